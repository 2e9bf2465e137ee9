#!/bin/bash
# Round 6 (as round 5): SQ counters for every kernel of the bench trace (four rocprofv3 --pmc passes, each within
# the per-block limits: <= 8 SQ, <= 2 GRBM), reduced per kernel by scripts/pmc_kernels.py into
# gpurun_out/r6_pmc_kernels.json (MFMA busy, WAIT_ANY, LDS busy, effective clock ...).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --knn-streams 1 --no-ingest --no-retrieve-pattern"
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P3="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VALU"
P4="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r6pmc_p$i -o run -- $CMD > $R/gpurun_out/r6pmc_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/r6pmc_p$i.log; exit $((10+i)); }
done
cd $R && python3 scripts/pmc_kernels.py gpurun_out/r6_pmc_kernels.json gpurun_out/r6pmc_p1 gpurun_out/r6pmc_p2 gpurun_out/r6pmc_p3 gpurun_out/r6pmc_p4 || exit 21
rm -rf gpurun_out/r6pmc_p1 gpurun_out/r6pmc_p2 gpurun_out/r6pmc_p3 gpurun_out/r6pmc_p4
python3 -c "
import json; d=json.load(open('gpurun_out/r6_pmc_kernels.json'))
for r in d['kernels'][:16]: print(r['kernel'][:60], r.get('avg_wall_ms'), r.get('mfma_busy_frac'), r.get('wait_any_frac'), r.get('eff_clock_ghz'))"
