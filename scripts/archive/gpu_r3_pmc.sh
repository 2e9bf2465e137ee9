#!/bin/bash
# Counter evidence for the kernels on today's path: three rocprofv3 --pmc passes
# (each within the per-block limits: <= 8 SQ, <= 2 GRBM counters) and one --kernel-trace --stats
# pass over the same bench command (every leg, one search in flight), reduced by
# scripts/pmc_kernels.py into profiles/r3_pmc_kernels.json.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --knn-streams 1"
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P3="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VALU"
P4="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r3pmc_p$i -o run -- $CMD > $R/gpurun_out/r3pmc_p$i.log 2>&1 || exit $((10+i))
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3pmc_stats -o run -- $CMD > $R/gpurun_out/r3pmc_stats.log 2>&1 || exit 20
cd $R && python3 scripts/pmc_kernels.py gpurun_out/r3_pmc_kernels.json gpurun_out/r3pmc_p1 gpurun_out/r3pmc_p2 gpurun_out/r3pmc_p3 gpurun_out/r3pmc_p4 || exit 21
# keep the reduced counters and the stats summary; the per-dispatch CSVs exceed what gpurun copies back
cp gpurun_out/r3pmc_stats/*kernel_stats.csv gpurun_out/r3_pmc_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/r3pmc_p1 gpurun_out/r3pmc_p2 gpurun_out/r3pmc_p3 gpurun_out/r3pmc_p4 gpurun_out/r3pmc_stats
ls -la gpurun_out; du -sh gpurun_out
