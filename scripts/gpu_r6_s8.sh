#!/bin/bash
# Round 6 session 8: counters of K3w against K3d on the CLIP-text q|k|v shape (M 16000): three SQ
# passes and one TA/TCP pass, merged per kernel (scripts/pmc_kernels.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/scripts/gemm_ws_probe.py 1536 512 0 k3w,k3d 16000"
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P3="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VALU"
P4="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r6s8_p$i -o run -- $CMD > $R/gpurun_out/r6s8_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/r6s8_p$i.log; exit $((10+i)); }
done
cd $R && python3 scripts/pmc_kernels.py gpurun_out/r6s8_pmc.json gpurun_out/r6s8_p1 gpurun_out/r6s8_p2 gpurun_out/r6s8_p3 gpurun_out/r6s8_p4 || exit 21
rm -rf gpurun_out/r6s8_p1 gpurun_out/r6s8_p2 gpurun_out/r6s8_p3 gpurun_out/r6s8_p4
python3 -c "
import json; d=json.load(open('gpurun_out/r6s8_pmc.json'))
for r in d['kernels'][:4]: print(json.dumps(r)[:1500])"
