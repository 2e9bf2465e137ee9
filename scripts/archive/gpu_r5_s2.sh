#!/bin/bash
# Round 5, session 2: K7 group-test fires inserted best value first (bf) vs register order with
# the chain-free insert (par), bf with a 1/32 sample pre-pass (bfs32); kNN tests on bf; stamps;
# counters of K3 (par) vs K3x (ax) on two GEMM shapes (why K3x was slower in s1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
MRAG_LIB=$R/$L/libmrag_bf.so timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s2_knn_tests.log 2>&1 || { echo "knn tests failed"; tail -30 gpurun_out/r5s2_knn_tests.log; exit 3; }
tail -1 gpurun_out/r5s2_knn_tests.log
for v in par bf bfs32 par bf bfs32 par bf bfs32; do
  MRAG_LIB=$R/$L/libmrag_$v.so timeout -k 10 240 python3 -u scripts/knn_scan_ab.py 40 > gpurun_out/r5s2_ab_$v.json 2>/dev/null || { echo "ab $v failed"; exit 4; }
  echo "$v $(cat gpurun_out/r5s2_ab_$v.json)" | tee -a gpurun_out/r5s2_ab.txt
done
MRAG_LIB=$R/$L/libmrag_k7stamp_bf.so timeout -k 10 240 python3 -u scripts/k7_stamps.py > gpurun_out/r5s2_stamps_bf.log 2>&1 || { echo "stamps failed"; exit 5; }
grep case gpurun_out/r5s2_stamps_bf.log | head -1 | cut -c1-400
cd /tmp && export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM"
P2="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
P3="FETCH_SIZE"
for v in par ax; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    MRAG_LIB=$R/$L/libmrag_$v.so timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r5s2_pmc_${v}_p$i -o run -- python3 $R/scripts/gemm_bench.py t_fc2 qkv > $R/gpurun_out/r5s2_pmc_${v}_p$i.log 2>&1 || { echo "pmc $v $i failed"; tail -5 $R/gpurun_out/r5s2_pmc_${v}_p$i.log; exit 6; }
  done
  cd $R && python3 scripts/pmc_kernels.py gpurun_out/r5s2_pmc_$v.json gpurun_out/r5s2_pmc_${v}_p1 gpurun_out/r5s2_pmc_${v}_p2 gpurun_out/r5s2_pmc_${v}_p3 > /dev/null 2>&1; cd /tmp
  rm -rf $R/gpurun_out/r5s2_pmc_${v}_p*/
done
cd $R; ls gpurun_out | grep r5s2
