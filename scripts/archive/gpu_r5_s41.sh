#!/bin/bash
# Round 5, session 41: K13a at 256 lanes x >= 4096 bits (the tree) vs 512 x 2048 and 1024 x 1024
# (lib/libmrag_par512.so, lib/libmrag_par1024.so): JPEG GPU tests on each, the device-decode
# stage alone per group, and a kernel trace of each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=$R/multimodal-rag-for-image-text-search_amd/lib
for v in par1024 par512; do
  MRAG_LIB=$L/libmrag_$v.so timeout -k 10 400 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s41_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/r5s41_tests_$v.log; exit 3; }
  tail -1 gpurun_out/r5s41_tests_$v.log
done
O=gpurun_out/r5s41_split.jsonl; : > $O
for i in 1 2; do
  for v in libmrag libmrag_par512 libmrag_par1024; do
    MRAG_LIB=$L/$v.so timeout -k 10 300 python3 -u scripts/decode_stage_split.py >> $O 2>> gpurun_out/r5s41.err || { echo "split $v failed"; tail gpurun_out/r5s41.err; exit 4; }
  done
done
cat $O
cd /tmp && export TMPDIR=/tmp
for v in libmrag libmrag_par512 libmrag_par1024; do
  MRAG_LIB=$L/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5s41_prof_$v -o run -- python3 $R/scripts/decode_stage_split.py > $R/gpurun_out/r5s41_prof_$v.log 2>&1 || { echo "prof $v failed"; exit 5; }
  f=$(find $R/gpurun_out/r5s41_prof_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; cut -d, -f1-4 "$f" | head -6
  find $R/gpurun_out/r5s41_prof_$v -name "*trace.csv" -delete
done
