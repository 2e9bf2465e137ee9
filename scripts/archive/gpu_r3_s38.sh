#!/bin/bash
# Round 3, session 38: K8 merge A/B on one box (prev = HEAD, nostage = loads-together rescoring +
# wave sort, cur = also the staged key fold): kernel timelines at Q = 1 and Q = 1000.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=$R/multimodal-rag-for-image-text-search_amd/lib
cd /tmp && export TMPDIR=/tmp && cd $R
for round in 1 2; do
for v in prev nostage cur; do
  lib=$L/libmrag_$v.so; [ $v = cur ] && lib=$L/libmrag.so
  for nq in 1 1000; do
    rm -rf gpurun_out/r3s38_prof
    MRAG_LIB=$lib NQ=$nq timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s38_prof -o q1 -- python3 scripts/q1_profile.py > gpurun_out/r3s38_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s38_prof.log; exit 3; }
    f=$(find gpurun_out/r3s38_prof -name "*kernel_trace.csv" | head -1)
    echo "== $v nq=$nq $(grep ms_per_search gpurun_out/r3s38_prof.log)" >> gpurun_out/r3s38_ab.log
    python3 scripts/q1_profile.py --trace "$f" | grep -v "pos\": 0" >> gpurun_out/r3s38_ab.log
  done
done
done
rm -rf gpurun_out/r3s38_prof
cat gpurun_out/r3s38_ab.log
