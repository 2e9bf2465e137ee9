#!/bin/bash
# Round 4, session 13: L2 hit rate and memory-side fetch of the encoder GEMMs (is the K3 / K3d
# fill served from L2 or from the Infinity Cache / HBM?). Two separate --pmc passes per shape.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for s in qkv out t_qkv t_out; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/l2h_$s -o run -- python3 $R/scripts/gemm_bench.py $s > $R/gpurun_out/l2h_$s.log 2>&1 || { echo "hits $s failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/l2f_$s -o run -- python3 $R/scripts/gemm_bench.py $s > $R/gpurun_out/l2f_$s.log 2>&1 || { echo "fetch $s failed"; exit 2; }
done
cd $R
for s in qkv out t_qkv t_out; do echo "== $s"; grep -h '"shape"' gpurun_out/l2h_$s.log | cut -c1-100; python3 scripts/l2_hits.py gpurun_out/l2h_$s gpurun_out/l2f_$s gemm; done | tee gpurun_out/r4s13_l2.txt
find gpurun_out/l2h_* gpurun_out/l2f_* -name "*.csv" -size +5M -delete
