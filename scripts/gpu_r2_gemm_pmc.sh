#!/bin/bash
# L2 behaviour of the encoder GEMMs (CLIP image leg + config-5 towers): TCC hit/miss, HBM fetch
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/r2_gpmc_l2 -o run -- python3 $R/scripts/clip_bench.py 3 > $R/gpurun_out/r2_gpmc_l2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r2_gpmc_fetch -o run -- python3 $R/scripts/clip_bench.py 3 > $R/gpurun_out/r2_gpmc_fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/r2_gpmc_l2f -o run -- python3 $R/scripts/fusion_bench.py 3 > $R/gpurun_out/r2_gpmc_l2f.log 2>&1 || exit 3
