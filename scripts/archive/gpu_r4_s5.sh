#!/bin/bash
# Round 4, session 5: K3 residual at the MiniLM fc2 shape (1134 us outlier in r4s4) under a kernel trace.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
MRAG_GEMM_BLASLT=0 timeout -k 10 200 python -u scripts/gemm_bench.py m_fc2 m_out t_fc2 m_fc2 > gpurun_out/r4s5_gemm.log 2>&1; rc=$?; echo "gemm rc=$rc"; fatal $rc gemm
cd /tmp && export TMPDIR=/tmp && MRAG_GEMM_BLASLT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4s5_prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py m_fc2 > $GRAFT_REPO_ROOT/gpurun_out/r4s5_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; cd $GRAFT_REPO_ROOT
grep -h shape gpurun_out/r4s5_gemm.log | cut -c1-100
find gpurun_out/r4s5_prof -name "*kernel_stats.csv" | head -2 | xargs -I{} head -5 {}
