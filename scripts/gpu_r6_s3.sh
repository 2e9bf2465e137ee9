#!/bin/bash
# Round 6 session 3: where the config-5 and CLIP legs spend their time on this tree: the config-5
# step serialised under a kernel trace, the CLIP tower one batch at a time under a kernel trace,
# the text-tower GEMMs alone per epilogue (is the erf-GELU epilogue the cost?), and one LDS
# counter pass over the CLIP bench (attention bank conflicts).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6s3_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r6s3_tests.log; exit 3; }
tail -1 gpurun_out/r6s3_tests.log
timeout -k 10 300 python3 scripts/gemm_roofline.py --only minilm:fc1,minilm:qkv,clip_text:fc1,clip_text:qkv > gpurun_out/r6s3_gemm_native.jsonl 2>&1 || { echo "gemm failed"; tail gpurun_out/r6s3_gemm_native.jsonl; exit 2; }
for e in 0 1 2; do timeout -k 10 300 python3 scripts/gemm_roofline.py --only minilm:fc1,clip_text:fc1 --epi $e >> gpurun_out/r6s3_gemm_epi.jsonl 2>&1 || exit 2; done
cat gpurun_out/r6s3_gemm_native.jsonl gpurun_out/r6s3_gemm_epi.jsonl | cut -c1-260
cd /tmp && export TMPDIR=/tmp
MRAG_FUSION_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6s3_fusion -o run -- python3 $R/scripts/fusion_profile.py 10 > $R/gpurun_out/r6s3_fusion.log 2>&1 || { echo "fusion prof failed"; tail -5 $R/gpurun_out/r6s3_fusion.log; exit 6; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6s3_clip -o run -- python3 $R/scripts/clip_bench.py 10 1 > $R/gpurun_out/r6s3_clip.log 2>&1 || { echo "clip prof failed"; exit 7; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/r6s3_clip_lds -o run -- python3 $R/scripts/clip_bench.py 3 1 > $R/gpurun_out/r6s3_clip_lds.log 2>&1 || { echo "lds pmc failed"; exit 8; }
cd $R
for d in r6s3_fusion r6s3_clip; do f=$(find gpurun_out/$d -name "*kernel_trace.csv" | head -1); python3 scripts/trace_by_grid.py "$f" > gpurun_out/${d}_by_grid.txt 2>/dev/null; head -25 gpurun_out/${d}_by_grid.txt; find gpurun_out/$d -name "*kernel_trace.csv" -delete; done
tail -2 gpurun_out/r6s3_fusion.log gpurun_out/r6s3_clip.log
f=$(find gpurun_out/r6s3_clip_lds -name "*counter_collection.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_LDS_IDX_ACTIVE", 0))[:12]:
    a = v.get("SQ_LDS_IDX_ACTIVE", 0)
    print(f"{k:60s} conflict/active {v.get('SQ_LDS_BANK_CONFLICT', 0) / max(a, 1):.3f} lds_insts {v.get('SQ_INSTS_LDS', 0):.3g}")
PY
find gpurun_out/r6s3_clip_lds -name "*counter_collection.csv" -size +5M -delete
