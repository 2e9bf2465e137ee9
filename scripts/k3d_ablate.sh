#!/bin/bash
# K3d timing ablations (results wrong by design), round 4: run on a checkout of commit 227f50e (the
# ablation bits were removed from the product kernel in round 5). Builds libs with -DMRAG_K3D_ABL=<mask> (bits in
# csrc/encoder_kernels.hip; 64 = one reduced value per lane instead of the epilogue stores, the
# MFMAs kept live) on the CPU side, then (GPU, "run") time the ViT / text GEMM shapes with
# each. Usage: scripts/k3d_ablate.sh build | run
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/multimodal-rag-for-image-text-search_amd
MASKS="${MASKS:-0 1 2 3 4 8 12 13 15 47 64 65 66 67 76 128}"
if [ "$1" = build ]; then
  make -C $P -j8 >/dev/null
  for m in $MASKS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DMRAG_K3D_ABL=$m -c $P/csrc/encoder_kernels.hip -o $P/build/ek_abl$m.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $P/lib/libmrag_abl$m.so $(ls $P/build/*.o | grep -v encoder_kernels.hip.o | grep -v ek_abl | grep -v knn_stamp) $P/build/ek_abl$m.o
  done
  ls -la $P/lib
else
  mkdir -p $R/gpurun_out
  for m in $MASKS; do
    MRAG_LIB=$P/lib/libmrag_abl$m.so timeout -k 10 120 python3 -u $R/scripts/gemm_bench.py qkv out fc2 t_qkv > $R/gpurun_out/k3d_abl$m.log 2>&1 || { echo "abl $m failed"; exit 1; }
    echo "mask $m: $(grep -h '"shape"' $R/gpurun_out/k3d_abl$m.log | python3 -c "
import sys, json
print(' '.join(f\"{d['shape']}={d['us']}\" for d in map(json.loads, sys.stdin)))")" | tee -a $R/gpurun_out/k3d_ablate.txt
  done
fi
