#!/bin/bash
# Build lib/libmrag_<name>.so from the csrc/ + include/ of git revision <rev>, for same-box A/B
# timing against the working tree (MRAG_LIB=.../lib/libmrag_<name>.so selects it at run time).
#   scripts/ab_lib.sh <rev|.> <name> [extra hipcc flags]   (. = the working tree)
# STAMP=1 also builds the K7 stamp library as lib/libmrag_k7stamp_<name>.so (scripts/k7_stamps.py).
set -e
rev=$1; name=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
P=multimodal-rag-for-image-text-search_amd
T=$(mktemp -d /tmp/ab_${name}_XXXX)
mkdir -p $T/$P $T/include
if [ "$rev" = "." ]; then  # the working tree as it is
  cp -r $R/$P/csrc $R/$P/Makefile $T/$P/ && cp -r $R/include $T/
else
  git -C $R archive $rev $P/csrc $P/Makefile include | tar -x -C $T
fi
make -C $T/$P -j8 CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*" > $T/build.log 2>&1 || { tail -20 $T/build.log; exit 1; }
cp $T/$P/lib/libmrag.so $R/$P/lib/libmrag_$name.so
if [ "${STAMP:-0}" = 1 ]; then
  make -C $T/$P -j8 stamp CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*" >> $T/build.log 2>&1 || { tail -20 $T/build.log; exit 1; }
  cp $T/$P/lib/libmrag_k7stamp.so $R/$P/lib/libmrag_k7stamp_$name.so
fi
rm -rf $T
echo "built $P/lib/libmrag_$name.so from $rev"
