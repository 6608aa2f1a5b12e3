#!/bin/bash
# Development build of the library (-DSM_DEV: SM_* A/B switches and ablation kernels)
# into build/dev/libsparsematrix_amd.so; bench.py / tests use it with SM_LIB_PATH.
# Extra flags (e.g. -DSM_CB_XAHEAD=3) through DEV_FLAGS; OUT overrides the directory.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-$ROOT/build/dev}
mkdir -p "$OUT/obj"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -Wall -I$ROOT/include -I$ROOT/sparsematrix_amd/csrc -DSM_DEV ${DEV_FLAGS:-}"
objs=()
for f in "$ROOT"/sparsematrix_amd/csrc/*.hip "$ROOT"/sparsematrix_amd/csrc/*.cpp; do
  b=$(basename "$f"); [[ $b == sblas_shim.cpp ]] && continue
  o="$OUT/obj/${b%.*}.o"; objs+=("$o")
  /opt/rocm/bin/hipcc $FLAGS -c "$f" -o "$o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libsparsematrix_amd.so" "${objs[@]}" -ldl
echo "built $OUT/libsparsematrix_amd.so"
