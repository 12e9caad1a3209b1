#!/bin/bash
# Build a variant of libcapsule_gpu.so into capsule_amd/var/<name>.so for A/B
# timing (bench.py honours CAPSULE_GPU_LIB).
# usage: bash scripts/build_variant.sh <name> <git-rev|WORKTREE> [extra hipcc flags...]
set -e
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/capsule_amd/csrc
TMP=$(mktemp -d)
for f in capi.hip parse.hip nat64.hip group_by.hip ingress.hip setip.hip device_common.hpp kernels.hpp; do
  if [ "$REV" = WORKTREE ]; then cp "$SRC/$f" "$TMP/$f"; else git -C "$ROOT" show "$REV:capsule_amd/csrc/$f" > "$TMP/$f"; fi
done
mkdir -p "$ROOT/capsule_amd/var"
OBJS=""
for f in capi parse nat64 group_by ingress setip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I"$ROOT/include" -Wno-unused-function "$@" -c "$TMP/$f.hip" -o "$TMP/$f.o" &
  OBJS="$OBJS $TMP/$f.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -o "$ROOT/capsule_amd/var/$NAME.so"
rm -rf "$TMP"
echo "built capsule_amd/var/$NAME.so"
