#!/bin/bash
# Build a timing variant of libcapsule_gpu.so into capsule_amd/var/<name>.so
# from the working tree with a sed expression applied to one source file
# (A/B builds that must not live in the product sources).
# usage: bash scripts/build_patched.sh <name> <file.hip> '<sed expr>' [extra hipcc flags...]
set -e
NAME=$1; FILE=$2; EXPR=$3; shift 3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp "$ROOT"/capsule_amd/csrc/*.hip "$ROOT"/capsule_amd/csrc/*.hpp "$TMP/"
sed -i "$EXPR" "$TMP/$FILE"
if cmp -s "$TMP/$FILE" "$ROOT/capsule_amd/csrc/$FILE"; then echo "sed changed nothing in $FILE" >&2; exit 1; fi
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
