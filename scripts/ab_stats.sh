#!/bin/bash
# rocprofv3 kernel stats of bench.py --config $CFG for library variants
# usage: CFG=nat64 bash scripts/ab_stats.sh variant...
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $REPO/gpurun_out
cd /tmp
for v in "$@"; do
  OUT=$REPO/gpurun_out/abstats_$v
  CAPSULE_GPU_LIB=$REPO/capsule_amd/var/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o s --output-format csv -- python3 $REPO/bench.py --config ${CFG:-nat64} --only --no-cpu --steps 1000 --warmup 500 > $OUT.log 2>&1 || { echo "$v failed"; tail -5 $OUT.log; exit 1; }
  f=$(find $OUT -name '*kernel_stats.csv' | head -1)
  echo "== $v"; cut -d, -f1-4 "$f" | head -6
done
