#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (TCC slots; never combined with traces).
# usage: bash scripts/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
ARGS="$*"
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
run() {  # name, limit, rocprof args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv \
      -- python3 "$REPO/bench.py" --no-cpu --only $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run stats 400 --kernel-trace --stats
run fetch 400 --pmc FETCH_SIZE
run write 400 --pmc WRITE_SIZE
find "$OUT" -name '*.csv' | head -20
