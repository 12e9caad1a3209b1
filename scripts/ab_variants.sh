#!/bin/bash
# A/B timing of capsule_amd/var/*.so variants: bench (+ optional PMC pass).
# usage: bash scripts/ab_variants.sh "<configs>" "<pmc counters or ->" variant...
# (several PMC passes: separate the counter sets with ';')
CFGS=$1; PMC=$2; shift 2
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $REPO/gpurun_out
for v in "$@"; do
  for c in $CFGS; do
    CAPSULE_GPU_LIB=$REPO/capsule_amd/var/$v.so timeout -k 10 200 python3 $REPO/bench.py --config $c --steps ${AB_STEPS:-2000} --warmup 1000 --no-cpu --only > $REPO/gpurun_out/ab_${v}_$c.log 2>&1 || { echo "$v $c failed"; tail -5 $REPO/gpurun_out/ab_${v}_$c.log; exit 1; }
    python3 - $REPO/gpurun_out/ab_${v}_$c.log $v $c <<'PY'
import json, sys
r = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
print(sys.argv[2], sys.argv[3], "Mpps", r["value"], "kernel_us", r["roofline"]["kernel_us"], "frac", r["roofline"]["frac"])
PY
    if [ "$PMC" != "-" ]; then
    IFS=';' read -ra PASSES <<< "$PMC"
    pi=0
    for P in "${PASSES[@]}"; do
      pi=$((pi+1))
      OUT=$REPO/gpurun_out/abpmc_${v}_${c}_$pi
      (cd /tmp && CAPSULE_GPU_LIB=$REPO/capsule_amd/var/$v.so timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT -o pmc --output-format csv -- python3 $REPO/bench.py --config $c --steps 20 --warmup 5 --no-cpu --only > $OUT.log 2>&1) || { echo "pmc $v $c failed"; tail -5 $OUT.log; exit 1; }
      python3 - $OUT <<'PY'
import csv, sys, glob, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if 'copyBuffer' in n or 'portmap_init' in n: continue
    n = n.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0].replace('cgpu::', '')[:40]
    agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    print("  ", k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
    done
    fi
  done
done
