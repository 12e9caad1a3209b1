#!/bin/bash
# rocprofv3 PMC pass(es) over bench.py for one config; per-kernel means.
# usage: bash scripts/pmc.sh <config> "<counters pass 1>" ["<counters pass 2>" ...]
CFG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
n=0
for ctrs in "$@"; do
  n=$((n+1))
  OUT=$REPO/gpurun_out/pmc_${CFG}_$n
  timeout -k 10 300 rocprofv3 --pmc $ctrs -d $OUT -o pmc --output-format csv -- python3 $REPO/bench.py --config $CFG --steps 30 --warmup 5 --no-cpu --only > $OUT.log 2>&1 || { echo "pmc pass $n rc=$?"; tail -5 $OUT.log; exit 1; }
  python3 - $OUT <<'PY'
import csv, sys, glob, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if 'copyBuffer' in r['Kernel_Name'] or 'portmap_init' in r['Kernel_Name']: continue
    name = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0].replace('cgpu::', '')[:48]
    agg[name][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    w = m.get('SQ_WAVES')
    extra = ''
    if w:
        extra = ' | per wave: ' + ' '.join(f"{c.replace('SQ_','')}={v / w:.0f}" for c, v in m.items() if c != 'SQ_WAVES')
    print(k, {c: round(v) for c, v in m.items()}, extra)
PY
done
