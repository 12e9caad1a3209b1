#!/bin/bash
# parity first, then microbench + instruction-count PMC of the parse kernel
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -m pytest tests/test_parse_gpu.py -q -m gpu -x > gpurun_out/parse_tests.log 2>&1
rc=$?; tail -3 gpurun_out/parse_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 tools/microbench > gpurun_out/micro.log 2>&1 || exit $?
cat gpurun_out/micro.log
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_insts -o pmc --output-format csv -- $R/tools/microbench 1048576 20 ${CASE:-parse_verify_hash} > $R/gpurun_out/pmc_insts.log 2>&1 || { echo pmc rc=$?; tail $R/gpurun_out/pmc_insts.log; exit 0; }
python3 - "$R/gpurun_out/pmc_insts/pmc_counter_collection.csv" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'parse_kernel' in r['Kernel_Name']]
agg = collections.defaultdict(list)
for r in rows: agg[r['Counter_Name']].append(float(r['Counter_Value']))
m = {k: sum(v)/len(v) for k, v in agg.items()}
print({k: round(v) for k, v in m.items()})
w = m.get('SQ_WAVES', 1)
print('per wave: VALU %.0f SALU %.0f VMEM_RD %.1f VMEM_WR %.1f' % (m.get('SQ_INSTS_VALU',0)/w, m.get('SQ_INSTS_SALU',0)/w, m.get('SQ_INSTS_VMEM_RD',0)/w, m.get('SQ_INSTS_VMEM_WR',0)/w))
PY
