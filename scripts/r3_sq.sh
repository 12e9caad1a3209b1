#!/bin/bash
# SQ counters of the rows/stream kernel (IMIX csum vs 1500 B) and the list of counters
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/avail.txt 2>&1 || { echo list failed; }
for c in imix_csum parse1500 parse64; do
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM"; do
    n=$(echo $P | cut -c1-12 | tr ' ' _)
    OUT=$GRAFT_REPO_ROOT/gpurun_out/sq_${c}_$n
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 5 --no-cpu --only > $OUT.log 2>&1
    rc=$?; echo "$c $n rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT.log; exit $rc; fi
  done
done
