#!/bin/bash
# The driver's multi-GPU launch (torch.distributed.run, one rank per GPU),
# rehearsed with N ranks sharing the one GPU of a test box.
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-2}
CGPU_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --steps 20 --warmup 5 \
  > gpurun_out/torchrun_$N.log 2> gpurun_out/torchrun_$N.err
rc=$?; echo "torchrun N=$N rc=$rc"; tail -1 gpurun_out/torchrun_$N.log | cut -c1-400; tail -3 gpurun_out/torchrun_$N.err
exit $rc
