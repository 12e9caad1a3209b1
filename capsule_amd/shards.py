"""One process per GPU, one independent RX-queue shard per process.

The reference scales by NIC RSS: one RX/TX queue pair per core, shared
nothing (core/src/dpdk/port.rs:35-36, 510-515, 556-622).  Here each rank
(= one MI355X, launched by torch.distributed.run) owns its own shard of
packets in its own HBM and runs the same kernels on it; there is no data-path
collective.  The process group exists only for the start/stop barrier and
the max-over-ranks reduction of the elapsed time that bench.py reports.
"""
import os
import time

import torch
import torch.distributed as dist


class ShardGroup:
    def __init__(self, backend=None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = False
        if self.world > 1:
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)
                dist.init_process_group(backend, device_id=torch.device("cuda", self.local_rank))
            else:
                dist.init_process_group(backend)
            self.backend = backend
            self.pg = True

    def shard_seed(self, base_seed):
        """Seed of this rank's RX queue: distinct, deterministic per rank."""
        return base_seed + 7919 * self.rank

    def barrier(self):
        if self.pg:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def _reduce(self, value, op):
        if not self.pg:
            return value
        dev = torch.device("cuda", self.local_rank) if self.backend == "nccl" else "cpu"
        t = torch.tensor([value], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, value):
        return self._reduce(value, dist.ReduceOp.MAX)

    def sum(self, value):
        return self._reduce(value, dist.ReduceOp.SUM)

    def timed(self, fn, steps, sync=None):
        """Barrier + sync, run `steps` calls of fn, sync + barrier; returns the
        max elapsed seconds over ranks."""
        if sync:
            sync()
        self.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        if sync:
            sync()
        self.barrier()
        return self.max(time.perf_counter() - t0)

    def close(self):
        if self.pg:
            dist.destroy_process_group()
            self.pg = False
