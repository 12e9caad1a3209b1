"""One process per GPU, one independent RX-queue shard per process.

The reference scales by NIC RSS: one RX/TX queue pair per core, shared
nothing (core/src/dpdk/port.rs:35-36, 510-515, 556-622; one worker thread per
core, core/src/runtime/core_map.rs:236-293).  Here each rank (= one MI355X)
owns its own shard of packets in its own HBM and runs the same kernels on
it; there is no data-path collective and RCCL is never initialised.  The
process group is a CPU (gloo) control plane: the start/stop barriers, the
max-over-ranks of the elapsed time and the gather of per-rank figures that
bench.py reports.

Ranks come from the environment (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT), as torch.distributed.run or bench.py's own
launcher (`launch_ranks`) set them.
"""
import os
import socket
import subprocess
import sys
import time


class ShardGroup:
    def __init__(self, backend="gloo"):
        if backend != "gloo":
            # the shards exchange no data: a device collective library has
            # nothing to carry
            raise ValueError("ShardGroup is a CPU control plane: backend must be gloo")
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.backend = backend
        self.pg = False
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo reports its connections on fd 1; rank 0's stdout carries
            # only bench.py's JSON line, so send those to stderr
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group(backend, rank=self.rank, world_size=self.world)
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.pg = True

    def shard_seed(self, base_seed):
        """Seed of this rank's RX queue: distinct, deterministic per rank."""
        return base_seed + 7919 * self.rank

    def barrier(self):
        if self.pg:
            import torch.distributed as dist

            dist.barrier()

    def _reduce(self, value, op):
        if not self.pg:
            return value
        import torch
        import torch.distributed as dist

        t = torch.tensor([value], dtype=torch.float64)
        dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
        return float(t.item())

    def max(self, value):
        return self._reduce(value, "MAX")

    def sum(self, value):
        return self._reduce(value, "SUM")

    def gather(self, value):
        """[value of rank 0, value of rank 1, ...] on every rank (floats)."""
        if not self.pg:
            return [float(value)]
        import torch
        import torch.distributed as dist

        out = [torch.zeros(1, dtype=torch.float64) for _ in range(self.world)]
        dist.all_gather(out, torch.tensor([float(value)], dtype=torch.float64))
        return [float(t.item()) for t in out]

    def gather_obj(self, value):
        """[value of rank 0, value of rank 1, ...] on every rank (any picklable
        value: the per-rank device identities of the bench line)."""
        if not self.pg:
            return [value]
        import torch.distributed as dist

        out = [None] * self.world
        dist.all_gather_object(out, value)
        return out

    def timed(self, fn, steps, sync=None):
        """sync + barrier, run `steps` calls of fn, sync; returns the max over
        ranks of the elapsed seconds (each rank's clock stops at its own
        sync, then the ranks meet at a barrier)."""
        if sync:
            sync()
        self.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        if sync:
            sync()
        el = time.perf_counter() - t0
        self.barrier()
        return self.max(el)

    def close(self):
        if self.pg:
            import torch.distributed as dist

            dist.destroy_process_group()
            self.pg = False


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv, script=None, env=None, timeout=None):
    """Start `n` rank processes of `script` (default: the running script)
    with `argv`, one per GPU, and wait for them; returns the worst exit code.

    The caller must not have touched the GPU: the ranks are new child
    processes (never an exec of this one), each with RANK = LOCAL_RANK = r,
    WORLD_SIZE = n and a loopback rendezvous (MASTER_ADDR 127.0.0.1).  If a
    rank fails, the others are terminated (by their own PIDs) so that none
    is left waiting at a barrier."""
    script = script or os.path.abspath(sys.argv[0])
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=e))
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0:
                rc = rc or code
                for q in pending:
                    q.terminate()
        if deadline is not None and time.monotonic() > deadline:
            for q in pending:
                q.kill()
            rc = rc or 124
        if pending:
            time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def _cpulist(text):
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11} (sysfs cpulist format)."""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def numa_bind(pci, sysfs="/sys"):
    """Bind the calling thread (and the threads it starts later) to the CPUs
    of the NUMA node its GPU hangs off, before the rank allocates any host
    buffer: one RX queue per core on the GPU's own socket, as capsule's core
    map pins each core's queues (runtime/core_map.rs:236-293), and page-locked
    buffers first touched on the node of the GPU's PCIe root.  `pci`:
    "dddd:bb:dd" (bench.py device_identity).  Returns what was done, for the
    bench line: {"node", "cpus", "bound", "reason"}."""
    info = {"node": None, "cpus": 0, "bound": False, "reason": None}
    try:
        dom, bus, dev = pci.split(":")
        path = os.path.join(sysfs, "bus", "pci", "devices", f"{dom}:{bus}:{dev}.0", "numa_node")
        with open(path) as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        info["reason"] = "no sysfs numa_node for the GPU"
        return info
    info["node"] = node
    if node < 0:
        info["reason"] = "the platform reports no NUMA node for the GPU"
        return info
    try:
        with open(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist")) as f:
            cpus = _cpulist(f.read())
    except (OSError, ValueError):
        info["reason"] = f"no cpulist for node {node}"
        return info
    allowed = cpus & os.sched_getaffinity(0)
    if not allowed:
        info["reason"] = f"none of node {node}'s CPUs is allowed to this process"
        return info
    os.sched_setaffinity(0, allowed)
    info.update(cpus=len(allowed), bound=True)
    return info
