"""Debug helper: 1M IMIX parse (checksums) vs the oracle; reports the failing
packets by wave position and whether the host thinks the wave streams."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import oracle_lib
from capsule_amd import _native as N, packets, synth

ctx = packets.Context(0)
arena, off, ln = synth.imix(1 << 20)
flags = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
for fields in (False, True):
    b = packets.PacketBatch.from_numpy(arena, off, ln, "cuda:0")
    r = packets.parse(ctx, b, flags=flags, fields=fields)
    torch.cuda.synchronize()
    gm = r.meta.cpu().numpy().view(np.uint32)
    gc = r.csum.cpu().numpy().view(np.uint32)
    om, oc, oh, _ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
    bad = np.nonzero((gm != om) | (gc != oc))[0]
    print("fields", fields, "bad", len(bad))
    if len(bad):
        w = bad // 64
        o = off.astype(np.int64); L = ln.astype(np.int64)
        for wi in np.unique(w)[:6]:
            s = slice(64 * wi, 64 * wi + 64)
            span = o[s][-1] + L[s][-1] - o[s][0]
            asc = (np.diff(o[s]) >= L[s][:-1]).all() and (o[s] % 16 == 0).all()
            print(" wave", wi, "span", span, "asc", asc, "anylong", (L[s] > 96).any(),
                  "bad lanes", (bad[w == wi] % 64).tolist()[:20])
            j = bad[w == wi][0]
            print("  pkt", j, "len", L[j], "off", o[j], "meta g/o", hex(gm[j]), hex(om[j]),
                  "csum g/o", hex(gc[j]), hex(oc[j]))
