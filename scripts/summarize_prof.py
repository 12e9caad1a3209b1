"""Summarize a scripts/profile.sh run into profiles/<tag>/ (committed).

usage: python scripts/summarize_prof.py <gpurun_out/prof_TAG> <profiles/TAG> <config>

Writes <config>_kernel_stats.csv (rocprofv3 --stats), <config>_pmc.json
(FETCH_SIZE / WRITE_SIZE per dispatch of the dominant kernel, corrected as
MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE counts half the bytes of a
wide coalesced read on gfx950, so bytes = 2 x FETCH_SIZE KiB x 1024;
WRITE_SIZE is exact for 16-B-per-lane stores) and, when the kernel sources
are unchanged, profiles/pmc_<config>.json that bench.py reads to fill
roofline.traffic.
"""
import csv
import hashlib
import json
import pathlib
import shutil
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


# the sources whose code a config's kernels are built from
_CONFIG_SOURCES = {"parse": ["parse.hip"], "nat64": ["nat64.hip"]}


def source_hash(config="parse64"):
    """Hash of the kernel sources a config runs (shared headers included)."""
    fam = "nat64" if config.startswith("nat64") else "parse"
    h = hashlib.sha256()
    csrc = ROOT / "capsule_amd" / "csrc"
    for name in sorted(_CONFIG_SOURCES[fam] + ["device_common.hpp", "kernels.hpp"]):
        h.update(name.encode())
        h.update((csrc / name).read_bytes())
    h.update((ROOT / "include" / "capsule_gpu.h").read_bytes())
    return h.hexdigest()[:16]


def main():
    src, dst, config = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2]), sys.argv[3]
    dst.mkdir(parents=True, exist_ok=True)
    stats = next(src.glob("stats/*kernel_stats.csv"))
    shutil.copy(stats, dst / f"{config}_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    kernel = top["Name"]
    out = {"config": config, "kernel": kernel, "calls": int(top["Calls"]),
           "avg_ns": float(top["AverageNs"]), "min_ns": float(top["MinNs"]),
           "src_hash": source_hash(config)}
    for name, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = next(src.glob(f"{name}/*counter_collection.csv"), None)
        if f is None:
            continue
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
             if r["Kernel_Name"] == kernel and r["Counter_Name"] == ctr]
        if v:
            out[ctr] = {"dispatches": len(v), "mean_kib": sum(v) / len(v)}
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        rd = 2 * out["FETCH_SIZE"]["mean_kib"] * 1024
        wr = out["WRITE_SIZE"]["mean_kib"] * 1024
        out["hbm_read_bytes"] = rd
        out["hbm_write_bytes"] = wr
        out["traffic_bytes"] = rd + wr
    (dst / f"{config}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
    (ROOT / "profiles" / f"pmc_{config}.json").write_text(json.dumps(out, indent=1) + "\n")
    for log in src.glob("*.log"):
        shutil.copy(log, dst / f"{config}_{log.name}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
