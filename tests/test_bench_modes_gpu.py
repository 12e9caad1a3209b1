"""Every mode bench.py runs, run the way the driver and DESIGN.md run it: a
fresh `python bench.py ...` process per mode, on a small batch (--n), whose
last stdout line must be one JSON object with the fields that mode reports.
This is what keeps a bench path from dying unnoticed (round 2: a NameError in
`--e2e --config nat64`)."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]
N = "65536"
SMALL = ["--n", N, "--steps", "6", "--warmup", "2", "--sub-steps", "6", "--cpu-seconds", "0.3"]


def _run(args, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, "bench.py"] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, (args, r.stderr[-3000:])
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, (args, r.stdout[-2000:])
    return json.loads(lines[0])


def test_bench_default_line():
    """The driver's own invocation, on a small batch: the metric line with
    every object (shards, sizes, rx_queues, cpu_baseline)."""
    d = _run(SMALL)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["config"] == "parse64"
    assert d["config"]["packets_per_step"] == int(N)
    assert {"roofline", "cpu_baseline", "shards", "sizes", "rx_queues"} <= set(d)
    import bench

    assert set(d["sizes"]) == set(bench.SIZES)
    for c, s in d["sizes"].items():
        assert s["kernel_us"] > 0 and s["frac"] > 0, c
    assert "line_floor_bytes" in d["shards"] and "frac_of_line_floor" in d["sizes"]["imix_csum"]
    assert "new keys per call" in d["sizes"]["nat64_cold"]["note"]
    assert d["roofline"]["per_rank"][0]["device"]["pci"]


@pytest.mark.parametrize("cfg", ["parse64", "parse256", "parse1500", "imix", "imix_csum", "nat64",
                                 "nat64_4to6", "nat64_cold"])
def test_bench_config(cfg):
    d = _run(SMALL + ["--config", cfg, "--only"])
    assert d["config"]["config"] == cfg and d["value"] > 0
    assert d["roofline"]["frac"] > 0 and d["cpu_baseline"]["value"] > 0


@pytest.mark.parametrize("cfg", ["parse64", "imix_csum", "nat64", "nat64_4to6"])
def test_bench_e2e(cfg):
    d = _run(["--e2e", "--config", cfg, "--n", N, "--steps", "20", "--warmup", "10"])
    assert d["value"] > 0 and d["h2d_GBps"] > 0 and d["config"] == cfg


@pytest.mark.parametrize("cfg,ingress", [("parse64", "stage"), ("parse64", "zero_copy"),
                                         ("parse64", "frames"), ("imix_csum", "zero_copy"),
                                         ("nat64", "zero_copy"), ("nat64", "frames"),
                                         ("nat64_4to6", "zero_copy"), ("nat64_4to6", "frames")])
def test_bench_e2e_ingress(cfg, ingress):
    d = _run(["--e2e", "--config", cfg, "--ingress", ingress, "--n", N, "--burst", "16384",
              "--steps", "20"])
    assert d["value"] > 0 and d["ingress"] == ingress and d["burst"] == 16384
    if cfg.startswith("nat64"):  # every frame of the stream (and every reply) is rewritten
        assert d["act_frac"] == 1.0
        assert ("4to6" in d["metric"]) == (cfg == "nat64_4to6")
