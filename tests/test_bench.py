"""bench.py's measurement plumbing: the roofline's kernel pick and its counter
provenance (a PMC summary is used only for the sources it was taken on), the
strong-scaling emulation (--emulate-ranks), and on the GPU one short bench run
with the parity leg and the emulation."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_emulated_scaling_fields():
    e = bench.emulated_scaling({2: [300.0, 320.0], 8: [80.0] * 7 + [90.0]}, 620.0, 530.8e6)
    assert e["frame_ms_1gpu"] == 620.0 and "ncclReduce" in e["excludes"]
    r2, r8 = e["ranks"]["2"], e["ranks"]["8"]
    assert r2["max_ms"] == 320.0 and r2["predicted_efficiency"] == round(620 / 2 / 320, 4)
    assert r8["imbalance"] == round(90 / (80 * 7 / 8 + 90 / 8), 4)
    assert r8["predicted_msamples_per_s"] == round(530.8e6 / 0.09 / 1e6, 2)
    for v in e["ranks"].values():
        assert set(v) == {"per_rank_ms", "max_ms", "mean_ms", "imbalance", "predicted_msamples_per_s",
                          "predicted_efficiency"}


def test_source_hash_stable():
    assert bench.source_hash() == bench.source_hash()
    assert len(bench.source_hash()) == 16


def test_kernel_match_is_exact():
    assert bench._kernel_match("void pt::k_shade_w3<16>", "k_shade_w3")
    assert not bench._kernel_match("void pt::k_shade_w3<16>", "k_shade")
    assert bench._kernel_match("pt::k_shade<0>", "k_shade")


def _timed(trace_ms, shade_ms):
    return {"trace_ms": trace_ms, "trace_launches": 100, "shade_ms": shade_ms, "shade_launches": 100,
            "node_visits": 10 ** 9, "prim_tests": 10 ** 8, "shade_bytes": 10 ** 12}


def test_roofline_kernel_is_timed_dominant_and_traffic_needs_same_sources(tmp_path, monkeypatch):
    """The roofline names the kernel with the most time in the TIMED steps
    (not in the isolated frame), and a PMC summary taken on other sources is
    reported as stale, never used as `traffic`."""
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    wl = "w"
    pmc = {"workload": wl, "source_hash": "old", "kernels": {
        "void pt::k_shade_w3<16>": {"launches": 10, "hbm_bytes_per_launch": 2.0e10}}}
    (tmp_path / "profiles" / "r3_pmc_traffic.json").write_text(json.dumps(pmc))
    timed = dict(_timed(400.0, 500.0), shade_bytes=0)  # shading dominates the timed region (bytes not counted there)
    iso = _timed(350.0, 270.0)            # ... though tracing dominates the isolated frame, which counts the bytes
    out = bench.rooflines(timed, iso, wl, "c2", True, ("k_trace_lds", "k_shade_w3"), "new")
    roof = out["roofline"]
    assert roof["kernel"] == "k_shade_w3"
    assert roof["avg_launch_ms"] == 5.0
    assert roof["achieved"] == round(1e10 / 5e-3 / 1e9, 1) and roof["frac"] == round(roof["achieved"] / 8000.0, 5)
    assert roof["traffic"] is None
    assert "other sources" in out["roofline_kernels"]["k_shade"]["traffic_stale"]
    lv = out["roofline_kernels"]["k_trace"]["lds_view"]
    assert lv["peak"] == 150000.0
    pmc["source_hash"] = "new"
    (tmp_path / "profiles" / "r4_pmc_traffic.json").write_text(json.dumps(pmc))
    out = bench.rooflines(timed, iso, wl, "c2", True, ("k_trace_lds", "k_shade_w3"), "new")
    assert out["roofline"]["traffic"] == 2.0e10
    assert out["roofline"]["traffic_source"].endswith("r4_pmc_traffic.json")


@pytest.mark.gpu
def test_bench_parity_and_emulation_fields(tmp_path):
    """A short bench run (C2 scene at 256x144 @16 spp): the line carries the
    parity leg (GPU film of the cpu_baseline's tiles bit-identical to the
    oracle's) and the --emulate-ranks prediction."""
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--res", "256x144", "--spp", "16",
                        "--steps", "1", "--warmup", "0", "--cpu-seconds", "1", "--emulate-ranks", "2,4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["parity"]["bit_exact_pixels"] == 1.0 and line["parity"]["counters_equal"]
    assert set(line["emulated_scaling"]["ranks"]) == {"2", "4"}
    assert line["roofline"]["kernel"] in {v["kernel"] for v in line["roofline_kernels"].values()}
    assert line["source_hash"] == bench.source_hash()
