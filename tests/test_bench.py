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
            "node_visits": 10 ** 9, "prim_tests": 10 ** 8, "shade_bytes": 10 ** 12,
            # the counting frame's reference counters (the binary traversal's visit order)
            "node_visits_ref": 10 ** 9, "prim_tests_ref": 10 ** 8, "trace_launches_counted": 100}


def test_roofline_kernel_is_isolated_dominant_and_traffic_needs_same_sources(tmp_path, monkeypatch):
    """The roofline names the kernel with the most time per frame in the
    ISOLATED frame (one pipeline: launch spans are kernel durations), not in
    the timed steps, where two pipelines overlap and a launch's span includes
    the co-running kernel (kept only as overlapped_span_ms); achieved / frac
    come from the isolated launch time.  A PMC summary taken on other sources
    is reported as stale, never used as `traffic`."""
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    wl = "w"
    pmc = {"workload": wl, "source_hash": "old", "kernels": {
        "void pt::k_shade_w3<16>": {"launches": 10, "hbm_bytes_per_launch": 2.0e10},
        "void pt::k_trace_pt<false, true, false>": {"launches": 10, "hbm_bytes_per_launch": 3.0e10}}}
    (tmp_path / "profiles" / "r3_pmc_traffic.json").write_text(json.dumps(pmc))
    timed = dict(_timed(400.0, 500.0), shade_bytes=0)  # shading dominates the overlapped timed spans ...
    iso = _timed(350.0, 270.0)            # ... tracing dominates the isolated frame
    # LDS-resident traversal dominant: bound lds/issue, the shading kernel's HBM fraction beside it
    out = bench.rooflines(timed, iso, wl, "c2", True, ("k_trace_lds", "k_shade_w3"), "new", ms_per_step=600.0)
    roof = out["roofline"]
    assert roof["kernel"] == "k_trace_lds" and roof["bound"] == "lds/issue"
    assert roof["avg_launch_ms"] == 3.5 and roof["per_frame_ms"] == 350.0 and roof["within_step"]
    alg = (32.0 * 10 ** 9 + 48.0 * 10 ** 8) / 100
    assert roof["achieved"] == round(alg / 3.5e-3 / 1e9, 1) and roof["peak"] == 150000.0
    assert roof["frac"] == round(roof["achieved"] / 150000.0, 5)
    assert roof["hbm_view"]["kernel"] == "k_shade_w3"
    assert roof["hbm_view"]["frac"] == round(round(1e10 / 2.7e-3 / 1e9, 1) / 8000.0, 5)
    assert out["roofline_kernels"]["k_shade"]["overlapped_span_ms"] == 5.0
    assert roof["traffic"] is None
    assert "other sources" in out["roofline_kernels"]["k_shade"]["traffic_stale"]
    # HBM-resident traversal dominant (C5): bound hbm from the isolated launch time
    out = bench.rooflines(timed, iso, wl, "c5", False, ("k_trace_pt", "k_shade"), "new")
    roof = out["roofline"]
    assert roof["kernel"] == "k_trace_pt" and roof["bound"] == "hbm"
    assert roof["frac"] == round(round(alg / 3.5e-3 / 1e9, 1) / 8000.0, 5)
    # shading dominant in the isolated frame
    out = bench.rooflines(timed, _timed(200.0, 270.0), wl, "c2", True, ("k_trace_lds", "k_shade_w3"), "new")
    assert out["roofline"]["kernel"] == "k_shade_w3" and out["roofline"]["bound"] == "hbm"
    assert out["roofline"]["achieved"] == round(1e10 / 2.7e-3 / 1e9, 1)
    pmc["source_hash"] = "new"
    (tmp_path / "profiles" / "r4_pmc_traffic.json").write_text(json.dumps(pmc))
    out = bench.rooflines(timed, _timed(200.0, 270.0), wl, "c2", True, ("k_trace_lds", "k_shade_w3"), "new")
    assert out["roofline"]["traffic"] == 2.0e10
    assert out["roofline"]["traffic_source"].endswith("r4_pmc_traffic.json")


def test_roofline_bound_check():
    """The dominant kernel's isolated time per frame may not exceed the step
    (round 4's line set a 632-ms overlapped span against a 597-ms step)."""
    timed, iso = _timed(400.0, 500.0), _timed(350.0, 270.0)
    ok = bench.rooflines(timed, iso, "w", "c2", True, ("k_trace_lds", "k_shade_w3"), "x", ms_per_step=340.0)
    assert ok["roofline"]["within_step"]  # 350 <= 1.05 * 340
    # beyond the step: reported on the line (within_step false + warning), the measurement is not thrown away
    bad = bench.rooflines(timed, iso, "w", "c2", True, ("k_trace_lds", "k_shade_w3"), "x", ms_per_step=300.0)
    assert not bad["roofline"]["within_step"] and "per frame > step" in bad["roofline"]["warning"]


def test_roofline_wide_traversal_view():
    """With the 4-wide traversal the algorithmic bytes stay the reference's
    (counting frame: 32 B per binary node visit + 48 B per primitive test)
    and the wide kernel's own LDS reads are reported beside them."""
    timed, iso = _timed(400.0, 500.0), _timed(350.0, 270.0)
    iso.update(wide_node_visits=3 * 10 ** 8, wide_prim_tests=10 ** 8, retraced_rays=10 ** 5, rays=10 ** 8)
    out = bench.rooflines(timed, iso, "w", "c2", True, ("k_trace_w", "k_shade_w3"), "x", ms_per_step=600.0)
    k = out["roofline_kernels"]["k_trace"]
    assert k["algorithmic_bytes_per_launch"] == round((32.0 * 10 ** 9 + 48.0 * 10 ** 8) / 100, 1)
    assert k["wide_view"]["bytes_per_launch"] == round((112.0 * 3 * 10 ** 8 + 48.0 * 10 ** 8) / 100, 1)
    assert k["wide_view"]["retraced_share"] == 0.001


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
