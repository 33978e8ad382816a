#!/usr/bin/env python3
"""bench.py -- headline benchmark (BASELINE.json metric) for the MI355X-native
wavefront path tracer.

Workload (BASELINE.json configs[1], "config 2"): scenes/portal_cornell.pbrt --
closed Cornell interior lit by an aaplane emitter behind one axis-aligned
portal, PathIntegrator maxdepth 5, 1920x1080, Halton 256 spp, box filter,
portal strategy "portal".  Synthetic scene (no downloads).

A step = one full 1920x1080 x 256-spp frame.  With N ranks (one process per
GPU) the 16x16 tiles are dealt round-robin (rank r renders tiles t % N == r:
strong scaling, the same frame at every N, independent units, no data-path
collective); the device films are summed once per step onto rank 0 with one
RCCL ncclReduce issued by the library (pt_render_frame_dist, the only
collective, inside the timed region).  --shard samples is the opt-in weak
scaling mode (rank r renders sample indices [r*spp, (r+1)*spp)).

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "pbrt-v3-light-portals_amd")
sys.path.insert(0, PKG)

METRIC = "Msamples/sec + Mrays/sec, 1920x1080 path integrator @256spp, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
LDS_B128_PEAK_GBS = 150000.0  # ds_read_b64/b128 aggregate, every CU streaming (MI355X_MICROARCH.md LDS section)
# BASELINE.json configs this bench can run: scene file, workload label
CONFIGS = {
    "c2": ("portal_cornell.pbrt", "portal Cornell (config 2)", "path maxdepth 5",
           "synthetic (scenes/portal_cornell.pbrt, procedural Cornell + portal; Halton sampler)"),
    "c3": ("cornell_dielectric.pbrt", "cornell dielectric (config 3)", "path maxdepth 5",
           "reference scenes/cornell_dielectric.pbrt (spectral params reduced to RGB) with Integrator path; file spp 1024"),
    "c3h": ("cornell_dielectric_hero.pbrt", "cornell dielectric as written (config 3)", "hero_path_mis",
            "reference scenes/cornell_dielectric.pbrt as written (SampledSpectrum, Integrator hero_path_mis; file spp 1024)"),
    "c4": ("portal_room.pbrt", "portal room (config 4)", "path maxdepth 8",
           "synthetic (scenes/portal_room.pbrt from scripts/make_portal_room.py: room + 4 portals + sky; Halton)"),
    "c5": ("killeroo_atrium.pbrt", "killeroo atrium 10M tris (config 5)", "path maxdepth 5",
           "synthetic (scenes/killeroo_atrium.pbrt from scripts/make_atrium.py: 300 loop-subdivided killeroos, "
           "9.98M triangles, skylight portal; Halton)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="c2: the headline workload (default); c3: cornell_dielectric (BASELINE configs[2]); "
                         "c4: portal room (BASELINE configs[3]); c5: 10M-triangle atrium (BASELINE configs[4])")
    ap.add_argument("--scene", default="", help="override the config's scene file")
    ap.add_argument("--spp", type=int, default=0, help="override samples per pixel per rank (0 = scene)")
    ap.add_argument("--res", default="", help="override WxH")
    ap.add_argument("--strategy", default="", help="override portal strategy")
    ap.add_argument("--batch-slots", type=int, default=0)
    ap.add_argument("--shard", default="tiles", help="tiles (strong, default) | samples-split (strong) | samples (weak)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-parity", action="store_true", help="skip the GPU-vs-oracle film check of the cpu_baseline tiles")
    ap.add_argument("--emulate-ranks", default="",
                    help="comma-separated rank counts (e.g. 2,4,8): time every rank's tile shard on this GPU, one "
                         "after the other, and predict the strong-scaling efficiency (single process only)")
    ap.add_argument("--print-source-hash", action="store_true", help="print source_hash() and exit")
    return ap.parse_args()


def scene_text(args) -> str:
    import re
    txt = open(args.scene or os.path.join(REPO, "scenes", CONFIGS[args.config][0])).read()
    if args.res:
        w, h = (int(v) for v in args.res.lower().split("x"))
        txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [%d]' % w, txt)
        txt = re.sub(r'"integer yresolution" \[\d+\]', '"integer yresolution" [%d]' % h, txt)
    if args.spp:
        txt = re.sub(r'"integer pixelsamples" \[\d+\]', '"integer pixelsamples" [%d]' % args.spp, txt)
    if args.strategy:
        txt = re.sub(r'"string strategy" "\w+"', '"string strategy" "%s"' % args.strategy, txt)
    # the copy is written to TMPDIR: keep relative Includes resolving against scenes/
    sdir = os.path.dirname(os.path.abspath(args.scene)) if args.scene else os.path.join(REPO, "scenes")
    txt = re.sub(r'Include "(?!/)([^"]+)"', lambda m: 'Include "%s/%s"' % (sdir, m.group(1)), txt)
    return txt


# The reference itself, timed by the survey in this container (SURVEY.md §6 /
# §8(d) [probe]): built from its sources with logging / EXR shims outside the
# repo, 8 threads on the draft C2 scene.  Reported beside the port's own rate.
REFERENCE_PROBE = {"value": 0.684, "unit": "Msamples/s", "cores": 8,
                   "source": "SURVEY.md §8(d) [probe]: reference pbrt-v3-light-portals, --nthreads 8, "
                             "draft C2 scene at 480x270 @16 spp scaled to the frame (not re-run here)"}


def _progress(msg: str) -> None:
    """A line on stderr between phases (long CPU phases -- a 10 M-triangle scene's load and the oracle's
    BVH build -- would otherwise leave a GPU job silent for minutes)."""
    print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def _heartbeat(period: float = 30.0) -> None:
    """A daemon thread that prints a line on stderr every `period` seconds: a 10 M-triangle scene's first
    frame (host subdivision + SAH build inside the library call) runs for minutes without returning."""
    import threading

    def beat():
        while True:
            time.sleep(period)
            _progress("still running")

    threading.Thread(target=beat, daemon=True).start()


# Frames of more than this many samples per pixel (C5 as written: 4096) take the CPU baseline, the parity
# check and the isolated / counting frames on the first CPU_SPP_CAP samples of every pixel (a bounded sample of
# the same frame: Halton indices [0, cap), HaltonSampler::StartPixelSample order) -- a full-spp CPU tile alone
# would run for minutes
CPU_SPP_CAP = 1024
CPU_SPP_SAMPLE = 64
ISO_SPP_SAMPLE = 16


def cpu_baseline(scene_path: str, seconds: float, hs=None, spp_cap: int = 0):
    """Reference CPU path restated in C (oracle/, 'port'), timed on this host's
    cores on a bounded sample of the same frame: the 16x16 tiles t with
    t % stride == 0, spread over the whole image (stride sized so the timed
    run takes about `seconds`), all samples of each pixel, or its first
    `spp_cap` (> 0) for the frames above CPU_SPP_CAP spp."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    import ptgpu
    if hs is None:
        hs = ptgpu.HostScene(scene_path)
    # Every core this process may run on, up to the box's declared CPU share
    # (OMP_NUM_THREADS: the GPU box gives one GPU's job 16 of the host's CPUs,
    # os.cpu_count() reports the whole machine)
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(affinity, share) if share > 0 else affinity)
    w, h = hs.film_size()
    ntiles = ((w + 15) // 16) * ((h + 15) // 16)
    stride = max(1, ntiles // (2 * threads))
    def oracle_tiles(stride_):
        if spp_cap > 0:
            return pyoracle.render_range(hs.desc, 0, spp_cap, nthreads=threads, tile_offset=0, tile_stride=stride_)
        return pyoracle.render_accum(hs.desc, nthreads=threads, tile_offset=0, tile_stride=stride_)

    _progress(f"cpu baseline: calibration run (tile stride {stride}, {threads} threads)")
    t0 = time.perf_counter()
    _, st = oracle_tiles(stride)
    dt = time.perf_counter() - t0
    per_tile = st["samples"] / max(1, (ntiles + stride - 1) // stride)
    want = max(2 * threads, min(ntiles, st["samples"] / dt * seconds / per_tile))
    stride = max(1, int(ntiles // want))
    _progress(f"cpu baseline: timed run (tile stride {stride})")
    t0 = time.perf_counter()
    film, st = oracle_tiles(stride)
    dt = time.perf_counter() - t0
    rate = st["samples"] / dt / 1e6
    host = os.cpu_count() or threads
    return {"value": round(rate, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "host_cpus": host, "affinity_cpus": affinity, "cpu_share": share or None,
            "threads_note": (f"timed on {threads} threads: the {affinity} CPUs in this process's affinity"
                             + (f", capped at the box's declared CPU share OMP_NUM_THREADS={share}" if share else "")
                             + f"; the host has {host} CPUs"),
            "all_host_cpus_linear_estimate": round(rate / threads * host, 3),
            "sample": f"every {stride}th 16x16 tile of the same frame (tiles t % {stride} == 0 over the whole image) "
                      + (f"at the first {spp_cap} samples of each pixel" if spp_cap > 0 else "at the scene's spp")
                      + f" ({st['samples']} samples, {dt:.1f} s, {threads} threads; oracle/pt_oracle.c)",
            "mrays_per_s": round((st["closest_rays"] + st["shadow_rays"]) / dt / 1e6, 3),
            "per_thread": round(rate / threads, 4),
            "reference_probe": dict(REFERENCE_PROBE, per_thread=round(REFERENCE_PROBE["value"] / 8, 4))}, \
        (stride, film, st)


def source_hash() -> str:
    """Hash of the sources libptgpu.so is built from (csrc/, include/pt.h, the
    Makefile): a profile summary records the hash of the tree it was taken on,
    and the bench uses its counters only when they match (no git on the GPU
    box, so no commit lookup)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(PKG, "csrc")
    files = [os.path.join(csrc, f) for f in sorted(os.listdir(csrc))]
    files += [os.path.join(REPO, "include", "pt.h"), os.path.join(PKG, "Makefile")]
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.basename(f).encode())
            h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def _profile_files(pattern: str):
    import glob
    import re
    files = glob.glob(os.path.join(REPO, "profiles", pattern))
    files.sort(key=lambda f: (int(re.search(r"r(\d+)_", os.path.basename(f)).group(1)), os.path.getmtime(f)))
    return list(reversed(files))


def _kernel_match(name: str, kernel: str) -> bool:
    """rocprof kernel names look like 'void pt::k_shade_w3<16>': match the
    exact kernel (k_shade must not match k_shade_w3)."""
    base = name.replace("void ", "").split("<")[0].split("::")[-1]
    return base == kernel


def pmc_traffic(workload: str, kernel: str, src: str):
    """HBM bytes per launch of `kernel` (the variant with the most launches)
    from the newest committed PMC summary (profiles/r*_pmc_traffic.json, made
    by scripts/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this bench on the same workload) taken on the same
    sources (source_hash).  Returns (bytes, file, stale_file): a summary of
    other sources is never used, only named in stale_file."""
    stale = None
    for f in _profile_files("r*_pmc_traffic.json"):
        d = json.load(open(f))
        if d.get("workload") != workload:
            continue
        ks = [(v["launches"], v["hbm_bytes_per_launch"]) for k, v in d.get("kernels", {}).items()
              if _kernel_match(k, kernel)]
        if not ks:
            continue
        if d.get("source_hash") != src:
            stale = stale or os.path.relpath(f, REPO)
            continue
        return max(ks)[1], os.path.relpath(f, REPO), None
    return None, None, stale


def sq_issue_view(config: str, kernel: str, src: str):
    """Issue / wait shares of `kernel` from the newest SQ-counter summary of
    this config taken on the same sources (profiles/r*_sq_counters.json,
    scripts/sq_summary.py), or None."""
    for f in _profile_files("r*_sq_counters.json"):
        d = json.load(open(f))
        if d.get("source_hash") != src or d.get("config") != config:
            continue
        for k, v in d.get("kernels", {}).items():
            if _kernel_match(k, kernel):
                keys = ("active_inst_any_share", "wait_any_share", "wait_inst_any_share", "insts_per_wave_valu",
                        "insts_per_wave_salu", "insts_per_wave_lds")
                return dict({x: round(v[x], 4) for x in keys if x in v}, source=os.path.relpath(f, REPO),
                            bench_args=d.get("bench_args"))
    return None


def rooflines(timed: dict, iso: dict, workload: str, config: str, lds_scene: bool, names: tuple, src: str,
              ms_per_step: float | None = None) -> dict:
    """roofline = the kernel with the most time per frame in the ISOLATED
    frame (pt_set_pipelines(1): the batches one after the other, so a launch's
    HIP-event span is that kernel's own duration -- what a rocprofv3
    --kernel-trace --stats pass at PT_PIPES=1 averages).  `achieved` and `frac`
    come from that isolated per-launch time.  In the timed steps two pipelines
    overlap one batch's trace with another's shading, so a timed launch span
    includes the co-running kernel: those spans are reported only as
    `overlapped_span_ms`.  Both kernels' figures are under roofline_kernels.

    * traversal: algorithmic bytes per SURVEY 8(d), 32 B per LinearBVHNode
      visit (bvh.cpp:95-104) + 48 B per primitive test (triangle.cpp:189-425),
      counted on the device.  For a scene whose BVH sits in LDS (C2-C4) those
      are LDS reads: bound "lds/issue", set against the ds_read_b128 aggregate
      (MI355X_MICROARCH LDS table, ~150 TB/s) with the SQ issue shares beside
      it, and the shading kernel's HBM fraction as the line's `hbm_view`.
    * shading: the path-state bytes each path step must read and write (the
      state PathIntegrator::Li carries between vertices + queue entries),
      counted on the device per step (kernels.hip shade_path) in the extra
      frame (pt_set_count_bytes).

    With ms_per_step given, the dominant kernel's isolated time per frame
    should not exceed the step (5 % tolerance for clock drift between the two
    measurements): otherwise the line says within_step false with a warning
    (raising threw the whole measurement away)."""
    trace_name, shade_name = names
    ks = {}
    # algorithmic bytes per launch: the reference's node visits / primitive tests of one frame, counted by the
    # counting frame (pt_set_count_bytes: the binary traversal in the reference's visit order, the same batches,
    # bounces and launches) -- also when the timed frames traverse the 4-wide BVH (k_trace_w), which does the
    # same work in fewer, wider steps; the shading kernel's count from the same frame
    parts = [("k_trace", trace_name, "trace", (32.0 * iso["node_visits_ref"] + 48.0 * iso["prim_tests_ref"]) /
              max(1, iso["trace_launches_counted"]))]
    if iso["shade_bytes"] > 0:
        parts.append(("k_shade", shade_name, "shade",
                      float(iso["shade_bytes"]) / max(1, iso.get("shade_launches_counted", iso["shade_launches"]))))
    for key, kname, p, alg in parts:
        il = max(1, iso[p + "_launches"])
        avg = iso[p + "_ms"] / il  # isolated: the kernel's own duration per launch
        span = timed[p + "_ms"] / max(1, timed[p + "_launches"])
        trf, trf_src, stale = pmc_traffic(workload, kname, src)
        e = {"kernel": kname, "launches_per_frame": iso[p + "_launches"], "avg_launch_ms": round(avg, 4),
             "per_frame_ms": round(iso[p + "_ms"], 3),
             "overlapped_span_ms": round(span, 4),
             "algorithmic_bytes_per_launch": round(alg, 1),
             "algorithmic_GBs": round(alg / (avg * 1e-3) / 1e9, 1) if avg > 0 else 0.0,
             "data": ("LDS (BVH + primitives staged per block)" if (p == "trace" and lds_scene) else
                      ("HBM (path state)" if p == "shade" else "HBM")),
             "hbm_traffic_per_launch": round(trf, 1) if trf is not None else None,
             "hbm_GBs": round(trf / (avg * 1e-3) / 1e9, 1) if (trf is not None and avg > 0) else None,
             "traffic_source": trf_src}
        if trf is not None:
            e["traffic_over_algorithmic"] = round(trf / alg, 3) if alg > 0 else None
        if stale:
            e["traffic_stale"] = stale + " (taken on other sources: not used)"
        if p == "trace" and iso.get("wide_node_visits"):
            nb = 128.0 if iso.get("wide_hbm") else 112.0  # one 128-B line per node from HBM, 112 B in LDS
            wb = (nb * iso["wide_node_visits"] + 48.0 * iso["wide_prim_tests"]) / il
            e["wide_view"] = {"bytes_per_launch": round(wb, 1), "GBs": round(wb / (avg * 1e-3) / 1e9, 1),
                              "retraced_share": round(iso["retraced_rays"] / max(1, iso["rays"]), 6),
                              "wide_nodes_per_ray": round(iso["wide_node_visits"] / max(1, iso["rays"]), 4),
                              "prim_tests_per_ray": round(iso["wide_prim_tests"] / max(1, iso["rays"]), 4),
                              "ref_nodes_per_ray": round(iso["node_visits_ref"] / max(1, iso["rays"]), 4),
                              "ref_prim_tests_per_ray": round(iso["prim_tests_ref"] / max(1, iso["rays"]), 4),
                              "note": "k_trace_w's own reads (112 B per 4-wide node from LDS, 128 from HBM; 48 B per "
                                      "primitive test) "
                                      "and the share of rays it handed back to the binary kernel; the launch time "
                                      "includes that retrace launch"}
        if p == "trace" and lds_scene:
            e["lds_view"] = {"achieved": e["algorithmic_GBs"], "peak": LDS_B128_PEAK_GBS, "unit": "GB/s",
                             "frac": round(e["algorithmic_GBs"] / LDS_B128_PEAK_GBS, 5),
                             "note": "SURVEY 8(d) bytes read from LDS vs the ds_read_b128 aggregate"}
            iv = sq_issue_view(config, kname, src)
            if iv:
                e["issue_view"] = iv
        else:
            e["hbm_view"] = {"achieved": e["algorithmic_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(e["algorithmic_GBs"] / HBM_PEAK_GBS, 5)}
        ks[key] = e
    dom = max(ks, key=lambda k: ks[k]["per_frame_ms"])
    k = ks[dom]
    on_chip = dom == "k_trace" and lds_scene
    if on_chip:
        roof = dict(bound="lds/issue", achieved=k["algorithmic_GBs"], peak=LDS_B128_PEAK_GBS, unit="GB/s",
                    frac=k["lds_view"]["frac"])
        if "issue_view" in k:
            roof["issue_share"] = k["issue_view"].get("active_inst_any_share")
            roof["wait_share"] = k["issue_view"].get("wait_any_share")
        other = ks.get("k_shade")
        if other is not None:
            roof["hbm_view"] = dict(other["hbm_view"], kernel=other["kernel"],
                                    note="the shading kernel (path state in HBM) against the HBM peak")
        roof["note"] = ("dominant kernel reads its SURVEY 8(d) bytes from LDS (scene staged per block): set against "
                        "the ds_read_b128 aggregate; it is bound by instruction issue and LDS latency "
                        "(issue_share / wait_share: SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY per wave cycle)")
    else:
        roof = dict(bound="hbm", achieved=k["algorithmic_GBs"], peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(k["algorithmic_GBs"] / HBM_PEAK_GBS, 5))
    roof.update({"traffic": k["hbm_traffic_per_launch"],
                 "traffic_unit": "HBM bytes per launch: rocprofv3 FETCH_SIZE x 0.9963 for per-slot gather kernels / "
                                 "x 2.0 for streaming kernels (profiles/r5_fetch_calib.json) + WRITE_SIZE, separate "
                                 "--pmc passes on the same sources",
                 "traffic_source": k["traffic_source"], "kernel": k["kernel"],
                 "algorithmic_bytes_per_launch": k["algorithmic_bytes_per_launch"], "avg_launch_ms": k["avg_launch_ms"],
                 "per_frame_ms": k["per_frame_ms"],
                 "dominant_by": "kernel time per frame in the isolated frame (one pipeline: launch spans are kernel "
                                "durations)",
                 "recipe": "achieved = algorithmic_bytes_per_launch / avg_launch_ms (HIP events on the launch stream, "
                           "isolated frame; = rocprofv3 --stats average at PT_PIPES=1); frac = achieved / peak"})
    if ms_per_step is not None:
        roof["ms_per_step"] = ms_per_step
        roof["within_step"] = k["per_frame_ms"] <= 1.05 * ms_per_step
        if not roof["within_step"]:  # reported, not raised: the measurement line is still printed
            roof["warning"] = f"{k['kernel']}: {k['per_frame_ms']} ms per frame > step {ms_per_step} ms"
    return {"roofline": roof, "roofline_kernels": ks}


def parity_check(sc, hs, stride: int, ref_acc, ref_st: dict, spp_cap: int = 0) -> dict:
    """The GPU film of the tiles t % stride == 0 (the cpu_baseline's sample of
    the same frame), rendered with the production batch size and pipelines,
    against the oracle's film of the same tiles: bit-exact pixels of the film
    (XYZ + weight, Film::Pixel), RMSE of the resolved image, and the
    reference's ray / node / primitive counters (integrator.cpp:526-637)."""
    import numpy as np
    def tiles():  # the same tiles (and sample range) as the cpu_baseline leg
        return sc.render_range(0, spp_cap, 0, stride) if spp_cap > 0 else sc.render_accum(0, stride)

    got, gst = tiles()
    # the counting frame's traversal (binary, the reference's visit order) for the node / primitive counters,
    # which the 4-wide k_trace_w does not reproduce; its film must be bit-exact too
    sc.set_count_bytes(True)
    got_c, gst_c = tiles()
    sc.set_count_bytes(False)
    same_c = bool(np.array_equal(got_c.view(np.uint32), ref_acc.view(np.uint32)))
    same = np.all(got.view(np.uint32) == ref_acc.view(np.uint32), axis=2)
    touched = np.any(ref_acc != 0, axis=2) | np.any(got != 0, axis=2)
    a = sc.resolve(got).astype(np.float64)
    b = sc.resolve(ref_acc).astype(np.float64)
    rmse = float(np.sqrt(np.mean((a - b) ** 2)))
    keys = ("samples", "closest_rays", "shadow_rays")
    order_keys = ("node_visits", "prim_tests")
    return {"tiles": f"t % {stride} == 0" + (f", samples [0, {spp_cap})" if spp_cap > 0 else ""),
            "samples": int(gst["samples"]),
            "bit_exact_pixels": round(float(np.mean(same)), 6),
            "bit_exact_rendered_pixels": round(float(np.mean(same[touched])), 6) if touched.any() else None,
            "rendered_pixels": int(touched.sum()), "rmse": rmse,
            "counters_equal": all(int(gst[k]) == int(ref_st[k]) for k in keys) and
                              all(int(gst_c[k]) == int(ref_st[k]) for k in keys + order_keys),
            "trace_wide": int(gst["trace_wide"]), "retraced_rays": int(gst["retraced_rays"]),
            "counting_frame_bit_exact": same_c,
            "batch_slots": int(sc.query("batch_slots")) or None, "pipelines": int(sc.query("pipelines")),
            "oracle": "oracle/pt_oracle.c render_accum of the same tiles"}


def emulated_scaling(rank_ms: dict, frame_ms: float, frame_samples: float) -> dict:
    """Strong-scaling prediction on one GPU (--emulate-ranks): rank_ms[N] is
    the device time of every rank's shard (tiles t % N == r) rendered one
    after the other; a step at N ranks takes the slowest shard (plus the
    film reduce, not included).  efficiency = (frame_ms / N) / max shard."""
    out = {}
    for n, times in sorted(rank_ms.items()):
        mx = max(times)
        out[str(n)] = {"per_rank_ms": [round(t, 2) for t in times], "max_ms": round(mx, 2),
                       "mean_ms": round(sum(times) / len(times), 2),
                       "imbalance": round(mx / (sum(times) / len(times)), 4),
                       "predicted_msamples_per_s": round(frame_samples / (mx * 1e-3) / 1e6, 2),
                       "predicted_efficiency": round(frame_ms / n / mx, 4)}
    return {"frame_ms_1gpu": round(frame_ms, 2), "excludes": "the per-step ncclReduce of the film", "ranks": out}


def main():
    args = parse()
    if args.print_source_hash:
        print(source_hash())
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import ptgpu
    import shard as shardmod

    tmpdir = os.environ.get("TMPDIR", "/tmp")
    spath = os.path.join(tmpdir, f"bench_scene_{os.getpid()}.pbrt")
    with open(spath, "w") as f:
        f.write(scene_text(args))
    _heartbeat()
    _progress(f"loading {args.config}")
    hs = ptgpu.HostScene(spath)
    sc = ptgpu.Scene(hs, device=local, batch_slots=args.batch_slots or None)
    _progress("scene on the device; warmup")
    w, h = sc.film_size()
    lds_scene = sc.query("trace_lds_bytes") > 0  # the library stages this BVH in LDS (PT_TRACE_LDS honoured)
    names = sc.kernel_names()
    import re
    spp = int(re.search(r'"integer pixelsamples" \[(\d+)\]', open(spath).read()).group(1))
    accum = torch.zeros((h, w, 4), dtype=torch.float32, device=f"cuda:{local}")
    stream = torch.cuda.current_stream().cuda_stream
    my = shardmod.plan(rank, world, spp, args.shard)
    render = shardmod.device_renderer(sc, accum.data_ptr(), stream)
    comm = None
    if world > 1:  # the library's own RCCL communicator (id handed over by torch.distributed)
        uid = [ptgpu.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = ptgpu.Comm(world, rank, uid[0])

    def step():
        if comm is not None and args.shard == "tiles":
            return comm.render_frame(sc, accum.data_ptr(), stream)
        return shardmod.render_frame(my, render, accum,
                                     (lambda a: comm.reduce(sc, a.data_ptr(), 0, stream)) if comm else None)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _progress(f"timed region: {args.steps} steps")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agg = {"samples": 0, "closest_rays": 0, "shadow_rays": 0, "node_visits": 0, "prim_tests": 0, "trace_ms": 0.0,
           "trace_launches": 0, "shade_ms": 0.0, "shade_launches": 0, "shade_bytes": 0, "render_ms": 0.0,
           "reduce_ms": 0.0}
    for _ in range(args.steps):
        st = step()
        for k in agg:
            agg[k] += st[k]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        tot = torch.tensor([agg["samples"], agg["closest_rays"] + agg["shadow_rays"]], dtype=torch.float64,
                           device=f"cuda:{local}")
        dist.all_reduce(tot)
        total_samples, total_rays = float(tot[0]), float(tot[1])
    else:
        total_samples, total_rays = float(agg["samples"]), float(agg["closest_rays"] + agg["shadow_rays"])
    # every rank's own render time and film-reduce time per step (max / min on rank 0)
    rank_times = shardmod.gather_rank_times(agg["render_ms"] / args.steps, agg["reduce_ms"] / args.steps, world,
                                            device=f"cuda:{local}")

    # One more frame with the batches run one after the other
    # (pt_set_pipelines(1)): per-launch times of each kernel alone, reported
    # beside the timed region's (where two pipelines overlap one batch's trace
    # with another's shading).  This rank's shard, no collective.
    iso = {"trace_ms": 0.0, "trace_launches": 0, "shade_ms": 0.0, "shade_launches": 0, "shade_bytes": 0,
           "node_visits": 0, "prim_tests": 0, "wide_node_visits": 0, "wide_prim_tests": 0, "retraced_rays": 0}
    _progress("isolated and byte-counting frames")
    # above CPU_SPP_CAP spp (C5 as written, 4096) both extra frames render the first ISO_SPP_SAMPLE samples of
    # every pixel: per-launch figures from the same batches, bounces and launches in both
    import dataclasses
    iso_shard = my if spp <= CPU_SPP_CAP else dataclasses.replace(
        my, sample_end=min(my.sample_end, my.sample_begin + ISO_SPP_SAMPLE))
    pipes = sc.query("pipelines")
    sc.set_pipelines(1)
    accum.zero_()
    st = render(iso_shard)
    torch.cuda.synchronize()
    sc.set_pipelines(pipes)
    for k in iso:
        iso[k] = st[k]
    iso["rays"] = st["closest_rays"] + st["shadow_rays"]
    iso["wide_hbm"] = sc.query("trace_kernel") == 7
    # and one frame with the shading build that also counts its algorithmic path-state bytes (one more
    # register: a separate instantiation, pt_set_count_bytes; the same batches, bounces and launches)
    sc.set_count_bytes(True)
    accum.zero_()
    st = render(iso_shard)
    torch.cuda.synchronize()
    sc.set_count_bytes(False)
    iso["shade_bytes"], iso["shade_launches_counted"] = st["shade_bytes"], st["shade_launches"]
    iso["node_visits_ref"], iso["prim_tests_ref"] = st["node_visits"], st["prim_tests"]
    iso["trace_launches_counted"] = st["trace_launches"]
    emul = None
    if args.emulate_ranks and world == 1:
        # every rank's tile shard at N ranks, one after the other, each timed like a step
        rank_ms = {}
        for n in sorted({int(v) for v in args.emulate_ranks.split(",") if v.strip()}):
            rank_ms[n] = []
            for r_ in range(n):
                accum.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                render(shardmod.plan(r_, n, spp, "tiles"))
                torch.cuda.synchronize()
                rank_ms[n].append((time.perf_counter() - t0) * 1e3)
        emul = emulated_scaling(rank_ms, dt / args.steps * 1e3, total_samples / args.steps)

    if rank == 0:
        cname, cdepth, cdata = CONFIGS[args.config][1:]
        workload = (f"{cname} {w}x{h} @{spp}spp{'/rank' if args.shard == 'samples' else ''}, "
                    f"{cdepth}, {args.shard}-sharded")
        out = {
            "metric": METRIC,
            "value": round(total_samples / dt / 1e6, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": shardmod.scaling(args.shard),
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"{cdata}; rendered at {spp} spp",
            "config": {"workload": workload, "resolution": [w, h],
                       "frame_spp": shardmod.frame_samples(spp, world, args.shard),
                       "parallelism": f"{args.shard} x{world}"},
            "mrays_per_s": round(total_rays / dt / 1e6, 2),
            "rays_per_sample": round(total_rays / max(1.0, total_samples), 3),
            "rank_times": rank_times,
        }
        src = source_hash()
        out["source_hash"] = src
        out.update(rooflines(agg, iso, workload, args.config, lds_scene, names, src,
                             ms_per_step=round(dt / args.steps * 1e3, 2)))
        out["isolated_frame_spp"] = iso_shard.samples_per_pixel
        if world == 1 and not args.no_cpu_baseline:
            cap = CPU_SPP_SAMPLE if spp > CPU_SPP_CAP else 0
            out["cpu_baseline"], (stride, ref_acc, ref_st) = cpu_baseline(spath, args.cpu_seconds, hs, cap)
            if not args.no_parity:
                _progress("parity: the sampled tiles on the GPU")
                out["parity"] = parity_check(sc, hs, stride, ref_acc, ref_st, cap)
        if emul is not None:
            out["emulated_scaling"] = emul
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()
    try:
        os.remove(spath)
    except OSError:
        pass


if __name__ == "__main__":
    main()
