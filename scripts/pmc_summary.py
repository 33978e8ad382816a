#!/usr/bin/env python3
"""Summarise a rocprofv3 bench profile into profiles/ (committed evidence).

Inputs (written by scripts/gpu_run*.sh under gpurun_out/):
  prof/bench_kernel_stats.csv            --kernel-trace --stats pass
  pmc_fetch/fetch_counter_collection.csv --pmc FETCH_SIZE pass
  pmc_write/write_counter_collection.csv --pmc WRITE_SIZE pass
Outputs:
  profiles/<round>_kernel_stats.csv      copy of the stats summary
  profiles/<round>_pmc_traffic.json      per-kernel HBM bytes per launch

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are reported in KiB per dispatch; on gfx950 FETCH_SIZE counts half
the bytes of wide coalesced streaming reads.  Narrow per-lane gathers are
calibrated by tools/fetch_calib (profiles/r5_fetch_calib.json, --calib): a
random 4-, 12-, 16- or 32-B read is counted as the 64-B request the memory
side serves, i.e. FETCH_SIZE counts those bytes one for one.  So each kernel's
reads get the factor of its access class (CLASS below): 2.0 for the streaming
kernels, the calibrated gather factor (1.0) for the per-slot gathers of the
trace / shading / film kernels; fetch_bytes_streaming_x2 keeps the old reading
beside it.  WRITE_SIZE counts bytes one for one for streaming stores and 32 B
per partial-sector store (calibration), so writes are taken as counted.
"""
import argparse
import collections
import csv
import json
import os
import shutil


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return d


# access class of each kernel's reads (name prefix -> class)
CLASS = [("k_film_prep", "stream"), ("k_camera", "stream"), ("k_hero_init", "stream"), ("k_film_add", "stream"),
         ("k_shade", "gather"), ("k_trace", "gather"), ("k_film", "gather"), ("k_hero", "gather")]


def read_class(kernel):
    base = kernel.replace("void ", "").split("<")[0].split("::")[-1]
    for pre, c in CLASS:
        if base.startswith(pre):
            return c
    return "stream"


def read_factors(calib_path):
    """bytes per counted FETCH byte per class: streaming 2.0 (MI355X_MICROARCH.md, and the calibration's
    coalesced 32-B reads), gather = the calibrated random-read requests' bytes per counted byte."""
    f = {"stream": 2.0, "gather": 2.0, "source": "MI355X_MICROARCH.md (streaming x2 for every class)"}
    if calib_path and os.path.exists(calib_path):
        c = json.load(open(calib_path))["classes"]
        # a random W-byte read is served as a 64-B request; counted bytes / request = 64 -> DRAM bytes = counted
        # a random W-byte read is served as one 64-B request, counted as 64 B: DRAM bytes per counted byte =
        # 64 / (W / bytes_per_counted_byte), averaged over the calibrated widths
        f["gather"] = round(sum(64.0 / (float(k.split("_")[1][:-1]) / v["bytes_per_counted_byte"]) for k, v in c.items()
                                if k.startswith("read_") and k.endswith("_random")) /
                            max(1, sum(1 for k in c if k.startswith("read_") and k.endswith("_random"))), 4)
        if "read_32B_coalesced" in c:
            f["stream"] = round(c["read_32B_coalesced"]["bytes_per_counted_byte"], 4)
        f["source"] = os.path.relpath(calib_path, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return f


def source_hash_of(a):
    if a.source_hash:
        return a.source_hash
    f = os.path.join(a.out, "source_hash.txt")
    if os.path.exists(f):
        return open(f).read().strip()
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    return bench.source_hash()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out")
    ap.add_argument("--round", default="r1")
    ap.add_argument("--prof-dir", default="prof", help="subdirectory of --out with bench_kernel_stats.csv")
    ap.add_argument("--fetch-dir", default="pmc_fetch")
    ap.add_argument("--write-dir", default="pmc_write")
    ap.add_argument("--workload", required=True, help="bench config workload string the profile was taken on")
    ap.add_argument("--source-hash", default="", help="bench.py source_hash() of the tree profiled "
                    "(default: <out>/source_hash.txt, else this tree's)")
    ap.add_argument("--calib", default="", help="FETCH_SIZE calibration (profiles/r5_fetch_calib.json; "
                    "default: the newest profiles/r*_fetch_calib.json)")
    a = ap.parse_args()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(a.out, a.prof_dir, "bench_kernel_stats.csv"),
                os.path.join(prof, f"{a.round}_kernel_stats.csv"))
    stats = {}
    for r in csv.DictReader(open(os.path.join(a.out, a.prof_dir, "bench_kernel_stats.csv"))):
        stats[r["Name"].split("(")[0]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                          "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                          "percent": float(r["Percentage"])}
    calib = a.calib
    if not calib:
        import glob
        cands = sorted(glob.glob(os.path.join(prof, "r*_fetch_calib.json")))
        calib = cands[-1] if cands else ""
    factors = read_factors(calib)
    fetch = per_kernel(os.path.join(a.out, a.fetch_dir, "fetch_counter_collection.csv"))
    write = per_kernel(os.path.join(a.out, a.write_dir, "write_counter_collection.csv"))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        counted = 1024.0 * sum(f) / len(f)
        cls = read_class(k)
        fb = factors[cls] * counted
        wb = 1024.0 * sum(w) / len(w)
        kernels[k] = {"launches": len(f), "read_class": cls, "fetch_counted_bytes_per_launch": counted,
                      "fetch_bytes_per_launch": fb, "fetch_bytes_streaming_x2": 2.0 * counted,
                      "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb,
                      **({"stats": stats[k]} if k in stats else {})}
    out = {"workload": a.workload, "source_hash": source_hash_of(a),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "bytes = factor[read class] * FETCH_SIZE[KiB]*1024 + WRITE_SIZE[KiB]*1024",
           "read_factors": factors,
           "kernels": kernels}
    with open(os.path.join(prof, f"{a.round}_pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k:20s} launches={v['launches']:5d} hbm/launch={v['hbm_bytes_per_launch'] / 1e6:10.2f} MB")


if __name__ == "__main__":
    main()
