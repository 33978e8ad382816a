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
the bytes of wide reads, so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
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
    fetch = per_kernel(os.path.join(a.out, a.fetch_dir, "fetch_counter_collection.csv"))
    write = per_kernel(os.path.join(a.out, a.write_dir, "write_counter_collection.csv"))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        fb = 2.0 * 1024.0 * sum(f) / len(f)
        wb = 1024.0 * sum(w) / len(w)
        kernels[k] = {"launches": len(f), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                      "hbm_bytes_per_launch": fb + wb, **({"stats": stats[k]} if k in stats else {})}
    out = {"workload": a.workload, "source_hash": source_hash_of(a),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "bytes = 2*FETCH_SIZE[KiB]*1024 + WRITE_SIZE[KiB]*1024 (gfx950 FETCH_SIZE half-count)",
           "kernels": kernels}
    with open(os.path.join(prof, f"{a.round}_pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k:20s} launches={v['launches']:5d} hbm/launch={v['hbm_bytes_per_launch'] / 1e6:10.2f} MB")


if __name__ == "__main__":
    main()
