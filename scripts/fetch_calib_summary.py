#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration (pbrt-v3-light-portals_amd/tools/fetch_calib.hip) into
profiles/<round>_fetch_calib.json.

Inputs under --out (scripts/gpu_r5.sh stage calib): calib.log (the tool's JSON lines: algorithmic bytes
per launch of each kernel), pmc_cfetch/cfetch_counter_collection.csv and pmc_cwrite/cwrite_counter_collection.csv
(separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes).  For every access class the factor is
    bytes per counted byte = algorithmic bytes / (counter KiB * 1024)
so HBM bytes = factor * counter bytes; MI355X_MICROARCH.md gives 2.0 for wide coalesced streaming reads.
"""
import argparse
import collections
import csv
import json
import os
import re


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    return d


def norm(name):
    return re.sub(r"\s+", "", name.replace("void ", ""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--round", default="r5")
    a = ap.parse_args()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tool = [json.loads(l) for l in open(os.path.join(a.out, "calib.log")) if l.startswith("{")]
    fetch = per_kernel(os.path.join(a.out, "pmc_cfetch", "cfetch_counter_collection.csv"))
    write = per_kernel(os.path.join(a.out, "pmc_cwrite", "cwrite_counter_collection.csv"))
    fetch = {norm(k): v for k, v in fetch.items()}
    write = {norm(k): v for k, v in write.items()}
    classes = {}
    for t in tool:
        rd = t["kernel"].startswith("k_rd")
        key = "%s_%dB_%s" % ("read" if rd else "write", t["width"], "random" if t["random"] else "coalesced")
        vals = (fetch if rd else write).get(norm(t["kernel"]))
        if not vals:
            continue
        counted = 1024.0 * sum(vals) / len(vals)
        classes[key] = {"kernel": t["kernel"], "algorithmic_bytes_per_launch": t["algorithmic_bytes_per_launch"],
                        "counter": "FETCH_SIZE" if rd else "WRITE_SIZE", "counted_bytes_per_launch": counted,
                        "bytes_per_counted_byte": round(t["algorithmic_bytes_per_launch"] / counted, 4) if counted else None,
                        "launches": len(vals), "avg_ms": t["avg_ms"], "GBs": t["GBs"]}
    out = {"method": "tools/fetch_calib: 64 M slots, 32-B records (2 GiB) and a 256-MiB SoA word array, zero-filled; "
                     "each kernel reads or writes W bytes per slot, slots in order or spread by i*0x9E3779B1 mod 2^26; "
                     "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes",
           "source_hash": open(os.path.join(a.out, "source_hash.txt")).read().strip()
           if os.path.exists(os.path.join(a.out, "source_hash.txt")) else None,
           "classes": classes}
    path = os.path.join(repo, "profiles", f"{a.round}_fetch_calib.json")
    json.dump(out, open(path, "w"), indent=1)
    for k, v in classes.items():
        print(f"{k:26s} bytes/counted={v['bytes_per_counted_byte']}  {v['GBs']} GB/s")


if __name__ == "__main__":
    main()
