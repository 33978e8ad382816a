#!/usr/bin/env python3
"""Summarise the SQ counter passes of scripts/gpu_r4.sh (stage sq) into
profiles/<round>_sq_counters.json: per kernel, the counters summed over its
dispatches and the ratios the DESIGN quotes (share of wave cycles spent
waiting, instructions per wave by kind).

usage: sq_summary.py --out gpurun_out --round r2 --workload "<bench workload>"
"""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out")
ap.add_argument("--round", default="r2")
ap.add_argument("--workload", required=True)
ap.add_argument("--args", default="--spp 16", help="bench args the passes ran with")
ap.add_argument("--config", default="c2", help="bench --config the passes ran")
ap.add_argument("--glob", default="pmc_sq*", help="pass directories under --out")
ap.add_argument("--source-hash", default="", help="default: <out>/source_hash.txt, else this tree's")
a = ap.parse_args()

sums = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(a.out, a.glob, "**", "*counter_collection.csv"), recursive=True)):
    part = collections.defaultdict(lambda: collections.defaultdict(float))  # this pass's sums
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not ("k_shade" in k or "k_trace" in k or "k_film" in k or "k_camera" in k):
            continue
        part[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
    for k, c in part.items():  # a counter collected in several passes: the later pass's sum
        sums[k].update(c)

src = a.source_hash
if not src and os.path.exists(os.path.join(a.out, "source_hash.txt")):
    src = open(os.path.join(a.out, "source_hash.txt")).read().strip()
if not src:
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench
    src = bench.source_hash()
out = {"workload": a.workload, "config": a.config, "source_hash": src, "bench_args": a.args,
       "method": "rocprofv3 --pmc, passes of 8 SQ counters each (scripts/gpu_r6.sh stage sq); sums over dispatches; counters in two passes (SQ_WAVES, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU) keep the last pass's value",
       "kernels": {}}
for k, c in sums.items():
    w = c.get("SQ_WAVES", 0) or 1
    cyc = c.get("SQ_WAVE_CYCLES", 0) or 1
    e = {"dispatches": len(disp[k]), "counters": dict(c)}
    e["wait_any_share"] = c.get("SQ_WAIT_ANY", 0) / cyc
    e["wait_inst_any_share"] = c.get("SQ_WAIT_INST_ANY", 0) / cyc
    e["active_inst_any_share"] = c.get("SQ_ACTIVE_INST_ANY", 0) / cyc
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        # rocprofv3's VALUUtilization: active lanes per VALU instruction cycle, of 64
        e["valu_lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM"):
        if n in c:
            e[n.replace("SQ_INSTS_", "insts_per_wave_").lower()] = c[n] / w
    out["kernels"][k] = e
    print("%-34s waves=%-9d wait_any=%.2f active_inst=%.2f valu/wave=%.0f vmem_rd/wave=%.0f" % (
        k[-34:], w, e["wait_any_share"], e["active_inst_any_share"], e.get("insts_per_wave_valu", 0),
        e.get("insts_per_wave_vmem_rd", 0)))
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", f"{a.round}_sq_counters.json")
json.dump(out, open(dst, "w"), indent=1)
print("wrote", os.path.relpath(dst))
