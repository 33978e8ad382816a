#!/usr/bin/env python3
"""Per-frame split of a rocprofv3 kernel trace of `bench.py --steps 1
--warmup 0`: the bench renders the timed frame (two pipelines overlapping
batches) and then one frame with the batches one after the other, whose HIP
event times give the roofline's avg_launch_ms.  The stats summary averages
both frames; this splits each kernel's dispatches (in start order) into the
two frames so the isolated-frame average can be set beside the bench line.

usage: trace_split.py gpurun_out/prof/bench_kernel_trace.csv profiles/<round>_kernel_split.json
"""
import collections
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {"source": sys.argv[1], "note": __doc__.split("\n\n")[0].replace("\n", " "), "kernels": {}}
for k, d in per.items():
    if len(d) < 2 or not ("k_shade" in k or "k_trace" in k or "k_film" in k or "k_camera" in k):
        continue
    h = len(d) // 2
    out["kernels"][k] = {"dispatches": len(d), "timed_frame_avg_ms": sum(d[:h]) / h,
                         "isolated_frame_avg_ms": sum(d[h:]) / (len(d) - h), "all_avg_ms": sum(d) / len(d)}
    print("%-40s %3d  timed(overlapped) %.3f ms  isolated %.3f ms  all %.3f ms" % (
        k[-40:], len(d), out["kernels"][k]["timed_frame_avg_ms"], out["kernels"][k]["isolated_frame_avg_ms"],
        out["kernels"][k]["all_avg_ms"]))
json.dump(out, open(sys.argv[2], "w"), indent=1)
