#!/bin/bash
# One bench line per environment setting (same bench args for all), e.g.
#   gpu_env_sweep.sh "--config c3h --spp 128" PT_HERO_WAVES=1 PT_HERO_WAVES=4
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
args="$1"; shift
for kv in "$@"; do
  env $kv timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > "gpurun_out/sweep_${kv//[^A-Za-z0-9_]/_}.log" 2>&1
  rc=$?
  echo "$kv rc=$rc $(tail -1 gpurun_out/sweep_${kv//[^A-Za-z0-9_]/_}.log | python3 -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); k=d.get("roofline_kernels",{}); print(d["value"], d["ms_per_step"], {n:(v["avg_launch_ms"],v.get("algorithmic_GBs")) for n,v in k.items()})
except Exception as e: print("parse error", e)')"
  case $rc in 0) ;; *) exit $rc;; esac
done
