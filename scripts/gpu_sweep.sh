#!/bin/bash
# Short C2 bench per value of an environment knob.  usage: bash scripts/gpu_sweep.sh VAR "v1 v2 ..." [bench args]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VAR=$1; VALS=$2; shift 2
for v in $VALS; do
  env "$VAR=$v" timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/sweep_$v.log 2>&1
  rc=$?; echo "$VAR=$v rc=$rc $(tail -1 gpurun_out/sweep_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' 2>&1)"
  [ $rc = 0 ] || exit $rc
done
