#!/bin/bash
# A/B of kernel variants on the bench workload (after the parity tests).
# usage: gpu_ab.sh "ENV=.. ENV=.." "ENV=.." ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$i.log 2>&1
  rc=$?
  echo "[$cfg] rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc;; esac
done
