#!/bin/bash
# Parity tests, then an A/B of environment variants on a bench workload.
# usage: BENCH_ARGS="--config c2" [SKIP_TESTS=1] gpu_ab3.sh "ENV=.." "ENV=.." ...
# prints per variant: Msamples/s, ms/step, isolated k_shade / k_trace avg launch ms
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --maxfail=5 --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  case $rc in 0) ;; *) exit $rc;; esac
fi
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_$i.log 2>&1
  rc=$?
  echo "[$cfg] rc=$rc $(python3 -c "
import json
d = json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1])
k = d['roofline_kernels']
print(d['value'], d['ms_per_step'], 'shade', k.get('k_shade', {}).get('avg_launch_ms'), 'trace', k['k_trace']['avg_launch_ms'])
" 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc;; esac
done
