#!/bin/bash
# Bench-only A/B of environment variants (no tests); prints Msamples/s, ms/step,
# isolated k_shade / k_trace avg launch ms.  BENCH_ARGS for the workload.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
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
