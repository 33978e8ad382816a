#!/bin/bash
# All GPU tests, then bench A/B items (gpu_ab_cfg.sh) and config benches.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --maxfail=5 --timeout 250 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0) ;; *) exit $rc;; esac
i=0
for item in "$@"; do
  i=$((i+1))
  cfg="${item%%|*}"; rest="${item#*|}"; envs="${rest%%|*}"; args="${rest#*|}"
  env $envs timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --config $cfg $args > gpurun_out/r3b_$i.log 2>&1
  rc=$?
  echo "[$cfg $envs $args] rc=$rc $(python3 -c "
import json
d = json.loads(open('gpurun_out/r3b_$i.log').read().strip().splitlines()[-1])
k = d['roofline_kernels']
print(d['value'], d['ms_per_step'], 'shade', k.get('k_shade', {}).get('avg_launch_ms'), 'trace', k['k_trace']['avg_launch_ms'])
" 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc;; esac
done
