#!/bin/bash
# Parity tests, then A/B of library builds on the C2 bench and the C5 bench.
# usage: [BENCH_SET='bench args;bench args'] gpu_ab2.sh "PT_LIB=a.so" "PT_LIB=b.so" ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_hero.py -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0) ;; *) exit $rc;; esac
i=0
for cfg in "$@"; do
  IFS=';' read -ra SETS <<< "${BENCH_SET:-;--config c5 --spp 16}"
  for bargs in "${SETS[@]}"; do
    i=$((i+1))
    env $cfg timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $bargs > gpurun_out/ab_$i.log 2>&1
    rc=$?
    echo "[$cfg $bargs] rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]); rk=d['roofline_kernels']; print(d['value'], d['ms_per_step'], {k: v['avg_launch_ms'] for k, v in rk.items()})" 2>/dev/null)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
