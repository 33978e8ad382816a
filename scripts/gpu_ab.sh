#!/bin/bash
# A/B of kernel variants on the bench workload (after the parity tests).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
for lds in 1 0; do
  for sv in 0 3 4; do
    PT_TRACE_LDS=$lds PT_SHADE_VARIANT=$sv timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${lds}_${sv}.log 2>&1
    rc=$?
    echo "lds=$lds shade=$sv rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${lds}_${sv}.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" 2>/dev/null)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
