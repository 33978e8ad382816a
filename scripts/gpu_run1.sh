#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ok() { case "$1" in 0|1) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
