#!/bin/bash
# GPU parity tests only.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -q -m gpu -s -p no:cacheprovider --maxfail=8 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_gpu.log | tail -5
exit $rc
