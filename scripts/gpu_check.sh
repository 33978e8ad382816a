#!/bin/bash
# GPU check: all gpu tests, smoke, c2 bench, kernel-trace stats of the bench.
# usage (via gpurun): bash scripts/gpu_check.sh [bench extra args]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
ok() { case "$1" in 0) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -q -m gpu --maxfail=10 -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-seconds 15 "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; ok $rc || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$R/gpurun_out/prof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 "$R/gpurun_out/prof_bench.log"; ok $rc || exit $rc
find "$R/gpurun_out/prof" -name "*stats*.csv"
exit 0
