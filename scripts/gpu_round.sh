#!/bin/bash
# Round evidence on one GPU: all -m gpu tests, smoke, the default bench line,
# its rocprofv3 kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes
# (separate runs, per MI355X_MICROARCH.md), summarised by scripts/pmc_summary.py.
# usage: gpu_round.sh [bench args]   (e.g. --config c5 --spp 16)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
ok() { case "$1" in 0) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --maxfail=5 --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; ok $rc || exit $rc
fi
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --cpu-seconds 15 "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400; ok $rc || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$R/gpurun_out/prof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; ok $rc || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$R/gpurun_out/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; ok $rc || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$R/gpurun_out/pmc_write.log" 2>&1
rc=$?; echo "pmc write rc=$rc"
exit $rc
