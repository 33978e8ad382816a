#!/bin/bash
# GPU: all gpu tests, then a bench (default: config 5, the 10M-triangle atrium, at a
# reduced spp; BENCH_ARGS overrides), its kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
ARGS="${BENCH_ARGS:---config c5 --spp ${C5_SPP:-16}}"
ok() { case "$1" in 0) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --cpu-seconds 15 $ARGS > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_c5.log; ok $rc || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $ARGS > "$R/gpurun_out/prof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; ok $rc || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $ARGS > "$R/gpurun_out/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; ok $rc || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $ARGS > "$R/gpurun_out/pmc_write.log" 2>&1
rc=$?; echo "pmc write rc=$rc"
find "$R/gpurun_out" -name "*.csv" | head -20
exit $rc
