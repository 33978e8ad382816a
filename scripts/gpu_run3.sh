#!/bin/bash
# GPU round: parity tests, smoke, bench, rocprofv3 kernel stats, PMC traffic passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
ok() { case "$1" in 0|1) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-seconds 15 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; ok $rc || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/prof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 "$R/gpurun_out/prof_bench.log"; ok $rc || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; tail -1 "$R/gpurun_out/pmc_fetch.log"; ok $rc || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_write.log" 2>&1
rc=$?; echo "pmc write rc=$rc"; tail -1 "$R/gpurun_out/pmc_write.log"
find "$R/gpurun_out" -name "*.csv" | head -20
exit 0
