#!/bin/bash
# Kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes (separate runs) of one
# bench step on a given config, laid out for scripts/pmc_summary.py --out.
# usage: gpu_pmc_cfg.sh outdir [bench args]
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o="$R/gpurun_out/$1"; shift
mkdir -p "$o"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$o/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$o/prof.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$o/pmc_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$o/fetch.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$o/pmc_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$o/write.log" 2>&1 || exit $?
echo "pmc cfg $o done"
