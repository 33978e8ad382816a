#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of one bench step with the
# library PT_LIB, summarised per kernel into gpurun_out/<tag>_pmc.txt.
# usage: PT_LIB=x.so gpu_pmc_lib.sh tag [bench args]
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
cd /tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/${tag}_fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$R/gpurun_out/${tag}_fetch.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/${tag}_write" -o write --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$R/gpurun_out/${tag}_write.log" 2>&1 || exit $?
echo "pmc $tag done"
