#!/bin/bash
# PC sampling (host trap, time-based) of a short bench run on the line-table
# build libptgpu_g.so (make EXTRA=-gline-tables-only B=build_g LIB=libptgpu_g.so).
# usage: bash scripts/gpu_pcsamp.sh [bench args]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
ARGS="${@:---spp 16}"
cd /tmp
PT_LIB=libptgpu_g.so timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1000 \
  -d "$R/gpurun_out/pcs" -o pcs --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $ARGS > "$R/gpurun_out/pcs.log" 2>&1
rc=$?; echo "pcsamp rc=$rc"; tail -3 "$R/gpurun_out/pcs.log"
find "$R/gpurun_out/pcs" -type f | head
exit $rc
