#!/bin/bash
# Instruction-mix / stall counters of the C2 kernels (one rocprofv3 --pmc pass
# each, at a reduced spp so a pass takes seconds).  usage: bash scripts/gpu_pmc_sq.sh [bench args]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
ARGS="${@:---spp 16}"
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > "$R/gpurun_out/pmc_avail.txt" 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  -d "$R/gpurun_out/pmc_sq1" -o sq1 --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $ARGS > "$R/gpurun_out/pmc_sq1.log" 2>&1
rc=$?; echo "pmc sq1 rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS \
  -d "$R/gpurun_out/pmc_sq2" -o sq2 --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $ARGS > "$R/gpurun_out/pmc_sq2.log" 2>&1
rc=$?; echo "pmc sq2 rc=$rc"
find "$R/gpurun_out" -name "*counter_collection*.csv"
exit 0
