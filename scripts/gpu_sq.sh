#!/bin/bash
# SQ/LDS counters for the trace and shade kernels on a reduced bench frame.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
n=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"; do
  n=$((n+1))
  env $EXTRA timeout -k 10 300 rocprofv3 --pmc $set -d "$R/gpurun_out/sq$n" -o sq --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --res 960x540 --spp 64 > "$R/gpurun_out/sq$n.log" 2>&1
  rc=$?; echo "sq$n rc=$rc"; case $rc in 0) ;; *) tail -5 "$R/gpurun_out/sq$n.log"; exit $rc;; esac
done
exit 0
