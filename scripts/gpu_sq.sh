#!/bin/bash
# SQ counters for the trace and shade kernels on a reduced bench frame.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d "$R/gpurun_out/sq1" -o sq --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --res 960x540 --spp 64 > "$R/gpurun_out/sq1.log" 2>&1
rc=$?; echo "sq1 rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d "$R/gpurun_out/sq2" -o sq --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --res 960x540 --spp 64 > "$R/gpurun_out/sq2.log" 2>&1
rc=$?; echo "sq2 rc=$rc"; tail -2 "$R/gpurun_out/sq2.log"
exit 0
