#!/bin/bash
# Bench lines + kernel-trace stats for the other BASELINE configs (one bench
# step each at the given spp; the headline C2 line comes from gpu_round.sh).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for c in "$@"; do
  name="${c%%:*}"; args="${c#*:}"; args="${args//,/ }"
  timeout -k 10 500 python -u bench.py --steps 1 --warmup 1 --cpu-seconds 10 $args > "gpurun_out/bench_$name.log" 2>&1
  rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/bench_$name.log | cut -c1-160)"
  case $rc in 0) ;; *) exit $rc;; esac
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$name" -o k --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $args > "$R/gpurun_out/prof_$name.log" 2>&1 )
  rc=$?; echo "$name rocprof rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
