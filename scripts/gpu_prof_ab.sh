#!/bin/bash
# rocprofv3 kernel-trace stats of one bench step per "label|ENV=.. ..|bench args" item.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for item in "$@"; do
  label="${item%%|*}"; rest="${item#*|}"; envs="${rest%%|*}"; args="${rest#*|}"
  ( cd /tmp && env $envs timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pab_$label" -o k --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $args > "$R/gpurun_out/pab_$label.log" 2>&1 )
  rc=$?; echo "$label rc=$rc $(tail -1 gpurun_out/pab_$label.log | cut -c1-120)"
  case $rc in 0) ;; *) exit $rc;; esac
  python3 - "$R/gpurun_out/pab_$label" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print("   %-40s calls=%5s avg=%9.3f ms total=%9.1f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
done
