#!/bin/bash
# A/B of library builds / env variants with per-kernel times (rocprofv3
# kernel-trace stats of one bench step each).
# usage: gpu_abk.sh "ENV=.. ENV=.." "ENV=.." ...   (PT_LIB=libptgpu_x.so selects a build)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
BARGS="${BARGS:---spp 64}"
i=0
for cfg in "$@"; do
  i=$((i+1))
  for kv in $cfg; do export "$kv"; done
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/abk_$i" -o abk --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline $BARGS > "$R/gpurun_out/abk_$i.log" 2>&1 )
  rc=$?
  for kv in $cfg; do unset "${kv%%=*}"; done
  echo "[$cfg] rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/abk_$i.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  python3 - "$R/gpurun_out/abk_$i" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:4] if f else []:
    print("   %-34s calls=%-4s total=%8.1f ms avg=%7.3f ms" % (r["Name"].split("(")[0][-34:], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6))
PY
  case $rc in 0) ;; *) exit $rc;; esac
done
