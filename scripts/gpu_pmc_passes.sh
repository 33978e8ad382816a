#!/bin/bash
# One rocprofv3 --pmc pass per argument (space-separated counter list), each
# on one bench step (BARGS, default --spp 8), summarised per kernel.
# usage: gpu_pmc_passes.sh "C1 C2 .." "C3 C4 .." ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
BARGS="${BARGS:---spp 8}"
i=0
for pass in "$@"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $pass -d "$R/gpurun_out/pp_$i" -o pp --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $BARGS > "$R/gpurun_out/pp_$i.log" 2>&1 )
  rc=$?; echo "pass $i [$pass] rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
python3 - "$R/gpurun_out" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(sys.argv[1] + "/pp_*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0][-30:]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if any(s in k for s in ("shade", "trace", "film", "camera")):
        print(k)
        for c, x in sorted(v.items()):
            print("    %-40s %.4g" % (c, x))
PY
