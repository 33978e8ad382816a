#!/bin/bash
# Film-pass A/B on one GPU: the film parity tests, then one kernel-trace
# profile per film environment in FILMENVS (';'-separated) on config CFG.
# Outputs under gpurun_out/film_$CFG/.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
CFG="${CFG:-c3}"
o="$R/gpurun_out/film_$CFG"
mkdir -p "$o"
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests -q -m gpu -k "film" -p no:cacheprovider -x --timeout 240 \
    --timeout-method thread > "$o/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$o/pytest.log"; [ $rc = 0 ] || exit $rc
fi
cd /tmp || exit 1
IFS=';' read -ra envs <<< "${FILMENVS:-PT_FILM_SK=0;PT_FILM_SK=1}"
i=0
for e in "${envs[@]}"; do
  i=$((i+1))
  env $e timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$o/prof_$i" -o b --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > "$o/bench_$i.log" 2>&1
  rc=$?
  echo "[$e] rc=$rc $(tail -1 "$o/bench_$i.log" | cut -c1-220)"
  [ $rc = 0 ] || exit $rc
  python3 - "$o/prof_$i" <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
for row in csv.DictReader(open(f[0])):
    n = row["Name"]
    if any(k in n for k in ("k_film", "k_camera", "k_shade", "k_trace")):
        print(f"   {n.split('(')[0][:40]:40s} calls={row['Calls']:>5s} avg_ms={float(row['AverageNs'])/1e6:8.3f}")
EOF
done
echo "gpu_film done"
