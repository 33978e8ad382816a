#!/bin/bash
# Round-6 evidence on one GPU.  Every GPU step has its own time limit; the
# script stops at the first failure.
#   STAGES (default "tests bench prof1 pmc sq"): any subset of tests bench ab prof prof1 pmc sq calib, run in that order
#          prof1: kernel-trace --stats with PT_PIPES=1 (one pipeline: every launch runs alone, so the averages
#          are kernel durations -- what the bench line's roofline uses); calib: tools/fetch_calib with
#          FETCH_SIZE / WRITE_SIZE passes (scripts/fetch_calib_summary.py); icache: SQC instruction-cache
#          hit / miss counters of the bench's kernels
#   CFG    bench --config for bench/prof/pmc/sq (default c2); OUT tag (default $CFG)
#   BARGS  extra bench args for prof/pmc (e.g. "--spp 64")
# Outputs under gpurun_out/r6_$OUT/: source_hash.txt, pytest_gpu.log, smoke.log,
# bench.log (JSON line last), prof/ (kernel-trace --stats), pmc_fetch/,
# pmc_write/ (separate --pmc passes), pmc_sq1/, pmc_sq2/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
CFG="${CFG:-c2}"
OUT="${OUT:-$CFG}"
STAGES="${STAGES:-tests bench prof1 pmc sq}"
o="$R/gpurun_out/r6_$OUT"
mkdir -p "$o"
python3 bench.py --print-source-hash > "$o/source_hash.txt" || exit 1
ok() { case "$1" in 0) return 0;; *) echo "STOP rc=$1 at $2"; exit "$1";; esac; }
has() { case " $STAGES " in *" $1 "*) return 0;; *) return 1;; esac; }
if has tests; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest ${TESTS:-tests} -q -m gpu -p no:cacheprovider -x --timeout 240 \
    --timeout-method thread ${TESTK:+-k "$TESTK"} > "$o/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$o/pytest_gpu.log"; ok $rc pytest
  if [ -z "$NOSMOKE" ]; then
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$o/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -1 "$o/smoke.log"; ok $rc smoke
  fi
fi
if has bench; then
  timeout -k 10 600 python -u bench.py --config "$CFG" --steps ${STEPS:-10} --warmup ${WARMUP:-2} --cpu-seconds 15 \
    ${EMUL:+--emulate-ranks $EMUL} $BARGS > "$o/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 "$o/bench.log" | cut -c1-600; ok $rc bench
fi
if has ab; then
  # A/B: one short bench per environment in ABENVS ("A=1 B=2;C=3;" -- ';'-separated, empty = default)
  IFS=';' read -ra envs <<< "${ABENVS:-}"
  i=0
  for e in "${envs[@]}"; do
    i=$((i+1))
    env $e timeout -k 10 300 python -u bench.py --config "$CFG" --steps ${ABSTEPS:-5} --warmup 1 --no-cpu-baseline $BARGS \
      > "$o/ab_$i.log" 2>&1
    rc=$?; echo "ab $i [$e] rc=$rc $(tail -1 "$o/ab_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline_kernels"]; print(d["value"], d["ms_per_step"], {x: (v["kernel"], v["avg_launch_ms"], v["overlapped_span_ms"]) for x, v in k.items()})' 2>/dev/null)"
    ok $rc "ab $i"
  done
fi
cd /tmp || exit 1
if has prof; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$o/prof" -o bench --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --steps ${PSTEPS:-5} --warmup 1 --no-cpu-baseline $BARGS > "$o/prof.log" 2>&1
  rc=$?; echo "rocprof stats rc=$rc"; tail -1 "$o/prof.log" | cut -c1-300; ok $rc prof
fi
if has prof1; then
  PT_PIPES=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$o/prof1" -o bench --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --steps ${PSTEPS:-3} --warmup 1 --no-cpu-baseline $BARGS > "$o/prof1.log" 2>&1
  rc=$?; echo "rocprof stats (1 pipeline) rc=$rc"; tail -1 "$o/prof1.log" | cut -c1-300; ok $rc prof1
fi
if has pmc; then
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$o/pmc_fetch" -o fetch --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline $BARGS > "$o/fetch.log" 2>&1
  rc=$?; echo "pmc fetch rc=$rc"; ok $rc fetch
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$o/pmc_write" -o write --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline $BARGS > "$o/write.log" 2>&1
  rc=$?; echo "pmc write rc=$rc"; ok $rc write
fi
if has sq; then
  SQ="${SQARGS:---spp 16}"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$o/pmc_sq1" -o sq1 --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline $SQ > "$o/sq1.log" 2>&1
  rc=$?; echo "pmc sq1 rc=$rc"; ok $rc sq1
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d "$o/pmc_sq2" -o sq2 \
    --output-format csv -- python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline $SQ \
    > "$o/sq2.log" 2>&1
  rc=$?; echo "pmc sq2 rc=$rc"; ok $rc sq2
  # VALU lane utilisation: thread-cycles of VALU work against 64 x the VALU instruction cycles
  timeout -s KILL 150 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS \
    SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES SQ_INSTS_VALU -d "$o/pmc_sq3" -o sq3 \
    --output-format csv -- python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline $SQ \
    > "$o/sq3.log" 2>&1
  rc=$?; echo "pmc sq3 rc=$rc"; ok $rc sq3
fi
if has icache; then
  # instruction-cache hits / misses of the bench's kernels (SQC block), beside the instruction counts
  timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_WAVES -d "$o/pmc_ic" -o ic --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline ${SQARGS:---spp 16} > "$o/ic.log" 2>&1
  rc=$?; echo "pmc icache rc=$rc"; ok $rc icache
fi
if has calib; then
  # FETCH_SIZE / WRITE_SIZE calibration: known bytes in the shading kernels' access shapes
  T="$R/pbrt-v3-light-portals_amd/tools/fetch_calib"
  timeout -k 10 120 "$T" 3 > "$o/calib.log" 2>&1
  rc=$?; echo "calib rc=$rc"; ok $rc calib
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$o/pmc_cfetch" -o cfetch --output-format csv -- "$T" 1 \
    > "$o/cfetch.log" 2>&1
  rc=$?; echo "calib fetch rc=$rc"; ok $rc cfetch
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$o/pmc_cwrite" -o cwrite --output-format csv -- "$T" 1 \
    > "$o/cwrite.log" 2>&1
  rc=$?; echo "calib write rc=$rc"; ok $rc cwrite
fi
echo "gpu_r6 $OUT done"
