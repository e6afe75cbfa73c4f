#!/bin/bash
# One GPU-box pass: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-10}
stage() { echo "[$(date +%T)] $*"; }
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

stage pytest-gpu
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; stage "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
ok $rc || exit $rc

stage smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; stage "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
ok $rc || exit $rc

if [ "${SKIP_BENCH:-0}" = "0" ]; then
stage bench
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; stage "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
ok $rc || exit $rc
fi

if [ "${SKIP_PROF:-0}" = "0" ]; then
stage rocprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-phase-timing > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; stage "rocprof rc=$rc"
find "$OUT/prof" -name "*stats*" | head
fi

if [ "${PROF_HENSMAN:-0}" = "1" ]; then
stage rocprof-hensman
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_h" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --regime hensman --steps 50 --warmup 5 --no-cpu-baseline --no-phase-timing > "$OUT/prof_h_bench.json" 2> "$OUT/prof_h.err"
rc=$?; stage "rocprof-hensman rc=$rc"
cat "$OUT/prof_h_bench.json"
fi
