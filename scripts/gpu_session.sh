#!/bin/bash
# One GPU-box session: selected parity tests, the default bench line (incl. CPU baseline), a
# rocprofv3 kernel-stats pass of the Regime B step, and a 2-rank gloo rehearsal of the multi-GPU
# paths on the one GPU.  Each step has its own time limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-s}
mkdir -p "$OUT"
stage() { echo "[$(date +%T)] $*"; }
if [ -n "$K" ]; then
  stage "pytest -k $K"
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "$K" > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; stage "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/${TAG}_pytest.log" | tail -30
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  stage bench
  timeout -k 10 420 python bench.py $BENCH_ARGS > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
  rc=$?; stage "bench rc=$rc"; cat "$OUT/${TAG}_bench.json"; tail -4 "$OUT/${TAG}_bench.err"
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROF:-1}" = "1" ]; then
  stage rocprof
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --regime ${PROF_REGIME:-closed} --steps 5 --warmup 2 --h-steps 20 --no-cpu-baseline \
    --no-phase-timing --no-c2 > "$OUT/${TAG}_prof_bench.json" 2> "$OUT/${TAG}_prof.err"
  rc=$?; stage "rocprof rc=$rc"
  rm -f "$OUT/${TAG}_prof"/*/*kernel_trace.csv "$OUT/${TAG}_prof"/*kernel_trace.csv 2>/dev/null
  cd "$ROOT"
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${REHEARSE:-0}" = "1" ]; then
  stage "2-rank gloo rehearsal on one GPU"
  LVAE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --h-steps 10 \
    > "$OUT/${TAG}_w2.json" 2> "$OUT/${TAG}_w2.err"
  rc=$?; stage "rehearsal rc=$rc"; cat "$OUT/${TAG}_w2.json"; grep -E "rank|Error|error" "$OUT/${TAG}_w2.err" | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
