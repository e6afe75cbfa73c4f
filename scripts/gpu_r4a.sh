#!/bin/bash
# Round-4 first call: the -m gpu suite, the default closed bench with C2 (no CPU leg), then the same
# bench command under rocprofv3 --kernel-trace --stats WITH the phase events on, so that the S GEMM's
# event average and its rocprof average come from the same launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
N=${PROF_NAME:-r4a}
OUT=$ROOT/gpurun_out/$N
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider --maxfail=5 ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
  # test failures (rc 1) do not stop the measurements; a crash, abort or time limit does
  [ $rc -le 1 ] || exit $rc
fi
echo "[$(date +%T)] bench (closed + c2)"
timeout -k 10 400 python3 bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); print('c2', json.dumps(d.get('c2'))[:900]); print('roof', json.dumps(d.get('roofline'))[:600])"
cd /tmp && export TMPDIR=/tmp
echo "[$(date +%T)] rocprofv3 default closed bench (phase events on)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 $BENCH_ARGS \
  > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 $ROOT/scripts/kstats.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/headline_kernel_stats.txt
cp $OUT/prof/run_kernel_stats.csv $OUT/headline_kernel_stats.csv
grep -h "syrk_c16" $OUT/prof/run_kernel_trace.csv > $OUT/syrk_trace.csv
rm -f $OUT/prof/run_kernel_trace.csv
head -12 $OUT/headline_kernel_stats.txt
python3 -c "import json; d=json.load(open('$OUT/prof.json')); r=d['roofline']; print('event avg us', r.get('avg_launch_us_event', r.get('avg_launch_us')), 'frac', r['frac'], r.get('frac_event'))"
cd $ROOT
for v in "closedL16:1:--regime closed" "sharded1:1:--regime closed --sharded-world1" "share8:1:--regime closed --rank-share 8" "share8_nopipe:0:--regime closed --rank-share 8" "L2full:1:--regime closed --L 2" "L2full_nopipe:0:--regime closed --L 2" "closedL16_pipe16:1:--regime closed"; do
  name=${v%%:*}; rest=${v#*:}; pipe=${rest%%:*}; args=${rest#*:}
  echo "[$(date +%T)] bench $name (LVAE_CI_PIPE=$pipe $args)"
  PL=4; [ $name = closedL16_pipe16 ] && PL=16
  LVAE_CI_PIPE_L=$PL LVAE_CI_PIPE=$pipe timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$name.json')); print('$name', round(d['ms_per_step'],3), 'ms', d['config']['parallelism'][:60], {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
done
# pivot phase stamps: this tree vs build_ab (the pending update before the triangular / shared-operand loads)
SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
for v in new old; do
  [ $v = old ] && cp $ROOT/build_ab/liblvae_hip.so $SO
  echo "[$(date +%T)] pivot_prof $v"
  LS=2,16 timeout -k 10 120 python3 scripts/pivot_prof.py > $OUT/pivot_prof_$v.txt 2>&1 || { cp /tmp/new.so $SO; tail -5 $OUT/pivot_prof_$v.txt; exit 1; }
  grep -E "^L=|^  (0|1|8|15) " $OUT/pivot_prof_$v.txt
done
cp /tmp/new.so $SO
