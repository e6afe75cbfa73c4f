#!/bin/bash
# Dev A/B: the second encoder conv's input gradient from lvae_conv3x3_pool_dgrad_f32 (the tree) vs MIOpen
# (LVAE_CONV_DGRAD=0): parity tests, the op alone, kernel stats, interleaved closed-regime bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/dgrad; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_regime_b.py \
  -x -k "dgrad or conv_relu_maxpool2" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head; exit $rc; }
timeout -k 10 120 python3 scripts/dgrad_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/scripts/dgrad_ab.py > $OUT/prof.log 2>&1 || exit 1
rm -f $OUT/prof/*kernel_trace.csv
python3 $ROOT/scripts/kstats.py $OUT/prof/run_kernel_stats.csv 12 8 | head -14
cd $ROOT
for r in 1 2 3; do
  for dg in 1 0; do
    LVAE_CONV_DGRAD=$dg timeout -k 10 240 python3 bench.py --regime closed --steps 30 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/b${dg}_$r.json 2> $OUT/b${dg}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('dgrad=$dg', d['ms_per_step'])" $OUT/b${dg}_$r.json
  done
done
