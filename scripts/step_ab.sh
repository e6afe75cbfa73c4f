#!/bin/bash
# Dev: same-box A/B of the closed step, build_ab/liblvae_hip.so ("old", scripts/build_variant.sh) vs the
# tree's library ("new"), interleaved rounds of bench.py (args: $BENCH_ARGS); with KERNELS set, rocprofv3
# kernel averages of both (name filters, comma-separated).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp $ROOT/build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
    timeout -k 10 300 python3 bench.py --regime closed --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-c2 \
      $BENCH_ARGS > $OUT/step_ab_$v$r.json 2> $OUT/step_ab_$v$r.err || { cp /tmp/new.so $SO; tail -5 $OUT/step_ab_$v$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/step_ab_$v$r.json'))
print('$v round $r: ms/step', round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()})"
  done
done
cp /tmp/new.so $SO
if [ -n "$KERNELS" ]; then
  for v in old new; do
    if [ $v = old ]; then cp $ROOT/build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/step_prof_$v -o run \
      --output-format csv -- python3 $ROOT/bench.py --regime closed --steps 5 --warmup 2 --no-cpu-baseline --no-c2 \
      $BENCH_ARGS > $OUT/step_prof_$v.log 2>&1) || { cp /tmp/new.so $SO; tail -5 $OUT/step_prof_$v.log; exit 1; }
    python3 - "$KERNELS" $v $OUT <<'PY'
import csv, glob, sys
keys = sys.argv[1].split(",")
f = sorted(glob.glob(f"{sys.argv[3]}/step_prof_{sys.argv[2]}/**/run_kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in keys):
        print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  done
  cp /tmp/new.so $SO
fi
