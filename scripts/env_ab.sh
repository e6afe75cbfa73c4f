#!/bin/bash
# Dev: same-box A/B of the closed step under an environment toggle of the one library: "old" runs with
# $OLD_ENV (e.g. LVAE_RESID_BINS=0), "new" without; interleaved rounds of bench.py ($BENCH_ARGS), then
# (KERNELS set) rocprofv3 kernel stats of a short "new" run filtered by KERNELS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in old new; do
    if [ $v = old ]; then E="$OLD_ENV"; else E=""; fi
    timeout -k 10 300 env $E python3 bench.py --regime closed --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-c2 \
      $BENCH_ARGS > $OUT/env_ab_$v$r.json 2> $OUT/env_ab_$v$r.err || { tail -5 $OUT/env_ab_$v$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/env_ab_$v$r.json'))
print('$v round $r: ms/step', round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()})"
  done
done
if [ -n "$KERNELS" ]; then
  for v in old new; do
    if [ $v = old ]; then E="$OLD_ENV"; else E=""; fi
    [ -n "$E" ] && export "$E"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OLDPWD/$OUT/env_prof_$v \
      -o run --output-format csv -- python3 $OLDPWD/bench.py --regime closed --steps 5 --warmup 2 --no-cpu-baseline \
      --no-c2 $BENCH_ARGS > $OLDPWD/$OUT/env_prof_$v.log 2>&1) || { tail -5 $OUT/env_prof_$v.log; exit 1; }
    [ -n "$E" ] && unset ${E%%=*}
    python3 - "$KERNELS" $v <<'PY'
import csv, glob, sys
keys = sys.argv[1].split(",")
f = sorted(glob.glob(f"gpurun_out/env_prof_{sys.argv[2]}/**/run_kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in keys):
        print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  done
fi
