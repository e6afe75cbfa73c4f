#!/bin/bash
# Dev: same-box A/B of library variants (VARIANTS="tree d2 d4": tree = the in-tree library, else
# variants/<name>/liblvae_hip.so via LVAE_LIB), interleaved ROUNDS of the closed bench ($BENCH_ARGS); with KERNELS
# set (comma-separated name filters), rocprofv3 kernel averages per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/lib_ab; mkdir -p $OUT
lib() { [ "$1" = tree ] && echo "" || echo "LVAE_LIB=$ROOT/variants/$1/liblvae_hip.so"; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    timeout -k 10 300 env $(lib $v) python3 bench.py --regime closed --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --no-c2 --no-dp-world1 $BENCH_ARGS > $OUT/$v$r.json 2> $OUT/$v$r.err || { tail -5 $OUT/$v$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/$v$r.json'))
print('$v round $r: ms/step', round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()})"
  done
done
if [ -n "$KERNELS" ]; then
  for v in $VARIANTS; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 env $(lib $v) rocprofv3 --kernel-trace --stats -d $OUT/prof_$v \
      -o run --output-format csv -- python3 $ROOT/bench.py --regime closed --steps 5 --warmup 2 --no-cpu-baseline \
      --no-c2 --no-dp-world1 $BENCH_ARGS > $OUT/prof_$v.log 2>&1) || { tail -5 $OUT/prof_$v.log; exit 1; }
    rm -f $OUT/prof_$v/*kernel_trace.csv
    python3 - "$KERNELS" $v $OUT <<'PY'
import csv, glob, sys
keys = sys.argv[1].split(",")
f = sorted(glob.glob(f"{sys.argv[3]}/prof_{sys.argv[2]}/**/run_kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in keys):
        print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  done
fi
