#!/bin/bash
# Dev: same-box A/B of the graphed Hensman step (bench.py --regime hensman), build_ab/liblvae_hip.so ("old")
# vs the tree's library ("new"), interleaved rounds; then rocprofv3 kernel averages (KERNELS filters) of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp $ROOT/build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
    timeout -k 10 300 python3 bench.py --regime hensman --h-steps ${HSTEPS:-200} --no-cpu-baseline \
      > $OUT/hab_$v$r.json 2> $OUT/hab_$v$r.err || { cp /tmp/new.so $SO; tail -5 $OUT/hab_$v$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/hab_$v$r.json')); a = d.get('regime_a', d)
print('$v round $r:', {k: a[k] for k in a if 'ms' in k or k == 'value'})"
  done
done
if [ -n "$KERNELS" ]; then
  for v in old new; do
    if [ $v = old ]; then cp $ROOT/build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/hprof_$v -o run \
      --output-format csv -- python3 $ROOT/bench.py --regime hensman --h-steps 50 --no-cpu-baseline \
      > $OUT/hprof_$v.log 2>&1) || { cp /tmp/new.so $SO; tail -5 $OUT/hprof_$v.log; exit 1; }
    python3 - "$KERNELS" $v $OUT <<'PY'
import csv, glob, sys
keys = sys.argv[1].split(",")
f = sorted(glob.glob(f"{sys.argv[3]}/hprof_{sys.argv[2]}/**/run_kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in keys):
        print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  done
fi
cp /tmp/new.so $SO
