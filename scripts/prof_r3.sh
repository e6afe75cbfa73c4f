#!/bin/bash
# Round-3 measurement: the headline bench line (closed regime), then rocprofv3 kernel stats of the
# closed step at the headline shape (N=4096, L=16) and at one C5 rank's share (N=16384, L=4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r3}
mkdir -p $OUT
echo "[$(date +%T)] bench (headline, closed regime)"
timeout -k 10 300 python3 $ROOT/bench.py --regime closed --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-c2 \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
summ() {
python3 - "$1" "$2" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time per step {tot/steps/1e3:.1f} us")
for r in rows[:32]:
    print(f"{float(r['TotalDurationNs'])/steps/1e3:9.1f} us/step {int(r['Calls'])/steps:6.1f}/step avg {float(r['AverageNs'])/1e3:9.1f}  {r['Name'][:120]}")
PY
}
cd /tmp && export TMPDIR=/tmp
declare -A ARGS=([headline]="--P 256 --L 16" [c5rank]="--P 1024 --L 4" [L2]="--P 256 --L 2")
for name in ${CFGS:-headline c5rank}; do
  args=${ARGS[$name]}
  echo "[$(date +%T)] rocprofv3 $name ($args)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run --output-format csv -- \
    python3 $ROOT/bench.py --regime closed $args --steps 5 --warmup 2 --no-cpu-baseline --no-phase-timing --no-c2 \
    > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  grep -h "ci_gemm\|ci_pivot\|ci_update\|ci_panel\|syrk\|kl_" $OUT/$name/run_kernel_trace.csv > $OUT/$name.trace_ci.csv 2>/dev/null
  rm -f $OUT/$name/run_kernel_trace.csv
  cat $OUT/$name.json
  summ $OUT/$name/run_kernel_stats.csv 7 | tee $OUT/$name.summary.txt
done
