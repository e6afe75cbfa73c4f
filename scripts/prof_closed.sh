#!/bin/bash
# rocprofv3 kernel stats of the Regime B bench step (env passes through, e.g. LVAE_X3 / LVAE_KL_LDLT)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-profc}
mkdir -p $OUT
# warm MIOpen's find database first (a fresh box benchmarks every conv algorithm on first use)
timeout -k 10 300 python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-phase-timing > /dev/null 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-phase-timing > $OUT/bench.json 2> $OUT/bench.err || exit $?
rm -f $OUT/run_kernel_trace.csv
python3 - "$OUT/run_kernel_stats.csv" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print(f"{float(r['TotalDurationNs'])/7/1e3:9.1f} us/step {int(r['Calls'])//7:4d}/step avg {float(r['AverageNs'])/1e3:9.1f}  {r['Name'][:110]}")
PY
