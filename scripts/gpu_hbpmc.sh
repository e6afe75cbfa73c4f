#!/bin/bash
# PMC pass on the KL micro (one iteration): SQ counters of the binned route's slab kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/hbpmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $ROOT/scripts/gram_micro.py 1 > $OUT/warm.log 2>&1 || exit $?
for m in ${MASKS:-0 3}; do
  LVAE_HB_DBG=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    -d $OUT/m$m -o run --output-format csv -- python3 $ROOT/scripts/gram_micro.py 1 > $OUT/pmc_$m.log 2>&1 || exit $?
  echo "== mask $m"
  python3 - $OUT/m$m <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "hb_slab" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc): print(f"  {k:24s} {acc[k] / max(n[k], 1):.4g} per dispatch-row ({n[k]} rows)")
PY
done
