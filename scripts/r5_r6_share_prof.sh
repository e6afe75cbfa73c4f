#!/bin/bash
# Kernel statistics of the W = 8 rank share, round-5 tree vs this tree (see r5_r6_share_ab.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$PWD; OUT=$ROOT/gpurun_out/r5r6p; mkdir -p $OUT
export TMPDIR=/tmp
for t in r5 r6; do
  D=$ROOT; [ $t = r5 ] && D=$ROOT/variants/r5tree
  (cd $D && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $OUT/$t -o run --output-format csv -- python3 bench.py --regime closed \
     --steps 30 --warmup 5 --no-cpu-baseline --no-c2 --rank-share 8 --no-phase-timing > $OUT/$t.json 2> $OUT/$t.err) \
     || { tail -5 $OUT/$t.err; exit 1; }
  python3 -c "import json; print('$t', json.load(open('$OUT/$t.json'))['ms_per_step'])"
done
