#!/bin/bash
# MIOpen's Winograd solvers vs the fp64 reference on the decoder's transposed conv (scripts/deconv_check.py),
# and the closed bench step time with them off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/wino; mkdir -p $OUT
MIOPEN_DEBUG_CONV_WINOGRAD=0 timeout -k 10 240 python3 scripts/deconv_check.py 2>/dev/null || exit $?
B="python3 -u bench.py --regime closed --no-cpu-baseline --no-c2 --steps 20 --warmup 5"
timeout -k 10 300 $B > $OUT/on.json 2> $OUT/on.err || exit $?
MIOPEN_DEBUG_CONV_WINOGRAD=0 timeout -k 10 300 $B > $OUT/off.json 2> $OUT/off.err || exit $?
for f in on off; do python3 -c "
import json
d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('winograd $f', round(d['ms_per_step'],3))"; done
