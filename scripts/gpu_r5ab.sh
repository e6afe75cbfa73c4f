#!/bin/bash
# Step-level A/B of the binned hyper-gradient route: the closed-form bench step with the route on (default)
# and off (LVAE_KL_HYPER=0), then the W=8 rank share (2 dims, 512 images) both ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r5ab; mkdir -p $OUT
B="python3 -u bench.py --regime closed --no-cpu-baseline --no-c2 --steps 20 --warmup 5"
timeout -k 10 300 $B > $OUT/on.json 2> $OUT/on.err || exit $?
LVAE_KL_HYPER=0 timeout -k 10 300 $B > $OUT/off.json 2> $OUT/off.err || exit $?
timeout -k 10 300 $B --rank-share 8 > $OUT/rs_on.json 2> $OUT/rs_on.err || exit $?
LVAE_KL_HYPER=0 timeout -k 10 300 $B --rank-share 8 > $OUT/rs_off.json 2> $OUT/rs_off.err || exit $?
for f in on off rs_on rs_off; do python3 -c "
import json,sys
d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1])
print('$f', d.get('ms_per_step'), d.get('value'), d.get('rank_share', ''))"; done
