#!/bin/bash
# A/B per-kernel averages of the exact-KL forward + backward alone (scripts/gram_micro.py under
# rocprofv3): build_ab/liblvae_hip.so ("old") vs the tree's library ("new"); KERNELS = name filters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gram_ab.sh > gpurun_out/kernel_ab.log 2>&1 || { tail -5 gpurun_out/kernel_ab.log; exit 1; }
for v in old new; do
  python3 - "$v" "${KERNELS:-kl_alpha,syrk}" <<'PY'
import csv, sys
v, keys = sys.argv[1], sys.argv[2].split(",")
rows = list(csv.DictReader(open(f"gpurun_out/ab_{v}/run_kernel_stats.csv")))
print(v, [(r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 1)) for r in rows if any(k in r["Name"] for k in keys)])
PY
done
