"""MFMA utilisation per kernel from one rocprofv3 --pmc pass (scripts/gpu_mfma_pmc.sh): SQ_VALU_MFMA_BUSY_CYCLES
summed over every SIMD of the chip (MI355X_MICROARCH.md: 32 busy cycles per 32x32x16 f16 MFMA, i.e. the SIMD-cycles
the matrix pipes ran), against the SIMD-cycles of the dispatch, 4 SIMDs x 256 CUs x (GRBM_GUI_ACTIVE / 8: that
counter is summed over the 8 XCDs).  Writes <out>/mfma_summary.json: per kernel name the mean per dispatch of
each counter, the dispatches, and mfma_busy_frac = busy / (1024 x GRBM_GUI_ACTIVE / 8)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


def main(out_dir):
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
    for path in glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            a = acc[row["Kernel_Name"]][row["Counter_Name"]]
            a[0] += float(row["Counter_Value"])
            a[1] += 1
    if not acc:
        sys.exit(f"no counter_collection.csv under {out_dir}")
    res = {}
    for name, cs in acc.items():
        d = {c: s / max(n, 1) for c, (s, n) in cs.items()}
        d["dispatches"] = max(n for _, n in cs.values())
        busy, grbm = d.get("SQ_VALU_MFMA_BUSY_CYCLES"), d.get("GRBM_GUI_ACTIVE")
        if busy is not None and grbm:
            d["mfma_busy_frac"] = busy / (SIMDS * grbm / XCDS)
        res[name] = d
    json.dump(res, open(os.path.join(out_dir, "mfma_summary.json"), "w"), indent=1)
    keys = sys.argv[2].split(",") if len(sys.argv) > 2 else []
    rows = sorted(res.items(), key=lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * kv[1]["dispatches"])
    for name, d in rows[:40]:
        if keys and not any(k in name for k in keys):
            continue
        print(f"{d.get('mfma_busy_frac', float('nan')):7.3f} busy {d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):14.4g} "
              f"grbm {d.get('GRBM_GUI_ACTIVE', 0):12.4g} x{d['dispatches']:4d}  {name[:80]}")


if __name__ == "__main__":
    main(sys.argv[1])
