"""Summarise rocprofv3 --pmc counter_collection.csv files into per-kernel mean counter values
(one row per dispatch in the raw file; the raw files are too big to keep)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(out_dir):
    res = {}
    for path in glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(lambda: [0.0, 0])
        counter = None
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                counter = row.get("Counter_Name", counter)
                v = float(row.get("Counter_Value", 0.0))
                a = acc[(name, counter)]
                a[0] += v
                a[1] += 1
        steps = int(os.environ.get("PMC_STEPS", "3"))  # bench steps + warm-up steps of each pass
        for (name, c), (s, n) in acc.items():
            res.setdefault(c, {})[name] = {"mean": s / n, "dispatches": n, "per_step": s / steps}
    with open(os.path.join(out_dir, "pmc_summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    keys = os.environ.get("PMC_KERNELS", "").split(",")
    for c, d in res.items():
        items = sorted(d.items(), key=lambda kv: -kv[1]["mean"] * kv[1]["dispatches"])
        if keys != [""]:
            items = [kv for kv in items if any(k in kv[0] for k in keys)]
        for name, v in items[:12]:
            print(f"{c:24s} {v['mean']:16.1f} x{v['dispatches']:4d}  {name[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])
