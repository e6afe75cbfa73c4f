"""Summarise a rocprofv3 --stats kernel CSV per step: kstats.py run_kernel_stats.csv [rows] [steps].

Steps default to the number of S-GEMM launches (one per closed step); every row gives the per-step
time, calls per step and the average launch duration."""
import csv
import sys


def main():
    path = sys.argv[1]
    nrows = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    rows = list(csv.DictReader(open(path)))
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if not steps:
        steps = sum(int(r["Calls"]) for r in rows if "syrk_c16_kernel" in r["Name"]) or 1
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time per step {tot / steps / 1e3:.1f} us over {steps} steps (all streams, summed)")
    for r in rows[:nrows]:
        print(f"{float(r['TotalDurationNs']) / steps / 1e3:9.1f} us/step {int(r['Calls']) / steps:6.1f}/step "
              f"avg {float(r['AverageNs']) / 1e3:9.1f}  {r['Name'][:120]}")


if __name__ == "__main__":
    main()
