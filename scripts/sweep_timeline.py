"""Per-pass kernel timeline of the last sweep in a rocprofv3 kernel-trace CSV (diagnostic)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
key = [("sw_pivot_kernel", "pivot"), ("sw_prep0_kernel", "prep0"), ("sw_prepw_kernel", "prepW"),
       ("sw_update_kernel<1", "U1"), ("sw_update_kernel<0", "U2"), ("sw_update_kernel<2", "LAST"),
       ("sw_finish_kernel", "finish")]
ev = []
for r in rows:
    name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
    for k, short in key:
        if k in name:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
ev.sort()
# the last sweep starts with the pivot before its prep0
starts = [i for i, e in enumerate(ev) if e[2] == "prep0"]
ev = ev[max(starts[-1] - 1, 0):]
t0 = ev[0][0]
tot = {}
for s, e, n in ev:
    tot.setdefault(n, []).append((e - s) / 1e3)
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  {(e - s) / 1e3:7.1f}  {n}")
print(f"sweep span {(ev[-1][1] - t0) / 1e3:.1f} us")
for n, v in tot.items():
    print(f"{n:7s} n={len(v):3d} mean {sum(v) / len(v):7.1f} us  total {sum(v):8.1f} us")
