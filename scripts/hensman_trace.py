"""Per-step kernel list of the graphed Hensman step from a rocprofv3 kernel trace (diagnostic):
the last complete step, delimited by the second spd_inv_small_kernel launch of each step."""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
names = [e[2] for e in ev]
with open(sys.argv[1].replace("run_kernel_trace.csv", "last_kernels.tsv"), "w") as f:
    for s_, e_, n_ in ev[-3000:]:
        f.write(f"{s_}\t{e_}\t{n_[:120]}\n")
# the replayed graph repeats one kernel sequence: its period is the smallest p with the last 2p names
# periodic (skipping a short non-graph tail); the step is one such period
tail = names[-4000:]
period, off = None, 0
for off in range(0, 200):
    t = tail[:len(tail) - off]
    period = next((p for p in range(20, len(t) // 3) if all(t[-1 - i] == t[-1 - i - p] for i in range(2 * p))), None)
    if period:
        break
step = ev[len(ev) - off - period:len(ev) - off]
span = (step[-1][1] - step[0][0]) / 1e3
busy = sum(e[1] - e[0] for e in step) / 1e3
print(f"kernels in one step: {len(step)}, span {span:.1f} us, summed kernel time {busy:.1f} us")
c = Counter()
t = Counter()
for s, e, n in step:
    key = n.split("(")[0][:90]
    c[key] += 1
    t[key] += (e - s) / 1e3
for k, v in sorted(c.items(), key=lambda kv: -t[kv[0]])[:40]:
    print(f"{v:4d} x {t[k] / v:7.1f} us = {t[k]:7.1f} us  {k}")
