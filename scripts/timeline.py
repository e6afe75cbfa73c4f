"""Dev: one step's kernel timeline from a rocprofv3 --kernel-trace CSV (the last complete step: from the
last-but-one to the last cov_int_check launch, the first kernel of a step).  Prints every kernel (start offset, duration, stream /
queue, name) and the union of busy time, so the idle stretches of the step show."""
import csv
import sys


def main(path, marker="cov_int_check"):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        ks.append((s, e, q, r["Kernel_Name"]))
    ks.sort()
    starts = [k[0] for k in ks if marker in k[3]]
    if len(starts) < 2:
        print("fewer than two steps in the trace")
        return
    t0, t1 = starts[-2], starts[-1]
    step = [k for k in ks if t0 <= k[0] < t1]
    print(f"step {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
    busy, cur_s, cur_e = 0, None, None
    for s, e, q, n in step:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"busy (union) {busy / 1e3:.1f} us")
    for s, e, q, n in step:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>4s}  {n[:110]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
