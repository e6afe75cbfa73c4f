"""One step's kernel timeline from a rocprofv3 kernel-trace CSV: timeline.py run_kernel_trace.csv [step_kernel]
[which].  Steps are delimited by the launches of step_kernel (default the Gram fill, one per closed step); the
which-th step (default: the middle one) is printed per queue with start / end times (us) relative to the step's
first kernel, plus each queue's busy time and the step's span."""
import csv
import sys


def main():
    path = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "gram_sq_fill_tab"
    rows = list(csv.DictReader(open(path)))
    key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "start"
    key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "end"
    rows.sort(key=lambda r: int(r[key_s]))
    marks = [int(r[key_s]) for r in rows if mark in r["Kernel_Name"]]
    which = int(sys.argv[3]) if len(sys.argv) > 3 else len(marks) // 2
    t0, t1 = marks[which], marks[which + 1]
    # the step: kernels starting in [t0 - 3 ms (the ConvVAE may start before the fill), t1)
    sel = [r for r in rows if t0 - 1000000 <= int(r[key_s]) < t1]
    q = {}
    for r in sel:
        q.setdefault(r.get("Queue_Id", r.get("Stream_Id", "?")), []).append(r)
    for qid, rs in sorted(q.items()):
        busy = sum(int(r[key_e]) - int(r[key_s]) for r in rs) / 1e3
        print(f"== queue {qid}: {len(rs)} kernels, busy {busy:.1f} us")
        for r in rs:
            s, e = (int(r[key_s]) - t0) / 1e3, (int(r[key_e]) - t0) / 1e3
            if e - s > 15:
                print(f"  {s:9.1f} {e:9.1f} {e - s:8.1f}  {r['Kernel_Name'][:90]}")
    print(f"step span (fill to fill): {(t1 - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
