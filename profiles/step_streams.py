"""Per-queue view of one step of a rocprofv3 kernel trace of bench.py (the
launches between two consecutive AdamW kernels): busy time per HW queue, the
union of busy intervals (time the GPU runs anything), and the main queue's
timeline with idle gaps >= GAP_US.
    python profiles/step_streams.py gpurun_out/prof/run_kernel_trace.csv [GAP_US]"""
import collections
import csv
import sys

from step_breakdown import short


def main(path, gap_us=3.0):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    # the fastest AdamW-to-AdamW window: a replayed (captured) step, not one of the eager
    # steps bench.py runs after its timed region (in-step kernel timing)
    spans = [(int(rows[j]["End_Timestamp"]) - int(rows[i + 1]["Start_Timestamp"]), i, j)
             for i, j in zip(idx[:-1], idx[1:]) if j - i > 50]
    _, i0, i1 = sorted(spans)[len(spans) // 4]
    step = rows[i0 + 1: i1 + 1]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in step)
    per_q = collections.defaultdict(list)
    for r in step:
        per_q[r["Queue_Id"]].append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0,
                                     short(r["Kernel_Name"])))
    iv = sorted((s, e) for q in per_q.values() for s, e, _ in q)
    union, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    print(f"span {(t1 - t0) / 1e3:.1f} us  union-busy {union / 1e3:.1f} us  idle {(t1 - t0 - union) / 1e3:.1f} us")
    for q, ks in sorted(per_q.items(), key=lambda x: -len(x[1])):
        busy = sum(e - s for s, e, _ in ks)
        print(f"queue {q}: {len(ks)} launches  busy {busy / 1e3:.1f} us")
    main_q = max(per_q, key=lambda q: len(per_q[q]))
    prev = 0
    print(f"--- queue {main_q} timeline (start us, dur us, gap before us) ---")
    for s, e, k in per_q[main_q]:
        g = (s - prev) / 1e3
        mark = "  <-- gap" if g >= gap_us else ""
        print(f"{s / 1e3:9.1f} {(e - s) / 1e3:8.1f} {g:7.1f}  {k}{mark}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 3.0)
