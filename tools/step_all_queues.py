"""All queues of one traced step (between consecutive AdamW launches), in start
order: start / end (us from the step start), queue, kernel.  Optional time window.
    python tools/step_all_queues.py run_kernel_trace.csv [t_from_us] [t_to_us]"""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles"))
from step_breakdown import short  # noqa: E402


def main(path, lo=0.0, hi=1e12):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    # the fastest AdamW-to-AdamW window: a replayed (captured) step, not one of the eager
    # steps bench.py runs after its timed region (in-step kernel timing)
    spans = [(int(rows[j]["End_Timestamp"]) - int(rows[i + 1]["Start_Timestamp"]), i, j)
             for i, j in zip(idx[:-1], idx[1:]) if j - i > 50]
    _, i0, i1 = sorted(spans)[len(spans) // 4]
    step = rows[i0 + 1: i1 + 1]
    t0 = int(step[0]["Start_Timestamp"])
    qs = sorted({r["Queue_Id"] for r in step})
    for r in step:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        if s < lo or s > hi:
            continue
        col = qs.index(r["Queue_Id"])
        print(f"{s:9.1f} {e:9.1f} {e - s:7.1f}  {'   ' * col}q{r['Queue_Id']}  {short(r['Kernel_Name'])[:70]}")


if __name__ == "__main__":
    main(sys.argv[1], *(float(a) for a in sys.argv[2:]))
