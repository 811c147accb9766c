"""Per-step kernel breakdown of a rocprofv3 kernel trace of bench.py: takes the
launches between two consecutive AdamW kernels (one graph replay = one step).
    python profiles/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv [N]"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"at::native::", "", n)
    return n.split("(")[0][:80]


def main(path, top=30):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    a, b = idx[-3] + 1, idx[-2] + 1
    step = rows[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    print(f"launches/step {len(step)}  span {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  "
          f"gaps {(t1 - t0 - busy) / 1e6:.3f} ms")
    c, t = collections.Counter(), collections.Counter()
    for r in step:
        k = short(r["Kernel_Name"])
        c[k] += 1
        t[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, v in t.most_common(top):
        print(f"{v / 1e6:8.3f} ms {c[k]:5d}x  avg {v / c[k] / 1e3:8.1f} us  {k}")




def by_grid(path, pattern="colsum"):
    """Launches of one kernel in one step, split by grid size (which call site)."""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    step = rows[idx[-3] + 1: idx[-2] + 1]
    c, t = collections.Counter(), collections.Counter()
    for r in step:
        if pattern in r["Kernel_Name"]:
            k = (r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Workgroup_Size_X"))
            c[k] += 1
            t[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, v in t.most_common():
        print(f"{v / 1e6:8.3f} ms {c[k]:5d}x  avg {v / c[k] / 1e3:8.1f} us  grid {k[0]} wg {k[1]}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and not sys.argv[2].isdigit():
        by_grid(sys.argv[1], sys.argv[2])
    else:
        main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
