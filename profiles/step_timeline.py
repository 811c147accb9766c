"""Timeline of one step (between two AdamW launches) of a rocprofv3 kernel trace:
    python profiles/step_timeline.py gpurun_out/prof/run_kernel_trace.csv [t_from_us] [t_to_us] [min_us]"""
import csv
import re
import sys


def short(n):
    return re.sub(r"\(anonymous namespace\)::|void |vaesne::|at::native::", "", n).split("(")[0][:44]


path = sys.argv[1]
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
hi = float(sys.argv[3]) if len(sys.argv) > 3 else 1e12
mn = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
step = rows[idx[-3] + 1:idx[-2] + 1]
t0 = int(step[0]["Start_Timestamp"])
for r in step:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if lo <= s <= hi and d >= mn:
        print(f"{s:9.1f} {s + d:9.1f} {d:7.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])} "
              f"{r['Grid_Size_X']}x{r.get('Grid_Size_Y', '')}")
