"""Per (kernel, grid, workgroup) launch durations of a rocprofv3 kernel trace:
    python tools/trace_kernels.py <run_kernel_trace.csv> [substring ...]"""
import collections
import csv
import sys


def main(path, subs):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if subs and not any(s in n for s in subs):
            continue
        short = n.replace("(anonymous namespace)::", "").replace("vaesne::", "").replace("void ", "")
        short = short.split("(")[0]
        key = (short, r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{k[0][:60]:60s} grid {k[1]:>8s} x {k[2]:>3s} wg {k[3]:>4s}  n {len(v):4d}  median {v[len(v) // 2]:8.1f} us  min {v[0]:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
