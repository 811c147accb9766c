"""Per-launch SQ counter summary (JSON) of the roofline kernels from the passes of
profiles/r06/sq.sh (bench.py --roofline-only), the input of bench.py's `valu` fields:
    python profiles/sq_json.py OUT.json gpurun_out/pmc_sq1/run_counter_collection.csv \
        gpurun_out/pmc_sq2/run_counter_collection.csv
Rows are the decoder-shape launches (grid of the step's N = 256 sequences x 982 tokens):
per kernel, every counter summed over a launch's rows (one row per XCD / dispatch record) and
averaged over the launches; the launch duration of pass 1 beside it."""
import collections
import csv
import json
import sys

# kernel -> grid size (work-items) of the decoder-shape launch
KERNELS = {"attn_fwd_sf16_kernel<4, 1, true>": 1048576, "attn_bwd_sf16_kernel<true>": 524288,
           "attn_fwd_sf16_kernel<1, 16, true>": 262144, "attn_rep_bwd_sf16_kernel<true>": 131072}


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("vaesne::", "").replace("void ", "").split("(")[0]


def main(out, paths):
    per = {}
    for pi, p in enumerate(paths):
        disp = collections.defaultdict(lambda: collections.defaultdict(float))
        dur = {}
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            if k not in KERNELS or int(r["Grid_Size"] if "Grid_Size" in r else r["Grid_Size_X"]) != KERNELS[k]:
                continue
            d = (k, r["Dispatch_Id"])
            disp[d][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        for (k, _), c in disp.items():
            e = per.setdefault(k, {"counters": collections.defaultdict(list), "us": []})
            for n, v in c.items():
                e["counters"][n].append(v)
        if pi == 0:
            for (k, _), us in dur.items():
                per[k]["us"].append(us)
    res = {"source": "profiles/r06/sq.sh: rocprofv3 --pmc passes over bench.py --roofline-only; "
                     "counters summed over a dispatch's rows, averaged over dispatches",
           "kernels": {}}
    for k, e in per.items():
        res["kernels"][k] = {"launches": len(e["us"]),
                             "launch_us_pass1": round(sum(e["us"]) / max(len(e["us"]), 1), 2),
                             "per_launch": {n: sum(v) / len(v) for n, v in sorted(e["counters"].items())}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
