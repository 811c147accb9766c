"""Per-kernel SQ counter summary of profiles/sq_pass.sh / pmc_step.sh output:
    python profiles/sq_summary.py [-k substr,substr] run_counter_collection.csv [...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
args = sys.argv[1:]
keys = ("attn_fwd", "attn_bwd", "keep_bits")
if args and args[0] == "-k":
    keys = tuple(args[1].split(","))
    args = args[2:]
for path in args:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for name, cs in agg.items():
    if not any(k in name for k in keys):
        continue
    avg = {k: sum(v) / len(v) for k, v in cs.items()}
    print(f"{name}: {sum(dur[name]) / len(dur[name]):.1f} us avg over {len(dur[name])} rows")
    for k in sorted(avg):
        print(f"   {k:24s} {avg[k]:.4g}")
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_VALU"):
            if k in avg:
                print(f"   {k} / WAVE_CYCLES = {avg[k] / wc:.3f}")
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        print(f"   VALU insts per wave = {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.0f}")
