"""MFMA / VALU balance per kernel from a full-step SQ counter pass (profiles/r05_session.sh,
pmc_sq3: SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES over three captured steps):
    python profiles/sq_mfma_summary.py run_counter_collection.csv
mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4 SIMDs x 256 CUs / 32 SEs):
the fraction of the busy cycles the matrix cores of the chip were busy (the counter sums
over the SIMDs; SQ_BUSY_CYCLES counts per shader engine)."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
dur = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("vaesne::", "")
    name = name.replace("void ", "").split("(")[0]
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES":
        n[name] += 1
        dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
rows = sorted(agg, key=lambda k: -dur[k])
print(f"{'kernel':60s} {'us/launch':>9s} {'launches':>8s} {'VALU/wave':>9s} {'MFMA/wave':>9s} "
      f"{'MFMA:VALU':>9s} {'mfma_busy':>9s}")
for k in rows[:30]:
    c = agg[k]
    w = max(c["SQ_WAVES"], 1)
    busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(c["SQ_BUSY_CYCLES"] * 1024 / 32, 1)
    print(f"{k[:60]:60s} {dur[k] / n[k]:9.1f} {n[k]:8d} {c['SQ_INSTS_VALU'] / w:9.0f} "
          f"{c['SQ_INSTS_MFMA'] / w:9.1f} {c['SQ_INSTS_MFMA'] / max(c['SQ_INSTS_VALU'], 1):9.4f} "
          f"{busy:9.3f}")
