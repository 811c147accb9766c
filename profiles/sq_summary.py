"""Per-kernel SQ counter summary of the two roofline passes of profiles/sq_pass.sh
(bench.py --roofline-only: the decoder-shape attention launches), the first section of a
profile set's sq_counters.txt:
    python profiles/sq_summary.py gpurun_out/pmc_sq1/run_counter_collection.csv \
        gpurun_out/pmc_sq2/run_counter_collection.csv"""
import collections
import csv
import sys

KERNELS = ("attn_fwd_sf16_kernel<true>", "attn_bwd_sf16_kernel<true>",
           "attn_rep_fwd_kernel<8, 256, 1, 2, true>", "attn_rep_bwd_kernel<256, 1, 16>")


def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    rows = collections.Counter()
    dur = collections.defaultdict(float)
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if not any(name.endswith(k) for k in KERNELS):
                continue
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
            if p == paths[0]:
                rows[name] += 1
                dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    print("# SQ counters, bench.py --roofline-only (decoder-shape launches), profiles/sq_pass.sh")
    for k in sorted(agg, key=lambda k: KERNELS.index(next(x for x in KERNELS if k.endswith(x)))):
        c = agg[k]
        print(f"{k}: {dur[k] / max(rows[k], 1):.1f} us avg over {rows[k]} rows")
        for n in sorted(c):
            print(f"   {n:24s} {c[n]:.4g}")
        wc = max(c["SQ_WAVE_CYCLES"], 1)
        for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_VALU"):
            if n in c:
                print(f"   {n} / WAVE_CYCLES = {c[n] / wc:.3f}")
        if c.get("SQ_WAVES"):
            print(f"   VALU insts per wave = {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}")


if __name__ == "__main__":
    main(sys.argv[1:])
