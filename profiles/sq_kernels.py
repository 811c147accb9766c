"""Per-kernel SQ summary of profiles/r06/sq_step.sh's two passes (every kernel of the step):
    python profiles/sq_kernels.py PASS1.csv PASS2.csv [name-substring ...]
Per kernel (all dispatches of one name and grid): mean duration, VALU / MFMA instructions per
wave, the issue model of bench.py (_sq_valu), MFMA busy and LDS conflict fractions."""
import collections
import csv
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("vaesne::", "").replace("void ", "").split("(")[0]


def load(p):
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(p)):
        d = r["Dispatch_Id"]
        disp[d][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[d] = (short(r["Kernel_Name"]), r.get("Grid_Size", r.get("Grid_Size_X")),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    return disp, meta


def main(p1, p2, subs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in (p1, p2):
        disp, meta = load(p)
        for d, c in disp.items():
            k, grid, us = meta[d]
            if subs and not any(s in k for s in subs):
                continue
            for n, v in c.items():
                agg[(k, grid)][n].append(v)
            if p == p1:
                agg[(k, grid)]["us"].append(us)
    rows = []
    for (k, grid), c in agg.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        if "GRBM_GUI_ACTIVE" not in m or "SQ_INSTS_VALU" not in m:
            continue
        valu, mf, tr = m["SQ_INSTS_VALU"], m.get("SQ_INSTS_MFMA", 0), m.get("SQ_INSTS_VALU_TRANS_F32", 0)
        act = m["GRBM_GUI_ACTIVE"] / 8
        cyc = (2 * (valu - mf) + 2 * tr + 8 * mf) / 1024
        rows.append((m["us"] * len(c["us"]), k, grid, len(c["us"]), m["us"], cyc / act,
                     m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / act,
                     m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_ACTIVE_INST_LDS", 1), 1),
                     valu / max(m.get("SQ_WAVES", 1), 1), mf / max(m.get("SQ_WAVES", 1), 1)))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'grid':>8s} {'n':>3s} {'us':>8s} {'issue':>6s} {'mfma':>6s} {'ldscf':>6s} {'valu/w':>8s} {'mfma/w':>7s}")
    for tot, k, grid, n, us, fr, mb, lc, vw, mw in rows[:40]:
        print(f"{k[:60]:60s} {grid:>8s} {n:3d} {us:8.1f} {fr:6.3f} {mb:6.3f} {lc:6.2f} {vw:8.0f} {mw:7.0f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
