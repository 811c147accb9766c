"""Print the VALU issue model and LDS figures of sq_json.py summaries side by side:
    python profiles/sq_show.py A.json [B.json ...]"""
import json
import sys

SCORES = 987467776   # scores per decoder-shape launch (2 K B H 982^2, K = 8, B = 16, H = 4)
for f in sys.argv[1:]:
    for k, v in json.load(open(f))["kernels"].items():
        c = v["per_launch"]
        valu, mf, tr = c["SQ_INSTS_VALU"], c.get("SQ_INSTS_MFMA", 0), c.get("SQ_INSTS_VALU_TRANS_F32", 0)
        cyc = (2 * (valu - mf) + 2 * tr + 8 * mf) / 1024
        fr = cyc * 8 / c["GRBM_GUI_ACTIVE"]
        print(f"{f[-24:]:24s} {k[:36]:36s} {v['launch_us_pass1']:7.1f} us  valu/score {valu * 64 / SCORES:5.2f}"
              f"  issue frac {fr:.3f}  lds conflict {c['SQ_LDS_BANK_CONFLICT'] / 1e6:6.2f}M"
              f" / active {c['SQ_ACTIVE_INST_LDS'] / 1e6:6.2f}M  mfma busy"
              f" {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 * 8 / c['GRBM_GUI_ACTIVE']:.3f}")
