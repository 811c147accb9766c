"""Phase split of one bench step from a rocprofv3 kernel trace: encoder
forward (step start -> first decoder self-attention), decoder forward + loss +
decoder backward, encoder backward (last decoder attention backward -> AdamW).
    python profiles/phase_times.py run_kernel_trace.csv"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    step = rows[idx[-3] + 1: idx[-2] + 1]
    t0 = int(step[0]["Start_Timestamp"])
    big = [r for r in step if "attn_fwd_kernel<8, 256, 2" in r["Kernel_Name"]]
    bwd = [r for r in step if "attn_bwd_kv_kernel<8, 256, 2" in r["Kernel_Name"]]
    t_dec0 = int(big[0]["Start_Timestamp"]) - t0
    t_dec1 = int(bwd[-1]["End_Timestamp"]) - t0
    t_end = max(int(r["End_Timestamp"]) for r in step) - t0
    n_enc_f = sum(1 for r in step if int(r["Start_Timestamp"]) - t0 < t_dec0)
    n_enc_b = sum(1 for r in step if int(r["Start_Timestamp"]) - t0 > t_dec1)
    print(f"encoder fwd {t_dec0 / 1e6:.3f} ms ({n_enc_f} launches) | decoders {(t_dec1 - t_dec0) / 1e6:.3f} ms"
          f" | encoder bwd + update {(t_end - t_dec1) / 1e6:.3f} ms ({n_enc_b} launches) | step {t_end / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
