"""Coarse phase split of one bench step from a rocprofv3 kernel trace: time to the
first spectra-decoder attention forward, decoder window, and the tail after the
last decoder attention backward (encoder backward + flush + optimizer).
    python profiles/step_phases.py gpurun_out/prof_X/run_kernel_trace.csv"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    for a, b in zip(idx[-4:-1], idx[-3:]):
        step = rows[a + 1:b + 1]
        t0 = int(step[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in step)
        big = [r for r in step if "attn_fwd_kernel<8, 256" in r["Kernel_Name"]]
        bwd = [r for r in step if "attn_bwd_kv_kernel<8, 256" in r["Kernel_Name"]]
        f0 = int(big[0]["Start_Timestamp"]) if big else t0
        b1 = int(bwd[-1]["End_Timestamp"]) if bwd else t1
        print(f"step {(t1 - t0) / 1e3:8.1f} us: to decoder {(f0 - t0) / 1e3:7.1f}  "
              f"decoders {(b1 - f0) / 1e3:7.1f}  tail {(t1 - b1) / 1e3:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
