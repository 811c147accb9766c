"""Untraced phase timeline of the captured bench step from device wall-clock stamps
(VAESNE_STAMPS=1; VAESNe/_stamps.py): the step is captured with one single-thread stamp
node at each phase boundary, replayed, and the stamps of the last replay are printed
in microseconds from the step's first stamp.  rocprofv3's kernel trace stretches the
latency-bound encoder phases with its per-dispatch cost; these nodes cost ~2 us each.
    VAESNE_STAMPS=1 python tools/stamps.py [--steps N] [--batch B]"""
import argparse
import os
import sys

os.environ.setdefault("VAESNE_STAMPS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=16, help="SN pairs per step (2: the DP script's per-GPU batch at 8 GPUs)")
    args = ap.parse_args()
    from VAESNe import _stamps
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = bench.make_model(dev, bench.CFG["dropout"])
    x = bench.synthetic_batch(args.batch, 1234, dev)
    st = bench.Step(model, x, dev, 1, True)
    st.capture()
    runs = []
    for _ in range(args.steps):
        st()
        torch.cuda.synchronize()
        runs.append(_stamps.read())
    names = list(runs[-1])
    print(f"{'stamp (us from the step start)':32s} {'min':>8s} {'median':>8s} {'max':>8s}")
    for n in names:
        v = sorted(r[n] for r in runs[2:] if n in r)
        print(f"{n:32s} {v[0]:8.1f} {v[len(v) // 2]:8.1f} {v[-1]:8.1f}")


if __name__ == "__main__":
    main()
