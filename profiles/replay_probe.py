"""Host-side cost of one hipGraph replay of the bench step: the time the
replay() call itself takes on the CPU vs the GPU time per step.
    python profiles/replay_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = bench.make_model(dev, bench.CFG["dropout"])
    x = bench.synthetic_batch(16, 1234, dev)
    st = bench.Step(model, x, dev, 1, True)
    st.capture()
    for _ in range(3):
        st()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(20):
        a = time.perf_counter()
        st()
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host replay() mean {1e3 * sum(host) / len(host):.3f} ms  min {1e3 * min(host):.3f}  "
          f"max {1e3 * max(host):.3f}; loop {1e3 * (t1 - t0) / 20:.3f} ms/step host, "
          f"{1e3 * (t2 - t0) / 20:.3f} ms/step incl. drain")
    print("first 5 host times (ms):", [round(1e3 * h, 3) for h in host[:5]])


if __name__ == "__main__":
    main()
