"""Host-side profile of the unchanged script's loop at 2 pairs per batch (bench.py
training_step_script's b2 leg): wall time per batch with and without cProfile, and the
functions the host spends it in.  Diagnostic, not product.
    python tools/b2_host_profile.py [--batches N]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=32)
    ap.add_argument("--bs", type=int, default=2)
    args = ap.parse_args()
    from torch.utils.data import DataLoader, TensorDataset
    from VAESNe.data_util import multimodalDataset
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = bench.make_model(dev, bench.CFG["dropout"])
    opt = torch.optim.AdamW(model.parameters(), lr=bench.CFG["lr"])
    x = bench.synthetic_batch(args.bs * args.batches, 2024, "cpu")
    loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                        batch_size=args.bs, shuffle=False)
    fn = lambda m, xx: m_iwae(m, xx, K=bench.CFG["K"])
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize(dev)
    for rep in range(2):
        t0 = time.perf_counter()
        training_step(model, opt, loader, loss_fn=fn, multimodal=True)
        torch.cuda.synchronize(dev)
        print(f"epoch {rep}: {(time.perf_counter() - t0) / args.batches * 1e3:.3f} ms per batch", flush=True)
    it = iter(loader)
    t0 = time.perf_counter()
    for _ in range(args.batches):
        next(it)
    print(f"DataLoader alone: {(time.perf_counter() - t0) / args.batches * 1e3:.3f} ms per batch")
    pr = cProfile.Profile()
    pr.enable()
    t0 = time.perf_counter()
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize(dev)
    pr.disable()
    print(f"profiled epoch: {(time.perf_counter() - t0) / args.batches * 1e3:.3f} ms per batch")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
