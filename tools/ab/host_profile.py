"""Host-side profile of the script loop (training_step, torch.optim.AdamW, host batches,
captured steps): per-batch wall time of the host thread and cProfile's top functions.
    python tools/ab/host_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    from torch.utils.data import DataLoader, TensorDataset
    from VAESNe.data_util import multimodalDataset
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    batches = 16
    model = bench.make_model(dev, bench.CFG["dropout"])
    opt = torch.optim.AdamW(model.parameters(), lr=bench.CFG["lr"])
    x = bench.synthetic_batch(16 * batches, 2024, "cpu")
    loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                        batch_size=16, shuffle=False)
    fn = lambda m, xx: m_iwae(m, xx, K=bench.CFG["K"])
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize(dev)
    print(f"epoch: {(time.perf_counter() - t0) / batches * 1e3:.3f} ms per batch")
    pr = cProfile.Profile()
    pr.enable()
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize(dev)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
