"""Host-side profile of the scripts' training loop (bench.training_step_script's setup:
training_step(model, torch.optim.AdamW, DataLoader(bs=16), m_iwae K=8) with captured
replays): cProfile of one timed epoch, top entries by cumulative and own time.
    python tools/profile_script_loop.py [batches]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main(batches=16):
    from torch.utils.data import DataLoader, TensorDataset
    from VAESNe.data_util import multimodalDataset
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = bench.make_model(dev, bench.CFG["dropout"])
    opt = torch.optim.AdamW(model.parameters(), lr=bench.CFG["lr"])
    x = bench.synthetic_batch(16 * batches, 2024, "cpu")
    loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                        batch_size=16, shuffle=False)
    fn = lambda m, xx: m_iwae(m, xx, K=bench.CFG["K"])
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize()
    print(f"{1e3 * (time.perf_counter() - t0) / batches:.3f} ms per batch (unprofiled)")
    pr = cProfile.Profile()
    pr.enable()
    training_step(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(35)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
