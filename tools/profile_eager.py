"""Host-side profile of the eager training_step the cannon scripts run
(bench.training_step_eager's loop): cProfile, top functions by cumulative and by
own time.  python tools/profile_eager.py > gpurun_out/eager_prof.txt"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from torch.utils.data import DataLoader, TensorDataset  # noqa: E402

from VAESNe import _lib  # noqa: E402
from VAESNe.data_util import multimodalDataset  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402
from VAESNe.training_util import training_step  # noqa: E402

_lib.load()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, 0.1)
opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
x = bench.synthetic_batch(64, 2024, "cpu")
loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])), batch_size=16)
fn = lambda m, xx: m_iwae(m, xx, K=8)
training_step(model, opt, loader, loss_fn=fn, multimodal=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
training_step(model, opt, loader, loss_fn=fn, multimodal=True)
torch.cuda.synchronize()
print(f"eager: {(time.perf_counter() - t0) / 4 * 1e3:.2f} ms per batch", flush=True)
pr = cProfile.Profile()
pr.enable()
training_step(model, opt, loader, loss_fn=fn, multimodal=True)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(45)
