"""Debug aid: capture bench.py's step once with a native SIGSEGV backtrace handler."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

BT = ctypes.CDLL(os.path.join(ROOT, "tools", "segv_bt.so"))
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = bench.make_model(dev, bench.CFG["dropout"])
x = bench.synthetic_batch(16, 1234, dev)
st = bench.Step(model, x, dev, 1, True)
BT.segv_bt_install()
st.capture()
st()
torch.cuda.synchronize()
print("captured ok")
