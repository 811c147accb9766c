"""Execution switches of the HIP path, read ONCE from the environment at import.

The forward never reads os.environ per call.  Every switch selects between two
parity-tested executions of the same arithmetic (tests set the attributes with
monkeypatch.setattr, not the environment):

  streams     VAESNE_STREAMS=0    one HIP stream for the whole step (default: the
                                  photometry branch and the encoders' context
                                  self-attention paths on side streams;
                                  tests/test_gpu_boundary.py: bitwise equal)
  ctx_streams VAESNE_CTX_STREAMS  side streams the per-block context paths share
                                  (round robin; default 2)
  ctx_merge   VAESNE_CTX_MERGE=0  per-block context self-attention paths instead of
                                  one batch-stacked launch (test_gpu_kernels.py)
  enc_chain   VAESNE_ENC_CHAIN=0  per-block encoder launches instead of the fused
                                  latent chain (test_gpu_enc_chain.py)
  fused_head  VAESNE_FUSED_HEAD=0 output head as two linears (test_gpu_kernels.py)
  rep_attn    VAESNE_REP_ATTN=0   decoder block 1 on the expanded input instead of
                                  once per distinct sequence (test_gpu_rep_attention.py)
  defer_grads VAESNE_DEFER_GRADS=0  parameter-gradient sums launched per op instead
                                  of one batched flush (test_gpu_defer.py)
  step_graph  VAESNE_STEP_GRAPH=0  training_step runs every batch eagerly instead of
                                  replaying a captured hipGraph (_stepgraph.py;
                                  test_gpu_stepgraph.py: bitwise equal)
  stamps      VAESNE_STAMPS=1     measurement only: device wall-clock stamps at the
                                  step's phase boundaries (_stamps.py, tools/stamps.py);
                                  off by default (no extra launches)
"""
import os


def _flag(name, default=True):
    return os.environ.get(name, "1" if default else "0") != "0"


streams = _flag("VAESNE_STREAMS")
ctx_streams = max(1, int(os.environ.get("VAESNE_CTX_STREAMS", "2") or 2))
ctx_merge = _flag("VAESNE_CTX_MERGE")
enc_chain = _flag("VAESNE_ENC_CHAIN")
fused_head = _flag("VAESNE_FUSED_HEAD")
rep_attn = _flag("VAESNE_REP_ATTN")
defer_grads = _flag("VAESNE_DEFER_GRADS")
step_graph = _flag("VAESNE_STEP_GRAPH")
stamps = _flag("VAESNE_STAMPS", default=False)
