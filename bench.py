"""Benchmark: the ZTF photometry+spectra MMVAE training step (BASELINE.json
configs[4], cannon/ZTF_photospect.py) on N MI355X GPUs, one process per GPU.

One step = m_iwae forward (K=8 importance samples, both encoders, the 2x2
cross-modal decoder matrix, dropout 0.1 in train mode) + backward + one RCCL
all-reduce of the flat gradient (N>1) + FusedAdamW update, on a fixed
per-GPU batch of 16 synthetic (light curve, spectrum) pairs already resident
in HBM (weak scaling).  The step is captured once as a hipGraph and replayed.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-graph]
                    [--no-cpu-baseline]

Multi-GPU: one process per GPU.  Under a launcher (torchrun sets WORLD_SIZE /
RANK / LOCAL_RANK) each process is one rank; with `--gpus N > 1` and no launcher
environment, this script starts the N rank processes itself (fresh children,
before anything touches the GPU) and exits with their status.  Backend "nccl"
(RCCL over xGMI); VAESNE_DP_BACKEND=gloo lets ranks share a GPU (rehearsing
`--gpus 2` on a 1-GPU box).  The headline is weak scaling (B pairs per GPU);
`strong_scaling` times the unchanged script's split of ONE global batch of 16
(cannon/ZTF_photospect.py:76 DataLoader(batch_size=16), sliced per rank as
training_util.training_step does).

Rank 0 prints ONE JSON line (value = whole-job SN pairs/s).  Beside it:
  roofline     : the dominant kernel (spectra-decoder masked self-attention
                 fused backward) timed with HIP events around its launches
                 INSIDE the training step (eager replay of the same step, on
                 the launch's own stream), its algorithmic FLOPs / average
                 launch time vs the FP32 peak; isolated launches beside it;
  cpu_baseline : the CPU oracle (pure-PyTorch restatement of the reference,
                 oracle/vaesne_oracle.py) timed on the host cores on a bounded
                 sample (rank 0, N=1 only);
  parity       : on the reference's own golden fixture of THIS configuration
                 (tests/golden/mmvae_cfg5_b16.npz: B=16, K=8, dropout off, injected
                 noise): elbo_rel_err = |loss_build - loss_ref| / |loss_ref|, the
                 max-rel errors of the latent mu / scale and decoder locs
                 (BASELINE.md §3), and the backward: grad_rel_err (full gradient
                 tensors) and grad_norm_rel_err (every parameter's gradient norm).
                 The cfg 2/3/4 side lines carry the same against their own fixtures
                 (elbo_spec_cfg2, elbo_photo_cfg3, mmvae_cfg4) and a CPU baseline each.
"""
import argparse
import contextlib
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.environ.get("VAESNE_PKG_DIR", os.path.join(ROOT, "vaesne-dev_amd")))   # A/B
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 matrix peak (spec)
F16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: BF16 / F16 dense MFMA peak (spec)
# f16 MFMA FLOPs the split-f16 attention issues per score: forward S^T and P V (P V as hi and lo
# B operands: 2 MFMAs per 16x16 output tile of 32 keys), backward S, dP, dV, dK, dQ -- each
# 16x16x32 MFMA = 16384 FLOPs over 256 (forward: 512) scores
SF16_MFMA_FLOPS_PER_SCORE = {"fwd": 4 * 16384 / 512, "bwd": 5 * 16384 / 256}
HBM_PEAK_GBS = 8000.0

CFG = dict(workload="ZTF_photospect MMVAE training step (cfg 5)", num_bands=2, latent_len=4,
           latent_dim=4, model_dim=32, num_heads=4, ff_dim=32, num_layers=4, dropout=0.1,
           beta=0.5, K=8, Lp=60, Ls=982, spectra_selfattn=True, lr=1e-3)


STEP_GFLOP_PER_PAIR = 29.214     # SURVEY.md §8(d), cfg 5, fwd + bwd matmul FLOPs
STEP_MSCORES_PER_PAIR = 262.4    # SURVEY.md §8(d), cfg 5, forward softmax scores


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_model(device, dropout):
    from VAESNe.PhotometricVAE import PhotometricVAE
    from VAESNe.SpectraVAE import SpectraVAE
    from VAESNe.mmVAE import photospecMMVAE
    c = CFG
    common = dict(latent_len=c["latent_len"], latent_dim=c["latent_dim"], model_dim=c["model_dim"],
                  num_heads=c["num_heads"], ff_dim=c["ff_dim"], num_layers=c["num_layers"],
                  dropout=dropout)
    spec = SpectraVAE(selfattn=c["spectra_selfattn"], spectra_length=c["Ls"], **common)
    photo = PhotometricVAE(num_bands=c["num_bands"], selfattn=False, photometric_length=c["Lp"],
                           **common)
    return photospecMMVAE(vaes=[photo, spec], beta=c["beta"]).to(device)


def synthetic_batch(B, seed, device, num_bands=None):
    """SURVEY.md §8(d) synthetic inputs (tests/golden/fill_rule.py recipe)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("fill_rule", os.path.join(ROOT, "tests", "golden", "fill_rule.py"))
    fr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fr)
    rng = np.random.default_rng(seed)
    pf, pt, pb, pm = fr.photo_inputs(rng, B, CFG["Lp"], num_bands or CFG["num_bands"])
    sf, sw, sp, sm = fr.spec_inputs(rng, B, CFG["Ls"])
    T = lambda a: torch.from_numpy(a).to(device)
    return [(T(pf), T(pt), T(pb), T(pm)), (T(sf), T(sw), T(sp), T(sm))]


def _mark(name):
    """Device wall-clock stamp of a phase boundary (VAESNE_STAMPS=1, tools/stamps.py)."""
    try:
        from VAESNe import _stamps
    except ImportError:            # an older package under profiles/ab_pkg.sh
        return
    _stamps.mark(name)


class Step:
    """fwd + bwd + pack (graph 1) | all-reduce (N>1) | AdamW update + RNG advance (graph 2)."""

    def __init__(self, model, x, device, world, use_graph, loss_fn=None, lr=None):
        from VAESNe import rng
        from VAESNe.distributed import GradAllReduce
        from VAESNe.losses import m_iwae
        from VAESNe.optim import FusedAdamW
        self.model, self.x, self.device, self.world = model, x, device, world
        self.loss_fn = loss_fn or (lambda m, x: m_iwae(m, x, K=CFG["K"]))
        self.rng = rng
        self.opt = FusedAdamW([p for p in model.parameters() if p.requires_grad],
                              lr=CFG["lr"] if lr is None else lr,
                              grad_hook=GradAllReduce("sum") if world > 1 else None)
        self._val = torch.zeros((), device=device)   # f of the last step (loss = -f)
        self.graphs = None
        self.use_graph = use_graph
        model.train()

    def fwd_bwd(self):
        try:
            from VAESNe._defer import deferred
        except ImportError:            # an older package under profiles/ab_pkg.sh
            deferred = contextlib.nullcontext
        try:
            from VAESNe.training_util import backward_negated
        except ImportError:
            def backward_negated(v, out=None, negate=True):
                loss = -v
                loss.backward()
                return v.detach()
        self.opt.zero_grad(set_to_none=True)
        _mark("step")
        with deferred():   # parameter-gradient sums: one batched launch at the end of backward
            value = self.loss_fn(self.model, self.x)
            _mark("loss")
            # = (-f).backward(); the loss -f is negated when read (no launch in the step)
            self._val = backward_negated(value, negate=False)
        _mark("backward")
        # the VAEs keep their last posterior parameters (the reference's `_qz_x_params`),
        # which would keep this step's autograd graph -- and its AccumulateGrad nodes,
        # bound to this step's stream -- alive into the next (captured) step
        for m in self.model.modules():
            if getattr(m, "_qz_x_params", None) is not None:
                m._qz_x_params = None
        self.opt.pack_grads()

    @property
    def loss(self):
        """The last step's loss -f (a device scalar)."""
        return -self._val

    def update(self):
        self.opt.apply_update()
        self.rng.advance(self.device)   # fresh sampler / dropout draws next step
        _mark("update")

    def eager(self):
        self.fwd_bwd()
        self.opt.reduce_grads()
        self.update()

    def capture(self):
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(3):
                self.eager()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        try:
            from VAESNe._capture import guarded   # refuses topologies that crash the capture
        except ImportError:            # an older package under profiles/ab_pkg.sh
            guarded = contextlib.nullcontext
        if self.world == 1:
            with torch.cuda.graph(g1):
                with guarded():
                    self.fwd_bwd()
                    self.update()
            self.graphs = (g1, None)
        else:
            with torch.cuda.graph(g1):
                with guarded():
                    self.fwd_bwd()
            with torch.cuda.graph(g2):
                self.update()
            self.graphs = (g1, g2)

    def __call__(self):
        if self.graphs is None:
            self.eager()
            return
        g1, g2 = self.graphs
        g1.replay()
        if g2 is not None:
            self.opt.reduce_grads()
            g2.replay()


def throughput_point(device, B, use_graph, steps=10, warmup=3):
    """The same cfg-5 step at a larger per-GPU batch (a capacity point beside
    the reference-batch `value`; not the headline metric)."""
    torch.manual_seed(1)
    model = make_model(device, CFG["dropout"])
    x = synthetic_batch(B, 4321, device)
    step = Step(model, x, device, 1, use_graph=use_graph)
    if use_graph:
        step.capture()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(device)
    dt = (time.perf_counter() - t0) / steps
    loss = step.loss.item()
    del step, model, x
    torch.cuda.empty_cache()
    return dict(per_gpu_batch=B, value=round(B / dt, 2), unit="SN pairs/s", ms_per_step=round(dt * 1e3, 3),
                steps=steps, finite_loss=math.isfinite(loss))


def time_kernel(fn, iters, device):
    """Average duration of fn's launches, HIP events on the stream they run on."""
    s = torch.cuda.Stream(device)
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(iters):
            fn()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def _usable_cores():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup
    CPU quota (cpu.max) when one is set (os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def _rocprof_avg_ms(kernel_prefix):
    """Average duration of a kernel in the committed rocprofv3 --kernel-trace --stats
    summary of the latest profile (profiles/LATEST names it), or None."""
    import csv
    import re
    try:
        d = open(os.path.join(ROOT, "profiles", "LATEST")).read().strip()
        # the decoder-shape launches picked from the trace by grid (roofline_launches.py):
        # the stats average also holds the encoder's context launches of the same
        # instantiation
        lj = os.path.join(ROOT, "profiles", d, "roofline_launches.json")
        if os.path.exists(lj):
            k = json.load(open(lj))["kernels"].get(kernel_prefix)
            if k:
                return k["avg_ms"], f"profiles/{d}/roofline_launches.json"
        path = os.path.join(ROOT, "profiles", d, "kernel_stats.csv")
        pat = re.compile(r"(^|::|\s)" + re.escape(kernel_prefix) + r"<")
        rows = [r for r in csv.DictReader(open(path)) if pat.search(r["Name"])]
        if rows:   # the instantiation with the most total time (the step's decoder launch)
            best = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            return float(best["AverageNs"]) * 1e-6, f"profiles/{d}/kernel_stats.csv"
    except (OSError, KeyError, ValueError):
        pass
    return None, None


def _sq_valu(kernel, scores):
    """VALU issue model of a roofline kernel from the committed SQ counter passes
    (profiles/<LATEST>/sq_counters.json, written by profiles/sq_json.py from
    profiles/r06/sq.sh): VALU lane-ops per score = (SQ_INSTS_VALU - SQ_INSTS_MFMA) * 64 /
    scores (SQ_INSTS_VALU counts the MFMAs too: reported apart, per score); issue cycles per
    SIMD = (2 * (VALU - MFMA) + 2 * TRANS + 8 * MFMA) / 1024 SIMDs (each VALU op issues in
    2 cycles on a 64-wide wave, transcendentals take 2 more, a 16x16x32 f16 MFMA 8);
    frac = issue cycles / active cycles (GRBM_GUI_ACTIVE / 8 XCDs); issue-bound ms =
    frac * the profiled launch duration.  None without the file."""
    try:
        d = open(os.path.join(ROOT, "profiles", "LATEST")).read().strip()
        path = os.path.join(ROOT, "profiles", d, "sq_counters.json")
        k = json.load(open(path))["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None
    c = k["per_launch"]
    valu, mfma = c["SQ_INSTS_VALU"], c.get("SQ_INSTS_MFMA", 0.0)
    trans = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
    cyc = (2 * (valu - mfma) + 2 * trans + 8 * mfma) / 1024
    frac = cyc * 8 / c["GRBM_GUI_ACTIVE"]
    return dict(valu_ops_per_score=round((valu - mfma) * 64 / scores, 2),
                mfma_insts_per_256_scores=round(mfma * 256 / scores, 3),
                valu_issue_frac=round(frac, 3),
                valu_issue_bound_ms=round(frac * k["launch_us_pass1"] * 1e-3, 4),
                sq_launch_ms=round(k["launch_us_pass1"] * 1e-3, 4),
                sq_source=f"profiles/{d}/sq_counters.json")


def roofline(device, B, in_step=None):
    """Spectra-decoder masked self-attention at its step shape (N = 2*K*B
    sequences x 982 tokens: the decoder runs once over both modalities'
    latents; 4 heads x dh 8, dropout 0.1, 5 % key padding),
    the dominant op of the step.  The roofline kernel is
    the fused attention backward (attn_bwd_kv_kernel<..., DQ=true>: dK, dV and
    dQ in one pass), the most expensive single kernel of the step; the forward
    is reported beside it.  Algorithmic FLOPs per score on SURVEY.md §8(d)'s
    FlopCounterMode basis: fwd 4*dh (QK^T, PV), bwd 8*dh (= 2x forward: dP, dV,
    dK, dQ).  The flash backward also recomputes S (2*dh more per score):
    reported separately as flops_incl_recompute, never in `achieved`.  The head_dim-8
    kernels are the split-f16 matrix-core ones (attention_sf16.hip): fp32-grade products
    (hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_f16), so `achieved` is fp32-basis
    algorithmic FLOP/s against the FP32 peak; `mfma_f16` reports the f16 matrix-core
    FLOP/s they issue against the f16 MFMA peak.
    `in_step`: {"attn_fwd" / "attn_bwd": (avg ms, launches)} timed with HIP events
    around the decoder-shape launches inside the training step (in_step_kernel_times);
    the headline `achieved` uses it, the isolated launches are reported beside it."""
    from VAESNe import _lib, rng
    N, L, E, H, dh = 2 * CFG["K"] * B, CFG["Ls"], CFG["model_dim"], CFG["num_heads"], 8
    pd = float(os.environ.get("VAESNE_ROOFLINE_PDROP", CFG["dropout"]))   # A/B studies only
    qkv = torch.randn(N, L, 3 * E, device=device)
    mask = (torch.rand(N, L, device=device) < 0.05)
    mask[:, 0] = False
    kbias = torch.where(mask, float("-inf"), 0.0).float().contiguous()
    o = torch.empty(N, L, E, device=device)
    lse = torch.empty(N, H, L, device=device)
    do = torch.randn(N, L, E, device=device)
    dqkv = torch.empty_like(qkv)
    st = rng.state(device)
    lib = _lib.lib
    bits = torch.empty(lib.attn_keep_bits_size(N, H, L, L), dtype=torch.uint8, device=device)
    b, d, s3 = qkv.data_ptr(), dqkv.data_ptr(), L * 3 * E
    # the fused backward's dQ partials (several key blocks per sequence), as _ops passes it
    wsb = torch.empty(max(1, lib.attn_workspace(N, H, L, L, dh, 1) // 4), device=device)

    def fwd():
        lib.attn_fwd(b, s3, 3 * E, b + 4 * E, s3, 3 * E, b + 8 * E, s3, 3 * E,
                     kbias.data_ptr(), L, o.data_ptr(), L * E, E, lse.data_ptr(),
                     N, H, L, L, dh, pd, st.data_ptr(), 7, bits.data_ptr(),
                     None, _lib.stream())

    def bwd(fn):
        return lambda: fn(b, s3, 3 * E, b + 4 * E, s3, 3 * E, b + 8 * E, s3, 3 * E,
                          kbias.data_ptr(), L, o.data_ptr(), L * E, E, lse.data_ptr(),
                          do.data_ptr(), L * E, E, d, s3, 3 * E, d + 4 * E, s3, 3 * E, d + 8 * E,
                          s3, 3 * E, N, H, L, L, dh, pd, st.data_ptr(), 7, bits.data_ptr(),
                          wsb.data_ptr(), _lib.stream())

    fwd()
    scores = N * H * L * L
    res = {}
    for name, kern, fn, fl in [("fwd", "attn_fwd_sf16_kernel", fwd, 4 * dh),
                               ("bwd", "attn_bwd_sf16_kernel", bwd(lib.attn_bwd), 8 * dh)]:
        t = time_kernel(fn, 20, device)
        res[name] = dict(kernel=kern, ms=t * 1e3, tflops=scores * fl / t / 1e12,
                         flops_per_launch=scores * fl,
                         mfma_f16_tflops=scores * SF16_MFMA_FLOPS_PER_SCORE[name] / t / 1e12)
        tr, src = _rocprof_avg_ms(kern)   # the committed kernel-trace average inside the step
        if tr is not None:
            res[name].update(ms_rocprof=tr, tflops_rocprof=scores * fl / (tr * 1e-3) / 1e12,
                             rocprof_source=src)
    # the decoders' first block: the same step shape as R = 2K copies of Bd = B distinct
    # sequences (attn_rep_*; scores, exponentials and dK/dQ products shared by the copies).
    # "equiv_tflops" counts the FLOPs of the R*Bd expanded sequences (the reference's work)
    R, Bd = 2 * CFG["K"], B
    qd = torch.randn(Bd, L, 3 * E, device=device)
    kbd = kbias[:Bd].contiguous()
    ord_ = torch.empty(N, L, E, device=device)
    lsed = torch.empty(Bd, H, L, device=device)
    dqd = torch.empty_like(qd)
    wsr = torch.empty(max(1, lib.attn_rep_workspace(Bd, R, H, L, dh, pd) // 4), device=device)
    qp, sp = qd.data_ptr(), L * 3 * E

    def rep_fwd():
        lib.attn_rep_fwd(qp, sp, 3 * E, kbd.data_ptr(), L, ord_.data_ptr(), L * E, E,
                         lsed.data_ptr(), Bd, R, H, L, dh, pd, st.data_ptr(), 9, bits.data_ptr(),
                         _lib.stream())

    def rep_bwd():
        lib.attn_rep_bwd(qp, sp, 3 * E, kbd.data_ptr(), L, ord_.data_ptr(), L * E, E,
                         lsed.data_ptr(), do.data_ptr(), dqd.data_ptr(), Bd, R, H, L, dh, pd,
                         st.data_ptr(), 9, bits.data_ptr(), wsr.data_ptr(), _lib.stream())

    rep_fwd()
    for name, kern, fn, fl in [("rep_fwd", "attn_fwd_sf16_kernel<1, 16, true>", rep_fwd, 4 * dh),
                               ("rep_bwd", "attn_rep_bwd_sf16_kernel", rep_bwd, 8 * dh)]:
        t = time_kernel(fn, 20, device)
        res[name] = dict(kernel=kern, ms=t * 1e3, equiv_tflops=scores * fl / t / 1e12,
                         note=f"{R} copies x {Bd} sequences (decoder block 1)")
    for name, sqk in (("fwd", "attn_fwd_sf16_kernel<4, 1, true>"),
                      ("bwd", "attn_bwd_sf16_kernel<true>"),
                      ("rep_fwd", "attn_fwd_sf16_kernel<1, 16, true>"),
                      ("rep_bwd", "attn_rep_bwd_sf16_kernel<true>")):
        v = _sq_valu(sqk, scores) if pd > 0 else None   # the counters are of the dropout launch
        if v is not None:
            res[name].update(v)
    for name, key, fl in (("fwd", "attn_fwd", 4 * dh), ("bwd", "attn_bwd", 8 * dh)):
        if in_step and key in in_step:
            ms, n = in_step[key]
            res[name].update(ms_in_step=ms, launches_in_step=n,
                             tflops_in_step=scores * fl / (ms * 1e-3) / 1e12,
                             mfma_f16_tflops_in_step=scores * SF16_MFMA_FLOPS_PER_SCORE[name]
                             / (ms * 1e-3) / 1e12)
    r = res["bwd"]
    a = r.get("tflops_in_step", r["tflops"])
    traffic, tsrc = None, None
    try:   # HBM bytes per launch from the committed rocprofv3 --pmc passes (gpu_run.sh pmc)
        t = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
        traffic = t["kernels"][r["kernel"]]["hbm_bytes_per_launch"]
        tsrc = t["source"] + "; " + t["correction"]
    except (OSError, KeyError, ValueError):
        pass
    mf = r.get("mfma_f16_tflops_in_step", r["mfma_f16_tflops"])
    out = dict(bound="fp32_flops", kernel=r["kernel"], achieved=round(a, 3), peak=FP32_PEAK_TFLOPS,
               unit="TFLOP/s", frac=round(a / FP32_PEAK_TFLOPS, 4), traffic=traffic,
               traffic_source=tsrc,
               launch_ms=round(r.get("ms_in_step", r["ms"]), 4),
               launch_ms_source=("HIP events around the step's own decoder-shape launches "
                                 "(eager replay of the training step, on the launch stream)"
                                 if "ms_in_step" in r else "HIP events, isolated launches"),
               launch_ms_isolated=round(r["ms"], 4),
               frac_isolated=round(r["tflops"] / FP32_PEAK_TFLOPS, 4),
               flops_per_launch=r["flops_per_launch"],
               flops_incl_recompute=scores * 10 * dh,
               algorithmic_bytes_per_launch=attn_bwd_algorithmic_bytes(N, H, L, dh, pd),
               detail={k: {kk: (round(vv, 4) if isinstance(vv, float) else vv)
                           for kk, vv in v.items()} for k, v in res.items()},
               mfma_f16=dict(achieved=round(mf, 2), peak=F16_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                             frac=round(mf / F16_MFMA_PEAK_TFLOPS, 4),
                             flops_per_score=SF16_MFMA_FLOPS_PER_SCORE["bwd"]),
               product_scheme=("split-f16 on v_mfma_f32_16x16x32_f16: x = hi + lo (f16 each, "
                               "2^-22 relative), x*y = hi*hi + hi*lo + lo*hi with fp32 "
                               "accumulation (<= 2^-20 relative per product, "
                               "tests/test_gpu_sf16.py)"),
               note="split-f16 matrix-core kernel, fp32-grade products; achieved = fp32-basis "
                    "algorithmic FLOP/s, peak = FP32 157.3 TF; FLOPs per score 8*dh "
                    "(FlopCounterMode: backward = "
                    "2x forward, S recompute excluded); scores per launch = 2*K*B*H*982^2 = %d; "
                    "launch_ms = in-step HIP events (headline), launch_ms_isolated = the same "
                    "launch alone on a stream, ms_rocprof = the committed kernel-trace "
                    "average inside the captured step" % scores)
    sp = softmax_peak(device, pd > 0)
    if sp is not None:
        f = res["fwd"]
        ach = scores / (f.get("ms_in_step", f["ms"]) * 1e-3) / 1e9
        out["softmax_frac"] = round(ach / sp, 4)
        out["softmax"] = dict(kernel=f["kernel"], achieved=round(ach, 1), peak=round(sp, 1),
                              unit="Gscores/s", frac=round(ach / sp, 4),
                              peak_source="tools/probe/softmax_peak.hip: the forward's key loop "
                                          "with every operand in registers (MFMAs, max test, "
                                          "exp2, sums, dropout hash and keep bits, f16 split), "
                                          "no LDS / HBM; achieved = scores per launch / the "
                                          "forward's in-step launch time")
    if "ms_rocprof" in r:
        out["launch_ms_rocprof"] = round(r["ms_rocprof"], 4)
        out["frac_rocprof"] = round(r["tflops_rocprof"] / FP32_PEAK_TFLOPS, 4)
    return out


def softmax_peak(device, drop, iters=1500):
    """Score-processing peak (Gscores/s) of the split-f16 forward's key loop with its
    operands in registers (tools/probe/softmax_peak.hip; SURVEY.md §8(d)'s softmax
    roofline), or None when the microbench library is absent (build_lib.build_probes)."""
    import ctypes
    path = os.path.join(ROOT, "tools", "probe", "libsoftmax_peak.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.softmax_peak_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p]
    grid = 256 * 3 * 4            # 4 rounds of 3 workgroups (12 waves) per CU
    out = torch.empty(grid * 256, device=device)

    def fn():
        rc = lib.softmax_peak_launch(grid, iters, int(drop), out.data_ptr(),
                                     torch.cuda.current_stream(device).cuda_stream)
        assert rc == 0, rc

    t = time_kernel(fn, 5, device)
    assert torch.isfinite(out).all()
    return grid * 4 * iters * 2048 / t / 1e9


def attn_bwd_algorithmic_bytes(N, H, L, dh, p):
    """HBM bytes the fused attention backward must move at least once: q|k|v read and
    dq|dk|dv written (fp32, 3*E each per token), o and dO read (E each), lse read
    (H per token), the key bias (1 per token) and, with dropout, the keep bitmap
    (1 bit per score)."""
    E = H * dh
    per_tok = 4 * (3 * E + 3 * E + 2 * E + H + 1)
    bits = N * H * L * L / 8 if p > 0 else 0
    return int(N * L * per_tok + bits)


class LaunchTimer:
    """_ops.launch_timer: HIP events around each launch of one attention shape
    (`work` = B*H*Lq*Lk scores) on the stream it is launched on."""

    def __init__(self, work):
        self.work = work
        self.ev = {}

    def run(self, name, work, fn):
        if work != self.work:
            return fn()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = fn()
        e1.record(s)
        self.ev.setdefault(name, []).append((e0, e1))
        return r

    def averages(self):
        torch.cuda.synchronize()
        return {k: (sum(a.elapsed_time(b) for a, b in v) / len(v), len(v))
                for k, v in self.ev.items()}


def in_step_kernel_times(step, B, reps=6):
    """Average duration of the spectra decoder's self-attention launches (blocks 2-4:
    N = 2*K*B sequences x 982 tokens) inside `reps` eager training steps, with the
    step's other streams running beside them.  Every rank runs it (the step's
    all-reduce is a collective)."""
    from VAESNe import _ops
    t = LaunchTimer(2 * CFG["K"] * B * CFG["num_heads"] * CFG["Ls"] * CFG["Ls"])
    step.eager()                       # settle allocations outside the timed launches
    _ops.launch_timer = t
    try:
        for _ in range(reps):
            step.eager()
    finally:
        _ops.launch_timer = None
    return t.averages()


def cpu_baseline(sample_B=4, steps=1):
    """The oracle (CPU restatement of the reference) on the same workload:
    cfg-5 shapes, K=8, dropout 0.1 train mode, AdamW; bounded sample: one step of
    4 pairs after a 1-pair warm-up step.  Every loss term is per sample (no
    cross-sample coupling), so the step's cost is linear in B and pairs/s at B=4
    extrapolates to the B=16 step (4x the work, 4x the time).  All cores this
    process may use (affinity, capped by the cgroup quota the box enforces)."""
    from oracle import vaesne_oracle as O
    cores, affinity, quota = _usable_cores()
    torch.set_num_threads(cores)
    c = CFG
    common = dict(latent_len=c["latent_len"], latent_dim=c["latent_dim"], model_dim=c["model_dim"],
                  num_heads=c["num_heads"], ff_dim=c["ff_dim"], num_layers=c["num_layers"])
    cfg = O.MMVAECfg(photo=O.VaeCfg("photo", num_bands=c["num_bands"], **common),
                     spec=O.VaeCfg("spec", selfattn=True, **common), beta=c["beta"])
    g = torch.Generator().manual_seed(0)
    p = O.make_params(cfg, lambda k, shp: (torch.randn(shp, generator=g) / math.sqrt(shp[-1])).numpy()
                      if "_pz" not in k else None, requires_grad=True)
    st = O.AdamWState(lr=c["lr"])
    eps = torch.finfo(torch.float32).eps

    def one(nb):
        x = synthetic_batch(nb, 99, "cpu")
        us = [torch.empty(c["K"], nb, c["latent_len"], c["latent_dim"]).uniform_(eps - 1, 1)
              for _ in range(2)]
        for v in p.values():
            v.grad = None
        loss, _, _ = O.m_iwae(p, cfg, x, c["K"], us, p_drop=c["dropout"], training=True)
        (-loss).backward()
        O.adamw_step(p, {k: v.grad for k, v in p.items() if v.requires_grad}, st)

    one(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        one(sample_B)
    dt = time.perf_counter() - t0
    v = sample_B * steps / dt
    return dict(value=round(v, 4), unit="SN pairs/s", cores=torch.get_num_threads(),
                kind="port", sample=f"{steps} oracle training step(s) of {sample_B} pairs (cfg-5 shapes, "
                                    f"K=8, dropout 0.1, AdamW) after a 1-pair warm-up step; {dt:.1f}s; "
                                    f"per-pair cost is linear in B, so the B=16 step takes "
                                    f"{16 / v:.1f}s on these cores",
                cores_affinity=affinity, cgroup_cpu_quota=quota, os_cpu_count=os.cpu_count(),
                cpu=_cpu_model())


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _rel(a, b):
    a = a.detach().double().cpu().numpy()
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-30))


def golden_parity(device, name, forward_detail=False):
    """One of the reference's own golden fixtures (tests/golden/<name>.npz, written by
    tests/golden/gen_golden.py from the reference package): identical parameters,
    inputs and Laplace noise, dropout off.  Forward AND backward on the HIP path, the
    backward under the training step's deferred gradient sums (training_util.py):
      elbo_rel_err      |loss - ref| / |ref|  (m_iwae for an MMVAE, losses.py:78-93;
                        elbo otherwise, losses.py:16-24)
      grad_rel_err      max over the fixture's full-gradient tensors of
                        max|g - ref| / max|ref|
      grad_norm_rel_err max over EVERY trainable parameter of
                        |‖g‖ - ref| / max(ref, 1e-3)  (tests/test_gpu_parity.py's bound)
    With forward_detail also the max-rel errors of the latent mu / scale and of the
    decoder locations."""
    from VAESNe import rng
    from VAESNe._defer import deferred
    from VAESNe.losses import elbo, m_iwae
    from VAESNe.training_util import backward_negated
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import build_model, golden_us, golden_x, load_golden
    g = load_golden(name)
    c = g["config"]
    mm = c["kind"] == "mmvae"
    model = build_model(c, device=device)
    model.train()
    x = golden_x(g, device)
    out = {}
    if forward_detail:
        with torch.no_grad(), rng.inject_uniform(golden_us(g)):
            qz, px, _ = model(x, K=c["K"])
        out.update(mu_rel_err=max(_rel(qz[m].loc, g[f"mu{m}"]) for m in range(2)),
                   scale_rel_err=max(_rel(qz[m].scale, g[f"scale{m}"]) for m in range(2)),
                   loc_rel_err=max(_rel(px[e][d].loc, g[f"loc{e}{d}"])
                                   for e in range(2) for d in range(2)))
        del qz, px
    for p in model.parameters():
        p.grad = None
    with deferred(), rng.inject_uniform(golden_us(g)):
        value = m_iwae(model, x, K=c["K"]) if mm else elbo(model, x, K=c["K"])
        loss = backward_negated(value)
    ref = float(g["loss"])
    params = dict(model.named_parameters())
    names = json.loads(str(g["grad_names"]))
    gn = max(abs(params[k].grad.norm().item() - n) / max(float(n), 1e-3)
             for k, n in zip(names, g["grad_norms"]))
    full = [k[5:] for k in g if k.startswith("grad:")]
    ge = max(_rel(params[k].grad, g["grad:" + k]) for k in full)
    out.update(elbo_rel_err=abs(loss.item() - ref) / abs(ref), grad_rel_err=ge,
               grad_norm_rel_err=gn, grad_tensors=len(full), grad_norms=len(names))
    return out


def parity(device):
    """The benchmarked configuration (B=16, K=8, cfg 5) on the reference's own golden
    fixture (mmvae_cfg5_b16): forward (loss, mu, scale, decoder locs) and backward
    (the fixture's 12 full gradient tensors and the gradient norm of every parameter
    tensor)."""
    out = golden_parity(device, "mmvae_cfg5_b16", forward_detail=True)
    out["parity_fixture"] = "tests/golden/mmvae_cfg5_b16.npz (B=16, K=8: this workload)"
    return out


def extras(device, use_graph, reps=10):
    """§8(f) paths beside the headline (N=1 only; not `value`):
    * reconstruct: photospecMMVAE.reconstruct(x, K=100) in eval mode (mmVAE.py:120-126,
      as test/goldstein/spect_cond_LC.py drives it), B=16 pairs, forward kernels only;
    * contrastive: one ContraPhotSpec + negInfoNCE training step (fwd, bwd, FusedAdamW)
      at cannon/test_photospectra_contrast.py's config (B=16, T=0.1, dropout 0.1), captured
      as a hipGraph like the headline step."""
    from VAESNe.contrastiveNets import ContraPhotSpec
    from VAESNe.losses import negInfoNCE
    out = {}
    torch.manual_seed(2)
    model = make_model(device, CFG["dropout"])
    model.eval()
    x = synthetic_batch(16, 99, device)
    with torch.no_grad():
        for _ in range(2):
            model.reconstruct(x, K=100)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(reps):
            rec = model.reconstruct(x, K=100)
        torch.cuda.synchronize(device)
    dt = (time.perf_counter() - t0) / reps
    ok = all(bool(torch.isfinite(rec[e][d]).all()) for e in range(2) for d in range(2))
    out["reconstruct_K100"] = dict(value=round(16 / dt, 2), unit="SN pairs/s", ms_per_call=round(dt * 1e3, 3),
                                   batch=16, K=100, finite=ok)
    del model, rec
    net = ContraPhotSpec(latent_len=4, latent_dim=4, proj_dim=8, num_bands=6, photo_model_dim=32,
                         photo_num_heads=4, photo_ff_dim=32, photo_num_layers=4, photo_dropout=0.1,
                         spec_model_dim=32, spec_num_heads=4, spec_num_layers=4, spec_ff_dim=32,
                         spec_dropout=0.1, selfattn=False).to(device)
    net.train()
    xc = synthetic_batch(16, 77, device)
    step = Step(net, xc, device, 1, use_graph, lr=2.5e-4,
                loss_fn=lambda m, x: negInfoNCE(m, x, temperature=0.1))
    graph = False
    if use_graph:
        try:
            step.capture()
            graph = True
        except Exception as e:
            log(f"[bench] contrastive hipGraph capture failed ({e!r}); timing eager steps")
            step.graphs = None
            torch.cuda.synchronize(device)
    for _ in range(3):
        step()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize(device)
    dt = (time.perf_counter() - t0) / reps
    out["contrastive_step"] = dict(value=round(16 / dt, 2), unit="SN pairs/s", ms_per_step=round(dt * 1e3, 3),
                                   batch=16, hipgraph=graph, finite_loss=math.isfinite(step.loss.item()))
    del net, step
    torch.cuda.empty_cache()
    return out


def time_steps(step, steps, warmup, device, world):
    """W untimed steps, then K timed steps bracketed by a barrier + device sync on both
    sides; the max over ranks (seconds)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64,
                         device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    return dt


def make_step(device, world, B, seed, use_graph, rank=0):
    """The cfg-5 training step on this rank's B pairs (captured when use_graph)."""
    from VAESNe.distributed import broadcast_parameters
    torch.manual_seed(0)
    model = make_model(device, CFG["dropout"])
    broadcast_parameters(model)
    x = synthetic_batch(B, seed + rank, device)
    step = Step(model, x, device, world, use_graph=use_graph)
    graph = False
    if use_graph:
        try:
            step.capture()
            graph = True
        except Exception as e:  # reported in the JSON line, never silent
            log(f"[bench] hipGraph capture failed ({e!r}); timing eager steps")
            step.graphs = None
            torch.cuda.synchronize(device)
    return step, graph


def strong_point(device, world, rank, args, global_batch=16):
    """The unchanged script's data parallelism: ONE DataLoader batch of 16 pairs
    (cannon/ZTF_photospect.py:76) split over the ranks as training_step does
    (training_util.py: torch.tensor_split's rule), so each rank runs global/N pairs."""
    from VAESNe.distributed import split_bounds
    lo, hi = split_bounds(global_batch, rank, world)
    step, graph = make_step(device, world, hi - lo, 4321, not args.no_graph, rank)
    dt = time_steps(step, args.steps, args.warmup, device, world)
    loss = step.loss.item()
    del step
    torch.cuda.empty_cache()
    return dict(global_batch=global_batch,
                per_gpu_batch=[b - a for a, b in (split_bounds(global_batch, r, world)
                                                  for r in range(world))],
                value=round(global_batch * args.steps / dt, 2), unit="SN pairs/s",
                ms_per_step=round(dt / args.steps * 1e3, 4), hipgraph=graph,
                finite_loss=math.isfinite(loss),
                note="total work fixed (one global batch of 16 per step, as the script's "
                     "DataLoader gives it) -- strong scaling; `value` above is weak scaling")


def config_lines(device, use_graph, steps=10, warmup=3):
    """BASELINE configs[1..3] (the other GPU configurations), each a captured training
    step (forward, backward, FusedAdamW) on synthetic inputs of its script's shape,
    with its matmul-FLOP basis from SURVEY.md §6 (FlopCounterMode, fwd + bwd):
      cfg 2  cannon/test_spectra.py:59-75      SpectraVAE 4x4, beta 1, B 32, elbo K=1
      cfg 3  cannon/test_photometry.py:52-66   PhotometricVAE 4x2, beta 0.5, B 32, elbo K=1
                                               (ZTF light curves: 2 bands, 60 epochs)
      cfg 4  cannon/test_photospectra.py:90-133 MMVAE 6 bands, beta 1, B 16, m_iwae K=2"""
    from VAESNe.PhotometricVAE import PhotometricVAE
    from VAESNe.SpectraVAE import SpectraVAE
    from VAESNe.losses import elbo, m_iwae
    from VAESNe.mmVAE import photospecMMVAE
    common = dict(model_dim=32, num_heads=4, ff_dim=32, num_layers=4, dropout=0.1, selfattn=False)
    cases = {
        "cfg2_spectra_elbo": dict(
            gf=1.783, B=32, lr=2.5e-4, loss=lambda m, x: elbo(m, x[1], K=1),
            make=lambda: SpectraVAE(latent_len=4, latent_dim=4, beta=1.0, **common),
            src="cannon/test_spectra.py:59-75"),
        "cfg3_photometry_elbo": dict(
            gf=0.027, B=32, lr=2.5e-4, loss=lambda m, x: elbo(m, x[0], K=1),
            make=lambda: PhotometricVAE(num_bands=2, latent_len=4, latent_dim=2, beta=0.5, **common),
            src="cannon/test_photometry.py:52-66 (2 ZTF bands)"),
        "cfg4_mmvae_K2": dict(
            gf=6.974, B=16, lr=1e-4, loss=lambda m, x: m_iwae(m, x, K=2),
            make=lambda: photospecMMVAE(vaes=[PhotometricVAE(num_bands=6, latent_len=4, latent_dim=4,
                                                             **common),
                                              SpectraVAE(latent_len=4, latent_dim=4, **common)],
                                        beta=1.0),
            src="cannon/test_photospectra.py:90-133"),
    }
    fixtures = {"cfg2_spectra_elbo": "elbo_spec_cfg2", "cfg3_photometry_elbo": "elbo_photo_cfg3",
                "cfg4_mmvae_K2": "mmvae_cfg4"}
    out = {}
    for name, c in cases.items():
        # parity first, on the reference's fixture of this config (its own batch of 4)
        try:
            par = golden_parity(device, fixtures[name])
            par["parity_fixture"] = f"tests/golden/{fixtures[name]}.npz"
        except Exception as e:
            par = dict(elbo_rel_err=None, parity_error=repr(e))
            log(f"[bench] {name}: parity failed: {e!r}")
        torch.cuda.empty_cache()
        torch.manual_seed(0)
        model = c["make"]().to(device)
        nb = 6 if name == "cfg4_mmvae_K2" else 2
        x = synthetic_batch(c["B"], 77, device, num_bands=nb)
        step = Step(model, x, device, 1, use_graph, loss_fn=c["loss"], lr=c["lr"])
        graph = False
        if use_graph:
            try:
                step.capture()
                graph = True
            except Exception as e:
                log(f"[bench] {name}: capture failed ({e!r}); eager")
                step.graphs = None
        dt = time_steps(step, steps, warmup, device, 1)
        v = c["B"] * steps / dt
        out[name] = dict(value=round(v, 2), unit="samples/s", batch=c["B"],
                         ms_per_step=round(dt / steps * 1e3, 4), hipgraph=graph,
                         finite_loss=math.isfinite(step.loss.item()), script=c["src"],
                         gflop_per_sample=c["gf"],
                         matmul_tflops=round(v * c["gf"] / 1e3, 3),
                         frac_fp32_peak=round(v * c["gf"] / 1e3 / FP32_PEAK_TFLOPS, 4), **par)
        del step, model, x
        torch.cuda.empty_cache()
    return out


def config_cpu_baselines():
    """the CPU oracle beside each of cfg 2/3/4 (the configs of
    config_lines), one training step (train mode, dropout 0.1, AdamW) on a bounded
    sample after a 1-sample warm-up.  Per-sample cost is linear in B (no cross-sample
    term in elbo or m_iwae)."""
    from oracle import vaesne_oracle as O
    cores, _, _ = _usable_cores()
    torch.set_num_threads(cores)
    eps = torch.finfo(torch.float32).eps
    cases = {
        "cfg2_spectra_elbo": (O.VaeCfg("spec", beta=1.0), 8, 1, 2, 2.5e-4),
        "cfg3_photometry_elbo": (O.VaeCfg("photo", num_bands=2, latent_dim=2, beta=0.5), 32, 1, 2, 2.5e-4),
        "cfg4_mmvae_K2": (O.MMVAECfg(photo=O.VaeCfg("photo", num_bands=6), spec=O.VaeCfg("spec"),
                                     beta=1.0), 4, 2, 6, 1e-4),
    }
    out = {}
    for name, (cfg, B, K, nb, lr) in cases.items():
        g = torch.Generator().manual_seed(0)
        p = O.make_params(cfg, lambda k, shp: (torch.randn(shp, generator=g) / math.sqrt(shp[-1])).numpy()
                          if "_pz" not in k else None, requires_grad=True)
        st = O.AdamWState(lr=lr)
        mm = isinstance(cfg, O.MMVAECfg)

        def one(nb_):
            x = synthetic_batch(nb_, 99, "cpu", num_bands=nb)
            for v in p.values():
                v.grad = None
            if mm:
                us = [torch.empty(K, nb_, 4, 4).uniform_(eps - 1, 1) for _ in range(2)]
                loss = O.m_iwae(p, cfg, x, K, us, p_drop=0.1, training=True)[0]
            else:
                u = torch.empty(K, nb_, cfg.latent_len, cfg.latent_dim).uniform_(eps - 1, 1)
                loss = O.elbo(p, cfg, x[1] if cfg.kind == "spec" else x[0], K, u, p_drop=0.1,
                              training=True)[0]
            (-loss).backward()
            O.adamw_step(p, {k: v.grad for k, v in p.items() if v.requires_grad}, st)
        one(1)
        t0 = time.perf_counter()
        one(B)
        dt = time.perf_counter() - t0
        out[name] = dict(value=round(B / dt, 3), unit="samples/s", cores=torch.get_num_threads(),
                         kind="port", sample=f"1 oracle training step of {B} samples after a "
                                             f"1-sample warm-up; {dt:.2f}s")
    return out


ALLREDUCE_MS_ASSUMED = 0.06   # 0.88 MB ring all-reduce over 8 GPUs' xGMI: latency-bound


def training_step_script(device, batches=32):
    """What the script runs, literally (cannon/ZTF_photospect.py:76,119-128):
    training_step(model, torch.optim.AdamW, DataLoader(multimodalDataset(...), 16),
    m_iwae K=8, multimodal=True) with HOST-resident batches (H2D copies, the loss read
    one batch late, torch's AdamW update applied behind the device skip), one timed
    epoch of `batches` batches after a warm-up epoch: as shipped (training_step
    replays its captured forward + backward, VAESNe._stepgraph) and with every batch
    eager (VAESNE_STEP_GRAPH=0).
    b2: the same loop at 2 pairs per batch, i.e. each rank's share when `torchrun
    --nproc-per-node 8` splits the script's batch of 16 (training_step shards every
    batch); with the flat-gradient all-reduce it bounds the unchanged script's 8-GPU
    strong-scaling speed-up: captured(16) / (b2 + all-reduce), the all-reduce time an
    assumption (one GPU here)."""
    from torch.utils.data import DataLoader, TensorDataset
    from VAESNe import _config, _stepgraph
    from VAESNe.data_util import multimodalDataset
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    out = {}
    saved = _config.step_graph
    try:
        for name, graph, bs in (("captured", True, 16), ("eager", False, 16), ("b2", True, 2)):
            _config.step_graph = graph
            torch.manual_seed(0)
            model = make_model(device, CFG["dropout"])
            opt = torch.optim.AdamW(model.parameters(), lr=CFG["lr"])
            x = synthetic_batch(bs * batches, 2024, "cpu")
            loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                                batch_size=bs, shuffle=False)
            fn = lambda m, xx: m_iwae(m, xx, K=CFG["K"])
            training_step(model, opt, loader, loss_fn=fn, multimodal=True)
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            loss = training_step(model, opt, loader, loss_fn=fn, multimodal=True)
            torch.cuda.synchronize(device)
            dt = (time.perf_counter() - t0) / batches
            out[name] = dict(value=round(bs / dt, 2), unit="SN pairs/s", ms_per_step=round(dt * 1e3, 3),
                             batch=bs, finite_loss=math.isfinite(loss))
            _stepgraph.clear(model)
            del model, opt
            torch.cuda.empty_cache()
    finally:
        _config.step_graph = saved
    b2 = out["b2"]["ms_per_step"]
    out["b2_ms_per_step"] = b2
    out["predicted_8gpu_strong_speedup"] = round(
        out["captured"]["ms_per_step"] / (b2 + ALLREDUCE_MS_ASSUMED), 2)
    out.update(batches=batches, optimizer="torch.optim.AdamW", allreduce_ms_assumed=ALLREDUCE_MS_ASSUMED,
               note="host-resident DataLoader batches; the headline times bench's own captured "
                    "step with FusedAdamW on HBM-resident inputs")
    return out


def launch_ranks(n, argv):
    """Start ranks 0..n-1 of this script as fresh child processes (nothing in this
    process touches the GPU), wait for them, and return the worst exit status.  A
    failing rank ends the others (their exact PIDs)."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for pr in list(live):
            code = pr.poll()
            if code is None:
                continue
            live.remove(pr)
            if code != 0:
                rc = rc or code
                for other in live:
                    other.terminate()
        time.sleep(0.2)
    return rc if rc >= 0 else 128 - rc


def rank_check(world):
    """Each rank (as launch_ranks or torchrun started it) joins a gloo group on the CPU
    and all-gathers (RANK, LOCAL_RANK, WORLD_SIZE); rank 0 prints them as JSON."""
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("VAESNE_RANK_CHECK_FAIL") == str(rank):
        sys.exit(3)        # the launcher test: one rank dies before the rendezvous
    me = [rank, int(os.environ.get("LOCAL_RANK", "0")), world]
    seen = [me]
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        seen = [None] * world
        dist.all_gather_object(seen, me)
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"world": world, "ranks": seen}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="per-GPU batch (SN pairs)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling point (N>1)")
    ap.add_argument("--throughput-batch", type=int, default=64,
                    help="also time the same step at this per-GPU batch (N=1 only; 0 = skip)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the side measurements (reconstruct K=100, contrastive step, "
                         "the scripts' training_step loop, BASELINE cfgs 2-4)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the roofline kernel launches (for rocprofv3 --pmc passes)")
    ap.add_argument("--rank-check", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group and rank 0 "
                         "prints the world it sees (tests/test_bench_launcher.py)")
    args = ap.parse_args()
    if args.roofline_only:
        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
        from VAESNe import _lib, rng
        _lib.load()
        rng.manual_seed(1234)
        print(json.dumps(roofline(device, args.batch)), flush=True)
        return

    env_ws = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if env_ws == 0 and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = max(1, env_ws)
    if args.rank_check:
        rank_check(world)
        return
    if world != args.gpus:
        log(f"[bench] --gpus {args.gpus} but the launcher describes {world} ranks: using {world}")
    rank = int(os.environ.get("RANK", "0"))
    from VAESNe.distributed import dp_backend, local_device_index
    device = torch.device("cuda", local_device_index())
    torch.cuda.set_device(device)
    backend = dp_backend() if world > 1 else None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    from VAESNe import _lib, rng
    _lib.load()
    rng.manual_seed(1234)        # each rank folds its rank in (rng.rank_seed): own noise / dropout
    step, graph = make_step(device, world, args.batch, 1234, not args.no_graph, rank)
    dt = time_steps(step, args.steps, args.warmup, device, world)
    loss = step.loss.item()
    if not math.isfinite(loss):
        raise RuntimeError(f"non-finite training loss {loss}")
    in_step = None
    if not args.no_roofline:
        in_step = in_step_kernel_times(step, args.batch)
    del step
    torch.cuda.empty_cache()
    strong = None
    if world > 1 and not args.no_strong:
        strong = strong_point(device, world, rank, args)
    ms = dt / args.steps * 1e3
    value = world * args.batch * args.steps / dt
    out = {
        "metric": "SN pairs/sec/GPU on ZTF photo+spec MMVAE step; ELBO rel-err vs CPU ref",
        "value": round(value, 2), "unit": "SN pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": CFG["workload"], "per_gpu_batch": args.batch,
                   "global_batch": args.batch * world, "K": CFG["K"], "seq_len": CFG["Ls"],
                   "photometry_len": CFG["Lp"], "num_bands": CFG["num_bands"], "beta": CFG["beta"],
                   "dropout": CFG["dropout"], "spectra_selfattn": True, "parallelism": f"dp{world}",
                   "dp_backend": backend, "hipgraph": graph},
        "value_per_gpu": round(value / world, 2),
        # whole-step rates from SURVEY.md §8(d)'s per-pair work at cfg 5 (FlopCounterMode on
        # the reference: 29.214 GFLOP of matmul fwd+bwd per pair; 262.4 M softmax scores per
        # pair in the forward), against the fp32 peak the step computes at
        "step_utilization": {
            "matmul_tflops": round(value * STEP_GFLOP_PER_PAIR / 1e3, 2),
            "frac_fp32_peak": round(value * STEP_GFLOP_PER_PAIR / 1e3 / FP32_PEAK_TFLOPS / world, 4),
            "softmax_gscores_per_s": round(value * STEP_MSCORES_PER_PAIR / 1e3, 1),
            "gflop_per_pair": STEP_GFLOP_PER_PAIR, "mscores_per_pair_fwd": STEP_MSCORES_PER_PAIR},
        "final_loss": loss,
    }
    if world == 1:
        out["strong_scaling"] = dict(global_batch=args.batch, per_gpu_batch=[args.batch],
                                     value=out["value"], unit="SN pairs/s", ms_per_step=out["ms_per_step"],
                                     note="one GPU: the headline step itself")
    elif strong is not None:
        out["strong_scaling"] = strong
    if rank == 0:
        try:
            out.update(parity(device))
        except Exception as e:
            out["elbo_rel_err"] = None
            log(f"[bench] parity failed: {e!r}")
        if not args.no_roofline:
            out["roofline"] = roofline(device, args.batch, in_step)
        if world == 1 and args.throughput_batch > 0:
            out["throughput_batch"] = throughput_point(device, args.throughput_batch, not args.no_graph)
        if world == 1 and not args.no_extras:
            ex = {}
            for name, fn in (("f", lambda: extras(device, not args.no_graph)),
                             ("configs", lambda: config_lines(device, not args.no_graph)),
                             ("training_step_script", lambda: training_step_script(device))):
                try:   # a side measurement never hides the headline line
                    r = fn()
                    ex.update(r) if name == "f" else ex.__setitem__(name, r)
                except Exception as e:
                    ex[name] = None
                    log(f"[bench] extras {name} failed: {e!r}")
            out["extras"] = ex
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
            cfgs = (out.get("extras") or {}).get("configs")
            if cfgs:
                try:
                    for name, cb in config_cpu_baselines().items():
                        if name in cfgs:
                            cfgs[name]["cpu_baseline"] = cb
                            cfgs[name]["vs_cpu"] = round(cfgs[name]["value"] / cb["value"], 1)
                except Exception as e:
                    log(f"[bench] config cpu baselines failed: {e!r}")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
