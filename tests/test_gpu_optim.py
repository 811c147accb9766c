"""FusedAdamW against torch.optim.AdamW (the cannon scripts' optimizer): per-parameter
step counts (a parameter that first gets a gradient late gets step-1 bias correction,
skipped while its .grad is None) and the state_dict format both ways."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(33, 7, generator=g), torch.randn(5, generator=g),
            torch.randn(4, 4, 4, generator=g)]


def _grads(step, seed):
    g = torch.Generator().manual_seed(1000 + step + seed)
    gs = [torch.randn(33, 7, generator=g), torch.randn(5, generator=g),
          torch.randn(4, 4, 4, generator=g)]
    if step == 0:
        gs[1] = None          # parameter 1 starts late: its first step is step 1
    if step == 2:
        gs[2] = None          # parameter 2 skips a step
    return gs


def _run(opt_cls, steps, seed=0, state=None, start=0):
    ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in _params(seed)]
    opt = opt_cls(ps, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.05)
    if state is not None:
        with torch.no_grad():
            for p, t in zip(ps, state[0]):
                p.copy_(t)
        opt.load_state_dict(state[1])
    for s in range(start, start + steps):
        for p, gr in zip(ps, _grads(s, seed)):
            p.grad = None if gr is None else gr.to(DEV)
        opt.step()
    torch.cuda.synchronize()
    return [p.detach().clone() for p in ps], opt


def test_fused_adamw_matches_torch_adamw_with_late_and_skipped_parameters():
    from VAESNe.optim import FusedAdamW
    ref, _ = _run(torch.optim.AdamW, 5)
    got, _ = _run(FusedAdamW, 5)
    for a, b in zip(got, ref):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (a - b).abs().max()


@pytest.mark.parametrize("src,dst", [("torch", "fused"), ("fused", "torch"), ("fused", "fused")])
def test_state_dict_round_trip_between_optimizers(src, dst):
    from VAESNe.optim import FusedAdamW
    cls = {"torch": torch.optim.AdamW, "fused": FusedAdamW}
    params, opt = _run(cls[src], 3)
    sd = opt.state_dict()
    assert set(sd["state"]) == {0, 1, 2}
    assert float(sd["state"][1]["step"]) == 2.0 and float(sd["state"][2]["step"]) == 2.0
    cont, _ = _run(cls[dst], 2, state=(params, sd), start=3)
    ref, _ = _run(torch.optim.AdamW, 5)
    for a, b in zip(cont, ref):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (a - b).abs().max()


def test_flagged_step_changes_nothing():
    """A set non-finite guard flag handed to the update kernels (training_step passes
    it as apply_update's skip) makes them no-ops: parameters, moments and step counts
    unchanged, as inside a captured step where nothing on the host can intervene.
    Clearing the flag lets the next step update as usual."""
    from VAESNe import guard
    from VAESNe.optim import FusedAdamW
    ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in _params(0)]
    opt = FusedAdamW(ps, lr=1e-2)
    for p, gr in zip(ps, _grads(1, 0)):
        p.grad = gr.to(DEV)
    fl = opt._flat[0]
    before = [fl[k].clone() for k in ("flat", "m", "v", "steps")]
    guard.flag(DEV)[1] = 1
    try:
        opt.pack_grads()
        opt.apply_update(skip=guard.ptr(fl["flat"]))
        torch.cuda.synchronize()
        for k, b in zip(("flat", "m", "v", "steps"), before):
            assert torch.equal(fl[k], b), k
    finally:
        guard.reset(DEV)
    opt.pack_grads()
    opt.apply_update(skip=guard.ptr(fl["flat"]))
    torch.cuda.synchronize()
    assert not torch.equal(fl["flat"], before[0]) and float(fl["steps"].max()) == 1.0


def test_plain_step_ignores_a_stale_flag():
    """a custom loop (the reference's *2goldstein_* scripts call
    optimizer.step() themselves) after an eval forward that flagged a NaN: FusedAdamW's
    plain step() updates, as torch.optim.AdamW would -- no silently dropped steps."""
    from VAESNe import guard
    from VAESNe.optim import FusedAdamW
    ref, _ = _run(torch.optim.AdamW, 3)
    guard.flag(DEV)[0] = 1           # left behind by an unchecked eval call
    try:
        got, opt = _run(FusedAdamW, 3)
        assert float(opt._flat[0]["steps"].max()) == 3.0
        for a, b in zip(got, ref):
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (a - b).abs().max()
    finally:
        guard.reset(DEV)


def test_load_state_dict_refuses_amsgrad_and_maximize():
    from VAESNe.optim import FusedAdamW
    for k in ("amsgrad", "maximize"):
        ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in _params(0)]
        sd = torch.optim.AdamW(ps, lr=1e-2, **{k: True}).state_dict()
        with pytest.raises(ValueError, match=k):
            FusedAdamW(ps, lr=1e-2).load_state_dict(sd)
    ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in _params(0)]
    sd = torch.optim.AdamW(ps, lr=3e-3, betas=(0.8, 0.9), foreach=False).state_dict()
    opt = FusedAdamW(ps, lr=1e-2)
    opt.load_state_dict(sd)
    g = opt.param_groups[0]
    assert g["lr"] == 3e-3 and tuple(g["betas"]) == (0.8, 0.9) and "foreach" not in g
