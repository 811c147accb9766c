"""Which fp32 rounding sequence does each torch._foreach op of torch.optim.AdamW's
foreach path use on this ROCm build?  Runs each op on the GPU and compares it with
candidate formulas evaluated exactly on the host (numpy fp32 per-op rounding; fma as
the fp64 sum of the exact fp64 product, then one fp32 rounding).  Debug aid for
vaesne_adamw_list (VAESNe._update): python tools/adamw_ops_probe.py"""
import numpy as np
import torch

N = 1 << 16
f32 = np.float32


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def report(name, got, cands):
    got = got.cpu().numpy()
    for cn, c in cands.items():
        print(f"{name:10s} {cn:28s} mismatches {int((got.view(np.int32) != c.view(np.int32)).sum())}")


def main():
    g = torch.Generator().manual_seed(0)
    t = lambda s=1.0: (torch.randn(N, generator=g) * s).float()
    p, gr, m, v = t(), t(1e-2), t(1e-3), t(1e-5).abs()
    P, G, M, V = (x.numpy() for x in (p, gr, m, v))
    dev = "cuda"
    lr, wd, b1, b2, eps, step = 1e-3, 1e-2, 0.9, 0.999, 1e-8, 3.0
    decay = 1 - lr * wd
    w = 1 - b1
    vb2 = 1 - b2
    bc1 = 1 - b1 ** step
    bc2s = (1 - b2 ** step) ** 0.5
    ss = (lr / bc1) * -1

    x = [p.to(dev)]
    torch._foreach_mul_(x, decay)
    report("mul", x[0], {"p*f32(decay)": P * f32(decay)})

    x = [m.to(dev)]
    torch._foreach_lerp_(x, [gr.to(dev)], w)
    d = G - M
    report("lerp", x[0], {"m + w*(g-m)": M + f32(w) * d, "fma(w, g-m, m)": fma(np.full_like(M, f32(w)), d, M)})

    x = [v.to(dev)]
    torch._foreach_mul_(x, b2)
    vv = V * f32(b2)
    report("mul_b2", x[0], {"v*b2": vv})
    y = [vv.copy()]
    y = [torch.from_numpy(vv).to(dev)]
    torch._foreach_addcmul_(y, [gr.to(dev)], [gr.to(dev)], vb2)
    gg = G * G
    report("addcmul", y[0], {"v + s*(g*g)": vv + f32(vb2) * gg,
                             "fma(s, g*g, v)": fma(np.full_like(G, f32(vb2)), gg, vv),
                             "v + (s*g)*g": vv + (f32(vb2) * G) * G,
                             "fma(s*g, g, v)": fma(f32(vb2) * G, G, vv)})

    z = torch._foreach_sqrt([torch.from_numpy(vv).to(dev)])
    report("sqrt", z[0], {"sqrt_rn": np.sqrt(vv)})
    sq = np.sqrt(vv)
    z = [torch.from_numpy(sq).to(dev)]
    torch._foreach_div_(z, [bc2s])
    report("div", z[0], {"x / f32(bc2s)": sq / f32(bc2s), "x * f32(1/bc2s)": sq * f32(1 / bc2s)})
    den = (sq / f32(bc2s)) + f32(eps)
    z = [torch.from_numpy(sq / f32(bc2s)).to(dev)]
    torch._foreach_add_(z, eps)
    report("add_eps", z[0], {"x + eps": den})
    mm = M + f32(w) * d
    z = [torch.from_numpy(P * f32(decay)).to(dev)]
    torch._foreach_addcdiv_(z, [torch.from_numpy(mm).to(dev)], [torch.from_numpy(den).to(dev)], [ss])
    q = mm / den
    pd = P * f32(decay)
    report("addcdiv", z[0], {"p + s*(m/d)": pd + f32(ss) * q,
                             "fma(s, m/d, p)": fma(np.full_like(q, f32(ss)), q, pd),
                             "p + (s*m)/d": pd + (f32(ss) * mm) / den,
                             "fma(s*m, 1/d, p)": fma(f32(ss) * mm, f32(1) / den, pd)})


if __name__ == "__main__":
    main()
