"""Fused encoder latent chain (include/vaesne_hip.h: vaesne_enc_chain_*).

The latent side of an encoder's transformer stack — for each block the
self-attention over the T bottleneck tokens, LN1, the cross-attention to the data
tokens, LN2, the FFN and LN3 (util_layers.py:285-309 as called by
PhotometricLayers.py:141-142 / SpectraLayers.py:135-136) — runs as ONE forward and
ONE backward launch for all blocks, and for up to two encoders side by side.  The
per-op path (vaesne_attn_* few-query kernels + vaesne_enc_block PRE / POST halves)
takes ~4 launches per block forward and ~8 backward; in a captured step those
latency-bound chains are on the critical path before and after the decoders, and
the graph executor runs the photometry chain before the spectra chain instead of
beside it.

The context k | v projections (rows [32, 96) of each block's cross in_proj) stay
wide token-wise GEMMs over B * Lk tokens on the linear kernels; their weight
gradient lands in place in the chain's flat gradient buffer, so every block
parameter's gradient is one view of it (deferred column sums as everywhere).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _defer, _lib, _stamps, rng
from . import _ops
from ._ops import _ws, key_bias_of
from ._lib import lib, ptr, stream

MAXB = 6          # VAESNE_ENC_CHAIN_MAXB
MAXT = 8
E = 32


class Group(C.Structure):
    _fields_ = [("w", (C.c_void_p * 18) * MAXB), ("kv", C.c_void_p * MAXB),
                ("dkv", C.c_void_p * MAXB), ("call_id", (C.c_uint32 * 4) * MAXB),
                ("B", C.c_int), ("T", C.c_int), ("Lk", C.c_int), ("nb", C.c_int),
                ("p_attn", C.c_float), ("p_res", C.c_float), ("p_cross", C.c_float),
                ("rng", C.c_void_p), ("kbias", C.c_void_p), ("kbias_bs", C.c_int64),
                ("x0", C.c_void_p), ("y", C.c_void_p), ("save", C.c_void_p),
                ("dy", C.c_void_p), ("dx0", C.c_void_p), ("wpart", C.c_void_p),
                ("gflat", C.c_void_p)]


_LAYOUT = None


def layout():
    """(save floats per block, gradient floats per block, the 18 gradient offsets)"""
    global _LAYOUT
    if _LAYOUT is None:
        sb, pb = C.c_int(), C.c_int()
        off = (C.c_int * 18)()
        lib.enc_chain_layout(C.byref(sb), C.byref(pb), off)
        _LAYOUT = (sb.value, pb.value, list(off))
    return _LAYOUT


def block_params(blk):
    """The 18 tensors of one encoder TransformerBlock in the C-ABI order."""
    sa, ca = blk.self_attn, blk.cross_attn
    return [sa.in_proj_weight, sa.in_proj_bias, sa.out_proj.weight, sa.out_proj.bias,
            blk.layernorm1.weight, blk.layernorm1.bias, ca.in_proj_weight, ca.in_proj_bias,
            ca.out_proj.weight, ca.out_proj.bias, blk.layernorm2.weight, blk.layernorm2.bias,
            blk.ffn[0].weight, blk.ffn[0].bias, blk.ffn[2].weight, blk.ffn[2].bias,
            blk.layernorm3.weight, blk.layernorm3.bias]


def fusable(blocks, x) -> bool:
    """Shapes the chain kernels cover: E 32, 4 heads, ff 32, LN eps 1e-5, biases,
    one dropout rate per kind across the blocks, T <= 8, nb <= MAXB."""
    if not blocks or len(blocks) > MAXB or x.dim() != 3 or x.shape[1] > MAXT or x.shape[-1] != E:
        return False
    b0 = blocks[0]
    for b in blocks:
        sa, ca = b.self_attn, b.cross_attn
        if (sa.embed_dim != E or sa.num_heads != 4 or ca.num_heads != 4 or ca.embed_dim != E
                or b.ffn[0].out_features != E or b.ffn[0].in_features != E
                or sa.in_proj_bias is None or ca.in_proj_bias is None
                or sa.out_proj.bias is None or ca.out_proj.bias is None
                or any(ln.eps != 1e-5 for ln in (b.layernorm1, b.layernorm2, b.layernorm3))
                or sa.dropout != b0.self_attn.dropout or ca.dropout != b0.cross_attn.dropout
                or b.dropout.p != b0.dropout.p or b.training != b0.training):
            return False
    return True


class Spec:
    """One encoder's chain: nb blocks, context shared by every block (`shared`) or
    one context per block, key bias (or None), dropout rates and call ids."""

    def __init__(self, nb, shared, kbias, probs, call_ids):
        self.nb, self.shared, self.kbias = nb, shared, kbias
        self.probs, self.call_ids = probs, call_ids


def reserve_call_ids(blocks):
    """The call ids the per-op path would draw for these blocks, in its order
    (per block: self-attention, PRE residual, cross-attention, POST residual;
    0 where that dropout is off): identical masks to the per-op path."""
    ids = []
    for b in blocks:
        pa = b.self_attn.dropout if b.training else 0.0
        p = b.dropout.p if b.training else 0.0
        pc = b.cross_attn.dropout if b.training else 0.0
        row = [rng.next_call_id() if pa > 0 else 0, rng.next_call_id() if p > 0 else 0,
               rng.next_call_id() if pc > 0 else 0, rng.next_call_id() if p > 0 else 0]
        ids.append(row)
    return ids


def make_spec(blocks, context_mask, shared, call_ids=None):
    b0 = blocks[0]
    tr = b0.training
    probs = (b0.self_attn.dropout if tr else 0.0, b0.dropout.p if tr else 0.0,
             b0.cross_attn.dropout if tr else 0.0)
    return Spec(len(blocks), shared, key_bias_of(context_mask), probs,
                call_ids if call_ids is not None else reserve_call_ids(blocks))


class EncChainFn(torch.autograd.Function):
    """specs (one Spec per encoder) + per encoder [x0 [B, T, 32], context(s) [B, Lk, 32]
    (1 if shared else nb), 18 * nb block tensors] -> one h [B, T, 32] per encoder."""

    @staticmethod
    def forward(ctx, specs, *flat):
        save_blk, _, _ = layout()
        G = len(specs)
        groups = (Group * G)()
        s = stream()
        per = []
        pos = 0
        outs = []
        kv_rows = []
        for gi, sp in enumerate(specs):
            nb = sp.nb
            x0 = flat[pos]
            nctx = 1 if sp.shared else nb
            ctxs = list(flat[pos + 1:pos + 1 + nctx])
            params = list(flat[pos + 1 + nctx:pos + 1 + nctx + 18 * nb])
            pos += 1 + nctx + 18 * nb
            _lib.require_device(x0, *ctxs, *params)
            _defer.count_uses(*params)
            x0 = x0.contiguous()
            ctxs = [c.contiguous() for c in ctxs]
            params = [t.contiguous() for t in params]
            B, T, _ = x0.shape
            Lk = ctxs[0].shape[1]
            if any(c.shape != (B, Lk, E) for c in ctxs):
                raise RuntimeError("EncChainFn: every context must be [B, Lk, 32]")
            dev = x0.device
            kv = torch.empty((nb, B, Lk, 2 * E), dtype=torch.float32, device=dev)
            for blk in range(nb):      # the k | v projections: one grouped launch below
                c = ctxs[0 if sp.shared else blk]
                Wc, bc = params[18 * blk + 6], params[18 * blk + 7]
                kv_rows.append((c.data_ptr(), E, Wc.data_ptr() + 4 * E * E, bc.data_ptr() + 4 * E,
                                kv[blk].data_ptr(), 2 * E, B * Lk, 0))
            y = torch.empty((B, T, E), dtype=torch.float32, device=dev)
            save = torch.empty((B, nb, save_blk), dtype=torch.float32, device=dev)
            st = rng.state(dev) if any(p > 0 for p in sp.probs) else None
            kb = sp.kbias.contiguous() if sp.kbias is not None else None
            g = groups[gi]
            for blk in range(nb):
                for j in range(18):
                    g.w[blk][j] = params[18 * blk + j].data_ptr()
                g.kv[blk] = kv[blk].data_ptr()
                for j in range(4):
                    g.call_id[blk][j] = sp.call_ids[blk][j]
            g.B, g.T, g.Lk, g.nb = B, T, Lk, nb
            g.p_attn, g.p_res, g.p_cross = (float(p) for p in sp.probs)
            g.rng = ptr(st)
            g.kbias = ptr(kb)
            g.kbias_bs = Lk if kb is None else kb.stride(0)
            g.x0, g.y, g.save = x0.data_ptr(), y.data_ptr(), save.data_ptr()
            per.append((sp, B, T, Lk, nctx, ctxs, params, kv, save, st, kb, x0.shape))
            outs.append(y)
        for i in range(0, len(kv_rows), 8):
            chunk = kv_rows[i:i + 8]
            lib.linear_fwd_group(len(chunk), _ops.lin_groups(chunk), E, 2 * E, s)
        lib.enc_chain_fwd(G, groups, s)
        ctx.per = [(sp, B, T, Lk, nctx, xs) for sp, B, T, Lk, nctx, _, _, _, _, _, _, xs in per]
        tensors = []
        for _, _, _, _, _, ctxs, params, kv, save, st, kb, _ in per:
            tensors += [kv, save, st, kb] + ctxs + params
        ctx.save_for_backward(*tensors)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *dys):
        _, pblk, offs = layout()
        saved = list(ctx.saved_tensors)
        G = len(ctx.per)
        groups = (Group * G)()
        s = stream()
        ng = ctx.needs_input_grad
        keep, all_params, all_out, res = [], [], [], []
        work = []
        pos_in = 1                     # needs_input_grad index (0 = specs)
        for gi, (sp, B, T, Lk, nctx, xshape) in enumerate(ctx.per):
            nb = sp.nb
            kv, save, st, kb = saved[:4]
            ctxs = saved[4:4 + nctx]
            params = saved[4 + nctx:4 + nctx + 18 * nb]
            del saved[:4 + nctx + 18 * nb]
            dev = kv.device
            dy = dys[gi]
            dy = torch.zeros(xshape, dtype=torch.float32, device=dev) if dy is None \
                else dy.contiguous()
            dx0 = torch.empty(xshape, dtype=torch.float32, device=dev)
            dkv = torch.empty_like(kv)
            wpart = torch.empty((B, nb * pblk), dtype=torch.float32, device=dev)
            gflat = torch.empty(nb * pblk, dtype=torch.float32, device=dev)
            gviews = []
            for blk in range(nb):
                for j in range(18):
                    o = blk * pblk + offs[j]
                    t = params[18 * blk + j]
                    gviews.append(gflat[o:o + t.numel()].view_as(t))
            need_p = ng[pos_in + 1 + nctx:pos_in + 1 + nctx + 18 * nb]
            all_params += params
            all_out += [gv if n else None for gv, n in zip(gviews, need_p)]
            wsk = _ws(lib.linear_bwd_weight_group_workspace(nb, B * Lk, 2 * E, E), dev)
            keep += [wpart, gflat, wsk]
            g = groups[gi]
            for blk in range(nb):
                for j in range(18):
                    g.w[blk][j] = params[18 * blk + j].data_ptr()
                g.kv[blk] = kv[blk].data_ptr()
                g.dkv[blk] = dkv[blk].data_ptr()
                for j in range(4):
                    g.call_id[blk][j] = sp.call_ids[blk][j]
            g.B, g.T, g.Lk, g.nb = B, T, Lk, nb
            g.p_attn, g.p_res, g.p_cross = (float(p) for p in sp.probs)
            g.rng = ptr(st)
            g.kbias = ptr(kb)
            g.kbias_bs = Lk if kb is None else kb.stride(0)
            g.x0 = 0
            g.y = 0
            g.save = save.data_ptr()
            g.dy, g.dx0 = dy.data_ptr(), dx0.data_ptr()
            g.wpart, g.gflat = wpart.data_ptr(), gflat.data_ptr()
            work.append((sp, B, Lk, nctx, ctxs, params, dkv, gflat, gviews, wsk, dx0, dy))
            pos_in += 1 + nctx + 18 * nb
        dfr = _defer.target(all_params, all_out, keep, entries=sum(
            5 * w[0].nb + 2 for w in work) + 2)
        _stamps.mark("enc_chain_bwd" + "_".join(str(w[2]) for w in work))
        lib.enc_chain_bwd(G, groups, dfr, s)
        _stamps.mark("enc_chain_bwd_end")
        grads = []
        # the context gradients first (the context paths' backward waits for them), the k | v
        # projection weight gradients (read only by the flush) after every item's
        for sp, B, Lk, nctx, ctxs, params, dkv, gflat, gviews, wsk, dx0, dy in work:
            nb = sp.nb
            M = B * Lk
            if sp.shared:
                # dctx = sum_blk dkv_blk Wkv_blk: per-block products in one launch, then one
                # fixed-order sum over the blocks
                part = torch.empty((nb, M, E), dtype=torch.float32, device=kv.device)
                rows = [(dkv[blk].data_ptr(), 2 * E, params[18 * blk + 6].data_ptr() + 4 * E * E,
                         None, part[blk].data_ptr(), E, M, 0) for blk in range(nb)]
                lib.linear_bwd_data_group(nb, _ops.lin_groups(rows), E, 2 * E, s)
                dctx = torch.empty_like(ctxs[0])
                lib.sum_leading(part.data_ptr(), nb, M * E, dctx.data_ptr(), 0, s)
                dctxs = [dctx]
            else:
                dctxs = [torch.empty_like(ctxs[blk]) for blk in range(nb)]
                rows = [(dkv[blk].data_ptr(), 2 * E, params[18 * blk + 6].data_ptr() + 4 * E * E,
                         None, dctxs[blk].data_ptr(), E, M, 0) for blk in range(nb)]
                lib.linear_bwd_data_group(nb, _ops.lin_groups(rows), E, 2 * E, s)
            grads += [dx0] + dctxs + gviews
            _stamps.mark(f"enc_dctx{Lk}")
        for sp, B, Lk, nctx, ctxs, params, dkv, gflat, gviews, wsk, dx0, dy in work:
            rows = []
            for blk in range(sp.nb):    # k | v projection weight gradients, in place in gflat
                c = ctxs[0 if sp.shared else blk]
                o = blk * pblk + offs[6]
                rows.append((dkv[blk].data_ptr(), 2 * E, c.data_ptr(), E,
                             gflat.data_ptr() + 4 * (o + E * E),
                             gflat.data_ptr() + 4 * (blk * pblk + offs[7] + E)))
            lib.linear_bwd_weight_group(sp.nb, _ops.wgt_groups(rows), B * Lk, 2 * E, E,
                                        wsk.data_ptr(), dfr, s)
        out = [None]
        for i, gr in enumerate(grads):
            out.append(gr if ng[1 + i] else None)
        return tuple(out)


def enc_chain(items):
    """items: list of (Spec, x0 [B, T, 32], contexts (list), blocks) -> list of h."""
    specs, flat = [], []
    for sp, x0, ctxs, blocks in items:
        specs.append(sp)
        flat.append(x0)
        flat += list(ctxs)
        for b in blocks:
            flat += block_params(b)
    return list(EncChainFn.apply(specs, *flat))


def drive(gens):
    """Run encoder generators (util_layers.encoder_stack_steps and the layers above
    it) together: advance each to its chain item in order, launch every item as ONE
    grouped chain (groups of two per kernel), resume each with its output in order,
    and return their results.  A generator that yields None computes its output
    itself."""
    items = [next(g) for g in gens]
    idx = [i for i, it in enumerate(items) if it is not None]
    hs = dict(zip(idx, enc_chain([items[i] for i in idx]))) if idx else {}
    out = []
    for i, g in enumerate(gens):
        try:
            g.send(hs.get(i))
        except StopIteration as e:
            out.append(e.value)
            continue
        raise RuntimeError("encoder step generator yielded more than once")
    return out
