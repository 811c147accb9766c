"""Host-galaxy image transformer encoder / decoders — reference ImageLayers.py
(HostImgTransformerEncoder :6-60, HostImgTransformerDecoder :63-110,
HostImgTransformerDecoderHybrid :116-180) and the image helpers of
util_layers.py (SinusoidalPositionalEmbedding2D :62-111, PatchEmbedding :399-412).

HOST (CPU) PATH.  The image VAE is BASELINE config 1 (cannon/mnist.py), "CPU
plumbing" in SURVEY.md §8(a) a16: it runs PyTorch's own host ops and no HIP
kernel.  Its blocks are therefore separate host classes here (HostTransformerBlock,
HostMLP, ...) with the reference's attribute names — so state_dict keys, and with
them checkpoints, are the reference's — and the reference's construction order,
so `torch.manual_seed(s)` initialises the same parameters.  The HIP model classes
of util_layers are never given a host path (they raise on host tensors).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


# ---------------------------------------------------------------------------
# host building blocks (arithmetic of util_layers.py)
# ---------------------------------------------------------------------------
class HostSingleLayerMLP(nn.Module):
    """singlelayerMLP (util_layers.py:9-18): fc2(relu(fc1(x)))."""

    def __init__(self, in_dim, out_dim):
        super().__init__()
        self.fc1 = nn.Linear(in_dim, in_dim)
        self.fc2 = nn.Linear(in_dim, out_dim)

    def forward(self, x):
        return self.fc2(F.relu(self.fc1(x)))


class HostMLP(nn.Module):
    """MLP (util_layers.py:20-34): (Linear, ReLU) per hidden width, then Linear;
    keys mlp.0, mlp.2, ..."""

    def __init__(self, in_dim, out_dim, hidden_dim=[64, 64]):
        super().__init__()
        widths = [in_dim] + list(hidden_dim)
        layers = []
        for a, b in zip(widths[:-1], widths[1:]):
            layers += [nn.Linear(a, b), nn.ReLU()]
        layers.append(nn.Linear(widths[-1], out_dim))
        self.mlp = nn.Sequential(*layers)

    def forward(self, x):
        return self.mlp(x)


class HostSinusoidalMLPPositionalEmbedding(nn.Module):
    """SinusoidalMLPPositionalEmbedding (util_layers.py:131-149): [sin | cos](x * d),
    d = exp(arange(dim) * -ln(1e4) / dim), then fc2(relu(fc1(.)))."""

    def __init__(self, dim=64):
        super().__init__()
        self.dim = dim
        self.div_term = torch.exp(torch.arange(0, dim).float() * (-torch.log(torch.tensor(10000.0)) / dim))
        self.fc1 = nn.Linear(2 * dim, dim)
        self.fc2 = nn.Linear(dim, dim)

    def forward(self, x):
        arg = x[:, :, None] * self.div_term.to(x.device)[None, None, :]
        return self.fc2(F.relu(self.fc1(torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1))))


class SinusoidalPositionalEmbedding2D(nn.Module):
    """util_layers.py:62-111: fixed (H*W, d_model) table; position (y, x) of the
    row-major grid gets [sin | cos](x * w) + [sin | cos](y * w),
    w = 10000^(-arange(d/2) / (d/2)).  Non-persistent buffer (not in state_dict)."""

    def __init__(self, d_model: int, height: int, width: int):
        super().__init__()
        if d_model % 4 != 0:
            raise ValueError("d_model must be divisible by 4 for 2D sinusoidal embeddings.")
        self.d_model, self.height, self.width = d_model, height, width
        self.register_buffer('pos_embed', self._table(), persistent=False)

    def _table(self):
        H, W, half = self.height, self.width, self.d_model // 2
        ys = torch.arange(H).unsqueeze(1).repeat(1, W).flatten()
        xs = torch.arange(W).unsqueeze(0).repeat(H, 1).flatten()
        omega = 1. / (10000 ** (torch.arange(half) / half))

        def feats(pos):
            a = pos[:, None] * omega[None, :]
            return torch.cat([torch.sin(a), torch.cos(a)], dim=-1)
        return feats(xs) + feats(ys)

    def forward(self):
        return self.pos_embed


class PatchEmbedding(nn.Module):
    """util_layers.py:399-412: non-overlapping patch_size^2 patches -> embed_dim
    (a stride-patch Conv2d), tokens in row-major patch order [B, N, E]."""

    def __init__(self, img_size=224, patch_size=16, in_channels=3, embed_dim=128):
        super().__init__()
        self.img_size = img_size
        self.patch_size = patch_size
        self.num_patches = (img_size // patch_size) ** 2
        self.proj = nn.Conv2d(in_channels, embed_dim, kernel_size=patch_size, stride=patch_size)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)


class HostTransformerBlock(nn.Module):
    """TransformerBlock (util_layers.py:257-309), post-LN, on host ops:
    x = LN1(x + Drop(SelfMHA(x, kpm=mask))); [ctx = LNc(ctx + Drop(MHA(ctx)))];
    x = LN2(x + Drop(MHA(x, ctx, kpm=context_mask))); x = LN3(x + Drop(FFN(x)))."""

    def __init__(self, embed_dim, num_heads, ff_dim, dropout=0.1, context_self_attn=False):
        super().__init__()
        mha = lambda: nn.MultiheadAttention(embed_dim, num_heads, dropout=dropout, batch_first=True)
        self.self_attn = mha()
        self.cross_attn = mha()
        if context_self_attn:
            self.context_self_attn = mha()
            self.layernorm_context = nn.LayerNorm(embed_dim)
        else:
            self.context_self_attn = None
        self.ffn = nn.Sequential(nn.Linear(embed_dim, ff_dim), nn.GELU(), nn.Linear(ff_dim, embed_dim))
        self.layernorm1 = nn.LayerNorm(embed_dim)
        self.layernorm2 = nn.LayerNorm(embed_dim)
        self.layernorm3 = nn.LayerNorm(embed_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, context=None, mask=None, context_mask=None):
        a, _ = self.self_attn(x, x, x, key_padding_mask=mask)
        x = self.layernorm1(x + self.dropout(a))
        if context is not None:
            if self.context_self_attn is not None:
                c, _ = self.context_self_attn(context, context, context, key_padding_mask=context_mask)
                context = self.layernorm_context(context + self.dropout(c))
            a, _ = self.cross_attn(x, context, context, key_padding_mask=context_mask)
            x = self.layernorm2(x + self.dropout(a))
        return self.layernorm3(x + self.dropout(self.ffn(x)))


def _blocks(num_layers, model_dim, num_heads, ff_dim, dropout, selfattn):
    return nn.ModuleList([HostTransformerBlock(model_dim, num_heads, ff_dim, dropout, selfattn)
                          for _ in range(num_layers)])


# ---------------------------------------------------------------------------
# image encoder / decoders
# ---------------------------------------------------------------------------
class HostImgTransformerEncoder(nn.Module):
    """ImageLayers.py:6-60: patch tokens (+ 2-D sinusoidal or learned positions,
    + 2 event-location tokens when focal_loc) are the context of bottleneck_length
    learned query tokens; 4 blocks; bottleneckfc(x + h)."""

    def __init__(self, img_size, bottleneck_length, bottleneck_dim, patch_size=4, in_channels=3,
                 focal_loc=False, model_dim=32, num_heads=4, ff_dim=32, num_layers=4, dropout=0.1,
                 selfattn=False, sincosin=True):
        super().__init__()
        assert img_size % patch_size == 0, "image size has to be divisible to patch size"
        self.focal_loc = focal_loc
        self.model_dim = model_dim
        self.initbottleneck = nn.Parameter(torch.randn(bottleneck_length, model_dim))
        self.patch_embed = PatchEmbedding(img_size, patch_size, in_channels, model_dim)
        if sincosin:
            g = img_size // patch_size
            self.pos_embed = SinusoidalPositionalEmbedding2D(model_dim, g, g)
        else:
            self.pos_embed = nn.Parameter(torch.zeros(1, self.patch_embed.num_patches, model_dim))
        self.eventloc_embd = HostSinusoidalMLPPositionalEmbedding(model_dim) if focal_loc else None
        self.transformerblocks = _blocks(num_layers, model_dim, num_heads, ff_dim, dropout, selfattn)
        self.bottleneckfc = HostSingleLayerMLP(model_dim, bottleneck_dim)

    def forward(self, image, event_loc=None):
        tokens = self.patch_embed(image)
        pos = self.pos_embed() if callable(self.pos_embed) else self.pos_embed
        context = tokens + pos
        if self.focal_loc:
            if event_loc is None:
                event_loc = torch.zeros(context.shape[0], 2)
            context = torch.cat([context, self.eventloc_embd(event_loc)], dim=1)
        x = self.initbottleneck[None, :, :].repeat(context.shape[0], 1, 1)
        h = x
        for blk in self.transformerblocks:
            h = blk(h, context, context_mask=None)
        return self.bottleneckfc(x + h)


class HostImgTransformerDecoder(nn.Module):
    """ImageLayers.py:63-110 (hybrid=False): one token per pixel (2-D sinusoidal
    queries) cross-attending to contextfc(z); pixel head MLP (or Linear)."""

    def __init__(self, img_size, bottleneck_dim, in_channels=3, model_dim=32, num_heads=4,
                 ff_dim=32, num_layers=4, dropout=0.1, selfattn=False, mlpdecoder=True):
        super().__init__()
        self.img_size = img_size
        self.in_channels = in_channels
        self.contextfc = HostMLP(bottleneck_dim, model_dim, [model_dim])
        self.init_img_embd = SinusoidalPositionalEmbedding2D(model_dim, img_size, img_size)
        self.transformerblocks = _blocks(num_layers, model_dim, num_heads, ff_dim, dropout, selfattn)
        self.decoder = HostMLP(model_dim, in_channels, [model_dim]) if mlpdecoder \
            else nn.Linear(model_dim, in_channels)

    def forward(self, bottleneck):
        x = self.init_img_embd()[None, :, :].expand(bottleneck.shape[0], -1, -1)
        ctx = self.contextfc(bottleneck)
        h = x
        for blk in self.transformerblocks:
            h = blk(h, ctx)
        h = self.decoder(h + x)
        return h.view(x.shape[0], self.img_size, self.img_size, self.in_channels).permute(0, 3, 1, 2)


class HostImgTransformerDecoderHybrid(nn.Module):
    """ImageLayers.py:116-180 (the default): one token per patch cross-attending to
    contextfc(z), each token -> a model_dim x patch x patch block (un-patchify), then
    two 'same' Conv2d refiners model_dim -> 4 model_dim -> in_channels (kernel patch)."""

    def __init__(self, img_size, bottleneck_dim, patch_size=4, in_channels=3, model_dim=64,
                 num_heads=4, ff_dim=128, num_layers=4, dropout=0.1, selfattn=False):
        super().__init__()
        assert img_size % patch_size == 0, "patch_size must divide img_size"
        self.img_size = img_size
        self.patch_size = patch_size
        self.grid_size = img_size // patch_size
        self.num_patches = self.grid_size ** 2
        self.in_channels = in_channels
        self.contextfc = HostMLP(bottleneck_dim, model_dim, [model_dim])
        self.init_img_embd = SinusoidalPositionalEmbedding2D(model_dim, self.grid_size, self.grid_size)
        self.transformerblocks = _blocks(num_layers, model_dim, num_heads, ff_dim, dropout, selfattn)
        self.decoder = nn.Linear(model_dim, model_dim * patch_size * patch_size)
        mid = model_dim * 4
        self.final_refine = nn.Sequential(
            nn.Conv2d(model_dim, mid, kernel_size=patch_size, padding='same'),
            nn.ReLU(),
            nn.Conv2d(mid, in_channels, kernel_size=patch_size, padding='same'))

    def forward(self, bottleneck):
        B = bottleneck.size(0)
        pos = self.init_img_embd()[None, :, :].expand(B, -1, -1)
        E = pos.shape[-1]
        ctx = self.contextfc(bottleneck)
        h = pos
        for blk in self.transformerblocks:
            h = blk(h, ctx)
        h = self.decoder(h + pos)
        # token (gy, gx) holds a [py, px, E] block (feature fastest) -> image [B, E, H, W]
        g, p = self.grid_size, self.patch_size
        h = h.view(B, g, g, p, p, E).permute(0, 5, 1, 3, 2, 4).contiguous()
        return self.final_refine(h.view(B, E, self.img_size, self.img_size))
