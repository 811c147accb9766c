"""Keep-decision statistics of the attention dropout hash (csrc/common.h attn_pair_bits_mixed,
attn_row_key, attn_keypair_mix) restated in numpy: keep rate, max |r| over key lags 1..128 and
row lags 1..64, and the (row, key) rectangle differences, for the r05 form and the r06 form.
    python tools/attn_hash_stats.py"""
import numpy as np

M = np.uint64(0xffffffff)
M24 = np.uint64(0xffffff)


def mix32(x):
    x = x.astype(np.uint64) & M
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7feb352d)) & M
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846ca68b)) & M
    x ^= x >> np.uint64(16)
    return x


def decisions(form, R=4096, KP=512, key=0x12345678, thr=6554):
    key = np.uint64(key)
    rk = mix32(key ^ ((np.arange(R, dtype=np.uint64) * np.uint64(0x9e3779b1)) & M))[:, None]
    kpm = mix32((key ^ np.uint64(0x5bd1e995)) ^ ((np.arange(KP, dtype=np.uint64) * np.uint64(0x9e3779b9)) & M))[None, :]
    if form == "r05":
        x = ((((rk ^ kpm) & M24) * np.uint64(0x9e3779)) & M)
    else:   # r06: the row key through the multiply, the key-pair mix added
        x = (((rk & M24) * np.uint64(0x9e3779)) + kpm) & M
    x ^= x >> np.uint64(13)
    x = ((x & M24) * np.uint64(0x68e31d)) & M
    x ^= x >> np.uint64(16)
    k0 = (x & np.uint64(0xffff)) >= thr
    k1 = (x >> np.uint64(16)) >= thr
    return np.stack([k0, k1], -1).reshape(R, 2 * KP).astype(np.float64)


def stats(k):
    z = k - k.mean()
    v = (z * z).mean()
    kl = max(abs((z[:, :-l] * z[:, l:]).mean() / v) for l in range(1, 129))
    rl = max(abs((z[:-l] * z[l:]).mean() / v) for l in range(1, 65))
    rect = 0.0
    for dr in (1, 2, 7):
        for dk in (2, 4, 6, 32):
            a = z[:-dr, :-dk] - z[dr:, :-dk]
            b = z[:-dr, dk:] - z[dr:, dk:]
            rect = max(rect, abs((a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean())))
    return 1 - k.mean(), kl, rl, rect, 1 / np.sqrt(k.size)


if __name__ == "__main__":
    for form in ("r05", "r06"):
        rate, kl, rl, rect, noise = stats(decisions(form))
        print(f"{form}: drop rate {rate:.5f} (p 0.1)  max|r| key lags {kl:.2e}  row lags {rl:.2e}  "
              f"rectangles {rect:.2e}  (noise {noise:.1e} per lag)")
