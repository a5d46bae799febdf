"""Statistics of LoRA-dropout mask hashes (ospo_amd/dropout.py drop_hash, common.h).

Round 5: the round-4 hash ('h3') multiplied only the low 24 bits of its state and dropped
the top byte, so pair indices p and p ^ 0x01000100 collide for every seed, and for two seeds
h(p, s1) = h(p ^ s1 ^ s2, s2).  'h4' (3 rounds) and 'h5' (4 rounds) keep every step a 32-bit bijection
(lo24(x) * c + top byte: v_and + v_mad_u32_u24 per round) and key the seed in after the first round; 'h6', the
round-5 hash, has h5's structure with each round x + lo24(x) * c (c even), one v_mad_u32_u24 (x, c, x).

Per hash, on [4800, 4096] (the q|k|v / o / gate|up inputs) and [4800, 11008] (the down input, 26.4 M pairs,
beyond 2^24) masks at p = 0.05 and 4 seeds, worst |value| x 1e-4 (sampling noise ~2.3e-4 / ~1.4e-4):
  rate    keep rate - 0.95
  adj     correlation of the two halves of one hash (adjacent elements)
  rowL    correlation of rows L apart (1 ... 64, and 3040-3056 around the old collision lag)
  colC    correlation of columns C apart
  coll    fraction of pairs p < n / 2 whose hash equals that of p ^ 0x01000100 (the old collision)
  xseed   correlation of mask(s1)[p] with mask(s2)[p ^ s1 ^ s2] (the old cross-seed re-indexing)
  aval    worst |P(output bit j flips when input bit i flips) - 0.5| over random inputs (x 1e-4)
  uniq    distinct hashes / pairs of the [4800, 11008] mask (1 = no two pairs share a hash)
"""
import sys

import numpy as np


def mul24(x, c):
    return (x & np.uint32(0xFFFFFF)) * np.uint32(c)


def mix24(x, c):
    return (x & np.uint32(0xFFFFFF)) * np.uint32(c) + (x & np.uint32(0xFF000000))


def h3(i, s):  # round 4
    with np.errstate(over="ignore"):
        x = i.astype(np.uint32) ^ np.uint32(s)
        x ^= x >> np.uint32(16)
        for c, sh in zip((0xED5AD5, 0xAC4C1B, 0x9E3779), (15, 13, 16)):
            x = mul24(x, c)
            x ^= x >> np.uint32(sh)
    return x


def _hk(i, s, rounds):
    with np.errstate(over="ignore"):
        x = mix24(i.astype(np.uint32), 0xED5AD5)
        x ^= x >> np.uint32(16)
        x ^= np.uint32(s)
        for c, sh in rounds:
            x = mix24(x, c)
            x ^= x >> np.uint32(sh)
    return x


def h4(i, s):  # 3 rounds
    return _hk(i, s, ((0xAC4C1B, 15), (0x9E3779, 16)))


def h5(i, s):  # 4 rounds, lo24(x) * c + top byte (and + mad per round)
    return _hk(i, s, ((0xAC4C1B, 15), (0x9E3779, 13), (0xC2B2AF, 16)))


def madself(x, c):  # x + lo24(x) * c, c even: one v_mad_u32_u24 (x, c, x); bijective since c + 1 is odd
    return (x & np.uint32(0xFFFFFF)) * np.uint32(c) + x


def h6(i, s):  # the round-5 hash (common.h drop_hash): h5's rounds as one mad each
    with np.errstate(over="ignore"):
        x = madself(i.astype(np.uint32), 0xED5AD4)
        x ^= x >> np.uint32(16)
        x ^= np.uint32(s)
        for c, sh in ((0xAC4C1A, 15), (0x9E3778, 13), (0xC2B2AE, 16)):
            x = madself(x, c)
            x ^= x >> np.uint32(sh)
    return x


def keep(h, thr):
    return np.stack([(h & np.uint32(0xFFFF)) >= thr, (h >> np.uint32(16)) >= thr], -1).reshape(-1)


def lagcorr(d, var, r=0, c=0):
    a = d[r:, c:]
    b = d[: d.shape[0] - r, : d.shape[1] - c]
    return (a * b).mean() / var


def stats(f, M, K, rng, thr, p):
    worst = {}
    i = np.arange(M * K // 2, dtype=np.uint64).astype(np.uint32)
    for trial in range(4):
        s = int(rng.integers(0, 2**32))
        k = keep(f(i, s), thr).reshape(M, K).astype(np.float32)
        rate = k.mean()
        d = k - rate
        var = rate * (1 - rate)
        res = {"rate": rate - (1 - p), "adj": (d[:, 0::2] * d[:, 1::2]).mean() / var}
        for r in (1, 2, 4, 8, 16, 64):
            res[f"row{r}"] = lagcorr(d, var, r=r)
        res["row3040-3056"] = max(abs(lagcorr(d, var, r=r)) for r in range(3040, 3057, 2)) if M > 3100 else 0.0
        for c in (2, 4, 8, 64, 256):
            res[f"col{c}"] = lagcorr(d, var, c=c)
        res["coll"] = float((f(i, s) == f(i ^ np.uint32(0x01000100), s)).mean())
        s2 = int(rng.integers(0, 2**32))
        k2 = keep(f(i ^ np.uint32(s ^ s2), s2), thr).astype(np.float32)
        res["xseed"] = ((k.reshape(-1) - rate) * (k2 - k2.mean())).mean() / var
        for kk, v in res.items():
            worst[kk] = max(worst.get(kk, 0), abs(float(v)))
    return worst


def avalanche(f, rng, n=1 << 16):
    worst = 0.0
    x = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for s in rng.integers(0, 2**32, 2, dtype=np.uint64):
        h = f(x, int(s))
        for b in range(32):
            d = h ^ f(x ^ np.uint32(1 << b), int(s))
            bits = (d[:, None] >> np.arange(32, dtype=np.uint32)) & np.uint32(1)
            worst = max(worst, float(np.abs(bits.mean(0) - 0.5).max()))
    return worst


def main():
    rng = np.random.default_rng(0)
    p = 0.05
    thr = int(p * 65536)
    for name, f in ((a, globals()[a]) for a in (sys.argv[1:] or ("h3", "h4", "h5", "h6"))):
        for M, K in ((4800, 4096), (4800, 11008)):
            w = stats(f, M, K, rng, thr, p)
            print(name, f"[{M},{K}]", " ".join(f"{k}:{v * 1e4:.1f}" for k, v in w.items()), "(x1e-4)")
        hh = f(np.arange(4800 * 11008 // 2, dtype=np.uint32), 12345)
        print(name, f"aval:{avalanche(f, rng) * 1e4:.0f} (x1e-4)  uniq:{np.unique(hh).size / hh.size:.6f}")


if __name__ == "__main__":
    main()
