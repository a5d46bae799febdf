"""Statistics of LoRA-dropout mask hashes (ospo_amd/dropout.py drop_hash, common.h): keep rate and the
correlation of keep decisions between the two halves of one hash, rows 1-64 and columns 2-256 apart, on a
[4800, 4096] mask at p = 0.05, 4 seeds, worst |value| x 1e-4 (sampling noise ~2.3e-4).  'old' = the round-3
hash (three 32-bit multiplies), 'h2' / 'h2b' = rejected cheaper candidates, 'h3' = the round-4 hash."""
import numpy as np
def mul24(x, c):
    return (x & np.uint32(0xFFFFFF)) * np.uint32(c)
def old(i, s):
    with np.errstate(over="ignore"):
        x = i.astype(np.uint32) * np.uint32(0x9E3779B1) + np.uint32(s)
        x ^= x >> np.uint32(16); x *= np.uint32(0x7FEB352D); x ^= x >> np.uint32(15); x *= np.uint32(0x846CA68B); x ^= x >> np.uint32(16)
    return x
def h2(i, s, cs=(0xED5AD5, 0xAC4C1B), shs=(16, 13, 16)):
    with np.errstate(over="ignore"):
        x = i.astype(np.uint32) ^ np.uint32(s)
        x ^= x >> np.uint32(shs[0])
        for c, sh in zip(cs, shs[1:]):
            x = mul24(x, c); x ^= x >> np.uint32(sh)
    return x
def h3(i, s):
    return h2(i, s, cs=(0xED5AD5, 0xAC4C1B, 0x9E3779), shs=(16, 15, 13, 16))
def h2b(i, s):  # seed added after the first multiply
    with np.errstate(over="ignore"):
        x = i.astype(np.uint32)
        x ^= x >> np.uint32(16); x = mul24(x, 0xED5AD5) + np.uint32(s); x ^= x >> np.uint32(15)
        x = mul24(x, 0xAC4C1B); x ^= x >> np.uint32(16)
    return x
def keep(h, thr):
    return np.stack([(h & np.uint32(0xFFFF)) >= thr, (h >> np.uint32(16)) >= thr], -1).reshape(-1)
rng = np.random.default_rng(0)
p = 0.05; thr = int(p * 65536)
M, K = 4800, 4096
i = np.arange(M * K // 2, dtype=np.uint64).astype(np.uint32)
for name, f in (("old", old), ("h2", h2), ("h3", h3), ("h2b", h2b)):
    worst = {}
    for trial in range(4):
        s = int(rng.integers(0, 2**32))
        k = keep(f(i, s), thr).reshape(M, K).astype(np.float32)
        rate = k.mean(); d = k - rate; var = rate * (1 - rate)
        res = {"rate": rate - 0.95, "adj": (d[:, 0::2] * d[:, 1::2]).mean() / var}
        for r in (1, 2, 4, 8, 16, 64):
            res[f"row{r}"] = (d[r:] * d[:-r]).mean() / var
        for c in (2, 4, 8, 64, 256):
            res[f"col{c}"] = (d[:, c:] * d[:, :-c]).mean() / var
        for kk, v in res.items():
            worst[kk] = max(worst.get(kk, 0), abs(float(v)))
    print(name, " ".join(f"{k}:{v*1e4:.1f}" for k, v in worst.items()), "(x1e-4)")
