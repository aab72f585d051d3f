"""numpy restatement of the device error sampler -- TEST INFRASTRUCTURE ONLY.

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3", SC'11; the Random123 reference algorithm), pinned by Random123's
published known-answer vectors (tests/test_philox.py), and the depolarising
sampler built on it exactly as qec_ldpc_amd/csrc/montecarlo.hip defines it:
qubit v of sample b uses counter (b_lo, b_hi, v, 0x51EC0DE5) and key
(seed_lo, seed_hi); hit if word0 < floor(p 2^32) (saturated), type = (word1*3)>>32.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
SALT = 0x51EC0DE5
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK for c in (c0, c1, c2, c3))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return tuple(x.astype(np.uint32) for x in (c0, c1, c2, c3))


def threshold(p):
    p = float(np.float32(p))
    if p <= 0.0:
        return 0
    if p >= 1.0:
        return 1 << 32
    return int(p * 4294967296.0)


def depolarizing(seed, start, count, n, p):
    """(x, z) uint8 [count, n] for samples [start, start+count) of stream `seed`."""
    b = np.arange(start, start + count, dtype=np.uint64)[:, None]
    v = np.arange(n, dtype=np.uint64)[None, :]
    shape = (count, n)
    c0 = np.broadcast_to(b & MASK, shape)
    c1 = np.broadcast_to(b >> np.uint64(32), shape)
    c2 = np.broadcast_to(v, shape)
    c3 = np.full(shape, SALT, dtype=np.uint64)
    w0, w1, _, _ = philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    hit = w0.astype(np.uint64) < np.uint64(threshold(p)) if threshold(p) < (1 << 32) else np.ones(shape, bool)
    typ = ((w1.astype(np.uint64) * np.uint64(3)) >> np.uint64(32)).astype(np.uint8)
    x = (hit & (typ != 2)).astype(np.uint8)
    z = (hit & (typ != 0)).astype(np.uint8)
    return x, z
