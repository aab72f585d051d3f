"""numpy restatement of the device error sampler -- TEST INFRASTRUCTURE ONLY.

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3", SC'11; the Random123 reference algorithm), pinned by Random123's
published known-answer vectors (tests/test_philox.py), and the depolarising
sampler built on it exactly as qec_ldpc_amd/csrc/montecarlo.hip defines it
(depolarizing4): qubits 4g..4g+3 of sample b use counter (b_lo, b_hi, g, 0x51EC0DE5)
and key (seed_lo, seed_hi), word j for qubit 4g + j; hit if w < thr = floor(p 2^32)
(saturated); type = floor(w mul / 2^64), mul = min(floor(3 2^64 / thr), 2^64 - 1).
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


def multiplier(thr):
    """mul = min(floor(3 2^64 / thr), 2^64 - 1) (0 for thr = 0)."""
    if thr == 0:
        return 0
    return min((3 << 64) // thr, (1 << 64) - 1)


def depolarizing(seed, start, count, n, p):
    """(x, z) uint8 [count, n] for samples [start, start+count) of stream `seed`."""
    ng = (n + 3) // 4
    b = np.arange(start, start + count, dtype=np.uint64)[:, None]
    g = np.arange(ng, dtype=np.uint64)[None, :]
    shape = (count, ng)
    c0 = np.broadcast_to(b & MASK, shape)
    c1 = np.broadcast_to(b >> np.uint64(32), shape)
    c2 = np.broadcast_to(g, shape)
    c3 = np.full(shape, SALT, dtype=np.uint64)
    words = philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    w = np.stack(words, axis=2).reshape(count, 4 * ng)[:, :n].astype(np.uint64)  # word j -> qubit 4g + j
    thr = threshold(p)
    mul = multiplier(thr)
    hit = w < np.uint64(thr) if thr < (1 << 32) else np.ones(w.shape, bool)
    hi = w * np.uint64(mul >> 32) + ((w * np.uint64(mul & 0xFFFFFFFF)) >> np.uint64(32))
    typ = (hi >> np.uint64(32)).astype(np.uint8)
    x = (hit & (typ != 2)).astype(np.uint8)
    z = (hit & (typ != 0)).astype(np.uint8)
    return x, z
