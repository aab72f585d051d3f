"""numpy restatement of the device error sampler -- TEST INFRASTRUCTURE ONLY.

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3", SC'11; the Random123 reference algorithm), pinned by Random123's
published known-answer vectors (tests/test_philox.py), and the depolarising
sampler built on it exactly as qec_ldpc_amd/csrc/montecarlo.hip defines it
(gap_sample):

* thr = floor(p 2^32) (saturated at 2^32); q = 1 - thr / 2^32 (exact in double);
  gap table T[g] = floor(q^g 2^32) for g = 1..n, q^g by right-to-left binary
  exponentiation in IEEE double (powsq below; the device runs the same operations).
* Sample b walks its qubits 0..n-1 in order, drawing 32-bit words from Philox calls
  k = 0, 1, ... with counter (b_lo, b_hi, k, 0x6A9C0DE5) and key (seed_lo, seed_hi),
  word 4k + j = output word j of call k.  Repeat: u = next word; the gap
  G = #{g in 1..n : u < T[g]} qubits are skipped (P(G >= g) = q^g to within 2^-32,
  i.e. each qubit is hit with probability thr / 2^32, independently); if the
  position passes n the sample is done; else the qubit there is hit, its type is
  t = floor(3 w / 2^32) of the next word w (0 = X, 1 = Y, 2 = Z; Y sets both bits),
  and the walk continues from the next qubit.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
SALT = 0x6A9C0DE5
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


def powsq(q, g):
    """q^g by right-to-left binary exponentiation (IEEE double, the device's order)."""
    r, b, e = 1.0, q, g
    while e:
        if e & 1:
            r = r * b
        e >>= 1
        if e:
            b = b * b
    return r


def gap_table(thr, n):
    """T[0..n] (T[0] unused, 0): T[g] = floor(q^g 2^32), q = 1 - thr / 2^32."""
    q = (4294967296.0 - thr) / 4294967296.0
    t = np.zeros(n + 1, dtype=np.int64)
    for g in range(1, n + 1):
        t[g] = int(powsq(q, g) * 4294967296.0)
    return t


def depolarizing(seed, start, count, n, p):
    """(x, z) uint8 [count, n] for samples [start, start+count) of stream `seed`."""
    x = np.zeros((count, n), dtype=np.uint8)
    z = np.zeros((count, n), dtype=np.uint8)
    thr = threshold(p)
    if thr == 0 or n == 0 or count == 0:
        return x, z
    negT = -gap_table(thr, n)[1:]  # ascending: G = #{g : u < T[g]} = #{g : -T[g] < -u}
    b = np.arange(start, start + count, dtype=np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF

    def word(idx, wi):
        k = (wi // 4).astype(np.uint64)
        o = philox4x32_10(b[idx] & MASK, b[idx] >> np.uint64(32), k, np.full(len(idx), SALT, np.uint64), k0, k1)
        return np.choose(wi % 4, o).astype(np.int64)

    pos = np.zeros(count, dtype=np.int64)
    wi = np.zeros(count, dtype=np.int64)
    idx = np.arange(count)
    while len(idx):
        u = word(idx, wi[idx])
        wi[idx] += 1
        pos[idx] += np.searchsorted(negT, -u, side="left")
        idx = idx[pos[idx] < n]
        if not len(idx):
            break
        t = (word(idx, wi[idx]) * 3) >> 32
        wi[idx] += 1
        v = pos[idx]
        x[idx, v] = t != 2
        z[idx, v] = t != 0
        pos[idx] += 1
        idx = idx[pos[idx] < n]
    return x, z
