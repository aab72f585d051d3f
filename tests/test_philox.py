"""The numpy restatement of the device sampler (oracle/philox.py): Philox4x32-10
pinned by Random123's published known-answer vectors, and the depolarising
sampler's basic properties."""
import numpy as np

from oracle.philox import SALT, depolarizing, gap_table, philox4x32_10, powsq, threshold

# Random123 kat_vectors, "philox4x32 10" lines: counter, key -> output
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_philox_known_answers():
    for c, k, out in KAT:
        got = philox4x32_10(*[np.array([x], dtype=np.uint64) for x in c], *k)
        assert tuple(int(w[0]) for w in got) == out


def test_threshold_edges():
    assert threshold(0.0) == 0 and threshold(-1) == 0
    assert threshold(1.0) == 1 << 32 and threshold(2.0) == 1 << 32
    assert threshold(0.5) == 1 << 31


def test_depolarizing_statistics_and_sharding():
    x, z = depolarizing(0x51EC0DE, 0, 4000, 610, 0.03)
    hit = x | z
    assert abs(hit.mean() - 0.03) < 0.002
    y = x & z
    # X, Y, Z each 1/3 of the hits
    for frac in ((x & ~z).sum() / hit.sum(), y.sum() / hit.sum(), (z & ~x).sum() / hit.sum()):
        assert abs(frac - 1 / 3) < 0.03
    xs, zs = depolarizing(0x51EC0DE, 1234, 100, 610, 0.03)
    assert np.array_equal(xs, x[1234:1334]) and np.array_equal(zs, z[1234:1334])
    x1, _ = depolarizing(0x51EC0DE, 0, 10, 42, 1.0)
    assert (depolarizing(0x51EC0DE, 0, 10, 42, 1.0)[0] | depolarizing(0x51EC0DE, 0, 10, 42, 1.0)[1]).all()
    x0, z0 = depolarizing(7, 0, 10, 42, 0.0)
    assert not x0.any() and not z0.any()


def test_gap_table_monotone_and_geometric():
    """T[g] = floor(q^g 2^32) is non-increasing for every p (so the count of entries above u is
    the gap), and equals the sequential product to within a unit."""
    for p in (1e-5, 1e-3, 2e-3, 0.01, 0.05, 0.1, 0.3, 0.75, 0.99):
        thr = threshold(p)
        t = gap_table(thr, 4096)
        assert (np.diff(t[1:]) <= 0).all()
        q = (2.0 ** 32 - thr) / 2.0 ** 32
        seq = 1.0
        for g in range(1, 300):
            seq *= q
            assert abs(t[g] - seq * 2.0 ** 32) <= 1.0 + 1e-9 * seq * 2.0 ** 32
    assert powsq(0.5, 10) == 0.5 ** 10 and powsq(0.0, 3) == 0.0 and powsq(0.9, 0) == 1.0


def _walk(seed, b, n, p):
    """The gap walk of one sample, word by word (pure Python, for the vectorised restatement)."""
    thr = threshold(p)
    x, z = [0] * n, [0] * n
    if thr == 0:
        return x, z
    t = gap_table(thr, n)
    words = []

    def nxt():
        k = len(words) // 4
        if len(words) == 4 * k:
            o = philox4x32_10(*[np.array([c], dtype=np.uint64) for c in (b & 0xFFFFFFFF, b >> 32, k, SALT)],
                              seed & 0xFFFFFFFF, seed >> 32)
            words.extend(int(w[0]) for w in o)
        w = words[nxt.i]
        nxt.i += 1
        return w
    nxt.i = 0
    pos = 0
    while True:
        u = nxt()
        pos += sum(1 for g in range(1, n + 1) if u < t[g])
        if pos >= n:
            break
        ty = (nxt() * 3) >> 32
        x[pos], z[pos] = int(ty != 2), int(ty != 0)
        pos += 1
        if pos >= n:
            break
    return x, z


def test_vectorised_walk_matches_word_by_word():
    for p, n, start in ((0.02, 610, 5), (0.3, 42, 2 ** 33 - 2), (1.0, 42, 0), (0.001, 610, 77)):
        x, z = depolarizing(0xC0FFEE, start, 6, n, p)
        for s in range(6):
            rx, rz = _walk(0xC0FFEE, start + s, n, p)
            assert list(x[s]) == rx and list(z[s]) == rz


def test_hits_independent_of_position():
    """Per-qubit hit rate flat over positions and no correlation between neighbours (the walk is a
    Bernoulli process, not a per-sample count)."""
    x, z = depolarizing(11, 0, 20000, 64, 0.1)
    hit = (x | z).astype(float)
    rate = hit.mean(0)
    assert np.abs(rate - 0.1).max() < 0.02
    c = np.corrcoef(hit[:, :-1].ravel(), hit[:, 1:].ravel())[0, 1]
    assert abs(c) < 0.01
