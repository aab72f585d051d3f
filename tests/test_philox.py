"""The numpy restatement of the device sampler (oracle/philox.py): Philox4x32-10
pinned by Random123's published known-answer vectors, and the depolarising
sampler's basic properties."""
import numpy as np

from oracle.philox import depolarizing, philox4x32_10, threshold

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
