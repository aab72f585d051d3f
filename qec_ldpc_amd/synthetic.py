"""Synthetic depolarising inputs for the benchmark and tests.

Each qubit is hit with probability p; a hit is X, Y or Z with probability 1/3 each
(Y sets both bits).  Randomness is counter-based so that any shard of the sample
index space can be generated independently and gives the same samples whatever
the number of ranks: samples are grouped in blocks of BLOCK, and block k is drawn
from numpy's Philox bit generator keyed by (seed, k).
"""
import numpy as np

BLOCK = 4096
DEFAULT_SEED = 0x51EC0DE


def depolarizing_errors(n, start, count, p, seed=DEFAULT_SEED):
    """Errors for samples [start, start+count) -> (x, z) uint8 [count, n]."""
    x = np.empty((count, n), dtype=np.uint8)
    z = np.empty((count, n), dtype=np.uint8)
    s = start
    while s < start + count:
        blk = s // BLOCK
        lo = s - blk * BLOCK
        hi = min(BLOCK, start + count - blk * BLOCK)
        g = np.random.Generator(np.random.Philox(key=[seed & 0xFFFFFFFFFFFFFFFF, blk]))
        u = g.random((BLOCK, n))[lo:hi]
        t = g.integers(0, 3, size=(BLOCK, n), dtype=np.uint8)[lo:hi]
        hit = u < p
        x[s - start: s - start + (hi - lo)] = hit & (t != 2)
        z[s - start: s - start + (hi - lo)] = hit & (t != 0)
        s = blk * BLOCK + hi
    return x, z


def syndromes(code, x, z):
    """(sX, sZ) = (HX x, HZ z) mod 2 through the product's code model."""
    return code.syndrome(0, x), code.syndrome(1, z)


def shard_range(total, rank, world):
    """Contiguous shard [lo, hi) of `total` samples for `rank` of `world`."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def bit_rows(s):
    """[B, m] 0/1 syndrome bytes (torch tensor) -> [B, ceil(m / 32)] int32 bit rows, bit c % 32 of
    word c / 32 = check c: the layout of qec_decode_bits_packed_dev and the Monte-Carlo pipeline."""
    import torch
    B, m = s.shape
    w = -(-m // 32)
    pad = torch.zeros((B, 32 * w), dtype=torch.int64, device=s.device)
    pad[:, :m] = (s != 0).to(torch.int64)
    v = (pad.view(B, w, 32) << torch.arange(32, device=s.device, dtype=torch.int64)).sum(2)
    return torch.where(v >= 2 ** 31, v - 2 ** 32, v).to(torch.int32).contiguous()
