"""Sparse-graph engine (bp_sparse.hip): parity with the oracle (CPU restatement of
DecoderCPU::Decode, QEC_LDPC/DecoderCPU.h:249-390) on codes the wave-circulant
engine cannot take -- non-circulant (column-permuted) codes, circulant codes with
P > 64 (LDS-resident and HBM-workspace modes) -- and on the shipped codes, where it
must also agree bit-for-bit with the wave-circulant engine.

Bar: bit-exact eX, eZ, flags, iteration counts and final messages (float32 bit
patterns; NaN matched by NaN).  No tolerance anywhere.
"""
import numpy as np
import pytest

import qec_ldpc_amd as q
from oracle.oracle import OracleCode
from qec_ldpc_amd.codes import write_code_file
from test_gpu_parity import mixed_inputs, same_floats

pytestmark = pytest.mark.gpu


def compare(g, o, what):
    for name, a, b in zip(("eX", "eZ", "flags", "iters"), g[:4], o[:4]):
        if not np.array_equal(a, b):
            bad = np.nonzero((a != b).reshape(len(a), -1).any(1))[0]
            raise AssertionError("%s: %s differs on %d/%d rows (first %s)" % (what, name, len(bad), len(a), bad[:5]))
    if g[4] is not None and o[4] is not None:
        assert same_floats(g[4], o[4]), "%s: final messages differ" % what


def permuted_code(path, tmp_path, seed):
    """The same code with its qubits (columns of HX, HZ and both halves of I-P) permuted:
    still regular (row weight L, column weight J / K) but no longer circulant."""
    c = q.Quantum_LDPC_Code.createFromFile(path)
    rng = np.random.default_rng(seed)
    perm = rng.permutation(c.n)
    HX, HZ = c.pcm(0)[:, perm], c.pcm(1)[:, perm]
    imp = None
    with open(path) as f:
        lines = f.read().split("\n")
    if len(lines) > 3 and lines[3].strip():
        IMP = np.array(lines[3].split(), dtype=np.uint8).reshape(2 * c.n, 2 * c.n)
        imp = IMP[:, np.concatenate([perm, c.n + perm])]
    out = tmp_path / ("perm_%d_%s.txt" % (seed, c.P))
    return write_code_file(str(out), c.J, c.K, c.L, c.P, c.sigma, c.tau, HX, HZ, imp)


def generated_file(tmp_path, J, K, L, P, s, t):
    c = q.QC_LDPC_CSS(J, K, L, P, s, t)
    out = tmp_path / ("gen_%d_%d_%d_%d.txt" % (J, K, L, P))
    return write_code_file(str(out), J, K, L, P, s, t, c.pcm(0), c.pcm(1)), c


@pytest.fixture(scope="module")
def shipped(code_paths):
    out = {}
    for k, path in code_paths.items():
        code = q.Quantum_LDPC_Code.createFromFile(path)
        out[k] = (code, q.DecoderGPU(code, 0, engine="sparse"), q.DecoderGPU(code, 0, engine="circulant"),
                  OracleCode(path))
    return out


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("stop", ["fixed", "ref", "syndrome"])
@pytest.mark.parametrize("N", [0, 1, 11, 50])
def test_sparse_engine_shipped_codes(shipped, key, stop, N):
    code, sp, _, orc = shipped[key]
    assert sp.describe().startswith("sparse-graph lds")
    sX, sZ = mixed_inputs(code, 96 if key == "P61" else 400, 1000 + N, 0.02)
    g = sp.decode_batch(sX, sZ, 0.02, N, stop, want_iters=True, want_q=True)
    o = orc.decode_batch(sX, sZ, 0.02, N, stop, want_q=True)
    compare(g, o, "%s sparse %s N=%d" % (key, stop, N))


@pytest.mark.parametrize("key,B,N", [("P61", 8192, 50), ("P7", 65536, 20)])
def test_sparse_equals_circulant(shipped, key, B, N):
    """Both engines are exact restatements, so they agree bit-for-bit at full batch size."""
    code, sp, wc, _ = shipped[key]
    sX, sZ = mixed_inputs(code, B, 77, 0.01)
    for stop in ("fixed", "ref"):
        g1 = sp.decode_batch(sX, sZ, 0.01, N, stop, want_iters=True, want_q=True)
        g2 = wc.decode_batch(sX, sZ, 0.01, N, stop, want_iters=True, want_q=True)
        compare(g1, g2, "%s sparse vs circulant %s" % (key, stop))


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("stop", ["fixed", "ref", "syndrome"])
def test_non_circulant_code(code_paths, tmp_path, key, stop):
    path = permuted_code(code_paths[key], tmp_path, 5)
    code = q.Quantum_LDPC_Code.createFromFile(path)
    with pytest.raises(q.QecError):
        code.exponents(0)  # not circulant any more
    dec = q.DecoderGPU(code, 0)  # auto -> sparse
    assert dec.describe().startswith("sparse-graph")
    with pytest.raises(q.QecError, match="wave-circulant"):
        q.DecoderGPU(code, 0, engine="circulant")
    orc = OracleCode(path)
    sX, sZ = mixed_inputs(code, 128, 3, 0.02)
    for N in (1, 20):
        g = dec.decode_batch(sX, sZ, 0.02, N, stop, want_iters=True, want_q=True)
        o = orc.decode_batch(sX, sZ, 0.02, N, stop, want_q=True)
        compare(g, o, "perm %s %s N=%d" % (key, stop, N))


@pytest.mark.parametrize("J,K,L,P,s,t,mode", [(3, 3, 6, 127, 2, 3, "lds"), (4, 5, 10, 467, 9, 49, "hbm")])
def test_large_circulant_code(tmp_path, J, K, L, P, s, t, mode):
    """P > 64: no wave-circulant kernel; the 467 code's messages (168 KB) exceed LDS."""
    path, code = generated_file(tmp_path, J, K, L, P, s, t)
    dec = q.DecoderGPU(code, 0)
    assert dec.describe().startswith("sparse-graph " + mode), dec.describe()
    orc = OracleCode(path)
    B = 48 if P < 200 else 12
    rng = np.random.default_rng(P)
    x = (rng.random((B, code.n)) < 0.01).astype(np.uint8)
    z = (rng.random((B, code.n)) < 0.01).astype(np.uint8)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    sX[0] = 0
    sZ[-1] = 1
    for stop, N in (("ref", 25), ("fixed", 11), ("syndrome", 30)):
        g = dec.decode_batch(sX, sZ, 0.015, N, stop, want_iters=True, want_q=True)
        o = orc.decode_batch(sX, sZ, 0.015, N, stop, want_q=True)
        compare(g, o, "P=%d %s" % (P, stop))


def test_large_code_front_end_full_width(tmp_path):
    """The fused front end's samples per wave are capped by the LDS the gap table leaves
    (montecarlo.hip launch_mc_gap): the n = 762 code (72 words of sample state) at 2^19 samples
    runs at 54 instead of 64 per wave and draws the same samples as a 1000-sample launch and the
    numpy restatement of the Philox stream (syndromes and packed errors)."""
    import torch
    from oracle.philox import depolarizing
    _, code = generated_file(tmp_path, 3, 3, 6, 127, 2, 3)
    dec = q.DecoderGPU(code, 0)
    dev = torch.device("cuda", 0)
    nb2 = 2 * ((code.n + 7) // 8)

    def bufs(B):
        return [torch.empty((B, w), dtype=torch.uint8, device=dev) for w in (code.numEqsX, code.numEqsZ, nb2)]

    B, lo, seed, p = 1 << 19, 300001, 5, 0.01
    big, small = bufs(B), bufs(1000)
    dec.sample_syndrome_dev(seed, 0, p, *big)
    dec.sample_syndrome_dev(seed, lo, p, *small)
    torch.cuda.synchronize()
    for a, b in zip(big, small):
        assert torch.equal(a[lo:lo + 1000], b)
    x, z = depolarizing(seed, lo, 1000, code.n, p)
    assert np.array_equal(small[0].cpu().numpy(), code.syndrome(0, x))
    assert np.array_equal(small[1].cpu().numpy(), code.syndrome(1, z))
    exp = np.concatenate([np.packbits(x, axis=1, bitorder="little"), np.packbits(z, axis=1, bitorder="little")], 1)
    assert np.array_equal(small[2].cpu().numpy(), exp)


def test_irregular_code_is_rejected(code_paths, tmp_path):
    c = q.Quantum_LDPC_Code.createFromFile(code_paths["P7"])
    HX = c.pcm(0).copy()
    HX[0, :] = 0
    HX[0, :3] = 1  # row 0 now has weight 3 != L
    path = write_code_file(str(tmp_path / "irr.txt"), c.J, c.K, c.L, c.P, c.sigma, c.tau, HX, c.pcm(1))
    bad = q.Quantum_LDPC_Code.createFromFile(path)
    with pytest.raises(q.QecError, match="irregular"):
        q.DecoderGPU(bad, 0)


def test_sparse_get_statistics_matches_oracle(code_paths, tmp_path):
    """GetStatistics (reference sampler, GPU decode + CSR syndromes + I-P check) on a
    non-circulant code equals the oracle's counting loop."""
    path = permuted_code(code_paths["P7"], tmp_path, 11)
    code = q.Quantum_LDPC_Code.createFromFile(path)
    dec = q.DecoderGPU(code, 0)
    orc = OracleCode(path)
    for W, count, seed in ((2, 4000, 1234), (4, 3000, 99)):
        g = dec.GetStatistics(W, count, 0.02, 100, seed=seed)
        o = orc.get_statistics(W, count, 0.02, 100, seed)
        assert g["numErrorsTested"] == o["tested"]
        for gk, ok in (("numXErrorsTested", "withX"), ("numZErrorsTested", "withZ"), ("corrected", "corrected"),
                       ("syndromeErrorsX", "synX"), ("syndromeErrorsZ", "synZ"), ("logicalErrors", "logical"),
                       ("convergenceFailX", "convX"), ("convergenceFailZ", "convZ")):
            assert g[gk] == o[ok], (W, gk, g[gk], o[ok])


def test_sparse_monte_carlo_equals_circulant(shipped):
    """Device Monte-Carlo (Philox sampler -> syndrome -> decode -> I-P check) gives the same
    counters through either engine (CSR vs circulant syndrome kernels included)."""
    _, sp, wc, _ = shipped["P61"]
    for stop in ("syndrome", "ref"):
        a = sp.monte_carlo(0x51EC0DE, 0, 20000, 0.03, 50, stop, batch=8192)
        b = wc.monte_carlo(0x51EC0DE, 0, 20000, 0.03, 50, stop, batch=8192)
        for k in ("tested", "withX", "withZ", "synX", "synZ", "logical", "corrected", "convX", "convZ",
                  "iterationsX", "iterationsZ"):
            assert a[k] == b[k], (stop, k, a[k], b[k])


@pytest.mark.parametrize("idx", [0, 4, 6])
def test_sparse_engine_reproduces_published_counters(idx, kat_records, shipped):
    """The sparse-graph engine reproduces the reference's published CodeStatistics blocks."""
    from conftest import COUNTERS, code_key, kat_subset
    from test_gpu_kat import MAP
    rec = kat_subset(kat_records)[idx]
    sp = shipped[code_key(rec)][1]
    st = sp.GetStatistics(rec["W"], rec["tested"], rec["p_run"], rec["MAX"], rec["seed"])
    assert {k: st[MAP[k]] for k in COUNTERS} == {k: rec[k] for k in COUNTERS}, (rec["file"], rec["block"])
