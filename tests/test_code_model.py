"""Host-side code model of the product (no GPU): loader, generator, circulant
extraction, syndromes, logical check and the reference's error sampler."""
import os

import numpy as np
import pytest

import qec_ldpc_amd as q
from oracle.oracle import OracleCode

# SURVEY.md section 8(a) row 11 (measured from the shipped files)
P61_EX = [[1, 9, 20, 58, 34, 42, 12, 47, 57, 25], [34, 1, 9, 20, 58, 12, 47, 57, 25, 42],
          [58, 34, 1, 9, 20, 47, 57, 25, 42, 12], [20, 58, 34, 1, 9, 57, 25, 42, 12, 47]]
P61_EZ = [[19, 49, 14, 4, 36, 60, 52, 41, 3, 27], [36, 19, 49, 14, 4, 52, 41, 3, 27, 60],
          [4, 36, 19, 49, 14, 41, 3, 27, 60, 52], [14, 4, 36, 19, 49, 3, 27, 60, 52, 41],
          [49, 14, 4, 36, 19, 27, 60, 52, 41, 3]]
P7_EX = [[1, 2, 4, 2, 4, 1], [4, 1, 2, 4, 1, 2], [2, 4, 1, 1, 2, 4]]
P7_EZ = [[5, 3, 6, 6, 5, 3], [6, 5, 3, 5, 3, 6], [3, 6, 5, 3, 6, 5]]


@pytest.fixture(scope="module")
def codes(code_paths):
    return {k: q.Quantum_LDPC_Code.createFromFile(v) for k, v in code_paths.items()}


def dense_file(path):
    lines = open(path).read().split("\n")
    J, K, L, P, s, t = map(int, lines[0].split())
    hx = np.array(lines[1].split(), dtype=np.uint8).reshape(J * P, L * P)
    hz = np.array(lines[2].split(), dtype=np.uint8).reshape(K * P, L * P)
    imp = np.array(lines[3].split(), dtype=np.uint8).reshape(2 * L * P, 2 * L * P)
    return hx, hz, imp


def test_params_and_describe(codes):
    c = codes["P61"]
    assert (c.J, c.K, c.L, c.P, c.sigma, c.tau, c.n, c.numEqsX, c.numEqsZ) == (4, 5, 10, 61, 9, 49, 610, 244, 305)
    assert c.describe() == "[J=4,K=5,L=10,P=61,s=9,t=49][[n=610,k=61]]"
    assert codes["P7"].describe() == "[J=3,K=3,L=6,P=7,s=2,t=3][[n=42,k=0]]"


def test_exponent_tables(codes):
    assert codes["P61"].exponents(0).tolist() == P61_EX
    assert codes["P61"].exponents(1).tolist() == P61_EZ
    assert codes["P7"].exponents(0).tolist() == P7_EX
    assert codes["P7"].exponents(1).tolist() == P7_EZ


@pytest.mark.parametrize("key,params", [("P7", (3, 3, 6, 7, 2, 3)), ("P61", (4, 5, 10, 61, 9, 49))])
def test_generator_regenerates_shipped_files(key, params, codes, code_paths):
    g = q.QC_LDPC_CSS(*params)
    hx, hz, _ = dense_file(code_paths[key])
    assert np.array_equal(g.pcm(0), hx)
    assert np.array_equal(g.pcm(1), hz)
    assert np.array_equal(codes[key].pcm(0), hx)
    # CSS condition HX HZ^T = 0 mod 2
    assert not ((hx.astype(np.int64) @ hz.T.astype(np.int64)) % 2).any()


def test_syndrome_matches_dense(codes, code_paths):
    rng = np.random.default_rng(1)
    for key in ("P7", "P61"):
        hx, hz, _ = dense_file(code_paths[key])
        e = (rng.random((50, codes[key].n)) < 0.05).astype(np.uint8)
        assert np.array_equal(codes[key].syndrome(0, e), (e.astype(np.int64) @ hx.T) % 2)
        assert np.array_equal(codes[key].syndrome(1, e), (e.astype(np.int64) @ hz.T) % 2)
        assert codes[key].GetSyndromeX(e[0]).tolist() == ((hx.astype(np.int64) @ e[0]) % 2).tolist()


def test_check_logical_matches_dense_and_oracle(codes, code_paths):
    rng = np.random.default_rng(2)
    for key in ("P7", "P61"):
        c = codes[key]
        _, _, imp = dense_file(code_paths[key])
        oc = OracleCode(code_paths[key])
        ex = (rng.random((40, c.n)) < 0.02).astype(np.uint8)
        ez = (rng.random((40, c.n)) < 0.02).astype(np.uint8)
        ex[0] = 0
        ez[0] = 0
        got = c.check_logical(ex, ez)
        dense = ((imp.astype(np.int64) @ np.concatenate([ex, ez], 1).T.astype(np.int64)) % 2).any(0)
        assert np.array_equal(got, dense)
        assert [oc.check_logical(ex[b], ez[b]) for b in range(40)] == got.tolist()
        assert not got[0]


def test_sampler_matches_oracle_stream():
    oc_x, oc_z = None, None
    from oracle.oracle import lib as olib  # noqa: F401  (oracle restates the same stream independently)
    for seed, W, n in ((2881811342, 3, 42), (12345, 60, 610), (0, 1, 42)):
        x, z = q.sample_fixed_weight(seed, W, 500, n)
        ox = np.empty_like(x)
        oz = np.empty_like(z)
        import ctypes
        olib().oc_sample_fixed_weight(seed, W, 500, n, ox.ctypes.data_as(ctypes.c_void_p),
                                      oz.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(x, ox) and np.array_equal(z, oz)
        assert (x | z).sum(1).max() <= W


def test_missing_file_raises_reference_message(tmp_path):
    with pytest.raises(q.QecError, match="Unable to find code file"):
        q.Quantum_LDPC_Code.createFromFile(str(tmp_path / "nope.txt"))


def test_malformed_header_raises(tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("3 3\n0 1\n")
    with pytest.raises(q.QecError):
        q.Quantum_LDPC_Code.createFromFile(str(p))


def test_generated_code_has_no_logical_matrix():
    g = q.QC_LDPC_CSS(3, 3, 6, 7, 2, 3)
    with pytest.raises(q.QecError, match="I-P"):
        g.check_logical(np.zeros((1, 42), np.uint8), np.zeros((1, 42), np.uint8))


def test_generator_bad_sigma():
    with pytest.raises(q.QecError):
        q.QC_LDPC_CSS(3, 3, 6, 8, 2, 3)  # 2 has no inverse mod 8


def test_non_qc_code_loads_but_has_no_exponents(tmp_path, code_paths):
    # perturb one entry of HX: still a valid file, no longer circulant
    lines = open(code_paths["P7"]).read().split("\n")
    vals = lines[1].split()
    vals[0] = "1" if vals[0] == "0" else "0"
    lines[1] = "\t".join(vals)
    p = tmp_path / "nonqc.txt"
    p.write_text("\n".join(lines))
    c = q.Quantum_LDPC_Code.createFromFile(str(p))
    with pytest.raises(q.QecError, match="circulant"):
        c.exponents(0)
    # dense syndrome path still matches numpy
    hx, _, _ = dense_file(str(p))
    e = (np.random.default_rng(3).random((5, 42)) < 0.2).astype(np.uint8)
    assert np.array_equal(c.syndrome(0, e), (e.astype(np.int64) @ hx.T) % 2)
