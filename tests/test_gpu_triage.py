"""Iteration-0 triage of the syndrome stop rule (triage.hip + the decode kernel's list mode, behind
QEC_OPT_TRIAGE) against the plain decode and the oracle (CPU restatement of DecoderCPU::Decode with
the syndrome stop, QEC_LDPC/DecoderCPU.h:249-390).

Bar: bit-identical decision records and iteration counts -- triage on, triage off, the byte-row entry
point -- and the oracle's answers; Monte-Carlo counters unchanged.
"""
import numpy as np
import pytest
import torch

import qec_ldpc_amd as q
from oracle.oracle import OracleCode
from qec_ldpc_amd.gather import pack_records
from qec_ldpc_amd.synthetic import depolarizing_errors

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def env(code_paths):
    out = {}
    for k, path in code_paths.items():
        code = q.Quantum_LDPC_Code.createFromFile(path)
        out[k] = (code, q.DecoderGPU(code, 0), OracleCode(path))
    return out


def bit_rows(s):
    """[B, m] 0/1 bytes -> [B, ceil(m/32)] int32 words, bit c = check c."""
    B, m = s.shape
    w = (m + 31) // 32
    pk = np.packbits(s, axis=1, bitorder="little")
    pad = np.zeros((B, 4 * w), np.uint8)
    pad[:, :pk.shape[1]] = pk
    return torch.from_numpy(pad.view(np.int32).copy()).to(DEV)


def decode_all(dec, code, sX, sZ, p, N):
    B = len(sX)
    out = {}
    for name, tri in (("on", 2), ("off", 0)):  # 2: triage at every p (1 only up to p = 0.01)
        dec.set_option("triage", tri)
        rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=DEV)
        its = torch.empty((B, 2), dtype=torch.int32, device=DEV)
        dec.decode_bits_packed_dev(bit_rows(sX), bit_rows(sZ), p, N, "syndrome", rec, its)
        torch.cuda.synchronize()
        out[name] = (rec.cpu().numpy(), its.cpu().numpy())
    dec.set_option("triage", 1)
    rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=DEV)
    its = torch.empty((B, 2), dtype=torch.int32, device=DEV)
    dec.decode_batch_packed_dev(torch.from_numpy(sX).to(DEV), torch.from_numpy(sZ).to(DEV), p, N, "syndrome", rec, its)
    torch.cuda.synchronize()
    out["bytes"] = (rec.cpu().numpy(), its.cpu().numpy())
    return out


def inputs(code, B, p, seed):
    x, z = depolarizing_errors(code.n, seed, B, p)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    rng = np.random.default_rng(seed)
    k = max(1, B // 50)
    sX[:k] = 0  # zero syndromes
    sZ[k:2 * k] = 0
    sX[-k:] = (rng.random((k, code.numEqsX)) < 0.3).astype(np.uint8)  # heavy random syndromes
    return sX, sZ


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("p", [0.001, 0.002, 0.005, 0.01, 0.05, 0.1])
def test_triage_identical_and_oracle(env, key, p):
    code, dec, orc = env[key]
    B = 3001 if key == "P61" else 20001
    sX, sZ = inputs(code, B, p, 17)
    out = decode_all(dec, code, sX, sZ, p, 50)
    for name in ("off", "bytes"):
        assert np.array_equal(out["on"][0], out[name][0]), name
        assert np.array_equal(out["on"][1], out[name][1]), name
    n = 600 if key == "P61" else 4000
    o = orc.decode_batch(sX[:n], sZ[:n], p, 50, "syndrome")
    assert np.array_equal(out["on"][0][:n], pack_records(o[0], o[1], o[2]))
    assert np.array_equal(out["on"][1][:n], o[3])


@pytest.mark.parametrize("p", [0.002, 0.01, 0.05])
def test_triage_count_form_equals_trees(env, p, monkeypatch):
    """Symmetric pattern masks (iteration-0 decisions that depend only on the number of unsatisfied
    checks, the usual case) take a bit-sliced adder tree in the triage kernel; the general pattern
    trees (QEC_TRIAGE_TREES=1) give the same records and counts."""
    code, dec, _ = env["P61"]
    sX, sZ = inputs(code, 5001, p, 23)
    a = decode_all(dec, code, sX, sZ, p, 50)
    monkeypatch.setenv("QEC_TRIAGE_TREES", "1")
    b = decode_all(dec, code, sX, sZ, p, 50)
    for name in ("on", "off"):
        assert np.array_equal(a[name][0], b[name][0]) and np.array_equal(a[name][1], b[name][1]), name
    assert np.array_equal(a["on"][0], a["off"][0])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("N,B", [(2, 777), (3, 64), (1, 100), (0, 65), (50, 1), (50, 63), (50, 129)])
def test_triage_edges(env, key, N, B):
    """N = 1 / 0 (no triage: iteration 0 is the last or none), N = 2, ragged batches around the
    64-lane waves, against the oracle."""
    code, dec, orc = env[key]
    sX, sZ = inputs(code, B, 0.01, 5 + N)
    out = decode_all(dec, code, sX, sZ, 0.01, N)
    o = orc.decode_batch(sX, sZ, 0.01, N, "syndrome")
    for name in ("on", "off", "bytes"):
        assert np.array_equal(out[name][0], pack_records(o[0], o[1], o[2])), name
        assert np.array_equal(out[name][1], o[3]), name


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("p", [0.002, 0.01, 0.05])
def test_monte_carlo_triage_counters(env, key, p):
    code, dec, _ = env[key]
    B = 1 << 18
    res = {}
    for tri in (2, 1, 3, 0):  # 2 / 1: the fused kernel (1 only up to p = 0.01), 3: triage kernel, 0: none
        dec.set_option("triage", tri)
        res[tri] = dec.monte_carlo(0x51EC0DE, 12345, B, p, 50, "syndrome")
    dec.set_option("triage", 1)
    for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
        assert res[2][k] == res[1][k] == res[3][k] == res[0][k], (k, res[2][k], res[1][k], res[3][k], res[0][k])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("p,count,batch", [(0.001, 100003, 32768), (0.005, 70001, 65536), (0.01, 4097, 1000),
                                           (0.0, 3000, 1024), (0.01, 1, 1)])
def test_monte_carlo_fused_ragged(env, key, p, count, batch):
    """The fused low-p pipeline (QEC_OPT_TRIAGE 1, triage.hip mc_fused_kernel + list decode + survivor
    statistics) over ragged multi-batch runs, p = 0 (no errors at all) and a single sample: counters
    equal the plain pipeline's (no triage) on the same samples."""
    code, dec, _ = env[key]
    res = {}
    for tri in (1, 0):
        dec.set_option("triage", tri)
        res[tri] = dec.monte_carlo(0xFEED, 777, count, p, 50, "syndrome", batch)
    dec.set_option("triage", 1)
    for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
        assert res[1][k] == res[0][k], (k, res[1][k], res[0][k])


def test_triage_option_roundtrip(env):
    _, dec, _ = env["P61"]
    assert dec.get_option("triage") == 1
    for v in (0, 2, 3, 1):
        dec.set_option("triage", v)
        assert dec.get_option("triage") == v
    with pytest.raises(q.QecError):
        dec.set_option("triage", 4)
