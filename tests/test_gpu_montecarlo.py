"""Device Monte-Carlo caller against the oracle:
Philox sampler vs its numpy restatement, circulant syndrome kernel vs the host
code model, statistics kernel and whole qec_monte_carlo runs vs counting with the
oracle's decoder and I-P check (DecoderCPU.h:464-521) on the same samples."""
import numpy as np
import pytest
import torch

import qec_ldpc_amd as q
from oracle.oracle import OracleCode
from oracle.philox import depolarizing

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def env(code_paths):
    out = {}
    for k, path in code_paths.items():
        code = q.Quantum_LDPC_Code.createFromFile(path)
        out[k] = (code, q.DecoderGPU(code, 0), OracleCode(path))
    return out


def dev_u8(*shape):
    return torch.empty(shape, dtype=torch.uint8, device=DEV)


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("seed,start,p", [(0x51EC0DE, 0, 0.01), (12345, (1 << 32) - 3, 0.2), (7, 99, 0.0),
                                          (7, 5, 1.0), (2 ** 63 + 5, 1 << 40, 0.05)])
def test_sampler_matches_numpy(env, key, seed, start, p):
    code, dec, _ = env[key]
    B = 300
    x, z = dev_u8(B, code.n), dev_u8(B, code.n)
    dec.sample_depolarizing_dev(seed, start, p, x, z)
    torch.cuda.synchronize()
    rx, rz = depolarizing(seed, start, B, code.n, p)
    assert np.array_equal(x.cpu().numpy(), rx) and np.array_equal(z.cpu().numpy(), rz)


@pytest.mark.parametrize("key", ["P7", "P61"])
def test_syndrome_kernel(env, key):
    code, dec, _ = env[key]
    rng = np.random.default_rng(4)
    ex = (rng.random((700, code.n)) < 0.05).astype(np.uint8)
    ez = (rng.random((700, code.n)) < 0.05).astype(np.uint8)
    sX, sZ = dev_u8(700, code.numEqsX), dev_u8(700, code.numEqsZ)
    dec.syndrome_dev(torch.from_numpy(ex).to(DEV), torch.from_numpy(ez).to(DEV), sX, sZ)
    torch.cuda.synchronize()
    assert np.array_equal(sX.cpu().numpy(), code.syndrome(0, ex))
    assert np.array_equal(sZ.cpu().numpy(), code.syndrome(1, ez))


def oracle_counters(orc, x, z, p, N, stop):
    sx, sz = orc.syndrome(0, x), orc.syndrome(1, z)
    eX, eZ, fl, it, _ = orc.decode_batch(sx, sz, p, N, stop)
    c = dict.fromkeys(q.MC_COUNTERS, 0)
    c["withX"] = int(x.any(1).sum())
    c["withZ"] = int(z.any(1).sum())
    c["synX"] = int((fl & 1 != 0).sum())
    c["synZ"] = int((fl & 2 != 0).sum())
    c["convX"] = int((fl & 4 != 0).sum())
    c["convZ"] = int((fl & 8 != 0).sum())
    for b in np.nonzero((fl & 3) == 0)[0]:
        if orc.check_logical(x[b] ^ eX[b], z[b] ^ eZ[b]):
            c["logical"] += 1
        else:
            c["corrected"] += 1
    return c, it


@pytest.mark.parametrize("key,B,p,N", [("P7", 4000, 0.06, 30), ("P61", 300, 0.03, 30)])
def test_statistics_kernel_matches_oracle(env, key, B, p, N):
    code, dec, orc = env[key]
    x, z = depolarizing(99, 0, B, code.n, p)
    xd, zd = torch.from_numpy(x).to(DEV), torch.from_numpy(z).to(DEV)
    sX, sZ = dev_u8(B, code.numEqsX), dev_u8(B, code.numEqsZ)
    dec.syndrome_dev(xd, zd, sX, sZ)
    eX, eZ, fl = dev_u8(B, code.n), dev_u8(B, code.n), dev_u8(B)
    dec.decode_batch_dev(sX, sZ, p, N, "ref", eX, eZ, fl)
    cnt = torch.zeros(8, dtype=torch.int64, device=DEV)
    dec.statistics_dev(xd, zd, eX, eZ, fl, cnt)
    torch.cuda.synchronize()
    got = dict(zip(q.MC_COUNTERS, cnt.cpu().tolist()))
    exp, _ = oracle_counters(orc, x, z, p, N, "ref")
    assert got == exp


@pytest.mark.parametrize("stop", ["ref", "syndrome", "fixed"])
@pytest.mark.parametrize("key,count,p", [("P7", 5000, 0.05), ("P61", 400, 0.04), ("P7", 20000, 0.005),
                                         ("P61", 3000, 0.01), ("P61", 3000, 0.002)])
def test_monte_carlo_matches_oracle(env, key, count, p, stop):
    """At p <= 0.01 the syndrome stop takes the fused low-p pipeline (triage.hip)."""
    code, dec, orc = env[key]
    r = dec.monte_carlo(0xBEEF, 17, count, p, 25, stop, batch=1000)
    x, z = depolarizing(0xBEEF, 17, count, code.n, p)
    exp, it = oracle_counters(orc, x, z, p, 25, stop)
    assert {k: r[k] for k in q.MC_COUNTERS} == exp
    assert r["tested"] == count
    assert r["iterationsX"] == int(it[:, 0].sum()) and r["iterationsZ"] == int(it[:, 1].sum())


@pytest.mark.parametrize("stop", ["ref", "syndrome", "fixed"])
def test_monte_carlo_other_code_with_i_minus_p(tmp_path, stop):
    """qec_monte_carlo on a code of neither shipped size (J=2,K=3,L=6,P=11, n = 66: records of 19 B,
    packed errors of 18 B) with an I-P line: the Philox pipeline keeps the public 2 ceil(n/8) + 1 record
    rows where the lane statistics kernel has no shape for padded ones, and its counters equal the
    oracle's counting over the same file (any 0/1 matrix on line 4 is a valid CheckLogicalError input,
    QEC_LDPC/Quantum_LDPC_Code.h:126-142)."""
    g = q.QC_LDPC_CSS(2, 3, 6, 11, 2, 3)
    rng = np.random.default_rng(11)
    imp = (rng.random((2 * g.n, 2 * g.n)) < 0.02).astype(np.uint8)
    path = str(tmp_path / "gen_imp.txt")
    with open(path, "w") as f:
        f.write("2 3 6 11 2 3\n")
        f.write("\t".join(map(str, g.pcm(0).ravel())) + "\n")
        f.write("\t".join(map(str, g.pcm(1).ravel())) + "\n")
        f.write("\t".join(map(str, imp.ravel())) + "\n")
    code = q.Quantum_LDPC_Code.createFromFile(path)
    dec = q.DecoderGPU(code, 0)
    assert "runtime-shift" in dec.describe()
    orc = OracleCode(path)
    count, p = 3000, 0.05
    r = dec.monte_carlo(0xC0DE, 5, count, p, 25, stop, batch=1024)
    x, z = depolarizing(0xC0DE, 5, count, code.n, p)
    exp, it = oracle_counters(orc, x, z, p, 25, stop)
    assert {k: r[k] for k in q.MC_COUNTERS} == exp
    assert exp["logical"] > 0 and exp["corrected"] > 0  # both outcomes of the I-P check occur
    assert r["iterationsX"] == int(it[:, 0].sum()) and r["iterationsZ"] == int(it[:, 1].sum())


def test_monte_carlo_shards_add_up(env):
    code, dec, _ = env["P61"]
    whole = dec.monte_carlo(5, 0, 6000, 0.03, 50, "syndrome", batch=2048)
    a = dec.monte_carlo(5, 0, 2500, 0.03, 50, "syndrome", batch=4096)
    b = dec.monte_carlo(5, 2500, 3500, 0.03, 50, "syndrome", batch=777)
    for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
        assert whole[k] == a[k] + b[k], k


def test_monte_carlo_fused_batches_and_empty_run(env):
    """The fused low-p pipeline over several batches of one call (the list lengths are zeroed again
    before every later batch; the first batch's memset also zeroes the counters) adds up to one
    batch, and a run of zero samples right after returns zero counters, not the last run's."""
    code, dec, _ = env["P61"]
    one = dec.monte_carlo(11, 0, 10000, 0.002, 50, "syndrome", batch=10000)
    many = dec.monte_carlo(11, 0, 10000, 0.002, 50, "syndrome", batch=4096)
    for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
        assert one[k] == many[k], k
    assert one["withX"] > 0 and one["corrected"] > 0
    empty = dec.monte_carlo(11, 0, 0, 0.002, 50, "syndrome")
    for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
        assert empty[k] == 0, k


def test_monte_carlo_without_decode_timing(env):
    """QEC_OPT_MC_DECODE_TIME 0 (tools/psweep.py's timed runs): the same counters on the fused low-p
    pipeline and the ordered one over several batches, decodeSeconds 0; back on, timed again."""
    code, dec, _ = env["P61"]
    for p, batch in ((0.002, 4096), (0.03, 2048)):
        timed = dec.monte_carlo(13, 0, 9000, p, 50, "syndrome", batch=batch)
        dec.set_option("mc_decode_time", 0)
        try:
            assert dec.get_option("mc_decode_time") == 0
            bare = dec.monte_carlo(13, 0, 9000, p, 50, "syndrome", batch=batch)
        finally:
            dec.set_option("mc_decode_time", 1)
        for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
            assert bare[k] == timed[k], (p, k)
        assert bare["decodeSeconds"] == 0.0 and timed["decodeSeconds"] > 0.0
        assert dec.monte_carlo(13, 0, 9000, p, 50, "syndrome", batch=batch)["decodeSeconds"] > 0.0


def test_monte_carlo_full_batch(env):
    """qec_monte_carlo at psweep's default shape (2^20 samples in one batch: 64-lane front-end waves,
    one decode launch) against oracle counting on its last 2 048 samples (the same launch shape minus
    them covers the rest), and eight contiguous shards adding up to it (BASELINE configs[4]/[5])."""
    code, dec, orc = env["P61"]
    B, p, tail, seed = 1 << 20, 0.005, 2048, 0x51EC0DE
    whole = dec.monte_carlo(seed, 0, B, p, 50, "syndrome")
    head = dec.monte_carlo(seed, 0, B - tail, p, 50, "syndrome")
    x, z = depolarizing(seed, B - tail, tail, code.n, p)
    exp, it = oracle_counters(orc, x, z, p, 50, "syndrome")
    for k in q.MC_COUNTERS:
        assert whole[k] == head[k] + exp[k], k
    assert whole["iterationsX"] == head["iterationsX"] + int(it[:, 0].sum())
    assert whole["iterationsZ"] == head["iterationsZ"] + int(it[:, 1].sum())
    parts = [dec.monte_carlo(seed, g * B // 8, B // 8, p, 50, "syndrome") for g in range(8)]
    for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
        assert whole[k] == sum(r[k] for r in parts), k


@pytest.mark.parametrize("key", ["P7", "P61"])
def test_pack_decisions_matches_host(env, key):
    """qec_pack_decisions_dev (the gather payload) equals the host packing of
    the same decoded batch, including the partial last byte (P7: n = 42)."""
    from qec_ldpc_amd.gather import pack_records, unpack_records
    code, dec, _ = env[key]
    B = 777
    rng = np.random.default_rng(8)
    sX = (rng.random((B, code.numEqsX)) < 0.05).astype(np.uint8)
    sZ = (rng.random((B, code.numEqsZ)) < 0.05).astype(np.uint8)
    eX, eZ, fl, _, _ = dec.decode_batch(sX, sZ, 0.02, 20, "fixed")
    tX, tZ, tf = (torch.from_numpy(a).to(DEV) for a in (eX, eZ, fl))
    rec = dev_u8(B, dec.record_bytes())
    dec.pack_decisions_dev(tX, tZ, tf, rec)
    torch.cuda.synchronize()
    got = rec.cpu().numpy()
    assert np.array_equal(got, pack_records(eX, eZ, fl))
    a, b, c = unpack_records(got, code.n)
    assert np.array_equal(a, eX) and np.array_equal(b, eZ) and np.array_equal(c, fl)
