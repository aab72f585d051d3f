"""Bit-packed decision records straight from the decode kernel (qec_decode_batch_packed_dev,
SURVEY.md 8(d)'s I/O model), the sector-split flag merge, the fused Monte-Carlo front end and
packed statistics, the device-buffer contract of the Python view (validation, streams, graph
capture) and the multi-device decoder (qec_decoder_create_multi).

Every packed output is compared with the oracle's decisions (packed on the host) and with the
byte-form entry point on the same inputs."""
import numpy as np
import pytest
import torch

import qec_ldpc_amd as q
from oracle.oracle import OracleCode
from oracle.philox import depolarizing
from qec_ldpc_amd.gather import pack_records, unpack_records
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


def inputs(code, B, p, seed=3):
    x, z = depolarizing_errors(code.n, seed * 1000, B, p)
    return code.syndrome(0, x), code.syndrome(1, z)


def u8(*shape):
    return torch.empty(shape, dtype=torch.uint8, device=DEV)


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("stop", ["ref", "fixed", "syndrome"])
@pytest.mark.parametrize("B", [1, 2, 28, 4097])
def test_packed_matches_oracle(env, key, stop, B):
    code, dec, orc = env[key]
    p, N = (0.03, 20) if key == "P7" else (0.02, 30)
    sX, sZ = inputs(code, B, p, seed=B)
    rec, its = dec.decode_batch_packed(sX, sZ, p, N, stop, want_iters=True)
    o = orc.decode_batch(sX, sZ, p, N, stop)
    assert np.array_equal(rec, pack_records(o[0], o[1], o[2]))
    assert np.array_equal(its, o[3])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("schedule,split", [(0, 0), (2, 0), (0, 2), (2, 2), (1, 1), (0, 3), (2, 3)])
def test_packed_dev_equals_byte_form(env, key, schedule, split):
    code, dec, _ = env[key]
    B = 5000
    sX, sZ = inputs(code, B, 0.03 if key == "P7" else 0.015, seed=11)
    dec.set_option("schedule", schedule)
    dec.set_option("sector_split", split)
    try:
        tX, tZ = torch.from_numpy(sX).to(DEV), torch.from_numpy(sZ).to(DEV)
        rec, it1 = u8(B, dec.record_bytes()), torch.empty((B, 2), dtype=torch.int32, device=DEV)
        dec.decode_batch_packed_dev(tX, tZ, 0.03, 25, "ref", rec, it1)
        eX, eZ, fl = u8(B, code.n), u8(B, code.n), u8(B)
        it2 = torch.empty((B, 2), dtype=torch.int32, device=DEV)
        dec.decode_batch_dev(tX, tZ, 0.03, 25, "ref", eX, eZ, fl, it2)
        torch.cuda.synchronize()
    finally:
        dec.set_option("schedule", 1)
        dec.set_option("sector_split", 1)
    a, b, c = unpack_records(rec.cpu().numpy(), code.n)
    assert np.array_equal(a, eX.cpu().numpy()) and np.array_equal(b, eZ.cpu().numpy())
    assert np.array_equal(c, fl.cpu().numpy())
    assert torch.equal(it1, it2)
    # padding bits of the last byte of each sector are zero
    r = rec.cpu().numpy()
    nb = (code.n + 7) // 8
    if code.n % 8:
        pad = np.uint8((0xFF << (code.n % 8)) & 0xFF)
        assert not (r[:, nb - 1] & pad).any() and not (r[:, 2 * nb - 1] & pad).any()


@pytest.mark.parametrize("offset", [0, 1, 2, 3])
def test_split_flags_stay_inside_the_buffer(env, offset):
    """The sector-split kernels merge their flags in the decoder's own words and store one byte
    per syndrome: a flags view at any byte offset is written exactly on its B bytes."""
    code, dec, orc = env["P7"]
    B = 4099
    sX, sZ = inputs(code, B, 0.05, seed=5)
    tX, tZ = torch.from_numpy(sX).to(DEV), torch.from_numpy(sZ).to(DEV)
    buf = torch.full((B + 8,), 0xAA, dtype=torch.uint8, device=DEV)
    fl = buf[offset:offset + B]
    eX, eZ = u8(B, code.n), u8(B, code.n)
    dec.set_option("sector_split", 2)
    try:
        dec.decode_batch_dev(tX, tZ, 0.05, 20, "ref", eX, eZ, fl)
        torch.cuda.synchronize()
    finally:
        dec.set_option("sector_split", 1)
    h = buf.cpu().numpy()
    assert (h[:offset] == 0xAA).all() and (h[offset + B:] == 0xAA).all()
    o = orc.decode_batch(sX, sZ, 0.05, 20, "ref")
    assert np.array_equal(h[offset:offset + B], o[2])


def test_two_streams_one_decoder(env):
    """Calls on one decoder from two streams are ordered through the workspace event."""
    code, dec, orc = env["P61"]
    B = 8192
    sX, sZ = inputs(code, B, 0.02, seed=21)
    s1, s2 = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    tX, tZ = torch.from_numpy(sX).to(DEV), torch.from_numpy(sZ).to(DEV)
    torch.cuda.synchronize()
    r1, r2 = u8(B, dec.record_bytes()), u8(B, dec.record_bytes())
    h = B // 2
    dec.decode_batch_packed_dev(tX, tZ, 0.02, 50, "fixed", r1, stream=s1)
    dec.decode_batch_packed_dev(tX[h:].contiguous(), tZ[h:].contiguous(), 0.02, 50, "fixed", r2[h:], stream=s2)
    dec.decode_batch_packed_dev(tX[:h].contiguous(), tZ[:h].contiguous(), 0.02, 50, "fixed", r2[:h], stream=s1)
    torch.cuda.synchronize()
    assert torch.equal(r1, r2)
    idx = np.arange(0, B, 37)
    o = orc.decode_batch(sX[idx], sZ[idx], 0.02, 50, "fixed")
    assert np.array_equal(r1.cpu().numpy()[idx], pack_records(o[0], o[1], o[2]))


def test_graph_capture_with_reserved_workspace(code_paths):
    """A decoder created with max_batch >= B allocates nothing in its device entry points, so
    the packed decode can be captured into a graph and replayed."""
    code = q.Quantum_LDPC_Code.createFromFile(code_paths["P61"])
    B = 6000
    dec = q.DecoderGPU(code, 0, max_batch=B)
    sX, sZ = inputs(code, B, 0.01, seed=31)
    tX, tZ = torch.from_numpy(sX).to(DEV), torch.from_numpy(sZ).to(DEV)
    ref = u8(B, dec.record_bytes())
    dec.decode_batch_packed_dev(tX, tZ, 0.01, 50, "fixed", ref)
    torch.cuda.synchronize()
    rec = u8(B, dec.record_bytes())
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            dec.decode_batch_packed_dev(tX, tZ, 0.01, 50, "fixed", rec, stream=s)
    rec.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(rec, ref)


# the refused call records nothing, so torch warns that the captured graph is empty: expected here
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
def test_capture_refuses_to_grow(code_paths):
    code = q.Quantum_LDPC_Code.createFromFile(code_paths["P61"])
    dec = q.DecoderGPU(code, 0, max_batch=16)
    B = 5000
    sX, sZ = inputs(code, B, 0.01, seed=32)
    tX, tZ = torch.from_numpy(sX).to(DEV), torch.from_numpy(sZ).to(DEV)
    rec = u8(B, dec.record_bytes())
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(DEV)
    err = None
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            try:
                dec.decode_batch_packed_dev(tX, tZ, 0.01, 50, "fixed", rec, stream=s)
            except q.QecError as e:
                err = e
    torch.cuda.synchronize()
    assert err is not None and "max_batch" in str(err)


def test_device_buffer_validation(env):
    code, dec, _ = env["P7"]
    B = 4
    sX, sZ = u8(B, code.numEqsX), u8(B, code.numEqsZ)
    rec = u8(B, dec.record_bytes())
    bad = [
        (dict(sX=sX.to(torch.int32)), "dtype"),
        (dict(sX=u8(B, code.numEqsX + 1)), "shape"),
        (dict(sZ=u8(2 * B, code.numEqsZ)[::2]), "shape|contiguous"),
        (dict(records=u8(B, dec.record_bytes() - 1)), "shape"),
        (dict(records=u8(B, dec.record_bytes() * 2)[:, ::2]), "contiguous"),
        (dict(sX=sX.cpu()), "cuda:0"),
        (dict(iters=torch.empty((B, 2), dtype=torch.int64, device=DEV)), "dtype"),
    ]
    for kw, msg in bad:
        args = dict(sX=sX, sZ=sZ, records=rec, iters=None)
        args.update(kw)
        with pytest.raises(q.QecError, match=msg):
            dec.decode_batch_packed_dev(args["sX"], args["sZ"], 0.02, 5, "fixed", args["records"], args["iters"])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("seed,start,p", [(0x51EC0DE, 0, 0.01), (12345, (1 << 32) - 3, 0.2), (7, 5, 1.0)])
def test_fused_front_end(env, key, seed, start, p):
    """qec_sample_syndrome_dev == syndromes of qec_sample_depolarizing_dev's errors (the numpy
    restatement of the Philox stream), and its packed errors == the host packing of them."""
    code, dec, _ = env[key]
    B = 1000
    sX, sZ, errp = u8(B, code.numEqsX), u8(B, code.numEqsZ), u8(B, 2 * ((code.n + 7) // 8))
    dec.sample_syndrome_dev(seed, start, p, sX, sZ, errp)
    torch.cuda.synchronize()
    x, z = depolarizing(seed, start, B, code.n, p)
    assert np.array_equal(sX.cpu().numpy(), code.syndrome(0, x))
    assert np.array_equal(sZ.cpu().numpy(), code.syndrome(1, z))
    exp = np.concatenate([np.packbits(x, axis=1, bitorder="little"), np.packbits(z, axis=1, bitorder="little")], 1)
    assert np.array_equal(errp.cpu().numpy(), exp)


@pytest.mark.parametrize("key", ["P7", "P61"])
def test_fused_front_end_wave_width(env, key):
    """The front end's samples per wave grow with the batch (16 .. 64 lanes, montecarlo.hip
    gap_spw); the samples do not depend on it: a 2^18-sample launch (64 per wave) equals the
    numpy restatement on a slice and a 1000-sample launch (16 per wave) of the same indices."""
    code, dec, _ = env[key]
    B, lo, seed, p = 1 << 18, 123456, 99, 0.02
    big = [u8(B, code.numEqsX), u8(B, code.numEqsZ), u8(B, 2 * ((code.n + 7) // 8))]
    dec.sample_syndrome_dev(seed, 0, p, *big)
    small = [u8(1000, code.numEqsX), u8(1000, code.numEqsZ), u8(1000, 2 * ((code.n + 7) // 8))]
    dec.sample_syndrome_dev(seed, lo, p, *small)
    torch.cuda.synchronize()
    for a, b in zip(big, small):
        assert torch.equal(a[lo:lo + 1000], b)
    x, z = depolarizing(seed, lo, 1000, code.n, p)
    assert np.array_equal(small[0].cpu().numpy(), code.syndrome(0, x))
    assert np.array_equal(small[1].cpu().numpy(), code.syndrome(1, z))


@pytest.mark.parametrize("key,B,p,N", [("P7", 4000, 0.06, 30), ("P61", 500, 0.03, 30)])
def test_statistics_packed_equals_byte_form(env, key, B, p, N):
    code, dec, _ = env[key]
    sX, sZ, errp = u8(B, code.numEqsX), u8(B, code.numEqsZ), u8(B, 2 * ((code.n + 7) // 8))
    dec.sample_syndrome_dev(77, 3, p, sX, sZ, errp)
    rec, its = u8(B, dec.record_bytes()), torch.empty((B, 2), dtype=torch.int32, device=DEV)
    dec.decode_batch_packed_dev(sX, sZ, p, N, "ref", rec, its)
    c10 = torch.zeros(10, dtype=torch.int64, device=DEV)
    dec.statistics_packed_dev(errp, rec, c10, iters=its)
    c8p = torch.zeros(8, dtype=torch.int64, device=DEV)
    dec.statistics_packed_dev(errp, rec, c8p)
    x, z = u8(B, code.n), u8(B, code.n)
    dec.sample_depolarizing_dev(77, 3, p, x, z)
    eX, eZ, fl = u8(B, code.n), u8(B, code.n), u8(B)
    dec.decode_batch_dev(sX, sZ, p, N, "ref", eX, eZ, fl)
    c8 = torch.zeros(8, dtype=torch.int64, device=DEV)
    dec.statistics_dev(x, z, eX, eZ, fl, c8)
    torch.cuda.synchronize()
    assert c10[:8].tolist() == c8.tolist() == c8p.tolist()
    itn = its.cpu().numpy()
    assert c10[8].item() == int(itn[:, 0].sum()) and c10[9].item() == int(itn[:, 1].sum())


# ---- multi-device decoder -------------------------------------------------------------------
@pytest.fixture(scope="module")
def multi(code_paths):
    out = {}
    for k, path in code_paths.items():
        code = q.Quantum_LDPC_Code.createFromFile(path)
        out[k] = q.DecoderGPU(code, devices=[0, 0, 0])
    return out


def test_multi_device_shape(multi):
    d = multi["P61"]
    assert d.num_parts == 3 and d.describe().startswith("multi-device [0,0,0]")
    assert [p.device for p in d.parts()] == [0, 0, 0]
    with pytest.raises(q.QecError, match="parts"):
        d.decode_batch_packed_dev(u8(1, 244), u8(1, 305), 0.01, 5, "fixed", u8(1, 155))


@pytest.mark.parametrize("key", ["P7", "P61"])
def test_multi_device_decode_equals_single(env, multi, key):
    code, dec, _ = env[key]
    B = 3001
    sX, sZ = inputs(code, B, 0.02, seed=41)
    a = dec.decode_batch(sX, sZ, 0.02, 30, "ref", want_iters=True)
    b = multi[key].decode_batch(sX, sZ, 0.02, 30, "ref", want_iters=True)
    for x, y in zip(a[:4], b[:4]):
        assert np.array_equal(x, y)
    ra, ia = dec.decode_batch_packed(sX, sZ, 0.02, 30, "fixed", want_iters=True)
    rb, ib = multi[key].decode_batch_packed(sX, sZ, 0.02, 30, "fixed", want_iters=True)
    assert np.array_equal(ra, rb) and np.array_equal(ia, ib)


def test_multi_device_statistics_reproduce_published(multi, kat_records):
    from conftest import COUNTERS, code_key, kat_subset
    from test_gpu_kat import MAP
    for rec in kat_subset(kat_records)[:6]:
        st = multi[code_key(rec)].GetStatistics(rec["W"], rec["tested"], rec["p_run"], rec["MAX"], rec["seed"])
        assert {k: st[MAP[k]] for k in COUNTERS} == {k: rec[k] for k in COUNTERS}, rec["file"]


def test_multi_device_monte_carlo_equals_single(env, multi):
    code, dec, _ = env["P61"]
    a = dec.monte_carlo(9, 100, 20000, 0.02, 50, "syndrome", batch=4096)
    b = multi["P61"].monte_carlo(9, 100, 20000, 0.02, 50, "syndrome", batch=4096)
    for k in q.MC_COUNTERS + ("tested", "iterationsX", "iterationsZ"):
        assert a[k] == b[k], k
