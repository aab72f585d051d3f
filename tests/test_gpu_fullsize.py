"""BASELINE.json configs at full size on the GPU (configs[1]: P7 x 65536 @ 20 fixed
iterations, configs[2]: P61 x 65536 @ 50 fixed iterations), checked through
size-independent properties: oracle parity on a random subsample, determinism,
batch-split invariance, device-pointer == host-pointer entry point, and the
decision syndrome identity (flags say SYNDROME_FAIL exactly when H e != s)."""
import numpy as np
import pytest

import qec_ldpc_amd as q
from oracle.oracle import OracleCode
from qec_ldpc_amd.synthetic import depolarizing_errors

pytestmark = pytest.mark.gpu

CONFIGS = [("P7", 65536, 20, 0.02), ("P61", 65536, 50, 0.01)]


@pytest.fixture(scope="module", params=CONFIGS, ids=[c[0] for c in CONFIGS])
def run(request, code_paths):
    key, B, N, p = request.param
    code = q.Quantum_LDPC_Code.createFromFile(code_paths[key])
    dec = q.DecoderGPU(code, 0)
    x, z = depolarizing_errors(code.n, 0, B, p)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    out = dec.decode_batch(sX, sZ, p, N, "fixed", want_iters=True)
    return dict(key=key, code=code, dec=dec, B=B, N=N, p=p, sX=sX, sZ=sZ, x=x, z=z, out=out,
                path=code_paths[key])


def test_oracle_subsample(run):
    """configs[1] (P7, ~0.1 s of oracle time): the whole batch; configs[2]: a 4 096-syndrome slice
    plus 256 syndromes drawn from the whole batch."""
    if run["key"] == "P7":
        idx = np.arange(run["B"])
    else:
        rng = np.random.default_rng(123)
        idx = np.unique(np.concatenate([np.arange(20000, 20000 + 4096), rng.choice(run["B"], 256, replace=False)]))
    o = OracleCode(run["path"]).decode_batch(run["sX"][idx], run["sZ"][idx], run["p"], run["N"], "fixed")
    for a, b in zip(run["out"][:4], o[:4]):
        assert np.array_equal(a[idx], b)


def test_deterministic(run):
    again = run["dec"].decode_batch(run["sX"], run["sZ"], run["p"], run["N"], "fixed", want_iters=True)
    for a, b in zip(run["out"][:4], again[:4]):
        assert np.array_equal(a, b)


def test_split_invariance(run):
    h = run["B"] // 2 + 5
    lo = run["dec"].decode_batch(run["sX"][:h], run["sZ"][:h], run["p"], run["N"], "fixed")
    hi = run["dec"].decode_batch(run["sX"][h:], run["sZ"][h:], run["p"], run["N"], "fixed")
    for k in range(3):
        assert np.array_equal(np.concatenate([lo[k], hi[k]]), run["out"][k])


def test_device_entry_point(run):
    import torch
    dev = torch.device("cuda:0")
    c = run["code"]
    B = run["B"]
    sX = torch.from_numpy(run["sX"]).to(dev)
    sZ = torch.from_numpy(run["sZ"]).to(dev)
    eX = torch.empty((B, c.n), dtype=torch.uint8, device=dev)
    eZ = torch.empty((B, c.n), dtype=torch.uint8, device=dev)
    fl = torch.empty(B, dtype=torch.uint8, device=dev)
    it = torch.empty((B, 2), dtype=torch.int32, device=dev)
    run["dec"].decode_batch_dev(sX, sZ, run["p"], run["N"], "fixed", eX, eZ, fl, it)
    torch.cuda.synchronize()
    for a, b in zip((eX, eZ, fl, it), run["out"][:4]):
        assert np.array_equal(a.cpu().numpy(), b)


def test_flags_consistent_with_syndromes(run):
    c = run["code"]
    eX, eZ, flags, iters, _ = run["out"]
    synx = (c.syndrome(0, eX) != run["sX"]).any(1)
    synz = (c.syndrome(1, eZ) != run["sZ"]).any(1)
    assert np.array_equal(synx, (flags & q.SYNDROME_FAIL_X) != 0)
    assert np.array_equal(synz, (flags & q.SYNDROME_FAIL_Z) != 0)
    assert (iters == run["N"]).all()
    # the decoder actually decodes: most low-p samples satisfy their syndromes
    assert synx.mean() < 0.5 and synz.mean() < 0.5


def test_hard_paths_off_identical(run):
    """The bench's full-size batch decodes to the same bits with the hard-message paths off."""
    dec = run["dec"]
    dec.set_option("hard_paths", 0)
    try:
        off = dec.decode_batch(run["sX"], run["sZ"], run["p"], run["N"], "fixed", want_iters=True)
    finally:
        dec.set_option("hard_paths", 1)
    for a, b in zip(run["out"][:4], off[:4]):
        assert np.array_equal(a, b)


def test_schedule_split_off_identical(run):
    """The full-size batch decodes to the same bits in batch order, one wave per syndrome
    (QEC_OPT_SCHEDULE = 0, QEC_OPT_SECTOR_SPLIT = 0), as with the defaults."""
    dec = run["dec"]
    dec.set_option("schedule", 0)
    dec.set_option("sector_split", 0)
    try:
        off = dec.decode_batch(run["sX"], run["sZ"], run["p"], run["N"], "fixed", want_iters=True)
    finally:
        dec.set_option("schedule", 1)
        dec.set_option("sector_split", 1)
    for a, b in zip(run["out"][:4], off[:4]):
        assert np.array_equal(a, b)


# ---- BASELINE configs[3]: 2^20 P61 syndromes @ 50 fixed iterations ---------------------------
@pytest.fixture(scope="module")
def mega(code_paths):
    """The whole configs[3] batch decoded on one GPU in one packed launch, plus its syndromes."""
    import torch
    code = q.Quantum_LDPC_Code.createFromFile(code_paths["P61"])
    B = 1 << 20
    dec = q.DecoderGPU(code, 0, max_batch=B)
    dev = torch.device("cuda", 0)
    sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_syndrome_dev(0x51EC0DE, 0, 0.01, sX, sZ)
    rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
    dec.decode_batch_packed_dev(sX, sZ, 0.01, 50, "fixed", rec)
    torch.cuda.synchronize()
    return dict(code=code, dec=dec, B=B, sX=sX, sZ=sZ, rec=rec, path=code_paths["P61"])


def test_configs3_oracle_subsample(mega):
    """A 4 096-syndrome slice at the end of the batch plus 192 syndromes drawn from all of it."""
    rng = np.random.default_rng(2020)
    idx = np.unique(np.concatenate([np.arange(mega["B"] - 4096, mega["B"]), rng.choice(mega["B"], 192, replace=False)]))
    sX = mega["sX"].cpu().numpy()[idx]
    sZ = mega["sZ"].cpu().numpy()[idx]
    o = OracleCode(mega["path"]).decode_batch(sX, sZ, 0.01, 50, "fixed")
    from qec_ldpc_amd.gather import pack_records
    assert np.array_equal(mega["rec"].cpu().numpy()[idx], pack_records(o[0], o[1], o[2]))


def test_configs3_shards_equal_single_launch(mega):
    """configs[3]'s sharding: 8 contiguous shards decoded separately and gathered (concatenated in
    rank order) give the single launch's records byte for byte."""
    import torch
    B, dec = mega["B"], mega["dec"]
    parts = []
    for g in range(8):
        lo, hi = g * B // 8, (g + 1) * B // 8
        r = torch.empty((hi - lo, dec.record_bytes()), dtype=torch.uint8, device=mega["rec"].device)
        dec.decode_batch_packed_dev(mega["sX"][lo:hi], mega["sZ"][lo:hi], 0.01, 50, "fixed", r)
        parts.append(r)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts), mega["rec"])


def test_configs3_flags_consistent(mega):
    """Flag bits against a recomputed H e on a 16 384-syndrome slice, and the batch decodes
    (most low-p syndromes are satisfied)."""
    from qec_ldpc_amd.gather import unpack_records
    code = mega["code"]
    sl = slice(500000, 500000 + 16384)
    eX, eZ, fl = unpack_records(mega["rec"][sl].cpu().numpy(), code.n)
    synx = (code.syndrome(0, eX) != mega["sX"][sl].cpu().numpy()).any(1)
    synz = (code.syndrome(1, eZ) != mega["sZ"][sl].cpu().numpy()).any(1)
    assert np.array_equal(synx, (fl & q.SYNDROME_FAIL_X) != 0)
    assert np.array_equal(synz, (fl & q.SYNDROME_FAIL_Z) != 0)
    assert synx.mean() < 0.01 and synz.mean() < 0.01
