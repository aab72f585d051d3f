"""The exact launch sequence bench.py times, checked at every per-GPU batch the driver's lines use.

bench.py's step is `decode_bits_packed_dev` with default options on device-sampled syndromes in bit
rows (BASELINE configs[3]: 2^20 P61 syndromes, 50 fixed iterations, p = 0.01; its N = 2/4/8 shards
524 288 / 262 144 / 131 072; configs[1]: P7, 65 536, 20 fixed, p = 0.02).  At those shapes the
decoder picks launch forms no smaller test reaches: the bit-row histogram of the per-sector dispatch
order, and the X and Z sector launches (P61 from 2^18) or split waves (P7).  Each case

  * asserts the launch sequence the call took (QEC_OPT_LAST_PATH), so the comparison below is of
    the timed path and not of a neighbour;
  * compares the records and iteration counts of the whole batch with the byte-row entry in batch
    order, one wave per syndrome (schedule 0, sector split 0) and with the byte-row entry's defaults;
  * compares an oracle slice (QEC_LDPC/DecoderCPU.h:317-390 restated in oracle/qec_oracle.c):
    a contiguous block, the heaviest syndromes of each sector (which the per-sector order dispatches
    first) and a random draw from the whole batch.

The reference stop rule through the bit-row entry is checked the same way at 2^20.
"""
import numpy as np
import pytest

import qec_ldpc_amd as q
from oracle.oracle import OracleCode
from qec_ldpc_amd.gather import pack_records
from qec_ldpc_amd.synthetic import bit_rows

pytestmark = pytest.mark.gpu

SEED = 0x51EC0DE  # bench.py's seed
FULL = 1 << 20
# (id, code, per-GPU batch, first sample (bench.py's last rank), p, iterations, launch sequence bench.py times)
BASE = {"bit_rows", "records", "ordered"}
CASES = [
    ("p61_2e20", "P61", FULL, 0, 0.01, 50, BASE | {"sector_order", "sector_launches"}),
    ("p61_n2", "P61", FULL // 2, FULL // 2, 0.01, 50, BASE | {"sector_order", "sector_launches"}),
    ("p61_n4", "P61", FULL // 4, FULL - FULL // 4, 0.01, 50, BASE | {"sector_order", "sector_launches"}),
    ("p61_n8", "P61", FULL // 8, FULL - FULL // 8, 0.01, 50, BASE),
    ("p7_65536", "P7", 65536, 0, 0.02, 20, BASE | {"sector_order", "split_waves"}),
]


def heaviest(w, k):
    """Indices of the k largest weights (ties by index)."""
    return np.argsort(-w, kind="stable")[:k]


@pytest.fixture(scope="module", params=CASES, ids=[c[0] for c in CASES])
def timed(request, code_paths):
    import torch
    cid, key, B, lo, p, N, path = request.param
    code = q.Quantum_LDPC_Code.createFromFile(code_paths[key])
    dev = torch.device("cuda", 0)
    dec = q.DecoderGPU(code, 0, max_batch=B)  # bench.py's decoder: default options
    sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_syndrome_dev(SEED, lo, p, sX, sZ)
    sXb, sZb = bit_rows(sX), bit_rows(sZ)
    rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
    its = torch.empty((B, 2), dtype=torch.int32, device=dev)
    dec.decode_bits_packed_dev(sXb, sZb, p, N, "fixed", rec, its)
    torch.cuda.synchronize()
    taken = dec.last_path()
    yield dict(id=cid, key=key, code=code, dec=dec, B=B, p=p, N=N, want=path, taken=taken, sX=sX, sZ=sZ,
               sXb=sXb, sZb=sZb, rec=rec, its=its, path=code_paths[key])
    del sX, sZ, sXb, sZb, rec, its
    torch.cuda.empty_cache()


def byte_row_decode(t, stop, **opts):
    import torch
    dec = q.DecoderGPU(t["code"], 0, max_batch=t["B"])
    for k, v in opts.items():
        dec.set_option(k, v)
    rec = torch.empty_like(t["rec"])
    its = torch.empty_like(t["its"])
    dec.decode_batch_packed_dev(t["sX"], t["sZ"], t["p"], t["N"], stop, rec, its)
    torch.cuda.synchronize()
    return rec, its, dec.last_path()


def oracle_slice(t, n_block, n_heavy, n_rand, seed):
    B = t["B"]
    if n_block >= B:
        return np.arange(B)
    sX = t["sX"].cpu().numpy()
    sZ = t["sZ"].cpu().numpy()
    wX, wZ = sX.sum(1, dtype=np.int64), sZ.sum(1, dtype=np.int64)
    rng = np.random.default_rng(seed)
    idx = np.concatenate([np.arange(B // 3, B // 3 + n_block), heaviest(wX, n_heavy), heaviest(wZ, n_heavy),
                          heaviest(wX + wZ, n_heavy), rng.choice(B, n_rand, replace=False)])
    return np.unique(idx)


def test_timed_launch_sequence(timed):
    assert timed["taken"] == timed["want"], (timed["id"], sorted(timed["taken"]))


def test_timed_path_equals_batch_order_whole_batch(timed):
    import torch
    rec, its, path = byte_row_decode(timed, "fixed", schedule=0, sector_split=0)
    assert path == {"records"}, sorted(path)
    assert torch.equal(rec, timed["rec"])
    assert torch.equal(its, timed["its"])
    assert bool((timed["its"] == timed["N"]).all())


def test_timed_path_equals_byte_row_defaults_whole_batch(timed):
    import torch
    rec, its, path = byte_row_decode(timed, "fixed")
    assert "bit_rows" not in path
    assert torch.equal(rec, timed["rec"])
    assert torch.equal(its, timed["its"])


def test_timed_path_oracle_slice(timed):
    """4 096 (P61 2^20) / 2 048 (shards) contiguous syndromes, the 256 heaviest of each sector and of
    both, and 192 from anywhere; P7 65 536: the whole batch."""
    t = timed
    n_block = 65536 if t["key"] == "P7" else (4096 if t["B"] == FULL else 2048)
    idx = oracle_slice(t, n_block, 256, 192, 77)
    o = OracleCode(t["path"]).decode_batch(t["sX"].cpu().numpy()[idx], t["sZ"].cpu().numpy()[idx], t["p"], t["N"],
                                           "fixed")
    assert np.array_equal(t["rec"].cpu().numpy()[idx], pack_records(o[0], o[1], o[2]))
    assert np.array_equal(t["its"].cpu().numpy()[idx], o[3])


def test_timed_path_ref_stop(timed):
    """The reference stop rule (DecoderCPU.h:280-291) through the bit-row entry: whole batch equal
    to the byte-row entry in batch order, and an oracle slice (P61 2^20 and P7 only)."""
    import torch
    t = timed
    if t["B"] not in (FULL, 65536):
        pytest.skip("reference stop checked at the N = 1 batch and P7")
    rec = torch.empty_like(t["rec"])
    its = torch.empty_like(t["its"])
    t["dec"].decode_bits_packed_dev(t["sXb"], t["sZb"], t["p"], t["N"], "ref", rec, its)
    torch.cuda.synchronize()
    assert {"bit_rows", "records", "ordered"} <= t["dec"].last_path()
    r0, i0, _ = byte_row_decode(t, "ref", schedule=0, sector_split=0)
    assert torch.equal(rec, r0) and torch.equal(its, i0)
    idx = oracle_slice(t, 4096 if t["key"] == "P61" else 65536, 128, 128, 78)
    o = OracleCode(t["path"]).decode_batch(t["sX"].cpu().numpy()[idx], t["sZ"].cpu().numpy()[idx], t["p"], t["N"], "ref")
    assert np.array_equal(rec.cpu().numpy()[idx], pack_records(o[0], o[1], o[2]))
    assert np.array_equal(its.cpu().numpy()[idx], o[3])
