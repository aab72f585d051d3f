"""Parity of the HIP engine (through the C ABI) with the oracle (CPU restatement of
DecoderCPU::Decode, QEC_LDPC/DecoderCPU.h:249-390) on identical inputs.

Bar: bit-exact decoded error strings, ErrorCode flags and iteration counts, and
bit-exact final variable->check messages (float32 compared as bit patterns; a NaN
only has to be matched by a NaN).  No tolerance is applied anywhere.
"""
import numpy as np
import pytest

import qec_ldpc_amd as q
from oracle.oracle import OracleCode
from qec_ldpc_amd.synthetic import depolarizing_errors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(code_paths):
    out = {}
    for k, path in code_paths.items():
        code = q.Quantum_LDPC_Code.createFromFile(path)
        out[k] = (code, q.DecoderGPU(code, 0), OracleCode(path))
    return out


def same_floats(a, b):
    an, bn = np.isnan(a), np.isnan(b)
    return np.array_equal(an, bn) and np.array_equal(a.view(np.uint32)[~an], b.view(np.uint32)[~bn])


def mixed_inputs(code, B, seed, p):
    """Depolarising samples, fixed-weight samples, random and extreme syndromes."""
    rng = np.random.default_rng(seed)
    k = B // 4
    x, z = depolarizing_errors(code.n, seed * 100000, k, p)
    sx1, sz1 = code.syndrome(0, x), code.syndrome(1, z)
    wx, wz = q.sample_fixed_weight(seed, int(rng.integers(1, max(2, code.n // 10))), k, code.n)
    sx2, sz2 = code.syndrome(0, wx), code.syndrome(1, wz)
    r = B - 2 * k
    sx3 = (rng.random((r, code.numEqsX)) < rng.random((r, 1))).astype(np.uint8)
    sz3 = (rng.random((r, code.numEqsZ)) < rng.random((r, 1))).astype(np.uint8)
    sx3[0] = 0
    sz3[0] = 0
    sx3[-1] = 1
    sz3[-1] = 1
    return np.concatenate([sx1, sx2, sx3]), np.concatenate([sz1, sz2, sz3])


def check(env, key, sX, sZ, p, N, stop, want_q=True):
    code, dec, orc = env[key]
    g = dec.decode_batch(sX, sZ, p, N, stop, want_iters=True, want_q=want_q)
    o = orc.decode_batch(sX, sZ, p, N, stop, want_q=want_q)
    for name, a, b in zip(("eX", "eZ", "flags", "iters"), g[:4], o[:4]):
        if not np.array_equal(a, b):
            bad = np.nonzero((a != b).reshape(len(a), -1).any(1))[0]
            raise AssertionError("%s %s N=%d p=%g: %s differs on %d/%d rows (first %s)"
                                 % (key, stop, N, p, name, len(bad), len(a), bad[:5]))
    if want_q:
        assert same_floats(g[4], o[4]), "%s %s N=%d: final messages differ" % (key, stop, N)
    return g


@pytest.mark.parametrize("stop", ["fixed", "ref", "syndrome"])
@pytest.mark.parametrize("N", [0, 1, 2, 10, 11, 20, 21, 50])
def test_p7_parity(env, stop, N):
    sX, sZ = mixed_inputs(env["P7"][0], 1003, 7 + N, 0.02)
    check(env, "P7", sX, sZ, 0.02, N, stop)


@pytest.mark.parametrize("stop", ["fixed", "ref", "syndrome"])
@pytest.mark.parametrize("N,p", [(1, 0.01), (11, 0.02), (50, 0.01)])
def test_p61_parity(env, stop, N, p):
    sX, sZ = mixed_inputs(env["P61"][0], 160, 61 + N, p)
    check(env, "P61", sX, sZ, p, N, stop)


@pytest.mark.parametrize("p", [0.0, 1e-30, 0.001, 0.05, 0.1, 0.75, 1.5, 3.0])
def test_extreme_error_probability(env, p):
    """Edge arithmetic: p' = 0, subnormal p', p' = 0.5, p' = 1 (1-p' = 0 -> 0/0 NaN paths)."""
    for key, B, N in (("P7", 300, 12), ("P61", 24, 12)):
        sX, sZ = mixed_inputs(env[key][0], B, 3, 0.05)
        for stop in ("fixed", "ref"):
            check(env, key, sX, sZ, p, N, stop)


@pytest.mark.parametrize("p", [1.4e-6, 1.5e-6, 1e-4, 0.7499999, 0.75, 0.7500001])
def test_scaled_division_domain_edges(env, p):
    """The guard-free scaled short division (bp_decode.hip, scaled_ok) holds for p' in [2^-20, 1/2]:
    p' just below and above both ends (1.4e-6 / 1.5e-6 straddle 2^-20; 0.75 gives p' = 1/2), with 50
    iterations of dense random syndromes driving messages towards 2^-25 and numerators towards their
    lower bound; final messages compared bit for bit."""
    for key, B in (("P7", 400), ("P61", 40)):
        sX, sZ = mixed_inputs(env[key][0], B, 17, 0.05)
        for stop in ("fixed", "ref"):
            check(env, key, sX, sZ, p, 50, stop)


@pytest.mark.parametrize("B", [1, 2, 8, 9, 10, 17, 63, 64, 65, 1000])
def test_ragged_batches(env, B):
    """Batch sizes that leave partial wavefront groups (P7 packs 9 syndromes per wave)."""
    for key in ("P7", "P61"):
        sX, sZ = mixed_inputs(env[key][0], max(B, 4), 11, 0.02)
        for stop in ("ref", "fixed", "syndrome"):
            check(env, key, sX[:B], sZ[:B], 0.02, 15, stop, want_q=False)


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("p", [0.001, 0.002, 0.005, 0.01, 0.05])
def test_syndrome_stop_without_messages(env, key, p):
    """The syndrome stop's shortcuts that apply only when no final messages are requested: a
    sector with a zero syndrome skips to its known outputs, and iteration 0 tests the syndrome
    before forming its messages (bp_decode.hip).  Low p (most sectors zero or stopping at
    iteration 0), a ragged batch whose last P7 wave holds one syndrome, against the oracle."""
    code = env[key][0]
    x, z = depolarizing_errors(code.n, 31337, 1000, p)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    sX[:50] = 0
    sZ[25:75] = 0
    check(env, key, sX, sZ, p, 30, "syndrome", want_q=False)
    check(env, key, sX[:10], sZ[:10], p, 30, "syndrome", want_q=False)


def test_empty_batch(env):
    code, dec, _ = env["P61"]
    eX, eZ, flags, _, _ = dec.decode_batch(np.zeros((0, code.numEqsX), np.uint8),
                                           np.zeros((0, code.numEqsZ), np.uint8), 0.01, 10)
    assert eX.shape == (0, code.n) and flags.shape == (0,)


def test_single_decode_api(env):
    """Decoder::Decode (one pair) == the batched result."""
    code, dec, orc = env["P61"]
    sX, sZ = mixed_inputs(code, 8, 5, 0.02)
    for b in range(8):
        f, ex, ez = dec.Decode(sX[b], sZ[b], 0.02, 30)
        o = orc.decode_batch(sX[b:b + 1], sZ[b:b + 1], 0.02, 30, "ref")
        assert f == o[2][0] and np.array_equal(ex, o[0][0]) and np.array_equal(ez, o[1][0])


def test_generated_code_runtime_shift_kernel(env):
    """A code served by the runtime-shift kernel (not the shipped tables): J=2,K=3,L=6,P=11."""
    g = q.QC_LDPC_CSS(2, 3, 6, 11, 2, 3)
    dec = q.DecoderGPU(g, 0)
    assert "runtime-shift" in dec.describe()
    # oracle needs a file: write the generated code in the reference format (no I-P line content needed)
    import os
    import tempfile
    d = tempfile.mkdtemp()
    path = os.path.join(d, "gen.txt")
    with open(path, "w") as f:
        f.write("2 3 6 11 2 3\n")
        f.write("\t".join(map(str, g.pcm(0).ravel())) + "\n")
        f.write("\t".join(map(str, g.pcm(1).ravel())) + "\n")
        f.write("0\n")
    orc = OracleCode(path)
    rng = np.random.default_rng(9)
    e = (rng.random((400, g.n)) < 0.04).astype(np.uint8)
    sX, sZ = g.syndrome(0, e), g.syndrome(1, e[::-1].copy())
    for stop in ("fixed", "ref", "syndrome"):
        a = dec.decode_batch(sX, sZ, 0.04, 25, stop, want_iters=True, want_q=True)
        b = orc.decode_batch(sX, sZ, 0.04, 25, stop, want_q=True)
        for x, y in zip(a[:4], b[:4]):
            assert np.array_equal(x, y)
        assert same_floats(a[4], b[4])


def test_runtime_shift_kernel_on_shipped_code(env, code_paths):
    """The shipped P61 code through the runtime-shift path (file with a header the generator
    does not reproduce -> no specialisation) gives the same bits."""
    import os
    import tempfile
    lines = open(code_paths["P61"]).read().split("\n")
    lines[0] = "4 5 10 61 9 50"  # tau changed in the header only
    d = tempfile.mkdtemp()
    path = os.path.join(d, "p61_rt.txt")
    with open(path, "w") as f:
        f.write("\n".join(lines))
    code = q.Quantum_LDPC_Code.createFromFile(path)
    dec = q.DecoderGPU(code, 0)
    assert "runtime-shift" in dec.describe()
    sX, sZ = mixed_inputs(code, 64, 21, 0.01)
    a = dec.decode_batch(sX, sZ, 0.01, 50, "fixed", want_iters=True, want_q=True)
    b = env["P61"][1].decode_batch(sX, sZ, 0.01, 50, "fixed", want_iters=True, want_q=True)
    for x, y in zip(a[:4], b[:4]):
        assert np.array_equal(x, y)
    assert same_floats(a[4], b[4])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("p", [0.001, 0.01, 0.05, 0.1])
def test_hard_paths_bit_identical(env, key, p):
    """QEC_OPT_HARD_PATHS (the exact hard-message forms of both updates, taken once every
    message of a sector is +0 or 1.0) changes no output bit: decisions, flags, iteration
    counts and final messages with the option on equal those with it off, and both equal
    the oracle.  Low p saturates almost every sector within a few iterations; high p
    leaves many sectors soft or NaN (0/0 in VarNodeUpdate), which must stay off the path."""
    code, dec, _ = env[key]
    x, z = depolarizing_errors(code.n, 777, 384, p)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    assert dec.get_option("hard_paths") == 1
    for stop in ("fixed", "ref", "syndrome"):
        on = check(env, key, sX, sZ, p, 50, stop)
        dec.set_option("hard_paths", 0)
        try:
            off = dec.decode_batch(sX, sZ, p, 50, stop, want_iters=True, want_q=True)
        finally:
            dec.set_option("hard_paths", 1)
        for a, b in zip(on[:4], off[:4]):
            assert np.array_equal(a, b)
        assert same_floats(on[4], off[4])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("N", [5, 7, 11, 12, 20, 21, 33])
@pytest.mark.parametrize("p", [0.01, 0.07])
def test_cycle_jump_bit_identical(env, key, N, p):
    """QEC_OPT_CYCLE_JUMP (a hard sector whose last two iterations agreed jumps to its last
    iteration, bp_decode.hip cycle_end) changes no output bit: even and odd remaining counts,
    the reference rule's next multiple of 10 before and after N - 1, every stop rule (p = 0.07: many
    syndrome-stop sectors cycle without satisfying their syndrome and jump through var_pass's identity
    passes).  The jump on equals the jump off, and both equal the oracle (final messages included)."""
    code, dec, _ = env[key]
    x, z = depolarizing_errors(code.n, 4242 + N, 256, p)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    for stop in ("fixed", "ref", "syndrome"):
        on = check(env, key, sX, sZ, p, N, stop)
        dec.set_option("cycle_jump", 0)
        try:
            off = dec.decode_batch(sX, sZ, p, N, stop, want_iters=True, want_q=True)
        finally:
            dec.set_option("cycle_jump", 1)
        for a, b in zip(on[:4], off[:4]):
            assert np.array_equal(a, b)
        assert same_floats(on[4], off[4])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("schedule,split", [(0, 0), (0, 2), (2, 0), (2, 2), (3, 0), (3, 2), (0, 3), (2, 3), (4, 0), (4, 2)])
@pytest.mark.parametrize("B", [1, 2, 383])
def test_schedule_and_split_bit_identical(env, key, schedule, split, B):
    """QEC_OPT_SCHEDULE (waves take syndromes heaviest-first, schedule.hip) and
    QEC_OPT_SECTOR_SPLIT (X and Z of a syndrome in two waves, flags merged by atomicOr; 3: two
    sector launches, the Z launch ORing its flags into the X launch's byte) change only which
    wave decodes what: every output bit equals the oracle's under every
    stop rule, for a single syndrome, two, and a ragged batch (P7 packs 9 per wave)."""
    code, dec, _ = env[key]
    sX, sZ = mixed_inputs(code, max(B, 4), 91 + B, 0.02)
    sX, sZ = sX[:B], sZ[:B]
    dec.set_option("schedule", schedule)
    dec.set_option("sector_split", split)
    try:
        for stop, N in (("fixed", 21), ("ref", 50), ("syndrome", 30)):
            check(env, key, sX, sZ, 0.02, N, stop)
    finally:
        dec.set_option("schedule", 1)
        dec.set_option("sector_split", 1)


@pytest.mark.parametrize("key", ["P7", "P61"])
def test_split_flags_unaligned_and_dirty(env, key):
    """With the sector split the launch zeroes flags[] and each sector ORs its bits into the
    aligned 32-bit word that holds the byte: an output buffer that starts with garbage and
    sits at an odd address must come out right, and the bytes either side must be untouched."""
    import torch
    code, dec, _ = env[key]
    B = 301
    sX, sZ = mixed_inputs(code, B, 5, 0.05)
    dev = torch.device("cuda", 0)
    ref = check(env, key, sX, sZ, 0.05, 20, "fixed", want_q=False)
    tX, tZ = torch.from_numpy(sX).to(dev), torch.from_numpy(sZ).to(dev)
    eX = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    eZ = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    # schedule 2: the order pass zeroes flags; split 3: sector launches (X stores, Z ORs into that byte)
    for off, sched, split in ((0, 0, 2), (1, 0, 2), (2, 0, 2), (3, 0, 2), (1, 2, 2), (2, 2, 2), (3, 3, 2),
                              (1, 0, 3), (3, 2, 3)):
        buf = torch.full((B + 8,), 0xA5, dtype=torch.uint8, device=dev)
        fl = buf[off:off + B]
        dec.set_option("sector_split", split)
        dec.set_option("schedule", sched)
        try:
            dec.decode_batch_dev(tX, tZ, 0.05, 20, "fixed", eX, eZ, fl)
            torch.cuda.synchronize()
        finally:
            dec.set_option("sector_split", 1)
            dec.set_option("schedule", 1)
        h = buf.cpu().numpy()
        assert np.array_equal(h[off:off + B], ref[2]), "offset %d" % off
        assert (h[:off] == 0xA5).all() and (h[off + B:] == 0xA5).all(), "offset %d: neighbours changed" % off
        assert np.array_equal(eX.cpu().numpy(), ref[0]) and np.array_equal(eZ.cpu().numpy(), ref[1])


@pytest.mark.parametrize("key", ["P7", "P61"])
def test_schedule_many_chunks_identical(env, key):
    """A ragged batch spread over many counting-sort chunks (schedule.hip) decodes to the
    same bits sorted, in the local (rank-interleaved chunk) order and in batch order."""
    code, dec, _ = env[key]
    B = 70001
    x, z = depolarizing_errors(code.n, 99, B, 0.03)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    outs = []
    for sched in (2, 3, 0):  # sorted, local order, batch order
        dec.set_option("schedule", sched)
        try:
            outs.append(dec.decode_batch(sX, sZ, 0.03, 20, "ref", want_iters=True))
        finally:
            dec.set_option("schedule", 1)
    for o in outs[1:]:
        for a, b in zip(outs[0][:4], o[:4]):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("key,B", [("P7", 70001), ("P7", 600001), ("P61", 70001)])
def test_per_sector_order_identical(env, key, B):
    """The sector-split launch (split waves, 2, or sector launches, 3) takes each sector's waves in
    the order of that sector's weight (schedule.hip, perm[0, B) for X and perm[B, 2 B) for Z; P7
    600 001 spreads the order pass over 147 chunks of the fused scatter): the same bits as one wave
    per syndrome group in total-weight order and as batch order."""
    code, dec, _ = env[key]
    x, z = depolarizing_errors(code.n, 7 + B, B, 0.03)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    outs = []
    for sched, split in ((2, 2), (2, 3), (2, 0), (0, 2), (0, 0)):
        dec.set_option("schedule", sched)
        dec.set_option("sector_split", split)
        try:
            outs.append(dec.decode_batch(sX, sZ, 0.03, 20, "fixed", want_iters=True))
        finally:
            dec.set_option("schedule", 1)
            dec.set_option("sector_split", 1)
    for o in outs[1:]:
        for a, b in zip(outs[0][:4], o[:4]):
            assert np.array_equal(a, b)


def test_schedule_workspace_across_calls(env):
    """The dispatch-order counters live in the decoder's workspace and are re-zeroed by the
    launches themselves (double-buffered by call parity): many ordered calls in a row, with
    the batch size changing (and the workspace growing) between them, each decode to the same
    bits as batch order."""
    code, dec, _ = env["P61"]
    x, z = depolarizing_errors(code.n, 31, 9000, 0.02)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    ref = {}
    dec.set_option("schedule", 0)
    try:
        for B in (5000, 9000, 4097):
            ref[B] = dec.decode_batch(sX[:B], sZ[:B], 0.02, 12, "fixed", want_iters=True)
    finally:
        dec.set_option("schedule", 1)
    dec.set_option("schedule", 2)
    try:
        for B in (5000, 9000, 4097, 5000, 9000, 9000, 4097, 2, 5000):
            if B not in ref:
                continue
            got = dec.decode_batch(sX[:B], sZ[:B], 0.02, 12, "fixed", want_iters=True)
            for a, b in zip(got[:4], ref[B][:4]):
                assert np.array_equal(a, b), "B=%d" % B
    finally:
        dec.set_option("schedule", 1)


def test_p7_order_across_calls(env):
    """Many ordered P7 calls in a row -- batch sizes changing, the local order (schedule 3) and batch
    order in between, the workspace growing -- each decode to the batch-order bits."""
    code, dec, _ = env["P7"]
    x, z = depolarizing_errors(code.n, 77, 70000, 0.03)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    ref = {}
    dec.set_option("schedule", 0)
    try:
        for B in (5000, 9001, 4097, 70000):
            ref[B] = dec.decode_batch(sX[:B], sZ[:B], 0.03, 20, "fixed", want_iters=True)
    finally:
        dec.set_option("schedule", 1)
    try:
        for B, sched in ((5000, 2), (9001, 2), (9001, 3), (4097, 2), (70000, 2), (5000, 0), (5000, 2), (9001, 2),
                         (70000, 1), (4097, 1)):
            dec.set_option("schedule", sched)
            got = dec.decode_batch(sX[:B], sZ[:B], 0.03, 20, "fixed", want_iters=True)
            for a, b in zip(got[:4], ref[B][:4]):
                assert np.array_equal(a, b), "B=%d schedule=%d" % (B, sched)
    finally:
        dec.set_option("schedule", 1)


@pytest.mark.parametrize("key,B", [("P7", 70001), ("P7", 1024 * 1024 + 3), ("P61", 70001), ("P61", 300001)])
def test_schedule_covers_every_syndrome(env, key, B):
    """The order pass (schedule.hip) is a permutation of the batch: with output buffers
    that start as garbage, an ordered decode writes every syndrome's eX, eZ, flags and
    iterations exactly as the batch-order decode does.  Sizes cover both histogram shapes
    (short rows: one thread per syndrome, 1 024-syndrome chunks; long rows: four threads,
    256-syndrome chunks), a ragged last chunk, and chunks longer than one histogram pass
    (more than 1 024 chunks' worth of minimum-size chunks)."""
    import torch
    code, dec, _ = env[key]
    dev = torch.device("cuda", 0)
    x = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    z = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_depolarizing_dev(7 + B, 0, 0.03, x, z)
    dec.syndrome_dev(x, z, sX, sZ)
    del x, z
    outs = []
    for sched in (0, 2):
        o = [torch.full((B, code.n), 0xA5, dtype=torch.uint8, device=dev),
             torch.full((B, code.n), 0xA5, dtype=torch.uint8, device=dev),
             torch.full((B,), 0xA5, dtype=torch.uint8, device=dev),
             torch.full((B, 2), -7, dtype=torch.int32, device=dev)]
        dec.set_option("schedule", sched)
        try:
            dec.decode_batch_dev(sX, sZ, 0.03, 12, "ref", *o)
            torch.cuda.synchronize()
        finally:
            dec.set_option("schedule", 1)
        outs.append(o)
    assert int(outs[0][3].min()) >= 1  # batch order wrote every syndrome
    for name, a, b in zip(("eX", "eZ", "flags", "iters"), outs[0], outs[1]):
        assert torch.equal(a, b), "%s B=%d: %s differs between batch and dispatch order" % (key, B, name)


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("engine", ["circulant", "sparse"])
@pytest.mark.parametrize("stop", ["ref", "fixed", "syndrome"])
def test_non_binary_syndrome_entries(env, key, engine, stop):
    """Syndrome bytes other than 0 / 1: the check update takes their truthiness (DecoderCPU.h:178),
    the syndrome tests their exact value (:381) -- such a sector decodes as with a 1 there and
    always reports SYNDROME_FAIL; the syndrome stop never stops on it.  Against the oracle, with
    and without final messages (the syndrome stop's message-free shortcuts)."""
    code, _, orc = env[key]
    dec = q.DecoderGPU(code, 0, engine=engine)
    B = 64 if key == "P61" else 500
    x, z = depolarizing_errors(code.n, 4242, B, 0.02)
    sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
    rng = np.random.default_rng(9)
    for s in (sX, sZ):
        rows = rng.choice(B, B // 3, replace=False)
        s[rows, rng.integers(0, s.shape[1], B // 3)] = rng.choice(np.array([2, 3, 128, 255], np.uint8), B // 3)
    sX[-1] = 0
    sX[-1, 0] = 7  # otherwise-zero syndrome with one non-binary entry
    for want_q in (True, False):
        g = dec.decode_batch(sX, sZ, 0.02, 12, stop, want_iters=True, want_q=want_q)
        o = orc.decode_batch(sX, sZ, 0.02, 12, stop, want_q=want_q)
        for name, a, b in zip(("eX", "eZ", "flags", "iters"), g[:4], o[:4]):
            assert np.array_equal(a, b), (name, want_q)
        if want_q:
            assert same_floats(g[4], o[4])
    assert (g[2][(sX > 1).any(1)] & 1).all()


@pytest.mark.parametrize("key,B", [("P7", 65536), ("P7", 5000), ("P61", 65536)])
def test_one_launch_order_repeated(env, key, B):
    """QEC_OPT_SCHEDULE = 4: the dispatch order in one launch with a software grid barrier (schedule.hip,
    schedule_one_launch_kernel; its barrier words must come back zeroed after every launch): five
    calls in a row give the records of the unordered decode."""
    import torch
    code, dec, _ = env[key]
    x, z = depolarizing_errors(code.n, 99 + B, B, 0.02)
    dev = torch.device("cuda", 0)
    tX = torch.from_numpy(code.syndrome(0, x)).to(dev)
    tZ = torch.from_numpy(code.syndrome(1, z)).to(dev)
    outs = []
    try:
        for sched in (0, 4, 4, 4, 4, 4):
            dec.set_option("schedule", sched)
            rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
            its = torch.empty((B, 2), dtype=torch.int32, device=dev)
            dec.decode_batch_packed_dev(tX, tZ, 0.02, 20, "fixed", rec, its)
            torch.cuda.synchronize()
            outs.append((rec.cpu().numpy(), its.cpu().numpy()))
    finally:
        dec.set_option("schedule", 1)
    for r, it in outs[1:]:
        assert np.array_equal(r, outs[0][0]) and np.array_equal(it, outs[0][1])


@pytest.mark.parametrize("key", ["P7", "P61"])
@pytest.mark.parametrize("stop", ["fixed", "ref"])
@pytest.mark.parametrize("N", [2, 3, 10, 11, 20, 21, 50])
def test_zero_syndrome_outcome(env, key, stop, N):
    """Zero-syndrome sectors under the fixed and reference stops take the launch's precomputed outcome
    (bp_decode.hip, zero_outcome) when no final messages are requested: whole waves of zero syndromes,
    zero X with nonzero Z and the reverse, mixed into nonzero rows, at p from 1e-4 to 1.4 (decisions,
    convergence and syndrome flags of either value) -- against the oracle."""
    code = env[key][0]
    rng = np.random.default_rng(N)
    for p in (1e-4, 0.01, 0.2, 0.74, 0.76, 1.4):
        B = 200
        x, z = depolarizing_errors(code.n, 7 * N, B, min(p, 0.3))
        sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
        sX[:64] = 0
        sZ[:64] = 0           # whole waves (P7: 9 per wave) of zero pairs
        sX[64:100] = 0        # zero X, nonzero Z
        sZ[100:130] = 0       # zero Z, nonzero X
        pick = rng.random(B) < 0.3
        sX[pick & (np.arange(B) >= 130)] = 0
        check(env, key, sX, sZ, p, N, stop, want_q=False)


@pytest.mark.parametrize("p", [0.03, 0.07, 0.1])
def test_syndrome_stop_sector_launches(env, p):
    """The syndrome stop through the sector launches (P61, 2^18 syndromes, QEC_OPT_SECTOR_SPLIT 3: ordered,
    an X and a Z launch, row-0-first tests, repeated-decision skips): the whole batch equals the
    one-wave-per-syndrome launch in batch order, the sector launches with the cycle jump off and the
    default choice, and a slice (the heaviest syndromes of each sector among it) equals the oracle."""
    import torch
    from qec_ldpc_amd.gather import pack_records
    code, _, orc = env["P61"]
    B = 1 << 18
    dev = torch.device("cuda", 0)
    dec = q.DecoderGPU(code, 0, max_batch=B)
    sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_syndrome_dev(0xC0DE, 0, p, sX, sZ)

    def run(**opts):
        for k, v in opts.items():
            dec.set_option(k, v)
        rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
        its = torch.empty((B, 2), dtype=torch.int32, device=dev)
        try:
            dec.decode_batch_packed_dev(sX, sZ, p, 50, "syndrome", rec, its)
            torch.cuda.synchronize()
            return rec, its, dec.last_path()
        finally:
            for k in opts:
                dec.set_option(k, 1)

    rec, its, path = run(sector_split=3)  # the sector launches (auto: at 2^20 and p >= 0.03)
    assert "sector_launches" in path, sorted(path)
    for opts in ({"schedule": 0, "sector_split": 0}, {"sector_split": 3, "cycle_jump": 0}, {}):
        r2, i2, _ = run(**opts)
        assert torch.equal(rec, r2) and torch.equal(its, i2), opts
    hX, hZ = sX.cpu().numpy(), sZ.cpu().numpy()
    wX, wZ = hX.sum(1, dtype=np.int64), hZ.sum(1, dtype=np.int64)
    idx = np.unique(np.concatenate([np.arange(512), np.argsort(-wX, kind="stable")[:128],
                                    np.argsort(-wZ, kind="stable")[:128]]))
    o = orc.decode_batch(hX[idx], hZ[idx], p, 50, "syndrome")
    assert np.array_equal(rec.cpu().numpy()[idx], pack_records(o[0], o[1], o[2]))
    assert np.array_equal(its.cpu().numpy()[idx], o[3])
