"""Multi-rank path on CPU (gloo, world size 2): each rank generates and processes its
own contiguous shard of the sample index space, so results are independent of the
number of ranks; the only collectives are the timing
MAX-reduction and (optionally) a gather of decisions / sum of counters."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from qec_ldpc_amd.synthetic import BLOCK, depolarizing_errors, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, path, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import qec_ldpc_amd as q
    code = q.Quantum_LDPC_Code.createFromFile(path)
    total = 3 * BLOCK + 77
    lo, hi = shard_range(total, rank, world)
    x, z = depolarizing_errors(code.n, lo, hi - lo, 0.02)
    s = torch.from_numpy(np.concatenate([code.syndrome(0, x), code.syndrome(1, z)], 1).astype(np.int64))
    # gather variable-size shards (pad to max), as the decision gather would
    n = torch.tensor([s.shape[0]])
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = int(max(t.item() for t in sizes))
    pad = torch.zeros((mx, s.shape[1]), dtype=torch.int64)
    pad[: s.shape[0]] = s
    parts = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    counters = torch.tensor([int(x.any(1).sum()), int(z.any(1).sum())], dtype=torch.int64)
    dist.all_reduce(counters)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        full = torch.cat([p[: int(sz.item())] for p, sz in zip(parts, sizes)]).numpy()
        np.savez(out, full=full, counters=counters.numpy(), tmax=t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_partition():
    for total in (1, 7, 65536, 2 ** 20 + 3):
        for world in (1, 2, 3, 8):
            r = [shard_range(total, k, world) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))


def test_generation_independent_of_sharding():
    x, z = depolarizing_errors(42, 0, 2 * BLOCK + 10, 0.05)
    for lo, hi in ((0, 5), (BLOCK - 3, BLOCK + 9), (100, 2 * BLOCK + 10)):
        xs, zs = depolarizing_errors(42, lo, hi - lo, 0.05)
        assert np.array_equal(xs, x[lo:hi]) and np.array_equal(zs, z[lo:hi])


def test_two_rank_gloo_matches_single_process(tmp_path, code_paths):
    out = str(tmp_path / "r.npz")
    mp.start_processes(_worker, args=(2, _free_port(), code_paths["P7"], out), nprocs=2, join=True,
                       start_method="spawn")
    import qec_ldpc_amd as q
    code = q.Quantum_LDPC_Code.createFromFile(code_paths["P7"])
    total = 3 * BLOCK + 77
    x, z = depolarizing_errors(code.n, 0, total, 0.02)
    ref = np.concatenate([code.syndrome(0, x), code.syndrome(1, z)], 1)
    r = np.load(out)
    assert np.array_equal(r["full"], ref)
    assert r["counters"].tolist() == [int(x.any(1).sum()), int(z.any(1).sum())]
    assert r["tmax"][0] == 2.0


def _gather_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qec_ldpc_amd.gather import gather_records
    rec = torch.full((5, 13), rank + 1, dtype=torch.uint8)
    rec[:, 0] = torch.arange(5, dtype=torch.uint8) + 10 * rank
    full = gather_records(rec)
    if rank == 0:
        np.save(out, full.numpy())
    else:
        assert full is None
    dist.barrier()
    dist.destroy_process_group()


def test_gather_records_two_ranks(tmp_path):
    """The decision gather (qec_ldpc_amd.gather): rank 0 receives every
    rank's records in rank order."""
    out = str(tmp_path / "g.npy")
    mp.start_processes(_gather_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    full = np.load(out)
    assert full.shape == (10, 13)
    assert (full[:5, 1:] == 1).all() and (full[5:, 1:] == 2).all()
    assert full[:, 0].tolist() == [0, 1, 2, 3, 4, 10, 11, 12, 13, 14]


def test_pack_unpack_records_roundtrip():
    from qec_ldpc_amd.gather import pack_records, unpack_records
    rng = np.random.default_rng(3)
    for n in (42, 610, 7, 8, 9):
        eX = (rng.random((17, n)) < 0.3).astype(np.uint8)
        eZ = (rng.random((17, n)) < 0.3).astype(np.uint8)
        fl = rng.integers(0, 16, 17).astype(np.uint8)
        rec = pack_records(eX, eZ, fl)
        assert rec.shape == (17, 2 * ((n + 7) // 8) + 1)
        a, b, c = unpack_records(rec, n)
        assert np.array_equal(a, eX) and np.array_equal(b, eZ) and np.array_equal(c, fl)
