"""The N > 1 path on the GPU: two ranks (gloo, both on GPU 0) each generate
and decode their contiguous shard of the sample index space straight into packed decision
records, and the records are gathered to rank 0 (qec_ldpc_amd.gather); rank 0's gathered batch
must equal a one-process decode of the whole batch byte for byte."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

TOTAL = 3 * 4096 + 77
P, N = 0.01, 50


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, path, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import qec_ldpc_amd as q
    from qec_ldpc_amd.gather import gather_records
    code = q.Quantum_LDPC_Code.createFromFile(path)
    dev = torch.device("cuda", 0)
    lo, hi = TOTAL * rank // world, TOTAL * (rank + 1) // world
    dec = q.DecoderGPU(code, 0)
    sX = torch.empty((hi - lo, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((hi - lo, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_syndrome_dev(0x51EC0DE, lo, P, sX, sZ)
    rec = torch.empty((hi - lo, dec.record_bytes()), dtype=torch.uint8, device=dev)
    dec.decode_batch_packed_dev(sX, sZ, P, N, "fixed", rec)
    torch.cuda.synchronize()
    # equal shard sizes for the gather: pad the shorter shard (TOTAL is odd)
    m = TOTAL - TOTAL * (world - 1) // world
    pad = torch.zeros((m, rec.shape[1]), dtype=torch.uint8, device=dev)
    pad[: hi - lo] = rec
    full = gather_records(pad)
    if rank == 0:
        parts = [full[k * m: k * m + (TOTAL * (k + 1) // world - TOTAL * k // world)] for k in range(world)]
        np.save(out, torch.cat(parts).cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_gather_equals_one_process(tmp_path, code_paths):
    import qec_ldpc_amd as q
    out = str(tmp_path / "rec.npy")
    mp.start_processes(_rank, args=(2, _free_port(), code_paths["P61"], out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    code = q.Quantum_LDPC_Code.createFromFile(code_paths["P61"])
    dec = q.DecoderGPU(code, 0)
    dev = torch.device("cuda", 0)
    sX = torch.empty((TOTAL, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((TOTAL, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_syndrome_dev(0x51EC0DE, 0, P, sX, sZ)
    rec = torch.empty((TOTAL, dec.record_bytes()), dtype=torch.uint8, device=dev)
    dec.decode_batch_packed_dev(sX, sZ, P, N, "fixed", rec)
    torch.cuda.synchronize()
    assert got.shape == (TOTAL, dec.record_bytes())
    assert np.array_equal(got, rec.cpu().numpy())
