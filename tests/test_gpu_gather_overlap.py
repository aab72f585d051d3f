"""The overlapped decode + gather of the multi-GPU path (qec_ldpc_amd.gather.GatherPipeline):
two gloo ranks on GPU 0 each decode K steps, step k being its contiguous shard of samples
[k T, (k + 1) T), into two alternating record buffers, while the previous step's records are gathered
to rank 0 on a communication stream.  Rank 0's gathered records of every step must equal a
one-process decode of that step's samples byte for byte (the reference's sample-parallel loop is
QEC_LDPC/DecoderCPU.h:419-438).  The RCCL branch of the same pipeline runs at world size 1 in
tests/test_gpu_rccl.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T = 2 * 3001  # samples per step over both ranks (equal shards)
K = 4
P, N = 0.02, 50


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
    from qec_ldpc_amd.gather import GatherPipeline
    code = q.Quantum_LDPC_Code.createFromFile(path)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dec = q.DecoderGPU(code, 0)
    m = T // world
    syn = []
    for k in range(K):  # step k: samples [k T + rank m, k T + (rank + 1) m)
        sX = torch.empty((m, code.numEqsX), dtype=torch.uint8, device=dev)
        sZ = torch.empty((m, code.numEqsZ), dtype=torch.uint8, device=dev)
        dec.sample_syndrome_dev(0x51EC0DE, k * T + rank * m, P, sX, sZ)
        syn.append((sX, sZ))
    torch.cuda.synchronize()
    pipe = GatherPipeline((m, dec.record_bytes()), dev)
    got = {}

    def decode(k, rec, stream):
        dec.decode_batch_packed_dev(syn[k][0], syn[k][1], P, N, "fixed", rec, stream=stream)

    pipe.run(decode, K, sink=lambda k, o: got.__setitem__(k, o.clone()))
    if rank == 0:
        assert sorted(got) == list(range(K)), sorted(got)
        np.save(out, torch.stack([got[k].cpu() for k in range(K)]).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_gather_equals_one_process(tmp_path, code_paths):
    import qec_ldpc_amd as q
    out = str(tmp_path / "rec.npy")
    mp.start_processes(_rank, args=(2, _free_port(), code_paths["P61"], out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    code = q.Quantum_LDPC_Code.createFromFile(code_paths["P61"])
    dec = q.DecoderGPU(code, 0)
    dev = torch.device("cuda", 0)
    assert got.shape == (K, T, dec.record_bytes())
    sX = torch.empty((K * T, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((K * T, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_syndrome_dev(0x51EC0DE, 0, P, sX, sZ)
    rec = torch.empty((K * T, dec.record_bytes()), dtype=torch.uint8, device=dev)
    dec.decode_batch_packed_dev(sX, sZ, P, N, "fixed", rec)
    torch.cuda.synchronize()
    want = rec.cpu().numpy().reshape(K, T, -1)
    for k in range(K):
        assert np.array_equal(got[k], want[k]), "step %d" % k
    # the steps differ (so a stale buffer could not pass)
    assert not np.array_equal(want[0], want[1])
