"""The RCCL code paths of the multi-GPU entry points, executed once on the GPU box before the
driver's 8-GPU run does: torch.distributed's "nccl" backend (RCCL on ROCm) at world size 1 (RCCL
allows one rank per GPU, and the box has one).  In a child process, so the process group never
outlives the test:

* gather_records' RCCL branch: a real dist.gather of device-resident decision records into the
  root's output (qec_ldpc_amd/gather.py), byte-equal to what was decoded; and the overlapped
  decode + gather pipeline (GatherPipeline) over three steps, every gathered step byte-equal;
* tools/psweep.py's counter reduction: the all-reduce (sum) of the counter vector and the
  all-reduce (max) of the timings on device tensors, on a real Monte-Carlo run's counters.

The reference's parallel axis is the sample loop of QEC_LDPC/DecoderCPU.h:419-438; the shards and
their gather are SURVEY.md 8(e).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["QEC_ROOT"])
sys.path.insert(0, os.path.join(os.environ["QEC_ROOT"], "tools"))
import torch
import torch.distributed as dist
import qec_ldpc_amd as q
from qec_ldpc_amd.codes import P61, code_path
from qec_ldpc_amd.gather import gather_records
import psweep

dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%s" % os.environ["QEC_PORT"], rank=0, world_size=1)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
code = q.Quantum_LDPC_Code.createFromFile(code_path(P61))
dec = q.DecoderGPU(code, 0)
B = 4096
sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
dec.sample_syndrome_dev(0x51EC0DE, 0, 0.01, sX, sZ, stream=st)
rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
its = torch.empty((B, 2), dtype=torch.int32, device=dev)
dec.decode_batch_packed_dev(sX, sZ, 0.01, 50, "fixed", rec, its, stream=st)
full = gather_records(rec)
torch.cuda.synchronize()
from qec_ldpc_amd.gather import GatherPipeline
pipe = GatherPipeline(tuple(rec.shape), dev)
piped = []
pipe.run(lambda k, r, s: dec.decode_batch_packed_dev(sX, sZ, 0.01, 50, "fixed", r, its, stream=s), 3,
         sink=lambda k, o: piped.append(o.clone()))
r = dec.monte_carlo(0x51EC0DE, 0, 8192, 0.01, 50, "syndrome", 8192)
c, tm = psweep.reduce_counters(r, [0.5, 0.25, 0.1, 0.9, 0.0], "nccl", dev)
out = {"backend": dist.get_backend(), "world": dist.get_world_size(),
       "gather_device": str(full.device), "gather_equal": bool(full is not rec and torch.equal(full, rec)),
       "gather_shape": list(full.shape),
       "pipeline_equal": len(piped) == 3 and all(torch.equal(x, rec) for x in piped),
       "pipeline_device": str(pipe.outs[0].device),
       "counters_equal": all(c[k] == r[k] for k in psweep.FIELDS), "tested": c["tested"], "times": tm}
dist.barrier()
dist.destroy_process_group()
print(json.dumps(out), flush=True)
"""


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_gather_and_counter_reduce_world1():
    env = dict(os.environ, QEC_ROOT=ROOT, QEC_PORT=str(free_port()), MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, "rc=%d\n%s\n%s" % (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["gather_equal"] and out["gather_device"] == "cuda:0" and out["gather_shape"][0] == 4096
    assert out["pipeline_equal"] and out["pipeline_device"] == "cuda:0"
    assert out["counters_equal"] and out["tested"] == 8192
    assert out["times"] == [0.5, 0.25, 0.1, 0.9, 0.0]


def test_bench_gather_world1():
    """bench.py --gather-world1: the gather measurements (alone, serialised, overlapped) in an RCCL group of
    one, the source of DESIGN.md section 9's world-1 rate; both record checks hold."""
    r = subprocess.run([sys.executable, "bench.py", "--gather-world1", "--no-extras", "--no-cpu",
                        "--global-batch", "65536", "--steps", "5"], cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, "rc=%d\n%s\n%s" % (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    g = out["gather"]
    assert "error" not in g, g
    assert g["backend"] == "nccl" and g["world_size"] == 1 and g["bytes_per_rank"] == 65536 * 155
    assert g["rank0_shard_intact"] and g["end_to_end_overlapped"]["rank0_last_step_intact"]
    assert g["gather_ms"] > 0 and g["end_to_end_overlapped"]["ms_per_step"] > 0
