"""The multi-GPU entry points under the launcher the driver uses (python -m torch.distributed.run,
one process per rank), rehearsed with two gloo ranks sharing GPU 0 (RCCL needs one GPU per rank).

bench.py: the JSON line reports both ranks, the global batch, the backend actually used and the
world size it saw, and rank 0's shard of the gathered records equals what it decoded.
tools/psweep.py: the counters summed over two ranks equal one rank's counters over the same
samples (the sample index space is sharded, so the totals do not depend on the rank count;
QEC_LDPC/DecoderCPU.h:419-438 is the reference's sample-parallel loop).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(cmd, env_extra, timeout=300):
    env = dict(os.environ, QEC_BENCH_BACKEND="gloo", **env_extra)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, "rc=%d\n%s\n%s" % (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


def launch(nproc, script, *args):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script, *args]


def test_bench_two_ranks():
    lines = run(launch(2, "bench.py", "--gpus", "2", "--global-batch", "16384", "--no-cpu", "--steps", "3",
                       "--warmup", "1", "--min-seconds", "0.05"), {})
    assert len(lines) == 1, lines
    b = lines[0]
    assert b["n_gpus"] == 2 and b["config"]["global_batch"] == 16384 and b["config"]["per_gpu_batch"] == 8192
    assert b["config"]["parallelism"] == "dp2" and b["value"] > 0 and b["steps"] == 3
    g = b["gather"]
    assert "error" not in g, g
    assert g["backend"] == "gloo" and g["backend_reported"] == "gloo" and g["world_size"] == 2
    assert g["rank0_shard_intact"] is True
    assert "gloo gather" in g["end_to_end"]["what"]
    o = g["end_to_end_overlapped"]
    assert o["rank0_last_step_intact"] is True and o["syndromes_per_s"] > 0
    assert o["gather_bytes_per_step"] == 16384 * g["record_bytes"]
    assert b["full_arithmetic"]["identical"] is True and b["ref_stop"]["syndromes_per_s"] > 0
    assert 0 < b["executed_iteration_fraction"] <= 1


def test_bench_plain_python_two_gpus():
    """`python bench.py --gpus 2` with no launcher starts the two ranks itself (a child
    torch.distributed.run) and reports them: never a one-GPU line labelled --gpus 2."""
    lines = run([sys.executable, "bench.py", "--gpus", "2", "--global-batch", "16384", "--no-cpu", "--no-extras",
                 "--steps", "3", "--warmup", "1"], {})
    assert len(lines) == 1, lines
    b = lines[0]
    assert b["n_gpus"] == 2 and b["config"]["parallelism"] == "dp2" and b["config"]["per_gpu_batch"] == 8192
    g = b["gather"]
    assert "error" not in g, g
    assert g["world_size"] == 2 and g["rank0_shard_intact"] is True


def test_psweep_two_ranks_equal_one():
    args = ["--total", "16384", "--ps", "0.01", "0.05", "--reps", "1", "--batch", "8192"]
    two = run(launch(2, "tools/psweep.py", *args), {})
    one = run([sys.executable, "tools/psweep.py", *args], {})
    per2 = [x for x in two if "p" in x]
    per1 = [x for x in one if "p" in x]
    assert [x["p"] for x in per2] == [0.01, 0.05] == [x["p"] for x in per1]
    for a, b in zip(per1, per2):
        assert b["n_gpus"] == 2 and a["n_gpus"] == 1 and b.get("backend") == "gloo"
        assert a["counters"] == b["counters"], (a["p"], a["counters"], b["counters"])
        assert a["counters"]["tested"] == 16384
