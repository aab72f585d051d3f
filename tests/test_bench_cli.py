"""bench.py's launcher contract on the CPU (no GPU is touched before these checks): a run whose
WORLD_SIZE disagrees with --gpus exits non-zero instead of printing a mislabelled line
(the reference's sample-parallel axis is QEC_LDPC/DecoderCPU.h:419-438)."""
import os
import subprocess
import sys

from conftest import ROOT


def bench(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=120)


def test_world_size_mismatch_refused():
    r = bench(["--gpus", "8", "--no-cpu"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr and not r.stdout.strip()


def test_launcher_world_smaller_than_gpus_refused():
    r = bench(["--gpus", "4", "--no-cpu"], {"WORLD_SIZE": "2", "RANK": "1"})
    assert r.returncode == 2 and "WORLD_SIZE 2" in r.stderr
