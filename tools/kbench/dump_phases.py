"""Per-syndrome phase counts (QEC_OPT_PHASE_STATS) and syndrome weights of a bench workload, saved
for offline analysis of dispatch orders (which grouping of syndromes into waves wastes the fewest
wave-iterations).  python tools/kbench/dump_phases.py --code p7 --batch 65536 --out f.npz"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import qec_ldpc_amd as q  # noqa: E402
from qec_ldpc_amd.codes import P7, P61, code_path  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--code", default="p7")
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--out", required=True)
a = ap.parse_args()
name, p, iters = {"p7": (P7, 0.02, 20), "p61": (P61, 0.01, 50)}[a.code]
code = q.Quantum_LDPC_Code.createFromFile(code_path(name))
dev = torch.device("cuda", 0)
dec = q.DecoderGPU(code, 0, max_batch=a.batch)
B = a.batch
sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
dec.sample_syndrome_dev(0x51EC0DE, 0, p, sX, sZ)
rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
its = torch.empty((B, 2), dtype=torch.int32, device=dev)
dec.set_option("phase_stats", 1)
dec.decode_batch_packed_dev(sX, sZ, p, iters, "fixed", rec, its)
torch.cuda.synchronize()
ph = its.cpu().numpy()
np.savez_compressed(a.out, phases=ph, wX=sX.sum(1).cpu().numpy(), wZ=sZ.sum(1).cpu().numpy(),
                    sX=sX.cpu().numpy(), sZ=sZ.cpu().numpy())
print("saved", a.out, ph.shape)
