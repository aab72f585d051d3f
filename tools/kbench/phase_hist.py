"""Where the iterations of a decode go, through the product library's instrumented kernels
(QEC_OPT_PHASE_STATS: iters[] holds per sector soft | hard << 8 | agreed << 16 | jumped << 24).
  python tools/kbench/phase_hist.py --p 0.1 --stop syndrome --stop fixed
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import qec_ldpc_amd as q  # noqa: E402
from qec_ldpc_amd.codes import P61, code_path  # noqa: E402
from qec_ldpc_amd.synthetic import depolarizing_errors  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--p", type=float, nargs="+", default=[0.1])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--stop", action="append", default=None)
    a = ap.parse_args()
    code = q.Quantum_LDPC_Code.createFromFile(code_path(P61))
    dec = q.DecoderGPU(code, 0)
    for p in a.p:
        x, z = depolarizing_errors(code.n, 0, a.batch, p)
        sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
        for stop in a.stop or ["syndrome", "fixed"]:
            dec.set_option("phase_stats", 1)
            v = dec.decode_batch(sX, sZ, p, a.iters, stop, want_iters=True)[3].astype(np.int64)
            dec.set_option("phase_stats", 0)
            out = {"p": p, "stop": stop, "batch": a.batch}
            for s, sec in enumerate("XZ"):
                w = v[:, s]
                ph = {"soft": w & 255, "hard": (w >> 8) & 255, "agreed": (w >> 16) & 255, "jumped": (w >> 24) & 255}
                o = {k: round(float(arr.mean()), 3) for k, arr in ph.items()}
                o["never_hard"] = int(np.sum(ph["hard"] + ph["agreed"] + ph["jumped"] == 0))
                o["soft_ge_40"] = int(np.sum(ph["soft"] >= 40))
                o["hard_hist"] = {str(i): int(c) for i, c in enumerate(np.bincount(ph["hard"], minlength=a.iters + 1)) if c}
                o["soft_hist10"] = np.bincount(ph["soft"] // 10, minlength=6).tolist()
                out[sec] = o
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
