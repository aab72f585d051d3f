"""Var-pass path statistics of an experiment build (-DQEC_PATH_STATS=1, P61 fixed-stop kernel):
per syndrome, the columns that took the agreement (same), zero, short-division and full-division
paths, on soft and on hard sector inputs.
  python tools/kbench/path_stats.py VARIANT [--batch B] [--p P ...]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from compare import bind  # noqa: E402
from qec_ldpc_amd.codes import P61, code_path  # noqa: E402
from qec_ldpc_amd.synthetic import depolarizing_errors  # noqa: E402

NAMES = ["same", "zero", "short", "full"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--p", type=float, nargs="+", default=[0.01, 0.05])
    ap.add_argument("--stop", type=int, default=1)
    a = ap.parse_args()
    L = bind(os.path.join(ROOT, "build", "variants", a.variant, "libqecldpc.so"))
    L.qec_debug_path_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    c = L.qec_code_load(code_path(P61).encode())
    prm = np.zeros(9, np.int32)
    L.qec_code_params(c, prm.ctypes.data)
    n, mX, mZ = int(prm[6]), int(prm[7]), int(prm[8])
    d = L.qec_decoder_create(c, 0, 0)
    B = a.batch
    st = np.zeros(24, np.uint64)
    for p in a.p:
        x, z = depolarizing_errors(n, 0, B, p)
        sx = np.empty((B, mX), np.uint8)
        sz = np.empty((B, mZ), np.uint8)
        L.qec_code_syndrome(c, 0, x.ctypes.data, B, sx.ctypes.data)
        L.qec_code_syndrome(c, 1, z.ctypes.data, B, sz.ctypes.data)
        sX, sZ = torch.from_numpy(sx).to(dev), torch.from_numpy(sz).to(dev)
        o = [torch.empty((B, n), dtype=torch.uint8, device=dev), torch.empty((B, n), dtype=torch.uint8, device=dev),
             torch.empty(B, dtype=torch.uint8, device=dev), torch.empty((B, 2), dtype=torch.int32, device=dev)]
        L.qec_debug_path_stats(st.ctypes.data, 1)
        rc = L.qec_decode_batch_dev(d, sX.data_ptr(), sZ.data_ptr(), B, p, 50, a.stop, o[0].data_ptr(),
                                    o[1].data_ptr(), o[2].data_ptr(), o[3].data_ptr(), None,
                                    torch.cuda.current_stream(dev).cuda_stream)
        assert rc == 0, L.qec_last_error()
        torch.cuda.synchronize()
        L.qec_debug_path_stats(st.ctypes.data, 1)
        print("p=%g stop=%d batch=%d: var-pass columns per syndrome" % (p, a.stop, B))
        for sec, sn in ((0, "X"), (1, "Z")):
            for h, hn in ((0, "soft in"), (4, "hard in")):
                row = {NAMES[k]: round(float(st[sec * 8 + h + k]) / B, 3) for k in range(4)}
                print("  %s %-8s %s" % (sn, hn, row))
            g = {k: round(float(st[16 + sec * 4 + i]) / B, 3) for i, k in enumerate(["all n big", "zeros only", "tiny n", "small d"])}
            print("  %s soft-column guard anatomy %s" % (sn, g))


if __name__ == "__main__":
    main()
