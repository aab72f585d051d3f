"""Where the iterations of a fixed-iteration decode go: run an experiment build compiled
with -DQEC_PHASE_STATS=1 (iters[] then holds, per sector, soft | hard << 8 |
agreed << 16 | jumped << 24) and print per-sector phase statistics.
  python tools/kbench/phase_stats.py --code p61 --p 0.01 stats_build
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from compare import CODES, ROOT, bind  # noqa: E402

sys.path.insert(0, ROOT)
from qec_ldpc_amd.codes import code_path  # noqa: E402
from qec_ldpc_amd.synthetic import depolarizing_errors  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="p61")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--p", type=float, default=None)
    ap.add_argument("--stop", type=int, default=1)
    ap.add_argument("variant")
    a = ap.parse_args()
    name, p, iters = CODES[a.code]
    p = a.p if a.p is not None else p
    L = bind(os.path.join(ROOT, "build", "variants", a.variant, "libqecldpc.so"))
    ch = L.qec_code_load(code_path(name).encode())
    prm = np.zeros(9, np.int32)
    L.qec_code_params(ch, prm.ctypes.data)
    n, mX, mZ = int(prm[6]), int(prm[7]), int(prm[8])
    B = a.batch
    x, z = depolarizing_errors(n, 0, B, p)
    sx = np.empty((B, mX), np.uint8)
    sz = np.empty((B, mZ), np.uint8)
    L.qec_code_syndrome(ch, 0, x.ctypes.data, B, sx.ctypes.data)
    L.qec_code_syndrome(ch, 1, z.ctypes.data, B, sz.ctypes.data)
    dev = torch.device("cuda", 0)
    sX, sZ = torch.from_numpy(sx).to(dev), torch.from_numpy(sz).to(dev)
    d = L.qec_decoder_create(ch, 0, 0)
    o = [torch.empty((B, n), dtype=torch.uint8, device=dev), torch.empty((B, n), dtype=torch.uint8, device=dev),
         torch.empty(B, dtype=torch.uint8, device=dev), torch.empty((B, 2), dtype=torch.int32, device=dev)]
    rc = L.qec_decode_batch_dev(d, sX.data_ptr(), sZ.data_ptr(), B, p, iters, a.stop, o[0].data_ptr(), o[1].data_ptr(),
                                o[2].data_ptr(), o[3].data_ptr(), None, torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0, L.qec_last_error()
    torch.cuda.synchronize()
    v = o[3].cpu().numpy().astype(np.int64)
    out = {"code": a.code, "p": p, "iters": iters, "batch": B}
    for s, sec in enumerate("XZ"):
        w = v[:, s]
        ph = {"soft": w & 255, "hard": (w >> 8) & 255, "agreed": (w >> 16) & 255, "jumped": (w >> 24) & 255}
        sec_out = {}
        for k, arr in ph.items():
            hist = np.bincount(arr, minlength=iters + 1)
            sec_out[k] = {"mean": round(float(arr.mean()), 3), "max": int(arr.max()),
                          "hist": {str(i): int(c) for i, c in enumerate(hist) if c}}
        sec_out["never_hard"] = int(np.sum(ph["soft"] == iters))
        out[sec] = sec_out
        print("%s: soft mean %.2f (never hard %d)  hard %.2f  agreed %.2f  jumped %.2f" % (
            sec, sec_out["soft"]["mean"], sec_out["never_hard"], sec_out["hard"]["mean"], sec_out["agreed"]["mean"],
            sec_out["jumped"]["mean"]))
        print("   soft hist", sec_out["soft"]["hist"])
        print("   hard hist", sec_out["hard"]["hist"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
