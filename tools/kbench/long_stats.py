"""Which syndromes never harden (run every iteration soft), and how early would candidate
dispatch keys start them?  Uses a -DQEC_PHASE_STATS=1 build (iters[] = per-phase counts).
  python tools/kbench/long_stats.py --code p61 stats
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
    ap.add_argument("--reps", type=int, default=4, help="batches of --batch (different seeds)")
    ap.add_argument("--p", type=float, default=None)
    ap.add_argument("stats")
    a = ap.parse_args()
    name, p, iters = CODES[a.code]
    p = a.p if a.p is not None else p
    dev = torch.device("cuda", 0)
    L = bind(os.path.join(ROOT, "build", "variants", a.stats, "libqecldpc.so"))
    ch = L.qec_code_load(code_path(name).encode())
    d = L.qec_decoder_create(ch, 0, 0)
    prm = np.zeros(9, np.int32)
    L.qec_code_params(ch, prm.ctypes.data)
    n, mX, mZ = int(prm[6]), int(prm[7]), int(prm[8])
    B = a.batch
    st = torch.cuda.current_stream(dev)
    rows = []
    for rep in range(a.reps):
        x, z = depolarizing_errors(n, rep * B, B, p)
        sx = np.empty((B, mX), np.uint8)
        sz = np.empty((B, mZ), np.uint8)
        L.qec_code_syndrome(ch, 0, x.ctypes.data, B, sx.ctypes.data)
        L.qec_code_syndrome(ch, 1, z.ctypes.data, B, sz.ctypes.data)
        o = [torch.empty((B, n), dtype=torch.uint8, device=dev), torch.empty((B, n), dtype=torch.uint8, device=dev),
             torch.empty(B, dtype=torch.uint8, device=dev), torch.empty((B, 2), dtype=torch.int32, device=dev)]
        sX, sZ = torch.from_numpy(sx).to(dev), torch.from_numpy(sz).to(dev)
        rc = L.qec_decode_batch_dev(d, sX.data_ptr(), sZ.data_ptr(), B, p, iters, 1, o[0].data_ptr(),
                                    o[1].data_ptr(), o[2].data_ptr(), o[3].data_ptr(), None, st.cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        w = o[3].cpu().numpy().astype(np.int64)
        softX, softZ = w[:, 0] & 255, w[:, 1] & 255
        wX, wZ = sx.sum(1, dtype=np.int64), sz.sum(1, dtype=np.int64)
        ex, ez = x.sum(1, dtype=np.int64), z.sum(1, dtype=np.int64)
        rows.append((wX, wZ, softX, softZ, ex, ez))
    wX, wZ, softX, softZ, ex, ez = (np.concatenate([r[k] for r in rows]) for k in range(6))
    longX, longZ = softX >= iters, softZ >= iters
    N = len(wX)
    print("batch %d x %d, long X %d, long Z %d, both %d" % (a.reps, B, longX.sum(), longZ.sum(), (longX & longZ).sum()))

    def pr(v):
        return np.argsort(np.argsort(v, kind="stable"), kind="stable") / (len(v) - 1.0)  # percentile rank

    keys = {
        "wX+wZ": wX + wZ,
        "max(wX,wZ)": np.maximum(wX, wZ),
        "max(prX,prZ)": np.maximum(pr(wX), pr(wZ)),
        "wX": wX, "wZ": wZ,
    }
    out = {"N": N, "long_x": int(longX.sum()), "long_z": int(longZ.sum()), "keys": {}}
    for k, v in keys.items():
        ahead = [(v > v[i]).mean() for i in np.nonzero(longX | longZ)[0]]  # fraction dispatched before it
        out["keys"][k] = {"mean_ahead": float(np.mean(ahead)), "max_ahead": float(np.max(ahead)),
                          "ahead": sorted(round(float(t), 3) for t in ahead)}
        print("%-14s long ones start after %.3f of the batch on average (worst %.3f)" % (k, np.mean(ahead), np.max(ahead)))
    for i in np.nonzero(longX | longZ)[0]:
        print("long %s%s  wX=%3d (pr %.2f) wZ=%3d (pr %.2f)  errX=%d errZ=%d  softX=%d softZ=%d"
              % ("X" if longX[i] else "-", "Z" if longZ[i] else "-", wX[i], pr(wX)[i], wZ[i], pr(wZ)[i], ex[i], ez[i],
                 softX[i], softZ[i]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
