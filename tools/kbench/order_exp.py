"""How much of a fixed-iteration launch is the tail of long-running syndromes?
Times one production build on the same batch in several orders, using an
-DQEC_PHASE_STATS=1 build to learn each syndrome's soft-iteration count:
  original | longest first | longest last | long ones replaced by the all-zero syndrome
  python tools/kbench/order_exp.py --code p61 cur stats
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
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("prod")
    ap.add_argument("stats")
    a = ap.parse_args()
    name, p, iters = CODES[a.code]
    p = a.p if a.p is not None else p
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    libs = {}
    for v in (a.prod, a.stats):
        L = bind(os.path.join(ROOT, "build", "variants", v, "libqecldpc.so"))
        c = L.qec_code_load(code_path(name).encode())
        libs[v] = (L, c, L.qec_decoder_create(c, 0, 0))
    L, ch, _ = libs[a.prod]
    prm = np.zeros(9, np.int32)
    L.qec_code_params(ch, prm.ctypes.data)
    n, mX, mZ = int(prm[6]), int(prm[7]), int(prm[8])
    B = a.batch
    x, z = depolarizing_errors(n, 0, B, p)
    sx = np.empty((B, mX), np.uint8)
    sz = np.empty((B, mZ), np.uint8)
    L.qec_code_syndrome(ch, 0, x.ctypes.data, B, sx.ctypes.data)
    L.qec_code_syndrome(ch, 1, z.ctypes.data, B, sz.ctypes.data)
    o = [torch.empty((B, n), dtype=torch.uint8, device=dev), torch.empty((B, n), dtype=torch.uint8, device=dev),
         torch.empty(B, dtype=torch.uint8, device=dev), torch.empty((B, 2), dtype=torch.int32, device=dev)]

    def run(v, sX, sZ):
        Lb, _, d = libs[v]
        rc = Lb.qec_decode_batch_dev(d, sX.data_ptr(), sZ.data_ptr(), B, p, iters, 1, o[0].data_ptr(),
                                     o[1].data_ptr(), o[2].data_ptr(), o[3].data_ptr(), None, st.cuda_stream)
        assert rc == 0, Lb.qec_last_error()

    sX0, sZ0 = torch.from_numpy(sx).to(dev), torch.from_numpy(sz).to(dev)
    run(a.stats, sX0, sZ0)
    torch.cuda.synchronize()
    w = o[3].cpu().numpy().astype(np.int64)
    soft = (w[:, 0] & 255) + (w[:, 1] & 255)
    long_ = soft >= iters  # at least one sector never hard
    orders = {
        "original": np.arange(B),
        "longest_first": np.argsort(-soft, kind="stable"),
        "longest_last": np.argsort(soft, kind="stable"),
        # a predictor available before decoding: syndrome weight, heaviest first
        "weight_first": np.argsort(-(sx.sum(1, dtype=np.int64) + sz.sum(1, dtype=np.int64)), kind="stable"),
    }
    wt = sx.sum(1, dtype=np.int64) + sz.sum(1, dtype=np.int64)
    for q in (50, 90, 99, 99.9):
        print("weight p%s = %d" % (q, np.percentile(wt, q)))
    print("long syndromes' weights:", sorted(wt[long_].tolist())[:40])
    print("corr(weight, soft) = %.3f" % np.corrcoef(wt, soft)[0, 1])
    res = {}
    for k, idx in orders.items():
        sX, sZ = sX0[torch.from_numpy(idx).to(dev)].contiguous(), sZ0[torch.from_numpy(idx).to(dev)].contiguous()
        res[k] = time_it(run, a.prod, sX, sZ, a.reps)
    sxz, szz = sx.copy(), sz.copy()
    sxz[long_] = 0
    szz[long_] = 0
    res["long_zeroed"] = time_it(run, a.prod, torch.from_numpy(sxz).to(dev), torch.from_numpy(szz).to(dev), a.reps)
    for k, ms in res.items():
        print("%-14s %8.4f ms  %12.0f syn/s" % (k, ms, B / ms * 1e3))
    print(json.dumps({"code": a.code, "p": p, "batch": B, "n_long": int(long_.sum()),
                      "soft_mean": float(soft.mean()), "ms": res}))


def time_it(run, v, sX, sZ, reps):
    run(v, sX, sZ)
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(v, sX, sZ)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return round(float(np.median(ms)), 4)


if __name__ == "__main__":
    main()
