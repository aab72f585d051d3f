"""Per-wave phase timing of the P61 decode from an experiment build compiled with
-DQEC_STAMPS=1 -DQEC_PHASE_STATS=1 (s_memtime stamps in the q_final buffer, soft-iteration
counts in iters[]).  Prints the average cycles per phase, the kernel span, wave
occupancy, and the cost per soft iteration (least squares over the batch).
  python tools/kbench/stamps.py --code p61 stamps_build"""
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

PHASES = ["table", "X it0", "X loop", "X post", "Z it0", "Z loop", "Z post", "end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="p61")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--p", type=float, default=None)
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--schedule", type=int, default=1)
    ap.add_argument("variant")
    a = ap.parse_args()
    name, p, iters = CODES[a.code]
    p = a.p if a.p is not None else p
    iters = a.iters if a.iters is not None else iters
    L = bind(os.path.join(ROOT, "build", "variants", a.variant, "libqecldpc.so"))
    ch = L.qec_code_load(code_path(name).encode())
    prm = np.zeros(9, np.int32)
    L.qec_code_params(ch, prm.ctypes.data)
    n, mX, mZ, Lc = int(prm[6]), int(prm[7]), int(prm[8]), int(prm[2])
    B = a.batch
    x, z = depolarizing_errors(n, 0, B, p)
    sx = np.empty((B, mX), np.uint8)
    sz = np.empty((B, mZ), np.uint8)
    L.qec_code_syndrome(ch, 0, x.ctypes.data, B, sx.ctypes.data)
    L.qec_code_syndrome(ch, 1, z.ctypes.data, B, sz.ctypes.data)
    dev = torch.device("cuda", 0)
    sX, sZ = torch.from_numpy(sx).to(dev), torch.from_numpy(sz).to(dev)
    d = L.qec_decoder_create(ch, 0, B)
    assert L.qec_decoder_set_option(d, 3, a.schedule) == 0
    o = [torch.empty((B, n), dtype=torch.uint8, device=dev), torch.empty((B, n), dtype=torch.uint8, device=dev),
         torch.empty(B, dtype=torch.uint8, device=dev), torch.empty((B, 2), dtype=torch.int32, device=dev)]
    q = torch.zeros((B, (mX + mZ) * Lc), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        rc = L.qec_decode_batch_dev(d, sX.data_ptr(), sZ.data_ptr(), B, p, iters, 1, o[0].data_ptr(), o[1].data_ptr(),
                                    o[2].data_ptr(), o[3].data_ptr(), q.data_ptr(), st)
        assert rc == 0, L.qec_last_error()
    torch.cuda.synchronize()
    nw = B  # G = 1, no sector split (P61)
    allst = q.view(torch.int64).cpu().numpy().reshape(-1)[: nw * 16].reshape(nw, 16).astype(np.float64)
    stamps = allst[:, :9]
    t0 = stamps[:, 0].min()
    span = stamps[:, 8].max() - t0
    dur = stamps[:, 8] - stamps[:, 0]
    ph = np.diff(stamps, axis=1)
    w = o[3].cpu().numpy().astype(np.int64)
    softX, softZ = w[:, 0] & 255, w[:, 1] & 255
    out = {"code": a.code, "p": p, "iters": iters, "schedule": a.schedule, "span_cycles": span,
           "mean_wave_cycles": float(dur.mean()), "sum_wave_cycles_over_span": float(dur.sum() / span),
           "phases_mean_cycles": {k: round(float(v), 1) for k, v in zip(PHASES, ph.mean(0))},
           "phases_share": {k: round(float(v), 4) for k, v in zip(PHASES, ph.sum(0) / dur.sum())}}
    for sec, soft, col in (("X", softX, 2), ("Z", softZ, 5)):
        A = np.stack([soft, np.ones_like(soft)], 1).astype(np.float64)
        coef, *_ = np.linalg.lstsq(A, ph[:, col], rcond=None)
        out["%s_loop_cycles_per_soft_iter" % sec] = round(float(coef[0]), 1)
        out["%s_loop_intercept_cycles" % sec] = round(float(coef[1]), 1)
    # soft part of each loop: from the loop's start to the first hard state (when it got hard)
    for sec, col, k in (("X", 2, 9), ("Z", 5, 10)):
        hard_at = allst[:, k]
        got = (hard_at >= stamps[:, col]) & (hard_at <= stamps[:, col + 1])
        out["%s_soft_part_cycles" % sec] = round(float((hard_at - stamps[:, col])[got].mean()), 1)
        out["%s_hard_part_cycles" % sec] = round(float((stamps[:, col + 1] - hard_at)[got].mean()), 1)
        out["%s_got_hard" % sec] = int(got.sum())
    start = stamps[:, 0] - t0
    out["start_quantiles"] = {str(qq): round(float(np.percentile(start, qq)) / span, 4) for qq in (0, 10, 50, 90, 99, 100)}
    end = stamps[:, 8] - t0
    out["end_quantiles"] = {str(qq): round(float(np.percentile(end, qq)) / span, 4) for qq in (50, 90, 99, 99.9, 100)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
