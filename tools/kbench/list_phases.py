"""Per-phase cycles of the list-mode decode from a build of a temporarily stamped copy of bp_decode.hip
(s_memtime around the phases of each listed sector; not part of the product).  Per wave row of
qec_debug_read_stamps: [0] iteration 0 (+ syndrome loads), [1] later iterations, [2] post-processing,
[3] decision output, [4] sectors, [5] later iterations executed, [6] whole sector incl. list entry and
merge / iteration stores, [7] waves.
  python tools/kbench/list_phases.py --p 0.005 VARIANT"""
import argparse
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from compare import ROOT, bind  # noqa: E402

sys.path.insert(0, ROOT)
from qec_ldpc_amd import MCResult  # noqa: E402
from qec_ldpc_amd.codes import P61, code_path  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=float, nargs="+", default=[0.005])
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("variant")
    a = ap.parse_args()
    L = bind(os.path.join(ROOT, "build", "variants", a.variant, "libqecldpc.so"))
    L.qec_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    c = L.qec_code_load(code_path(P61).encode())
    d = L.qec_decoder_create(c, 0, 0)
    buf = np.zeros(8192 * 8, np.uint64)
    for p in a.p:
        r = MCResult()
        assert L.qec_monte_carlo(d, 0x51EC0DE, 0, a.batch, p, 50, 2, a.batch, ctypes.byref(r)) == 0
        L.qec_debug_read_stamps(buf.ctypes.data, 1)
        assert L.qec_monte_carlo(d, 0x51EC0DE, 0, a.batch, p, 50, 2, a.batch, ctypes.byref(r)) == 0
        L.qec_debug_read_stamps(buf.ctypes.data, 1)
        v = buf.reshape(8192, 8).astype(np.float64)
        waves = v[:, 7] > 0
        tot = v[waves].sum(0)
        n = tot[4]
        per = {k: round(tot[i] / n) for i, k in enumerate(["iter0", "later_iters", "post", "emit"])}
        per["per_later_iter"] = round(tot[1] / max(tot[5], 1))
        per["sector_total"] = round(tot[6] / n)
        print("p", p, "sectors", int(n), "later iters/sector", round(tot[5] / n, 3), "cycles/sector", per,
              "waves", int(waves.sum()), "decode_s", r.decodeSeconds,
              "wave busy cycles max/mean", round(v[waves, 6].max()), round(v[waves, 6].mean()))
        busy = v[:4096, 6]
        print("   busy percentiles 10/50/90/99/max", [round(np.percentile(busy, q)) for q in (10, 50, 90, 99, 100)])
        print("   mean busy by XCD (wave % 8)", [round(busy[k::8].mean()) for k in range(8)])
        print("   sectors per wave min/max", int(v[:4096, 4].min()), int(v[:4096, 4].max()),
              "busy per sector by XCD", [round(busy[k::8].sum() / v[:4096, 4][k::8].sum()) for k in range(8)])
        print("   mean busy by wave // 1024 (launch order quarter)", [round(busy[k * 1024:(k + 1) * 1024].mean()) for k in range(4)])


if __name__ == "__main__":
    main()
