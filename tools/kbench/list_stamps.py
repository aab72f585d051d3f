"""Per-phase cycle spans of the syndrome-stop sectors (list-mode decode of the Monte-Carlo pipeline),
from an experiment build compiled with -DQEC_LIST_STAMPS=1 (tools/kbench/build_variants.sh
stamps:-DQEC_LIST_STAMPS=1): iteration 0 (syndrome loads, table iteration), the remaining iterations
(per iteration), the post-processing, the decision output, per sector X / Z.
  python tools/kbench/list_stamps.py --p 0.005 stamps"""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from compare import CODES, ROOT, bind  # noqa: E402

sys.path.insert(0, ROOT)
from qec_ldpc_amd import MCResult  # noqa: E402
from qec_ldpc_amd.codes import code_path  # noqa: E402

PHASES = ["iteration 0 (+ loads)", "iterations 1.. (per iteration)", "post-processing", "decision output"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="p61")
    ap.add_argument("--p", type=float, default=0.005)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("variant")
    a = ap.parse_args()
    name, _, iters = CODES[a.code]
    L = bind(os.path.join(ROOT, "build", "variants", a.variant, "libqecldpc.so"))
    L.qec_debug_list_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    c = L.qec_code_load(code_path(name).encode())
    d = L.qec_decoder_create(c, 0, 0)
    buf = (ctypes.c_ulonglong * 16)()
    r = MCResult()
    assert L.qec_monte_carlo(d, 0x51EC0DE, 0, a.batch, a.p, iters, 2, a.batch, ctypes.byref(r)) == 0
    L.qec_debug_list_stamps(buf, 1)
    t0 = r.decodeSeconds
    assert L.qec_monte_carlo(d, 0x51EC0DE, 0, a.batch, a.p, iters, 2, a.batch, ctypes.byref(r)) == 0
    L.qec_debug_list_stamps(buf, 0)
    v = list(buf)
    print("p=%g batch %d decode %.3f ms (warm-up %.3f ms)" % (a.p, a.batch, r.decodeSeconds * 1e3, t0 * 1e3))
    for sec in range(2):
        cnt = v[8 + 4 * sec]
        print("sector %s: %d sectors" % ("XZ"[sec], cnt))
        for k, ph in enumerate(PHASES):
            tot, n = v[4 * sec + k], v[8 + 4 * sec + k]
            per = tot / max(n, 1)
            print("  %-32s %10.0f cycles per %s  (count %d, total %.3g)" % (ph, per, "iteration" if k == 1 else "sector", n, tot))


if __name__ == "__main__":
    main()
