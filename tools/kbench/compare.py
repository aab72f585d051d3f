"""Time several builds of libqecldpc.so (build/variants/<name>/) on the same resident
batch in one process, interleaved, and check that every variant's outputs are
bit-identical to the first one's.  Usage:
  python tools/kbench/compare.py --code p61 --reps 5 v0 v1 ...
  python tools/kbench/compare.py --mc --stop 2 --p 0.002 --batch 1048576 v0 v1 ...   (qec_monte_carlo runs)
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from qec_ldpc_amd.codes import P7, P61, code_path  # noqa: E402
from qec_ldpc_amd.synthetic import depolarizing_errors  # noqa: E402

CODES = {"p61": (P61, 0.01, 50), "p7": (P7, 0.02, 20)}
OPTIONS = {"hard_paths": 1, "cycle_jump": 2, "schedule": 3, "sector_split": 4, "phase_stats": 5, "triage": 6,
           "mc_decode_time": 8}


def bind(path):
    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    vp = ctypes.c_void_p
    L.qec_code_load.restype = vp
    L.qec_code_load.argtypes = [ctypes.c_char_p]
    L.qec_decoder_create.restype = vp
    L.qec_decoder_create.argtypes = [vp, ctypes.c_int, ctypes.c_size_t]
    L.qec_decode_batch_dev.restype = ctypes.c_int
    L.qec_decode_batch_dev.argtypes = [vp, vp, vp, ctypes.c_size_t, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                       vp, vp, vp, vp, vp, vp]
    L.qec_code_syndrome.argtypes = [vp, ctypes.c_int, vp, ctypes.c_size_t, vp]
    L.qec_code_params.argtypes = [vp, vp]
    L.qec_decoder_describe.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
    L.qec_last_error.restype = ctypes.c_char_p
    L.qec_decoder_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    from qec_ldpc_amd import MCResult
    L.qec_monte_carlo.restype = ctypes.c_int
    L.qec_monte_carlo.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_float, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(MCResult)]
    return L


def mc_main(a, name, p, iters):
    """--mc: whole qec_monte_carlo runs (the psweep step) of every variant, interleaved; counters must
    be identical; wall time of the call and its decode-kernel time."""
    import time
    from qec_ldpc_amd import MCResult
    opts = {v: [kv.split("=") for kv in v.split(":", 1)[1].split(",")] if ":" in v else [] for v in a.variants}
    runs = {}
    for v in a.variants:
        L = bind(os.path.join(ROOT, "build", "variants", v.split(":")[0], "libqecldpc.so"))
        c = L.qec_code_load(code_path(name).encode())
        d = L.qec_decoder_create(c, 0, 0)
        for k, val in opts[v]:
            assert L.qec_decoder_set_option(d, OPTIONS[k], int(val)) == 0, L.qec_last_error()
        runs[v] = (L, d)
    res = {v: [] for v in a.variants}
    cnt = {}
    for rep in range(a.reps + 1):
        for v, (L, d) in runs.items():
            r = MCResult()
            t = time.perf_counter()
            rc = L.qec_monte_carlo(d, 0x51EC0DE, 0, a.batch, p, iters, a.stop, a.batch, ctypes.byref(r))
            dt = time.perf_counter() - t
            assert rc == 0, L.qec_last_error()
            c = r.as_dict()
            key = tuple(c[k] for k in ("tested", "withX", "withZ", "synX", "synZ", "logical", "corrected", "convX",
                                       "convZ", "iterationsX", "iterationsZ"))
            cnt.setdefault(v, key)
            assert cnt[v] == key
            if rep:
                res[v].append((dt, c["decodeSeconds"]))
    ref = cnt[a.variants[0]]
    for v in a.variants:
        ms = float(np.median([x[0] for x in res[v]])) * 1e3
        dms = float(np.median([x[1] for x in res[v]])) * 1e3
        print("%-22s %9.3f ms  %12.0f syn/s  decode %.3f ms  identical=%s" % (v, ms, a.batch / ms * 1e3, dms, cnt[v] == ref))
        print(json.dumps({"variant": v, "counters": dict(zip(("tested", "withX", "withZ", "synX", "synZ", "logical",
                                                               "corrected", "convX", "convZ", "iterationsX",
                                                               "iterationsZ"), cnt[v]))}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="p61")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stop", type=int, default=1)
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--p", type=float, default=None, help="depolarising rate (default: the code's bench p)")
    ap.add_argument("--mc", action="store_true", help="whole Monte-Carlo runs (qec_monte_carlo, --batch samples)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    name, p, iters = CODES[a.code]
    if a.iters is not None:
        iters = a.iters
    if a.p is not None:
        p = a.p
    if a.mc:
        return mc_main(a, name, p, iters)
    dev = torch.device("cuda", 0)
    # a variant is "<build dir>" or "<build dir>:<option>=<value>,..." (decoder options, e.g.
    # cur:cycle_jump=0), so one build can be timed with several option settings
    opts = {v: [kv.split("=") for kv in v.split(":", 1)[1].split(",")] if ":" in v else [] for v in a.variants}
    libs = {v: bind(os.path.join(ROOT, "build", "variants", v.split(":")[0], "libqecldpc.so")) for v in a.variants}
    first = libs[a.variants[0]]
    ch = first.qec_code_load(code_path(name).encode())
    prm = np.zeros(9, np.int32)
    first.qec_code_params(ch, prm.ctypes.data)
    n, mX, mZ = int(prm[6]), int(prm[7]), int(prm[8])
    B = a.batch
    x, z = depolarizing_errors(n, 0, B, p)
    sx = np.empty((B, mX), np.uint8)
    sz = np.empty((B, mZ), np.uint8)
    first.qec_code_syndrome(ch, 0, x.ctypes.data, B, sx.ctypes.data)
    first.qec_code_syndrome(ch, 1, z.ctypes.data, B, sz.ctypes.data)
    sX = torch.from_numpy(sx).to(dev)
    sZ = torch.from_numpy(sz).to(dev)
    decs, outs = {}, {}
    for v, L in libs.items():
        c = L.qec_code_load(code_path(name).encode())
        d = L.qec_decoder_create(c, 0, 0)
        if not d:
            raise SystemExit("%s: %s" % (v, L.qec_last_error()))
        for k, val in opts[v]:
            assert L.qec_decoder_set_option(d, OPTIONS[k], int(val)) == 0, L.qec_last_error()
        buf = ctypes.create_string_buffer(256)
        L.qec_decoder_describe(d, buf, 256)
        decs[v] = (L, d, buf.value.decode())
        outs[v] = [torch.empty((B, n), dtype=torch.uint8, device=dev), torch.empty((B, n), dtype=torch.uint8, device=dev),
                   torch.empty(B, dtype=torch.uint8, device=dev), torch.empty((B, 2), dtype=torch.int32, device=dev)]
    st = torch.cuda.current_stream(dev)
    times = {v: [] for v in a.variants}

    def run(v):
        L, d, _ = decs[v]
        o = outs[v]
        rc = L.qec_decode_batch_dev(d, sX.data_ptr(), sZ.data_ptr(), B, p, iters, a.stop, o[0].data_ptr(),
                                    o[1].data_ptr(), o[2].data_ptr(), o[3].data_ptr(), None, st.cuda_stream)
        assert rc == 0, L.qec_last_error()

    for v in a.variants:
        run(v)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        for v in a.variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run(v)
            e1.record(st)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
    ref = [t.cpu().numpy() for t in outs[a.variants[0]]]
    res = {}
    for v in a.variants:
        same = all(np.array_equal(r, t.cpu().numpy()) for r, t in zip(ref, outs[v]))
        ms = float(np.median(times[v]))
        res[v] = {"ms": round(ms, 4), "min_ms": round(float(np.min(times[v])), 4), "syn_per_s": round(B / ms * 1e3),
                  "identical": same, "kernel": decs[v][2]}
        print("%-14s %9.3f ms  %12.0f syn/s  identical=%s  %s" % (v, ms, B / ms * 1e3, same, decs[v][2]))
    print(json.dumps({"code": a.code, "batch": B, "iters": iters, "stop": a.stop, "results": res}))


if __name__ == "__main__":
    main()
