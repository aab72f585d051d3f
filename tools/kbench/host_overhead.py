"""Host cost of one decode step on the GPU box: wall time of K back-to-back steps through the Python
wrapper, through a bound call (DecoderGPU.bind), and the bound call with a HIP event pair per step,
beside the GPU time of a step (events around K steps).
  python tools/kbench/host_overhead.py --code p7 --batch 65536"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import qec_ldpc_amd as q  # noqa: E402
from qec_ldpc_amd.codes import P7, P61, code_path  # noqa: E402
from qec_ldpc_amd.synthetic import bit_rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="p7")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    name, p, N = (P7, 0.02, 20) if a.code == "p7" else (P61, 0.01, 50)
    code = q.Quantum_LDPC_Code.createFromFile(code_path(name))
    dev = torch.device("cuda", 0)
    B = a.batch
    dec = q.DecoderGPU(code, 0, max_batch=B)
    sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_syndrome_dev(0x51EC0DE, 0, p, sX, sZ)
    sXb, sZb = bit_rows(sX), bit_rows(sZ)
    rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
    its = torch.empty((B, 2), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    wrapped = lambda: dec.decode_bits_packed_dev(sXb, sZb, p, N, "fixed", rec, its, stream=st)  # noqa: E731
    bound = dec.bind(dec.decode_bits_packed_dev, sXb, sZb, p, N, "fixed", rec, its, stream=st)

    def run(fn, events):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        e0.record(st)
        for _ in range(a.steps):
            if events:
                x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                x.record(st)
                fn()
                y.record(st)
            else:
                fn()
        e1.record(st)
        host = time.perf_counter() - t
        torch.cuda.synchronize()
        wall = time.perf_counter() - t
        return host / a.steps * 1e6, wall / a.steps * 1e6, e0.elapsed_time(e1) / a.steps * 1e3

    for label, fn, ev in (("wrapper", wrapped, False), ("bound", bound, False), ("bound+events", bound, True),
                          ("wrapper+events", wrapped, True)):
        h, w, g = run(fn, ev)
        print("%-16s host enqueue %.1f us/step  wall %.1f us/step  gpu %.1f us/step" % (label, h, w, g))
    # the host cost of the C call alone: a zero-size batch enqueues nothing
    t = time.perf_counter()
    for _ in range(a.steps):
        dec.decode_bits_packed_dev(sXb[:0], sZb[:0], p, N, "fixed", rec[:0], its[:0], stream=st)
    print("empty batch through the wrapper: %.1f us/call" % ((time.perf_counter() - t) / a.steps * 1e6))


if __name__ == "__main__":
    main()
