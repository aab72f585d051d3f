"""Faithfulness of the CPU restatement (oracle/qec_oracle.c) as a stand-in for the compiled reference
DecoderCPU (SURVEY.md 8(d) "Faithfulness check"): the oracle's decode rate on this
container's cores, same configs, same threads (1 and all), i.i.d. depolarising inputs, beside the
compiled reference's rates that BASELINE.md section 2 records for the same container.

The reference itself is not built here (its headers need cusp / thrust), so the
reference side of the ratio is the recorded BASELINE.md section 2 range, not a same-run measurement.
The oracle's fixed-N rows include Decode's post-processing (hard decision, convergence and syndrome
flags; DecoderCPU.h:354-384), the reference's fixed-N rows do not (the update
functions looped), so those ratios understate the restatement's speed slightly.
  python tools/faithfulness.py [--seconds 6] [--out profiles/r06/faithfulness.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# BASELINE.md section 2 (compiled reference DecoderCPU, this container, g++ 11.4 -O2 -fopenmp)
REFERENCE = {
    ("p61", "fixed"): {"1": (147, 199), "8": (1100, 1220)},
    ("p61", "ref"): {"1": (455, 599), "8": (2850, 3620)},
    ("p7", "fixed"): {"1": (7200, 10100), "8": (51900, 61200)},
    ("p7", "ref"): {"1": (21700, 31400), "8": (169000, 196000)},
}
CONFIGS = {"p61": ("J_4_K_5_L_10_P_61_s_9_t_49", 0.01, 50), "p7": ("J_3_K_3_L_6_P_7_s_2_t_3", 0.02, 20)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0, help="target length of each timed run")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import qec_ldpc_amd as q
    from oracle.oracle import OracleCode
    from qec_ldpc_amd.codes import code_path
    from qec_ldpc_amd.synthetic import depolarizing_errors
    allthreads = os.cpu_count() or 1
    rows = []
    for key, (fname, p, iters) in CONFIGS.items():
        code = q.Quantum_LDPC_Code.createFromFile(code_path(fname))
        orc = OracleCode(code_path(fname))
        x, z = depolarizing_errors(code.n, 0, 65536, p)
        sX, sZ = code.syndrome(0, x), code.syndrome(1, z)
        for stop in ("fixed", "ref"):
            for nt in (1, allthreads):
                probe = 16 * nt
                t = time.perf_counter()
                orc.decode_batch(sX[:probe], sZ[:probe], p, iters, stop, nthreads=nt)
                n = int(min(len(sX), max(probe, probe / (time.perf_counter() - t) * a.seconds)))
                rates = []
                for _ in range(a.reps):
                    t = time.perf_counter()
                    orc.decode_batch(sX[:n], sZ[:n], p, iters, stop, nthreads=nt)
                    rates.append(n / (time.perf_counter() - t))
                ref = REFERENCE[(key, stop)].get(str(nt))
                row = {"code": key, "stop": stop, "iters": iters, "p": p, "threads": nt, "samples": n,
                       "oracle_per_s": [round(r, 1) for r in rates]}
                if ref:
                    mid = (ref[0] + ref[1]) / 2
                    med = sorted(rates)[len(rates) // 2]
                    row.update({"reference_per_s": list(ref), "ratio_to_reference_mid": round(med / mid, 3),
                                "ratio_range": [round(min(rates) / ref[1], 3), round(max(rates) / ref[0], 3)]})
                rows.append(row)
                print(json.dumps(row), flush=True)
    out = {"what": "oracle (CPU restatement) decode rate / compiled-reference DecoderCPU rate (BASELINE.md 2)",
           "cpu": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), ""),
           "threads_all": allthreads, "command": "python tools/faithfulness.py", "rows": rows}
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
