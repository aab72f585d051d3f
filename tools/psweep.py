"""Physical error-rate sweep (BASELINE.json configs[4]): P61 code, early-termination
BP (--stop syndrome: stop once the hard decision satisfies the syndrome, cap 50
iterations), i.i.d. depolarising errors, on N GPUs.

One process per GPU (python -m torch.distributed.run --nproc-per-node N
tools/psweep.py ...).  Each rank runs qec_monte_carlo on its contiguous shard of
the sample index space (device sampler -> syndromes -> decode -> I-P check ->
counters, all on its GPU); the per-p counters are summed across ranks with one
all-reduce (RCCL over xGMI) and the wall time is the max over ranks.  Rank 0
prints one JSON line per p and a final summary line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT_PS = [1e-3, 2e-3, 5e-3, 1e-2, 2e-2, 5e-2, 1e-1]
FIELDS = ("tested", "withX", "withZ", "synX", "synZ", "logical", "corrected", "convX", "convZ", "iterationsX",
          "iterationsZ")


def summarize(p, c, seconds, world):
    """Rates from summed counters (also used by the CPU test of the reduction)."""
    t = max(c["tested"], 1)
    failed = c["tested"] - c["corrected"]
    return {
        "p": p, "samples": c["tested"], "n_gpus": world,
        "syndromes_per_s": round(c["tested"] / seconds, 1) if seconds > 0 else None,
        "seconds": round(seconds, 4),
        "logical_error_rate": c["logical"] / t,
        "decoder_failure_rate": failed / t,  # syndrome fail or logical error
        "syndrome_fail_rate_x": c["synX"] / t, "syndrome_fail_rate_z": c["synZ"] / t,
        "mean_iterations_x": c["iterationsX"] / t, "mean_iterations_z": c["iterationsZ"] / t,
        "counters": {k: int(c[k]) for k in FIELDS},
    }


def mc_roofline(p, samples, stop, iters, batch, code_name):
    """The roofline of a sweep point from its rocprofv3 profile (profiles/pmc_mc_p61_p<p>.json; other stop
    rules than the syndrome stop pmc_mc_p61_<stop>_p<p>.json;
    tools/gpu/run_mc_profile.sh): per kernel its dispatch time and VALU / LDS issue fractions, and the
    dominant kernel's bound -- only from a profile of this workload (p, samples, batch, stop, cap) taken
    on this very build of the library (else the reason)."""
    import qec_ldpc_amd as q
    sfx = "" if stop == "syndrome" else stop + "_"
    path = os.path.join(ROOT, "profiles", "pmc_mc_p61_%sp%g.json" % (sfx, p))
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return {"frac": None, "note": "no %s" % os.path.relpath(path, ROOT)}
    if "P_61" not in code_name or (pm.get("stop"), pm.get("iters"), pm.get("samples"), pm.get("batch")) != \
            (stop, iters, samples, batch):
        return {"frac": None, "note": "%s: other workload" % os.path.basename(path)}
    if pm.get("build_id") != q.build_id():
        return {"frac": None, "note": "%s: collected on another build of the library" % os.path.basename(path)}
    dom = pm["dominant"]
    k = pm["kernels"][dom]
    lds = k.get("lds_issue_frac") or 0.0
    valu = k.get("valu_issue_frac") or 0.0
    return {"dominant_kernel": dom, "bound": "lds" if lds > valu else "valu",
            "frac": max(lds, valu),  # the bound's issue fraction
            "valu_issue_frac": k.get("valu_issue_frac"), "lds_issue_frac": k.get("lds_issue_frac"),
            "wait_over_issue": k.get("wait_over_issue"),
            "kernels_us": {n: round(v["avg_ns"] / 1e3, 1) for n, v in pm["kernels"].items()},
            "basis": "profiled dispatch times: SQ_INSTS_VALU x 2 / (1024 SIMDs x 2.4 GHz x time); LDS: SQ_INSTS_LDS "
                     "x 6 CU-cycles / (256 CUs x 2.4 GHz x time)",
            "profile": os.path.relpath(path, ROOT)}


def reduce_counters(r, times, backend, dev):
    """Sums the per-rank counters and takes the max of the per-rank times across ranks (one
    all-reduce each, on the device for RCCL, on the host for gloo); without an initialised
    process group (one process) returns them as they are."""
    import torch
    import torch.distributed as dist
    cdev = dev if backend in (None, "nccl") else torch.device("cpu")  # gloo reduces host tensors
    vec = torch.tensor([r[k] for k in FIELDS], dtype=torch.int64, device=cdev)
    tm = torch.tensor(times, dtype=torch.float64, device=cdev)
    if dist.is_initialized():
        dist.all_reduce(vec)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    return dict(zip(FIELDS, vec.cpu().tolist())), [float(x) for x in tm.cpu().tolist()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="J_4_K_5_L_10_P_61_s_9_t_49")
    ap.add_argument("--total", type=int, default=1 << 20, help="samples per p over all GPUs")
    ap.add_argument("--ps", type=float, nargs="*", default=DEFAULT_PS)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--stop", default="syndrome", choices=["syndrome", "ref", "fixed"])
    # one batch per p per GPU: batches of 65 536 ran 25-35 % slower (five launches and their gaps
    # per batch, and a launch tail each; profiles/r02/psweep_batch_r02s3zd.json)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--seed", type=lambda v: int(v, 0), default=0x51EC0DE)
    ap.add_argument("--reps", type=int, default=3, help="runs per p (the median is reported, min and max beside it)")
    ap.add_argument("--out", default=None, help="write the per-p lines to this JSON file (rank 0)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="decoder option (qec_decoder_set_option), e.g. schedule=0")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import qec_ldpc_amd as q
    from qec_ldpc_amd.codes import code_path
    from qec_ldpc_amd.synthetic import shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # this rank's GPU first, so RCCL's communicator and the barriers run on it
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    backend = None
    if world > 1:
        # RCCL ("nccl") over xGMI; QEC_BENCH_BACKEND=gloo rehearses the multi-rank path with several
        # ranks sharing one GPU (RCCL needs one GPU per rank)
        backend = os.environ.get("QEC_BENCH_BACKEND") or "nccl"
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    code = q.Quantum_LDPC_Code.createFromFile(code_path(args.code))
    dec = q.DecoderGPU(code, local)
    for kv in args.opt:
        k, v = kv.split("=")
        dec.set_option(k, int(v))
    lo, hi = shard_range(args.total, rank, world)
    # warm-up at the full batch size, so the workspace is reserved before the timed runs
    dec.monte_carlo(args.seed, lo, min(hi - lo, args.batch), args.ps[0], args.iters, args.stop, args.batch)
    lines = []
    for p in args.ps:
        if world > 1:
            dist.barrier()
        # the same samples --reps times (identical counters, checked); the median run's time is
        # reported, the fastest and slowest beside it
        # The timed runs carry no decode-timing events (QEC_OPT_MC_DECODE_TIME 0: each event record
        # costs the GPU a few microseconds between launches); one more run of the same samples with
        # them gives decode_seconds.
        runs = []
        dec.set_option("mc_decode_time", 0)
        for _ in range(max(1, args.reps)):
            t0 = time.perf_counter()
            r = dec.monte_carlo(args.seed, lo, hi - lo, p, args.iters, args.stop, args.batch)
            runs.append((time.perf_counter() - t0, r))
        dec.set_option("mc_decode_time", 1)
        rt = dec.monte_carlo(args.seed, lo, hi - lo, p, args.iters, args.stop, args.batch)
        same = all(all(r[k] == runs[0][1][k] for k in FIELDS) for _, r in runs + [(0, rt)])
        order = sorted(range(len(runs)), key=lambda i: runs[i][0])
        dt, r = runs[order[len(order) // 2]]
        c, tm = reduce_counters(r, [dt, rt["decodeSeconds"], runs[order[0]][0], runs[order[-1]][0], 0.0 if same else 1.0],
                                backend, dev)
        line = summarize(p, c, tm[0], world)
        line["decode_seconds"] = round(tm[1], 4)  # decode kernels only (the rest: front end + counts), untimed run
        line["reps"] = {"n": len(runs), "reported": "median", "min_seconds": round(tm[2], 4),
                        "max_seconds": round(tm[3], 4), "counters_identical": tm[4] == 0.0}
        if backend:
            line["backend"] = backend
        line.update({"code": code.describe(), "stop": args.stop, "max_iters": args.iters, "seed": args.seed})
        line["roofline"] = mc_roofline(p, hi - lo, args.stop, args.iters, args.batch, args.code)
        lines.append(line)
        if rank == 0:
            print(json.dumps(line), flush=True)
    if rank == 0:
        tot = sum(l["samples"] for l in lines)
        sec = sum(l["seconds"] for l in lines)
        print(json.dumps({"sweep": "psweep", "n_gpus": world, "total_samples": tot, "seconds": round(sec, 3),
                          "syndromes_per_s": round(tot / sec, 1)}), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(lines, f, indent=1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
