"""Headline benchmark: syndromes decoded per second at a fixed number of BP
iterations (BASELINE.json "metric"), on N MI355X with one process per GPU.

One step = one batched decode (both sectors, `--iters` fixed iterations, reference
update rules) of the rank's resident batch of synthetic depolarising syndromes.
Inputs are generated and copied to HBM before the timed region.  Ranks decode
disjoint shards of the sample index space; there is no collective in the data
path (syndromes are independent), only the timing barrier and a MAX reduction.

Prints one JSON line (rank 0).  Extra objects:
  roofline      -- the decode kernel's algorithmic bytes (16 B per
                   edge-iteration + bit-packed I/O, i.e. an HBM-resident flooding
                   schedule) over its HIP-event-timed launch duration, vs 8 TB/s;
                   the engine keeps messages in VGPRs, so frac > 1 means it moves
                   less than that schedule's bytes.
  full_arithmetic -- the same batch re-timed with QEC_OPT_HARD_PATHS off (every
                   iteration in full fp32 arithmetic, no hard-message forms), with a
                   bit-identity check against the timed run's outputs.
  no_cycle_jump -- the same with only QEC_OPT_CYCLE_JUMP off (hard-message forms, but
                   every iteration executed one by one), also bit-identity checked.
  valu          -- analytical full-arithmetic VALU lane-ops per launch over the
                   full_arithmetic launch time, vs the fp32 VALU issue ceiling (on the
                   hard-path launch the analytical count would over-count the work).
  cpu_baseline  -- oracle (CPU restatement of DecoderCPU, OpenMP) on host cores,
                   rank 0 at N = 1 only, bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CODES = {
    # name: (code file, default p, default iters, config label)
    "p61": ("J_4_K_5_L_10_P_61_s_9_t_49", 0.01, 50,
            "BASELINE configs[2]: J=4,K=5,L=10,P=61 code, batch 65536 per GPU, 50 fixed BP iters"),
    "p7": ("J_3_K_3_L_6_P_7_s_2_t_3", 0.02, 20,
           "BASELINE configs[1]: J=3,K=3,L=6,P=7 code, batch 65536 per GPU, 20 fixed BP iters"),
}
SEED = 0x51EC0DE
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, chip-level parameters
VALU_PEAK_TOPS = 78.64          # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz lane-ops/s (fp32 non-FMA issue ceiling)


def algorithmic_bytes_per_syndrome(code, iters):
    """16 B per edge-iteration (q read + r write, r read + q write)
    plus bit-packed I/O (syndrome bits in, correction bits out, one flag byte)."""
    EX, EZ = code.numEqsX * code.L, code.numEqsZ * code.L
    io = -(-(code.numEqsX + code.numEqsZ) // 8) + -(-(2 * code.n) // 8) + 1
    return 16 * (EX + EZ) * iters + io


def lane_ops_per_syndrome(code, iters):
    """Analytical VALU lane-operations per syndrome of the fixed-iteration decode
    ('Roofline'): per check (dc = L) L fma(1-2q), 2(L-2) prefix/first-slot
    muls, (L-1)(L-2)/2 leave-one-out muls, L output fmas, 1 select; per variable
    (dv = R) R subs, 2(R-1) prefix and R(R-1) leave-one-out muls, R adds and R
    correctly rounded divisions of 11 instructions."""
    L = code.L
    chk = L + 2 * (L - 2) + (L - 1) * (L - 2) // 2 + L + 1

    def var(R):
        return R + 2 * (R - 1) + R * (R - 1) + R + 11 * R

    per_iter = (code.numEqsX + code.numEqsZ) * chk + code.n * (var(code.J) + var(code.K))
    return per_iter * iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--code", choices=sorted(CODES), default="p61")
    ap.add_argument("--batch", type=int, default=65536, help="syndromes per GPU per step")
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--p", type=float, default=None)
    ap.add_argument("--stop", choices=["fixed", "ref", "syndrome"], default="fixed")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--hard-paths", type=int, default=1, help="QEC_OPT_HARD_PATHS for the timed run")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: skip the (untimed-step) RCCL gather of bit-packed decisions to rank 0")
    ap.add_argument("--no-full-arith", action="store_true",
                    help="skip the full_arithmetic re-timing (profiling runs: keeps the launch average clean)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import qec_ldpc_amd as q
    from qec_ldpc_amd.codes import code_path

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # RCCL ("nccl") over xGMI; QEC_BENCH_BACKEND=gloo rehearses the multi-rank path with
        # several ranks sharing one GPU (RCCL needs one GPU per rank)
        dist.init_process_group(os.environ.get("QEC_BENCH_BACKEND") or "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    fname, p_def, it_def, label = CODES[args.code]
    p = args.p if args.p is not None else p_def
    iters = args.iters if args.iters is not None else it_def
    code = q.Quantum_LDPC_Code.createFromFile(code_path(fname))
    dec = q.DecoderGPU(code, local)
    dec.set_option("hard_paths", args.hard_paths)
    B = args.batch

    # rank's shard of the sample index space, [rank*B, (rank+1)*B), drawn on the device
    # (Philox depolarising sampler + circulant syndrome kernel) before the timed region
    x = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    z = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
    dec.sample_depolarizing_dev(SEED, rank * B, p, x, z)
    dec.syndrome_dev(x, z, sX, sZ)
    torch.cuda.synchronize(dev)
    del x, z
    eX = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    eZ = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
    fl = torch.empty(B, dtype=torch.uint8, device=dev)
    its = torch.empty((B, 2), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        dec.decode_batch_dev(sX, sZ, p, iters, args.stop, eX, eZ, fl, its, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])

    total = B * world * args.steps
    value = total / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # executed iterations (fixed: == iters); mean over the batch for the other rules
    it_np = its.cpu().numpy()
    it_mean = (float(it_np[:, 0].mean()), float(it_np[:, 1].mean()))
    EX, EZ = code.numEqsX * code.L, code.numEqsZ * code.L
    io = -(-(code.numEqsX + code.numEqsZ) // 8) + -(-(2 * code.n) // 8) + 1
    bytes_per_syn = 16 * (EX * it_mean[0] + EZ * it_mean[1]) + io
    achieved_gbs = bytes_per_syn * B / (kernel_ms * 1e-3) / 1e9
    ops = lane_ops_per_syndrome(code, 1) * (it_mean[0] + it_mean[1]) / 2.0
    full = None
    nojump = None
    if args.hard_paths and not args.no_full_arith:
        full = full_arithmetic(dec, step, stream, B, (eX, eZ, fl, its))
        nojump = full_arithmetic(dec, step, stream, B, (eX, eZ, fl, its), option="cycle_jump")
    # the analytical count is the full-arithmetic work: only a launch without the
    # hard-message paths can be priced against it
    valu_ms = full["kernel_ms"] if full else (kernel_ms if not args.hard_paths else None)
    achieved_tops = ops * B / (valu_ms * 1e-3) / 1e12 if valu_ms else None
    traffic = None
    prof = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.code)
    if os.path.exists(prof):
        try:
            with open(prof) as f:
                pm = json.load(f)
            if pm.get("batch") == B and pm.get("iters") == iters and pm.get("stop") == args.stop:
                traffic = pm.get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    out = {
        "metric": "syndromes decoded/sec (fixed BP iters)",
        "value": round(value, 1),
        "unit": "syndromes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic i.i.d. depolarising errors (device Philox4x32-10 sampler, seed 0x51EC0DE), "
                "syndromes resident in HBM",
        "config": {"workload": label if world == 1 else label + " (BASELINE configs[3] shape, sharded)",
                   "code": code.describe(), "global_batch": B * world, "per_gpu_batch": B,
                   "bp_iters": iters, "stop": args.stop, "p": p, "parallelism": "dp%d" % world,
                   "kernel": dec.describe()},
        "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": int(bytes_per_syn * B), "kernel_ms": round(kernel_ms, 4)},
        "valu": None if achieved_tops is None else
                {"achieved": round(achieved_tops, 2), "peak": VALU_PEAK_TOPS, "unit": "Tlane-op/s",
                 "frac": round(achieved_tops / VALU_PEAK_TOPS, 4), "kernel_ms": round(valu_ms, 4),
                 "launch": "full_arithmetic" if full else "timed (hard paths off)"},
    }
    if full:
        out["full_arithmetic"] = full
        out["no_cycle_jump"] = nojump
    if args.stop != "fixed":
        hist = np.bincount(it_np.ravel(), minlength=iters + 1)
        out["iteration_histogram"] = {str(k): int(v) for k, v in enumerate(hist) if v}

    if world > 1 and not args.no_gather:
        # measured after the timed steps; a failure here must not cost the bench line
        try:
            out["gather"] = gather_step(dec, eX, eZ, fl, B, world, rank, dev, stream)
        except Exception as exc:  # noqa: BLE001
            out["gather"] = {"error": "%s: %s" % (type(exc).__name__, exc)}

    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(code, fname, sX.cpu().numpy(), sZ.cpu().numpy(), p, iters, args, eX, eZ, fl)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def gather_step(dec, eX, eZ, fl, B, world, rank, dev, stream):
    """every rank bit-packs its decoded shard on the device and the records
    are gathered to rank 0 over RCCL.  Measured after (not inside) the timed decode steps:
    the decode itself needs no exchange."""
    import torch
    import torch.distributed as dist
    from qec_ldpc_amd.gather import gather_records
    rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    dec.pack_decisions_dev(eX, eZ, fl, rec, stream=stream)
    b.record(stream)
    torch.cuda.synchronize(dev)
    pack_ms = a.elapsed_time(b)
    gather_records(rec)  # warm-up (communicator set-up)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    full = gather_records(rec)
    torch.cuda.synchronize(dev)
    dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3
    t = torch.tensor([ms, pack_ms], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = True
    if rank == 0:
        ok = bool(torch.equal(full[:B], rec))
    nbytes = B * rec.shape[1]
    return {"record_bytes": int(rec.shape[1]), "bytes_per_rank": int(nbytes), "pack_ms": round(float(t[1]), 4),
            "gather_ms": round(float(t[0]), 4), "root_GBps": round(world * nbytes / (float(t[0]) * 1e-3) / 1e9, 2),
            "rank0_shard_intact": ok}


def full_arithmetic(dec, step, stream, B, outs, reps=3, option="hard_paths"):
    """Re-time the step with a shortcut option off (hard_paths: every iteration in full
    arithmetic; cycle_jump: hard iterations run one by one) and check the outputs are the
    same bits."""
    import torch
    ref = [t.clone() for t in outs]
    dec.set_option(option, 0)
    try:
        step()
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            step()
            b.record(stream)
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
    finally:
        dec.set_option(option, 1)
    same = all(torch.equal(r, t) for r, t in zip(ref, outs))
    k = float(np.median(ms))
    return {"kernel_ms": round(k, 4), "syndromes_per_s": round(B / k * 1e3, 1), "identical": bool(same)}


def cpu_baseline(code, fname, sX_h, sZ_h, p, iters, args, eX, eZ, fl):
    """Oracle (CPU restatement of DecoderCPU, one decoder per OpenMP thread) on a bounded
    sample of the same batch; also checks the GPU's answers on that sample."""
    from oracle.oracle import OracleCode
    from qec_ldpc_amd.codes import code_path
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    orc = OracleCode(code_path(fname))
    probe = min(64 * threads, len(sX_h))
    t = time.perf_counter()
    orc.decode_batch(sX_h[:probe], sZ_h[:probe], p, iters, args.stop, nthreads=threads)
    rate = probe / max(time.perf_counter() - t, 1e-9)
    n = int(min(len(sX_h), max(probe, rate * args.cpu_seconds)))
    t = time.perf_counter()
    o = orc.decode_batch(sX_h[:n], sZ_h[:n], p, iters, args.stop, nthreads=threads)
    dt = time.perf_counter() - t
    same = (np.array_equal(o[0], eX[:n].cpu().numpy()) and np.array_equal(o[1], eZ[:n].cpu().numpy())
            and np.array_equal(o[2], fl[:n].cpu().numpy()))
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(n / dt, 2), "unit": "syndromes/s", "cores": threads, "kind": "port",
            "sample": "first %d syndromes of rank 0's batch, %s stop, %d iters (%.1f s)" % (n, args.stop, iters, dt),
            "cpu": cpu_model, "gpu_matches_oracle_on_sample": bool(same)}


if __name__ == "__main__":
    main()
