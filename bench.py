"""Headline benchmark: syndromes decoded per second at a fixed number of BP iterations
(BASELINE.json "metric"), on N MI355X with one process per GPU.

Workload (BASELINE.json configs[3]): the J=4,K=5,L=10,P=61 code, a global batch of 2^20
depolarising syndromes (p = 0.01), 50 fixed BP iterations, sharded contiguously over the N
GPUs: rank g decodes samples [g B / N, (g + 1) B / N) (strong scaling: the same 2^20 syndromes
at every N).  `--batch` instead fixes the per-GPU batch (weak scaling), labelled as such.

One step = one batched decode of the rank's resident shard (both sectors, reference update
rules, exactly `--iters` iterations) writing bit-packed decision records (eX bits, eZ bits,
flags byte: SURVEY.md 8(d)'s I/O model).  Syndromes are generated on the device (fused
gap-walk sampler + syndrome kernel) before the timed region.  There is no collective in the
decode step (syndromes are independent); at N > 1 the RCCL gather of every rank's records to
rank 0 is timed separately, as its own component and end to end (decode + gather per step).

Prints one JSON line (rank 0).  Extra objects:
  roofline        the dominant kernel (the decode) against its real bound, VALU issue:
                  SQ_INSTS_VALU per launch (rocprofv3 PMC, profiles/pmc_<code>.json, per syndrome
                  x the batch) x 2 cycles / (1024 SIMDs x 2.4 GHz x step time); step time = the GPU
                  span per step from one HIP event pair on the launch stream around the K timed
                  steps, so it includes any idle gap between launches (frac is then a lower bound;
                  the rocprofv3 kernel trace under profiles/ gives the launches alone); traffic =
                  PMC HBM bytes.
                  frac is the counter-exact figure; cost-weighted figures, the LDS issue fraction and
                  the LDS bank-conflict share sit beside it (LDS is a co-bound of the P61 kernels).
  roofline_hbm_alg  SURVEY.md 8(d)'s HBM-resident flooding-schedule bytes over the launch time:
                  valid only if frac <= 1 (the engine keeps messages in VGPRs and takes exact
                  shortcuts, so it does far less than that schedule's traffic).
  value_full_arithmetic / full_arithmetic  the same batch re-timed with every iteration in full
                  fp32 arithmetic (QEC_OPT_HARD_PATHS = 0), bit-identity checked: the "50 BP
                  iterations executed" rate.
  sector_iterations  executed sector-iterations of one launch by phase (soft / hard / agreed /
                  jumped), from the instrumented kernel (QEC_OPT_PHASE_STATS).
  executed_iteration_fraction  executed / nominal sector-iterations of the timed launch (the rest are
                  exact jumps; 1.0 for value_full_arithmetic).
  ref_stop        the same batch under the reference stop rule (DecoderCPU::Decode unmodified): rate,
                  per-sector iteration histogram, oracle check on a slice.
  published_blocks  DecoderGPU::GetStatistics on two of the reference's published results blocks
                  (seeded MSVC sampler, same samples): rate vs the published duration, counters checked,
                  on one decoder and on a two-part (multi-device API) decoder.
  sustained       a >= 1 s window of the same step (clock-settled rate).
  cpu_baseline    the oracle (CPU restatement of DecoderCPU, OpenMP) on host cores, rank 0 at
                  N = 1 only, bounded sample of the same workload; also 1 thread and
                  BASELINE configs[0] (P7, 1k syndromes, 20 iterations).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CODES = {
    # name: (code file, default p, default iters)
    "p61": ("J_4_K_5_L_10_P_61_s_9_t_49", 0.01, 50),
    "p7": ("J_3_K_3_L_6_P_7_s_2_t_3", 0.02, 20),
}
SEED = 0x51EC0DE
GLOBAL_BATCH = 1 << 20          # BASELINE configs[3]
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, chip-level parameters
VALU_PEAK_TOPS = 78.64          # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz lane-ops/s (fp32 non-FMA issue ceiling)
SIMDS = 1024                    # 256 CU x 4 SIMD
CLOCK_GHZ = 2.4                 # peak engine clock
VALU_ISSUE_CYCLES = 2           # one wave64 VALU instruction per 2 cycles on a SIMD-32 (MI355X_MICROARCH.md)


def algorithmic_bytes_per_syndrome(code, it_x, it_z):
    """16 B per edge-iteration (q read + r write, r read + q write)
    plus bit-packed I/O (syndrome bits in, correction bits out, one flag byte)."""
    EX, EZ = code.numEqsX * code.L, code.numEqsZ * code.L
    io = -(-(code.numEqsX + code.numEqsZ) // 8) + -(-(2 * code.n) // 8) + 1
    return 16 * (EX * it_x + EZ * it_z) + io


def lane_ops_per_syndrome(code, iters):
    """Analytical VALU lane-operations per syndrome of the fixed-iteration decode
    ('Roofline'): per check (dc = L) L fma(1-2q), 2(L-2) prefix/first-slot
    muls, (L-1)(L-2)/2 leave-one-out muls, L output fmas, 1 select; per variable
    (dv = R) R subs, 2(R-1) prefix and R(R-1) leave-one-out muls, R adds and R
    correctly rounded divisions of 6 instructions (the kernel's short form)."""
    L = code.L
    chk = L + 2 * (L - 2) + (L - 1) * (L - 2) // 2 + L + 1

    def var(R):
        return R + 2 * (R - 1) + R * (R - 1) + R + 6 * R

    per_iter = (code.numEqsX + code.numEqsZ) * chk + code.n * (var(code.J) + var(code.K))
    return per_iter * iters


def shard(total, rank, world):
    return total * rank // world, total * (rank + 1) // world


def library_build_id():
    import qec_ldpc_amd as q
    return q.build_id()


def load_pmc(code_name, iters, stop, p, batch, hard_paths=1, input_form="bits"):
    """profiles/pmc_<code>_<batch>[_hp0].json or profiles/pmc_<code>[_hp0].json if it was collected on
    this workload (code, iters, stop, p, batch, hard paths on / off) with a library built from these
    very sources (tools/gpu/pmc_summary.py stamps qec_build_id(), a hash of the sources and flags): a
    profile of another build or batch would mis-state the roofline."""
    why = []
    lib = library_build_id()
    sfx = "" if hard_paths else "_hp0"
    for name in ("pmc_%s_%d%s.json" % (code_name, batch, sfx), "pmc_%s%s.json" % (code_name, sfx)):
        path = os.path.join(ROOT, "profiles", name)
        try:
            with open(path) as f:
                pm = json.load(f)
        except (OSError, ValueError):
            continue
        if (pm.get("iters") != iters or pm.get("stop") != stop or abs(float(pm.get("p", -1)) - p) > 1e-12
                or int(pm.get("hard_paths", 1)) != (1 if hard_paths else 0) or pm.get("input", "bytes") != input_form):
            why.append("%s: other workload" % name)
        elif pm.get("batch") != batch:
            why.append("%s: batch %s" % (name, pm.get("batch")))
        elif pm.get("build_id") != lib:
            why.append("%s: collected on another build of the library" % name)
        else:
            return pm, path
    return None, "; ".join(why) or "no profiles/pmc_%s*%s.json" % (code_name, sfx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: enough for a >= 1 s window)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--code", choices=sorted(CODES), default="p61")
    ap.add_argument("--global-batch", type=int, default=GLOBAL_BATCH,
                    help="syndromes per step over all GPUs (strong scaling)")
    ap.add_argument("--batch", type=int, default=None, help="syndromes per GPU per step (weak scaling instead)")
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--p", type=float, default=None)
    ap.add_argument("--stop", choices=["fixed", "ref", "syndrome"], default="fixed")
    ap.add_argument("--output", choices=["packed", "bytes"], default="packed",
                    help="decision records (default) or eX/eZ/flags byte arrays")
    ap.add_argument("--input", choices=["bits", "bytes"], default="bits",
                    help="syndromes as bit rows (default; SURVEY.md 8(d)'s bit-packed I/O, "
                         "qec_decode_bits_packed_dev) or as 0/1 bytes (qec_decode_batch_packed_dev)")
    ap.add_argument("--min-seconds", type=float, default=1.0, help="sustained window / auto --steps target")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--hard-paths", type=int, default=1, help="QEC_OPT_HARD_PATHS for the timed run")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="decoder option for the timed run (qec_decoder_set_option), e.g. schedule=0")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip the RCCL gather measurements")
    ap.add_argument("--gather-world1", action="store_true",
                    help="N = 1: measure the gather paths in an RCCL group of one (the gather is rank 0's own copy; "
                         "DESIGN.md section 9's world-1 rate)")
    ap.add_argument("--graph", action="store_true",
                    help="time the step as a replay of one captured HIP graph of it (same kernels, no per-launch "
                         "host work or inter-launch gaps); without it the replay is reported in `graph`")
    ap.add_argument("--no-extras", action="store_true",
                    help="only the timed steps (profiling runs: no full-arithmetic / phase / sustained re-timings)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and "RANK" not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks (one process per GPU) under
        # torch.distributed.run as children, before anything here touches a GPU, and pass on their
        # exit status; rank 0 prints the JSON line
        sys.exit(relaunch(args.gpus))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE %d: refusing to report a %d-GPU run as %d" %
              (args.gpus, world, world, args.gpus), file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    import qec_ldpc_amd as q
    from qec_ldpc_amd.codes import code_path
    from qec_ldpc_amd.synthetic import bit_rows

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # this rank's GPU first, so RCCL's communicator and the barriers run on it
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    backend = None
    if world > 1:
        # RCCL ("nccl") over xGMI; QEC_BENCH_BACKEND=gloo rehearses the multi-rank path with
        # several ranks sharing one GPU (RCCL needs one GPU per rank)
        backend = os.environ.get("QEC_BENCH_BACKEND") or "nccl"
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    fname, p_def, it_def = CODES[args.code]
    p = args.p if args.p is not None else p_def
    iters = args.iters if args.iters is not None else it_def
    code = q.Quantum_LDPC_Code.createFromFile(code_path(fname))
    if args.batch is not None:
        scaling, lo, hi = "weak", rank * args.batch, (rank + 1) * args.batch
        global_batch = args.batch * world
    else:
        scaling, global_batch = "strong", args.global_batch
        lo, hi = shard(global_batch, rank, world)
    B = hi - lo
    dec = q.DecoderGPU(code, local, max_batch=B)
    dec.set_option("hard_paths", args.hard_paths)
    for kv in args.opt:
        k, v = kv.split("=")
        dec.set_option(k, int(v))

    # the rank's shard of the sample index space, drawn and turned into syndromes on the device
    # (fused gap-walk sampler + syndrome kernel) before the timed region
    sX = torch.empty((B, code.numEqsX), dtype=torch.uint8, device=dev)
    sZ = torch.empty((B, code.numEqsZ), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    dec.sample_syndrome_dev(SEED, lo, p, sX, sZ, stream=stream)
    S = {"stream": stream}  # the step's launch stream (a capture stream while a graph is recorded)
    its = torch.empty((B, 2), dtype=torch.int32, device=dev)
    packed = args.output == "packed"
    bits = args.input == "bits"
    if bits and not packed:
        raise SystemExit("--input bits decodes into records (--output packed)")
    sXb, sZb = bit_rows(sX), bit_rows(sZ)  # bit c of word c / 32 = check c (the Monte-Carlo pipeline's layout)
    if packed:
        rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=dev)
        outs = (rec, its)

        def step_bytes():
            dec.decode_batch_packed_dev(sX, sZ, p, iters, args.stop, rec, its, stream=S["stream"])

        def step_bits():
            dec.decode_bits_packed_dev(sXb, sZb, p, iters, args.stop, rec, its, stream=S["stream"])

        step = step_bits if bits else step_bytes
        # the timed step: the same call with its tensors validated once (DecoderGPU.bind), so the host
        # side of a step is the C ABI call alone
        def bound_into(r):
            return (dec.bind(dec.decode_bits_packed_dev, sXb, sZb, p, iters, args.stop, r, its, stream=stream) if bits
                    else dec.bind(dec.decode_batch_packed_dev, sX, sZ, p, iters, args.stop, r, its, stream=stream))

        bound = bound_into(rec)
    else:
        eX = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
        eZ = torch.empty((B, code.n), dtype=torch.uint8, device=dev)
        fl = torch.empty(B, dtype=torch.uint8, device=dev)
        outs = (eX, eZ, fl, its)

        def step():
            dec.decode_batch_dev(sX, sZ, p, iters, args.stop, eX, eZ, fl, its, stream=S["stream"])

        bound = dec.bind(dec.decode_batch_dev, sX, sZ, p, iters, args.stop, eX, eZ, fl, its, stream=stream)

    eager_step = step
    step = capture_graph(eager_step, S, dev) if args.graph else bound
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    steps = args.steps
    if steps is None:  # enough steps for a >= min-seconds window (probe 3 steps)
        t = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize(dev)
        per = (time.perf_counter() - t) / 3
        steps = max(5, int(math.ceil(args.min_seconds / max(per, 1e-6))))
        if world > 1:
            s = torch.tensor([steps], dtype=torch.int64, device=dev)
            dist.all_reduce(s, op=dist.ReduceOp.MAX)
            steps = int(s.item())

    elapsed, kernel_ms = timed_steps(step, steps, stream, dev, world)
    total = B * world * steps if scaling == "weak" else global_batch * steps
    value = total / elapsed
    ms_per_step = elapsed / steps * 1e3

    # executed iterations of the timed batch (fixed: == iters)
    it_np = its.cpu().numpy()
    it_mean = (float(it_np[:, 0].mean()), float(it_np[:, 1].mean()))
    workload = ("BASELINE configs[3]: J=4,K=5,L=10,P=61 code, 2^20 syndromes sharded over %d GPU(s)" % world
                if args.code == "p61" and scaling == "strong" and global_batch == GLOBAL_BATCH else
                "%s code, %d syndromes %s" % (code.describe(), global_batch,
                                              "per step over %d GPU(s)" % world if scaling == "strong"
                                              else "(%d per GPU, weak scaling)" % B))
    stop_label = {"fixed": "%d fixed BP iters" % iters, "ref": "reference stop rule (DecoderCPU::Decode), cap %d" % iters,
                  "syndrome": "syndrome stop, cap %d" % iters}[args.stop]
    metric = {"fixed": "syndromes decoded/sec (fixed BP iters)",
              "ref": "syndromes decoded/sec (reference stop rule)",
              "syndrome": "syndromes decoded/sec (syndrome stop)"}[args.stop]
    out = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "syndromes/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic i.i.d. depolarising errors (device gap-walk sampler over Philox4x32-10, seed 0x51EC0DE), "
                "syndromes resident in HBM",
        "config": {"workload": workload + ", " + stop_label, "code": code.describe(), "global_batch": global_batch,
                   "per_gpu_batch": B, "bp_iters": iters, "stop": args.stop, "p": p, "output": args.output,
                   "input": args.input,
                   "parallelism": "dp%d" % world, "kernel": dec.describe(), "hard_paths": args.hard_paths,
                   **({"options": args.opt} if args.opt else {})},
        "p": p,
        "mean_iterations": {"X": round(it_mean[0], 4), "Z": round(it_mean[1], 4)},
        "decode_ms": round(kernel_ms, 4),
        "decode_ms_basis": "GPU time of a step (dispatch order + decode launches): one HIP event pair on the launch "
                           "stream around the timed steps, / steps",
    }
    pm, pm_path = load_pmc(args.code, iters, args.stop, p, B, args.hard_paths, args.input)
    out["roofline"] = valu_roofline(pm, pm_path, B, kernel_ms)
    if out["roofline"].get("traffic") is not None:
        # SURVEY.md 8(d)'s bit-packed I/O per syndrome (syndrome bits in, correction bits out, flag byte)
        io = -(-(code.numEqsX + code.numEqsZ) // 8) + -(-(2 * code.n) // 8) + 1
        out["roofline"]["traffic_per_syndrome"] = round(out["roofline"]["traffic"] / B, 1)
        out["roofline"]["io_bytes_per_syndrome_8d"] = io
    ab = algorithmic_bytes_per_syndrome(code, it_mean[0], it_mean[1]) * B
    gbs = ab / (kernel_ms * 1e-3) / 1e9
    out["roofline_hbm_alg"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(gbs / HBM_PEAK_GBS, 4), "valid": gbs <= HBM_PEAK_GBS,
                               "algorithmic_bytes_per_launch": int(ab),
                               "note": "SURVEY 8(d) HBM-resident flooding schedule; the engine keeps messages in "
                                       "VGPRs, so this is not its bound when frac > 1"}

    if not args.no_extras:
        if args.hard_paths:
            full = retime(dec, step, stream, B, outs, {"hard_paths": 0}, world=world)
            # whole job: every rank's shard at the slowest rank's kernel time
            out["value_full_arithmetic"] = full["syndromes_per_s"]
            pmf, pmf_path = load_pmc(args.code, iters, args.stop, p, B, 0, args.input)
            full["roofline"] = valu_roofline(pmf, pmf_path, B, full["kernel_ms"])
            ops = lane_ops_per_syndrome(code, 1) * (it_mean[0] + it_mean[1]) / 2.0
            tops = ops * B / (full["kernel_ms"] * 1e-3) / 1e12
            full["valu_lane_ops"] = {"achieved": round(tops, 2), "peak": VALU_PEAK_TOPS, "unit": "Tlane-op/s",
                                     "frac": round(tops / VALU_PEAK_TOPS, 4),
                                     "basis": "secondary: analytical lane-ops of full-arithmetic BP (bench.py "
                                              "lane_ops_per_syndrome, 6-instruction divisions); the counter "
                                              "figure is full_arithmetic.roofline"}
            out["full_arithmetic"] = full
        if packed:
            # the other syndrome layout, same outputs (bytes: 549 B per P61 syndrome in, bits: 72 B)
            other = step_bytes if bits else step_bits
            out["other_input"] = dict(retime_step(other, stream, B, outs, world=world),
                                      input="bytes" if bits else "bits")
            out["no_cycle_jump"] = retime(dec, step, stream, B, outs, {"cycle_jump": 0}, world=world)
        out["sector_iterations"] = phase_counts(dec, step, stream, its, B)
        pl = out["sector_iterations"].get("per_launch")
        if pl:
            out["executed_iteration_fraction"] = round(pl["sector_iterations_executed"] / pl["sector_iterations_nominal"], 4)
        if args.stop == "fixed" and packed:
            out["ref_stop"] = ref_stop(dec, sX, sZ, p, iters, B, stream, world, fname, rank == 0 and not args.no_cpu)
        out["sustained"] = sustained(step, stream, dev, world, ms_per_step, args.min_seconds,
                                     global_batch if scaling == "strong" else B * world)

    if not args.no_extras and not args.graph:
        out["graph"] = graph_retime(eager_step, S, dev, stream, B, outs, world, global_batch if scaling == "strong"
                                    else B * world, steps)
    if args.graph:
        out["config"]["launch"] = "hip graph replay"

    solo = world == 1 and args.gather_world1 and packed
    if solo:  # an RCCL group of one, after every timed measurement above
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % free_port(), rank=0, world_size=1)
        backend = "nccl"
    if (world > 1 or solo) and not args.no_gather and packed:
        try:
            out["gather"] = gather_measure(dec, step, rec, B, world, rank, dev, stream, steps, global_batch, backend,
                                           bound_into)
        except Exception as exc:  # noqa: BLE001 -- a failure here must not cost the bench line
            out["gather"] = {"error": "%s: %s" % (type(exc).__name__, exc)}
    if solo:
        dist.destroy_process_group()

    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(code, fname, sX, sZ, p, iters, args, outs, packed)
    if rank == 0 and world == 1 and not args.no_extras:
        out["published_blocks"] = published_blocks(local)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def capture_graph(step, S, dev):
    """One step captured into a HIP graph (torch.cuda.CUDAGraph: hipStreamBeginCapture on a side stream;
    the decoder's device entry points are capture-safe and allocate nothing at max_batch); returns its
    replay on the current stream."""
    import torch
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):  # one eager step on the side stream first (workspace already sized)
        S["stream"] = cap
        step()
    torch.cuda.current_stream(dev).wait_stream(cap)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=cap):
            step()
    finally:
        S["stream"] = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    return g.replay


def graph_retime(step, S, dev, stream, B, outs, world, per_step_units, steps):
    """The same step replayed from one captured HIP graph: K replays between synchronisations (max over
    ranks), outputs compared with the eager step's."""
    import torch
    ref = [t.clone() for t in outs]
    try:
        replay = capture_graph(step, S, dev)
    except Exception as exc:  # noqa: BLE001 -- reported, the eager line stands
        return {"error": "%s: %s" % (type(exc).__name__, exc)}
    for t in outs:
        t.zero_()
    replay()
    torch.cuda.synchronize(dev)
    same = all(torch.equal(r, t) for r, t in zip(ref, outs))
    elapsed, kernel_ms = timed_steps(replay, steps, stream, dev, world)
    return {"what": "the timed step replayed from one captured HIP graph", "steps": steps,
            "ms_per_step": round(elapsed / steps * 1e3, 4), "syndromes_per_s": round(per_step_units * steps / elapsed, 1),
            "kernel_ms": round(kernel_ms, 4), "identical": bool(same)}


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(nproc):
    """Runs this script under `python -m torch.distributed.run --nproc-per-node nproc` (rendezvous on
    127.0.0.1) as a child process with the same arguments; returns its exit status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def timed_steps(step, steps, stream, dev, world):
    """K steps between barrier + synchronize on both sides; wall time max over ranks, and the GPU time
    of a step from one HIP event pair on the launch stream around the K steps (an event pair around
    every step costs a P7 configs[1] step ~10 us of GPU time: tools/kbench/host_overhead.py)."""
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = e0.elapsed_time(e1) / steps
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
    return elapsed, kernel_ms


def valu_roofline(pm, path, B, kernel_ms):
    """VALU-issue roofline of the decode kernel: PMC SQ_INSTS_VALU (wave instructions) per
    syndrome x B, each taking VALU_ISSUE_CYCLES of a SIMD, over this run's GPU step span (includes inter-launch gaps)."""
    peak = SIMDS * CLOCK_GHZ * 1e9 / VALU_ISSUE_CYCLES / 1e12  # T wave-instructions/s
    base = {"bound": "valu", "peak": round(peak, 4), "unit": "Twave-instr/s",
            "peak_basis": "1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction"}
    if pm is None or "valu_insts_per_syndrome" not in pm:
        base.update({"achieved": None, "frac": None, "traffic": None,
                     "note": "no PMC profile for this workload and library (%s)" % path})
        return base
    insts = pm["valu_insts_per_syndrome"] * B
    ach = insts / (kernel_ms * 1e-3) / 1e12
    base.update({"achieved": round(ach, 4), "frac": round(ach / peak, 4),
                 "traffic": int(round(pm["hbm_bytes_per_syndrome"] * B)) if pm.get("hbm_bytes_per_syndrome") else None,
                 "valu_insts_per_launch": int(insts), "kernel_ms": round(kernel_ms, 4),
                 "profile": os.path.relpath(path, ROOT), "profile_batch": pm.get("batch"),
                 "profile_frac": pm.get("valu_issue_frac")})
    if pm.get("valu_weighted_slots_per_syndrome"):
        # secondary: cost-weighted issue, a transcendental (v_rcp_f32, SQ_INSTS_VALU_TRANS_F32) priced at
        # 4 slots (this repo's probe: 8.1 vs 2.1-2.4 cycles at full occupancy) and at 2 slots
        # (MI355X_MICROARCH.md's issue-cost row: 8 vs 4 cycles for one wave)
        trans = pm["valu_trans_per_launch"] * B / pm["batch"]
        for label, w in (("frac_weighted_probe4x", 4), ("frac_weighted_guide2x", 2)):
            wach = (insts + (w - 1) * trans) / (kernel_ms * 1e-3) / 1e12
            base[label] = round(wach / peak, 4)
        base["weighting"] = ("frac is the counter-exact SQ_INSTS_VALU issue; the weighted figures count each "
                             "SQ_INSTS_VALU_TRANS_F32 as 4 (probe) or 2 (guide) issue slots")
        base["valu_trans_per_launch"] = int(round(trans))
    if pm.get("lds_issue_frac") is not None and pm.get("kernel_trace_avg_ns"):
        base["lds_issue_frac"] = round(pm["lds_issue_frac"] * pm["kernel_trace_avg_ns"] * 1e-6 / kernel_ms, 4)
    if pm.get("lds_bank_conflict_share") is not None:
        base["lds_bank_conflict_share"] = pm["lds_bank_conflict_share"]
    return base


def gpu_ms_per_step(step, stream, reps=3, window_ms=20.0):
    """GPU time of one step: the median over reps of one HIP event pair around n back-to-back steps,
    n enough for a ~window_ms window (a pair around each single step would add its own cost)."""
    import torch
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    step()
    b.record(stream)
    torch.cuda.synchronize()
    n = max(1, int(math.ceil(window_ms / max(a.elapsed_time(b), 1e-3))))
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(n):
            step()
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b) / n)
    return float(np.median(ms))


def retime_step(step, stream, B, outs, reps=3, world=1):
    """Time another step function on the same batch; outputs checked against the timed step's."""
    import torch
    import torch.distributed as dist
    ref = [t.clone() for t in outs]
    step()
    k = gpu_ms_per_step(step, stream, reps)
    same = all(torch.equal(r, t) for r, t in zip(ref, outs))
    if world > 1:
        t = torch.tensor([k, 0.0 if same else 1.0], dtype=torch.float64, device=outs[0].device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        k, same = float(t[0]), float(t[1]) == 0.0
    return {"kernel_ms": round(k, 4), "syndromes_per_s": round(B * world / k * 1e3, 1), "identical": bool(same)}


def retime(dec, step, stream, B, outs, opts, reps=3, world=1):
    """Re-time the step with decoder options changed (e.g. hard_paths 0: every iteration in full
    arithmetic) and check the outputs are the same bits.  At N > 1 the kernel time is the max over
    ranks (as timed_steps) and the rate is the whole job's."""
    import torch
    import torch.distributed as dist
    ref = [t.clone() for t in outs]
    old = {k: dec.get_option(k) for k in opts}
    for k, v in opts.items():
        dec.set_option(k, v)
    try:
        step()
        k = gpu_ms_per_step(step, stream, reps)
    finally:
        for k_, v in old.items():
            dec.set_option(k_, v)
    same = all(torch.equal(r, t) for r, t in zip(ref, outs))
    if world > 1:
        t = torch.tensor([k, 0.0 if same else 1.0], dtype=torch.float64, device=outs[0].device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        k, same = float(t[0]), float(t[1]) == 0.0
    return {"kernel_ms": round(k, 4), "syndromes_per_s": round(B * world / k * 1e3, 1), "identical": bool(same)}


def phase_counts(dec, step, stream, its, B):
    """One launch of the instrumented kernel (QEC_OPT_PHASE_STATS): iters[] then packs, per
    sector, soft | hard << 8 | agreed << 16 | jumped << 24 iterations."""
    import torch
    try:
        dec.set_option("phase_stats", 1)
    except Exception as exc:  # noqa: BLE001
        return {"error": str(exc)}
    try:
        step()
        torch.cuda.synchronize()
        v = its.cpu().numpy().astype(np.int64)
    finally:
        dec.set_option("phase_stats", 0)
    out = {}
    for name, shift in (("soft", 0), ("hard", 8), ("agreed", 16), ("jumped", 24)):
        c = (v >> shift) & 0xFF
        out[name] = {"X": int(c[:, 0].sum()), "Z": int(c[:, 1].sum())}
    executed = sum(out[k]["X"] + out[k]["Z"] for k in ("soft", "hard", "agreed"))
    out["per_launch"] = {"syndromes": B, "sector_iterations_executed": executed,
                         "sector_iterations_nominal": executed + out["jumped"]["X"] + out["jumped"]["Z"]}
    step()  # restore the timed outputs
    torch.cuda.synchronize()
    return out


def sustained(step, stream, dev, world, ms_per_step, min_seconds, per_step_units):
    n = max(5, int(math.ceil(min_seconds * 1e3 / max(ms_per_step, 1e-3))))
    elapsed, _ = timed_steps(step, n, stream, dev, world)
    return {"steps": n, "seconds": round(elapsed, 3), "syndromes_per_s": round(per_step_units * n / elapsed, 1)}


def gather_measure(dec, step, rec, B, world, rank, dev, stream, steps, global_batch, backend, bound_into):
    """every rank's decision records (decoded straight into bit-packed form) are
    gathered to rank 0.  Timed alone, end to end serialised (decode, then gather, each step), and end to
    end overlapped (qec_ldpc_amd.gather.GatherPipeline: step k + 1 decodes into a second record buffer
    while step k's records are gathered on a communication stream, events only)."""
    import torch
    import torch.distributed as dist
    from qec_ldpc_amd.gather import GatherPipeline, gather_records
    gather_records(rec)  # warm-up (communicator set-up)
    torch.cuda.synchronize(dev)

    def timed(fn, n):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        return (time.perf_counter() - t0) / n

    g = timed(lambda: gather_records(rec), max(3, min(steps, 20)))

    def e2e():
        step()
        gather_records(rec)

    e = timed(e2e, steps)
    full = gather_records(rec)
    ok = True
    if rank == 0:
        ok = bool(torch.equal(full[:B], rec))
    pipe = GatherPipeline(tuple(rec.shape), dev)
    calls = [bound_into(pipe.bufs[0]), bound_into(pipe.bufs[1])]

    def decode(k, r, s):
        calls[k % 2]()

    pipe.run(decode, 2)  # warm-up
    o = timed(lambda: pipe.run(decode, steps), 1) / steps
    ok_o = True
    if rank == 0:  # every step decodes the same shard: the last gathered batch starts with rank 0's records
        ok_o = bool(torch.equal(pipe.outs[(steps - 1) % 2][:B].to(rec.device), rec))
    t = torch.tensor([g, e, o], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    g, e, o = float(t[0]), float(t[1]), float(t[2])
    nbytes = B * rec.shape[1]
    coll = "RCCL" if backend == "nccl" else backend
    rccl = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001
            rccl = None
    return {"backend": backend, "backend_reported": dist.get_backend(), "world_size": dist.get_world_size(),
            "rccl_version": rccl, "record_bytes": int(rec.shape[1]), "bytes_per_rank": int(nbytes),
            "gather_ms": round(g * 1e3, 4), "root_GBps": round(world * nbytes / g / 1e9, 2),
            "end_to_end": {"ms_per_step": round(e * 1e3, 4), "syndromes_per_s": round(global_batch / e, 1),
                           "what": "packed decode of every shard + %s gather of all records to rank 0" % coll},
            "end_to_end_overlapped": {
                "ms_per_step": round(o * 1e3, 4), "syndromes_per_s": round(global_batch / o, 1),
                "gather_bytes_per_step": int(world * nbytes),
                "what": "packed decode of step k + 1 overlapped with the %s gather of step k's records to rank 0 "
                        "(two record buffers, a communication stream, events only; qec_ldpc_amd.gather."
                        "GatherPipeline)" % coll,
                "rank0_last_step_intact": ok_o},
            "rank0_shard_intact": ok}


def ref_stop(dec, sX, sZ, p, iters, B, stream, world, fname, check):
    """the same resident batch under the reference stop rule (DecoderCPU::Decode
    unmodified, QEC_LDPC/DecoderCPU.h:280-291): rate, per-sector iteration histogram, and on rank 0
    the oracle's answers on a slice."""
    import torch
    import torch.distributed as dist
    rec = torch.empty((B, dec.record_bytes()), dtype=torch.uint8, device=sX.device)
    its = torch.empty((B, 2), dtype=torch.int32, device=sX.device)

    def step():
        dec.decode_batch_packed_dev(sX, sZ, p, iters, "ref", rec, its, stream=stream)

    step()
    torch.cuda.synchronize()
    k = gpu_ms_per_step(step, stream, 5)
    it = its.cpu().numpy()
    if world > 1:
        t = torch.tensor([k], dtype=torch.float64, device=sX.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        k = float(t[0])
    hist = {sec: {str(v): int(c) for v, c in enumerate(np.bincount(it[:, j])) if c}
            for j, sec in enumerate(("X", "Z"))}
    out = {"syndromes_per_s": round(B * world / k * 1e3, 1), "kernel_ms": round(k, 4), "cap": iters,
           "iterations_hist_rank0": hist, "mean_iterations": {"X": round(float(it[:, 0].mean()), 4),
                                                              "Z": round(float(it[:, 1].mean()), 4)}}
    if check:
        from oracle.oracle import OracleCode
        from qec_ldpc_amd.codes import code_path
        from qec_ldpc_amd.gather import unpack_records
        n = min(B, 4096)
        o = OracleCode(code_path(fname)).decode_batch(sX[:n].cpu().numpy(), sZ[:n].cpu().numpy(), p, iters, "ref")
        gX, gZ, gF = unpack_records(rec[:n].cpu().numpy(), dec.code.n)
        out["gpu_matches_oracle_on_sample"] = bool(np.array_equal(o[0], gX) and np.array_equal(o[1], gZ)
                                                   and np.array_equal(o[2], gF) and np.array_equal(o[3], it[:n]))
        out["oracle_sample"] = n
    return out


# The reference's published results blocks timed here (seed and counters from tests/golden/kat.json,
# extracted from QEC_LDPC/results/**): the P61 block of init.txt (code610, W=15, 100 000 samples,
# MAX 100, p 0.01: 112.73 s, results/[J=4,K=5,L=10,P=61,s=9,t=49][[n=610,k=61]]_W_15_MAX_100_p_0.01.txt:1-4)
# and the P7 W=3 MAX 100 p 0.02 block (results/[2,3,6,7,2,3]/..._W_3_MAX_100_p_0.02.txt:1-4).
PUBLISHED = [("J_4_K_5_L_10_P_61_s_9_t_49", 15, 100, 2287037912), ("J_3_K_3_L_6_P_7_s_2_t_3", 3, 100, 2596423950)]
KAT_FIELDS = {"tested": "numErrorsTested", "withX": "numXErrorsTested", "withZ": "numZErrorsTested",
              "corrected": "corrected", "synX": "syndromeErrorsX", "synZ": "syndromeErrorsZ",
              "logical": "logicalErrors", "convX": "convergenceFailX", "convZ": "convergenceFailZ"}


def published_blocks(device):
    """DecoderGPU::GetStatistics (QEC_LDPC/main.cu:101's call, the reference's seeded VS2015 sampler
    on the host, decode + I-P check on the GPU) on the published blocks: samples/s against the
    block's own Duration, every counter compared; one decoder and a two-part decoder on this GPU."""
    import qec_ldpc_amd as q
    from qec_ldpc_amd.codes import code_path
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        kat = json.load(f)
    out = []
    for fname, W, MAX, seed in PUBLISHED:
        rec = next(r for r in kat if r["code"] == fname and r["W"] == W and r["MAX"] == MAX and r["seed"] == seed)
        code = q.Quantum_LDPC_Code.createFromFile(code_path(fname))
        line = {"block": "%s block %d" % (rec["file"], rec["block"]), "W": W, "MAX": MAX, "p": rec["p_run"],
                "seed": seed, "samples": rec["tested"],
                "reference": {"seconds": rec["duration_us"] / 1e6,
                              "samples_per_s": round(rec["tested"] / (rec["duration_us"] / 1e6), 1),
                              "hardware": "Intel i7-4720HQ, 8 OpenMP threads (SURVEY.md section 6)"}}
        for label, devs in (("one_decoder", None), ("two_part_decoder", [device, device])):
            dec = q.DecoderGPU(code, device) if devs is None else q.DecoderGPU(code, devices=devs)
            dec.GetStatistics(W, 2000, rec["p_run"], MAX, seed)  # warm-up (workspace, code upload)
            t = time.perf_counter()
            st = dec.GetStatistics(W, rec["tested"], rec["p_run"], MAX, seed)
            dt = time.perf_counter() - t
            line[label] = {"seconds": round(dt, 4), "samples_per_s": round(rec["tested"] / dt, 1),
                           "vs_reference": round(rec["duration_us"] / 1e6 / dt, 1),
                           "counters_match": all(st[v] == rec[k] for k, v in KAT_FIELDS.items())}
            del dec
        out.append(line)
    return out


def host_threads():
    """OpenMP threads for the CPU baseline and where the number comes from: OMP_NUM_THREADS if set
    (the GPU box sets it to its CPU share), else the smaller of the CPU affinity set and the cgroup
    CPU quota; os.cpu_count() (the whole machine) is reported beside them."""
    env = os.environ.get("OMP_NUM_THREADS")
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    if env and env.isdigit() and int(env) > 0:
        n, src = int(env), "OMP_NUM_THREADS"
    else:
        n = max(1, min(aff, int(quota) if quota else aff))
        src = "cgroup cpu.max quota" if quota and int(quota) < aff else "CPU affinity set"
    return n, {"source": src, "OMP_NUM_THREADS": env, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
               "os_cpu_count": os.cpu_count()}


def cpu_baseline(code, fname, sX, sZ, p, iters, args, outs, packed):
    """Oracle (CPU restatement of DecoderCPU, one decoder per OpenMP thread) on a bounded sample of
    the same batch, all host threads and 1 thread; checks the GPU's answers on that sample; and
    BASELINE configs[0] (P7, 1k depolarising syndromes, 20 iterations) on all threads."""
    from oracle.oracle import OracleCode
    from qec_ldpc_amd.codes import P7, code_path
    from qec_ldpc_amd.gather import unpack_records
    import qec_ldpc_amd as q
    from qec_ldpc_amd.synthetic import depolarizing_errors
    threads, thread_source = host_threads()
    orc = OracleCode(code_path(fname))
    sX_h, sZ_h = sX.cpu().numpy(), sZ.cpu().numpy()

    def rate(nthreads, seconds, cap):
        probe = min(8 * nthreads, cap)
        t = time.perf_counter()
        orc.decode_batch(sX_h[:probe], sZ_h[:probe], p, iters, args.stop, nthreads=nthreads)
        r = probe / max(time.perf_counter() - t, 1e-9)
        n = int(min(cap, max(probe, r * seconds)))
        t = time.perf_counter()
        o = orc.decode_batch(sX_h[:n], sZ_h[:n], p, iters, args.stop, nthreads=nthreads)
        return n, time.perf_counter() - t, o

    n, dt, o = rate(threads, args.cpu_seconds, len(sX_h))
    if packed:
        gX, gZ, gF = unpack_records(outs[0][:n].cpu().numpy(), code.n)
    else:
        gX, gZ, gF = (t[:n].cpu().numpy() for t in outs[:3])
    same = np.array_equal(o[0], gX) and np.array_equal(o[1], gZ) and np.array_equal(o[2], gF)
    n1, dt1, _ = rate(1, max(2.0, args.cpu_seconds / 4), len(sX_h))
    # BASELINE configs[0]: P7, 1k depolarising syndromes (p = 0.02), 20 iterations, all threads
    c7 = q.Quantum_LDPC_Code.createFromFile(code_path(P7))
    x7, z7 = depolarizing_errors(c7.n, 0, 1000, 0.02)
    o7 = OracleCode(code_path(P7))
    s7 = (c7.syndrome(0, x7), c7.syndrome(1, z7))
    cfg0 = {}
    for stop in ("fixed", "ref"):
        t = time.perf_counter()
        reps = 0
        while time.perf_counter() - t < 1.0 or reps < 3:
            o7.decode_batch(s7[0], s7[1], 0.02, 20, stop, nthreads=threads)
            reps += 1
        cfg0[stop] = round(1000 * reps / (time.perf_counter() - t), 1)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(n / dt, 2), "unit": "syndromes/s", "cores": threads, "cores_source": thread_source,
            "kind": "port",
            "sample": "first %d syndromes of rank 0's batch, %s stop, %d iters (%.1f s)" % (n, args.stop, iters, dt),
            "cpu": cpu_model, "gpu_matches_oracle_on_sample": bool(same),
            "one_thread": {"value": round(n1 / dt1, 2), "sample": "first %d syndromes (%.1f s)" % (n1, dt1)},
            "configs0_p7_1k_20iters": {"fixed": cfg0["fixed"], "ref": cfg0["ref"], "unit": "syndromes/s",
                                       "cores": threads, "p": 0.02}}


if __name__ == "__main__":
    main()
