#!/usr/bin/env python3
"""Benchmark: timesteps/s of the RSW 2048² FilteredAB3 fp64 step (BASELINE.json
metric) on N MI355X, plus the roofline of the dominant kernel and the CPU
baseline (the oracle restatement, scipy.fft on the host cores).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode slab|ensemble] [--grid N]

Defaults: 200 untimed + 2000 timed steps (state resident in HBM).  When the
W untimed steps take less than --min-warmup-s (0.1 s) of stepping, more
untimed steps follow until they have (the GPU's steady state; the count is
reported as `warmup_extra_steps`); the K timed steps are exactly K.

N > 1: one process per GPU.  Started as `python bench.py --gpus N` (no
WORLD_SIZE in the environment) the script launches `torch.distributed.run
--nproc-per-node N` on itself as a child process, before any GPU call, and
exits with its status; the driver's own torch.distributed.run launch lands
directly in the rank code.
  --mode slab (default): ONE problem slab-decomposed over the N GPUs, the
      transposes as RCCL all-to-alls over xGMI; value = that
      problem's steps / max-over-ranks time; scaling "strong".
  --mode ensemble: every rank steps its own independent problem (the
      reference's job-array usage); value = all ranks' steps / time; "weak".
Extra keys on the same JSON line (never `value`):
  `ensemble` — the ensemble throughput of the same configuration on the N GPUs;
  `config5` — BASELINE config 5 (TwoLayerQG 8192² IFMRK4) decomposed over the
      N GPUs (one GPU at N = 1), steps/s (--no-config5 to skip);
  `config4` — BASELINE config 4 (RSW 4096² FilteredAB3) decomposed over
      min(N, 4) GPUs, as BASELINE names it ("across 4 MI355X"; one GPU at
      N = 1; at N = 8 ranks 4-7 only join the barriers), steps/s
      (--no-config4 to skip);
  `host_boundary` — one state download/upload through the C ABI over PCIe,
      and the rate with the driver's per-frame download;
  `comm` (N > 1, slab) — the exchange explained (sw_comm_profile): transport,
      RCCL rank count, schedule (pipelined / sequential, row chunks) and per
      rank the compute-stream µs per step spent waiting for transposes, the
      step's µs and the bytes sent per step (also in `config5` / `config4`);
  `kernels_cold`, `roofline.hbm_only` — the per-kernel table again with L2
      and the 256 MiB Infinity Cache evicted before every launch (libsw's
      SW_PROF_COLD), i.e. each kernel's inputs from HBM alone; the warm table
      (`kernels`, `roofline.achieved`) is the step as it runs, where a kernel
      reads part of what the previous one wrote from the Infinity Cache
      (--no-cold-profile to skip);
  `box` — the GPU box's state (tools/box_state.py, amdsmi in-process):
      product, serial, partition mode, power cap, clock ranges, and over each
      timed region the sampled gfx / memory clocks, socket power, hotspot and
      HBM temperatures, the energy-counter average power and the fraction of
      the region spent power- or thermally-limited — per rank at N > 1 —
      so a box-to-box swing can be attributed from the line itself;
  `roofline.traffic` — PMC bytes per launch of the dominant kernel from the
      newest round's profiles/rNN/traffic_<config>.json (`traffic_source`);
  `cpu_baseline` — rank 0 at N = 1 only.
"""
import argparse
import glob
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
CONFIG4_MAX_RANKS = 4  # BASELINE config 4: "RSW 4096² slab-decomposed across 4 MI355X"
SHORT = {'FilteredAB3': 'fab3', 'IFMAB3': 'ifmab3', 'IFMRK4': 'ifmrk4', 'ETDRK4': 'etdrk4',
         'FilteredRK4': 'frk4'}


# SURVEY §8(d) B_alg model (fp64): b_T = 16 Ns + 8 Np per logical 2D transform
def b_alg(model, stepper, n):
    Ns, Np = (n // 2 + 1) * n, n * n
    bT = 16 * Ns + 8 * Np
    if model == "rsw":
        return 13 * bT + (18 if stepper == "FilteredAB3" else 15) * 16 * Ns
    if model == "mlqg":
        # 4 calcN of 2-layer batched 3 c2r + 2 r2c (GF calcN_advection!) and
        # 4 FilteredRK4 stages of 4.25·2 state + 2 N fields
        return 4 * 10 * bT + 4 * (4.25 * 2 + 2) * 16 * Ns
    if model == "ty":
        # 4 calcN of 11 c2r + 13 r2c (thomasyamada/ThomasYamada.jl:129-262) and
        # 4 ETDRK4 stages of (3.75·4 state + 4 N) fields + 1.25 coefficient planes
        return 96 * bT + 4 * (4.75 * 4 + 1.25) * 16 * Ns
    if stepper == "IFMRK4":
        return 40 * bT + 30 * 16 * Ns
    return 10 * bT + 10 * 16 * Ns


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(model, stepper, n, grids=(128, 1024, 2048), samples=5, warm_steps=10, sample_s=1.0,
                 sample_steps=200):
    """The oracle — the fp64 numpy/scipy restatement of the reference op
    sequence, NOT FourierFlows/FFTW (Julia is absent) — on the host cores, by
    BASELINE.md §3's protocol: at each grid 10 untimed steps (past the AB3
    Euler start-up), then `samples` timed samples, each of 200 steps or as
    many as take >= 1 s, whichever comes first; the median.  About 20 s of
    CPU work in all (the 2048² samples are 3 steps of ≈ 0.45 s)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import statistics

    import sw_cases
    import sw_oracle as O

    affinity = len(os.sched_getaffinity(0))
    # the box's CPU share: the harness sets OMP_NUM_THREADS to it (16 per GPU);
    # sched_getaffinity shows the whole machine there
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cores = min(affinity, share) if share > 0 else affinity
    O.set_fft_workers(cores)
    grids = sorted(set(grids) | {n})
    by_grid = {}
    for g in grids:
        p = sw_cases.case_params(f"{model}_{SHORT[stepper]}", g)
        pr = sw_cases.oracle_problem(p)
        pr.set_solution(sw_cases.initial_condition(p, pr.grid))
        pr.stepforward(warm_steps)  # untimed
        rates, counts = [], []
        for _ in range(samples):
            k, t0 = 0, time.perf_counter()
            while k < sample_steps and time.perf_counter() - t0 < sample_s:
                pr.stepforward(1)
                k += 1
            rates.append(k / (time.perf_counter() - t0))
            counts.append(k)
        by_grid[str(g)] = {"steps_per_s": statistics.median(rates), "steps_per_sample": counts,
                           "warmup_steps": warm_steps, "samples": samples, "min": min(rates), "max": max(rates)}
    O.set_fft_workers(None)
    # BASELINE.md §3's optional extra: the reference's own CPU path if the box
    # has it (`julia -e 'using FourierFlows'`); recorded either way
    import shutil

    jl = shutil.which("julia")
    probe = "julia not on PATH: the reference's FourierFlows/FFTW path cannot run on this box"
    if jl:
        try:
            r = subprocess.run([jl, "-e", "using FourierFlows"], capture_output=True, text=True, timeout=120)
            probe = ("julia found, `using FourierFlows` succeeded (not timed by this script)" if r.returncode == 0
                     else f"julia found, `using FourierFlows` failed: {r.stderr.strip()[-200:]}")
        except Exception as exc:  # noqa: BLE001 - recorded
            probe = f"julia found, probe failed: {exc}"
    return dict(value=by_grid[str(n)]["steps_per_s"], unit="timesteps/s", cores=cores, kind="port",
                reference_probe=probe,
                nproc=os.cpu_count(), affinity_cores=affinity, cpu_model=_cpu_model(), by_grid=by_grid,
                sample=f"{stepper} steps of the {model.upper()} oracle: the repo's fp64 numpy/scipy restatement of "
                       f"the reference op sequence (numpy elementwise + scipy.fft workers={cores}), not "
                       f"FourierFlows/FFTW (Julia is not in the image); at {', '.join(f'{g}²' for g in grids)}: "
                       f"{warm_steps} untimed steps, then the median of {samples} samples of {sample_steps} steps "
                       f"or >= {sample_s:g} s each (BASELINE.md §3); value = the {n}² median")


def latest_traffic_file(model, n, stepper):
    """The newest round's PMC traffic file of this configuration
    (profiles/rNN/traffic_<model><n>_<stepper>.json, tools/profile_round.sh)."""
    def rnd(path):
        d = os.path.basename(os.path.dirname(path))
        return int(d[1:]) if d[1:].isdigit() else -1

    c = glob.glob(os.path.join(ROOT, "profiles", "r*", f"traffic_{model}{n}_{stepper}.json"))
    return max(c, key=rnd) if c else None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start torch.distributed.run on
    this script as a child (no exec, no GPU touched here) and return its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def make_problem(model, n, stepper, local, dec, over=None):
    from juliaraytracingsw_amd import drivers

    if model == "rsw":
        return drivers.rsw_problem(n, stepper, device=local, decomposition=dec, **(over or {}))
    if model == "ty":
        return drivers.ty_problem(n, device=local, decomposition=dec)
    if model == "mlqg":
        return drivers.mlqg_problem(n, device=local, decomposition=dec)
    return drivers.qg2_problem(n, stepper, device=local, decomposition=dec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    # (no option may be a prefix of a torch.distributed.run option: the ranks'
    # command line passes through its parser)
    ap.add_argument("--grid", dest="n", type=int, default=2048)
    ap.add_argument("--model", default="rsw", choices=["rsw", "qg2", "ty", "mlqg"])
    ap.add_argument("--stepper", default="FilteredAB3",
                    choices=["FilteredAB3", "IFMAB3", "IFMRK4", "ETDRK4", "FilteredRK4"])
    ap.add_argument("--profile-steps", type=int, default=50)
    ap.add_argument("--no-cold-profile", action="store_true",
                    help="skip the per-kernel table with caches evicted before each launch")
    ap.add_argument("--min-warmup-s", type=float, default=0.1,
                    help="untimed steps after the W warm-up steps until this much stepping has run (steady state)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config5", action="store_true")
    ap.add_argument("--config5-steps", type=int, default=20)
    ap.add_argument("--no-config4", action="store_true")
    ap.add_argument("--config4-steps", type=int, default=100)
    ap.add_argument("--mode", default="slab", choices=["ensemble", "slab"])
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic file for roofline.traffic (default: the newest profiles/rNN/ file of the "
                         "configuration)")
    ap.add_argument("--no-box-state", action="store_true", help="skip the amdsmi box-state record")
    ap.add_argument("--nutune", type=float, default=None,
                    help="RSW: override RSWParameters' νtune (FilteredAB3 below 2048² is linearly unstable at the "
                         "driver's νtune = 20, DESIGN §4; the kernels' work does not depend on it)")
    ap.add_argument("--cfltune", type=float, default=None, help="RSW: override RSWParameters' cfltune")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the rank plan (n_gpus, parallelism, scaling) and exit, touching no GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    # stdout carries exactly one line, the JSON result: everything else a
    # library prints there (Gloo's connection report, HIP/RCCL notices) goes
    # to stderr, the result through a duplicate of the original stdout
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    def emit(obj):
        result_out.write(json.dumps(obj) + "\n")
        result_out.flush()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; n_gpus = {world}", file=sys.stderr)
    slab = args.mode == "slab" and world > 1
    parallelism = (f"slab{world}" if slab else f"ensemble{world}") if world > 1 else "single-gpu"
    if args.dry_run:
        if rank == 0:
            emit({"n_gpus": world, "parallelism": parallelism,
                  "scaling": ("strong" if slab else "weak") if world > 1 else None, "rank0_of": world,
                  "config5_ranks": world, "config4_ranks": min(world, CONFIG4_MAX_RANKS)})
        return

    import torch

    dist = None
    # SW_BENCH_BACKEND=gloo: rehearse the N-rank path with several ranks
    # sharing the box's GPU and the host-staged slab transport (RCCL refuses
    # two ranks on one GPU); the driver's multi-GPU runs use the default,
    # RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("SW_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier_sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if backend == "gloo" else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    from juliaraytracingsw_amd import slab_comm

    monitor = None
    box_regions = {}
    if not args.no_box_state:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        try:
            import box_state

            monitor = box_state.BoxMonitor(local)
        except Exception as exc:  # noqa: BLE001 - the measurement never depends on it
            print(f"[bench] box state unavailable: {exc}", file=sys.stderr)
    box_static = monitor.static() if monitor is not None else None

    def comm_report(prob, nsteps=10):
        """sw_comm_profile on every rank of the problem (collective), gathered
        to every rank; prob None on a rank outside the problem"""
        if world == 1:
            return None
        st = prob.ctx.comm_profile(nsteps) if prob is not None else None
        # the link probe libsw ran at sw_create (per-peer GB/s, α, β, n½) and
        # the schedule it chose (VERDICT r05 #4b-c)
        lm = prob.ctx.link_model() if prob is not None else None
        per = [None] * world
        dist.all_gather_object(per, None if st is None else dict(
            rank=rank, exposed_transpose_us_per_step=st["exposed_transpose_us"], step_us=st["step_us"],
            sent_MB_per_step=st["sent_bytes_per_step"] / 1e6, peer_GBps=lm["peer_GBps"]))
        per = [r for r in per if r is not None]
        if st is None:
            return None
        ex = max(r["exposed_transpose_us_per_step"] for r in per)
        link = {k: lm[k] for k in ("probed", "transport", "latency_us", "GBps_per_peer_direction", "nhalf_bytes",
                                    "msg_bytes", "pipelined", "row_chunks")}
        return {"transport": st["transport"], "rccl_ranks": st["rccl_ranks"], "nranks": st["nranks"],
                "schedule": st["schedule"], "row_chunks": st["row_chunks"], "profiled_steps": nsteps,
                "exposed_transpose_us_per_step_max": ex,
                "exposed_fraction_of_step": ex / max(r["step_us"] for r in per), "link": link, "per_rank": per}

    def decomposition():
        if world == 1:
            return None
        if backend == "gloo":
            return slab_comm.host_decomposition(rank, world)
        return slab_comm.rccl_decomposition(rank, world)

    extra_warmup = {}

    def timed(prob, warmup, steps, tag="headline"):
        """max-over-ranks seconds of `steps` steps; prob None: a rank that
        only joins the barriers (config 4 on 4 of 8 GPUs)"""
        # W warm-up steps, then — if they took less than --min-warmup-s of
        # stepping — more untimed steps until they have: the GPU's clocks and
        # caches reach their steady state only after tens of ms of load (K =
        # 20, W = 5: 0.181 ms/step; W = 200: 0.167).  Every rank runs the same
        # number (the slab transposes are collective); the count is reported.
        barrier_sync()
        t0 = time.perf_counter()
        if prob is not None:
            prob.stepforward(warmup)
        barrier_sync()
        dt = max_over_ranks(time.perf_counter() - t0)
        extra = 0
        # the box monitor covers the extra warm-up and the timed steps (a
        # 20-step region alone is ~3 ms, one amdsmi sample): regions[tag] is
        # the whole window, tag_warmup and tag_timed its two parts
        if monitor is not None:
            monitor.start()
        if args.min_warmup_s > 0 and dt < args.min_warmup_s:
            per = dt / warmup if warmup > 0 else 1e-3
            extra = int(min(100000, math.ceil((args.min_warmup_s - dt) / max(per, 1e-6))))
            if prob is not None:
                prob.stepforward(extra)
        extra_warmup[tag] = extra
        barrier_sync()
        if monitor is not None:
            box_regions[tag + "_warmup"] = dict(monitor.lap(), steps=extra)
        t0 = time.perf_counter()
        if prob is not None:
            prob.stepforward(steps)  # sw_step returns when its stream is drained
        barrier_sync()
        el = time.perf_counter() - t0
        if monitor is not None:
            box_regions[tag + "_timed"] = dict(monitor.lap(), steps=steps)
            whole = monitor.stop(whole=True)
            n = extra + steps
            whole.update(steps=n, energy_J_per_step=(whole["energy_J"] / n if whole.get("energy_J") and n else None))
            box_regions[tag] = whole
        return max_over_ranks(el)

    over = {k: v for k, v in (("nutune", args.nutune), ("cfltune", args.cfltune)) if v is not None}
    if args.model == "ty":
        args.stepper = "ETDRK4"  # the only Thomas-Yamada stepper
    if args.model == "mlqg":
        args.stepper = "FilteredRK4"  # TwoLayerSimulation's stepper

    # headline: the configured problem, slab-decomposed over the N GPUs
    # (or one independent problem per GPU with --mode ensemble).  Should the
    # slab run fail on any rank (the RCCL transport first runs on the
    # driver's multi-GPU node), every rank falls back to the ensemble
    # headline, labelled as such, with the error in "slab_error".
    slab_error = None
    if slab:
        # every rank passes each stage's agreement point (an all-reduce of
        # the failure flag) before the next collective, so a failure on one
        # rank cannot leave the others waiting in a transpose
        prob = None

        def stage(fn):
            nonlocal slab_error
            if slab_error is None:
                try:
                    fn()
                except Exception as exc:  # noqa: BLE001 - reported in the JSON line
                    slab_error = f"{type(exc).__name__}: {exc}"
            return max_over_ranks(1.0 if slab_error else 0.0) == 0

        box = {}

        def create():
            dec = decomposition()  # collective: the RCCL unique id broadcast
            # test hook of the fallback path: every rank fails its slab problem,
            # as an RCCL communicator that cannot be created fails on every rank
            if os.environ.get("SW_BENCH_FAIL_SLAB") == "1":
                raise RuntimeError("SW_BENCH_FAIL_SLAB")
            box["prob"], box["P"] = make_problem(args.model, args.n, args.stepper, local, dec, over)

        if stage(create) and stage(lambda: box.__setitem__("t", timed(box["prob"], args.warmup, args.steps))):
            prob, P, elapsed = box["prob"], box["P"], box["t"]
        else:
            print(f"[bench] slab headline failed ({slab_error or 'on another rank'}); "
                  "reporting the ensemble", file=sys.stderr)
            slab_error = slab_error or "failed on another rank"
            slab = False
            parallelism = f"ensemble{world}"
            if "prob" in box:
                try:
                    box["prob"].close()
                except Exception:  # noqa: BLE001
                    pass
    if not slab:
        prob, P = make_problem(args.model, args.n, args.stepper, local, None, over)
        elapsed = timed(prob, args.warmup, args.steps)

    comm = comm_report(prob) if slab else None
    # roofline: per-kernel HIP-event durations on libsw's stream
    stats = prob.ctx.profile(args.profile_steps)
    # the same kernels with L2 and the 256 MiB Infinity Cache evicted before
    # each launch (SW_PROF_COLD): every input from HBM.  In the step a kernel
    # reads what the previous one wrote, partly from the Infinity Cache, so
    # the warm table above is the step's rate and this one the HBM-only rate
    stats_cold = None
    if not args.no_cold_profile:
        os.environ["SW_PROF_COLD"] = "1"
        try:
            stats_cold = prob.ctx.profile(max(3, args.profile_steps // 5))
        finally:
            os.environ.pop("SW_PROF_COLD", None)
            prob.ctx.profile(1)  # (frees the eviction buffer)
    step_alg = prob.ctx.step_alg_bytes()
    # the boundary's host-buffer cost: one state download and
    # upload through the C ABI, i.e. over PCIe (after the timed region)
    tg, tu = [], []
    st = prob.ctx.get_state()  # the caller's prob.sol buffer, reused per frame
    for _ in range(3):
        t0 = time.perf_counter()
        prob.ctx.get_state(out=st)
        tg.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        prob.ctx.set_state(st)
        tu.append(time.perf_counter() - t0)
    prob.close()
    del prob

    # extra: the ensemble throughput of the same configuration (N > 1)
    ensemble = None
    if slab:
        e, _ = make_problem(args.model, args.n, args.stepper, local, None)
        k = max(1, args.steps // 4)
        te = timed(e, min(args.warmup, 50), k, "ensemble")
        ensemble = {"value": world * k / te, "unit": "timesteps/s", "steps_per_rank": k,
                    "scaling": "weak", "workload": f"{world} independent {args.model.upper()} {args.n}^2 "
                                                  f"{args.stepper} problems, one per GPU"}
        e.close()
        del e

    # extras: BASELINE configs 5 (TwoLayerQG 8192² IFMRK4) and 4 (RSW 4096²
    # FilteredAB3), each one problem slab-decomposed over the N GPUs (one GPU
    # at N = 1)
    def extra_config(model, n, stepper, steps, warmup, label, max_ranks=None):
        """one problem slab-decomposed over min(world, max_ranks) GPUs (ranks
        [0, used)); the other ranks only join the barriers"""
        used = world if max_ranks is None else min(world, max_ranks)
        active = rank < used
        dec = None
        if world > 1:
            if backend == "gloo":
                # the host-staged all-to-all runs over a group of the used ranks
                # (new_group is collective on every rank)
                grp = dist.new_group(ranks=list(range(used))) if used < world else None
                dec = slab_comm.host_decomposition(rank, used, grp) if active and used > 1 else None
            else:
                dec = slab_comm.rccl_decomposition(rank, world, used)
                if used == 1:
                    dec = None
        ex = make_problem(model, n, stepper, local, dec)[0] if active else None
        te = timed(ex, warmup, steps, label)
        cx = comm_report(ex, 3) if used > 1 else None
        sx = ex.ctx.profile(3) if active else []
        if ex is not None:
            ex.close()
        del ex
        return {"value": steps / te, "unit": "timesteps/s", "n_gpus": used, "steps": steps,
                "ms_per_step": te / steps * 1e3, "scaling": "strong" if used > 1 else None,
                "ranks_idle": world - used,
                "workload": f"{label} fp64, " + (f"slab{used}" if used > 1 else "single-gpu"),
                "kernels": [{"name": s["name"], "avg_us": s["avg_ms"] * 1e3, "per_step": s["launches"] / 3}
                            for s in sx], "comm": cx}

    headline_cfg = (args.model, args.n, args.stepper) == ("rsw", 2048, "FilteredAB3")
    config5 = config4 = None
    if not args.no_config5 and not slab_error and headline_cfg:
        config5 = extra_config("qg2", 8192, "IFMRK4", args.config5_steps, 3,
                               "TwoLayerQG 8192^2 IFMRK4 (BASELINE config 5)")
    if not args.no_config4 and not slab_error and headline_cfg:
        config4 = extra_config("rsw", 4096, "FilteredAB3", args.config4_steps, 20,
                               "RSW 4096^2 FilteredAB3 (BASELINE config 4)", CONFIG4_MAX_RANKS)

    box = None
    if monitor is not None:
        mine = {"rank": rank, "static": box_static, "regions": box_regions}
        if dist is not None:
            per = [None] * world
            dist.all_gather_object(per, mine)
        else:
            per = [mine]
        box = {"source": "amdsmi in-process (tools/box_state.py)", "per_rank": per}

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    kern = [s for s in stats if s["name"] != "transpose"]
    dom = max(kern, key=lambda s: s["avg_ms"] * s["launches"])
    achieved = dom["alg_bytes"] / (dom["avg_ms"] * 1e-3) / 1e9
    dom_cold = next((s for s in stats_cold or [] if s["name"] == dom["name"]), None)
    achieved_cold = dom_cold["alg_bytes"] / (dom_cold["avg_ms"] * 1e-3) / 1e9 if dom_cold else None
    traffic = None
    traffic_src = args.traffic_json or latest_traffic_file(args.model, args.n, args.stepper)
    try:
        tj = json.load(open(traffic_src))
        if tj.get("config") == f"{args.model}{args.n}_{args.stepper}" and world == 1:
            traffic = tj["kernels"].get(dom["name"])
    except Exception:
        traffic = None
    if traffic is None:
        traffic_src = None
    for s in stats:
        gbps = s["alg_bytes"] / (s["avg_ms"] * 1e-3) / 1e9
        print(f"[bench] {s['name']:>10s}: {s['avg_ms'] * 1e3:8.1f} us/launch  x{s['launches'] / args.profile_steps:.0f}/step"
              f"  alg {s['alg_bytes'] / 1e6:7.1f} MB  -> {gbps:7.0f} GB/s ({gbps / HBM_PEAK_GBPS:.1%} of HBM peak)",
              file=sys.stderr)

    ms_per_step = elapsed / args.steps * 1e3
    value = (1 if slab else world) * args.steps / elapsed
    balg = b_alg(args.model, args.stepper, args.n)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.model, args.stepper, args.n)
    metric = f"timesteps/sec, {args.model.upper()} {args.n}^2 {args.stepper} fp64"
    if (args.model, args.n, args.stepper) == ("rsw", 2048, "FilteredAB3"):
        try:  # the BASELINE.json metric this default configuration measures
            metric = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
        except Exception:
            pass
    per_gpu_rate = value / world if slab else args.steps / elapsed
    out = {
        "metric": metric,
        "value": value,
        "unit": "timesteps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_extra_steps": extra_warmup.get("headline", 0),
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        # fixed per-GPU work (ensemble) is weak scaling, one problem over N
        # GPUs strong; a single GPU scales neither way
        "scaling": ("strong" if slab else "weak") if world > 1 else None,
        "vs_baseline": None,
        "dtype": "f64",
        "data": {"rsw": "synthetic random-phase IC (set_shafer_initial_condition!, seeded)",
                 "qg2": "synthetic randn PV IC (set_seed_initial_condition!, seeded)",
                 "ty": "synthetic random-phase IC (TYdriver set_initial_condition, seeded)",
                 "mlqg": "synthetic filtered randn PV IC (TwoLayerSimulation, seeded)"}[args.model],
        "config": {"workload": f"{args.model.upper()} {args.n}^2 {args.stepper} fp64 step, dt={P['dt']:.6g}"
                               + (f" ({', '.join(f'{k}={v:g}' for k, v in over.items())})" if over else ""),
                   "grid": args.n,
                   "parallelism": parallelism},
        # bytes the libsw kernels move per step (live modes only, physical
        # space never in HBM) and the resulting HBM rate per GPU
        "libsw_alg_bytes_per_step": step_alg,
        "libsw_alg_GBps_per_gpu": step_alg * per_gpu_rate / 1e9,
        # SURVEY §8(d)'s byte model of a full-array FFT implementation (13
        # full transforms + 18 state passes per RSW step): bytes libsw does
        # NOT move; the rate is an equivalence, not a measured bandwidth
        "reference_byte_model": {"bytes_per_step": balg, "equivalent_GBps_per_gpu": balg * per_gpu_rate / 1e9},
        "roofline": {"bound": "hbm", "kernel": dom["name"], "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "traffic_source": None if traffic_src is None else os.path.relpath(traffic_src, ROOT),
                     "alg_bytes_per_launch": dom["alg_bytes"], "avg_us_per_launch": dom["avg_ms"] * 1e3,
                     # in the step some of its input comes from the Infinity
                     # Cache; with L2 and that cache evicted before the launch
                     # (SW_PROF_COLD) every byte comes from HBM:
                     "hbm_only": None if dom_cold is None else {
                         "achieved": achieved_cold, "frac": achieved_cold / HBM_PEAK_GBPS,
                         "avg_us_per_launch": dom_cold["avg_ms"] * 1e3}},
        "kernels": [{"name": s["name"], "avg_us": s["avg_ms"] * 1e3, "per_step": s["launches"] / args.profile_steps,
                     "alg_bytes": s["alg_bytes"]} for s in stats],
        "kernels_cold": None if stats_cold is None else [
            {"name": s["name"], "avg_us": s["avg_ms"] * 1e3, "alg_bytes": s["alg_bytes"]} for s in stats_cold],
        "ensemble": ensemble,
        "slab_error": slab_error,
        "comm": comm,
        "config5": config5,
        "config4": config4,
        "cpu_baseline": cpu,
        "box": box,
        # RSWDriver saves a frame every output_freq = floor(output_dt/dt) steps
        # (rsw/RSWDriver.jl:152, output_dt = 0.025/f): 81 steps at 2048²
        "host_boundary": {"state_bytes": int(st.nbytes), "get_state_ms": min(tg) * 1e3,
                          "set_state_ms": min(tu) * 1e3,
                          "steps_per_s_with_state_download_every_81_steps":
                              81 / (81 * ms_per_step * 1e-3 + min(tg))},
    }
    emit(out)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
