#!/usr/bin/env python3
"""Benchmark: timesteps/s of the RSW 2048² FilteredAB3 fp64 step (BASELINE.json
metric) on N MI355X, plus the roofline of the dominant kernel and the CPU
baseline (the oracle restatement, scipy.fft on the host cores).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode ensemble|slab]

Defaults: 200 untimed + 2000 timed steps (state resident in HBM).  Also
reported, never in `value`: `host_boundary` (one state download/upload
through the C ABI, over PCIe, and the rate with the driver's per-frame
download).

N > 1 is launched by torch.distributed.run, one process per GPU.
  --mode ensemble (default): every rank steps its own independent 2048²
      problem (an ensemble of seeded runs, the reference's job-array usage);
      no collective on the data path; value = all ranks' steps / max-over-ranks
      time; scaling "weak".
  --mode slab: ONE problem slab-decomposed over the N GPUs, transposes as RCCL
      all-to-alls; value = that problem's steps / time; scaling
      "strong".  Meant for the large configurations (4096², 8192²): at 2048²
      the transposes cost more than the step.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

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


def cpu_baseline(model, stepper, n, budget_s=20.0, max_steps=20):
    """Time the oracle (fp64 numpy/scipy restatement) on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import sw_cases
    import sw_oracle as O

    cores = min(16, len(os.sched_getaffinity(0)))
    O.set_fft_workers(cores)
    short = {'FilteredAB3': 'fab3', 'IFMAB3': 'ifmab3', 'IFMRK4': 'ifmrk4', 'ETDRK4': 'etdrk4',
             'FilteredRK4': 'frk4'}[stepper]
    p = sw_cases.case_params(f"{model}_{short}", n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    pr.stepforward(3)  # the Euler start-up steps (AB3 steppers), untimed
    t0 = time.perf_counter()
    k = 0
    while k < max_steps and (time.perf_counter() - t0) < budget_s:
        pr.stepforward(1)
        k += 1
    dt = time.perf_counter() - t0
    O.set_fft_workers(None)
    return dict(value=k / dt, unit="timesteps/s", cores=cores, kind="port",
                sample=f"{k} {stepper} steps of the {n}² oracle restatement (numpy elementwise + scipy.fft "
                       f"workers={cores}) after 3 untimed steps")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--model", default="rsw", choices=["rsw", "qg2", "ty", "mlqg"])
    ap.add_argument("--stepper", default="FilteredAB3",
                    choices=["FilteredAB3", "IFMAB3", "IFMRK4", "ETDRK4", "FilteredRK4"])
    ap.add_argument("--profile-steps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default="ensemble", choices=["ensemble", "slab"])
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_rsw2048_fab3.json"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    # SW_BENCH_BACKEND=gloo: rehearse the N-rank ensemble path with several
    # ranks sharing the box's GPUs (RCCL refuses two ranks on one GPU); the
    # driver's multi-GPU runs use the default, RCCL ("nccl"), one GPU per rank
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

    from juliaraytracingsw_amd import drivers, slab_comm

    slab = args.mode == "slab" and world > 1
    dec = slab_comm.rccl_decomposition(rank, world) if slab else None
    if args.model == "ty":
        args.stepper = "ETDRK4"  # the only Thomas-Yamada stepper
    if args.model == "mlqg":
        args.stepper = "FilteredRK4"  # TwoLayerSimulation's stepper
    if args.model == "rsw":
        prob, P = drivers.rsw_problem(args.n, args.stepper, device=local, decomposition=dec)
    elif args.model == "ty":
        prob, P = drivers.ty_problem(args.n, device=local, decomposition=dec)
    elif args.model == "mlqg":
        prob, P = drivers.mlqg_problem(args.n, device=local, decomposition=dec)
    else:
        prob, P = drivers.qg2_problem(args.n, args.stepper, device=local, decomposition=dec)

    prob.stepforward(args.warmup)
    barrier_sync()
    t0 = time.perf_counter()
    prob.stepforward(args.steps)  # sw_step returns when its stream is drained
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # roofline: per-kernel HIP-event durations on libsw's stream
    stats = prob.ctx.profile(args.profile_steps)
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

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    dom = max(stats, key=lambda s: s["avg_ms"] * s["launches"])
    achieved = dom["alg_bytes"] / (dom["avg_ms"] * 1e-3) / 1e9
    traffic = None
    try:
        tj = json.load(open(args.traffic_json))
        if tj.get("config") == f"{args.model}{args.n}_{args.stepper}":
            traffic = tj["kernels"].get(dom["name"])
    except Exception:
        traffic = None
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
    out = {
        "metric": metric,
        "value": value,
        "unit": "timesteps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if slab else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": {"rsw": "synthetic random-phase IC (set_shafer_initial_condition!, seeded)",
                 "qg2": "synthetic randn PV IC (set_seed_initial_condition!, seeded)",
                 "ty": "synthetic random-phase IC (TYdriver set_initial_condition, seeded)",
                 "mlqg": "synthetic filtered randn PV IC (TwoLayerSimulation, seeded)"}[args.model],
        "config": {"workload": f"{args.model.upper()} {args.n}^2 {args.stepper} fp64 step, dt={P['dt']:.6g}",
                   "grid": args.n,
                   "parallelism": (f"slab{world}" if slab else f"ensemble{world}") if world > 1 else "single-gpu"},
        "b_alg_bytes_per_step": balg,
        "b_alg_GBps": balg * value / world / 1e9,  # per GPU
        "b_alg_frac_of_peak": balg * value / world / 1e9 / HBM_PEAK_GBPS,
        "libsw_alg_bytes_per_step": step_alg,
        "roofline": {"bound": "hbm", "kernel": dom["name"], "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "alg_bytes_per_launch": dom["alg_bytes"], "avg_us_per_launch": dom["avg_ms"] * 1e3},
        "kernels": [{"name": s["name"], "avg_us": s["avg_ms"] * 1e3, "per_step": s["launches"] / args.profile_steps,
                     "alg_bytes": s["alg_bytes"]} for s in stats],
        "cpu_baseline": cpu,
        # RSWDriver saves a frame every output_freq = floor(output_dt/dt) steps
        # (rsw/RSWDriver.jl:152, output_dt = 0.025/f): 81 steps at 2048²
        "host_boundary": {"state_bytes": int(st.nbytes), "get_state_ms": min(tg) * 1e3,
                          "set_state_ms": min(tu) * 1e3,
                          "steps_per_s_with_state_download_every_81_steps":
                              81 / (81 * ms_per_step * 1e-3 + min(tg))},
    }
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
