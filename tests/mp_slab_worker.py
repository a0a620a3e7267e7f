"""Worker for tests/test_gpu_multiprocess.py (launched by torch.distributed.run).

Every rank holds one slab of the problem in its own process and its own libsw
context on the same GPU; the transposes go through the host-staged transport
hook over gloo (RCCL refuses several ranks on one GPU).  Rank 0 also runs the
undecomposed problem and checks the gathered state, calcN, physical fields
and energies against it."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE, os.path.join(os.path.dirname(HERE), "oracle")]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="rsw_fab3")
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--freq", type=int, default=2)
    ap.add_argument("--out", required=True)
    ap.add_argument("--aliased", action="store_true", help="aliased_state: the full (nkr, nl) array")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import sw_cases
    import sw_oracle as O
    from juliaraytracingsw_amd import multilayer_qg as MLQG, rotating_shallow_water as RSW, slab_comm
    from juliaraytracingsw_amd import two_layer_qg as QG2

    M = RSW if a.case.startswith("rsw") else MLQG if a.case.startswith("mlqg") else QG2
    p = sw_cases.case_params(a.case, a.n)
    grid = O.TwoDGrid(a.n, aliased_fraction=p.get("af", 1 / 3))

    def energies(pb):  # (ΣKE, PE) of the model's energy functions
        if M is MLQG:
            (k1, k2), (pe,) = MLQG.energies(pb)
            return k1 + k2, pe
        return np.sum(M.kinetic_energy(pb)), M.potential_energy(pb)
    ic = sw_cases.initial_condition(p, grid)
    kw = dict(aliased_state=True) if a.aliased else {}
    prob = sw_cases.libsw_problem(p, decomposition=slab_comm.host_decomposition(rank, world), **kw)
    prob.sol = ic
    N = prob.calcN(ic)
    cap = a.steps // a.freq + 1
    prob.ctx.set_energy_diagnostics(a.freq, cap)
    half = a.steps // 2
    prob.stepforward(half)
    mid = prob.ctx.energy_diagnostics()  # gathered once; the rest incrementally below
    prob.stepforward(a.steps - half)
    sol = prob.sol
    # (energies of prob.sol before updatevars!, which dealiases it: with
    # aliased_state they include the aliased modes)
    ke, pe = energies(prob)
    phys = M.updatevars(prob)
    recs, cfl = prob.ctx.energy_diagnostics(), M.cfl(prob)
    res = {}
    if rank == 0:
        ref = sw_cases.libsw_problem(p, **kw)
        ref.sol = ic
        Nr = ref.calcN(ic)
        ref.ctx.set_energy_diagnostics(a.freq, cap)
        ref.stepforward(a.steps)
        rsol = ref.sol
        rke, rpe = energies(ref)
        pr = M.updatevars(ref)
        res = dict(
            state_equal=bool(np.array_equal(sol, rsol)),
            calcN_equal=bool(np.array_equal(N, Nr)),
            physical_equal=bool(all(np.array_equal(phys[k], pr[k]) for k in pr)),
            ke_rel=abs(ke / rke - 1),
            pe_rel=abs(pe / rpe - 1),
            records_equal=bool(recs == ref.ctx.energy_diagnostics() and len(recs) == a.steps // a.freq
                               and mid == recs[:len(mid)] and len(mid) == half // a.freq),
            n_records=len(recs),
            cfl_equal=bool(cfl == M.cfl(ref)),
            world=world,
            # the largest aliased mode of the state (aliased_state: nonzero)
            aliased_max=float(np.max(np.abs(np.where(grid.dealias(np.ones_like(sol)) == 0, sol, 0)))),
        )
        ref.close()
        res["link"] = prob.ctx.link_model()  # the probe of sw_create (host-staged here)
    prob.close()
    dist.barrier()
    if rank == 0:
        with open(a.out, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
