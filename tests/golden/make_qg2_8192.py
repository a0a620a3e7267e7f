"""Oracle reference for BASELINE config 5 at full size:
TwoLayerQG 8192² IFMRK4 from the seeded driver IC (sw_cases "qg2_ifmrk4",
swqg/TwoLayerDriver.jl:10-15 amplitude 1e-2), two full IFMRK4 steps of the
oracle (utils/IFMRK4.jl:157-163 as SURVEY A9 defines it, swqg/TwoLayerQG.jl
:152-198 calcN and L), with the 2×2 integrating factors from scipy's expm on
every live mode (round 5, VERDICT r04 weak #1: independent of the device's
closed-form ExpOf; forked worker processes, sw_oracle.set_expm_workers; the
round-4 fixture used the closed form sw_oracle.expm_2x2, which
tests/test_oracle.py pins to scipy on these rows).

    python tests/golden/make_qg2_8192.py        (≈ 8 min, ≈ 30 GB, 8 cores)

The state is 1.07 GB, so the fixture keeps a sample: every live kr of 24 l
rows (low, middle, high, negative), both layers, after 2 steps; the full
state's per-layer sums of |q̂|²; a check of the same rows of the seeded IC
(sum of |q̂|², a seeded projection, max) so the test knows it regenerated
the same IC; and the size of the nonlinear part of the sample (its
distance from the linear-only propagation exp(2 dt L)·sol0).  tests/test_gpu_large.py compares libsw (one slab and eight) with
it.  Data only: no reference source.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))

import sw_cases  # noqa: E402
import sw_oracle as O  # noqa: E402

N = 8192
STEPS = 2
ROWS = [0, 1, 2, 3, 5, 8, 13, 34, 89, 233, 610, 1597, 2000, 2500, 2729,
        N - 1, N - 2, N - 7, N - 55, N - 377, N - 987, N - 1900, N - 2600, N - 2729]


def main():
    t0 = time.time()
    O.set_fft_workers(os.cpu_count())
    O.set_expm_workers(os.cpu_count())
    p = sw_cases.case_params("qg2_ifmrk4", N)
    pr = sw_cases.oracle_problem(p, expm="scipy")
    g = pr.grid
    ic = sw_cases.initial_condition(p, g)
    pr.set_solution(ic)
    kc = int(np.count_nonzero(g.dealias(np.ones((1, 1, g.nkr), np.complex128))[0, 0]))
    rows = np.array(ROWS)
    s0 = pr.sol[:, rows, :kc].copy()
    lin = O.mvmul(O.expm_2x2(pr.L[rows] * (STEPS * p["dt"])), pr.sol[:, rows])[:, :, :kc]
    print(f"setup {time.time() - t0:.0f} s", flush=True)
    for s in range(STEPS):
        pr.stepforward(1)
        print(f"step {s + 1} {time.time() - t0:.0f} s", flush=True)
    sol = g.dealias(pr.sol.copy())
    srows = sol[:, rows, :kc]
    out = {"params": np.array(json.dumps(p)), "rows": rows, "kc": np.array(kc), "steps": np.array(STEPS),
           "expm": np.array(pr.ts.expm),
           "sol_rows": srows, "sumsq": np.array([float(np.sum(np.abs(sol[f]) ** 2)) for f in range(2)]),
           "ic_check": ic_check(s0),
           "nonlinear_part": np.array(np.max(np.abs(srows - lin)) / np.max(np.abs(srows)))}
    fn = os.path.join(HERE, f"qg2_ifmrk4_{N}_rows.npz")
    np.savez_compressed(fn, **out)
    print(f"wrote {fn}; nonlinear part of the sample: {float(out['nonlinear_part']):.2e} of its max; "
          f"{time.time() - t0:.0f} s")


def ic_check(ic_rows):
    """sum |q̂|², a seeded projection (re, im) and the max of the IC sample"""
    w = np.random.default_rng(99).standard_normal(ic_rows.shape)
    z = np.sum(ic_rows * w)
    return np.array([np.sum(np.abs(ic_rows) ** 2), z.real, z.imag, np.max(np.abs(ic_rows))])


if __name__ == "__main__":
    main()
