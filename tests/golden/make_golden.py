"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

Fixtures hold data only: the seeded initial condition, the first calcN output
N(sol0) and the dealiased state after 1, 10 and 100 steps (32²), plus 10
steps at 64².  The reference itself cannot run in this container (no Julia /
FourierFlows / FFTW), so these vectors come from the oracle
restatement, which tests/test_oracle.py pins to the reference's known answers.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))

import sw_cases  # noqa: E402


def make(name, n, steps):
    p = sw_cases.case_params(name, n)
    pr = sw_cases.oracle_problem(p)
    ic = sw_cases.initial_condition(p, pr.grid)
    pr.set_solution(ic)
    out = {"params": np.array(json.dumps(p)), "ic": pr.sol.copy()}
    out["N0"] = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    done = 0
    for s in steps:
        pr.stepforward(s - done)
        done = s
        out[f"sol{s}"] = pr.grid.dealias(pr.sol.copy())
    fn = os.path.join(HERE, f"{name}_{n}.npz")
    np.savez_compressed(fn, **out)
    return fn


if __name__ == "__main__":
    only = sys.argv[1:]  # optional case names
    for name in sw_cases.ALL_CASES:
        if only and name not in only:
            continue
        print(make(name, 32, [1, 10, 100]))
        print(make(name, 64, [10]))
