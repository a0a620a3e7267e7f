"""Debug helper: compare fused / unfused / repeated runs of one case bitwise."""
import os
import sys

sys.path[:0] = ['.', 'tests', 'oracle']
import numpy as np  # noqa: E402

import sw_cases  # noqa: E402


def run(name, fused, n=128, steps=2):
    p = sw_cases.case_params(name, n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    if fused:
        os.environ['SW_FUSE_ALL'] = '1'
    a = sw_cases.libsw_problem(p, unfused=not fused)
    os.environ.pop('SW_FUSE_ALL', None)
    a.sol = pr.sol
    out = []
    for _ in range(steps):
        a.stepforward(1)
        out.append(a.sol)
    a.close()
    return out


for name in sys.argv[1:] or ['qg2_ifmrk4']:
    f1, f2, u1, u2 = run(name, True), run(name, True), run(name, False), run(name, False)
    for i in range(len(f1)):
        print(name, i, 'ff', np.abs(f1[i] - f2[i]).max(), 'uu', np.abs(u1[i] - u2[i]).max(),
              'fu', np.abs(f1[i] - u1[i]).max())
