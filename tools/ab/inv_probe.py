"""RSW 2048² calcN against the oracle mode by mode (the η invariant probe)."""
import sys
sys.path[:0] = ['tests', 'oracle', '.']
import numpy as np
import invariants as I, sw_oracle as O, sw_cases
O.set_fft_workers(16)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
g = O.TwoDGrid(n); s = I.rsw_state(g, n + 1); p = sw_cases.case_params("rsw_fab3", n)
No = O.rsw_calcN(s.copy(), g, O.RSWParams(p["nu"], p["nnu"], p["f"], p["Cg"]))
prob = sw_cases.libsw_problem(p)
Ng = prob.calcN(s)
prob.close()
print("gpu", I.rsw_residuals(g, s, Ng)); print("oracle", I.rsw_residuals(g, s, No))
live = g.dealias(np.ones(Ng.shape[1:], complex)) != 0
for f in range(3):
    d = np.where(live, np.abs(Ng[f] - No[f]), 0); sc = np.max(np.abs(np.where(live, No[f], 0)))
    idx = np.argsort(d.ravel())[::-1][:12]
    print(f"field {f}: max|d|/max|N| = {d.max() / sc:.3e}, median {np.median(d[live]) / sc:.3e}")
    for i in idx:
        j, k = np.unravel_index(i, d.shape)
        print(f"   l-row {j:5d} kr {k:5d}  |d|/max {d[j, k] / sc:.3e}  |N| {abs(No[f][j, k]) / sc:.3e}  gpu {Ng[f][j, k]:.6e} or {No[f][j, k]:.6e}")
