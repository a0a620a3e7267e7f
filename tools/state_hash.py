"""sha256 of a problem's state after N steps from its driver IC (the A/B
scripts compare variant builds bitwise: LIBSW_PATH=… python
tools/state_hash.py [N] [grid] [model] [stepper]; default RSW 2048²
FilteredAB3)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from juliaraytracingsw_amd import drivers  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
grid = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
model = sys.argv[3] if len(sys.argv) > 3 else "rsw"
stepper = sys.argv[4] if len(sys.argv) > 4 else "FilteredAB3"
if model == "rsw":
    prob, _ = drivers.rsw_problem(grid, stepper)
elif model == "qg2":
    prob, _ = drivers.qg2_problem(grid, stepper)
elif model == "mlqg":
    prob, _ = drivers.mlqg_problem(grid)
else:
    prob, _ = drivers.ty_problem(grid)
prob.stepforward(n)
print(os.path.basename(os.environ.get("LIBSW_PATH", "libsw.so")), model, grid, stepper, n,
      hashlib.sha256(prob.sol.tobytes()).hexdigest()[:16])
prob.close()
