"""sha256 of the RSW 2048² FilteredAB3 state after N steps from the driver IC
(the A/B scripts compare variant builds bitwise: LIBSW_PATH=… python
tools/state_hash.py [N] [grid])."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from juliaraytracingsw_amd import drivers  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
grid = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
prob, _ = drivers.rsw_problem(grid, "FilteredAB3")
prob.stepforward(n)
print(os.path.basename(os.environ.get("LIBSW_PATH", "libsw.so")), n, hashlib.sha256(prob.sol.tobytes()).hexdigest()[:16])
prob.close()
