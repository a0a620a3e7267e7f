"""CPU test of bench.py's N-rank launch: `bench.py --gpus N`
without a launcher starts torch.distributed.run on itself as a child, and the
ranks report n_gpus = N with the slab-decomposed (strong-scaling) headline.
--dry-run stops before any GPU call."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _plan(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", *args],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_launches_n_ranks_slab(n):
    # config 5 runs over every rank, config 4 over min(N, 4) (BASELINE: "RSW
    # 4096² slab-decomposed across 4 MI355X")
    assert _plan("--gpus", str(n)) == {"n_gpus": n, "parallelism": f"slab{n}", "scaling": "strong",
                                        "rank0_of": n, "config5_ranks": n, "config4_ranks": min(n, 4)}


def test_ensemble_mode_and_single_gpu():
    assert _plan("--gpus", "2", "--mode", "ensemble")["parallelism"] == "ensemble2"
    assert _plan()["parallelism"] == "single-gpu"
    assert _plan()["scaling"] is None  # one GPU scales neither way
