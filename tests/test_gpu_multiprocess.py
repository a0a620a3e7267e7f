"""One process per slab on the GPU box: torch.distributed.run starts `world`
ranks, each with its own libsw context holding one slab, exchanging through
the host-staged transport (gloo).  The gathered results must equal the
undecomposed run bitwise, the device-recorded energy diagnostics and the CFL
reduction included."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("case,world,steps,freq", [("rsw_fab3", 2, 6, 2), ("qg2_ifmrk4", 2, 6, 2),
                                                   ("rsw_ifmab3", 4, 6, 2),
                                                   # more records than one host-staged gather holds
                                                   # before the chunked, incremental gather
                                                   ("rsw_fab3", 2, 240, 1)])
def test_one_process_per_slab(case, world, steps, freq, tmp_path):
    out = tmp_path / "res.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "mp_slab_worker.py"), "--case", case, "--out", str(out),
           "--steps", str(steps), "--freq", str(freq)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["world"] == world
    assert res["state_equal"] and res["calcN_equal"] and res["physical_equal"], res
    assert res["ke_rel"] == 0 and res["pe_rel"] == 0, res
    assert res["records_equal"] and res["cfl_equal"], res
