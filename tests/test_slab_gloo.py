"""Multi-process (gloo, CPU) tests of the slab decomposition's host path:
the product's exchange hook (slab_comm.torch_exchange, the host-staged
transport of sw_config.exchange) moves blocks correctly between ranks, and
a numpy rehearsal of libsw's slab-decomposed RSW calcN built on that hook
(tests/slab_emulation.py) equals the oracle's single-process calcN."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    try:
        sys.path[:0] = [os.path.dirname(HERE), HERE, os.path.join(os.path.dirname(HERE), "oracle")]
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from juliaraytracingsw_amd import slab_comm

        hook = slab_comm.torch_exchange()
        # 1) block routing: block q of rank r's send arrives as block r of rank q's recv
        blk = 24
        send = np.zeros((world, blk), np.uint8)
        for dst in range(world):
            send[dst] = 16 * rank + dst
        recv = np.empty_like(send)
        assert hook(None, send.ctypes.data, recv.ctypes.data, blk, world) == 0
        for src in range(world):
            assert np.all(recv[src] == 16 * src + rank), (src, recv[src, 0])
        # 2) slab-decomposed RSW calcN vs the oracle
        import slab_emulation as E
        import sw_cases
        import sw_oracle as O

        p = sw_cases.case_params("rsw_fab3", n)
        grid = O.TwoDGrid(n)
        ic = grid.dealias(sw_cases.initial_condition(p, grid))
        N_loc, kr0 = E.slab_calcN_rsw(ic, grid, world, rank, hook)
        N = E.gather_full(N_loc, kr0, grid, world, hook)
        ref = O.rsw_calcN(ic.copy(), grid, O.RSWParams(p["nu"], p["nnu"], p["f"], p["Cg"]))
        err = O.parity_error(N, ref, grid)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", float(err)))
    except Exception as e:  # report, never hang the parent
        import traceback

        q.put((rank, "fail", traceback.format_exc()))


@pytest.mark.parametrize("world,n", [(2, 64), (2, 128), (4, 128)])
def test_slab_decomposition_gloo(world, n):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    for rank, status, info in res:
        assert status == "ok", info
        assert info < 1e-12, (rank, info)
