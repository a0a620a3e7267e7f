"""Host-side plumbing of the slab decomposition.

libsw does the transposes itself (RCCL all-to-all over xGMI); the host only
has to agree on the communicator.  ``rccl_decomposition`` broadcasts the RCCL
unique id with ``torch.distributed`` (one process per GPU, the bench layout).
``torch_exchange`` builds the optional host-staged transport hook of
``sw_config.exchange``: every exchange becomes a ``torch.distributed``
all-to-all of host buffers, which runs over gloo where RCCL cannot (several
ranks on one GPU, CPU tests).  ``slab_geometry`` mirrors ``make_geom`` in
``csrc/sw_api.cpp`` for reporting and for the CPU emulation tests.
"""
from __future__ import annotations

import ctypes as C
import math
import traceback

from . import _lib


def rccl_decomposition(rank: int, world: int, nranks: int | None = None) -> dict | None:
    """Problem(decomposition=...) kwargs for slab `rank` of `world`, one GPU
    per process, RCCL transposes.  Collective: every rank of the default
    group must call it.  With `nranks` < world only ranks [0, nranks) form
    the problem (BASELINE config 4 on 4 of 8 GPUs); the others get None."""
    import torch.distributed as dist

    n = world if nranks is None else nranks
    box = [_lib.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    if rank >= n:
        return None
    return dict(nranks=n, rank=rank, local_slabs=1, comm_unique_id=box[0])


def _as_tensor(addr: int, nbytes: int):
    import torch

    return torch.frombuffer((C.c_char * nbytes).from_address(addr), dtype=torch.uint8)


def torch_exchange(group=None):
    """An ``sw_exchange_fn`` doing ``dist.all_to_all_single`` on the staged
    host blocks (block q of send -> rank q; block p of recv <- rank p)."""
    import torch.distributed as dist

    def _fn(user, send, recv, block_bytes, nranks):
        try:
            n = int(block_bytes) * int(nranks)
            dist.all_to_all_single(_as_tensor(recv, n), _as_tensor(send, n), group=group)
            return 0
        except Exception:  # an exception must not cross the C ABI
            traceback.print_exc()
            return 1

    return _lib.EXCHANGE_FN(_fn)


def host_decomposition(rank: int, world: int, group=None) -> dict:
    """Problem(decomposition=...) kwargs for slab `rank` of `world` with the
    host-staged transport over the current torch.distributed group."""
    return dict(nranks=world, rank=rank, local_slabs=1, exchange=torch_exchange(group))


# threads per column-pass block (SW_BLK_THREADS, csrc/sw_internal.hpp); the
# library reports its own value through sw_slab_geometry (checked by
# tests/test_abi.py)
SW_BLK_THREADS = 64


def _alias_range(n, af):
    return math.floor((1 - af) / 2 * n) + 1, math.ceil((1 + af) / 2 * n)


def slab_geometry(nx: int, ny: int, aliased_fraction: float, P: int, s: int) -> dict:
    """Columns and rows of slab s of P (make_geom in csrc/sw_api.cpp)."""
    iLx, _ = _alias_range(nx, aliased_fraction)
    kc = iLx - 1
    if P == 1:
        kcl = (kc + 63) // 64 * 64
    else:
        NT = ny // 8
        nb = 1 if NT >= SW_BLK_THREADS else min(SW_BLK_THREADS // NT, 32)
        gran = max(8, nb)
        kcl = ((kc + P - 1) // P + gran - 1) // gran * gran
    kr0 = s * kcl
    return dict(kc=kc, kcl=kcl, kr0=kr0, kcn=max(0, min(kcl, kc - kr0)), nyl=ny // P, y0=s * (ny // P))
