"""CPU rehearsal of libsw's slab-decomposed calcN (TEST INFRASTRUCTURE).

One rank of the decomposition of DESIGN.md §6, written with numpy FFTs but
with exactly libsw's data movement and field set: the tiled mixed layouts of
sw_internal.hpp (mtile_c / mtile_x, both directions), the staging order
[peer][field][block] of the host-staged transport and the product's own
exchange hook (``juliaraytracingsw_amd.slab_comm.torch_exchange``) moving
the blocks between processes.  RSW calcN (rsw/RotatingShallowWater.jl:140-230)
is restated per slab and gathered; the tests compare it with the oracle.
"""
from __future__ import annotations

import numpy as np

from juliaraytracingsw_amd.slab_comm import slab_geometry


def _exchange(hook, send: np.ndarray, P: int) -> np.ndarray:
    """Call the C-ABI exchange hook on contiguous host buffers."""
    send = np.ascontiguousarray(send)
    recv = np.empty_like(send)
    rc = hook(None, send.ctypes.data, recv.ctypes.data, send.nbytes // P, P)
    if rc != 0:
        raise RuntimeError("exchange hook failed")
    return recv


# libsw's tile shapes (sw_internal.hpp): (kr extent A of a 128-B line, line order)
TILE_F, LORD_F = 2, 1  # forward fields (row outputs)
TILE_I, LORD_I = 2, 0  # inverse fields (column outputs)
CM_F, CM_I = 0, 1  # inside a line: row-major (forward), column-major (inverse; Geom::tcm)


def _tile_local(krl, yl, A, order, kcl, nyl, cm=0):
    """mtile_local: element offset of (krl, yl) inside one kcl x nyl block."""
    B = 8 // A
    line = (yl // B) * (kcl // A) + krl // A if order == 0 else (krl // A) * (nyl // B) + yl // B
    return line * 8 + ((krl % A) * B + yl % B if cm else (yl % B) * A + krl % A)


def _to_col_phase(X, A, order, P, nyl, cm=0):
    """[y][krl] (ny x kcl) -> the column-phase buffer (mtile_c), blocks q contiguous."""
    ny, kcl = X.shape
    y, krl = np.meshgrid(np.arange(ny), np.arange(kcl), indexing="ij")
    off = (y // nyl) * nyl * kcl + _tile_local(krl, y % nyl, A, order, kcl, nyl, cm)
    buf = np.empty(ny * kcl, X.dtype)
    buf[off.ravel()] = X.ravel()
    return buf.reshape(P, nyl * kcl)


def _from_row_phase(blocks, A, order, kcl, nyl, cm=0):
    """blocks [p][nyl*kcl] (mtile_x) -> [yl][kr] (nyl x P*kcl)."""
    P = blocks.shape[0]
    yl, kr = np.meshgrid(np.arange(nyl), np.arange(P * kcl), indexing="ij")
    off = (kr // kcl) * nyl * kcl + _tile_local(kr % kcl, yl, A, order, kcl, nyl, cm)
    return blocks.reshape(-1)[off]


def _to_row_phase(Y, A, order, kcl, nyl, cm=0):
    """[yl][kr] (nyl x P*kcl) -> blocks [q][nyl*kcl] (mtile_x), block q = slab q's columns."""
    P = Y.shape[1] // kcl
    yl, kr = np.meshgrid(np.arange(nyl), np.arange(P * kcl), indexing="ij")
    off = (kr // kcl) * nyl * kcl + _tile_local(kr % kcl, yl, A, order, kcl, nyl, cm)
    buf = np.empty(P * nyl * kcl, Y.dtype)
    buf[off.ravel()] = Y.ravel()
    return buf.reshape(P, nyl * kcl)


def _from_col_phase(blocks, A, order, kcl, nyl, cm=0):
    """blocks [q][nyl*kcl] (mtile_c) -> [y][krl] (ny x kcl)."""
    P = blocks.shape[0]
    y, krl = np.meshgrid(np.arange(P * nyl), np.arange(kcl), indexing="ij")
    off = (y // nyl) * nyl * kcl + _tile_local(krl, y % nyl, A, order, kcl, nyl, cm)
    return blocks.reshape(-1)[off]


def slab_calcN_rsw(sol, grid, P, r, hook):
    """N on slab r's live columns: (3, ny, kcn) complex, plus kr0."""
    nx, ny = grid.nx, grid.ny
    geo = slab_geometry(nx, ny, grid.aliased_fraction, P, r)
    kc, kcl, kr0, kcn, nyl = geo["kc"], geo["kcl"], geo["kr0"], geo["kcn"], geo["nyl"]
    kr_all = grid.kr  # (nkr,)
    l = grid.l        # (ny,)
    scale = 1.0 / (nx * ny)

    # --- column phase: this slab's spectral columns (dealiased state)
    S = np.zeros((3, ny, kcl), complex)
    S[:, :, :kcn] = grid.dealias(sol.copy())[:, :, kr0:kr0 + kcn]
    U, V, H = S
    # inverse fields U, V, H, Uy (sw_kernels.hip k_col_inv)
    inv_in = [U, V, H, 1j * l[:, None] * U]
    colph = [np.fft.ifft(X, axis=0) * ny * scale for X in inv_in]  # unnormalised inverse / (nx ny)
    # inverse-direction layout midc_i; staging [q][field][block]
    send = np.stack([_to_col_phase(c, TILE_I, LORD_I, P, nyl, CM_I) for c in colph], axis=1)
    recv = _exchange(hook, send, P)  # [p][field][block]

    # --- row phase (midx_i) -> [yl][kr]
    def row_field(f):
        t = _from_row_phase(recv[:, f], TILE_I, LORD_I, kcl, nyl, CM_I)
        full = np.zeros((nyl, nx // 2 + 1), complex)
        full[:, :kc] = t[:, :kc]
        return full

    def phys(Xh):  # unnormalised c2r along x (numpy rule: DC imaginary part dropped)
        return np.fft.irfft(Xh, n=nx, axis=1) * nx

    Ur, Vr, Hr, Uyr = (row_field(f) for f in range(4))
    ik = 1j * kr_all[None, :]
    u, v, eta = phys(Ur), phys(Vr), phys(Hr)
    zeta = phys(ik * Vr - Uyr)

    def spec(a):
        return np.fft.rfft(a, axis=1)

    # vorticity form (k_row): P = -ik K^ + (ζv)^, K^, (ζu)^, Q = -ik (uη)^, (vη)^
    Kh = spec(0.5 * (u * u + v * v))
    outs = [-ik * Kh + spec(zeta * v), Kh, spec(zeta * u), -ik * spec(u * eta), spec(v * eta)]
    fwd = []
    for a in outs:
        Y = np.zeros((nyl, P * kcl), complex)
        Y[:, :kc] = a[:, :kc]
        fwd.append(_to_row_phase(Y, TILE_F, LORD_F, kcl, nyl, CM_F))  # midx: [q][block]
    send = np.stack(fwd, axis=1)  # [q][field][block]
    recv = _exchange(hook, send, P)  # [p][field][block]

    # --- column phase (midc) -> [y][krl], forward y-FFT, combine
    def col_field(f):
        return _from_col_phase(recv[:, f], TILE_F, LORD_F, kcl, nyl, CM_F)

    FP, FK, FZU, FQ, FVE = (np.fft.fft(col_field(f), axis=0) for f in range(5))
    il = 1j * l[:, None]
    N = np.stack([FP, -il * FK - FZU, FQ - il * FVE])[:, :, :kcn]
    return N, kr0


def gather_full(N_local, kr0, grid, P, hook):
    """Assemble the full (3, nl, nkr) array from every rank's columns."""
    import torch.distributed as dist

    parts = [None] * P
    dist.all_gather_object(parts, (kr0, N_local))
    out = np.zeros((3, grid.ny, grid.nx // 2 + 1), complex)
    for k0, n in parts:
        out[:, :, k0:k0 + n.shape[2]] = n
    return grid.dealias(out)
