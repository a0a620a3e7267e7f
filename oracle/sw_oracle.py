"""CPU oracle for the pseudo-spectral time-step hot path (TEST INFRASTRUCTURE ONLY).

This module is the *checker*, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``juliaraytracingsw_amd`` + ``libsw.so``) never calls
into this file and fails loudly when the HIP library is missing.

It is a plain fp64 numpy/scipy restatement of the reference algorithm, written
to mirror the reference op sequence one broadcast / one transform at a time:

* FourierFlows.jl ``TwoDGrid`` / ``dealias!`` / ``makefilter`` / FFT plan
  semantics (FF is not vendored in the reference; formulas restated from its
  call sites).
* ``rsw/RotatingShallowWater.jl`` calcN! (140-230), L (242-307).
* ``swqg/TwoLayerQG.jl`` streamfunctionfrompv! (101-111), calcN! (152-182),
  L_kernel! (184-198) including its Complex{Float32} literal quirk.
* ``utils/IFMAB3.jl`` (9-11, 26-30, 125-169) and FF ``FilteredAB3`` (A7, with
  ``addlinearterm!`` generalised to the per-mode matvec).
* ``utils/IFMRK4.jl`` structure (13-22, 157-163) -> Lawson IF-RK4.
* ``thomasyamada/ThomasYamada.jl`` calcN! (129-262), L (265-277),
  ``thomasyamada/TYUtils.jl`` bases, ``TYdriver.jl:36-87`` IC, and FF
  ``ETDRK4``/``getetdcoeffs`` (restated: FF not vendored).
* GeophysicalFlows ``MultiLayerQG`` (2 layers) + FF ``FilteredRK4`` as
  ``simulation/TwoLayerSimulation.jl`` runs it (GF not vendored: restated from
  its published equations, PARITY UNPINNED against GF; pinned by the
  analytic Phillips baroclinic growth rate).
* Driver parameter formulas and initial conditions: ``rsw/RSWDriver.jl:88-176``,
  ``swqg/TwoLayerDriver.jl:10-68``, ``simulation/Parameters.jl``.

Parity pinning.  The reference cannot run here (no Julia / FourierFlows /
FFTW).  This restatement is pinned by every known answer the
reference holds for the path: the Julia ``exp`` of ``Lop(1,1)``
(rsw/Notebooks/MatrixExponentialTest.ipynb:64,197-199), the per-mode matvec
assertion (same notebook :498), the ``TwoDGrid`` display (:17-20) and the
``dt``/``ν`` driver numbers (rsw/Notebooks/RSW_Test.ipynb:228-229), plus the
analytic known answers listed in SURVEY §8c (linear exactness of IFMAB3 via the
reference's NOPcalcN! hook, energy conservation of the linear propagator,
convergence order).  No reference test pins a *stepped* nonlinear state, so
stepped-state parity against FourierFlows itself is "parity unpinned"; the
GPU path is checked against this restatement.

Array layout: numpy C order ``[field][l][kr]`` == Julia column-major
``(nkr, nl, nfield)`` byte for byte.  Physical ``[y][x]`` == Julia ``(nx, ny)``.
"""
from __future__ import annotations

import math
import numpy as np

try:  # scipy's batched expm is the oracle's matrix exponential
    import scipy.linalg as _sla
except Exception:  # pragma: no cover
    _sla = None

# FFT backend: numpy (default, used for golden vectors) or scipy.fft with a
# worker pool (the timed CPU-baseline leg in bench.py)
_FFT_WORKERS = None


def set_fft_workers(n):
    """Use scipy.fft with ``n`` threads for the transforms (None: numpy.fft)."""
    global _FFT_WORKERS
    _FFT_WORKERS = n


def _irfft2(a, s):
    if _FFT_WORKERS:
        import scipy.fft as sf
        return sf.irfft2(a, s=s, axes=(-2, -1), workers=_FFT_WORKERS)
    return np.fft.irfft2(a, s=s, axes=(-2, -1))


def _rfft2(a):
    if _FFT_WORKERS:
        import scipy.fft as sf
        return sf.rfft2(a, axes=(-2, -1), workers=_FFT_WORKERS)
    return np.fft.rfft2(a, axes=(-2, -1))


# utils/IFMAB3.jl:9-11
AB3H1 = 23 / 12
AB3H2 = 16 / 12
AB3H3 = 5 / 12


# --------------------------------------------------------------------------
# FourierFlows TwoDGrid restatement
# --------------------------------------------------------------------------
def aliased_index_range(n: int, aliased_fraction: float):
    """FF ``getaliasedwavenumbers``: 1-based (iL, iR) of the aliased band.

    L = (1-af)/2, R = (1+af)/2, iL = floor(L n) + 1, iR = ceil(R n)
    (SURVEY A1).  kralias = iL:nkr, lalias = iL:iR (1-based, inclusive).
    """
    if not (0.0 <= aliased_fraction < 1.0):
        raise ValueError("aliased_fraction must be in [0, 1)")
    L = (1 - aliased_fraction) / 2
    R = (1 + aliased_fraction) / 2
    iL = math.floor(L * n) + 1
    iR = math.ceil(R * n)
    return iL, iR


class TwoDGrid:
    """Restatement of FF ``TwoDGrid(dev; nx, Lx, ny, Ly, aliased_fraction, T)``.

    Called at rsw/RotatingShallowWater.jl:87 and swqg/TwoLayerQG.jl:75.
    """

    def __init__(self, nx, Lx=2 * np.pi, ny=None, Ly=None, aliased_fraction=1 / 3):
        ny = nx if ny is None else ny
        Ly = Lx if Ly is None else Ly
        if nx % 2 or ny % 2:
            raise ValueError("nx, ny must be even")
        self.nx, self.ny, self.Lx, self.Ly = int(nx), int(ny), float(Lx), float(Ly)
        self.aliased_fraction = float(aliased_fraction)
        self.dx = self.Lx / self.nx
        self.dy = self.Ly / self.ny
        self.x = -self.Lx / 2 + self.dx * np.arange(self.nx)
        self.y = -self.Ly / 2 + self.dy * np.arange(self.ny)
        self.nkr = self.nx // 2 + 1
        self.nl = self.ny
        # rfftfreq(nx, 2π/Lx*nx) / fftfreq(ny, 2π/Ly*ny): element j = j*(fs/n)
        mk = (2 * np.pi / self.Lx * self.nx) / self.nx
        ml = (2 * np.pi / self.Ly * self.ny) / self.ny
        self.kr = np.arange(self.nkr) * mk
        lidx = np.concatenate([np.arange(0, self.ny // 2), np.arange(-self.ny // 2, 0)])
        self.l = lidx * ml
        self.Krsq = self.kr[None, :] ** 2 + self.l[:, None] ** 2
        with np.errstate(divide="ignore"):
            self.invKrsq = np.where(self.Krsq == 0, 0.0, 1.0 / self.Krsq)
        # dealias index ranges (0-based, half-open)
        iLx, _ = aliased_index_range(self.nx, self.aliased_fraction)
        iLy, iRy = aliased_index_range(self.ny, self.aliased_fraction)
        self.kralias = (iLx - 1, self.nkr)        # zeroed kr columns
        self.lalias = (iLy - 1, iRy)              # zeroed l rows [a, b)
        if self.aliased_fraction == 0:
            # FF getaliasedwavenumbers with aliased_fraction = 0: only the
            # Nyquist column kr = nx/2 and row l = -ny/2 are zeroed
            self.kralias = (self.nkr - 1, self.nkr)
            self.lalias = (self.ny // 2, self.ny // 2 + 1)
        mask = np.ones((self.nl, self.nkr), dtype=bool)
        mask[:, self.kralias[0]:self.kralias[1]] = False
        mask[self.lalias[0]:self.lalias[1], :] = False
        self.live = mask
        # number of live kr columns and live l rows
        self.kc = self.kralias[0]
        self.live_rows = np.concatenate(
            [np.arange(0, self.lalias[0]), np.arange(self.lalias[1], self.ny)])

    def dealias(self, fh):
        """FF ``dealias!(fh, grid)`` in place."""
        fh[..., :, self.kralias[0]:self.kralias[1]] = 0
        fh[..., self.lalias[0]:self.lalias[1], :] = 0
        return fh

    # FF rfftplan semantics
    def irfft(self, fh):
        """``ldiv!(u, grid.rfftplan, uh)``: normalised c2r (numpy rule for
        non-Hermitian DC/Nyquist columns: c2c along l then c2r along x)."""
        return _irfft2(fh, (self.ny, self.nx))

    def rfft(self, f):
        """``mul!(uh, grid.rfftplan, u)``: unnormalised r2c."""
        return _rfft2(f)


def makefilter(grid: TwoDGrid, order=4, innerK=0.65, outerK=1.0, tol=1e-15):
    """FF ``makefilter(grid; realvars=true, order, innerK, outerK, tol)`` (A8)."""
    K = np.sqrt((grid.kr[None, :] * grid.dx / np.pi) ** 2
                + (grid.l[:, None] * grid.dy / np.pi) ** 2)
    decay = -np.log(tol) / (outerK - innerK) ** order
    filt = np.exp(-decay * (K - innerK) ** order)
    filt[K < innerK] = 1.0
    return filt


def expm_batched(A):
    """Per-mode matrix exponential (utils/IFMAB3.jl:26-30 ``mapslices(exp, …)``)."""
    if _sla is None:  # pragma: no cover
        raise RuntimeError("scipy is required for the oracle's expm")
    sh = A.shape
    flat = A.reshape(-1, sh[-2], sh[-1])
    if _EXPM_WORKERS > 1 and flat.shape[0] > 400_000:
        # scipy's per-slice loop holds the GIL: large batches (the 8192²
        # fixture's 30 M matrices) go to forked worker processes
        import multiprocessing as mp

        with mp.get_context("fork").Pool(_EXPM_WORKERS) as pool:
            parts = pool.map(_sla.expm, np.array_split(flat, 4 * _EXPM_WORKERS))
        out = np.concatenate(parts)
    else:
        out = _sla.expm(flat)
    return out.reshape(sh)


_EXPM_WORKERS = 1


def set_expm_workers(n):
    """processes for scipy's expm over large batches (None/1: in process)"""
    global _EXPM_WORKERS
    _EXPM_WORKERS = max(1, int(n or 1))


def expm_2x2(A):
    """exp of a batch of 2×2 matrices in closed form (the 2LQG/MLQG operators;
    utils/IFMAB3.jl:26-30 takes Julia's Padé ``exp`` per mode): with m the
    half trace and B = A − m I (traceless, B² = δ² I, δ² = p² + b c),
    exp(A) = e^m (cosh δ I + sinh(δ)/δ B), both even in δ (no branch), series
    for small |δ|.  Checked against scipy's expm per mode in
    tests/test_oracle.py; it makes the 8192² oracle run affordable (scipy's
    expm over 33.5 M matrices is not)."""
    a, b, c, d = A[..., 0, 0], A[..., 0, 1], A[..., 1, 0], A[..., 1, 1]
    m = 0.5 * (a + d)
    p = 0.5 * (a - d)
    d2 = p * p + b * c
    dl = np.sqrt(d2)
    small = np.abs(d2) < 1e-6
    with np.errstate(invalid="ignore", divide="ignore"):
        ch = np.where(small, 1 + d2 / 2 + d2 * d2 / 24 + d2 ** 3 / 720, np.cosh(dl))
        sh = np.where(small, 1 + d2 / 6 + d2 * d2 / 120 + d2 ** 3 / 5040, np.sinh(dl) / np.where(small, 1, dl))
    em = np.exp(m)
    out = np.empty(A.shape, np.complex128)
    out[..., 0, 0] = em * (ch + sh * p)
    out[..., 1, 1] = em * (ch - sh * p)
    out[..., 0, 1] = em * (sh * b)
    out[..., 1, 0] = em * (sh * c)
    return out


def expm_modes(A, method="scipy", live=None):
    """Per-mode exp (utils/IFMAB3.jl:26-30: Julia's Padé ``exp`` per mode).

    method "scipy" (default): scipy's expm (Al-Mohy & Higham scaling and
    squaring; scipy >= 1.11 has no 2×2 special case), independent of the
    device's closed-form ``ExpOf`` — with `live` (a
    mask of the modes the 2/3 rule keeps), scipy on those modes and the
    closed form on the aliased ones, whose values never reach a live mode
    (calcN! dealiases its input); the Problems pass `live` only above
    SCIPY_ALL_MODES (scipy_split), so every aliased_state comparison, which
    reads the aliased modes, runs on scipy's values there.  method "closed": ``expm_2x2`` for 2×2
    operators — the 8192² fixture (tests/golden/make_qg2_8192.py), where
    scipy over 33.5 M matrices is not affordable; it is pinned to scipy on
    that fixture's own operator rows (tests/test_oracle.py)."""
    if A.shape[-2:] != (2, 2):
        return expm_batched(A)
    if method == "closed":
        return expm_2x2(A)
    if method != "scipy":
        raise ValueError(method)
    if live is None:
        return expm_batched(A)
    out = expm_2x2(A)
    out[live] = expm_batched(A[live])
    return out


# modes up to which scipy's expm runs on every mode, the aliased ones too
# (the aliased_state tests compare those modes, and the closed
# form there is the device's own formula); above it (2048² and up, the live
# modes alone are ~1 M matrices) scipy on the live modes, the closed form on
# the aliased ones, which no default-context comparison reads
SCIPY_ALL_MODES = 1 << 20


def scipy_split(grid):
    """the `live` argument of expm_modes for this grid (None: scipy everywhere)"""
    return None if grid.nkr * grid.nl <= SCIPY_ALL_MODES else live_mask(grid)


def mvmul(A, x):
    """``mvmul!`` (utils/IFMAB3.jl:90-100, 124-127): y[…,r] = Σ_c A[…,r,c] x[…,c].

    ``A`` has shape [nl, nkr, nf, nf]; ``x`` has shape [nf, nl, nkr]."""
    return np.einsum("lkrc,clk->rlk", A, x)


# --------------------------------------------------------------------------
# Rotating shallow water (rsw/RotatingShallowWater.jl)
# --------------------------------------------------------------------------
class RSWParams:
    """rsw/RotatingShallowWater.jl:18-23 (ν, nν, f, Cg2)."""

    def __init__(self, nu, nnu, f, Cg):
        self.nu, self.nnu, self.f, self.Cg2 = float(nu), int(nnu), float(f), float(Cg) ** 2


def rsw_L(grid: TwoDGrid, p: RSWParams):
    """Per-mode 3×3 L (rsw/RotatingShallowWater.jl:242-289), shape [nl,nkr,3,3]."""
    D = -p.nu * grid.Krsq ** p.nnu
    k = np.broadcast_to(grid.kr[None, :], D.shape)
    l = np.broadcast_to(grid.l[:, None], D.shape)
    L = np.zeros(D.shape + (3, 3), dtype=np.complex128)
    L[..., 0, 0] = D
    L[..., 0, 1] = p.f
    L[..., 0, 2] = -1j * k * p.Cg2
    L[..., 1, 0] = -p.f
    L[..., 1, 1] = D
    L[..., 1, 2] = -1j * l * p.Cg2
    L[..., 2, 0] = -1j * k
    L[..., 2, 1] = -1j * l
    L[..., 2, 2] = D
    return L


def rsw_calcN(sol, grid: TwoDGrid, p: RSWParams):
    """rsw/RotatingShallowWater.jl:140-230, op for op.  ``sol`` is dealiased
    IN PLACE (line 141), exactly as the reference does."""
    grid.dealias(sol)
    kr = grid.kr[None, :]
    l = grid.l[:, None]
    uh, vh, etah = sol[0].copy(), sol[1].copy(), sol[2].copy()
    N = np.empty_like(sol)
    u = grid.irfft(uh)                                   # :154-156
    v = grid.irfft(vh)                                   # :159-161
    uux = grid.irfft(1j * kr * uh) * u                   # :170-172
    N[0] = -grid.rfft(uux)                               # :173-174
    vvy = grid.irfft(1j * l * vh) * v                    # :179-181
    N[1] = -grid.rfft(vvy)                               # :182-183
    vuy = grid.irfft(1j * l * uh) * v                    # :193-195
    N[0] += -grid.rfft(vuy)                              # :196-197
    uvx = grid.irfft(1j * kr * vh) * u                   # :202-204
    N[1] += -grid.rfft(uvx)                              # :205-206
    eta = grid.irfft(etah)                               # :212-214
    N[2] = -1j * kr * grid.rfft(u * eta)                 # :218-220
    N[2] += -1j * l * grid.rfft(v * eta)                 # :224-226
    return N


def rsw_NOPcalcN(sol, grid, p):
    """rsw/RotatingShallowWater.jl:135-138 (N .= 0) — the linear-only hook."""
    return np.zeros_like(sol)


def rsw_updatevars(sol, grid: TwoDGrid, p: RSWParams):
    """rsw/RotatingShallowWater.jl:101-116 -> dict of physical fields."""
    grid.dealias(sol)
    kr = grid.kr[None, :]
    l = grid.l[:, None]
    zh = 1j * kr * sol[1] - 1j * l * sol[0] - p.f * sol[2]
    return {"u": grid.irfft(sol[0]), "v": grid.irfft(sol[1]),
            "eta": grid.irfft(sol[2]), "zeta": grid.irfft(zh)}


def parsevalsum2(uh, grid: TwoDGrid):
    """FF ``parsevalsum2`` (copy at thomasyamada/ThomasYamada.jl:319-331)."""
    U = np.abs(uh) ** 2
    s = 2 * U.sum() - U[:, 0].sum()
    if grid.nx % 2 == 0:
        s -= U[:, -1].sum()
    norm = grid.Lx * grid.Ly / (grid.nx ** 2 * grid.ny ** 2)
    return norm * s


def rsw_energies(sol, grid, p):
    """KE, PE (rsw/RotatingShallowWater.jl:323-336) of the dealiased state."""
    s = grid.dealias(sol.copy())
    KE = (parsevalsum2(s[0], grid) + parsevalsum2(s[1], grid)) / (2 * grid.Lx * grid.Ly)
    PE = 0.5 * p.Cg2 * parsevalsum2(s[2], grid) / (grid.Lx * grid.Ly)
    return KE, PE


# --------------------------------------------------------------------------
# Two-layer QG (swqg/TwoLayerQG.jl)
# --------------------------------------------------------------------------
class QG2Params:
    """swqg/TwoLayerQG.jl:23-30, F = 2 f0²/Cg²/δρρ0 (:79)."""

    def __init__(self, U, mu, nu, nnu, f0=3.0, Cg=1.0, drhorho0=0.2, F=None):
        self.U, self.mu, self.nu, self.nnu = float(U), float(mu), float(nu), int(nnu)
        self.F = float(2 * f0 ** 2 / Cg ** 2 / drhorho0) if F is None else float(F)


def qg2_streamfunction(qh, grid: TwoDGrid, p: QG2Params):
    """swqg/TwoLayerQG.jl:101-111 (same evaluation order)."""
    K2 = grid.Krsq
    q1, q2 = qh[0], qh[1]
    psi = np.empty_like(qh)
    psi[0] = -(K2 * q1 + p.F * (q1 + q2))
    psi[1] = -(K2 * q2 + p.F * (q1 + q2))
    psi /= K2 + 2 * p.F
    psi *= grid.invKrsq
    return psi


def qg2_L(grid: TwoDGrid, p: QG2Params):
    """swqg/TwoLayerQG.jl:184-206, with the Complex{Float32} literal quirk
    (SURVEY A11): PV_term, drag_term and the Sinv numerators are rounded to
    fp32 before being widened back to fp64.  Shape [nl, nkr, 2, 2]."""
    k = np.broadcast_to(grid.kr[None, :], grid.Krsq.shape).astype(np.float64)
    K2 = k ** 2 + np.broadcast_to(grid.l[:, None], grid.Krsq.shape) ** 2
    with np.errstate(divide="ignore"):
        K2inv = np.where(K2 == 0, 0.0, 1.0 / K2)
    D = -p.nu * grid.Krsq ** p.nnu
    f32 = np.float32
    pv1_im = (((-2.0 * k) * p.F) * p.U).astype(f32).astype(np.float64)
    pv2_im = (((2.0 * k) * p.F) * p.U).astype(f32).astype(np.float64)
    drag2 = (p.mu * K2).astype(f32).astype(np.float64)
    psi_re = [np.zeros_like(K2), drag2]
    psi_im = [pv1_im, pv2_im]
    a = ((-K2) - p.F).astype(f32).astype(np.float64)
    b = np.full_like(K2, f32(-p.F), dtype=np.float64)
    den = K2 + 2 * p.F
    S = [[(a / den) * K2inv, (b / den) * K2inv],
         [(b / den) * K2inv, (a / den) * K2inv]]
    L = np.zeros(K2.shape + (2, 2), dtype=np.complex128)
    for r in range(2):
        for c in range(2):
            L[..., r, c] = psi_re[r] * S[r][c] + 1j * (psi_im[r] * S[r][c])
    L[..., 0, 0] = (L[..., 0, 0].real + D) + 1j * (L[..., 0, 0].imag + (-k * p.U))
    L[..., 1, 1] = (L[..., 1, 1].real + D) + 1j * (L[..., 1, 1].imag + (k * p.U))
    return L


def qg2_calcN(sol, grid: TwoDGrid, p: QG2Params):
    """swqg/TwoLayerQG.jl:152-182 (batched over both layers), sol dealiased in place."""
    grid.dealias(sol)
    kr = grid.kr[None, :]
    l = grid.l[:, None]
    qh = sol.copy()
    psih = qg2_streamfunction(qh, grid, p)
    q = grid.irfft(qh)                                   # :157-159
    psixq = grid.irfft(1j * kr * psih) * q               # :167-169
    N = -1j * l * grid.rfft(psixq)                       # :170-171
    psiyq = grid.irfft(1j * l * psih) * q                # :175-177
    N += 1j * kr * grid.rfft(psiyq)                      # :178-179
    return N


def qg2_energies(sol, grid, p):
    """KE per layer and PE (swqg/TwoLayerQG.jl:230-252); reads sol as is."""
    psih = qg2_streamfunction(sol, grid, p)
    a = grid.Krsq * np.abs(psih) ** 2

    def parsevalsum(fh):
        s = 2 * fh.sum() - fh[:, 0].sum()
        if grid.nx % 2 == 0:
            s -= fh[:, -1].sum()
        return (grid.Lx * grid.Ly / (grid.nx ** 2 * grid.ny ** 2)) * s.real

    KE1 = parsevalsum(a[0]) / (grid.Lx * grid.Ly)
    KE2 = parsevalsum(a[1]) / (grid.Lx * grid.Ly)
    PE = 1 / (2 * grid.Lx * grid.Ly) * p.F * parsevalsum(np.abs(psih[0] - psih[1]) ** 2)
    return (KE1, KE2), PE


# --------------------------------------------------------------------------
# Thomas–Yamada barotropic/baroclinic model (thomasyamada/ThomasYamada.jl)
# --------------------------------------------------------------------------
class TYParams:
    """thomasyamada/ThomasYamada.jl:21-25 (ν, nν, Ro)."""

    def __init__(self, nu, nnu, Ro):
        self.nu, self.nnu, self.Ro = float(nu), int(nnu), float(Ro)


def ty_L(grid: TwoDGrid, p: TYParams):
    """thomasyamada/ThomasYamada.jl:265-277: real diagonal L = D on all four
    fields, shape [4, nl, nkr]."""
    D = -p.nu * grid.Krsq ** p.nnu
    return np.stack([D, D, D, D])


def ty_calcN(sol, grid: TwoDGrid, p: TYParams):
    """thomasyamada/ThomasYamada.jl:129-262 (calcN! + calcN_vorticity!,
    calcN_baroclinic!, calcN_pressure!) op for op; ``sol`` = (ζ_T, u_c, v_c,
    p_c) is dealiased IN PLACE (line 130)."""
    grid.dealias(sol)
    kr = grid.kr[None, :]
    l = grid.l[:, None]
    Ro = p.Ro
    zth, uch, vch, pch = sol[0].copy(), sol[1].copy(), sol[2].copy(), sol[3].copy()
    psith = -zth * grid.invKrsq                           # :125-127
    uth = -1j * l * psith                                 # :138
    vth = 1j * kr * psith                                 # :139
    N = np.empty_like(sol)
    N[0] = 0.0                                            # :142
    N[1] = vch - 1j * kr * pch                            # :143
    N[2] = -uch - 1j * l * pch                            # :144
    N[3] = -1j * kr * uch - 1j * l * vch                  # :145
    zt = grid.irfft(zth)                                  # :148-149
    ut = grid.irfft(uth)                                  # :150-152
    vt = grid.irfft(vth)                                  # :153
    uc = grid.irfft(uch)                                  # :154-156
    vc = grid.irfft(vch)                                  # :157
    # calcN_vorticity! (:166-202)
    vzh = grid.rfft(vt * zt)                              # :174-177
    uzh = grid.rfft(ut * zt)                              # :179-182
    N[0] += -Ro * (1j * l * vzh + 1j * kr * uzh)          # :183
    uvh = grid.rfft(uc * vc)                              # :186-189
    N[0] += -Ro * (-kr ** 2 + l ** 2) * uvh               # :190
    v2h = grid.rfft(vc * vc)                              # :192-199
    u2h = grid.rfft(uc * uc)
    N[0] += -Ro * (-kr * l * v2h + kr * l * u2h)          # :201
    # calcN_baroclinic! (:204-243)
    ucuth = grid.rfft(ut * uc)                            # :212-217
    vcvth = grid.rfft(vt * vc)
    N[1] += -Ro * (1j * kr * ucuth)                       # :218
    N[2] += -Ro * (1j * l * vcvth)                        # :219
    vtucy = grid.irfft(1j * l * uch) * vt                 # :225-231
    vcuty = grid.irfft(1j * l * uth) * vc
    N[1] += -Ro * (grid.rfft(vtucy) + grid.rfft(vcuty))   # :232-234
    utvcx = grid.irfft(1j * kr * vch) * ut                # :240-246
    ucvtx = grid.irfft(1j * kr * vth) * uc
    N[2] += -Ro * (grid.rfft(utvcx) + grid.rfft(ucvtx))   # :247-249
    # calcN_pressure! (:251-262), pch restored from sol at :161
    utpcx = grid.irfft(1j * kr * pch) * ut                # :257-264
    vtpcy = grid.irfft(1j * l * pch) * vt
    N[3] += -Ro * (grid.rfft(utpcx) + grid.rfft(vtpcy))   # :265-266
    return N


def ty_updatevars(sol, grid: TwoDGrid, p: TYParams):
    """thomasyamada/ThomasYamada.jl:67-92 -> dict of physical fields."""
    grid.dealias(sol)
    kr = grid.kr[None, :]
    l = grid.l[:, None]
    psith = -sol[0] * grid.invKrsq
    qch = 1j * kr * sol[2] - 1j * l * sol[1] - sol[3]
    return {"zt": grid.irfft(sol[0]), "uc": grid.irfft(sol[1]), "vc": grid.irfft(sol[2]),
            "pc": grid.irfft(sol[3]), "ut": grid.irfft(-1j * l * psith),
            "vt": grid.irfft(1j * kr * psith), "qc": grid.irfft(qch)}


def ty_balanced_basis(grid: TwoDGrid):
    """thomasyamada/TYUtils.jl:10-20 (Φ₀), shape [3, nl, nkr]."""
    kr = np.broadcast_to(grid.kr[None, :], grid.Krsq.shape)
    l = np.broadcast_to(grid.l[:, None], grid.Krsq.shape)
    om = np.sqrt(1 + kr ** 2 + l ** 2)
    P = np.stack([1j * l / om, -1j * kr / om, -1 / om + 0j])
    P[:, 0, 0] = [0, 0, 1]
    return P


def ty_wave_bases(grid: TwoDGrid):
    """thomasyamada/TYUtils.jl:22-38 (Φ₊, Φ₋), each [3, nl, nkr]."""
    kr = np.broadcast_to(grid.kr[None, :], grid.Krsq.shape)
    l = np.broadcast_to(grid.l[:, None], grid.Krsq.shape)
    om = np.sqrt(1 + kr ** 2 + l ** 2)
    s = np.sqrt(grid.invKrsq / 2) / om
    Pp = np.stack([(om * kr + 1j * l) * s, (om * l - 1j * kr) * s, (om ** 2 - 1) * s + 0j])
    Pm = np.stack([(-om * kr + 1j * l) * s, (-om * l - 1j * kr) * s, (om ** 2 - 1) * s + 0j])
    Pp[:, 0, 0] = np.array([1j, 1, 0]) / np.sqrt(2)
    Pm[:, 0, 0] = np.array([1j, -1, 0]) / np.sqrt(2)
    return Pp, Pm


def ty_decompose(sol, grid: TwoDGrid):
    """thomasyamada/TYUtils.jl:40-51: balanced (G) and wave (W) parts of
    (u_c, v_c, p_c)."""
    b = sol[1:4]
    P0 = ty_balanced_basis(grid)
    Pp, Pm = ty_wave_bases(grid)
    G = (b * np.conj(P0)).sum(0)[None] * P0
    W = (b * np.conj(Pp)).sum(0)[None] * Pp + (b * np.conj(Pm)).sum(0)[None] * Pm
    return G, W


def ty_energies(sol, grid: TwoDGrid):
    """barotropic_energy, baroclinic_energy, wave_geostrophic_energy
    (thomasyamada/ThomasYamada.jl:333-367) of ``sol`` as is."""
    bt = parsevalsum2(np.sqrt(grid.invKrsq) * sol[0], grid)
    bc = (parsevalsum2(sol[1], grid) + parsevalsum2(sol[2], grid), parsevalsum2(sol[3], grid))
    G, W = ty_decompose(sol, grid)
    wg = ((parsevalsum2(W[0], grid) + parsevalsum2(W[1], grid), parsevalsum2(W[2], grid)),
          (parsevalsum2(G[0], grid) + parsevalsum2(G[1], grid), parsevalsum2(G[2], grid)))
    return bt, bc, wg


def ty_initial_condition(grid: TwoDGrid, rng, k0w_range=(0.0, 5 / 3), k0g_range=(10 / 3, 13 / 3),
                         at=0.0, ag=0.3, aw=0.1):
    """thomasyamada/TYdriver.jl:36-87 (set_initial_condition): random phases
    on the wave / geostrophic annuli projected on the TYUtils bases, each part
    scaled by its physical max.  Julia's RNG stream is not reproducible here:
    ``rng`` is a seeded numpy Generator drawing θ, θ₀, θ₊, θ₋ over (nkr, nl)
    in Julia column-major order.  Returns sol (4, nl, nkr)."""
    K2 = grid.Krsq
    wf = (k0w_range[0] ** 2 <= K2) & (K2 <= k0w_range[1] ** 2)
    gf = (k0g_range[0] ** 2 <= K2) & (K2 <= k0g_range[1] ** 2)
    th = [rng.random((grid.nkr, grid.nl)).T for _ in range(4)]
    ph, ph0, php, phm = [np.exp(2 * np.pi * 1j * t) for t in th]
    P0 = ty_balanced_basis(grid)
    Pp, Pm = ty_wave_bases(grid)
    psith = ph * gf
    g = [P0[i] * ph0 * gf for i in range(3)]
    w = [(Pp[i] * php + Pm[i] * phm) * wf for i in range(3)]
    mt = np.max(np.abs(grid.irfft(psith)))
    mg = np.max(np.abs(grid.irfft(g[0])))
    mw = np.max(np.abs(grid.irfft(w[0])))
    psith = psith * at / mt if mt > 0 else psith * 0
    g = [x * ag / mg for x in g] if mg > 0 else [x * 0 for x in g]
    w = [x * aw / mw for x in w] if mw > 0 else [x * 0 for x in w]
    zh = -K2 * psith
    return np.stack([zh, w[0] + g[0], w[1] + g[1], w[2] + g[2]])


# --------------------------------------------------------------------------
# GeophysicalFlows MultiLayerQG, nlayers = 2 (simulation/TwoLayerSimulation.jl)
# --------------------------------------------------------------------------
# GeophysicalFlows.jl is not vendored in the reference (no Manifest; SURVEY
# §8c): its MultiLayerQG is restated here from the package's published
# equations and call sequence (GF ≥ 0.15 keyword set: f₀, H, b, U, μ, β, ν,
# nν).  PARITY UNPINNED against GF itself; pinned instead by the analytic
# baroclinic-instability growth rate of the two-layer (Phillips) problem and
# by the shared J(ψ, q) term of TwoLayerQG (tests/test_oracle.py).
class MLQGParams:
    """MultiLayerQG.Params for 2 layers: g′ = b₁ − b₂, F_j = f₀²/(g′ H_j),
    background PV gradients Qy₁ = β − F₁(U₂ − U₁), Qy₂ = β − F₂(U₁ − U₂)
    (no topography: Qx = 0)."""

    def __init__(self, f0, H, b, U, mu, beta=0.0, nu=0.0, nnu=1):
        self.f0, self.mu, self.beta, self.nu, self.nnu = float(f0), float(mu), float(beta), float(nu), int(nnu)
        self.H = [float(h) for h in H]
        self.b = [float(x) for x in b]
        self.U = [float(u) for u in U]
        self.gp = self.b[0] - self.b[1]
        self.F1 = self.f0 ** 2 / (self.gp * self.H[0])
        self.F2 = self.f0 ** 2 / (self.gp * self.H[1])
        self.Qy = [self.beta - self.F1 * (self.U[1] - self.U[0]), self.beta - self.F2 * (self.U[0] - self.U[1])]


def mlqg_streamfunction(qh, grid: TwoDGrid, p: MLQGParams):
    """streamfunctionfrompv!: ψ̂ = S⁻¹ q̂ per mode, S = [[-K²-F₁, F₁],
    [F₂, -K²-F₂]]; S⁻¹ = [[-(K²+F₂), -F₁], [-F₂, -(K²+F₁)]] / (K²(K²+F₁+F₂)),
    0 at K = 0."""
    K2 = grid.Krsq
    den = K2 * (K2 + p.F1 + p.F2)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = np.where(K2 == 0, 0.0, 1.0 / den)
    q1, q2 = qh[0], qh[1]
    return np.stack([(-(K2 + p.F2) * q1 - p.F1 * q2) * inv, (-p.F2 * q1 - (K2 + p.F1) * q2) * inv])


def mlqg_pvfromstreamfunction(psih, grid: TwoDGrid, p: MLQGParams):
    """pvfromstreamfunction!: q̂ = S ψ̂ (simulation / raytracing set-up)."""
    K2 = grid.Krsq
    return np.stack([(-K2 - p.F1) * psih[0] + p.F1 * psih[1], p.F2 * psih[0] + (-K2 - p.F2) * psih[1]])


def mlqg_calcN(sol, grid: TwoDGrid, p: MLQGParams):
    """MultiLayerQG calcN! (calcN_advection! + bottom drag), op sequence of GF:
    N = -(U+u)·Qx^ - (v Qy)^ - ik((U+u) q)^ - il(v q)^, then
    N_n += μ K² ψ̂_n.  ``sol`` dealiased in place (aliased_fraction = 0 zeroes
    only the Nyquist row and column)."""
    grid.dealias(sol)
    kr = grid.kr[None, :]
    l = grid.l[:, None]
    qh = sol.copy()
    psih = mlqg_streamfunction(qh, grid, p)
    u = grid.irfft(-1j * l * psih) + np.array(p.U)[:, None, None]
    v = grid.irfft(1j * kr * psih)
    N = -grid.rfft(v * np.array(p.Qy)[:, None, None])
    q = grid.irfft(qh)
    N -= 1j * kr * grid.rfft(u * q) + 1j * l * grid.rfft(v * q)
    N[1] += p.mu * grid.Krsq * psih[1]
    return N


def mlqg_L(grid: TwoDGrid, p: MLQGParams):
    """MultiLayerQG Equation: L = -ν K^(2nν) on each layer (the mean-flow,
    background-gradient and drag terms are in calcN), as [2, nl, nkr]."""
    D = -p.nu * grid.Krsq ** p.nnu
    return np.stack([D, D])


def mlqg_linear_operator(grid: TwoDGrid, p: MLQGParams):
    """The full per-mode linearisation of MultiLayerQG about rest (L plus the
    linear part of calcN), [nl, nkr, 2, 2] acting on q̂ — what libsw applies
    as its matvec (the nonlinear J(ψ, q) alone goes through the transforms)."""
    K2 = grid.Krsq
    k = np.broadcast_to(grid.kr[None, :], K2.shape)
    den = K2 * (K2 + p.F1 + p.F2)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = np.where(K2 == 0, 0.0, 1.0 / den)
    Si = np.zeros(K2.shape + (2, 2))
    Si[..., 0, 0] = -(K2 + p.F2) * inv
    Si[..., 0, 1] = -p.F1 * inv
    Si[..., 1, 0] = -p.F2 * inv
    Si[..., 1, 1] = -(K2 + p.F1) * inv
    A = np.zeros(K2.shape + (2, 2), np.complex128)
    D = -p.nu * K2 ** p.nnu
    for j in range(2):
        A[..., j, j] += D - 1j * k * p.U[j]
        A[..., j, :] += -1j * k[..., None] * p.Qy[j] * Si[..., j, :]
    A[..., 1, :] += p.mu * K2[..., None] * Si[..., 1, :]
    return A


def mlqg_energies(sol, grid: TwoDGrid, p: MLQGParams):
    """MultiLayerQG.energies: KE_j = 1/(2 Lx Ly) parsevalsum(K²|ψ̂_j|²) H_j/H,
    PE = 1/(2 Lx Ly) f₀²/g′ parsevalsum(|ψ̂₂ − ψ̂₁|²)/H."""
    psih = mlqg_streamfunction(sol, grid, p)
    Ht = sum(p.H)

    def parsevalsum(fh):
        s = 2 * fh.sum() - fh[:, 0].sum()
        if grid.nx % 2 == 0:
            s -= fh[:, -1].sum()
        return (grid.Lx * grid.Ly / (grid.nx ** 2 * grid.ny ** 2)) * s.real

    KE = [1 / (2 * grid.Lx * grid.Ly) * parsevalsum(grid.Krsq * np.abs(psih[j]) ** 2) * p.H[j] / Ht
          for j in range(2)]
    PE = 1 / (2 * grid.Lx * grid.Ly) * p.f0 ** 2 / p.gp * parsevalsum(np.abs(psih[1] - psih[0]) ** 2) / Ht
    return KE, PE


def mlqg_simulation_params(nx, Lx=2 * np.pi, f=1.0, rd=1 / 15, lv=1 / 2, avg_U=0.1, H0=1.0, nnu=8, nu=0.0):
    """simulation/Parameters.jl compute_parameters and the derived values."""
    c1, c2 = 3.2, 0.36
    l_star = lv / rd
    b2 = 1.0
    kappa_star = c2 / np.log(l_star / c1)
    U = avg_U / l_star
    mu = 2 * U * kappa_star / rd
    b1 = 4 * f ** 2 * rd ** 2 / H0 + b2
    dx = Lx / nx
    return dict(f0=f, H=[H0 / 2, H0 / 2], b=[b1, b2], U=[U, -U], mu=mu, beta=0.0, nu=nu, nnu=nnu,
                dt=0.02 * dx / avg_U, q0_amplitude=1e-2 * avg_U)


# --------------------------------------------------------------------------
# Time steppers
# --------------------------------------------------------------------------
class Clock:
    def __init__(self, dt):
        self.dt, self.t, self.step = float(dt), 0.0, 0


class FilteredAB3:
    """FF ``FilteredAB3TimeStepper`` with ``addlinearterm!`` generalised to the
    per-mode matvec.  Filter kwargs as keywords."""

    def __init__(self, L, grid, nf, order=4, innerK=0.65, outerK=1.0, tol=1e-15):
        self.L = L
        self.filter = makefilter(grid, order=order, innerK=innerK, outerK=outerK, tol=tol)[None]
        shape = (nf, grid.nl, grid.nkr)
        self.RHS = np.zeros(shape, np.complex128)
        self.RHSm1 = np.zeros(shape, np.complex128)
        self.RHSm2 = np.zeros(shape, np.complex128)

    def stepforward(self, sol, clock, calcN, grid, params):
        self.RHS = calcN(sol, grid, params)
        # addlinearterm! (matvec; a diagonal L — MultiLayerQG's — per field)
        self.RHS += mvmul(self.L, sol) if self.L.ndim == 4 else self.L * sol
        if clock.step < 3:
            sol += clock.dt * self.RHS
        else:
            sol += clock.dt * (AB3H1 * self.RHS - AB3H2 * self.RHSm1 + AB3H3 * self.RHSm2)
        sol *= self.filter
        clock.t += clock.dt
        clock.step += 1
        self.RHSm2 = self.RHSm1.copy()
        self.RHSm1 = self.RHS.copy()


class FilteredRK4:
    """FF ``FilteredRK4TimeStepper`` (TwoLayerSimulation's stepper,
    simulation/Parameters.jl:25): RHS = calcN + L·sol (``addlinearterm!``,
    a per-mode matvec for matrix L), RK4 substeps with sol₁ = sol + dt/2 RHS₁,
    sol + dt/2 RHS₂, sol + dt RHS₃, then
    sol += dt (RHS₁/6 + RHS₂/3 + RHS₃/3 + RHS₄/6); sol .*= filter."""

    def __init__(self, L, grid, nf, order=4, innerK=0.65, outerK=1.0, tol=1e-15):
        self.L = L
        self.filter = makefilter(grid, order=order, innerK=innerK, outerK=outerK, tol=tol)[None]

    def _rhs(self, x, calcN, grid, params):
        N = calcN(x, grid, params)
        if self.L.ndim == 4:
            return N + mvmul(self.L, x)
        return N + self.L * x

    def stepforward(self, sol, clock, calcN, grid, params):
        dt = clock.dt
        R1 = self._rhs(sol, calcN, grid, params)
        R2 = self._rhs(sol + dt / 2 * R1, calcN, grid, params)
        R3 = self._rhs(sol + dt / 2 * R2, calcN, grid, params)
        R4 = self._rhs(sol + dt * R3, calcN, grid, params)
        sol += dt * (R1 / 6 + R2 / 3 + R3 / 3 + R4 / 6)
        sol *= self.filter
        clock.t += dt
        clock.step += 1


def live_mask(grid):
    """the (nl, nkr) modes FF's dealias! keeps"""
    return grid.dealias(np.ones((1, grid.nl, grid.nkr), np.complex128))[0] != 0


class IFMAB3:
    """utils/IFMAB3.jl:68-88, 128-169 (CPU method)."""

    def __init__(self, L, dt, grid, nf, use_filter=False, diagonal=False, expm="scipy", **filter_kw):
        self.expm = expm
        self.expLdt = expm_modes(L * dt, expm, scipy_split(grid))
        self.exp2Ldt = expm_modes(L * 2 * dt, expm, scipy_split(grid))
        shape = (nf, grid.nl, grid.nkr)
        self.N = np.zeros(shape, np.complex128)
        self.Nm1 = np.zeros(shape, np.complex128)
        self.Nm2 = np.zeros(shape, np.complex128)
        if use_filter:
            self.filter = makefilter(grid, **filter_kw)[None]
        else:
            self.filter = np.ones((1, grid.nl, grid.nkr))

    def stepforward(self, sol, clock, calcN, grid, params):
        self.N = calcN(sol, grid, params)                            # :158
        if clock.step < 3:                                           # :130-132
            sol += clock.dt * self.N
            sol[...] = mvmul(self.expLdt, sol)
        else:                                                        # :134-137
            eN1 = mvmul(self.expLdt, self.Nm1)
            e2N2 = mvmul(self.exp2Ldt, self.Nm2)
            sol += clock.dt * (AB3H1 * self.N - AB3H2 * eN1 + AB3H3 * e2N2)
            sol[...] = mvmul(self.expLdt, sol)
        sol *= self.filter                                           # :160
        clock.t += clock.dt
        clock.step += 1
        self.Nm2 = self.Nm1.copy()                                   # :165-166
        self.Nm1 = self.N.copy()


class IFMRK4:
    """Lawson integrating-factor RK4, the build's definition of the draft
    utils/IFMRK4.jl (struct fields expLdt, expL½dt, k₁..k₄, filter at :13-22;
    four calcN! evaluations at :157-163).  SURVEY §8a A9:
      k1 = N(u); k2 = N(H(u + dt/2 k1)); k3 = N(H u + dt/2 k2);
      k4 = N(E u + dt H k3); u <- E u + dt/6 (E k1 + 2H(k2 + k3) + k4); filter.
    """

    def __init__(self, L, dt, grid, nf, use_filter=False, expm="scipy", **filter_kw):
        self.expm = expm
        self.expLdt = expm_modes(L * dt, expm, scipy_split(grid))
        self.expLhdt = expm_modes(L * 0.5 * dt, expm, scipy_split(grid))
        if use_filter:
            self.filter = makefilter(grid, **filter_kw)[None]
        else:
            self.filter = np.ones((1, grid.nl, grid.nkr))

    def stepforward(self, sol, clock, calcN, grid, params):
        dt = clock.dt
        E, H = self.expLdt, self.expLhdt
        k1 = calcN(sol, grid, params)                 # dealiases sol in place
        x = mvmul(H, sol + 0.5 * dt * k1)
        k2 = calcN(x, grid, params)
        x = mvmul(H, sol) + 0.5 * dt * k2
        k3 = calcN(x, grid, params)
        x = mvmul(E, sol) + dt * mvmul(H, k3)
        k4 = calcN(x, grid, params)
        sol[...] = mvmul(E, sol) + dt / 6 * (mvmul(E, k1) + 2 * mvmul(H, k2 + k3) + k4)
        sol *= self.filter
        clock.t += dt
        clock.step += 1


def etdrk4_coeffs(dt, L, ncirc=32, rcirc=1.0):
    """FF ``getetdcoeffs(dt, L; ncirc=32, rcirc=1)`` for a real diagonal L
    (FourierFlows.jl timesteppers; not vendored in the reference — restated
    from its published Cox–Matthews / Kassam–Trefethen contour form): the
    mean over ``ncirc`` points z = dt L + r e^{2πi (j+1/2)/ncirc} of
      ζ = (e^{z/2} - 1)/z,  α = (-4 - z + e^z (4 - 3z + z²))/z³,
      β = (2 + z + e^z (z - 2))/z³,  Γ = (-4 - 3z - z² + e^z (4 - z))/z³,
    each times dt, real part (L real)."""
    circ = rcirc * np.exp(2j * np.pi / ncirc * (np.arange(ncirc) + 0.5))
    zc = dt * L[..., None] + circ
    ez = np.exp(zc)
    z3 = zc ** 3
    zeta = (np.exp(zc / 2) - 1) / zc
    alpha = (-4 - zc + ez * (4 - 3 * zc + zc ** 2)) / z3
    beta = (2 + zc + ez * (-2 + zc)) / z3
    gamma = (-4 - 3 * zc - zc ** 2 + ez * (4 - zc)) / z3
    return tuple(dt * np.real(c.mean(axis=-1)) for c in (zeta, alpha, beta, gamma))


class ETDRK4:
    """FF ``ETDRK4TimeStepper`` (the stepper ThomasYamada.Problem defaults to,
    thomasyamada/ThomasYamada.jl:60, cpu-setup/Parameters.jl:12): with
    E = e^{dt L}, E2 = e^{dt L/2} and the contour coefficients
      N1 = N(u);        s1 = E2 u + ζ N1
      N2 = N(s1);       s2 = E2 u + ζ N2
      N3 = N(s2);       s2 = E2 s1 + ζ (2 N3 - N1)
      N4 = N(s2);       u  = E u + α N1 + 2β (N2 + N3) + Γ N4."""

    def __init__(self, L, dt, grid, nf):
        self.expLdt = np.exp(dt * L)
        self.expLdt2 = np.exp(dt * L / 2)
        self.zeta, self.alpha, self.beta, self.gamma = etdrk4_coeffs(dt, L)

    def stepforward(self, sol, clock, calcN, grid, params):
        E, E2, z = self.expLdt, self.expLdt2, self.zeta
        N1 = calcN(sol, grid, params)
        s1 = E2 * sol + z * N1
        N2 = calcN(s1, grid, params)
        s2 = E2 * sol + z * N2
        N3 = calcN(s2, grid, params)
        s2 = E2 * s1 + z * (2 * N3 - N1)
        N4 = calcN(s2, grid, params)
        sol[...] = E * sol + self.alpha * N1 + 2 * self.beta * (N2 + N3) + self.gamma * N4
        clock.t += clock.dt
        clock.step += 1


# --------------------------------------------------------------------------
# Problems and driver formulas
# --------------------------------------------------------------------------
class Problem:
    """Mirror of ``RotatingShallowWater.Problem`` / ``TwoLayerQG.Problem`` for
    the oracle (model in {"rsw", "qg2"}, stepper in {"FilteredAB3", "IFMAB3",
    "IFMRK4"}, or "NOP" calcN for the linear-only check)."""

    def __init__(self, model, stepper, nx, dt, Lx=2 * np.pi, aliased_fraction=1 / 3,
                 params=None, use_filter=False, calcN=None, ny=None, Ly=None, expm="scipy", **filter_kw):
        # expm: the integrating factors' matrix exponential (expm_modes)
        # model "ty" (thomasyamada/ThomasYamada.jl:55-74) takes stepper "ETDRK4"
        self.grid = TwoDGrid(nx, Lx, ny=ny, Ly=Ly, aliased_fraction=aliased_fraction)
        self.params = params
        self.model = model
        if model == "rsw":
            self.nf = 3
            self.L = rsw_L(self.grid, params)
            self.calcN = rsw_calcN if calcN is None else calcN
        elif model == "qg2":
            self.nf = 2
            self.L = qg2_L(self.grid, params)
            self.calcN = qg2_calcN if calcN is None else calcN
        elif model == "ty":
            self.nf = 4
            self.L = ty_L(self.grid, params)
            self.calcN = ty_calcN if calcN is None else calcN
            if stepper != "ETDRK4":
                raise ValueError("the Thomas-Yamada model is stepped with ETDRK4")
        elif model == "mlqg":
            self.nf = 2
            self.L = mlqg_L(self.grid, params)
            self.calcN = mlqg_calcN if calcN is None else calcN
        else:
            raise ValueError(model)
        self.clock = Clock(dt)
        if stepper == "ETDRK4":
            if model != "ty":
                raise ValueError("ETDRK4 needs a diagonal L (Thomas-Yamada)")
            self.ts = ETDRK4(self.L, dt, self.grid, self.nf)
        elif stepper == "FilteredAB3":
            self.ts = FilteredAB3(self.L, self.grid, self.nf, **filter_kw)
        elif stepper == "FilteredRK4":
            self.ts = FilteredRK4(self.L, self.grid, self.nf, **filter_kw)
        elif stepper == "IFMAB3":
            self.ts = IFMAB3(self.L, dt, self.grid, self.nf, use_filter=use_filter, expm=expm, **filter_kw)
        elif stepper == "IFMRK4":
            self.ts = IFMRK4(self.L, dt, self.grid, self.nf, use_filter=use_filter, expm=expm, **filter_kw)
        else:
            raise ValueError(stepper)
        self.sol = np.zeros((self.nf, self.grid.nl, self.grid.nkr), np.complex128)

    def set_solution(self, solh):
        """set_solution! (rsw/RotatingShallowWater.jl:309-321): copies then
        updatevars! which dealiases the state in place (:104)."""
        self.sol[...] = solh
        self.grid.dealias(self.sol)

    def stepforward(self, nsteps=1):
        for _ in range(nsteps):
            self.ts.stepforward(self.sol, self.clock, self.calcN, self.grid, self.params)


def rsw_driver_params(nx, Lx=2 * np.pi, aliased_fraction=1 / 3, nnu=4, nutune=20.0,
                      cfltune=0.01, ag=0.2, aw=0.1):
    """rsw/RSWDriver.jl:134-148 (defaults from rsw/RSWParameters.jl)."""
    dx = Lx / nx
    kmax = (nx / 2 - 1) * Lx / (2 * np.pi) * (1 - aliased_fraction)
    umax = ag + aw
    dt = cfltune / umax * dx
    nu = nutune * dx / (kmax ** (2 * nnu)) / dt
    return dt, nu


def fab3_linear_growth(grid: TwoDGrid, p: RSWParams, dt, order=8):
    """Largest per-step amplification |z| over the live modes of the linear
    RSW FilteredAB3 scheme (FF FilteredAB3, SURVEY A7, with the filter applied
    after the update): sol_{n+1} = filt·(sol_n + dt(23/12 λ sol_n − 16/12 λ
    sol_{n−1} + 5/12 λ sol_{n−2})) for each eigenvalue λ of the per-mode L
    (rsw/RotatingShallowWater.jl:242-260): D and D ± iω, D = −ν K^(2nν),
    ω² = f² + Cg² K².  |z| > 1 means the explicit hyperviscosity outruns the
    filter and the driver's run blows up (rsw/RSWDriver.jl:213-218)."""
    K2 = grid.Krsq
    D = -p.nu * K2 ** p.nnu
    w = np.sqrt(p.f ** 2 + p.Cg2 * K2)
    filt = makefilter(grid, order=order)
    live = grid.live
    worst = 0.0
    for lam in (D, D + 1j * w, D - 1j * w):
        a = dt * lam[live]
        F = filt[live]
        co = np.stack([-F * (1 + 23 / 12 * a), F * 16 / 12 * a, -F * 5 / 12 * a], -1)
        C = np.zeros((a.size, 3, 3), complex)
        C[:, 0, :] = -co
        C[:, 1, 0] = 1
        C[:, 2, 1] = 1
        worst = max(worst, float(np.abs(np.linalg.eigvals(C)).max()))
    return worst


def qg2_compute_parameters(deformation_radius, intervortex_radius, avg_eddy_velocity, H, f0):
    """swqg/TwoLayerDriver.jl:17-27."""
    c1, c2 = 3.2, 0.36
    l_star = intervortex_radius / deformation_radius
    kappa_star = c2 / np.log(l_star / c1)
    U = avg_eddy_velocity / l_star
    mu = 2 * U * kappa_star / deformation_radius
    db = 4 * f0 ** 2 * deformation_radius ** 2 / H
    return mu, db, U


def qg2_driver_params(nx, Lx=2 * np.pi, aliased_fraction=1 / 3, nnu=4, nutune=40.0,
                      cfltune=0.025, ug=0.025, f=3.0, Cg=1.0, rd=1 / 6, lv=1.0, H=1.0):
    """swqg/TwoLayerDriver.jl:29-63 (defaults from swqg/TwoLayerParameters.jl)."""
    dx = Lx / nx
    kmax = (nx / 2 - 1) * (1 - aliased_fraction)
    mu, db, U = qg2_compute_parameters(rd, lv, ug, H, f)
    drr0 = db / (Cg / H)
    dt = cfltune / ug * dx
    nu = nutune * 2 * np.pi / nx / (kmax ** (2 * nnu)) / dt
    F = 2 * f ** 2 / Cg ** 2 / drr0
    return dict(dt=dt, nu=nu, U=U, mu=mu, drhorho0=drr0, F=F, f0=f, Cg=Cg)


def shafer_ic_parts(grid: TwoDGrid, Kg, Kw, f, Cg2, rng):
    """Spectral pieces of ``set_shafer_initial_condition!`` before the Umax
    normalisation (rsw/RSWDriver.jl:93-106, 118-120).  Julia's RNG stream is
    not reproducible here: ``rng`` is a numpy Generator (seeded by the caller)
    drawing phase = 2π·U[0,1) then sgn = sign(U[0,1) - 0.5), each over
    (nkr, nl) in Julia column-major order."""
    K2 = grid.Krsq
    geo = (Kg[0] ** 2 <= K2) & (K2 <= Kg[1] ** 2) & (K2 > 0)
    wav = (Kw[0] ** 2 <= K2) & (K2 <= Kw[1] ** 2) & (K2 > 0)
    phase = 2 * np.pi * rng.random((grid.nkr, grid.nl)).T
    sgn = np.sign(rng.random((grid.nkr, grid.nl)).T - 0.5)
    shift = np.exp(1j * phase)
    om = np.sqrt(f ** 2 + Cg2 * K2)
    gamp = 1 / om
    with np.errstate(divide="ignore", invalid="ignore"):
        wamp = np.sqrt(grid.invKrsq) / (2 * om)
    kr = np.broadcast_to(grid.kr[None, :], K2.shape)
    l = np.broadcast_to(grid.l[:, None], K2.shape)
    z = np.zeros(K2.shape, np.complex128)
    ugh, vgh, egh = z.copy(), z.copy(), z.copy()
    uwh, vwh, ewh = z.copy(), z.copy(), z.copy()
    egh[geo] += (gamp * f * shift)[geo]
    ugh[geo] += (-gamp * 1j * Cg2 * l * shift)[geo]
    vgh[geo] += (gamp * 1j * Cg2 * kr * shift)[geo]
    ewh[wav] += (wamp * K2 * shift)[wav]
    uwh[wav] += (wamp * (sgn * kr * om * shift + 1j * f * l * shift))[wav]
    vwh[wav] += (wamp * (sgn * l * om * shift - 1j * f * kr * shift))[wav]
    return (ugh, vgh, egh), (uwh, vwh, ewh)


def shafer_ic(grid: TwoDGrid, Kg, Kw, ag, aw, f, Cg2, rng):
    """rsw/RSWDriver.jl:88-132 with numpy's c2r for the Umax normalisation."""
    (ugh, vgh, egh), (uwh, vwh, ewh) = shafer_ic_parts(grid, Kg, Kw, f, Cg2, rng)
    ug, vg = grid.irfft(ugh), grid.irfft(vgh)
    Umax = np.max(np.sqrt(ug ** 2 + vg ** 2))
    ugh, vgh, egh = ugh * (ag / Umax), vgh * (ag / Umax), egh * (ag / Umax)
    uw, vw = grid.irfft(uwh), grid.irfft(vwh)
    Umax = np.max(np.sqrt(uw ** 2 + vw ** 2))
    uwh, vwh, ewh = uwh * (aw / Umax), vwh * (aw / Umax), ewh * (aw / Umax)
    return np.stack([ugh + uwh, vgh + vwh, egh + ewh])


def qg2_seed_ic(grid: TwoDGrid, rng):
    """swqg/TwoLayerDriver.jl:10-15: q0 = 1e-2·randn(nx, ny, 2); rfft over (1,2)."""
    q0 = 1e-2 * rng.standard_normal((2, grid.ny, grid.nx))
    return grid.rfft(q0)


def parity_error(a, b, grid: TwoDGrid):
    """SURVEY §8c metric: max|a-b| / max|b| over the dealias-masked state."""
    m = grid.live[None]
    den = np.max(np.abs(np.where(m, b, 0)))
    num = np.max(np.abs(np.where(m, a - b, 0)))
    return num / den if den > 0 else num
