"""Galerkin invariants of the dealiased nonlinear terms (test helper).

The 2/3 rule makes every retained mode of a quadratic product exact, so the
retained part of the nonlinear term N is the exact Galerkin projection of the
continuous one.  Paired with a field that is itself retained-only, N then
obeys the continuous identities exactly (up to roundoff):

* TwoLayerQG (swqg/TwoLayerQG.jl:152-182, N_j = -J(ψ_j, q_j) per layer):
  ⟨q_j, N_j⟩ = 0 (enstrophy) and ⟨ψ_j, N_j⟩ = 0 (energy), any q;
* RotatingShallowWater (rsw/RotatingShallowWater.jl:140-230, advective form)
  for a divergence-free velocity (u, v) = (-∂y ψ, ∂x ψ) and any η:
  ⟨u, N_u⟩ = 0 and ⟨v, N_v⟩ = 0 (each is ∫ (u²/2) ∇·u, resp. v²),
  ⟨ζ, ∂x N_v - ∂y N_u⟩ = 0 and ⟨η, N_η⟩ = 0;
* ThomasYamada (thomasyamada/ThomasYamada.jl:129-262; N holds the rotation
  and pressure terms too), any state: the total energy
  ½∫(|∇ψ_T|² + u_c² + v_c² + p_c²) is conserved by N,
  -⟨ψ_T, N_ζ⟩ + ⟨u_c, N_u⟩ + ⟨v_c, N_v⟩ + ⟨p_c, N_p⟩ = 0 (ψ_T = -ζ_T/K²).

These identities are independent of the oracle (and of the reference): they
pin the nonlinear transform chain against the equations themselves, at any
size.  They do not see a constant factor on N; the oracle comparisons do.
⟨a, b⟩ is the real inner product over the full Hermitian spectrum held in
the rfft half (weight 2 on 0 < kr < nx/2)."""
import numpy as np


def inner(a, b):
    nkr = a.shape[-1]
    w = np.full(nkr, 2.0)
    w[0] = 1.0
    w[-1] = 1.0  # kr = nx/2 (nkr = nx/2 + 1)
    return float(np.sum(w * (np.conj(a) * b).real))


def rel(a, b):
    """|⟨a, b⟩| / (‖a‖ ‖b‖)"""
    return abs(inner(a, b)) / np.sqrt(inner(a, a) * inner(b, b))


def random_real_spectrum(grid, nf, seed):
    """rfft of seeded white noise, dealiased: nf real fields."""
    rng = np.random.default_rng(seed)
    fh = grid.rfft(rng.standard_normal((nf, grid.ny, grid.nx)))
    return grid.dealias(fh)


def rsw_state(grid, seed):
    """(û, v̂, η̂) with (u, v) = (-∂y ψ, ∂x ψ): divergence-free."""
    f = random_real_spectrum(grid, 2, seed)
    kr, l = grid.kr[None, :], grid.l[:, None]
    return np.stack([-1j * l * f[0], 1j * kr * f[0], f[1]])


def rsw_residuals(grid, sol, N):
    kr, l = grid.kr[None, :], grid.l[:, None]
    zeta = 1j * kr * sol[1] - 1j * l * sol[0]
    Nzeta = 1j * kr * N[1] - 1j * l * N[0]
    return {"u": rel(sol[0], N[0]), "v": rel(sol[1], N[1]), "vorticity": rel(zeta, Nzeta), "eta": rel(sol[2], N[2])}


def qg2_residuals(grid, q, psi, N):
    out = {}
    for j in range(2):
        out[f"enstrophy{j + 1}"] = rel(q[j], N[j])
        out[f"energy{j + 1}"] = rel(psi[j], N[j])
    return out


def ty_residuals(grid, sol, N):
    """the energy budget of N relative to the size of its terms"""
    psi = -sol[0] * grid.invKrsq
    t = [-inner(psi, N[0])] + [inner(sol[f], N[f]) for f in (1, 2, 3)]
    return {"energy": abs(sum(t)) / sum(abs(x) for x in t)}
