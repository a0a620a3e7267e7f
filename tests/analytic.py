"""Closed-form nonlinear terms of few-mode states (test infrastructure).

An independent pin of calcN, built on neither the oracle nor an FFT: each
physical field is a short sum of trigonometric terms ``a·cos(m·x)`` /
``a·sin(m·x)`` with integer wavevectors m = (m_x, m_y) on the 2π-periodic
domain.  Derivatives and products are expanded with the product-to-sum
identities, and the result is written straight into the rfft2 (FFTW r2c,
unnormalised) array the reference's ``calcN!`` fills:

* RSW (rsw/RotatingShallowWater.jl:140-230):
  N_u = −(u u_x + v u_y)^, N_v = −(u v_x + v v_y)^,
  N_η = −ik (u η)^ − il (v η)^;
* 2LQG (swqg/TwoLayerQG.jl:152-182, 101-111): ψ̂ = S⁻¹ q̂ per mode,
  N = −il (ψ_x q)^ + ik (ψ_y q)^;
* Thomas–Yamada (thomasyamada/ThomasYamada.jl:129-262), ty_N;
* GeophysicalFlows MultiLayerQG (two layers, simulation/TwoLayerSimulation.jl),
  mlqg_N (restated: GF is not vendored).

With every sum and difference wavevector inside the 2/3-rule live band, the
pseudo-spectral product is exact, so calcN must reproduce these arrays to
rounding.
"""
from __future__ import annotations

import numpy as np

# a term: (amplitude, kind "c" | "s", (mx, my)); a field: list of terms


def _canon(term):
    a, kind, (mx, my) = term
    if (mx, my) == (0, 0):
        return [(a, "c", (0, 0))] if kind == "c" else []
    if mx < 0 or (mx == 0 and my < 0):  # cos(-θ) = cos θ, sin(-θ) = -sin θ
        return [(a if kind == "c" else -a, kind, (-mx, -my))]
    return [(a, kind, (mx, my))]


def simplify(f):
    acc = {}
    for t in f:
        for a, kind, m in _canon(t):
            acc[(kind, m)] = acc.get((kind, m), 0.0) + a
    return [(a, k, m) for (k, m), a in acc.items() if a != 0.0]


def dx(f, axis):
    """∂/∂x (axis 0) or ∂/∂y (axis 1) of a trig field."""
    out = []
    for a, kind, m in f:
        k = m[axis]
        out.append((-a * k, "s", m) if kind == "c" else (a * k, "c", m))
    return simplify(out)


def mul(f, g):
    """Product of two trig fields (product-to-sum identities)."""
    out = []
    for a, ka, ma in f:
        for b, kb, mb in g:
            s = (ma[0] + mb[0], ma[1] + mb[1])
            d = (ma[0] - mb[0], ma[1] - mb[1])
            h = 0.5 * a * b
            if ka == "c" and kb == "c":
                out += [(h, "c", d), (h, "c", s)]
            elif ka == "s" and kb == "s":
                out += [(h, "c", d), (-h, "c", s)]
            elif ka == "s" and kb == "c":
                out += [(h, "s", s), (h, "s", d)]
            else:  # cos · sin
                out += [(h, "s", s), (-h, "s", d)]
    return simplify(out)


def add(*fs, scale=None):
    out = []
    for i, f in enumerate(fs):
        c = 1.0 if scale is None else scale[i]
        out += [(c * a, k, m) for a, k, m in f]
    return simplify(out)


def spectrum(f, nx, ny):
    """rfft2 array [ny][nx/2+1] of a trig field sampled on the nx × ny grid
    (x = 2π i/nx): a cos(m·x) puts a·nx·ny/2 at ±m, a sin(m·x) puts
    ∓i a·nx·ny/2 at ±m; only m_x >= 0 is stored (both ±m_y at m_x = 0)."""
    out = np.zeros((ny, nx // 2 + 1), np.complex128)
    half = nx * ny / 2
    for a, kind, (mx, my) in simplify(f):  # canonical: mx > 0, or mx == 0 < my
        if (mx, my) == (0, 0):
            out[0, 0] += a * nx * ny
            continue
        cp = a * half if kind == "c" else -1j * a * half  # sin θ = (e^{iθ} - e^{-iθ}) / 2i
        out[my % ny, mx] += cp
        if mx == 0:  # the -m partner is stored too in the kr = 0 column
            out[(-my) % ny, 0] += np.conj(cp)
    return out


def scale_field(f, c):
    return [(c * a, k, m) for a, k, m in f]


# --- model nonlinear terms ---------------------------------------------------

def rsw_N(u, v, eta):
    """(N_u, N_v, N_η) trig fields (rsw/RotatingShallowWater.jl:140-230)."""
    nu = add(mul(u, dx(u, 0)), mul(v, dx(u, 1)), scale=(-1.0, -1.0))
    nv = add(mul(u, dx(v, 0)), mul(v, dx(v, 1)), scale=(-1.0, -1.0))
    ne = add(dx(mul(u, eta), 0), dx(mul(v, eta), 1), scale=(-1.0, -1.0))
    return nu, nv, ne


def qg2_psi(q1, q2, F):
    """ψ per layer from q per mode (swqg/TwoLayerQG.jl:101-111):
    ψ̂ = −[(K²+F) q̂1 + F q̂2, F q̂1 + (K²+F) q̂2] / (K²+2F) / K², 0 at K = 0.
    Both layers must be built on the same wavevector set."""
    p1, p2 = [], []
    d2 = {(k, m): a for a, k, m in simplify(q2)}
    keys = {(k, m) for _, k, m in simplify(q1)} | set(d2)
    d1 = {(k, m): a for a, k, m in simplify(q1)}
    for k, m in keys:
        K2 = float(m[0] ** 2 + m[1] ** 2)
        if K2 == 0:
            continue
        a1, a2 = d1.get((k, m), 0.0), d2.get((k, m), 0.0)
        den = (K2 + 2 * F) * K2
        p1.append((-((K2 + F) * a1 + F * a2) / den, k, m))
        p2.append((-(F * a1 + (K2 + F) * a2) / den, k, m))
    return simplify(p1), simplify(p2)


def qg2_N(q1, q2, F):
    """N_j = −∂y(ψ_x q)_j + ∂x(ψ_y q)_j (swqg/TwoLayerQG.jl:152-182)."""
    out = []
    for q, psi in zip((q1, q2), qg2_psi(q1, q2, F)):
        out.append(add(dx(mul(dx(psi, 0), q), 1), dx(mul(dx(psi, 1), q), 0), scale=(-1.0, 1.0)))
    return out


def _K2(m):
    return float(m[0] ** 2 + m[1] ** 2)


def ty_N(zt, uc, vc, pc, Ro):
    """(N_ζ, N_uc, N_vc, N_pc) of Thomas–Yamada (thomasyamada/ThomasYamada.jl
    :129-262) on the 2π domain: ψ_T = −ζ/K² per mode (:125-127), u_T = −∂y ψ_T,
    v_T = ∂x ψ_T (:138-139); linear terms (:142-145) plus
      N_ζ  −= Ro [∂y(v_T ζ) + ∂x(u_T ζ) + (∂xx − ∂yy)(u_c v_c) + ∂x∂y(v_c² − u_c²)]   (:166-202)
      N_uc −= Ro [∂x(u_T u_c) + v_T ∂y u_c + v_c ∂y u_T]                            (:204-234)
      N_vc −= Ro [∂y(v_T v_c) + u_T ∂x v_c + u_c ∂x v_T]                            (:235-249)
      N_pc −= Ro [u_T ∂x p_c + v_T ∂y p_c]                                          (:251-266)"""
    psi = simplify([(-a / _K2(m), k, m) for a, k, m in simplify(zt) if m != (0, 0)])
    ut, vt = scale_field(dx(psi, 1), -1.0), dx(psi, 0)
    uv = mul(uc, vc)
    nz = add(dx(mul(vt, zt), 1), dx(mul(ut, zt), 0), dx(dx(uv, 0), 0), scale_field(dx(dx(uv, 1), 1), -1.0),
             dx(dx(mul(vc, vc), 0), 1), scale_field(dx(dx(mul(uc, uc), 0), 1), -1.0),
             scale=(-Ro,) * 6)
    nu = add(vc, scale_field(dx(pc, 0), -1.0),
             dx(mul(ut, uc), 0), mul(vt, dx(uc, 1)), mul(vc, dx(ut, 1)), scale=(1.0, 1.0, -Ro, -Ro, -Ro))
    nv = add(scale_field(uc, -1.0), scale_field(dx(pc, 1), -1.0),
             dx(mul(vt, vc), 1), mul(ut, dx(vc, 0)), mul(uc, dx(vt, 0)), scale=(1.0, 1.0, -Ro, -Ro, -Ro))
    npc = add(scale_field(dx(uc, 0), -1.0), scale_field(dx(vc, 1), -1.0),
              mul(ut, dx(pc, 0)), mul(vt, dx(pc, 1)), scale=(1.0, 1.0, -Ro, -Ro))
    return nz, nu, nv, npc


def mlqg_psi(q1, q2, F1, F2):
    """GeophysicalFlows MultiLayerQG streamfunctionfrompv! for two layers:
    ψ̂ = S⁻¹ q̂, S = [[−K²−F₁, F₁], [F₂, −K²−F₂]], 0 at K = 0."""
    d1 = {(k, m): a for a, k, m in simplify(q1)}
    d2 = {(k, m): a for a, k, m in simplify(q2)}
    p1, p2 = [], []
    for k, m in set(d1) | set(d2):
        K2 = _K2(m)
        if K2 == 0:
            continue
        a1, a2 = d1.get((k, m), 0.0), d2.get((k, m), 0.0)
        den = K2 * (K2 + F1 + F2)
        p1.append((-((K2 + F2) * a1 + F1 * a2) / den, k, m))
        p2.append((-(F2 * a1 + (K2 + F1) * a2) / den, k, m))
    return simplify(p1), simplify(p2)


def mlqg_N(q1, q2, F1, F2, U, Qy, mu):
    """MultiLayerQG calcN! (two layers, no topography): per layer j with
    u_j = −∂y ψ_j, v_j = ∂x ψ_j,
      N_j = −Qy_j v_j − ∂x((U_j + u_j) q_j) − ∂y(v_j q_j),
    and the bottom drag N₂ += μ K² ψ̂₂ (= −μ ∇²ψ₂)."""
    out = []
    psis = mlqg_psi(q1, q2, F1, F2)
    for j, (q, psi) in enumerate(zip((q1, q2), psis)):
        u, v = scale_field(dx(psi, 1), -1.0), dx(psi, 0)
        out.append(add(v, dx(q, 0), dx(mul(u, q), 0), dx(mul(v, q), 1), scale=(-Qy[j], -U[j], -1.0, -1.0)))
    out[1] = add(out[1], [(mu * _K2(m) * a, k, m) for a, k, m in psis[1]])
    return out


# --- the few-mode states used by the tests ----------------------------------

def rsw_triad():
    """u, v, η on three wavevectors whose sums and differences stay below
    K = 12 (inside the live band of a 64² grid, kmax = 21)."""
    u = [(0.7, "c", (1, 2)), (-0.3, "s", (3, -1))]
    v = [(0.5, "s", (2, 1)), (0.2, "c", (1, 2))]
    eta = [(0.4, "c", (3, -1)), (-0.25, "s", (0, 4)), (0.1, "c", (2, 1))]
    return u, v, eta


def qg2_triad():
    q1 = [(0.8, "c", (1, 3)), (-0.4, "s", (4, -2)), (0.3, "c", (2, 2))]
    q2 = [(0.5, "s", (1, 3)), (0.6, "c", (4, -2)), (-0.2, "s", (0, 5))]
    return q1, q2


def qg2_shell(c=0.7):
    """q2 = c·q1 on one |K|² = 25 shell: ψ_j ∝ q1, so J(ψ_j, q_j) = 0 exactly
    although each product ψ_x q_y, ψ_y q_x is O(1)."""
    q1 = [(0.6, "c", (3, 4)), (-0.5, "s", (5, 0)), (0.45, "c", (4, -3)), (0.3, "s", (0, 5))]
    return q1, scale_field(q1, c)


def ty_quad():
    """ζ_T, u_c, v_c, p_c on a few wavevectors (all sums and differences
    below K = 12: inside the live band of a 64² grid)."""
    zt = [(0.9, "c", (1, 2)), (-0.5, "s", (2, -1)), (0.3, "c", (0, 3))]
    uc = [(0.4, "s", (1, 1)), (0.25, "c", (3, 0))]
    vc = [(-0.35, "c", (1, 1)), (0.2, "s", (2, 2))]
    pc = [(0.15, "c", (2, 1)), (-0.1, "s", (1, -3))]
    return zt, uc, vc, pc


def mlqg_pair():
    q1 = [(0.8, "c", (1, 2)), (-0.3, "s", (3, -1)), (0.25, "c", (0, 2))]
    q2 = [(0.4, "s", (1, 2)), (0.5, "c", (2, 2)), (-0.2, "s", (3, 0))]
    return q1, q2


def state(fields, n):
    return np.stack([spectrum(f, n, n) for f in fields])
