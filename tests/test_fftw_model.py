"""Host model of the wave-decimated row transforms (csrc/sw_fft.hpp
fftw_dif / fftw_dit / fftw_dit_split), checked against numpy's FFT.

The GPU kernels are checked against the oracle by the -m gpu parity tests;
this is the index algebra alone, thread by thread, so a change to the
register/region mapping is caught on CPU.  N = 512·W points over W waves
(NT = 64 W threads, 8 points each, Q = 512 per wave):

  DIF  X[W m + c] = Σ_n ω_Q^(nm) ω^(nc) Σ_q x[n + Qq] ω_W^(qc)
       thread t holds x[t + NT s]; n = t + NT h (h < 8/W) and x[n + Qq] is
       register h + (8/W) q; on exit lane j of wave c holds X[W (j + 64 r) + c]
  DIT  X[k + Qp] = Σ_c ω_W^(cp) ω^(ck) DFT_Q(x[W m + c])[k], natural out
  split (two real signals z = a + i b): A_c[k] = (Y_c[k] + conj Y_c[Q-k]) / 2 …
"""
import numpy as np
import pytest

Q = 512


def _omega(n, sign):
    return np.exp(sign * 2j * np.pi / n)


def dif_model(x, W, sign):
    """Registers after fftw_dif: out[c][j, r] = X[W (j + 64 r) + c]."""
    N, NT, HN = Q * W, 64 * W, 8 // W
    v = np.array([[x[t + NT * s] for s in range(8)] for t in range(NT)])  # thread t, slot s
    regions = np.zeros((W, Q), complex)
    w = _omega(N, sign)
    for t in range(NT):
        for h in range(HN):
            a = np.array([v[t, h + HN * q] for q in range(W)])
            y = np.array([sum(a[q] * _omega(W, sign) ** (q * c) for q in range(W)) for c in range(W)])
            n = t + NT * h
            for c in range(W):
                regions[c, n] = y[c] * w ** (n * c)  # ω^(ct) ω_8^(hc) = ω^(c n)
    out = np.zeros((W, 64, 8), complex)
    for c in range(W):
        Y = np.fft.fft(regions[c]) if sign < 0 else np.fft.ifft(regions[c]) * Q  # the wave's Q-point transform
        for j in range(64):
            for r in range(8):
                out[c, j, r] = Y[j + 64 * r]
    return out


def dit_model(dec, W, sign):
    """fftw_dit from the DIF's order: returns v[t, s] = X[t + NT s]."""
    N, NT, HN = Q * W, 64 * W, 8 // W
    w = _omega(N, sign)
    Y = np.zeros((W, Q), complex)
    for c in range(W):
        xc = np.array([dec[c, j, s] for s in range(8) for j in range(64)])  # m = j + 64 s ↔ index
        m = np.array([j + 64 * s for s in range(8) for j in range(64)])
        seq = np.zeros(Q, complex)
        seq[m] = xc
        Y[c] = np.fft.fft(seq) if sign < 0 else np.fft.ifft(seq) * Q
    v = np.zeros((NT, 8), complex)
    for t in range(NT):
        for h in range(HN):
            k = t + NT * h
            a = np.array([Y[c, k] * w ** (c * k) for c in range(W)])
            for p in range(W):
                v[t, h + HN * p] = sum(a[c] * _omega(W, sign) ** (c * p) for c in range(W))
    return v


@pytest.mark.parametrize("W", [2, 4, 8])
def test_dif_decimated_order(W):
    rng = np.random.default_rng(W)
    N = Q * W
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    X = np.fft.ifft(x) * N  # inverse, unnormalised (DIR = +1)
    out = dif_model(x, W, +1)
    for c in range(W):
        for j in range(0, 64, 7):
            for r in range(8):
                assert abs(out[c, j, r] - X[W * (j + 64 * r) + c]) < 1e-9 * N


@pytest.mark.parametrize("W", [2, 4, 8])
def test_dit_from_dif_order_is_natural(W):
    """Inverse DIF then forward DIT: the round trip is N·x in natural order,
    i.e. the DIT reads exactly the order the DIF leaves."""
    rng = np.random.default_rng(10 + W)
    N, NT = Q * W, 64 * W
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    dec = dif_model(x, W, +1)
    v = dit_model(dec, W, -1)
    got = np.array([v[t % NT, t // NT] for t in range(N)])
    assert np.max(np.abs(got - N * x)) < 1e-9 * N


def test_split_fold_identity():
    """fftw_dit_split: splitting each wave's sub-spectrum before the radix-W
    combination equals splitting the natural-order spectrum after it."""
    W = 4
    N, NT = Q * W, 64 * W
    rng = np.random.default_rng(3)
    a, b = rng.standard_normal(N), rng.standard_normal(N)
    Z = np.fft.fft(a + 1j * b)
    A_ref, B_ref = np.fft.fft(a), np.fft.fft(b)
    w = _omega(N, -1)
    Y = np.array([np.fft.fft((a + 1j * b)[c::W]) for c in range(W)])  # wave c: x[W m + c]
    for k in range(0, Q, 37):
        km = (Q - k) % Q
        Ac = (Y[:, k] + np.conj(Y[:, km])) / 2
        Bc = (Y[:, k] - np.conj(Y[:, km])) / 2j
        for p in range(W):
            K = k + Q * p
            A = sum(_omega(W, -1) ** (c * p) * w ** (c * k) * Ac[c] for c in range(W))
            B = sum(_omega(W, -1) ** (c * p) * w ** (c * k) * Bc[c] for c in range(W))
            assert abs(A - A_ref[K]) < 1e-9 * N and abs(B - B_ref[K]) < 1e-9 * N
            assert abs(Z[K] - (A + 1j * B)) < 1e-9 * N
