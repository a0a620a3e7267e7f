"""CPU model of the generic engine's line transform (csrc/sw_generic.hip
fft_lds): the radix sequence of `radices` and the mixed-radix Stockham DIF
index algebra — y[q + s(rp + u)] = ω_len^(pu) Σ_t x[q + s(p + tm)] ω_r^(tu),
the r-point DFTs as dft_small writes them and ω_len^(pu) from the n-point
table (k_twiddles) —
checked against numpy's FFT in both directions on the grids the engine
accepts (2^a·3^b·5^c, even, 16 … 4096), and the c2r row rule (the DC and
Nyquist bins' imaginary parts dropped, numpy's irfft convention)."""
import numpy as np
import pytest


def radices(n):
    """sw_generic.hip radices(): 4s, then a 2, 3s, 5s; None if n does not factor"""
    if n < 16 or n > 4096 or n % 2:
        return None
    out = []
    for r in (4, 2, 3, 5):
        while n % r == 0:
            out.append(r)
            n //= r
    return out if n == 1 else None


def dft_small(v, d):
    """sw_generic.hip dft_small: the r-point DFTs as written there (exact ±1/±i
    for r = 2, 4; the radix-3/5 constants); v: [r, ...] complex, d = DIR"""
    r = len(v)
    rot = lambda a: 1j * d * a  # noqa: E731
    if r == 4:
        a, b, c, e = v[0] + v[2], v[0] - v[2], v[1] + v[3], rot(v[1] - v[3])
        return np.stack([a + c, b + e, a - c, b - e])
    if r == 2:
        return np.stack([v[0] + v[1], v[0] - v[1]])
    if r == 3:
        s3 = 0.86602540378443864676
        sm, df = v[1] + v[2], v[1] - v[2]
        t, e = v[0] - 0.5 * sm, rot(s3 * df)
        return np.stack([v[0] + sm, t + e, t - e])
    c1, c2, s1, s2 = 0.30901699437494742410, -0.80901699437494742410, 0.95105651629515357212, 0.58778525229247312917
    p1, d1, p2, d2 = v[1] + v[4], v[1] - v[4], v[2] + v[3], v[2] - v[3]
    a1, a2 = v[0] + c1 * p1 + c2 * p2, v[0] + c2 * p1 + c1 * p2
    b1, b2 = rot(s1 * d1 + s2 * d2), rot(s2 * d1 - s1 * d2)
    return np.stack([v[0] + p1 + p2, a1 + b1, a2 + b2, a2 - b2, a1 - b1])


def fft_lds(x, d):
    n = len(x)
    tw = np.exp(-2j * np.pi * np.arange(n) / n)  # k_twiddles: the forward table, conj for d = +1
    if d > 0:
        tw = tw.conj()
    X, Y = x.astype(complex).copy(), np.zeros(n, complex)
    L, s = n, 1
    for r in radices(n):
        m = L // r
        i = np.arange(m * s)
        p, q = i // s, i % s
        v = dft_small(np.stack([X[q + s * (p + t * m)] for t in range(r)]), d)
        for u in range(r):
            Y[q + s * (r * p + u)] = v[u] * tw[p * u * (n // L)]
        X, Y = Y, X
        L, s = m, s * r
    return X


@pytest.mark.parametrize("n", [16, 30, 96, 120, 384, 750, 3072, 4096])
def test_stockham_model_matches_numpy(n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    assert np.max(np.abs(fft_lds(x, -1) - np.fft.fft(x))) < 1e-12 * np.max(np.abs(np.fft.fft(x)))
    assert np.max(np.abs(fft_lds(x, +1) - n * np.fft.ifft(x))) < 1e-12 * n * np.max(np.abs(np.fft.ifft(x)))


def test_radices_accept_and_refuse():
    assert radices(384) == [4, 4, 4, 2, 3]
    assert radices(120) == [4, 2, 3, 5]
    for n in (98, 14, 6144, 8, 385):
        assert radices(n) is None


def test_c2r_row_rule_is_numpys():
    """k_c2r_rows: z[k] = X[k] (k ≤ n/2, imaginary parts of k = 0, n/2
    dropped), z[n-k] = conj X[k]; inverse transform; real part / n"""
    n = 96
    rng = np.random.default_rng(1)
    X = rng.standard_normal(n // 2 + 1) + 1j * rng.standard_normal(n // 2 + 1)
    z = np.empty(n, complex)
    z[: n // 2 + 1] = X
    z[0], z[n // 2] = X[0].real, X[n // 2].real
    z[n // 2 + 1:] = np.conj(X[1: n // 2][::-1])
    got = fft_lds(z, +1).real / n
    assert np.max(np.abs(got - np.fft.irfft(X, n))) < 1e-14
