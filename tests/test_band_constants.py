"""The compile-time live bands of the kernels (round 6): the
rows specialise on kc = N/3 (the 2/3 rule) or N/2 (aliased_fraction = 0), the
column kernels on lc = N/3, lr2 = N − N/3 (or N/2, N/2 + 1), and the launch
predicates (`row_kc`, `rowh_kc`, `band_of` in csrc/sw_kernels.hip) compare the
run-time geometry with exactly these integers.  libsw's geometry follows
FourierFlows' dealias ranges (csrc/sw_api.cpp alias_range / make_geom, the
oracle's grid): this pins that, for every power-of-two line the kernels are
built for, the 2/3 rule's fp64 ranges give those integers, so the specialised
kernels are the ones the BASELINE configurations launch."""
import math

import pytest


def alias_range(n, af):
    """csrc/sw_api.cpp alias_range: iL = ⌊(1−af)/2·n⌋ + 1, iR = ⌈(1+af)/2·n⌉"""
    L, R = (1 - af) / 2, (1 + af) / 2
    return math.floor(L * n) + 1, math.ceil(R * n)


@pytest.mark.parametrize("log2n", range(5, 14))
def test_two_thirds_rule_band_is_n_over_3(log2n):
    n = 1 << log2n
    iL, iR = alias_range(n, 1 / 3)
    kc, lc, lr2 = iL - 1, iL - 1, iR  # make_geom: kc = iLx - 1, lc = iLy - 1, lr2 = iRy
    assert kc == n // 3 and lc == n // 3
    assert lr2 == n - n // 3


@pytest.mark.parametrize("log2n", range(5, 14))
def test_aliased_fraction_zero_band(log2n):
    """aliased_fraction = 0 (MultiLayerQG in TwoLayerSimulation): kc = nx/2
    (the Nyquist column dropped), lc = ny/2, lr2 = ny/2 + 1 (make_geom's
    special case)"""
    n = 1 << log2n
    iL, _ = alias_range(n, 0.0)
    assert iL - 1 == n // 2
