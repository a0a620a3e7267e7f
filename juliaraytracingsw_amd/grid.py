"""Host-side grid description (FF ``TwoDGrid``) used by the drivers
to build initial conditions.  Pure setup code: no hot-path work happens here.
"""
from __future__ import annotations

import math

import numpy as np


class TwoDGrid:
    """Mirror of FF ``TwoDGrid(dev; nx, Lx, ny, Ly, aliased_fraction, T)``
    (rsw/RotatingShallowWater.jl:87).  Arrays use numpy ``[l][kr]`` order."""

    def __init__(self, nx, Lx=2 * np.pi, ny=None, Ly=None, aliased_fraction=1 / 3):
        ny = nx if ny is None else ny
        Ly = Lx if Ly is None else Ly
        self.nx, self.ny, self.Lx, self.Ly = int(nx), int(ny), float(Lx), float(Ly)
        self.aliased_fraction = float(aliased_fraction)
        self.dx, self.dy = self.Lx / self.nx, self.Ly / self.ny
        self.x = -self.Lx / 2 + self.dx * np.arange(self.nx)
        self.y = -self.Ly / 2 + self.dy * np.arange(self.ny)
        self.nkr, self.nl = self.nx // 2 + 1, self.ny
        self.kr = np.arange(self.nkr) * ((2 * np.pi / self.Lx * self.nx) / self.nx)
        lidx = np.concatenate([np.arange(0, self.ny // 2), np.arange(-self.ny // 2, 0)])
        self.l = lidx * ((2 * np.pi / self.Ly * self.ny) / self.ny)
        self.Krsq = self.kr[None, :] ** 2 + self.l[:, None] ** 2
        with np.errstate(divide="ignore"):
            self.invKrsq = np.where(self.Krsq == 0, 0.0, 1.0 / self.Krsq)
        af = self.aliased_fraction
        iLx = math.floor((1 - af) / 2 * self.nx) + 1
        iLy = math.floor((1 - af) / 2 * self.ny) + 1
        iRy = math.ceil((1 + af) / 2 * self.ny)
        self.kralias = (iLx - 1, self.nkr)
        self.lalias = (iLy - 1, iRy)
        m = np.ones((self.nl, self.nkr), bool)
        m[:, self.kralias[0]:] = False
        m[self.lalias[0]:self.lalias[1], :] = False
        self.live = m
