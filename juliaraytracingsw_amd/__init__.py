"""juliaraytracingsw_amd — MI355X-native pseudo-spectral time-step core.

The hot path (calcN + stepper update of the FourierFlows models used by
ndefilippis/JuliaRaytracingSW) runs in ``libsw.so``: hand-written HIP kernels
for gfx950 behind the C ABI of ``include/sw.h``.  This package is the host-side
mirror of the reference's module interfaces:

* ``rotating_shallow_water`` — rsw/RotatingShallowWater.jl
* ``two_layer_qg``           — swqg/TwoLayerQG.jl
* ``thomas_yamada``          — thomasyamada/ThomasYamada.jl (ETDRK4)
* ``multilayer_qg``          — GeophysicalFlows MultiLayerQG (FilteredRK4), simulation/TwoLayerSimulation.jl
* ``output``                 — snapshot output / restart (FF Output, utils/SequencedOutputs.jl)
* ``drivers``                — rsw/RSWDriver.jl, swqg/TwoLayerDriver.jl setup
"""
from ._lib import LibSWError, load, LIB_PATH  # noqa: F401

__all__ = ["LibSWError", "load", "LIB_PATH"]
