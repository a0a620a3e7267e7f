# Run-directory RotatingShallowWater.jl under libsw: the reference module
# (rsw/RotatingShallowWater.jl, copied as RotatingShallowWater.ref.jl), then its
# libsw methods.  RSWMain.jl and RSWDriver.jl run unchanged.
include("RotatingShallowWater.ref.jl")
include("SWLib.jl")
SWLib.attach!(RotatingShallowWater)
