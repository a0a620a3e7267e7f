# Run-directory TwoLayerQG.jl under libsw: the reference module
# (swqg/TwoLayerQG.jl, copied as TwoLayerQG.ref.jl), then its libsw methods.
# TwoLayerMain.jl and TwoLayerDriver.jl run unchanged.
include("TwoLayerQG.ref.jl")
include("SWLib.jl")
SWLib.attach!(TwoLayerQG)
