# Run-directory TwoLayerQG.jl under libsw: the reference module
# (swqg/TwoLayerQG.jl, copied as TwoLayerQG.ref.jl), then its libsw methods.
# TwoLayerMain.jl and TwoLayerDriver.jl run unchanged.
include("TwoLayerQG.ref.jl")
include("SWLib.jl")
SWLib.attach!(TwoLayerQG)
# The driver's device_array(GPU()) (swqg/TwoLayerDriver.jl:11) -> host Array
# (SWLib.device_array; bound before TwoLayerDriver.jl's `using FourierFlows`)
const device_array = SWLib.device_array
