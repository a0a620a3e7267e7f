# Run-directory Parameters.jl of simulation/ under libsw: the reference
# parameters module (simulation/Parameters.jl, copied as Parameters.ref.jl:
# device = GPU(), stepper = "FilteredRK4"), then libsw's methods on
# GeophysicalFlows' MultiLayerQG, the package TwoLayerSimulation.jl loads.
# Driver.jl and TwoLayerSimulation.jl run unchanged.
include("Parameters.ref.jl")
include("SWLib.jl")
import GeophysicalFlows
SWLib.attach!(GeophysicalFlows.MultiLayerQG)
# The driver's device_array(GPU()) (simulation/TwoLayerSimulation.jl:43) ->
# host Array (SWLib.device_array; bound before its `using GeophysicalFlows`)
const device_array = SWLib.device_array
