# Run-directory ThomasYamada.jl under libsw: the reference module
# (thomasyamada/ThomasYamada.jl, copied as ThomasYamada.ref.jl), then its libsw
# methods.  TYdriver.jl includes this file inside its module Driver and runs
# unchanged; `TYdriver.jl GPU` builds the start-up problem on libsw, and
# LIBSW_CPU=1 puts its second Problem(CPU()) (:181) there too.
include("ThomasYamada.ref.jl")
include("SWLib.jl")
SWLib.attach!(ThomasYamada)
