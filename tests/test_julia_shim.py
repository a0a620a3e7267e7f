"""CPU checks of the Julia drop-in (integration/julia/SWLib.jl).

Julia is not installed here, so the binding is checked by reading it:

* INTEGRATION.md carries SWLib.jl verbatim;
* ``SWStepper{A} <: AbstractTimeStepper{A}`` — FourierFlows' parametric
  supertype, as utils/IFMAB3.jl:13 subtypes it — with the ``filter`` field
  simulation/TwoLayerSimulation.jl:44 reads;
* a ``Problem(dev::GPU; …)`` method per driver model (RSWDriver.jl,
  TYdriver.jl, TwoLayerSimulation.jl, TwoLayerDriver.jl) plus the run-directory
  wrapper that attaches it;
* every ``ccall`` binds an include/sw.h prototype with the same number of
  arguments, and ``SWConfig`` is ``struct sw_config`` field for field;
* each SWLib.jl function that reaches libsw issues the same C entry points,
  in the same order, as its Python twin in tests/driver_replay.py (which the
  GPU replay tests run);
* no type piracy: every FourierFlows function SWLib extends
  has an ``::SWStepper`` argument, and the per-step seam FF's own
  ``stepforward!(prob, diags, n)`` loop calls makes no C call and no host copy.
"""
import inspect
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = os.path.join(ROOT, "integration", "julia")
SWLIB = os.path.join(JL, "SWLib.jl")
HEADER = os.path.join(ROOT, "include", "sw.h")


def _src():
    return open(SWLIB).read()


def _strip_comments(s):
    return re.sub(r"#[^\n]*", "", s)


def _prototypes():
    """sw.h: name -> number of parameters of every extern "C" function."""
    hdr = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"^\s*(int|void|double|const char\*)\s+(sw_\w+)\(([^)]*)\);", hdr, flags=re.M):
        a = args.strip()
        out[name] = 0 if a in ("", "void") else a.count(",") + 1
    return out


def test_integration_md_embeds_the_binding_verbatim():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "```julia\n" + _src() + "```" in doc


def test_stepper_type_is_parametric_with_filter():
    s = _strip_comments(_src())
    m = re.search(r"mutable struct SWStepper\{A<:AbstractArray, Tf\} <: AbstractTimeStepper\{A\}(.*?)\nend", s, re.S)
    assert m, "SWStepper must subtype FourierFlows.AbstractTimeStepper{A} (utils/IFMAB3.jl:13)"
    assert re.search(r"^\s*filter::Tf", m.group(1), re.M)
    # the stepper type parameter is the array type of prob.sol
    assert "A = Array{equation.T, length(equation.dims)}" in s


@pytest.mark.parametrize("module,sig,builder", [
    ("RotatingShallowWater", r"Problem\(dev::FourierFlows\.GPU; kw\.\.\.\) = \$rsw_problem", "rsw_problem"),
    ("TwoLayerQG", r"Problem\(dev::FourierFlows\.GPU; kw\.\.\.\) = \$qg2_problem", "qg2_problem"),
    ("ThomasYamada", r"Problem\(dev::FourierFlows\.GPU; kw\.\.\.\) = \$ty_problem", "ty_problem"),
    ("MultiLayerQG", r"Problem\(nlayers::Int, dev::FourierFlows\.GPU; kw\.\.\.\) = \$mlqg_problem", "mlqg_problem"),
])
def test_problem_method_per_driver(module, sig, builder):
    s = _strip_comments(_src())
    branch = re.search(rf"name === :{module}\n(.*?)(?:\n    elseif|\n    else)", s, re.S)
    assert branch, module
    assert re.search(sig, branch.group(1)), f"{module}: no Problem(GPU) method"
    # the CPU() method falls back to the reference's own (invoke), unless LIBSW_CPU=1
    assert "invoke(Problem, Tuple{" in branch.group(1) and "$use_libsw(dev)" in branch.group(1)
    assert re.search(rf"^function {builder}\(M::Module", s, re.M)


@pytest.mark.parametrize("path,module", [
    ("rsw/RotatingShallowWater.jl", "RotatingShallowWater"),
    ("swqg/TwoLayerQG.jl", "TwoLayerQG"),
    ("thomasyamada/ThomasYamada.jl", "ThomasYamada"),
    ("simulation/Parameters.jl", "GeophysicalFlows.MultiLayerQG"),
])
def test_run_directory_wrappers(path, module):
    s = _strip_comments(open(os.path.join(JL, path)).read())
    ref = os.path.basename(path).replace(".jl", ".ref.jl")
    lines = [x.strip() for x in s.splitlines() if x.strip()]
    assert lines[0] == f'include("{ref}")'
    assert 'include("SWLib.jl")' in lines
    assert f"SWLib.attach!({module})" in lines
    # the two drivers that draw their PV with device_array(GPU()) see SWLib's
    # own host device_array (bound in Main), not a FourierFlows method
    if path.startswith(("swqg/", "simulation/")):
        assert lines[-1] == "const device_array = SWLib.device_array"
    else:
        assert lines[-1] == f"SWLib.attach!({module})"


def test_every_ccall_binds_a_header_prototype():
    protos = _prototypes()
    s = _strip_comments(_src())
    calls = re.findall(r"ccall\(\(:(sw_\w+), libsw\), (\w+(?:\{\w+\})?), \(([^()]*(?:\([^()]*\)[^()]*)*)\)", s)
    assert len(calls) >= 13
    seen = set()
    for name, ret, argtypes in calls:
        assert name in protos, f"{name} is not declared in include/sw.h"
        n = len([a for a in argtypes.split(",") if a.strip()])
        assert n == protos[name], f"{name}: {n} Julia argument types vs {protos[name]} C parameters"
        seen.add(name)
    # the entry points the drivers' call sequences need
    need = {"sw_config_default", "sw_create", "sw_destroy", "sw_last_error", "sw_set_state", "sw_get_state",
            "sw_set_clock", "sw_step", "sw_step_record", "sw_diag", "sw_get_physical", "sw_comm_unique_id"}
    assert need <= seen


def test_swconfig_is_sw_config_field_for_field():
    hdr = open(HEADER).read()
    body = re.search(r"typedef struct sw_config \{(.*?)\} sw_config;", hdr, flags=re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    ctype = {}
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        m = re.match(r"(const void\*|sw_exchange_fn|void\*|int32_t|double)\s+(.*)", decl)
        assert m, decl
        for name in m.group(2).split(","):
            name = name.strip()
            arr = re.match(r"(\w+)\[(\d+)\]", name)
            ctype[arr.group(1) if arr else name] = (m.group(1), int(arr.group(2)) if arr else 1)
    hnames = list(ctype)
    js = re.search(r"Base\.@kwdef mutable struct SWConfig(.*?)\nend", _src(), flags=re.S).group(1)
    jfields = re.findall(r"\b([A-Za-z_]\w*)::([\w{},]+)", js)
    assert [f for f, _ in jfields] == hnames
    jmap = {"int32_t": "Int32", "double": "Float64", "const void*": "Ptr{Cvoid}", "void*": "Ptr{Cvoid}",
            "sw_exchange_fn": "Ptr{Cvoid}"}
    for f, jt in jfields:
        ct, n = ctype[f]
        want = jmap[ct] if n == 1 else f"NTuple{{{n},{jmap[ct]}}}"
        assert jt == want, (f, jt, want)


def _julia_functions(src):
    """name -> body of every top-level `function name(...)` … `end` and
    one-line `name(...) = …` definition in SWLib.jl."""
    out = {}
    lines = _strip_comments(src).splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        m = re.match(r"^function ([\w!.]+)\(", ln)
        if m:
            j = i + 1
            while not lines[j].startswith("end"):
                j += 1
            out.setdefault(m.group(1).split(".")[-1], "\n".join(lines[i:j]))
            i = j + 1
            continue
        m = re.match(r"^([\w!]+)\([^=]*\)(?: where \{[^}]*\})? =", ln)
        if m:
            j = i + 1
            while j < len(lines) and lines[j].startswith(" "):
                j += 1
            out.setdefault(m.group(1), "\n".join(lines[i:j]))
            i = j
            continue
        i += 1
    return out


def _c_sequence(text, pattern):
    return re.findall(pattern, text)


HELPERS_JL = r"\b(upload!|download!|push_clock!|flush!|sync!|blowup!|diag_record)\("
HELPERS_PY = r"self\.(upload|download|push_clock|flush|sync|blowup|diag_record)\("


@pytest.mark.parametrize("jname,pyname", [
    ("config", "config"), ("SWStepper", "SWStepper"), ("upload!", "upload"), ("download!", "download"),
    ("push_clock!", "push_clock"), ("load_solution!", "load_solution"), ("stepforward!", "stepforward_seam"),
    ("flush!", "flush"), ("sync!", "sync"), ("device_energy", "device_energy"), ("diag_record", "diag_record"),
    ("settle!", "settle"),
])
def test_julia_function_matches_its_python_twin(jname, pyname):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import driver_replay

    jf = _julia_functions(_src())
    assert jname in jf, f"SWLib.jl has no function {jname}"
    jseq = _c_sequence(jf[jname], r"ccall\(\(:(sw_\w+)")
    # helper calls inside the Julia body
    body = jf[jname].split("\n", 1)[1] if "\n" in jf[jname] else ""  # without the definition line
    jhelp = _c_sequence(body, HELPERS_JL)
    py = inspect.getsource(getattr(driver_replay.Twin, pyname))
    pseq = _c_sequence(py, r'self\.c\("(sw_\w+)"')
    phelp = _c_sequence(py.split("\n", 1)[1], HELPERS_PY)
    assert jseq == pseq, (jname, jseq, pseq)
    assert [h.rstrip("!") for h in jhelp] == phelp, (jname, jhelp, phelp)


def test_no_fourierflows_method_on_fourierflows_types():
    """Every method SWLib adds to a FourierFlows function dispatches on an
    argument typed ::SWStepper (the reference's own seam, utils/IFMAB3.jl:157,
    dispatches on its stepper type); FF's stepforward!(prob, diags, n),
    stepforward!(prob, n) and device_array(::GPU) are left as FF defines them."""
    s = _strip_comments(_src())
    defs = re.findall(r"^(?:function\s+)?FourierFlows\.([\w!]+)\(([^)]*)\)(?:\s*=|\s*$)", s, re.M)
    assert defs, "the per-step seam"
    for name, args in defs:
        assert "::SWStepper" in args, f"FourierFlows.{name}({args}) is defined for FourierFlows' own types"
    assert [n for n, _ in defs] == ["stepforward!"]
    assert not re.search(r"FourierFlows\.device_array\([^)]*\)\s*=", s)
    assert not re.search(r"FourierFlows\.(increment!|Diagnostic)\(", s)


def test_per_step_seam_is_lazy():
    """FF's stepforward!(prob, diags, n) calls the seam once per step: it only
    counts the step (no ccall, no download!/sync!/flush!), in Julia and in the
    twin; the counted steps run at the next energy Diagnostic (sw_step_record)
    or updatevars!/set_solution! (sw_step, one sw_get_state)."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import driver_replay

    s = _strip_comments(_src())
    body = re.search(r"^function FourierFlows\.stepforward!\(sol, clock, ts::SWStepper, (.*?)\nend", s,
                     re.S | re.M).group(1)
    assert "ccall" not in body and not re.search(r"\b(download!|sync!|flush!|upload!)\(", body)
    assert "ts.pending += 1" in body and "clock.step += 1" in body
    py = inspect.getsource(driver_replay.Twin.stepforward_seam)
    assert "self.c(" not in py and "ts.pending += 1" in py
    # every libsw updatevars! shim syncs first (and dealiases the host sol as
    # the reference's :104 / :115 and GF's updatevars! do — ADVICE r03)
    for f in ("rsw_updatevars!", "qg2_updatevars!", "ty_updatevars!", "mlqg_updatevars!"):
        fb = re.search(rf"^function {re.escape(f)}\((.*?)\nend", s, re.S | re.M).group(1)
        assert "sync!(prob)" in fb, f
    for f in ("rsw_updatevars!", "qg2_updatevars!", "ty_updatevars!", "mlqg_updatevars!"):
        fb = re.search(rf"^function {re.escape(f)}\((.*?)\nend", s, re.S | re.M).group(1)
        assert fb.index("sync!(prob)") < fb.index("FourierFlows.dealias!(sol, grid)") < fb.index("@. vars.")
    # after updatevars! the energy functions read the updated state (sw_diag),
    # not the last step's record
    for f in ("rsw_updatevars!", "qg2_updatevars!", "ty_updatevars!", "mlqg_updatevars!"):
        fb = re.search(rf"^function {re.escape(f)}\((.*?)\nend", s, re.S | re.M).group(1)
        assert "ts.rec_step = -1" in fb, f


def test_physical_vars_run_the_counted_steps_when_read():
    """the drivers scan vars.η / vars.q for NaN right after
    stepforward!(prob, diags, n) (rsw/RSWDriver.jl:213, swqg/TwoLayerDriver.jl:106).
    The physical fields of a libsw problem's vars are SWFields whose reads run
    the pending steps first (settle! -> flush!), for RSW, 2LQG and TY; the
    twin's DeviceVars does the same on attribute access."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import driver_replay

    s = _strip_comments(_src())
    assert re.search(r"^struct SWField\{T,N\} <: AbstractArray\{T,N\}", s, re.M)
    settle = re.search(r"^function settle!\(a::SWField\)(.*?)\nend", s, re.S | re.M).group(1)
    assert "pending == 0 || flush!(prob)" in settle
    # every read path settles: indexing, broadcasting (isnan.(vars.η)), deepcopy
    assert re.search(r"Base\.getindex\(a::SWField, i::Int\) = \(settle!\(a\);", s)
    assert re.search(r"Base\.Broadcast\.broadcastable\(a::SWField\) = parent\(settle!\(a\)\)", s)
    assert re.search(r"Base\.deepcopy_internal\(a::SWField, d::IdDict\) = .*settle!\(a\)", s)
    # writes do not
    assert re.search(r"Base\.setindex!\(a::SWField, x, i::Int\) = \(a\.data\[i\] = x; a\)", s)
    for builder in ("rsw_problem", "qg2_problem", "ty_problem"):
        body = re.search(rf"^function {builder}\((.*?)\nend", s, re.S | re.M).group(1)
        assert "vars = device_vars(M.Vars(grid), owner)" in body, builder
        assert "owned_problem(owner, sol, clock, equation, grid, vars, params, ts)" in body, builder
    # blowup! fills the SWFields in place (fill! writes the host array)
    assert re.search(r"Base\.fill!\(a::SWField, x\) = \(fill!\(a\.data, x\); a\)", s)
    py = inspect.getsource(driver_replay.DeviceVars)
    assert "owner.tw.settle(owner.prob)" in py


@pytest.mark.parametrize("module,names", [
    ("RotatingShallowWater", ["kinetic_energy", "potential_energy"]),
    ("TwoLayerQG", ["kinetic_energy", "potential_energy"]),
    ("ThomasYamada", ["barotropic_energy", "baroclinic_energy", "wave_geostrophic_energy"]),
    ("MultiLayerQG", ["energies"]),
])
def test_energy_functions_have_libsw_methods(module, names):
    s = _strip_comments(_src())
    branch = re.search(rf"name === :{module}\n(.*?)(?:\n    elseif|\n    else)", s, re.S).group(1)
    m = re.search(r"energy_methods!\(M, (.*?)\)(?:\n|$)", branch + "\n", re.S)
    assert m, module
    assert re.findall(r":(\w+) =>", m.group(1)) == names
