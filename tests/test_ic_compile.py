"""f1 for any icond formula: the program compiled for the device (pft_ic_compile, csrc/pft_ic_ops.h),
checked on the CPU.

pft_ic_compile folds every subexpression of constants and one coordinate into host-evaluated
tables (the C library's own values) and leaves a residual program of operators the device
evaluates as the host does.  pft_ic_eval_compiled runs that residual program with the device's
operator code compiled for the host; it must give pft_ic_eval's bits (the host path, pinned to the
reference's IC by tests/test_frontend.py) at every node -- for every formula the reference's
published cases use (tests/golden/icond_published.json, from its results/ archives), the default
Params, multi-pass formulas over u/p/gl, math errors at some nodes (0 there, as the reference's
Eval()), and on several Z-slabs.  The GPU test (tests/test_device_ic.py) runs the same programs
through ic_prog_kernel."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import porousfreezethaw_amd as P
from porousfreezethaw_amd import frontend as FE

# formulas written for this test: every operator class, multi-pass reads, per-node math errors
SYNTHETIC = [
    {"u": "293.15 + 5*tanh((x-L1/2)/L1) * (y > L2/3)", "p": "sqrt(x*y) < 0.01 or z > L3/2",
     "gl": "(0.5*(1.0 + tanh(0.5/xi_gl*(z-0.055)))) max p"},
    {"u": "top_temp1", "p": "(x-L1/2)^2 + (y-L2/2)^2 < (L1/3)^2 and z > 0.052",
     "gl": "floor(p*3.7) + round(_x*10)/10 - abs(_y - 0.5) + sgn(_z - 0.5)"},
    {"p": "1/(x - L1/2) min 50", "gl": "ln(_x) * 0 + _y", "u": "p*2 + gl + exp(_z)"},          # 1/0 nowhere
    # math errors at some nodes (0 there): 1/0 where 0.25 <= _x < 0.5, sqrt of a negative below _y = 0.45,
    # a table entry's error inside a residual program (u)
    {"p": "1/(floor(_x*4) - 1)", "gl": "sqrt(_y - 0.45)", "u": "gl + p + sqrt(_z - 0.3)*x"},
    {"u": "x*y*z*1e9 + not (p) + 3! + (5 C 2) - toDeg(toRad(y))", "p": "(_x+_y+_z)/3 > 0.5",
     "gl": "(1 - p) * 0.25"},
]


def _lib():
    L = P.lib()
    L.pft_ic_eval_compiled.argtypes = [C.POINTER(P.pft_grid), C.c_int, C.c_int, C.POINTER(C.c_int),
                                      C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.pft_ic_device_ok.argtypes = [C.POINTER(P.pft_grid), C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.pft_ic_eval.argtypes = L.pft_ic_eval_compiled.argtypes
    return L


def _minimal(extra=""):
    lines = ["L1 0.03", "L2 0.03", "L3 0.06", "saved_files 1", "tau 1", "final_time 1", "delta 1e-3",
             "xi_gl 0.0004", "beads_offset_x 0.002", "beads_offset_y 0.002", "beads_offset_z 0.004",
             "top_temp1 268.15"]
    lines += [f"{n} 1" for n in P.PARAM_NAMES if n not in ("xi_gl",)]
    return "\n".join(lines) + "\n" + extra


def _programs(formulas):
    text = "".join(f'icond {k} = "{v}"\n' for k, v in formulas.items())
    case = FE.load_params(text=_minimal(text))
    return case.icond_programs()


def _published():
    """the distinct formula sets of the reference's published cases and its default Params
    (tests/golden/icond_published.json, made from the reference's files by gen_icond.py)"""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "icond_published.json")
    d = json.load(open(path))
    return [c["icond"] for c in d["published"]] + [d["default"]]


def _both(progs, n1, n2, total_n3, nprocs, rank):
    L = _lib()
    g = P.pft_grid()
    assert L.pft_grid_init(C.byref(g), n1, n2, total_n3, nprocs, rank, 0.03, 0.03, 0.06, 0) == 0
    S = (n1 + 4) * (n2 + 4) * (g.n3 + 4)
    host, dev = np.zeros(3 * S), np.zeros(3 * S)
    for q, prog in progs:
        ops = np.array([o for o, _ in prog], dtype=np.int32)
        args = np.array([a for _, a in prog], dtype=np.float64)
        ip, dp = ops.ctypes.data_as(C.POINTER(C.c_int)), args.ctypes.data_as(C.POINTER(C.c_double))
        assert L.pft_ic_device_ok(C.byref(g), len(prog), ip, dp) == 1
        assert L.pft_ic_eval(C.byref(g), q, len(prog), ip, dp, host.ctypes.data_as(C.POINTER(C.c_double))) == 0
        assert L.pft_ic_eval_compiled(C.byref(g), q, len(prog), ip, dp,
                                      dev.ctypes.data_as(C.POINTER(C.c_double))) == 0
    return host, dev


def _same(a, b):
    assert np.array_equal(a, b, equal_nan=True) and np.array_equal(np.signbit(a), np.signbit(b))


@pytest.mark.parametrize("which", range(len(SYNTHETIC)))
@pytest.mark.parametrize("dims,nprocs", [((14, 9, 22), 1), ((14, 9, 22), 3), ((7, 12, 5), 1)])
def test_compiled_equals_host_synthetic(which, dims, nprocs):
    progs = _programs(SYNTHETIC[which])
    for r in range(nprocs):
        _same(*_both(progs, *dims, nprocs, r))


def test_compiled_equals_host_published():
    cases = _published()
    assert len(cases) >= 5
    for f in cases:
        progs = _programs(f)
        for nprocs, r in ((1, 0), (4, 2)):
            _same(*_both(progs, 20, 16, 36, nprocs, r))


def test_stays_on_host_where_not_device_exact():
    """pow or another libm call over several coordinates (or the node's fields) is not folded:
    the program stays on the host"""
    L = _lib()
    g = P.pft_grid()
    assert L.pft_grid_init(C.byref(g), 6, 5, 4, 1, 0, 0.03, 0.03, 0.06, 0) == 0
    for formula, ok in (("(x*y)^2", 0), ("exp(x + y)", 0), ("exp(x) + exp(y)", 1), ("x^2 + y^2", 1),
                        ("tanh(x*y)", 1), ("sin(u)", 0)):
        ev = FE.Evaluator()
        for n in ("L1", "L2", "L3"):
            ev.define(n, 0.03)
        for v in ("x", "y", "z", "_x", "_y", "_z", "u", "p", "gl"):
            ev.define(v, 0.5)
        prog = ev.compile(formula, ("x", "y", "z", "_x", "_y", "_z", "u", "p", "gl"))
        ops = np.array([o for o, _ in prog], dtype=np.int32)
        args = np.array([a for _, a in prog], dtype=np.float64)
        got = L.pft_ic_device_ok(C.byref(g), len(prog), ops.ctypes.data_as(C.POINTER(C.c_int)),
                                 args.ctypes.data_as(C.POINTER(C.c_double)))
        assert got == ok, formula
