"""Params front end (porousfreezethaw_amd/frontend.py, pft_ic_eval), CPU only.

Pinned three ways:
- the default Params (grid_nodes 20) evaluates to the bits of the reference's own parameter dump
  (tests/golden/g20.json, from the reference compiled in place);
- its icond formulas, compiled and evaluated at every node by pft_ic_eval, give the reference's
  initial condition bit for bit (golden g20 "ic", glass beads applied afterwards as the reference
  does);
- every published case under the reference's results/ archives evaluates to the values its own
  intertrack.log printed (%g) -- read from /root/reference when it exists (this container), skipped
  elsewhere; nothing is copied from there.
"""
import glob
import math
import os
import re
import tarfile

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P
from porousfreezethaw_amd import frontend as FE

REF_APP = "/root/reference/apps/intertrack-hybrid-S-freezing"


def test_evaluator_precedence_and_functions():
    ev = FE.Evaluator()
    cases = {
        "1+2*3": 7.0, "2^3^2": 64.0,              # equal precedence reduces left to right
        "-2^2": -4.0, "2*-3": -6.0, "10 max 3 max 7": 10.0, "3! + 1": 7.0, "5 C 2": 10.0,
        "(1<2) and (3>2)": 1.0, "not 0": 1.0, "2 = 2": 1.0, "sqrt 16": 4.0,
        "tanh(0.5)": math.tanh(0.5), "ln(e)": math.log(math.e), "abs -3": 3.0, "round 2.5": 3.0,
        "(1+2": 3.0,                              # unbalanced '(' closed at the end (exp_all.cc:856)
        "1e-3": O.lib().pft_or_float_val(b"1e-3"), "2.5e+2": 250.0,
    }
    for expr, want in cases.items():
        got = ev.eval(expr)
        assert got == want and math.copysign(1, got) == math.copysign(1, want), (expr, got, want)
    ev.define("a_1", 2.0)
    assert ev.eval("a_1*a_1") == 4.0
    for bad in ("1+", "(", "1 2", "undefined_name", "1/0", "sqrt -1", ")"):
        with pytest.raises(FE.EvalError):
            ev.eval(bad)


def _default_params_text():
    path = os.path.join(REF_APP, "Params")
    if not os.path.exists(path):
        pytest.skip("reference Params not available here")
    with open(path) as f:
        return f.read()


def test_default_params_bitwise_vs_reference_dump():
    meta, _ = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    case = FE.load_params(text=_default_params_text(), env={"OUTPUT": "out"}, overrides={"grid_nodes": 20})
    assert np.array_equal(case.params, Pm)
    assert case.n == (info["n1"], info["n2"], info["n3"])
    assert case.L == (info["L1"], info["L2"], info["L3"])
    assert (case.tau_min, case.delta) == (info["tau_min"], info["delta"])
    assert case.settings["out_file"] == "out/image" and case.settings["out_file_suffix"] == ".ncd"
    assert case.settings["comment"] == "Testing run"


def test_icond_formulas_bitwise_vs_reference_ic():
    meta, A = O.load_case("g20")
    case = FE.load_params(text=_default_params_text(), env={"OUTPUT": "out"}, overrides={"grid_nodes": 20})
    progs = case.icond_programs()
    assert [q for q, _ in progs] == [0, 1, 2]
    for nprocs in (1, 3):
        parts = []
        for r in range(nprocs):
            sim = case.simulation(nprocs=nprocs, rank=r, beads=O.beads(), init_solver=False)
            parts.append(sim.interior())
            sim.close()
        assert np.array_equal(np.concatenate(parts, axis=1), A["ic"])


def test_multipass_icond():
    """a formula may use another quantity's initial value (intertrack.c:1831-1847 multi-pass)"""
    text = "icond u = \"p*2 + gl\"\nicond p = \"x + y\"\nicond gl = \"p max z\"\n"
    case = FE.Case.__new__(FE.Case)
    case.ev, case.icond = FE.Evaluator(), FE.load_params(text=text + _minimal()).icond
    progs = case.icond_programs()
    assert [q for q, _ in progs] == [1, 2, 0]          # p first, then gl (uses p), then u
    meta, _ = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    sim = P.Simulation(4, 3, 5, (info["L1"], info["L2"], info["L3"]), 0, Pm, icond=progs, init_solver=False)
    u, p, gl = sim.interior()
    x = info["L1"] * ((0.5 + np.arange(4)) / 4)
    y = info["L2"] * ((0.5 + np.arange(3)) / 3)
    z = info["L3"] * ((0.5 + np.arange(5)) / 5)
    pe = x[None, None, :] + y[None, :, None] + 0 * z[:, None, None]
    assert np.array_equal(p, pe)
    assert np.array_equal(gl, np.where(pe > z[:, None, None], pe, z[:, None, None] + 0 * pe))
    assert np.array_equal(u, pe * 2 + gl)
    sim.close()


def _minimal():
    names = ["L1 0.03", "L2 0.03", "L3 0.06", "saved_files 1", "tau 1", "final_time 1", "delta 1e-3"]
    names += [f"{n} 1" for n in P.PARAM_NAMES]
    return "\n".join(names) + "\n"


def _log_values(log):
    vals = {}
    for line in log.splitlines():
        m = re.match(r".{70} : (\S+)\s+= (\S+)$", line)
        if m:
            vals[m.group(1)] = m.group(2)
        for key, pat in (("L1", r"Domain base width: (\S+)"), ("L2", r"Domain base height: (\S+)"),
                         ("L3", r"Domain depth: (\S+)"), ("calc_mode", r"Calculation mode: (\S+)"),
                         ("n1", r"Grid X inner nodes: (\S+)"), ("n2", r"Grid Y inner nodes: (\S+)"),
                         ("n3", r"Grid Z inner nodes: (\S+)"), ("tau", r"Initial time step: (\S+)"),
                         ("final_time", r"Final time : (\S+)"),
                         ("delta", r"Runge-Kutta-Merson solver tolerance \(delta\) : (\S+)"),
                         ("tau_min", r"Time step lower bound .* : (\S+)")):
            m = re.match(pat, line)
            if m and key not in vals:
                vals[key] = m.group(1)
    return vals


def test_published_cases_match_their_logs():
    archives = sorted(glob.glob(os.path.join(REF_APP, "results", "*", "*.tgz")))
    if not archives:
        pytest.skip("reference result archives not available here")
    checked = 0
    for arc in archives:
        with tarfile.open(arc) as tf:
            members = {m.name: m for m in tf.getmembers() if m.isfile()}
            for name in members:
                if not name.endswith("/Params"):
                    continue
                logname = os.path.join(os.path.dirname(name), "OUTPUT", "intertrack.log")
                if logname not in members:
                    continue
                text = tf.extractfile(members[name]).read().decode("latin-1")
                log = tf.extractfile(members[logname]).read().decode("latin-1")
                want = _log_values(log)
                case = FE.load_params(text=text, env={"OUTPUT": "OUTPUT"})
                got = {k: case.ev.value(k) for k in want if k not in ("n1", "n2", "n3", "calc_mode", "tau_min")}
                got.update(n1=case.n[0], n2=case.n[1], n3=case.n[2], calc_mode=case.calc_mode, tau_min=case.tau_min)
                for k, v in want.items():
                    g = got[k]
                    assert ("%d" % g if isinstance(g, int) else "%g" % g) == v, (name, k, g, v)
                checked += 1
    assert checked >= 5
