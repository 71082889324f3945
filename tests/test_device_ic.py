"""f1: the default Params' initial condition and the glass beads computed on the device
(pft_solver_ic_default_device: intertrack.c:1880-2010 with Params:9-21, and PrecalculateData,
equation.c:459-530), against the reference's own IC digests at every BASELINE single-GPU size
(tests/golden/g100, g200, g400: SHA-256 of the harness' IC) and against libpft's host IC, bit for
bit; on several slabs; and the reference's g100 trajectory started from it on the device."""
import hashlib

import numpy as np
import pytest

import _multi as M
import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def _sim(grid_nodes, device_ic, nprocs=1, rank=0, beads=True, mode=0):
    base, Pm, info = M.full_size_case(grid_nodes, mode)
    return P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode, Pm,
                        nprocs=nprocs, rank=rank, beads=O.beads() if beads else None, tau=1.0,
                        tau_min=info["tau_min"], delta=info["delta"], device_ic=device_ic)


@pytest.mark.parametrize("case,grid_nodes,key", [("g100", 100, "ic_sha256"), ("g200", 200, "m0_ic_sha256"),
                                                 ("g400", 400, "m0_ic_sha256")])
def test_device_ic_equals_reference(case, grid_nodes, key):
    """BASELINE configs[0..2]: the device IC's digest is the reference's"""
    meta, _ = O.load_case(case)
    sim = _sim(grid_nodes, True)
    x = sim.interior()
    sim.close()
    assert _sha(x) == meta[key]


@pytest.mark.parametrize("grid_nodes", [20, 30, 100])
@pytest.mark.parametrize("beads", [True, False])
def test_device_ic_equals_host_ic(grid_nodes, beads):
    host = _sim(grid_nodes, False, beads=beads)
    a = host.interior()
    host.close()
    dev = _sim(grid_nodes, True, beads=beads)
    b = dev.interior()
    dev.close()
    assert np.array_equal(a, b) and np.array_equal(np.signbit(a), np.signbit(b))


@pytest.mark.parametrize("nprocs", [3, 4])
def test_device_ic_multislab(nprocs):
    """each slab computes its own planes (first_row), on loopback slabs: the global field is the
    single-slab host IC"""
    host = _sim(40, False)
    ref = host.interior()
    host.close()
    out = M.loopback_run(nprocs, lambda r: _sim(40, True, nprocs, r), lambda sim: sim.interior())
    assert np.array_equal(np.concatenate(out, axis=1), ref)


def test_device_ic_g100_trajectory():
    """BASELINE configs[0] from the device IC without any host upload (PFT_SOLVE_REUSE_DEVICE):
    the reference's trajectory to t = 3 s (152 attempted steps)"""
    meta, A = O.load_case("g100")
    sim = _sim(100, True)
    rc = sim.solve_ex(meta["traj_times"][0], 0, P.PFT_SOLVE_REUSE_DEVICE)
    ref = meta["traj_m0"][0]
    assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
        (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
    x = sim.interior()
    sim.close()
    assert np.array_equal(x[:, -1], A["traj_m0_state0_top"])
    assert _sha(x) == meta["traj_m0_sha256"][0]


# ---- f1 for any icond formula (pft_solver_ic_formulas_device) --------------------------------

def _formula_sets():
    import test_ic_compile as T
    return [("published", f) for f in T._published()] + [("synthetic", f) for f in T.SYNTHETIC]


def _formula_sim(formulas, dims, device_ic, nprocs=1, rank=0, beads=True):
    import test_ic_compile as T
    from porousfreezethaw_amd import frontend as FE
    text = "".join(f'icond {k} = "{v}"\n' for k, v in formulas.items())
    case = FE.load_params(text=T._minimal(text))
    n1, n2, n3 = dims
    return P.Simulation(n1, n2, n3, case.L, 0, case.params, nprocs=nprocs, rank=rank,
                        beads=O.beads() if beads else None, icond=case.icond_programs(), tau=1.0,
                        device_ic=device_ic)


@pytest.mark.parametrize("which", range(10))
@pytest.mark.parametrize("beads", [True, False])
def test_device_formulas_equal_host(which, beads):
    """every published formula set (and the synthetic ones of tests/test_ic_compile.py: every
    operator class, multi-pass reads, math errors at some nodes) on the device, beads overlaid
    there too: the host's IC (pft_ic_eval + PrecalculateData) bit for bit"""
    sets = _formula_sets()
    if which >= len(sets):
        pytest.skip("fewer formula sets")
    _, f = sets[which]
    host = _formula_sim(f, (26, 18, 30), False, beads=beads)
    a = host.interior()
    assert host.ic_where == "host"
    host.close()
    dev = _formula_sim(f, (26, 18, 30), True, beads=beads)
    assert dev.ic_where == "device"
    b = dev.interior()
    dev.close()
    assert np.array_equal(a, b, equal_nan=True) and np.array_equal(np.signbit(a), np.signbit(b))


@pytest.mark.parametrize("nprocs", [3])
def test_device_formulas_multislab(nprocs):
    """each slab evaluates its own planes (z tables with its first_row): the global field is the
    single-slab host IC"""
    f = _formula_sets()[0][1]
    host = _formula_sim(f, (24, 20, 33), False)
    ref = host.interior()
    host.close()
    out = M.loopback_run(nprocs, lambda r: _formula_sim(f, (24, 20, 33), True, nprocs, r), lambda sim: sim.interior())
    assert np.array_equal(np.concatenate(out, axis=1), ref)


def test_device_formulas_default_params_g100():
    """the default Params' formulas (Params:9-21) compiled for the device at g100 (BASELINE
    configs[0]), beads overlaid on the device: the reference's own IC digest -- the general path
    reproduces what the fixed-function kernel and the reference give"""
    import test_ic_compile as T
    from porousfreezethaw_amd import frontend as FE
    meta, _ = O.load_case("g100")
    base, Pm, info = M.full_size_case(100, 0)
    ev = FE.Evaluator()
    for k, v in base.items():
        if isinstance(v, (int, float)):
            ev.define(k, float(v))
    case = FE.Case.__new__(FE.Case)
    case.ev, case.icond = ev, T._published()[-1]     # the default Params' formulas
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                       beads=O.beads(), icond=case.icond_programs(), tau=1.0, tau_min=info["tau_min"],
                       delta=info["delta"], device_ic=True)
    assert sim.ic_where == "device"
    x = sim.interior()
    sim.close()
    assert _sha(x) == meta["ic_sha256"]
