"""RK_MPI_SA_solve control flow on the HIP path against the reference's own runs (tests/golden/ctl,
made by oracle/ref_harness.c `solvex` from /root/reference compiled in place):

  - NaN handling (RK_MPI_SA_handle_NAN(1), hybrid2.c:464-504, 624-646): a NaN / inf in the state
    makes every attempt non-finite; h /= 10 until h/(T-t) < 1e-11, then return -4 with t, h left
    as they were and steps_total counting the retries.  Three (state, t0, h0, T) variants.
  - NaN retries that recover: h0 = 1e8 s overflows the stage values to inf/NaN; the reference
    retries with h/10 until the error norm is finite, then steps on.  A Service_Callback logs
    (steps, t, h) after every accepted step (hybrid2.c:676-685) and interrupts at the 10th.
  - Service_Callback break and resume (hybrid2.c:697-705): interrupt at the 25th accepted step
    (return 1, t and h = new_h left in the system), resume to T; every callback call, both
    returned rows and both states equal the reference's -- and the resumed state equals the
    uninterrupted golden trajectory (g20 traj_m0_state0).
Every comparison is bit for bit (hex floats, integer counters, array_equal with NaN = NaN)."""
import ctypes as C

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


def _run(name, flavour_tile=None, pair=1):
    """pair 2: stages 2+3 and 4+5 as pair kernels (PFT_OPT_PAIR; needs an LDS-tiled flavour)"""
    P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, pair)
    meta, A = O.load_case("ctl")
    run = meta["runs"][name]
    Pm, info = O.params_from_meta(meta)
    state = A.get(f"{name}_ic", A["ic"])
    kw = {} if flavour_tile is None else {"tile": flavour_tile}
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                       initial=state, tau=run["h0"], t0=run["t0"], tau_min=info["tau_min"],
                       delta=info["delta"], **kw)
    L = sim.lib
    log = []

    @P.SERVICE_FN
    def cb(final, s):
        log.append([s.contents.steps, s.contents.t.hex(), s.contents.h.hex()])
        return 1 if run["break_at"] > 0 and len(log) == run["break_at"] else 0

    if run["break_at"] >= 0:
        sim.system.Service_Callback = C.cast(cb, C.c_void_p).value
    L.RK_MPI_SA_handle_NAN(run["handle_nan"])
    rows, states = [], []
    try:
        for T in run["T"]:
            rc = L.RK_MPI_SA_solve(T, C.byref(sim.system))
            rows.append([sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc,
                         L.RK_MPI_SA_check_NAN()])
            states.append(sim.interior())
    finally:
        L.RK_MPI_SA_handle_NAN(0)
        path = sim.stats().path
        pairs = sim.stats().pairs
        sim.close()
        L.pft_solver_set_option(P.PFT_OPT_PAIR, 1)
    assert pairs == (pair == 2)
    return run, A, rows, log, states, path


def _ref_rows(run):
    return [[float.fromhex(r[0]).hex(), float.fromhex(r[1]).hex()] + r[2:] for r in run["traj"]]


@pytest.mark.parametrize("tile,pair", [(None, 1), (2, 2)])
@pytest.mark.parametrize("name", ["nan_giveup_a", "nan_giveup_b", "nan_giveup_c"])
def test_nan_gives_up_like_the_reference(name, tile, pair):
    run, A, rows, log, states, path = _run(name, tile, pair)
    assert path == 1
    assert rows == _ref_rows(run)
    assert rows[0][4] == -4 and rows[0][5] == 1
    assert np.array_equal(states[0], A[f"{name}_state0"], equal_nan=True)


@pytest.mark.parametrize("tile,pair", [(None, 1), (32, 1), (32, 2)])
def test_nan_retries_then_recovers_like_the_reference(tile, pair):
    """tile None: the automatic choice (the cache kernel, aux arrays, for this 10-cell plane); 32: the
    fused LDS-tiled recompute kernel with the speculative stage 1; pair 2: and the pair kernels"""
    run, A, rows, log, states, path = _run("nan_retry", tile, pair)
    assert rows == _ref_rows(run)
    assert rows[0][3] - rows[0][2] > 1 and rows[0][5] == 1      # retries happened, NaN seen
    assert log == [[c[0], float.fromhex(c[1]).hex(), float.fromhex(c[2]).hex()] for c in run["cb"]]
    assert np.array_equal(states[0], A["nan_retry_state0"])


@pytest.mark.parametrize("tile,pair", [(None, 1), (32, 1), (32, 2)])
def test_service_callback_break_and_resume_like_the_reference(tile, pair):
    run, A, rows, log, states, path = _run("cb_break", tile, pair)
    assert rows == _ref_rows(run)
    assert rows[0][4] == 1 and rows[1][4] == 0
    assert log == [[c[0], float.fromhex(c[1]).hex(), float.fromhex(c[2]).hex()] for c in run["cb"]]
    assert len(log) == run["traj"][1][2]                      # one call per accepted step
    assert np.array_equal(states[0], A["cb_break_state0"])
    assert np.array_equal(states[1], A["cb_break_state1"])
    g20, G = O.load_case("g20")
    assert np.array_equal(states[1], G["traj_m0_state0"])   # = the uninterrupted trajectory
