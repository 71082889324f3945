"""The reference ABI's edge behaviour on the GPU (include/RK_MPI_SAsolver.h, reference
RK_MPI_SAsolver.h:291-392, RK_MPI_SAsolver_hybrid2.c):

  - RK_MPI_SA_init allocates the solver's buffers (hybrid2.c:101-112) and returns -1 when the
    memory is not there (here: HBM filled first), leaving the solver uninitialised;
  - meta_f() switching to another right-hand side after an accepted step (hybrid2.c:732): the
    integration continues with the new f (libpft: from the fused device path onto the host-staged
    path) and ends on the reference trajectory;
  - a Service_Callback on the fused path can fetch the current x (pft_solver_download);
  - the host-staged path leaves the ghost layers the last f(t, x) wrote in x, as the reference's
    in-place update does (hybrid2.c:657-668)."""
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


def _g20_sim(**kw):
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                       initial=A["traj_m0_ic"], tau=1.0, tau_min=info["tau_min"], delta=info["delta"], **kw)
    return sim, meta, A, Pm, info


def test_init_returns_minus_one_when_hbm_is_full():
    L = P.lib()
    from porousfreezethaw_amd import params as PR
    base = PR.default_params(grid_nodes=400)
    Pm = P.params_array(base)
    sim = P.Simulation(base["n1"], base["n2"], base["n3"], (base["L1"], base["L2"], base["L3"]), 0, Pm,
                       initial=np.zeros((3, base["n3"], base["n2"], base["n1"])), init_solver=False)
    hold = []
    try:
        chunk = 8 << 30
        while len(hold) < 64:              # at most 512 GB requested; the card has 288 GB
            p = C.c_void_p()
            if L.pft_dev_alloc(C.byref(p), C.c_size_t(chunk)) != 0:
                if chunk <= (256 << 20):
                    break
                chunk //= 2
                continue
            hold.append(p)
        assert L.RK_MPI_SA_init(3 * sim.S, P.MPI_COMM_WORLD, 0) == -1
        assert L.pft_solver_last_status() <= -1000              # the HIP error behind it
        assert L.RK_MPI_SA_cleanup() == -3                       # not initialised
    finally:
        for p in hold:
            L.pft_dev_free(p)
    assert L.RK_MPI_SA_init(3 * sim.S, P.MPI_COMM_WORLD, 0) == 0
    assert L.RK_MPI_SA_cleanup() == 0
    sim.close()


def test_meta_f_switch_continues_on_the_host_path():
    """after 40 accepted steps on the device, meta_f hands out the oracle's RHS as a host
    callback (same bits as the reference's); the solve goes on and ends on golden g20"""
    sim, meta, A, Pm, info = _g20_sim(tile=32)
    g = O.make_grid(info)
    OL = O.lib()
    dev_f = sim.lib.mf_single()                     # libpft's device RHS (restype c_void_p: an int)
    accepted = []

    @P.RHS_FN
    def host_f(t, w, dw):
        OL.pft_or_rhs(C.byref(g), O.ptr(Pm), 0, t, w, dw)

    host_addr = C.cast(host_f, C.c_void_p).value

    @P.META_FN
    def meta_f():
        return dev_f if len(accepted) < 40 else host_addr

    @P.SERVICE_FN
    def cb(final, s):
        accepted.append(s.contents.steps)
        return 0

    sim.system.meta_f = C.cast(meta_f, C.c_void_p).value
    sim.system.Service_Callback = C.cast(cb, C.c_void_p).value
    T = meta["traj_times"][0]
    rc = sim.solve(T)
    ref = meta["traj_m0"][0]
    assert sim.stats().path == 2                     # ended on the host-staged path
    assert (sim.t, sim.system.steps, sim.system.steps_total, rc) == \
        (float.fromhex(ref[0]), ref[2], ref[3], ref[4])
    # with a Service_Callback installed the reference leaves system->h = the last (truncated) step
    # (hybrid2.c:680 runs before the FINISHED break): the ctl fixture's callback run to 36 s
    ctl, _ = O.load_case("ctl")
    assert sim.h == float.fromhex(ctl["runs"]["cb_break"]["traj"][1][1])
    assert np.array_equal(sim.interior(), A["traj_m0_state0"])
    sim.close()


def test_callback_downloads_current_x():
    """the 25th callback call downloads x: the reference's state after 25 accepted steps
    (tests/golden/ctl cb_break_state0)"""
    meta, A = O.load_case("ctl")
    sim, _, _, _, _ = _g20_sim(tile=32)
    got = []

    @P.SERVICE_FN
    def cb(final, s):
        if s.contents.steps == 25:
            assert sim.lib.pft_solver_download(s) == 0
            got.append(sim.interior())
        return 0

    sim.system.Service_Callback = C.cast(cb, C.c_void_p).value
    sim.solve(36.0)
    assert sim.stats().path == 1
    assert len(got) == 1 and np.array_equal(got[0], A["cb_break_state0"])
    assert sim.lib.pft_solver_download(C.byref(sim.system)) == 0   # after the call: still valid
    sim.close()


def test_host_staged_path_keeps_the_ghosts_f_wrote():
    """a foreign RHS (the oracle's, which runs bcond_setup on its input like equation.c:624):
    after the solve every value of the padded x, ghosts included, equals the oracle's own x"""
    sim, meta, A, Pm, info = _g20_sim()
    g = O.make_grid(info)
    OL = O.lib()

    @P.RHS_FN
    def f(t, w, dw):
        OL.pft_or_rhs(C.byref(g), O.ptr(Pm), 0, t, w, dw)

    @P.META_FN
    def meta_f():
        return C.cast(f, C.c_void_p).value

    sim.system.meta_f = C.cast(meta_f, C.c_void_p).value
    T = meta["traj_times"][0]
    sim.solve(T)
    assert sim.stats().path == 2
    x = O.pad(g, A["traj_m0_ic"]).ravel()
    t, h = C.c_double(0.0), C.c_double(1.0)
    steps, total = C.c_long(0), C.c_long(0)
    OL.pft_or_solve(C.byref(g), O.ptr(Pm), 0, T, C.byref(t), C.byref(h), info["tau_min"], info["delta"], 0,
                    O.ptr(x), C.byref(steps), C.byref(total), 0, O.EXCHANGE_FN(), O.ALLREDUCE_FN(), None)
    assert np.array_equal(sim.x, x)
    sim.close()


def test_device_failure_in_own_rhs_on_host_path_is_a_device_error():
    """libpft's own f (f_generic_model01) called by the host-staged path -- a DDLBF_Rearrange
    callback keeps the solve off the fused path (hybrid2.c:726-729) -- whose device evaluation
    fails (PFT_OPT_FAIL_RHS): the solve must return PFT_SOLVE_DEVICE_ERROR, not accept the NaN
    state f leaves behind (the reference driver runs with NaN handling off, intertrack.c:2193)"""
    sim, meta, A, Pm, info = _g20_sim()

    @P.REARRANGE_FN
    def same(n):
        return n

    sim.system.DDLBF_Rearrange = C.cast(same, C.c_void_p).value
    L = sim.lib
    try:
        assert L.pft_solver_set_option(P.PFT_OPT_FAIL_RHS, 7) == 0    # the 2nd step's second stage
        rc = L.RK_MPI_SA_solve(meta["traj_times"][0], C.byref(sim.system))
        assert sim.stats().path == 2
        assert rc == P.PFT_SOLVE_DEVICE_ERROR
        assert L.pft_solver_last_status() <= -1000
        assert sim.system.steps_total == 1
    finally:
        L.pft_solver_set_option(P.PFT_OPT_FAIL_RHS, 0)
        sim.close()


def test_rearrange_callback_host_path_matches_golden():
    """the same host-staged run with libpft's own f and no failure ends on golden g20"""
    sim, meta, A, Pm, info = _g20_sim()

    @P.REARRANGE_FN
    def same(n):
        return n

    sim.system.DDLBF_Rearrange = C.cast(same, C.c_void_p).value
    T = meta["traj_times"][0]
    rc = sim.solve(T)
    ref = meta["traj_m0"][0]
    assert sim.stats().path == 2
    assert (sim.t, sim.system.steps, sim.system.steps_total, rc) == \
        (float.fromhex(ref[0]), ref[2], ref[3], ref[4])
    assert np.array_equal(sim.interior(), A["traj_m0_state0"])
    sim.close()


def test_meta_f_switch_on_the_capped_step_returns_2():
    """meta_f switches to a foreign RHS on the very attempted step that reaches the cap of
    pft_solve_ex: the call returns 2 (not a run to final_time), and the next call continues on
    the host-staged path to the reference trajectory"""
    # the attempted-step count at which the 10th step is accepted (uninterrupted device run)
    probe = []

    @P.SERVICE_FN
    def cnt(final, s):
        probe.append(s.contents.steps_total)
        return 0

    sim2, meta, A, Pm, info = _g20_sim(tile=32)
    sim2.system.Service_Callback = C.cast(cnt, C.c_void_p).value
    T = meta["traj_times"][0]
    sim2.solve(T)
    sim2.close()
    sim, meta, A, Pm, info = _g20_sim(tile=32)
    g = O.make_grid(info)
    OL = O.lib()
    dev_f = sim.lib.mf_single()
    accepted = []

    @P.RHS_FN
    def host_f(t, w, dw):
        OL.pft_or_rhs(C.byref(g), O.ptr(Pm), 0, t, w, dw)

    host_addr = C.cast(host_f, C.c_void_p).value

    @P.META_FN
    def meta_f():
        return dev_f if len(accepted) < 10 else host_addr

    @P.SERVICE_FN
    def cb(final, s):
        accepted.append(s.contents.steps)
        return 0

    sim.system.meta_f = C.cast(meta_f, C.c_void_p).value
    sim.system.Service_Callback = C.cast(cb, C.c_void_p).value
    cap = probe[9]                              # attempted steps when the 10th step is accepted
    rc = sim.solve_ex(T, cap, 0)
    assert rc == 2 and sim.system.steps_total == cap and sim.system.steps == 10
    rc = sim.solve(T)
    ref = meta["traj_m0"][0]
    assert sim.stats().path == 2
    assert (sim.t, sim.system.steps, sim.system.steps_total, rc) == \
        (float.fromhex(ref[0]), ref[2], ref[3], ref[4])
    assert np.array_equal(sim.interior(), A["traj_m0_state0"])
    sim.close()
