"""HIP path vs the reference: golden vectors produced by the reference itself and the pinned CPU
oracle, bit for bit for calc_mode 0/1/10/11 (mode 2: device cosh, tolerance stated per test).
Every call goes through libpft's C ABI (RK_MPI_SA_*, f_generic_model*, pft_solve_ex)."""
import ctypes as C
import threading

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu

# mode 2 only: device cosh (ROCm ocml) vs glibc cosh differ by <= 1 ulp -> a few ulp in K
MODE2_RTOL = 1e-13


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


# kernel flavours: (tile width, recompute stage inputs)
FLAVOURS = {"cache": (0, False), "fused32": (32, True), "fused16": (16, True), "default": (1, True),
            "fusedauto": (2, True)}   # the fused kernel with the tile fitted to n1 x n2, at any size


def make_sim(meta, initial, mode=None, flavour=None, **kw):
    if flavour is not None:
        kw["tile"], kw["recompute"] = FLAVOURS[flavour]
    Pm, info = O.params_from_meta(meta)
    mode = info["calc_mode"] if mode is None else mode
    return P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode, Pm,
                        initial=initial, tau=kw.pop("tau", 1.0), tau_min=info["tau_min"],
                        delta=info["delta"], **kw), Pm, info


def assert_rhs(K, ref, mode):
    if mode == 2:
        scale = np.abs(ref).max(axis=(1, 2, 3), keepdims=True) + 1e-300
        assert np.all(np.abs(K - ref) <= MODE2_RTOL * scale)
    else:
        assert np.array_equal(K, ref)


@pytest.mark.parametrize("case,key", [("g20", "ic"), ("ragged", "state")])
@pytest.mark.parametrize("mode", [0, 1, 2, 10, 11])
@pytest.mark.parametrize("tag", ["t0", "t1"])
@pytest.mark.parametrize("flavour", sorted(FLAVOURS))
def test_rhs_device(case, key, mode, tag, flavour):
    meta, A = O.load_case(case)
    sim, Pm, info = make_sim(meta, A[key], mode=mode, init_solver=False, flavour=flavour)
    dw, _ = P.rhs(sim, meta["rhs_times"][tag])
    K = dw.reshape((3,) + sim.N)[:, 2:-2, 2:-2, 2:-2]
    assert_rhs(K, A[f"rhs_m{mode}_{tag}"], mode)
    sim.close()


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("gl_static", [False, True])
@pytest.mark.parametrize("flavour", sorted(FLAVOURS))
def test_trajectory_bitwise(mode, gl_static, flavour):
    """RK_MPI_SA_solve to several snapshot times (intertrack.c:2272-2283): t, h, step counts and
    the fields equal the reference's after 1171 attempted steps (mode 0)"""
    meta, A = O.load_case("g20")
    sim, Pm, info = make_sim(meta, A[f"traj_m{mode}_ic"], mode=mode, gl_static=gl_static, flavour=flavour)
    for i, T in enumerate(meta["traj_times"]):
        rc = sim.solve(T)
        ref = meta[f"traj_m{mode}"][i]
        assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
            (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        assert np.array_equal(sim.interior(), A[f"traj_m{mode}_state{i}"])
    assert sim.stats().path == 1
    sim.close()


@pytest.mark.parametrize("mode", [10, 11])
@pytest.mark.parametrize("flavour", sorted(FLAVOURS) + ["pairs"])
def test_trajectory_no_flux_modes_bitwise(mode, flavour):
    """calc_mode 10 and 11 on the device to the g20 snapshot times: the reference's own trajectory
    (tests/golden/g20nf) bit for bit, every kernel flavour and the pair kernels forced"""
    meta, A = O.load_case("g20nf")
    m = {"params": meta[f"m{mode}_params"]}
    pair = flavour == "pairs"
    P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 2 if pair else 1)
    try:
        sim, Pm, info = make_sim(m, A[f"traj_m{mode}_ic"], mode=mode, flavour="fusedauto" if pair else flavour)
        for i, T in enumerate(meta["traj_times"]):
            rc = sim.solve(T)
            ref = meta[f"traj_m{mode}"][i]
            assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
            assert np.array_equal(sim.interior(), A[f"traj_m{mode}_state{i}"])
        st = sim.stats()
        assert st.path == 1 and bool(st.pairs) == pair
        sim.close()
    finally:
        P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 1)


def test_trajectory_mode2_tolerance():
    meta, A = O.load_case("g20")
    sim, Pm, info = make_sim(meta, A["traj_m2_ic"], mode=2)
    T = meta["traj_times"][0]
    sim.solve(T)
    ref = meta["traj_m2"][0]
    assert sim.t == float.fromhex(ref[0])
    assert abs(sim.system.steps_total - ref[3]) <= 2
    got, exp = sim.interior(), A["traj_m2_state0"]
    assert np.all(np.abs(got - exp) <= 1e-10 * np.abs(exp).max(axis=(1, 2, 3), keepdims=True))
    sim.close()


@pytest.mark.parametrize("tag", ["small", "large"])
def test_single_step(tag):
    meta, A = O.load_case("ragged")
    m = meta[f"step_{tag}"]
    sim, Pm, info = make_sim(meta, A["state"], mode=0, tau=m["h0"], t0=m["t0"])
    rc = sim.solve(m["T"])
    r = m["result"]
    assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
        (float.fromhex(r[0]).hex(), float.fromhex(r[1]).hex(), r[2], r[3], r[4])
    assert np.array_equal(sim.interior(), A[f"step_{tag}"])
    sim.close()


def test_step_limited_resident_equals_continuous():
    """pft_solve_ex in chunks of attempted steps with x kept on the device == one solve"""
    meta, A = O.load_case("g20")
    sim, Pm, info = make_sim(meta, A["traj_m0_ic"])
    flags = P.PFT_SOLVE_KEEP_DEVICE
    for i, T in enumerate(meta["traj_times"][:2]):     # same snapshot times as the golden run
        while True:
            rc = sim.solve_ex(T, 37, flags)
            flags = P.PFT_SOLVE_KEEP_DEVICE | P.PFT_SOLVE_REUSE_DEVICE
            if rc != 2:
                break
        ref = meta["traj_m0"][i]
        assert (sim.t, sim.system.steps, sim.system.steps_total) == (float.fromhex(ref[0]), ref[2], ref[3])
    sim.download()
    assert np.array_equal(sim.interior(), A["traj_m0_state1"])
    sim.close()


# fusedauto grids and the tile fused_geometry picks (wx pairs x ty rows): 50x50 -> 25x10 (exact),
# 252x14 -> 18x14, 318x10 -> 25x10 (partial x tile), 130x70 and 66x38 -> 33x7 (one tile wide),
# 100x36 -> 28x9
@pytest.mark.parametrize("dims,flavour", [((30, 30, 60), "fused32"), ((30, 30, 60), "fused16"),
                                          ((66, 38, 21), "fused32"), ((17, 9, 13), "fused32"),
                                          ((130, 70, 9), "fused16"), ((66, 38, 21), "cache"),
                                          ((130, 70, 9), "cache"), ((50, 50, 20), "fusedauto"),
                                          ((252, 14, 6), "fusedauto"), ((318, 10, 5), "fusedauto"),
                                          ((130, 70, 9), "fusedauto"), ((66, 38, 21), "fusedauto"),
                                          ((100, 36, 12), "fusedauto")])
def test_matches_oracle_larger_grid(dims, flavour):
    """default Params on several grids (odd n1 falls back to the cache-based kernel; tiles with
    partial x/y coverage; automatic tiles of any width), from the default IC, 12 attempted steps
    vs the oracle"""
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    n1, n2, n3 = dims
    info = dict(info, n1=n1, n2=n2, n3=n3)
    sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), 0, Pm, beads=O.beads(),
                       tau=1.0, tau_min=info["tau_min"], delta=info["delta"], tile=FLAVOURS[flavour][0],
                       recompute=FLAVOURS[flavour][1])
    ic = sim.interior()
    rc = sim.solve_ex(1e9, 12, 0)
    assert rc == 2
    res = O.solve(info, Pm, 0, ic, 0.0, 1.0, [1e9], max_steps_total=12)[0]
    assert (sim.t, sim.h, sim.system.steps, sim.system.steps_total) == (res[0], res[1], res[2], res[3])
    assert np.array_equal(sim.interior(), res[5])
    sim.close()


def _loopback_run(meta, initial, nprocs, times, mode=0, gl_static=False, flavour="fused32"):
    L = P.lib()
    group = C.c_void_p()
    assert L.pft_comm_init_loopback(C.byref(group), nprocs) == 0
    out, errs = [None] * nprocs, []

    def worker(r):
        try:
            mine = C.c_void_p()
            assert L.pft_comm_loopback_rank(group, r, C.byref(mine)) == 0
            L.pft_comm_set_current(mine)
            Pm, info = O.params_from_meta(meta)
            sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode,
                               Pm, nprocs=nprocs, rank=r, initial=initial, tau=1.0, tau_min=info["tau_min"],
                               delta=info["delta"], gl_static=gl_static, tile=FLAVOURS[flavour][0],
                               recompute=FLAVOURS[flavour][1])
            res = []
            for T in times:
                rc = sim.solve(T)
                res.append((sim.t, sim.h, sim.system.steps, sim.system.steps_total, rc, sim.interior()))
            out[r] = res
            sim.close()
            L.pft_comm_set_current(None)
            L.pft_comm_destroy(mine)
        except BaseException as e:   # noqa: BLE001 -- surfaced below
            errs.append(e)

    ths = [threading.Thread(target=worker, args=(r,)) for r in range(nprocs)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    L.pft_comm_destroy(group)
    if errs:
        raise errs[0]
    return out


@pytest.mark.parametrize("nprocs", [2, 4])
@pytest.mark.parametrize("gl_static", [False, True])
@pytest.mark.parametrize("flavour", ["default", "fused32", "fused16", "cache"])
def test_multislab_loopback_bitwise(nprocs, gl_static, flavour):
    """Z-slab decomposition with halo exchange (boundary planes first, interior overlapped) over
    the loopback transport on one GPU: identical to the single-slab reference trajectory (F6)"""
    meta, A = O.load_case("g20")
    times = meta["traj_times"][:2]
    out = _loopback_run(meta, A["traj_m0_ic"], nprocs, times, gl_static=gl_static, flavour=flavour)
    for i in range(len(times)):
        ref = meta["traj_m0"][i]
        for r in range(nprocs):
            t, h, s, st, rc, _ = out[r][i]
            assert (t, s, st, rc) == (float.fromhex(ref[0]), ref[2], ref[3], ref[4])
        full = np.concatenate([out[r][i][5] for r in range(nprocs)], axis=1)
        assert np.array_equal(full, A[f"traj_m0_state{i}"])


def _self_exchange_comm():
    L = P.lib()
    uid = (C.c_char * 128)()
    assert L.pft_comm_get_unique_id(uid) == 0
    comm = C.c_void_p()
    assert L.pft_comm_init_rccl(C.byref(comm), 1, 0, uid, 0) == 0
    assert L.pft_comm_set_self_exchange(comm, 1) == 0
    assert L.pft_comm_splits(comm) == 1
    return comm


@pytest.mark.parametrize("gl_static", [False, True])
@pytest.mark.parametrize("flavour", ["default", "fusedauto", "fused16", "fused32", "cache"])
def test_rccl_stage_pipeline_self_exchange_bitwise(gl_static, flavour):
    """the N > 1 stage pipeline through real RCCL calls on one GPU (pft_comm_set_self_exchange):
    both boundary planes in one launch, ncclSend/ncclRecv on the priority comm stream beside the
    interior sweep, the eps max by ncclAllReduce and its publication on the comm stream.  The
    exchanged planes land in the slab's own ghost planes, which one slab never reads, so the
    trajectory must equal the reference's bit for bit"""
    L = P.lib()
    comm = _self_exchange_comm()
    L.pft_comm_set_current(comm)
    try:
        meta, A = O.load_case("g20")
        sim, Pm, info = make_sim(meta, A["traj_m0_ic"], mode=0, gl_static=gl_static, flavour=flavour)
        for i, T in enumerate(meta["traj_times"][:2]):
            rc = sim.solve(T)
            ref = meta["traj_m0"][i]
            assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
            assert np.array_equal(sim.interior(), A[f"traj_m0_state{i}"])
        sim.close()
    finally:
        L.pft_comm_set_current(None)
        L.pft_comm_destroy(comm)


def test_rccl_stage_pipeline_self_exchange_larger_grid():
    """the same pipeline on a 100 x 36 x 40 grid with the automatic fused tile (several z-chunks,
    boundary launch of two one-plane chunks) vs the oracle, 12 attempted steps"""
    L = P.lib()
    comm = _self_exchange_comm()
    L.pft_comm_set_current(comm)
    try:
        meta, A = O.load_case("g20")
        Pm, info = O.params_from_meta(meta)
        n1, n2, n3 = 100, 36, 40
        info = dict(info, n1=n1, n2=n2, n3=n3)
        sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), 0, Pm, beads=O.beads(), tau=1.0,
                           tau_min=info["tau_min"], delta=info["delta"], tile=2)
        ic = sim.interior()
        assert sim.solve_ex(1e9, 12, 0) == 2
        assert sim.stats().kernel_launches > 0
        res = O.solve(info, Pm, 0, ic, 0.0, 1.0, [1e9], max_steps_total=12)[0]
        assert (sim.t, sim.h, sim.system.steps, sim.system.steps_total) == (res[0], res[1], res[2], res[3])
        assert np.array_equal(sim.interior(), res[5])
        geo = sim.tile_geometry()
        assert geo[5] == (2, 28, 9)      # fused kernel, fused_geometry's tile for 100 x 36
        sim.close()
    finally:
        L.pft_comm_set_current(None)
        L.pft_comm_destroy(comm)


def test_host_staged_path_with_foreign_rhs():
    """an RK_RightHandSide the library does not know (here: the oracle's RHS as a host callback)
    takes the host-staged path: host f, HIP combines/error/update over the chunk table"""
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    sim, _, _ = make_sim(meta, A["traj_m0_ic"], mode=0)
    g = O.make_grid(info)
    n = 3 * sim.S
    OL = O.lib()

    @P.RHS_FN
    def f(t, w, dw):
        OL.pft_or_rhs(C.byref(g), O.ptr(Pm), 0, t, w, dw)

    @P.META_FN
    def meta_f():
        return C.cast(f, C.c_void_p).value

    sim.system.meta_f = C.cast(meta_f, C.c_void_p).value
    T = meta["traj_times"][0]
    rc = sim.solve(T)
    ref = meta["traj_m0"][0]
    assert sim.stats().path == 2
    assert (sim.t, sim.h, sim.system.steps, sim.system.steps_total, rc) == \
        (float.fromhex(ref[0]), float.fromhex(ref[1]), ref[2], ref[3], ref[4])
    assert np.array_equal(sim.interior(), A["traj_m0_state0"])
    assert n == sim.x.size
    sim.close()


def _full_size_case():
    from porousfreezethaw_amd import params as PR
    base = PR.default_params(grid_nodes=400, calc_mode=0)
    info = {k: base[k] for k in ("n1", "n2", "n3", "L1", "L2", "L3", "tau_min", "delta")}
    return base, P.params_array(base), info


def test_full_size_400_bitwise_and_rank_invariant():
    """BASELINE's 400^3 (200x200x400, default Params, beads) at full size: 3 attempted steps of the
    device path equal the oracle bit for bit, and a 2-slab loopback run (halo exchange, boundary
    planes first) equals the single-slab one (rank-count invariance)"""
    base, Pm, info = _full_size_case()
    L3s = (info["L1"], info["L2"], info["L3"])
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], L3s, 0, Pm, beads=O.beads(), tau=1.0,
                       tau_min=info["tau_min"], delta=info["delta"])
    ic = sim.interior()
    assert sim.solve_ex(1e9, 3, 0) == 2
    got = (sim.t, sim.h, sim.system.steps, sim.system.steps_total)
    x1 = sim.interior()
    sim.close()
    res = O.solve(info, Pm, 0, ic, 0.0, 1.0, [1e9], max_steps_total=3)[0]
    assert got == tuple(res[:4])
    assert np.array_equal(x1, res[5])
    del res

    L = P.lib()
    group = C.c_void_p()
    assert L.pft_comm_init_loopback(C.byref(group), 2) == 0
    out, errs = [None, None], []

    def worker(r):
        try:
            mine = C.c_void_p()
            assert L.pft_comm_loopback_rank(group, r, C.byref(mine)) == 0
            L.pft_comm_set_current(mine)
            s = P.Simulation(info["n1"], info["n2"], info["n3"], L3s, 0, Pm, nprocs=2, rank=r, initial=ic,
                             tau=1.0, tau_min=info["tau_min"], delta=info["delta"])
            assert s.solve_ex(1e9, 3, 0) == 2
            out[r] = ((s.t, s.h, s.system.steps, s.system.steps_total), s.interior())
            s.close()
            L.pft_comm_set_current(None)
            L.pft_comm_destroy(mine)
        except BaseException as e:  # noqa: BLE001 -- surfaced below
            errs.append(e)

    ths = [threading.Thread(target=worker, args=(r,)) for r in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    L.pft_comm_destroy(group)
    if errs:
        raise errs[0]
    for r in range(2):
        assert out[r][0] == got
    assert np.array_equal(np.concatenate([out[0][1], out[1][1]], axis=1), x1)


def test_snapshot_restart_continues_trajectory(tmp_path):
    """continue_series (intertrack.c:1584-1669): a snapshot written at t = 36 s and read back into
    a fresh solver (t, tau and the parameters from the dataset) continues the reference's
    trajectory bit for bit to t = 360 s"""
    meta, A = O.load_case("g20")
    sim, Pm, info = make_sim(meta, A["traj_m0_ic"], mode=0)
    T0, T1 = meta["traj_times"][:2]
    sim.solve(T0)
    path = str(tmp_path / "image.001.000.ncd")
    P.save_snapshot(sim, path, P.snapshot_info(t=sim.t, tau=sim.h, final_time=T1, delta=info["delta"], calc_mode=0,
                                               snapshot=1, total_snapshots=10, comment="restart test"))
    s0, st0 = sim.system.steps, sim.system.steps_total
    sim.close()
    n1, n2, n3, inf, prm = P.read_snapshot_info(path)
    assert (inf.L1, inf.L2, inf.L3) == (info["L1"], info["L2"], info["L3"])
    sim2 = P.Simulation(n1, n2, n3, (inf.L1, inf.L2, inf.L3), inf.calc_mode, prm,
                        initial=np.zeros((3, n3, n2, n1)), tau=inf.tau, t0=inf.t, tau_min=info["tau_min"],
                        delta=inf.delta)
    P.load_snapshot(sim2, path)
    sim2.solve(inf.final_time)
    ref = meta["traj_m0"][1]
    assert (sim2.t, sim2.h, s0 + sim2.system.steps, st0 + sim2.system.steps_total) == \
        (float.fromhex(ref[0]), float.fromhex(ref[1]), ref[2], ref[3])
    assert np.array_equal(sim2.interior(), A["traj_m0_state1"])
    sim2.close()


@pytest.mark.parametrize("mode", [0, 1, 10, 11])
@pytest.mark.parametrize("flavour", ["default", "fused32", "fused16", "cache"])
def test_rhs_with_temperature_noise(mode, flavour):
    """u_noise (u_noise_amp != 0, equation.c:450-456, 676-687): the device RHS with the slab's
    noise field equals the oracle's stencil given the same field"""
    meta, A = O.load_case("ragged")
    Pm, info = O.params_from_meta(meta)
    Pm = Pm.copy()
    Pm[O.PARAM_NAMES.index("u_noise_amp")] = 0.5
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode, Pm,
                       initial=A["state"], init_solver=False, tile=FLAVOURS[flavour][0],
                       recompute=FLAVOURS[flavour][1])
    n = info["n1"] * info["n2"] * info["n3"]
    noise = np.ctypeslib.as_array(P.lib().pft_model_noise(), shape=(n,)).copy()
    assert np.abs(noise).max() > 0
    t = meta["rhs_times"]["t1"]
    dw, _ = P.rhs(sim, t)
    K = dw.reshape((3,) + sim.N)[:, 2:-2, 2:-2, 2:-2]
    sim.close()
    g = O.make_grid(info)
    w = O.pad(g, A["state"])
    O.lib().pft_or_bcond(C.byref(g), O.ptr(Pm), t, O.ptr(w))
    dwo = np.zeros_like(w)
    O.lib().pft_or_stencil(C.byref(g), O.ptr(Pm), mode, O.ptr(w), O.ptr(noise), O.ptr(dwo))
    assert np.array_equal(K, O.unpad(g, dwo))


@pytest.mark.parametrize("flavour", ["default", "fusedauto"])
def test_gl_negative_zero_keeps_reference_bits(flavour):
    """stage 5 skips storing gl's x(t+h) = x + coef*0.0 when that is x bit for bit
    (pft_slab_set_gl_keep); a -0.0 in gl (-0.0 + 0.0 = +0.0) must turn that off: 12 attempted
    steps from a state with -0.0 and +0.0 in gl equal the oracle's bit for bit"""
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    n1, n2, n3 = 30, 30, 24
    info = dict(info, n1=n1, n2=n2, n3=n3)
    sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), 0, Pm, beads=O.beads(), tau=1.0,
                       tau_min=info["tau_min"], delta=info["delta"], init_solver=False)
    ic = sim.interior().copy()
    sim.close()
    ic[2, :, :5, :] = 0.0
    ic[2, 3:9, :3, 2:11] = -0.0
    assert np.signbit(ic[2]).sum() > 0
    sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), 0, Pm, initial=ic, tau=1.0,
                       tau_min=info["tau_min"], delta=info["delta"], tile=FLAVOURS[flavour][0],
                       recompute=FLAVOURS[flavour][1])
    assert sim.solve_ex(1e9, 12, 0) == 2
    res = O.solve(info, Pm, 0, ic, 0.0, 1.0, [1e9], max_steps_total=12)[0]
    assert (sim.t, sim.h, sim.system.steps, sim.system.steps_total) == (res[0], res[1], res[2], res[3])
    got = sim.interior()
    assert np.array_equal(got, res[5])
    assert np.array_equal(np.signbit(got[2]), np.signbit(res[5][2]))
    sim.close()


# ---- u_noise pinned to the reference (tests/golden/gnoise, u_noise_amp = 0.5 K, one rank) ------

def _noise_sim(meta, A, mode, initial, **kw):
    """libpft's model set up as the reference's: its PrecalculateData draws the noise field from
    the C library's rand() (equation.c:450-456), seeded here as the reference harness leaves it"""
    C.CDLL("libc.so.6").srand(1)
    sim, Pm, info = make_sim({"params": meta[f"m{mode}_params"]}, initial, mode=mode, **kw)
    n = info["n1"] * info["n2"] * info["n3"]
    noise = np.ctypeslib.as_array(P.lib().pft_model_noise(), shape=(n,)).copy()
    assert np.array_equal(noise.reshape(A["noise"].shape), A["noise"]), "libpft's noise field differs"
    return sim


@pytest.mark.parametrize("mode", [0, 10, 1, 11])
@pytest.mark.parametrize("flavour", ["default", "fused32", "fusedauto", "cache"])
def test_noise_rhs_equals_reference(mode, flavour):
    """libpft's noise field and the device RHS of the four models that add it (equation.c:676,
    687) equal the reference's, at a state with mixed phases"""
    meta, A = O.load_case("gnoise")
    sim = _noise_sim(meta, A, mode, A[meta["rhs_state"]], init_solver=False, flavour=flavour)
    dw, _ = P.rhs(sim, meta["rhs_time"])
    K = dw.reshape((3,) + sim.N)[:, 2:-2, 2:-2, 2:-2]
    sim.close()
    assert np.array_equal(K, A[f"rhs_m{mode}"])


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("flavour", ["default", "fusedauto", "cache", "pairs"])
def test_noise_trajectory_equals_reference(mode, flavour):
    """RK_MPI_SA_solve with u_noise to t = 36 and 360 s: t, h, step counts and fields equal the
    reference's (the pair kernels forced: both stages of a pair see the noise)"""
    meta, A = O.load_case("gnoise")
    pair = flavour == "pairs"
    P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 2 if pair else 0)
    try:
        sim = _noise_sim(meta, A, mode, A["ic"], flavour="fusedauto" if pair else flavour)
        for i, T in enumerate(meta["traj_times"]):
            rc = sim.solve(T)
            ref = meta[f"traj_m{mode}"][i]
            assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
            assert np.array_equal(sim.interior(), A[f"traj_m{mode}_state{i}"])
        st = sim.stats()
        sim.close()
    finally:
        P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 1)
    assert st.path == 1 and st.pairs == (1 if pair else 0)
