"""Pair kernels (merson_pair, pft_slab_pair): stages 2+3 and 4+5 of the Merson step in one launch
each, stage A evaluated on the tile plus a one-cell ring inside stage B's z-march and never stored.
Bit for bit what the five stage launches give (RK_MPI_SAsolver_hybrid2.c:392-524,657-668), on grids
whose pair tiles fit exactly, leave partial tiles, are one tile wide or narrower than a tile, with
forced z-chunks (interior chunks recompute stage A on the plane below and above), every calc_mode,
gl_static, u_noise, and against the oracle and the reference's golden trajectory."""
import ctypes as C
import threading

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


def _run(dims, mode, pair, steps, kz=None, gl_static=False, noise=0.0, tile=2):
    meta, _ = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    Pm = Pm.copy()
    if noise:
        Pm[O.PARAM_NAMES.index("u_noise_amp")] = noise
    n1, n2, n3 = dims
    L = P.lib()
    L.pft_solver_set_option(P.PFT_OPT_PAIR, 2 if pair else 0)   # 2: also below the size threshold
    # u_noise comes from the C library's rand() (PrecalculateData, equation.c:450-456): the same
    # field for both runs
    C.CDLL("libc.so.6").srand(1)
    try:
        sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), mode, Pm, beads=O.beads(),
                           tau=1.0, tau_min=info["tau_min"], delta=info["delta"], tile=tile, recompute=True,
                           kz=kz, gl_static=gl_static)
        ic = sim.interior()
        rc = sim.solve_ex(1e9, steps, 0)
        assert rc == 2
        st = sim.stats()
        out = (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, sim.interior())
        sim.close()
    finally:
        L.pft_solver_set_option(P.PFT_OPT_PAIR, 1)
    assert st.path == 1
    return out, st.pairs, ic, info, Pm


def _same(a, b):
    assert a[:4] == b[:4]
    assert np.array_equal(a[4], b[4])


# pair tiles (pair_geometry): 30 -> 30 cells wide (one tile), 100x36 -> 20 x 36, 18x12 one
# tile, 66x38 partial x tile, 252x14 / 318x10 wide planes, 2 x 6 and 4 x 130 narrow ones; the 40 x 20
# tile of the 400^3 bench, whose last ring row holds 16 positions beyond the 512 threads (LDS DMA):
# 80x40 (2 x 2 tiles, every one at two walls), 120x60 (3 x 3, an interior tile), 40x40 (one column)
GRIDS = [(30, 30, 60), (100, 36, 40), (18, 12, 30), (66, 38, 21), (252, 14, 6), (318, 10, 5), (2, 6, 5),
         (4, 130, 9), (50, 50, 100), (30, 30, 2), (80, 40, 30), (120, 60, 20), (40, 40, 8)]
TALL = [(80, 40, 30), (120, 60, 20), (40, 40, 8)]


@pytest.mark.parametrize("dims", TALL)
def test_tall_tile_geometry(dims):
    """those grids do run the 40 x 20 tile (pft_slab_pair_geometry)"""
    meta, _ = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    n1, n2, n3 = dims
    L = P.lib()
    L.pft_solver_set_option(P.PFT_OPT_PAIR, 2)
    try:
        sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), 0, Pm, beads=O.beads(), tau=1.0,
                           tau_min=info["tau_min"], delta=info["delta"], tile=2)
        assert sim.solve_ex(1e9, 1, 0) == 2
        tx, ty = C.c_int(), C.c_int()
        L.pft_solver_slab.restype = C.c_void_p
        L.pft_slab_pair_geometry.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        assert L.pft_slab_pair_geometry(L.pft_solver_slab(), C.byref(tx), C.byref(ty)) == 0
        assert (tx.value, ty.value) == (40, 20)
        assert sim.stats().pairs == 1
        sim.close()
    finally:
        L.pft_solver_set_option(P.PFT_OPT_PAIR, 1)


@pytest.mark.parametrize("dims", GRIDS)
@pytest.mark.parametrize("mode", [0, 1, 2, 10, 11])
def test_pair_equals_stage_kernels(dims, mode):
    """12 attempted steps (rejections included: h starts at tau = 1 s) with and without pairs"""
    got, used, *_ = _run(dims, mode, True, 12)
    ref, unused, *_ = _run(dims, mode, False, 12)
    assert used == 1 and unused == 0
    _same(got, ref)


@pytest.mark.parametrize("kz", [1, 2, 3, 7])
@pytest.mark.parametrize("dims", [(30, 30, 60), (66, 38, 21), (2, 6, 5), (80, 40, 30)])
def test_pair_z_chunks(dims, kz):
    """forced z-chunks: every chunk but the first recomputes stage A on the plane below its first,
    every chunk but the last on the plane above its last (one plane per chunk at kz = 1)"""
    got, used, *_ = _run(dims, 0, True, 8, kz=kz)
    ref, *_ = _run(dims, 0, False, 8)
    assert used == 1
    _same(got, ref)


@pytest.mark.parametrize("gl_static", [False, True])
@pytest.mark.parametrize("noise", [0.0, 0.5])
@pytest.mark.parametrize("mode", [0, 1])
def test_pair_gl_static_and_noise(gl_static, noise, mode):
    """gl read from x (gl_static) and u_noise (equation.c:450-456, 676-687) seen by both stages"""
    got, used, *_ = _run((66, 38, 21), mode, True, 10, gl_static=gl_static, noise=noise)
    ref, *_ = _run((66, 38, 21), mode, False, 10, gl_static=gl_static, noise=noise)
    assert used == 1
    _same(got, ref)


@pytest.mark.parametrize("kz", [None, 2])
@pytest.mark.parametrize("dims", [(66, 38, 21), (30, 30, 60), (120, 60, 20)])
def test_pair_gl_negative_zero(dims, kz):
    """a -0.0 in gl turns gl_keep off (pft_slab_set_gl_keep): the pair kernels without GLX, whose
    stage B keeps gl in its own ring and re-loads the operands of its outputs (no lO), against the
    stage launches and the oracle, bit for bit and sign for sign"""
    meta, _ = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    n1, n2, n3 = dims
    info = dict(info, n1=n1, n2=n2, n3=n3)
    sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), 0, Pm, beads=O.beads(), tau=1.0,
                       tau_min=info["tau_min"], delta=info["delta"], init_solver=False)
    ic = sim.interior().copy()
    sim.close()
    ic[2, :, :5, :] = 0.0
    ic[2, 3:9, :3, 2:11] = -0.0
    assert np.signbit(ic[2]).sum() > 0
    L = P.lib()
    outs = []
    for pair in (2, 0):
        L.pft_solver_set_option(P.PFT_OPT_PAIR, pair)
        try:
            sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), 0, Pm, initial=ic, tau=1.0,
                               tau_min=info["tau_min"], delta=info["delta"], tile=2, recompute=True, kz=kz)
            assert sim.solve_ex(1e9, 10, 0) == 2
            st = sim.stats()
            outs.append((sim.t, sim.h, sim.system.steps, sim.system.steps_total, sim.interior(), st.pairs))
            sim.close()
        finally:
            L.pft_solver_set_option(P.PFT_OPT_PAIR, 1)
    got, ref = outs
    assert got[5] == 1 and ref[5] == 0
    assert got[:4] == ref[:4]
    assert np.array_equal(got[4], ref[4]) and np.array_equal(np.signbit(got[4]), np.signbit(ref[4]))
    res = O.solve(info, Pm, 0, ic, 0.0, 1.0, [1e9], max_steps_total=10)[0]
    assert got[:4] == (res[0], res[1], res[2], res[3])
    assert np.array_equal(got[4], res[5]) and np.array_equal(np.signbit(got[4][2]), np.signbit(res[5][2]))


@pytest.mark.parametrize("dims", [(30, 30, 60), (100, 36, 40), (18, 12, 30), (80, 40, 30)])
def test_pair_matches_oracle(dims):
    got, used, ic, info, Pm = _run(dims, 0, True, 12)
    n1, n2, n3 = dims
    res = O.solve(dict(info, n1=n1, n2=n2, n3=n3), Pm, 0, ic, 0.0, 1.0, [1e9], max_steps_total=12)[0]
    assert used == 1
    assert (got[0], got[1], got[2], got[3]) == (res[0].hex(), res[1].hex(), res[2], res[3])
    assert np.array_equal(got[4], res[5])


@pytest.mark.parametrize("mode", [0, 1, 10, 11])
@pytest.mark.parametrize("gl_static", [False, True])
def test_pair_golden_trajectory(mode, gl_static):
    """the reference's own trajectory (g20, 10x10x20) through the pair kernels to every snapshot
    time, where the golden holds it (modes 0/1); modes 10/11 against the stage kernels"""
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    ic = A["traj_m0_ic"] if mode not in (0, 1) else A[f"traj_m{mode}_ic"]
    runs = {}
    for pair in (1, 0):
        P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 2 if pair else 0)
        sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode, Pm,
                           initial=ic, tau=1.0, tau_min=info["tau_min"], delta=info["delta"], tile=2,
                           recompute=True, gl_static=gl_static)
        res = []
        for T in meta["traj_times"]:
            rc = sim.solve(T)
            res.append((sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc, sim.interior()))
        runs[pair] = (res, sim.stats().pairs)
        sim.close()
    P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 1)
    assert runs[1][1] == 1 and runs[0][1] == 0
    for a, b in zip(runs[1][0], runs[0][0]):
        assert a[:5] == b[:5]
        assert np.array_equal(a[5], b[5])
    if mode in (0, 1):
        for i, a in enumerate(runs[1][0]):
            ref = meta[f"traj_m{mode}"][i]
            assert a[:5] == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
            assert np.array_equal(a[5], A[f"traj_m{mode}_state{i}"])


def test_pair_full_size_400():
    """BASELINE configs[1] (200 x 200 x 400, beads): 20 attempted steps with and without pairs, and
    the pair tile the bench runs (40 x 20 cells, 16 DMA-staged positions)"""
    got, used, *_ = _run((200, 200, 400), 0, True, 20, tile=1)
    ref, *_ = _run((200, 200, 400), 0, False, 20, tile=1)
    assert used == 1
    _same(got, ref)


def _loopback_pairs(meta, initial, nprocs, times, dims=None, steps=0, gl_static=False, mode=0):
    """nprocs slabs on one GPU (loopback transport, one host thread each), pair kernels forced"""
    L = P.lib()
    group = C.c_void_p()
    assert L.pft_comm_init_loopback(C.byref(group), nprocs) == 0
    out, errs = [None] * nprocs, []

    def worker(r):
        try:
            mine = C.c_void_p()
            assert L.pft_comm_loopback_rank(group, r, C.byref(mine)) == 0
            L.pft_comm_set_current(mine)
            L.pft_solver_set_option(P.PFT_OPT_PAIR, 2)         # per host thread
            Pm, info = O.params_from_meta(meta)
            n1, n2, n3 = dims or (info["n1"], info["n2"], info["n3"])
            sim = P.Simulation(n1, n2, n3, (info["L1"], info["L2"], info["L3"]), mode, Pm, nprocs=nprocs, rank=r,
                               initial=initial, beads=None if initial is not None else O.beads(), tau=1.0,
                               tau_min=info["tau_min"], delta=info["delta"], gl_static=gl_static, tile=2)
            res = []
            for T in times:
                rc = sim.solve_ex(T, steps, 0) if steps else sim.solve(T)
                res.append((sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc, sim.interior()))
            out[r] = (res, sim.stats().pairs)
            sim.close()
            L.pft_solver_set_option(P.PFT_OPT_PAIR, 1)
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


@pytest.mark.parametrize("nprocs", [2, 3, 4])
@pytest.mark.parametrize("gl_static", [False, True])
def test_pair_multislab_loopback_golden(nprocs, gl_static):
    """g20 (n3 = 20) on 2-4 slabs with the pair kernels: the reference's own trajectory bit for bit
    (stage A on each ghost plane from the neighbour's two boundary planes)"""
    meta, A = O.load_case("g20")
    times = meta["traj_times"][:2]
    out = _loopback_pairs(meta, A["traj_m0_ic"], nprocs, times, gl_static=gl_static)
    assert all(o[1] == 1 for o in out)
    for i in range(len(times)):
        ref = meta["traj_m0"][i]
        for o in out:
            assert o[0][i][:5] == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        assert np.array_equal(np.concatenate([o[0][i][5] for o in out], axis=1), A[f"traj_m0_state{i}"])


@pytest.mark.parametrize("nprocs,dims", [(3, (30, 30, 60)), (4, (66, 38, 21)), (2, (100, 36, 40)), (3, (80, 40, 30)),
                                          (4, (30, 30, 12)), (3, (18, 12, 8))])
def test_pair_multislab_loopback_equals_one_slab(nprocs, dims):
    """default IC on grids with partial tiles and uneven slabs (21 planes over 4: 6/5/5/5; slabs of
    2-3 planes, where the whole slab is launched before its two-plane exchange), 10 attempted
    steps, against the single-slab pair run"""
    ref, used, *_ = _run(dims, 0, True, 10)
    meta, _ = O.load_case("g20")
    out = _loopback_pairs(meta, None, nprocs, [1e9], dims=dims, steps=10)
    assert used == 1 and all(o[1] == 1 for o in out)
    for o in out:
        assert o[0][0][:4] == ref[:4]
    assert np.array_equal(np.concatenate([o[0][0][5] for o in out], axis=1), ref[4])


def test_pair_multislab_k1_carried_from_stage_launch_call():
    """a resident call with one launch per stage (PFT_OPT_PAIR 0: K1's first ghost plane
    only) followed by a REUSE_DEVICE call with the pair kernels between slabs, whose stage A reads
    K1's far ghost planes: the carried K1 must not be used there (R.k1_deep), so the two calls
    equal 10 continuous single-slab pair steps bit for bit"""
    dims, nprocs = (30, 30, 60), 3
    ref, used, *_ = _run(dims, 0, True, 10)
    meta, _ = O.load_case("g20")
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
            sim = P.Simulation(*dims, (info["L1"], info["L2"], info["L3"]), 0, Pm, nprocs=nprocs, rank=r,
                               beads=O.beads(), tau=1.0, tau_min=info["tau_min"], delta=info["delta"], tile=2)
            L.pft_solver_set_option(P.PFT_OPT_PAIR, 0)          # per host thread
            assert sim.solve_ex(1e9, 5, P.PFT_SOLVE_KEEP_DEVICE) == 2
            p0 = sim.stats().pairs
            L.pft_solver_set_option(P.PFT_OPT_PAIR, 2)
            assert sim.solve_ex(1e9, 5, P.PFT_SOLVE_REUSE_DEVICE) == 2
            out[r] = (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, sim.interior(),
                      p0, sim.stats().pairs)
            sim.close()
            L.pft_solver_set_option(P.PFT_OPT_PAIR, 1)
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
    assert used == 1 and all(o[5] == 0 and o[6] == 1 for o in out)
    for o in out:
        assert o[:4] == ref[:4]
    assert np.array_equal(np.concatenate([o[4] for o in out], axis=1), ref[4])


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
def test_pair_self_exchange(transport):
    """one slab, a 1-rank communicator exchanging with itself: the two-plane halo of every launch
    runs through the transport (RCCL send/recv on the comm stream; ipc put kernel + flags) and
    lands in planes a single slab never reads"""
    import os
    import uuid
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    if transport == "rccl":
        L = P.lib()
        uid = (C.c_char * 128)()
        assert L.pft_comm_get_unique_id(uid) == 0
        comm = C.c_void_p()
        assert L.pft_comm_init_rccl(C.byref(comm), 1, 0, uid, 0) == 0
        L.pft_comm_set_current(comm)
    else:
        comm = P.comm_init_ipc(1, 0, f"/pft_pselfx_{os.getpid()}_{uuid.uuid4().hex[:12]}")
    try:
        assert P.lib().pft_comm_set_self_exchange(comm, 1) == 0
        P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 2)
        sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                           initial=A["traj_m0_ic"], tau=1.0, tau_min=info["tau_min"], delta=info["delta"], tile=2)
        for i, T in enumerate(meta["traj_times"][:2]):
            rc = sim.solve(T)
            ref = meta["traj_m0"][i]
            assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
            assert np.array_equal(sim.interior(), A[f"traj_m0_state{i}"])
        assert sim.stats().pairs == 1
        sim.close()
    finally:
        P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 1)
        P.lib().pft_comm_set_current(None)
        P.comm_destroy(comm)
