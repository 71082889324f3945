"""The N > 1 path between separate processes: the ipc transport (pft_comm.h) with one process per
Z-slab, all on one GPU here (the same code maps a neighbour on another GPU over xGMI).  Each rank
is its own Python process started before it touches the GPU (tests/_ipc_worker.py); the slabs
exchange boundary planes through IPC-mapped device memory and flag words, the eps max and the
broadcasts through a shared-memory segment -- the reference's sync_solution (equation.c:290-326),
MPI_Allreduce of eps (RK_MPI_SAsolver_hybrid2.c:572) and command broadcasts (:328-336, :690).

Checked bit for bit (results do not depend on the decomposition):
  - golden g20 (the reference's own trajectory, 1171 attempted steps to t = 720 s) on 2, 3 and 4
    processes, default and fused-tile kernels;
  - BASELINE's 400^3 split over 2 and 4 processes against the single-slab run, 12 attempted steps;
  - the one-process ipc self exchange (the per-rank rehearsal of bench.py --self-exchange)."""
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

import _multi as M
import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


def _run_ranks(tmp_path, nranks, timeout=240, rank_env=None, ipc_timeout="120", **spec):
    spec = dict(spec, nranks=nranks, shm=f"/pft_test_{os.getpid()}_{uuid.uuid4().hex[:12]}",
                out=str(tmp_path / "rank"))
    path = tmp_path / "spec.json"
    path.write_text(json.dumps(spec))
    env = dict(os.environ, PFT_IPC_TIMEOUT=ipc_timeout)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_ipc_worker.py"), str(path), str(r)],
                              env=dict(env, **((rank_env or {}).get(r, {}))), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(nranks)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed ({p.returncode}):\n{outs[r][-3000:]}"
    return [dict(np.load(f"{spec['out']}.{r}.npz")) for r in range(nranks)]


@pytest.mark.parametrize("nranks,tile", [(2, None), (3, 32), (4, None), (4, 32), (2, 2)])
def test_g20_processes_equal_reference(tmp_path, nranks, tile):
    """tile 32 / 2: the fused kernels with fixed / fitted tiles (the default picks the cache
    kernel for the 10-cell-wide plane)"""
    meta, A = O.load_case("g20")
    times = meta["traj_times"]
    res = _run_ranks(tmp_path, nranks, case="g20", times=times, tile=tile)
    for r in res:
        assert int(r["path"]) == 1
    for i in range(len(times)):
        ref = meta["traj_m0"][i]
        for r in res:
            t, h, s, st, rc = r["rows"][i]
            assert (t.hex(), h.hex(), int(s), int(st), int(rc)) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        full = np.concatenate([r["states"][i] for r in res], axis=1)
        assert np.array_equal(full, A[f"traj_m0_state{i}"])


@pytest.mark.parametrize("nranks,tile,pair", [(2, 2, 2), (3, 2, 2), (4, 32, 2)])
def test_g20_processes_pair_kernels_equal_reference(tmp_path, nranks, tile, pair):
    """the pair kernels between processes (PFT_OPT_PAIR 2): stage A also on the ghost planes, from
    the two-plane halo exchanged after every launch (pft_comm_halo_deep)"""
    meta, A = O.load_case("g20")
    times = meta["traj_times"][:2]
    res = _run_ranks(tmp_path, nranks, case="g20", times=times, tile=tile, pair=pair)
    for r in res:
        assert int(r["path"]) == 1 and int(r["pairs"]) == 1
    for i in range(len(times)):
        ref = meta["traj_m0"][i]
        for r in res:
            t, h, s, st, rc = r["rows"][i]
            assert (t.hex(), h.hex(), int(s), int(st), int(rc)) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        full = np.concatenate([r["states"][i] for r in res], axis=1)
        assert np.array_equal(full, A[f"traj_m0_state{i}"])


@pytest.mark.parametrize("nranks", [2, 4])
def test_400_processes_equal_one_slab(tmp_path, nranks):
    steps = 12
    base, Pm, info = M.full_size_case(400, 0)
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                       beads=O.beads(), tau=1.0, tau_min=info["tau_min"], delta=info["delta"])
    assert sim.solve_ex(1e9, steps, 0) == 2
    got = (sim.t, sim.h, sim.system.steps, sim.system.steps_total)
    x = sim.interior()
    sim.close()
    assert got[2] < got[3]                                    # a rejected step in the window
    res = _run_ranks(tmp_path, nranks, case="default", grid_nodes=400, times=[1e9], steps=steps, pair=2)
    for r in res:
        assert int(r["pairs"]) == 1                           # the pair kernels between the slabs
        t, h, s, st, rc = r["rows"][0]
        assert (t, h, int(s), int(st), int(rc)) == got + (2,)
    assert [int(r["n3"]) for r in res] == [400 // nranks] * nranks
    assert np.array_equal(np.concatenate([r["states"][0] for r in res], axis=1), x)


@pytest.mark.parametrize("nranks,pair,staged_ranks", [(2, 0, (0, 1)), (3, 2, (0, 1, 2)), (3, 2, (1,))])
def test_g20_processes_staged_receive_equal_reference(tmp_path, nranks, pair, staged_ranks):
    """the staged receive a neighbour on another GPU gets (here forced between processes on one
    GPU, PFT_IPC_STAGED=1): planes into the receiver's uncached receive buffer, copied into its
    ghost (and far ghost) planes after the flag wait -- golden g20 bit for bit, one launch per
    stage and pair kernels (two-plane halo).  staged_ranks (1,): only the middle rank asks for it;
    its neighbours learn it at attach (IpcSlot.staged), so both ends of each link stage"""
    meta, A = O.load_case("g20")
    times = meta["traj_times"][:2]
    env = {r: {"PFT_IPC_STAGED": "1"} for r in staged_ranks}
    res = _run_ranks(tmp_path, nranks, rank_env=env, case="g20", times=times, tile=2, pair=pair)
    for r in res:
        assert int(r["path"]) == 1 and int(r["pairs"]) == (1 if pair else 0)
    for i in range(len(times)):
        ref = meta["traj_m0"][i]
        for r in res:
            t, h, s, st, rc = r["rows"][i]
            assert (t.hex(), h.hex(), int(s), int(st), int(rc)) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        full = np.concatenate([r["states"][i] for r in res], axis=1)
        assert np.array_equal(full, A[f"traj_m0_state{i}"])


def test_400_processes_staged_receive_equal_one_slab(tmp_path):
    """400^3 over 2 processes with the pair kernels and the staged receive (PFT_IPC_STAGED=1)"""
    steps = 8
    base, Pm, info = M.full_size_case(400, 0)
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                       beads=O.beads(), tau=1.0, tau_min=info["tau_min"], delta=info["delta"])
    assert sim.solve_ex(1e9, steps, 0) == 2
    got = (sim.t, sim.h, sim.system.steps, sim.system.steps_total)
    x = sim.interior()
    sim.close()
    env = {r: {"PFT_IPC_STAGED": "1"} for r in range(2)}
    res = _run_ranks(tmp_path, 2, rank_env=env, case="default", grid_nodes=400, times=[1e9], steps=steps, pair=2)
    for r in res:
        assert int(r["pairs"]) == 1
        t, h, s, st, rc = r["rows"][0]
        assert (t, h, int(s), int(st), int(rc)) == got + (2,)
    assert np.array_equal(np.concatenate([r["states"][0] for r in res], axis=1), x)


@pytest.mark.parametrize("staged", [0, 1])
@pytest.mark.parametrize("tile", [None, 32])
def test_ipc_self_exchange_equals_reference(tile, staged, monkeypatch):
    """one process, ipc communicator of size 1 exchanging with itself: the put kernel, the flag
    words and the stream waits of every stage run; the planes land in ghost planes one slab never
    reads, so the trajectory is the reference's"""
    if staged:
        monkeypatch.setenv("PFT_IPC_STAGED", "1")      # the receive-buffer path (read at set_peer)
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    comm = P.comm_init_ipc(1, 0, f"/pft_selfx_{os.getpid()}_{uuid.uuid4().hex[:12]}")
    try:
        assert P.lib().pft_comm_set_self_exchange(comm, 1) == 0
        assert P.lib().pft_comm_device_halo(comm) == 1
        sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                           initial=A["traj_m0_ic"], tau=1.0, tau_min=info["tau_min"], delta=info["delta"],
                           tile=tile)
        for i, T in enumerate(meta["traj_times"][:2]):
            rc = sim.solve(T)
            ref = meta["traj_m0"][i]
            assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
            assert np.array_equal(sim.interior(), A[f"traj_m0_state{i}"])
        sim.close()
    finally:
        P.comm_destroy(comm)


def test_lost_ipc_halo_ends_in_device_error_not_a_hang(tmp_path):
    """rank 1 never delivers its halo (fault injection PFT_IPC_DROP_PUTS=1: its puts and flag
    raises are skipped), so rank 0's compute stream blocks on a flag word that never comes.  Every
    host wait of the slab is bounded by PFT_IPC_TIMEOUT (here 5 s): both ranks return
    PFT_SOLVE_DEVICE_ERROR and exit, with the raw status an ipc timeout (-5000 host round,
    -5002 device halo) -- not a hang"""
    res = _run_ranks(tmp_path, 2, timeout=240, case="g20", times=[36.0], raw_rc=True, ipc_timeout="5",
                     second_call=True, rank_env={1: {"PFT_IPC_DROP_PUTS": "1"}})
    for r in res:
        assert int(r["rc"]) == P.PFT_SOLVE_DEVICE_ERROR
        assert int(r["status"]) in (-5000, -5002)
        assert float(r["seconds"]) < 60
    assert int(res[0]["status"]) == -5002            # rank 0 waited on the device flag
    # a second solve on the same comm and slab: the timed-out slab's flag words were
    # forced past every sequence number, so without the refusal its halo waits would all pass and
    # it would run on stale ghost planes; it must fail again, within the bound
    for r in res:
        assert int(r["rc2"]) == P.PFT_SOLVE_DEVICE_ERROR
        assert int(r["status2"]) in (-5000, -5002)
        assert float(r["seconds2"]) < 60


# ---- the exchange on the copy engines (PFT_IPC_CE=1: pft_slab_halo_put_ce) --------------------

# copy-engine options (pft_slab_set_boundary_stream): PFT_CE_BND 3, round 5's boundary pipeline (the
# pair kernels' boundary launch beside their interior launch, the halo waits on the boundary
# stream, so no pair interior launch waits for a neighbour); 2: the same with the waits on the
# compute stream; 0: every boundary launch before its interior; 1: every one beside; 4: the pair
# kernels' boundary chunks inline, leading their interior launch's grid (PFT_K_INLINE); 5 (the
# default since round 6): pair 2+3 as the whole slab in one launch, every tile column's first and
# last z-chunk leading (PFT_K_ENDS_FIRST), pair 4+5 as 4 (PFT_CE_BND45=5: ends-first too)
_SERIAL = {"PFT_CE_BND": "0"}
_INLINE = {"PFT_CE_BND": "4"}
_ENDS = {"PFT_CE_BND": "5"}
_PIPE = {"PFT_CE_BND": "2"}
_BESIDE_ALL = {"PFT_CE_BND": "1"}


@pytest.mark.parametrize("nranks,pair,staged,ce_ranks,xenv", [(2, 2, 0, (0, 1), {}), (3, 2, 0, (0, 1, 2), {}),
                                                              (3, 2, 1, (0, 1, 2), {}), (2, 0, 0, (0, 1), {}),
                                                              (3, 0, 1, (0, 1, 2), {}), (3, 2, 0, (1,), {}),
                                                              (3, 2, 1, (0, 1, 2), {"PFT_CE_SEQTAB": "5"}),
                                                              (2, 2, 0, (0, 1), _SERIAL), (3, 2, 1, (0, 1, 2), _SERIAL),
                                                              (3, 0, 0, (0, 1, 2), _BESIDE_ALL),
                                                              (3, 2, 1, (0, 2), _BESIDE_ALL),
                                                              (3, 2, 0, (0, 1, 2), _PIPE), (3, 2, 1, (0, 1, 2), _PIPE),
                                                              (3, 0, 1, (0, 1, 2), _PIPE), (3, 2, 1, (1,), _PIPE),
                                                              (2, 2, 0, (0, 1), dict(_PIPE, PFT_CE_SEQTAB="3")),
                                                              (3, 2, 1, (0, 1, 2), {"PFT_CE_FENCE": "0"}),
                                                              (2, 2, 0, (0, 1), {"PFT_CE_FENCE": "0"}),
                                                              (3, 2, 0, (0, 2), {"PFT_CE_SEQTAB": "3"}),
                                                              (2, 2, 0, (0, 1), _INLINE), (3, 2, 1, (0, 1, 2), _INLINE),
                                                              (3, 2, 0, (1,), _INLINE), (3, 2, 1, (0, 2), _INLINE),
                                                              (2, 2, 1, (0, 1), dict(_INLINE, PFT_CE_SEQTAB="3")),
                                                              (2, 2, 0, (0, 1), _ENDS), (3, 2, 1, (0, 1, 2), _ENDS),
                                                              (3, 2, 0, (1,), _ENDS), (3, 2, 1, (0, 2), _ENDS),
                                                              (3, 0, 0, (0, 1, 2), _ENDS),
                                                              (2, 2, 1, (0, 1), dict(_ENDS, PFT_CE_SEQTAB="3")),
                                                              (3, 2, 1, (0, 1, 2), dict(_ENDS, PFT_CE_BND45="5")),
                                                              (3, 2, 0, (0, 1, 2), dict(_ENDS, PFT_CE_STAGE_INLINE="1")),
                                                              (2, 0, 1, (0, 1), dict(_INLINE, PFT_CE_STAGE_INLINE="1")),
                                                              (3, 2, 1, (0, 1, 2), {"PFT_CE_BND": "3"})])
def test_g20_processes_copy_engine_equal_reference(tmp_path, nranks, pair, staged, ce_ranks, xenv):
    """the boundary planes first, their exchange as SDMA copies and 8-byte flag copies on the comm
    stream beside the interior launch, the receiver's flag wait before the next launch: golden g20
    bit for bit with the pair kernels (two-plane halo) and one launch per stage, direct and staged.
    ce_ranks (1,): only the middle rank puts on the copy engines, its neighbours with the put
    kernel -- the receiving side is the same for both.  PFT_CE_SEQTAB 5: the flags' table of
    sequence numbers refilled every 5 exchanges, hundreds of times over the run (each refill
    waits for the copy that last read its pinned half).  _SERIAL, _BESIDE_ALL: the boundary
    launches' placement.  PFT_CE_FENCE: each side's flag on the other copy stream behind an event
    after that side's planes (1, the default), or right behind them on the same stream (0)"""
    meta, A = O.load_case("g20")
    times = meta["traj_times"][:2]
    env = {r: dict({"PFT_IPC_CE": "1"} if r in ce_ranks else {}, **({"PFT_IPC_STAGED": "1"} if staged else {}),
                   **(xenv if r in ce_ranks else {}))
           for r in range(nranks)}
    res = _run_ranks(tmp_path, nranks, rank_env=env, case="g20", times=times, tile=2, pair=pair)
    for r in res:
        assert int(r["path"]) == 1 and int(r["pairs"]) == (1 if pair else 0)
    for i in range(len(times)):
        ref = meta["traj_m0"][i]
        for r in res:
            t, h, s, st, rc = r["rows"][i]
            assert (t.hex(), h.hex(), int(s), int(st), int(rc)) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        full = np.concatenate([r["states"][i] for r in res], axis=1)
        assert np.array_equal(full, A[f"traj_m0_state{i}"])


@pytest.mark.parametrize("staged,xenv", [(0, {}), (1, {}), (0, _SERIAL), (1, _SERIAL), (0, _PIPE), (1, _PIPE),
                                         (0, _INLINE), (1, _INLINE), (0, _ENDS), (1, _ENDS)])
def test_400_processes_copy_engine_equal_one_slab(tmp_path, staged, xenv):
    """400^3 over 2 processes with the pair kernels, the exchange on the copy engines"""
    steps = 10
    base, Pm, info = M.full_size_case(400, 0)
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                       beads=O.beads(), tau=1.0, tau_min=info["tau_min"], delta=info["delta"])
    assert sim.solve_ex(1e9, steps, 0) == 2
    got = (sim.t, sim.h, sim.system.steps, sim.system.steps_total)
    x = sim.interior()
    sim.close()
    env = {r: dict({"PFT_IPC_CE": "1"}, **({"PFT_IPC_STAGED": "1"} if staged else {}), **xenv) for r in range(2)}
    res = _run_ranks(tmp_path, 2, rank_env=env, case="default", grid_nodes=400, times=[1e9], steps=steps, pair=2)
    for r in res:
        assert int(r["pairs"]) == 1
        t, h, s, st, rc = r["rows"][0]
        assert (t, h, int(s), int(st), int(rc)) == got + (2,)
    assert np.array_equal(np.concatenate([r["states"][0] for r in res], axis=1), x)


@pytest.mark.parametrize("xenv", [{}, _SERIAL, _BESIDE_ALL, _PIPE, _INLINE, _ENDS])
@pytest.mark.parametrize("staged", [0, 1])
@pytest.mark.parametrize("pair", [2, 0])
def test_ipc_copy_engine_self_exchange_equals_reference(pair, staged, xenv, monkeypatch):
    """one process exchanging with itself on the copy engines (bench.py --self-exchange
    --transport ipc-ce): every exchange's SDMA copies, flag copies and waits run"""
    monkeypatch.setenv("PFT_IPC_CE", "1")
    for k, v in xenv.items():
        monkeypatch.setenv(k, v)
    if staged:
        monkeypatch.setenv("PFT_IPC_STAGED", "1")
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    comm = P.comm_init_ipc(1, 0, f"/pft_ceselfx_{os.getpid()}_{uuid.uuid4().hex[:12]}")
    P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, pair)
    try:
        assert P.lib().pft_comm_set_self_exchange(comm, 1) == 0
        assert P.lib().pft_comm_copy_engine(comm) == 1 and P.lib().pft_comm_boundary_first(comm) == 1
        sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                           initial=A["traj_m0_ic"], tau=1.0, tau_min=info["tau_min"], delta=info["delta"], tile=2)
        for i, T in enumerate(meta["traj_times"][:2]):
            rc = sim.solve(T)
            ref = meta["traj_m0"][i]
            assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
                (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
            assert np.array_equal(sim.interior(), A[f"traj_m0_state{i}"])
        assert sim.stats().pairs == (1 if pair else 0)
        sim.close()
    finally:
        P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, 1)
        P.comm_destroy(comm)


def test_lost_copy_engine_halo_ends_in_device_error(tmp_path):
    """as test_lost_ipc_halo_ends_in_device_error_not_a_hang, with the copy-engine put"""
    env = {0: {"PFT_IPC_CE": "1"}, 1: {"PFT_IPC_CE": "1", "PFT_IPC_DROP_PUTS": "1"}}
    res = _run_ranks(tmp_path, 2, timeout=240, case="g20", times=[36.0], raw_rc=True, ipc_timeout="5",
                     second_call=True, rank_env=env)
    for r in res:
        assert int(r["rc"]) == P.PFT_SOLVE_DEVICE_ERROR
        assert int(r["status"]) in (-5000, -5002)
        assert float(r["seconds"]) < 60
        assert int(r["rc2"]) == P.PFT_SOLVE_DEVICE_ERROR


def test_failed_attach_fails_every_rank_at_once(tmp_path):
    """rank 1 cannot map its neighbour's buffers (fault injection PFT_IPC_FAIL_ATTACH=1): the attach
    agrees its outcome across ranks, so both ranks' RK_MPI_SA_init (which attaches the slab) fails at
    once -- rank 0 is not left in the attach's second round until PFT_IPC_TIMEOUT (here 120 s)"""
    import time
    spec = dict(nranks=2, shm=f"/pft_test_{os.getpid()}_{uuid.uuid4().hex[:12]}", out=str(tmp_path / "rank"),
                case="g20", times=[36.0], raw_rc=True)
    path = tmp_path / "spec.json"
    path.write_text(json.dumps(spec))
    env = dict(os.environ, PFT_IPC_TIMEOUT="120")
    rank_env = {1: {"PFT_IPC_FAIL_ATTACH": "1"}, 0: {"PFT_IPC_CE": "1"}}
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_ipc_worker.py"), str(path), str(r)],
                              env=dict(env, **rank_env[r]), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(2)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    el = time.time() - t0
    for r, p in enumerate(procs):
        assert p.returncode != 0 and "RK_MPI_SA_init failed" in outs[r], outs[r][-2000:]
    assert el < 90, el          # the import of torch-free workers plus the failed attach, not the 120 s bound


@pytest.mark.gpu
def test_device_phys_id_names_the_gpu():
    """pft_hip_device_phys_id: the PCI location, stable, distinct per visible GPU -- the ipc
    transport compares it (not the device index) to decide whether a neighbour shares the GPU"""
    import ctypes as C
    import torch
    L = P.lib()
    ids = []
    for d in range(torch.cuda.device_count()):
        a, b = C.c_int(-1), C.c_int(-2)
        assert L.pft_hip_device_phys_id(d, C.byref(a)) == 0 and L.pft_hip_device_phys_id(d, C.byref(b)) == 0
        assert a.value == b.value and a.value >= 0
        ids.append(a.value)
    assert len(set(ids)) == len(ids)


@pytest.mark.gpu
def test_device_ident_names_the_gpu():
    """pft_hip_device_ident: PCI bus id with the function, then the UUID; stable, distinct per
    visible GPU.  The ipc attach counts a neighbour as on this GPU only when the identities are
    equal (partitions of one package differ in the function or the UUID)."""
    import ctypes as C
    import re
    import torch
    L = P.lib()
    ids = []
    for d in range(torch.cuda.device_count()):
        a, b = C.create_string_buffer(80), C.create_string_buffer(80)
        assert L.pft_hip_device_ident(d, a, 80) == 0 and L.pft_hip_device_ident(d, b, 80) == 0
        assert a.value == b.value
        assert re.fullmatch(rb"[0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-9a-fA-F]/[0-9a-f]{32}", a.value), a.value
        ids.append(a.value)
    assert len(set(ids)) == len(ids)
    assert L.pft_hip_device_ident(0, C.create_string_buffer(16), 16) == -2     # too small a buffer
