"""Bounded waits on RCCL-fed work (pft_comm.hip rccl_watch / rccl_abort, pft_slab_set_watch).

A peer that dies or diverges leaves the compute stream waiting on an exchange that never ends.  The
reference has MPI's error negotiation for this (intertrack.c:534-629, CheckErrorAcrossRanks); libpft
bounds every host wait on an RCCL-fed stream by PFT_COMM_TIMEOUT, watches ncclCommGetAsyncError,
aborts the communicator (ncclCommAbort) and returns PFT_SOLVE_DEVICE_ERROR; later solves on it refuse.
On one GPU the lost peer is the test hook PFT_COMM_STALL=n: the n-th exchange's comm stream waits on
a word only the abort releases (a 1-rank RCCL communicator exchanging with itself)."""
import ctypes as C
import os
import time

import pytest

import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu

PFT_ERR_COMM_ABORTED = -5003


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


@pytest.mark.parametrize("pair", [2, 0])
def test_rccl_stalled_exchange_returns_device_error(pair, monkeypatch):
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    L = P.lib()
    monkeypatch.setenv("PFT_COMM_TIMEOUT", "2")
    monkeypatch.setenv("PFT_COMM_STALL", "4")
    uid = (C.c_char * 128)()
    assert L.pft_comm_get_unique_id(uid) == 0
    comm = C.c_void_p()
    assert L.pft_comm_init_rccl(C.byref(comm), 1, 0, uid, 0) == 0
    monkeypatch.delenv("PFT_COMM_STALL")
    L.pft_comm_set_current(comm)
    try:
        assert L.pft_comm_set_self_exchange(comm, 1) == 0
        L.pft_solver_set_option(P.PFT_OPT_PAIR, pair)
        sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                           initial=A["traj_m0_ic"], tau=1.0, tau_min=info["tau_min"], delta=info["delta"], tile=2)
        t0 = time.time()
        rc = L.RK_MPI_SA_solve(meta["traj_times"][0], C.byref(sim.system))
        el = time.time() - t0
        assert rc == P.PFT_SOLVE_DEVICE_ERROR, rc
        assert L.pft_solver_last_status() == PFT_ERR_COMM_ABORTED
        assert el < 2 + 20, el             # the bound, plus the abort itself
        # the communicator is gone: the next solve refuses at once instead of waiting again
        t0 = time.time()
        rc = L.RK_MPI_SA_solve(meta["traj_times"][0], C.byref(sim.system))
        assert rc == P.PFT_SOLVE_DEVICE_ERROR, rc
        assert L.pft_solver_last_status() == PFT_ERR_COMM_ABORTED
        assert time.time() - t0 < 2
        sim.close()
    finally:
        L.pft_solver_set_option(P.PFT_OPT_PAIR, 1)
        L.pft_comm_set_current(None)
        P.comm_destroy(comm)
