"""Multi-slab helpers for the GPU tests: the same Z-slab decomposition (intertrack.c:1776-1800)
run by several slabs of libpft, either as host threads of this process (loopback transport) or as
separate processes (ipc transport, tests/_ipc_worker.py)."""
import ctypes as C
import threading

import porousfreezethaw_amd as P
from porousfreezethaw_amd import params as PR


def full_size_case(grid_nodes, calc_mode=0):
    """default Params at grid_nodes G: (params dict, param[] array, geometry info)"""
    base = PR.default_params(grid_nodes=grid_nodes, calc_mode=calc_mode)
    info = {k: base[k] for k in ("n1", "n2", "n3", "L1", "L2", "L3", "tau_min", "delta")}
    return base, P.params_array(base), info


def loopback_run(nprocs, make_sim, run, timeout=900):
    """nprocs slabs on host threads sharing one GPU (pft_comm_init_loopback).  make_sim(rank)
    builds rank r's Simulation (nprocs, rank set), run(sim) solves and returns what to collect;
    returns the per-rank results in rank order."""
    L = P.lib()
    group = C.c_void_p()
    assert L.pft_comm_init_loopback(C.byref(group), nprocs) == 0
    out, errs = [None] * nprocs, []

    def worker(r):
        mine = C.c_void_p()
        try:
            assert L.pft_comm_loopback_rank(group, r, C.byref(mine)) == 0
            L.pft_comm_set_current(mine)
            sim = make_sim(r)
            try:
                out[r] = run(sim)
            finally:
                sim.close()
        except BaseException as e:  # noqa: BLE001 -- surfaced below
            errs.append(e)
        finally:
            L.pft_comm_set_current(None)
            if mine:
                L.pft_comm_destroy(mine)

    ths = [threading.Thread(target=worker, args=(r,)) for r in range(nprocs)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=timeout)
    L.pft_comm_destroy(group)
    if errs:
        raise errs[0]
    return out
