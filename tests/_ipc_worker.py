"""One rank of a multi-process run over the ipc transport (tests/test_ipc_multiprocess.py,
bench-like rehearsals).  Started as its own process -- never forked from a process that uses the
GPU -- with:

    python tests/_ipc_worker.py <spec.json> <rank>

spec: {"nranks", "shm", "case": "g20" | "default", "grid_nodes", "mode", "times": [...],
       "steps": max attempted steps per call (0 = none), "out": output prefix, "tile", "self_x",
       "pair": PFT_OPT_PAIR (default 1: automatic)}
Writes <out>.<rank>.npz: per call (t, h, steps, steps_total, rc) and this slab's interior."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import _oracle as O  # noqa: E402
import porousfreezethaw_amd as P  # noqa: E402


def main():
    spec = json.load(open(sys.argv[1]))
    rank = int(sys.argv[2])
    n = spec["nranks"]
    comm = P.comm_init_ipc(n, rank, spec["shm"], spec.get("device", 0))
    if spec.get("self_x"):
        assert P.lib().pft_comm_set_self_exchange(comm, 1) == 0
    P.lib().pft_solver_set_option(P.PFT_OPT_PAIR, spec.get("pair", 1))
    if spec["case"] == "g20":
        meta, A = O.load_case("g20")
        Pm, info = O.params_from_meta(meta)
        ic, beads = A["traj_m0_ic"], None
    else:
        import _multi as M
        base, Pm, info = M.full_size_case(spec["grid_nodes"], spec.get("mode", 0))
        ic, beads = None, O.beads()
        if spec.get("ic"):
            ic, beads = np.load(spec["ic"]), None
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]),
                       spec.get("mode", 0), Pm, nprocs=n, rank=rank, initial=ic, beads=beads, tau=1.0,
                       tau_min=info["tau_min"], delta=info["delta"], tile=spec.get("tile"))
    rows, states = [], []
    if spec.get("raw_rc"):
        # fault-injection runs: one pft_solve_ex call, its raw return code and timing recorded
        import ctypes as C
        import time
        t0 = time.time()
        rc = P.lib().pft_solve_ex(spec["times"][0], C.byref(sim.system), spec.get("steps", 0), 0)
        el = time.time() - t0
        status = P.lib().pft_solver_last_status()
        extra = {}
        if spec.get("second_call"):
            # the same solver and comm again after the failure: it must fail again (a slab whose
            # halo wait timed out refuses every later exchange), not run on released flag words
            t0 = time.time()
            extra["rc2"] = P.lib().pft_solve_ex(spec["times"][0], C.byref(sim.system), spec.get("steps", 0), 0)
            extra["seconds2"] = time.time() - t0
            extra["status2"] = P.lib().pft_solver_last_status()
        sim.close()
        P.comm_destroy(comm)
        np.savez(f"{spec['out']}.{rank}.npz", rc=rc, status=status, seconds=el, **extra)
        return
    for T in spec["times"]:
        if spec.get("steps"):
            rc = sim.solve_ex(T, spec["steps"], 0)
        else:
            rc = sim.solve(T)
        rows.append([sim.t, sim.h, sim.system.steps, sim.system.steps_total, rc])
        states.append(sim.interior())
    st = sim.stats()
    assert P.lib().pft_comm_device_halo(comm) == 1
    sim.close()
    P.comm_destroy(comm)
    np.savez(f"{spec['out']}.{rank}.npz", rows=np.array(rows), states=np.array(states),
             path=st.path, launches=st.kernel_launches, first_row=sim.grid.first_row, n3=sim.grid.n3,
             pairs=st.pairs)


if __name__ == "__main__":
    main()
