#!/usr/bin/env python3
"""Calibrate bench.py's cpu_baseline (the oracle port, oracle/pft_oracle.c) against the reference
itself, on the same cores and the same 400^3 state.  Test/measurement infrastructure: runs only in
the build container, where /root/reference and MPICH exist.

  reference: oracle/_ref/pft_ref (RK_MPI_SAsolver_hybrid2.c + equation.c compiled in place with
             the reference's flags, -O1 -std=c99 -fopenmp) under `mpirun -np P`, 1 OpenMP thread
             per rank (P ranks x 1 thread beat 4 x 2 in SURVEY section 6); the harness reports the
             wall time of the RK_MPI_SA_solve call itself (solvex, wall0.txt)
  port:      oracle/lib/libpft_oracle.so, P OpenMP threads, the same number of attempted steps
             from the same state
Output: profiles/r02_cpu_calibration.json with both rates and their ratio (reference / port):
bench.py multiplies the box's port figure by that ratio to state the reference-equivalent rate.

    python scripts/calibrate_cpu.py [P] [grid_nodes] [T]
"""
import ctypes as C
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import gen_golden as G  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    gn = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    T = float(sys.argv[3]) if len(sys.argv) > 3 else 0.05
    w = G.Work({"grid_nodes": gn})
    try:
        t0 = time.time()
        out = w.run(P, "setup", timeout=3600)
        p = G.read_params(out)
        shape = (3, p["n3"], p["n2"], p["n1"])
        ic = G.load(os.path.join(out, "ic.f64"), shape)
        icp = os.path.join(w.dir, "ic0.f64")
        ic.tofile(icp)
        print(f"setup {time.time() - t0:.1f} s", flush=True)
        o = w.run(P, "solvex", icp, 0.0, 1.0, 0, -1, T, timeout=3600)
        row = open(os.path.join(o, "traj.txt")).read().split()
        steps_ref = int(row[3])
        wall_ref = float(open(os.path.join(o, "wall0.txt")).read())
        cells = p["n1"] * p["n2"] * p["n3"]
        ref_rate = cells * steps_ref / wall_ref / 1e6
        print(f"reference {P}x1: {steps_ref} attempted steps in {wall_ref:.2f} s = {ref_rate:.2f} Mcells*steps/s",
              flush=True)

        os.environ["OMP_NUM_THREADS"] = str(P)
        import _oracle as O
        import numpy as np
        Pm = np.array([p[k] for k in O.PARAM_NAMES], dtype=np.float64)
        info = {k: p[k] for k in ("n1", "n2", "n3", "L1", "L2", "L3", "tau_min", "delta")}
        g = O.make_grid(info)
        x = O.pad(g, ic)
        t, h = C.c_double(0.0), C.c_double(1.0)
        s, st = C.c_long(0), C.c_long(0)
        w0 = time.perf_counter()
        O.lib().pft_or_solve(C.byref(g), O.ptr(Pm), 0, T, C.byref(t), C.byref(h), info["tau_min"], info["delta"], 0,
                             O.ptr(x), C.byref(s), C.byref(st), 0, O.EXCHANGE_FN(), O.ALLREDUCE_FN(), None)
        wall_port = time.perf_counter() - w0
        assert st.value == steps_ref, (st.value, steps_ref)
        assert np.array_equal(O.unpad(g, x), G.load(os.path.join(o, "state0.f64"), shape)), "port != reference"
        port_rate = cells * st.value / wall_port / 1e6
        print(f"port {P} threads: {wall_port:.2f} s = {port_rate:.2f} Mcells*steps/s", flush=True)
        res = {"cores": P, "grid": f"{p['n1']}x{p['n2']}x{p['n3']}", "attempted_steps": steps_ref,
               "reference": {"layout": f"{P} MPI ranks x 1 OpenMP thread, -O1 (reference flags)",
                             "wall_s": round(wall_ref, 3), "Mcells_steps_per_s": round(ref_rate, 3)},
               "port": {"layout": f"{P} OpenMP threads, gcc -O2 -ffp-contract=off",
                        "wall_s": round(wall_port, 3), "Mcells_steps_per_s": round(port_rate, 3)},
               "reference_over_port": round(ref_rate / port_rate, 4),
               "bitwise_equal": True,
               "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" :\t")}
        dst = os.path.join(REPO, "profiles", "r02_cpu_calibration.json")
        with open(dst, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
    finally:
        w.close()


if __name__ == "__main__":
    main()
