"""Per-launch time of the pair kernels alone at 400^3 (default Params, device IC), independent of the
results (for timing ablations whose arithmetic is wrong on purpose): N back-to-back launches of
pft_slab_pair(first = 2, then 4) on the solver's slab after one warm-up solve, timed with a device
sync around them.  Library: PFT_LIB.  Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402

import porousfreezethaw_amd as P  # noqa: E402
from porousfreezethaw_amd import params as PR  # noqa: E402

N = int(os.environ.get("N", "200"))
base = PR.default_params(grid_nodes=400)
beads = np.load(os.path.join(P.REPO, "tests", "golden", "beads.npy"))
L = P.lib()
sim = P.Simulation(base["n1"], base["n2"], base["n3"], (base["L1"], base["L2"], base["L3"]), 0,
                   P.params_array(base), beads=beads, tau=base["tau"], tau_min=base["tau_min"],
                   delta=base["delta"], device_ic=True)
sim.solve_ex(base["final_time"], 3, P.PFT_SOLVE_KEEP_DEVICE | P.PFT_SOLVE_REUSE_DEVICE)
L.pft_solver_slab.restype = C.c_void_p
slab = C.c_void_p(L.pft_solver_slab())
L.pft_slab_pair.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double]
h = 1e-4
out = {}
for first in (2, 4):
    for _ in range(10):
        L.pft_slab_pair(slab, first, 0.0, h / 3, h, h / 3)
    L.pft_hip_device_sync()
    t0 = time.perf_counter()
    for _ in range(N):
        assert L.pft_slab_pair(slab, first, 0.0, h / 3, h, h / 3) == 0
    L.pft_hip_device_sync()
    out[f"pair{first}{first + 1}_ms"] = round((time.perf_counter() - t0) / N * 1e3, 4)
sim.close()
print(json.dumps(dict(out, lib=os.environ.get("PFT_LIB", "lib"), launches=N)))
