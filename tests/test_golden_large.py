"""BASELINE configs[1] and [2] pinned to the reference itself (tests/golden/g200, g400: the
reference compiled in place by oracle/Makefile, run with MPICH on 8 ranks and re-checked on 3 / 5
ranks, tests/golden/gen_golden.py).  CPU side:

- the benchmark's parameters at grid_nodes 200 and 400 (porousfreezethaw_amd/params.py) equal the
  reference's parameter dump bit for bit;
- libpft's host initial condition (the default icond formulas + the 200 glass beads,
  intertrack_model.c) has the reference's SHA-256 at both sizes;
- the CPU oracle (oracle/pft_oracle.c) reaches the reference's g200 state after 35 attempted steps.

The GPU side (RK_MPI_SA_solve on the MI355X to the same times) is
tests/test_baseline_configs.py::test_full_size_reference_trajectory_bitwise."""
import hashlib

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P
from porousfreezethaw_amd import params as PR


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


CASES = [("g200", 200, 0), ("g200", 200, 1), ("g400", 400, 0)]


@pytest.mark.parametrize("case,gn,mode", CASES)
def test_bench_params_equal_reference(case, gn, mode):
    meta, _ = O.load_case(case)
    ref = {k: (float.fromhex(v) if isinstance(v, str) else v) for k, v in meta[f"m{mode}_params"].items()}
    mine = PR.default_params(grid_nodes=gn, calc_mode=mode)
    for k in P.PARAM_NAMES + ["L1", "L2", "L3", "tau", "tau_min", "delta", "final_time", "n1", "n2", "n3",
                              "calc_mode"]:
        assert mine[k] == ref[k], (k, mine[k], ref[k])


@pytest.mark.parametrize("case,gn,mode", CASES)
def test_host_ic_equals_reference(case, gn, mode):
    meta, _ = O.load_case(case)
    Pm, info = O.params_from_meta({"params": meta[f"m{mode}_params"]})
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode, Pm,
                       beads=O.beads(), tau=1.0, tau_min=info["tau_min"], delta=info["delta"], init_solver=False)
    try:
        assert _sha(sim.interior()) == meta[f"m{mode}_ic_sha256"]
    finally:
        sim.close()


def test_oracle_reaches_reference_g200():
    """the CPU restatement at full configs[1] size: 35 attempted steps to t = 0.01 s, bit for bit"""
    meta, A = O.load_case("g200")
    Pm, info = O.params_from_meta({"params": meta["m0_params"]})
    ic = O.ic_default(info, Pm, O.beads())
    assert _sha(ic) == meta["m0_ic_sha256"]
    T = meta["traj_m0_times"][0]
    t, h, s, st, rc, x = O.solve(info, Pm, 0, ic, 0.0, 1.0, [T])[0]
    ref = meta["traj_m0"][0]
    assert (t.hex(), h.hex(), s, st, rc) == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(),
                                             ref[2], ref[3], ref[4])
    assert np.array_equal(x[:, x.shape[1] // 2], A["traj_m0_state0_mid"])
    assert np.array_equal(x[:, -1], A["traj_m0_state0_top"])
    assert _sha(x) == meta["traj_m0_sha256"][0]
