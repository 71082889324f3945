"""BASELINE configs[0] at the reference's own size: default Params at grid_nodes 100 (50x50x100
cells), pinned by tests/golden/g100.json, which the reference compiled in place produced
(tests/golden/gen_golden.py, case g100).  The states are kept as SHA-256 digests of their
little-endian float64 bytes plus two sampled planes (a full state is 6 MB).

- CPU: the bench's parameters and libpft's default initial condition (the bench's synthetic
  input) equal the reference's; the oracle's trajectory equals the reference's.
- GPU: RK_MPI_SA_solve on the MI355X reaches the reference's t, h, step counts and field bits at
  every snapshot time (225 attempted steps), on the default fused path with the tile geometry it
  fits to n1 = 50.
"""
import hashlib

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P
from porousfreezethaw_amd import params as PR


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def g100():
    return O.load_case("g100")


def _sim(meta, **kw):
    Pm, info = O.params_from_meta(meta)
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]),
                       info["calc_mode"], Pm, beads=O.beads(), tau=1.0, tau_min=info["tau_min"],
                       delta=info["delta"], **kw)
    return sim, Pm, info


def _check_state(x, meta, A, i):
    n3 = x.shape[1]
    # the sampled planes first: a mismatch there says where, the digest says whether
    assert np.array_equal(x[:, n3 // 2], A[f"traj_m0_state{i}_mid"])
    assert np.array_equal(x[:, -1], A[f"traj_m0_state{i}_top"])
    assert _sha(x) == meta["traj_m0_sha256"][i]


def test_g100_bench_params_bitwise(g100):
    meta, _ = g100
    ref = {k: (float.fromhex(v) if isinstance(v, str) else v) for k, v in meta["params"].items()}
    mine = PR.default_params(grid_nodes=100)
    assert (mine["n1"], mine["n2"], mine["n3"]) == (50, 50, 100)
    for k in P.PARAM_NAMES + ["L1", "L2", "L3", "tau", "tau_min", "delta", "final_time", "n1", "n2", "n3",
                              "calc_mode"]:
        assert mine[k] == ref[k], (k, mine[k], ref[k])


def test_g100_default_ic_bitwise(g100):
    meta, _ = g100
    sim, _, _ = _sim(meta, init_solver=False)
    assert _sha(sim.interior()) == meta["ic_sha256"]
    sim.close()


def test_g100_oracle_trajectory(g100):
    meta, A = g100
    Pm, info = O.params_from_meta(meta)
    ic = O.ic_default(info, Pm, O.beads())
    assert _sha(ic) == meta["ic_sha256"]
    res = O.solve(info, Pm, 0, ic, 0.0, 1.0, meta["traj_times"])
    for i, (t, h, s, st, rc, x) in enumerate(res):
        ref = meta["traj_m0"][i]
        assert (t.hex(), h.hex(), s, st, rc) == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(),
                                                 ref[2], ref[3], ref[4])
        _check_state(x, meta, A, i)


@pytest.mark.gpu
def test_g100_device_trajectory(g100):
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")
    meta, A = g100
    sim, _, _ = _sim(meta)
    assert _sha(sim.interior()) == meta["ic_sha256"]
    for i, T in enumerate(meta["traj_times"]):
        rc = sim.solve(T)
        ref = meta["traj_m0"][i]
        assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
            (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        _check_state(sim.interior(), meta, A, i)
    assert sim.stats().path == 1
    geo = sim.tile_geometry()
    assert geo[5][0] == 2              # the fused kernel (tiles fitted to the 50 x 50 plane)
    sim.close()
