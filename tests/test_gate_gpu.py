"""f4, gated steps (PFT_OPT_GATE, rk_solver.c run_fused, pft_slab_gate_*; off by default): on a
small single slab the launches of the next attempted step are enqueued before this step's error
norm is known and run on the device's own step decision (the speculative stage 1 reduces the error
norm and decides as hybrid2.c:578-611, with a correctly rounded x^0.2); the host takes its own
decision with glibc's pow and keeps the gated step only if both agree bit for bit.  Every test
compares against the reference itself (tests/golden/g100.json, BASELINE configs[0], produced by
the reference compiled in place) or against the same solve with gating off: t, h, step counts and
the fields bit for bit.

Paths covered: accepted steps (kept), rejected steps (the gated launches exit at once; the next
attempt ungated), the last step to final_time (NEXTFINISH / FINISHED: no gated step after it),
step caps of pft_solve_ex at every phase of the pipeline, calls that continue a resident state,
and RK_MPI_SA_solve's host boundary after a discarded gated step.
"""
import hashlib
import os

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def g100():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")
    return O.load_case("g100")


@pytest.fixture(autouse=True)
def _gate_on():
    P.lib().pft_solver_set_option(P.PFT_OPT_GATE, 1)      # off by default
    yield
    P.lib().pft_solver_set_option(P.PFT_OPT_GATE, 0)


def _sim(meta):
    Pm, info = O.params_from_meta(meta)
    return P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]),
                        info["calc_mode"], Pm, beads=O.beads(), tau=1.0, tau_min=info["tau_min"],
                        delta=info["delta"])


def _rec(sim):
    return (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total)


def test_gated_g100_reference_trajectory(g100):
    """the reference's own g100 trajectory (225 attempted steps, rejections among them, both
    snapshot times reached exactly) with the gated pipeline on, and most steps gated"""
    meta, A = g100
    sim = _sim(meta)
    gated = 0
    for i, T in enumerate(meta["traj_times"]):
        rc = sim.solve(T)
        ref = meta["traj_m0"][i]
        assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
            (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        x = sim.interior()
        n3 = x.shape[1]
        assert np.array_equal(x[:, n3 // 2], A[f"traj_m0_state{i}_mid"])
        assert _sha(x) == meta["traj_m0_sha256"][i]
        st = sim.stats()
        assert st.path == 1 and not st.pairs
        gated += st.gated_steps
        # the device's x^0.2 is correctly rounded: it differs from glibc's only where glibc
        # misrounds (~0.06% of random arguments), and each difference costs one discarded step
        assert st.gate_misses <= max(2, st.gated_steps // 50), (st.gate_misses, st.gated_steps)
    accepted = meta["traj_m0"][-1][2]
    assert gated >= accepted // 2, (gated, accepted)
    sim.close()


def test_gated_equals_ungated_with_step_caps(g100):
    """capped calls of every length 1..9 (the cap lands on every phase of the pipeline: an armed
    decision pending, a pre-enqueued step in flight) continuing a resident state, gated vs ungated"""
    meta, _ = g100
    caps = [1, 2, 3, 4, 5, 6, 7, 8, 9, 3, 1, 40]
    out = {}
    for gate in (0, 1):
        P.lib().pft_solver_set_option(P.PFT_OPT_GATE, gate)
        sim = _sim(meta)
        recs = []
        for k in caps:
            rc = sim.solve_ex(1e9, k, P.PFT_SOLVE_KEEP_DEVICE | (P.PFT_SOLVE_REUSE_DEVICE if recs else 0))
            assert rc == 2
            recs.append(_rec(sim))
        sim.download()
        out[gate] = (recs, _sha(sim.interior()), sim.stats().gated_steps)
        sim.close()
    assert out[0][0] == out[1][0]
    assert out[0][1] == out[1][1]
    assert out[0][2] == 0 and out[1][2] > 0


def test_gated_host_boundary_calls(g100):
    """RK_MPI_SA_solve's own boundary (x up and down every call) to short snapshot times: the
    armed decision is released before the state leaves the device"""
    meta, _ = g100
    times = [0.5, 0.75, 1.0, 2.0, 3.0]
    out = {}
    for gate in (0, 1):
        P.lib().pft_solver_set_option(P.PFT_OPT_GATE, gate)
        sim = _sim(meta)
        recs = []
        for T in times:
            assert sim.solve(T) == 0
            recs.append(_rec(sim) + (_sha(sim.interior()),))
        out[gate] = recs
        sim.close()
    assert out[0] == out[1]


def test_gated_discards_a_differing_decision(g100):
    """the host's check of the device's decision: with every 5th accepted device decision's h off
    by one bit (test hook PFT_GATE_FLIP), each such gated step is discarded and relaunched with the
    host's h, and the trajectory is still the reference's, bit for bit"""
    meta, A = g100
    os.environ["PFT_GATE_FLIP"] = "5"
    try:
        sim = _sim(meta)
    finally:
        del os.environ["PFT_GATE_FLIP"]
    misses = gated = 0
    for i, T in enumerate(meta["traj_times"]):
        rc = sim.solve(T)
        ref = meta["traj_m0"][i]
        assert (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc) == \
            (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
        assert _sha(sim.interior()) == meta["traj_m0_sha256"][i]
        st = sim.stats()
        misses += st.gate_misses
        gated += st.gated_steps
    sim.close()
    assert misses >= 10 and gated > 0, (misses, gated)
