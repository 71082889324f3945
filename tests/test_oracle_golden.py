"""Pin the CPU oracle (oracle/pft_oracle.c) to the reference's own outputs, bit for bit.

Golden vectors come from the reference compiled in place (tests/golden/gen_golden.py).
"""
import numpy as np
import pytest

import _oracle as O


@pytest.fixture(scope="module")
def g20():
    return O.load_case("g20")


@pytest.fixture(scope="module")
def ragged():
    return O.load_case("ragged")


def test_float_val_matches_reference_params(g20):
    meta, _ = g20
    _, info = O.params_from_meta(meta)
    fv = O.lib().pft_or_float_val
    # Params:130 "tau_min 1e-6" is NOT the correctly rounded 1e-6 in the reference
    assert fv(b"1e-6") == info["tau_min"]
    assert fv(b"1e-6") != 1e-6
    assert fv(b"1e-3") == info["delta"]
    assert fv(b"0.03") == info["L1"]


def test_ic_default_bitwise(g20):
    meta, A = g20
    P, info = O.params_from_meta(meta)
    ic = O.ic_default(info, P, O.beads())
    assert np.array_equal(ic, A["ic"])


def test_ic_default_slabs_bitwise(g20):
    meta, A = g20
    P, info = O.params_from_meta(meta)
    parts = [O.ic_default(info, P, O.beads(), 3, r) for r in range(3)]
    assert np.array_equal(np.concatenate(parts, axis=1), A["ic"])


@pytest.mark.parametrize("mode", [0, 1, 2, 10, 11])
@pytest.mark.parametrize("tag", ["t0", "t1"])
def test_rhs_g20_bitwise(g20, mode, tag):
    meta, A = g20
    P, info = O.params_from_meta(meta)
    K, _ = O.rhs(info, P, mode, meta["rhs_times"][tag], A["ic"])
    assert np.array_equal(K, A[f"rhs_m{mode}_{tag}"])


@pytest.mark.parametrize("mode", [0, 1, 2, 10, 11])
@pytest.mark.parametrize("tag", ["t0", "t1"])
@pytest.mark.parametrize("nprocs", [1, 4])
def test_rhs_ragged_bitwise(ragged, mode, tag, nprocs):
    meta, A = ragged
    P, info = O.params_from_meta(meta)
    K, _ = O.rhs(info, P, mode, meta["rhs_times"][tag], A["state"], nprocs)
    assert np.array_equal(K, A[f"rhs_m{mode}_{tag}"])


@pytest.mark.parametrize("tag", ["t0", "t1"])
def test_boundary_kat(ragged, tag):
    """every rank's padded input after bcond_setup + sync_solution (equation.c:266-326)"""
    meta, A = ragged
    P, info = O.params_from_meta(meta)
    _, ws = O.rhs(info, P, 0, meta["rhs_times"][tag], A["state"], 4)
    for r in range(4):
        ref = A[f"w4_{tag}_rank{r}"].reshape(ws[r].shape)
        assert np.array_equal(ws[r], ref), r
    _, ws1 = O.rhs(info, P, 0, meta["rhs_times"][tag], A["state"], 1)
    assert np.array_equal(ws1[0], A[f"w1_{tag}_rank0"].reshape(ws1[0].shape))


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_trajectory_bitwise(g20, mode):
    meta, A = g20
    P, info = O.params_from_meta(meta)
    res = O.solve(info, P, mode, A[f"traj_m{mode}_ic"], 0.0, 1.0, meta["traj_times"])
    for i, (t, h, s, st, rc, x) in enumerate(res):
        ref = meta[f"traj_m{mode}"][i]
        assert (t.hex(), h.hex(), s, st, rc) == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(),
                                                 ref[2], ref[3], ref[4])
        assert np.array_equal(x, A[f"traj_m{mode}_state{i}"])


@pytest.mark.parametrize("tag", ["small", "large"])
def test_single_step_bitwise(ragged, tag):
    meta, A = ragged
    P, info = O.params_from_meta(meta)
    m = meta[f"step_{tag}"]
    (t, h, s, st, rc, x), = O.solve(info, P, 0, A["state"], m["t0"], m["h0"], [m["T"]])
    r = m["result"]
    assert (t.hex(), h.hex(), s, st, rc) == (float.fromhex(r[0]).hex(), float.fromhex(r[1]).hex(), r[2], r[3], r[4])
    assert np.array_equal(x, A[f"step_{tag}"])


@pytest.mark.parametrize("mode", [10, 11])
def test_trajectory_no_flux_modes_bitwise(mode):
    """calc_mode 10 and 11 (no heat-flux term, du = 0): the oracle's trajectory to the g20 snapshot
    times equals the reference's own (tests/golden/g20nf, from gen_golden.py)"""
    meta, A = O.load_case("g20nf")
    P, info = O.params_from_meta({"params": meta[f"m{mode}_params"]})
    assert info["calc_mode"] == mode
    res = O.solve(info, P, mode, A[f"traj_m{mode}_ic"], 0.0, 1.0, meta["traj_times"])
    for i, (t, h, s, st, rc, x) in enumerate(res):
        ref = meta[f"traj_m{mode}"][i]
        assert (t.hex(), h.hex(), s, st, rc) == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(),
                                                 ref[2], ref[3], ref[4])
        assert np.array_equal(x, A[f"traj_m{mode}_state{i}"])


# ---- u_noise (tests/golden/gnoise: the reference with u_noise_amp = 0.5 K on one rank) ----------

def test_noise_field_is_glibc_rand_from_seed_1():
    """the reference's noise field (equation.c:450-456, rand() never seeded by the harness) is
    amp (rand()/RAND_MAX - 0.5) of glibc's sequence from seed 1, node by node in [k][j][i] order --
    what libpft draws after srand(1) (intertrack_model.c PrecalculateData)"""
    meta, A = O.load_case("gnoise")
    noise = O.glibc_noise(meta["u_noise_amp"], A["noise"].size)
    assert np.abs(A["noise"]).max() > 0.2
    assert np.array_equal(noise.reshape(A["noise"].shape), A["noise"])


@pytest.mark.parametrize("mode", [0, 10, 1, 11])
def test_noise_rhs_equals_reference(mode):
    """the four models that add u_noise to u in their reaction term (equation.c:676, 687), at a
    state with mixed phases"""
    meta, A = O.load_case("gnoise")
    P, info = O.params_from_meta({"params": meta[f"m{mode}_params"]})
    assert info["calc_mode"] == mode and P[O.PARAM_NAMES.index("u_noise_amp")] == meta["u_noise_amp"]
    x, t = A[meta["rhs_state"]], meta["rhs_time"]
    K, _ = O.rhs(info, P, mode, t, x, noise=A["noise"])
    assert np.array_equal(K, A[f"rhs_m{mode}"])
    K0, _ = O.rhs(info, P, mode, t, x)
    assert not np.array_equal(K0, A[f"rhs_m{mode}"])        # the noise is seen


@pytest.mark.parametrize("mode", [0, 1])
def test_noise_trajectory_equals_reference(mode):
    meta, A = O.load_case("gnoise")
    P, info = O.params_from_meta({"params": meta[f"m{mode}_params"]})
    res = O.solve(info, P, mode, A["ic"], 0.0, 1.0, meta["traj_times"], noise=A["noise"])
    for i, (t, h, s, st, rc, x) in enumerate(res):
        ref = meta[f"traj_m{mode}"][i]
        assert (t.hex(), h.hex(), s, st, rc) == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(),
                                                 ref[2], ref[3], ref[4])
        assert np.array_equal(x, A[f"traj_m{mode}_state{i}"])
