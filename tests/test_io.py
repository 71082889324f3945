"""Snapshot / restart datasets (include/pft_io.h), CPU only.

The reference writes its snapshots through the NetCDF library in classic format
(intertrack.c:2326-2548).  No NetCDF library exists in this image and the reference ships no
snapshot files, so the writer is checked against an independent reader of the classic format
(scipy.io.netcdf_file): dimensions, coordinate variables, the u/p/gl arrays and the global
attributes in the reference's order.  Parity with a reference-written file is unpinned.
"""
import os

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P

netcdf = pytest.importorskip("scipy.io").netcdf_file

# intertrack.c:2382-2406 with param_info[] order (model.c:85-137)
ATTR_ORDER = (["L1", "L2", "L3", "u_star", "L", "water_cp", "ice_cp", "glass_cp", "water_lambda", "ice_lambda",
               "glass_lambda", "water_rho", "ice_rho", "glass_rho", "ball_radius", "beads_scaling",
               "beads_offset_x", "beads_offset_y", "beads_offset_z", "xi_gl", "zeta", "xi", "a", "b", "alpha",
               "mu", "p_eps0", "p_eps1", "gamma", "top_temp1", "top_temp2", "phase_switch_time",
               "u_noise_amp"] + ["calc_mode", "delta", "tau", "t", "final_time", "snapshot", "total_snapshots",
                                 "title"])


def _sim(meta, state, nprocs=1, rank=0):
    Pm, info = O.params_from_meta(meta)
    return P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                        nprocs=nprocs, rank=rank, initial=state, init_solver=False), Pm, info


@pytest.fixture(scope="module")
def ragged():
    return O.load_case("ragged")


def _info(meta):
    _, info = O.params_from_meta(meta)
    return P.snapshot_info(t=1234.5, tau=0.25, final_time=36000.0, delta=info["delta"], calc_mode=0,
                           snapshot=7, total_snapshots=100, comment="Testing run")


def test_snapshot_matches_classic_netcdf_reader(tmp_path, ragged):
    meta, A = ragged
    sim, Pm, info = _sim(meta, A["state"])
    path = str(tmp_path / "image.007.000.ncd")
    P.save_snapshot(sim, path, _info(meta))
    sim.close()
    with netcdf(path, "r", mmap=False) as f:
        assert f.version_byte == 1
        assert list(f.dimensions.items()) == [("n3", info["n3"]), ("n2", info["n2"]), ("n1", info["n1"])]
        assert list(f.variables) == ["n3", "n2", "n1", "u", "p", "gl"]
        assert list(f._attributes) == ATTR_ORDER
        for q, v in enumerate(("u", "p", "gl")):
            assert np.array_equal(f.variables[v][:], A["state"][q])
        # coordinates, intertrack.c:2441-2443
        for name, L, n in (("n3", info["L3"], info["n3"]), ("n2", info["L2"], info["n2"]), ("n1", info["L1"], info["n1"])):
            assert np.array_equal(f.variables[name][:], np.array([L * (0.5 + k - 0) / n for k in range(n)]))
        at = f._attributes
        assert at["t"] == 1234.5 and at["tau"] == 0.25 and at["final_time"] == 36000.0
        assert at["snapshot"] == 7 and at["total_snapshots"] == 100 and at["calc_mode"] == 0
        assert at["title"] == b"Intertrack simulation (Testing run). Time: 1234.5"
        for k, name in enumerate(O.PARAM_NAMES):
            assert at[name] == Pm[k], name


@pytest.mark.parametrize("nw,nr", [(3, 1), (1, 4), (4, 2)])
def test_slab_parallel_write_and_restart_read(tmp_path, ragged, nw, nr):
    """each rank writes only its Z-slab planes into the shared file (no gather); reading back with
    another decomposition restores every slab (continue_series restart, intertrack.c:1584-1669)"""
    meta, A = ragged
    path = str(tmp_path / "snap.ncd")
    sims = [_sim(meta, A["state"], nw, r)[0] for r in range(nw)]
    info = _info(meta)
    L = P.lib()
    assert L.pft_snapshot_create(path.encode(), P.C.byref(sims[0].grid), P._dp(sims[0].params), P.C.byref(info), 0) == 0
    for s in reversed(sims):
        assert L.pft_snapshot_write_slab(path.encode(), P.C.byref(s.grid), P._dp(s.x)) == 0
        s.close()
    with netcdf(path, "r", mmap=False) as f:
        for q, v in enumerate(("u", "p", "gl")):
            assert np.array_equal(f.variables[v][:], A["state"][q])
    n1, n2, n3, got, prm = P.read_snapshot_info(path)
    assert (n1, n2, n3) == (A["state"].shape[3], A["state"].shape[2], A["state"].shape[1])
    assert (got.t, got.tau, got.snapshot, got.total_snapshots) == (1234.5, 0.25, 7, 100)
    assert np.array_equal(prm, sims[0].params)
    parts = []
    for r in range(nr):
        s, _, _ = _sim(meta, np.zeros_like(A["state"]), nr, r)
        P.load_snapshot(s, path)
        parts.append(s.interior())
        s.close()
    assert np.array_equal(np.concatenate(parts, axis=1), A["state"])


def test_cdf2_and_errors(tmp_path, ragged):
    meta, A = ragged
    sim, Pm, info = _sim(meta, A["state"])
    L = P.lib()
    path = str(tmp_path / "snap64.ncd")
    inf = _info(meta)
    assert L.pft_snapshot_create(path.encode(), P.C.byref(sim.grid), P._dp(sim.params), P.C.byref(inf), 2) == 0
    assert L.pft_snapshot_write_slab(path.encode(), P.C.byref(sim.grid), P._dp(sim.x)) == 0
    with netcdf(path, "r", mmap=False) as f:
        assert f.version_byte == 2
        assert np.array_equal(f.variables["gl"][:], A["state"][2])
    # not a dataset / wrong grid
    bad = tmp_path / "bad.ncd"
    bad.write_bytes(b"not netcdf at all")
    assert L.pft_snapshot_read_slab(str(bad).encode(), P.C.byref(sim.grid), P._dp(sim.x)) == -3
    other, _, _ = _sim(O.load_case("g20")[0], O.load_case("g20")[1]["ic"])
    assert L.pft_snapshot_read_slab(path.encode(), P.C.byref(other.grid), P._dp(other.x)) == -4
    assert L.pft_snapshot_read_slab(str(tmp_path / "missing.ncd").encode(), P.C.byref(sim.grid), P._dp(sim.x)) == -1
    other.close()
    sim.close()
    assert os.path.getsize(path) > A["state"].nbytes
