"""The Python restatement of the default Params evaluation equals the reference's own dump."""
import _oracle as O
from porousfreezethaw_amd import PARAM_NAMES, params


def test_default_params_bitwise():
    meta, _ = O.load_case("g20")
    ref = {k: (float.fromhex(v) if isinstance(v, str) else v) for k, v in meta["params"].items()}
    mine = params.default_params(grid_nodes=20)
    for k in PARAM_NAMES + ["L1", "L2", "L3", "tau", "tau_min", "delta", "final_time"]:
        assert mine[k] == ref[k], (k, mine[k], ref[k])
    for k in ("n1", "n2", "n3", "calc_mode"):
        assert mine[k] == ref[k]


def test_grid_nodes_family():
    for g, dims in [(100, (50, 50, 100)), (200, (100, 100, 200)), (400, (200, 200, 400)), (800, (400, 400, 800))]:
        p = params.default_params(grid_nodes=g)
        assert (p["n1"], p["n2"], p["n3"]) == dims


def test_float_val_matches_c():
    import porousfreezethaw_amd as P
    for s in ["1e-6", "293.15", "0.052", "4.18e3", "-2.5E-3", "0.03", "1", "273.15", "0.84e3", "3.34e5"]:
        assert params.float_val(s) == P.lib().pft_float_val(s.encode())
