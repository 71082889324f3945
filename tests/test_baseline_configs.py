"""BASELINE.json's configurations at full size on the HIP path (SURVEY F5 grids, default Params
initial condition with the 200 glass beads, t = 0, h = tau = 1 s):

  configs[1]  400^3 = 200 x 200 x 400, 1 GPU      -> >= 50 attempted steps vs the oracle, calc_mode
                                                   0 and 1 bit for bit, mode 2 to 1e-10
  configs[2]  200^3 = 100 x 100 x 200, 1 GPU      -> 60 attempted steps vs the oracle, bit for bit
  configs[3]  400^3, 4-way Z-slab split           -> 4 slabs (loopback transport on one GPU) equal
                                                   the single-slab run bit for bit
  configs[4]  800^3 = 400 x 400 x 800, 8-way      -> 8 slabs of 400 x 400 x 100 equal the single-slab
                                                   800^3 device run and the oracle bit for bit

(configs[0], 100^3, is tests/test_g100.py.)  The attempted steps start from h = 1 s, far above
what the error norm admits, so every run includes rejected steps (asserted).  The decomposition
is the reference's (intertrack.c:1776-1800); SURVEY F6: results do not depend on it."""
import numpy as np
import pytest

import _multi as M
import _oracle as O
import porousfreezethaw_amd as P

pytestmark = pytest.mark.gpu

# calc_mode 2 calls cosh: ROCm's ocml and glibc differ by <= 1 ulp
MODE2_RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


def _device_run(grid_nodes, mode, steps, **kw):
    base, Pm, info = M.full_size_case(grid_nodes, mode)
    sim = P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode, Pm,
                       beads=O.beads(), tau=1.0, tau_min=info["tau_min"], delta=info["delta"], **kw)
    ic = sim.interior()
    assert sim.solve_ex(1e9, steps, 0) == 2
    st = sim.stats()
    assert st.path == 1 and st.steps_total == steps
    got = (sim.t, sim.h, sim.system.steps, sim.system.steps_total)
    x = sim.interior()
    sim.close()
    return Pm, info, ic, got, x


@pytest.mark.parametrize("grid_nodes,mode,steps", [(200, 0, 60), (400, 0, 50), (400, 1, 50)])
def test_full_size_vs_oracle_bitwise(grid_nodes, mode, steps):
    Pm, info, ic, got, x = _device_run(grid_nodes, mode, steps)
    assert got[2] < got[3], "no rejected step in the window"
    res = O.solve(info, Pm, mode, ic, 0.0, 1.0, [1e9], max_steps_total=steps)[0]
    assert (got[0].hex(), got[1].hex(), got[2], got[3]) == (res[0].hex(), res[1].hex(), res[2], res[3])
    assert np.array_equal(x, res[5])


def test_full_size_400_mode2_tolerance():
    """calc_mode 2 (Temp, device cosh): 50 attempted steps at 400^3, same accept/reject sequence,
    t, h and every field within MODE2_RTOL of the oracle (normwise per field)"""
    steps = 50
    Pm, info, ic, got, x = _device_run(400, 2, steps)
    res = O.solve(info, Pm, 2, ic, 0.0, 1.0, [1e9], max_steps_total=steps)[0]
    assert (got[2], got[3]) == (res[2], res[3])
    assert abs(got[0] - res[0]) <= MODE2_RTOL * abs(res[0])
    assert abs(got[1] - res[1]) <= MODE2_RTOL * abs(res[1])
    assert np.all(np.abs(x - res[5]) <= MODE2_RTOL * np.abs(res[5]).max(axis=(1, 2, 3), keepdims=True))


def _multislab(grid_nodes, nprocs, steps, ic):
    base, Pm, info = M.full_size_case(grid_nodes, 0)

    def make(r):
        return P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), 0, Pm,
                            nprocs=nprocs, rank=r, initial=ic, tau=1.0, tau_min=info["tau_min"],
                            delta=info["delta"])

    def run(sim):
        assert sim.solve_ex(1e9, steps, 0) == 2
        return (sim.t, sim.h, sim.system.steps, sim.system.steps_total), sim.interior(), sim.grid.n3

    return M.loopback_run(nprocs, make, run)


def test_400_four_slabs_equal_one_slab():
    """configs[3]: 400^3 split 4-way (4 x 100 planes), halo exchange per stage, 12 attempted steps"""
    steps = 12
    Pm, info, ic, got, x = _device_run(400, 0, steps)
    out = _multislab(400, 4, steps, ic)
    assert [o[2] for o in out] == [100] * 4
    for o in out:
        assert o[0] == got
    assert np.array_equal(np.concatenate([o[1] for o in out], axis=1), x)


def test_800_eight_slabs_equal_one_slab_and_oracle():
    """configs[4]: 800^3 = 400 x 400 x 800 (128 M cells), 8 slabs of 400 x 400 x 100 on one GPU,
    4 attempted steps: the 8-slab run equals the single-slab device run and the oracle bit for bit"""
    steps = 4
    Pm, info, ic, got, x = _device_run(800, 0, steps)
    assert info["n1"] == 400 and info["n3"] == 800
    out = _multislab(800, 8, steps, ic)
    assert [o[2] for o in out] == [100] * 8
    for o in out:
        assert o[0] == got
    assert np.array_equal(np.concatenate([o[1] for o in out], axis=1), x)
    del out
    res = O.solve(info, Pm, 0, ic, 0.0, 1.0, [1e9], max_steps_total=steps)[0]
    assert (got[0].hex(), got[1].hex(), got[2], got[3]) == (res[0].hex(), res[1].hex(), res[2], res[3])
    assert np.array_equal(x, res[5])
