"""SURVEY 8(f) f3 on the GPU: a parameter file goes through the front end (the pparser/exprsion
restatement in porousfreezethaw_amd/frontend.py: line grammar pparser.c:27-114, expression
evaluator ee_wrapper.cc:304-336, value extraction intertrack.c:1491-1575, icond formulas
intertrack.c:1831-2012) into RK_MPI_SA_solve on the HIP path, and lands on the reference's own
trajectory bit for bit (tests/golden/g20: the reference compiled in place, default model at
grid_nodes 20, t = 0 -> 36 s).

The parameter text below is this repository's own: the default model written with helper
variables and a different layout (cap centre and radius, one reusable wall steepness, the
cooling/heating temperatures relative to u_star).  It evaluates to the same numbers because every
quantity is the same chain of operations on the same literals."""
import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P
from porousfreezethaw_amd import frontend as FE

pytestmark = pytest.mark.gpu

PARAMS = """\
# libpft front-end check: the freezing-around-glass-beads model, default values
grid_nodes      20
L1 0.03
L2 0.03
L3 0.06
multiplier      grid_nodes / (L1 max L2 max L3)
n1 L1 * multiplier
n2 L2 * multiplier
n3 L3 * multiplier

hours           60*60
final_time      10*hours
saved_files     100
tau             1
tau_min         1e-6
delta           1e-3
calc_mode       0

# water / ice / glass
water_rho 997
ice_rho 917
glass_rho 2500
water_cp 4.18e3
ice_cp 2.05e3
glass_cp 0.84e3
water_lambda 0.6
ice_lambda 2.22
glass_lambda 1.1
u_star          273.15
L               3.34e5
u_noise_amp     0

# phase field
xi      L3/100
a       2
b       1
alpha   water_rho*water_cp
mu      1e-4
p_eps0  0.05
p_eps1  0.2
gamma   2

# container walls and beads
wall_thickness  0.05
beads_offset_x  wall_thickness*L1
beads_offset_y  beads_offset_x
beads_offset_z  beads_offset_x
beads_scaling   (1-2*wall_thickness)*L1
ball_radius     0.1*beads_scaling
xi_gl           L3/500
zeta            1.05
steep           0.5/xi_gl

# boundary temperature programme
top_temp1         u_star - 25
top_temp2         u_star + 20
phase_switch_time 5*hours

# initial state: room temperature, an ice lens under the lid, glass lid + walls
cap_x  L1/2
cap_y  L2/2
cap_r2 (L1/3)^2
icond u = "293.15"
icond p = "(z>0.052) and (z<0.058) and ((x-cap_x)^2+(y-cap_y)^2 < cap_r2)"
icond gl = "(0.5*(1.0 + tanh(steep*(beads_offset_y-y)))) max (0.5*(1.0 + tanh(steep*(z-0.055)))) max (0.5*(1.0 + tanh(steep*(beads_offset_x-x)))) max (0.5*(1.0 + tanh(steep*(beads_offset_z-z)))) max (0.5*(1.0 + tanh(steep*(y-L2+beads_offset_y)))) max (0.5*(1.0 + tanh(steep*(x-L1+beads_offset_x))))"

set out_file = $OUTPUT/image out_file_suffix = .ncd
set comment = "on-box front-end test"
"""


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if P.device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback exists)")


@pytest.mark.parametrize("nprocs", [1, 2])
def test_params_text_to_hip_solve_equals_reference(nprocs, tmp_path):
    meta, A = O.load_case("g20")
    Pm, info = O.params_from_meta(meta)
    case = FE.load_params(text=PARAMS, env={"OUTPUT": str(tmp_path)})
    assert np.array_equal(case.params, Pm)
    assert case.n == (info["n1"], info["n2"], info["n3"]) and case.L == (info["L1"], info["L2"], info["L3"])
    assert (case.tau, case.tau_min, case.delta, case.calc_mode) == (1.0, info["tau_min"], info["delta"], 0)
    assert case.settings["out_file"] == str(tmp_path) + "/image"
    T = meta["traj_times"][0]
    ref = meta["traj_m0"][0]
    if nprocs == 1:
        sim = case.simulation(beads=O.beads())
        assert np.array_equal(sim.interior(), A["traj_m0_ic"])      # icond formulas + beads
        rc = sim.solve(T)
        assert sim.stats().path == 1
        got = [(sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc)]
        x = sim.interior()
        sim.close()
    else:
        import _multi as M

        def run(sim):
            rc = sim.solve(T)
            return (sim.t.hex(), sim.h.hex(), sim.system.steps, sim.system.steps_total, rc), sim.interior()

        out = M.loopback_run(nprocs, lambda r: case.simulation(nprocs=nprocs, rank=r, beads=O.beads()), run)
        got = [o[0] for o in out]
        x = np.concatenate([o[1] for o in out], axis=1)
    for g in got:
        assert g == (float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
    assert np.array_equal(x, A["traj_m0_state0"])
