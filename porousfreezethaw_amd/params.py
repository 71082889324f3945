"""The reference's default Params file (apps/intertrack-hybrid-S-freezing/Params:43-144) evaluated
with the reference front end's arithmetic.

pparse (modules/pparser/pparser.c:70-108) evaluates every `name expression` line with the
Digithell expression evaluator, whose numeric literals go through float_val
(libsource/strings/str_fval.c:13-88) -- NOT strtod: `1e-6` becomes 1/10/10/10/10/10/10, which
differs from the C literal in the last bit.  Since trajectories are rounding-sensitive (SURVEY
F7), parameters must be bit-identical to the reference's; tests/test_params.py checks this module
against the parameter dump the reference itself produced (tests/golden/g20.json).
"""


def float_val(s):
    """str_fval.c:13-88: integer digits accumulated, fraction digits accumulated as an integer
    and divided by pow(10, count), exponent applied by repeated *10 or /10."""
    out = decimal = 0.0
    decnum = expnum = 0
    point = neg = expneg = expsign = False
    expflag = 0
    x = 0
    if s[:1] == "-":
        neg, x = True, 1
    elif s[:1] == "+":
        x = 1
    while x < len(s):
        c = s[x]
        x += 1
        if c == ".":
            if not (point or expflag):
                point = True
            continue
        if c in "eE":
            if not expflag:
                expflag = 1
            continue
        if c == "-" and expflag == 1:
            expsign = expneg = True
            expflag += 1
            continue
        if c == "+" and expflag == 1:
            expsign = True
            expflag += 1
            continue
        if c.isdigit():
            d = ord(c) - 48
            if not expflag:
                if not point:
                    out = out * 10 + d
                else:
                    decimal = decimal * 10 + d
                    decnum += 1
            else:
                expnum = expnum * 10 + d
                expflag += 1
    out += decimal / (10.0 ** decnum)
    while expnum > 0:
        expnum -= 1
        out = out / 10 if expneg else out * 10
    return -out if neg else out


def to_int(x):
    """intertrack.c:673-681"""
    import math
    r = math.floor(x)
    if x - r >= 0.5:
        r += 1
    return int(r)


def default_params(grid_nodes=100, calc_mode=0, L=None):
    """Evaluate the default Params (in file order, left-to-right like the evaluator).
    Returns (param dict, geometry dict).  L=(L1,L2,L3) overrides the domain size."""
    f = float_val
    v = {}
    v["hours"] = f("60") * f("60")
    v["L1"], v["L2"], v["L3"] = f("0.03"), f("0.03"), f("0.06")
    if L is not None:
        v["L1"], v["L2"], v["L3"] = L
    v["u_noise_amp"] = f("0")
    v["water_cp"], v["ice_cp"], v["glass_cp"] = f("4.18e3"), f("2.05e3"), f("0.84e3")
    v["water_lambda"], v["ice_lambda"], v["glass_lambda"] = f("0.6"), f("2.22"), f("1.1")
    v["water_rho"], v["ice_rho"], v["glass_rho"] = f("997"), f("917"), f("2500")
    v["u_star"], v["L"] = f("273.15"), f("3.34e5")
    v["wall_thickness"] = f("0.05")
    v["beads_scaling"] = (f("1") - f("2") * v["wall_thickness"]) * v["L1"]
    v["ball_radius"] = f("0.1") * v["beads_scaling"]
    v["beads_offset_x"] = v["wall_thickness"] * v["L1"]
    v["beads_offset_y"] = v["beads_offset_x"]
    v["beads_offset_z"] = v["beads_offset_x"]
    v["xi_gl"] = v["L3"] / f("500")
    v["zeta"] = f("1.05")
    v["xi"] = v["L3"] / f("100")
    v["a"], v["b"] = f("2"), f("1")
    v["alpha"] = v["water_rho"] * v["water_cp"]
    v["mu"] = f("1e-4")
    v["p_eps0"], v["p_eps1"] = f("0.05"), f("0.2")
    v["gamma"] = f("2")
    v["top_temp1"] = f("273.15") - f("25")
    v["top_temp2"] = f("273.15") + f("20")
    v["phase_switch_time"] = f("5") * v["hours"]
    v["calc_mode"] = calc_mode
    v["final_time"] = f("10") * v["hours"]
    v["saved_files"] = f("100")
    v["delta"], v["tau_min"], v["tau"] = f("1e-3"), f("1e-6"), f("1")
    v["grid_nodes"] = float(grid_nodes)
    m = max(v["L1"], v["L2"], v["L3"])        # "L1 max L2 max L3"
    v["multiplier"] = v["grid_nodes"] / m
    v["n1"] = to_int(v["L1"] * v["multiplier"])
    v["n2"] = to_int(v["L2"] * v["multiplier"])
    v["n3"] = to_int(v["L3"] * v["multiplier"])
    return v
