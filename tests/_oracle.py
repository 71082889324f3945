"""ctypes access to the CPU oracle (oracle/lib/libpft_oracle.so).

Test infrastructure only: the oracle is the checker, never the thing measured or shipped.
"""
import ctypes as C
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
LIB_PATH = os.path.join(REPO, "oracle", "lib", "libpft_oracle.so")

# parameter order of model.c:44-59 (include/pft_model.h)
PARAM_NAMES = [
    "u_star", "L", "xi", "a", "b", "alpha", "mu",
    "beads_scaling", "beads_offset_x", "beads_offset_y", "beads_offset_z",
    "xi_gl", "zeta", "p_eps0", "p_eps1", "gamma",
    "water_cp", "ice_cp", "glass_cp", "water_lambda", "ice_lambda", "glass_lambda",
    "water_rho", "ice_rho", "glass_rho", "top_temp1", "top_temp2", "phase_switch_time",
    "u_noise_amp", "ball_radius",
]
BT = 2


class Grid(C.Structure):
    _fields_ = [("n1", C.c_int), ("n2", C.c_int), ("n3", C.c_int), ("total_n3", C.c_int),
                ("first_row", C.c_int), ("rank", C.c_int), ("nprocs", C.c_int),
                ("L1", C.c_double), ("L2", C.c_double), ("L3", C.c_double)]


EXCHANGE_FN = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_void_p)
ALLREDUCE_FN = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_void_p)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: make -C oracle port")
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        L.pft_or_bcond.argtypes = [C.POINTER(Grid), dp, C.c_double, dp]
        L.pft_or_stencil.argtypes = [C.POINTER(Grid), dp, C.c_int, dp, dp, dp]
        L.pft_or_rhs.argtypes = [C.POINTER(Grid), dp, C.c_int, C.c_double, dp, dp]
        L.pft_or_solve.argtypes = [C.POINTER(Grid), dp, C.c_int, C.c_double, dp, dp, C.c_double,
                                   C.c_double, C.c_int, dp, C.POINTER(C.c_long), C.POINTER(C.c_long),
                                   C.c_long, EXCHANGE_FN, ALLREDUCE_FN, C.c_void_p]
        L.pft_or_solve.restype = C.c_int
        L.pft_or_ic_default.argtypes = [C.POINTER(Grid), dp, dp, C.c_int, dp]
        L.pft_or_set_noise.argtypes = [dp]
        L.pft_or_set_noise.restype = None
        L.pft_or_float_val.argtypes = [C.c_char_p]
        L.pft_or_float_val.restype = C.c_double
        L.pft_or_decompose.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.pft_or_exchange_local.argtypes = [C.POINTER(Grid), C.POINTER(dp), C.c_int]
        _lib = L
    return _lib


def ptr(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_double))


def load_case(name):
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    arrays = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    return meta, arrays


def params_from_meta(meta):
    p = meta["params"]
    P = np.array([float.fromhex(p[k]) for k in PARAM_NAMES], dtype=np.float64)
    info = {k: (float.fromhex(v) if isinstance(v, str) else v) for k, v in p.items()}
    return P, info


def decompose(total_n3, nprocs, rank):
    n3, fr = C.c_int(), C.c_int()
    lib().pft_or_decompose(total_n3, nprocs, rank, C.byref(n3), C.byref(fr))
    return n3.value, fr.value


def make_grid(info, nprocs=1, rank=0):
    n3, fr = decompose(info["n3"], nprocs, rank)
    return Grid(info["n1"], info["n2"], n3, info["n3"], fr, rank, nprocs,
                info["L1"], info["L2"], info["L3"])


def pad(g, interior_global):
    """global interior [3][total_n3][n2][n1] -> this slab's padded host-layout array (zeros in ghosts)"""
    N1, N2, N3 = g.n1 + 2 * BT, g.n2 + 2 * BT, g.n3 + 2 * BT
    w = np.zeros((3, N3, N2, N1))
    w[:, BT:BT + g.n3, BT:BT + g.n2, BT:BT + g.n1] = interior_global[:, g.first_row:g.first_row + g.n3]
    return np.ascontiguousarray(w)


def unpad(g, w):
    N1, N2, N3 = g.n1 + 2 * BT, g.n2 + 2 * BT, g.n3 + 2 * BT
    w = w.reshape(3, N3, N2, N1)
    return np.ascontiguousarray(w[:, BT:BT + g.n3, BT:BT + g.n2, BT:BT + g.n1])


def rhs(info, P, mode, t, state, nprocs=1, noise=None):
    """K = f(t, state) on `nprocs` slabs held in this process (local exchange); noise: the single
    slab's u_noise field [k][j][i] (equation.c:450-456) or None"""
    assert noise is None or nprocs == 1
    grids = [make_grid(info, nprocs, r) for r in range(nprocs)]
    ws = [pad(g, state) for g in grids]
    dws = [np.zeros_like(w) for w in ws]
    L = lib()
    for g, w in zip(grids, ws):
        L.pft_or_bcond(C.byref(g), ptr(P), t, ptr(w))
    if nprocs > 1:
        arr = (Grid * nprocs)(*grids)
        wp = (C.POINTER(C.c_double) * nprocs)(*[ptr(w) for w in ws])
        L.pft_or_exchange_local(arr, wp, nprocs)
    for g, w, dw in zip(grids, ws, dws):
        L.pft_or_stencil(C.byref(g), ptr(P), mode, ptr(w),
                         None if noise is None else ptr(np.ascontiguousarray(noise, dtype=np.float64)), ptr(dw))
    out = np.concatenate([unpad(g, dw) for g, dw in zip(grids, dws)], axis=1)
    return out, ws


def solve(info, P, mode, state, t0, h0, times, max_steps_total=0, noise=None):
    """single-slab Merson solve to each time in `times`; returns [(t,h,steps,total,rc,state)];
    noise: the u_noise field [k][j][i] its right-hand side adds (equation.c:676-687) or None"""
    g = make_grid(info)
    x = pad(g, state)
    t, h = C.c_double(t0), C.c_double(h0)
    steps, total = C.c_long(0), C.c_long(0)
    res = []
    nz = None if noise is None else np.ascontiguousarray(noise, dtype=np.float64)
    lib().pft_or_set_noise(None if nz is None else ptr(nz))
    try:
        for T in times:
            rc = lib().pft_or_solve(C.byref(g), ptr(P), mode, T, C.byref(t), C.byref(h), info["tau_min"],
                                    info["delta"], 0, ptr(x), C.byref(steps), C.byref(total),
                                    max_steps_total, EXCHANGE_FN(), ALLREDUCE_FN(), None)
            res.append((t.value, h.value, steps.value, total.value, rc, unpad(g, x)))
    finally:
        lib().pft_or_set_noise(None)
    return res


def glibc_noise(amp, n, seed=1):
    """u_noise = amp (rand()/RAND_MAX - 0.5) for n nodes (equation.c:450-456) from glibc's rand()
    after srand(seed) -- what the reference draws when nothing seeded rand() (seed 1)"""
    libc = C.CDLL("libc.so.6")
    libc.srand(seed)
    r = np.array([libc.rand() for _ in range(n)], dtype=np.float64)
    return amp * (r / 2147483647.0 - 0.5)


def ic_default(info, P, beads, nprocs=1, rank=0):
    g = make_grid(info, nprocs, rank)
    w = np.zeros(3 * (g.n1 + 4) * (g.n2 + 4) * (g.n3 + 4))
    b = np.ascontiguousarray(beads, dtype=np.float64)
    lib().pft_or_ic_default(C.byref(g), ptr(P), ptr(b), b.shape[0], ptr(w))
    return unpad(g, w)


def beads():
    return np.load(os.path.join(GOLDEN, "beads.npy"))
