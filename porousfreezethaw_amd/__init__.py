"""porousfreezethaw_amd -- MI355X-native RK-Merson solver + intertrack freezing model.

The product is the C library ``lib/libpft.so`` (host C + HIP kernels for gfx950); this module is
a thin ctypes view of its C ABI for tests, the benchmark and scripting.  Names and argument
meaning follow the reference's C interface (include/RK_MPI_SAsolver.h, equation.c, model.c).
There is no CPU fallback: if the library (or a GPU, for the solving calls) is missing, the calls
fail loudly.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.environ.get("PFT_LIB") or os.path.join(HERE, "lib", "libpft.so")

PARAM_NAMES = [  # model.c:44-59, the order of param[] (include/pft_model.h)
    "u_star", "L", "xi", "a", "b", "alpha", "mu",
    "beads_scaling", "beads_offset_x", "beads_offset_y", "beads_offset_z",
    "xi_gl", "zeta", "p_eps0", "p_eps1", "gamma",
    "water_cp", "ice_cp", "glass_cp", "water_lambda", "ice_lambda", "glass_lambda",
    "water_rho", "ice_rho", "glass_rho", "top_temp1", "top_temp2", "phase_switch_time",
    "u_noise_amp", "ball_radius",
]
BCOND_THICKNESS = 2
DELTA_LOCAL, DELTA_GLOBAL = 0, 1
RKA_CMD_FINISHED = 8
PFT_SOLVE_KEEP_DEVICE, PFT_SOLVE_REUSE_DEVICE = 1, 2
PFT_OPT_GL_STATIC, PFT_OPT_KZ, PFT_OPT_DEVICE, PFT_OPT_TIMING, PFT_OPT_TILE, PFT_OPT_RECOMPUTE = 1, 2, 3, 4, 5, 6
PFT_OPT_LAZY_ALLOC = 9
PFT_OPT_PAIR = 10
PFT_OPT_GATE = 12
PFT_OPT_FAIL_RHS = 11
PFT_SOLVE_DEVICE_ERROR = -7
MPI_COMM_WORLD = 0x44000000

# every function of the public headers, for the "library exports its ABI" check
ABI_FUNCTIONS = [
    "RK_MPI_SA_init", "RK_MPI_SA_cleanup", "RK_MPI_SA_handle_NAN", "RK_MPI_SA_check_NAN",
    "RK_MPI_SA_check_mem", "RK_MPI_SA_solve",
]


class RK_MEM_DIST(C.Structure):
    _fields_ = [("n_chunks", C.c_int), ("chunk_start", C.POINTER(C.c_int)),
                ("chunk_size", C.POINTER(C.c_int)), ("chunk_eps_mult", C.POINTER(C.c_double))]


RHS_FN = C.CFUNCTYPE(None, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double))
META_FN = C.CFUNCTYPE(C.c_void_p)


class RK_MPI_S_SOLUTION(C.Structure):
    pass


SERVICE_FN = C.CFUNCTYPE(C.c_int, C.c_double, C.POINTER(RK_MPI_S_SOLUTION))
REARRANGE_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p)   # RK_MEM_DIST* (*)(RK_MEM_DIST*)
RK_MPI_S_SOLUTION._fields_ = [
    ("n", C.POINTER(RK_MEM_DIST)), ("t", C.c_double), ("x", C.POINTER(C.c_double)),
    ("meta_f", C.c_void_p), ("h", C.c_double), ("h_min", C.c_double), ("delta", C.c_double),
    ("delta_mode", C.c_int), ("DDLBF_Rearrange", C.c_void_p), ("Service_Callback", C.c_void_p),
    ("steps", C.c_long), ("steps_total", C.c_long)]


class pft_grid(C.Structure):
    _fields_ = [("n1", C.c_int), ("n2", C.c_int), ("n3", C.c_int), ("total_n3", C.c_int),
                ("first_row", C.c_int), ("rank", C.c_int), ("nprocs", C.c_int),
                ("L1", C.c_double), ("L2", C.c_double), ("L3", C.c_double), ("calc_mode", C.c_int)]


class pft_snapshot_info(C.Structure):
    """include/pft_io.h: the attributes of a snapshot dataset (intertrack.c:2393-2406)"""
    _fields_ = [("t", C.c_double), ("tau", C.c_double), ("final_time", C.c_double), ("delta", C.c_double),
                ("snapshot", C.c_int), ("total_snapshots", C.c_int), ("calc_mode", C.c_int),
                ("title", C.c_char * 256), ("L1", C.c_double), ("L2", C.c_double), ("L3", C.c_double)]


class pft_solver_stats(C.Structure):
    _fields_ = [("path", C.c_int), ("nprocs", C.c_int), ("rank", C.c_int),
                ("kernel_launches", C.c_long), ("steps_total", C.c_long), ("last_eps", C.c_double),
                ("stage_ms", C.c_double * 6), ("stage_n", C.c_long * 6), ("pairs", C.c_int),
                ("gated_steps", C.c_long), ("gate_misses", C.c_long)]


_lib = None


def lib():
    """Load libpft.so (built in-tree by __graft_entry__.build() / make -C porousfreezethaw_amd)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libpft.so is not built ({LIB_PATH}); run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)   # RTLD_LOCAL: its ROCm 7.2 runtime must not interpose on torch's
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int)
        L.RK_MPI_SA_init.argtypes = [C.c_int, C.c_int, C.c_int]
        L.RK_MPI_SA_check_mem.argtypes = [C.POINTER(RK_MEM_DIST)]
        L.RK_MPI_SA_solve.argtypes = [C.c_double, C.POINTER(RK_MPI_S_SOLUTION)]
        L.RK_MPI_SA_handle_NAN.argtypes = [C.c_int]
        L.RK_MPI_SA_handle_NAN.restype = None
        L.pft_solve_ex.argtypes = [C.c_double, C.POINTER(RK_MPI_S_SOLUTION), C.c_long, C.c_int]
        L.pft_solver_download.argtypes = [C.POINTER(RK_MPI_S_SOLUTION)]
        L.pft_solver_set_option.argtypes = [C.c_int, C.c_long]
        L.pft_solver_get_stats.argtypes = [C.POINTER(pft_solver_stats)]
        L.pft_solver_last_status.restype = C.c_int
        L.pft_solver_slab.restype = C.c_void_p
        L.pft_slab_tile_geometry.argtypes = [C.c_void_p, C.c_int, ip, ip]
        L.pft_decompose.argtypes = [C.c_int, C.c_int, C.c_int, ip, ip]
        L.pft_decompose.restype = None
        L.pft_grid_init.argtypes = [C.POINTER(pft_grid), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_double, C.c_double, C.c_double, C.c_int]
        L.pft_grid_block.argtypes = [C.POINTER(pft_grid)]
        L.pft_grid_block.restype = C.c_long
        L.pft_model_configure.argtypes = [C.POINTER(pft_grid), dp]
        L.bcond_setup.argtypes = [C.c_double, dp]
        L.bcond_setup.restype = None
        L.pft_model_set_beads.argtypes = [dp, C.c_int]
        L.pft_model_load_beads.argtypes = [C.c_char_p]
        L.PrecalculateData.argtypes = [dp]
        L.pft_model_set_solution.argtypes = [dp]
        L.pft_model_chunks.argtypes = [ip, ip, dp]
        L.pft_model_ic_default.argtypes = [dp]
        L.pft_float_val.argtypes = [C.c_char_p]
        L.pft_float_val.restype = C.c_double
        for name in ("f_generic_model01", "f_generic_model2"):
            getattr(L, name).argtypes = [C.c_double, dp, dp]
            getattr(L, name).restype = None
        for name in ("mf_single", "mf_top", "mf_middle", "mf_bottom"):
            getattr(L, name).restype = C.c_void_p
        L.pft_hip_device_count.argtypes = [ip]
        L.pft_hip_set_device.argtypes = [C.c_int]
        L.pft_ic_device_ok.argtypes = [C.POINTER(pft_grid), C.c_int, ip, dp]
        L.pft_solver_ic_formulas_device.argtypes = [C.c_int, ip, ip, ip, dp, C.c_int]
        L.pft_hip_last_error.restype = C.c_char_p
        L.pft_comm_get_unique_id.argtypes = [C.c_void_p]
        L.pft_comm_init_rccl.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_void_p, C.c_int]
        L.pft_comm_init_loopback.argtypes = [C.POINTER(C.c_void_p), C.c_int]
        L.pft_comm_init_ipc.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_char_p, C.c_int]
        L.pft_comm_device_halo.argtypes = [C.c_void_p]
        L.pft_comm_boundary_first.argtypes = [C.c_void_p]
        L.pft_comm_copy_engine.argtypes = [C.c_void_p]
        L.pft_comm_set_copy_engine.argtypes = [C.c_void_p, C.c_int]
        L.pft_comm_loopback_rank.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        L.pft_comm_set_current.argtypes = [C.c_void_p]
        L.pft_comm_destroy.argtypes = [C.c_void_p]
        L.pft_comm_set_self_exchange.argtypes = [C.c_void_p, C.c_int]
        L.pft_comm_splits.argtypes = [C.c_void_p]
        L.pft_comm_barrier.argtypes = [C.c_void_p]
        L.pft_comm_current.restype = C.c_void_p
        L.pft_comm_kind.argtypes = [C.c_void_p]
        L.pft_comm_kind.restype = C.c_char_p
        L.pft_slab_stream.argtypes = [C.c_void_p]
        L.pft_slab_stream.restype = C.c_void_p
        L.pft_hip_device_sync.restype = C.c_int
        gp, sp = C.POINTER(pft_grid), C.POINTER(pft_snapshot_info)
        L.pft_ic_eval.argtypes = [gp, C.c_int, C.c_int, ip, dp, dp]
        L.pft_model_noise.restype = dp
        L.pft_snapshot_create.argtypes = [C.c_char_p, gp, dp, sp, C.c_int]
        L.pft_snapshot_write_slab.argtypes = [C.c_char_p, gp, dp]
        L.pft_snapshot_write.argtypes = [C.c_char_p, gp, dp, sp, dp]
        L.pft_snapshot_read_info.argtypes = [C.c_char_p, ip, ip, ip, sp, dp]
        L.pft_snapshot_read_slab.argtypes = [C.c_char_p, gp, dp]
        L.pft_snapshot_title.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_double]
        _lib = L
    return _lib


def _dp(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_int))


def device_count():
    n = C.c_int(0)
    rc = lib().pft_hip_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def decompose(total_n3, nprocs, rank):
    n3, fr = C.c_int(), C.c_int()
    lib().pft_decompose(total_n3, nprocs, rank, C.byref(n3), C.byref(fr))
    return n3.value, fr.value


def comm_init_ipc(nranks, rank, name, device=0):
    """the ipc communicator of rank `rank` (pft_comm.h): every rank passes the same shared-memory
    name ("/..."), rank 0 creates it; bound to this thread (pft_comm_set_current).  Returns the handle."""
    c = C.c_void_p()
    rc = lib().pft_comm_init_ipc(C.byref(c), nranks, rank, name.encode(), device)
    if rc:
        raise RuntimeError(f"pft_comm_init_ipc(rank {rank}) failed ({rc}): {lib().pft_hip_last_error()}")
    lib().pft_comm_set_current(c)
    return c


def comm_destroy(c):
    lib().pft_comm_set_current(None)
    lib().pft_comm_destroy(c)


def params_array(values):
    """dict name -> value  ->  param[] in model.c order"""
    return np.array([float(values[k]) for k in PARAM_NAMES], dtype=np.float64)


class Simulation:
    """One slab of an intertrack run, driven exactly like intertrack.c drives the reference.

    Sets up the grid (intertrack.c:1776-1800), the host solution array and chunk table
    (:1803-1827, :2144-2157), the model (equation.c contract), and the solver
    (RK_MPI_SA_init :2192, check_mem :2208, PrecalculateData :2218), then solves with
    RK_MPI_SA_solve (:2283) or the device-resident pft_solve_ex.
    """

    def __init__(self, n1, n2, total_n3, L, calc_mode, params, nprocs=1, rank=0, beads=None,
                 initial=None, tau=1.0, tau_min=0.0, delta=1e-3, t0=0.0, gl_static=False, kz=None,
                 init_solver=True, tile=None, recompute=True, icond=None, device_ic=False):
        if device_ic and (initial is not None or not init_solver):
            # checked before any host IC work: the device IC overwrites X/XN and the host copy
            raise ValueError("device_ic computes the IC (the default Params', or icond=) on an initialised "
                             "solver: it cannot be combined with initial= or init_solver=False")
        L1, L2, L3 = L
        self.lib = L_ = lib()
        self.grid = pft_grid()
        rc = L_.pft_grid_init(C.byref(self.grid), n1, n2, total_n3, nprocs, rank, L1, L2, L3, calc_mode)
        if rc:
            raise ValueError(f"pft_grid_init failed ({rc})")
        self.params = np.ascontiguousarray(params, dtype=np.float64)
        if L_.pft_model_configure(C.byref(self.grid), _dp(self.params)):
            raise ValueError("pft_model_configure failed")
        g = self.grid
        self.N = (g.n3 + 4, g.n2 + 4, g.n1 + 4)
        self.S = int(np.prod(self.N))
        self.x = np.zeros(3 * self.S)
        # where the IC is computed: "device" (f1: the default IC, or icond programs that compile for
        # the device, pft_ic_compile), else "host"
        self.ic_where = "host"
        if device_ic and icond is not None:
            ok = []
            for q, prog in icond:
                ops = np.array([o for o, _ in prog], dtype=np.int32)
                args = np.array([a for _, a in prog], dtype=np.float64)
                ok.append(L_.pft_ic_device_ok(C.byref(self.grid), len(prog), _ip(ops), _dp(args)))
            if any(v < 0 for v in ok):
                raise ValueError(f"pft_ic_device_ok: a bad icond program ({ok})")
            device_ic = all(v == 1 for v in ok)   # one that is not device-exact: all on the host
        if device_ic:
            self.ic_where = "device"
        if icond is not None and device_ic:
            pass                # the programs run on the device after RK_MPI_SA_init (below)
        elif icond is not None:
            # the parameter file's icond formulas, compiled by frontend.py (intertrack.c:1831-2012)
            for q, prog in icond:
                ops = np.array([o for o, _ in prog], dtype=np.int32)
                args = np.array([a for _, a in prog], dtype=np.float64)
                rc = L_.pft_ic_eval(C.byref(self.grid), q, len(prog), _ip(ops), _dp(args), _dp(self.x))
                if rc:
                    raise ValueError(f"pft_ic_eval failed ({rc})")
        elif initial is None:
            if not device_ic:   # (device_ic: computed on the device below, then downloaded)
                L_.pft_model_ic_default(_dp(self.x))
        else:
            self.set_interior(initial)
        nch = 3 * g.n2 * g.n3
        self.chunk_start = np.zeros(nch, dtype=np.int32)
        self.chunk_size = np.zeros(nch, dtype=np.int32)
        self.chunk_mult = np.zeros(nch, dtype=np.float64)
        L_.pft_model_chunks(_ip(self.chunk_start), _ip(self.chunk_size), _dp(self.chunk_mult))
        self.mem = RK_MEM_DIST(nch, _ip(self.chunk_start), _ip(self.chunk_size), _dp(self.chunk_mult))
        meta = {1: "mf_single"}.get(nprocs) or ("mf_bottom" if rank == 0 else
                                                ("mf_top" if rank == nprocs - 1 else "mf_middle"))
        self.meta_addr = C.cast(getattr(L_, meta), C.c_void_p).value
        self.system = RK_MPI_S_SOLUTION(C.pointer(self.mem), t0, _dp(self.x), self.meta_addr, tau,
                                        tau_min, delta, DELTA_GLOBAL, None, None, 0, 0)
        L_.pft_solver_set_option(PFT_OPT_GL_STATIC, 1 if gl_static else 0)
        L_.pft_solver_set_option(PFT_OPT_KZ, kz or 0)   # 0: automatic
        L_.pft_solver_set_option(PFT_OPT_TILE, 1 if tile is None else tile)   # 1: per stage
        L_.pft_solver_set_option(PFT_OPT_RECOMPUTE, 1 if recompute else 0)
        self.initialised = False
        if L_.AllocPrecalcData():
            raise RuntimeError("AllocPrecalcData failed")
        if beads is not None and initial is None:   # (also after icond formulas)
            b = np.ascontiguousarray(beads, dtype=np.float64)
            L_.pft_model_set_beads(_dp(b), b.shape[0])
            # device_ic: the beads are overlaid on the device (pft_solver_ic_default_device)
            L_.pft_model_set_solution(None if device_ic else _dp(self.x))
        else:
            L_.pft_model_set_solution(None)
        if L_.PrecalculateData(_dp(self.chunk_mult)):
            raise RuntimeError("PrecalculateData failed")
        if init_solver:
            rc = L_.RK_MPI_SA_init(3 * self.S, MPI_COMM_WORLD, 0)
            if rc:
                raise RuntimeError(f"RK_MPI_SA_init failed ({rc})")
            self.initialised = True
            rc = L_.RK_MPI_SA_check_mem(C.byref(self.mem))
            if rc:
                raise RuntimeError(f"RK_MPI_SA_check_mem failed ({rc})")
        if device_ic:
            # f1: the default Params' IC (or the icond programs) and the beads computed on the device
            # (bit for bit the host's); the host array receives a copy, so every later call works
            # as after a host IC
            if icond is not None:
                qs = np.array([q for q, _ in icond], dtype=np.int32)
                lens = np.array([len(prog) for _, prog in icond], dtype=np.int32)
                ops = np.array([o for _, prog in icond for o, _ in prog], dtype=np.int32)
                args = np.array([a for _, prog in icond for _, a in prog], dtype=np.float64)
                rc = L_.pft_solver_ic_formulas_device(len(icond), _ip(qs), _ip(lens), _ip(ops), _dp(args),
                                                      1 if beads is not None else 0)
            else:
                rc = L_.pft_solver_ic_default_device(1 if beads is not None else 0)
            if rc:
                raise RuntimeError(f"pft_solver_ic_default_device failed ({rc}): {L_.pft_hip_last_error()}")
            if L_.pft_solver_download(C.byref(self.system)):
                raise RuntimeError("pft_solver_download failed")

    # -- host array views ------------------------------------------------------------------
    def padded(self):
        return self.x.reshape((3,) + self.N)

    def interior(self):
        g = self.grid
        return np.ascontiguousarray(self.padded()[:, 2:2 + g.n3, 2:2 + g.n2, 2:2 + g.n1])

    def set_interior(self, a):
        """a: this slab's interior [3][n3][n2][n1], or the global [3][total_n3][n2][n1]"""
        g = self.grid
        if a.shape[1] != g.n3:
            a = a[:, g.first_row:g.first_row + g.n3]
        self.padded()[:, 2:2 + g.n3, 2:2 + g.n2, 2:2 + g.n1] = a

    # -- solving ---------------------------------------------------------------------------
    def solve(self, final_time):
        rc = self.lib.RK_MPI_SA_solve(final_time, C.byref(self.system))
        if rc < 0:
            raise RuntimeError(f"RK_MPI_SA_solve failed ({rc}): {self.lib.pft_hip_last_error()}")
        return rc

    def solve_ex(self, final_time, max_steps_total=0, flags=0):
        rc = self.lib.pft_solve_ex(final_time, C.byref(self.system), max_steps_total, flags)
        if rc < 0:
            raise RuntimeError(f"pft_solve_ex failed ({rc}): {self.lib.pft_hip_last_error()}")
        return rc

    def download(self):
        rc = self.lib.pft_solver_download(C.byref(self.system))
        if rc:
            raise RuntimeError(f"pft_solver_download failed ({rc})")

    def tile_geometry(self):
        """{stage: (kernel kind, wx cell pairs, ty rows)} of the slab's stage launches (kind 0 cache,
        1 LDS tile with aux arrays, 2 fused recompute); the slab exists after the first solve"""
        slab = self.lib.pft_solver_slab()
        if not slab:
            return None
        out = {}
        for st in range(1, 6):
            wx, ty = C.c_int(), C.c_int()
            kind = self.lib.pft_slab_tile_geometry(slab, st, C.byref(wx), C.byref(ty))
            out[st] = (kind, wx.value, ty.value)
        return out

    def stats(self):
        s = pft_solver_stats()
        self.lib.pft_solver_get_stats(C.byref(s))
        return s

    @property
    def t(self):
        return self.system.t

    @property
    def h(self):
        return self.system.h

    def close(self):
        if self.initialised:
            self.lib.RK_MPI_SA_cleanup()
            self.initialised = False
        self.lib.FreePrecalcData()


def snapshot_info(t, tau, final_time, delta, calc_mode, snapshot=0, total_snapshots=0, comment=""):
    """pft_snapshot_info; its title is the reference's "Intertrack simulation (<comment>). Time: <t>"."""
    info = pft_snapshot_info(t, tau, final_time, delta, snapshot, total_snapshots, calc_mode)
    info.title = ("Intertrack simulation (%s). Time: %g" % (comment, t)).encode()[:255]   # C's %g
    return info


def save_snapshot(sim, path, info):
    """Write this slab's part of a NetCDF-classic snapshot (pft_io.h); the host array must hold the
    state (Simulation.download() after a device-resident solve).  Multi-rank: every rank calls it."""
    rc = lib().pft_snapshot_write(os.fsencode(path), C.byref(sim.grid), _dp(sim.params), C.byref(info), _dp(sim.x))
    if rc:
        raise OSError(f"pft_snapshot_write({path}) failed ({rc})")


def read_snapshot_info(path):
    """(n1, n2, total_n3, pft_snapshot_info, params[PFT_PARAM_COUNT]) of a snapshot dataset"""
    n1, n2, n3 = C.c_int(), C.c_int(), C.c_int()
    info = pft_snapshot_info()
    prm = np.full(len(PARAM_NAMES), np.nan)
    rc = lib().pft_snapshot_read_info(os.fsencode(path), C.byref(n1), C.byref(n2), C.byref(n3), C.byref(info), _dp(prm))
    if rc:
        raise OSError(f"pft_snapshot_read_info({path}) failed ({rc})")
    return n1.value, n2.value, n3.value, info, prm


def load_snapshot(sim, path):
    """Fill this slab's interior from a snapshot dataset (restart / icond_file, intertrack.c:2040-2069)"""
    rc = lib().pft_snapshot_read_slab(os.fsencode(path), C.byref(sim.grid), _dp(sim.x))
    if rc:
        raise OSError(f"pft_snapshot_read_slab({path}) failed ({rc})")


def rhs(sim, t, state_padded=None):
    """K = f(t, w) through the model's RHS meta-pointer (equation.c contract) on host arrays."""
    L_ = sim.lib
    w = sim.x.copy() if state_padded is None else np.ascontiguousarray(state_padded, dtype=np.float64)
    dw = np.zeros_like(w)
    fname = "f_generic_model2" if sim.grid.calc_mode == 2 else "f_generic_model01"
    getattr(L_, fname)(t, _dp(w), _dp(dw))
    return dw, w
