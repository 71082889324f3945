"""CPU-only checks of libpft: the C ABI is exported, and the host-side logic (decomposition,
chunk table, boundary conditions on host arrays, initial condition, solver argument checks)
matches the reference bit for bit.  No GPU needed: nothing here launches a kernel."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

import _oracle as O
import porousfreezethaw_amd as P

HEADERS = sorted(glob.glob(os.path.join(P.REPO, "include", "*.h")))


def declared_functions():
    names = set()
    for h in HEADERS:
        if h.endswith("pft_equation_adapter.h"):
            continue
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//.*", "", src)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", src, re.M):
            line = m.group(0)
            if line.lstrip().startswith(("typedef", "return", "#")):
                continue
            names.add(m.group(1))
    return sorted(names)


def test_headers_found():
    assert any(h.endswith("RK_MPI_SAsolver.h") for h in HEADERS)
    fns = declared_functions()
    for f in P.ABI_FUNCTIONS + ["bcond_setup", "PrecalculateData", "mf_single", "pft_comm_init_rccl"]:
        assert f in fns, f


@pytest.mark.parametrize("name", declared_functions())
def test_library_exports(name):
    lib = C.CDLL(P.LIB_PATH)
    assert hasattr(lib, name), f"{name} declared in include/ but not exported by libpft.so"


@pytest.mark.parametrize("total,nprocs", [(20, 1), (20, 3), (30, 4), (400, 8), (400, 3), (7, 3)])
def test_decompose_matches_reference(total, nprocs):
    covered = 0
    for r in range(nprocs):
        assert P.decompose(total, nprocs, r) == O.decompose(total, nprocs, r)
        n3, fr = P.decompose(total, nprocs, r)
        assert fr == covered
        covered += n3
    assert covered == total


def test_float_val():
    L = P.lib()
    for s in [b"1e-6", b"293.15", b"0.052", b"4.18e3", b"-2.5E-3", b"0.03", b"1", b"273.15"]:
        assert L.pft_float_val(s) == O.lib().pft_or_float_val(s)


def _sim_from_case(meta, arrays, key, nprocs=1, rank=0, mode=None, **kw):
    Pm, info = O.params_from_meta(meta)
    mode = info["calc_mode"] if mode is None else mode
    return P.Simulation(info["n1"], info["n2"], info["n3"], (info["L1"], info["L2"], info["L3"]), mode, Pm,
                        nprocs=nprocs, rank=rank, initial=arrays[key] if key else None,
                        beads=O.beads(), init_solver=False, **kw)


def test_chunk_table_is_intertrack_layout():
    meta, A = O.load_case("ragged")
    sim = _sim_from_case(meta, A, "state", nprocs=4, rank=2)
    g = sim.grid
    N1, N2 = g.n1 + 4, g.n2 + 4
    exp = [q * sim.S + (k + 2) * N1 * N2 + (j + 2) * N1 + 2
           for q in range(3) for k in range(g.n3) for j in range(g.n2)]
    assert np.array_equal(sim.chunk_start, np.array(exp, dtype=np.int32))
    assert np.all(sim.chunk_size == g.n1) and np.all(sim.chunk_mult == 1.0)
    sim.close()


@pytest.mark.parametrize("tag", ["t0", "t1"])
def test_bcond_setup_host_bitwise(tag):
    """bcond_setup (equation.c:266-284) on host arrays, every rank of a 4-slab split, vs the
    reference's arrays after bcond_setup+sync_solution (interface ghosts come from the
    exchange, so they are copied over from the reference before comparing)."""
    meta, A = O.load_case("ragged")
    t = meta["rhs_times"][tag]
    for r in range(4):
        sim = _sim_from_case(meta, A, "state", nprocs=4, rank=r)
        ref = A[f"w4_{tag}_rank{r}"].reshape((3,) + sim.N)
        w = sim.padded()
        if r > 0:
            w[:, :2] = ref[:, :2]
        if r < 3:
            w[:, -2:] = ref[:, -2:]
        P.lib().bcond_setup(t, P._dp(sim.x))
        assert np.array_equal(w, ref), r
        sim.close()


def test_initial_condition_bitwise():
    """pft_model_ic_default + PrecalculateData glass beads vs the reference's IC (Params:9-21
    through its expression evaluator, equation.c:459-530)"""
    meta, A = O.load_case("g20")
    for nprocs in (1, 3):
        parts = []
        for r in range(nprocs):
            sim = _sim_from_case(meta, A, None, nprocs=nprocs, rank=r)
            parts.append(sim.interior())
            sim.close()
        assert np.array_equal(np.concatenate(parts, axis=1), A["ic"]), nprocs


def test_init_allocates_and_reports_no_memory():
    """RK_MPI_SA_init allocates the device buffers (hybrid2.c:101-112): on this CPU-only host
    there is no device memory, so it returns -1 and leaves the solver uninitialised; an unknown
    communicator is -4 (hybrid2.c:95)"""
    L = P.lib()
    if P.device_count() > 0:
        pytest.skip("a HIP device is visible: the no-memory case is the GPU test's")
    assert L.RK_MPI_SA_init(100, P.MPI_COMM_WORLD + 1, 0) == -4
    assert L.RK_MPI_SA_init(100, P.MPI_COMM_WORLD, 0) == -1
    assert L.pft_solver_last_status() <= -1000          # the HIP error behind it
    assert L.RK_MPI_SA_cleanup() == -3


def test_solver_argument_codes():
    L = P.lib()
    assert L.pft_solver_set_option(P.PFT_OPT_LAZY_ALLOC, 1) == 0   # argument checks only
    assert L.RK_MPI_SA_cleanup() == -3
    mem = P.RK_MEM_DIST(0, None, None, None)
    assert L.RK_MPI_SA_init(0, P.MPI_COMM_WORLD, 0) == -2
    assert L.RK_MPI_SA_init(100, P.MPI_COMM_WORLD, 5) == -4      # master rank outside the communicator
    assert L.RK_MPI_SA_init(100, P.MPI_COMM_WORLD, 0) == 0
    assert L.RK_MPI_SA_init(100, P.MPI_COMM_WORLD, 0) == -3
    assert L.RK_MPI_SA_check_mem(C.byref(mem)) == -7
    cs = np.array([0, 10, 20], dtype=np.int32)
    cz = np.array([10, 10, 10], dtype=np.int32)
    cm = np.ones(3)
    mem = P.RK_MEM_DIST(3, P._ip(cs), P._ip(cz), P._dp(cm))
    assert L.RK_MPI_SA_check_mem(C.byref(mem)) == 0
    cz[2] = 90
    assert L.RK_MPI_SA_check_mem(C.byref(mem)) == -5
    cz[2] = 10
    cs[1] = 5
    assert L.RK_MPI_SA_check_mem(C.byref(mem)) == -6
    cs[1] = 10
    cz[1] = 0
    assert L.RK_MPI_SA_check_mem(C.byref(mem)) == -6
    cz[1] = 10
    x = np.zeros(100)
    sysm = P.RK_MPI_S_SOLUTION(C.pointer(mem), 0.0, P._dp(x), C.cast(L.mf_single, C.c_void_p).value,
                               1.0, 0.0, 0.0, P.DELTA_GLOBAL, None, None, 0, 0)
    assert L.RK_MPI_SA_solve(1.0, C.byref(sysm)) == -2          # delta <= 0 on the master
    sysm.delta = 1e-3
    sysm.x = None
    assert L.RK_MPI_SA_solve(1.0, C.byref(sysm)) == -2          # x == NULL
    sysm.x = P._dp(x)
    cz[2] = 90
    assert L.RK_MPI_SA_solve(1.0, C.byref(sysm)) == -5          # last chunk beyond max_block_size
    cz[2] = 10
    assert L.RK_MPI_SA_cleanup() == 0
    assert L.RK_MPI_SA_solve(1.0, C.byref(sysm)) == -3          # not initialised
    assert L.RK_MPI_SA_check_NAN() == 0
    if P.device_count() == 0:
        # with the arguments valid, the first device allocation fails: the added code -7
        assert L.RK_MPI_SA_init(100, P.MPI_COMM_WORLD, 0) == 0
        assert L.RK_MPI_SA_solve(1.0, C.byref(sysm)) == P.PFT_SOLVE_DEVICE_ERROR
        assert L.pft_solver_last_status() <= -1000
        assert L.RK_MPI_SA_cleanup() == 0
    assert L.pft_solver_set_option(P.PFT_OPT_LAZY_ALLOC, 0) == 0


@pytest.mark.parametrize("kw", [{"initial": np.zeros((3, 10, 10, 20))}, {"init_solver": False}])
def test_device_ic_rejects_conflicting_inputs(kw):
    """device_ic overwrites X/XN and the host copy: combining it with a caller's state, icond
    formulas or an uninitialised solver is refused up front (ValueError, also under python -O)"""
    with pytest.raises(ValueError, match="device_ic"):
        P.Simulation(10, 10, 20, (1e-3, 1e-3, 2e-3), 0, np.zeros(len(P.PARAM_NAMES)), device_ic=True, **kw)


@pytest.mark.parametrize("n,local_staged,gpu_ranks,bnd,want", [
    (4 * 2 * 160000, 0, 1, 0, 1024),    # alone on its GPU, remote neighbours, compute stream: up to 1024
    (4 * 2 * 160000, 0, 1, 1, 128),     # the boundary pipeline: beside an interior launch
    (4 * 2 * 160000, 1, 2, 0, 32),      # a staged neighbour on this GPU (PFT_IPC_STAGED)
    (4 * 2 * 160000, 0, 2, 0, 32),      # N ranks per GPU, remote neighbours: bounded all the same
    (4 * 2 * 160000, 0, 4, 1, 32),
    (1000, 0, 1, 0, 4),                 # small receives: one block per 256 doubles
    (1, 1, 3, 1, 1),
])
def test_halo_wait_blocks_bound_every_layout(n, local_staged, gpu_ranks, bnd, want):
    """pft_halo_wait_blocks: the spinning workgroups of a staged receive's wait, bounded so that they
    never hold the CUs a neighbour's pair workgroup needs -- 32 whenever the GPU is shared by ranks
    (any layout: a staged neighbour on it, or N ranks per GPU with neighbours elsewhere), 128 beside
    an interior launch"""
    L = P.lib()
    L.pft_halo_wait_blocks.argtypes = [C.c_long, C.c_int, C.c_int, C.c_int]
    assert L.pft_halo_wait_blocks(n, local_staged, gpu_ranks, bnd) == want
