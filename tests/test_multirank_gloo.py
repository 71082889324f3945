"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo), SURVEY 8(e).

The GPU path splits the grid into Z-slabs (intertrack.c:1776-1800), exchanges the interface
planes of every stage input with the z-neighbours (equation.c:290-326 sync_solution; libpft:
RCCL grouped send/recv, pft_comm.hip) and takes one max-allreduce of the error norm per
attempted step (RK_MPI_SAsolver_hybrid2.c:572).  Here two processes run that protocol over
torch.distributed/gloo around the CPU oracle's Merson loop, and the gathered result must equal
the reference's single-rank trajectory bit for bit (the reference is rank-count invariant,
SURVEY F6).  This is the oracle's protocol, not libpft's: libpft needs a GPU for every solve.
libpft's own cross-process path is tests/test_ipc_multiprocess.py (2-4 processes over the ipc
transport, GPU), its threads-in-one-process path the loopback cases of test_gpu_parity.py /
test_pair_gpu.py, and its RCCL calls the 1-rank self-exchange cases; the bench's gloo-side
decomposition parity check is test_bench_parity_gloo below.
"""
import ctypes as C
import os
import socket
import sys

import numpy as np
import pytest

import _oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, T, outdir, parity=None):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    import _oracle as Ow
    os.environ["OMP_NUM_THREADS"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    meta, A = Ow.load_case("g20")
    P, info = Ow.params_from_meta(meta)
    g = Ow.make_grid(info, world, rank)
    x = Ow.pad(g, A[f"traj_m{mode}_ic"])
    BT = Ow.BT
    N1, N2, N3 = g.n1 + 2 * BT, g.n2 + 2 * BT, g.n3 + 2 * BT
    n3 = g.n3

    def exchange(wp, user):
        # sync_solution: 2 interface planes of every variable to/from each z-neighbour
        w = np.ctypeslib.as_array(wp, shape=(3 * N3 * N2 * N1,)).reshape(3, N3, N2, N1)
        reqs, recv = [], []
        if rank + 1 < world:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(w[:, BT + n3 - 2:BT + n3])), rank + 1))
            buf = torch.empty((3, 2, N2, N1), dtype=torch.float64)
            reqs.append(dist.irecv(buf, rank + 1))
            recv.append((slice(BT + n3, BT + n3 + 2), buf))
        if rank > 0:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(w[:, BT:BT + 2])), rank - 1))
            buf = torch.empty((3, 2, N2, N1), dtype=torch.float64)
            reqs.append(dist.irecv(buf, rank - 1))
            recv.append((slice(0, 2), buf))
        for r in reqs:
            r.wait()
        for sl, buf in recv:
            w[:, sl] = buf.numpy()

    def allreduce(vp, user):
        t = torch.tensor([vp[0]], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vp[0] = float(t.item())

    ex, ar = Ow.EXCHANGE_FN(exchange), Ow.ALLREDUCE_FN(allreduce)
    t, h = C.c_double(0.0), C.c_double(1.0)
    s, st = C.c_long(0), C.c_long(0)
    rc = Ow.lib().pft_or_solve(C.byref(g), Ow.ptr(P), mode, T, C.byref(t), C.byref(h), info["tau_min"],
                               info["delta"], 0, Ow.ptr(x), C.byref(s), C.byref(st), 0, ex, ar, None)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), x=Ow.unpad(g, x),
             ctl=np.array([t.value, h.value, s.value, st.value, rc], dtype=np.float64))
    if parity is not None:
        # bench.py --gpus N's decomposition check, as its ranks run it: every rank hands rank 0 its
        # record (all_gather_object), rank 0 compares them with the single-slab state -- here the
        # reference's own golden state; `parity` names a rank whose state is put off by one ulp
        sys.path.insert(0, REPO)
        import json
        import bench
        mine = Ow.unpad(g, x)
        if parity == rank:
            mine.reshape(-1)[mine.size // 2] = np.nextafter(mine.reshape(-1)[mine.size // 2], np.inf)
        rec = bench.slab_record(mine, t.value, h.value, s.value, st.value, g.first_row, g.n3)
        ranks = [None] * world
        dist.all_gather_object(ranks, rec)
        if rank == 0:
            ref = meta[f"traj_m{mode}"][0]
            bad = bench.compare_records(ranks, A[f"traj_m{mode}_state0"], float.fromhex(ref[0]),
                                        float.fromhex(ref[1]), ref[2], ref[3])
            with open(os.path.join(outdir, "parity.json"), "w") as f:
                json.dump(bad, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", [0, 2])
def test_two_rank_trajectory_equals_single_rank_reference(tmp_path, mode):
    mp = pytest.importorskip("torch.multiprocessing")
    meta, A = O.load_case("g20")
    T = meta["traj_times"][0]
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), mode, T, str(tmp_path)), nprocs=world, join=True)
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    x = np.concatenate([p["x"] for p in parts], axis=1)
    ref = meta[f"traj_m{mode}"][0]
    for p in parts:
        t, h, s, st, rc = p["ctl"]
        assert (t.hex(), h.hex(), int(s), int(st), int(rc)) == (
            float.fromhex(ref[0]).hex(), float.fromhex(ref[1]).hex(), ref[2], ref[3], ref[4])
    assert np.array_equal(x, A[f"traj_m{mode}_state0"])


@pytest.mark.parametrize("perturb", [-1, 1])
def test_bench_parity_gloo(tmp_path, perturb):
    """bench.py's N > 1 self-check over gloo with 2 ranks: the gathered per-rank records equal the
    single-slab (reference) state when the run is right, and name the rank that is one ulp off
    when it is not"""
    import json
    mp = pytest.importorskip("torch.multiprocessing")
    meta, A = O.load_case("g20")
    T = meta["traj_times"][0]
    mp.spawn(_worker, args=(2, _free_port(), 0, T, str(tmp_path), perturb), nprocs=2, join=True)
    bad = json.load(open(tmp_path / "parity.json"))
    if perturb < 0:
        assert bad == []
    else:
        assert bad == [{"rank": perturb, "fields": ["sha256"]}]


def test_decomposition_matches_reference_rule():
    """libpft's pft_decompose == the oracle's restatement of intertrack.c:1780-1787 for the
    benchmark's multi-GPU shapes"""
    sys.path.insert(0, REPO)
    import porousfreezethaw_amd as P
    if not os.path.exists(P.LIB_PATH):
        pytest.skip("libpft not built")
    L = P.lib()
    for total, world in [(400, 1), (504, 2), (636, 4), (800, 8), (20, 3), (30, 4), (13, 5)]:
        first = 0
        for r in range(world):
            n3, fr = C.c_int(), C.c_int()
            L.pft_decompose(total, world, r, C.byref(n3), C.byref(fr))
            assert (n3.value, fr.value) == O.decompose(total, world, r)
            assert fr.value == first
            first += n3.value
        assert first == total


def test_bench_weak_scaling_shapes():
    """the bench's N-GPU workloads: N = 8 is the 800^3 8-way configuration of BASELINE.json"""
    sys.path.insert(0, REPO)
    import bench
    assert bench.workload(400, 1)[2] == (200, 200, 400)
    assert bench.workload(400, 8)[2] == (400, 400, 800)
    for N in (2, 4, 8):
        gn, _, (n1, n2, n3), _ = bench.workload(400, N)
        assert gn % 4 == 0 and n1 % 2 == 0                  # even n1: the LDS-tiled kernels
        assert abs(n1 * n2 * n3 / N / 16e6 - 1) < 0.01      # ~16 M cells per GPU
        assert bench.workload(400, N, "tall")[2] == (200, 200, 400 * N)
