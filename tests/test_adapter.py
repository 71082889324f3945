"""The drop-in boundary as the reference driver sees it.

tests/adapter/mock_intertrack.c stands where intertrack.c stands: the driver statics the model
file reads, `#include "pft_equation_adapter.c"` in place of equation.c (intertrack.c:633), and the
driver's call sequence (AllocPrecalcData, PrecalculateData, chunk table, RK_MPI_SA_init /
check_mem / solve / cleanup).  CPU: it compiles and links against libpft with MPI's headers.
GPU: run on the default Params at 10x10x20 to t = 36 s it must reproduce the reference's
trajectory (golden g20, produced by the reference itself) bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

import _oracle as O

REPO = O.REPO
SRC = os.path.join(REPO, "tests", "adapter", "mock_intertrack.c")
LIBDIR = os.path.join(REPO, "porousfreezethaw_amd", "lib")
MPI_INC, MPI_LIB = "/opt/conda/include", "/opt/conda/lib"


def _build(tmp, extra=()):
    if not os.path.exists(os.path.join(MPI_INC, "mpi.h")):
        pytest.skip("no MPI headers in this image")
    if not os.path.exists(os.path.join(LIBDIR, "libpft.so")):
        pytest.skip("libpft not built")
    exe = os.path.join(tmp, "mock_intertrack" + "".join(e.replace("-D", "_") for e in extra))
    # the system libstdc++ must win over the MPI distribution's older copy (ROCm needs it)
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-Wno-unused-variable", "-DPFT_USE_MPI", *extra,
           f"-I{MPI_INC}", f"-I{os.path.join(REPO, 'include')}", SRC, f"-L{LIBDIR}", "-lpft",
           os.path.join(MPI_LIB, "libmpi.so"),
           f"-Wl,-rpath,{LIBDIR}:/usr/lib/x86_64-linux-gnu:{MPI_LIB}", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return exe


def test_adapter_compiles_into_driver(tmp_path):
    _build(str(tmp_path))


MPIRUN = "/opt/conda/bin/mpirun"


def _driver_args(exe, tmp_path):
    meta, A = O.load_case("g20")
    P, info = O.params_from_meta(meta)
    (tmp_path / "params.txt").write_text("".join(float(v).hex() + "\n" for v in P))
    (tmp_path / "data").mkdir(exist_ok=True)
    (tmp_path / "data" / "spheres_positions.txt").write_text(
        "".join("%.17g %.17g %.17g\n" % tuple(b) for b in O.beads()))
    h = lambda v: float(v).hex()  # noqa: E731
    return [exe, "params.txt", str(info["n1"]), str(info["n2"]), str(info["n3"]), h(info["L1"]),
            h(info["L2"]), h(info["L3"]), "0", h(1.0), h(info["tau_min"]), h(info["delta"]),
            h(meta["traj_times"][0]), "out.bin"]


@pytest.mark.parametrize("test_uid", [True, False])
def test_adapter_multirank_without_device_fails_cleanly(tmp_path, test_uid):
    """The adapter's multi-rank branch (pft_equation_adapter.c: the RCCL unique id broadcast over the
    driver's MPI_COMM_WORLD) under `mpirun -np 2` on a host without a GPU: with a fixed id from the
    master (test hook) both ranks receive the same 128 bytes, then agree that a rank has no device
    and fail -- the driver's AllocPrecalcData error -- instead of blocking in RCCL's init; without
    the hook RCCL gives the master no id, which every rank learns from the broadcast.  Either way
    the run ends, well within the timeout."""
    import glob
    if not os.path.exists(MPIRUN):
        pytest.skip("no mpirun in this image")
    import porousfreezethaw_amd as PA
    if PA.device_count() > 0:
        pytest.skip("a GPU is visible: this test covers the no-device failure path")
    exe = _build(str(tmp_path), ("-DPFT_ADAPTER_TEST_UID",) if test_uid else ())
    # the RCCL transport named explicitly: its missing unique id is the failure the no-hook case
    # exercises (the default, auto, needs no id on one node and fails on the device check instead)
    env = dict(os.environ, PFT_ADAPTER_TRACE="1", OMP_NUM_THREADS="1", PFT_ADAPTER_TRANSPORT="rccl")
    r = subprocess.run([MPIRUN, "-np", "2"] + _driver_args(exe, tmp_path), cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    trace = [l for l in r.stderr.splitlines() if "unique id digest" in l]
    assert len(trace) == 2, r.stderr
    digests = {l.split()[-1] for l in trace}
    assert len(digests) == 1                                   # the same 128 bytes on both ranks
    status = {l.split("master status")[1].split(",")[0].strip() for l in trace}
    if test_uid:
        assert status == {"1"}
        assert sum("no HIP device" in l for l in r.stderr.splitlines()) == 2, r.stderr
    else:
        assert status == {"0"}
        assert sum("has no RCCL unique id" in l for l in r.stderr.splitlines()) == 2, r.stderr
    assert "AllocPrecalcData failed" in r.stderr
    assert not glob.glob(str(tmp_path / "out.bin"))


@pytest.mark.gpu
def test_adapter_driver_reproduces_reference_trajectory(tmp_path):
    exe = _build(str(tmp_path))
    meta, A = O.load_case("g20")
    P, info = O.params_from_meta(meta)
    (tmp_path / "params.txt").write_text("".join(float(v).hex() + "\n" for v in P))
    (tmp_path / "data").mkdir()
    (tmp_path / "data" / "spheres_positions.txt").write_text(
        "".join("%.17g %.17g %.17g\n" % tuple(b) for b in O.beads()))
    T = meta["traj_times"][0]
    h = lambda v: float(v).hex()  # noqa: E731
    args = [exe, "params.txt", str(info["n1"]), str(info["n2"]), str(info["n3"]), h(info["L1"]),
            h(info["L2"]), h(info["L3"]), "0", h(1.0), h(info["tau_min"]), h(info["delta"]), h(T), "out.bin"]
    r = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    raw = (tmp_path / "out.bin").read_bytes()
    line, body = raw.split(b"\n", 1)
    t, hh, s, st, rc = line.decode().split()
    ref = meta["traj_m0"][0]
    assert (float.fromhex(t), float.fromhex(hh), int(s), int(st), int(rc)) == (
        float.fromhex(ref[0]), float.fromhex(ref[1]), ref[2], ref[3], ref[4])
    x = np.frombuffer(body, dtype=np.float64).reshape(A["traj_m0_state0"].shape)
    assert np.array_equal(A["traj_m0_ic"], A["ic"])           # the driver starts from the default IC
    assert np.array_equal(x, A["traj_m0_state0"])


def test_adapter_auto_without_device_fails_cleanly(tmp_path):
    """The default transport (auto, the bench's rule) under `mpirun -np 2` on a host without a GPU:
    no RCCL id is needed on one node, so the ranks get as far as the device check, agree that a
    rank has no device and fail together."""
    if not os.path.exists(MPIRUN):
        pytest.skip("no mpirun in this image")
    import porousfreezethaw_amd as PA
    if PA.device_count() > 0:
        pytest.skip("a GPU is visible: this test covers the no-device failure path")
    exe = _build(str(tmp_path))
    env = dict(os.environ, PFT_ADAPTER_TRACE="1", OMP_NUM_THREADS="1")
    env.pop("PFT_ADAPTER_TRANSPORT", None)
    r = subprocess.run([MPIRUN, "-np", "2"] + _driver_args(exe, tmp_path), cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert sum("no HIP device" in l for l in r.stderr.splitlines()) == 2, r.stderr
    assert "AllocPrecalcData failed" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["auto", "ipc-ce"])
def test_adapter_mpirun_two_ranks_reproduce_reference(tmp_path, transport):
    """The drop-in as `mpirun -np 2 ./intertrack` runs it: the mock driver with the adapter, two MPI
    ranks on this box's GPU, the adapter's default transport (auto: both ranks share the GPU, so the
    IPC-mapped slabs with the put kernel) and the copy-engine one forced.  The two Z-slabs together
    must be the reference's 10x10x20 trajectory to t = 36 s (golden g20) bit for bit, with the
    reference's t, h and step counts on both ranks."""
    if not os.path.exists(MPIRUN):
        pytest.skip("no mpirun in this image")
    exe = _build(str(tmp_path))
    meta, A = O.load_case("g20")
    env = dict(os.environ, PFT_ADAPTER_TRACE="1", OMP_NUM_THREADS="1", PFT_IPC_TIMEOUT="60")
    if transport == "auto":
        env.pop("PFT_ADAPTER_TRANSPORT", None)
    else:
        env["PFT_ADAPTER_TRANSPORT"] = transport
    r = subprocess.run([MPIRUN, "-np", "2"] + _driver_args(exe, tmp_path), cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    if transport == "auto":
        assert sum("transport ipc" in l and "ipc-ce" not in l for l in r.stderr.splitlines()) == 2, r.stderr
    ref = meta["traj_m0"][0]
    full = A["traj_m0_state0"]
    slabs = []
    for rank in range(2):
        raw = (tmp_path / f"out.bin.{rank}").read_bytes()
        line, body = raw.split(b"\n", 1)
        t, hh, s, st, rc = line.decode().split()
        assert (float.fromhex(t), float.fromhex(hh), int(s), int(st), int(rc)) == (
            float.fromhex(ref[0]), float.fromhex(ref[1]), ref[2], ref[3], ref[4])
        slabs.append(np.frombuffer(body, dtype=np.float64).reshape(3, -1, full.shape[2], full.shape[3]))
    assert np.array_equal(np.concatenate(slabs, axis=1), full)
