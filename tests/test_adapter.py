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


def _build(tmp):
    if not os.path.exists(os.path.join(MPI_INC, "mpi.h")):
        pytest.skip("no MPI headers in this image")
    if not os.path.exists(os.path.join(LIBDIR, "libpft.so")):
        pytest.skip("libpft not built")
    exe = os.path.join(tmp, "mock_intertrack")
    # the system libstdc++ must win over the MPI distribution's older copy (ROCm needs it)
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-Wno-unused-variable", "-DPFT_USE_MPI",
           f"-I{MPI_INC}", f"-I{os.path.join(REPO, 'include')}", SRC, f"-L{LIBDIR}", "-lpft",
           os.path.join(MPI_LIB, "libmpi.so"),
           f"-Wl,-rpath,{LIBDIR}:/usr/lib/x86_64-linux-gnu:{MPI_LIB}", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return exe


def test_adapter_compiles_into_driver(tmp_path):
    _build(str(tmp_path))


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
