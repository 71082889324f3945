"""libpft against the reference's OWN solver header (CPU, build container only).

The reference driver (intertrack.c) cannot be compiled here: it includes <netcdf.h>, which the
image lacks, and the task forbids stand-in headers for building reference code (DESIGN.md
section 7).  What the driver needs from libpft is the solver ABI of
/root/reference/include/RK_MPI_SAsolver.h (its calls at intertrack.c:2192, 2208, 2283, 2672,
2725) and the equation.c model contract (include/pft_equation_adapter.c, tests/test_adapter.py).
This test compiles a small program against the reference header IN PLACE (with MPICH's mpi.h, as
the driver is built), takes the address of every solver entry point with the reference's own
prototype types, calls the host-only ones, and links it against libpft.so; a second program does
the same through libpft's header.  Both print the struct layouts and macro values, which must
agree field for field.  Nothing from /root/reference is copied."""
import os
import subprocess

import pytest

import _oracle as O

REPO = O.REPO
REF_INC = "/root/reference/include"
MPI_INC = "/opt/conda/include"
LIBDIR = os.path.join(REPO, "porousfreezethaw_amd", "lib")

PROG = r'''
#include <stddef.h>
#include <stdio.h>
#include "RK_MPI_SAsolver.h"
/* every solver entry point through the prototype types of the header above */
static int (*p_init)(int, MPI_Comm, int) = RK_MPI_SA_init;
static int (*p_cleanup)(void) = RK_MPI_SA_cleanup;
static void (*p_handle)(int) = RK_MPI_SA_handle_NAN;
static int (*p_check_nan)() = RK_MPI_SA_check_NAN;
static int (*p_check_mem)(RK_MEM_DIST *) = RK_MPI_SA_check_mem;
static int (*p_solve)(FLOAT, RK_MPI_S_SOLUTION *) = RK_MPI_SA_solve;
int main(void)
{
	RK_MEM_DIST md = { 0, NULL, NULL, NULL };
	RK_MPI_S_SOLUTION s;
	printf("FLOAT %zu\n", sizeof(FLOAT));
	printf("RK_MEM_DIST %zu %zu %zu %zu %zu\n", sizeof(RK_MEM_DIST), offsetof(RK_MEM_DIST, n_chunks),
	       offsetof(RK_MEM_DIST, chunk_start), offsetof(RK_MEM_DIST, chunk_size), offsetof(RK_MEM_DIST, chunk_eps_mult));
	printf("RK_MPI_S_SOLUTION %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(RK_MPI_S_SOLUTION),
	       offsetof(RK_MPI_S_SOLUTION, n), offsetof(RK_MPI_S_SOLUTION, t), offsetof(RK_MPI_S_SOLUTION, x),
	       offsetof(RK_MPI_S_SOLUTION, meta_f), offsetof(RK_MPI_S_SOLUTION, h), offsetof(RK_MPI_S_SOLUTION, h_min),
	       offsetof(RK_MPI_S_SOLUTION, delta), offsetof(RK_MPI_S_SOLUTION, delta_mode),
	       offsetof(RK_MPI_S_SOLUTION, DDLBF_Rearrange), offsetof(RK_MPI_S_SOLUTION, Service_Callback),
	       offsetof(RK_MPI_S_SOLUTION, steps), offsetof(RK_MPI_S_SOLUTION, steps_total));
	printf("sizeof_delta_mode %zu DELTA %d %d\n", sizeof(s.delta_mode), (int)DELTA_LOCAL, (int)DELTA_GLOBAL);
	printf("RKA_CMD %d %d %d %d %d %d\n", RKA_CMD_h_TOO_SMALL, RKA_CMD_NAN, RKA_CMD_UPDATE, RKA_CMD_FINISHED,
	       RKA_CMD_NEXTFINISH, RKA_CMD_BREAK);
	/* host-only entry points, as a driver calls them before RK_MPI_SA_init (no device needed) */
	p_handle(1);
	printf("calls %d %d %d\n", p_cleanup(), p_check_nan(), p_check_mem(&md));
	return (p_init && p_solve) ? 0 : 1;
}
'''


def _run(tmp, tag, flags):
    src = os.path.join(tmp, f"{tag}.c")
    exe = os.path.join(tmp, tag)
    with open(src, "w") as f:
        f.write(PROG)
    cmd = ["gcc", "-std=c99", "-Wall", "-Werror", "-D__GNU_SYSTEM", f"-I{MPI_INC}"] + flags + \
          [src, f"-L{LIBDIR}", "-lpft", f"-Wl,-rpath,{LIBDIR}:/usr/lib/x86_64-linux-gnu", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_libpft_links_under_reference_header(tmp_path):
    if not os.path.exists(os.path.join(REF_INC, "RK_MPI_SAsolver.h")):
        pytest.skip("the reference is not present (build container only)")
    if not os.path.exists(os.path.join(MPI_INC, "mpi.h")):
        pytest.skip("no MPI headers in this image")
    if not os.path.exists(os.path.join(LIBDIR, "libpft.so")):
        pytest.skip("libpft not built")
    ref = _run(str(tmp_path), "ref_abi", [f"-I{REF_INC}"])
    ours = _run(str(tmp_path), "pft_abi", ["-DPFT_USE_MPI", f"-I{os.path.join(REPO, 'include')}"])
    assert ref == ours, (ref, ours)
    # before RK_MPI_SA_init: cleanup -3 and check_mem -3 (hybrid2.c:130, :191), no NaN recorded
    assert "calls -3 0 -3" in ref
