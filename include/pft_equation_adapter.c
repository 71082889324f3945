/*
 * pft_equation_adapter.c -- drop-in replacement for apps/intertrack-hybrid-S-freezing/equation.c.
 *
 * The reference driver pulls its model in textually (intertrack.c:633 `#include "equation.c"`),
 * so the model reads the driver's statics.  Switching the driver to libpft is one changed line,
 *
 *     #include "pft_equation_adapter.c"        (was: #include "equation.c")
 *
 * plus the link line of INTEGRATION.md (libpft.so instead of RK_MPI_SAsolver_hybrid2.o, and
 * -DPFT_USE_MPI -I<repo>/include so that RK_MPI_SAsolver.h, intertrack.c:109, is libpft's copy).
 * Everything else in intertrack.c -- Params, IC, snapshots, the master/worker protocol, the
 * RK_MPI_SA_* calls (:2192, :2208, :2283, :2672, :2725) -- stays unchanged.
 *
 * This file only compiles in that context: it uses the driver globals of intertrack.c:233-428
 * (n1, n2, total_n3, L1, L2, L3, param[], solution, calc_mode, MPIrank, MPIprocs, MPIrankmap).
 * What it adds to the reference contract (equation.c:35-38, 266-284, 427-558, 955-973):
 *   - AllocPrecalcData() (called at :1814, after the sizes :1776-1800 and `solution` :1813) first
 *     hands the driver's grid to libpft (pft_model_configure) and creates the slab communicator:
 *     RCCL over xGMI in VIRTUAL rank order (slab r talks to r-1 and r+1), its unique id broadcast
 *     over the driver's MPI_COMM_WORLD from the master, as intertrack.c:544 broadcasts commands;
 *   - PrecalculateData() (:646) reads the glass-bead file like equation.c:474-506 (every rank
 *     reads it instead of rank 0 + MPI_Bcast);
 *   - RK_MPI_SA_init()'s master argument is the master's REAL rank (intertrack.c:246); libpft's
 *     communicator is in virtual order, where the master is always 0;
 *   - RK_MPI_SA_cleanup() also releases the communicator.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include "pft_model.h"
#include "pft_solver.h"
#include "pft_comm.h"

/* equation.c:38 -- read by the driver (:1555, :1776-1800); libpft's host layout uses 2 */
static int bcond_thickness = PFT_BCOND_THICKNESS;

/* equation.c:35 */
static const char * pft_ball_positions_file = "data/spheres_positions.txt";

static pft_comm * pft_adapter_comm = NULL;

static int pft_adapter_comm_init(void)
{
	/* [0]: the master's status, [1..128]: the RCCL unique id.  The master broadcasts even when it
	   has no id, and every rank agrees that it has a device before the (collective, blocking) RCCL
	   init: a rank that cannot take part makes all of them fail here, as the driver's
	   CheckErrorAcrossRanks after AllocPrecalcData (intertrack.c:1814-1826) expects, instead of
	   leaving the others blocked in MPI_Bcast or ncclCommInitRank. */
	char msg[1 + 128];
	int ndev = 0, ok = 0, i;
	if(MPIprocs == 1) return pft_comm_init_self(&pft_adapter_comm) ? 1 : 0;
	memset(msg, 0, sizeof(msg));
#ifdef PFT_ADAPTER_TEST_UID
	/* test hook (tests/test_adapter.py runs the driver on CPU-only hosts, where RCCL has no id) */
	if(MPIrank == 0) { for(i = 0; i < 128; i++) msg[1 + i] = (char)(i * 37 + 11); msg[0] = 1; }
#else
	if(MPIrank == 0) msg[0] = pft_comm_get_unique_id(msg + 1) == 0;
#endif
	MPI_Bcast(msg, (int)sizeof(msg), MPI_BYTE, MPIrankmap[0], MPI_COMM_WORLD);
	if(getenv("PFT_ADAPTER_TRACE")) {
		unsigned long h = 5381;
		for(i = 1; i <= 128; i++) h = h * 33 + (unsigned char)msg[i];
		fprintf(stderr, "pft_adapter: rank %d of %d: master status %d, unique id digest %016lx\n", MPIrank,
		        MPIprocs, msg[0], h);
	}
	if(!msg[0]) {
		fprintf(stderr, "pft_adapter: rank %d: the master has no RCCL unique id (%s)\n", MPIrank, pft_hip_last_error());
		return 1;
	}
	ok = pft_hip_device_count(&ndev) == 0 && ndev >= 1;
	MPI_Allreduce(MPI_IN_PLACE, &ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
	if(!ok) {
		fprintf(stderr, "pft_adapter: rank %d: no HIP device on %s rank\n", MPIrank, ndev >= 1 ? "another" : "this");
		return 1;
	}
	{
		/* PFT_ADAPTER_TRANSPORT=ipc-ce (or ipc): every rank on ONE node, the exchange over IPC-mapped
		   slabs -- on the copy engines beside the interior launch with ipc-ce;
		   the shared-memory name comes from the master.  Default: RCCL, which also spans nodes. */
		const char * tr = getenv("PFT_ADAPTER_TRANSPORT");
		if(tr && (strcmp(tr, "ipc-ce") == 0 || strcmp(tr, "ipc") == 0)) {
			char name[64];
			int rc;
			memset(name, 0, sizeof(name));
			if(MPIrank == 0) snprintf(name, sizeof(name), "/pft_adapter_%ld", (long)getpid());
			MPI_Bcast(name, (int)sizeof(name), MPI_CHAR, MPIrankmap[0], MPI_COMM_WORLD);
			rc = pft_comm_init_ipc(&pft_adapter_comm, MPIprocs, MPIrank, name, MPIrank % ndev);
			if(!rc && strcmp(tr, "ipc-ce") == 0) rc = pft_comm_set_copy_engine(pft_adapter_comm, 1);
			if(rc) return 1;
			return pft_comm_set_current(pft_adapter_comm) ? 1 : 0;
		}
	}
	/* one process per GPU, ranks packed per node */
	if(pft_comm_init_rccl(&pft_adapter_comm, MPIprocs, MPIrank, msg + 1, MPIrank % ndev)) return 1;
	return pft_comm_set_current(pft_adapter_comm) ? 1 : 0;
}

static int pft_adapter_alloc(void)
{
	pft_grid g;
	if(pft_grid_init(&g, n1, n2, total_n3, MPIprocs, MPIrank, L1, L2, L3, calc_mode)) return 1;
	if(pft_model_configure(&g, param)) return 1;
	if(pft_model_set_solution(solution)) return 1;
	if(pft_adapter_comm_init()) return 1;
	return AllocPrecalcData();
}

static int pft_adapter_precalc(FLOAT * var_eps_mult)
{
	if(pft_model_load_beads(pft_ball_positions_file) < 0) return 1;
	return PrecalculateData(var_eps_mult);
}

static int pft_adapter_cleanup(void)
{
	int rc = RK_MPI_SA_cleanup();
	if(pft_adapter_comm) {
		pft_comm_set_current(NULL);
		pft_comm_destroy(pft_adapter_comm);
		pft_adapter_comm = NULL;
	}
	return rc;
}

/* the driver's calls below this point reach the adapter */
#define AllocPrecalcData() pft_adapter_alloc()
#define PrecalculateData(m) pft_adapter_precalc(m)
/* libpft's communicator stands for the driver's MPI_COMM_WORLD; its handle is MPICH's value, passed
   as such whatever the MPI library's MPI_Comm type is */
#define RK_MPI_SA_init(size, comm, master) RK_MPI_SA_init((size), (MPI_Comm)(long)0x44000000, 0)
#define RK_MPI_SA_cleanup() pft_adapter_cleanup()
