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
 *     hands the driver's grid to libpft (pft_model_configure) and creates the slab communicator in
 *     VIRTUAL rank order (slab r talks to r-1 and r+1): by default bench.py's rule -- on one node
 *     the IPC-mapped slabs (copy engines with a GPU per rank, the put kernel when ranks share a
 *     GPU), across nodes RCCL, whose unique id is broadcast over the driver's MPI_COMM_WORLD from
 *     the master, as intertrack.c:544 broadcasts commands; PFT_ADAPTER_TRANSPORT picks one;
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

/* the slab transport (PFT_ADAPTER_TRANSPORT = auto | rccl | ipc | ipc-ce; default auto), the rule
   bench.py's `auto` uses:
     - every rank on one node, each on a GPU of its own: ipc-ce (IPC-mapped slabs, the halo planes
       as copy-engine transfers beside the interior launch);
     - every rank on one node, some sharing a GPU: ipc (the put kernel: a local copy there);
     - ranks on several nodes: RCCL.
   "One node" is MPI_COMM_TYPE_SHARED spanning MPI_COMM_WORLD; "a GPU of its own" compares the
   GPUs' full identities (pft_hip_device_ident: PCI bus id with function, and UUID).  If an ipc
   communicator cannot be created on some rank, every rank falls back to RCCL (auto only). */
enum { PFT_TR_AUTO = 0, PFT_TR_RCCL = 1, PFT_TR_IPC = 2, PFT_TR_IPC_CE = 3 };

static int pft_adapter_transport_env(void)
{
	const char * tr = getenv("PFT_ADAPTER_TRANSPORT");
	if(!tr || !*tr || strcmp(tr, "auto") == 0) return PFT_TR_AUTO;
	if(strcmp(tr, "rccl") == 0) return PFT_TR_RCCL;
	if(strcmp(tr, "ipc") == 0) return PFT_TR_IPC;
	if(strcmp(tr, "ipc-ce") == 0) return PFT_TR_IPC_CE;
	return -1;
}

/* auto: one node? then a GPU per rank (ipc-ce) or shared GPUs (ipc); else RCCL.  Collective. */
static int pft_adapter_auto_transport(int ndev)
{
	MPI_Comm node;
	int nl = 0, one = 0, shared = 0, i;
	char * all;
	char me[PFT_DEV_IDENT_BYTES];
	if(MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node) == MPI_SUCCESS) {
		MPI_Comm_size(node, &nl);
		MPI_Comm_free(&node);
	}
	one = nl == MPIprocs;
	MPI_Allreduce(MPI_IN_PLACE, &one, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
	if(!one) return PFT_TR_RCCL;
	memset(me, 0, sizeof(me));
	if(pft_hip_device_ident(MPIrank % ndev, me, (int)sizeof(me))) me[0] = 0;
	all = (char *)calloc((size_t)MPIprocs, sizeof(me));
	if(!all) return PFT_TR_IPC;
	MPI_Allgather(me, (int)sizeof(me), MPI_CHAR, all, (int)sizeof(me), MPI_CHAR, MPI_COMM_WORLD);
	/* a rank whose identity is unknown counts as sharing (the put kernel is correct either way) */
	for(i = 0; i < MPIprocs && !shared; i++) {
		int j;
		if(!all[i * sizeof(me)]) shared = 1;
		for(j = 0; j < i && !shared; j++)
			if(strncmp(all + i * sizeof(me), all + j * sizeof(me), sizeof(me)) == 0) shared = 1;
	}
	free(all);
	return shared ? PFT_TR_IPC : PFT_TR_IPC_CE;
}

static int pft_adapter_comm_init(void)
{
	/* [0]: the master's status, [1..128]: the RCCL unique id.  The master broadcasts even when it
	   has no id, and every rank agrees that it has a device before any (collective, blocking)
	   communicator init: a rank that cannot take part makes all of them fail here, as the driver's
	   CheckErrorAcrossRanks after AllocPrecalcData (intertrack.c:1814-1826) expects, instead of
	   leaving the others blocked in MPI_Bcast or ncclCommInitRank. */
	char msg[1 + 128];
	int ndev = 0, ok = 0, i, tr = pft_adapter_transport_env();
	if(MPIprocs == 1) return pft_comm_init_self(&pft_adapter_comm) ? 1 : 0;
	if(tr < 0) {
		fprintf(stderr, "pft_adapter: rank %d: PFT_ADAPTER_TRANSPORT must be auto, rccl, ipc or ipc-ce\n", MPIrank);
		return 1;
	}
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
	if(tr == PFT_TR_RCCL && !msg[0]) {
		fprintf(stderr, "pft_adapter: rank %d: the master has no RCCL unique id (%s)\n", MPIrank, pft_hip_last_error());
		return 1;
	}
	ok = pft_hip_device_count(&ndev) == 0 && ndev >= 1;
	MPI_Allreduce(MPI_IN_PLACE, &ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
	if(!ok) {
		fprintf(stderr, "pft_adapter: rank %d: no HIP device on %s rank\n", MPIrank, ndev >= 1 ? "another" : "this");
		return 1;
	}
	if(tr == PFT_TR_AUTO) {
		tr = pft_adapter_auto_transport(ndev);
		if(getenv("PFT_ADAPTER_TRACE"))
			fprintf(stderr, "pft_adapter: rank %d: transport %s\n", MPIrank,
			        tr == PFT_TR_IPC_CE ? "ipc-ce" : (tr == PFT_TR_IPC ? "ipc" : "rccl"));
		if(tr != PFT_TR_RCCL) {
			/* the shared-memory name comes from the master; the init's outcome is agreed, and a
			   failure anywhere sends every rank to RCCL */
			char name[64];
			int rc, bad;
			memset(name, 0, sizeof(name));
			if(MPIrank == 0) snprintf(name, sizeof(name), "/pft_adapter_%ld", (long)getpid());
			MPI_Bcast(name, (int)sizeof(name), MPI_CHAR, MPIrankmap[0], MPI_COMM_WORLD);
			rc = pft_comm_init_ipc(&pft_adapter_comm, MPIprocs, MPIrank, name, MPIrank % ndev);
			if(!rc && tr == PFT_TR_IPC_CE) rc = pft_comm_set_copy_engine(pft_adapter_comm, 1);
			bad = rc != 0;
			MPI_Allreduce(MPI_IN_PLACE, &bad, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
			if(!bad) return pft_comm_set_current(pft_adapter_comm) ? 1 : 0;
			if(pft_adapter_comm) { pft_comm_destroy(pft_adapter_comm); pft_adapter_comm = NULL; }
			fprintf(stderr, "pft_adapter: rank %d: the ipc communicator failed on a rank; RCCL instead\n", MPIrank);
			if(!msg[0]) return 1;
		}
	} else if(tr == PFT_TR_IPC || tr == PFT_TR_IPC_CE) {
		char name[64];
		int rc;
		memset(name, 0, sizeof(name));
		if(MPIrank == 0) snprintf(name, sizeof(name), "/pft_adapter_%ld", (long)getpid());
		MPI_Bcast(name, (int)sizeof(name), MPI_CHAR, MPIrankmap[0], MPI_COMM_WORLD);
		rc = pft_comm_init_ipc(&pft_adapter_comm, MPIprocs, MPIrank, name, MPIrank % ndev);
		if(!rc && tr == PFT_TR_IPC_CE) rc = pft_comm_set_copy_engine(pft_adapter_comm, 1);
		if(rc) return 1;
		return pft_comm_set_current(pft_adapter_comm) ? 1 : 0;
	}
	/* RCCL: one process per GPU, ranks packed per node */
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
