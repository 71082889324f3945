/*
 * RK_MPI_SAsolver.h -- drop-in C ABI of the reference's adaptive Runge-Kutta-Merson solver,
 * implemented by libpft on MI355X (porousfreezethaw_amd/csrc/rk_solver.c).
 *
 * Replaces include/RK_MPI_SAsolver.h of radixsorth/PorousFreezeThaw (shared by
 * RK_MPI_SAsolver_hybrid.h / RK_MPI_SAsolver_hybrid2.h, which are symlinks to it):
 *   types    RK_RightHandSide (:173), RK_MEM_DIST (:184-194), RK_MPI_S_SOLUTION (:196-289)
 *   macros   MPI__FLOAT (:20-27), RKA_CMD_* (:29-35)
 *   entries  RK_MPI_SA_init (:291-313), RK_MPI_SA_cleanup (:315-322),
 *            RK_MPI_SA_handle_NAN (:324-352), RK_MPI_SA_check_NAN (:354-360),
 *            RK_MPI_SA_check_mem (:362-373), RK_MPI_SA_solve (:375-392)
 * Struct layouts, field order, argument meaning and return codes are identical, so a driver
 * built against the reference header links against libpft unchanged.
 *
 * Differences a caller can observe (all documented in DESIGN.md):
 *  - MPI is not required.  Without <mpi.h> MPI_Comm is an int handle; the ranks of a multi-GPU
 *    run are the ranks of the pft communicator (pft_comm.h, RCCL over xGMI), and `comm`
 *    must be MPI_COMM_WORLD (or PFT_COMM_WORLD).
 *  - When meta_f returns one of libpft's registered device right-hand sides (pft_model.h), the
 *    whole step runs on the GPU with x mirrored host->device at entry and device->host at exit.
 *    Any other RK_RightHandSide is called on the host with host pointers (host-staged path);
 *    the stage combines, the error norm and the update still run as HIP kernels.
 */
#ifndef PFT_RK_MPI_SASOLVER_H
#define PFT_RK_MPI_SASOLVER_H

/* FLOAT (the reference's common.h:26,63-72 with _DEFAULT_FP_PRECISION == FP_DOUBLE) */
#ifndef __common
typedef double FLOAT;
#endif

#if defined(PFT_USE_MPI) || defined(MPI_VERSION)
#include <mpi.h>
#define MPI__FLOAT MPI_DOUBLE
#else
typedef int MPI_Comm;
#ifndef MPI_COMM_WORLD
#define MPI_COMM_WORLD ((MPI_Comm)0x44000000)
#endif
#endif
#define PFT_COMM_WORLD MPI_COMM_WORLD

/* commands of the master rank, may be OR-ed */
#define RKA_CMD_h_TOO_SMALL  1
#define RKA_CMD_NAN          2
#define RKA_CMD_UPDATE       4
#define RKA_CMD_FINISHED     8
#define RKA_CMD_NEXTFINISH   16
#define RKA_CMD_BREAK        32

#ifdef __cplusplus
extern "C" {
#endif

/* f(t, x, dest): fill dest (same layout as x) at every chunk position */
typedef void (*RK_RightHandSide)(FLOAT, const FLOAT *, FLOAT *);

/* which parts of x are unknowns: ascending, non-overlapping chunks */
typedef struct {
	int n_chunks;
	int * chunk_start;        /* offset of each chunk in x */
	int * chunk_size;         /* length of each chunk */
	FLOAT * chunk_eps_mult;   /* per-chunk multiplier of the error estimate */
} RK_MEM_DIST;

typedef struct __struct_RK_MPI_S_SOLUTION {
	RK_MEM_DIST * n;                                   /* chunk layout of this rank */
	FLOAT t;                                           /* current time (master) */
	FLOAT * x;                                         /* the solution, caller-owned */
	RK_RightHandSide (*meta_f)();                      /* returns the RHS for the next step */
	FLOAT h;                                           /* current step (master) */
	FLOAT h_min;                                       /* steps below this are always accepted */
	FLOAT delta;                                       /* error tolerance (master) */
	enum { DELTA_LOCAL, DELTA_GLOBAL } delta_mode;     /* per-step or per-unit-time error */
	RK_MEM_DIST * (* DDLBF_Rearrange)(RK_MEM_DIST *); /* block rearrangement hook (may be NULL) */
	int (* Service_Callback)(FLOAT, const struct __struct_RK_MPI_S_SOLUTION * const);
	long steps;                                        /* accepted steps (caller resets) */
	long steps_total;                                  /* attempted steps */
} RK_MPI_S_SOLUTION;

/* 0 ok, -1 no memory, -2 bad size, -3 already initialised, -4 communicator not initialised.
   libpft allocates the solver's device buffers here (the fused path's slab when the model is
   configured and max_block_size holds its block, else the host-staged arrays): -1 when that
   fails (HBM exhausted, or no HIP device).  -4 also for a `comm` other than MPI_COMM_WORLD. */
int RK_MPI_SA_init(int max_block_size, MPI_Comm comm, int master_rank);
/* 0 ok, -3 not initialised */
int RK_MPI_SA_cleanup(void);
void RK_MPI_SA_handle_NAN(int hN);
int RK_MPI_SA_check_NAN();
/* 0 ok, -3 not initialised, -5 beyond max_block_size, -6 bad chunk order/size, -7 no chunks */
int RK_MPI_SA_check_mem(RK_MEM_DIST * n);
/* 0 ok, 1 interrupted by Service_Callback, -2 bad system, -3 not initialised,
   -4 NaN persists (NaN handling on), -5 last chunk beyond max_block_size, -6 error on another rank,
   and one code the reference does not have: -7 device / communication failure (HIP or RCCL,
   PFT_SOLVE_DEVICE_ERROR in pft_solver.h, details from pft_solver_last_status()) */
int RK_MPI_SA_solve(FLOAT final_time, RK_MPI_S_SOLUTION * system);

#ifdef __cplusplus
}
#endif
#endif
