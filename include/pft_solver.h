/*
 * pft_solver.h -- libpft extensions around the reference solver ABI (RK_MPI_SAsolver.h).
 *
 * RK_MPI_SA_solve() keeps the reference contract: x is a host array, mirrored host->device at
 * entry and device->host at exit.  Drivers that keep the state on the GPU across calls (the
 * benchmark, long runs with rare snapshots) use pft_solve_ex() with the flags below; the loop,
 * its arithmetic and its control decisions are exactly those of RK_MPI_SA_solve().
 */
#ifndef PFT_SOLVER_H
#define PFT_SOLVER_H

#include "RK_MPI_SAsolver.h"
#include "pft_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PFT_SOLVE_KEEP_DEVICE   1   /* leave x on the device at exit (no device->host copy) */
#define PFT_SOLVE_REUSE_DEVICE  2   /* the device already holds x from the previous call */

/* RK_MPI_SA_solve with an optional cap on attempted steps in this call (0 = none; returns 2
   when the cap stops the loop, with system->t and system->h set so that the next call
   continues the identical trajectory) and the flags above. */
int pft_solve_ex(FLOAT final_time, RK_MPI_S_SOLUTION * system, long max_steps_total, int flags);

/* copy the device-resident x back into system->x (host layout): after a pft_solve_ex call with
   PFT_SOLVE_KEEP_DEVICE, or from inside a Service_Callback on the fused path -- there the state
   lives on the device and system->x is only refreshed when solve returns, so a callback that
   reads x (a snapshot, say) downloads it first.  The reference's RKService (intertrack.c:1072-1116)
   reads only t and h. */
int pft_solver_download(RK_MPI_S_SOLUTION * system);

/* f1 (after RK_MPI_SA_init): the default Params' initial condition (Params:9-21,
   intertrack.c:1880-2010) and, with with_beads, the glass beads (PrecalculateData,
   equation.c:459-530) computed on the device straight into the solver's state, bit for bit what
   pft_model_ic_default + PrecalculateData give on the host; system->x is not written (download it
   with pft_solver_download).  The next pft_solve_ex(..., PFT_SOLVE_REUSE_DEVICE) starts from it.
   Collective when the communicator has several ranks.  0, -3 (no RK_MPI_SA_init), -1 (beads
   requested but none set) or PFT_SOLVE_DEVICE_ERROR. */
int pft_solver_ic_default_device(int with_beads);
/* f1 for any icond formulas (intertrack.c:1831-2012): nprog compiled programs in the multi-pass
   order (frontend.py icond_programs), program p for field qs[p] with lens[p] entries, concatenated
   in ops/args (pft_frontend.h), then with with_beads the glass beads, all on the device into the
   solver's state -- bit for bit pft_ic_eval + PrecalculateData on the host.  Returns 1 without
   touching the device when a program is not device-exact (pft_ic_compile; every rank decides
   alike: evaluate on the host), else as pft_solver_ic_default_device; -2 a bad program. */
int pft_solver_ic_formulas_device(int nprog, const int * qs, const int * lens, const int * ops,
                                  const double * args, int with_beads);

/* RK_MPI_SA_solve / pft_solve_ex return value added to the reference's codes
   (RK_MPI_SAsolver.h:384-392): a HIP or RCCL failure (out of device memory, a device fault, a
   lost peer).  pft_solver_last_status() gives the raw status (-1000 - hipError_t, -3000 -
   ncclResult_t, -1 host allocation) and pft_hip_last_error() the HIP error text. */
#define PFT_SOLVE_DEVICE_ERROR  (-7)
int pft_solver_last_status(void);

enum {
	PFT_OPT_GL_STATIC = 1,  /* 1: exploit dgl == 0 (equation.c:731,874): gl neither stored in K
	                           nor combined -- bit-identical results, less traffic. Default 0. */
	PFT_OPT_KZ = 2,         /* planes per workgroup z-march; 0 (default) = automatic: the z-chunk
	                           cost model of pft_slab_set_kz */
	PFT_OPT_DEVICE = 3,     /* HIP device of this thread's slab (default: current device) */
	PFT_OPT_TIMING = 4,     /* N > 0: time the stages of every N-th attempted step with HIP events
	                           (stats.stage_ms / stage_n); each timed stage adds ~3 us of
	                           event-packet overhead, so benchmarks sample (N = 10) */
	PFT_OPT_TILE = 5,       /* stage kernel: 1 (default) = automatic, 2 = LDS-tiled at any size with
	                           the automatic tile, 32 / 16 = LDS-tiled 64x8 / 32x16 tiles, 0 =
	                           cache-based kernel (pft_slab_set_tile) */
	PFT_OPT_RECOMPUTE = 6,  /* 1 (default): rebuild stage inputs from x and the K's inside the
	                           stencil, 0: materialise the aux arrays (pft_slab_set_recompute) */
	/* 7, 8: retired (the two-stream / comm-boundary N > 1 orders and the z-wavefront stage
	   schedule, measured slower: DESIGN.md section 8) */
	PFT_OPT_LAZY_ALLOC = 9, /* 1: RK_MPI_SA_init only checks its arguments and the device buffers
	                           are allocated by the first solve (host-only checks of the ABI);
	                           0 (default): RK_MPI_SA_init allocates them, as hybrid2.c:101-112
	                           allocates K1..K5 and aux, and returns -1 when that fails */
	PFT_OPT_PAIR = 10       /* stages 2+3 and 4+5 as pair kernels (pft_slab_pair: stage A evaluated
	                           inside stage B's stencil, never stored -- 21 instead of 39 doubles
	                           per cell-step, bit-identical): 1 (default) = on slabs of at least
	                           4 Ki cells per CU (1 M cells on MI355X), 2 = on any slab they fit,
	                           0 = one launch per stage */
	,
	PFT_OPT_FAIL_RHS = 11,  /* test hook: N > 0 makes the N-th device evaluation of libpft's own
	                           right-hand side on a host array (f_generic_model01/2 called by the
	                           host-staged path) fail as a device fault would; 0 (default) off */
	PFT_OPT_GATE = 12       /* gated steps (f4): 1 = on one slab with one launch per stage and no
	                           Service_Callback, the next attempted step's launches are enqueued
	                           before this step's error norm is read and run on the device's step
	                           decision, which the host checks bit for bit (pft_slab_gate_*);
	                           0 (default) = off: measured neutral at 100^3 (38.2 vs 37.4-38.5 us
	                           per attempted step) and -2% at 200^3, where the step is bound by its
	                           kernels, not by the host.  Bit-identical. */
};
int pft_solver_set_option(int opt, long value);

typedef struct {
	int path;               /* 0 none yet, 1 fused device path, 2 host-staged path */
	int nprocs, rank;
	long kernel_launches;   /* stage kernels launched by the last call */
	long steps_total;       /* attempted steps of the last call */
	double last_eps;        /* max error norm of the last attempted step */
	double stage_ms[6];     /* PFT_OPT_TIMING: summed HIP-event time of stages 1..5 */
	long stage_n[6];        /* number of timed stage executions */
	int pairs;              /* 1: the last fused call ran stages 2+3 and 4+5 as pair kernels
	                           (timed as stages 3 and 5) */
	long gated_steps;       /* attempted steps of the last call that ran as pre-enqueued gated
	                           launches (PFT_OPT_GATE) */
	long gate_misses;       /* ... that were discarded because the device's step size differed
	                           from the host's in the last bit (pow) and were launched again */
} pft_solver_stats;
int pft_solver_get_stats(pft_solver_stats * st);

/* the slab of the fused path (benchmarks / profilers); NULL before the first fused solve */
pft_slab * pft_solver_slab(void);

#ifdef __cplusplus
}
#endif
#endif
