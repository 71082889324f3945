/*
 * rk_solver.c -- libpft's RK_MPI_SAsolver ABI (include/RK_MPI_SAsolver.h): the adaptive
 * 4th-order Runge-Kutta-Merson solver of modules/RK_MPI_SAsolver_hybrid2/RK_MPI_SAsolver_hybrid2.c
 * (and its twin _hybrid), re-designed for MI355X.
 *
 * Host C.  The control logic -- step size, accept/reject, finish/next-finish, NaN retries,
 * service callback, meta-pointer refresh, return codes -- is restated line for line from
 * hybrid2.c:215-770 (citations inline); every decision uses the same fp64 expressions, so
 * trajectories are identical to the reference's.  The array work runs on the GPU:
 *
 *  - fused path (the hot path): when meta_f() returns libpft's intertrack right-hand side and
 *    the chunk table is the driver's canonical one (intertrack.c:2144-2157), x lives on the
 *    device and each attempted step is 5 fused stage kernels (pft_kernels.hip) + one 16-byte
 *    device->host read of the global error norm; with several ranks the stage outputs' boundary
 *    planes travel by RCCL while the interior planes are computed (pft_comm.h).
 *  - host-staged path: any other RK_RightHandSide is called on the host with host arrays; the
 *    stage combines, the error norm and the update run as HIP kernels over the chunk table.
 *
 * Solver state is per host thread (the reference's is per MPI process: one static instance).
 */
#include "pft_internal.h"
#include "../../include/pft_frontend.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
	int max_n;                    /* hybrid2.c:61; 0 = not initialised */
	int master;
	int handle_nan, last_nan;     /* :63-64 */
	pft_comm * self_comm;
	/* fused path */
	pft_slab * slab;
	pft_grid slab_grid;
	int slab_gls, slab_dev;
	int device_valid;             /* slab X holds the solution left by the previous call */
	/* host-staged path */
	double *d_x, *d_k1, *d_k3, *d_k4, *d_k5, *d_aux, *d_eps;
	int *d_cs, *d_cz; double * d_cm; int d_nch, d_cap;
	double *h_k, *h_aux; int h_cap;
	/* options */
	int opt_gls, opt_kz, opt_dev, opt_timing, opt_tile, opt_norecompute;
	int opt_lazy;               /* PFT_OPT_LAZY_ALLOC: device buffers at the first solve, not at init */
	int opt_pair;               /* PFT_OPT_PAIR: stages 2+3 and 4+5 as pair kernels where the slab can */
	int opt_gate;               /* PFT_OPT_GATE: gated steps on small single slabs (f4) */
	/* K1 = f(t, x) left on the device by the last fused call (its speculative stage 1, swapped in
	   on the last accepted step, or the current one after a rejection): the next call that keeps
	   x resident from the same t, with the same constants and no u_noise, starts at stage 2 */
	int k1_keep;
	double k1_t;
	pft_consts k1_c;
	pft_slab * k1_slab;
	int k1_deep;                /* ... and its far ghost planes are current: the call that left it ran
	                               the deep (pair, between slabs) exchange, not one launch per stage */
	int deep;                   /* this call runs the pair kernels on z-neighbouring slabs: every stage
	                               launch covers the whole slab and is followed by the two-plane halo
	                               exchange of its output (pft_comm_halo_deep) */
	int tstep;                  /* this attempted step's stages are timed (every opt_timing-th) */
	int last_status;            /* raw status of the last device / communication failure */
	int in_callback;            /* inside Service_Callback on the fused path (x is on the device) */
	int rhs_failed;             /* sticky: a device evaluation of libpft's RHS on a host array failed
	                               (f_generic_model01/2 cannot report it: the reference's f is void);
	                               the host-staged loop checks it after every f() */
	long fail_rhs_after, rhs_calls;   /* PFT_OPT_FAIL_RHS test hook */
	pft_solver_stats stats;
} solver_state;

static __thread solver_state R = { .slab_dev = -1, .opt_kz = 0, .opt_dev = -1, .opt_tile = 1, .opt_pair = 1, .opt_gate = 0 };

static pft_comm * comm(void)
{
	pft_comm * c = pft_comm_current();
	if(c) return c;
	if(!R.self_comm) pft_comm_init_self(&R.self_comm);
	return R.self_comm;
}

/* ---------------------------------------------------------------------------------------- */
/* lifecycle, hybrid2.c:72-212 */

static int ensure_slab(void);
static int alloc_staged(void);
static void free_staged(void);

/* the device buffers RK_MPI_SA_init allocates (hybrid2.c:101-112 allocates K1, K3, K4, K5, aux):
   the fused path's slab when the model is configured and max_block_size holds its intertrack
   block (intertrack.c:2192 passes 3 * subgridSIZE), otherwise the host-staged path's arrays */
static int alloc_at_init(void)
{
	pft_grid g;
	int rc;
	if(pft_model_get_grid(&g) == 0) {
		const long S = (g.n1 + 2L*PFT_BCOND_THICKNESS) * (g.n2 + 2L*PFT_BCOND_THICKNESS) *
		               (g.n3 + 2L*PFT_BCOND_THICKNESS);
		if(R.max_n >= PFT_VAR_COUNT*S) return ensure_slab();
	}
	rc = alloc_staged();
	return rc;
}

int RK_MPI_SA_init(int max_block_size, MPI_Comm comm_handle, int master_rank)
{
	pft_comm * c = comm();
	int rc;
	/* :95; the ranks are those of the pft communicator (pft_comm.h), which stands for the
	   driver's MPI_COMM_WORLD -- any other communicator is unknown to libpft */
	if(!c || comm_handle != PFT_COMM_WORLD) return -4;
	if(R.max_n) return -3;                                  /* :98 */
	if(max_block_size <= 0) return -2;                      /* :99 */
	if(master_rank < 0 || master_rank >= pft_comm_size(c)) return -4;
	R.max_n = max_block_size;                               /* :114-118 */
	R.last_nan = 0;
	R.master = master_rank;
	if(!R.opt_lazy && (rc = alloc_at_init())) {             /* :101-112: -1, not enough memory */
		R.last_status = rc;
		if(R.slab) { pft_comm_attach(comm(), NULL); pft_slab_destroy(R.slab); R.slab = NULL; R.k1_keep = 0; }
		free_staged();
		R.max_n = 0;
		return -1;
	}
	return 0;
}

static void free_staged(void)
{
	pft_flat_free(R.d_x); pft_flat_free(R.d_k1); pft_flat_free(R.d_k3); pft_flat_free(R.d_k4);
	pft_flat_free(R.d_k5); pft_flat_free(R.d_aux); pft_flat_free(R.d_eps);
	pft_dev_free(R.d_cs); pft_dev_free(R.d_cz); pft_flat_free(R.d_cm);
	R.d_x = R.d_k1 = R.d_k3 = R.d_k4 = R.d_k5 = R.d_aux = R.d_eps = R.d_cm = NULL;
	R.d_cs = R.d_cz = NULL; R.d_cap = 0; R.d_nch = 0;
	free(R.h_k); free(R.h_aux); R.h_k = R.h_aux = NULL; R.h_cap = 0;
}

int RK_MPI_SA_cleanup(void)
{
	if(R.max_n == 0) return -3;                             /* :130 */
	if(R.slab) { pft_comm_attach(comm(), NULL); pft_slab_destroy(R.slab); R.slab = NULL; R.k1_keep = 0; }
	free_staged();
	R.device_valid = 0;
	R.max_n = 0;                                            /* :134 */
	return 0;
}

void RK_MPI_SA_handle_NAN(int hN) { R.handle_nan = (hN == 0) ? 0 : 1; }   /* :165 */
int RK_MPI_SA_check_NAN() { return R.last_nan; }                           /* :176 */

int RK_MPI_SA_check_mem(RK_MEM_DIST * n)
{
	/* :191-211 */
	int offset = 0, prev, i;
	if(R.max_n == 0) return -3;
	if(n->n_chunks <= 0) return -7;
	for(i=0;i<n->n_chunks;i++) {
		prev = offset;
		offset = n->chunk_start[i];
		if(offset < prev) return -6;
		prev = offset;
		offset += n->chunk_size[i];
		if(offset <= prev) return -6;
	}
	if(offset > R.max_n) return -5;
	return 0;
}

int pft_solver_set_option(int opt, long value)
{
	switch(opt) {
		case PFT_OPT_GL_STATIC: R.opt_gls = value ? 1 : 0; return 0;
		case PFT_OPT_KZ: if(value < 0) return -2; R.opt_kz = (int)value; if(R.slab) pft_slab_set_kz(R.slab, R.opt_kz); return 0;
		case PFT_OPT_DEVICE: R.opt_dev = (int)value; return 0;
		case PFT_OPT_TIMING: if(value < 0) return -2; R.opt_timing = (int)value; return 0;
		case PFT_OPT_LAZY_ALLOC: R.opt_lazy = value ? 1 : 0; return 0;
		case PFT_OPT_FAIL_RHS: if(value < 0) return -2; R.fail_rhs_after = value; R.rhs_calls = 0; return 0;
		case PFT_OPT_PAIR: if(value < 0 || value > 2) return -2; R.opt_pair = (int)value; return 0;
		case PFT_OPT_GATE: if(value < 0 || value > 1) return -2; R.opt_gate = (int)value; return 0;
		case PFT_OPT_RECOMPUTE:
			R.opt_norecompute = value ? 0 : 1; if(R.slab) pft_slab_set_recompute(R.slab, !R.opt_norecompute); return 0;
		case PFT_OPT_TILE:
			if(value != 0 && value != 1 && value != 2 && value != 16 && value != 32) return -2;
			R.opt_tile = (int)value; if(R.slab) pft_slab_set_tile(R.slab, R.opt_tile); return 0;
	}
	return -2;
}

int pft_solver_get_stats(pft_solver_stats * st) { *st = R.stats; return 0; }
int pft_solver_last_status(void) { return R.last_status; }
pft_slab * pft_solver_slab(void) { return R.slab; }

/* ---------------------------------------------------------------------------------------- */
/* fused device path */

static int ensure_slab(void)
{
	pft_grid g;
	pft_consts c;
	pft_slab_desc d;
	int rc;
	if(pft_model_get_grid(&g) || pft_model_get_consts(&c)) return -2;
	if(R.slab && R.slab_grid.n1 == g.n1 && R.slab_grid.n2 == g.n2 && R.slab_grid.n3 == g.n3 &&
	   R.slab_grid.rank == g.rank && R.slab_grid.nprocs == g.nprocs && R.slab_grid.calc_mode == g.calc_mode &&
	   R.slab_gls == R.opt_gls && R.slab_dev == R.opt_dev) {
		/* parameters may change between calls: refresh the constants */
		pft_slab_set_consts(R.slab, &c);
	} else if(R.slab) {
		pft_comm_attach(comm(), NULL);
		pft_slab_destroy(R.slab); R.slab = NULL; R.device_valid = 0; R.k1_keep = 0;
	}
	if(!R.slab) {
		if(R.opt_dev >= 0 && (rc = pft_hip_set_device(R.opt_dev))) return rc;
		memset(&d, 0, sizeof(d));
		d.n1 = g.n1; d.n2 = g.n2; d.n3 = g.n3;
		d.has_below = g.rank > 0;
		d.has_above = g.rank < g.nprocs - 1;
		d.calc_mode = g.calc_mode;
		d.gl_static = R.opt_gls;
		d.eps_mult[0] = d.eps_mult[1] = d.eps_mult[2] = 1.0;
		if((rc = pft_slab_create(&R.slab, &d, &c))) return rc;
		pft_slab_set_kz(R.slab, R.opt_kz);
		pft_slab_set_tile(R.slab, R.opt_tile);
		pft_slab_set_recompute(R.slab, !R.opt_norecompute);
		R.slab_grid = g; R.slab_gls = R.opt_gls; R.slab_dev = R.opt_dev;
		R.device_valid = 0;
	}
	if((rc = pft_comm_attach(comm(), R.slab))) return rc;
	return pft_slab_set_noise(R.slab, pft_model_noise());
}

static int canonical_chunks(const RK_MEM_DIST * n, double em[3])
{
	/* the intertrack chunk table (intertrack.c:2144-2157) for the configured grid */
	pft_grid g;
	int q, k, j, c = 0;
	long N1, row, S;
	if(pft_model_get_grid(&g)) return 0;
	N1 = g.n1 + 2*PFT_BCOND_THICKNESS; row = N1*(g.n2 + 2*PFT_BCOND_THICKNESS);
	S = row*(g.n3 + 2*PFT_BCOND_THICKNESS);
	if(n->n_chunks != PFT_VAR_COUNT*g.n2*g.n3) return 0;
	for(q=0;q<PFT_VAR_COUNT;q++) {
		em[q] = n->chunk_eps_mult ? n->chunk_eps_mult[c] : 1.0;
		for(k=0;k<g.n3;k++) for(j=0;j<g.n2;j++, c++) {
			const long s0 = q*S + (k+PFT_BCOND_THICKNESS)*row + (long)(j+PFT_BCOND_THICKNESS)*N1 + PFT_BCOND_THICKNESS;
			if(n->chunk_start[c] != s0 || n->chunk_size[c] != g.n1) return 0;
			if(n->chunk_eps_mult && n->chunk_eps_mult[c] != em[q]) return 0;
		}
	}
	return R.max_n >= PFT_VAR_COUNT*S;
}

/* one stage of the step on this slab; stage 6 = the speculative stage 1 of the next step
   (K1' = f(ts, XN) into A1, pft_slab_stage_spec) */
static int run1(int stage, double ts, double coef, double h, int kb, int ke)
{
	return stage == 6 ? pft_slab_stage_spec(R.slab, ts, kb, ke) : pft_slab_stage(R.slab, stage, ts, coef, h, kb, ke);
}

static int do_stage(int stage, double ts, double coef, double h, long * launches)
{
	pft_comm * c = comm();
	const int out_buf = stage == 6 ? PFT_BUF_A1 : pft_slab_stage_output(R.slab, stage);
	const int nfields = pft_slab_stage_fields(R.slab, stage);
	const int tstage = stage == 6 ? 1 : stage;
	int rc, n3;
	if(R.tstep) pft_slab_timing_mark(R.slab, tstage, 0);
	if(R.deep) {
		/* pair path between slabs: the output's two-plane halo (the next pair kernel evaluates its
		   stage A on the ghost planes too).  RCCL and ipc on the copy engines: the two planes at each
		   end first, their exchange on the comm stream beside the interior launch; ipc with put
		   kernels: the whole slab, then the put. */
		n3 = R.slab_grid.n3;
		if(pft_comm_boundary_first(c) && n3 >= 5 && (rc = pft_slab_stage_inline(R.slab))) {
			/* one launch whose leading workgroups produce the planes the exchange sends (as do_pair) */
			if((rc = run1(stage, ts, coef, h, rc, 0))) return rc;
			if((rc = pft_comm_halo_start_deep(c, out_buf, 0, nfields))) return rc;
			if(R.tstep) pft_slab_timing_mark(R.slab, tstage, 1);
			(*launches)++;
			return pft_comm_halo_finish(c);
		}
		if(pft_comm_boundary_first(c) && n3 >= 5) {
			if((rc = run1(stage, ts, coef, h, PFT_K_BOUNDARY2, 0))) return rc;
			if((rc = pft_comm_halo_start_deep(c, out_buf, 0, nfields))) return rc;
			if((rc = run1(stage, ts, coef, h, 2, n3-2))) return rc;
			if(R.tstep) pft_slab_timing_mark(R.slab, tstage, 1);
			*launches += 2;
			return pft_comm_halo_finish(c);
		}
		(*launches)++;
		if((rc = run1(stage, ts, coef, h, -1, -1))) return rc;
		if(R.tstep) pft_slab_timing_mark(R.slab, tstage, 1);
		return pft_comm_halo_deep(c, out_buf, 0, nfields);
	}
	if(pft_comm_device_halo(c) && !pft_comm_boundary_first(c)) {
		/* ipc: the whole slab in one launch, then (stream-ordered) the boundary planes into the
		   neighbours' ghost planes and the wait for theirs in ours */
		(*launches)++;
		if((rc = run1(stage, ts, coef, h, -1, -1))) return rc;
		if(R.tstep) pft_slab_timing_mark(R.slab, tstage, 1);
		return pft_comm_halo(c, out_buf, 0, nfields);
	}
	if(!pft_comm_splits(c)) {
		(*launches)++;
		rc = run1(stage, ts, coef, h, -1, -1);
		if(R.tstep) pft_slab_timing_mark(R.slab, tstage, 1);
		return rc;
	}
	/* SURVEY 8e.  Stage s reads the stage-(s-1) values of planes -1..n3 and writes its own; only
	   its two boundary planes read ghost planes: they are launched first, exchanged on the comm
	   stream beside the interior sweep, and the compute stream waits for the exchange before the
	   next stage.  (Measured slower and removed: the boundary launch on the comm stream with the
	   interior sweep waiting for it, and two-stream orders) */
	n3 = R.slab_grid.n3;
	if((rc = run1(stage, ts, coef, h, PFT_K_BOUNDARY, 0))) return rc;
	if((rc = pft_comm_halo_start(c, out_buf, 0, nfields))) return rc;
	if(n3 > 2 && (rc = run1(stage, ts, coef, h, 1, n3-1))) return rc;
	if(R.tstep) pft_slab_timing_mark(R.slab, tstage, 1);
	*launches += 2;
	return pft_comm_halo_finish(c);
}

/* stages first, first+1 (2+3 or 4+5) of the step as ONE pair kernel (pft_slab_pair; one slab):
   timed as stage first+1 */
static int do_pair(int first, double ta, double tb, double h, double coef, long * launches)
{
	pft_comm * c = comm();
	const int out_buf = first == 2 ? PFT_BUF_K3 : PFT_BUF_XN, n3 = R.slab_grid.n3;
	int rc;
	if(R.tstep) pft_slab_timing_mark(R.slab, first+1, 0);
	if(R.deep && pft_comm_boundary_first(c) && n3 >= 5) {
		/* between slabs over RCCL or the copy engines: the two planes at each end first, their
		   exchange (K3, or x(t+h): gl only where stored) beside the interior launch, which reads no
		   ghost plane */
		const int nf = pft_slab_stage_fields(R.slab, first+1);
		const int inl = pft_slab_pair_inline(R.slab, first);
		if(inl) {
			/* one launch whose leading workgroups produce the planes the exchange sends; the copies
			   start when they are done (PFT_K_INLINE, PFT_K_ENDS_FIRST) */
			(*launches)++;
			if((rc = pft_slab_pair_range(R.slab, first, ta, tb, h, coef, inl, 0))) return rc;
			if((rc = pft_comm_halo_start_deep(c, out_buf, 0, nf))) return rc;
			if(R.tstep) pft_slab_timing_mark(R.slab, first+1, 1);
			return pft_comm_halo_finish(c);
		}
		*launches += 2;
		if((rc = pft_slab_pair_range(R.slab, first, ta, tb, h, coef, PFT_K_BOUNDARY2, 0))) return rc;
		if((rc = pft_comm_halo_start_deep(c, out_buf, 0, nf))) return rc;
		if((rc = pft_slab_pair_range(R.slab, first, ta, tb, h, coef, 2, n3-2))) return rc;
		if(R.tstep) pft_slab_timing_mark(R.slab, first+1, 1);
		return pft_comm_halo_finish(c);
	}
	(*launches)++;
	rc = pft_slab_pair(R.slab, first, ta, tb, h, coef);
	if(R.tstep) pft_slab_timing_mark(R.slab, first+1, 1);
	if(rc || !R.deep) return rc;
	/* between slabs (ipc): the whole slab, then the two-plane halo */
	return pft_comm_halo_deep(c, out_buf, 0, pft_slab_stage_fields(R.slab, first+1));
}

/* gl evolves by dgl == 0 (equation.c:731,874), so x(t+h) of gl is x + coef*0.0: x itself, bit for
   bit, unless x is -0.0 (-0.0 + 0.0 = +0.0) or NaN.  When no gl value of the uploaded state is
   either, X and XN (both uploaded from it) keep identical gl for good and stage 5 skips that store
   (pft_slab_set_gl_keep); one step turns any -0.0 into +0.0, so the check only looks at input. */
static int gl_clean(const double * x)
{
	/* host layout: [q][k][j][i] with 2 ghost cells on every side; only the interior is uploaded */
	const int n1 = R.slab_grid.n1, n2 = R.slab_grid.n2, n3 = R.slab_grid.n3;
	const long N1 = n1 + 4, N2 = n2 + 4;
	const double * g = x + 2 * N1 * N2 * (n3 + 4);
	int k, bad = 0;
	#pragma omp parallel for reduction(|:bad) schedule(static)
	for(k = 2; k < n3 + 2; k++) {
		int j, i;
		for(j = 2; j < n2 + 2; j++) {
			const double * r = g + ((long)k * N2 + j) * N1;
			for(i = 2; i < n1 + 2; i++) bad |= (r[i] != r[i]) || (r[i] == 0.0 && signbit(r[i]));
		}
	}
	return !bad;
}

/* shared prologue results */
typedef struct {
	double final_time, t, h, h_min, delta;
	int delta_mode, handle_nan, any_cb;
} solve_bcast;

static int run_staged(RK_MPI_S_SOLUTION * system, RK_RightHandSide f, solve_bcast * B, int command,
                      long max_steps_total, int flags);

/* PFT_GATE_TRACE=1: host-side timeline of the gated pipeline (stderr at the end of a call) */
static double gt_now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int run_fused(RK_MPI_S_SOLUTION * system, RK_RightHandSide f, solve_bcast * B, int command,
                     long max_steps_total, int flags, const double * em)
{
	pft_comm * c = comm();
	const int rank = pft_comm_rank(c), nprocs = pft_comm_size(c);
	double t = B->t, h = B->h, new_h = 0.0, h2, h3, h6, h8, eps;
	const double final_time = B->final_time, delta = B->delta, h_min = B->h_min;
	int nonfinite, rc, ret = 0, to_host = 0;
	long attempted = 0, launches = 0;
	int spec, k1_valid = 0;               /* K1 holds f(t, x) for the current t and x */
	int pair;                             /* stages 2+3 and 4+5 as pair kernels */
	int gate, pre = 0, acc, enq;          /* gated steps; this attempt was pre-enqueued; accepted;
	                                         the next attempt is pre-enqueued */
	unsigned long long gcur = 0, gnext;   /* decisions on this attempt (by its speculative stage 1)
	                                         and on the pre-enqueued one */

	if((rc = ensure_slab())) return rc;
	pft_slab_set_eps_mult(R.slab, em);
	/* The next step's K1 is computed speculatively right after stage 5 (recompute path): the
	   kernel runs while the host reads the error norm and decides, so the GPU does not idle
	   between steps.  Accepted: it is f(t+h, x(t+h)), exactly the next stage 1.  Rejected: x and t
	   are unchanged, so the current K1 is still exactly f(t, x) -- the reference recomputes the
	   same bits (hybrid2.c:373) -- and the speculative one is dropped. */
	spec = pft_slab_can_speculate(R.slab);
	/* pair kernels (pft_slab_pair_ok: slab size, n3 >= 2 and no u_noise between slabs); every rank
	   must take the same path -- the exchanges differ */
	pft_slab_set_pair(R.slab, R.opt_pair);
	pair = spec && pft_slab_pair_ok(R.slab);
	if(nprocs > 1) {
		long long no = !pair;
		if((rc = pft_comm_allreduce_max_i64(c, &no))) return rc;
		pair = !no;
	}
	R.deep = pair && pft_comm_splits(c);
	{
		/* K1 from the previous call (R.k1_keep): x resident and unchanged since (no upload), the
		   same slab, t, constants, and no u_noise (re-uploaded every call); for the pair kernels
		   between slabs also its far ghost planes (R.k1_deep: a call with one launch per stage
		   exchanged only the first ghost plane, and the deep prologue below re-exchanges only X
		   and XN).  Every rank takes the same decision (the same calls, flags and t). */
		pft_consts cc;
		if(spec && (flags & PFT_SOLVE_REUSE_DEVICE) && R.device_valid && R.k1_keep && R.k1_slab == R.slab &&
		   (!R.deep || R.k1_deep) && !pft_model_noise() && memcmp(&R.k1_t, &t, sizeof t) == 0 && !pft_model_get_consts(&cc) &&
		   memcmp(&cc, &R.k1_c, sizeof cc) == 0)
			k1_valid = 1;
		R.k1_keep = 0;
	}
	R.stats.pairs = pair;
	R.stats.gated_steps = 0;
	R.stats.gate_misses = 0;
	if(!(flags & PFT_SOLVE_REUSE_DEVICE) || !R.device_valid) {
		if((rc = pft_slab_upload_host(R.slab, PFT_BUF_X, system->x))) return rc;
		if((rc = pft_slab_upload_host(R.slab, PFT_BUF_XN, system->x))) return rc;
		{
			/* every rank must agree: the stage-5 exchange carries gl only when some rank stores it */
			long long unclean = !gl_clean(system->x);
			if(nprocs > 1 && (rc = pft_comm_allreduce_max_i64(c, &unclean))) return rc;
			pft_slab_set_gl_keep(R.slab, !unclean);
		}
		if(nprocs > 1 && !R.deep) {
			if((rc = pft_comm_halo(c, PFT_BUF_X, 0, 3))) return rc;
			if((rc = pft_comm_halo(c, PFT_BUF_XN, 0, 3))) return rc;
		}
	}
	if(R.deep) {
		/* two planes deep, also when x stayed on the device (the previous call may have run one
		   launch per stage, which keeps only the first ghost plane current) */
		if((rc = pft_comm_halo_deep(c, PFT_BUF_X, 0, 3))) return rc;
		if((rc = pft_comm_halo_deep(c, PFT_BUF_XN, 0, 3))) return rc;
	}
	R.device_valid = 0;
	R.stats.path = 1;
	/* the error norm goes to the host from stage 5 itself (no publish kernel, no event) where no
	   device collective sits between stage 5 and the host (one slab, or ipc); env
	   PFT_INKERNEL_PUBLISH=0 turns it off (A/B) */
	{
		const char * e = getenv("PFT_INKERNEL_PUBLISH");
		const int on = spec && (!pft_comm_splits(c) || pft_comm_device_halo(c)) &&
		               !(e && atoi(e) == 0);
		pft_slab_set_inkernel_publish(R.slab, on);
	}

	/* f4, gated steps (PFT_OPT_GATE, pft_slab_gate_*): on one slab with one launch per stage, the
	   next attempted step's launches are enqueued before this step's error norm is read, as if the
	   step were accepted.  This step's speculative stage 1 reduces the error norm and decides the
	   step on the device (hybrid2.c:578-611, the expressions below); the gated launches run on
	   that decision, so the GPU waits neither for the host's round trip nor for its launch latency.
	   The host still takes the decision below (glibc pow) and keeps the gated step only if the
	   device's (ocml pow) is the same bit for bit; otherwise that step is discarded -- it wrote only
	   buffers nothing reads afterwards (XN, A0, K3, K4, A1) -- and launched again.  Not with a
	   Service_Callback (it may read x between steps) or per-stage timing. */
	{
		/* env PFT_GATE=0/1 overrides PFT_OPT_GATE (whole-suite runs with gating forced on) */
		const char * eg = getenv("PFT_GATE");
		gate = eg ? atoi(eg) != 0 : R.opt_gate;
	}
	gate = gate && spec && !pair && nprocs == 1 && !pft_comm_splits(c) &&
	       system->Service_Callback == NULL && !R.opt_timing;
	if(gate) pft_slab_gate_config(R.slab, final_time, delta, h_min, B->delta_mode == DELTA_LOCAL, B->handle_nan);
	const int gtrace = getenv("PFT_GATE_TRACE") != NULL;
	double gt_t0 = 0.0, gt_enq = 0.0, gt_wait = 0.0, gt_dec = 0.0, gt_a, gt_b;
	long gt_n = 0;
	if(gtrace) gt_t0 = gt_now();

	while(1) {
		h2 = h/2.0; h3 = h/3.0; h6 = h/6.0; h8 = h/8.0;                          /* :355 */
		R.tstep = R.opt_timing > 0 && attempted % R.opt_timing == 0;
		acc = 0;
		if(!pre) {
			/* the error norm accumulator is reset by its publication on the speculative path */
			if((!spec || attempted == 0) && (rc = pft_slab_eps_reset(R.slab))) return rc;
			/* K1 = f(t,x); aux = x + K1 h/3 ... K5 = f(t+h, aux); error norm; x(t+h) candidate */
			if(pair) {
				/* the same arithmetic: stage A of each pair is evaluated inside stage B's stencil */
				if(!k1_valid && (rc = do_stage(1, t, h3, h, &launches))) return rc;      /* :373-389 */
				if((rc = do_pair(2, t+h3, t+h3, h, h3, &launches))) return rc;          /* :392-429 */
				if((rc = do_pair(4, t+h2, t+h, h, h3, &launches))) return rc;           /* :432-524,657-668 */
			} else {
				if(!(spec && k1_valid) && (rc = do_stage(1, t, h3, h, &launches))) return rc;  /* :373-389 */
				if((rc = do_stage(2, t+h3, h6, h, &launches))) return rc;    /* :392-409 */
				if((rc = do_stage(3, t+h3, h8, h, &launches))) return rc;    /* :412-429 */
				if((rc = do_stage(4, t+h2, h,  h, &launches))) return rc;    /* :432-450 */
				if((rc = do_stage(5, t+h,  h3, h, &launches))) return rc;    /* :453,507-524,657-668 */
			}
			k1_valid = 1;
			if(spec) {
				/* eps max over ranks (:572) and its publication beside the speculative stage 1 */
				if((rc = pft_comm_eps_publish(c))) return rc;
				if(gate) gcur = pft_slab_gate_arm(R.slab, t, h);
				if((rc = do_stage(6, t+h, 0.0, h, &launches))) return rc;
			} else {
				/* the boundary launch of stage 5 (comm stream) adds to the error norm too */
				if(pft_comm_splits(c) && (rc = pft_slab_order(R.slab, 1))) return rc;
				if((rc = pft_comm_allreduce_eps(c))) return rc;                      /* :572 */
			}
		}
		pre = 0;
		gnext = 0;
		gt_a = gtrace ? gt_now() : 0.0;
		/* pre-enqueue the next attempt unless this one ends the solve if accepted (FINISHED) or the
		   step cap stops before it */
		enq = gate && gcur && !(command & RKA_CMD_FINISHED) &&
		      !(max_steps_total > 0 && attempted + 1 >= max_steps_total);
		if(enq) {
			/* the next attempted step, enqueued now as if this one were accepted (the buffers
			   swapped as the accept below swaps them, for the enqueue only): stages 2-5 and its
			   speculative stage 1, gated on the device's decision gcur.  The scalars passed here
			   are not used: the launches derive theirs from the decided (t, h). */
			pft_slab_book_save(R.slab, 0);
			pft_slab_accept(R.slab);
			pft_slab_swap_buffers(R.slab, PFT_BUF_K1, PFT_BUF_A1);
			pft_slab_gate_use(R.slab, gcur);
			rc = 0;
			if(!rc) rc = do_stage(2, 0.0, 0.0, 0.0, &launches);
			if(!rc) rc = do_stage(3, 0.0, 0.0, 0.0, &launches);
			if(!rc) rc = do_stage(4, 0.0, 0.0, 0.0, &launches);
			if(!rc) rc = do_stage(5, 0.0, 0.0, 0.0, &launches);
			if(!rc) rc = pft_comm_eps_publish(c);
			if(!rc) gnext = pft_slab_gate_arm(R.slab, 0.0, 0.0);   /* (t, h) from its own gate */
			if(!rc) rc = do_stage(6, 0.0, 0.0, 0.0, &launches);
			pft_slab_gate_use(R.slab, 0);
			pft_slab_accept(R.slab);
			pft_slab_swap_buffers(R.slab, PFT_BUF_K1, PFT_BUF_A1);
			pft_slab_book_save(R.slab, 1);
			pft_slab_book_load(R.slab, 0);
			if(rc) return rc;
		}
		gt_b = gtrace ? gt_now() : 0.0;
		if((rc = pft_slab_eps_fetch(R.slab, &eps, &nonfinite))) return rc;
		if(gtrace) {
			const double n = gt_now();
			gt_enq += gt_b - gt_a;
			gt_wait += n - gt_b;
			gt_a = n;
			gt_n++;
		}
		if((rc = pft_comm_eps_host(c, &eps, &nonfinite))) return rc;                 /* :572 (ipc) */
		if(R.opt_timing) pft_slab_timing_collect(R.slab, R.stats.stage_ms, R.stats.stage_n);
		system->steps_total++;                                                   /* :460 */
		attempted++;
		R.stats.last_eps = eps;

		if(B->handle_nan && nonfinite) {                                         /* :493-503 */
			command |= RKA_CMD_NAN;
			if(h/(final_time-t) < 1e-11) command |= RKA_CMD_h_TOO_SMALL;
		}
		if(B->delta_mode == DELTA_LOCAL) eps *= fabs(h3);                        /* :578 */
		new_h = ((eps > 0.0) ? pow((delta/eps), 0.2)*0.8 : 2.0) * h;            /* :580 */
		if(eps < delta || fabs(h) < h_min) {                                     /* :599-611 */
			command |= RKA_CMD_UPDATE;
			if(fabs(final_time-(t+h)) <= fabs(new_h)) command |= RKA_CMD_NEXTFINISH;
		}

		if(command & RKA_CMD_NAN) {                                              /* :626-646 */
			R.last_nan = 1;
			if(command & RKA_CMD_h_TOO_SMALL) { system->t = t; ret = -4; break; }
			h /= 10;
			command = 0;
		} else {
			if(command & RKA_CMD_UPDATE) {                                       /* :651-668 */
				t += h;
				acc = 1;
				pft_slab_accept(R.slab);
				if(spec) pft_slab_swap_buffers(R.slab, PFT_BUF_K1, PFT_BUF_A1);  /* K1 = f(t, x) */
				else k1_valid = 0;
				system->steps++;
				if(system->Service_Callback != NULL) {                           /* :676-685 */
					/* x stays on the device: a callback that reads it calls
					   pft_solver_download(system) first (pft_solver.h) */
					system->t = t;
					system->h = h;
					R.in_callback = 1;
					if(system->Service_Callback(final_time, system)) command |= RKA_CMD_BREAK;
					R.in_callback = 0;
				}
				if(nprocs > 1 && B->any_cb && (rc = pft_comm_bcast(c, &command, sizeof(int), R.master))) return rc;   /* :690 */
				if(command & RKA_CMD_FINISHED) break;                            /* :695 */
				if(command & RKA_CMD_BREAK) {                                    /* :697-705 */
					system->t = t;
					system->h = new_h;
					ret = 1;
					break;
				}
				f = system->meta_f();                                            /* :732 */
				/* another right-hand side from the next step on: the state leaves the device
				   and the loop continues on the host-staged path (below) */
				if(!pft_model_is_device_rhs(f)) to_host = 1;
			}
			if(command & RKA_CMD_NEXTFINISH) {                                   /* :743-761 */
				system->h = new_h;
				h = final_time - t;
				command = RKA_CMD_FINISHED;
			} else {
				command = 0;
				h = new_h;
			}
		}
		if(max_steps_total > 0 && attempted >= max_steps_total) {
			/* extension: stop between two attempted steps; the next call continues the
			   identical trajectory (its prologue re-derives FINISHED from t, h) */
			system->h = h;
			ret = 2;
			break;
		}
		if(to_host) break;
		if(enq) {
			/* keep the pre-enqueued attempt iff the device took this decision, bit for bit:
			   accepted, and the same next t and h (its launches ran on them); otherwise it
			   exited at once (device: rejected) or ran on a different h (pow) and is discarded */
			int go = 0;
			double td = 0.0, hd = 0.0;
			if((rc = pft_slab_gate_decision(R.slab, gcur, &go, &td, &hd))) return rc;
			if(gtrace) gt_dec += gt_now() - gt_a;
			if(acc && go && memcmp(&td, &t, sizeof t) == 0 && memcmp(&hd, &h, sizeof h) == 0) {
				pft_slab_book_load(R.slab, 1);
				pre = 1;
				R.stats.gated_steps++;
				gcur = gnext;
			} else {
				if(acc && go) R.stats.gate_misses++;
				gcur = 0;
			}
		} else {
			gcur = 0;
		}
	}
	if(gtrace && gt_n)
		fprintf(stderr, "libpft gate trace: %ld attempts, %.2f us each: enqueue %.2f, eps wait %.2f, "
		        "decide+compare %.2f (gated %ld, pow misses %ld)\n", gt_n, (gt_now() - gt_t0) / gt_n,
		        gt_enq / gt_n, gt_wait / gt_n, gt_dec / gt_n, R.stats.gated_steps, R.stats.gate_misses);
	(void)rank;
	/* join the comm stream (the last boundary launch and exchange) before the state leaves */
	if(pft_comm_splits(c) && (rc = pft_slab_order(R.slab, 1))) return rc;
	if(ret != 1 && ret != -4) system->t = t;                                     /* :768 */
	if(spec && k1_valid && ret != -4 && !to_host && !pft_model_get_consts(&R.k1_c)) {
		/* K1 = f(t, x) for the state this call leaves on the device (see R.k1_keep) */
		R.k1_keep = 1;
		R.k1_t = t;
		R.k1_slab = R.slab;
		R.k1_deep = R.deep;
	}
	if(R.opt_timing) pft_slab_timing_flush(R.slab, R.stats.stage_ms, R.stats.stage_n);
	R.tstep = 0;
	R.device_valid = 1;
	R.stats.kernel_launches = launches;
	R.stats.steps_total = attempted;
	if(!(flags & PFT_SOLVE_KEEP_DEVICE) || to_host) {
		if((rc = pft_slab_download_host(R.slab, PFT_BUF_X, system->x))) return rc;
	}
	if(to_host) {
		/* meta_f() returned a right-hand side that is not libpft's: carry on from t, h and the
		   pending command with it, on the host-staged path (hybrid2.c:732 keeps integrating with
		   the new f) -- unless the step cap ended this call on that very step: then it returns 2
		   like any capped call, and the next call (its prologue calls meta_f()) takes the
		   host-staged path from the start */
		R.device_valid = 0;
		if(ret == 2) return ret;
		B->t = t;
		B->h = h;
		return run_staged(system, f, B, command, max_steps_total > 0 ? max_steps_total - attempted : 0, flags);
	}
	return ret;
}

int pft_solver_download(RK_MPI_S_SOLUTION * system)
{
	if(!R.slab || !(R.device_valid || R.in_callback) || !system || !system->x) return -2;
	return pft_slab_download_host(R.slab, PFT_BUF_X, system->x);
}

/* the common end of the device IC paths: every rank's outcome agreed (a rank that failed locally
   still takes part, so that no other rank is left inside a collective: every rank returns the same,
   most negative, code), then the ghost planes exchanged as at an upload and gl_keep agreed */
static int ic_device_finish(int ret, int unclean)
{
	pft_comm * c = comm();
	const long long FAILED = 1LL << 40;
	long long u = ret ? FAILED - ret : unclean;
	int rc;
	if(pft_comm_size(c) > 1 && (rc = pft_comm_allreduce_max_i64(c, &u))) {
		R.last_status = rc;
		return PFT_SOLVE_DEVICE_ERROR;
	}
	if(u >= FAILED) return (int)(FAILED - u);
	if(pft_comm_size(c) > 1) {
		if((rc = pft_comm_halo(c, PFT_BUF_X, 0, 3)) || (rc = pft_comm_halo(c, PFT_BUF_XN, 0, 3))) {
			R.last_status = rc;
			return PFT_SOLVE_DEVICE_ERROR;
		}
	}
	pft_slab_set_gl_keep(R.slab, !u);
	R.device_valid = 1;
	R.k1_keep = 0;
	return 0;
}

int pft_solver_ic_default_device(int with_beads)
{
	/* f1: the default Params' IC (and the glass beads) computed on the device into X and XN, bit
	   for bit what pft_model_ic_default + PrecalculateData give on the host; the next
	   pft_solve_ex(..., PFT_SOLVE_REUSE_DEVICE) starts from it.  Collective with nprocs > 1 (the
	   ghost planes are exchanged, as at an upload, and the ranks agree on gl_keep). */
	pft_ic_tables tb;
	double * store = NULL;
	int * istore = NULL, unclean = 0, rc, ret = 0;
	if(R.max_n == 0) return -3;
	if((rc = ensure_slab())) { R.last_status = rc; ret = PFT_SOLVE_DEVICE_ERROR; }
	else if((rc = pft_model_ic_tables(&tb, with_beads, &store, &istore))) ret = rc;
	else {
		rc = pft_slab_ic_default(R.slab, &tb, &unclean);
		if(rc) { R.last_status = rc; ret = PFT_SOLVE_DEVICE_ERROR; }
	}
	free(store);
	free(istore);
	return ic_device_finish(ret, unclean);
}

int pft_solver_ic_formulas_device(int nprog, const int * qs, const int * lens, const int * ops,
                                  const double * args, int with_beads)
{
	pft_grid g;
	pft_ic_tables tb;
	pft_ic_prog * pr;
	double * store = NULL;
	int * istore = NULL, unclean = 0, rc = 0, ret = 0, p, off = 0, ok = 1;
	if(R.max_n == 0) return -3;
	if(nprog < 1 || !qs || !lens || !ops || !args || pft_model_get_grid(&g)) return -2;
	pr = (pft_ic_prog*)calloc(nprog, sizeof(pft_ic_prog));
	if(!pr) return -1;
	/* compile every program first: the device is not touched unless all of them compile.  The
	   outcome is agreed across ranks before anything collective: 1 (stays on the host) and -2 (bad
	   program) are the same on every rank, but -1 (out of memory in the compiler's tables) is local,
	   and a rank returning early would leave the others in ensure_slab's attach rounds or the
	   allreduce of ic_device_finish until the transport's timeout.  Every rank returns the same code:
	   -1 over -2 over 1. */
	for(p = 0; p < nprog && ok; p++) {
		if(qs[p] < 0 || qs[p] > 2 || lens[p] < 1) { ok = 0; rc = -2; break; }
		rc = pft_ic_compile(&g, lens[p], ops + off, args + off, &pr[p]);
		off += lens[p];
		if(rc) ok = 0;
	}
	if(pft_comm_size(comm()) > 1) {
		long long v = rc == -1 ? 3 : (rc == -2 ? 2 : (rc == 1 ? 1 : (rc ? 3 : 0)));
		int crc = pft_comm_allreduce_max_i64(comm(), &v);
		if(crc) {
			for(p = 0; p < nprog; p++) pft_ic_prog_free(&pr[p]);
			free(pr);
			R.last_status = crc;
			return PFT_SOLVE_DEVICE_ERROR;
		}
		rc = v == 3 ? -1 : (v == 2 ? -2 : (v == 1 ? 1 : 0));
		ok = rc == 0;
	}
	if(!ok) {
		for(p = 0; p < nprog; p++) pft_ic_prog_free(&pr[p]);
		free(pr);
		return rc;
	}
	if((rc = ensure_slab())) { R.last_status = rc; ret = PFT_SOLVE_DEVICE_ERROR; }
	for(p = 0; p < nprog && !ret; p++)
		if((rc = pft_slab_ic_program(R.slab, qs[p], &pr[p], p == 0))) { R.last_status = rc; ret = PFT_SOLVE_DEVICE_ERROR; }
	for(p = 0; p < nprog; p++) pft_ic_prog_free(&pr[p]);
	free(pr);
	/* the beads over gl (PrecalculateData, equation.c:459-530), or only the gl scan without them */
	if(!ret && (rc = pft_model_ic_tables(&tb, with_beads, &store, &istore))) ret = rc;
	else if(!ret && (rc = pft_slab_ic_beads(R.slab, &tb, &unclean))) { R.last_status = rc; ret = PFT_SOLVE_DEVICE_ERROR; }
	free(store);
	free(istore);
	return ic_device_finish(ret, unclean);
}

int pft_solver_eval_rhs(FLOAT t, const FLOAT * w, FLOAT * dw)
{
	/* f(t, w, dw) on host arrays: stage w into A0, exchange its boundary planes, K into K1 */
	pft_comm * c = comm();
	int rc;
	R.k1_keep = 0;                       /* K1's buffer receives this K */
	if(R.fail_rhs_after > 0 && ++R.rhs_calls >= R.fail_rhs_after) {
		R.fail_rhs_after = 0;
		rc = -1000 - 999;                    /* as a hipError_t the runtime reports for a fault */
	} else if(!(rc = ensure_slab()) && !(rc = pft_slab_upload_host(R.slab, PFT_BUF_A0, w)) &&
	   !(pft_comm_size(c) > 1 && (rc = pft_comm_halo(c, PFT_BUF_A0, 0, 3))) &&
	   !(rc = pft_slab_rhs(R.slab, PFT_BUF_A0, PFT_BUF_K1, t)))
		rc = pft_slab_download_host(R.slab, PFT_BUF_K1, dw);
	if(rc) {
		R.last_status = rc;
		R.rhs_failed = 1;
	}
	return rc;
}

/* ---------------------------------------------------------------------------------------- */
/* host-staged path: any right-hand side, combines on the GPU over the chunk table */

static int alloc_staged(void)
{
	int rc;
	if(R.d_cap >= R.max_n) return 0;
	free_staged();
	if((rc = pft_flat_alloc(&R.d_x, R.max_n)) || (rc = pft_flat_alloc(&R.d_k1, R.max_n)) ||
	   (rc = pft_flat_alloc(&R.d_k3, R.max_n)) || (rc = pft_flat_alloc(&R.d_k4, R.max_n)) ||
	   (rc = pft_flat_alloc(&R.d_k5, R.max_n)) || (rc = pft_flat_alloc(&R.d_aux, R.max_n)) ||
	   (rc = pft_flat_alloc(&R.d_eps, 2))) return rc;
	R.d_cap = R.max_n;
	R.h_k = (double*)calloc(R.max_n, sizeof(double));
	R.h_aux = (double*)calloc(R.max_n, sizeof(double));
	if(!R.h_k || !R.h_aux) return -1;
	return 0;
}

static int ensure_staged(const RK_MEM_DIST * n)
{
	int rc;
	if((rc = alloc_staged())) return rc;
	if(R.d_nch < n->n_chunks) {
		pft_dev_free(R.d_cs); pft_dev_free(R.d_cz); pft_flat_free(R.d_cm);
		if((rc = pft_dev_alloc((void**)&R.d_cs, sizeof(int)*n->n_chunks)) ||
		   (rc = pft_dev_alloc((void**)&R.d_cz, sizeof(int)*n->n_chunks)) ||
		   (rc = pft_flat_alloc(&R.d_cm, n->n_chunks))) return rc;
		R.d_nch = n->n_chunks;
	}
	if((rc = pft_h2d(R.d_cs, n->chunk_start, sizeof(int)*n->n_chunks, NULL))) return rc;
	if((rc = pft_h2d(R.d_cz, n->chunk_size, sizeof(int)*n->n_chunks, NULL))) return rc;
	if(n->chunk_eps_mult) {
		if((rc = pft_flat_h2d(R.d_cm, n->chunk_eps_mult, n->n_chunks, NULL))) return rc;
	} else {
		double * ones = (double*)malloc(sizeof(double)*n->n_chunks);
		int i;
		for(i=0;i<n->n_chunks;i++) ones[i] = 1.0;
		rc = pft_flat_h2d(R.d_cm, ones, n->n_chunks, NULL);
		free(ones);
		if(rc) return rc;
	}
	return pft_stream_sync(NULL);
}

static int staged_rhs(RK_RightHandSide f, double t, const double * d_in, double * host_in, double * d_out)
{
	int rc;
	if(d_in) {
		if((rc = pft_flat_d2h(host_in, d_in, R.max_n, NULL)) || (rc = pft_stream_sync(NULL))) return rc;
	}
	R.rhs_failed = 0;
	f(t, host_in, R.h_k);
	if(R.rhs_failed) {
		/* libpft's own f failed on the device and left NaN in h_k: never let that pass as a step
		   (the reference driver leaves NaN handling off, intertrack.c:2193) */
		R.rhs_failed = 0;
		return R.last_status <= -1000 ? R.last_status : -1;
	}
	if((rc = pft_flat_h2d(d_out, R.h_k, R.max_n, NULL))) return rc;
	return 0;
}

static int run_staged(RK_MPI_S_SOLUTION * system, RK_RightHandSide f, solve_bcast * B, int command,
                      long max_steps_total, int flags)
{
	R.k1_keep = 0;                       /* this path computes K1 in the slab's buffers */
	pft_comm * c = comm();
	const int nprocs = pft_comm_size(c);
	RK_MEM_DIST * n = system->n;
	double * x = system->x;
	double t = B->t, h = B->h, new_h = 0.0, h2, h3, h6, h8, eps;
	const double final_time = B->final_time, delta = B->delta, h_min = B->h_min;
	int rc, ret = 0, nch = n->n_chunks;
	long attempted = 0;
	double zero2[2] = {0.0, 0.0};
	(void)flags;

	if((rc = ensure_staged(n))) return rc;
	if((rc = pft_flat_h2d(R.d_x, x, R.max_n, NULL))) return rc;
	R.stats.path = 2;

	while(1) {
		long long bits[2];
		h2 = h/2.0; h3 = h/3.0; h6 = h/6.0; h8 = h/8.0;
		if((rc = staged_rhs(f, t, NULL, x, R.d_k1))) return rc;                                   /* :373 */
		if((rc = pft_flat_combine(1, nch, R.d_cs, R.d_cz, R.d_cm, h3, h, R.d_x, R.d_k1, R.d_k3, R.d_k3,
		                          R.d_k4, R.d_k5, R.d_aux, R.d_eps, NULL))) return rc;          /* :378-389 */
		if((rc = staged_rhs(f, t+h3, R.d_aux, R.h_aux, R.d_k3))) return rc;                       /* K2 in K3, :392 */
		if((rc = pft_flat_combine(2, nch, R.d_cs, R.d_cz, R.d_cm, h6, h, R.d_x, R.d_k1, R.d_k3, R.d_k3,
		                          R.d_k4, R.d_k5, R.d_aux, R.d_eps, NULL))) return rc;          /* :397-409 */
		if((rc = staged_rhs(f, t+h3, R.d_aux, R.h_aux, R.d_k3))) return rc;                       /* :412 */
		if((rc = pft_flat_combine(3, nch, R.d_cs, R.d_cz, R.d_cm, h8, h, R.d_x, R.d_k1, R.d_k3, R.d_k3,
		                          R.d_k4, R.d_k5, R.d_aux, R.d_eps, NULL))) return rc;          /* :417-429 */
		if((rc = staged_rhs(f, t+h2, R.d_aux, R.h_aux, R.d_k4))) return rc;                       /* :432 */
		if((rc = pft_flat_combine(4, nch, R.d_cs, R.d_cz, R.d_cm, h, h, R.d_x, R.d_k1, R.d_k3, R.d_k3,
		                          R.d_k4, R.d_k5, R.d_aux, R.d_eps, NULL))) return rc;          /* :437-450 */
		if((rc = staged_rhs(f, t+h, R.d_aux, R.h_aux, R.d_k5))) return rc;                        /* :453 */
		if((rc = pft_flat_h2d(R.d_eps, zero2, 2, NULL))) return rc;
		if((rc = pft_flat_combine(5, nch, R.d_cs, R.d_cz, R.d_cm, h3, h, R.d_x, R.d_k1, R.d_k3, R.d_k3,
		                          R.d_k4, R.d_k5, R.d_aux, R.d_eps, NULL))) return rc;          /* :507-524 */
		if((rc = pft_flat_d2h((double*)bits, R.d_eps, 2, NULL)) || (rc = pft_stream_sync(NULL))) return rc;
		if(nprocs > 1) {
			if((rc = pft_comm_allreduce_max_i64(c, &bits[0]))) return rc;                      /* :572 */
			bits[1] &= 0xffffffffLL;
			if((rc = pft_comm_allreduce_max_i64(c, &bits[1]))) return rc;
		}
		memcpy(&eps, &bits[0], sizeof(double));
		system->steps_total++;
		attempted++;
		R.stats.last_eps = eps;
		if(B->handle_nan && (bits[1] & 0xffffffffLL)) {
			command |= RKA_CMD_NAN;
			if(h/(final_time-t) < 1e-11) command |= RKA_CMD_h_TOO_SMALL;
		}
		if(B->delta_mode == DELTA_LOCAL) eps *= fabs(h3);
		new_h = ((eps > 0.0) ? pow((delta/eps), 0.2)*0.8 : 2.0) * h;
		if(eps < delta || fabs(h) < h_min) {
			command |= RKA_CMD_UPDATE;
			if(fabs(final_time-(t+h)) <= fabs(new_h)) command |= RKA_CMD_NEXTFINISH;
		}
		if(command & RKA_CMD_NAN) {
			R.last_nan = 1;
			if(command & RKA_CMD_h_TOO_SMALL) { system->t = t; ret = -4; break; }
			h /= 10;
			command = 0;
		} else {
			if(command & RKA_CMD_UPDATE) {
				t += h;
				if((rc = pft_flat_combine(6, nch, R.d_cs, R.d_cz, R.d_cm, h3, h, R.d_x, R.d_k1, R.d_k3, R.d_k3,
				                          R.d_k4, R.d_k5, R.d_x, R.d_eps, NULL))) return rc;    /* :657-668 */
				/* the right-hand side of the next step reads the host x: only the chunks (the
				   unknowns) come back, the ghost values the last f(t, x) wrote stay (the
				   reference updates x in place, hybrid2.c:657-668) */
				if((rc = pft_flat_d2h(R.h_aux, R.d_x, R.max_n, NULL)) || (rc = pft_stream_sync(NULL))) return rc;
				{
					int ch;
					for(ch = 0; ch < nch; ch++)
						memcpy(x + n->chunk_start[ch], R.h_aux + n->chunk_start[ch], sizeof(double)*n->chunk_size[ch]);
				}
				system->steps++;
				if(system->Service_Callback != NULL) {
					system->t = t;
					system->h = h;
					if(system->Service_Callback(final_time, system)) command |= RKA_CMD_BREAK;
				}
				if(nprocs > 1 && B->any_cb && (rc = pft_comm_bcast(c, &command, sizeof(int), R.master))) return rc;
				if(command & RKA_CMD_FINISHED) break;
				if(command & RKA_CMD_BREAK) { system->t = t; system->h = new_h; ret = 1; break; }
				if(system->DDLBF_Rearrange != NULL) {                                              /* :726-729 */
					n = system->n = system->DDLBF_Rearrange(n);
					nch = n->n_chunks;
					if((rc = ensure_staged(n))) return rc;
				}
				f = system->meta_f();
			}
			if(command & RKA_CMD_NEXTFINISH) {
				system->h = new_h;
				h = final_time - t;
				command = RKA_CMD_FINISHED;
			} else {
				command = 0;
				h = new_h;
			}
		}
		if(max_steps_total > 0 && attempted >= max_steps_total) { system->h = h; ret = 2; break; }
	}
	if(ret != 1 && ret != -4) system->t = t;
	R.stats.steps_total = attempted;
	R.stats.kernel_launches = 6*attempted;
	return ret;
}

/* ---------------------------------------------------------------------------------------- */
/* solve, hybrid2.c:215-337 prologue */

int pft_solve_ex(FLOAT final_time, RK_MPI_S_SOLUTION * system, long max_steps_total, int flags)
{
	pft_comm * c = comm();
	const int rank = pft_comm_rank(c);
	int error_code = 0, command = 0, crc;
	long long neg;
	RK_RightHandSide f = NULL;
	solve_bcast B;
	RK_MEM_DIST * n;

	if(system == NULL) return -2;                                               /* :249 */
	n = system->n;
	if(system->meta_f != NULL) f = system->meta_f();                            /* :268 */
	if(n == NULL || n->n_chunks <= 0) error_code = -5;                          /* :276-280 */
	else if(n->chunk_start[n->n_chunks-1] + n->chunk_size[n->n_chunks-1] > R.max_n) error_code = -5;
	if(R.max_n == 0) error_code = -3;                                           /* :282 */
	if(system->x == NULL || system->meta_f == NULL) error_code = -2;            /* :284 */
	if(rank == R.master && system->delta <= 0) error_code = -2;                 /* :286 */
	neg = -error_code;                                                          /* :294 Allreduce(MIN) */
	/* a failed collective (a lost peer, an aborted communicator) is a device error on every rank
	   that sees it; the bounded waits inside make sure each one returns */
	if((crc = pft_comm_allreduce_max_i64(c, &neg))) { R.last_status = crc; return PFT_SOLVE_DEVICE_ERROR; }
	if(error_code) return error_code;                                           /* :295 */
	if(neg > 0) return -6;                                                      /* :299 */

	R.last_nan = 0;                                                             /* :316 */
	B.final_time = final_time; B.t = system->t; B.h = system->h;
	B.h_min = system->h_min; B.delta = system->delta; B.delta_mode = (int)system->delta_mode;
	B.handle_nan = R.handle_nan;
	B.any_cb = system->Service_Callback != NULL;
	if(rank == R.master) {                                                      /* :319-325 */
		if((B.final_time > B.t && B.h < 0) || (B.final_time < B.t && B.h > 0)) B.h *= -1;
		if(B.h == 0 || fabs(B.final_time - B.t) <= fabs(B.h)) {
			B.h = B.final_time - B.t;
			command |= RKA_CMD_FINISHED;
		}
	}
	if(pft_comm_size(c) > 1) {                                                  /* :328-336 */
		long long cmd = command;
		if((crc = pft_comm_bcast(c, &B, sizeof(B), R.master)) || (crc = pft_comm_allreduce_max_i64(c, &cmd))) {
			R.last_status = crc;
			return PFT_SOLVE_DEVICE_ERROR;
		}
		command = (int)cmd;
	}
	R.stats.nprocs = pft_comm_size(c);
	R.stats.rank = rank;

	{
		int rc;
		double em[3];
		if(pft_model_is_device_rhs(f) && system->DDLBF_Rearrange == NULL && canonical_chunks(n, em))
			rc = run_fused(system, f, &B, command, max_steps_total, flags, em);
		else
			rc = run_staged(system, f, &B, command, max_steps_total, flags);
		/* a HIP or RCCL failure (out of device memory, a lost peer, ...) is reported as
		   PFT_SOLVE_DEVICE_ERROR; the raw status stays in pft_solver_last_status() and the HIP
		   text in pft_hip_last_error() */
		if(rc <= -1000 || rc == -1) {
			R.last_status = rc;
			R.device_valid = 0;
			return PFT_SOLVE_DEVICE_ERROR;
		}
		return rc;
	}
}

int RK_MPI_SA_solve(FLOAT final_time, RK_MPI_S_SOLUTION * system)
{
	return pft_solve_ex(final_time, system, 0, 0);
}
