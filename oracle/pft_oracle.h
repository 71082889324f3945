/*
 * pft_oracle.h -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * oracle/lib/libpft_oracle.so, and only as the checker / the timed CPU baseline.  The
 * product (porousfreezethaw_amd) never links or calls it.
 *
 * Parity pinned: every function here is checked bit-for-bit against golden vectors produced
 * by the reference itself (oracle/ref_harness.c driving /root/reference sources compiled in
 * place; tests/golden/gen_golden.py) in tests/test_oracle_golden.py.
 *
 * Layout: the reference's own host layout (intertrack.c:431,1776-1800): per variable a padded
 * block of (n1+4)(n2+4)(n3+4) doubles, variable blocks consecutive, i fastest; interior cell
 * (i,j,k) of variable q sits at q*S + (k+2)*N1*N2 + (j+2)*N1 + (i+2).
 */
#ifndef PFT_ORACLE_H
#define PFT_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	int n1, n2, n3;        /* interior cells of this slab (n3 = local planes) */
	int total_n3;          /* global planes */
	int first_row;         /* global index of local plane 0 */
	int rank, nprocs;      /* slab position (rank 0 = bottom, z = 0) */
	double L1, L2, L3;     /* domain size */
} pft_or_grid;

/* intertrack.c:1780-1787 */
void pft_or_decompose(int total_n3, int nprocs, int rank, int * n3, int * first_row);
long pft_or_block_size(const pft_or_grid * g);        /* S = N1*N2*N3 (one variable) */

/* equation.c:266-284 (bcond_setup) */
void pft_or_bcond(const pft_or_grid * g, const double * param, double t, double * w);
/* equation.c:290-326 semantics for P slabs held in one process: copy the 2 interface planes of
   every variable between neighbouring slabs */
void pft_or_exchange_local(const pft_or_grid * gs, double ** ws, int nslabs);
/* the 7-point sweep of f_generic_model01 (equation.c:628-738) / f_generic_model2 (:808-881);
   noise may be NULL (u_noise == 0) */
void pft_or_stencil(const pft_or_grid * g, const double * param, int calc_mode,
                    const double * w, const double * noise, double * dw);
/* PrecalculateData constants (equation.c:442-447) are derived inside pft_or_stencil */

/* the u_noise field ([k][j][i] of the slab, equation.c:450-456) that pft_or_solve's right-hand
   side adds (equation.c:676-687); NULL (the default) for u_noise_amp == 0.  Single slab only. */
void pft_or_set_noise(const double * noise);

/* full single-slab RHS: bcond + stencil */
void pft_or_rhs(const pft_or_grid * g, const double * param, int calc_mode, double t,
                double * w, double * dw);

/* Multi-slab hooks for the Merson loop: exchange(w) performs sync_solution on the stage input
   (after the local bcond); allreduce_max(&eps) replaces MPI_Allreduce(MAX).  Both may be NULL
   for a single slab. */
typedef void (*pft_or_exchange_fn)(double * w, void * user);
typedef void (*pft_or_allreduce_fn)(double * value, void * user);

/* RK_MPI_SA_solve (RK_MPI_SAsolver_hybrid2.c:215-770) restated for the intertrack chunk table
   (one chunk per interior row, eps multiplier 1), DELTA_GLOBAL (delta_local=0) or DELTA_LOCAL.
   max_steps_total > 0 stops after that many attempted steps (returns 2).  Returns the reference
   codes 0 / -2 otherwise. */
int pft_or_solve(const pft_or_grid * g, const double * param, int calc_mode,
                 double final_time, double * t, double * h, double h_min, double delta,
                 int delta_local, double * x, long * steps, long * steps_total,
                 long max_steps_total, pft_or_exchange_fn exchange, pft_or_allreduce_fn allreduce,
                 void * user);

/* default Params initial condition (Params:9-21 evaluated as the reference evaluator does) +
   PrecalculateData glass beads (equation.c:459-530); beads = nbeads x 3 unit-cube centres */
void pft_or_ic_default(const pft_or_grid * g, const double * param, const double * beads,
                       int nbeads, double * w);

/* the reference's number parser float_val (libsource/strings/str_fval.c:13-88) */
double pft_or_float_val(const char * s);

#ifdef __cplusplus
}
#endif
#endif
