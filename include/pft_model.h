/*
 * pft_model.h -- the intertrack-hybrid-S-freezing model (u, p, gl) on MI355X.
 *
 * Replaces the reference's model contract: apps/intertrack-hybrid-S-freezing/model.c (variable
 * and parameter enums, model.c:32-59) and equation.c (bcond_setup :266-284, AllocPrecalcData
 * :427-432, FreePrecalcData :434-437, PrecalculateData :439-558, mf_single/top/middle/bottom
 * :955-973).  In the reference that file is #included into the driver and reads the driver's
 * globals (n1, N1, first_row, param[], solution, MPIrank, ...); here the driver hands the same
 * facts over once through pft_model_configure(), and include/pft_equation_adapter.c shows the
 * few lines an unchanged intertrack.c needs to do so.
 *
 * Host memory layout is the reference's (intertrack.c:431,1776-1800): per variable a padded
 * block of N1*N2*N3 doubles (Ni = ni + 2*bcond_thickness, bcond_thickness = 2), variable-major.
 */
#ifndef PFT_MODEL_H
#define PFT_MODEL_H

#include "RK_MPI_SAsolver.h"

#ifdef __cplusplus
extern "C" {
#endif

/* variables, model.c:32-40 */
enum { PFT_VAR_U = 0, PFT_VAR_P = 1, PFT_VAR_GL = 2, PFT_VAR_COUNT = 3 };

/* parameters, in the order of model.c:44-59 (param[] indices are ABI) */
enum {
	PFT_P_u_star, PFT_P_L, PFT_P_xi, PFT_P_a, PFT_P_b, PFT_P_alpha, PFT_P_mu,
	PFT_P_beads_scaling, PFT_P_beads_offset_x, PFT_P_beads_offset_y, PFT_P_beads_offset_z,
	PFT_P_xi_gl, PFT_P_zeta,
	PFT_P_p_eps0, PFT_P_p_eps1,
	PFT_P_gamma,
	PFT_P_water_cp, PFT_P_ice_cp, PFT_P_glass_cp,
	PFT_P_water_lambda, PFT_P_ice_lambda, PFT_P_glass_lambda,
	PFT_P_water_rho, PFT_P_ice_rho, PFT_P_glass_rho,
	PFT_P_top_temp1, PFT_P_top_temp2, PFT_P_phase_switch_time,
	PFT_P_u_noise_amp,
	PFT_P_ball_radius,
	PFT_PARAM_COUNT
};

/* thickness of the ghost layer in the HOST layout (equation.c:38) */
#define PFT_BCOND_THICKNESS 2

/* Everything the reference's equation.c reads from the driver's globals. */
typedef struct {
	int n1, n2;            /* interior cells in x, y */
	int n3;                /* interior planes held by this rank */
	int total_n3;          /* interior planes of the whole grid */
	int first_row;         /* global index of this rank's first plane */
	int rank, nprocs;      /* virtual rank (0 = bottom slab) and slab count */
	double L1, L2, L3;     /* domain size [m] */
	int calc_mode;         /* 0, 1, 2, 10, 11 (Params:115-122) */
} pft_grid;

/* Z-slab split, intertrack.c:1780-1787: floor(total/P) planes, one more for rank < total%P. */
void pft_decompose(int total_n3, int nprocs, int rank, int * n3, int * first_row);

/* Fill a pft_grid and the reference's derived sizes (intertrack.c:1776-1800). */
int pft_grid_init(pft_grid * g, int n1, int n2, int total_n3, int nprocs, int rank,
                  double L1, double L2, double L3, int calc_mode);
long pft_grid_block(const pft_grid * g);   /* subgridSIZE = N1*N2*N3 */

/* The model's view of the driver (replaces the textual #include): must precede everything below.
   param has PFT_PARAM_COUNT entries (copied). Returns 0, or -1 for an invalid grid / calc_mode. */
int pft_model_configure(const pft_grid * g, const double * param);

/* equation.c:266-284 -- boundary conditions on a host array in the host layout (used by the
   driver before full-grid snapshots, intertrack.c:2511,2700). */
void bcond_setup(FLOAT t, FLOAT * w);

/* equation.c:427-558 -- allocate the noise field, precompute constants, overlay the glass beads
   on VAR(w, gl) (max-blend, :507-530).  beads: nbeads x 3 unit-cube centres (the reference reads
   data/spheres_positions.txt on rank 0; pft_model_set_beads() takes them from the caller).
   Return 0 = OK, as the reference. */
int AllocPrecalcData(void);
void FreePrecalcData(void);
int pft_model_set_beads(const double * beads, int nbeads);
int pft_model_load_beads(const char * path);             /* same file format as the reference */
int PrecalculateData(FLOAT * var_eps_mult);              /* overlays beads on the configured solution */
int pft_model_set_solution(FLOAT * solution);            /* the driver's `solution` array */
/* the slab's u_noise field (equation.c:450-456: u_noise_amp*(rand()/RAND_MAX - 0.5) per interior
   node, [k][j][i]); NULL when u_noise_amp == 0.  The reference seeds rand() with the time
   (intertrack.c:1278), so its noise is not reproducible; libpft draws from the process's rand()
   stream as it stands (srand() before PrecalculateData to fix it). */
const FLOAT * pft_model_noise(void);

/* Right-hand sides with the reference signature (RK_RightHandSide).  Called on HOST arrays they
   run the device kernels on a staged copy; the solver recognises them and runs its fused
   device-resident path instead.  f_generic_model01: calc_mode 0/1/10/11; f_generic_model2: 2. */
void f_generic_model01(FLOAT t, const FLOAT * w, FLOAT * dw_dt);
void f_generic_model2(FLOAT t, const FLOAT * w, FLOAT * dw_dt);

/* meta-pointers, equation.c:955-973 */
RK_RightHandSide mf_single(void);
RK_RightHandSide mf_top(void);
RK_RightHandSide mf_middle(void);
RK_RightHandSide mf_bottom(void);

/* Build the reference chunk table (intertrack.c:2144-2157) for the configured grid:
   3*n2*n3 chunks of n1 doubles, eps multiplier 1.  Arrays must hold 3*n2*n3 entries. */
int pft_model_chunks(int * chunk_start, int * chunk_size, FLOAT * chunk_eps_mult);

/* Initial condition of the default Params (Params:9-21), evaluated with the reference
   evaluator's arithmetic (libsource/exprsion) on the configured slab's interior; the glass
   beads are applied afterwards by PrecalculateData().  Host layout. */
int pft_model_ic_default(FLOAT * w);

/* The reference's number parser (libsource/strings/str_fval.c:13-88): Params constants are
   parsed by it, not by strtod, and differ from C literals in the last bit (e.g. 1e-6). */
double pft_float_val(const char * s);

#ifdef __cplusplus
}
#endif
#endif
