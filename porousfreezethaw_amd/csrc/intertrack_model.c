/*
 * intertrack_model.c -- libpft's implementation of the intertrack model contract (pft_model.h).
 *
 * Host C.  Restates, for the driver-facing parts of apps/intertrack-hybrid-S-freezing/equation.c
 * and model.c: the grid bookkeeping the driver does (intertrack.c:1776-1800, 2144-2157), the
 * boundary conditions on host arrays (equation.c:113-284), PrecalculateData (equation.c:427-558:
 * constants, u_noise, glass beads) and the meta-pointers (equation.c:945-973).  The right-hand
 * side itself runs on the GPU (pft_kernels.hip); f_generic_model01/2 below are the host-callable
 * entries with the reference signature, and the solver recognises them to run its fused path.
 *
 * State is per host thread (as the reference's is per MPI process): every thread that drives a
 * slab configures its own model.
 */
#include "pft_internal.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BT PFT_BCOND_THICKNESS
#define MAX_BALLS_COUNT 1000                 /* equation.c:34 */

typedef struct {
	int configured;
	pft_grid g;
	double param[PFT_PARAM_COUNT];
	int N1, N2, N3;
	long row, S;
	FLOAT * solution;
	double * noise;                       /* AllocPrecalcData: n1*n2*n3 */
	double beads[3*MAX_BALLS_COUNT];
	int nbeads, beads_set;
	/* PrecalculateData constants, equation.c:78-82,442-447 */
	double xi2a, xibs, e23, e32;
} model_state;

static __thread model_state M;

/* ---------------------------------------------------------------------------------------- */
/* grid */

void pft_decompose(int total_n3, int nprocs, int rank, int * n3, int * first_row)
{
	/* intertrack.c:1780-1787: the remaining planes go one each to the lowest ranks */
	int n = total_n3/nprocs, f = rank*n;
	if(rank < total_n3%nprocs) { n++; f += rank; }
	else f += total_n3%nprocs;
	*n3 = n;
	*first_row = f;
}

int pft_grid_init(pft_grid * g, int n1, int n2, int total_n3, int nprocs, int rank,
                  double L1, double L2, double L3, int calc_mode)
{
	if(n1 < 1 || n2 < 1 || total_n3 < 1 || nprocs < 1 || rank < 0 || rank >= nprocs) return -1;
	/* intertrack.c:1555-1558: every slab must hold at least bcond_thickness planes */
	if(total_n3/nprocs < BT) return -1;
	memset(g, 0, sizeof(*g));
	g->n1 = n1; g->n2 = n2; g->total_n3 = total_n3;
	pft_decompose(total_n3, nprocs, rank, &g->n3, &g->first_row);
	g->rank = rank; g->nprocs = nprocs;
	g->L1 = L1; g->L2 = L2; g->L3 = L3;
	g->calc_mode = calc_mode;
	return 0;
}

long pft_grid_block(const pft_grid * g)
{
	return (long)(g->n1 + 2*BT)*(g->n2 + 2*BT)*(g->n3 + 2*BT);
}

static int valid_mode(int m) { return m == 0 || m == 1 || m == 2 || m == 10 || m == 11; }

int pft_model_configure(const pft_grid * g, const double * param)
{
	double de;
	if(!g || !param || g->n1 < 1 || g->n2 < 1 || g->n3 < 1 || !valid_mode(g->calc_mode)) return -1;
	free(M.noise); M.noise = NULL;
	M.g = *g;
	memcpy(M.param, param, sizeof(M.param));
	M.N1 = g->n1 + 2*BT; M.N2 = g->n2 + 2*BT; M.N3 = g->n3 + 2*BT;
	M.row = (long)M.N1*M.N2; M.S = M.row*M.N3;
	/* equation.c:442-447 */
	M.xi2a = param[PFT_P_a] / (param[PFT_P_xi]*param[PFT_P_xi]);
	M.xibs = param[PFT_P_b] * sqrt(0.5*param[PFT_P_a]) / param[PFT_P_xi];
	de = param[PFT_P_p_eps1] - param[PFT_P_p_eps0];
	M.e23 = 3.0 / (de*de);
	M.e32 = 2.0 / (de*de*de);
	M.configured = 1;
	return 0;
}

int pft_model_get_grid(pft_grid * g)
{
	if(!M.configured) return -3;
	*g = M.g;
	return 0;
}

int pft_model_get_consts(pft_consts * c)
{
	const double * P = M.param;
	double h1, h2, h3;
	if(!M.configured) return -3;
	memset(c, 0, sizeof(*c));
	/* equation.c:605-612; h3 uses the GLOBAL total_n3 */
	h1 = ((double)M.g.n1) / M.g.L1;
	h2 = ((double)M.g.n2) / M.g.L2;
	h3 = ((double)M.g.total_n3) / M.g.L3;
	c->h1_2 = h1*h1; c->h1d2 = 0.5*h1;
	c->h2_2 = h2*h2; c->h2d2 = 0.5*h2;
	c->h3_2 = h3*h3; c->h3d2 = 0.5*h3;
	c->xi2a = M.xi2a;
	/* left-to-right prefixes of f_GradP / f_SigmaP1_P (equation.c:370,387) */
	c->bam = P[PFT_P_b]*P[PFT_P_alpha]*P[PFT_P_mu];
	c->sam = M.xibs*P[PFT_P_alpha]*P[PFT_P_mu];
	c->alpha = P[PFT_P_alpha]; c->L = P[PFT_P_L]; c->zeta = P[PFT_P_zeta]; c->u_star = P[PFT_P_u_star];
	c->p_eps0 = P[PFT_P_p_eps0]; c->p_eps1 = P[PFT_P_p_eps1]; c->e23 = M.e23; c->e32 = M.e32;
	c->gamma = P[PFT_P_gamma];
	c->mhg = -0.5*P[PFT_P_gamma];                      /* equation.c:420: -0.5*param[gamma] */
	c->rho_g = P[PFT_P_glass_rho]; c->rho_i = P[PFT_P_ice_rho]; c->rho_w = P[PFT_P_water_rho];
	c->cp_g = P[PFT_P_glass_cp]; c->cp_i = P[PFT_P_ice_cp]; c->cp_w = P[PFT_P_water_cp];
	c->lam_g = P[PFT_P_glass_lambda]; c->lam_i = P[PFT_P_ice_lambda]; c->lam_w = P[PFT_P_water_lambda];
	c->top_temp1 = P[PFT_P_top_temp1]; c->top_temp2 = P[PFT_P_top_temp2];
	c->phase_switch_time = P[PFT_P_phase_switch_time];
	return 0;
}

const double * pft_model_noise(void)
{
	return (M.configured && M.param[PFT_P_u_noise_amp] != 0.0) ? M.noise : NULL;
}

int pft_model_chunks(int * chunk_start, int * chunk_size, FLOAT * chunk_eps_mult)
{
	/* intertrack.c:2144-2157 */
	int q, k, j, c = 0;
	if(!M.configured) return -3;
	for(q=0;q<PFT_VAR_COUNT;q++)
		for(k=0;k<M.g.n3;k++)
			for(j=0;j<M.g.n2;j++) {
				chunk_start[c] = (int)(q*M.S + (k+BT)*M.row + (long)(j+BT)*M.N1 + BT);
				chunk_size[c] = M.g.n1;
				chunk_eps_mult[c] = 1.0;
				c++;
			}
	return 0;
}

/* ---------------------------------------------------------------------------------------- */
/* boundary conditions on a host array, equation.c:113-284 */

static void neumann_xy(FLOAT * w)
{
	int i, j, k;
	for(k=0;k<M.g.n3;k++) {
		FLOAT * pl = w + (BT+k)*M.row;
		for(j=0;j<M.g.n2;j++) {
			FLOAT * r = pl + (long)(BT+j)*M.N1 + BT;
			for(i=0;i<BT;i++) { r[-1-i] = r[i]; r[M.g.n1+i] = r[M.g.n1-1-i]; }
		}
		for(j=0;j<BT;j++) {
			memcpy(pl + (long)(BT-1-j)*M.N1, pl + (long)(BT+j)*M.N1, sizeof(FLOAT)*M.N1);
			memcpy(pl + (long)(BT+M.g.n2+j)*M.N1, pl + (long)(BT+M.g.n2-1-j)*M.N1, sizeof(FLOAT)*M.N1);
		}
	}
}

void bcond_setup(FLOAT t, FLOAT * w)
{
	int q, k;
	long i;
	if(!M.configured || !w) return;
	for(q=0;q<PFT_VAR_COUNT;q++) {
		FLOAT * v = w + q*M.S;
		neumann_xy(v);
		if(M.g.rank == 0)            /* z front mirror, equation.c:164-174 */
			for(k=0;k<BT;k++) memcpy(v + (BT-1-k)*M.row, v + (BT+k)*M.row, sizeof(FLOAT)*M.row);
		if(M.g.rank == M.g.nprocs-1) {
			if(q == PFT_VAR_U) {     /* Dirichlet top, equation.c:96-111,175-183 */
				const double T = t < M.param[PFT_P_phase_switch_time] ? M.param[PFT_P_top_temp1]
				                                                       : M.param[PFT_P_top_temp2];
				for(k=0;k<BT;k++) { FLOAT * pl = v + (BT+M.g.n3+k)*M.row; for(i=0;i<M.row;i++) pl[i] = T; }
			} else {                 /* Neumann top, equation.c:251-261 */
				for(k=0;k<BT;k++)
					memcpy(v + (BT+M.g.n3+k)*M.row, v + (BT+M.g.n3-1-k)*M.row, sizeof(FLOAT)*M.row);
			}
		}
	}
}

/* ---------------------------------------------------------------------------------------- */
/* PrecalculateData, equation.c:427-558 */

int AllocPrecalcData(void)
{
	if(!M.configured) return 1;
	free(M.noise);
	M.noise = (double*)malloc(sizeof(double)*(size_t)M.g.n1*M.g.n2*(M.g.n3 > 0 ? M.g.n3 : 1));
	return M.noise == NULL;
}

void FreePrecalcData(void)
{
	free(M.noise);
	M.noise = NULL;
}

int pft_model_set_beads(const double * beads, int nbeads)
{
	if(nbeads < 0) return -1;
	if(nbeads > MAX_BALLS_COUNT) nbeads = MAX_BALLS_COUNT;
	memcpy(M.beads, beads, sizeof(double)*3*nbeads);
	M.nbeads = nbeads;
	M.beads_set = 1;
	return 0;
}

int pft_model_load_beads(const char * path)
{
	/* equation.c:476-484: up to MAX_BALLS_COUNT lines of "x y z" read with %lg */
	FILE * f = fopen(path, "r");
	int n = 0;
	if(!f) return -1;
	while(n < MAX_BALLS_COUNT && fscanf(f, "%lg %lg %lg", M.beads+3*n, M.beads+3*n+1, M.beads+3*n+2) == 3) n++;
	fclose(f);
	M.nbeads = n;
	M.beads_set = 1;
	return 0;
}

int pft_model_set_solution(FLOAT * solution)
{
	M.solution = solution;
	return 0;
}

static void overlay_beads(FLOAT * w)
{
	/* the model state is thread-local: OpenMP workers reach the caller's through m */
	const model_state * const m = &M;
	/* equation.c:507-530: gl = max(gl, 0.5*(1 - tanh(0.5/xi_gl*(|x-b_q| + 1e-10 - R)))).
	   A bead whose tanh argument is >= 22 contributes exactly 0 (glibc tanh returns 1.0 there)
	   and gl >= 0, so such beads are skipped: the result is bit-identical and init at 800^3
	   takes seconds instead of minutes. */
	const double * P = M.param;
	const double s = 0.5/P[PFT_P_xi_gl], R = P[PFT_P_ball_radius];
	const double reach = R + 2.0*P[PFT_P_xi_gl]*30.0;      /* argument >= 30 beyond this */
	const double reach2 = reach*reach;
	double bx[MAX_BALLS_COUNT], by[MAX_BALLS_COUNT], bz[MAX_BALLS_COUNT];
	int q, k;
	for(q=0;q<M.nbeads;q++) {
		bx[q] = M.beads[3*q+0]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_x];
		by[q] = M.beads[3*q+1]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_y];
		bz[q] = M.beads[3*q+2]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_z];
	}
	#pragma omp parallel for schedule(dynamic, 1)
	for(k=0;k<m->g.n3;k++) {
		const double z = m->g.L3 * (0.5+k+m->g.first_row) / m->g.total_n3;
		int j, i, qq, near[MAX_BALLS_COUNT], nn = 0;
		for(qq=0;qq<m->nbeads;qq++) { const double dz = z - bz[qq]; if(dz*dz < reach2*1.0001) near[nn++] = qq; }
		FLOAT * ptr = w + 2*m->S + (BT+k)*m->row;
		for(j=0;j<m->g.n2;j++) {
			const double y = m->g.L2 * (0.5+j) / m->g.n2;
			FLOAT * row = ptr + (long)(BT+j)*m->N1 + BT;
			for(i=0;i<m->g.n1;i++) {
				const double x = m->g.L1 * (0.5+i) / m->g.n1;
				double gl = row[i];
				int t;
				for(t=0;t<nn;t++) {
					const int b = near[t];
					const double v1 = x-bx[b], v2 = y-by[b], v3 = z-bz[b];
					const double d2 = v1*v1 + v2*v2 + v3*v3;
					double nrm, phf;
					if(d2 > reach2*1.0001) continue;
					nrm = sqrt(d2) + 1E-10;
					phf = 0.5*(1.0 - tanh(s*(nrm - R)));
					if(gl < phf) gl = phf;
				}
				row[i] = gl;
			}
		}
	}
}

int PrecalculateData(FLOAT * var_eps_mult)
{
	(void)var_eps_mult;       /* the reference leaves the multipliers at 1 (equation.c:533) */
	if(!M.configured) return 1;
	/* equation.c:450-456: rand() stream from the default seed, per rank */
	if(M.noise) {
		long i, n = (long)M.g.n1*M.g.n2*M.g.n3;
		for(i=0;i<n;i++) M.noise[i] = M.param[PFT_P_u_noise_amp] * (((double)rand() / (double)RAND_MAX) - 0.5);
	}
	if(M.solution) {
		if(!M.beads_set) return 1;      /* the reference fails when the bead file is missing */
		overlay_beads(M.solution);
	}
	return 0;
}

/* ---------------------------------------------------------------------------------------- */
/* initial condition of the default Params (Params:9-21) */

double pft_float_val(const char * s)
{
	/* libsource/strings/str_fval.c:13-88 */
	double out = 0, decimal = 0;
	int decnum = 0, expnum = 0, pointflag = 0, expflag = 0, negflag = 0, expneg = 0, expsign = 0;
	size_t x = 0, len = strlen(s);
	if(s[0] == '-') { negflag = 1; x++; }
	if(s[0] == '+') x++;
	for(; x < len; x++) {
		const char c = s[x];
		if(c == '.') { if(!(pointflag || expflag)) pointflag = 1; continue; }
		if(c == 'E' || c == 'e') { if(!expflag) expflag = 1; continue; }
		if(c == '-' && expflag == 1) { expsign = expneg = 1; expflag++; continue; }
		if(c == '+' && expflag == 1) { expsign = 1; expflag++; continue; }
		if(c >= '0' && c <= '9') {
			const int d = c - '0';
			if(!expflag) {
				if(!pointflag) { out *= 10; out += d; }
				else { decimal *= 10; decimal += d; decnum++; }
			} else {
				expnum *= 10; expnum += d;
				if(expflag++ == (4+expsign)) continue;
			}
		}
	}
	out += decimal/pow(10, decnum);
	while(expnum--) { if(expneg) out /= 10; else out *= 10; }
	return negflag ? -out : out;
}

static double evmax(double a, double b) { return a > b ? a : b; }   /* ee_wrapper.cc:246-250 */

int pft_model_ic_default(FLOAT * w)
{
	/* formula coordinates as intertrack.c:1958-1971 (x = L1*((0.5+i)/n1)); operators of the
	   reference evaluator: ^ is pow (exp_all.cc:50-65), max returns an operand, and/< yield 1/0 */
	const model_state * const m = &M;      /* thread-local state, shared with the OpenMP workers */
	const double * P = M.param;
	const double c293 = pft_float_val("293.15"), c052 = pft_float_val("0.052"),
	             c058 = pft_float_val("0.058"), c055 = pft_float_val("0.055");
	int k;
	if(!M.configured || !w) return -3;
	{
		const double s = 0.5 / P[PFT_P_xi_gl];
		const double r2 = pow(M.g.L1/3.0, 2.0);
		#pragma omp parallel for schedule(static)
		for(k=0;k<m->g.n3;k++) {
			const double z = m->g.L3 * ((0.5+k+m->g.first_row) / m->g.total_n3);
			int i, j;
			for(j=0;j<m->g.n2;j++) {
				const double y = m->g.L2 * ((0.5+j) / m->g.n2);
				const long o = (BT+k)*m->row + (long)(BT+j)*m->N1 + BT;
				for(i=0;i<m->g.n1;i++) {
					const double x = m->g.L1 * ((0.5+i) / m->g.n1);
					double gl;
					w[o+i] = c293;
					w[m->S+o+i] = ((z > c052) && (z < c058) &&
					              (pow(x - m->g.L1/2.0, 2.0) + pow(y - m->g.L2/2.0, 2.0) < r2)) ? 1.0 : 0.0;
					gl = 0.5*(1.0 + tanh(s*(z - c055)));
					gl = evmax(gl, 0.5*(1.0 + tanh(s*(P[PFT_P_beads_offset_z] - z))));
					gl = evmax(gl, 0.5*(1.0 + tanh(s*(x - m->g.L1 + P[PFT_P_beads_offset_x]))));
					gl = evmax(gl, 0.5*(1.0 + tanh(s*(y - m->g.L2 + P[PFT_P_beads_offset_y]))));
					gl = evmax(gl, 0.5*(1.0 + tanh(s*(P[PFT_P_beads_offset_x] - x))));
					gl = evmax(gl, 0.5*(1.0 + tanh(s*(P[PFT_P_beads_offset_y] - y))));
					w[2*m->S+o+i] = gl;
				}
			}
		}
	}
	return 0;
}

/* f1: the per-axis tables of the device initial condition (pft_slab_ic_default).  Every term of
   pft_model_ic_default and overlay_beads that depends on one coordinate only is evaluated here,
   with the same expressions and the C library's tanh / pow; the device combines them in the same
   order and evaluates the beads' tanh with the C library's algorithm (pft_tanh.h).  with_beads:
   overlay the beads (PrecalculateData after the IC).  *store / *istore: the tables' memory, for
   pft_model_ic_tables_free. */
int pft_model_ic_tables(pft_ic_tables * t, int with_beads, double ** store, int ** istore)
{
	const model_state * const m = &M;
	const double * P = M.param;
	const double c293 = pft_float_val("293.15"), c052 = pft_float_val("0.052"),
	             c058 = pft_float_val("0.058"), c055 = pft_float_val("0.055");
	const int n1 = M.g.n1, n2 = M.g.n2, n3 = M.g.n3;
	const double s = 0.5 / P[PFT_P_xi_gl];
	double * d, bxyz[3*MAX_BALLS_COUNT];
	int * iv, i, j, k, q, nb = 0, cnt = 0;
	if(!M.configured) return -3;
	if(with_beads) {
		if(!M.beads_set) return -1;          /* the reference fails without the bead file */
		nb = M.nbeads;
	}
	d = (double*)malloc(sizeof(double)*(4*(size_t)(n1 + n2 + n3) + 3*(size_t)nb));
	iv = (int*)malloc(sizeof(int)*((size_t)(n3 + 1) + (size_t)n3*(nb > 0 ? nb : 1)));
	if(!d || !iv) { free(d); free(iv); return -1; }
	memset(t, 0, sizeof(*t));
	t->n1 = n1; t->n2 = n2; t->n3 = n3;
	t->tx1 = d; t->tx2 = d + n1; t->px2 = d + 2*n1; t->xb = d + 3*n1;
	t->ty1 = d + 4*n1; t->ty2 = t->ty1 + n2; t->py2 = t->ty1 + 2*n2; t->yb = t->ty1 + 3*n2;
	t->tz1 = t->ty1 + 4*n2; t->tz2 = t->tz1 + n3; t->pz = t->tz1 + 2*n3; t->zb = t->tz1 + 3*n3;
	t->bxyz = t->tz1 + 4*n3;
	t->u0 = c293;
	t->r2 = pow(M.g.L1/3.0, 2.0);
	for(i=0;i<n1;i++) {
		const double x = m->g.L1 * ((0.5+i) / m->g.n1);                  /* pft_model_ic_default */
		d[i] = 0.5*(1.0 + tanh(s*(x - m->g.L1 + P[PFT_P_beads_offset_x])));
		d[n1+i] = 0.5*(1.0 + tanh(s*(P[PFT_P_beads_offset_x] - x)));
		d[2*n1+i] = pow(x - m->g.L1/2.0, 2.0);
		d[3*n1+i] = m->g.L1 * (0.5+i) / m->g.n1;                        /* overlay_beads */
	}
	for(j=0;j<n2;j++) {
		double * e = (double*)t->ty1;
		const double y = m->g.L2 * ((0.5+j) / m->g.n2);
		e[j] = 0.5*(1.0 + tanh(s*(y - m->g.L2 + P[PFT_P_beads_offset_y])));
		e[n2+j] = 0.5*(1.0 + tanh(s*(P[PFT_P_beads_offset_y] - y)));
		e[2*n2+j] = pow(y - m->g.L2/2.0, 2.0);
		e[3*n2+j] = m->g.L2 * (0.5+j) / m->g.n2;
	}
	for(k=0;k<n3;k++) {
		double * e = (double*)t->tz1;
		const double z = m->g.L3 * ((0.5+k+m->g.first_row) / m->g.total_n3);
		e[k] = 0.5*(1.0 + tanh(s*(z - c055)));
		e[n3+k] = 0.5*(1.0 + tanh(s*(P[PFT_P_beads_offset_z] - z)));
		e[2*n3+k] = ((z > c052) && (z < c058)) ? 1.0 : 0.0;
		e[3*n3+k] = m->g.L3 * (0.5+k+m->g.first_row) / m->g.total_n3;
	}
	if(nb) {
		/* overlay_beads: the same centres, cull distance and per-plane candidate lists */
		const double R = P[PFT_P_ball_radius];
		const double reach = R + 2.0*P[PFT_P_xi_gl]*30.0;
		const double reach2 = reach*reach;
		for(q=0;q<nb;q++) {
			bxyz[3*q+0] = M.beads[3*q+0]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_x];
			bxyz[3*q+1] = M.beads[3*q+1]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_y];
			bxyz[3*q+2] = M.beads[3*q+2]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_z];
		}
		memcpy((double*)t->bxyz, bxyz, sizeof(double)*3*nb);
		for(k=0;k<n3;k++) {
			const double z = t->zb[k];
			iv[k] = cnt;
			for(q=0;q<nb;q++) { const double dz = z - bxyz[3*q+2]; if(dz*dz < reach2*1.0001) iv[n3+1+cnt++] = q; }
		}
		iv[n3] = cnt;
		t->nbeads = nb;
		t->plane_off = iv;
		t->plane_beads = iv + n3 + 1;
		t->s = s;
		t->R = R;
		t->reach2 = reach2*1.0001;
	}
	*store = d;
	*istore = iv;
	return 0;
}

/* ---------------------------------------------------------------------------------------- */
/* right-hand sides and meta-pointers */

/* implemented in rk_solver.c: evaluate the device RHS on a host array */
int pft_solver_eval_rhs(FLOAT t, const FLOAT * w, FLOAT * dw);

/* The reference's right-hand side cannot fail (void, equation.c:566); a device failure here leaves
   NaN in every entry of dw, which a caller's NaN handling (RK_MPI_SA_handle_NAN) sees, and the
   status in pft_solver_last_status() / the text in pft_hip_last_error(). */
static void rhs_failed(const char * who, FLOAT * dw)
{
	long i, n = PFT_VAR_COUNT * M.S;
	for(i = 0; i < n; i++) dw[i] = NAN;
	fprintf(stderr, "libpft: %s: device evaluation failed (%s)\n", who, pft_hip_last_error());
}

void f_generic_model01(FLOAT t, const FLOAT * w, FLOAT * dw_dt)
{
	/* the reference writes the ghost layers of its input (equation.c:622-626) */
	bcond_setup(t, (FLOAT*)w);
	if(pft_solver_eval_rhs(t, w, dw_dt)) rhs_failed("f_generic_model01", dw_dt);
}

void f_generic_model2(FLOAT t, const FLOAT * w, FLOAT * dw_dt)
{
	bcond_setup(t, (FLOAT*)w);
	if(pft_solver_eval_rhs(t, w, dw_dt)) rhs_failed("f_generic_model2", dw_dt);
}

static RK_RightHandSide mf_generic(void)
{
	/* equation.c:945-953 */
	return M.g.calc_mode == 2 ? f_generic_model2 : f_generic_model01;
}

RK_RightHandSide mf_single(void) { return mf_generic(); }
RK_RightHandSide mf_top(void) { return mf_generic(); }
RK_RightHandSide mf_middle(void) { return mf_generic(); }
RK_RightHandSide mf_bottom(void) { return mf_generic(); }

int pft_model_is_device_rhs(RK_RightHandSide f)
{
	if(!M.configured) return 0;
	if(f == f_generic_model2) return M.g.calc_mode == 2;
	if(f == f_generic_model01) return M.g.calc_mode != 2;
	return 0;
}
