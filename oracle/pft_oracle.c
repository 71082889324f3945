/*
 * pft_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY
 * (see pft_oracle.h: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * it; the product never does).  Plain scalar C, IEEE fp64, no contraction, the reference's
 * operation order; parity is pinned bit-for-bit against the reference's own outputs
 * (tests/golden/, produced by oracle/ref_harness.c from /root/reference compiled in place).
 *
 * Each function cites the reference lines it restates.
 */
#include "pft_oracle.h"
#include "../include/pft_model.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define BT 2                              /* bcond_thickness, equation.c:38 */
#define NV 3

typedef struct { int N1, N2, N3; long row, S; } dims;

static dims dims_of(const pft_or_grid * g)
{
	dims d;
	d.N1 = g->n1 + 2*BT; d.N2 = g->n2 + 2*BT; d.N3 = g->n3 + 2*BT;
	d.row = (long)d.N1*d.N2; d.S = d.row*d.N3;
	return d;
}

void pft_or_decompose(int total_n3, int nprocs, int rank, int * n3, int * first_row)
{
	/* intertrack.c:1780-1787 */
	int n = total_n3/nprocs, f = rank*n;
	if(rank < total_n3%nprocs) { n++; f += rank; } else f += total_n3%nprocs;
	*n3 = n; *first_row = f;
}

long pft_or_block_size(const pft_or_grid * g) { return dims_of(g).S; }

/* ---------------------------------------------------------------------------------------- */
/* boundary conditions, equation.c:113-284 */

static void neumann_xy(const pft_or_grid * g, const dims * d, double * w)
{
	/* equation.c:137-161: x edges of every interior row, then 2 full-width y rows */
	int i, j, k;
	for(k=0;k<g->n3;k++) {
		double * pl = w + (BT+k)*d->row;
		for(j=0;j<g->n2;j++) {
			double * r = pl + (long)(BT+j)*d->N1 + BT;
			for(i=0;i<BT;i++) { r[-1-i] = r[i]; r[g->n1+i] = r[g->n1-1-i]; }
		}
		for(j=0;j<BT;j++) {
			memcpy(pl + (long)(BT-1-j)*d->N1, pl + (long)(BT+j)*d->N1, sizeof(double)*d->N1);
			memcpy(pl + (long)(BT+g->n2+j)*d->N1, pl + (long)(BT+g->n2-1-j)*d->N1, sizeof(double)*d->N1);
		}
	}
}

static void neumann_z_front(const dims * d, double * w)
{
	/* equation.c:164-174 (rank 0): plane -1-k <- plane k, full N1*N2 */
	int k;
	for(k=0;k<BT;k++) memcpy(w + (BT-1-k)*d->row, w + (BT+k)*d->row, sizeof(double)*d->row);
}

void pft_or_bcond(const pft_or_grid * g, const double * param, double t, double * w)
{
	dims d = dims_of(g);
	int q, k;
	long i;
	for(q=0;q<NV;q++) {
		double * v = w + q*d.S;
		neumann_xy(g, &d, v);
		if(g->rank == 0) neumann_z_front(&d, v);
		if(g->rank == g->nprocs-1) {
			if(q == PFT_VAR_U) {
				/* equation.c:96-111,175-183: Dirichlet T_top(t) on 2 full planes */
				double T = t < param[PFT_P_phase_switch_time] ? param[PFT_P_top_temp1] : param[PFT_P_top_temp2];
				for(k=0;k<BT;k++) { double * pl = v + (BT+g->n3+k)*d.row; for(i=0;i<d.row;i++) pl[i] = T; }
			} else {
				/* equation.c:251-261: plane n3+k <- plane n3-1-k */
				for(k=0;k<BT;k++)
					memcpy(v + (BT+g->n3+k)*d.row, v + (BT+g->n3-1-k)*d.row, sizeof(double)*d.row);
			}
		}
	}
}

void pft_or_exchange_local(const pft_or_grid * gs, double ** ws, int nslabs)
{
	/* equation.c:290-326: bcond_size = 2 planes per variable to/from each z-neighbour */
	int r, q;
	for(r=0;r+1<nslabs;r++) {
		dims a = dims_of(&gs[r]), b = dims_of(&gs[r+1]);
		for(q=0;q<NV;q++) {
			double * lo = ws[r] + q*a.S, * hi = ws[r+1] + q*b.S;
			/* upper slab's first 2 interior planes -> lower slab's top ghosts */
			memcpy(lo + (BT+gs[r].n3)*a.row, hi + BT*b.row, sizeof(double)*BT*b.row);
			/* lower slab's last 2 interior planes -> upper slab's bottom ghosts */
			memcpy(hi, lo + gs[r].n3*a.row, sizeof(double)*BT*a.row);
		}
	}
}

/* ---------------------------------------------------------------------------------------- */
/* material functions, equation.c:330-421 */

static double rho_of(const double * P, double p, double gl)
{ return gl*P[PFT_P_glass_rho] + (1.0-gl)*(p*P[PFT_P_ice_rho] + (1.0-p)*P[PFT_P_water_rho]); }
static double cp_of(const double * P, double p, double gl)
{ return gl*P[PFT_P_glass_cp] + (1.0-gl)*(p*P[PFT_P_ice_cp] + (1.0-p)*P[PFT_P_water_cp]); }
static double lambda_of(const double * P, double p, double gl)
{ return gl*P[PFT_P_glass_lambda] + (1.0-gl)*(p*P[PFT_P_ice_lambda] + (1.0-p)*P[PFT_P_water_lambda]); }
static double water_ind(const double * P, double gl)
{ return fmax(0.0, 1.0 - P[PFT_P_zeta]*gl); }

static double sshape(const double * P, double e23, double e32, double x)
{
	/* equation.c:375-382 */
	if(x <= P[PFT_P_p_eps0]) return 0.0;
	if(x >= P[PFT_P_p_eps1]) return 1.0;
	x -= P[PFT_P_p_eps0];
	return x*x*(e23 - e32*x);
}

void pft_or_stencil(const pft_or_grid * g, const double * P, int calc_mode,
                    const double * w, const double * noise, double * dw)
{
	dims d = dims_of(g);
	/* PrecalculateData constants, equation.c:442-447 */
	const double xi2a = P[PFT_P_a] / (P[PFT_P_xi]*P[PFT_P_xi]);
	const double xibs = P[PFT_P_b] * sqrt(0.5*P[PFT_P_a]) / P[PFT_P_xi];
	const double de = P[PFT_P_p_eps1] - P[PFT_P_p_eps0];
	const double e23 = 3.0 / (de*de);
	const double e32 = 2.0 / (de*de*de);
	/* equation.c:605-612 (note the GLOBAL total_n3 in h3) */
	const double h1 = ((double)g->n1) / g->L1, h2 = ((double)g->n2) / g->L2, h3 = ((double)g->total_n3) / g->L3;
	const double h1_2 = h1*h1, h1d2 = 0.5*h1, h2_2 = h2*h2, h2d2 = 0.5*h2, h3_2 = h3*h3, h3d2 = 0.5*h3;
	const long X = 1, Y = d.N1, Z = d.row;
	int i, j, k;

	#pragma omp parallel for private(i, j) schedule(static)
	for(k=0;k<g->n3;k++)
		for(j=0;j<g->n2;j++) {
			long off = (BT+k)*d.row + (long)(BT+j)*d.N1 + BT;
			const double * u = w + off, * p = w + d.S + off, * gl = w + 2*d.S + off;
			const double * nz = noise ? noise + ((long)k*g->n2 + j)*g->n1 : NULL;
			double * du = dw + off, * dp = dw + d.S + off, * dg = dw + 2*d.S + off;
			for(i=0;i<g->n1;i++) {
				const double pc = p[i], gc = gl[i], uc = u[i];
				const double rho = rho_of(P, pc, gc), cp = cp_of(P, pc, gc);
				/* face conductivities: lambda of the face-averaged composition; minus side
				   averages (neighbour + centre), plus side (centre + neighbour) */
				const double lxm = lambda_of(P, 0.5*(p[i-X]+pc), 0.5*(gl[i-X]+gc));
				const double lxp = lambda_of(P, 0.5*(pc+p[i+X]), 0.5*(gc+gl[i+X]));
				const double lym = lambda_of(P, 0.5*(p[i-Y]+pc), 0.5*(gl[i-Y]+gc));
				const double lyp = lambda_of(P, 0.5*(pc+p[i+Y]), 0.5*(gc+gl[i+Y]));
				const double lzm = lambda_of(P, 0.5*(p[i-Z]+pc), 0.5*(gl[i-Z]+gc));
				const double lzp = lambda_of(P, 0.5*(pc+p[i+Z]), 0.5*(gc+gl[i+Z]));
				const double flux =
					h1_2 * ( -lxm*(-u[i-X]+uc) + lxp*(-uc+u[i+X]) ) +
					h2_2 * ( -lym*(-u[i-Y]+uc) + lyp*(-uc+u[i+Y]) ) +
					h3_2 * ( -lzm*(-u[i-Z]+uc) + lzp*(-uc+u[i+Z]) );
				if(calc_mode == 2) {
					/* equation.c:835-874 */
					const double c = cosh(P[PFT_P_gamma]*(uc - P[PFT_P_u_star]));
					const double dpdu = (-0.5*P[PFT_P_gamma]/(c*c)) * water_ind(P, gc);
					const double dudt = flux / (rho*(cp - P[PFT_P_L]*dpdu));
					du[i] = dudt;
					dp[i] = dpdu*dudt;
				} else {
					/* equation.c:650-724 */
					const double un = nz ? uc + nz[i] : uc;
					double dpdt = h1_2*( -(-p[i-X]+pc) + (-pc+p[i+X]) )
					            + h2_2*( -(-p[i-Y]+pc) + (-pc+p[i+Y]) )
					            + h3_2*( -(-p[i-Z]+pc) + (-pc+p[i+Z]) );
					if(calc_mode == 0 || calc_mode == 10) {
						const double v1 = h1d2*(-p[i-X]+p[i+X]), v2 = h2d2*(-p[i-Y]+p[i+Y]),
						             v3 = h3d2*(-p[i-Z]+p[i+Z]);
						const double gn = sqrt(v1*v1 + v2*v2 + v3*v3) + 1E-10;
						dpdt += xi2a*pc*(1.0-pc)*(pc-0.5)
						      - P[PFT_P_b]*P[PFT_P_alpha]*P[PFT_P_mu]*gn*(un - P[PFT_P_u_star]);
					} else if(calc_mode == 1 || calc_mode == 11) {
						dpdt += xi2a*pc*(1.0-pc)*(pc-0.5)
						      - xibs*P[PFT_P_alpha]*P[PFT_P_mu]*sshape(P,e23,e32,pc)*sshape(P,e23,e32,1.0-pc)
						        *fmax(pc*(1.0-pc),0.0)*(un - P[PFT_P_u_star]);
					}
					dpdt /= P[PFT_P_alpha];
					dpdt *= water_ind(P, gc);
					dp[i] = dpdt;
					du[i] = (calc_mode == 10 || calc_mode == 11) ? 0.0 : (flux/rho + P[PFT_P_L]*dpdt)/cp;
				}
				dg[i] = 0.0;
			}
		}
}

void pft_or_rhs(const pft_or_grid * g, const double * param, int calc_mode, double t,
                double * w, double * dw)
{
	pft_or_bcond(g, param, t, w);
	pft_or_stencil(g, param, calc_mode, w, NULL, dw);
}

/* ---------------------------------------------------------------------------------------- */
/* RK-Merson, RK_MPI_SAsolver_hybrid2.c:215-770 over the intertrack chunk table
   (intertrack.c:2144-2157: one chunk per interior row, chunk_eps_mult = 1) */

#define CMD_UPDATE 4
#define CMD_FINISHED 8
#define CMD_NEXTFINISH 16

typedef struct { const pft_or_grid * g; dims d; } rows_t;

/* apply `body` to every interior element index */
#define FOR_CHUNKS(R, IDX, BODY) do { \
	int q_, k_, j_, i_; \
	for(q_=0;q_<NV;q_++) { \
		_Pragma("omp parallel for private(j_, i_) schedule(static)") \
		for(k_=0;k_<(R)->g->n3;k_++) for(j_=0;j_<(R)->g->n2;j_++) { \
			long b_ = q_*(R)->d.S + (BT+k_)*(R)->d.row + (long)(BT+j_)*(R)->d.N1 + BT; \
			for(i_=0;i_<(R)->g->n1;i_++) { long IDX = b_ + i_; BODY; } \
		} \
	} } while(0)

/* the u_noise field the solve's RHS adds (equation.c:450-456, 676-687); NULL: u_noise_amp == 0 */
static const double * or_noise = NULL;

void pft_or_set_noise(const double * noise) { or_noise = noise; }

static void rhs_stage(const pft_or_grid * g, const double * P, int cm, double t, double * w,
                      double * dw, pft_or_exchange_fn ex, void * user)
{
	pft_or_bcond(g, P, t, w);
	if(ex) ex(w, user);
	pft_or_stencil(g, P, cm, w, or_noise, dw);
}

static double eps_max(const rows_t * R, const double * K1, const double * K3, const double * K4,
                      const double * K5)
{
	/* hybrid2.c:507-524 (OpenMP 3.1 max reduction); NaN never wins (e>eps is false) */
	double eps = 0.0;
	int q, k, j, i;
	for(q=0;q<NV;q++) {
		#pragma omp parallel for private(j, i) reduction(max:eps) schedule(static)
		for(k=0;k<R->g->n3;k++) for(j=0;j<R->g->n2;j++) {
			long b = q*R->d.S + (BT+k)*R->d.row + (long)(BT+j)*R->d.N1 + BT;
			for(i=0;i<R->g->n1;i++) {
				double e = 1.0 * fabs(0.2*K1[b+i] - 0.9*K3[b+i] + 0.8*K4[b+i] - 0.1*K5[b+i]);
				if(e > eps) eps = e;
			}
		}
	}
	return eps;
}

int pft_or_solve(const pft_or_grid * g, const double * P, int cm,
                 double final_time, double * tp, double * hp, double h_min, double delta,
                 int delta_local, double * x, long * steps, long * steps_total,
                 long max_steps_total, pft_or_exchange_fn ex, pft_or_allreduce_fn ar, void * user)
{
	rows_t R; long n;
	double *K1, *K3, *K4, *K5, *aux, *K2;
	double t = *tp, h = *hp, new_h = 0.0, h2, h3, h6, h8, eps;
	int command = 0, ret = 0;
	long attempted = 0;

	R.g = g; R.d = dims_of(g); n = NV*R.d.S;
	if(delta <= 0) return -2;
	K1 = (double*)calloc(n, sizeof(double)); K3 = (double*)calloc(n, sizeof(double));
	K4 = (double*)calloc(n, sizeof(double)); K5 = (double*)calloc(n, sizeof(double));
	aux = (double*)calloc(n, sizeof(double));
	K2 = K3;                                                      /* :301 */

	/* :319-325 */
	if((final_time>t && h<0) || (final_time<t && h>0)) h *= -1;
	if(h==0 || fabs(final_time-t)<=fabs(h)) { h = final_time-t; command |= CMD_FINISHED; }

	while(1) {
		h2 = h/2.0; h3 = h/3.0; h6 = h/6.0; h8 = h/8.0;          /* :355 */
		rhs_stage(g, P, cm, t, x, K1, ex, user);                        /* :373 */
		FOR_CHUNKS(&R, e, aux[e] = K1[e]*h3 + x[e]);                   /* :378-389 */
		rhs_stage(g, P, cm, t+h3, aux, K2, ex, user);                   /* :392 */
		FOR_CHUNKS(&R, e, aux[e] = (K1[e] + K2[e])*h6 + x[e]);         /* :397-409 */
		rhs_stage(g, P, cm, t+h3, aux, K3, ex, user);                   /* :412 */
		FOR_CHUNKS(&R, e, aux[e] = (K1[e] + 3.0*K3[e])*h8 + x[e]);     /* :417-429 */
		rhs_stage(g, P, cm, t+h2, aux, K4, ex, user);                   /* :432 */
		FOR_CHUNKS(&R, e, aux[e] = (0.5*K1[e] - 1.5*K3[e] + 2.0*K4[e])*h + x[e]);  /* :437-450 */
		rhs_stage(g, P, cm, t+h, aux, K5, ex, user);                    /* :453 */

		(*steps_total)++; attempted++;                                  /* :460 */
		eps = eps_max(&R, K1, K3, K4, K5);
		if(ar) ar(&eps, user);                                          /* :572 */
		if(delta_local) eps *= fabs(h3);                               /* :578 */
		new_h = ((eps>0.0) ? pow((delta/eps),0.2)*0.8 : 2.0) * h;      /* :580 */
		if(eps<delta || fabs(h)<h_min) {                               /* :599-611 */
			command |= CMD_UPDATE;
			if(fabs(final_time-(t+h)) <= fabs(new_h)) command |= CMD_NEXTFINISH;
		}
		if(command & CMD_UPDATE) {                                      /* :651-668 */
			t += h;
			FOR_CHUNKS(&R, e, x[e] += h3*( 0.5*(K1[e] + K5[e]) + 2.0*K4[e] ));
			(*steps)++;
			if(command & CMD_FINISHED) break;                           /* :695 */
		}
		if(command & CMD_NEXTFINISH) {                                  /* :743-761 */
			*hp = new_h; h = final_time-t; command = CMD_FINISHED;
		} else { command = 0; h = new_h; }
		if(max_steps_total > 0 && attempted >= max_steps_total) { ret = 2; *hp = h; break; }
	}
	*tp = t;
	free(K1); free(K3); free(K4); free(K5); free(aux);
	return ret;
}

/* ---------------------------------------------------------------------------------------- */
/* initial condition: Params:9-21 through the reference evaluator's arithmetic */

double pft_or_float_val(const char * s)
{
	/* str_fval.c:13-88: integer digits accumulated, fraction digits accumulated as an integer
	   and divided by pow(10, count), exponent applied by repeated *10 or /10 */
	double out = 0, decimal = 0;
	int decnum = 0, expnum = 0, pointflag = 0, expflag = 0, negflag = 0, expneg = 0, expsign = 0;
	size_t x = 0, len = strlen(s);
	if(s[0] == '-') { negflag = 1; x++; }
	if(s[0] == '+') x++;
	for(; x < len; x++) {
		char c = s[x];
		if(c == '.') { if(!(pointflag || expflag)) pointflag = 1; continue; }
		if(c == 'E' || c == 'e') { if(!expflag) expflag = 1; continue; }
		if(c == '-' && expflag == 1) { expsign = expneg = 1; expflag++; continue; }
		if(c == '+' && expflag == 1) { expsign = 1; expflag++; continue; }
		if(c >= '0' && c <= '9') {
			int no = c - '0';
			if(!expflag) {
				if(!pointflag) { out *= 10; out += no; }
				else { decimal *= 10; decimal += no; decnum++; }
			} else {
				expnum *= 10; expnum += no;
				if(expflag++ == (4+expsign)) continue;
			}
		}
	}
	out += decimal/pow(10, decnum);
	while(expnum--) { if(expneg) out /= 10; else out *= 10; }
	return negflag ? -out : out;
}

static double emax(double a, double b) { return a > b ? a : b; }   /* ee_wrapper.cc:246-250 */

void pft_or_ic_default(const pft_or_grid * g, const double * P, const double * beads,
                       int nbeads, double * w)
{
	dims d = dims_of(g);
	const double c293 = pft_or_float_val("293.15"), c052 = pft_or_float_val("0.052"),
	             c058 = pft_or_float_val("0.058"), c055 = pft_or_float_val("0.055");
	const double half = 0.5, one = 1.0;
	const double s = half / P[PFT_P_xi_gl];              /* "0.5/xi_gl" */
	double bx[1000], by[1000], bz[1000];
	int i, j, k, q;
	if(nbeads > 1000) nbeads = 1000;                     /* MAX_BALLS_COUNT, equation.c:34 */
	for(q=0;q<nbeads;q++) {                              /* equation.c:480-482 */
		bx[q] = beads[3*q+0]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_x];
		by[q] = beads[3*q+1]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_y];
		bz[q] = beads[3*q+2]*P[PFT_P_beads_scaling] + P[PFT_P_beads_offset_z];
	}
	for(k=0;k<g->n3;k++) {
		/* formula coordinates, intertrack.c:1958-1971: x = L1*((0.5+i)/n1) */
		const double fz = g->L3 * ((0.5+k+g->first_row) / g->total_n3);
		/* PrecalculateData coordinates, equation.c:510-516: x = (L1*(0.5+i))/n1 */
		const double cz = g->L3 * (0.5+k+g->first_row) / g->total_n3;
		for(j=0;j<g->n2;j++) {
			const double fy = g->L2 * ((0.5+j) / g->n2);
			const double cy = g->L2 * (0.5+j) / g->n2;
			for(i=0;i<g->n1;i++) {
				const double fx = g->L1 * ((0.5+i) / g->n1);
				const double cx = g->L1 * (0.5+i) / g->n1;
				long o = (BT+k)*d.row + (long)(BT+j)*d.N1 + BT + i;
				double gl, dx, dy;
				w[o] = c293;                                                    /* Params:9 */
				dx = fx - g->L1/2.0; dy = fy - g->L2/2.0;                      /* Params:11 */
				w[d.S+o] = ((fz > c052) && (fz < c058) &&
				            (pow(dx, 2.0) + pow(dy, 2.0) < pow(g->L1/3.0, 2.0))) ? 1.0 : 0.0;
				gl = half*(one + tanh(s*(fz - c055)));                            /* Params:21 */
				gl = emax(gl, half*(one + tanh(s*(P[PFT_P_beads_offset_z] - fz))));
				gl = emax(gl, half*(one + tanh(s*(fx - g->L1 + P[PFT_P_beads_offset_x]))));
				gl = emax(gl, half*(one + tanh(s*(fy - g->L2 + P[PFT_P_beads_offset_y]))));
				gl = emax(gl, half*(one + tanh(s*(P[PFT_P_beads_offset_x] - fx))));
				gl = emax(gl, half*(one + tanh(s*(P[PFT_P_beads_offset_y] - fy))));
				for(q=0;q<nbeads;q++) {                                          /* equation.c:517-523 */
					const double v1 = cx-bx[q], v2 = cy-by[q], v3 = cz-bz[q];
					const double nrm = sqrt(v1*v1 + v2*v2 + v3*v3) + 1E-10;
					const double phf = 0.5*(1.0 - tanh(0.5/P[PFT_P_xi_gl]*(nrm - P[PFT_P_ball_radius])));
					if(gl < phf) gl = phf;
				}
				w[2*d.S+o] = gl;
			}
		}
	}
}
