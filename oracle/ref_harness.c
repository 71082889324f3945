/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
 *
 * A minimal stand-in for the *driver* (apps/intertrack-hybrid-S-freezing/intertrack.c) that
 * drives the reference's own model and solver, compiled IN PLACE from /root/reference:
 *
 *   - model.c / equation.c are #included textually, exactly as intertrack.c does
 *     (intertrack.c:279 and :633), after this file defines the driver globals they use;
 *   - modules/RK_MPI_SAsolver_hybrid2/RK_MPI_SAsolver_hybrid2.c is linked as the solver;
 *   - modules/pparser + libsource/exprsion + libsource/strings parse the Params file and
 *     evaluate the initial-condition formulas (intertrack.c:1425, :1880-2010).
 *
 * Nothing from the reference is copied into this repository: oracle/Makefile compiles the
 * reference sources where they lie, and only this harness' OUTPUTS (golden vectors) are
 * committed under tests/golden/.  Run it under `mpirun -np P` for multi-rank fixtures.
 *
 * Commands (all outputs are raw little-endian fp64 files plus a text key/value file):
 *   pft_ref setup <Params> <outdir>
 *        parse Params, build the grid, evaluate the IC formulas, run PrecalculateData
 *        (glass beads) -> <outdir>/params.txt, <outdir>/ic.f64 (global interior [q][k][j][i])
 *   pft_ref rhs   <Params> <outdir> <state.f64> <t>
 *        K = f(t, state) through the reference meta-pointer -> <outdir>/rhs.f64 (interior),
 *        <outdir>/w_rank<r>.f64 (each rank's full padded input array after bcond+sync),
 *        <outdir>/noise_rank<r>.f64 (each rank's u_noise field, equation.c:450-456, [k][j][i];
 *        rand() is not seeded here, so it is glibc's sequence from seed 1)
 *   pft_ref solve <Params> <outdir> <state.f64> <t0> <h0> <T1> [<T2> ...]
 *        RK_MPI_SA_solve() to each T_i in turn (like intertrack.c:2283) -> <outdir>/traj.txt
 *        (t, h, steps, steps_total, return code per call, hex floats) and
 *        <outdir>/state<i>.f64 (global interior after call i)
 *   pft_ref solvex <Params> <outdir> <state.f64> <t0> <h0> <handle_nan> <break_at> <T1> [<T2> ...]
 *        as solve, with RK_MPI_SA_handle_NAN(handle_nan) (hybrid2.c:138-166) and, when break_at
 *        >= 0, a Service_Callback (hybrid2.c:670-705) that logs every call (steps, t, h) to
 *        <outdir>/cb.txt and returns 1 on its break_at-th call (0 = never); traj.txt rows gain
 *        RK_MPI_SA_check_NAN(); <outdir>/wall<i>.txt holds the wall seconds of call i
 */

#include "common.h"
#include "strings.h"
#include "mprintf.h"
#include "pparser.h"
#include "ee_wrapper.h"
#include "RK_MPI_SAsolver.h"
#include "mathspec.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- driver globals used by model.c / equation.c (names fixed by the reference contract) ---- */
MEMSTREAM * logfile = NULL;
#define MPIMSG_BOUNDARY 200            /* intertrack.c:208 */
static int * MPIrankmap;
static int MPIrank, MPIprocs;
static FLOAT L1, L2, L3;

#include "model.c"

static int calc_mode;
static int N1, N2, N3, n1, n2, n3, total_N3, total_n3, first_row;
static int rowsize, bcond_size, subgridSIZE, subgridSize;
static FLOAT * solution;
static FLOAT model_parameters[PARAM_COUNT];
static FLOAT * param = model_parameters;
#define VAR(var_vector,var_no) ((var_vector) + (var_no)*subgridSIZE)

void CheckErrorAcrossRanks(int error, int code, char ** err_messg)
{
	int any = 0;
	MPI_Allreduce(&error, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
	if(any) {
		if(error) fprintf(stderr, "rank %d error: %s\n", MPIrank, err_messg[error-1]);
		MPI_Finalize();
		exit(code);
	}
}

#include "equation.c"

/* ------------------------------------------------------------------------------------------ */

static char icond_formula[VAR_COUNT][4096];
static double tau, tau_min, delta_, final_time_;
static int saved_files;

static PP_STAT harness_line(_conststring_ line, int l)
{
	const char * s = line;
	(void)l;
	while(*s==' ' || *s=='\t') s++;
	if(*s=='\0' || *s=='\n' || *s=='\r' || *s=='#') return PP_SPECIAL;
	if(!strncmp(s, "set", 3) && (s[3]==' ' || s[3]=='\t')) return PP_SPECIAL;
	if(!strncmp(s, "grid", 4) && (s[4]==' ' || s[4]=='\t')) return PP_SPECIAL;
	if(!strncmp(s, "icond", 5) && (s[5]==' ' || s[5]=='\t')) {
		/* icond <var> = "<formula>"   (intertrack.c:726-732 via cparser) */
		char name[64]; int q;
		const char * p = s+5, *a, *b;
		while(*p==' ' || *p=='\t') p++;
		sscanf(p, "%63[^ \t=]", name);
		a = strchr(p, '"'); if(!a) return PP_ERROR;
		b = strchr(a+1, '"'); if(!b) return PP_ERROR;
		for(q=0;q<VAR_COUNT;q++) if(!strcmp(name, variable[q].name)) break;
		if(q==VAR_COUNT) return PP_ERROR;
		memcpy(icond_formula[q], a+1, b-a-1); icond_formula[q][b-a-1] = 0;
		return PP_SPECIAL;
	}
	return PP_DEFAULT;
}

static double evreq(const char * name)
{
	double x = eval(name);
	if(ev_error()) { fprintf(stderr, "undefined variable %s\n", name); MPI_Abort(MPI_COMM_WORLD, 3); }
	return x;
}

static double evdef(const char * name, double d)
{
	double x = eval(name);
	return ev_error() ? d : x;
}

static int to_int(double x)   /* intertrack.c:673-681 */
{
	double r = floor(x);
	if(x - r >= 0.5) r += 1;
	return (int)r;
}

static void load_params(const char * path)
{
	int q;
	install_evaluator_extensions();
	for(q=0;q<VAR_COUNT;q++) icond_formula[q][0] = 0;
	if(pparse(path, harness_line, NULL)) { fprintf(stderr, "pparse failed\n"); MPI_Abort(MPI_COMM_WORLD, 2); }
	L1 = evreq("L1"); L2 = evreq("L2"); L3 = evreq("L3");
	for(q=0;q<(int)PARAM_INFO_SIZE;q++)
		if(param_info[q].index >= 0) model_parameters[param_info[q].index] = evreq(param_info[q].name);
	calc_mode = to_int(evdef("calc_mode", 0));
	n1 = to_int(evdef("n1", 0)); n2 = to_int(evdef("n2", 0)); total_n3 = to_int(evdef("n3", 0));
	saved_files = to_int(evreq("saved_files"));
	tau = evreq("tau"); final_time_ = evreq("final_time"); delta_ = evreq("delta");
	tau_min = evdef("tau_min", 0.0);
}

/* Z-slab decomposition, as intertrack.c:1776-1800 */
static void decompose(void)
{
	N1 = n1 + 2*bcond_thickness;
	N2 = n2 + 2*bcond_thickness;
	total_N3 = total_n3 + 2*bcond_thickness;
	n3 = total_n3/MPIprocs;
	first_row = MPIrank*n3;
	if(MPIrank < total_n3%MPIprocs) { n3++; first_row += MPIrank; }
	else first_row += total_n3%MPIprocs;
	N3 = n3 + 2*bcond_thickness;
	rowsize = N1*N2;
	bcond_size = bcond_thickness*rowsize;
	subgridSIZE = rowsize*N3;
	subgridSize = rowsize*n3;
	solution = (FLOAT*)malloc(sizeof(FLOAT)*VAR_COUNT*subgridSIZE);
	{ size_t i; for(i=0;i<(size_t)VAR_COUNT*subgridSIZE;i++) solution[i] = 0.0; }
	if(AllocPrecalcData()) { fprintf(stderr, "alloc precalc\n"); MPI_Abort(MPI_COMM_WORLD, 4); }
}

static size_t gidx(int q, int k, int j, int i)   /* global interior index */
{ return (((size_t)q*total_n3 + k)*n2 + j)*n1 + i; }

static size_t lidx(int k, int j, int i)          /* local padded index (k,j,i are interior-relative) */
{ return (size_t)(k+bcond_thickness)*rowsize + (size_t)(j+bcond_thickness)*N1 + (i+bcond_thickness); }

static double * read_global(const char * path)
{
	size_t n = (size_t)VAR_COUNT*n1*n2*total_n3;
	double * g = (double*)malloc(n*sizeof(double));
	FILE * f = fopen(path, "rb");
	if(!f || fread(g, sizeof(double), n, f) != n) { fprintf(stderr, "read %s\n", path); MPI_Abort(MPI_COMM_WORLD, 5); }
	fclose(f);
	return g;
}

static void scatter_interior(const double * g, FLOAT * w)
{
	int q,k,j,i;
	for(q=0;q<VAR_COUNT;q++) for(k=0;k<n3;k++) for(j=0;j<n2;j++) for(i=0;i<n1;i++)
		VAR(w,q)[lidx(k,j,i)] = g[gidx(q,first_row+k,j,i)];
}

/* gather each rank's interior of w into a global array on rank 0 and write it */
static void gather_write(const FLOAT * w, const char * path)
{
	size_t plane = (size_t)n1*n2;
	double * loc = (double*)malloc(sizeof(double)*VAR_COUNT*plane*(n3>0?n3:1));
	int q,k,j,i,r;
	for(q=0;q<VAR_COUNT;q++) for(k=0;k<n3;k++) for(j=0;j<n2;j++) for(i=0;i<n1;i++)
		loc[(((size_t)q*n3+k)*n2+j)*n1+i] = VAR(w,q)[lidx(k,j,i)];
	if(MPIrank==0) {
		double * g = (double*)malloc(sizeof(double)*VAR_COUNT*plane*total_n3);
		for(r=0;r<MPIprocs;r++) {
			int rn3 = total_n3/MPIprocs, rfirst = r*rn3;
			double * buf = loc;
			if(r < total_n3%MPIprocs) { rn3++; rfirst += r; } else rfirst += total_n3%MPIprocs;
			if(r) {
				buf = (double*)malloc(sizeof(double)*VAR_COUNT*plane*rn3);
				MPI_Recv(buf, VAR_COUNT*plane*rn3, MPI_DOUBLE, r, 900, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
			}
			for(q=0;q<VAR_COUNT;q++) memcpy(g + ((size_t)q*total_n3 + rfirst)*plane, buf + (size_t)q*rn3*plane, sizeof(double)*rn3*plane);
			if(r) free(buf);
		}
		{ FILE * f = fopen(path, "wb"); fwrite(g, sizeof(double), VAR_COUNT*plane*total_n3, f); fclose(f); }
		free(g);
	} else {
		MPI_Send(loc, VAR_COUNT*plane*n3, MPI_DOUBLE, 0, 900, MPI_COMM_WORLD);
	}
	free(loc);
}

static void write_params(const char * path)
{
	int q;
	FILE * f;
	if(MPIrank) return;
	f = fopen(path, "w");
	fprintf(f, "L1 %a\nL2 %a\nL3 %a\n", L1, L2, L3);
	for(q=0;q<(int)PARAM_INFO_SIZE;q++)
		if(param_info[q].index >= 0) fprintf(f, "%s %a\n", param_info[q].name, model_parameters[param_info[q].index]);
	fprintf(f, "calc_mode %d\nn1 %d\nn2 %d\nn3 %d\nsaved_files %d\n", calc_mode, n1, n2, total_n3, saved_files);
	fprintf(f, "tau %a\ntau_min %a\ndelta %a\nfinal_time %a\n", tau, tau_min, delta_, final_time_);
	fclose(f);
}

/* initial conditions from formulas, as intertrack.c:1880-2010 (single pass: the default Params
   formulas do not reference other fields) */
static void eval_ic(void)
{
	int q, i, j, k, xi_, yi_, zi_, _xi, _yi, _zi;
	ev_reset();
	{ char b[8]; for(q=0;q<20;q++) { sprintf(b, "i%d", q+1); ev_def_var(b, 1); } }
	ev_def_var("L1", L1); ev_def_var("L2", L2); ev_def_var("L3", L3);
	for(q=0;q<(int)PARAM_INFO_SIZE;q++) if(param_info[q].index >= 0)
		ev_def_var(param_info[q].name, model_parameters[param_info[q].index]);
	ev_def_var("x", 0); xi_ = ev_get_index("x");
	ev_def_var("y", 0); yi_ = ev_get_index("y");
	ev_def_var("z", 0); zi_ = ev_get_index("z");
	ev_def_var("_x", 0); _xi = ev_get_index("_x");
	ev_def_var("_y", 0); _yi = ev_get_index("_y");
	ev_def_var("_z", 0); _zi = ev_get_index("_z");
	for(q=0;q<VAR_COUNT;q++) {
		FLOAT * var = VAR(solution, q);
		if(!icond_formula[q][0]) continue;
		if(ev_parse(icond_formula[q])) { fprintf(stderr, "IC formula syntax error (%d)\n", q); MPI_Abort(MPI_COMM_WORLD, 6); }
		for(k=0;k<n3;k++) {
			double _z = (0.5+k+first_row) / total_n3;
			ev_set_var_value(_zi, _z); ev_set_var_value(zi_, L3*_z);
			for(j=0;j<n2;j++) {
				double _y = (0.5+j) / n2;
				ev_set_var_value(_yi, _y); ev_set_var_value(yi_, L2*_y);
				for(i=0;i<n1;i++) {
					double _x = (0.5+i) / n1;
					ev_set_var_value(_xi, _x); ev_set_var_value(xi_, L1*_x);
					var[lidx(k,j,i)] = ev_evaluate();
				}
			}
		}
	}
}

/* solvex's Service_Callback: log every call, interrupt on the break_at-th */
static FILE * cb_file;
static long cb_calls, cb_break_at;

static int logging_callback(FLOAT final_time, RK_MPI_S_SOLUTION * s)
{
	(void)final_time;
	cb_calls++;
	if(cb_file) fprintf(cb_file, "%ld %a %a\n", s->steps, s->t, s->h);
	return (cb_break_at > 0 && cb_calls == cb_break_at) ? 1 : 0;
}

static RK_RightHandSide (*pick_meta(void))()
{
	/* intertrack.c:2131-2135 */
	if(MPIrank==0) return (MPIprocs==1) ? mf_single : mf_bottom;
	if(MPIrank==MPIprocs-1) return mf_top;
	return mf_middle;
}

int main(int argc, char ** argv)
{
	int q;
	char path[4096];
	FLOAT eps_mult[VAR_COUNT];

	MPI_Init(&argc, &argv);
	MPI_Comm_rank(MPI_COMM_WORLD, &MPIrank);
	MPI_Comm_size(MPI_COMM_WORLD, &MPIprocs);
	MPIrankmap = (int*)malloc(sizeof(int)*MPIprocs);
	for(q=0;q<MPIprocs;q++) MPIrankmap[q] = q;
	if(argc < 4) { fprintf(stderr, "usage: pft_ref setup|rhs|solve <Params> <outdir> ...\n"); return 1; }

	load_params(argv[2]);
	decompose();

	if(!strcmp(argv[1], "setup")) {
		eval_ic();
		if(PrecalculateData(eps_mult)) MPI_Abort(MPI_COMM_WORLD, 7);
		sprintf(path, "%s/params.txt", argv[3]); write_params(path);
		sprintf(path, "%s/ic.f64", argv[3]); gather_write(solution, path);
	} else if(!strcmp(argv[1], "rhs")) {
		double t = strtod(argv[5], NULL);
		double * g;
		FLOAT * K = (FLOAT*)malloc(sizeof(FLOAT)*VAR_COUNT*subgridSIZE);
		size_t s;
		if(PrecalculateData(eps_mult)) MPI_Abort(MPI_COMM_WORLD, 7);   /* constants (overwrites gl: reloaded below) */
		for(s=0;s<(size_t)VAR_COUNT*subgridSIZE;s++) { solution[s] = 0.0/0.0; K[s] = 0.0/0.0; }
		g = read_global(argv[4]);
		scatter_interior(g, solution);
		pick_meta()()(t, solution, K);
		sprintf(path, "%s/rhs.f64", argv[3]); gather_write(K, path);
		sprintf(path, "%s/w_rank%d.f64", argv[3], MPIrank);
		{ FILE * f = fopen(path, "wb"); fwrite(solution, sizeof(FLOAT), VAR_COUNT*subgridSIZE, f); fclose(f); }
		sprintf(path, "%s/noise_rank%d.f64", argv[3], MPIrank);
		{
			FILE * f = fopen(path, "wb");
			int i;
			for(i=0;i<n1*n2*n3;i++) fwrite(&precalc[i].u_noise, sizeof(FLOAT), 1, f);
			fclose(f);
		}
	} else if(!strcmp(argv[1], "solve") || !strcmp(argv[1], "solvex")) {
		const int ext = !strcmp(argv[1], "solvex");
		const int first_T = ext ? 9 : 7;
		double * g;
		int c = 0, j, k, call;
		int n_chunks = VAR_COUNT*n2*n3;
		int * cs = (int*)malloc(sizeof(int)*n_chunks), * cz = (int*)malloc(sizeof(int)*n_chunks);
		FLOAT * cm = (FLOAT*)malloc(sizeof(FLOAT)*n_chunks);
		FILE * tf = NULL;
		if(PrecalculateData(eps_mult)) MPI_Abort(MPI_COMM_WORLD, 7);
		g = read_global(argv[4]);
		scatter_interior(g, solution);
		/* chunk table, intertrack.c:2144-2157 */
		for(q=0;q<VAR_COUNT;q++) for(k=0;k<n3;k++) for(j=0;j<n2;j++) {
			cs[c] = q*subgridSIZE + (k+bcond_thickness)*rowsize + (j+bcond_thickness)*N1 + bcond_thickness;
			cz[c] = n1; cm[c] = 1.0; c++;
		}
		{
			RK_MEM_DIST md = { n_chunks, cs, cz, cm };
			RK_MPI_S_SOLUTION sys = { &md, strtod(argv[5], NULL), solution, NULL, strtod(argv[6], NULL),
			                          tau_min, delta_, DELTA_GLOBAL, NULL, NULL, 0L, 0L };
			sys.meta_f = pick_meta();
			if(RK_MPI_SA_init(VAR_COUNT*subgridSIZE, MPI_COMM_WORLD, 0)) MPI_Abort(MPI_COMM_WORLD, 8);
			if(RK_MPI_SA_check_mem(&md)) MPI_Abort(MPI_COMM_WORLD, 9);
			if(MPIrank==0) { sprintf(path, "%s/traj.txt", argv[3]); tf = fopen(path, "w"); }
			if(ext) {
				RK_MPI_SA_handle_NAN(atoi(argv[7]));
				cb_break_at = atol(argv[8]);
				if(cb_break_at >= 0) {
					sys.Service_Callback = logging_callback;
					if(MPIrank==0) { sprintf(path, "%s/cb.txt", argv[3]); cb_file = fopen(path, "w"); }
				}
			}
			for(call=first_T; call<argc; call++) {
				double w0 = MPI_Wtime(), w1;
				int rc = RK_MPI_SA_solve(strtod(argv[call], NULL), &sys);
				w1 = MPI_Wtime();
				if(ext && MPIrank==0) {   /* wall time of the call (the CPU-baseline calibration) */
					FILE * wf; sprintf(path, "%s/wall%d.txt", argv[3], call-first_T);
					if((wf = fopen(path, "w"))) { fprintf(wf, "%.6f\n", w1 - w0); fclose(wf); }
				}
				if(tf && ext) fprintf(tf, "%a %a %ld %ld %d %d\n", sys.t, sys.h, sys.steps, sys.steps_total, rc, RK_MPI_SA_check_NAN());
				else if(tf) fprintf(tf, "%a %a %ld %ld %d\n", sys.t, sys.h, sys.steps, sys.steps_total, rc);
				sprintf(path, "%s/state%d.f64", argv[3], call-first_T); gather_write(solution, path);
			}
			if(tf) fclose(tf);
			if(cb_file) fclose(cb_file);
			RK_MPI_SA_cleanup();
		}
	} else {
		fprintf(stderr, "unknown command %s\n", argv[1]);
		MPI_Abort(MPI_COMM_WORLD, 1);
	}
	MPI_Finalize();
	return 0;
}
