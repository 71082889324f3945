/*
 * pft_frontend.c -- per-node evaluation of compiled `icond` formulas (include/pft_frontend.h).
 *
 * The postfix program comes from porousfreezethaw_amd/frontend.py, which restates the parse and
 * evaluation order of the reference's expression evaluator (libsource/exprsion/exp_all.cc,
 * ee_wrapper.cc).  Each operator below is the reference's handler (exp_all.cc:21-250,
 * ee_wrapper.cc:255-301) in C: same libm calls, same tests.  The node loop restates
 * intertrack.c:1950-1991 (node coordinates, padded host layout).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pft_frontend.h"
#include "pft_ic_ops.h"

#define STACK 64
#define PI_ 3.14159265358979323846   /* M_PI (exp_all.cc:406, 261-269) */

static double fact(double x, int * e)
{
	double r = 1;
	if(x < 0 || x != floor(x)) { *e = 1; return 0; }
	if(x > 170) { *e = 1; return 0; }
	while(x) r *= x--;
	return r;
}

static double power(double x, double y, int * e)
{
	/* exp_all.cc:53-64 */
	if(x == 0 && y <= 0) { *e = 1; return 0; }
	if(x < 0 && y != floor(y)) {
		if(fmod(1/y - 1, 2) != 0) { *e = 1; return 0; }
		return -pow(-x, y);
	}
	{
		const double r = pow(x, y);
		if(isinf(r) && !isinf(x)) { *e = 1; return 0; }         /* ERANGE */
		return r;
	}
}

static double binary(int op, double x, double y, int * e)
{
	double r = 1;
	switch(op) {
		case 1: return x - y;
		case 2: return x + y;
		case 3: return x * y;
		case 4: if(y == 0) { *e = 1; return 0; } return x / y;
		case 5: case 6:                                         /* C, P (exp_all.cc:223-239) */
			if(x < 0 || x != floor(x) || y < 0 || y != floor(y) || x < y) { *e = 1; return 0; }
			while(y) { r *= x--; if(op == 5) r /= y; y--; }
			return r;
		case 7: return power(x, y, e);
		case 8: if(x == 0) { *e = 1; return 0; } return power(y, 1/x, e);
		case 9: return x > y ? x : y;                           /* max */
		case 10: return x < y ? x : y;                          /* min */
		case 11: return x < y ? 1 : 0;
		case 12: return x > y ? 1 : 0;
		case 13: return x == y ? 1 : 0;
		case 14: return (x != 0 && y != 0) ? 1 : 0;
		case 15: return (x != 0 || y != 0) ? 1 : 0;
	}
	*e = 1;
	return 0;
}

static double unary(int op, double x, int * e)
{
	double r;
	switch(op) {
		case 20: return -x;
		case 21: return x;
		case 22: return x > 0 ? floor(x) : ceil(x);
		case 23: return floor(x);
		case 24: return ceil(x);
		case 25: r = floor(x); if(x - r >= 0.5) r += 1; return r;
		case 26: return fabs(x);
		case 27: if(fabs(x) > 1e12) { *e = 1; return 0; } return sin(x);
		case 28: if(fabs(x) > 1e12) { *e = 1; return 0; } return cos(x);
		case 29: if(fabs(x) > 1e12 || cos(x) == 0) { *e = 1; return 0; } return tan(x);
		case 30: if(fabs(x) > 1) { *e = 1; return 0; } return asin(x);
		case 31: if(fabs(x) > 1) { *e = 1; return 0; } return acos(x);
		case 32: return atan(x);
		case 33: r = sinh(x); if(isinf(r)) { *e = 1; return 0; } return r;   /* ERANGE */
		case 34: r = cosh(x); if(isinf(r)) { *e = 1; return 0; } return r;   /* ERANGE */
		case 35: return tanh(x);
		case 36: return log(x + sqrt(pow(x, 2) + 1));
		case 37: if(x < 1) { *e = 1; return 0; } return log(x + sqrt(pow(x, 2) - 1));
		case 38: if(fabs(x) >= 1) { *e = 1; return 0; } return log((1 + x)/(1 - x))/2;
		case 39: if(x <= 0) { *e = 1; return 0; } return log10(x);
		case 40: if(x <= 0) { *e = 1; return 0; } return log(x);
		case 41: if(x < 0) { *e = 1; return 0; } return sqrt(x);
		case 42: r = exp(x); if(isinf(r)) { *e = 1; return 0; } return r;
		case 43: if(x > 308) { *e = 1; return 0; } return pow(10, x);
		case 44: return fact(x, e);
		case 45: return x/PI_*180;
		case 46: return x/180*PI_;
		case 47: return x > 0 ? 1 : (x < 0 ? -1 : 0);
		case 48: return x != 0 ? 0 : 1;
	}
	*e = 1;
	return 0;
}

/* *err = 1 when a math error ended the evaluation (the result is then 0) */
static double run_e(int n, const int * op, const double * arg, const double * in, int * err)
{
	double st[STACK];
	int sp = 0, i, e = 0;
	*err = 0;
	for(i = 0; i < n; i++) {
		const int o = op[i];
		if(o == 100) st[sp++] = arg[i];
		else if(o == 101) st[sp++] = in[(int)arg[i]];
		else if(o < 20) { sp--; st[sp-1] = binary(o, st[sp-1], st[sp], &e); }
		else st[sp-1] = unary(o, st[sp-1], &e);
		if(e) { *err = 1; return 0; }                           /* the reference's Eval() returns 0 */
	}
	return st[0];
}

static double run(int n, const int * op, const double * arg, const double * in)
{
	int e;
	return run_e(n, op, arg, in, &e);
}

/* a valid program: known operators, inputs 0..8, a stack that never underflows and ends at one value */
static int validate(int n, const int * op, const double * arg)
{
	int i, depth = 0, maxdepth = 0;
	if(!op || !arg || n < 1) return -2;
	for(i = 0; i < n; i++) {
		if(op[i] == 100 || op[i] == 101) {
			if(op[i] == 101 && (arg[i] < 0 || arg[i] > 8 || arg[i] != floor(arg[i]))) return -2;
			depth++;
		} else if(op[i] >= 1 && op[i] <= 15) depth--;
		else if(op[i] < 20 || op[i] > 48) return -2;
		if(depth < 1) return -2;
		if(depth > maxdepth) maxdepth = depth;
	}
	return (depth != 1 || maxdepth > STACK) ? -2 : 0;
}

int pft_ic_eval(const pft_grid * g, int q, int n, const int * op, const double * arg, double * w)
{
	const long N1 = g->n1 + 2*PFT_BCOND_THICKNESS, N2 = g->n2 + 2*PFT_BCOND_THICKNESS;
	const long N3 = g->n3 + 2*PFT_BCOND_THICKNESS, S = N1*N2*N3;
	int k;
	if(!g || !w || q < 0 || q > 2 || validate(n, op, arg)) return -2;
	#pragma omp parallel for schedule(static)
	for(k = 0; k < g->n3; k++) {
		double in[9];
		int j, ii;
		const double _z = (0.5 + k + g->first_row) / g->total_n3;    /* intertrack.c:1958-1960 */
		in[5] = _z; in[2] = g->L3 * _z;
		for(j = 0; j < g->n2; j++) {
			const double _y = (0.5 + j) / g->n2;
			in[4] = _y; in[1] = g->L2 * _y;
			for(ii = 0; ii < g->n1; ii++) {
				const long idx = (k + PFT_BCOND_THICKNESS)*N1*N2 + (j + PFT_BCOND_THICKNESS)*N1 + ii + PFT_BCOND_THICKNESS;
				const double _x = (0.5 + ii) / g->n1;
				in[3] = _x; in[0] = g->L1 * _x;
				in[6] = w[idx]; in[7] = w[S + idx]; in[8] = w[2*S + idx];
				w[q*S + idx] = run(n, op, arg, in);
			}
		}
	}
	return 0;
}

/* ---------------------------------------------------------------------------------------- */
/* f1, general formulas: the program compiled for the device (pft_frontend.h) */

/* the node inputs of axis a at index t (intertrack.c:1958-1971, as pft_ic_eval forms them); the
   other inputs are not read by a one-axis subexpression */
static void axis_inputs(const pft_grid * g, int a, int t, double * in)
{
	int c;
	for(c = 0; c < 9; c++) in[c] = 0.0;
	if(a == 0) { const double _x = (0.5 + t) / g->n1; in[3] = _x; in[0] = g->L1 * _x; }
	if(a == 1) { const double _y = (0.5 + t) / g->n2; in[4] = _y; in[1] = g->L2 * _y; }
	if(a == 2) { const double _z = (0.5 + t + g->first_row) / g->total_n3; in[5] = _z; in[2] = g->L3 * _z; }
}

typedef struct {
	const pft_grid * g;
	const int * op;
	const double * arg;
	int * start;       /* first program entry of each node's subtree (postfix: a contiguous slice) */
	int * kid;         /* two children per node (-1: none) */
	int * dep;         /* inputs the subtree reads: 1 x, 2 y, 4 z, 8 the node's u/p/gl */
	pft_ic_prog * p;
	int cap_tab;
	long cap_val;
	int status;        /* 0, 1 (not device-exact), -1 (out of memory) */
} ic_comp;

static int axis_of(int dep) { return dep == 1 ? 0 : (dep == 2 ? 1 : (dep == 4 ? 2 : -1)); }

static void emit(ic_comp * c, int o, double a)
{
	c->p->op[c->p->n] = o;
	c->p->arg[c->p->n] = a;
	c->p->n++;
}

/* a new table of m entries on axis a; its first entry's index in tab_val, or -1 (out of memory) */
static long new_table(ic_comp * c, int a, int m)
{
	pft_ic_prog * p = c->p;
	if(p->ntab == c->cap_tab || p->tab_len + m > c->cap_val) {
		const int ct = c->cap_tab ? 2 * c->cap_tab : 8;
		const long cv = 2 * (c->cap_val + m);
		int * ax = (int*)realloc(p->tab_axis, sizeof(int) * ct);
		long * off = ax ? (long*)realloc(p->tab_off, sizeof(long) * ct) : NULL;
		double * val = off ? (double*)realloc(p->tab_val, sizeof(double) * cv) : NULL;
		unsigned char * err = val ? (unsigned char*)realloc(p->tab_err, cv) : NULL;
		if(ax) p->tab_axis = ax;
		if(off) p->tab_off = off;
		if(val) p->tab_val = val;
		if(err) p->tab_err = err;
		if(!err) { c->status = -1; return -1; }
		c->cap_tab = ct;
		c->cap_val = cv;
	}
	p->tab_axis[p->ntab] = a;
	p->tab_off[p->ntab] = p->tab_len;
	p->tab_len += m;
	emit(c, 102, (double)p->ntab);
	p->ntab++;
	return p->tab_len - m;
}

static void compile_node(ic_comp * c, int i)
{
	const int d = c->dep[i], o = c->op[i];
	pft_ic_prog * p = c->p;
	double in[9];
	int e, t;
	if(c->status) return;
	if(o == 100) { emit(c, 100, c->arg[i]); return; }
	if(o == 101) {
		const int v = (int)c->arg[i];
		if(v >= 6) { emit(c, 101, (double)v); return; }      /* the node's u, p or gl */
		{
			/* a bare coordinate: a table of the node input itself, as pft_ic_eval forms it */
			const int a = v % 3, m = a == 0 ? c->g->n1 : (a == 1 ? c->g->n2 : c->g->n3);
			const long b = new_table(c, a, m);
			if(b < 0) return;
			for(t = 0; t < m; t++) {
				axis_inputs(c->g, a, t, in);
				p->tab_val[b + t] = in[v];
				p->tab_err[b + t] = 0;
			}
		}
		return;
	}
	if(!(d & 8) && (d == 0 || axis_of(d) >= 0)) {
		/* an operator over constants and one coordinate at most: the host evaluates the subtree with
		   the C library, once (a constant) or once per index of its axis (a table) */
		const int len = i - c->start[i] + 1;
		const int * sop = c->op + c->start[i];
		const double * sarg = c->arg + c->start[i];
		if(d == 0) {
			double v;
			axis_inputs(c->g, 0, 0, in);
			v = run_e(len, sop, sarg, in, &e);
			if(e) p->const_err = 1;
			emit(c, 100, e ? 0.0 : v);
		} else {
			const int a = axis_of(d), m = a == 0 ? c->g->n1 : (a == 1 ? c->g->n2 : c->g->n3);
			const long b = new_table(c, a, m);
			if(b < 0) return;
			for(t = 0; t < m; t++) {
				axis_inputs(c->g, a, t, in);
				p->tab_val[b + t] = run_e(len, sop, sarg, in, &e);
				p->tab_err[b + t] = (unsigned char)e;
			}
		}
		return;
	}
	/* an operator over the node's fields or several coordinates: evaluated on the device */
	if(!pft_ic_op_device(o)) { c->status = 1; return; }
	compile_node(c, c->kid[2*i]);
	if(c->kid[2*i+1] >= 0) compile_node(c, c->kid[2*i+1]);
	emit(c, o, 0.0);
}

void pft_ic_prog_free(pft_ic_prog * p)
{
	if(!p) return;
	free(p->op); free(p->arg); free(p->tab_axis); free(p->tab_off); free(p->tab_val); free(p->tab_err);
	memset(p, 0, sizeof(*p));
}

int pft_ic_compile(const pft_grid * g, int n, const int * op, const double * arg, pft_ic_prog * out)
{
	ic_comp c;
	int * stack, sp = 0, i, depth, maxdepth;
	if(!g || !out) return -2;
	memset(out, 0, sizeof(*out));
	if(validate(n, op, arg)) return -2;
	memset(&c, 0, sizeof(c));
	c.g = g; c.op = op; c.arg = arg; c.p = out;
	c.start = (int*)malloc(sizeof(int) * n);
	c.kid = (int*)malloc(sizeof(int) * 2 * n);
	c.dep = (int*)malloc(sizeof(int) * n);
	stack = (int*)malloc(sizeof(int) * n);
	out->op = (int*)malloc(sizeof(int) * n);
	out->arg = (double*)malloc(sizeof(double) * n);
	if(!c.start || !c.kid || !c.dep || !stack || !out->op || !out->arg) {
		free(c.start); free(c.kid); free(c.dep); free(stack);
		pft_ic_prog_free(out);
		return -1;
	}
	/* the expression tree of the postfix program */
	for(i = 0; i < n; i++) {
		c.kid[2*i] = c.kid[2*i+1] = -1;
		if(op[i] == 100 || op[i] == 101) {
			const int v = op[i] == 101 ? (int)arg[i] : -1;
			c.start[i] = i;
			c.dep[i] = v < 0 ? 0 : (v >= 6 ? 8 : 1 << (v % 3));
		} else if(op[i] <= 15) {
			const int b = stack[--sp], a = stack[--sp];
			c.kid[2*i] = a; c.kid[2*i+1] = b;
			c.start[i] = c.start[a];
			c.dep[i] = c.dep[a] | c.dep[b];
		} else {
			const int a = stack[--sp];
			c.kid[2*i] = a;
			c.start[i] = c.start[a];
			c.dep[i] = c.dep[a];
		}
		stack[sp++] = i;
	}
	compile_node(&c, n - 1);
	free(c.start); free(c.kid); free(c.dep); free(stack);
	if(c.status) { pft_ic_prog_free(out); return c.status; }
	/* the device stack */
	for(i = 0, depth = 0, maxdepth = 0; i < out->n; i++) {
		const int o = out->op[i];
		depth += (o >= 100) ? 1 : (o <= 15 ? -1 : 0);
		if(depth > maxdepth) maxdepth = depth;
	}
	if(maxdepth > PFT_IC_STACK) { pft_ic_prog_free(out); return 1; }
	if(out->const_err) {
		/* a constant subexpression erred: the formula is 0 at every node (the reference's Eval()) */
		out->n = 1;
		out->op[0] = 100;
		out->arg[0] = 0.0;
		out->ntab = 0;
		out->tab_len = 0;
	}
	return 0;
}

int pft_ic_prog_eval_host(const pft_grid * g, int q, const pft_ic_prog * p, double * w)
{
	const long N1 = g->n1 + 2*PFT_BCOND_THICKNESS, N2 = g->n2 + 2*PFT_BCOND_THICKNESS;
	const long N3 = g->n3 + 2*PFT_BCOND_THICKNESS, S = N1*N2*N3;
	int k;
	if(!g || !p || !w || q < 0 || q > 2 || p->n < 1) return -2;
	#pragma omp parallel for schedule(static)
	for(k = 0; k < g->n3; k++) {
		int j, i;
		for(j = 0; j < g->n2; j++)
			for(i = 0; i < g->n1; i++) {
				const long idx = (k + PFT_BCOND_THICKNESS)*N1*N2 + (j + PFT_BCOND_THICKNESS)*N1 + i + PFT_BCOND_THICKNESS;
				double node[3];
				node[0] = w[idx]; node[1] = w[S + idx]; node[2] = w[2*S + idx];
				w[q*S + idx] = pft_ic_run(p->n, p->op, p->arg, node, p->tab_axis, p->tab_off, p->tab_val,
				                          p->tab_err, i, j, k);
			}
	}
	return 0;
}

int pft_ic_device_ok(const pft_grid * g, int n, const int * op, const double * arg)
{
	pft_ic_prog p;
	const int rc = pft_ic_compile(g, n, op, arg, &p);
	pft_ic_prog_free(&p);
	return rc == 0 ? 1 : (rc == 1 ? 0 : rc);
}

int pft_ic_eval_compiled(const pft_grid * g, int q, int n, const int * op, const double * arg, double * w)
{
	pft_ic_prog p;
	int rc = pft_ic_compile(g, n, op, arg, &p);
	if(rc) return rc;
	rc = pft_ic_prog_eval_host(g, q, &p, w);
	pft_ic_prog_free(&p);
	return rc;
}
