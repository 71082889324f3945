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
#include <string.h>

#include "../../include/pft_frontend.h"

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

static double run(int n, const int * op, const double * arg, const double * in)
{
	double st[STACK];
	int sp = 0, i, e = 0;
	for(i = 0; i < n; i++) {
		const int o = op[i];
		if(o == 100) st[sp++] = arg[i];
		else if(o == 101) st[sp++] = in[(int)arg[i]];
		else if(o < 20) { sp--; st[sp-1] = binary(o, st[sp-1], st[sp], &e); }
		else st[sp-1] = unary(o, st[sp-1], &e);
		if(e) return 0;                                         /* the reference's Eval() returns 0 */
	}
	return st[0];
}

int pft_ic_eval(const pft_grid * g, int q, int n, const int * op, const double * arg, double * w)
{
	const long N1 = g->n1 + 2*PFT_BCOND_THICKNESS, N2 = g->n2 + 2*PFT_BCOND_THICKNESS;
	const long N3 = g->n3 + 2*PFT_BCOND_THICKNESS, S = N1*N2*N3;
	int i, k, depth = 0, maxdepth = 0;
	if(!g || !op || !arg || !w || q < 0 || q > 2 || n < 1) return -2;
	for(i = 0; i < n; i++) {                                     /* validate the program */
		if(op[i] == 100 || op[i] == 101) {
			if(op[i] == 101 && (arg[i] < 0 || arg[i] > 8 || arg[i] != floor(arg[i]))) return -2;
			depth++;
		} else if(op[i] >= 1 && op[i] <= 15) depth--;
		else if(op[i] < 20 || op[i] > 48) return -2;
		if(depth < 1) return -2;
		if(depth > maxdepth) maxdepth = depth;
	}
	if(depth != 1 || maxdepth > STACK) return -2;
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
