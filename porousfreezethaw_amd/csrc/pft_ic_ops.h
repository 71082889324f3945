/*
 * pft_ic_ops.h -- the operators of a compiled `icond` program that the device evaluates bit for bit
 * as the host does (f1, general formulas: pft_ic_compile in pft_frontend.c, ic_prog_kernel in
 * pft_kernels.hip).  Compiled both as C (the host restatement pft_ic_prog_eval_host that the CPU
 * tests compare with pft_ic_eval) and as HIP device code; always without contraction.
 *
 * Each operator is the reference evaluator's handler (exp_all.cc:21-250, ee_wrapper.cc:255-301) as
 * pft_frontend.c states it for the host, restricted to the operators whose result is the same
 * bits on both sides: IEEE + - * / and sqrt (correctly rounded on both), comparisons, max/min,
 * and/or/not, the integer-valued rounding functions, the factorial and C/P loops (sequences of IEEE
 * operations), toDeg/toRad, sgn, and tanh (pft_tanh.h restates the C library's).  pow (^, root)
 * and the other libm functions are not: a formula applies them only to subexpressions of one
 * coordinate (or constants), which the host folds into per-axis tables with the C library
 * itself; anywhere else the program stays on the host (pft_ic_compile returns 1).
 */
#ifndef PFT_IC_OPS_H
#define PFT_IC_OPS_H

#include <math.h>

#include "pft_tanh.h"

#define PFT_IC_STACK 16          /* device evaluation stack (pft_ic_compile checks the depth) */
#define PFT_IC_PI 3.14159265358979323846

/* 1 when the device evaluates operator o exactly as the host */
static inline PFT_HD int pft_ic_op_device(int o)
{
	return (o >= 1 && o <= 6) || (o >= 9 && o <= 15) || (o >= 20 && o <= 26) || o == 35 || o == 41 ||
	       (o >= 44 && o <= 48);
}

static inline PFT_HD double pft_ic_binary(int op, double x, double y, int * e)
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

static inline PFT_HD double pft_ic_unary(int op, double x, int * e)
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
		case 35: return pft_tanh(x);
		case 41: if(x < 0) { *e = 1; return 0; } return sqrt(x);
		case 44:                                                /* factorial */
			r = 1;
			if(x < 0 || x != floor(x) || x > 170) { *e = 1; return 0; }
			while(x) r *= x--;
			return r;
		case 45: return x/PFT_IC_PI*180;
		case 46: return x/180*PFT_IC_PI;
		case 47: return x > 0 ? 1 : (x < 0 ? -1 : 0);
		case 48: return x != 0 ? 0 : 1;
	}
	*e = 1;
	return 0;
}

/* the compiled program at node (i, j, k) of the slab: op 100 push arg; 101 push the node's field
   (int)arg - 6 (u, p, gl); 102 push table t = (int)arg at the node's index on the table's axis
   (taxis[t]: 0 x, 1 y, 2 z; entries from toff[t] in tval, their math-error flags in terr); binary
   1..15 and unary 20..48 as above.  A math error anywhere yields 0, as the reference's Eval() (and
   pft_ic_eval). */
static inline PFT_HD double pft_ic_run(int n, const int * op, const double * arg, const double * node,
                                       const int * taxis, const long * toff, const double * tval,
                                       const unsigned char * terr, int i, int j, int k)
{
	double st[PFT_IC_STACK];
	int sp = 0, c, e = 0;
	for(c = 0; c < n; c++) {
		const int o = op[c];
		if(o == 100) st[sp++] = arg[c];
		else if(o == 101) st[sp++] = node[(int)arg[c] - 6];
		else if(o == 102) {
			const int t = (int)arg[c];
			const long x = toff[t] + (taxis[t] == 0 ? i : (taxis[t] == 1 ? j : k));
			if(terr[x]) return 0;
			st[sp++] = tval[x];
		}
		else if(o < 20) { sp--; st[sp-1] = pft_ic_binary(o, st[sp-1], st[sp], &e); }
		else st[sp-1] = pft_ic_unary(o, st[sp-1], &e);
		if(e) return 0;
	}
	return st[0];
}

#endif
