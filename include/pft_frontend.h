/*
 * pft_frontend.h -- per-node evaluation of the reference's `icond` formulas.
 *
 * intertrack.c:1831-2012 evaluates every `icond <var> = "<formula>"` of the parameter file at each
 * interior node with the Digithell expression evaluator (libsource/exprsion/exp_all.cc).
 * porousfreezethaw_amd/frontend.py parses a formula exactly as that evaluator does and emits the
 * postfix program its evaluation executes; pft_ic_eval() runs the program at every node of this
 * slab with the reference's node variables and C's libm, so the values are bit-identical.
 *
 * Program: n entries (op[i], arg[i]).  op 100: push the constant arg; op 101: push input (int)arg
 * with inputs 0..8 = x, y, z, _x, _y, _z, u, p, gl (x = L1*_x, _x = (0.5+i)/n1; y, z alike, z with
 * the slab's first_row and total_n3, intertrack.c:1958-1971; u/p/gl: the node's value of an
 * already initialised quantity, the multi-pass rule of :1976-1987).  Binary operators
 * (pop y, pop x, push x OP y): 1 -, 2 +, 3 *, 4 /, 5 C, 6 P, 7 ^, 8 root, 9 max, 10 min, 11 <,
 * 12 >, 13 =, 14 and, 15 or.  Unary: 20 -, 21 +, 22 int, 23 floor, 24 ceil, 25 round, 26 abs,
 * 27 sin, 28 cos, 29 tan, 30 asin, 31 acos, 32 atan, 33 sinh, 34 cosh, 35 tanh, 36 asinh,
 * 37 acosh, 38 atanh, 39 log, 40 ln, 41 sqrt, 42 exp, 43 pow10, 44 ! (factorial), 45 toDeg,
 * 46 toRad, 47 sgn, 48 not.  A math error at a node yields 0 there, as the reference's Eval().
 */
#ifndef PFT_FRONTEND_H
#define PFT_FRONTEND_H

#include "pft_hip.h"
#include "pft_model.h"

#ifdef __cplusplus
extern "C" {
#endif

/* fill the interior of variable q of the host padded array w; returns 0, -2 bad program/args */
int pft_ic_eval(const pft_grid * g, int q, int n, const int * op, const double * arg, double * w);

/* f1 for any formula: the program compiled for the device.  Every subexpression
   that reads constants and at most one coordinate (x or _x, y or _y, z or _z) is evaluated here, on
   the host, with the C library -- once (a constant) or once per index of its axis (a table of n1,
   n2 or this slab's n3 entries, with each entry's math-error flag) -- and the rest, over the node's
   u/p/gl and several coordinates, is a residual program whose operators the device evaluates bit
   for bit as the host (csrc/pft_ic_ops.h: IEEE arithmetic, sqrt, comparisons, max/min, logic,
   rounding, factorial, tanh).  Residual program: op 100 push arg, 101 push the node's field arg
   (6 u, 7 p, 8 gl), 102 push table arg at the node's index on that table's axis; the operator
   codes of pft_ic_eval.  All the published formulas (the 86 Params of results/) compile. */
typedef struct {
	int n;                     /* residual program */
	int * op;
	double * arg;
	int ntab;                  /* tables: axis (0 x, 1 y, 2 z), first entry in tab_val / tab_err */
	int * tab_axis;
	long * tab_off;
	double * tab_val;
	unsigned char * tab_err;
	long tab_len;
	int const_err;             /* a constant subexpression erred: the program is the constant 0 */
} pft_ic_prog;
/* 0: compiled; 1: not device-exact (pow or another libm function over the node's fields or
   several coordinates, or a deeper stack than the device's): evaluate it with pft_ic_eval;
   -2 bad program; -1 out of memory */
int pft_ic_compile(const pft_grid * g, int n, const int * op, const double * arg, pft_ic_prog * out);
void pft_ic_prog_free(pft_ic_prog * p);
/* 1 when the program compiles for the device, 0 when it stays on the host, < 0 bad program */
int pft_ic_device_ok(const pft_grid * g, int n, const int * op, const double * arg);
/* the compiled program's semantics run on the host (the check of the compiler against pft_ic_eval) */
int pft_ic_prog_eval_host(const pft_grid * g, int q, const pft_ic_prog * p, double * w);
/* compile + pft_ic_prog_eval_host: the device's result for a program, computed on the host (tests);
   returns pft_ic_compile's code */
int pft_ic_eval_compiled(const pft_grid * g, int q, int n, const int * op, const double * arg, double * w);
/* on the device: the compiled program p (for this slab's grid) into field q of the slab's X and XN
   at every interior node, reading the node's u, p, gl from X; clear = 1 first zeroes X and XN (the
   host array the reference's IC loop fills starts zeroed) */
int pft_slab_ic_program(pft_slab * s, int q, const pft_ic_prog * p, int clear);

#ifdef __cplusplus
}
#endif
#endif
