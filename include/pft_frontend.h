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

#include "pft_model.h"

#ifdef __cplusplus
extern "C" {
#endif

/* fill the interior of variable q of the host padded array w; returns 0, -2 bad program/args */
int pft_ic_eval(const pft_grid * g, int q, int n, const int * op, const double * arg, double * w);

#ifdef __cplusplus
}
#endif
#endif
