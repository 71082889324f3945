/* tests/native/tanh_check.c -- TEST INFRASTRUCTURE: compares libpft's restated tanh / expm1
   (porousfreezethaw_amd/csrc/pft_tanh.h, the device initial condition's) with the C library's
   on n pseudo-random arguments; prints the mismatch counts.  Built and run by tests/test_tanh.py:
     gcc -O2 -std=c99 -ffp-contract=off tanh_check.c -lm && ./a.out n */
#define _DEFAULT_SOURCE
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../porousfreezethaw_amd/csrc/pft_tanh.h"

int main(int argc, char ** argv)
{
	const long n = argc > 1 ? atol(argv[1]) : 1000000;
	long bad_tanh = 0, bad_expm1 = 0, i;
	srand48(20261017);
	for(i = 0; i < n; i++) {
		double x, a, b;
		switch(i % 5) {
			case 0: x = (drand48() * 2 - 1) * 25; break;                  /* tanh's whole range */
			case 1: x = (drand48() * 2 - 1) * 2; break;                   /* the |x| ~ 1 switch */
			case 2: x = (drand48() * 2 - 1) * ldexp(1.0, -(int)(drand48() * 60)); break;
			case 3: x = (drand48() * 2 - 1) * 60; break;                  /* expm1's k > 56 */
			default: x = -drand48() * 45; break;                          /* the beads' arguments */
		}
		a = pft_tanh(x); b = tanh(x);
		if(memcmp(&a, &b, 8)) bad_tanh++;
		a = pft_expm1(x); b = expm1(x);
		if(memcmp(&a, &b, 8)) bad_expm1++;
	}
	printf("%ld %ld %ld\n", n, bad_tanh, bad_expm1);
	return 0;
}
