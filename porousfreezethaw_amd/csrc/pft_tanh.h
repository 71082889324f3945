/*
 * pft_tanh.h -- tanh() exactly as the host's C library computes it, for the device initial
 * condition (f1: the glass walls and beads of PrecalculateData, equation.c:459-530, and the default
 * Params' gl formula).  Compiled both as C (gcc, the CPU check tests/test_tanh.py) and as HIP
 * device code (pft_kernels.hip); always without contraction (-ffp-contract=off).
 *
 * glibc 2.35's x86_64 tanh is the generic sysdeps/ieee754/dbl-64 code: fdlibm's s_tanh.c on top of
 * fdlibm's s_expm1.c, whose polynomial glibc evaluates in the split form
 *     r1 = (1 + hxs Q1) + hxs^2 (Q2 + hxs Q3) + hxs^4 (Q4 + hxs Q5)
 * (not fdlibm's Horner chain, which differs from glibc in 450 of 10^7 tanh results).  Restated
 * here from the published algorithm (argument reduction by ln2 in hi/lo parts, the scaled
 * rational correction, reconstruction by exponent arithmetic); the CPU test compares it with the
 * C library on 10^7 arguments (uniform on +-25, +-2, +-60 and log-uniform down to 2^-60): equal
 * bit for bit.  Division, multiplication, addition and the int conversion are IEEE on both sides.
 * Attribution: the algorithm and its polynomial constants are fdlibm's (Sun Microsystems, 1993),
 * as carried in the GNU C Library; none of /root/reference's code is involved.
 */
#ifndef PFT_TANH_H
#define PFT_TANH_H

#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#define PFT_HD __host__ __device__
#else
#define PFT_HD
#endif

static inline PFT_HD uint32_t pft_hi32(double x)
{
	uint64_t u;
	memcpy(&u, &x, 8);
	return (uint32_t)(u >> 32);
}
static inline PFT_HD uint32_t pft_lo32(double x)
{
	uint64_t u;
	memcpy(&u, &x, 8);
	return (uint32_t)u;
}
static inline PFT_HD double pft_with_hi32(double x, uint32_t h)
{
	uint64_t u;
	memcpy(&u, &x, 8);
	u = (u & 0xffffffffULL) | ((uint64_t)h << 32);
	memcpy(&x, &u, 8);
	return x;
}

/* expm1(x), fdlibm s_expm1.c with glibc's polynomial evaluation */
static inline PFT_HD double pft_expm1(double x)
{
	const double one = 1.0, huge = 1.0e+300, tiny = 1.0e-300;
	const double o_threshold = 7.09782712893383973096e+02;
	const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
	const double invln2 = 1.44269504088896338700e+00;
	const double Q1 = -3.33333333333331316428e-02, Q2 = 1.58730158725481460165e-03,
	             Q3 = -7.93650757867487942473e-05, Q4 = 4.00821782732936239552e-06,
	             Q5 = -2.01099218183624371326e-07;
	double y, hi, lo, c = 0.0, t, e, hxs, hfx, r1;
	int k;
	uint32_t hx = pft_hi32(x);
	const uint32_t xsb = hx & 0x80000000u;      /* sign of x */
	hx &= 0x7fffffffu;                           /* high word of |x| */
	if(hx >= 0x4043687Au) {                      /* |x| >= 56 ln2 */
		if(hx >= 0x40862E42u) {                  /* |x| >= 709.78... */
			if(hx >= 0x7ff00000u) {
				if(((hx & 0xfffffu) | pft_lo32(x)) != 0) return x + x;   /* NaN */
				return xsb == 0 ? x : -1.0;                                /* +-inf */
			}
			if(x > o_threshold) return huge * huge;                        /* overflow */
		}
		if(xsb != 0 && x + tiny < 0.0) return tiny - one;                  /* x < -56 ln2: -1 */
	}
	if(hx > 0x3fd62e42u) {                       /* |x| > 0.5 ln2: argument reduction */
		if(hx < 0x3FF0A2B2u) {                   /* and |x| < 1.5 ln2 */
			if(xsb == 0) { hi = x - ln2_hi; lo = ln2_lo; k = 1; }
			else { hi = x + ln2_hi; lo = -ln2_lo; k = -1; }
		} else {
			k = (int)(invln2 * x + ((xsb == 0) ? 0.5 : -0.5));
			t = k;
			hi = x - t * ln2_hi;                 /* t ln2_hi is exact here */
			lo = t * ln2_lo;
		}
		x = hi - lo;
		c = (hi - x) - lo;
	} else if(hx < 0x3c900000u) {                /* |x| < 2^-54: x */
		t = huge + x;
		return x - (t - (huge + x));
	} else {
		k = 0;
	}
	/* x is now in the primary range */
	hfx = 0.5 * x;
	hxs = x * hfx;
	{
		const double R1 = one + hxs * Q1, h2 = hxs * hxs, R2 = Q2 + hxs * Q3, h4 = h2 * h2, R3 = Q4 + hxs * Q5;
		r1 = R1 + h2 * R2 + h4 * R3;
	}
	t = 3.0 - r1 * hfx;
	e = hxs * ((r1 - t) / (6.0 - x * t));
	if(k == 0) return x - (x * e - hxs);         /* c is 0 */
	e = (x * (e - c) - c);
	e -= hxs;
	if(k == -1) return 0.5 * (x - e) - 0.5;
	if(k == 1) {
		if(x < -0.25) return -2.0 * (e - (x + 0.5));
		return one + 2.0 * (x - e);
	}
	if(k <= -2 || k > 56) {                      /* exp(x) - 1 */
		y = one - (e - x);
		if(k == 1024) y = y * 2.0 * 0x1p1023;
		else y = pft_with_hi32(y, pft_hi32(y) + ((uint32_t)k << 20));
		return y - one;
	}
	if(k < 20) {
		t = pft_with_hi32(one, 0x3ff00000u - (0x200000u >> k));   /* 1 - 2^-k */
		y = t - (e - x);
	} else {
		t = pft_with_hi32(one, (uint32_t)(0x3ff - k) << 20);       /* 2^-k */
		y = x - (e + t);
		y += one;
	}
	return pft_with_hi32(y, pft_hi32(y) + ((uint32_t)k << 20));
}

/* tanh(x), fdlibm s_tanh.c (glibc sysdeps/ieee754/dbl-64/s_tanh.c) */
static inline PFT_HD double pft_tanh(double x)
{
	const double one = 1.0, two = 2.0, tiny = 1.0e-300;
	double t, z;
	const int32_t jx = (int32_t)pft_hi32(x);
	const uint32_t ix = (uint32_t)jx & 0x7fffffffu;
	if(ix >= 0x7ff00000u) return jx >= 0 ? one / x + one : one / x - one;   /* inf, NaN */
	if(ix < 0x40360000u) {                       /* |x| < 22 */
		if((ix | pft_lo32(x)) == 0) return x;    /* +-0 */
		if(ix < 0x3c800000u) return x * (one + x);   /* |x| < 2^-55 */
		if(ix >= 0x3ff00000u) {                  /* |x| >= 1 */
			t = pft_expm1(two * (jx >= 0 ? x : -x));
			z = one - two / (t + two);
		} else {
			t = pft_expm1(-two * (jx >= 0 ? x : -x));
			z = -t / (t + two);
		}
	} else {
		z = one - tiny;                          /* |x| >= 22: +-1 */
	}
	return jx >= 0 ? z : -z;
}

#endif
