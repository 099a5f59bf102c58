/*
 * icw_libm.h -- sin / cos bit-identical to the glibc 2.35 libm the reference's CPU path calls.
 *
 * dsp_shift and dsp_pm (adv_modulator.c:537-539, 569-573) take cos / sin of the modulator phase.
 * Built with gcc on Linux (the oracle, and any gcc build of the reference) the pair
 * cos(phase); sin(phase) becomes one sincos() call (gcc's sincos pass), and PM's inner
 * sin(phase + fphase*PI) stays a sin() call.  glibc 2.35 implements both with the IBM Accurate
 * Mathematical Library algorithm (sysdeps/ieee754/dbl-64/s_sin.c, s_sincos.c) *without* its old
 * correctly-rounding slow paths, so results are within ~0.52 ulp, not correctly rounded: a
 * correctly rounded device sin/cos (or ocml's) disagrees with it in a few % of arguments.  This
 * header restates the two entry points the oracle binds, exactly:
 *
 *   icw_lm_sincos(x, &s, &c) -- glibc `sincos`, not an ifunc: the generic x86-64 build, plain
 *                               IEEE double operations in source order (no contraction);
 *   icw_lm_sin_fma(x)        -- glibc `sin` as its ifunc resolves on an x86-64 host with FMA and
 *                               AVX2 (every GPU host of this pool): __sin_fma, the same source
 *                               compiled with -mfma, where gcc fused every product feeding an add
 *                               into an fma.  The fma() calls below are exactly those fusions
 *                               (read off the disassembly of /lib/x86_64-linux-gnu/libm.so.6).
 *
 * Both use glibc's 440-entry table (icw_libm_tab.inc, tools/gen_libm_tab.py) and reduce
 * |x| >= 2.426 with a 4-part pi/2 (reduce_sincos).  glibc switches to Payne-Hanek (__branred)
 * at |x| >= 105414350, which no argument reaches inside the reference's parameter ranges
 * (|fr_shift| <= 20 Hz, PM freq <= 40 Hz, phase / angle in [-1, 1], level <= 1: in_cwave.h:164-182,
 * so |phase + fphase*PI| < 3 pi and |psi| <= 2 pi); beyond that bound this code keeps the
 * 4-part reduction and is no longer glibc-identical.
 *
 * Exactness rests on IEEE-754 double +, -, *, / and fma being correctly rounded (gfx950 VALU and
 * x86-64 SSE/FMA both are) and on nothing here being contracted or reassociated: the kernels are
 * built with -ffp-contract=off.  tests/test_libm.py compiles this header for the host and checks
 * it against libm bit for bit on millions of arguments; the GPU tests check the device build.
 *
 * ICW_LIBM_FN / ICW_LIBM_TAB default to device qualifiers; the host check defines them.
 */
#ifndef ICW_LIBM_H_
#define ICW_LIBM_H_

#ifndef ICW_LIBM_FN
#define ICW_LIBM_FN __device__ __forceinline__
#endif
#ifndef ICW_LIBM_TAB
#define ICW_LIBM_TAB static __device__ const
#endif

ICW_LIBM_TAB unsigned long long icw_sincostab[440] = {
#include "icw_libm_tab.inc"
};

typedef union { double d; unsigned long long u; } icw_lm_bits;

ICW_LIBM_FN double icw_lm_tab(int i) { icw_lm_bits b; b.u = icw_sincostab[i]; return b.d; }
ICW_LIBM_FN unsigned long long icw_lm_u(double d) { icw_lm_bits b; b.d = d; return b.u; }

/* usncs.h constants (glibc's own bit patterns) */
#define ICW_LM_HP0   0x1.921fb54442d18p+0      /* pi/2 high */
#define ICW_LM_HP1   0x1.1a62633145c07p-54     /* pi/2 low */
#define ICW_LM_HPINV 0x1.45f306dc9c883p-1      /* 2/pi */
#define ICW_LM_TOINT 0x1.8p+52
#define ICW_LM_MP1   0x1.921fb58p+0            /* 4-part pi/2 of reduce_sincos */
#define ICW_LM_MP2   -0x1.dde973cp-27
#define ICW_LM_PP3   -0x1.cb3b398p-55
#define ICW_LM_PP4   -0x1.d747f23e32ed7p-83
#define ICW_LM_BIG   0x1.8p+45                 /* rounds |x| to a multiple of 1/128 */
#define ICW_LM_SN3   -0x1.5555555555515p-3
#define ICW_LM_SN5   0x1.11110e829872fp-7
#define ICW_LM_CS2   0x1p-1
#define ICW_LM_CS4   -0x1.5555555555535p-5
#define ICW_LM_CS6   0x1.6c16bedd9e239p-10
#define ICW_LM_S1    -0x1.5555555555555p-3     /* TAYLOR_SIN */
#define ICW_LM_S2    0x1.1111111110ecep-7
#define ICW_LM_S3    -0x1.a01a019db08b8p-13
#define ICW_LM_S4    0x1.71de27b9a7ed9p-19
#define ICW_LM_S5    -0x1.addffc2fcdf59p-26
#define ICW_LM_TAYLOR 0x1.020c49ba5e354p-3     /* 0.126 */

/* table row of |x| (0 <= |x| < 0.86): u = big + |x|, row = low word of u; returns |x| - row/128 */
ICW_LIBM_FN double icw_lm_row(double ax, int &k)
{
    const double u = ICW_LM_BIG + ax;
    k = (int)(unsigned)(icw_lm_u(u) & 0xffffffffull) << 2;
    return ax - (u - ICW_LM_BIG);
}

/* ------------------------------------------------ generic build (sincos) ------ */
/* TAYLOR_SIN: sin(a + da) for |a| < 0.126 */
ICW_LIBM_FN double icw_lm_taylor(double a, double da)
{
    const double xx = a * a;
    const double p = (((ICW_LM_S5 * xx + ICW_LM_S4) * xx + ICW_LM_S3) * xx + ICW_LM_S2) * xx + ICW_LM_S1;
    const double t = (p * a - 0.5 * da) * xx + da;
    return a + t;
}

/* do_sin: sin(x + dx), |x| < 0.855469 */
ICW_LIBM_FN double icw_lm_dosin(double x, double dx)
{
    if (fabs(x) < ICW_LM_TAYLOR) return icw_lm_taylor(x, dx);
    const double xold = x;
    if (x <= 0) dx = -dx;
    int k;
    x = icw_lm_row(fabs(x), k);
    const double xx = x * x;
    const double s = x + (dx + x * xx * (ICW_LM_SN3 + xx * ICW_LM_SN5));
    const double c = x * dx + xx * (ICW_LM_CS2 + xx * (ICW_LM_CS4 + xx * ICW_LM_CS6));
    const double sn = icw_lm_tab(k), ssn = icw_lm_tab(k + 1), cs = icw_lm_tab(k + 2), ccs = icw_lm_tab(k + 3);
    const double cor = (ssn + s * ccs - sn * c) + cs * s;
    return copysign(sn + cor, xold);
}

/* do_cos: cos(x + dx), |x| < 0.855469 */
ICW_LIBM_FN double icw_lm_docos(double x, double dx)
{
    if (x < 0) dx = -dx;
    int k;
    x = icw_lm_row(fabs(x), k) + dx;
    const double xx = x * x;
    const double s = x + x * xx * (ICW_LM_SN3 + xx * ICW_LM_SN5);
    const double c = xx * (ICW_LM_CS2 + xx * (ICW_LM_CS4 + xx * ICW_LM_CS6));
    const double sn = icw_lm_tab(k), ssn = icw_lm_tab(k + 1), cs = icw_lm_tab(k + 2), ccs = icw_lm_tab(k + 3);
    const double cor = (ccs - s * ssn - cs * c) - sn * s;
    return cs + cor;
}

/* reduce_sincos: x = n pi/2 + (a + da), |x| < 105414350 */
ICW_LIBM_FN int icw_lm_reduce(double x, double &a, double &da)
{
    const double t = x * ICW_LM_HPINV + ICW_LM_TOINT;
    const double xn = t - ICW_LM_TOINT;
    const double y = (x - xn * ICW_LM_MP1) - xn * ICW_LM_MP2;
    double t1 = xn * ICW_LM_PP3;
    const double t2 = y - t1;
    double db = (y - t2) - t1;
    t1 = xn * ICW_LM_PP4;
    const double b = t2 - t1;
    db += (t2 - b) - t1;
    a = b;
    da = db;
    return (int)(icw_lm_u(t) & 3u);
}

/* glibc sincos (s_sincos.c, generic x86-64 build) */
ICW_LIBM_FN void icw_lm_sincos(double x, double &sinx, double &cosx)
{
    const unsigned k = (unsigned)(icw_lm_u(x) >> 32) & 0x7fffffffu;
    if (k < 0x400368fdu) {
        if (k < 0x3e400000u) { sinx = x; cosx = 1.0; return; }
        if (k < 0x3feb6000u) { sinx = icw_lm_dosin(x, 0.0); cosx = icw_lm_docos(x, 0.0); return; }
        const double y = ICW_LM_HP0 - fabs(x);
        const double a = y + ICW_LM_HP1;
        const double da = (y - a) + ICW_LM_HP1;
        sinx = copysign(icw_lm_docos(a, da), x);
        cosx = icw_lm_dosin(a, da);
        return;
    }
    if (k >= 0x7ff00000u) { sinx = cosx = x - x; return; }       /* Inf / NaN -> NaN */
    double a, da;
    const int n = icw_lm_reduce(x, a, da);
    if (n == 1 || n == 2) { a = -a; da = -da; }
    const double s = icw_lm_dosin(a, da);
    double c = icw_lm_docos(a, da);
    if (n & 2) c = -c;
    if (n & 1) { sinx = c; cosx = s; }
    else { sinx = s; cosx = c; }
}

/* ------------------------------------------------ FMA build (sin) ------------ */
ICW_LIBM_FN double icw_lm_taylor_f(double a, double da)
{
    const double xx = a * a;
    double p = fma(xx, ICW_LM_S5, ICW_LM_S4);
    p = fma(xx, p, ICW_LM_S3);
    p = fma(xx, p, ICW_LM_S2);
    p = fma(xx, p, ICW_LM_S1);
    const double t = fma(xx, fma(p, a, -(da * 0.5)), da);
    return a + t;
}

ICW_LIBM_FN double icw_lm_dosin_f(double x, double dx)
{
    if (fabs(x) < ICW_LM_TAYLOR) return icw_lm_taylor_f(x, dx);
    const double xold = x;
    if (x <= 0) dx = -dx;
    int k;
    x = icw_lm_row(fabs(x), k);
    const double xx = x * x;
    const double s = x + fma(x * xx, fma(xx, ICW_LM_SN5, ICW_LM_SN3), dx);
    const double c = fma(x, dx, xx * fma(xx, fma(xx, ICW_LM_CS6, ICW_LM_CS4), ICW_LM_CS2));
    const double sn = icw_lm_tab(k), ssn = icw_lm_tab(k + 1), cs = icw_lm_tab(k + 2), ccs = icw_lm_tab(k + 3);
    const double cor = fma(s, cs, fma(-c, sn, fma(s, ccs, ssn)));
    return copysign(sn + cor, xold);
}

ICW_LIBM_FN double icw_lm_docos_f(double x, double dx)
{
    if (x < 0) dx = -dx;
    int k;
    x = icw_lm_row(fabs(x), k) + dx;
    const double xx = x * x;
    const double s = fma(x * xx, fma(xx, ICW_LM_SN5, ICW_LM_SN3), x);
    const double c = xx * fma(xx, fma(xx, ICW_LM_CS6, ICW_LM_CS4), ICW_LM_CS2);
    const double sn = icw_lm_tab(k), ssn = icw_lm_tab(k + 1), cs = icw_lm_tab(k + 2), ccs = icw_lm_tab(k + 3);
    const double cor = fma(-s, sn, fma(-c, cs, fma(-s, ssn, ccs)));
    return cs + cor;
}

ICW_LIBM_FN int icw_lm_reduce_f(double x, double &a, double &da)
{
    const double t = fma(x, ICW_LM_HPINV, ICW_LM_TOINT);
    const double xn = t - ICW_LM_TOINT;
    double y = fma(-xn, ICW_LM_MP1, x);
    y = fma(-xn, ICW_LM_MP2, y);
    const double t2 = fma(-xn, ICW_LM_PP3, y);
    double db = fma(-ICW_LM_PP3, xn, y - t2);
    const double b = fma(-xn, ICW_LM_PP4, t2);
    db = db + fma(-xn, ICW_LM_PP4, t2 - b);
    a = b;
    da = db;
    return (int)(icw_lm_u(t) & 3u);
}

/* glibc sin (s_sin.c as __sin_fma) */
ICW_LIBM_FN double icw_lm_sin_fma(double x)
{
    const unsigned k = (unsigned)(icw_lm_u(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e500000u) return x;
    if (k < 0x3feb6000u) return icw_lm_dosin_f(x, 0.0);
    if (k < 0x400368fdu) return copysign(icw_lm_docos_f(ICW_LM_HP0 - fabs(x), ICW_LM_HP1), x);
    if (k >= 0x7ff00000u) return x - x;
    double a, da;
    const int n = icw_lm_reduce_f(x, a, da);
    const double r = (n & 1) ? icw_lm_docos_f(a, da) : icw_lm_dosin_f(a, da);
    return (n & 2) ? -r : r;
}

#endif /* ICW_LIBM_H_ */
