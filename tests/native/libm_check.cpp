// Host check of in_cwave_amd/csrc/icw_libm.h against the system libm (test infrastructure).
// Usage: libm_check N SEED  -- prints "mismatches <sincos> <sin> of <count>" and the first few.
// Compiled by tests/test_libm.py with g++ -O2 -ffp-contract=off (no -mfma: fma() is libm's).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>

#define ICW_LIBM_FN static inline
#define ICW_LIBM_TAB static const
#include "../../in_cwave_amd/csrc/icw_libm.h"

static uint64_t rs;
static uint64_t rnd() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
static double uni(double lo, double hi) { return lo + (hi - lo) * ((rnd() >> 11) * 0x1p-53); }
static uint64_t bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

// libm entry points through volatile pointers: gcc knows sin / sincos and would otherwise merge
// the two calls on one argument (its sincos pass) and compare one libm routine with itself
static void (*volatile p_sincos)(double, double *, double *) = sincos;
static double (*volatile p_sin)(double) = sin;

static long n_sc, n_s, n_all;
static void check(double x)
{
    double s, c, s2, c2;
    p_sincos(x, &s, &c);                     // libm sincos (generic build)
    icw_lm_sincos(x, s2, c2);
    if (bits(s) != bits(s2) || bits(c) != bits(c2)) {
        if (n_sc < 5) printf("sincos %a: libm %a %a  icw %a %a\n", x, s, c, s2, c2);
        ++n_sc;
    }
    const double f = p_sin(x);               // libm sin (ifunc: __sin_fma on FMA hosts)
    const double f2 = icw_lm_sin_fma(x);
    if (bits(f) != bits(f2)) {
        if (n_s < 5) printf("sin %a: libm %a icw %a\n", x, f, f2);
        ++n_s;
    }
    ++n_all;
}

int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    rs = argc > 2 ? strtoull(argv[2], 0, 0) : 0x9E3779B97F4A7C15ull;
    if (!rs) rs = 1;
    const double PI = 3.14159265358979323846;
    for (long i = 0; i < n; ++i) {
        check(uni(0.0, 2.0 * PI));                       // Shift phases
        check(uni(-PI, 3.0 * PI));                       // PM inner sin(phase + fphase*PI)
        check(uni(-2.0 * PI, 2.0 * PI));                 // PM psi
        check(std::ldexp(uni(1.0, 2.0), -(int)(rnd() % 40)) * ((rnd() & 1) ? 1 : -1));   // small
        const double edges[] = {0.126, 0.85546875, 2.426265, PI / 2, PI, 3 * PI / 2, 2 * PI, 3 * PI};
        const double e = edges[rnd() % 8];
        check(e + std::ldexp(uni(-1.0, 1.0), -(int)(rnd() % 50)));                         // branch edges
        check(uni(-1.0e4, 1.0e4));                                                          // wide
    }
    // the modulator's own phases: fmod(norm_omega * f, 2 pi) along the frame counter
    // (adv_modulator.c:611-625, 537), scaled mode, a few rates and shift frequencies
    const unsigned rates[] = {44100, 48000, 96000, 192000};
    const double fr[] = {2000.0, 4000.0, 20000.0, 1.0, 333.0};
    for (unsigned r : rates)
        for (double f : fr)
            for (long t = 0; t < n / 8; ++t) {
                const unsigned ssr = r * 1000u;
                const uint64_t nf = (uint64_t)((t * 7919ull) % ssr);
                const double om = (2.0 * PI) * ((double)nf) / ((double)ssr);
                check(fmod(om * f, 2.0 * PI));
            }
    printf("mismatches %ld %ld of %ld\n", n_sc, n_s, n_all);
    return (n_sc || n_s) ? 1 : 0;
}
