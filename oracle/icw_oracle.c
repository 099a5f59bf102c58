/*
 * oracle/icw_oracle.c -- TEST INFRASTRUCTURE ONLY (never linked into, called by, or shipped
 * with the product library).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / the timed CPU baseline.
 *
 * A scalar C restatement of the in_cwave (V2.4.4) per-block hot path, written from the
 * reference's behaviour with the SAME floating-point operation order, so that a build with
 * `gcc -O2 -ffp-contract=off` (no fast-math) reproduces the reference's doubles bit for bit:
 *
 *   orc_iir_*        <- iir_rp_process_kahan / _baseline   hblpf.c:1008-1099 / 894-953
 *                       (incl. the omitted d0*x term of the Kahan form, hblpf.c:1026-1043, and
 *                        the `fabs(sum) < is_subnorm_reject` (== 1.0) threshold, hblpf.c:915/1046)
 *   orc_hq_process   <- hq_rp_process                       lpf_hilbert_quad.c:129-156
 *   unpack / fade    <- xwave_unpack_csample + unpackers   xwave_reader.c:908-1009, 205-239,
 *                                                           unpack_lsb.h:53-125
 *   graph            <- amod_process_samples DSP loop       adv_modulator.c:604-753,
 *                       dsp_master/shift/pm                 adv_modulator.c:485-583
 *   render           <- sound_render_value / _recalc        sound_render.c:691-915 / 499-581,
 *                       ns_fir / ns_iir                     sound_render.c:403-489
 *   MT19937          <- mt_jrnd.c:28-256
 *
 * PARITY STATUS (see DESIGN.md "Oracle"):
 *   - MT19937: pinned bit-exact against the reference's own known-answer test
 *     (mersene_twister/test_mt_jrnd, 1000 outputs of init_by_array) and against
 *     oracle/_ref/libref_mt.so compiled from the reference mt_jrnd.c.
 *   - Filter / shaper coefficient tables: extracted bit-exactly from hblpf.c / sound_render.c
 *     (tools/gen_tables.py, tests/golden/tables.json).
 *   - IIR / Hilbert: cross-checked against scipy.signal.lfilter (an independent implementation of
 *     the same difference equation) to floating-point tolerance, and by the analytic-signal
 *     property of SURVEY 4.  The remaining stages (graph, render) are PARITY UNPINNED at bit
 *     level: the reference keeps no fixtures for them and its sources cannot be built here
 *     without Win32 stand-in headers (cmalloc.h/fp_check.h/atomic.h include <windows.h>), which
 *     this build is not allowed to write.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/icw.h"
#include "orc_tables.inc"

#define ORC_PI     (3.1415926535897932384626433832795029)   /* in_cwave.h:144 */
#define ORC_SQRT2  (1.4142135623730950488016887242097)      /* adv_modulator.c:44 */
#define ORC_SQRT6  (2.4494897427831780981972840747059)      /* sound_render.c:50 */

static double u2d(unsigned long long u) { double d; memcpy(&d, &u, 8); return d; }

/* ------------------------------------------------------------------ MT19937 (mt_jrnd.c) -- */
#define MT_N 624
#define MT_M 397
typedef struct { uint32_t st[MT_N]; int next; int left; } orc_mt;

static void mt_seed(orc_mt *m, uint32_t seed)
{
    m->st[0] = seed;
    for (uint32_t j = 1; j < MT_N; ++j)
        m->st[j] = 1812433253u * (m->st[j - 1] ^ (m->st[j - 1] >> 30)) + j;
    m->left = 1;
    m->next = 0;
}

static void mt_init_key(orc_mt *m, const uint32_t *key, uint32_t klen)
{
    mt_seed(m, 19650218u);
    uint32_t i = 1, j = 0, k = (MT_N > klen ? MT_N : klen);
    for (; k; --k) {
        m->st[i] = (m->st[i] ^ ((m->st[i - 1] ^ (m->st[i - 1] >> 30)) * 1664525u)) + key[j] + j;
        if (++i >= MT_N) { m->st[0] = m->st[MT_N - 1]; i = 1; }
        if (++j >= klen) j = 0;
    }
    for (k = MT_N - 1; k; --k) {
        m->st[i] = (m->st[i] ^ ((m->st[i - 1] ^ (m->st[i - 1] >> 30)) * 1566083941u)) - i;
        if (++i >= MT_N) { m->st[0] = m->st[MT_N - 1]; i = 1; }
    }
    m->st[0] = 0x80000000u;
    m->left = 1;
}

static uint32_t mt_twist(uint32_t u, uint32_t v)
{
    uint32_t y = (u & 0x80000000u) | (v & 0x7fffffffu);
    return (y >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
}

static uint32_t mt_u32(orc_mt *m)
{
    if (--m->left == 0) {
        int i;
        for (i = 0; i < MT_N - MT_M; ++i) m->st[i] = m->st[i + MT_M] ^ mt_twist(m->st[i], m->st[i + 1]);
        for (; i < MT_N - 1; ++i) m->st[i] = m->st[i + MT_M - MT_N] ^ mt_twist(m->st[i], m->st[i + 1]);
        m->st[MT_N - 1] = m->st[MT_M - 1] ^ mt_twist(m->st[MT_N - 1], m->st[0]);
        m->left = MT_N;
        m->next = 0;
    }
    uint32_t y = m->st[m->next++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static double mt_dsemi(orc_mt *m)
{
    uint32_t a = mt_u32(m) >> 5, b = mt_u32(m) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

static double mt_dsopen(orc_mt *m)
{
    double r;
    do { r = mt_dsemi(m) * 2.0 - 1.0; } while (-1.0 == r || 1.0 == r);
    return r;
}

/* ------------------------------------------ FP-exception census (fp_check.c:52-100) ------ */
/* FP_EXCEPT_STATS (fp_check.h:62-72): total, snan, qnan, ninf, nden, pden, pinf.  FC(v) returns v
 * unless it is a NaN / denormal (-> 0.0) or an infinity (-> +-INF_HUGE_VALUE = +-65535.0,
 * fp_check.h:60), counting the class when the census is enabled.  _fpclass: a NaN with the quiet
 * bit (mantissa bit 51) clear is signaling. */
typedef struct { int on; uint32_t c[ICW_FES_N]; } orc_fes;

static double fc(double v, orc_fes *f)
{
    if (!f->on) return v;
    uint64_t u;
    memcpy(&u, &v, 8);
    const unsigned ex = (unsigned)((u >> 52) & 0x7ffu);
    const uint64_t man = u & 0xfffffffffffffULL;
    const int neg = (int)(u >> 63);
    if (ex == 0x7ffu) {
        ++f->c[0];
        if (man) { ++f->c[(man >> 51) & 1u ? 2 : 1]; return 0.0; }
        if (neg) { ++f->c[3]; return -65535.0; }
        ++f->c[6];
        return 65535.0;
    }
    if (ex == 0u && man) { ++f->c[0]; ++f->c[neg ? 4 : 5]; return 0.0; }
    return v;
}

/* ------------------------------------------------------------ HB LPF IIR (hblpf.c) -------- */
typedef struct {
    double pc[ICW_MAX_IIR_ORDER], pd[ICW_MAX_IIR_ORDER], pz[ICW_MAX_IIR_ORDER], d0;
    int nord, ix, kahan, subn;
    uint64_t sncnt;
    orc_fes *fes;                      /* the converter's census (mc->fes_hilb_left / _right) */
} orc_iir;

static void iir_init(orc_iir *f, int type, int kahan, int subn)
{
    memset(f, 0, sizeof(*f));
    f->nord = orc_hb_order[type];
    double a0 = u2d(orc_hb_a[type][0]);
    f->d0 = u2d(orc_hb_b[type][0]) / a0;
    for (int i = 0; i < f->nord; ++i) {
        f->pc[i] = -u2d(orc_hb_a[type][i + 1]) / a0;
        f->pd[i] = u2d(orc_hb_b[type][i + 1]) / a0;
    }
    f->kahan = kahan;
    f->subn = subn;
}

static void iir_reset(orc_iir *f)
{
    for (int i = 0; i < f->nord; ++i) f->pz[i] = 0.0;
    f->ix = 0;
    f->sncnt = 0;
}

typedef struct { double S, C, Y, T; } kh;
static inline void kh_step(double x, kh *k)
{
    k->Y = x - k->C;
    k->T = k->S + k->Y;
    k->C = (k->T - k->S) - k->Y;
    k->S = k->T;
}

/* kahan_step_fes (hblpf.c:995-1005) */
static inline void kh_step_fc(double x, kh *k, orc_fes *fe)
{
    k->Y = fc(x - k->C, fe);
    k->T = fc(k->S + k->Y, fe);
    k->C = fc(fc(k->T - k->S, fe) - k->Y, fe);
    k->S = k->T;
}

/* the WITH FP CHECKS branches of iir_rp_process_baseline / _kahan (hblpf.c:928-950, 1058-1095) */
static double iir_baseline_fc(double x, orc_iir *f)
{
    orc_fes *fe = f->fes;
    double si = x, so = 0.0;
    int k = f->ix;
    for (int i = 0; i < f->nord; ++i) {
        if (k == 0) k = f->nord;
        --k;
        si = fc(si + fc(f->pz[k] * f->pc[i], fe), fe);
        so = fc(so + fc(f->pz[k] * f->pd[i], fe), fe);
    }
    if (f->subn && fabs(si) < 1.0) { si = 0.0; ++f->sncnt; }
    f->pz[f->ix] = si;
    if (++f->ix >= f->nord) f->ix = 0;
    return fc(fc(si * f->d0, fe) + so, fe);
}

static double iir_kahan_fc(double x, orc_iir *f)
{
    orc_fes *fe = f->fes;
    kh si, so;
    double t;
    int k = f->ix;
    si.S = x; si.C = 0.0;
    if (k == 0) k = f->nord;
    --k;
    t = fc(f->pz[k] * f->pc[0], fe);
    kh_step_fc(t, &si, fe);
    so.S = fc(f->pz[k] * f->pd[0], fe); so.C = 0.0;
    kh_step_fc(fc(t * f->d0, fe), &so, fe);
    for (int i = 1; i < f->nord; ++i) {
        if (k == 0) k = f->nord;
        --k;
        t = fc(f->pz[k] * f->pc[i], fe);
        kh_step_fc(t, &si, fe);
        kh_step_fc(fc(f->pz[k] * f->pd[i], fe), &so, fe);
        kh_step_fc(fc(t * f->d0, fe), &so, fe);
    }
    if (f->subn && fabs(si.S) < 1.0) { si.S = 0.0; ++f->sncnt; }
    f->pz[f->ix] = si.S;
    if (++f->ix >= f->nord) f->ix = 0;
    return so.S;
}

static double iir_baseline(double x, orc_iir *f)
{
    double si = x, so = 0.0;
    int k = f->ix;
    for (int i = 0; i < f->nord; ++i) {
        if (k == 0) k = f->nord;
        --k;
        si += f->pz[k] * f->pc[i];
        so += f->pz[k] * f->pd[i];
    }
    if (f->subn && fabs(si) < 1.0) { si = 0.0; ++f->sncnt; }
    f->pz[f->ix] = si;
    if (++f->ix >= f->nord) f->ix = 0;
    return si * f->d0 + so;
}

static double iir_kahan(double x, orc_iir *f)
{
    kh si, so;
    double t;
    int k = f->ix;
    si.S = x; si.C = 0.0;
    if (k == 0) k = f->nord;
    --k;
    t = f->pz[k] * f->pc[0];
    kh_step(t, &si);
    so.S = f->pz[k] * f->pd[0]; so.C = 0.0;
    kh_step(t * f->d0, &so);
    for (int i = 1; i < f->nord; ++i) {
        if (k == 0) k = f->nord;
        --k;
        t = f->pz[k] * f->pc[i];
        kh_step(t, &si);
        kh_step(f->pz[k] * f->pd[i], &so);
        kh_step(t * f->d0, &so);
    }
    if (f->subn && fabs(si.S) < 1.0) { si.S = 0.0; ++f->sncnt; }
    f->pz[f->ix] = si.S;
    if (++f->ix >= f->nord) f->ix = 0;
    return so.S;
}

static inline double iir_run(double x, orc_iir *f)
{
    if (f->fes && f->fes->on) return f->kahan ? iir_kahan_fc(x, f) : iir_baseline_fc(x, f);
    return f->kahan ? iir_kahan(x, f) : iir_baseline(x, f);
}

/* ------------------------------------------------- quadrature Hilbert (lpf_hilbert_quad.c) */
typedef struct { orc_iir I, Q; unsigned k; } orc_hq;

static void hq_process(double x, double *oI, double *oQ, orc_hq *h)
{
    switch (h->k) {
    case 0: *oI =  iir_run( x, &h->I) * 2.0; *oQ =  iir_run(0.0, &h->Q) * 2.0; break;
    case 1: *oI = -iir_run(-x, &h->Q) * 2.0; *oQ =  iir_run(0.0, &h->I) * 2.0; break;
    case 2: *oI = -iir_run(-x, &h->I) * 2.0; *oQ = -iir_run(0.0, &h->Q) * 2.0; break;
    default:*oI =  iir_run( x, &h->Q) * 2.0; *oQ = -iir_run(0.0, &h->I) * 2.0; break;
    }
    h->k = (h->k + 1) & 3;
}

/* -------------------------------------------------------------- render (sound_render.c) --- */
typedef struct {
    icw_render_cfg cfg;
    int is24;
    double dth_mul, prev_rnd, hi, lo, norm_mul, round_offset, prev_ns_err;
    int sign_delta, norm_shift;
    int ns_kind, ns_n, ns_ix;
    double ns_c[2 * ICW_MAX_NS_TAPS], ns_e[ICW_MAX_NS_TAPS], ns_o[ICW_MAX_NS_TAPS];
    orc_mt mt;
    orc_fes fes;                       /* mc->fes_sr_left / _right */
} orc_render;

static void render_recalc(orc_render *r)
{
    r->dth_mul = pow(2.0, r->cfg.dth_bits) - 1.0;
    r->prev_rnd = 0.0;
    if (r->cfg.quantz_type == ICW_QUANTZ_MID_TREAD) { r->round_offset = 0.5; r->sign_delta = 0; }
    else { r->round_offset = 0.0; r->sign_delta = -1; }
    if (r->is24) {
        int64_t hib = 0x800000LL;
        r->norm_shift = 24 - (int)r->cfg.sign_bits24;
        hib >>= r->norm_shift;
        r->hi = (double)hib;
        r->lo = -(double)(hib + 1 + r->sign_delta);
        r->norm_mul = (r->norm_shift < 8) ? (double)(0x100 >> r->norm_shift)
                                           : 1.0 / (double)(1ULL << (r->norm_shift - 8));
    } else {
        int64_t hib = 0x8000LL;
        r->norm_shift = 16 - (int)r->cfg.sign_bits16;
        hib >>= r->norm_shift;
        r->hi = (double)hib;
        r->lo = -(double)(hib + 1 + r->sign_delta);
        r->norm_mul = 1.0 / (double)(1ULL << r->norm_shift);
    }
    r->lo -= (double)r->sign_delta;
    if (r->cfg.nshape_type > ICW_NSHAPE_MAX) r->cfg.nshape_type = ICW_NSHAPE_FLAT;
    int t = (int)r->cfg.nshape_type;
    r->ns_kind = orc_ns_kind[t];
    r->ns_n = orc_ns_n[t];
    int nc = r->ns_kind == 2 ? 2 * r->ns_n : r->ns_n;
    for (int i = 0; i < nc; ++i) r->ns_c[i] = u2d(orc_ns_c[t][i]);
    for (int i = 0; i < ICW_MAX_NS_TAPS; ++i) r->ns_e[i] = r->ns_o[i] = 0.0;
    r->ns_ix = 0;
    r->prev_ns_err = 0.0;
}

static void render_init(orc_render *r, const icw_render_cfg *cfg, int is24, uint32_t seed)
{
    memset(r, 0, sizeof(*r));
    mt_seed(&r->mt, seed);
    r->cfg = *cfg;
    r->is24 = is24;
    render_recalc(r);
}

/* ns_empty / ns_fir / ns_iir (sound_render.c:396-489); FC branches at 428-433, 474-486 */
static double ns_filter(double val, orc_render *r)
{
    double res = 0.0;
    unsigned ib, ic, n = (unsigned)r->ns_n;
    orc_fes *fe = &r->fes;
    if (r->ns_kind == 0) return 0.0;
    if (r->ns_ix) --r->ns_ix; else r->ns_ix = (int)n - 1;
    if (fe->on) {
        r->ns_e[ib = (unsigned)r->ns_ix] = fc(val, fe);
        if (r->ns_kind == 1) {
            for (ic = 0; ic < n; ++ic) {
                res = fc(res + fc(r->ns_c[ic] * r->ns_e[ib], fe), fe);
                if (++ib >= n) ib = 0;
            }
        } else {
            for (ic = 0; ic < n; ++ic) {
                res = fc(res + fc(fc(r->ns_c[ic] * r->ns_e[ib], fe) - fc(r->ns_c[ic + n] * r->ns_o[ib], fe), fe), fe);
                if (++ib >= n) ib = 0;
            }
            r->ns_o[(r->ns_ix ? r->ns_ix : (int)n) - 1] = res;
        }
        return res;
    }
    r->ns_e[ib = (unsigned)r->ns_ix] = val;
    if (r->ns_kind == 1) {
        for (ic = 0; ic < n; ++ic) {
            res += r->ns_c[ic] * r->ns_e[ib];
            if (++ib >= n) ib = 0;
        }
    } else {
        for (ic = 0; ic < n; ++ic) {
            res += r->ns_c[ic] * r->ns_e[ib] - r->ns_c[ic + n] * r->ns_o[ib];
            if (++ib >= n) ib = 0;
        }
        r->ns_o[(r->ns_ix ? r->ns_ix : (int)n) - 1] = res;
    }
    return res;
}

/* returns the integer sample (before the norm_shift) and writes 2/3 bytes */
static int render_value(unsigned char **buf, double input, uint32_t *clips, double *peak, orc_render *r)
{
    double rnd = 0.0, tr, q;
    int delta, val;
    switch (r->cfg.render_type) {
    case ICW_RENDER_RPDF: rnd = mt_dsopen(&r->mt) / ORC_SQRT2; break;
    case ICW_RENDER_TPDF: rnd = mt_dsopen(&r->mt); rnd += mt_dsopen(&r->mt); rnd /= 2.0; break;
    case ICW_RENDER_STPDF: rnd = ((tr = mt_dsopen(&r->mt)) - r->prev_rnd) / 2.0; r->prev_rnd = tr; break;
    case ICW_RENDER_GAUSS:
        rnd = mt_dsopen(&r->mt);
        for (int i = 1; i < 12; ++i) rnd += mt_dsopen(&r->mt);
        rnd /= (2.0 * ORC_SQRT6);
        break;
    default: break;
    }
    orc_fes *fe = &r->fes;
    if (fe->on) {
        /* sound_render.c:815-870 with FC: the dither sums are multiples of 2^-53 below 12 in
         * magnitude (never special), so their FC() are identities and are not restated */
        input = fc(fc(input * r->norm_mul, fe) - r->prev_ns_err, fe);
        q = fc(input + fc(rnd * r->dth_mul, fe), fe);
        if (q < 0.0) { q = fc(q - r->round_offset, fe); delta = r->sign_delta; }
        else { q = fc(q + r->round_offset, fe); delta = 0; }
    } else {
        input = (input * r->norm_mul) - r->prev_ns_err;
        q = input + (rnd * r->dth_mul);
        if (q < 0.0) { q -= r->round_offset; delta = r->sign_delta; }
        else { q += r->round_offset; delta = 0; }
    }
    if (peak) {
        double cv = fabs(q) / r->hi;
        cv = cv ? 20.0 * log10(cv) : ICW_SR_ZERO_SIGNAL_DB;
        if (cv > *peak) *peak = cv;
    }
    if (q >= r->hi) { q = r->hi - 1.0; if (clips) ++*clips; }
    if (q <= r->lo) { q = r->lo + 1.0; if (clips) ++*clips; }
    val = ((int)q) + delta;
    r->prev_ns_err = ns_filter(fe->on ? fc((double)val - input, fe) : (double)val - input, r);
    val <<= r->norm_shift;
    *(*buf)++ = (unsigned char)(val);
    *(*buf)++ = (unsigned char)(val >> 8);
    if (r->is24) *(*buf)++ = (unsigned char)(val >> 16);
    return val;
}

/* ------------------------------------------------------------------- one stream ---------- */
typedef struct { double lre, lim, rre, rim; } lrc;

/* FIR Hilbert converter (icw_set_fir_hilbert; the CWAVE converter cwave.h:40,56-58 names by its
 * order k_M and Kaiser parameter k_beta -- no reference implementation, parity unpinned).  Per
 * channel a ring of the last M+1 inputs (newest at head), kept twice (slots h and h + M + 1), so
 * every read of the last M+1 is one contiguous index -- no modulo per tap (a test-speed change only:
 * the same values in the same fma order) */
#define ORC_FIR_MAX 4096
typedef struct {
    int M, nt, head;
    double g[ORC_FIR_MAX / 4 + 1];
    double x[2][2 * (ORC_FIR_MAX + 1)];
} orc_fir;

typedef struct orc_stream {
    icw_config cfg;
    orc_fir fir;
    orc_fes fes_hilb[2];               /* mc->fes_hilb_left / _right (in_cwave.c:72-79) */
    icw_node nodes[64];
    int n_nodes;
    uint64_t n_frame;
    lrc bus[ICW_N_INPUTS];
    orc_hq hq[2];
    orc_render rd[2];
    int64_t pos, n_samples, n_fade_in, n_fade_out;
    uint32_t clips[2];
    double peak[2];
    /* the meters render_value updates: this stream's own clips / peak, or another stream's when
     * orc_share_meters makes them one accumulator -- the reference's single am.l/r_clips and
     * am.l/r_peak, which every decoding context feeds (adv_modulator.c:54-55, 757-758) */
    uint32_t *am_clips;
    double *am_peak;
} orc_stream;

static double unpack1(const unsigned char *p, unsigned fmt)
{
    switch (fmt) {
    case ICW_FMT_U8: return 256.0 * (double)((int8_t)(p[0] - 0x80u));
    case ICW_FMT_I16: return (double)(int16_t)(p[0] | (p[1] << 8));
    case ICW_FMT_I24: {
        int v = ((int)(((uint32_t)p[0] << 8) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 24))) >> 8;
        return ((double)v) / 256.0;
    }
    case ICW_FMT_I32: {
        int v = (int)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
        return ((double)v) / 65536.0;
    }
    default: {
        uint32_t u = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        float f; memcpy(&f, &u, 4);
        return 32768.0 * (double)f;
    }
    }
}

/* CWAVE unpackers (xwave_reader.c:171-200; unpack_lsb.h:53-125): I/Q as stored, no scaling */
static uint32_t le32(const unsigned char *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static double le_f32(const unsigned char *p)
{
    uint32_t u = le32(p);
    float f;
    memcpy(&f, &u, 4);
    return (double)f;
}

static void unpack_iq(const unsigned char *p, unsigned fmt, double *vI, double *vQ)
{
    switch (fmt) {
    case ICW_FMT_CW_F64: {
        uint64_t a = (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32);
        uint64_t b = (uint64_t)le32(p + 8) | ((uint64_t)le32(p + 12) << 32);
        memcpy(vI, &a, 8);
        memcpy(vQ, &b, 8);
        break;
    }
    case ICW_FMT_CW_I16:
        *vI = (double)(int16_t)(p[0] | (p[1] << 8));
        *vQ = (double)(int16_t)(p[2] | (p[3] << 8));
        break;
    case ICW_FMT_CW_I16_F32:
        *vI = (double)(int16_t)(p[0] | (p[1] << 8));
        *vQ = le_f32(p + 2);
        break;
    default:
        *vI = le_f32(p);
        *vQ = le_f32(p + 4);
        break;
    }
}

/* test hooks: n samples of real format fmt at src -> the scaled doubles unpack1 gives (pre-fade),
 * and n complex samples of CWAVE format fmt -> I / Q (tests/test_reader_pinned.py pins both against
 * the reference's own unpack_lsb.h, compiled by `make -C oracle ref`) */
static unsigned fmt_size(unsigned fmt);
void orc_unpack_real(unsigned fmt, const unsigned char *src, size_t n, double *dst)
{
    for (size_t i = 0; i < n; ++i) dst[i] = unpack1(src + i * fmt_size(fmt), fmt);
}

void orc_unpack_cw(unsigned fmt, const unsigned char *src, size_t n, double *vI, double *vQ)
{
    for (size_t i = 0; i < n; ++i) unpack_iq(src + i * fmt_size(fmt), fmt, vI + i, vQ + i);
}

/* HRW_FMT_* sample sizes and CWAVE cw_slen (xwave_reader.c:246-252) */
static unsigned fmt_size(unsigned fmt)
{
    static const unsigned sz[9] = {1, 2, 3, 4, 4, 16, 4, 6, 8};
    return fmt < 9 ? sz[fmt] : 0;
}

/* I0(x) = sum_k ((x/2)^k / k!)^2 */
static double orc_i0(double x)
{
    double half = x / 2.0, sum = 1.0, term = 1.0;
    int k;
    for (k = 1; k < 1000; ++k) {
        double t2;
        term *= half / (double)k;
        t2 = term * term;
        sum += t2;
        if (t2 < sum * 1e-17) break;
    }
    return sum;
}

/* taps g[k] of odd tap m = 2k+1 <= M/2: 2 w(m) / (pi m), Kaiser w(m) = I0(beta sqrt(1-(m/c)^2)) / I0(beta) */
int orc_fir_taps(int M, double beta, double *g, int n)
{
    int c = M / 2, nt = (c + 1) / 2, k;
    double ib;
    if (M < 2 || M > ORC_FIR_MAX || (M & 1) || n < nt || beta < 0.0) return -1;
    ib = orc_i0(beta);
    for (k = 0; k < nt; ++k) {
        int m = 2 * k + 1;
        double r = (double)m / (double)c;
        g[k] = (2.0 / (ORC_PI * (double)m)) * (orc_i0(beta * sqrt(1.0 - r * r)) / ib);
    }
    return nt;
}

static void fir_reset(orc_fir *f)
{
    memset(f->x, 0, sizeof(f->x));
    f->head = 0;
}

/* one input of channel ch -> (I, Q): I = x[n-c], Q = sum over odd m <= c of g_m (x[n-c-m] - x[n-c+m]),
 * ascending m, one fma per tap from +0.0 */
static void fir_process(orc_fir *f, int ch, double x, double *oI, double *oQ)
{
    int L = f->M + 1, c = f->M / 2, k;
    double *r = f->x[ch];
    int h = f->head;                                /* slot of x[n]; advanced after both channels */
    const double *p = r + h + L;                    /* x[n - j] = p[-j] for 0 <= j <= M */
    double acc = 0.0;
    r[h] = x;
    r[h + L] = x;
    for (k = 0; k < f->nt; ++k) {
        int m = 2 * k + 1;
        double a = p[-(c + m)], b = p[-(c - m)];
        acc = fma(f->g[k], a - b, acc);
    }
    *oI = p[-c];
    *oQ = acc;
}

int orc_set_fir(orc_stream *s, int M, double beta)
{
    if (M == 0) { s->fir.M = 0; return 0; }
    if (orc_fir_taps(M, beta, s->fir.g, ORC_FIR_MAX / 4 + 1) < 0) return -1;
    s->fir.M = M;
    s->fir.nt = (M / 2 + 1) / 2;
    fir_reset(&s->fir);
    return 0;
}

/* amod_init normalisation (adv_modulator.c:216-331), shared with the product by semantics */
static int graph_accept(icw_node *n, int cnt)
{
    if (cnt <= 0 || n[0].mode != ICW_MODE_MASTER) return 0;
    int was_master = 0;
    for (int i = 0; i < cnt; ++i) {
        icw_node *t = &n[i];
        if (t->lock_gain) { t->gain[1] = t->gain[0]; t->iq_invert[1] = t->iq_invert[0]; }
        switch (t->mode) {
        case ICW_MODE_MASTER: if (was_master) return 0; was_master = 1; break;
        case ICW_MODE_SHIFT:
            if (t->lock_shift) {
                t->fr_shift[1] = t->sign_lock_shift ? -t->fr_shift[0] : t->fr_shift[0];
                t->is_shift[1] = t->is_shift[0];
            }
            break;
        case ICW_MODE_PM:
            if (t->lock_freq) { t->pm_freq[1] = t->pm_freq[0]; t->is_pm[1] = t->is_pm[0]; }
            if (t->lock_phase) t->pm_phase[1] = t->pm_phase[0];
            if (t->lock_level) t->pm_level[1] = t->pm_level[0];
            if (t->lock_angle) t->pm_angle[1] = t->pm_angle[0];
            break;
        case ICW_MODE_MIX: break;
        default: return 0;
        }
    }
    return 1;
}

static void default_master(icw_node *n)
{
    memset(n, 0, sizeof(*n));
    n->mode = ICW_MODE_MASTER;
    n->gain[0] = n->gain[1] = 0.8;           /* DEF_GAIN_MASTER in_cwave.h:167 */
    n->tout[0] = n->tout[1] = ICW_S_ADD_REIM;
    n->inputs[0] = 1;
    n->lock_gain = 1;
}

orc_stream *orc_stream_new(const icw_config *cfg, const icw_node *nodes, int n_nodes, int *accepted)
{
    orc_stream *s = (orc_stream *)calloc(1, sizeof(orc_stream));
    if (!s) return NULL;
    s->cfg = *cfg;
    if (n_nodes > 64) n_nodes = 0;
    if (n_nodes > 0) memcpy(s->nodes, nodes, sizeof(icw_node) * (size_t)n_nodes);
    int ok = graph_accept(s->nodes, n_nodes);
    if (!ok) { default_master(&s->nodes[0]); s->n_nodes = 1; }
    else s->n_nodes = n_nodes;
    if (accepted) *accepted = ok;
    for (int c = 0; c < 2; ++c) {
        iir_init(&s->hq[c].I, (int)cfg->hilbert_type, cfg->iir_kahan, cfg->iir_subnorm_reject);
        iir_init(&s->hq[c].Q, (int)cfg->hilbert_type, cfg->iir_kahan, cfg->iir_subnorm_reject);
        s->hq[c].k = 0;
        s->fes_hilb[c].on = cfg->fp_check != 0;
        s->hq[c].I.fes = s->hq[c].Q.fes = &s->fes_hilb[c];
    }
    render_init(&s->rd[0], &cfg->render, cfg->need24bits, cfg->seed_left);
    render_init(&s->rd[1], &cfg->render, cfg->need24bits, cfg->seed_right);
    s->rd[0].fes.on = s->rd[1].fes.on = cfg->fp_check != 0;
    s->peak[0] = s->peak[1] = ICW_SR_ZERO_SIGNAL_DB;
    s->am_clips = s->clips;
    s->am_peak = s->peak;
    s->n_samples = INT64_MAX / 4;
    return s;
}

void orc_stream_free(orc_stream *s) { free(s); }

/* raw MT19937 state of render channel ch (test hook): 624 words and the index of the next word
 * (624: the next draw twists first), the device's representation */
void orc_set_mt(orc_stream *s, int ch, const uint32_t *words, int idx)
{
    orc_mt *m = &s->rd[ch].mt;
    memcpy(m->st, words, sizeof(m->st));
    m->next = idx >= MT_N ? 0 : idx;
    m->left = idx >= MT_N ? 1 : MT_N + 1 - idx;
}

/* a new track's sample format (mod_context_fopen -> xwave_reader_create, in_cwave.c:207-236) */
void orc_set_input(orc_stream *s, uint32_t sample_rate, uint32_t fmt, uint32_t channels)
{
    s->cfg.sample_rate = sample_rate;
    s->cfg.in_format = fmt;
    s->cfg.in_channels = channels;
}

/* Live edits, applied between blocks as the GUI thread's edits land between frames
 * of amod_process_samples at block granularity.
 * The DSP list: amod_add_lastdsp / amod_del_* (adv_modulator.c:358-400) and the node-field
 * writes, as a whole new list normalised like amod_init; a list amod_init would reject is refused
 * and the running one stays.  am.is_bypass_list: amod_set_bypass_list_flag (:422-425).
 * Bus slots: amod_del_lastdsp / amod_del_dsplist and amod_set_output_plug go through
 * replace_output_plug (adv_modulator.c:176-209), which zeroes the removed or re-plugged node's old
 * output slot in every context (mod_context_clear_all_inouts, in_cwave.c:255-261).  A whole-list
 * edit is matched to those primitives by position: an old Shift / PM / Mix node whose position is
 * gone, holds a node of another mode, or whose n_out changed had its old slot cleared.  Any other
 * slot keeps its value (orc_clear_inout is the primitive itself). */
void orc_clear_inout(orc_stream *s, int slot)
{
    if (slot >= 0 && slot < ICW_N_INPUTS) memset(&s->bus[slot], 0, sizeof(s->bus[slot]));
}

int orc_set_graph(orc_stream *s, const icw_node *nodes, int n_nodes, int bypass)
{
    icw_node tmp[64];
    if (n_nodes <= 0 || n_nodes > 64) return 0;
    memcpy(tmp, nodes, sizeof(icw_node) * (size_t)n_nodes);
    if (!graph_accept(tmp, n_nodes)) return 0;
    for (int i = 0; i < s->n_nodes; ++i) {
        const icw_node *o = &s->nodes[i];
        if (o->mode != ICW_MODE_SHIFT && o->mode != ICW_MODE_PM && o->mode != ICW_MODE_MIX) continue;
        if (i >= n_nodes || tmp[i].mode != o->mode || tmp[i].n_out != o->n_out) orc_clear_inout(s, o->n_out);
    }
    memcpy(s->nodes, tmp, sizeof(icw_node) * (size_t)n_nodes);
    s->n_nodes = n_nodes;
    s->cfg.bypass_list = bypass ? 1 : 0;
    return 1;
}

/* The list primitives themselves, as the GUI calls them (amod_gui_control.c:1125, 1165, 1172,
 * 1858), one at a time.  replace_output_plug (adv_modulator.c:176-209): a Shift / PM / Mix node's
 * old output slot is cleared -- also when it is re-plugged to the same slot, and with n = -1 the
 * node keeps its n_out but the slot is cleared all the same; a Master clears nothing. */
static void replace_output_plug(orc_stream *s, icw_node *n, int to)
{
    int nrem = -1;
    if (n->mode == ICW_MODE_SHIFT || n->mode == ICW_MODE_PM || n->mode == ICW_MODE_MIX) {
        nrem = n->n_out;
        if (to >= 0) n->n_out = to;
    }
    if (nrem >= 0) orc_clear_inout(s, nrem);
}

/* amod_del_lastdsp (adv_modulator.c:378-390): the head (Master) stays */
void orc_del_lastdsp(orc_stream *s)
{
    if (s->n_nodes > 1) {
        --s->n_nodes;
        replace_output_plug(s, &s->nodes[s->n_nodes], -1);
    }
}

/* amod_del_dsplist (adv_modulator.c:360-374): tail first, down to the head */
void orc_del_dsplist(orc_stream *s)
{
    while (s->n_nodes > 1) orc_del_lastdsp(s);
}

/* amod_add_lastdsp (adv_modulator.c:394-411) and the GUI's field writes of the new node (a Master
 * cannot be created there: create_node_dsp returns NULL, :112-123); the L/R locks are applied as
 * amod_init applies them.  Returns 0 if refused. */
int orc_add_lastdsp(orc_stream *s, const icw_node *node)
{
    icw_node tmp[64];
    if (!node || node->mode == ICW_MODE_MASTER || s->n_nodes >= 64) return 0;
    memcpy(tmp, s->nodes, sizeof(icw_node) * (size_t)s->n_nodes);
    tmp[s->n_nodes] = *node;
    if (!graph_accept(tmp, s->n_nodes + 1)) return 0;
    s->nodes[s->n_nodes] = tmp[s->n_nodes];
    ++s->n_nodes;
    return 1;
}

/* amod_set_output_plug (adv_modulator.c:436-441) on node `index` of the list */
void orc_set_output_plug(orc_stream *s, int index, int to)
{
    if (index >= 0 && index < s->n_nodes) replace_output_plug(s, &s->nodes[index], to);
}

/* srenders_set_vcfg (in_cwave.c:457-469) -> sound_render_setup (sound_render.c:625-629): copy the
 * config, sound_render_recalc (prev_rnd, shaper rings, prev_ns_err restart; the MT goes on) */
void orc_set_render(orc_stream *s, const icw_render_cfg *cfg)
{
    for (int c = 0; c < 2; ++c) {
        s->rd[c].cfg = *cfg;
        render_recalc(&s->rd[c]);
    }
    s->cfg.render = *cfg;
}

/* mod_context_change_all_hilberts_filter (in_cwave.c:186-199): a different type destroys and
 * re-creates both converters (hq_rp_create, lpf_hilbert_quad.c:80-88: iir_rp_create ->
 * iir_rp_setcfg + iir_rp_reset, hblpf.c:828-860; sampe_ix = 0) */
void orc_set_hilbert_filter(orc_stream *s, unsigned type)
{
    if (type == s->cfg.hilbert_type || type > 5) return;
    s->cfg.hilbert_type = type;
    for (int c = 0; c < 2; ++c) {
        iir_init(&s->hq[c].I, (int)type, s->cfg.iir_kahan, s->cfg.iir_subnorm_reject);
        iir_init(&s->hq[c].Q, (int)type, s->cfg.iir_kahan, s->cfg.iir_subnorm_reject);
        s->hq[c].k = 0;
        s->hq[c].I.fes = s->hq[c].Q.fes = &s->fes_hilb[c];
    }
}

/* mod_context_change_all_hilberts_config (in_cwave.c:171-182) -> hq_rp_setcfg -> iir_rp_setcfg
 * (hblpf.c:1117-1127): summation and reject switched, rings kept, subnorm_cnt = 0 */
void orc_set_hilbert_config(orc_stream *s, int kahan, int subn)
{
    s->cfg.iir_kahan = kahan ? 1 : 0;
    s->cfg.iir_subnorm_reject = subn ? 1 : 0;
    for (int c = 0; c < 2; ++c) {
        orc_iir *f[2] = {&s->hq[c].I, &s->hq[c].Q};
        for (int q = 0; q < 2; ++q) {
            f[q]->kahan = s->cfg.iir_kahan;
            f[q]->subn = s->cfg.iir_subnorm_reject;
            f[q]->sncnt = 0;
        }
    }
}

/* sound_render_set_outbits (sound_render.c:617-621) on both renders: is24bits, then
 * sound_render_recalc (new bounds; prev_rnd, shaper rings, prev_ns_err restart; the MT goes on).
 * mod_context_fopen applies it with the.cfg.need24bits at every track open (in_cwave.c:212, 233-234). */
void orc_set_outbits(orc_stream *s, int need24bits)
{
    for (int c = 0; c < 2; ++c) {
        s->rd[c].is24 = need24bits ? 1 : 0;
        render_recalc(&s->rd[c]);
    }
    s->cfg.need24bits = need24bits ? 1 : 0;
}

/* mod_context_fopen + xwave_reader_create fade/tail arithmetic; returns n_tail */
int64_t orc_stream_open(orc_stream *s, int64_t n_samples, uint32_t fade_in, uint32_t fade_out,
                        uint32_t sec_align, int clr_nframe, int clr_hilb)
{
    int64_t n_tail = 0;
    s->n_samples = n_samples;
    if (sec_align) {
        int64_t mt = (int64_t)s->cfg.sample_rate * (int64_t)sec_align;
        int64_t fr = n_samples % mt;
        n_tail = fr ? mt - fr : 0;
    }
    s->n_fade_in = (int64_t)(((uint64_t)fade_in * (uint64_t)s->cfg.sample_rate) / 1000ULL);
    s->n_fade_out = (int64_t)(((uint64_t)fade_out * (uint64_t)s->cfg.sample_rate) / 1000ULL);
    if (s->n_fade_in + s->n_fade_out >= n_samples) {
        if (n_samples < 300LL) s->n_fade_in = s->n_fade_out = 0;
        else {
            if (s->n_fade_in) s->n_fade_in = n_samples / 3;
            if (s->n_fade_out) s->n_fade_out = n_samples / 3;
        }
    }
    s->pos = 0;
    if (clr_nframe) s->n_frame = 0;
    if (clr_hilb) {
        for (int c = 0; c < 2; ++c) { iir_reset(&s->hq[c].I); iir_reset(&s->hq[c].Q); s->hq[c].k = 0; }
        fir_reset(&s->fir);
    }
    render_recalc(&s->rd[0]);
    render_recalc(&s->rd[1]);
    return n_tail;
}

static double dsp_master(int tout, double re, double im)
{
    switch (tout) {
    case ICW_S_RE: return re;
    case ICW_S_IM: return im;
    case ICW_S_ADD_REIM: return (re + im) / ORC_SQRT2;
    case ICW_S_SUB_REIM: return (re - im) / ORC_SQRT2;
    }
    return 0.0;
}

static void dsp_shift(const icw_node *n, int c, int scaled, double *ore, double *oim, double re, double im, double omega)
{
    if (n->is_shift[c]) {
        double f = n->fr_shift[c], cs, sn, ph;
        int neg = 0;
        if (f < 0.0) { f = -f; neg = 1; }
        if (scaled) f = (double)((unsigned)(f * ((double)ICW_HZ_SCALE) + 0.5));
        ph = fmod(omega * f, 2.0 * ORC_PI);
        cs = cos(ph);
        sn = sin(ph);
        if (neg) sn = -sn;
        *ore = re * cs - im * sn;
        *oim = re * sn + im * cs;
    } else { *ore = re; *oim = im; }
}

static void dsp_pm(const icw_node *n, int c, int scaled, double *ore, double *oim, double re, double im, double omega)
{
    if (n->is_pm[c]) {
        double f = n->pm_freq[c], fp = n->pm_phase[c], fl = n->pm_level[c], fa = n->pm_angle[c], ph;
        if (scaled) f = (double)((unsigned)(f * ((double)ICW_HZ_SCALE) + 0.5));
        ph = fmod(omega * f, 2.0 * ORC_PI);
        double psi = fl * ORC_PI * (sin(ph + fp * ORC_PI) + fa);
        double cs = cos(psi), sn = sin(psi);
        *ore = re * cs - im * sn;
        *oim = re * sn + im * cs;
    } else { *ore = re; *oim = im; }
}

/* Process n_frames frames of raw interleaved input.  out: 2/3-byte LE samples L,R per frame.
 * pre (nullable): the two pre-render doubles per frame.  Returns the frames rendered. */
int orc_process(orc_stream *s, const void *in, unsigned n_frames, void *out, double *pre)
{
    const unsigned char *ip = (const unsigned char *)in;
    unsigned char *op = (unsigned char *)out;
    const icw_config *cfg = &s->cfg;
    unsigned csz = fmt_size(cfg->in_format);
    unsigned nch = cfg->in_channels ? cfg->in_channels : 1;
    unsigned fsz = csz * nch;
    for (unsigned f = 0; f < n_frames; ++f) {
        double omega, lOut = 0.0, rOut = 0.0;
        if (cfg->frmod_scaled) {
            unsigned ssr = cfg->sample_rate * ICW_HZ_SCALE;
            omega = (2.0 * ORC_PI) * ((double)s->n_frame) / ((double)ssr);
            s->n_frame = (s->n_frame + 1) % (uint64_t)ssr;
        } else {
            omega = (2.0 * ORC_PI) * ((double)s->n_frame) / (double)cfg->sample_rate;
            ++s->n_frame;
        }
        /* unpack + fade + Hilbert (xwave_unpack_csample) */
        double fade = -1.0;
        int64_t ix = s->pos;
        if (ix < s->n_fade_in) fade = ((double)ix) / ((double)s->n_fade_in);
        else if (ix > s->n_samples - s->n_fade_out && ix < s->n_samples)
            fade = ((double)(s->n_samples - ix)) / ((double)s->n_fade_out);
        const unsigned char *fp = ip + (size_t)f * fsz;
        if (cfg->in_format >= ICW_FMT_CW_F64) {
            /* complex sample: no Hilbert; mono -> R = L; fade on all four (xwave_reader.c:939-966) */
            lrc *b = &s->bus[0];
            unpack_iq(fp, cfg->in_format, &b->lre, &b->lim);
            if (nch > 1) unpack_iq(fp + csz, cfg->in_format, &b->rre, &b->rim);
            else { b->rre = b->lre; b->rim = b->lim; }
            if (fade >= 0.0) { b->lre *= fade; b->lim *= fade; b->rre *= fade; b->rim *= fade; }
        } else if (s->fir.M) {
            /* FIR Hilbert converter: the analytic signal of a CWAVE file, then as complex input */
            double val = unpack1(fp, cfg->in_format);
            if (fade >= 0.0) val *= fade;
            fir_process(&s->fir, 0, val, &s->bus[0].lre, &s->bus[0].lim);
            if (nch > 1) {
                val = unpack1(fp + csz, cfg->in_format);
                if (fade >= 0.0) val *= fade;
            }
            fir_process(&s->fir, 1, val, &s->bus[0].rre, &s->bus[0].rim);
            s->fir.head = (s->fir.head + 1) % (s->fir.M + 1);
        } else {
            double val = unpack1(fp, cfg->in_format);
            if (fade >= 0.0) val *= fade;
            hq_process(val, &s->bus[0].lre, &s->bus[0].lim, &s->hq[0]);
            if (nch > 1) {
                val = unpack1(fp + csz, cfg->in_format);
                if (fade >= 0.0) val *= fade;
            }
            hq_process(val, &s->bus[0].rre, &s->bus[0].rim, &s->hq[1]);
        }
        ++s->pos;
        /* DSP list, tail -> head */
        for (int ni = cfg->bypass_list ? 0 : s->n_nodes - 1; ni >= 0; --ni) {
            const icw_node *n = &s->nodes[ni];
            lrc d;
            double xt;
            if (cfg->bypass_list) d = s->bus[0];
            else {
                d.lre = d.lim = d.rre = d.rim = 0.0;
                for (int k = 0; k < ICW_N_INPUTS; ++k)
                    if (n->inputs[k]) {
                        d.lre += s->bus[k].lre; d.lim += s->bus[k].lim;
                        d.rre += s->bus[k].rre; d.rim += s->bus[k].rim;
                    }
            }
            switch (n->xch_mode) {
            case ICW_XCH_SWAP:
                xt = d.lre; d.lre = d.rre; d.rre = xt;
                xt = d.lim; d.lim = d.rim; d.rim = xt;
                break;
            case ICW_XCH_LEFTONLY: d.rre = d.lre; d.rim = d.lim; break;
            case ICW_XCH_RIGHTONLY: d.lre = d.rre; d.lim = d.rim; break;
            case ICW_XCH_MIXLR:
                d.lre = d.rre = (d.lre + d.rre) / 2.0;
                d.lim = d.rim = (d.lim + d.rim) / 2.0;
                break;
            default: break;
            }
            if (n->iq_invert[0]) { xt = d.lre; d.lre = d.lim; d.lim = xt; }
            if (n->iq_invert[1]) { xt = d.rre; d.rre = d.rim; d.rim = xt; }
            d.lre *= n->gain[0]; d.lim *= n->gain[0];
            d.rre *= n->gain[1]; d.rim *= n->gain[1];
            lrc *po;
            switch (n->mode) {
            case ICW_MODE_MASTER:
                lOut = dsp_master(n->tout[0], d.lre, d.lim);
                rOut = dsp_master(n->tout[1], d.rre, d.rim);
                break;
            case ICW_MODE_SHIFT:
                po = &s->bus[n->n_out];
                dsp_shift(n, 0, cfg->frmod_scaled, &po->lre, &po->lim, d.lre, d.lim, omega);
                dsp_shift(n, 1, cfg->frmod_scaled, &po->rre, &po->rim, d.rre, d.rim, omega);
                break;
            case ICW_MODE_PM:
                po = &s->bus[n->n_out];
                dsp_pm(n, 0, cfg->frmod_scaled, &po->lre, &po->lim, d.lre, d.lim, omega);
                dsp_pm(n, 1, cfg->frmod_scaled, &po->rre, &po->rim, d.rre, d.rim, omega);
                break;
            case ICW_MODE_MIX:
                s->bus[n->n_out] = d;
                break;
            }
        }
        if (pre) { pre[2 * f] = lOut; pre[2 * f + 1] = rOut; }
        render_value(&op, lOut, &s->am_clips[0], &s->am_peak[0], &s->rd[0]);
        render_value(&op, rOut, &s->am_clips[1], &s->am_peak[1], &s->rd[1]);
    }
    return (int)n_frames;
}

/* s renders into owner's meters from now on (owner: s itself to separate them again): the two
 * decoding contexts of the reference, the.mc_playback and the.mc_transcode (in_cwave.h:473-474),
 * both pass &am.l_clips / &am.l_peak ... to sound_render_value (adv_modulator.c:757-758) */
void orc_share_meters(orc_stream *s, orc_stream *owner)
{
    s->am_clips = owner->clips;
    s->am_peak = owner->peak;
}

/* amod_get_clips_peaks (adv_modulator.c:445-465) on the accumulator s renders into: with reset
 * the clips and peaks are cleared first and the cleared values read back */
void orc_get_clips_peaks(orc_stream *s, int reset, icw_meters *m)
{
    if (reset) {
        s->am_clips[0] = s->am_clips[1] = 0;
        s->am_peak[0] = s->am_peak[1] = ICW_SR_ZERO_SIGNAL_DB;
    }
    m->clips[0] = s->am_clips[0]; m->clips[1] = s->am_clips[1];
    m->peak_db[0] = s->am_peak[0]; m->peak_db[1] = s->am_peak[1];
    m->desubnorm = s->hq[0].I.sncnt + s->hq[0].Q.sncnt + s->hq[1].I.sncnt + s->hq[1].Q.sncnt;
}

void orc_get_meters(orc_stream *s, icw_meters *m)
{
    m->clips[0] = s->am_clips[0]; m->clips[1] = s->am_clips[1];
    m->peak_db[0] = s->am_peak[0]; m->peak_db[1] = s->am_peak[1];
    m->desubnorm = s->hq[0].I.sncnt + s->hq[0].Q.sncnt + s->hq[1].I.sncnt + s->hq[1].Q.sncnt;
}

uint64_t orc_stream_nframe(orc_stream *s) { return s->n_frame; }
/* test hook: place the modulator frame counter (mc->n_frame, in_cwave.h:413) anywhere, e.g. just
 * below the scaled-mode wrap or above a lower rate's scale after a track switch */
void orc_set_nframe(orc_stream *s, uint64_t n) { s->n_frame = n; }

/* census [4][ICW_FES_N]: Hilbert left, right, render left, right */
void orc_get_fp_census(orc_stream *s, uint32_t *out)
{
    const orc_fes *f[4] = {&s->fes_hilb[0], &s->fes_hilb[1], &s->rd[0].fes, &s->rd[1].fes};
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < ICW_FES_N; ++k) out[i * ICW_FES_N + k] = f[i]->c[k];
}

/* Process many independent streams back to back (the timed CPU baseline, bench.py). */
int orc_process_many(orc_stream **ss, int n_streams, const void *in, size_t in_stride,
                     void *out, size_t out_stride, unsigned n_frames)
{
    for (int i = 0; i < n_streams; ++i)
        orc_process(ss[i], (const char *)in + (size_t)i * in_stride, n_frames,
                    (char *)out + (size_t)i * out_stride, NULL);
    return n_streams;
}

/* ------------------------------------------------------------ component entry points ------ */
/* IIR over a block from fresh state; y = filter output, w = post-reject DF-II state (nullable) */
int orc_iir_block(int type, int kahan, int subn, const double *x, int n, double *y, double *w, uint64_t *sncnt)
{
    orc_iir f;
    iir_init(&f, type, kahan, subn);
    iir_reset(&f);
    for (int i = 0; i < n; ++i) {
        y[i] = iir_run(x[i], &f);
        if (w) w[i] = f.pz[(f.ix + f.nord - 1) % f.nord];
    }
    if (sncnt) *sncnt = f.sncnt;
    return 0;
}

/* raw filter coefficients as the IIR uses them: pc[n], pd[n], d0 */
int orc_iir_coeffs(int type, double *pc, double *pd, double *d0)
{
    orc_iir f;
    iir_init(&f, type, 1, 1);
    for (int i = 0; i < f.nord; ++i) { pc[i] = f.pc[i]; pd[i] = f.pd[i]; }
    *d0 = f.d0;
    return f.nord;
}

int orc_hilbert_block(int type, int kahan, int subn, const double *x, int n, double *oI, double *oQ)
{
    orc_hq h;
    iir_init(&h.I, type, kahan, subn); iir_reset(&h.I);
    iir_init(&h.Q, type, kahan, subn); iir_reset(&h.Q);
    h.k = 0;
    for (int i = 0; i < n; ++i) hq_process(x[i], &oI[i], &oQ[i], &h);
    return 0;
}

int orc_render_block(const icw_render_cfg *cfg, int is24, uint32_t seed, const double *x, int n,
                     void *out, int *ival, uint32_t *clips, double *peak)
{
    orc_render r;
    render_init(&r, cfg, is24, seed);
    unsigned char *op = (unsigned char *)out;
    for (int i = 0; i < n; ++i) {
        int v = render_value(&op, x[i], clips, peak, &r);
        if (ival) ival[i] = v;
    }
    return 0;
}

/* MT entry points for the known-answer test */
void *orc_mt_new(void) { return calloc(1, sizeof(orc_mt)); }
void orc_mt_free(void *m) { free(m); }
void orc_mt_seed(void *m, uint32_t seed) { mt_seed((orc_mt *)m, seed); }
void orc_mt_init_key(void *m, const uint32_t *key, uint32_t n) { mt_init_key((orc_mt *)m, key, n); }
uint32_t orc_mt_u32(void *m) { return mt_u32((orc_mt *)m); }
double orc_mt_dsemi(void *m) { return mt_dsemi((orc_mt *)m); }
double orc_mt_dsopen(void *m) { return mt_dsopen((orc_mt *)m); }
double orc_mt_dlclosed(void *m) { return ((double)mt_u32((orc_mt *)m)) * (1.0 / 4294967295.0); }
double orc_mt_dlsemi(void *m) { return ((double)mt_u32((orc_mt *)m)) * (1.0 / 4294967296.0); }
double orc_mt_dclosed(void *m)
{
    uint32_t a = mt_u32((orc_mt *)m) >> 5, b = mt_u32((orc_mt *)m) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740991.0);
}

/* ------------------------------------------------------------------------ CRC-32 ---------- */
/* crc32.c restated.  The reference builds the reflected table of POLYNOMIAL 0xEDB88320
 * (crc32init), feeds the first four data bytes inverted into the register while shifting the
 * inversion mask out (crc32update, first loop), runs them through four table steps when the mask
 * empties (ini_), continues byte-wise, and inverts at the end (crc32final, which also finishes
 * data shorter than four bytes).  Equivalent to the zlib CRC-32 -- tests/test_oracle.py pins it
 * against zlib and against crc32.c itself compiled by oracle/Makefile. */
typedef struct { uint32_t xor_mask, reg; } orc_crc;

static uint32_t orc_crc_tab[256];

static uint32_t orc_crc_4steps(uint32_t r)
{
    for (int i = 0; i < 4; ++i) r = (r >> 8) ^ orc_crc_tab[r & 255u];
    return r;
}

void orc_crc32_init(orc_crc *t)
{
    if (!orc_crc_tab[1])
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t r = i;
            for (int j = 0; j < 8; ++j) r = (r >> 1) ^ ((r & 1u) ? 0xEDB88320u : 0u);
            orc_crc_tab[i] = r;
        }
    t->xor_mask = ~0u;
    t->reg = 0;
}

void orc_crc32_update(orc_crc *t, const void *data, size_t len)
{
    const uint8_t *p = (const uint8_t *)data;
    for (; t->xor_mask && len; --len, ++p) {
        t->reg = (t->reg >> 8) | ((uint32_t)(uint8_t)~*p << 24);
        t->xor_mask >>= 8;
        if (!t->xor_mask) t->reg = orc_crc_4steps(t->reg);
    }
    for (; len; --len, ++p) t->reg = orc_crc_tab[(t->reg ^ *p) & 255u] ^ (t->reg >> 8);
}

uint32_t orc_crc32_final(orc_crc *t)
{
    return ~(t->xor_mask ? t->xor_mask ^ orc_crc_4steps(t->reg) : t->reg);
}

uint32_t orc_crc32(const void *data, size_t len)
{
    orc_crc t;
    orc_crc32_init(&t);
    orc_crc32_update(&t, data, len);
    return orc_crc32_final(&t);
}
