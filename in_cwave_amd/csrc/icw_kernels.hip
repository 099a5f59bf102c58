/*
 * icw_kernels.hip -- gfx950 (CDNA4) kernels of the in_cwave Hilbert -> modulator -> render path.
 *
 * Built with `-ffp-contract=off` and no fast-math; every floating-point expression below keeps
 * the operand order of the reference so that results are bit-identical to the x86 SSE2 build
 * of in_cwave (IEEE binary64, round-to-nearest, no FMA contraction, denormals preserved).
 *
 * Kernel roles (DESIGN.md "Kernels"; the serial IIR recurrence K1 lives in icw_iir.hip):
 *   icw_unpack_frames  K0: unpack + fade + the quadrature mix into per-chain filter inputs.
 *   icw_output      one thread per frame.  Everything that is NOT on the recurrence: the output
 *                   Kahan sum y[n] = sum d_i z_i + d0*c_i z_i (hblpf.c:1029-1043) from the w
 *                   window (frame-parallel), the fs/4 un-mix (lpf_hilbert_quad.c:129-156), the
 *                   DSP graph (adv_modulator.c:637-751) and the elementwise render
 *                   (sound_render.c:691-809, ROUND/flat).  Coalesced tile loads via LDS.
 *   icw_graph_serial / icw_dither_coop / icw_render_serial   K4 / K3a / K3b (serial forms).
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/icw.h"
#include "icw_device.h"
#include "icw_iir_dev.h"
#include "icw_libm.h"

#pragma clang fp contract(off)

#define ICW_PI (3.1415926535897932384626433832795029)
#define ICW_SQRT2 (1.4142135623730950488016887242097)

/* ------------------------------------------------------------------ input unpack --------- */
/* xwave_reader.c:205-239 + unpack_lsb.h:53-125 (little-endian, exact conversions) */
__device__ __forceinline__ double icw_unpack(const unsigned char *p, uint32_t fmt)
{
    switch (fmt) {
    case ICW_FMT_I16: {
        int v = (int)(short)((unsigned)p[0] | ((unsigned)p[1] << 8));
        return (double)v;
    }
    case ICW_FMT_U8:
        return 256.0 * (double)((signed char)(unsigned char)(p[0] - 0x80u));
    case ICW_FMT_I24: {
        int v = ((int)(((unsigned)p[0] << 8) | ((unsigned)p[1] << 16) | ((unsigned)p[2] << 24))) >> 8;
        return ((double)v) / 256.0;
    }
    case ICW_FMT_I32: {
        int v = (int)((unsigned)p[0] | ((unsigned)p[1] << 8) | ((unsigned)p[2] << 16) | ((unsigned)p[3] << 24));
        return ((double)v) / 65536.0;
    }
    default: {
        unsigned u = (unsigned)p[0] | ((unsigned)p[1] << 8) | ((unsigned)p[2] << 16) | ((unsigned)p[3] << 24);
        return 32768.0 * (double)__uint_as_float(u);
    }
    }
}

/* CWAVE unpackers (xwave_reader.c:171-200): no scaling, values already on the 16-bit scale */
__device__ __forceinline__ uint32_t icw_le32(const unsigned char *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ __forceinline__ void icw_unpack_iq(const unsigned char *p, uint32_t fmt, double &vI, double &vQ)
{
    switch (fmt) {
    case ICW_FMT_CW_F64: {
        const unsigned long long lo = icw_le32(p), hi = icw_le32(p + 4);
        const unsigned long long lo2 = icw_le32(p + 8), hi2 = icw_le32(p + 12);
        vI = __longlong_as_double((long long)(lo | (hi << 32)));
        vQ = __longlong_as_double((long long)(lo2 | (hi2 << 32)));
        break;
    }
    case ICW_FMT_CW_I16:
        vI = (double)(short)((unsigned)p[0] | ((unsigned)p[1] << 8));
        vQ = (double)(short)((unsigned)p[2] | ((unsigned)p[3] << 8));
        break;
    case ICW_FMT_CW_I16_F32:
        vI = (double)(short)((unsigned)p[0] | ((unsigned)p[1] << 8));
        vQ = (double)__uint_as_float(icw_le32(p + 2));
        break;
    default:
        vI = (double)__uint_as_float(icw_le32(p));
        vQ = (double)__uint_as_float(icw_le32(p + 4));
        break;
    }
}

/* one sample of format FMT; AL: the address is aligned to the sample's size, so one typed load
 * replaces the byte loads and their shifts */
template <int FMT, bool AL>
__device__ __forceinline__ double icw_unpack_f(const unsigned char *p)
{
    if constexpr (AL && FMT == ICW_FMT_I16) return (double)*(const short *)p;
    else if constexpr (AL && FMT == ICW_FMT_I32) return ((double)*(const int *)p) / 65536.0;
    else if constexpr (AL && FMT == ICW_FMT_F32) return 32768.0 * (double)*(const float *)p;
    else return icw_unpack(p, FMT);
}

template <int V> struct icw_ic { static constexpr int value = V; };

/* calls f(icw_ic<FMT>, icw_ic<AL>) for a uniform real format: the unpack specialised once per
 * workgroup instead of a format switch per sample.  al: the OR of the base address and the strides
 * the samples are read at (aligned when its low bits below the sample size are clear) */
template <typename F>
__device__ __forceinline__ void icw_fmt_dispatch(uint32_t fmt, uintptr_t al, F &&f)
{
    switch (fmt) {
    case ICW_FMT_I16:
        if (al & 1) f(icw_ic<ICW_FMT_I16>(), icw_ic<0>());
        else f(icw_ic<ICW_FMT_I16>(), icw_ic<1>());
        break;
    case ICW_FMT_U8: f(icw_ic<ICW_FMT_U8>(), icw_ic<0>()); break;
    case ICW_FMT_I24: f(icw_ic<ICW_FMT_I24>(), icw_ic<0>()); break;
    case ICW_FMT_I32:
        if (al & 3) f(icw_ic<ICW_FMT_I32>(), icw_ic<0>());
        else f(icw_ic<ICW_FMT_I32>(), icw_ic<1>());
        break;
    default:
        if (al & 3) f(icw_ic<ICW_FMT_F32>(), icw_ic<0>());
        else f(icw_ic<ICW_FMT_F32>(), icw_ic<1>());
        break;
    }
}

/* fade factor of xwave_unpack_csample (xwave_reader.c:918-936); < 0 means "no fade" */
__device__ __forceinline__ double icw_fade(long long ix, long long ns, long long fi, long long fo)
{
    double fade = -1.0;
    if (ix < fi)
        fade = ((double)ix) / ((double)fi);
    else if (ix > ns - fo && ix < ns)
        fade = ((double)(ns - ix)) / ((double)fo);
    return fade;
}

/* input of the I (f=0) / Q (f=1) filter for Hilbert phase k (lpf_hilbert_quad.c:133-151):
 *   I: {x, +0, -x, +0}   Q: {+0, -x, +0, x}.  K0 writes the nonzero values of both into one row per
 * channel; the recurrences supply the +0.0 (icw_iir_dev.h: icw_chain_x). */

/* the fade and the signed filter-input row of one real frame (v: the unpacked L, R samples) */
__device__ __forceinline__ void icw_store_frame(const IcwK0Args &a, int t, int s, double (&v)[2])
{
    const long long ix = a.pos[s] + a.t0 + t;
    const double fd = icw_fade(ix, a.fade[s * 3 + 0], a.fade[s * 3 + 1], a.fade[s * 3 + 2]);
    if (fd >= 0.0) {
        v[0] *= fd;
        v[1] *= fd;
    }
    /* one row per channel, s*2 + ch: the I filter's nonzero inputs sit at the even phases, the Q
     * filter's at the odd ones, so the channel's signed sample {x, -x, -x, x}[k] serves both -- the
     * I filter reads it where k is even (x, -x), the Q filter where k is odd (-x, x), and each takes
     * the literal +0.0 at the other phases itself (icw_chain_x): 16 B per stereo frame, not 32 */
    double *xs = a.xd + (size_t)s * 2 * a.x_pitch + t;
    const int nchw = a.dedup ? 1 : 2;          /* mono dedup: K1 reads the left row only */
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
        if (ch < nchw) {
            const unsigned k = (a.hq_phase[s * 2 + ch] + (unsigned)(a.t0 + t)) & 3u;
            xs[(size_t)ch * a.x_pitch] = (k == 0u || k == 3u) ? v[ch] : -v[ch];
        }
    }
}

/* Input prep (K0): unpack + fade each frame once (xwave_unpack_csample, xwave_reader.c:908-1001)
 * and lay out the filter inputs of the quadrature mix of hq_rp_process (lpf_hilbert_quad.c:129-156):
 * the I filter {x, +0, -x, +0} and the Q filter {+0, -x, +0, x} by sample phase, both in one row
 * s*2 + ch of signed samples (below).  Mono input feeds the right converter with the left value,
 * exactly the reference's reuse of `val` (xwave_reader.c:988).  Complex input: four rows
 * s*4 + ch*2 + {I, Q}. */
__device__ __forceinline__ void icw_unpack_frame(const IcwK0Args &a, int t, int s)
{
    const unsigned char *fp = a.in + (size_t)s * a.in_stride + (size_t)t * a.fsz;
    const long long ix = a.pos[s] + a.t0 + t;
    const double fd = icw_fade(ix, a.fade[s * 3 + 0], a.fade[s * 3 + 1], a.fade[s * 3 + 2]);
    if (a.fmt >= ICW_FMT_CW_F64) {
        /* complex (CWAVE) sample: I/Q per channel, mono -> R = L, fade on all four
         * (xwave_reader.c:939-966); rows s*4 + ch*2 + {I, Q} */
        double q[4];
        icw_unpack_iq(fp, a.fmt, q[0], q[1]);
        if (a.nch > 1) icw_unpack_iq(fp + a.csz, a.fmt, q[2], q[3]);
        else { q[2] = q[0]; q[3] = q[1]; }
        if (fd >= 0.0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] *= fd;
        }
        double *xs = a.xd + (size_t)s * 4 * a.x_pitch + t;
#pragma unroll
        for (int i = 0; i < 4; ++i) xs[(size_t)i * a.x_pitch] = q[i];
        return;
    }
    const uintptr_t al = (uintptr_t)(a.in + (size_t)s * a.in_stride) | (uintptr_t)a.fsz;
    icw_fmt_dispatch(a.fmt, al, [&](auto fc, auto ac) {
        constexpr int F = decltype(fc)::value;
        constexpr bool AL = decltype(ac)::value != 0;
        double v[2];
        v[0] = icw_unpack_f<F, AL>(fp);
        v[1] = a.nch > 1 ? icw_unpack_f<F, AL>(fp + a.csz) : v[0];
        icw_store_frame(a, t, s, v);
    });
}

__global__ __launch_bounds__(256) void icw_unpack_frames(IcwK0Args a)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t < a.T) icw_unpack_frame(a, t, blockIdx.y);
}

/* FIR Hilbert converter: real PCM -> the analytic signal a CWAVE file holds (cwave.h:40,56-58:
 * "Hilbert FIR filter order" k_M, "filter parameter" k_beta; the converter itself is not part of
 * in_cwave).  Order M (even, M + 1 taps), centre c = M/2, odd taps only:
 *     I[n] = x[n - c],   Q[n] = sum_{m = 1, 3, .., <= c} g_m * (x[n - c - m] - x[n - c + m])
 * with the sum taken in ascending m as acc = fma(g_m, d_m, acc) from +0.0 -- the oracle's order, so
 * the result is bit-identical.  x is the unpacked, faded input of K0 (xwave_unpack_csample,
 * xwave_reader.c:908-936), mono feeding R with L.
 *
 * Register blocking.  A lane sums 8 consecutive outputs of one channel.  For 8 taps at a time it
 * loads the 22 inputs their left operands span and the 22 of the right ones, then runs the 64
 * subtract + FMA pairs from registers: 44 LDS reads per 64 output-taps instead of 128.  The staged
 * inputs carry one pad double after every 8 (physical index i + i/8), so the 32 lanes of a
 * ds_read_b64 group, 9 doubles apart, hit 64 distinct banks; a staging shift `sh` puts every lane's
 * window at the same phase of that pattern, so all offsets inside a block are immediates.  Taps past
 * the last multiple of 8 run one at a time. */
#define ICW_FIR_R 8                                  /* outputs per lane */
#ifndef ICW_FIR_VEC
#define ICW_FIR_VEC 1                                /* FIR staging: 16-byte loads, one LDS base per thread */
#endif
#ifndef ICW_FIR_INTERIOR
#define ICW_FIR_INTERIOR 1                           /* FIR staging: the interior tiles' short form */
#endif
#ifndef ICW_FIR_OCC
#define ICW_FIR_OCC 4                                /* KF2 workgroups per CU the register budget is sized for */
#endif
#ifndef ICW_FIR_CUT
#define ICW_FIR_CUT 0                                /* diagnostic: 1 no graph, 2 no sums either (VALU by phase) */
#endif
#ifndef ICW_FIR_DIAG
#define ICW_FIR_DIAG 0                               /* diagnostic, not exact: 1 no division slow path, 2 no render */
#endif
#ifndef ICW_FIR_STAMPS
#define ICW_FIR_STAMPS 0                             /* diagnostic: KF2 phase stamps (tools/fir_phases.py) */
#endif
#ifndef ICW_CHAIN4
#define ICW_CHAIN4 1                                 /* KF2: chain programs op by op over a lane's frames */
#endif

/* The staged inputs carry ICW_FIR_PAD pad doubles after every 8 (physical index i + PAD (i / 8)).  With
 * 2 a lane's window (8 outputs apart: 10 doubles = 20 dwords) starts 16-byte aligned at every lane, and
 * the sums read it two doubles at a time (ds_read_b128, conflict-free over each 16-lane group: 20 l
 * mod 64 covers the 64 banks once), half the LDS instructions of the 1-pad layout's ds_read_b64. */
#ifndef ICW_FIR_PAD
#define ICW_FIR_PAD 2
#endif
#if ICW_FIR_PAD != 1 && ICW_FIR_PAD != 2
#error "ICW_FIR_PAD: icw_fir_block's window reads are written for 1 or 2 pad doubles per 8"
#endif
#ifndef ICW_SCALAR_UNIT
#define ICW_SCALAR_UNIT 1                            /* A/B: unit gains / norm_mul tested on scalar flags */
#endif
#ifndef ICW_RENDER_SH0
#define ICW_RENDER_SH0 1                             /* A/B: the render-only form specialised for norm_shift 0 */
#endif
__device__ __forceinline__ int icw_fir_phys(int i) { return i + ICW_FIR_PAD * (i >> 3); }


/* inputs of NC channels from ch0 for the outputs [tt, tt + nout) of a launch block, at logical
 * index i <-> frame j = tt - M + i - sh (zero outside [-M, T)), channel k at xs + k * px; the
 * history after the block is written by the tile that owns each of its frames.  The stereo form
 * computes a frame's address, validity and fade once for both channels. */
template <int FMT, bool AL, int NC>
__device__ __forceinline__ void icw_fir_stage_t(const IcwFirArgs &f, int s, int ch0, double *xs, int px, int tt,
                                                int nout, int sh, int tid, int nthr)
{
    const int T = f.T, M = f.M;
    const unsigned char *src = f.in + (size_t)s * f.in_stride + (size_t)ch0 * f.csz;
    const long long p0 = f.pos[s] + f.t0;
    const long long ns = f.fade[s * 3 + 0], fi = f.fade[s * 3 + 1], fo = f.fade[s * 3 + 2];
    const double *hin = f.hist_in + ((size_t)s * 2 + ch0) * M;
    double *hout = f.hist_out + ((size_t)s * 2 + ch0) * M;
    const bool mono = f.nch == 1;
    const int nl = sh + M + nout + 24;               /* logical extent: pad, history, tile, margin */
    const int nf = min(nout, T - tt);
    /* uniform over the tile: no fade anywhere in the frames it stages (icw_fade returns "none" for
     * fi <= ix <= ns - fo and for ix >= ns), and whether any staged frame precedes the block (the
     * history).  The fade's two FP64 divisions and the history loads were computed for every input
     * and made the staging ~half of the kernel's VALU instructions (r03_c2fir_sq.json). */
    const long long ja = max(tt - M, 0), jb = (long long)tt + nf - 1;
    const bool nofade = p0 + ja >= fi && (p0 + jb <= ns - fo || p0 + ja >= ns);
    const bool need_hist = tt < M + sh;
    /* 8 consecutive frames per thread and pass, their loads issued together (clamped in range,
     * selected after): the staging is load-latency bound otherwise */
    constexpr int V = 8;
    /* An interior tile of a packed typed format (i16 / i32 / f32, the file frame exactly the computed
     * channels): a thread's 8 frames are 8 * frame-size contiguous bytes, read by 16-byte loads from
     * one address, unpacked from the registers (the same conversions as icw_unpack_f), and written to
     * 8 consecutive LDS doubles per channel (logical 8t..8t+7 sit at physical 9t..9t+7) from one base.
     * Only the threads at the ends of the staged range select zeros.  With M >= 32 every frame a
     * thread loads lies in [0, T) (tt >= M + sh, and the last load ends 30 frames past the tile's
     * outputs, tt + nout <= T - M).  The per-frame address, clamp and select of the general form were
     * most of the staging's VALU instructions (c2fir: ~150 per wave). */
    if constexpr (ICW_FIR_VEC && AL && (FMT == ICW_FMT_I16 || FMT == ICW_FMT_I32 || FMT == ICW_FMT_F32)) {
        constexpr int CS = FMT == ICW_FMT_I16 ? 2 : 4;
        constexpr int FB = NC * CS;                       /* bytes per frame */
        constexpr int NW = V * FB / 4;                    /* 32-bit words per thread and pass */
        const unsigned char *b0 = src + (size_t)(tt - M - sh) * f.fsz;
        if (nofade && !need_hist && tt + nf <= T - M && M >= 32 && f.fsz == FB && !((uintptr_t)b0 & 15)) {
            const int lim = sh + M + nf;                  /* logical [sh, lim) holds inputs, the rest zeros */
            for (int i0 = tid * V; i0 < nl; i0 += nthr * V) {
                const uint4 *p = (const uint4 *)(b0 + (size_t)i0 * FB);
                uint32_t w[NW];
#pragma unroll
                for (int k = 0; k < NW / 4; ++k) {
                    const uint4 q4 = p[k];
                    w[4 * k] = q4.x; w[4 * k + 1] = q4.y; w[4 * k + 2] = q4.z; w[4 * k + 3] = q4.w;
                }
                double v[NC][V];
#pragma unroll
                for (int e = 0; e < V; ++e) {
#pragma unroll
                    for (int k = 0; k < NC; ++k) {
                        const int si = e * NC + k;            /* sample index in the thread's run */
                        if constexpr (FMT == ICW_FMT_I16) {
                            const uint32_t u = w[si >> 1];
                            v[k][e] = (double)((si & 1) ? ((int)u >> 16) : (int)(short)(u & 0xffffu));
                        } else if constexpr (FMT == ICW_FMT_I32) {
                            v[k][e] = ((double)(int)w[si]) / 65536.0;
                        } else {
                            v[k][e] = 32768.0 * (double)__uint_as_float(w[si]);
                        }
                    }
                }
                double *d = xs + icw_fir_phys(i0);
                if (i0 >= sh && i0 + V <= lim) {
#pragma unroll
                    for (int k = 0; k < NC; ++k)
#pragma unroll
                        for (int e = 0; e < V; ++e) d[k * px + e] = v[k][e];
                } else {
#pragma unroll
                    for (int e = 0; e < V; ++e) {
                        const int i = i0 + e;
                        if (i < nl) {
#pragma unroll
                            for (int k = 0; k < NC; ++k) d[k * px + e] = (i >= sh && i < lim) ? v[k][e] : 0.0;
                        }
                    }
                }
            }
            return;
        }
    }
    if (ICW_FIR_INTERIOR && NC == 2 && nofade && !need_hist && tt + nf <= T - M) {
        /* an interior tile (most of them): no fade, no history to read or write -- a frame is its
         * input inside [tt - M, tt + nf) and zero outside (c2fir +3 %, c4fir +3 %; the mono form
         * measured 1 % slower with it, so it keeps the general one) */
        for (int i0 = tid * V; i0 < nl; i0 += nthr * V) {
            double raw[NC][V];
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const int jr = min(tt - M + i0 + e - sh, T - 1);
                const unsigned char *p = src + (size_t)jr * f.fsz;
#pragma unroll
                for (int k = 0; k < NC; ++k) raw[k][e] = icw_unpack_f<FMT, AL>(p + k * f.csz);
            }
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const int i = i0 + e;
                const bool in = i >= sh && i < sh + M + nf;
                if (i < nl) {
#pragma unroll
                    for (int k = 0; k < NC; ++k) xs[k * px + icw_fir_phys(i)] = in ? raw[k][e] : 0.0;
                }
            }
        }
        return;
    }
    for (int i0 = tid * V; i0 < nl; i0 += nthr * V) {
        double raw[NC][V], his[NC][V];
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const int j = tt - M + i0 + e - sh;
            const int jr = min(max(j, 0), T - 1);
            const unsigned char *p = src + (size_t)jr * f.fsz;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                raw[k][e] = icw_unpack_f<FMT, AL>(p + k * f.csz);
                his[k][e] = 0.0;
            }
        }
        if (need_hist) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const int h = min(max(tt + i0 + e - sh, 0), M - 1);
#pragma unroll
                for (int k = 0; k < NC; ++k) his[k][e] = hin[k * M + h];
            }
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const int i = i0 + e;
            const int j = tt - M + i - sh;
            double v[NC];
#pragma unroll
            for (int k = 0; k < NC; ++k) v[k] = 0.0;
            if (i >= sh && j < tt + nf) {
                if (j < 0) {
#pragma unroll
                    for (int k = 0; k < NC; ++k) v[k] = his[k][e];
                } else {
#pragma unroll
                    for (int k = 0; k < NC; ++k) v[k] = raw[k][e];
                    if (!nofade) {
                        const double fd = icw_fade(p0 + j, ns, fi, fo);
                        if (fd >= 0.0) {
#pragma unroll
                            for (int k = 0; k < NC; ++k) v[k] *= fd;
                        }
                    }
                }
                if (j >= T - M && (j >= tt || tt == 0)) {
#pragma unroll
                    for (int k = 0; k < NC; ++k) hout[k * M + j - (T - M)] = v[k];
                    if (NC == 1 && mono) hout[M + j - (T - M)] = v[0];
                }
            }
            if (i < nl) {
#pragma unroll
                for (int k = 0; k < NC; ++k) xs[k * px + icw_fir_phys(i)] = v[k];
            }
        }
    }
}

/* the staging of NC channels, its format and alignment resolved once (uniform) per workgroup */
template <int NC>
__device__ __forceinline__ void icw_fir_stage(const IcwFirArgs &f, int s, int ch0, double *xs, int px, int tt,
                                              int nout, int sh, int tid, int nthr)
{
    const uintptr_t al = (uintptr_t)(f.in + (size_t)s * f.in_stride) | (uintptr_t)f.fsz;
    icw_fmt_dispatch(f.fmt, al, [&](auto fc, auto ac) {
        icw_fir_stage_t<decltype(fc)::value, decltype(ac)::value != 0, NC>(f, s, ch0, xs, px, tt, nout, sh, tid,
                                                                           nthr);
    });
}

/* The taps through the constant address space: every lane of a wave reads the same tap, so they
 * come in by scalar loads into SGPRs (the FMA takes one SGPR operand) and leave the LDS pipe to the
 * inputs -- which bounds the sums: 52 -> 44 LDS reads per 8-tap block of a lane's 8 outputs. */
typedef const __attribute__((address_space(4))) double icw_ctap;

/* one NTAP-tap block (k0 = NTAP b) of a lane's 8 outputs: bl / br = physical index of the first input
 * of the left / right window (both at phase 2 of the pad pattern; NTAP 4 or 8 keeps it there) */
#ifndef ICW_FIR_NTAP
#define ICW_FIR_NTAP 8                               /* taps per register block of the sums */
#endif
template <int NTAP>
__device__ __forceinline__ void icw_fir_block(const double *xs, icw_ctap *gs, int k0, int bl, int br,
                                              double (&acc)[ICW_FIR_R])
{
    static_assert(NTAP == 4 || NTAP == 8, "a window step of whole pad groups");
    constexpr int W = ICW_FIR_R + 2 * NTAP - 2;
    double L[W], Rt[W], g[NTAP];
    if constexpr (ICW_FIR_PAD == 2) {
        /* elements e, e + 1 (e even) never straddle a pad: the window starts at logical phase 2 */
#pragma unroll
        for (int e = 0; e < W; e += 2) {
            const double2 v = *(const double2 *)(xs + bl + e + 2 * ((e + 2) >> 3));
            L[e] = v.x;
            L[e + 1] = v.y;
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int e = 0; e < W; e += 2) {
            const double2 v = *(const double2 *)(xs + br + e + 2 * ((e + 2) >> 3));
            Rt[e] = v.x;
            Rt[e + 1] = v.y;
            asm volatile("" ::: "memory");
        }
    } else {
#pragma unroll
        for (int e = 0; e < W; ++e) {
            L[e] = xs[bl + e + ((e + 2) >> 3)];
            asm volatile("" ::: "memory");               /* no ds_read2 pairing: 2 x 2 cycles, not 8 */
        }
#pragma unroll
        for (int e = 0; e < W; ++e) {
            Rt[e] = xs[br + e + ((e + 2) >> 3)];
            asm volatile("" ::: "memory");
        }
    }
#pragma unroll
    for (int j = 0; j < NTAP; ++j) g[j] = gs[k0 + j];
#pragma unroll
    for (int j = 0; j < NTAP; ++j) {
#pragma unroll
        for (int r = 0; r < ICW_FIR_R; ++r)
            acc[r] = __builtin_fma(g[j], L[r - 2 * j + 2 * NTAP - 2] - Rt[r + 2 * j], acc[r]);
    }
}

/* Q of a lane's 8 outputs tt + 8 ll + r; a = (c - 1 + sh) / 8.  The taps in ascending order, in
 * register blocks of ICW_FIR_NTAP, then one by one */
template <int NB = ICW_FIR_NTAP>
__device__ __forceinline__ void icw_fir_sums(const double *xs, icw_ctap *gs, int nt, int ll, int a, int sh, int c,
                                             double (&acc)[ICW_FIR_R])
{
#pragma unroll
    for (int r = 0; r < ICW_FIR_R; ++r) acc[r] = 0.0;
    const int nb = nt / NB;
    constexpr int G = 8 + ICW_FIR_PAD;                  /* physical doubles per group of 8 */
    constexpr int GS = G * NB / 4;                      /* physical step of a window per block */
    int bl = G * (ll + a - NB / 4) + 2, br = G * (ll + a) + 2;
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        icw_fir_block<NB>(xs, gs, NB * b, bl, br, acc);
        bl -= GS;
        br += GS;
    }
    const int A = 8 * a;
#pragma unroll 1
    for (int k = nb * NB; k < nt; ++k) {
        const double gk = gs[k];
#pragma unroll
        for (int r = 0; r < ICW_FIR_R; ++r) {
            const int li = 8 * ll + A + r - 2 * k, ri = 8 * ll + A + 2 + r + 2 * k;
            acc[r] = __builtin_fma(gk, xs[icw_fir_phys(li)] - xs[icw_fir_phys(ri)], acc[r]);
        }
    }
    (void)sh; (void)c;
}

/* KF: the converter alone, one workgroup per channel and 2048-frame tile of a stream; I / Q rows
 * go out coalesced through LDS to the CWAVE rows K2 reads */
__global__ __launch_bounds__(256) void icw_fir_hilbert(IcwFirArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double xs[];   /* staged inputs (padded), taps, Q */
    constexpr int TF = 256 * ICW_FIR_R;
    const int ch = blockIdx.y, s = blockIdx.z;
    const int tt = blockIdx.x * TF;
    const int M = a.M, c = M >> 1;
    const int sh = (8 - ((c - 1) & 7)) & 7;          /* c - 1 + sh = 8 a */
    const int av = (c - 1 + sh) >> 3;
    const int nf = min(TF, a.T - tt);
    icw_fir_stage<1>(a, s, ch, xs, 0, tt, TF, sh, threadIdx.x, 256);
    const int px = (icw_fir_phys(sh + M + TF + 24) + 2) & ~1;   /* even: the next row stays 16-byte aligned */
    double *qs = xs + px + ((a.nt + 1) & ~1);
    icw_ctap *gs = (icw_ctap *)a.g;
    __syncthreads();
    double acc[ICW_FIR_R];
    icw_fir_sums(xs, gs, a.nt, threadIdx.x, av, sh, c, acc);
#pragma unroll
    for (int r = 0; r < ICW_FIR_R; ++r) qs[ICW_FIR_R * threadIdx.x + r] = acc[r];
    __syncthreads();
    double *rowI = a.xd + ((size_t)s * 4 + ch * 2) * a.x_pitch + tt;
    double *rowQ = rowI + a.x_pitch;
    const bool mono = a.nch == 1;
    for (int f = threadIdx.x; f < nf; f += 256) {
        const double vi = xs[icw_fir_phys(f + 8 * av + 1)], vq = qs[f];
        rowI[f] = vi;
        rowQ[f] = vq;
        if (mono) {
            rowI[f + 2 * a.x_pitch] = vi;
            rowQ[f + 2 * a.x_pitch] = vq;
        }
    }
}


/* ------------------------------------------------------------- output kernel (K2) ------- */
struct IcwLR { double lre, lim, rre, rim; };

/* output Kahan sum of iir_rp_process_kahan (hblpf.c:1029-1043) for the sample whose delay line
 * is z_i = win[N-1-i] (win = w[t-N .. t-1]); baseline form (hblpf.c:898-925) needs w[t]=win[N] */
/* the same sums for NC chains at once, interleaved by term: each coefficient is live for one
 * term of all NC chains instead of across NC whole sums (with the chains back to back, all 2N
 * coefficients stay live in SGPRs and spill to VGPR lanes -- a v_readlane per use) */
/* FP_CHECK on: the output half of the WITH FP CHECKS branches of iir_rp_process_kahan / _baseline
 * (hblpf.c:1058-1095, 928-950) for one chain, whose delay line is z_i = win[N-1-i].  ti = FC(z * c_i)
 * is the loop-back kernel's product (counted there), so here it is only applied.  Compact on
 * purpose (run-time loops, FC() not inlined): a diagnostic mode. */
__device__ __noinline__ double icw_iir_out_fc(const double *win, int N, int kahan, const double *pc,
                                              const double *pd, double d0, IcwFes &f)
{
    if (kahan) {
        double z = win[N - 1];
        double t = icw_fc_nc(z * pc[0]);
        double S = icw_fc(z * pd[0], f), C = 0.0, Y, T;
#pragma unroll 1
        for (int k = 0; k < 2 * N - 1; ++k) {
            /* steps: t0 * d0, then per i >= 1: z * d_i, t_i * d0 */
            const int i = (k + 1) >> 1;
            double x;
            if (k == 0) x = icw_fc(t * d0, f);
            else if (k & 1) { z = win[N - 1 - i]; t = icw_fc_nc(z * pc[i]); x = icw_fc(z * pd[i], f); }
            else x = icw_fc(t * d0, f);
            Y = icw_fc(x - C, f);                            /* kahan_step_fes, hblpf.c:995-1005 */
            T = icw_fc(S + Y, f);
            C = icw_fc(icw_fc(T - S, f) - Y, f);
            S = T;
        }
        return S;
    }
    double so = 0.0;
#pragma unroll 1
    for (int i = 0; i < N; ++i) so = icw_fc(so + icw_fc(win[N - 1 - i] * pd[i], f), f);
    return icw_fc(icw_fc(win[N] * d0, f) + so, f);
}

template <int N, bool KAHAN, int NC>
__device__ __forceinline__ void icw_iir_out_n(const double *const (&win)[NC], const double *pc, const double *pd,
                                              double d0, double (&y)[NC])
{
    if (KAHAN) {
        double S[NC], C[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const double z = win[c][N - 1];
            const double t0 = z * pc[0];
            double Y, T;
            S[c] = z * pd[0];
            C[c] = 0.0;
            const double x = t0 * d0;
            Y = x - C[c]; T = S[c] + Y; C[c] = (T - S[c]) - Y; S[c] = T;
        }
#pragma unroll
        for (int i = 1; i < N; ++i) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const double z = win[c][N - 1 - i];
                const double ti = z * pc[i];
                double x = z * pd[i], Y, T;
                Y = x - C[c]; T = S[c] + Y; C[c] = (T - S[c]) - Y; S[c] = T;
                x = ti * d0;
                Y = x - C[c]; T = S[c] + Y; C[c] = (T - S[c]) - Y; S[c] = T;
            }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) y[c] = S[c];
    } else {
        double so[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) so[c] = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
#pragma unroll
            for (int c = 0; c < NC; ++c) so[c] += win[c][N - 1 - i] * pd[i];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) y[c] = win[c][N] * d0 + so[c];
    }
}

template <int N, bool KAHAN>
__device__ __forceinline__ double icw_iir_out(const double *win, const double (&pc)[20],
                                              const double (&pd)[20], double d0)
{
    if (KAHAN) {
        double z = win[N - 1];
        double t0 = z * pc[0];
        double S = z * pd[0], C = 0.0, Y, T;
        double x = t0 * d0;
        Y = x - C; T = S + Y; C = (T - S) - Y; S = T;
#pragma unroll
        for (int i = 1; i < N; ++i) {
            z = win[N - 1 - i];
            const double ti = z * pc[i];
            x = z * pd[i];
            Y = x - C; T = S + Y; C = (T - S) - Y; S = T;
            x = ti * d0;
            Y = x - C; T = S + Y; C = (T - S) - Y; S = T;
        }
        return S;
    } else {
        double so = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) so += win[N - 1 - i] * pd[i];
        return win[N] * d0 + so;
    }
}

/* x / SQRT2 correctly rounded, as dsp_master divides (adv_modulator.c:498-501), in 3 FP64 operations
 * instead of the 11 of a general division (div_scale x 2, rcp, 5 fma, mul, div_fmas, div_fixup):
 *     q0 = RN(x r),  e = RN(x - q0 c) (one fma),  q = RN(q0 + e r) (one fma),  r = RN(1/c).
 * Error: |q0 + e r - x/c| < 2^-51 ulp(x/c) for 2^-900 <= |x| <= DBL_MAX (q0 is within 2 ulp, e within
 * one rounding of the exact remainder, r within half an ulp of 1/c), so q can differ from RN(x/c)
 * only where x/c lies within 2^-51 ulp of a rounding midpoint.  With c = C 2^-52 (C odd) those
 * are the significands X with (2M + 1) C - 2^53 X = k (X >= C) or (2M + 1) C - 2^54 X = k (X < C)
 * for an odd |k| < 8 -- one residue class mod C each, a handful of X in [2^52, 2^53); every one of
 * them, up to |k| <= 63, gives RN(x/c) here (tests/test_libm.py::test_div_sqrt2_hard_cases, which
 * solves for them and checks this arithmetic in exact rationals).  Zeros (a -0.0 would come out
 * +0.0), tiny values (a subnormal remainder or quotient), infinities and NaNs take the division. */
/* The range test is on the result: |q| >= 2^-900 holds for no NaN (an infinite x gives a NaN q) and
 * implies |x| >= 2^-899.5 (q is within a few ulp of x / c wherever it is not a NaN), so it keeps q
 * only inside the range above, in one compare. */
__device__ __forceinline__ double icw_div_sqrt2_fast(double x)
{
    constexpr double rc = 0x1.6a09e667f3bccp-1;          /* RN(1 / c) */
    const double q0 = x * rc;
    const double e = __builtin_fma(-q0, ICW_SQRT2, x);
    return __builtin_fma(e, rc, q0);
}

__device__ __forceinline__ bool icw_div_sqrt2_ok(double q)
{
#if ICW_FIR_DIAG & 1
    return true;
#else
    return fabs(q) >= 0x1p-900;
#endif
}

__device__ __forceinline__ double icw_div_sqrt2(double x)
{
    double q = icw_div_sqrt2_fast(x);
    if (!icw_div_sqrt2_ok(q)) q = x / ICW_SQRT2;
    return q;
}

__device__ __forceinline__ double icw_master(int tout, double re, double im)
{
    switch (tout) {
    case ICW_S_RE: return re;
    case ICW_S_IM: return im;
    case ICW_S_ADD_REIM: return icw_div_sqrt2(re + im);
    case ICW_S_SUB_REIM: return icw_div_sqrt2(re - im);
    }
    return 0.0;
}

/* The value registers of the DSP program live in LDS, [reg][component][thread]: a register index
 * is wave-uniform and data-dependent, and a register array in VGPRs is demoted to scratch memory
 * by the compiler (measured: 256 B per frame written to HBM, 4.5 GB WRITE_SIZE per 16.8 M-frame
 * launch).  Lane-contiguous LDS rows are bank-conflict free. */
struct IcwRegFile {
    double *base;   /* lds + tid */
    __device__ __forceinline__ void get(int r, IcwLR &v) const
    {
        const double *p = base + (size_t)r * 4 * ICW_K2_TILE;
        v.lre = p[0]; v.lim = p[ICW_K2_TILE]; v.rre = p[2 * ICW_K2_TILE]; v.rim = p[3 * ICW_K2_TILE];
    }
    __device__ __forceinline__ void set(int r, const IcwLR &v) const
    {
        double *p = base + (size_t)r * 4 * ICW_K2_TILE;
        p[0] = v.lre; p[ICW_K2_TILE] = v.lim; p[2 * ICW_K2_TILE] = v.rre; p[3 * ICW_K2_TILE] = v.rim;
    }
};

/* row of frame t in the rotation table: frame-major, or (perm_q > 0, the fused FIR kernel, whose
 * lanes hold 4 or 8 consecutive frames) frames 8 apart in consecutive rows, so that a wave's loads
 * of one frame slot cover 1-2 KB contiguously instead of one row every 128 / 256 B */
__device__ __forceinline__ size_t icw_trig_index(int t, int perm_q)
{
    return perm_q ? (size_t)(t & 7) * (size_t)perm_q + (size_t)(t >> 3) : (size_t)t;
}

/* rotate (re,im) by e^{j phi} given cos/sin (adv_modulator.c:546-547, 576-577) */
__device__ __forceinline__ void icw_rot(double re, double im, double cs, double sn, double &ore, double &oim)
{
    ore = re * cs - im * sn;
    oim = re * sn + im * cs;
}

/* The rounding step of sound_render_value (sound_render.c:757-767) in fewer instructions, same bits:
 * q - ro is q + (-ro) in IEEE arithmetic, and ro / -ro differ only in the sign bit of the high
 * word, so one 32-bit select replaces the two 64-bit ones.  Then the peak: `aq > pk ? aq : pk`
 * equals fmax(pk, aq) here, because pk never holds a NaN and fmax returns the number when aq is
 * NaN (the reference's `cv > pv` is false for a NaN as well, sound_render.c:770-779). */
__device__ __forceinline__ double icw_round_q(double q, double round_offset, int sign_delta, int &delta)
{
    const bool neg = q < 0.0;
    const unsigned long long rb = (unsigned long long)__double_as_longlong(round_offset);
    const unsigned hi = (unsigned)(rb >> 32) ^ (neg ? 0x80000000u : 0u);
    delta = neg ? sign_delta : 0;
    return q + __longlong_as_double((long long)(((unsigned long long)hi << 32) | (rb & 0xffffffffull)));
}

/* The clip stage of sound_render_value (sound_render.c:782-797) as it reaches the integer:
 * q >= hi -> hi - 1, q <= lo -> lo + 1, then (int) truncation.  hi and lo are integers (hi >= 1,
 * lo <= -2), so for q in [hi-1, hi) the reference keeps q and truncates it to hi - 1, and for q in
 * (lo, lo+1] to lo + 1: min(q, hi - 1) / max(., lo + 1) give the same integer for every q, with
 * two instructions on the render's serial chain instead of two compares and four selects.  The
 * clip counts come from the same comparisons, off the chain.  A NaN q is the caller's case. */
__device__ __forceinline__ int icw_clamp_int(double q, const IcwRenderK &k, unsigned &clips)
{
    clips += (q >= k.hi ? 1u : 0u) + (q <= k.lo ? 1u : 0u);
    return (int)fmax(fmin(q, k.hi - 1.0), k.lo + 1.0);
}

/* The q of sound_render_value for ROUND render + flat shaper (sound_render.c:747-767): x * norm_mul
 * - prev_ns_err (0.0) + rnd * dth_mul (0.0 * dth_mul = +0.0), then +- round_offset by the sign.
 * x - 0.0 is x; the + 0.0, and a mid-riser's +- 0.0 (round_offset 0, sign_delta -1), change only a
 * zero's sign, which nothing downstream sees -- the peak takes fabs, the clip stage compares and
 * truncates, and (int) +-0.0 is 0 -- so they are not executed; a mid-tread's +- 0.5 of a -0.0 is +0.5
 * either way (-0.0 < 0 is false).  A norm_mul of 1.0 (16 sign bits) is not multiplied: x is a sum
 * or product, never a signalling NaN, and x * 1.0 is x. */
__device__ __forceinline__ double icw_round_in(double x, const IcwRenderK &k, int &delta)
{
    if (k.norm_mul != 1.0) x = x * k.norm_mul;
    if (k.sign_delta) {
        delta = x < 0.0 ? k.sign_delta : 0;
        return x;
    }
    return icw_round_q(x, k.round_offset, k.sign_delta, delta);
}

/* the rendered integer of one channel-sample (ROUND + flat), q for the caller's meters */
__device__ __forceinline__ int icw_render_round_q(double input, const IcwRenderK &k, double &q)
{
    int delta;
    q = icw_round_in(input, k, delta);
    /* x86 cvttsd2si semantics: NaN -> INT_MIN ("integer indefinite") */
    const int vc = (int)fmax(fmin(q, k.hi - 1.0), k.lo + 1.0);   /* icw_clamp_int without the counts */
    const int v = isnan(q) ? (int)0x80000000 : vc;
    return (v + delta) << k.norm_shift;
}

/* The q of a dithered render with the flat shaper (sound_render.c:711-767): the dither term d =
 * rnd * dth_mul comes from K3a (the same product), input = x * norm_mul - prev_ns_err is x * norm_mul
 * exactly (ns_empty keeps prev_ns_err at 0.0, sound_render.c:396-400, and x - 0.0 is x, a -0.0
 * included), qinput = input + d; then the rounding offset as icw_round_in (a mid-riser's +- 0.0
 * changes only a zero's sign, which nothing downstream sees). */
__device__ __forceinline__ double icw_round_in_d(double x, double d, const IcwRenderK &k, int &delta)
{
    if (k.norm_mul != 1.0) x = x * k.norm_mul;
    x = x + d;
    if (k.sign_delta) {
        delta = x < 0.0 ? k.sign_delta : 0;
        return x;
    }
    return icw_round_q(x, k.round_offset, k.sign_delta, delta);
}

/* sound_render_value for a flat-shaper render (sound_render.c:691-809): elementwise.  DITH: the
 * dither term d of a RPDF / TPDF / STPDF / GAUSS render (K3a's); ROUND has none. */
template <bool DITH = false>
__device__ __forceinline__ int icw_render_round(double input, const IcwRenderK &k, unsigned &clips, double &pk,
                                                double d = 0.0)
{
    int delta;
    const double q = DITH ? icw_round_in_d(input, d, k, delta) : icw_round_in(input, k, delta);
    pk = fmax(pk, fabs(q));
    /* x86 cvttsd2si semantics: NaN -> INT_MIN ("integer indefinite") */
    const int vc = icw_clamp_int(q, k, clips);    /* unconditional: a NaN counts no clip */
    int v = isnan(q) ? (int)0x80000000 : vc;
    return (v + delta) << k.norm_shift;
}

/* modulator frame counter -> norm_omega of frame t of the call (adv_modulator.c:611-625).
 * n0 is the call-start counter.  In scaled mode the reference takes the first frame's omega from
 * the raw counter and wraps only when it advances (n = (n + 1) % scale_sr), so a counter left at or
 * above a new, lower scale by a track switch (icw_set_input without clr_nframe) is used as is once,
 * and frame t >= 1 sees (n0 + t) mod scale_sr. */
__device__ __forceinline__ double icw_omega(unsigned long long n0, long long t, int scaled, unsigned long long ssr,
                                            uint32_t sample_rate)
{
    if (scaled) {
        /* n0 < ssr except after a rate change, so one subtraction covers any call shorter than ssr
         * frames (1000 s of audio) -- the 64-bit remainder is the rare path */
        unsigned long long n = n0 + (unsigned long long)t;
        if (t != 0 && n >= ssr) n = (n - ssr < ssr) ? n - ssr : n % ssr;
        return (2.0 * ICW_PI) * ((double)n) / ((double)ssr);
    }
    return (2.0 * ICW_PI) * ((double)(n0 + (unsigned long long)t)) / (double)sample_rate;
}

/* The rotation factor e^{j phi} of channel c of an active Shift / PM node at norm_omega
 * (dsp_shift adv_modulator.c:519-550, dsp_pm adv_modulator.c:554-583).  The one definition used by
 * the per-frame table kernel and by the inline path, so both produce the same bits.  fmod is exact;
 * cos / sin are glibc's own (icw_libm.h): the reference's cos + sin pair is one sincos() call in a
 * gcc build, PM's inner sin() is glibc's FMA variant -- so the factors, and everything after them,
 * are bit-identical to the CPU path. */
/* The compiled DSP program is read through the constant address space: its fields are wave-uniform
 * and the kernels never write it, so they come in by scalar loads into SGPRs.  Through a plain
 * pointer the compiler could not prove the kernel's own stores (output, bus, pre-render) leave it
 * alone, and every op field became a vector load, a full vmcnt(0) wait and a v_readfirstlane per
 * use -- in KF2's graph phase ~half of its 1 050 VALU instructions per wave (c2fir SQ pass,
 * profiles/r04_c2fir_phases.json). */
typedef const __attribute__((address_space(4))) IcwProg icw_cprog;
typedef const __attribute__((address_space(4))) IcwOp icw_cop;
__device__ __forceinline__ icw_cprog *icw_prog_c(const IcwProg *p) { return (icw_cprog *)p; }

__device__ __forceinline__ void icw_trig(icw_cop &op, int c, double omega, double &cs, double &sn)
{
    const double ph = fmod(omega * op.f[c], 2.0 * ICW_PI);
    if (op.mode == ICW_MODE_SHIFT) {
        icw_lm_sincos(ph, sn, cs);
        if (op.neg[c]) sn = -sn;
    } else {
        const double psi = op.lp[c] * (icw_lm_sin_fma(ph + op.pp[c]) + op.fa[c]);
        icw_lm_sincos(psi, sn, cs);
    }
}

/* icw_trig out of line, for the per-stream fallback of K2 / K4 (a stream whose frame counter is
 * not stream 0's): inlined, glibc's sincos path added ~45 VGPRs to K2 and cost it a wave per SIMD
 * (141 -> 3 waves) although the per-frame rotation table serves every stream in step. */
__device__ __noinline__ double2 icw_trig_call(icw_cop &op, int c, double omega)
{
    double cs, sn;
    icw_trig(op, c, omega, cs, sn);
    return make_double2(cs, sn);
}

/* One DSP node on its mixed input d (adv_modulator.c:669-751): channel exchange, I/Q swap,
 * gains, then Master (-> lOut/rOut) or Shift / PM / Mix (-> o, returns true).  trow: this frame's
 * row of the rotation table (nullable: compute the factors inline). */
template <bool TRIG = true, bool TAB = false>
__device__ __forceinline__ bool icw_exec_op(icw_cop &op, IcwLR d, double omega, IcwLR &o, double &lOut,
                                            double &rOut, const double *trow = nullptr)
{
    double xt;
    switch (op.xch) {
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
    if (op.iqinv[0]) { xt = d.lre; d.lre = d.lim; d.lim = xt; }
    if (op.iqinv[1]) { xt = d.rre; d.rre = d.rim; d.rim = xt; }
    d.lre *= op.gain[0]; d.lim *= op.gain[0];
    d.rre *= op.gain[1]; d.rim *= op.gain[1];
    switch (op.mode) {
    case ICW_MODE_MASTER:
        lOut = icw_master(op.tout[0], d.lre, d.lim);
        rOut = icw_master(op.tout[1], d.rre, d.rim);
        return false;
    case ICW_MODE_SHIFT:
    case ICW_MODE_PM: {
        if constexpr (!TRIG) { o = d; return true; }   /* no active Shift/PM in the program */
        double cs, sn;
        if (op.act[0]) {
            if (TAB || trow) { cs = trow[op.tslot[0] * 2]; sn = trow[op.tslot[0] * 2 + 1]; }
            else { const double2 f = icw_trig_call(op, 0, omega); cs = f.x; sn = f.y; }
            icw_rot(d.lre, d.lim, cs, sn, o.lre, o.lim);
        } else { o.lre = d.lre; o.lim = d.lim; }
        if (op.act[1]) {
            if (TAB || trow) { cs = trow[op.tslot[1] * 2]; sn = trow[op.tslot[1] * 2 + 1]; }
            else { const double2 f = icw_trig_call(op, 1, omega); cs = f.x; sn = f.y; }
            icw_rot(d.rre, d.rim, cs, sn, o.rre, o.rim);
        } else { o.rre = d.rre; o.rim = d.rim; }
        return true;
    }
    default: /* MIX */
        o = d;
        return true;
    }
}

/* One frame's `in` through the rest of the block (K2 and the fused converter KF2): the bus-form
 * hand-off, or the DSP list (adv_modulator.c:637-751) on the LDS register file, the pre-render
 * doubles and the elementwise ROUND render with the meters' per-thread parts. */
/* DEFER: the rendered integers go to dv[0..1] instead of the output row (KF2 stores 4 frames at once) */
/* Chain-program signatures compiled straight (IcwProg.sig, the host's encoding: the op count in bits
 * 0-3, then per op in execution order (tail first) 4 bits: mode | chain_in << 2).  Each is one of
 * the BASELINE graphs: Master on `in` (C3 / C5), Shift -> Master (C1 / C2), PM -> Shift ->
 * Mix(in + B) -> Master (C4).  Any other chain runs the generic op loop.  (icw_chain_sig below.) */
#define ICW_SIG_M    0x41
#define ICW_SIG_SM   0x852
#define ICW_SIG_PSXM 0x8F964
/* flag: every op but the Master has gain 1.0 on both channels (the BASELINE lists' Shift / PM / Mix,
 * DEF_GAIN_MOD in_cwave.h:166), so the render-only form skips those multiplies at compile time */
#define ICW_SIG_UNIT (1 << 30)
template <bool TRIG, int R, bool ROWP, int SIG, int I>
__device__ __forceinline__ void icw_chain_sig(const IcwK2Args &a, icw_cprog *P, int t0, int T, const IcwLR (&in)[R],
                                              IcwLR (&prev)[R], double (&lOut)[R], double (&rOut)[R], double *bus_s,
                                              bool has_last, int lastr, uint32_t tro_lane, size_t tro_u, size_t tro_step);

/* one frame's rendered integers to the output row (16-bit: one dword per frame; 24-bit: 6 bytes) */
__device__ __forceinline__ void icw_frame_store(const IcwK2Args &a, int s, int t, int vl, int vr)
{
    unsigned char *o = a.out + (size_t)s * a.out_stride;
    if (a.rk.is24) {
        unsigned char *q = o + (size_t)t * 6;
        q[0] = (unsigned char)vl; q[1] = (unsigned char)(vl >> 8); q[2] = (unsigned char)(vl >> 16);
        q[3] = (unsigned char)vr; q[4] = (unsigned char)(vr >> 8); q[5] = (unsigned char)(vr >> 16);
    } else {
        const unsigned pk = ((unsigned)vl & 0xffffu) | ((unsigned)vr << 16);
        *(unsigned *)(o + (size_t)t * 4) = pk;
    }
}

/* (K2 keeps the exact form for every frame: its render-only form, KF2's icw_sig_fast per frame,
 * measured C3 -0.3 %, C4 -0.5 % on one box -- K2 runs beside the recurrence, which bounds C3 / C4) */
template <bool TRIG, bool TAB = false, bool DEFER = false>
__device__ __forceinline__ void icw_frame_graph(const IcwK2Args &a, icw_cprog *P, const IcwRegFile &R, int s,
                                                int t, const IcwLR &in, bool use_tab, unsigned &clip_l,
                                                unsigned &clip_r, double &pk_l, double &pk_r, int *dv = nullptr)
{
    const int T = a.T;
    if (a.iq_out) {
        /* bus-form graph: the serial graph kernel takes it from here (do_render == 0) */
        double *q = a.iq_out + ((size_t)s * T + t) * 4;
        q[0] = in.lre; q[1] = in.lim; q[2] = in.rre; q[3] = in.rim;
    } else {
        const double *trow = use_tab ? a.trig_tab + icw_trig_index(t, a.trig_perm_q) * a.trig_pitch : nullptr;
        const double omega = (TRIG && !use_tab) ? icw_omega(a.n_frame[s], a.t0 + t, a.scaled, a.ssr, a.sample_rate)
                                                : 0.0;
        /* DSP list (adv_modulator.c:637-751) */
        /* persistent bus at the block's last frame: slot 0 = in, then each written slot's
         * final value from the op that writes it (compile_graph: op.wb_slot) */
        const bool last = t == T - 1;
        double *bus_s = a.bus + (size_t)s * ICW_N_INPUTS * 4;
        if (last) { bus_s[0] = in.lre; bus_s[1] = in.lim; bus_s[2] = in.rre; bus_s[3] = in.rim; }
        double lOut = 0.0, rOut = 0.0;
        const int sig = P->sig & ~ICW_SIG_UNIT;
        if (P->chain && (sig == ICW_SIG_M || sig == ICW_SIG_SM || sig == ICW_SIG_PSXM) && (!TRIG || use_tab)) {
            /* a specialised chain signature, factors from the table (or none): the ops straight */
            IcwLR inr[1] = {in}, pv[1] = {in};
            double lo[1] = {0.0}, ro[1] = {0.0};
            const uint32_t tro = TRIG ? (uint32_t)(icw_trig_index(t, a.trig_perm_q) * a.trig_pitch) : 0u;
            if (sig == ICW_SIG_M)
                icw_chain_sig<TRIG, 1, true, ICW_SIG_M, 0>(a, P, t, T, inr, pv, lo, ro, bus_s, last, 0, tro, 0, 0);
            else if (sig == ICW_SIG_SM)
                icw_chain_sig<TRIG, 1, true, ICW_SIG_SM, 0>(a, P, t, T, inr, pv, lo, ro, bus_s, last, 0, tro, 0, 0);
            else
                icw_chain_sig<TRIG, 1, true, ICW_SIG_PSXM, 0>(a, P, t, T, inr, pv, lo, ro, bus_s, last, 0, tro, 0, 0);
            lOut = lo[0];
            rOut = ro[0];
        } else if (P->chain) {
            /* chain program: `in` and the previous op's output in registers, no register file */
            IcwLR prev = in;
            for (int oi = 0; oi < P->n_ops; ++oi) {
                icw_cop &op = P->ops[oi];
                IcwLR d;
                if (P->bypass) {
                    d = in;
                } else {
                    d.lre = d.lim = d.rre = d.rim = 0.0;
                    if (op.chain_in & 1) { d.lre += in.lre; d.lim += in.lim; d.rre += in.rre; d.rim += in.rim; }
                    if (op.chain_in & 2) { d.lre += prev.lre; d.lim += prev.lim; d.rre += prev.rre; d.rim += prev.rim; }
                }
                IcwLR o;
                if (icw_exec_op<TRIG, TAB>(op, d, omega, o, lOut, rOut, trow)) {
                    prev = o;
                    if (last && op.wb_slot >= 0) {
                        double *b = bus_s + op.wb_slot * 4;
                        b[0] = o.lre; b[1] = o.lim; b[2] = o.rre; b[3] = o.rim;
                    }
                }
            }
        } else {
        R.set(0, in);
        for (int oi = 0; oi < P->n_ops; ++oi) {
            icw_cop &op = P->ops[oi];
            IcwLR d;
            if (P->bypass) {
                d = in;
            } else {
                d.lre = d.lim = d.rre = d.rim = 0.0;
                for (int q = 0; q < op.n_in; ++q) {
                    IcwLR v;
                    R.get(op.in_reg[q], v);
                    d.lre += v.lre; d.lim += v.lim; d.rre += v.rre; d.rim += v.rim;
                }
            }
            IcwLR o;
            if (icw_exec_op<TRIG, TAB>(op, d, omega, o, lOut, rOut, trow)) {
                R.set(op.out_reg, o);
                if (last && op.wb_slot >= 0) {
                    double *b = bus_s + op.wb_slot * 4;
                    b[0] = o.lre; b[1] = o.lim; b[2] = o.rre; b[3] = o.rim;
                }
            }
        }
        }   /* register file */

        if (a.pre) {
            double *p = a.pre + (size_t)s * a.pre_stride + (size_t)t * 2;
            p[0] = lOut; p[1] = rOut;
        }
        if (a.do_render) {
            int vl, vr;
            if (a.dith) {
                /* a dithered render with the flat shaper: K3a's terms of this frame, rows 2s, 2s + 1 */
                const double *dd = a.dith + (size_t)(2 * s) * a.dith_pitch + t;
                const double dl = dd[0], dr = dd[a.dith_pitch];
                vl = icw_render_round<true>(lOut, a.rk, clip_l, pk_l, dl);
                vr = icw_render_round<true>(rOut, a.rk, clip_r, pk_r, dr);
            } else {
                vl = icw_render_round(lOut, a.rk, clip_l, pk_l);
                vr = icw_render_round(rOut, a.rk, clip_r, pk_r);
            }
            if constexpr (DEFER) {
                dv[0] = vl;
                dv[1] = vr;
                return;
            }
            icw_frame_store(a, s, t, vl, vr);
        }
    }
}

/* A chain program's op fields as the frame loop uses them, read once per op for all the frames a
 * lane holds (not per frame: the op list lives in global memory, and the loads came back after
 * every store of the frame loop) */
struct IcwOpK {
    int mode, chain_in, xch, iq0, iq1, tout0, tout1, act0, act1, ts0, ts1, wb;
    double g0, g1;
};

__device__ __forceinline__ IcwOpK icw_op_k(icw_cop &op)
{
    IcwOpK k;
    k.mode = op.mode; k.chain_in = op.chain_in; k.xch = op.xch;
    k.iq0 = op.iqinv[0]; k.iq1 = op.iqinv[1];
    k.tout0 = op.tout[0]; k.tout1 = op.tout[1];
    k.act0 = op.act[0]; k.act1 = op.act[1];
    k.ts0 = op.tslot[0]; k.ts1 = op.tslot[1];
    k.wb = op.wb_slot;
    k.g0 = op.gain[0]; k.g1 = op.gain[1];
    return k;
}

/* R frames of one lane (t0 + r; the first nv are in the block) through a chain program, op by op:
 * the op's fields are read once for the R frames and their rotation factors (the per-frame table,
 * every stream in step) are loaded together before the arithmetic.  Per frame the arithmetic of
 * icw_frame_graph + icw_exec_op in the same order, so the bits are the same; the rendered integers
 * go to dv (0 for frames past the block).
 * ROWP: the caller knows where the R frames' table rows are -- frame r's row at
 * a.trig_tab + tro_u + r * tro_step + tro_lane, the first two wave-uniform, the last the lane's (KF2's
 * lanes hold consecutive frames of a tile inside the block, icw_fir_graph) -- so a load needs no
 * per-frame index arithmetic and no clamp.
 * Three shortcuts, each exact: a gain of 1.0 is not multiplied (x * 1.0 is x for every value that is
 * not a signalling NaN, and d is a sum or a converted input here, never one); the bus writes of the
 * block's last frame are tested once per call (one lane of the launch holds it); and the clip
 * counters take one compare per call -- a clip needs |q| >= min(hi, -lo) (clip_abs), so only a call
 * whose largest |q| reaches that counts its samples one by one (a NaN q clips nothing, and fmax
 * passes it over, as the per-sample compares did). */
/* One op of a chain program over the R frames (the body of icw_chain_frames).  MODE / CIN >= 0: the
 * op's mode and chain inputs known at compile time (a specialised signature, ICW_SIG_*), so the
 * compiler keeps only that op's arithmetic and no merges between the modes' results; -1: read from
 * the program (the generic loop).  The other fields are wave-uniform scalars either way. */
template <bool TRIG, int R, bool ROWP, int MODE, int CIN>
__device__ __forceinline__ void icw_chain_op(const IcwK2Args &a, icw_cop &op, bool bypass, int t0, int T,
                                             const IcwLR (&in)[R], IcwLR (&prev)[R], double (&lOut)[R],
                                             double (&rOut)[R], double *bus_s, bool has_last, int lastr,
                                             uint32_t tro_lane, size_t tro_u, size_t tro_step)
{
    constexpr bool plain = MODE >= 0;   /* a signature op: plain fields (compile_graph, IcwProg.sig) */
    const IcwOpK k = icw_op_k(op);
    const int mode = MODE >= 0 ? MODE : k.mode;
    const int cin = CIN >= 0 ? CIN : k.chain_in;
    const bool rot = TRIG && (mode == ICW_MODE_SHIFT || mode == ICW_MODE_PM);
    const bool act0 = plain || k.act0, act1 = plain || k.act1;
    double cs[R][2], sn[R][2];
    if (rot) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            /* (cos, sin) of a channel: one 16-byte load (rows and columns are 16-byte aligned) */
            const double *trow = ROWP ? a.trig_tab + tro_u + (size_t)r * tro_step + tro_lane
                                      : a.trig_tab + icw_trig_index(min(t0 + r, T - 1), a.trig_perm_q) * a.trig_pitch;
            const double2 f0 = act0 ? *(const double2 *)(trow + k.ts0 * 2) : make_double2(0.0, 0.0);
            const double2 f1 = act1 ? *(const double2 *)(trow + k.ts1 * 2) : make_double2(0.0, 0.0);
            cs[r][0] = f0.x; sn[r][0] = f0.y;
            cs[r][1] = f1.x; sn[r][1] = f1.y;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        IcwLR d;
        if (bypass) {
            d = in[r];
        } else {
            d.lre = d.lim = d.rre = d.rim = 0.0;
            if (cin & 1) { d.lre += in[r].lre; d.lim += in[r].lim; d.rre += in[r].rre; d.rim += in[r].rim; }
            if (cin & 2) { d.lre += prev[r].lre; d.lim += prev[r].lim; d.rre += prev[r].rre; d.rim += prev[r].rim; }
        }
        double xt;
        if (!plain) {
            switch (k.xch) {
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
            if (k.iq0) { xt = d.lre; d.lre = d.lim; d.lim = xt; }
            if (k.iq1) { xt = d.rre; d.rre = d.rim; d.rim = xt; }
        }
        if (k.g0 != 1.0) { d.lre *= k.g0; d.lim *= k.g0; }
        if (k.g1 != 1.0) { d.rre *= k.g1; d.rim *= k.g1; }
        if (mode == ICW_MODE_MASTER) {
            lOut[r] = icw_master(plain ? ICW_S_ADD_REIM : k.tout0, d.lre, d.lim);
            rOut[r] = icw_master(plain ? ICW_S_ADD_REIM : k.tout1, d.rre, d.rim);
            continue;
        }
        IcwLR o = d;
        if (rot) {
            if (act0) icw_rot(d.lre, d.lim, cs[r][0], sn[r][0], o.lre, o.lim);
            if (act1) icw_rot(d.rre, d.rim, cs[r][1], sn[r][1], o.rre, o.rim);
        }
        prev[r] = o;
    }
    if (mode != ICW_MODE_MASTER && k.wb >= 0 && has_last) {
        double *b = bus_s + k.wb * 4;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r == lastr) { b[0] = prev[r].lre; b[1] = prev[r].lim; b[2] = prev[r].rre; b[3] = prev[r].rim; }
    }
}

/* op I of signature SIG (ICW_SIG_*, above) */
template <int SIG, int I>
struct icw_sig_op {
    static constexpr int mode = (SIG >> (4 + 4 * I)) & 3;
    static constexpr int cin = (SIG >> (6 + 4 * I)) & 3;
};

template <bool TRIG, int R, bool ROWP, int SIG, int I>
__device__ __forceinline__ void icw_chain_sig(const IcwK2Args &a, icw_cprog *P, int t0, int T, const IcwLR (&in)[R],
                                              IcwLR (&prev)[R], double (&lOut)[R], double (&rOut)[R], double *bus_s,
                                              bool has_last, int lastr, uint32_t tro_lane, size_t tro_u, size_t tro_step)
{
    if constexpr (I < (SIG & 15)) {
        icw_chain_op<TRIG, R, ROWP, icw_sig_op<SIG, I>::mode, icw_sig_op<SIG, I>::cin>(
            a, P->ops[I], false, t0, T, in, prev, lOut, rOut, bus_s, has_last, lastr, tro_lane, tro_u, tro_step);
        icw_chain_sig<TRIG, R, ROWP, SIG, I + 1>(a, P, t0, T, in, prev, lOut, rOut, bus_s, has_last, lastr, tro_lane,
                                                 tro_u, tro_step);
    }
}

/* The render-only form of a signature pass (no pre-render doubles requested, no lane holding the
 * block's last frame): the same rendered integers and meters in about half the instructions (KF2's
 * graph phase, c2fir: ~800 -> ~410 VALU per wave, profiles/r04_c2fir_sq.json).
 *  - An op's input is the sum in + prev without the reference's leading 0.0 + (adv_modulator.c:655-665).
 *    0.0 + x differs from x only for x = -0.0, and in this arithmetic (products, sums, the division by
 *    SQRT2 -- no reciprocal, no sign test) a zero's sign changes nothing but zero signs downstream.
 *    The render cannot see one (below), so the integers and meters are the exact pass's; the pre-render
 *    doubles and the bus state can, which is why those calls and frames take icw_chain_frames' path.
 *  - Gains of 1.0 on every op but the Master (ICW_SIG_UNIT, the BASELINE lists) are left out at
 *    compile time; any other gain of 1.0 is branched over (the compiler had turned the uniform test
 *    into a multiply and two selects per double).
 *  - The division by SQRT2: icw_div_sqrt2's three operations for every value, then one test per value
 *    and one divergent branch per op for those outside its range.
 *  - The render (sound_render_value, ROUND + flat shaper, sound_render.c:747-797): q = x * norm_mul +
 *    copysign(round_offset, x) -- for the mid-riser (offset 0) x + +-0 with x's own sign is x exactly,
 *    for the mid-tread it is the reference's x +- 0.5 except at x = -0.0, where -0.5 and +0.5 both
 *    truncate to 0 and have the same magnitude for the peak and the clip tests; the truncation as
 *    v_cvt_i32_f64 (saturating), and the clip stage (an integer clamp into [lo + 1, hi - 1]: the same
 *    integer as min(q, hi - 1), max(., lo + 1), then (int), for every q that is not a NaN) only in a pass whose
 *    largest |q| reaches min(hi, -lo) -- below it the clamp changes nothing; a NaN q -- INT_MIN, as
 *    x86's cvttsd2si gives -- takes a divergent branch of its own (icw_fast_render). */
__device__ __forceinline__ int icw_cvt_sat_i32(double q)
{
    int v;
    asm("v_cvt_i32_f64_e32 %0, %1" : "=v"(v) : "v"(q));
    return v;
}

__device__ __forceinline__ int icw_med3_i32(int x, int lo, int hi)
{
    int v;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(v) : "v"(x), "v"(lo), "v"(hi));
    return v;
}

/* max(m, |q|) and max(a, b) as one v_max_f64 each: IEEE maxNum returns the number for a quiet NaN
 * operand, as fmax; written out because the compiler canonicalised both operands of every fmax here
 * (two more v_max_f64 per sample).  The operands are sums and products, never signalling NaNs. */
__device__ __forceinline__ double icw_vmax_abs(double m, double q)
{
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(q));
    return r;
}

__device__ __forceinline__ double icw_vmax(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

/* max(|a|, |b|) as one v_max_f64: a NaN operand gives the other magnitude (maxNum), two NaNs a NaN */
__device__ __forceinline__ double icw_vmax_abs2(double a, double b)
{
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

/* The render of the R frames (see above).  MR: mid-riser, q = x (x + +-0.0 with x's sign is x) and
 * delta = -1 below zero; mid-tread: q = copysign(|x| + 0.5, x), the reference's x +- 0.5 (-0.0 gives
 * -0.5, harmless as above), delta 0.  The integer is the saturating conversion; the clamp to
 * [lo + 1, hi - 1] is needed only where |q| reaches clip_abs = min(hi, -lo) -- the pass's meter test
 * -- so it is applied there with the clip counts.  Then the NaN samples: INT_MIN (delta 0). */
template <bool MR, bool SH0, int R>
__device__ __forceinline__ void icw_fast_render(const IcwRenderK &rk, const double (&x)[R][2], int (&dv)[R][2],
                                                double &lm_l, double &lm_r, unsigned &clip_l, unsigned &clip_r)
{
    /* SH0: norm_shift 0 (full sign bits, the usual case) -- no shift after the integer, so the
     * mid-riser's delta folds into one subtract-with-borrow of the compare */
    const int sh = SH0 ? 0 : rk.norm_shift;
    static_assert(R >= 2, "the meters start from the first two frames");
    double q[R][2];
    int del[R][2];
    bool nan = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if constexpr (MR) {
                q[r][c] = x[r][c];
                del[r][c] = x[r][c] < 0.0 ? -1 : 0;               /* sign_delta -1 (icw_launch_fir_graph checks) */
            } else {
                q[r][c] = __builtin_copysign(fabs(x[r][c]) + rk.round_offset, x[r][c]);
                del[r][c] = 0;
            }
            dv[r][c] = (int)((unsigned)(icw_cvt_sat_i32(q[r][c]) + del[r][c]) << sh);
            nan |= q[r][c] != q[r][c];
        }
    }
    /* the largest |q| of the frames (a NaN q counts as nothing, as fmax from 0.0 does; all-NaN
     * frames give a NaN here, which no comparison passes and the peak's v_max_f64 skips) */
    lm_l = icw_vmax_abs2(q[0][0], q[1][0]);
    lm_r = icw_vmax_abs2(q[0][1], q[1][1]);
#pragma unroll
    for (int r = 2; r < R; ++r) {
        lm_l = icw_vmax_abs(lm_l, q[r][0]);
        lm_r = icw_vmax_abs(lm_r, q[r][1]);
    }
    if (icw_vmax(lm_l, lm_r) >= rk.clip_abs) {
        /* the host's integer bounds (SGPRs), integer min / max: (int)rk.lo is a VALU conversion, whose
         * result the compiler hoisted to the kernel entry and spilled (+1.6 B of scratch writes per
         * c2fir frame), and a v_med3_i32 wants VGPR operands */
        const int lo1 = rk.lo1, hi1 = rk.hi1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            clip_l += (q[r][0] >= rk.hi ? 1u : 0u) + (q[r][0] <= rk.lo ? 1u : 0u);
            clip_r += (q[r][1] >= rk.hi ? 1u : 0u) + (q[r][1] <= rk.lo ? 1u : 0u);
#pragma unroll
            for (int c = 0; c < 2; ++c)
                dv[r][c] = (int)((unsigned)(min(max(icw_cvt_sat_i32(q[r][c]), lo1), hi1) + del[r][c]) << sh);
        }
    }
    if (nan) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c)
                if (q[r][c] != q[r][c]) dv[r][c] = (int)(0x80000000u << sh);
    }
}

/* 16 bytes at a wave-uniform base + a lane's 32-bit byte offset, as a raw buffer load: the base goes
 * into the descriptor (SGPRs), so no address arithmetic runs on the VALU -- a global load took a
 * v_lshl_add_u64 per load (the lane offset held as 64 bits), 4-8 per pass of the fused converter */
__device__ __forceinline__ double2 icw_ld_row2(const double *base, uint32_t lane_bytes)
{
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7fffffff, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)lane_bytes, 0, 0);
    double2 d;
    d.x = __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
    d.y = __longlong_as_double((long long)(((unsigned long long)v[3] << 32) | v[2]));
    return d;
}

template <bool TRIG, int R, int SIG, int I>
__device__ __forceinline__ void icw_sig_fast_ops(const IcwK2Args &a, icw_cprog *P, const IcwLR (&in)[R],
                                                 IcwLR (&prev)[R], double (&lOut)[R], double (&rOut)[R],
                                                 uint32_t tro_lane, size_t tro_u, size_t tro_step)
{
    if constexpr (I < (SIG & 15)) {
        constexpr int mode = icw_sig_op<SIG, I>::mode, cin = icw_sig_op<SIG, I>::cin;
        constexpr bool rot = TRIG && (mode == ICW_MODE_SHIFT || mode == ICW_MODE_PM);
        icw_cop &op = P->ops[I];
        double cs[R][2], sn[R][2];
        if constexpr (rot) {
            const int ts0 = op.tslot[0], ts1 = op.tslot[1];
            /* a wave-uniform row base (SGPRs) + the lane's 32-bit byte offset */
            const uint32_t lane_b = tro_lane * 8u;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const double2 f0 = icw_ld_row2(a.trig_tab + tro_u + (size_t)r * tro_step + ts0 * 2, lane_b);
                const double2 f1 = icw_ld_row2(a.trig_tab + tro_u + (size_t)r * tro_step + ts1 * 2, lane_b);
                cs[r][0] = f0.x; sn[r][0] = f0.y;
                cs[r][1] = f1.x; sn[r][1] = f1.y;
            }
        }
        IcwLR d[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if constexpr (cin == 1) d[r] = in[r];
            else if constexpr (cin == 2) d[r] = prev[r];
            else if constexpr (cin == 3) {
                d[r].lre = in[r].lre + prev[r].lre; d[r].lim = in[r].lim + prev[r].lim;
                d[r].rre = in[r].rre + prev[r].rre; d[r].rim = in[r].rim + prev[r].rim;
            } else {
                d[r].lre = d[r].lim = d[r].rre = d[r].rim = 0.0;
            }
        }
        constexpr bool unit = (SIG & ICW_SIG_UNIT) && mode != ICW_MODE_MASTER;
        const double g0 = op.gain[0], g1 = op.gain[1];
        if (!unit && (ICW_SCALAR_UNIT ? !op.unit_gain[0] : g0 != 1.0)) {
            asm volatile("");
#pragma unroll
            for (int r = 0; r < R; ++r) { d[r].lre *= g0; d[r].lim *= g0; }
        }
        if (!unit && (ICW_SCALAR_UNIT ? !op.unit_gain[1] : g1 != 1.0)) {
            asm volatile("");
#pragma unroll
            for (int r = 0; r < R; ++r) { d[r].rre *= g1; d[r].rim *= g1; }
        }
        if constexpr (mode == ICW_MODE_MASTER) {
            double x[R][2];
            bool slow = false;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                x[r][0] = d[r].lre + d[r].lim;
                x[r][1] = d[r].rre + d[r].rim;
                lOut[r] = icw_div_sqrt2_fast(x[r][0]);
                rOut[r] = icw_div_sqrt2_fast(x[r][1]);
                slow |= !icw_div_sqrt2_ok(lOut[r]) || !icw_div_sqrt2_ok(rOut[r]);
            }
            if (slow) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (!icw_div_sqrt2_ok(lOut[r])) lOut[r] = x[r][0] / ICW_SQRT2;
                    if (!icw_div_sqrt2_ok(rOut[r])) rOut[r] = x[r][1] / ICW_SQRT2;
                }
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if constexpr (rot) {
                    icw_rot(d[r].lre, d[r].lim, cs[r][0], sn[r][0], prev[r].lre, prev[r].lim);
                    icw_rot(d[r].rre, d[r].rim, cs[r][1], sn[r][1], prev[r].rre, prev[r].rim);
                } else {
                    prev[r] = d[r];
                }
            }
        }
        icw_sig_fast_ops<TRIG, R, SIG, I + 1>(a, P, in, prev, lOut, rOut, tro_lane, tro_u, tro_step);
    }
}

template <bool TRIG, int R, int SIG>
__device__ __forceinline__ void icw_sig_fast(const IcwK2Args &a, icw_cprog *P, const IcwLR (&in)[R], unsigned &clip_l,
                                             unsigned &clip_r, double &pk_l, double &pk_r, int (&dv)[R][2],
                                             uint32_t tro_lane, size_t tro_u, size_t tro_step)
{
    IcwLR prev[R];
    double lOut[R], rOut[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        prev[r] = in[r];
        lOut[r] = rOut[r] = 0.0;
    }
    icw_sig_fast_ops<TRIG, R, SIG, 0>(a, P, in, prev, lOut, rOut, tro_lane, tro_u, tro_step);
    const IcwRenderK &rk = a.rk;
    double x[R][2];
#pragma unroll
    for (int r = 0; r < R; ++r) { x[r][0] = lOut[r]; x[r][1] = rOut[r]; }
    if (ICW_SCALAR_UNIT ? !rk.unit_mul : rk.norm_mul != 1.0) {
        asm volatile("");
#pragma unroll
        for (int r = 0; r < R; ++r) { x[r][0] *= rk.norm_mul; x[r][1] *= rk.norm_mul; }
    }
    double lm_l, lm_r;
    if (ICW_RENDER_SH0 && rk.norm_shift == 0) {
        if (rk.sign_delta != 0) icw_fast_render<true, true, R>(rk, x, dv, lm_l, lm_r, clip_l, clip_r);
        else icw_fast_render<false, true, R>(rk, x, dv, lm_l, lm_r, clip_l, clip_r);
    } else {
        if (rk.sign_delta != 0) icw_fast_render<true, false, R>(rk, x, dv, lm_l, lm_r, clip_l, clip_r);
        else icw_fast_render<false, false, R>(rk, x, dv, lm_l, lm_r, clip_l, clip_r);
    }
    pk_l = icw_vmax(pk_l, lm_l);
    pk_r = icw_vmax(pk_r, lm_r);
}

template <bool TRIG, int R, bool ROWP = false, int SIG = 0>
__device__ __forceinline__ void icw_chain_frames(const IcwK2Args &a, icw_cprog *P, int s, int t0, int nv,
                                                 const IcwLR (&in)[R], unsigned &clip_l, unsigned &clip_r,
                                                 double &pk_l, double &pk_r, int (&dv)[R][2], uint32_t tro_lane = 0,
                                                 size_t tro_u = 0, size_t tro_step = 0)
{
    const int T = a.T;
    double *bus_s = a.bus + (size_t)s * ICW_N_INPUTS * 4;
    const int lastr = T - 1 - t0;                    /* the block's last frame is frame lastr here */
    const bool has_last = lastr >= 0 && lastr < nv;
    if constexpr (SIG != 0 && ROWP) {
        /* the render-only form when no lane of the wave needs the exact doubles */
        if (!a.pre && __all(nv == R && !has_last)) {
            icw_sig_fast<TRIG, R, SIG>(a, P, in, clip_l, clip_r, pk_l, pk_r, dv, tro_lane, tro_u, tro_step);
            return;
        }
    }
    IcwLR prev[R];
    double lOut[R], rOut[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        prev[r] = in[r];
        lOut[r] = rOut[r] = 0.0;
    }
    if (has_last) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r == lastr) { bus_s[0] = in[r].lre; bus_s[1] = in[r].lim; bus_s[2] = in[r].rre; bus_s[3] = in[r].rim; }
    }
    if constexpr (SIG != 0) {
        /* a signature has no bypass: a bypassed list is the Master alone reading nothing (chain_in 0) */
        icw_chain_sig<TRIG, R, ROWP, SIG & ~ICW_SIG_UNIT, 0>(a, P, t0, T, in, prev, lOut, rOut, bus_s, has_last, lastr,
                                                             tro_lane, tro_u, tro_step);
    } else {
        const bool bypass = P->bypass != 0;
        for (int oi = 0; oi < P->n_ops; ++oi)
            icw_chain_op<TRIG, R, ROWP, -1, -1>(a, P->ops[oi], bypass, t0, T, in, prev, lOut, rOut, bus_s, has_last, lastr,
                                                tro_lane, tro_u, tro_step);
    }
    const IcwRenderK &rk = a.rk;
    double q[R][2], lm_l = 0.0, lm_r = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        dv[r][0] = dv[r][1] = 0;
        q[r][0] = q[r][1] = 0.0;
        if (r < nv) {
            if (a.pre) {
                double *p = a.pre + (size_t)s * a.pre_stride + (size_t)(t0 + r) * 2;
                p[0] = lOut[r]; p[1] = rOut[r];
            }
#if ICW_FIR_DIAG & 2
            q[r][0] = lOut[r]; q[r][1] = rOut[r];
            dv[r][0] = (int)lOut[r]; dv[r][1] = (int)rOut[r];
#else
            dv[r][0] = icw_render_round_q(lOut[r], rk, q[r][0]);
            dv[r][1] = icw_render_round_q(rOut[r], rk, q[r][1]);
#endif
            lm_l = fmax(lm_l, fabs(q[r][0]));
            lm_r = fmax(lm_r, fabs(q[r][1]));
        }
    }
    pk_l = fmax(pk_l, lm_l);
    pk_r = fmax(pk_r, lm_r);
    if (fmax(lm_l, lm_r) >= rk.clip_abs) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            clip_l += (q[r][0] >= rk.hi ? 1u : 0u) + (q[r][0] <= rk.lo ? 1u : 0u);
            clip_r += (q[r][1] >= rk.hi ? 1u : 0u) + (q[r][1] <= rk.lo ? 1u : 0u);
        }
    }
}

/* the chain frames of one call through the program's signature when it is a specialised one */
template <bool TRIG, int R>
__device__ __forceinline__ void icw_chain_frames_rowp(const IcwK2Args &a, icw_cprog *P, int sig, int s, int t0, int nv,
                                                      const IcwLR (&in)[R], unsigned &clip_l, unsigned &clip_r,
                                                      double &pk_l, double &pk_r, int (&dv)[R][2], uint32_t tro_lane,
                                                      size_t tro_u, size_t tro_step)
{
    /* a plain Shift / PM always rotates, so a kernel without TRIG sees only the Master signature and
     * carries only that one: with all of them the mono kernel spilled in its loop (c3fir WRITE_SIZE
     * 1.98 against 1.09 GB per launch).  The TRIG kernels keep the Master case they never take: without
     * it the stereo kernel's allocation spilled instead (c2fir 96 against 67 MB). */
    if constexpr (TRIG) {
        switch (sig) {
        case ICW_SIG_M:
        case ICW_SIG_M | ICW_SIG_UNIT:
            icw_chain_frames<TRIG, R, true, ICW_SIG_M | ICW_SIG_UNIT>(a, P, s, t0, nv, in, clip_l, clip_r, pk_l, pk_r,
                                                                    dv, tro_lane, tro_u, tro_step);
            return;
        case ICW_SIG_SM:
            icw_chain_frames<TRIG, R, true, ICW_SIG_SM>(a, P, s, t0, nv, in, clip_l, clip_r, pk_l, pk_r, dv, tro_lane,
                                                        tro_u, tro_step);
            return;
        case ICW_SIG_SM | ICW_SIG_UNIT:
            icw_chain_frames<TRIG, R, true, ICW_SIG_SM | ICW_SIG_UNIT>(a, P, s, t0, nv, in, clip_l, clip_r, pk_l, pk_r,
                                                                     dv, tro_lane, tro_u, tro_step);
            return;
        case ICW_SIG_PSXM:
            icw_chain_frames<TRIG, R, true, ICW_SIG_PSXM>(a, P, s, t0, nv, in, clip_l, clip_r, pk_l, pk_r, dv, tro_lane,
                                                          tro_u, tro_step);
            return;
        case ICW_SIG_PSXM | ICW_SIG_UNIT:
            icw_chain_frames<TRIG, R, true, ICW_SIG_PSXM | ICW_SIG_UNIT>(a, P, s, t0, nv, in, clip_l, clip_r, pk_l,
                                                                       pk_r, dv, tro_lane, tro_u, tro_step);
            return;
        default: break;
        }
    } else {
        if (sig == ICW_SIG_M || sig == (ICW_SIG_M | ICW_SIG_UNIT)) {
            icw_chain_frames<TRIG, R, true, ICW_SIG_M | ICW_SIG_UNIT>(a, P, s, t0, nv, in, clip_l, clip_r, pk_l, pk_r, dv,
                                                                    tro_lane, tro_u, tro_step);
            return;
        }
    }
    icw_chain_frames<TRIG, R, true>(a, P, s, t0, nv, in, clip_l, clip_r, pk_l, pk_r, dv, tro_lane, tro_u, tro_step);
}

/* The stereo I / Q exchange between lane l (channel L) and lane l + 32 (channel R) of a wave: with
 * a = x[r] and b = x[r + 4] of each lane, afterwards a = L's value and b = R's value of the lane's
 * frame (lane l: frame r, lane l + 32: frame r + 4).  v_permlane32_swap trades the upper half of one
 * VGPR with the lower half of another on the VALU, two per double, where __shfl_xor(x, 32) took two
 * ds_bpermute round trips through the LDS plus a select (c2fir kernel 0.331 -> 0.328 ms, c4fir
 * 3.114 -> 3.084 ms, profiles/r03_fir_swap_ab.jsonl). */
__device__ __forceinline__ void icw_swap32(double &a, double &b)
{
    const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    a = __longlong_as_double(((unsigned long long)hi[0] << 32) | lo[0]);
    b = __longlong_as_double(((unsigned long long)hi[1] << 32) | lo[1]);
}

/* peak / clip reduction slots of a workgroup: per channel two per wave, one per 16-lane row (icw_meters_wg;
 * every caller runs ICW_K2_TILE threads, KF2's launch bound included) */
#define ICW_PK_SLOTS (ICW_K2_TILE / 32)
static_assert(ICW_K2_TILE == 256, "icw_fir_graph launches 256 threads and shares icw_meters_wg's slots");

/* every lane of a 16-lane row gets the row's largest value, for doubles >= +0.0 that are never a NaN
 * (so v_max_f64 without canonicalising, and any order gives the same value): DPP row_ror 8, 4, 2, 1,
 * each two v_mov_b32_dpp and one v_max_f64.  Full EXEC. */
template <int CTRL>
__device__ __forceinline__ double icw_dpp_max_nn(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return icw_vmax(v, __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo)));
}

__device__ __forceinline__ double icw_row_max_nn(double v)
{
    v = icw_dpp_max_nn<0x128>(v);                    /* row_ror:8 */
    v = icw_dpp_max_nn<0x124>(v);                    /* row_ror:4 */
    v = icw_dpp_max_nn<0x122>(v);                    /* row_ror:2 */
    return icw_dpp_max_nn<0x121>(v);                 /* row_ror:1 */
}

/* the sum over a 16-lane row, in every lane of it (the same rotations) */
__device__ __forceinline__ unsigned icw_row_sum_u32(unsigned v)
{
    v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x122, 0xf, 0xf, false);
    return v + (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xf, 0xf, false);
}

/* per-workgroup meters (ICW_K2_TILE threads, full EXEC): row reduce, LDS, one atomic per
 * stream/channel.  The peaks are maxima of |q| from +0.0 (fmax / v_max_f64 return the number for a
 * NaN operand), so they are >= +0.0 and never a NaN, and their maximum is the same in any order; the
 * clip counts are sums of integers.  The two channels share one reduction: v_permlane32_swap leaves
 * lanes 0-31 with channel L's values of lanes l and l + 32 and lanes 32-63 with channel R's (one
 * max), each 16-lane row is reduced by DPP, and lanes 0 and 16 (L) / 32 and 48 (R) hand their row's
 * maximum to the final reduction -- ~15 VALU per wave where two device-library wave reductions
 * (-inf fills, canonicalising maxima, cross-row steps) took ~75 in the fused converter's graph phase.
 * The counts are reduced only when a lane of the wave clipped (a ballot), the usual case being none. */
__device__ __forceinline__ void icw_meters_wg(const IcwK2Args &a, int s, unsigned clip_l, unsigned clip_r, double pk_l,
                                              double pk_r, unsigned (*red_clip)[ICW_PK_SLOTS],
                                              double (*red_pk)[ICW_PK_SLOTS])
{
    const int tl = threadIdx.x, ln = tl & 63, wv = tl >> 6;
    const bool any_clip = __any((clip_l | clip_r) != 0u);
    if (any_clip) {
        const auto c = __builtin_amdgcn_permlane32_swap(clip_l, clip_r, false, false);
        const unsigned cs = icw_row_sum_u32(c[0] + c[1]);
        if ((ln & 15) == 0) red_clip[ln >> 5][2 * wv + ((ln >> 4) & 1)] = cs;
    } else if ((ln & 15) == 0) {
        red_clip[ln >> 5][2 * wv + ((ln >> 4) & 1)] = 0u;
    }
    icw_swap32(pk_l, pk_r);
    const double pk = icw_row_max_nn(icw_vmax(pk_l, pk_r));
    if ((ln & 15) == 0) red_pk[ln >> 5][2 * wv + ((ln >> 4) & 1)] = pk;
    __syncthreads();
    if (tl < 2) {
        unsigned cs = 0; double pm = 0.0;
        for (int i = 0; i < ICW_PK_SLOTS; ++i) { cs += red_clip[tl][i]; pm = fmax(pm, red_pk[tl][i]); }
        if (cs) atomicAdd(&a.clips[s * 2 + tl], cs);
        if (pm > 0.0) atomicMax(&a.peak_bits[s * 2 + tl], (unsigned long long)__double_as_longlong(pm));
    }
}

/* One frame of K2: the four chains' output sums from their w rows (w[c]: the row at the frame's
 * window, w[c][N] the state after the frame), the de-subnorm counts, the fs/4 un-mix, then the
 * frame graph.  dup: mono input with bit-identical converters, chains 2-3 are copies of 0-1. */
template <int N, bool KAHAN, bool TRIG, bool FCK>
__device__ __forceinline__ void icw_output_frame(const IcwK2Args &a, icw_cprog *P, const IcwRegFile &R, int s,
                                                 int t, const double *const (&w)[4], bool dup, const double *lc,
                                                 IcwFes (&fes)[2], bool count_sn, unsigned (&sn)[4], bool use_tab,
                                                 unsigned &clip_l, unsigned &clip_r, double &pk_l, double &pk_r)
{
    IcwLR in;
    if (a.cw) {
        /* complex (CWAVE) input: the analytic signal as read (xwave_reader.c:939-966) */
        const double *xs = a.xin + (size_t)s * 4 * a.x_pitch + t;
        in.lre = xs[0]; in.lim = xs[a.x_pitch]; in.rre = xs[2 * a.x_pitch]; in.rim = xs[3 * a.x_pitch];
    } else {
        const int nc = dup ? 2 : 4;
        if (count_sn) {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < nc) sn[c] += (w[c][N] == 0.0) ? 1u : 0u;
        }
        /* filter outputs of the 4 chains (L-I, L-Q, R-I, R-Q) */
        double y[4];
        if constexpr (FCK) {
#pragma unroll 1
            for (int c = 0; c < 4; ++c) y[c] = icw_iir_out_fc(w[c], N, KAHAN, lc, lc + 20, a.d0, fes[c >> 1]);
        } else if (dup) {
            const double *const wins[2] = {w[0], w[1]};
            double y2[2];
            icw_iir_out_n<N, KAHAN, 2>(wins, lc, lc + 20, a.d0, y2);
            y[0] = y[2] = y2[0];
            y[1] = y[3] = y2[1];
        } else {
            icw_iir_out_n<N, KAHAN, 4>(w, lc, lc + 20, a.d0, y);
        }
        /* fs/4 un-mix (lpf_hilbert_quad.c:129-156) */
        double oI[2], oQ[2];
#pragma unroll
        for (int ch = 0; ch < 2; ++ch) {
            const double yi = y[ch * 2], yq = y[ch * 2 + 1];
            const unsigned kq = (a.hq_phase[s * 2 + ch] + (unsigned)(a.t0 + t)) & 3u;
            switch (kq) {
            case 0: oI[ch] = yi * 2.0; oQ[ch] = yq * 2.0; break;
            case 1: oI[ch] = -yq * 2.0; oQ[ch] = yi * 2.0; break;
            case 2: oI[ch] = -yi * 2.0; oQ[ch] = -yq * 2.0; break;
            default: oI[ch] = yq * 2.0; oQ[ch] = -yi * 2.0; break;
            }
        }
        in.lre = oI[0]; in.lim = oQ[0]; in.rre = oI[1]; in.rim = oQ[1];
    }
    icw_frame_graph<TRIG>(a, P, R, s, t, in, use_tab, clip_l, clip_r, pk_l, pk_r);
}

/* the workgroup's de-subnorm counts, one atomic per chain (nc chains computed; dup: the right
 * converters ran identically, so they rejected the same samples) */
__device__ __forceinline__ void icw_sn_wg(const IcwK2Args &a, int s, const unsigned (&sn)[4], int nc,
                                          unsigned (*red_sn)[ICW_K2_TILE / 64])
{
    const int tl = threadIdx.x, wv = tl >> 6;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        unsigned v = sn[c];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((tl & 63) == 0) red_sn[c][wv] = v;
    }
    __syncthreads();
    if (tl < 4) {
        unsigned long long tot = 0;
        for (int i = 0; i < ICW_K2_TILE / 64; ++i) tot += red_sn[tl < nc ? tl : tl - 2][i];
        if (tot) atomicAdd(&a.sncnt[(size_t)s * 4 + tl], tot);
    }
}

/* Output kernel (K2).  A workgroup owns a.tpw (<= ICW_K2_TPW) consecutive 256-frame tiles of one
 * stream (fewer when a launch would have too few workgroups to spread over the chip).
 * The w window of tile k+1 is loaded into registers while tile k is computed, then written to the
 * other half of a double-buffered LDS window: the global-load latency hides behind FP64 work and
 * the meters reduce once per workgroup.  TRIG = the program has an active Shift / PM node. */
#ifndef ICW_K2_MINWG
#define ICW_K2_MINWG 1
#endif
template <int N, bool KAHAN, bool TRIG, bool FCK = false>
__device__ __forceinline__ void icw_output_body(const IcwK2Args &a, int bx, int s, double *lregs)
{
    constexpr int TILE = ICW_K2_TILE;
    constexpr int NR = N + 1;                        /* window rows past the tile (row N+t: w[t]) */
    __shared__ double lw[2][4][TILE + 24];
    /* lregs: the DSP register file [n_regs][4][TILE] in dynamic LDS */
    __shared__ unsigned red_clip[2][ICW_PK_SLOTS];
    __shared__ double red_pk[2][ICW_PK_SLOTS];
    const int tl = threadIdx.x;
    const int T = a.T;
    const int tw0 = bx * TILE * a.tpw;
    const int ntile = min(a.tpw, (T - tw0 + TILE - 1) / TILE);

    /* mono input, converters bit-identical at block start (K1's flag) and in phase: the right
     * filter outputs are copies of the left ones this block */
    const bool dup = !FCK && !a.cw && a.nch == 1 && a.info_dup && a.info_dup[s * 2] && a.info_dup[s * 2 + 1] &&
                     a.hq_phase[s * 2] == a.hq_phase[s * 2 + 1];
    IcwFes fes[2] = {};
    const int nc = dup ? 2 : 4;
    /* the per-frame rotation table holds this stream's factors when its counter is in step */
    const bool use_tab = TRIG && a.trig_tab && a.n_frame[s] == a.n_frame[0];
    double pf[4][2];
    auto load_tile = [&](int k) {
        const int tt = tw0 + k * TILE;
        const int nrow = min(TILE, T - tt) + NR;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < nc) {
                const double *src = a.w + (size_t)(s * 4 + c) * a.w_pitch + tt;
                pf[c][0] = tl < nrow ? src[tl] : 0.0;
                pf[c][1] = (tl < NR && tl + TILE < nrow) ? src[tl + TILE] : 0.0;
            }
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < nc) {
                lw[buf][c][tl] = pf[c][0];
                if (tl < NR) lw[buf][c][tl + TILE] = pf[c][1];
            }
        }
    };
    if (!a.cw) {
        load_tile(0);
        store_tile(0);
        __syncthreads();
    }

    icw_cprog *P = icw_prog_c(a.prog);
    IcwRegFile R;
    R.base = lregs + tl;
    /* slots read but never written in the frame hold their block-start values */
    for (int r = 0; r < P->n_persist; ++r) {
        const double *b = a.bus + ((size_t)s * ICW_N_INPUTS + P->persist_slot[r]) * 4;
        IcwLR v; v.lre = b[0]; v.lim = b[1]; v.rre = b[2]; v.rim = b[3];
        R.set(P->persist_reg[r], v);
    }
    /* the 2N output-sum coefficients are read from LDS (broadcast) at their one use per frame:
     * held in SGPRs they crowd out the program's operands and spill to VGPR lanes, a v_readlane
     * per use.  `zk` (a runtime zero) keeps the loads inside the tile loop. */
    __shared__ double lcoef[40];
    if (tl < 40) lcoef[tl] = tl < 20 ? a.pc[tl] : a.pd[tl - 20];
    __syncthreads();

    unsigned clip_l = 0, clip_r = 0;
    double pk_l = 0.0, pk_r = 0.0;
    /* de-subnorm rejections of this workgroup's frames, per chain: the reject stores exactly +0.0
     * (hblpf.c:1046-1050) and every |sum| < 1 is rejected, so a w row equal to 0.0 is one count */
    const bool count_sn = !a.cw && a.sncnt;
    unsigned sn[4] = {0u, 0u, 0u, 0u};
    for (int k = 0; k < ntile; ++k) {
        const bool more = !a.cw && k + 1 < ntile;
        if (more) load_tile(k + 1);
        const int t = tw0 + k * TILE + tl;
        const double (&W)[4][TILE + 24] = lw[k & 1];
        const int zk = a.zero * k;
        if (t < T) {
            const double *const w[4] = {&W[0][tl], &W[1][tl], &W[2][tl], &W[3][tl]};
            icw_output_frame<N, KAHAN, TRIG, FCK>(a, P, R, s, t, w, dup, lcoef + zk, fes, count_sn, sn, use_tab, clip_l,
                                                  clip_r, pk_l, pk_r);
        }
        if (more) {
            /* the other half was last read in tile k-1, before the previous barrier */
            store_tile((k + 1) & 1);
            __syncthreads();
        }
    }

    if constexpr (FCK) {
        icw_fes_flush(fes[0], a.fes + (size_t)s * 4 * ICW_FES_PITCH);
        icw_fes_flush(fes[1], a.fes + ((size_t)s * 4 + 1) * ICW_FES_PITCH);
    }
    if (count_sn) {
        __shared__ unsigned red_sn[4][TILE / 64];
        icw_sn_wg(a, s, sn, nc, red_sn);
    }
    if (a.do_render) icw_meters_wg(a, s, clip_l, clip_r, pk_l, pk_r, red_clip, red_pk);
}

template <int N, bool KAHAN, bool TRIG, bool FCK = false>
__global__ __launch_bounds__(ICW_K2_TILE, ICW_K2_MINWG) void icw_output(IcwK2Args a)
{
    extern __shared__ __attribute__((aligned(16))) double lregs[];   /* [n_regs][4][TILE] */
    icw_output_body<N, KAHAN, TRIG, FCK>(a, blockIdx.x, blockIdx.y, lregs);
}

/* Fused FIR converter + graph + render (KF2): one workgroup per stream and 1024-frame tile (2048
 * for mono).  Wave w owns frames [256 w, 256 w + 256) of the tile: lanes 0-31 sum channel L's
 * outputs and lanes 32-63 channel R's, 8 consecutive frames each (icw_fir_sums).  A lane pair
 * (l, l + 32) then swaps half of its I / Q values (v_permlane32_swap), so lane l holds both channels
 * of frames 0-3 of its eight and lane l + 32 of frames 4-7, and each takes its 4 frames straight
 * through K2's per-frame code (icw_frame_graph: DSP list, pre-render, ROUND render, meters).  The
 * analytic signal never leaves the registers (KF + K2 move 32 B per frame through HBM twice); the
 * sums are KF's, in the same order, so the results are KF + K2's bit for bit.  Dynamic LDS: the
 * padded inputs of each computed channel, the taps, the DSP register file. */
/* Occupancy: 4 workgroups per CU (4 waves per SIMD, <= 128 VGPRs).  TAB: every stream of the launch
 * is in step with the rotation table (the host's frame-counter mirror says so), so the per-stream
 * fallback (icw_trig_call) is compiled out.  With the call in the kernel the allocator kept values
 * live across it in scratch -- 44 B per thread written to HBM, most of the kernel's 2.95x write
 * traffic (profiles/r02_c2fir_pmc.json: 198 MB per launch against 67 MB of output); giving that
 * variant 168 VGPRs instead (3 workgroups per CU) removed the spills but cost c2fir 22 %. */

/* NC: computed channels (1: mono input, 2: stereo), a template parameter so that each form gets its
 * own register allocation (the mono graph phase holds 8 frames per lane, the stereo one 4) */
#if ICW_FIR_STAMPS
/* diagnostic build only (tools/fir_phases.py): per workgroup of the last KF2 launch, wave 0's
 * shader-clock stamps at the phase boundaries and the 100 MHz clock at its start and end */
__device__ unsigned long long icw_fir_stp[(1 << 16) * 8];
#define ICW_FIR_STAMP(k)                                                                              \
    do {                                                                                              \
        if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < (1u << 16))                     \
            icw_fir_stp[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (k)] =                            \
                ((k) == 0 || (k) == 7) ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime(); \
    } while (0)
extern "C" int icw_fir_stamps_read(unsigned long long *dst, size_t n)
{
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(icw_fir_stp), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#else
#define ICW_FIR_STAMP(k) do { } while (0)
#endif

/* KF2's mono chain form: the lane's ICW_FIR_R frames (from t0, nv of them in the block) two at a time
 * through one signature (SIG; 0: the generic op loop, ROWP: rows at known offsets), the rendered
 * frames packed into w (16-bit: w[0..8), 24-bit: 12 words).  B24 is a template parameter: with a
 * runtime flag the compiler merged the two packings' stores into one store at a selected index, which
 * put w in scratch -- c3fir wrote 6.3 GB per launch against 4.3 GB of output (profiles/r05_c3fir_pmc.json) */
template <bool TRIG, int SIG, bool ROWP, bool B24>
__device__ __forceinline__ void icw_mono_passes(const IcwK2Args &a, icw_cprog *P, int s, int t0, int nv,
                                                const double (&vi)[ICW_FIR_R], const double (&q)[ICW_FIR_R],
                                                unsigned &clip_l, unsigned &clip_r, double &pk_l, double &pk_r,
                                                unsigned (&w)[ICW_FIR_R / 2 * 3], uint32_t tro_lane, size_t pq)
{
#pragma unroll
    for (int hh = 0; hh < ICW_FIR_R; hh += 2) {
        IcwLR in2[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            in2[r].lre = in2[r].rre = vi[hh + r];
            in2[r].lim = in2[r].rim = q[hh + r];
        }
        int dv[2][2];
        const int n2 = min(2, max(nv - hh, 0));
        if constexpr (!ROWP)
            icw_chain_frames<TRIG, 2>(a, P, s, t0 + hh, n2, in2, clip_l, clip_r, pk_l, pk_r, dv);
        else if constexpr (SIG != 0)
            icw_chain_frames<TRIG, 2, true, SIG>(a, P, s, t0 + hh, n2, in2, clip_l, clip_r, pk_l, pk_r, dv, tro_lane,
                                                 (size_t)hh * pq, pq);
        else
            icw_chain_frames<TRIG, 2, true>(a, P, s, t0 + hh, n2, in2, clip_l, clip_r, pk_l, pk_r, dv, tro_lane,
                                            (size_t)hh * pq, pq);
        if constexpr (B24) {
            const unsigned l0 = (unsigned)dv[0][0] & 0xffffffu, r0 = (unsigned)dv[0][1] & 0xffffffu;
            const unsigned l1 = (unsigned)dv[1][0] & 0xffffffu, r1 = (unsigned)dv[1][1] & 0xffffffu;
            w[hh / 2 * 3 + 0] = l0 | (r0 << 24);
            w[hh / 2 * 3 + 1] = (r0 >> 8) | (l1 << 16);
            w[hh / 2 * 3 + 2] = (l1 >> 16) | (r1 << 8);
        } else {
            w[hh] = ((unsigned)dv[0][0] & 0xffffu) | ((unsigned)dv[0][1] << 16);
            w[hh + 1] = ((unsigned)dv[1][0] & 0xffffu) | ((unsigned)dv[1][1] << 16);
        }
    }
}

/* ICW_FIR_OCC 5 (96 VGPRs) spills and ran 2.4x slower (profiles/r03_fir_swap_ab.jsonl) */
template <bool TRIG, bool TAB, int NC>
__global__ __launch_bounds__(256, ICW_FIR_OCC) void icw_fir_graph(IcwFirArgs f, IcwK2Args a)
{
    ICW_FIR_STAMP(0);
    ICW_FIR_STAMP(1);                                /* diagnostic build: 0 / 7 = 100 MHz clock, 1-6 shader clock */
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ unsigned red_clip[2][ICW_PK_SLOTS];
    __shared__ double red_pk[2][ICW_PK_SLOTS];
    /* workgroups in stream-fastest order (the grid is streams x tiles): the workgroups of one tile run
     * together, so its rotation-table rows come from the L2 for every stream, where tile-fastest order
     * swept the whole block's table once per stream (a 2^20-frame block's table is 32 MB: c2fir 37 HBM
     * bytes per frame against 9.4) */
    const int s = blockIdx.x;
    constexpr int nchc = NC;
    const int TF = 256 * ICW_FIR_R / nchc;
    const int tt = (blockIdx.y + f.tile0) * TF;
    const int M = f.M, c = M >> 1;
    const int sh = (8 - ((c - 1) & 7)) & 7;
    const int av = (c - 1 + sh) >> 3;
    const int nf = min(TF, f.T - tt);
    const int px = (icw_fir_phys(sh + M + TF + 24) + 2) & ~1;   /* doubles per staged channel (even) */
    double *lregs = lds + nchc * px + ((f.nt + 1) & ~1);
    icw_ctap *gs = (icw_ctap *)f.g;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ch = nchc == 2 ? lane >> 5 : 0;
    const int ll = nchc == 2 ? wv * 32 + (lane & 31) : threadIdx.x;   /* lane index within the channel */
    if (nchc == 2) icw_fir_stage<2>(f, s, 0, lds, px, tt, TF, sh, threadIdx.x, 256);
    else icw_fir_stage<1>(f, s, 0, lds, px, tt, TF, sh, threadIdx.x, 256);
    ICW_FIR_STAMP(2);
    __syncthreads();
    ICW_FIR_STAMP(3);
    double q[ICW_FIR_R], vi[ICW_FIR_R];
#if ICW_FIR_CUT >= 2
#pragma unroll
    for (int r = 0; r < ICW_FIR_R; ++r) q[r] = 0.0;
#else
    icw_fir_sums(lds + ch * px, gs, f.nt, ll, av, sh, c, q);
#endif
    const int ix = 8 * av + 1;                               /* logical index of x[tt - c] */
#pragma unroll
    for (int r = 0; r < ICW_FIR_R; ++r) vi[r] = lds[ch * px + icw_fir_phys(ICW_FIR_R * ll + r + ix)];
#if ICW_FIR_STAMPS
    if (threadIdx.x == 0 && q[0] + vi[0] == 1.2345e300) icw_fir_stp[0] = 1;     /* the sums before stamp 4 */
#endif
    ICW_FIR_STAMP(4);
#if ICW_FIR_CUT
    /* diagnostic build only (VALU accounting by phase): no graph, no render */
    {
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < ICW_FIR_R; ++r) acc += q[r] + vi[r];
        if (acc == 1.2345e300) a.out[threadIdx.x] = 1;
        return;
    }
#endif

    icw_cprog *P = icw_prog_c(a.prog);
    IcwRegFile Rf;
    Rf.base = lregs + threadIdx.x;
    for (int r = 0; r < P->n_persist; ++r) {
        const double *b = a.bus + ((size_t)s * ICW_N_INPUTS + P->persist_slot[r]) * 4;
        IcwLR v; v.lre = b[0]; v.lim = b[1]; v.rre = b[2]; v.rim = b[3];
        Rf.set(P->persist_reg[r], v);
    }
    const bool use_tab = TAB || (TRIG && a.trig_tab && a.n_frame[s] == a.n_frame[0]);
    unsigned clip_l = 0, clip_r = 0;
    double pk_l = 0.0, pk_r = 0.0;
    if (nchc == 2) {
        /* lane l (L) keeps frames 0-3 and gets R's values of them; lane l + 32 (R) frames 4-7.  Their
         * rendered frames are stored together: lane l's four at byte 32 ll, lane l + 32's at 32 ll + 16
         * (16-bit output), so one 16-byte store per lane covers the wave's 1 KB contiguously.  One
         * 4-byte store per frame instead put 2 of every 32 bytes in each store instruction, and the L2
         * wrote the partial sectors out 2.3x over (r03_c2fir_pmc.json before this change: WRITE_SIZE
         * 153 MB per launch against 67 MB of output). */
        const int h = ch ? 4 : 0;
        int dv[4][2];
        const int fr0 = ICW_FIR_R * ll + h;
        if (ICW_CHAIN4 && P->chain && (TAB || !TRIG) && !a.iq_out && a.do_render && !a.dith) {
            /* chain program, factors from the table (or none): the four frames op by op, two per
             * pass (four at once spill at 128 VGPRs), each pass's I / Q exchange just before it.
             * Frame tt + fr0 + hh + j (tt a multiple of 8, fr0 = 8 ll + h) sits in table row
             * (h + hh + j) q + tt / 8 + ll (icw_trig_index, q = trig_perm_q): a per-lane part and a
             * uniform one.  The last tile of a launch block keeps the clamped index (frames past
             * the block would point past the table). */
            const bool rowp = (TRIG || P->sig) && tt + TF <= f.T;
            const int sig = P->sig;
            const size_t pq = (size_t)a.trig_perm_q * a.trig_pitch;
            const uint32_t tro_lane = (uint32_t)(((size_t)h * a.trig_perm_q + (size_t)(tt >> 3) + ll) * a.trig_pitch);
#pragma unroll
            for (int hh = 0; hh < 4; hh += 2) {
                IcwLR in2[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int r = hh + j;
                    double xl = vi[r], xr = vi[r + 4], yl = q[r], yr = q[r + 4];
                    icw_swap32(xl, xr);
                    icw_swap32(yl, yr);
                    in2[j].lre = xl; in2[j].lim = yl; in2[j].rre = xr; in2[j].rim = yr;
                }
                int dv2[2][2];
                if (rowp)
                    icw_chain_frames_rowp<TRIG, 2>(a, P, sig, s, tt + fr0 + hh, min(2, max(nf - fr0 - hh, 0)), in2, clip_l,
                                                   clip_r, pk_l, pk_r, dv2, tro_lane, (size_t)hh * pq, pq);
                else
                    icw_chain_frames<TRIG, 2>(a, P, s, tt + fr0 + hh, min(2, max(nf - fr0 - hh, 0)), in2, clip_l, clip_r,
                                              pk_l, pk_r, dv2);
                dv[hh][0] = dv2[0][0]; dv[hh][1] = dv2[0][1];
                dv[hh + 1][0] = dv2[1][0]; dv[hh + 1][1] = dv2[1][1];
            }
        } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double xl = vi[r], xr = vi[r + 4], yl = q[r], yr = q[r + 4];
            icw_swap32(xl, xr);
            icw_swap32(yl, yr);
            const int fr = fr0 + r;
            dv[r][0] = dv[r][1] = 0;
            if (fr < nf) {
                IcwLR in;
                in.lre = xl; in.lim = yl; in.rre = xr; in.rim = yr;
                icw_frame_graph<TRIG, TAB, true>(a, P, Rf, s, tt + fr, in, use_tab, clip_l, clip_r, pk_l, pk_r, dv[r]);
            }
        }
        }
        if (a.do_render && !a.iq_out) {
            unsigned char *o = a.out + (size_t)s * a.out_stride;
            const int nv = min(4, nf - fr0);
            if (a.rk.is24) {
                /* 6 bytes per frame: 24 contiguous bytes per lane */
                unsigned char *p = o + (size_t)(tt + fr0) * 6;
                if (nv == 4 && !((uintptr_t)p & 7)) {
                    unsigned w[6];
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const unsigned l0 = (unsigned)dv[r][0] & 0xffffffu, r0 = (unsigned)dv[r][1] & 0xffffffu;
                        const unsigned l1 = (unsigned)dv[r + 1][0] & 0xffffffu, r1 = (unsigned)dv[r + 1][1] & 0xffffffu;
                        w[r / 2 * 3 + 0] = l0 | (r0 << 24);
                        w[r / 2 * 3 + 1] = (r0 >> 8) | (l1 << 16);
                        w[r / 2 * 3 + 2] = (l1 >> 16) | (r1 << 8);
                    }
                    uint2 *q2 = (uint2 *)p;
                    q2[0] = make_uint2(w[0], w[1]);
                    q2[1] = make_uint2(w[2], w[3]);
                    q2[2] = make_uint2(w[4], w[5]);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if (r >= nv) break;
                        unsigned char *b = p + r * 6;
                        const int vl = dv[r][0], vr = dv[r][1];
                        b[0] = (unsigned char)vl; b[1] = (unsigned char)(vl >> 8); b[2] = (unsigned char)(vl >> 16);
                        b[3] = (unsigned char)vr; b[4] = (unsigned char)(vr >> 8); b[5] = (unsigned char)(vr >> 16);
                    }
                }
            } else {
                unsigned pk[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) pk[r] = ((unsigned)dv[r][0] & 0xffffu) | ((unsigned)dv[r][1] << 16);
                unsigned *p = (unsigned *)(o + (size_t)(tt + fr0) * 4);
                if (nv == 4 && !((uintptr_t)p & 15)) {
                    *(uint4 *)p = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (r < nv) p[r] = pk[r];
                }
            }
        }
    } else if (ICW_CHAIN4 && P->chain && (TAB || !TRIG) && !a.iq_out && a.do_render && !a.dith) {
        /* mono input, chain program: the lane's 8 frames op by op, two at a time, and their 8
         * rendered frames stored together (32 / 48 contiguous bytes per lane) */
        const int fr0 = ICW_FIR_R * ll;
        const bool b24 = a.rk.is24;
        unsigned w[ICW_FIR_R / 2 * 3];               /* packed output: 16-bit frames in w[0..8) */
        /* table rows as in the stereo form: frame tt + 8 ll + hh + j at row (hh + j) q + tt / 8 + ll */
        const bool rowp = (TRIG || P->sig) && tt + TF <= f.T;
        const int sig = P->sig;
        const size_t pq = (size_t)a.trig_perm_q * a.trig_pitch;
        const uint32_t tro_lane = (uint32_t)(((size_t)(tt >> 3) + ll) * a.trig_pitch);
        /* the signature is chosen once for the lane's four passes (inside the pass loop every pass
         * carried all variants while the eight inputs stayed live, and the rotating kernel spilled) */
#define ICW_MONO(SIGV, RP)                                                                                    \
    do {                                                                                                      \
        if (b24) icw_mono_passes<TRIG, SIGV, RP, true>(a, P, s, tt + fr0, nf - fr0, vi, q, clip_l, clip_r, pk_l,  \
                                                       pk_r, w, tro_lane, pq);                                \
        else icw_mono_passes<TRIG, SIGV, RP, false>(a, P, s, tt + fr0, nf - fr0, vi, q, clip_l, clip_r, pk_l,    \
                                                    pk_r, w, tro_lane, pq);                                   \
    } while (0)
        if (!rowp) {
            ICW_MONO(0, false);
        } else if constexpr (TRIG) {
            switch (sig) {
            case ICW_SIG_M:
            case ICW_SIG_M | ICW_SIG_UNIT: ICW_MONO(ICW_SIG_M | ICW_SIG_UNIT, true); break;
            case ICW_SIG_SM: ICW_MONO(ICW_SIG_SM, true); break;
            case ICW_SIG_SM | ICW_SIG_UNIT: ICW_MONO(ICW_SIG_SM | ICW_SIG_UNIT, true); break;
            case ICW_SIG_PSXM: ICW_MONO(ICW_SIG_PSXM, true); break;
            case ICW_SIG_PSXM | ICW_SIG_UNIT: ICW_MONO(ICW_SIG_PSXM | ICW_SIG_UNIT, true); break;
            default: ICW_MONO(0, true); break;
            }
        } else {
            if (sig == ICW_SIG_M || sig == (ICW_SIG_M | ICW_SIG_UNIT)) ICW_MONO(ICW_SIG_M | ICW_SIG_UNIT, true);
            else ICW_MONO(0, true);
        }
#undef ICW_MONO
        unsigned char *o = a.out + (size_t)s * a.out_stride;
        const int nv = min(ICW_FIR_R, max(nf - fr0, 0));
        if (b24) {
            unsigned char *p = o + (size_t)(tt + fr0) * 6;
            if (nv == ICW_FIR_R && !((uintptr_t)p & 7)) {
                uint2 *q2 = (uint2 *)p;
#pragma unroll
                for (int i = 0; i < ICW_FIR_R / 2 * 3 / 2; ++i) q2[i] = make_uint2(w[2 * i], w[2 * i + 1]);
            } else {
                /* byte r of the packed run is byte r of the output */
#pragma unroll
                for (int i = 0; i < ICW_FIR_R * 6; ++i)
                    if (i < nv * 6) p[i] = (unsigned char)(w[i >> 2] >> (8 * (i & 3)));
            }
        } else {
            unsigned *p = (unsigned *)(o + (size_t)(tt + fr0) * 4);
            if (nv == ICW_FIR_R && !((uintptr_t)p & 15)) {
                *(uint4 *)p = make_uint4(w[0], w[1], w[2], w[3]);
                *(uint4 *)(p + 4) = make_uint4(w[4], w[5], w[6], w[7]);
            } else {
#pragma unroll
                for (int r = 0; r < ICW_FIR_R; ++r)
                    if (r < nv) p[r] = w[r];
            }
        }
    } else {
#pragma unroll 1
        for (int r = 0; r < ICW_FIR_R; ++r) {
            const int fr = ICW_FIR_R * ll + r;
            if (fr < nf) {
                IcwLR in;
                in.lre = in.rre = vi[r];
                in.lim = in.rim = q[r];
                icw_frame_graph<TRIG, TAB>(a, P, Rf, s, tt + fr, in, use_tab, clip_l, clip_r, pk_l, pk_r);
            }
        }
    }
    ICW_FIR_STAMP(5);
    if (a.do_render) icw_meters_wg(a, s, clip_l, clip_r, pk_l, pk_r, red_clip, red_pk);
    ICW_FIR_STAMP(6);
    ICW_FIR_STAMP(7);
}

/* KF2's signature form (icw_fir_sig): the tiles of a launch block before the one holding its last
 * frame, for a chain program of one of the specialised signatures (ICW_SIG_*), a ROUND / flat render
 * and no pre-render doubles -- the production form of the BASELINE FIR legs.  Every lane then takes
 * icw_chain_frames' render-only branch (full frames, no block-end bus write), so the kernel holds only
 * the staging, the sums, that branch (SIG and the output depth B24 at compile time) and the meters:
 * icw_fir_graph's register allocation is set by its generic paths (the per-frame graph, the exact
 * chain pass, the runtime signature switch), and their scalars spilled to VGPR lanes in the hot
 * phases.  icw_launch_fir_graph runs the last tile of each stream through icw_fir_graph (tile0).
 * Same staging, sums and render arithmetic, so the bytes and meters are icw_fir_graph's. */
/* Occupancy of the signature form: without the generic paths it fits 114 VGPRs at 4 workgroups per CU,
 * no scratch.  It also fits 96 (5 per CU) with 4-tap register blocks in the sums, and the mono form 80
 * (6 per CU): measured the same within the box noise (c2fir -1 / +1.7 %, c4fir +0.5 / +0.8 %, c3fir
 * -1.9 / +0.2 %, profiles/r06_fir_sig_ab.txt) with 24 more VALU and 48 more LDS instructions per wave,
 * so the FP64 pipe, not latency, bounds it at 4. */
#ifndef ICW_FIR_SIG_OCC
#define ICW_FIR_SIG_OCC 4
#endif
#ifndef ICW_FIR_SIG_OCC1
#define ICW_FIR_SIG_OCC1 4                           /* the mono form */
#endif
#ifndef ICW_FIR_SIG_NTAP
#define ICW_FIR_SIG_NTAP ICW_FIR_NTAP
#endif
template <int SIG, int NC, bool B24>
__global__ __launch_bounds__(256, NC == 2 ? ICW_FIR_SIG_OCC : ICW_FIR_SIG_OCC1) void icw_fir_sig(IcwFirArgs f, IcwK2Args a)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ unsigned red_clip[2][ICW_PK_SLOTS];
    __shared__ double red_pk[2][ICW_PK_SLOTS];
    constexpr bool TRIG = (SIG & ~ICW_SIG_UNIT) != ICW_SIG_M;
    constexpr int TF = 256 * ICW_FIR_R / NC;
    const int s = blockIdx.x;
    const int tt = blockIdx.y * TF;
    const int M = f.M, c = M >> 1;
    const int sh = (8 - ((c - 1) & 7)) & 7;
    const int av = (c - 1 + sh) >> 3;
    const int px = (icw_fir_phys(sh + M + TF + 24) + 2) & ~1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ch = NC == 2 ? lane >> 5 : 0;
    const int ll = NC == 2 ? wv * 32 + (lane & 31) : threadIdx.x;
    icw_fir_stage<NC>(f, s, 0, lds, px, tt, TF, sh, threadIdx.x, 256);
    __syncthreads();
    double q[ICW_FIR_R], vi[ICW_FIR_R];
    icw_fir_sums<ICW_FIR_SIG_NTAP>(lds + ch * px, (icw_ctap *)f.g, f.nt, ll, av, sh, c, q);
    const int ix = 8 * av + 1;
#pragma unroll
    for (int r = 0; r < ICW_FIR_R; ++r) vi[r] = lds[ch * px + icw_fir_phys(ICW_FIR_R * ll + r + ix)];
    icw_cprog *P = icw_prog_c(a.prog);
    unsigned clip_l = 0, clip_r = 0;
    double pk_l = 0.0, pk_r = 0.0;
    const size_t pq = (size_t)a.trig_perm_q * a.trig_pitch;
    unsigned char *o = a.out + (size_t)s * a.out_stride;
    if constexpr (NC == 2) {
        /* lane l (L) frames 0-3 of its eight with R's values swapped in, lane l + 32 frames 4-7 */
        const int h = ch ? 4 : 0;
        const int fr0 = ICW_FIR_R * ll + h;
        const uint32_t tro_lane = (uint32_t)(((size_t)h * a.trig_perm_q + (size_t)(tt >> 3) + ll) * a.trig_pitch);
        int dv[4][2];
#pragma unroll
        for (int hh = 0; hh < 4; hh += 2) {
            IcwLR in2[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = hh + j;
                double xl = vi[r], xr = vi[r + 4], yl = q[r], yr = q[r + 4];
                icw_swap32(xl, xr);
                icw_swap32(yl, yr);
                in2[j].lre = xl; in2[j].lim = yl; in2[j].rre = xr; in2[j].rim = yr;
            }
            int dv2[2][2];
            icw_sig_fast<TRIG, 2, SIG>(a, P, in2, clip_l, clip_r, pk_l, pk_r, dv2, tro_lane, (size_t)hh * pq, pq);
            dv[hh][0] = dv2[0][0]; dv[hh][1] = dv2[0][1];
            dv[hh + 1][0] = dv2[1][0]; dv[hh + 1][1] = dv2[1][1];
        }
        if constexpr (B24) {
            unsigned char *p = o + (size_t)(tt + fr0) * 6;
            unsigned w[6];
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
                const unsigned l0 = (unsigned)dv[r][0] & 0xffffffu, r0 = (unsigned)dv[r][1] & 0xffffffu;
                const unsigned l1 = (unsigned)dv[r + 1][0] & 0xffffffu, r1 = (unsigned)dv[r + 1][1] & 0xffffffu;
                w[r / 2 * 3 + 0] = l0 | (r0 << 24);
                w[r / 2 * 3 + 1] = (r0 >> 8) | (l1 << 16);
                w[r / 2 * 3 + 2] = (l1 >> 16) | (r1 << 8);
            }
            if (!((uintptr_t)p & 7)) {
                uint2 *q2 = (uint2 *)p;
                q2[0] = make_uint2(w[0], w[1]);
                q2[1] = make_uint2(w[2], w[3]);
                q2[2] = make_uint2(w[4], w[5]);
            } else {
#pragma unroll
                for (int i = 0; i < 24; ++i) p[i] = (unsigned char)(w[i >> 2] >> (8 * (i & 3)));
            }
        } else {
            unsigned pk[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) pk[r] = ((unsigned)dv[r][0] & 0xffffu) | ((unsigned)dv[r][1] << 16);
            unsigned *p = (unsigned *)(o + (size_t)(tt + fr0) * 4);
            if (!((uintptr_t)p & 15)) {
                *(uint4 *)p = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) p[r] = pk[r];
            }
        }
    } else {
        /* mono: the lane's 8 frames two at a time, packed as icw_mono_passes does */
        const int fr0 = ICW_FIR_R * ll;
        const uint32_t tro_lane = (uint32_t)(((size_t)(tt >> 3) + ll) * a.trig_pitch);
        int dl[ICW_FIR_R], dr[ICW_FIR_R];
        if (!TRIG && f.lr_same) {
            /* both channels run the same arithmetic on the same inputs (mono input, a Master whose two
             * gains are the same double: icw_launch_fir_graph's lr_same), so a pass takes two frames in
             * its L / R slots and each result serves both channels: half the graph and render */
#pragma unroll
            for (int hh = 0; hh < ICW_FIR_R; hh += 4) {
                IcwLR in2[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    in2[r].lre = vi[hh + 2 * r];
                    in2[r].lim = q[hh + 2 * r];
                    in2[r].rre = vi[hh + 2 * r + 1];
                    in2[r].rim = q[hh + 2 * r + 1];
                }
                int dv[2][2];
                icw_sig_fast<TRIG, 2, SIG>(a, P, in2, clip_l, clip_r, pk_l, pk_r, dv, tro_lane, 0, pq);
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int c = 0; c < 2; ++c) dl[hh + 2 * r + c] = dr[hh + 2 * r + c] = dv[r][c];
            }
            /* the slots held frames: every frame's clips and peak count for both channels */
            clip_l = clip_r = clip_l + clip_r;
            pk_l = pk_r = icw_vmax(pk_l, pk_r);
        } else {
#pragma unroll
            for (int hh = 0; hh < ICW_FIR_R; hh += 2) {
                IcwLR in2[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    in2[r].lre = in2[r].rre = vi[hh + r];
                    in2[r].lim = in2[r].rim = q[hh + r];
                }
                int dv[2][2];
                icw_sig_fast<TRIG, 2, SIG>(a, P, in2, clip_l, clip_r, pk_l, pk_r, dv, tro_lane, (size_t)hh * pq, pq);
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    dl[hh + r] = dv[r][0];
                    dr[hh + r] = dv[r][1];
                }
            }
        }
        unsigned w[ICW_FIR_R / 2 * 3];
#pragma unroll
        for (int hh = 0; hh < ICW_FIR_R; hh += 2) {
            if constexpr (B24) {
                const unsigned l0 = (unsigned)dl[hh] & 0xffffffu, r0 = (unsigned)dr[hh] & 0xffffffu;
                const unsigned l1 = (unsigned)dl[hh + 1] & 0xffffffu, r1 = (unsigned)dr[hh + 1] & 0xffffffu;
                w[hh / 2 * 3 + 0] = l0 | (r0 << 24);
                w[hh / 2 * 3 + 1] = (r0 >> 8) | (l1 << 16);
                w[hh / 2 * 3 + 2] = (l1 >> 16) | (r1 << 8);
            } else {
                w[hh] = ((unsigned)dl[hh] & 0xffffu) | ((unsigned)dr[hh] << 16);
                w[hh + 1] = ((unsigned)dl[hh + 1] & 0xffffu) | ((unsigned)dr[hh + 1] << 16);
            }
        }
        if constexpr (B24) {
            unsigned char *p = o + (size_t)(tt + fr0) * 6;
            if (!((uintptr_t)p & 7)) {
                uint2 *q2 = (uint2 *)p;
#pragma unroll
                for (int i = 0; i < ICW_FIR_R / 2 * 3 / 2; ++i) q2[i] = make_uint2(w[2 * i], w[2 * i + 1]);
            } else {
#pragma unroll
                for (int i = 0; i < ICW_FIR_R * 6; ++i) p[i] = (unsigned char)(w[i >> 2] >> (8 * (i & 3)));
            }
        } else {
            unsigned *p = (unsigned *)(o + (size_t)(tt + fr0) * 4);
            if (!((uintptr_t)p & 15)) {
                *(uint4 *)p = make_uint4(w[0], w[1], w[2], w[3]);
                *(uint4 *)(p + 4) = make_uint4(w[4], w[5], w[6], w[7]);
            } else {
#pragma unroll
                for (int r = 0; r < ICW_FIR_R; ++r) p[r] = w[r];
            }
        }
    }
    icw_meters_wg(a, s, clip_l, clip_r, pk_l, pk_r, red_clip, red_pk);
}

/* Per-frame rotation table: the Shift / PM factors of frame t depend only on the modulator frame
 * counter, which all streams of a batch share while they are in step (same call-start counter).
 * One thread per frame evaluates each active channel's factor once (icw_trig, the same code as
 * the inline path); K2 reads the row instead of running fmod / sin / sincos per stream. */
__device__ __forceinline__ void icw_trig_row(const IcwTrigArgs &a, int t)
{
    icw_cprog *P = icw_prog_c(a.prog);
    const double omega = icw_omega(a.n_frame[0], a.t0 + t, a.scaled, a.ssr, a.sample_rate);
    double *row = a.tab + icw_trig_index(t, a.perm_q) * a.trig_pitch;
    for (int oi = 0; oi < P->n_ops; ++oi) {
        icw_cop &op = P->ops[oi];
        if (op.mode != ICW_MODE_SHIFT && op.mode != ICW_MODE_PM) continue;
        for (int c = 0; c < 2; ++c) {
            if (!op.act[c]) continue;
            double cs, sn;
            icw_trig(op, c, omega, cs, sn);
            row[op.tslot[c] * 2] = cs;
            row[op.tslot[c] * 2 + 1] = sn;
        }
    }
}

__global__ __launch_bounds__(256) void icw_trig_table(IcwTrigArgs a)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t < a.T) icw_trig_row(a, t);
}

/* ------------------------------------------------------- serial graph kernel (K4) ------ */
/* Bus form of the DSP list, for lists whose nodes read a slot before it is written in the frame
 * (a one-frame delay -- feedback loops included): the reference's own per-frame semantics
 * (adv_modulator.c:636-751) with the 27-slot bus of the stream held in LDS, one lane per stream,
 * frames in order.  `in` comes from the output kernel (Hilbert or complex input), lOut/rOut go
 * to the serial render kernel. */
__global__ __launch_bounds__(64) void icw_graph_serial(IcwK4Args a)
{
    __shared__ double bus[ICW_N_INPUTS * 4][64];
    const int lane = threadIdx.x;
    const int s = blockIdx.x * 64 + lane;
    if (s >= a.n_streams) return;
    double *gb = a.bus + (size_t)s * ICW_N_INPUTS * 4;
    for (int k = 0; k < ICW_N_INPUTS * 4; ++k) bus[k][lane] = gb[k];
    icw_cprog *P = icw_prog_c(a.prog);
    const unsigned long long n0 = a.n_frame[s];
    const double *iq = a.iq + (size_t)s * a.T * 4;
    double *pre = a.pre + (size_t)s * a.pre_stride;
    for (int t = 0; t < a.T; ++t) {
        const double omega = P->needs_omega ? icw_omega(n0, a.t0 + t, a.scaled, a.ssr, a.sample_rate) : 0.0;
        bus[0][lane] = iq[(size_t)t * 4 + 0];
        bus[1][lane] = iq[(size_t)t * 4 + 1];
        bus[2][lane] = iq[(size_t)t * 4 + 2];
        bus[3][lane] = iq[(size_t)t * 4 + 3];
        double lOut = 0.0, rOut = 0.0;
        for (int oi = 0; oi < P->n_ops; ++oi) {
            icw_cop &op = P->ops[oi];
            IcwLR d;
            if (P->bypass) {
                d.lre = bus[0][lane]; d.lim = bus[1][lane]; d.rre = bus[2][lane]; d.rim = bus[3][lane];
            } else {
                d.lre = d.lim = d.rre = d.rim = 0.0;
                const uint32_t m = op.in_mask;
                for (int k = 0; k < ICW_N_INPUTS; ++k) {
                    if (!((m >> k) & 1u)) continue;
                    d.lre += bus[k * 4 + 0][lane]; d.lim += bus[k * 4 + 1][lane];
                    d.rre += bus[k * 4 + 2][lane]; d.rim += bus[k * 4 + 3][lane];
                }
            }
            IcwLR o;
            if (icw_exec_op(op, d, omega, o, lOut, rOut)) {
                const int q = op.out_slot * 4;
                bus[q + 0][lane] = o.lre; bus[q + 1][lane] = o.lim; bus[q + 2][lane] = o.rre; bus[q + 3][lane] = o.rim;
            }
        }
        pre[(size_t)t * 2] = lOut;
        pre[(size_t)t * 2 + 1] = rOut;
    }
    for (int k = 0; k < ICW_N_INPUTS * 4; ++k) gb[k] = bus[k][lane];
}

/* Call-end bookkeeping: the reader position, the Hilbert phases (not for complex input -- the
 * converters were not called) and the modulator frame counter advance by the call's frames. */
__device__ __forceinline__ void icw_advance_stream(const IcwAdvArgs &a, int s)
{
    a.pos[s] += a.n;
    if (!a.cw) {
        a.hq_phase[s * 2 + 0] = (a.hq_phase[s * 2 + 0] + (unsigned)a.n) & 3u;
        a.hq_phase[s * 2 + 1] = (a.hq_phase[s * 2 + 1] + (unsigned)a.n) & 3u;
    }
    const unsigned long long n0 = a.n_frame[s];
    a.n_frame[s] = a.scaled ? (n0 + (unsigned long long)a.n) % a.ssr : n0 + (unsigned long long)a.n;
    if (s == 0 && a.err_copy) *a.err_copy = *a.err;
}

__global__ __launch_bounds__(64) void icw_advance(IcwAdvArgs a)
{
    const int s = blockIdx.x * 64 + threadIdx.x;
    if (s < a.n_streams) icw_advance_stream(a, s);
}

/* K5's overlapped form (a.ovl, the launcher checks that the rows fit in LDS): after K0, waves 0-1
 * run the recurrence with its w rows in LDS and publish how many frames are final
 * (icw_iir_row_body<N, true>); waves 2-3 take the output phase frame by frame behind it -- wave w
 * the 64-frame groups g = w, w + 2, ..: the group's rotation factors (no dependence on the
 * recurrence), then, once its rows are final, its outputs.  The output phase's ~20 us (576 frames)
 * but its last group hide behind the recurrence.  Per frame the same code as K2 (icw_output_frame),
 * so the results are the pipeline's bit for bit. */
__device__ __forceinline__ void icw_s1_stamp(unsigned long long *stp, int k)
{
    if (stp && threadIdx.x == 0) {
        stp[2 * k] = __builtin_amdgcn_s_memtime();
        stp[2 * k + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

template <int N, bool TRIG>
__device__ __forceinline__ void icw_s1_overlapped(const IcwS1Args &a, double *lregs)
{
    auto stamp = [&a](int k) { icw_s1_stamp(a.stamps, k); };
    __shared__ double coef[40];
    __shared__ unsigned red_clip[2][ICW_PK_SLOTS], red_sn[4][ICW_K2_TILE / 64];
    __shared__ double red_pk[2][ICW_PK_SLOTS];
    const IcwK2Args &a2 = a.k2;
    const int tid = threadIdx.x, T = a2.T;
    double *rows = lregs + a.rows_off;
    int *prog = (int *)(rows + (size_t)4 * a.lpitch);
    if (tid < 2) prog[tid] = 0;
    if (tid < 40) coef[tid] = tid < 20 ? a2.pc[tid] : a2.pd[tid - 20];
    /* mono input with bit-identical converters in phase (K2's `dup`): the flags as the block starts,
     * read before the recurrence updates them */
    const bool dup = a2.nch == 1 && a.k1.lr_equal[0] && a.k1.lr_equal[1] && a2.hq_phase[0] == a2.hq_phase[1];
    __syncthreads();
    stamp(1);
    unsigned clip_l = 0, clip_r = 0;
    double pk_l = 0.0, pk_r = 0.0;
    unsigned sn[4] = {0u, 0u, 0u, 0u};
    const bool count_sn = a2.sncnt != nullptr;
    if (tid < 128) {
        icw_iir_row_body<N, true>(a.k1, tid, rows, a.lpitch, prog);
    } else {
        const int k = tid - 128, w2 = k >> 6, lane = k & 63;
        icw_cprog *P = icw_prog_c(a2.prog);
        IcwRegFile R;
        R.base = lregs + tid;
        for (int r = 0; r < P->n_persist; ++r) {
            const double *b = a2.bus + (size_t)P->persist_slot[r] * 4;
            IcwLR v; v.lre = b[0]; v.lim = b[1]; v.rre = b[2]; v.rim = b[3];
            R.set(P->persist_reg[r], v);
        }
        const bool use_tab = TRIG && a2.trig_tab;
        IcwFes fes[2] = {};
        const volatile __attribute__((address_space(3))) int *vp = (__attribute__((address_space(3))) int *)prog;
        for (int g = w2; g * 64 < T; g += 2) {
            const int t = g * 64 + lane;
            const int need = min(g * 64 + 64, T);
            if (a.has_trig && t < T) icw_trig_row(a.trig, t);
            /* bounded: a recurrence that never published (never in a healthy run) flags the call's
             * error and the wave goes on, so the grid drains */
            for (unsigned spin = 0; min(vp[0], vp[1]) < need; ++spin) {
                if (spin >= (1u << 24)) {
                    if (lane == 0 && a.k1.err) atomicOr(a.k1.err, 1);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            asm volatile("" ::: "memory");
            if (t < T) {
                const size_t lp = a.lpitch;
                const double *const w[4] = {rows + t, rows + lp + t, rows + 2 * lp + t, rows + 3 * lp + t};
                icw_output_frame<N, true, TRIG, false>(a2, P, R, 0, t, w, dup, coef + a2.zero * g, fes, count_sn,
                                                       sn, use_tab, clip_l, clip_r, pk_l, pk_r);
            }
        }
    }
    __syncthreads();
    stamp(2);
    if (count_sn) icw_sn_wg(a2, 0, sn, dup ? 2 : 4, red_sn);
    icw_meters_wg(a2, 0, clip_l, clip_r, pk_l, pk_r, red_clip, red_pk);
    stamp(3);
}

/* K5 icw_stream1: one stream's whole launch block in ONE workgroup -- the per-call form of the
 * drop-in boundary (icw_amod_process_samples: playback.c:619 renders 576-frame blocks, NS_PERTIME,
 * in_cwave.h:133).  The pipeline's four launches (K0, K1r, K2, icw_advance) and their ~6 us gaps
 * become phases of one kernel, separated by workgroup barriers; each phase runs the same device
 * code as its kernel, so the results are the pipeline's bit for bit:
 *   1. all 256 threads: unpack + fade + quadrature mix of the block (K0) into the xd rows;
 *   2. waves 0-1: the row-broadcast recurrence (K1r: filter f = wave, one 16-lane row per channel);
 *   3. all threads: output sums, un-mix, DSP list, ROUND render, meters (K2, a.tpw tiles of 256);
 *   4. thread 0: reader position, Hilbert phases, frame counter (icw_advance).
 * The stores of one phase reach the next one's loads through the barrier's workgroup-scope
 * release / acquire (one CU, one vector L1). */
template <int N, bool TRIG>
__global__ __launch_bounds__(ICW_K2_TILE) void icw_stream1(IcwS1Args a)
{
    extern __shared__ __attribute__((aligned(16))) double lregs[];   /* K2's register file */
    /* diagnostic build only (ICW_S1_STAMPS, tools/s1_phases.py): shader-clock and 100 MHz stamps at
     * the phase boundaries */
    auto stamp = [&a](int k) { icw_s1_stamp(a.stamps, k); };
    stamp(0);
    /* K0: all the block's loads first (the zero-copy input is read across PCIe: one round trip per
     * pass instead of one per frame -- a frame's stores could alias the next frame's loads), then the
     * fades and the stores */
    const IcwK0Args &a0 = a.k0;
    const bool mono = a0.nch == 1;
    icw_fmt_dispatch(a0.fmt, (uintptr_t)a0.in | (uintptr_t)a0.fsz, [&](auto fc, auto ac) {
        constexpr int F = decltype(fc)::value;
        constexpr bool AL = decltype(ac)::value != 0;
        for (int t0 = 0; t0 < a0.T; t0 += 4 * ICW_K2_TILE) {
            double v[4][2];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int t = t0 + k * ICW_K2_TILE + (int)threadIdx.x;
                if (t < a0.T) {
                    const unsigned char *fp = a0.in + (size_t)t * a0.fsz;
                    v[k][0] = icw_unpack_f<F, AL>(fp);
                    v[k][1] = mono ? v[k][0] : icw_unpack_f<F, AL>(fp + a0.csz);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int t = t0 + k * ICW_K2_TILE + (int)threadIdx.x;
                if (t < a0.T) icw_store_frame(a0, t, 0, v[k]);
            }
        }
    });
    if (a.ovl) {
        icw_s1_overlapped<N, TRIG>(a, lregs);
    } else {
        __syncthreads();
        stamp(1);
        /* waves 0-1 (SIMDs 0, 1): the recurrence; waves 2-3 (SIMDs 2, 3), idle otherwise: the block's
         * Shift / PM rotation factors, which depend only on the frame counter, for the output phase */
        if (threadIdx.x < 128) icw_iir_row_body<N>(a.k1, threadIdx.x);
        else if (a.has_trig)
            for (int t = (int)threadIdx.x - 128; t < a.trig.T; t += 128) icw_trig_row(a.trig, t);
        __syncthreads();
        stamp(2);
        icw_output_body<N, true, TRIG>(a.k2, 0, 0, lregs);
        __syncthreads();
        stamp(3);
    }
    if (a.adv.done) {
        /* every wave waits for its own zero-copy output stores to be acknowledged before the barrier
         * (a workgroup-scope release need not wait on vmcnt outside threadgroup-split mode), so thread
         * 0's system-scope fence below covers the whole workgroup's output, not only wave 0's */
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        icw_advance_stream(a.adv, 0);
        if (a.adv.done) {
            /* write the output and the error flag back to host memory, then the call's sequence
             * number the host polls for */
            __threadfence_system();
            __hip_atomic_store(a.adv.done, a.adv.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

/* ------------------------------------------------------ serial render kernel (K3) ------ */
/* sound_render_value (sound_render.c:691-809) for the dithered / noise-shaped renders, whose
 * state (MT19937 position, sloped-TPDF memory, noise-shaper feedback) is serial per channel:
 * one lane per channel, the channel's MT19937 state held in LDS ([624][64] words, 156 KB: the
 * twist of mt_jrnd.c:99-124 runs in place per lane), shaper history in registers as shift
 * registers (age 0 = newest, identical sums to the ring of ns_fir/ns_iir, sound_render.c:403-489). */
__device__ __forceinline__ uint32_t icw_mt_twist_word(uint32_t u, uint32_t v)
{
    const uint32_t y = (u & 0x80000000u) | (v & 0x7fffffffu);
    return (y >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
}

__device__ __forceinline__ void icw_mt_regen(uint32_t *mt, int lane)
{
    /* in-place generation of the next 624 words (mtrnd_gen_ui32, mt_jrnd.c:105-120), 8 words per
     * batch: a batch's LDS reads are independent of its writes (they read words >= i and, in the
     * second part, words written >= 220 positions earlier), so its loads issue back to back */
    uint32_t *m = mt + lane;
    int i = 0;
    for (; i + 8 <= 227; i += 8) {
        uint32_t u[9], f[8];
#pragma unroll
        for (int j = 0; j < 9; ++j) u[j] = m[(i + j) * 64];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = m[(i + j + 397) * 64];
#pragma unroll
        for (int j = 0; j < 8; ++j) m[(i + j) * 64] = f[j] ^ icw_mt_twist_word(u[j], u[j + 1]);
    }
    for (; i < 227; ++i) m[i * 64] = m[(i + 397) * 64] ^ icw_mt_twist_word(m[i * 64], m[(i + 1) * 64]);
    for (; i + 8 <= 623; i += 8) {
        uint32_t u[9], f[8];
#pragma unroll
        for (int j = 0; j < 9; ++j) u[j] = m[(i + j) * 64];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = m[(i + j - 227) * 64];
#pragma unroll
        for (int j = 0; j < 8; ++j) m[(i + j) * 64] = f[j] ^ icw_mt_twist_word(u[j], u[j + 1]);
    }
    for (; i < 623; ++i) m[i * 64] = m[(i - 227) * 64] ^ icw_mt_twist_word(m[i * 64], m[(i + 1) * 64]);
    m[623 * 64] = m[396 * 64] ^ icw_mt_twist_word(m[623 * 64], m[0]);
}

__device__ __forceinline__ uint32_t icw_mt_temper(uint32_t y)
{
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t icw_mt_u32(uint32_t *mt, int lane, int &idx)
{
    if (idx >= 624) {
        icw_mt_regen(mt, lane);
        idx = 0;
    }
    const uint32_t y = mt[idx * 64 + lane];
    ++idx;
    return icw_mt_temper(y);
}

/* mtrnd_gen_dsopen (mt_jrnd.c:218-256): (-1, 1) with 53-bit resolution, +-1 rejected */
__device__ __forceinline__ double icw_mt_dsopen(uint32_t *mt, int lane, int &idx)
{
    double r;
    do {
        const uint32_t a = icw_mt_u32(mt, lane, idx) >> 5;
        const uint32_t b = icw_mt_u32(mt, lane, idx) >> 6;
        r = ((a * 67108864.0 + b) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
    } while (-1.0 == r || 1.0 == r);
    return r;
}

#define ICW_SQRT6 (2.4494897427831780981972840747059)

/* Dither generation (K3a): the random term rnd * dth_mul of sound_render_value
 * (sound_render.c:711-756) for every sample of the block.  It depends only on the channel's MT19937
 * state and the sloped-TPDF memory, never on the audio, so it runs on its own stream ahead of /
 * beside the Hilbert and output kernels; one lane per render channel, MT words in LDS. */
/* dsopen from two tempered words (mtrnd_gen_dsopen, mt_jrnd.c:218-256) without the rejection */
__device__ __forceinline__ double icw_dsopen2(uint32_t ua, uint32_t ub)
{
    const uint32_t a = ua >> 5, b = ub >> 6;
    return ((a * 67108864.0 + b) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
}

template <int RT>
struct IcwDith {
    static constexpr int W = RT == ICW_RENDER_GAUSS ? 24 : (RT == ICW_RENDER_TPDF ? 4 : 2);   /* words/sample */
    static constexpr int C = RT == ICW_RENDER_GAUSS ? 2 : (RT == ICW_RENDER_TPDF ? 8 : 16);  /* samples/chunk */
};

/* the dither of one sample from its words (no rejection among them) */
template <int RT>
__device__ __forceinline__ double icw_dith_from_words(const uint32_t *u, double &prev_rnd)
{
    double rnd, tr;
    if (RT == ICW_RENDER_RPDF) {
        rnd = icw_dsopen2(u[0], u[1]) / ICW_SQRT2;
    } else if (RT == ICW_RENDER_TPDF) {
        rnd = icw_dsopen2(u[0], u[1]);
        rnd += icw_dsopen2(u[2], u[3]);
        rnd /= 2.0;
    } else if (RT == ICW_RENDER_STPDF) {
        rnd = ((tr = icw_dsopen2(u[0], u[1])) - prev_rnd) / 2.0;
        prev_rnd = tr;
    } else {
        rnd = icw_dsopen2(u[0], u[1]);
#pragma unroll
        for (int i = 1; i < 12; ++i) rnd += icw_dsopen2(u[2 * i], u[2 * i + 1]);
        rnd /= (2.0 * ICW_SQRT6);
    }
    return rnd;
}

/* the reference's sequential form, rejection and twist included */
template <int RT>
__device__ __forceinline__ double icw_dith_slow(uint32_t *mt, int lane, int &idx, double &prev_rnd)
{
    double rnd, tr;
    if (RT == ICW_RENDER_RPDF) {
        rnd = icw_mt_dsopen(mt, lane, idx) / ICW_SQRT2;
    } else if (RT == ICW_RENDER_TPDF) {
        rnd = icw_mt_dsopen(mt, lane, idx);
        rnd += icw_mt_dsopen(mt, lane, idx);
        rnd /= 2.0;
    } else if (RT == ICW_RENDER_STPDF) {
        rnd = ((tr = icw_mt_dsopen(mt, lane, idx)) - prev_rnd) / 2.0;
        prev_rnd = tr;
    } else {
        rnd = icw_mt_dsopen(mt, lane, idx);
        for (int i = 1; i < 12; ++i) rnd += icw_mt_dsopen(mt, lane, idx);
        rnd /= (2.0 * ICW_SQRT6);
    }
    return rnd;
}

/* Dither generation (K3a): the random term rnd * dth_mul of sound_render_value
 * (sound_render.c:711-756) for every sample of the block.  It depends only on the channel's MT19937
 * state and the sloped-TPDF memory, never on the audio, so it runs on its own stream beside the
 * Hilbert and output kernels; one lane per render channel, MT words in LDS.  Fast path: a chunk of
 * C samples whose W*C words are all left before the next twist is read as one batch of
 * independent LDS loads; a chunk that would hit a rejected draw (probability ~2^-53 per draw) or
 * the twist runs through the sequential form instead. */
template <int RT>
__global__ __launch_bounds__(64) void icw_dither_gen(IcwK3Args a)
{
    using D = IcwDith<RT>;
    constexpr int NW = D::W * D::C;
    __shared__ uint32_t mt[624 * 64];
    const int lane = threadIdx.x;
    const int g0 = blockIdx.x * 64 + lane;
    const bool valid = g0 < a.n_gen;
    const int g = valid ? g0 : a.n_gen - 1;
    for (int i = 0; i < 624; ++i) mt[i * 64 + lane] = a.mt[(size_t)i * a.mt_pitch + g];
    int idx = a.mt_idx[g];
    double *rs = a.rs + (size_t)g * ICW_RSTATE;
    double prev_rnd = rs[0];
    const double dth_mul = a.rk.dth_mul;
    /* time-major [t][dith_pitch]: one store per sample is coalesced; generator-major: a lane's own run */
    double *dd = a.dith_gm ? a.dith + (size_t)g * a.dith_pitch : a.dith + g;
    const size_t dp = a.dith_gm ? 1 : a.dith_pitch;
    const int T = a.T;
    int t = 0;
    while (t < T) {
        if (t + D::C <= T && idx + NW <= 624) {
            uint32_t u[NW];
#pragma unroll
            for (int j = 0; j < NW; ++j) u[j] = icw_mt_temper(mt[(idx + j) * 64 + lane]);
            bool rej = false;
#pragma unroll
            for (int j = 0; j < NW; j += 2) rej |= ((u[j] >> 5) == 0u) && ((u[j + 1] >> 6) == 0u);
            if (!rej) {
                double pr = prev_rnd;
#pragma unroll
                for (int c = 0; c < D::C; ++c) {
                    const double rnd = icw_dith_from_words<RT>(u + c * D::W, pr);
                    if (valid) dd[(size_t)(t + c) * dp] = rnd * dth_mul;
                }
                prev_rnd = pr;
                idx += NW;
                t += D::C;
                continue;
            }
        }
        /* one sample the sequential way (twists, rejections) */
        const double rnd = icw_dith_slow<RT>(mt, lane, idx, prev_rnd);
        if (valid) dd[(size_t)t * dp] = rnd * dth_mul;
        ++t;
    }
    if (!valid) return;
    for (int i = 0; i < 624; ++i) a.mt[(size_t)i * a.mt_pitch + g] = mt[i * 64 + lane];
    a.mt_idx[g] = idx;
    rs[0] = prev_rnd;
}

/* Cooperative dither generation (K3a): one wave per render channel.  The random term of
 * sound_render_value (sound_render.c:711-756) depends only on the channel's MT19937 stream, so the
 * stream is produced 624 words at a time by the whole wave:
 *   twist     the 624-word regeneration (mt_jrnd.c:105-120) in three dependency phases
 *             ([0,227) from old words; [227,454) and [454,623) from words new by then; then 623);
 *   window    words idx..623 tempered in parallel; word pairs -> dsopen values (mt_jrnd.c:218-256);
 *             a rejected pair (+-1.0) yields no value -- the reference just draws the next pair --
 *             so accepted values are compacted with a ballot prefix count;
 *   samples   V consecutive values per sample (RPDF 1, TPDF 2, STPDF 1 + the previous, GAUSS 12),
 *             one lane per sample.
 * A pair or a sample may straddle windows (one carried word, < V carried values).  The block ends
 * exactly after its last sample, so idx is where the reference's would be. */
__device__ __forceinline__ void icw_coop_twist(uint32_t *mt, int lane)
{
    uint32_t r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = lane + 64 * q;
        if (i < 227) r[q] = mt[i + 397] ^ icw_mt_twist_word(mt[i], mt[i + 1]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = lane + 64 * q;
        if (i < 227) mt[i] = r[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = 227 + lane + 64 * q;
        if (i < 454) r[q] = mt[i - 227] ^ icw_mt_twist_word(mt[i], mt[i + 1]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = 227 + lane + 64 * q;
        if (i < 454) mt[i] = r[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int i = 454 + lane + 64 * q;
        if (i < 623) r[q] = mt[i - 227] ^ icw_mt_twist_word(mt[i], mt[i + 1]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int i = 454 + lane + 64 * q;
        if (i < 623) mt[i] = r[q];
    }
    __syncthreads();
    if (lane == 0) mt[623] = mt[396] ^ icw_mt_twist_word(mt[623], mt[0]);
    __syncthreads();
}

/* the generator g's samples of the block (or chunk) the sequential way: from the state in a.mt /
 * a.mt_idx / rs[0], or (bk) from the chunk's backup K3t made -- K3f's redo of a channel whose words
 * held a rejected pair */
template <int RT>
__device__ __forceinline__ void icw_dither_coop_body(const IcwK3Args &a, int g, const uint32_t *bk)
{
    constexpr int V = RT == ICW_RENDER_GAUSS ? 12 : (RT == ICW_RENDER_TPDF ? 2 : 1);
    __shared__ uint32_t mt[624];
    __shared__ uint32_t tw[626];           /* the window's word list: [carried word] + tempered mt[idx..623] */
    __shared__ double vals[313 + 16];      /* [carried values] + the window's accepted values */
    __shared__ short pidx[313];            /* pair index of each accepted value of the window */
    const int lane = threadIdx.x;          /* one wave per generator: everything below is wave-uniform */
    double *rs = a.rs + (size_t)g * ICW_RSTATE;
    int idx;
    double prev_rnd;
    if (bk) {
        for (int i = lane; i < 624; i += 64) mt[i] = bk[i];
        idx = (int)bk[624];
        prev_rnd = *(const double *)(bk + 626);
    } else {
        for (int i = lane; i < 624; i += 64) mt[i] = a.mt[(size_t)i * a.mt_pitch + g];
        idx = a.mt_idx[g];
        prev_rnd = rs[0];
    }
    const double dth_mul = a.rk.dth_mul;
    /* generator-major (dith_gm): the wave's samples of a window are one contiguous run, each store
     * instruction writes 64 consecutive doubles; time-major: one double per row (K3b's layout) */
    double *dd = a.dith_gm ? a.dith + (size_t)g * a.dith_pitch : a.dith + g;
    const size_t dp = a.dith_gm ? 1 : a.dith_pitch;
    const int T = a.T;
    int t = 0, k = 0, c = 0;               /* samples done, carried values, carried word (0/1) */
    uint32_t cword = 0;
    __syncthreads();
    while (t < T) {
        if (idx >= 624) {
            icw_coop_twist(mt, lane);
            idx = 0;
        }
        const int nw = 624 - idx, nl = nw + c, np = nl >> 1;
        for (int j = lane; j < nw; j += 64) tw[c + j] = icw_mt_temper(mt[idx + j]);
        if (lane == 0 && c) tw[0] = cword;
        __syncthreads();
        int nacc = 0;
        for (int p0 = 0; p0 < np; p0 += 64) {
            const int pp = p0 + lane;
            bool acc = false;
            double d = 0.0;
            if (pp < np) {
                const uint32_t ua = tw[2 * pp] >> 5, ub = tw[2 * pp + 1] >> 6;
                acc = !(ua == 0u && ub == 0u);                  /* dsopen rejects exactly -1.0 */
                d = ((ua * 67108864.0 + ub) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
            }
            const unsigned long long m = __ballot(acc);
            const int pos = nacc + __popcll(m & ((1ull << lane) - 1ull));
            if (acc) { vals[k + pos] = d; pidx[pos] = (short)pp; }
            nacc += __popcll(m);
        }
        __syncthreads();
        const int nv = k + nacc;
        const int ns = min(nv / V, T - t);
        for (int sm = lane; sm < ns; sm += 64) {
            const double *v = vals + sm * V;
            double rnd;
            if (RT == ICW_RENDER_RPDF) {
                rnd = v[0] / ICW_SQRT2;
            } else if (RT == ICW_RENDER_TPDF) {
                rnd = v[0];
                rnd += v[1];
                rnd /= 2.0;
            } else if (RT == ICW_RENDER_STPDF) {
                rnd = (v[0] - (sm == 0 ? prev_rnd : v[-1])) / 2.0;
            } else {
                rnd = v[0];
#pragma unroll
                for (int i = 1; i < 12; ++i) rnd += v[i];
                rnd /= (2.0 * ICW_SQRT6);
            }
            dd[(size_t)(t + sm) * dp] = rnd * dth_mul;
        }
        if (RT == ICW_RENDER_STPDF && ns > 0) prev_rnd = vals[ns - 1];
        t += ns;
        if (t >= T) {
            /* the block ends inside this window: consume exactly through its last value's pair */
            const int need = ns * V - k;                        /* >= 1: carried values are < V */
            const int plast = pidx[need - 1];
            idx += 2 * (plast + 1) - c;
            c = 0;
        } else {
            /* everything consumed; carry the partial sample's values and an odd last word */
            const int kn = nv - ns * V;
            __syncthreads();
            double cv = 0.0;
            if (lane < kn) cv = vals[ns * V + lane];
            __syncthreads();
            if (lane < kn) vals[lane] = cv;
            k = kn;
            if (nl & 1) { cword = tw[nl - 1]; c = 1; }
            else c = 0;
            idx = 624;
        }
        __syncthreads();
    }
    for (int i = lane; i < 624; i += 64) a.mt[(size_t)i * a.mt_pitch + g] = mt[i];
    if (lane == 0) {
        a.mt_idx[g] = idx;
        rs[0] = prev_rnd;
    }
}

template <int RT>
__global__ __launch_bounds__(64) void icw_dither_coop(IcwK3Args a)
{
    icw_dither_coop_body<RT>(a, blockIdx.x, nullptr);
}

/* ------------------------------------------------------ split dither generator (K3t/K3s/K3f) ---- */
/* The dither term of sound_render_value (sound_render.c:711-751) consumes the channel's MT19937 words
 * in a fixed order: sample t of a chunk takes words [W t, W t + W) after the chunk's starting
 * position (W = 2 V: V dsopen values of two words each, mt_jrnd.c:218-256) -- unless a pair is
 * rejected (exactly -1.0, probability 2^-53 per pair), which shifts every later sample.  So
 *   K3t  icw_dith_twist    one wave per generator: saves the starting state (the backup), then runs
 *                          the twists (mt_jrnd.c:99-124) and writes the chunk's W T tempered words,
 *                          coalesced, and the generator's state after them (mt, idx);
 *   K3s  icw_dith_samples  a thread per sample, frame-parallel: its W words -> the V values -> rnd *
 *                          dth_mul (STPDF: the previous sample's value, or the backup's prev_rnd);
 *                          a rejected pair flags the generator;
 *   K3f  icw_dith_fix      a wave per flagged generator only: the chunk again from the backup, the
 *                          sequential way (icw_dither_coop_body, rejections and all), output and state.
 * The serial part left is the twist chain itself; K3a did the windows' tempering, pairing, ballots and
 * samples on the same wave between twists.  Chunks of at most a.wcap / W frames (icw_launch_dither). */
__global__ __launch_bounds__(64) void icw_dith_twist(IcwK3Args a, int W)
{
    __shared__ uint32_t mt[624];
    const int lane = threadIdx.x, g = blockIdx.x;
    uint32_t *bk = a.dbk + (size_t)g * ICW_DBK;
    double *rs = a.rs + (size_t)g * ICW_RSTATE;
    for (int i = lane; i < 624; i += 64) {
        const uint32_t v = a.mt[(size_t)i * a.mt_pitch + g];
        mt[i] = v;
        bk[i] = v;
    }
    int idx = a.mt_idx[g];
    if (lane == 0) {
        bk[624] = (uint32_t)idx;
        *(double *)(bk + 626) = rs[0];
        a.dflag[g] = 0;
    }
    __syncthreads();
    uint32_t *wr = a.wbuf + (size_t)g * a.wpitch;
    const long long nw = (long long)W * a.T;
    long long pos = 0;
    bool twisted = false;
    while (pos < nw) {
        if (idx >= 624) {
            icw_coop_twist(mt, lane);
            idx = 0;
            twisted = true;
        }
        const int n = (int)min((long long)(624 - idx), nw - pos);
        for (int j = lane; j < n; j += 64) wr[pos + j] = icw_mt_temper(mt[idx + j]);
        pos += n;
        idx += n;
    }
    if (twisted)
        for (int i = lane; i < 624; i += 64) a.mt[(size_t)i * a.mt_pitch + g] = mt[i];
    if (lane == 0) a.mt_idx[g] = idx;
}

/* the dsopen value of a word pair (mt_jrnd.c:218-256); rej: the pair is the rejected -1.0 */
__device__ __forceinline__ double icw_dsopen_pair(uint32_t wa, uint32_t wb, bool &rej)
{
    const uint32_t ua = wa >> 5, ub = wb >> 6;
    rej |= ua == 0u && ub == 0u;
    return ((ua * 67108864.0 + ub) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
}

/* gm: a thread per (generator, sample), samples fastest (generator-major rows, coalesced); tm: the
 * generators fastest (time-major rows, K3b / K3f) */
template <int RT>
__global__ __launch_bounds__(256) void icw_dith_samples(IcwK3Args a)
{
    constexpr int V = RT == ICW_RENDER_GAUSS ? 12 : (RT == ICW_RENDER_TPDF ? 2 : 1);
    constexpr int W = 2 * V;
    const long long id = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long tot = (long long)a.n_gen * a.T;
    if (id >= tot) return;
    int g, t;
    if (a.dith_gm) { g = (int)(id / a.T); t = (int)(id - (long long)g * a.T); }
    else { t = (int)(id / a.n_gen); g = (int)(id - (long long)t * a.n_gen); }
    const uint32_t *w = a.wbuf + (size_t)g * a.wpitch + (size_t)t * W;
    uint32_t u[W];
    if constexpr (W % 4 == 0) {
#pragma unroll
        for (int i = 0; i < W; i += 4) {
            const uint4 q = *(const uint4 *)(w + i);
            u[i] = q.x; u[i + 1] = q.y; u[i + 2] = q.z; u[i + 3] = q.w;
        }
    } else {
        const uint2 q = *(const uint2 *)w;
        u[0] = q.x; u[1] = q.y;
    }
    bool rej = false;
    double rnd;
    if constexpr (RT == ICW_RENDER_RPDF) {
        rnd = icw_dsopen_pair(u[0], u[1], rej) / ICW_SQRT2;
    } else if constexpr (RT == ICW_RENDER_TPDF) {
        rnd = icw_dsopen_pair(u[0], u[1], rej);
        rnd += icw_dsopen_pair(u[2], u[3], rej);
        rnd /= 2.0;
    } else if constexpr (RT == ICW_RENDER_STPDF) {
        double prev;
        if (t == 0) {
            prev = *(const double *)(a.dbk + (size_t)g * ICW_DBK + 626);
        } else {
            bool r2 = false;               /* the previous sample's own pair is flagged by its thread */
            prev = icw_dsopen_pair(w[-2], w[-1], r2);
        }
        const double tr = icw_dsopen_pair(u[0], u[1], rej);
        rnd = (tr - prev) / 2.0;
        if (t == a.T - 1) a.rs[(size_t)g * ICW_RSTATE] = tr;     /* prev_rnd after the chunk */
    } else {
        rnd = icw_dsopen_pair(u[0], u[1], rej);
#pragma unroll
        for (int i = 1; i < 12; ++i) rnd += icw_dsopen_pair(u[2 * i], u[2 * i + 1], rej);
        rnd /= (2.0 * ICW_SQRT6);
    }
    const size_t o = a.dith_gm ? (size_t)g * a.dith_pitch + t : (size_t)t * a.dith_pitch + g;
    a.dith[o] = rnd * a.rk.dth_mul;
    if (rej) atomicOr(&a.dflag[g], 1);
}

template <int RT>
__global__ __launch_bounds__(64) void icw_dith_fix(IcwK3Args a)
{
    const int g = blockIdx.x;
    if (!a.dflag[g]) return;               /* wave-uniform: the usual case, no rejected pair */
    icw_dither_coop_body<RT>(a, g, a.dbk + (size_t)g * ICW_DBK);
    if (threadIdx.x == 0) a.dflag[g] = 0;
}

/* Shaper history as a ring of R values (R = ICW_MAX_NS_TAPS for the FIR shapers, 4 for the
 * order-4 IIR shapers; R divides the unroll length ICW_MAX_NS_TAPS): at unrolled step J the newest
 * value goes to slot J mod R, so age i lives in slot (J - i) mod R -- compile-time indices, no
 * register moves (the reference's ring with a decrementing write pointer, sound_render.c:403-489). */
template <int R>
__device__ __forceinline__ void icw_ring_rotate1(double (&X)[R])
{
    const double r0 = X[0];
#pragma unroll
    for (int k = 0; k < R - 1; ++k) X[k] = X[k + 1];
    X[R - 1] = r0;
}

/* One sample of sound_render_value after the dither term (sound_render.c:754-809).  NN is the
 * shaper's tap count (a template parameter: a runtime count would predicate all 20 taps). */
template <int KIND, int R, int NN, int J>
__device__ __forceinline__ int icw_render_step(double input, double d, double &prev_err, double (&E)[R],
                                               double (&O)[R], const IcwRenderK &k, const double (&cf)[2 * NN + 1],
                                               unsigned &clips, double &pk)
{
    input = (input * k.norm_mul) - prev_err;
    double q = input + d;
    int delta;
    q = icw_round_q(q, k.round_offset, k.sign_delta, delta);
    pk = fmax(pk, fabs(q));
    const int vc = icw_clamp_int(q, k, clips);    /* unconditional: a NaN counts no clip */
    int val = (isnan(q) ? (int)0x80000000 : vc) + delta;
    /* noise shaping for the next sample (ns_empty / ns_fir / ns_iir) */
    const double ev = (double)val - input;
    double res = 0.0;
    if (KIND == 1) {
        E[J % R] = ev;
#pragma unroll
        for (int i = 0; i < NN; ++i) res += cf[i] * E[(J - i + 2 * R) % R];
    } else if (KIND == 2) {
        E[J % R] = ev;
#pragma unroll
        for (int i = 0; i < NN; ++i) res += cf[i] * E[(J - i + 2 * R) % R] - cf[i + NN] * O[(J - 1 - i + 2 * R) % R];
        O[J % R] = res;
    }
    prev_err = res;
    return val << k.norm_shift;
}

template <int KIND, int R, int NN, int J0>
__device__ __forceinline__ void icw_render_block(const double (&xin)[ICW_MAX_NS_TAPS], const double (&dv)[ICW_MAX_NS_TAPS],
                                                 double &prev_err, double (&E)[R], double (&O)[R], const IcwRenderK &k,
                                                 const double (&cf)[2 * NN + 1], unsigned &clips, double &pk, int *vrow,
                                                 int lim)
{
    if constexpr (J0 < ICW_MAX_NS_TAPS) {
        if (J0 < lim) {
            vrow[J0] = icw_render_step<KIND, R, NN, J0>(xin[J0], dv[J0], prev_err, E, O, k, cf, clips, pk);
            icw_render_block<KIND, R, NN, J0 + 1>(xin, dv, prev_err, E, O, k, cf, clips, pk, vrow, lim);
        }
    }
}

/* a full block whose step J refills xin[J] / dv[J] with the next block's sample right after
 * consuming it, so the loads run a block ahead of use (clamped indices stay in bounds) */
template <int KIND, int R, int NN, int J0>
__device__ __forceinline__ void icw_render_block_pf(double (&xin)[ICW_MAX_NS_TAPS], double (&dv)[ICW_MAX_NS_TAPS],
                                                    double &prev_err, double (&E)[R], double (&O)[R],
                                                    const IcwRenderK &k, const double (&cf)[2 * NN + 1],
                                                    unsigned &clips, double &pk, int *vrow, const double *pp,
                                                    const double *dp, size_t dpitch, int tn, int tmax)
{
    if constexpr (J0 < ICW_MAX_NS_TAPS) {
        vrow[J0] = icw_render_step<KIND, R, NN, J0>(xin[J0], dv[J0], prev_err, E, O, k, cf, clips, pk);
        const int tj = min(tn + J0, tmax);
        xin[J0] = pp[(size_t)tj * 2];
        dv[J0] = dp ? dp[(size_t)tj * dpitch] : 0.0;
        icw_render_block_pf<KIND, R, NN, J0 + 1>(xin, dv, prev_err, E, O, k, cf, clips, pk, vrow, pp, dp, dpitch, tn,
                                                 tmax);
    }
}

/* Write frames [f0, f1) of a block: the lane pair (L = even lane, R = odd lane) of a stream owns
 * the interleaved L,R frames; values come from the pair's LDS rows.  16-bit frames are one dword;
 * 24-bit frames are three 16-bit words (2-byte aligned for every stride). */
__device__ __forceinline__ void icw_put_frames(const int *vl, const int *vr, unsigned char *o, int osz, int f0, int f1)
{
    if (osz == 2) {
        for (int f = f0; f < f1; ++f)
            *(uint32_t *)(o + (size_t)f * 4) = ((uint32_t)vl[f] & 0xffffu) | ((uint32_t)vr[f] << 16);
    } else {
        for (int f = f0; f < f1; ++f) {
            const uint32_t l = (uint32_t)vl[f], r = (uint32_t)vr[f];
            uint16_t *q = (uint16_t *)(o + (size_t)f * 6);
            q[0] = (uint16_t)(l & 0xffffu);
            q[1] = (uint16_t)(((l >> 16) & 0xffu) | ((r & 0xffu) << 8));
            q[2] = (uint16_t)((r >> 8) & 0xffffu);
        }
    }
}

/* Render (K3b): the serial remainder of sound_render_value -- scale, error feedback, rounding,
 * clips, peak, noise shaper -- with the dither term from K3a.  One lane per channel, samples in
 * blocks of ICW_MAX_NS_TAPS (a multiple of the ring period): the block's inputs are loaded
 * before use.  rs keeps the shaper history by age (0 = newest), 20 + 20 slots. */
template <int KIND, int R, int NN>
__global__ __launch_bounds__(64) void icw_render_serial(IcwK3Args a)
{
    constexpr int NM = ICW_MAX_NS_TAPS;
    static_assert(NM % R == 0, "ring period must divide the unroll");
    __shared__ int vals[64][NM + 1];    /* the block's rendered values, one row per lane */
    const int lane = threadIdx.x;
    const int g0 = blockIdx.x * 64 + lane;
    const bool valid = g0 < a.n_gen;
    const int g = valid ? g0 : a.n_gen - 1;
    const int s = g >> 1, ch = g & 1;
    double *rs = a.rs + (size_t)g * ICW_RSTATE;
    double prev_err = rs[1];
    double E[R], O[R];
    /* block start: age i sits in slot (-1 - i) mod R */
#pragma unroll
    for (int i = 0; i < R; ++i) { E[(R - 1 - i) % R] = rs[2 + i]; O[(R - 1 - i) % R] = rs[2 + NM + i]; }
    const IcwRenderK &k = a.rk;
    double cf[2 * NN + 1];                                    /* shaper coefficients in registers */
#pragma unroll
    for (int i = 0; i < 2 * NN; ++i) cf[i] = k.ns_c[i];
    cf[2 * NN] = 0.0;
    const int osz = k.is24 ? 3 : 2;
    const double *pp = a.pre + (size_t)s * a.pre_stride + ch;
    const double *dp = a.dith ? a.dith + g : nullptr;         /* time-major [t][dith_pitch] */
    const size_t dpitch = a.dith_pitch;
    unsigned char *op = a.out + (size_t)s * a.out_stride;     /* the stream's frames */
    int *vrow = vals[lane];
    const int *vl = vals[lane & ~1], *vr = vals[lane | 1];
    const int half = (lane & 1) * (NM / 2);
    unsigned clips = 0;
    double pk = 0.0;
    const int T = a.T;
    int t = 0;
    double xin[NM], dv[NM];
    if (T >= NM) {
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            xin[j] = pp[(size_t)j * 2];
            dv[j] = dp ? dp[(size_t)j * dpitch] : 0.0;         /* ROUND: rnd * dth_mul == 0.0 * dth_mul */
        }
    }
    for (; t + NM <= T; t += NM) {
        icw_render_block_pf<KIND, R, NN, 0>(xin, dv, prev_err, E, O, k, cf, clips, pk, vrow, pp, dp, dpitch, t + NM,
                                            T - 1);
        __builtin_amdgcn_wave_barrier();
        if (valid) icw_put_frames(vl, vr, op + (size_t)t * 2 * osz, osz, half, half + NM / 2);
        __builtin_amdgcn_wave_barrier();
    }
    const int rem = T - t;
    if (rem > 0) {
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            xin[j] = j < rem ? pp[(size_t)(t + j) * 2] : 0.0;
            dv[j] = (j < rem && dp) ? dp[(size_t)(t + j) * dpitch] : 0.0;
        }
        icw_render_block<KIND, R, NN, 0>(xin, dv, prev_err, E, O, k, cf, clips, pk, vrow, rem);
        __builtin_amdgcn_wave_barrier();
        const int h = (rem + 1) / 2;
        if (valid) icw_put_frames(vl, vr, op + (size_t)t * 2 * osz, osz, (lane & 1) ? h : 0, (lane & 1) ? rem : h);
        /* back to the block-start mapping: rotate left by rem mod R */
#pragma unroll
        for (int r = 1; r < NM; ++r)
            if (r <= rem) { icw_ring_rotate1<R>(E); icw_ring_rotate1<R>(O); }
    }
    if (!valid) return;
    rs[1] = prev_err;
#pragma unroll
    for (int i = 0; i < R; ++i) { rs[2 + i] = E[(R - 1 - i) % R]; rs[2 + NM + i] = O[(R - 1 - i) % R]; }
    if (clips) atomicAdd(&a.clips[g], clips);
    if (pk > 0.0) atomicMax(&a.peak_bits[g], (unsigned long long)__double_as_longlong(pk));
}

/* ------------------------------------------------------- render, row broadcast (K3r) ------- */
/* The serial render of K3b with one 16-lane DPP row per channel instead of one lane, built like the
 * IIR kernel K1r (icw_iir.hip): every lane of a row runs the channel's chain redundantly, so each
 * value is row-uniform, and what is not on the chain leaves the per-sample instruction stream --
 * K3b spends ~51 instructions per sample for a ~22-instruction dependent chain:
 *   - the shaper terms: right after the error ev of sample n is known, ONE lane-parallel multiply
 *     makes lane l hold cf[l+1] * ev (P2: cf[l+17]), term l+1 of sample n+l+1; the sum adds it
 *     from that lane with `v_fmac_f64_dpp ... row_newbcast` (icw_render_asm.inc).  The IIR shaper's
 *     term cf[i]*E - cf[i+NN]*O is formed the same way, three lane-parallel ops per sample;
 *   - clips and peak: each lane stages q in its own LDS slot; at the end of a 20-sample block lane
 *     l counts samples l and l+16 (every row holds all of them) -- ~0.5 instead of ~6 per sample;
 *   - the frames: the shifted values are staged alike and a block's frames are written by 40
 *     lanes at once.
 * Sums keep the reference's order (res = 0.0; res += t_0; res += t_1 ...), products are rounded
 * before they are added, so every value is the reference's (sound_render.c:754-809, ns_fir
 * :403-438, ns_iir :442-489).  Small batches (the host's choice): 4 channels per wave. */
__device__ __forceinline__ double icw_rmul(double a, double b)
{
    double r;
    asm volatile("v_mul_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ double icw_rsub(double a, double b)
{
    double r;
    asm volatile("v_add_f64 %0, %1, -%2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

#include "icw_render_asm.inc"

struct IcwRowNs {
    double c0, cN;      /* row-uniform: cf[0]; IIR: cf[NN] (the O term of t_0) */
    double pl, pl2;     /* per lane: FIR cf[l+1], cf[l+17]; IIR cf[l+1], cf[l+1+NN] (0 past the taps) */
    double one;
};

/* one sample at unroll step J (0..ICW_MAX_NS_TAPS-1); rings of R slots, the newest at J mod R.
 *
 * The integer never sits on the error-feedback chain.  The reference forms val = (int)q' + delta
 * (q' the clipped q, sound_render.c:782-797) and feeds back ev = (double)val - input (:800).  q' lies
 * in [lo + 1, hi - 1] (|q'| < 2^24) and delta is 0 or -1, so (double)val = trunc(q') + (double)delta
 * exactly -- an integer-valued sum of two integers, no rounding; the trunc of a negative q' in (-1, 0)
 * is -0.0, and -0.0 + 0.0 = +0.0 = (double)0, -0.0 + -1.0 = -1.0 = (double)-1.  A NaN q (only from a
 * NaN input, which makes ev NaN either way) clamps to a number here; its stored value is fixed up in
 * the flush from the staged q, as the reference's (int)NaN = INT_MIN (cvttsd2si) + delta 0.  The
 * double val (vst) is converted to the integer off the chain, in the flush.
 * MR: mid-riser (round_offset 0, sign_delta -1: sound_render_recalc, sound_render.c:527-540) -- the
 * rounding add q + (+-0.0) changes nothing but a -0.0 (to +0.0), which neither the clip stage, the
 * peak (fabs) nor trunc + delta can tell apart, so it is skipped and only delta's select remains,
 * beside the clamp.  Mid-tread (round_offset 0.5, sign_delta 0): q +- 0.5 by the sign of q, both
 * sums formed beside the compare, delta 0.
 * The FIR shaper's first term 0.0 + c0 * ev (ns_fir, sound_render.c:420-427: the sum starts at 0.0)
 * is one fma(c0, ev, +0.0): the exact product plus +0.0, rounded once, is round(c0 * ev) with an
 * exact zero's sign made +, what 0.0 + round(c0 * ev) gives -- except where c0 * ev is nonzero but
 * rounds to zero (|ev| below ~2^-1022 / |c0|: a subnormal input with vd = 0): the fma then gives the
 * product's sign, -0.0 for a negative one, where the reference's 0.0 + (-0.0) is +0.0.  Only the sign
 * of a zero differs, in res (prev_ns_err), and nothing downstream can see it: input = xs - res, then
 * q = input + d, differ at most in a zero's sign, which trunc + delta, the clip stage and the peak
 * (fabs) all map alike, so ev, the integer and the meters are the reference's (the saved prev_ns_err
 * of the state blob may hold -0.0 for its +0.0).  On the chain per sample: the input and q, clamp
 * (2), trunc, + delta, ev, the fma and the shaper's DPP sum -- 16 ops for MEW44 where the integer
 * round trip and the rounding's compare / select / add made it 23 (14 in a clamp-free block). */
/* qst: the lane's slot for sample 0 in the q stage qs[row][U / 2][16][2] -- samples 2i and 2i + 1 of a
 * lane side by side, written together by one ds_write_b128 at the odd sample (qh holds the even one) */
template <int KIND, int NN, int R, int J, bool MR, bool FAST>
__device__ __forceinline__ void icw_rrow_step(double xs, double d, double &prev_err, double (&E)[R], double (&O)[R],
                                              double (&P)[R], double (&P2)[R], const IcwRowNs &c,
                                              const IcwRenderK &k, double *qst, double &qh, double &mq)
{
    constexpr int S = J % R;
    const double input = xs - prev_err;                /* xs = x * norm_mul, formed in the staging */
    double q = input + d;
    double dd;                                         /* (double)delta */
    if constexpr (MR) {
        dd = q < 0.0 ? -1.0 : 0.0;
    } else {
        const double qa = q + 0.5, qb = q - 0.5;       /* q + round_offset, q - round_offset */
        q = q < 0.0 ? qb : qa;
        dd = 0.0;
    }
    /* the clip stage as it reaches the integer (icw_clamp_int); clips and peak from the staged q.  A
     * clamp-free block (FAST, icw_render_row) has lo < q < hi for every sample, where the reference's
     * clip stage changes nothing and trunc(q) is already in [lo + 1, hi - 1] */
    double vd;
    if constexpr (FAST) {
        vd = __builtin_trunc(q) + dd;
    } else {
        vd = __builtin_trunc(fmax(fmin(q, k.hi - 1.0), k.lo + 1.0)) + dd;
        mq = icw_vmax_abs(mq, q);       /* the block's largest |q| (icw_render_rowc's calm test; unused otherwise) */
    }
    if constexpr (J & 1) *(double2 *)(qst + (J >> 1) * 32) = make_double2(qh, q);   /* the integer is the flush's */
    else qh = q;
    const double ev = vd - input;
    double res = 0.0;
    /* the new products go out before this sample's sum, whose volatile fmac block then separates
     * them from their first DPP read in the next sample (a VALU write -> DPP read needs two
     * instructions in between, and the compiler does not look into the asm) */
    if constexpr (KIND == 1) {
        E[S] = ev;
        P[S] = icw_rmul(c.pl, ev);
        if constexpr (NN > 17) P2[S] = icw_rmul(c.pl2, ev);
        res = __builtin_fma(c.c0, ev, 0.0);
        res = icw_ns_row_sum<NN, R, S>(res, c.one, P, P2);
    } else if constexpr (KIND == 2) {
        E[S] = ev;
        const double op = O[(S + R - 1) % R];
        P[S] = icw_rsub(icw_rmul(c.pl, ev), icw_rmul(c.pl2, op));
        res = 0.0 + (c.c0 * ev - c.cN * op);
        res = icw_ns_row_sum<NN, R, S>(res, c.one, P, P2);
        O[S] = res;
    }
    prev_err = res;
}

/* look-ahead reads: the next block's inputs and dither values of the row's channel, staged in LDS
 * (icw_rrow_stage_*): sample J of this block reads sample J of the next -- a whole block ahead of
 * its use, at an immediate offset (no address arithmetic per sample, no wait on global memory) */
template <int KIND, int NN, int R, int J, bool MR, bool FAST>
__device__ __forceinline__ void icw_rrow_block(double (&xin)[ICW_MAX_NS_TAPS], double (&dv)[ICW_MAX_NS_TAPS],
                                               double &prev_err, double (&E)[R], double (&O)[R], double (&P)[R],
                                               double (&P2)[R], const IcwRowNs &c, const IcwRenderK &k, double *qst,
                                               const double *xn, const double *dn, double &mq)
{
    if constexpr (J < ICW_MAX_NS_TAPS) {
        /* the next block's samples J, J + 1 by one ds_read_b128 each for x and d (16-byte aligned rows) */
        double qh;
        icw_rrow_step<KIND, NN, R, J, MR, FAST>(xin[J], dv[J], prev_err, E, O, P, P2, c, k, qst, qh, mq);
        icw_rrow_step<KIND, NN, R, J + 1, MR, FAST>(xin[J + 1], dv[J + 1], prev_err, E, O, P, P2, c, k, qst, qh, mq);
        /* after both steps, so the 16 bytes land in the pair's own registers (no moves) */
        const double2 x2 = *(const double2 *)(xn + J), d2 = *(const double2 *)(dn + J);
        xin[J] = x2.x;
        xin[J + 1] = x2.y;
        dv[J] = d2.x;
        dv[J + 1] = d2.y;
        icw_rrow_block<KIND, NN, R, J + 2, MR, FAST>(xin, dv, prev_err, E, O, P, P2, c, k, qst, xn, dn, mq);
    }
}

template <int KIND, int NN, int R, int J, bool MR>
__device__ __forceinline__ void icw_rrow_block_lim(const double (&xin)[ICW_MAX_NS_TAPS], const double (&dv)[ICW_MAX_NS_TAPS],
                                                   double &prev_err, double (&E)[R], double (&O)[R], double (&P)[R],
                                                   double (&P2)[R], const IcwRowNs &c, const IcwRenderK &k, double *qst,
                                                   int lim, double &mq)
{
    if constexpr (J < ICW_MAX_NS_TAPS) {
        if (J < lim) {
            double qh;
            icw_rrow_step<KIND, NN, R, J, MR, false>(xin[J], dv[J], prev_err, E, O, P, P2, c, k, qst, qh, mq);
            if (J + 1 < lim) {
                icw_rrow_step<KIND, NN, R, J + 1, MR, false>(xin[J + 1], dv[J + 1], prev_err, E, O, P, P2, c, k, qst, qh, mq);
                icw_rrow_block_lim<KIND, NN, R, J + 2, MR>(xin, dv, prev_err, E, O, P, P2, c, k, qst, lim, mq);
            } else {
                qst[(J >> 1) * 32] = qh;                 /* the last sample, an even one, alone */
            }
        }
    }
}

/* The staging of one block's inputs (frames t0 .. t0 + U - 1 of the wave's two streams, both
 * channels: lanes 0-19 / 32-51 load frame i of stream A / B, L and R in 16 bytes) and dither values
 * (its four channels: lanes 0-39 half a dither row each, 16 bytes); frames past T, streams past the
 * batch and channels past n_gen load nothing.  A block is loaded one block before it is stored to
 * LDS and stored one block before it is read, so no per-sample wait reaches global memory -- the
 * per-sample loads they replace ended each block in a full drain (s_waitcnt vmcnt(0)). */
struct IcwRowStage {
    double2 x, d;
};

/* What a lane stages, fixed for the launch: its source rows at t0 = 0 (the addresses then advance by
 * t0, no per-block 64-bit multiplies), its frame within a block for the t0 + i < T test, whether it
 * loads at all, and its LDS offsets inside one buffer (the buffer's own offset is a scalar) */
struct IcwRowLane {
    const double *xp, *dp;
    size_t dstr;                 /* dither elements per frame: dith_pitch (time-major) or 1 (generator-major) */
    int xi, di, di1;             /* frame of the x pair; frames of the dither pair's two values */
    bool xv, dvv;
    uint32_t xo, dof, d2;        /* LDS byte offsets of the x pair and the dither pair; d2 the second value's in doubles */
};

/* dither values, 40 lanes x 16 bytes: time-major, lane 2i + h loads channels 2h, 2h + 1 at frame i (LDS rows
 * 2h, 2h + 1); generator-major (dith_gm), lane 10c + p loads frames 2p, 2p + 1 of channel c (LDS row c) */
__device__ __forceinline__ IcwRowLane icw_rrow_lane(const IcwK3Args &a, int lane)
{
    constexpr int U = ICW_MAX_NS_TAPS;
    IcwRowLane L;
    const int sb = lane >> 5, i = lane & 31;
    const int s = blockIdx.x * 2 + sb;
    L.xi = i;
    L.xv = i < U && 2 * s < a.n_gen;
    L.xp = L.xv ? a.pre + (size_t)s * a.pre_stride + (size_t)i * 2 : a.pre;
    L.xo = (uint32_t)(((2 * sb) * U + (i < U ? i : 0)) * sizeof(double));
    const int ld = lane < 2 * U ? lane : 0;
    if (a.dith_gm) {
        const int ch = ld / (U / 2), p = ld % (U / 2);
        L.di = 2 * p;
        L.di1 = 2 * p + 1;
        L.dvv = a.dith && lane < 2 * U && (int)blockIdx.x * 4 + ch < a.n_gen;
        L.dp = L.dvv ? a.dith + (size_t)(blockIdx.x * 4 + ch) * a.dith_pitch + 2 * p : a.dith;
        L.dstr = 1;
        L.dof = (uint32_t)((ch * U + 2 * p) * sizeof(double));
        L.d2 = 1;
    } else {
        const int tt = ld >> 1, h = ld & 1;
        L.di = L.di1 = tt;
        L.dvv = a.dith && lane < 2 * U && (int)blockIdx.x * 4 + 2 * h < a.n_gen;
        L.dp = L.dvv ? a.dith + (size_t)tt * a.dith_pitch + blockIdx.x * 4 + 2 * h : a.dith;
        L.dstr = a.dith_pitch;
        L.dof = (uint32_t)(((2 * h) * U + tt) * sizeof(double));
        L.d2 = U;
    }
    return L;
}

__device__ __forceinline__ void icw_rrow_stage_load(const IcwK3Args &a, const IcwRowLane &L, int t0, IcwRowStage &st)
{
#ifdef ICW_K3R_NOLOAD
    if (t0 >= 3 * ICW_MAX_NS_TAPS) return;          /* diagnostic build (timing only): no staging loads */
#endif
    st.x = make_double2(0.0, 0.0);
    st.d = make_double2(0.0, 0.0);
    if (L.xv && t0 + L.xi < a.T) st.x = *(const double2 *)(L.xp + (size_t)t0 * 2);
    if (L.dvv && t0 + L.di1 < a.T) st.d = *(const double2 *)(L.dp + (size_t)t0 * L.dstr);
    else if (L.dvv && t0 + L.di < a.T) st.d.x = L.dp[(size_t)t0 * L.dstr];   /* generator-major: the last, odd frame */
}

/* The inputs go to LDS as x * norm_mul (sound_render.c:754's product, formed here lane-parallel: two
 * multiplies per block instead of one per sample on the chain).  Returns, wave-uniform, whether every
 * staged |x * norm_mul| <= thr (render_consts' spec_thr; NaN fails): the block may run clamp-free.
 * xs / ds: the buffer's x rows [4][U] and dither rows [4][U]. */
__device__ __forceinline__ bool icw_rrow_stage_store(double (*xs)[ICW_MAX_NS_TAPS], double (*ds)[ICW_MAX_NS_TAPS],
                                                     int lane, const IcwRowLane &L, const IcwRowStage &st, double nm,
                                                     double thr)
{
    constexpr int U = ICW_MAX_NS_TAPS;
    const int i = lane & 31;
    bool ok = true;
    if (i < U) {
        const double a = st.x.x * nm, b = st.x.y * nm;
        double *p = (double *)((char *)&xs[0][0] + L.xo);
        p[0] = a;
        p[U] = b;
        ok = fabs(a) <= thr && fabs(b) <= thr;
    }
    if (lane < 2 * U) {
        double *p = (double *)((char *)&ds[0][0] + L.dof);
        p[0] = st.d.x;
        p[L.d2] = st.d.y;
    }
    return __all(ok);
}

/* End of a block of nf samples: clips and peak of the staged q (lane l: samples l, l + 16 of its
 * row), then the block's frames -- lanes 0-31 write stream A's (rows 0, 1), 32-63 stream B's.  The
 * integer is the chain's trunc(q') + delta formed again from q, off the chain: the saturating
 * conversion, the clamp into [lo + 1, hi - 1] and the mid-riser's delta (q < 0); a NaN q gives
 * (int)NaN = INT_MIN (x86 cvttsd2si) with delta 0, as icw_render_round. */
template <bool MR>
__device__ __forceinline__ int icw_rrow_val(double q, int lo1, int hi1)
{
    const int v = icw_med3_i32(icw_cvt_sat_i32(q), lo1, hi1) + (MR && q < 0.0 ? -1 : 0);
    return q != q ? (int)0x80000000 : v;
}

/* (the exact form; returns, wave-uniform, whether every q of the block had |q| < clip_abs -- no clip,
 * so the next block may run clamp-free) */
template <bool MR>
__device__ __forceinline__ bool icw_rrow_flush(const double (*qs)[ICW_MAX_NS_TAPS / 2][16][2], int r, int lr, int lane,
                                               int nf, const IcwRenderK &k, unsigned &clips, double &pk,
                                               unsigned char *o0, unsigned char *o1, int osz)
{
    __builtin_amdgcn_wave_barrier();
    bool calm = true;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lr + 16 * h;
        if (j < nf) {
            const double q = qs[r][j >> 1][lr][j & 1];
            clips += (q >= k.hi ? 1u : 0u) + (q <= k.lo ? 1u : 0u);
            pk = fmax(pk, fabs(q));
            calm &= fabs(q) < k.clip_abs;
        }
    }
    calm = __all(calm);
    const int sb = lane >> 5, f = lane & 31;
    unsigned char *o = sb ? o1 : o0;
    if (o && f < nf) {
        const int lo1 = k.lo1, hi1 = k.hi1;
        const int vl = icw_rrow_val<MR>(qs[2 * sb][f >> 1][0][f & 1], lo1, hi1);
        const int vr = icw_rrow_val<MR>(qs[2 * sb + 1][f >> 1][0][f & 1], lo1, hi1);
        const uint32_t l = (uint32_t)(vl << k.norm_shift);
        const uint32_t rr = (uint32_t)(vr << k.norm_shift);
        if (osz == 2) {
            *(uint32_t *)(o + (size_t)f * 4) = (l & 0xffffu) | (rr << 16);
        } else {
            uint16_t *p = (uint16_t *)(o + (size_t)f * 6);
            p[0] = (uint16_t)(l & 0xffffu);
            p[1] = (uint16_t)(((l >> 16) & 0xffu) | ((rr & 0xffu) << 8));
            p[2] = (uint16_t)((rr >> 8) & 0xffffu);
        }
    }
    __builtin_amdgcn_wave_barrier();
    return calm;
}

/* the flush of a clamp-free block: every |q| < clip_abs, finite -- no clip to count, the integer is the
 * plain conversion (exact below 2^31) + the mid-riser's delta, no clamp, no NaN */
template <bool MR>
__device__ __forceinline__ void icw_rrow_flush_fast(const double (*qs)[ICW_MAX_NS_TAPS / 2][16][2], int r, int lr, int lane,
                                                    const IcwRenderK &k, double &pk, unsigned char *o, int osz)
{
    constexpr int U = ICW_MAX_NS_TAPS;
    __builtin_amdgcn_wave_barrier();
    /* the four reads first, unconditionally (clamped indices; a lane's second peak sample repeats its
     * first where lr + 16 >= U, which changes no maximum), so they share one wait */
    const int f = lane & 31, sb = lane >> 5, fc = f < U ? f : U - 1;
    const int j1 = lr + 16 < U ? lr + 16 : lr;
    const double q0 = qs[r][lr >> 1][lr][lr & 1];
    const double q1 = qs[r][j1 >> 1][lr][j1 & 1];
    const double ql = qs[2 * sb][fc >> 1][0][fc & 1], qr = qs[2 * sb + 1][fc >> 1][0][fc & 1];
    pk = icw_vmax_abs(icw_vmax_abs(pk, q0), q1);
    const int vl = icw_cvt_sat_i32(ql) + (MR && ql < 0.0 ? -1 : 0);
    const int vr = icw_cvt_sat_i32(qr) + (MR && qr < 0.0 ? -1 : 0);
    const uint32_t l = (uint32_t)(vl << k.norm_shift);
    const uint32_t rr = (uint32_t)(vr << k.norm_shift);
    /* o: this lane's frame in the block's output (null: no frame to write) */
    if (o) {
        if (osz == 2) {
            *(uint32_t *)o = (l & 0xffffu) | (rr << 16);
        } else {
            uint16_t *p = (uint16_t *)o;
            p[0] = (uint16_t)(l & 0xffffu);
            p[1] = (uint16_t)(((l >> 16) & 0xffu) | ((rr & 0xffu) << 8));
            p[2] = (uint16_t)((rr >> 8) & 0xffffu);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

template <int KIND, int NN, bool MR>
__global__ __launch_bounds__(64) void icw_render_row(IcwK3Args a)
{
    constexpr int U = ICW_MAX_NS_TAPS;                 /* samples per unrolled block */
    constexpr int R = KIND == 1 ? U : (KIND == 2 ? 4 : 1);
    static_assert(U % R == 0, "ring period must divide the unroll");
    static_assert(U % 2 == 0, "samples go in pairs");
    __shared__ __attribute__((aligned(16))) double qs[4][U / 2][16][2];   /* q of each sample, every lane its own slots */
    const int lane = threadIdx.x, r = lane >> 4, lr = lane & 15;
    const int g0 = blockIdx.x * 4 + r;
    const bool valid = g0 < a.n_gen;
    const int g = valid ? g0 : a.n_gen - 1;            /* spare rows run on zeros, store nothing */
    const IcwRenderK &k = a.rk;
    double *rs = a.rs + (size_t)g * ICW_RSTATE;
    double prev_err = rs[1];
    double E[R], O[R], P[R], P2[R];
    IcwRowNs c;
    c.one = 1.0;
    c.c0 = k.ns_c[0];
    c.cN = KIND == 2 ? k.ns_c[NN] : 0.0;
    if constexpr (KIND == 2) {
        c.pl = lr + 1 < NN ? k.ns_c[lr + 1] : 0.0;
        c.pl2 = lr + 1 < NN ? k.ns_c[lr + 1 + NN] : 0.0;
    } else {
        c.pl = lr + 1 < NN ? k.ns_c[lr + 1] : 0.0;
        c.pl2 = lr + 17 < NN ? k.ns_c[lr + 17] : 0.0;
    }
    /* block start: age i sits in slot (-1 - i) mod R; the products of those ages */
#pragma unroll
    for (int i = 0; i < R; ++i) {
        E[(R - 1 - i) % R] = rs[2 + i];
        O[(R - 1 - i) % R] = rs[2 + U + i];
    }
    if constexpr (KIND == 1) {
#pragma unroll
        for (int m = 0; m < R; ++m) {
            P[m] = icw_rmul(c.pl, E[m]);
            if constexpr (NN > 17) P2[m] = icw_rmul(c.pl2, E[m]);
        }
    } else if constexpr (KIND == 2) {
#pragma unroll
        for (int m = 0; m < R; ++m) P[m] = icw_rsub(icw_rmul(c.pl, E[m]), icw_rmul(c.pl2, O[(m + R - 1) % R]));
    }
    asm volatile("s_nop 1");                           /* VALU write -> DPP read of P / P2 */
    const int osz = k.is24 ? 3 : 2;
    /* the wave's two streams (channels 4b..4b+3); a stream past the batch writes nothing */
    const int sA = blockIdx.x * 2, sB = sA + 1;
    unsigned char *oA = 2 * sA < a.n_gen ? a.out + (size_t)sA * a.out_stride : nullptr;
    unsigned char *oB = 2 * sB < a.n_gen ? a.out + (size_t)sB * a.out_stride : nullptr;
    double *qst = &qs[r][0][lr][0];
    unsigned clips = 0;
    double pk = 0.0;
    const int T = a.T;
    /* block j's inputs in LDS buffer j & 1: loaded at the end of block j - 3, stored at the end of
     * block j - 2, read (a block ahead) during block j - 1 */
    __shared__ __attribute__((aligned(16))) double xsl[2][4][U];
    __shared__ __attribute__((aligned(16))) double dsl[2][4][U];
    const double nm = k.norm_mul, thr = k.spec_thr;
    IcwRowStage stg;
    const IcwRowLane sl = icw_rrow_lane(a, lane);
    /* the frame this lane writes in a clamp-free block's flush: frame lane & 31 of stream A / B */
    unsigned char *const olane = (lane & 31) < U && ((lane >> 5) ? oB : oA) ? ((lane >> 5) ? oB : oA) + (size_t)(lane & 31) * 2 * osz
                                                                          : nullptr;
    icw_rrow_stage_load(a, sl, 0, stg);
    bool x_ok0 = icw_rrow_stage_store(xsl[0], dsl[0], lane, sl, stg, nm, thr);
    icw_rrow_stage_load(a, sl, U, stg);
    bool x_ok1 = icw_rrow_stage_store(xsl[1], dsl[1], lane, sl, stg, nm, thr);
    icw_rrow_stage_load(a, sl, 2 * U, stg);
    __builtin_amdgcn_wave_barrier();
    double xin[U], dv[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        xin[j] = xsl[0][r][j];
        dv[j] = dsl[0][r][j];
    }
    /* Clamp-free blocks (render_consts: spec_thr).  A block runs without the clip stage when the block
     * before it clipped nowhere (every |q| < clip_abs: `calm`) and its own inputs are all within
     * spec_thr; it then clips nowhere itself, so the next block's history is calm too.  The first block
     * of a launch starts from a saved history and takes the exact form.  Wave-uniform (__all).
     * The two forms run in loops of their own, each with its own back edge: with one loop and the form
     * chosen per block, the register allocation of the two unrolled bodies met at the loop's end, and
     * every block paid ~80 AGPR / VGPR moves for it (more than the clamp it saved). */
    bool calm = false;
    int t = 0, kb = 0;
    double mq_unused = 0.0;             /* this kernel's calm test is the flush's */
    /* one block of either form, the staging of block kb + 2 (into the buffer block kb has left), the
     * block's flush, and block kb + 3 on its way.  The staging comes before the flush: its stores to
     * LDS wait for the registers loaded one block ago, and on gfx950 that wait (vmcnt) also counts
     * the global stores issued before it -- after the flush it waited for the block's own output
     * stores to complete. */
    auto step = [&](auto fast) {
        constexpr bool FAST = decltype(fast)::value;
        const int nb = (kb + 1) & 1;
        unsigned char *ot0 = oA ? oA + (size_t)t * 2 * osz : nullptr, *ot1 = oB ? oB + (size_t)t * 2 * osz : nullptr;
        icw_rrow_block<KIND, NN, R, 0, MR, FAST>(xin, dv, prev_err, E, O, P, P2, c, k, qst, &xsl[nb][r][0],
                                                 &dsl[nb][r][0], mq_unused);
        x_ok0 = x_ok1;
        x_ok1 = icw_rrow_stage_store(xsl[kb & 1], dsl[kb & 1], lane, sl, stg, nm, thr);
        if constexpr (FAST) {
            icw_rrow_flush_fast<MR>(qs, r, lr, lane, k, pk, olane ? olane + (size_t)t * 2 * osz : nullptr, osz);
#ifdef ICW_K3R_COUNT
            if (lr == 0 && valid) atomicAdd(&a.clips[g], 1u);   /* diagnostic build: clamp-free blocks */
#endif
        } else {
            calm = icw_rrow_flush<MR>(qs, r, lr, lane, U, k, clips, pk, ot0, ot1, osz);
        }
        icw_rrow_stage_load(a, sl, t + 3 * U, stg);
        __builtin_amdgcn_wave_barrier();
        t += U;
        ++kb;
    };
    while (t + U <= T) {
        while (t + U <= T && !(KIND != 2 && calm && x_ok0)) step(icw_ic<0>());
        if constexpr (KIND != 2) {
            while (t + U <= T && x_ok0) step(icw_ic<1>());
        }
    }
    const int rem = T - t;
    if (rem > 0) {
        icw_rrow_block_lim<KIND, NN, R, 0, MR>(xin, dv, prev_err, E, O, P, P2, c, k, qst, rem, mq_unused);
        icw_rrow_flush<MR>(qs, r, lr, lane, rem, k, clips, pk, oA ? oA + (size_t)t * 2 * osz : nullptr,
                           oB ? oB + (size_t)t * 2 * osz : nullptr, osz);
        /* back to the block-start mapping: rotate left by rem mod R */
#pragma unroll
        for (int q = 1; q < U; ++q)
            if (q <= rem) { icw_ring_rotate1<R>(E); icw_ring_rotate1<R>(O); }
    }
    /* meters: the row's lanes hold disjoint samples */
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
        clips += __shfl_xor(clips, off);
        pk = fmax(pk, __shfl_xor(pk, off));
    }
    if (!valid || lr != 0) return;
    rs[1] = prev_err;
#pragma unroll
    for (int i = 0; i < R; ++i) { rs[2 + i] = E[(R - 1 - i) % R]; rs[2 + U + i] = O[(R - 1 - i) % R]; }
    if (clips) atomicAdd(&a.clips[g], clips);
    if (pk > 0.0) atomicMax(&a.peak_bits[g], (unsigned long long)__double_as_longlong(pk));
}

/* ------------------------------------------- render, row broadcast + companion wave (K3c) ------ */
/* icw_render_row with everything that is not the error-feedback chain moved to a second wave of the
 * workgroup, which the dispatcher puts on another SIMD of the CU.  A lone wave issues one FP64 op per
 * ~5 cycles, so in K3r every staging load, LDS store, integer conversion, meter update and
 * output store was issue time taken from the chain: 18.9 VALU + 2.5 SALU + 1.8 LDS per sample for a
 * 16-op chain (MEW44).  Here
 *   wave 0 (chain)      runs only the chain of sound_render.c:754-809 on its four channels: per sample
 *                       the row-uniform chain, one ds_read_b128 per two samples for x and for the
 *                       dither value (the next block, staged), one ds_write_b128 per two samples for q;
 *                       per block one counter read and one counter write;
 *   wave 1 (companion)  stages block n (global loads issued four blocks ahead, x * norm_mul, the
 *                       clamp-free input test) into staging buffer n mod 4 and publishes `staged`;
 *                       flushes block n - 4 once the chain has published it `done` (the exact flush of
 *                       icw_rrow_flush: integers, clips, peak, packed frames) and publishes `flushed`.
 * The hand-offs are LDS counters.  The LDS executes one wave's DS instructions in order, so a counter
 * written after a block's data is seen only once the data is there; the compiler is kept from
 * moving memory accesses across a counter access by a fence of its own.  The chain checks, at each
 * block start, the counters it read at the previous one (the companion runs a block ahead), so the
 * check costs no wait; it spins (s_sleep) only if the companion fell behind.  Every spin is bounded:
 * a hand-off that never comes flags a.err and the wave goes on, so the grid drains.
 * The clamp-free decision needs the block before to have been calm (no |q| >= clip_abs, no NaN):
 * the chain itself keeps max |q| in an exact block (one v_max_f64 per sample, only there); a NaN q
 * makes the chain's error, and so prev_ns_err, NaN for good (the shaper's sum of a NaN), which the
 * block-end test also sees; a FIR shaper's NaN is never self-clearing, a flat one has no history.
 * Results are icw_render_row's bit for bit: the same chain code, the same exact flush for every
 * block (a clamp-free block gives the same integers through it: no clip, no NaN). */
#define ICW_K3C_NSB 4                  /* staging buffers (blocks) */
#define ICW_K3C_NQB 4                  /* q buffers (blocks) */
#define ICW_K3C_SPIN (1u << 24)        /* spin bound: ~2^24 s_sleep(1), far beyond any healthy wait */

__device__ __forceinline__ void icw_cfence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ unsigned long long icw_lds_ld64(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ int icw_lds_ld32(const int *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void icw_lds_st32(int *p, int v)
{
    icw_cfence();
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* chain side: the counters (staged word | flushed << 32) once staged >= ns and flushed >= nf.  The
 * staged word is (blocks staged) << 4 | the clamp-free input tests of the last four staged blocks (bit
 * n mod 4 for block n), so one 64-bit read per block brings the chain both counters and block j + 1's
 * test (inline, as every hand-off here: a call would make the callee wait for all memory traffic) */
__device__ __forceinline__ unsigned long long icw_k3c_wait(const unsigned long long *sf, int ns, int nf, int32_t *err)
{
    unsigned long long v = icw_lds_ld64(sf);
    for (unsigned spin = 0;; ++spin) {
        const int st = __builtin_amdgcn_readfirstlane((int)(uint32_t)v) >> 4;
        const int fl = __builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
        if (st >= ns && fl >= nf) break;
        if (spin >= ICW_K3C_SPIN) {
            if (err && threadIdx.x == 0) atomicOr(err, 1);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = icw_lds_ld64(sf);
    }
    icw_cfence();
    return v;
}

/* companion side: wait until the chain has published at least n blocks done */
__device__ __forceinline__ void icw_k3c_wait_done(const int *dn, int n, int32_t *err)
{
    for (unsigned spin = 0; __builtin_amdgcn_readfirstlane(icw_lds_ld32(dn)) < n; ++spin) {
        if (spin >= ICW_K3C_SPIN) {
            if (err && threadIdx.x == 64) atomicOr(err, 1);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    icw_cfence();
}

/* The companion's staging (generator-major dither rows).  Loads are issued by every lane from a
 * clamped, always valid address (the frame index held to T - 1, a spare lane on its row's first frame)
 * and the values a lane has no business loading are zeroed only at the store, four blocks later: a load
 * under a branch, or a select right after it, made the compiler wait for all memory traffic
 * (vmcnt(0)) every block.  A dither pair starting at the block's last, even frame reads the row's
 * padding (dith_pitch is T rounded up to even). */
struct IcwCompLane {
    const double *xr, *dr;       /* the lane's x row and dither row (frame 0; a spare lane: row 0 of the batch) */
    int xi, di;                  /* frame offsets in a block: x frame, first frame of the dither pair */
    bool xv, dvv;
    uint32_t xo, dof;            /* LDS byte offsets in a staging buffer */
};

__device__ __forceinline__ IcwCompLane icw_k3c_lane(const IcwK3Args &a, int lane)
{
    constexpr int U = ICW_MAX_NS_TAPS;
    IcwCompLane L;
    const int sb = lane >> 5, i = lane & 31;
    const int s = blockIdx.x * 2 + sb;
    L.xi = i < U ? i : 0;
    L.xv = i < U && 2 * s < a.n_gen;
    L.xr = L.xv ? a.pre + (size_t)s * a.pre_stride : a.pre;
    L.xo = (uint32_t)(((2 * sb) * U + L.xi) * sizeof(double));
    const int ld = lane < 2 * U ? lane : 0;
    const int ch = ld / (U / 2), p = ld % (U / 2);
    L.di = 2 * p;
    L.dvv = a.dith && lane < 2 * U && (int)blockIdx.x * 4 + ch < a.n_gen;
    L.dr = L.dvv ? a.dith + (size_t)(blockIdx.x * 4 + ch) * a.dith_pitch : a.pre;
    L.dof = (uint32_t)((ch * U + 2 * p) * sizeof(double));
    return L;
}

__device__ __forceinline__ void icw_k3c_stage_load(const IcwK3Args &a, const IcwCompLane &L, int t0, IcwRowStage &st)
{
    const int T1 = a.T - 1;
    const int fx = t0 + L.xi < T1 ? t0 + L.xi : T1;
    const int fd = t0 + L.di < T1 ? t0 + L.di : (T1 & ~1);
    st.x = *(const double2 *)(L.xr + (size_t)fx * 2);
    st.d = *(const double2 *)(L.dr + fd);
}

/* block t0's values to staging buffer (xs, ds); returns, wave-uniform, the clamp-free input test.
 * Branch-free: the lanes without a slot store into dum (a scratch area of 64 x 32 bytes), so every
 * loaded register is consumed on every path (a skipped store left its pending load's register free for
 * reuse, and the write to it waited for all memory traffic). */
__device__ __forceinline__ bool icw_k3c_stage_store(double (*xs)[ICW_MAX_NS_TAPS], double (*ds)[ICW_MAX_NS_TAPS], double *dum,
                                                    int lane, const IcwCompLane &L, const IcwRowStage &st, int t0, int T,
                                                    double nm, double thr)
{
    constexpr int U = ICW_MAX_NS_TAPS;
    const bool xl = (lane & 31) < U, dl = lane < 2 * U;
    const bool v = L.xv && t0 + L.xi < T;
    const double a = (v ? st.x.x : 0.0) * nm, b = (v ? st.x.y : 0.0) * nm;
    double *px = xl ? (double *)((char *)&xs[0][0] + L.xo) : dum + lane * 4;
    px[0] = a;
    px[xl ? U : 1] = b;
    const bool ok = !xl || (fabs(a) <= thr && fabs(b) <= thr);
    const bool v0 = L.dvv && t0 + L.di < T, v1 = L.dvv && t0 + L.di + 1 < T;
    double *pd = dl ? (double *)((char *)&ds[0][0] + L.dof) : dum + lane * 4 + 2;
    *(double2 *)pd = make_double2(v0 ? st.d.x : 0.0, v1 ? st.d.y : 0.0);
    return __all(ok);
}

template <int KIND, int NN, bool MR>
__global__ __launch_bounds__(128) void icw_render_rowc(IcwK3Args a)
{
    constexpr int U = ICW_MAX_NS_TAPS, NSB = ICW_K3C_NSB, NQB = ICW_K3C_NQB;
    constexpr int R = KIND == 1 ? U : (KIND == 2 ? 4 : 1);
    constexpr int QSTR = 4 * (U / 2) * 16 * 2;          /* doubles per q buffer */
    static_assert(U % R == 0, "ring period must divide the unroll");
    static_assert(U % 2 == 0, "samples go in pairs");
    static_assert(NSB == 4 && NQB == 4, "the companion's schedule below assumes four buffers of each");
    __shared__ __attribute__((aligned(16))) double qsb[NQB][4][U / 2][16][2];
    __shared__ __attribute__((aligned(16))) double xsl[NSB][4][U];
    __shared__ __attribute__((aligned(16))) double dsl[NSB][4][U];
    __shared__ __attribute__((aligned(8))) int cnt[4];  /* staged word (icw_k3c_wait), flushed, done (blocks) */
    __shared__ __attribute__((aligned(16))) double dum[64 * 4];   /* the companion's slotless stores */
    const int T = a.T;
    if (T <= 0) return;
    const int nbk = (T + U - 1) / U, nfull = T / U;
    const IcwRenderK &k = a.rk;
    const int osz = k.is24 ? 3 : 2;
    if (threadIdx.x == 0) { cnt[0] = 0; cnt[1] = 0; cnt[2] = 0; cnt[3] = 0; }
    __syncthreads();
    const unsigned long long *sfp = (const unsigned long long *)&cnt[0];
    if (threadIdx.x < 64) {
        /* ------------------------------------------------------------------ the chain ------ */
        const int lane = threadIdx.x, r = lane >> 4, lr = lane & 15;
        const int g0 = blockIdx.x * 4 + r;
        const bool valid = g0 < a.n_gen;
        const int g = valid ? g0 : a.n_gen - 1;
        double *rs = a.rs + (size_t)g * ICW_RSTATE;
        double prev_err = rs[1];
        double E[R], O[R], P[R], P2[R];
        IcwRowNs c;
        c.one = 1.0;
        c.c0 = k.ns_c[0];
        c.cN = KIND == 2 ? k.ns_c[NN] : 0.0;
        if constexpr (KIND == 2) {
            c.pl = lr + 1 < NN ? k.ns_c[lr + 1] : 0.0;
            c.pl2 = lr + 1 < NN ? k.ns_c[lr + 1 + NN] : 0.0;
        } else {
            c.pl = lr + 1 < NN ? k.ns_c[lr + 1] : 0.0;
            c.pl2 = lr + 17 < NN ? k.ns_c[lr + 17] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
            E[(R - 1 - i) % R] = rs[2 + i];
            O[(R - 1 - i) % R] = rs[2 + U + i];
        }
        if constexpr (KIND == 1) {
#pragma unroll
            for (int m = 0; m < R; ++m) {
                P[m] = icw_rmul(c.pl, E[m]);
                if constexpr (NN > 17) P2[m] = icw_rmul(c.pl2, E[m]);
            }
        } else if constexpr (KIND == 2) {
#pragma unroll
            for (int m = 0; m < R; ++m) P[m] = icw_rsub(icw_rmul(c.pl, E[m]), icw_rmul(c.pl2, O[(m + R - 1) % R]));
        }
        asm volatile("s_nop 1");                       /* VALU write -> DPP read of P / P2 */
        double *const qst = &qsb[0][r][0][lr][0];
        /* blocks 0 and 1 staged: block 0 into registers, block 1 is read during block 0 */
        unsigned long long sf = icw_k3c_wait(sfp, nbk < 2 ? nbk : 2, 0, a.err);
        double xin[U], dv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            xin[j] = xsl[0][r][j];
            dv[j] = dsl[0][r][j];
        }
        bool okn = (__builtin_amdgcn_readfirstlane((int)(uint32_t)sf) & 1) != 0;   /* block j's clamp-free input test */
        bool calm = false;                             /* the block before j clipped nowhere (no NaN) */
        int j = 0;
        auto step = [&](auto fast) {
            constexpr bool FAST = decltype(fast)::value;
            /* the counters read one block ago: block j + 1 staged, block j - NQB flushed */
            const int ns = j + 2 < nbk ? j + 2 : nbk, nf = j + 1 - NQB;
            if ((__builtin_amdgcn_readfirstlane((int)(uint32_t)sf) >> 4) < ns ||
                __builtin_amdgcn_readfirstlane((int)(uint32_t)(sf >> 32)) < nf)
                sf = icw_k3c_wait(sfp, ns, nf, a.err);
            icw_cfence();
            /* for the next block's check, and block j + 1's input test: staged then covers blocks up to
             * at most j + 3 (the companion stages block n after the chain's block n - 4), j + 1 among its
             * last four */
            sf = icw_lds_ld64(sfp);
            const int nb = (j + 1) & (NSB - 1);
            double mq = 0.0;
            icw_rrow_block<KIND, NN, R, 0, MR, FAST>(xin, dv, prev_err, E, O, P, P2, c, k, qst + (j & (NQB - 1)) * QSTR,
                                                     &xsl[nb][r][0], &dsl[nb][r][0], mq);
            if constexpr (!FAST) calm = __all(mq < k.clip_abs && prev_err == prev_err);
            icw_lds_st32(&cnt[2], j + 1);
            __builtin_amdgcn_sched_barrier(0);         /* the read of sf stays a block ahead of this use */
            okn = ((__builtin_amdgcn_readfirstlane((int)(uint32_t)sf) >> nb) & 1) != 0;
            ++j;
        };
        while (j < nfull) {
            while (j < nfull && !(KIND != 2 && calm && okn)) step(icw_ic<0>());
            if constexpr (KIND != 2) {
                while (j < nfull && okn) step(icw_ic<1>());
            }
        }
        const int rem = T - nfull * U;
        if (rem > 0) {
            const int nf = j + 1 - NQB;
            if (__builtin_amdgcn_readfirstlane((int)(uint32_t)(sf >> 32)) < nf) sf = icw_k3c_wait(sfp, nbk, nf, a.err);
            icw_cfence();
            double mq = 0.0;
            icw_rrow_block_lim<KIND, NN, R, 0, MR>(xin, dv, prev_err, E, O, P, P2, c, k, qst + (j & (NQB - 1)) * QSTR,
                                                   rem, mq);
            icw_lds_st32(&cnt[2], j + 1);
#pragma unroll
            for (int q = 1; q < U; ++q)
                if (q <= rem) { icw_ring_rotate1<R>(E); icw_ring_rotate1<R>(O); }
        }
        if (!valid || lr != 0) return;
        rs[1] = prev_err;
#pragma unroll
        for (int i = 0; i < R; ++i) { rs[2 + i] = E[(R - 1 - i) % R]; rs[2 + U + i] = O[(R - 1 - i) % R]; }
    } else {
        /* -------------------------------------------------------------- the companion ------ */
        const int lane = threadIdx.x - 64, r = lane >> 4, lr = lane & 15;
        const bool valid = (int)blockIdx.x * 4 + r < a.n_gen;
        const IcwCompLane sl = icw_k3c_lane(a, lane);
        const double nm = k.norm_mul, thr = k.spec_thr;
        const int sA = blockIdx.x * 2, sB = sA + 1;
        unsigned char *oA = 2 * sA < a.n_gen ? a.out + (size_t)sA * a.out_stride : nullptr;
        unsigned char *oB = 2 * sB < a.n_gen ? a.out + (size_t)sB * a.out_stride : nullptr;
        unsigned clips = 0;
        double pk = 0.0;
        IcwRowStage rg[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) icw_k3c_stage_load(a, sl, i * U, rg[i]);
        unsigned okm = 0;                              /* clamp-free input tests of the last four staged blocks */
        /* iteration n: flush block n - 4 (the chain has moved on to n - 3), then stage block n into
         * buffer n mod 4 (its last reader, block n - 5, is done) and send its registers for block n + 4 */
        auto iter = [&](int n, IcwRowStage &st) {
            if (n >= 4 && n - 4 < nbk) {
                const int jf = n - 4;
                icw_k3c_wait_done(&cnt[2], jf + 1, a.err);
                const int t = jf * U, nf = T - t < U ? T - t : U;
                (void)icw_rrow_flush<MR>(qsb[jf & (NQB - 1)], r, lr, lane, nf, k, clips, pk,
                                         oA ? oA + (size_t)t * 2 * osz : nullptr, oB ? oB + (size_t)t * 2 * osz : nullptr, osz);
                icw_lds_st32(&cnt[1], jf + 1);
            }
            /* unconditional, past the last block too (zeros into a buffer nobody reads any more, a
             * staged count past nbk): with the loads under a branch, the compiler's wait for a register
             * set assumed the path without the later loads and waited for everything */
            const int b = n & (NSB - 1);
            const bool ok = icw_k3c_stage_store(xsl[b], dsl[b], dum, lane, sl, st, n * U, T, nm, thr);
            okm = (okm & ~(1u << b)) | ((ok ? 1u : 0u) << b);
            icw_lds_st32(&cnt[0], (int)(((unsigned)(n + 1) << 4) | okm));
            icw_k3c_stage_load(a, sl, (n + 4) * U, st);
        };
        for (int n0 = 0; n0 < nbk + 4; n0 += 4) {
            iter(n0, rg[0]);
            iter(n0 + 1, rg[1]);
            iter(n0 + 2, rg[2]);
            iter(n0 + 3, rg[3]);
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            clips += __shfl_xor(clips, off);
            pk = fmax(pk, __shfl_xor(pk, off));
        }
        if (!valid || lr != 0) return;
        const int g = blockIdx.x * 4 + r;
        if (clips) atomicAdd(&a.clips[g], clips);
        if (pk > 0.0) atomicMax(&a.peak_bits[g], (unsigned long long)__double_as_longlong(pk));
    }
}

/* Render with FP_CHECK (K3f): sound_render_value's WITH FC CHECKS arithmetic (sound_render.c:
 * 857-903) and ns_fir / ns_iir's (428-433, 474-486), counting into the render census.  One lane per
 * channel like K3b, but compact (run-time loops, the reference's own decrementing ring in private
 * memory): a diagnostic mode.  The dither term comes from K3a; its FC() are identities (the sums of
 * dsopen values are multiples of 2^-56 below 12 in magnitude, never special). */
__global__ __launch_bounds__(64) void icw_render_fc(IcwK3Args a)
{
    constexpr int NM = ICW_MAX_NS_TAPS;
    const int g = blockIdx.x * 64 + threadIdx.x;
    if (g >= a.n_gen) return;
    const int s = g >> 1, ch = g & 1;
    const IcwRenderK &k = a.rk;
    const int n = k.ns_n;
    double *rs = a.rs + (size_t)g * ICW_RSTATE;
    double prev_err = rs[1];
    /* rs keeps the history by age (0 = newest); the reference ring: ebuf[(pos + age) mod n] */
    double E[NM], O[NM];
    int pos = 0;                                         /* E age j at slot (pos + j) mod n, O age j at (pos - 1 + j) */
#pragma unroll 1
    for (int i = 0; i < NM; ++i) E[i] = O[i] = 0.0;
#pragma unroll 1
    for (int i = 0; i < n; ++i) { E[i] = rs[2 + i]; O[(i - 1 + n) % n] = rs[2 + NM + i]; }
    const double *pp = a.pre + (size_t)s * a.pre_stride + ch;
    const double *dp = a.dith ? a.dith + g : nullptr;
    unsigned char *op = a.out + (size_t)s * a.out_stride;
    const int osz = k.is24 ? 3 : 2;
    unsigned clips = 0;
    double pk = 0.0;
    IcwFes fe = {};
#pragma unroll 1
    for (int t = 0; t < a.T; ++t) {
        const double d = dp ? dp[(size_t)t * a.dith_pitch] : 0.0;
        const double input = icw_fc(icw_fc(pp[(size_t)t * 2] * k.norm_mul, fe) - prev_err, fe);
        int delta;
        double q = icw_fc(input + icw_fc(d, fe), fe);
        q = icw_fc(icw_round_q(q, k.round_offset, k.sign_delta, delta), fe);
        pk = fmax(pk, fabs(q));
        const int vc = icw_clamp_int(q, k, clips);
        const int val = (isnan(q) ? (int)0x80000000 : vc) + delta;
        const double ev = icw_fc((double)val - input, fe);
        double res = 0.0;
        if (k.ns_kind != 0) {
            pos = pos ? pos - 1 : n - 1;                 /* ns_ix_pos decrement (sound_render.c:410-413) */
            /* ages shift by one: the ring slot of age j is (pos + j) mod n */
            E[pos] = icw_fc(ev, fe);
            int ib = pos;
#pragma unroll 1
            for (int ic = 0; ic < n; ++ic) {
                if (k.ns_kind == 1) res = icw_fc(res + icw_fc(k.ns_c[ic] * E[ib], fe), fe);
                else res = icw_fc(res + icw_fc(icw_fc(k.ns_c[ic] * E[ib], fe) - icw_fc(k.ns_c[ic + n] * O[ib], fe), fe), fe);
                if (++ib >= n) ib = 0;
            }
            if (k.ns_kind == 2) O[(pos ? pos : n) - 1] = res;
        }
        prev_err = res;
        const int v = val << k.norm_shift;
        unsigned char *o = op + ((size_t)t * 2 + ch) * osz;
        o[0] = (unsigned char)v;
        o[1] = (unsigned char)(v >> 8);
        if (osz == 3) o[2] = (unsigned char)(v >> 16);
    }
    rs[1] = prev_err;
    /* back to the by-age layout: age j at slot (pos + j) mod n (E) and (pos - 1 + j) mod n (O: the
     * newest output sits one slot behind the newest error) */
    if (k.ns_kind != 0) {
        double e2[NM], o2[NM];
#pragma unroll 1
        for (int j = 0; j < n; ++j) { e2[j] = E[(pos + j) % n]; o2[j] = O[(pos - 1 + n + j) % n]; }
#pragma unroll 1
        for (int j = 0; j < n; ++j) { rs[2 + j] = e2[j]; rs[2 + NM + j] = o2[j]; }
    }
    if (clips) atomicAdd(&a.clips[g], clips);
    if (pk > 0.0) atomicMax(&a.peak_bits[g], (unsigned long long)__double_as_longlong(pk));
    icw_fes_flush(fe, a.fes + ((size_t)s * 4 + 2 + ch) * ICW_FES_PITCH);
}

/* ---------------------------------------------------------------- launch wrappers ------- */
extern "C" hipError_t icw_launch_unpack(const IcwK0Args *a, hipStream_t st)
{
    dim3 grid((a->T + 255) / 256, a->n_streams);
    hipLaunchKernelGGL(icw_unpack_frames, grid, dim3(256), a->lds_guard, st, *a);
    return hipGetLastError();
}

/* dynamic LDS of the FIR kernels: staged channels (padded), taps, Q, the DSP register file */
static size_t fir_lds(int M, int nt, int nchc, int tf, int n_regs)
{
    const int sh = (8 - ((M / 2 - 1) & 7)) & 7;
    const int nl = sh + M + tf + 24;
    const size_t px = (size_t)(nl + ICW_FIR_PAD * (nl >> 3) + 2) & ~(size_t)1;
    return ((size_t)nchc * px + (size_t)((nt + 1) & ~1) + (size_t)nchc * tf + (size_t)n_regs * 4 * ICW_K2_TILE) *
           sizeof(double);
}

static bool fir_ok(int M, int nt)
{
    return M >= 2 && M <= ICW_FIR_MAX_M && !(M & 1) && nt >= 1 && 2 * nt - 1 <= M / 2;
}

/* LDS above 64 KB per workgroup needs the kernel attribute (gfx950: 160 KB per CU) */
static hipError_t fir_lds_attr(const void *fn, size_t lds)
{
    return lds > 64 * 1024 ? hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) : hipSuccess;
}

extern "C" hipError_t icw_launch_fir(const IcwFirArgs *a, hipStream_t st)
{
    if (!fir_ok(a->M, a->nt)) return hipErrorInvalidValue;
    constexpr int TF = 256 * ICW_FIR_R;
    const size_t lds = fir_lds(a->M, a->nt, 1, TF, 0);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (fir_lds_attr((const void *)icw_fir_hilbert, lds) != hipSuccess) return hipErrorInvalidValue;
    dim3 grid((a->T + TF - 1) / TF, a->nch > 1 ? 2 : 1, a->n_streams);
    hipLaunchKernelGGL(icw_fir_hilbert, grid, dim3(256), lds, st, *a);
    return hipGetLastError();
}

/* bytes of dynamic LDS the fused converter needs (0: more than a workgroup may hold -- run KF + K2) */
extern "C" size_t icw_fir_graph_lds(int M, int nt, int nch, int n_regs)
{
    const int nchc = nch > 1 ? 2 : 1;
    const size_t lds = fir_lds(M, nt, nchc, 256 * ICW_FIR_R / nchc, n_regs) - (size_t)256 * ICW_FIR_R * sizeof(double);
    return lds <= 96 * 1024 ? lds : 0;
}

/* in_step: every stream of the launch is in step with the rotation table (a->trig_tab) */
template <int NC>
static hipError_t launch_fir_graph_nc(const IcwFirArgs *f, const IcwK2Args *a, int in_step, size_t lds, hipStream_t st)
{
    const int TF = 256 * ICW_FIR_R / NC;
    dim3 grid(f->n_streams, (f->T + TF - 1) / TF - f->tile0);  /* stream-fastest (icw_fir_graph); <= 1 024 tiles */
    const void *fn = !a->trig ? (const void *)icw_fir_graph<false, false, NC>
                   : in_step ? (const void *)icw_fir_graph<true, true, NC> : (const void *)icw_fir_graph<true, false, NC>;
    if (fir_lds_attr(fn, lds) != hipSuccess) return hipErrorInvalidValue;
    if (!a->trig) hipLaunchKernelGGL((icw_fir_graph<false, false, NC>), grid, dim3(256), lds, st, *f, *a);
    else if (in_step) hipLaunchKernelGGL((icw_fir_graph<true, true, NC>), grid, dim3(256), lds, st, *f, *a);
    else hipLaunchKernelGGL((icw_fir_graph<true, false, NC>), grid, dim3(256), lds, st, *f, *a);
    return hipGetLastError();
}

/* the signature form over tiles [0, ntile) of every stream */
template <int SIG, int NC, bool B24>
static hipError_t launch_fir_sig_t(const IcwFirArgs *f, const IcwK2Args *a, int ntile, size_t lds, hipStream_t st)
{
    const void *fn = (const void *)icw_fir_sig<SIG, NC, B24>;
    if (fir_lds_attr(fn, lds) != hipSuccess) return hipErrorInvalidValue;
    hipLaunchKernelGGL((icw_fir_sig<SIG, NC, B24>), dim3(f->n_streams, ntile), dim3(256), lds, st, *f, *a);
    return hipGetLastError();
}

template <int NC, bool B24>
static hipError_t launch_fir_sig_d(const IcwFirArgs *f, const IcwK2Args *a, int sig, int ntile, size_t lds,
                                   hipStream_t st)
{
    switch (sig) {
    case ICW_SIG_M:
    case ICW_SIG_M | ICW_SIG_UNIT: return launch_fir_sig_t<ICW_SIG_M | ICW_SIG_UNIT, NC, B24>(f, a, ntile, lds, st);
    case ICW_SIG_SM: return launch_fir_sig_t<ICW_SIG_SM, NC, B24>(f, a, ntile, lds, st);
    case ICW_SIG_SM | ICW_SIG_UNIT: return launch_fir_sig_t<ICW_SIG_SM | ICW_SIG_UNIT, NC, B24>(f, a, ntile, lds, st);
    case ICW_SIG_PSXM: return launch_fir_sig_t<ICW_SIG_PSXM, NC, B24>(f, a, ntile, lds, st);
    case ICW_SIG_PSXM | ICW_SIG_UNIT: return launch_fir_sig_t<ICW_SIG_PSXM | ICW_SIG_UNIT, NC, B24>(f, a, ntile, lds, st);
    default: return hipErrorInvalidValue;
    }
}

static bool fir_sig_known(int sig)
{
    switch (sig) {
    case ICW_SIG_M: case ICW_SIG_M | ICW_SIG_UNIT: case ICW_SIG_SM: case ICW_SIG_SM | ICW_SIG_UNIT:
    case ICW_SIG_PSXM: case ICW_SIG_PSXM | ICW_SIG_UNIT: return true;
    default: return false;
    }
}

extern "C" hipError_t icw_launch_fir_graph(const IcwFirArgs *f, const IcwK2Args *a, int in_step, hipStream_t st)
{
    if (!fir_ok(f->M, f->nt)) return hipErrorInvalidValue;
    /* the render-only form (icw_fast_render) takes the quantiser from sign_delta alone: mid-riser
     * (sign_delta -1, round_offset 0) or mid-tread (0, 0.5), the only pairs render_consts gives */
    if (a->rk.sign_delta != 0 ? (a->rk.sign_delta != -1 || a->rk.round_offset != 0.0) : a->rk.round_offset != 0.5)
        return hipErrorInvalidValue;
    const size_t lds = icw_fir_graph_lds(f->M, f->nt, f->nch, a->n_regs);
    if (!lds) return hipErrorInvalidValue;
    if (in_step && !(a->trig && a->trig_tab)) return hipErrorInvalidValue;
    const int nc = f->nch > 1 ? 2 : 1, TF = 256 * ICW_FIR_R / nc;
    IcwFirArgs fl = *f;
    fl.tile0 = 0;
    /* the signature form takes the tiles before the one holding the block's last frame when every
     * lane of them would take icw_chain_frames' render-only branch: a chain program of a known
     * signature, its rotation factors (if any) from the table, a render here, no pre-render doubles,
     * no I / Q hand-off, no dither rows.  ICW_FIR_SIG=0: icw_fir_graph for every tile (A/B). */
    const char *sig_env = getenv("ICW_FIR_SIG");
    const bool sig_on = !sig_env || atoi(sig_env) != 0;
    const int sig = f->sig;
    const bool rot = (sig & ~ICW_SIG_UNIT) != ICW_SIG_M;
    if (sig_on && ICW_CHAIN4 && fir_sig_known(sig) && (rot ? (a->trig && in_step) : !a->trig) && a->do_render &&
        !a->iq_out && !a->pre && !a->dith) {
        const int nsig = (f->T - 1) / TF;
        if (nsig > 0) {
            const bool b24 = a->rk.is24 != 0;
            const size_t ls = icw_fir_graph_lds(f->M, f->nt, f->nch, 0);   /* no DSP register file */
            const hipError_t e = nc == 2 ? (b24 ? launch_fir_sig_d<2, true>(f, a, sig, nsig, ls, st)
                                                : launch_fir_sig_d<2, false>(f, a, sig, nsig, ls, st))
                                         : (b24 ? launch_fir_sig_d<1, true>(f, a, sig, nsig, ls, st)
                                                : launch_fir_sig_d<1, false>(f, a, sig, nsig, ls, st));
            if (e != hipSuccess) return e;
            fl.tile0 = nsig;
        }
    }
    return nc == 2 ? launch_fir_graph_nc<2>(&fl, a, in_step, lds, st) : launch_fir_graph_nc<1>(&fl, a, in_step, lds, st);
}

template <int N, bool K>
static hipError_t launch_k2_t(IcwK2Args a, hipStream_t st)
{
    /* ICW_K2_TPW tiles per workgroup (the next window loads hide behind a tile's work, one meter
     * atomic per 1024 frames); a small launch (the one-stream drop-in: 576 frames) uses fewer
     * tiles per workgroup so that its tiles run side by side */
    int tpw = ICW_K2_TPW;
    while (tpw > 1 && (long)((a.T + ICW_K2_TILE * tpw - 1) / (ICW_K2_TILE * tpw)) * a.n_streams < 512) tpw >>= 1;
    a.tpw = tpw;
    const int span = ICW_K2_TILE * tpw;
    dim3 grid((a.T + span - 1) / span, a.n_streams);
    const size_t lds = (size_t)a.n_regs * 4 * ICW_K2_TILE * sizeof(double);
    if (a.fes && !a.cw) hipLaunchKernelGGL((icw_output<N, K, true, true>), grid, dim3(ICW_K2_TILE), lds, st, a);
    else if (a.trig) hipLaunchKernelGGL((icw_output<N, K, true>), grid, dim3(ICW_K2_TILE), lds, st, a);
    else hipLaunchKernelGGL((icw_output<N, K, false>), grid, dim3(ICW_K2_TILE), lds, st, a);
    return hipGetLastError();
}

template <int RT>
static hipError_t icw_launch_dither_t(const IcwK3Args *a, hipStream_t st)
{
    if (!a->wbuf) {                        /* the one-kernel K3a (ICW_DITHER=coop, A/B) */
        hipLaunchKernelGGL(icw_dither_coop<RT>, dim3(a->n_gen), dim3(64), 0, st, *a);
        return hipGetLastError();
    }
    constexpr int W = 2 * (RT == ICW_RENDER_GAUSS ? 12 : (RT == ICW_RENDER_TPDF ? 2 : 1));
    const int chunk = (int)std::min<size_t>((size_t)a->T, a->wcap / W);
    if (chunk <= 0) return hipErrorInvalidValue;
    for (int t0 = 0; t0 < a->T; t0 += chunk) {
        IcwK3Args c = *a;
        c.T = std::min(chunk, a->T - t0);
        c.dith = a->dith + (a->dith_gm ? (size_t)t0 : (size_t)t0 * a->dith_pitch);
        hipLaunchKernelGGL(icw_dith_twist, dim3(c.n_gen), dim3(64), 0, st, c, W);
        const long long tot = (long long)c.n_gen * c.T;
        hipLaunchKernelGGL(icw_dith_samples<RT>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, c);
        hipLaunchKernelGGL(icw_dith_fix<RT>, dim3(c.n_gen), dim3(64), 0, st, c);
    }
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_dither(const IcwK3Args *a, hipStream_t st)
{
    if (a->T <= 0) return hipSuccess;
    switch (a->rk.render_type) {
    case ICW_RENDER_RPDF: return icw_launch_dither_t<ICW_RENDER_RPDF>(a, st);
    case ICW_RENDER_TPDF: return icw_launch_dither_t<ICW_RENDER_TPDF>(a, st);
    case ICW_RENDER_STPDF: return icw_launch_dither_t<ICW_RENDER_STPDF>(a, st);
    case ICW_RENDER_GAUSS: return icw_launch_dither_t<ICW_RENDER_GAUSS>(a, st);
    default: return hipErrorInvalidValue;
    }
}

/* the lane-per-channel generator, kept for A/B timing (ICW_DITHER=lane) */
extern "C" hipError_t icw_launch_dither_lane(const IcwK3Args *a, hipStream_t st)
{
    const int blocks = (a->n_gen + 63) / 64;
    switch (a->rk.render_type) {
    case ICW_RENDER_RPDF: hipLaunchKernelGGL(icw_dither_gen<ICW_RENDER_RPDF>, dim3(blocks), dim3(64), 0, st, *a); break;
    case ICW_RENDER_TPDF: hipLaunchKernelGGL(icw_dither_gen<ICW_RENDER_TPDF>, dim3(blocks), dim3(64), 0, st, *a); break;
    case ICW_RENDER_STPDF: hipLaunchKernelGGL(icw_dither_gen<ICW_RENDER_STPDF>, dim3(blocks), dim3(64), 0, st, *a); break;
    case ICW_RENDER_GAUSS: hipLaunchKernelGGL(icw_dither_gen<ICW_RENDER_GAUSS>, dim3(blocks), dim3(64), 0, st, *a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int KIND, int NN, bool MR>
static void icw_launch_rr(const IcwK3Args *a, int rb, hipStream_t st)
{
    /* K3c (a companion wave beside the chain, 128 threads) or K3r (one wave).  ICW_K3C_LDS (A/B): dynamic
     * LDS bytes K3c reserves on top of its own, so that fewer other workgroups share its CUs */
    if (a->comp) {
        const char *e = getenv("ICW_K3C_LDS");
        size_t pad = e ? (size_t)atol(e) : 0;
        if (pad > 150 * 1024) pad = 150 * 1024;
        if (pad > 64 * 1024)
            (void)hipFuncSetAttribute((const void *)icw_render_rowc<KIND, NN, MR>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
        hipLaunchKernelGGL((icw_render_rowc<KIND, NN, MR>), dim3(rb), dim3(128), pad, st, *a);
    } else {
        hipLaunchKernelGGL((icw_render_row<KIND, NN, MR>), dim3(rb), dim3(64), 0, st, *a);
    }
}

template <bool MR>
static hipError_t icw_launch_render_row(const IcwK3Args *a, int rb, int nn, hipStream_t st)
{
    if (a->comp && a->dith && !a->dith_gm) return hipErrorInvalidValue;   /* K3c stages generator-major rows */
    if (a->rk.ns_kind == 0) {
        icw_launch_rr<0, 0, MR>(a, rb, st);
    } else if (a->rk.ns_kind == 1) {
        switch (nn) {
        case 5: icw_launch_rr<1, 5, MR>(a, rb, st); break;
        case 9: icw_launch_rr<1, 9, MR>(a, rb, st); break;
        case 15: icw_launch_rr<1, 15, MR>(a, rb, st); break;
        case 16: icw_launch_rr<1, 16, MR>(a, rb, st); break;
        case 20: icw_launch_rr<1, 20, MR>(a, rb, st); break;
        default: return hipErrorInvalidValue;
        }
    } else {
        if (nn != 4) return hipErrorInvalidValue;
        icw_launch_rr<2, 4, MR>(a, rb, st);
    }
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_render(const IcwK3Args *a, hipStream_t st)
{
    const int blocks = (a->n_gen + 63) / 64;
    if (a->fes) {
        hipLaunchKernelGGL(icw_render_fc, dim3(blocks), dim3(64), 0, st, *a);
        return hipGetLastError();
    }
    /* the tap counts of the canned shapers (sound_render.c:75-235): FIR 5, 9, 15, 16, 20; IIR 4 */
    const int nn = a->rk.ns_n;
    if (a->row) {
        const int rb = (a->n_gen + 3) / 4;          /* four channels (two streams) per wave */
        /* the quantiser as a template flag: mid-riser (sign_delta -1, round_offset 0) or mid-tread
         * (sign_delta 0, round_offset 0.5) -- render_consts gives no other pair */
        if (a->rk.sign_delta != 0 ? a->rk.round_offset != 0.0 : a->rk.round_offset != 0.5) return hipErrorInvalidValue;
        return a->rk.sign_delta ? icw_launch_render_row<true>(a, rb, nn, st) : icw_launch_render_row<false>(a, rb, nn, st);
    }
    if (a->rk.ns_kind == 0) {
        hipLaunchKernelGGL((icw_render_serial<0, 1, 0>), dim3(blocks), dim3(64), 0, st, *a);
    } else if (a->rk.ns_kind == 1) {
        switch (nn) {
        case 5: hipLaunchKernelGGL((icw_render_serial<1, ICW_MAX_NS_TAPS, 5>), dim3(blocks), dim3(64), 0, st, *a); break;
        case 9: hipLaunchKernelGGL((icw_render_serial<1, ICW_MAX_NS_TAPS, 9>), dim3(blocks), dim3(64), 0, st, *a); break;
        case 15: hipLaunchKernelGGL((icw_render_serial<1, ICW_MAX_NS_TAPS, 15>), dim3(blocks), dim3(64), 0, st, *a); break;
        case 16: hipLaunchKernelGGL((icw_render_serial<1, ICW_MAX_NS_TAPS, 16>), dim3(blocks), dim3(64), 0, st, *a); break;
        case 20: hipLaunchKernelGGL((icw_render_serial<1, ICW_MAX_NS_TAPS, 20>), dim3(blocks), dim3(64), 0, st, *a); break;
        default: return hipErrorInvalidValue;
        }
    } else {
        if (nn != 4) return hipErrorInvalidValue;
        hipLaunchKernelGGL((icw_render_serial<2, 4, 4>), dim3(blocks), dim3(64), 0, st, *a);
    }
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_output(const IcwK2Args *a, int nord, int kahan, hipStream_t st)
{
    switch (nord) {
    case 15: return kahan ? launch_k2_t<15, true>(*a, st) : launch_k2_t<15, false>(*a, st);
    case 18: return kahan ? launch_k2_t<18, true>(*a, st) : launch_k2_t<18, false>(*a, st);
    case 19: return kahan ? launch_k2_t<19, true>(*a, st) : launch_k2_t<19, false>(*a, st);
    case 20: return kahan ? launch_k2_t<20, true>(*a, st) : launch_k2_t<20, false>(*a, st);
    }
    return hipErrorInvalidValue;
}

extern "C" hipError_t icw_launch_trig_table(const IcwTrigArgs *a, hipStream_t st)
{
    hipLaunchKernelGGL(icw_trig_table, dim3((a->T + 255) / 256), dim3(256), a->lds_guard, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_graph_serial(const IcwK4Args *a, hipStream_t st)
{
    hipLaunchKernelGGL(icw_graph_serial, dim3((a->n_streams + 63) / 64), dim3(64), a->lds_guard, st, *a);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_s1_t(IcwS1Args a, hipStream_t st)
{
    a.k2.tpw = (a.k2.T + ICW_K2_TILE - 1) / ICW_K2_TILE;
    const size_t regs = (size_t)a.k2.n_regs * 4 * ICW_K2_TILE * sizeof(double);
    a.lpitch = (a.k2.T + N + 2) & ~1;
    a.rows_off = a.k2.n_regs * 4 * ICW_K2_TILE;
    const size_t rows = (size_t)4 * a.lpitch * sizeof(double) + 16;
    a.ovl = a.ovl && regs + rows <= ICW_S1_OVL_LDS;
    const size_t lds = regs + (a.ovl ? rows : 0);
    if (lds > 64 * 1024) {
        const hipError_t e = a.k2.trig ? hipFuncSetAttribute((const void *)icw_stream1<N, true>,
                                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
                                       : hipFuncSetAttribute((const void *)icw_stream1<N, false>,
                                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    if (a.k2.trig) hipLaunchKernelGGL((icw_stream1<N, true>), dim3(1), dim3(ICW_K2_TILE), lds, st, a);
    else hipLaunchKernelGGL((icw_stream1<N, false>), dim3(1), dim3(ICW_K2_TILE), lds, st, a);
    return hipGetLastError();
}

/* K5: one stream, one launch block of at most ICW_S1_MAX frames, real input, Kahan + reject (the
 * row recurrence), register-form graph, ROUND / flat render, no FP_CHECK -- the host checks */
extern "C" hipError_t icw_launch_stream1(const IcwS1Args *a, int nord, hipStream_t st)
{
    if (a->k0.T != a->k2.T || a->k1.T != a->k2.T || a->k2.T <= 0 || a->k2.T > ICW_S1_MAX || a->k2.n_streams != 1 ||
        a->k2.cw || a->k2.fes || a->k2.iq_out || !a->k2.do_render)
        return hipErrorInvalidValue;
    switch (nord) {
    case 15: return launch_s1_t<15>(*a, st);
    case 18: return launch_s1_t<18>(*a, st);
    case 19: return launch_s1_t<19>(*a, st);
    case 20: return launch_s1_t<20>(*a, st);
    }
    return hipErrorInvalidValue;
}

extern "C" hipError_t icw_launch_advance(const IcwAdvArgs *a, hipStream_t st)
{
    hipLaunchKernelGGL(icw_advance, dim3((a->n_streams + 63) / 64), dim3(64), a->lds_guard, st, *a);
    return hipGetLastError();
}
