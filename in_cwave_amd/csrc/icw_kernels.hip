/*
 * icw_kernels.hip -- gfx950 (CDNA4) kernels of the in_cwave Hilbert -> modulator -> render path.
 *
 * Built with `-ffp-contract=off` and no fast-math; every floating-point expression below keeps
 * the operand order of the reference so that results are bit-identical to the x86 SSE2 build
 * of in_cwave (IEEE binary64, round-to-nearest, no FMA contraction, denormals preserved).
 *
 * Kernel roles (DESIGN.md "Kernels"):
 *   icw_iir_state   one lane per DF-II chain (stream x channel x {I,Q} filter).  Runs the
 *                   serial part of iir_rp_process_kahan (hblpf.c:1017-1054) -- the loop-back
 *                   Kahan sum that produces the delay-line value w[n] -- with the delay line held
 *                   in VGPRs as a compile-time-rotated ring (unrolled by the filter order N).
 *                   Writes w[] per chain to HBM.  This is the latency-bound critical path.
 *   icw_output      one thread per frame.  Everything that is NOT on the recurrence: the output
 *                   Kahan sum y[n] = sum d_i z_i + d0*c_i z_i (hblpf.c:1029-1043) from the w
 *                   window (frame-parallel), the fs/4 un-mix (lpf_hilbert_quad.c:129-156), the
 *                   DSP graph (adv_modulator.c:637-751) and the elementwise render
 *                   (sound_render.c:691-809, ROUND/flat).  Coalesced tile loads via LDS.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/icw.h"
#include "icw_device.h"

#pragma clang fp contract(off)

/* diagnostic build only (tools/k1_probe.hip): s_memtime stamps of workgroup 0, lane 0 */
#ifdef ICW_STAMPS
__device__ unsigned long long icw_stamps[8][1024];
#define ICW_STAMP(k, n) do { if (blockIdx.x == 0 && lane == 0 && (n) < 1024) icw_stamps[k][n] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define ICW_STAMP(k, n) do { } while (0)
#endif

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
 *   I: {x, +0, -x, +0}   Q: {+0, -x, +0, x}   ==  k' = (k+f)&3: {x, +0, -x, +0}[k'] */
__device__ __forceinline__ double icw_filter_in(double x, unsigned kq)
{
    return kq == 0 ? x : (kq == 2 ? -x : 0.0);
}

/* ------------------------------------------------------------ IIR state kernel (K1) ----- */
/* One unrolled step of the loop-back sum for sample J of an N-block.  The delay line lives in
 * R[]: at step J the logical z_i (i = 0 most recent) is R[(J-1-i) mod N]; the new w is written
 * to R[J], overwriting the oldest value.  All indices are compile-time constants. */
template <int N, bool KAHAN, bool SUBN, int J>
__device__ __forceinline__ void icw_iir_step(double (&R)[N], double xin, const double (&pc)[20],
                                             unsigned &cnt)
{
    double S;
    if (KAHAN) {
        /* kahan_init(sample); i = 0 term first (hblpf.c:1017-1027) then i = 1..N-1 */
        double t0 = R[(J - 1 + N) % N] * pc[0];
        double C = 0.0, Y, T;
        S = xin;
        Y = t0 - C; T = S + Y; C = (T - S) - Y; S = T;
#pragma unroll
        for (int i = 1; i < N; ++i) {
            double ti = R[(J - 1 - i + 2 * N) % N] * pc[i];
            Y = ti - C; T = S + Y; C = (T - S) - Y; S = T;
        }
    } else {
        /* baseline: sum_i = sample; sum_i += z_k * c_i (hblpf.c:898-913) */
        S = xin;
#pragma unroll
        for (int i = 0; i < N; ++i) S += R[(J - 1 - i + 2 * N) % N] * pc[i];
    }
    if (SUBN) {
        /* fabs(sum) < is_subnorm_reject, a BOOL == 1 -> threshold 1.0 (hblpf.c:915, 1046) */
        const bool z = fabs(S) < 1.0;
        cnt += z ? 1u : 0u;
        S = z ? 0.0 : S;
    }
    R[J] = S;
}


template <int N, int J>
__device__ __forceinline__ void icw_store_hist(const double (&R)[N], double *hist, int g, int n_chains)
{
    /* after J steps of a block, logical z_i = R[(J-1-i) mod N] */
#pragma unroll
    for (int i = 0; i < N; ++i) hist[(size_t)g * ICW_HIST_PITCH + i] = R[(J - 1 - i + 2 * N) % N];
}

/* R[k] <- R[k+1 mod N]: one static rotation of the ring (moves only) */
template <int N>
__device__ __forceinline__ void icw_rotate1(double (&R)[N])
{
    const double r0 = R[0];
#pragma unroll
    for (int k = 0; k < N - 1; ++k) R[k] = R[k + 1];
    R[N - 1] = r0;
}

/* After `rem` (< N) steps the logical order is R[(rem-1-i) mod N].  Rotating left by rem
 * restores the block-start mapping R[(N-1-i)] without any runtime-indexed register access
 * (which the compiler would otherwise demote to scratch). */
template <int N>
__device__ __forceinline__ void icw_normalise_ring(double (&R)[N], int rem)
{
#pragma unroll
    for (int k = 1; k < N; ++k)
        if (k <= rem) icw_rotate1<N>(R);
}

template <int N, int J0, bool KAHAN, bool SUBN>
__device__ __forceinline__ void icw_block_steps(double (&R)[N], const double (&xv)[N],
                                                const double (&pc)[20], unsigned &cnt, int lim)
{
    if constexpr (J0 < N) {
        if (J0 < lim) {
            icw_iir_step<N, KAHAN, SUBN, J0>(R, xv[J0], pc, cnt);
            icw_block_steps<N, J0 + 1, KAHAN, SUBN>(R, xv, pc, cnt, lim);
        }
    }
}

/* full block of N steps; after step J consumes xv[J], refill it with the input N samples ahead
 * (rows are padded by >= N doubles, so the last block's look-ahead loads stay in bounds) */
template <int N, int J0, bool KAHAN, bool SUBN>
__device__ __forceinline__ void icw_block_steps_pf(double (&R)[N], double (&xv)[N], const double *xnext,
                                                   const double (&pc)[20], unsigned &cnt)
{
    if constexpr (J0 < N) {
        icw_iir_step<N, KAHAN, SUBN, J0>(R, xv[J0], pc, cnt);
        xv[J0] = xnext[J0];
        icw_block_steps_pf<N, J0 + 1, KAHAN, SUBN>(R, xv, xnext, pc, cnt);
    }
}

/* Input prep (K0): unpack + fade each frame once (xwave_unpack_csample, xwave_reader.c:908-1001)
 * and lay out every DF-II chain's own input sequence: the quadrature mix of hq_rp_process
 * (lpf_hilbert_quad.c:129-156) feeds the I filter {x, +0, -x, +0} and the Q filter {+0, -x, +0, x}
 * by sample phase.  Mono input feeds the right converter with the left value, exactly the
 * reference's reuse of `val` (xwave_reader.c:988).  Row g = s*4 + ch*2 + {0:I, 1:Q}. */
__global__ __launch_bounds__(256) void icw_unpack_frames(IcwK0Args a)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int s = blockIdx.y;
    if (t >= a.T) return;
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
    double v[2];
    v[0] = icw_unpack(fp, a.fmt);
    if (fd >= 0.0) v[0] *= fd;
    if (a.nch > 1) {
        v[1] = icw_unpack(fp + a.csz, a.fmt);
        if (fd >= 0.0) v[1] *= fd;
    } else {
        v[1] = v[0];
    }
    double *xs = a.xd + (size_t)s * 4 * a.x_pitch + t;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
        const unsigned k = (a.hq_phase[s * 2 + ch] + (unsigned)(a.t0 + t)) & 3u;
        xs[(size_t)(ch * 2 + 0) * a.x_pitch] = icw_filter_in(v[ch], k);
        xs[(size_t)(ch * 2 + 1) * a.x_pitch] = icw_filter_in(v[ch], (k + 1u) & 3u);
    }
}

template <int N>
__device__ __forceinline__ void icw_load_x(double (&xv)[N], const double *xp)
{
#pragma unroll
    for (int j = 0; j < N; ++j) xv[j] = xp[j];
}

template <int N, bool KAHAN, bool SUBN>
__global__ __launch_bounds__(64) void icw_iir_state(IcwK1Args a)
{
    const int g = blockIdx.x * 64 + threadIdx.x;
    if (g >= a.n_chains) return;
    const int s = g >> 2, c = (g >> 1) & 1, f = g & 1;
    const int n_chains = a.n_chains;
    double pc[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) pc[i] = a.pc[i];

    double R[N];
#pragma unroll
    for (int i = 0; i < N; ++i) R[N - 1 - i] = a.hist[(size_t)g * ICW_HIST_PITCH + i];

    if (f == 0 && c == 0) a.info_dup[s] = a.lr_equal[s];     /* this block's start (for K2) */
    const double *xp = a.xd + (size_t)g * a.x_pitch;
    double *wrow = a.w + (size_t)g * a.w_pitch;
    /* history rows [0, N): row j = z_{N-1-j} = R[j] */
#pragma unroll
    for (int j = 0; j < N; ++j) wrow[j] = R[j];

    const int T = a.T;
    unsigned cnt = 0;
    int t = 0;
    if (T >= N) {
        /* xv[j] holds the input of step j of the current block; right after a step consumes it the
         * same register is refilled with the next block's input, so loads run N samples ahead
         * with no register copies */
        double xv[N];
        icw_load_x<N>(xv, xp);
        for (; t + N <= T; t += N) {
            icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt);
            double *wo = wrow + N + t;
#pragma unroll
            for (int j = 0; j < N; ++j) wo[j] = R[j];
        }
    }
    const int rem = T - t;
    if (rem > 0) {
        double xv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) xv[j] = (j < rem) ? xp[t + j] : 0.0;
        icw_block_steps<N, 0, KAHAN, SUBN>(R, xv, pc, cnt, rem);
        double *wo = wrow + N + t;
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (j < rem) wo[j] = R[j];
        icw_normalise_ring<N>(R, rem);
    }
    icw_store_hist<N, 0>(R, a.hist, g, n_chains);
    a.sncnt[g] += cnt;
    /* are the stream's right converters still bit-identical to its left ones?  The 4 chains of a
     * stream are lanes 4k..4k+3 of this wave; lane ^ 2 is the same filter of the other channel */
    bool eq = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double o = __shfl_xor(R[i], 2);
        eq = eq && (__double_as_longlong(o) == __double_as_longlong(R[i]));
    }
    const bool eq_q = __shfl_xor((int)eq, 1) != 0;
    if (f == 0 && c == 0) a.lr_equal[s] = (eq && eq_q) ? 1u : 0u;
}

/* ---------------------------------------- IIR state kernel, chain+helper wave pair (K1p) ---- */
/* Latency/issue-bound regime (few chains per SIMD, e.g. BASELINE C2: 1024 chains on 1024 SIMDs).
 * A single wave issues ~1 FP64 instruction per ~4.7 cycles whether or not the instructions depend
 * on each other (tools/lat_probe), so a chain's time per sample is its instruction count.  The
 * workgroup pairs a CHAIN wave with a HELPER wave on another SIMD:
 *   chain : the loop-back Kahan sum (hblpf.c:1017-1046) -- the 4 products that depend on the
 *           newest / oldest states, the 73 dependent adds, the subnorm reject -- and nothing else;
 *   helper: every other product w[m]*c_i (i in [3, N-KT)), the Hilbert input selection, and the
 *           store of w[] to HBM; it publishes them through an LDS ring indexed by target sample.
 * Hand-off: the chain writes w[n] to wring and bumps chain_done; the helper bumps help_done once
 * w[m]'s products are in LDS.  Slot n needs help_done >= n-3; the chain checks the slot of sample
 * n+1 in the middle of sample n and prefetches it in two halves (after the entries are consumed),
 * so LDS latency is off the critical path and the helper has ~2 samples of slack. */
template <int N>
struct IcwPair {
    static constexpr int KT = (N >= 20) ? 2 : 1;   /* oldest products computed by the chain */
    static constexpr int RING = N - KT;            /* product slots, indexed by target % RING */
    static constexpr int NH = N - KT - 3;          /* helper products i in [3, N-KT) */
    static constexpr int NE = NH + 1;              /* + the filter input x_in (entry 0) */
    static constexpr int WR = 8;                   /* w hand-off ring */
    static constexpr int HALF = 7;                 /* entries [0,HALF) prefetched mid-sample */
    static constexpr int IMID = 3 + HALF - 1;      /* steps i < IMID consume entries < HALF */
};

__device__ __forceinline__ int icw_lds_ld(const int *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
/* blocking LDS poll issued by hand: the compiler's own atomic-load lowering placed a
 * vector-memory drain (s_waitcnt vmcnt(0)) at every poll-loop header, which would wait for the
 * helper's HBM prefetches each sample */
__device__ __forceinline__ int icw_poll(unsigned off)
{
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(off));
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void icw_lds_st(int *p, int v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int N, int J, int I>
__device__ __forceinline__ double icw_pair_prod(const double (&R)[N], const double (&pf)[IcwPair<N>::NE],
                                                const double (&pc)[20])
{
    using P = IcwPair<N>;
    if constexpr (I < 3 || I >= N - P::KT) return R[(J - 1 - I + 2 * N) % N] * pc[I];
    else return pf[1 + I - 3];
}

template <int N, bool KAHAN, int J, int I>
__device__ __forceinline__ void icw_pair_sum(double &S, double &C, const double (&R)[N],
                                             const double (&pf)[IcwPair<N>::NE], const double (&pc)[20], int I1)
{
    if constexpr (I < N) {
        if (I < I1) {
            const double t = icw_pair_prod<N, J, I>(R, pf, pc);
            if (KAHAN) {
                const double Y = t - C;
                const double T = S + Y;
                C = (T - S) - Y;
                S = T;
            } else {
                S += t;
            }
            icw_pair_sum<N, KAHAN, J, I + 1>(S, C, R, pf, pc, I1);
        }
    }
}

/* steps i in [I0, N) starting at template index I0 */
template <int N, bool KAHAN, int J, int I0>
__device__ __forceinline__ void icw_pair_range(double &S, double &C, const double (&R)[N],
                                               const double (&pf)[IcwPair<N>::NE], const double (&pc)[20], int I1)
{
    icw_pair_sum<N, KAHAN, J, I0>(S, C, R, pf, pc, I1);
}

struct IcwPairLds;   /* layout documented in icw_iir_pair */

template <int N, bool KAHAN, bool SUBN, int J>
__device__ __forceinline__ void icw_pair_sample(double (&R)[N], double (&pf)[IcwPair<N>::NE], const double (&pc)[20],
                                                unsigned &cnt, const int n, double *prod, double *wring,
                                                int *chain_done, const int *help_done, const int lane, int *err,
                                                const unsigned hd_off)
{
    using P = IcwPair<N>;
    /* The poll of help_done is issued by hand at the start of the sample and waited for by hand
     * in the middle, so its LDS latency hides under the first half of the Kahan chain.  (A plain
     * load would be sunk by the compiler to its use, with the first half of the sum moved below
     * the check -- an exposed LDS round trip every sample.)  Extra hand-issued LDS ops only make
     * the compiler's in-order lgkmcnt waits stronger, never weaker. */
    int pv;
    double S = pf[0], C = 0.0;
    ICW_STAMP(0, n);
    asm volatile("ds_read_b32 %0, %2" : "=v"(pv), "+v"(S) : "v"(hd_off));
    icw_pair_range<N, KAHAN, J, 0>(S, C, R, pf, pc, P::IMID);
    asm volatile("" : "+v"(S), "+v"(C));                       /* first half stays above the check */
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pv) : : "memory");
    /* mid-sample: slot n+1 must be complete (help_done >= n-2), then prefetch its first half
     * (x_in and products 3..IMID-1, whose registers were just consumed) */
    pv = __builtin_amdgcn_readfirstlane(pv);
    for (int spin = 0; pv < n - 2; ++spin) {          /* bounded: a broken hand-off ends the kernel */
        if (spin > (1 << 22)) { *err = 1; break; }
        __builtin_amdgcn_s_sleep(1);
        pv = icw_poll(hd_off);
    }
    ICW_STAMP(1, n);
    const double *slot = prod + (size_t)((n + 1) % P::RING) * P::NE * 64 + lane;
#pragma unroll
    for (int e = 0; e < P::HALF; ++e) pf[e] = slot[e * 64];
    icw_pair_range<N, KAHAN, J, P::IMID>(S, C, R, pf, pc, N);
    asm volatile("" : "+v"(S));                                 /* second half above its refill */
#pragma unroll
    for (int e = P::HALF; e < P::NE; ++e) pf[e] = slot[e * 64];
    if (SUBN) {
        const bool z = fabs(S) < 1.0;
        cnt += z ? 1u : 0u;
        S = z ? 0.0 : S;
    }
    R[J] = S;
    /* publish w[n]: LDS operations of one wave are performed in order, so the counter store
     * cannot overtake the data store; the asm barrier keeps the compiler from reordering them */
    wring[(n % P::WR) * 64 + lane] = S;
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (lane == 0) icw_lds_st(chain_done, n + 1);
    ICW_STAMP(2, n);
}

template <int N, bool KAHAN, bool SUBN, int J0>
__device__ __forceinline__ void icw_pair_block(double (&R)[N], double (&pf)[IcwPair<N>::NE], const double (&pc)[20],
                                               unsigned &cnt, const int n0, const int lim, double *prod, double *wring,
                                               int *chain_done, const int *help_done, const int lane, int *err,
                                               const unsigned hd_off)
{
    if constexpr (J0 < N) {
        if (J0 < lim) {
            icw_pair_sample<N, KAHAN, SUBN, J0>(R, pf, pc, cnt, n0 + J0, prod, wring, chain_done, help_done, lane, err,
                                                hd_off);
            icw_pair_block<N, KAHAN, SUBN, J0 + 1>(R, pf, pc, cnt, n0, lim, prod, wring, chain_done, help_done, lane,
                                                   err, hd_off);
        }
    }
}

template <int N, bool KAHAN, bool SUBN>
__global__ __launch_bounds__(128) void icw_iir_pair(IcwK1Args a)
{
    using P = IcwPair<N>;
    __shared__ double prod[P::RING * P::NE * 64];   /* [slot][entry][lane] */
    __shared__ double wring[P::WR * 64];             /* [n % WR][lane] */
    __shared__ int counters[2];                       /* chain_done, help_done */
    int *chain_done = &counters[0];
    int *help_done = &counters[1];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g0 = blockIdx.x * 64 + lane;
    const bool valid = g0 < a.n_chains;
    const int g = valid ? g0 : a.n_chains - 1;
    const int s = g >> 2, c = (g >> 1) & 1, f = g & 1;
    const int T = a.T;
    double pc[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) pc[i] = a.pc[i];
    if (threadIdx.x == 0) {
        icw_lds_st(chain_done, 0);
        icw_lds_st(help_done, -0x40000000);
    }
    __syncthreads();

    if (wave == 1) {
        /* ------------------------------- helper wave ------------------------------- */
        const double *xp = a.xd + (size_t)g * a.x_pitch;
        double *wrow = a.w + (size_t)g * a.w_pitch;
        double z[N];   /* z[k] = w[-1-k] (history, most recent first) */
#pragma unroll
        for (int k = 0; k < N; ++k) z[k] = a.hist[(size_t)g * ICW_HIST_PITCH + k];
        if (valid) {
#pragma unroll
            for (int j = 0; j < N; ++j) wrow[j] = z[N - 1 - j];
        }
        /* prefill: products of history w[m] (m = -1-k) for targets n = m+1+i = i-k >= 0 */
#pragma unroll
        for (int k = 0; k < N; ++k)
#pragma unroll
            for (int i = 3; i < N - P::KT; ++i) {
                const int n = i - k;
                if (n >= 0 && n < T) prod[((size_t)(n % P::RING) * P::NE + 1 + i - 3) * 64 + lane] = z[k] * pc[i];
            }
#pragma unroll
        for (int n = 0; n < 4; ++n)
            if (n < T) prod[((size_t)(n % P::RING) * P::NE) * 64 + lane] = xp[n];
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (lane == 0) icw_lds_st(help_done, 0);

        /* All HBM traffic of the helper happens at 16-sample group boundaries (filter inputs
         * read a group ahead into registers, the group's w[] written back as one 128-B run per
         * lane), and the per-sample hand-off is branch-free apart from the poll, so the loop
         * carries no vector-memory waits.  Products for targets >= T land in ring slots whose
         * previous targets are already consumed, so they are written unconditionally. */
        constexpr int U = 16;
        double xa[U], xb[U], wg[U];
#pragma unroll
        for (int u = 0; u < U; ++u) xa[u] = (4 + u < T) ? xp[4 + u] : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) xb[u] = (U + 4 + u < T) ? xp[U + 4 + u] : 0.0;
        int cd = 0;
        const unsigned cd_off = (unsigned)(uintptr_t)chain_done;
        for (int m0 = 0; m0 < T; m0 += U) {
            const int ulim = min(U, T - m0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int m = m0 + u;
                if (u < ulim) {
                    for (int spin = 0; cd < m + 1; ++spin) {
                        if (spin > (1 << 24)) { *a.err = 2; return; }
                        cd = icw_poll(cd_off);
                    }
                    ICW_STAMP(3, m);
                    const double w = wring[(m % P::WR) * 64 + lane];
                    wg[u] = w;
                    const int sb = (m + 4) % P::RING;   /* slot of target m+1+i for i = 3 */
                    double *pb = prod + lane;
#pragma unroll
                    for (int i = 3; i < N - P::KT; ++i) {
                        int sl = sb + (i - 3);
                        sl = sl >= P::RING ? sl - P::RING : sl;
                        pb[((size_t)sl * P::NE + 1 + i - 3) * 64] = w * pc[i];
                    }
                    pb[((size_t)sb * P::NE) * 64] = xa[u];
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    if (lane == 0) icw_lds_st(help_done, m + 1);
                    ICW_STAMP(4, m);
                }
            }
            if (valid) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (u < ulim) wrow[N + m0 + u] = wg[u];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) xa[u] = xb[u];
#pragma unroll
            for (int u = 0; u < U; ++u) xb[u] = (m0 + 2 * U + 4 + u < T) ? xp[m0 + 2 * U + 4 + u] : 0.0;
        }
        return;
    }

    /* ---------------------------------- chain wave ---------------------------------- */
    double R[N];
#pragma unroll
    for (int i = 0; i < N; ++i) R[N - 1 - i] = a.hist[(size_t)g * ICW_HIST_PITCH + i];
    for (int spin = 0; __builtin_amdgcn_readfirstlane(icw_lds_ld(help_done)) < 0; ++spin) {
        if (spin > (1 << 22)) { *a.err = 3; break; }
        __builtin_amdgcn_s_sleep(1);
    }
    double pf[P::NE];
#pragma unroll
    for (int e = 0; e < P::NE; ++e) pf[e] = prod[(size_t)e * 64 + lane];
    const unsigned hd_off = (unsigned)(uintptr_t)help_done;   /* LDS byte offset (flat low bits) */
    unsigned cnt = 0;
    int t = 0;
    for (; t + N <= T; t += N)
        icw_pair_block<N, KAHAN, SUBN, 0>(R, pf, pc, cnt, t, N, prod, wring, chain_done, help_done, lane, a.err, hd_off);
    const int rem = T - t;
    if (rem > 0) {
        icw_pair_block<N, KAHAN, SUBN, 0>(R, pf, pc, cnt, t, rem, prod, wring, chain_done, help_done, lane, a.err, hd_off);
        icw_normalise_ring<N>(R, rem);
    }
    if (!valid) return;
    icw_store_hist<N, 0>(R, a.hist, g, a.n_chains);
    a.sncnt[g] += cnt;
    if (f == 0 && c == 0) {   /* the pair kernel does not track converter identity: no shortcut */
        a.info_dup[s] = 0u;
        a.lr_equal[s] = 0u;
    }
}

/* ------------------------------------------------------------- output kernel (K2) ------- */
struct IcwLR { double lre, lim, rre, rim; };

/* output Kahan sum of iir_rp_process_kahan (hblpf.c:1029-1043) for the sample whose delay line
 * is z_i = win[N-1-i] (win = w[t-N .. t-1]); baseline form (hblpf.c:898-925) needs w[t]=win[N] */
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

__device__ __forceinline__ double icw_master(int tout, double re, double im)
{
    switch (tout) {
    case ICW_S_RE: return re;
    case ICW_S_IM: return im;
    case ICW_S_ADD_REIM: return (re + im) / ICW_SQRT2;
    case ICW_S_SUB_REIM: return (re - im) / ICW_SQRT2;
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

/* rotate (re,im) by e^{j phi} given cos/sin (adv_modulator.c:546-547, 576-577) */
__device__ __forceinline__ void icw_rot(double re, double im, double cs, double sn, double &ore, double &oim)
{
    ore = re * cs - im * sn;
    oim = re * sn + im * cs;
}

/* sound_render_value for ROUND render + flat shaper (sound_render.c:691-809): elementwise */
__device__ __forceinline__ int icw_render_round(double input, const IcwRenderK &k, unsigned &clips, double &pk)
{
    input = (input * k.norm_mul) - 0.0;           /* prev_ns_err == 0.0 for the flat shaper */
    double q = input + (0.0 * k.dth_mul);         /* rnd_dth == 0.0 for ROUND */
    int delta;
    if (q < 0.0) { q -= k.round_offset; delta = k.sign_delta; }
    else { q += k.round_offset; delta = 0; }
    const double aq = fabs(q);
    pk = aq > pk ? aq : pk;
    if (q >= k.hi) { q = k.hi - 1.0; ++clips; }
    if (q <= k.lo) { q = k.lo + 1.0; ++clips; }
    /* x86 cvttsd2si semantics: NaN -> INT_MIN ("integer indefinite") */
    int v = isnan(q) ? (int)0x80000000 : (int)q;
    return (v + delta) << k.norm_shift;
}

/* modulator frame counter -> norm_omega of frame t of the block (adv_modulator.c:611-625);
 * n0 is the block-start counter (< ssr in scaled mode) */
__device__ __forceinline__ double icw_omega(unsigned long long n0, long long t, int scaled, unsigned long long ssr,
                                            uint32_t sample_rate)
{
    /* n0: the counter at the call's start (< ssr when scaled); t: frames since then */
    if (scaled) {
        const unsigned long long n = (n0 + (unsigned long long)t) % ssr;
        return (2.0 * ICW_PI) * ((double)n) / ((double)ssr);
    }
    return (2.0 * ICW_PI) * ((double)(n0 + (unsigned long long)t)) / (double)sample_rate;
}

/* One DSP node on its mixed input d (adv_modulator.c:669-751): channel exchange, I/Q swap,
 * gains, then Master (-> lOut/rOut) or Shift / PM / Mix (-> o, returns true). */
__device__ __forceinline__ bool icw_exec_op(const IcwOp &op, IcwLR d, double omega, IcwLR &o, double &lOut,
                                            double &rOut)
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
    case ICW_MODE_SHIFT: {
        double cs, sn;
        if (op.act[0]) {
            const double ph = fmod(omega * op.f[0], 2.0 * ICW_PI);
            sincos(ph, &sn, &cs);
            if (op.neg[0]) sn = -sn;
            icw_rot(d.lre, d.lim, cs, sn, o.lre, o.lim);
        } else { o.lre = d.lre; o.lim = d.lim; }
        if (op.act[1]) {
            const double ph = fmod(omega * op.f[1], 2.0 * ICW_PI);
            sincos(ph, &sn, &cs);
            if (op.neg[1]) sn = -sn;
            icw_rot(d.rre, d.rim, cs, sn, o.rre, o.rim);
        } else { o.rre = d.rre; o.rim = d.rim; }
        return true;
    }
    case ICW_MODE_PM: {
        double cs, sn;
        if (op.act[0]) {
            const double ph = fmod(omega * op.f[0], 2.0 * ICW_PI);
            const double psi = op.lp[0] * (sin(ph + op.pp[0]) + op.fa[0]);
            sincos(psi, &sn, &cs);
            icw_rot(d.lre, d.lim, cs, sn, o.lre, o.lim);
        } else { o.lre = d.lre; o.lim = d.lim; }
        if (op.act[1]) {
            const double ph = fmod(omega * op.f[1], 2.0 * ICW_PI);
            const double psi = op.lp[1] * (sin(ph + op.pp[1]) + op.fa[1]);
            sincos(psi, &sn, &cs);
            icw_rot(d.rre, d.rim, cs, sn, o.rre, o.rim);
        } else { o.rre = d.rre; o.rim = d.rim; }
        return true;
    }
    default: /* MIX */
        o = d;
        return true;
    }
}

template <int N, bool KAHAN>
__global__ __launch_bounds__(ICW_K2_TILE) void icw_output(IcwK2Args a)
{
    __shared__ double lw[4][ICW_K2_TILE + 24];
    extern __shared__ __attribute__((aligned(16))) double lregs[];   /* [n_regs][4][ICW_K2_TILE] */
    __shared__ unsigned red_clip[2][ICW_K2_TILE / 64];
    __shared__ double red_pk[2][ICW_K2_TILE / 64];
    const int s = blockIdx.y;
    const int t0 = blockIdx.x * ICW_K2_TILE;
    const int tl = threadIdx.x;
    const int t = t0 + tl;
    const int T = a.T;

    if (!a.cw) {
        /* stage the w windows of the stream's 4 chains: rows [t0, t0+nrow) */
        const int nrow = min(ICW_K2_TILE, T - t0) + N + (KAHAN ? 0 : 1);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double *src = a.w + (size_t)(s * 4 + c) * a.w_pitch + t0;
            for (int r = tl; r < nrow; r += ICW_K2_TILE) lw[c][r] = src[r];
        }
        __syncthreads();
    }

    unsigned clip_l = 0, clip_r = 0;
    double pk_l = 0.0, pk_r = 0.0;
    if (t < T) {
        IcwLR in;
        if (a.cw) {
            /* complex (CWAVE) input: the analytic signal as read (xwave_reader.c:939-966) */
            const double *xs = a.xin + (size_t)s * 4 * a.x_pitch + t;
            in.lre = xs[0]; in.lim = xs[a.x_pitch]; in.rre = xs[2 * a.x_pitch]; in.rim = xs[3 * a.x_pitch];
        } else {
            double pc[20], pd[20];
#pragma unroll
            for (int i = 0; i < 20; ++i) { pc[i] = a.pc[i]; pd[i] = a.pd[i]; }
            /* filter outputs of the 4 chains (L-I, L-Q, R-I, R-Q); the right pair is a copy when the
             * converters are provably identical this block (mono, equal state: K0's flag) */
            double y[4];
            y[0] = icw_iir_out<N, KAHAN>(&lw[0][tl], pc, pd, a.d0);
            y[1] = icw_iir_out<N, KAHAN>(&lw[1][tl], pc, pd, a.d0);
            if (a.nch == 1 && a.info_dup && a.info_dup[s] && a.hq_phase[s * 2] == a.hq_phase[s * 2 + 1]) {
                y[2] = y[0];
                y[3] = y[1];
            } else {
                y[2] = icw_iir_out<N, KAHAN>(&lw[2][tl], pc, pd, a.d0);
                y[3] = icw_iir_out<N, KAHAN>(&lw[3][tl], pc, pd, a.d0);
            }

            /* fs/4 un-mix (lpf_hilbert_quad.c:129-156) */
            double oI[2], oQ[2];
#pragma unroll
            for (int ch = 0; ch < 2; ++ch) {
                const double yi = y[ch * 2], yq = y[ch * 2 + 1];
                const unsigned k = (a.hq_phase[s * 2 + ch] + (unsigned)(a.t0 + t)) & 3u;
                switch (k) {
                case 0: oI[ch] = yi * 2.0; oQ[ch] = yq * 2.0; break;
                case 1: oI[ch] = -yq * 2.0; oQ[ch] = yi * 2.0; break;
                case 2: oI[ch] = -yi * 2.0; oQ[ch] = -yq * 2.0; break;
                default: oI[ch] = yq * 2.0; oQ[ch] = -yi * 2.0; break;
                }
            }
            in.lre = oI[0]; in.lim = oQ[0]; in.rre = oI[1]; in.rim = oQ[1];
        }

        if (a.iq_out) {
            /* bus-form graph: the serial graph kernel takes it from here */
            double *q = a.iq_out + ((size_t)s * T + t) * 4;
            q[0] = in.lre; q[1] = in.lim; q[2] = in.rre; q[3] = in.rim;
            return;   /* do_render == 0 in this mode: no barrier follows */
        }

        const double omega = icw_omega(a.n_frame[s], a.t0 + t, a.scaled, a.ssr, a.sample_rate);

        /* DSP list (adv_modulator.c:637-751) */
        const IcwProg *P = a.prog;
        IcwRegFile R;
        R.base = lregs + tl;
        R.set(0, in);
        for (int r = 0; r < P->n_persist; ++r) {
            const double *b = a.bus + ((size_t)s * ICW_N_INPUTS + P->persist_slot[r]) * 4;
            IcwLR v; v.lre = b[0]; v.lim = b[1]; v.rre = b[2]; v.rim = b[3];
            R.set(P->persist_reg[r], v);
        }
        double lOut = 0.0, rOut = 0.0;
        for (int oi = 0; oi < P->n_ops; ++oi) {
            const IcwOp &op = P->ops[oi];
            IcwLR d;
            if (P->bypass) {
                d = in;
            } else {
                d.lre = d.lim = d.rre = d.rim = 0.0;
                for (int k = 0; k < op.n_in; ++k) {
                    IcwLR v;
                    R.get(op.in_reg[k], v);
                    d.lre += v.lre; d.lim += v.lim; d.rre += v.rre; d.rim += v.rim;
                }
            }
            IcwLR o;
            if (icw_exec_op(op, d, omega, o, lOut, rOut)) R.set(op.out_reg, o);
        }

        if (a.pre) {
            double *p = a.pre + (size_t)s * a.pre_stride + (size_t)t * 2;
            p[0] = lOut; p[1] = rOut;
        }
        if (a.do_render) {
            const int vl = icw_render_round(lOut, a.rk, clip_l, pk_l);
            const int vr = icw_render_round(rOut, a.rk, clip_r, pk_r);
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
        /* persistent bus write-back from the block's last frame */
        if (t == T - 1) {
            double *b0 = a.bus + (size_t)s * ICW_N_INPUTS * 4;
            b0[0] = in.lre; b0[1] = in.lim; b0[2] = in.rre; b0[3] = in.rim;
            for (int k = 0; k < P->n_wb; ++k) {
                IcwLR v;
                R.get(P->wb_reg[k], v);
                double *b = b0 + P->wb_slot[k] * 4;
                b[0] = v.lre; b[1] = v.lim; b[2] = v.rre; b[3] = v.rim;
            }
        }
    }

    if (a.do_render) {
        /* per-workgroup meters: wave reduce, LDS, one atomic per stream/channel */
        for (int off = 32; off > 0; off >>= 1) {
            clip_l += __shfl_xor(clip_l, off);
            clip_r += __shfl_xor(clip_r, off);
            pk_l = fmax(pk_l, __shfl_xor(pk_l, off));
            pk_r = fmax(pk_r, __shfl_xor(pk_r, off));
        }
        const int wv = tl >> 6;
        if ((tl & 63) == 0) {
            red_clip[0][wv] = clip_l; red_clip[1][wv] = clip_r;
            red_pk[0][wv] = pk_l; red_pk[1][wv] = pk_r;
        }
        __syncthreads();
        if (tl < 2) {
            unsigned cs = 0; double pm = 0.0;
            for (int i = 0; i < ICW_K2_TILE / 64; ++i) { cs += red_clip[tl][i]; pm = fmax(pm, red_pk[tl][i]); }
            if (cs) atomicAdd(&a.clips[s * 2 + tl], cs);
            if (pm > 0.0) atomicMax(&a.peak_bits[s * 2 + tl], (unsigned long long)__double_as_longlong(pm));
        }
    }
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
    const IcwProg *P = a.prog;
    const unsigned long long n0 = a.n_frame[s];
    const double *iq = a.iq + (size_t)s * a.T * 4;
    double *pre = a.pre + (size_t)s * a.pre_stride;
    for (int t = 0; t < a.T; ++t) {
        const double omega = icw_omega(n0, a.t0 + t, a.scaled, a.ssr, a.sample_rate);
        bus[0][lane] = iq[(size_t)t * 4 + 0];
        bus[1][lane] = iq[(size_t)t * 4 + 1];
        bus[2][lane] = iq[(size_t)t * 4 + 2];
        bus[3][lane] = iq[(size_t)t * 4 + 3];
        double lOut = 0.0, rOut = 0.0;
        for (int oi = 0; oi < P->n_ops; ++oi) {
            const IcwOp &op = P->ops[oi];
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
__global__ __launch_bounds__(64) void icw_advance(IcwAdvArgs a)
{
    const int s = blockIdx.x * 64 + threadIdx.x;
    if (s >= a.n_streams) return;
    a.pos[s] += a.n;
    if (!a.cw) {
        a.hq_phase[s * 2 + 0] = (a.hq_phase[s * 2 + 0] + (unsigned)a.n) & 3u;
        a.hq_phase[s * 2 + 1] = (a.hq_phase[s * 2 + 1] + (unsigned)a.n) & 3u;
    }
    const unsigned long long n0 = a.n_frame[s];
    a.n_frame[s] = a.scaled ? (n0 + (unsigned long long)a.n) % a.ssr : n0 + (unsigned long long)a.n;
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
    double *dd = a.dith + g;            /* time-major [t][dith_pitch]: one store per sample is coalesced */
    const size_t dp = a.dith_pitch;
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

template <int RT>
__global__ __launch_bounds__(64) void icw_dither_coop(IcwK3Args a)
{
    constexpr int V = RT == ICW_RENDER_GAUSS ? 12 : (RT == ICW_RENDER_TPDF ? 2 : 1);
    __shared__ uint32_t mt[624];
    __shared__ uint32_t tw[626];           /* the window's word list: [carried word] + tempered mt[idx..623] */
    __shared__ double vals[313 + 16];      /* [carried values] + the window's accepted values */
    __shared__ short pidx[313];            /* pair index of each accepted value of the window */
    const int lane = threadIdx.x;
    const int g = blockIdx.x;              /* one wave per generator: everything below is wave-uniform */
    for (int i = lane; i < 624; i += 64) mt[i] = a.mt[(size_t)i * a.mt_pitch + g];
    int idx = a.mt_idx[g];
    double *rs = a.rs + (size_t)g * ICW_RSTATE;
    double prev_rnd = rs[0];
    const double dth_mul = a.rk.dth_mul;
    double *dd = a.dith + g;
    const size_t dp = a.dith_pitch;
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
    if (q < 0.0) { q -= k.round_offset; delta = k.sign_delta; }
    else { q += k.round_offset; delta = 0; }
    const double aq = fabs(q);
    pk = aq > pk ? aq : pk;
    if (q >= k.hi) { q = k.hi - 1.0; ++clips; }
    if (q <= k.lo) { q = k.lo + 1.0; ++clips; }
    int val = (isnan(q) ? (int)0x80000000 : (int)q) + delta;
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

/* ---------------------------------------------------------------- launch wrappers ------- */
template <int N, bool K, bool S>
static hipError_t launch_k1_t(const IcwK1Args &a, hipStream_t st)
{
    const int blocks = (a.n_chains + 63) / 64;
    hipLaunchKernelGGL((icw_iir_state<N, K, S>), dim3(blocks), dim3(64), 0, st, a);
    return hipGetLastError();
}

template <int N, bool K, bool S>
static hipError_t launch_k1p_t(const IcwK1Args &a, hipStream_t st)
{
    const int blocks = (a.n_chains + 63) / 64;
    hipLaunchKernelGGL((icw_iir_pair<N, K, S>), dim3(blocks), dim3(128), 0, st, a);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_k1p_n(const IcwK1Args &a, bool kahan, bool subn, hipStream_t st)
{
    if (kahan) return subn ? launch_k1p_t<N, true, true>(a, st) : launch_k1p_t<N, true, false>(a, st);
    return subn ? launch_k1p_t<N, false, true>(a, st) : launch_k1p_t<N, false, false>(a, st);
}

extern "C" hipError_t icw_launch_iir_pair(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st)
{
    switch (nord) {
    case 15: return launch_k1p_n<15>(*a, kahan, subn, st);
    case 18: return launch_k1p_n<18>(*a, kahan, subn, st);
    case 19: return launch_k1p_n<19>(*a, kahan, subn, st);
    case 20: return launch_k1p_n<20>(*a, kahan, subn, st);
    }
    return hipErrorInvalidValue;
}

template <int N>
static hipError_t launch_k1_n(const IcwK1Args &a, bool kahan, bool subn, hipStream_t st)
{
    if (kahan) return subn ? launch_k1_t<N, true, true>(a, st) : launch_k1_t<N, true, false>(a, st);
    return subn ? launch_k1_t<N, false, true>(a, st) : launch_k1_t<N, false, false>(a, st);
}

extern "C" hipError_t icw_launch_unpack(const IcwK0Args *a, hipStream_t st)
{
    dim3 grid((a->T + 255) / 256, a->n_streams);
    hipLaunchKernelGGL(icw_unpack_frames, grid, dim3(256), 0, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_iir_state(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st)
{
    switch (nord) {
    case 15: return launch_k1_n<15>(*a, kahan, subn, st);
    case 18: return launch_k1_n<18>(*a, kahan, subn, st);
    case 19: return launch_k1_n<19>(*a, kahan, subn, st);
    case 20: return launch_k1_n<20>(*a, kahan, subn, st);
    }
    return hipErrorInvalidValue;
}

template <int N, bool K>
static hipError_t launch_k2_t(const IcwK2Args &a, hipStream_t st)
{
    dim3 grid((a.T + ICW_K2_TILE - 1) / ICW_K2_TILE, a.n_streams);
    const size_t lds = (size_t)a.n_regs * 4 * ICW_K2_TILE * sizeof(double);
    hipLaunchKernelGGL((icw_output<N, K>), grid, dim3(ICW_K2_TILE), lds, st, a);
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_dither(const IcwK3Args *a, hipStream_t st)
{
    const int blocks = a->n_gen;           /* one wave per render channel */
    switch (a->rk.render_type) {
    case ICW_RENDER_RPDF: hipLaunchKernelGGL(icw_dither_coop<ICW_RENDER_RPDF>, dim3(blocks), dim3(64), 0, st, *a); break;
    case ICW_RENDER_TPDF: hipLaunchKernelGGL(icw_dither_coop<ICW_RENDER_TPDF>, dim3(blocks), dim3(64), 0, st, *a); break;
    case ICW_RENDER_STPDF: hipLaunchKernelGGL(icw_dither_coop<ICW_RENDER_STPDF>, dim3(blocks), dim3(64), 0, st, *a); break;
    case ICW_RENDER_GAUSS: hipLaunchKernelGGL(icw_dither_coop<ICW_RENDER_GAUSS>, dim3(blocks), dim3(64), 0, st, *a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
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

extern "C" hipError_t icw_launch_render(const IcwK3Args *a, hipStream_t st)
{
    const int blocks = (a->n_gen + 63) / 64;
    /* the tap counts of the canned shapers (sound_render.c:75-235): FIR 5, 9, 15, 16, 20; IIR 4 */
    const int nn = a->rk.ns_n;
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

extern "C" hipError_t icw_launch_graph_serial(const IcwK4Args *a, hipStream_t st)
{
    hipLaunchKernelGGL(icw_graph_serial, dim3((a->n_streams + 63) / 64), dim3(64), 0, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_advance(const IcwAdvArgs *a, hipStream_t st)
{
    hipLaunchKernelGGL(icw_advance, dim3((a->n_streams + 63) / 64), dim3(64), 0, st, *a);
    return hipGetLastError();
}
