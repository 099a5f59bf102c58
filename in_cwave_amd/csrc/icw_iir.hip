/*
 * icw_iir.hip -- gfx950 (CDNA4) kernels of the serial IIR recurrence (K1 and its variants).
 *
 * Built with `-ffp-contract=off` and no fast-math: the loop-back sum keeps the operand order of
 * iir_rp_process_kahan / iir_rp_process_baseline (hblpf.c:894-953, 1008-1099) bit for bit.
 *
 *   icw_iir_state     one lane per DF-II chain (stream x channel x {I,Q} filter); the delay line
 *                     is a VGPR ring rotated at compile time (unrolled by the filter order N).
 *   icw_iir_state_fc  the FP_CHECK variant (FC() arithmetic and census).
 *   icw_iir_row       one 16-lane DPP row per chain: the products lane-parallel (small batches).
 *
 * Two slower experiments (MFMA product feed, chain + helper wave pair) are archived, not built
 * into the library: tools/k1_experimental.hip.
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

#include "icw_iir_dev.h"


/* One unrolled step of the loop-back sum for sample J of an N-block.  The delay line lives in
 * R[]: at step J the logical z_i (i = 0 most recent) is R[(J-1-i) mod N]; the new w is written
 * to R[J], overwriting the oldest value.  All indices are compile-time constants. */
template <int N, bool KAHAN, bool SUBN, int J, bool SPEC = false>
__device__ __forceinline__ void icw_iir_step(double (&R)[N], double xin, const double (&pc)[20],
                                             unsigned &cnt, double *mn = nullptr)
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
    if constexpr (SPEC) {
        *mn = icw_minabs(*mn, S);                /* the reject speculated away ("Speculative blocks") */
    } else if (SUBN) {
        /* fabs(sum) < is_subnorm_reject, a BOOL == 1 -> threshold 1.0 (hblpf.c:915, 1046) */
        const bool z = fabs(S) < 1.0;
        cnt += z ? 1u : 0u;
        S = z ? 0.0 : S;
    }
    R[J] = S;
}



/* generic steps (every input read, the zero ones supplied by icw_chain_x; qodd: the block starts
 * on an odd (phi + t), see icw_chain_x) */
template <int N, int J0, bool KAHAN, bool SUBN>
__device__ __forceinline__ void icw_block_steps(double (&R)[N], const double (&xv)[N],
                                                const double (&pc)[20], unsigned &cnt, int lim, bool qodd)
{
    if constexpr (J0 < N) {
        if (J0 < lim) {
            icw_iir_step<N, KAHAN, SUBN, J0>(R, icw_chain_x<J0>(xv[J0], qodd), pc, cnt);
            icw_block_steps<N, J0 + 1, KAHAN, SUBN>(R, xv, pc, cnt, lim, qodd);
        }
    }
}


template <int N, int J0, bool KAHAN, bool SUBN, bool SPEC = false>
__device__ __forceinline__ void icw_block_steps_pf(double (&R)[N], double (&xv)[N], const double *xnext,
                                                   const double (&pc)[20], unsigned &cnt, bool qodd,
                                                   double *mn = nullptr)
{
    if constexpr (J0 < N) {
        icw_iir_step<N, KAHAN, SUBN, J0, SPEC>(R, icw_chain_x<J0>(xv[J0], qodd), pc, cnt, mn);
        xv[J0] = xnext[J0];
        icw_block_steps_pf<N, J0 + 1, KAHAN, SUBN, SPEC>(R, xv, xnext, pc, cnt, qodd, mn);
    }
}

/* Zero-input step (Kahan, subnorm reject on).  Every other sample of a chain's input is the
 * literal +0.0 of hq_rp_process (lpf_hilbert_quad.c:136-151).  With sample = +0:
 *   kahan_init(+0): S = +0, C = 0;  i = 0: Y = t0, T = +0 + t0, C = (T - 0) - t0 = +0, S = T;
 *   i = 1: Y = t1 - (+0) = t1.
 * So S = t0 and C = +0 after step 0, and step 1's Y is t1: 4 adds fewer.  S can differ from the
 * reference only in the sign of a zero (t0 = -0 gives T = +0); a zero's sign is absorbed by the
 * first nonzero term, and a sum that stays zero is rejected to +0.0 (|S| < 1, hblpf.c:1046), so
 * w is bit-identical.  (With the reject off the sign would survive: that mode takes icw_iir_step.) */
template <int N, int J, bool SPEC = false>
__device__ __forceinline__ void icw_iir_step_z(double (&R)[N], const double (&pc)[20], unsigned &cnt,
                                               double *mn = nullptr)
{
    double S = R[(J - 1 + N) % N] * pc[0];
    double C, Y, T;
    Y = R[(J - 2 + 2 * N) % N] * pc[1];
    T = S + Y; C = (T - S) - Y; S = T;
#pragma unroll
    for (int i = 2; i < N; ++i) {
        const double ti = R[(J - 1 - i + 2 * N) % N] * pc[i];
        Y = ti - C; T = S + Y; C = (T - S) - Y; S = T;
    }
    if constexpr (SPEC) {
        *mn = icw_minabs(*mn, S);
    } else {
        const bool z = fabs(S) < 1.0;
        cnt += z ? 1u : 0u;
        S = z ? 0.0 : S;
    }
    R[J] = S;
}

/* A block of N steps whose input is zero at the steps J with (J & 1) == Z; the look-ahead refill
 * of xv[J] happens where the NEXT block's step J consumes an input (its zero parity ZN: the other
 * one for odd N, the same one for even N) */
template <int N, int J0, int Z, bool SUBN, bool SPEC = false, int ZN = 1 - Z>
__device__ __forceinline__ void icw_block_steps_zpf(double (&R)[N], double (&xv)[N], const double *xnext,
                                                    const double (&pc)[20], unsigned &cnt, double *mn = nullptr)
{
    if constexpr (J0 < N) {
        if constexpr ((J0 & 1) == Z) icw_iir_step_z<N, J0, SPEC>(R, pc, cnt, mn);
        else icw_iir_step<N, true, SUBN, J0, SPEC>(R, xv[J0], pc, cnt, mn);
        if constexpr ((J0 & 1) != ZN) xv[J0] = xnext[J0];
        icw_block_steps_zpf<N, J0 + 1, Z, SUBN, SPEC, ZN>(R, xv, xnext, pc, cnt, mn);
    }
}

/* even orders: every block of N (even) steps has the same zero steps, (J & 1) == Z; speculative
 * blocks first, then (after a block whose smallest |sum| fell below 1) the exact ones from its start */
template <int N, int Z, bool SUBN>
__device__ __forceinline__ void icw_even_blocks(double (&R)[N], double (&xv)[N], const double *xp, double *wrow,
                                                const double (&pc)[20], unsigned &cnt, int &t, int T)
{
    double mn = __builtin_inf();
    bool fail = false;
    ICW_DRAIN_VMEM();
    while (!fail && t + N <= T) {
        icw_block_steps_zpf<N, 0, Z, SUBN, true, Z>(R, xv, xp + t + N, pc, cnt, &mn);
        icw_store_block<N>(R, wrow + N + t);
        fail = __any(mn < 1.0);
        if (!fail) t += N;
    }
    if (fail) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll
        for (int j = 0; j < N; ++j) R[j] = wrow[t + j];
        icw_load_x<N>(xv, xp + t);
        ICW_DRAIN_VMEM();
        for (; t + N <= T; t += N) {
            icw_block_steps_zpf<N, 0, Z, SUBN, false, Z>(R, xv, xp + t + N, pc, cnt);
            icw_store_block<N>(R, wrow + N + t);
        }
    }
    icw_load_x<N>(xv, xp + t);   /* the zero steps left part of xv unloaded */
}


/* Speculative blocks (icw_iir_state, icw_iir_row): the loop-back sums run without the
 * reject's compare-and-select (hblpf.c:1046), i.e. w = S, which is exact unless some |S| < 1.  The
 * smallest |S| is checked once per loop iteration (a pair of blocks for odd orders); if any chain
 * of the wave fell below 1, the wave drops the iteration and runs the rest of the launch with the
 * exact steps, starting from the iteration's start state: the ring is the N w values just before
 * it, which the w row already holds, and the inputs are reloaded.  (Silence rejects every sample; a wave that meets it runs at the
 * exact kernel's speed.)  Only the zero-input loops speculate.  The exact loops follow the
 * speculative one instead of sharing a loop with it: one loop nest with both made the register
 * allocator keep ~80 more VGPRs live and spill to AGPRs (accvgpr moves cost VALU slots). */
/* Lane layout: a group of 128 lanes (two waves) covers 32 streams (64 with the mono dedup); wave
 * f of the group holds filter f (0: I, 1: Q) of every channel, lane l = stream (l >> 1), channel
 * (l & 1) -- or stream l, left channel, under the dedup.  A wave's chains then share the phase
 * parity of their zero inputs whenever the streams' Hilbert phases agree in parity (the usual
 * case: streams started together), which the zero-input fast path needs. */
__device__ __forceinline__ bool icw_k1_chain(int gi, int count, bool dedup, int &s, int &ch, int &f)
{
    const int grp = gi >> 7, w = (gi >> 6) & 1, l = gi & 63;
    f = w;
    if (dedup) { s = grp * 64 + l; ch = 0; }
    else { s = grp * 32 + (l >> 1); ch = l & 1; }
    return s < count;
}

/* XCD-aware order of one-wave workgroups (A/B build only: -DICW_K1_XCD_REMAP=1).  Workgroup b goes
 * to XCD b mod 8 (the dispatcher's round robin on MI355X), so making the I and Q waves of a 128-lane
 * group -- which read the same channel rows since K0 writes one row per channel -- workgroups
 * 16c + j and 16c + j + 8 puts them on one XCD, and the second wave's reads hit the L2 the first one
 * filled: C4's K1 fetch halves (FETCH_SIZE 16.1 -> 8.05 B/frame, the pipeline 121.6 -> 105.5 B/frame).
 * It does not pay: K1 2.91 -> 2.99 ms per launch, C3 -1.6 %, C4 -2.3 % (two runs each, one box),
 * the same direction as two-wave K1 workgroups (-2 to -2.5 %).  So the lane kernel keeps its order. */
#ifndef ICW_K1_XCD_REMAP
#define ICW_K1_XCD_REMAP 0
#endif
__device__ __forceinline__ int icw_k1_block(int b, int nb, int tpb)
{
    if (!ICW_K1_XCD_REMAP || tpb != 64 || b >= (nb & ~15)) return b;
    const int c = b >> 4, j = b & 15;
    return ((c * 8 + (j & 7)) << 1) | (j >> 3);
}

template <int N, bool KAHAN, bool SUBN>
__global__ __launch_bounds__(256) void icw_iir_state(IcwK1Args a)
{
    int s, ch, f;
    if (!icw_k1_chain(icw_k1_block(blockIdx.x, gridDim.x, blockDim.x) * blockDim.x + threadIdx.x, a.n_streams,
                      a.dedup != 0, s, ch, f))
        return;
    const int g = s * 4 + ch * 2 + f;
    const int n_chains = a.n_chains;
    double pc[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) pc[i] = a.pc[i];

    double R[N];
#pragma unroll
    for (int i = 0; i < N; ++i) R[N - 1 - i] = a.hist[(size_t)g * ICW_HIST_PITCH + i];

    /* this block's start (for K2); each (stream, filter) flag is read and written by one wave */
    if (ch == 0) a.info_dup[s * 2 + f] = a.lr_equal[s * 2 + f];
    const double *xp = a.xd + (size_t)(s * 2 + ch) * a.x_pitch;     /* the channel's signed row (K0) */
    double *wrow = a.w + (size_t)g * a.w_pitch;
    /* block-relative sample n has a zero input iff (phi + n) is odd (I: k = hq + t0 + n odd;
     * Q: k + 1 odd) */
    const unsigned phi = (a.hq_phase[s * 2 + ch] + (unsigned)a.t0 + (unsigned)f) & 1u;
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
        bool zfast = false;
        unsigned phi0 = 0;
        if constexpr (KAHAN && SUBN) {
            /* the fast path needs one zero-input parity across the wave */
            phi0 = __builtin_amdgcn_readfirstlane(phi);
            zfast = __all(phi == phi0) && T >= 3 * N;
        }
        if constexpr (KAHAN && SUBN && !(N & 1)) {
            /* even order: block-relative step J of every block (t a multiple of N) is a zero input
             * iff (phi0 + J) is odd */
            if (zfast) {
                if (phi0) icw_even_blocks<N, 0, SUBN>(R, xv, xp, wrow, pc, cnt, t, T);
                else icw_even_blocks<N, 1, SUBN>(R, xv, xp, wrow, pc, cnt, t, T);
            }
        }
        if constexpr (KAHAN && SUBN && (N & 1)) {
            if (zfast) {
                /* speculative pairs of blocks ("Speculative blocks") that start on a nonzero sample; a
                 * failed block ends them and the exact loops below take over at its start */
                if ((phi0 + (unsigned)t) & 1u) {
                    icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt, true);
                    icw_store_block<N>(R, wrow + N + t);
                    t += N;
                }
                double mn = __builtin_inf();       /* smallest |sum| of the speculative block */
                bool fail = false;
                ICW_DRAIN_VMEM();
                while (!fail && t + 2 * N <= T) {
                    /* a failed pair's stores land past [t, t + N), the restart state, and the
                     * exact re-run overwrites them */
                    icw_block_steps_zpf<N, 0, 1, SUBN, true>(R, xv, xp + t + N, pc, cnt, &mn);
                    icw_store_block<N>(R, wrow + N + t);
                    icw_block_steps_zpf<N, 0, 0, SUBN, true>(R, xv, xp + t + 2 * N, pc, cnt, &mn);
                    icw_store_block<N>(R, wrow + 2 * N + t);
                    fail = __any(mn < 1.0);
                    if (!fail) t += 2 * N;
                }
                if (fail) {
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll
                    for (int j = 0; j < N; ++j) R[j] = wrow[t + j];
                }
                icw_load_x<N>(xv, xp + t);   /* the block's inputs (the zero steps left slots unloaded) */
                if (fail) {
                    /* exact from here: the same zero-input pairs with the reject */
                    ICW_DRAIN_VMEM();
                    if (((phi0 + (unsigned)t) & 1u) && t + N <= T) {
                        icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt, true);
                        icw_store_block<N>(R, wrow + N + t);
                        t += N;
                    }
                    for (; t + 2 * N <= T; t += 2 * N) {
                        icw_block_steps_zpf<N, 0, 1, SUBN>(R, xv, xp + t + N, pc, cnt);
                        icw_store_block<N>(R, wrow + N + t);
                        icw_block_steps_zpf<N, 0, 0, SUBN>(R, xv, xp + t + 2 * N, pc, cnt);
                        icw_store_block<N>(R, wrow + 2 * N + t);
                    }
                    icw_load_x<N>(xv, xp + t);
                }
            }
        }
        for (; t + N <= T; t += N) {
            icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt, ((phi + (unsigned)t) & 1u) != 0u);
            icw_store_block<N>(R, wrow + N + t);
        }
    }
    const int rem = T - t;
    if (rem > 0) {
        double xv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) xv[j] = (j < rem) ? xp[t + j] : 0.0;
        icw_block_steps<N, 0, KAHAN, SUBN>(R, xv, pc, cnt, rem, ((phi + (unsigned)t) & 1u) != 0u);
        double *wo = wrow + N + t;
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (j < rem) wo[j] = R[j];
        icw_normalise_ring<N>(R, rem);
    }
    /* the de-subnorm count is taken by K2 from the w rows (a rejected w is exactly 0.0), so the
     * recurrence does not spend issue slots on it: cnt is dead here and compiled away */
    (void)cnt;
    icw_store_hist<N, 0>(R, a.hist, g, n_chains);
    if (a.dedup) {
        icw_store_hist<N, 0>(R, a.hist, g + 2, n_chains);
        a.lr_equal[s * 2 + f] = 1u;
        return;
    }
    /* is this (stream, filter)'s right converter still bit-identical to its left one?  The two
     * channels of a stream are lanes l, l ^ 1 of this wave */
    bool eq = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double o = __shfl_xor(R[i], 1);
        eq = eq && (__double_as_longlong(o) == __double_as_longlong(R[i]));
    }
    if (ch == 0) a.lr_equal[s * 2 + f] = eq ? 1u : 0u;
}

/* ----------------------------------------------- IIR state kernel with FC() (K1f) -------- */
/* FP_CHECK on: the WITH FP CHECKS branches of iir_rp_process_kahan / _baseline for the loop-back
 * sum (hblpf.c:1058-1095 / 928-950): ti = FC(z * c_i), kahan_step_fes (hblpf.c:995-1005), or
 * sum_i = FC(sum_i + FC(z * c_i)).  A diagnostic mode, so the plain form: one lane per chain,
 * no zero-input steps, no mono shortcuts (the census must count every converter's own events). */
/* one sample; the delay line is a ring in private memory indexed at run time (this mode favours
 * code size over speed): logical z_i = R[(j - 1 - i) mod N] at step j, the new w goes to R[j mod N] */
template <bool KAHAN, bool SUBN>
__device__ __noinline__ double icw_iir_step_fc(double *R, int N, int j, double xin, const double *pc, IcwFes &fe)
{
    double S = xin;
    if (KAHAN) {
        double C = 0.0, Y, T;
#pragma unroll 1
        for (int i = 0; i < N; ++i) {
            const double ti = icw_fc(R[(j - 1 - i + 2 * N) % N] * pc[i], fe);
            Y = icw_fc(ti - C, fe);
            T = icw_fc(S + Y, fe);
            C = icw_fc(icw_fc(T - S, fe) - Y, fe);
            S = T;
        }
    } else {
#pragma unroll 1
        for (int i = 0; i < N; ++i) S = icw_fc(S + icw_fc(R[(j - 1 - i + 2 * N) % N] * pc[i], fe), fe);
    }
    if (SUBN && fabs(S) < 1.0) S = 0.0;
    R[j % N] = S;
    return S;
}

template <bool KAHAN, bool SUBN>
__global__ __launch_bounds__(64) void icw_iir_state_fc(IcwK1Args a, int N)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.n_chains) return;
    const int s = g >> 2, ch = (g >> 1) & 1, f = g & 1;
    double pc[20], R[20];
#pragma unroll 1
    for (int i = 0; i < 20; ++i) pc[i] = a.pc[i];
#pragma unroll 1
    for (int i = 0; i < N; ++i) R[N - 1 - i] = a.hist[(size_t)g * ICW_HIST_PITCH + i];
    const double *xp = a.xd + (size_t)(s * 2 + ch) * a.x_pitch;     /* the channel's signed row (K0) */
    const unsigned phi = (a.hq_phase[s * 2 + ch] + (unsigned)a.t0 + (unsigned)f) & 1u;
    double *wrow = a.w + (size_t)g * a.w_pitch;
#pragma unroll 1
    for (int j = 0; j < N; ++j) wrow[j] = R[j];
    IcwFes fe = {};
    const int T = a.T;
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
        const double x = ((phi + (unsigned)t) & 1u) ? 0.0 : xp[t];     /* hq_rp_process's literal +0.0 */
        wrow[N + t] = icw_iir_step_fc<KAHAN, SUBN>(R, N, t, x, pc, fe);
    }
    /* after T steps logical z_i = R[(T - 1 - i) mod N] */
#pragma unroll 1
    for (int i = 0; i < N; ++i) a.hist[(size_t)g * ICW_HIST_PITCH + i] = R[((T - 1 - i) % N + N) % N];
    if (ch == 0) {                /* no converter-identity shortcuts in this mode */
        a.info_dup[s * 2 + f] = 0u;
        a.lr_equal[s * 2 + f] = 0u;
    }
    icw_fes_flush(fe, a.fes + ((size_t)s * 4 + ch) * ICW_FES_PITCH);
}

template <int N>
__global__ __launch_bounds__(256) void icw_iir_row(IcwK1Args a)
{
    icw_iir_row_body<N>(a, blockIdx.x * blockDim.x + threadIdx.x);
}


/* ---------------------------------------------------------------- launch wrappers ------- */
/* dynamic LDS that makes a workgroup of kernel f hold a.lds_hold bytes in all */
static size_t k1_dyn_lds(const void *f, const IcwK1Args &a)
{
    if (!a.lds_hold) return 0;
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, f) != hipSuccess) return 0;
    return a.lds_hold > fa.sharedSizeBytes ? a.lds_hold - fa.sharedSizeBytes : 0;
}

template <int N, bool K, bool S>
static hipError_t launch_k1_t(const IcwK1Args &a, hipStream_t st)
{
    /* 128-lane groups of 32 streams (64 under the mono dedup), see icw_k1_chain */
    const int spg = a.dedup ? 64 : 32;
    const long lanes = (long)((a.n_streams + spg - 1) / spg) * 128;
    const int tpb = 64 * a.wg_waves;
    const int blocks = (int)((lanes + tpb - 1) / tpb);
    hipLaunchKernelGGL((icw_iir_state<N, K, S>), dim3(blocks), dim3(tpb),
                       k1_dyn_lds((const void *)icw_iir_state<N, K, S>, a), st, a);
    return hipGetLastError();
}

template <bool K, bool S>
static hipError_t launch_k1f_t(const IcwK1Args &a, int N, hipStream_t st)
{
    hipLaunchKernelGGL((icw_iir_state_fc<K, S>), dim3((a.n_chains + 63) / 64), dim3(64), 0, st, a, N);
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_iir_fc(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st)
{
    if (!a->fes || a->dedup || nord < 1 || nord > 20) return hipErrorInvalidValue;
    if (kahan) return subn ? launch_k1f_t<true, true>(*a, nord, st) : launch_k1f_t<true, false>(*a, nord, st);
    return subn ? launch_k1f_t<false, true>(*a, nord, st) : launch_k1f_t<false, false>(*a, nord, st);
}

/* K1r: four chain slots per wave and filter (see icw_iir_row); Kahan with the reject only */
template <int N>
static hipError_t launch_k1r_t(const IcwK1Args &a, hipStream_t st)
{
    const long slots = a.dedup ? a.n_streams : 2L * a.n_streams;
    const long lanes = ((slots + 3) / 4) * 2 * 64;
    const int tpb = 64 * a.wg_waves;
    const int blocks = (int)((lanes + tpb - 1) / tpb);
    hipLaunchKernelGGL((icw_iir_row<N>), dim3(blocks), dim3(tpb), k1_dyn_lds((const void *)icw_iir_row<N>, a), st, a);
    return hipGetLastError();
}

extern "C" hipError_t icw_launch_iir_row(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st)
{
    if (!kahan || !subn) return hipErrorInvalidValue;
    switch (nord) {
    case 15: return launch_k1r_t<15>(*a, st);
    case 18: return launch_k1r_t<18>(*a, st);
    case 19: return launch_k1r_t<19>(*a, st);
    case 20: return launch_k1r_t<20>(*a, st);
    }
    return hipErrorInvalidValue;
}

template <int N>
static hipError_t launch_k1_n(const IcwK1Args &a, bool kahan, bool subn, hipStream_t st)
{
    if (kahan) return subn ? launch_k1_t<N, true, true>(a, st) : launch_k1_t<N, true, false>(a, st);
    return subn ? launch_k1_t<N, false, true>(a, st) : launch_k1_t<N, false, false>(a, st);
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

