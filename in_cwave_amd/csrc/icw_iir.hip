/*
 * icw_iir.hip -- gfx950 (CDNA4) kernels of the serial IIR recurrence (K1 and its variants).
 *
 * Built with `-ffp-contract=off` and no fast-math: the loop-back sum keeps the operand order of
 * iir_rp_process_kahan / iir_rp_process_baseline (hblpf.c:894-953, 1008-1099) bit for bit.
 *
 *   icw_iir_state     one lane per DF-II chain (stream x channel x {I,Q} filter); the delay line
 *                     is a VGPR ring rotated at compile time (unrolled by the filter order N).
 *   icw_iir_state_mf  the same recurrence with the off-critical-path products fed by the matrix
 *                     core (v_mfma_f64_16x16x4_f64), leaving the VALU to the dependent adds.
 *   icw_iir_pair      experimental chain + helper wave pair (off by default).
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

/* Zero-input step (Kahan, subnorm reject on).  Every other sample of a chain's input is the
 * literal +0.0 of hq_rp_process (lpf_hilbert_quad.c:136-151).  With sample = +0:
 *   kahan_init(+0): S = +0, C = 0;  i = 0: Y = t0, T = +0 + t0, C = (T - 0) - t0 = +0, S = T;
 *   i = 1: Y = t1 - (+0) = t1.
 * So S = t0 and C = +0 after step 0, and step 1's Y is t1: 4 adds fewer.  S can differ from the
 * reference only in the sign of a zero (t0 = -0 gives T = +0); a zero's sign is absorbed by the
 * first nonzero term, and a sum that stays zero is rejected to +0.0 (|S| < 1, hblpf.c:1046), so
 * w is bit-identical.  (With the reject off the sign would survive: that mode takes icw_iir_step.) */
template <int N, int J>
__device__ __forceinline__ void icw_iir_step_z(double (&R)[N], const double (&pc)[20], unsigned &cnt)
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
    const bool z = fabs(S) < 1.0;
    cnt += z ? 1u : 0u;
    S = z ? 0.0 : S;
    R[J] = S;
}

/* A block of N steps whose input is zero at the steps J with (J & 1) == Z.  The next block's
 * zero steps are the other parity (N is odd), so the look-ahead refill of xv[J] is needed exactly
 * where this block's step J had a zero input. */
template <int N, int J0, int Z, bool SUBN>
__device__ __forceinline__ void icw_block_steps_zpf(double (&R)[N], double (&xv)[N], const double *xnext,
                                                    const double (&pc)[20], unsigned &cnt)
{
    if constexpr (J0 < N) {
        if constexpr ((J0 & 1) == Z) {
            icw_iir_step_z<N, J0>(R, pc, cnt);
            xv[J0] = xnext[J0];
        } else {
            icw_iir_step<N, true, SUBN, J0>(R, xv[J0], pc, cnt);
        }
        icw_block_steps_zpf<N, J0 + 1, Z, SUBN>(R, xv, xnext, pc, cnt);
    }
}

template <int N>
__device__ __forceinline__ void icw_load_x(double (&xv)[N], const double *xp)
{
#pragma unroll
    for (int j = 0; j < N; ++j) xv[j] = xp[j];
}

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

template <int N, bool KAHAN, bool SUBN>
__global__ __launch_bounds__(256) void icw_iir_state(IcwK1Args a)
{
    int s, ch, f;
    if (!icw_k1_chain(blockIdx.x * blockDim.x + threadIdx.x, a.n_streams, a.dedup != 0, s, ch, f)) return;
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
        if constexpr (KAHAN && SUBN && (N & 1)) {
            /* block-relative sample n has a zero input iff (phi + n) is odd (I: k = hq + t0 + n odd;
             * Q: k + 1 odd); the fast path needs one parity across the wave */
            const unsigned phi = (a.hq_phase[s * 2 + ch] + (unsigned)a.t0 + (unsigned)f) & 1u;
            const unsigned phi0 = __builtin_amdgcn_readfirstlane(phi);
            if (__all(phi == phi0) && T >= 3 * N) {
                if (phi0) {   /* align: pairs start on a nonzero sample */
                    icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt);
                    double *wo = wrow + N + t;
#pragma unroll
                    for (int j = 0; j < N; ++j) wo[j] = R[j];
                    t += N;
                }
                for (; t + 2 * N <= T; t += 2 * N) {
                    icw_block_steps_zpf<N, 0, 1, SUBN>(R, xv, xp + t + N, pc, cnt);
                    double *wo = wrow + N + t;
#pragma unroll
                    for (int j = 0; j < N; ++j) wo[j] = R[j];
                    icw_block_steps_zpf<N, 0, 0, SUBN>(R, xv, xp + t + 2 * N, pc, cnt);
#pragma unroll
                    for (int j = 0; j < N; ++j) wo[N + j] = R[j];
                }
                icw_load_x<N>(xv, xp + t);   /* the zero steps left half of xv unloaded */
            }
        }
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
    const double *xp = a.xd + (size_t)g * a.x_pitch;
    double *wrow = a.w + (size_t)g * a.w_pitch;
#pragma unroll 1
    for (int j = 0; j < N; ++j) wrow[j] = R[j];
    IcwFes fe = {};
    const int T = a.T;
#pragma unroll 1
    for (int t = 0; t < T; ++t) wrow[N + t] = icw_iir_step_fc<KAHAN, SUBN>(R, N, t, xp[t], pc, fe);
    /* after T steps logical z_i = R[(T - 1 - i) mod N] */
#pragma unroll 1
    for (int i = 0; i < N; ++i) a.hist[(size_t)g * ICW_HIST_PITCH + i] = R[((T - 1 - i) % N + N) % N];
    if (ch == 0) {                /* no converter-identity shortcuts in this mode */
        a.info_dup[s * 2 + f] = 0u;
        a.lr_equal[s * 2 + f] = 0u;
    }
    icw_fes_flush(fe, a.fes + ((size_t)s * 4 + ch) * ICW_FES_PITCH);
}

/* ------------------------------------------ IIR state kernel, row broadcast (K1r) -------- */
/* The same Kahan loop-back sum (iir_rp_process_kahan, hblpf.c:1017-1046, subnorm reject on) with
 * one DF-II chain per 16-lane DPP row instead of one per lane.  What it buys: a wave issues ~one
 * FP64 VALU op per 5 cycles no matter how many lanes do useful work (tools/dpp_probe.hip), so the
 * 18 products c_i * w[n-1-i] of the plain kernel (18 of its 93 instructions per sample) are
 * replaced by ONE lane-parallel multiply per sample:
 *
 *   - every lane of a row runs the chain's Kahan sequence redundantly, so w[n] is row-uniform;
 *   - right after w[n] is known, lane l computes P[n mod N] = c[l+1] * w[n]: term i = l+1 of the
 *     sample n+1+i.  Terms 17..19 (orders 18..20) use a second register P2 (lanes 0..3);
 *   - term i's step Y = t_i - C takes t_i straight from lane i-1 of the row through
 *     `v_fmac_f64_dpp ... row_newbcast:(i-1)` as Y = t_i * 1.0 + NC with NC = -C: one rounding
 *     of t_i - C, the same value (a DPP fmac issues like a v_add_f64: 20.0 cycles per Kahan step
 *     either way, profiles/r01_dpp_probe.txt);
 *   - NC = Y - (T - S) is -((T - S) - Y) exactly, except that an exact-zero difference comes out
 *     +0 on both sides: intermediate values then differ at most in the sign of a zero, which the
 *     first nonzero term absorbs, and a sum that stays zero is rejected to +0.0 (|S| < 1,
 *     hblpf.c:1046).  So w is bit-identical when the reject is on, the only mode this kernel runs.
 *   - the newest term t0 = c0 * w[n-1] is on the critical path and stays a row-uniform multiply
 *     (zero-input steps, below, also need t1 row-uniform).
 *
 * Per sample: 1 + P-muls (1 or 2) + 73 add/fmac + cmp + 2 cndmask, against 19 mul + 73 add + cmp +
 * 2 cndmask; the zero-input steps (every other input of a filter is the literal +0.0,
 * lpf_hilbert_quad.c:136-151) save 4 adds as in icw_iir_state, now for every filter order.  The
 * price is 16 lanes per chain: 4 chains per wave.  The host takes this kernel only when the
 * resulting waves fit one per SIMD on at most half the chip (C2, C5); bigger batches keep the
 * lane-per-chain kernel, whose 64 chains per wave fill the chip at the issue floor. */

/* Products of a new w: r = a * b.  Volatile, like the term chains (icw_row_asm.inc): program order
 * keeps every DPP read of a product register many instructions after its write (the VALU-write
 * -> DPP-read hazard needs two). */
__device__ __forceinline__ double icw_vmul(double a, double b)
{
    double r;
    asm volatile("v_mul_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

#include "icw_row_asm.inc"

struct IcwRowC {
    double c0, c1;      /* row-uniform: newest two loop-back coefficients */
    double pl, pl2;     /* per lane: c[l+1], c[l+17] (0 past the order) */
    double one;         /* 1.0 in a VGPR (VOP2 src1) */
};

/* one sample at unroll step J; zero-input step when Z != 2 and (J & 1) == Z.  Logical z_i =
 * W[(J-1-i) mod N] (row-uniform); the new w goes to W[J] and its products to P[J] / P2[J]. */
template <int N, int J, int Z>
__device__ __forceinline__ void icw_row_step(double (&W)[N], double (&P)[N], double (&P2)[N], double xin,
                                             const IcwRowC &c)
{
    constexpr bool ZS = Z != 2 && (J & 1) == Z;
    double S, Y;
    if constexpr (ZS) {
        /* kahan_init(+0) and term 0 collapse to S = t0, C = +0; term 1's Y is t1 */
        S = W[(J - 1 + N) % N] * c.c0;
        Y = W[(J - 2 + 2 * N) % N] * c.c1;
    } else {
        S = xin;                               /* kahan_init(sample) */
        Y = W[(J - 1 + N) % N] * c.c0;         /* term 0: t0 - 0 */
    }
    const double T = S + Y;
    double NC = Y - (T - S);
    /* terms I0..N-1: Y = t_i - C with t_i = lane i-1 of P (i-17 of P2), one asm block */
    S = icw_row_chain<N, ZS ? 2 : 1, J>(T, NC, c.one, P, P2);
    S = fabs(S) < 1.0 ? 0.0 : S;               /* hblpf.c:1046 */
    W[J] = S;
    P[J] = icw_vmul(c.pl, S);
    if constexpr (N > 17) P2[J] = icw_vmul(c.pl2, S);
}

/* a block of N samples; xv[J] is refilled with the input N samples ahead right after step J when
 * the next block's step J (zero parity ZN) consumes an input */
template <int N, int J, int Z, int ZN>
__device__ __forceinline__ void icw_row_block(double (&W)[N], double (&P)[N], double (&P2)[N], double (&xv)[N],
                                              const double *xnext, const IcwRowC &c)
{
    if constexpr (J < N) {
        icw_row_step<N, J, Z>(W, P, P2, xv[J], c);
        if constexpr (!(ZN != 2 && (J & 1) == ZN)) xv[J] = xnext[J];
        icw_row_block<N, J + 1, Z, ZN>(W, P, P2, xv, xnext, c);
    }
}

template <int N, int J>
__device__ __forceinline__ void icw_row_block_lim(double (&W)[N], double (&P)[N], double (&P2)[N],
                                                  const double (&xv)[N], const IcwRowC &c, int lim)
{
    if constexpr (J < N) {
        if (J < lim) {
            icw_row_step<N, J, 2>(W, P, P2, xv[J], c);
            icw_row_block_lim<N, J + 1>(W, P, P2, xv, c, lim);
        }
    }
}

template <int N>
__device__ __forceinline__ void icw_row_store(const double (&W)[N], double *wo, bool writer)
{
    if (writer) {
#pragma unroll
        for (int j = 0; j < N; ++j) wo[j] = W[j];
    }
}

/* Row layout: wave v holds filter f = v & 1 of the four chain slots 4 (v >> 1) + r, r = row;
 * slot = 2 stream + channel (stream, left channel under the dedup).  The two channels of a
 * stream are rows r, r ^ 1 of one wave; a wave's chains share a filter kind, hence the
 * zero-input parity whenever their Hilbert phases agree in parity. */
template <int N>
__global__ __launch_bounds__(256) void icw_iir_row(IcwK1Args a)
{
    const int gl = blockIdx.x * blockDim.x + threadIdx.x;
    const int wv = gl >> 6, r = (gl >> 4) & 3, lr = gl & 15;
    const int f = wv & 1;
    const int slot = (wv >> 1) * 4 + r;
    const bool dedup = a.dedup != 0;
    const int s = dedup ? slot : (slot >> 1), ch = dedup ? 0 : (slot & 1);
    if (s >= a.n_streams) return;
    const int g = s * 4 + ch * 2 + f;
    const bool writer = lr == 0;

    IcwRowC c;
    c.c0 = a.pc[0];
    c.c1 = a.pc[1];
    c.pl = (lr + 1 < N) ? a.pc[lr + 1] : 0.0;
    c.pl2 = (lr + 17 < N) ? a.pc[lr + 17] : 0.0;
    c.one = 1.0;

    double W[N], P[N], P2[N];
#pragma unroll
    for (int i = 0; i < N; ++i) W[N - 1 - i] = a.hist[(size_t)g * ICW_HIST_PITCH + i];
    if constexpr (N > 17) {
#pragma unroll
        for (int k = 0; k < N; ++k) P2[k] = icw_vmul(c.pl2, W[k]);
    }
#pragma unroll
    for (int k = 0; k < N; ++k) P[k] = icw_vmul(c.pl, W[k]);
    asm volatile("s_nop 1");

    if (writer && ch == 0) a.info_dup[s * 2 + f] = a.lr_equal[s * 2 + f];
    const double *xp = a.xd + (size_t)g * a.x_pitch;
    double *wrow = a.w + (size_t)g * a.w_pitch;
    icw_row_store<N>(W, wrow, writer);

    const int T = a.T;
    int t = 0;
    if (T >= N) {
        double xv[N];
        icw_load_x<N>(xv, xp);
        /* block-relative sample n has a zero input iff (phi + n) is odd (see icw_iir_state) */
        const unsigned phi = (a.hq_phase[s * 2 + ch] + (unsigned)a.t0 + (unsigned)f) & 1u;
        const unsigned phi0 = __builtin_amdgcn_readfirstlane(phi);
        if (__all(phi == phi0) && T >= 3 * N) {
            if constexpr (N & 1) {
                /* odd order: the zero parity alternates block to block */
                if (phi0) {
                    icw_row_block<N, 0, 0, 1>(W, P, P2, xv, xp + t + N, c);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    t += N;
                }
                for (; t + 2 * N <= T; t += 2 * N) {
                    icw_row_block<N, 0, 1, 0>(W, P, P2, xv, xp + t + N, c);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    icw_row_block<N, 0, 0, 1>(W, P, P2, xv, xp + t + 2 * N, c);
                    icw_row_store<N>(W, wrow + 2 * N + t, writer);
                }
            } else if (phi0) {
                /* even order: the same zero steps in every block */
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 0, 0>(W, P, P2, xv, xp + t + N, c);
                    icw_row_store<N>(W, wrow + N + t, writer);
                }
            } else {
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 1, 1>(W, P, P2, xv, xp + t + N, c);
                    icw_row_store<N>(W, wrow + N + t, writer);
                }
            }
            icw_load_x<N>(xv, xp + t);   /* the zero steps left part of xv unloaded */
        }
        for (; t + N <= T; t += N) {
            icw_row_block<N, 0, 2, 2>(W, P, P2, xv, xp + t + N, c);
            icw_row_store<N>(W, wrow + N + t, writer);
        }
    }
    const int rem = T - t;
    if (rem > 0) {
        double xv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) xv[j] = (j < rem) ? xp[t + j] : 0.0;
        icw_row_block_lim<N, 0>(W, P, P2, xv, c, rem);
        if (writer) {
            double *wo = wrow + N + t;
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j < rem) wo[j] = W[j];
        }
        icw_normalise_ring<N>(W, rem);
    }
    if (writer) {
        icw_store_hist<N, 0>(W, a.hist, g, a.n_chains);
        if (dedup) icw_store_hist<N, 0>(W, a.hist, g + 2, a.n_chains);
    }
    if (dedup) {
        if (writer) a.lr_equal[s * 2 + f] = 1u;
        return;
    }
    /* right converter still bit-identical to the left one?  Its row is r ^ 1 (lane ^ 16) */
    bool eq = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double o = __shfl_xor(W[i], 16);
        eq = eq && (__double_as_longlong(o) == __double_as_longlong(W[i]));
    }
    if (writer && ch == 0) a.lr_equal[s * 2 + f] = eq ? 1u : 0u;
}

/* ------------------------------------------- IIR state kernel, MFMA product feed (K1m) ---- */
/* Same recurrence as icw_iir_state, but the products c_i * w[n-1-i], i >= 1, which are off the
 * critical path, come from the matrix core instead of the chain's own VALU issue slots.  A wave
 * issues ~1 FP64 VALU op per ~4.7 cycles whether or not the ops depend on each other, so every
 * product taken off the VALU shortens the sample.
 *
 * v_mfma_f64_16x16x4_f64 (gfx950): lane l holds A[l&15][l>>4], B[l>>4][l&15] and
 * D[(l>>4) + 4r][l&15], r = 0..3.  With B = the lane's own w[m] and
 *     A[rho][k] = (k == (rho & 3)) ? c[4G + 1 + (rho >> 2)] : 0,
 * D[h + 4r][col] = sum_k A[h+4r][k] * B[k][col] = c[4G+1+r] * (B of lane 16h+col = this lane):
 * every lane receives the four products c[4G+1..4G+4] * w[m] of its OWN chain.  The three other
 * k terms are exact zeros (w is finite), so each result is the correctly rounded product, i.e.
 * bit-identical to v_mul_f64 (a zero-signed product may come out as +0 instead of -0; that only
 * matters for an exactly-zero sum, which the subnorm reject turns into +0 anyway, and the
 * GPU parity tests cover both sum modes bit for bit).
 *
 * Schedule: at sample n the wave issues, for each group G, the MFMA of w[n-1-4G]; its product
 * r is consumed at sample n+1+r (i = 4G+1+r:  w[(n+1+r)-1-i] = w[n-1-4G]).  So every product is
 * ready ~a sample ahead of use and at most 4 samples x NG groups of results are live.  Results
 * are kept in P[G][J] with J = sample mod N (the unroll), so the loop carries them without moves.
 * MFMA ignores EXEC: every lane of the wave must hold a finite w, so lanes past n_chains shadow
 * the last chain and store nothing of their own. */
typedef double icw_d4 __attribute__((ext_vector_type(4)));

template <int N>
struct IcwMf {
    static constexpr int NG = (N - 1 + 3) / 4;     /* product groups of 4 */
};

template <int N, bool KAHAN, bool SUBN, int J>
__device__ __forceinline__ void icw_iir_step_mf(double (&R)[N], double xin, const double (&pc)[20],
                                                const double (&A)[IcwMf<N>::NG],
                                                icw_d4 (&P)[IcwMf<N>::NG][N], unsigned &cnt)
{
    constexpr int NG = IcwMf<N>::NG;
    const icw_d4 z4 = {0.0, 0.0, 0.0, 0.0};
    /* products of this sample's issue: group G of w[n-1-4G] = R[(J-1-4G) mod N] */
#pragma unroll
    for (int G = 0; G < NG; ++G)
        P[G][J] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[G], R[(J - 1 - 4 * G + 2 * N) % N], z4, 0, 0, 0);
    double S;
    const double t0 = R[(J - 1 + N) % N] * pc[0];
    if (KAHAN) {
        double C = 0.0, Y, T;
        S = xin;
        Y = t0 - C; T = S + Y; C = (T - S) - Y; S = T;
#pragma unroll
        for (int i = 1; i < N; ++i) {
            const int r = (i - 1) & 3, G = (i - 1) >> 2;
            const double ti = P[G][(J - 1 - r + N) % N][r];
            Y = ti - C; T = S + Y; C = (T - S) - Y; S = T;
        }
    } else {
        S = xin;
        S += t0;
#pragma unroll
        for (int i = 1; i < N; ++i) {
            const int r = (i - 1) & 3, G = (i - 1) >> 2;
            S += P[G][(J - 1 - r + N) % N][r];
        }
    }
    if (SUBN) {
        const bool z = fabs(S) < 1.0;
        cnt += z ? 1u : 0u;
        S = z ? 0.0 : S;
    }
    R[J] = S;
}

template <int N, int J0, bool KAHAN, bool SUBN>
__device__ __forceinline__ void icw_block_steps_mf(double (&R)[N], double (&xv)[N], const double *xnext,
                                                   const double (&pc)[20], const double (&A)[IcwMf<N>::NG],
                                                   icw_d4 (&P)[IcwMf<N>::NG][N], unsigned &cnt)
{
    if constexpr (J0 < N) {
        icw_iir_step_mf<N, KAHAN, SUBN, J0>(R, xv[J0], pc, A, P, cnt);
        xv[J0] = xnext[J0];
        icw_block_steps_mf<N, J0 + 1, KAHAN, SUBN>(R, xv, xnext, pc, A, P, cnt);
    }
}

/* MFMAs of the four virtual samples before the loop (J = N-4 .. N-1): block-start ring mapping
 * R[N-1-i] = w[-1-i], so w[n'-1-4G] = R[J-1-4G]; an index below 0 is a product never consumed */
template <int N, int J>
__device__ __forceinline__ void icw_mf_prime(const double (&R)[N], const double (&A)[IcwMf<N>::NG],
                                             icw_d4 (&P)[IcwMf<N>::NG][N])
{
    if constexpr (J < N) {
        const icw_d4 z4 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int G = 0; G < IcwMf<N>::NG; ++G) {
            const int idx = J - 1 - 4 * G;
            P[G][J] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[G], idx >= 0 ? R[idx < 0 ? 0 : idx] : 0.0, z4, 0, 0, 0);
        }
        icw_mf_prime<N, J + 1>(R, A, P);
    }
}

template <int N, bool KAHAN, bool SUBN>
__global__ __launch_bounds__(256) void icw_iir_state_mf(IcwK1Args a)
{
    constexpr int NG = IcwMf<N>::NG;
    const int lane = threadIdx.x & 63;
    const int g0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool own = g0 < a.n_chains;
    const int g = own ? g0 : a.n_chains - 1;       /* shadow lanes: finite data, no stores */
    const int s = g >> 2, c = (g >> 1) & 1, f = g & 1;
    const int n_chains = a.n_chains;
    double pc[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) pc[i] = a.pc[i];
    double A[NG];
    {
        const int rho = lane & 15, k = lane >> 4;
#pragma unroll
        for (int G = 0; G < NG; ++G) {
            const int i = 4 * G + 1 + (rho >> 2);
            double v = 0.0;
#pragma unroll
            for (int q = 1; q < N; ++q) v = (q == i) ? pc[q] : v;
            A[G] = (k == (rho & 3)) ? v : 0.0;
        }
    }

    double R[N];
#pragma unroll
    for (int i = 0; i < N; ++i) R[N - 1 - i] = a.hist[(size_t)g * ICW_HIST_PITCH + i];

    if (own && c == 0) a.info_dup[s * 2 + f] = a.lr_equal[s * 2 + f];
    const double *xp = a.xd + (size_t)g * a.x_pitch;
    double *wrow = a.w + (size_t)g * a.w_pitch;
    if (own) {
#pragma unroll
        for (int j = 0; j < N; ++j) wrow[j] = R[j];
    }

    const int T = a.T;
    unsigned cnt = 0;
    int t = 0;
    if (T >= N) {
        icw_d4 P[NG][N];
        icw_mf_prime<N, N - 4>(R, A, P);
        double xv[N];
        icw_load_x<N>(xv, xp);
        for (; t + N <= T; t += N) {
            icw_block_steps_mf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, A, P, cnt);
            if (own) {
                double *wo = wrow + N + t;
#pragma unroll
                for (int j = 0; j < N; ++j) wo[j] = R[j];
            }
        }
    }
    const int rem = T - t;
    if (rem > 0) {
        double xv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) xv[j] = (j < rem) ? xp[t + j] : 0.0;
        icw_block_steps<N, 0, KAHAN, SUBN>(R, xv, pc, cnt, rem);
        if (own) {
            double *wo = wrow + N + t;
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j < rem) wo[j] = R[j];
        }
        icw_normalise_ring<N>(R, rem);
    }
    bool eq = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double o = __shfl_xor(R[i], 2);
        eq = eq && (__double_as_longlong(o) == __double_as_longlong(R[i]));
    }
    const bool eq_q = __shfl_xor((int)eq, 1) != 0;
    if (!own) return;
    icw_store_hist<N, 0>(R, a.hist, g, n_chains);
    (void)cnt;   /* counted by K2 */
    if (c == 0) a.lr_equal[s * 2 + f] = (eq && eq_q) ? 1u : 0u;
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
    (void)cnt;   /* counted by K2 */
    if (c == 0) {   /* the pair kernel does not track converter identity: no shortcut */
        a.info_dup[s * 2 + f] = 0u;
        a.lr_equal[s * 2 + f] = 0u;
    }
}
/* ---------------------------------------------------------------- launch wrappers ------- */
template <int N, bool K, bool S>
static hipError_t launch_k1_t(const IcwK1Args &a, hipStream_t st)
{
    /* 128-lane groups of 32 streams (64 under the mono dedup), see icw_k1_chain */
    const int spg = a.dedup ? 64 : 32;
    const long lanes = (long)((a.n_streams + spg - 1) / spg) * 128;
    const int tpb = 64 * a.wg_waves;
    const int blocks = (int)((lanes + tpb - 1) / tpb);
    hipLaunchKernelGGL((icw_iir_state<N, K, S>), dim3(blocks), dim3(tpb), 0, st, a);
    return hipGetLastError();
}

template <int N, bool K, bool S>
static hipError_t launch_k1m_t(const IcwK1Args &a, hipStream_t st)
{
    const int tpb = 64 * a.wg_waves;
    const int blocks = (a.n_chains + tpb - 1) / tpb;
    hipLaunchKernelGGL((icw_iir_state_mf<N, K, S>), dim3(blocks), dim3(tpb), 0, st, a);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_k1m_n(const IcwK1Args &a, bool kahan, bool subn, hipStream_t st)
{
    if (kahan) return subn ? launch_k1m_t<N, true, true>(a, st) : launch_k1m_t<N, true, false>(a, st);
    return subn ? launch_k1m_t<N, false, true>(a, st) : launch_k1m_t<N, false, false>(a, st);
}

extern "C" hipError_t icw_launch_iir_mfma(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st)
{
    switch (nord) {
    case 15: return launch_k1m_n<15>(*a, kahan, subn, st);
    case 18: return launch_k1m_n<18>(*a, kahan, subn, st);
    case 19: return launch_k1m_n<19>(*a, kahan, subn, st);
    case 20: return launch_k1m_n<20>(*a, kahan, subn, st);
    }
    return hipErrorInvalidValue;
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
    hipLaunchKernelGGL((icw_iir_row<N>), dim3(blocks), dim3(tpb), 0, st, a);
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

