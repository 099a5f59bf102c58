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

/* ------------------------------------------------------------ IIR state kernel (K1) ----- */
/* mn = min(mn, |s|) in one instruction: v_min_f64 with the abs modifier (the fmin builtin adds a
 * NaN-quieting v_max_f64 per operand in IEEE mode).  A NaN s leaves mn unchanged, as it leaves the
 * reference's `fabs(sum) < 1` false. */
__device__ __forceinline__ double icw_minabs(double m, double s)
{
    double r;
    asm("v_min_f64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(s));
    return r;
}

/* the same, volatile: K1r keeps it in program order among its volatile term chains (placed freely
 * there, the scheduler's choices pushed the kernel past 256 VGPRs) -- and K1 must not use this one:
 * memory operations do not move across a volatile asm, so the mins dragged K1's look-ahead loads
 * to the end of each block, and block 2 waited on them (C4 K1 3.18 -> 3.29 ms per launch) */
__device__ __forceinline__ double icw_minabs_v(double m, double s)
{
    double r;
    asm volatile("v_min_f64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(s));
    return r;
}

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
/* Before a loop over blocks: wait for every outstanding global access, once.  The loop's first
 * iteration can be entered straight from a block whose last look-ahead loads were just issued; the
 * waitcnt pass then sizes the in-loop waits for that path (vmcnt(0)-(2) a few steps in) and every
 * iteration pays them, waiting on the previous block's stores -- in K1 those are 10 stores over
 * 64 rows each (C4: K1 3.18 -> 3.29-3.40 ms per launch).  Drained here, the loop's waits follow
 * the steady state (vmcnt(19) down to (10)). */
#define ICW_DRAIN_VMEM() __builtin_amdgcn_s_waitcnt(0x0F70)   /* vmcnt(0), expcnt / lgkmcnt free */

template <int N, int J0, bool KAHAN, bool SUBN, bool SPEC = false>
__device__ __forceinline__ void icw_block_steps_pf(double (&R)[N], double (&xv)[N], const double *xnext,
                                                   const double (&pc)[20], unsigned &cnt, double *mn = nullptr)
{
    if constexpr (J0 < N) {
        icw_iir_step<N, KAHAN, SUBN, J0, SPEC>(R, xv[J0], pc, cnt, mn);
        xv[J0] = xnext[J0];
        icw_block_steps_pf<N, J0 + 1, KAHAN, SUBN, SPEC>(R, xv, xnext, pc, cnt, mn);
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

/* A block of N steps whose input is zero at the steps J with (J & 1) == Z.  The next block's
 * zero steps are the other parity (N is odd), so the look-ahead refill of xv[J] is needed exactly
 * where this block's step J had a zero input. */
template <int N, int J0, int Z, bool SUBN, bool SPEC = false>
__device__ __forceinline__ void icw_block_steps_zpf(double (&R)[N], double (&xv)[N], const double *xnext,
                                                    const double (&pc)[20], unsigned &cnt, double *mn = nullptr)
{
    if constexpr (J0 < N) {
        if constexpr ((J0 & 1) == Z) {
            icw_iir_step_z<N, J0, SPEC>(R, pc, cnt, mn);
            xv[J0] = xnext[J0];
        } else {
            icw_iir_step<N, true, SUBN, J0, SPEC>(R, xv[J0], pc, cnt, mn);
        }
        icw_block_steps_zpf<N, J0 + 1, Z, SUBN, SPEC>(R, xv, xnext, pc, cnt, mn);
    }
}

template <int N>
__device__ __forceinline__ void icw_load_x(double (&xv)[N], const double *xp)
{
#pragma unroll
    for (int j = 0; j < N; ++j) xv[j] = xp[j];
}

/* a block's w values to its row: after a full block R[j] is the block's sample j */
template <int N>
__device__ __forceinline__ void icw_store_block(const double (&R)[N], double *wo)
{
#pragma unroll
    for (int j = 0; j < N; ++j) wo[j] = R[j];
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
        bool zfast = false;
        unsigned phi0 = 0;
        if constexpr (KAHAN && SUBN && (N & 1)) {
            /* block-relative sample n has a zero input iff (phi + n) is odd (I: k = hq + t0 + n odd;
             * Q: k + 1 odd); the fast path needs one parity across the wave */
            const unsigned phi = (a.hq_phase[s * 2 + ch] + (unsigned)a.t0 + (unsigned)f) & 1u;
            phi0 = __builtin_amdgcn_readfirstlane(phi);
            zfast = __all(phi == phi0) && T >= 3 * N;
        }
        if constexpr (KAHAN && SUBN && (N & 1)) {
            if (zfast) {
                /* speculative pairs of blocks ("Speculative blocks") that start on a nonzero sample; a
                 * failed block ends them and the exact loops below take over at its start */
                if ((phi0 + (unsigned)t) & 1u) {
                    icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt);
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
                        icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt);
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
            icw_block_steps_pf<N, 0, KAHAN, SUBN>(R, xv, xp + t + N, pc, cnt);
            icw_store_block<N>(R, wrow + N + t);
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
    double pl, pl2;     /* per lane: c[l+1], c[l+17] (0 past the order); orders > 17 also c0 in lane
                           N - 17 of pl2 (icw_row_c0_lane) */
    double one;         /* 1.0 in a VGPR (VOP2 src1) */
};

/* Orders > 17 keep c0 * w in a spare lane of the second product row, so a nonzero-input step reads
 * its newest term t0 through the DPP operand like the others (icw_row_asm.inc, I0 = 0) instead of
 * a row-uniform multiply: 77 -> 76 FP64 VALU on those steps.  Orders <= 17 have no second row to
 * spare (its multiply would cost what it saves). */
template <int N>
constexpr bool icw_row_c0p() { return N > 17; }
template <int N>
constexpr int icw_row_c0_lane() { return N - 17; }


/* one sample at unroll step J; zero-input step when Z != 2 and (J & 1) == Z.  Logical z_i =
 * W[(J-1-i) mod N] (row-uniform); the new w goes to W[J] and its products to P[J] / P2[J].
 * SPEC: the reject (hblpf.c:1046) is speculated away -- w = S unconditionally, and mn tracks the
 * smallest |S| so the block can be re-run exactly if any sum fell below 1 ("Speculative blocks").
 * xin2: a second register holding the same input (the zero-input loops of orders > 17 load it
 * twice), which the I0 = 0 chain turns into T in place. */
template <int N, int J, int Z, bool SPEC>
__device__ __forceinline__ void icw_row_step(double (&W)[N], double (&P)[N], double (&P2)[N], double xin,
                                             double xin2, const IcwRowC &c, double &mn)
{
    constexpr bool ZS = Z != 2 && (J & 1) == Z;
    constexpr bool C0P = icw_row_c0p<N>() && Z != 2 && !ZS;
    double S;
    if constexpr (C0P) {
        /* kahan_init(sample), then every term from a product lane */
        S = icw_row_chain<N, 0, J>(xin, 0.0, xin2, c.one, P, P2);
    } else {
        double Y;
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
        S = icw_row_chain<N, ZS ? 2 : 1, J>(T, NC, 0.0, c.one, P, P2);
    }
    if constexpr (!SPEC) S = fabs(S) < 1.0 ? 0.0 : S;          /* hblpf.c:1046 */
    W[J] = S;
    /* P2 first: the next step's I0 = 0 chain reads lane c0 of P2[J] through DPP, which must come
     * two VALU instructions after the write (P[J] and the minimum, all volatile asm in order) */
    if constexpr (N > 17) P2[J] = icw_vmul(c.pl2, S);
    P[J] = icw_vmul(c.pl, S);
    if constexpr (SPEC) mn = icw_minabs_v(mn, S);
    else if constexpr (icw_row_c0p<N>()) asm volatile("s_nop 1");   /* exact loops: no minimum */
}

/* a block of N samples; xv[J] is refilled with the input N samples ahead right after step J when
 * the next block's step J (zero parity ZN) consumes an input */
template <int N, int J, int Z, int ZN, bool SPEC>
__device__ __forceinline__ void icw_row_block(double (&W)[N], double (&P)[N], double (&P2)[N], double (&xv)[N],
                                              double (&xv2)[N], const double *xnext, const double *xnext2,
                                              const IcwRowC &c, double &mn)
{
    if constexpr (J < N) {
        icw_row_step<N, J, Z, SPEC>(W, P, P2, xv[J], xv2[J], c, mn);
        if constexpr (!(ZN != 2 && (J & 1) == ZN)) {
            xv[J] = xnext[J];
            if constexpr (icw_row_c0p<N>() && ZN != 2) xv2[J] = xnext2[J];
        }
        icw_row_block<N, J + 1, Z, ZN, SPEC>(W, P, P2, xv, xv2, xnext, xnext2, c, mn);
    }
}

template <int N, int J>
__device__ __forceinline__ void icw_row_block_lim(double (&W)[N], double (&P)[N], double (&P2)[N],
                                                  const double (&xv)[N], const IcwRowC &c, int lim)
{
    if constexpr (J < N) {
        if (J < lim) {
            double mn;
            icw_row_step<N, J, 2, false>(W, P, P2, xv[J], 0.0, c, mn);
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

/* the lane-parallel products of the whole ring: P[k] = c[l+1] * W[k], P2[k] = c[l+17] * W[k] */
template <int N>
__device__ __forceinline__ void icw_row_products(const double (&W)[N], double (&P)[N], double (&P2)[N],
                                                 const IcwRowC &c)
{
    if constexpr (N > 17) {
#pragma unroll
        for (int k = 0; k < N; ++k) P2[k] = icw_vmul(c.pl2, W[k]);
    }
#pragma unroll
    for (int k = 0; k < N; ++k) P[k] = icw_vmul(c.pl, W[k]);
    asm volatile("s_nop 1");   /* VALU write -> DPP read of P / P2 */
}

/* after a failed speculative block at t: the ring from the w row, its products, the block's inputs */
template <int N>
__device__ __forceinline__ void icw_row_restart(double (&W)[N], double (&P)[N], double (&P2)[N], double (&xv)[N],
                                                double (&xv2)[N], const double *xp, const double *xp2,
                                                const double *wrow, int t, const IcwRowC &c)
{
    /* the writer lane stored the row [t, t + N): block start or the previous block */
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll
    for (int j = 0; j < N; ++j) W[j] = wrow[t + j];
    icw_row_products<N>(W, P, P2, c);
    icw_load_x<N>(xv, xp + t);
    if constexpr (icw_row_c0p<N>()) icw_load_x<N>(xv2, xp2 + t);
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
    c.pl2 = (lr + 17 < N) ? a.pc[lr + 17] : (icw_row_c0p<N>() && lr == icw_row_c0_lane<N>()) ? a.pc[0] : 0.0;
    c.one = 1.0;

    double W[N], P[N], P2[N];
#pragma unroll
    for (int i = 0; i < N; ++i) W[N - 1 - i] = a.hist[(size_t)g * ICW_HIST_PITCH + i];
    icw_row_products<N>(W, P, P2, c);

    if (writer && ch == 0) a.info_dup[s * 2 + f] = a.lr_equal[s * 2 + f];
    const double *xp = a.xd + (size_t)g * a.x_pitch;
    /* the same row through a pointer the compiler cannot equate with xp: the zero-input loops of
     * orders > 17 load each input into two registers (icw_row_step's xin2), not load + copy */
    int zoff = 0;
    asm volatile("" : "+s"(zoff));
    const double *xp2 = xp + zoff;             /* still a global-memory pointer (no flat loads) */
    double *wrow = a.w + (size_t)g * a.w_pitch;
    icw_row_store<N>(W, wrow, writer);

    const int T = a.T;
    int t = 0;
    if (T >= N) {
        double xv[N], xv2[N];
        icw_load_x<N>(xv, xp);
        if constexpr (icw_row_c0p<N>()) icw_load_x<N>(xv2, xp2);
        /* block-relative sample n has a zero input iff (phi + n) is odd (see icw_iir_state) */
        const unsigned phi = (a.hq_phase[s * 2 + ch] + (unsigned)a.t0 + (unsigned)f) & 1u;
        const unsigned phi0 = __builtin_amdgcn_readfirstlane(phi);
        const bool zfast = __all(phi == phi0) && T >= 3 * N;
        double mn = __builtin_inf();               /* smallest |sum| of the speculative block */
        bool fail = false;
        ICW_DRAIN_VMEM();
        if (zfast) {
            /* speculative zero-input blocks ("Speculative blocks" above); a failed block ends them
             * and the exact loops below take over at its start */
            if constexpr (N & 1) {
                /* odd order: the zero parity alternates block to block; pairs start on a nonzero
                 * sample */
                if ((phi0 + (unsigned)t) & 1u) {
                    icw_row_block<N, 0, 0, 1, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    t += N;
                }
                for (; t + 2 * N <= T; t += 2 * N) {
                    /* a failed pair's stores land past [t, t + N), the restart state, and the
                     * exact re-run overwrites them */
                    icw_row_block<N, 0, 1, 0, true>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    icw_row_block<N, 0, 0, 1, true>(W, P, P2, xv, xv2, xp + t + 2 * N, xp2 + t + 2 * N, c, mn);
                    icw_row_store<N>(W, wrow + 2 * N + t, writer);
                    if (__any(mn < 1.0)) { fail = true; break; }
                }
            } else if (phi0) {
                /* even order: the same zero steps in every block */
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 0, 0, true>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    if (__any(mn < 1.0)) { fail = true; break; }
                }
            } else {
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 1, 1, true>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    if (__any(mn < 1.0)) { fail = true; break; }
                }
            }
            if (fail) icw_row_restart<N>(W, P, P2, xv, xv2, xp, xp2, wrow, t, c);
            else icw_load_x<N>(xv, xp + t);   /* the zero steps left part of xv unloaded */
        }
        if (fail) {
            /* exact from here: the same zero-input blocks with the reject */
            ICW_DRAIN_VMEM();
            if constexpr (N & 1) {
                if (((phi0 + (unsigned)t) & 1u) && t + N <= T) {
                    icw_row_block<N, 0, 0, 1, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    t += N;
                }
                for (; t + 2 * N <= T; t += 2 * N) {
                    icw_row_block<N, 0, 1, 0, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    icw_row_block<N, 0, 0, 1, false>(W, P, P2, xv, xv2, xp + t + 2 * N, xp2 + t + 2 * N, c, mn);
                    icw_row_store<N>(W, wrow + 2 * N + t, writer);
                }
            } else if (phi0) {
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 0, 0, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                }
            } else {
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 1, 1, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                }
            }
            icw_load_x<N>(xv, xp + t);
        }
        for (; t + N <= T; t += N) {
            icw_row_block<N, 0, 2, 2, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
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

