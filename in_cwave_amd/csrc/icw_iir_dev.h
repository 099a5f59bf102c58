/*
 * icw_iir_dev.h -- device code of the row-broadcast IIR recurrence K1r (icw_iir_row) and the
 * helpers it shares with the lane-per-chain K1, included by icw_iir.hip (the K1 kernels) and by
 * icw_kernels.hip (the one-stream fused kernel icw_stream1, which runs K1r inside one workgroup).
 * Built with -ffp-contract=off: the loop-back sum keeps the operand order of iir_rp_process_kahan
 * (hblpf.c:1008-1056) bit for bit.
 */
#ifndef ICW_IIR_DEV_H_
#define ICW_IIR_DEV_H_

#pragma clang fp contract(off)

/* Filter input of a chain at step J of a block (K0 writes one signed row per channel, holding the I
 * filter's nonzero inputs at the even Hilbert phases and the Q filter's at the odd ones): the row's
 * value, or the literal +0.0 that hq_rp_process feeds the filter at the other phases
 * (lpf_hilbert_quad.c:133-151).  Block-relative sample n is a zero input iff (phi + n) is odd; qodd
 * says (phi + t) is odd for the block at t, so step J is a zero input iff (J odd) != qodd.  Only the
 * generic loops call this: the zero-input loops never read a zero step's input. */
template <int J>
__device__ __forceinline__ double icw_chain_x(double v, bool qodd)
{
    return (((J & 1) != 0) != qodd) ? 0.0 : v;
}

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

/* full block of N steps; after step J consumes xv[J], refill it with the input N samples ahead
 * (rows are padded by >= N doubles, so the last block's look-ahead loads stay in bounds) */
/* Before a loop over blocks: wait for every outstanding global access, once.  The loop's first
 * iteration can be entered straight from a block whose last look-ahead loads were just issued; the
 * waitcnt pass then sizes the in-loop waits for that path (vmcnt(0)-(2) a few steps in) and every
 * iteration pays them, waiting on the previous block's stores -- in K1 those are 10 stores over
 * 64 rows each (C4: K1 3.18 -> 3.29-3.40 ms per launch).  Drained here, the loop's waits follow
 * the steady state (vmcnt(19) down to (10)). */
#define ICW_DRAIN_VMEM() __builtin_amdgcn_s_waitcnt(0x0F70)   /* vmcnt(0), expcnt / lgkmcnt free */

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
                                             double xin2, const IcwRowC &c, double &mn, bool qodd = false)
{
    if constexpr (Z == 2) xin = icw_chain_x<J>(xin, qodd);   /* generic steps: the zero inputs supplied */
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
                                              const IcwRowC &c, double &mn, bool qodd = false)
{
    if constexpr (J < N) {
        icw_row_step<N, J, Z, SPEC>(W, P, P2, xv[J], xv2[J], c, mn, qodd);
        if constexpr (!(ZN != 2 && (J & 1) == ZN)) {
            xv[J] = xnext[J];
            if constexpr (icw_row_c0p<N>() && ZN != 2) xv2[J] = xnext2[J];
        }
        icw_row_block<N, J + 1, Z, ZN, SPEC>(W, P, P2, xv, xv2, xnext, xnext2, c, mn, qodd);
    }
}

template <int N, int J>
__device__ __forceinline__ void icw_row_block_lim(double (&W)[N], double (&P)[N], double (&P2)[N],
                                                  const double (&xv)[N], const IcwRowC &c, int lim, bool qodd)
{
    if constexpr (J < N) {
        if (J < lim) {
            double mn;
            icw_row_step<N, J, 2, false>(W, P, P2, xv[J], 0.0, c, mn, qodd);
            icw_row_block_lim<N, J + 1>(W, P, P2, xv, c, lim, qodd);
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
/* PUB (K5's overlapped form, one stream): the w rows go to the LDS rows lw (chain c = ch*2 + f at
 * lw + c * lpitch) instead of a.w, and lane 0 of each wave publishes in prog[f] how many of the
 * block's frames have final rows, after each checked block: the output waves poll it and take
 * those frames while the recurrence runs on.  One wave's LDS operations are performed in issue
 * order, so a reader that sees the count also sees the rows stored before it. */
template <bool PUB>
__device__ __forceinline__ void icw_row_publish(int *prog, int gl, int f, int done)
{
    if constexpr (PUB) {
        asm volatile("" ::: "memory");
        if ((gl & 63) == 0) *(volatile __attribute__((address_space(3))) int *)(prog + f) = done;
    }
}

template <int N, bool PUB = false>
__device__ __forceinline__ void icw_iir_row_body(const IcwK1Args &a, int gl, double *lw = nullptr, int lpitch = 0,
                                                 int *prog = nullptr)
{
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
    const double *xp = a.xd + (size_t)(s * 2 + ch) * a.x_pitch;     /* the channel's signed row (K0) */
    /* block-relative sample n has a zero input iff (phi + n) is odd (see icw_iir_state) */
    const unsigned phi = (a.hq_phase[s * 2 + ch] + (unsigned)a.t0 + (unsigned)f) & 1u;
    /* the same row through a pointer the compiler cannot equate with xp: the zero-input loops of
     * orders > 17 load each input into two registers (icw_row_step's xin2), not load + copy */
    int zoff = 0;
    asm volatile("" : "+s"(zoff));
    const double *xp2 = xp + zoff;             /* still a global-memory pointer (no flat loads) */
    double *wrow = PUB ? lw + (size_t)(ch * 2 + f) * lpitch : a.w + (size_t)g * a.w_pitch;
    icw_row_store<N>(W, wrow, writer);

    const int T = a.T;
    int t = 0;
    if (T >= N) {
        double xv[N], xv2[N];
        icw_load_x<N>(xv, xp);
        if constexpr (icw_row_c0p<N>()) icw_load_x<N>(xv2, xp2);
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
                    icw_row_publish<PUB>(prog, gl, f, t + 2 * N);
                }
            } else if (phi0) {
                /* even order: the same zero steps in every block */
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 0, 0, true>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    if (__any(mn < 1.0)) { fail = true; break; }
                    icw_row_publish<PUB>(prog, gl, f, t + N);
                }
            } else {
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 1, 1, true>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    if (__any(mn < 1.0)) { fail = true; break; }
                    icw_row_publish<PUB>(prog, gl, f, t + N);
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
                    icw_row_publish<PUB>(prog, gl, f, t + 2 * N);
                }
            } else if (phi0) {
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 0, 0, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    icw_row_publish<PUB>(prog, gl, f, t + N);
                }
            } else {
                for (; t + N <= T; t += N) {
                    icw_row_block<N, 0, 1, 1, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn);
                    icw_row_store<N>(W, wrow + N + t, writer);
                    icw_row_publish<PUB>(prog, gl, f, t + N);
                }
            }
            icw_load_x<N>(xv, xp + t);
        }
        for (; t + N <= T; t += N) {
            icw_row_block<N, 0, 2, 2, false>(W, P, P2, xv, xv2, xp + t + N, xp2 + t + N, c, mn,
                                             ((phi + (unsigned)t) & 1u) != 0u);
            icw_row_store<N>(W, wrow + N + t, writer);
            icw_row_publish<PUB>(prog, gl, f, t + N);
        }
    }
    const int rem = T - t;
    if (rem > 0) {
        double xv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) xv[j] = (j < rem) ? xp[t + j] : 0.0;
        icw_row_block_lim<N, 0>(W, P, P2, xv, c, rem, ((phi + (unsigned)t) & 1u) != 0u);
        if (writer) {
            double *wo = wrow + N + t;
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j < rem) wo[j] = W[j];
        }
        icw_normalise_ring<N>(W, rem);
    }
    icw_row_publish<PUB>(prog, gl, f, T);
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

#endif /* ICW_IIR_DEV_H_ */
