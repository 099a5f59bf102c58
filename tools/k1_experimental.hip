/*
 * k1_experimental.hip -- ARCHIVED K1 variants, not part of libicw.so.
 *
 *   icw_iir_state_mf  the loop-back recurrence with the 18 off-critical-path products fed by the
 *                     matrix core (v_mfma_f64_16x16x4_f64): bit-exact, but 20.5 ms against 13.7 ms
 *                     per 65 536-frame launch (the FP64 MFMA shares the VALU's FP64 pipe).
 *   icw_iir_pair      chain + helper wave pair, products handed over through an LDS ring:
 *                     bit-exact, 24 ms against 13 ms per launch (hand-off waits).
 *
 * Both were GPU-parity green when they lived in the library (round 1).  They compile on top of
 * the product's K1 helpers:  make -C tools k1x   (tools/k1_probe.hip times icw_iir_pair).
 */
#include "../in_cwave_amd/csrc/icw_iir.hip"

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

