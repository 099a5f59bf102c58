// tools/k1_probe.hip -- diagnostic harness for the IIR state kernels (plain vs chain+helper pair).
// Includes the kernels with ICW_STAMPS so workgroup 0 records s_memtime stamps per sample.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/k1_probe tools/k1_probe.hip
#define ICW_STAMPS
#include "k1_experimental.hip"
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv)
{
    const int S = argc > 1 ? atoi(argv[1]) : 256, T = argc > 2 ? atoi(argv[2]) : 8192;
    const int C = S * 4;
    const size_t xp = T + 2, wp = T + 21;
    std::vector<double> hx((size_t)S * 2 * xp);
    for (size_t i = 0; i < hx.size(); ++i) hx[i] = (double)((int)(rand() % 65536) - 32768);
    double *xd, *hist, *w;
    unsigned long long *sn, *nf, *inf;
    unsigned *ph, *iph;
    long long *pos;
    int *err;
    CK(hipMalloc(&xd, hx.size() * 8));
    CK(hipMemcpy(xd, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&hist, (size_t)C * 20 * 8));
    CK(hipMalloc(&w, (size_t)C * wp * 8));
    CK(hipMalloc(&sn, C * 8)); CK(hipMalloc(&nf, S * 8)); CK(hipMalloc(&inf, S * 8));
    CK(hipMalloc(&ph, S * 8)); CK(hipMalloc(&iph, S * 8)); CK(hipMalloc(&pos, S * 8)); CK(hipMalloc(&err, 4));
    IcwK1Args a;
    memset(&a, 0, sizeof(a));
    a.xd = xd; a.x_pitch = xp; a.nch = 2; a.n_streams = S; a.n_chains = C; a.T = T;
    a.hist = hist; a.sncnt = sn; a.hq_phase = ph; a.pos = pos; a.n_frame = nf; a.ssr = 48000000ull; a.scaled = 1;
    a.w = w; a.w_pitch = wp; a.info_phase = iph; a.info_nframe = inf; a.err = err;
    const double pcv[19] = {0.5, -0.4, 0.3, -0.2, 0.1, -0.05, 0.02, -0.01, 0.005, -0.002, 0.001, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 19; ++i) a.pc[i] = pcv[i];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 2; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemset(hist, 0, (size_t)C * 20 * 8));
            CK(hipEventRecord(e0, 0));
            if (mode == 0) hipLaunchKernelGGL((icw_iir_state<19, true, true>), dim3((C + 63) / 64), dim3(64), 0, 0, a);
            else hipLaunchKernelGGL((icw_iir_pair<19, true, true>), dim3((C + 63) / 64), dim3(128), 0, 0, a);
            CK(hipEventRecord(e1, 0));
            CK(hipDeviceSynchronize());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%s: %d chains x %d samples: %.3f ms  = %.1f ns/sample = %.0f cyc@2.4GHz\n", mode ? "pair " : "plain",
               C, T, best, best * 1e6 / T, best * 1e6 / T * 2.4);
    }
    unsigned long long st[8][1024];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(icw_stamps), sizeof(st)));
    printf("stamps (s_memtime ticks), samples 200..215: chain[start, mid-ok, published] helper[seen, done]\n");
    for (int n = 200; n < 216; ++n)
        printf("n=%4d  c_mid-c_start %6lld  c_pub-c_mid %6lld  c_next-c_start %6lld | h_seen-c_pub %6lld  h_done-h_seen %6lld\n", n,
               (long long)(st[1][n] - st[0][n]), (long long)(st[2][n] - st[1][n]), (long long)(st[0][n + 1] - st[0][n]),
               (long long)(st[3][n] - st[2][n]), (long long)(st[4][n] - st[3][n]));
    double acc[5] = {0};
    int cnt = 0;
    for (int n = 100; n < 1000; ++n, ++cnt) {
        acc[0] += (double)(st[1][n] - st[0][n]); acc[1] += (double)(st[2][n] - st[1][n]);
        acc[2] += (double)(st[0][n + 1] - st[0][n]); acc[3] += (double)(st[3][n] - st[2][n]); acc[4] += (double)(st[4][n] - st[3][n]);
    }
    printf("mean over 100..999: mid %.0f pub %.0f period %.0f | seen-lag %.0f helper-work %.0f\n", acc[0] / cnt, acc[1] / cnt,
           acc[2] / cnt, acc[3] / cnt, acc[4] / cnt);
    int he = 0;
    CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
    printf("err flag %d\n", he);
    return 0;
}
