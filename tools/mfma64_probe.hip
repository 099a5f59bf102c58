// Probe: does v_mfma_f64_16x16x4_f64 run beside FP64 VALU work (separate pipes) or in the same pipe,
// and how does it round (which order of fused steps)?  Diagnostic only (tools/mfma64_probe.py reads
// gpurun_out/mfma64_round.bin).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/mfma64_probe tools/mfma64_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <cmath>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

/* MODE 0: MFMA only, 1: VALU only, 2: both in every wave, 3: waves 0-3 of a 512-thread block MFMA,
 * waves 4-7 VALU.  Per iteration: 4 independent MFMAs (4 096 FMAs) and/or 64 VALU FMAs (4 096 lane FMAs). */
template <int MODE>
__global__ __launch_bounds__(512) void tk(double *out, int n, double s)
{
    const int w = threadIdx.x >> 6;
    const bool doM = MODE == 0 || MODE == 2 || (MODE == 3 && (w & 4) == 0);
    const bool doV = MODE == 1 || MODE == 2 || (MODE == 3 && (w & 4) != 0);
    const double a = threadIdx.x * 1e-3 + s, b = 1.0 + threadIdx.x * 1e-9;
    d4 c0 = {0, 0, 0, 0}, c1 = {1, 0, 0, 0}, c2 = {2, 0, 0, 0}, c3 = {3, 0, 0, 0};
    double v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = i * s;
    if (MODE == 2) {
        for (int it = 0; it < n; ++it) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = __builtin_fma(v[i], b, a);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = __builtin_fma(v[i], b, a);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = __builtin_fma(v[i], b, a);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = __builtin_fma(v[i], b, a);
        }
    } else {
        if (doM) {
            for (int it = 0; it < n; ++it) {
                c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
            }
        }
        if (doV) {
            for (int it = 0; it < n; ++it) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int i = 0; i < 16; ++i) v[i] = __builtin_fma(v[i], b, a);
            }
        }
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += v[i];
    acc += c0[0] + c0[1] + c0[2] + c0[3] + c1[0] + c1[1] + c1[2] + c1[3];
    acc += c2[0] + c2[1] + c2[2] + c2[3] + c3[0] + c3[1] + c3[2] + c3[3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

/* rounding: wave g computes D = A B + C for its own A (16x4), B (4x16), C (16x16) */
__global__ void rk(const double *A, const double *B, const double *C, double *D)
{
    const int l = threadIdx.x & 63, g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const double *Ag = A + g * 64, *Bg = B + g * 64, *Cg = C + g * 256;
    double *Dg = D + g * 256;
    const double a = Ag[(l & 15) * 4 + (l >> 4)];          /* A[i = l & 15][k = l >> 4], row-major 16x4 */
    const double b = Bg[(l >> 4) * 16 + (l & 15)];         /* B[k = l >> 4][j = l & 15], row-major 4x16 */
    d4 c;
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = Cg[((l >> 4) + 4 * r) * 16 + (l & 15)];
    const d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) Dg[((l >> 4) + 4 * r) * 16 + (l & 15)] = d[r];
}

template <int MODE>
static float timeit(double *out, int blocks, int threads, int n)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(tk<MODE>, dim3(blocks), dim3(threads), 0, 0, out, n, 1e-7);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(tk<MODE>, dim3(blocks), dim3(threads), 0, 0, out, n, 1e-7);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

int main(int argc, char **argv)
{
    const char *path = argc > 1 ? argv[1] : "gpurun_out/mfma64_round.bin";
    double *out;
    CK(hipMalloc(&out, sizeof(double) * 2048 * 512));
    const int n = 1000;
    /* same total work per mode: MODE 0 and 1 do one kind each, MODE 2 / 3 both kinds */
    const float t0 = timeit<0>(out, 2048, 256, n), t1 = timeit<1>(out, 2048, 256, n);
    const float t2 = timeit<2>(out, 2048, 256, n), t3 = timeit<3>(out, 1024, 512, n);
    const double fm = 2048.0 * 4 * 4 * 1024.0 * n * 2;   /* MFMA flops of MODE 0 */
    printf("{\"mfma_ms\": %.3f, \"valu_ms\": %.3f, \"both_same_wave_ms\": %.3f, \"both_split_waves_ms\": %.3f, "
           "\"mfma_tflops\": %.2f, \"valu_tflops\": %.2f}\n", t0, t1, t2, t3, fm / t0 / 1e9, fm / t1 / 1e9);

    const int G = 4096;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(1.0, 2.0);
    std::uniform_int_distribution<int> E(-40, 40), S(0, 1);
    auto rnd = [&]() { return (S(rng) ? -1.0 : 1.0) * std::ldexp(U(rng), E(rng)); };
    std::vector<double> A(G * 64), B(G * 64), C(G * 256), D(G * 256);
    for (auto &x : A) x = rnd();
    for (auto &x : B) x = rnd();
    for (auto &x : C) x = rnd();
    /* a quarter of the groups: cancellation-heavy (products of similar size, opposite signs) */
    for (int g = 0; g < G / 4; ++g)
        for (int i = 0; i < 64; ++i) {
            A[g * 64 + i] = (S(rng) ? -1.0 : 1.0) * std::ldexp(U(rng), E(rng) / 8);
            B[g * 64 + i] = (S(rng) ? -1.0 : 1.0) * std::ldexp(U(rng), E(rng) / 8);
        }
    double *dA, *dB, *dC, *dD;
    CK(hipMalloc(&dA, A.size() * 8));
    CK(hipMalloc(&dB, B.size() * 8));
    CK(hipMalloc(&dC, C.size() * 8));
    CK(hipMalloc(&dD, D.size() * 8));
    CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(rk, dim3(G / 4), dim3(256), 0, 0, dA, dB, dC, dD);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost));
    FILE *f = fopen(path, "wb");
    if (!f) { printf("cannot write %s\n", path); return 1; }
    fwrite(A.data(), 8, A.size(), f);
    fwrite(B.data(), 8, B.size(), f);
    fwrite(C.data(), 8, C.size(), f);
    fwrite(D.data(), 8, D.size(), f);
    fclose(f);
    printf("wrote %d groups to %s\n", G, path);
    return 0;
}
