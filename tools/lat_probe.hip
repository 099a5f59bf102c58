// tools/lat_probe.hip -- gfx950 FP64 VALU latency / throughput probe for the IIR critical path.
// Measures, with s_memtime inside one wave: cycles per dependent v_add_f64, per dependent
// v_mul_f64, per Kahan step (4 dependent adds), and independent-add issue rate.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/lat_probe tools/lat_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#pragma clang fp contract(off)

#define REPS 4096

__global__ void dep_add(const double *in, double *out, long long *cyc)
{
    double a = in[threadIdx.x], c = in[64 + threadIdx.x];
    long long t0 = clock64();
#pragma unroll 64
    for (int i = 0; i < REPS; ++i) a = a + c;
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void dep_mul(const double *in, double *out, long long *cyc)
{
    double a = in[threadIdx.x], c = in[64 + threadIdx.x];
    long long t0 = clock64();
#pragma unroll 64
    for (int i = 0; i < REPS; ++i) a = a * c;
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void kahan(const double *in, double *out, long long *cyc)
{
    double S = in[threadIdx.x], C = 0.0, x = in[64 + threadIdx.x];
    long long t0 = clock64();
#pragma unroll 64
    for (int i = 0; i < REPS; ++i) {
        double Y = x - C;
        double T = S + Y;
        C = (T - S) - Y;
        S = T;
    }
    long long t1 = clock64();
    out[threadIdx.x] = S + C;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void dep_add_lanes(const double *in, double *out, long long *cyc, int lanes)
{
    double a = in[threadIdx.x & 63], c = in[64 + (threadIdx.x & 63)];
    long long t0 = clock64();
    if ((int)(threadIdx.x & 63) < lanes) {
#pragma unroll 64
        for (int i = 0; i < REPS; ++i) a = a + c;
    }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void kahan_lanes(const double *in, double *out, long long *cyc, int lanes)
{
    double S = in[threadIdx.x & 63], C = 0.0, x = in[64 + (threadIdx.x & 63)];
    long long t0 = clock64();
    if ((int)(threadIdx.x & 63) < lanes) {
#pragma unroll 64
        for (int i = 0; i < REPS; ++i) {
            double Y = x - C;
            double T = S + Y;
            C = (T - S) - Y;
            S = T;
        }
    }
    long long t1 = clock64();
    out[threadIdx.x] = S + C;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void indep_add(const double *in, double *out, long long *cyc)
{
    double a0 = in[threadIdx.x], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7, c = in[64 + threadIdx.x];
    long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < REPS / 8; ++i) {
        a0 = a0 + c; a1 = a1 + c; a2 = a2 + c; a3 = a3 + c;
        a4 = a4 + c; a5 = a5 + c; a6 = a6 + c; a7 = a7 + c;
    }
    long long t1 = clock64();
    out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*K)(const double *, double *, long long *);

static void run(const char *name, K k, int waves_per_block, const double *din, double *dout,
                long long *dcyc, double ops)
{
    long long h[256];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves_per_block), 0, 0, din, dout, dcyc);
        hipDeviceSynchronize();
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves_per_block), 0, 0, din, dout, dcyc);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, dcyc, sizeof(long long), hipMemcpyDeviceToHost);
    printf("%-10s waves/WG=%d  cycles/op=%.2f  (s_memtime cyc %lld, kernel %.3f us, %.2f ns/op)\n", name,
           waves_per_block, h[0] / ops, h[0], ms * 1e3, ms * 1e6 / ops);
}

int main()
{
    double *din, *dout;
    long long *dcyc;
    hipMalloc(&din, 128 * 8);
    hipMalloc(&dout, 64 * 8 * 16);
    hipMalloc(&dcyc, 256 * 8);
    double h[128];
    for (int i = 0; i < 128; ++i) h[i] = 1.0 + i * 1e-3;
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("device %s clock %d kHz CUs %d\n", p.gcnArchName, p.clockRate, p.multiProcessorCount);
    run("dep_add", dep_add, 1, din, dout, dcyc, REPS);
    run("dep_mul", dep_mul, 1, din, dout, dcyc, REPS);
    run("kahan4", kahan, 1, din, dout, dcyc, REPS * 4.0);
    run("indep_add", indep_add, 1, din, dout, dcyc, REPS);
    for (int lanes = 64; lanes >= 1; lanes /= 2) {
        long long h1[2];
        hipLaunchKernelGGL(dep_add_lanes, dim3(1), dim3(64), 0, 0, din, dout, dcyc, lanes);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(dep_add_lanes, dim3(1), dim3(64), 0, 0, din, dout, dcyc, lanes);
        hipDeviceSynchronize();
        hipMemcpy(h1, dcyc, 8, hipMemcpyDeviceToHost);
        long long h2[2];
        hipLaunchKernelGGL(kahan_lanes, dim3(1), dim3(64), 0, 0, din, dout, dcyc, lanes);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(kahan_lanes, dim3(1), dim3(64), 0, 0, din, dout, dcyc, lanes);
        hipDeviceSynchronize();
        hipMemcpy(h2, dcyc, 8, hipMemcpyDeviceToHost);
        printf("active lanes %2d: dep_add %.2f cyc/op, kahan %.2f cyc/add\n", lanes, h1[0] / (double)REPS,
               h2[0] / (4.0 * REPS));
    }
    // two waves sharing one SIMD (8 waves per WG -> 2 per SIMD)
    run("dep_add", dep_add, 8, din, dout, dcyc, REPS);
    run("kahan4", kahan, 8, din, dout, dcyc, REPS * 4.0);
    run("dep_add", dep_add, 4, din, dout, dcyc, REPS);
    run("kahan4", kahan, 4, din, dout, dcyc, REPS * 4.0);
    return 0;
}
