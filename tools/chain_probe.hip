// tools/chain_probe.hip -- gfx950 dependent-chain latency of the instructions on the serial render's
// error-feedback chain (K3r): one wave, a chain of 16 dependent instructions per loop trip, 512
// trips, s_memtime around it.  Prints shader-clock cycles per dependent instruction.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/chain_probe tools/chain_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define TRIPS 512
#define X4(s) s s s s
#define X16(s) X4(s) X4(s) X4(s) X4(s)

#define PROBE(name, ...)                                                                    \
    __global__ void name(const double *in, double *out, long long *cyc)                     \
    {                                                                                       \
        double a = in[threadIdx.x], b = in[64 + threadIdx.x], one = 1.0;                    \
        int ia = (int)threadIdx.x, lo = -100, hi = 100;                                     \
        long long t0 = clock64();                                                           \
        for (int i = 0; i < TRIPS; ++i) {                                                   \
            __VA_ARGS__;                                                                    \
        }                                                                                   \
        long long t1 = clock64();                                                           \
        out[threadIdx.x] = a + b + one + (double)ia + lo + hi;                              \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                    \
    }

PROBE(p_add, asm volatile(X16("v_add_f64 %0, %0, %1\n") : "+v"(a) : "v"(b)))
PROBE(p_fma, asm volatile(X16("v_fma_f64 %0, %0, %1, %1\n") : "+v"(a) : "v"(b)))
PROBE(p_max, asm volatile(X16("v_max_f64 %0, %0, %1\n") : "+v"(a) : "v"(b)))
PROBE(p_trunc, asm volatile(X16("v_trunc_f64 %0, %0\n") : "+v"(a)))
PROBE(p_fmac_dpp, asm volatile(X16("v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n")
                               : "+v"(a) : "v"(b), "v"(one)))
PROBE(p_add_dpp_src, asm volatile(X16("v_fmac_f64_dpp %0, %0, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\ns_nop 1\n")
                                  : "+v"(a) : "v"(b), "v"(one)))
PROBE(p_cvt_pair, asm volatile(X16("v_cvt_i32_f64 %1, %0\nv_cvt_f64_i32 %0, %1\n") : "+v"(a), "+v"(ia)))
PROBE(p_med3, asm volatile(X16("v_med3_i32 %0, %0, %1, %2\n") : "+v"(ia) : "v"(lo), "v"(hi)))
PROBE(p_add_i32, asm volatile(X16("v_add_u32 %0, %0, %1\n") : "+v"(ia) : "v"(lo)))
PROBE(p_cndmask, asm volatile(X16("v_cmp_gt_i32 vcc, 0, %0\nv_cndmask_b32 %0, %0, %1, vcc\n") : "+v"(ia) : "v"(lo) : "vcc"))
PROBE(p_indep_add, { double c1, c2, c3, c4;
      asm volatile(X4("v_add_f64 %0, %4, %4\nv_add_f64 %1, %4, %4\nv_add_f64 %2, %4, %4\nv_add_f64 %3, %4, %4\n")
                   : "=v"(c1), "=v"(c2), "=v"(c3), "=v"(c4) : "v"(b)); a += c1 + c2 + c3 + c4; })

typedef void (*K)(const double *, double *, long long *);

int main()
{
    double *in, *out;
    long long *cyc;
    hipMalloc(&in, 128 * sizeof(double));
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, sizeof(long long));
    double h[128];
    for (int i = 0; i < 128; ++i) h[i] = 1.0 + i * 1e-9;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    struct { const char *n; K k; double per; } ks[] = {
        {"v_add_f64 dep", p_add, 16}, {"v_fma_f64 dep", p_fma, 16}, {"v_max_f64 dep", p_max, 16},
        {"v_trunc_f64 dep", p_trunc, 16}, {"v_fmac_f64_dpp (acc dep)", p_fmac_dpp, 16},
        {"v_fmac_f64_dpp (dpp src dep, +s_nop 1)", p_add_dpp_src, 16},
        {"cvt_i32_f64 + cvt_f64_i32 pair", p_cvt_pair, 16}, {"v_med3_i32 dep", p_med3, 16},
        {"v_add_u32 dep", p_add_i32, 16}, {"v_cmp_f64 + v_cndmask pair", p_cndmask, 16},
        {"v_add_f64 independent (issue)", p_indep_add, 16},
    };
    for (auto &k : ks) {
        long long c = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, in, out, cyc);
            hipDeviceSynchronize();
            hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        }
        printf("%-44s %6.2f cycles per instruction (group)\n", k.n, (double)c / (TRIPS * k.per));
    }
    return 0;
}
