// tools/exec_probe.hip -- does a wave64 FP64 VALU op issue faster when EXEC has fewer lanes?
// A chain of dependent v_add_f64 (and v_fma_f64 / v_mul_f64) runs under EXEC = the first L lanes
// (L = 64, 48, 32, 16, 8, 1, and lanes 16..31 only); cycles per op from s_memtime (clock64).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/exec_probe tools/exec_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP "512"
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7"

#define PROBE(name, body)                                                                   \
__global__ void name(long long *cyc, double *out, int lo, int hi)                           \
{                                                                                           \
    long long t0 = 0, t1 = 0;                                                               \
    double r = 0.0;                                                                         \
    const int l = threadIdx.x;                                                              \
    if (l >= lo && l < hi) {                                                                \
        asm volatile("v_mov_b64 v[0:1], 1.0\n v_mov_b64 v[2:3], 0.5\n v_mov_b64 v[4:5], 1.0" ::: CLOB); \
        t0 = clock64();                                                                     \
        asm volatile(".rept " REP "\n" body "\n.endr" ::: CLOB);                            \
        t1 = clock64();                                                                     \
        asm volatile("v_mov_b64 %0, v[0:1]" : "=v"(r) :: CLOB);                             \
        out[l] = r;                                                                         \
        if (l == lo) cyc[0] = t1 - t0;                                                      \
    }                                                                                       \
}

PROBE(dep_add, "v_add_f64 v[0:1], v[0:1], v[2:3]\n v_add_f64 v[0:1], v[0:1], v[2:3]")
PROBE(dep_fma, "v_fma_f64 v[0:1], v[0:1], v[4:5], v[2:3]\n v_fma_f64 v[0:1], v[0:1], v[4:5], v[2:3]")
PROBE(ind_add, "v_add_f64 v[0:1], v[0:1], v[2:3]\n v_add_f64 v[6:7], v[4:5], v[2:3]")
PROBE(dep_add32, "v_add_f32 v0, v0, v2\n v_add_f32 v0, v0, v2")

typedef void (*K)(long long *, double *, int, int);

int main()
{
    long long *dcyc; double *dout;
    hipMalloc(&dcyc, 64); hipMalloc(&dout, 64 * 8);
    const int rng[][2] = {{0, 64}, {0, 48}, {0, 32}, {0, 16}, {16, 32}, {32, 48}, {0, 8}, {0, 1}, {63, 64}};
    const char *nm[] = {"dep_add_f64", "dep_fma_f64", "ind_add_f64", "dep_add_f32"};
    K ks[] = {dep_add, dep_fma, ind_add, dep_add32};
    for (int k = 0; k < 4; ++k)
        for (auto &r : rng) {
            long long h = 0;
            for (int i = 0; i < 3; ++i) {
                hipLaunchKernelGGL(ks[k], dim3(1), dim3(64), 0, 0, dcyc, dout, r[0], r[1]);
                hipDeviceSynchronize();
            }
            hipMemcpy(&h, dcyc, 8, hipMemcpyDeviceToHost);
            printf("%-12s lanes [%2d,%2d)  cyc/op %.2f\n", nm[k], r[0], r[1], h / (512.0 * 2));
        }
    return 0;
}
