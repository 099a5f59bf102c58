// tools/bank_probe.hip -- gfx950 FP64 VALU probe: does the VGPR bank of the two 64-bit source
// operands change the issue interval of dependent v_add_f64 chains (the IIR critical path)?
// Register numbers are fixed in inline asm so the bank (reg index mod 4) is under control.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bank_probe tools/bank_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP "256"
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15"

#define PROBE(name, init, body, nops)                                                        \
__global__ void name(long long *cyc, double *out)                                           \
{                                                                                           \
    long long t0, t1;                                                                       \
    double r;                                                                               \
    asm volatile(init ::: CLOB);                                                            \
    t0 = clock64();                                                                         \
    asm volatile(".rept " REP "\n" body "\n.endr" ::: CLOB);                                \
    t1 = clock64();                                                                         \
    asm volatile("v_mov_b64 %0, v[4:5]" : "=v"(r) :: CLOB);                                 \
    out[threadIdx.x] = r;                                                                   \
    if (threadIdx.x % 64 == 0) cyc[threadIdx.x / 64] = t1 - t0;                             \
}

#define INIT "v_mov_b64 v[0:1], 1.0\n v_mov_b64 v[2:3], 1.0\n v_mov_b64 v[4:5], 1.0\n v_mov_b64 v[6:7], 0.5\n" \
             "v_mov_b64 v[8:9], 0.5\n v_mov_b64 v[10:11], 0.5\n v_mov_b64 v[12:13], 0.5\n v_mov_b64 v[14:15], 0.5"

/* 4 dependent adds per rep */
PROBE(dep_b02, INIT, "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[4:5], v[4:5], v[6:7]", 4)
PROBE(dep_b00, INIT, "v_add_f64 v[4:5], v[4:5], v[8:9]\n v_add_f64 v[4:5], v[4:5], v[8:9]\n v_add_f64 v[4:5], v[4:5], v[8:9]\n v_add_f64 v[4:5], v[4:5], v[8:9]", 4)
/* dependent, alternating destination (ping-pong) banks 0/2 */
PROBE(dep_pp02, INIT, "v_add_f64 v[6:7], v[4:5], v[10:11]\n v_add_f64 v[4:5], v[6:7], v[8:9]\n v_add_f64 v[6:7], v[4:5], v[10:11]\n v_add_f64 v[4:5], v[6:7], v[8:9]", 4)
/* two independent chains interleaved */
PROBE(ind2_nc, INIT, "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[8:9], v[8:9], v[10:11]\n v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[8:9], v[8:9], v[10:11]", 4)
PROBE(ind2_c, INIT, "v_add_f64 v[4:5], v[4:5], v[8:9]\n v_add_f64 v[12:13], v[12:13], v[0:1]\n v_add_f64 v[4:5], v[4:5], v[8:9]\n v_add_f64 v[12:13], v[12:13], v[0:1]", 4)
/* four independent chains, no conflicts */
PROBE(ind4_nc, INIT, "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[8:9], v[8:9], v[10:11]\n v_add_f64 v[12:13], v[12:13], v[14:15]\n v_add_f64 v[0:1], v[0:1], v[2:3]", 4)
/* dependent mul */
PROBE(mul_b02, INIT, "v_mul_f64 v[4:5], v[4:5], v[6:7]\n v_mul_f64 v[4:5], v[4:5], v[6:7]\n v_mul_f64 v[4:5], v[4:5], v[6:7]\n v_mul_f64 v[4:5], v[4:5], v[6:7]", 4)
/* Kahan step, bank-aware: S v[0:1](b0) Y v[2:3](b2) T v[6:7](b2) D v[4:5](b0) C v[8:9](b0) t v[10:11](b2)
 *   Y = t - C ; T = S + Y ; D = T - S ; C = D - Y ; S = T (copy-free by swapping roles each rep) */
PROBE(kahan_nc, INIT,
      "v_add_f64 v[2:3], v[10:11], -v[8:9]\n v_add_f64 v[6:7], v[0:1], v[2:3]\n v_add_f64 v[4:5], v[6:7], -v[0:1]\n v_add_f64 v[8:9], v[4:5], -v[2:3]\n"
      "v_add_f64 v[2:3], v[10:11], -v[8:9]\n v_add_f64 v[0:1], v[6:7], v[2:3]\n v_add_f64 v[4:5], v[0:1], -v[6:7]\n v_add_f64 v[8:9], v[4:5], -v[2:3]", 8)
/* the compiler's K1 pattern: S v[12:13]? mixed banks (as emitted in icw_iir_state) */
PROBE(kahan_cc, INIT,
      "v_add_f64 v[4:5], v[12:13], -v[4:5]\n v_add_f64 v[0:1], v[8:9], v[4:5]\n v_add_f64 v[8:9], v[0:1], -v[8:9]\n v_add_f64 v[4:5], v[8:9], -v[4:5]\n"
      "v_add_f64 v[4:5], v[12:13], -v[4:5]\n v_add_f64 v[8:9], v[0:1], v[4:5]\n v_add_f64 v[0:1], v[8:9], -v[0:1]\n v_add_f64 v[4:5], v[0:1], -v[4:5]", 8)

/* the K1 mix: per 5 instructions, 4 dependent adds (the Kahan chain) + 1 independent mul (a product) */
PROBE(kahan_mix, INIT,
      "v_mul_f64 v[10:11], v[12:13], v[14:15]\n v_add_f64 v[2:3], v[10:11], -v[8:9]\n v_add_f64 v[6:7], v[0:1], v[2:3]\n v_add_f64 v[4:5], v[6:7], -v[0:1]\n v_add_f64 v[8:9], v[4:5], -v[2:3]\n"
      "v_mul_f64 v[10:11], v[14:15], v[12:13]\n v_add_f64 v[2:3], v[10:11], -v[8:9]\n v_add_f64 v[0:1], v[6:7], v[2:3]\n v_add_f64 v[4:5], v[0:1], -v[6:7]\n v_add_f64 v[8:9], v[4:5], -v[2:3]", 10)
/* independent muls only */
PROBE(ind_mul, INIT, "v_mul_f64 v[4:5], v[6:7], v[8:9]\n v_mul_f64 v[10:11], v[12:13], v[14:15]\n v_mul_f64 v[0:1], v[6:7], v[14:15]\n v_mul_f64 v[2:3], v[8:9], v[12:13]", 4)

typedef void (*K)(long long *, double *);

static void run(const char *name, K k, int waves, int ops_per_rep, long long *dcyc, double *dout)
{
    long long h[16];
    for (int i = 0; i < 3; ++i) { hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves), 0, 0, dcyc, dout); hipDeviceSynchronize(); }
    hipMemcpy(h, dcyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
    const double ops = 256.0 * ops_per_rep;
    printf("%-9s waves=%d  cyc/op wave0 %.2f  wave%d %.2f\n", name, waves, h[0] / ops, waves - 1, h[waves - 1] / ops);
}

int main()
{
    long long *dcyc; double *dout;
    hipMalloc(&dcyc, 64 * 8); hipMalloc(&dout, 1024 * 8);
    for (int w = 1; w <= 8; w *= 2) {
        run("dep_b02", dep_b02, w, 4, dcyc, dout);
        run("dep_b00", dep_b00, w, 4, dcyc, dout);
        run("dep_pp02", dep_pp02, w, 4, dcyc, dout);
        run("ind2_nc", ind2_nc, w, 4, dcyc, dout);
        run("ind2_c", ind2_c, w, 4, dcyc, dout);
        run("ind4_nc", ind4_nc, w, 4, dcyc, dout);
        run("mul_b02", mul_b02, w, 4, dcyc, dout);
        run("kahan_nc", kahan_nc, w, 8, dcyc, dout);
        run("kahan_cc", kahan_cc, w, 8, dcyc, dout);
        run("kahan_mix", kahan_mix, w, 10, dcyc, dout);
        run("ind_mul", ind_mul, w, 4, dcyc, dout);
    }
    return 0;
}
