// tools/dpp_probe.hip -- gfx950 issue-cost probe for a row-broadcast Kahan step.
// Question: can the Kahan term operand t_i come from another lane of the row through a DPP
// row_newbcast on v_fmac_f64 (Y = t*1 + (-C)) at the cost of a plain v_add_f64, and what do the
// 32-bit v_cndmask_b32 (ring write / reject) and a v_mul_f64 cost between the dependent adds?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/dpp_probe tools/dpp_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP "256"
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","s40","s41"

#define PROBE(name, body)                                                                     \
__global__ void name(long long *cyc, double *out)                                           \
{                                                                                           \
    long long t0, t1;                                                                       \
    double r;                                                                               \
    asm volatile(INIT ::: CLOB);                                                            \
    t0 = clock64();                                                                         \
    asm volatile(".rept " REP "\n" body "\n.endr" ::: CLOB);                                \
    t1 = clock64();                                                                         \
    asm volatile("v_mov_b64 %0, v[4:5]" : "=v"(r) :: CLOB);                                 \
    out[threadIdx.x] = r;                                                                   \
    if (threadIdx.x % 64 == 0) cyc[threadIdx.x / 64] = t1 - t0;                             \
}

#define INIT "v_mov_b64 v[0:1], 1.0\n v_mov_b64 v[2:3], 1.0\n v_mov_b64 v[4:5], 1.0\n v_mov_b64 v[6:7], 0.5\n" \
             "v_mov_b64 v[8:9], 0.5\n v_mov_b64 v[10:11], 0.5\n v_mov_b64 v[12:13], 0.5\n v_mov_b64 v[14:15], 1.0\n" \
             "s_mov_b64 s[40:41], 0x10001"

/* reference: plain Kahan step, 4 dependent adds (S v0 / T v6 alternate) */
PROBE(kahan_plain,
      "v_add_f64 v[2:3], v[10:11], -v[8:9]\n v_add_f64 v[6:7], v[0:1], v[2:3]\n v_add_f64 v[4:5], v[6:7], -v[0:1]\n v_add_f64 v[8:9], v[4:5], -v[2:3]\n"
      "v_add_f64 v[2:3], v[10:11], -v[8:9]\n v_add_f64 v[0:1], v[6:7], v[2:3]\n v_add_f64 v[4:5], v[0:1], -v[6:7]\n v_add_f64 v[8:9], v[4:5], -v[2:3]")
/* row-broadcast Kahan step: Y = fma(t[lane 3 of the row], 1.0, NC) in NC's register v[8:9];
 * T = S + Y; D = T - S; NC = Y - D */
PROBE(kahan_dpp,
      "v_fmac_f64_dpp v[8:9], v[10:11], v[14:15] row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_add_f64 v[6:7], v[0:1], v[8:9]\n v_add_f64 v[4:5], v[6:7], -v[0:1]\n v_add_f64 v[8:9], v[8:9], -v[4:5]\n"
      "v_fmac_f64_dpp v[8:9], v[10:11], v[14:15] row_newbcast:7 row_mask:0xf bank_mask:0xf\n v_add_f64 v[0:1], v[6:7], v[8:9]\n v_add_f64 v[4:5], v[0:1], -v[6:7]\n v_add_f64 v[8:9], v[8:9], -v[4:5]")
/* a dependent chain of DPP fmacs alone */
PROBE(fmac_dpp_dep,
      "v_fmac_f64_dpp v[4:5], v[10:11], v[14:15] row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp v[4:5], v[10:11], v[14:15] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f64_dpp v[4:5], v[10:11], v[14:15] row_newbcast:9 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp v[4:5], v[10:11], v[14:15] row_newbcast:1 row_mask:0xf bank_mask:0xf")
/* 4 dependent adds + 2 independent v_cndmask_b32 (6 instructions) */
PROBE(add4_cnd2,
      "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_cndmask_b32 v12, v12, v0, s[40:41]\n v_add_f64 v[4:5], v[4:5], v[6:7]\n v_cndmask_b32 v13, v13, v1, s[40:41]\n"
      "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[4:5], v[4:5], v[6:7]")
/* 4 dependent adds + 1 independent v_mul_f64 (5 instructions) */
PROBE(add4_mul1,
      "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_mul_f64 v[10:11], v[12:13], v[14:15]\n v_add_f64 v[4:5], v[4:5], v[6:7]\n"
      "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[4:5], v[4:5], v[6:7]")
/* independent 32-bit ops only */
PROBE(cnd_only,
      "v_cndmask_b32 v12, v12, v0, s[40:41]\n v_cndmask_b32 v13, v13, v1, s[40:41]\n v_cndmask_b32 v2, v2, v0, s[40:41]\n v_cndmask_b32 v3, v3, v1, s[40:41]")
/* 4 dependent adds + 2 SALU ops */
PROBE(add4_salu2,
      "v_add_f64 v[4:5], v[4:5], v[6:7]\n s_add_u32 s40, s40, 1\n v_add_f64 v[4:5], v[4:5], v[6:7]\n s_add_u32 s41, s41, 1\n"
      "v_add_f64 v[4:5], v[4:5], v[6:7]\n v_add_f64 v[4:5], v[4:5], v[6:7]")

typedef void (*K)(long long *, double *);

static void run(const char *name, K k, int waves, double per_rep, const char *unit, long long *dcyc, double *dout)
{
    long long h[16];
    for (int i = 0; i < 3; ++i) { hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves), 0, 0, dcyc, dout); hipDeviceSynchronize(); }
    hipMemcpy(h, dcyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
    printf("%-13s waves=%d  cycles per %s: wave0 %.2f  wave%d %.2f\n", name, waves, unit,
           h[0] / (256.0 * per_rep), waves - 1, h[waves - 1] / (256.0 * per_rep));
}

int main()
{
    long long *dcyc; double *dout;
    hipMalloc(&dcyc, 64 * 8); hipMalloc(&dout, 1024 * 8);
    for (int w = 1; w <= 4; w *= 4) {
        run("kahan_plain", kahan_plain, w, 2, "Kahan step (4 adds)", dcyc, dout);
        run("kahan_dpp", kahan_dpp, w, 2, "Kahan step (fmac_dpp + 3 adds)", dcyc, dout);
        run("fmac_dpp_dep", fmac_dpp_dep, w, 4, "dependent fmac_dpp", dcyc, dout);
        run("add4_cnd2", add4_cnd2, w, 1, "4 dep adds + 2 cndmask", dcyc, dout);
        run("add4_mul1", add4_mul1, w, 1, "4 dep adds + 1 mul", dcyc, dout);
        run("cnd_only", cnd_only, w, 4, "cndmask", dcyc, dout);
        run("add4_salu2", add4_salu2, w, 1, "4 dep adds + 2 salu", dcyc, dout);
    }
    return 0;
}
