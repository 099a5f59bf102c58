// cumask_probe.hip -- where do the workgroups of a CU-masked stream run?  (diagnostic tool)
// Builds the same masks as icw_host.cpp cu_split (K1 on every (n / k)-th CU bit, the rest on the
// complement), launches one-wave workgroups on each stream and records HW_REG_XCC_ID and
// HW_REG_HW_ID (SE, SH, CU, SIMD) per workgroup.
//   hipcc --offload-arch=gfx950 -O2 -o tools/cumask_probe tools/cumask_probe.hip
//   ./tools/cumask_probe [k1_cus=32]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <map>
#include <set>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__global__ void where(unsigned *out, int spin)
{
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    long long t0 = clock64();
    while (clock64() - t0 < spin) { }
    if (threadIdx.x == 0) {
        out[blockIdx.x * 2] = hw;
        out[blockIdx.x * 2 + 1] = xcc;
    }
}

static void run(const char *name, hipStream_t st, int nblk)
{
    unsigned *d, *h = (unsigned *)malloc(sizeof(unsigned) * 2 * nblk);
    hipMalloc(&d, sizeof(unsigned) * 2 * nblk);
    hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, st, d, 200000);
    hipStreamSynchronize(st);
    hipMemcpy(h, d, sizeof(unsigned) * 2 * nblk, hipMemcpyDeviceToHost);
    std::map<int, std::set<int>> cus;   // xcc -> {se*64 + sh*16 + cu}
    std::map<int, std::set<int>> ses;   // xcc -> {se*2 + sh}
    for (int b = 0; b < nblk; ++b) {
        unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        cus[xcc].insert(se * 64 + sh * 16 + cu);
        ses[xcc].insert(se * 2 + sh);
    }
    printf("%s:", name);
    int tot = 0;
    for (auto &kv : cus) {
        printf(" x%d:%zu/%zu", kv.first, kv.second.size(), ses[kv.first].size());
        tot += (int)kv.second.size();
    }
    printf("  (distinct CUs %d; per XCC: CUs/SE-SH groups)\n", tot);
    hipFree(d);
    free(h);
}

int main(int argc, char **argv)
{
    int k = argc > 1 ? atoi(argv[1]) : 32;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int n = p.multiProcessorCount, words = (n + 31) / 32;
    std::vector<uint32_t> mk(words, 0u), mr(words, 0u);
    std::vector<char> used(n, 0);
    for (int i = 0; i < k; ++i) used[(int)((long)i * n / k)] = 1;
    for (int cu = 0; cu < n; ++cu) (used[cu] ? mk : mr)[cu / 32] |= 1u << (cu % 32);
    hipStream_t sk, sr, sp;
    hipExtStreamCreateWithCUMask(&sk, words, mk.data());
    hipExtStreamCreateWithCUMask(&sr, words, mr.data());
    hipStreamCreate(&sp);
    // contiguous low bits as a second pattern: which CUs does mask bit range [0, k) select?
    std::vector<uint32_t> ml(words, 0u);
    for (int cu = 0; cu < k; ++cu) ml[cu / 32] |= 1u << (cu % 32);
    hipStream_t sl;
    hipExtStreamCreateWithCUMask(&sl, words, ml.data());
    // icw_host.cpp layout: bit b -> XCC b % 8; per XCC k/8 CUs at evenly spaced in-XCC indices
    std::vector<uint32_t> mx(words, 0u), mxr(words, 0u);
    const int per = k / 8, step = (n / 8) / (per > 0 ? per : 1);
    for (int i = 0; i < k; ++i) { int b = (i % 8) + 8 * ((i / 8) * step); mx[b / 32] |= 1u << (b % 32); }
    for (int w = 0; w < words; ++w) mxr[w] = ~mx[w];
    hipStream_t sx, sxr;
    hipExtStreamCreateWithCUMask(&sx, words, mx.data());
    hipExtStreamCreateWithCUMask(&sxr, words, mxr.data());
    printf("CUs %d, k1 mask = every %d-th bit (%d bits)\n", n, n / k, k);
    run("spread k1     ", sx, 4096);
    run("spread rest   ", sxr, 4096);
    run("plain stream  ", sp, 4096);
    run("k1 mask       ", sk, 4096);
    run("rest mask     ", sr, 4096);
    run("low k bits    ", sl, 4096);
    return 0;
}
