/*
 * icw_crc.hip -- gfx950 CRC-32 of many byte ranges (the CWAVE data-part check, gui_cwave.c:82-129
 * with crc32.c's CRC: reflected poly 0xEDB88320, register preset ~0, final inversion).
 *
 * HBM-bound byte work, so no GEMM reshaping: the CRC register is linear over GF(2), which lets
 * every lane compute the "raw" CRC (preset 0, no inversion) of its own 256-byte segment with
 * slice-by-16 table lookups (tables in LDS), and the segments be stitched together by
 * multiplying with x^(8*distance) mod P:
 *     raw(A || B) = raw(A) * x^(8|B|)  xor  raw(B)
 * Each range is cut on a 64 KB grid ("cells"); a workgroup of 256 lanes owns one cell, lane t one
 * 256 B segment of it (16 x 16 B coalesced-by-line loads, all issued before use).  Bytes outside
 * the range read as zero: leading zeros do not change a raw CRC, trailing zeros are undone on the
 * host by x^(-8 pad).  Cells combine by atomicXor, so the kernel needs no second pass.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icw_crc.h"

#define ICW_CRC_POLY 0xEDB88320u

typedef uint32_t icw_u32x4 __attribute__((ext_vector_type(4)));

/* a * b mod P in the reflected representation (bit 31 = x^0), zlib's multmodp without early exit */
__device__ __forceinline__ uint32_t icw_gf_mul(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        p ^= ((a >> (31 - i)) & 1u) ? b : 0u;
        b = (b >> 1) ^ ((b & 1u) ? ICW_CRC_POLY : 0u);
    }
    return p;
}

/* 16 bytes through the register: byte j of the word uses table 15 - j (slice-by-16) */
__device__ __forceinline__ uint32_t icw_crc16b(uint32_t c, icw_u32x4 w, const uint32_t (*T)[256])
{
    const uint32_t a = w.x ^ c;
    return T[15][a & 255u] ^ T[14][(a >> 8) & 255u] ^ T[13][(a >> 16) & 255u] ^ T[12][a >> 24] ^
           T[11][w.y & 255u] ^ T[10][(w.y >> 8) & 255u] ^ T[9][(w.y >> 16) & 255u] ^ T[8][w.y >> 24] ^
           T[7][w.z & 255u] ^ T[6][(w.z >> 8) & 255u] ^ T[5][(w.z >> 16) & 255u] ^ T[4][w.z >> 24] ^
           T[3][w.w & 255u] ^ T[2][(w.w >> 8) & 255u] ^ T[1][(w.w >> 16) & 255u] ^ T[0][w.w >> 24];
}

/* keep the bytes of a 16 B word at addresses [lo, hi), zero the rest */
__device__ __forceinline__ uint32_t icw_mask_dword(uint32_t v, uint64_t a, uint64_t lo, uint64_t hi)
{
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
        if (a + b >= lo && a + b < hi) m |= 0xffu << (8 * b);
    return v & m;
}

__global__ __launch_bounds__(256) void icw_crc32_cells(IcwCrcArgs a)
{
    __shared__ uint32_t T[16][256];
    __shared__ uint32_t red[4];
    const int t = threadIdx.x;
    for (int i = t; i < 16 * 256; i += 256) T[i >> 8][i & 255] = a.tab[i];
    const uint32_t xs = a.xseg[255 - t];   /* x^(8*256*(255-t)): segment end -> cell end */
    __syncthreads();

    for (uint64_t chunk = blockIdx.x; chunk < a.n_chunks; chunk += gridDim.x) {
        /* which range: last i with first_chunk <= chunk (wave-uniform binary search) */
        int lo_i = 0, hi_i = a.n_bufs - 1;
        while (lo_i < hi_i) {
            const int mid = (lo_i + hi_i + 1) >> 1;
            if (a.bufs[mid].first_chunk <= chunk) lo_i = mid;
            else hi_i = mid - 1;
        }
        const IcwCrcBuf B = a.bufs[lo_i];
        const uint64_t cell = B.cell0 + (chunk - B.first_chunk);
        const uint64_t seg_lo = cell * ICW_CRC_CELL + (uint64_t)t * ICW_CRC_SEG;
        const uint64_t seg_hi = seg_lo + ICW_CRC_SEG;
        uint32_t c = 0;
        if (seg_lo >= B.start && seg_hi <= B.end) {
            const icw_u32x4 *p = (const icw_u32x4 *)(a.base + seg_lo);
            icw_u32x4 w[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) w[j] = __builtin_nontemporal_load(p + j);
#pragma unroll
            for (int j = 0; j < 16; ++j) c = icw_crc16b(c, w[j], T);
        } else if (seg_hi > B.start && seg_lo < B.end) {
            /* range edge: aligned 16 B words, bytes outside the range zeroed; words wholly
             * outside are not loaded (a partial word never crosses a page) */
            for (int j = 0; j < 16; ++j) {
                const uint64_t wa = seg_lo + 16u * (uint64_t)j;
                icw_u32x4 w = {0u, 0u, 0u, 0u};
                if (wa + 16 > B.start && wa < B.end) {
                    w = *(const icw_u32x4 *)(a.base + wa);
                    w.x = icw_mask_dword(w.x, wa, B.start, B.end);
                    w.y = icw_mask_dword(w.y, wa + 4, B.start, B.end);
                    w.z = icw_mask_dword(w.z, wa + 8, B.start, B.end);
                    w.w = icw_mask_dword(w.w, wa + 12, B.start, B.end);
                }
                c = icw_crc16b(c, w, T);
            }
        }
        uint32_t v = icw_gf_mul(c, xs);
        for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
        if ((t & 63) == 0) red[t >> 6] = v;
        __syncthreads();
        if (t == 0) {
            uint32_t r = red[0] ^ red[1] ^ red[2] ^ red[3];
            /* cell end -> the range's last cell end: x^(8 * CELL * m) by square-and-multiply */
            uint64_t m = B.last_cell - cell;
            uint32_t k = 0x80000000u;
            for (int b = 0; m; ++b, m >>= 1)
                if (m & 1u) k = icw_gf_mul(k, a.xcell[b]);
            if (r) atomicXor(&a.raw[B.index], icw_gf_mul(r, k));
        }
        __syncthreads();
    }
}

extern "C" hipError_t icw_launch_crc32(const IcwCrcArgs *a, int n_cu, hipStream_t st)
{
    uint64_t blocks = (uint64_t)n_cu * 8;
    if (a->n_chunks < blocks) blocks = a->n_chunks;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(icw_crc32_cells, dim3((unsigned)blocks), dim3(256), 0, st, *a);
    return hipGetLastError();
}
