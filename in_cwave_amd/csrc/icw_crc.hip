/*
 * icw_crc.hip -- gfx950 CRC-32 of many byte ranges (the CWAVE data-part check, gui_cwave.c:82-129
 * with crc32.c's CRC: reflected poly 0xEDB88320, register preset ~0, final inversion).
 *
 * HBM-bound byte work, so no GEMM reshaping: the CRC register is linear over GF(2), which lets
 * every lane compute the "raw" CRC (preset 0, no inversion) of its own 256-byte segment with
 * slice-by-16 table lookups (tables in LDS), and the segments be stitched together by
 * multiplying with x^(8*distance) mod P:
 *     raw(A || B) = raw(A) * x^(8|B|)  xor  raw(B)
 * Each range is cut on a 64 KB grid ("cells"); a workgroup of 256 lanes owns one cell (16 x 16 B
 * coalesced loads per lane, all issued before use).  Bytes outside the range read as zero:
 * leading zeros do not change a raw CRC, trailing zeros are undone on the host by x^(-8 pad).
 * Cells combine by atomicXor after a shift by a precomputed x^(8 * CELL * m), so the data pass
 * needs no second kernel.
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

/* raw CRC of one 16 B word with the register at 0: byte j of the word uses table 15 - j */
__device__ __forceinline__ uint32_t icw_crc16b(icw_u32x4 w, const uint32_t (*T)[256])
{
    return T[15][w.x & 255u] ^ T[14][(w.x >> 8) & 255u] ^ T[13][(w.x >> 16) & 255u] ^ T[12][w.x >> 24] ^
           T[11][w.y & 255u] ^ T[10][(w.y >> 8) & 255u] ^ T[9][(w.y >> 16) & 255u] ^ T[8][w.y >> 24] ^
           T[7][w.z & 255u] ^ T[6][(w.z >> 8) & 255u] ^ T[5][(w.z >> 16) & 255u] ^ T[4][w.z >> 24] ^
           T[3][w.w & 255u] ^ T[2][(w.w >> 8) & 255u] ^ T[1][(w.w >> 16) & 255u] ^ T[0][w.w >> 24];
}

/* r * x^(8 * 1024) mod P: the register carried over one 1 KB stride, as 4 byte-table lookups */
__device__ __forceinline__ uint32_t icw_crc_stride(uint32_t r, const uint32_t (*D)[256])
{
    return D[0][r & 255u] ^ D[1][(r >> 8) & 255u] ^ D[2][(r >> 16) & 255u] ^ D[3][r >> 24];
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

/* x^(8 * CELL * m) for m < n: the shift of a cell to the end of its range */
__global__ __launch_bounds__(256) void icw_crc32_powers(const uint32_t *xcell, uint32_t *pw, uint64_t n)
{
    const uint64_t m0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (m0 >= n) return;
    uint64_t m = m0;
    uint32_t k = 0x80000000u;
    for (int b = 0; m; ++b, m >>= 1)
        if (m & 1u) k = icw_gf_mul(k, xcell[b]);
    pw[m0] = k;
}

/* One workgroup per 64 KB cell.  Wave w owns the cell's w-th 16 KB; load j of lane l reads word
 * j*64 + l, so every load instruction is one contiguous 1 KB (coalesced).  A lane's words are
 * 1 KB apart: its register is carried across the other lanes' bytes with one x^8192 multiply
 * (4 lookups) before each word's 16 lookups.  At the end each lane shifts its register to the
 * cell end (x^(8 * distance), per-lane constant) and the cell XOR-reduces. */
__global__ __launch_bounds__(256) void icw_crc32_cells(IcwCrcArgs a)
{
    __shared__ uint32_t T[16][256];
    __shared__ uint32_t D[4][256];
    __shared__ uint32_t red[4];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int i = t; i < 16 * 256; i += 256) T[i >> 8][i & 255] = a.tab[i];
    for (int i = t; i < 4 * 256; i += 256) D[i >> 8][i & 255] = a.dstride[i];
    const uint32_t xs = a.xlane[t];      /* x^(8 * (16384 (3 - w) + 16 (63 - l))) */
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
        const uint64_t wbase = cell * ICW_CRC_CELL + (uint64_t)wv * 16384u;
        uint32_t c = 0;
        if (wbase >= B.start && wbase + 16384u <= B.end) {
            const icw_u32x4 *p = (const icw_u32x4 *)(a.base + wbase) + lane;
            icw_u32x4 w[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) w[j] = __builtin_nontemporal_load(p + j * 64);
#pragma unroll
            for (int j = 0; j < 16; ++j) c = icw_crc_stride(c, D) ^ icw_crc16b(w[j], T);
        } else if (wbase + 16384u > B.start && wbase < B.end) {
            /* range edge: bytes outside the range read as zero; words wholly outside are not
             * loaded (a partially covered aligned 16 B word never crosses a page) */
            for (int j = 0; j < 16; ++j) {
                const uint64_t wa = wbase + 16u * (uint64_t)(j * 64 + lane);
                icw_u32x4 w = {0u, 0u, 0u, 0u};
                if (wa + 16 > B.start && wa < B.end) {
                    w = *(const icw_u32x4 *)(a.base + wa);
                    w.x = icw_mask_dword(w.x, wa, B.start, B.end);
                    w.y = icw_mask_dword(w.y, wa + 4, B.start, B.end);
                    w.z = icw_mask_dword(w.z, wa + 8, B.start, B.end);
                    w.w = icw_mask_dword(w.w, wa + 12, B.start, B.end);
                }
                c = icw_crc_stride(c, D) ^ icw_crc16b(w, T);
            }
        }
        uint32_t v = c ? icw_gf_mul(c, xs) : 0u;
        for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off);
        if (lane == 0) red[wv] = v;
        __syncthreads();
        if (t == 0) {
            const uint32_t r = red[0] ^ red[1] ^ red[2] ^ red[3];
            if (r) atomicXor(&a.raw[B.index], icw_gf_mul(r, a.pw[B.last_cell - cell]));
        }
        __syncthreads();
    }
}

extern "C" hipError_t icw_launch_crc32(const IcwCrcArgs *a, uint64_t max_cells, int n_cu, hipStream_t st)
{
    if (max_cells) {
        hipLaunchKernelGGL(icw_crc32_powers, dim3((unsigned)((max_cells + 255) / 256)), dim3(256), 0, st, a->xcell,
                           a->pw, max_cells);
    }
    uint64_t blocks = (uint64_t)n_cu * 8;
    if (a->n_chunks < blocks) blocks = a->n_chunks;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(icw_crc32_cells, dim3((unsigned)blocks), dim3(256), 0, st, *a);
    return hipGetLastError();
}
