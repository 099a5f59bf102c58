/*
 * icw_crc.h -- structures shared by the CRC-32 host code (icw_cwave.cpp) and kernel (icw_crc.hip).
 */
#ifndef ICW_CRC_H_
#define ICW_CRC_H_

#include <stdint.h>

#define ICW_CRC_CELL 65536u      /* bytes per workgroup cell */

/* one non-empty byte range [start, end), offsets from the (16 B aligned) base */
struct IcwCrcBuf {
    uint64_t start, end;
    uint64_t cell0, last_cell;     /* first / last 64 KB cell the range touches */
    uint64_t first_chunk;          /* index of its first cell in the launch's chunk list */
    uint32_t index;                /* slot in raw[] */
    uint32_t pad_;
};

struct IcwCrcArgs {
    const unsigned char *base;
    const IcwCrcBuf *bufs;
    int32_t n_bufs;
    uint64_t n_chunks;
    const uint32_t *tab;           /* [16][256] slice-by-16 tables */
    const uint32_t *dstride;       /* [4][256] byte tables of r -> r * x^(8*1024) */
    const uint32_t *xlane;         /* [256] x^(8 * (16384 (3 - w) + 16 (63 - l))), t = 64 w + l */
    const uint32_t *xcell;         /* [64] x^(8*CELL*2^k) mod P */
    uint32_t *pw;                  /* [max cells per range] x^(8*CELL*m), filled by icw_crc32_powers */
    uint32_t *raw;                 /* [n] raw CRC (preset 0, no inversion), padded to the cell grid */
};

#endif
