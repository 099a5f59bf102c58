/*
 * icw_cwave.h -- CWAVE (complex wave) file support: the header checks of the reference's CWAVE
 * reader, and a batched GPU CRC32 for the integrity check of CWAVE data parts.
 *
 * Reference interfaces replaced (file:line into the reference tree):
 *   icw_cwave_parse    <- cwave_reader_create (xwave_reader.c:243-300): header field checks, the
 *                         sample format -> unpacker choice (xwave_reader.c:311-335)
 *   icw_crc32_batch    <- crc32init / crc32update / crc32final (crc32.c) as driven by check_cwave
 *                         (gui_cwave.c:82-129): CRC-32 (poly 0xEDB88320, reflected, init and final
 *                         inversion) over the data part, compared with HCWAVE_V2.n_CRC32
 *   icw_cwave_check    <- check_cwave (gui_cwave.c:82-129) on a file image in host or HBM memory
 *   icw_crc32_combine  <- the block-by-block crc32update chaining of check_cwave
 * The CWAVE sample data itself is decoded by icw_process_* with cfg.in_format = ICW_FMT_CW_*.
 */
#ifndef ICW_CWAVE_H_
#define ICW_CWAVE_H_

#include "icw.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ICW_CWAVE_HEADER_BYTES 48      /* 8 + 7 * 4 + 4 + 8: the known part, xwave_reader.c:255-256 */

/* HCWAVE_V2 (cwave.h:48-60).  A V1 header (cwave.h:31-43) has the same field positions, with pad0
 * where V2 has n_CRC32; the reference reads both the same way. */
typedef struct icw_cwave_header {
    char     magic[8];                 /* "cPLXwAVE" */
    uint32_t hsize;                    /* header size, data part starts here */
    uint32_t version;                  /* 1 or 2 */
    uint32_t format;                   /* HCW_FMT_PCM_* 0..3 */
    uint32_t n_channels;               /* 1 or 2 */
    uint32_t n_samples;                /* frames */
    uint32_t sample_rate;
    int32_t  k_M;                      /* external Hilbert FIR order (informational) */
    uint32_t n_crc32;                  /* CRC32 of the data part (V2) */
    double   k_beta;                   /* external Hilbert FIR parameter (informational) */
} icw_cwave_header;

/* Decode and validate the first ICW_CWAVE_HEADER_BYTES of a CWAVE file of file_size bytes, with
 * the reference's checks in the reference's order: magic, hsize (>= 48 and < file size), version
 * (1 or 2), format (<= 3), channels (1..2), n_samples (>= 2 and data part inside the file),
 * sample_rate != 0.  On success fills *h, the ICW_FMT_CW_* input format and the frame size in
 * bytes, and returns ICW_OK; returns ICW_EINVAL for a file the reference refuses. */
int icw_cwave_parse(const void *hdr, size_t hdr_len, int64_t file_size, icw_cwave_header *h,
                    uint32_t *icw_fmt, uint32_t *frame_bytes);

/* CRC-32 of n byte ranges [base + offsets[i], + lengths[i]) on the GPU, one pass over HBM.
 * crc_in[i] (nullable: 0) continues an earlier CRC the way zlib's crc32(crc, buf, len) does;
 * crc_out[i] receives the result.  With ICW_F_DEVICE_PTRS base is a device pointer (the ranges
 * are resident in HBM); otherwise it is a host pointer and the ranges are staged over PCIe.
 * offsets/lengths/crc_in/crc_out are host arrays.  device: HIP device (-1: current);
 * hip_stream: hipStream_t or NULL.  Returns ICW_OK when crc_out is filled. */
int icw_crc32_batch(const void *base, const uint64_t *offsets, const uint64_t *lengths, int n,
                    const uint32_t *crc_in, uint32_t *crc_out, unsigned flags, int device,
                    void *hip_stream);

/* CRC-32 of A||B from crc(A), crc(B) and |B| (GF(2) arithmetic on the host, no data access). */
uint32_t icw_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* check_cwave on a whole CWAVE file image (host or, with ICW_F_DEVICE_PTRS, device memory):
 * parses the header, CRCs the data part (n_samples * frame bytes from hsize) on the GPU.
 * *crc gets the computed CRC; *crc_ok is 1 if it equals n_CRC32, 0 if not, -1 for a V1 file
 * (no CRC stored; the reference only reports the value, gui_cwave.c:124-127). */
int icw_cwave_check(const void *file, uint64_t file_size, unsigned flags, int device, uint32_t *crc,
                    int *crc_ok);

#ifdef __cplusplus
}
#endif
#endif /* ICW_CWAVE_H_ */
