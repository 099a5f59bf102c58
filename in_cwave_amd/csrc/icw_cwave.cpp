/*
 * icw_cwave.cpp -- CWAVE header checks and the host side of the GPU CRC-32 (include/icw_cwave.h).
 *
 * Mirrors: cwave_reader_create (xwave_reader.c:243-300, 311-335), crc32init / crc32update /
 * crc32final (crc32.c) as used by check_cwave (gui_cwave.c:82-129).  The CRC data pass runs in
 * icw_crc32_cells (icw_crc.hip); the host only does GF(2) arithmetic on 32-bit values.
 */
#include <hip/hip_runtime_api.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/icw_cwave.h"
#include "icw_crc.h"

extern "C" hipError_t icw_launch_crc32(const IcwCrcArgs *a, uint64_t max_cells, int n_cu, hipStream_t st);

namespace {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kOne = 0x80000000u;        /* x^0 in the reflected representation */
constexpr uint32_t kXinv = 0xDB710641u;       /* x^-1 mod P: (P - 1) / x, reflected */

uint32_t gf_mul(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 0; i < 32; ++i) {
        if ((a >> (31 - i)) & 1u) p ^= b;
        b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
    }
    return p;
}

/* base^n by square-and-multiply */
uint32_t gf_pow(uint32_t base, uint64_t n)
{
    uint32_t r = kOne;
    while (n) {
        if (n & 1u) r = gf_mul(r, base);
        base = gf_mul(base, base);
        n >>= 1;
    }
    return r;
}

uint32_t x8n(uint64_t n) { return gf_pow(1u << 23, n); }                 /* x^(8n) */
uint32_t xinv8n(uint64_t n) { return gf_pow(gf_pow(kXinv, 8), n); }      /* x^(-8n) */

struct Tables {
    uint32_t tab[16][256];
    uint32_t dstride[4][256];
    uint32_t xlane[256];
    uint32_t xcell[64];
};

const Tables &tables()
{
    static Tables t;
    static std::once_flag once;
    std::call_once(once, [] {
        for (uint32_t b = 0; b < 256; ++b) {      /* the table of crc32init (crc32.c) */
            uint32_t c = b;
            for (int j = 0; j < 8; ++j) c = (c >> 1) ^ ((c & 1u) ? kPoly : 0u);
            t.tab[0][b] = c;
        }
        for (int k = 1; k < 16; ++k)
            for (int b = 0; b < 256; ++b) t.tab[k][b] = (t.tab[k - 1][b] >> 8) ^ t.tab[0][t.tab[k - 1][b] & 255u];
        /* r * x^8192 is linear in r: one table per byte of r (bit i of r is x^(31-i)) */
        const uint32_t k1k = x8n(1024);
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b) t.dstride[k][b] = gf_mul(b << (8 * k), k1k);
        for (int w = 0; w < 4; ++w)
            for (int l = 0; l < 64; ++l) t.xlane[w * 64 + l] = x8n(16384ull * (3 - w) + 16ull * (63 - l));
        t.xcell[0] = x8n(ICW_CRC_CELL);
        for (int k = 1; k < 64; ++k) t.xcell[k] = gf_mul(t.xcell[k - 1], t.xcell[k - 1]);
    });
    return t;
}

uint32_t le32(const unsigned char *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

}  // namespace

extern "C" {

uint32_t icw_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    return gf_mul(x8n(len_b), crc_a) ^ crc_b;
}

int icw_cwave_parse(const void *hdr, size_t hdr_len, int64_t file_size, icw_cwave_header *h, uint32_t *icw_fmt,
                    uint32_t *frame_bytes)
{
    /* supported one channel sample lengths (cw_slen, xwave_reader.c:246-252) */
    static const uint32_t cw_slen[4] = {16, 4, 6, 8};
    static const char magic[8] = {'c', 'P', 'L', 'X', 'w', 'A', 'V', 'E'};
    if (!hdr || !h) return ICW_EINVAL;
    const unsigned char *b = (const unsigned char *)hdr;
    const int64_t hsize = ICW_CWAVE_HEADER_BYTES;
    memset(h, 0, sizeof(*h));
    if (file_size < hsize || (int64_t)hdr_len < hsize) return ICW_EINVAL;
    memcpy(h->magic, b, 8);
    if (memcmp(h->magic, magic, 8)) return ICW_EINVAL;
    h->hsize = le32(b + 8);
    if ((int64_t)h->hsize < hsize || (int64_t)h->hsize >= file_size) return ICW_EINVAL;
    h->version = le32(b + 12);
    if (h->version != 1 && h->version != 2) return ICW_EINVAL;
    h->format = le32(b + 16);
    if (h->format > 3) return ICW_EINVAL;
    h->n_channels = le32(b + 20);
    if (h->n_channels > 2 || h->n_channels == 0) return ICW_EINVAL;
    h->n_samples = le32(b + 24);
    if (h->n_samples < 2) return ICW_EINVAL;                           /* MIN_FILE_SAMPLES */
    if ((int64_t)h->n_samples * h->n_channels * cw_slen[h->format] + h->hsize > file_size) return ICW_EINVAL;
    h->sample_rate = le32(b + 28);
    h->k_M = (int32_t)le32(b + 32);
    h->n_crc32 = le32(b + 36);
    uint64_t kb = (uint64_t)le32(b + 40) | ((uint64_t)le32(b + 44) << 32);
    memcpy(&h->k_beta, &kb, 8);
    if (h->sample_rate == 0) return ICW_EINVAL;
    if (icw_fmt) *icw_fmt = ICW_FMT_CW_F64 + h->format;
    if (frame_bytes) *frame_bytes = cw_slen[h->format] * h->n_channels;
    return ICW_OK;
}

int icw_crc32_batch(const void *base, const uint64_t *offsets, const uint64_t *lengths, int n, const uint32_t *crc_in,
                    uint32_t *crc_out, unsigned flags, int device, void *hip_stream)
{
    if (n < 0 || (n > 0 && (!offsets || !lengths || !crc_out))) return ICW_EINVAL;
    if (n == 0) return ICW_OK;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return ICW_EDEVICE;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return ICW_EDEVICE;
    int n_cu = 256;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n_cu = 256;
    hipStream_t st = (hipStream_t)hip_stream;
    const bool devp = flags & ICW_F_DEVICE_PTRS;

    /* device view of the ranges: 16 B aligned base, offsets relative to it */
    std::vector<uint64_t> start(n), end(n);
    unsigned char *stage = nullptr;
    const unsigned char *dbase;
    if (devp) {
        const uintptr_t b = (uintptr_t)base, al = b & ~(uintptr_t)15;
        dbase = (const unsigned char *)al;
        for (int i = 0; i < n; ++i) {
            start[i] = offsets[i] + (b - al);
            end[i] = start[i] + lengths[i];
        }
    } else {
        /* stage the host ranges back to back (16 B aligned) */
        uint64_t tot = 0;
        for (int i = 0; i < n; ++i) {
            start[i] = tot;
            end[i] = tot + lengths[i];
            tot = (end[i] + 15) & ~(uint64_t)15;
        }
        if (hipMalloc((void **)&stage, tot ? tot : 16) != hipSuccess) return ICW_ENOMEM;
        for (int i = 0; i < n; ++i)
            if (lengths[i] && hipMemcpyAsync(stage + start[i], (const unsigned char *)base + offsets[i], lengths[i],
                                             hipMemcpyHostToDevice, st) != hipSuccess) {
                (void)hipFree(stage);
                return ICW_EDEVICE;
            }
        dbase = stage;
    }
    std::vector<IcwCrcBuf> bufs;
    uint64_t n_chunks = 0, max_cells = 0;
    for (int i = 0; i < n; ++i) {
        if (!lengths[i]) continue;
        IcwCrcBuf B;
        memset(&B, 0, sizeof(B));
        B.start = start[i];
        B.end = end[i];
        B.cell0 = start[i] / ICW_CRC_CELL;
        B.last_cell = (end[i] - 1) / ICW_CRC_CELL;
        B.first_chunk = n_chunks;
        B.index = (uint32_t)i;
        n_chunks += B.last_cell - B.cell0 + 1;
        if (B.last_cell - B.cell0 + 1 > max_cells) max_cells = B.last_cell - B.cell0 + 1;
        bufs.push_back(B);
    }
    const Tables &T = tables();
    /* one device block: tables | raw[n] | bufs | pw[max_cells] */
    const size_t tab_b = sizeof(Tables), raw_b = (size_t)n * 4, buf_b = bufs.size() * sizeof(IcwCrcBuf);
    const size_t raw_off = (tab_b + 255) & ~(size_t)255, buf_off = (raw_off + raw_b + 255) & ~(size_t)255;
    const size_t pw_off = (buf_off + buf_b + 255) & ~(size_t)255;
    unsigned char *blk = nullptr;
    int rc = ICW_OK;
    std::vector<uint32_t> raw(n, 0);
    if (hipMalloc((void **)&blk, pw_off + max_cells * 4 + 16) != hipSuccess) rc = ICW_ENOMEM;
    if (rc == ICW_OK &&
        (hipMemcpyAsync(blk, &T, tab_b, hipMemcpyHostToDevice, st) != hipSuccess ||
         hipMemsetAsync(blk + raw_off, 0, raw_b, st) != hipSuccess ||
         (buf_b && hipMemcpyAsync(blk + buf_off, bufs.data(), buf_b, hipMemcpyHostToDevice, st) != hipSuccess)))
        rc = ICW_EDEVICE;
    if (rc == ICW_OK && !bufs.empty()) {
        IcwCrcArgs a;
        memset(&a, 0, sizeof(a));
        a.base = dbase;
        a.bufs = (const IcwCrcBuf *)(blk + buf_off);
        a.n_bufs = (int32_t)bufs.size();
        a.n_chunks = n_chunks;
        a.tab = (const uint32_t *)(blk + offsetof(Tables, tab));
        a.dstride = (const uint32_t *)(blk + offsetof(Tables, dstride));
        a.xlane = (const uint32_t *)(blk + offsetof(Tables, xlane));
        a.xcell = (const uint32_t *)(blk + offsetof(Tables, xcell));
        a.pw = (uint32_t *)(blk + pw_off);
        a.raw = (uint32_t *)(blk + raw_off);
        if (icw_launch_crc32(&a, max_cells, n_cu, st) != hipSuccess) rc = ICW_EDEVICE;
    }
    if (rc == ICW_OK && (hipMemcpyAsync(raw.data(), blk + raw_off, raw_b, hipMemcpyDeviceToHost, st) != hipSuccess ||
                         hipStreamSynchronize(st) != hipSuccess))
        rc = ICW_EDEVICE;
    if (blk) (void)hipFree(blk);
    if (stage) (void)hipFree(stage);
    if (rc != ICW_OK) return rc;
    for (int i = 0; i < n; ++i) {
        const uint32_t c0 = crc_in ? crc_in[i] : 0u;
        if (!lengths[i]) { crc_out[i] = c0; continue; }
        const uint64_t pad = (end[i] - 1) / ICW_CRC_CELL * ICW_CRC_CELL + ICW_CRC_CELL - end[i];
        const uint32_t r = gf_mul(raw[i], xinv8n(pad));
        /* register preset ~crc_in shifted over the range, plus the data's raw CRC, inverted */
        crc_out[i] = ~(gf_mul(~c0, x8n(lengths[i])) ^ r);
    }
    return ICW_OK;
}

int icw_cwave_check(const void *file, uint64_t file_size, unsigned flags, int device, uint32_t *crc, int *crc_ok)
{
    if (!file || !crc || !crc_ok) return ICW_EINVAL;
    unsigned char hdr[ICW_CWAVE_HEADER_BYTES];
    if (file_size < sizeof(hdr)) return ICW_EINVAL;
    if (flags & ICW_F_DEVICE_PTRS) {
        if (device >= 0 && hipSetDevice(device) != hipSuccess) return ICW_EDEVICE;
        if (hipMemcpy(hdr, file, sizeof(hdr), hipMemcpyDeviceToHost) != hipSuccess) return ICW_EDEVICE;
    } else {
        memcpy(hdr, file, sizeof(hdr));
    }
    icw_cwave_header h;
    uint32_t fmt = 0, fb = 0;
    int rc = icw_cwave_parse(hdr, sizeof(hdr), (int64_t)file_size, &h, &fmt, &fb);
    if (rc != ICW_OK) return rc;
    const uint64_t off = h.hsize, len = (uint64_t)h.n_samples * fb;
    rc = icw_crc32_batch(file, &off, &len, 1, nullptr, crc, flags, device, nullptr);
    if (rc != ICW_OK) return rc;
    *crc_ok = h.version > 1 ? (*crc == h.n_crc32 ? 1 : 0) : -1;
    return ICW_OK;
}

}  /* extern "C" */
