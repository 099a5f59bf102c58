/*
 * ref_unpack.c -- TEST INFRASTRUCTURE ONLY (a checker; nothing in the product loads it).
 *
 * An original driver that compiles the REFERENCE's own little-endian unpackers and CWAVE header
 * layout where they lie: `make -C oracle ref` builds it with -I /root/reference/src into
 * oracle/_ref/libref_unpack.so (git-ignored).  Both headers include only <stdint.h>
 * (unpack_lsb.h:39, cwave.h:27), so no stand-in header is involved.  tools/gen_golden.py runs it on
 * random and edge-case byte patterns and commits the results (tests/golden/unpack_ref.npz,
 * cwave_layout.json); the oracle's unpackers (icw_oracle.c unpack1 / unpack_iq) and the device's
 * (K0, ICW_F_DEBUG_INPUT; the CWAVE path) are checked against those fixtures.
 *
 * Pinned here: unpack_int16 / unpack_int24 / unpack_int32 / unpack_float / unpack_double
 * (unpack_lsb.h:53-125) bit for bit, and sizeof / offsetof of HCWAVE_V1 / HCWAVE_V2 with the
 * HCW_* constants (cwave.h:31-87).  Not pinned here: the sample scaling of xwave_reader.c:205-239
 * (i24 / 256, i32 / 65536, f32 * 32768, u8 256 (b - 128)) -- that file includes <windows.h>.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "unpack_lsb.h"
#include "cwave.h"

enum { REF_I16 = 0, REF_I24 = 1, REF_I32 = 2, REF_F32 = 3, REF_F64 = 4 };

/* n samples of `kind` packed back to back at src (2, 3, 4, 4, 8 bytes each); dst gets the decoded
 * value's bits: int32 for the integer kinds (sign-extended), the float's / double's own bits for
 * the floating kinds (a register move, no conversion that could quiet a signalling NaN) */
int ref_unpack_batch(int kind, const uint8_t *src, size_t n, void *dst)
{
    static const size_t sz[5] = {2, 3, 4, 4, 8};
    if (kind < 0 || kind > 4) return -1;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *p = src + i * sz[kind];
        switch (kind) {
        case REF_I16: ((int32_t *)dst)[i] = unpack_int16(p); break;
        case REF_I24: ((int32_t *)dst)[i] = unpack_int24(p); break;
        case REF_I32: ((int32_t *)dst)[i] = unpack_int32(p); break;
        case REF_F32: { float f = unpack_float(p); memcpy((uint32_t *)dst + i, &f, 4); break; }
        case REF_F64: { double d = unpack_double(p); memcpy((uint64_t *)dst + i, &d, 8); break; }
        }
    }
    return 0;
}

/* the header layout: {sizeof, offsetof each field} of HCWAVE_V1 then HCWAVE_V2, then the constants */
int ref_cwave_layout(int64_t *out, int n)
{
    const int64_t v[] = {
        (int64_t)sizeof(HCWAVE_V1), offsetof(HCWAVE_V1, magic), offsetof(HCWAVE_V1, hsize),
        offsetof(HCWAVE_V1, version), offsetof(HCWAVE_V1, format), offsetof(HCWAVE_V1, n_channels),
        offsetof(HCWAVE_V1, n_samples), offsetof(HCWAVE_V1, sample_rate), offsetof(HCWAVE_V1, k_M),
        offsetof(HCWAVE_V1, pad0), offsetof(HCWAVE_V1, k_beta),
        (int64_t)sizeof(HCWAVE_V2), offsetof(HCWAVE_V2, magic), offsetof(HCWAVE_V2, hsize),
        offsetof(HCWAVE_V2, version), offsetof(HCWAVE_V2, format), offsetof(HCWAVE_V2, n_channels),
        offsetof(HCWAVE_V2, n_samples), offsetof(HCWAVE_V2, sample_rate), offsetof(HCWAVE_V2, k_M),
        offsetof(HCWAVE_V2, n_CRC32), offsetof(HCWAVE_V2, k_beta),
        HCW_VERSION_BAD, HCW_VERSION_V1, HCW_VERSION_V2, HCW_VERSION_CUR,
        (int64_t)HCW_FMT_BAD_FMT, HCW_FMT_PCM_DBL64, HCW_FMT_PCM_INT16, HCW_FMT_PCM_INT16_FLT32, HCW_FMT_PCM_FLT32,
    };
    const int m = (int)(sizeof(v) / sizeof(v[0]));
    for (int i = 0; i < m && i < n; ++i) out[i] = v[i];
    return m;
}

const char *ref_cwave_magic(void) { return HCW_MAGIC; }
