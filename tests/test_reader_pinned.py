"""The reader's sample decode, pinned to the reference's own code (missing #2).

tests/golden/unpack_ref.npz holds the outputs of the REFERENCE's unpack_int16 / unpack_int24 /
unpack_int32 / unpack_float / unpack_double (unpack_lsb.h:53-125), compiled where they lie by
`make -C oracle ref` (oracle/ref_unpack.c, an original driver; unpack_lsb.h and cwave.h include only
<stdint.h>, so no stand-in header is involved) and run by tools/gen_golden.py on random bytes and
edge cases: i24 sign extension, integer extremes, signed zeros, infinities, quiet / signalling /
negative NaNs with payloads, denormals.  tests/golden/cwave_layout.json holds sizeof / offsetof of
HCWAVE_V1 / V2 and the HCW_* constants (cwave.h:31-87) from the same build.

Checked here (no GPU): the oracle's unpackers (icw_oracle.c unpack1 / unpack_iq) against those
values, with the reader's scaling of xwave_reader.c:205-239 applied (i16 as is, i24 / 256, i32 /
65536, f32 * 32768; the CWAVE samples unscaled, xwave_reader.c:171-200) -- that scaling lives in
xwave_reader.c, which needs <windows.h>, so it is restated, not reference-built; and the product's
CWAVE header struct, writer and parser against the reference's layout.  tests/test_gpu_reader_pinned.py
checks the device's decode (K0 and the CWAVE path) against the same fixtures."""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

from in_cwave_amd import abi, cwave

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"
REF_UNPACK = ROOT / "oracle" / "_ref" / "libref_unpack.so"


def fixtures():
    with np.load(GOLD / "unpack_ref.npz") as z:
        return {k: z[k] for k in z.files}


def expected_real(fx, name):
    """the reader's scaled doubles (xwave_reader.c:213-239) from the reference's raw decode"""
    v = fx[name + "_val"]
    if name == "i16":
        return v.astype(np.float64)
    if name == "i24":
        return v.astype(np.float64) / 256.0
    if name == "i32":
        return v.astype(np.float64) / 65536.0
    if name == "f32":
        with np.errstate(invalid="ignore"):          # signalling NaNs become quiet ones, as in C
            return 32768.0 * v.view(np.float32).astype(np.float64)
    raise KeyError(name)


REAL_FMT = {"i16": abi.FMT_I16, "i24": abi.FMT_I24, "i32": abi.FMT_I32, "f32": abi.FMT_F32}


def same_bits(a, b):
    """bit-identical doubles; NaNs compare as a class (a payload is not an audio value; the
    reference's x86 build and the device both return a quiet NaN)"""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    nan = np.isnan(a)
    return bool(np.array_equal(nan, np.isnan(b)) and np.array_equal(a[~nan].view(np.uint64), b[~nan].view(np.uint64)))


def _orc():
    from oracle import oracle as O
    lib = O.load()
    lib.orc_unpack_real.argtypes = [C.c_uint, C.c_void_p, C.c_size_t, C.c_void_p]
    lib.orc_unpack_cw.argtypes = [C.c_uint, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    return lib


def cw_cases(fx):
    """CWAVE sample images built from the reference fixtures, with the expected I / Q
    (unpack_cwave_dbl / _sht / _sht_flt / _flt, xwave_reader.c:171-200)"""
    f64 = fx["f64_bytes"].reshape(-1, 8)
    i16 = fx["i16_bytes"].reshape(-1, 2)
    f32 = fx["f32_bytes"].reshape(-1, 4)
    f64v = fx["f64_val"].view(np.float64)
    i16v = fx["i16_val"].astype(np.float64)
    with np.errstate(invalid="ignore"):
        f32v = fx["f32_val"].view(np.float32).astype(np.float64)
    n = len(f64) // 2
    yield abi.FMT_CW_F64, f64[:2 * n].reshape(n, 16), f64v[0:2 * n:2], f64v[1:2 * n:2]
    n = len(i16) // 2
    yield abi.FMT_CW_I16, i16[:2 * n].reshape(n, 4), i16v[0:2 * n:2], i16v[1:2 * n:2]
    n = min(len(i16), len(f32))
    yield abi.FMT_CW_I16_F32, np.concatenate([i16[:n], f32[:n]], axis=1), i16v[:n], f32v[:n]
    n = len(f32) // 2
    yield abi.FMT_CW_F32, f32[:2 * n].reshape(n, 8), f32v[0:2 * n:2], f32v[1:2 * n:2]


def test_fixture_covers_edge_cases():
    fx = fixtures()
    i24 = fx["i24_val"]
    assert i24.min() == -(1 << 23) and i24.max() == (1 << 23) - 1 and (i24 == -1).any()
    f32 = fx["f32_val"].view(np.float32)
    assert np.isnan(f32).any() and np.isinf(f32).any()
    assert ((fx["f32_val"] & 0x7F800000) == 0).sum() > 3          # zeros and denormals
    f64 = fx["f64_val"]
    assert (f64 == 1 << 63).any() and np.isnan(f64.view(np.float64)).any()


@pytest.mark.parametrize("name", ["i16", "i24", "i32", "f32"])
def test_oracle_real_unpack_matches_reference(name):
    fx = fixtures()
    raw = np.ascontiguousarray(fx[name + "_bytes"])
    want = expected_real(fx, name)
    got = np.zeros(want.size)
    _orc().orc_unpack_real(REAL_FMT[name], raw.ctypes.data, want.size, got.ctypes.data)
    assert same_bits(got, want)
    # the integer kinds carry no NaN: bit for bit outright
    if name != "f32":
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_oracle_cwave_unpack_matches_reference():
    fx = fixtures()
    lib = _orc()
    for fmt, img, wi, wq in cw_cases(fx):
        img = np.ascontiguousarray(img)
        gi, gq = np.zeros(len(img)), np.zeros(len(img))
        lib.orc_unpack_cw(fmt, img.ctypes.data, len(img), gi.ctypes.data, gq.ctypes.data)
        assert same_bits(gi, wi) and same_bits(gq, wq), fmt


def test_cwave_header_layout_matches_reference():
    """the product's header struct (include/icw_cwave.h, abi.CwaveHeader), its writer
    (in_cwave_amd/cwave.py) and its parser (icw_cwave_parse) against cwave.h's own layout"""
    from in_cwave_amd import lib as L
    doc = json.loads((GOLD / "cwave_layout.json").read_text())
    v2, v1 = doc["HCWAVE_V2"], doc["HCWAVE_V1"]
    assert v2["sizeof"] == v1["sizeof"] == abi.CWAVE_HEADER_BYTES == C.sizeof(abi.CwaveHeader)
    ours = {"magic": "magic", "hsize": "hsize", "version": "version", "format": "format",
            "n_channels": "n_channels", "n_samples": "n_samples", "sample_rate": "sample_rate", "k_M": "k_M",
            "n_CRC32": "n_crc32", "k_beta": "k_beta"}
    for ref_name, our_name in ours.items():
        assert getattr(abi.CwaveHeader, our_name).offset == v2[ref_name], ref_name
    assert v1["pad0"] == v2["n_CRC32"] and v1["k_beta"] == v2["k_beta"]
    assert doc["HCW_MAGIC"] == "cPLXwAVE" and doc["HCW_VERSION"] == {"BAD": 0, "V1": 1, "V2": 2, "CUR": 2}
    fmts = doc["HCW_FMT"]
    assert [fmts[k] + 5 for k in ("PCM_DBL64", "PCM_INT16", "PCM_INT16_FLT32", "PCM_FLT32")] == \
        [abi.FMT_CW_F64, abi.FMT_CW_I16, abi.FMT_CW_I16_F32, abi.FMT_CW_F32]
    # the writer puts every field where cwave.h has it
    hdr = cwave.header_bytes(abi.FMT_CW_I16_F32, 2, 1234, 48000, crc=0xDEADBEEF)
    import struct
    assert hdr[v2["magic"]:v2["magic"] + 8] == b"cPLXwAVE"
    for field, val in (("hsize", abi.CWAVE_HEADER_BYTES), ("version", 2), ("format", fmts["PCM_INT16_FLT32"]),
                       ("n_channels", 2), ("n_samples", 1234), ("sample_rate", 48000), ("n_CRC32", 0xDEADBEEF)):
        assert struct.unpack_from("<I", hdr, v2[field])[0] == val, field
    # the parser reads a header laid out by the reference's offsets
    img = bytearray(v2["sizeof"])
    img[0:8] = doc["HCW_MAGIC"].encode()
    for field, val in (("hsize", 48), ("version", 1), ("format", fmts["PCM_FLT32"]), ("n_channels", 1),
                       ("n_samples", 10), ("sample_rate", 96000)):
        struct.pack_into("<I", img, v1[field], val)
    struct.pack_into("<i", img, v1["k_M"], 1022)
    struct.pack_into("<d", img, v1["k_beta"], 8.5)
    h, fmt, fb = L.cwave_parse(bytes(img), 48 + 10 * 8)
    assert (h.version, h.n_channels, h.n_samples, h.sample_rate, h.k_M, h.k_beta) == (1, 1, 10, 96000, 1022, 8.5)
    assert fmt == abi.FMT_CW_F32 and fb == 8


@pytest.mark.skipif(not REF_UNPACK.exists(), reason="reference build absent (oracle/_ref is built where "
                                                    "/root/reference exists)")
def test_reference_unpackers_live():
    """where the reference build exists (this container), fresh random bytes through the reference's
    unpackers and the oracle's: the fixture is not a one-off"""
    ref = C.CDLL(str(REF_UNPACK))
    ref.ref_unpack_batch.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_void_p]
    lib = _orc()
    rng = np.random.default_rng(777)
    for name, kind, size in (("i16", 0, 2), ("i24", 1, 3), ("i32", 2, 4), ("f32", 3, 4)):
        raw = rng.integers(0, 256, 50_000 * size, dtype=np.uint8)
        val = np.zeros(50_000, dtype=np.uint32 if name == "f32" else np.int32)
        ref.ref_unpack_batch(kind, raw.ctypes.data, val.size, val.ctypes.data)
        want = expected_real({name + "_val": val}, name)
        got = np.zeros(val.size)
        lib.orc_unpack_real(REAL_FMT[name], raw.ctypes.data, val.size, got.ctypes.data)
        assert same_bits(got, want), name
