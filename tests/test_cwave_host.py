"""CPU tests for the CWAVE side: the oracle's CRC-32 restatement pinned against the reference's
crc32.c (golden vectors from the reference build, and the build itself when present), zlib and
the standard check value; the product's host-only pieces (CWAVE header checks, CRC combine) --
no GPU call is made here."""
import ctypes as C
import json
import zlib
from pathlib import Path

import numpy as np
import pytest

from in_cwave_amd import abi, cwave, synth
from in_cwave_amd import lib as L

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"
REF_CRC = ROOT / "oracle" / "_ref" / "libref_crc32.so"


def golden_crc_cases():
    doc = json.loads((GOLD / "crc32_ref.json").read_text())
    rng = np.random.default_rng(32)
    for c in doc["cases"]:
        yield rng.integers(0, 256, c["n"], dtype=np.uint8).tobytes(), c["parts"], c["crc"]


class _OrcCrc(C.Structure):
    _fields_ = [("xor_mask", C.c_uint32), ("reg", C.c_uint32)]


def _orc():
    from oracle import oracle as O
    lib = O.load()
    lib.orc_crc32_update.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    lib.orc_crc32_final.restype = C.c_uint32
    lib.orc_crc32.restype = C.c_uint32
    lib.orc_crc32.argtypes = [C.c_char_p, C.c_size_t]
    return lib


def test_oracle_crc_matches_reference_golden():
    lib = _orc()
    doc = json.loads((GOLD / "crc32_ref.json").read_text())
    for data, parts, want in golden_crc_cases():
        t = _OrcCrc()
        lib.orc_crc32_init(C.byref(t))
        off = 0
        for k in parts:
            lib.orc_crc32_update(C.byref(t), data[off:off + k], k)
            off += k
        assert lib.orc_crc32_final(C.byref(t)) == want
        assert zlib.crc32(data) == want
    assert lib.orc_crc32(b"123456789", 9) == doc["check_123456789"] == 0xCBF43926


def test_oracle_crc_random_vs_zlib():
    lib = _orc()
    rng = np.random.default_rng(5)
    for n in list(range(0, 40)) + [1000, 4097, 70001]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert lib.orc_crc32(d, n) == zlib.crc32(d)


@pytest.mark.skipif(not REF_CRC.exists(), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_crc_vs_reference_build():
    ref = C.CDLL(str(REF_CRC))
    ref.crc32final.restype = C.c_uint32
    lib = _orc()
    rng = np.random.default_rng(6)
    for n in (0, 1, 2, 3, 5, 17, 333):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        t = (C.c_uint32 * 2)()
        ref.crc32init(t)
        ref.crc32update(d, C.c_uint(n), t)
        assert ref.crc32final(t) == lib.orc_crc32(d, n)


def test_crc_combine_vs_zlib():
    rng = np.random.default_rng(7)
    for _ in range(50):
        a = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        assert L.crc32_combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)
    assert L.crc32_combine(0x12345678, 0, 0) == 0x12345678


@pytest.mark.parametrize("fmt", abi.CW_FORMATS)
@pytest.mark.parametrize("ch", [1, 2])
@pytest.mark.parametrize("version", [1, 2])
def test_cwave_parse_accepts(fmt, ch, version):
    d = synth.stream_cwave(0, 50, 44100, channels=ch, fmt=fmt)
    img = cwave.make_image(d, fmt, ch, 44100, version=version, trailer=b"xyz")
    h, f, fb = L.cwave_parse(img.tobytes(), img.size)
    assert (h.version, h.n_channels, h.n_samples, h.sample_rate) == (version, ch, 50, 44100)
    assert f == fmt and fb == abi.FMT_BYTES[fmt] * ch and h.hsize == 48
    assert h.n_crc32 == (zlib.crc32(d.tobytes()) if version == 2 else 0)


def _hdr(**kw):
    f = dict(magic=b"cPLXwAVE", hsize=48, version=2, format=1, ch=2, n=100, sr=48000)
    f.update(kw)
    import struct
    return f["magic"] + struct.pack("<7I", f["hsize"], f["version"], f["format"], f["ch"], f["n"], f["sr"], 0) + \
        struct.pack("<Id", 0, 0.0)


@pytest.mark.parametrize("kw,size", [
    (dict(magic=b"cPLXwAVf"), 1000), (dict(hsize=47), 1000), (dict(hsize=1000), 1000), (dict(hsize=900), 1000), (dict(version=0), 1000),
    (dict(version=3), 1000), (dict(format=4), 1000), (dict(ch=0), 1000), (dict(ch=3), 1000), (dict(n=1), 1000),
    (dict(n=100), 48 + 799), (dict(sr=0), 1000), (dict(), 47)])
def test_cwave_parse_rejects_what_the_reference_rejects(kw, size):
    """cwave_reader_create's checks (xwave_reader.c:258-299)"""
    with pytest.raises(L.IcwError):
        L.cwave_parse(_hdr(**kw), size)
    L.cwave_parse(_hdr(), 48 + 800)       # the unmodified header is fine (100 x 2 x 4 B)
