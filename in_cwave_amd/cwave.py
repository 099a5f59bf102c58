"""CWAVE file images (cwave.h): header layout HCWAVE_V2 (cwave.h:48-60), magic "cPLXwAVE",
little-endian fields, data part right after the header.  The writer is what the reference's
external CWAVE converter produces; n_CRC32 is the CRC-32 of the data part (gui_cwave.c:82-129).
Used to make test and benchmark inputs; decoding is icw_process_* with ICW_FMT_CW_*."""
import struct
import zlib

import numpy as np

from . import abi

HCW_FMT = {abi.FMT_CW_F64: 0, abi.FMT_CW_I16: 1, abi.FMT_CW_I16_F32: 2, abi.FMT_CW_F32: 3}


def header_bytes(fmt, channels, n_samples, sample_rate, crc=0, version=2, hsize=abi.CWAVE_HEADER_BYTES,
                 k_M=-1, k_beta=0.0):
    return (b"cPLXwAVE" + struct.pack("<7I", hsize, version, HCW_FMT[fmt], channels, n_samples, sample_rate,
                                      k_M & 0xffffffff) + struct.pack("<I", crc) + struct.pack("<d", k_beta))


def make_image(data, fmt, channels, sample_rate, version=2, hsize=abi.CWAVE_HEADER_BYTES, trailer=b""):
    """a CWAVE file image (uint8 array) around interleaved sample data in an ICW_FMT_CW_* format"""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    fb = abi.FMT_BYTES[fmt] * channels
    assert data.size % fb == 0
    crc = zlib.crc32(data.tobytes()) if version >= 2 else 0
    hdr = header_bytes(fmt, channels, data.size // fb, sample_rate, crc, version, hsize)
    hdr = hdr + b"\0" * (hsize - len(hdr))
    return np.frombuffer(hdr + data.tobytes() + trailer, dtype=np.uint8).copy()
