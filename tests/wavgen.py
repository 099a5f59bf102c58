"""Test helper: RIFF/WAVE file images in every header variant rwave_reader_create accepts
(xwave_reader.c:362-585), plus broken ones.  Pure byte assembly, no audio library."""
import struct

from in_cwave_amd import abi

BPS = {abi.FMT_U8: 8, abi.FMT_I16: 16, abi.FMT_I24: 24, abi.FMT_I32: 32, abi.FMT_F32: 32}
GUID_TAIL = bytes([0x00, 0x00, 0x00, 0x00, 0x10, 0x00, 0x80, 0x00, 0x00, 0xaa, 0x00, 0x38, 0x9b, 0x71])


def chunk(tag, body):
    return tag + struct.pack("<I", len(body)) + body


def fmt_body(fmt, ch, rate, kind="pcm", bps=None, align=None, guid_code=None, cb=22):
    bps = BPS[fmt] if bps is None else bps
    align = ch * ((bps + 7) // 8) if align is None else align
    tag = {"pcm": 1, "float": 3, "ext": 0xFFFE, "wfonly": 1}[kind]
    if kind == "float" or (kind == "ext" and fmt == abi.FMT_F32 and guid_code is None):
        guid_code = 3 if kind == "ext" else None
    base = struct.pack("<HHIIH", tag, ch, rate, rate * align, align)
    if kind == "wfonly":
        return base                                   # WAVEFORMAT: 14 bytes, no wBitsPerSample
    body = base + struct.pack("<H", bps)
    if kind == "ext":
        code = 1 if guid_code is None else guid_code
        body += struct.pack("<HHI", cb, bps, (1 << ch) - 1) + struct.pack("<H", code) + GUID_TAIL
    return body


def wav_bytes(data, fmt, ch, rate, kind="pcm", pre_chunks=(), post_fmt_chunks=(), **kw):
    body = b"WAVE"
    for c in pre_chunks:
        body += c
    body += chunk(b"fmt ", fmt_body(fmt, ch, rate, kind, **kw))
    for c in post_fmt_chunks:
        body += c
    body += chunk(b"data", bytes(data))
    return b"RIFF" + struct.pack("<I", len(body)) + body


def write(path, data, fmt, ch, rate, **kw):
    path.write_bytes(wav_bytes(data, fmt, ch, rate, **kw))
    return path
