"""CPU tests for icw_wav_parse_file: the reference's reader acceptance rules
(xwave_reader_create / rwave_reader_create / cwave_reader_create, xwave_reader.c:123-131,
243-339, 362-585, 672-674), on file images built by tests/wavgen.py.  No GPU call is made."""
import struct

import numpy as np
import pytest

from in_cwave_amd import abi, cwave, synth
from in_cwave_amd import lib as L

import wavgen as W


def data_for(fmt, ch, n=100):
    return synth.stream_pcm(0, n, 48000, channels=ch, fmt=fmt)


@pytest.mark.parametrize("fmt", [abi.FMT_U8, abi.FMT_I16, abi.FMT_I24, abi.FMT_I32, abi.FMT_F32])
@pytest.mark.parametrize("ch", [1, 2])
def test_accepts_pcm_float_and_extensible(tmp_path, fmt, ch):
    d = data_for(fmt, ch)
    kinds = ["float", "ext"] if fmt == abi.FMT_F32 else ["pcm", "ext", "wfonly"]
    for kind in kinds:
        p = W.write(tmp_path / f"a_{kind}.wav", d, fmt, ch, 44100, kind=kind,
                    pre_chunks=[W.chunk(b"LIST", b"abcd")], post_fmt_chunks=[W.chunk(b"fact", b"\0" * 4)])
        i = L.wav_parse_file(p)
        assert (i.fmt, i.channels, i.sample_rate, i.n_samples) == (fmt, ch, 44100, 100), kind
        assert i.frame_bytes == abi.FMT_BYTES[fmt] * ch
        assert i.htype == {"pcm": abi.HTYPE_PCMW, "float": abi.HTYPE_PCMW, "ext": abi.HTYPE_EXT,
                           "wfonly": abi.HTYPE_WFONLY}[kind]
        raw = p.read_bytes()
        assert raw[i.data_offset:i.data_offset + d.size] == d.tobytes()


def test_bits_rounded_up_to_bytes(tmp_path):
    """wBitsPerSample 12 reads as 16 (xwave_reader.c:440-442)"""
    d = data_for(abi.FMT_I16, 2)
    i = L.wav_parse_file(W.write(tmp_path / "b.wav", d, abi.FMT_I16, 2, 8000, bps=12))
    assert i.fmt == abi.FMT_I16


@pytest.mark.parametrize("case", ["no_riff", "data_first", "fmt_beyond_eof", "three_ch", "zero_rate", "bps_12_float",
                                  "bad_guid", "align_mismatch", "one_sample", "rate_over_max", "ext_cb_small",
                                  "data_beyond_eof", "wfonly_align_odd", "bad_ext"])
def test_rejects(tmp_path, case):
    d = data_for(abi.FMT_I16, 2)
    name = "x.wav"
    if case == "no_riff":
        img = b"RIFX" + W.wav_bytes(d, abi.FMT_I16, 2, 48000)[4:]
    elif case == "data_first":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 48000, pre_chunks=[W.chunk(b"data", b"\0" * 8)])
    elif case == "fmt_beyond_eof":
        img = b"RIFF" + struct.pack("<I", 100) + b"WAVE" + b"fmt " + struct.pack("<I", 1000) + b"\0" * 16
    elif case == "three_ch":
        img = W.wav_bytes(synth.stream_pcm(0, 100, 48000, channels=3), abi.FMT_I16, 3, 48000)
    elif case == "zero_rate":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 0)
    elif case == "bps_12_float":
        img = W.wav_bytes(d, abi.FMT_F32, 2, 48000, kind="float", bps=24)
    elif case == "bad_guid":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 48000, kind="ext", guid_code=2)
    elif case == "align_mismatch":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 48000, align=6)
    elif case == "one_sample":
        img = W.wav_bytes(d[:4], abi.FMT_I16, 2, 48000)
    elif case == "rate_over_max":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 2_000_001)
    elif case == "ext_cb_small":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 48000, kind="ext", cb=21)
    elif case == "data_beyond_eof":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 48000)[:-10]
    elif case == "wfonly_align_odd":
        img = W.wav_bytes(d, abi.FMT_I16, 2, 48000, kind="wfonly", align=3)
    else:
        img, name = W.wav_bytes(d, abi.FMT_I16, 2, 48000), "x.flac"
    p = tmp_path / name
    p.write_bytes(img)
    with pytest.raises(L.IcwError):
        L.wav_parse_file(p)


def test_cwave_by_extension(tmp_path):
    d = synth.stream_cwave(0, 64, 48000, fmt=abi.FMT_CW_F32)
    img = cwave.make_image(d, abi.FMT_CW_F32, 2, 48000)
    p = tmp_path / "t.CWAVE"
    p.write_bytes(img.tobytes())
    i = L.wav_parse_file(p)
    assert (i.fmt, i.n_samples, i.data_offset, i.htype) == (abi.FMT_CW_F32, 64, 48, abi.HTYPE_CWAVE)
    (tmp_path / "t.wav").write_bytes(img.tobytes())           # CWAVE bytes under .wav: refused
    with pytest.raises(L.IcwError):
        L.wav_parse_file(tmp_path / "t.wav")
    ok = tmp_path / "w.rwave"
    ok.write_bytes(W.wav_bytes(synth.stream_pcm(0, 10, 48000), abi.FMT_I16, 2, 48000))
    assert L.wav_parse_file(ok).n_samples == 10
