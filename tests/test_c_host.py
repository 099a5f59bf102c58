"""The C host (examples/icw_transcode.c) drives the drop-in boundary (include/icw_amod.h) the way
playback.c / transcode.c drive amod_process_samples: 576-frame blocks from a WAV reader.
BASELINE C1 shape (44.1 kHz 16-bit stereo, Shift + Master, 16-bit render)."""
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "examples" / "icw_transcode"


def write_wav(path, raw, rate, channels, bits, fmt_tag=1):
    data = raw.tobytes()
    ba = channels * bits // 8
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVEfmt " + struct.pack(
        "<IHHIIHH", 16, fmt_tag, channels, rate, rate * ba, ba, bits) + b"data" + struct.pack("<I", len(data))
    path.write_bytes(hdr + data)


def read_wav_data(path):
    b = path.read_bytes()
    i = b.index(b"data")
    n = struct.unpack("<I", b[i + 4:i + 8])[0]
    return np.frombuffer(b[i + 8:i + 8 + n], np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("gname,nodes", [
    ("master", graph.graph_master_only()),
    ("shift", graph.graph_shift_master()),
    ("pmmix", graph.graph_pm_shift_mix()),
])
def test_c_host_transcode_c1(oracle, tmp_path, gname, nodes):
    assert EXE.exists(), "build() builds examples/icw_transcode"
    n = 44100 * 2 + 123
    raw = synth.stream_pcm(7, n, 44100)
    write_wav(tmp_path / "in.wav", raw, 44100, 2, 16)
    r = subprocess.run([str(EXE), str(tmp_path / "in.wav"), str(tmp_path / "out.wav"), "576", gname],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = read_wav_data(tmp_path / "out.wav")
    cfg = graph.default_config(44100)
    st = oracle.Stream(cfg, nodes)
    st.open(n)
    ref, _ = st.process(raw, n)
    assert got.size == ref.size
    assert np.array_equal(got, ref)        # Shift / PM included: glibc-identical sin / cos


@pytest.mark.gpu
def test_c_host_mono_f32_24bit(oracle, tmp_path):
    n = 9000
    raw = synth.stream_pcm(3, n, 96000, channels=1, fmt=abi.FMT_F32)
    write_wav(tmp_path / "in.wav", raw, 96000, 1, 32, fmt_tag=3)
    r = subprocess.run([str(EXE), str(tmp_path / "in.wav"), str(tmp_path / "out.wav"), "1000", "master", "24"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    cfg = graph.default_config(96000, fmt=abi.FMT_F32, channels=1, need24bits=True)
    st = oracle.Stream(cfg, graph.graph_master_only())
    st.open(n)
    ref, _ = st.process(raw, n)
    assert np.array_equal(read_wav_data(tmp_path / "out.wav"), ref)
