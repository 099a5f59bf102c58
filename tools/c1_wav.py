#!/usr/bin/env python3
"""Write the C1 track (30 s, 44.1 kHz, 16-bit stereo, SURVEY 8(d) generator) as a WAV file:
    python tools/c1_wav.py out.wav [seconds]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from in_cwave_amd import synth  # noqa: E402

sec = float(sys.argv[2]) if len(sys.argv) > 2 else 30.0
n = int(44100 * sec)
bench._wav_i16(sys.argv[1], synth.stream_pcm(0, n, 44100), 44100, 2)
