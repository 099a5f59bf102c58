"""Synthetic stream generator of SURVEY 8(d): per stream s, numpy.random.default_rng(1000+s),
two sines with frequencies uniform in [40 Hz, 0.4*fs] at -12 dBFS each with random phases, plus
white Gaussian noise at -40 dBFS; quantised (round, clip) to int16 or kept float32.  Output is
the raw interleaved little-endian byte layout a WAV reader leaves in xr->tbuff."""
import numpy as np

from . import abi


def stream_pcm(s, n_frames, fs, channels=2, fmt=abi.FMT_I16, seed_base=1000):
    rng = np.random.default_rng(seed_base + s)
    t = np.arange(n_frames, dtype=np.float64) / fs
    a = 10 ** (-12 / 20)
    sig = np.zeros((n_frames, channels))
    for ch in range(channels):
        f = rng.uniform(40.0, 0.4 * fs, size=2)
        ph = rng.uniform(0, 2 * np.pi, size=2)
        sig[:, ch] = a * (np.sin(2 * np.pi * f[0] * t + ph[0]) + np.sin(2 * np.pi * f[1] * t + ph[1]))
        sig[:, ch] += 10 ** (-40 / 20) * rng.standard_normal(n_frames)
    if fmt == abi.FMT_I16:
        q = np.clip(np.round(sig * 32767.0), -32768, 32767).astype("<i2")
        return q.reshape(-1).view(np.uint8)
    if fmt == abi.FMT_F32:
        return sig.astype("<f4").reshape(-1).view(np.uint8)
    if fmt == abi.FMT_I24:
        q = np.clip(np.round(sig * 8388607.0), -8388608, 8388607).astype("<i4").reshape(-1)
        b = q.view(np.uint8).reshape(-1, 4)[:, :3]
        return np.ascontiguousarray(b).reshape(-1)
    if fmt == abi.FMT_I32:
        q = np.clip(np.round(sig * 2147483647.0), -2147483648, 2147483647).astype("<i4")
        return q.reshape(-1).view(np.uint8)
    if fmt == abi.FMT_U8:
        q = np.clip(np.round(sig * 127.0) + 128, 0, 255).astype(np.uint8)
        return q.reshape(-1)
    raise ValueError(fmt)


def stream_cwave(s, n_frames, fs, channels=2, fmt=abi.FMT_CW_I16, seed_base=2000):
    """Analytic (complex) test signal in a CWAVE sample format: per channel two complex
    exponentials (positive and negative frequency, -12 dBFS each) plus complex Gaussian noise at
    -40 dBFS, on the 16-bit scale the CWAVE formats use (cwave.h:70-80).  Interleaved per frame:
    Re(L), Im(L)[, Re(R), Im(R)] in the format's own field widths."""
    rng = np.random.default_rng(seed_base + s)
    t = np.arange(n_frames, dtype=np.float64) / fs
    a = 32767.0 * 10 ** (-12 / 20)
    z = np.zeros((n_frames, channels), dtype=np.complex128)
    for ch in range(channels):
        f = rng.uniform(40.0, 0.4 * fs, size=2) * np.array([1.0, -1.0])
        ph = rng.uniform(0, 2 * np.pi, size=2)
        z[:, ch] = a * (np.exp(1j * (2 * np.pi * f[0] * t + ph[0])) + np.exp(1j * (2 * np.pi * f[1] * t + ph[1])))
        z[:, ch] += 32767.0 * 10 ** (-40 / 20) * (rng.standard_normal(n_frames) + 1j * rng.standard_normal(n_frames))
    re, im = z.real, z.imag
    if fmt == abi.FMT_CW_F64:
        dt = np.dtype([("re", "<f8"), ("im", "<f8")])
    elif fmt == abi.FMT_CW_I16:
        dt = np.dtype([("re", "<i2"), ("im", "<i2")])
        re = np.clip(np.round(re), -32768, 32767)
        im = np.clip(np.round(im), -32768, 32767)
    elif fmt == abi.FMT_CW_I16_F32:
        dt = np.dtype([("re", "<i2"), ("im", "<f4")])
        re = np.clip(np.round(re), -32768, 32767)
    elif fmt == abi.FMT_CW_F32:
        dt = np.dtype([("re", "<f4"), ("im", "<f4")])
    else:
        raise ValueError(fmt)
    rec = np.zeros((n_frames, channels), dtype=dt)
    rec["re"] = re
    rec["im"] = im
    return rec.reshape(-1).view(np.uint8)


def batch_pcm(n_streams, n_frames, fs, channels=2, fmt=abi.FMT_I16, first=0):
    gen = stream_cwave if fmt in abi.CW_FORMATS else stream_pcm
    rows = [gen(first + s, n_frames, fs, channels, fmt) for s in range(n_streams)]
    return np.stack(rows)
