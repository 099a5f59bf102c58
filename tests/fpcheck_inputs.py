"""Inputs and configurations for the FP_CHECK tests (fp_check.c:52-100, the FC() census): PCM with
NaN, +-Inf and denormal samples at seeded positions."""
import numpy as np

from in_cwave_amd import abi, graph, synth


def fc_cfg(fmt=abi.FMT_F32, kahan=1, subn=1, render=abi.RENDER_TPDF, ns=abi.NSHAPE_MEW44, need24=True,
           channels=2):
    cfg = graph.default_config(48000, fmt=fmt, channels=channels, need24bits=need24)
    cfg.iir_kahan, cfg.iir_subnorm_reject = kahan, subn
    cfg.render.render_type, cfg.render.nshape_type = render, ns
    cfg.fp_check = 1
    return cfg


def special_f32(n_streams, n_frames, seed=0):
    """float32 stereo PCM with NaN, +-Inf and f32-denormal samples"""
    raw = synth.batch_pcm(n_streams, n_frames, 48000, fmt=abi.FMT_F32)
    f = raw.view(np.float32).reshape(n_streams, n_frames, 2)
    rng = np.random.default_rng(seed)
    for s in range(n_streams):
        for v in (np.nan, np.inf, -np.inf, np.float32(1e-45), np.float32(-3e-42)):
            f[s, rng.integers(0, n_frames), rng.integers(0, 2)] = v
    return raw


def special_cw64(n_streams, n_frames, seed=1):
    """CWAVE float64 I/Q (no Hilbert: the values reach the render as they are) with NaN, +-Inf and
    double denormals that stay denormal after the 24-bit norm_mul (x256)"""
    raw = synth.batch_pcm(n_streams, n_frames, 48000, fmt=abi.FMT_CW_F64)
    d = raw.view(np.float64).reshape(n_streams, n_frames, 4)
    rng = np.random.default_rng(seed)
    for s in range(n_streams):
        for v in (np.nan, np.inf, -np.inf):
            d[s, rng.integers(0, n_frames), rng.integers(0, 4)] = v
        for v in (3e-321, -1e-320):      # both components of a channel: the Master's (re + im) stays tiny
            t, c = rng.integers(0, n_frames), rng.integers(0, 2)
            d[s, t, 2 * c] = d[s, t, 2 * c + 1] = v
    return raw
