"""The device's sample decode against the REFERENCE's own unpackers (tests/golden/unpack_ref.npz:
unpack_lsb.h:53-125 compiled where it lies, see tests/test_reader_pinned.py).

  - real input: K0's pre-Hilbert doubles (ICW_F_DEBUG_INPUT: the unpacked, faded samples the
    quadrature converters get, xwave_unpack_csample, xwave_reader.c:974-998) for i16 / i24 / i32 /
    f32, stereo and mono, in one-block and multi-block calls -- the reference's raw decode with the
    reader's scaling (xwave_reader.c:213-239) applied;
  - complex (CWAVE) input: the analytic samples as K0 unpacks them (xwave_reader.c:171-200), read
    back through a bypassed list whose Master passes Re or Im at gain 1.0 (adv_modulator.c:644-651:
    with the bypass the Master runs on `in` itself, no 0.0 + sum, so even a zero's sign survives).
Integer kinds are bit for bit; a NaN compares as a NaN (its payload is not an audio value)."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph
from tests.test_reader_pinned import REAL_FMT, cw_cases, expected_real, fixtures, same_bits

pytestmark = pytest.mark.gpu

SIZE = {"i16": 2, "i24": 3, "i32": 4, "f32": 4}


@pytest.mark.parametrize("name", ["i16", "i24", "i32", "f32"])
@pytest.mark.parametrize("ch", [2, 1])
@pytest.mark.parametrize("block", [0, 256])
def test_k0_decode_matches_reference(icw, name, ch, block, monkeypatch):
    if block:
        monkeypatch.setenv("ICW_BLOCK", str(block))       # several launch blocks in one call
    fx = fixtures()
    raw = np.ascontiguousarray(fx[name + "_bytes"])
    want = expected_real(fx, name)
    n = want.size // ch
    cfg = graph.default_config(48000, fmt=REAL_FMT[name], channels=ch)
    S = 3
    # stream s carries the fixture rotated by s frames (every stream its own input)
    img = np.stack([np.roll(raw[:n * ch * SIZE[name]], -s * ch * SIZE[name]) for s in range(S)])
    ctx = icw.Context(cfg, graph.graph_shift_master(), S)
    x, _ = ctx.unpacked_input(img, n)
    for s in range(S):
        w = np.roll(want[:n * ch], -s * ch).reshape(n, ch)
        assert same_bits(x[s, :, 0], w[:, 0]), (name, ch, s)
        assert same_bits(x[s, :, 1], w[:, ch - 1]), (name, ch, s)       # mono: R = L
        if name != "f32":
            assert np.array_equal(x[s].view(np.uint64)[:, 0], w[:, 0].view(np.uint64))
    ctx.close()


def test_k0_decode_with_fades(icw, oracle):
    """a track with fades: K0's doubles are the reference decode times the fade factor of
    xwave_unpack_csample (xwave_reader.c:922-936), as the oracle computes it"""
    fx = fixtures()
    raw = np.ascontiguousarray(fx["i24_bytes"])
    want = expected_real(fx, "i24")
    n = want.size // 2
    cfg = graph.default_config(44100, fmt=abi.FMT_I24, channels=2)
    ctx = icw.Context(cfg, graph.graph_master_only(), 1)
    ctx.stream_open(0, n, fade_in_ms=3, fade_out_ms=4)
    x, _ = ctx.unpacked_input(raw[None, :n * 6], n)
    nfi, nfo = 3 * 44100 // 1000, 4 * 44100 // 1000
    fade = np.full(n, -1.0)
    ix = np.arange(n)
    fade[ix < nfi] = ix[ix < nfi] / nfi
    m = (ix > n - nfo) & (ix < n)
    fade[m] = (n - ix[m]) / nfo
    w = want[:2 * n].reshape(n, 2).copy()
    w[fade >= 0] *= fade[fade >= 0, None]
    assert same_bits(x[0], w)
    ctx.close()


@pytest.mark.parametrize("ch", [2, 1])
def test_cwave_decode_matches_reference(icw, ch):
    fx = fixtures()
    for fmt, img, wi, wq in cw_cases(fx):
        n = len(img) // ch
        data = np.ascontiguousarray(img[:n * ch].reshape(1, -1))
        got = []
        for tout in (abi.S_RE, abi.S_IM):
            cfg = graph.default_config(48000, fmt=fmt, channels=ch)
            cfg.bypass_list = 1
            ctx = icw.Context(cfg, [graph.master(gain=1.0, tout=tout)], 1)
            _, pre = ctx.process(data, n, want_pre=True)
            got.append(pre[0])
            ctx.close()
        for tout, g, w in ((abi.S_RE, got[0], wi), (abi.S_IM, got[1], wq)):
            w = w[:n * ch].reshape(n, ch)
            assert same_bits(g[:, 0], w[:, 0]), (fmt, ch, tout)
            assert same_bits(g[:, 1], w[:, ch - 1]), (fmt, ch, tout)
