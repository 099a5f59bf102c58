"""GPU parity of K3r's clamp-free blocks (icw_render_row, render_consts' spec_thr).

The row render runs a 20-sample block without the clip stage when the block before it clipped
nowhere and the block's own inputs x * norm_mul are all within spec_thr: the error fed back is then
bounded, no |q| can reach the clip bounds, and the clamp is the identity (sound_render.c:782-797).
These cases drive the switch both ways inside one launch: quiet stretches (clamp-free), bursts past
full scale (clips; the next block runs exact and re-arms), inputs hovering at the threshold, a NaN and
an infinity in float input, for FIR shapers of every tap count, the flat shaper with dither, the IIR
shaper (never clamp-free), both quantisers, 16 / 24 bit and reduced sign bits, every dither type.
Bytes, pre-render doubles and meters equal the oracle's."""
import os

import numpy as np
import pytest

from in_cwave_amd import abi, graph

pytestmark = pytest.mark.gpu

N = 9000
REPS = int(os.environ.get("ICW_SPEC_REPS", 1))       # inputs per case (wider sweeps: the env)


def bursty_f32(n_streams, n, seed, amp):
    """stereo float input: a tone at `amp` of full scale with bursts far past it, stretches right at
    it, and (stream 1) a NaN and an infinity"""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 48000.0
    x = np.zeros((n_streams, n, 2))
    for s in range(n_streams):
        for c in range(2):
            f = rng.uniform(200, 9000)
            x[s, :, c] = amp[s % len(amp)] * np.sin(2 * np.pi * f * t + rng.uniform(0, 6))
            x[s, :, c] += 1e-3 * rng.standard_normal(n)
        for _ in range(4):                                   # bursts: clip for a few dozen samples
            i = int(rng.integers(100, n - 200))
            x[s, i:i + int(rng.integers(1, 80))] *= rng.uniform(1.5, 6.0)
        i = int(rng.integers(100, n - 400))                  # right at full scale for a while
        x[s, i:i + 300] = np.clip(x[s, i:i + 300] * 4.0, -1.0, 1.0) * rng.uniform(0.995, 1.0)
    x[1 % n_streams, 4321, 0] = np.nan
    x[1 % n_streams, 6543, 1] = np.inf
    return x.astype(np.float32).reshape(n_streams, -1).view(np.uint8)


def run(oracle, icw, cfg, nodes, raw, n, blocks=(N,)):
    ctx = icw.Context(cfg, nodes, raw.shape[0])
    outs, pres, t = [], [], 0
    fsz = ctx.fsz
    for b in blocks:
        o, p = ctx.process(np.ascontiguousarray(raw[:, t * fsz:(t + b) * fsz]), b, want_pre=True)
        outs.append(o)
        pres.append(p)
        t += b
    out, pre = np.concatenate(outs, axis=1), np.concatenate(pres, axis=1)
    meters = [ctx.meters(s) for s in range(raw.shape[0])]
    ctx.close()
    for s in range(raw.shape[0]):
        st = oracle.Stream(cfg, nodes)
        ro, rp = st.process(raw[s], n, want_pre=True)
        bad = np.flatnonzero(pre[s].view(np.uint64) != rp.view(np.uint64))
        bad = bad[~(np.isnan(pre[s].reshape(-1)[bad]) & np.isnan(rp.reshape(-1)[bad]))]
        assert bad.size == 0, (s, bad[:5])
        badb = np.flatnonzero(out[s] != ro)
        assert badb.size == 0, (s, badb[:8])
        assert meters[s] == st.meters(), (s, meters[s], st.meters())


# shapers: 0 flat, 4 FIR 5, 2 FIR 9 (MEW44), 14 FIR 15, 5 FIR 16, 6 FIR 20, 16 IIR 4; ROUND + flat is not a
# serial render (K2 renders it), so that pair is left out
RENDERS = [(ns, rt) for ns in (0, 4, 2, 14, 5, 6, 16) for rt in (abi.RENDER_ROUND, abi.RENDER_TPDF, abi.RENDER_GAUSS)
           if (ns, rt) != (0, abi.RENDER_ROUND)]


@pytest.mark.parametrize("rep", range(REPS))
@pytest.mark.parametrize("ns,rtype", RENDERS)
@pytest.mark.parametrize("quantz", [abi.QUANTZ_MID_RISER, abi.QUANTZ_MID_TREAD])
@pytest.mark.parametrize("b24", [False, True])
def test_clamp_free_blocks(oracle, icw, monkeypatch, ns, rtype, quantz, b24, rep):
    monkeypatch.setenv("ICW_RENDER", "row")
    cfg = graph.default_config(48000, fmt=abi.FMT_F32, need24bits=b24)
    cfg.render.render_type = rtype
    cfg.render.nshape_type = ns
    cfg.render.quantz_type = quantz
    nodes = [graph.master(gain=1.0, tout=abi.S_RE)]          # the I channel: the input, delayed
    raw = bursty_f32(6, N, seed=ns * 100 + rtype * 10 + quantz * 2 + b24 + 100003 * rep, amp=(0.2, 0.6, 0.93, 0.99))
    run(oracle, icw, cfg, nodes, raw, N, blocks=(4007, N - 4007))


@pytest.mark.parametrize("ns", [2, 6])
@pytest.mark.parametrize("rtype", [abi.RENDER_RPDF, abi.RENDER_STPDF])
@pytest.mark.parametrize("sign_bits,dth", [(12, 1.0), (16, 3.0), (16, 0.0)])
def test_clamp_free_blocks_sign_bits_dither(oracle, icw, monkeypatch, ns, rtype, sign_bits, dth):
    """norm_mul != 1 (sign bits), larger dither (spec_thr shrinks), dth_bits 0 (dth_mul 0)"""
    monkeypatch.setenv("ICW_RENDER", "row")
    cfg = graph.default_config(48000, fmt=abi.FMT_F32)
    cfg.render.render_type = rtype
    cfg.render.nshape_type = ns
    cfg.render.sign_bits16 = sign_bits
    cfg.render.dth_bits = dth
    nodes = [graph.master(gain=1.0, tout=abi.S_RE)]
    raw = bursty_f32(4, N, seed=ns + rtype * 7 + sign_bits, amp=(0.5, 0.97))
    run(oracle, icw, cfg, nodes, raw, N)
