"""GPU parity of the dithered renders with the flat noise shaper, rendered frame-parallel.

With NSHAPE_FLAT the shaper returns 0.0 (ns_empty, sound_render.c:396-400), so prev_ns_err stays 0.0
(:800) and sound_render_value (:711-809) is a per-sample function of the sample and its dither term
rnd * dth_mul.  The dither terms come from K3a (the channel's MT19937 stream, serial per channel);
the render itself runs inside the output kernel of each path -- K2 (quadrature IIR), KF2 (the fused
FIR converter) and K5 (the one-kernel drop-in call) -- instead of the serial render.  Every case is
checked bit for bit against the oracle: the rendered bytes, the pre-render doubles and the meters,
over several calls (state carried), and ICW_DITH_PAR=0 (the same renders through the serial render)
gives the same bytes.  Forced dsopen rejections (zeroed MT words via the state blob) check that the
generator state the render consumes stays the reference's."""
import ctypes as C

import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

pytestmark = pytest.mark.gpu

DITHERS = [abi.RENDER_RPDF, abi.RENDER_TPDF, abi.RENDER_STPDF, abi.RENDER_GAUSS]


def flat_cfg(fs, rtype, quantz, b24, reduced, fmt=abi.FMT_I16, ch=2):
    cfg = graph.default_config(fs, fmt=fmt, channels=ch, need24bits=b24)
    cfg.render.render_type, cfg.render.quantz_type = rtype, quantz
    cfg.render.nshape_type = abi.NSHAPE_FLAT
    cfg.render.dth_bits = 1.5
    if reduced:
        if b24:
            cfg.render.sign_bits24 = 19
        else:
            cfg.render.sign_bits16 = 13
    return cfg


def run_calls(oracle, icw, cfg, nodes, n_streams, lens, fir=None, want_pre=True, first=3):
    """the calls of `lens` frames through one context, against one oracle stream per stream"""
    ctx = icw.Context(cfg, nodes, n_streams)
    if fir:
        ctx.set_fir_hilbert(*fir)
    n = sum(lens)
    raw = synth.batch_pcm(n_streams, n, cfg.sample_rate, channels=cfg.in_channels, fmt=cfg.in_format, first=first)
    fsz = ctx.fsz
    outs, pres, t = [], [], 0
    for b in lens:
        o, p = ctx.process(np.ascontiguousarray(raw[:, t * fsz:(t + b) * fsz]), b, want_pre=want_pre)
        outs.append(o)
        pres.append(p)
        t += b
    out = np.concatenate(outs, axis=1)
    ref_out, ref_pre = oracle.process_streams(cfg, nodes, raw, n, want_pre=True, fir=fir)
    assert np.array_equal(out, ref_out), "rendered bytes differ"
    if want_pre:
        pre = np.concatenate(pres, axis=1)
        bad = np.flatnonzero(pre.view(np.uint64) != ref_pre.view(np.uint64))
        assert bad.size == 0, f"{bad.size} pre-render doubles differ, first at {bad[:5]}"
    meters = [ctx.meters(s) for s in range(n_streams)]
    ctx.close()
    return out, meters


def ref_meters(oracle, cfg, nodes, raw_list, lens, fir=None):
    out = []
    for raw in raw_list:
        st = oracle.Stream(cfg, nodes)
        if fir:
            st.set_fir(*fir)
        t, fsz = 0, len(raw) // sum(lens)
        for b in lens:
            st.process(raw[t * fsz:(t + b) * fsz], b)
            t += b
        out.append(st.meters())
    return out


@pytest.mark.parametrize("rtype", DITHERS)
@pytest.mark.parametrize("quantz", [abi.QUANTZ_MID_TREAD, abi.QUANTZ_MID_RISER])
@pytest.mark.parametrize("b24", [False, True])
@pytest.mark.parametrize("reduced", [False, True])
def test_iir_path(oracle, icw, rtype, quantz, b24, reduced):
    """K2: every dither type x quantiser x 16 / 24 bit x full / reduced sign bits, three calls"""
    cfg = flat_cfg(44100, rtype, quantz, b24, reduced)
    nodes = graph.graph_shift_master()
    lens = [700, 801, 1]
    out, meters = run_calls(oracle, icw, cfg, nodes, 3, lens)
    raw = synth.batch_pcm(3, sum(lens), 44100, first=3)
    assert meters == ref_meters(oracle, cfg, nodes, list(raw), lens)


@pytest.mark.parametrize("rtype", DITHERS)
@pytest.mark.parametrize("quantz", [abi.QUANTZ_MID_TREAD, abi.QUANTZ_MID_RISER])
@pytest.mark.parametrize("b24", [False, True])
@pytest.mark.parametrize("ch", [1, 2])
def test_fir_path(oracle, icw, rtype, quantz, b24, ch):
    """KF2 (the fused converter, stereo and mono kernels): the render pass takes K3a's rows; two calls,
    the production form (no pre-render copy) and the checked one"""
    fir = (254, 8.0)
    cfg = flat_cfg(48000, rtype, quantz, b24, ch == 1, ch=ch)
    nodes = graph.graph_shift_master()
    lens = [1500, 2600]
    o1, m1 = run_calls(oracle, icw, cfg, nodes, 3, lens, fir=fir, want_pre=False)
    o2, m2 = run_calls(oracle, icw, cfg, nodes, 3, lens, fir=fir, want_pre=True)
    assert np.array_equal(o1, o2)
    raw = synth.batch_pcm(3, sum(lens), 48000, channels=ch, first=3)
    assert m1 == m2 == ref_meters(oracle, cfg, nodes, list(raw), lens, fir=fir)


@pytest.mark.parametrize("rtype", DITHERS)
@pytest.mark.parametrize("quantz", [abi.QUANTZ_MID_TREAD, abi.QUANTZ_MID_RISER])
@pytest.mark.parametrize("b24", [False, True])
def test_stream1_path(oracle, icw, rtype, quantz, b24, monkeypatch):
    """K5 (one stream, one launch block per call: the drop-in's 576-frame calls), K3a launched ahead
    of it on the same stream"""
    monkeypatch.setenv("ICW_STREAM1", "1")
    monkeypatch.setenv("ICW_K1_MODE", "row")
    cfg = flat_cfg(44100, rtype, quantz, b24, b24)
    nodes = graph.graph_pm_shift_mix()
    lens = [576] * 6 + [1, 19, 1000]
    out, meters = run_calls(oracle, icw, cfg, nodes, 1, lens, want_pre=True)
    raw = synth.batch_pcm(1, sum(lens), 44100, first=3)
    assert meters == ref_meters(oracle, cfg, nodes, list(raw), lens)


@pytest.mark.parametrize("path", ["iir", "fir", "stream1"])
@pytest.mark.parametrize("rtype", DITHERS)
def test_same_bytes_as_serial_render(oracle, icw, path, rtype, monkeypatch):
    """ICW_DITH_PAR=0 renders the same configuration through the serial render (K3a + K3r): the bytes
    and meters are the frame-parallel render's"""
    monkeypatch.setenv("ICW_K1_MODE", "row")
    cfg = flat_cfg(48000, rtype, abi.QUANTZ_MID_RISER, True, False)
    nodes = graph.graph_shift_master()
    n_streams, lens, fir = (1, [576, 576, 300], None) if path == "stream1" else (4, [1200, 3000], None)
    if path == "fir":
        fir = (510, 8.0)
    res = []
    for par in ("1", "0"):
        monkeypatch.setenv("ICW_DITH_PAR", par)
        res.append(run_calls(oracle, icw, cfg, nodes, n_streams, lens, fir=fir, want_pre=False))
    assert np.array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]


@pytest.mark.parametrize("rtype", DITHERS)
@pytest.mark.parametrize("where", ["mid", "edge"])
@pytest.mark.parametrize("path", ["iir", "fir"])
def test_forced_rejects_via_state_blob(oracle, icw, rtype, where, path):
    """mtrnd_gen_dsopen rejects a draw of exactly -1.0 and draws again (mt_jrnd.c:245-256): zeroed raw
    MT words temper to 0 and force rejected pairs, mid-window or straddling the next twist; the state
    blob hands the same words to the GPU context and the oracle stream"""
    cfg = flat_cfg(48000, rtype, abi.QUANTZ_MID_RISER, True, False)
    nodes = graph.graph_master_only()
    fir = (254, 8.0) if path == "fir" else None
    raw = synth.batch_pcm(2, 3000, 48000)
    ctx = icw.Context(cfg, nodes, 2)
    if fir:
        ctx.set_fir_hilbert(*fir)
    o1, _ = ctx.process(raw[:, :700 * 4], 700)
    full = ctx.get_state(1)                              # the blob, then the FIR history if on
    blob = abi.StateBlob.from_buffer_copy(full)
    assert blob.has_render == 1
    words, idx = [], []
    for ch in range(2):
        w = np.frombuffer(bytes(blob.mt[ch]), dtype=np.uint32).copy()
        i0 = blob.mt_idx[ch]
        start = i0 + 5 if where == "mid" else 621
        w[min(start, 623):min(start + 6, 624)] = 0
        if where == "mid" and i0 + 5 >= 624:
            w[:6] = 0
        words.append(w)
        idx.append(i0)
        C.memmove(C.addressof(blob.mt[ch]), w.ctypes.data, 624 * 4)
    ctx.set_state(1, bytes(blob) + full[C.sizeof(blob):])
    o2, p2 = ctx.process(np.ascontiguousarray(raw[:, 700 * 4:]), 2300, want_pre=True)
    st = oracle.Stream(cfg, nodes)
    if fir:
        st.set_fir(*fir)
    r1, _ = st.process(raw[1, :700 * 4], 700)
    assert np.array_equal(o1[1], r1)
    for ch in range(2):
        st.set_mt(ch, words[ch], idx[ch])
    r2, rp2 = st.process(raw[1, 700 * 4:], 2300, want_pre=True)
    assert np.array_equal(p2[1].view(np.uint64), rp2.view(np.uint64))
    assert np.array_equal(o2[1], r2)
    assert ctx.meters(1) == st.meters()
    ctx.close()


def test_render_switch_keeps_generator(oracle, icw):
    """icw_set_render between a frame-parallel dithered render, a noise-shaped one and ROUND: the MT19937
    words carry on through every form (sound_render_setup keeps them), the shaper state restarts"""
    nodes = graph.graph_shift_master()
    cfg = flat_cfg(44100, abi.RENDER_TPDF, abi.QUANTZ_MID_RISER, False, False)
    ctx = icw.Context(cfg, nodes, 2)
    st = [oracle.Stream(cfg, nodes) for _ in range(2)]
    raw = synth.batch_pcm(2, 4000, 44100)
    t = 0
    for i, (rt, ns, n) in enumerate([(abi.RENDER_TPDF, abi.NSHAPE_FLAT, 900), (abi.RENDER_TPDF, abi.NSHAPE_MEW44, 700),
                                     (abi.RENDER_GAUSS, abi.NSHAPE_FLAT, 800), (abi.RENDER_ROUND, abi.NSHAPE_FLAT, 500),
                                     (abi.RENDER_STPDF, abi.NSHAPE_FLAT, 1100)]):
        r = abi.RenderCfg.from_buffer_copy(bytes(cfg.render))
        r.render_type, r.nshape_type = rt, ns
        ctx.set_render(r)
        seg = np.ascontiguousarray(raw[:, t * 4:(t + n) * 4])
        out, _ = ctx.process(seg, n)
        for s in range(2):
            st[s].set_render(r)
            ro, _ = st[s].process(seg[s], n)
            assert np.array_equal(out[s], ro), (i, s)
        t += n
    for s in range(2):
        assert ctx.meters(s) == st[s].meters()
    ctx.close()
