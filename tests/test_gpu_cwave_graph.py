"""GPU parity for the second input format and the general DSP-list form.

CWAVE (complex) input, xwave_reader.c:171-200 and 939-966: the analytic signal is used as read.
The Hilbert converters are bypassed and keep their state across tracks. Fades scale I and Q, and
mono feeds R with L.

Bus-form graphs, adv_modulator.c:636-751: these lists read a slot before it is written in the
frame, which is a one-frame delay and includes feedback loops. They run in the serial graph
kernel with the reference's own bus semantics.
"""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

from test_gpu_parity import assert_parity, run_both

pytestmark = pytest.mark.gpu

CW = [abi.FMT_CW_F64, abi.FMT_CW_I16, abi.FMT_CW_I16_F32, abi.FMT_CW_F32]


@pytest.fixture(autouse=True, params=["plain", "row"])
def k1_mode(request, monkeypatch):
    monkeypatch.setenv("ICW_K1_MODE", request.param)
    return request.param


@pytest.mark.parametrize("fmt", CW)
@pytest.mark.parametrize("ch", [1, 2])
def test_cwave_formats_master_exact(oracle, icw, fmt, ch):
    cfg = graph.default_config(44100, fmt=fmt, channels=ch, need24bits=True)
    raw = synth.batch_pcm(3, 2500, 44100, channels=ch, fmt=fmt)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 2500)
    assert_parity(out, pre, ro, rp, 3, exact_pre=True)


@pytest.mark.parametrize("fmt", CW)
def test_cwave_shift_master(oracle, icw, fmt):
    cfg = graph.default_config(48000, fmt=fmt)
    raw = synth.batch_pcm(8, 4000, 48000, fmt=fmt)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_shift_master(), raw, 4000,
                                   blocks=[576, 1000, 2424])
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


def test_cwave_fades_and_tpdf(oracle, icw):
    cfg = graph.default_config(48000, fmt=abi.FMT_CW_F32)
    cfg.render.render_type = abi.RENDER_TPDF
    n = 30000
    raw = synth.batch_pcm(2, n, 48000, fmt=abi.FMT_CW_F32)
    ctx = icw.Context(cfg, graph.graph_master_only(), 2)
    for s in range(2):
        ctx.stream_open(s, n, fade_in_ms=100, fade_out_ms=200)
    out, pre = ctx.process(raw, n, want_pre=True)
    for s in range(2):
        st = oracle.Stream(cfg, graph.graph_master_only())
        st.open(n, 100, 200)
        ro, rp = st.process(raw[s], n, want_pre=True)
        assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64))
        assert np.array_equal(out[s], ro)


def test_track_switch_keeps_hilbert_state(oracle, icw):
    """WAV track -> CWAVE track -> WAV track in one context: the converters are idle during the
    CWAVE track, and the second WAV track continues from their state (is_clr_hilb_trk FALSE)"""
    fs = 48000
    cfg = graph.default_config(fs)
    nodes = graph.graph_master_only()
    tracks = [(abi.FMT_I16, 2, 3000), (abi.FMT_CW_I16_F32, 1, 2000), (abi.FMT_I16, 2, 2500)]
    ctx = icw.Context(cfg, nodes, 2)
    sts = [oracle.Stream(cfg, nodes) for _ in range(2)]
    for i, (fmt, ch, n) in enumerate(tracks):
        raw = np.stack([synth.batch_pcm(1, n, fs, channels=ch, fmt=fmt, first=10 * i + s)[0] for s in range(2)])
        ctx.set_input(fs, fmt, ch)
        for s in range(2):
            ctx.stream_open(s, n)
        out, pre = ctx.process(raw, n, want_pre=True)
        for s in range(2):
            sts[s].set_input(fs, fmt, ch)
            sts[s].open(n)
            ro, rp = sts[s].process(raw[s], n, want_pre=True)
            assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), f"track {i} stream {s}"
            assert np.array_equal(out[s], ro)


# ------------------------------------------------------------------ bus-form DSP lists --------
@pytest.mark.parametrize("mk,exact", [(graph.graph_pure_delay, False), (graph.graph_leaky_feedback, True),
                                      (graph.graph_feedback_pm_shift, False), (graph.graph_long_chain, True)])
def test_bus_form_graphs(oracle, icw, mk, exact):
    cfg = graph.default_config(48000)
    raw = synth.batch_pcm(6, 3000, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, mk(), raw, 3000, blocks=[576, 1, 1423, 1000])
    assert_parity(out, pre, ro, rp, 2, exact_pre=exact)


def test_bus_form_cwave_gauss(oracle, icw):
    cfg = graph.default_config(48000, fmt=abi.FMT_CW_F64, need24bits=True)
    cfg.render.render_type = abi.RENDER_GAUSS
    cfg.render.nshape_type = abi.NSHAPE_MEW44
    raw = synth.batch_pcm(3, 2000, 48000, fmt=abi.FMT_CW_F64)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_leaky_feedback(), raw, 2000)
    assert_parity(out, pre, ro, rp, 3, exact_pre=True)


def test_bus_form_more_streams_than_a_wave(oracle, icw):
    cfg = graph.default_config(44100)
    raw = synth.batch_pcm(70, 700, 44100)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_leaky_feedback(), raw, 700)
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


# ------------------------------------------------------- dither rejections, state round trip ----
@pytest.mark.parametrize("rtype", [abi.RENDER_TPDF, abi.RENDER_STPDF, abi.RENDER_GAUSS, abi.RENDER_RPDF])
@pytest.mark.parametrize("where", ["mid", "edge"])
def test_dither_rejected_draws_and_state_round_trip(oracle, icw, rtype, where):
    """mtrnd_gen_dsopen rejects a draw of exactly -1.0 and draws again (mt_jrnd.c:245-256).  A raw
    MT word 0 tempers to 0, so zeroed words force rejected pairs; the state blob carries the
    render state, so the same words go into the GPU context and the oracle stream."""
    import ctypes as C
    cfg = graph.default_config(48000, need24bits=True)
    cfg.render.render_type = rtype
    cfg.render.nshape_type = abi.NSHAPE_FW44 if rtype != abi.RENDER_RPDF else abi.NSHAPE_FLAT
    nodes = graph.graph_master_only()
    raw = synth.batch_pcm(2, 3000, 48000)
    ctx = icw.Context(cfg, nodes, 2)
    o1, _ = ctx.process(raw[:, :700 * 4], 700)
    blob = abi.StateBlob.from_buffer_copy(ctx.get_state(1))
    assert blob.has_render == 1
    words, idx = [], []
    for ch in range(2):
        w = np.frombuffer(bytes(blob.mt[ch]), dtype=np.uint32).copy()
        i0 = blob.mt_idx[ch]
        start = i0 + 5 if where == "mid" else 621            # a pair straddling the next twist
        w[min(start, 623):min(start + 6, 624)] = 0
        if where == "mid" and i0 + 5 >= 624:
            w[:6] = 0
        words.append(w)
        idx.append(i0)
        C.memmove(C.addressof(blob.mt[ch]), w.ctypes.data, 624 * 4)
    ctx.set_state(1, bytes(blob))
    o2, p2 = ctx.process(np.ascontiguousarray(raw[:, 700 * 4:]), 2300, want_pre=True)
    st = oracle.Stream(cfg, nodes)
    r1, _ = st.process(raw[1, :700 * 4], 700)
    assert np.array_equal(o1[1], r1)
    for ch in range(2):
        st.set_mt(ch, words[ch], idx[ch])
    r2, rp2 = st.process(raw[1, 700 * 4:], 2300, want_pre=True)
    assert np.array_equal(p2[1].view(np.uint64), rp2.view(np.uint64))
    assert np.array_equal(o2[1], r2)


def test_mono_after_stereo_track(oracle, icw):
    """a mono track right after a stereo one: the converters' states differ, so the right outputs
    must be computed, not copied (the output kernel's mono shortcut needs identical state)"""
    fs = 48000
    cfg = graph.default_config(fs)
    nodes = graph.graph_shift_master()
    ctx = icw.Context(cfg, nodes, 3)
    sts = [oracle.Stream(cfg, nodes) for _ in range(3)]
    for i, (ch, n) in enumerate([(2, 1500), (1, 4000), (1, 2000)]):
        raw = synth.batch_pcm(3, n, fs, channels=ch, first=5 * i)
        ctx.set_input(fs, abi.FMT_I16, ch)
        out, pre = ctx.process(raw, n, want_pre=True)
        for s in range(3):
            sts[s].set_input(fs, abi.FMT_I16, ch)
            ro, rp = sts[s].process(raw[s], n, want_pre=True)
            assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), (i, s)
            assert np.array_equal(out[s], ro), (i, s)
    # the mono tracks after a fresh start do take the shortcut: left == right exactly
    ctx2 = icw.Context(graph.default_config(fs, channels=1), graph.graph_master_only(), 2)
    raw = synth.batch_pcm(2, 3000, fs, channels=1)
    _, pre = ctx2.process(raw, 3000, want_pre=True)
    assert np.array_equal(pre[:, :, 0].view(np.uint64), pre[:, :, 1].view(np.uint64))


@pytest.mark.parametrize("fmt", CW)
def test_dropin_boundary_takes_cwave(oracle, icw, fmt):
    """icw_amod_process_samples (the amod_process_samples drop-in) fed CWAVE blocks the way the
    reader hands them over (576-frame blocks of raw complex samples): WAV track first, then a
    CWAVE track in the same context -- the converters keep their state across it"""
    import ctypes as C
    lib = icw.load()
    fs = 48000
    cfg = graph.default_config(fs)
    nodes = graph.graph_shift_master()
    arr = graph.node_array(nodes)
    st = C.c_int()
    mc = lib.icw_mod_context_create(C.byref(cfg), arr, len(nodes), 0, C.byref(st))
    assert mc and st.value == abi.OK
    ref = oracle.Stream(cfg, nodes)
    osz = lib.icw_mod_context_out_size(mc)
    for track, (f, n) in enumerate([(abi.FMT_I16, 1700), (fmt, 2300)]):
        raw = synth.batch_pcm(1, n, fs, channels=2, fmt=f, first=11 + track)[0]
        assert lib.icw_mod_context_fopen(mc, fs, f, 2, n, 0, 0, 0, 0, 0, cfg.need24bits) == abi.OK
        ref.set_input(fs, f, 2)
        ref.open(n)
        fsz = abi.FMT_BYTES[f] * 2
        got = []
        for t in range(0, n, 576):
            k = min(576, n - t)
            blk = np.ascontiguousarray(raw[t * fsz:(t + k) * fsz])
            buf = np.zeros(k * osz, np.uint8)
            assert lib.icw_amod_process_samples(buf.ctypes.data, mc, blk.ctypes.data, k) == k
            got.append(buf)
        ro, _ = ref.process(raw, n)
        assert np.array_equal(np.concatenate(got), ro), track     # Shift factors glibc-identical
    lib.icw_mod_context_destroy(mc)
