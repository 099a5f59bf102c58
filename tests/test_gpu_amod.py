"""The drop-in boundary as the reference's plugin uses it: two decoding contexts at once (playback and
transcode, the.mc_playback / the.mc_transcode, in_cwave.h:473-474), one DSP list and one set of
clip / peak meters shared by both (the `am` singleton, adv_modulator.c:49-60), and the GUI's list
primitives applied one at a time (amod_gui_control.c:1125, 1165, 1172, 1858).

The oracle side is driven the reference's way: two streams render into ONE meter accumulator
(orc_share_meters: sound_render_value(&buf, lOut, &am.l_clips, &am.l_peak, ...),
adv_modulator.c:757-758), amod_get_clips_peaks reads and resets it (adv_modulator.c:445-465), and
each list primitive runs replace_output_plug itself (adv_modulator.c:176-209) -- not the position
diff icw_set_graph uses for whole-list edits."""
import ctypes as C

import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

pytestmark = pytest.mark.gpu


def _loud_i16(n, fs, first, amp):
    """stereo int16 at `amp` of full scale (two sines per channel): the Master's gain drives it into
    the render's clip bounds now and then"""
    raw = synth.stream_pcm(first, n, fs).view(np.int16).astype(np.float64)
    raw *= amp / max(1.0, np.abs(raw).max() / 32767.0)
    return np.clip(np.round(raw), -32768, 32767).astype(np.int16).view(np.uint8)


class _Mod:
    """one icw_mod_context (the product) beside one oracle stream (the reference context)"""

    def __init__(self, icw, oracle, cfg, nodes, fs, fmt, ch, n_samples):
        self.lib = icw.load()
        arr = graph.node_array(nodes)
        st = C.c_int()
        self.mc = self.lib.icw_mod_context_create(C.byref(cfg), arr, len(nodes), 0, C.byref(st))
        assert self.mc and st.value == abi.OK
        assert self.lib.icw_mod_context_fopen(self.mc, fs, fmt, ch, n_samples, 0, 0, 0, 0, 0, cfg.need24bits) == abi.OK
        self.ref = oracle.Stream(cfg, nodes)
        self.ref.set_input(fs, fmt, ch)
        self.ref.open(n_samples)
        self.fsz = abi.FMT_BYTES[fmt] * ch
        self.osz = self.lib.icw_mod_context_out_size(self.mc)

    def block(self, raw, n):
        buf = np.zeros(n * self.osz, np.uint8)
        blk = np.ascontiguousarray(raw[:n * self.fsz])
        assert self.lib.icw_amod_process_samples(buf.ctypes.data, self.mc, blk.ctypes.data, n) == n
        ro, _ = self.ref.process(blk, n)
        assert np.array_equal(buf, ro)

    def close(self):
        self.lib.icw_mod_context_destroy(self.mc)


def _clips_peaks(lib, mods, reset):
    arr = (C.c_void_p * len(mods))(*[m.mc for m in mods])
    lc, rc, lp, rp = C.c_uint(), C.c_uint(), C.c_double(), C.c_double()
    assert lib.icw_amod_get_clips_peaks(arr, len(mods), C.byref(lc), C.byref(rc), C.byref(lp), C.byref(rp),
                                        int(reset)) == abi.OK
    return {"clips": (lc.value, rc.value), "peak_db": (lp.value, rp.value)}


def _amod(lib, mods, name, *args):
    arr = (C.c_void_p * len(mods))(*[m.mc for m in mods])
    return getattr(lib, "icw_amod_" + name)(arr, len(mods), *args)


def test_global_meters_two_contexts(oracle, icw):
    """amod_get_clips_peaks over the playback and the transcode context, decoding different tracks in
    interleaved calls (576-frame playback blocks, 1000-frame transcode reads): clips summed, peaks
    maxed, and a reset in the middle clears both -- against one oracle accumulator fed by both
    streams in call order"""
    cfg = graph.default_config(44100)
    nodes = [graph.master(inputs=("A",), gain=1.9), graph.shift(inputs=("in",), out="A")]
    n_pb, n_tc = 576 * 16, 1000 * 10
    pb = _Mod(icw, oracle, cfg, nodes, 44100, abi.FMT_I16, 2, n_pb)
    tc = _Mod(icw, oracle, cfg, nodes, 48000, abi.FMT_F32, 1, n_tc)
    tc.ref.share_meters(pb.ref)                     # the reference's one `am` accumulator
    a = _loud_i16(n_pb, 44100, 3, 0.9)
    b = (0.6 * np.sin(np.arange(n_tc) * 0.031)).astype(np.float32).view(np.uint8)
    lib = pb.lib
    saw_clips = False
    for k in range(16):
        pb.block(a[k * 576 * 4:], 576)
        if k < 10:
            tc.block(b[k * 1000 * 4:], 1000)
        reset = k == 7
        got = _clips_peaks(lib, [pb, tc], reset)
        want = pb.ref.clips_peaks(reset)
        assert got == want, (k, got, want)
        saw_clips = saw_clips or got["clips"][0] > 0
        if reset:
            assert got == {"clips": (0, 0), "peak_db": (abi.SR_ZERO_SIGNAL_DB, abi.SR_ZERO_SIGNAL_DB)}
    assert saw_clips, "the test input never clipped"
    for m in (pb, tc):
        m.close()


def test_list_primitives_two_contexts(oracle, icw):
    """The GUI's list edits over both contexts (icw_amod_*), primitive by primitive, between blocks:
    delete the tail and add an identical node back (same mode, same slot: the reference clears the
    slot, a position diff would not), re-plug to the same slot, a removal-only plug, a new node, the
    whole list deleted.  The tail is a Mix feeding itself, C = 0.5 (in + C[t-1]): a bus-form reader
    of its own slot, so every clear shows in the output."""
    cfg = graph.default_config(44100)
    feedback = graph.mix(inputs=("in", "C"), out="C", gain=0.5)
    nodes = [graph.master(inputs=("C", "A")), graph.shift(inputs=("in",), out="A", gain=0.3), feedback]
    n = 576 * 14
    pb = _Mod(icw, oracle, cfg, nodes, 44100, abi.FMT_I16, 2, n)
    tc = _Mod(icw, oracle, cfg, nodes, 48000, abi.FMT_I16, 1, n)
    tc.ref.share_meters(pb.ref)
    a = synth.stream_pcm(8, n, 44100)
    b = synth.stream_pcm(9, n, 48000, channels=1)
    lib = pb.lib
    mods = [pb, tc]
    edits = {
        2: [("del_lastdsp",), ("add_lastdsp", feedback)],        # same mode, same slot C
        4: [("set_output_plug", 2, graph.slot("C"))],             # re-plug to the same slot
        6: [("set_output_plug", 1, -1)],                          # remove-only: A cleared, n_out kept
        8: [("add_lastdsp", graph.pm(inputs=("C",), out="D"))],
        10: [("del_dsplist",), ("add_lastdsp", feedback)],
        12: [("del_lastdsp",)],
    }
    for k in range(14):
        for e in edits.get(k, []):
            name, args = e[0], e[1:]
            c_args = [C.byref(x) if isinstance(x, abi.Node) else x for x in args]
            assert _amod(lib, mods, name, *c_args) == abi.OK, e
            for m in mods:
                getattr(m.ref, name)(*args)
        pb.block(a[k * 576 * 4:], 576)
        tc.block(b[k * 576 * 2:], 576)
        assert _clips_peaks(lib, mods, False) == pb.ref.clips_peaks(False), k
    # a Master cannot be added (create_node_dsp returns NULL for it)
    assert _amod(lib, mods, "add_lastdsp", C.byref(graph.master())) == abi.EGRAPH
    for m in mods:
        m.close()


def test_graph_primitives_batched_context(oracle, icw):
    """the icw.h primitives on a many-stream context (icw_graph_*), streams with different inputs,
    checked frame for frame against per-stream oracles driven primitive by primitive"""
    cfg = graph.default_config(48000)
    fb = graph.mix(inputs=("in", "B"), out="B", gain=0.25)
    nodes = [graph.master(inputs=("B",)), graph.pm(inputs=("in",), out="A"), fb]
    S = 5
    raw = synth.batch_pcm(S, 6000, 48000, first=40)
    ctx = icw.Context(cfg, nodes, S)
    refs = [oracle.Stream(cfg, nodes) for _ in range(S)]
    steps = [None, ("graph_del_last", "del_lastdsp", ()), ("graph_add_last", "add_lastdsp", (fb,)),
             ("graph_set_output_plug", "set_output_plug", (2, graph.slot("B"))),
             ("graph_set_output_plug", "set_output_plug", (1, graph.slot("E"))),
             ("graph_del_all", "del_dsplist", ())]
    for k, stp in enumerate(steps):
        if stp:
            getattr(ctx, stp[0])(*stp[2])
            for r in refs:
                getattr(r, stp[1])(*stp[2])
        seg = np.ascontiguousarray(raw[:, k * 1000 * 4:(k + 1) * 1000 * 4])
        out, pre = ctx.process(seg, 1000, want_pre=True)
        for s in range(S):
            ro, rp = refs[s].process(seg[s], 1000, want_pre=True)
            assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), (k, s)
            assert np.array_equal(out[s], ro), (k, s)
    ctx.close()


def _meters_equal(lib, m):
    got = abi.Meters()
    assert lib.icw_mod_context_meters(m.mc, 0, C.byref(got)) == abi.OK
    want = m.ref.meters()
    assert (got.clips[0], got.clips[1]) == want["clips"]
    assert (got.peak_db[0], got.peak_db[1]) == want["peak_db"]
    assert got.desubnorm == want["desubnorm"]


def test_track_bit_depth_follows_fopen(oracle, icw):
    """mod_context_fopen applies the.cfg.need24bits to both renders at every track open
    (in_cwave.c:212, 233-234 -> sound_render_set_outbits, sound_render.c:617-621), and the GUI flips the
    flag between tracks (amod_gui_control.c:1641).  One drop-in context, three tracks: 16-bit, then
    24-bit, then 16-bit, 576-frame blocks (playback.c:619) with a short last block, a TPDF + MEW44
    render (the generators go on across the tracks, the shaper state restarts at each open), no
    is_clr_*: the Hilbert rings and the frame counter carry over.  Bytes and meters equal the oracle's
    after every block, and out_size follows each track (playback.c:215 sizes the buffer from it)."""
    cfg = graph.default_config(44100)
    cfg.render.render_type = abi.RENDER_TPDF
    cfg.render.nshape_type = abi.NSHAPE_MEW44
    nodes = [graph.master(inputs=("A",), gain=1.6), graph.shift(inputs=("in",), out="A")]
    lib = icw.load()
    st = C.c_int()
    mc = lib.icw_mod_context_create(C.byref(cfg), graph.node_array(nodes), len(nodes), 0, C.byref(st))
    assert mc and st.value == abi.OK
    ref = oracle.Stream(cfg, nodes)
    m = type("M", (), {})()
    m.mc, m.ref = mc, ref
    tracks = [(44100, abi.FMT_I16, 2, False), (48000, abi.FMT_F32, 1, True), (44100, abi.FMT_I16, 2, False),
              (96000, abi.FMT_I24, 2, True)]
    for t, (fs, fmt, ch, b24) in enumerate(tracks):
        n = 576 * 5 + 100
        assert lib.icw_mod_context_fopen(mc, fs, fmt, ch, n, 0, 0, 0, 0, 0, int(b24)) == abi.OK
        ref.set_input(fs, fmt, ch)
        ref.open(n, need24bits=b24)
        osz = lib.icw_mod_context_out_size(mc)
        assert osz == (6 if b24 else 4)
        if fmt == abi.FMT_I16:
            raw = _loud_i16(n, fs, 20 + t, 0.95)
        else:
            raw = synth.stream_pcm(20 + t, n, fs, channels=ch, fmt=fmt)
        fsz = abi.FMT_BYTES[fmt] * ch
        for k in range(0, n, 576):
            nb = min(576, n - k)
            blk = np.ascontiguousarray(raw[k * fsz:(k + nb) * fsz])
            buf = np.zeros(nb * osz, np.uint8)
            assert lib.icw_amod_process_samples(buf.ctypes.data, mc, blk.ctypes.data, nb) == nb
            ro, _ = ref.process(blk, nb)
            assert np.array_equal(buf, ro), (t, k)
            _meters_equal(lib, m)
    lib.icw_mod_context_destroy(mc)


@pytest.mark.parametrize("rtype,ns", [(abi.RENDER_ROUND, abi.NSHAPE_FLAT), (abi.RENDER_GAUSS, abi.NSHAPE_FLAT),
                                      (abi.RENDER_RPDF, abi.NSHAPE_FW44)])
def test_set_outbits_batched(oracle, icw, rtype, ns):
    """icw_set_outbits on a many-stream context between calls (a new track on every stream): the
    render-in-K2 ROUND path and the serial render, 24 -> 16 -> 24 bit, against per-stream oracles
    given sound_render_set_outbits at the same points; pre-render doubles, bytes and meters"""
    cfg = graph.default_config(48000, need24bits=True)
    cfg.render.render_type = rtype
    cfg.render.nshape_type = ns
    nodes = graph.graph_pm_shift_mix()
    S = 3
    raw = synth.batch_pcm(S, 9000, 48000, first=60)
    ctx = icw.Context(cfg, nodes, S)
    refs = [oracle.Stream(cfg, nodes) for _ in range(S)]
    for k, b24 in enumerate([True, False, True]):
        if k:
            ctx.set_outbits(b24)
            for r in refs:
                r.set_outbits(b24)
        assert ctx.render_size == (3 if b24 else 2)
        seg = np.ascontiguousarray(raw[:, k * 3000 * 4:(k + 1) * 3000 * 4])
        out, pre = ctx.process(seg, 3000, want_pre=k == 1)
        for s in range(S):
            ro, rp = refs[s].process(seg[s], 3000, want_pre=k == 1)
            assert np.array_equal(out[s], ro), (k, s)
            if k == 1:
                assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), (k, s)
            got, want = ctx.meters(s), refs[s].meters()
            assert got["clips"] == want["clips"] and got["peak_db"] == want["peak_db"], (k, s)
    ctx.close()
