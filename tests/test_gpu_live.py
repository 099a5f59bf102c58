"""GPU parity of live parameter changes: the DSP list, the renders and the Hilbert
converters edited between calls while the streams keep their state, against the oracle given the
same edits at the same frames, bit for bit (pre-render doubles, rendered bytes, meters).

Edits (include/icw.h):
  icw_set_graph          amod_add_lastdsp / amod_del_* / node writes, amod_set_bypass_list_flag
                         (adv_modulator.c:358-425): register form <-> bus form, bypass on / off
  icw_set_render         srenders_set_vcfg -> sound_render_setup (in_cwave.c:457-469,
                         sound_render.c:625-629): ROUND <-> dithered / shaped, sign bits (peaks)
  icw_set_hilbert_filter mod_context_change_all_hilberts_filter (in_cwave.c:186-199)
  icw_set_hilbert_config mod_context_change_all_hilberts_config -> iir_rp_setcfg (hblpf.c:1117-1127)
"""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth
from tests import graphgen
from tests.test_gpu_graph_random import differing

pytestmark = pytest.mark.gpu

N_STREAMS = 3


def random_render(rng):
    r = abi.RenderCfg()
    r.dth_bits = float(rng.choice([0.5, 1.0, 2.0]))
    r.quantz_type = int(rng.integers(0, 2))
    r.render_type = int(rng.choice([abi.RENDER_ROUND, abi.RENDER_ROUND, abi.RENDER_RPDF, abi.RENDER_TPDF,
                                    abi.RENDER_STPDF, abi.RENDER_GAUSS]))
    r.nshape_type = int(rng.choice([abi.NSHAPE_FLAT, abi.NSHAPE_FLAT, abi.NSHAPE_MEW44,
                                    int(rng.integers(0, abi.NSHAPE_MAX + 1))]))
    r.sign_bits16 = int(rng.choice([16, 16, 12, 8]))
    r.sign_bits24 = int(rng.choice([24, 24, 20, 16]))
    return r


def bad_list(rng):
    """a list amod_init rejects: two Masters, or none at the head"""
    nodes = graphgen.random_list(rng, int(rng.integers(2, 5)))
    if rng.random() < 0.5:
        nodes[1] = graph.master(inputs=("in",))
    else:
        nodes = nodes[1:] + nodes[:1]
    return nodes


def random_edit(rng, ctx, refs, log):
    kind = str(rng.choice(["graph", "graph", "render", "render", "filter", "config", "feedback"]))
    if kind in ("graph", "feedback"):
        r = rng.random()
        if kind == "feedback":
            mk = (graph.graph_leaky_feedback, graph.graph_feedback_pm_shift, graph.graph_pure_delay)
            nodes, bypass = mk[int(rng.integers(0, 3))](), 0
        elif r < 0.12:
            nodes, bypass = bad_list(rng), 0
        else:
            nodes, bypass = graphgen.random_list(rng), int(rng.random() < 0.2)
        ok = ctx.set_graph(nodes, bypass)
        for st in refs:
            assert st.set_graph(nodes, bypass) == ok
        log.append(f"graph({len(nodes)} nodes, bypass={bypass}, accepted={ok})")
    elif kind == "render":
        r = random_render(rng)
        ctx.set_render(r)
        for st in refs:
            st.set_render(r)
        log.append(f"render(type={r.render_type}, ns={r.nshape_type}, q={r.quantz_type}, "
                   f"sb={r.sign_bits16}/{r.sign_bits24})")
    elif kind == "filter":
        t = int(rng.integers(0, 6))
        ctx.set_hilbert_filter(t)
        for st in refs:
            st.set_hilbert_filter(t)
        log.append(f"filter({t})")
    else:
        k, sn = int(rng.random() < 0.6), int(rng.random() < 0.7)
        ctx.set_hilbert_config(k, sn)
        for st in refs:
            st.set_hilbert_config(k, sn)
        log.append(f"config(kahan={k}, subn={sn})")


def check_meters(ctx, refs, where):
    for s, st in enumerate(refs):
        m, r = ctx.meters(s), st.meters()
        assert m["clips"] == r["clips"], (where, s, m, r)
        assert m["desubnorm"] == r["desubnorm"], (where, s, m, r)
        assert m["peak_db"] == r["peak_db"], (where, s, m, r)


def run_sequence(oracle, icw, seed, n_calls=6):
    rng = np.random.default_rng(7919 * seed + 3)
    cfg = graphgen.random_config(rng)
    cfg.need24bits = int(rng.random() < 0.4)
    if rng.random() < 0.5:
        cfg.render = random_render(rng)
    nodes = graphgen.random_list(rng)
    lens = [int(x) for x in rng.integers(100, 700, size=n_calls)]
    raw = synth.batch_pcm(N_STREAMS, sum(lens), cfg.sample_rate, first=300 + seed * N_STREAMS)
    ctx = icw.Context(cfg, nodes, N_STREAMS)
    refs = [oracle.Stream(cfg, nodes) for _ in range(N_STREAMS)]
    log, t = [], 0
    for call, n in enumerate(lens):
        if call:
            for _ in range(int(rng.integers(1, 3))):
                random_edit(rng, ctx, refs, log)
        seg = np.ascontiguousarray(raw[:, t * 4:(t + n) * 4])
        out, pre = ctx.process(seg, n, want_pre=True)
        for s, st in enumerate(refs):
            ro, rp = st.process(seg[s], n, want_pre=True)
            bad = differing(pre[s], rp)
            assert bad.size == 0, (f"seed {seed} call {call} stream {s} after {log}: {bad.size} pre-render "
                                   f"doubles differ, first {bad[:4]}")
            assert np.array_equal(out[s], ro), f"seed {seed} call {call} stream {s} after {log}: bytes differ"
        t += n
        if call % 2:
            check_meters(ctx, refs, (seed, call, tuple(log)))
    check_meters(ctx, refs, (seed, "end", tuple(log)))
    ctx.close()
    return log


@pytest.mark.parametrize("batch", range(8))
def test_live_edit_sequences(oracle, icw, batch):
    """random edit sequences: 8 x 10 seeds, 6 calls each, 1-2 edits before every call after the first"""
    kinds = set()
    for seed in range(batch * 10, (batch + 1) * 10):
        for e in run_sequence(oracle, icw, seed):
            kinds.add(e.split("(")[0])
    assert kinds >= {"graph", "render", "filter"}, kinds


def test_graph_register_bus_register_keeps_bus(oracle, icw):
    """register form -> bus form (one-frame feedback) -> register form reading a slot the bus form
    wrote: the 27-slot bus carries across both switches"""
    cfg = graph.default_config(48000)
    reg1 = graph.graph_pm_shift_mix()
    bus = graph.graph_leaky_feedback()
    # a register-form list that reads slot "B" without writing it: the bus form's last value
    reg2 = [graph.master(inputs=("in", "B")), graph.shift(inputs=("in",), out="A", fr=1.5)]
    raw = synth.batch_pcm(2, 1800, 48000, first=41)
    ctx = icw.Context(cfg, reg1, 2)
    refs = [oracle.Stream(cfg, reg1) for _ in range(2)]
    t = 0
    for nodes, n in ((None, 600), (bus, 600), (reg2, 600)):
        if nodes is not None:
            assert ctx.set_graph(nodes)
            for st in refs:
                assert st.set_graph(nodes)
        seg = np.ascontiguousarray(raw[:, t * 4:(t + n) * 4])
        out, pre = ctx.process(seg, n, want_pre=True)
        for s, st in enumerate(refs):
            ro, rp = st.process(seg[s], n, want_pre=True)
            assert differing(pre[s], rp).size == 0 and np.array_equal(out[s], ro), (s, t)
        t += n
    ctx.close()


def test_rejected_graph_keeps_running_list(oracle, icw):
    cfg = graph.default_config(44100)
    nodes = graph.graph_shift_master()
    ctx = icw.Context(cfg, nodes, 1)
    ref = oracle.Stream(cfg, nodes)
    raw = synth.batch_pcm(1, 800, 44100, first=3)
    ctx.process(np.ascontiguousarray(raw[:, :1600]), 400)
    ref.process(raw[0, :1600], 400)
    assert not ctx.set_graph([graph.shift(inputs=("in",), out="A"), graph.master(inputs=("A",))])
    assert not ref.set_graph([graph.shift(inputs=("in",), out="A"), graph.master(inputs=("A",))])
    out, _ = ctx.process(np.ascontiguousarray(raw[:, 1600:]), 400)
    ro, _ = ref.process(raw[0, 1600:], 400)
    assert np.array_equal(out[0], ro)
    ctx.close()


def test_render_change_folds_peaks_and_restarts_shaper(oracle, icw):
    """16-bit ROUND (elementwise, no render state) -> TPDF + MEW44 with 12 sign bits (the serial
    render's state is created on the fly, seeded as the reference's never-used generators) -> back;
    the peak meters keep the maxima measured against each bound"""
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    ctx = icw.Context(cfg, nodes, 2)
    refs = [oracle.Stream(cfg, nodes) for _ in range(2)]
    raw = synth.batch_pcm(2, 1500, 48000, first=61)
    r2 = abi.RenderCfg.from_buffer_copy(cfg.render)
    r2.render_type, r2.nshape_type, r2.sign_bits16 = abi.RENDER_TPDF, abi.NSHAPE_MEW44, 12
    t = 0
    for r, n in ((None, 500), (r2, 500), (cfg.render, 500)):
        if r is not None:
            ctx.set_render(r)
            for st in refs:
                st.set_render(r)
        seg = np.ascontiguousarray(raw[:, t * 4:(t + n) * 4])
        out, _ = ctx.process(seg, n)
        for s, st in enumerate(refs):
            ro, _ = st.process(seg[s], n)
            assert np.array_equal(out[s], ro), (s, t)
        check_meters(ctx, refs, t)
        t += n
    ctx.close()


@pytest.mark.parametrize("dedup", [False, True])
def test_hilbert_filter_and_config_changes(oracle, icw, dedup):
    """type 1 -> 4 (order 20) -> 0 (order 15) -> 0 (no-op) mid-stream, then baseline summation and
    back to Kahan with the reject off: rings re-created, counters restarted.  Mono input exercises
    the K1 dedup, whose identical-converter bookkeeping the re-creation must restore."""
    cfg = graph.default_config(96000, channels=1 if dedup else 2)
    nodes = graph.graph_master_only()
    ctx = icw.Context(cfg, nodes, 4)
    refs = [oracle.Stream(cfg, nodes) for _ in range(4)]
    fsz = 2 * cfg.in_channels
    raw = synth.batch_pcm(4, 6 * 700, 96000, channels=cfg.in_channels, first=80)
    edits = [None, ("f", 4), ("f", 0), ("f", 0), ("c", (0, 1)), ("c", (1, 0))]
    t = 0
    for e in edits:
        if e is not None:
            for tgt in [ctx] + refs:
                if e[0] == "f":
                    tgt.set_hilbert_filter(e[1])
                else:
                    tgt.set_hilbert_config(*e[1])
        seg = np.ascontiguousarray(raw[:, t * fsz:(t + 700) * fsz])
        out, pre = ctx.process(seg, 700, want_pre=True)
        for s, st in enumerate(refs):
            ro, rp = st.process(seg[s], 700, want_pre=True)
            assert differing(pre[s], rp).size == 0 and np.array_equal(out[s], ro), (e, s)
        check_meters(ctx, refs, e)
        t += 700
    ctx.close()


@pytest.mark.parametrize("mono", [False, True])
def test_edits_between_multi_block_calls(oracle, icw, mono):
    """calls long enough for several launch blocks (the multi-stream pipeline, block scratch sets,
    the serial render one block behind): ROUND register form -> TPDF + MEW44 behind a bus-form
    list (serial render state created between calls) -> filter type 4 -> back to ROUND + register
    form; every block of every call bit for bit"""
    ch = 1 if mono else 2
    cfg = graph.default_config(48000, channels=ch)
    nodes = graph.graph_shift_master()
    n = 36000
    raw = synth.batch_pcm(3, 4 * n, 48000, channels=ch, first=500)
    fsz = 2 * ch
    ctx = icw.Context(cfg, nodes, 3)
    refs = [oracle.Stream(cfg, nodes) for _ in range(3)]
    r2 = abi.RenderCfg.from_buffer_copy(cfg.render)
    r2.render_type, r2.nshape_type = abi.RENDER_TPDF, abi.NSHAPE_MEW44

    def edit_graph(t, nn):
        assert t.set_graph(nn)

    edits = [None,
             [lambda t: t.set_render(r2), lambda t: edit_graph(t, graph.graph_feedback_pm_shift())],
             [lambda t: t.set_hilbert_filter(4)],
             [lambda t: t.set_render(cfg.render), lambda t: edit_graph(t, graph.graph_pm_shift_mix())]]
    for k, e in enumerate(edits):
        for f in (e or []):
            for tgt in [ctx] + refs:
                f(tgt)
        seg = np.ascontiguousarray(raw[:, k * n * fsz:(k + 1) * n * fsz])
        out, pre = ctx.process(seg, n, want_pre=True)
        for s, st in enumerate(refs):
            ro, rp = st.process(seg[s], n, want_pre=True)
            bad = differing(pre[s], rp)
            assert bad.size == 0, (k, s, bad[:4])
            assert np.array_equal(out[s], ro), (k, s)
        check_meters(ctx, refs, k)
    ctx.close()


def test_edits_with_fir_converter(oracle, icw):
    """the FIR Hilbert converter on (fused KF2 while the list fits its LDS, KF + K2 otherwise):
    list and render edits between calls, the converter's history carried; a Hilbert-type change
    leaves the FIR converter alone (it replaces the quadrature IIR)"""
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    ctx = icw.Context(cfg, nodes, 2)
    ctx.set_fir_hilbert(254, 8.0)
    refs = [oracle.Stream(cfg, nodes) for _ in range(2)]
    for st in refs:
        st.set_fir(254, 8.0)
    r2 = abi.RenderCfg.from_buffer_copy(cfg.render)
    r2.render_type, r2.nshape_type = abi.RENDER_RPDF, abi.NSHAPE_FLAT
    edits = [None,
             [lambda t: t.set_graph(graph.graph_pm_shift_mix())],
             [lambda t: t.set_render(r2), lambda t: t.set_hilbert_filter(3)],
             [lambda t: t.set_graph(graph.graph_leaky_feedback())],
             [lambda t: t.set_graph(graph.graph_master_only())]]
    n = 5000
    raw = synth.batch_pcm(2, n * len(edits), 48000, first=700)
    for k, e in enumerate(edits):
        for f in (e or []):
            for tgt in [ctx] + refs:
                f(tgt)
        seg = np.ascontiguousarray(raw[:, k * n * 4:(k + 1) * n * 4])
        out, pre = ctx.process(seg, n, want_pre=True)
        for s, st in enumerate(refs):
            ro, rp = st.process(seg[s], n, want_pre=True)
            assert differing(pre[s], rp).size == 0 and np.array_equal(out[s], ro), (k, s)
        check_meters(ctx, refs, k)
    ctx.close()


def test_dropin_context_live_edits(oracle, icw):
    """the drop-in boundary: icw_amod_process_samples in 576-frame blocks (playback.c:619), with
    the GUI's edits applied between blocks through icw_mod_context_ctx -- list, render, filter"""
    import ctypes as C
    lib = icw.load()
    fs = 44100
    cfg = graph.default_config(fs)
    nodes = graph.graph_shift_master()
    arr = graph.node_array(nodes)
    st = C.c_int()
    mc = lib.icw_mod_context_create(C.byref(cfg), arr, len(nodes), 0, C.byref(st))
    assert mc and st.value == abi.OK
    ctx = lib.icw_mod_context_ctx(mc)
    assert ctx
    ref = oracle.Stream(cfg, nodes)
    osz = lib.icw_mod_context_out_size(mc)
    n = 576 * 12
    raw = synth.batch_pcm(1, n, fs, first=31)[0]
    r2 = abi.RenderCfg.from_buffer_copy(cfg.render)
    r2.render_type, r2.nshape_type = abi.RENDER_TPDF, abi.NSHAPE_MEW44
    pm = graph.graph_pm_shift_mix()
    got, ro = [], []
    for b in range(12):
        if b == 3:
            acc = C.c_int()
            assert lib.icw_set_graph(ctx, graph.node_array(pm), len(pm), 0, C.byref(acc)) == abi.OK and acc.value
            assert ref.set_graph(pm)
        if b == 6:
            assert lib.icw_set_render(ctx, C.byref(r2)) == abi.OK
            ref.set_render(r2)
        if b == 9:
            assert lib.icw_set_hilbert_filter(ctx, 2) == abi.OK
            ref.set_hilbert_filter(2)
        blk = np.ascontiguousarray(raw[b * 576 * 4:(b + 1) * 576 * 4])
        buf = np.zeros(576 * osz, np.uint8)
        assert lib.icw_amod_process_samples(buf.ctypes.data, mc, blk.ctypes.data, 576) == 576
        got.append(buf)
        o, _ = ref.process(blk, 576)
        ro.append(o)
    for b in range(12):
        assert np.array_equal(got[b], ro[b]), b
    lib.icw_mod_context_destroy(mc)


@pytest.mark.parametrize("form", ["register", "bus"])
def test_deleted_writer_slot_reads_zero(oracle, icw, form):
    """amod_del_lastdsp / amod_set_output_plug -> replace_output_plug (adv_modulator.c:176-209): the
    removed or re-plugged node's old slot is zeroed in every stream (mod_context_clear_all_inouts,
    in_cwave.c:255-261) while a Mix still reads it; icw_clear_bus_slot is the primitive itself.  The
    bus form (a one-frame delay: the Mix reads A before the Shift writes it) reads the cleared slot
    in the first frame of the next call."""
    cfg = graph.default_config(48000)
    if form == "register":
        l1 = [graph.master(inputs=("C",)), graph.mix(inputs=("in", "A"), out="C"),
              graph.shift(inputs=("in",), out="A", fr=3.0)]
    else:
        l1 = [graph.master(inputs=("C",)), graph.shift(inputs=("in",), out="A", fr=3.0),
              graph.mix(inputs=("in", "A"), out="C")]
    # register form: the writer deleted; bus form: a parameter edit keeps A, the explicit clear zeroes it
    l2 = l1[:2] if form == "register" else [l1[0], graph.shift(inputs=("in",), out="A", fr=5.0), l1[2]]
    l3 = [l2[0], l2[1], graph.mix(inputs=("in", "A"), out="D")]      # re-plugged C -> D: C cleared
    raw = synth.batch_pcm(3, 2400, 48000, first=77)
    ctx = icw.Context(cfg, l1, 3)
    refs = [oracle.Stream(cfg, l1) for _ in range(3)]
    t = 0
    for step in ("none", "l2", "clear", "l3"):
        if step in ("l2", "l3"):
            nn = l2 if step == "l2" else l3
            assert ctx.set_graph(nn)
            for st in refs:
                assert st.set_graph(nn)
        elif step == "clear":
            ctx.clear_bus_slot(graph.slot("A"))
            for st in refs:
                st.clear_bus_slot(graph.slot("A"))
        seg = np.ascontiguousarray(raw[:, t * 4:(t + 600) * 4])
        out, pre = ctx.process(seg, 600, want_pre=True)
        for s, st in enumerate(refs):
            ro, rp = st.process(seg[s], 600, want_pre=True)
            assert differing(pre[s], rp).size == 0 and np.array_equal(out[s], ro), (step, s)
        t += 600
    ctx.close()
