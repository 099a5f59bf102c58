"""Live parameter changes, CPU side: the oracle's restatement of the edits checked by
properties that follow from the reference's own definitions, and the C-ABI argument checks that
need no GPU.  The GPU parity of the same edits is tests/test_gpu_live.py.

  mod_context_change_all_hilberts_filter (in_cwave.c:186-199) re-creates the converters: after it, a
    stateless graph and render give what a fresh stream of the new type gives on the same input;
  mod_context_change_all_hilberts_config -> iir_rp_setcfg (hblpf.c:1117-1127) keeps the rings and
    restarts the de-subnorm counters;
  srenders_set_vcfg -> sound_render_setup (sound_render.c:625-629): after ROUND (which draws nothing)
    the new render runs as a freshly seeded one on the same pre-render doubles;
  amod_del_* / amod_set_output_plug zero the removed / re-plugged node's old slot (replace_output_plug,
    adv_modulator.c:176-209); every other slot keeps its value.
"""
import numpy as np

from in_cwave_amd import abi, graph, synth


def test_filter_change_equals_fresh_converters(oracle):
    cfg = graph.default_config(48000)
    nodes = graph.graph_master_only()
    raw = synth.batch_pcm(1, 1200, 48000, first=11)[0]
    a = oracle.Stream(cfg, nodes)
    a.process(raw[:600 * 4], 600)
    for t in (4, 0, 5):
        a.set_hilbert_filter(t)
        cfg_t = graph.default_config(48000, hilbert_type=t)
        b = oracle.Stream(cfg_t, nodes)
        oa, pa = a.process(raw[600 * 4:], 600, want_pre=True)
        ob, pb = b.process(raw[600 * 4:], 600, want_pre=True)
        assert np.array_equal(pa.view(np.uint64), pb.view(np.uint64)), t
        assert np.array_equal(oa, ob), t


def test_same_filter_is_a_no_op(oracle):
    cfg = graph.default_config(44100)
    nodes = graph.graph_shift_master()
    raw = synth.batch_pcm(1, 800, 44100, first=12)[0]
    a, b = oracle.Stream(cfg, nodes), oracle.Stream(cfg, nodes)
    a.process(raw[:1600], 400)
    b.process(raw[:1600], 400)
    a.set_hilbert_filter(1)
    oa, _ = a.process(raw[1600:], 400)
    ob, _ = b.process(raw[1600:], 400)
    assert np.array_equal(oa, ob)


def test_config_change_keeps_rings_restarts_counter(oracle):
    cfg = graph.default_config(48000)
    nodes = graph.graph_master_only()
    # silence after a burst drives the DF-II states below the reject threshold
    raw = np.zeros(60000 * 4, dtype=np.uint8)
    raw[:400 * 4] = synth.batch_pcm(1, 400, 48000, first=13)[0][:400 * 4]
    a, b = oracle.Stream(cfg, nodes), oracle.Stream(cfg, nodes)
    a.process(raw, 60000)
    b.process(raw, 60000)
    assert a.meters()["desubnorm"] > 0
    a.set_hilbert_config(1, 1)                   # same summation: rings kept, counters restart
    assert a.meters()["desubnorm"] == 0
    tail = synth.batch_pcm(1, 500, 48000, first=14)[0]
    oa, pa = a.process(tail, 500, want_pre=True)
    ob, pb = b.process(tail, 500, want_pre=True)
    assert np.array_equal(pa.view(np.uint64), pb.view(np.uint64))
    a.set_hilbert_config(0, 1)                   # baseline sums from the same rings
    oa2, pa2 = a.process(tail, 500, want_pre=True)
    ob2, pb2 = b.process(tail, 500, want_pre=True)
    assert not np.array_equal(pa2.view(np.uint64), pb2.view(np.uint64))
    # the same signal: the baseline adds the d0 * w term the Kahan form omits (hblpf.c:1026-1043)
    assert np.max(np.abs(pa2 - pb2)) < 0.02 * np.max(np.abs(pb2))


def test_render_change_after_round_is_a_fresh_render(oracle):
    cfg = graph.default_config(48000, need24bits=True)
    nodes = graph.graph_shift_master()
    raw = synth.batch_pcm(1, 1000, 48000, first=15)[0]
    a = oracle.Stream(cfg, nodes)
    a.process(raw[:400 * 4], 400)
    r = abi.RenderCfg.from_buffer_copy(cfg.render)
    r.render_type, r.nshape_type = abi.RENDER_TPDF, abi.NSHAPE_MEW44
    a.set_render(r)
    out, pre = a.process(raw[400 * 4:], 600, want_pre=True)
    osz = 3
    got = out.reshape(600, 2, osz)
    for ch, seed in ((0, abi.SEED_LEFT), (1, abi.SEED_RIGHT)):
        ref, _, _, _ = oracle.render_block(pre[:, ch], r, is24=True, seed=seed)
        assert np.array_equal(got[:, ch, :].reshape(-1), ref), ch


def test_graph_change_clears_removed_writers_and_rejects_bad_lists(oracle):
    """amod_del_lastdsp -> replace_output_plug (adv_modulator.c:176-209, 377-390): the deleted node's
    output slot is zeroed in every context (mod_context_clear_all_inouts, in_cwave.c:255-261), so a
    node still reading it reads 0 from then on"""
    cfg = graph.default_config(48000)
    writer = [graph.master(inputs=("A",)), graph.shift(inputs=("in",), out="A", fr=2.5)]
    reader = [graph.master(inputs=("A",))]        # the Shift deleted: A is cleared
    raw = synth.batch_pcm(1, 600, 48000, first=16)[0]
    a = oracle.Stream(cfg, writer)
    _, p1 = a.process(raw[:300 * 4], 300, want_pre=True)
    assert np.any(p1 != 0.0)
    assert not a.set_graph([graph.shift(inputs=("in",), out="A"), graph.master(inputs=("A",))])
    assert not a.set_graph([graph.master(), graph.master()])
    assert a.set_graph(reader)
    _, p2 = a.process(raw[300 * 4:], 300, want_pre=True)
    assert np.all(p2 == 0.0)


def test_graph_change_keeps_other_slots(oracle):
    """a parameter edit keeps every slot: a one-frame delay (Mix reads A before the Shift writes it
    in the frame, doc 3.1) sees last call's A in the first frame of the next call; an explicit
    mod_context_clear_all_inouts of A makes that first frame read 0 instead"""
    cfg = graph.default_config(48000)
    delay = [graph.master(inputs=("B",)), graph.shift(inputs=("in",), out="A", fr=2.0),
             graph.mix(inputs=("A",), out="B")]
    edited = [graph.master(inputs=("B",)), graph.shift(inputs=("in",), out="A", fr=3.0),
              graph.mix(inputs=("A",), out="B", gain=0.7)]
    raw = synth.batch_pcm(1, 600, 48000, first=17)[0]
    a, b = oracle.Stream(cfg, delay), oracle.Stream(cfg, delay)
    for st in (a, b):
        st.process(raw[:300 * 4], 300)
        assert st.set_graph(edited)
    b.clear_bus_slot(graph.slot("A"))
    _, pa = a.process(raw[300 * 4:], 300, want_pre=True)
    _, pb = b.process(raw[300 * 4:], 300, want_pre=True)
    assert np.any(pa[0] != 0.0) and np.all(pb[0] == 0.0)
    assert np.array_equal(pa[1:], pb[1:])
    # position matching: the Mix re-plugged to C clears B (the Master reads it, nobody writes it)
    c = oracle.Stream(cfg, delay)
    c.process(raw[:300 * 4], 300)
    assert c.set_graph(edited[:2] + [graph.mix(inputs=("A",), out="C")])
    _, pc = c.process(raw[300 * 4:], 300, want_pre=True)
    assert np.all(pc == 0.0)


def test_live_setters_reject_bad_arguments_without_gpu(icw):
    """argument checks come before any device call"""
    lib = icw.load()
    assert lib.icw_set_hilbert_filter(None, 1) == abi.EINVAL
    assert lib.icw_set_hilbert_config(None, 1, 1) == abi.EINVAL
    assert lib.icw_set_render(None, None) == abi.EINVAL
    assert lib.icw_set_graph(None, None, 0, 0, None) == abi.EINVAL
    assert lib.icw_clear_bus_slot(None, 1) == abi.EINVAL
