"""CPU side of the drop-in's shared-state semantics (tests/test_gpu_amod.py runs the GPU half): the
oracle's list primitives and its one meter accumulator for several decoding contexts."""
import numpy as np

from in_cwave_amd import abi, graph, synth


def test_del_add_same_slot_differs_from_position_diff(oracle):
    """the case the primitives exist for: del_lastdsp + add_lastdsp of an identical self-feeding Mix
    clears its slot in the reference, while a whole-list edit matched by position keeps it -- the two
    oracle runs must differ, or the GPU test above could not tell the rules apart"""
    cfg = graph.default_config(44100)
    fb = graph.mix(inputs=("in", "C"), out="C", gain=0.5)
    nodes = [graph.master(inputs=("C",)), fb]
    raw = synth.stream_pcm(5, 2000, 44100)
    outs = []
    for prim in (True, False):
        st = oracle.Stream(cfg, nodes)
        st.process(raw[:1000 * 4], 1000)
        if prim:
            st.del_lastdsp()
            st.add_lastdsp(fb)
        else:
            assert st.set_graph(nodes)
        outs.append(st.process(raw[1000 * 4:], 1000)[0])
    assert not np.array_equal(outs[0], outs[1])


def test_shared_meter_accumulator(oracle):
    """two oracle streams rendering into one accumulator (orc_share_meters, the reference's `am`
    meters, adv_modulator.c:757-758): clips add up and the peak is the larger one; a reset through
    either stream clears the one accumulator (amod_get_clips_peaks, adv_modulator.c:445-465)"""
    cfg = graph.default_config(44100)
    nodes = [graph.master(gain=3.0)]
    loud = synth.stream_pcm(1, 3000, 44100)
    quiet = (synth.stream_pcm(2, 3000, 44100).view(np.int16) // 64).view(np.uint8)
    a, b, a1, b1 = (oracle.Stream(cfg, nodes) for _ in range(4))
    b.share_meters(a)
    a.process(loud, 3000)
    b.process(quiet, 3000)
    a1.process(loud, 3000)
    b1.process(quiet, 3000)
    g, ma, mb = a.clips_peaks(), a1.meters(), b1.meters()
    assert ma["clips"][0] > 0
    assert g["clips"] == (ma["clips"][0] + mb["clips"][0], ma["clips"][1] + mb["clips"][1])
    assert g["peak_db"] == (max(ma["peak_db"][0], mb["peak_db"][0]), max(ma["peak_db"][1], mb["peak_db"][1]))
    assert b.clips_peaks() == g
    z = b.clips_peaks(reset=True)
    assert z == {"clips": (0, 0), "peak_db": (abi.SR_ZERO_SIGNAL_DB, abi.SR_ZERO_SIGNAL_DB)}
    assert a.clips_peaks() == z


def test_list_primitives_clear_rules(oracle):
    """replace_output_plug (adv_modulator.c:176-209) as the oracle restates it: del_lastdsp clears
    the removed node's slot, a Master removal is impossible (the head stays), set_output_plug clears
    the old slot also for a re-plug to the same slot and for the remove-only form (n_out kept), and
    add_lastdsp clears nothing and refuses a Master"""
    cfg = graph.default_config(44100)
    nodes = [graph.master(inputs=("A",)), graph.mix(inputs=("in", "A"), out="A", gain=0.5)]
    raw = synth.stream_pcm(6, 4000, 44100)

    def run(edit):
        st = oracle.Stream(cfg, nodes)
        st.process(raw[:2000 * 4], 2000)
        edit(st)
        return st.process(raw[2000 * 4:], 2000)[0]

    base = run(lambda st: None)
    replug = run(lambda st: st.set_output_plug(1, graph.slot("A")))
    remove_only = run(lambda st: st.set_output_plug(1, -1))
    assert not np.array_equal(base, replug)
    assert np.array_equal(replug, remove_only)       # both clear A; the node keeps writing A
    st = oracle.Stream(cfg, nodes)
    assert not st.add_lastdsp(graph.master())
    st.del_lastdsp()
    st.del_lastdsp()                                 # the Master alone stays
    out, _ = st.process(raw[:100 * 4], 100)
    assert not out.any()                             # Master reads A: cleared, never written again
