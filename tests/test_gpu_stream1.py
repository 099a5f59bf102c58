"""GPU parity of K5 `icw_stream1`: a one-stream call of one launch block (the drop-in's 576-frame
calls, playback.c:619, NS_PERTIME in_cwave.h:133) runs K0, K1r, K2 and icw_advance as phases of
one workgroup.  Its results must be the four-kernel pipeline's and the oracle's bit for bit: every
filter order, the mono dedup, every register-form graph kind, block lengths from 1 frame to the
fused limit (ICW_S1_MAX = 4096) and past it, and state carried across calls of mixed forms."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth
from tests.graphgen import random_list

pytestmark = pytest.mark.gpu


def calls(oracle, icw, cfg, nodes, lens, monkeypatch, fused, first=5):
    monkeypatch.setenv("ICW_STREAM1", "1" if fused else "0")
    monkeypatch.setenv("ICW_K1_MODE", "row")
    ctx = icw.Context(cfg, nodes, 1)
    ref = oracle.Stream(cfg, nodes)
    fsz = ctx.fsz
    raw = synth.batch_pcm(1, sum(lens), cfg.sample_rate, channels=cfg.in_channels, fmt=cfg.in_format,
                          first=first)
    t, outs = 0, []
    for n in lens:
        seg = np.ascontiguousarray(raw[:, t * fsz:(t + n) * fsz])
        out, pre = ctx.process(seg, n, want_pre=True)
        ro, rp = ref.process(seg[0], n, want_pre=True)
        bad = np.flatnonzero(pre[0].view(np.uint64) != rp.view(np.uint64))
        assert bad.size == 0, (n, t, bad[:5])
        assert np.array_equal(out[0], ro), (n, t)
        outs.append(out[0])
        t += n
    m, r = ctx.meters(0), ref.meters()
    assert m == r, (m, r)
    assert ctx.n_frame(0) == ref.n_frame()
    ctx.close()
    return np.concatenate(outs)


@pytest.mark.parametrize("htype", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("ch", [1, 2])
def test_stream1_filters_and_dedup(oracle, icw, htype, ch, monkeypatch):
    cfg = graph.default_config(44100, channels=ch, hilbert_type=htype)
    lens = [576] * 5 + [1, 18, 19, 57, 700]
    calls(oracle, icw, cfg, graph.graph_shift_master(), lens, monkeypatch, True)


@pytest.mark.parametrize("seed", range(8))
def test_stream1_random_lists(oracle, icw, seed, monkeypatch):
    rng = np.random.default_rng(4000 + seed)
    cfg = graph.default_config(48000)
    nodes = random_list(rng)
    calls(oracle, icw, cfg, nodes, [576, 576, 1152, 4096, 4097, 576], monkeypatch, True, first=seed)


def test_stream1_equals_pipeline(oracle, icw, monkeypatch):
    """the fused kernel and the four-kernel pipeline give the same bytes, call by call"""
    cfg = graph.default_config(44100)
    nodes = graph.graph_pm_shift_mix()
    lens = [576] * 8 + [3000, 2, 576]
    a = calls(oracle, icw, cfg, nodes, lens, monkeypatch, True)
    b = calls(oracle, icw, cfg, nodes, lens, monkeypatch, False)
    assert np.array_equal(a, b)


def test_stream1_drop_in_boundary(oracle, icw):
    """icw_amod_process_samples (the C drop-in) in 576-frame blocks with a track open: fades, the
    pinned zero-copy staging, the error flag copied by the fused kernel's advance phase"""
    import ctypes as C
    lib = icw.load()
    fs = 44100
    cfg = graph.default_config(fs)
    nodes = graph.graph_shift_master()
    arr = graph.node_array(nodes)
    st = C.c_int()
    mc = lib.icw_mod_context_create(C.byref(cfg), arr, len(nodes), 0, C.byref(st))
    assert mc and st.value == abi.OK
    n = 576 * 20
    assert lib.icw_mod_context_fopen(mc, fs, abi.FMT_I16, 2, n, 20, 30, 0, 0, 0, cfg.need24bits) == abi.OK
    ref = oracle.Stream(cfg, nodes)
    ref.open(n, 20, 30)
    raw = synth.batch_pcm(1, n, fs, first=77)[0]
    osz = lib.icw_mod_context_out_size(mc)
    for b in range(20):
        blk = np.ascontiguousarray(raw[b * 576 * 4:(b + 1) * 576 * 4])
        buf = np.zeros(576 * osz, np.uint8)
        assert lib.icw_amod_process_samples(buf.ctypes.data, mc, blk.ctypes.data, 576) == 576
        ro, _ = ref.process(blk, 576)
        assert np.array_equal(buf, ro), b
    lib.icw_mod_context_destroy(mc)


@pytest.mark.parametrize("fmt,ch,b24", [(abi.FMT_I24, 1, True), (abi.FMT_I16, 2, False), (abi.FMT_U8, 1, False)])
@pytest.mark.parametrize("spin", ["1", "0"])
def test_stream1_polled_completion(oracle, icw, fmt, ch, b24, spin, monkeypatch):
    """zero-copy calls (no pre-render doubles requested): the host polls for the sequence number K5
    stores after the output and the error flag (ICW_SPIN=0: a stream wait instead).  Odd block
    lengths and frame sizes put the word at every offset of the staging buffer"""
    monkeypatch.setenv("ICW_SPIN", spin)
    monkeypatch.setenv("ICW_STREAM1", "1")
    monkeypatch.setenv("ICW_K1_MODE", "row")
    cfg = graph.default_config(44100, fmt=fmt, channels=ch, need24bits=b24)
    nodes = graph.graph_shift_master()
    ctx = icw.Context(cfg, nodes, 1)
    ref = oracle.Stream(cfg, nodes)
    lens = [576, 1, 3, 577, 2, 4096, 575, 576, 576]
    raw = synth.batch_pcm(1, sum(lens), cfg.sample_rate, channels=ch, fmt=fmt, first=11)
    t = 0
    for n in lens:
        seg = np.ascontiguousarray(raw[:, t * ctx.fsz:(t + n) * ctx.fsz])
        out, _ = ctx.process(seg, n)
        ro, _ = ref.process(seg[0], n)
        assert np.array_equal(out[0], ro), (n, t)
        t += n
    assert ctx.n_frame(0) == ref.n_frame()
    ctx.close()


def test_stream1_stale_completion_word(oracle, icw, monkeypatch):
    """the completion word lives in the reused staging buffer.  A ramp input (frame n =
    (L = n, R = 0): the little-endian word n) in two 4000-frame calls (sequence numbers 1, 2) leaves
    word 3 at byte 12, where a 1-frame call (number 3: 4 B in, 4 B out, the word at 8 + 4) polls.  The
    host stores a value that cannot match before the launch, so the call returns the kernel's output,
    not the stale bytes."""
    monkeypatch.setenv("ICW_SPIN", "1")
    monkeypatch.setenv("ICW_STREAM1", "1")
    monkeypatch.setenv("ICW_K1_MODE", "row")
    cfg = graph.default_config(44100)
    nodes = graph.graph_shift_master()
    ctx = icw.Context(cfg, nodes, 1)
    ref = oracle.Stream(cfg, nodes)
    ramp = np.zeros((1, 4000, 2), np.int16)
    ramp[0, :, 0] = np.arange(4000)
    ramp = ramp.view(np.uint8).reshape(1, -1)
    for n, seg in ((4000, ramp), (4000, ramp), (1, ramp[:, :4]), (2, ramp[:, 8:16]), (1, ramp[:, 4:8])):
        out, _ = ctx.process(np.ascontiguousarray(seg), n)
        ro, _ = ref.process(np.ascontiguousarray(seg[0]), n)
        assert np.array_equal(out[0], ro), n
    assert ctx.n_frame(0) == ref.n_frame()
    ctx.close()


@pytest.mark.parametrize("ovl", ["1", "0"])
@pytest.mark.parametrize("kind", ["shift_master", "pm_shift_mix", "long_chain", "random"])
@pytest.mark.parametrize("ch", [1, 2])
def test_stream1_overlapped_output_phase(oracle, icw, ovl, kind, ch, monkeypatch):
    """K5's output phase beside the recurrence (ICW_S1_OVL=1, the default: the w rows in LDS, the
    output waves polling the recurrence's published frame count) and after it (ICW_S1_OVL=0): both
    the oracle's bytes, for block lengths around the 64-frame groups and the recurrence's blocks,
    register-file and chain programs, stereo and mono (dedup)"""
    monkeypatch.setenv("ICW_S1_OVL", ovl)
    cfg = graph.default_config(48000, channels=ch)
    if kind == "random":
        nodes = random_list(np.random.default_rng(77))
    else:
        nodes = {"shift_master": graph.graph_shift_master, "pm_shift_mix": graph.graph_pm_shift_mix,
                 "long_chain": graph.graph_long_chain}[kind]()
    lens = [576, 1, 19, 38, 63, 64, 65, 128, 129, 2048, 2500, 576]
    calls(oracle, icw, cfg, nodes, lens, monkeypatch, True)


def test_prepare_leaves_fresh_state(oracle, icw):
    """icw_prepare (the drop-in's warm-up, called by icw_mod_context_create): one call of silence, then
    the fresh state back -- the first real call equals the oracle's from a fresh stream, meters and
    frame counter included; a second icw_prepare, after a call, is refused"""
    cfg = graph.default_config(44100)
    nodes = graph.graph_pm_shift_mix()
    ctx = icw.Context(cfg, nodes, 1)
    ctx.prepare(576)
    ref = oracle.Stream(cfg, nodes)
    raw = synth.batch_pcm(1, 576 * 3, 44100, first=21)
    for b in range(3):
        seg = np.ascontiguousarray(raw[:, b * 576 * 4:(b + 1) * 576 * 4])
        out, _ = ctx.process(seg, 576)
        ro, _ = ref.process(seg[0], 576)
        assert np.array_equal(out[0], ro), b
    assert ctx.meters(0) == ref.meters() and ctx.n_frame(0) == ref.n_frame()
    with pytest.raises(icw.IcwError):
        ctx.prepare(576)
    ctx.close()
