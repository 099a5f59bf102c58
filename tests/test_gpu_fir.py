"""GPU parity of the FIR Hilbert converter (icw_set_fir_hilbert: kernel KF2 `icw_fir_graph`, or KF
`icw_fir_hilbert` + K2)
against the oracle's restatement (oracle/icw_oracle.c fir_process): pre-render doubles and
rendered bytes bit for bit.

The converter is the one CWAVE headers name (cwave.h:40,56-58, k_M / k_beta); in_cwave does not
ship it, so the oracle is pinned only by the design's definition (tests/test_fir.py: scipy's
Kaiser window, numpy convolution, the analytic-signal property) -- parity unpinned against any
reference output.  After the converter the block runs the CWAVE path (graph, render), which
tests/test_gpu_cwave_graph.py checks against the reference restatement.
"""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu

BETA = 8.0


@pytest.fixture(autouse=True, params=["fused", "split"])
def fir_form(request, monkeypatch):
    """KF2 (converter, graph and render in one kernel) and KF + K2 (ICW_FIR_FUSED=0)"""
    monkeypatch.setenv("ICW_FIR_FUSED", "1" if request.param == "fused" else "0")
    return request.param


def run_fir(oracle, icw, cfg, nodes, raw, n_frames, order, beta=BETA, blocks=None):
    ctx = icw.Context(cfg, nodes, raw.shape[0])
    ctx.set_fir_hilbert(order, beta)
    if blocks is None:
        out, pre = ctx.process(raw, n_frames, want_pre=True)
    else:
        outs, pres, t = [], [], 0
        for b in blocks:
            o, p = ctx.process(np.ascontiguousarray(raw[:, t * ctx.fsz:(t + b) * ctx.fsz]), b, want_pre=True)
            outs.append(o)
            pres.append(p)
            t += b
        out, pre = np.concatenate(outs, axis=1), np.concatenate(pres, axis=1)
    ref_out, ref_pre = oracle.process_streams(cfg, nodes, raw, n_frames, want_pre=True, fir=(order, beta))
    return ctx, out, pre, ref_out, ref_pre


@pytest.mark.parametrize("order", [2, 30, 254, 510, 1022])
@pytest.mark.parametrize("fmt,ch", [(abi.FMT_I16, 2), (abi.FMT_F32, 2), (abi.FMT_U8, 1), (abi.FMT_I24, 2),
                                    (abi.FMT_I32, 1)])
def test_fir_formats_shift_master(oracle, icw, order, fmt, ch):
    cfg = graph.default_config(48000, fmt=fmt, channels=ch)
    raw = synth.batch_pcm(3, 3000, 48000, channels=ch, fmt=fmt)
    ctx, out, pre, ro, rp = run_fir(oracle, icw, cfg, graph.graph_shift_master(), raw, 3000, order)
    assert_parity(out, pre, ro, rp)
    ctx.close()


@pytest.mark.parametrize("order", [30, 254, 1022])
def test_fir_launch_blocks_and_calls(oracle, icw, order, monkeypatch):
    """263-frame launch blocks (shorter than the 1022-order history) and ragged calls: the history
    hand-off between blocks and calls is exact"""
    monkeypatch.setenv("ICW_BLOCK", "263")
    cfg = graph.default_config(44100)
    raw = synth.batch_pcm(4, 5000, 44100)
    ctx, out, pre, ro, rp = run_fir(oracle, icw, cfg, graph.graph_shift_master(), raw, 5000, order,
                                    blocks=[100, 1, 577, 2322, 2000])
    assert_parity(out, pre, ro, rp)
    ctx.close()


def test_fir_many_tiles_c4_graph(oracle, icw):
    """several 1024-frame tiles per launch block, the PM -> Shift -> Mix -> Master list"""
    cfg = graph.default_config(48000)
    raw = synth.batch_pcm(6, 20000, 48000)
    ctx, out, pre, ro, rp = run_fir(oracle, icw, cfg, graph.graph_pm_shift_mix(), raw, 20000, 254)
    assert_parity(out, pre, ro, rp)
    ctx.close()


@pytest.mark.parametrize("order", [254, 1022])
def test_fir_dithered_noise_shaped_24bit(oracle, icw, order):
    """the C5 render (24-bit TPDF + MEW44) after the converter: serial render path"""
    cfg = graph.default_config(192000, fmt=abi.FMT_F32, need24bits=True)
    cfg.render.render_type = abi.RENDER_TPDF
    cfg.render.nshape_type = abi.NSHAPE_MEW44
    raw = synth.batch_pcm(3, 6000, 192000, fmt=abi.FMT_F32)
    ctx, out, pre, ro, rp = run_fir(oracle, icw, cfg, graph.graph_master_only(), raw, 6000, order)
    assert_parity(out, pre, ro, rp)
    ctx.close()


def test_fir_bus_form_graph(oracle, icw):
    cfg = graph.default_config(48000)
    raw = synth.batch_pcm(3, 3000, 48000)
    ctx, out, pre, ro, rp = run_fir(oracle, icw, cfg, graph.graph_feedback_pm_shift(), raw, 3000, 30)
    assert_parity(out, pre, ro, rp)
    ctx.close()


def test_fir_fades(oracle, icw):
    cfg = graph.default_config(48000)
    n = 30000
    raw = synth.batch_pcm(2, n, 48000)
    nodes = graph.graph_shift_master()
    ctx = icw.Context(cfg, nodes, 2)
    ctx.set_fir_hilbert(254, BETA)
    for s in range(2):
        ctx.stream_open(s, n, fade_in_ms=100, fade_out_ms=200)
    out, pre = ctx.process(raw, n, want_pre=True)
    for s in range(2):
        st = oracle.Stream(cfg, nodes)
        st.set_fir(254, BETA)
        st.open(n, 100, 200)
        ro, rp = st.process(raw[s], n, want_pre=True)
        assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64))
        assert np.array_equal(out[s], ro)
    ctx.close()


def test_fir_mono_then_stereo_track(oracle, icw):
    """a mono track then a stereo one without clearing the converter: R's history follows L's"""
    cfg = graph.default_config(48000, channels=1)
    nodes = graph.graph_shift_master()
    mono = synth.batch_pcm(2, 1500, 48000, channels=1)
    stereo = synth.batch_pcm(2, 1500, 48000, channels=2, first=7)
    ctx = icw.Context(cfg, nodes, 2)
    ctx.set_fir_hilbert(254, BETA)
    o1, p1 = ctx.process(mono, 1500, want_pre=True)
    ctx.set_input(48000, abi.FMT_I16, 2)
    o2, p2 = ctx.process(stereo, 1500, want_pre=True)
    for s in range(2):
        st = oracle.Stream(cfg, nodes)
        st.set_fir(254, BETA)
        r1, q1 = st.process(mono[s], 1500, want_pre=True)
        st.set_input(48000, abi.FMT_I16, 2)
        r2, q2 = st.process(stereo[s], 1500, want_pre=True)
        assert np.array_equal(p1[s].view(np.uint64), q1.view(np.uint64))
        assert np.array_equal(p2[s].view(np.uint64), q2.view(np.uint64))
        assert np.array_equal(o2[s], r2)
    ctx.close()


def test_fir_state_roundtrip(oracle, icw):
    """checkpoint after 2500 frames (the FIR history travels in the state blob), resume in a new
    context: the continuation equals an uninterrupted run"""
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    raw = synth.batch_pcm(2, 5000, 48000)
    full = icw.Context(cfg, nodes, 2)
    full.set_fir_hilbert(510, BETA)
    ref, refp = full.process(raw, 5000, want_pre=True)
    a = icw.Context(cfg, nodes, 2)
    a.set_fir_hilbert(510, BETA)
    a.process(np.ascontiguousarray(raw[:, :2500 * 4]), 2500)
    blobs = [a.get_state(s) for s in range(2)]
    b = icw.Context(cfg, nodes, 2)
    b.set_fir_hilbert(510, BETA)
    for s in range(2):
        b.set_state(s, blobs[s])
    for s in range(2):
        assert b.n_frame(s) == a.n_frame(s) == 2500      # set_state moves the host mirror too
    out, pre = b.process(np.ascontiguousarray(raw[:, 2500 * 4:]), 2500, want_pre=True)
    assert np.array_equal(pre.view(np.uint64), refp[:, 2500:].view(np.uint64))
    assert np.array_equal(out, ref[:, 2500 * 4:])
    for c in (full, a, b):
        c.close()


def test_fir_off_restores_quadrature_iir(oracle, icw):
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    raw = synth.batch_pcm(3, 2000, 48000)
    ctx = icw.Context(cfg, nodes, 3)
    ctx.set_fir_hilbert(254, BETA)
    ctx.set_fir_hilbert(0, 0.0)
    out, pre = ctx.process(raw, 2000, want_pre=True)
    ro, rp = oracle.process_streams(cfg, nodes, raw, 2000, want_pre=True)
    assert_parity(out, pre, ro, rp)
    ctx.close()


def test_fir_pinned_host_buffers_many_blocks(oracle, icw):
    """pinned host in / out buffers (icw_host_alloc) on a call of several launch blocks: each block's
    input slice goes H2D on the copy stream before the block's converter reads it (KF or the fused
    KF2), and three blocks leave the history in the second buffer, which the call copies back"""
    from in_cwave_amd import lib as L
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    n = 3 * 65536 - 1000
    raw = synth.batch_pcm(2, n, 48000)
    ctx = icw.Context(cfg, nodes, 2)
    ctx.set_fir_hilbert(254, BETA)
    h_in = L.host_array(raw.shape)
    h_in[:] = raw
    h_out = L.host_array((2, n * 4))
    for call in range(2):          # the second call starts from the history the first one left
        seg = raw if call == 0 else np.ascontiguousarray(raw[:, ::-1])
        h_in[:] = seg
        ctx.process(h_in, n, out=h_out)
        if call == 0:
            ro, _ = oracle.process_streams(cfg, nodes, seg, n, fir=(254, BETA))
            assert np.array_equal(np.asarray(h_out), ro)
    refs = [oracle.Stream(cfg, nodes) for _ in range(2)]
    for s, st in enumerate(refs):
        st.set_fir(254, BETA)
        st.process(raw[s], n)
        r2, _ = st.process(np.ascontiguousarray(raw[s, ::-1]), n)
        assert np.array_equal(np.asarray(h_out)[s], r2), s
    ctx.close()


def test_fir_subset_calls_keep_other_streams_history(oracle, icw, monkeypatch):
    """icw_process_streams on subsets with odd and even block counts: every stream's history stays
    its own (a subset call must not move the other streams' current history buffer)"""
    monkeypatch.setenv("ICW_BLOCK", "4096")
    cfg = graph.default_config(48000)
    nodes = graph.graph_pm_shift_mix()
    S = 3
    calls = [(0, 1, 3000), (0, 3, 2500), (1, 2, 9000), (0, 3, 4100), (2, 1, 5000), (0, 3, 700)]
    total = [0] * S
    for f, cnt, n in calls:
        for s in range(f, f + cnt):
            total[s] += n
    raw = synth.batch_pcm(S, max(total), 48000, first=900)
    ctx = icw.Context(cfg, nodes, S)
    ctx.set_fir_hilbert(510, BETA)
    refs = [oracle.Stream(cfg, nodes) for _ in range(S)]
    for st in refs:
        st.set_fir(510, BETA)
    pos = [0] * S
    for k, (f, cnt, n) in enumerate(calls):
        seg = np.stack([raw[s, pos[s] * 4:(pos[s] + n) * 4] for s in range(f, f + cnt)])
        out, pre = ctx.process(seg, n, first=f, count=cnt, want_pre=True)
        for i, s in enumerate(range(f, f + cnt)):
            ro, rp = refs[s].process(seg[i], n, want_pre=True)
            assert np.array_equal(pre[i].view(np.uint64), rp.view(np.uint64)), (k, s)
            assert np.array_equal(out[i], ro), (k, s)
            pos[s] += n
        # the host mirror of the frame counters (in_step) follows every subset call: icw_n_frame
        # fails loudly on a divergence
        for s in range(S):
            assert ctx.n_frame(s) == refs[s].n_frame(), (k, s)
    ctx.close()


def test_fir_state_blob_records_order(icw):
    """the blob carries the FIR order in force; a blob of another order (or of the IIR) is refused"""
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    a = icw.Context(cfg, nodes, 1)
    a.set_fir_hilbert(254, BETA)
    assert icw.load().icw_state_size(a.h) == C_sizeof_blob() + 2 * 254 * 8
    blob = a.get_state(0)
    assert abi.StateBlob.from_buffer_copy(blob).fir_M == 254
    b = icw.Context(cfg, nodes, 1)
    b.set_fir_hilbert(510, BETA)
    big = blob + bytes(2 * 256 * 8)
    with pytest.raises(Exception):
        b.set_state(0, big)
    b.set_fir_hilbert(0, 0.0)
    with pytest.raises(Exception):
        b.set_state(0, blob)
    for c in (a, b):
        c.close()


def C_sizeof_blob():
    import ctypes
    return ctypes.sizeof(abi.StateBlob)


@pytest.mark.parametrize("ch", [1, 2])
@pytest.mark.parametrize("b24", [False, True])
@pytest.mark.parametrize("nodes", ["shift_master", "pm_shift_mix", "master"])
def test_fir_chain_frames_round_renders(oracle, icw, ch, b24, nodes):
    """KF2's chain programs op by op over a lane's frames (icw_chain_frames): mono and stereo, 16-
    and 24-bit ROUND output, ragged block ends (the last lane's frames partly past the block: the
    packed stores fall back to per-frame / per-byte stores)"""
    cfg = graph.default_config(48000, fmt=abi.FMT_I16, channels=ch, need24bits=b24)
    nodes = {"shift_master": graph.graph_shift_master, "pm_shift_mix": graph.graph_pm_shift_mix,
             "master": graph.graph_master_only}[nodes]()
    raw = synth.batch_pcm(3, 5003, 48000, channels=ch)
    ctx, out, pre, ro, rp = run_fir(oracle, icw, cfg, nodes, raw, 5003, 254, blocks=[2049, 7, 2947])
    assert_parity(out, pre, ro, rp)
    ctx.close()


def test_fir_long_blocks_device_buffers(oracle, icw):
    """device buffers, nothing after the converter: launch blocks of 2^20 frames (icw_host.cpp
    kMaxFirBlockFrames) -- a call of two blocks (the history hand-off between them in the device's
    double buffer, no copy-back) and then a call of one (odd: copy-back), against the oracle with the
    stream-fastest grid of three streams"""
    import torch
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    S, n1, n2 = 3, (1 << 20) + 3000, 70000
    raw = synth.batch_pcm(S, n1 + n2, 48000, first=41)
    dev = torch.device("cuda", 0)
    ctx = icw.Context(cfg, nodes, S, device=0)
    ctx.set_fir_hilbert(254, BETA)
    osz = 2 * ctx.render_size
    outs = []
    t = 0
    for n in (n1, n2):
        d_in = torch.from_numpy(np.ascontiguousarray(raw[:, t * 4:(t + n) * 4])).to(dev)
        d_out = torch.empty((S, n * osz), dtype=torch.uint8, device=dev)
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), n)
        torch.cuda.synchronize()
        outs.append(d_out.cpu().numpy())
        t += n
    meters = [ctx.meters(s) for s in range(S)]
    ctx.close()
    for s in range(S):
        st = oracle.Stream(cfg, nodes)
        st.set_fir(254, BETA)
        t = 0
        for k, n in enumerate((n1, n2)):
            ro, _ = st.process(raw[s, t * 4:(t + n) * 4], n)
            assert np.array_equal(outs[k][s], ro), (s, k)
            t += n
        m, r = meters[s], st.meters()
        assert tuple(m["clips"]) == tuple(r["clips"]) and tuple(m["peak_db"]) == tuple(r["peak_db"]), s
