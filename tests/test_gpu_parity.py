"""GPU parity: libicw.so (hand-written gfx950 kernels) against the C restatement oracle on the
same seeded inputs.  Everything is bit-exact: the pre-render (Hilbert / modulator) doubles and
the rendered integers.  The north star allows 1e-6 relative on the float stages; the Shift / PM
factors use glibc's own sin / cos algorithm on the device (icw_libm.h), so no tolerance is
needed anywhere."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

pytestmark = pytest.mark.gpu



@pytest.fixture(autouse=True, params=["plain", "row"])
def k1_mode(request, monkeypatch):
    """run every case through both shipped forms of the two serial kernels: lane per chain / per
    render channel (large batches: K1, K3b) and the 16-lane row broadcast (small batches: K1r, K3r;
    K1r takes Kahan + reject only, other modes fall back to the lane-per-chain kernel)"""
    monkeypatch.setenv("ICW_K1_MODE", request.param)
    monkeypatch.setenv("ICW_RENDER", "serial" if request.param == "plain" else "row")
    return request.param


def run_both(oracle, icw, cfg, nodes, raw, n_frames, blocks=None):
    ctx = icw.Context(cfg, nodes, raw.shape[0])
    if blocks is None:
        out, pre = ctx.process(raw, n_frames, want_pre=True)
    else:
        outs, pres = [], []
        fsz = ctx.fsz
        t = 0
        for b in blocks:
            o, p = ctx.process(np.ascontiguousarray(raw[:, t * fsz:(t + b) * fsz]), b, want_pre=True)
            outs.append(o)
            pres.append(p)
            t += b
        out, pre = np.concatenate(outs, axis=1), np.concatenate(pres, axis=1)
    ref_out, ref_pre = oracle.process_streams(cfg, nodes, raw, n_frames, want_pre=True)
    return ctx, out, pre, ref_out, ref_pre


def assert_parity(out, pre, ref_out, ref_pre, rs=2, exact_pre=True):
    """bit-exact pre-render doubles and rendered bytes (exact_pre / rs kept for the callers)"""
    bad = np.flatnonzero(pre.view(np.uint64) != ref_pre.view(np.uint64))
    assert bad.size == 0, f"{bad.size} pre-render doubles differ, first at {bad[:5]}"
    assert np.array_equal(out, ref_out)


def test_master_only_bit_exact(oracle, icw):
    cfg = graph.default_config(48000)
    raw = synth.batch_pcm(8, 4000, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 4000)
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


def test_hilbert_I_channel_bit_exact(oracle, icw):
    cfg = graph.default_config(44100)
    nodes = [graph.master(tout=abi.S_RE, gain=1.0)]
    raw = synth.batch_pcm(4, 3001, 44100)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, nodes, raw, 3001)
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


def test_c2_shape_shift_master(oracle, icw):
    cfg = graph.default_config(48000)
    raw = synth.batch_pcm(16, 6000, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_shift_master(), raw, 6000)
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


def test_c4_shape_pm_shift_mix(oracle, icw):
    cfg = graph.default_config(48000)
    raw = synth.batch_pcm(8, 5000, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_pm_shift_mix(), raw, 5000)
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


@pytest.mark.parametrize("htype", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("kahan,subn", [(1, 1), (0, 1), (1, 0), (0, 0)])
def test_all_filters_modes(oracle, icw, htype, kahan, subn):
    cfg = graph.default_config(48000, hilbert_type=htype)
    cfg.iir_kahan, cfg.iir_subnorm_reject = kahan, subn
    raw = synth.batch_pcm(4, 1500, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 1500)
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


@pytest.mark.parametrize("htype", [1, 2])
def test_speculative_reject_fallback(oracle, icw, htype):
    """The zero-input loops of K1 / K1r run without the reject's select and fall back to exact
    blocks from a failed block's start when some |sum| < 1 (icw_iir.hip, "Speculative blocks").
    Stream 0 falls silent after 2000 frames: its decaying states dip below 1 now and then from
    ~50 000 frames on, so speculation fails in the middle of a launch; stream 1 starts silent
    (every sum rejected) and fails at a launch's first block; streams 2-5 stay speculative in the
    same waves.  Orders 19 (pairs of blocks) and 18 (one zero parity per block)."""
    cfg = graph.default_config(48000, hilbert_type=htype)
    T = 64000
    raw = synth.batch_pcm(6, T, 48000)
    x = raw.view(np.int16).reshape(6, T, 2)
    x[0, 2000:] = 0
    x[1, :3000] = 0
    x[4, 30000:30500] = 0
    ctx, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, T)
    assert_parity(out, pre, ro, rp)
    sts = [oracle.Stream(cfg, graph.graph_master_only()) for _ in range(2)]
    for s in range(2):
        sts[s].process(raw[s], T, want_pre=False)
        r = sts[s].meters()
        assert r["desubnorm"] > (2 if s == 0 else 3000)      # the fallback did run
        assert ctx.meters(s)["desubnorm"] == r["desubnorm"], s


@pytest.mark.parametrize("htype", [0, 1, 2, 4])
def test_block_split_invariance(oracle, icw, htype):
    """state carried across blocks of odd sizes == one pass (and == oracle); orders 15 / 19 / 18 /
    20, block lengths around the zero-input path's 3N minimum, both start parities"""
    cfg = graph.default_config(48000, hilbert_type=htype)
    raw = synth.batch_pcm(4, 5000, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 5000,
                                   blocks=[576, 1, 18, 19, 20, 44, 45, 54, 57, 60, 61, 2000, 2045])
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


@pytest.mark.parametrize("htype", [1, 2])
def test_launch_blocks_inside_one_call(oracle, icw, htype, monkeypatch):
    """one call cut into many 263-frame launch blocks (ICW_BLOCK): every K1 launch starts at a block
    offset t0 of either parity and reads the call-start phases"""
    monkeypatch.setenv("ICW_BLOCK", "263")
    cfg = graph.default_config(48000, hilbert_type=htype)
    raw = synth.batch_pcm(6, 3001, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 3001)
    assert_parity(out, pre, ro, rp, 2, exact_pre=True)


@pytest.mark.parametrize("graph_name", ["shift_master", "pm_shift_mix"])
def test_block_schedule_first_and_tail(oracle, icw, graph_name, monkeypatch):
    """a long call's launch blocks: a short first block, full blocks, then a geometric tail of
    shrinking blocks (plan_blocks in icw_host.cpp), here 640 | 2048 x k | 1728, 1408, ..., 128 --
    every block offset and size reaches K0 / K1 / K2 / the rotation table like a uniform block"""
    monkeypatch.setenv("ICW_BLOCK", "2048")
    monkeypatch.setenv("ICW_FIRST_BLOCK", "640")
    monkeypatch.setenv("ICW_TAPER", "0.85")
    monkeypatch.setenv("ICW_TAPER_MIN", "128")
    cfg = graph.default_config(48000)
    nodes = getattr(graph, "graph_" + graph_name)()
    raw = synth.batch_pcm(6, 20011, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, nodes, raw, 20011)
    assert_parity(out, pre, ro, rp)


@pytest.mark.parametrize("fmt", [abi.FMT_U8, abi.FMT_I16, abi.FMT_I24, abi.FMT_I32, abi.FMT_F32])
@pytest.mark.parametrize("ch", [1, 2])
def test_input_formats(oracle, icw, fmt, ch):
    cfg = graph.default_config(44100, fmt=fmt, channels=ch, need24bits=True)
    raw = synth.batch_pcm(3, 2000, 44100, channels=ch, fmt=fmt)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 2000)
    assert_parity(out, pre, ro, rp, 3, exact_pre=True)


@pytest.mark.parametrize("rtype", [abi.RENDER_ROUND, abi.RENDER_RPDF, abi.RENDER_TPDF, abi.RENDER_STPDF,
                                   abi.RENDER_GAUSS])
@pytest.mark.parametrize("quantz", [abi.QUANTZ_MID_TREAD, abi.QUANTZ_MID_RISER])
@pytest.mark.parametrize("is24", [False, True])
def test_render_matrix(oracle, icw, rtype, quantz, is24):
    """sound_render_value: every render type x quantiser x 16/24 bit, flat and F-weighted shaper"""
    for ns in (abi.NSHAPE_FLAT, abi.NSHAPE_FW44):
        cfg = graph.default_config(44100, need24bits=is24)
        cfg.render.render_type, cfg.render.quantz_type, cfg.render.nshape_type = rtype, quantz, ns
        cfg.render.dth_bits = 1.5
        raw = synth.batch_pcm(3, 1500, 44100)
        ctx, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 1500,
                                         blocks=[700, 800])
        assert_parity(out, pre, ro, rp, 3 if is24 else 2, exact_pre=True)


@pytest.mark.parametrize("ns", list(range(abi.NSHAPE_MAX + 1)))
def test_every_noise_shaper(oracle, icw, ns):
    cfg = graph.default_config(48000, need24bits=(ns % 2 == 1))
    cfg.render.render_type = abi.RENDER_TPDF
    cfg.render.nshape_type = ns
    raw = synth.batch_pcm(2, 1200, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 1200)
    assert_parity(out, pre, ro, rp, 3 if ns % 2 == 1 else 2, exact_pre=True)


@pytest.mark.parametrize("bits", [(16, 2), (16, 11), (24, 18), (24, 5)])
def test_sign_bits_reduction(oracle, icw, bits):
    width, sb = bits
    cfg = graph.default_config(48000, need24bits=(width == 24))
    if width == 24:
        cfg.render.sign_bits24 = sb
    else:
        cfg.render.sign_bits16 = sb
    cfg.render.render_type = abi.RENDER_STPDF
    raw = synth.batch_pcm(2, 1000, 48000)
    _, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 1000)
    assert_parity(out, pre, ro, rp, 3 if width == 24 else 2, exact_pre=True)


def test_c5_shape_tpdf_mew44_24bit(oracle, icw):
    """BASELINE C5: 192 kHz float32 stereo, Hilbert + Master, 24-bit TPDF (1 bit) + MEW44 shaper"""
    cfg = graph.default_config(192000, fmt=abi.FMT_F32, need24bits=True)
    cfg.render.render_type = abi.RENDER_TPDF
    cfg.render.nshape_type = abi.NSHAPE_MEW44
    raw = synth.batch_pcm(4, 3000, 192000, fmt=abi.FMT_F32)
    ctx, out, pre, ro, rp = run_both(oracle, icw, cfg, graph.graph_master_only(), raw, 3000)
    assert_parity(out, pre, ro, rp, 3, exact_pre=True)


def test_meters_match_oracle(oracle, icw):
    cfg = graph.default_config(48000)
    cfg.render.render_type = abi.RENDER_TPDF
    raw = synth.batch_pcm(3, 2000, 48000)
    nodes = [graph.master(gain=2.0)]            # drive into clipping
    ctx = icw.Context(cfg, nodes, 3)
    ctx.process(raw, 2000)
    for s in range(3):
        st = oracle.Stream(cfg, nodes)
        st.process(raw[s], 2000)
        m, r = ctx.meters(s), st.meters()
        assert m["clips"] == r["clips"] and m["desubnorm"] == r["desubnorm"]
        assert m["peak_db"] == r["peak_db"]


def test_mono_dedup_state_and_meters(oracle, icw):
    """mono input on fresh streams: K1 runs the left chains only and writes the right converters'
    state as a copy -- outputs, meters (de-subnorm counts of all four filters) and the state blob
    must equal the full computation's, and a later stereo track must still match the oracle"""
    fs = 48000
    cfg = graph.default_config(fs, channels=1)
    nodes = graph.graph_master_only()
    raw = synth.batch_pcm(5, 3000, fs, channels=1)
    raw[2, :] = 0                                    # digital silence: every w rejected (sncnt)
    ctx = icw.Context(cfg, nodes, 5)
    out, pre = ctx.process(raw, 3000, want_pre=True)
    sts = [oracle.Stream(cfg, nodes) for _ in range(5)]
    for s in range(5):
        ro, rp = sts[s].process(raw[s], 3000, want_pre=True)
        assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), s
        assert np.array_equal(out[s], ro), s
        m, r = ctx.meters(s), sts[s].meters()
        assert m["desubnorm"] == r["desubnorm"] and m["clips"] == r["clips"], s
    # the blob holds identical halves (the copy), so a stereo continuation stays exact
    for s in range(5):
        blob = abi.StateBlob.from_buffer_copy(ctx.get_state(s))
        h = np.ctypeslib.as_array(blob.hist)
        assert np.array_equal(h[0].view(np.uint64), h[2].view(np.uint64))
        assert np.array_equal(h[1].view(np.uint64), h[3].view(np.uint64))
        assert blob.sncnt[0] == blob.sncnt[2] and blob.sncnt[1] == blob.sncnt[3]
    raw2 = synth.batch_pcm(5, 2000, fs, channels=2, first=9)
    ctx.set_input(fs, abi.FMT_I16, 2)
    out2, pre2 = ctx.process(raw2, 2000, want_pre=True)
    for s in range(5):
        sts[s].set_input(fs, abi.FMT_I16, 2)
        ro, rp = sts[s].process(raw2[s], 2000, want_pre=True)
        assert np.array_equal(pre2[s].view(np.uint64), rp.view(np.uint64)), s
        assert np.array_equal(out2[s], ro), s


def test_trig_table_streams_out_of_step(oracle, icw):
    """the per-frame rotation table serves streams whose frame counter equals stream 0's; a stream
    reset to another counter takes the inline path -- both must match the oracle"""
    fs = 44100
    cfg = graph.default_config(fs)
    nodes = graph.graph_pm_shift_mix()
    ctx = icw.Context(cfg, nodes, 4)
    sts = [oracle.Stream(cfg, nodes) for _ in range(4)]
    raw = synth.batch_pcm(4, 1700, fs)
    ctx.process(raw, 1700)
    for s in range(4):
        sts[s].process(raw[s], 1700)
    # stream 2 restarts its modulator counter (a track change with is_clr_nframe_trk)
    ctx.stream_open(2, 1 << 40, clr_nframe=1)
    sts[2].open(1 << 40, clr_nframe=1)
    raw2 = synth.batch_pcm(4, 2500, fs, first=4)
    out, pre = ctx.process(raw2, 2500, want_pre=True)
    for s in range(4):
        ro, rp = sts[s].process(raw2[s], 2500, want_pre=True)
        assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), s
        assert np.array_equal(out[s], ro), s


def test_zero_input_fast_path_mixed_phases(oracle, icw):
    """K1's zero-input fast path needs one phase parity per wave: after an odd-length block and a
    Hilbert reset of one stream, a wave mixes parities (generic path) while other waves do not --
    every stream must still match the oracle bit for bit (Master only: exact pre-render)"""
    fs = 48000
    cfg = graph.default_config(fs)
    nodes = graph.graph_master_only()
    S = 40                                              # two 32-stream lane groups, one partial
    ctx = icw.Context(cfg, nodes, S)
    sts = [oracle.Stream(cfg, nodes) for _ in range(S)]
    raw = synth.batch_pcm(S, 1001, fs)
    ctx.process(raw, 1001)
    for s in range(S):
        sts[s].process(raw[s], 1001)
    for s in (1, 35):                                   # phase 0 among streams at phase 1001 & 3
        ctx.stream_open(s, 1 << 40, clr_hilb=1)
        sts[s].open(1 << 40, clr_hilb=1)
    raw2 = synth.batch_pcm(S, 3000, fs, first=S)
    out, pre = ctx.process(raw2, 3000, want_pre=True)
    for s in range(S):
        ro, rp = sts[s].process(raw2[s], 3000, want_pre=True)
        assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), s
        assert np.array_equal(out[s], ro), s


@pytest.mark.parametrize("streams,ch", [(4096, 1), (2048, 2)])
def test_large_batch_sampled_against_oracle(oracle, icw, streams, ch):
    """BASELINE C3 / C4 shard sizes (4096 mono, 2048 stereo streams per GPU) on a short run: many
    lane groups, the mono dedup, several CU-partitioned K1 workgroups.  A sample of streams from
    the start, the middle, the last lane group and the very end is checked bit for bit."""
    fs = 96000 if ch == 1 else 48000
    cfg = graph.default_config(fs, channels=ch)
    nodes = graph.graph_master_only() if ch == 1 else graph.graph_shift_master()
    n = 1200
    gen = synth.batch_pcm(8, n, fs, channels=ch)          # 8 generated streams tiled over the batch
    raw = np.ascontiguousarray(np.tile(gen, (streams // 8, 1)))
    ctx = icw.Context(cfg, nodes, streams)
    out, pre = ctx.process(raw, n, want_pre=True)
    for s in (0, 1, 7, streams // 2 + 3, streams - 33, streams - 1):
        st = oracle.Stream(cfg, nodes)
        ro, rp = st.process(raw[s], n, want_pre=True)
        assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), s
        assert np.array_equal(out[s], ro), s
    # streams built from the same generated row produce the same bytes
    assert np.array_equal(out[3], out[3 + 8 * (streams // 16)])


def test_meters_reset_order_matches_reference(oracle, icw):
    """amod_get_clips_peaks (adv_modulator.c:445-465) clears the clips and peaks first and returns
    the cleared values; the de-subnorm count is not touched (in_cwave.c:300-310)"""
    cfg = graph.default_config(48000)
    nodes = [graph.master(inputs=("A",), gain=2.0), graph.mix(inputs=("in",), out="A", gain=2.0)]  # x4: clips
    raw = synth.batch_pcm(2, 3000, 48000)
    ctx = icw.Context(cfg, nodes, 2)
    ctx.process(np.ascontiguousarray(raw[:, :1500 * 4]), 1500)
    before = ctx.meters(0)
    assert before["clips"][0] > 0
    m = ctx.meters(0, reset=True)
    assert m["clips"] == (0, 0)
    assert m["peak_db"] == (abi.SR_ZERO_SIGNAL_DB, abi.SR_ZERO_SIGNAL_DB)
    assert m["desubnorm"] == before["desubnorm"]
    ctx.process(np.ascontiguousarray(raw[:, 1500 * 4:]), 1500)
    full, half = oracle.Stream(cfg, nodes), oracle.Stream(cfg, nodes)
    full.process(raw[0], 3000)
    half.process(raw[0], 1500)
    # clip counts are additive: after the reset they count the second half only
    want = tuple(f - h for f, h in zip(full.meters()["clips"], half.meters()["clips"]))
    after = ctx.meters(0)
    assert after["clips"] == want
    assert after["peak_db"][0] <= full.meters()["peak_db"][0]
    other = oracle.Stream(cfg, nodes)                   # the other stream is untouched by the reset
    other.process(raw[1], 3000)
    assert ctx.meters(1)["clips"] == other.meters()["clips"]


def test_meters_and_output_after_device_call_without_sync(oracle, icw):
    """ICW_F_DEVICE_PTRS with a NULL stream handle (torch's default stream): the call returns while
    the kernels run; icw_get_meters must wait for them, and torch's default stream must see the
    finished output (the call is ordered on the legacy default stream)"""
    import torch
    fs, S, T = 48000, 3, 65536
    cfg = graph.default_config(fs)
    cfg.render.render_type = abi.RENDER_TPDF
    nodes = [graph.master(inputs=("A",), gain=1.9), graph.shift(inputs=("in",), out="A")]
    raw = synth.batch_pcm(S, T, fs)
    ctx = icw.Context(cfg, nodes, S)
    d_in = torch.from_numpy(raw).cuda()
    d_out = torch.zeros((S, T * 4), dtype=torch.uint8, device="cuda")
    ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T)
    meters = [ctx.meters(s) for s in range(S)]          # no synchronize in between
    out = d_out.cpu().numpy()                            # torch's default stream
    for s in range(S):
        st = oracle.Stream(cfg, nodes)
        ro, _ = st.process(raw[s], T)
        assert np.array_equal(out[s], ro), s
        r = st.meters()
        assert meters[s]["clips"] == r["clips"] and meters[s]["peak_db"] == r["peak_db"], s
        assert meters[s]["desubnorm"] == r["desubnorm"], s


@pytest.mark.parametrize("ns", [abi.NSHAPE_FLAT, abi.NSHAPE_FW44, abi.NSHAPE_MEW44, 9, abi.NSHAPE_MAX])
def test_serial_render_short_and_ragged_calls(oracle, icw, ns):
    """the serial renders over calls shorter than one, two and three 20-sample blocks and around
    their multiples -- K3r stages a block's inputs in LDS two blocks ahead (its prologue reads past a
    short call's end, its last block is partial) and rotates the shaper ring by the remainder; three
    streams leave two spare rows in the second K3r wave; the state carries across the calls"""
    cfg = graph.default_config(48000, need24bits=(ns % 2 == 1))
    cfg.render.render_type = abi.RENDER_TPDF
    cfg.render.nshape_type = ns
    nodes = graph.graph_master_only()
    lens = [1, 7, 19, 20, 21, 39, 40, 41, 59, 61, 100]
    S = 3
    raw = synth.batch_pcm(S, sum(lens), 48000, first=31)
    ctx = icw.Context(cfg, nodes, S)
    refs = [oracle.Stream(cfg, nodes) for _ in range(S)]
    t = 0
    for n in lens:
        seg = np.ascontiguousarray(raw[:, t * 4:(t + n) * 4])
        out, pre = ctx.process(seg, n, want_pre=True)
        for s, st in enumerate(refs):
            ro, rp = st.process(seg[s], n, want_pre=True)
            assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), (n, s)
            assert np.array_equal(out[s], ro), (n, s)
        t += n
    for s, st in enumerate(refs):
        assert ctx.meters(s) == st.meters(), s
    ctx.close()
