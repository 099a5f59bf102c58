"""CPU tests of the oracle (C restatement) against the reference's own fixtures and independent
checks.  These are what pins the oracle before it is trusted as the GPU checker:

  * MT19937: reference known-answer test (mt19937ar_out.c, 1000 values) and the outputs of the
    reference mt_jrnd.c itself, compiled by oracle/Makefile (tests/golden/mt_ref_seeds.npz);
  * coefficient tables: bit patterns extracted from hblpf.c / sound_render.c;
  * IIR: scipy.signal.lfilter (independent implementation of the same difference equation);
    the Kahan form equals lfilter(b, a, x) - b0*x (its d0*x omission, hblpf.c:1026-1043);
  * Hilbert: analytic-signal property of SURVEY 4 (|I+jQ|/A in [0.818, 0.902], positive rotation);
  * render / reader / graph arithmetic: quirks stated in SURVEY 0 (subnorm threshold 1.0,
    MID_RISER range [-32767, 32767], clip counting).
"""
import ctypes as C
import json
import struct
from pathlib import Path

import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

GOLD = Path(__file__).resolve().parent / "golden"


def h2d(h):
    return struct.unpack("<d", bytes.fromhex(h)[::-1])[0]


def test_mt_known_answer(oracle):
    kat = json.loads((GOLD / "mt19937ar_kat.json").read_text())
    mt = oracle.MT(key=kat["init_key"])
    got = [mt.u32() for _ in range(len(kat["u32"]))]
    assert got == kat["u32"]


def test_mt_matches_reference_build_outputs(oracle):
    g = np.load(GOLD / "mt_ref_seeds.npz")
    for name, seed in (("left", abi.SEED_LEFT), ("right", abi.SEED_RIGHT)):
        mt = oracle.MT(seed=seed)
        assert np.array_equal(np.array([mt.u32() for _ in range(2000)], np.uint32), g[f"{name}_u32"])
        mt = oracle.MT(seed=seed)
        assert np.array_equal(np.array([mt.dsemi() for _ in range(2000)]).view(np.uint64),
                              g[f"{name}_dsemi"].view(np.uint64))
        mt = oracle.MT(seed=seed)
        assert np.array_equal(np.array([mt.dsopen() for _ in range(2000)]).view(np.uint64),
                              g[f"{name}_dsopen"].view(np.uint64))


def test_mt_dsemi_equals_numpy_randomstate(oracle):
    """numpy's RandomState(seed).random_sample() is the same 53-bit construction"""
    mt = oracle.MT(seed=abi.SEED_LEFT)
    rs = np.random.RandomState(abi.SEED_LEFT)
    assert np.array_equal(np.array([mt.dsemi() for _ in range(3000)]), rs.random_sample(3000))


@pytest.mark.skipif(not Path("/root/reference/src/mersene_twister/mt_jrnd.c").exists(), reason="reference absent")
def test_reference_kat_binary_passes():
    import subprocess
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "test_mt_jrnd"
    if not exe.exists():
        subprocess.run(["make", "-C", str(exe.parents[1]), "ref"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, check=True)
    assert "EVERYTHING WENT OK" in r.stdout


@pytest.mark.skipif(not Path("/root/reference/src/hblpf.c").exists(), reason="reference absent")
def test_tables_match_reference_text():
    import re
    tb = json.loads((GOLD / "tables.json").read_text())
    src = Path("/root/reference/src/hblpf.c").read_text(errors="replace").split("#else")[0]
    for t, f in enumerate(tb["hb"]):
        for ab, key in (("B", "b"), ("A", "a")):
            body = re.search(rf"IIR_LOEL_TYPE{t}_{ab}\[\]\s*=\s*[^{{]*\{{(.*?)\}};", src, re.S).group(1)
            ref = [h.lower() for h in re.findall(r"0x([0-9A-Fa-f]{16})U", body)]
            assert ref == f[key]


def test_tables_orders_and_a0():
    tb = json.loads((GOLD / "tables.json").read_text())
    assert [f["order"] for f in tb["hb"]] == [15, 19, 18, 19, 20, 20]       # hblpf.c:740-820
    for f in tb["hb"]:
        assert h2d(f["a"][0]) == 1.0                                       # a0 == 1 -> exact copies
    assert [d["n"] for d in tb["ns"]][:3] == [0, 9, 9]


def test_product_and_oracle_tables_identical():
    root = Path(__file__).resolve().parents[1]
    a = (root / "in_cwave_amd/csrc/icw_tables.inc").read_text().replace("icw_", "X_")
    b = (root / "oracle/orc_tables.inc").read_text().replace("orc_", "X_")
    assert a == b


def _ba(t):
    tb = json.loads((GOLD / "tables.json").read_text())
    return (np.array([h2d(x) for x in tb["hb"][t]["b"]]), np.array([h2d(x) for x in tb["hb"][t]["a"]]))


@pytest.mark.parametrize("t,tol", [(0, 1e-7), (1, 2e-3), (2, 2e-3), (3, 5e-3), (4, 2e-2), (5, 2e-2)])
@pytest.mark.parametrize("kahan", [0, 1])
def test_iir_against_scipy_lfilter(oracle, t, tol, kahan):
    from scipy.signal import lfilter
    b, a = _ba(t)
    x = np.random.default_rng(t).standard_normal(6000) * 8000.0
    y, w, cnt = oracle.iir_block(x, t, kahan, 0)
    ref = lfilter(b, a, x)
    if kahan:
        ref = ref - b[0] * x          # the Kahan form omits d0*x (hblpf.c:1026-1043)
    assert np.max(np.abs(y - ref)) / np.max(np.abs(ref)) < tol
    assert cnt == 0


def test_iir_kahan_vs_baseline_differ_by_d0x(oracle):
    x = np.random.default_rng(5).standard_normal(3000) * 8000.0
    yk, _, _ = oracle.iir_block(x, 0, 1, 0)
    yb, _, _ = oracle.iir_block(x, 0, 0, 0)
    b, _ = _ba(0)
    np.testing.assert_allclose(yb - yk, b[0] * x, rtol=0, atol=1e-3)   # rounding of two sum orders


def test_subnorm_threshold_is_one(oracle):
    """`fabs(sum) < is_subnorm_reject` compares against BOOL 1 -> every |w| < 1 is zeroed"""
    x = np.full(500, 0.4)
    y, w, cnt = oracle.iir_block(x, 1, 1, 1)
    assert cnt == 500 and np.all(w == 0.0)
    y2, w2, cnt2 = oracle.iir_block(x, 1, 1, 0)
    assert cnt2 == 0 and np.any(w2 != 0.0)


@pytest.mark.parametrize("f", [30.0, 1000.0, 10000.0, 23500.0])
def test_hilbert_analytic_property(oracle, f):
    fs, n, amp = 48000, 120000, 8000.0
    x = amp * np.sin(2 * np.pi * f * np.arange(n) / fs)
    I, Q = oracle.hilbert_block(x)
    z = I[n // 2:] + 1j * Q[n // 2:]
    m = np.abs(z) / amp
    assert 0.81 <= m.min() and m.max() <= 0.91
    assert (m.max() - m.min()) / m.mean() < 0.013
    assert np.mean(np.diff(np.unwrap(np.angle(z)))) > 0        # e^{+j w t}: positive frequency


def test_render_mid_riser_range_and_clips(oracle):
    cfg = graph.default_config().render
    x = np.array([-40000.0, -32767.4, -0.5, -0.0, 0.0, 0.4, 32766.9, 32768.0, 1e9])
    out, iv, clips, peak = oracle.render_block(x, cfg)
    assert iv.tolist() == [-32767, -32767, -1, 0, 0, 0, 32766, 32767, 32767]
    assert clips == 4
    assert peak == pytest.approx(20 * np.log10(1e9 / 32768.0))


def test_render_mid_tread_24bit_signbits(oracle):
    cfg = graph.default_config().render
    cfg.quantz_type = abi.QUANTZ_MID_TREAD
    cfg.sign_bits24 = 18
    x = np.array([1.0, -1.0, 100.25, -100.75])
    out, iv, clips, _ = oracle.render_block(x, cfg, is24=True)
    # 24-bit, 18 significant bits: norm_shift 6, norm_mul 256/64 = 4; rounds half away (mid-tread)
    assert iv.tolist() == [4 << 6, -4 << 6, 401 << 6, -403 << 6]
    assert out.size == 12


def test_e2e_golden_regression(oracle):
    """the committed oracle vectors still reproduce (guards the restatement against drift)"""
    for p in sorted(GOLD.glob("e2e_*.npz")):
        g = np.load(p)
        raw_cfg = g["cfg"].tobytes()        # fixtures predate cfg.fp_check: zero-extend (off)
        cfg = abi.Config.from_buffer_copy(raw_cfg + bytes(C.sizeof(abi.Config) - len(raw_cfg)))
        nodes = list((abi.Node * (g["nodes"].size // C_sizeof_node())).from_buffer_copy(g["nodes"].tobytes()))
        raw = g["raw"]
        fsz = abi.FMT_BYTES[cfg.in_format] * cfg.in_channels
        out, pre = oracle.process_streams(cfg, nodes, raw, raw.shape[1] // fsz, want_pre=True)
        assert np.array_equal(out, g["out"]), p.name
        assert np.array_equal(pre.view(np.uint64), g["pre"].view(np.uint64)), p.name


def C_sizeof_node():
    import ctypes
    return ctypes.sizeof(abi.Node)


def test_quirk_minus100dbfs_is_silence():
    g = np.load(GOLD / "e2e_quirk_minus100dbfs_f32.npz")
    assert np.all(g["out"] == 0)                  # default config renders silence
    assert g["desubnorm"][0] == 4 * 4800


def test_quirk_square_clips():
    g = np.load(GOLD / "e2e_quirk_fullscale_square.npz")
    v = g["out"].view("<i2")
    assert v.max() == 32767 and v.min() == -32767 and g["clips"][0][0] > 0


def test_block_independence_oracle(oracle):
    """results do not depend on the block partition (state fully carried)"""
    cfg = graph.default_config(48000)
    nodes = graph.graph_pm_shift_mix()
    raw = synth.stream_pcm(3, 3000, 48000)
    a = oracle.Stream(cfg, nodes)
    o1, _ = a.process(raw, 3000)
    b = oracle.Stream(cfg, nodes)
    parts = []
    t = 0
    for n in (576, 1, 1000, 1423):
        o, _ = b.process(raw[t * 4:(t + n) * 4], n)
        parts.append(o)
        t += n
    assert np.array_equal(o1, np.concatenate(parts))


def test_graph_normalisation_amod_init(oracle):
    """amod_init: list without a Master at its head is rejected and replaced by the default
    Master (S_ADD_REIM, 0.8, in)  (adv_modulator.c:225-312)"""
    cfg = graph.default_config()
    bad = [graph.shift(), graph.master()]
    s = oracle.Stream(cfg, bad)
    assert not s.accepted
    d = oracle.Stream(cfg, [graph.master()])
    raw = synth.stream_pcm(0, 500, 48000)
    assert np.array_equal(s.process(raw, 500)[0], d.process(raw, 500)[0])
    two = oracle.Stream(cfg, [graph.master(), graph.master()])
    assert not two.accepted


# ---------------------------------------------------------------- CWAVE input / bus form -------
def _cw_config(fmt, ch, fs=48000):
    return graph.default_config(fs, fmt=fmt, channels=ch)


@pytest.mark.parametrize("fmt", [abi.FMT_CW_F64, abi.FMT_CW_I16, abi.FMT_CW_I16_F32, abi.FMT_CW_F32])
def test_cwave_reads_analytic_signal_as_is(oracle, fmt):
    """xwave_reader.c:171-200, 939-966: CWAVE samples go to the bus unscaled, without Hilbert;
    Master S_RE / S_IM with gain 1 returns Re / Im exactly; mono feeds R with L"""
    for ch in (1, 2):
        raw = synth.stream_cwave(7, 1000, 48000, channels=ch, fmt=fmt)
        rec = {abi.FMT_CW_F64: [("re", "<f8"), ("im", "<f8")], abi.FMT_CW_I16: [("re", "<i2"), ("im", "<i2")],
               abi.FMT_CW_I16_F32: [("re", "<i2"), ("im", "<f4")], abi.FMT_CW_F32: [("re", "<f4"), ("im", "<f4")]}[fmt]
        v = raw.view(np.dtype(rec)).reshape(1000, ch)
        re, im = v["re"].astype(np.float64), v["im"].astype(np.float64)
        if ch == 1:
            re, im = np.repeat(re, 2, axis=1), np.repeat(im, 2, axis=1)
        for tout, want in ((abi.S_RE, re), (abi.S_IM, im)):
            st = oracle.Stream(_cw_config(fmt, ch), [graph.master(tout=tout, gain=1.0)])
            _, pre = st.process(raw, 1000, want_pre=True)
            assert np.array_equal(pre.view(np.uint64), want.view(np.uint64))


def test_cwave_fade_scales_both_components(oracle):
    raw = synth.stream_cwave(1, 9600, 48000, fmt=abi.FMT_CW_F32)
    st = oracle.Stream(_cw_config(abi.FMT_CW_F32, 2), [graph.master(tout=abi.S_IM, gain=1.0)])
    st.open(9600, fade_in_ms=50)
    _, pre = st.process(raw, 9600, want_pre=True)
    im = raw.view(np.dtype([("re", "<f4"), ("im", "<f4")])).reshape(9600, 2)["im"].astype(np.float64)
    n_in = 50 * 48000 // 1000
    fade = np.arange(n_in, dtype=np.float64) / n_in
    # the node's mix starts from 0.0 (adv_modulator.c:655), so a faded -0.0 comes out as +0.0
    assert np.array_equal(pre[:n_in].view(np.uint64), (0.0 + im[:n_in] * fade[:, None]).view(np.uint64))
    assert np.array_equal(pre[n_in:].view(np.uint64), (0.0 + im[n_in:]).view(np.uint64))


def test_bus_leaky_feedback_recurrence(oracle):
    """a Mix node reading its own slot sees last frame's value (adv_modulator.c:655-665):
    C[t] = ((0.0 + in[t]) + C[t-1]) * 0.5, then Master S_RE gain 1"""
    raw = synth.stream_cwave(2, 800, 48000, fmt=abi.FMT_CW_F64)
    nodes = [graph.master(inputs=("C",), tout=abi.S_RE, gain=1.0), graph.mix(inputs=("in", "C"), out="C", gain=0.5)]
    st = oracle.Stream(_cw_config(abi.FMT_CW_F64, 2), nodes)
    _, pre = st.process(raw, 800, want_pre=True)
    x = raw.view(np.dtype([("re", "<f8"), ("im", "<f8")])).reshape(800, 2)["re"]
    c = np.zeros(2)
    want = np.zeros((800, 2))
    for t in range(800):
        c = ((0.0 + x[t]) + c) * 0.5
        want[t] = c
    assert np.array_equal(pre.view(np.uint64), want.view(np.uint64))


def test_bus_pure_delay_is_one_frame_late(oracle):
    """Mix(A->B) executes before Shift(in->A): B is last frame's A"""
    raw = synth.stream_pcm(4, 1500, 48000)
    cfg = graph.default_config(48000)
    _, p1 = oracle.Stream(cfg, graph.graph_shift_master()).process(raw, 1500, want_pre=True)
    _, p2 = oracle.Stream(cfg, graph.graph_pure_delay()).process(raw, 1500, want_pre=True)
    assert np.all(p2[0] == 0.0)
    assert np.array_equal(p2[1:].view(np.uint64), p1[:-1].view(np.uint64))


@pytest.mark.parametrize("type_", [0, 1, 4])
def test_restarted_recurrence_never_resynchronizes(oracle, type_):
    """Why K1 cannot split a stream's time axis: a chain restarted from a zero state part
    way through a track never falls back onto the true trajectory bit for bit -- the DF-II states
    are large (|w| ~ 1e7..1e13) and the rounding noise they carry keeps two trajectories apart at a
    plateau, so no window of N equal states (which would make the rest identical) ever appears"""
    fs, n, s0 = 48000, 160000, 40000
    raw = synth.stream_pcm(3, n, fs).view("<i2").reshape(n, 2)[:, 0].astype(np.float64)
    k = np.arange(n) % 4
    x = np.where(k == 0, raw, np.where(k == 2, -raw, 0.0))          # the I chain's input
    _, w, _ = oracle.iir_block(x, type_, 1, 1)
    _, w2, _ = oracle.iir_block(x[s0:], type_, 1, 1)
    eq = (w[s0:].view(np.uint64) == w2.view(np.uint64)).astype(np.int64)
    run = np.convolve(eq, np.ones(20, dtype=np.int64), mode="valid")   # order <= 20
    assert run.max() < 20
    tail = slice(-20000, None)
    assert np.max(np.abs(w[s0:][tail] - w2[tail])) > 0.0
