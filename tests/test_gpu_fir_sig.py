"""GPU parity of KF2's signature form (icw_fir_sig in icw_kernels.hip): the tiles of a launch block
before the one holding its last frame go through a kernel holding only the staging, the sums, the
render-only signature pass and the meters, and icw_fir_graph takes the rest (icw_launch_fir_graph,
IcwFirArgs.tile0).  Calls of lengths around the tile size (1024 stereo / 2048 mono frames: no tile for
the signature form, exactly one, one plus a frame) in sequence through one context must give the
oracle's bytes and meters, and the same as ICW_FIR_SIG=0 (icw_fir_graph for every tile)."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

pytestmark = pytest.mark.gpu

ORDER, BETA = 254, 8.0


def calls(ch):
    tf = 1024 if ch == 2 else 2048
    return [tf - 1, tf, tf + 1, 3 * tf, 1, 2 * tf + 5]


def run(icw, cfg, nodes, raw, lens, monkeypatch, sig):
    monkeypatch.setenv("ICW_FIR_SIG", sig)
    S = raw.shape[0]
    fsz = raw.shape[1] // sum(lens)
    ctx = icw.Context(cfg, nodes, S)
    ctx.set_fir_hilbert(ORDER, BETA)
    outs, t = [], 0
    for n in lens:
        o, _ = ctx.process(np.ascontiguousarray(raw[:, t * fsz:(t + n) * fsz]), n, want_pre=False)
        outs.append(o)
        t += n
    meters = [ctx.meters(s) for s in range(S)]
    ctx.close()
    return np.concatenate(outs, axis=1), meters


@pytest.mark.parametrize("gname", ["master", "shift_master", "pm_shift_mix"])
@pytest.mark.parametrize("ch", [1, 2])
@pytest.mark.parametrize("b24", [False, True])
@pytest.mark.parametrize("quantz", [abi.QUANTZ_MID_RISER, abi.QUANTZ_MID_TREAD])
def test_signature_form_calls(oracle, icw, gname, ch, b24, quantz, monkeypatch):
    nodes = {"master": graph.graph_master_only, "shift_master": graph.graph_shift_master,
             "pm_shift_mix": graph.graph_pm_shift_mix}[gname]()
    cfg = graph.default_config(48000, fmt=abi.FMT_I16, channels=ch, need24bits=b24)
    cfg.render.quantz_type = quantz
    lens = calls(ch)
    n = sum(lens)
    raw = synth.batch_pcm(3, n, 48000, channels=ch, first=11)
    on, m_on = run(icw, cfg, nodes, raw, lens, monkeypatch, "1")
    off, m_off = run(icw, cfg, nodes, raw, lens, monkeypatch, "0")
    assert np.array_equal(on, off)
    assert m_on == m_off
    ref, _ = oracle.process_streams(cfg, nodes, raw, n, want_pre=False, fir=(ORDER, BETA))
    bad = np.flatnonzero(on != ref)
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}"
    for s in range(3):
        st = oracle.Stream(cfg, nodes)
        st.set_fir(ORDER, BETA)
        t = 0
        fsz = raw.shape[1] // n
        for b in lens:
            st.process(raw[s, t * fsz:(t + b) * fsz], b)
            t += b
        assert m_on[s] == st.meters(), s


@pytest.mark.parametrize("gains", [(1.0, 1.0), (0.5, 0.5), (0.5, 0.75), (0.0, 0.0), (-0.0, 0.0)])
@pytest.mark.parametrize("b24", [False, True])
def test_mono_master_one_computation(oracle, icw, gains, b24, monkeypatch):
    """mono input through a Master whose two gains are the same double: icw_fir_sig computes both
    channels once, two frames per pass in the L / R slots (IcwFirArgs.lr_same); unequal gains, and
    +0.0 against -0.0, keep the two-channel passes.  Bytes and meters are the oracle's and the
    ICW_FIR_SIG=0 form's"""
    nodes = graph.graph_master_only()
    nodes[0].gain[0], nodes[0].gain[1] = gains
    cfg = graph.default_config(48000, fmt=abi.FMT_F32, channels=1, need24bits=b24)
    lens = [5 * 2048 + 7, 2048, 3 * 2048 + 1]
    n = sum(lens)
    rng = np.random.default_rng(int(gains[0] * 1000 + gains[1] * 10 + b24))
    x = (rng.standard_normal((2, n)) * 1.7).astype(np.float32)     # past full scale: clips counted
    x[:, 100:140] = -0.0
    x[0, 3000] = np.nan
    raw = x.view(np.uint8)
    on, m_on = run(icw, cfg, nodes, raw, lens, monkeypatch, "1")
    off, m_off = run(icw, cfg, nodes, raw, lens, monkeypatch, "0")
    assert np.array_equal(on, off)
    assert m_on == m_off
    ref, _ = oracle.process_streams(cfg, nodes, raw, n, want_pre=False, fir=(ORDER, BETA))
    assert np.array_equal(on, ref)
    for s in range(2):
        st = oracle.Stream(cfg, nodes)
        st.set_fir(ORDER, BETA)
        t = 0
        for b in lens:
            st.process(raw[s, t * 4:(t + b) * 4], b)
            t += b
        assert m_on[s] == st.meters(), s
