"""Bit-exact cross-check of the oracle against a second, independently written restatement in pure
Python: the IIR and quadrature Hilbert (tests/pyref_iir.py) for all 6 filter types x Kahan/baseline
x subnorm reject on/off, and the whole per-frame chain (tests/pyref_chain.py: unpack, fades, DSP
list, render, MT19937, noise shapers) over random graphs and the render matrix.  Both follow hblpf.c:894-1056 and lpf_hilbert_quad.c:129-156; agreement bit
for bit on inputs that exercise the reject (small and zero samples) pins the C restatement's
operation order, which the scipy lfilter check (test_oracle.py) can only bound by a tolerance.
"""
import numpy as np
import pytest

from pyref_iir import PyHilbert, PyIIR


def _signal(seed, n):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n) * 8000.0
    x[:40] = rng.standard_normal(40) * 0.3                  # from rest, sub-threshold: rejected
    x[n // 3: n // 3 + 60] = 0.0                            # decaying tail
    x[n // 2: n // 2 + 40] = rng.standard_normal(40) * 0.3
    x[-25:] = 0.0
    return x


@pytest.mark.parametrize("type_", range(6))
@pytest.mark.parametrize("kahan", [0, 1])
@pytest.mark.parametrize("subn", [0, 1])
def test_iir_bit_exact_vs_python_restatement(oracle, type_, kahan, subn):
    x = _signal(100 + type_, 900)
    y, w, cnt = oracle.iir_block(x, type_, kahan, subn)
    f = PyIIR(type_, kahan, subn)
    yp = np.empty_like(x)
    wp = np.empty_like(x)
    for i, v in enumerate(x.tolist()):
        yp[i] = f.step(v)
        wp[i] = f.hist[0]
    assert np.array_equal(y.view(np.uint64), yp.view(np.uint64))
    assert np.array_equal(w.view(np.uint64), wp.view(np.uint64))
    assert cnt == f.subnorm_cnt
    if subn:
        assert cnt > 0                                      # the reject branch was exercised


@pytest.mark.parametrize("type_", range(6))
@pytest.mark.parametrize("kahan", [0, 1])
def test_hilbert_bit_exact_vs_python_restatement(oracle, type_, kahan):
    x = _signal(200 + type_, 700)
    oi, oq = oracle.hilbert_block(x, type_, kahan, 1)
    h = PyHilbert(type_, kahan, 1)
    got = np.array([h.step(v) for v in x.tolist()])
    assert np.array_equal(oi.view(np.uint64), got[:, 0].copy().view(np.uint64))
    assert np.array_equal(oq.view(np.uint64), got[:, 1].copy().view(np.uint64))


def test_python_restatement_coefficients_match_oracle(oracle):
    for t in range(6):
        pc, pd, d0 = oracle.iir_coeffs(t)
        f = PyIIR(t)
        assert np.array_equal(pc, np.array(f.c)) and np.array_equal(pd, np.array(f.d)) and d0 == f.d0


# ------------------------------------------------------------------ the whole chain -------------
def _chain_case(oracle, cfg, nodes, raw, n, n_frame0=0, fades=None):
    from pyref_chain import PyStream
    st = oracle.Stream(cfg, nodes)
    py = PyStream(cfg, nodes)
    if fades:
        st.open(n, *fades)
        py.open(n, *fades)
    if n_frame0:
        st.set_n_frame(n_frame0)
        py.n_frame = n_frame0
    assert st.accepted == py.accepted
    out, pre = st.process(raw, n, want_pre=True)
    pout, ppre = py.process(raw, n)
    ppre = np.array(ppre)
    a, b = pre.view(np.uint64), ppre.view(np.uint64)
    same = (a == b) | (np.isnan(pre) & np.isnan(ppre))
    assert same.all(), f"{(~same).sum()} pre-render doubles differ, first at {np.argwhere(~same)[:3].tolist()}"
    assert bytes(out) == pout
    m = st.meters()
    assert list(m["clips"]) == py.meters["clips"]
    assert list(m["peak_db"]) == py.meters["peak"]


@pytest.mark.parametrize("seed", range(40))
def test_chain_random_graphs_vs_python_restatement(oracle, seed):
    """random DSP lists over the modulator's option space (tests/graphgen.py), both frame-counter
    modes, the list bypass, counters near the scaled wrap: the oracle's pre-render doubles, bytes
    and meters equal a second, independent restatement's"""
    from in_cwave_amd import synth
    from tests import graphgen
    rng = np.random.default_rng(9000 + seed)
    cfg = graphgen.random_config(rng)
    nodes = graphgen.random_list(rng)
    n = 160
    raw = synth.stream_pcm(seed, n, cfg.sample_rate)
    n0 = cfg.sample_rate * 1000 - int(rng.integers(1, 100)) if (cfg.frmod_scaled and seed % 3 == 0) else \
        (int(rng.integers(1, 1 << 40)) if seed % 3 == 1 else 0)
    _chain_case(oracle, cfg, nodes, raw, n, n_frame0=n0)


RENDER_CASES = [(rt, q, b24, ns, sb) for rt in range(5) for q in (0, 1) for b24 in (0, 1)
                for ns, sb in ((0, 0), (2, 0), (16, 1), (7, 0))]


@pytest.mark.parametrize("rt,q,b24,ns,sb", RENDER_CASES)
def test_chain_render_matrix_vs_python_restatement(oracle, rt, q, b24, ns, sb):
    """every render type x quantiser x 16/24 bit, FIR and IIR shapers, reduced sign bits, loud
    (clipping) input: sound_render_value and its MT19937 draws restated independently"""
    from in_cwave_amd import abi, graph, synth
    cfg = graph.default_config(44100, need24bits=bool(b24))
    cfg.render.render_type, cfg.render.quantz_type, cfg.render.nshape_type = rt, q, ns
    cfg.render.dth_bits = 1.5 if rt else 1.0
    if sb:
        cfg.render.sign_bits16, cfg.render.sign_bits24 = 12, 18
    nodes = [graph.master(gain=2.0)]
    n = 200
    raw = synth.stream_pcm(rt * 7 + ns, n, 44100)
    _chain_case(oracle, cfg, nodes, raw, n)


@pytest.mark.parametrize("fmt", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("ch", [1, 2])
def test_chain_formats_and_fades_vs_python_restatement(oracle, fmt, ch):
    """the five WAV sample formats, mono (R fed with L) and stereo, fade in and out"""
    from in_cwave_amd import graph, synth
    cfg = graph.default_config(8000, fmt=fmt, channels=ch)
    nodes = graph.graph_shift_master()
    n = 400
    raw = synth.stream_pcm(fmt + 10 * ch, n, 8000, channels=ch, fmt=fmt)
    _chain_case(oracle, cfg, nodes, raw, n, fades=(10, 10))
