"""FIR Hilbert converter (icw_set_fir_hilbert), CPU side: the product's taps against the oracle's
own and against scipy's Kaiser window, and the oracle's converter against numpy convolution and
the analytic-signal property.

The converter is the one a CWAVE header names (cwave.h:40,56-58: "Hilbert FIR filter order" k_M,
"filter parameter" k_beta); in_cwave does not ship it, so no reference output exists and this
stage's parity is unpinned.  These tests pin the oracle to the design's definition:
taps from the Kaiser formula (scipy), the sum from a plain convolution, and |I + jQ| ~ A for a sine
in the pass band.
"""
import numpy as np
import pytest
from scipy.signal import windows

from in_cwave_amd import abi, graph
from in_cwave_amd import lib as L
from oracle import oracle as O

ORDERS = [2, 6, 30, 254, 510, 1022, 4096]


@pytest.mark.parametrize("order", ORDERS)
@pytest.mark.parametrize("beta", [0.0, 4.5, 8.0])
def test_taps_product_equal_oracle(order, beta):
    g_prod = L.fir_taps(order, beta)
    g_orc = O.fir_taps(order, beta)
    assert g_prod.size == (order // 2 + 1) // 2
    assert np.array_equal(g_prod.view(np.uint64), g_orc.view(np.uint64))


@pytest.mark.parametrize("order", [30, 254, 1022])
@pytest.mark.parametrize("beta", [0.0, 8.0])
def test_taps_against_scipy_kaiser(order, beta):
    c = order // 2
    w = windows.kaiser(order + 1, beta, sym=True)
    m = np.arange(1, c + 1, 2)
    ref = 2.0 / (np.pi * m) * w[c + m]
    g = O.fir_taps(order, beta)
    np.testing.assert_allclose(g, ref, rtol=1e-13, atol=0)


def test_bad_orders_rejected():
    for order in (0, 1, 3, 4097, 8192):
        with pytest.raises(ValueError):
            O.fir_taps(order, 8.0)
        with pytest.raises(L.IcwError):
            L.fir_taps(order, 8.0)


def _iq_config(fs=48000):
    """mono i16, Master with L = Re (S_RE) and R = Im (S_IM) at gain 1: the pre-render doubles are
    the converter's I and Q exactly"""
    cfg = graph.default_config(fs, fmt=abi.FMT_I16, channels=1)
    nodes = [graph.master(gain=1.0, tout=abi.S_RE, tout_r=abi.S_IM)]
    return cfg, nodes


def _pcm(x):
    return np.clip(np.round(x), -32768, 32767).astype("<i2").view(np.uint8)


@pytest.mark.parametrize("order", [2, 30, 254, 1022])
def test_oracle_converter_is_the_convolution(order):
    rng = np.random.default_rng(order)
    n = 6000
    x = rng.normal(0, 6000, n)
    raw = _pcm(x)
    xv = raw.view("<i2").astype(np.float64)
    cfg, nodes = _iq_config()
    st = O.Stream(cfg, nodes)
    st.set_fir(order, 8.0)
    _, pre = st.process(raw, n, want_pre=True)
    c = order // 2
    g = O.fir_taps(order, 8.0)
    h = np.zeros(order + 1)
    for k, gm in enumerate(g):
        m = 2 * k + 1
        h[c + m] = gm          # x[n - c - m] weight (delay c + m)
        h[c - m] = -gm         # x[n - c + m] weight (delay c - m)
    q_ref = np.convolve(xv, h)[:n]
    i_ref = np.concatenate([np.zeros(c), xv[:n - c]])
    assert np.array_equal(pre[:, 0], i_ref)
    np.testing.assert_allclose(pre[:, 1], q_ref, rtol=0, atol=1e-9 * np.abs(xv).max())


@pytest.mark.parametrize("order", [254, 1022])
def test_oracle_converter_analytic_signal(order):
    fs, f0, a = 48000, 6000.0, 10000.0
    n = 4 * order + 2000
    t = np.arange(n)
    raw = _pcm(a * np.cos(2 * np.pi * f0 / fs * t))
    cfg, nodes = _iq_config(fs)
    st = O.Stream(cfg, nodes)
    st.set_fir(order, 8.0)
    _, pre = st.process(raw, n, want_pre=True)
    env = np.hypot(pre[order:, 0], pre[order:, 1])
    assert np.abs(env / a - 1.0).max() < 2e-3
    # the analytic signal turns counter-clockwise: Q lags I by a quarter period (sin after cos)
    c = order // 2
    q = pre[order:, 1]
    s_ref = a * np.sin(2 * np.pi * f0 / fs * (t[order:] - c))
    assert np.abs(q - s_ref).max() < 2e-3 * a


def test_oracle_block_split_and_mono_right_history():
    """two calls equal one; a mono track followed by a stereo one continues R from L's history"""
    order = 30
    rng = np.random.default_rng(5)
    cfg, nodes = _iq_config()
    one = O.Stream(cfg, nodes)
    one.set_fir(order, 6.0)
    two = O.Stream(cfg, nodes)
    two.set_fir(order, 6.0)
    raw = _pcm(rng.normal(0, 3000, 500))
    a, pa = one.process(raw, 500, want_pre=True)
    b1, p1 = two.process(raw[:2 * 123], 123, want_pre=True)
    b2, p2 = two.process(raw[2 * 123:], 377, want_pre=True)
    assert np.array_equal(pa, np.concatenate([p1, p2]))
    assert np.array_equal(a, np.concatenate([b1, b2]))
