"""dsp_master's (re +- im) / SQRT2 (adv_modulator.c:498-501) on the device (icw_div_sqrt2: the
FMA-corrected reciprocal product, true division outside 2^-900 <= |x| <= DBL_MAX) against the
oracle's division, bit for bit, on the inputs that stress it: every near-midpoint significand of
tests/test_libm.py::test_div_sqrt2_hard_cases in several binades, both signs, zeros, the edges of the
fast range, subnormals, infinities and NaNs.  The values enter as CWAVE f64 samples (I = x, Q = 0)
through a bypassed list whose Master (gain 1.0) adds re + im, so the Master divides x itself."""
import math

import numpy as np
import pytest

from in_cwave_amd import abi, graph

pytestmark = pytest.mark.gpu


def hard_values():
    c = float("1.4142135623730950488016887242097")
    m, ex = math.frexp(c)
    C = int(m * 2 ** 53)
    xs = []
    for s in (53, 54):
        inv = pow(2 ** s, -1, C)
        lo, hi = (C, 2 ** 53) if s == 53 else (2 ** 52, C)
        for k in range(-15, 16, 2):
            X = (-k * inv) % C
            while X < hi:
                if X >= lo:
                    for e2 in (-899, -300, -20, 0, 14, 15, 300, 1020):
                        xs += [X * 2.0 ** (e2 - 52), -X * 2.0 ** (e2 - 52)]
                X += C
    edge = [0.0, -0.0, 2.0 ** -900, -2.0 ** -900, 2.0 ** -900 * (1 - 2 ** -53), 2.0 ** -1000, 5e-324,
            -5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, -1.7976931348623157e308,
            math.inf, -math.inf, math.nan, 32767.0, -32768.0, 1.0, c, 2 * c]
    rng = np.random.default_rng(9)
    rnd = list(rng.standard_normal(2000) * 2.0 ** rng.integers(-40, 40, 2000))
    return np.array(xs + edge + rnd, dtype=np.float64)


@pytest.mark.parametrize("tout", [abi.S_ADD_REIM, abi.S_SUB_REIM])
def test_master_division_matches_oracle(icw, oracle, tout):
    x = hard_values()
    iq = np.zeros((x.size, 2))
    iq[:, 0] = x                                    # I = x, Q = +0: re + im = x, re - im = x
    raw = iq.view(np.uint8).reshape(1, -1)
    cfg = graph.default_config(48000, fmt=abi.FMT_CW_F64, channels=1)
    cfg.bypass_list = 1
    nodes = [graph.master(gain=1.0, tout=tout)]
    ctx = icw.Context(cfg, nodes, 1)
    out, pre = ctx.process(np.ascontiguousarray(raw), x.size, want_pre=True)
    ro, rp = oracle.process_streams(cfg, nodes, raw, x.size, want_pre=True)
    got, want = pre[0, :, 0], rp[0, :, 0]
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan)
    bad = np.flatnonzero(got[~nan].view(np.uint64) != want[~nan].view(np.uint64))
    assert bad.size == 0, (x[~nan][bad[:5]], got[~nan][bad[:5]], want[~nan][bad[:5]])
    assert np.array_equal(out, ro)
    ctx.close()
