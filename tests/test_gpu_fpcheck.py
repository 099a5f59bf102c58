"""FP_CHECK on the GPU: cfg.fp_check runs the FC() arithmetic of fp_check.c:52-100
in the IIR (K1f + K2's output sums) and the render (K3f).  Output bytes, pre-render doubles and the
per-stream census (Hilbert L/R, render L/R x 7 classes) must equal the oracle's on inputs carrying
NaN, +-Inf and denormal samples -- every IIR mode, three render / shaper kinds, CWAVE input, block
splits."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph
from fpcheck_inputs import fc_cfg, special_cw64, special_f32

pytestmark = pytest.mark.gpu


def _run(oracle, icw, cfg, raw, n_frames, nodes=None, blocks=None):
    nodes = graph.graph_master_only() if nodes is None else nodes
    S = raw.shape[0]
    ctx = icw.Context(cfg, nodes, S)
    fsz = ctx.fsz
    outs, pres = [], []
    t = 0
    for b in (blocks or [n_frames]):
        o, p = ctx.process(np.ascontiguousarray(raw[:, t * fsz:(t + b) * fsz]), b, want_pre=True)
        outs.append(o)
        pres.append(p)
        t += b
    out, pre = np.concatenate(outs, axis=1), np.concatenate(pres, axis=1)
    cen = []
    ref_out, ref_pre = oracle.process_streams(cfg, nodes, raw, n_frames, want_pre=True, census=cen)
    assert ctx.last_k1_kernel() == (abi.K1_FC if cfg.in_format < abi.FMT_CW_F64 else ctx.last_k1_kernel())
    assert np.array_equal(pre.view(np.uint64), ref_pre.view(np.uint64))
    assert np.array_equal(out, ref_out)
    for s in range(S):
        assert np.array_equal(ctx.fp_census(s), cen[s]), (s, ctx.fp_census(s).tolist(), cen[s].tolist())
    return cen


@pytest.mark.parametrize("kahan,subn", [(1, 1), (1, 0), (0, 1), (0, 0)])
def test_fp_check_iir_modes_specials(oracle, icw, kahan, subn):
    cen = _run(oracle, icw, fc_cfg(kahan=kahan, subn=subn), special_f32(3, 3000), 3000)
    assert sum(int(c[:2, 0].sum()) for c in cen) > 0          # the Hilbert census saw the specials


@pytest.mark.parametrize("render,ns,need24", [(abi.RENDER_ROUND, abi.NSHAPE_FLAT, False),
                                              (abi.RENDER_RPDF, 5, False),
                                              (abi.RENDER_TPDF, abi.NSHAPE_MEW44, True)])
def test_fp_check_render_kinds_cwave(oracle, icw, render, ns, need24):
    """CWAVE float64: NaN / Inf / denormal values reach the render unfiltered"""
    cfg = fc_cfg(abi.FMT_CW_F64, render=render, ns=ns, need24=need24)
    cen = _run(oracle, icw, cfg, special_cw64(3, 2500), 2500)
    assert sum(int(c[2:, 0].sum()) for c in cen) > 0


def test_fp_check_ordinary_input_matches_plain_path(oracle, icw):
    """no specials: FP_CHECK renders what the plain kernels render, with an empty census"""
    from in_cwave_amd import synth
    raw = synth.batch_pcm(4, 4000, 48000)
    cfg = fc_cfg(abi.FMT_I16, render=abi.RENDER_ROUND, ns=abi.NSHAPE_FLAT, need24=False)
    cen = _run(oracle, icw, cfg, raw, 4000)                 # Master only: pure arithmetic, bit-exact
    assert all(int(c.sum()) == 0 for c in cen)
    fc_out, _ = icw.Context(cfg, graph.graph_master_only(), 4).process(raw, 4000)
    cfg.fp_check = 0
    out_plain, _ = icw.Context(cfg, graph.graph_master_only(), 4).process(raw, 4000)
    assert np.array_equal(out_plain, fc_out)


def test_fp_check_block_splits(oracle, icw):
    """census and shaper ring carried across calls of odd sizes"""
    _run(oracle, icw, fc_cfg(), special_f32(2, 3000, seed=5), 3000, blocks=[576, 1, 19, 20, 1000, 1384])
