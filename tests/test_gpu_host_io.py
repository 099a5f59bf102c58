"""Host-buffer calls whose buffers are pinned (icw_host_alloc): each launch block's input slice is
copied in and its output slice out on the context's copy stream, beside the other blocks' kernels
(icw_process_streams, pipe_io).  Output must equal the oracle and the pageable-buffer call."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth
from in_cwave_amd import lib as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("render", ["round", "tpdf_mew44"])
def test_pinned_host_buffers_block_pipeline(oracle, icw, render, monkeypatch):
    monkeypatch.setenv("ICW_BLOCK", "2048")           # 11 launch blocks, first block 640
    monkeypatch.setenv("ICW_FIRST_BLOCK", "640")
    cfg = graph.default_config(48000, need24bits=render != "round")
    if render != "round":
        cfg.render.render_type = abi.RENDER_TPDF
        cfg.render.nshape_type = abi.NSHAPE_MEW44
    nodes = graph.graph_shift_master()
    S, T = 16, 20011
    raw = synth.batch_pcm(S, T, 48000)
    ctx = icw.Context(cfg, nodes, S)
    osz = 2 * ctx.render_size
    h_in = L.host_array(raw.shape)
    h_in[:] = raw
    h_out = L.host_array((S, T * osz))
    h_out[:] = 0xEE
    ctx.process(h_in, T, out=h_out)
    ref, _ = oracle.process_streams(cfg, nodes, raw, T)
    assert np.array_equal(np.asarray(h_out), ref)
    # the same call over pageable buffers, on a fresh context
    ctx2 = icw.Context(cfg, nodes, S)
    out2, _ = ctx2.process(raw, T)
    assert np.array_equal(out2, ref)
    # and a second pinned call continues the streams' state
    raw2 = synth.batch_pcm(S, T, 48000, first=S)
    h_in[:] = raw2
    ctx.process(h_in, T, out=h_out)
    out3, _ = ctx2.process(raw2, T)
    assert np.array_equal(np.asarray(h_out), out3)
    ctx.close()
    ctx2.close()
