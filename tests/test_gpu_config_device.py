"""In_cwave.cfg ingestion on the device path: the text of a configuration file
with NODE_DSP= lines goes through icw_config_load -> icw_create -> the HIP path, and the same text
goes through the independent Python reader (oracle/orc_config.py) into the oracle; the rendered
bytes and the pre-render doubles must agree bit for bit.

The lines are written here from the reference's file format (handle_node_dsp, config.c:565-652:
name with % escapes, doubles as 0x<16 hex digits>), not with the product's own formatter.  The
graphs come from tests/graphgen.py (locks off and on, channel exchange, I/Q inversion, 1-6 nodes,
register and bus forms); the keys cover the Hilbert filter and sum mode, the frame-counter mode,
the render (type, shaper, dither bits, quantiser, 16/24 bit, sign bits) and the fades
(load_config, config.c:813-915; amod_init locks, adv_modulator.c:216-299)."""
import numpy as np
import pytest

from in_cwave_amd import abi, synth
from tests import graphgen
from tests.cfggen import config_text, oracle_side

pytestmark = pytest.mark.gpu

N_CASES = 48
N_STREAMS = 3
N_FRAMES = 2400


@pytest.mark.parametrize("seed", range(N_CASES))
def test_config_text_through_libicw_equals_oracle(oracle, icw, seed):
    rng = np.random.default_rng(4242 + seed)
    fs = int(rng.choice(graphgen.RATES))
    nodes = graphgen.random_list(rng)
    text = config_text(rng, nodes)

    ok, fc, bad = icw.config_load(text, sample_rate=fs, fmt=abi.FMT_I16, channels=2)
    assert ok and bad == 0
    cfg_o, nodes_o, v = oracle_side(text, fs)
    assert (fc.fade_in, fc.fade_out) == (v["FADE_IN"], v["FADE_OUT"])

    raw = synth.batch_pcm(N_STREAMS, N_FRAMES, fs, first=100 + seed * N_STREAMS)
    ctx = icw.Context(fc.cfg, icw.config_nodes(fc), N_STREAMS)
    for s in range(N_STREAMS):
        ctx.stream_open(s, N_FRAMES, fc.fade_in, fc.fade_out, 0)
    out, pre = ctx.process(raw, N_FRAMES, want_pre=True)
    for s in range(N_STREAMS):
        st = oracle.Stream(cfg_o, nodes_o)
        assert st.accepted == ctx.accepted
        st.open(N_FRAMES, v["FADE_IN"], v["FADE_OUT"], 0)
        ro, rp = st.process(raw[s], N_FRAMES, want_pre=True)
        a, b = pre[s], rp
        bad = np.flatnonzero((a.view(np.uint64) != b.view(np.uint64)) & ~(np.isnan(a) & np.isnan(b)))
        assert bad.size == 0, f"seed {seed} stream {s}: {bad.size} pre-render doubles differ"
        assert np.array_equal(out[s], ro), f"seed {seed} stream {s}: rendered bytes differ"
    ctx.close()
