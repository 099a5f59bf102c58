"""CPU tests for in_cwave.cfg ingestion (icw_config.c).  The product parser is checked against
the rules of config.c, and against an independent Python restatement of them
(oracle/orc_config.py) on generated files.  Parity unpinned: the reference ships no
configuration file and config.c does not build here."""
import math
import random

import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth
from in_cwave_amd import lib as L
from oracle import orc_config as R


def node_line(n, name="node"):
    return L.node_dsp_format(n, name)


def sample_config():
    nodes = [graph.master(inputs=("C",), gain=0.7), graph.mix(inputs=("in", "B"), out="C"),
             graph.shift(inputs=("A",), out="B", fr=3.5), graph.pm(inputs=("in",), out="A", freq=5.0, level=0.25)]
    names = ["Master", "Mix% C", "Shift B", "PM A"]
    lines = ["VER_CONFIG=10", "WAV_SUPPORT=1", "IBOX_PARENT=1", "FADE_IN=250", "FADE_OUT=99999",
             "IIR_HBLPF_IX=4", "IIR_SUM_KAHAN=0", "IIR_SUBN_THR=0x2A9E7A3B3B4E8B1C", "NEED24BITS=0",
             "DITHER_BITS=0x3FF8000000000000", "RENDER_TYPE=2", "NOISE_SHAPING=5", "SIGNBITS16=14"]
    lines += [node_line(n, nm) for n, nm in zip(nodes, names)]
    return "\r\n".join(lines) + "\r\n", nodes, names


def test_sample_config_loads():
    text, nodes, names = sample_config()
    ok, fc, bad = L.config_load(text)
    assert ok and bad == 0
    c = fc.cfg
    assert (c.hilbert_type, c.iir_kahan, c.need24bits, c.render.render_type, c.render.nshape_type) == (4, 0, 0, 2, 5)
    assert c.render.dth_bits == 1.5 and c.render.sign_bits16 == 14
    assert fc.fade_in == 250 and fc.fade_out == 10000            # clamped to MAX_FADE_INOUT
    assert fc.n_nodes == 4
    for i, (n, nm) in enumerate(zip(nodes, names)):
        assert fc.names[i].value.decode() == nm
        assert node_line(fc.nodes[i], nm) == node_line(n, nm)


def test_round_trip_every_mode():
    for n in (graph.master(tout=abi.S_SUB_REIM, tout_r=abi.S_IM), graph.shift(fr=-7.25, lock=False),
              graph.pm(freq=1.5, level=0.75, phase=-0.5, angle=0.25), graph.mix(inputs=("in", "Q", "Z"), out="Y")):
        line = node_line(n, "a name with blanks")
        m, name = L.node_dsp_parse(line.split("=", 1)[1])
        assert name == "a name with blanks"
        assert node_line(m, name) == line


def test_clamps_like_handle_chk():
    n = graph.shift()
    n.gain[0], n.gain[1] = 9.0, -3.0
    n.fr_shift[0], n.fr_shift[1] = 50.0, -50.0
    n.n_out = 40
    n.xch_mode = 9
    m, _ = L.node_dsp_parse(node_line(n).split("=", 1)[1])
    assert (m.gain[0], m.gain[1], m.fr_shift[0], m.fr_shift[1], m.n_out, m.xch_mode) == (2.0, 0.0, 20.0, -20.0, 27, 4)
    p = graph.pm(freq=99.0, level=3.0, phase=-4.0, angle=4.0)
    q, _ = L.node_dsp_parse(node_line(p).split("=", 1)[1])
    assert (q.pm_freq[0], q.pm_level[0], q.pm_phase[0], q.pm_angle[0]) == (40.0, 1.0, -1.0, 1.0)


@pytest.mark.parametrize("text,bad_line", [
    ("NEED24BITS=0\n", 0),                                  # no VER_CONFIG -> version 0 -> defaults
    ("VER_CONFIG=9\nNEED24BITS=0\n", 0),                    # wrong version
    ("VER_CONFIG=10\nNO_SUCH_KEY=1\n", 2),                  # unknown key
    ("VER_CONFIG=10\nNEED24BITS\n", 2),                     # no '='
    ("VER_CONFIG=10\nNEED24BITS=x\n", 2),                   # not a number
    ("VER_CONFIG=10\nNODE_DSP=m 0x0 0x0 1\n", 2),           # truncated node
    ("VER_CONFIG=10\nNEED24BITS=0\x01\n", 2),               # control character
    ("VER_CONFIG=10\nNEED24BITS=0 " + "x" * 2100 + "\n", 2),  # over-long line
])
def test_failures_reset_to_defaults(text, bad_line):
    ok, fc, bad = L.config_load(text)
    assert not ok and bad == bad_line
    assert fc.cfg.need24bits == 1 and fc.n_nodes == 0 and fc.ver_config == 10
    rok, vals, nodes = R.load(text)
    assert not rok and vals["NEED24BITS"] == 1 and nodes == []


def test_blank_lines_tabs_case_and_escapes():
    text = "\n   \n\tver_config\t=\t10\n\nneed24bits= 0 trailing junk\n"
    ok, fc, _ = L.config_load(text)
    assert ok and fc.cfg.need24bits == 0
    assert R.load(text)[0]


def test_too_many_nodes():
    line = node_line(graph.mix(out="A"), "m")
    text = "VER_CONFIG=10\n" + "\n".join([node_line(graph.master(), "M")] + [line] * 64) + "\n"
    ok, fc, bad = L.config_load(text)
    assert not ok and fc.n_nodes == 0


def _rand_token(rng):
    k = rng.random()
    if k < 0.3:
        return str(rng.randint(-3, 40))
    if k < 0.55:
        return "0x%016X" % struct_d2u(rng.uniform(-60, 60))
    if k < 0.8:
        return repr(round(rng.uniform(-60, 60), rng.randint(0, 6)))
    return rng.choice(["0", "1", "abc", "-0", "+7", "12abc", "0x", "0xZZ", "2.5e1", "-1e-2"])


def struct_d2u(x):
    import struct
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def test_node_parser_vs_restatement_fuzz():
    """product parser == the Python restatement on generated NODE_DSP argument strings"""
    rng = random.Random(2024)
    for _ in range(3000):
        mode = rng.randint(-1, 4)
        n_fields = {0: 2, 1: 7, 2: 15, 3: 1}.get(max(0, min(3, mode)), 1)
        toks = ["nm%%%d" % rng.randint(0, 9)] + [_rand_token(rng) for _ in range(2)] + \
               [str(rng.randint(0, 1)) for _ in range(28)] + [str(rng.randint(-2, 6))] + \
               [str(rng.randint(0, 1)) for _ in range(2)] + [str(mode)] + \
               [_rand_token(rng) for _ in range(n_fields - rng.randint(0, 1))]
        args = " " + " ".join(toks)
        want = R.parse_node(args)
        try:
            got, name = L.node_dsp_parse(args)
        except L.IcwError:
            got = None
        if want is None:
            assert got is None, args
            continue
        assert got is not None, args
        assert name == want["name"]
        assert [got.gain[0], got.gain[1]] == want["gain"]
        assert list(got.inputs) == want["inputs"][:27]
        assert got.mode == want["mode"] and got.xch_mode == want["xch_mode"]
        if got.mode == abi.MODE_SHIFT:
            assert [got.fr_shift[0], got.fr_shift[1]] == want["fr_shift"] and got.n_out == want["n_out"]
        if got.mode == abi.MODE_PM:
            for k in ("pm_freq", "pm_phase", "pm_level", "pm_angle"):
                assert list(getattr(got, k)) == want[k], (k, args)
        if got.mode == abi.MODE_MASTER:
            assert list(got.tout) == want["tout"]


def test_config_drives_the_oracle_graph(oracle):
    """a loaded config yields the DSP list and render settings that icw_create / the oracle use"""
    text, nodes, _ = sample_config()
    ok, fc, _ = L.config_load(text, sample_rate=48000)
    assert ok
    cfg = fc.cfg
    raw = synth.stream_pcm(1, 2000, 48000)
    a = oracle.Stream(cfg, L.config_nodes(fc)).process(raw, 2000, want_pre=True)
    ref_cfg = graph.default_config(48000, hilbert_type=4)
    ref_cfg.iir_kahan = 0
    ref_cfg.render.render_type, ref_cfg.render.nshape_type = abi.RENDER_TPDF, 5
    ref_cfg.render.dth_bits, ref_cfg.render.sign_bits16 = 1.5, 14
    b = oracle.Stream(ref_cfg, nodes).process(raw, 2000, want_pre=True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_generated_config_texts_agree_with_restatement():
    """the texts tests/test_gpu_config_device.py feeds to the GPU: the product reader and the
    Python restatement give byte-identical icw_config / icw_node structures, equal to the graph
    the text was written from"""
    from tests import graphgen
    from tests.cfggen import config_text, oracle_side
    for seed in range(48):
        rng = np.random.default_rng(4242 + seed)
        fs = int(rng.choice(graphgen.RATES))
        nodes = graphgen.random_list(rng)
        text = config_text(rng, nodes)
        ok, fc, bad = L.config_load(text, sample_rate=fs)
        assert ok and bad == 0
        cfg_o, nodes_o, _ = oracle_side(text, fs)
        assert bytes(fc.cfg) == bytes(cfg_o)
        assert fc.n_nodes == len(nodes_o) == len(nodes)
        for i in range(fc.n_nodes):
            assert bytes(fc.nodes[i]) == bytes(nodes_o[i]) == bytes(nodes[i])
