"""In_cwave.cfg texts for tests (test helper): NODE_DSP= lines written from the reference's file
format (handle_node_dsp, config.c:565-652: name with % escapes, doubles as 0x<16 hex digits>),
independently of the product's formatter, plus the hot-path keys of load_config
(config.c:113-296); and the oracle side of such a text, read by oracle/orc_config.py."""
import struct

from in_cwave_amd import abi
from oracle import orc_config as R


def _hexd(x):
    return "0x%016X" % struct.unpack("<Q", struct.pack("<d", float(x)))[0]


def _esc(name):
    return name.replace("%", "%%").replace(" ", "% ").replace("\t", "%\t")


def node_line(n, name):
    f = [_esc(name), _hexd(n.gain[0]), _hexd(n.gain[1]), str(n.lock_gain)]
    f += [str(int(n.inputs[k])) for k in range(abi.N_INPUTS)]
    f += [str(n.xch_mode), str(n.iq_invert[0]), str(n.iq_invert[1]), str(n.mode)]
    if n.mode == abi.MODE_MASTER:
        f += [str(n.tout[0]), str(n.tout[1])]
    elif n.mode == abi.MODE_SHIFT:
        for c in range(2):
            f += [_hexd(n.fr_shift[c]), str(n.is_shift[c])]
        f += [str(n.n_out), str(n.lock_shift), str(n.sign_lock_shift)]
    elif n.mode == abi.MODE_PM:
        for c in range(2):
            f += [_hexd(n.pm_freq[c]), _hexd(n.pm_phase[c]), _hexd(n.pm_level[c]), _hexd(n.pm_angle[c]),
                  str(n.is_pm[c])]
        f += [str(n.n_out), str(n.lock_freq), str(n.lock_phase), str(n.lock_level), str(n.lock_angle)]
    else:
        f += [str(n.n_out)]
    return "NODE_DSP=" + " ".join(f)


def config_text(rng, nodes):
    keys = {
        "VER_CONFIG": 10, "FADE_IN": int(rng.choice([0, 0, 10, 25])), "FADE_OUT": int(rng.choice([0, 0, 15])),
        "FRMOD_SCALED": int(rng.random() < 0.6), "IIR_HBLPF_IX": int(rng.integers(0, 6)),
        "IIR_SUM_KAHAN": int(rng.random() < 0.7), "IIR_SUBN_ZERO": int(rng.random() < 0.8),
        "NEED24BITS": int(rng.random() < 0.5), "QUANTIZE_TYPE": int(rng.integers(0, 2)),
        "RENDER_TYPE": int(rng.choice([0, 0, 1, 2, 3, 4])), "NOISE_SHAPING": int(rng.integers(0, 18)),
        "SIGNBITS16": int(rng.choice([16, 16, 12])), "SIGNBITS24": int(rng.choice([24, 24, 20])),
    }
    lines = ["%s=%d" % (k, v) for k, v in keys.items()]
    lines.append("DITHER_BITS=" + _hexd(rng.choice([1.0, 1.0, 0.5, 2.0])))
    lines += [node_line(n, "node %d%%" % i) for i, n in enumerate(nodes)]
    return "\r\n".join(lines) + "\r\n"


def oracle_side(text, fs):
    """orc_config.load -> abi.Config + abi.Node list, the fields as load_config fills the.cfg"""
    ok, v, dicts = R.load(text)
    assert ok
    cfg = abi.Config()
    cfg.sample_rate, cfg.in_format, cfg.in_channels = fs, abi.FMT_I16, 2
    cfg.hilbert_type, cfg.iir_kahan, cfg.iir_subnorm_reject = v["IIR_HBLPF_IX"], v["IIR_SUM_KAHAN"], v["IIR_SUBN_ZERO"]
    cfg.frmod_scaled, cfg.need24bits, cfg.fp_check = v["FRMOD_SCALED"], v["NEED24BITS"], v["FP_CHECK"]
    cfg.seed_left, cfg.seed_right = abi.SEED_LEFT, abi.SEED_RIGHT
    r = cfg.render
    r.dth_bits, r.quantz_type, r.render_type = v["DITHER_BITS"], v["QUANTIZE_TYPE"], v["RENDER_TYPE"]
    r.nshape_type, r.sign_bits16, r.sign_bits24 = v["NOISE_SHAPING"], v["SIGNBITS16"], v["SIGNBITS24"]
    nodes = []
    for d in dicts:
        n = abi.Node()
        n.mode, n.xch_mode, n.lock_gain = d["mode"], d["xch_mode"], d["lock_gain"]
        n.gain[0], n.gain[1] = d["gain"]
        n.iq_invert[0], n.iq_invert[1] = d["iq_invert"]
        for k in range(abi.N_INPUTS):
            n.inputs[k] = d["inputs"][k]
        n.n_out = d.get("n_out", 0)
        for key in ("tout", "fr_shift", "is_shift", "pm_freq", "pm_phase", "pm_level", "pm_angle", "is_pm"):
            if key in d:
                getattr(n, key)[0], getattr(n, key)[1] = d[key]
        for key in ("lock_shift", "sign_lock_shift", "lock_freq", "lock_phase", "lock_level", "lock_angle"):
            if key in d:
                setattr(n, key, d[key])
        nodes.append(n)
    return cfg, nodes, v
