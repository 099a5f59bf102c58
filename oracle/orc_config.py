"""TEST INFRASTRUCTURE -- an independent Python restatement of the reference's config file reader
(config.c), used to cross-check the product's C parser (icw_config.c) on generated inputs.

Follows: read_conf_line (config.c:307-363), handle_string read side (config.c:410-441),
handle_bool / _int / _unsigned / _double (config.c:445-541), handle_node_dsp read side
(config.c:663-774), load_config (config.c:813-915) and the config_list bounds
(config.c:113-207).  Parity unpinned: the reference ships no configuration file and config.c
cannot be compiled here (it needs <windows.h>); the rules are restated from the source text.
"""
import re
import struct

MAX_LINE, MAX_KEYW = 2048, 80
MAX_ARGS = MAX_LINE - MAX_KEYW
N_INPUTS = 27


def next_token(s, pos, max_size):
    """handle_string: returns (token, new_pos)"""
    n = len(s)
    while pos < n and s[pos] in " \t":
        pos += 1
    out = []
    while pos < n and s[pos] not in " \t":
        if s[pos] == "%":
            pos += 1
            if pos < n and s[pos] in " \t%":
                if len(out) < max_size - 2:
                    out.append(s[pos])
                pos += 1
        else:
            if len(out) < max_size - 2:
                out.append(s[pos])
            pos += 1
    if pos < n:
        pos += 1
    return "".join(out), pos


_INT = re.compile(r"\s*([+-]?\d+)")
_FLT = re.compile(r"\s*([+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)")
_HEX = re.compile(r"\s*(?:0[xX])?([0-9a-fA-F]+)")


def scan_int(tok):
    m = _INT.match(tok)
    if not m:
        return None
    v = int(m.group(1))
    return ((v + 2 ** 31) % 2 ** 32) - 2 ** 31          # C int wrap on overflow


def scan_unsigned(tok):
    m = _INT.match(tok)
    return None if not m else int(m.group(1)) % 2 ** 32


def scan_double(tok):
    if tok[:2] in ("0x", "0X"):
        m = _HEX.match(tok[2:])
        if not m:
            return None
        return struct.unpack("<d", struct.pack("<Q", int(m.group(1), 16) % 2 ** 64))[0]
    m = _FLT.match(tok)
    return None if not m else float(m.group(1))


def clamp(v, lo, hi):
    if v < lo:
        v = lo
    if v > hi:
        v = hi
    return v


def parse_node(args):
    """handle_node_dsp read side -> dict, or None if a field is missing"""
    pos = 0
    name, pos = next_token(args, pos, 96)
    d = {"name": name}

    def tok():
        nonlocal pos
        t, pos = next_token(args, pos, MAX_ARGS)
        return t

    def rd(kind, lo=None, hi=None):
        v = {"bool": scan_int, "int": scan_int, "double": scan_double}[kind](tok())
        if v is None:
            raise ValueError
        if kind == "bool":
            return 1 if v else 0
        return v if lo is None else clamp(v, lo, hi)

    try:
        d["gain"] = [rd("double", 0.0, 2.0), rd("double", 0.0, 2.0)]
        d["lock_gain"] = rd("bool")
        d["inputs"] = [rd("bool") for _ in range(N_INPUTS)]
        d["xch_mode"] = rd("int", 0, 4)
        d["iq_invert"] = [rd("bool"), rd("bool")]
        d["mode"] = rd("int", 0, 3)
        if d["mode"] == 0:
            d["tout"] = [rd("int", 0, 3), rd("int", 0, 3)]
        elif d["mode"] == 1:
            d["fr_shift"], d["is_shift"] = [0.0, 0.0], [0, 0]
            for c in range(2):
                d["fr_shift"][c] = rd("double", -20.0, 20.0)
                d["is_shift"][c] = rd("bool")
            d["n_out"] = rd("int", 1, N_INPUTS)
            d["lock_shift"], d["sign_lock_shift"] = rd("bool"), rd("bool")
        elif d["mode"] == 2:
            for k in ("pm_freq", "pm_phase", "pm_level", "pm_angle", "is_pm"):
                d[k] = [0, 0]
            for c in range(2):
                d["pm_freq"][c] = rd("double", 0.0, 40.0)
                d["pm_phase"][c] = rd("double", -1.0, 1.0)
                d["pm_level"][c] = rd("double", 0.0, 1.0)
                d["pm_angle"][c] = rd("double", -1.0, 1.0)
                d["is_pm"][c] = rd("bool")
            d["n_out"] = rd("int", 1, N_INPUTS)
            d["lock_freq"], d["lock_phase"], d["lock_level"], d["lock_angle"] = (rd("bool") for _ in range(4))
        else:
            d["n_out"] = rd("int", 1, N_INPUTS)
    except ValueError:
        return None
    return d


KEYS = {  # name: (kind, lo, hi)
    "VER_CONFIG": ("unsigned", 0, 2 ** 32 - 1), "WAV_SUPPORT": ("bool",), "RWAVE_SUPPORT": ("bool",),
    "IBOX_PARENT": ("unsigned", 0, 2), "LAST_CHANCE": ("bool",), "PLAY_SLEEP": ("unsigned", 0, 100),
    "DISABLE_SLEEP": ("bool",), "SEC_ALIGN": ("unsigned", 0, 20), "FADE_IN": ("unsigned", 0, 10000),
    "FADE_OUT": ("unsigned", 0, 10000), "FRMOD_SCALED": ("bool",), "IIR_HBLPF_IX": ("unsigned", 0, 5),
    "IIR_SUM_KAHAN": ("bool",), "IIR_SUBN_ZERO": ("bool",), "IIR_SUBN_THR": ("double", 1e-300, 1e-40),
    "CLR_NFRAME_PT": ("bool",), "CLR_HILB_PT": ("bool",), "SHOW_LONGNUMB": ("bool",), "FP_CHECK": ("bool",),
    "NEED24BITS": ("bool",), "DITHER_BITS": ("double", 0.0, 23.0), "QUANTIZE_TYPE": ("unsigned", 0, 1),
    "RENDER_TYPE": ("unsigned", 0, 4), "NOISE_SHAPING": ("unsigned", 0, 17), "SIGNBITS16": ("unsigned", 2, 16),
    "SIGNBITS24": ("unsigned", 2, 24),
}

DEFAULTS = {"VER_CONFIG": 0, "SEC_ALIGN": 0, "FADE_IN": 0, "FADE_OUT": 0, "FRMOD_SCALED": 1, "IIR_HBLPF_IX": 1,
            "IIR_SUM_KAHAN": 1, "IIR_SUBN_ZERO": 1, "IIR_SUBN_THR": 1e-150, "CLR_NFRAME_PT": 0, "CLR_HILB_PT": 0,
            "FP_CHECK": 0, "NEED24BITS": 1, "DITHER_BITS": 1.0, "QUANTIZE_TYPE": 1, "RENDER_TYPE": 0,
            "NOISE_SHAPING": 0, "SIGNBITS16": 16, "SIGNBITS24": 24}


def load(text):
    """load_config -> (ok, values dict, nodes list)"""
    vals, nodes = dict(DEFAULTS), []
    ok = True
    lines = text.split("\n")
    if lines and lines[-1] == "":
        lines = lines[:-1]
    for raw in lines:
        line = raw.replace("\r", "").replace("\t", " ")
        if len(line) >= MAX_LINE:
            ok = False
            break
        if any(ord(c) < 32 or ord(c) == 127 for c in line):
            ok = False
            break
        if not any(33 <= ord(c) <= 126 for c in line):
            continue
        if "=" not in line:
            ok = False
            break
        kpart, args = line.split("=", 1)
        key, _ = next_token(kpart, 0, MAX_KEYW)
        key = key.upper()
        if key == "NODE_DSP":
            n = parse_node(args)
            if n is None or len(nodes) >= 64:
                ok = False
                break
            nodes.append(n)
            continue
        if key not in KEYS:
            ok = False
            break
        kind = KEYS[key]
        t, _ = next_token(args, 0, MAX_ARGS)
        v = {"bool": scan_int, "unsigned": scan_unsigned, "double": scan_double}[kind[0]](t)
        if v is None:
            ok = False
            break
        if kind[0] == "bool":
            v = 1 if v else 0
        else:
            v = clamp(v, kind[1], kind[2])
        vals[key] = v
    if not ok or vals["VER_CONFIG"] != 10:
        vals, nodes = dict(DEFAULTS), []
        vals["VER_CONFIG"] = 10
        return False, vals, nodes
    return True, vals, nodes
