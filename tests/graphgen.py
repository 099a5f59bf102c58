"""Seeded random DSP lists over the whole modulator option space (test helper).

Draws what adv_modulator.c lets a configuration hold (NODE_DSP, in_cwave.h:207-287, ranges
in_cwave.h:164-182): Master / Shift / PM / Mix nodes with 1-3 input slots, every channel exchange
(adv_modulator.c:669-700), per-channel I/Q inversion (:703-714), locked and unlocked L/R gains
(:240-244, 717-722), Shift / PM channels switched off (is_shift / is_pm = 0, :523, :558), PM
phase / angle != 0 (:569), all four Master conversions with L != R (:485-507), plus the
context-wide list bypass (:637, 644-651) and frame-counter mode (:611-625).  Lists come out in
the register form (every slot a node reads is written earlier in the frame or never) and in the
bus form (one-frame delays, feedback).
"""
import numpy as np

from in_cwave_amd import abi, graph

RATES = (8000, 22050, 44100, 48000, 96000, 192000)


def _channel_pair(rng, lo, hi, p_equal=0.3):
    a = float(rng.uniform(lo, hi))
    b = a if rng.random() < p_equal else float(rng.uniform(lo, hi))
    return a, b


def _common(rng, n, slots):
    """input mask, exchange, I/Q inversion and gains of a node"""
    k = int(rng.integers(1, 4))
    for s in rng.choice(slots, size=min(k, len(slots)), replace=False):
        n.inputs[int(s)] = 1
    n.xch_mode = int(rng.choice([abi.XCH_NORMAL, abi.XCH_SWAP, abi.XCH_LEFTONLY, abi.XCH_RIGHTONLY,
                                 abi.XCH_MIXLR], p=[0.4, 0.15, 0.15, 0.15, 0.15]))
    n.iq_invert[0] = int(rng.random() < 0.3)
    n.iq_invert[1] = int(rng.random() < 0.3)
    n.gain[0], n.gain[1] = _channel_pair(rng, 0.0, 2.0)          # MAX_GAIN 2.0
    n.lock_gain = int(rng.random() < 0.4)


def random_node(rng, mode, out_slot, slots):
    n = abi.Node()
    n.mode = mode
    _common(rng, n, slots)
    if mode == abi.MODE_MASTER:
        n.tout[0] = int(rng.integers(0, 4))
        n.tout[1] = int(rng.integers(0, 4))
        return n
    n.n_out = out_slot
    if mode == abi.MODE_SHIFT:
        # integer Hz, fractions, negative (mirrored) shifts; |fr| <= MAX_FSHIFT 20
        for c in range(2):
            f = float(rng.choice([rng.integers(-20, 21), rng.uniform(-20, 20), rng.uniform(-1, 1)]))
            n.fr_shift[c] = f
            n.is_shift[c] = int(rng.random() < 0.85)
        n.lock_shift = int(rng.random() < 0.5)
        n.sign_lock_shift = int(rng.random() < 0.5)
    elif mode == abi.MODE_PM:
        n.pm_freq[0], n.pm_freq[1] = _channel_pair(rng, 0.0, 40.0)    # MAX_PMFREQ
        n.pm_phase[0], n.pm_phase[1] = _channel_pair(rng, -1.0, 1.0)  # MIN/MAX_PMPHASE
        n.pm_level[0], n.pm_level[1] = _channel_pair(rng, 0.0, 1.0)   # MAX_PMLEVEL
        n.pm_angle[0], n.pm_angle[1] = _channel_pair(rng, -1.0, 1.0)  # MIN/MAX_PMANGLE
        n.is_pm[0] = int(rng.random() < 0.85)
        n.is_pm[1] = int(rng.random() < 0.85)
        n.lock_freq, n.lock_phase, n.lock_level, n.lock_angle = (int(rng.random() < 0.4) for _ in range(4))
    return n


def random_list(rng, n_nodes=None):
    """head first: Master, then Shift / PM / Mix nodes (executed tail -> head)"""
    n_nodes = int(rng.integers(1, 7)) if n_nodes is None else n_nodes
    outs = [int(x) for x in rng.choice(np.arange(1, abi.N_INPUTS), size=n_nodes - 1, replace=False)]
    spare = int(rng.integers(1, abi.N_INPUTS))          # a slot that may never be written
    slots = [0] + outs + [spare]
    nodes = [random_node(rng, abi.MODE_MASTER, 0, slots)]
    for o in outs:
        mode = int(rng.choice([abi.MODE_SHIFT, abi.MODE_PM, abi.MODE_MIX]))
        nodes.append(random_node(rng, mode, o, slots))
    return nodes


def random_config(rng):
    fs = int(rng.choice(RATES))
    cfg = graph.default_config(fs)
    cfg.frmod_scaled = int(rng.random() < 0.6)
    cfg.bypass_list = int(rng.random() < 0.2)
    return cfg


# ---- plain chains: the production fast paths ---------------------------------------------------
# The host compiles a *chain* (every op reads only `in` and / or the op just before it) with no channel
# exchange, no I/Q inversion, both channels of every Shift / PM rotating and a Master summing re + im
# into a signature (icw_host.cpp compile_graph, IcwProg.sig); the three BASELINE structures among them
# run specialised code (ICW_SIG_M / _SM / _PSXM, icw_kernels.hip), and KF2 runs those in the render-only
# form (icw_sig_fast) when a call asks for no pre-render doubles.  Structures, as (mode, reads) per op
# in execution order (tail first); reads: 1 = in, 2 = the previous op, 3 = both.
SIG_STRUCTS = {
    "M": [(abi.MODE_MASTER, 1)],
    "SM": [(abi.MODE_SHIFT, 1), (abi.MODE_MASTER, 2)],
    "PSXM": [(abi.MODE_PM, 1), (abi.MODE_SHIFT, 2), (abi.MODE_MIX, 3), (abi.MODE_MASTER, 2)],
}


def _gain_pair(rng, unit_p):
    """a node's L / R gains: exactly 1.0 now and then (the ICW_SIG_UNIT lists), locked or not"""
    if rng.random() < unit_p:
        return 1.0, 1.0, 1
    a, b = _channel_pair(rng, 0.0, 2.0, p_equal=0.2)
    lock = int(rng.random() < 0.5)
    return a, b, lock


def plain_node(rng, mode, out_slot, reads, prev_slot, rotate_p=0.93):
    """one node of a plain chain: reads `in` (bit 1) and / or prev_slot (bit 2)"""
    n = abi.Node()
    n.mode = mode
    if reads & 1:
        n.inputs[0] = 1
    if reads & 2:
        n.inputs[prev_slot] = 1
    n.xch_mode = abi.XCH_NORMAL
    if mode == abi.MODE_MASTER:
        n.gain[0], n.gain[1], n.lock_gain = _gain_pair(rng, 0.15)
        n.tout[0] = n.tout[1] = abi.S_ADD_REIM
        return n
    n.gain[0], n.gain[1], n.lock_gain = _gain_pair(rng, 0.5)
    n.n_out = out_slot
    if mode == abi.MODE_SHIFT:
        for c in range(2):
            kind = rng.integers(0, 4)
            if kind == 0:
                f = float(rng.integers(-20, 21))                 # integer Hz, either sign
            elif kind == 1:
                f = float(rng.uniform(-20, 20))                  # fractional
            elif kind == 2:
                f = float(rng.uniform(-1, 1))                    # below 1 Hz
            else:
                f = float(rng.choice([2.0, -2.0, 0.5, -0.25, 19.999]))
            n.fr_shift[c] = f
            n.is_shift[c] = int(rng.random() < rotate_p)
        n.lock_shift = int(rng.random() < 0.5)
        n.sign_lock_shift = int(rng.random() < 0.5)
    elif mode == abi.MODE_PM:
        n.pm_freq[0], n.pm_freq[1] = _channel_pair(rng, 0.0, 40.0)
        n.pm_phase[0], n.pm_phase[1] = _channel_pair(rng, -1.0, 1.0)
        n.pm_level[0], n.pm_level[1] = _channel_pair(rng, 0.0, 1.0)
        n.pm_angle[0], n.pm_angle[1] = _channel_pair(rng, -1.0, 1.0)
        if rng.random() < 0.2:                                  # the create_node_dsp defaults
            n.pm_phase[0] = n.pm_phase[1] = n.pm_angle[0] = n.pm_angle[1] = 0.0
        n.is_pm[0] = int(rng.random() < rotate_p)
        n.is_pm[1] = int(rng.random() < rotate_p)
        n.lock_freq, n.lock_phase, n.lock_level, n.lock_angle = (int(rng.random() < 0.4) for _ in range(4))
    return n


def plain_chain(rng, p_sig=0.6):
    """(name, nodes head first): one of the BASELINE structures with random parameters (p_sig), or a
    random plain chain of 1-6 ops; every op reads `in` and / or the op before it"""
    if rng.random() < p_sig:
        name = str(rng.choice(sorted(SIG_STRUCTS)))
        struct = SIG_STRUCTS[name]
    else:
        name = "chain"
        k = int(rng.integers(0, 6))
        struct = [(int(rng.choice([abi.MODE_SHIFT, abi.MODE_PM, abi.MODE_MIX])), 1 if i == 0 else int(rng.integers(1, 4)))
                  for i in range(k)]
        struct.append((abi.MODE_MASTER, 1 if k == 0 else int(rng.integers(1, 4))))
    outs = [int(x) for x in rng.choice(np.arange(1, abi.N_INPUTS), size=len(struct) - 1, replace=False)]
    exec_order, prev = [], 0
    for i, (mode, reads) in enumerate(struct):
        out = outs[i] if mode != abi.MODE_MASTER else 0
        if i == 0:
            reads = 1
        exec_order.append(plain_node(rng, mode, out, reads, prev))
        prev = out
    return name, exec_order[::-1]


def plain_config(rng, fir=False):
    """frame-counter mode, rate, input format / channels, quantiser, depth and sign bits of a plain-chain
    case; ROUND + flat (the render K2 / KF2 do themselves)"""
    fs = int(rng.choice(RATES))
    fmt, ch = [(abi.FMT_I16, 2), (abi.FMT_I16, 1), (abi.FMT_F32, 2), (abi.FMT_I24, 2)][int(rng.choice(4, p=[0.5, 0.2, 0.2, 0.1]))]
    cfg = graph.default_config(fs, fmt=fmt, channels=ch, need24bits=bool(rng.random() < 0.4))
    cfg.frmod_scaled = int(rng.random() < 0.6)
    cfg.render.quantz_type = int(rng.integers(0, 2))
    cfg.render.sign_bits16 = int(rng.choice([16, 16, 12]))
    cfg.render.sign_bits24 = int(rng.choice([24, 24, 20]))
    return cfg
