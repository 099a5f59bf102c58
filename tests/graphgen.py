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
