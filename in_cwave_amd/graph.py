"""DSP-list (NODE_DSP) builders with the reference's defaults and the default configuration.

Mirrors create_node_dsp (adv_modulator.c:89-172), amod_add_lastdsp (adv_modulator.c:381-399) and
load_config_default's hot-path defaults (config.c:118-207).  The list is head first: element 0
is the Master; amod_add_lastdsp appends at the tail, and the list is EXECUTED tail -> head
(adv_modulator.c:637).
"""
from . import abi

DEF_GAIN_MOD = 1.0          # in_cwave.h:166
DEF_GAIN_MASTER = 0.8       # in_cwave.h:167
DEF_FSHIFT = 2.0            # in_cwave.h:163
DEF_PMFREQ = 4.0            # in_cwave.h:170
DEF_PMLEVEL = 0.5           # in_cwave.h:182
DEF_PMPHASE = 0.0
DEF_PMANGLE = 0.0


def slot(name):
    """'in' -> 0, 'A' -> 1 ... 'Z' -> 26 (in_cwave.h:244)."""
    if name == "in":
        return 0
    return ord(name.upper()) - ord("A") + 1


def _base(mode, inputs, gain):
    n = abi.Node()
    n.mode = mode
    n.gain[0] = n.gain[1] = gain
    for k in inputs:
        n.inputs[k if isinstance(k, int) else slot(k)] = 1
    n.xch_mode = abi.XCH_NORMAL
    n.lock_gain = 1
    return n


def master(inputs=("in",), gain=DEF_GAIN_MASTER, tout=abi.S_ADD_REIM, tout_r=None):
    n = _base(abi.MODE_MASTER, inputs, gain)
    n.tout[0] = tout
    n.tout[1] = tout if tout_r is None else tout_r
    return n


def shift(inputs=("in",), out="Z", fr=DEF_FSHIFT, fr_r=None, gain=DEF_GAIN_MOD, lock=True, sign_lock=True):
    """Shift node; defaults: +2 Hz left, mirrored -2 Hz right (adv_modulator.c:127-135)."""
    n = _base(abi.MODE_SHIFT, inputs, gain)
    n.n_out = out if isinstance(out, int) else slot(out)
    n.fr_shift[0] = fr
    n.fr_shift[1] = (-fr if sign_lock else fr) if fr_r is None else fr_r
    n.is_shift[0] = n.is_shift[1] = 1
    n.lock_shift = 1 if lock else 0
    n.sign_lock_shift = 1 if sign_lock else 0
    return n


def pm(inputs=("in",), out="Z", freq=DEF_PMFREQ, level=DEF_PMLEVEL, phase=DEF_PMPHASE, angle=DEF_PMANGLE,
       phase_r=DEF_PMPHASE, angle_r=DEF_PMANGLE, gain=DEF_GAIN_MOD):
    """PM node with the create_node_dsp defaults (adv_modulator.c:138-156)."""
    n = _base(abi.MODE_PM, inputs, gain)
    n.n_out = out if isinstance(out, int) else slot(out)
    n.pm_freq[0] = n.pm_freq[1] = freq
    n.pm_level[0] = n.pm_level[1] = level
    n.pm_phase[0], n.pm_phase[1] = phase, phase_r
    n.pm_angle[0], n.pm_angle[1] = angle, angle_r
    n.is_pm[0] = n.is_pm[1] = 1
    n.lock_freq, n.lock_phase, n.lock_level, n.lock_angle = 1, 0, 1, 0
    return n


def mix(inputs=("in",), out="Z", gain=DEF_GAIN_MOD):
    n = _base(abi.MODE_MIX, inputs, gain)
    n.n_out = out if isinstance(out, int) else slot(out)
    return n


def node_array(nodes):
    arr = (abi.Node * max(1, len(nodes)))()
    for i, n in enumerate(nodes):
        arr[i] = n
    return arr


# ---- the BASELINE.json graphs -------------------------------------------------
def graph_shift_master():
    """C1/C2: Shift(in -> A, +2/-2 Hz) + Master(A, S_ADD_REIM, 0.8).  Head first."""
    return [master(inputs=("A",)), shift(inputs=("in",), out="A")]


def graph_master_only():
    """C3/C5: Hilbert + Master only (default Master on `in`)."""
    return [master()]


def graph_pm_shift_mix():
    """C4: PM(in -> A, 4 Hz, L=0.5) -> Shift(A -> B) -> Mix(in + B -> C) -> Master(C).
    Executed tail -> head, so the list head-first is Master, Mix, Shift, PM."""
    return [master(inputs=("C",)), mix(inputs=("in", "B"), out="C"), shift(inputs=("A",), out="B"),
            pm(inputs=("in",), out="A")]


# ---- lists with one-frame delays (bus form, serial graph kernel) -----------------------------
def graph_pure_delay():
    """Master(B) <- Mix(A -> B) <- Shift(in -> A).  Executed tail -> head, the Mix runs first and
    reads A before the Shift writes it, so B is the shifted signal one frame late."""
    return [master(inputs=("B",)), shift(inputs=("in",), out="A"), mix(inputs=("A",), out="B")]


def graph_leaky_feedback():
    """C = 0.5 * (in + C[t-1]): a Mix node feeding itself, then Master(C)."""
    return [master(inputs=("C",)), mix(inputs=("in", "C"), out="C", gain=0.5)]


def graph_feedback_pm_shift():
    """PM and Shift inside a loop: A = PM(0.25 (in + B[t-1])); B = Shift(A); Master(in + B)."""
    return [master(inputs=("in", "B")), shift(inputs=("A",), out="B"), pm(inputs=("in", "B"), out="A", gain=0.25)]


def graph_long_chain(n=24):
    """More nodes than the register program holds: Master(X) <- n Mix hops from `in`."""
    slots = "ABCDEFGHIJKLMNOPQRSTUVWX"
    nodes = [master(inputs=("X",)), mix(inputs=(slots[n - 2],), out="X", gain=1.0)]
    for i in range(n - 2, 0, -1):
        nodes.append(mix(inputs=(slots[i - 1],), out=slots[i], gain=1.0))
    nodes.append(mix(inputs=("in",), out="A", gain=0.999))
    return nodes


def default_config(sample_rate=48000, fmt=abi.FMT_I16, channels=2, need24bits=False, hilbert_type=1):
    """load_config_default hot-path fields (config.c:153-207); NEED24BITS defaults to TRUE in the
    reference, the BASELINE configs C1-C4 use 16-bit output."""
    c = abi.Config()
    c.sample_rate = sample_rate
    c.in_format = fmt
    c.in_channels = channels
    c.hilbert_type = hilbert_type
    c.iir_kahan = 1
    c.iir_subnorm_reject = 1
    c.frmod_scaled = 1
    c.need24bits = 1 if need24bits else 0
    c.bypass_list = 0
    c.seed_left, c.seed_right = abi.SEED_LEFT, abi.SEED_RIGHT
    c.render.dth_bits = 1.0
    c.render.quantz_type = abi.QUANTZ_MID_RISER
    c.render.render_type = abi.RENDER_ROUND
    c.render.nshape_type = abi.NSHAPE_FLAT
    c.render.sign_bits16 = 16
    c.render.sign_bits24 = 24
    return c
