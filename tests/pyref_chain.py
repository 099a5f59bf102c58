"""Second, independent restatement of the whole per-frame chain in pure Python (test infrastructure).

Written from the reference's text, sharing no code with oracle/icw_oracle.c, and used only to
cross-check that oracle bit for bit on small inputs (tests/test_oracle_pyref.py).  Python floats
are IEEE binary64 without FMA contraction; math.sin / math.cos / math.fmod / math.log10 and
float.__pow__ are the platform libm's (glibc), the same functions the oracle links.

  unpack + fade        xwave_unpack_csample (xwave_reader.c:908-1001), unpackers (:205-239,
                       unpack_lsb.h:53-125), fade lengths (xwave_reader.c:712-725)
  Hilbert              tests/pyref_iir.py (hblpf.c, lpf_hilbert_quad.c)
  frame counter        amod_process_samples (adv_modulator.c:611-625)
  DSP list             adv_modulator.c:637-751 (mix, exchange, I/Q swap, gains, modes),
                       dsp_master / dsp_shift / dsp_pm (:485-583), amod_init (:216-331)
  render               sound_render_value (sound_render.c:691-809), sound_render_recalc
                       (:499-581), ns_empty / ns_fir / ns_iir (:396-489)
  MT19937              init_genrand / genrand_int32, dsemi / dsopen (mt_jrnd.c:28-47, 99-134,
                       218-256)

libm: the reference's `cos_v = cos(x); sin_v = sin(x);` pairs (adv_modulator.c:537-538, 573-574)
are one sincos(x) call in a gcc build (gcc merges them at -O1 and up), and glibc's sincos differs
from its separate sin / cos in ~0.1 % of arguments, so the pairs call libm's sincos through ctypes;
PM's inner sin (:569) is a lone sin() call, math.sin.
"""
import ctypes
import json
import math
import struct
from pathlib import Path

from pyref_iir import PyHilbert

_TABLES = json.loads((Path(__file__).resolve().parent / "golden" / "tables.json").read_text())
PI = 3.1415926535897932384626433832795029
SQRT2 = 1.4142135623730950488016887242097
SQRT6 = 2.4494897427831780981972840747059
ZERO_DB = -555.0
N_INPUTS = 27


_LIBM = ctypes.CDLL("libm.so.6")
_LIBM.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
_LIBM.sincos.restype = None


def _sincos(x):
    s, c = ctypes.c_double(), ctypes.c_double()
    _LIBM.sincos(x, ctypes.byref(s), ctypes.byref(c))
    return c.value, s.value


def _hex2d(h):
    return struct.unpack(">d", bytes.fromhex(h))[0]


# ------------------------------------------------------------------------------ MT19937 ----
class PyMT:
    def __init__(self, seed):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            p = self.mt[i - 1]
            self.mt[i] = (1812433253 * (p ^ (p >> 30)) + i) & 0xFFFFFFFF
        self.i = 624

    def u32(self):
        if self.i >= 624:
            mt = self.mt
            for k in range(624):
                y = (mt[k] & 0x80000000) | (mt[(k + 1) % 624] & 0x7FFFFFFF)
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y

    def dsemi(self):
        a = self.u32() >> 5
        b = self.u32() >> 6
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0)

    def dsopen(self):
        while True:
            r = self.dsemi() * 2.0 - 1.0
            if r != -1.0 and r != 1.0:
                return r


# ------------------------------------------------------------------------------ render -----
class PyRender:
    def __init__(self, rcfg, is24, seed):
        self.mt = PyMT(seed)
        self.rtype = rcfg.render_type
        self.dth_mul = 2.0 ** rcfg.dth_bits - 1.0
        self.prev_rnd = 0.0
        if rcfg.quantz_type == 0:             # mid tread
            self.round_offset, self.sign_delta = 0.5, 0
        else:
            self.round_offset, self.sign_delta = 0.0, -1
        self.is24 = is24
        if is24:
            self.norm_shift = 24 - rcfg.sign_bits24
            hib = 0x800000 >> self.norm_shift
            self.norm_mul = float(0x100 >> self.norm_shift) if self.norm_shift < 8 else \
                1.0 / float(1 << (self.norm_shift - 8))
        else:
            self.norm_shift = 16 - rcfg.sign_bits16
            hib = 0x8000 >> self.norm_shift
            self.norm_mul = 1.0 / float(1 << self.norm_shift)
        self.hi = float(hib)
        self.lo = -float(hib + 1 + self.sign_delta) - float(self.sign_delta)
        ns = rcfg.nshape_type if rcfg.nshape_type <= 17 else 0
        d = _TABLES["ns"][ns]
        self.ns_kind, self.ns_n = d["kind"], d["n"]
        self.ns_c = [_hex2d(h) for h in d["coeffs"]]
        self.eb = [0.0] * self.ns_n
        self.ob = [0.0] * self.ns_n
        self.ix = 0
        self.prev_ns_err = 0.0

    def _shape(self, v):
        if self.ns_kind == "flat":
            return 0.0
        n = self.ns_n
        self.ix = self.ix - 1 if self.ix else n - 1
        self.eb[self.ix] = v
        res = 0.0
        b = self.ix
        for k in range(n):
            if self.ns_kind == "fir":
                res += self.ns_c[k] * self.eb[b]
            else:
                res += self.ns_c[k] * self.eb[b] - self.ns_c[k + n] * self.ob[b]
            b = b + 1 if b + 1 < n else 0
        if self.ns_kind == "iir":
            self.ob[(self.ix if self.ix else n) - 1] = res
        return res

    def value(self, x, meters, ch):
        """-> output bytes of one sample; meters = {'clips': [l, r], 'peak': [l, r]}"""
        rnd = 0.0
        t = self.rtype
        if t == 1:
            rnd = self.mt.dsopen() / SQRT2
        elif t == 2:
            rnd = self.mt.dsopen()
            rnd += self.mt.dsopen()
            rnd /= 2.0
        elif t == 3:
            tr = self.mt.dsopen()
            rnd = (tr - self.prev_rnd) / 2.0
            self.prev_rnd = tr
        elif t == 4:
            rnd = self.mt.dsopen()
            for _ in range(11):
                rnd += self.mt.dsopen()
            rnd /= (2.0 * SQRT6)
        inp = (x * self.norm_mul) - self.prev_ns_err
        q = inp + (rnd * self.dth_mul)
        if q < 0.0:
            q -= self.round_offset
            delta = self.sign_delta
        else:
            q += self.round_offset
            delta = 0
        cv = abs(q) / self.hi
        cv = 20.0 * math.log10(cv) if cv else ZERO_DB
        if cv > meters["peak"][ch]:
            meters["peak"][ch] = cv
        if q >= self.hi:
            q = self.hi - 1.0
            meters["clips"][ch] += 1
        if q <= self.lo:
            q = self.lo + 1.0
            meters["clips"][ch] += 1
        iv = -2147483648 if math.isnan(q) else int(q)          # cvttsd2si: NaN -> INT_MIN
        val = ((iv + delta + 2 ** 31) % 2 ** 32) - 2 ** 31
        self.prev_ns_err = self._shape(float(val) - inp)
        val = (val << self.norm_shift) & 0xFFFFFFFF
        return bytes([val & 0xFF, (val >> 8) & 0xFF] + ([(val >> 16) & 0xFF] if self.is24 else []))


# ------------------------------------------------------------------------------ graph ------
def amod_init(nodes):
    """adv_modulator.c:216-331 on a copy: locks fanned out to the right channel; a list whose head
    is not the one Master (or with a bad mode) is replaced by the default Master.  -> (list, ok)"""
    import copy
    lst = [copy.copy(n) for n in nodes]
    ok = bool(lst) and lst[0].mode == 0
    seen_master = False
    for n in lst if ok else []:
        if n.lock_gain:
            n.gain[1] = n.gain[0]
            n.iq_invert[1] = n.iq_invert[0]
        if n.mode == 0:
            if seen_master:
                ok = False
            seen_master = True
        elif n.mode == 1:
            if n.lock_shift:
                n.fr_shift[1] = -n.fr_shift[0] if n.sign_lock_shift else n.fr_shift[0]
                n.is_shift[1] = n.is_shift[0]
        elif n.mode == 2:
            if n.lock_freq:
                n.pm_freq[1] = n.pm_freq[0]
                n.is_pm[1] = n.is_pm[0]
            if n.lock_phase:
                n.pm_phase[1] = n.pm_phase[0]
            if n.lock_level:
                n.pm_level[1] = n.pm_level[0]
            if n.lock_angle:
                n.pm_angle[1] = n.pm_angle[0]
        elif n.mode != 3:
            ok = False
        if not ok:
            break
    if ok:
        return lst, True
    from in_cwave_amd import abi
    m = abi.Node()
    m.mode = 0
    m.gain[0] = m.gain[1] = 0.8
    m.tout[0] = m.tout[1] = 0
    m.inputs[0] = 1
    m.lock_gain = 1
    return [m], False


def _master(tout, re, im):
    if tout == 2:
        return re
    if tout == 3:
        return im
    if tout == 0:
        return (re + im) / SQRT2
    if tout == 1:
        return (re - im) / SQRT2
    return 0.0


def _scaled(f):
    return float(int(f * 1000.0 + 0.5) & 0xFFFFFFFF)


def _shift(n, c, re, im, omega, scaled):
    if not n.is_shift[c]:
        return re, im
    f = n.fr_shift[c]
    neg = f < 0.0
    if neg:
        f = -f
    if scaled:
        f = _scaled(f)
    ph = math.fmod(omega * f, 2.0 * PI)
    cs, sn = _sincos(ph)
    if neg:
        sn = -sn
    return re * cs - im * sn, re * sn + im * cs


def _pm(n, c, re, im, omega, scaled):
    if not n.is_pm[c]:
        return re, im
    f = n.pm_freq[c]
    if scaled:
        f = _scaled(f)
    ph = math.fmod(omega * f, 2.0 * PI)
    psi = n.pm_level[c] * PI * (math.sin(ph + n.pm_phase[c] * PI) + n.pm_angle[c])
    cs, sn = _sincos(psi)
    return re * cs - im * sn, re * sn + im * cs


# ------------------------------------------------------------------------------ stream -----
_FMT = {0: 1, 1: 2, 2: 3, 3: 4, 4: 4}


def _unpack(b, fmt):
    if fmt == 0:
        return 256.0 * float(((b[0] - 0x80) & 0xFF) - (256 if ((b[0] - 0x80) & 0xFF) >= 128 else 0))
    if fmt == 1:
        return float(struct.unpack("<h", bytes(b[:2]))[0])
    if fmt == 2:
        v = b[0] | (b[1] << 8) | (b[2] << 16)
        return float(v - (1 << 24) if v & 0x800000 else v) / 256.0
    if fmt == 3:
        return float(struct.unpack("<i", bytes(b[:4]))[0]) / 65536.0
    return 32768.0 * float(struct.unpack("<f", bytes(b[:4]))[0])


class PyStream:
    """One stream: MOD_CONTEXT + reader position + the two renders, real (WAV) input."""

    def __init__(self, cfg, nodes):
        self.cfg = cfg
        self.nodes, self.accepted = amod_init(nodes)
        self.hl = PyHilbert(cfg.hilbert_type, cfg.iir_kahan, cfg.iir_subnorm_reject)
        self.hr = PyHilbert(cfg.hilbert_type, cfg.iir_kahan, cfg.iir_subnorm_reject)
        self.bus = [[0.0, 0.0, 0.0, 0.0] for _ in range(N_INPUTS)]
        self.n_frame = 0
        self.rl = PyRender(cfg.render, cfg.need24bits, cfg.seed_left)
        self.rr = PyRender(cfg.render, cfg.need24bits, cfg.seed_right)
        self.meters = {"clips": [0, 0], "peak": [ZERO_DB, ZERO_DB]}
        self.pos = 0
        self.n_samples, self.fin, self.fout = 1 << 62, 0, 0

    def open(self, n_samples, fade_in_ms=0, fade_out_ms=0):
        fs = self.cfg.sample_rate
        self.n_samples = n_samples
        self.fin, self.fout = fade_in_ms * fs // 1000, fade_out_ms * fs // 1000
        if self.fin + self.fout >= n_samples:
            if n_samples < 300:
                self.fin = self.fout = 0
            else:
                self.fin = n_samples // 3 if self.fin else 0
                self.fout = n_samples // 3 if self.fout else 0
        self.pos = 0

    def _fade(self, ix):
        if ix < self.fin:
            return float(ix) / float(self.fin)
        if self.n_samples - self.fout < ix < self.n_samples:
            return float(self.n_samples - ix) / float(self.fout)
        return -1.0

    def process(self, raw, n_frames):
        cfg = self.cfg
        csz = _FMT[cfg.in_format]
        fsz = csz * cfg.in_channels
        out = bytearray()
        pre = []
        raw = bytes(raw)
        scale_sr = cfg.sample_rate * 1000
        for t in range(n_frames):
            if cfg.frmod_scaled:
                omega = (2.0 * PI) * float(self.n_frame) / float(scale_sr)
                self.n_frame = (self.n_frame + 1) % scale_sr
            else:
                omega = (2.0 * PI) * float(self.n_frame) / float(cfg.sample_rate)
                self.n_frame += 1
            fb = raw[t * fsz:(t + 1) * fsz]
            fade = self._fade(self.pos)
            self.pos += 1
            v = _unpack(fb, cfg.in_format)
            if fade >= 0.0:
                v *= fade
            li, lq = self.hl.step(v)
            if cfg.in_channels > 1:
                v = _unpack(fb[csz:], cfg.in_format)
                if fade >= 0.0:
                    v *= fade
            ri, rq = self.hr.step(v)
            self.bus[0] = [li, lq, ri, rq]
            lout = rout = 0.0
            order = [0] if cfg.bypass_list else range(len(self.nodes) - 1, -1, -1)
            for k in order:
                n = self.nodes[k]
                if cfg.bypass_list:
                    d = list(self.bus[0])
                else:
                    d = [0.0, 0.0, 0.0, 0.0]
                    for s in range(N_INPUTS):
                        if n.inputs[s]:
                            b = self.bus[s]
                            d = [d[0] + b[0], d[1] + b[1], d[2] + b[2], d[3] + b[3]]
                x = n.xch_mode
                if x == 1:
                    d = [d[2], d[3], d[0], d[1]]
                elif x == 2:
                    d = [d[0], d[1], d[0], d[1]]
                elif x == 3:
                    d = [d[2], d[3], d[2], d[3]]
                elif x == 4:
                    mr, mi = (d[0] + d[2]) / 2.0, (d[1] + d[3]) / 2.0
                    d = [mr, mi, mr, mi]
                if n.iq_invert[0]:
                    d[0], d[1] = d[1], d[0]
                if n.iq_invert[1]:
                    d[2], d[3] = d[3], d[2]
                lg, rg = n.gain[0], n.gain[1]
                d = [d[0] * lg, d[1] * lg, d[2] * rg, d[3] * rg]
                if n.mode == 0:
                    lout = _master(n.tout[0], d[0], d[1])
                    rout = _master(n.tout[1], d[2], d[3])
                elif n.mode == 1:
                    self.bus[n.n_out] = [*_shift(n, 0, d[0], d[1], omega, cfg.frmod_scaled),
                                         *_shift(n, 1, d[2], d[3], omega, cfg.frmod_scaled)]
                elif n.mode == 2:
                    self.bus[n.n_out] = [*_pm(n, 0, d[0], d[1], omega, cfg.frmod_scaled),
                                         *_pm(n, 1, d[2], d[3], omega, cfg.frmod_scaled)]
                else:
                    self.bus[n.n_out] = d
            pre.append((lout, rout))
            out += self.rl.value(lout, self.meters, 0)
            out += self.rr.value(rout, self.meters, 1)
        return bytes(out), pre
