"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline; the product (in_cwave_amd) never does.
See icw_oracle.c for what the restatement follows (file:line) and its parity status.
"""
import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

from in_cwave_amd import abi

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = C.CDLL(str(LIB))
        vp = C.c_void_p
        lib.orc_stream_new.restype = vp
        lib.orc_stream_new.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.Node), C.c_int, C.POINTER(C.c_int)]
        lib.orc_stream_free.argtypes = [vp]
        lib.orc_set_input.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32]
        lib.orc_set_mt.argtypes = [vp, C.c_int, vp, C.c_int]
        lib.orc_stream_open.restype = C.c_int64
        lib.orc_stream_open.argtypes = [vp, C.c_int64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int]
        lib.orc_process.restype = C.c_int
        lib.orc_process.argtypes = [vp, vp, C.c_uint, vp, vp]
        lib.orc_process_many.restype = C.c_int
        lib.orc_process_many.argtypes = [C.POINTER(vp), C.c_int, vp, C.c_size_t, vp, C.c_size_t, C.c_uint]
        lib.orc_get_meters.argtypes = [vp, C.POINTER(abi.Meters)]
        lib.orc_get_fp_census.argtypes = [vp, C.POINTER(C.c_uint32)]
        lib.orc_stream_nframe.restype = C.c_uint64
        lib.orc_stream_nframe.argtypes = [vp]
        lib.orc_set_nframe.argtypes = [vp, C.c_uint64]
        lib.orc_iir_block.argtypes = [C.c_int, C.c_int, C.c_int, vp, C.c_int, vp, vp, C.POINTER(C.c_uint64)]
        lib.orc_iir_coeffs.restype = C.c_int
        lib.orc_iir_coeffs.argtypes = [C.c_int, vp, vp, C.POINTER(C.c_double)]
        lib.orc_hilbert_block.argtypes = [C.c_int, C.c_int, C.c_int, vp, C.c_int, vp, vp]
        lib.orc_render_block.argtypes = [C.POINTER(abi.RenderCfg), C.c_int, C.c_uint32, vp, C.c_int, vp, vp,
                                         C.POINTER(C.c_uint32), C.POINTER(C.c_double)]
        lib.orc_set_graph.restype = C.c_int
        lib.orc_set_graph.argtypes = [vp, C.POINTER(abi.Node), C.c_int, C.c_int]
        lib.orc_set_render.argtypes = [vp, C.POINTER(abi.RenderCfg)]
        lib.orc_set_outbits.argtypes = [vp, C.c_int]
        lib.orc_clear_inout.argtypes = [vp, C.c_int]
        lib.orc_share_meters.argtypes = [vp, vp]
        lib.orc_get_clips_peaks.argtypes = [vp, C.c_int, C.POINTER(abi.Meters)]
        lib.orc_del_lastdsp.argtypes = [vp]
        lib.orc_del_dsplist.argtypes = [vp]
        lib.orc_add_lastdsp.restype = C.c_int
        lib.orc_add_lastdsp.argtypes = [vp, C.POINTER(abi.Node)]
        lib.orc_set_output_plug.argtypes = [vp, C.c_int, C.c_int]
        lib.orc_set_hilbert_filter.argtypes = [vp, C.c_uint]
        lib.orc_set_hilbert_config.argtypes = [vp, C.c_int, C.c_int]
        lib.orc_set_fir.restype = C.c_int
        lib.orc_set_fir.argtypes = [vp, C.c_int, C.c_double]
        lib.orc_fir_taps.restype = C.c_int
        lib.orc_fir_taps.argtypes = [C.c_int, C.c_double, vp, C.c_int]
        lib.orc_mt_new.restype = vp
        lib.orc_mt_free.argtypes = [vp]
        lib.orc_mt_seed.argtypes = [vp, C.c_uint32]
        lib.orc_mt_init_key.argtypes = [vp, C.POINTER(C.c_uint32), C.c_uint32]
        for n in ("orc_mt_u32",):
            getattr(lib, n).restype = C.c_uint32
            getattr(lib, n).argtypes = [vp]
        for n in ("orc_mt_dsemi", "orc_mt_dsopen", "orc_mt_dlclosed", "orc_mt_dlsemi", "orc_mt_dclosed"):
            getattr(lib, n).restype = C.c_double
            getattr(lib, n).argtypes = [vp]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class Stream:
    """One reference-semantics stream (MOD_CONTEXT + reader position + renders)."""

    def __init__(self, cfg, nodes):
        lib = load()
        arr = (abi.Node * max(1, len(nodes)))(*nodes) if nodes else (abi.Node * 1)()
        acc = C.c_int()
        self.h = lib.orc_stream_new(C.byref(cfg), arr, len(nodes), C.byref(acc))
        self.accepted = bool(acc.value)
        self.cfg = cfg
        self.fsz = abi.FMT_BYTES[cfg.in_format] * cfg.in_channels
        self.osz = 2 * (3 if cfg.need24bits else 2)

    def __del__(self):
        try:
            load().orc_stream_free(self.h)
        except Exception:
            pass

    def set_mt(self, ch, words, idx):
        w = np.ascontiguousarray(words, dtype=np.uint32)
        load().orc_set_mt(self.h, ch, w.ctypes.data, idx)

    def set_fir(self, order, beta):
        """the FIR Hilbert converter (icw_set_fir_hilbert); order 0: the quadrature IIR"""
        if load().orc_set_fir(self.h, order, beta) != 0:
            raise ValueError("bad FIR order / beta")

    def set_graph(self, nodes, bypass_list=0):
        """live DSP-list edit (amod_add_lastdsp / amod_del_* / field writes); False if refused"""
        arr = (abi.Node * max(1, len(nodes)))(*nodes) if nodes else (abi.Node * 1)()
        return bool(load().orc_set_graph(self.h, arr, len(nodes), int(bypass_list)))

    def clear_bus_slot(self, slot):
        """mod_context_clear_all_inouts (in_cwave.c:255-261): bus slot `slot` to zero"""
        load().orc_clear_inout(self.h, int(slot))

    def del_lastdsp(self):
        """amod_del_lastdsp (adv_modulator.c:378-390), with replace_output_plug's clear"""
        load().orc_del_lastdsp(self.h)

    def del_dsplist(self):
        """amod_del_dsplist (adv_modulator.c:360-374)"""
        load().orc_del_dsplist(self.h)

    def add_lastdsp(self, node):
        """amod_add_lastdsp (adv_modulator.c:394-411) + the GUI's field writes; False if refused"""
        return bool(load().orc_add_lastdsp(self.h, C.byref(node)))

    def set_output_plug(self, index, n):
        """amod_set_output_plug (adv_modulator.c:436-441) on list node `index` (n = -1: clear only)"""
        load().orc_set_output_plug(self.h, int(index), int(n))

    def share_meters(self, owner):
        """render into owner's clips / peaks: the reference's one `am` accumulator that both decoding
        contexts feed (adv_modulator.c:54-55, 757-758); owner = self separates them again"""
        load().orc_share_meters(self.h, owner.h)
        self._meters_owner = owner           # keeps the accumulator's memory alive

    def clips_peaks(self, reset=False):
        """amod_get_clips_peaks (adv_modulator.c:445-465) of the accumulator this stream feeds"""
        m = abi.Meters()
        load().orc_get_clips_peaks(self.h, int(bool(reset)), C.byref(m))
        return {"clips": (m.clips[0], m.clips[1]), "peak_db": (m.peak_db[0], m.peak_db[1])}

    def set_render(self, render):
        """srenders_set_vcfg"""
        load().orc_set_render(self.h, C.byref(render))

    def set_hilbert_filter(self, type_):
        """mod_context_change_all_hilberts_filter"""
        load().orc_set_hilbert_filter(self.h, type_)

    def set_hilbert_config(self, kahan, subn):
        """mod_context_change_all_hilberts_config"""
        load().orc_set_hilbert_config(self.h, int(kahan), int(subn))

    def set_input(self, sample_rate, fmt, channels):
        load().orc_set_input(self.h, sample_rate, fmt, channels)
        self.fsz = abi.FMT_BYTES[fmt] * channels

    def set_outbits(self, need24bits):
        """sound_render_set_outbits on both renders (sound_render.c:617-621)"""
        load().orc_set_outbits(self.h, int(bool(need24bits)))
        self.osz = 2 * (3 if need24bits else 2)

    def open(self, n_samples, fade_in_ms=0, fade_out_ms=0, sec_align=0, clr_nframe=0, clr_hilb=0,
             need24bits=None):
        """mod_context_fopen (in_cwave.c:207-236).  need24bits: the.cfg.need24bits as the track opens,
        applied to both renders last (:233-234); None keeps the depth the stream has"""
        n_tail = load().orc_stream_open(self.h, n_samples, fade_in_ms, fade_out_ms, sec_align, clr_nframe,
                                        clr_hilb)
        if need24bits is not None:
            self.set_outbits(need24bits)
        return n_tail

    def process(self, raw, n_frames, want_pre=False):
        raw = np.ascontiguousarray(raw, dtype=np.uint8)
        assert raw.size >= n_frames * self.fsz
        out = np.zeros(n_frames * self.osz, dtype=np.uint8)
        pre = np.zeros((n_frames, 2), dtype=np.float64) if want_pre else None
        load().orc_process(self.h, _p(raw), n_frames, _p(out), _p(pre))
        return out, pre

    def meters(self):
        m = abi.Meters()
        load().orc_get_meters(self.h, C.byref(m))
        return {"clips": (m.clips[0], m.clips[1]), "peak_db": (m.peak_db[0], m.peak_db[1]),
                "desubnorm": m.desubnorm}

    def n_frame(self):
        return load().orc_stream_nframe(self.h)

    def set_n_frame(self, n):
        load().orc_set_nframe(self.h, n)

    def fp_census(self):
        """FP_EXCEPT_STATS [4, 7]: Hilbert L, R, render L, R (fp_check.h:62-72)"""
        buf = (C.c_uint32 * (4 * abi.FES_N))()
        load().orc_get_fp_census(self.h, buf)
        return np.frombuffer(bytes(buf), dtype=np.uint32).reshape(4, abi.FES_N).copy()


def iir_block(x, type_=1, kahan=1, subn=1):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros_like(x)
    w = np.zeros_like(x)
    cnt = C.c_uint64()
    load().orc_iir_block(type_, kahan, subn, _p(x), x.size, _p(y), _p(w), C.byref(cnt))
    return y, w, cnt.value


def iir_coeffs(type_):
    pc = np.zeros(20)
    pd = np.zeros(20)
    d0 = C.c_double()
    n = load().orc_iir_coeffs(type_, _p(pc), _p(pd), C.byref(d0))
    return pc[:n], pd[:n], d0.value


def hilbert_block(x, type_=1, kahan=1, subn=1):
    x = np.ascontiguousarray(x, dtype=np.float64)
    oi = np.zeros_like(x)
    oq = np.zeros_like(x)
    load().orc_hilbert_block(type_, kahan, subn, _p(x), x.size, _p(oi), _p(oq))
    return oi, oq


def render_block(x, cfg_render, is24=False, seed=abi.SEED_LEFT):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros(x.size * (3 if is24 else 2), dtype=np.uint8)
    iv = np.zeros(x.size, dtype=np.int32)
    clips = C.c_uint32()
    peak = C.c_double(abi.SR_ZERO_SIGNAL_DB)
    load().orc_render_block(C.byref(cfg_render), 1 if is24 else 0, seed, _p(x), x.size, _p(out), _p(iv),
                            C.byref(clips), C.byref(peak))
    return out, iv, clips.value, peak.value


class MT:
    def __init__(self, seed=None, key=None):
        self.lib = load()
        self.h = self.lib.orc_mt_new()
        if key is not None:
            k = (C.c_uint32 * len(key))(*key)
            self.lib.orc_mt_init_key(self.h, k, len(key))
        else:
            self.lib.orc_mt_seed(self.h, seed)

    def __del__(self):
        try:
            self.lib.orc_mt_free(self.h)
        except Exception:
            pass

    def u32(self):
        return self.lib.orc_mt_u32(self.h)

    def dsemi(self):
        return self.lib.orc_mt_dsemi(self.h)

    def dsopen(self):
        return self.lib.orc_mt_dsopen(self.h)


def fir_taps(order, beta):
    """the oracle's own taps g_m (m = 1, 3, ..) of the FIR Hilbert converter"""
    g = np.zeros((order // 2 + 1) // 2, dtype=np.float64)
    nt = load().orc_fir_taps(order, beta, g.ctypes.data, g.size)
    if nt < 0:
        raise ValueError("bad FIR order / beta")
    return g


def process_streams(cfg, nodes, raw, n_frames, want_pre=False, n_samples=None, census=None, fir=None):
    """Run every row of raw [S, bytes] through its own fresh oracle stream.  census (a list):
    receives each stream's FP-exception census [4, 7].  fir: (order, beta) of the FIR Hilbert
    converter."""
    outs, pres = [], []
    for s in range(raw.shape[0]):
        st = Stream(cfg, nodes)
        if fir:
            st.set_fir(*fir)
        if n_samples is not None:
            st.open(n_samples)
        o, p = st.process(raw[s], n_frames, want_pre)
        outs.append(o)
        pres.append(p)
        if census is not None:
            census.append(st.fp_census())
    return np.stack(outs), (np.stack(pres) if want_pre else None)
