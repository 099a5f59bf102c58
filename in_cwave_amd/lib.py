"""Loader for the in-tree HIP library in_cwave_amd/libicw.so and a thin Pythonic wrapper of the
C ABI (include/icw.h).  There is no CPU fallback: if the library or a HIP device is missing the
calls raise."""
import ctypes as C
import os
from pathlib import Path

import numpy as np

from . import abi

LIB_PATH = Path(__file__).resolve().parent / "libicw.so"
# A/B runs only: ICW_LIB=<name> loads in_cwave_amd/<name> (an alternative in-tree build) instead
if os.environ.get("ICW_LIB"):
    LIB_PATH = Path(__file__).resolve().parent / Path(os.environ["ICW_LIB"]).name
_lib = None


class IcwError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise IcwError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        # PyTorch-ROCm bundles its own HIP runtime; when both live in one process (torch tensors as
        # device buffers) torch's must come up first, or its later initialisation finds no GPU.
        try:
            import torch
            torch.cuda.is_available()
        except ImportError:
            pass
        lib = C.CDLL(str(LIB_PATH))
        for name, (res, args) in abi.SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                if os.environ.get("ICW_LIB"):      # an older A/B build may lack newer entry points
                    continue
                raise IcwError(f"{LIB_PATH} does not export {name}")
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _check(rc, what):
    if rc != abi.OK:
        msg = load().icw_strerror(rc).decode()
        raise IcwError(f"{what} failed: {rc} ({msg})")


def _ptr(x):
    """device/host pointer of a numpy array, torch tensor or int"""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(type(x))


class _HostBuffer:
    """owner of an icw_host_alloc block; freed when the last array view over it goes away"""

    def __init__(self, nbytes):
        p = C.c_void_p()
        _check(load().icw_host_alloc(nbytes, C.byref(p)), "icw_host_alloc")
        self.ptr = p.value

    def __del__(self):
        if self.ptr and _lib is not None:
            _lib.icw_host_free(self.ptr)
            self.ptr = None


class HostArray(np.ndarray):
    """a numpy array over an icw_host_alloc block; the block lives as long as the array or any view"""
    _icw_owner = None


def host_array(shape, dtype=np.uint8):
    """a numpy array in pinned host memory (icw_host_alloc): as a call's in / out buffer its copies
    run block by block beside the kernels"""
    dt = np.dtype(dtype)
    n = max(1, int(np.prod(shape)) * dt.itemsize)
    owner = _HostBuffer(n)
    buf = (C.c_uint8 * n).from_address(owner.ptr)
    a = np.frombuffer(buf, dtype=np.uint8, count=int(np.prod(shape)) * dt.itemsize).view(dt).reshape(shape)
    a = a.view(HostArray)
    a._icw_owner = owner
    return a


class Context:
    """One icw_ctx: n_streams streams sharing a config and a DSP list, state resident in HBM."""

    def __init__(self, cfg, nodes, n_streams, device=-1):
        lib = load()
        self._lib = lib
        arr = (abi.Node * max(1, len(nodes)))(*nodes) if nodes else (abi.Node * 1)()
        h = C.c_void_p()
        acc = C.c_int()
        _check(lib.icw_create(C.byref(cfg), arr, len(nodes), n_streams, device, C.byref(h), C.byref(acc)),
               "icw_create")
        self.h = h
        self.accepted = bool(acc.value)
        self.cfg = cfg
        self.n_streams = n_streams
        self.render_size = lib.icw_render_size(h)
        self.fsz = abi.FMT_BYTES[cfg.in_format] * cfg.in_channels

    def close(self):
        if self.h:
            self._lib.icw_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream_init(self, first=0, count=None):
        _check(self._lib.icw_stream_init(self.h, first, self.n_streams - first if count is None else count),
               "icw_stream_init")

    def set_input(self, sample_rate, fmt, channels):
        """a new track's sample format for every stream (icw_set_input)"""
        _check(self._lib.icw_set_input(self.h, sample_rate, fmt, channels), "icw_set_input")
        self.fsz = abi.FMT_BYTES[fmt] * channels

    def set_fir_hilbert(self, order, beta=8.0):
        """icw_set_fir_hilbert: real input through the FIR Hilbert converter (order k_M, Kaiser
        beta k_beta, cwave.h:56-58) instead of the quadrature IIR; order 0 restores the IIR"""
        _check(self._lib.icw_set_fir_hilbert(self.h, order, beta), "icw_set_fir_hilbert")

    def _own_cfg(self):
        """the live setters record the context's parameters in a copy, never in the caller's Config"""
        self.cfg = abi.Config.from_buffer_copy(self.cfg)

    def set_graph(self, nodes, bypass_list=0):
        """live DSP-list edit for the next calls (icw_set_graph); returns False when the list is
        one amod_init would reject (the running list stays)"""
        arr = (abi.Node * max(1, len(nodes)))(*nodes) if nodes else (abi.Node * 1)()
        acc = C.c_int()
        rc = self._lib.icw_set_graph(self.h, arr, len(nodes), int(bypass_list), C.byref(acc))
        if rc == abi.EGRAPH:
            return False
        _check(rc, "icw_set_graph")
        self._own_cfg()
        self.cfg.bypass_list = int(bool(bypass_list))
        return True

    def clear_bus_slot(self, slot):
        """mod_context_clear_all_inouts for every stream (icw_clear_bus_slot): slot 0..26 to zero"""
        _check(self._lib.icw_clear_bus_slot(self.h, int(slot)), "icw_clear_bus_slot")

    def graph_del_last(self):
        """amod_del_lastdsp (icw_graph_del_last): the tail goes, its output slot is cleared"""
        _check(self._lib.icw_graph_del_last(self.h), "icw_graph_del_last")

    def graph_del_all(self):
        """amod_del_dsplist (icw_graph_del_all): every node but the Master, each slot cleared"""
        _check(self._lib.icw_graph_del_all(self.h), "icw_graph_del_all")

    def graph_add_last(self, node):
        """amod_add_lastdsp + the GUI's field writes (icw_graph_add_last); False if refused"""
        rc = self._lib.icw_graph_add_last(self.h, C.byref(node))
        if rc == abi.EGRAPH:
            return False
        _check(rc, "icw_graph_add_last")
        return True

    def graph_set_output_plug(self, index, n):
        """amod_set_output_plug (icw_graph_set_output_plug): node `index`'s slot to n (-1: clear only)"""
        _check(self._lib.icw_graph_set_output_plug(self.h, int(index), int(n)), "icw_graph_set_output_plug")

    def prepare(self, n_frames=0):
        """icw_prepare: warm a fresh context (one call of silence, then the fresh state back)"""
        _check(self._lib.icw_prepare(self.h, int(n_frames)), "icw_prepare")

    def set_render(self, render):
        """srenders_set_vcfg for every stream (icw_set_render): an abi.RenderCfg"""
        _check(self._lib.icw_set_render(self.h, C.byref(render)), "icw_set_render")
        self._own_cfg()
        self.cfg.render = render

    def set_outbits(self, need24bits):
        """sound_render_set_outbits for every stream (icw_set_outbits): 16 or 24 output bits"""
        _check(self._lib.icw_set_outbits(self.h, int(bool(need24bits))), "icw_set_outbits")
        self._own_cfg()
        self.cfg.need24bits = int(bool(need24bits))
        self.render_size = self._lib.icw_render_size(self.h)

    def set_hilbert_filter(self, type_):
        """mod_context_change_all_hilberts_filter (icw_set_hilbert_filter)"""
        _check(self._lib.icw_set_hilbert_filter(self.h, type_), "icw_set_hilbert_filter")
        self._own_cfg()
        self.cfg.hilbert_type = type_

    def set_hilbert_config(self, kahan, subnorm_reject):
        """mod_context_change_all_hilberts_config (icw_set_hilbert_config)"""
        _check(self._lib.icw_set_hilbert_config(self.h, int(kahan), int(subnorm_reject)), "icw_set_hilbert_config")
        self._own_cfg()
        self.cfg.iir_kahan, self.cfg.iir_subnorm_reject = int(bool(kahan)), int(bool(subnorm_reject))

    def stream_open(self, s, n_samples, fade_in_ms=0, fade_out_ms=0, sec_align=0, clr_nframe=0, clr_hilb=0):
        _check(self._lib.icw_stream_open(self.h, s, n_samples, fade_in_ms, fade_out_ms, sec_align,
                                         clr_nframe, clr_hilb), "icw_stream_open")

    def process(self, inp, n_frames, first=0, count=None, want_pre=False, out=None):
        """Host numpy path: inp uint8 [count, >= n_frames*fsz]; returns (out uint8 [count, n_frames*2*rs],
        pre float64 [count, n_frames, 2] or None).  out: a preallocated output array (reused)."""
        count = self.n_streams - first if count is None else count
        inp = np.ascontiguousarray(inp)
        assert inp.dtype == np.uint8 and inp.shape[0] == count and inp.shape[1] >= n_frames * self.fsz
        osz = 2 * self.render_size
        if out is None:
            out = np.zeros((count, n_frames * osz), dtype=np.uint8)
        assert out.dtype == np.uint8 and out.flags.c_contiguous and out.shape[0] == count
        assert out.shape[1] >= n_frames * osz
        pre = np.zeros((count, n_frames, 2), dtype=np.float64) if want_pre else None
        flags = abi.F_DEBUG_PRE if want_pre else 0
        # a length-1 leading axis may carry stride 0 (x[None, :]): the row length is the stride then
        in_stride = inp.strides[0] if count > 1 else inp.shape[1]
        _check(self._lib.icw_process_streams(self.h, first, count, _ptr(inp), in_stride, _ptr(out),
                                             out.strides[0], n_frames, flags, _ptr(pre), None),
               "icw_process_streams")
        return out, pre

    def unpacked_input(self, inp, n_frames, first=0, count=None):
        """Test hook (ICW_F_DEBUG_INPUT): process like `process` and return float64 [count, n_frames, 2],
        the unpacked, faded samples K0 hands the Hilbert converters (pre-Hilbert, R = L for mono)"""
        count = self.n_streams - first if count is None else count
        inp = np.ascontiguousarray(inp)
        assert inp.dtype == np.uint8 and inp.shape[0] == count and inp.shape[1] >= n_frames * self.fsz
        out = np.zeros((count, n_frames * 2 * self.render_size), dtype=np.uint8)
        x = np.zeros((count, n_frames, 2), dtype=np.float64)
        in_stride = inp.strides[0] if count > 1 else inp.shape[1]
        _check(self._lib.icw_process_streams(self.h, first, count, _ptr(inp), in_stride, _ptr(out), out.strides[0],
                                             n_frames, abi.F_DEBUG_INPUT, _ptr(x), None), "icw_process_streams")
        return x, out

    def process_device(self, d_in, in_stride, d_out, out_stride, n_frames, first=0, count=None,
                       timing=False, hip_stream=None):
        count = self.n_streams - first if count is None else count
        flags = abi.F_DEVICE_PTRS | (abi.F_TIMING if timing else 0)
        _check(self._lib.icw_process_streams(self.h, first, count, _ptr(d_in), in_stride, _ptr(d_out),
                                             out_stride, n_frames, flags, None, hip_stream),
               "icw_process_streams")

    def synchronize(self):
        _check(self._lib.icw_synchronize(self.h), "icw_synchronize")

    def meters(self, s, reset=False):
        m = abi.Meters()
        _check(self._lib.icw_get_meters(self.h, s, 1 if reset else 0, C.byref(m)), "icw_get_meters")
        return {"clips": (m.clips[0], m.clips[1]), "peak_db": (m.peak_db[0], m.peak_db[1]),
                "desubnorm": m.desubnorm}

    def n_frame(self, s):
        v = C.c_uint64()
        _check(self._lib.icw_n_frame(self.h, s, C.byref(v)), "icw_n_frame")
        return v.value

    def get_state(self, s):
        n = self._lib.icw_state_size(self.h)
        buf = (C.c_uint8 * n)()
        _check(self._lib.icw_get_state(self.h, s, buf, n), "icw_get_state")
        return bytes(buf)

    def set_state(self, s, blob):
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        _check(self._lib.icw_set_state(self.h, s, buf, len(blob)), "icw_set_state")

    def fp_census(self, s, reset=False):
        """icw_get_fp_census: uint32 [4, 7] (Hilbert L, R, render L, R) x (total, snan, qnan, ninf,
        nden, pden, pinf)"""
        buf = (C.c_uint32 * (4 * abi.FES_N))()
        _check(self._lib.icw_get_fp_census(self.h, s, 1 if reset else 0, buf), "icw_get_fp_census")
        return np.frombuffer(bytes(buf), dtype=np.uint32).reshape(4, abi.FES_N).copy()

    def last_k1_kernel(self):
        """ICW_K1_* of the last real-input call: 0 lane-per-chain, 1 pair, 2 MFMA, 3 row broadcast"""
        return int(self._lib.icw_last_k1_kernel(self.h))

    def last_timing(self):
        ms = (C.c_double * 2)()
        n = (C.c_int * 2)()
        _check(self._lib.icw_last_timing(self.h, ms, n), "icw_last_timing")
        return (ms[0], ms[1]), (n[0], n[1])


def fir_taps(order, beta=8.0):
    """icw_fir_taps: the converter's taps g_m, m = 1, 3, .. (host arithmetic, no device call)"""
    g = np.zeros((order // 2 + 1) // 2, dtype=np.float64)
    nt = load().icw_fir_taps(order, beta, _ptr(g), g.size)
    if nt < 0:
        _check(nt, "icw_fir_taps")
    return g


# ------------------------------------------------------------------ CWAVE files / CRC-32 -------
def cwave_parse(header, file_size):
    """icw_cwave_parse: the reference's CWAVE header checks (xwave_reader.c:243-300).  Returns
    (header struct, ICW_FMT_CW_* format, frame bytes); raises IcwError for a refused file."""
    lib = load()
    b = np.frombuffer(bytes(header[:abi.CWAVE_HEADER_BYTES]), dtype=np.uint8).copy()
    h = abi.CwaveHeader()
    fmt, fb = C.c_uint32(), C.c_uint32()
    _check(lib.icw_cwave_parse(_ptr(b), b.size, file_size, C.byref(h), C.byref(fmt), C.byref(fb)), "icw_cwave_parse")
    return h, fmt.value, fb.value


def crc32_batch(base, offsets, lengths, crc_in=None, device_ptrs=False, device=-1, hip_stream=None):
    """icw_crc32_batch: CRC-32 (crc32.c) of the byte ranges [base+offsets[i], +lengths[i]) on the
    GPU.  base: numpy uint8 array (host) or a torch uint8 CUDA tensor / int pointer (device_ptrs)."""
    lib = load()
    n = len(offsets)
    off = (C.c_uint64 * max(1, n))(*[int(v) for v in offsets])
    ln = (C.c_uint64 * max(1, n))(*[int(v) for v in lengths])
    cin = (C.c_uint32 * max(1, n))(*[int(v) for v in crc_in]) if crc_in is not None else None
    out = (C.c_uint32 * max(1, n))()
    flags = abi.F_DEVICE_PTRS if device_ptrs else 0
    _check(lib.icw_crc32_batch(_ptr(base), off, ln, n, cin, out, flags, device, hip_stream), "icw_crc32_batch")
    return [int(out[i]) for i in range(n)]


def crc32_combine(crc_a, crc_b, len_b):
    return int(load().icw_crc32_combine(crc_a, crc_b, len_b))


def cwave_check(image, device_ptrs=False, device=-1, size=None):
    """icw_cwave_check: (crc, ok) with ok 1 / 0, or -1 for a V1 file without a stored CRC"""
    lib = load()
    size = image.numel() if hasattr(image, "numel") else (len(image) if size is None else size)
    crc, ok = C.c_uint32(), C.c_int()
    _check(lib.icw_cwave_check(_ptr(image), size, abi.F_DEVICE_PTRS if device_ptrs else 0, device,
                               C.byref(crc), C.byref(ok)), "icw_cwave_check")
    return crc.value, ok.value


# ------------------------------------------------------------------ in_cwave.cfg ingestion -----
def config_load(text, sample_rate=48000, fmt=abi.FMT_I16, channels=2):
    """icw_config_load on the text of an in_cwave.cfg (load_config, config.c:813-915).
    Returns (ok, FileConfig, bad_line); on failure the FileConfig holds the defaults, as the
    reference falls back to them."""
    data = text.encode() if isinstance(text, str) else bytes(text)
    fc = abi.FileConfig()
    fc.cfg.sample_rate, fc.cfg.in_format, fc.cfg.in_channels = sample_rate, fmt, channels
    bad = C.c_int()
    rc = load().icw_config_load(data, len(data), C.byref(fc), C.byref(bad))
    return rc == abi.OK, fc, bad.value


def config_nodes(fc):
    """the DSP list of a loaded config, head first, as icw_create takes it"""
    return [fc.nodes[i] for i in range(fc.n_nodes)]


def node_dsp_parse(args):
    n = abi.Node()
    name = C.create_string_buffer(abi.DSP_NAME_SIZE)
    _check(load().icw_node_dsp_parse(args.encode() if isinstance(args, str) else args, C.byref(n), name,
                                     abi.DSP_NAME_SIZE), "icw_node_dsp_parse")
    return n, name.value.decode(errors="replace")


def node_dsp_format(node, name=""):
    buf = C.create_string_buffer(4096)
    k = load().icw_node_dsp_format(C.byref(node), name.encode(), buf, 4096)
    if k < 0:
        _check(k, "icw_node_dsp_format")
    return buf.value.decode()


# ------------------------------------------------------------------ WAV / CWAVE files ---------
def wav_parse_file(path):
    """icw_wav_parse_file: the reference's reader acceptance (xwave_reader_create); raises for a
    refused file"""
    info = abi.WavInfo()
    _check(load().icw_wav_parse_file(str(path).encode(), C.byref(info)), "icw_wav_parse_file")
    return info


def transcode_files(cfg, nodes, in_paths, out_paths, fade_in_ms=0, fade_out_ms=0, sec_align=0,
                    block_frames=0, device=-1):
    """icw_transcode_files: many files through the GPU path; returns (stats, per-file status)"""
    n = len(in_paths)
    ins = (C.c_char_p * max(1, n))(*[str(p).encode() for p in in_paths])
    outs = (C.c_char_p * max(1, n))(*[str(p).encode() for p in out_paths])
    arr = graph_nodes(nodes)
    o = abi.BatchOpts(fade_in_ms, fade_out_ms, sec_align, block_frames, device, 0)
    st = abi.BatchStats()
    status = (C.c_int * max(1, n))()
    rc = load().icw_transcode_files(C.byref(cfg), arr, len(nodes), ins, outs, n, C.byref(o), C.byref(st), status)
    return rc, st, [status[i] for i in range(n)]


def transcode_files_devices(cfg, nodes, in_paths, out_paths, devices, fade_in_ms=0, fade_out_ms=0, sec_align=0,
                            block_frames=0):
    """icw_transcode_files_devices: the files split over `devices` (one host thread each)"""
    n = len(in_paths)
    ins = (C.c_char_p * max(1, n))(*[str(p).encode() for p in in_paths])
    outs = (C.c_char_p * max(1, n))(*[str(p).encode() for p in out_paths])
    arr = graph_nodes(nodes)
    o = abi.BatchOpts(fade_in_ms, fade_out_ms, sec_align, block_frames, -1, 0)
    dv = (C.c_int * len(devices))(*devices)
    st = abi.BatchStats()
    status = (C.c_int * max(1, n))()
    rc = load().icw_transcode_files_devices(C.byref(cfg), arr, len(nodes), ins, outs, n, C.byref(o), dv,
                                            len(devices), C.byref(st), status)
    return rc, st, [status[i] for i in range(n)]


class Group:
    """icw_group: n_streams streams sharded over several devices, one context and one host
    thread per device (include/icw_group.h)"""

    def __init__(self, cfg, nodes, n_streams, devices):
        lib = load()
        self._lib = lib
        arr = graph_nodes(nodes)
        dv = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        acc = C.c_int()
        _check(lib.icw_group_create(C.byref(cfg), arr, len(nodes), n_streams, dv, len(devices), C.byref(h),
                                    C.byref(acc)), "icw_group_create")
        self.h, self.accepted, self.n_streams = h, bool(acc.value), n_streams
        self.fsz = abi.FMT_BYTES[cfg.in_format] * cfg.in_channels
        self.osz = 2 * (3 if cfg.need24bits else 2)

    def close(self):
        if self.h:
            self._lib.icw_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def shard(self, d):
        f, c, dev, ctx = C.c_int(), C.c_int(), C.c_int(), C.c_void_p()
        _check(self._lib.icw_group_shard(self.h, d, C.byref(f), C.byref(c), C.byref(dev), C.byref(ctx)),
               "icw_group_shard")
        return f.value, c.value, dev.value

    def process(self, inp, n_frames, want_pre=False, out=None):
        """out: an optional [n_streams, >= n_frames * osz] uint8 array (e.g. host_array: pinned, so every
        shard copies its slices block by block on its own device)"""
        inp = np.ascontiguousarray(inp)
        assert inp.dtype == np.uint8 and inp.shape[0] == self.n_streams and inp.shape[1] >= n_frames * self.fsz
        if out is None:
            out = np.zeros((self.n_streams, n_frames * self.osz), dtype=np.uint8)
        assert out.dtype == np.uint8 and out.shape[0] == self.n_streams and out.shape[1] >= n_frames * self.osz
        pre = np.zeros((self.n_streams, n_frames, 2), dtype=np.float64) if want_pre else None
        _check(self._lib.icw_group_process(self.h, _ptr(inp), inp.strides[0], _ptr(out), out.strides[0], n_frames,
                                           abi.F_DEBUG_PRE if want_pre else 0, _ptr(pre)), "icw_group_process")
        return out, pre

    def meters(self, s, reset=False):
        m = abi.Meters()
        _check(self._lib.icw_group_get_meters(self.h, s, 1 if reset else 0, C.byref(m)), "icw_group_get_meters")
        return {"clips": (m.clips[0], m.clips[1]), "peak_db": (m.peak_db[0], m.peak_db[1]),
                "desubnorm": m.desubnorm}

    def n_frame(self, s):
        v = C.c_uint64()
        _check(self._lib.icw_group_n_frame(self.h, s, C.byref(v)), "icw_group_n_frame")
        return v.value


def graph_nodes(nodes):
    arr = (abi.Node * max(1, len(nodes)))()
    for i, nd in enumerate(nodes):
        arr[i] = nd
    return arr
