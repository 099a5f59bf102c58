"""ctypes mirror of include/icw.h (the C ABI).  Kept field-for-field identical to the header;
tests/test_abi.py checks sizes/offsets against the header's layout rules."""
import ctypes as C

N_INPUTS = 27
MAX_IIR_ORDER = 20

# status codes
OK, EINVAL, ENOMEM, EDEVICE, EGRAPH, EUNSUPPORTED = 0, -1, -2, -3, -4, -5

# node modes / master outputs / channel exchange (in_cwave.h:152-287)
MODE_MASTER, MODE_SHIFT, MODE_PM, MODE_MIX = 0, 1, 2, 3
S_ADD_REIM, S_SUB_REIM, S_RE, S_IM = 0, 1, 2, 3
XCH_NORMAL, XCH_SWAP, XCH_LEFTONLY, XCH_RIGHTONLY, XCH_MIXLR = 0, 1, 2, 3, 4
# input formats (HRW_FMT_*)
FMT_U8, FMT_I16, FMT_I24, FMT_I32, FMT_F32 = 0, 1, 2, 3, 4
K1_LANE, K1_ROW, K1_FC = 0, 3, 4      # icw_last_k1_kernel (include/icw.h)
FES_N = 7     # FP_EXCEPT_STATS counters: total, snan, qnan, ninf, nden, pden, pinf
# complex CWAVE formats: ICW_FMT_CW_F64 + HCW_FMT_* (cwave.h:70-80), Hilbert bypassed
FMT_CW_F64, FMT_CW_I16, FMT_CW_I16_F32, FMT_CW_F32 = 5, 6, 7, 8
FMT_BYTES = {FMT_U8: 1, FMT_I16: 2, FMT_I24: 3, FMT_I32: 4, FMT_F32: 4,
             FMT_CW_F64: 16, FMT_CW_I16: 4, FMT_CW_I16_F32: 6, FMT_CW_F32: 8}
CW_FORMATS = (FMT_CW_F64, FMT_CW_I16, FMT_CW_I16_F32, FMT_CW_F32)
# render (sound_render.h)
QUANTZ_MID_TREAD, QUANTZ_MID_RISER = 0, 1
RENDER_ROUND, RENDER_RPDF, RENDER_TPDF, RENDER_STPDF, RENDER_GAUSS = 0, 1, 2, 3, 4
NSHAPE_FLAT, NSHAPE_FW44, NSHAPE_MEW44 = 0, 1, 2
NSHAPE_MAX = 17
SEED_LEFT, SEED_RIGHT = 0x13579BDF, 0x479B22AB
SR_ZERO_SIGNAL_DB = -555.0

F_DEVICE_PTRS, F_DEBUG_PRE, F_TIMING, F_DEBUG_INPUT = 1, 2, 4, 8


class Node(C.Structure):
    _fields_ = [
        ("mode", C.c_int32), ("n_out", C.c_int32),
        ("gain", C.c_double * 2),
        ("inputs", C.c_uint8 * N_INPUTS), ("pad_", C.c_uint8 * 1),
        ("xch_mode", C.c_int32), ("iq_invert", C.c_int32 * 2),
        ("tout", C.c_int32 * 2),
        ("fr_shift", C.c_double * 2), ("is_shift", C.c_int32 * 2),
        ("pm_freq", C.c_double * 2), ("pm_phase", C.c_double * 2),
        ("pm_level", C.c_double * 2), ("pm_angle", C.c_double * 2),
        ("is_pm", C.c_int32 * 2),
        ("lock_gain", C.c_int32), ("lock_shift", C.c_int32), ("sign_lock_shift", C.c_int32),
        ("lock_freq", C.c_int32), ("lock_phase", C.c_int32), ("lock_level", C.c_int32),
        ("lock_angle", C.c_int32), ("reserved_", C.c_int32),
    ]


class RenderCfg(C.Structure):
    _fields_ = [("dth_bits", C.c_double), ("quantz_type", C.c_uint32), ("render_type", C.c_uint32),
                ("nshape_type", C.c_uint32), ("sign_bits16", C.c_uint32), ("sign_bits24", C.c_uint32)]


class Config(C.Structure):
    _fields_ = [
        ("sample_rate", C.c_uint32), ("in_format", C.c_uint32), ("in_channels", C.c_uint32),
        ("hilbert_type", C.c_uint32), ("iir_kahan", C.c_int32), ("iir_subnorm_reject", C.c_int32),
        ("frmod_scaled", C.c_int32), ("need24bits", C.c_int32), ("bypass_list", C.c_int32),
        ("seed_left", C.c_uint32), ("seed_right", C.c_uint32),
        ("render", RenderCfg),
        ("fp_check", C.c_int32),
    ]


class Meters(C.Structure):
    _fields_ = [("clips", C.c_uint32 * 2), ("peak_db", C.c_double * 2), ("desubnorm", C.c_uint64)]


class CwaveHeader(C.Structure):
    """icw_cwave_header (include/icw_cwave.h) = HCWAVE_V2 (cwave.h:48-60)"""
    _fields_ = [("magic", C.c_char * 8), ("hsize", C.c_uint32), ("version", C.c_uint32), ("format", C.c_uint32),
                ("n_channels", C.c_uint32), ("n_samples", C.c_uint32), ("sample_rate", C.c_uint32),
                ("k_M", C.c_int32), ("n_crc32", C.c_uint32), ("k_beta", C.c_double)]


CWAVE_HEADER_BYTES = 48

CFG_VERSION = 10
CFG_MAX_NODES = 64
DSP_NAME_SIZE = 96


class FileConfig(C.Structure):
    """icw_file_config (include/icw_config.h): what an in_cwave.cfg defines"""
    _fields_ = [("cfg", Config), ("sec_align", C.c_uint32), ("fade_in", C.c_uint32), ("fade_out", C.c_uint32),
                ("clr_nframe", C.c_int32), ("clr_hilb", C.c_int32), ("subnorm_thr", C.c_double),
                ("fp_check", C.c_int32), ("ver_config", C.c_uint32), ("n_nodes", C.c_int32),
                ("nodes", Node * CFG_MAX_NODES), ("names", (C.c_char * DSP_NAME_SIZE) * CFG_MAX_NODES)]

HTYPE_WFONLY, HTYPE_PCMW, HTYPE_EXT, HTYPE_CWAVE = 0, 1, 2, 3
RSTATE = 42


class StateBlob(C.Structure):
    """the per-stream state blob of icw_get_state / icw_set_state"""
    _fields_ = [("magic", C.c_uint64), ("n_frame", C.c_uint64), ("pos", C.c_int64), ("n_samples", C.c_int64),
                ("n_fade_in", C.c_int64), ("n_fade_out", C.c_int64), ("hq_phase", C.c_uint32 * 2),
                ("nord", C.c_uint32), ("has_render", C.c_uint32), ("fir_M", C.c_uint32), ("reserved", C.c_uint32),
                ("hist", (C.c_double * 20) * 4),
                ("sncnt", C.c_uint64 * 4), ("bus", (C.c_double * 4) * N_INPUTS),
                ("mt", (C.c_uint32 * 624) * 2), ("mt_idx", C.c_int32 * 2), ("rs", (C.c_double * RSTATE) * 2)]


class WavInfo(C.Structure):
    """icw_wav_info (include/icw_reader.h)"""
    _fields_ = [("fmt", C.c_uint32), ("channels", C.c_uint32), ("sample_rate", C.c_uint32),
                ("frame_bytes", C.c_uint32), ("n_samples", C.c_int64), ("data_offset", C.c_int64),
                ("htype", C.c_uint32), ("reserved_", C.c_uint32)]


class BatchOpts(C.Structure):
    _fields_ = [("fade_in_ms", C.c_uint32), ("fade_out_ms", C.c_uint32), ("sec_align", C.c_uint32),
                ("block_frames", C.c_int32), ("device", C.c_int32), ("reserved_", C.c_int32)]


class BatchStats(C.Structure):
    _fields_ = [("n_files", C.c_int32), ("n_groups", C.c_int32), ("frames_in", C.c_uint64),
                ("frames_out", C.c_uint64), ("wall_s", C.c_double), ("io_s", C.c_double)]


# every function declared in include/icw.h, icw_amod.h, icw_cwave.h: name -> (restype, argtypes)
_vp, _sz, _i, _u = C.c_void_p, C.c_size_t, C.c_int, C.c_uint
SIGNATURES = {
    "icw_create": (_i, [C.POINTER(Config), C.POINTER(Node), _i, _i, _i, C.POINTER(_vp), C.POINTER(_i)]),
    "icw_destroy": (_i, [_vp]),
    "icw_stream_init": (_i, [_vp, _i, _i]),
    "icw_stream_open": (_i, [_vp, _i, C.c_int64, C.c_uint32, C.c_uint32, C.c_uint32, _i, _i]),
    "icw_stream_reset_hilbert": (_i, [_vp, _i]),
    "icw_stream_reset_framecnt": (_i, [_vp, _i]),
    "icw_stream_seek": (_i, [_vp, _i, C.c_int64]),
    "icw_set_input": (_i, [_vp, C.c_uint32, C.c_uint32, C.c_uint32]),
    "icw_set_fir_hilbert": (_i, [_vp, C.c_int32, C.c_double]),
    "icw_set_graph": (_i, [_vp, C.POINTER(Node), _i, _i, C.POINTER(_i)]),
    "icw_set_render": (_i, [_vp, C.POINTER(RenderCfg)]),
    "icw_set_outbits": (_i, [_vp, _i]),
    "icw_clear_bus_slot": (_i, [_vp, _i]),
    "icw_graph_del_last": (_i, [_vp]),
    "icw_graph_del_all": (_i, [_vp]),
    "icw_graph_add_last": (_i, [_vp, C.POINTER(Node)]),
    "icw_graph_set_output_plug": (_i, [_vp, _i, _i]),
    "icw_prepare": (_i, [_vp, _i]),
    "icw_set_hilbert_filter": (_i, [_vp, C.c_uint32]),
    "icw_set_hilbert_config": (_i, [_vp, _i, _i]),
    "icw_fir_taps": (_i, [C.c_int32, C.c_double, _vp, C.c_int]),
    "icw_mod_context_create": (_vp, [C.POINTER(Config), C.POINTER(Node), _i, _i, C.POINTER(_i)]),
    "icw_mod_context_destroy": (None, [_vp]),
    "icw_mod_context_ctx": (_vp, [_vp]),
    "icw_mod_context_fopen": (_i, [_vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int64, C.c_uint32, C.c_uint32,
                                   C.c_uint32, _i, _i, _i]),
    "icw_amod_process_samples": (_i, [_vp, _vp, _vp, _u]),
    "icw_mod_context_seek": (_i, [_vp, C.c_int64, _i]),
    "icw_mod_context_out_size": (_i, [_vp]),
    "icw_mod_context_meters": (_i, [_vp, _i, C.POINTER(Meters)]),
    "icw_amod_get_clips_peaks": (_i, [C.POINTER(_vp), _i, C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                                      C.POINTER(C.c_double), C.POINTER(C.c_double), _i]),
    "icw_amod_del_lastdsp": (_i, [C.POINTER(_vp), _i]),
    "icw_amod_del_dsplist": (_i, [C.POINTER(_vp), _i]),
    "icw_amod_add_lastdsp": (_i, [C.POINTER(_vp), _i, C.POINTER(Node)]),
    "icw_amod_set_output_plug": (_i, [C.POINTER(_vp), _i, _i, _i]),
    "icw_process_batch": (_i, [_vp, _vp, _sz, _vp, _sz, _i, _u, _vp, _vp]),
    "icw_process_streams": (_i, [_vp, _i, _i, _vp, _sz, _vp, _sz, _i, _u, _vp, _vp]),
    "icw_synchronize": (_i, [_vp]),
    "icw_host_alloc": (_i, [C.c_size_t, C.POINTER(_vp)]),
    "icw_host_free": (_i, [_vp]),
    "icw_host_pinned": (_i, [_vp, _i]),
    "icw_get_meters": (_i, [_vp, _i, _i, C.POINTER(Meters)]),
    "icw_render_size": (_i, [_vp]),
    "icw_n_frame": (_i, [_vp, _i, C.POINTER(C.c_uint64)]),
    "icw_state_size": (_sz, [_vp]),
    "icw_get_state": (_i, [_vp, _i, _vp, _sz]),
    "icw_set_state": (_i, [_vp, _i, _vp, _sz]),
    "icw_last_timing": (_i, [_vp, C.POINTER(C.c_double), C.POINTER(_i)]),
    "icw_last_k1_kernel": (_i, [_vp]),
    "icw_get_fp_census": (_i, [_vp, _i, _i, C.POINTER(C.c_uint32)]),
    "icw_cwave_parse": (_i, [_vp, _sz, C.c_int64, C.POINTER(CwaveHeader), C.POINTER(C.c_uint32),
                             C.POINTER(C.c_uint32)]),
    "icw_crc32_batch": (_i, [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), _i, C.POINTER(C.c_uint32),
                             C.POINTER(C.c_uint32), _u, _i, _vp]),
    "icw_crc32_combine": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint64]),
    "icw_cwave_check": (_i, [_vp, C.c_uint64, _u, _i, C.POINTER(C.c_uint32), C.POINTER(_i)]),
    "icw_config_load": (_i, [C.c_char_p, _sz, C.POINTER(FileConfig), C.POINTER(_i)]),
    "icw_node_dsp_parse": (_i, [C.c_char_p, C.POINTER(Node), C.c_char_p, _sz]),
    "icw_node_dsp_format": (_i, [C.POINTER(Node), C.c_char_p, C.c_char_p, _sz]),
    "icw_wav_parse_file": (_i, [C.c_char_p, C.POINTER(WavInfo)]),
    "icw_transcode_files": (_i, [C.POINTER(Config), C.POINTER(Node), _i, C.POINTER(C.c_char_p),
                                 C.POINTER(C.c_char_p), _i, C.POINTER(BatchOpts), C.POINTER(BatchStats),
                                 C.POINTER(_i)]),
    "icw_group_create": (_i, [C.POINTER(Config), C.POINTER(Node), _i, _i, C.POINTER(_i), _i, C.POINTER(_vp),
                              C.POINTER(_i)]),
    "icw_group_destroy": (_i, [_vp]),
    "icw_group_shard": (_i, [_vp, _i, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i), C.POINTER(_vp)]),
    "icw_group_process": (_i, [_vp, _vp, _sz, _vp, _sz, _i, _u, _vp]),
    "icw_group_get_meters": (_i, [_vp, _i, _i, C.POINTER(Meters)]),
    "icw_group_n_frame": (_i, [_vp, _i, C.POINTER(C.c_uint64)]),
    "icw_transcode_files_devices": (_i, [C.POINTER(Config), C.POINTER(Node), _i, C.POINTER(C.c_char_p),
                                         C.POINTER(C.c_char_p), _i, C.POINTER(BatchOpts), C.POINTER(_i), _i,
                                         C.POINTER(BatchStats), C.POINTER(_i)]),
    "icw_version": (C.c_char_p, []),
    "icw_abi_version": (C.c_int, []),
    "icw_strerror": (C.c_char_p, [_i]),
}
