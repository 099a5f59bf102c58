#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Reference-pinned (produced from the reference's own files / reference-built code):
  mt19937ar_kat.json   -- the reference's known-answer data (test_mt_jrnd/mt19937ar_out.c:
                          init_by_array {0x123,0x234,0x345,0x456}, first 1000 genrand_int32)
  unpack_ref.npz       -- the REFERENCE's unpack_int16/24/32/float/double (unpack_lsb.h:53-125) on
                          random and edge-case bytes (oracle/_ref/libref_unpack.so: oracle/ref_unpack.c
                          compiled with -I /root/reference/src, no stand-in headers)
  cwave_layout.json    -- sizeof / offsetof of HCWAVE_V1 / V2 and the HCW_* constants of cwave.h
  mt_ref_seeds.npz     -- outputs of the REFERENCE mt_jrnd.c (oracle/_ref/libref_mt.so, compiled
                          from /root/reference/src/mersene_twister/mt_jrnd.c by oracle/Makefile)
                          for the two render seeds 0x13579BDF / 0x479B22AB (in_cwave.c:69-70):
                          u32, dsemi and dsopen streams
Oracle regression vectors (produced by oracle/liboracle.so; they pin the GPU path and guard the
restatement against regressions -- NOT reference outputs, see DESIGN.md "Oracle"):
  e2e_*.npz            -- small end-to-end cases of the BASELINE config shapes + quirk inputs

Run in the build container (needs /root/reference for the first two):  python tools/gen_golden.py
"""
import ctypes as C
import json
import re
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
GOLD = ROOT / "tests" / "golden"
REF = Path("/root/reference/src")


def kat():
    src = (REF / "mersene_twister/test_mt_jrnd/mt19937ar_out.c").read_text()
    init = [int(x, 16) for x in re.search(r"test_init\[4\]\s*=\s*\{([^}]*)\}", src).group(1).replace(" ", "").split(",")]
    body = re.search(r"test_u32\[1000\]\s*=\s*\{(.*?)\};", src, re.S).group(1)
    vals = [int(v) for v in re.findall(r"(\d+)U", body)]
    assert len(vals) == 1000
    (GOLD / "mt19937ar_kat.json").write_text(json.dumps({"init_key": init, "u32": vals}) + "\n")


class _St(C.Structure):
    _fields_ = [("state", C.c_uint32 * 624), ("next", C.c_void_p), ("left", C.c_int)]


def ref_seeds():
    lib = C.CDLL(str(ROOT / "oracle/_ref/libref_mt.so"))
    lib.mtrnd_init_seed.argtypes = [C.c_void_p, C.c_uint32]
    lib.mtrnd_gen_ui32.restype = C.c_uint32
    lib.mtrnd_gen_dsemi.restype = C.c_double
    lib.mtrnd_gen_dsopen.restype = C.c_double
    out = {}
    for name, seed in (("left", 0x13579BDF), ("right", 0x479B22AB)):
        for kind, fn in (("u32", lib.mtrnd_gen_ui32), ("dsemi", lib.mtrnd_gen_dsemi), ("dsopen", lib.mtrnd_gen_dsopen)):
            st = _St()
            lib.mtrnd_init_seed(C.byref(st), seed)
            fn.argtypes = [C.c_void_p]
            out[f"{name}_{kind}"] = np.array([fn(C.byref(st)) for _ in range(2000)])
    out["left_u32"] = out["left_u32"].astype(np.uint32)
    out["right_u32"] = out["right_u32"].astype(np.uint32)
    np.savez_compressed(GOLD / "mt_ref_seeds.npz", **out)


def crc_ref():
    """CRC-32 of seeded random data by the REFERENCE crc32.c (oracle/_ref/libref_crc32.so), fed in
    the block partitions given (crc32update chaining across reads, as check_cwave does)."""
    lib = C.CDLL(str(ROOT / "oracle/_ref/libref_crc32.so"))

    class Tmp(C.Structure):
        _fields_ = [("xOr", C.c_uint32), ("temp", C.c_uint32)]

    lib.crc32final.restype = C.c_uint32
    cases = []
    rng = np.random.default_rng(32)
    for n, parts in [(0, [0]), (1, [1]), (3, [1, 2]), (4, [4]), (7, [2, 2, 3]), (9, [9]), (255, [100, 155]),
                     (4096, [576 * 4, 4096 - 576 * 4]), (65537, [65537]), (100003, [3, 1, 99999])]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        t = Tmp()
        lib.crc32init(C.byref(t))
        off = 0
        for k in parts:
            lib.crc32update(data[off:off + k], C.c_uint(k), C.byref(t))
            off += k
        cases.append({"seed_index": len(cases), "n": n, "parts": parts, "crc": int(lib.crc32final(C.byref(t)))})
    check = b"123456789"
    t = Tmp()
    lib.crc32init(C.byref(t))
    lib.crc32update(check, C.c_uint(9), C.byref(t))
    doc = {"generator": "numpy.random.default_rng(32).integers(0, 256, n, uint8), cases in order",
           "cases": cases, "check_123456789": int(lib.crc32final(C.byref(t)))}
    (GOLD / "crc32_ref.json").write_text(json.dumps(doc, indent=1) + "\n")


# edge-case patterns per unpacker, little-endian values: i24 sign extension, integer extremes,
# signed zeros, infinities, quiet / signalling / negative NaNs with payloads, denormals
UNPACK_EDGES = {
    "i16": [0x0000, 0x0001, 0x7FFF, 0x8000, 0x8001, 0xFFFF, 0x00FF, 0xFF00],
    "i24": [0x000000, 0x000001, 0x7FFFFF, 0x800000, 0x800001, 0xFFFFFF, 0x00FF80, 0xFF007F],
    "i32": [0, 1, 0x7FFFFFFF, 0x80000000, 0x80000001, 0xFFFFFFFF, 0x00008000, 0xFFFF8000],
    "f32": [0x00000000, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00000, 0x7FA00001, 0xFFC00123, 0xFF800001,
            0x00000001, 0x007FFFFF, 0x80000001, 0x807FFFFF, 0x00800000, 0x3F800000, 0xBF800000, 0x7F7FFFFF],
    "f64": [0, 1 << 63, 0x7FF0000000000000, 0xFFF0000000000000, 0x7FF8000000000000, 0x7FF4000000000001,
            0xFFF8000000000123, 0x0000000000000001, 0x000FFFFFFFFFFFFF, 0x8000000000000001,
            0x0010000000000000, 0x3FF0000000000000, 0x40DFFFC000000000, 0xC0E0000000000000, 0x7FEFFFFFFFFFFFFF],
}
UNPACK_KINDS = {"i16": (0, 2), "i24": (1, 3), "i32": (2, 4), "f32": (3, 4), "f64": (4, 8)}


def unpack_ref():
    """the REFERENCE's LE unpackers (unpack_lsb.h:53-125) and CWAVE header layout (cwave.h:31-87),
    compiled where they lie by oracle/Makefile (`ref`: oracle/ref_unpack.c includes them), run on
    random bytes (numpy.random.default_rng(53), 1024 samples per kind) followed by the edge cases"""
    lib = C.CDLL(str(ROOT / "oracle/_ref/libref_unpack.so"))
    lib.ref_unpack_batch.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_void_p]
    lib.ref_cwave_layout.argtypes = [C.c_void_p, C.c_int]
    lib.ref_cwave_magic.restype = C.c_char_p
    rng = np.random.default_rng(53)
    out = {}
    for name, (kind, size) in UNPACK_KINDS.items():
        rnd = rng.integers(0, 256, 1024 * size, dtype=np.uint8)
        edge = np.concatenate([np.frombuffer(int(v).to_bytes(size, "little"), np.uint8) for v in UNPACK_EDGES[name]])
        raw = np.ascontiguousarray(np.concatenate([rnd, edge]))
        n = raw.size // size
        val = np.zeros(n, dtype=np.uint64 if name == "f64" else (np.uint32 if name == "f32" else np.int32))
        assert lib.ref_unpack_batch(kind, raw.ctypes.data, n, val.ctypes.data) == 0
        out[name + "_bytes"] = raw
        out[name + "_val"] = val
    np.savez_compressed(GOLD / "unpack_ref.npz", **out)
    lay = np.zeros(64, dtype=np.int64)
    m = lib.ref_cwave_layout(lay.ctypes.data, lay.size)
    fields = ["sizeof", "magic", "hsize", "version", "format", "n_channels", "n_samples", "sample_rate", "k_M"]
    doc = {"generator": "oracle/ref_unpack.c on cwave.h (reference, compiled where it lies)",
           "HCWAVE_V1": dict(zip(fields + ["pad0", "k_beta"], map(int, lay[0:11]))),
           "HCWAVE_V2": dict(zip(fields + ["n_CRC32", "k_beta"], map(int, lay[11:22]))),
           "HCW_VERSION": dict(zip(["BAD", "V1", "V2", "CUR"], map(int, lay[22:26]))),
           "HCW_FMT": dict(zip(["BAD_FMT", "PCM_DBL64", "PCM_INT16", "PCM_INT16_FLT32", "PCM_FLT32"],
                               map(int, lay[26:31]))),
           "HCW_MAGIC": lib.ref_cwave_magic().decode()}
    assert m == 31
    (GOLD / "cwave_layout.json").write_text(json.dumps(doc, indent=1) + "\n")


def e2e():
    from in_cwave_amd import abi, graph, synth
    from oracle import oracle as O
    cases = {
        "c1_shift_44k": (graph.default_config(44100), graph.graph_shift_master(), synth.batch_pcm(1, 4410, 44100)),
        "c2_shift_48k": (graph.default_config(48000), graph.graph_shift_master(), synth.batch_pcm(2, 4800, 48000)),
        "c3_mono_96k": (graph.default_config(96000, channels=1), graph.graph_master_only(),
                        synth.batch_pcm(2, 4800, 96000, channels=1)),
        "c4_pm_shift_mix": (graph.default_config(48000), graph.graph_pm_shift_mix(), synth.batch_pcm(2, 4800, 48000)),
    }
    # quirk inputs: -100 dBFS float (subnorm threshold 1.0 -> silence), full-scale square (clips),
    # digital silence, DC, impulse
    n = 4800
    t = np.arange(n)
    quiet = (10 ** (-100 / 20) * np.sin(2 * np.pi * 997 * t / 48000)).astype("<f4")
    quiet = np.repeat(quiet, 2).view(np.uint8)[None, :]
    cases["quirk_minus100dbfs_f32"] = (graph.default_config(48000, fmt=abi.FMT_F32), graph.graph_master_only(), quiet)
    sq = np.where((t // 24) % 2 == 0, 32767, -32768).astype("<i2")
    sq = np.repeat(sq, 2).view(np.uint8)[None, :]
    cases["quirk_fullscale_square"] = (graph.default_config(48000), [graph.master(gain=2.0)], sq)
    cases["quirk_silence"] = (graph.default_config(48000), graph.graph_master_only(), np.zeros((1, n * 4), np.uint8))
    dc = np.full(2 * n, 12000, dtype="<i2").view(np.uint8)[None, :]
    cases["quirk_dc"] = (graph.default_config(48000), graph.graph_master_only(), dc)
    imp = np.zeros(2 * n, dtype="<i2")
    imp[0] = imp[1] = 32767
    cases["quirk_impulse"] = (graph.default_config(48000), [graph.master(tout=abi.S_RE, gain=1.0)],
                              imp.view(np.uint8)[None, :])
    # complex (CWAVE) input and lists with one-frame delays / feedback (bus form)
    cases["cw_i16f32_shift"] = (graph.default_config(48000, fmt=abi.FMT_CW_I16_F32), graph.graph_shift_master(),
                                synth.batch_pcm(2, 2400, 48000, fmt=abi.FMT_CW_I16_F32))
    cases["cw_f64_mono_24"] = (graph.default_config(44100, fmt=abi.FMT_CW_F64, channels=1, need24bits=True),
                               graph.graph_master_only(), synth.batch_pcm(1, 2205, 44100, channels=1, fmt=abi.FMT_CW_F64))
    cases["fb_leaky"] = (graph.default_config(48000), graph.graph_leaky_feedback(), synth.batch_pcm(2, 2400, 48000))
    cases["fb_pm_shift"] = (graph.default_config(48000), graph.graph_feedback_pm_shift(), synth.batch_pcm(2, 2400, 48000))
    cases["delay_shift"] = (graph.default_config(48000), graph.graph_pure_delay(), synth.batch_pcm(2, 2400, 48000))
    for name, (cfg, nodes, raw) in cases.items():
        fsz = abi.FMT_BYTES[cfg.in_format] * cfg.in_channels
        nf = raw.shape[1] // fsz
        out, pre = O.process_streams(cfg, nodes, raw, nf, want_pre=True)
        metas = []
        for s in range(raw.shape[0]):
            st = O.Stream(cfg, nodes)
            st.process(raw[s], nf)
            metas.append(st.meters())
        np.savez_compressed(GOLD / f"e2e_{name}.npz", raw=raw, out=out, pre=pre,
                            cfg=np.frombuffer(bytes(cfg), np.uint8),
                            nodes=np.frombuffer(bytes((abi.Node * len(nodes))(*nodes)), np.uint8),
                            clips=np.array([m["clips"] for m in metas]),
                            peak=np.array([m["peak_db"] for m in metas]),
                            desubnorm=np.array([m["desubnorm"] for m in metas]))


if __name__ == "__main__":
    GOLD.mkdir(parents=True, exist_ok=True)
    if REF.is_dir():
        kat()
        ref_seeds()
        crc_ref()
        unpack_ref()
    e2e()
    print("golden fixtures written to", GOLD)
