#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Reference-pinned (produced from the reference's own files / reference-built code):
  mt19937ar_kat.json   -- the reference's known-answer data (test_mt_jrnd/mt19937ar_out.c:
                          init_by_array {0x123,0x234,0x345,0x456}, first 1000 genrand_int32)
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
    e2e()
    print("golden fixtures written to", GOLD)
