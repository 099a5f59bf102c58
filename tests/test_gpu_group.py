"""GPU: one host process driving several device shards (include/icw_group.h) -- contiguous stream
ranges, one context and one host thread per shard.  On the one-GPU box every shard maps to device 0;
the 8-GPU node runs the same code with devices 0..7.  Results must be byte-identical to one
context over all streams and equal the oracle."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth
from in_cwave_amd import lib as L

from test_gpu_transcode import make_inputs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", ["c4", "c5"])
def test_group_equals_one_context_and_oracle(oracle, icw, shape):
    if shape == "c4":
        fs, fmt = 48000, abi.FMT_I16
        cfg = graph.default_config(fs)
        nodes = graph.graph_pm_shift_mix()
    else:
        fs, fmt = 192000, abi.FMT_F32
        cfg = graph.default_config(fs, fmt=fmt, need24bits=True)
        cfg.render.render_type = abi.RENDER_TPDF
        cfg.render.nshape_type = abi.NSHAPE_MEW44
        nodes = graph.graph_master_only()
    S, n = 7, 2500
    raw = synth.batch_pcm(S, n, fs, fmt=fmt)
    grp = L.Group(cfg, nodes, S, [0, 0, 0])
    assert [grp.shard(d)[:2] for d in range(3)] == [(0, 3), (3, 2), (5, 2)]
    out, pre = grp.process(raw, n, want_pre=True)
    ctx = icw.Context(cfg, nodes, S)
    out1, pre1 = ctx.process(raw, n, want_pre=True)
    assert np.array_equal(out, out1)
    assert np.array_equal(pre.view(np.uint64), pre1.view(np.uint64))
    for s in range(S):
        st = oracle.Stream(cfg, nodes)
        ro, rp = st.process(raw[s], n, want_pre=True)
        assert np.array_equal(out[s], ro), s
        assert np.array_equal(pre[s].view(np.uint64), rp.view(np.uint64)), s
        assert grp.meters(s) == ctx.meters(s) and grp.meters(s)["clips"] == st.meters()["clips"]
        assert grp.n_frame(s) == ctx.n_frame(s) == st.n_frame()
    grp.close()
    ctx.close()


def test_group_pinned_host_buffers(oracle, icw):
    """one caller buffer pair in pinned memory (icw_host_alloc: portable, so pinned for every device),
    sliced over the shards: each shard takes the per-block copy pipeline (several launch blocks per
    call) on its own device, and the bytes equal one context over all streams and the oracle.  On this
    box every shard is device 0; on an 8-GPU node the same slices go to devices 0..7 (host_pinned
    accepts them there because the block is portable)."""
    fs = 48000
    cfg = graph.default_config(fs)
    nodes = graph.graph_shift_master()
    S, n = 5, 40000                                   # 40 000 frames: three launch blocks per call
    raw = synth.batch_pcm(S, n, fs, first=31)
    inp = L.host_array(raw.shape)
    inp[:] = raw
    out = L.host_array((S, n * 4))
    grp = L.Group(cfg, nodes, S, [0, 0])
    grp.process(inp, n, out=out)
    ctx = icw.Context(cfg, nodes, S)
    out1, _ = ctx.process(raw, n)
    assert np.array_equal(np.asarray(out), out1)
    for s in range(S):
        ro, _ = oracle.Stream(cfg, nodes).process(raw[s], n)
        assert np.array_equal(np.asarray(out)[s], ro), s
    grp.close()
    ctx.close()


def test_host_pinned_query():
    """icw_host_pinned is the check each shard context makes before it pipelines a caller slice
    (host_pinned): a portable block (icw_host_alloc) counts for the allocating device 0 and, through
    the allocation-flags branch, for device 1 as well (the query compares indices, so device 1 need
    not exist); pageable memory counts for neither; memory registered while device 0 was current
    counts for device 0"""
    import ctypes as C
    lib = L.load()
    pin = L.host_array((4096,))
    p = pin.ctypes.data
    assert lib.icw_host_pinned(p, 0) == 1
    assert lib.icw_host_pinned(p, 1) == 1
    assert lib.icw_host_pinned(p + 100, 1) == 1        # an interior slice, as a shard gets
    pageable = np.zeros(1 << 16, dtype=np.uint8)
    assert lib.icw_host_pinned(pageable.ctypes.data, 0) == 0
    assert lib.icw_host_pinned(pageable.ctypes.data, 1) == 0
    assert lib.icw_host_pinned(None, 0) == 0
    hip = C.CDLL("libamdhip64.so.7")                    # the runtime libicw links (the same handle)
    buf = np.zeros(1 << 16, dtype=np.uint8)
    assert hip.hipHostRegister(C.c_void_p(buf.ctypes.data), C.c_size_t(buf.nbytes), C.c_uint(0)) == 0
    try:
        assert lib.icw_host_pinned(buf.ctypes.data, 0) == 1
    finally:
        assert hip.hipHostUnregister(C.c_void_p(buf.ctypes.data)) == 0


def test_transcode_files_devices_byte_identical(tmp_path):
    """the many-file transcoder split over two 'devices' (both device 0) writes the same files as
    one device"""
    files = make_inputs(tmp_path)
    cfg = graph.default_config(48000)
    cfg.render.render_type = abi.RENDER_TPDF
    nodes = graph.graph_shift_master()
    ins = [f[0] for f in files]
    one = [tmp_path / f"one_{i}.wav" for i in range(len(ins))]
    two = [tmp_path / f"two_{i}.wav" for i in range(len(ins))]
    rc1, st1, s1 = L.transcode_files(cfg, nodes, ins, one, fade_in_ms=30, fade_out_ms=30, sec_align=1,
                                     block_frames=16384)
    rc2, st2, s2 = L.transcode_files_devices(cfg, nodes, ins, two, [0, 0], fade_in_ms=30, fade_out_ms=30,
                                             sec_align=1, block_frames=16384)
    assert rc1 == rc2 == abi.OK and s1 == s2 == [abi.OK] * len(ins)
    assert st2.n_files == st1.n_files == len(ins) and st2.frames_out == st1.frames_out
    for a, b in zip(one, two):
        assert a.read_bytes() == b.read_bytes(), a.name
