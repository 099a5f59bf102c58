"""GPU: the batched many-file transcoder (icw_transcode_files) against the oracle, file by file.
Mixed formats (grouped into several contexts), lengths spanning several blocks, fades, the
sec_align virtual zero tail, a CWAVE input and a refused file in the same batch."""
import numpy as np
import pytest

from in_cwave_amd import abi, cwave, graph, synth
from in_cwave_amd import lib as L

import wavgen as W

pytestmark = pytest.mark.gpu


def make_inputs(tmp_path):
    files = []
    specs = [("a.wav", abi.FMT_I16, 2, 48000, 70000), ("b.wav", abi.FMT_I16, 2, 48000, 150001),
             ("c.wav", abi.FMT_I16, 2, 48000, 1000), ("d.wav", abi.FMT_F32, 1, 44100, 90000),
             ("e.rwave", abi.FMT_F32, 1, 44100, 333), ("f.wav", abi.FMT_U8, 2, 22050, 40000)]
    for i, (name, fmt, ch, fs, n) in enumerate(specs):
        d = synth.stream_pcm(i, n, fs, channels=ch, fmt=fmt)
        W.write(tmp_path / name, d, fmt, ch, fs, kind="ext" if i == 1 else ("float" if fmt == abi.FMT_F32 else "pcm"))
        files.append((tmp_path / name, fmt, ch, fs, n, d))
    cw = synth.stream_cwave(9, 50000, 48000, fmt=abi.FMT_CW_I16)
    (tmp_path / "g.cwave").write_bytes(cwave.make_image(cw, abi.FMT_CW_I16, 2, 48000).tobytes())
    files.append((tmp_path / "g.cwave", abi.FMT_CW_I16, 2, 48000, 50000, cw))
    return files


@pytest.mark.parametrize("need24", [False, True])
def test_transcode_batch_vs_oracle(tmp_path, oracle, need24):
    files = make_inputs(tmp_path)
    bad = tmp_path / "broken.wav"
    bad.write_bytes(b"RIFF\0\0\0\0WAVEjunk")
    cfg = graph.default_config(48000, need24bits=need24)
    cfg.render.render_type = abi.RENDER_TPDF
    nodes = graph.graph_master_only()
    ins = [f[0] for f in files] + [bad]
    outs = [tmp_path / f"out_{i}.wav" for i in range(len(ins))]
    rc, st, status = L.transcode_files(cfg, nodes, ins, outs, fade_in_ms=50, fade_out_ms=80, sec_align=1,
                                       block_frames=32768)
    assert status[:-1] == [abi.OK] * len(files) and status[-1] == abi.EINVAL and rc == abi.EINVAL
    assert st.n_files == len(files) and st.n_groups == 4
    rs = 3 if need24 else 2
    for (path, fmt, ch, fs, n, data), out in zip(files, outs):
        c = graph.default_config(fs, fmt=fmt, channels=ch, need24bits=need24)
        c.render.render_type = abi.RENDER_TPDF
        total = n + ((fs - n % fs) % fs)
        zero = 0x80 if fmt == abi.FMT_U8 else 0
        fsz = abi.FMT_BYTES[fmt] * ch
        raw = np.concatenate([data, np.full((total - n) * fsz, zero, np.uint8)])
        s = oracle.Stream(c, nodes)
        s.open(n, 50, 80, 1)
        ref, _ = s.process(raw, total)
        got = np.frombuffer(out.read_bytes(), np.uint8)
        hdr = got[:44].tobytes()
        assert hdr[:4] == b"RIFF" and hdr[8:16] == b"WAVEfmt " and int.from_bytes(hdr[24:28], "little") == fs
        assert int.from_bytes(hdr[34:36], "little") == 8 * rs and int.from_bytes(hdr[40:44], "little") == total * 2 * rs
        assert np.array_equal(got[44:], ref), path.name
