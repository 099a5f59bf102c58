"""GPU CRC-32 (icw_crc32_cells) and the CWAVE file path end to end.

The CRC is pinned against zlib.crc32, the reference-build golden vectors
(tests/golden/crc32_ref.json, from crc32.c itself) and the oracle restatement. The CWAVE path
starts from a file image: the header is checked, the CRC verified, and the data part decoded by
the HIP kernels against the oracle.
"""
import zlib

import numpy as np
import pytest

from in_cwave_amd import abi, cwave, graph, synth
from in_cwave_amd import lib as L

from test_cwave_host import golden_crc_cases

pytestmark = pytest.mark.gpu


def test_crc_golden_reference_vectors():
    data, want = [], []
    for d, _, crc in golden_crc_cases():
        data.append(d)
        want.append(crc)
    offs = np.cumsum([0] + [len(d) for d in data[:-1]])
    base = np.frombuffer(b"".join(data), dtype=np.uint8).copy() if sum(map(len, data)) else np.zeros(1, np.uint8)
    assert L.crc32_batch(base, offs, [len(d) for d in data]) == want


def test_crc_lengths_and_alignments_host():
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    cases = []
    for n in [0, 1, 2, 3, 4, 15, 16, 17, 255, 256, 257, 4095, 65535, 65536, 65537, 131072 + 5, (1 << 20) + 13]:
        for off in (0, 1, 7, 16, 65535, 1 << 20):
            if off + n <= buf.size:
                cases.append((off, n))
    got = L.crc32_batch(buf, [c[0] for c in cases], [c[1] for c in cases])
    want = [zlib.crc32(buf[o:o + n].tobytes()) for o, n in cases]
    assert got == want


def test_crc_device_pointers_and_chaining():
    import torch
    rng = np.random.default_rng(12)
    host = rng.integers(0, 256, (8 << 20) + 3, dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    offs = [3, 1000, (4 << 20) + 1]
    lens = [1 << 20, (3 << 20) + 77, (4 << 20) - 9]
    got = L.crc32_batch(dev, offs, lens, device_ptrs=True)
    assert got == [zlib.crc32(host[o:o + n].tobytes()) for o, n in zip(offs, lens)]
    # crc_in continues a CRC: crc(A || B) with A done earlier
    a, b = host[:12345].tobytes(), host[12345:12345 + 99999]
    got = L.crc32_batch(dev, [12345], [99999], crc_in=[zlib.crc32(a)], device_ptrs=True)
    assert got == [zlib.crc32(a + b.tobytes())]


def test_crc_many_small_ranges():
    rng = np.random.default_rng(13)
    lens = rng.integers(0, 3000, 4000)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    buf = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    got = L.crc32_batch(buf, offs, lens)
    assert got == [zlib.crc32(buf[o:o + n].tobytes()) for o, n in zip(offs, lens)]


def test_crc_large_range_device():
    import torch
    n = 256 << 20
    dev = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    host = dev.cpu().numpy()
    assert L.crc32_batch(dev, [0], [n], device_ptrs=True) == [zlib.crc32(host.tobytes())]


@pytest.mark.parametrize("fmt", abi.CW_FORMATS)
def test_cwave_check_and_decode(oracle, icw, fmt):
    """check_cwave (gui_cwave.c:82-129) + decoding the data part (xwave_reader.c:171-200)"""
    import torch
    fs, n, ch = 48000, 7000, 2
    data = synth.stream_cwave(4, n, fs, channels=ch, fmt=fmt)
    img = cwave.make_image(data, fmt, ch, fs, trailer=b"\x01\x02")
    crc, ok = L.cwave_check(img)
    assert ok == 1 and crc == zlib.crc32(data.tobytes())
    crc_d, ok_d = L.cwave_check(torch.from_numpy(img).cuda(), device_ptrs=True)
    assert (crc_d, ok_d) == (crc, 1)
    bad = img.copy()
    bad[48 + 1234] ^= 0x40
    assert L.cwave_check(bad)[1] == 0
    v1 = cwave.make_image(data, fmt, ch, fs, version=1)
    assert L.cwave_check(v1) == (crc, -1)

    h, f, fb = L.cwave_parse(img.tobytes(), img.size)
    cfg = graph.default_config(h.sample_rate, fmt=f, channels=h.n_channels)
    payload = img[h.hsize:h.hsize + h.n_samples * fb][None, :]
    ctx = icw.Context(cfg, graph.graph_shift_master(), 1)
    ctx.stream_open(0, h.n_samples, fade_in_ms=20, fade_out_ms=20)
    out, pre = ctx.process(payload, h.n_samples, want_pre=True)
    st = oracle.Stream(cfg, graph.graph_shift_master())
    st.open(h.n_samples, 20, 20)
    ro, rp = st.process(payload[0], h.n_samples, want_pre=True)
    assert np.array_equal(pre[0].view(np.uint64), rp.view(np.uint64))
    assert np.array_equal(out[0], ro)
