"""GPU parity with misaligned input: the unpack is specialised per format (icw_kernels.hip
icw_fmt_dispatch) and reads a sample with one typed load when the base address and the strides keep
every sample aligned to its size, with byte loads otherwise.  The reader's buffers carry no such
promise (xwave_reader.c:205-239 reads bytes), so both forms must give the oracle's bytes: device
input at byte offsets 0-3 with odd and even row strides, through K0 (quadrature IIR), the FIR
converter (KF2 and KF + K2) and the one-stream kernel K5."""
import numpy as np
import pytest

from in_cwave_amd import abi, graph, synth

pytestmark = pytest.mark.gpu


def run(oracle, icw, cfg, nodes, S, T, off, pad, fir=None):
    import torch
    raw = synth.batch_pcm(S, T, cfg.sample_rate, channels=cfg.in_channels, fmt=cfg.in_format, first=3)
    row = raw.shape[1] + pad
    buf = np.zeros((S, row + 4), dtype=np.uint8)
    buf[:, off:off + raw.shape[1]] = raw
    d_buf = torch.from_numpy(buf).cuda()
    d_in = d_buf[:, off:]
    ctx = icw.Context(cfg, nodes, S)
    if fir:
        ctx.set_fir_hilbert(fir, 8.0)
    osz = 2 * ctx.render_size
    d_out = torch.zeros((S, T * osz), dtype=torch.uint8, device="cuda")
    assert d_in.data_ptr() % 8 == off
    ctx.process_device(d_in, d_buf.stride(0), d_out, d_out.stride(0), T)
    ctx.synchronize()
    out = d_out.cpu().numpy()
    for s in range(S):
        st = oracle.Stream(cfg, nodes)
        if fir:
            st.set_fir(fir, 8.0)
        ro, _ = st.process(raw[s], T)
        assert np.array_equal(out[s], ro), (s, off, pad)
    ctx.close()


FORMATS = [(abi.FMT_I16, 2), (abi.FMT_I16, 1), (abi.FMT_I32, 2), (abi.FMT_F32, 1), (abi.FMT_I24, 2),
           (abi.FMT_U8, 2)]


@pytest.mark.parametrize("off,pad", [(0, 0), (1, 0), (2, 1), (3, 2), (2, 0)])
@pytest.mark.parametrize("fmt,ch", FORMATS)
def test_iir_unaligned_input(oracle, icw, fmt, ch, off, pad):
    cfg = graph.default_config(48000, fmt=fmt, channels=ch)
    run(oracle, icw, cfg, graph.graph_shift_master(), 3, 1500, off, pad)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("off,pad", [(1, 0), (2, 1), (2, 0)])
@pytest.mark.parametrize("fmt,ch", FORMATS)
def test_fir_unaligned_input(oracle, icw, fmt, ch, off, pad, fused, monkeypatch):
    monkeypatch.setenv("ICW_FIR_FUSED", fused)
    cfg = graph.default_config(48000, fmt=fmt, channels=ch)
    run(oracle, icw, cfg, graph.graph_shift_master(), 2, 2500, off, pad, fir=254)


@pytest.mark.parametrize("off", [0, 1, 2])
@pytest.mark.parametrize("fmt,ch", FORMATS)
def test_stream1_unaligned_input(oracle, icw, fmt, ch, off, monkeypatch):
    monkeypatch.setenv("ICW_STREAM1", "1")
    monkeypatch.setenv("ICW_K1_MODE", "row")
    cfg = graph.default_config(44100, fmt=fmt, channels=ch)
    run(oracle, icw, cfg, graph.graph_shift_master(), 1, 576, off, 0)
