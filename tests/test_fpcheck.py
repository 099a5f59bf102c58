"""FP_CHECK (fp_check.c:52-100): the oracle's FC() arithmetic and census, CPU only.  FC() returns
its argument unless it is a NaN / denormal (-> 0.0) or an infinity (-> +-65535.0), counting the
class (FP_EXCEPT_STATS, fp_check.h:62-72); the GPU path is checked against it in
test_gpu_fpcheck.py.  Parity unpinned against the reference itself (its FC path needs <windows.h>,
DESIGN.md 1): these tests pin the restatement's own invariants."""
import numpy as np

from in_cwave_amd import abi, graph, synth
from fpcheck_inputs import fc_cfg, special_cw64, special_f32


def test_fp_check_is_identity_on_ordinary_input(oracle):
    """on ordinary audio nothing is special: same bytes as the plain path, an empty census"""
    raw = synth.batch_pcm(2, 3000, 48000)
    for kahan in (1, 0):
        cfg = fc_cfg(abi.FMT_I16, kahan=kahan)
        cen = []
        on, _ = oracle.process_streams(cfg, graph.graph_shift_master(), raw, 3000, census=cen)
        cfg.fp_check = 0
        off, _ = oracle.process_streams(cfg, graph.graph_shift_master(), raw, 3000)
        assert np.array_equal(on, off)
        assert all(int(c.sum()) == 0 for c in cen)


def test_fp_check_counts_hilbert_specials(oracle):
    cen = []
    oracle.process_streams(fc_cfg(), graph.graph_master_only(), special_f32(2, 2000), 2000, census=cen)
    h = sum(c[:2] for c in cen)
    assert h[:, 2].sum() > 0                                  # NaN products / sums -> qNaN
    assert h[:, 3].sum() > 0 and h[:, 6].sum() > 0            # -Inf, +Inf -> -+65535
    for c in cen:
        assert (c[:, 0] == c[:, 1:].sum(axis=1)).all()        # total = sum of the classes


def test_fp_check_counts_render_specials(oracle):
    cen = []
    oracle.process_streams(fc_cfg(abi.FMT_CW_F64), graph.graph_master_only(), special_cw64(2, 2000), 2000,
                           census=cen)
    r = sum(c[2:] for c in cen)
    assert r[:, 2].sum() > 0 and r[:, 3].sum() > 0 and r[:, 6].sum() > 0
    assert r[:, 4].sum() + r[:, 5].sum() > 0                   # denormals -> 0.0
    for c in cen:
        assert (c[:, 0] == c[:, 1:].sum(axis=1)).all()
