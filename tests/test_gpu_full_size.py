"""Parity at the BASELINE shapes' full per-GPU sizes, exactly as bench.py runs
them: device-resident input of the workload's shape, one full step through libicw with device
pointers -- but every stream gets its own generated input (synth.stream_pcm(s), no tiling), and
EVERY stream is checked bit-exact against the oracle over its FULL length, with its meters.

The pre-render doubles are not exported by this path, so the comparison is on the rendered bytes
(and the clip / peak / de-subnorm meters).  The oracle runs one stream per worker thread (its
ctypes calls release the GIL), one worker per CPU the box gives this process, at most 16.

The c2fir-c5fir variants run the same shapes through the FIR Hilbert converter (bench.py's FIR
legs, DESIGN 4d: no reference implementation, parity against the oracle's restatement only).
Every stream of every shape is checked, c3fir's 4096 included (511 taps over 2^30 frames: about a
minute on 16 cores since the oracle's FIR ring reads without a modulo per tap).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STRIDE = {}                     # every stream of every shape (a stride per shape, if ever needed)


def _workload(name):
    import bench
    return bench.WORKLOADS[name], bench.workload_config(bench.WORKLOADS[name])


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5", "c2fir", "c3fir", "c4fir", "c5fir"])
def test_full_size_step(oracle, icw, name):
    import bench
    import torch
    from in_cwave_amd import synth
    W, (cfg, nodes, fmt) = _workload(name)
    S, T = W["streams"], W["frames"]
    fir = (W["fir"], bench.FIR_BETA) if W.get("fir") else None
    dev = torch.device("cuda", 0)
    nw = synth.cpu_workers()
    with ThreadPoolExecutor(nw) as pool:
        inp = synth.batch_pcm(S, T, W["fs"], channels=W["ch"], fmt=fmt, workers=nw)
        d_in = torch.from_numpy(inp).to(dev)
        ctx = icw.Context(cfg, nodes, S, device=0)
        if fir:
            ctx.set_fir_hilbert(*fir)
        osz = 2 * ctx.render_size
        d_out = torch.empty((S, T * osz), dtype=torch.uint8, device=dev)
        ctx.process_device(d_in, d_in.stride(0), d_out, d_out.stride(0), T)
        torch.cuda.synchronize()
        got = d_out.cpu().numpy()
        meters = [ctx.meters(s) for s in range(S)]
        ctx.close()
        del d_in, d_out

        def check(s):
            st = oracle.Stream(cfg, nodes)
            if fir:
                st.set_fir(*fir)
            ref, _ = st.process(inp[s], T)
            bad = np.flatnonzero(got[s] != ref)
            if bad.size:
                return f"stream {s}: {bad.size} output bytes differ, first at {bad[:4]}"
            m, r = meters[s], st.meters()
            if not (tuple(m["clips"]) == tuple(r["clips"]) and tuple(m["peak_db"]) == tuple(r["peak_db"])
                    and m["desubnorm"] == r["desubnorm"]):
                return f"stream {s}: meters {m} != oracle {r}"
            return None
        checked = list(range(0, S, STRIDE.get(name, 1)))
        if S - 1 not in checked:
            checked.append(S - 1)
        errs = [e for e in pool.map(check, checked) if e]
    assert not errs, f"{name}: {len(errs)} of {len(checked)} streams differ: {errs[:3]}"
    # no two streams share an output (each got its own input): nothing cross-wired or duplicated
    w = got[:, : (got.shape[1] // 8) * 8].view(np.int64)
    sig = np.stack([w.sum(axis=1), (w * 0x9E3779B1).sum(axis=1)], axis=1)
    assert len({tuple(r) for r in sig}) == S
