"""GPU parity of the PRODUCTION paths over random DSP lists: calls that ask for no pre-render doubles,
as the bench (process_device) and the drop-in (dbg = NULL) make them.  Those calls take the
render-only form of the signature-specialised chain programs in KF2 (icw_sig_fast), and the
signature / chain / register-file programs of K2 and K5 without the pre-render store.  Every case
compares the rendered bytes and the meters with the oracle (adv_modulator.c:519-583, 611-751;
sound_render.c:747-800).

Two list generators (tests/graphgen.py):
  - plain_chain: the BASELINE structures (Master on in, Shift -> Master, PM -> Shift -> Mix(in + B)
    -> Master) with random gains (1.0 included), Shift frequencies (negative, fractional, < 1 Hz, locked
    and not), PM frequency / phase / level / angle, now and then a channel that does not rotate, and
    random plain chains of 1-6 ops; both frame-counter modes (counters fresh, near the scaled wrap, far
    out in exact mode, in step or staggered), both quantisers, 16 and 24 bit, sign bits;
  - random_list: the whole option space (exchange, I/Q inversion, one-frame delays, bypass).
Paths: "k2" (3 streams, the quadrature IIR, K2's frame graph), "kf2" (the FIR converter fused with the
graph, order 254, beta 8: KF2 with its render-only passes), "k5" (one stream, one launch per call: the
drop-in's K5).  FIR parity is unpinned: its oracle is the design's own restatement."""
import ctypes as C
import os

import numpy as np
import pytest

from in_cwave_amd import abi, synth
from tests import graphgen
from tests.test_gpu_graph_random import counter_start

pytestmark = pytest.mark.gpu

SEEDS = int(os.environ.get("ICW_RANDOM_SEEDS", 64))   # per generator and path (a multiple of BATCH)
BATCH = 8
FIR_ORDER, FIR_BETA = 254, 8.0
CALLS = {"k2": (1500, 2117), "kf2": (2560, 3190), "k5": (576, 1900)}
STREAMS = {"k2": 3, "kf2": 3, "k5": 1}

_SEEN = {}


def set_counter(ctx, s, n):
    """the stream's frame counter through its state blob (the FIR history after the fixed part stays)"""
    blob = bytes(ctx.get_state(s))
    b = abi.StateBlob.from_buffer_copy(blob)
    b.n_frame = n
    ctx.set_state(s, bytes(b) + blob[C.sizeof(abi.StateBlob):])


def _count(key):
    _SEEN[key] = _SEEN.get(key, 0) + 1


def run_case(oracle, icw, path, gen, seed):
    rng = np.random.default_rng(7_000_003 * seed + (11 if gen == "plain" else 23) + len(path))
    if gen == "plain":
        name, nodes = graphgen.plain_chain(rng)
        cfg = graphgen.plain_config(rng)
    else:
        nodes = graphgen.random_list(rng)
        cfg = graphgen.random_config(rng)
        cfg.need24bits = int(rng.random() < 0.4)
        cfg.render.quantz_type = int(rng.integers(0, 2))
        name = "random"
    S = STREAMS[path]
    kind, n0 = counter_start(rng, cfg)
    n0 = n0[:S] + [n0[-1]] * max(0, S - len(n0))
    calls = CALLS[path]
    fsz = abi.FMT_BYTES[cfg.in_format] * cfg.in_channels
    raw = synth.batch_pcm(S, sum(calls), cfg.sample_rate, channels=cfg.in_channels, fmt=cfg.in_format,
                          first=100 + seed * S)
    if cfg.in_format == abi.FMT_I16 and rng.random() < 0.5:
        v = raw.view(np.int16).copy()          # past full scale now and then: clips and the clamp
        v *= 3
        raw = v.view(np.uint8)
    ctx = icw.Context(cfg, nodes, S)
    if path == "kf2":
        ctx.set_fir_hilbert(FIR_ORDER, FIR_BETA)
    if kind != "fresh":
        for s in range(S):
            set_counter(ctx, s, n0[s])
    outs, t = [], 0
    for n in calls:
        o, _ = ctx.process(np.ascontiguousarray(raw[:, t * fsz:(t + n) * fsz]), n, want_pre=False)
        outs.append(o)
        t += n
    out = np.concatenate(outs, axis=1)
    meters = [ctx.meters(s) for s in range(S)]
    nf = [ctx.n_frame(s) for s in range(S)]
    ctx.close()
    for s in range(S):
        st = oracle.Stream(cfg, nodes)
        assert st.accepted == ctx.accepted
        if path == "kf2":
            st.set_fir(FIR_ORDER, FIR_BETA)
        st.set_n_frame(n0[s])
        ro, _ = st.process(raw[s], sum(calls))
        bad = np.flatnonzero(out[s] != ro)
        where = (f"{path} {gen} seed {seed} stream {s} ({name}, {len(nodes)} nodes, {kind}, "
                 f"scaled={cfg.frmod_scaled}, 24bit={cfg.need24bits}, quantz={cfg.render.quantz_type}, "
                 f"fmt={cfg.in_format}x{cfg.in_channels})")
        assert bad.size == 0, f"{where}: {bad.size} bytes differ, first {bad[:6]}"
        assert meters[s] == st.meters(), f"{where}: meters {meters[s]} vs {st.meters()}"
        assert nf[s] == st.n_frame(), where
    _count((path, gen, name))
    _count((path, gen, kind))
    _count((path, gen, "24bit" if cfg.need24bits else "16bit"))
    _count((path, gen, "exact" if not cfg.frmod_scaled else "scaled"))


@pytest.mark.parametrize("batch", range(SEEDS // BATCH))
@pytest.mark.parametrize("gen", ["plain", "random"])
@pytest.mark.parametrize("path", ["k2", "kf2", "k5"])
def test_production_random_lists(oracle, icw, path, gen, batch, monkeypatch):
    monkeypatch.setenv("ICW_FIR_FUSED", "1")
    for seed in range(batch * BATCH, (batch + 1) * BATCH):
        run_case(oracle, icw, path, gen, seed)


def test_production_random_lists_covered():
    """the plain generator reached every signature, both depths and both counter modes on every path
    (runs after the batches)"""
    if not _SEEN:
        pytest.skip("batches not run in this session")
    for path in ("k2", "kf2", "k5"):
        for key in ("M", "SM", "PSXM", "chain", "16bit", "24bit", "exact", "scaled", "fresh", "in-step"):
            assert _SEEN.get((path, "plain", key), 0) >= 2, (path, key, _SEEN)
