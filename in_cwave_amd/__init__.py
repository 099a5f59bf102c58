"""in_cwave_amd -- MI355X-native (gfx950) batched implementation of the in_cwave per-block
Hilbert -> modulator-graph -> dithered render hot path, behind a C ABI (include/icw.h).

    from in_cwave_amd import graph, lib
    cfg = graph.default_config(48000)
    ctx = lib.Context(cfg, graph.graph_shift_master(), n_streams=256)
    out, _ = ctx.process(pcm_bytes, n_frames)

The compute runs only in libicw.so (hand-written HIP kernels); importing this package never
falls back to a CPU implementation.
"""
from . import abi, graph  # noqa: F401

__version__ = "0.1.0"

