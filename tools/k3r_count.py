import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from in_cwave_amd import lib as L, graph, synth, abi
cfg = graph.default_config(192000, fmt=abi.FMT_F32, need24bits=True)
cfg.render.render_type = abi.RENDER_TPDF
cfg.render.nshape_type = abi.NSHAPE_MEW44
S, n = 8, 200000
raw = synth.batch_pcm(S, n, 192000, fmt=abi.FMT_F32)
ctx = L.Context(cfg, graph.graph_master_only(), S)
ctx.set_fir_hilbert(1022, 8.0)
ctx.process(raw, n)
print("fast blocks per channel:", [ctx.meters(s)["clips"] for s in range(S)], "of", n // 20)
