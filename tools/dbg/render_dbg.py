import sys, numpy as np
sys.path.insert(0, '.')
from in_cwave_amd import abi, graph, synth, lib as L
from oracle import oracle as O
cfg = graph.default_config(44100)
cfg.render.render_type = abi.RENDER_RPDF
cfg.render.dth_bits = 1.5
raw = synth.batch_pcm(1, 64, 44100)
ctx = L.Context(cfg, graph.graph_master_only(), 1)
out, pre = ctx.process(raw, 64, want_pre=True)
ro, rp = O.process_streams(cfg, graph.graph_master_only(), raw, 64, want_pre=True)
g = out.view('<i2').reshape(-1, 2); r = ro.view('<i2').reshape(-1, 2)
print("pre equal", np.array_equal(pre.view(np.uint64), rp.view(np.uint64)))
for t in range(12):
    print(t, pre[0, t], g[t], r[t])
mt = O.MT(seed=abi.SEED_LEFT)
print("first dsopen L:", [mt.dsopen() for _ in range(4)])
