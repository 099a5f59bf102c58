"""CPU tests of the host side: the C ABI library loads and exports every symbol include/*.h
declares (no compute calls without a GPU), ctypes layouts equal the C layouts, graph builders
carry the reference defaults, and the multi-rank sharding/gather path (gloo, world size 2)."""
import ctypes
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np
import pytest

from in_cwave_amd import abi, graph, shard, synth

ROOT = Path(__file__).resolve().parents[1]


def header_functions():
    names = []
    for h in sorted((ROOT / "include").glob("*.h")):
        txt = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(icw_\w+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_header_symbol():
    lib = ROOT / "in_cwave_amd" / "libicw.so"
    assert lib.exists(), "build() must have produced the in-tree library"
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (\w+)", out))
    missing = [n for n in header_functions() if n not in exported]
    assert not missing, missing
    assert set(abi.SIGNATURES) <= set(header_functions())


def test_library_loads_without_gpu():
    from in_cwave_amd import lib as L
    l = L.load()
    assert l.icw_version().startswith(b"in_cwave_amd")
    assert l.icw_strerror(abi.EUNSUPPORTED)
    # the header's ICW_ABI_VERSION is the library's (2: icw_mod_context_fopen takes need24bits)
    hdr = (ROOT / "include" / "icw.h").read_text()
    assert l.icw_abi_version() == int(re.search(r"#define ICW_ABI_VERSION (\d+)", hdr).group(1)) == 2


def test_ctypes_layout_matches_c():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "icw.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(icw_node), sizeof(icw_config), sizeof(icw_render_cfg),
   sizeof(icw_meters), offsetof(icw_node, xch_mode), offsetof(icw_node, fr_shift), offsetof(icw_node, lock_gain),
   offsetof(icw_config, render));
 return 0; }
"""
    with tempfile.TemporaryDirectory() as d:
        c = Path(d) / "l.c"
        c.write_text(src)
        exe = Path(d) / "l"
        subprocess.run(["gcc", "-I", str(ROOT / "include"), "-o", str(exe), str(c)], check=True)
        got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(abi.Node), ctypes.sizeof(abi.Config), ctypes.sizeof(abi.RenderCfg),
            ctypes.sizeof(abi.Meters), abi.Node.xch_mode.offset, abi.Node.fr_shift.offset,
            abi.Node.lock_gain.offset, abi.Config.render.offset]
    assert got == want


def test_graph_defaults_match_reference():
    s = graph.shift()
    assert (s.fr_shift[0], s.fr_shift[1]) == (2.0, -2.0) and s.lock_shift and s.sign_lock_shift
    p = graph.pm()
    assert (p.pm_freq[0], p.pm_level[0]) == (4.0, 0.5) and p.lock_freq and p.lock_level and not p.lock_phase
    m = graph.master()
    assert m.gain[0] == 0.8 and m.tout[0] == abi.S_ADD_REIM and m.inputs[0] == 1
    assert graph.slot("in") == 0 and graph.slot("A") == 1 and graph.slot("Z") == 26


def test_default_config_fields():
    c = graph.default_config()
    assert c.iir_kahan == 1 and c.iir_subnorm_reject == 1 and c.frmod_scaled == 1 and c.hilbert_type == 1
    assert c.render.quantz_type == abi.QUANTZ_MID_RISER and c.render.render_type == abi.RENDER_ROUND
    assert (c.seed_left, c.seed_right) == (0x13579BDF, 0x479B22AB)


@pytest.mark.parametrize("n,w", [(256, 1), (256, 8), (16384, 8), (7, 3), (3, 8)])
def test_shard_range_partition(n, w):
    got = [shard.shard_range(n, r, w) for r in range(w)]
    assert sum(c for _, c in got) == n
    pos = 0
    for f, c in got:
        assert f == pos
        pos += c


def _rank_main(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    from oracle import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_total, n_frames = 5, 700
    first, count = shard.shard_range(n_total, rank, world)
    cfg = graph.default_config(48000)
    nodes = graph.graph_shift_master()
    raw = synth.batch_pcm(count, n_frames, 48000, first=first)
    out, _ = O.process_streams(cfg, nodes, raw, n_frames)        # compute stand-in (test only)
    full = shard.gather_pcm(dist, out, n_total, rank, world)
    clips, peak, dsn = shard.reduce_meters(dist, [[rank, 1]], [[-3.0 - rank, -1.0]], 5)
    if rank == 0:
        np.save(Path(outdir) / "full.npy", full)
        np.save(Path(outdir) / "meters.npy", np.concatenate([clips, peak, [dsn]]))
    dist.barrier()
    dist.destroy_process_group()


def test_multirank_shard_gather_gloo(oracle, tmp_path):
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    full = np.load(tmp_path / "full.npy")
    raw = synth.batch_pcm(5, 700, 48000)
    ref, _ = oracle.process_streams(graph.default_config(48000), graph.graph_shift_master(), raw, 700)
    assert np.array_equal(full, ref)            # sharded == single-process, byte for byte
    m = np.load(tmp_path / "meters.npy")
    assert m.tolist() == [1, 2, -3.0, -1.0, 10]
