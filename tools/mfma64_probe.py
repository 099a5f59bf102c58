"""Reads gpurun_out/mfma64_round.bin (tools/mfma64_probe.hip) and tests rounding models of
v_mfma_f64_16x16x4_f64: D[i][j] = C[i][j] + sum_k A[i][k] B[k][j], per model the fraction of the
256 x G results it reproduces bit for bit.  Diagnostic only."""
import sys
from fractions import Fraction

import numpy as np

G = 4096


def rnd(q):
    """a Fraction rounded to the nearest double (ties to even)"""
    return float(q) if q != 0 else 0.0


def models(a, b, c):
    p = [Fraction(a[k]) * Fraction(b[k]) for k in range(4)]
    C = Fraction(c)
    out = {}
    # sequential fused steps, k ascending / descending
    for name, order in (("fma_k0123", (0, 1, 2, 3)), ("fma_k3210", (3, 2, 1, 0))):
        acc = c
        for k in order:
            acc = rnd(Fraction(acc) + p[k])
        out[name] = acc
    out["fused_dot"] = rnd(C + sum(p))
    # products exact, then a tree, then + c
    s01 = rnd(p[0] + p[1]); s23 = rnd(p[2] + p[3])
    out["tree_then_c"] = rnd(Fraction(rnd(Fraction(s01) + Fraction(s23))) + C)
    out["dot_exact_then_c"] = rnd(Fraction(rnd(sum(p))) + C)
    # rounded products, sequential adds from c
    acc = c
    for k in range(4):
        acc = rnd(Fraction(acc) + Fraction(rnd(p[k])))
    out["mul_add_k0123"] = acc
    return out


def main(path):
    raw = np.fromfile(path, dtype=np.float64)
    A = raw[:G * 64].reshape(G, 16, 4)
    B = raw[G * 64:G * 128].reshape(G, 4, 16)
    C = raw[G * 128:G * 384].reshape(G, 16, 16)
    D = raw[G * 384:].reshape(G, 16, 16)
    hits, n = {}, 0
    for g in range(0, G, 29):
        for i in range(16):
            for j in range(16):
                m = models(A[g, i], B[g, :, j], C[g, i, j])
                n += 1
                for k, v in m.items():
                    hits[k] = hits.get(k, 0) + (np.float64(v).view(np.uint64) == D[g, i, j].view(np.uint64))
    for k, v in sorted(hits.items(), key=lambda kv: -kv[1]):
        print(f"{k:18s} {v}/{n} = {v / n:.6f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mfma64_round.bin")
