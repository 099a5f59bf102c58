"""Second, independent restatement of the quadrature Hilbert converter, in pure Python.

Test infrastructure only.  Python floats are IEEE-754 binary64 and the interpreter never
contracts a*b+c into an FMA, so every operation below rounds exactly once, as the reference's
x87-free SSE2 build does.  It is written from the reference's text, not from oracle/icw_oracle.c,
and shares no code with it: the delay line is a Python list kept newest-first instead of the
reference's decrementing ring, and the coefficients come from tests/golden/tables.json (the bit
patterns of hblpf.c:81-402), not from the oracle's table include.

  * coefficients   iir_rp_create          hblpf.c:828-863   pc = -a[j]/a0, pd = b[j]/a0, d0 = b0/a0
  * baseline       iir_rp_process_baseline hblpf.c:894-926  plain sums, reject, sum_i*d0 + sum_o
  * Kahan          iir_rp_process_kahan   hblpf.c:1008-1056 Kahan sums (kahan_step :987-993),
                                                            output sum without a d0*sample term
  * reject         `fabs(S) < is_subnorm_reject` with a BOOL threshold, i.e. 1.0 (hblpf.c:1046)
  * quadrature     hq_rp_process          lpf_hilbert_quad.c:129-156
"""
import json
import struct
from pathlib import Path

_TABLES = json.loads((Path(__file__).resolve().parent / "golden" / "tables.json").read_text())


def _hex2d(h):
    return struct.unpack(">d", bytes.fromhex(h))[0]


class PyIIR:
    """One DF-II section of order N; `hist[0]` is the newest state (the reference's pz[ix-1])."""

    def __init__(self, type_, kahan=1, subn=1):
        f = _TABLES["hb"][type_]
        n = f["order"]
        a = [_hex2d(h) for h in f["a"][: n + 1]]
        b = [_hex2d(h) for h in f["b"][: n + 1]]
        a0 = a[0]
        self.n = n
        self.d0 = b[0] / a0
        self.c = [-a[j] / a0 for j in range(1, n + 1)]
        self.d = [b[j] / a0 for j in range(1, n + 1)]
        self.kahan = kahan
        self.thr = 1.0 if subn else 0.0
        self.hist = [0.0] * n
        self.subnorm_cnt = 0

    def _reject(self, s):
        if self.thr and abs(s) < self.thr:
            self.subnorm_cnt += 1
            return 0.0
        return s

    def step(self, x):
        h = self.hist
        if self.kahan:
            # input sum: S = x, C = 0, then one Kahan step per c_i*z_i, newest state first
            s, cc = x, 0.0
            # output sum: S = z_0*d_0, C = 0, then d0*(c_0 z_0), then per i>0: d_i z_i, d0*(c_i z_i)
            so, co = None, 0.0
            for i in range(self.n):
                ti = h[i] * self.c[i]
                y = ti - cc
                t = s + y
                cc = (t - s) - y
                s = t
                if i == 0:
                    so = h[0] * self.d[0]
                    terms = (ti * self.d0,)
                else:
                    terms = (h[i] * self.d[i], ti * self.d0)
                for xj in terms:
                    y = xj - co
                    t = so + y
                    co = (t - so) - y
                    so = t
            w = self._reject(s)
            out = so
        else:
            si, so = x, 0.0
            for i in range(self.n):
                si = si + h[i] * self.c[i]
                so = so + h[i] * self.d[i]
            w = self._reject(si)
            out = w * self.d0 + so
        self.hist = [w] + h[:-1]
        return out


class PyHilbert:
    """fs/4 quadrature converter: filter I gets {x, 0, -x, 0}, filter Q gets {0, -x, 0, x}."""

    def __init__(self, type_=1, kahan=1, subn=1):
        self.fi = PyIIR(type_, kahan, subn)
        self.fq = PyIIR(type_, kahan, subn)
        self.k = 0

    def step(self, x):
        fi, fq, k = self.fi, self.fq, self.k
        if k == 0:
            oi, oq = fi.step(x) * 2.0, fq.step(0.0) * 2.0
        elif k == 1:
            oi, oq = -fq.step(-x) * 2.0, fi.step(0.0) * 2.0
        elif k == 2:
            oi, oq = -fi.step(-x) * 2.0, -fq.step(0.0) * 2.0
        else:
            oi, oq = fq.step(x) * 2.0, -fi.step(0.0) * 2.0
        self.k = (k + 1) & 3
        return oi, oq
