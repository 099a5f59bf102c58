"""The device sin / cos (in_cwave_amd/csrc/icw_libm.h) against the system libm, bit for bit, on the
host: the header compiled with g++ -ffp-contract=off is checked against glibc's sincos (generic
build) and sin (the FMA ifunc variant this pool's hosts resolve) on random arguments over every
branch of both routines and on the modulator's own phases (tests/native/libm_check.cpp).  The
same header compiles into the kernels; the GPU tests check the device build through the graph."""
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = tmp_path_factory.mktemp("libm") / "libm_check"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-o", str(exe),
                    str(HERE / "native" / "libm_check.cpp"), "-lm"], check=True)
    return exe


@pytest.mark.parametrize("seed", ["0x9E3779B97F4A7C15", "12345", "0xDEADBEEF"])
def test_sin_cos_bit_identical_to_glibc(checker, seed):
    r = subprocess.run([str(checker), "400000", seed], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("of 3400000") and "mismatches 0 0" in r.stdout


def test_checker_detects_variant_mix(tmp_path):
    """negative control: the generic-build sin is NOT the FMA build's on some arguments, so the
    check above can tell them apart"""
    src = (HERE / "native" / "libm_check.cpp").read_text()
    src = src.replace("const double f2 = icw_lm_sin_fma(x);", "double f2, cd; icw_lm_sincos(x, f2, cd);")
    src = src.replace('"../../in_cwave_amd', f'"{HERE.parent}/in_cwave_amd')
    (tmp_path / "neg.cpp").write_text(src)
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-o", str(tmp_path / "neg"), str(tmp_path / "neg.cpp"),
                    "-lm"], check=True)
    r = subprocess.run([str(tmp_path / "neg"), "100000"], capture_output=True, text=True)
    assert r.returncode == 1
    n_sc, n_s = (int(v) for v in r.stdout.strip().split("\n")[-1].split()[1:3])
    assert n_sc == 0 and n_s > 0


def test_div_sqrt2_hard_cases():
    """icw_div_sqrt2 (icw_kernels.hip): dsp_master's x / SQRT2 (adv_modulator.c:498-501) as
    q0 = RN(x r), e = RN(x - q0 c), q = RN(q0 + e r) with r = RN(1/c).  Its error is below 2^-51 ulp,
    so it can miss RN(x/c) only where x/c is that close to a rounding midpoint: for c = C 2^-52
    (C odd) those significands X solve (2M + 1) C - 2^s X = k, s = 53 (X >= C) or 54 (X < C), odd
    |k| < 8 -- one residue class mod C each.  Every such X (|k| <= 63, several binades) must give
    RN(x/c), computed here in exact rationals; plus random values, and the range test on the result."""
    import math
    import random
    from fractions import Fraction as Fr
    c = float("1.4142135623730950488016887242097")        # SQRT2, adv_modulator.c:43
    r = float.fromhex("0x1.6a09e667f3bccp-1")
    assert c == math.sqrt(2.0) and r == 1.0 / c
    m, ex = math.frexp(c)
    C = int(m * 2 ** 53)
    assert C * 2.0 ** (ex - 53) == c and C % 2 == 1

    def fast(x):
        q0 = x * r
        e = float(Fr(x) - Fr(q0) * Fr(c))                  # one fma: exact, then rounded
        return float(Fr(q0) + Fr(e) * Fr(r))                # one fma

    n = 0
    for s in (53, 54):
        inv = pow(2 ** s, -1, C)
        lo, hi = (C, 2 ** 53) if s == 53 else (2 ** 52, C)
        for k in range(-63, 64, 2):
            X = (-k * inv) % C
            while X < hi:
                if X >= lo:
                    for e2 in (-800, -60, -1, 0, 7, 300, 1000):
                        x = X * 2.0 ** (e2 - 52)
                        assert fast(x) == float(Fr(x) / Fr(c)), (s, k, X, e2)
                        assert fast(-x) == float(Fr(-x) / Fr(c)), (s, k, X, e2)
                        n += 1
                X += C
    assert n > 100
    rng = random.Random(2)
    for _ in range(20000):
        x = rng.uniform(-1e5, 1e5) * 2.0 ** rng.randint(-800, 900)
        assert fast(x) == float(Fr(x) / Fr(c)), x
    # the device keeps the fast value only where |q| >= 2^-900 (icw_div_sqrt2_ok): around that bound
    # and far below it, every kept value is RN(x / c), and from 2^-899.5 up every value is kept
    kept = 0
    for _ in range(4000):
        x = rng.choice((-1.0, 1.0)) * rng.uniform(1.0, 2.0) * 2.0 ** rng.randint(-1074, -896)
        q = fast(x)
        if abs(q) >= 2.0 ** -900:
            assert q == float(Fr(x) / Fr(c)), x
            kept += 1
        if abs(x) >= 2.0 ** -899.5:
            assert abs(q) >= 2.0 ** -900, x
    assert kept > 50
