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
