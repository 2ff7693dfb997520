"""The C++ host mirror (binius-ntt_amd/host/ulvt: AdditiveNTT<T,P>, NTTData, AdditiveNTTConf,
FanPaarTowerField, BitsliceUtils, Sumcheck<N,d,T>) builds against the C-ABI alone (CPU), and on
the GPU runs the reference's own test flows (tests/cpp/test_surface.cpp): the GF(2^32) MD5 table
of test_ntt.cu, GF(2^128) vs the oracle, and the sumcheck verifier loop of test.cu."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "binius-ntt_amd", "lib")
ORACLE = os.path.join(ROOT, "oracle")
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_surface")


def _build():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "binius-ntt_amd", "host", "ulvt"),
           os.path.join(ROOT, "tests", "cpp", "test_surface.cpp"), "-o", BIN,
           "-L", LIBDIR, "-lbinius_ntt_amd", "-L", ORACLE, "-loracle",
           "-Wl,-rpath," + LIBDIR, "-Wl,-rpath," + ORACLE, "-Wl,--allow-shlib-undefined"]
    subprocess.check_call(cmd)


def test_cpp_mirror_builds_against_the_c_abi():
    _build()
    assert os.path.exists(BIN)


@pytest.mark.gpu
def test_cpp_mirror_runs_reference_flows(ntt_md5):
    _build()
    p = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    out = p.stdout.splitlines()
    assert p.returncode == 0, p.stdout + p.stderr
    n = 0
    for line in out:
        if line.startswith("md5 "):
            _, r, log_h, h = line.split()
            want = ntt_md5[r][int(log_h)]
            if want:
                assert h == want, line
                n += 1
    assert n >= 30
    assert not [l for l in out if l.startswith("FAIL")]
