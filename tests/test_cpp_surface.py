"""The C++ host mirror (binius-ntt_amd/host/ulvt: AdditiveNTT<T,P>, NTTData, AdditiveNTTConf,
FanPaarTowerField, BitsliceUtils, Sumcheck<N,d,T>; and the prime-field siblings NTT<BB31>,
NTTConfRad2, BB31, QM31, Sumcheck<N>, interpolate_at) builds against the C-ABI alone (CPU), and on
the GPU runs the reference's own test flows (tests/cpp/test_surface.cpp: the GF(2^32) MD5 table
of test_ntt.cu, GF(2^128) vs the oracle, the sumcheck verifier loop of test.cu;
tests/cpp/test_prime_field.cpp: the BabyBear MD5 table and round trip of test_ntt.cu and the
"Prime Field Sumcheck Test")."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "binius-ntt_amd", "lib")
ORACLE = os.path.join(ROOT, "oracle")
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_surface")


PRIME_BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_prime_field")


ROCM = "/opt/rocm"


def _build(src="test_surface.cpp", out=BIN):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "binius-ntt_amd", "host", "ulvt"),
           os.path.join(ROOT, "tests", "cpp", src), "-o", out,
           "-L", LIBDIR, "-lbinius_ntt_amd", "-L", ORACLE, "-loracle",
           "-Wl,-rpath," + LIBDIR, "-Wl,-rpath," + ORACLE, "-Wl,--allow-shlib-undefined"]
    if src == "test_surface.cpp":  # device message sinks of the sharded test (HIP host API)
        cmd += ["-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROCM, "include"), "-L", os.path.join(ROCM, "lib"),
                "-lamdhip64", "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    subprocess.check_call(cmd)


BENCH = os.path.join(ROOT, "tests", "cpp", "build", "benchmark_antt")


def _build_bench():
    os.makedirs(os.path.dirname(BENCH), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "binius-ntt_amd", "host", "ulvt"),
                           os.path.join(ROOT, "tools", "cpp", "benchmark_antt.cpp"), "-o", BENCH,
                           "-L", LIBDIR, "-lbinius_ntt_amd", "-L", ORACLE, "-loracle",
                           "-Wl,-rpath," + LIBDIR, "-Wl,-rpath," + ORACLE, "-Wl,--allow-shlib-undefined"])


def test_cpp_mirror_builds_against_the_c_abi():
    _build()
    assert os.path.exists(BIN)
    _build("test_prime_field.cpp", PRIME_BIN)
    assert os.path.exists(PRIME_BIN)
    _build_bench()
    assert os.path.exists(BENCH)


@pytest.mark.gpu
def test_benchmark_antt_harness_all_pass(ntt_md5, tmp_path):
    # the benchmark_antt.cu table (both kernel variants, every row checked against the MD5 table)
    _build_bench()
    hashes = tmp_path / "hashes.txt"
    hashes.write_text("".join("%d %s\n" % (i, h) for i, h in enumerate(ntt_md5["0"]) if h))
    p = subprocess.run([BENCH, str(hashes), "20"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "Modified tests passed: 20/20" in p.stdout


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


@pytest.mark.gpu
def test_cpp_prime_field_mirror_runs_reference_flows():
    _build("test_prime_field.cpp", PRIME_BIN)
    with open(os.path.join(ROOT, "tests", "golden", "bb31_ntt_md5.json")) as f:
        want = json.load(f)["hashes"]
    p = subprocess.run([PRIME_BIN], capture_output=True, text=True, timeout=300)
    out = p.stdout.splitlines()
    assert p.returncode == 0, p.stdout + p.stderr
    n = 0
    for line in out:
        if line.startswith("bbmd5 "):
            _, log_n, h = line.split()
            assert h == want[int(log_n)], line
            n += 1
    assert n == 22
    assert not [l for l in out if l.startswith("FAIL")]
    assert len([l for l in out if l.startswith("ok Prime Field Sumcheck Test")]) == 3


CIRCUITS_BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_circuits")


def test_generated_constant_operand_circuits_match_oracle():
    """bsm6_fma_w2 (the fold's scalar-challenge GF(2^64) product, sc_fold_pair), bsm5_fma_tw (the
    NTT's per-lane compact-twiddle product) and bsm5_mul_w (its scalar-twiddle top stage) run on
    the host against the oracle's tower product (CPU)."""
    os.makedirs(os.path.dirname(CIRCUITS_BIN), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROCM, "include"),
                           "-I", os.path.join(ROOT, "binius-ntt_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "test_circuits.cpp"), "-o", CIRCUITS_BIN,
                           "-L", ORACLE, "-loracle", "-Wl,-rpath," + ORACLE])
    p = subprocess.run([CIRCUITS_BIN], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "ok bsm6_fma_w2" in p.stdout and "ok bsm5_fma_tw" in p.stdout and "ok bsm5_mul_w" in p.stdout
