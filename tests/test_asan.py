"""Host-side sanitizer run (CPU; SURVEY.md section 5 "race detection / sanitizers"): the oracle, the
C++ host mirror and the library's host code built with AddressSanitizer + UBSan
(`make -C tests/cpp asan`: binius-ntt_amd/lib-asan + tests/cpp/build/test_host_asan) and run
without a GPU. tests/cpp/test_host_asan.cpp cross-checks the oracle's forms against each other, the
mirror's host classes and the library's host circuits against the oracle, and the C-ABI's error
paths; its MD5 lines are compared here with the reference's golden tables (test_ntt.cu:52-152)."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_host_asan")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_host_code_under_address_sanitizer():
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.check_call(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "tests", "cpp"), "asan"],
                          timeout=1500)
    env = dict(os.environ)
    # leak checking stays on; the HIP runtime's own allocations are not reported because the
    # library never initialises a device here
    env["ASAN_OPTIONS"] = "abort_on_error=0:halt_on_error=1:detect_leaks=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    p = subprocess.run([BIN], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-5000:]
    lines = p.stdout.splitlines()
    assert not [l for l in lines if l.startswith("FAIL")]
    assert sum(1 for l in lines if l.startswith("ok ")) >= 30
    with open(os.path.join(GOLDEN, "additive_ntt_md5.json")) as f:
        ntt = json.load(f)["hashes"]
    with open(os.path.join(GOLDEN, "bb31_ntt_md5.json")) as f:
        bb = json.load(f)["hashes"]
    n = 0
    for l in lines:
        w = l.split()
        if w[0] == "md5":
            assert w[3] == ntt[w[1]][int(w[2])], l
            n += 1
        elif w[0] == "bb31md5":
            assert w[2] == bb[int(w[1])], l
            n += 1
    assert n == 3
