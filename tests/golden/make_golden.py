#!/usr/bin/env python3
"""Regenerate the golden fixtures in this directory.

Data only: known-answer values and MD5 digests held by the reference's own tests,
parsed out of the reference test sources as text (no reference code is run or kept).

  additive_ntt_md5.json  <- src/ulvt/ntt/tests/test_ntt.cu:52-124   (additive_ntt_hashes[r][log_h])
  bb31_ntt_md5.json      <- src/ulvt/ntt/tests/test_ntt.cu:21-50    (bb31_ntt_hashes[log_len])
  field_kats.json        <- src/ulvt/finite_fields/tests/test_fanpaartower.cu:9-273
                            src/ulvt/finite_fields/tests/tests.cu:17-201
The reference holds no GF(2^128) NTT or sumcheck vectors; those paths are pinned by the
MD5 tables above (every limb plane of a GF(2^128) transform) and by the reference test's
protocol invariants (tests/test_gpu_sumcheck*.py), checked against the CPU oracle.

Usage: python tests/golden/make_golden.py [/root/reference]
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _read(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def ntt_hashes():
    src = _read("src/ulvt/ntt/tests/test_ntt.cu")
    start = src.index("additive_ntt_hashes[3][31][16]")
    body = src[start:src.index("};", start)]
    # split into the three log-rate groups by the top-level '// Log rate' comments
    groups = re.split(r"//\s*Log rate\s*(\d)", body)[1:]
    out = {}
    for i in range(0, len(groups), 2):
        r = int(groups[i])
        rows = re.findall(r"\{([^{}]*)\}", groups[i + 1])
        table = []
        for row in rows:
            vals = [int(v, 16) for v in re.findall(r"0x[0-9a-fA-F]+", row)]
            table.append(bytes(vals).hex() if len(vals) == 16 else None)
        out[str(r)] = table
    return out


def bb31_hashes():
    src = _read("src/ulvt/ntt/tests/test_ntt.cu")
    start = src.index("bb31_ntt_hashes[28][16]")
    body = src[start:src.index("};", start)]
    table = []
    for row in re.findall(r"\{([^{}]*)\}", body[body.index("=") + 1:]):
        vals = [int(v, 16) for v in re.findall(r"0x[0-9a-fA-F]+", row)]
        table.append(bytes(vals).hex() if len(vals) == 16 else None)
    return table


def field_kats():
    fp = _read("src/ulvt/finite_fields/tests/test_fanpaartower.cu")
    kats = {"mul32": [], "sqr32": [], "inv32": [], "simd16": [], "simd8": []}
    for a, b, c in re.findall(r"FanPaarTowerField<5>::multiply\((0x[0-9a-f]+),\s*(0x[0-9a-f]+)\)\s*==\s*(0x[0-9a-f]+)", fp):
        kats["mul32"].append([int(a, 16), int(b, 16), int(c, 16)])
    for a, c in re.findall(r"FanPaarTowerField<5>::square\((0x[0-9a-f]+)\)\s*==\s*(0x[0-9a-f]+)", fp):
        kats["sqr32"].append([int(a, 16), int(c, 16)])
    for a, c in re.findall(r"FanPaarTowerField<5>::inverse\((0x[0-9a-f]+)\)\s*==\s*(0x[0-9a-f]+)", fp):
        kats["inv32"].append([int(a, 16), int(c, 16)])
    for h, a, b, c in re.findall(r"mul_binary_tower_32b_simd<(\d)>\((0x[0-9a-f]+),\s*(0x[0-9a-f]+)\)\s*==\s*(0x[0-9a-f]+)", fp):
        key = {"4": "simd16", "3": "simd8"}.get(h)
        if key:
            kats[key].append([int(a, 16), int(b, 16), int(c, 16)])
    # bitsliced 128-bit KAT block (test_fanpaartower.cu:199-273): 4 elements a[], b[], results
    blk = fp[fp.index('TEST_CASE("Bitsliced 128-bit multiplications")'):]
    a_arr = re.search(r"uint32_t a\[WIDTH\] = \{([^}]*)\}", blk).group(1)
    b_arr = re.search(r"uint32_t b\[WIDTH\] = \{([^}]*)\}", blk).group(1)
    res = re.findall(r"results\[(\d+)\] == (0x[0-9a-f]+)", blk)
    kats["mul128_block"] = {
        "a": [int(v, 16) for v in re.findall(r"0x[0-9a-f]+", a_arr)],
        "b": [int(v, 16) for v in re.findall(r"0x[0-9a-f]+", b_arr)],
        "out": [int(v, 16) for _, v in sorted(res, key=lambda t: int(t[0]))],
    }
    t = _read("src/ulvt/finite_fields/tests/tests.cu")
    sa = re.search(r'field_elem_a_str = "(0x[0-9a-f]+)"', t).group(1)
    sb = re.search(r'field_elem_b_str = "(0x[0-9a-f]+)"', t).group(1)
    blk = t[t.index('TEST_CASE("mul_binary_tower_128b_bitsliced_unrolled"'):]
    res = re.findall(r"REQUIRE\(result\[(\d)\] == (0x[0-9a-f]+)\)", blk)
    words = [int(v, 16) for _, v in sorted(res)]
    c = sum(w << (32 * i) for i, w in enumerate(words))
    kats["mul128"] = [[int(sa, 16), int(sb, 16), c]]
    # packed-subfield products at heights 0, 2, 5 (tests.cu:68-95) and the interleave_32b KATs
    # (tests.cu:17-53: a/b/c/d assignments followed by REQUIREs in both directions)
    for h, a, b, c in re.findall(r"mul_binary_tower_32b_simd<(\d)>\((0x[0-9a-f]+),\s*(0x[0-9a-f]+)\)\s*==\s*(0x[0-9a-f]+)", t):
        kats.setdefault("simd_h%s" % h, []).append([int(a, 16), int(b, 16), int(c, 16)])
    blk = t[t.index('TEST_CASE("interleave_32b"'):t.index('TEST_CASE("interleave"')]
    env = {}
    kats["interleave32"] = []
    for m in re.finditer(r"(\w) = (0x[0-9a-f]+);|REQUIRE\(interleave_32b<(\d)>\((\w), (\w)\) == make_pair\((\w), (\w)\)\)", blk):
        if m.group(1):
            env[m.group(1)] = int(m.group(2), 16)
        else:
            h, x, y, u, v = m.group(3), m.group(4), m.group(5), m.group(6), m.group(7)
            kats["interleave32"].append([int(h), env[x], env[y], env[u], env[v]])
    return kats


if __name__ == "__main__":
    with open(os.path.join(HERE, "additive_ntt_md5.json"), "w") as f:
        json.dump({"source": "src/ulvt/ntt/tests/test_ntt.cu:52-124 (additive_ntt_hashes[log_rate][log_h]); "
                             "input std::mt19937(0xdeadbeef+log_h+log_rate), MD5 over output u32 words",
                   "hashes": ntt_hashes()}, f, indent=1)
    with open(os.path.join(HERE, "bb31_ntt_md5.json"), "w") as f:
        json.dump({"source": "src/ulvt/ntt/tests/test_ntt.cu:21-50 (bb31_ntt_hashes[log_len]); input "
                             "BB31(std::mt19937(0xdeadbeef+log_len)()), NTTConfRad2(BB31(137), 27, log_len), "
                             "MD5 over output asUInt32() words (test_ntt.cu:126-152)",
                   "hashes": bb31_hashes()}, f, indent=1)
    with open(os.path.join(HERE, "field_kats.json"), "w") as f:
        json.dump({"source": "src/ulvt/finite_fields/tests/test_fanpaartower.cu:9-273, tests.cu:17-95,172-201",
                   "kats": field_kats()}, f, indent=1)
    print("wrote", os.listdir(HERE))
