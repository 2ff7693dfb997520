#!/usr/bin/env python3
"""Generator of the wave-uniform-twiddle GF(2^32) bitsliced product.

When every lane of a wave multiplies by the same twiddle t (a stage whose butterflies all share one
twiddle within the wave), the product u ^= t * v need not run the variable-operand Karatsuba
circuit (1022 gates per 32 products, 243 of them ANDs with twiddle-bit masks). Instead:

  * the tower's top two levels are Karatsuba over GF(2^8) coefficients: GF(2^32) = GF(2^8)[X3][X4],
    so t * v is 9 products of a GF(2^8) constant c_k (a byte of t, or an XOR of bytes: scalar work)
    by an 8-word bitsliced GF(2^8) operand a_k (an XOR of v's coordinates);
  * each of those is a product by a KNOWN constant: an 8x8 GF(2) matrix, emitted as straight-line
    code for all 256 constants and selected by a uniform switch on c_k (scalar branches), with
    common pairs shared inside each case (Paar's greedy CSE) and XOR3 fusion;
  * the pre-sums and the recombination of the 9 products are emitted with the same XOR3 fusion as
    the multiplier circuits (gen_bitsliced.py's Emitter), the accumulation into u included.

Output: binius-ntt_amd/tools/uniform_gen.hpp (bn::gf8c_mul, bn::bsm5_fma_uniform; microbench6 only, not committed).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_bitsliced as G  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "uniform_gen.hpp")


def mul_alpha_int(a, h):
    if h == 0:
        return a & 1
    half = 1 << (h - 1)
    m = (1 << half) - 1
    a0, a1 = a & m, (a >> half) & m
    return a1 | ((a0 ^ mul_alpha_int(a1, h - 1)) << half)


def mul_int(a, b, h):
    """Fan-Paar tower product (binary_tower.cuh:35-50) on integers."""
    if h == 0:
        return a & b & 1
    half = 1 << (h - 1)
    m = (1 << half) - 1
    a0, a1, b0, b1 = a & m, (a >> half) & m, b & m, (b >> half) & m
    z0, z2 = mul_int(a0, b0, h - 1), mul_int(a1, b1, h - 1)
    z1 = mul_int(a0 ^ a1, b0 ^ b1, h - 1) ^ z0 ^ z2
    return (z0 ^ z2) | ((z1 ^ mul_alpha_int(z2, h - 1)) << half)


def paar(rows, nin):
    """Greedy common-pair elimination (Paar): rows are sets of input indices; returns (gates, rows)
    with gates = [(new_index, a, b)] defining new variables x_new = x_a ^ x_b."""
    rows = [set(r) for r in rows]
    gates = []
    nxt = nin
    while True:
        cnt = {}
        for r in rows:
            rl = sorted(r)
            for i in range(len(rl)):
                for j in range(i + 1, len(rl)):
                    cnt[(rl[i], rl[j])] = cnt.get((rl[i], rl[j]), 0) + 1
        if not cnt:
            break
        (a, b), c = max(cnt.items(), key=lambda kv: (kv[1], -kv[0][0], -kv[0][1]))
        if c < 2:
            break
        gates.append((nxt, a, b))
        for r in rows:
            if a in r and b in r:
                r.discard(a)
                r.discard(b)
                r.add(nxt)
        nxt += 1
    return gates, rows


def emit_const_case(c, acc=False, coords=1):
    """Statements computing out[i] = (c * x)_i (acc: out[i] ^= ...) for `coords` consecutive 8-word
    GF(2^8) coordinates of x, c a constant (every coordinate uses the same shared-pair plan)."""
    if coords > 1:
        lines, ng = [], 0
        for g in range(coords):
            l1, n1 = emit_const_case(c, acc, 1)
            off = 8 * g
            import re
            l1 = [re.sub(r"x\[(\d+)\]", lambda m: "x[%d]" % (int(m.group(1)) + off), l) for l in l1]
            l1 = [re.sub(r"out\[(\d+)\]", lambda m: "out[%d]" % (int(m.group(1)) + off), l) for l in l1]
            l1 = [re.sub(r"\bg(\d+)\b", lambda m: "g%d_%d" % (int(m.group(1)), g), l) for l in l1]
            lines += l1
            ng += n1
        return lines, ng
    # column j = c * e_j; row i has bit j set iff bit i of column j is set
    cols = [mul_int(c, 1 << j, 3) for j in range(8)]
    rows = [{j for j in range(8) if (cols[j] >> i) & 1} for i in range(8)]
    gates, rows = paar(rows, 8)
    # all 3-term XORs are fused (v_bitop3 XOR3); names: x0..x7 inputs, g8.. shared pairs
    name = {i: "x[%d]" % i for i in range(8)}
    lines = []
    for (k, a, b) in gates:
        name[k] = "g%d" % k
        lines.append("const uint32_t g%d = %s ^ %s;" % (k, name[a], name[b]))
    for i, r in enumerate(rows):
        terms = [name[t] for t in sorted(r)]
        if acc:
            if not terms:
                continue
            terms = ["out[%d]" % i] + terms
        if not terms:
            lines.append("out[%d] = 0u;" % i)
            continue
        acc = terms[0]
        rest = terms[1:]
        while rest:
            if len(rest) >= 2:
                acc = "BN_XOR3(%s, %s, %s)" % (acc, rest[0], rest[1])
                rest = rest[2:]
            else:
                acc = "(%s ^ %s)" % (acc, rest[0])
                rest = rest[1:]
        lines.append("out[%d] = %s;" % (i, acc))
    ngates = len(gates) + sum(max(0, (len(r) - 1 + 1) // 2) for r in rows)
    return lines, ngates


def gen_gf8c(acc=False, coords=1):
    body = ["switch (c & 255u) {"]
    total = 0
    for c in range(256):
        lines, ng = emit_const_case(c, acc, coords)
        total += ng
        body.append("case %d: {" % c)
        body += ["\t" + l for l in lines]
        body.append("\tbreak;")
        body.append("}")
    body.append("default: break;")
    body.append("}")
    return body, total / 256.0


def gen_fma_uniform():
    """u ^= t * v on 32 bitsliced GF(2^32) words with t uniform: the 9 GF(2^8)-coefficient
    Karatsuba products; returns (pre lines, post lines, the 9 (constant expr, operand index) pairs)."""
    # pre: operands a_k = 8-word XOR combinations of v's GF(2^8) coordinates v[8q .. 8q+7]
    d = G.DAG()
    v = [d.inp("v%d" % i) for i in range(32)]
    q = [v[8 * i: 8 * i + 8] for i in range(4)]  # coordinates of 1, X3, X4, X3X4
    lo16, hi16 = q[0] + q[1], q[2] + q[3]
    mid16 = G.vadd(d, lo16, hi16)
    ops = []
    for x in (lo16, hi16, mid16):  # level-16 products P_lo, P_hi, P_mid
        x0, x1 = x[:8], x[8:]
        ops += [x0, x1, G.vadd(d, x0, x1)]  # level-8 products q0, q2, q1
    pre_roots = [n for op in ops for n in op]
    imap = {"v%d" % i: "v[%d]" % i for i in range(32)}
    # operands that are plain input words need no instruction: keep their expressions
    e = G.Emitter(d, pre_roots)
    pre = e.emit(imap, [("a[%d]" % i, r) for i, r in enumerate(pre_roots)])
    # constants (scalar): t = t0 + t1 X3 + t2 X4 + t3 X3 X4 (bytes)
    cexpr = []
    for (c0, c1) in (("tb0", "tb1"), ("tb2", "tb3"), ("(tb0 ^ tb2)", "(tb1 ^ tb3)")):
        cexpr += [c0, c1, "(%s ^ %s)" % (c0, c1)]
    # post: from the 9 products p_k (8 words each) and u, form u ^= t * v
    d2 = G.DAG()
    p = [[d2.inp("p%d_%d" % (k, i)) for i in range(8)] for k in range(9)]
    u = [d2.inp("u%d" % i) for i in range(32)]

    def comb8(z0, z2, z1):  # level-16 recombination (Karatsuba as in gen_bitsliced.karatsuba)
        lo = G.vadd(d2, z0, z2)
        hi = G.vadd(d2, G.vadd(d2, z1, lo), G.mul_alpha(d2, z2, 3))
        return lo + hi

    P = [comb8(p[3 * m], p[3 * m + 1], p[3 * m + 2]) for m in range(3)]  # P_lo, P_hi, P_mid
    lo = G.vadd(d2, P[0], P[1])
    hi = G.vadd(d2, G.vadd(d2, P[2], lo), G.mul_alpha(d2, P[1], 4))
    res = lo + hi
    roots = [d2.xor(u[i], res[i]) for i in range(32)]
    imap2 = {"p%d_%d" % (k, i): "p[%d]" % (8 * k + i) for k in range(9) for i in range(8)}
    imap2.update({"u%d" % i: "u[%d]" % i for i in range(32)})
    e2 = G.Emitter(d2, roots)
    post = e2.emit(imap2, [("u[%d]" % i, r) for i, r in enumerate(roots)])
    return pre, post, cexpr


def main():
    gf8, avg = gen_gf8c()
    pre, post, cexpr = gen_fma_uniform()
    parts = ["// GENERATED by binius-ntt_amd/tools/gen_uniform.py -- do not edit.",
             "// Products by a wave-uniform GF(2^8)/GF(2^32) constant on bitsliced operands (see the generator).",
             "#pragma once", "#include <hip/hip_runtime.h>", "#include <stdint.h>", '#include "bitsliced_gen.hpp"', "",
             "namespace bn {", ""]
    parts.append("// out = c * x for one bitsliced GF(2^8) coordinate (8 words), c uniform (0..255): one straight-line")
    parts.append("// case per constant (%.1f gates on average, XOR3-fused, shared pairs), scalar dispatch. Alias-unsafe." % avg)
    parts.append("__device__ __forceinline__ void gf8c_mul(uint32_t c, const uint32_t* __restrict__ x, uint32_t* __restrict__ out) {")
    parts += ["\t" + l for l in gf8] + ["}", ""]
    gf8x4, avg4 = gen_gf8c(acc=True, coords=4)
    parts.append("// out ^= c * x on the four GF(2^8) coordinates of a 32-word GF(2^32) limb (a GF(2^8) twiddle acts on")
    parts.append("// each coordinate alone), c uniform: %.1f gates on average, one scalar dispatch." % avg4)
    parts.append("__device__ __forceinline__ void gf8c_fma4(uint32_t c, const uint32_t* __restrict__ x, uint32_t* __restrict__ out) {")
    parts += ["\t" + l for l in gf8x4] + ["}", ""]
    parts.append("__device__ __forceinline__ void bsm3x4_fma_uniform(const uint32_t* __restrict__ v, uint32_t t, uint32_t* __restrict__ u) {")
    parts.append("\tgf8c_fma4(__builtin_amdgcn_readfirstlane(t), v, u);")
    parts += ["}", ""]
    npre, npost = G.count_ops(pre), G.count_ops(post)
    parts.append("// u ^= t * v, 32 bitsliced GF(2^32) words, t wave-uniform: %d pre-sum gates, 9 gf8c_mul, %d" % (npre, npost))
    parts.append("// recombination + accumulation gates (vs 1022 + 32 for the variable-operand circuit).")
    parts.append("__device__ __forceinline__ void bsm5_fma_uniform(const uint32_t* __restrict__ v, uint32_t t, uint32_t* __restrict__ u) {")
    parts.append("\tconst uint32_t ts = __builtin_amdgcn_readfirstlane(t);")
    parts.append("\tconst uint32_t tb0 = ts & 255u, tb1 = (ts >> 8) & 255u, tb2 = (ts >> 16) & 255u, tb3 = ts >> 24;")
    parts.append("\tuint32_t a[72], p[72];")
    parts += ["\t{"] + ["\t\t" + l for l in pre] + ["\t}"]
    for k in range(9):
        parts.append("\tgf8c_mul(%s, a + %d, p + %d);" % (cexpr[k], 8 * k, 8 * k))
    parts += ["\t{"] + ["\t\t" + l for l in post] + ["\t}"]
    parts += ["}", "", "}  // namespace bn", ""]
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print("gf8c average gates %.2f, pre %d, post %d, total ~%.0f" % (avg, npre, npost, npre + npost + 9 * avg), file=sys.stderr)


if __name__ == "__main__":
    main()
