#!/usr/bin/env python3
"""Bitsliced binary-tower multiplier generator (gfx950 flavour).

MI355X-native successor of the reference's circuit generator
(src/ulvt/finite_fields/circuit_generator/multiply_and_generate_circuit.cpp:86-241, which
symbolically executes the recursive Karatsuba tower multiply and prints one C statement per
gate). Differences that matter on CDNA4:

* gates are hash-consed (common subexpressions are computed once);
* XOR chains and AND->XOR pairs are fused into gfx950's 3-input v_bitop3_b32
  (XOR3 = 0x96, (a&b)^c = 0x6a) through __builtin_amdgcn_bitop3_b32 — hipcc does not form
  XOR3 on its own;
* every multiplier is alias-safe (all inputs are read before any output is written).

Word i of a bitsliced operand holds bit i (tower basis) of 32 independent field elements.
Output: binius-ntt_amd/csrc/bitsliced_gen.hpp
"""
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "bitsliced_gen.hpp")


class DAG:
    def __init__(self):
        self.nodes = []  # (op, args)  op in {'in','and','xor'}
        self.index = {}

    def node(self, op, args):
        if op == "xor":
            args = tuple(sorted(args))
        elif op == "and":
            args = tuple(sorted(args))
        key = (op, args)
        if key in self.index:
            return self.index[key]
        self.nodes.append(key)
        self.index[key] = len(self.nodes) - 1
        return len(self.nodes) - 1

    def inp(self, name):
        return self.node("in", (name,))

    def xor(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        if a == b:
            return None  # zero
        return self.node("xor", (a, b))

    def and_(self, a, b):
        if a is None or b is None:
            return None
        return self.node("and", (a, b))


def vadd(d, a, b):
    return [d.xor(x, y) for x, y in zip(a, b)]


def mul_alpha(d, a, h):
    """(a0 + a1 X)X = a1 + (a0 + a1 alpha_{h-1}) X   (binary_tower.cuh:83-93)."""
    if h == 0:
        return list(a)
    half = 1 << (h - 1)
    a0, a1 = a[:half], a[half:]
    return a1 + vadd(d, a0, mul_alpha(d, a1, h - 1))


def karatsuba(d, a, b, h):
    """Recursive Karatsuba tower product (binary_tower.cuh:35-50), built depth-first so that
    node creation order == a low-register-pressure evaluation order."""
    if h == 0:
        return [d.and_(a[0], b[0])]
    half = 1 << (h - 1)
    a0, a1, b0, b1 = a[:half], a[half:], b[:half], b[half:]
    z0 = karatsuba(d, a0, b0, h - 1)
    z2 = karatsuba(d, a1, b1, h - 1)
    z1 = karatsuba(d, vadd(d, a0, a1), vadd(d, b0, b1), h - 1)
    lo = vadd(d, z0, z2)
    hi = vadd(d, vadd(d, z1, lo), mul_alpha(d, z2, h - 1))
    return lo + hi


class Emitter:
    """Emit a DAG as straight-line HIP with XOR3 / ANDXOR fusion."""

    def __init__(self, dag, roots):
        self.d = dag
        self.roots = roots
        uses = [0] * len(dag.nodes)
        for i, (op, args) in enumerate(dag.nodes):
            if op != "in":
                for a in args:
                    uses[a] += 1
        for r in roots:
            if r is not None:
                uses[r] += 1
        self.uses = uses

    def emit(self, input_map, outputs, barrier_every=0):
        """input_map: name -> C expression; outputs: list of (C lvalue, node or None).
        barrier_every > 0 inserts a scheduling barrier every that many gates, which keeps the
        machine scheduler close to the (depth-first, low register pressure) emission order."""
        d = self.d
        live = set()
        stack = [r for _, r in outputs if r is not None]
        while stack:
            n = stack.pop()
            if n in live:
                continue
            live.add(n)
            op, args = d.nodes[n]
            if op != "in":
                stack.extend(args)
        # fusion decisions
        absorbed = set()
        fused = {}
        for n in sorted(live):
            op, args = d.nodes[n]
            if op != "xor":
                continue
            a, b = args
            cand = []
            for x, y in ((a, b), (b, a)):
                ox = d.nodes[x][0]
                if self.uses[x] == 1 and x not in absorbed and x not in fused and ox in ("xor", "and"):
                    cand.append((x, y))
            # prefer absorbing an XOR (saves a full gate) over an AND
            cand.sort(key=lambda t: 0 if d.nodes[t[0]][0] == "xor" else 1)
            if cand:
                x, y = cand[0]
                absorbed.add(x)
                fused[n] = (x, y)
        lines = []
        name = {}
        cnt = [0]

        def nm(n):
            return name[n]

        for n in sorted(live):
            op, args = d.nodes[n]
            if op == "in":
                name[n] = input_map[args[0]]
                continue
            if n in absorbed:
                continue
            v = "t%d" % cnt[0]
            cnt[0] += 1
            if op == "and":
                lines.append("const uint32_t %s = %s & %s;" % (v, nm(args[0]), nm(args[1])))
            elif n in fused:
                x, y = fused[n]
                ox, xargs = d.nodes[x]
                if ox == "xor":
                    lines.append("const uint32_t %s = BN_XOR3(%s, %s, %s);" % (v, nm(xargs[0]), nm(xargs[1]), nm(y)))
                else:
                    lines.append("const uint32_t %s = BN_ANDXOR(%s, %s, %s);" % (v, nm(xargs[0]), nm(xargs[1]), nm(y)))
            else:
                lines.append("const uint32_t %s = %s ^ %s;" % (v, nm(args[0]), nm(args[1])))
            name[n] = v
            if barrier_every and cnt[0] % barrier_every == 0:
                lines.append("BN_SCHED_BARRIER();")
        for lv, r in outputs:
            lines.append("%s = %s;" % (lv, "0u" if r is None else nm(r)))
        return lines


class LutEmitter:
    """Technology mapping of the AND/XOR DAG onto gfx950's v_bitop3_b32, which evaluates ANY
    3-input boolean function in one VALU instruction: enumerate the 3-feasible cuts of every node,
    pick a cover by area flow (a node whose value several cuts would recompute is kept when that
    is cheaper, re-derived inside each consumer's 3-input function when it is not), refine with
    the mapping's real reference counts, and emit one instruction per chosen cut with its truth
    table as the bitop3 immediate (imm bit (a<<2 | b<<1 | c) = f(a, b, c)). The result is
    checked against the DAG by random simulation before it is written."""

    K = 3
    CUTS_PER_NODE = 16

    def __init__(self, dag, roots):
        self.d = dag
        self.roots = [r for r in roots if r is not None]

    def _live(self):
        d = self.d
        live = set()
        stack = list(self.roots)
        while stack:
            n = stack.pop()
            if n in live:
                continue
            live.add(n)
            op, args = d.nodes[n]
            if op != "in":
                stack.extend(args)
        return sorted(live)

    def _cuts(self, order):
        d = self.d
        cuts = {}
        for n in order:
            op, args = d.nodes[n]
            if op == "in":
                cuts[n] = [frozenset([n])]
                continue
            a, b = args
            cs = set()
            for ca in cuts[a]:
                for cb in cuts[b]:
                    u = ca | cb
                    if len(u) <= self.K:
                        cs.add(u)
            cs = sorted(cs, key=lambda c: (len(c), sorted(c)))[: self.CUTS_PER_NODE]
            cuts[n] = cs + [frozenset([n])]
        return cuts

    def _map(self, order, cuts, refs):
        d = self.d
        af = {}
        best = {}
        for n in order:
            if d.nodes[n][0] == "in":
                af[n] = 0.0
                continue
            bc, bv = None, None
            for c in cuts[n]:
                if n in c:
                    continue
                v = 1.0 + sum(af[l] / max(1, refs.get(l, 1)) for l in c)
                if bv is None or v < bv - 1e-9 or (abs(v - bv) <= 1e-9 and len(c) < len(bc)):
                    bc, bv = c, v
            best[n] = bc
            af[n] = bv
        mapped = {}
        need = list(self.roots)
        while need:
            n = need.pop()
            if n in mapped or d.nodes[n][0] == "in":
                continue
            mapped[n] = best[n]
            need.extend(best[n])
        return mapped

    def _truth(self, n, leaves):
        d = self.d
        pats = (0xF0, 0xCC, 0xAA)
        val = {l: pats[i] for i, l in enumerate(leaves)}

        def ev(x):
            if x in val:
                return val[x]
            op, args = d.nodes[x]
            va, vb = ev(args[0]), ev(args[1])
            r = (va & vb) if op == "and" else (va ^ vb)
            val[x] = r
            return r
        return ev(n) & 0xFF

    def build(self):
        order = self._live()
        cuts = self._cuts(order)
        refs = {}
        for n in order:
            op, args = self.d.nodes[n]
            if op != "in":
                for a in args:
                    refs[a] = refs.get(a, 0) + 1
        mapped = self._map(order, cuts, refs)
        for _ in range(3):  # re-estimate fanouts from the current cover
            refs = {}
            for n, c in mapped.items():
                for l in c:
                    refs[l] = refs.get(l, 0) + 1
            for r in self.roots:
                refs[r] = refs.get(r, 0) + 1
            m2 = self._map(order, cuts, refs)
            if len(m2) >= len(mapped):
                break
            mapped = m2
        self.mapped = mapped
        return mapped

    def emit(self, input_map, outputs, barrier_every=0):
        mapped = self.build()
        d = self.d
        name = {}
        lines = []
        cnt = 0
        for n in sorted(mapped):
            leaves = sorted(mapped[n])
            tt = self._truth(n, leaves)
            args = []
            for l in leaves:
                args.append(input_map[d.nodes[l][1][0]] if d.nodes[l][0] == "in" else name[l])
            v = "t%d" % cnt
            cnt += 1
            if len(leaves) == 2 and tt == 0xF0 ^ 0xCC:
                expr = "%s ^ %s" % tuple(args)
            elif len(leaves) == 2 and tt == 0xF0 & 0xCC:
                expr = "%s & %s" % tuple(args)
            else:
                while len(args) < 3:
                    args.append(args[0])  # the truth table ignores the padding operand
                expr = "BN_BITOP3(%s, %s, %s, 0x%02x)" % (args[0], args[1], args[2], tt)
            lines.append("const uint32_t %s = %s;" % (v, expr))
            name[n] = v
            if barrier_every and cnt % barrier_every == 0:
                lines.append("BN_SCHED_BARRIER();")
        for lv, r in outputs:
            if r is None:
                lines.append("%s = 0u;" % lv)
            elif d.nodes[r][0] == "in":
                lines.append("%s = %s;" % (lv, input_map[d.nodes[r][1][0]]))
            else:
                lines.append("%s = %s;" % (lv, name[r]))
        self._selfcheck(outputs)
        return lines

    def _selfcheck(self, outputs, trials=4):
        """Random 64-bit simulation: the mapped network equals the DAG on every output."""
        import random
        d = self.d
        rnd = random.Random(1234)
        for _ in range(trials):
            ref = {}
            for i, (op, args) in enumerate(d.nodes):
                if op == "in":
                    ref[i] = rnd.getrandbits(64)
            inputs = dict(ref)

            def ev_ref(x):
                if x in ref:
                    return ref[x]
                op, args = d.nodes[x]
                a, b = ev_ref(args[0]), ev_ref(args[1])
                ref[x] = (a & b) if op == "and" else (a ^ b)
                return ref[x]
            got = dict(inputs)
            for n in sorted(self.mapped):
                leaves = sorted(self.mapped[n])
                tt = self._truth(n, leaves)
                vals = [got[l] for l in leaves]
                while len(vals) < 3:
                    vals.append(vals[0])
                a, b, c = vals
                r = 0
                for i in range(8):
                    if (tt >> i) & 1:
                        ma = a if (i >> 2) & 1 else ~a
                        mb = b if (i >> 1) & 1 else ~b
                        mc = c if i & 1 else ~c
                        r |= ma & mb & mc
                got[n] = r & ((1 << 64) - 1)
            for _, r in outputs:
                if r is not None and got[r] != ev_ref(r):
                    raise AssertionError("LUT mapping differs from the DAG")


EMITTER = os.environ.get("BN_GEN_EMITTER", "auto")


def make_emitter(dag, roots, low_pressure=False):
    """auto: XOR3 / AND-XOR fusion (Emitter) for the circuits that run inside register-hungry
    kernels (the full GF(2^8..2^32) multiplies of the NTT passes and the sumcheck's quad product:
    the LUT cover re-derives nodes and reorders, and there it costs more in spills than it saves in
    gates — c4 d=3 4.5 -> 6.0 ms measured), the LUT mapping everywhere else."""
    if EMITTER == "lut" or (EMITTER == "auto" and not low_pressure):
        return LutEmitter(dag, roots)
    return Emitter(dag, roots)


def count_ops(lines):
    return sum(1 for l in lines if l.startswith("const uint32_t t"))


BARRIER_EVERY = int(os.environ.get("BN_GEN_BARRIER_EVERY", "0"))


def gen_full(h):
    """out = a * b, both bitsliced, alias-safe (every input word is read before any output word is
    written)."""
    d = DAG()
    n = 1 << h
    a = [d.inp("a%d" % i) for i in range(n)]
    b = [d.inp("b%d" % i) for i in range(n)]
    res = karatsuba(d, a, b, h)
    imap = {"a%d" % i: "a%d_" % i for i in range(n)}
    imap.update({"b%d" % i: "b%d_" % i for i in range(n)})
    e = make_emitter(d, res, low_pressure=h <= 5)
    body = e.emit(imap, [("out[%d]" % i, res[i]) for i in range(n)], BARRIER_EVERY if h <= 5 else 0)
    pre = ["const uint32_t a%d_ = a[%d];" % (i, i) for i in range(n)]
    pre += ["const uint32_t b%d_ = b[%d];" % (i, i) for i in range(n)]
    return pre + body


def fn(sig, lines):
    # host + device: the device build maps BN_BITOP3 onto v_bitop3_b32, the host build (the
    # reference's __host__ multiply_unrolled<H>, binary_tower_unrolled.cuh:4-5) onto plain logic
    return "__host__ __device__ __forceinline__ " + sig + " {\n\t" + "\n\t".join(lines) + "\n}\n"


def main():
    parts = ["// GENERATED by binius-ntt_amd/tools/gen_bitsliced.py -- do not edit.",
             "// Bitsliced binary-tower multipliers (Karatsuba tower, gfx950 v_bitop3 fusion).",
             "#pragma once", "#include <hip/hip_runtime.h>", "#include <stdint.h>", "",
             "// BN_BITOP3(a, b, c, imm): any 3-input boolean function, imm bit (a<<2 | b<<1 | c) = f(a, b, c)",
             "#if defined(__HIP_DEVICE_COMPILE__)",
             "#define BN_BITOP3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))",
             "#define BN_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)",
             "#else",
             "__host__ __device__ constexpr uint32_t bn_bitop3_host(uint32_t a, uint32_t b, uint32_t c, unsigned imm) {",
             "\tuint32_t r = 0;",
             "\tfor (unsigned i = 0; i < 8; i++)",
             "\t\tif ((imm >> i) & 1u) r |= ((i & 4u) ? a : ~a) & ((i & 2u) ? b : ~b) & ((i & 1u) ? c : ~c);",
             "\treturn r;",
             "}",
             "#define BN_BITOP3(a, b, c, imm) bn_bitop3_host((a), (b), (c), (imm))",
             "#define BN_SCHED_BARRIER()",
             "#endif",
             "#define BN_XOR3(a, b, c) BN_BITOP3((a), (b), (c), 0x96)",
             "#define BN_ANDXOR(a, b, c) BN_BITOP3((a), (b), (c), 0x6a)",
             "",
             "namespace bn {", ""]
    stats = []
    for h in (2, 3, 4, 5, 6, 7):
        fl = gen_full(h)
        parts.append("// full multiply: %d gates for 32 products" % count_ops(fl))
        parts.append(fn("void bsm%d_mul(const uint32_t* a, const uint32_t* b, uint32_t* out)" % h, fl))
        stats.append((h, "full", count_ops(fl)))
    parts.append("}  // namespace bn")
    with open(OUT, "w") as f:
        f.write("\n".join(parts) + "\n")
    for s in stats:
        print(s, file=sys.stderr)


if __name__ == "__main__":
    main()
