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
            if op.startswith("csum:"):
                # compact twiddle combination: bits [0, half) of p ^ (p >> half)
                lines.append("const uint32_t %s = %s ^ (%s >> %s);" % (v, nm(args[0]), nm(args[0]), op[5:]))
            elif op.startswith("wleaf:"):
                # one twiddle bit broadcast to a whole word
                lines.append("const uint32_t %s = BN_BIT(%s, %s);" % (v, nm(args[0]), op[6:]))
            elif op == "and":
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


class ScalarLutEmitter(LutEmitter):
    """LutEmitter for circuits with a wave-uniform compact operand (gen_fma_w2): the nodes that
    depend on that operand only (its leaves, Karatsuba sums and their XORs) are scalar work and
    enter the 3-input cover as free inputs; the cover maps the vector network alone."""

    def __init__(self, dag, roots, scalar_inputs):
        super().__init__(dag, roots)
        self.scalar = set()
        for n, (op, args) in enumerate(dag.nodes):
            if op == "in":
                if args[0] in scalar_inputs:
                    self.scalar.add(n)
            elif all(a in self.scalar for a in args):
                self.scalar.add(n)

    def _cuts(self, order):
        d = self.d
        cuts = {}
        for n in order:
            op, args = d.nodes[n]
            if op == "in" or n in self.scalar:
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
            if d.nodes[n][0] == "in" or n in self.scalar:
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
            if n in mapped or d.nodes[n][0] == "in" or n in self.scalar:
                continue
            mapped[n] = best[n]
            need.extend(best[n])
        return mapped

    def emit(self, input_map, outputs, barrier_every=0):
        mapped = self.build()
        d = self.d
        # scalar nodes the cover reads, with their scalar arguments
        sneed = set()
        stack = [l for c in mapped.values() for l in c if l in self.scalar]
        while stack:
            n = stack.pop()
            if n in sneed or d.nodes[n][0] == "in":
                continue
            sneed.add(n)
            stack.extend(d.nodes[n][1])
        name = {}
        lines = []
        cnt = 0

        def nm(x):
            op, args = d.nodes[x]
            return input_map[args[0]] if op == "in" else name[x]
        for n in sorted(set(mapped) | sneed):
            v = "t%d" % cnt
            cnt += 1
            op, args = d.nodes[n]
            if n in sneed:
                if op.startswith("csum:"):
                    expr = "%s ^ (%s >> %s)" % (nm(args[0]), nm(args[0]), op[5:])
                elif op.startswith("wleaf:"):
                    expr = "BN_BIT(%s, %s)" % (nm(args[0]), op[6:])
                else:
                    expr = "%s %s %s" % (nm(args[0]), "&" if op == "and" else "^", nm(args[1]))
            else:
                leaves = sorted(mapped[n])
                tt = self._truth(n, leaves)
                a = [nm(l) for l in leaves]
                if len(leaves) == 2 and tt == 0xF0 ^ 0xCC:
                    expr = "%s ^ %s" % tuple(a)
                elif len(leaves) == 2 and tt == 0xF0 & 0xCC:
                    expr = "%s & %s" % tuple(a)
                else:
                    while len(a) < 3:
                        a.append(a[0])
                    expr = "BN_BITOP3(%s, %s, %s, 0x%02x)" % (a[0], a[1], a[2], tt)
            lines.append("const uint32_t %s = %s;" % (v, expr))
            name[n] = v
            if barrier_every and cnt % barrier_every == 0:
                lines.append("BN_SCHED_BARRIER();")
        for lv, r in outputs:
            lines.append("%s = %s;" % (lv, "0u" if r is None else nm(r)))
        self._selfcheck(outputs)
        return lines

    def _selfcheck(self, outputs, trials=4):
        """As LutEmitter's, with the scalar nodes as free random inputs on both sides."""
        import random
        d = self.d
        rnd = random.Random(1234)
        for _ in range(trials):
            ref = {}
            for i, (op, args) in enumerate(d.nodes):
                if op == "in" or i in self.scalar:
                    ref[i] = rnd.getrandbits(64)
            got = dict(ref)

            def ev_ref(x):
                if x in ref:
                    return ref[x]
                op, args = d.nodes[x]
                a, b = ev_ref(args[0]), ev_ref(args[1])
                ref[x] = (a & b) if op == "and" else (a ^ b)
                return ref[x]
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
                        r |= (a if (i >> 2) & 1 else ~a) & (b if (i >> 1) & 1 else ~b) & (c if i & 1 else ~c)
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
# gen_fma_w2: scheduling barriers keep the scalar leaf extractions next to their uses (without
# them the scheduler hoists the SALU work and its SGPRs spill)
W2_BARRIER_EVERY = int(os.environ.get("BN_GEN_W2_BARRIER_EVERY", "32"))
W2_LUT = int(os.environ.get("BN_GEN_W2_LUT", "1"))


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


def kara_w(d, a, cid, off, h):
    """Karatsuba product of bitsliced a (2^h words) with a twiddle given COMPACTLY: bits
    [off, off + 2^h) of the per-lane word node cid (the same value in all 32 bit-lanes). The
    twiddle side never exists as broadcast words: a sub-operand is a bit offset into a compact
    word (lo, hi halves) or a compact XOR of halves (one shift + XOR), and a leaf is one bit
    broadcast by v_bfe_i32. Costs ~80 more instructions than the broadcast-word form for GF(2^32)
    but keeps ~40 fewer registers live."""
    if h == 0:
        return [d.and_(a[0], d.node("wleaf:%d" % off, (cid,)))]
    half = 1 << (h - 1)
    a0, a1 = a[:half], a[half:]
    z0 = kara_w(d, a0, cid, off, h - 1)
    z2 = kara_w(d, a1, cid, off + half, h - 1)
    if h == 1:
        wsum = d.xor(d.node("wleaf:%d" % off, (cid,)), d.node("wleaf:%d" % (off + 1), (cid,)))
        z1 = [d.and_(d.xor(a0[0], a1[0]), wsum)]
    else:
        z1 = kara_w(d, vadd(d, a0, a1), d.node("csum:%d" % half, (cid,)), off, h - 1)
    lo = vadd(d, z0, z2)
    hi = vadd(d, vadd(d, z1, lo), mul_alpha(d, z2, h - 1))
    return lo + hi


def kara_w_multi(d, aa, cid, off, h):
    """kara_w for several data operands sharing one compact twiddle, recursing over all of them in
    lockstep: every twiddle leaf is extracted once and used at once by each operand, so no leaf
    outlives its uses (the compiler CSEs the leaves of separately inlined products and keeps all
    of them live)."""
    if h == 0:
        leaf = d.node("wleaf:%d" % off, (cid,))
        return [[d.and_(a[0], leaf)] for a in aa]
    half = 1 << (h - 1)
    z0 = kara_w_multi(d, [a[:half] for a in aa], cid, off, h - 1)
    z2 = kara_w_multi(d, [a[half:] for a in aa], cid, off + half, h - 1)
    if h == 1:
        wsum = d.xor(d.node("wleaf:%d" % off, (cid,)), d.node("wleaf:%d" % (off + 1), (cid,)))
        z1 = [[d.and_(d.xor(a[0], a[1]), wsum)] for a in aa]
    else:
        z1 = kara_w_multi(d, [vadd(d, a[:half], a[half:]) for a in aa], d.node("csum:%d" % half, (cid,)), off, h - 1)
    out = []
    for k in range(len(aa)):
        lo = vadd(d, z0[k], z2[k])
        hi = vadd(d, vadd(d, z1[k], lo), mul_alpha(d, z2[k], h - 1))
        out.append(lo + hi)
    return out


def gen_fma_tw_multi(h, cnt):
    """out ^= a * w on cnt consecutive 2^h-word coordinates of a 32-bit limb (a GF(2^(2^h)) twiddle
    acts on each sub-field coordinate of the tower representation on its own), twiddle leaves
    shared by the cnt products; eager accumulation at the top level as gen_fma_tw."""
    d = DAG()
    n = 1 << h
    half = n >> 1
    a = [[d.inp("a%d" % (c * n + i)) for i in range(n)] for c in range(cnt)]
    w = d.inp("w")
    o = [[d.inp("o%d" % (c * n + i)) for i in range(n)] for c in range(cnt)]
    z2 = kara_w_multi(d, [x[half:] for x in a], w, half, h - 1)
    for c in range(cnt):
        az2 = mul_alpha(d, z2[c], h - 1)
        o[c] = [d.xor(o[c][i], z2[c][i]) for i in range(half)] + [d.xor(d.xor(o[c][half + i], z2[c][i]), az2[i]) for i in range(half)]
    z0 = kara_w_multi(d, [x[:half] for x in a], w, 0, h - 1)
    for c in range(cnt):
        o[c] = [d.xor(o[c][i], z0[c][i]) for i in range(half)] + [d.xor(o[c][half + i], z0[c][i]) for i in range(half)]
    z1 = kara_w_multi(d, [vadd(d, x[:half], x[half:]) for x in a], d.node("csum:%d" % half, (w,)), 0, h - 1)
    for c in range(cnt):
        o[c] = o[c][:half] + [d.xor(o[c][half + i], z1[c][i]) for i in range(half)]
    flat = [x for oc in o for x in oc]
    imap = {"a%d" % i: "a[%d]" % i for i in range(cnt * n)}
    imap["w"] = "w"
    imap.update({"o%d" % i: "out[%d]" % i for i in range(cnt * n)})
    e = Emitter(d, flat)
    return e.emit(imap, [("out[%d]" % i, flat[i]) for i in range(cnt * n)], BARRIER_EVERY)


def kara_multi(d, aa, b, h):
    """karatsuba() for several a operands sharing one b, in lockstep (see kara_w_multi)."""
    if h == 0:
        return [[d.and_(a[0], b[0])] for a in aa]
    half = 1 << (h - 1)
    z0 = kara_multi(d, [a[:half] for a in aa], b[:half], h - 1)
    z2 = kara_multi(d, [a[half:] for a in aa], b[half:], h - 1)
    z1 = kara_multi(d, [vadd(d, a[:half], a[half:]) for a in aa], vadd(d, b[:half], b[half:]), h - 1)
    out = []
    for k in range(len(aa)):
        lo = vadd(d, z0[k], z2[k])
        hi = vadd(d, vadd(d, z1[k], lo), mul_alpha(d, z2[k], h - 1))
        out.append(lo + hi)
    return out


def gen_acc_multi(h, cnt):
    """out ^= a * b on cnt consecutive 2^h-word coordinates of a, b (2^h words) shared, in lockstep
    with eager top-level accumulation (the in-word stages' sub-field twiddle words)."""
    d = DAG()
    n = 1 << h
    half = n >> 1
    a = [[d.inp("a%d" % (c * n + i)) for i in range(n)] for c in range(cnt)]
    b = [d.inp("b%d" % i) for i in range(n)]
    o = [[d.inp("o%d" % (c * n + i)) for i in range(n)] for c in range(cnt)]
    z2 = kara_multi(d, [x[half:] for x in a], b[half:], h - 1)
    for c in range(cnt):
        az2 = mul_alpha(d, z2[c], h - 1)
        o[c] = [d.xor(o[c][i], z2[c][i]) for i in range(half)] + [d.xor(d.xor(o[c][half + i], z2[c][i]), az2[i]) for i in range(half)]
    z0 = kara_multi(d, [x[:half] for x in a], b[:half], h - 1)
    for c in range(cnt):
        o[c] = [d.xor(o[c][i], z0[c][i]) for i in range(half)] + [d.xor(o[c][half + i], z0[c][i]) for i in range(half)]
    z1 = kara_multi(d, [vadd(d, x[:half], x[half:]) for x in a], vadd(d, b[:half], b[half:]), h - 1)
    for c in range(cnt):
        o[c] = o[c][:half] + [d.xor(o[c][half + i], z1[c][i]) for i in range(half)]
    flat = [x for oc in o for x in oc]
    imap = {"a%d" % i: "a[%d]" % i for i in range(cnt * n)}
    imap.update({"b%d" % i: "b[%d]" % i for i in range(n)})
    imap.update({"o%d" % i: "out[%d]" % i for i in range(cnt * n)})
    e = Emitter(d, flat)
    return e.emit(imap, [("out[%d]" % i, flat[i]) for i in range(cnt * n)], BARRIER_EVERY)


def gen_fma_tw(h):
    """out ^= a * w with w a compact GF(2^(2^h)) value per lane (the same twiddle for the lane's
    32 bitsliced elements). Top level accumulated eagerly (z2, z0, z1 go into out as soon as each
    is formed), so at most one half-size partial product is live beside a and out."""
    d = DAG()
    n = 1 << h
    half = n >> 1
    a = [d.inp("a%d" % i) for i in range(n)]
    w = d.inp("w")
    o = [d.inp("o%d" % i) for i in range(n)]
    a0, a1 = a[:half], a[half:]
    z2 = kara_w(d, a1, w, half, h - 1)
    az2 = mul_alpha(d, z2, h - 1)
    o = [d.xor(o[i], z2[i]) for i in range(half)] + [d.xor(d.xor(o[half + i], z2[i]), az2[i]) for i in range(half)]
    z0 = kara_w(d, a0, w, 0, h - 1)
    o = [d.xor(o[i], z0[i]) for i in range(half)] + [d.xor(o[half + i], z0[i]) for i in range(half)]
    z1 = kara_w(d, vadd(d, a0, a1), d.node("csum:%d" % half, (w,)), 0, h - 1)
    o = o[:half] + [d.xor(o[half + i], z1[i]) for i in range(half)]
    imap = {"a%d" % i: "a[%d]" % i for i in range(n)}
    imap["w"] = "w"
    imap.update({"o%d" % i: "out[%d]" % i for i in range(n)})
    e = Emitter(d, o)
    return e.emit(imap, [("out[%d]" % i, o[i]) for i in range(n)], BARRIER_EVERY)


def gen_fma_w2():
    """out ^= a * (w0 + w1 X) in GF(2^64): a is 64 bitsliced words, w0 and w1 are the compact
    GF(2^32) halves of a constant that is the same for every lane of the wave (the sumcheck fold's
    challenge, sc_fold_pair). The twiddle side (leaves, Karatsuba sums of the halves) is then
    scalar work; the vector side is the three GF(2^32) circuits' data half only. Top level
    accumulated eagerly as gen_fma_tw."""
    d = DAG()
    n, half = 64, 32
    a = [d.inp("a%d" % i) for i in range(n)]
    w0, w1 = d.inp("w0"), d.inp("w1")
    o = [d.inp("o%d" % i) for i in range(n)]
    a0, a1 = a[:half], a[half:]
    z2 = kara_w(d, a1, w1, 0, 5)
    az2 = mul_alpha(d, z2, 5)
    o = [d.xor(o[i], z2[i]) for i in range(half)] + [d.xor(d.xor(o[half + i], z2[i]), az2[i]) for i in range(half)]
    z0 = kara_w(d, a0, w0, 0, 5)
    o = [d.xor(o[i], z0[i]) for i in range(half)] + [d.xor(o[half + i], z0[i]) for i in range(half)]
    z1 = kara_w(d, vadd(d, a0, a1), d.xor(w0, w1), 0, 5)
    o = o[:half] + [d.xor(o[half + i], z1[i]) for i in range(half)]
    imap = {"a%d" % i: "a[%d]" % i for i in range(n)}
    imap.update({"w0": "w0", "w1": "w1"})
    imap.update({"o%d" % i: "out[%d]" % i for i in range(n)})
    e = ScalarLutEmitter(d, o, ("w0", "w1")) if W2_LUT else Emitter(d, o)
    return e.emit(imap, [("out[%d]" % i, o[i]) for i in range(n)], W2_BARRIER_EVERY)


def gen_mul_w(h):
    """out = a * w in GF(2^(2^h)), w compact and wave-uniform (the NTT's top block stage of a tile,
    whose twiddle depends on no tile bit): the twiddle side is scalar work as in gen_fma_w2."""
    d = DAG()
    n = 1 << h
    a = [d.inp("a%d" % i) for i in range(n)]
    w = d.inp("w")
    res = kara_w(d, a, w, 0, h)
    imap = {"a%d" % i: "a[%d]" % i for i in range(n)}
    imap["w"] = "w"
    e = ScalarLutEmitter(d, res, ("w",))
    return e.emit(imap, [("out[%d]" % i, res[i]) for i in range(n)], W2_BARRIER_EVERY)


def gen_acc(h):
    """out ^= a * b (out must not alias a or b): the product's last XOR per word also takes the
    accumulator, so the register-tile butterflies (u ^= w*v) need no product array."""
    d = DAG()
    n = 1 << h
    half = n >> 1
    a = [d.inp("a%d" % i) for i in range(n)]
    b = [d.inp("b%d" % i) for i in range(n)]
    o = [d.inp("o%d" % i) for i in range(n)]
    # top level accumulated eagerly (as gen_fma_tw): z2, z0, z1 go into out as soon as formed
    a0, a1, b0, b1 = a[:half], a[half:], b[:half], b[half:]
    z2 = karatsuba(d, a1, b1, h - 1)
    az2 = mul_alpha(d, z2, h - 1)
    o = [d.xor(o[i], z2[i]) for i in range(half)] + [d.xor(d.xor(o[half + i], z2[i]), az2[i]) for i in range(half)]
    z0 = karatsuba(d, a0, b0, h - 1)
    o = [d.xor(o[i], z0[i]) for i in range(half)] + [d.xor(o[half + i], z0[i]) for i in range(half)]
    z1 = karatsuba(d, vadd(d, a0, a1), vadd(d, b0, b1), h - 1)
    roots = o[:half] + [d.xor(o[half + i], z1[i]) for i in range(half)]
    imap = {"a%d" % i: "a[%d]" % i for i in range(n)}
    imap.update({"b%d" % i: "b[%d]" % i for i in range(n)})
    imap.update({"o%d" % i: "out[%d]" % i for i in range(n)})
    e = make_emitter(d, roots, low_pressure=True)
    return e.emit(imap, [("out[%d]" % i, roots[i]) for i in range(n)], BARRIER_EVERY)


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
             "#define BN_BIT(x, i) ((uint32_t)__builtin_amdgcn_sbfe((int)(x), (i), 1))",
             "#else",
             "#define BN_BIT(x, i) (0u - (((x) >> (i)) & 1u))",
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
        # the register-tile NTT kernels (antt_rr.hip) use: the GF(2^32) limb products with a compact
        # twiddle (h = 5) or with twiddle words (in-word stages), and the sub-field forms on all the
        # coordinates of a limb at once (h = 3, 4)
        if h == 5:
            tl = gen_fma_tw(h)
            parts.append("// out ^= a * w, w compact (bits 0 .. 2^%d - 1 of a per-lane word); out must not alias a: %d gates" % (h, count_ops(tl)))
            parts.append(fn("void bsm%d_fma_tw(const uint32_t* __restrict__ a, uint32_t w, uint32_t* __restrict__ out)" % h, tl))
            stats.append((h, "fma_tw", count_ops(tl)))
            al = gen_acc(h)
            parts.append("// out ^= a * b (out must not alias a or b): %d gates" % count_ops(al))
            parts.append(fn("void bsm%d_mul_acc(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint32_t* __restrict__ out)" % h, al))
            stats.append((h, "acc", count_ops(al)))
        elif h in (3, 4):
            cnt = 32 >> h
            ml = gen_fma_tw_multi(h, cnt)
            parts.append("// out ^= a * w on the %d GF(2^%d) coordinates of 32-word limbs, w compact (bits 0 .. 2^%d - 1), twiddle leaves shared: %d gates" % (cnt, 1 << h, h, count_ops(ml)))
            parts.append(fn("void bsm%dx%d_fma_tw(const uint32_t* __restrict__ a, uint32_t w, uint32_t* __restrict__ out)" % (h, cnt), ml))
            stats.append((h, "fma_tw x%d" % cnt, count_ops(ml)))
            ml = gen_acc_multi(h, cnt)
            parts.append("// out ^= a * b on the %d GF(2^%d) coordinates of 32-word limbs, b shared (2^%d words): %d gates" % (cnt, 1 << h, h, count_ops(ml)))
            parts.append(fn("void bsm%dx%d_mul_acc(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint32_t* __restrict__ out)" % (h, cnt), ml))
            stats.append((h, "acc x%d" % cnt, count_ops(ml)))
    ml = gen_mul_w(5)
    parts.append("// out = a * w in GF(2^32), w compact and wave-uniform (scalar leaves); out must not alias a: %d gates" % count_ops(ml))
    parts.append(fn("void bsm5_mul_w(const uint32_t* __restrict__ a, uint32_t w, uint32_t* __restrict__ out)", ml))
    stats.append((5, "mul_w", count_ops(ml)))
    wl = gen_fma_w2()
    parts.append("// out ^= a * (w0 + w1 X) in GF(2^64), w0 / w1 compact and wave-uniform (scalar leaves); out must not alias a: %d gates" % count_ops(wl))
    parts.append(fn("void bsm6_fma_w2(const uint32_t* __restrict__ a, uint32_t w0, uint32_t w1, uint32_t* __restrict__ out)", wl))
    stats.append((6, "fma_w2", count_ops(wl)))
    parts.append("}  // namespace bn")
    with open(OUT, "w") as f:
        f.write("\n".join(parts) + "\n")
    for s in stats:
        print(s, file=sys.stderr)


if __name__ == "__main__":
    main()
