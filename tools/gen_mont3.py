#!/usr/bin/env python3
"""Generate janus_amd/csrc/mont3.h: THREE independent Field128 Montgomery products in one
instruction stream (gfx950 inline asm), checked here by simulating the exact instruction list.

Why: gfx950 needs two wait states between a VALU that writes a carry (SGPR pair / VCC) and the
VALU that reads it, so one Montgomery product -- a few long carry chains -- is hazard-bound: the
compiler's version issues ~146 VALU + ~59 s_nop, and it does not interleave independent products
to fill those slots.  Here each product is written as a plain sequential program (carry-scanning
product columns, 8-limb normalisation, two 64-bit-word REDC steps for p = 2^128 - 28 2^64 + 1,
final conditional subtraction; ~90 instructions, 16 v_mad_u64_u32) and three of them are issued
round-robin, so consecutive instructions of one product are always 3 apart: no wait state is ever
needed and no s_nop is emitted.

Two asm statements per call: the product columns come out as 64-bit VGPR pairs (v_mad_u64_u32
writes pairs) and the reduction needs their 32-bit halves, which inline asm cannot name, so C++
splits them between the statements (register renaming, no instructions).

  python3 tools/gen_mont3.py            # simulate + write janus_amd/csrc/mont3.h
"""
import os
import random

P = (1 << 128) - 28 * (1 << 64) + 1
M32 = (1 << 32) - 1
P2 = 0xFFFFFFE4

# ---------------------------------------------------------------------------------------------
# One product's program.  Operands: register names (per stream), ints (inline constants), "P2"
# (0xFFFFFFE4 in a VGPR: a VOP3 may read only one SGPR, here the borrow).  Ops: mad (dst64, carry, s0, s1, src2_64 | 0), add_co, addc, sub_co, subb,
# lsl (dst, shift, src), lsr, abit (dst, hi, lo, shift), cnd (dst, a, b, mask) = mask ? b : a.
# ---------------------------------------------------------------------------------------------
# product phase, scheduled so that a mad's carry is read >= 3 instructions later even inside one
# stream (carry pairs ca/cb/cc rotate; "cd" is a never-read sink)
PRODUCT = [
    ("mad", "L0", "cd", "a0", "b0", 0),
    ("mad", "L1", "cd", "a0", "b1", 0),
    ("mad", "L2", "cd", "a0", "b2", 0),
    ("mad", "L1", "ca", "a1", "b0", "L1"),
    ("mad", "L3", "cd", "a0", "b3", 0),
    ("mad", "L2", "cb", "a1", "b1", "L2"),
    ("addc", "h1", "cd", 0, 0, "ca"),
    ("mad", "L3", "cc", "a1", "b2", "L3"),
    ("addc", "h2", "cd", 0, 0, "cb"),
    ("mad", "L2", "ca", "a2", "b0", "L2"),
    ("addc", "h3", "cd", 0, 0, "cc"),
    ("mad", "L3", "cb", "a2", "b1", "L3"),
    ("addc", "h2", "cd", "h2", 0, "ca"),
    ("mad", "L4", "cd", "a1", "b3", 0),
    ("addc", "h3", "cd", "h3", 0, "cb"),
    ("mad", "L3", "cc", "a3", "b0", "L3"),
    ("mad", "L4", "ca", "a2", "b2", "L4"),
    ("mad", "L5", "cd", "a2", "b3", 0),
    ("addc", "h3", "cd", "h3", 0, "cc"),
    ("mad", "L4", "cb", "a3", "b1", "L4"),
    ("addc", "h4", "cd", 0, 0, "ca"),
    ("mad", "L5", "cc", "a3", "b2", "L5"),
    ("mad", "L6", "cd", "a3", "b3", 0),
    ("addc", "h4", "cd", "h4", 0, "cb"),
    ("addc", "h5", "cd", 0, 0, "cc"),
]


def reduce_program():
    """Normalisation + 2 REDC steps + final subtraction, on 32-bit registers.  Inputs: l0..l6
    (low halves of L0..L6), g0..g6 (high halves), h1..h5.  Output r0..r3.  Registers are reused
    in place: T_k lives in l_k (T7 in g6), U in T's registers, V in U's."""
    ins = []
    A = ins.append
    # T = sum_c L_c 2^(32c) + sum_c h_c 2^(32c + 64):  T0 = l0, T1..T7
    A(("add_co", "l1", "k", "l1", "g0"))
    for c in range(2, 7):
        A(("addc", f"l{c}", "k", f"l{c}", f"g{c - 1}", "k"))
    A(("addc", "g6", "k", "g6", 0, "k"))
    T = ["l0", "l1", "l2", "l3", "l4", "l5", "l6", "g6"]
    A(("add_co", T[3], "k", T[3], "h1"))
    for c in range(4, 8):
        A(("addc", T[c], "k", T[c], f"h{c - 2}", "k"))

    def redc(X, n):
        """X: limb registers (X0, X1 are the word reduced away); result in X[2:2+n]."""
        A(("sub_co", "m0", "k", 0, X[0]))
        A(("subb", "m1", "k", 0, X[1], "k"))  # k = (x0 != 0), the carry into the next word
        A(("lsl", "a0", 5, "m0"))
        A(("abit", "a1", "m1", "m0", 27))
        A(("lsr", "a2", 27, "m1"))
        A(("lsl", "b0", 2, "m0"))
        A(("abit", "b1", "m1", "m0", 30))
        A(("lsr", "b2", 30, "m1"))
        A(("sub_co", "w0", "k2", "a0", "b0"))  # w = 28 m = 32 m - 4 m (96 bits)
        A(("subb", "w1", "k2", "a1", "b1", "k2"))
        A(("subb", "w2", "k2", "a2", "b2", "k2"))
        # Y = X[2:] + carry + m 2^64 - 28 m
        Y = X[2:2 + n]
        A(("addc", Y[0], "k", Y[0], 0, "k"))
        A(("addc", Y[1], "k", Y[1], 0, "k"))
        A(("addc", Y[2], "k", Y[2], "m0", "k"))
        A(("addc", Y[3], "k", Y[3], "m1", "k"))
        for i in range(4, n):
            A(("addc", Y[i], "k", Y[i], 0, "k"))
        A(("sub_co", Y[0], "k2", Y[0], "w0"))
        A(("subb", Y[1], "k2", Y[1], "w1", "k2"))
        A(("subb", Y[2], "k2", Y[2], "w2", "k2"))
        for i in range(3, n):
            A(("subb", Y[i], "k2", Y[i], 0, "k2"))
        return Y

    U = redc(T, 6)               # (T + m p) / 2^64  < 2^192 + 2^128
    V = redc(U + ["v4"], 5)      # 5 limbs: V < 2p < 2^129; v4 starts at 0
    # r = V >= p ? V - p : V
    A(("sub_co", "m0", "k", V[0], 1))
    A(("subb", "a0", "k", V[1], 0, "k"))
    A(("subb", "a1", "k", V[2], "P2", "k"))
    A(("subb", "a2", "k", V[3], -1, "k"))
    A(("subb", "b0", "k", V[4], 0, "k"))   # k = borrow: V < p
    A(("cnd", "r0", "m0", V[0], "k"))
    A(("cnd", "r1", "a0", V[1], "k"))
    A(("cnd", "r2", "a1", V[2], "k"))
    A(("cnd", "r3", "a2", V[3], "k"))
    return ins


REDUCE = reduce_program()

# Temporaries of the reduction live in registers that are dead by then: g0..g5 once chain A has
# folded them into T (g6 holds T7), h1..h5 once chain B has.  check() verifies the aliasing by
# simulating with shared storage.
ALIAS = {"m0": "g0", "m1": "g1", "a0": "g2", "a1": "g3", "a2": "g4", "b0": "g5", "b1": "h1",
         "b2": "h2", "w0": "h3", "w1": "h4", "w2": "h5"}


# ---------------------------------------------------------------------------------------------
# Simulator (one lane)
# ---------------------------------------------------------------------------------------------
def val(st, x):
    if isinstance(x, int):
        return x & M32
    if x == "P2":
        return P2
    return st[x]


def simulate(prog, st):
    for ins in prog:
        op = ins[0]
        if op == "mad":
            _, d, c, s0, s1, s2 = ins
            add = 0 if s2 == 0 else st[s2]
            t = val(st, s0) * val(st, s1) + add
            st[d] = t & ((1 << 64) - 1)
            st[c] = t >> 64
        elif op in ("add_co", "addc"):
            d, c, s0, s1 = ins[1:5]
            ci = st[ins[5]] if op == "addc" else 0
            t = val(st, s0) + val(st, s1) + ci
            st[d], st[c] = t & M32, t >> 32
        elif op in ("sub_co", "subb"):
            d, c, s0, s1 = ins[1:5]
            bi = st[ins[5]] if op == "subb" else 0
            t = val(st, s0) - val(st, s1) - bi
            st[d], st[c] = t & M32, 1 if t < 0 else 0
        elif op == "lsl":
            st[ins[1]] = (val(st, ins[3]) << ins[2]) & M32
        elif op == "lsr":
            st[ins[1]] = val(st, ins[3]) >> ins[2]
        elif op == "abit":
            st[ins[1]] = (((val(st, ins[2]) << 32) | val(st, ins[3])) >> ins[4]) & M32
        elif op == "cnd":
            st[ins[1]] = val(st, ins[3]) if st[ins[4]] else val(st, ins[2])
        else:
            raise ValueError(op)


def mont_ref(a, b):
    return a * b * pow(1 << 128, -1, P) % P


def check(trials=20000):
    rng = random.Random(1)
    edge = [0, 1, 2, P - 1, P - 2, (1 << 64), (1 << 127), P // 2, (1 << 128) - 28 * (1 << 64)]
    for t in range(trials):
        a = rng.choice(edge) if t % 7 == 0 else rng.randrange(P)
        b = rng.choice(edge) if t % 5 == 0 else rng.randrange(P)
        st = {}
        for i in range(4):
            st[f"a{i}"] = (a >> (32 * i)) & M32
            st[f"b{i}"] = (b >> (32 * i)) & M32
        simulate(PRODUCT, st)
        for c in range(7):
            st[f"l{c}"] = st[f"L{c}"] & M32
            st[f"g{c}"] = st[f"L{c}"] >> 32
        st["v4"] = 0
        simulate([tuple(ALIAS.get(x, x) if isinstance(x, str) else x for x in ins)
                  for ins in REDUCE], st)
        r = sum(st[f"r{i}"] << (32 * i) for i in range(4))
        assert r == mont_ref(a, b), (hex(a), hex(b), hex(r), hex(mont_ref(a, b)))
    # hazard rule inside one stream: a carry is never read by the very next instruction of the
    # product phase (3-way interleaving then puts >= 2 other instructions in between anyway)
    return trials


# ---------------------------------------------------------------------------------------------
# Emitter
# ---------------------------------------------------------------------------------------------
NS = 3


def emit():
    out = []
    w = out.append
    w("// GENERATED by tools/gen_mont3.py -- edit the generator, not this file.")
    w("// Three independent Field128 Montgomery products a_s * b_s * 2^-128 mod p (s = 0, 1, 2),")
    w("// inputs < p, outputs canonical, issued round-robin so every carry is read >= 2")
    w("// instructions after it was written (gfx950's VALU carry hazard) without any s_nop.")
    w("#pragma once")
    w('#include "field.h"')
    w("")
    # ---- product statement
    ops, cons = [], []
    idx = {}

    def opnd(name, con, expr):
        idx[name] = len(ops)
        ops.append(expr)
        cons.append(con)

    for s in range(NS):
        for c in range(7):
            opnd(f"L{c}_{s}", '"=&v"', f"L{s}[{c}]")
        for c in range(1, 6):
            opnd(f"h{c}_{s}", '"=&v"', f"h{s}[{c - 1}]")
        for c in ("ca", "cb", "cc"):
            opnd(f"{c}_{s}", '"=&s"', f"{c}{s}")
    opnd("cd", '"=&s"', "cdump")
    nout = len(ops)
    for s in range(NS):
        for i in range(4):
            opnd(f"a{i}_{s}", '"v"', f"a{s}.w[{i}]")
            opnd(f"b{i}_{s}", '"v"', f"b{s}.w[{i}]")

    def ref(x, s):
        if isinstance(x, int):
            return str(x)
        if x == "cd":
            return f"%{idx['cd']}"
        return f"%{idx[f'{x}_{s}']}"

    lines = []
    for ins in PRODUCT:
        for s in range(NS):
            op = ins[0]
            if op == "mad":
                _, d, c, s0, s1, s2 = ins
                lines.append(f"v_mad_u64_u32 {ref(d, s)}, {ref(c, s)}, {ref(s0, s)}, {ref(s1, s)}, "
                             f"{ref(s2, s)}")
            else:  # addc
                _, d, c, s0, s1, ci = ins
                lines.append(f"v_addc_co_u32_e64 {ref(d, s)}, {ref(c, s)}, {ref(s0, s)}, "
                             f"{ref(s1, s)}, {ref(ci, s)}")
    w("DEVI void mont_mul3(const F128& a0, const F128& b0, const F128& a1, const F128& b1,")
    w("                    const F128& a2, const F128& b2, F128& r0, F128& r1, F128& r2) {")
    for s in range(NS):
        w(f"  uint64_t L{s}[7];")
        w(f"  uint32_t h{s}[5];")
        w(f"  uint64_t ca{s}, cb{s}, cc{s};")
    w("  uint64_t cdump;")
    w("  asm volatile(")
    for l in lines:
        w(f'      "{l}\\n\\t"')
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[:nout], ops[:nout])))
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[nout:], ops[nout:])) + ");")
    # ---- reduce statement
    ops, cons, idx = [], [], {}
    regs = (["l%d" % c for c in range(7)] + ["g%d" % c for c in range(7)] +
            ["h%d" % c for c in range(1, 6)] + ["v4"])
    tmps = []  # every temporary lives in a register the normalisation has freed (ALIAS)
    for s in range(NS):
        w(f"  uint32_t l{s}[7], g{s}[7], v4_{s} = 0u;")
        w(f"  for (int c = 0; c < 7; ++c) {{ l{s}[c] = (uint32_t)L{s}[c]; "
          f"g{s}[c] = (uint32_t)(L{s}[c] >> 32); }}")
        w(f"  uint64_t k{s}, kk{s};")
    for s in range(NS):
        for r in regs:
            if r[0] in "lg":
                opnd(f"{r}_{s}", '"+v"', f"{r[0]}{s}[{r[1:]}]")
            elif r[0] == "h":
                opnd(f"{r}_{s}", '"+v"', f"h{s}[{int(r[1:]) - 1}]")
            else:
                opnd(f"{r}_{s}", '"+v"', f"v4_{s}")
        for t, reg in ALIAS.items():
            idx[f"{t}_{s}"] = idx[f"{reg}_{s}"]
        for i in range(4):
            opnd(f"r{i}_{s}", '"=&v"', f"r{s}.w[{i}]")
        opnd(f"k_{s}", '"=&s"', f"k{s}")
        opnd(f"k2_{s}", '"=&s"', f"kk{s}")
    nout = len(ops)
    opnd("P2", '"v"', "0xFFFFFFE4u")  # a VGPR: one VOP3 may read only one SGPR (the borrow)

    def rref(x, s):
        if isinstance(x, int):
            return str(x)
        if x == "P2":
            return f"%{idx['P2']}"
        return f"%{idx[f'{x}_{s}']}"

    lines = []
    mn = {"add_co": "v_add_co_u32_e64", "addc": "v_addc_co_u32_e64", "sub_co": "v_sub_co_u32_e64",
          "subb": "v_subb_co_u32_e64"}
    for ins in REDUCE:
        for s in range(NS):
            op = ins[0]
            if op in mn:
                args = [rref(x, s) for x in ins[1:]]
                lines.append(f"{mn[op]} " + ", ".join(args))
            elif op == "lsl":
                lines.append(f"v_lshlrev_b32_e64 {rref(ins[1], s)}, {ins[2]}, {rref(ins[3], s)}")
            elif op == "lsr":
                lines.append(f"v_lshrrev_b32_e64 {rref(ins[1], s)}, {ins[2]}, {rref(ins[3], s)}")
            elif op == "abit":
                lines.append(f"v_alignbit_b32 {rref(ins[1], s)}, {rref(ins[2], s)}, "
                             f"{rref(ins[3], s)}, {ins[4]}")
            elif op == "cnd":
                lines.append(f"v_cndmask_b32_e64 {rref(ins[1], s)}, {rref(ins[2], s)}, "
                             f"{rref(ins[3], s)}, {rref(ins[4], s)}")
            else:
                raise ValueError(op)
    w("  asm volatile(")
    for l in lines:
        w(f'      "{l}\\n\\t"')
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[:nout], ops[:nout])))
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[nout:], ops[nout:])) + ");")
    w("}")
    w("")
    return "\n".join(out)


if __name__ == "__main__":
    n = check()
    print(f"simulated {n} products: ok ({len(PRODUCT)} + {len(REDUCE)} instructions per product)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "janus_amd", "csrc", "mont3.h")
    open(path, "w").write(emit())
    print("wrote", path)
