#!/usr/bin/env python3
"""Generate janus_amd/csrc/mont_fma.h: Field128 Montgomery products and FUSED product sums
    fma:  r = (a b + c d) 2^-128 mod p        mul:  r = a b 2^-128 mod p
issued as three interleaved instruction streams (gfx950 inline asm), every program checked here by
simulating the exact instruction list, including the register aliasing, and every carry read
checked against gfx950's VALU carry hazard (a VALU that writes an SGPR carry / VCC needs two wait
states before a VALU reads it): where the interleaving does not provide them, s_nop is emitted.

Why fused: a Montgomery product is 16 v_mad_u64_u32 + ~74 carry / shift instructions, of which
the two REDC steps and the final subtraction are ~2/3.  The fraction and Horner recurrences of
the FLP query (N d + a D, t pt + t^m c) are sums of two products: accumulating both products'
columns before ONE reduction saves ~30 % of their instructions (the sum is < 2 p^2 < 2^257, so
the reduction takes nine input words and ends with up to two conditional subtractions).

The operations of one function ("F" fused / "M" single) are independent and issue as one stream
each, round-robin; their product phases go into the first asm statement (64-bit column
accumulators, v_mad_u64_u32 writes pairs), their reductions into the second (32-bit halves: C++
splits the pairs between the statements, register renaming only).

  python3 tools/gen_mont_fma.py          # simulate + write janus_amd/csrc/mont_fma.h
"""
import os
import random

P = (1 << 128) - 28 * (1 << 64) + 1
M32 = (1 << 32) - 1
P2 = 0xFFFFFFE4
R = 1 << 128


# ---------------------------------------------------------------------------------------------
# programs of one operation (register names local to the operation, prefix added later)
# ---------------------------------------------------------------------------------------------
# operand pairs of a product sum: M = a b, F = a b + c d, Q = a b + c d + e f + i j
PAIRS = [("a", "b"), ("c", "d"), ("e", "f"), ("i", "j")]
KIND_PAIRS = {"M": 1, "F": 2, "Q": 4}


def npairs(fused):
    """number of operand pairs of an operation given as bool (fused) or int"""
    if isinstance(fused, bool):
        return 2 if fused else 1
    return fused


def product(fused, rename=False):
    """Column sums of a b (+ c d): L0..L6 (64-bit), carries h0..h6 (32-bit; h_c sits at
    2^(32 c + 64)).  Each mad's carry is read by the addc right after it (the interleave or the
    emitter's s_nop gives the wait states)."""
    ins = []
    first, hset = set(), set()
    pairs = PAIRS[:npairs(fused)]
    for (x, y) in pairs:
        for c in range(7):
            for i in range(4):
                j = c - i
                if not 0 <= j < 4:
                    continue
                if c not in first:
                    first.add(c)
                    ins.append(("mad", f"L{c}", "cd", f"{x}{i}", f"{y}{j}", 0))
                else:
                    cy = f"cy{c}" if rename else "cy"  # per-column carries let columns interleave
                    ins.append(("mad", f"L{c}", cy, f"{x}{i}", f"{y}{j}", f"L{c}"))
                    # the first carry into h_c sets it (h_c = 0 + 0 + carry), later ones add
                    ins.append(("addc", f"h{c}", "cd", f"h{c}" if c in hset else 0, 0, cy))
                    hset.add(c)
    return ins


def product_inits(fused):
    """carry words no mad of the product writes (a single product's outer columns hold one
    partial product each): zero-initialised in C, the rest are pure asm outputs"""
    written = {ins[1] for ins in product(fused) if ins[0] == "addc"}
    return [f"h{c}" for c in range(7) if f"h{c}" not in written]


def reduce_program(fused):
    """T = sum_c L_c 2^(32c) + sum_c h_c 2^(32c+64) -> (T / 2^128) mod p, canonical, in r0..r3.
    Inputs l0..l6 / g0..g6 (halves of L0..L6), h0..h6."""
    ins = []
    A = ins.append
    A(("add_co", "l1", "k", "l1", "g0"))
    for c in range(2, 7):
        A(("addc", f"l{c}", "k", f"l{c}", f"g{c - 1}", "k"))
    A(("addc", "g6", "k", "g6", 0, "k"))
    A(("addc", "h6", "k", "h6", 0, "k"))
    T = ["l0", "l1", "l2", "l3", "l4", "l5", "l6", "g6", "h6"]
    A(("add_co", T[2], "k", T[2], "h0"))
    for c in range(3, 8):
        A(("addc", T[c], "k", T[c], f"h{c - 2}", "k"))
    A(("addc", T[8], "k", T[8], 0, "k"))

    def redc(X, n):
        A(("sub_co", "m0", "k", 0, X[0]))
        A(("subb", "m1", "k", 0, X[1], "k"))
        A(("lsl", "a0", 5, "m0"))
        A(("abit", "a1", "m1", "m0", 27))
        A(("lsr", "a2", 27, "m1"))
        A(("lsl", "b0", 2, "m0"))
        A(("abit", "b1", "m1", "m0", 30))
        A(("lsr", "b2", 30, "m1"))
        A(("sub_co", "w0", "k2", "a0", "b0"))  # 28 m = 32 m - 4 m (96 bits)
        A(("subb", "w1", "k2", "a1", "b1", "k2"))
        A(("subb", "w2", "k2", "a2", "b2", "k2"))
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

    U = redc(T, 7)  # (T + m p) / 2^64 < 2^195: 7 words
    V = redc(U, 5)  # < (np + 1) p: 5 words
    if npairs(fused) == 4:
        # V < 5p: fold the top word with 2^128 = c (mod p), c = 28 2^64 - 1, then the modular
        # add's tail (exclusive flags: a wrap past 2^128 | W >= p) -- V = [l4, l5, l6, g6, h6]
        A(("lsl", "l0", 5, "h6"))
        A(("lsl", "l1", 2, "h6"))
        A(("vsub", "l0", "l0", "l1"))          # t = 28 V4
        A(("sub_co", "r0", "k", "l4", "h6"))   # W = V_lo - V4 ...
        A(("subb", "r1", "k", "l5", 0, "k"))
        A(("subb", "r2", "k", "l6", 0, "k"))
        A(("subb", "r3", "k", "g6", 0, "k"))
        A(("subb", "l1", "k", 0, 0, "k"))      # -borrow
        A(("add_co", "r2", "k2", "r2", "l0"))  # ... + t 2^64
        A(("addc", "r3", "k2", "r3", 0, "k2"))
        A(("addc", "l1", "k2", "l1", 0, "k2"))  # e = carry - borrow: W = W_lo + e 2^128
        A(("add_co", "l2", "k", "r0", -1))     # carry of W_lo + c: W_lo >= p
        A(("addc", "l2", "k", "r1", -1, "k"))
        A(("addc", "l2", "k", "r2", 27, "k"))
        A(("addc", "l2", "k", "r3", 0, "k"))
        A(("addc", "l1", "k", "l1", 0, "k"))   # sel = e + (W_lo >= p)
        A(("vsub", "l3", 0, "l1"))
        A(("and", "l2", 27, "l3"))
        A(("add_co", "r0", "k", "r0", "l3"))   # r = W_lo + (c & -sel) mod 2^128
        A(("addc", "r1", "k", "r1", "l3", "k"))
        A(("addc", "r2", "k", "r2", "l2", "k"))
        A(("addc", "r3", "k", "r3", 0, "k"))
        return ins
    # up to two conditional subtractions of p (one suffices for a single product: V < 2p)
    nsub = 1 if npairs(fused) == 1 else 2
    for rnd in range(nsub):
        A(("sub_co", "m0", "k", V[0], 1))
        A(("subb", "a0", "k", V[1], 0, "k"))
        A(("subb", "a1", "k", V[2], "P2", "k"))
        A(("subb", "a2", "k", V[3], -1, "k"))
        A(("subb", "b0", "k", V[4], 0, "k"))  # k = borrow: V < p
        dst = ["r0", "r1", "r2", "r3", None] if rnd == nsub - 1 else V
        A(("cnd", dst[0], "m0", V[0], "k"))
        A(("cnd", dst[1], "a0", V[1], "k"))
        A(("cnd", dst[2], "a1", V[2], "k"))
        A(("cnd", dst[3], "a2", V[3], "k"))
        if dst is V:
            A(("cnd", V[4], "b0", V[4], "k"))
    return ins


# temporaries of the reduction in registers the normalisation has freed
ALIAS = {"m0": "g0", "m1": "g1", "a0": "g2", "a1": "g3", "a2": "g4", "b0": "g5", "b1": "h1",
         "b2": "h2", "w0": "h3", "w1": "h4", "w2": "h5"}


# ---------------------------------------------------------------------------------------------
# simulator (one lane)
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
            t = val(st, s0) * val(st, s1) + (0 if s2 == 0 else st[s2])
            st[d] = t & ((1 << 64) - 1)
            st[c] = t >> 64
        elif op in ("add_co", "addc"):
            d, c, s0, s1 = ins[1:5]
            t = val(st, s0) + val(st, s1) + (st[ins[5]] if op == "addc" else 0)
            st[d], st[c] = t & M32, t >> 32
        elif op in ("sub_co", "subb"):
            d, c, s0, s1 = ins[1:5]
            t = val(st, s0) - val(st, s1) - (st[ins[5]] if op == "subb" else 0)
            st[d], st[c] = t & M32, 1 if t < 0 else 0
        elif op == "lsl":
            st[ins[1]] = (val(st, ins[3]) << ins[2]) & M32
        elif op == "lsr":
            st[ins[1]] = val(st, ins[3]) >> ins[2]
        elif op == "abit":
            st[ins[1]] = (((val(st, ins[2]) << 32) | val(st, ins[3])) >> ins[4]) & M32
        elif op == "cnd":
            st[ins[1]] = val(st, ins[3]) if st[ins[4]] else val(st, ins[2])
        elif op == "vsub":
            st[ins[1]] = (val(st, ins[2]) - val(st, ins[3])) & M32
        elif op == "and":
            st[ins[1]] = val(st, ins[2]) & val(st, ins[3])
        elif op == "nop":
            pass
        else:
            raise ValueError(op)


def aliased(prog):
    return [tuple(ALIAS.get(x, x) if isinstance(x, str) else x for x in ins) for ins in prog]


def run_op(fused, *vals):
    """vals: 2 np operands (a, b[, c, d[, e, f, i, j]])"""
    st = {}
    names = [x for pr in PAIRS[:npairs(fused)] for x in pr]
    for nm, v in zip(names, vals):
        for i in range(4):
            st[f"{nm}{i}"] = (v >> (32 * i)) & M32
    for c in range(7):
        st[f"h{c}"] = 0xDEADBEEF  # garbage: only product_inits are zeroed
    for h in product_inits(fused):
        st[h] = 0
    simulate(product(fused), st)
    for k in range(7):
        st[f"l{k}"], st[f"g{k}"] = st[f"L{k}"] & M32, st[f"L{k}"] >> 32
    simulate(aliased(reduce_program(fused)), st)
    return sum(st[f"r{i}"] << (32 * i) for i in range(4))


def check(trials=20000):
    rng = random.Random(7)
    edge = [0, 1, 2, P - 1, P - 2, 1 << 64, 1 << 127, P // 2, (1 << 128) - 28 * (1 << 64)]
    rinv = pow(R, -1, P)
    pick = lambda t, k: rng.choice(edge) if t % k == 0 else rng.randrange(P)
    for t in range(trials):
        a, b, c, d = pick(t, 7), pick(t, 5), pick(t, 3), pick(t, 11)
        assert run_op(False, a, b) == a * b * rinv % P, (a, b)
        assert run_op(True, a, b, c, d) == (a * b + c * d) * rinv % P, (a, b, c, d)
    for a, b in [(P - 1, P - 1), (P - 2, P - 1)]:  # the largest sums
        assert run_op(True, a, b, a, b) == 2 * a * b * rinv % P
        assert run_op(4, a, b, a, b, a, b, a, b) == 4 * a * b * rinv % P
    for t in range(trials):
        v = [pick(t + k, 3 + k) for k in range(8)]
        exp = (v[0] * v[1] + v[2] * v[3] + v[4] * v[5] + v[6] * v[7]) * rinv % P
        assert run_op(4, *v) == exp, v
    return trials


# ---------------------------------------------------------------------------------------------
# emitter: streams interleaved round-robin; s_nop wherever a carry would be read too early
# ---------------------------------------------------------------------------------------------
CARRY_OPS = {"mad": 2, "add_co": 2, "addc": 2, "sub_co": 2, "subb": 2}  # index of carry-out
WAIT = 2  # wait states between a VALU carry write and a VALU carry read


def interleave(streams):
    """streams: lists of (ins, stream_id).  Round-robin; returns the issue order with ("nop", n)
    entries so that every read of a carry register is >= WAIT + 1 slots after its write."""
    out = []
    last_write = {}  # register (stream-qualified) -> issue slot
    pos = [0] * len(streams)
    slot = 0
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k, s in enumerate(streams):
            if pos[k] >= len(s):
                continue
            ins, sid = s[pos[k]]
            pos[k] += 1
            reads = []
            op = ins[0]
            if op in ("addc", "subb"):
                reads.append(ins[5])
            elif op == "cnd":
                reads.append(ins[4])
            need = 0
            for r in reads:
                key = (sid, r)
                if key in last_write:
                    need = max(need, last_write[key] + WAIT + 1 - slot)
            if need > 0:
                out.append((("nop", need - 1), None))  # s_nop N waits N + 1 slots
                slot += need
            out.append((ins, sid))
            if op in CARRY_OPS:
                last_write[(sid, ins[CARRY_OPS[op]])] = slot
            slot += 1
    return out


def rw_sets(ins):
    """(registers read, registers written) of one instruction; the carry dump "cd" and the
    constant P2 carry no dependencies."""
    op = ins[0]
    if op == "mad":
        R, W = [ins[3], ins[4], ins[5]], [ins[1], ins[2]]
    elif op in ("add_co", "sub_co"):
        R, W = [ins[3], ins[4]], [ins[1], ins[2]]
    elif op in ("addc", "subb"):
        R, W = [ins[3], ins[4], ins[5]], [ins[1], ins[2]]
    elif op in ("lsl", "lsr"):
        R, W = [ins[3]], [ins[1]]
    elif op == "abit":
        R, W = [ins[2], ins[3]], [ins[1]]
    elif op == "cnd":
        R, W = [ins[2], ins[3], ins[4]], [ins[1]]
    elif op in ("vsub", "and"):
        R, W = [ins[2], ins[3]], [ins[1]]
    else:
        raise ValueError(op)
    R = [r for r in R if isinstance(r, str) and r not in ("P2", "cd")]
    W = [x for x in W if x != "cd"]
    return R, W


def carry_reads(ins):
    op = ins[0]
    return [ins[5]] if op in ("addc", "subb") else [ins[4]] if op == "cnd" else []


def list_schedule(streams):
    """streams: lists of (ins, stream_id), independent of each other.  Greedy list scheduling in
    round-robin priority: each slot issues the first instruction whose predecessors (RAW, WAR,
    WAW within its stream) have issued and whose carry inputs were written >= WAIT + 1 slots
    earlier; s_nop only when nothing is ready.  Same output form as interleave()."""
    order, pos = [], [0] * len(streams)
    while any(p < len(st) for p, st in zip(pos, streams)):
        for k, st in enumerate(streams):
            if pos[k] < len(st):
                order.append(st[pos[k]])
                pos[k] += 1
    n = len(order)
    deps = [[] for _ in range(n)]
    last_w, readers = {}, {}
    for i, (ins, sid) in enumerate(order):
        R, W = rw_sets(ins)
        cr = set(carry_reads(ins))
        for r in R:
            if (sid, r) in last_w:
                deps[i].append((last_w[(sid, r)], WAIT + 1 if r in cr else 1))
        for x in W:
            if (sid, x) in last_w:
                deps[i].append((last_w[(sid, x)], 1))
            deps[i] += [(j, 1) for j in readers.get((sid, x), []) if j != i]
        for r in R:
            readers.setdefault((sid, r), []).append(i)
        for x in W:
            last_w[(sid, x)] = i
            readers[(sid, x)] = []
    at = [None] * n
    out, slot, left = [], 0, list(range(n))
    while left:
        pick, wait = None, None
        for i in left:
            need, ok = 0, True
            for j, d in deps[i]:
                if at[j] is None:
                    ok = False
                    break
                need = max(need, at[j] + d - slot)
            if not ok:
                continue
            if need <= 0:
                pick = i
                break
            wait = need if wait is None else min(wait, need)
        if pick is None:
            out.append((("nop", wait - 1), None))
            slot += wait
            continue
        at[pick] = slot
        out.append(order[pick])
        left.remove(pick)
        slot += 1
    return out


def qualify(ins, sid):
    """register names of one instruction prefixed with its stream (the opcode and P2 kept)"""
    return (ins[0],) + tuple(f"{sid}.{x}" if isinstance(x, str) and x != "P2" else x
                             for x in ins[1:])


def check_schedule(sched, init, expect):
    """Run a scheduled stream (registers qualified by stream) on the simulator and check every
    carry read's distance to its write: init = {(sid, reg): value}, expect = {(sid, reg): value}."""
    st = {f"{sid}.{r}": v for (sid, r), v in init.items()}
    last, slot = {}, 0
    for ins, sid in sched:
        if ins[0] == "nop":
            slot += ins[1] + 1
            continue
        q = qualify(ins, sid)
        for r in carry_reads(ins):
            assert slot - last[(sid, r)] >= WAIT + 1, ("carry hazard", ins, sid)
        simulate([q], st)
        if ins[0] in CARRY_OPS:
            last[(sid, ins[CARRY_OPS[ins[0]]])] = slot
        slot += 1
    for (sid, r), v in expect.items():
        assert st[f"{sid}.{r}"] == v, ("schedule result", sid, r)


def verify_function(ops, progs, sched, rsched, trials=40):
    """The scheduled product and reduction streams of one generated function against Python
    integers, on random and edge operands, with the carry-hazard check of check_schedule."""
    rng = random.Random(len(sched) * 7 + len(rsched))
    edge = [0, 1, P - 1, P - 2, (1 << 128) - 28 * (1 << 64)]
    rinv = pow(R, -1, P)
    for t in range(trials):
        init, want, mid = {}, {}, {}
        for s, q, fused, tag in ops:
            names = [x for pr in PAIRS[:npairs(fused)] for x in pr]
            vals = [rng.choice(edge) if (t + k) % 5 == 0 else rng.randrange(P)
                    for k in range(len(names))]
            for i in range(4):
                for nm, v in zip(names, vals):
                    init[(tag, f"{nm}{i}")] = (v >> (32 * i)) & M32
            for c in range(7):
                init[(tag, f"h{c}")] = 0xDEADBEEF
            for h in product_inits(fused):
                init[(tag, h)] = 0
            want[tag] = sum(vals[2 * k] * vals[2 * k + 1] for k in range(len(names) // 2)) \
                * rinv % P
        st = {f"{sid}.{r}": v for (sid, r), v in init.items()}
        check_schedule(sched, init, {})
        # rerun to read the product state, split L into halves for the reduction
        for ins, sid in sched:
            if ins[0] != "nop":
                simulate([qualify(ins, sid)], st)
        rin = {}
        for s, q, fused, tag in ops:
            for c in range(7):
                Lc = st[f"{tag}.L{c}"]
                rin[(tag, f"l{c}")], rin[(tag, f"g{c}")] = Lc & M32, Lc >> 32
                rin[(tag, f"h{c}")] = st[f"{tag}.h{c}"]
        exp = {}
        for s, q, fused, tag in ops:
            for i in range(4):
                exp[(tag, f"r{i}")] = (want[tag] >> (32 * i)) & M32
        check_schedule(rsched, rin, exp)


def gen_function(name, spec, volatile=True):
    """spec: one string per stream of "M" (a b), "F" (a b + c d) or "Q" (a b + c d + e f + i j)
    operations, e.g. ["F", "F", "MM"].  Signature: for every operation in stream order, its
    operand pairs then its output."""
    ops = []  # (stream, op index in stream, number of operand pairs, tag)
    for s, st in enumerate(spec):
        for q, kind in enumerate(st):
            ops.append((s, q, KIND_PAIRS[kind], f"{s}{q}"))
    out = []
    w = out.append
    params = []
    for s, q, fused, tag in ops:
        for x, y in PAIRS[:fused]:
            params += [f"const F128& {x}{tag}", f"const F128& {y}{tag}"]
        params.append(f"F128& r{tag}")
    w(f"DEVI void {name}(" + ", ".join(params) + ") {")
    # ---- products ----
    ops_e, cons = [], []
    idx = {}

    def opnd(key, con, expr):
        idx[key] = len(ops_e)
        ops_e.append(expr)
        cons.append(con)

    rename = len(ops) <= 2  # per-column carries (7 SGPR pairs per product) for 1-2 products
    progs = {tag: product(fused, rename) for s, q, fused, tag in ops}
    carries = {tag: sorted({i[2] for i in pr if i[0] == "mad" and i[2] != "cd"})
               for tag, pr in progs.items()}
    for s, q, fused, tag in ops:
        w(f"  uint64_t L{tag}[7];")
        w(f"  uint32_t h{tag}[7];")
        for h in product_inits(fused):
            w(f"  h{tag}[{h[1:]}] = 0u;")
        w(f"  uint64_t " + ", ".join(f"{cy}_{tag}" for cy in carries[tag]) + ";")
    w("  uint64_t cdump;")
    for s, q, fused, tag in ops:
        for c in range(7):
            opnd(f"L{c}_{tag}", '"=&v"', f"L{tag}[{c}]")
        zero = product_inits(fused)
        for c in range(7):
            opnd(f"h{c}_{tag}", '"+v"' if f"h{c}" in zero else '"=&v"', f"h{tag}[{c}]")
        for cy in carries[tag]:
            opnd(f"{cy}_{tag}", '"=&s"', f"{cy}_{tag}")
    opnd("cd", '"=&s"', "cdump")
    nout = len(ops_e)
    for s, q, fused, tag in ops:
        for i in range(4):
            for x, y in PAIRS[:fused]:
                opnd(f"{x}{i}_{tag}", '"v"', f"{x}{tag}.w[{i}]")
                opnd(f"{y}{i}_{tag}", '"v"', f"{y}{tag}.w[{i}]")

    def ref(x, tag):
        if isinstance(x, int):
            return str(x)
        if x == "cd":
            return f"%{idx['cd']}"
        return f"%{idx[f'{x}_{tag}']}"

    # every operation is its own stream (they are independent); list-scheduled, then re-run on
    # the simulator and hazard-checked (verify_function)
    sched = list_schedule([[(ins, tag) for ins in progs[tag]] for (ss, q, fused, tag) in ops])
    rsched = list_schedule([[(ins, tag) for ins in aliased(reduce_program(fused))]
                            for (ss, q, fused, tag) in ops])
    verify_function(ops, progs, sched, rsched)
    lines = []
    for ins, tag in sched:
        if ins[0] == "nop":
            lines.append(f"s_nop {ins[1]}")
        elif ins[0] == "mad":
            _, d, c, s0, s1, s2 = ins
            lines.append(f"v_mad_u64_u32 {ref(d, tag)}, {ref(c, tag)}, {ref(s0, tag)}, "
                         f"{ref(s1, tag)}, {ref(s2, tag)}")
        else:
            _, d, c, s0, s1, ci = ins
            lines.append(f"v_addc_co_u32_e64 {ref(d, tag)}, {ref(c, tag)}, {ref(s0, tag)}, "
                         f"{ref(s1, tag)}, {ref(ci, tag)}")
    w("  asm volatile(" if volatile else "  asm(")
    for l in lines:
        w(f'      "{l}\\n\\t"')
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[:nout], ops_e[:nout])))
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[nout:], ops_e[nout:])) + ");")
    # ---- reductions ----
    ops_e, cons, idx = [], [], {}
    for s, q, fused, tag in ops:
        w(f"  uint32_t l{tag}[7], g{tag}[7];")
        w(f"  for (int c = 0; c < 7; ++c) {{ l{tag}[c] = (uint32_t)L{tag}[c]; "
          f"g{tag}[c] = (uint32_t)(L{tag}[c] >> 32); }}")
        w(f"  uint64_t k{tag}, kk{tag};")
    for s, q, fused, tag in ops:
        for c in range(7):
            opnd(f"l{c}_{tag}", '"+v"', f"l{tag}[{c}]")
            opnd(f"g{c}_{tag}", '"+v"', f"g{tag}[{c}]")
            opnd(f"h{c}_{tag}", '"+v"', f"h{tag}[{c}]")
        for t, reg in ALIAS.items():
            idx[f"{t}_{tag}"] = idx[f"{reg}_{tag}"]
        for i in range(4):
            opnd(f"r{i}_{tag}", '"=&v"', f"r{tag}.w[{i}]")
        opnd(f"k_{tag}", '"=&s"', f"k{tag}")
        opnd(f"k2_{tag}", '"=&s"', f"kk{tag}")
    nout = len(ops_e)
    opnd("P2", '"v"', "0xFFFFFFE4u")

    def rref(x, tag):
        if isinstance(x, int):
            return str(x)
        if x == "P2":
            return f"%{idx['P2']}"
        return f"%{idx[f'{x}_{tag}']}"

    sched = rsched
    mn = {"add_co": "v_add_co_u32_e64", "addc": "v_addc_co_u32_e64", "sub_co": "v_sub_co_u32_e64",
          "subb": "v_subb_co_u32_e64"}
    lines = []
    for ins, tag in sched:
        op = ins[0]
        if op == "nop":
            lines.append(f"s_nop {ins[1]}")
        elif op in mn:
            lines.append(f"{mn[op]} " + ", ".join(rref(x, tag) for x in ins[1:]))
        elif op == "lsl":
            lines.append(f"v_lshlrev_b32_e64 {rref(ins[1], tag)}, {ins[2]}, {rref(ins[3], tag)}")
        elif op == "lsr":
            lines.append(f"v_lshrrev_b32_e64 {rref(ins[1], tag)}, {ins[2]}, {rref(ins[3], tag)}")
        elif op == "abit":
            lines.append(f"v_alignbit_b32 {rref(ins[1], tag)}, {rref(ins[2], tag)}, "
                         f"{rref(ins[3], tag)}, {ins[4]}")
        elif op == "cnd":
            lines.append(f"v_cndmask_b32_e64 {rref(ins[1], tag)}, {rref(ins[2], tag)}, "
                         f"{rref(ins[3], tag)}, {rref(ins[4], tag)}")
        elif op == "vsub":
            lines.append(f"v_sub_u32_e64 {rref(ins[1], tag)}, {rref(ins[2], tag)}, "
                         f"{rref(ins[3], tag)}")
        elif op == "and":
            lines.append(f"v_and_b32_e64 {rref(ins[1], tag)}, {rref(ins[2], tag)}, "
                         f"{rref(ins[3], tag)}")
        else:
            raise ValueError(op)
    w("  asm volatile(" if volatile else "  asm(")
    for l in lines:
        w(f'      "{l}\\n\\t"')
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[:nout], ops_e[:nout])))
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[nout:], ops_e[nout:])) + ");")
    w("}")
    w("")
    nops = sum(int(l.split()[1]) + 1 for l in lines if l.startswith("s_nop"))
    return "\n".join(out), nops


# ---------------------------------------------------------------------------------------------
# modular additions / subtractions (inputs < p, outputs canonical), c = 2^128 - p = [-1, -1, 27, 0]
# ---------------------------------------------------------------------------------------------
def modadd_program():
    """r = a + b mod p: s = a + b (carry k1); k2 = carry of s + c; sel = k1 + k2 (they exclude
    each other: k1 = 1 means s - 2^128 < p - c); r = s + (c & -sel) mod 2^128.  16 VALU."""
    ins = [("add_co", "r0", "k", "a0", "b0")]
    for i in range(1, 4):
        ins.append(("addc", f"r{i}", "k", f"a{i}", f"b{i}", "k"))
    ins.append(("addc", "q", "k", 0, 0, "k"))  # q = k1
    # the detect chain has its own carry, so it can start as soon as r0 is formed
    ins.append(("add_co", "x", "k2", "r0", -1))
    ins.append(("addc", "x", "k2", "r1", -1, "k2"))
    ins.append(("addc", "x", "k2", "r2", 27, "k2"))
    ins.append(("addc", "x", "k2", "r3", 0, "k2"))
    ins.append(("addc", "q", "k2", "q", 0, "k2"))  # q = k1 + k2
    ins.append(("vsub", "m", 0, "q"))
    ins.append(("and", "x", 27, "m"))
    ins.append(("add_co", "r0", "k", "r0", "m"))
    ins.append(("addc", "r1", "k", "r1", "m", "k"))
    ins.append(("addc", "r2", "k", "r2", "x", "k"))
    ins.append(("addc", "r3", "k", "r3", 0, "k"))
    return ins


def modsub_program():
    """r = a - b mod p: d = a - b (borrow k); r = d - (c & -k) mod 2^128 (= d + p - 2^128).
    10 VALU."""
    ins = [("sub_co", "r0", "k", "a0", "b0")]
    for i in range(1, 4):
        ins.append(("subb", f"r{i}", "k", f"a{i}", f"b{i}", "k"))
    ins.append(("subb", "m", "k", 0, 0, "k"))  # m = -borrow
    ins.append(("and", "x", 27, "m"))
    ins.append(("sub_co", "r0", "k", "r0", "m"))
    ins.append(("subb", "r1", "k", "r1", "m", "k"))
    ins.append(("subb", "r2", "k", "r2", "x", "k"))
    ins.append(("subb", "r3", "k", "r3", 0, "k"))
    return ins


def run_addsub(kind, a, b):
    st = {}
    for i in range(4):
        st[f"a{i}"], st[f"b{i}"] = (a >> (32 * i)) & M32, (b >> (32 * i)) & M32
    simulate(modadd_program() if kind == "A" else modsub_program(), st)
    return sum(st[f"r{i}"] << (32 * i) for i in range(4))


def check_addsub(trials=20000):
    rng = random.Random(11)
    edge = [0, 1, 2, P - 1, P - 2, P // 2, P // 2 + 1, (1 << 128) - 28 * (1 << 64), 1 << 127,
            28 * (1 << 64) - 1, 28 * (1 << 64)]
    pick = lambda t, k: rng.choice(edge) if t % k == 0 else rng.randrange(P)
    for t in range(trials):
        a, b = pick(t, 3), pick(t, 2)
        assert run_addsub("A", a, b) == (a + b) % P, (a, b)
        assert run_addsub("S", a, b) == (a - b) % P, (a, b)
    for a in edge:
        for b in edge:
            assert run_addsub("A", a, b) == (a + b) % P and run_addsub("S", a, b) == (a - b) % P
    return trials


def gen_addsub(name, spec, volatile=True):
    """spec: a string of "A" (r = a + b) / "S" (r = a - b) operations, one stream each, issued
    round-robin in one asm statement.  Signature: (a, b, r) per operation.  volatile=False leaves
    the compiler free to schedule / drop the statement like any pure expression."""
    ops = [(q, kind, f"{q}") for q, kind in enumerate(spec)]
    out = []
    w = out.append
    params = []
    for q, kind, tag in ops:
        params += [f"const F128& a{tag}", f"const F128& b{tag}", f"F128& r{tag}"]
    w(f"DEVI void {name}(" + ", ".join(params) + ") {")
    ops_e, cons, idx = [], [], {}

    def opnd(key, con, expr):
        idx[key] = len(ops_e)
        ops_e.append(expr)
        cons.append(con)

    for q, kind, tag in ops:
        w(f"  uint32_t x{tag}, m{tag}" + (f", q{tag};" if kind == "A" else ";"))
        w(f"  uint64_t k{tag}" + (f", kk{tag};" if kind == "A" else ";"))
    for q, kind, tag in ops:
        for i in range(4):
            opnd(f"r{i}_{tag}", '"=&v"', f"r{tag}.w[{i}]")
        opnd(f"x_{tag}", '"=&v"', f"x{tag}")
        opnd(f"m_{tag}", '"=&v"', f"m{tag}")
        if kind == "A":
            opnd(f"q_{tag}", '"=&v"', f"q{tag}")
            opnd(f"k2_{tag}", '"=&s"', f"kk{tag}")
        opnd(f"k_{tag}", '"=&s"', f"k{tag}")
    nout = len(ops_e)
    for q, kind, tag in ops:
        for i in range(4):
            opnd(f"a{i}_{tag}", '"v"', f"a{tag}.w[{i}]")
            opnd(f"b{i}_{tag}", '"v"', f"b{tag}.w[{i}]")

    def ref(x, tag):
        return str(x) if isinstance(x, int) else f"%{idx[f'{x}_{tag}']}"

    progs = [[(ins, tag) for ins in (modadd_program() if kind == "A" else modsub_program())]
             for (q, kind, tag) in ops]
    sched = list_schedule(progs)
    rng = random.Random(len(spec))
    for t in range(200):
        init, exp = {}, {}
        for q, kind, tag in ops:
            a, b = rng.randrange(P), rng.randrange(P)
            if t % 7 == 0:
                a, b = P - 1, P - 1 - (t % 3)
            for i in range(4):
                init[(tag, f"a{i}")], init[(tag, f"b{i}")] = (a >> 32 * i) & M32, (b >> 32 * i) & M32
                exp[(tag, f"r{i}")] = (((a + b) if kind == "A" else (a - b)) % P >> 32 * i) & M32
        check_schedule(sched, init, exp)
    mn = {"add_co": "v_add_co_u32_e64", "addc": "v_addc_co_u32_e64", "sub_co": "v_sub_co_u32_e64",
          "subb": "v_subb_co_u32_e64"}
    lines = []
    for ins, tag in sched:
        op = ins[0]
        if op == "nop":
            lines.append(f"s_nop {ins[1]}")
        elif op in mn:
            lines.append(f"{mn[op]} " + ", ".join(ref(x, tag) for x in ins[1:]))
        elif op == "vsub":
            lines.append(f"v_sub_u32_e64 {ref(ins[1], tag)}, {ref(ins[2], tag)}, {ref(ins[3], tag)}")
        elif op == "and":
            lines.append(f"v_and_b32_e64 {ref(ins[1], tag)}, {ref(ins[2], tag)}, {ref(ins[3], tag)}")
        else:
            raise ValueError(op)
    w("  asm volatile(" if volatile else "  asm(")
    for l in lines:
        w(f'      "{l}\\n\\t"')
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[:nout], ops_e[:nout])))
    w("      : " + ", ".join(f"{c}({e})" for c, e in zip(cons[nout:], ops_e[nout:])) + ");")
    w("}")
    w("")
    nops = sum(int(l.split()[1]) + 1 for l in lines if l.startswith("s_nop"))
    return "\n".join(out), nops


# one iteration of the Sum FLP query's additions (prio3_kernels.h sum_query_pair)
ADDSUB = {
    "modaddsub_AASS": "AASS",    # F_i, F_j, r^2 - beta^2, t - alpha^i
    "modaddsub_ASAA": "ASAA",    # F_i + F_j, F_i - F_j, X + x, Horner + c_(i+1)
    "modaddsub_A": "A",
}


FUNCTIONS = {
    # one iteration of the Sum FLP query (prio3_kernels.h sum_query_pair), two calls:
    #   the Horner step (four products, one reduction) + the paired numerator + the gadget-output
    #   denominator,
    "mont_q1_fma1_mul1": ["Q", "F", "M"],
    #   then the gadget-output fraction's numerator + the wire fraction (numerator, denominator)
    "mont_fma2_mul1": ["F", "F", "M"],
    # k_flp_weights: the forward pass (prefix product + r^j), the backward pass (L_k, the inverse
    # and weight chains, q <- q / r^c and the previous entry's MM), Horner in t^3
    "mont_mul2": ["M", "M"],
    "mont_mul5": ["M", "M", "M", "M", "M"],
}


def generate(trials=20000, log=print):
    """Simulate every program, then return {path: text} of the two generated headers (every
    generated function is also list-scheduled, re-simulated and hazard-checked on the way)."""
    n = check(trials)
    log(f"simulated {n} single + {n} fused products: ok "
        f"(single {len(product(False))} + {len(reduce_program(False))}, "
        f"fused {len(product(True))} + {len(reduce_program(True))} instructions)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    path = os.path.join(root, "janus_amd", "csrc", "mont_fma.h")
    parts = ["// GENERATED by tools/gen_mont_fma.py -- edit the generator, not this file.",
             "// Field128 Montgomery products r = a b 2^-128 and fused sums r = (a b + c d [+ e f + i j])",
             "// 2^-128",
             "// (mod p, inputs < p, outputs canonical), several independent operations issued as",
             "// interleaved streams; s_nop only where the interleave leaves a carry hazard.",
             "#pragma once", '#include "field.h"', ""]
    for name, spec in FUNCTIONS.items():
        code, nops = gen_function(name, spec)
        parts.append(f"// streams: {spec}; {nops} s_nop")
        parts.append(code)
        log(f"{name}: {spec}, {nops} s_nop")
    n = check_addsub(trials)
    log(f"simulated {n} modular additions + subtractions: ok "
        f"({len(modadd_program())} / {len(modsub_program())} instructions)")
    parts.append("// modular additions (A) / subtractions (S), one stream each")
    for name, spec in ADDSUB.items():
        code, nops = gen_addsub(name, spec)
        parts.append(f"// streams: {spec}; {nops} s_nop")
        parts.append(code)
        log(f"{name}: {spec}, {nops} s_nop")
    out[path] = "\n".join(parts)
    # Field128Ops::add / sub (field.h): one operation, s_nop where its own chain needs them
    path = os.path.join(root, "janus_amd", "csrc", "modadd.h")
    parts = ["// GENERATED by tools/gen_mont_fma.py -- edit the generator, not this file.",
             "// Field128 r = a + b / a - b mod p and r = a b 2^-128 mod p (inputs < p, outputs canonical) as",
             "// 32-bit carry chains; included by field.h for Field128Ops::add / sub / mul.",
             "#pragma once", ""]
    for name, spec in {"f128_add_chain": "A", "f128_sub_chain": "S"}.items():
        code, nops = gen_addsub(name, spec, volatile=False)
        parts.append(f"// {nops} s_nop")
        parts.append(code)
        log(f"{name}: {spec}, {nops} s_nop")
    # Field128Ops::mul: one Montgomery product
    code, nops = gen_function("f128_mont_mul1", ["M"], volatile=False)
    parts.append(f"// one Montgomery product; {nops} s_nop")
    parts.append(code)
    log(f"f128_mont_mul1: {nops} s_nop")
    out[path] = "\n".join(parts)
    return out


if __name__ == "__main__":
    for path, text in generate().items():
        open(path, "w").write(text)
        print("wrote", path)
