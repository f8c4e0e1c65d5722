#!/usr/bin/env python3
"""Generate keccak_asm.h (default build/keccak_asm.h, or --out PATH; an A/B study, not product code): Keccak-f[1600] rounds as inline gfx950 assembly with a
VGPR-bank-aware register assignment.

Why: a VALU instruction whose source operands sit in the same VGPR bank (register index mod 4)
issues at about 60 % of the rate of a conflict-free one once two or more waves share a SIMD
(tools/mb_bank.hip: v_bitop3_b32 2.8 vs 4.4-4.5 cycles per wave-instruction at 4 waves/SIMD; no
difference for a lone wave, and none for the half-rate v_alignbit_b32).  hipcc's allocation of
keccak.h's C++ rounds leaves ~1,900 of a permutation's 2,880 v_bitop3 with a bank conflict.  Here
the state lives in fixed registers whose banks, and those of the theta / rho temporaries, come
from a small search that leaves 10 conflicting v_bitop3 per half and round (the chi rows: three
cyclically adjacent lanes out of five cannot all take distinct banks among four).

Round structure (per 32-bit half; the same as keccak.h's keccak_round32, 180 VALU per round):
  theta  C[x] = A[x] ^ A[x+5] ^ A[x+10] ^ A[x+15] ^ A[x+20]      (2 v_bitop3)
         R[x] = rotl64(C[x], 1)                                  (2 v_alignbit per x, both halves)
         A[i] ^= C[x-1] ^ R[x+1]                                 (1 v_bitop3, in place)
  rho/pi B[pi(i)] = rotl64(A[i], r_i)   (2 v_alignbit; B[0] = A[0] stays in A[0]'s register;
         the B registers reuse C / R's once theta is done)
  chi    A[x+5y] = B[x] ^ (~B[x+1] & B[x+2])                     (1 v_bitop3 0xd2)
  iota   A[0] ^= RC                                              (v_xor_b32 with a literal)

Run: python3 tools/gen_keccak_asm.py  (deterministic).  `--selftest` interprets the generated
instructions on 32-bit integers against a plain Keccak-f[1600] (tests/test_keccak_asm.py); built
with -DP3G_KECCAK_ASM=1 the engine passed all 237 GPU tests.

Measured (profiles/r05/kasm/): no gain -- SumVec k_jr 72.4-72.8 vs 71.4-71.8 ms/step, k_expand
38.9 vs 38.5, i.e. in the sponge kernels (a third of whose VALU work is the half-rate
v_alignbit_b32) the bank conflicts of hipcc's allocation are hidden, and the copies into the fixed
registers cost a little.  The engine keeps keccak.h's C++ rounds (P3G_KECCAK_ASM=0).
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "keccak_asm.h")
if "--out" in sys.argv:
    OUT = sys.argv[sys.argv.index("--out") + 1]

RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808a, 0x8000000080008000,
      0x000000000000808b, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
      0x000000000000008a, 0x0000000000000088, 0x0000000080008009, 0x000000008000000a,
      0x000000008000808b, 0x800000000000008b, 0x8000000000008089, 0x8000000000008003,
      0x8000000000008002, 0x8000000000000080, 0x000000000000800a, 0x800000008000000a,
      0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
# rho offsets r[x + 5y] and pi: lane (x, y) -> (y, 2x + 3y)
ROT = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]


def pi(i):
    x, y = i % 5, i // 5
    return y + 5 * ((2 * x + 3 * y) % 5)


def cost(a, c, r, b):
    """Bank conflicts (operands sharing a bank) of one half-round's v_bitop3 instructions."""
    B = [a[0]] + b  # b[j - 1] = bank of B[j], j >= 1

    def t(*xs):
        return len(xs) - len(set(xs))

    tot = 0
    for x in range(5):
        tot += t(a[x], a[x + 5], a[x + 10])
        tot += t(c[x], a[x + 15], a[x + 20])
    for i in range(25):
        x = i % 5
        tot += t(a[i], c[(x + 4) % 5], r[(x + 1) % 5])
    for y in range(5):
        for x in range(5):
            tot += t(B[x + 5 * y], B[(x + 1) % 5 + 5 * y], B[(x + 2) % 5 + 5 * y])
    return tot


def usage(a, c, r, b):
    """Registers per bank of one half: A, plus a pool that holds C / R, then B (shared per bank)."""
    u = []
    for k in range(4):
        ncr = sum(1 for x in c + r if x == k)
        nb = sum(1 for x in b if x == k)
        u.append(sum(1 for x in a if x == k) + max(ncr, nb))
    return u


def objective(v):
    # conflicts first; then the most-used bank (the register block is 4 x that, per half)
    return 100 * cost(*v) + max(usage(*v))


def search(seed=1, restarts=24, iters=20000):
    rng = random.Random(seed)
    best = None
    for _ in range(restarts):
        v = [[rng.randrange(4) for _ in range(n)] for n in (25, 5, 5, 24)]
        cur = objective(v)
        temp = 2.0
        for _ in range(iters):
            w = rng.randrange(4)
            k = rng.randrange(len(v[w]))
            old = v[w][k]
            v[w][k] = rng.randrange(4)
            nc = objective(v)
            if nc <= cur or rng.random() < 2.718281828 ** (-(nc - cur) / temp):
                cur = nc
            else:
                v[w][k] = old
            temp *= 0.9997
        if best is None or cur < best[0]:
            best = (cur, [list(x) for x in v])
    return cost(*best[1]), best[1]


ROLL_U = 2  # rounds per body of the rolled loop


def allocate(banks_a, banks_c, banks_r, banks_b, base):
    """Physical registers for one half: A[25], then a pool T holding C[5], R[5] during theta and
    B[1..24] afterwards (a B value may take a dead C / R register of its bank)."""
    nxt = {k: None for k in range(4)}
    used = []

    def fresh(bank):
        # next free register index >= base with index % 4 == bank
        v = nxt[bank]
        if v is None:
            v = base + ((bank - base) % 4)
        while v in used:
            v += 4
        used.append(v)
        nxt[bank] = v + 4
        return v

    A = [fresh(bk) for bk in banks_a]
    C = [fresh(bk) for bk in banks_c]
    R = [fresh(bk) for bk in banks_r]
    pool = {k: [reg for reg in C + R if reg % 4 == k] for k in range(4)}
    B = [None] * 25
    for j in range(1, 25):
        bk = banks_b[j - 1]
        B[j] = pool[bk].pop(0) if pool[bk] else fresh(bk)
    return A, C, R, B, used


def round_asm(R_, lo, hi, iota=True):
    """Instructions of round R_ (lo / hi: dicts of register lists A, C, R, B); iota=False leaves
    the round constant to the caller (the rolled loop xors it from SGPRs)."""
    ins = []
    v = lambda n: "v%d" % n
    # theta parities: first all 3-input halves, then the rest (the second reads the first)
    for half in (lo, hi):
        for x in range(5):
            ins.append("v_bitop3_b32 %s, %s, %s, %s bitop3:0x96" % (
                v(half["C"][x]), v(half["A"][x]), v(half["A"][x + 5]), v(half["A"][x + 10])))
    for half in (lo, hi):
        for x in range(5):
            ins.append("v_bitop3_b32 %s, %s, %s, %s bitop3:0x96" % (
                v(half["C"][x]), v(half["C"][x]), v(half["A"][x + 15]), v(half["A"][x + 20])))
    # R = rotl64(C, 1): lo' = (lo << 1) | (hi >> 31) = alignbit(lo, hi, 31)
    for x in range(5):
        ins.append("v_alignbit_b32 %s, %s, %s, 31" % (v(lo["R"][x]), v(lo["C"][x]), v(hi["C"][x])))
        ins.append("v_alignbit_b32 %s, %s, %s, 31" % (v(hi["R"][x]), v(hi["C"][x]), v(lo["C"][x])))
    # theta apply, in place
    for i in range(25):
        x = i % 5
        for half in (lo, hi):
            ins.append("v_bitop3_b32 %s, %s, %s, %s bitop3:0x96" % (
                v(half["A"][i]), v(half["A"][i]), v(half["C"][(x + 4) % 5]), v(half["R"][(x + 1) % 5])))
    # rho + pi into the B registers (C / R are dead now)
    for i in range(1, 25):
        n, j = ROT[i], pi(i)
        al, ah = v(lo["A"][i]), v(hi["A"][i])
        bl, bh = v(lo["B"][j]), v(hi["B"][j])
        if n < 32:
            s = 32 - n
            ins.append("v_alignbit_b32 %s, %s, %s, %d" % (bl, al, ah, s))
            ins.append("v_alignbit_b32 %s, %s, %s, %d" % (bh, ah, al, s))
        else:
            s = 64 - n
            ins.append("v_alignbit_b32 %s, %s, %s, %d" % (bl, ah, al, s))
            ins.append("v_alignbit_b32 %s, %s, %s, %d" % (bh, al, ah, s))
    # chi: B[0] lives in A[0]'s register, so row 0 writes A[0] last (its readers: x = 3, 4, 0)
    Bl = [lo["A"][0]] + lo["B"][1:]
    Bh = [hi["A"][0]] + hi["B"][1:]
    for y in range(5):
        order = [3, 4, 1, 2, 0] if y == 0 else [0, 1, 2, 3, 4]
        for x in order:
            for half, Bx in ((lo, Bl), (hi, Bh)):
                ins.append("v_bitop3_b32 %s, %s, %s, %s bitop3:0xd2" % (
                    v(half["A"][x + 5 * y]), v(Bx[x + 5 * y]), v(Bx[(x + 1) % 5 + 5 * y]),
                    v(Bx[(x + 2) % 5 + 5 * y])))
    rc = RC[R_]
    if not iota:
        return ins
    if rc & 0xFFFFFFFF:
        ins.append("v_xor_b32 %s, 0x%x, %s" % (v(lo["A"][0]), rc & 0xFFFFFFFF, v(lo["A"][0])))
    if rc >> 32:
        ins.append("v_xor_b32 %s, 0x%x, %s" % (v(hi["A"][0]), rc >> 32, v(hi["A"][0])))
    return ins


def main(path=None):
    path = path or OUT
    best_cost, (ba, bc, br, bb) = search()
    assert best_cost <= 10, best_cost
    base = 8  # registers v8 .. : the kernel keeps v0-v7 and everything above the block
    lo_A, lo_C, lo_R, lo_B, used_lo = allocate(ba, bc, br, bb, base)
    base_hi = max(used_lo) + 1
    hi_A, hi_C, hi_R, hi_B, used_hi = allocate(ba, bc, br, bb, base_hi)
    lo = dict(A=lo_A, C=lo_C, R=lo_R, B=lo_B)
    hi = dict(A=hi_A, C=hi_C, R=hi_R, B=hi_B)
    state = set(lo_A + hi_A)
    temps = sorted((set(used_lo) | set(used_hi)) - state)
    top = max(used_lo + used_hi)
    out = []
    out.append("// Generated by tools/gen_keccak_asm.py -- do not edit.\n")
    out.append("// Keccak-f[1600] rounds as gfx950 inline assembly, VGPR-bank-aware registers\n")
    out.append("// (%d conflicting v_bitop3 per half and round; registers v%d..v%d).\n"
               % (best_cost, base, top))
    out.append("#pragma once\n#include <stdint.h>\n\n")
    out.append("#define P3G_KECCAK_ASM_CLOBBERS " + ", ".join('"v%d"' % t for t in temps) + "\n\n")
    # one asm statement per round range [R0, R1)
    for r0, r1 in ((0, 12), (12, 24)):
        out.append("__device__ __forceinline__ void keccak_asm_rounds_%d_%d(uint32_t l[25], uint32_t h[25]) {\n"
                   % (r0, r1))
        body = []
        for R_ in range(r0, r1):
            body += round_asm(R_, lo, hi)
        out.append("  asm volatile(\n")
        for k, line in enumerate(body):
            sep = "\\n\\t" if k + 1 < len(body) else ""
            out.append('      "%s%s"\n' % (line, sep))
        ops = []
        for i in range(25):
            ops.append('"+{v%d}"(l[%d])' % (lo_A[i], i))
        for i in range(25):
            ops.append('"+{v%d}"(h[%d])' % (hi_A[i], i))
        out.append("      : " + ",\n        ".join(", ".join(ops[k:k + 5]) for k in range(0, 50, 5)) + "\n")
        out.append("      :\n      : P3G_KECCAK_ASM_CLOBBERS);\n}\n\n")
    # rolled form: every round uses the same registers, so one loop body of ROLL_U rounds serves
    # all 24 (or TurboSHAKE's last 12); the round constants come from a device table by scalar
    # loads issued at the top of the body.  ~3 KB of code instead of ~35 KB unrolled.
    out.append("__device__ const uint64_t p3g_keccak_rc[24] = {\n")
    for k in range(0, 24, 4):
        out.append("    " + ", ".join("0x%016xull" % x for x in RC[k:k + 4]) + ",\n")
    out.append("};\n\n")
    U = ROLL_U
    out.append("// nr = 24 (Keccak-f) or 12 (its last 12 rounds); nr %% %d == 0\n" % U)
    out.append("__device__ __forceinline__ void keccak_asm_rolled(uint32_t l[25], uint32_t h[25], bool full) {\n")
    out.append("  const uint64_t* t = full ? p3g_keccak_rc : p3g_keccak_rc + 12;\n")
    out.append("  const uint32_t iters = (full ? 24u : 12u) / %du;\n" % U)
    body = ["s_mov_b64 s[90:91], %[t]", "s_mov_b32 s92, %[it]", "L_keccak_%=:"]
    body.append("s_load_dwordx%d s[80:%d], s[90:91], 0x0" % (2 * U, 80 + 2 * U - 1))
    for u in range(U):
        body += round_asm(0, lo, hi, iota=False)
        if u == 0:
            body.append("s_waitcnt lgkmcnt(0)")
        body.append("v_xor_b32 v%d, s%d, v%d" % (lo_A[0], 80 + 2 * u, lo_A[0]))
        body.append("v_xor_b32 v%d, s%d, v%d" % (hi_A[0], 81 + 2 * u, hi_A[0]))
    body += ["s_add_u32 s90, s90, %d" % (8 * U), "s_addc_u32 s91, s91, 0", "s_sub_u32 s92, s92, 1",
             "s_cmp_lg_u32 s92, 0", "s_cbranch_scc1 L_keccak_%="]
    out.append("  asm volatile(\n")
    for k, line in enumerate(body):
        sep = "\\n\\t" if k + 1 < len(body) else ""
        if line.endswith(":"):
            sep = "\\n"
        out.append('      "%s%s"\n' % (line, sep))
    out.append("      : " + ",\n        ".join(", ".join(ops[k:k + 5]) for k in range(0, 50, 5)) + "\n")
    sg = ", ".join('"s%d"' % k for k in list(range(80, 80 + 2 * U)) + [90, 91, 92])
    out.append("      : [t] \"s\"(t), [it] \"s\"(iters)\n")
    out.append("      : P3G_KECCAK_ASM_CLOBBERS, %s, \"scc\");\n}\n" % sg)
    text = "".join(out)
    if "--check" in sys.argv:
        cur = open(path).read() if os.path.exists(path) else ""
        sys.exit(0 if cur == text else 1)
    with open(path, "w") as f:
        f.write(text)
    print("wrote %s: %d instructions per 12 rounds, conflicts/half-round %d, v%d..v%d (%d temps)"
          % (path, len(body), best_cost, base, top, len(temps)))


if __name__ == "__main__" and "--selftest" not in sys.argv:
    main()


# ------------------------------------------------------------------------------------------------
# Self-check (tests/test_gen_arith.py): interpret the generated instructions on 32-bit registers and
# compare 24 rounds with a plain Keccak-f[1600].
def keccak_f_ref(a):
    M = (1 << 64) - 1
    rot = lambda v, n: ((v << n) | (v >> (64 - n))) & M if n else v
    a = list(a)
    for R_ in range(24):
        C = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        D = [C[(x + 4) % 5] ^ rot(C[(x + 1) % 5], 1) for x in range(5)]
        a = [a[i] ^ D[i % 5] for i in range(25)]
        B = [0] * 25
        for i in range(25):
            B[pi(i)] = rot(a[i], ROT[i])
        a = [B[i] ^ ((~B[(i % 5 + 1) % 5 + 5 * (i // 5)]) & B[(i % 5 + 2) % 5 + 5 * (i // 5)]) & M
             for i in range(25)]
        a[0] ^= RC[R_]
    return a


def interpret(text, l, h):
    """Run the generated asm statements of `text` on a register file seeded from the state."""
    import re
    reg = {}
    blocks = re.findall(r"keccak_asm_rounds_(\d+)_(\d+)\(.*?asm volatile\((.*?)\s*:\s*(\"\+\{.*?)\s*:\s*\n", text,
                        re.S)
    M32 = 0xFFFFFFFF
    for r0, r1, body, ops in blocks:
        regs = [int(x) for x in re.findall(r'"\+\{v(\d+)\}"', ops)]
        for i in range(25):
            reg[regs[i]] = l[i]
            reg[regs[25 + i]] = h[i]
        for line in re.findall(r'"([^"]*)"', body):
            line = line.replace("\\n\\t", "").strip()
            if not line:
                continue
            op, rest = line.split(" ", 1)
            args = [x.strip() for x in rest.replace(" bitop3:", ", bitop3:").split(",")]
            val = lambda t: reg[int(t[1:])] if t.startswith("v") else int(t, 0)
            d = int(args[0][1:])
            if op == "v_bitop3_b32":
                a_, b_, c_ = val(args[1]), val(args[2]), val(args[3])
                lut = int(args[4].split(":")[1], 0)
                r = 0
                for bit in range(32):
                    idx = (((a_ >> bit) & 1) << 2) | (((b_ >> bit) & 1) << 1) | ((c_ >> bit) & 1)
                    r |= ((lut >> idx) & 1) << bit
                reg[d] = r
            elif op == "v_alignbit_b32":
                hi_, lo_, s = val(args[1]), val(args[2]), int(args[3])
                reg[d] = (((hi_ << 32) | lo_) >> s) & M32
            elif op == "v_xor_b32":
                reg[d] = val(args[1]) ^ val(args[2])
            else:
                raise ValueError(op)
        l = [reg[regs[i]] for i in range(25)]
        h = [reg[regs[25 + i]] for i in range(25)]
    return l, h


def interpret_rolled(text, l, h, full=True):
    """Run keccak_asm_rolled's loop body on a register file (round constants from RC)."""
    import re
    m = re.search(r"keccak_asm_rolled\(.*?asm volatile\((.*?)\s*:\s*(\"\+\{.*?)\s*:\s*\[t\]", text, re.S)
    body, ops = m.group(1), m.group(2)
    regs = [int(x) for x in re.findall(r'"\+\{v(\d+)\}"', ops)]
    reg = {}
    for i in range(25):
        reg[regs[i]] = l[i]
        reg[regs[25 + i]] = h[i]
    lines = [x.replace("\\n\\t", "").replace("\\n", "").strip() for x in re.findall(r'"([^"]*)"', body)]
    start = [k for k, x in enumerate(lines) if x.startswith("L_keccak")][0] + 1
    loop = lines[start:]
    r0 = 0 if full else 12
    M32 = 0xFFFFFFFF
    for it in range((24 - r0) // ROLL_U):
        sg = {}
        for k in range(ROLL_U):
            rc = RC[r0 + it * ROLL_U + k]
            sg[80 + 2 * k], sg[81 + 2 * k] = rc & M32, rc >> 32
        for line in loop:
            if not line.startswith("v_"):
                continue
            op, rest = line.split(" ", 1)
            args = [x.strip() for x in rest.replace(" bitop3:", ", bitop3:").split(",")]

            def val(t):
                if t.startswith("v"):
                    return reg[int(t[1:])]
                if t.startswith("s"):
                    return sg[int(t[1:])]
                return int(t, 0)
            d = int(args[0][1:])
            if op == "v_bitop3_b32":
                a_, b_, c_ = val(args[1]), val(args[2]), val(args[3])
                lut = int(args[4].split(":")[1], 0)
                r = 0
                for bit in range(32):
                    idx = (((a_ >> bit) & 1) << 2) | (((b_ >> bit) & 1) << 1) | ((c_ >> bit) & 1)
                    r |= ((lut >> idx) & 1) << bit
                reg[d] = r
            elif op == "v_alignbit_b32":
                hi_, lo_, s = val(args[1]), val(args[2]), int(args[3])
                reg[d] = (((hi_ << 32) | lo_) >> s) & M32
            elif op == "v_xor_b32":
                reg[d] = val(args[1]) ^ val(args[2])
            else:
                raise ValueError(op)
    return [reg[regs[i]] for i in range(25)], [reg[regs[25 + i]] for i in range(25)]


def selftest_rolled(path=OUT, seed=7):
    rng = random.Random(seed)
    a = [rng.getrandbits(64) for _ in range(25)]
    l, h = [x & 0xFFFFFFFF for x in a], [x >> 32 for x in a]
    l, h = interpret_rolled(open(path).read(), l, h)
    got = [(hh << 32) | ll for ll, hh in zip(l, h)]
    return got == keccak_f_ref(a)


def selftest(path=OUT, seed=7):
    rng = random.Random(seed)
    a = [rng.getrandbits(64) for _ in range(25)]
    l, h = [x & 0xFFFFFFFF for x in a], [x >> 32 for x in a]
    l, h = interpret(open(path).read(), l, h)
    got = [(hh << 32) | ll for ll, hh in zip(l, h)]
    return got == keccak_f_ref(a)


if __name__ == "__main__" and "--selftest" in sys.argv:
    ok = selftest() and selftest_rolled()
    print("selftest", "ok" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)
