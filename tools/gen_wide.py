"""Regenerates the inline-asm product schedule in janus_amd/csrc/wide.h (see that file).
The 16 (i, j) limb products go column-major; product k's carry lands in SGPR pair k % 3 and is
consumed (v_addc into hi[col]) two mads later, so every carry read is >= 3 issue slots after its
write (gfx950's two wait states between a VALU carry write and a VALU carry read) with no s_nop.
Operands: %0..%6 lo, %7..%13 hi, %14..%16 carries, %17..%20 a, %21..%24 x.

  python3 tools/gen_wide.py          # prints the asm lines (paste into wide.h)
"""
prods = [(0,0),(0,1),(1,0),(0,2),(1,1),(2,0),(0,3),(1,2),(2,1),(3,0),(1,3),(2,2),(3,1),(2,3),(3,2),(3,3)]
NC = 7
NCARRY = 3
A0, X0 = 2 * NC + NCARRY, 2 * NC + NCARRY + 4


def schedule():
    """(kind, k) in issue order: mads lead their carry reads by two products."""
    out, pending = [], []
    for k in range(len(prods)):
        out.append(("mad", k))
        pending.append(k)
        if len(pending) == 3:
            out.append(("addc", pending.pop(0)))
    out += [("addc", k) for k in pending]
    return out


def check(sched):
    """every addc reads a carry written >= 3 slots earlier and not overwritten since"""
    slot, wrote = {}, {}
    for t, (kind, k) in enumerate(sched):
        creg = k % NCARRY
        if kind == "mad":
            wrote[creg] = (k, t)
        else:
            wk, wt = wrote[creg]
            assert wk == k and t - wt >= 3, (k, t, wt)


if __name__ == "__main__":
    sched = schedule()
    check(sched)
    for kind, k in sched:
        i, j = prods[k]
        c, creg = i + j, 2 * NC + (k % NCARRY)
        if kind == "mad":
            print(f'      "v_mad_u64_u32 %{c}, %{creg}, %{A0 + i}, %{X0 + j}, %{c}\\n\\t"   // ({i},{j}) col {c}')
        else:
            print(f'      "v_addc_co_u32_e64 %{NC + c}, %{creg}, 0, %{NC + c}, %{creg}\\n\\t"')
