"""Regenerates the inline-asm product schedule in janus_amd/csrc/wide.h (see that file).
The 16 (i, j) limb products go column-major; the carry of product k lands in SGPR pair k%2 and is
consumed (v_addc into hi[col]) one instruction later, after the next product's mad."""
prods = [(0,0),(0,1),(1,0),(0,2),(1,1),(2,0),(0,3),(1,2),(2,1),(3,0),(1,3),(2,2),(3,1),(2,3),(3,2),(3,3)]
NC = 7
if __name__ == "__main__":
    pending = None
    for k, (i, j) in enumerate(prods):
        c, creg = i + j, 2 * NC + (k % 2)
        print(f'"v_mad_u64_u32 %{c}, %{creg}, %{2*NC+2+i}, %{2*NC+6+j}, %{c}\\n\\t"')
        if pending:
            print(f'"v_addc_co_u32_e64 %{NC+pending[0]}, %{pending[1]}, 0, %{NC+pending[0]}, %{pending[1]}\\n\\t"')
        pending = (c, creg)
    print('"s_nop 0\\n\\t"')
    print(f'"v_addc_co_u32_e64 %{NC+pending[0]}, %{pending[1]}, 0, %{NC+pending[0]}, %{pending[1]}\\n\\t"')
