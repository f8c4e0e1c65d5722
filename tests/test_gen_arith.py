"""The generated Field128 arithmetic (tools/gen_mont_fma.py -> janus_amd/csrc/mont_fma.h,
modadd.h): every program simulated against Python integers (single / fused / four-pair Montgomery
products, modular additions and subtractions, on random and edge operands), every generated
function's list schedule re-simulated and checked for gfx950's carry hazard (>= 2 wait states
between a VALU carry write and read), and the committed headers equal to what the generator emits
now.  CPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_mont_fma as G  # noqa: E402


def test_generated_headers_are_current_and_verified():
    out = G.generate(trials=1500, log=lambda *_: None)
    assert len(out) == 2
    for path, text in out.items():
        with open(path) as f:
            assert f.read() == text, f"{os.path.basename(path)} is stale: run tools/gen_mont_fma.py"


def test_four_pair_product_sum_edges():
    P, R = G.P, G.R
    rinv = pow(R, -1, P)
    for v in ([P - 1] * 8, [0] * 8, [1] * 8, [P - 1, 1] * 4, [P // 2] * 8):
        exp = sum(v[2 * k] * v[2 * k + 1] for k in range(4)) * rinv % P
        assert G.run_op(4, *v) == exp
