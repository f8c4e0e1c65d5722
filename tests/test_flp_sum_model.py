"""The algebra behind k_flp_query_lane's fused Sum path (prio3_kernels.h sum_query_half): the
gadget-output sum as two parity-split fractions sum F_i/(y_i - 1) plus plain sums of F, the wire
as t sum x_k/(t - alpha^k) - sum x_k, p(t) folded mod x^m - 1 -- restated in plain modular
arithmetic and checked against the oracle's direct flp_query (oracle/prio3.py, prio's Type::query
for Prio3Sum) on random measurement / proof shares and randomness.  CPU only."""
import random

import pytest

from oracle import prio3 as O

P = O.Field128.MODULUS


def sum_query_half_model(bits, meas, proof, t, r):
    calls = bits
    m = 1
    while m < calls + 1:
        m <<= 1
    assert 2 * calls == m
    gp_len = 2 * (m - 1) + 1
    alpha = pow(7, (P - 1) // m, P)
    s0, gp = proof[0], proof[1:]
    tmm, rc = pow(t, m, P), pow(r, calls, P)
    pt, N, D, S, Nw, Dw, X = 0, [0, 0], [1, 1], [0, 0], 0, 1, 0
    for i in range(m - 1, -1, -1):
        ci, ch = gp[i], (gp[i + m] if i + m < gp_len else 0)
        f = (ci + ch) % P
        e = (r * pow(alpha, i, P) - 1) % P
        par = i & 1
        S[par] = (S[par] + f) % P
        if i <= calls:
            x = meas[i - 1] if i else s0
            X = (X + x) % P
            d = (t - pow(alpha, i, P)) % P
            Nw, Dw = (Nw * d + x * Dw) % P, Dw * d % P
        pt = (t * pt + tmm * ch + ci) % P
        N[par], D[par] = (N[par] * e + f * D[par]) % P, D[par] * e % P
    inv = pow(Dw * D[0] * D[1] % P, P - 2, P)
    qw, q0, q1 = Nw * inv * D[0] * D[1] % P, N[0] * inv * Dw * D[1] % P, N[1] * inv * Dw * D[0] % P
    w0 = (tmm - 1) * pow(m, P - 2, P) * (t * qw - X) % P
    v = ((rc - 1) * (S[0] + q0) + (-rc - 1) * (S[1] + q1)) % P
    return [v, w0, pt]


@pytest.mark.parametrize("bits", [1, 2, 8, 32, 64])
def test_fused_sum_query_algebra_matches_flp_query(bits):
    rng = random.Random(bits)
    typ = O.Sum(bits)
    m = 1
    while m < bits + 1:
        m <<= 1
    for _ in range(4):
        meas = [rng.randrange(P) for _ in range(bits)]
        proof = [rng.randrange(P) for _ in range(1 + 2 * (m - 1) + 1)]
        t, r = rng.randrange(P), rng.randrange(P)
        assert sum_query_half_model(bits, meas, proof, t, r) == \
            O.flp_query(typ, meas, proof, [t], [r], 2)[:3]
