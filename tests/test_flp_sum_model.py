"""The algebra behind k_flp_query_lane's fused Sum path (prio3_kernels.h sum_query_pair): the
gadget-output sum as r * sum_par c_par Q_par with Q_par = sum_(i = par) F_i/(r - alpha^-i), the
terms i and i + m/2 paired over r^2 - alpha^-2i; the wire as t sum x_k/(t - alpha^k) - sum x_k;
p(t) folded mod x^m - 1 and then mod x^(m/2) + 1 into m/2 Horner steps -- restated in plain modular
arithmetic and checked against the oracle's direct flp_query (oracle/prio3.py, prio's Type::query
for Prio3Sum) on random measurement / proof shares and randomness.  CPU only."""
import random

import pytest

from oracle import prio3 as O

P = O.Field128.MODULUS


def sum_query_pair_model(bits, meas, proof, t, r):
    calls = bits
    m = 1
    while m < calls + 1:
        m <<= 1
    h = m // 2
    assert calls == h and h % 2 == 0
    gp_len = 2 * (m - 1) + 1
    alpha = pow(7, (P - 1) // m, P)

    def tw(k):
        return pow(alpha, k % m, P)

    s0, gp = proof[0], proof[1:]

    def c(d):
        return gp[d] if d < gp_len else 0

    tmm, th = pow(t, m, P), pow(t, h, P)
    t3h, rc, r2 = tmm * th % P, pow(r, calls, P), r * r % P
    X = Nw = meas[calls - 1]
    Dw = (t - tw(calls)) % P
    pt, N, D = 0, [0, 0], [1, 1]
    for i in range(h - 1, -1, -1):
        par = i & 1
        x = meas[i - 1] if i else s0
        fi, fj = (c(i) + c(i + m)) % P, (c(i + h) + c(i + h + m)) % P
        beta = tw(m - i)
        u = (r * (fi + fj) + beta * (fi - fj)) % P
        d2 = (r2 - beta * beta) % P
        dw = (t - tw(i)) % P
        N[par], D[par] = (N[par] * d2 + u * D[par]) % P, D[par] * d2 % P
        Nw, Dw = (Nw * dw + x * Dw) % P, Dw * dw % P
        X = (X + x) % P
        pt = (t * pt + tmm * c(i + m) + th * c(i + h) + t3h * c(i + h + m) + c(i)) % P

    def inv(a):
        return pow(a, P - 2, P)

    qw, q0, q1 = Nw * inv(Dw) % P, N[0] * inv(D[0]) % P, N[1] * inv(D[1]) % P
    w0 = (tmm - 1) * inv(m) * (t * qw - X) % P
    v = r * ((rc - 1) * q0 + (-rc - 1) * q1) % P
    return [v, w0, pt]


@pytest.mark.parametrize("bits", [2, 4, 8, 32, 64])
def test_paired_sum_query_algebra_matches_flp_query(bits):
    rng = random.Random(bits)
    typ = O.Sum(bits)
    m = 1
    while m < bits + 1:
        m <<= 1
    for _ in range(4):
        meas = [rng.randrange(P) for _ in range(bits)]
        proof = [rng.randrange(P) for _ in range(1 + 2 * (m - 1) + 1)]
        t, r = rng.randrange(P), rng.randrange(P)
        assert sum_query_pair_model(bits, meas, proof, t, r) == \
            O.flp_query(typ, meas, proof, [t], [r], 2)[:3]
