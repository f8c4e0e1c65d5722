"""CPU model of k_flp_wires_mfma's arithmetic (janus_amd/csrc/wires_mfma.h), checked against the
plain field computation it replaces: REDC(sum_k w_k x_k) = sum_k w_k x_k 2^-128 mod p.

Mirrors the kernel step by step -- signed byte digits of the weights (w + 0x80..80, bytes ^ 0x80,
the carry out as digit 16), offset-binary share bytes (x_a ^ 0x80), the 32 x 16 Toeplitz A
operand, int32 limb accumulators (bound-checked), the two lane halves' word assembly, the
0x80..80 * (sum w mod p + calls p) correction and one REDC -- on random and extreme values."""
import random

import numpy as np
import pytest

P = 2**128 - 28 * 2**64 + 1
R_INV = pow(2**128, -1, P)
K128 = int.from_bytes(b"\x80" * 16, "little")


def weight_digits(w):
    y = w + K128
    d = [((y >> (8 * b)) & 0xFF) ^ 0x80 for b in range(16)]
    d = [i8(v) for v in d]  # as the MFMA reads the byte (signed i8)
    d.append(y >> 128)  # carry out: 0 or 1
    assert sum(v << (8 * b) for b, v in enumerate(d)) == w
    return d


def i8(v):
    return v - 256 if v >= 128 else v


def share_bytes(x):
    out = [i8(((x >> (8 * a)) & 0xFF) ^ 0x80) for a in range(16)]  # the MFMA's reading of x_a ^ 0x80
    assert out == [((x >> (8 * a)) & 0xFF) - 128 for a in range(16)]
    return out


def mfma_wire(ws, xs):
    """sum_k w_k x_k 2^-128 mod p the way the kernel computes it (one column, one wire)."""
    calls = len(ws)
    acc = np.zeros(32, dtype=np.int64)
    for k in range(calls):
        d = weight_digits(ws[k])
        # A[s][a] = d_(s - a) (zero outside 0..16), B[a] = x'_a: one MFMA K-slice
        A = np.array([[d[s - a] if 0 <= s - a <= 16 else 0 for a in range(16)] for s in range(32)],
                     dtype=np.int64)
        acc += A @ np.array(share_bytes(xs[k]), dtype=np.int64)
        assert np.abs(acc).max() < 2**31  # int32 accumulators never overflow
    # lane half h holds rows 8g + 4h + i: word 2g + h = sum_i acc[row] << 8i
    words = [sum(int(acc[8 * g + 4 * h + i]) << (8 * i) for i in range(4)) for g in range(4)
             for h in range(2)]  # index 2g + h
    V = sum(v << (32 * w) for w, v in enumerate(words))
    assert V == sum(w * (x - K128) for w, x in zip(ws, xs))
    wsum_mod = sum(ws) % P  # what k_flp_weights stores (SMM / SLM)
    S = V + K128 * (wsum_mod + calls * P)
    assert 0 <= S < 2**288  # the Wide accumulator's range
    assert S % P == sum(w * x for w, x in zip(ws, xs)) % P
    return S * R_INV % P


def _cases():
    rng = random.Random(7)
    extremes = [0, 1, P - 1, P - 2, 2**127, 2**128 - 29 * 2**64, K128, K128 - 1]
    out = []
    for calls in (1, 2, 7, 90, 300):
        ws = [rng.choice(extremes) if rng.random() < 0.3 else rng.randrange(P) for _ in range(calls)]
        xs = [rng.choice(extremes) if rng.random() < 0.3 else rng.randrange(P) for _ in range(calls)]
        out.append((ws, xs))
    out.append(([P - 1] * 300, [P - 1] * 300))  # every product at its maximum
    out.append(([0] * 16, [P - 1] * 16))
    out.append(([P - 1] * 16, [0] * 16))
    return out


@pytest.mark.parametrize("ws,xs", _cases())
def test_mfma_wire_arithmetic_is_exact(ws, xs):
    want = sum(w * x for w, x in zip(ws, xs)) * R_INV % P
    assert mfma_wire(ws, xs) == want


def test_accumulator_bound_at_the_call_limit():
    """|acc| <= calls * 16 * 2^14: the kernel's limit of 8,000 calls keeps it below 2^31."""
    assert 8000 * 16 * 2**14 < 2**31
    assert 8192 * 16 * 2**14 == 2**31
