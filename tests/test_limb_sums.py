"""k_flp_wires_cols' Histogram sum (prio3_kernels.h f128_reduce_limb_sums): the lane's elements
summed as four 64-bit sums of their 32-bit limbs, reduced once.  The same steps in Python integers
against the plain modular sum, on random, boundary (p - 1, 0) and worst-case-count inputs.  CPU
only."""
import random

P = (1 << 128) - 28 * (1 << 64) + 1
CC = (1 << 128) - P
M64 = (1 << 64) - 1
M128 = (1 << 128) - 1


def reduce_limb_sums(xs):
    """mirror of f128_reduce_limb_sums (u128 arithmetic wraps mod 2^128)"""
    acc = xs[0] + (xs[1] << 32)
    c64, w0 = acc >> 64, acc & M64
    hi = c64 + xs[2] + (xs[3] << 32)
    lo = ((hi & M64) << 64) | w0
    top = hi >> 64
    v = (lo + top * CC) & M128
    if v < lo:
        v = (v + CC) & M128
    if v >= P:
        v -= P
    return v


def limb_sums(vals):
    xs = [0, 0, 0, 0]
    for v in vals:
        for q in range(4):
            xs[q] += (v >> (32 * q)) & 0xFFFFFFFF
    return xs


def test_limb_sums_reduce_to_the_modular_sum():
    rng = random.Random(5)
    for n in (0, 1, 2, 16, 89, 1000):
        for _ in range(200):
            vals = [rng.randrange(P) for _ in range(n)]
            assert reduce_limb_sums(limb_sums(vals)) == sum(vals) % P


def test_limb_sums_extremes():
    for n in (1, 16, 4096, 1 << 16):
        for v in (P - 1, P - 2, 0, 1, 1 << 127, (1 << 128) - 28 * (1 << 64)):
            xs = [((v >> (32 * q)) & 0xFFFFFFFF) * n for q in range(4)]
            assert reduce_limb_sums(xs) == v * n % P
