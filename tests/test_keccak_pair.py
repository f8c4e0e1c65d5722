"""The lane-pair Keccak of the config E chains (janus_amd/csrc/keccak_pair.h, kp_bits.h) on the CPU:
  * the bit-interleaving helpers (even / odd bit halves, the delta-swap zip / unzip), built from
    the same header with g++, against a bit-by-bit restatement;
  * the pair round's decomposition -- each lane rotates its own half by k + p for an odd rotation
    2k + 1 and the pair swaps, by k for an even one 2k; iota XORs the round constant's halves --
    as a Python model, against the oracle's Keccak-p (oracle/prio3.py keccak_p) for SHAKE128's 24
    rounds and TurboSHAKE128's 12.
The GPU kernels themselves are pinned by the FixedPoint transcripts (tests/test_gpu_parity.py)."""
import os
import random
import subprocess

import pytest

from oracle import prio3 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M32 = 0xFFFFFFFF


def half(w, p):
    return sum(((w >> (2 * j + p)) & 1) << j for j in range(32))


def spread(h, p):
    return sum(((h >> j) & 1) << (2 * j + p) for j in range(32))


@pytest.fixture(scope="module")
def kp_bin(tmp_path_factory):
    out = tmp_path_factory.mktemp("kp") / "kp_bits_host"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-o", str(out),
                    os.path.join(ROOT, "tests", "native", "kp_bits_host.cpp")], check=True)
    return str(out)


def test_zip_unzip_match_bitwise(kp_bin):
    rng = random.Random(2)
    ws = [0, (1 << 64) - 1, 0x5555555555555555, 0xAAAAAAAAAAAAAAAA, 0x0123456789ABCDEF]
    ws += [1 << i for i in range(64)] + [rng.getrandbits(64) for _ in range(3000)]
    out = subprocess.run([kp_bin], input="".join(f"{w:x}\n" for w in ws).encode(),
                         capture_output=True, check=True).stdout.decode().split("\n")
    for w, line in zip(ws, out):
        e, o, h0, h1, z, sp = (int(t, 16) for t in line.split())
        assert e == h0 == half(w, 0) and o == h1 == half(w, 1), hex(w)
        assert z == sp == w, hex(w)


def _rotl32(x, n):
    n %= 32
    return ((x << n) | (x >> (32 - n))) & M32 if n else x


def pair_round(E, Od, rnd):
    """One round on the two halves, written the way keccak_pair.h's lanes compute it."""
    def rotl(e, o, n):  # lane p rotates its own half by k + p (odd n) or n / 2, then the swap
        if n % 2 == 0:
            return _rotl32(e, n // 2), _rotl32(o, n // 2)
        k = (n - 1) // 2
        re, ro = _rotl32(e, k), _rotl32(o, k + 1)  # own word by k + p
        return ro, re                              # DPP swap with the partner lane
    ce = [E[x] ^ E[x + 5] ^ E[x + 10] ^ E[x + 15] ^ E[x + 20] for x in range(5)]
    co = [Od[x] ^ Od[x + 5] ^ Od[x + 10] ^ Od[x + 15] ^ Od[x + 20] for x in range(5)]
    r1 = [rotl(ce[x], co[x], 1) for x in range(5)]
    be, bo = [0] * 25, [0] * 25
    rho = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61,
           56, 14]
    for i in range(25):
        x, y = i % 5, i // 5
        ve = E[i] ^ ce[(x + 4) % 5] ^ r1[(x + 1) % 5][0]
        vo = Od[i] ^ co[(x + 4) % 5] ^ r1[(x + 1) % 5][1]
        dst = y + 5 * ((2 * x + 3 * y) % 5)
        be[dst], bo[dst] = rotl(ve, vo, rho[i])
    for i in range(25):
        x, y = i % 5, i // 5
        a1, a2 = (x + 1) % 5 + 5 * y, (x + 2) % 5 + 5 * y
        E[i] = be[i] ^ (~be[a1] & be[a2] & M32)
        Od[i] = bo[i] ^ (~bo[a1] & bo[a2] & M32)
    E[0] ^= half(O._RC[rnd], 0)
    Od[0] ^= half(O._RC[rnd], 1)


@pytest.mark.parametrize("nr", [24, 12])
def test_pair_permutation_matches_oracle(nr):
    rng = random.Random(nr)
    for _ in range(20):
        a = [rng.getrandbits(64) for _ in range(25)]
        E, Od = [half(w, 0) for w in a], [half(w, 1) for w in a]
        for rnd in range(24 - nr, 24):
            pair_round(E, Od, rnd)
        assert [spread(e, 0) | spread(o, 1) for e, o in zip(E, Od)] == O.keccak_p(a, nr)
