"""CPU oracle: restatement of Prio3 (draft-irtf-cfrg-vdaf-07) as implemented by prio 0.15.1.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import this module, and only as the checker.  The product path
(`janus_amd/`) never imports it; it fails loudly when the HIP library is missing.

PARITY UNPINNED (Prio3 arithmetic).  The reference (`/root/reference`, Janus 0.6) only *calls*
Prio3; the arithmetic lives in the third-party crate `prio` 0.15.1 (`Cargo.toml:46`,
`Cargo.lock:2939-2963`), which is not vendored, not buildable here (no cargo/rustc/network) and has
no Python binding.  The reference's own tests compute every Prio3 expectation at run time by calling
prio (`core/src/test_util/mod.rs:87-233`), so no golden Prio3 bytes exist to pin against.  What IS
pinned:
  * the SHAKE128 sponge, against `hashlib.shake_128` (FIPS 202) and the FIPS 202 empty-input KAT;
  * the field moduli / generators / 2-adic orders (checked numerically in tests);
  * end-to-end semantics: unshard(aggregate) == plaintext sum, as the reference's integration tests
    check (`integration_tests/tests/common/mod.rs:225-398`);
  * DAP framing of ping-pong messages (`messages/src/lib.rs:4094-4280`).
Everything else follows VDAF-07 as restated in SURVEY.md Appendix A, with the prio-0.15.1 code
structure recalled per function below ("prio" = prio 0.15.1 source file, not in this container).

Call sites in the reference that this oracle stands behind:
  * helper prepare: `aggregator/src/aggregator.rs:1775-1797` (helper_initialized + evaluate)
  * leader prepare: `aggregator/src/aggregator/aggregation_job_driver.rs:362-380`, `:579-593`
  * accumulation:   `aggregator/src/aggregator/accumulator.rs:76-122`,
                    `aggregator_core/src/datastore/models.rs:962-991`
  * transcript:     `core/src/test_util/mod.rs:87-233` (run_vdaf / VdafTranscript)
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field as dc_field
from typing import List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------------------------
# Fields (prio src/field.rs, src/fp.rs; VDAF-07 §6.1.2).  Canonical integers; the encoding is the
# little-endian canonical value, so Montgomery vs canonical internal form does not matter.
# ---------------------------------------------------------------------------------------------


class Field:
    MODULUS: int
    ENCODED_SIZE: int
    GEN_ORDER_LOG: int
    GEN: int

    @classmethod
    def root(cls, log_n: int) -> int:
        """Principal 2^log_n-th root of unity: GEN^(2^(GEN_ORDER_LOG - log_n)) (prio fp.rs roots)."""
        assert 0 <= log_n <= cls.GEN_ORDER_LOG
        return pow(cls.GEN, 1 << (cls.GEN_ORDER_LOG - log_n), cls.MODULUS)

    @classmethod
    def inv(cls, x: int) -> int:
        return pow(x, cls.MODULUS - 2, cls.MODULUS)

    @classmethod
    def encode_vec(cls, v: Sequence[int]) -> bytes:
        return b"".join(int(x).to_bytes(cls.ENCODED_SIZE, "little") for x in v)

    @classmethod
    def decode_vec(cls, b: bytes) -> List[int]:
        n = cls.ENCODED_SIZE
        if len(b) % n:
            raise ValueError("bad field-vector length")
        out = []
        for i in range(0, len(b), n):
            x = int.from_bytes(b[i:i + n], "little")
            if x >= cls.MODULUS:
                raise ValueError("field element out of range")
            out.append(x)
        return out


class Field64(Field):
    MODULUS = 2**32 * 4294967295 + 1  # 2^64 - 2^32 + 1
    ENCODED_SIZE = 8
    GEN_ORDER_LOG = 32
    GEN = pow(7, (MODULUS - 1) >> 32, MODULUS)


class Field128(Field):
    MODULUS = 2**66 * 4611686018427387897 + 1  # 2^128 - 28*2^64 + 1
    ENCODED_SIZE = 16
    GEN_ORDER_LOG = 66
    GEN = pow(7, (MODULUS - 1) >> 66, MODULUS)


def next_pow2(n: int) -> int:
    return 1 << (n - 1).bit_length() if n > 1 else 1


# ---------------------------------------------------------------------------------------------
# XOF: XofShake128 (prio src/vdaf/xof.rs; VDAF-07 §6.2.1).
#   stream = SHAKE128( u8(len(dst)) || dst || seed || binder )
# ---------------------------------------------------------------------------------------------

SEED_SIZE = 16
VERSION = 7


class XofShake128:
    def __init__(self, seed: bytes, dst: bytes, binder: bytes = b""):
        assert len(seed) == SEED_SIZE and len(dst) < 256
        self.msg = bytes([len(dst)]) + dst + seed + binder

    def stream(self, n: int) -> bytes:
        return hashlib.shake_128(self.msg).digest(n)

    def next_vec(self, fld, length: int) -> List[int]:
        """prio `into_field_vec` over the XOF stream (see field_vec_from_stream)."""
        nbytes = fld.ENCODED_SIZE * length + 64
        while True:
            out = field_vec_from_stream(fld, self.stream(nbytes), length)
            if out is not None:
                return out
            nbytes *= 2


# XofTurboShake128 (draft-irtf-cfrg-vdaf-08 §6.2.1; TurboSHAKE128 = RFC 9861):
#   stream = TurboSHAKE128( u8(len(dst)) || dst || seed || binder, D = 0x01 )
# TurboSHAKE128 = the SHAKE128 sponge (rate 168) over Keccak-p[1600, 12] -- the LAST 12 rounds of
# Keccak-f -- with the domain byte D in place of SHAKE's 0x1F.  A pure-Python permutation (no
# library in this image implements TurboSHAKE); pinned in tests by (a) the 24-round form of the
# same code == hashlib.shake_128 and (b) the RFC 9861 TurboSHAKE128(M = empty, D = 0x1F) vectors.
# Janus 0.6 runs XofShake128; this mode is forward compatibility only: PARITY UNPINNED.
_RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
       0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
       0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
       0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
       0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
       0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
_ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56],
        [27, 20, 39, 8, 14]]
_M64 = (1 << 64) - 1


def _rotl(x: int, n: int) -> int:
    return ((x << n) | (x >> (64 - n))) & _M64 if n else x


def keccak_p(a: List[int], nr: int) -> List[int]:
    """Keccak-p[1600, nr] on 25 lanes (lane x + 5y): rounds 24 - nr .. 23 of Keccak-f."""
    for rnd in range(24 - nr, 24):
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rotl(c[(x + 1) % 5], 1) for x in range(5)]
        a = [a[i] ^ d[i % 5] for i in range(25)]
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = _rotl(a[x + 5 * y], _ROT[x][y])
        a = [b[i] ^ (~b[(i % 5 + 1) % 5 + 5 * (i // 5)] & b[(i % 5 + 2) % 5 + 5 * (i // 5)])
             for i in range(25)]
        a[0] ^= _RC[rnd]
    return a


def keccak_sponge(msg: bytes, pad: int, n: int, nr: int, rate: int = 168) -> bytes:
    """Sponge over Keccak-p[1600, nr]: msg || pad || 0.. || 0x80 (pad 0x1F, nr 24 = SHAKE128;
    pad D, nr 12 = TurboSHAKE128(msg, D))."""
    m = bytearray(msg) + bytes([pad])
    while len(m) % rate:
        m.append(0)
    m[-1] ^= 0x80
    a = [0] * 25
    for off in range(0, len(m), rate):
        for i in range(rate // 8):
            a[i] ^= int.from_bytes(m[off + 8 * i:off + 8 * i + 8], "little")
        a = keccak_p(a, nr)
    out = bytearray()
    while True:
        out += b"".join(a[i].to_bytes(8, "little") for i in range(rate // 8))
        if len(out) >= n:
            return bytes(out[:n])
        a = keccak_p(a, nr)


def turboshake128(msg: bytes, d: int, n: int) -> bytes:
    return keccak_sponge(msg, d, n, 12)


class XofTurboShake128(XofShake128):
    """draft-irtf-cfrg-vdaf-08 XofTurboShake128: TurboSHAKE128(u8(len(dst)) || dst || seed ||
    binder, D = 1).  Same message and next_vec as XofShake128."""
    DOMAIN = 0x01

    def stream(self, n: int) -> bytes:
        return turboshake128(self.msg, self.DOMAIN, n)


def field_vec_from_stream(fld, buf: bytes, length: int) -> Optional[List[int]]:
    """prio 0.15.1 `into_field_vec` (src/field.rs, via XofShake128::next_vec): read
    ENCODED_SIZE-byte LE chunks of the stream in order and keep those < p (rejection sampling; the
    mask is all-ones for Field64/Field128, so masking is a no-op).  None if `buf` runs out first."""
    es = fld.ENCODED_SIZE
    out, off = [], 0
    while len(out) < length and off + es <= len(buf):
        x = int.from_bytes(buf[off:off + es], "little")
        off += es
        if x < fld.MODULUS:
            out.append(x)
    return out if len(out) == length else None


def derive_seed(seed: bytes, dst: bytes, binder: bytes, xof=None) -> bytes:
    return (xof or XofShake128)(seed, dst, binder).stream(SEED_SIZE)


# Usage constants (prio src/vdaf/prio3.rs; VDAF-07 §7.2)
DST_MEASUREMENT_SHARE = 1
DST_PROOF_SHARE = 2
DST_JOINT_RANDOMNESS = 3
DST_PROVE_RANDOMNESS = 4
DST_QUERY_RANDOMNESS = 5
DST_JOINT_RAND_SEED = 6
DST_JOINT_RAND_PART = 7


def domain_separation_tag(algo_id: int, usage: int) -> bytes:
    """prio `Vdaf::domain_separation_tag`: [VERSION, class=0, algo_id u32 BE, usage u16 BE]."""
    return bytes([VERSION, 0]) + algo_id.to_bytes(4, "big") + usage.to_bytes(2, "big")


# ---------------------------------------------------------------------------------------------
# Polynomials / NTT (prio src/fft.rs, src/polynomial.rs) -- natural-order DFT over 2^k roots.
# ---------------------------------------------------------------------------------------------


def ntt(fld, coeffs: Sequence[int], n: int) -> List[int]:
    """out[i] = sum_j coeffs[j] * w^(i*j), w = fld.root(log2 n); coeffs zero-padded to n."""
    p = fld.MODULUS
    a = list(coeffs) + [0] * (n - len(coeffs))
    assert len(a) == n and n & (n - 1) == 0
    logn = n.bit_length() - 1
    # bit reversal
    j = 0
    for i in range(1, n):
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j |= bit
        if i < j:
            a[i], a[j] = a[j], a[i]
    length = 2
    while length <= n:
        w_len = fld.root(length.bit_length() - 1)
        half = length >> 1
        ws = [1] * half
        for k in range(1, half):
            ws[k] = ws[k - 1] * w_len % p
        for start in range(0, n, length):
            for k in range(half):
                u = a[start + k]
                v = a[start + k + half] * ws[k] % p
                a[start + k] = (u + v) % p
                a[start + k + half] = (u - v) % p
        length <<= 1
    del logn
    return a


def intt(fld, vals: Sequence[int], n: int) -> List[int]:
    """Interpolate: coefficients c with sum_j c_j w^(ij) = vals[i] (prio DFT + inv_finish)."""
    p = fld.MODULUS
    a = ntt(fld, vals, n)
    n_inv = fld.inv(n)
    out = [0] * n
    out[0] = a[0] * n_inv % p
    for i in range(1, n):
        out[i] = a[n - i] * n_inv % p
    return out


def poly_eval(fld, coeffs: Sequence[int], x: int) -> int:
    p = fld.MODULUS
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % p
    return acc


def poly_mul(fld, a: Sequence[int], b: Sequence[int]) -> List[int]:
    p = fld.MODULUS
    n = next_pow2(len(a) + len(b) - 1)
    fa, fb = ntt(fld, a, n), ntt(fld, b, n)
    c = intt(fld, [x * y % p for x, y in zip(fa, fb)], n)
    return c[:len(a) + len(b) - 1]


# ---------------------------------------------------------------------------------------------
# Gadgets (prio src/flp/gadgets.rs)
# ---------------------------------------------------------------------------------------------


class Mul:
    """prio `Mul`: arity 2, degree 2."""

    def __init__(self, calls: int):
        self.ARITY, self.DEGREE, self.CALLS = 2, 2, calls

    def eval(self, fld, inp):
        return inp[0] * inp[1] % fld.MODULUS

    def eval_poly(self, fld, polys):
        return poly_mul(fld, polys[0], polys[1])


class PolyEval:
    """prio `PolyEval`: arity 1, degree len(poly)-1."""

    def __init__(self, poly: Sequence[int], calls: int):
        self.poly = list(poly)
        self.ARITY, self.DEGREE, self.CALLS = 1, len(poly) - 1, calls

    def eval(self, fld, inp):
        return poly_eval(fld, [c % fld.MODULUS for c in self.poly], inp[0])

    def eval_poly(self, fld, polys):
        p = fld.MODULUS
        x = polys[0]
        out = [0]
        xp = [1]
        for c in self.poly:
            c %= p
            if c:
                term = [c * v % p for v in xp]
                out = poly_add(fld, out, term)
            xp = poly_mul(fld, xp, x)
        return out


def poly_add(fld, a, b):
    p = fld.MODULUS
    n = max(len(a), len(b))
    a = list(a) + [0] * (n - len(a))
    b = list(b) + [0] * (n - len(b))
    return [(x + y) % p for x, y in zip(a, b)]


class ParallelSumMul:
    """prio `ParallelSum<F, Mul<F>>` (and `...Multithreaded`, identical output): arity 2*chunk."""

    def __init__(self, chunk: int, calls: int):
        self.chunk = chunk
        self.ARITY, self.DEGREE, self.CALLS = 2 * chunk, 2, calls

    def eval(self, fld, inp):
        p = fld.MODULUS
        return sum(inp[2 * j] * inp[2 * j + 1] for j in range(self.chunk)) % p

    def eval_poly(self, fld, polys):
        # Evaluate every wire poly at 2m points, multiply pointwise, interpolate (NTT form).
        p = fld.MODULUS
        m = len(polys[0])
        n = next_pow2(2 * m - 1)
        acc = [0] * n
        for j in range(self.chunk):
            fa, fb = ntt(fld, polys[2 * j], n), ntt(fld, polys[2 * j + 1], n)
            for i in range(n):
                acc[i] = (acc[i] + fa[i] * fb[i]) % p
        return intt(fld, acc, n)[:2 * m - 1]


class ParallelSumPolyEval:
    """prio `ParallelSum<F, PolyEval<F>>` (and `...Multithreaded`): arity chunk, degree
    len(poly)-1; G(x_0..x_{c-1}) = sum_j poly(x_j)."""

    def __init__(self, poly: Sequence[int], chunk: int, calls: int):
        self.poly = list(poly)
        self.chunk = chunk
        self.ARITY, self.DEGREE, self.CALLS = chunk, len(poly) - 1, calls

    def eval(self, fld, inp):
        p = fld.MODULUS
        cs = [c % p for c in self.poly]
        return sum(poly_eval(fld, cs, x) for x in inp) % p

    def eval_poly(self, fld, polys):
        # Every wire poly evaluated at n >= DEGREE*(m-1)+1 points, poly applied pointwise, summed,
        # interpolated (the result is the unique polynomial of that degree).
        p = fld.MODULUS
        m = len(polys[0])
        want = self.DEGREE * (m - 1) + 1
        n = next_pow2(want)
        cs = [c % p for c in self.poly]
        acc = [0] * n
        for j in range(self.chunk):
            fv = ntt(fld, polys[j], n)
            for i in range(n):
                acc[i] = (acc[i] + poly_eval(fld, cs, fv[i])) % p
        return intt(fld, acc, n)[:want]


def optimal_chunk_length(measurement_length: int) -> int:
    """prio `optimal_chunk_length` (src/vdaf/prio3.rs): among gadget_calls = 2^k - 1 (k = 1 ..
    round(log2(len+1))), the chunk length minimising the ParallelSum(Mul) proof length
    2*chunk + 2*((1 + calls).next_power_of_two() - 1) + 1 (first minimum from the largest k)."""
    if measurement_length <= 1:
        return 1
    import math
    max_log2 = round(math.log2(measurement_length + 1))
    best = None
    for log2 in range(max_log2, 0, -1):
        calls = (1 << log2) - 1
        chunk = (measurement_length + calls - 1) // calls
        cost = 2 * chunk + 2 * (next_pow2(1 + calls) - 1) + 1
        if best is None or cost < best[0]:
            best = (cost, chunk)
    return best[1]


# ---------------------------------------------------------------------------------------------
# Validity circuits (prio src/flp/types.rs, VDAF-07 §7.4)
# ---------------------------------------------------------------------------------------------


def parallel_sum_range_checks(fld, g, calls, meas, r, chunk, num_shares):
    """prio `parallel_sum_range_checks` (0.15.1: ONE joint-rand value, r_power runs across all
    chunks; padding slots use measurement value 0, i.e. args (0, -1/num_shares))."""
    p = fld.MODULUS
    shares_inv = fld.inv(num_shares)
    out = 0
    r_power = r
    for i in range(calls):
        inputs = [0] * (2 * chunk)
        for j in range(chunk):
            idx = i * chunk + j
            if idx < len(meas):
                x = meas[idx]
                inputs[2 * j] = r_power * x % p
                inputs[2 * j + 1] = (x - shares_inv) % p
                r_power = r_power * r % p
            else:
                inputs[2 * j] = 0
                inputs[2 * j + 1] = (-shares_inv) % p
        out = (out + g(inputs)) % p
    return out


class Count:
    ID = 0x00000000
    Field = Field64

    def __init__(self):
        self.MEAS_LEN = 1
        self.OUTPUT_LEN = 1
        self.JOINT_RAND_LEN = 0
        self.QUERY_RAND_LEN = 1
        self.gadgets = [Mul(1)]
        self.PROVE_RAND_LEN = 2

    def encode(self, m: int) -> List[int]:
        assert m in (0, 1)
        return [m]

    def valid(self, g, meas, joint_rand, num_shares):
        p = self.Field.MODULUS
        return (g[0]([meas[0], meas[0]]) - meas[0]) % p

    def truncate(self, meas):
        return list(meas)

    def decode_result(self, agg):
        return agg[0]


class Sum:
    ID = 0x00000001
    Field = Field128

    def __init__(self, bits: int):
        self.bits = bits
        self.MEAS_LEN = bits
        self.OUTPUT_LEN = 1
        self.JOINT_RAND_LEN = 1
        self.QUERY_RAND_LEN = 1
        # poly_range_check(0, 2) = x*(x-1) = [0, -1, 1]
        self.gadgets = [PolyEval([0, -1, 1], bits)]
        self.PROVE_RAND_LEN = 1

    def encode(self, m: int) -> List[int]:
        assert 0 <= m < (1 << self.bits)
        return [(m >> i) & 1 for i in range(self.bits)]

    def valid(self, g, meas, joint_rand, num_shares):
        """prio `call_gadget_on_vec_entries`: sum_i r^(i+1) * g(x_i)."""
        p = self.Field.MODULUS
        r = joint_rand[0]
        rp = r
        out = 0
        for x in meas:
            out = (out + rp * g[0]([x])) % p
            rp = rp * r % p
        return out

    def truncate(self, meas):
        p = self.Field.MODULUS
        return [sum((1 << i) * x for i, x in enumerate(meas)) % p]

    def decode_result(self, agg):
        return agg[0]


class SumVec:
    ID = 0x00000002
    Field = Field128

    def __init__(self, bits: int, length: int, chunk: int):
        self.bits, self.length, self.chunk = bits, length, chunk
        self.MEAS_LEN = bits * length
        self.OUTPUT_LEN = length
        self.JOINT_RAND_LEN = 1
        self.QUERY_RAND_LEN = 1
        calls = (self.MEAS_LEN + chunk - 1) // chunk
        self.gadgets = [ParallelSumMul(chunk, calls)]
        self.PROVE_RAND_LEN = 2 * chunk

    def encode(self, m: Sequence[int]) -> List[int]:
        assert len(m) == self.length
        out = []
        for v in m:
            assert 0 <= v < (1 << self.bits)
            out += [(v >> i) & 1 for i in range(self.bits)]
        return out

    def valid(self, g, meas, joint_rand, num_shares):
        return parallel_sum_range_checks(self.Field, g[0], self.gadgets[0].CALLS, meas,
                                         joint_rand[0], self.chunk,
                                         num_shares)

    def truncate(self, meas):
        p = self.Field.MODULUS
        out = []
        for e in range(self.length):
            chunk = meas[e * self.bits:(e + 1) * self.bits]
            out.append(sum((1 << i) * x for i, x in enumerate(chunk)) % p)
        return out

    def decode_result(self, agg):
        return list(agg)


class Histogram:
    ID = 0x00000003
    Field = Field128

    def __init__(self, length: int, chunk: int):
        self.length, self.chunk = length, chunk
        self.MEAS_LEN = length
        self.OUTPUT_LEN = length
        self.JOINT_RAND_LEN = 2
        self.QUERY_RAND_LEN = 1
        calls = (length + chunk - 1) // chunk
        self.gadgets = [ParallelSumMul(chunk, calls)]
        self.PROVE_RAND_LEN = 2 * chunk

    def encode(self, m: int) -> List[int]:
        assert 0 <= m < self.length
        return [1 if i == m else 0 for i in range(self.length)]

    def valid(self, g, meas, joint_rand, num_shares):
        p = self.Field.MODULUS
        range_check = parallel_sum_range_checks(self.Field, g[0], self.gadgets[0].CALLS, meas,
                                                joint_rand[0], self.chunk,
                                                num_shares)
        sum_check = (-self.Field.inv(num_shares)) % p
        for x in meas:
            sum_check = (sum_check + x) % p
        r = joint_rand[1]
        return (r * range_check + r * r % p * sum_check) % p

    def truncate(self, meas):
        return list(meas)

    def decode_result(self, agg):
        return list(agg)


def decode_bitvector(fld, bits: Sequence[int]) -> int:
    """prio `decode_bitvector`: sum_l 2^l x_l (mod p)."""
    p = fld.MODULUS
    return sum((1 << l) * x for l, x in enumerate(bits)) % p


class FixedPointBoundedL2VecSum:
    """prio `FixedPointBoundedL2VecSum<FixedI{16,32,64}<U{15,31,63}>, ParallelSum<PolyEval>,
    ParallelSum<Mul>>` (prio src/flp/types/fixedpoint_l2.rs, feature `experimental`), as
    instantiated by Janus for `Prio3FixedPoint{16,32,64}BitBoundedL2VecSum { length }`
    (`aggregator/src/aggregator.rs:839-861`, `Prio3::new_fixedpoint_boundedl2_vec_sum_multithreaded
    (2, length)`).  Recalled structure (confidence M):
      * entry x (fixed point, n bits, value in [-1, 1)) -> integer z = bits(x) + 2^(n-1) in
        [0, 2^n), encoded as n LE bits; then the squared L2 norm of the integer entries
        sum_e (z_e - 2^(n-1))^2 (< 2^(2n-2), i.e. norm < 1) as 2n-2 LE bits;
      * gadget 0 = ParallelSum(Mul, c0): range check of all n*entries + 2n-2 bits with
        `parallel_sum_range_checks` on joint_rand[0];
      * gadget 1 = ParallelSum(PolyEval([2^(2n-2), -2^n, 1]), c1) over the decoded entries (padding
        = share of the encoded zero 2^(n-1)/num_shares) = computed norm;
      * valid = jr[1] * range + jr[1]^2 * (computed norm - submitted norm);
      * c0 = optimal_chunk_length(n*entries + 2n-2), c1 = optimal_chunk_length(entries);
      * truncate = decoded entries; decode_result(d, c) = d * 2^(1-n) - c  (to_float_bits).
    Measurements are the fixed-point values' raw two's-complement integers (x * 2^(n-1))."""
    ID = 0xFFFF0000
    Field = Field128

    def __init__(self, bits: int, entries: int):
        assert bits in (16, 32, 64) and entries >= 1
        self.bits, self.entries = bits, entries
        self.bits_for_norm = 2 * bits - 2
        self.range_norm_begin = bits * entries
        self.range_norm_end = bits * entries + self.bits_for_norm
        self.MEAS_LEN = self.range_norm_end
        self.OUTPUT_LEN = entries
        self.JOINT_RAND_LEN = 2
        self.QUERY_RAND_LEN = 2
        self.chunk0 = optimal_chunk_length(self.range_norm_end)
        self.calls0 = (self.range_norm_end + self.chunk0 - 1) // self.chunk0
        self.chunk1 = optimal_chunk_length(entries)
        self.calls1 = (entries + self.chunk1 - 1) // self.chunk1
        one = 1 << (bits - 1)
        self.norm_summand_poly = [one * one, -2 * one, 1]
        self.gadgets = [ParallelSumMul(self.chunk0, self.calls0),
                        ParallelSumPolyEval(self.norm_summand_poly, self.chunk1, self.calls1)]
        self.PROVE_RAND_LEN = 2 * self.chunk0 + self.chunk1

    def encode(self, m: Sequence[int]) -> List[int]:
        assert len(m) == self.entries
        n = self.bits
        out = []
        norm = 0
        for v in m:
            assert -(1 << (n - 1)) <= v < (1 << (n - 1))
            z = v + (1 << (n - 1))
            out += [(z >> l) & 1 for l in range(n)]
            norm += v * v
        if norm >= 1 << self.bits_for_norm:
            raise ValueError("measurement L2 norm exceeds 1")
        out += [(norm >> l) & 1 for l in range(self.bits_for_norm)]
        return out

    def valid(self, g, meas, joint_rand, num_shares):
        fld = self.Field
        p = fld.MODULUS
        range_check = parallel_sum_range_checks(fld, g[0], self.calls0,
                                                meas[:self.range_norm_end], joint_rand[0],
                                                self.chunk0, num_shares)
        n = self.bits
        decoded = [decode_bitvector(fld, meas[e * n:(e + 1) * n]) for e in range(self.entries)]
        zero_share = (1 << (n - 1)) * fld.inv(num_shares) % p
        computed = 0
        c1 = self.chunk1
        for i in range(0, self.entries, c1):
            chunk = decoded[i:i + c1]
            chunk = chunk + [zero_share] * (c1 - len(chunk))
            computed = (computed + g[1](chunk)) % p
        submitted = decode_bitvector(fld, meas[self.range_norm_begin:self.range_norm_end])
        norm_check = (computed - submitted) % p
        r = joint_rand[1]
        return (r * range_check + r * r % p * norm_check) % p

    def truncate(self, meas):
        n = self.bits
        return [decode_bitvector(self.Field, meas[e * n:(e + 1) * n]) for e in range(self.entries)]

    def decode_result(self, agg, num_measurements: int = None):
        """prio `CompatibleFloat::to_float` -> to_float_bits(d, c, n) = d * 2^(1-n) - c."""
        assert num_measurements is not None, "FixedPoint decode needs the report count"
        return [float(d) * 2.0 ** (1 - self.bits) - num_measurements for d in agg]


# ---------------------------------------------------------------------------------------------
# FLP (prio src/flp.rs: Type::prove / query / decide with ProveShimGadget / QueryShimGadget)
# ---------------------------------------------------------------------------------------------


def gadget_m(g) -> int:
    return next_pow2(1 + g.CALLS)


def proof_len(typ) -> int:
    return sum(g.ARITY + g.DEGREE * (gadget_m(g) - 1) + 1 for g in typ.gadgets)


def verifier_len(typ) -> int:
    return 1 + sum(g.ARITY + 1 for g in typ.gadgets)


def flp_prove(typ, meas, prove_rand, joint_rand) -> List[int]:
    fld = typ.Field
    p = fld.MODULUS
    records = []
    shims = []
    off = 0
    for g in typ.gadgets:
        rec = [[prove_rand[off + w]] for w in range(g.ARITY)]
        off += g.ARITY
        records.append(rec)

        def shim(inp, g=g, rec=rec):
            for w in range(g.ARITY):
                rec[w].append(inp[w])
            return g.eval(fld, inp)
        shims.append(shim)
    typ.valid(shims, meas, joint_rand, 1)
    proof = []
    for g, rec in zip(typ.gadgets, records):
        m = gadget_m(g)
        assert all(len(r) == 1 + g.CALLS for r in rec)
        wire_polys = [intt(fld, r + [0] * (m - len(r)), m) for r in rec]
        proof += [r[0] for r in rec]
        gp = g.eval_poly(fld, wire_polys)
        want = g.DEGREE * (m - 1) + 1
        gp = (gp + [0] * want)[:want]
        proof += [c % p for c in gp]
    return proof


def flp_query(typ, meas, proof, query_rand, joint_rand, num_shares) -> List[int]:
    fld = typ.Field
    p = fld.MODULUS
    records, shims, gpolys = [], [], []
    off = 0
    for gi, g in enumerate(typ.gadgets):
        m = gadget_m(g)
        t = query_rand[gi]
        if pow(t, m, p) == 1:
            raise ValueError("invalid query randomness: encountered root of unity")
        seeds = proof[off:off + g.ARITY]
        gp = proof[off + g.ARITY: off + g.ARITY + g.DEGREE * (m - 1) + 1]
        off += g.ARITY + g.DEGREE * (m - 1) + 1
        rec = [[s] for s in seeds]
        records.append(rec)
        gpolys.append(gp)
        alpha = fld.root(m.bit_length() - 1)
        ctr = [1]

        def shim(inp, g=g, rec=rec, gp=gp, alpha=alpha, ctr=ctr):
            for w in range(g.ARITY):
                rec[w].append(inp[w])
            out = poly_eval(fld, gp, pow(alpha, ctr[0], p))
            ctr[0] += 1
            return out
        shims.append(shim)
    v = typ.valid(shims, meas, joint_rand, num_shares)
    verifier = [v]
    for gi, (g, rec, gp) in enumerate(zip(typ.gadgets, records, gpolys)):
        m = gadget_m(g)
        t = query_rand[gi]
        for r in rec:
            coeffs = intt(fld, r + [0] * (m - len(r)), m)
            verifier.append(poly_eval(fld, coeffs, t))
        verifier.append(poly_eval(fld, gp, t))
    return verifier


def flp_decide(typ, verifier) -> bool:
    fld = typ.Field
    if verifier[0] != 0:
        return False
    off = 1
    for g in typ.gadgets:
        wires = verifier[off:off + g.ARITY]
        if g.eval(fld, wires) != verifier[off + g.ARITY]:
            return False
        off += g.ARITY + 1
    return True


# ---------------------------------------------------------------------------------------------
# Prio3 (prio src/vdaf/prio3.rs; VDAF-07 §7.2), NUM_SHARES = 2 (Janus: leader 0, helper 1 --
# `messages/src/lib.rs:511-517`).
# ---------------------------------------------------------------------------------------------


@dataclass
class InputShare:
    meas_share: Optional[List[int]] = None   # leader (explicit)
    proof_share: Optional[List[int]] = None  # leader (explicit)
    meas_seed: Optional[bytes] = None        # helper
    proof_seed: Optional[bytes] = None       # helper
    blind: Optional[bytes] = None


@dataclass
class PrepState:
    out_share: List[int]
    corrected_seed: Optional[bytes]


@dataclass
class PrepShare:
    verifier: List[int]
    part: Optional[bytes]


class Prio3:
    SHARES = 2

    def __init__(self, typ, xof=None):
        """`xof`: the XOF class (XofShake128 = prio 0.15.1 / VDAF-07, the default;
        XofTurboShake128 = the VDAF-08+ forward-compatibility mode, parity unpinned)."""
        self.typ = typ
        self.xof = xof or XofShake128
        self.fld = typ.Field
        self.PROOF_LEN = proof_len(typ)
        self.VERIFIER_LEN = verifier_len(typ)

    # -- constructors mirroring prio `Prio3::new_*` (as called at aggregator.rs:797-840) --------
    @classmethod
    def new_count(cls):
        return cls(Count())

    @classmethod
    def new_sum(cls, bits):
        return cls(Sum(bits))

    @classmethod
    def new_sum_vec(cls, bits, length, chunk_length):
        return cls(SumVec(bits, length, chunk_length))

    @classmethod
    def new_histogram(cls, length, chunk_length):
        return cls(Histogram(length, chunk_length))

    @classmethod
    def new_fixedpoint_boundedl2_vec_sum(cls, bits, entries):
        """Janus `VdafInstance::Prio3FixedPoint{16,32,64}BitBoundedL2VecSum { length }`."""
        return cls(FixedPointBoundedL2VecSum(bits, entries))

    def dst(self, usage):
        return domain_separation_tag(self.typ.ID, usage)

    @property
    def uses_jr(self):
        return self.typ.JOINT_RAND_LEN > 0

    # -- sizes of the DAP/VDAF encodings ----------------------------------------------------------
    def leader_input_share_len(self):
        es = self.fld.ENCODED_SIZE
        return es * (self.typ.MEAS_LEN + self.PROOF_LEN) + (SEED_SIZE if self.uses_jr else 0)

    def helper_input_share_len(self):
        return SEED_SIZE * (3 if self.uses_jr else 2)

    def public_share_len(self):
        return 2 * SEED_SIZE if self.uses_jr else 0

    def prep_share_len(self):
        return self.fld.ENCODED_SIZE * self.VERIFIER_LEN + (SEED_SIZE if self.uses_jr else 0)

    def prep_msg_len(self):
        return SEED_SIZE if self.uses_jr else 0

    def random_size(self):
        # per helper: meas seed, proof seed, [blind]; [leader blind]; prove seed
        n = 2 * (self.SHARES - 1) + 1
        if self.uses_jr:
            n += self.SHARES
        return n * SEED_SIZE

    # -- helpers -------------------------------------------------------------------------------
    def joint_rand_part(self, j: int, blind: bytes, meas_share, nonce: bytes) -> bytes:
        return derive_seed(blind, self.dst(DST_JOINT_RAND_PART),
                           bytes([j]) + nonce + self.fld.encode_vec(meas_share), self.xof)

    def joint_rand_seed(self, parts: Sequence[bytes]) -> bytes:
        return derive_seed(bytes(SEED_SIZE), self.dst(DST_JOINT_RAND_SEED), b"".join(parts),
                           self.xof)

    def joint_rand(self, seed: bytes) -> List[int]:
        return self.xof(seed, self.dst(DST_JOINT_RANDOMNESS)).next_vec(
            self.fld, self.typ.JOINT_RAND_LEN)

    def query_rand(self, verify_key: bytes, nonce: bytes) -> List[int]:
        return self.xof(verify_key, self.dst(DST_QUERY_RANDOMNESS), nonce).next_vec(
            self.fld, self.typ.QUERY_RAND_LEN)

    def expand_meas_share(self, seed: bytes, j: int) -> List[int]:
        return self.xof(seed, self.dst(DST_MEASUREMENT_SHARE), bytes([j])).next_vec(
            self.fld, self.typ.MEAS_LEN)

    def expand_proof_share(self, seed: bytes, j: int) -> List[int]:
        return self.xof(seed, self.dst(DST_PROOF_SHARE), bytes([j])).next_vec(
            self.fld, self.PROOF_LEN)

    # -- Client::shard (prio `shard_with_random`) ------------------------------------------------
    def shard(self, measurement, nonce: bytes, rand: bytes):
        assert len(rand) == self.random_size() and len(nonce) == 16
        p = self.fld.MODULUS
        seeds = [rand[i:i + SEED_SIZE] for i in range(0, len(rand), SEED_SIZE)]
        encoded = self.typ.encode(measurement)
        leader_meas = list(encoded)
        helpers = []
        parts = []
        it = iter(seeds)
        for j in range(1, self.SHARES):
            k_meas, k_proof = next(it), next(it)
            hm = self.expand_meas_share(k_meas, j)
            leader_meas = [(x - y) % p for x, y in zip(leader_meas, hm)]
            blind = None
            if self.uses_jr:
                blind = next(it)
                parts.append(self.joint_rand_part(j, blind, hm, nonce))
            helpers.append(InputShare(meas_seed=k_meas, proof_seed=k_proof, blind=blind))
        leader_blind = None
        public_parts = None
        joint_rand = []
        if self.uses_jr:
            leader_blind = next(it)
            public_parts = [self.joint_rand_part(0, leader_blind, leader_meas, nonce)] + parts
            joint_rand = self.joint_rand(self.joint_rand_seed(public_parts))
        k_prove = next(it)
        prove_rand = self.xof(k_prove, self.dst(DST_PROVE_RANDOMNESS)).next_vec(
            self.fld, self.typ.PROVE_RAND_LEN)
        proof = flp_prove(self.typ, encoded, prove_rand, joint_rand)
        leader_proof = list(proof)
        for j, h in enumerate(helpers, start=1):
            hp = self.expand_proof_share(h.proof_seed, j)
            leader_proof = [(x - y) % p for x, y in zip(leader_proof, hp)]
        leader = InputShare(meas_share=leader_meas, proof_share=leader_proof, blind=leader_blind)
        return public_parts, [leader] + helpers

    # -- Aggregator::prepare_init ------------------------------------------------------------------
    def prepare_init(self, verify_key: bytes, agg_id: int, nonce: bytes, public_parts, share):
        query_rand = self.query_rand(verify_key, nonce)
        if agg_id == 0:
            meas, proof = share.meas_share, share.proof_share
        else:
            meas = self.expand_meas_share(share.meas_seed, agg_id)
            proof = self.expand_proof_share(share.proof_seed, agg_id)
        corrected_seed, own_part, joint_rand = None, None, []
        if self.uses_jr:
            own_part = self.joint_rand_part(agg_id, share.blind, meas, nonce)
            parts = list(public_parts)
            parts[agg_id] = own_part
            corrected_seed = self.joint_rand_seed(parts)
            joint_rand = self.joint_rand(corrected_seed)
        verifier = flp_query(self.typ, meas, proof, query_rand, joint_rand, self.SHARES)
        out_share = self.typ.truncate(meas)
        return PrepState(out_share, corrected_seed), PrepShare(verifier, own_part)

    # -- Aggregator::prepare_shares_to_prepare_message -----------------------------------------
    def prep_shares_to_prep(self, prep_shares: Sequence[PrepShare]) -> Optional[bytes]:
        p = self.fld.MODULUS
        verifier = [0] * self.VERIFIER_LEN
        for s in prep_shares:
            verifier = [(x + y) % p for x, y in zip(verifier, s.verifier)]
        if not flp_decide(self.typ, verifier):
            raise ValueError("proof verifier check failed")
        if self.uses_jr:
            return self.joint_rand_seed([s.part for s in prep_shares])
        return None

    # -- Aggregator::prepare_next -------------------------------------------------------------------
    def prepare_next(self, state: PrepState, prep_msg: Optional[bytes]) -> List[int]:
        if self.uses_jr and state.corrected_seed != prep_msg:
            raise ValueError("joint randomness mismatch")
        return state.out_share

    # -- Aggregator::aggregate / Collector::unshard ---------------------------------------------
    def aggregate(self, out_shares) -> List[int]:
        p = self.fld.MODULUS
        agg = [0] * self.typ.OUTPUT_LEN
        for o in out_shares:
            agg = [(x + y) % p for x, y in zip(agg, o)]
        return agg

    def unshard(self, agg_shares, num_measurements: int = None):
        """Collector::unshard (collector/src/lib.rs:539): decode_result(sum of shares); the
        fixed-point type also needs the report count (prio to_float_bits)."""
        agg = self.aggregate(agg_shares)
        if isinstance(self.typ, FixedPointBoundedL2VecSum):
            return self.typ.decode_result(agg, num_measurements)
        return self.typ.decode_result(agg)

    # -- codecs (prio `Encode` impls; Janus decodes with (vdaf, agg_id) at aggregator.rs:1738) ---
    def encode_input_share(self, s: InputShare) -> bytes:
        if s.meas_share is not None:
            b = self.fld.encode_vec(s.meas_share) + self.fld.encode_vec(s.proof_share)
        else:
            b = s.meas_seed + s.proof_seed
        return b + (s.blind if self.uses_jr else b"")

    def decode_input_share(self, agg_id: int, b: bytes) -> InputShare:
        es = self.fld.ENCODED_SIZE
        if len(b) != (self.leader_input_share_len() if agg_id == 0 else
                      self.helper_input_share_len()):
            raise ValueError("bad input share length")
        blind = b[-SEED_SIZE:] if self.uses_jr else None
        if agg_id == 0:
            ml = es * self.typ.MEAS_LEN
            pl = es * self.PROOF_LEN
            return InputShare(meas_share=self.fld.decode_vec(b[:ml]),
                              proof_share=self.fld.decode_vec(b[ml:ml + pl]), blind=blind)
        return InputShare(meas_seed=b[:16], proof_seed=b[16:32], blind=blind)

    def encode_public_share(self, parts) -> bytes:
        return b"".join(parts) if self.uses_jr else b""

    def decode_public_share(self, b: bytes):
        if len(b) != self.public_share_len():
            raise ValueError("bad public share length")
        return [b[:16], b[16:32]] if self.uses_jr else None

    def encode_prep_share(self, s: PrepShare) -> bytes:
        return self.fld.encode_vec(s.verifier) + (s.part if self.uses_jr else b"")

    def decode_prep_share(self, b: bytes) -> PrepShare:
        es = self.fld.ENCODED_SIZE
        vl = es * self.VERIFIER_LEN
        if len(b) != self.prep_share_len():
            raise ValueError("bad prep share length")
        return PrepShare(self.fld.decode_vec(b[:vl]), b[vl:] if self.uses_jr else None)


# ---------------------------------------------------------------------------------------------
# Transcript (mirror of `core/src/test_util/mod.rs:50-233` run_vdaf / VdafTranscript)
# ---------------------------------------------------------------------------------------------


def run_vdaf(vdaf: Prio3, verify_key: bytes, nonce: bytes, measurement, rand: bytes) -> dict:
    public_parts, shares = vdaf.shard(measurement, nonce, rand)
    l_state, l_share = vdaf.prepare_init(verify_key, 0, nonce, public_parts, shares[0])
    h_state, h_share = vdaf.prepare_init(verify_key, 1, nonce, public_parts, shares[1])
    prep_msg = vdaf.prep_shares_to_prep([l_share, h_share])
    h_out = vdaf.prepare_next(h_state, prep_msg)
    l_out = vdaf.prepare_next(l_state, prep_msg)
    return dict(
        public_share=vdaf.encode_public_share(public_parts),
        leader_input_share=vdaf.encode_input_share(shares[0]),
        helper_input_share=vdaf.encode_input_share(shares[1]),
        leader_prep_share=vdaf.encode_prep_share(l_share),
        helper_prep_share=vdaf.encode_prep_share(h_share),
        prep_msg=prep_msg if prep_msg is not None else b"",
        leader_out_share=vdaf.fld.encode_vec(l_out),
        helper_out_share=vdaf.fld.encode_vec(h_out),
    )


# ---------------------------------------------------------------------------------------------
# Deterministic synthetic reports:
#   rand_i = SHAKE128("janus-prio3-bench" || cfg_id || u64le(i))
#   verify key = SHAKE128("verify-key" || cfg_id)[:16]
# ---------------------------------------------------------------------------------------------


def synth_verify_key(cfg_id: bytes) -> bytes:
    return hashlib.shake_128(b"verify-key" + cfg_id).digest(16)


def synth_report_rand(cfg_id: bytes, i: int, nbytes: int) -> bytes:
    return hashlib.shake_128(b"janus-prio3-bench" + cfg_id + i.to_bytes(8, "little")).digest(nbytes)


def synth_measurement(vdaf: Prio3, stream: bytes):
    """Measurement drawn from the tail of the per-report stream (deterministic)."""
    typ = vdaf.typ
    if isinstance(typ, Count):
        return stream[0] & 1
    if isinstance(typ, Sum):
        return int.from_bytes(stream[:8], "little") % (1 << typ.bits)
    if isinstance(typ, Histogram):
        return int.from_bytes(stream[:8], "little") % typ.length
    if isinstance(typ, SumVec):
        nb = (typ.bits + 7) // 8
        return [int.from_bytes(stream[i * nb:(i + 1) * nb], "little") % (1 << typ.bits)
                for i in range(typ.length)]
    if isinstance(typ, FixedPointBoundedL2VecSum):
        return synth_fixedpoint(typ.bits, typ.entries, stream)
    raise TypeError(typ)


def synth_fixedpoint(bits: int, entries: int, stream: bytes) -> List[int]:
    """x_j = u_j / sqrt(entries), u_j uniform in [-1, 1], quantized:
    integer entries uniform in [-B, B] with entries * B^2 <= (2^(n-1) - 1)^2, so the L2 norm < 1.
    8 stream bytes per entry."""
    import math
    one = (1 << (bits - 1)) - 1
    B = math.isqrt(one * one // entries)
    return [int.from_bytes(stream[8 * j:8 * j + 8], "little") % (2 * B + 1) - B
            for j in range(entries)]


def synth_meas_bytes(typ) -> int:
    if isinstance(typ, SumVec):
        return typ.length * ((typ.bits + 7) // 8)
    if isinstance(typ, FixedPointBoundedL2VecSum):
        return 8 * typ.entries
    return 8


def synth_report(vdaf: Prio3, cfg_id: bytes, i: int):
    """(nonce, measurement, rand) for report i; nonce = first 16 bytes of the stream."""
    meas_bytes = synth_meas_bytes(vdaf.typ)
    total = 16 + vdaf.random_size() + meas_bytes
    s = synth_report_rand(cfg_id, i, total)
    nonce = s[:16]
    rand = s[16:16 + vdaf.random_size()]
    meas = synth_measurement(vdaf, s[16 + vdaf.random_size():])
    return nonce, meas, rand
