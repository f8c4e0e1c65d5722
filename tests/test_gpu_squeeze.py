"""XOF squeeze parity: prio 0.15.1 `into_field_vec` rejection sampling (XofShake128::next_vec).

Real SHAKE128 output hits a non-canonical Field128 chunk with probability 28/2^64, so the exact
per-element branches of the device squeeze (janus_amd/csrc/prio3_kernels.h SqueezeVec: Field128
even/odd block parity with the element that straddles two rate blocks, Field64) never run on real
reports.  Two checks close that gap:
  * `prio3gpu_test_squeeze` runs the very same SqueezeVec code over caller-crafted rate blocks that
    are dense in non-canonical chunks and edge values (p - 1, p, 2^128 - 1, high word exactly
    2^64 - 28), against the oracle's `field_vec_from_stream` on the same bytes, with and without
    the forced exact path;
  * the engine option exact_squeeze = 1 forces the exact path in every real XOF kernel (query randomness,
    helper expansion, joint randomness, shard): every golden config must stay byte-identical.
"""
import ctypes

import numpy as np
import pytest

from oracle.prio3 import Field64, Field128, XofShake128, field_vec_from_stream

P128, P64 = Field128.MODULUS, Field64.MODULUS
RATE = 168


def _edge_chunks128(rng, nchunks):
    """16-byte chunks, ~40 % non-canonical or on the p boundary."""
    hi_max = (1 << 64) - 1
    out = []
    for _ in range(nchunks):
        u = rng.random()
        if u < 0.5:
            x = int.from_bytes(rng.bytes(16), "little") % P128          # canonical
        elif u < 0.6:
            x = P128 - 1                                                 # largest canonical
        elif u < 0.7:
            x = P128 + int(rng.integers(0, 1 << 20))                     # p .. p + 2^20
        elif u < 0.8:
            x = (1 << 128) - 1 - int(rng.integers(0, 1 << 16))
        elif u < 0.9:
            x = ((hi_max - 27) << 64) | int.from_bytes(rng.bytes(8), "little")  # hi = 2^64 - 28
        else:
            x = ((hi_max - 28) << 64) | hi_max                            # hi just below: canonical
        out.append(x.to_bytes(16, "little"))
    return b"".join(out)


def _edge_words64(rng, nwords):
    out = []
    for _ in range(nwords):
        u = rng.random()
        if u < 0.55:
            x = int(rng.integers(0, P64, dtype=np.uint64))
        elif u < 0.65:
            x = P64 - 1
        elif u < 0.8:
            x = P64 + int(rng.integers(0, (1 << 32) - 1))
        else:
            x = (1 << 64) - 1
        out.append(x.to_bytes(8, "little"))
    return b"".join(out)


def _blocks(stream: bytes) -> np.ndarray:
    """Rate blocks as the 25-word states the test kernel feeds (capacity words zero)."""
    nb = len(stream) // RATE
    w = np.frombuffer(stream[:nb * RATE], dtype="<u8").reshape(nb, 21)
    st = np.zeros((nb, 25), np.uint64)
    st[:, :21] = w
    return np.ascontiguousarray(st)


def test_field_vec_from_stream_matches_next_vec():
    x = XofShake128(bytes(range(16)), b"\x07\x00\x00\x00\x00\x02\x00\x01", b"\x01")
    for fld in (Field64, Field128):
        assert field_vec_from_stream(fld, x.stream(16 * 100), 50) == x.next_vec(fld, 50)
    # the boundary: p - 1 kept, p and 2^128 - 1 rejected
    s = b"".join(v.to_bytes(16, "little") for v in (P128 - 1, P128, (1 << 128) - 1, 5))
    assert field_vec_from_stream(Field128, s, 2) == [P128 - 1, 5]
    assert field_vec_from_stream(Field128, s, 3) is None


def _gpu_squeeze(es, blocks, n, exact):
    from janus_amd._lib import check, lib
    out = np.zeros(n * es, np.uint8)
    check(lib().prio3gpu_test_squeeze(es, blocks.ctypes.data, blocks.shape[0], n,
                                      out.ctypes.data, exact), "test_squeeze")
    return out.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [0, 1])
@pytest.mark.parametrize("seed", range(6))
def test_crafted_stream_field128(seed, exact):
    rng = np.random.default_rng(100 + seed)
    stream = _edge_chunks128(rng, 12 * RATE // 16)  # 12 rate blocks, straddling chunks included
    blocks = _blocks(stream)
    usable = stream[:blocks.shape[0] * RATE]
    avail = sum(1 for i in range(0, len(usable) - 15, 16)
                if int.from_bytes(usable[i:i + 16], "little") < P128)
    for n in sorted({1, 2, 9, 10, 11, 12, 21, 22, 23, avail // 2, avail - 1, avail}):
        if n < 1 or n > avail:
            continue
        exp = field_vec_from_stream(Field128, usable, n)
        got = _gpu_squeeze(16, blocks, n, exact)
        assert got == Field128.encode_vec(exp), (seed, n, exact)


@pytest.mark.gpu
def test_crafted_stream_field128_all_canonical_fast_path():
    """Canonical chunks only: the fast block path (bulk stores) and the exact path agree."""
    rng = np.random.default_rng(7)
    stream = b"".join((int.from_bytes(rng.bytes(16), "little") % P128).to_bytes(16, "little")
                      for _ in range(20 * RATE // 16))
    blocks = _blocks(stream)
    for n in (10, 11, 21, 22, 32, 100, 200):
        exp = Field128.encode_vec(field_vec_from_stream(Field128, stream, n))
        assert _gpu_squeeze(16, blocks, n, 0) == exp == _gpu_squeeze(16, blocks, n, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_crafted_stream_field64(seed):
    rng = np.random.default_rng(200 + seed)
    stream = _edge_words64(rng, 10 * 21)
    blocks = _blocks(stream)
    avail = sum(1 for i in range(0, len(stream), 8) if int.from_bytes(stream[i:i + 8], "little") < P64)
    for n in sorted({1, 20, 21, 22, avail - 1, avail}):
        exp = field_vec_from_stream(Field64, stream, n)
        assert _gpu_squeeze(8, blocks, n, 0) == Field64.encode_vec(exp), (seed, n)


@pytest.mark.gpu
def test_crafted_stream_overrun_is_an_error():
    from janus_amd._lib import Prio3GpuError
    rng = np.random.default_rng(1)
    blocks = _blocks(_edge_chunks128(rng, 2 * RATE // 16))
    with pytest.raises(Prio3GpuError, match="more blocks"):
        _gpu_squeeze(16, blocks, 1000, 0)


# ---- the real kernels with the exact path forced ------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["count", "sum8", "sum32", "sumvec_small", "countvec15", "hist4",
                                  "hist256", "sumvec_8_1000", "fp16_3", "fp32_5", "fp64_4",
                                  "fp16_300", "fp16_5000"])
def test_exact_squeeze_forced_transcript_bit_exact(name):
    from tests.test_gpu_parity import batch, gpu_vdaf
    from tests.reports import meas_array
    b = batch(name)
    v = gpu_vdaf(b)
    v.set_option("exact_squeeze", 1)
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    hp, hst = v.prepare_init(hs, b.nonces, b.public, b.helper_in)
    assert (lst == 0).all() and (hst == 0).all()
    np.testing.assert_array_equal(lp, b.leader_prep)
    np.testing.assert_array_equal(hp, b.helper_prep)
    msgs, st = v.prepare_shares_to_prepare_message(lp, hp)
    np.testing.assert_array_equal(msgs, b.prep_msg)
    ho, hst = v.prepare_next(hs, msgs, hst.copy())
    np.testing.assert_array_equal(ho, b.helper_out)
    if not name.startswith("fp"):  # Client::shard (k_shard_jr: joint rand + prove rand squeezes)
        pub, lead, helper = v.shard(v.new_state(1, b.n), b.nonces, meas_array(b), b.rand)
        np.testing.assert_array_equal(lead, b.leader_in)
        if v.sizes.public_share:
            np.testing.assert_array_equal(pub, b.public)
