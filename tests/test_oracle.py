"""CPU checks of the oracle (test infrastructure): SHAKE128 against FIPS 202 / hashlib, field
constants, the committed golden transcripts, the C restatement against the Python restatement,
and the end-to-end property unshard(aggregate) == plaintext sum
(integration_tests/tests/common/mod.rs:225-398)."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import prio3 as O
from tests.reports import CONFIGS, make_batch, plaintext_sum

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "prio3_transcripts.json")))


def test_shake128_fips202_kat():
    # FIPS 202 / NIST example: SHAKE128("") first 16 bytes
    assert hashlib.shake_128(b"").hexdigest(16) == "7f9c2ba4e88f827d616045507605853e"
    x = O.XofShake128(bytes(16), O.domain_separation_tag(2, 1), b"\x01")
    assert x.stream(32) == hashlib.shake_128(b"\x08" + O.domain_separation_tag(2, 1) +
                                             bytes(16) + b"\x01").digest(32)


def test_c_keccak_matches_hashlib():
    from oracle.ref import lib
    l = lib()
    l.p3ref_shake128.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    rng = np.random.default_rng(1)
    for n in [0, 1, 167, 168, 169, 336, 1000]:
        msg = rng.integers(0, 256, n, dtype=np.uint8)
        out = np.zeros(500, np.uint8)
        l.p3ref_shake128(msg.ctypes.data, n, out.ctypes.data, 500)
        assert out.tobytes() == hashlib.shake_128(msg.tobytes()).digest(500)


def test_field_constants():
    for F, k in ((O.Field64, 32), (O.Field128, 66)):
        p = F.MODULUS
        assert (p - 1) % (1 << k) == 0
        g = F.GEN
        assert pow(g, 1 << k, p) == 1 and pow(g, 1 << (k - 1), p) != 1
    assert O.Field64.MODULUS == 18446744069414584321
    assert O.Field128.MODULUS == 340282366920938462946865773367900766209
    assert O.Field64.GEN == 1753635133440165772
    assert O.Field128.GEN == 145091266659756586618791329697897684742


def test_domain_separation_tag():
    # [VERSION=7, class=0, algo id u32 BE, usage u16 BE]
    assert O.domain_separation_tag(0x00000002, 7) == bytes([7, 0, 0, 0, 0, 2, 0, 7])


def _enc(b):
    if len(b) > 4096:
        return {"sha256": hashlib.sha256(b).hexdigest(), "len": len(b)}
    return b.hex()


@pytest.mark.parametrize("cfg", GOLD["configs"], ids=[c["name"] for c in GOLD["configs"]])
def test_oracle_reproduces_golden(cfg):
    v = CONFIGS[cfg["name"]]["ctor"]()
    vk = bytes.fromhex(cfg["verify_key"])
    if cfg["name"] == "sumvec_8_1000":
        pass  # one report, ~0.5 s
    lo, ho = [], []
    for rep in cfg["reports"]:
        t = O.run_vdaf(v, vk, bytes.fromhex(rep["nonce"]), rep["measurement"],
                       bytes.fromhex(rep["rand"]))
        for k, val in t.items():
            assert _enc(val) == rep[k], (cfg["name"], k)
        lo.append(v.fld.decode_vec(t["leader_out_share"]))
        ho.append(v.fld.decode_vec(t["helper_out_share"]))
    assert _enc(v.fld.encode_vec(v.aggregate(lo))) == cfg["leader_agg_share"]
    assert v.unshard([v.aggregate(lo), v.aggregate(ho)], len(lo)) == cfg["unsharded"]


@pytest.mark.parametrize("name", ["count", "sum8", "sum32", "sumvec_small", "countvec15", "hist4",
                                  "hist256", "fp16_3", "fp32_5", "fp64_4", "fp16_300"])
def test_c_restatement_matches_python(name):
    from oracle.ref import Prio3Ref
    b = make_batch(name, 5)
    c = CONFIGS[name]
    r = Prio3Ref(c["kind"], b.verify_key, c["bits"], c["length"], c["chunk"])
    g = r.gen(name.encode(), 0, 5, threads=2)
    for k in ["nonces", "public", "leader_in", "helper_in"]:
        np.testing.assert_array_equal(g[k], getattr(b, k))
    if c["kind"] == 4:  # fixed-point measurements are signed (two's complement in the u64 words)
        np.testing.assert_array_equal(g["meas"].view(np.int64), np.array(b.measurements))
    res = r.prepare_batch(b.nonces, b.public, b.leader_in, b.helper_in, threads=2)
    np.testing.assert_array_equal(res["lprep"], b.leader_prep)
    np.testing.assert_array_equal(res["hprep"], b.helper_prep)
    np.testing.assert_array_equal(res["msgs"], b.prep_msg)
    assert (res["status"] == 0).all() and res["count"] == 5


@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_small", "hist4", "fp16_3", "fp32_5"])
def test_unshard_equals_plaintext(name):
    b = make_batch(name, 12)
    v = b.vdaf
    la = v.aggregate([v.fld.decode_vec(x.tobytes()) for x in b.leader_out])
    ha = v.aggregate([v.fld.decode_vec(x.tobytes()) for x in b.helper_out])
    assert v.unshard([la, ha], b.n) == plaintext_sum(b)


def _fp_run(bits, vecs):
    v = O.Prio3.new_fixedpoint_boundedl2_vec_sum(bits, len(vecs[0]))
    q = lambda x: int(x * (1 << (bits - 1)))
    lo, ho = [], []
    for i, m in enumerate(vecs):
        t = O.run_vdaf(v, bytes(range(16)), bytes([i]) * 16, [q(x) for x in m],
                       bytes([0x11 * (i + 1) & 0xFF]) * v.random_size())
        lo.append(v.fld.decode_vec(t["leader_out_share"]))
        ho.append(v.fld.decode_vec(t["helper_out_share"]))
    return v.unshard([v.aggregate(lo), v.aggregate(ho)], len(vecs))


def test_fixedpoint16_e2e_kat():
    """interop_binaries/tests/end_to_end.rs:689-723: FixedI16 vectors -> ["0.5","0.5","0.6875"]."""
    got = _fp_run(16, [[.25, .125, .125], [.0625, .125, .0625], [.125, .125, .25],
                       [.0625, .125, .25]])
    assert [repr(x) for x in got] == ["0.5", "0.5", "0.6875"]


def test_fixedpoint32_collector_kat():
    """collector/src/lib.rs:1033-1110: one FixedI32 report [1/16, 1/8, 1/4] -> same values;
    end_to_end.rs e2e_prio3_fixed32vec uses the FP16 vectors at 32 bits -> same sums."""
    assert _fp_run(32, [[.0625, .125, .25]]) == [0.0625, 0.125, 0.25]
    got = _fp_run(32, [[.25, .125, .125], [.0625, .125, .0625], [.125, .125, .25],
                       [.0625, .125, .25]])
    assert got == [0.5, 0.5, 0.6875]


def test_fixedpoint_shapes():
    """Chunk lengths from prio's optimal_chunk_length; proof/verifier lengths of the two gadgets."""
    v = O.Prio3.new_fixedpoint_boundedl2_vec_sum(16, 100000)
    t = v.typ
    assert t.MEAS_LEN == 16 * 100000 + 30
    assert (t.chunk0, t.calls0, t.chunk1, t.calls1) == (1565, 1023, 393, 255)
    assert v.PROOF_LEN == 2 * 1565 + 2 * 1023 + 1 + 393 + 2 * 255 + 1
    assert v.VERIFIER_LEN == 1 + 2 * 1565 + 1 + 393 + 1
    with pytest.raises(ValueError):  # norm >= 1 is not encodable
        O.FixedPointBoundedL2VecSum(16, 2).encode([-(1 << 15), 0])


def test_tampered_share_rejected_by_oracle():
    b = make_batch("sumvec_small", 1)
    v = b.vdaf
    share = v.decode_input_share(0, b.leader_in[0].tobytes())
    share.meas_share[0] = (share.meas_share[0] + 1) % v.fld.MODULUS
    pub = v.decode_public_share(b.public[0].tobytes())
    nonce = b.nonces[0].tobytes()
    _, lps = v.prepare_init(b.verify_key, 0, nonce, pub, share)
    _, hps = v.prepare_init(b.verify_key, 1, nonce, pub,
                            v.decode_input_share(1, b.helper_in[0].tobytes()))
    with pytest.raises(ValueError):
        v.prep_shares_to_prep([lps, hps])


def test_noncanonical_decode_rejected():
    b = make_batch("hist4", 1)
    raw = bytearray(b.leader_in[0].tobytes())
    raw[:16] = b"\xff" * 16
    with pytest.raises(ValueError):
        b.vdaf.decode_input_share(0, bytes(raw))


# ---- XofTurboShake128 (VDAF-08+ forward-compatibility mode; parity unpinned) ---------------------

def test_keccak_sponge_24_rounds_is_shake128():
    """The pure-Python Keccak-p behind the TurboSHAKE oracle, run with 24 rounds and SHAKE's pad
    byte, is hashlib's SHAKE128 (FIPS 202) -- multi-block absorb and squeeze included."""
    import hashlib
    from oracle.prio3 import keccak_sponge
    for msg in (b"", b"abc", bytes(range(167)), bytes(range(168)), bytes(500)):
        assert keccak_sponge(msg, 0x1F, 400, 24) == hashlib.shake_128(msg).digest(400)


def test_turboshake128_rfc9861_vectors():
    """RFC 9861 TurboSHAKE128(M = empty, D = 0x1F): 32- and 64-byte outputs."""
    from oracle.prio3 import turboshake128
    v32 = bytes.fromhex("1e415f1c5983aff2169217277d17bb538cd945a397ddec541f1ce41af2c1b74c")
    v64 = v32 + bytes.fromhex("3e8ccae2a4dae56c84a04c2385c03c15e8193bdf58737363321691c05462c8df")
    assert turboshake128(b"", 0x1F, 32) == v32
    assert turboshake128(b"", 0x1F, 64) == v64


@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_small", "hist4"])
def test_turboshake_mode_round_trip(name):
    """Prio3 over XofTurboShake128: the transcript differs from XofShake128's, every report
    verifies, and unshard(aggregate) == plaintext sum."""
    from oracle import prio3 as O
    from tests.reports import make_batch, plaintext_sum
    bt = make_batch(name, 4, xof=O.XofTurboShake128)
    bs = make_batch(name, 4)
    assert (bt.leader_prep != bs.leader_prep).any()
    v = bt.vdaf
    agg_l = v.aggregate([v.fld.decode_vec(bt.leader_out[r].tobytes()) for r in range(bt.n)])
    agg_h = v.aggregate([v.fld.decode_vec(bt.helper_out[r].tobytes()) for r in range(bt.n)])
    assert v.unshard([agg_l, agg_h]) == plaintext_sum(bt)
