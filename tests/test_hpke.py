"""HPKE on host threads (janus_amd/hpke.py -> native hpke.cpp in libprio3gpu.so).

Pinned by the RFC 9180 vectors the reference's own test opens (core/src/hpke.rs:539-615, data in
tests/golden/hpke_rfc9180_vectors.json made by tests/golden/make_hpke_vectors.py), the reference's
behavioural tests (exchange_message, wrong_private_key, wrong_application_info,
wrong_associated_data, round_trip_all_algorithms: hpke.rs:345-535), and the helper loop's
per-report mapping (aggregator.rs:1634-1700).  Host-only: no GPU needed, except the last test,
which runs the pipelined helper driver through the engine."""
import json
import os

import numpy as np
import pytest

from janus_amd import codec as C
from janus_amd import hpke as H

VECTORS = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                      "hpke_rfc9180_vectors.json")))
h = bytes.fromhex
SUITES = [(k, d, a) for k in (H.KEM_X25519_HKDF_SHA256, H.KEM_P256_HKDF_SHA256)
          for d in (1, 2, 3) for a in (1, 2, 3)]


def test_vectors_cover_both_kems():
    assert len(VECTORS) == 12
    assert {v["kem_id"] for v in VECTORS} == {0x10, 0x20}


@pytest.mark.parametrize("i", range(12))
def test_decrypt_rfc9180_vector(i):
    v = VECTORS[i]
    kp = H.HpkeKeypair(H.HpkeConfig(0, v["kem_id"], v["kdf_id"], v["aead_id"], h(v["pkRm"])),
                       h(v["skRm"]))
    assert H.open_(kp, h(v["info"]), h(v["enc"]), h(v["ct"]), h(v["aad"])) == h(v["pt"])
    # the serialized public key is pk(skRm)
    assert H.public_key(v["kem_id"], h(v["skRm"])) == h(v["pkRm"])


@pytest.mark.parametrize("kem,kdf,aead", SUITES)
def test_round_trip_all_algorithms(kem, kdf, aead):
    kp = H.generate_hpke_config_and_private_key(7, kem, kdf, aead)
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_LEADER)
    for pt in (b"", b"plaintext", os.urandom(5000)):
        cid, enc, ct = H.seal(kp.config, info, pt, b"aad")
        assert cid == 7 and len(ct) == len(pt) + 16
        assert H.open_(kp, info, enc, ct, b"aad") == pt


def test_seal_with_fixed_ephemeral_key_is_deterministic():
    kp = H.generate_hpke_config_and_private_key(1)
    ske = bytes(range(1, 33))
    a = H.seal(kp.config, b"info", b"message", b"aad", ske)
    b = H.seal(kp.config, b"info", b"message", b"aad", ske)
    assert a == b and a[1] == H.public_key(kp.config.kem_id, ske)


@pytest.mark.parametrize("what", ["private_key", "info", "aad", "ct", "enc"])
def test_wrong_inputs_fail(what):
    kp = H.generate_hpke_config_and_private_key(1)
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
    _, enc, ct = H.seal(kp.config, info, b"a message that is secret", b"associated data")
    args = dict(keypair=kp, info=info, enc=enc, payload=ct, aad=b"associated data")
    if what == "private_key":
        args["keypair"] = H.HpkeKeypair(kp.config,
                                        H.generate_hpke_config_and_private_key(1).private_key)
    elif what == "info":
        args["info"] = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_LEADER)
    elif what == "aad":
        args["aad"] = b"wrong associated data"
    elif what == "ct":
        args["payload"] = ct[:-1] + bytes([ct[-1] ^ 1])
    else:
        args["enc"] = bytes([enc[0] ^ 1]) + enc[1:]
    with pytest.raises(H.HpkeError):
        H.open_(**args)


def test_unsupported_suite_is_a_configuration_error():
    kp = H.generate_hpke_config_and_private_key(1)
    bad = H.HpkeConfig(1, 0x21, 1, 1, kp.config.public_key)  # X448: not a Janus KEM
    with pytest.raises(ValueError):
        H.seal(bad, b"", b"x", b"")


def _request(task_id, nonces, times, public, payloads, keypairs, prep_share_len=4):
    """AggregationJobInitializeReq whose encrypted input shares are sealed to keypairs[i] (None:
    unknown config id 99)."""
    n = len(nonces)
    cts = []
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
    for i in range(n):
        pt = b"\x00\x00" + len(payloads[i]).to_bytes(4, "big") + payloads[i]
        aad = H.input_share_aad(task_id, nonces[i].tobytes(), times[i], public[i].tobytes())
        kp = keypairs[i]
        cts.append(H.seal(kp.config, info, pt, aad) if kp else (99, b"\x01" * 32, b"\x02" * 40))
    lps = np.zeros((n, prep_share_len), np.uint8)
    return C.encode_agg_init_req(C.TIME_INTERVAL, None, b"", nonces, times, public, cts, lps)


def test_open_report_shares_key_selection_and_errors():
    rng = np.random.default_rng(5)
    n = 40
    task_id = bytes(range(32))
    tk = H.generate_hpke_config_and_private_key(1)
    gk = H.generate_hpke_config_and_private_key(2, H.KEM_P256_HKDF_SHA256, 1, 3)
    gk_same_id = H.generate_hpke_config_and_private_key(1)  # global key sharing the task key's id
    nonces = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    times = [1_700_000_000 + i for i in range(n)]
    public = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    payloads = [bytes(rng.integers(0, 256, 48, dtype=np.uint8)) for _ in range(n)]
    kps = [tk if i % 3 == 0 else gk if i % 3 == 1 else gk_same_id for i in range(n)]
    kps[5] = None  # unknown config id
    req = C.decode_agg_init_req(bytearray(_request(task_id, nonces, times, public, payloads, kps)))
    # corrupt report 7's payload in place (AEAD tag check fails)
    v = req.views[7]
    req.raw[v.payload_off + 3] ^= 0x40
    st = np.zeros(n, np.uint8)
    st[9] = 8  # rejected by an earlier stage: skipped
    pts, offs, st = H.open_report_shares(task_id, req, [tk], [gk, gk_same_id], st, threads=4)
    for i in range(n):
        if i == 5:
            assert st[i] == 3
        elif i == 7:
            assert st[i] == 4
        elif i == 9:
            assert st[i] == 8
        else:
            # reports sealed to gk_same_id are opened by the global key after the task key
            # (same config id) fails to decrypt -- the reference's second trial
            assert st[i] == 0, i
            pt = pts[int(offs[i]):int(offs[i + 1])].tobytes()
            assert pt[6:] == payloads[i]
    # without the global keys: gk's reports have an unknown id, gk_same_id's fail to decrypt
    st2 = np.zeros(n, np.uint8)
    _, _, st2 = H.open_report_shares(task_id, req, [tk], [], st2, threads=1)
    assert all(st2[i] == 3 for i in range(n) if i % 3 == 1 and i not in (5, 7))
    assert all(st2[i] == 4 for i in range(n) if i % 3 == 2 and i not in (5, 7))
    # a wrong task id changes the AAD: every open fails
    st3 = np.zeros(n, np.uint8)
    _, _, st3 = H.open_report_shares(bytes(32), req, [tk], [gk, gk_same_id], st3)
    assert set(st3.tolist()) == {3, 4}


@pytest.mark.gpu
def test_pipelined_helper_driver_with_hpke():
    """Three aggregation jobs through HelperAggregateInit.handle_jobs (HPKE open of job k + 1 on
    host threads while the GPU prepares job k): aggregates equal the oracle's over the reports
    that survive, and the rejected ones carry the HPKE error codes."""
    from janus_amd import messages as M  # noqa: F401
    from janus_amd.helper import HelperAggregateInit
    from janus_amd.prio3 import Prio3Gpu
    from tests.reports import CONFIGS, expected_aggregate, make_batch
    name = "sumvec_small"
    b = make_batch(name, 24)
    c = CONFIGS[name]
    v = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                 chunk_length=c["chunk"])
    ls = v.new_state(0, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    task_id = os.urandom(32)
    tk = H.generate_hpke_config_and_private_key(3)
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
    times = list(range(1000, 1000 + b.n))
    cts = []
    for r in range(b.n):
        pt = b"\x00\x00" + len(b.helper_in[r]).to_bytes(4, "big") + b.helper_in[r].tobytes()
        aad = H.input_share_aad(task_id, b.nonces[r].tobytes(), times[r], b.public[r].tobytes())
        cts.append(H.seal(tk.config, info, pt, aad))
    cts[4] = (9, cts[4][1], cts[4][2])  # unknown config id
    cts[13] = (cts[13][0], cts[13][1], cts[13][2][:-1] + b"\x00")  # bad tag
    jobs = [slice(0, 8), slice(8, 16), slice(16, 24)]
    reqs = [C.encode_agg_init_req(C.TIME_INTERVAL, None, b"", b.nonces[j], times[j], b.public[j],
                                  cts[j], lp[j]) for j in jobs]
    drv = HelperAggregateInit(v, task_id, [tk], hpke_threads=4)
    hagg = v.new_aggregate(1)
    resps = drv.handle_jobs(reqs, hagg)
    st = np.zeros(b.n, np.uint8)
    for j, resp in zip(jobs, resps):
        _, st_j = C.gather_helper_resps(v.sizes, resp, b.nonces[j], np.zeros(8, np.uint8))
        st[j] = st_j
    assert st[4] == 3 and st[13] == 4 and (np.delete(st, [4, 13]) == 0).all()
    got, cnt = hagg.read(0)
    exp, ecnt = expected_aggregate(b, "helper", mask=st == 0)
    assert got == exp and cnt == ecnt == b.n - 2
    drv.close()


def test_open_report_shares_empty_request():
    empty = C.encode_agg_init_req(C.TIME_INTERVAL, None, b"", np.zeros((0, 16), np.uint8), [],
                                  np.zeros((0, 32), np.uint8), [], np.zeros((0, 4), np.uint8))
    req = C.decode_agg_init_req(empty)
    assert req.n == 0
    pts, offs, st = H.open_report_shares(bytes(32), req, [H.generate_hpke_config_and_private_key(1)])
    assert offs.tolist() == [0] and st.size == 0


def _x25519_batch(sk: bytes, points: bytes, simd: int) -> bytes:
    import ctypes
    from janus_amd._lib import lib
    n = len(points) // 32
    out = ctypes.create_string_buffer(32 * max(n, 1))
    rc = lib().prio3gpu_x25519_batch(sk, points, n, out, simd)
    if rc == -6:
        pytest.skip("host CPU has no AVX-512 IFMA")
    assert rc == 0
    return out.raw[:32 * n]


@pytest.mark.parametrize("n", [1, 3, 8, 13, 64])
def test_x25519_ifma_ladder_matches_scalar(n):
    """The 8-way IFMA ladder the batched open uses == the scalar radix-2^51 ladder, including
    points with bit 255 set and non-canonical u-coordinates (>= p), and ragged groups."""
    rng = np.random.default_rng(n)
    sk = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    pts = bytearray(rng.integers(0, 256, 32 * n, dtype=np.uint8).tobytes())
    pts[31] |= 0x80
    if n > 1:  # u = p + 3 (non-canonical) and u = 2^255 - 1
        pts[32:64] = ((1 << 255) - 19 + 3).to_bytes(32, "little")
    if n > 2:
        pts[64:96] = b"\xff" * 32
    assert _x25519_batch(sk, bytes(pts), 1) == _x25519_batch(sk, bytes(pts), 0)


def test_x25519_ifma_rfc7748_vectors():
    # RFC 7748 §5.2 test vectors 1 and 2, both through one 8-way group
    k1 = bytes.fromhex("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4")
    u1 = bytes.fromhex("e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c")
    r1 = "c3da55379de9c6908e94ea4df28d084f32eccf03491c71f754b4075577a28552"
    k2 = bytes.fromhex("4b66e9d4d1b4673c5ad22691957d6af5c11b6421e0ea01d42ca4169e7918ba0d")
    u2 = bytes.fromhex("e5210f12786811d3f4b7959d0538ae2c31dbe7106fc03c3efc4cd549c715a493")
    r2 = "95cbde9476e8907d7aade45cb4b873f88b595a68799fa152e6f8f7647aac7957"
    assert _x25519_batch(k1, u1 * 3, 1).hex() == r1 * 3
    assert _x25519_batch(k2, u2 * 9, 1).hex() == r2 * 9


def test_open_report_shares_one_key_batch_matches_single_opens():
    """A batch sealed to one X25519 key (the helper's common case: every chunk of 8 goes through
    the IFMA ladder, with a ragged tail) opens exactly like per-report hpke::open."""
    rng = np.random.default_rng(11)
    n = 37
    task_id = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    tk = H.generate_hpke_config_and_private_key(4)
    nonces = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    times = [1_600_000_000 + 7 * i for i in range(n)]
    public = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    payloads = [bytes(rng.integers(0, 256, 48, dtype=np.uint8)) for _ in range(n)]
    req = C.decode_agg_init_req(bytearray(_request(task_id, nonces, times, public, payloads,
                                                   [tk] * n)))
    v = req.views[20]
    req.raw[v.payload_off] ^= 1  # one bad tag inside a full SIMD group
    pts, offs, st = H.open_report_shares(task_id, req, [tk], [], np.zeros(n, np.uint8), threads=3)
    for i in range(n):
        if i == 20:
            assert st[i] == 4
            continue
        assert st[i] == 0, i
        assert pts[int(offs[i]):int(offs[i + 1])].tobytes()[6:] == payloads[i]


@pytest.mark.gpu
def test_pipelined_helper_driver_isolates_bad_requests():
    """handle_jobs with a duplicate-report-ID request and an empty request between valid ones:
    those entries are InvalidMessage / EmptyAggregation, the other jobs are answered and
    accumulated, and no staging buffer stays busy (one bad request must not abort
    the stream or leak the buffer of the job opened ahead)."""
    from janus_amd._lib import EmptyAggregation, InvalidMessage
    from janus_amd.helper import HelperAggregateInit
    from janus_amd.prio3 import Prio3Gpu
    from tests.reports import CONFIGS, expected_aggregate, make_batch
    name = "sum8"
    b = make_batch(name, 16)
    c = CONFIGS[name]
    v = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                 chunk_length=c["chunk"])
    task_id = os.urandom(32)
    tk = H.generate_hpke_config_and_private_key(3)
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
    times = list(range(1000, 1000 + b.n))
    cts = []
    for r in range(b.n):
        pt = b"\x00\x00" + len(b.helper_in[r]).to_bytes(4, "big") + b.helper_in[r].tobytes()
        aad = H.input_share_aad(task_id, b.nonces[r].tobytes(), times[r], b.public[r].tobytes())
        cts.append(H.seal(tk.config, info, pt, aad))

    def req(idx):
        return C.encode_agg_init_req(C.TIME_INTERVAL, None, b"", b.nonces[idx],
                                     [times[i] for i in idx], b.public[idx],
                                     [cts[i] for i in idx], b.leader_prep[idx])

    a, d = list(range(0, 8)), list(range(8, 16))
    dup = [0, 1, 2, 1]
    empty = C.encode_agg_init_req(C.TIME_INTERVAL, None, b"", np.zeros((0, 16), np.uint8), [],
                                  np.zeros((0, b.public.shape[1]), np.uint8), [],
                                  np.zeros((0, b.leader_prep.shape[1]), np.uint8))
    drv = HelperAggregateInit(v, task_id, [tk], hpke_threads=2)
    hagg = v.new_aggregate(1)
    out = drv.handle_jobs([req(a), req(dup), empty, req(d)], hagg)
    assert isinstance(out[1], InvalidMessage) and isinstance(out[2], EmptyAggregation)
    for idx, resp in ((a, out[0]), (d, out[3])):
        _, st = C.gather_helper_resps(v.sizes, resp, b.nonces[idx], np.zeros(len(idx), np.uint8))
        assert (st == 0).all()
    got, cnt = hagg.read(0)
    exp, ecnt = expected_aggregate(b, "helper")
    assert got == exp and cnt == ecnt == b.n
    assert not any(drv._pinned._busy)
    drv.close()
