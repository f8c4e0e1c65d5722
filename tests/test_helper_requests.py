"""Helper aggregate-init request handling on the host (no GPU): the request-level checks of
`handle_aggregate_init_generic` and the per-report error precedence of its loop.

Reference: aggregator/src/aggregator.rs
  :1586        AggregationJobInitializeReq::get_decoded (malformed -> whole request fails)
  :1588-1598   duplicate report IDs -> Error::InvalidMessage (whole request)
  :1605        A::AggregationParam::get_decoded: Prio3's `()` accepts only empty bytes
  :1663-1700   HpkeUnknownConfigId (3), then HpkeDecryptError (4)
  :1702-1753   PlaintextInputShare / duplicate extensions / input share decode -> InvalidMessage (8)
  :1755-1770   public share decode -> InvalidMessage (8), checked only once the input share decoded
  :1775-1797   ping-pong (message type, prep share decode) -> VdafPrepError (5)
  :1851-1863   no reports -> Error::EmptyAggregation
"""
import json
import os
import struct

import numpy as np
import pytest

from janus_amd import codec as C
from janus_amd import hpke as H
from janus_amd import messages as M
from janus_amd._lib import EmptyAggregation, InvalidMessage
from janus_amd.helper import HelperAggregateInit
from janus_amd.prio3 import _Sizes

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dap_framing_kats.json")))

PUB, PREP, HIN = 32, 64, 48  # public share, leader prep share, helper input share (bytes)


def _sizes():
    s = _Sizes()
    s.public_share, s.prep_share, s.prep_msg = PUB, PREP, 16
    s.helper_input_share, s.leader_input_share = HIN, HIN
    return s


class _StubVdaf:
    """Only what HelperAggregateInit.open reads (the engine itself is not called here)."""
    sizes = _sizes()


def _req(agg_param, prepare_inits):
    body = b"".join(prepare_inits)
    return struct.pack(">I", len(agg_param)) + agg_param + b"\x01" + struct.pack(">I", len(body)) + body


def test_duplicate_report_ids_fail_the_request():
    rng = np.random.default_rng(3)
    n = 5000
    ids = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    pis = [M.encode_prepare_init(M.encode_report_share(ids[i].tobytes(), i, bytes(PUB), 1, b"e",
                                                       b"p"),
                                 M.encode_ping_pong(M.PING_PONG_INITIALIZE, prep_share=bytes(PREP)))
           for i in range(n)]
    ok = C.decode_agg_init_req(_req(b"", pis))
    C.check_agg_init_req(ok)  # distinct ids pass
    dup = list(pis)
    dup[4321] = dup[17]  # the same PrepareInit twice
    with pytest.raises(InvalidMessage, match="duplicate report IDs"):
        C.check_agg_init_req(C.decode_agg_init_req(_req(b"", dup)))
    # ids differing only in the last byte are distinct
    a = bytes(15) + b"\x01"
    b = bytes(15) + b"\x02"
    two = [M.encode_prepare_init(M.encode_report_share(x, 0, bytes(PUB), 1, b"", b""),
                                 M.encode_ping_pong(M.PING_PONG_INITIALIZE, prep_share=b""))
           for x in (a, b)]
    C.check_agg_init_req(C.decode_agg_init_req(_req(b"", two)))


def test_non_empty_aggregation_parameter_fails_the_request():
    # the reference's own KAT request carries agg_param "012345": decodable DAP, but not Prio3's ()
    k = KATS["agg_init_req"]
    req = C.decode_agg_init_req(bytes.fromhex(k["time_interval"]))
    assert req.agg_param == bytes.fromhex(k["agg_param"])
    with pytest.raises(InvalidMessage, match="aggregation parameter"):
        C.check_agg_init_req(req)


def test_empty_and_invalid_requests_through_the_driver():
    drv = HelperAggregateInit(_StubVdaf(), bytes(32), [H.generate_hpke_config_and_private_key(1)])
    with pytest.raises(EmptyAggregation):
        drv.open(_req(b"", []))
    pi = M.encode_prepare_init(M.encode_report_share(bytes(16), 0, bytes(PUB), 1, b"", b""),
                               M.encode_ping_pong(M.PING_PONG_INITIALIZE, prep_share=bytes(PREP)))
    with pytest.raises(InvalidMessage):
        drv.open(_req(b"", [pi, pi]))
    with pytest.raises(InvalidMessage):
        drv.open(_req(b"\x00", [pi]))


def test_error_precedence_with_two_faults_per_report():
    """Reports carrying two faults each get the status of the one Janus checks first."""
    rng = np.random.default_rng(9)
    task_id = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    kp = H.generate_hpke_config_and_private_key(7)
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
    good_pt = lambda payload: b"\x00\x00" + struct.pack(">I", len(payload)) + payload
    dup_ext_pt = (struct.pack(">H", 8) + b"\x00\x01\x00\x00" * 2 + struct.pack(">I", HIN)
                  + bytes(HIN))
    init = lambda n: M.encode_ping_pong(M.PING_PONG_INITIALIZE, prep_share=bytes(n))
    finish = M.encode_ping_pong(M.PING_PONG_FINISH, prep_msg=bytes(16))
    cont = M.encode_ping_pong(M.PING_PONG_CONTINUE, prep_msg=bytes(16), prep_share=bytes(PREP))
    # (plaintext, public share length, ping-pong message, seal mode, expected status)
    cases = [
        (good_pt(bytes(HIN)), PUB, init(PREP), "ok", 0),
        (good_pt(bytes(HIN)), PUB, finish, "bad_tag", 4),        # HPKE before ping-pong
        (good_pt(bytes(HIN)), PUB - 1, init(PREP), "unknown_id", 3),  # HPKE id before public share
        (b"\x00", PUB, init(PREP - 1), "ok", 8),                  # plaintext before ping-pong
        (dup_ext_pt, PUB, cont, "ok", 8),                         # duplicate extension before ping-pong
        (good_pt(bytes(HIN - 1)), PUB + 1, init(PREP), "ok", 8),  # input share, then public share
        (good_pt(bytes(HIN)), PUB + 3, finish, "ok", 8),          # public share before ping-pong
        (good_pt(bytes(HIN)), PUB, cont, "ok", 5),                # ping-pong alone
        (good_pt(bytes(HIN)), PUB, init(PREP + 1), "ok", 5),      # wrong prep share length
        (good_pt(bytes(HIN)), PUB, init(PREP), "bad_tag", 4),
    ]
    pis = []
    for i, (pt, plen, pp, mode, _) in enumerate(cases):
        rid = bytes([i + 1]) * 16
        pub = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
        aad = H.input_share_aad(task_id, rid, 1000 + i, pub)
        cid, enc, payload = H.seal(kp.config, info, pt, aad)
        if mode == "bad_tag":
            payload = payload[:-1] + bytes([payload[-1] ^ 1])
        if mode == "unknown_id":
            cid = (cid + 1) % 256
        pis.append(M.encode_prepare_init(M.encode_report_share(rid, 1000 + i, pub, cid, enc,
                                                               payload), pp))
    drv = HelperAggregateInit(_StubVdaf(), task_id, [kp], hpke_threads=2)
    o = drv.open(_req(b"", pis))
    assert o.status.tolist() == [c[-1] for c in cases]
    assert o.nonces[0].tobytes() == bytes([1]) * 16 and (o.times == 1000 + np.arange(len(cases))).all()
    # rows of the reports with a structural fault are zeroed; the good report's prep share is kept
    assert not o.leader_prep[[3, 6, 7, 8]].any()
    drv.close()


def test_staging_buffers_survive_opens_ahead_of_prepare():
    """opening several jobs before preparing any must not overwrite a previous job's
    leader prep shares (each opened job owns its staging buffer until prepare)."""
    from janus_amd.helper import _PinnedPool
    pool = _PinnedPool(8)
    # without a GPU the pool hands out nothing (gather allocates per job): still no aliasing
    k1, b1 = pool.acquire(4)
    k2, b2 = pool.acquire(4)
    assert (k1, b1) == (-1, None) or (k1 != k2 and b1 is not b2)
    pool.release(k1)
    pool.release(k2)
