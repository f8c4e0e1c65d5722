"""DAP framing of the aggregate-init messages (janus_amd/messages.py) against the reference's own
KATs (messages/src/lib.rs:4094-4280), stored as data in tests/golden/dap_framing_kats.json."""
import json
import os

from janus_amd import messages as M

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dap_framing_kats.json")))


def h(s):
    return bytes.fromhex(s.replace(" ", ""))


def test_prepare_init_kats():
    for k in KATS["prepare_init"]:
        rs = M.encode_report_share(h(k["report_id"]), k["time"], h(k["public_share"]),
                                   k["config_id"], h(k["enc"]), h(k["payload"]))
        msg = k["message"]
        if msg["type"] == 0:
            pp = M.encode_ping_pong(M.PING_PONG_INITIALIZE, prep_share=h(msg["prep_share"]))
        else:
            pp = M.encode_ping_pong(M.PING_PONG_FINISH, prep_msg=h(msg["prep_msg"]))
        got = M.encode_prepare_init(rs, pp)
        exp = h(k["expected"]) + h(k["expected_tail"]) + h(k["expected_message"])
        assert got == exp


def test_prepare_resp_kats():
    for k in KATS["prepare_resp"]:
        rid = h(k["report_id"])
        if k["step"] == 0:
            m = k["message"]
            pp = M.encode_ping_pong(M.PING_PONG_CONTINUE, prep_msg=h(m["prep_msg"]),
                                    prep_share=h(m["prep_share"]))
            got = M.encode_prepare_resp(rid, M.STEP_CONTINUE, message=pp)
        elif k["step"] == 1:
            got = M.encode_prepare_resp(rid, M.STEP_FINISHED)
        else:
            got = M.encode_prepare_resp(rid, M.STEP_REJECT, error=k["error"])
        assert got == h(k["expected"])


def test_prepare_error_codes_match_status_codes():
    from janus_amd.prio3 import STATUS_INVALID_MESSAGE, STATUS_VDAF_PREP_ERROR
    assert int(KATS["prepare_error"]["VdafPrepError"], 16) == STATUS_VDAF_PREP_ERROR
    assert STATUS_INVALID_MESSAGE == 8  # PrepareError::InvalidMessage (lib.rs:2288-2298)


def test_helper_batch_responses():
    nonces = [bytes([i]) * 16 for i in range(3)]
    msgs = [bytes([0xA0 + i]) * 16 for i in range(3)]
    out = M.helper_prepare_resps(nonces, msgs, [0, 5, 0])
    assert out[0] == nonces[0] + b"\x00\x02" + (16).to_bytes(4, "big") + msgs[0]
    assert out[1] == nonces[1] + b"\x02\x05"
