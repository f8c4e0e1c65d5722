"""DAP-07 framing for the aggregate-init messages that carry the engine's batch outputs.

Mirrors `messages/src/lib.rs` (Janus 0.6): `PingPongMessage` (`Initialize` = 0x00 + u32-len
prep_share; `Continue` = 0x01 + u32-len prep_msg + u32-len prep_share; `Finish` = 0x02 + u32-len
prep_msg), `PrepareResp` (report_id[16] + PrepareStepResult: 0x00 Continue{msg} | 0x01 Finished |
0x02 Reject{PrepareError u8}, lib.rs:2187-2317), `PrepareInit` (ReportShare + PingPongMessage,
lib.rs:2136-2185).  Pinned by the reference's own KATs (lib.rs:4094-4280) in tests/test_messages.py.
"""
from __future__ import annotations

import struct
from typing import Iterable, List, Optional

PING_PONG_INITIALIZE, PING_PONG_CONTINUE, PING_PONG_FINISH = 0, 1, 2
STEP_CONTINUE, STEP_FINISHED, STEP_REJECT = 0, 1, 2


def _u32_opaque(b: bytes) -> bytes:
    return struct.pack(">I", len(b)) + bytes(b)


def encode_ping_pong(kind: int, prep_msg: Optional[bytes] = None,
                     prep_share: Optional[bytes] = None) -> bytes:
    if kind == PING_PONG_INITIALIZE:
        return b"\x00" + _u32_opaque(prep_share)
    if kind == PING_PONG_CONTINUE:
        return b"\x01" + _u32_opaque(prep_msg) + _u32_opaque(prep_share)
    if kind == PING_PONG_FINISH:
        return b"\x02" + _u32_opaque(prep_msg)
    raise ValueError(kind)


def encode_prepare_resp(report_id: bytes, step: int, message: Optional[bytes] = None,
                        error: Optional[int] = None) -> bytes:
    assert len(report_id) == 16
    if step == STEP_CONTINUE:
        return bytes(report_id) + b"\x00" + message
    if step == STEP_FINISHED:
        return bytes(report_id) + b"\x01"
    if step == STEP_REJECT:
        return bytes(report_id) + b"\x02" + bytes([error])
    raise ValueError(step)


def encode_report_share(report_id: bytes, time: int, public_share: bytes, config_id: int,
                        encapsulated_key: bytes, payload: bytes) -> bytes:
    return (bytes(report_id) + struct.pack(">Q", time) + _u32_opaque(public_share)
            + bytes([config_id]) + struct.pack(">H", len(encapsulated_key)) + encapsulated_key
            + _u32_opaque(payload))


def encode_prepare_init(report_share: bytes, ping_pong: bytes) -> bytes:
    return report_share + ping_pong


def helper_prepare_resps(nonces, prep_msgs, status) -> List[bytes]:
    """The helper's per-report responses for one aggregate-init batch (aggregator.rs:1811-1830):
    ok -> Continue{Finish{prep_msg}}, else Reject(status as PrepareError)."""
    out = []
    for r in range(len(status)):
        rid = bytes(nonces[r])
        st = int(status[r])
        if st == 0:
            msg = bytes(prep_msgs[r]) if prep_msgs is not None and len(prep_msgs) else b""
            out.append(encode_prepare_resp(rid, STEP_CONTINUE,
                                           encode_ping_pong(PING_PONG_FINISH, prep_msg=msg)))
        else:
            out.append(encode_prepare_resp(rid, STEP_REJECT, error=st))
    return out


def leader_prepare_inits(nonces, prep_shares, status) -> List[Optional[bytes]]:
    """PingPong `Initialize{prep_share}` messages the leader sends (aggregation_job_driver.rs:
    362-411); None for reports that failed prepare_init."""
    return [encode_ping_pong(PING_PONG_INITIALIZE, prep_share=bytes(prep_shares[r]))
            if int(status[r]) == 0 else None for r in range(len(status))]
