"""Batched DAP-07 codec edge around the engine, calling the native codec in
libprio3gpu.so (janus_amd/csrc/codec.cpp; C ABI include/prio3gpu.h):

  helper  AggregationJobInitializeReq -> (nonces, public shares, leader prep shares, HPKE
          ciphertexts) -> [HPKE open on CPU] -> PlaintextInputShare -> helper input shares
          -> prio3gpu_helper_init -> AggregationJobResp
  leader  (reports, leader prep shares) -> AggregationJobInitializeReq; AggregationJobResp ->
          prep msgs + per-report status -> prio3gpu_prepare_next

Reference: messages/src/lib.rs (Janus 0.6) encodings; per-report error mapping of the helper loop
aggregator/src/aggregator.rs:1702-1797 and the leader's aggregation_job_driver.rs:530-600.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from ._lib import EmptyAggregation, InvalidMessage, check, lib  # noqa: F401 (re-exported)

TIME_INTERVAL, FIXED_SIZE = 1, 2


class PrepareInitView(ctypes.Structure):
    _fields_ = [("report_id_off", ctypes.c_uint64), ("time", ctypes.c_uint64),
                ("public_share_off", ctypes.c_uint64), ("enc_off", ctypes.c_uint64),
                ("payload_off", ctypes.c_uint64), ("prep_share_off", ctypes.c_uint64),
                ("prep_msg_off", ctypes.c_uint64), ("public_share_len", ctypes.c_uint32),
                ("enc_len", ctypes.c_uint32), ("payload_len", ctypes.c_uint32),
                ("prep_share_len", ctypes.c_uint32), ("prep_msg_len", ctypes.c_uint32),
                ("hpke_config_id", ctypes.c_uint8), ("message_type", ctypes.c_uint8)]


class PrepareRespView(ctypes.Structure):
    _fields_ = [("report_id_off", ctypes.c_uint64), ("prep_share_off", ctypes.c_uint64),
                ("prep_msg_off", ctypes.c_uint64), ("prep_share_len", ctypes.c_uint32),
                ("prep_msg_len", ctypes.c_uint32), ("result", ctypes.c_uint8),
                ("message_type", ctypes.c_uint8), ("error", ctypes.c_uint8)]


def _u8(b) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b


def _p(a):
    return None if a is None else a.ctypes.data


@dataclass
class AggInitReq:
    """A decoded AggregationJobInitializeReq: raw bytes + one view per PrepareInit."""
    raw: np.ndarray
    views: ctypes.Array
    n: int
    agg_param: bytes
    batch_id: Optional[bytes]

    def field(self, i: int, off: str, ln: str) -> bytes:
        v = self.views[i]
        o, l = getattr(v, off), getattr(v, ln)
        return self.raw[o:o + l].tobytes()

    def hpke_ciphertexts(self):
        """(config id, encapsulated key, payload) per report, for the CPU HPKE stage."""
        return [(self.views[i].hpke_config_id, self.field(i, "enc_off", "enc_len"),
                 self.field(i, "payload_off", "payload_len")) for i in range(self.n)]

    def times(self) -> np.ndarray:
        if self.n == 0:
            return np.zeros(0, np.uint64)
        # the views' `time` column read straight from the ctypes array (no per-report loop)
        sz, off = ctypes.sizeof(PrepareInitView), PrepareInitView.time.offset
        rows = np.frombuffer(self.views, dtype=np.uint8)[:self.n * sz].reshape(self.n, sz)
        return np.ascontiguousarray(rows[:, off:off + 8]).view("<u8").reshape(self.n)


def decode_agg_init_req(msg: bytes, query_type: int = TIME_INTERVAL) -> AggInitReq:
    """Decode an AggregationJobInitializeReq (aggregator.rs:1586); Prio3GpuError for a malformed
    request.  The helper then runs `check_agg_init_req`."""
    # no copy of the (up to hundreds of MB) request: bytes give a read-only view, a bytearray or
    # ndarray a writable one that aliases the caller's buffer
    raw = msg if isinstance(msg, np.ndarray) else np.frombuffer(msg, dtype=np.uint8)
    n = ctypes.c_size_t()
    check(lib().prio3gpu_decode_agg_init_req(_p(raw), raw.size, query_type, None, None, None, 0,
                                             ctypes.byref(n)), "decode AggregationJobInitializeReq")
    views = (PrepareInitView * max(1, n.value))()
    bid = np.zeros(32, np.uint8)
    ap = (ctypes.c_uint64 * 2)()
    check(lib().prio3gpu_decode_agg_init_req(_p(raw), raw.size, query_type, _p(bid), ap, views,
                                             n.value, ctypes.byref(n)),
          "decode AggregationJobInitializeReq")
    return AggInitReq(raw, views, n.value, raw[ap[0]:ap[0] + ap[1]].tobytes(),
                      bid.tobytes() if query_type == FIXED_SIZE else None)


def check_agg_init_req(req: AggInitReq) -> None:
    """Helper request-level checks (aggregator.rs:1588-1605): raises `InvalidMessage` when two
    PrepareInits carry the same report ID or the aggregation parameter is not Prio3's empty `()`."""
    check(lib().prio3gpu_check_agg_init_req(_p(req.raw), req.views, req.n, len(req.agg_param)),
          "aggregate-init request")


def gather_prepare_inits(sizes, req: AggInitReq, lps_out: Optional[np.ndarray] = None):
    """(nonces, public shares, leader prep shares, faults) for prio3gpu_helper_init.  `faults[i]`
    is the status report i gets if it survives HPKE open and the plaintext decode (8: public share
    of the wrong length, 5: not Initialize{prep share}); apply it with `apply_faults` after those
    stages, which is Janus's precedence (aggregator.rs:1663-1797).  `lps_out`: optional
    (>= n, prep_share) uint8 buffer (e.g. pinned host memory) for the prep shares."""
    n = req.n
    st = np.zeros(n, np.uint8)
    nonces = np.zeros((n, 16), np.uint8)
    pub = np.zeros((n, sizes.public_share), np.uint8)
    if lps_out is not None:
        assert lps_out.dtype == np.uint8 and lps_out.flags.c_contiguous
        assert lps_out.shape[0] >= n and lps_out.shape[1] == sizes.prep_share
        lps = lps_out[:n]
    else:
        lps = np.zeros((n, sizes.prep_share), np.uint8)
    check(lib().prio3gpu_gather_prepare_inits(ctypes.byref(sizes), _p(req.raw), req.views, n,
                                              _p(nonces), _p(pub), _p(lps), _p(st)), "gather")
    return nonces, pub, lps, st


def apply_faults(status: np.ndarray, faults: np.ndarray) -> np.ndarray:
    """status[i] = faults[i] where status[i] is still 0 (in place; returns status)."""
    assert status.dtype == np.uint8 and faults.dtype == np.uint8 and len(status) == len(faults)
    check(lib().prio3gpu_apply_faults(len(status), _p(faults), _p(status)), "apply faults")
    return status


def decode_plaintext_input_shares(sizes, plaintexts: Sequence[bytes], agg_id: int = 1,
                                  status: Optional[np.ndarray] = None):
    """HPKE-opened PlaintextInputShares -> (n, input share) array + status."""
    n = len(plaintexts)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in plaintexts])
    buf = np.frombuffer(b"".join(plaintexts) or b"\0", np.uint8).copy()
    return decode_plaintext_input_shares_raw(sizes, buf, offs, agg_id, status)


def decode_plaintext_input_shares_raw(sizes, buf: np.ndarray, offs: np.ndarray, agg_id: int = 1,
                                      status: Optional[np.ndarray] = None):
    """As decode_plaintext_input_shares, over one buffer + (n + 1) offsets (the layout
    hpke.open_report_shares produces)."""
    n = len(offs) - 1
    st = np.zeros(n, np.uint8) if status is None else status
    w = sizes.leader_input_share if agg_id == 0 else sizes.helper_input_share
    out = np.zeros((n, w), np.uint8)
    check(lib().prio3gpu_decode_plaintext_input_shares(ctypes.byref(sizes), _p(buf), _p(offs), n,
                                                       agg_id, _p(out), _p(st)),
          "decode PlaintextInputShare")
    return out, st


def encode_agg_job_resp(nonces: np.ndarray, prep_msgs: Optional[np.ndarray], prep_msg_len: int,
                        status: np.ndarray) -> bytes:
    n = len(status)
    ln = ctypes.c_size_t()
    nonces = np.ascontiguousarray(nonces, np.uint8)
    pm = None if prep_msgs is None else np.ascontiguousarray(prep_msgs, np.uint8)
    st = np.ascontiguousarray(status, np.uint8)
    check(lib().prio3gpu_encode_agg_job_resp(_p(nonces), _p(pm), prep_msg_len, _p(st), n, None,
                                             0, ctypes.byref(ln)), "encode AggregationJobResp")
    out = np.zeros(ln.value, np.uint8)
    check(lib().prio3gpu_encode_agg_job_resp(_p(nonces), _p(pm), prep_msg_len, _p(st), n,
                                             _p(out), out.size, ctypes.byref(ln)),
          "encode AggregationJobResp")
    return out.tobytes()


def encode_agg_init_req(query_type: int, batch_id: Optional[bytes], agg_param: bytes,
                        nonces: np.ndarray, times: Sequence[int], public_shares: np.ndarray,
                        ciphertexts: Sequence[tuple], prep_shares: np.ndarray,
                        status: Optional[np.ndarray] = None) -> bytes:
    """Leader: AggregationJobInitializeReq for the reports whose status is 0."""
    n = len(nonces)
    nonces = np.ascontiguousarray(nonces, np.uint8)
    tm = np.ascontiguousarray(times, np.uint64)
    pub = np.ascontiguousarray(public_shares, np.uint8)
    cids = np.array([c[0] for c in ciphertexts], np.uint8)
    encs = [bytes(c[1]) for c in ciphertexts]
    pays = [bytes(c[2]) for c in ciphertexts]
    eo = np.zeros(n + 1, np.uint64)
    eo[1:] = np.cumsum([len(e) for e in encs])
    po = np.zeros(n + 1, np.uint64)
    po[1:] = np.cumsum([len(x) for x in pays])
    eb = np.frombuffer(b"".join(encs) or b"\0", np.uint8).copy()
    pb = np.frombuffer(b"".join(pays) or b"\0", np.uint8).copy()
    ps = np.ascontiguousarray(prep_shares, np.uint8)
    st = None if status is None else np.ascontiguousarray(status, np.uint8)
    ap = np.frombuffer(bytes(agg_param) or b"\0", np.uint8).copy()
    bid = None if batch_id is None else np.frombuffer(bytes(batch_id), np.uint8).copy()
    args = lambda out, cap, ln: (query_type, _p(bid), _p(ap), len(agg_param), n, _p(nonces),
                                 _p(tm), _p(pub), pub.shape[1] if pub.ndim == 2 else 0, _p(cids),
                                 _p(eb), _p(eo), _p(pb), _p(po), _p(ps), ps.shape[1], _p(st), out,
                                 cap, ctypes.byref(ln))
    ln = ctypes.c_size_t()
    check(lib().prio3gpu_encode_agg_init_req(*args(None, 0, ln)), "encode init req")
    out = np.zeros(ln.value, np.uint8)
    check(lib().prio3gpu_encode_agg_init_req(*args(_p(out), out.size, ln)), "encode init req")
    return out.tobytes()


def encode_agg_init_req_packed(query_type: int, batch_id: Optional[bytes], agg_param: bytes,
                               nonces: np.ndarray, times, public_shares: Optional[np.ndarray],
                               hpke_config_ids: np.ndarray, encs: np.ndarray,
                               enc_offsets: np.ndarray, payloads: np.ndarray,
                               payload_offsets: np.ndarray, prep_shares: np.ndarray,
                               status: Optional[np.ndarray] = None) -> bytes:
    """As encode_agg_init_req, with the helper ciphertexts already packed (config ids, one buffer
    of encapsulated keys + (n + 1) offsets, one buffer of payloads + offsets): no per-report
    Python work, for whole aggregation jobs."""
    n = len(nonces)
    nonces = np.ascontiguousarray(nonces, np.uint8)
    tm = np.ascontiguousarray(times, np.uint64)
    pub = None if public_shares is None else np.ascontiguousarray(public_shares, np.uint8)
    pub_len = pub.shape[1] if pub is not None and pub.ndim == 2 else 0
    cids = np.ascontiguousarray(hpke_config_ids, np.uint8)
    eb = np.ascontiguousarray(encs, np.uint8)
    eo = np.ascontiguousarray(enc_offsets, np.uint64)
    pb = np.ascontiguousarray(payloads, np.uint8)
    po = np.ascontiguousarray(payload_offsets, np.uint64)
    ps = np.ascontiguousarray(prep_shares, np.uint8)
    if len(tm) != n or len(cids) != n or len(eo) != n + 1 or len(po) != n + 1 or len(ps) != n:
        raise ValueError("per-report arrays disagree on the report count")
    st = None if status is None else np.ascontiguousarray(status, np.uint8)
    ap = np.frombuffer(bytes(agg_param) or b"\0", np.uint8).copy()
    bid = None if batch_id is None else np.frombuffer(bytes(batch_id), np.uint8).copy()
    args = lambda out, cap, ln: (query_type, _p(bid), _p(ap), len(agg_param), n, _p(nonces),
                                 _p(tm), _p(pub), pub_len, _p(cids), _p(eb), _p(eo), _p(pb),
                                 _p(po), _p(ps), ps.shape[1], _p(st), out, cap, ctypes.byref(ln))
    ln = ctypes.c_size_t()
    check(lib().prio3gpu_encode_agg_init_req(*args(None, 0, ln)), "encode init req")
    out = np.empty(ln.value, np.uint8)
    check(lib().prio3gpu_encode_agg_init_req(*args(_p(out), out.size, ln)), "encode init req")
    return out.tobytes()


def decode_agg_job_resp(msg: bytes):
    raw = _u8(msg).copy()
    n = ctypes.c_size_t()
    check(lib().prio3gpu_decode_agg_job_resp(_p(raw), raw.size, None, 0, ctypes.byref(n)),
          "decode AggregationJobResp")
    views = (PrepareRespView * max(1, n.value))()
    check(lib().prio3gpu_decode_agg_job_resp(_p(raw), raw.size, views, n.value, ctypes.byref(n)),
          "decode AggregationJobResp")
    return raw, views, n.value


def gather_helper_resps(sizes, msg: bytes, nonces: np.ndarray, status: np.ndarray):
    """Leader: helper responses -> (prep msgs, status) for prio3gpu_prepare_next."""
    raw, views, nv = decode_agg_job_resp(msg)
    n = len(status)
    pm = np.zeros((n, sizes.prep_msg), np.uint8)
    nonces = np.ascontiguousarray(nonces, np.uint8)
    check(lib().prio3gpu_gather_helper_resps(ctypes.byref(sizes), _p(raw), views, nv, _p(nonces), n,
                                             _p(pm), _p(status)), "gather helper responses")
    return pm, status
