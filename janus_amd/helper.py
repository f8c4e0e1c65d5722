"""Batched helper aggregate-init driver: the host-side mirror of Janus's
`VdafOps::handle_aggregate_init_generic` (aggregator/src/aggregator.rs:1561-2045) for one task,
minus the datastore transaction (out of scope).

Per aggregation job (one AggregationJobInitializeReq):
  1. decode the request; request-level checks: duplicate report IDs and a non-empty aggregation
     parameter fail the whole request (`InvalidMessage`, aggregator.rs:1588-1605), an empty job
     fails it too (`EmptyAggregation`, aggregator.rs:1851-1863); gather the engine inputs and
     each report's structural faults                                 codec.cpp   (aggregator.rs:1561-1612)
  2. HPKE-open every encrypted input share on host threads            hpke.cpp    (aggregator.rs:1634-1700)
  3. decode the PlaintextInputShares into the input-share array, then apply the structural
     faults to the reports still OK (Janus's precedence: HPKE 3/4, plaintext/input share 8,
     public share 8, ping-pong 5)                                                 (aggregator.rs:1702-1797)
  4. prio3gpu_helper_init: prepare_init + decide + prepare_next + accumulate on the GPU, and
     prio3gpu_agg_update_reports: report-ID checksum + client-timestamp interval per batch
                                                                                  (aggregator.rs:1775-1819,
                                                                                   accumulator.rs:76-122)
  5. encode the AggregationJobResp                                                (aggregator.rs:1811-1848)

`handle_jobs` pipelines a stream of jobs: while the GPU runs job k (step 4, the ctypes call
releases the GIL and blocks on the engine's stream), a host worker thread runs steps 1-3 of job
k + 1 -- the north star's "HPKE open stays on pipelined CPU threads".  Per-report errors keep the
reference's mapping: status 3 HpkeUnknownConfigId, 4 HpkeDecryptError, 5 VdafPrepError,
8 InvalidMessage, each rejecting that report alone.
"""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import codec as C
from . import hpke
from ._lib import EmptyAggregation, Prio3GpuError
from .prio3 import AggregateShares, Prio3Gpu


@dataclass
class _Opened:
    n: int
    nonces: np.ndarray
    public: np.ndarray
    leader_prep: np.ndarray
    helper_in: np.ndarray
    status: np.ndarray
    slots: Optional[np.ndarray]
    times: np.ndarray
    buf: int = -1  # index of the pinned staging buffer holding leader_prep (-1: none)


class _PinnedPool:
    """Pinned host buffers for the leader prep shares of jobs in flight.  A buffer is owned by one
    opened job from `acquire` until `release` (after its GPU stage), so any number of jobs may be
    opened ahead of preparation without one overwriting another's rows."""

    def __init__(self, row_bytes: int):
        self.row_bytes = row_bytes
        self._bufs: List[np.ndarray] = []
        self._keep: List[object] = []
        self._busy: List[bool] = []
        self._lock = threading.Lock()

    def acquire(self, n: int):
        import torch
        if n == 0 or not torch.cuda.is_available():
            return -1, None
        with self._lock:
            for k, b in enumerate(self._bufs):
                if not self._busy[k] and b.shape[0] >= n:
                    self._busy[k] = True
                    return k, b
            t = torch.empty((max(n, 1024), self.row_bytes), dtype=torch.uint8, pin_memory=True)
            self._keep.append(t)
            self._bufs.append(t.numpy())
            self._busy.append(True)
            return len(self._bufs) - 1, self._bufs[-1]

    def release(self, k: int):
        if k < 0:
            return
        with self._lock:
            assert self._busy[k], "staging buffer released twice"
            self._busy[k] = False

    def clear(self):
        with self._lock:
            self._bufs, self._keep, self._busy = [], [], []


class HelperAggregateInit:
    def __init__(self, vdaf: Prio3Gpu, task_id: bytes, task_keys: Sequence[hpke.HpkeKeypair],
                 global_keys: Sequence[hpke.HpkeKeypair] = (), query_type: int = C.TIME_INTERVAL,
                 hpke_threads: int = 0,
                 batch_slot_of: Optional[Callable[[np.ndarray], np.ndarray]] = None):
        """`batch_slot_of(times) -> slots` maps report times to aggregate slots (Janus's
        Q::to_batch_identifier, aggregator.rs:1614-1619); None = one slot."""
        self.vdaf = vdaf
        self.task_id = bytes(task_id)
        self.task_keys = list(task_keys)
        self.global_keys = list(global_keys)
        self.query_type = query_type
        self.hpke_threads = hpke_threads
        self.batch_slot_of = batch_slot_of
        self._state = None
        self._cap = 0
        # pinned staging for the leader prep shares (the largest per-report input, 2,896 B for
        # SumVec): job k+1 is gathered into one buffer while job k's is copied to the GPU from
        # another; pageable memory would make that copy the slowest step.
        self._pinned = _PinnedPool(vdaf.sizes.prep_share)

    def open(self, req_bytes: bytes) -> _Opened:
        """Steps 1-3 (host only).  Raises InvalidMessage / EmptyAggregation for the request."""
        s = self.vdaf.sizes
        req = C.decode_agg_init_req(req_bytes, self.query_type)
        C.check_agg_init_req(req)
        if req.n == 0:
            raise EmptyAggregation("aggregation job contains no reports")
        k, buf = self._pinned.acquire(req.n)
        try:
            nonces, pub, lps, faults = C.gather_prepare_inits(s, req, lps_out=buf)
            pts, offs, st = hpke.open_report_shares(self.task_id, req, self.task_keys,
                                                    self.global_keys, None, self.hpke_threads)
            hin, st = C.decode_plaintext_input_shares_raw(s, pts, offs, 1, st)
            C.apply_faults(st, faults)
            slots = None
            times = req.times()
            if self.batch_slot_of is not None:
                slots = np.ascontiguousarray(self.batch_slot_of(times), np.uint32)
        except BaseException:
            self._pinned.release(k)
            raise
        return _Opened(req.n, nonces, pub, lps, hin, st, slots, times, k)

    def prepare(self, o: _Opened, agg: AggregateShares) -> bytes:
        """Steps 4-5 (GPU + encode)."""
        try:
            if o.n > self._cap:
                if self._state is not None:
                    self._state.close()
                self._cap = max(o.n, 2 * self._cap)
                self._state = self.vdaf.new_state(1, self._cap)
            msgs, st = self.vdaf.helper_init(self._state, o.nonces, o.public, o.helper_in,
                                             o.leader_prep, agg=agg, batch_slots=o.slots,
                                             status=o.status)
        finally:
            self._pinned.release(o.buf)  # helper_init returns after its stream has synchronised
            o.buf = -1
        # Accumulator::update bookkeeping: report-ID checksum + client-timestamp interval
        agg.update_reports(o.nonces, o.times, st, o.slots)
        return C.encode_agg_job_resp(o.nonces, msgs, self.vdaf.sizes.prep_msg, st)

    def handle(self, req_bytes: bytes, agg: AggregateShares) -> bytes:
        return self.prepare(self.open(req_bytes), agg)

    def handle_jobs(self, reqs: Sequence[bytes], agg: AggregateShares) -> List[object]:
        """Pipelined: host decode + HPKE of job k + 1 overlaps the GPU preparation of job k.

        Entry k is job k's AggregationJobResp bytes, or the Prio3GpuError that failed that request
        alone (InvalidMessage: duplicate report IDs or a non-empty aggregation parameter;
        EmptyAggregation): Janus answers such a request with an error and the other jobs carry
        on (aggregator.rs:1588-1605, :1851-1863).  An engine failure while preparing a job ends
        the stream (re-raised), after the staging buffer of the job opened ahead is released."""
        out: List[object] = []
        if not reqs:
            return out
        with ThreadPoolExecutor(max_workers=1) as pool:
            nxt = pool.submit(self.open, reqs[0])
            for k in range(len(reqs)):
                try:
                    cur = nxt.result()
                except Prio3GpuError as e:  # this request alone is rejected
                    cur = e
                if k + 1 < len(reqs):
                    nxt = pool.submit(self.open, reqs[k + 1])
                if isinstance(cur, Prio3GpuError):
                    out.append(cur)
                    continue
                try:
                    out.append(self.prepare(cur, agg))
                except BaseException:
                    if k + 1 < len(reqs):  # drain the job opened ahead and free its buffer
                        try:
                            ahead = nxt.result()
                        except BaseException:
                            ahead = None
                        if isinstance(ahead, _Opened):
                            self._pinned.release(ahead.buf)
                    raise
        return out

    def close(self):
        if self._state is not None:
            self._state.close()
            self._state = None
        self._pinned.clear()
