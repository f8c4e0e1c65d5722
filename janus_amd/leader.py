"""Batched leader aggregate-init driver: the host-side mirror of Janus's
`AggregationJobDriver::step_aggregation_job_aggregate_init` + `process_response_from_helper`
(aggregator/src/aggregator/aggregation_job_driver.rs:290-437, :530-727) for one task, minus the
datastore transactions and the HTTP client (out of scope): the helper round trip is
a caller-supplied `send(request_bytes) -> response_bytes`.

Per aggregation job (the job's `LeaderStoredReport`s, models.rs:78, already decoded from the
datastore as in aggregator_core/src/datastore.rs:1298-1304):
  1. per-report pre-checks: a missing client report -> ReportDropped (2) (:330-342), repeated
     leader extensions -> InvalidMessage (8) (:344-359)
  2. prio3gpu_prepare_init(agg_id 0) on the GPU (`leader_initialized`, :362-380); reports it
     rejects -> VdafPrepError (5) / InvalidMessage (8), never sent
  3. AggregationJobInitializeReq of the surviving reports: ReportShare (metadata, public share,
     the helper's encrypted input share) + PingPongMessage::Initialize{prep share} (:382-411)
  4. send to the helper
  5. AggregationJobResp: the response must answer exactly the sent reports, in order, else the
     whole job fails (:556-573); Continue{Finish{prep msg}} -> prio3gpu_prepare_next
     (`leader_continued` -> FinishedNoMessage) + accumulate (:575-627); Finished while the
     leader is not finished -> VdafPrepError (:632-664); Reject(e) -> e (:666-677)
  6. Accumulator::update bookkeeping: report-ID checksum + client-timestamp interval per batch
     slot (accumulator.rs:76-122)

`run_jobs` pipelines a stream of jobs the way Janus runs aggregation jobs concurrently
(job_driver.rs:119-216): the host -> GPU copy of job k+1's leader input shares (the dominant
input, 134,944 B per SumVec(8,1000) report; pinned host memory, its own copy stream) overlaps
the GPU preparation of job k, and the helper round trip of job k overlaps the GPU work of job
k+1.  Returns per-report final statuses (0 = Finished).
"""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import codec as C
from ._lib import EmptyAggregation, Prio3GpuError
from .prio3 import AggregateShares, PrepareState, Prio3Gpu

REPORT_DROPPED, VDAF_PREP_ERROR, INVALID_MESSAGE = 2, 5, 8


@dataclass
class LeaderJob:
    """One aggregation job's reports, columnar (report i = row i)."""
    nonces: np.ndarray               # (n, 16) report IDs (the VDAF nonces)
    times: np.ndarray                # (n,) u64 client timestamps
    public: np.ndarray               # (n, public_share) encoded public shares
    leader_in: object                # (n, leader_input_share) uint8: numpy (pinned: see
                                     # LeaderAggregateInit.pinned) or a torch tensor on the GPU
    hpke_config_ids: np.ndarray      # (n,) helper ciphertext config ids
    encs: np.ndarray                 # concatenated encapsulated keys
    enc_offsets: np.ndarray          # (n + 1,) u64
    payloads: np.ndarray             # concatenated helper ciphertext payloads
    payload_offsets: np.ndarray      # (n + 1,) u64
    present: Optional[np.ndarray] = None         # (n,) bool; False: report garbage-collected
    dup_extensions: Optional[np.ndarray] = None  # (n,) bool; True: repeated leader extension

    @property
    def n(self) -> int:
        return len(self.nonces)

    @staticmethod
    def pack_ciphertexts(cts: Sequence[tuple]):
        """[(config id, enc, payload)] -> (ids, encs, enc_offsets, payloads, payload_offsets)."""
        n = len(cts)
        ids = np.array([c[0] for c in cts], np.uint8)
        eo = np.zeros(n + 1, np.uint64)
        eo[1:] = np.cumsum([len(c[1]) for c in cts])
        po = np.zeros(n + 1, np.uint64)
        po[1:] = np.cumsum([len(c[2]) for c in cts])
        eb = np.frombuffer(b"".join(bytes(c[1]) for c in cts) or b"\0", np.uint8).copy()
        pb = np.frombuffer(b"".join(bytes(c[2]) for c in cts) or b"\0", np.uint8).copy()
        return ids, eb, eo, pb, po


@dataclass
class LeaderStepped:
    """A job between its request and the helper's response (Janus: SteppedAggregation list)."""
    job: LeaderJob
    state: PrepareState
    status: np.ndarray
    request: bytes
    d_in: object = None              # device copy of the leader input shares (kept alive)
    slots: Optional[np.ndarray] = None
    times_ms: dict = field(default_factory=dict)
    prep: object = None              # prep shares between prepare and encode (pinned buffer view)
    pbuf: object = None


class LeaderAggregateInit:
    def __init__(self, vdaf: Prio3Gpu, query_type: int = C.TIME_INTERVAL,
                 batch_id: Optional[bytes] = None,
                 batch_slot_of: Optional[Callable[[np.ndarray], np.ndarray]] = None):
        """`batch_slot_of(times) -> slots` maps report times to aggregate slots (Janus's
        partial batch identifier per report); None = one slot."""
        if query_type == C.FIXED_SIZE and batch_id is None:
            raise ValueError("fixed-size aggregation jobs carry a batch id")
        self.vdaf = vdaf
        self.query_type = query_type
        self.batch_id = batch_id
        self.batch_slot_of = batch_slot_of
        self._copy_stream = None
        self._lock = threading.Lock()
        self._prep_bufs: List[np.ndarray] = []  # pinned prep-share buffers, one per job in flight
        # prepare states of the jobs in flight, reused: creating / destroying one allocates /
        # frees device memory, and hipFree waits for the whole device (the next job's H2D copy)
        self._states: List[PrepareState] = []

    # -- host staging --------------------------------------------------------------------------------
    @staticmethod
    def pinned(n: int, width: int) -> np.ndarray:
        """A pinned (page-locked) (n, width) uint8 host array, for decoding leader input shares
        into so that the host -> GPU copy is DMA."""
        import torch
        # the ndarray's base keeps the tensor (and its pinned allocation) alive
        return torch.empty((n, width), dtype=torch.uint8, pin_memory=True).numpy()

    def stage(self, job: LeaderJob):
        """Copy the job's leader input shares to the GPU on the driver's copy stream (blocking
        this thread only); a torch CUDA tensor is used as is."""
        import torch
        li = job.leader_in
        if isinstance(li, torch.Tensor) and li.is_cuda:
            return li
        with self._lock:
            if self._copy_stream is None:
                self._copy_stream = torch.cuda.Stream(device=self.vdaf.device)
        s = self._copy_stream
        src = torch.from_numpy(np.ascontiguousarray(li))
        with torch.cuda.stream(s):
            d = torch.empty(src.shape, dtype=torch.uint8, device=f"cuda:{self.vdaf.device}")
            d.copy_(src, non_blocking=True)
        s.synchronize()
        return d

    def _state(self, n: int) -> PrepareState:
        with self._lock:
            for k, st in enumerate(self._states):
                if st.capacity >= n:
                    return self._states.pop(k)
        return self.vdaf.new_state(0, n)

    def _release(self, st: PrepareState):
        with self._lock:
            self._states.append(st)

    def close(self):
        with self._lock:
            for st in self._states:
                st.close()
            self._states = []
            self._prep_bufs = []

    def _return_prep_buf(self, b):
        if b is not None:
            with self._lock:
                self._prep_bufs.append(b)

    def _prep_buf(self, n: int) -> np.ndarray:
        """A pinned (>= n, prep_share) buffer for prepare_init's output (the device -> host copy
        of 2,896 B per SumVec report is then DMA); buffers are reused once the request that
        copied them out has been encoded."""
        w = self.vdaf.sizes.prep_share
        with self._lock:
            for k, b in enumerate(self._prep_bufs):
                if b.shape[0] >= n:
                    return self._prep_bufs.pop(k)
        try:
            return self.pinned(max(n, 1024), w)
        except RuntimeError:  # no GPU runtime for pinning: pageable memory
            return np.zeros((max(n, 1024), w), np.uint8)

    # -- steps ---------------------------------------------------------------------------------------
    def init(self, job: LeaderJob, d_in=None) -> LeaderStepped:
        """Steps 1-3: pre-checks, GPU prepare_init, request bytes."""
        st = self.prepare(job, d_in)
        try:
            self.encode(st)
        except BaseException:
            self._release(st.state)
            raise
        return st

    def prepare(self, job: LeaderJob, d_in=None) -> LeaderStepped:
        """Steps 1-2: pre-checks and GPU prepare_init; the prep shares wait in a pinned buffer
        for `encode` (which may run on another thread while the GPU takes the next job)."""
        import time
        n = job.n
        if n == 0:
            raise EmptyAggregation("aggregation job contains no reports")
        s = self.vdaf.sizes
        t0 = time.perf_counter()
        status = np.zeros(n, np.uint8)
        if job.present is not None:
            status[~np.asarray(job.present, bool)] = REPORT_DROPPED
        if job.dup_extensions is not None:
            status[(status == 0) & np.asarray(job.dup_extensions, bool)] = INVALID_MESSAGE
        if d_in is None:
            d_in = self.stage(job)
        t1 = time.perf_counter()
        state = self._state(n)
        pbuf = self._prep_buf(n)
        try:
            prep, status = self.vdaf.prepare_init(state, job.nonces,
                                                  job.public if s.public_share else None, d_in,
                                                  status=status, out_prep_shares=pbuf)
        except BaseException:
            self._release(state)
            self._return_prep_buf(pbuf)
            raise
        t2 = time.perf_counter()
        slots = None
        if self.batch_slot_of is not None:
            slots = np.ascontiguousarray(self.batch_slot_of(np.asarray(job.times)), np.uint32)
        st = LeaderStepped(job, state, status, b"", d_in, slots,
                           {"stage": (t1 - t0) * 1e3, "prepare_init": (t2 - t1) * 1e3})
        st.prep = prep
        st.pbuf = pbuf
        return st

    def encode(self, st: LeaderStepped) -> bytes:
        """Step 3: the AggregationJobInitializeReq of a prepared job (its prep-share buffer is
        returned to the pool: the shares live on in the request bytes)."""
        import time
        t0 = time.perf_counter()
        job = st.job
        try:
            st.request = C.encode_agg_init_req_packed(
                self.query_type, self.batch_id, b"", job.nonces, job.times, job.public,
                job.hpke_config_ids, job.encs, job.enc_offsets, job.payloads, job.payload_offsets,
                st.prep, st.status)
        finally:
            self._return_prep_buf(st.pbuf)
            st.prep = st.pbuf = None
        st.times_ms["encode"] = (time.perf_counter() - t0) * 1e3
        return st.request

    def finish(self, st: LeaderStepped, resp: bytes, agg: AggregateShares) -> np.ndarray:
        """Steps 5-6.  Raises Prio3GpuError when the response does not answer exactly the sent
        reports in order (the whole job fails, aggregation_job_driver.rs:556-573)."""
        import time
        t0 = time.perf_counter()
        try:
            pm, status = C.gather_helper_resps(self.vdaf.sizes, resp, st.job.nonces,
                                               st.status.copy())
            t1 = time.perf_counter()
            self.vdaf.prepare_next(st.state, pm, status, want_output_shares=False, agg=agg,
                                   batch_slots=st.slots)
            agg.update_reports(st.job.nonces, st.job.times, status, st.slots)
            t2 = time.perf_counter()
        finally:
            self._release(st.state)
            st.d_in = None
        st.times_ms.update({"decode": (t1 - t0) * 1e3, "prepare_next": (t2 - t1) * 1e3})
        return status

    def handle(self, job: LeaderJob, send: Callable[[bytes], bytes],
               agg: AggregateShares) -> np.ndarray:
        st = self.init(job)
        return self.finish(st, send(st.request), agg)

    def run_jobs(self, jobs: Sequence[LeaderJob], send: Callable[[bytes], bytes],
                 agg: AggregateShares, stats: Optional[list] = None,
                 stage_ahead: int = 2) -> List[object]:
        """Pipelined over jobs: the H2D copies of the next `stage_ahead` jobs queue on the copy
        stream behind the current one (the copy engine never waits for the driver thread), GPU
        prepare_init of job k runs while job k-1's request is encoded and sent on the network
        worker, and job k-1's response is finished after job k is queued.  `stats`, if given,
        receives each job's stage times.

        Entry k is job k's per-report final statuses, or the exception that failed job k alone:
        an empty job (EmptyAggregation), a response that does not answer the sent reports
        (Prio3GpuError, aggregation_job_driver.rs:556-573), a failed helper round trip.  Janus
        steps each aggregation job on its own (job_driver.rs:119-216), so a failing job never
        strands the one in flight: the request already sent for job k-1 is still finished, so
        the leader's aggregate keeps the reports the helper has accumulated."""
        out: List[object] = [None] * len(jobs)
        if not jobs:
            return out
        ahead = max(1, stage_ahead)
        with ThreadPoolExecutor(max_workers=1) as h2d, ThreadPoolExecutor(max_workers=1) as net:
            staged = [h2d.submit(self.stage, jobs[i]) for i in range(min(ahead, len(jobs)))]
            inflight = None  # (job index, LeaderStepped, response future)

            def encode_send(st):
                return send(self.encode(st))

            def finish_inflight():
                k0, st0, fut0 = inflight
                try:
                    resp = fut0.result()
                except Exception as e:  # encoding or the helper round trip failed: this job alone
                    self._release(st0.state)
                    self._return_prep_buf(st0.pbuf)
                    st0.d_in = None
                    out[k0] = e
                    return
                try:
                    out[k0] = self.finish(st0, resp, agg)
                except Prio3GpuError as e:
                    out[k0] = e
                if stats is not None:
                    stats.append(st0.times_ms)

            try:
                for k in range(len(jobs)):
                    try:
                        d_in = staged.pop(0).result()
                    except Exception as e:
                        d_in = e
                    if k + ahead < len(jobs):
                        staged.append(h2d.submit(self.stage, jobs[k + ahead]))
                    started = None
                    if isinstance(d_in, Exception):
                        out[k] = d_in
                    else:
                        try:
                            st = self.prepare(jobs[k], d_in)
                            started = (k, st, net.submit(encode_send, st))
                        except Prio3GpuError as e:  # EmptyAggregation, a rejected batch
                            out[k] = e
                    if inflight is not None:
                        finish_inflight()
                    inflight = started
            finally:
                if inflight is not None:  # also on abort: never leave a sent job unfinished
                    finish_inflight()
        return out
