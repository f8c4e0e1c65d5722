"""Host-side mirror of prio 0.15.1's `prio::vdaf::{Aggregator, Collector}` surface for Prio3,
batched over whole aggregation jobs and executed by the MI355X HIP engine (libprio3gpu.so).

Reference surface:
  * `Prio3::new_count / new_sum / new_sum_vec / new_histogram /
    new_fixedpoint_boundedl2_vec_sum` as constructed by Janus at
    `aggregator/src/aggregator.rs:797-861`; chunk length = floor(sqrt(len)) (`core/src/task.rs:84-86`).
  * `Aggregator::prepare_init`, `prepare_shares_to_prepare_message`, `prepare_next`, `aggregate`
    (fake-VDAF mirror: `core/src/test_util/dummy_vdaf.rs:80-141`).
  * `Aggregatable::merge` (`dummy_vdaf.rs:230-242`), `Collector::unshard` (`collector/src/lib.rs:539`).
  * Per-report errors map to `PrepareError` (`aggregator/src/aggregator/error.rs:240-300`,
    `messages/src/lib.rs:2288-2298`); one bad report never fails the batch.

Inputs are (n, len) uint8 arrays (numpy, host) or torch uint8 tensors on the GPU (device pointers
are used directly, no PCIe copy).  There is no CPU fallback: without the HIP library every call
raises `Prio3GpuError`.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from ._lib import Prio3GpuError, check, lib

COUNT, SUM, SUMVEC, HISTOGRAM, FPVEC = 0, 1, 2, 3, 4
# XOF behind every Prio3 stream (include/prio3gpu.h): XofShake128 = prio 0.15.1 / VDAF-07 (Janus
# 0.6, the default); XofTurboShake128 = draft-irtf-cfrg-vdaf-08+ (forward compatibility, parity
# unpinned)
XOF_SHAKE128, XOF_TURBOSHAKE128 = 0, 1
SLOT_UNUSED = 0xFFFFFFFF  # PRIO3GPU_SLOT_UNUSED (prio3gpu_agg_epoch_merge)
STATUS_OK, STATUS_VDAF_PREP_ERROR, STATUS_INVALID_MESSAGE = 0, 5, 8

FIELD64_MODULUS = 2**64 - 2**32 + 1
FIELD128_MODULUS = 2**128 - 28 * 2**64 + 1


class _Sizes(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "field_size", "meas_len", "proof_len", "verifier_len", "joint_rand_len", "output_len",
        "leader_input_share", "helper_input_share", "public_share", "prep_share", "prep_msg",
        "aggregate_share")]


def chunk_size(measurement_length: int) -> int:
    """Janus `VdafInstance::chunk_size` (core/src/task.rs:84-86): floor(sqrt(len))."""
    return int(math.floor(math.sqrt(measurement_length)))


def vdaf_instance_params(instance):
    """(kind, bits, length, chunk_length) for a Janus VdafInstance in its serde form, as
    `TaskAggregator::new` constructs the VDAF (aggregator/src/aggregator.rs:797-861):
    CountVec = SumVec with bits 1 and chunk_size(length); SumVec chunk_size(bits * length);
    Histogram chunk_size(length); FixedPoint{16,32,64}BitBoundedL2VecSum -> bits 16/32/64.
    Poplar1 and the test-only Fake VDAFs are not Prio3 and are rejected."""
    if isinstance(instance, str):
        name, p = instance, {}
    elif isinstance(instance, dict) and len(instance) == 1:
        (name, p), = instance.items()
        p = p or {}
    else:
        raise ValueError(f"not a VdafInstance: {instance!r}")
    if name == "Prio3Count":
        return COUNT, 0, 0, 0
    if name == "Prio3CountVec":
        return SUMVEC, 1, p["length"], chunk_size(p["length"])
    if name == "Prio3Sum":
        return SUM, p["bits"], 0, 0
    if name == "Prio3SumVec":
        return SUMVEC, p["bits"], p["length"], chunk_size(p["bits"] * p["length"])
    if name == "Prio3Histogram":
        return HISTOGRAM, 0, p["length"], chunk_size(p["length"])
    fp = {"Prio3FixedPoint16BitBoundedL2VecSum": 16, "Prio3FixedPoint32BitBoundedL2VecSum": 32,
          "Prio3FixedPoint64BitBoundedL2VecSum": 64}
    if name in fp:
        return FPVEC, fp[name], p["length"], 0
    raise ValueError(f"VdafInstance {name} is not served by the Prio3 engine")


def _ptr(a) -> Optional[int]:
    """Raw pointer of a numpy array or torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("arrays must be C-contiguous")
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        if not a.is_contiguous():
            raise ValueError("tensors must be contiguous")
        return a.data_ptr()
    raise TypeError(f"unsupported buffer type {type(a)}")


def _pitched_rows(a, n: int, width: int, what: str):
    """(buffer, row pitch) of an (n, width) uint8 view whose rows may sit `pitch` >= width bytes
    apart (a column slice of a wider, e.g. 128-B-aligned, buffer: numpy or torch, host or
    device).  Only a positive pitch >= width that is a multiple of 16 (what
    prio3gpu_state_set_input_pitch accepts) is passed through; any other layout -- broadcast
    (stride 0), negative or unaligned strides, non-contiguous rows -- is packed (pitch = width)."""
    shp = getattr(a, "shape", None)
    if shp is not None and len(shp) == 2 and tuple(shp) == (n, width) and n > 1:
        pitch = None
        if isinstance(a, np.ndarray) and a.dtype == np.uint8 and a.strides[1] == 1:
            pitch = a.strides[0]
        elif hasattr(a, "data_ptr") and getattr(a, "element_size", lambda: 0)() == 1 and \
                a.stride(1) == 1:
            pitch = a.stride(0)
        if pitch is not None and pitch >= width and (pitch == width or pitch % 16 == 0):
            return a, pitch
    return _as_u8(a, n, width, what), width


def _row_ptr(a) -> Optional[int]:
    """Pointer of row 0 of a `_pitched_rows` buffer (rows need only be contiguous inside)."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return _ptr(a)


def _nbytes(a) -> int:
    if isinstance(a, np.ndarray):
        return a.nbytes
    return a.numel() * a.element_size()


def _as_u8(a, n: int, width: int, what: str):
    if a is None:
        return None
    if isinstance(a, (bytes, bytearray)):
        a = np.frombuffer(bytes(a), dtype=np.uint8)
    if isinstance(a, (list, tuple)):
        a = np.frombuffer(b"".join(a), dtype=np.uint8)
    if _nbytes(a) != n * width:
        raise ValueError(f"{what}: expected {n}x{width} bytes, got {_nbytes(a)}")
    if isinstance(a, np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.uint8)
    elif hasattr(a, "is_contiguous") and not a.is_contiguous():
        a = a.contiguous()  # torch: packed rows (the engine reads n * width bytes from row 0)
    return a


class PrepareState:
    """Batch `Prio3PrepareState` for one aggregator (device scratch for up to `capacity`)."""

    def __init__(self, vdaf: "Prio3Gpu", agg_id: int, capacity: int):
        self.vdaf, self.agg_id, self.capacity = vdaf, agg_id, capacity
        h = ctypes.c_void_p()
        check(lib().prio3gpu_state_create(vdaf._ctx, agg_id, capacity, ctypes.byref(h)),
              "state_create")
        self._h = h
        self._keep = None  # keeps device inputs referenced until prepare_next
        self._pitch = 0

    def set_input_pitch(self, pitch: int):
        """Row pitch of the input shares the next calls read (0 = packed; else a multiple of 16
        that is >= the share length): prio3gpu_state_set_input_pitch."""
        if pitch != self._pitch:
            check(lib().prio3gpu_state_set_input_pitch(self._h, pitch), "state_set_input_pitch")
            self._pitch = pitch

    def close(self):
        if getattr(self, "_h", None):
            lib().prio3gpu_state_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class AggregateShares:
    """Per-batch-identifier aggregate shares kept in HBM (`num_slots` batch identifiers)."""

    def __init__(self, vdaf: "Prio3Gpu", num_slots: int = 1):
        self.vdaf, self.num_slots = vdaf, num_slots
        h = ctypes.c_void_p()
        check(lib().prio3gpu_agg_create(vdaf._ctx, num_slots, ctypes.byref(h)), "agg_create")
        self._h = h

    def reset(self):
        check(lib().prio3gpu_agg_reset(self._h), "agg_reset")

    def read(self, slot: int = 0):
        """(aggregate share bytes, report count) for one batch slot."""
        out = np.zeros(self.vdaf.sizes.aggregate_share, dtype=np.uint8)
        cnt = ctypes.c_uint64()
        check(lib().prio3gpu_agg_read(self._h, slot, _ptr(out), ctypes.byref(cnt)), "agg_read")
        return out.tobytes(), cnt.value

    def update_reports(self, report_ids, times, status=None, batch_slots=None):
        """Accumulator::update's bookkeeping (accumulator.rs:76-122): per slot, the report-ID
        checksum (XOR of SHA-256(report id)) and client-timestamp interval of the reports whose
        status is 0.  Arrays may be numpy (host) or torch/device tensors."""
        n = _nbytes(report_ids) // 16
        ids = _as_u8(report_ids, n, 16, "report ids")
        tm = times if not isinstance(times, (list, tuple)) else np.asarray(times, np.uint64)
        if isinstance(tm, np.ndarray):
            tm = np.ascontiguousarray(tm, dtype=np.uint64)
        st = status
        if isinstance(st, np.ndarray):
            st = np.ascontiguousarray(st, dtype=np.uint8)
        sl = batch_slots
        if isinstance(sl, np.ndarray):
            sl = np.ascontiguousarray(sl, dtype=np.uint32)
        check(lib().prio3gpu_agg_update_reports(self._h, n, _ptr(ids), _ptr(tm), _ptr(st),
                                                _ptr(sl)), "agg_update_reports")

    def read_reports(self, slot: int = 0):
        """(ReportIdChecksum bytes, (interval start, duration)) for one batch slot."""
        ck = np.zeros(32, np.uint8)
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().prio3gpu_agg_read_reports(self._h, slot, _ptr(ck), ctypes.byref(a),
                                              ctypes.byref(b)), "agg_read_reports")
        return ck.tobytes(), (a.value, b.value)

    def merge(self, slot: int, share: bytes, count: int):
        """`Aggregatable::merge` with an encoded aggregate share."""
        buf = np.frombuffer(bytes(share), dtype=np.uint8).copy()
        check(lib().prio3gpu_agg_merge_bytes(self._h, slot, _ptr(buf), count), "agg_merge")

    def close(self):
        if getattr(self, "_h", None):
            lib().prio3gpu_agg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Prio3Gpu:
    """Prio3 with NUM_SHARES = 2 bound to one verify key (one Janus task) and one GPU."""

    def __init__(self, kind: int, verify_key: bytes, bits: int = 0, length: int = 0,
                 chunk_length: int = 0, device: int = 0, xof: int = XOF_SHAKE128):
        if len(verify_key) != 16:
            raise ValueError("verify key must be 16 bytes")
        self.kind, self.bits, self.length, self.chunk_length = kind, bits, length, chunk_length
        self.verify_key = bytes(verify_key)
        self.device = device
        self.xof = xof
        h = ctypes.c_void_p()
        check(lib().prio3gpu_ctx_create2(kind, bits, length, chunk_length, self.verify_key, device,
                                         xof, ctypes.byref(h)), "ctx_create")
        self._ctx = h
        s = _Sizes()
        check(lib().prio3gpu_ctx_sizes(self._ctx, ctypes.byref(s)), "ctx_sizes")
        self.sizes = s
        self.modulus = FIELD64_MODULUS if s.field_size == 8 else FIELD128_MODULUS

    # -- constructors mirroring prio (Janus passes num_aggregators = 2) -------------------------
    @classmethod
    def from_vdaf_instance(cls, instance, verify_key, device=0):
        """`TaskAggregator::new`'s VdafInstance -> VDAF mapping (aggregator.rs:797-861).
        `instance` is Janus's serde form: "Prio3Count" or {"Prio3SumVec": {"bits": 8,
        "length": 1000}} (core/src/task.rs:24-59)."""
        kind, bits, length, chunk = vdaf_instance_params(instance)
        return cls(kind, verify_key, bits=bits, length=length, chunk_length=chunk, device=device)

    @classmethod
    def new_count(cls, verify_key, device=0):
        return cls(COUNT, verify_key, device=device)

    @classmethod
    def new_sum(cls, bits, verify_key, device=0):
        return cls(SUM, verify_key, bits=bits, device=device)

    @classmethod
    def new_sum_vec(cls, bits, length, chunk_length, verify_key, device=0):
        return cls(SUMVEC, verify_key, bits=bits, length=length, chunk_length=chunk_length,
                   device=device)

    @classmethod
    def new_count_vec(cls, length, chunk_length, verify_key, device=0):
        """Janus `Prio3CountVec` = SumVec with bits = 1 (aggregator.rs:805-813)."""
        return cls.new_sum_vec(1, length, chunk_length, verify_key, device)

    @classmethod
    def new_histogram(cls, length, chunk_length, verify_key, device=0):
        return cls(HISTOGRAM, verify_key, length=length, chunk_length=chunk_length, device=device)

    @classmethod
    def new_fixedpoint_boundedl2_vec_sum(cls, bits, length, verify_key, device=0):
        """Janus `Prio3FixedPoint{16,32,64}BitBoundedL2VecSum { length }` (aggregator.rs:839-861):
        `Prio3::new_fixedpoint_boundedl2_vec_sum_multithreaded(2, length)` over FixedI{bits}."""
        return cls(FPVEC, verify_key, bits=bits, length=length, device=device)

    def close(self):
        if getattr(self, "_ctx", None):
            lib().prio3gpu_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self) -> int:
        return lib().prio3gpu_ctx_stream(self._ctx) or 0

    def sync(self):
        check(lib().prio3gpu_ctx_sync(self._ctx), "sync")

    def set_option(self, name: str, value: int):
        """Engine option of this context (prio3gpu_ctx_set_option: "speculate", "wires_mfma",
        "wires_cols", "fused_helper", "helper_snap", "snap_chunk", "jr_ring", "spread",
        "expand_lds", "jr_lds", "exact_squeeze")."""
        check(lib().prio3gpu_ctx_set_option(self._ctx, name.encode(), int(value)),
              f"ctx_set_option({name})")

    # -- asynchronous use (include/prio3gpu.h: prio3gpu_ctx_set_async / _wait / _mark) -----------
    def set_async(self, on: bool = True):
        """Calls over device buffers return once queued (host buffers still wait)."""
        check(lib().prio3gpu_ctx_set_async(self._ctx, int(bool(on))), "ctx_set_async")

    def wait_for(self, other: "Prio3Gpu", mark: Optional[int] = None):
        """Work queued here from now on starts after `other`'s work queued so far (or up to
        `mark`, from other.mark())."""
        if mark is None:
            check(lib().prio3gpu_ctx_wait(self._ctx, other._ctx), "ctx_wait")
        else:
            check(lib().prio3gpu_ctx_wait_mark(self._ctx, other._ctx, mark), "ctx_wait_mark")

    def mark(self) -> int:
        m = ctypes.c_int()
        check(lib().prio3gpu_ctx_mark(self._ctx, ctypes.byref(m)), "ctx_mark")
        return m.value

    def prepare_init_xof(self, state: PrepareState, nonces, public_shares, input_shares, status):
        """prepare_init's XOF phase (query + joint randomness, helper expansion); `status` (n,)
        uint8, host or device; inputs must stay valid until prepare_init_query."""
        n = _nbytes(status)
        s = self.sizes
        in_len = s.leader_input_share if state.agg_id == 0 else s.helper_input_share
        input_shares, pitch = _pitched_rows(input_shares, n, in_len, "input shares")
        state.set_input_pitch(0 if pitch == in_len else pitch)
        check(lib().prio3gpu_prepare_init_xof(self._ctx, state._h, n, _ptr(nonces),
                                              _ptr(public_shares), _row_ptr(input_shares),
                                              _ptr(status)), "prepare_init_xof")
        state._keep = input_shares

    def prepare_init_query(self, state: PrepareState, out_prep_shares, status):
        """prepare_init's FLP-query phase -> prep shares into `out_prep_shares` (n, prep_share)."""
        n = _nbytes(status)
        check(lib().prio3gpu_prepare_init_query(self._ctx, state._h, n, _ptr(out_prep_shares),
                                                _ptr(status)), "prepare_init_query")

    def prepare_init_weights(self, state: PrepareState, status):
        """Optional step between the XOF and query phases: the first (latency-bound) half of a
        ParallelSum FLP query (k_flp_weights); a no-op for the other types."""
        n = _nbytes(status)
        check(lib().prio3gpu_prepare_init_weights(self._ctx, state._h, n, _ptr(status)),
              "prepare_init_weights")

    def new_state(self, agg_id: int, capacity: int) -> PrepareState:
        return PrepareState(self, agg_id, capacity)

    def new_aggregate(self, num_slots: int = 1) -> AggregateShares:
        return AggregateShares(self, num_slots)

    # -- Aggregator --------------------------------------------------------------------------------
    def prepare_init(self, state: PrepareState, nonces, public_shares, input_shares,
                     status=None, want_prep_shares: bool = True, out_prep_shares=None):
        """Batched `prepare_init` -> (prep_shares (n, prep_share) uint8, status (n,) uint8).
        `out_prep_shares`: optional (>= n, prep_share) uint8 destination (e.g. pinned host
        memory, so the device -> host copy is DMA)."""
        s = self.sizes
        n = _nbytes(nonces) // 16
        in_len = s.leader_input_share if state.agg_id == 0 else s.helper_input_share
        nonces = _as_u8(nonces, n, 16, "nonces")
        public_shares = _as_u8(public_shares, n, s.public_share, "public shares") \
            if s.public_share else None
        input_shares, pitch = _pitched_rows(input_shares, n, in_len, "input shares")
        state.set_input_pitch(0 if pitch == in_len else pitch)
        st = np.zeros(n, dtype=np.uint8) if status is None else status
        if out_prep_shares is not None:
            prep = out_prep_shares[:n]
            if prep.shape != (n, s.prep_share) or prep.dtype != np.uint8 or \
                    not prep.flags.c_contiguous:
                raise ValueError("out_prep_shares must be a contiguous (n, prep_share) uint8 array")
        else:
            prep = np.zeros((n, s.prep_share), dtype=np.uint8) if want_prep_shares else None
        check(lib().prio3gpu_prepare_init(self._ctx, state._h, n, _ptr(nonces),
                                          _ptr(public_shares), _row_ptr(input_shares), _ptr(prep),
                                          _ptr(st)), "prepare_init")
        state._keep = input_shares
        return prep, st

    def prepare_shares_to_prepare_message(self, leader_prep_shares, helper_prep_shares,
                                          status=None):
        s = self.sizes
        n = _nbytes(leader_prep_shares) // s.prep_share
        lp = _as_u8(leader_prep_shares, n, s.prep_share, "leader prep shares")
        hp = _as_u8(helper_prep_shares, n, s.prep_share, "helper prep shares")
        st = np.zeros(n, dtype=np.uint8) if status is None else status
        msgs = np.zeros((n, max(1, s.prep_msg)), dtype=np.uint8)[:, :s.prep_msg].copy()
        check(lib().prio3gpu_prepare_shares_to_prepare_message(
            self._ctx, n, _ptr(lp), _ptr(hp), _ptr(msgs) if s.prep_msg else None, _ptr(st)),
            "prepare_shares_to_prepare_message")
        return msgs, st

    def prepare_next(self, state: PrepareState, prep_msgs, status, want_output_shares=True,
                     agg: Optional[AggregateShares] = None, batch_slots=None):
        s = self.sizes
        n = _nbytes(status)
        msgs = _as_u8(prep_msgs, n, s.prep_msg, "prep msgs") if s.prep_msg else None
        outs = np.zeros((n, s.aggregate_share), dtype=np.uint8) if want_output_shares else None
        slots = None
        if batch_slots is not None:
            slots = batch_slots if not isinstance(batch_slots, np.ndarray) else \
                np.ascontiguousarray(batch_slots, dtype=np.uint32)
        check(lib().prio3gpu_prepare_next(self._ctx, state._h, n, _ptr(msgs), _ptr(status),
                                          _ptr(outs), _ptr(slots), agg._h if agg else None),
              "prepare_next")
        return outs, status

    def helper_init(self, state: PrepareState, nonces, public_shares, helper_input_shares,
                    leader_prep_shares, agg: Optional[AggregateShares] = None, batch_slots=None,
                    status=None, out_prep_msgs=None):
        """Helper aggregate-init for a whole job (aggregator.rs:1613-1848): returns
        (prep_msgs, status); output shares are accumulated into `agg`."""
        s = self.sizes
        n = _nbytes(nonces) // 16
        nonces = _as_u8(nonces, n, 16, "nonces")
        pub = _as_u8(public_shares, n, s.public_share, "public shares") if s.public_share else None
        hs, pitch = _pitched_rows(helper_input_shares, n, s.helper_input_share,
                                  "helper input shares")
        state.set_input_pitch(0 if pitch == s.helper_input_share else pitch)
        lp = _as_u8(leader_prep_shares, n, s.prep_share, "leader prep shares")
        st = np.zeros(n, dtype=np.uint8) if status is None else status
        msgs = out_prep_msgs
        if msgs is None and s.prep_msg:
            msgs = np.zeros((n, s.prep_msg), dtype=np.uint8)
        slots = None
        if batch_slots is not None:
            slots = batch_slots if not isinstance(batch_slots, np.ndarray) else \
                np.ascontiguousarray(batch_slots, dtype=np.uint32)
        check(lib().prio3gpu_helper_init(self._ctx, state._h, n, _ptr(nonces), _ptr(pub),
                                         _row_ptr(hs), _ptr(lp), _ptr(slots), _ptr(msgs), _ptr(st),
                                         agg._h if agg else None), "helper_init")
        return msgs, st

    # -- Client ------------------------------------------------------------------------------------
    def random_size(self) -> int:
        return lib().prio3gpu_random_size(self._ctx)

    def shard(self, state: PrepareState, nonces, measurements, rand, out=None):
        """Batched `Client::shard` (prio shard_with_random) on the GPU -> (public shares, leader
        input shares, helper input shares).  `measurements`: (n,) or (n, length) uint64; for
        FixedPointBoundedL2VecSum the (n, length) raw two's-complement fixed-point integers
        (int64 accepted), whose L2 norm must be < 1 as prio's shard requires."""
        s = self.sizes
        n = _nbytes(nonces) // 16
        nonces = _as_u8(nonces, n, 16, "nonces")
        rand = _as_u8(rand, n, self.random_size(), "rand")
        if isinstance(measurements, np.ndarray):
            if measurements.dtype == np.int64:
                measurements = np.ascontiguousarray(measurements).view(np.uint64)
            measurements = np.ascontiguousarray(measurements, dtype=np.uint64)
        if out is None:
            out = (np.zeros((n, s.public_share), np.uint8) if s.public_share else None,
                   np.zeros((n, s.leader_input_share), np.uint8),
                   np.zeros((n, s.helper_input_share), np.uint8))
        pub, lead, helper = out
        check(lib().prio3gpu_shard(self._ctx, state._h, n, _ptr(nonces), _ptr(measurements),
                                   _ptr(rand), _ptr(pub), _ptr(lead), _ptr(helper)), "shard")
        return pub, lead, helper

    # -- Collector ---------------------------------------------------------------------------------
    def decode_field_vec(self, b: bytes):
        es = self.sizes.field_size
        return [int.from_bytes(b[i:i + es], "little") for i in range(0, len(b), es)]

    def unshard(self, aggregate_shares: Sequence[bytes], num_measurements: int = None):
        """`Collector::unshard` (collector/src/lib.rs:539) via prio3gpu_unshard: sum the aggregate
        shares mod p and decode the result (integers; fixed-point vectors decode each sum d of
        `num_measurements` encoded entries as d * 2^(1-bits) - num_measurements)."""
        s = self.sizes
        shares = b"".join(bytes(a) for a in aggregate_shares)
        if len(shares) != len(aggregate_shares) * s.aggregate_share or not aggregate_shares:
            raise ValueError("aggregate shares must be aggregate_share bytes each")
        buf = np.frombuffer(shares, np.uint8).copy()
        if self.kind == FPVEC:
            if num_measurements is None:
                raise ValueError("fixed-point unshard needs the report count")
            out = np.zeros(s.output_len, np.float64)
            check(lib().prio3gpu_unshard(self._ctx, _ptr(buf), len(aggregate_shares),
                                         num_measurements, None, _ptr(out)), "unshard")
            return [float(x) for x in out]
        out = np.zeros((s.output_len, 16), np.uint8)
        check(lib().prio3gpu_unshard(self._ctx, _ptr(buf), len(aggregate_shares),
                                     num_measurements or 0, _ptr(out), None), "unshard")
        vals = [int.from_bytes(out[e].tobytes(), "little") for e in range(s.output_len)]
        if self.kind in (COUNT, SUM):
            return vals[0]
        return vals


class Comm:
    """RCCL communicator for the per-GPU partial-aggregate merge (one process per GPU)."""

    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int):
        h = ctypes.c_void_p()
        buf = np.frombuffer(bytes(unique_id), dtype=np.uint8).copy()
        check(lib().prio3gpu_comm_init(_ptr(buf), nranks, rank, device, ctypes.byref(h)),
              "comm_init")
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        buf = np.zeros(128, dtype=np.uint8)
        check(lib().prio3gpu_comm_unique_id(_ptr(buf)), "comm_unique_id")
        return buf.tobytes()

    def allreduce(self, vdaf: Prio3Gpu, local: AggregateShares,
                  total: Optional[AggregateShares] = None):
        """total += sum over ranks of `local` (then `local` is reset); without `total`, `local`
        becomes the sum over ranks."""
        check(lib().prio3gpu_agg_allreduce(self._h, vdaf._ctx, local._h,
                                           total._h if total is not None else None),
              "agg_allreduce")

    def epoch_merge(self, vdaf: Prio3Gpu, local: AggregateShares, slot_map,
                    total: AggregateShares):
        """prio3gpu_agg_epoch_merge: total[slot_map[s]] += sum over ranks of local[s] (one entry
        per local slot; SLOT_UNUSED for a slot the epoch's jobs did not use), local reset.  A
        collective: every rank, once per epoch, epochs in the same order."""
        m = np.ascontiguousarray(slot_map, dtype=np.uint32)
        if m.shape != (local.num_slots,):
            raise ValueError(f"slot_map needs {local.num_slots} entries, got {m.shape}")
        check(lib().prio3gpu_agg_epoch_merge(self._h, vdaf._ctx, local._h, _ptr(m),
                                             total.num_slots, total._h), "agg_epoch_merge")

    def close(self):
        if getattr(self, "_h", None):
            lib().prio3gpu_comm_destroy(self._h)
            self._h = None
