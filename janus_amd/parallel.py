"""Report sharding across GPUs: one process per GPU, contiguous report ranges,
no data-path collective; the only exchange is the merge of per-GPU partial aggregate shares (RCCL
all-gather of raw LE field-element bytes + mod-p add kernel) with the checksum / interval half of
`BatchAggregation::merged_with`.

Two merge contracts:
  * per job, `Comm.allreduce` (prio3gpu_agg_allreduce): every rank flushes every job in lockstep
    (the bench's step, one job per rank per step);
  * per epoch, `EpochPartials` (host) / `epoch_merge_device` (prio3gpu_agg_epoch_merge): each
    rank keeps its partials across ANY number of independent jobs, keyed by batch identifier, and
    the ranks merge once at an epoch boundary (a collection), every rank calling the merge for
    epochs in the same order -- the shape Janus's independent job drivers can run
    (binary_utils/job_driver.rs:119-216) and the shard merge of aggregate_share.rs:44-66.

Janus analogue: independent aggregation jobs on concurrent job-driver workers
(`aggregator/src/binary_utils/job_driver.rs:119-216`) whose partial batch aggregations are merged
(`aggregator_core/src/datastore/models.rs:962-991`, `aggregate_share.rs:47-65`).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Iterable, Tuple

from ._lib import check, lib


def world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n: int, world_size: int, rank: int):
    """GPU `rank` takes reports [rank*n/G, (rank+1)*n/G)."""
    return (n * rank) // world_size, (n * (rank + 1)) // world_size


class _BA(ctypes.Structure):
    _fields_ = [("aggregate_share", ctypes.c_void_p), ("report_count", ctypes.c_uint64),
                ("checksum", ctypes.c_uint8 * 32), ("interval_start", ctypes.c_uint64),
                ("interval_duration", ctypes.c_uint64)]


@dataclass
class BatchAggregation:
    """One batch identifier's aggregation (Janus `BatchAggregation`, models.rs:843-991):
    encoded aggregate share, report count, ReportIdChecksum, client-timestamp interval."""
    aggregate_share: bytes
    report_count: int
    checksum: bytes = bytes(32)
    interval: Tuple[int, int] = (0, 0)  # (start, duration); duration 0 = Interval::EMPTY


def merge_batch_aggregations(field_size: int, parts: Iterable[BatchAggregation]) -> BatchAggregation:
    """`merged_with` folded left over `parts` in order (rank order for per-GPU partials) through
    prio3gpu_batch_aggregation_merge: mod-p share sum, count sum, checksum XOR, Interval::merge."""
    parts = list(parts)
    if not parts:
        raise ValueError("nothing to merge")
    n = len(parts[0].aggregate_share) // field_size
    acc_buf = ctypes.create_string_buffer(bytes(parts[0].aggregate_share), len(parts[0].aggregate_share))
    acc = _BA(ctypes.cast(acc_buf, ctypes.c_void_p), parts[0].report_count,
              (ctypes.c_uint8 * 32)(*parts[0].checksum), *parts[0].interval)
    L = lib()
    for p in parts[1:]:
        if len(p.aggregate_share) != n * field_size:
            raise ValueError("aggregate shares of different lengths")
        sb = ctypes.create_string_buffer(bytes(p.aggregate_share), len(p.aggregate_share))
        src = _BA(ctypes.cast(sb, ctypes.c_void_p), p.report_count,
                  (ctypes.c_uint8 * 32)(*p.checksum), *p.interval)
        check(L.prio3gpu_batch_aggregation_merge(field_size, n, ctypes.byref(acc),
                                                 ctypes.byref(src)), "batch aggregation merge")
    return BatchAggregation(acc_buf.raw[:n * field_size], acc.report_count, bytes(acc.checksum),
                            (acc.interval_start, acc.interval_duration))


def epoch_union(epoch: int, local_keys, all_gather):
    """The epoch's union slot table: the sorted union of every rank's batch identifiers, agreed
    over the host channel `all_gather(obj) -> [obj of each rank]` (e.g.
    torch.distributed.all_gather_object).  Every rank must be at the same epoch."""
    got = all_gather((epoch, sorted(bytes(k) for k in local_keys)))
    epochs = sorted(set(e for e, _ in got))
    if len(epochs) != 1:
        raise RuntimeError(f"epoch merge: ranks are at epochs {epochs}")
    return sorted(set().union(*(set(k) for _, k in got)))


class EpochPartials:
    """One rank's partial `BatchAggregation`s, kept across any number of aggregation jobs and
    keyed by batch identifier (bytes), merged across ranks once per epoch (host path: the
    prio3gpu_batch_aggregation_merge fold; the device path is `epoch_merge_device`)."""

    def __init__(self, field_size: int):
        self.field_size = field_size
        self.parts = {}
        self.epoch = 0

    def add(self, key: bytes, ba: BatchAggregation):
        """Accumulator::update_aggregated of one job's slot into this rank's partial."""
        key = bytes(key)
        cur = self.parts.get(key)
        self.parts[key] = ba if cur is None else merge_batch_aggregations(self.field_size,
                                                                          [cur, ba])

    def merge_epoch(self, all_gather):
        """The epoch's merged aggregations on every rank ({key: BatchAggregation}, each key
        folded over the ranks that hold it, in rank order); the partials are reset and the
        epoch advances."""
        got = all_gather((self.epoch, self.parts))
        epochs = sorted(set(e for e, _ in got))
        if len(epochs) != 1:
            raise RuntimeError(f"epoch merge: ranks are at epochs {epochs}")
        union = sorted(set().union(*(set(p) for _, p in got)))
        out = {k: merge_batch_aggregations(self.field_size, [p[k] for _, p in got if k in p])
               for k in union}
        self.parts = {}
        self.epoch += 1
        return out


class OrdShardStore:
    """The batch-aggregation shards of Janus's datastore, as the patched Janus uses them with one
    process per GPU ("The contract the Janus binding runs"): no collective.

    * `flush` is `Accumulator::flush_to_datastore` (accumulator.rs:133-215) for one batch
      identifier: the job's aggregation goes to shard `ord` (drawn by the writer in
      [0, shard_count), accumulator.rs:88-95); an existing shard (same batch identifier and
      `ord`, written by any process) is `merged_with` the new one and updated, else the new one is
      put.
    * `collect` is `compute_aggregate_share` (aggregate_share.rs:44-80): every shard of the batch
      identifier folded -- checksums XORed, counts summed, shares merged (mod p).

    The store is the shared medium (Janus's Postgres); `tests/test_multirank_cpu.py` feeds it the
    flushes of two gloo ranks."""

    def __init__(self, field_size: int, shard_count: int):
        if shard_count < 1:
            raise ValueError("shard_count must be >= 1")
        self.field_size = field_size
        self.shard_count = shard_count
        self.rows = {}  # (batch identifier, ord) -> BatchAggregation

    def flush(self, key: bytes, ord_: int, ba: BatchAggregation):
        if not 0 <= ord_ < self.shard_count:
            raise ValueError(f"ord {ord_} outside [0, {self.shard_count})")
        k = (bytes(key), int(ord_))
        cur = self.rows.get(k)
        self.rows[k] = ba if cur is None else merge_batch_aggregations(self.field_size, [cur, ba])

    def shards(self, key: bytes):
        return sorted(o for (k, o) in self.rows if k == bytes(key))

    def collect(self, key: bytes) -> BatchAggregation:
        parts = [self.rows[(bytes(key), o)] for o in self.shards(key)]
        if not parts:
            raise KeyError("no batch aggregations for this batch identifier")
        return merge_batch_aggregations(self.field_size, parts)


def epoch_merge_device(comm, vdaf, local, local_keys, epoch: int, all_gather):
    """prio3gpu_agg_epoch_merge over a device partial `local` (AggregateShares whose slot i holds
    batch identifier local_keys[i]; slots past len(local_keys) unused): returns (union keys,
    AggregateShares of the merged totals, one slot per union key).  Every rank calls it once per
    epoch, epochs in the same order."""
    from .prio3 import SLOT_UNUSED
    union = epoch_union(epoch, local_keys, all_gather)
    idx = {k: i for i, k in enumerate(union)}
    slot_map = [idx[bytes(k)] for k in local_keys]
    slot_map += [SLOT_UNUSED] * (local.num_slots - len(slot_map))
    total = vdaf.new_aggregate(len(union))
    comm.epoch_merge(vdaf, local, slot_map, total)
    return union, total
