"""Report sharding across GPUs: one process per GPU, contiguous report ranges,
no data-path collective; the only exchange is the end-of-job merge of per-GPU partial aggregate
shares (RCCL all-gather of raw LE field-element bytes + mod-p add kernel, `Comm.allreduce`) with
the checksum / interval half of `BatchAggregation::merged_with` folded on the host
(`merge_batch_aggregations`, the same C-ABI function the GPU merge calls).

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
