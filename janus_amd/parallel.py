"""Report sharding across GPUs: one process per GPU, contiguous report ranges,
no data-path collective; the only exchange is the end-of-job merge of per-GPU partial aggregate
shares (RCCL all-gather of raw LE field-element bytes + mod-p add kernel, `Comm.allreduce`).

Janus analogue: independent aggregation jobs on concurrent job-driver workers
(`aggregator/src/binary_utils/job_driver.rs:119-216`) whose partial batch aggregations are merged
(`aggregator_core/src/datastore/models.rs:962-991`, `aggregate_share.rs:47-65`).
"""
from __future__ import annotations

import os


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n: int, world_size: int, rank: int):
    """GPU `rank` takes reports [rank*n/G, (rank+1)*n/G)."""
    return (n * rank) // world_size, (n * (rank + 1)) // world_size
