"""N > 1 path on CPU (gloo, world_size 2).  Reports are sharded by janus_amd.parallel.shard_range;
each rank aggregates its shard (the C restatement stands in for the GPU, which this container
lacks) into a `BatchAggregation` per aggregator (aggregate share, count, ReportIdChecksum,
client-timestamp interval); the partials are all-gathered and folded in rank order by the
product's merge, prio3gpu_batch_aggregation_merge (janus_amd.parallel.merge_batch_aggregations)
-- the host half of the exchange Comm.allreduce performs after its RCCL all-gather.  The merged
result must equal the single-process aggregation over all reports, bit for bit.

Reference semantics: BatchAggregation::merged_with (aggregator_core/src/datastore/models.rs:
962-991), Interval::merge (core/src/time.rs:289-302, test cases :357-406), ReportIdChecksum
(core/src/report_id.rs:18-44), batch-aggregation shard merge (aggregate_share.rs:47-65)."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N = 24
NAME = "hist4"
T0 = 1_600_000_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _checksum(nonces):
    ck = np.zeros(32, np.uint8)
    for r in range(len(nonces)):
        ck ^= np.frombuffer(hashlib.sha256(nonces[r].tobytes()).digest(), np.uint8)
    return ck.tobytes()


def _times(lo, hi):
    return [T0 + 37 * i + (i % 5) for i in range(lo, hi)]


def _partials(lo, hi):
    """(leader, helper) BatchAggregations of reports [lo, hi) from the C restatement."""
    from janus_amd.parallel import BatchAggregation
    from oracle import prio3 as O
    from oracle.ref import Prio3Ref
    from tests.reports import CONFIGS
    c = CONFIGS[NAME]
    r = Prio3Ref(c["kind"], O.synth_verify_key(b"mr"), c["bits"], c["length"], c["chunk"])
    g = r.gen(b"mr", lo, hi - lo, threads=1)
    res = r.prepare_batch(g["nonces"], g["public"], g["leader_in"], g["helper_in"], threads=1,
                          outputs=False)
    ck = _checksum(g["nonces"])
    t = _times(lo, hi)
    iv = (min(t), max(t) - min(t) + 1) if t else (0, 0)
    return tuple(BatchAggregation(res[k].tobytes(), res["count"], ck, iv)
                 for k in ("agg_l", "agg_h"))


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from janus_amd.parallel import merge_batch_aggregations, shard_range
    lo, hi = shard_range(N, world, rank)
    mine = _partials(lo, hi)
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    merged = [merge_batch_aggregations(16, [p[which] for p in parts]) for which in (0, 1)]
    q.put((rank, merged))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_merge():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    want = _partials(0, N)  # one process over every report
    for rank in (0, 1):  # every rank holds the same merged totals
        for which in (0, 1):
            g, w = got[rank][which], want[which]
            assert g.aggregate_share == w.aggregate_share
            assert g.report_count == w.report_count == N
            assert g.checksum == w.checksum
            assert g.interval == w.interval


def test_merge_interval_reference_cases():
    """Interval::merge as the reference's own test pins it (core/src/time.rs:357-406)."""
    from janus_amd.parallel import BatchAggregation, merge_batch_aggregations
    cases = [((0, 10), (20, 10), (0, 30)), ((0, 10), (5, 10), (0, 15)), ((0, 10), (2, 8), (0, 10)),
             ((0, 10), (0, 10), (0, 10)), ((0, 0), (0, 10), (0, 10)), ((0, 10), (0, 0), (0, 10)),
             ((0, 0), (0, 0), (0, 0))]
    for lhs, rhs, want in cases:
        a = BatchAggregation(bytes(16), 1, bytes(32), lhs)
        b = BatchAggregation(bytes(16), 2, bytes(32), rhs)
        m = merge_batch_aggregations(16, [a, b])
        assert m.interval == want and m.report_count == 3


def test_merge_mod_p_and_checksum():
    from janus_amd.parallel import BatchAggregation, merge_batch_aggregations
    from janus_amd.prio3 import FIELD64_MODULUS as P64, FIELD128_MODULUS as P128
    from janus_amd._lib import Prio3GpuError
    for es, p in ((16, P128), (8, P64)):
        xs = [p - 1, p - 2, 5, 0]
        ys = [p - 1, 3, p - 5, 0]
        enc = lambda v: b"".join(int(x).to_bytes(es, "little") for x in v)
        a = BatchAggregation(enc(xs), 1, bytes(range(32)), (5, 1))
        b = BatchAggregation(enc(ys), 1, bytes(32 * [0xFF]), (9, 1))
        m = merge_batch_aggregations(es, [a, b])
        assert m.aggregate_share == enc([(x + y) % p for x, y in zip(xs, ys)])
        assert m.checksum == bytes(i ^ 0xFF for i in range(32)) and m.interval == (5, 5)
        with pytest.raises(Prio3GpuError):  # a non-canonical element is refused
            merge_batch_aggregations(es, [a, BatchAggregation(enc([p, 0, 0, 0]), 1)])


def test_shard_ranges_cover():
    from janus_amd.parallel import shard_range
    for n in [0, 1, 7, 1000, 262144]:
        for w in [1, 2, 3, 8]:
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


# ---- epoch merge: independent job counts per rank, one merge per epoch -------------------------
# Reports r = 0..N_EPOCH-1 arrive in jobs of JOB reports; rank 0 drives 3 jobs, rank 1 drives 5
# (independent job drivers: no per-job collective).  Report r falls in batch identifier
# r // BUCKET (time-interval buckets), so the ranks hold different key sets.
N_EPOCH, JOB, BUCKET = 40, 5, 7
JOBS_OF = {0: [0, 1, 2], 1: [3, 4, 5, 6, 7]}


def _key_partials(reports):
    """{key: (leader, helper) BatchAggregation} of the given report indices, per batch
    identifier, from the C restatement."""
    from janus_amd.parallel import BatchAggregation
    from oracle import prio3 as O
    from oracle.ref import Prio3Ref
    from tests.reports import CONFIGS
    c = CONFIGS[NAME]
    r = Prio3Ref(c["kind"], O.synth_verify_key(b"ep"), c["bits"], c["length"], c["chunk"])
    g = r.gen(b"ep", 0, N_EPOCH, threads=1)
    out = {}
    for key in sorted(set(i // BUCKET for i in reports)):
        idx = [i for i in reports if i // BUCKET == key]
        res = r.prepare_batch(g["nonces"][idx], g["public"][idx], g["leader_in"][idx],
                              g["helper_in"][idx], threads=1, outputs=False)
        t = [T0 + 37 * i for i in idx]
        iv = (min(t), max(t) - min(t) + 1)
        ck = _checksum(g["nonces"][idx])
        out[key.to_bytes(4, "big")] = tuple(BatchAggregation(res[k].tobytes(), res["count"], ck, iv)
                                            for k in ("agg_l", "agg_h"))
    return out


def _epoch_rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from janus_amd.parallel import EpochPartials

    def all_gather(obj):
        got = [None] * world
        dist.all_gather_object(got, obj)
        return got
    parts = [EpochPartials(16), EpochPartials(16)]  # leader, helper
    for job in JOBS_OF[rank]:  # each job flushes into this rank's partials, no collective
        for key, bas in _key_partials(range(job * JOB, (job + 1) * JOB)).items():
            for which in (0, 1):
                parts[which].add(key, bas[which])
    merged = [p.merge_epoch(all_gather) for p in parts]
    # a second, empty epoch: the partials were reset and the epochs advance together
    empty = [p.merge_epoch(all_gather) for p in parts]
    q.put((rank, merged, empty, [p.epoch for p in parts]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_epoch_merge_different_job_counts():
    """Ranks drive 3 and 5 jobs, keep per-key partials across their jobs and merge ONCE at the
    epoch boundary: every rank's merged BatchAggregations (share, count, checksum, interval) equal
    the single-process aggregation of all 40 reports per batch identifier, bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_epoch_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=180) for _ in procs))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    want = _key_partials(range(N_EPOCH))
    assert len(want) == -(-N_EPOCH // BUCKET)
    for rank in (0, 1):
        merged, empty, epochs = got[rank]
        assert epochs == [2, 2] and empty == [{}, {}]
        for which in (0, 1):
            assert sorted(merged[which]) == sorted(want)
            for key, w in want.items():
                g = merged[which][key]
                assert g.aggregate_share == w[which].aggregate_share
                assert g.report_count == w[which].report_count
                assert g.checksum == w[which].checksum and g.interval == w[which].interval


def test_epoch_merge_refuses_ranks_at_different_epochs():
    from janus_amd.parallel import EpochPartials, epoch_union
    p = EpochPartials(16)
    with pytest.raises(RuntimeError):
        p.merge_epoch(lambda obj: [obj, (obj[0] + 1, {})])
    with pytest.raises(RuntimeError):
        epoch_union(3, [b"a"], lambda obj: [obj, (2, [b"b"])])
    assert epoch_union(3, [b"b", b"a"], lambda obj: [obj, (3, [b"c", b"a"])]) == [b"a", b"b", b"c"]


# ---- the contract the Janus binding runs: per-job flushes into `ord` shards, no collective -----
# Each rank flushes every job's per-batch-identifier aggregation into the shared datastore as the
# patched Janus does (Accumulator::update_aggregated, then flush_to_datastore into a random shard
# `ord`, accumulator.rs:88-95 / :133-215); collection merges the shards (aggregate_share.rs:44-80).
# The "datastore" is janus_amd.parallel.OrdShardStore; the rows reach it over gloo.
SHARD_COUNT = 2  # small, so both ranks write some (batch identifier, ord) rows: the merge path


def _ord_rank_main(rank, world, port, q):
    import random

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = random.Random(1000 + rank)  # thread_rng().gen_range(0..shard_count) of the writer
    rows = []
    for job in JOBS_OF[rank]:
        for key, bas in _key_partials(range(job * JOB, (job + 1) * JOB)).items():
            rows.append((key, rng.randrange(SHARD_COUNT), bas))
    got = [None] * world
    dist.all_gather_object(got, rows)  # stands in for the rows both processes write to Postgres
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_ord_shard_flush_matches_single_process():
    """Two GPU processes flush their jobs (3 and 5) into batch-aggregation shards with random
    `ord`, without any collective; the collection-time merge of every batch identifier's shards
    equals the single-process aggregation of all 40 reports, bit for bit, for both aggregators."""
    from janus_amd.parallel import OrdShardStore
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ord_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    assert got[0] == got[1]
    writes = got[0]
    stores = [OrdShardStore(16, SHARD_COUNT), OrdShardStore(16, SHARD_COUNT)]
    writers = {}
    for rank, rows in enumerate(writes):
        for key, ord_, bas in rows:
            writers.setdefault((key, ord_), set()).add(rank)
            for which in (0, 1):
                stores[which].flush(key, ord_, bas[which])
    # the shards were really shared: some row was written by both processes (merged_with path)
    # and some batch identifier spans more than one shard (the collection-time merge)
    assert any(len(w) == 2 for w in writers.values())
    want = _key_partials(range(N_EPOCH))
    assert any(len(stores[0].shards(k)) > 1 for k in want)
    for which in (0, 1):
        for key, w in want.items():
            g = stores[which].collect(key)
            assert g.aggregate_share == w[which].aggregate_share
            assert g.report_count == w[which].report_count
            assert g.checksum == w[which].checksum and g.interval == w[which].interval


def test_ord_shard_store_rejects_out_of_range_ord():
    from janus_amd.parallel import BatchAggregation, OrdShardStore
    s = OrdShardStore(16, 4)
    with pytest.raises(ValueError):
        s.flush(b"k", 4, BatchAggregation(bytes(16), 1))
    with pytest.raises(KeyError):
        s.collect(b"k")
