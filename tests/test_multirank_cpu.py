"""N > 1 path on CPU (gloo, world_size 2): reports sharded by janus_amd.parallel.shard_range, each
rank aggregates its shard (C restatement as the stand-in for the GPU, which this container lacks),
partial aggregate shares are all-gathered as raw LE bytes and merged mod p in rank order -- the
exchange Comm.allreduce performs with RCCL on the GPU.  The merged result must equal the
single-process aggregate over all reports, for both aggregators, bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N = 24
NAME = "hist4"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from janus_amd.parallel import shard_range
    from oracle.ref import Prio3Ref
    from tests.reports import CONFIGS
    from oracle import prio3 as O
    c = CONFIGS[NAME]
    vk = O.synth_verify_key(b"mr")
    r = Prio3Ref(c["kind"], vk, c["bits"], c["length"], c["chunk"])
    lo, hi = shard_range(N, world, rank)
    g = r.gen(b"mr", lo, hi - lo, threads=1)
    res = r.prepare_batch(g["nonces"], g["public"], g["leader_in"], g["helper_in"], threads=1,
                          outputs=False)
    parts = [None] * world
    dist.all_gather_object(parts, (res["agg_l"].tobytes(), res["agg_h"].tobytes(), res["count"]))
    p, es = O.Field128.MODULUS, 16
    merged = []
    for which in (0, 1):
        acc = [0] * (len(parts[0][which]) // es)
        for part in parts:  # rank order
            vec = O.Field128.decode_vec(part[which])
            acc = [(a + b) % p for a, b in zip(acc, vec)]
        merged.append(O.Field128.encode_vec(acc))
    count = sum(part[2] for part in parts)
    if rank == 0:
        q.put((merged[0], merged[1], count))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_merge():
    from oracle.ref import Prio3Ref
    from tests.reports import CONFIGS
    from oracle import prio3 as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    got = q.get(timeout=120)
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    c = CONFIGS[NAME]
    r = Prio3Ref(c["kind"], O.synth_verify_key(b"mr"), c["bits"], c["length"], c["chunk"])
    g = r.gen(b"mr", 0, N, threads=1)
    res = r.prepare_batch(g["nonces"], g["public"], g["leader_in"], g["helper_in"], threads=1,
                          outputs=False)
    assert got[0] == res["agg_l"].tobytes() and got[1] == res["agg_h"].tobytes()
    assert got[2] == N == res["count"]


def test_shard_ranges_cover():
    from janus_amd.parallel import shard_range
    for n in [0, 1, 7, 1000, 262144]:
        for w in [1, 2, 3, 8]:
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
