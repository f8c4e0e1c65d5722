#!/usr/bin/env python3
"""Config E stress bench: Prio3FixedPoint16BitBoundedL2VecSum, entries = 100k (BASELINE.json
configs[4], "large-vector FLP query stress") on one MI355X.

One step = B reports through the leader and helper aggregate-init path (leader prepare_init,
helper prepare_init, prep_shares_to_prep, both prepare_next + accumulate).  The two aggregators'
prepare_init run concurrently on two engine contexts (two HIP streams): they are independent until
decide, like Janus's leader and helper processes.  Inputs: U distinct reports from the C
restatement (SURVEY §8(d) recipe, oracle/prio3_ref.c), tiled to B on the GPU -- every tile is
processed in full; the aggregate is checked against the C restatement's aggregate x tiles.
With --distinct 1 the B reports are all distinct: the SURVEY §8(d) recipe's nonces, randomness
and measurements (C restatement) go through the GPU client shard (prio3gpu_shard, Client::shard
+ FLP prove; the first U are checked byte for byte against the C restatement's shard) and the
check is unshard(leader + helper aggregate) == the plaintext fixed-point sum.
CPU baseline: the C restatement on U reports, 16 threads.

python tools/bench_fpvec.py [--reports B --unique U --steps K --entries E --bits N --distinct 1]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entries", type=int, default=100000)
    ap.add_argument("--bits", type=int, default=16)
    ap.add_argument("--reports", type=int, default=1024)
    ap.add_argument("--unique", type=int, default=16)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--overlap", type=int, default=1)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--distinct", type=int, default=0)
    ap.add_argument("--shard-chunk", type=int, default=512)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option for both contexts (prio3gpu_ctx_set_option), repeatable")
    ap.add_argument("--no-check", type=int, default=0,
                    help="timing-only diagnostic libraries: skip the status / aggregate checks")
    ap.add_argument("--lopt", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option for the leader's context only, repeatable")
    ap.add_argument("--hopt", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option for the helper's context only, repeatable")
    args = ap.parse_args()

    import torch
    from janus_amd._lib import check, lib
    from janus_amd.prio3 import Prio3Gpu
    from oracle import prio3 as O
    from oracle.ref import Prio3Ref

    B, U = args.reports, min(args.unique, args.reports)
    assert args.distinct or B % U == 0
    cid = b"cfgE-%d-%d" % (args.bits, args.entries)
    vk = O.synth_verify_key(cid)
    ref = Prio3Ref(4, vk, args.bits, args.entries, 0)
    t0 = time.time()
    g = ref.gen(cid, 0, U, threads=args.threads)
    t_gen = time.time() - t0
    t0 = time.time()
    res = ref.prepare_batch(g["nonces"], g["public"], g["leader_in"], g["helper_in"],
                            threads=args.threads)
    t_cpu = time.time() - t0
    assert res["count"] == U
    cpu_rate = U / t_cpu
    print(f"# C restatement: gen {U} in {t_gen:.1f}s, prepare+aggregate {U} in {t_cpu:.2f}s "
          f"({cpu_rate:.1f} reports/s, {args.threads} threads)", flush=True)

    dev = torch.device("cuda:0")
    tiles = B // U if not args.distinct else 1
    vl = Prio3Gpu.new_fixedpoint_boundedl2_vec_sum(args.bits, args.entries, vk)
    vh = Prio3Gpu.new_fixedpoint_boundedl2_vec_sum(args.bits, args.entries, vk)
    def parse(lst):
        return dict((o.split("=", 1)[0], int(o.split("=", 1)[1])) for o in lst)

    opts = parse(args.opt)
    lopts, hopts = {**opts, **parse(args.lopt)}, {**opts, **parse(args.hopt)}
    for v_, o_ in ((vl, lopts), (vh, hopts)):
        for k_, val in o_.items():
            v_.set_option(k_, val)
    s = vl.sizes
    shard_info = None
    if args.distinct:
        # B distinct reports: recipe inputs from the C restatement, shares from the GPU shard
        d_nonces = torch.empty((B, 16), dtype=torch.uint8, device=dev)
        d_pub = torch.empty((B, s.public_share), dtype=torch.uint8, device=dev)
        d_lin = torch.empty((B, s.leader_input_share), dtype=torch.uint8, device=dev)
        d_hin = torch.empty((B, s.helper_input_share), dtype=torch.uint8, device=dev)
        plain = np.zeros(args.entries, np.int64)
        CH = min(args.shard_chunk, B)
        sst = vh.new_state(1, CH)
        t_syn = t_sh = 0.0
        for i in range(0, B, CH):
            k = min(CH, B - i)
            t0 = time.time()
            syn = ref.synth(cid, i, k, threads=args.threads)
            t_syn += time.time() - t0
            plain += syn["meas"].view(np.int64).sum(axis=0)
            d_nonces[i:i + k] = torch.from_numpy(syn["nonces"]).to(dev)
            t0 = time.time()
            vh.shard(sst, d_nonces[i:i + k], torch.from_numpy(syn["meas"].view(np.int64)).to(dev),
                     torch.from_numpy(syn["rand"]).to(dev),
                     out=(d_pub[i:i + k], d_lin[i:i + k], d_hin[i:i + k]))
            torch.cuda.synchronize()
            t_sh += time.time() - t0
        sst.close()
        del sst
        k = min(U, B)
        assert np.array_equal(d_lin[:k].cpu().numpy(), g["leader_in"][:k]), "GPU shard != C"
        assert np.array_equal(d_hin[:k].cpu().numpy(), g["helper_in"][:k]), "GPU shard != C"
        assert np.array_equal(d_pub[:k].cpu().numpy(), g["public"][:k]), "GPU shard != C"
        shard_info = {"reports": B, "synth_s": round(t_syn, 2), "gpu_shard_s": round(t_sh, 2),
                      "gpu_shard_reports_per_s": round(B / t_sh, 1),
                      "cpu_gen_reports_per_s": round(U / t_gen, 2),
                      "check": f"first {k} GPU shares == C restatement bytes"}
        print("# " + json.dumps(shard_info), flush=True)
    else:
        def tile(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev).repeat(tiles, 1).contiguous()

        d_nonces, d_pub, d_lin, d_hin = (tile(g[k]) for k in ("nonces", "public", "leader_in",
                                                              "helper_in"))
    ls, hs = vl.new_state(0, B), vh.new_state(1, B)
    lagg, hagg = vl.new_aggregate(1), vh.new_aggregate(1)
    d_lprep = torch.empty((B, s.prep_share), dtype=torch.uint8, device=dev)
    d_hprep = torch.empty((B, s.prep_share), dtype=torch.uint8, device=dev)
    d_msgs = torch.empty((B, s.prep_msg), dtype=torch.uint8, device=dev)
    d_lst = torch.zeros(B, dtype=torch.uint8, device=dev)
    d_hst = torch.zeros(B, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    L = lib()
    P = lambda t: ctypes.c_void_p(t.data_ptr())

    def leader_init():
        check(L.prio3gpu_prepare_init(vl._ctx, ls._h, B, P(d_nonces), P(d_pub), P(d_lin),
                                      P(d_lprep), P(d_lst)), "leader prepare_init")
        check(L.prio3gpu_ctx_sync(vl._ctx), "sync")

    def helper_init():
        check(L.prio3gpu_prepare_init(vh._ctx, hs._h, B, P(d_nonces), P(d_pub), P(d_hin),
                                      P(d_hprep), P(d_hst)), "helper prepare_init")
        check(L.prio3gpu_ctx_sync(vh._ctx), "sync")

    def step():
        d_lst.zero_()
        d_hst.zero_()
        torch.cuda.synchronize()
        if args.overlap:
            th = threading.Thread(target=helper_init)
            th.start()
            leader_init()
            th.join()
        else:
            leader_init()
            helper_init()
        check(L.prio3gpu_prepare_shares_to_prepare_message(vh._ctx, B, P(d_lprep), P(d_hprep),
                                                           P(d_msgs), P(d_hst)), "decide")
        check(L.prio3gpu_prepare_next(vh._ctx, hs._h, B, P(d_msgs), P(d_hst), None, None,
                                      hagg._h), "helper prepare_next")
        check(L.prio3gpu_ctx_sync(vh._ctx), "sync")
        check(L.prio3gpu_prepare_next(vl._ctx, ls._h, B, P(d_msgs), P(d_hst), None, None,
                                      lagg._h), "leader prepare_next")
        check(L.prio3gpu_ctx_sync(vl._ctx), "sync")

    for _ in range(args.warmup):
        step()
    lagg.reset()
    hagg.reset()
    for v in (vl, vh):
        check(L.prio3gpu_prof_enable(v._ctx, 1), "prof")
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.time() - t0) / args.steps
    kern = {}
    for v in (vl, vh):
        ms, nl = (ctypes.c_double * 64)(), (ctypes.c_uint64 * 64)()
        nk = min(64, L.prio3gpu_prof_read(v._ctx, ms, nl, 64))
        for i in range(nk):
            if nl[i]:
                name = L.prio3gpu_prof_kernel_name(i).decode()
                a = kern.setdefault(name, [0.0, 0])
                a[0] += ms[i] / args.steps
                a[1] += nl[i] // args.steps
    # parity: every tile's reports accepted, aggregates = C aggregate x tiles x steps
    if args.no_check:
        print(json.dumps({"reports_per_step": B, "ms_per_step": dt * 1e3, "no_check": True,
                          "kernels_ms_per_step": {k: round(v[0], 3) for k, v in kern.items()}}),
              flush=True)
        return
    assert int(d_hst.eq(0).sum()) == B, "reports rejected"
    la, lc = lagg.read(0)
    ha, hc = hagg.read(0)
    assert lc == hc == B * args.steps
    mult = tiles * args.steps
    p = O.Field128.MODULUS
    if args.distinct:
        # unshard(leader + helper) == plaintext sum of the fixed-point values (x steps)
        got = vl.unshard([la, ha], num_measurements=B * args.steps)
        want = [float(x) * args.steps * 2.0 ** (1 - args.bits) for x in plain]
        assert got == want, "aggregate != plaintext sum"
    else:
        for got, exp in ((la, res["agg_l"]), (ha, res["agg_h"])):
            e = O.Field128.decode_vec(exp.tobytes())
            assert O.Field128.decode_vec(got) == [(x * mult) % p for x in e], "aggregate mismatch"
    out = {"config": f"Prio3FixedPoint{args.bits}BitBoundedL2VecSum entries={args.entries}",
           "reports_per_step": B, "unique": B if args.distinct else U,
           "gpu_shard": shard_info, "ms_per_step": dt * 1e3,
           "reports_per_sec": B / dt, "overlap_leader_helper": bool(args.overlap),
           "engine_options": {"leader": lopts, "helper": hopts},
           "cpu_baseline": {"reports_per_sec": cpu_rate, "threads": args.threads,
                            "kind": "port", "sample": f"{U} reports"},
           "speedup_vs_cpu": (B / dt) / cpu_rate,
           "kernels_ms_per_step": {k: round(v[0], 3) for k, v in kern.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
