#!/usr/bin/env python3
"""Time the sponge kernels alone (measurement tooling, not a parity check): the leader's and the
helper's prepare_init XOF phase (k_query_rand + k_jr; k_query_rand + k_expand + k_jr) over B
SumVec(8,1000) reports of random bytes, per-kernel milliseconds from the engine's HIP-event
profiler.  Variant builds are selected with PRIO3GPU_LIB (tools/build_variant.sh); variants that
change what is absorbed or stored give wrong bytes, which this harness never looks at.

    python tools/sponge_ab.py [--reports B] [--reps R] [--pitch P]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reports", type=int, default=0, help="default: 393216 SumVec, else 2^20")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pitch", type=int, default=0)
    ap.add_argument("--label", default=os.path.basename(os.environ.get("PRIO3GPU_LIB", "base")))
    ap.add_argument("--config", default="sumvec", choices=["sumvec", "histogram", "sum"])
    ap.add_argument("--query", type=int, default=0,
                    help="also time the FLP query phase (prepare_init_query) of both aggregators")
    a = ap.parse_args()
    import torch
    from janus_amd._lib import check, lib
    from janus_amd.prio3 import HISTOGRAM, SUM, SUMVEC, Prio3Gpu
    kind, bits, length, chunk = {"sumvec": (SUMVEC, 8, 1000, 89), "histogram": (HISTOGRAM, 0, 256, 16),
                                 "sum": (SUM, 32, 0, 0)}[a.config]
    v = Prio3Gpu(kind, bytes(range(16)), bits=bits, length=length, chunk_length=chunk, device=0)
    s = v.sizes
    B = a.reports or (393216 if a.config == "sumvec" else 1 << 20)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    pitch = a.pitch or s.leader_input_share
    lin = torch.randint(0, 256, (B, pitch), dtype=torch.uint8, device=dev, generator=g)
    hin = torch.randint(0, 256, (B, s.helper_input_share), dtype=torch.uint8, device=dev,
                        generator=g)
    nonces = torch.randint(0, 256, (B, 16), dtype=torch.uint8, device=dev, generator=g)
    pub = torch.randint(0, 256, (B, s.public_share), dtype=torch.uint8, device=dev, generator=g)
    lst = torch.zeros(B, dtype=torch.uint8, device=dev)
    hst = torch.zeros(B, dtype=torch.uint8, device=dev)
    ls, hs = v.new_state(0, B), v.new_state(1, B)
    L = lib()
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    ls.set_input_pitch(0 if pitch == s.leader_input_share else pitch)
    cx = v._ctx
    check(L.prio3gpu_prof_enable(cx, 1), "prof")

    prep = torch.empty((B, s.prep_share), dtype=torch.uint8, device=dev)

    def run(leader):
        lst.zero_()
        hst.zero_()
        torch.cuda.synchronize()
        st, stt, inp = (ls, lst, lin) if leader else (hs, hst, hin)
        check(L.prio3gpu_prepare_init_xof(cx, st._h, B, P(nonces), P(pub), P(inp), P(stt)), "xof")
        if a.query:
            stt.zero_()  # random shares: keep every report in the query
            check(L.prio3gpu_prepare_init_query(cx, st._h, B, P(prep), P(stt)), "query")
        check(L.prio3gpu_ctx_sync(cx), "sync")

    def read():
        ms, nl = (ctypes.c_double * 64)(), (ctypes.c_uint64 * 64)()
        nk = L.prio3gpu_prof_read(cx, ms, nl, 64)
        return {L.prio3gpu_prof_kernel_name(i).decode(): (ms[i], nl[i]) for i in range(nk) if nl[i]}

    run(True)
    run(False)
    read()
    out = {}
    for _ in range(a.reps):
        for leader in (True, False):
            run(leader)
            for k, (t, n) in read().items():
                out.setdefault(k + ("_leader" if leader else ""), []).append(t / n)
    res = {k: round(min(x), 3) for k, x in out.items()}
    perms = {"k_jr": 765, "k_jr_leader": 765, "k_expand": 804} if a.config == "sumvec" else {}
    rate = {k: round(perms[k] * B / (res[k] * 1e-3) / 1e9, 3) for k in perms if k in res}
    print(json.dumps({"label": a.label, "config": a.config, "reports": B, "pitch": pitch,
                      "ms_per_launch_min": res, "G_perms_per_s": rate}))


if __name__ == "__main__":
    main()
