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
    ap.add_argument("--reports", type=int, default=393216)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pitch", type=int, default=0)
    ap.add_argument("--label", default=os.path.basename(os.environ.get("PRIO3GPU_LIB", "base")))
    a = ap.parse_args()
    import torch
    from janus_amd._lib import check, lib
    from janus_amd.prio3 import SUMVEC, Prio3Gpu
    v = Prio3Gpu(SUMVEC, bytes(range(16)), bits=8, length=1000, chunk_length=89, device=0)
    s = v.sizes
    B = a.reports
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

    def run(leader):
        lst.zero_()
        hst.zero_()
        torch.cuda.synchronize()
        if leader:
            check(L.prio3gpu_prepare_init_xof(cx, ls._h, B, P(nonces), P(pub), P(lin), P(lst)),
                  "leader xof")
        else:
            check(L.prio3gpu_prepare_init_xof(cx, hs._h, B, P(nonces), P(pub), P(hin), P(hst)),
                  "helper xof")
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
                out.setdefault(k + ("_leader" if leader and k == "k_jr" else ""), []).append(t / n)
    res = {k: round(min(x), 3) for k, x in out.items()}
    perms = {"k_jr": 765, "k_jr_leader": 765, "k_expand": 804}
    rate = {k: round(perms[k] * B / (res[k] * 1e-3) / 1e9, 3) for k in perms if k in res}
    print(json.dumps({"label": a.label, "reports": B, "pitch": pitch, "ms_per_launch_min": res,
                      "G_perms_per_s": rate}))


if __name__ == "__main__":
    main()
