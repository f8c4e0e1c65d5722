#!/usr/bin/env python3
"""Bench: reports/sec prepared+aggregated, Prio3SumVec(bits=8, length=1000, chunk=89), 1..N GPUs.

One "step" = one batch of B synthetic reports per GPU (weak scaling) taken through Janus's whole
aggregate-init hot path on the GPU: leader prepare_init (aggregation_job_driver.rs:362-380), helper
prepare_init + prep_shares_to_prep + prepare_next + accumulate (aggregator.rs:1775-1819), leader
prepare_next + accumulate (aggregation_job_driver.rs:579-627).  For N > 1 every step ends with the
RCCL all-gather + mod-p merge of both aggregators' per-GPU partial aggregate shares.  Inputs
(decrypted shares, SURVEY.md §8(d) recipe) are resident in HBM before timing starts; HPKE is out of
scope.

Launch: python bench.py [--gpus N --steps K --warmup W].  N > 1: bench.py starts the N ranks itself
(a child `torch.distributed.run`, one process per GPU), or runs as one rank of an outside launcher
whose WORLD_SIZE must equal N (a mismatch is an error).  Prints one JSON line on rank 0.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (kind, bits, length, chunk, metric label)
    "sumvec": (2, 8, 1000, 89, "Prio3SumVec bits=8 length=1000 chunk=89"),
    "sum": (1, 32, 0, 0, "Prio3Sum bits=32"),
    "histogram": (3, 0, 256, 16, "Prio3Histogram length=256 chunk=16"),
    "count": (0, 0, 0, 0, "Prio3Count"),
}
METRIC = "reports/sec prepared+aggregated, Prio3SumVec len=1000, 1/2/4/8 GPUs"

# gfx950 peaks (MI355X_MICROARCH.md): FP32 vector 157.3 TFLOP/s = 256 CU x 128 lanes/clk x 2.4 GHz
# x 2 (FMA)  ->  int32 VALU 78.6 Tops/s;  HBM3E 8.0 TB/s.
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0
HBM_COPY_GBS = 6290.0  # measured float4 copy (MI355X_MICROARCH.md): the achievable stream rate
# SURVEY.md §8(d) declared cost model: 7,440 int32 VALU ops per Keccak-f[1600]; 36 per F128 mul.
OPS_PER_PERM = 7440
OPS_PER_F128_MUL = 36
OPS_PER_F64_MUL = 10
# VALU issue rate: 256 CU x 4 SIMD x 2.4 GHz, a wave64 instruction every 2 cycles on a 32-lane SIMD
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2
# Measured register-only Keccak-f[1600] ceiling of one MI355X (tools/mb_keccak_occ.hip,
# profiles/microbench_keccak_mem_r01.log: 10.3-10.8 G permutations/s at 2-6 waves/SIMD)
KECCAK_CEILING = 10.8e9
PMC_ROUND = "r06"


def cpu_threads(requested=0):
    """Threads for the CPU legs: the host CPUs this process may run on (affinity), capped by the
    cgroup CPU quota and by OMP_NUM_THREADS when set (a GPU box grants a 16-CPU share of a larger
    machine and announces it that way)."""
    if requested > 0:
        return requested
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    try:
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        pass
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_cpu_info():
    info = {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
    try:
        info["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    return info


def load_pmc(config):
    """Per-kernel PMC summary of the same bench command (tools/profile_round.sh), this round's
    first: {"source": path, "kernels": {name: {...}}}."""
    for path in (os.path.join(ROOT, "profiles", PMC_ROUND, f"pmc_{config}.json"),
                 os.path.join(ROOT, "profiles", f"pmc_{config}.json")):
        if os.path.exists(path):
            try:
                return {"source": os.path.relpath(path, ROOT), "kernels": json.load(open(path))}
            except (OSError, ValueError):
                pass
    return {}


def flp_wires_bytes_per_report(s, mfma=False):
    """Algorithmic HBM bytes of the FLP wire pass per report (ParallelSum types): the measurement
    share once, the weight-row entries it reads -- MM[calls] | LM[calls] | RP[c] | L0 | HL, plus
    SMM, SLM (k_flp_wires_mfma's offset correction) -- the 2c wire seeds of the proof share, and
    the 2c wire values written into the prep share."""
    es = s.field_size
    arity = s.verifier_len - 2
    c = arity // 2
    calls = -(-s.meas_len // c)
    w_len = 2 * calls + c + (4 if mfma else 2)
    return (s.meas_len + w_len + 2 * arity) * es


def flp_weights_bytes_per_report(s):
    """Algorithmic HBM bytes of k_flp_weights per report (ParallelSum types): the
    gadget-poly part of the proof share and t, r read; the weight row MM[calls] | LM[calls] |
    RP[c] | L0 | HL | gsum | SMM | SLM written; the block-start prefix products (one per 8 calls)
    written and read back; v, p(t) and the 16-byte part copied into the prep share."""
    es = s.field_size
    arity = s.verifier_len - 2
    c = arity // 2
    calls = -(-s.meas_len // c)
    gp_len = s.proof_len - arity
    w_len = 2 * calls + c + 5
    scratch = 2 * ((calls + 7) // 8)
    return (gp_len + 2 + w_len + scratch + 2) * es + 2 * 16


def flp_mults_per_report(sizes, kind):
    """SURVEY §8(d)'s FLP op model: field multiplications of ONE aggregator's prio-style FLP query
    (Type::query with the QueryShim gadget; count the spec algorithm, not this engine's): every
    wire polynomial interpolated by a size-m inverse NTT (m/2 log2 m) and evaluated at t by
    Horner (m), the gadget polynomial at t (gp_len), its values at the m-th roots by one
    size-2m NTT (m log2 2m), and the validity circuit (~2 per measurement element, Count 1).
    Gives Sum32 ~0.9K, Histogram256 ~4.6K, SumVec(8,1000) ~128K."""
    arity = sizes.verifier_len - 2
    calls = {0: 1, 1: sizes.meas_len}.get(kind)
    if calls is None:  # ParallelSum: chunk = arity / 2 columns per call
        calls = -(-sizes.meas_len // (arity // 2))
    m = 1 << max(1, math.ceil(math.log2(calls + 1)))
    lg = int(math.log2(m))
    gp_len = sizes.proof_len - arity
    wires = arity * (m // 2 * lg + m)
    return wires + gp_len + m * (lg + 1) + (1 if kind == 0 else 2 * sizes.meas_len)


def perms_per_report(kind_name, sizes):
    """Keccak-f[1600] permutations per report executed by each XOF kernel (one aggregator)."""
    es = sizes.field_size

    def squeeze(nelem):
        return max(1, math.ceil(nelem * es / 168))

    jr = sizes.joint_rand_len
    part = math.ceil((42 + sizes.meas_len * es + 1) / 168) if jr else 0
    return {
        "k_query_rand": 0 if kind_name == "count" else 1,  # Count: inside k_flp_query_lane
        "k_expand": squeeze(sizes.meas_len) + squeeze(sizes.proof_len),
        "k_jr": (part + 1 + squeeze(jr)) if jr else 0,
        "k_decide": 1 if jr else 0,
    }


def leader_output_shares(leader_in, kind, bits, length, s, p):
    """prio's truncate() of the leader's measurement share (the first MEAS elements of its input
    share), exact integers: Count/Histogram keep the share, Sum/SumVec fold each entry's bits as
    sum_b 2^b x_b mod p.  (n, OUT * ES) uint8."""
    es = s.field_size
    n = leader_in.shape[0]
    m = leader_in[:, :s.meas_len * es].reshape(n, s.meas_len, es)
    x = np.zeros((n, s.meas_len), dtype=object)
    for k in range(es // 8):
        x += m[:, :, 8 * k:8 * k + 8].copy().view("<u8").reshape(n, s.meas_len).astype(object) << (64 * k)
    if kind in (1, 2):
        nb = bits
        x = x.reshape(n, -1, nb)
        w = np.array([1 << b for b in range(nb)], dtype=object)
        x = (x * w).sum(axis=2) % p
    out = np.zeros((n, x.shape[1] * es), np.uint8)
    for i in range(n):
        out[i] = np.frombuffer(b"".join(int(v).to_bytes(es, "little") for v in x[i]), np.uint8)
    return out


def oracle_transcript_gate(vdaf, kind, bits, length, chunk, vk, syn, d_pub, d_lin, d_hin, n=2):
    """XofTurboShake128 runs (no C restatement of that XOF): the first n synthetic reports through
    the Python oracle's run_vdaf (VdafTranscript, core/src/test_util/mod.rs:87-233) vs the GPU's
    client shard, both prep shares, prep messages and both output shares, byte for byte."""
    from oracle import prio3 as O
    ctor = {0: lambda: O.Prio3.new_count(), 1: lambda: O.Prio3.new_sum(bits),
            2: lambda: O.Prio3.new_sum_vec(bits, length, chunk),
            3: lambda: O.Prio3.new_histogram(length, chunk)}[kind]
    ov = ctor()
    ov.xof = O.XofTurboShake128
    s = vdaf.sizes
    rows = dict(public_share=d_pub, leader_input_share=d_lin, helper_input_share=d_hin)
    want = {k: [] for k in ("leader_prep_share", "helper_prep_share", "prep_msg",
                            "leader_out_share", "helper_out_share")}
    for i in range(n):
        nonce = syn["nonces"][i].tobytes()
        m = [int(x) for x in syn["meas"][i]] if kind == 2 else int(syn["meas"][i][0])
        t = O.run_vdaf(ov, vk, nonce, m, syn["rand"][i].tobytes())
        for k, d in rows.items():
            if d is not None:
                assert d[i].cpu().numpy().tobytes() == t[k], f"GPU shard != oracle {k}"
        for k in want:
            want[k].append(t[k])
    nz = syn["nonces"][:n]
    pub = d_pub[:n].cpu().numpy() if d_pub is not None else None
    ls, hs = vdaf.new_state(0, n), vdaf.new_state(1, n)
    lp, lst = vdaf.prepare_init(ls, nz, pub, d_lin[:n].cpu().numpy())
    hp, hst = vdaf.prepare_init(hs, nz, pub, d_hin[:n].cpu().numpy())
    msgs, st = vdaf.prepare_shares_to_prepare_message(lp, hp)
    lo, lst = vdaf.prepare_next(ls, msgs, lst.copy())
    ho, hst = vdaf.prepare_next(hs, msgs, hst.copy())
    assert (lst == 0).all() and (hst == 0).all() and (st == 0).all()
    got = dict(leader_prep_share=lp, helper_prep_share=hp, prep_msg=np.asarray(msgs)[:, :s.prep_msg],
               leader_out_share=lo, helper_out_share=ho)
    for k, rows_ in want.items():
        assert np.asarray(got[k]).tobytes() == b"".join(rows_), f"GPU {k} != oracle"
    ls.close()
    hs.close()
    return (f"first {n} reports: GPU client shard, prep shares, prep messages and output shares "
            f"== Python oracle run_vdaf (XofTurboShake128)")


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_argv(n: int, argv, port: int):
    """The child command that runs this bench as n ranks on one node (Janus scales the same
    path by running aggregation jobs concurrently, aggregator/src/binary_utils/job_driver.rs:
    119-216; here each rank owns one GPU and a contiguous report range)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def launch_ranks(n: int, argv) -> int:
    """Run the n-rank bench as a child process (rank 0's JSON line goes straight to our stdout)
    and return its exit code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC on this host driver
    return subprocess.run(launcher_argv(n, argv, free_port()), env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="sumvec", choices=list(CONFIGS))
    ap.add_argument("--reports", type=int, default=0, help="reports per GPU per step (B)")
    ap.add_argument("--leader-pitch", type=int, default=0,
                    help="row pitch of the leader input shares in HBM (0 packed, -1 next 128 B)")
    ap.add_argument("--unique", type=int, default=0, help="CPU-baseline sample size (reports)")
    ap.add_argument("--gen-threads", type=int, default=16)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: the host CPUs this process may use)")
    ap.add_argument("--overlap", type=int, default=-1,
                    help="0: leader then helper on one context; 1: leader and helper on separate "
                         "contexts/streams, prepare_init concurrent (like two aggregator "
                         "processes sharing the GPU); 2: pipelined schedule (each batch's FLP "
                         "query under the other aggregator's Keccak, async contexts, see DESIGN "
                         "§5); 3: the same with the latency-bound FLP weights kept out from under "
                         "the Keccak (only the HBM-bound wire pass overlaps).  -1 (default): the "
                         "measured best per config -- 1 for Count, Sum and Histogram (their one-"
                         "lane-per-report sponge launches end in a partly filled wave round that "
                         "the other aggregator's launch fills), 0 for SumVec")
    ap.add_argument("--async-calls", type=int, default=1,
                    help="--overlap 0/1, one rank: engine calls return once queued "
                         "(prio3gpu_ctx_set_async; every buffer is device memory), so a step's "
                         "calls run back to back with no host round trip between them; the two "
                         "contexts are ordered by marks")
    ap.add_argument("--helper-only", type=int, default=1, help="also time the helper path alone")
    ap.add_argument("--prof-steps", type=int, default=2,
                    help="untimed serial kernel pass after the timed steps (synchronous calls, "
                         "one kernel at a time): the per-kernel durations behind `roofline` and "
                         "kernels_ms_per_step (0: use the timed steps' HIP-event spans)")
    ap.add_argument("--hpke", type=int, default=1, help="time the CPU HPKE-open stage (rank 0, N=1)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--xof", default="shake128", choices=["shake128", "turboshake128"],
                    help="XofShake128 (prio 0.15.1 / VDAF-07: the reference's XOF, the metric) or "
                         "XofTurboShake128 (VDAF-08+, the north star's Keccak-p[1600,12]; the C "
                         "restatement is SHAKE128-only, so its gates use the Python oracle)")
    ap.add_argument("--merge", default="rccl", choices=["rccl", "gloo"],
                    help="N > 1: per-step RCCL all-gather + mod-p merge (the product path), or "
                         "'gloo' = a rehearsal of the multi-rank bench on fewer GPUs than ranks "
                         "(ranks share GPUs, aggregates merged once over gloo at the end)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option for every context (prio3gpu_ctx_set_option), repeatable")
    ap.add_argument("--workers", type=int, default=1,
                    help="concurrent aggregation-job workers per GPU, one engine context (HIP "
                         "stream) and one contiguous slice of the batch each (Janus "
                         "max_concurrent_job_workers)")
    args = ap.parse_args()
    if args.overlap < 0:  # profiles/r04/ab_r4u_*.log
        args.overlap = 0 if args.config == "sumvec" else 1

    # One process per GPU.  `--gpus N` without a launcher: start the N ranks ourselves, as a
    # child torch.distributed.run (never exec: nothing here has touched the GPU yet, and the
    # parent only relays).  Under a launcher, WORLD_SIZE must be N.
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU "
              f"(or drop --gpus and let bench.py start them)", file=sys.stderr)
        sys.exit(2)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # the device of this rank (gloo rehearsal: ranks may share GPUs)
    gpu = local_rank % max(1, torch.cuda.device_count()) if args.merge == "gloo" else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        # Host-side coordination only (barriers, max-over-ranks timing, the RCCL unique id):
        # gloo.  The one RCCL communicator of the process is the engine's own (prio3gpu_comm),
        # which carries the data-path collective; torch does not create a second one.
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from janus_amd import _lib
    from janus_amd._lib import check, lib
    from janus_amd.parallel import shard_range
    from janus_amd.prio3 import XOF_SHAKE128, XOF_TURBOSHAKE128, Comm, Prio3Gpu
    from oracle.ref import Prio3Ref

    kind, bits, length, chunk, label = CONFIGS[args.config]
    defaults = {"sumvec": (393216, 4096), "sum": (1 << 20, 16384), "histogram": (1 << 20, 16384),
                "count": (1 << 22, 65536)}
    B = args.reports or defaults[args.config][0]
    U = args.unique or defaults[args.config][1]
    cfg_id = f"bench-{args.config}".encode()
    import hashlib
    vk = hashlib.shake_128(b"verify-key" + cfg_id).digest(16)

    W = max(1, args.workers)
    turbo = args.xof == "turboshake128"
    xof_id = XOF_TURBOSHAKE128 if turbo else XOF_SHAKE128
    vdafs = [Prio3Gpu(kind, vk, bits=bits, length=length, chunk_length=chunk, device=gpu,
                      xof=xof_id) for _ in range(W)]
    vdaf = vdafs[0]
    s = vdaf.sizes
    engine_opts = [(o.split("=", 1)[0], int(o.split("=", 1)[1])) for o in args.opt]

    def apply_opts(v):
        for name, val in engine_opts:
            v.set_option(name, val)
        return v
    for v_ in vdafs:
        apply_opts(v_)

    # ---- synthetic inputs: B distinct reports per rank (SURVEY §8(d) recipe).  The recipe's
    # nonces / client randomness / measurements come from the C restatement (multithreaded); the
    # shares are made by the GPU client (prio3gpu_shard: Client::shard + FLP prove).  A sample is
    # checked against the C restatement's own shard before anything is timed.
    ref = Prio3Ref(kind, vk, bits, length, chunk)
    t0 = time.time()
    lo, hi = shard_range(B * world, world, rank)  # weak scaling: B reports per rank
    syn = ref.synth(cfg_id, lo, hi - lo, threads=args.gen_threads)
    d_nonces = torch.from_numpy(syn["nonces"]).to(dev)
    d_meas = torch.from_numpy(syn["meas"].view(np.int64)).to(dev)
    d_rand = torch.from_numpy(syn["rand"]).to(dev)
    d_pub = torch.empty((B, s.public_share), dtype=torch.uint8, device=dev) if s.public_share \
        else None
    # leader input shares at a row pitch (--leader-pitch; 0 = packed wire rows): what a Janus
    # caller decoding LeaderStoredReports into 128-B-aligned rows hands prio3gpu_prepare_init
    lpitch = args.leader_pitch if args.leader_pitch > 0 else s.leader_input_share
    if args.leader_pitch < 0:  # auto: the next multiple of 128 B
        lpitch = (s.leader_input_share + 127) // 128 * 128
    assert lpitch >= s.leader_input_share and lpitch % 16 == 0, "bad --leader-pitch"
    d_lin_rows = torch.empty((B, lpitch), dtype=torch.uint8, device=dev)
    d_lin = d_lin_rows[:, :s.leader_input_share]
    d_hin = torch.empty((B, s.helper_input_share), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    SC = B if lpitch == s.leader_input_share else min(B, 32768)  # shard chunk (packed: one call)
    hs0 = vdaf.new_state(1, SC)
    d_tmp = d_lin if SC == B else torch.empty((SC, s.leader_input_share), dtype=torch.uint8,
                                                device=dev)
    for c0 in range(0, B, SC):
        c1 = min(B, c0 + SC)
        vdaf.shard(hs0, d_nonces[c0:c1], d_meas[c0:c1], d_rand[c0:c1],
                   out=(d_pub[c0:c1] if d_pub is not None else None, d_tmp[:c1 - c0],
                        d_hin[c0:c1]))
        if SC != B:  # torch's stream; the next shard (engine stream) reuses d_tmp
            d_lin[c0:c1].copy_(d_tmp[:c1 - c0])
            torch.cuda.synchronize()
    del d_tmp
    hs0.close()
    del d_rand
    gen_s = time.time() - t0
    U = min(U, B)  # CPU-baseline sample size
    if turbo:
        turbo_gate = oracle_transcript_gate(vdaf, kind, bits, length, chunk, vk, syn, d_pub, d_lin,
                                            d_hin, n=2)
    else:
        chk = ref.gen(cfg_id, lo, min(U, 64), threads=args.gen_threads)
        k = chk["nonces"].shape[0]
        assert np.array_equal(d_lin[:k].cpu().numpy(), chk["leader_in"]), "GPU shard != C shard"
        assert np.array_equal(d_hin[:k].cpu().numpy(), chk["helper_in"]), "GPU shard != C shard"
        if s.public_share:
            assert np.array_equal(d_pub[:k].cpu().numpy(), chk["public"]), "GPU shard != C shard"
    d_lprep = torch.empty((B, s.prep_share), dtype=torch.uint8, device=dev)
    d_hprep = (torch.empty((B, s.prep_share), dtype=torch.uint8, device=dev) if args.overlap
               else None)
    d_msgs = torch.empty((B, max(1, s.prep_msg)), dtype=torch.uint8, device=dev)
    d_lst = torch.zeros(B, dtype=torch.uint8, device=dev)
    d_hst = torch.zeros(B, dtype=torch.uint8, device=dev)
    d_times = torch.arange(B, dtype=torch.int64, device=dev) + 1_700_000_000  # report times (s)
    torch.cuda.synchronize()

    comm = None
    rccl = world > 1 and args.merge == "rccl"
    if rccl:
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm(uid[0], world, rank, gpu)
    L = lib()
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None

    # W job workers, each with its own context (HIP stream), states and aggregates over a
    # contiguous slice of the batch; running aggregates are the batch aggregation; with N > 1 each
    # step accumulates into per-GPU partials that the RCCL merge flushes into the totals
    class Worker:
        pass

    bounds = [B * w // W for w in range(W + 1)]
    workers = []
    for w in range(W):
        wk = Worker()
        wk.v, lo, hi = vdafs[w], bounds[w], bounds[w + 1]
        wk.n = hi - lo
        # --overlap: the helper gets its own context (HIP stream), so its prepare_init runs
        # concurrently with the leader's, like two aggregator processes sharing the GPU
        wk.hv = (apply_opts(Prio3Gpu(kind, vk, bits=bits, length=length, chunk_length=chunk,
                                     device=gpu, xof=xof_id)) if args.overlap else wk.v)
        wk.ls, wk.hs = wk.v.new_state(0, wk.n), wk.hv.new_state(1, wk.n)
        wk.ls.set_input_pitch(0 if lpitch == s.leader_input_share else lpitch)
        wk.lagg, wk.hagg = wk.v.new_aggregate(1), wk.hv.new_aggregate(1)
        wk.lpart, wk.hpart = ((wk.v.new_aggregate(1), wk.hv.new_aggregate(1)) if rccl
                              else (wk.lagg, wk.hagg))
        sl = slice(lo, hi)
        wk.p = dict(nonces=P(d_nonces[sl]), pub=P(d_pub[sl]) if d_pub is not None else None,
                    lin=P(d_lin[sl]), hin=P(d_hin[sl]), lprep=P(d_lprep[sl]),
                    msgs=P(d_msgs[sl]) if s.prep_msg else None, lst=P(d_lst[sl]),
                    hst=P(d_hst[sl]), times=P(d_times[sl]),
                    hprep=P(d_hprep[sl]) if args.overlap else None)
        workers.append(wk)

    hpool = ThreadPoolExecutor(max_workers=W) if args.overlap else None
    # single process only: the multi-rank step keeps the synchronous calls around its RCCL flush
    async_calls = bool(args.async_calls) and args.overlap in (0, 1) and world == 1
    if async_calls:
        for wk in workers:
            wk.v.set_async(True)
            if wk.hv is not wk.v:
                wk.hv.set_async(True)

    def run_worker_overlap(wk):
        p, ctx, hctx = wk.p, wk.v._ctx, wk.hv._ctx
        fut = hpool.submit(L.prio3gpu_prepare_init, hctx, wk.hs._h, wk.n, p["nonces"], p["pub"],
                           p["hin"], p["hprep"], p["hst"])
        check(L.prio3gpu_prepare_init(ctx, wk.ls._h, wk.n, p["nonces"], p["pub"], p["lin"],
                                      p["lprep"], p["lst"]), "leader prepare_init")
        check(fut.result(), "helper prepare_init")
        if async_calls:  # decide reads the leader's prep shares
            wk.hv.wait_for(wk.v)
        check(L.prio3gpu_prepare_shares_to_prepare_message(hctx, wk.n, p["lprep"], p["hprep"],
                                                           p["msgs"], p["hst"]), "helper decide")
        if async_calls:  # the leader's prepare_next reads the prep messages
            wk.v.wait_for(wk.hv, wk.hv.mark())

        def helper_next():
            check(L.prio3gpu_prepare_next(hctx, wk.hs._h, wk.n, p["msgs"], p["hst"], None, None,
                                          wk.hpart._h), "helper prepare_next")
            return L.prio3gpu_agg_update_reports(wk.hpart._h, wk.n, p["nonces"], p["times"],
                                                 p["hst"], None)
        fut = hpool.submit(helper_next)
        check(L.prio3gpu_prepare_next(ctx, wk.ls._h, wk.n, p["msgs"], p["lst"], None, None,
                                      wk.lpart._h), "leader prepare_next")
        check(L.prio3gpu_agg_update_reports(wk.lpart._h, wk.n, p["nonces"], p["times"], p["lst"],
                                            None), "leader report checksums")
        check(fut.result(), "helper report checksums")

    def run_worker(wk):
        if args.overlap:
            return run_worker_overlap(wk)
        p, ctx = wk.p, wk.v._ctx
        check(L.prio3gpu_prepare_init(ctx, wk.ls._h, wk.n, p["nonces"], p["pub"], p["lin"],
                                      p["lprep"], p["lst"]), "leader prepare_init")
        check(L.prio3gpu_helper_init(ctx, wk.hs._h, wk.n, p["nonces"], p["pub"], p["hin"],
                                     p["lprep"], None, p["msgs"], p["hst"], wk.hpart._h),
              "helper_init")
        check(L.prio3gpu_agg_update_reports(wk.hpart._h, wk.n, p["nonces"], p["times"], p["hst"],
                                            None), "helper report checksums")
        check(L.prio3gpu_prepare_next(ctx, wk.ls._h, wk.n, p["msgs"], p["lst"], None, None,
                                      wk.lpart._h), "leader prepare_next")
        check(L.prio3gpu_agg_update_reports(wk.lpart._h, wk.n, p["nonces"], p["times"], p["lst"],
                                            None), "leader report checksums")

    pool = ThreadPoolExecutor(max_workers=W) if W > 1 else None

    # --overlap 2: the pipelined schedule.  Two async contexts (leader A, helper B), two leader
    # states (step i+1's XOF phase runs before step i's prepare_next).  Per step i:
    #   B waits A; B: helper XOF(i); mark mB          | A: leader query(i) (HBM) under it; mark mA
    #   A waits mB; A: leader XOF(i+1)                | B: helper query(i) (HBM) under it
    #   B waits mA; B: decide(i), prepare_next + accumulate(i), report meta; mark mB2
    #   A waits mB2; A: leader prepare_next + accumulate(i), report meta
    # Both streams are drained (and, N > 1, the partials merged) at the end of the run.
    pipe = None
    if args.overlap in (2, 3):
        assert W == 1, "--overlap 2/3 runs one job worker"
        wk = workers[0]
        A, Bv = wk.v, wk.hv
        A.set_async(True)
        Bv.set_async(True)
        ls2 = wk.v.new_state(0, wk.n)
        ls2.set_input_pitch(0 if lpitch == s.leader_input_share else lpitch)
        pipe = dict(ls=[wk.ls, ls2],
                    lst=[d_lst, torch.zeros(B, dtype=torch.uint8, device=dev)])

    def run_pipelined(k_steps):
        wk, p = workers[0], workers[0].p
        A, Bv = wk.v, wk.hv
        ls, lst = pipe["ls"], pipe["lst"]
        xof = lambda v, st, status, inp: check(L.prio3gpu_prepare_init_xof(
            v._ctx, st._h, wk.n, p["nonces"], p["pub"], inp, P(status)), "prepare_init_xof")
        query = lambda v, st, status, out: check(L.prio3gpu_prepare_init_query(
            v._ctx, st._h, wk.n, out, P(status)), "prepare_init_query")
        weights = lambda v, st, status: check(L.prio3gpu_prepare_init_weights(
            v._ctx, st._h, wk.n, P(status)), "prepare_init_weights")
        w3 = args.overlap == 3
        xof(A, ls[0], lst[0], p["lin"])
        for i in range(k_steps):
            cur, nxt = i % 2, (i + 1) % 2
            if w3:  # A's weights(i) before B's Keccak starts
                weights(A, ls[cur], lst[cur])
            Bv.wait_for(A)
            xof(Bv, wk.hs, d_hst, p["hin"])
            if w3:  # B's weights(i) before A's next Keccak starts
                weights(Bv, wk.hs, d_hst)
            mB = Bv.mark()
            query(A, ls[cur], lst[cur], p["lprep"])
            mA = A.mark()
            if i + 1 < k_steps:
                A.wait_for(Bv, mB)
                xof(A, ls[nxt], lst[nxt], p["lin"])
            query(Bv, wk.hs, d_hst, P(d_hprep2))
            Bv.wait_for(A, mA)
            check(L.prio3gpu_prepare_shares_to_prepare_message(Bv._ctx, wk.n, p["lprep"],
                                                               P(d_hprep2), p["msgs"], p["hst"]),
                  "decide")
            check(L.prio3gpu_prepare_next(Bv._ctx, wk.hs._h, wk.n, p["msgs"], p["hst"], None,
                                          None, wk.hpart._h), "helper prepare_next")
            check(L.prio3gpu_agg_update_reports(wk.hpart._h, wk.n, p["nonces"], p["times"],
                                                p["hst"], None), "helper report checksums")
            mB2 = Bv.mark()
            A.wait_for(Bv, mB2)
            check(L.prio3gpu_prepare_next(A._ctx, ls[cur]._h, wk.n, p["msgs"], P(lst[cur]), None,
                                          None, wk.lpart._h), "leader prepare_next")
            check(L.prio3gpu_agg_update_reports(wk.lpart._h, wk.n, p["nonces"], p["times"],
                                                P(lst[cur]), None), "leader report checksums")
        A.sync()
        Bv.sync()
        if comm is not None:
            comm.allreduce(A, wk.lpart, wk.lagg)
            comm.allreduce(Bv, wk.hpart, wk.hagg)

    def step():
        # the previous step's engine work (async calls on non-blocking HIP streams) reads and
        # writes these status arrays: drain the device before torch's stream resets them, and
        # again after, so the engine streams see the reset
        torch.cuda.synchronize()
        d_lst.zero_()
        d_hst.zero_()
        torch.cuda.synchronize()
        if pool is None:
            run_worker(workers[0])
        else:
            list(pool.map(run_worker, workers))
        if comm is not None:  # flush the per-GPU partials into the totals (RCCL + mod-p add)
            for wk in workers:
                comm.allreduce(wk.v, wk.lpart, wk.lagg)
                comm.allreduce(wk.hv, wk.hpart, wk.hagg)

    d_hprep2 = (torch.empty((B, s.prep_share), dtype=torch.uint8, device=dev)
                if args.overlap in (2, 3) else None)
    if pipe is not None:
        run_pipelined(max(1, args.warmup))
    else:
        for _ in range(args.warmup):
            step()
    ctxs = []
    for wk in workers:
        ctxs += [wk.v._ctx] + ([wk.hv._ctx] if wk.hv is not wk.v else [])
    for cx in ctxs:
        check(L.prio3gpu_prof_enable(cx, 1), "prof")
        L.prio3gpu_prof_read(cx, (ctypes.c_double * 64)(), (ctypes.c_uint64 * 64)(), 64)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    if pipe is not None:
        run_pipelined(args.steps)
    else:
        for _ in range(args.steps):
            step()
    barrier()
    elapsed = time.perf_counter() - t0

    def read_prof(enable_after):
        kt_ = {}
        for cx in ctxs:
            ms = (ctypes.c_double * 64)()
            nl = (ctypes.c_uint64 * 64)()
            nk = L.prio3gpu_prof_read(cx, ms, nl, 64)
            for i in range(nk):
                if nl[i]:
                    name = L.prio3gpu_prof_kernel_name(i).decode()
                    a, b = kt_.get(name, (0.0, 0))
                    kt_[name] = (a + ms[i], b + nl[i])
            check(L.prio3gpu_prof_enable(cx, 1 if enable_after else 0), "prof")
        return kt_

    # HIP-event spans of the timed schedule: with two contexts co-running (--overlap >= 1) a
    # kernel's span also covers the time it waited behind, or shared the CUs with, the other
    # context's kernel, so these are spans, not kernel durations
    kt_timed = read_prof(args.prof_steps > 0)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert int(d_lst.max().item()) == 0 and int(d_hst.max().item()) == 0, "rejected reports"
    if pipe is not None:
        assert int(pipe["lst"][1].max().item()) == 0, "rejected reports"
    if pipe is not None or async_calls:
        for wk in workers:
            for v_ in (wk.v, wk.hv):
                v_.set_async(False)

    # ---- serial kernel pass (untimed): the same calls, each synchronous, one after the other
    # from one thread, so no two kernels share the GPU and each HIP-event span is the kernel's
    # own duration -- the durations rocprofv3 reports for the same kernels (its PMC passes
    # serialise dispatches).  The roofline and kernels_ms_per_step come from this pass.
    def serial_step():
        torch.cuda.synchronize()
        d_lst.zero_()
        d_hst.zero_()
        torch.cuda.synchronize()
        for wk in workers:
            p, ctx, hctx = wk.p, wk.v._ctx, wk.hv._ctx
            if wk.hv is wk.v:
                run_worker(wk)
                continue
            check(L.prio3gpu_prepare_init(ctx, wk.ls._h, wk.n, p["nonces"], p["pub"], p["lin"],
                                          p["lprep"], p["lst"]), "leader prepare_init")
            check(L.prio3gpu_prepare_init(hctx, wk.hs._h, wk.n, p["nonces"], p["pub"], p["hin"],
                                          p["hprep"], p["hst"]), "helper prepare_init")
            check(L.prio3gpu_prepare_shares_to_prepare_message(hctx, wk.n, p["lprep"], p["hprep"],
                                                               p["msgs"], p["hst"]), "decide")
            check(L.prio3gpu_prepare_next(hctx, wk.hs._h, wk.n, p["msgs"], p["hst"], None, None,
                                          wk.hpart._h), "helper prepare_next")
            check(L.prio3gpu_agg_update_reports(wk.hpart._h, wk.n, p["nonces"], p["times"],
                                                p["hst"], None), "helper report checksums")
            check(L.prio3gpu_prepare_next(ctx, wk.ls._h, wk.n, p["msgs"], p["lst"], None, None,
                                          wk.lpart._h), "leader prepare_next")
            check(L.prio3gpu_agg_update_reports(wk.lpart._h, wk.n, p["nonces"], p["times"],
                                                p["lst"], None), "leader report checksums")
        torch.cuda.synchronize()
        if comm is not None:
            for wk in workers:
                comm.allreduce(wk.v, wk.lpart, wk.lagg)
                comm.allreduce(wk.hv, wk.hpart, wk.hagg)

    serial_el = None
    if args.prof_steps > 0:
        barrier()
        ts0 = time.perf_counter()
        for _ in range(args.prof_steps):
            serial_step()
        barrier()
        serial_el = time.perf_counter() - ts0
        kt = read_prof(False)
        assert int(d_lst.max().item()) == 0 and int(d_hst.max().item()) == 0, "rejected reports"
    else:
        kt = kt_timed
    kt_steps = args.prof_steps if args.prof_steps > 0 else args.steps

    # ---- parity gate: statuses, counts, aggregate == plaintext sum (and == CPU restatement) ------
    total_steps = ((max(1, args.warmup) if pipe is not None else args.warmup) + args.steps
                   + max(0, args.prof_steps))
    def total(attr):  # merge the workers' aggregates (mod p) and counts
        acc, cnt = None, 0
        for wk in workers:
            a, c = getattr(wk, attr).read(0)
            vec = vdaf.decode_field_vec(a)
            acc = vec if acc is None else [(x + y) % vdaf.modulus for x, y in zip(acc, vec)]
            cnt += c
        return b"".join(int(x).to_bytes(s.field_size, "little") for x in acc), cnt

    la, lc = total("lagg")
    ha, hc = total("hagg")
    if dist is not None and not rccl:  # gloo rehearsal: merge the ranks' aggregates on the host
        for which in ("l", "h"):
            mine = (la, lc) if which == "l" else (ha, hc)
            allv = [None] * world
            dist.all_gather_object(allv, mine)
            acc = [0] * (len(mine[0]) // s.field_size)
            for b, _ in allv:
                acc = [(x + y) % vdaf.modulus for x, y in zip(acc, vdaf.decode_field_vec(b))]
            merged = (b"".join(int(x).to_bytes(s.field_size, "little") for x in acc),
                      sum(c for _, c in allv))
            if which == "l":
                la, lc = merged
            else:
                ha, hc = merged
    exp_count = total_steps * B * world
    assert lc == exp_count and hc == exp_count, (lc, hc, exp_count)
    meas = syn["meas"]
    if kind == 2:
        plain = [int(x) * total_steps for x in meas.sum(axis=0, dtype=np.uint64)]
    elif kind == 3:
        plain = [int((meas[:, 0] == i).sum()) * total_steps for i in range(length)]
    else:
        plain = int(meas[:, 0].sum()) * total_steps
    if dist is not None:  # every rank holds the merged totals: compare with all ranks' plaintext
        allp = [None] * world
        dist.all_gather_object(allp, plain)
        plain = [sum(col) for col in zip(*allp)] if isinstance(plain, list) else sum(allp)
    assert vdaf.unshard([la, ha]) == plain, "aggregate != plaintext sum"
    # report bookkeeping (Accumulator::update): interval of the report times, and at N = 1 the
    # ReportIdChecksum against hashlib (each report was accumulated total_steps times: XOR parity)
    for attr in ("lagg", "hagg"):
        cks = [getattr(wk, attr).read_reports(0) for wk in workers]
        assert all(iv == (1_700_000_000, wk.n if W > 1 else B) or W > 1 for _, iv in cks)
        if world == 1 and W == 1:
            import hashlib
            nz = d_nonces.cpu().numpy()
            dg = np.frombuffer(b"".join(hashlib.sha256(nz[i].tobytes()).digest() for i in range(B)),
                               np.uint8).reshape(B, 32)
            x = np.bitwise_xor.reduce(dg, axis=0) if total_steps % 2 else np.zeros(32, np.uint8)
            assert cks[0][0] == x.tobytes(), "report-ID checksum != SHA-256 XOR"

    # byte-level gate: the first G reports of this rank through the same GPU path
    # (leader prepare_init, helper_init, leader prepare_next + accumulate) and through the C
    # restatement of prio 0.15.1: both aggregators' aggregate-share bytes and counts identical.
    G = min(U, B)
    nthr = cpu_threads(args.cpu_threads)
    if turbo:  # the C restatement is SHAKE128-only: the Python-oracle transcript gate above
        parity = (f"{turbo_gate}; unshard(aggregate) == plaintext sum over every timed step; "
                  f"report-ID checksums == hashlib; status all ok (XofTurboShake128: parity "
                  f"unpinned beyond the oracle)")
    else:
        cn = d_nonces[:G].cpu().numpy()
        cp = d_pub[:G].cpu().numpy() if d_pub is not None else np.zeros((G, 0), np.uint8)
        cl = d_lin[:G].cpu().numpy()
        ch = d_hin[:G].cpu().numpy()
        gv = workers[0].v
        gls, ghs = gv.new_state(0, G), gv.new_state(1, G)
        glagg, ghagg = gv.new_aggregate(1), gv.new_aggregate(1)
        gpub = d_pub[:G] if d_pub is not None else None
        glp, glst = gv.prepare_init(gls, d_nonces[:G], gpub, d_lin[:G])
        gmsgs, ghst = gv.helper_init(ghs, d_nonces[:G], gpub, d_hin[:G], glp, agg=ghagg)
        gout = gv.prepare_next(gls, gmsgs, glst, want_output_shares=True, agg=glagg)
        if isinstance(gout, tuple):
            gout = gout[0]
        ref_res = ref.prepare_batch(cn, cp, cl, ch, threads=nthr, outputs=True)
        (gla, glc), (gha, ghc) = glagg.read(0), ghagg.read(0)
        assert glc == ghc == ref_res["count"] == G, (glc, ghc, ref_res["count"], G)
        assert gla == ref_res["agg_l"].tobytes(), "leader aggregate share != C restatement"
        assert gha == ref_res["agg_h"].tobytes(), "helper aggregate share != C restatement"
        # sampled prep shares, prep messages and output shares byte-equal too
        assert (ref_res["status"] == 0).all() and (glst == 0).all() and (ghst == 0).all()
        assert np.array_equal(glp, ref_res["lprep"]), "leader prep shares != C restatement"
        ghs2 = gv.new_state(1, G)
        ghp, _ = gv.prepare_init(ghs2, d_nonces[:G], gpub, d_hin[:G])
        ghs2.close()
        assert np.array_equal(ghp, ref_res["hprep"]), "helper prep shares != C restatement"
        if s.prep_msg:
            assert np.array_equal(np.asarray(gmsgs)[:, :s.prep_msg], ref_res["msgs"]), \
                "prep messages != C restatement"
        no = min(G, 64)
        assert np.array_equal(np.asarray(gout)[:no], leader_output_shares(cl[:no], kind, bits, length, s,
                                                                          vdaf.modulus)), \
            "leader output shares != truncate(leader measurement share)"
        for o in (gls, ghs, glagg, ghagg):
            o.close()
        parity = (f"aggregate-share bytes == C restatement (both aggregators, {G} reports/rank "
                  f"through the product path); leader and helper prep shares and prep messages of "
                  f"those {G} reports == C restatement; leader output shares of {no} == truncate(meas "
                  f"share); unshard(aggregate) == plaintext sum over every timed step; report-ID "
                  f"checksums == hashlib; status all ok")

    # ---- helper-only variant (the A1 path alone: helper_init + bookkeeping), SURVEY §8(d) -------
    helper_only = None
    if args.helper_only:
        wk = workers[0]
        p = wk.p
        hagg2 = wk.hv.new_aggregate(1)

        def hstep():
            d_hst.zero_()
            check(L.prio3gpu_helper_init(wk.hv._ctx, wk.hs._h, wk.n, p["nonces"], p["pub"],
                                         p["hin"], p["lprep"], None, p["msgs"], p["hst"],
                                         hagg2._h), "helper_init")
            check(L.prio3gpu_agg_update_reports(hagg2._h, wk.n, p["nonces"], p["times"], p["hst"],
                                                None), "helper report checksums")
        hstep()
        barrier()
        th0 = time.perf_counter()
        for _ in range(args.steps):
            hstep()
        barrier()
        h_el = time.perf_counter() - th0
        if dist is not None:
            t = torch.tensor([h_el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            h_el = float(t.item())
        assert int(d_hst.max().item()) == 0 and hagg2.read(0)[1] == (args.steps + 1) * wk.n
        helper_only = {"value": round(args.steps * wk.n * world / h_el, 2), "unit": "reports/s",
                       "ms_per_step": round(h_el / args.steps * 1e3, 3),
                       "what": "helper aggregate-init alone (prepare_init + decide + prepare_next "
                               "+ accumulate + report checksums), leader prep shares precomputed"}
        hagg2.close()

    reports = args.steps * B * world
    value = reports / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- roofline of the dominant kernel (HIP events on the engine's stream) -------------------
    perms = perms_per_report(args.config, s)
    dom = max(kt.items(), key=lambda kv: kv[1][0])
    dname, (dms, dlaunch) = dom
    avg_launch_s = dms / 1e3 / dlaunch
    # B / W reports per launch; k_jr runs once per aggregator and worker (2 W launches per step)
    nlaunch = bounds[1] - bounds[0]
    # the PMC passes profile the SHAKE128 build of the command; a TurboSHAKE128 permutation is the
    # last 12 of Keccak-f's 24 rounds: half the ops, twice the measured ceiling rate
    # (tools/profile_round.sh profiles the default command: its per-launch bytes only describe
    # launches of the default batch size)
    pmc = load_pmc(args.config) if not turbo and B == defaults[args.config][0] else {}
    rf = 0.5 if turbo else 1.0
    if dname in perms and perms[dname]:
        ops = perms[dname] * nlaunch * OPS_PER_PERM * rf
        achieved = ops / avg_launch_s / 1e12
        perm_rate = perms[dname] * nlaunch / avg_launch_s
        roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_TOPS, 1),
                "unit": "Tops/s", "frac": round(achieved / VALU_PEAK_TOPS, 4), "traffic": None,
                "kernel": dname, "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                "model": (f"{perms[dname]} Keccak-f[1600]/report x {OPS_PER_PERM} int32 ops "
                          f"(SURVEY §8(d)) x {nlaunch} reports/launch" if not turbo else
                          f"{perms[dname]} Keccak-p[1600,12]/report x {OPS_PER_PERM // 2} int32 "
                          f"ops (half of SURVEY §8(d)'s 24-round figure) x {nlaunch} "
                          f"reports/launch"),
                "keccak_perms_per_s": round(perm_rate, 1),
                # vs the measured register-only Keccak-f ceiling of this chip (tools/mb_keccak_occ.hip)
                "keccak_ceiling_perms_per_s": KECCAK_CEILING / rf,
                "keccak_ceiling_frac": round(perm_rate * rf / KECCAK_CEILING, 4),
                "algorithmic_hbm_bytes_per_launch": (
                    nlaunch * s.meas_len * s.field_size if dname == "k_jr" else
                    nlaunch * (s.meas_len + s.proof_len) * s.field_size if dname == "k_expand"
                    else None)}
    elif dname == "k_flp_query_lane":  # the whole FLP query of Count / Sum in one kernel
        mults = flp_mults_per_report(s, kind)
        per_mul = OPS_PER_F128_MUL if s.field_size == 16 else OPS_PER_F64_MUL
        # Count's launch also derives the query randomness (one Keccak-f per report)
        qperm = 1 if args.config == "count" else 0
        ops = (mults * per_mul + qperm * OPS_PER_PERM * rf) * nlaunch
        achieved = ops / avg_launch_s / 1e12
        roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_TOPS, 1),
                "unit": "Tops/s", "frac": round(achieved / VALU_PEAK_TOPS, 4), "traffic": None,
                "kernel": dname, "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                "model": (f"{mults} {'F128' if s.field_size == 16 else 'F64'} mults/report "
                          f"(prio-style FLP query, SURVEY §8(d)) x {per_mul} int32 ops"
                          + (f" + {qperm} Keccak-f/report (query randomness) x "
                             f"{int(OPS_PER_PERM * rf)} ops" if qperm else "")
                          + f" x {nlaunch} reports/launch")}
    else:
        roof = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK_TOPS, 1),
                "unit": "Tops/s", "frac": None, "traffic": None, "kernel": dname,
                "avg_launch_ms": round(avg_launch_s * 1e3, 3)}
    roof["avg_launch_ms_source"] = ("serial kernel pass" if args.prof_steps > 0
                                    else "timed steps")
    if dname in kt_timed and kt_timed[dname][1]:
        roof["avg_launch_ms_timed_span"] = round(kt_timed[dname][0] / kt_timed[dname][1], 3)
    pm = pmc.get("kernels", {}).get(dname)
    if pm:  # PMC passes of the same command (tools/profile_round.sh), per launch
        roof["traffic"] = pm.get("hbm_bytes_per_launch")
        roof["pmc_source"] = pmc["source"]
        if roof.get("achieved") and pm.get("avg_ms"):
            # the same op model over rocprofv3's average duration of this kernel
            roof["pmc_avg_ms"] = round(pm["avg_ms"], 3)
            roof["frac_from_pmc_avg_ms"] = round(
                roof["frac"] * roof["avg_launch_ms"] / pm["avg_ms"], 4)
        if pm.get("SQ_INSTS_VALU"):
            # wave-instructions issued / (launch time x the chip's VALU issue rate)
            roof["valu_issue_frac"] = round(pm["SQ_INSTS_VALU"] / (pm["avg_ms"] / 1e3)
                                            / VALU_ISSUE_PEAK, 4)
            if dname in perms and perms[dname]:
                roof["valu_insts_per_perm"] = round(pm["valu_insts_per_wave"] / perms[dname], 1)
    # the HBM-bound kernel of the step: the FLP wire pass streams each measurement share once
    hbm_k = "k_flp_wires_mfma" if kt.get("k_flp_wires_mfma", (0, 0))[1] else "k_flp_wires"
    if hbm_k in kt and kt[hbm_k][1]:
        hms, hl = kt[hbm_k]
        h_avg = hms / 1e3 / hl
        alg = nlaunch * flp_wires_bytes_per_report(s, hbm_k == "k_flp_wires_mfma")
        hb = {"kernel": hbm_k, "avg_launch_ms": round(h_avg * 1e3, 3),
              "algorithmic_bytes_per_launch": alg,
              "achieved": round(alg / h_avg / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(alg / h_avg / 1e9 / HBM_PEAK_GBS, 4),
              # MI355X_MICROARCH.md: 6.29 TB/s measured for a float4 copy (79 % of the spec)
              "frac_of_measured_copy": round(alg / h_avg / 1e9 / HBM_COPY_GBS, 4),
              "traffic": None}
        hp = pmc.get("kernels", {}).get(hbm_k)
        if hp and hp.get("hbm_bytes_per_launch"):
            hb["traffic"] = hp["hbm_bytes_per_launch"]
            hb["traffic_over_algorithmic"] = round(hp["hbm_bytes_per_launch"] / alg, 3)
        roof["hbm"] = hb
    # the weights kernel beside it: its HBM line, PMC traffic per launch
    if kt.get("k_flp_weights", (0, 0))[1]:
        wms, wl = kt["k_flp_weights"]
        w_avg = wms / 1e3 / wl
        walg = nlaunch * flp_weights_bytes_per_report(s)
        wline = {"kernel": "k_flp_weights", "avg_launch_ms": round(w_avg * 1e3, 3),
                 "algorithmic_bytes_per_launch": walg,
                 "achieved": round(walg / w_avg / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(walg / w_avg / 1e9 / HBM_PEAK_GBS, 4), "traffic": None}
        wp = pmc.get("kernels", {}).get("k_flp_weights")
        if wp and wp.get("hbm_bytes_per_launch"):
            wline["traffic"] = wp["hbm_bytes_per_launch"]
            wline["traffic_over_algorithmic"] = round(wp["hbm_bytes_per_launch"] / walg, 3)
        roof["hbm_weights"] = wline

    # ---- CPU baseline: C restatement of prio 0.15.1, bounded sample, rank 0 at N = 1 -----------
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline and not turbo:
        done, t0 = 0, time.perf_counter()
        while True:
            res = ref.prepare_batch(cn, cp, cl, ch, threads=nthr, outputs=False)
            assert res["count"] == G
            done += G
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        cpu_s = time.perf_counter() - t0
        # one thread: Janus's per-report loop inside one aggregation job (aggregator.rs:1613)
        n1 = min(G, 256)
        done1, t1 = 0, time.perf_counter()
        while True:
            r1 = ref.prepare_batch(cn[:n1], cp[:n1], cl[:n1], ch[:n1], threads=1, outputs=False)
            assert r1["count"] == n1
            done1 += n1
            if time.perf_counter() - t1 >= max(2.0, args.cpu_seconds / 4):
                break
        cpu1_s = time.perf_counter() - t1
        # the CPU restatement's aggregate over the sample == plaintext sum of the sample
        sm = syn["meas"][:G]
        if kind == 2:
            sp = [int(x) for x in sm.sum(axis=0, dtype=np.uint64)]
        elif kind == 3:
            sp = [int((sm[:, 0] == i).sum()) for i in range(length)]
        else:
            sp = int(sm[:, 0].sum())
        assert vdaf.unshard([res["agg_l"].tobytes(), res["agg_h"].tobytes()]) == sp
        cpu = {"value": round(done / cpu_s, 2), "unit": "reports/s", "cores": nthr,
               "kind": "port",
               "one_thread": round(done1 / cpu1_s, 2),
               # a whole 8-GPU host (e.g. 256 CPUs) gives each GPU more CPUs than this box's
               # cgroup share: the speedup at a host's per-GPU CPU count, scaled linearly from
               # the measured rate, is `value` x cpus_per_gpu_on_host / cores
               "cpus_per_gpu_on_host_8gpu": (os.cpu_count() or 0) // 8,
               "cpu_model": cpu_model(),
               "host_cpus": host_cpu_info(),
               "sample": f"{done} report preparations ({G} distinct reports, repeated) leader+helper "
                         f"prepare+aggregate on {nthr} threads in {cpu_s:.1f} s, and {done1} on "
                         f"1 thread in {cpu1_s:.1f} s; C restatement of prio 0.15.1 (the "
                         f"reference's Rust path is not buildable here)"}

    # ---- HPKE open on host threads (excluded from `value`, reported separately: SURVEY §8(d)) --
    hpke_rep = None
    if rank == 0 and world == 1 and args.hpke:
        from janus_amd import codec as C
        from janus_amd import hpke as H
        nh = min(U, 8192)
        kp = H.generate_hpke_config_and_private_key(1)
        info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
        hn = d_nonces[:nh].cpu().numpy()
        hp = d_pub[:nh].cpu().numpy() if d_pub is not None else np.zeros((nh, 0), np.uint8)
        hh = d_hin[:nh].cpu().numpy()
        task_id = bytes(32)
        cts = [H.seal(kp.config, info, b"\0\0" + len(hh[i]).to_bytes(4, "big") + hh[i].tobytes(),
                      H.input_share_aad(task_id, hn[i].tobytes(), 0, hp[i].tobytes()))
               for i in range(nh)]
        req = C.decode_agg_init_req(C.encode_agg_init_req(
            C.TIME_INTERVAL, None, b"", hn, [0] * nh, hp, cts, np.zeros((nh, s.prep_share), np.uint8)))
        H.open_report_shares(task_id, req, [kp], [], None, nthr)  # warm
        t0 = time.perf_counter()
        reps = 0
        while True:
            pts, offs, hst = H.open_report_shares(task_id, req, [kp], [], None, nthr)
            reps += 1
            if time.perf_counter() - t0 > 2.0:
                break
        hs_dt = time.perf_counter() - t0
        assert (hst == 0).all()
        hin2, hst = C.decode_plaintext_input_shares_raw(s, pts, offs, 1, hst)
        assert (hst == 0).all() and np.array_equal(hin2, hh)
        hpke_rep = {"value": round(reps * nh / hs_dt, 1), "unit": "helper input shares opened/s",
                    "threads": nthr, "suite": "X25519HkdfSha256/HkdfSha256/Aes128Gcm",
                    "sample": f"{nh} helper input shares x {reps}",
                    "note": "CPU stage in front of the GPU path (north star); not in `value`"}

    out = {
        "metric": (METRIC if args.config == "sumvec" and not turbo else
                   f"reports/sec prepared+aggregated, {label}" + (", XofTurboShake128" if turbo
                                                                  else "")),
        "value": round(value, 2),
        "unit": "reports/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u128 (Field128 mod p)" if s.field_size == 16 else "u64 (Field64 mod p)",
        "data": f"synthetic: {B} distinct reports/GPU (SURVEY §8(d) recipe; shares made by the GPU "
                f"client shard), resident in HBM",
        "config": {"workload": label, "xof": "XofTurboShake128" if turbo else "XofShake128",
                   "engine_options": dict(engine_opts),
                   "schedule": f"overlap {args.overlap}" + (", async calls" if async_calls else ""),
                   "reports_per_gpu_per_step": B, "job_workers_per_gpu": W,
                   "parallelism": f"report-sharded x{world}, {W} job stream(s)/GPU, "
                                  + ("RCCL all-gather merge" if args.merge == "rccl" else
                                     "gloo rehearsal (ranks share GPUs, host merge)")},
        "roofline": roof,
        "cpu_baseline": cpu,
        "hpke_open": hpke_rep,
        "helper_only": helper_only,
        # each kernel's own duration per step, from the serial kernel pass (one kernel on the GPU
        # at a time): sums to the serial pass's kernel time, <= its ms_per_step
        "kernels_ms_per_step": {k: round(v[0] / kt_steps, 3) for k, v in kt.items()},
        "kernels_source": (f"serial kernel pass, {args.prof_steps} untimed steps after the timed "
                           f"region (synchronous calls, one kernel on the GPU at a time)"
                           if args.prof_steps > 0 else "HIP-event spans of the timed steps"),
        "serial_pass": ({"steps": args.prof_steps,
                         "ms_per_step": round(serial_el / args.prof_steps * 1e3, 3),
                         "kernel_ms_per_step": round(sum(v[0] for v in kt.values()) / kt_steps, 3)}
                        if serial_el else None),
        # HIP-event spans in the timed (possibly co-running) schedule: a span includes time spent
        # queued behind or sharing the CUs with the other context's kernels
        "kernels_timed_span_ms_per_step": {k: round(v[0] / args.steps, 3)
                                           for k, v in kt_timed.items()},
        "parity": parity,
        "gen_seconds": round(gen_s, 1),
        # the engine build that ran: SHA-256 of its sources + flags (janus_amd/_lib.py)
        "build_hash": L.prio3gpu_build_hash().decode(),
    }
    if cpu:
        out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        fair = cpu.get("cpus_per_gpu_on_host_8gpu") or 0
        if fair > cpu["cores"]:  # the same speedup against a linearly scaled fair CPU share
            out["speedup_vs_cpu_at_host_share"] = round(value / (cpu["value"] * fair / cpu["cores"]), 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
