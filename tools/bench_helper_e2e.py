"""End-to-end helper aggregate-init throughput on one GPU (SURVEY §8(a) A1 with its host stages):
AggregationJobInitializeReq bytes in -> batched decode -> HPKE open of every helper input share on
host threads -> GPU prepare_init + decide + prepare_next + accumulate -> AggregationJobResp bytes
out, pipelined over jobs by HelperAggregateInit.handle_jobs (decode + HPKE of job k+1 on the host
while the GPU prepares job k).  Prio3SumVec(8, 1000, 89).  Inputs: seeded random nonces, client
randomness and measurements, shares from the GPU client shard, leader prep shares from the GPU leader prepare_init, helper shares sealed to
one X25519/HKDF-SHA256/AES-128-GCM key -- all made before timing.

  python tools/bench_helper_e2e.py --jobs 8 --job-size 16384 --threads 16
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from janus_amd import codec as C  # noqa: E402
from janus_amd import hpke as H  # noqa: E402
from janus_amd.helper import HelperAggregateInit  # noqa: E402
from janus_amd.prio3 import Prio3Gpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--job-size", type=int, default=16384)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    kind, bits, length, chunk, label = CONFIGS["sumvec"]
    cfg_id = b"bench-sumvec"
    vk = hashlib.shake_128(b"verify-key" + cfg_id).digest(16)
    v = Prio3Gpu(kind, vk, bits=bits, length=length, chunk_length=chunk, device=0)
    s = v.sizes
    M, J = args.job_size, args.jobs
    rng = np.random.default_rng(2024)
    tk = H.generate_hpke_config_and_private_key(7)
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
    task_id = hashlib.sha256(b"e2e task").digest()
    t0 = time.time()
    reqs, job_nonces = [], []
    ls = v.new_state(0, M)
    hs0 = v.new_state(1, M)
    for j in range(J):
        nonces = rng.integers(0, 256, (M, 16), dtype=np.uint8)
        d_nonces = torch.from_numpy(nonces).to(dev)
        d_meas = torch.from_numpy(rng.integers(0, 1 << bits, (M, length), dtype=np.int64)).to(dev)
        d_rand = torch.from_numpy(rng.integers(0, 256, (M, v.random_size()), dtype=np.uint8)).to(dev)
        d_pub = torch.empty((M, s.public_share), dtype=torch.uint8, device=dev)
        d_lin = torch.empty((M, s.leader_input_share), dtype=torch.uint8, device=dev)
        d_hin = torch.empty((M, s.helper_input_share), dtype=torch.uint8, device=dev)
        v.shard(hs0, d_nonces, d_meas, d_rand, out=(d_pub, d_lin, d_hin))
        lp, lst = v.prepare_init(ls, d_nonces, d_pub, d_lin)
        assert (lst == 0).all()
        pub, hin = d_pub.cpu().numpy(), d_hin.cpu().numpy()
        job_nonces.append(nonces)
        times = [1_700_000_000 + (j * M + i) % 3600 for i in range(M)]
        cts = []
        for i in range(M):
            pt = b"\0\0" + len(hin[i]).to_bytes(4, "big") + hin[i].tobytes()
            aad = H.input_share_aad(task_id, nonces[i].tobytes(), times[i], pub[i].tobytes())
            cts.append(H.seal(tk.config, info, pt, aad))
        reqs.append(C.encode_agg_init_req(C.TIME_INTERVAL, None, b"", nonces, times, pub, cts, lp))
        del d_lin, d_rand, d_meas
    ls.close()
    hs0.close()
    gen_s = time.time() - t0
    drv = HelperAggregateInit(v, task_id, [tk], hpke_threads=args.threads)
    agg = v.new_aggregate(1)
    drv.handle_jobs(reqs[:1], agg)  # warm (allocates the state)
    agg = v.new_aggregate(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        resps = drv.handle_jobs(reqs, agg)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = J * M * args.reps
    for j, resp in enumerate(resps):
        _, st = C.gather_helper_resps(s, resp, job_nonces[j], np.zeros(M, np.uint8))
        assert (st == 0).all(), f"job {j}: {int((st != 0).sum())} reports rejected"
    _, cnt = agg.read(0)
    assert cnt == n, (cnt, n)
    # unpipelined per-stage times of one job (host stages one by one, then the GPU stage)
    stages = {}
    req = C.decode_agg_init_req(reqs[0])
    t = time.perf_counter()
    req = C.decode_agg_init_req(reqs[0])
    stages["decode_req"] = time.perf_counter() - t
    t = time.perf_counter()
    C.check_agg_init_req(req)
    nonces_, pub_, lps_, faults_ = C.gather_prepare_inits(s, req)
    stages["check_gather"] = time.perf_counter() - t
    t = time.perf_counter()
    pts, offs, st_ = H.open_report_shares(task_id, req, [tk], [], None, args.threads)
    stages["hpke_open"] = time.perf_counter() - t
    t = time.perf_counter()
    C.decode_plaintext_input_shares_raw(s, pts, offs, 1, st_)
    stages["decode_plaintext"] = time.perf_counter() - t
    t = time.perf_counter()
    o = drv.open(reqs[0])
    stages["open_total"] = time.perf_counter() - t
    a2 = v.new_aggregate(1)
    t = time.perf_counter()
    drv.prepare(o, a2)
    torch.cuda.synchronize()
    stages["prepare_gpu_encode"] = time.perf_counter() - t
    stages = {k: round(x * 1e3, 2) for k, x in stages.items()}
    drv.close()
    print(json.dumps({
        "what": "helper aggregate-init end to end: request bytes -> decode -> HPKE open (host "
                "threads) -> GPU prepare+decide+prepare_next+accumulate -> response bytes, "
                "pipelined over jobs",
        "value": round(n / dt, 1), "unit": "reports/s", "jobs": J, "job_size": M,
        "reps": args.reps, "hpke_threads": args.threads, "seconds": round(dt, 3),
        "request_mb_per_job": round(len(reqs[0]) / 1e6, 1), "gen_seconds": round(gen_s, 1),
        "workload": label, "stage_ms_per_job": stages}))


if __name__ == "__main__":
    main()
