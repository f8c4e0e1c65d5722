"""Batched leader aggregate-init driver (janus_amd/leader.py) against Janus's
step_aggregation_job_aggregate_init / process_response_from_helper
(aggregator/src/aggregator/aggregation_job_driver.rs:290-437, :530-727)."""
import os

import numpy as np
import pytest

from janus_amd import codec as C
from janus_amd import hpke as H


def _sizes(**kw):
    from janus_amd.prio3 import _Sizes
    s = _Sizes()
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def test_packed_request_encoder_matches_list_encoder():
    """encode_agg_init_req_packed == encode_agg_init_req (the list form pinned by the reference's
    message KATs in test_codec.py), with reports that failed leader preparation left out."""
    from janus_amd.leader import LeaderJob
    rng = np.random.default_rng(5)
    n = 7
    nonces = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    pub = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    prep = rng.integers(0, 256, (n, 48), dtype=np.uint8)
    times = [1000 + 3 * i for i in range(n)]
    cts = [(i % 3, os.urandom(32), os.urandom(10 + i)) for i in range(n)]
    st = np.array([0, 5, 0, 0, 8, 0, 2], np.uint8)
    ref = C.encode_agg_init_req(C.TIME_INTERVAL, None, b"", nonces, times, pub, cts, prep, st)
    ids, eb, eo, pb, po = LeaderJob.pack_ciphertexts(cts)
    got = C.encode_agg_init_req_packed(C.TIME_INTERVAL, None, b"", nonces, times, pub, ids, eb,
                                       eo, pb, po, prep, st)
    assert got == ref
    d = C.decode_agg_init_req(got)
    assert d.n == 4 and d.times().tolist() == [times[i] for i in (0, 2, 3, 5)]
    with pytest.raises(ValueError):
        C.encode_agg_init_req_packed(C.TIME_INTERVAL, None, b"", nonces, times[:-1], pub, ids, eb,
                                     eo, pb, po, prep, st)


def test_leader_response_must_answer_sent_reports_in_order():
    """process_response_from_helper: a response that skips, repeats or reorders the sent reports
    fails the whole job (aggregation_job_driver.rs:556-573); Reject(e) passes e through; a
    Finished result while the leader is not finished is VdafPrepError (:632-664)."""
    from janus_amd import messages as M
    nonces = np.arange(48, dtype=np.uint8).reshape(3, 16)
    msgs = np.full((3, 16), 7, np.uint8)
    sz = _sizes(prep_msg=16)
    resp = C.encode_agg_job_resp(nonces, msgs, 16, np.array([0, 4, 0], np.uint8))
    pm, st = C.gather_helper_resps(sz, resp, nonces, np.zeros(3, np.uint8))
    assert st.tolist() == [0, 4, 0] and (pm[0] == 7).all()
    # report 1 was not sent (failed at the leader): the two answers map to reports 0 and 2
    resp2 = C.encode_agg_job_resp(nonces[[0, 2]], msgs[[0, 2]], 16, np.zeros(2, np.uint8))
    pm, st = C.gather_helper_resps(sz, resp2, nonces, np.array([0, 5, 0], np.uint8))
    assert st.tolist() == [0, 5, 0]
    for bad in (resp2, C.encode_agg_job_resp(nonces[[2, 0, 1]], msgs, 16, np.zeros(3, np.uint8))):
        with pytest.raises(Exception):
            C.gather_helper_resps(sz, bad, nonces, np.zeros(3, np.uint8))
    # PrepareStepResult::Finished (result 1) for a leader that has not finished
    fin = b"".join(nonces[i].tobytes() + b"\x01" for i in range(3))
    resp3 = len(fin).to_bytes(4, "big") + fin
    _, st = C.gather_helper_resps(sz, resp3, nonces, np.zeros(3, np.uint8))
    assert st.tolist() == [5, 5, 5]
    assert M is not None


def _leader_setup(name, n):
    from janus_amd.leader import LeaderJob
    from janus_amd.prio3 import Prio3Gpu
    from tests.reports import CONFIGS, make_batch
    b = make_batch(name, n)
    c = CONFIGS[name]
    mk = lambda: Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                          chunk_length=c["chunk"])
    task_id = os.urandom(32)
    tk = H.generate_hpke_config_and_private_key(3)
    info = H.application_info(H.Label.INPUT_SHARE, H.ROLE_CLIENT, H.ROLE_HELPER)
    times = np.arange(1000, 1000 + b.n, dtype=np.uint64)
    cts = []
    for r in range(b.n):
        pt = b"\x00\x00" + len(b.helper_in[r]).to_bytes(4, "big") + b.helper_in[r].tobytes()
        aad = H.input_share_aad(task_id, b.nonces[r].tobytes(), int(times[r]),
                                b.public[r].tobytes())
        cts.append(H.seal(tk.config, info, pt, aad))
    return b, mk, task_id, tk, times, cts, LeaderJob


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["sumvec_small", "hist256"])
def test_leader_driver_round_trip_with_helper(name):
    """Three jobs through LeaderAggregateInit.run_jobs (pinned staging, H2D of job k+1 under the
    GPU work of job k, helper round trip of job k under job k+1) against the helper driver
    (HPKE open + prio3gpu_helper_init) on its own context: per-report statuses follow Janus's
    leader rules and both aggregates equal the oracle's over the finished reports."""
    from janus_amd.helper import HelperAggregateInit
    from janus_amd.leader import LeaderAggregateInit
    from tests.reports import expected_aggregate
    b, mk, task_id, tk, times, cts, LeaderJob = _leader_setup(name, 30)
    cts[4] = (cts[4][0], cts[4][1], cts[4][2][:-1] + bytes([cts[4][2][-1] ^ 1]))  # helper: bad tag
    present = np.ones(b.n, bool)
    present[11] = False              # garbage-collected client report -> ReportDropped
    dup = np.zeros(b.n, bool)
    dup[17] = True                   # repeated leader extension -> InvalidMessage
    lin_bad = b.leader_in.copy()
    lin_bad[23, :16] = 0xFF          # non-canonical leader measurement share -> InvalidMessage
    lv, hv = mk(), mk()
    drv = LeaderAggregateInit(lv)
    jobs = []
    for j in (slice(0, 10), slice(10, 20), slice(20, 30)):
        k = j.stop - j.start
        pin = drv.pinned(k, lv.sizes.leader_input_share)
        pin[:] = lin_bad[j]
        ids, eb, eo, pb, po = LeaderJob.pack_ciphertexts(cts[j])
        jobs.append(LeaderJob(b.nonces[j], times[j], b.public[j], pin, ids, eb, eo, pb, po,
                              present[j], dup[j]))
    helper = HelperAggregateInit(hv, task_id, [tk], hpke_threads=2)
    hagg, lagg = hv.new_aggregate(1), lv.new_aggregate(1)
    sent = []

    def send(req):
        sent.append(C.decode_agg_init_req(req).n)
        return helper.handle(req, hagg)

    stats = []
    st = np.concatenate(drv.run_jobs(jobs, send, lagg, stats=stats))
    exp = np.zeros(b.n, np.uint8)
    exp[[4, 11, 17, 23]] = [4, 2, 8, 8]
    assert st.tolist() == exp.tolist()
    assert sent == [10, 8, 9] and len(stats) == 3
    mask = exp == 0
    for agg, which in ((lagg, "leader"), (hagg, "helper")):
        got, cnt = agg.read(0)
        want, wcnt = expected_aggregate(b, which, mask=mask)
        assert got == want and cnt == wcnt == int(mask.sum())
    # ReportIdChecksum / interval over the finished reports only (Accumulator::update)
    import hashlib
    ck = bytes(32)
    for i in np.flatnonzero(mask):
        ck = bytes(x ^ y for x, y in zip(ck, hashlib.sha256(b.nonces[i].tobytes()).digest()))
    lck, liv = lagg.read_reports(0)
    assert lck == ck and liv[0] == int(times[mask].min())
    helper.close()


@pytest.mark.gpu
def test_leader_driver_rejects_mismatched_response():
    """A helper response that does not answer the sent reports fails the job (and frees its
    state); the next job on the same driver still runs."""
    from janus_amd.leader import LeaderAggregateInit
    from janus_amd.prio3 import Prio3GpuError
    b, mk, task_id, tk, times, cts, LeaderJob = _leader_setup("sum8", 6)
    lv = mk()
    drv = LeaderAggregateInit(lv)
    ids, eb, eo, pb, po = LeaderJob.pack_ciphertexts(cts)
    job = LeaderJob(b.nonces, times, b.public, b.leader_in, ids, eb, eo, pb, po)
    lagg = lv.new_aggregate(1)
    short = C.encode_agg_job_resp(b.nonces[:5], np.zeros((5, 16), np.uint8), 16,
                                  np.zeros(5, np.uint8))
    with pytest.raises(Prio3GpuError):
        drv.handle(job, lambda req: short, lagg)
    assert lagg.read(0)[1] == 0
    good = C.encode_agg_job_resp(b.nonces, b.prep_msg, 16, np.zeros(b.n, np.uint8))
    st = drv.handle(job, lambda req: good, lagg)
    assert (st == 0).all() and lagg.read(0)[1] == b.n


@pytest.mark.gpu
def test_leader_run_jobs_isolates_failing_jobs():
    """run_jobs with an empty job and a job whose helper answers the wrong reports between valid
    ones: those two entries are the jobs' errors, the job in flight before each failure is still
    finished (its request already reached the helper, which accumulated it), and the leader's
    aggregate covers exactly the finished jobs (a failing init must not strand job
    k-1)."""
    from janus_amd._lib import EmptyAggregation, Prio3GpuError
    from janus_amd.helper import HelperAggregateInit
    from janus_amd.leader import LeaderAggregateInit
    from tests.reports import expected_aggregate
    b, mk, task_id, tk, times, cts, LeaderJob = _leader_setup("sum8", 24)
    lv, hv = mk(), mk()
    drv = LeaderAggregateInit(lv)

    def job(j):
        ids, eb, eo, pb, po = LeaderJob.pack_ciphertexts(cts[j])
        return LeaderJob(b.nonces[j], times[j], b.public[j], b.leader_in[j], ids, eb, eo, pb, po)

    e = slice(0, 0)
    jobs = [job(slice(0, 8)), job(e), job(slice(8, 16)), job(slice(16, 24))]
    helper = HelperAggregateInit(hv, task_id, [tk], hpke_threads=2)
    hagg, lagg = hv.new_aggregate(1), lv.new_aggregate(1)
    calls = []

    def send(req):
        calls.append(len(calls))
        resp = helper.handle(req, hagg)
        if len(calls) == 3:  # the fourth job's helper answers only its first report
            return C.encode_agg_job_resp(b.nonces[16:17], b.prep_msg[16:17], 16,
                                         np.zeros(1, np.uint8))
        return resp

    out = drv.run_jobs(jobs, send, lagg)
    assert isinstance(out[1], EmptyAggregation)
    assert isinstance(out[3], Prio3GpuError)
    assert (out[0] == 0).all() and (out[2] == 0).all()
    mask = np.zeros(b.n, bool)
    mask[:16] = True
    got, cnt = lagg.read(0)
    want, wcnt = expected_aggregate(b, "leader", mask=mask)
    assert got == want and cnt == wcnt == 16
    # the driver keeps working after the failures
    st = drv.handle(job(slice(0, 8)), lambda req: helper.handle(req, hagg), lagg)
    assert (st == 0).all() and lagg.read(0)[1] == 24
    helper.close()
    drv.close()
