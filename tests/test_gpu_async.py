"""Asynchronous engine use (include/prio3gpu.h: prio3gpu_ctx_set_async / _mark / _wait_mark and
prepare_init split into its XOF and FLP-query phases): a leader context and a helper context
queue two batches with cross-context marks only (no host waits between calls), and the results
equal the synchronous path's / the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["sumvec_small", "hist256", "sum8", "count"])
def test_async_two_context_pipeline_matches_oracle(name):
    import torch
    from janus_amd._lib import check, lib
    from janus_amd.prio3 import Prio3Gpu
    from tests.reports import CONFIGS, expected_aggregate, make_batch
    b = make_batch(name, 40)
    c = CONFIGS[name]
    mk = lambda: Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                          chunk_length=c["chunk"])
    A, H = mk(), mk()
    s = A.sizes
    dev = torch.device("cuda", 0)
    halves = [slice(0, 20), slice(20, 40)]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    nz, pub, lin, hin = d(b.nonces), d(b.public), d(b.leader_in), d(b.helper_in)
    times = torch.arange(b.n, dtype=torch.int64, device=dev) + 5000
    lprep = torch.zeros((b.n, s.prep_share), dtype=torch.uint8, device=dev)
    hprep = torch.zeros((b.n, s.prep_share), dtype=torch.uint8, device=dev)
    msgs = torch.zeros((b.n, max(1, s.prep_msg)), dtype=torch.uint8, device=dev)
    lst = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    hst = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    A.set_async(True)
    H.set_async(True)
    P = lambda t: t.data_ptr()
    ls = [A.new_state(0, 20), A.new_state(0, 20)]
    hs = H.new_state(1, 20)
    lagg, hagg = A.new_aggregate(1), H.new_aggregate(1)
    for i, j in enumerate(halves):
        A.prepare_init_xof(ls[i], nz[j], pub[j] if s.public_share else None, lin[j], lst[j])
        A.prepare_init_query(ls[i], lprep[j], lst[j])
        mA = A.mark()
        H.prepare_init_xof(hs, nz[j], pub[j] if s.public_share else None, hin[j], hst[j])
        H.prepare_init_query(hs, hprep[j], hst[j])
        H.wait_for(A, mA)
        check(lib().prio3gpu_prepare_shares_to_prepare_message(
            H._ctx, 20, P(lprep[j]), P(hprep[j]), P(msgs[j]) if s.prep_msg else None,
            P(hst[j])), "decide")
        check(lib().prio3gpu_prepare_next(H._ctx, hs._h, 20, P(msgs[j]) if s.prep_msg else None,
                                          P(hst[j]), None, None, hagg._h), "helper next")
        check(lib().prio3gpu_agg_update_reports(hagg._h, 20, P(nz[j]), P(times[j]), P(hst[j]),
                                                None), "helper meta")
        mH = H.mark()
        A.wait_for(H, mH)
        check(lib().prio3gpu_prepare_next(A._ctx, ls[i]._h, 20, P(msgs[j]) if s.prep_msg else None,
                                          P(lst[j]), None, None, lagg._h), "leader next")
    A.sync()
    H.sync()
    A.set_async(False)
    H.set_async(False)
    assert int(lst.max()) == 0 and int(hst.max()) == 0
    np.testing.assert_array_equal(lprep.cpu().numpy(), b.leader_prep)
    np.testing.assert_array_equal(hprep.cpu().numpy(), b.helper_prep)
    if s.prep_msg:
        np.testing.assert_array_equal(msgs.cpu().numpy(), b.prep_msg)
    for agg, which in ((lagg, "leader"), (hagg, "helper")):
        got, cnt = agg.read(0)
        want, wcnt = expected_aggregate(b, which)
        assert got == want and cnt == wcnt == b.n
    ck, (start, dur) = hagg.read_reports(0)
    assert start == 5000 and dur == b.n


@pytest.mark.gpu
def test_query_phase_without_xof_phase_is_an_error():
    from janus_amd.prio3 import Prio3Gpu, Prio3GpuError
    from tests.reports import CONFIGS, make_batch
    b = make_batch("sum8", 4)
    c = CONFIGS["sum8"]
    v = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"])
    st = v.new_state(0, 4)
    status = np.zeros(4, np.uint8)
    with pytest.raises(Prio3GpuError):
        v.prepare_init_query(st, np.zeros((4, v.sizes.prep_share), np.uint8), status)
    v.prepare_init_xof(st, b.nonces, b.public, b.leader_in, status)
    out = np.zeros((4, v.sizes.prep_share), np.uint8)
    v.prepare_init_query(st, out, status)
    assert (status == 0).all() and (out == b.leader_prep).all()


def test_stale_mark_is_rejected_and_ctx_wait_takes_no_mark():
    """Marks carry a generation: a mark re-recorded by 16 newer ones is refused
    instead of silently waiting on newer work, and prio3gpu_ctx_wait records a private event, so
    it never consumes the other context's mark ring."""
    from janus_amd.prio3 import Prio3Gpu, Prio3GpuError
    from tests.reports import CONFIGS, make_batch
    b = make_batch("sum8", 4)
    c = CONFIGS["sum8"]
    A = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"])
    B = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"])
    m = A.mark()
    for _ in range(40):
        B.wait_for(A)  # no marks taken on A
    B.wait_for(A, m)   # still valid
    for _ in range(16):
        A.mark()
    with pytest.raises(Prio3GpuError, match="stale mark"):
        B.wait_for(A, m)
    B.wait_for(A, A.mark())
    with pytest.raises(Prio3GpuError):
        B.wait_for(A, 3)  # never a mark (generation 0)
    A.sync()
    B.sync()


@pytest.mark.parametrize("with_total", [True, False])
def test_rccl_flush_is_stream_ordered_in_async_mode(with_total):
    """prio3gpu_agg_allreduce queues like every other all-device call: two jobs
    accumulated and flushed back to back on an async context with no host wait in between give
    the same aggregate, count, checksum and interval as the host-side
    BatchAggregation::merged_with of the two jobs' partials (prio3gpu_batch_aggregation_merge)."""
    import torch
    from janus_amd._lib import check, lib
    from janus_amd.prio3 import Comm, Prio3Gpu
    from tests.reports import CONFIGS, expected_aggregate, make_batch
    name = "sumvec_small"
    b = make_batch(name, 24)
    c = CONFIGS[name]
    v = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                 chunk_length=c["chunk"])
    s = v.sizes
    dev = torch.device("cuda", 0)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    nz, pub, lin, msgs = d(b.nonces), d(b.public), d(b.leader_in), d(b.prep_msg)
    times = torch.arange(b.n, dtype=torch.int64, device=dev) + 7000
    lst = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    P = lambda t: t.data_ptr()
    jobs = [slice(0, 10), slice(10, 24)]
    states = [v.new_state(0, 14) for _ in jobs]
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    local = v.new_aggregate(1)
    total = v.new_aggregate(1) if with_total else None
    torch.cuda.synchronize()
    v.set_async(True)
    for st, j in zip(states, jobs):
        n = j.stop - j.start
        check(lib().prio3gpu_prepare_init(v._ctx, st._h, n, P(nz[j]), P(pub[j]), P(lin[j]), None,
                                          P(lst[j])), "prepare_init")
        check(lib().prio3gpu_prepare_next(v._ctx, st._h, n, P(msgs[j]), P(lst[j]), None, None,
                                          local._h), "prepare_next")
        check(lib().prio3gpu_agg_update_reports(local._h, n, P(nz[j]), P(times[j]), P(lst[j]),
                                                None), "report meta")
        comm.allreduce(v, local, total)  # queued: no host wait
    v.sync()
    v.set_async(False)
    assert int(lst.max()) == 0
    got = (total if with_total else local).read(0)
    want = expected_aggregate(b, "leader")
    assert got[0] == want[0] and got[1] == want[1] == b.n
    ck, iv = (total if with_total else local).read_reports(0)
    import hashlib
    exp_ck = bytes(32)
    for i in range(b.n):
        exp_ck = bytes(x ^ y for x, y in zip(exp_ck, hashlib.sha256(b.nonces[i].tobytes()).digest()))
    assert ck == exp_ck and iv == (7000, b.n)
    # the same through the host merge of the two jobs' partials
    parts = []
    for j in jobs:
        m = np.zeros(b.n, bool)
        m[j] = True
        sh, cnt = expected_aggregate(b, "leader", mask=m)
        pck = bytes(32)
        for i in np.flatnonzero(m):
            pck = bytes(x ^ y for x, y in zip(pck, hashlib.sha256(b.nonces[i].tobytes()).digest()))
        parts.append((sh, cnt, pck, 7000 + j.start, j.stop - j.start))
    from janus_amd.parallel import BatchAggregation, merge_batch_aggregations
    merged = merge_batch_aggregations(s.field_size, [BatchAggregation(sh, cnt, pck, (t0, dur))
                                                     for sh, cnt, pck, t0, dur in parts])
    assert (merged.aggregate_share, merged.report_count, merged.checksum, merged.interval) == \
        (got[0], got[1], ck, iv)
    if with_total:
        assert local.read(0)[1] == 0 and local.read_reports(0) == (bytes(32), (0, 0))
    comm.close()


def test_rccl_flushes_of_two_async_contexts_on_one_comm():
    """One communicator shared by two async contexts (one comm per process, one
    context per job worker; Janus runs jobs concurrently, job_driver.rs:119-216).  Both contexts
    flush different partials back to back with no host wait: the comm's shared all-gather scratch
    must not be overwritten by the second flush while the first one's k_merge_ranks reads it, so
    each total equals its own partial (aggregate bytes, count, checksum, interval) -- the
    BatchAggregation::merged_with of one partial (aggregate_share.rs:47-65)."""
    import hashlib

    import torch
    from janus_amd._lib import check, lib
    from janus_amd.parallel import BatchAggregation, merge_batch_aggregations
    from janus_amd.prio3 import Comm, Prio3Gpu
    from tests.reports import CONFIGS, expected_aggregate, make_batch
    name = "sumvec_small"
    b = make_batch(name, 48)
    c = CONFIGS[name]
    mk = lambda: Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                          chunk_length=c["chunk"])
    ctxs = [mk(), mk()]
    s = ctxs[0].sizes
    dev = torch.device("cuda", 0)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    nz, pub, lin, msgs = d(b.nonces), d(b.public), d(b.leader_in), d(b.prep_msg)
    times = torch.arange(b.n, dtype=torch.int64, device=dev) + 9000
    lst = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    P = lambda t: t.data_ptr()
    jobs = [slice(0, 30), slice(30, 48)]
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    states = [v.new_state(0, j.stop - j.start) for v, j in zip(ctxs, jobs)]
    locals_ = [v.new_aggregate(1) for v in ctxs]
    totals = [v.new_aggregate(1) for v in ctxs]
    torch.cuda.synchronize()
    for rep in range(3):  # repeated: each round flushes into the running totals
        for v in ctxs:
            v.set_async(True)
        for v, st, loc, j in zip(ctxs, states, locals_, jobs):
            n = j.stop - j.start
            check(lib().prio3gpu_prepare_init(v._ctx, st._h, n, P(nz[j]), P(pub[j]), P(lin[j]),
                                              None, P(lst[j])), "prepare_init")
            check(lib().prio3gpu_prepare_next(v._ctx, st._h, n, P(msgs[j]), P(lst[j]), None, None,
                                              loc._h), "prepare_next")
            check(lib().prio3gpu_agg_update_reports(loc._h, n, P(nz[j]), P(times[j]), P(lst[j]),
                                                    None), "report meta")
        for v, loc, tot in zip(ctxs, locals_, totals):
            comm.allreduce(v, loc, tot)  # back to back, queued on two streams, no host wait
        for v in ctxs:
            v.sync()
            v.set_async(False)
    assert int(lst.max()) == 0
    for tot, j in zip(totals, jobs):
        m = np.zeros(b.n, bool)
        m[j] = True
        sh, cnt = expected_aggregate(b, "leader", mask=m)
        # three flushes of the same partial: 3x the share mod p, 3x the count, checksum XOR'd 3x
        vec = [(3 * x) % ctxs[0].modulus for x in ctxs[0].decode_field_vec(sh)]
        want = b"".join(int(x).to_bytes(s.field_size, "little") for x in vec)
        got_sh, got_cnt = tot.read(0)
        assert got_sh == want and got_cnt == 3 * cnt
        pck = bytes(32)
        for i in np.flatnonzero(m):
            pck = bytes(x ^ y for x, y in zip(pck, hashlib.sha256(b.nonces[i].tobytes()).digest()))
        ck, iv = tot.read_reports(0)
        assert ck == pck and iv == (9000 + j.start, j.stop - j.start)
        one = merge_batch_aggregations(s.field_size, [BatchAggregation(sh, cnt, pck,
                                                                      (9000 + j.start,
                                                                       j.stop - j.start))] * 3)
        assert (one.aggregate_share, one.report_count, one.checksum, one.interval) == \
            (got_sh, got_cnt, ck, iv)
    for loc in locals_:
        assert loc.read(0)[1] == 0
    comm.close()


@pytest.mark.parametrize("name", ["sumvec_small", "hist256", "sumvec_8_1000", "sum8", "fp16_3",
                                  "count"])
def test_three_phase_prepare_init_matches_oracle(name):
    """prepare_init as XOF phase -> weights phase (prio3gpu_prepare_init_weights: ParallelSum
    types' k_flp_weights; a no-op otherwise) -> query phase, for both aggregators: the oracle's
    prep shares; the weights phase twice is harmless, and the query phase alone still works.
    (Count: the XOF phase runs the whole query, the query phase copies the prep shares out.)"""
    from tests.test_gpu_parity import batch, gpu_vdaf
    b = batch(name)  # the transcript tests' cached oracle batch
    v = gpu_vdaf(b)
    s = v.sizes
    for agg_id, inp, want in ((0, b.leader_in, b.leader_prep), (1, b.helper_in, b.helper_prep)):
        for weights in (0, 1, 2):
            st = v.new_state(agg_id, b.n)
            status = np.zeros(b.n, np.uint8)
            v.prepare_init_xof(st, b.nonces, b.public if s.public_share else None, inp, status)
            for _ in range(weights):
                v.prepare_init_weights(st, status)
            out = np.zeros((b.n, s.prep_share), np.uint8)
            v.prepare_init_query(st, out, status)
            assert (status == 0).all()
            np.testing.assert_array_equal(out, want)
            st.close()
