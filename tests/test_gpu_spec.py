"""Speculative accumulation (k_jr column sums + k_accum_spec) vs the direct accumulation path.

Large batches (several 64-report waves) are made by the GPU client shard, which is itself
parity-tested against the oracle (test_gpu_parity.py::test_gpu_shard_matches_oracle).  Batch slots
mix uniform waves (speculative) with a mixed wave (direct), the last wave is partial (clamped rows
are subtracted again), and tampered reports are rejected after k_jr has already counted them.
Expected aggregates = plaintext sums of the accepted reports per slot
(integration_tests/tests/common/mod.rs:225-398 semantics), and both paths agree byte for byte.
"""
import numpy as np
import pytest

from tests.reports import CONFIGS

pytestmark = pytest.mark.gpu


def _vdaf(name, speculate):
    from janus_amd.prio3 import Prio3Gpu
    c = CONFIGS[name]
    v = Prio3Gpu(c["kind"], bytes(range(16)), bits=c["bits"], length=c["length"],
                 chunk_length=c["chunk"])
    v.set_option("speculate", int(speculate))
    return v


def _meas(name, n, rng):
    c = CONFIGS[name]
    if c["kind"] == 2:
        return rng.integers(0, 1 << c["bits"], size=(n, c["length"]), dtype=np.uint64)
    if c["kind"] == 3:
        return rng.integers(0, c["length"], size=(n, 1), dtype=np.uint64)
    return rng.integers(0, 1 << c["bits"], size=(n, 1), dtype=np.uint64)


def _plain(name, meas, sel):
    c = CONFIGS[name]
    m = meas[sel]
    if c["kind"] == 2:
        return [int(x) for x in m.sum(axis=0, dtype=np.uint64)] if len(m) else [0] * c["length"]
    if c["kind"] == 3:
        return [int((m[:, 0] == i).sum()) for i in range(c["length"])]
    return int(m[:, 0].sum())


def test_sumvec_8_1000_multichunk_fold_bytes_vs_c_restatement():
    """The headline config at a size that reaches the multi-chunk speculative fold (WCH = 32 waves
    = 2,048 reports per chunk, engine.hip launch_accumulate): 4,200 SumVec(8, 1000) reports,
    slot 0 over 36 whole waves (two speculative chunks), slot 1 over 28 waves, one mixed-slot wave
    (direct path) and a partial last wave of 40 rows on slot 2; six reports tampered inside the
    column-summed window (element 500) so k_accum_spec must subtract their rows.  Both
    aggregators' aggregate shares and counts per slot must equal the C restatement's bytes."""
    from janus_amd.prio3 import Prio3Gpu
    from oracle import prio3 as O
    from oracle.ref import Prio3Ref
    n = 4200
    vk = O.synth_verify_key(b"spec-fold")
    ref = Prio3Ref(2, vk, 8, 1000, 89)
    g = ref.gen(b"spec-fold", 0, n, threads=16)
    lin = g["leader_in"].copy()
    bad = [5, 70, 2100, 3000, 4130, 4199]
    for r in bad:
        off = 500 * 16
        x = (int.from_bytes(lin[r, off:off + 16].tobytes(), "little") + 1) % O.Field128.MODULUS
        lin[r, off:off + 16] = np.frombuffer(x.to_bytes(16, "little"), np.uint8)
    slots = np.zeros(n, np.uint32)
    slots[2304:4096] = 1
    slots[4096:4160] = np.random.default_rng(3).integers(0, 3, 64)
    slots[4160:] = 2
    v = Prio3Gpu.new_sum_vec(8, 1000, 89, vk)
    ls, hs = v.new_state(0, n), v.new_state(1, n)
    lp, lst = v.prepare_init(ls, g["nonces"], g["public"], lin)
    hagg, lagg = v.new_aggregate(3), v.new_aggregate(3)
    msgs, hst = v.helper_init(hs, g["nonces"], g["public"], g["helper_in"], lp, agg=hagg,
                              batch_slots=slots)
    _, lst = v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg, batch_slots=slots)
    ok = np.ones(n, bool)
    ok[bad] = False
    assert (hst[bad] == 5).all() and (hst[ok] == 0).all() and (lst == hst).all()
    for q in range(3):
        sel = np.nonzero(slots == q)[0]
        res = ref.prepare_batch(np.ascontiguousarray(g["nonces"][sel]),
                                np.ascontiguousarray(g["public"][sel]),
                                np.ascontiguousarray(lin[sel]),
                                np.ascontiguousarray(g["helper_in"][sel]), threads=16,
                                outputs=False)
        (la, lc), (ha, hc) = lagg.read(q), hagg.read(q)
        assert lc == hc == res["count"] == int(ok[sel].sum())
        assert la == res["agg_l"].tobytes(), f"leader slot {q}"
        assert ha == res["agg_h"].tobytes(), f"helper slot {q}"


@pytest.mark.parametrize("name", ["hist256", "sumvec_small", "sum32", "countvec15"])
def test_speculative_matches_direct_and_plaintext(name):
    n = 300
    rng = np.random.default_rng(11)
    vs, vd = _vdaf(name, True), _vdaf(name, False)
    s = vs.sizes
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rand = rng.integers(0, 256, size=(n, vs.random_size()), dtype=np.uint8)
    meas = _meas(name, n, rng)
    pub, lin, hin = vs.shard(vs.new_state(1, n), nonces, meas, rand)
    es = s.field_size
    bad = [5, 70, 199, 299]
    lin = lin.copy()
    for r in bad:  # first leader meas element + 1: decide fails for these reports only
        x = (int.from_bytes(lin[r, :es].tobytes(), "little") + 1) % vs.modulus
        lin[r, :es] = np.frombuffer(x.to_bytes(es, "little"), dtype=np.uint8)
    slots = np.zeros(n, dtype=np.uint32)
    slots[128:192] = rng.integers(0, 3, size=64)  # wave 2 mixed -> direct chunks
    slots[192:256] = 2
    slots[256:] = 1                              # partial last wave (44 rows)
    out = {}
    for tag, v in (("spec", vs), ("direct", vd)):
        ls, hs = v.new_state(0, n), v.new_state(1, n)
        lp, lst = v.prepare_init(ls, nonces, pub, lin)
        hagg, lagg = v.new_aggregate(3), v.new_aggregate(3)
        msgs, hst = v.helper_init(hs, nonces, pub, hin, lp, agg=hagg, batch_slots=slots)
        _, lst2 = v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg,
                                 batch_slots=slots)
        out[tag] = (hst.copy(), lst2.copy(), [lagg.read(q) for q in range(3)],
                    [hagg.read(q) for q in range(3)])
    assert (out["spec"][0] == out["direct"][0]).all()
    assert (out["spec"][1] == out["direct"][1]).all()
    assert out["spec"][2] == out["direct"][2]
    assert out["spec"][3] == out["direct"][3]
    hst = out["spec"][0]
    ok = np.ones(n, dtype=bool)
    ok[bad] = False
    assert (hst[bad] == 5).all() and (hst[ok] == 0).all()
    for q in range(3):
        sel = ok & (slots == q)
        (la, lc), (ha, hc) = out["spec"][2][q], out["spec"][3][q]
        assert lc == hc == int(sel.sum())
        assert vs.unshard([la, ha]) == _plain(name, meas, sel)


@pytest.mark.parametrize("kind,bits,label", [(0, 0, "count"), (1, 32, "sum32"), (1, 8, "sum8")])
def test_small_types_multichunk_slots_bytes_vs_c_restatement(kind, bits, label):
    """Count / Sum at a size with several 2,048-report accumulation chunks per batch slot: the
    lane-per-report FLP query and decide (k_flp_query_lane, k_decide's lane path) and the merge
    that splits each slot's chunk run over otherwise idle threads (k_accum_merge, runs found by
    binary search, counts by atomics).  10,000 reports over 3 randomly interleaved slots, a few
    tampered; per-slot aggregate bytes and counts of both aggregators == the C restatement."""
    from janus_amd.prio3 import Prio3Gpu
    from oracle import prio3 as O
    from oracle.ref import Prio3Ref
    n = 10000
    cfg = f"merge-{label}".encode()
    vk = O.synth_verify_key(cfg)
    ref = Prio3Ref(kind, vk, bits, 0, 0)
    g = ref.gen(cfg, 0, n, threads=16)
    es = 8 if kind == 0 else 16
    p = O.Field64.MODULUS if kind == 0 else O.Field128.MODULUS
    lin = g["leader_in"].copy()
    bad = [3, 2047, 2048, 6001, 9999]
    for r in bad:  # + 2: a bit becomes 2 or 3 (+ 1 could turn Count's 0 into a valid 1)
        x = (int.from_bytes(lin[r, :es].tobytes(), "little") + 2) % p
        lin[r, :es] = np.frombuffer(x.to_bytes(es, "little"), np.uint8)
    slots = np.random.default_rng(5).integers(0, 3, n).astype(np.uint32)
    v = Prio3Gpu(kind, vk, bits=bits)
    pub = g["public"] if g["public"].shape[1] else None
    ls, hs = v.new_state(0, n), v.new_state(1, n)
    lp, lst = v.prepare_init(ls, g["nonces"], pub, lin)
    hagg, lagg = v.new_aggregate(3), v.new_aggregate(3)
    msgs, hst = v.helper_init(hs, g["nonces"], pub, g["helper_in"], lp, agg=hagg,
                              batch_slots=slots)
    # the helper's Reject reaches the leader in the AggregationJobResp (Count has no prep message
    # to disagree on): the leader driver carries it into prepare_next's status
    lst = np.where(hst != 0, hst, lst).astype(np.uint8)
    _, lst = v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg, batch_slots=slots)
    ok = np.ones(n, bool)
    ok[bad] = False
    assert (hst[bad] == 5).all() and (hst[ok] == 0).all() and (lst == hst).all()
    for q in range(3):
        sel = np.nonzero(slots == q)[0]
        res = ref.prepare_batch(np.ascontiguousarray(g["nonces"][sel]),
                                np.ascontiguousarray(g["public"][sel]),
                                np.ascontiguousarray(lin[sel]),
                                np.ascontiguousarray(g["helper_in"][sel]), threads=16,
                                outputs=False)
        (la, lc), (ha, hc) = lagg.read(q), hagg.read(q)
        assert lc == hc == res["count"] == int(ok[sel].sum())
        assert la == res["agg_l"].tobytes(), f"leader slot {q}"
        assert ha == res["agg_h"].tobytes(), f"helper slot {q}"
