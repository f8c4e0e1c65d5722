"""GPU parity: the HIP engine (through the C ABI) vs the CPU oracle, bit-exact.

Every byte the reference path produces per report -- prep shares (both aggregators), prep
messages, output shares, aggregate shares -- is compared with the oracle's VdafTranscript
(core/src/test_util/mod.rs:50-233).  Negative cases follow the reference's per-report error
mapping (aggregator/src/aggregator/error.rs:240-300): a bad report is rejected alone.
"""
import numpy as np
import pytest

from tests.reports import CONFIGS, expected_aggregate, make_batch, plaintext_sum

pytestmark = pytest.mark.gpu

SIZES = {"count": 64, "sum8": 40, "sum32": 24, "sum5": 24, "sum1": 16, "sum64": 16, "sum2": 70,
         "sum4": 70, "sum16": 70, "sumvec_small": 40, "countvec15": 24, "hist4": 40,
         "hist256": 24, "sumvec_8_1000": 6, "sumvec_odd_calls": 8, "sumvec_chunk128": 8, "sumvec_chunk65": 8, "fp16_3": 12, "fp32_5": 8, "fp64_4": 8, "fp16_300": 6,
         "fp16_5000": 2, "sumvec_calls1": 8, "hist_calls1": 8, "sumvec_calls3": 8}
FPVEC = [k for k in SIZES if k.startswith("fp")]

_cache = {}


def batch(name):
    if name not in _cache:
        _cache[name] = make_batch(name, SIZES[name])
    return _cache[name]


def gpu_vdaf(b):
    from janus_amd.prio3 import Prio3Gpu
    c = CONFIGS[b.name]
    return Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                    chunk_length=c["chunk"])


@pytest.mark.parametrize("name", list(SIZES))
def test_prepare_transcript_bit_exact(name):
    b = batch(name)
    v = gpu_vdaf(b)
    s = v.sizes
    assert s.leader_input_share == b.leader_in.shape[1]
    assert s.prep_share == b.leader_prep.shape[1]
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    assert (lst == 0).all()
    np.testing.assert_array_equal(lp, b.leader_prep)
    hp, hst = v.prepare_init(hs, b.nonces, b.public, b.helper_in)
    assert (hst == 0).all()
    np.testing.assert_array_equal(hp, b.helper_prep)
    msgs, st = v.prepare_shares_to_prepare_message(lp, hp)
    assert (st == 0).all()
    np.testing.assert_array_equal(msgs, b.prep_msg)
    lo, lst = v.prepare_next(ls, msgs, lst.copy())
    ho, hst = v.prepare_next(hs, msgs, hst.copy())
    assert (lst == 0).all() and (hst == 0).all()
    np.testing.assert_array_equal(lo, b.leader_out)
    np.testing.assert_array_equal(ho, b.helper_out)


@pytest.mark.parametrize("name", list(SIZES))
def test_aggregate_and_unshard(name):
    b = batch(name)
    v = gpu_vdaf(b)
    ls = v.new_state(0, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    # helper: fused aggregate-init
    hs = v.new_state(1, b.n)
    hagg = v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, b.nonces, b.public, b.helper_in, lp, agg=hagg)
    assert (hst == 0).all()
    np.testing.assert_array_equal(msgs, b.prep_msg)
    lagg = v.new_aggregate(1)
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    la, lc = lagg.read(0)
    ha, hc = hagg.read(0)
    assert lc == hc == b.n
    assert la == expected_aggregate(b, "leader")[0]
    assert ha == expected_aggregate(b, "helper")[0]
    if name in FPVEC:
        assert v.unshard([la, ha], lc) == pytest.approx(plaintext_sum(b), rel=1e-12, abs=1e-12)
    else:
        assert v.unshard([la, ha]) == plaintext_sum(b)


@pytest.mark.parametrize("name", ["sum8", "hist4", "sumvec_small", "count", "fp16_300"])
def test_batch_slots_segmentation(name):
    b = batch(name)
    v = gpu_vdaf(b)
    rng = np.random.default_rng(7)
    slots = rng.integers(0, 3, size=b.n).astype(np.uint32)
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    hagg = v.new_aggregate(3)
    msgs, hst = v.helper_init(hs, b.nonces, b.public, b.helper_in, lp, agg=hagg,
                              batch_slots=slots)
    lagg = v.new_aggregate(3)
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg, batch_slots=slots)
    for s in range(3):
        for agg, which in ((lagg, "leader"), (hagg, "helper")):
            got, cnt = agg.read(s)
            exp, ecnt = expected_aggregate(b, which, slots=slots, slot=s)
            assert got == exp and cnt == ecnt


def _oracle_prep_share(b, agg_id, r, leader_in=None, public=None):
    v = b.vdaf
    share_b = (leader_in if leader_in is not None else b.leader_in)[r].tobytes() if agg_id == 0 \
        else b.helper_in[r].tobytes()
    share = v.decode_input_share(agg_id, share_b)
    pub = v.decode_public_share((public if public is not None else b.public)[r].tobytes())
    _, ps = v.prepare_init(b.verify_key, agg_id, b.nonces[r].tobytes(), pub, share)
    return v.encode_prep_share(ps)


@pytest.mark.parametrize("name", ["sum8", "hist4", "sumvec_small", "count", "fp16_3", "fp64_4"])
def test_tampered_reports_rejected_alone(name):
    """A tampered leader measurement share fails decide for that report only; the GPU prep
    shares of the tampered report still match the oracle bit for bit."""
    b = batch(name)
    v = gpu_vdaf(b)
    es = b.vdaf.fld.ENCODED_SIZE
    bad = [1, 5]
    lin = b.leader_in.copy()
    for r in bad:
        x = int.from_bytes(lin[r, :es].tobytes(), "little")
        x = (x + 1) % b.vdaf.fld.MODULUS
        lin[r, :es] = np.frombuffer(x.to_bytes(es, "little"), dtype=np.uint8)
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, lin)
    assert (lst == 0).all()
    for r in bad:
        assert lp[r].tobytes() == _oracle_prep_share(b, 0, r, leader_in=lin)
    hagg = v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, b.nonces, b.public, b.helper_in, lp, agg=hagg)
    mask = np.ones(b.n, dtype=bool)
    mask[bad] = False
    assert (hst[bad] == 5).all() and (hst[mask] == 0).all()
    ha, hc = hagg.read(0)
    exp, ecnt = expected_aggregate(b, "helper", mask=mask)
    assert ha == exp and hc == ecnt


def test_noncanonical_leader_share_is_invalid_message():
    b = batch("hist4")
    v = gpu_vdaf(b)
    lin = b.leader_in.copy()
    lin[3, :16] = 0xFF  # >= p: decode error
    ls = v.new_state(0, b.n)
    _, lst = v.prepare_init(ls, b.nonces, b.public, lin)
    assert lst[3] == 8 and (np.delete(lst, 3) == 0).all()


@pytest.mark.parametrize("name", ["hist256", "sumvec_small", "countvec15", "sumvec_8_1000",
                                  "sumvec_odd_calls", "sum8", "sum32"])
def test_noncanonical_element_inside_a_lane_group(name):
    """A non-canonical measurement element deep inside the share (not the first element) rejects
    only its report, whichever lane of a multi-report wave (k_flp_wires_cols: G lanes per report)
    it lands in; every other report's prep share stays bit-exact."""
    b = batch(name)
    v = gpu_vdaf(b)
    es = b.vdaf.fld.ENCODED_SIZE
    meas_len = b.vdaf.typ.MEAS_LEN
    lin = b.leader_in.copy()
    bad = {1: meas_len - 1, 3: meas_len // 2, 5: 1}
    for r, e in bad.items():
        lin[r, e * es:(e + 1) * es] = 0xFF
    ls = v.new_state(0, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, lin)
    for r in range(b.n):
        if r in bad:
            assert lst[r] == 8, (r, lst[r])
        else:
            assert lst[r] == 0, (r, lst[r])
            np.testing.assert_array_equal(lp[r], b.leader_prep[r])


@pytest.mark.parametrize("name", ["sum8", "sum32", "sum64"])
def test_noncanonical_gadget_coefficient_rejects_its_report(name):
    """A non-canonical gadget-polynomial coefficient of the proof share (first, middle, last)
    rejects only its report in the paired Sum query; every other report's prep share stays
    bit-exact."""
    b = batch(name)
    v = gpu_vdaf(b)
    es = b.vdaf.fld.ENCODED_SIZE
    meas_len, proof_len = b.vdaf.typ.MEAS_LEN, b.vdaf.PROOF_LEN
    lin = b.leader_in.copy()
    bad = {0: meas_len + 1, 2: meas_len + proof_len // 2, 7: meas_len + proof_len - 1}
    for r, e in bad.items():
        lin[r, e * es:(e + 1) * es] = 0xFF
    ls = v.new_state(0, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, lin)
    for r in range(b.n):
        if r in bad:
            assert lst[r] == 8, (r, lst[r])
        else:
            assert lst[r] == 0, (r, lst[r])
            np.testing.assert_array_equal(lp[r], b.leader_prep[r])


def test_tampered_public_share_rejected():
    b = batch("sum8")
    v = gpu_vdaf(b)
    pub = b.public.copy()
    pub[2, 20] ^= 1  # helper's joint-rand part as seen by the leader
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, pub, b.leader_in)
    assert lp[2].tobytes() == _oracle_prep_share(b, 0, 2, public=pub)
    hp, hst = v.prepare_init(hs, b.nonces, pub, b.helper_in)
    assert hp[2].tobytes() == _oracle_prep_share(b, 1, 2, public=pub)
    msgs, st = v.prepare_shares_to_prepare_message(lp, hp)
    # helper's part is honest, so prep msg == H(part_L, part_H) is the honest one, but the
    # leader's corrected seed used the tampered part: decide fails (different joint rand)
    assert st[2] == 5 and (np.delete(st, 2) == 0).all()


def test_wrong_prep_msg_fails_prepare_next():
    b = batch("sumvec_small")
    v = gpu_vdaf(b)
    ls = v.new_state(0, b.n)
    _, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    msgs = b.prep_msg.copy()
    msgs[4, 0] ^= 0x80
    lagg = v.new_aggregate(1)
    _, st = v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    assert st[4] == 5 and (np.delete(st, 4) == 0).all()
    _, cnt = lagg.read(0)
    assert cnt == b.n - 1


def test_empty_batch():
    b = batch("sum8")
    v = gpu_vdaf(b)
    ls = v.new_state(0, 4)
    prep, st = v.prepare_init(ls, np.zeros((0, 16), np.uint8), np.zeros((0, 32), np.uint8),
                              np.zeros((0, v.sizes.leader_input_share), np.uint8))
    assert prep.shape == (0, v.sizes.prep_share) and st.shape == (0,)


def test_device_resident_inputs_torch():
    import torch
    b = batch("hist256")
    v = gpu_vdaf(b)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ls = v.new_state(0, b.n)
    lp, lst = v.prepare_init(ls, t(b.nonces), t(b.public), t(b.leader_in))
    np.testing.assert_array_equal(lp, b.leader_prep)


def test_agg_merge_bytes():
    b = batch("hist4")
    v = gpu_vdaf(b)
    agg = v.new_aggregate(2)
    exp, _ = expected_aggregate(b, "leader")
    agg.merge(1, exp, 7)
    agg.merge(1, exp, 3)
    got, cnt = agg.read(1)
    x = v.decode_field_vec(exp)
    assert v.decode_field_vec(got) == [(2 * a) % v.modulus for a in x] and cnt == 10


def test_rccl_merge_single_rank():
    """RCCL all-gather + mod-p merge path with one rank: total += local, local reset."""
    from janus_amd.prio3 import Comm
    b = batch("hist4")
    v = gpu_vdaf(b)
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    ls = v.new_state(0, b.n)
    _, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    local, total = v.new_aggregate(1), v.new_aggregate(1)
    v.prepare_next(ls, b.prep_msg, lst, want_output_shares=False, agg=local)
    times = np.arange(100, 100 + b.n, dtype=np.uint64)
    local.update_reports(b.nonces, times, lst)
    ck_local = local.read_reports(0)
    comm.allreduce(v, local, total)
    comm.allreduce(v, local, total)  # local was reset: no double counting
    got, cnt = total.read(0)
    assert got == expected_aggregate(b, "leader")[0] and cnt == b.n
    assert local.read(0)[1] == 0
    # checksums and intervals travel with the merge (all-gather + XOR / min-max fold)
    assert total.read_reports(0) == ck_local and ck_local[1] == (100, b.n)
    assert local.read_reports(0) == (bytes(32), (0, 0))
    comm.close()


def test_rccl_epoch_merge_remaps_slots():
    """prio3gpu_agg_epoch_merge with one rank: two jobs accumulate into ONE pooled partial whose
    slots hold batch identifiers in first-seen order (k2, k0, k5; slot 3 unused); the epoch merge
    lands each slot in the union table (k0, k1, k2, k5; k1 seen only by another rank) -- shares,
    counts, checksums and intervals -- and resets the partial.  Reference: the batch-aggregation
    shard merge, aggregate_share.rs:44-66."""
    from janus_amd.parallel import epoch_merge_device
    from janus_amd.prio3 import Comm
    b = batch("hist4")
    v = gpu_vdaf(b)
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    h = b.n // 2
    keys = [b"k2", b"k0", b"k5"]
    # report -> local slot: job A (first half) sees k2, k0; job B sees k0, k5
    slots = np.array([(r % 2) if r < h else 1 + (r % 2) for r in range(b.n)], np.uint32)
    times = np.arange(500, 500 + b.n, dtype=np.uint64)
    local = v.new_aggregate(4)
    for lo, hi in ((0, h), (h, b.n)):  # two independent jobs, no collective between them
        ls = v.new_state(0, hi - lo)
        _, lst = v.prepare_init(ls, b.nonces[lo:hi], b.public[lo:hi], b.leader_in[lo:hi])
        v.prepare_next(ls, b.prep_msg[lo:hi], lst, want_output_shares=False, agg=local,
                       batch_slots=slots[lo:hi])
        local.update_reports(b.nonces[lo:hi], times[lo:hi], lst, slots[lo:hi])
        ls.close()
    before = [(local.read(s), local.read_reports(s)) for s in range(3)]
    union, total = epoch_merge_device(comm, v, local, keys, 0,
                                      lambda obj: [obj, (0, [b"k1"])])
    assert union == [b"k0", b"k1", b"k2", b"k5"]
    for s, k in enumerate(keys):
        u = union.index(k)
        assert (total.read(u), total.read_reports(u)) == before[s]
        want, cnt = expected_aggregate(b, "leader", slots=slots, slot=s)
        assert total.read(u) == (want, cnt) and cnt > 0
    assert total.read(union.index(b"k1"))[1] == 0  # another rank's key: empty here
    assert all(local.read(s)[1] == 0 for s in range(4))
    assert local.read_reports(0) == (bytes(32), (0, 0))
    with pytest.raises(Exception):  # a slot map that sends two slots to one union slot
        comm.epoch_merge(v, local, [0, 0, 1, 2], v.new_aggregate(3))
    total.close()
    local.close()
    comm.close()


@pytest.mark.parametrize("name", list(SIZES))
def test_gpu_shard_matches_oracle(name):
    """Client::shard + FLP prove on the GPU reproduce the oracle's public/leader/helper shares."""
    from tests.reports import meas_array
    b = batch(name)
    v = gpu_vdaf(b)
    assert v.random_size() == b.rand.shape[1]
    st = v.new_state(1, b.n)
    pub, lead, helper = v.shard(st, b.nonces, meas_array(b), b.rand)
    np.testing.assert_array_equal(helper, b.helper_in)
    if v.sizes.public_share:
        np.testing.assert_array_equal(pub, b.public)
    np.testing.assert_array_equal(lead, b.leader_in)


def test_fixedpoint16_end_to_end_kat():
    """interop_binaries/tests/end_to_end.rs:689-723 (e2e_prio3_fixed16vec): four FixedI16 vectors
    of length 3 -> ["0.5", "0.5", "0.6875"], through the GPU leader + helper paths."""
    from oracle import prio3 as O
    from janus_amd.prio3 import Prio3Gpu
    q = lambda x: int(x * (1 << 15))
    ms = [[q(.25), q(.125), q(.125)], [q(.0625), q(.125), q(.0625)],
          [q(.125), q(.125), q(.25)], [q(.0625), q(.125), q(.25)]]
    ov = O.Prio3.new_fixedpoint_boundedl2_vec_sum(16, 3)
    vk = bytes(range(16))
    rows = {k: [] for k in ("nonce", "public_share", "leader_input_share", "helper_input_share")}
    for i, m in enumerate(ms):
        nonce = bytes([i + 1]) * 16
        pub, shares = ov.shard(m, nonce, bytes([0x40 + i]) * ov.random_size())
        rows["nonce"].append(nonce)
        rows["public_share"].append(ov.encode_public_share(pub))
        rows["leader_input_share"].append(ov.encode_input_share(shares[0]))
        rows["helper_input_share"].append(ov.encode_input_share(shares[1]))
    arr = {k: np.frombuffer(b"".join(v), np.uint8).reshape(len(v), -1).copy()
           for k, v in rows.items()}
    v = Prio3Gpu.new_fixedpoint_boundedl2_vec_sum(16, 3, vk)
    ls, hs = v.new_state(0, 4), v.new_state(1, 4)
    lp, lst = v.prepare_init(ls, arr["nonce"], arr["public_share"], arr["leader_input_share"])
    hagg, lagg = v.new_aggregate(1), v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, arr["nonce"], arr["public_share"], arr["helper_input_share"], lp,
                              agg=hagg)
    assert (lst == 0).all() and (hst == 0).all()
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    (la, lc), (ha, hc) = lagg.read(0), hagg.read(0)
    assert lc == hc == 4
    assert [repr(x) for x in v.unshard([la, ha], 4)] == ["0.5", "0.5", "0.6875"]


def test_fixedpoint_norm_violation_rejected():
    """A client that claims a smaller norm than its entries have (bit-encoded claim != computed
    norm) is rejected by decide; the other reports of the batch are unaffected."""
    from oracle import prio3 as O
    b = batch("fp16_3")
    v = gpu_vdaf(b)
    ov = b.vdaf
    typ = ov.typ
    r = 2
    # re-shard report r with a forged encoding: the norm bits claim 0
    enc = typ.encode(b.measurements[r])
    forged = enc[:typ.range_norm_begin] + [0] * typ.bits_for_norm
    orig = typ.encode
    typ.encode = lambda m: forged
    try:
        pub, shares = ov.shard(b.measurements[r], b.nonces[r].tobytes(), b.rand[r].tobytes())
    finally:
        typ.encode = orig
    lin, hin, pb = b.leader_in.copy(), b.helper_in.copy(), b.public.copy()
    lin[r] = np.frombuffer(ov.encode_input_share(shares[0]), np.uint8)
    hin[r] = np.frombuffer(ov.encode_input_share(shares[1]), np.uint8)
    pb[r] = np.frombuffer(ov.encode_public_share(pub), np.uint8)
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, pb, lin)
    assert lp[r].tobytes() == _oracle_prep_share(b, 0, r, leader_in=lin, public=pb)
    msgs, hst = v.helper_init(hs, b.nonces, pb, hin, lp, agg=v.new_aggregate(1))
    assert hst[r] == 5 and (np.delete(hst, r) == 0).all()


def test_fixedpoint16_100k_entries_config_e():
    """BASELINE config E (FixedI16 BoundedL2VecSum, 100k entries: 1.6M-element shares, 25.7 MB
    per leader share): GPU prep shares, prep msgs and both aggregate shares bit-exact against the
    C restatement; unshard == the plaintext sum."""
    from oracle import prio3 as O
    from oracle.ref import Prio3Ref
    from janus_amd.prio3 import Prio3Gpu
    vk = O.synth_verify_key(b"cfgE")
    ref = Prio3Ref(4, vk, 16, 100000, 0)
    n = 3
    g = ref.gen(b"cfgE", 0, n, threads=16)
    res = ref.prepare_batch(g["nonces"], g["public"], g["leader_in"], g["helper_in"], threads=16)
    assert (res["status"] == 0).all()
    v = Prio3Gpu.new_fixedpoint_boundedl2_vec_sum(16, 100000, vk)
    ls, hs = v.new_state(0, n), v.new_state(1, n)
    lp, lst = v.prepare_init(ls, g["nonces"], g["public"], g["leader_in"])
    assert (lst == 0).all()
    np.testing.assert_array_equal(lp, res["lprep"])
    hagg, lagg = v.new_aggregate(1), v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, g["nonces"], g["public"], g["helper_in"], lp, agg=hagg)
    assert (hst == 0).all()
    np.testing.assert_array_equal(msgs, res["msgs"])
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    (la, lc), (ha, hc) = lagg.read(0), hagg.read(0)
    assert lc == hc == n
    assert la == res["agg_l"].tobytes() and ha == res["agg_h"].tobytes()
    plain = g["meas"].view(np.int64).sum(axis=0) * 2.0 ** -15
    assert v.unshard([la, ha], n) == pytest.approx(list(plain), abs=1e-12)


@pytest.mark.parametrize("name", ["fp16_3", "fp64_4", "fp16_300"])
def test_fpvec_helper_two_pass_path_bit_exact(name):
    """The FixedPoint helper runs its two sponges fused (k_helper_xof) by default and falls back
    to the exact two-pass k_expand + k_jr when a squeezed element is non-canonical.  The fallback
    cannot be provoked with real seeds (probability ~28/2^64 per element), so force the two-pass
    path through the context option and check it too against the oracle's transcript."""
    b = batch(name)
    v = gpu_vdaf(b)
    v.set_option("fused_helper", 0)
    hs = v.new_state(1, b.n)
    hp, hst = v.prepare_init(hs, b.nonces, b.public, b.helper_in)
    assert (hst == 0).all()
    np.testing.assert_array_equal(hp, b.helper_prep)
    ho, hst = v.prepare_next(hs, b.prep_msg, hst.copy())
    assert (hst == 0).all()
    np.testing.assert_array_equal(ho, b.helper_out)


@pytest.mark.parametrize("opts", [{}, {"snap_chunk": 1}, {"snap_chunk": 5}, {"helper_snap": 0},
                                  {"pair_chains": 0, "chain_pairs": 2},
                                  {"snap_chunk": 5, "query_overlap": 1},
                                  {"snap_chunk": 1, "query_overlap": 1},
                                  {"pair_chains": 0}, {"pair_chains": 0, "helper_snap": 0},
                                  {"snap_chunk": 5, "query_overlap": 0}],
                         ids=["snap", "snap_chunk1", "snap_chunk5", "rows", "pairs2", "overlap5",
                              "overlap1", "unpaired", "unpaired_rows", "inturn5"])
@pytest.mark.parametrize("name", ["fp16_3", "fp64_4", "fp16_300"])
def test_fpvec_helper_snapshot_mode(name, opts):
    """Snapshot mode (helper_snap, the default): the FixedPoint helper keeps k_helper_xof's sponge
    snapshots instead of the expanded share and k_fpv_regen rewrites each query / accumulation
    chunk's rows (with query_overlap 1, the default, the query's half-chunks regenerated on a
    second stream beside the previous half-chunk's query; 0: in turn).  Prep shares, output shares and the
    aggregate with a rejected row (regenerated rows summed directly) equal the oracle's, for one
    chunk, several chunks and the stored-rows mode."""
    b = batch(name)
    v = gpu_vdaf(b)
    for k, val in opts.items():
        v.set_option(k, val)
    hs = v.new_state(1, b.n)
    hp, hst = v.prepare_init(hs, b.nonces, b.public, b.helper_in)
    assert (hst == 0).all()
    np.testing.assert_array_equal(hp, b.helper_prep)
    ho, hst2 = v.prepare_next(hs, b.prep_msg, hst.copy())
    assert (hst2 == 0).all()
    np.testing.assert_array_equal(ho, b.helper_out)
    hst = hst.copy()
    hst[1] = 5
    hagg = v.new_aggregate(1)
    v.prepare_next(hs, b.prep_msg, hst, want_output_shares=False, agg=hagg)
    slots = np.zeros(b.n, np.uint32)
    slots[1] = 1
    exp, ecnt = expected_aggregate(b, "helper", slots=slots, slot=0)
    assert hagg.read(0) == (exp, ecnt) and ecnt == b.n - 1


def test_fpvec_helper_snapshot_whole_waves():
    """64 FixedPoint reports, all accepted, one slot: the snapshot-mode helper aggregates from the
    storer's column sums alone (every element, no row read or regenerated); the aggregate equals
    the oracle's and the stored-rows mode's."""
    b = make_batch("fp16_3", 64)
    aggs = []
    for snap in (1, 0):
        v = gpu_vdaf(b)
        v.set_option("helper_snap", snap)
        ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
        lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
        hagg = v.new_aggregate(1)
        msgs, hst = v.helper_init(hs, b.nonces, b.public, b.helper_in, lp, agg=hagg)
        assert (hst == 0).all()
        np.testing.assert_array_equal(msgs, b.prep_msg)
        aggs.append(hagg.read(0))
    assert aggs[0] == aggs[1] == expected_aggregate(b, "helper")


@pytest.mark.parametrize("pairs,n", [(1, 100), (2, 100), (0, 100), (0, 161)],
                         ids=["pairs1", "pairs2", "lane_pairs", "lane_pairs_161"])
def test_fpvec_chain_pairs(pairs, n):
    """k_helper_xof / k_jr_ring with one or two 64-report chains per workgroup (option
    chain_pairs, pair_chains 0): 100 reports, so the second workgroup's pair is partial and, with
    two pairs, the first workgroup's second pair too; and the lane-pair kernels (pairs = 0 here:
    k_helper_xof_pair, 64 reports per workgroup, k_jr_ring_pair, 128) with 100 and 161 reports
    (161 = a last helper workgroup of 33: one full and one 1-report sponge wave).  Both
    aggregators' prep shares, the prep messages and both aggregates (the chains' column sums)
    equal the oracle's."""
    b = make_batch("fp16_3", n)
    v = gpu_vdaf(b)
    if pairs:
        v.set_option("pair_chains", 0)
        v.set_option("chain_pairs", pairs)
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    assert (lst == 0).all()
    np.testing.assert_array_equal(lp, b.leader_prep)
    lagg, hagg = v.new_aggregate(1), v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, b.nonces, b.public, b.helper_in, lp, agg=hagg)
    assert (hst == 0).all()
    np.testing.assert_array_equal(msgs, b.prep_msg)
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    assert lagg.read(0) == expected_aggregate(b, "leader")
    assert hagg.read(0) == expected_aggregate(b, "helper")


@pytest.mark.parametrize("opts", [{}, {"jr_ring": 0}, {"spread": 0},
                                  {"pair_chains": 0, "chain_pairs": 2}, {"pair_chains": 0}],
                         ids=["ring", "k_jr_spread", "k_jr_packed", "ring_pairs2", "ring_unpaired"])
@pytest.mark.parametrize("name", ["fp16_3", "fp16_300"])
def test_fpvec_leader_jr_variants(name, opts):
    """The leader's FixedPoint joint-rand part runs k_jr_ring (sponge wave + loader wave writing
    the speculative column sums) when few waves fit one per CU, else k_jr.  Every variant gives
    the oracle's prep shares, and its column sums fold into the exact aggregate with a rejected
    row subtracted (report 1's status set before prepare_next; rows past n are clamped copies)."""
    b = batch(name)
    v = gpu_vdaf(b)
    for k, val in opts.items():
        v.set_option(k, val)
    ls = v.new_state(0, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    assert (lst == 0).all()
    np.testing.assert_array_equal(lp, b.leader_prep)
    lst = lst.copy()
    lst[1] = 5
    lagg = v.new_aggregate(1)
    v.prepare_next(ls, b.prep_msg, lst, want_output_shares=False, agg=lagg)
    got, cnt = lagg.read(0)
    slots = np.zeros(b.n, np.uint32)
    slots[1] = 1
    exp, ecnt = expected_aggregate(b, "leader", slots=slots, slot=0)
    assert got == exp and cnt == ecnt == b.n - 1


def test_report_checksum_and_interval():
    """Accumulator::update's per-batch bookkeeping next to the aggregate share: ReportIdChecksum
    = XOR of SHA-256(report id) (core/src/report_id.rs:18-44, hashlib as the oracle) and the
    client-timestamp interval [min, max + 1) (core/src/time.rs:289-312) over the reports whose
    status is 0, per batch slot; whole waves on one slot and mixed-slot waves both covered."""
    import hashlib
    from janus_amd.prio3 import Prio3Gpu
    rng = np.random.default_rng(11)
    n = 1000
    ids = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    times = rng.integers(1_600_000_000, 1_700_000_000, n, dtype=np.uint64)
    status = np.where(rng.random(n) < 0.1, 5, 0).astype(np.uint8)
    slots = np.zeros(n, np.uint32)
    slots[512:] = rng.integers(0, 3, n - 512)
    v = Prio3Gpu.new_sum(8, bytes(16))
    agg = v.new_aggregate(4)
    agg.update_reports(ids[:700], times[:700], status[:700], slots[:700])
    agg.update_reports(ids[700:], times[700:], status[700:], slots[700:])  # two calls accumulate
    for slot in range(4):
        sel = [i for i in range(n) if status[i] == 0 and slots[i] == slot]
        ck = bytearray(32)
        for i in sel:
            for k, x in enumerate(hashlib.sha256(ids[i].tobytes()).digest()):
                ck[k] ^= x
        got_ck, (start, dur) = agg.read_reports(slot)
        assert got_ck == bytes(ck)
        if sel:
            assert (start, dur) == (int(times[sel].min()), int(times[sel].max() - times[sel].min()) + 1)
        else:
            assert (start, dur) == (0, 0)
    agg.reset()
    assert agg.read_reports(0) == (bytes(32), (0, 0))


@pytest.mark.parametrize("name", ["sumvec_small", "hist256", "sum32", "count", "fp16_3"])
def test_pitched_input_shares_bit_exact(name):
    """Input shares at a row pitch > the share length (prio3gpu_state_set_input_pitch): a caller
    decoding leader shares into 128-B-aligned rows gets the same prep shares, prep messages and
    aggregates as with packed rows; host and device buffers; the helper's seeds too."""
    import torch
    from janus_amd._lib import Prio3GpuError
    b = batch(name)
    v = gpu_vdaf(b)
    s = v.sizes
    lp_pitch = (s.leader_input_share + 127) // 128 * 128 + 128
    rows = np.zeros((b.n, lp_pitch), np.uint8)
    rows[:, :s.leader_input_share] = b.leader_in
    ls = v.new_state(0, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, rows[:, :s.leader_input_share])
    assert (lst == 0).all()
    np.testing.assert_array_equal(lp, b.leader_prep)
    d_rows = torch.from_numpy(rows).cuda()
    ls2 = v.new_state(0, b.n)
    lp2, lst2 = v.prepare_init(ls2, b.nonces, b.public, d_rows[:, :s.leader_input_share])
    assert (lst2 == 0).all()
    np.testing.assert_array_equal(lp2, b.leader_prep)
    hrows = torch.zeros((b.n, 64), dtype=torch.uint8)
    hrows[:, :s.helper_input_share] = torch.from_numpy(b.helper_in)
    hs = v.new_state(1, b.n)
    hagg = v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, b.nonces, b.public, hrows.cuda()[:, :s.helper_input_share], lp,
                              agg=hagg)
    assert (hst == 0).all()
    np.testing.assert_array_equal(msgs, b.prep_msg)
    lagg = v.new_aggregate(1)
    v.prepare_next(ls2, msgs, lst2, want_output_shares=False, agg=lagg)
    assert lagg.read(0)[0] == expected_aggregate(b, "leader")[0]
    assert hagg.read(0)[0] == expected_aggregate(b, "helper")[0]
    # a packed call on the same state after a pitched one reads packed rows again
    lp3, _ = v.prepare_init(ls2, b.nonces, b.public, b.leader_in)
    np.testing.assert_array_equal(lp3, b.leader_prep)
    for bad in (s.leader_input_share - 16, lp_pitch + 8):
        with pytest.raises(Prio3GpuError):
            ls2.set_input_pitch(bad)


@pytest.mark.parametrize("name,capacity,opts", [("fp16_300", 10_000_000, {"helper_snap": 0}),
                                                ("fp16_5000", 8_000_000, {}),
                                                ("sumvec_8_1000", 3_000_000, {})],
                         ids=["fp16_300_rows", "fp16_5000_snap", "sumvec_8_1000"])
def test_state_beyond_device_memory_is_capacity_error(name, capacity, opts):
    """A helper state sized past the device's HBM is refused by prio3gpu_state_create with
    PRIO3GPU_E_CAPACITY (-4) before anything is allocated -- not a HIP out-of-memory error from a
    call halfway through a batch -- and the same context then prepares a normal batch bit-exact
    (every per-state buffer is sized at creation, so calls never allocate)."""
    import torch
    from janus_amd._lib import Prio3GpuError
    b = batch(name)
    v = gpu_vdaf(b)
    for k, val in opts.items():
        v.set_option(k, val)
    free, total = torch.cuda.mem_get_info()
    with pytest.raises(Prio3GpuError) as e:
        v.new_state(1, capacity)
    assert "(-4)" in str(e.value) and "bytes of device memory" in str(e.value), str(e.value)
    assert torch.cuda.mem_get_info()[0] >= free - (64 << 20)  # nothing was left allocated
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    assert (lst == 0).all()
    np.testing.assert_array_equal(lp, b.leader_prep)
    hagg, lagg = v.new_aggregate(1), v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, b.nonces, b.public, b.helper_in, lp, agg=hagg)
    assert (hst == 0).all()
    np.testing.assert_array_equal(msgs, b.prep_msg)
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    assert lagg.read(0) == expected_aggregate(b, "leader")
    assert hagg.read(0) == expected_aggregate(b, "helper")


@pytest.mark.parametrize("name,n", [("sumvec_8_1000", 129), ("sumvec_8_1000", 200),
                                    ("hist256", 191), ("countvec15", 257),
                                    ("sumvec_odd_calls", 130), ("fp16_300", 130),
                                    ("fp64_4", 200), ("sum32", 300), ("count", 1000),
                                    ("sumvec_calls1", 70), ("hist_calls1", 70),
                                    ("sumvec_calls3", 70)])
def test_ragged_multiwave_batches_match_c_restatement(name, n):
    """Batches that end inside a wave and inside a block (k_flp_weights: 2 waves per block, lane
    per report, dead lanes computing on a clamped row; k_jr / k_expand: 4 waves per block; the
    FixedPoint chain kernels: 64 / 128 reports per workgroup, several workgroups): both
    aggregators' prep shares, the prep messages and both aggregates equal the C restatement's
    (oracle/prio3_ref.c, itself cross-checked against the Python oracle), report for report."""
    from oracle import prio3 as O
    from oracle.ref import Prio3Ref
    from janus_amd.prio3 import Prio3Gpu
    c = CONFIGS[name]
    vk = O.synth_verify_key(b"ragged")
    ref = Prio3Ref(c["kind"], vk, c["bits"], c["length"], c["chunk"])
    g = ref.gen(b"ragged-" + name.encode(), 0, n, threads=8)
    res = ref.prepare_batch(g["nonces"], g["public"], g["leader_in"], g["helper_in"], threads=8)
    assert (res["status"] == 0).all() and res["count"] == n
    v = Prio3Gpu(c["kind"], vk, bits=c["bits"], length=c["length"], chunk_length=c["chunk"])
    ls, hs = v.new_state(0, n), v.new_state(1, n)
    lp, lst = v.prepare_init(ls, g["nonces"], g["public"], g["leader_in"])
    assert (lst == 0).all()
    np.testing.assert_array_equal(lp, res["lprep"])
    hp, hst = v.prepare_init(hs, g["nonces"], g["public"], g["helper_in"])
    assert (hst == 0).all()
    np.testing.assert_array_equal(hp, res["hprep"])
    hs2 = v.new_state(1, n)
    hagg, lagg = v.new_aggregate(1), v.new_aggregate(1)
    msgs, hst = v.helper_init(hs2, g["nonces"], g["public"], g["helper_in"], lp, agg=hagg)
    assert (hst == 0).all()
    np.testing.assert_array_equal(msgs, res["msgs"])
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    (la, lc), (ha, hc) = lagg.read(0), hagg.read(0)
    assert lc == hc == n
    assert la == res["agg_l"].tobytes() and ha == res["agg_h"].tobytes()
