"""XofTurboShake128 mode (prio3gpu_ctx_create2(..., PRIO3GPU_XOF_TURBOSHAKE128, ...)): the GPU's
Keccak-p[1600, 12] streams against the oracle's XofTurboShake128 (RFC 9861 TurboSHAKE128, domain
byte 0x01; tests/test_oracle.py pins the permutation and the RFC vectors).  Janus 0.6 runs
XofShake128 (aggregator/src/aggregator.rs:73); this draft-irtf-cfrg-vdaf-08+ mode is forward
compatibility: PARITY UNPINNED against any Prio3 implementation -- only against the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAMES = ["count", "sum8", "sumvec_small", "countvec15", "hist4", "hist256", "fp16_3"]


def _setup(name, n=6):
    from oracle import prio3 as O
    from janus_amd.prio3 import XOF_TURBOSHAKE128, Prio3Gpu
    from tests.reports import CONFIGS, make_batch
    b = make_batch(name, n, xof=O.XofTurboShake128)
    c = CONFIGS[name]
    v = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                 chunk_length=c["chunk"], xof=XOF_TURBOSHAKE128)
    return b, v


@pytest.mark.parametrize("name", NAMES)
def test_turboshake_transcript_bit_exact(name):
    """prepare_init (both aggregators), prep msgs and output shares == the oracle's transcript."""
    b, v = _setup(name)
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    hp, hst = v.prepare_init(hs, b.nonces, b.public, b.helper_in)
    assert (lst == 0).all() and (hst == 0).all()
    np.testing.assert_array_equal(lp, b.leader_prep)
    np.testing.assert_array_equal(hp, b.helper_prep)
    msgs, st = v.prepare_shares_to_prepare_message(lp, hp)
    assert (st == 0).all()
    np.testing.assert_array_equal(msgs, b.prep_msg)
    lo, lst = v.prepare_next(ls, msgs, lst.copy())
    ho, hst = v.prepare_next(hs, msgs, hst.copy())
    assert (lst == 0).all() and (hst == 0).all()
    np.testing.assert_array_equal(lo, b.leader_out)
    np.testing.assert_array_equal(ho, b.helper_out)


@pytest.mark.parametrize("name", ["count", "sum8", "sumvec_small", "hist4"])
def test_turboshake_helper_init_and_shard(name):
    """Fused helper aggregate-init and the GPU client shard in TurboSHAKE mode; a SHAKE128
    context rejects every TurboSHAKE report (the two XOFs do not interoperate)."""
    from janus_amd.prio3 import Prio3Gpu
    from tests.reports import CONFIGS, expected_aggregate, meas_array, plaintext_sum
    b, v = _setup(name)
    st = v.new_state(1, b.n)
    pub, lead, helper = v.shard(st, b.nonces, meas_array(b), b.rand)
    np.testing.assert_array_equal(helper, b.helper_in)
    np.testing.assert_array_equal(lead, b.leader_in)
    if v.sizes.public_share:
        np.testing.assert_array_equal(pub, b.public)
    ls, hs = v.new_state(0, b.n), v.new_state(1, b.n)
    lp, lst = v.prepare_init(ls, b.nonces, b.public, b.leader_in)
    hagg, lagg = v.new_aggregate(1), v.new_aggregate(1)
    msgs, hst = v.helper_init(hs, b.nonces, b.public, b.helper_in, lp, agg=hagg)
    assert (hst == 0).all()
    v.prepare_next(ls, msgs, lst, want_output_shares=False, agg=lagg)
    la, ha = lagg.read(0)[0], hagg.read(0)[0]
    assert la == expected_aggregate(b, "leader")[0] and ha == expected_aggregate(b, "helper")[0]
    assert v.unshard([la, ha]) == plaintext_sum(b)
    c = CONFIGS[name]
    vs = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                  chunk_length=c["chunk"])
    ls2, hs2 = vs.new_state(0, b.n), vs.new_state(1, b.n)
    lp2, _ = vs.prepare_init(ls2, b.nonces, b.public, b.leader_in)
    _, hst2 = vs.helper_init(hs2, b.nonces, b.public, b.helper_in, lp2)
    assert (hst2 == 5).all()
