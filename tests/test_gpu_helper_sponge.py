"""The helper's fused expansion + joint-rand-part pass (k_helper_sponge) vs the oracle, in its
three modes: fused (PRIO3GPU_HELPER_SPONGE=1), fused with every lane forced onto the exact
fallback (PRIO3GPU_TEST_FALLBACK=1: k_expand + k_jr re-run gated on the device flag), and the
two-pass path (the default).  Helper prep shares, prep messages and aggregates must be the oracle's
bytes in every mode (prio's helper prepare_init, aggregator.rs:1775-1797)."""
import numpy as np
import pytest

from tests.reports import CONFIGS, expected_aggregate, make_batch

pytestmark = pytest.mark.gpu

MODES = {"fused": {"PRIO3GPU_HELPER_SPONGE": "1"},
         "fallback": {"PRIO3GPU_HELPER_SPONGE": "1", "PRIO3GPU_TEST_FALLBACK": "1"},
         "twopass": {"PRIO3GPU_HELPER_SPONGE": "0"}}
SIZES = {"sum32": 70, "sum5": 24, "sumvec_small": 80, "hist256": 66, "countvec15": 24,
         "sumvec_8_1000": 6}
_cache = {}


def batch(name):
    if name not in _cache:
        _cache[name] = make_batch(name, SIZES[name])
    return _cache[name]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", list(SIZES))
def test_helper_paths_bit_exact(name, mode, monkeypatch):
    from janus_amd.prio3 import Prio3Gpu
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    b = batch(name)
    c = CONFIGS[name]
    v = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                 chunk_length=c["chunk"])
    hs = v.new_state(1, b.n)
    hp, hst = v.prepare_init(hs, b.nonces, b.public, b.helper_in)
    assert (hst == 0).all()
    np.testing.assert_array_equal(hp, b.helper_prep)
    ho, hst = v.prepare_next(hs, b.prep_msg, hst.copy())
    np.testing.assert_array_equal(ho, b.helper_out)
    hs2 = v.new_state(1, b.n)
    hagg = v.new_aggregate(1)
    msgs, st = v.helper_init(hs2, b.nonces, b.public, b.helper_in, b.leader_prep, agg=hagg)
    assert (st == 0).all()
    np.testing.assert_array_equal(msgs, b.prep_msg)
    assert hagg.read(0)[0] == expected_aggregate(b, "helper")[0]
