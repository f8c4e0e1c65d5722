"""Speculative accumulation (k_jr column sums + k_accum_spec) vs the direct accumulation path.

Large batches (several 64-report waves) are made by the GPU client shard, which is itself
parity-tested against the oracle (test_gpu_parity.py::test_gpu_shard_matches_oracle).  Batch slots
mix uniform waves (speculative) with a mixed wave (direct), the last wave is partial (clamped rows
are subtracted again), and tampered reports are rejected after k_jr has already counted them.
Expected aggregates = plaintext sums of the accepted reports per slot
(integration_tests/tests/common/mod.rs:225-398 semantics), and both paths agree byte for byte.
"""
import os

import numpy as np
import pytest

from tests.reports import CONFIGS

pytestmark = pytest.mark.gpu


def _vdaf(name, speculate):
    from janus_amd.prio3 import Prio3Gpu
    c = CONFIGS[name]
    old = os.environ.get("PRIO3GPU_SPECULATE")
    os.environ["PRIO3GPU_SPECULATE"] = "1" if speculate else "0"
    try:
        return Prio3Gpu(c["kind"], bytes(range(16)), bits=c["bits"], length=c["length"],
                        chunk_length=c["chunk"])
    finally:
        if old is None:
            del os.environ["PRIO3GPU_SPECULATE"]
        else:
            os.environ["PRIO3GPU_SPECULATE"] = old


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
