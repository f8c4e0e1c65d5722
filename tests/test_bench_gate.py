"""The bench's parity gate helpers (CPU): bench.leader_output_shares, the exact truncate() the gate
compares the GPU's leader output shares with, against the oracle's VdafTranscript output shares."""
import numpy as np
import pytest

from bench import leader_output_shares
from tests.reports import make_batch

KINDS = {"Count": 0, "Sum": 1, "SumVec": 2, "Histogram": 3}


@pytest.mark.parametrize("name", ["count", "sum8", "sum32", "sumvec_small", "countvec15",
                                  "sumvec_8_1000", "hist4", "hist256"])
def test_leader_output_shares_match_oracle(name):
    b = make_batch(name, 3)
    typ = b.vdaf.typ

    class Sizes:
        field_size = b.leader_out.shape[1] // typ.OUTPUT_LEN
        meas_len = typ.MEAS_LEN

    got = leader_output_shares(b.leader_in, KINDS[type(typ).__name__], getattr(typ, "bits", 0),
                               getattr(typ, "length", 0), Sizes, b.vdaf.fld.MODULUS)
    assert np.array_equal(got, b.leader_out)


def test_flp_op_model_matches_survey_appendix_b():
    """bench.py's FLP op model (the roofline of k_flp_query_lane-bound configs) gives
    Appendix B's per-aggregator multiplication counts: Sum32 ~900, Histogram256 ~4.6K,
    SumVec(8,1000) ~128K, Count ~14."""
    import bench
    from types import SimpleNamespace as NS
    mk = lambda fs, ml, pl, vl: NS(field_size=fs, meas_len=ml, proof_len=pl, verifier_len=vl)
    assert bench.flp_mults_per_report(mk(16, 32, 128, 3), 1) == 895
    assert 4000 <= bench.flp_mults_per_report(mk(16, 256, 95, 34), 3) <= 4700
    assert 115000 <= bench.flp_mults_per_report(mk(16, 8000, 433, 180), 2) <= 130000
    assert bench.flp_mults_per_report(mk(8, 1, 5, 4), 0) == 14


def test_flp_weights_bytes_model():
    """k_flp_weights' algorithmic bytes per report (bench.py roofline.hbm_weights): SumVec(8,1000)
    reads 255 gadget coefficients + t, r and writes a 274-entry weight row, 12 block-start prefix
    products (written and read back), v, p(t) and the 16-byte part copy."""
    import bench
    from types import SimpleNamespace as NS
    s = NS(field_size=16, meas_len=8000, proof_len=433, verifier_len=180)
    assert bench.flp_weights_bytes_per_report(s) == (255 + 2 + 274 + 24 + 2) * 16 + 32
    assert 3.4e9 < 393216 * bench.flp_weights_bytes_per_report(s) < 3.6e9
