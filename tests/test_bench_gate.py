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
