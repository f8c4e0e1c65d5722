"""Host mirror: which input-share layouts janus_amd.prio3 hands the engine as pitched rows
(prio3gpu_state_set_input_pitch) and which it packs first.  CPU only: no engine
call is made."""
import numpy as np
import pytest
import torch

from janus_amd.prio3 import _as_u8, _pitched_rows


def test_column_slice_of_a_16b_aligned_buffer_is_passed_through():
    buf = np.zeros((5, 128), np.uint8)
    a, pitch = _pitched_rows(buf[:, :100], 5, 100, "x")
    assert pitch == 128 and a.base is buf


def test_packed_rows_keep_their_width():
    a, pitch = _pitched_rows(np.zeros((4, 48), np.uint8), 4, 48, "x")
    assert pitch == 48


@pytest.mark.parametrize("extra", [8, 4, 1])
def test_unaligned_pitch_is_packed(extra):
    buf = np.arange(5 * (100 + extra), dtype=np.uint64).astype(np.uint8).reshape(5, 100 + extra)
    view = buf[:, :100]
    a, pitch = _pitched_rows(view, 5, 100, "x")
    assert pitch == 100 and a.flags.c_contiguous and np.array_equal(a, view)


def test_broadcast_rows_are_packed():
    row = np.arange(48, dtype=np.uint8)
    view = np.broadcast_to(row, (6, 48))
    assert view.strides[0] == 0
    a, pitch = _pitched_rows(view, 6, 48, "x")
    assert pitch == 48 and a.flags.c_contiguous and a.nbytes == 6 * 48
    assert np.array_equal(a, view)


def test_negative_stride_is_packed():
    buf = np.arange(4 * 64, dtype=np.uint64).astype(np.uint8).reshape(4, 64)
    view = buf[::-1]
    assert view.strides[0] < 0
    a, pitch = _pitched_rows(view, 4, 64, "x")
    assert pitch == 64 and a.flags.c_contiguous and np.array_equal(a, view)


def test_torch_views():
    t = torch.zeros((4, 160), dtype=torch.uint8)
    a, pitch = _pitched_rows(t[:, :144], 4, 144, "x")
    assert pitch == 160 and a.data_ptr() == t.data_ptr()
    u = torch.arange(4 * 150, dtype=torch.int64).to(torch.uint8).reshape(4, 150)
    a, pitch = _pitched_rows(u[:, :144], 4, 144, "x")
    assert pitch == 144 and a.is_contiguous() and torch.equal(a, u[:, :144])
    e = torch.arange(48, dtype=torch.uint8).expand(3, 48)
    a, pitch = _pitched_rows(e, 3, 48, "x")
    assert pitch == 48 and a.is_contiguous() and torch.equal(a, e)


def test_wrong_size_is_an_error():
    with pytest.raises(ValueError):
        _as_u8(np.zeros((3, 10), np.uint8), 3, 11, "x")
