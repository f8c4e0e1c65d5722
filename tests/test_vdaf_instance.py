"""Janus VdafInstance -> engine parameters, as TaskAggregator::new builds the VDAF
(aggregator/src/aggregator.rs:797-861; VdafInstance core/src/task.rs:24-59, chunk_size :84-86)."""
import pytest

from janus_amd.prio3 import COUNT, FPVEC, HISTOGRAM, SUM, SUMVEC, vdaf_instance_params


@pytest.mark.parametrize("instance,expected", [
    ("Prio3Count", (COUNT, 0, 0, 0)),
    ({"Prio3Count": None}, (COUNT, 0, 0, 0)),
    ({"Prio3CountVec": {"length": 15}}, (SUMVEC, 1, 15, 3)),
    ({"Prio3Sum": {"bits": 32}}, (SUM, 32, 0, 0)),
    ({"Prio3SumVec": {"bits": 8, "length": 1000}}, (SUMVEC, 8, 1000, 89)),  # BASELINE config D
    ({"Prio3Histogram": {"length": 256}}, (HISTOGRAM, 0, 256, 16)),        # BASELINE config C
    ({"Prio3FixedPoint16BitBoundedL2VecSum": {"length": 100000}}, (FPVEC, 16, 100000, 0)),
    ({"Prio3FixedPoint32BitBoundedL2VecSum": {"length": 3}}, (FPVEC, 32, 3, 0)),
    ({"Prio3FixedPoint64BitBoundedL2VecSum": {"length": 3}}, (FPVEC, 64, 3, 0)),
])
def test_vdaf_instance_params(instance, expected):
    assert vdaf_instance_params(instance) == expected


@pytest.mark.parametrize("instance", [{"Poplar1": {"bits": 8}}, "Fake", {"a": 1, "b": 2}, 3])
def test_non_prio3_instances_rejected(instance):
    with pytest.raises(ValueError):
        vdaf_instance_params(instance)


@pytest.mark.gpu
def test_from_vdaf_instance_matches_direct_constructor():
    from janus_amd.prio3 import Prio3Gpu
    a = Prio3Gpu.from_vdaf_instance({"Prio3SumVec": {"bits": 8, "length": 1000}}, bytes(16))
    b = Prio3Gpu.new_sum_vec(8, 1000, 89, bytes(16))
    fields = [f for f, _ in type(a.sizes)._fields_]
    assert [getattr(a.sizes, f) for f in fields] == [getattr(b.sizes, f) for f in fields]
    assert a.sizes.leader_input_share == 134944 and a.sizes.prep_share == 2896
