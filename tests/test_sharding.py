"""Shard planners vs the reference formulas and the SURVEY.md §2.8 golden tables."""
import pytest

from ddl_amd.models.layout import TENSORS, NUM_TENSORS, TOTAL_NUMEL, TOTAL_BYTES
from ddl_amd.parallel.sharding import (make_plan, greedy_order, reference_route, balance_table,
                                       contiguous_counts, segment_aligned_num_ps, host_imbalance,
                                       segment_ps_counts)


def test_layout_constants():
    # SURVEY.md §2.5
    assert NUM_TENSORS == 14
    assert TOTAL_NUMEL == 2_656_010
    assert TOTAL_BYTES == 10_624_040
    assert [t.numel for t in TENSORS][:4] == [800, 32, 51200, 64]


def test_greedy_order_golden():
    # mnist_sync_sharding_greedy/worker.py:13-37 replayed
    assert greedy_order([t.numel for t in TENSORS]) == [13, 8, 1, 6, 3, 10, 5, 4, 7, 2, 11, 12, 0, 9]


def test_greedy_order_odd_count():
    assert greedy_order([5, 1, 3]) == [1, 0, 2]


@pytest.mark.parametrize("P,expect", [
    (1, [1.00, 1.00]), (2, [1.19, 1.80]), (3, [1.78, 2.11]), (4, [2.81, 2.02]),
    (5, [2.97, 1.97]), (6, [2.37, 2.37]), (7, [2.77, 2.76]), (8, [4.76, 3.16])])
def test_balance_table_matches_survey(P, expect):
    c = make_plan("contiguous", P).imbalance()
    g = make_plan("greedy", P).imbalance()
    assert round(c, 2) == pytest.approx(expect[0], abs=0.011)
    assert round(g, 2) == pytest.approx(expect[1], abs=0.011)


def test_contiguous_p2_shard_sizes():
    mib = [b / 2**20 for b in make_plan("contiguous", 2).shard_bytes()]
    assert mib[0] == pytest.approx(4.11, abs=0.01) and mib[1] == pytest.approx(6.03, abs=0.01)


@pytest.mark.parametrize("P", range(1, 15))
def test_contiguous_matches_reference_routing(P):
    plan = make_plan("contiguous", P)
    for i in range(NUM_TENSORS):
        owner, tag = reference_route(i, NUM_TENSORS, P)
        assert plan.owner[i] == owner
        # tag = index local to the owning PS, as the reference PS receives it
        assert plan.tensors_of(owner).index(i) == tag


@pytest.mark.parametrize("P", range(1, 15))
def test_greedy_matches_reference_routing(P):
    plan = make_plan("greedy", P)
    order = plan.meta["reference_order"]
    for pos, i in enumerate(order):
        owner, _ = reference_route(pos, NUM_TENSORS, P)
        assert plan.owner[i] == owner


@pytest.mark.parametrize("policy", ["contiguous", "greedy", "lpt", "flat"])
@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_plan_is_a_partition(policy, P):
    plan = make_plan(policy, P)
    covered = []
    for p in range(P):
        for lo, hi in plan.ps_segments(p):
            covered.extend(range(lo, hi))
    assert sorted(covered) == list(range(plan.total))
    # every tensor lies inside the buffer, tensors don't overlap
    spans = sorted((plan.tensor_offsets[t.index], plan.tensor_offsets[t.index] + t.numel) for t in TENSORS)
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b <= c
    assert spans[-1][1] <= plan.total


def test_flat_bucketed_plan():
    buckets = [list(range(8, 14)), [6, 7], [4, 5], [0, 1, 2, 3]]
    plan = make_plan("flat", 8, buckets=buckets)
    assert plan.imbalance() == 1.0
    assert len(plan.bucket_ranges) == 4
    for lo, hi in plan.bucket_ranges:
        assert (hi - lo) % (8 * 64) == 0
    assert all(len(plan.ps_segments(p)) == 4 for p in range(8))


def test_flat_balance_is_perfect():
    for row in balance_table():
        assert row["flat"] == 1.0


def test_invalid_plans():
    with pytest.raises(ValueError):
        make_plan("contiguous", 15)      # reference divides by zero (Q8)
    with pytest.raises(ValueError):
        make_plan("none", 2)             # Q7
    with pytest.raises(ValueError):
        make_plan("bogus", 1)
    assert contiguous_counts(14, 4) == [3, 3, 3, 5]


def test_host_ranks_colocated():
    plan = make_plan("contiguous", 8)
    assert [plan.host_rank(p, 8) for p in range(8)] == list(range(8))
    assert [plan.host_rank(p, 2) for p in range(4)] == [0, 1, 0, 1]


def test_replicated_bucket_is_the_last_backward_segments():
    """the replicated (all-reduce / xGMI all-to-all) bucket of the native sync
    exchange must be the one the LAST backward segment completes — conv1 + conv2, bucket 0 in
    make_plan's min-tensor-id order — not the last index (the fc bucket, first to complete);
    an unbucketed plan (no overlap) replicates its one bucket."""
    from ddl_amd.models.layout import CANON_OFFSETS, TENSORS
    from ddl_amd.parallel.native_exchange import last_segment_bucket
    segs = [[8, 9, 10, 11, 12, 13], [6, 7], [4, 5], [0, 1, 2, 3]]  # HIP engine order
    for W in (1, 2, 4, 8):
        plan = make_plan("flat", W, buckets=segs)
        b = last_segment_bucket(plan, segs)
        lo, hi = plan.bucket_ranges[b]
        assert sorted(plan.meta["buckets"][b]) == [0, 1, 2, 3]
        assert hi - lo < 60000  # 52,160 parameters (+ padding to a multiple of 4 W)
    plan = make_plan("flat", 2)
    assert last_segment_bucket(plan, segs) == 0 and len(plan.bucket_ranges) == 1


SEGS = [list(range(8, 14)), [6, 7], [4, 5], [0, 1, 2, 3]]  # models.HIP_SEGMENTS until round 5


@pytest.mark.parametrize("P", [4, 5, 6, 8, 16])
def test_segment_aligned_flat_plan(P):
    """Async flat plan: one range per PS, every range inside one backward segment, ranges
    tile the buffer, 16-B aligned, every tensor inside its segment's ranges."""
    plan = make_plan("flat", P, buckets=SEGS, segment_aligned=True)
    assert plan.num_ps == P and len(plan.ps_ranges) == P
    assert sum(plan.meta["ps_per_group"]) == P and min(plan.meta["ps_per_group"]) >= 1
    pos = 0
    for p in range(P):
        lo, hi = plan.ps_segments(p)[0]
        assert lo == pos and hi > lo and lo % 4 == 0 and (hi - lo) % 4 == 0
        pos = hi
        segs = {s for s, ts in enumerate(SEGS) for t in ts
                if plan.tensor_offsets[t] < hi and plan.tensor_offsets[t] + TENSORS[t].numel > lo}
        assert len(segs) == 1, (p, segs)
    assert pos == plan.total
    for t in TENSORS:
        o = plan.tensor_offsets[t.index]
        assert o % 64 == 0 and o + t.numel <= plan.total


def test_segment_aligned_ps_counts():
    """P is the smallest multiple of W with a PS per segment and per-host load within 1.25x
    (the async critical path then carries only the last segment's 52 K-element shard)."""
    got = {W: segment_aligned_num_ps(W, SEGS) for W in (1, 2, 3, 4, 8)}
    assert got == {1: 4, 2: 6, 3: 9, 4: 8, 8: 8}
    for W, P in got.items():
        plan = make_plan("flat", P, buckets=SEGS, segment_aligned=True)
        assert host_imbalance(plan, W) <= 1.25
    assert segment_ps_counts([10, 10, 80], 3) == [1, 1, 1]
    assert segment_ps_counts([10, 10, 80], 10) == [1, 1, 8]
    with pytest.raises(ValueError):
        make_plan("flat", 3, buckets=SEGS, segment_aligned=True)
    with pytest.raises(ValueError):
        make_plan("contiguous", 4, buckets=SEGS, segment_aligned=True)


def test_async_groups_merge_the_tiny_head_segment():
    """The HIP engine's segment 0 holds only fc3 (5,130 parameters: fc1 / fc2's weight
    gradients run in the conv4 dual launch since round 6); the async plan folds it into the
    segment completed after it instead of spending a PS per host on it."""
    from ddl_amd.models import HIP_SEGMENTS
    from ddl_amd.parallel.sharding import async_groups
    g = async_groups(HIP_SEGMENTS)
    assert g == [list(range(6, 14)), [4, 5], [0, 1, 2, 3]]
    got = {W: segment_aligned_num_ps(W, g) for W in (1, 2, 4, 8)}
    assert got == {1: 3, 2: 4, 4: 8, 8: 8}
    for W, P in got.items():
        plan = make_plan("flat", P, buckets=g, segment_aligned=True)
        assert host_imbalance(plan, W) <= 1.25
    # a plan whose groups are all large is left alone
    assert async_groups(SEGS) == [sorted(x) for x in SEGS]
