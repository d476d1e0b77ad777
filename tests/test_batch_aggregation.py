"""Host-side half of the batch-aggregation contract (janus_amd/batch_aggregation.py) against the
reference semantics of BatchAggregation::merged_with (aggregator_core/src/datastore/models.rs:
1275-1320), Interval merging (core/src/time.rs:294-317) and the AggregationJobWriter counters
(aggregator/src/aggregator/aggregation_job_writer.rs:335-420, 608-708)."""
import pytest

from janus_amd.batch_aggregation import (AlreadyCollected, BatchAggregation, BatchAggregationWriter, Interval,
                                         Scrubbed)

P128 = 2**128 - 28 * 2**64 + 1


def enc(vals):
    return b"".join(v.to_bytes(16, "little") for v in vals)


def test_interval_merge_semantics():
    e = Interval.EMPTY
    a = Interval.from_time(100)
    assert (a.start, a.duration) == (100, 1)
    assert e.merge(a) == a and a.merge(e) == a
    b = Interval.from_time(250)
    assert a.merge(b) == Interval(100, 151) == b.merge(a)  # end is exclusive: [100, 251)
    assert Interval(10, 5).merge(Interval(12, 1)) == Interval(10, 5)


def test_merged_with_none_shares_and_counters():
    x = BatchAggregation(7, aggregate_share=None, client_timestamp_interval=Interval.from_time(5),
                         aggregation_jobs_created=1)
    y = BatchAggregation(7, aggregate_share=enc([P128 - 1, 3]), report_count=2, checksum=bytes([1]) * 32,
                         client_timestamp_interval=Interval.from_time(9), aggregation_jobs_terminated=1)
    m = x.merged_with(y)
    assert m.aggregate_share == y.aggregate_share and m.report_count == 2
    assert (m.aggregation_jobs_created, m.aggregation_jobs_terminated) == (1, 1)
    assert m.client_timestamp_interval == Interval(5, 5)
    m2 = m.merged_with(y)
    assert m2.aggregate_share == enc([P128 - 2, 6]) and m2.checksum == bytes(32) and m2.report_count == 4
    assert x.merged_with(BatchAggregation(7)).aggregate_share is None  # (None, None) -> None
    with pytest.raises(AlreadyCollected):
        m.collected().merged_with(y)
    with pytest.raises(Scrubbed):
        y.merged_with(m.scrubbed())


class _FakeEngine:
    """Stands in for HelperEngine.aggregate_share (the device half)."""

    def __init__(self, rows):
        self.rows = rows

    def aggregate_share(self, seg):
        return self.rows.get(seg, (enc([0, 0]), 0, bytes(32)))


def test_writer_records_all_reports_and_none_share():
    w = BatchAggregationWriter(field_bytes=16)
    # helper job: 4 reports in two batch identifiers, one of which only has a failed report
    w.observe_report_aggregations([1, 1, 2, 1], [1000, 1030, 2000, 990])
    w.observe_job([1, 1, 2, 1], initial_write=True, terminal=True)  # one-round helper: no counter moves
    eng = _FakeEngine({1: (enc([5, 6]), 2, bytes([3]) * 32)})
    b1, b2 = w.batch_aggregation(eng, 1), w.batch_aggregation(eng, 2)
    assert b1.client_timestamp_interval == Interval(990, 41) and b1.report_count == 2
    assert b2.client_timestamp_interval == Interval(2000, 1)  # the failed report's time still counts
    assert b2.aggregate_share is None and b2.report_count == 0
    assert (b1.aggregation_jobs_created, b1.aggregation_jobs_terminated) == (0, 0)
    # leader: creation in progress, then the update into a terminal state
    w.observe_job([1, 2], initial_write=True, terminal=False)
    w.observe_job([1, 2, 2], initial_write=False, terminal=True)
    assert (w.batch_aggregation(eng, 2).aggregation_jobs_created, w.batch_aggregation(eng, 2).aggregation_jobs_terminated) == (1, 1)
    assert w.segments() == [1, 2]
