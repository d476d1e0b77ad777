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
    """Stands in for HelperEngine.aggregate_records (the device half): per-row output shares of one
    resident batch, reduced per dense segment index under the accept mask. Counts its calls."""

    def __init__(self, outs, ids):
        self.outs, self.ids, self.calls = outs, ids, 0

    def aggregate_records(self, batch_id, n, accept, seg_index, nseg):
        import hashlib
        self.calls += 1
        recs = []
        for k in range(nseg):
            rows = [r for r in range(n) if accept[r] and seg_index[r] == k]
            share = enc([sum(self.outs[r][j] for r in rows) % P128 for j in range(2)])
            cs = bytes(32)
            for r in rows:
                cs = bytes(x ^ y for x, y in zip(cs, hashlib.sha256(self.ids[r]).digest()))
            recs.append((share, len(rows), cs))
        return recs


def _job(w, eng, inject=0):
    # 4 rows in two batch identifiers (dense 0 -> id 1, 1 -> id 2); row 2 (id 2) failed
    return w.write_job(eng, 7, 4, [1, 1, 0, 1], [0, 0, 1, 0], [1, 2], [(1, 1000), (1, 1030), (2, 2000), (1, 990)],
                       initial_write=True, terminal=True, inject_failures=inject)


def test_writer_records_all_reports_and_none_share():
    w = BatchAggregationWriter(field_bytes=16)
    eng = _FakeEngine([[5, 6], [1, 1], [9, 9], [P128 - 1, 0]], [bytes([i]) * 16 for i in range(4)])
    assert _job(w, eng) == set()
    b1, b2 = w.batch_aggregation(1), w.batch_aggregation(2)
    assert b1.client_timestamp_interval == Interval(990, 41) and b1.report_count == 3
    assert b1.aggregate_share == enc([5, 7])
    assert b2.client_timestamp_interval == Interval(2000, 1)  # the failed report's time still counts
    assert b2.aggregate_share is None and b2.report_count == 0
    assert (b1.aggregation_jobs_created, b1.aggregation_jobs_terminated) == (0, 0)  # one-round helper
    # leader: creation in progress, then the update into a terminal state
    w.write_job(eng, 0, 0, None, None, [], [(1, 5), (2, 6)], initial_write=True, terminal=False)
    w.write_job(eng, 0, 0, None, None, [], [(1, 5), (2, 6)], initial_write=False, terminal=True)
    b2 = w.batch_aggregation(2)
    assert (b2.aggregation_jobs_created, b2.aggregation_jobs_terminated) == (1, 1)
    assert w.segments() == [1, 2]


def test_retried_transaction_writes_what_one_attempt_writes():
    """ADVICE/VERDICT r2: the run_tx closure is pure. Two rolled-back attempts recompute the deltas from
    the resident batch (the engine is asked three times) and the committed rows equal a single attempt's;
    nothing of the failed attempts is double counted."""
    outs, ids = [[5, 6], [1, 1], [9, 9], [P128 - 1, 0]], [bytes([i]) * 16 for i in range(4)]
    once, twice = BatchAggregationWriter(seed=3), BatchAggregationWriter(seed=3)
    e1, e2 = _FakeEngine(outs, ids), _FakeEngine(outs, ids)
    for _ in range(2):  # two jobs, so the second merges into the rows the first wrote
        _job(once, e1)
        _job(twice, e2, inject=2)
    assert e1.calls == 2 and e2.calls == 6 and twice.datastore.attempts == 6
    assert once.datastore.rows == twice.datastore.rows
    assert twice.batch_aggregation(1).report_count == 6


def test_shard_ords_merge_at_collection():
    """Rows are written at a random ord per transaction; collection merges every ord."""
    w = BatchAggregationWriter(shard_count=4, seed=11)
    eng = _FakeEngine([[1, 2], [3, 4], [0, 0], [5, 6]], [bytes([i]) * 16 for i in range(4)])
    for _ in range(8):
        _job(w, eng)
    ords = {o for (s, o) in w.datastore.rows if s == 1}
    assert len(ords) > 1
    b1 = w.batch_aggregation(1)
    assert b1.report_count == 24 and b1.aggregate_share == enc([8 * 9, 8 * 12])


def test_collected_batch_is_not_updated():
    w = BatchAggregationWriter()
    eng = _FakeEngine([[1, 2], [3, 4], [0, 0], [5, 6]], [bytes([i]) * 16 for i in range(4)])
    _job(w, eng)
    w.datastore.rows[(1, 0)] = w.datastore.rows[(1, 0)].collected()
    before = w.datastore.rows[(1, 0)]
    assert _job(w, eng) == {1}  # reports of batch 1 fail with BatchCollected
    assert w.datastore.rows[(1, 0)] == before
    assert w.batch_aggregation(2).client_timestamp_interval == Interval(2000, 1)
