"""BatchAggregation records: the host-owned half of the accumulation contract.

The engine accumulates what is arithmetic (aggregate share, report count, ReportIdChecksum) per
segment on the device. The rest of a Janus batch aggregation row is bookkeeping that stays on the
host, mirrored here:

  * client_timestamp_interval: the smallest interval holding Interval::from_time(t) of EVERY report
    aggregation written for the batch identifier, failed ones included
    (aggregation_job_writer.rs:641-663; Interval merge core/src/time.rs:294-317);
  * aggregation_jobs_created / aggregation_jobs_terminated: +1 per job first written while in
    progress (InitialWrite, aggregation_job_writer.rs:335-363) / per job updated into a terminal
    state (UpdateWrite, :394-420);
  * aggregate_share = None while no finished report has been merged
    (BatchAggregationState::Aggregating, models.rs:1275-1320);
  * merged_with: only Aggregating rows merge; Collected -> AlreadyCollected, Scrubbed -> Scrubbed.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

from .distributed import merge_aggregate_shares


@dataclass(frozen=True)
class Interval:
    """DAP Interval (messages/src/lib.rs:220-260): [start, start + duration), seconds."""
    start: int = 0
    duration: int = 0

    EMPTY = None  # set below

    @staticmethod
    def from_time(t: int) -> "Interval":
        """A length-1 interval containing exactly t (core/src/time.rs:313-317)."""
        return Interval(t, 1)

    @property
    def end(self) -> int:
        return self.start + self.duration

    def merge(self, other: "Interval") -> "Interval":
        """Smallest interval holding both; a zero-length interval is the identity (time.rs:294-307)."""
        if self.duration == 0:
            return other
        if other.duration == 0:
            return self
        lo, hi = min(self.start, other.start), max(self.end, other.end)
        return Interval(lo, hi - lo)


Interval.EMPTY = Interval(0, 0)


class AlreadyCollected(Exception):
    pass


class Scrubbed(Exception):
    pass


AGGREGATING, COLLECTED, SCRUBBED = "aggregating", "collected", "scrubbed"


@dataclass
class BatchAggregation:
    """models.rs:1152-1330 (BatchAggregation + BatchAggregationState)."""
    batch_identifier: int
    ord: int = 0
    client_timestamp_interval: Interval = Interval(0, 0)
    state: str = AGGREGATING
    aggregate_share: bytes | None = None
    report_count: int = 0
    checksum: bytes = bytes(32)
    aggregation_jobs_created: int = 0
    aggregation_jobs_terminated: int = 0
    field_bytes: int = 16

    def merged_with(self, other: "BatchAggregation") -> "BatchAggregation":
        if SCRUBBED in (self.state, other.state):
            raise Scrubbed("batch aggregation was scrubbed")
        if COLLECTED in (self.state, other.state):
            raise AlreadyCollected("batch aggregation was already collected")
        a, b = self.aggregate_share, other.aggregate_share
        share = merge_aggregate_shares([a, b], self.field_bytes) if a is not None and b is not None else \
            (a if b is None else b)
        return replace(self, aggregate_share=share, report_count=self.report_count + other.report_count,
                       checksum=bytes(x ^ y for x, y in zip(self.checksum, other.checksum)),
                       aggregation_jobs_created=self.aggregation_jobs_created + other.aggregation_jobs_created,
                       aggregation_jobs_terminated=self.aggregation_jobs_terminated + other.aggregation_jobs_terminated,
                       client_timestamp_interval=self.client_timestamp_interval.merge(other.client_timestamp_interval))

    def collected(self) -> "BatchAggregation":
        if self.state == SCRUBBED:
            raise Scrubbed("batch aggregation was scrubbed")
        return replace(self, state=COLLECTED)

    def scrubbed(self) -> "BatchAggregation":
        return replace(self, state=SCRUBBED, aggregate_share=None)


class Datastore:
    """In-memory stand-in for the batch_aggregations table and Datastore::run_tx
    (aggregator_core/src/datastore.rs:225-282): rows keyed by (batch identifier, ord). A transaction
    runs its closure on a snapshot of the committed rows; a serialization failure discards the
    snapshot and runs the closure again, so the closure must be pure (Janus's writer is copy-on-write
    for exactly this reason, aggregation_job_writer.rs:497-500). `inject_failures` makes the first k
    attempts fail after the closure ran (tests)."""

    def __init__(self):
        self.rows: dict[tuple[int, int], BatchAggregation] = {}
        self.attempts = 0

    def run_tx(self, fn, inject_failures: int = 0):
        tries = 0
        while True:
            tx = dict(self.rows)
            result = fn(tx)
            tries += 1
            self.attempts += 1
            if tries <= inject_failures:
                continue  # rolled back: nothing of this attempt is kept
            self.rows = tx
            return result


@dataclass
class BatchAggregationWriter:
    """AggregationJobWriter's batch-aggregation half for one engine (aggregation_job_writer.rs:
    476-553, 608-708). Per aggregation job, the engine turns the job's resident batch into one delta
    per batch identifier (share, count, checksum of the job's finished reports:
    jx_batch_aggregate_records, which changes nothing on the engine); inside a datastore transaction
    the writer reads the rows at a random shard `ord` in [0, shard_count) and merges each delta into
    the row it read (merged_with), together with the host-side bookkeeping: the client timestamp
    interval over every report aggregation of the job (failed ones included) and the job counters.
    Rows that are collected or scrubbed are not updated, and their reports fail with BatchCollected.
    A retried transaction recomputes everything from the resident batch, so a retry writes exactly
    what one attempt would."""
    field_bytes: int = 16
    shard_count: int = 1
    datastore: Datastore = field(default_factory=Datastore)
    seed: int = 0

    def __post_init__(self):
        import random
        self._rng = random.Random(self.seed)

    def write_job(self, engine, batch_id: int, n: int, accept, segment_index, segment_ids: list[int],
                  report_times: list[tuple[int, int]], initial_write: bool, terminal: bool,
                  inject_failures: int = 0) -> set[int]:
        """Write one aggregation job's batch aggregations. accept / segment_index: per row of the
        engine batch (None: no engine batch, e.g. a job whose reports all failed before the
        engine); segment_ids[k]: the batch identifier of dense index k; report_times: (batch
        identifier, client time) of every report aggregation the job writes. Returns the batch
        identifiers that were already collected (their reports fail with BatchCollected)."""
        ids = list(dict.fromkeys(int(s) for s in segment_ids))
        intervals: dict[int, Interval] = {}
        for s, t in report_times:
            s = int(s)
            intervals[s] = intervals.get(s, Interval.EMPTY).merge(Interval.from_time(int(t)))
            if s not in ids:
                ids.append(s)
        dense = {s: k for k, s in enumerate(segment_ids)}
        created = 1 if initial_write and not terminal else 0
        terminated = 1 if not initial_write and terminal else 0

        def closure(tx) -> set[int]:
            ord_ = self._rng.randrange(self.shard_count)
            recs = (engine.aggregate_records(batch_id, n, accept, segment_index, len(segment_ids))
                    if batch_id and n and segment_ids else [])
            collected = set()
            for s in ids:
                row = tx.get((s, ord_))
                if row is not None and row.state != AGGREGATING:
                    collected.add(s)
                    continue
                share, cnt, cs = recs[dense[s]] if s in dense and recs else (None, 0, bytes(32))
                delta = BatchAggregation(s, ord_, intervals.get(s, Interval.EMPTY), AGGREGATING,
                                         share if cnt else None, cnt, cs, created, terminated, self.field_bytes)
                tx[(s, ord_)] = delta if row is None else row.merged_with(delta)
            return collected

        return self.datastore.run_tx(closure, inject_failures)

    def batch_aggregation(self, segment: int) -> BatchAggregation:
        """The batch identifier's rows merged over every shard ord (as collection merges them,
        aggregate_share.rs:55-96)."""
        rows = [r for (s, _), r in sorted(self.datastore.rows.items()) if s == segment]
        if not rows:
            return BatchAggregation(segment, field_bytes=self.field_bytes)
        out = rows[0]
        for r in rows[1:]:
            out = out.merged_with(r)
        return out

    def segments(self) -> list[int]:
        return sorted({s for s, _ in self.datastore.rows})
