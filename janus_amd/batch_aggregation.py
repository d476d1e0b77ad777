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


@dataclass
class BatchAggregationWriter:
    """The batch-aggregation bookkeeping of AggregationJobWriter for one engine: the device holds the
    per-segment share / count / checksum; this object holds the per-segment interval and job counters
    and assembles BatchAggregation rows (segment = batch identifier)."""
    field_bytes: int = 16
    ord: int = 0
    intervals: dict[int, Interval] = field(default_factory=dict)
    jobs_created: dict[int, int] = field(default_factory=dict)
    jobs_terminated: dict[int, int] = field(default_factory=dict)

    def observe_report_aggregations(self, segments, times) -> None:
        """Every report aggregation written for a batch identifier widens its client timestamp
        interval, whatever its state (aggregation_job_writer.rs:641-663)."""
        for s, t in zip(segments, times):
            s = int(s)
            self.intervals[s] = self.intervals.get(s, Interval.EMPTY).merge(Interval.from_time(int(t)))

    def observe_job(self, segments, initial_write: bool, terminal: bool) -> None:
        """One aggregation job touching `segments`: InitialWrite of an in-progress job counts as
        created, UpdateWrite into a terminal state as terminated (aggregation_job_writer.rs:335-420)."""
        for s in set(int(x) for x in segments):
            if initial_write and not terminal:
                self.jobs_created[s] = self.jobs_created.get(s, 0) + 1
            elif not initial_write and terminal:
                self.jobs_terminated[s] = self.jobs_terminated.get(s, 0) + 1

    def batch_aggregation(self, engine, segment: int) -> BatchAggregation:
        agg, count, checksum = engine.aggregate_share(segment)
        return BatchAggregation(segment, self.ord, self.intervals.get(segment, Interval.EMPTY), AGGREGATING,
                                agg if count else None, count, checksum, self.jobs_created.get(segment, 0),
                                self.jobs_terminated.get(segment, 0), self.field_bytes)

    def segments(self) -> list[int]:
        return sorted(set(self.intervals) | set(self.jobs_created) | set(self.jobs_terminated))
