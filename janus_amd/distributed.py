"""Report sharding across GPUs and the combine of per-GPU batch-aggregation shards.

Janus spreads one batch's accumulation over `batch_aggregation_shard_count` rows: each
aggregation-job writer adds into a random shard `ord` (aggregation_job_writer.rs:527) and
`compute_aggregate_share` later merges every shard with `Aggregatable::merge`, sums the
report counts and XORs the report-id checksums (aggregator/src/aggregator/aggregate_share.rs:
55-96). Here a shard is one GPU: reports are split into contiguous ranges, every rank
prepares and accumulates its own range with no data-path communication, and the partials
are combined once at the end. RCCL's reduction ops know nothing of field arithmetic, so
the exchange is an all-gather of fixed-size shard records followed by a mod-p merge
(SURVEY.md §8(e)).

Shard record (the unit that crosses xGMI), little-endian:
    aggregate share  OUT x FB bytes (encoded field elements, the BYTEA of
                     batch_aggregations.aggregate_share, db/00000000000001_initial_schema.up.sql:308)
    report count     8 bytes (u64)
    checksum         32 bytes (ReportIdChecksum, core/src/report_id.rs:19-42)

The device merge runs in the engine (jx_shard_record_combine_device); `merge_records` is
the same merge on the host, used where Janus itself merges on the host (the collection
side) and by the gloo tests.
"""
from __future__ import annotations

import numpy as np

P64 = 2**64 - 2**32 + 1
P128 = 2**128 - 28 * 2**64 + 1
RECORD_TAIL = 8 + 32


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous report range [start, stop) owned by `rank` of `world` (remainder to the first ranks)."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError(f"bad shard request n={n} rank={rank} world={world}")
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def record_bytes(output_len: int, field_bytes: int) -> int:
    return output_len * field_bytes + RECORD_TAIL


def pack_record(aggregate_share: bytes, count: int, checksum: bytes) -> np.ndarray:
    if len(checksum) != 32:
        raise ValueError("checksum must be 32 bytes")
    return np.frombuffer(bytes(aggregate_share) + int(count).to_bytes(8, "little") + bytes(checksum),
                         np.uint8).copy()


def unpack_record(rec, field_bytes: int) -> tuple[bytes, int, bytes]:
    b = bytes(np.asarray(rec, dtype=np.uint8).tobytes())
    agg_len = len(b) - RECORD_TAIL
    if agg_len < 0 or agg_len % field_bytes:
        raise ValueError("malformed shard record")
    return b[:agg_len], int.from_bytes(b[agg_len:agg_len + 8], "little"), b[agg_len + 8:]


def merge_aggregate_shares(parts: list[bytes], field_bytes: int) -> bytes:
    """Element-wise mod-p sum of encoded aggregate shares (Aggregatable::merge).

    A non-canonical element (>= p) is a decode error, as in prio's field decoding."""
    p = P64 if field_bytes == 8 else P128
    if not parts:
        raise ValueError("nothing to merge")
    n = len(parts[0])
    if any(len(x) != n for x in parts) or n % field_bytes:
        raise ValueError("aggregate shares of different lengths")
    acc = [0] * (n // field_bytes)
    for part in parts:
        for i in range(len(acc)):
            v = int.from_bytes(part[i * field_bytes:(i + 1) * field_bytes], "little")
            if v >= p:
                raise ValueError("aggregate share element is not canonical")
            acc[i] += v
    return b"".join((v % p).to_bytes(field_bytes, "little") for v in acc)


def merge_records(records, field_bytes: int) -> tuple[bytes, int, bytes]:
    """compute_aggregate_share over shard records: (aggregate share, report count, checksum)."""
    parts, count, cs = [], 0, bytearray(32)
    for rec in records:
        agg, c, k = unpack_record(rec, field_bytes)
        parts.append(agg)
        count += c
        for i in range(32):
            cs[i] ^= k[i]
    return merge_aggregate_shares(parts, field_bytes), count, bytes(cs)


def all_gather_records(record, group=None):
    """All-gather one fixed-size uint8 shard record per rank (a torch tensor on the
    backend's device: CUDA for RCCL, CPU for gloo). Returns a [world, record_bytes] tensor."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    out = torch.empty((world, record.numel()), dtype=torch.uint8, device=record.device)
    dist.all_gather(list(out.unbind(0)), record.contiguous(), group=group)
    return out


class ShardCombiner:
    """Device-side gather + merge of an engine's batch aggregation across ranks.

    export -> RCCL all-gather (one collective of world x record_bytes) -> device merge.
    Every rank ends up with the merged record (all-gather, not gather: any rank can serve
    the aggregate share). The engine runs on its own HIP stream; the three steps are ordered
    with stream waits (engine stream -> torch's current stream, on which the collective's
    result is ready -> engine stream), so a combine never blocks the host. The record, gather
    and merge buffers are allocated once and live as long as the combiner, so no buffer the
    engine stream may still read is ever handed back to torch's allocator mid-flight."""

    def __init__(self, engine, group=None):
        import torch
        import torch.distributed as dist

        self.engine = engine
        self.group = group
        self.nbytes = record_bytes(engine.output_len, engine.field_bytes)
        self.dev = torch.device("cuda", engine.device)
        self.world = dist.get_world_size(group)
        self.record = torch.zeros(self.nbytes, dtype=torch.uint8, device=self.dev)
        self.gathered = torch.zeros((self.world, self.nbytes), dtype=torch.uint8, device=self.dev)
        self.merged = torch.zeros(self.nbytes, dtype=torch.uint8, device=self.dev)
        self.stream = torch.cuda.ExternalStream(engine.stream(), device=self.dev)

    def combine(self, segment: int = 0):
        """Queue export -> all-gather -> merge; the merged record is ready on the engine stream
        (engine.sync() or any later engine call orders after it)."""
        import torch
        import torch.distributed as dist

        cur = torch.cuda.current_stream(self.dev)
        self.engine.export_record_device(segment, self.record.data_ptr(), stream=False)
        # the all-gather reads the exported record and overwrites `gathered`, which the previous merge
        # (queued before the export on the engine stream) has read
        cur.wait_stream(self.stream)
        if dist.get_backend(self.group) == "gloo":  # gloo gathers host tensors (CPU tests, 1-GPU boxes)
            self.gathered.copy_(all_gather_records(self.record.cpu(), self.group))
        else:  # RCCL over xGMI into the persistent buffer; ready on the current stream when the call returns
            dist.all_gather(list(self.gathered.unbind(0)), self.record, group=self.group)
        self.stream.wait_stream(cur)  # the merge reads the gathered records
        self.engine.combine_records_device(self.gathered.data_ptr(), self.world, self.merged.data_ptr(), stream=False)
        return self.merged

    def result(self) -> tuple[bytes, int, bytes]:
        self.engine.sync()
        return unpack_record(self.merged.cpu().numpy(), self.engine.field_bytes)
