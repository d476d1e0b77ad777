"""Helper aggregate-init over a batch of PrepareInits — the hot loop of Janus, batched.

Mirror of VdafOps::handle_aggregate_init_generic, /root/reference/aggregator/src/
aggregator.rs:1712-2161, minus what stays on the host and is out of scope here
(HPKE open :1772-1832, the datastore transaction :2051-2156). Per report, the
reference:
  * decodes the helper input share and public share -> PrepareError::InvalidMessage on
    failure (:1896-1926),
  * runs helper_initialized + evaluate (:1945-1967); any PingPongError becomes
    PrepareError::VdafPrepError via handle_ping_pong_error (error.rs:365-427),
  * answers PrepareStepResult::Continue{Finish{prep_msg}} or Reject(error) (:1969-1993),
  * later fails replayed reports with ReportReplayed (:2101-2136) and accumulates the
    rest into batch aggregations (aggregation_job_writer.rs:608-708).
Here the per-report prio call is one engine batch call and accumulation is one masked,
segmented device reduction.
"""
from __future__ import annotations

from collections import Counter
from dataclasses import dataclass, field

import numpy as np

from .engine import FINISHED, VERDICT_LABELS, HelperEngine
from .messages import CodecError, PingPongMessage, PrepareError, PrepareInit, PrepareResp, PrepareStepResult


@dataclass
class AggregateInitOutcome:
    responses: list[PrepareResp]
    finished: np.ndarray                 # bool per PrepareInit: accumulated
    step_failures: Counter = field(default_factory=Counter)  # janus_step_failures{type=...}


def handle_aggregate_init(engine: HelperEngine, prepare_inits: list[PrepareInit], input_shares: list[bytes],
                          segments: list[int] | None = None, replayed: set[bytes] | None = None
                          ) -> AggregateInitOutcome:
    """Prepare and aggregate one AggregationJobInitializeReq worth of reports.

    input_shares[i] is the HPKE-decrypted PlaintextInputShare payload of report i (the
    encoded Prio3 helper input share). segments[i] names the batch aggregation the report
    belongs to (batch identifier; default 0). replayed holds report ids the datastore
    already saw (check_other_report_aggregation_exists)."""
    n = len(prepare_inits)
    if len(input_shares) != n:
        raise ValueError("one input share per PrepareInit")
    ids = [p.report_share.metadata.report_id for p in prepare_inits]
    if len(set(ids)) != n:  # aggregator.rs:1750-1758
        raise ValueError("aggregate request contains duplicate report IDs (invalidMessage)")
    v = engine.vdaf
    failures: Counter = Counter()
    results: list[PrepareStepResult | None] = [None] * n
    batch_idx: list[int] = []
    for i, (pi, ins) in enumerate(zip(prepare_inits, input_shares)):
        if len(ins) != v.helper_input_share_len:
            failures["input_share_decode_failure"] += 1
            results[i] = PrepareStepResult(2, error=PrepareError.InvalidMessage)
            continue
        if len(pi.report_share.public_share) != v.public_share_len:
            failures["public_share_decode_failure"] += 1
            results[i] = PrepareStepResult(2, error=PrepareError.InvalidMessage)
            continue
        msg = pi.message
        if msg.kind != PingPongMessage.INITIALIZE:  # PingPongError::PeerMessageMismatch
            failures["leader_ping_pong_message_mismatch"] += 1
            results[i] = PrepareStepResult(2, error=PrepareError.VdafPrepError)
            continue
        if len(msg.prep_share) != v.prep_share_len:  # PingPongError::CodecPrepShare
            failures["leader_prep_share_decode_failure"] += 1
            results[i] = PrepareStepResult(2, error=PrepareError.VdafPrepError)
            continue
        batch_idx.append(i)
    finished = np.zeros(n, bool)
    m = len(batch_idx)
    if m:
        nonces = np.frombuffer(b"".join(ids[i] for i in batch_idx), np.uint8).reshape(m, 16)
        ps = np.frombuffer(b"".join(prepare_inits[i].report_share.public_share for i in batch_idx), np.uint8)
        his = np.frombuffer(b"".join(input_shares[i] for i in batch_idx), np.uint8)
        lps = np.frombuffer(b"".join(prepare_inits[i].message.prep_share for i in batch_idx), np.uint8)
        res = engine.helper_initialized_batch(nonces, ps, his, lps)
        accept = np.zeros(m, np.uint8)
        seg = np.zeros(m, np.uint32)
        for j, i in enumerate(batch_idx):
            verdict = int(res.verdicts[j])
            if verdict != FINISHED:
                failures[VERDICT_LABELS[verdict]] += 1
                results[i] = PrepareStepResult(2, error=PrepareError.VdafPrepError)
                continue
            if replayed and ids[i] in replayed:  # aggregator.rs:2127-2132
                results[i] = PrepareStepResult(2, error=PrepareError.ReportReplayed)
                continue
            results[i] = PrepareStepResult(0, message=PingPongMessage.finish(res.prep_msgs[j].tobytes()))
            accept[j] = 1
            seg[j] = segments[i] if segments else 0
            finished[i] = True
        engine.accumulate(m, accept, seg)
    responses = [PrepareResp(ids[i], results[i]) for i in range(n)]
    return AggregateInitOutcome(responses, finished, failures)
