"""Helper aggregate-init over a batch of PrepareInits — the hot loop of Janus, batched.

Mirror of VdafOps::handle_aggregate_init_generic, /root/reference/aggregator/src/
aggregator.rs:1712-2161, minus the datastore transaction itself (:2051-2156).
handle_aggregate_init_encrypted starts from the encrypted report shares (the HPKE open runs inside the
prepare launch on the GPU); handle_aggregate_init from opened ones. Per report, the reference:
  * decodes the helper input share and public share -> PrepareError::InvalidMessage on
    failure (:1896-1926),
  * runs helper_initialized + evaluate (:1945-1967); any PingPongError becomes
    PrepareError::VdafPrepError via handle_ping_pong_error (error.rs:365-427),
  * answers PrepareStepResult::Continue{Finish{prep_msg}} or Reject(error) (:1969-1993),
  * later fails replayed reports with ReportReplayed (:2101-2136) and accumulates the
    rest into batch aggregations (aggregation_job_writer.rs:608-708).
Here the per-report prio call is one engine batch call that leaves a resident batch (one
per aggregation job in flight), and accumulation is one masked, segmented device reduction:
with a BatchAggregationWriter, into per-batch-identifier deltas merged inside a retryable
datastore transaction (aggregation_job_writer.rs:476-553, 608-708); without one, into the
engine's running aggregations.
"""
from __future__ import annotations

from collections import Counter
from dataclasses import dataclass, field

import numpy as np

from .engine import FINISHED, VERDICT_LABELS, HelperEngine
from .messages import (EXTENSION_TASKPROV, CodecError, HpkeCiphertext, PingPongMessage,  # noqa: F401
                       PlaintextInputShare, PrepareError, PrepareInit, PrepareResp, PrepareStepResult, ReportMetadata,
                       ReportShare)


@dataclass
class AggregateInitOutcome:
    responses: list[PrepareResp]
    finished: np.ndarray                 # bool per PrepareInit: accumulated
    step_failures: Counter = field(default_factory=Counter)  # janus_step_failures{type=...}


def _dense(seg_of_row: list[int]) -> tuple[np.ndarray, list[int]]:
    """Dense per-row indices into the list of distinct batch identifiers (first-seen order)."""
    ids: dict[int, int] = {}
    idx = np.array([ids.setdefault(int(s), len(ids)) for s in seg_of_row], np.uint32)
    return idx, list(ids)


def handle_aggregate_init(engine: HelperEngine, prepare_inits: list[PrepareInit], input_shares: list[bytes],
                          segments: list[int] | None = None, replayed: set[bytes] | None = None,
                          writer=None, extra_report_times: list[tuple[int, int]] = (),
                          inject_tx_failures: int = 0) -> AggregateInitOutcome:
    """Prepare and aggregate one AggregationJobInitializeReq worth of reports.

    input_shares[i] is the HPKE-decrypted PlaintextInputShare payload of report i (the
    encoded Prio3 helper input share). segments[i] names the batch aggregation the report
    belongs to (batch identifier; default 0). replayed holds report ids the datastore
    already saw (check_other_report_aggregation_exists).

    writer (a batch_aggregation.BatchAggregationWriter): the job's batch aggregations are
    written in one retryable transaction (a one-round Prio3 helper job is written already
    finished: neither job counter moves); every report's timestamp widens its batch's
    interval, failed ones included (extra_report_times: report aggregations of the request
    that never reached this call, e.g. HPKE failures). Reports landing in an already
    collected batch fail with BatchCollected. The engine batch is released afterwards.
    Without a writer the finished reports go into the engine's running aggregations."""
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
    res = None
    accept = np.zeros(m, np.uint8)
    if m:
        nonces = np.frombuffer(b"".join(ids[i] for i in batch_idx), np.uint8).reshape(m, 16)
        ps = np.frombuffer(b"".join(prepare_inits[i].report_share.public_share for i in batch_idx), np.uint8)
        his = np.frombuffer(b"".join(input_shares[i] for i in batch_idx), np.uint8)
        lps = np.frombuffer(b"".join(prepare_inits[i].message.prep_share for i in batch_idx), np.uint8)
        res = engine.helper_initialized_batch(nonces, ps, his, lps)
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
            finished[i] = True
    times = [(int(segments[i]) if segments else 0, p.report_share.metadata.time)
             for i, p in enumerate(prepare_inits)] + list(extra_report_times)
    _write_job(engine, res.batch_id if m else 0, batch_idx, accept, segments, writer, times, inject_tx_failures,
               finished, results)
    responses = [PrepareResp(ids[i], results[i]) for i in range(n)]
    return AggregateInitOutcome(responses, finished, failures)


def _write_job(engine: HelperEngine, batch_id: int, batch_idx: list[int], accept: np.ndarray, segments, writer,
               times, inject_tx_failures: int, finished: np.ndarray, results: list) -> None:
    """Accumulate a helper job's accepted rows (engine row j = report batch_idx[j]): with a writer, as
    per-batch-identifier deltas in one retryable transaction (aggregation_job_writer.rs:476-553, 608-708; the
    batch is released after), else into the engine's running aggregations (which consume the batch). Reports of
    an already collected batch fail with BatchCollected."""
    m = len(batch_idx)
    row_seg = [int(segments[i]) if segments else 0 for i in batch_idx]
    if writer is None:
        if m:
            seg = np.array(row_seg, np.uint32)
            with engine.resident(batch_id):  # accumulate consumes the batch; on an error it is released
                engine.accumulate(m, accept, seg, batch_id=batch_id)
        return
    if m:
        idx, seg_ids = _dense(row_seg)
        try:
            collected = writer.write_job(engine, batch_id, m, accept, idx, seg_ids, times,
                                         initial_write=True, terminal=True, inject_failures=inject_tx_failures)
        finally:
            engine.release(batch_id)
    else:
        collected = writer.write_job(engine, 0, 0, None, None, [], times, initial_write=True, terminal=True,
                                     inject_failures=inject_tx_failures)
    for j, i in enumerate(batch_idx):  # fail_report_aggregations_for_collected_batches
        if finished[i] and row_seg[j] in collected:
            finished[i] = False
            results[i] = PrepareStepResult(2, error=PrepareError.BatchCollected)


# ----------------------------------------------------------------------------- leader side
# Mirror of AggregationJobDriver::step_aggregation_job_aggregate_init and
# process_response_from_helper (aggregator/src/aggregator/aggregation_job_driver.rs:259-436,
# 540-701) minus the HTTP exchange and the datastore: the leader's per-report
# leader_initialized / leader_continued calls become two engine batch calls.


@dataclass
class LeaderReport:
    metadata: ReportMetadata
    public_share: bytes
    leader_input_share: bytes                  # decoded at upload time in Janus; encoded here
    helper_encrypted_input_share: HpkeCiphertext


@dataclass
class LeaderStep:
    prepare_inits: list[PrepareInit]           # the AggregationJobInitializeReq body
    stepped: list[int]                         # report index of each PrepareInit
    failed: dict[int, PrepareError]            # reports that failed before the helper
    n: int                                     # reports in the engine's leader batch
    step_failures: Counter = field(default_factory=Counter)
    init: object = None                        # the engine's LeaderInit (its batch id) when n > 0


def leader_aggregate_init(engine: HelperEngine, reports: list[LeaderReport], segments: list[int] | None = None,
                          writer=None) -> LeaderStep:
    """Prepare every report of a new aggregation job on the leader (agg_id 0) and build the
    PrepareInits to send to the helper (aggregation_job_driver.rs:301-386). writer: the job is
    written in progress (aggregation_jobs_created + 1 per batch identifier) with every report's
    timestamp."""
    v = engine.vdaf
    n = len(reports)
    failures: Counter = Counter()
    failed: dict[int, PrepareError] = {}
    ok = [i for i, r in enumerate(reports) if len(r.leader_input_share) == engine.leader_input_share_len
          and len(r.public_share) == v.public_share_len]
    for i in set(range(n)) - set(ok):
        failed[i] = PrepareError.InvalidMessage
        failures["input_share_decode_failure"] += 1
    inits: list[PrepareInit] = []
    stepped: list[int] = []
    if ok:
        nonces = np.frombuffer(b"".join(reports[i].metadata.report_id for i in ok), np.uint8).reshape(len(ok), 16)
        ps = np.frombuffer(b"".join(reports[i].public_share for i in ok), np.uint8)
        lis = np.frombuffer(b"".join(reports[i].leader_input_share for i in ok), np.uint8)
        res = engine.leader_initialized_batch(nonces, ps, lis)
        for j, i in enumerate(ok):
            if res.verdicts[j] != FINISHED:  # handle_ping_pong_error(Role::Leader, ...)
                failed[i] = PrepareError.VdafPrepError
                failures[VERDICT_LABELS[int(res.verdicts[j])]] += 1
                continue
            r = reports[i]
            inits.append(PrepareInit(ReportShare(r.metadata, r.public_share, r.helper_encrypted_input_share),
                                     PingPongMessage.initialize(res.prep_shares[j].tobytes())))
            stepped.append(i)
    times = [(int(segments[i]) if segments else 0, r.metadata.time) for i, r in enumerate(reports)]
    if writer is not None:  # InitialWrite of the in-progress job: no finished report yet
        try:
            collected = writer.write_job(engine, 0, 0, None, None, [], times, initial_write=True, terminal=False)
        except BaseException:
            if ok:
                engine.release(res.batch_id, missing_ok=True)
            raise
        # fail_report_aggregations_for_collected_batches on the initial write (aggregation_job_writer.rs:
        # 557-605): a report of an already collected batch fails with BatchCollected and is not sent to
        # the helper (its engine row is never continued, so it is never accumulated)
        if collected:
            keep = [k for k, i in enumerate(stepped) if (int(segments[i]) if segments else 0) not in collected]
            for k, i in enumerate(stepped):
                if (int(segments[i]) if segments else 0) in collected:
                    failed[i] = PrepareError.BatchCollected
            inits = [inits[k] for k in keep]
            stepped = [stepped[k] for k in keep]
    step = LeaderStep(inits, stepped, failed, len(ok), failures, res if ok else None)
    step._batch_index = {i: j for j, i in enumerate(ok)}  # report index -> engine batch row
    step._times = times
    return step


def leader_abandon(engine: HelperEngine, step: LeaderStep) -> None:
    """Drop an aggregation job's leader state (the job was abandoned, or its helper exchange failed
    for good): its resident engine batch is released. A later leader_process_helper_response for
    the step fails with JX_E_STATE."""
    if step.init is not None:
        engine.release(step.init.batch_id, missing_ok=True)


def leader_process_helper_response(engine: HelperEngine, step: LeaderStep, prepare_resps: list[PrepareResp],
                                   segments: list[int] | None = None, writer=None) -> AggregateInitOutcome:
    """Finish the leader's reports from the helper's AggregationJobResp and accumulate the
    finished ones (process_response_from_helper, aggregation_job_driver.rs:540-701). writer: the
    job is updated into a terminal state (aggregation_jobs_terminated + 1 per batch identifier),
    its finished reports merged as deltas in one retryable transaction, and the engine batch is
    released. Without a writer they go into the engine's running aggregations."""
    if len(prepare_resps) != len(step.stepped) or any(
            resp.report_id != step.prepare_inits[k].report_share.metadata.report_id
            for k, resp in enumerate(prepare_resps)):
        # the job step fails (process_response_from_helper's error): its device state is released, and
        # the job is stepped again from leader_aggregate_init
        leader_abandon(engine, step)
        raise ValueError("missing, duplicate, out-of-order, or unexpected prepare steps in response")
    failures = Counter(step.step_failures)
    nrep = max([*step.stepped, *step.failed, -1]) + 1
    finished = np.zeros(nrep, bool)
    results: dict[int, PrepareError | None] = dict(step.failed)
    pm = engine.prep_msg_len
    msgs = np.zeros((step.n, max(pm, 1)), np.uint8)
    continued = np.zeros(step.n, bool)
    for k, resp in enumerate(prepare_resps):
        i = step.stepped[k]
        row = step._batch_index[i]
        res = resp.result
        if res.kind == 2:                        # Reject(err): the helper's error
            results[i] = res.error
            failures["helper_step_failure"] += 1
        elif res.kind == 1:                      # Finished, but a 1-round leader is still Continued
            results[i] = PrepareError.VdafPrepError
            failures["finish_mismatch"] += 1
        elif res.message.kind != PingPongMessage.FINISH or len(res.message.prep_msg) != pm:
            results[i] = PrepareError.VdafPrepError  # PingPongError::PeerMessageMismatch / CodecPrepMessage
            failures["leader_ping_pong_message_mismatch"] += 1
        else:
            if pm:
                msgs[row, :pm] = np.frombuffer(res.message.prep_msg, np.uint8)
            continued[row] = True
    if step.n == 0:  # no report reached the engine: nothing to continue or accumulate
        if writer is not None:
            writer.write_job(engine, 0, 0, None, None, [], step._times, initial_write=False, terminal=True)
        responses = [PrepareResp(step.prepare_inits[k].report_share.metadata.report_id,
                                 PrepareStepResult(2, error=results[i])) for k, i in enumerate(step.stepped)]
        return AggregateInitOutcome(responses, finished, failures)
    try:
        fin = engine.leader_continued_batch(msgs[:, :pm] if pm else None, init=step.init)
    except BaseException:
        leader_abandon(engine, step)
        raise
    accept = np.zeros(step.n, np.uint8)
    seg = np.zeros(step.n, np.uint32)
    for i, row in step._batch_index.items():
        if not continued[row]:
            continue
        if fin.verdicts[row] != FINISHED:
            results[i] = PrepareError.VdafPrepError
            failures[VERDICT_LABELS[int(fin.verdicts[row])]] += 1
            continue
        results[i] = None
        accept[row] = 1
        seg[row] = segments[i] if segments else 0
        finished[i] = True
    if writer is None:
        with engine.resident(step.init.batch_id):
            engine.accumulate(step.n, accept, seg, batch_id=step.init.batch_id)
    else:
        row_seg = [0] * step.n
        for i, row in step._batch_index.items():
            row_seg[row] = int(segments[i]) if segments else 0
        idx, seg_ids = _dense(row_seg)
        try:
            collected = writer.write_job(engine, step.init.batch_id, step.n, accept, idx, seg_ids, step._times,
                                         initial_write=False, terminal=True)
        finally:
            engine.release(step.init.batch_id)
        for i, row in step._batch_index.items():
            if finished[i] and row_seg[row] in collected:
                finished[i] = False
                results[i] = PrepareError.BatchCollected
    responses = [PrepareResp(step.prepare_inits[k].report_share.metadata.report_id,
                             PrepareStepResult(1) if results[i] is None else
                             PrepareStepResult(2, error=results[i]))
                 for k, i in enumerate(step.stepped)]
    return AggregateInitOutcome(responses, finished, failures)


# ----------------------------------------------------------------------------- HPKE + prepare


def handle_aggregate_init_encrypted(engine: HelperEngine, opener, hpke_config_id: int, task_id: bytes,
                                    prepare_inits: list[PrepareInit], segments: list[int] | None = None,
                                    replayed: set[bytes] | None = None, writer=None, global_keypairs=None,
                                    require_taskprov: bool = False, report_deadline: int | None = None,
                                    inject_tx_failures: int = 0) -> AggregateInitOutcome:
    """The helper's aggregate-init loop from the encrypted report shares (aggregator.rs:1763-2013), with the
    HPKE open inside the prepare launch (jx_helper_prep_encrypted_batch; coalesced with other jobs when the
    engine coalesces): per report, the task's keypair (opener, config id hpke_config_id) and then the
    aggregator's global keypair for the report's config id (global_keypairs: {config_id: HpkeOpener}) are
    tried (:1781-1832), the PlaintextInputShare is decoded and its extensions checked (:1834-1893), the payload
    decoded as the helper input share (:1895-1910), the public share decoded (:1912-1925), reports from after
    report_deadline rejected (:1929-1940), then helper_initialized + evaluate (:1945-1967). Failures map as in
    the reference: HpkeUnknownConfigId, HpkeDecryptError, InvalidMessage (plaintext / extension / input share /
    public share), ReportTooEarly, VdafPrepError. A report whose public share has the wrong length cannot ride
    the fixed-stride device rows: it is opened alone (janus_amd.hpke) and fails with InvalidMessage unless an
    earlier check fails it first."""
    from .engine import KEY_MALFORMED, KEY_NONE, OPEN_STATUS

    v = engine.vdaf
    n = len(prepare_inits)
    ids = [p.report_share.metadata.report_id for p in prepare_inits]
    if len(set(ids)) != n:  # aggregator.rs:1750-1758
        raise ValueError("aggregate request contains duplicate report IDs (invalidMessage)")
    globals_ = dict(global_keypairs or {})
    keypairs = [opener]
    slot: dict[int, int] = {}

    def key_slot(k) -> int:
        if id(k) not in slot:
            slot[id(k)] = len(keypairs) if k is not opener else 0
            if k is not opener:
                keypairs.append(k)
        return slot[id(k)]

    slot[id(opener)] = 0
    failures: Counter = Counter()
    results: list[PrepareStepResult | None] = [None] * n
    rows: list[int] = []           # reports on the device, in row order
    odd: list[int] = []            # public share of the wrong length: opened alone
    key_index = []
    for i, pi in enumerate(prepare_inits):
        ct = pi.report_share.encrypted_input_share
        task_k = opener if ct.config_id == hpke_config_id else None
        glob_k = globals_.get(ct.config_id)
        first, second = (task_k, glob_k) if task_k is not None else (glob_k, None)
        if len(pi.report_share.public_share) != v.public_share_len:
            odd.append(i)
            continue
        if first is None:
            k0, k1 = KEY_NONE, KEY_NONE
        elif len(ct.encapsulated_key) != 32:
            k0, k1 = KEY_MALFORMED, KEY_NONE
        else:
            k0, k1 = key_slot(first), (key_slot(second) if second is not None else KEY_NONE)
        if len(keypairs) > 8:
            raise ValueError("more than JX_ENC_MAX_KEYPAIRS distinct keypairs in one request")
        rows.append(i)
        key_index.append((k0, k1))
    finished = np.zeros(n, bool)
    m = len(rows)
    accept = np.zeros(m, np.uint8)
    res = None
    if m:
        md = [prepare_inits[i].report_share.metadata for i in rows]
        nonces = np.frombuffer(b"".join(x.report_id for x in md), np.uint8).reshape(m, 16)
        times = np.array([x.time for x in md], np.uint64)
        ps = np.frombuffer(b"".join(prepare_inits[i].report_share.public_share for i in rows), np.uint8)
        encs = np.frombuffer(b"".join(
            (lambda e: e if len(e) == 32 else bytes(32))(prepare_inits[i].report_share.encrypted_input_share
                                                           .encapsulated_key) for i in rows), np.uint8).reshape(m, 32)
        payloads = [prepare_inits[i].report_share.encrypted_input_share.payload for i in rows]
        # a leader message that is not Initialize, or a prep share of the wrong length, fails inside
        # helper_initialized, after the open: the row rides with a zero prep share and is fixed up below
        msg_fail: dict[int, str] = {}
        lps_rows = []
        for j, i in enumerate(rows):
            msg = prepare_inits[i].message
            if msg.kind != PingPongMessage.INITIALIZE:  # PingPongError::PeerMessageMismatch
                msg_fail[j] = "leader_ping_pong_message_mismatch"
            elif len(msg.prep_share) != v.prep_share_len:  # PingPongError::CodecPrepShare
                msg_fail[j] = "leader_prep_share_decode_failure"
            lps_rows.append(msg.prep_share if j not in msg_fail else bytes(v.prep_share_len))
        lps = np.frombuffer(b"".join(lps_rows), np.uint8)
        res = engine.helper_initialized_encrypted_batch(nonces, times, ps, task_id, keypairs,
                                                        np.array(key_index, np.uint8), encs, payloads, lps,
                                                        require_taskprov=require_taskprov)
        for j, i in enumerate(rows):
            st = int(res.open_status[j])
            if st:
                label, err = OPEN_STATUS[st]
                failures[label] += 1
                results[i] = PrepareStepResult(2, error=PrepareError(err))
            elif report_deadline is not None and md[j].time > report_deadline:
                results[i] = PrepareStepResult(2, error=PrepareError.ReportTooEarly)
            elif j in msg_fail:
                failures[msg_fail[j]] += 1
                results[i] = PrepareStepResult(2, error=PrepareError.VdafPrepError)
            elif int(res.verdicts[j]) != FINISHED:
                failures[VERDICT_LABELS[int(res.verdicts[j])]] += 1
                results[i] = PrepareStepResult(2, error=PrepareError.VdafPrepError)
            elif replayed and ids[i] in replayed:  # aggregator.rs:2127-2132
                results[i] = PrepareStepResult(2, error=PrepareError.ReportReplayed)
            else:
                results[i] = PrepareStepResult(0, message=PingPongMessage.finish(res.prep_msgs[j].tobytes()))
                accept[j] = 1
                finished[i] = True
    for i in odd:
        results[i] = PrepareStepResult(2, error=_open_alone(prepare_inits[i], opener, hpke_config_id, globals_,
                                                            task_id, v, require_taskprov, failures))
    times_all = [(int(segments[i]) if segments else 0, p.report_share.metadata.time) for i, p in enumerate(prepare_inits)]
    _write_job(engine, res.batch_id if m else 0, rows, accept, segments, writer, times_all, inject_tx_failures,
               finished, results)
    responses = [PrepareResp(ids[i], results[i]) for i in range(n)]
    return AggregateInitOutcome(responses, finished, failures)


def _open_alone(pi: PrepareInit, opener, hpke_config_id: int, globals_: dict, task_id: bytes, v, require_taskprov: bool,
                failures: Counter) -> PrepareError:
    """A report whose public share has the wrong length (it cannot ride the fixed-stride device rows): the
    reference's checks in order on the host (batched HPKE open on the GPU for this one share); it always fails,
    with public_share_decode_failure at the latest."""
    from .hpke import input_share_aad

    rs = pi.report_share
    ct = rs.encrypted_input_share
    keys = [k for k in ((opener if ct.config_id == hpke_config_id else None), globals_.get(ct.config_id)) if k]
    if not keys:
        failures["unknown_hpke_config_id"] += 1
        return PrepareError.HpkeUnknownConfigId
    aad = input_share_aad(task_id, rs.metadata.report_id, rs.metadata.time, rs.public_share)
    pt = None
    for k in keys:
        pt = k.open_batch([ct.encapsulated_key], [ct.payload], [aad])[0]
        if pt is not None:
            break
    if pt is None:
        failures["decrypt_failure"] += 1
        return PrepareError.HpkeDecryptError
    try:
        pis = PlaintextInputShare.decode(pt)
    except CodecError:
        failures["plaintext_input_share_decode_failure"] += 1
        return PrepareError.InvalidMessage
    types = [e.extension_type for e in pis.extensions]
    if len(set(types)) != len(types):
        failures["duplicate_extension"] += 1
    elif require_taskprov and not any(e.extension_type == EXTENSION_TASKPROV and not e.extension_data
                                      for e in pis.extensions):
        failures["missing_or_malformed_taskprov_extension"] += 1
    elif not require_taskprov and EXTENSION_TASKPROV in types:
        failures["unexpected_taskprov_extension"] += 1
    elif len(pis.payload) != v.helper_input_share_len:
        failures["input_share_decode_failure"] += 1
    else:
        failures["public_share_decode_failure"] += 1
    return PrepareError.InvalidMessage
