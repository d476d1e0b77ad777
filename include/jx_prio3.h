/*
 * jx_prio3.h — C ABI of the MI355X batched Prio3 helper prepare + aggregate engine.
 *
 * Drop-in boundary. In Janus the hot path is reached through the
 * `prio::vdaf::Aggregator<16, 16>` trait + `PingPongTopology`, called once per
 * report from the helper's aggregate-init loop:
 *   /root/reference/aggregator/src/aggregator.rs:1945-1967
 *     vdaf.helper_initialized(verify_key, agg_param, nonce = report_id,
 *                             public_share, input_share, leader_msg).evaluate(vdaf)
 * and the per-report accumulation
 *   /root/reference/aggregator/src/aggregator/aggregation_job_writer.rs:608-708
 *   /root/reference/aggregator_core/src/datastore/models.rs:1275-1330 (merged_with)
 * plus the shard merge of compute_aggregate_share
 *   /root/reference/aggregator/src/aggregator/aggregate_share.rs:55-96.
 * This ABI replaces that loop body with one call per batch. HPKE-open, plaintext
 * decode, replay / collected-batch checks and the datastore stay on the host.
 *
 * Conventions:
 *  - Every function returns int32 status: 0 = OK, < 0 = engine error (JX_E_*).
 *    Per-report preparation failures are NOT errors: they are verdict bytes.
 *  - The caller owns every host buffer; it is borrowed for the duration of the call.
 *  - An engine is one task's handle on one device (VdafOps per task, aggregator/src/aggregator.rs:
 *    1156-1183): its verify key, its resident batches, its running aggregations and one HIP stream.
 *    It holds no launch staging between calls: staging is checked out of the device's arena per call
 *    and handed back stream-ordered, and resident batches come from the same arena (jx_engine_memory),
 *    so any number of engines (tasks) share one GPU's HBM. Every entry point takes the engine's mutex
 *    for the duration of the call, so one engine can serve concurrent aggregation jobs from several
 *    host threads; the device work of the calls is serialized on the engine stream. What a job keeps
 *    between calls (its prepared reports) is a batch handle. (A helper launch past one lane-split K1
 *    wave per SIMD, while no other engine on the device runs a large K1 launch, puts part of its K1 on
 *    a second stream of the engine, forked from and joined back into the engine stream by events: the
 *    ordering below is unchanged.)
 *  - Coalesced prepares (jx_engine_coalesce): with coalescing on, jx_helper_prep_batch and
 *    jx_leader_prep_init_batch of jobs up to a quarter of a launch join the device's next shared launch
 *    with the concurrent jobs of every coalescing engine of the same Prio3 instance on the device (each
 *    report with its own engine's verify key), and wait for it without holding the engine mutex. Results,
 *    batches and errors are per job, exactly as without coalescing.
 *  - Host-buffer entry points are synchronous. Device-pointer entry points (*_device) are
 *    asynchronous on the engine stream, a NON-BLOCKING stream that orders itself after nothing:
 *    PRODUCER ORDERING is the caller's. Before a *_device call whose inputs were written by work
 *    queued on another stream, call jx_engine_wait_stream(e, producer) (or jx_engine_wait_event on an
 *    event recorded after the producer's writes); after it, jx_engine_join_stream(e, consumer) (or
 *    jx_engine_record_event + a wait) before the consumer reads the outputs or reuses the inputs.
 *    Neither blocks the host. Creating an engine synchronizes only the engine stream.
 *  - jx_last_error returns the message of the calling thread's last failed call.
 *  - Byte layouts are the DAP/VDAF encodings (fixed stride per report):
 *      nonces               n x 16   (report ids; VDAF nonce, aggregator.rs:1951)
 *      public_shares        n x PS   (Prio3PublicShare: joint-rand parts, 0 or 32 B)
 *      helper_input_shares  n x HIS  (k_meas || k_proofs || [k_blind])
 *      leader_prep_shares   n x LPS  (the prep_share inside PingPongMessage::Initialize)
 *      prep_msgs            n x PM   (prep_msg inside PingPongMessage::Finish; 0 or 16 B)
 *      output shares        n x OUT x FB, aggregate shares OUT x FB, field elements LE.
 */
#ifndef JX_PRIO3_H
#define JX_PRIO3_H

#include <stdint.h>

#include "jx_hpke.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes */
#define JX_OK 0
#define JX_E_INVALID (-1)     /* bad argument */
#define JX_E_UNSUPPORTED (-2) /* parameter set not supported by the engine */
#define JX_E_HIP (-3)         /* HIP runtime error (see jx_last_error) */
#define JX_E_NOMEM (-4)       /* device allocation failed */
#define JX_E_STATE (-5)       /* call out of order (e.g. accumulate without a prepared batch) */
#define JX_E_NODEVICE (-6)

/* Verdict bytes. Labels match handle_ping_pong_error, aggregator/src/aggregator/error.rs:379-424;
 * every non-zero verdict goes on the wire as PrepareError::VdafPrepError (messages/src/lib.rs:2344). */
#define JX_FINISHED 0
#define JX_PREPARE_INIT_FAILURE 1          /* PingPongError::VdafPrepareInit */
#define JX_PREP_SHARE_DECODE_FAILURE 2     /* PingPongError::CodecPrepShare (leader share malformed) */
#define JX_PREPARE_MESSAGE_FAILURE 3       /* PingPongError::VdafPrepareSharesToPrepareMessage */
#define JX_PREPARE_NEXT_FAILURE 4          /* PingPongError::VdafPrepareNext */
/* Leader only: the helper answered PrepareStepResult::Reject for this report (label
 * helper_step_failure, aggregation_job_driver.rs:646-660). */
#define JX_HELPER_STEP_FAILURE 5
/* Helper, encrypted inputs only: the report's input share did not open or decode; its out_open_status byte
 * names why (not a prepare failure: the report never reached helper_initialized). */
#define JX_OPEN_FAILURE 6

/* Open status of an encrypted report share (jx_helper_prep_encrypted_batch out_open_status): the checks of
 * the helper's loop before helper_initialized, in its order (aggregator/src/aggregator.rs:1781-1910), with the
 * PrepareError each goes on the wire as and its janus_step_failures label. */
#define JX_OPEN_OK 0
#define JX_OPEN_HPKE_DECRYPT_ERROR 1         /* HpkeDecryptError, "decrypt_failure" */
#define JX_OPEN_PLAINTEXT_DECODE_FAILURE 2   /* InvalidMessage, "plaintext_input_share_decode_failure" */
#define JX_OPEN_DUPLICATE_EXTENSION 3        /* InvalidMessage, "duplicate_extension" */
#define JX_OPEN_UNEXPECTED_TASKPROV 4        /* InvalidMessage, "unexpected_taskprov_extension" */
#define JX_OPEN_MISSING_TASKPROV 5           /* InvalidMessage, "missing_or_malformed_taskprov_extension" */
#define JX_OPEN_INPUT_SHARE_DECODE_FAILURE 6 /* InvalidMessage, "input_share_decode_failure" */
#define JX_OPEN_UNKNOWN_CONFIG 7             /* HpkeUnknownConfigId, "unknown_hpke_config_id" */
/* key_index values besides keypair indices */
#define JX_KEY_NONE 0xFF      /* no keypair (first: the config id is unknown; second: no fallback) */
#define JX_KEY_MALFORMED 0xFE /* first only: the encapsulated key is not 32 bytes (HpkeDecryptError) */
#define JX_ENC_MAX_KEYPAIRS 8
/* flags */
#define JX_ENC_REQUIRE_TASKPROV 1u /* the task is provisioned by taskprov (aggregator.rs:1869-1879) */

/* Prio3 instance, mirroring janus_core::vdaf::VdafInstance (core/src/vdaf.rs:65-108).
 * algo_id: 0 Prio3Count, 1 Prio3Sum{bits}, 2 Prio3SumVec{bits,length,chunk_length},
 *          3 Prio3Histogram{length,chunk_length}  (== Prio3 algorithm ids, messages/src/taskprov.rs:358-363)
 *          4 Prio3SumVecField64MultiproofHmacSha256Aes128{proofs,bits,length,chunk_length}
 *            (core/src/vdaf.rs:173-199: Field64, XofHmacSha256Aes128, 32-byte seeds and verify key;
 *            DST algorithm id 0xFFFF1003; prep messages and joint-rand parts are 32 bytes)
 *          5 Prio3FixedPointBoundedL2VecSum{bitsize, length} (core/src/vdaf.rs:86-91; built at
 *            aggregator/src/aggregator.rs:916-932): bits = 16 (BitSize16, FixedI16<U15>) or 32
 *            (BitSize32, FixedI32<U31>), length = entries, chunk_length ignored (prio derives both
 *            gadgets' chunk lengths); Field128, TurboSHAKE, DST algorithm id 0xFFFF0000. The
 *            dp_strategy is applied at collection time and is not part of this ABI.
 * num_proofs: 1 for ids 0-3 and 5 (the TurboSHAKE variants, core/src/vdaf.rs:203-262); 2..8 for id 4. */
#define JX_ALGO_COUNT 0
#define JX_ALGO_SUM 1
#define JX_ALGO_SUMVEC 2
#define JX_ALGO_HISTOGRAM 3
#define JX_ALGO_SUMVEC_F64_MULTIPROOF_HMACSHA256_AES128 4
#define JX_ALGO_FIXEDPOINT_BOUNDED_L2_VEC_SUM 5
typedef struct {
  uint32_t algo_id;
  uint32_t bits;
  uint32_t length;
  uint32_t chunk_length;
  uint32_t num_proofs;
} jx_prio3_params;

typedef struct jx_engine jx_engine;

/* Create an engine for one Prio3 instance and one verify key (VERIFY_KEY_LENGTH = 16,
 * core/src/vdaf.rs:16) on HIP device `device`. */
int32_t jx_engine_create(const jx_prio3_params* params, const uint8_t verify_key[16], int32_t device,
                         jx_engine** out);
/* Same with an explicit verify key length: 16 (VERIFY_KEY_LENGTH) or, for algo_id 4, 32
 * (VERIFY_KEY_LENGTH_HMACSHA256_AES128, core/src/vdaf.rs:24). */
int32_t jx_engine_create_ex(const jx_prio3_params* params, const uint8_t* verify_key, uint32_t verify_key_len,
                            int32_t device, jx_engine** out);
void jx_engine_destroy(jx_engine* e);

/* Encoded sizes (bytes) for this instance. Any pointer may be NULL. */
int32_t jx_engine_sizes(const jx_engine* e, uint32_t* public_share, uint32_t* helper_input_share,
                        uint32_t* leader_prep_share, uint32_t* prep_msg, uint32_t* output_len,
                        uint32_t* field_bytes);

/* Reserve staging for `reports` reports (two-phase API needs n <= capacity; grows on demand). */
int32_t jx_engine_set_capacity(jx_engine* e, uint64_t reports);

/* ---- Resident prepared batches (one per aggregation job in flight).
 * Every prepare call (jx_helper_prep_batch, jx_leader_prep_init_*) creates a NEW resident batch and
 * returns its handle (batch id, never reused, never 0); it does not disturb other resident batches,
 * so any number of aggregation jobs can be prepared, finished and aggregated interleaved on one
 * engine (Janus steps max_concurrent_job_workers jobs at once, aggregator/src/binary_utils/
 * job_driver.rs:116-138; the leader holds each job's prepare state across the helper round trip,
 * aggregation_job_driver.rs:396-416 -> :540-701). A batch holds its output shares, verdicts, prep
 * messages (leader: the corrected joint-rand seeds) and report ids in HBM until it is released
 * (jx_batch_release) or accumulated into the running aggregations (jx_accumulate*, which releases it).
 * Calls naming a released or unknown batch return JX_E_STATE; a report count other than the
 * batch's returns JX_E_INVALID. */

/* Device memory of the engine and of its device's arena (shared by every engine on the device), and
 * the engine's coalescer (jx_engine_coalesce). */
typedef struct {
  uint64_t resident_batches;   /* this engine's resident batches */
  uint64_t batch_bytes;        /* device bytes they hold (arena slabs) */
  uint64_t arena_budget;       /* bytes the device arena may hold (JX_ARENA_GB, default 90% of HBM) */
  uint64_t arena_allocated;    /* bytes it holds: checked out + idle */
  uint64_t arena_in_use;       /* checked out now (staging of calls in progress + resident batches) */
  uint64_t arena_peak;         /* max arena_in_use */
  uint64_t arena_allocs;       /* device allocations it made */
  uint64_t arena_reuses;       /* check-outs served from idle slabs */
  uint64_t arena_waits;        /* check-outs that waited for another call's staging */
  uint64_t arena_engines;      /* live engines on the device */
  uint64_t last_pipelines;     /* pipelines the engine's last fused call ran */
  uint64_t coalesced_launches; /* launches of the device coalescer this engine uses (all its engines) */
  uint64_t coalesced_jobs;
  uint64_t coalesced_reports;
  uint64_t coalesce_window_us; /* its current gathering window */
  /* phase totals over the coalescer's launches (us): gathering (first job -> closed), the callers' input
   * copies after the close, queueing the launch, the device (queued -> done) */
  uint64_t coalesce_gather_us;
  uint64_t coalesce_copy_us;
  uint64_t coalesce_enqueue_us;
  uint64_t coalesce_device_us;
  uint64_t arena_cross_stream_waits; /* check-outs that had to wait for another stream's work */
  /* the coalescer's pinned host rows (all its lanes; released after 2 s without jobs) and its launches / jobs
   * by role (one gathering lane per role: leader and helper jobs never close each other's gathers) */
  uint64_t coalesce_pinned_bytes;
  uint64_t coalesced_helper_launches;
  uint64_t coalesced_helper_jobs;
  uint64_t coalesced_leader_launches;
  uint64_t coalesced_leader_jobs;
  uint64_t coalesced_encrypted_jobs;  /* helper jobs whose input shares were opened inside the launch */
  uint64_t arena_frees;               /* slabs the arena returned to the device (trims) */
} jx_memory_stats;
int32_t jx_engine_memory(const jx_engine* e, jx_memory_stats* out);

/* Coalesced prepares (Conventions). enable != 0 joins the device coalescer of this Prio3 instance;
 * window_us: the longest a launch gathers jobs after its first one arrives (0 = automatic: 1.5x the recent
 * launch latency, 0.1 .. 20 ms). A launch closes earlier when it is full, or once no job has joined for
 * 100 us while no other launch of the coalescer is running (or it already holds a quarter of a full
 * launch). Calls already waiting are unaffected by a later disable. The window is a setting of the device
 * coalescer, which every coalescing engine of the same Prio3 instance on the device shares: the last call
 * sets it for all of them. */
int32_t jx_engine_coalesce(jx_engine* e, int32_t enable, uint32_t window_us);

/* Batched helper_initialized + evaluate for n reports (host buffers).
 * out_verdicts[n] receives JX_FINISHED or a failure code; out_prep_msgs[n x PM] the outbound
 * Finish{prep_msg} payload (meaningful where verdict == JX_FINISHED); out_output_shares
 * (nullable) the output shares; *out_batch_id (nullable) the new batch's handle. */
int32_t jx_helper_prep_batch(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                             const uint8_t* helper_input_shares, const uint8_t* leader_prep_shares,
                             uint8_t* out_prep_msgs, uint8_t* out_verdicts, uint8_t* out_output_shares,
                             uint64_t* out_batch_id);
/* The same prepare for report shares still under HPKE, the helper's whole per-report loop up to
 * helper_initialized (aggregator/src/aggregator.rs:1763-1967): on the device, report i's encrypted input share
 * is opened with keypairs[key_index[2i]] and, if that fails to decrypt, keypairs[key_index[2i + 1]] (the
 * task's keypair, then the global one for the same config id, :1807-1820), the PlaintextInputShare is decoded
 * and its extensions checked (:1834-1893), its payload decoded as the helper input share (:1895-1910), and the
 * report prepared in the same launch (coalesced with other jobs like jx_helper_prep_batch). A report that fails
 * before helper_initialized gets verdict JX_OPEN_FAILURE and out_open_status[i] (JX_OPEN_*); every other
 * report gets JX_OPEN_OK and its verdict as from jx_helper_prep_batch.
 *   times[n]            ReportMetadata.time (seconds); InputShareAad = task_id || id || time || public share
 *   task_id             32 bytes
 *   keypairs            nkeypairs (<= JX_ENC_MAX_KEYPAIRS) HPKE contexts on the engine's device, created with
 *                       the input-share application info (Label::InputShare, Client -> Helper)
 *   key_index[n x 2]    per report: first keypair, fallback keypair (JX_KEY_NONE / JX_KEY_MALFORMED above)
 *   encs[n x 32]        HpkeCiphertext.encapsulated_key
 *   payloads            ciphertexts back to back; report i's is [payload_offsets[i], payload_offsets[i+1])
 *   flags               JX_ENC_REQUIRE_TASKPROV or 0
 * Public shares are fixed-length rows: a report whose public share has another length cannot go here (the
 * caller opens it alone and fails it with public_share_decode_failure, :1912-1925). out_open_status nullable. */
int32_t jx_helper_prep_encrypted_batch(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint64_t* times,
                                       const uint8_t* public_shares, const uint8_t task_id[32],
                                       jx_hpke* const* keypairs, uint32_t nkeypairs, const uint8_t* key_index,
                                       const uint8_t* encs, const uint8_t* payloads, const uint64_t* payload_offsets,
                                       uint32_t flags, const uint8_t* leader_prep_shares, uint8_t* out_prep_msgs,
                                       uint8_t* out_verdicts, uint8_t* out_open_status, uint64_t* out_batch_id);
/* Handle of the most recently prepared batch if it is still resident (0 otherwise). */
int32_t jx_engine_batch_id(const jx_engine* e, uint64_t* batch_id);
/* Resident batches and the device bytes they hold (either pointer nullable). */
int32_t jx_engine_batches(const jx_engine* e, uint64_t* resident, uint64_t* device_bytes);
/* Drop a resident batch (its device memory returns to the engine). */
int32_t jx_batch_release(jx_engine* e, uint64_t batch_id);

/* Per-job batch-aggregation deltas (the retry-safe accumulation contract).
 * Aggregates the finished reports of batch `batch_id` (helper; leader after finish) with
 * accept_mask[i] != 0 (nullable = all) into nsegments ZEROED aggregations, report i into aggregation
 * segment_index[i] (nullable = all into 0; indices >= nsegments are skipped), and writes them as
 * nsegments back-to-back shard records (encoded aggregate share OUT x FB || report count u64 LE ||
 * ReportIdChecksum 32 B, see jx_shard_record_bytes) to out_records. Nothing in the engine changes: the
 * batch stays resident and the running aggregations are untouched, so the call can be repeated with
 * the same or another mask (a retried run_tx closure, aggregator_core/src/datastore.rs:225-282) and the
 * host merges each record into the batch-aggregation row it read at its shard `ord`
 * (BatchAggregation::merged_with, aggregation_job_writer.rs:527,615-690). */
int32_t jx_batch_aggregate_records(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* accept_mask,
                                   const uint32_t* segment_index, uint32_t nsegments, uint8_t* out_records);
/* Same with device arrays and a device output (asynchronous on the engine stream). */
int32_t jx_batch_aggregate_records_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_accept_mask,
                                          const void* d_segment_index, uint32_t nsegments, void* d_out_records);

/* ---- Leader role: the leader side of the same ping-pong exchange.
 * jx_leader_prep_init_batch replaces the per-report vdaf.leader_initialized(verify_key, agg_param,
 * nonce = report id, public_share, leader_input_share) of step_aggregation_job_aggregate_init
 * (aggregator/src/aggregator/aggregation_job_driver.rs:344-362): prepare_init with agg_id 0 on the
 * explicit leader input share (meas share || proofs share || [k_blind], LIS bytes each, see
 * jx_engine_leader_sizes). out_prep_shares[n x LPS] receives the prep_share that goes into
 * PingPongMessage::Initialize; out_verdicts[n]: JX_FINISHED (0) = initialized, or
 * JX_PREPARE_INIT_FAILURE (an input-share element >= p, or t a P-th root of unity). The prepare
 * state (output share + corrected joint-rand seed) stays on the device in the new batch.
 * jx_leader_prep_finish_batch replaces leader_continued on the helper's Finish{prep_msg}
 * (aggregation_job_driver.rs:588-602): prepare_next fails (JX_PREPARE_NEXT_FAILURE) unless prep_msg
 * equals the corrected seed. prep_msgs: n x PM (PM = 0: nullable). out_output_shares nullable.
 * *out_batch_id names the leader batch; finish, records and accumulate pass it back. A batch is
 * finished once (a second finish returns JX_E_STATE); its records / accumulation need the finish. */
int32_t jx_engine_leader_sizes(const jx_engine* e, uint32_t* leader_input_share);
int32_t jx_leader_prep_init_batch(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                                  const uint8_t* leader_input_shares, uint8_t* out_prep_shares, uint8_t* out_verdicts,
                                  uint64_t* out_batch_id);
int32_t jx_leader_prep_finish_batch(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* prep_msgs,
                                    uint8_t* out_verdicts, uint8_t* out_output_shares);
/* Device-pointer leader role (inputs resident in HBM; asynchronous on the engine stream, n <= the
 * engine capacity, grown on demand; the report ids are copied into the batch). For Prio3Sum, SumVec
 * and FixedPointBoundedL2VecSum the FLP kernels read the measurement share in place from
 * d_leader_input_shares in 16-byte vectors: that pointer must be 16-byte aligned (JX_E_INVALID
 * otherwise); the stride LIS is a multiple of 16 for every Field128 instance.
 * d_out_verdicts nullable. Finish: d_peer_verdicts (nullable) are the helper's verdicts; a report
 * the helper rejected gets JX_HELPER_STEP_FAILURE. */
int32_t jx_leader_prep_init_device(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_public_shares,
                                   const void* d_leader_input_shares, void* d_out_prep_shares, void* d_out_verdicts,
                                   uint64_t* out_batch_id);
int32_t jx_leader_prep_finish_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_prep_msgs,
                                     const void* d_peer_verdicts, void* d_out_verdicts);
/* jx_leader_prep_init_device with an explicit row stride of d_leader_input_shares (0 = LIS; otherwise
 * >= LIS and a multiple of 16). The leader assembles these rows after HPKE open, so it can pad them for
 * free: with a stride that is a multiple of 128 the in-place FLP kernels read whole cache lines. */
int32_t jx_leader_prep_init_device_ex(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_public_shares,
                                      const void* d_leader_input_shares, uint64_t lis_stride, void* d_out_prep_shares,
                                      void* d_out_verdicts, uint64_t* out_batch_id);

/* Accumulate the output shares of the resident batch `batch_id` (helper, or leader after finish) into
 * the engine's running batch aggregations (the engine as one shard, §8e): report i is added iff
 * verdict == FINISHED and accept_mask[i] != 0 (accept_mask nullable = all), into aggregation
 * `segment[i]` (any u32 batch-aggregation id; segment nullable = 0). Adds to the aggregate share, the
 * report count and the ReportIdChecksum (XOR of SHA-256(report id)). Any number of segments is handled
 * in one pass over the batch (device counting sort by segment). The batch is released: it is
 * accumulated at most once (a second call returns JX_E_STATE). The call returns once the accumulation is
 * queued on the engine stream (the host arrays are consumed before it returns); later calls on the engine
 * see its result (jx_aggregate_read / jx_engine_sync wait for it). A job-sized batch (<= 1,024 reports, no
 * accept_mask, one segment) is deferred: the engine keeps it and adds up to 64 such batches per aggregation
 * in one launch, when its queue is full or at the next call that reads, exports, resets or orders work
 * against the aggregations (jx_aggregate_*, jx_shard_record_export_device, jx_engine_sync,
 * jx_engine_record_event, jx_engine_join_stream, jx_engine_stream). */
int32_t jx_accumulate(jx_engine* e, uint64_t batch_id, uint64_t n, const uint8_t* accept_mask,
                      const uint32_t* segment);
/* Same with device arrays: d_accept_mask (nullable) and d_segment (nullable = all reports into
 * segment_ids[0]) holding, per report, an index into the host array segment_ids[nsegments]; reports
 * whose index is >= nsegments are skipped. segment_ids must not repeat an id (JX_E_INVALID).
 * Asynchronous on the engine stream. */
int32_t jx_accumulate_device(jx_engine* e, uint64_t batch_id, uint64_t n, const void* d_accept_mask,
                             const void* d_segment, const uint32_t* segment_ids, uint32_t nsegments);

/* Fused prep + accumulate (the metric's unit of work): prepare n reports and add every
 * finished one into aggregation `segment`. Host buffers; processed in capacity-sized chunks.
 * out_prep_msgs / out_verdicts nullable. */
int32_t jx_helper_prep_aggregate(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* public_shares,
                                 const uint8_t* helper_input_shares, const uint8_t* leader_prep_shares,
                                 uint32_t segment, uint8_t* out_prep_msgs, uint8_t* out_verdicts);

/* Same with DEVICE pointers (inputs already resident in HBM, e.g. from a torch tensor).
 * Report i goes to aggregation segment_ids[d_segment[i]] (d_segment nullable: all into
 * segment_ids[0]; indices >= nsegments are skipped; ids must not repeat); every finished report is
 * added. No batch is created (staging holds one launch at a time).
 * d_out_prep_msgs / d_out_verdicts are device pointers (nullable). Asynchronous on the engine
 * stream; call jx_engine_sync before reading results. */
int32_t jx_helper_prep_aggregate_device(jx_engine* e, uint64_t n, const void* d_nonces, const void* d_public_shares,
                                        const void* d_helper_input_shares, const void* d_leader_prep_shares,
                                        const void* d_segment, const uint32_t* segment_ids, uint32_t nsegments,
                                        void* d_out_prep_msgs, void* d_out_verdicts);

/* Read aggregation `segment`: encoded aggregate share (OUT x FB, LE), report count, checksum. */
int32_t jx_aggregate_read(jx_engine* e, uint32_t segment, uint8_t* out_agg, uint64_t* count);
int32_t jx_aggregate_checksum(jx_engine* e, uint32_t segment, uint8_t out_checksum[32]);
/* Zero every aggregation. */
int32_t jx_aggregate_reset(jx_engine* e);

/* Multi-GPU combine (compute_aggregate_share, aggregate_share.rs:87-95): write the encoded
 * aggregate share of `segment` to device buffer d_dst (OUT x FB bytes), and sum `nparts`
 * encoded shares laid out back to back at d_parts into d_out (mod p; RCCL's sum is not
 * field addition). Both asynchronous on the engine stream. */
int32_t jx_aggregate_export_device(jx_engine* e, uint32_t segment, void* d_dst);
int32_t jx_aggregate_combine_device(jx_engine* e, const void* d_parts, uint32_t nparts, void* d_out);

/* Shard records for the multi-GPU combine. A record is the encoded aggregate
 * share (OUT x FB) || report count (u64 LE) || checksum (32 B) of one aggregation: the state of
 * one batch_aggregations shard row that compute_aggregate_share merges
 * (aggregator/src/aggregator/aggregate_share.rs:55-96). Export writes this engine's record for
 * `segment` to device memory; combine merges `nrecords` records laid out back to back (e.g. the
 * output of an RCCL all-gather) into one: mod-p sum, count sum, checksum XOR. Both asynchronous
 * on the engine stream. jx_shard_record_bytes gives the record size. */
int32_t jx_shard_record_bytes(const jx_engine* e, uint32_t* bytes);
int32_t jx_shard_record_export_device(jx_engine* e, uint32_t segment, void* d_dst);
int32_t jx_shard_record_combine_device(jx_engine* e, const void* d_records, uint32_t nrecords, void* d_out);

/* Wait for all work on the engine stream. Returns JX_E_INVALID if a combine since the last sync
 * met a non-canonical field element (>= p) in its inputs (the host merge rejects those too). */
int32_t jx_engine_sync(jx_engine* e);
/* The engine's HIP stream (hipStream_t), for callers that order their own work after it. */
int32_t jx_engine_stream(jx_engine* e, void** stream);

/* Producer / consumer ordering of the device-pointer entry points (see Conventions). None blocks the
 * host; all are stream-ordered.
 * jx_engine_wait_stream: engine work queued after this call starts only after all work queued on
 *   `stream` (hipStream_t; NULL = the null stream) so far has completed.
 * jx_engine_join_stream: work queued on `stream` after this call starts only after all engine work
 *   queued so far has completed.
 * jx_engine_wait_event / jx_engine_record_event: the same with a caller-owned hipEvent_t (the engine
 *   stream waits on the event's last record / records the event). With several host threads on one
 *   engine, a wait or join issued by one thread may also order another thread's calls: that only
 *   adds ordering, never removes it.
 * The reference needs none of this: Janus calls prio synchronously on owned values
 * (aggregator/src/aggregator.rs:1945-1967). */
int32_t jx_engine_wait_stream(jx_engine* e, void* stream);
int32_t jx_engine_join_stream(jx_engine* e, void* stream);
int32_t jx_engine_wait_event(jx_engine* e, void* event);
int32_t jx_engine_record_event(jx_engine* e, void* event);

/* Kernel timing with HIP events recorded on the engine stream around each stage.
 * enable != 0 starts collecting (and clears the totals). ms[0] = XOF stage (K1),
 * ms[1] = FLP stage (K3), ms[2] = accumulate (K4), ms[3] = slow-path kernel;
 * launches[0..3] = launch counts. Reading synchronizes the stream. */
int32_t jx_engine_timing(jx_engine* e, int32_t enable);
int32_t jx_engine_timing_read(jx_engine* e, float ms[4], uint64_t launches[4]);

/* Debug knobs (tests and measurements); any other option returns JX_E_INVALID.
 *   option 1: value != 0 routes every report through the slow XOF kernel K1';
 *   option 2: accumulate report chunks, 1..4096 (frees the staging);
 *   option 3: helper K1 kernel: 0 automatic (the fused two-sponge kernel; the lane-split kernel for
 *             launches under one fused wave per SIMD; the lane-pair kernel under one lane-split wave
 *             per SIMD; a word per lane up to one report-wave per SIMD), 3 lane-split, 5 fused,
 *             6 lane pairs, 7 a word per lane (6 and 7: bits <= 32).
 *   option 4: pipelines of jx_helper_prep_aggregate_device / jx_helper_prep_aggregate: 0 automatic
 *             (when a call of one segment spans two or more launches: 2 for the device form, 3 for the
 *             host form), 1 one stream, 2..4 that many (each with its own stream and staging; the
 *             launches alternate over them, their accumulations stay in launch order). A call runs with
 *             fewer when the arena cannot stage them all at once (jx_engine_memory: last_pipelines);
 *   option 5: reports per launch of the fused paths: 0 automatic (whole K1 rounds within ~48 GiB of
 *             staging), else >= 64 (rounded down to a multiple of 64);
 *   option 6: lane-split K1 workgroups per CU (its placement for chain-latency-bound launches): 2 default
 *             (at most two waves per SIMD), 0 no cap, 1..8;
 *   option 7: tests: the device coalescer's gathers wait, up to their window, until `value` jobs have joined
 *             (0: off); needs coalescing on (JX_E_STATE otherwise). Applies to the whole device coalescer;
 *   option 8: jx_accumulate of job-sized batches: 1 deferred and added together (default), 0 one launch per call
 *             (queued deferrals run first);
 *   option 9: run the deferred accumulations now. */
int32_t jx_engine_debug(jx_engine* e, int32_t option, int64_t value);

const char* jx_status_str(int32_t status);
const char* jx_last_error(const jx_engine* e);

#ifdef __cplusplus
}
#endif
#endif /* JX_PRIO3_H */
