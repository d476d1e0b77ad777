// jx_engine_internal.h — engine internals shared by jx_engine.cpp (the C ABI and launch sequencing),
// jx_arena.cpp (the per-device memory arena) and jx_coalesce.cpp (the per-device job coalescer).
// Not part of the ABI: include/jx_prio3.h is.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/jx_prio3.h"
#include "jx_kernels.h"

namespace jxi {

using jx::Cfg;

// ---------------------------------------------------------------------------- device arena (jx_arena.cpp)
// One per HIP device, shared by every engine (every task) on it: launch staging is checked out per call and
// handed back stream-ordered, and resident batches are carved from the same pool. A slab handed back is
// reused by another stream only after that stream waits on the slab's event (recorded where its last user
// finished), so reuse never blocks the host.
struct Slab {
  void* p = nullptr;
  size_t bytes = 0;
  hipEvent_t ev = nullptr;  // recorded on the stream of the slab's last user when it was handed back
  hipStream_t last = nullptr;  // that stream
  bool staging = false;     // per-call staging (comes back soon) vs. a resident batch (comes back on release)
};

struct Arena {
  int device = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t budget = 0;           // bytes the arena may hold (free + checked out)
  uint64_t allocated = 0;        // bytes held (free + checked out + being freed)
  uint64_t freeing = 0;          // bytes of slabs taken off the free list and being destroyed (lock dropped)
  uint64_t in_use = 0;           // checked out
  uint64_t in_use_staging = 0;   // checked out as per-call staging
  uint64_t peak = 0;             // max in_use
  uint64_t allocs = 0, reuses = 0, waits = 0, frees = 0, cross_waits = 0;
  uint32_t engines = 0;          // live engines on this device (the last one out trims the free slabs)
  std::multimap<size_t, Slab> free;
  // per engine (owner pointer): an event recorded after its latest large K1 launch (more reports than a
  // lane-split wave per SIMD), so a launch can tell whether it would share the device with one
  std::map<const void*, hipEvent_t> big;
};

Arena* arena_for(int device);
// Check out `bytes` for work on stream `s` (the stream waits on the slab's last user). may_wait: when the
// budget is held by other callers' staging, wait for a hand-back (a caller that holds no slab may wait;
// one that already holds one must not). hipErrorOutOfMemory when it cannot be satisfied.
hipError_t arena_get(Arena* A, size_t bytes, hipStream_t s, bool staging, bool may_wait, Slab& out);
// Hand a slab back after queueing its last use on stream `s`.
void arena_put(Arena* A, Slab& slab, hipStream_t s);
// Free every slab on the free list (waits for their last users).
void arena_trim(Arena* A);
void arena_engine_add(Arena* A);
void arena_engine_remove(Arena* A);
// Large K1 launches on the device: record one of `owner`'s after it on stream s; is one of another owner's
// still running; forget an owner (engine teardown).
hipError_t arena_big_record(Arena* A, const void* owner, hipStream_t s);
bool arena_big_busy(Arena* A, const void* owner);
void arena_big_forget(Arena* A, const void* owner);

// ---------------------------------------------------------------------------- engine state

// One batch aggregation's device state (aggregate share, report count, ReportIdChecksum).
struct Segment {
  uint4* agg = nullptr;                 // [out_len] canonical
  uint32_t* checksum = nullptr;         // [8]
  unsigned long long* count = nullptr;  // [1]
};

// A resident prepared batch: one aggregation job's reports after prepare_init, holding what
// prepare_next and the accumulation need once the prepare call has returned. Staging (measurement
// and proof shares, coefficients, FLP partials) is per-call scratch from the arena; the output
// shares, verdicts, prep messages (leader: the corrected joint-rand seeds, its prepare state) and
// report ids live here until jx_batch_release / jx_accumulate. Any number of batches can be
// resident, so the aggregation jobs Janus steps concurrently (max_concurrent_job_workers,
// aggregator/src/binary_utils/job_driver.rs:116-138; a leader job holds its prepare state across
// the helper round trip, aggregation_job_driver.rs:396-416 -> :540-701) each keep their own.
struct Batch {
  uint64_t n = 0;
  bool leader = false;
  bool finished = false;      // leader: prepare_next has run (once)
  // a coalesced launch is still writing it (not visible to other calls yet); cleared by the job's caller without
  // the engine mutex (atomic builtins; other calls read it under the mutex)
  bool pending = false;
  Slab slab;                  // one arena allocation: outs | verdicts | msgs | nonces
  hipEvent_t wait_ev = nullptr;  // a slab recycled by a deferred-accumulate flush: that flush (else slab.ev)
  uint4* outs = nullptr;      // interleaved [n/64][out_len][64] (Histogram: the measurement share)
  uint8_t* verdicts = nullptr;
  uint8_t* msgs = nullptr;
  uint8_t* nonces = nullptr;  // report ids, for the checksums
};

// What an accumulation reads: output shares, verdicts, report ids of n reports.
struct AccSrc {
  uint64_t n;
  const uint4* outs;
  const uint8_t* verdicts;
  const uint8_t* nonces;
};

enum { ST_XOF = 0, ST_FLP = 1, ST_ACC = 2, ST_SLOW = 3, NST = 4 };

// Per-call staging regions (stage_acquire flags)
enum : uint32_t {
  SG_IN = 1,     // host-path inputs: nonces, public shares
  SG_HIN = 256,  // host-path helper inputs: helper input shares, leader prep shares
  SG_MEAS = 2,   // measurement-share staging
  SG_PREP = 4,   // proof shares, output shares, FLP coefficients, flags, FLP partials
  SG_RES = 8,    // per-launch verdicts and prep messages of the fused paths
  SG_ACC = 16,   // accumulation: mask, dense segment index, partials
  SG_LEAD = 32,  // host-path leader: input shares (rows of lis_stride) and outbound prep shares
  SG_LMSG = 64,  // host-path leader finish: inbound prep messages
  SG_VK = 128,   // coalesced launches: one verify key per report (16 B; multiproof: HMAC pads, 64 B)
  SG_JOBS = 512, // coalesced launches: the job table (MAX_JOBS_PER_LAUNCH slices)
  SG_ENC = 1024, // encrypted helper inputs: EncRows, ciphertext + plaintext bytes (enc_ct_bytes each), key table,
                 // open status
};

// One job's encrypted input shares (jx_helper_prep_encrypted_batch), as the caller passed them.
struct EncJob {
  const uint64_t* times = nullptr;
  const uint8_t* task_id = nullptr;
  jx_hpke* const* keypairs = nullptr;
  uint32_t nkeys = 0;
  const uint8_t* key_index = nullptr;  // n x 2
  const uint8_t* encs = nullptr;
  const uint8_t* payloads = nullptr;
  const uint64_t* payload_offsets = nullptr;  // n + 1
  uint32_t flags = 0;
  uint64_t ct_bytes(uint64_t n) const { return payload_offsets[n] - payload_offsets[0]; }
};
// The job's EncRows, ciphertexts at ct_base + their offset within the job; key_map: the job's keypair
// index -> the launch's key-table row.
void fill_enc_rows(const EncJob& j, uint64_t n, jx::EncRow* rows, uint64_t ct_base, const uint8_t* key_map);
// jx_hpke.hip
int hpke_device(const jx_hpke* h);
void hpke_key_row(const jx_hpke* h, jx::HpkeKeyRow* out);
hipError_t launch_hpke_rows(const jx::HpkeRowsArgs& a, hipStream_t s);
hipError_t launch_open_mask(const uint8_t* status, uint8_t* verdicts, uint64_t n, hipStream_t s);

struct Coalescer;  // jx_coalesce.cpp

// The engine mutex, bounded-fair: an engine serves many host threads (one per job in flight). With
// std::mutex a thread could wait behind a stream of others (measured: 2 s tail latency at 64 threads); handing
// the lock over in strict arrival order instead makes every contended acquisition wait for the next waiter's
// wake-up (a convoy: three acquisitions per coalesced job). So a running thread may take a free lock unless the
// oldest waiter has waited kBargeUs; waiters queue in arrival order, each on its own condition variable, and
// unlock wakes only the oldest.
class FairMutex {
 public:
  void lock() {
    std::unique_lock<std::mutex> l(m_);
    if (!locked_ && (q_.empty() || std::chrono::steady_clock::now() < q_.front()->since + kBarge)) {
      locked_ = true;
      return;
    }
    Waiter w;
    w.since = std::chrono::steady_clock::now();
    q_.push_back(&w);
    w.cv.wait(l, [&] { return !locked_ && q_.front() == &w; });
    q_.pop_front();
    locked_ = true;
  }
  void unlock() {
    std::lock_guard<std::mutex> l(m_);
    locked_ = false;
    if (!q_.empty()) q_.front()->cv.notify_one();
  }

 private:
  static constexpr std::chrono::microseconds kBarge{1000};
  struct Waiter {
    std::condition_variable cv;
    std::chrono::steady_clock::time_point since;
  };
  std::mutex m_;
  bool locked_ = false;
  std::deque<Waiter*> q_;
};

}  // namespace jxi

struct jx_engine {
  jxi::Cfg cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  // helper K1 launches split over two kernels (prep_core): the lane-pair part runs on this side stream,
  // forked from and joined back into `stream` by events
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_side = nullptr;
  jxi::FairMutex mu;  // held by every entry point for the duration of the call (coalesced prepares: not while waiting)
  jxi::Arena* arena = nullptr;
  // per-call staging, carved from an arena slab by stage_acquire and cleared by its release
  uint64_t cap = 0;       // reports the current staging holds (0: none checked out)
  uint32_t stage_flags = 0;
  uint64_t default_chunk = 0;  // reports per launch of the fused paths (debug option 5 overrides auto_chunk)
  uint64_t auto_chunk = 0;
  uint64_t round_reports = 0;  // reports that fill every K1 wave slot once (0: unknown)
  uint64_t lis_stride = 0;     // row stride of the staged leader input shares (host leader path)
  uint8_t *d_nonces = nullptr, *d_ps = nullptr, *d_his = nullptr, *d_lps = nullptr;
  uint4 *d_meas = nullptr, *d_proof = nullptr, *d_outs = nullptr, *d_coef = nullptr, *d_consts = nullptr;
  uint32_t* d_flags = nullptr;
  uint4* d_part = nullptr;
  uint8_t *d_verdicts = nullptr, *d_msgs = nullptr;  // the fused paths' per-launch results
  uint64_t* d_partials = nullptr;
  uint8_t* d_mask = nullptr;
  uint32_t* d_seg = nullptr;
  uint8_t *d_lis = nullptr, *d_lps_out = nullptr, *d_in_msgs = nullptr;
  uint8_t* d_vkeys = nullptr;
  jx::JobSlice* d_jobs = nullptr;
  // SG_ENC: encrypted helper inputs (enc_ct_bytes: the ciphertext region's size, set before stage_acquire)
  jx::EncRow* d_encrows = nullptr;
  uint8_t *d_ct = nullptr, *d_pt = nullptr, *d_status = nullptr;
  jx::HpkeKeyRow* d_keys = nullptr;
  uint64_t enc_ct_bytes = 0;
  uint32_t acc_chunks = 0;  // report chunks of the accumulate kernel (0: acc_nchunks picks)
  std::map<uint32_t, jxi::Segment> segs;  // running batch aggregations (the engine as one shard)
  std::vector<jxi::Slab> seg_slabs;       // their states, kSegsPerSlab per arena slab
  uint32_t seg_next = 0;                  // next free state in seg_slabs.back()
  // resident prepared batches by handle; handles are never reused
  std::map<uint64_t, jxi::Batch> batches;
  uint64_t batch_gen = 0;
  std::atomic<uint64_t> last_batch{0};  // a coalesced prepare sets it without the engine mutex
  // segmented accumulation: pointers into the call's arena scratch while it runs (accumulate_many)
  uint32_t* d_segx = nullptr;  // cnt, off, cursor [SEG_MAX each], ioff [SEG_MAX + 1], nitems [2]
  uint32_t* d_perm = nullptr;
  uint4* d_items = nullptr;
  uint64_t* d_spart = nullptr;
  void** d_ptrs = nullptr;  // [3][nptrs]: aggs, counts, checksums of the call's segments (upload_targets)
  // pinned host copies of the pointer table, double-buffered: buffer k is rewritten only after the
  // upload that last read it has completed (ev_ptrs[k]), so no call waits for its own work
  void** h_ptrs[2] = {nullptr, nullptr};
  uint64_t h_ptrs_cap[2] = {0, 0};
  hipEvent_t ev_ptrs[2] = {nullptr, nullptr};
  int ptrs_k = 0;
  // pinned host staging for the small host arrays of jx_accumulate (mask, dense segment index), so the
  // call returns once queued: reused after ev_hacc (the last upload that read it) has completed
  uint8_t* h_acc = nullptr;
  uint64_t h_acc_cap = 0;
  hipEvent_t ev_hacc = nullptr;
  std::vector<uint32_t> h_dense;
  // deferred small accumulations: jx_accumulate of an unmasked batch of <= ACC_SMALL reports into one
  // aggregation parks the batch here; a flush runs one accumulate_multi launch per aggregation (a full queue,
  // or any call that reads, exports, resets or orders work against the aggregations)
  std::vector<std::pair<jxi::Batch, uint32_t>> accq;  // (batch, aggregation id)
  uint64_t accq_reports = 0;
  bool acc_defer = true;      // debug option 8
  // batch slabs the flushes read, kept for the engine's next batches (no arena round trip, one event per flush)
  std::multimap<size_t, jxi::Slab> recycle;
  size_t recycle_bytes = 0;
  hipEvent_t ev_flush = nullptr;
  uint64_t acc_flushes = 0, acc_deferred = 0;
  uint32_t* d_err = nullptr;  // combine kernels: non-canonical input seen (reported by jx_engine_sync)
  // timing
  bool timing = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  double ms[jxi::NST] = {0, 0, 0, 0};
  uint64_t launches[jxi::NST] = {0, 0, 0, 0};
  uint32_t force_slow = 0;
  uint32_t k1_split = 0;  // helper K1: 0 automatic, 3 lane-split, 5 fused, 6 lane pairs (debug option 3)
  uint32_t lanes_wg_cap = 2;  // lane-split K1 workgroups per CU (debug option 6; 0: no cap)
  // producer / consumer ordering (jx_engine_wait_stream / jx_engine_join_stream): reused events
  hipEvent_t ev_wait = nullptr, ev_join = nullptr;
  // Concurrent pipelines of the fused paths (pipes_for): child engines with their own stream run
  // K1 -> K3 -> K4 of alternate launches, so launches of different phases share the device; the K4s stay
  // in launch order through ev_pipe. Their staging comes from the arena per call.
  std::vector<jx_engine*> pipes;
  uint32_t npipes = 0;  // 0: automatic (debug option 4)
  uint32_t last_pipes = 0;  // pipelines the last fused call ran (fewer than asked when staging was short)
  bool is_pipe = false;  // a child: d_consts belongs to the parent
  hipEvent_t ev_pipe = nullptr;
  // coalesced prepares (jx_engine_coalesce): the device's coalescer for this engine's Prio3 instance
  jxi::Coalescer* coal = nullptr;
  bool coalesce = false;
};

namespace jxi {

// errors: per calling thread (jx_last_error)
int32_t fail(jx_engine* e, int32_t code, const std::string& msg);
std::string& thread_error();

#define HIPCHK(e, call)                                                                                   \
  do {                                                                                                    \
    hipError_t _st = (call);                                                                              \
    if (_st != hipSuccess)                                                                                \
      return ::jxi::fail((e), _st == hipErrorOutOfMemory ? JX_E_NOMEM : JX_E_HIP,                         \
                         std::string(#call) + ": " + hipGetErrorString(_st));                             \
  } while (0)

// Per-call staging: an arena slab carved into the engine's d_* regions named by the flags; released
// (handed back stream-ordered on the engine's stream) when the Stage goes out of scope.
struct Stage {
  jx_engine* e = nullptr;
  Slab slab;
  Stage() = default;
  Stage(const Stage&) = delete;
  Stage& operator=(const Stage&) = delete;
  ~Stage() { release(); }
  void release();
};
int32_t stage_acquire(jx_engine* e, uint64_t n, uint32_t flags, Stage& st, bool may_wait = true);
size_t stage_bytes(const jx_engine* e, uint64_t cap, uint32_t flags);

int32_t prep_core(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* his,
                  const uint8_t* lps, uint8_t* verdicts, uint8_t* msgs, uint4* outs, const uint8_t* lis = nullptr,
                  uint8_t* lps_out = nullptr, uint64_t lis_rs = 0, const uint8_t* vkeys = nullptr,
                  hipEvent_t before_flp = nullptr,  // the FLP stage (K3) also waits on this event
                  const std::function<int32_t()>* after_k1 = nullptr);  // queued right after K1 (before K1', K3)
uint4* staging_outs(jx_engine* e);
int32_t batch_new(jx_engine* e, uint64_t n, bool leader, uint64_t* id, Batch** out);
void batch_free(jx_engine* e, std::map<uint64_t, Batch>::iterator it);
int32_t drain_timing(jx_engine* e);
size_t align256(size_t v);
uint32_t vk_row_bytes(const Cfg& c);
void vk_row(const Cfg& c, uint8_t* dst);  // this engine's verify key as one SG_VK row
jx_engine* new_child(jx_engine* parent);  // a pipeline / coalescer lane: own stream, shared consts

// ---------------------------------------------------------------------------- coalescer (jx_coalesce.cpp)
Coalescer* coalescer_for(jx_engine* e);
// A coalesced helper prepare / leader prepare_init of a job of n reports: joins the device's next launch
// with other engines' (tasks') jobs of the same Prio3 instance. Blocks the calling thread until its results
// are in the caller's buffers; the engine mutex is not held while waiting.
// enc (nullable): the job's input shares are encrypted (his unused); out_status (nullable): their open status.
int32_t coalesced_helper_prep(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* his,
                              const uint8_t* lps, uint8_t* out_msgs, uint8_t* out_verdicts, uint64_t* out_batch_id,
                              const EncJob* enc = nullptr, uint8_t* out_status = nullptr);
// Whether a job of n reports (ct_bytes of ciphertexts when encrypted) fits one of the coalescer's launches for
// its role; larger jobs take the direct path.
bool coalescer_accepts(const jx_engine* e, bool leader, uint64_t n, bool encrypted, uint64_t ct_bytes);
int32_t coalesced_leader_init(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* lis,
                              uint8_t* out_prep_shares, uint8_t* out_verdicts, uint64_t* out_batch_id);
void coalescer_stats(const jx_engine* e, uint64_t out[16]);
void coalescer_set_window(jx_engine* e, uint32_t window_us);  // 0: automatic
void coalescer_set_min_jobs(jx_engine* e, uint32_t jobs);     // debug option 7
void coalescer_release(jx_engine* e);

}  // namespace jxi
