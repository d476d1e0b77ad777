// jx_coalesce.cpp — coalesced prepares: the aggregation jobs of every task of one Prio3 instance on one GPU
// share launches.
//
// Janus prepares one aggregation job per request: the helper's handle_aggregate_init_generic runs one
// AggregationJobInitializeReq (aggregator/src/aggregator.rs:1712-2013), jobs hold 10-100 reports
// (docs/samples/basic_config/aggregation_job_creator.yaml:23-26), and many are in flight (tokio workers
// on the helper; the leader steps max_concurrent_job_workers jobs at once, binary_utils/job_driver.rs:116).
// A GPU launch of 100 SumVec reports is bound by one report's chain of ~800 dependent Keccak
// permutations (~3 ms) and leaves the device nearly empty; one engine call at a time serialises those
// latencies. Here the jobs that arrive together become ONE launch:
//
//   caller thread (jx_helper_prep_batch / jx_helper_prep_encrypted_batch / jx_leader_prep_init_batch with
//   coalescing on):
//     1. creates its job's resident batch on its own engine (its task: verify key, batches, aggregations);
//     2. reserves rows in the lane that is gathering for its role, and copies its inputs and its verify key
//        into the lane's pinned host rows itself (callers copy in parallel); an encrypted job copies its
//        ciphertexts and EncRows instead of helper input shares (its keypairs join the launch's key table);
//     3. waits (without its engine's mutex) until the launch is done, then copies its verdicts / prep
//        messages / prep shares / open status out of the lane's pinned result rows and returns its batch.
//   dispatcher thread, one per role (leader and helper jobs gather in lanes of their own, so interleaved
//     traffic of an aggregator that is leader for some tasks and helper for others, aggregator_core/src/
//     task.rs:598, never closes the other role's gather): closes its gathering lane when it holds a full
//     launch, once no job has joined for a quiet period while no other launch of the role runs (a running
//     launch's callers join this one when it returns), or when the gathering window has passed; then, on
//     the lane's stream: one upload per input region, the HPKE open of the encrypted reports into the helper
//     input-share rows (jx_hpke.hip), K1 -> K1' -> K3 over all jobs (each report with its own task's verify
//     key, Bufs::vkeys), the open-status mask, one scatter kernel that copies every job's slice into its
//     batch, one download of the results, a host flag (launch_host_signal).
//   completer thread: spins on the running launches' host flags (no runtime call) and wakes their callers.
// Up to kLanes launches are gathering or in flight, so jobs that arrive while one runs start on the next lane
// at once. A lane's pinned rows are sized to the role's recent launches and returned after kIdleFreeMs
// without jobs (jx_engine_memory: coalesce_pinned_bytes).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <thread>

#include "jx_engine_internal.h"

using namespace jx;

namespace jxi {

namespace {

using clk = std::chrono::steady_clock;
constexpr uint32_t kLanes = 4;                   // one gathering lane per role + launches in flight
constexpr uint32_t kMaxLanes = 8;                // JX_COAL_LANES (measurement) may raise the lanes up to this
constexpr size_t kPinnedBudget = 512ull << 20;   // the largest lane: pinned input rows
constexpr uint32_t kIdleFreeMs = 2000;           // pinned rows go back to the OS after this long without jobs
constexpr uint64_t kMinLaneReports = 1024;
constexpr uint32_t kFlagStride = 16;             // uint32 per lane flag: one 64-byte line each
enum Role { HELPER = 0, LEADER = 1, NROLES = 2 };

struct CReq {
  jx_engine* e = nullptr;
  int role = HELPER;
  uint64_t n = 0, first = 0, id = 0;
  const EncJob* enc = nullptr;  // encrypted helper inputs
  uint64_t ct_first = 0, ct_bytes = 0;
  uint8_t key_map[JX_ENC_MAX_KEYPAIRS] = {0};
  JobSlice dst{};
  hipEvent_t batch_ev = nullptr;  // the batch slab's last user (the lane waits on it)
  uint8_t* out_msgs = nullptr;
  uint8_t* out_verdicts = nullptr;
  uint8_t* out_prep_shares = nullptr;
  uint8_t* out_status = nullptr;
  int32_t rc = 0;
  std::string err;
  bool done = false;
  // this job's caller waits here for its launch: its own mutex and condition variable (no herd of wake-ups, and
  // the callers of a completed launch do not queue on the coalescer's mutex to leave their wait)
  std::mutex m;
  std::condition_variable cv;
};

enum LaneState { FREE, GATHER, SEALED, RUNNING, DONE };

struct Lane {
  jx_engine* q = nullptr;  // child engine: own stream, staging from the arena per launch
  uint8_t* h_in = nullptr;
  size_t h_in_cap = 0;
  uint8_t* h_out = nullptr;  // host-coherent: the launch's download kernel writes it over PCIe
  size_t h_out_cap = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr;  // the same pinned rows as the device addresses them
  clk::time_point grown;  // when the pinned rows were last (re)allocated
  hipEvent_t ev_done = nullptr;
  uint32_t seq = 0;       // launches queued on this lane (the host flag's value once the latest is done)
  // the leader prep shares' upload beside K1 (K1 reads only their joint-rand parts; K3 the rest)
  hipStream_t up = nullptr;
  hipEvent_t ev_up0 = nullptr, ev_up = nullptr;
  bool all_back = false;  // every caller of the role's completed launches has joined: close without a quiet period
  LaneState state = FREE;
  int role = HELPER;
  bool full = false;      // a caller could not fit: close now
  bool enc = false;       // the layout holds the encrypted-input regions
  bool has_enc = false;   // a job of this gather is encrypted
  uint64_t reports = 0, cap_reports = 0, ct_bytes = 0, ct_cap = 0;
  uint32_t copying = 0;
  std::atomic<uint32_t> unconsumed{0};  // callers still to copy their results out (the last one frees the lane)
  std::vector<CReq*> reqs;
  std::vector<const jx_hpke*> keys;  // the launch's key table
  clk::time_point opened, launched, last_arrival;
  // region offsets in h_in (rows of cap_reports)
  size_t o_non = 0, o_ps = 0, o_his = 0, o_lps = 0, o_lis = 0, o_vk = 0, o_jobs = 0, o_enc = 0, o_ct = 0, o_keys = 0;
  // region offsets in h_out
  size_t r_ver = 0, r_msg = 0, r_lps = 0, r_st = 0;
};

// per role: its gathering lane, its dispatcher and the close policy's state
struct RoleState {
  int open = -1;
  std::condition_variable cv;  // the role's dispatcher: a job joined, copies done, a launch completed
  uint32_t nrunning = 0;       // the role's launches queued on the device and not yet done
  uint64_t run_reports = 0;    // their reports
  uint32_t expect = 0;         // jobs of completed launches not yet back (closed-loop callers return)
  clk::time_point expect_until;  // ... expected until then
  double ewma_us = 0;          // launch latency
  uint64_t peak = 0;           // largest launch of the last second (lane sizing)
  clk::time_point peak_at;
  uint64_t launches = 0, jobs = 0;
  std::thread dispatcher;
};

}  // namespace

struct Coalescer {
  std::string key;
  int device = 0;
  jx_engine* base = nullptr;  // owns the constant tables the lanes share
  std::mutex mu;
  std::condition_variable cv_comp, cv_lane;  // the completer (a launch queued); callers waiting for a free lane
  Lane lanes[kMaxLanes];
  uint32_t nlanes = kLanes;
  RoleState role[NROLES];
  std::vector<int> running;
  // per lane, a host-coherent pinned flag (one per 64-byte line) the lane's launch sets to its seq when done
  uint32_t* hflag = nullptr;
  uint32_t* dflag = nullptr;  // the same memory as the device addresses it
  std::thread completer;
  bool stop = false;
  uint32_t refs = 0;
  uint32_t window_us = 0;   // 0: automatic
  uint32_t min_jobs = 0;    // debug option 7 (tests): a gather waits (up to its window) for this many jobs
  uint64_t max_reports = 0; // reports per launch
  uint64_t flat_reports = 0;  // launches up to this size take the same device time (merge_groups)
  std::atomic<bool> enc_seen{false};  // helper lanes lay out the encrypted-input regions from now on
  clk::time_point last_job;
  size_t pinned = 0;        // bytes of pinned host rows held by the lanes
  uint64_t launches = 0, jobs = 0, reports = 0, enc_jobs = 0;
  // per-phase totals (microseconds, summed over launches): gathering (first job -> closed), the callers'
  // input copies after the close, queueing the launch, and the device (queued -> done event)
  double t_gather = 0, t_copy = 0, t_enqueue = 0, t_device = 0;
};

static std::mutex g_mu;
static std::map<std::string, Coalescer*> g_coal;

static std::string coal_key(const jx_engine* e) {
  const Cfg& c = e->cfg;
  return std::to_string(e->device) + "/" + std::to_string(c.algo) + "/" + std::to_string(c.bits) + "/" +
         std::to_string(c.length) + "/" + std::to_string(c.chunk) + "/" + std::to_string(c.np);
}

// A gathering lane closes at once while no launch of its role runs and no caller of a completed launch is
// still due back (a lone caller, or the device idle: nothing to wait for). Otherwise it closes once no job
// has joined it for kQuietUs, fewer than kMaxRunning launches of its role are on the device, and the callers
// of the launches that completed meanwhile have come back (up to kRejoinUs after the completion: copying
// their results, accumulating, preparing their next job), so closed-loop callers share a launch per round
// trip instead of splitting into fragments; open-loop arrivals wait at most the window. A launch's device
// time is nearly flat in its size below a K1 round (the per-report sponge chain), so two launches in flight,
// each carrying every job that is back, is the measured optimum (DESIGN.md §5.4:
// profiles/r05_coalesce_policy_ab.jsonl, 1 / 2 / 3 running; profiles/r05_coalesce_rejoin_retune.jsonl, the
// rejoin window re-measured on the final kernels and host path: 1 ms, against 1.5 / 2 / 3 ms).
constexpr uint32_t kQuietUs = 100;
constexpr uint32_t kRejoinUs = 1000;
// The rejoin window grows to 30 % of the role's launch latency when that is longer than kRejoinUs: callers come
// back later when the host is busy, e.g. beside a leader role's multi-MB input copies. 32 helper + 32 leader
// threads of 100-report SumVec jobs on one Prio3 instance (profiles/r06_rejoin_ab.jsonl): helper 183-198k ->
// 291-320k reports/s, leader 98-99k -> 110-124k, leader jobs per launch 16-20 -> 31 (as many as alone); one role
// alone unchanged. JX_COAL_REJOIN_FRAC (percent, 0 = the fixed 1 ms) overrides it for A/B.
static uint32_t rejoin_us(const RoleState& R) {
  static const uint32_t pct = [] {
    const char* s = getenv("JX_COAL_REJOIN_FRAC");
    const int x = s ? atoi(s) : 30;
    return x >= 0 && x <= 100 ? (uint32_t)x : 30u;
  }();
  const double w = R.ewma_us * pct / 100.0;
  return w > kRejoinUs ? (uint32_t)w : kRejoinUs;
}
constexpr uint32_t kMaxRunning = 2;
// Below flat_reports (the word-per-lane K1's range, 1,024 SumVec reports) a launch takes the same time whatever its
// size. A gather that opens while a launch of its role runs, and that fits that range together with it, waits for
// that launch's callers instead of closing as a group of its own: a late caller would otherwise split a few
// workers into two groups that alternate for good, each launch sharing the CUs with the other's (10 x 100-report
// jobs: 5.3-7.4 jobs per launch and 292-317k reports/s in the runs that split, 10 and ~330k otherwise). A
// completion also clears the gathering lane's all-back mark, which was stale and closed such a gather before the
// callers it now expects were back. Measured (profiles/r06_jobs_merge_ab.jsonl, runs r06mgc/d): every 10-worker
// run at 10 jobs per launch, 64 x 100 unchanged (1.15-1.21M), sealed 64 x 100 0.90-0.91M against 0.84-0.87M. An
// 8,192-report range instead (the lane-pair kernel's) made 64 x 100 take turns on the device: 0.89M.
// JX_COAL_MERGE=0 turns it off (A/B).
static bool merge_groups() {
  static const bool v = [] {
    const char* s = getenv("JX_COAL_MERGE");
    return !(s && atoi(s) == 0);
  }();
  return v;
}
// JX_COAL_MAX_RUNNING (measurement): launches of a role in flight before a gather waits for one to complete
static uint32_t max_running() {
  static const uint32_t v = [] {
    const char* s = getenv("JX_COAL_MAX_RUNNING");
    const int x = s ? atoi(s) : 0;
    return x >= 1 && x <= (int)kMaxLanes - 1 ? (uint32_t)x : kMaxRunning;
  }();
  return v;
}

// The longest a gathering lane waits for more jobs (automatic: 1.5x the role's recent launch latency,
// 0.1-20 ms). It matters while another launch runs: the jobs that launch returns join this one instead of
// starting a fragment of their own (closed-loop callers then share one launch per round trip).
static uint32_t cur_window_us(const Coalescer* C, int role) {
  if (C->window_us) return C->window_us;
  const double ew = C->role[role].ewma_us;
  if (ew <= 0) return 2000;
  double w = 1.5 * ew;
  return (uint32_t)(w < 100 ? 100 : (w > 20000 ? 20000 : w));
}

// bytes of one report's pinned input row / result row
static size_t in_row(const Cfg& c, int role, bool enc) {
  size_t b = 16 + c.ps_bytes + vk_row_bytes(c);
  b += role == LEADER ? c.lis_bytes : (size_t)c.his_bytes + c.lps_bytes;
  if (enc) b += sizeof(EncRow);
  return b;
}
// the ciphertext bytes a lane budgets per report: a PlaintextInputShare with no extensions (2 + 4 + HIS) and
// the GCM tag, plus 64 bytes of extensions
static uint64_t ct_row(const Cfg& c) { return (c.his_bytes + 6 + 16 + 64 + 15) / 16 * 16; }
static uint64_t lane_max_reports(const Coalescer* C, int role, bool enc) {
  uint64_t cap = kPinnedBudget / in_row(C->base->cfg, role, enc);
  if (cap > C->max_reports) cap = C->max_reports;
  return cap < 64 ? 64 : cap / 64 * 64;
}

static void lane_free_pinned(Coalescer* C, Lane& L) {
  if (L.h_in) (void)hipHostFree(L.h_in);
  if (L.h_out) (void)hipHostFree(L.h_out);
  C->pinned -= L.h_in_cap + L.h_out_cap;
  L.h_in = L.h_out = L.d_in = L.d_out = nullptr;
  L.h_in_cap = L.h_out_cap = 0;
}

// Lay a FREE lane's pinned rows out for a gather of `role` that must take a job of n reports (ct bytes of
// ciphertexts): capacity for twice the role's largest recent launch (at least kMinLaneReports and the job,
// at most a launch within the pinned budget), grown (or shrunk, when 4x too large for over a second) to fit.
// With C->mu held. JX_E_INVALID when the job is larger than any lane of its role.
static int32_t lane_layout(Coalescer* C, Lane& L, int role, uint64_t n, uint64_t ct) {
  const Cfg& c = C->base->cfg;
  const bool enc = role == HELPER && C->enc_seen;
  const uint64_t cmax = lane_max_reports(C, role, enc);
  if (n > cmax || ct > kPinnedBudget / 2) return JX_E_INVALID;
  RoleState& R = C->role[role];
  const auto now = clk::now();
  const uint64_t recent = now - R.peak_at < std::chrono::seconds(1) ? R.peak : 0;
  uint64_t cap = kMinLaneReports;
  while (cap < 2 * recent || cap < n) cap <<= 1;
  if (cap > cmax || C->min_jobs) cap = cmax;  // a test holding the gather for its jobs (option 7): room for all
  size_t off = 0;
  auto take = [&](size_t& o, size_t bytes) {
    o = off;
    off += align256(bytes ? bytes : 1);
  };
  take(L.o_non, cap * 16);
  take(L.o_ps, cap * c.ps_bytes);
  if (role == LEADER) {
    take(L.o_lis, cap * c.lis_bytes);
    L.o_his = L.o_lps = 0;
  } else {
    take(L.o_his, cap * c.his_bytes);
    take(L.o_lps, cap * c.lps_bytes);
    L.o_lis = 0;
  }
  take(L.o_vk, cap * vk_row_bytes(c));
  take(L.o_jobs, (size_t)MAX_JOBS_PER_LAUNCH * sizeof(JobSlice));
  uint64_t ct_cap = 0;
  if (enc) {
    ct_cap = cap * ct_row(c);
    if (ct_cap < ct) ct_cap = ct;
    take(L.o_enc, cap * sizeof(EncRow));
    take(L.o_ct, ct_cap);
    take(L.o_keys, ENC_MAX_KEYS * sizeof(HpkeKeyRow));
  }
  const size_t in_bytes = off;
  off = 0;
  take(L.r_ver, cap);
  take(L.r_msg, cap * c.seed);
  if (role == LEADER) take(L.r_lps, cap * c.lps_bytes);
  if (enc) take(L.r_st, cap);
  const size_t out_bytes = off;
  const bool oversized = L.h_in_cap > 4 * in_bytes && now - L.grown > std::chrono::seconds(1);
  if (L.h_in_cap < in_bytes || L.h_out_cap < out_bytes || oversized) {
    lane_free_pinned(C, L);
    // mapped: the launch's upload and download kernels address the rows directly (launch_copy_regions)
    if (hipHostMalloc((void**)&L.h_in, in_bytes, hipHostMallocMapped) != hipSuccess) {
      L.h_in = nullptr;
      return JX_E_NOMEM;
    }
    L.h_in_cap = in_bytes;
    if (hipHostMalloc((void**)&L.h_out, out_bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      L.h_out = nullptr;
      C->pinned += L.h_in_cap;
      lane_free_pinned(C, L);
      return JX_E_NOMEM;
    }
    L.h_out_cap = out_bytes;
    if (hipHostGetDevicePointer((void**)&L.d_in, L.h_in, 0) != hipSuccess ||
        hipHostGetDevicePointer((void**)&L.d_out, L.h_out, 0) != hipSuccess) {
      C->pinned += in_bytes + out_bytes;
      lane_free_pinned(C, L);
      return JX_E_HIP;
    }
    C->pinned += in_bytes + out_bytes;
    L.grown = now;
  }
  L.cap_reports = cap;
  L.ct_cap = ct_cap;
  L.role = role;
  L.enc = enc;
  return JX_OK;
}

// Queue one closed gather on its lane's stream. Returns JX_OK or an error for every job of the launch.
static int32_t launch_lane(Coalescer* C, Lane& L, std::string& err) {
  jx_engine* q = L.q;
  const Cfg& c = q->cfg;
  const uint64_t m = L.reports;
  const bool leader = L.role == LEADER;
  bool queued = false;  // device work of this launch is on the lane stream
  auto bad = [&](hipError_t st, const char* what) {
    err = std::string("coalesced launch: ") + what + ": " + hipGetErrorString(st);
    // the callers free their batches on the error: let the work already queued into them finish first (their
    // slabs' events are recorded on their engines' streams, not on this one)
    if (queued) {
      (void)hipStreamSynchronize(L.up);
      (void)hipStreamSynchronize(q->stream);
    }
    return st == hipErrorOutOfMemory ? JX_E_NOMEM : JX_E_HIP;
  };
  if (hipSetDevice(C->device) != hipSuccess) return JX_E_HIP;
  const bool inpl = leader && (c.algo == ALGO_SUM || c.algo == ALGO_SUMVEC || c.algo == ALGO_FIXEDPOINT_L2);
  uint32_t fl = SG_IN | SG_PREP | SG_RES | SG_VK | SG_JOBS;
  fl |= leader ? SG_LEAD : SG_HIN;
  if (!inpl) fl |= SG_MEAS;
  if (L.has_enc) {
    fl |= SG_ENC;
    q->enc_ct_bytes = L.ct_cap;  // the lane's budget: launches of varying size reuse the lane's slab
  }
  // staging for a power of two of reports (>= 1,024): launches of varying size reuse the lane's slab
  uint64_t cap = 1024;
  while (cap < m) cap <<= 1;
  Stage st;
  int32_t rc = stage_acquire(q, cap, fl, st);
  if (rc) {
    err = thread_error();
    return rc;
  }
  // Transfers are kernels on the lane's streams reading / writing the mapped pinned rows (launch_copy_regions): a
  // copy-engine command of this lane could queue behind another lane's download, which waits for that lane's
  // K1 (measured 1-2 ms stalls per launch at 64 x 100-report jobs, profiles/r06_jobs_trace_*).
  const uint8_t* hin = L.d_in;
  auto add = [](CopyArgs& a, void* dst, uint64_t dstride, const void* src, uint64_t sstride, uint64_t width,
                uint64_t rows) {
    if (width && rows) a.r[a.nr++] = CopyRegion{(uint8_t*)dst, (const uint8_t*)src, dstride, sstride, rows, width};
  };
  auto flat = [&](CopyArgs& a, void* dst, size_t off, uint64_t bytes) { add(a, dst, 0, hin + off, 0, bytes, 1); };
  queued = true;
  CopyArgs ua{};
  flat(ua, q->d_nonces, L.o_non, m * 16);
  if (c.ps_bytes) flat(ua, q->d_ps, L.o_ps, m * c.ps_bytes);
  if (!leader) flat(ua, q->d_his, L.o_his, m * c.his_bytes);
  // Helper: the leader prep shares are most of the bytes (SumVec 8x1000/88: 2,864 of 2,960 per report) and only
  // the FLP stage reads them whole; K1 reads each row's last 16 bytes (the leader's joint-rand part). Those go
  // first on the lane stream, the rest of the rows on the lane's upload stream beside K1, and K3 waits for it.
  const bool split_lps = !leader && c.lps_bytes > 16 && c.algo != ALGO_COUNT && c.algo != ALGO_SUMVEC_F64_MULTIPROOF;
  const size_t P = c.lps_bytes;
  if (!leader && !split_lps) flat(ua, q->d_lps, L.o_lps, m * P);
  if (split_lps) add(ua, q->d_lps + P - 16, P, hin + L.o_lps + P - 16, P, 16, m);
  if (leader) add(ua, q->d_lis, q->lis_stride, hin + L.o_lis, c.lis_bytes, c.lis_bytes, m);
  flat(ua, q->d_vkeys, L.o_vk, m * vk_row_bytes(c));
  if (L.has_enc) {
    flat(ua, q->d_encrows, L.o_enc, m * sizeof(EncRow));
    flat(ua, q->d_ct, L.o_ct, L.ct_bytes);
    flat(ua, q->d_keys, L.o_keys, L.keys.size() * sizeof(HpkeKeyRow));
  }
  JobSlice* h_jobs = reinterpret_cast<JobSlice*>(L.h_in + L.o_jobs);
  uint64_t max_job = 0;
  for (size_t k = 0; k < L.reqs.size(); k++) {
    h_jobs[k] = L.reqs[k]->dst;
    if (L.reqs[k]->n > max_job) max_job = L.reqs[k]->n;
  }
  flat(ua, q->d_jobs, L.o_jobs, L.reqs.size() * sizeof(JobSlice));
  hipError_t s = launch_copy_regions(ua, q->stream);
  // the rest of the leader prep-share rows: on the lane's upload stream once the lane's previous launch has read
  // d_lps (ev_up0), queued right after K1 so that nothing but the upload and this record precede K1
  hipEvent_t before_flp = nullptr;
  std::function<int32_t()> side;
  if (s == hipSuccess && split_lps) {
    s = hipEventRecord(L.ev_up0, q->stream);
    before_flp = L.ev_up;
    side = [&]() -> int32_t {
      CopyArgs ra{};
      add(ra, q->d_lps, P, hin + L.o_lps, P, P - 16, m);
      hipError_t t = hipStreamWaitEvent(L.up, L.ev_up0, 0);
      if (t == hipSuccess) t = launch_copy_regions(ra, L.up);
      if (t == hipSuccess) t = hipEventRecord(L.ev_up, L.up);
      if (t != hipSuccess)  // prep_core returns it; the launch's error path synchronises the lane's streams
        return fail(q, t == hipErrorOutOfMemory ? JX_E_NOMEM : JX_E_HIP,
                    std::string("coalesced launch: upload: ") + hipGetErrorString(t));
      return JX_OK;
    };
  }
  if (s != hipSuccess) return bad(s, "upload");
  if (L.has_enc) {  // open the encrypted reports into their helper input-share rows
    HpkeRowsArgs ha{m, q->d_encrows, q->d_ct, q->d_pt, q->d_keys, (uint32_t)L.keys.size(), q->d_nonces, q->d_ps,
                    c.ps_bytes, q->d_his, c.his_bytes, q->d_status};
    s = launch_hpke_rows(ha, q->stream);
    if (s != hipSuccess) return bad(s, "hpke open");
  }
  rc = prep_core(q, m, q->d_nonces, q->d_ps, q->d_his, q->d_lps, q->d_verdicts, q->d_msgs, staging_outs(q),
                 leader ? q->d_lis : nullptr, leader ? q->d_lps_out : nullptr, leader ? q->lis_stride : 0, q->d_vkeys,
                 before_flp, side ? &side : nullptr);
  if (rc) {
    err = thread_error();
    (void)hipStreamSynchronize(L.up);
    (void)hipStreamSynchronize(q->stream);
    return rc;
  }
  if (L.has_enc) {
    s = launch_open_mask(q->d_status, q->d_verdicts, m, q->stream);
    if (s != hipSuccess) return bad(s, "open mask");
  }
  // every job's batch slab (only the scatter writes it): after its previous user
  for (CReq* r : L.reqs) {
    s = hipStreamWaitEvent(q->stream, r->batch_ev, 0);
    if (s != hipSuccess) return bad(s, "hipStreamWaitEvent");
  }
  s = launch_scatter_jobs(c, q->d_jobs, (uint32_t)L.reqs.size(), max_job,
                          staging_outs(q), q->d_verdicts, q->d_msgs, q->d_nonces, q->stream);
  if (s != hipSuccess) return bad(s, "scatter");
  CopyArgs da{};
  add(da, L.d_out + L.r_ver, 0, q->d_verdicts, 0, m, 1);
  if (c.jr_len) add(da, L.d_out + L.r_msg, 0, q->d_msgs, 0, m * c.seed, 1);
  if (leader) add(da, L.d_out + L.r_lps, 0, q->d_lps_out, 0, m * c.lps_bytes, 1);
  if (L.has_enc) add(da, L.d_out + L.r_st, 0, q->d_status, 0, m, 1);
  s = launch_copy_regions(da, q->stream);
  if (s == hipSuccess) s = hipEventRecord(L.ev_done, q->stream);
  if (s == hipSuccess) s = launch_host_signal(C->dflag + kFlagStride * (&L - C->lanes), ++L.seq, q->stream);
  if (s != hipSuccess) return bad(s, "download");
  return JX_OK;  // st hands the staging back stream-ordered
}

static void finish_lane(Coalescer* C, Lane& L, int32_t rc, const std::string& err) {
  L.unconsumed.store((uint32_t)L.reqs.size());
  L.state = DONE;
  if (L.reqs.empty()) {
    L.state = FREE;
    C->cv_lane.notify_all();
  }
  for (CReq* r : L.reqs) {
    r->rc = rc;
    if (rc) r->err = err;
    // notify under the caller's mutex: once it sees done it may return and destroy r
    std::lock_guard<std::mutex> g(r->m);
    r->done = true;
    r->cv.notify_one();
  }
}

// After kIdleFreeMs without a job, hand the FREE lanes' pinned rows back (outside the lock: hipHostFree may
// wait for the device).
static void maybe_release_idle(Coalescer* C, std::unique_lock<std::mutex>& lk) {
  if (clk::now() - C->last_job < std::chrono::milliseconds(kIdleFreeMs)) return;
  std::vector<void*> give;
  for (Lane& L : C->lanes) {
    if (L.state != FREE || !L.h_in) continue;
    give.push_back(L.h_in);
    give.push_back(L.h_out);
    C->pinned -= L.h_in_cap + L.h_out_cap;
    L.h_in = L.h_out = nullptr;
    L.h_in_cap = L.h_out_cap = 0;
  }
  if (give.empty()) return;
  lk.unlock();
  for (void* p : give)
    if (p) (void)hipHostFree(p);
  lk.lock();
}

static void dispatcher_main(Coalescer* C, int role) {
  (void)hipSetDevice(C->device);
  RoleState& R = C->role[role];
  std::unique_lock<std::mutex> lk(C->mu);
  for (;;) {
    while (!C->stop && !(R.open >= 0 && C->lanes[R.open].reports > 0)) {
      if (R.cv.wait_for(lk, std::chrono::milliseconds(kIdleFreeMs)) == std::cv_status::timeout)
        maybe_release_idle(C, lk);
    }
    if (C->stop) return;
    Lane& L = C->lanes[R.open];
    const auto deadline = L.opened + std::chrono::microseconds(cur_window_us(C, role));
    // Close when full; otherwise once the arrivals have gone quiet, the callers of completed launches are back
    // and fewer than kMaxRunning launches of the role run (or this one is already big enough to fill the device
    // with its own phases); at the latest at the window's end.
    for (;;) {
      if (C->stop || L.full || L.reports >= L.cap_reports || L.reqs.size() >= MAX_JOBS_PER_LAUNCH) break;
      const auto now = clk::now();
      if (now >= deadline) break;
      if (L.reqs.size() < C->min_jobs) {  // a test holds the gather for its jobs
        R.cv.wait_until(lk, deadline);
        continue;
      }
      if (merge_groups() && R.nrunning > 0 && L.reports + R.run_reports <= C->flat_reports) {
        R.cv.wait_until(lk, deadline);
        continue;
      }
      // every caller of the completed launches is back: nobody else is expected, close without a quiet period
      if (L.all_back && R.nrunning < max_running()) break;
      const auto quiet_at = L.last_arrival + std::chrono::microseconds(kQuietUs);
      const bool back = R.expect == 0 || now >= R.expect_until;
      // nothing of this role on the device and no caller of a completed launch still to come: waiting buys nothing
      if (R.nrunning == 0 && R.expect == 0) break;
      if (now >= quiet_at && ((back && R.nrunning < max_running()) || L.reports >= C->max_reports / 4)) break;
      auto until = deadline;
      if (now < quiet_at && quiet_at < until) until = quiet_at;
      if (!back && R.expect_until < until) until = R.expect_until;
      R.cv.wait_until(lk, until);
    }
    if (C->stop) return;
    L.state = SEALED;  // no more reservations; new callers open the next lane
    R.open = -1;
    C->cv_lane.notify_all();
    const auto t_sealed = clk::now();
    R.cv.wait(lk, [&] { return L.copying == 0; });
    lk.unlock();
    std::string err;
    L.launched = clk::now();
    const int32_t rc = launch_lane(C, L, err);
    const auto t_queued = clk::now();
    lk.lock();
    using us = std::chrono::duration<double, std::micro>;
    C->t_gather += us(t_sealed - L.opened).count();
    C->t_copy += us(L.launched - t_sealed).count();
    C->t_enqueue += us(t_queued - L.launched).count();
    C->launches++;
    C->jobs += L.reqs.size();
    C->reports += L.reports;
    R.launches++;
    R.jobs += L.reqs.size();
    if (L.reports >= R.peak || t_queued - R.peak_at > std::chrono::seconds(1)) {
      R.peak = L.reports;
      R.peak_at = t_queued;
    }
    for (CReq* r : L.reqs) C->enc_jobs += r->enc != nullptr;
    if (rc) {
      finish_lane(C, L, rc, err);
    } else {
      L.state = RUNNING;
      R.nrunning++;
      R.run_reports += L.reports;
      C->running.push_back((int)(&L - C->lanes));
      C->cv_comp.notify_one();
    }
  }
}

// Waits for the running launches (of both roles, which complete in any order) and wakes each one's callers. It
// spins on the lanes' host flags (launch_host_signal), so it makes no runtime call while launches run: a loop of
// hipEventQuery measured ~1 ms stalls of the other threads' HIP calls (the dispatcher's uploads, the callers'
// next batches) behind the runtime's locks. Each running lane's event is still queried every
// kEventCheckUs, to see a launch that failed (its flag never comes).
constexpr uint32_t kEventCheckUs = 2000;
static void completer_main(Coalescer* C) {
  (void)hipSetDevice(C->device);
  std::unique_lock<std::mutex> lk(C->mu);
  std::vector<clk::time_point> checked(kMaxLanes);
  for (;;) {
    C->cv_comp.wait(lk, [&] { return C->stop || !C->running.empty(); });
    if (C->running.empty() && C->stop) return;
    std::vector<std::pair<int, uint32_t>> snap;
    for (int k : C->running) snap.push_back({k, C->lanes[k].seq});
    lk.unlock();
    std::vector<std::pair<int, hipError_t>> done;
    const auto t_poll = clk::now();
    for (int spin = 0; done.empty(); spin++) {
      for (auto& ks : snap)
        if (__atomic_load_n(C->hflag + kFlagStride * ks.first, __ATOMIC_ACQUIRE) == ks.second)
          done.push_back({ks.first, hipSuccess});
      if (!done.empty()) break;
      const auto now = clk::now();
      for (auto& ks : snap) {
        if (now - checked[ks.first] < std::chrono::microseconds(kEventCheckUs)) continue;
        checked[ks.first] = now;
        const hipError_t st = hipEventQuery(C->lanes[ks.first].ev_done);
        if (st != hipSuccess && st != hipErrorNotReady) done.push_back({ks.first, st});
        (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
      }
      if (!done.empty()) break;
      // a launch queued meanwhile joins the poll
      if (now - t_poll > std::chrono::microseconds(200)) break;
      if (spin & 63) {
        __builtin_ia32_pause();
      } else {
        std::this_thread::yield();
      }
    }
    const auto now = clk::now();
    lk.lock();
    for (auto& d : done) {
      Lane& L = C->lanes[d.first];
      C->running.erase(std::find(C->running.begin(), C->running.end(), d.first));
      RoleState& R = C->role[L.role];
      const double us = std::chrono::duration<double, std::micro>(now - L.launched).count();
      R.ewma_us = R.ewma_us > 0 ? 0.8 * R.ewma_us + 0.2 * us : us;
      C->t_device += us;
      R.nrunning--;
      R.run_reports -= L.reports;
      R.expect += (uint32_t)L.reqs.size();  // this launch's callers will be back with their next jobs
      R.expect_until = now + std::chrono::microseconds(rejoin_us(R));
      if (R.open >= 0) C->lanes[R.open].all_back = false;  // the gathering lane now expects these callers too
      R.cv.notify_one();  // a gathering lane may close now
      finish_lane(C, L, d.second == hipSuccess ? JX_OK : JX_E_HIP,
                  d.second == hipSuccess ? std::string() : std::string("coalesced launch: ") + hipGetErrorString(d.second));
    }
  }
}

Coalescer* coalescer_for(jx_engine* e) {
  std::lock_guard<std::mutex> gl(g_mu);
  const std::string key = coal_key(e);
  auto it = g_coal.find(key);
  if (it != g_coal.end()) {
    it->second->refs++;
    return it->second;
  }
  Coalescer* C = new Coalescer();
  C->key = key;
  C->device = e->device;
  // the base: the engine state the lanes copy, with its own copy of the constant tables (e may go away
  // before the coalescer) and no stream of its own (the device has few hardware queues: the lanes get them)
  jx_engine* base = new jx_engine();
  base->cfg = e->cfg;
  base->device = e->device;
  base->is_pipe = true;
  base->arena = e->arena;
  base->default_chunk = e->default_chunk;
  base->auto_chunk = e->auto_chunk;
  base->round_reports = e->round_reports;
  base->lis_stride = e->lis_stride;
  const Cfg& cc = e->cfg;
  const size_t cbytes = (size_t)(cc.P + cc.gpoly_len + jx::NMISC + cc.P1 + cc.gpoly1_len) * sizeof(uint4);
  uint4* consts = nullptr;
  if (hipMalloc((void**)&consts, cbytes) != hipSuccess ||
      hipMemcpyAsync(consts, e->d_consts, cbytes, hipMemcpyDeviceToDevice, e->stream) != hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess) {
    if (consts) (void)hipFree(consts);
    delete base;
    delete C;
    return nullptr;
  }
  base->d_consts = consts;
  base->is_pipe = true;  // destroy: the consts are freed by the coalescer
  C->base = base;
  // a launch: up to half the fused path's launch size (its staging comes from the arena per launch)
  C->max_reports = e->auto_chunk / 2 < 4096 ? 4096 : e->auto_chunk / 2;
  // the word-per-lane K1's range (one report-wave per SIMD, 1,024 SumVec reports): a launch of all of them takes
  // the time of a launch of a few (prep_core)
  C->flat_reports = e->round_reports / 128;
  C->last_job = clk::now();
  if (hipHostMalloc((void**)&C->hflag, kMaxLanes * kFlagStride * sizeof(uint32_t),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&C->dflag, C->hflag, 0) != hipSuccess) {
    if (C->hflag) (void)hipHostFree(C->hflag);
    jx_engine_destroy(base);
    (void)hipFree(consts);
    delete C;
    return nullptr;
  }
  memset(C->hflag, 0, kMaxLanes * kFlagStride * sizeof(uint32_t));
  if (const char* env = getenv("JX_COAL_LANES")) {
    const int x = atoi(env);
    if (x >= 2 && x <= (int)kMaxLanes) C->nlanes = (uint32_t)x;
  }
  for (uint32_t k = 0; k < C->nlanes; k++) {
    Lane& L = C->lanes[k];
    L.q = new_child(base);
    // the completer polls this event (a blocking-sync event's interrupt wake-up measured ms late)
    if (!L.q || hipEventCreateWithFlags(&L.ev_done, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&L.up, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&L.ev_up0, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&L.ev_up, hipEventDisableTiming) != hipSuccess) {
      for (uint32_t j = 0; j <= k; j++) {
        Lane& J = C->lanes[j];
        if (J.q) jx_engine_destroy(J.q);
        if (J.ev_done) (void)hipEventDestroy(J.ev_done);
        if (J.up) (void)hipStreamDestroy(J.up);
        if (J.ev_up0) (void)hipEventDestroy(J.ev_up0);
        if (J.ev_up) (void)hipEventDestroy(J.ev_up);
      }
      jx_engine_destroy(base);
      (void)hipFree(consts);
      (void)hipHostFree(C->hflag);
      delete C;
      return nullptr;
    }
  }
  C->refs = 1;
  for (int r = 0; r < NROLES; r++) C->role[r].dispatcher = std::thread(dispatcher_main, C, r);
  C->completer = std::thread(completer_main, C);
  g_coal.emplace(key, C);
  return C;
}

void coalescer_release(jx_engine* e) {
  Coalescer* C = e->coal;
  e->coal = nullptr;
  e->coalesce = false;
  if (!C) return;
  {
    std::lock_guard<std::mutex> gl(g_mu);
    if (--C->refs > 0) return;
    g_coal.erase(C->key);
  }
  {
    std::lock_guard<std::mutex> lk(C->mu);
    C->stop = true;
  }
  for (RoleState& R : C->role) R.cv.notify_all();
  C->cv_comp.notify_all();
  C->cv_lane.notify_all();
  for (RoleState& R : C->role) R.dispatcher.join();
  C->completer.join();
  uint4* consts = C->base->d_consts;
  for (Lane& L : C->lanes) {
    if (L.q) jx_engine_destroy(L.q);
    if (L.ev_done) (void)hipEventDestroy(L.ev_done);
    if (L.up) {
      (void)hipStreamSynchronize(L.up);
      (void)hipStreamDestroy(L.up);
    }
    if (L.ev_up0) (void)hipEventDestroy(L.ev_up0);
    if (L.ev_up) (void)hipEventDestroy(L.ev_up);
    lane_free_pinned(C, L);
  }
  jx_engine_destroy(C->base);
  if (consts) (void)hipFree(consts);
  if (C->hflag) (void)hipHostFree(C->hflag);
  delete C;
}

void coalescer_set_window(jx_engine* e, uint32_t window_us) {
  if (!e->coal) return;
  std::lock_guard<std::mutex> lk(e->coal->mu);
  e->coal->window_us = window_us;
}

void coalescer_set_min_jobs(jx_engine* e, uint32_t jobs) {
  if (!e->coal) return;
  std::lock_guard<std::mutex> lk(e->coal->mu);
  e->coal->min_jobs = jobs;
}

bool coalescer_accepts(const jx_engine* e, bool leader, uint64_t n, bool encrypted, uint64_t ct_bytes) {
  Coalescer* C = e->coal;
  if (!C || n == 0) return false;
  const int role = leader ? LEADER : HELPER;  // no lock: the lane limits are fixed, enc_seen only turns on
  return n <= lane_max_reports(C, role, role == HELPER && (C->enc_seen || encrypted)) &&
         (!encrypted || ct_bytes <= kPinnedBudget / 2);
}

void coalescer_stats(const jx_engine* e, uint64_t out[16]) {
  for (int i = 0; i < 16; i++) out[i] = 0;
  Coalescer* C = e->coal;
  if (!C) return;
  std::lock_guard<std::mutex> lk(C->mu);
  out[0] = C->launches;
  out[1] = C->jobs;
  out[2] = C->reports;
  out[3] = cur_window_us(C, HELPER);
  out[4] = (uint64_t)C->role[HELPER].ewma_us;
  out[5] = (uint64_t)C->t_gather;
  out[6] = (uint64_t)C->t_copy;
  out[7] = (uint64_t)C->t_enqueue;
  out[8] = (uint64_t)C->t_device;
  out[9] = C->pinned;
  out[10] = C->role[HELPER].launches;
  out[11] = C->role[HELPER].jobs;
  out[12] = C->role[LEADER].launches;
  out[13] = C->role[LEADER].jobs;
  out[14] = C->enc_jobs;
}

// Whether r joins the gathering lane L (with C->mu held); if so, its rows (and ciphertext bytes and keypairs)
// are reserved.
static bool try_join(Coalescer* C, Lane& L, CReq* r) {
  (void)C;
  if (L.reports + r->n > L.cap_reports || L.reqs.size() >= MAX_JOBS_PER_LAUNCH) return false;
  if (r->enc) {
    if (!L.enc || L.ct_bytes + r->ct_bytes > L.ct_cap) return false;
    size_t add = 0;
    for (uint32_t k = 0; k < r->enc->nkeys; k++)
      if (std::find(L.keys.begin(), L.keys.end(), r->enc->keypairs[k]) == L.keys.end()) add++;
    if (L.keys.size() + add > ENC_MAX_KEYS) return false;
    for (uint32_t k = 0; k < r->enc->nkeys; k++) {
      const jx_hpke* h = r->enc->keypairs[k];
      auto it = std::find(L.keys.begin(), L.keys.end(), h);
      if (it == L.keys.end()) {
        hpke_key_row(h, reinterpret_cast<HpkeKeyRow*>(L.h_in + L.o_keys) + L.keys.size());
        L.keys.push_back(h);
        it = L.keys.end() - 1;
      }
      r->key_map[k] = (uint8_t)(it - L.keys.begin());
    }
    r->ct_first = L.ct_bytes;
    L.ct_bytes += r->ct_bytes;
    L.has_enc = true;
  }
  r->first = L.reports;
  L.reports += r->n;
  L.last_arrival = clk::now();
  return true;
}

// Reserve rows for r in its role's gathering lane (opening one if none gathers). With C->mu held.
static Lane* reserve(Coalescer* C, std::unique_lock<std::mutex>& lk, CReq* r, int32_t* rc) {
  RoleState& R = C->role[r->role];
  if (r->enc) C->enc_seen = true;  // helper lanes opened from now on carry the encrypted-input regions
  C->last_job = clk::now();
  for (;;) {
    if (C->stop) {
      *rc = JX_E_STATE;
      return nullptr;
    }
    if (R.open >= 0) {
      Lane& L = C->lanes[R.open];
      if (try_join(C, L, r)) {
        if (R.expect && --R.expect == 0) L.all_back = true;
        L.reqs.push_back(r);
        L.copying++;
        R.cv.notify_one();
        return &L;
      }
      L.full = true;  // close it now; wait for the next lane
      R.cv.notify_one();
    } else {
      for (uint32_t k = 0; k < C->nlanes; k++) {
        Lane& L = C->lanes[k];
        if (L.state != FREE) continue;
        int32_t lr = lane_layout(C, L, r->role, r->n, r->ct_bytes);
        if (lr) {  // JX_E_INVALID: larger than a lane (the caller runs it directly); JX_E_NOMEM
          *rc = lr;
          return nullptr;
        }
        L.state = GATHER;
        L.full = false;
        L.all_back = false;
        L.has_enc = false;
        L.reports = 0;
        L.ct_bytes = 0;
        L.keys.clear();
        L.reqs.clear();
        L.copying = 0;
        L.opened = L.last_arrival = clk::now();
        R.open = (int)k;
        break;
      }
      if (R.open >= 0) continue;
    }
    C->cv_lane.wait(lk);
  }
}

// Lay out one job's EncRows (its ciphertexts at ct_base + their offset within the job).
void fill_enc_rows(const EncJob& j, uint64_t n, EncRow* rows, uint64_t ct_base, const uint8_t* key_map) {
  const uint64_t c0 = j.payload_offsets[0];
  for (uint64_t i = 0; i < n; i++) {
    EncRow& w = rows[i];
    memset(&w, 0, sizeof w);
    memcpy(w.enc, j.encs + 32 * i, 32);
    memcpy(w.task_id, j.task_id, 32);
    const uint64_t t = j.times[i];
    for (int b = 0; b < 8; b++) w.time_be[b] = (uint8_t)(t >> (56 - 8 * b));
    w.ct_off = ct_base + (j.payload_offsets[i] - c0);
    w.ct_len = (uint32_t)(j.payload_offsets[i + 1] - j.payload_offsets[i]);
    const uint8_t k0 = j.key_index[2 * i], k1 = j.key_index[2 * i + 1];
    w.flags = ENC_ROW_ENCRYPTED | ((j.flags & JX_ENC_REQUIRE_TASKPROV) ? ENC_ROW_REQUIRE_TASKPROV : 0);
    if (k0 == JX_KEY_MALFORMED) w.flags |= ENC_ROW_MALFORMED;
    w.key0 = k0 < j.nkeys ? key_map[k0] : (k0 == JX_KEY_MALFORMED ? (uint8_t)0 : (uint8_t)JX_KEY_NONE);
    w.key1 = k1 < j.nkeys ? key_map[k1] : (uint8_t)JX_KEY_NONE;
  }
}

// The coalesced prepare of one job (both roles).
static int32_t coalesced(jx_engine* e, bool leader, uint64_t n, const uint8_t* nonces, const uint8_t* ps,
                         const uint8_t* his, const uint8_t* lps, const uint8_t* lis, uint8_t* out_msgs,
                         uint8_t* out_verdicts, uint8_t* out_prep_shares, uint64_t* out_batch_id,
                         const EncJob* enc = nullptr, uint8_t* out_status = nullptr) {
  Coalescer* C = e->coal;
  const Cfg& c = e->cfg;
  CReq r;
  r.e = e;
  r.role = leader ? LEADER : HELPER;
  r.n = n;
  r.enc = enc;
  r.ct_bytes = enc ? enc->ct_bytes(n) : 0;
  r.out_msgs = out_msgs;
  r.out_verdicts = out_verdicts;
  r.out_prep_shares = out_prep_shares;
  r.out_status = out_status;
  Batch* Bp = nullptr;
  {
    std::lock_guard<FairMutex> el(e->mu);
    HIPCHK(e, hipSetDevice(e->device));
    Batch* B = nullptr;
    int32_t rc = batch_new(e, n, leader, &r.id, &B);
    if (rc) return rc;
    B->pending = true;
    Bp = B;
    r.dst = JobSlice{0, n, B->outs, B->verdicts, B->msgs, B->nonces};
    r.batch_ev = B->wait_ev ? B->wait_ev : B->slab.ev;
  }
  auto drop = [&](int32_t rc) {
    std::lock_guard<FairMutex> el(e->mu);
    auto it = e->batches.find(r.id);
    if (it != e->batches.end()) batch_free(e, it);
    return rc;
  };
  std::unique_lock<std::mutex> lk(C->mu);
  int32_t rc = JX_OK;
  Lane* L = reserve(C, lk, &r, &rc);
  if (!L) {
    lk.unlock();
    fail(e, rc, rc == JX_E_INVALID ? "coalesced prepare: the job does not fit a coalesced launch"
                                   : "coalesced prepare: no lane (pinned host memory or shutdown)");
    return drop(rc);
  }
  r.dst.first = r.first;
  lk.unlock();
  // copy this job's rows into the lane's pinned input (in parallel with the other callers)
  const uint64_t f = r.first;
  memcpy(L->h_in + L->o_non + f * 16, nonces, n * 16);
  if (c.ps_bytes) memcpy(L->h_in + L->o_ps + f * c.ps_bytes, ps, n * c.ps_bytes);
  if (leader) {
    memcpy(L->h_in + L->o_lis + f * c.lis_bytes, lis, n * c.lis_bytes);
  } else {
    if (!enc) memcpy(L->h_in + L->o_his + f * c.his_bytes, his, n * c.his_bytes);
    memcpy(L->h_in + L->o_lps + f * c.lps_bytes, lps, n * c.lps_bytes);
    EncRow* rows = L->enc ? reinterpret_cast<EncRow*>(L->h_in + L->o_enc) + f : nullptr;
    if (enc) {
      fill_enc_rows(*enc, n, rows, r.ct_first, r.key_map);
      memcpy(L->h_in + L->o_ct + r.ct_first, enc->payloads + enc->payload_offsets[0], r.ct_bytes);
    } else if (rows) {
      memset(rows, 0, n * sizeof(EncRow));  // plain reports: the open kernel leaves their rows alone
    }
  }
  {
    const uint32_t vb = vk_row_bytes(c);
    uint8_t row[64];
    vk_row(c, row);
    uint8_t* dst = L->h_in + L->o_vk + f * vb;
    for (uint64_t i = 0; i < n; i++) memcpy(dst + i * vb, row, vb);
  }
  lk.lock();
  if (--L->copying == 0) C->role[r.role].cv.notify_one();
  lk.unlock();
  {
    std::unique_lock<std::mutex> rl(r.m);
    r.cv.wait(rl, [&] { return r.done; });
  }
  if (r.rc == JX_OK) {
    memcpy(out_verdicts, L->h_out + L->r_ver + f, n);
    if (out_msgs && c.jr_len) memcpy(out_msgs, L->h_out + L->r_msg + f * c.seed, n * c.seed);
    if (leader) memcpy(out_prep_shares, L->h_out + L->r_lps + f * c.lps_bytes, n * c.lps_bytes);
    if (out_status) {
      if (L->has_enc)
        memcpy(out_status, L->h_out + L->r_st + f, n);
      else
        memset(out_status, 0, n);
    }
  }
  if (L->unconsumed.fetch_sub(1) == 1) {
    lk.lock();
    L->state = FREE;
    C->cv_lane.notify_all();
    lk.unlock();
  }
  if (r.rc) {
    fail(e, r.rc, r.err);
    return drop(r.rc);
  }
  // the batch is ready: no engine mutex (the callers of a completed launch return together; each lock hand-off
  // was a wake-up on the way back to the next job). Its map node is stable and no other call touches a pending
  // batch.
  __atomic_store_n(&Bp->pending, false, __ATOMIC_RELEASE);
  e->last_batch.store(r.id);
  if (out_batch_id) *out_batch_id = r.id;
  return JX_OK;
}

int32_t coalesced_helper_prep(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* his,
                              const uint8_t* lps, uint8_t* out_msgs, uint8_t* out_verdicts, uint64_t* out_batch_id,
                              const EncJob* enc, uint8_t* out_status) {
  return coalesced(e, false, n, nonces, ps, his, lps, nullptr, out_msgs, out_verdicts, nullptr, out_batch_id, enc,
                   out_status);
}

int32_t coalesced_leader_init(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* lis,
                              uint8_t* out_prep_shares, uint8_t* out_verdicts, uint64_t* out_batch_id) {
  return coalesced(e, true, n, nonces, ps, nullptr, nullptr, lis, nullptr, out_verdicts, out_prep_shares, out_batch_id);
}

}  // namespace jxi
