// jx_coalesce.cpp — coalesced prepares: the aggregation jobs of every task of one Prio3 instance on one GPU
// share launches.
//
// Janus prepares one aggregation job per request: the helper's handle_aggregate_init_generic runs one
// AggregationJobInitializeReq (aggregator/src/aggregator.rs:1712-2013), jobs hold 10-100 reports
// (docs/samples/basic_config/aggregation_job_creator.yaml:23-26), and many are in flight (tokio workers
// on the helper; the leader steps max_concurrent_job_workers jobs at once, binary_utils/job_driver.rs:116).
// A GPU launch of 100 SumVec reports is bound by one report's chain of ~800 dependent Keccak
// permutations (~4 ms) and leaves the device nearly empty; one engine call at a time serialises those
// latencies. Here the jobs that arrive together become ONE launch:
//
//   caller thread (jx_helper_prep_batch / jx_leader_prep_init_batch with coalescing on):
//     1. creates its job's resident batch on its own engine (its task: verify key, batches, aggregations);
//     2. reserves rows in the lane that is gathering, and copies its inputs and its verify key into the
//        lane's pinned host rows itself (callers copy in parallel);
//     3. waits (without its engine's mutex) until the launch is done, then copies its verdicts / prep
//        messages / prep shares out of the lane's pinned result rows and returns its batch handle.
//   dispatcher thread: closes the gathering lane when it holds a full launch, once no job has joined for
//     a quiet period while no other launch runs (a running launch's callers join this one when it
//     returns), or when the gathering window has passed; then, on the lane's stream: one upload per input
//     region, K1 -> K1' -> K3
//     over all jobs (each report with its own task's verify key, Bufs::vkeys), one scatter kernel that
//     copies every job's slice into its batch, one download of the results, an event.
//   completer thread: waits for launches in order and wakes their callers.
// Up to kLanes launches are in flight, so jobs that arrive while one runs start on the next lane at once.
#include <chrono>
#include <cstring>
#include <deque>
#include <thread>

#include "jx_engine_internal.h"

using namespace jx;

namespace jxi {

namespace {

using clk = std::chrono::steady_clock;
constexpr uint32_t kLanes = 3;
constexpr size_t kPinnedBudget = 512ull << 20;  // pinned input rows per lane

struct CReq {
  jx_engine* e = nullptr;
  bool leader = false;
  uint64_t n = 0, first = 0, id = 0;
  JobSlice dst{};
  hipEvent_t batch_ev = nullptr;  // the batch slab's last user (the lane waits on it)
  uint8_t* out_msgs = nullptr;
  uint8_t* out_verdicts = nullptr;
  uint8_t* out_prep_shares = nullptr;
  int32_t rc = 0;
  std::string err;
  bool done = false;
  std::condition_variable cv;  // this job's caller waits here for its launch (no herd of wake-ups)
};

enum LaneState { FREE, GATHER, SEALED, RUNNING, DONE };

struct Lane {
  jx_engine* q = nullptr;  // child engine: own stream, staging from the arena per launch
  uint8_t* h_in = nullptr;
  size_t h_in_cap = 0;
  uint8_t* h_out = nullptr;
  size_t h_out_cap = 0;
  hipEvent_t ev_done = nullptr;
  LaneState state = FREE;
  bool leader = false;
  bool full = false;  // a caller could not fit: close now
  uint64_t reports = 0, cap_reports = 0;
  uint32_t copying = 0, unconsumed = 0;
  std::vector<CReq*> reqs;
  clk::time_point opened, launched, last_arrival;
  // region offsets in h_in (rows of cap_reports)
  size_t o_non = 0, o_ps = 0, o_his = 0, o_lps = 0, o_lis = 0, o_vk = 0, o_jobs = 0;
  // region offsets in h_out
  size_t r_ver = 0, r_msg = 0, r_lps = 0;
};

}  // namespace

struct Coalescer {
  std::string key;
  int device = 0;
  jx_engine* base = nullptr;  // owns the constant tables the lanes share
  std::mutex mu;
  // one condition variable per kind of waiter: the dispatcher (a job joined, copies done), the completer (a
  // launch queued), callers waiting for a lane to gather in; callers waiting for their launch use their own
  std::condition_variable cv_disp, cv_comp, cv_lane;
  Lane lanes[kLanes];
  int open = -1;
  std::deque<int> running;
  std::thread dispatcher, completer;
  bool stop = false;
  uint32_t refs = 0;
  uint32_t window_us = 0;         // 0: automatic
  uint32_t min_jobs = 0;          // debug option 7 (tests): a gather waits (up to its window) for this many jobs
  double ewma_us = 0;             // launch latency
  uint32_t nrunning = 0;          // launches queued on the device and not yet done
  uint32_t expect = 0;            // jobs of completed launches not yet back (closed-loop callers return)
  clk::time_point expect_until;   // ... expected until then
  uint64_t max_reports = 0;       // reports per launch
  uint64_t launches = 0, jobs = 0, reports = 0;
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

// A gathering lane closes at once while no launch runs and no caller of a completed launch is still due back
// (a lone caller, or the device idle: nothing to wait for). Otherwise it closes once no job has joined it for
// kQuietUs, fewer than kMaxRunning launches are on the device, and the callers of the launches that completed
// meanwhile have come back (up to kRejoinUs after the
// completion: copying their results, accumulating, preparing their next job), so closed-loop callers share a
// launch per round trip instead of splitting into fragments; open-loop arrivals wait at most the window. A
// launch's device time is nearly flat in its size below a K1 round (the per-report sponge chain), so two
// launches in flight, each carrying every job that is back, is the measured optimum (DESIGN.md §5.4:
// profiles/r05_coalesce_policy_ab.jsonl, 1 / 2 / 3 running; profiles/r05_coalesce_rejoin_retune.jsonl, the
// rejoin window re-measured on the final kernels and host path: 1 ms, against 1.5 / 2 / 3 ms).
constexpr uint32_t kQuietUs = 100;
constexpr uint32_t kRejoinUs = 1000;
constexpr uint32_t kMaxRunning = 2;

// The longest a gathering lane waits for more jobs (automatic: 1.5x the recent launch latency, 0.1-20 ms). It
// matters while another launch runs: the jobs that launch returns join this one instead of starting a
// fragment of their own (closed-loop callers then share one launch per round trip).
static uint32_t cur_window_us(const Coalescer* C) {
  if (C->window_us) return C->window_us;
  if (C->ewma_us <= 0) return 2000;
  double w = 1.5 * C->ewma_us;
  return (uint32_t)(w < 100 ? 100 : (w > 20000 ? 20000 : w));
}

// bytes of one report's pinned input row / result row
static size_t in_row(const Cfg& c, bool leader) {
  size_t b = 16 + c.ps_bytes + vk_row_bytes(c);
  b += leader ? c.lis_bytes : (size_t)c.his_bytes + c.lps_bytes;
  return b;
}

// Lay the lane's pinned rows out for a gather of `leader` kind (capacity cap reports); grows the buffers.
static int32_t lane_layout(Coalescer* C, Lane& L, bool leader) {
  const Cfg& c = C->base->cfg;
  const uint64_t want = C->max_reports;
  uint64_t cap = kPinnedBudget / in_row(c, leader);
  if (cap > want) cap = want;
  cap = cap < 64 ? 64 : cap / 64 * 64;
  size_t off = 0;
  auto take = [&](size_t& o, size_t bytes) {
    o = off;
    off += align256(bytes ? bytes : 1);
  };
  take(L.o_non, cap * 16);
  take(L.o_ps, cap * c.ps_bytes);
  if (leader) {
    take(L.o_lis, cap * c.lis_bytes);
    L.o_his = L.o_lps = 0;
  } else {
    take(L.o_his, cap * c.his_bytes);
    take(L.o_lps, cap * c.lps_bytes);
    L.o_lis = 0;
  }
  take(L.o_vk, cap * vk_row_bytes(c));
  take(L.o_jobs, (size_t)MAX_JOBS_PER_LAUNCH * sizeof(JobSlice));
  const size_t in_bytes = off;
  off = 0;
  take(L.r_ver, cap);
  take(L.r_msg, cap * c.seed);
  if (leader) take(L.r_lps, cap * c.lps_bytes);
  const size_t out_bytes = off;
  if (L.h_in_cap < in_bytes) {
    if (L.h_in) (void)hipHostFree(L.h_in);
    L.h_in = nullptr;
    L.h_in_cap = 0;
    if (hipHostMalloc((void**)&L.h_in, in_bytes, hipHostMallocDefault) != hipSuccess) return JX_E_NOMEM;
    L.h_in_cap = in_bytes;
  }
  if (L.h_out_cap < out_bytes) {
    if (L.h_out) (void)hipHostFree(L.h_out);
    L.h_out = nullptr;
    L.h_out_cap = 0;
    if (hipHostMalloc((void**)&L.h_out, out_bytes, hipHostMallocDefault) != hipSuccess) return JX_E_NOMEM;
    L.h_out_cap = out_bytes;
  }
  L.cap_reports = cap;
  L.leader = leader;
  return JX_OK;
}

// Queue one closed gather on its lane's stream. Returns JX_OK or an error for every job of the launch.
static int32_t launch_lane(Coalescer* C, Lane& L, std::string& err) {
  jx_engine* q = L.q;
  const Cfg& c = q->cfg;
  const uint64_t m = L.reports;
  const bool leader = L.leader;
  auto bad = [&](hipError_t st, const char* what) {
    err = std::string("coalesced launch: ") + what + ": " + hipGetErrorString(st);
    return st == hipErrorOutOfMemory ? JX_E_NOMEM : JX_E_HIP;
  };
  if (hipSetDevice(C->device) != hipSuccess) return JX_E_HIP;
  const bool inpl = leader && (c.algo == ALGO_SUM || c.algo == ALGO_SUMVEC || c.algo == ALGO_FIXEDPOINT_L2);
  uint32_t fl = SG_IN | SG_PREP | SG_RES | SG_VK | SG_JOBS;
  fl |= leader ? SG_LEAD : SG_HIN;
  if (!inpl) fl |= SG_MEAS;
  // staging for a power of two of reports (>= 1,024): launches of varying size reuse the lane's slab
  uint64_t cap = 1024;
  while (cap < m) cap <<= 1;
  Stage st;
  int32_t rc = stage_acquire(q, cap, fl, st);
  if (rc) {
    err = thread_error();
    return rc;
  }
  // every job's batch slab: after its previous user
  for (CReq* r : L.reqs) {
    hipError_t s = hipStreamWaitEvent(q->stream, r->batch_ev, 0);
    if (s != hipSuccess) return bad(s, "hipStreamWaitEvent");
  }
  auto up = [&](void* dst, size_t off, size_t bytes) -> hipError_t {
    return bytes ? hipMemcpyAsync(dst, L.h_in + off, bytes, hipMemcpyHostToDevice, q->stream) : hipSuccess;
  };
  hipError_t s = up(q->d_nonces, L.o_non, m * 16);
  if (s == hipSuccess && c.ps_bytes) s = up(q->d_ps, L.o_ps, m * c.ps_bytes);
  if (s == hipSuccess && !leader) s = up(q->d_his, L.o_his, m * c.his_bytes);
  if (s == hipSuccess && !leader) s = up(q->d_lps, L.o_lps, m * c.lps_bytes);
  if (s == hipSuccess && leader) {
    if (q->lis_stride == c.lis_bytes)
      s = up(q->d_lis, L.o_lis, m * c.lis_bytes);
    else
      s = hipMemcpy2DAsync(q->d_lis, q->lis_stride, L.h_in + L.o_lis, c.lis_bytes, c.lis_bytes, m,
                           hipMemcpyHostToDevice, q->stream);
  }
  if (s == hipSuccess) s = up(q->d_vkeys, L.o_vk, m * vk_row_bytes(c));
  JobSlice* h_jobs = reinterpret_cast<JobSlice*>(L.h_in + L.o_jobs);
  uint64_t max_job = 0;
  for (size_t k = 0; k < L.reqs.size(); k++) {
    h_jobs[k] = L.reqs[k]->dst;
    if (L.reqs[k]->n > max_job) max_job = L.reqs[k]->n;
  }
  if (s == hipSuccess) s = up(q->d_jobs, L.o_jobs, L.reqs.size() * sizeof(JobSlice));
  if (s != hipSuccess) return bad(s, "upload");
  rc = prep_core(q, m, q->d_nonces, q->d_ps, q->d_his, q->d_lps, q->d_verdicts, q->d_msgs, staging_outs(q),
                 leader ? q->d_lis : nullptr, leader ? q->d_lps_out : nullptr, leader ? q->lis_stride : 0, q->d_vkeys);
  if (rc) {
    err = thread_error();
    return rc;
  }
  s = launch_scatter_jobs(c, q->d_jobs, (uint32_t)L.reqs.size(), max_job,
                          staging_outs(q), q->d_verdicts, q->d_msgs, q->d_nonces, q->stream);
  if (s != hipSuccess) return bad(s, "scatter");
  s = hipMemcpyAsync(L.h_out + L.r_ver, q->d_verdicts, m, hipMemcpyDeviceToHost, q->stream);
  if (s == hipSuccess && c.jr_len)
    s = hipMemcpyAsync(L.h_out + L.r_msg, q->d_msgs, m * c.seed, hipMemcpyDeviceToHost, q->stream);
  if (s == hipSuccess && leader)
    s = hipMemcpyAsync(L.h_out + L.r_lps, q->d_lps_out, m * c.lps_bytes, hipMemcpyDeviceToHost, q->stream);
  if (s == hipSuccess) s = hipEventRecord(L.ev_done, q->stream);
  if (s != hipSuccess) return bad(s, "download");
  return JX_OK;  // st hands the staging back stream-ordered
}

static void finish_lane(Coalescer* C, Lane& L, int32_t rc, const std::string& err) {
  for (CReq* r : L.reqs) {
    r->rc = rc;
    if (rc) r->err = err;
    r->done = true;
    r->cv.notify_one();
  }
  L.unconsumed = (uint32_t)L.reqs.size();
  L.state = DONE;
  if (L.unconsumed == 0) {
    L.state = FREE;
    C->cv_lane.notify_all();
  }
}

static void dispatcher_main(Coalescer* C) {
  (void)hipSetDevice(C->device);
  std::unique_lock<std::mutex> lk(C->mu);
  for (;;) {
    C->cv_disp.wait(lk, [&] { return C->stop || (C->open >= 0 && C->lanes[C->open].reports > 0); });
    if (C->stop) return;
    Lane& L = C->lanes[C->open];
    const auto deadline = L.opened + std::chrono::microseconds(cur_window_us(C));
    // Close when full; otherwise once the arrivals have gone quiet, the callers of completed launches are back
    // and fewer than kMaxRunning launches run (or this one is already big enough to fill the device with its own
    // phases); at the latest at the window's end.
    for (;;) {
      if (C->stop || L.full || L.reports >= L.cap_reports || L.reqs.size() >= MAX_JOBS_PER_LAUNCH) break;
      const auto now = clk::now();
      if (now >= deadline) break;
      if (L.reqs.size() < C->min_jobs) {  // a test holds the gather for its jobs
        C->cv_disp.wait_until(lk, deadline);
        continue;
      }
      const auto quiet_at = L.last_arrival + std::chrono::microseconds(kQuietUs);
      const bool back = C->expect == 0 || now >= C->expect_until;
      // nothing on the device and no caller of a completed launch still to come: waiting buys nothing
      if (C->nrunning == 0 && C->expect == 0) break;
      if (now >= quiet_at && ((back && C->nrunning < kMaxRunning) || L.reports >= C->max_reports / 4)) break;
      auto until = deadline;
      if (now < quiet_at && quiet_at < until) until = quiet_at;
      if (!back && C->expect_until < until) until = C->expect_until;
      C->cv_disp.wait_until(lk, until);
    }
    if (C->stop) return;
    L.state = SEALED;  // no more reservations; new callers open the next lane
    C->open = -1;
    C->cv_lane.notify_all();
    const auto t_sealed = clk::now();
    C->cv_disp.wait(lk, [&] { return L.copying == 0; });
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
    if (rc) {
      finish_lane(C, L, rc, err);
    } else {
      L.state = RUNNING;
      C->nrunning++;
      C->running.push_back((int)(&L - C->lanes));
      C->cv_comp.notify_one();
    }
  }
}

static void completer_main(Coalescer* C) {
  (void)hipSetDevice(C->device);
  std::unique_lock<std::mutex> lk(C->mu);
  for (;;) {
    C->cv_comp.wait(lk, [&] { return C->stop || !C->running.empty(); });
    if (C->running.empty() && C->stop) return;
    Lane& L = C->lanes[C->running.front()];
    C->running.pop_front();
    lk.unlock();
    const hipError_t s = hipEventSynchronize(L.ev_done);
    const double us = std::chrono::duration<double, std::micro>(clk::now() - L.launched).count();
    lk.lock();
    C->ewma_us = C->ewma_us > 0 ? 0.8 * C->ewma_us + 0.2 * us : us;
    C->t_device += us;
    C->nrunning--;
    C->expect += (uint32_t)L.reqs.size();  // this launch's callers will be back with their next jobs
    C->expect_until = clk::now() + std::chrono::microseconds(kRejoinUs);
    C->cv_disp.notify_one();  // a gathering lane may close now
    finish_lane(C, L, s == hipSuccess ? JX_OK : JX_E_HIP,
                s == hipSuccess ? std::string() : std::string("coalesced launch: ") + hipGetErrorString(s));
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
  for (uint32_t k = 0; k < kLanes; k++) {
    Lane& L = C->lanes[k];
    L.q = new_child(base);
    // the completer spin-waits on this event (a blocking-sync event's interrupt wake-up measured ms late)
    if (!L.q || hipEventCreateWithFlags(&L.ev_done, hipEventDisableTiming) != hipSuccess) {
      for (uint32_t j = 0; j <= k; j++) {
        if (C->lanes[j].q) jx_engine_destroy(C->lanes[j].q);
        if (C->lanes[j].ev_done) (void)hipEventDestroy(C->lanes[j].ev_done);
      }
      jx_engine_destroy(base);
      (void)hipFree(consts);
      delete C;
      return nullptr;
    }
  }
  C->refs = 1;
  C->dispatcher = std::thread(dispatcher_main, C);
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
  C->cv_disp.notify_all();
  C->cv_comp.notify_all();
  C->cv_lane.notify_all();
  C->dispatcher.join();
  C->completer.join();
  uint4* consts = C->base->d_consts;
  for (Lane& L : C->lanes) {
    if (L.q) jx_engine_destroy(L.q);
    if (L.ev_done) (void)hipEventDestroy(L.ev_done);
    if (L.h_in) (void)hipHostFree(L.h_in);
    if (L.h_out) (void)hipHostFree(L.h_out);
  }
  jx_engine_destroy(C->base);
  if (consts) (void)hipFree(consts);
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

void coalescer_stats(const jx_engine* e, uint64_t out[12]) {
  for (int i = 0; i < 12; i++) out[i] = 0;
  Coalescer* C = e->coal;
  if (!C) return;
  std::lock_guard<std::mutex> lk(C->mu);
  out[0] = C->launches;
  out[1] = C->jobs;
  out[2] = C->reports;
  out[3] = cur_window_us(C);
  out[4] = (uint64_t)C->ewma_us;
  out[5] = (uint64_t)C->t_gather;
  out[6] = (uint64_t)C->t_copy;
  out[7] = (uint64_t)C->t_enqueue;
  out[8] = (uint64_t)C->t_device;
}

// Reserve rows for r in the gathering lane (opening one if none gathers). With C->mu held.
static Lane* reserve(Coalescer* C, std::unique_lock<std::mutex>& lk, CReq* r, int32_t* rc) {
  for (;;) {
    if (C->stop) {
      *rc = JX_E_STATE;
      return nullptr;
    }
    if (C->open >= 0) {
      Lane& L = C->lanes[C->open];
      if (L.leader == r->leader && L.reports + r->n <= L.cap_reports && L.reqs.size() < MAX_JOBS_PER_LAUNCH) {
        r->first = L.reports;
        L.reports += r->n;
        L.last_arrival = clk::now();
        if (C->expect) C->expect--;
        L.reqs.push_back(r);
        L.copying++;
        C->cv_disp.notify_one();
        return &L;
      }
      L.full = true;  // close it now; wait for the next lane
      C->cv_disp.notify_one();
    } else {
      for (uint32_t k = 0; k < kLanes; k++) {
        Lane& L = C->lanes[k];
        if (L.state != FREE) continue;
        int32_t lr = lane_layout(C, L, r->leader);
        if (lr) {
          *rc = lr;
          return nullptr;
        }
        if (r->n > L.cap_reports) {  // larger than a launch (callers route such jobs directly)
          *rc = JX_E_INVALID;
          return nullptr;
        }
        L.state = GATHER;
        L.full = false;
        L.reports = 0;
        L.reqs.clear();
        L.copying = 0;
        L.opened = L.last_arrival = clk::now();
        C->open = (int)k;
        break;
      }
      if (C->open >= 0) continue;
    }
    C->cv_lane.wait(lk);
  }
}

// The coalesced prepare of one job (both roles).
static int32_t coalesced(jx_engine* e, bool leader, uint64_t n, const uint8_t* nonces, const uint8_t* ps,
                         const uint8_t* his, const uint8_t* lps, const uint8_t* lis, uint8_t* out_msgs,
                         uint8_t* out_verdicts, uint8_t* out_prep_shares, uint64_t* out_batch_id) {
  Coalescer* C = e->coal;
  const Cfg& c = e->cfg;
  CReq r;
  r.e = e;
  r.leader = leader;
  r.n = n;
  r.out_msgs = out_msgs;
  r.out_verdicts = out_verdicts;
  r.out_prep_shares = out_prep_shares;
  {
    std::lock_guard<FairMutex> el(e->mu);
    HIPCHK(e, hipSetDevice(e->device));
    Batch* B = nullptr;
    int32_t rc = batch_new(e, n, leader, &r.id, &B);
    if (rc) return rc;
    B->pending = true;
    r.dst = JobSlice{0, n, B->outs, B->verdicts, B->msgs, B->nonces};
    r.batch_ev = B->slab.ev;
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
    fail(e, rc, "coalesced prepare: the job does not fit a coalesced launch");
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
    memcpy(L->h_in + L->o_his + f * c.his_bytes, his, n * c.his_bytes);
    memcpy(L->h_in + L->o_lps + f * c.lps_bytes, lps, n * c.lps_bytes);
  }
  {
    const uint32_t vb = vk_row_bytes(c);
    uint8_t row[64];
    vk_row(c, row);
    uint8_t* dst = L->h_in + L->o_vk + f * vb;
    for (uint64_t i = 0; i < n; i++) memcpy(dst + i * vb, row, vb);
  }
  lk.lock();
  if (--L->copying == 0) C->cv_disp.notify_one();
  r.cv.wait(lk, [&] { return r.done; });
  lk.unlock();
  if (r.rc == JX_OK) {
    memcpy(out_verdicts, L->h_out + L->r_ver + f, n);
    if (out_msgs && c.jr_len) memcpy(out_msgs, L->h_out + L->r_msg + f * c.seed, n * c.seed);
    if (leader) memcpy(out_prep_shares, L->h_out + L->r_lps + f * c.lps_bytes, n * c.lps_bytes);
  }
  lk.lock();
  if (--L->unconsumed == 0) {
    L->state = FREE;
    C->cv_lane.notify_all();
  }
  lk.unlock();
  if (r.rc) {
    fail(e, r.rc, r.err);
    return drop(r.rc);
  }
  {
    std::lock_guard<FairMutex> el(e->mu);
    auto it = e->batches.find(r.id);
    if (it != e->batches.end()) it->second.pending = false;
    e->last_batch = r.id;
  }
  if (out_batch_id) *out_batch_id = r.id;
  return JX_OK;
}

int32_t coalesced_helper_prep(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* his,
                              const uint8_t* lps, uint8_t* out_msgs, uint8_t* out_verdicts, uint64_t* out_batch_id) {
  return coalesced(e, false, n, nonces, ps, his, lps, nullptr, out_msgs, out_verdicts, nullptr, out_batch_id);
}

int32_t coalesced_leader_init(jx_engine* e, uint64_t n, const uint8_t* nonces, const uint8_t* ps, const uint8_t* lis,
                              uint8_t* out_prep_shares, uint8_t* out_verdicts, uint64_t* out_batch_id) {
  return coalesced(e, true, n, nonces, ps, nullptr, nullptr, lis, nullptr, out_verdicts, out_prep_shares, out_batch_id);
}

}  // namespace jxi
