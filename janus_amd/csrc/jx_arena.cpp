// jx_arena.cpp — the per-device memory arena every engine on a GPU draws from.
//
// Janus runs one VdafOps per task (aggregator/src/aggregator.rs:1156-1183), so an aggregator with many
// tasks of one Prio3 instance holds many engines on one GPU. Per-engine staging sized for full-device
// launches (tens of GB for SumVec 8x1000/88) would exhaust the 288 GB of HBM after a handful of tasks.
// Instead, staging is checked out of this arena per call and handed back stream-ordered when the call
// has queued its last use: the slab's event is recorded on the user's stream, and the next user's stream
// waits on that event before touching it. The host never blocks on a reuse. Resident batches (a job's
// output shares between its prepare and its accumulation) come from the same arena, so the arena's
// budget bounds everything the engines hold.
//
// Budget: JX_ARENA_GB, or 90 % of the device's memory at first use. A request that does not fit first
// frees idle slabs (those whose last user has finished first; the waits and hipFree run outside the arena's
// lock, so one trim never stalls another engine's check-out), then (for per-call staging, by a caller that
// holds no slab) waits for another caller's staging to come back; otherwise JX_E_NOMEM.
#include <cstdio>
#include <cstdlib>
#include <ctime>

#include "jx_engine_internal.h"

namespace jxi {

static std::mutex g_mu;
static std::map<int, Arena*> g_arenas;  // process lifetime

Arena* arena_for(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_arenas.find(device);
  if (it != g_arenas.end()) return it->second;
  Arena* A = new Arena();
  A->device = device;
  size_t fr = 0, tot = 0;
  (void)hipSetDevice(device);
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) tot = 0;
  A->budget = tot ? (uint64_t)(tot * 0.9) : (64ull << 30);
  if (const char* env = getenv("JX_ARENA_GB")) {
    const uint64_t gb = strtoull(env, nullptr, 10);
    if (gb >= 1) A->budget = gb << 30;
  }
  g_arenas.emplace(device, A);
  return A;
}

// JX_ARENA_TRIM_LOG=<path> (measurement): one line per freed slab, "monotonic <free start> <free end> boottime
// <free start> <free end> <bytes> <wait ns>": the hipFree's interval in both clocks (to line it up with a kernel
// trace, tools/stream_gaps.py --trims) and how long the trimming thread first waited for the slab's last user.
static uint64_t now_ns(clockid_t id) {
  timespec t;
  clock_gettime(id, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}
static void log_free(uint64_t m0, uint64_t b0, uint64_t wait_ns, size_t bytes) {
  static const char* path = getenv("JX_ARENA_TRIM_LOG");
  if (!path) return;
  const uint64_t m1 = now_ns(CLOCK_MONOTONIC), b1 = now_ns(CLOCK_BOOTTIME);
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (FILE* f = fopen(path, "a")) {
    fprintf(f, "monotonic %llu %llu boottime %llu %llu %zu %llu\n", (unsigned long long)m0, (unsigned long long)m1,
            (unsigned long long)b0, (unsigned long long)b1, bytes, (unsigned long long)wait_ns);
    fclose(f);
  }
}

// Waits for the slab's last user and frees it. Never with A->mu held: the wait can be a 100 ms K1 launch, and
// every engine's check-outs on the device would stall behind it.
static void slab_destroy(Slab& s) {
  const uint64_t w0 = now_ns(CLOCK_MONOTONIC);
  if (s.ev) {
    (void)hipEventSynchronize(s.ev);  // its last user's work
    (void)hipEventDestroy(s.ev);
  }
  const uint64_t m0 = now_ns(CLOCK_MONOTONIC), b0 = now_ns(CLOCK_BOOTTIME);
  (void)hipFree(s.p);
  log_free(m0, b0, m0 - w0, s.bytes);
  s = Slab{};
}

// With A->mu held: take idle slabs off the free list for destruction until `need` more bytes fit the budget
// (need = ~0: all of them), those whose last user has finished first, largest first. Their bytes stay counted
// in `allocated` (and in `freeing`) until free_slabs has returned them.
static void take_idle(Arena* A, size_t need, std::vector<Slab>& dead) {
  auto over = [&] { return need == ~(size_t)0 || A->allocated - A->freeing + need > A->budget; };
  for (int pass = 0; pass < 2 && over(); pass++) {
    for (auto it = A->free.end(); it != A->free.begin() && over();) {
      --it;
      const bool idle = !it->second.last || hipEventQuery(it->second.ev) == hipSuccess;
      if (pass == 0 && !idle) continue;
      dead.push_back(it->second);
      A->freeing += it->second.bytes;
      it = A->free.erase(it);
    }
    (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
  }
}

// Destroy slabs taken by take_idle: drops the lock for the waits and frees, then accounts them.
static void free_slabs(Arena* A, std::vector<Slab>& dead, std::unique_lock<std::mutex>& lk) {
  if (dead.empty()) return;
  lk.unlock();
  size_t bytes = 0;
  for (Slab& s : dead) {
    bytes += s.bytes;
    slab_destroy(s);
  }
  lk.lock();
  A->allocated -= bytes;
  A->freeing -= bytes;
  A->frees += dead.size();
  dead.clear();
  A->cv.notify_all();
}

static void account_out(Arena* A, const Slab& s) {
  A->in_use += s.bytes;
  if (s.staging) A->in_use_staging += s.bytes;
  if (A->in_use > A->peak) A->peak = A->in_use;
}

// Staging sizes round up to size classes (4 per octave, <= 19 % slack) so that launches of varying report
// counts find idle slabs to reuse instead of allocating a new size each time.
static size_t size_class(size_t b) {
  if (b <= (1u << 20)) return align256(b);
  int e = 63 - __builtin_clzll((unsigned long long)b);  // 2^e <= b < 2^(e+1)
  const size_t step = (size_t)1 << (e - 2);
  return (b + step - 1) / step * step;
}

hipError_t arena_get(Arena* A, size_t bytes, hipStream_t s, bool staging, bool may_wait, Slab& out) {
  bytes = staging ? size_class(bytes ? bytes : 1) : align256(bytes ? bytes : 1);
  std::unique_lock<std::mutex> lk(A->mu);
  for (;;) {
    // Idle slabs at most 2x (+1 MiB) larger (a small request does not pin a big slab). Prefer, best fit
    // first, one whose last user is this stream or has finished: taking a slab another stream is still
    // using would make this stream wait for that work (two concurrent launches would run one after the
    // other). Such a slab is taken only when the budget leaves no room for a new one.
    auto lo = A->free.lower_bound(bytes);
    auto hi = A->free.upper_bound(2 * bytes + (1u << 20));
    auto pick = A->free.end(), busy = A->free.end();
    for (auto it = lo; it != hi; ++it) {
      if (it->second.last == s || !it->second.last || hipEventQuery(it->second.ev) == hipSuccess) {
        pick = it;
        break;
      }
      if (busy == A->free.end()) busy = it;
    }
    const bool room = A->allocated + bytes <= A->budget;
    // With no room for a new slab, any larger idle slab before freeing one: a trim stalls its caller for the
    // slab's last user and the hipFree (72 + 49 ms for a 640 MB slab; 7 -> 1 trims in the two-engine trace,
    // profiles/r06_arena_stream_gaps.json, where the other engine kept launching through the free).
    if (pick == A->free.end() && !room) {
      for (auto it = hi; it != A->free.end(); ++it) {
        if (it->second.last == s || !it->second.last || hipEventQuery(it->second.ev) == hipSuccess) {
          pick = it;
          break;
        }
        if (busy == A->free.end()) busy = it;
      }
    }
    (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
    if (pick == A->free.end() && busy != A->free.end() && !room) pick = busy;
    if (pick != A->free.end()) {
      out = pick->second;
      A->free.erase(pick);
      out.staging = staging;
      account_out(A, out);
      A->reuses++;
      if (out.last && out.last != s) A->cross_waits += pick == busy;
      // after the slab's last user (a never-recorded event: no wait); on its own stream, stream order does it
      return out.last == s ? hipSuccess : hipStreamWaitEvent(s, out.ev, 0);
    }
    if (A->allocated + bytes > A->budget && !A->free.empty()) {  // make room from idle slabs, outside the lock
      std::vector<Slab> dead;
      take_idle(A, bytes, dead);
      if (!dead.empty()) {
        free_slabs(A, dead, lk);
        continue;
      }
    }
    if (A->allocated + bytes <= A->budget) {
      // the budget is reserved under the lock and the device allocation made outside it: a large hipMalloc
      // takes milliseconds, and every other engine's check-outs (batches, staging) must not wait for it
      A->allocated += bytes;
      lk.unlock();
      void* p = nullptr;
      hipError_t st = hipMalloc(&p, bytes);
      hipEvent_t ev = nullptr;
      if (st == hipSuccess) {
        st = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (st != hipSuccess) (void)hipFree(p);
      }
      lk.lock();
      if (st == hipSuccess) {
        out = Slab{p, bytes, ev, nullptr, staging};
        A->allocs++;
        account_out(A, out);
        return hipSuccess;
      }
      A->allocated -= bytes;
      if (st != hipErrorOutOfMemory) return st;
      (void)hipGetLastError();
      // the device (other users, torch) is fuller than the budget: give back the idle slabs and retry once
      if (!A->free.empty()) {
        std::vector<Slab> dead;
        take_idle(A, ~(size_t)0, dead);
        free_slabs(A, dead, lk);
        continue;
      }
    }
    // slabs being freed by another caller come back to the budget shortly
    if (A->freeing) {
      A->cv.wait(lk);
      continue;
    }
    // what is checked out holds the memory: staging comes back when its call has queued its work
    if (!may_wait || A->in_use_staging == 0) return hipErrorOutOfMemory;
    A->waits++;
    A->cv.wait(lk);
  }
}

void arena_put(Arena* A, Slab& slab, hipStream_t s) {
  if (!slab.p) return;
  (void)hipEventRecord(slab.ev, s);
  slab.last = s;
  {
    std::lock_guard<std::mutex> lk(A->mu);
    A->in_use -= slab.bytes;
    if (slab.staging) A->in_use_staging -= slab.bytes;
    A->free.emplace(slab.bytes, slab);
  }
  A->cv.notify_all();
  slab = Slab{};
}

void arena_trim(Arena* A) {
  std::unique_lock<std::mutex> lk(A->mu);
  std::vector<Slab> dead;
  take_idle(A, ~(size_t)0, dead);
  free_slabs(A, dead, lk);
}

void arena_engine_add(Arena* A) {
  std::lock_guard<std::mutex> lk(A->mu);
  A->engines++;
}

void arena_engine_remove(Arena* A) {
  std::unique_lock<std::mutex> lk(A->mu);
  if (A->engines) A->engines--;
  if (A->engines == 0) {  // nothing left to reuse the idle slabs: give the memory back to the device
    std::vector<Slab> dead;
    take_idle(A, ~(size_t)0, dead);
    free_slabs(A, dead, lk);
  }
}

hipError_t arena_big_record(Arena* A, const void* owner, hipStream_t s) {
  std::lock_guard<std::mutex> lk(A->mu);
  hipEvent_t& ev = A->big[owner];
  if (!ev) {
    const hipError_t st = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (st != hipSuccess) {
      A->big.erase(owner);
      return st;
    }
  }
  return hipEventRecord(ev, s);
}

bool arena_big_busy(Arena* A, const void* owner) {
  std::lock_guard<std::mutex> lk(A->mu);
  bool busy = false;
  for (auto& kv : A->big)
    if (kv.first != owner && hipEventQuery(kv.second) == hipErrorNotReady) busy = true;
  (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
  return busy;
}

void arena_big_forget(Arena* A, const void* owner) {
  std::lock_guard<std::mutex> lk(A->mu);
  auto it = A->big.find(owner);
  if (it == A->big.end()) return;
  (void)hipEventDestroy(it->second);
  A->big.erase(it);
}

}  // namespace jxi
