// jobs_driver.cpp — load generator for tools/bench_jobs.py (--driver cpp): T native threads submit
// aggregation jobs of n reports to ONE engine through the C ABI (jx_helper_prep_batch -> jx_accumulate, or
// from the encrypted report shares jx_helper_prep_encrypted_batch -> jx_accumulate), the way Janus's helper
// (Rust, tokio worker threads) would call it, with no interpreter in the loop. Optionally L more threads
// submit leader prepare_init jobs (jx_leader_prep_init_batch) of another task on the same Prio3 instance: an
// aggregator that is leader for some tasks and helper for others (aggregator_core/src/task.rs:598).
//
// Input file (written by bench_jobs.py): header of 8 u64 [K, PS, HIS, LPS, PM, mode, CT, 0], then K x 16
// nonces, K x PS public shares, K x HIS helper input shares, K x LPS leader prep shares, K expected verdicts,
// K x PM expected prep messages; mode 1 (encrypted report shares) adds sk[32], pk[32], task_id[32], K x 8 times,
// K x 32 encapsulated keys, (K + 1) x 8 ciphertext offsets, CT ciphertext bytes, K x 2 key indices (0 or
// JX_KEY_NONE) and K expected open statuses. Leader file: header [K, PS, LIS, LPS, 0, 0, 0, 0], K x 16
// nonces, K x PS public shares, K x LIS leader input shares, K expected verdicts, K x LPS expected prep shares.
// Output file: u64 [jobs, reports, bad_jobs, count] + the engine's aggregate (OUT x FB) + K x u64
// multiplicities of the pool reports prepared, for the caller to check the aggregate against the oracle; the
// JSON line on stdout carries rate and latencies (and the leader side's, with leader threads).
//
//   jobs_driver IN OUT algo bits length chunk proofs vk_hex n threads seconds coalesce window_us warmup
//               [accumulate=1 [leader_in leader_vk_hex leader_threads]]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/jx_prio3.h"

using clk = std::chrono::steady_clock;

static void die(const char* what, int32_t st, const jx_engine* e) {
  fprintf(stderr, "jobs_driver: %s: %s (%d) %s\n", what, jx_status_str(st), st, e ? jx_last_error(e) : "");
  exit(1);
}

static std::vector<uint8_t> hex(const char* h) {
  std::vector<uint8_t> v;
  for (; h[0] && h[1]; h += 2) {
    char b[3] = {h[0], h[1], 0};
    v.push_back((uint8_t)strtoul(b, nullptr, 16));
  }
  return v;
}

struct Reader {
  FILE* f;
  void rd(void* p, size_t n) {
    if (n && fread(p, 1, n, f) != n) exit(3);
  }
  template <class T>
  void rd(std::vector<T>& v) {
    rd(v.data(), v.size() * sizeof(T));
  }
};

int main(int argc, char** argv) {
  if (argc < 15) {
    fprintf(stderr, "usage: jobs_driver IN OUT algo bits length chunk proofs vk_hex n threads seconds coalesce window_us "
                    "warmup [accumulate [leader_in leader_vk_hex leader_threads]]\n");
    return 2;
  }
  const char* in_path = argv[1];
  const char* out_path = argv[2];
  jx_prio3_params p{(uint32_t)atoi(argv[3]), (uint32_t)atoi(argv[4]), (uint32_t)atoi(argv[5]), (uint32_t)atoi(argv[6]),
                    (uint32_t)atoi(argv[7])};
  const std::vector<uint8_t> vk = hex(argv[8]);
  const uint64_t n = strtoull(argv[9], nullptr, 10);
  const int T = atoi(argv[10]);
  const double seconds = atof(argv[11]);
  const int coalesce = atoi(argv[12]);
  const uint32_t window = (uint32_t)atoi(argv[13]);
  const int warm = atoi(argv[14]);
  const bool no_acc = argc > 15 && atoi(argv[15]) == 0;  // measurement: prepare only, batches released unaccumulated
  const char* lead_path = argc > 18 ? argv[16] : nullptr;
  const std::vector<uint8_t> lvk = argc > 18 ? hex(argv[17]) : std::vector<uint8_t>();
  const int TL = argc > 18 ? atoi(argv[18]) : 0;

  FILE* f = fopen(in_path, "rb");
  if (!f) return 3;
  Reader R{f};
  uint64_t hdr[8];
  R.rd(hdr, sizeof hdr);
  const uint64_t K = hdr[0], PS = hdr[1], HIS = hdr[2], LPS = hdr[3], PM = hdr[4];
  const bool encrypted = hdr[5] == 1;
  const uint64_t CT = hdr[6];
  std::vector<uint8_t> non(K * 16), ps(K * PS), his(K * HIS), lps(K * LPS), wv(K), wm(K * PM);
  R.rd(non), R.rd(ps), R.rd(his), R.rd(lps), R.rd(wv), R.rd(wm);
  std::vector<uint8_t> sk(32), pk(32), task(32), encs, cts, kidx, wst;
  std::vector<uint64_t> times, cto;
  if (encrypted) {
    times.resize(K), encs.resize(K * 32), cto.resize(K + 1), cts.resize(CT), kidx.resize(K * 2), wst.resize(K);
    R.rd(sk), R.rd(pk), R.rd(task), R.rd(times), R.rd(encs), R.rd(cto), R.rd(cts), R.rd(kidx), R.rd(wst);
  }
  fclose(f);
  // the leader pool
  uint64_t KL = 0, LIS = 0;
  std::vector<uint8_t> lnon, lps_in, lis, lwv, lwp;
  if (lead_path && TL > 0) {
    FILE* g = fopen(lead_path, "rb");
    if (!g) return 3;
    Reader L{g};
    uint64_t h[8];
    L.rd(h, sizeof h);
    KL = h[0];
    LIS = h[2];
    if (h[1] != PS || h[3] != LPS) return 3;
    lnon.resize(KL * 16), lps_in.resize(KL * PS), lis.resize(KL * LIS), lwv.resize(KL), lwp.resize(KL * LPS);
    L.rd(lnon), L.rd(lps_in), L.rd(lis), L.rd(lwv), L.rd(lwp);
    fclose(g);
  }

  jx_engine* e = nullptr;
  int32_t st = jx_engine_create_ex(&p, vk.data(), (uint32_t)vk.size(), 0, &e);
  if (st) die("create", st, nullptr);
  if (coalesce && (st = jx_engine_coalesce(e, 1, window))) die("coalesce", st, e);
  // measurement: JX_JOBS_DEFER=0 accumulates every job at once (jx_engine_debug option 8) instead of deferred
  if (getenv("JX_JOBS_DEFER") && atoi(getenv("JX_JOBS_DEFER")) == 0 && (st = jx_engine_debug(e, 8, 0)))
    die("debug 8", st, e);
  jx_engine* el = nullptr;
  if (TL > 0) {
    if ((st = jx_engine_create_ex(&p, lvk.data(), (uint32_t)lvk.size(), 0, &el))) die("create leader", st, nullptr);
    if (coalesce && (st = jx_engine_coalesce(el, 1, window))) die("coalesce leader", st, el);
  }
  jx_hpke* hk = nullptr;
  if (encrypted) {
    const char info[] = "dap-09 input share\x01\x03";
    if (jx_hpke_create(sk.data(), pk.data(), (const uint8_t*)info, (uint32_t)(sizeof info - 1), 0, &hk)) {
      fprintf(stderr, "jobs_driver: jx_hpke_create failed\n");
      return 1;
    }
  }

  // per thread: 4 jobs of n reports at distinct pool offsets, contiguous copies
  struct Job {
    std::vector<uint64_t> idx;
    std::vector<uint8_t> non, ps, his, lps, lis, encs, cts, kidx;
    std::vector<uint64_t> times, cto;
  };
  const int TT = T + TL;
  std::vector<std::vector<Job>> jobs(TT);
  for (int t = 0; t < TT; t++) {
    const bool lead = t >= T;
    const uint64_t KK = lead ? KL : K;
    for (int j = 0; j < 4; j++) {
      Job jb;
      const uint64_t off = ((uint64_t)(t * 4 + j) * 7919ull * n) % KK;
      jb.idx.resize(n);
      jb.non.resize(n * 16), jb.ps.resize(n * PS);
      if (lead) {
        jb.lis.resize(n * LIS);
      } else {
        jb.his.resize(n * HIS), jb.lps.resize(n * LPS);
      }
      if (encrypted && !lead) jb.encs.resize(n * 32), jb.kidx.resize(n * 2), jb.times.resize(n), jb.cto.assign(1, 0);
      for (uint64_t i = 0; i < n; i++) {
        const uint64_t r = (off + i) % KK;
        jb.idx[i] = r;
        memcpy(&jb.non[i * 16], lead ? &lnon[r * 16] : &non[r * 16], 16);
        if (PS) memcpy(&jb.ps[i * PS], lead ? &lps_in[r * PS] : &ps[r * PS], PS);
        if (lead) {
          memcpy(&jb.lis[i * LIS], &lis[r * LIS], LIS);
          continue;
        }
        memcpy(&jb.his[i * HIS], &his[r * HIS], HIS);
        memcpy(&jb.lps[i * LPS], &lps[r * LPS], LPS);
        if (encrypted) {
          memcpy(&jb.encs[i * 32], &encs[r * 32], 32);
          memcpy(&jb.kidx[i * 2], &kidx[r * 2], 2);
          jb.times[i] = times[r];
          jb.cts.insert(jb.cts.end(), cts.begin() + cto[r], cts.begin() + cto[r + 1]);
          jb.cto.push_back(jb.cts.size());
        }
      }
      jobs[t].push_back(std::move(jb));
    }
  }

  auto run = [&](double secs, bool record, std::vector<double>* lat_prep, std::vector<double>* lat_job,
                 std::vector<double>* lat_lead, std::vector<uint64_t>* mult, uint64_t* njobs, uint64_t* nbad,
                 uint64_t* nlead, uint64_t* nlead_bad, double* wall) {
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::vector<double>> lp(TT), lj(TT);
    std::vector<std::vector<uint64_t>> per(TT, std::vector<uint64_t>(4, 0));
    std::vector<uint64_t> bad(TT, 0);
    std::vector<clk::time_point> ends(TT);
    std::vector<std::string> errs(TT);
    clk::time_point t0;
    std::vector<std::thread> th;
    for (int t = 0; t < TT; t++)
      th.emplace_back([&, t] {
        const bool lead = t >= T;
        std::vector<uint8_t> v(n), m(n * (PM ? PM : 1)), stt(n), shares(lead ? n * LPS : 0);
        jx_engine* eng = lead ? el : e;
        ready++;
        while (!go.load()) std::this_thread::yield();
        const auto stop = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(secs));
        for (uint64_t k = 0; clk::now() < stop; k++) {
          Job& jb = jobs[t][k % 4];
          uint64_t bid = 0;
          const auto a = clk::now();
          int32_t s;
          if (lead)
            s = jx_leader_prep_init_batch(el, n, jb.non.data(), PS ? jb.ps.data() : nullptr, jb.lis.data(),
                                          shares.data(), v.data(), &bid);
          else if (encrypted)
            s = jx_helper_prep_encrypted_batch(e, n, jb.non.data(), jb.times.data(), PS ? jb.ps.data() : nullptr,
                                               task.data(), &hk, 1, jb.kidx.data(), jb.encs.data(), jb.cts.data(),
                                               jb.cto.data(), 0, jb.lps.data(), PM ? m.data() : nullptr, v.data(),
                                               stt.data(), &bid);
          else
            s = jx_helper_prep_batch(e, n, jb.non.data(), PS ? jb.ps.data() : nullptr, jb.his.data(), jb.lps.data(),
                                     PM ? m.data() : nullptr, v.data(), nullptr, &bid);
          const auto b = clk::now();
          if (s == 0) s = (no_acc || lead) ? jx_batch_release(eng, bid) : jx_accumulate(e, bid, n, nullptr, nullptr);
          const auto c = clk::now();
          if (s) {
            errs[t] = std::string(jx_status_str(s)) + " " + jx_last_error(eng);
            break;
          }
          if (record) {
            lp[t].push_back(std::chrono::duration<double, std::milli>(b - a).count());
            lj[t].push_back(std::chrono::duration<double, std::milli>(c - a).count());
            per[t][k % 4]++;
            bool ok = true;
            for (uint64_t i = 0; i < n && ok; i++) {
              const uint64_t r = jb.idx[i];
              if (lead) {
                ok = v[i] == lwv[r] && (lwv[r] != 0 || memcmp(&shares[i * LPS], &lwp[r * LPS], LPS) == 0);
              } else {
                ok = v[i] == wv[r] && (wv[r] != 0 || !PM || memcmp(&m[i * PM], &wm[r * PM], PM) == 0);
                if (encrypted) ok = ok && stt[i] == wst[r];
              }
            }
            bad[t] += ok ? 0 : 1;
          }
        }
        ends[t] = clk::now();
      });
    while (ready.load() < TT) std::this_thread::yield();
    t0 = clk::now();
    go = true;
    for (auto& x : th) x.join();
    for (int t = 0; t < TT; t++)
      if (!errs[t].empty()) {
        fprintf(stderr, "jobs_driver: thread %d: %s\n", t, errs[t].c_str());
        exit(4);
      }
    *wall = std::chrono::duration<double>(*std::max_element(ends.begin(), ends.end()) - t0).count();
    if (!record) return;
    for (int t = 0; t < TT; t++) {
      const bool lead = t >= T;
      if (lead) {
        lat_lead->insert(lat_lead->end(), lp[t].begin(), lp[t].end());
        for (int j = 0; j < 4; j++) *nlead += per[t][j];
        *nlead_bad += bad[t];
        continue;
      }
      lat_prep->insert(lat_prep->end(), lp[t].begin(), lp[t].end());
      lat_job->insert(lat_job->end(), lj[t].begin(), lj[t].end());
      for (int j = 0; j < 4; j++) {
        *njobs += per[t][j];
        for (uint64_t r : jobs[t][j].idx) (*mult)[r] += per[t][j];
      }
      *nbad += bad[t];
    }
  };

  std::vector<double> lat_prep, lat_job, lat_lead;
  std::vector<uint64_t> mult(K, 0);
  uint64_t njobs = 0, nbad = 0, nlead = 0, nlead_bad = 0;
  double wall = 0;
  if (warm) run(0.3, false, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &wall);
  if ((st = jx_aggregate_reset(e))) die("reset", st, e);
  jx_memory_stats m0{}, m1{};
  jx_engine_memory(e, &m0);
  run(seconds, true, &lat_prep, &lat_job, &lat_lead, &mult, &njobs, &nbad, &nlead, &nlead_bad, &wall);
  jx_engine_memory(e, &m1);
  uint32_t out_len = 0, fb = 0;
  jx_engine_sizes(e, nullptr, nullptr, nullptr, nullptr, &out_len, &fb);
  std::vector<uint8_t> agg((size_t)out_len * fb);
  uint64_t count = 0;
  if ((st = jx_aggregate_read(e, 0, agg.data(), &count))) die("read", st, e);
  jx_engine_destroy(e);
  if (el) jx_engine_destroy(el);
  if (hk) jx_hpke_destroy(hk);

  FILE* o = fopen(out_path, "wb");
  const uint64_t head[4] = {njobs, njobs * n, nbad, count};
  fwrite(head, 8, 4, o);
  fwrite(agg.data(), 1, agg.size(), o);
  fwrite(mult.data(), 8, K, o);
  fclose(o);

  auto pct = [](std::vector<double> v, double q) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
  };
  const uint64_t la = m1.coalesced_launches - m0.coalesced_launches;
  const uint64_t hl = m1.coalesced_helper_launches - m0.coalesced_helper_launches,
                 hj = m1.coalesced_helper_jobs - m0.coalesced_helper_jobs,
                 ll = m1.coalesced_leader_launches - m0.coalesced_leader_launches,
                 lj = m1.coalesced_leader_jobs - m0.coalesced_leader_jobs;
  printf("{\"jobs\": %llu, \"reports\": %llu, \"wall_s\": %.4f, \"reports_per_s\": %.1f, \"prep_ms_p50\": %.3f, "
         "\"prep_ms_p99\": %.3f, \"job_ms_p50\": %.3f, \"job_ms_p99\": %.3f, \"bad_jobs\": %llu, \"launches\": %llu, "
         "\"jobs_per_launch\": %.2f, \"gather_ms\": %.3f, \"copy_ms\": %.3f, \"enqueue_ms\": %.3f, \"device_ms\": %.3f, "
         "\"window_us\": %llu, \"arena_cross_stream_waits\": %llu, \"arena_allocs\": %llu, \"arena_peak_gb\": %.2f, "
         "\"encrypted\": %s, \"helper_jobs_per_launch\": %.2f, \"leader_threads\": %d, \"leader_jobs\": %llu, "
         "\"leader_reports_per_s\": %.1f, \"leader_bad_jobs\": %llu, \"leader_prep_ms_p50\": %.3f, "
         "\"leader_jobs_per_launch\": %.2f, \"pinned_mb\": %.1f}\n",
         (unsigned long long)njobs, (unsigned long long)(njobs * n), wall, njobs * n / wall, pct(lat_prep, 0.5),
         pct(lat_prep, 0.99), pct(lat_job, 0.5), pct(lat_job, 0.99), (unsigned long long)nbad, (unsigned long long)la,
         la ? (double)(m1.coalesced_jobs - m0.coalesced_jobs) / la : 0.0,
         la ? (m1.coalesce_gather_us - m0.coalesce_gather_us) / 1e3 / la : 0.0,
         la ? (m1.coalesce_copy_us - m0.coalesce_copy_us) / 1e3 / la : 0.0,
         la ? (m1.coalesce_enqueue_us - m0.coalesce_enqueue_us) / 1e3 / la : 0.0,
         la ? (m1.coalesce_device_us - m0.coalesce_device_us) / 1e3 / la : 0.0, (unsigned long long)m1.coalesce_window_us,
         (unsigned long long)(m1.arena_cross_stream_waits - m0.arena_cross_stream_waits),
         (unsigned long long)(m1.arena_allocs - m0.arena_allocs), m1.arena_peak / 1e9, encrypted ? "true" : "false",
         hl ? (double)hj / hl : 0.0, TL, (unsigned long long)nlead, nlead * n / wall, (unsigned long long)nlead_bad,
         pct(lat_lead, 0.5), ll ? (double)lj / ll : 0.0, m1.coalesce_pinned_bytes / 1e6);
  return 0;
}
