// jobs_driver.cpp — load generator for tools/bench_jobs.py (--driver cpp): T native threads submit
// aggregation jobs of n reports to ONE engine through the C ABI (jx_helper_prep_batch -> jx_accumulate),
// the way Janus's helper (Rust, tokio worker threads) would call it, with no interpreter in the loop.
//
// Input file (written by bench_jobs.py): header of 8 u64 [K, PS, HIS, LPS, PM, 0, 0, 0], then K x 16
// nonces, K x PS public shares, K x HIS helper input shares, K x LPS leader prep shares, K expected
// verdicts, K x PM expected prep messages. Output file: u64 [jobs, reports, bad_jobs, count] + the
// engine's aggregate (OUT x FB) + K x u64 multiplicities of the pool reports prepared, for the caller to
// check the aggregate against the oracle; the JSON line on stdout carries rate and latencies.
//
//   jobs_driver IN OUT algo bits length chunk proofs vk_hex n threads seconds coalesce window_us warmup
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

int main(int argc, char** argv) {
  if (argc < 15) {
    fprintf(stderr, "usage: jobs_driver IN OUT algo bits length chunk proofs vk_hex n threads seconds coalesce window_us warmup\n");
    return 2;
  }
  const char* in_path = argv[1];
  const char* out_path = argv[2];
  jx_prio3_params p{(uint32_t)atoi(argv[3]), (uint32_t)atoi(argv[4]), (uint32_t)atoi(argv[5]), (uint32_t)atoi(argv[6]),
                    (uint32_t)atoi(argv[7])};
  std::vector<uint8_t> vk;
  for (const char* h = argv[8]; h[0] && h[1]; h += 2) {
    char b[3] = {h[0], h[1], 0};
    vk.push_back((uint8_t)strtoul(b, nullptr, 16));
  }
  const uint64_t n = strtoull(argv[9], nullptr, 10);
  const int T = atoi(argv[10]);
  const double seconds = atof(argv[11]);
  const int coalesce = atoi(argv[12]);
  const uint32_t window = (uint32_t)atoi(argv[13]);
  const int warm = atoi(argv[14]);
  const bool no_acc = argc > 15 && atoi(argv[15]) == 0;  // measurement: prepare only, batches released unaccumulated

  FILE* f = fopen(in_path, "rb");
  if (!f) return 3;
  uint64_t hdr[8];
  if (fread(hdr, 8, 8, f) != 8) return 3;
  const uint64_t K = hdr[0], PS = hdr[1], HIS = hdr[2], LPS = hdr[3], PM = hdr[4];
  std::vector<uint8_t> non(K * 16), ps(K * PS), his(K * HIS), lps(K * LPS), wv(K), wm(K * PM);
  auto rd = [&](std::vector<uint8_t>& v) {
    if (!v.empty() && fread(v.data(), 1, v.size(), f) != v.size()) exit(3);
  };
  rd(non), rd(ps), rd(his), rd(lps), rd(wv), rd(wm);
  fclose(f);

  jx_engine* e = nullptr;
  int32_t st = jx_engine_create_ex(&p, vk.data(), (uint32_t)vk.size(), 0, &e);
  if (st) die("create", st, nullptr);
  if (coalesce && (st = jx_engine_coalesce(e, 1, window))) die("coalesce", st, e);

  // per thread: 4 jobs of n reports at distinct pool offsets, contiguous copies
  struct Job {
    std::vector<uint64_t> idx;
    std::vector<uint8_t> non, ps, his, lps;
  };
  std::vector<std::vector<Job>> jobs(T);
  for (int t = 0; t < T; t++)
    for (int j = 0; j < 4; j++) {
      Job jb;
      const uint64_t off = ((uint64_t)(t * 4 + j) * 7919ull * n) % K;
      jb.idx.resize(n);
      jb.non.resize(n * 16), jb.ps.resize(n * PS), jb.his.resize(n * HIS), jb.lps.resize(n * LPS);
      for (uint64_t i = 0; i < n; i++) {
        const uint64_t r = (off + i) % K;
        jb.idx[i] = r;
        memcpy(&jb.non[i * 16], &non[r * 16], 16);
        if (PS) memcpy(&jb.ps[i * PS], &ps[r * PS], PS);
        memcpy(&jb.his[i * HIS], &his[r * HIS], HIS);
        memcpy(&jb.lps[i * LPS], &lps[r * LPS], LPS);
      }
      jobs[t].push_back(std::move(jb));
    }

  auto run = [&](double secs, bool record, std::vector<double>* lat_prep, std::vector<double>* lat_job,
                 std::vector<uint64_t>* mult, uint64_t* njobs, uint64_t* nbad, double* wall) {
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::vector<double>> lp(T), lj(T);
    std::vector<std::vector<uint64_t>> per(T, std::vector<uint64_t>(4, 0));
    std::vector<uint64_t> bad(T, 0);
    std::vector<clk::time_point> ends(T);
    std::vector<std::string> errs(T);
    clk::time_point t0;
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        std::vector<uint8_t> v(n), m(n * (PM ? PM : 1));
        ready++;
        while (!go.load()) std::this_thread::yield();
        const auto stop = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(secs));
        for (uint64_t k = 0; clk::now() < stop; k++) {
          Job& jb = jobs[t][k % 4];
          uint64_t bid = 0;
          const auto a = clk::now();
          int32_t s = jx_helper_prep_batch(e, n, jb.non.data(), PS ? jb.ps.data() : nullptr, jb.his.data(), jb.lps.data(),
                                           PM ? m.data() : nullptr, v.data(), nullptr, &bid);
          const auto b = clk::now();
          if (s == 0) s = no_acc ? jx_batch_release(e, bid) : jx_accumulate(e, bid, n, nullptr, nullptr);
          const auto c = clk::now();
          if (s) {
            errs[t] = std::string(jx_status_str(s)) + " " + jx_last_error(e);
            break;
          }
          if (record) {
            lp[t].push_back(std::chrono::duration<double, std::milli>(b - a).count());
            lj[t].push_back(std::chrono::duration<double, std::milli>(c - a).count());
            per[t][k % 4]++;
            bool ok = true;
            for (uint64_t i = 0; i < n && ok; i++) {
              const uint64_t r = jb.idx[i];
              ok = v[i] == wv[r] && (wv[r] != 0 || !PM || memcmp(&m[i * PM], &wm[r * PM], PM) == 0);
            }
            bad[t] += ok ? 0 : 1;
          }
        }
        ends[t] = clk::now();
      });
    while (ready.load() < T) std::this_thread::yield();
    t0 = clk::now();
    go = true;
    for (auto& x : th) x.join();
    for (int t = 0; t < T; t++)
      if (!errs[t].empty()) {
        fprintf(stderr, "jobs_driver: thread %d: %s\n", t, errs[t].c_str());
        exit(4);
      }
    *wall = std::chrono::duration<double>(*std::max_element(ends.begin(), ends.end()) - t0).count();
    if (!record) return;
    for (int t = 0; t < T; t++) {
      lat_prep->insert(lat_prep->end(), lp[t].begin(), lp[t].end());
      lat_job->insert(lat_job->end(), lj[t].begin(), lj[t].end());
      for (int j = 0; j < 4; j++) {
        *njobs += per[t][j];
        for (uint64_t r : jobs[t][j].idx) (*mult)[r] += per[t][j];
      }
      *nbad += bad[t];
    }
  };

  std::vector<double> lat_prep, lat_job;
  std::vector<uint64_t> mult(K, 0);
  uint64_t njobs = 0, nbad = 0;
  double wall = 0;
  if (warm) run(0.3, false, nullptr, nullptr, nullptr, nullptr, nullptr, &wall);  // first-touch allocations
  if ((st = jx_aggregate_reset(e))) die("reset", st, e);
  jx_memory_stats m0{}, m1{};
  jx_engine_memory(e, &m0);
  run(seconds, true, &lat_prep, &lat_job, &mult, &njobs, &nbad, &wall);
  jx_engine_memory(e, &m1);
  uint32_t out_len = 0, fb = 0;
  jx_engine_sizes(e, nullptr, nullptr, nullptr, nullptr, &out_len, &fb);
  std::vector<uint8_t> agg((size_t)out_len * fb);
  uint64_t count = 0;
  if ((st = jx_aggregate_read(e, 0, agg.data(), &count))) die("read", st, e);
  jx_engine_destroy(e);

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
  printf("{\"jobs\": %llu, \"reports\": %llu, \"wall_s\": %.4f, \"reports_per_s\": %.1f, \"prep_ms_p50\": %.3f, "
         "\"prep_ms_p99\": %.3f, \"job_ms_p50\": %.3f, \"job_ms_p99\": %.3f, \"bad_jobs\": %llu, \"launches\": %llu, "
         "\"jobs_per_launch\": %.2f, \"gather_ms\": %.3f, \"copy_ms\": %.3f, \"enqueue_ms\": %.3f, \"device_ms\": %.3f, "
         "\"window_us\": %llu, \"arena_cross_stream_waits\": %llu, \"arena_allocs\": %llu, \"arena_peak_gb\": %.2f}\n",
         (unsigned long long)njobs, (unsigned long long)(njobs * n), wall, njobs * n / wall, pct(lat_prep, 0.5),
         pct(lat_prep, 0.99), pct(lat_job, 0.5), pct(lat_job, 0.99), (unsigned long long)nbad, (unsigned long long)la,
         la ? (double)(m1.coalesced_jobs - m0.coalesced_jobs) / la : 0.0,
         la ? (m1.coalesce_gather_us - m0.coalesce_gather_us) / 1e3 / la : 0.0,
         la ? (m1.coalesce_copy_us - m0.coalesce_copy_us) / 1e3 / la : 0.0,
         la ? (m1.coalesce_enqueue_us - m0.coalesce_enqueue_us) / 1e3 / la : 0.0,
         la ? (m1.coalesce_device_us - m0.coalesce_device_us) / 1e3 / la : 0.0, (unsigned long long)m1.coalesce_window_us,
         (unsigned long long)(m1.arena_cross_stream_waits - m0.arena_cross_stream_waits),
         (unsigned long long)(m1.arena_allocs - m0.arena_allocs), m1.arena_peak / 1e9);
  return 0;
}
