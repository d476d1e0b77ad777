// jx_kernels.h — kernel argument structs and launchers shared by jx_kernels.hip and
// jx_engine.cpp.  See DESIGN.md for the HBM layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jx {

enum Algo : uint32_t {
  ALGO_COUNT = 0,
  ALGO_SUM = 1,
  ALGO_SUMVEC = 2,
  ALGO_HISTOGRAM = 3,
  // Prio3SumVecField64MultiproofHmacSha256Aes128 (core/src/vdaf.rs:173-199): Field64, num_proofs
  // >= 2, XofHmacSha256Aes128 with 32-byte seeds (kernels: jx_mp64.hip)
  ALGO_SUMVEC_F64_MULTIPROOF = 4,
  // Prio3FixedPointBoundedL2VecSum{bitsize 16 | 32, length} (core/src/vdaf.rs:86-91, aggregator.rs:916-932):
  // Field128, TurboSHAKE, two gadgets: ParallelSum(Mul, chunk) range check over every input bit and
  // ParallelSum(PolyEval(2^(2n-2) - 2^n y + y^2), chunk1) over the decoded entries (the squared norm)
  ALGO_FIXEDPOINT_L2 = 5,
};
constexpr uint32_t MP_MAX_PROOFS = 8;  // num_proofs supported by the multiproof kernels

// per-report flag bits written by the XOF stage, consumed by the FLP stage
enum : uint32_t {
  FLAG_INIT_FAIL = 1u,  // query randomness t is a P-th root of unity -> prepare_init_failure
  FLAG_NEXT_FAIL = 2u,  // leader's joint-rand part disagrees with the public share -> prepare_next_failure
  FLAG_SLOW = 4u,       // a rejected XOF sample shifted a stream: the slow kernel redoes this report
  FLAG_DFAIL = 8u,      // a leader verifier element is >= p -> leader_prep_share_decode_failure
  FLAG_INPUT_FAIL = 16u,  // leader: an explicit input-share element is >= p -> prepare_init_failure
};

// Interleaved staging: element e of report r lives at [(r/64)][e][r%64] (16 bytes each),
// so a wave (64 reports, one per lane) touching element e moves one coalesced 1 KiB.
constexpr int IL = 64;

struct Cfg {
  uint32_t algo, bits, length, chunk;
  uint32_t meas_len, out_len, jr_len, proof_len, ver_len, calls, P, logP, gpoly_len;
  uint32_t ps_bytes, his_bytes, lps_bytes;
  uint32_t lis_bytes;    // leader input share: meas || proofs || [k_blind]
  uint32_t ncoef;        // coefficient slots per report
  uint32_t out_is_meas;  // truncate == identity (Histogram): output share aliases the meas staging
  uint32_t ppw, ngroups; // ParallelSum FLP: chunk slots per group, groups per 64-report block
  uint32_t ngt;          // partial-sum groups per block over all gadgets (ngroups [+ ngroups1])
  uint32_t vk[4];
  // constant table offsets (uint4 units) in Bufs::consts
  uint32_t c_omega, c_S, c_misc;
  uint32_t fb;      // field element bytes (8: Field64, 16: Field128)
  uint32_t seed;    // XOF SEED_SIZE (16 TurboSHAKE128, 32 HmacSha256Aes128) = prep message bytes
  uint32_t np;      // num_proofs
  uint32_t dst_id;  // algorithm id in the XOF domain-separation tags
  uint32_t nco;     // multiproof: coefficient slots per proof
  // multiproof: HMAC-SHA256 inner/outer states after the key block, for the 32-byte verify key
  // (query randomness) and the all-zero key (joint-rand seed derivations)
  uint32_t vk_ist[8], vk_ost[8], zero_ist[8], zero_ost[8];
  uint32_t trunc_len;  // measurement elements that truncate into the output share (SumVec/Sum/FixedPoint)
  uint32_t qr_len;     // query randomness elements (= gadgets)
  // FixedPointBoundedL2VecSum: the norm bits and gadget 1 (ParallelSum(PolyEval), arity chunk1)
  uint32_t norm_bits;
  uint32_t chunk1, calls1, P1, logP1, gpoly1_len, ppw1, ngroups1;
  uint32_t proof1_off;  // first element of gadget 1's sub-proof [seeds (chunk1) || gadget poly]
  uint32_t coef1;       // first coefficient slot of gadget 1 (G1_* below)
  uint32_t c_omega1, c_S1;  // constant-table offsets of gadget 1's roots and S1_m
  // ParallelSum(Mul) gadget 0 (SumVec, Histogram, FixedPoint): per-report power tables K1 writes so that
  // the FLP group finish needs no exponentiation: c_rpow + j = L r^(j+1) canonical (j < chunk), c_tpow + g
  // = t^(g * per) R, per = ceil(gpoly_len / ngroups) (the group's first gadget-polynomial coefficient)
  uint32_t c_rpow, c_tpow;
};

// coefficient slots (Montgomery form unless noted) for the ParallelSum / Sum FLP. Prio3Sum: as named;
// ParallelSum (SumVec, Histogram, FixedPoint gadget 0) stores them scaled by L for the group finish:
// COEF_L = L canonical, COEF_C0 = c_0 L R, COEF_HALFSUM = L (1/2) sum c_k canonical (xof_tail)
enum : uint32_t {
  COEF_L = 0,        // L = (t^P - 1)/P
  COEF_C0 = 1,       // c_0 = 1/(t - 1)
  COEF_HALFSUM = 2,  // (1/2) * sum_{k>=1} c_k   [canonical]
  COEF_T = 3,        // t
  COEF_R = 4,        // joint_rand[0]
  COEF_R2 = 5,       // joint_rand[1] (Histogram)
  COEF_K = 6,        // first per-call slot
};
// FixedPoint gadget-1 coefficient slots, relative to Cfg::coef1 (Montgomery form)
enum : uint32_t {
  G1_L = 0,   // (t1^P1 - 1)/P1
  G1_C0 = 1,  // c'_0 = 1/(t1 - 1)
  G1_T = 2,   // t1
  G1_K = 3,   // c'_k, k = 1..calls1
};
// misc constants (uint4 slots at Cfg::c_misc): 0 (1/P)R, 1 1/2, 2 R, 3 (1/2)R; FixedPoint: 4 2^n,
// 5 2^(2n-2) R^-1, 6 2^(n-2) (gadget-1 padding, a share of the encoded 0.0), 7 (1/P1)R; 8 zero (the
// source of the FLP ring's loads for measurement elements past the share and for padded slots)
constexpr uint32_t NMISC = 9;
constexpr uint32_t MISC_ZERO = 8;

struct Bufs {
  uint64_t n;  // reports in this launch
  const uint8_t* nonces;
  const uint8_t* ps;
  const uint8_t* his;
  const uint8_t* lps;
  const uint8_t* lis;   // leader role: explicit leader input shares (n rows of lis_rs bytes)
  uint64_t lis_rs;      // leader role: row stride of lis (>= lis_bytes, a multiple of 16)
  // per-report verify keys (nullable: every report uses Cfg::vk / vk_ist, vk_ost): a coalesced launch
  // prepares the jobs of several tasks (engines) of one Prio3 instance. Row r: the 16-byte key
  // (TurboSHAKE instances) or the HMAC-SHA256 pads ist[8] || ost[8] of the 32-byte key (multiproof).
  const uint8_t* vkeys;
  uint8_t* lps_out;     // leader role: outbound prep shares (n x lps_bytes)
  uint32_t leader;      // 1: run prepare_init for agg_id 0 (leader_initialized)
  uint4* meas;
  // leader, read in place: the FLP kernels read measurement element e of report r at
  // meas_src + r * meas_rs + 16 e (the explicit leader input share) instead of the interleaved
  // staging, which K1 then does not write (meas_rs == 0: the staging)
  const uint8_t* meas_src;
  uint64_t meas_rs;
  uint4* proof;
  uint4* outs;
  uint4* coef;
  uint32_t* flags;
  uint4* part;  // ParallelSum FLP partial sums [blk][group][4][lane] (multiproof: uint2 [blk][proof][group][3][lane])
  uint8_t* verdicts;
  uint8_t* msgs;
  const uint4* consts;
  uint32_t force_slow;  // debug: route every report through the slow XOF kernel
  uint32_t k1_split;    // helper K1 kernel: 3 = lane-split (xof_lanes_kernel), 6 = lane pairs (xof_pairs_kernel,
                        // bits <= 32), 8 = lane pairs with unrolled rounds, 7 = a word per lane (xof_words_kernel,
                        // bits <= 32), otherwise the fused kernel
  uint32_t k1_lds;      // dynamic LDS of the lane-split kernel: caps its workgroups per CU (lanes_lds_bytes)
  uint32_t k1_pairs_lds;  // dynamic LDS of the lane-pair kernel (0: none): one workgroup per CU, so two small
                          // launches in flight (coalesced jobs) take disjoint CUs instead of sharing SIMDs
};

struct AccArgs {
  uint64_t n;
  const uint4* outs;
  uint32_t out_len;
  const uint8_t* verdicts;
  const uint8_t* mask;     // nullable
  const uint32_t* seg;     // nullable
  uint32_t seg_id;
  uint64_t* partials;      // [nchunks][out_len][3]
  uint32_t blocks_per_chunk;
  uint32_t nchunks;
  const uint8_t* nonces;
  uint32_t* checksum;      // [8] (XOR)
  unsigned long long* count;
};

// Segmented accumulation (batch aggregations of several batch identifiers in one pass,
// aggregation_job_writer.rs:608-708): reports are counting-sorted by dense segment index on the
// device, then summed per (segment, run of <= L sorted positions) work item, then per segment.
constexpr uint32_t SEG_MAX = 4096;
constexpr uint32_t SELECT_WGS = 1024;  // grid-stride workgroups of the select / segment-count kernels  // dense segment indices handled per pass (LDS histogram size)
struct SegArgs {
  uint64_t n;
  const uint4* outs;
  uint32_t out_len;
  uint32_t fb;
  const uint8_t* verdicts;
  const uint8_t* mask;     // nullable
  const uint32_t* seg;     // dense segment index per report
  uint32_t s0, ns;         // this pass: dense indices [s0, s0 + ns)
  const uint8_t* nonces;
  uint32_t* cnt;           // [ns] selected reports per segment (zeroed by the host)
  uint32_t* off;           // [ns] first sorted position of each segment
  uint32_t* cursor;        // [ns] scatter cursors
  uint32_t* ioff;          // [ns + 1] first work item of each segment
  uint32_t* perm;          // [n] selected report indices grouped by segment
  uint32_t L;              // sorted positions per work item
  uint4* items;            // [wmax] (segment, p0, p1, 0)
  uint32_t* nitems;        // [2]: work items, selected reports
  uint32_t wmax;
  uint64_t* partials;      // [wmax][out_len][3]
  uint4* const* aggs;                  // [ns] the segments' aggregate shares
  unsigned long long* const* counts;   // [ns]
  uint32_t* const* checksums;          // [ns] [8]
};
hipError_t launch_accumulate_segmented(const Cfg& c, const SegArgs& a, uint32_t grid, hipStream_t s);

// multiproof coefficient slots (canonical Field64), per proof
enum : uint32_t { MCOEF_L = 0, MCOEF_C0 = 1, MCOEF_HALFSUM = 2, MCOEF_T = 3, MCOEF_R = 4, MCOEF_K = 5 };

// launchers (jx_kernels.hip)
hipError_t launch_count(const Cfg& c, const Bufs& b, hipStream_t s);
hipError_t launch_xof(const Cfg& c, const Bufs& b, hipStream_t s);
hipError_t launch_xof_slow(const Cfg& c, const Bufs& b, hipStream_t s);
hipError_t launch_leader_finish(const Cfg& c, const Bufs& b, const uint8_t* prep_msgs, const uint8_t* peer,
                                hipStream_t s);
hipError_t launch_flp(const Cfg& c, const Bufs& b, hipStream_t s);
hipError_t launch_accumulate(const Cfg& c, const AccArgs& a, uint4* agg, hipStream_t s);
// Accumulations of at most ACC_SMALL reports: one kernel, no partials or selection scratch (a.partials unused).
constexpr uint64_t ACC_SMALL = 1024;
hipError_t launch_accumulate_small(const Cfg& c, const AccArgs& a, uint4* agg, hipStream_t s);
// Several small batches into ONE aggregation in one kernel (jx_accumulate calls the engine deferred and
// flushes together): every finished report of every batch is added. The table travels as the kernel argument.
constexpr uint32_t ACC_MULTI_MAX = 64;
struct AccDesc {
  const uint4* outs;
  const uint8_t* verdicts;
  const uint8_t* nonces;
  uint64_t n;
};
struct AccMultiArgs {
  AccDesc d[ACC_MULTI_MAX];
  uint32_t nb;
  uint4* agg;
  unsigned long long* count;
  uint32_t* checksum;
};
hipError_t launch_accumulate_multi(const Cfg& c, const AccMultiArgs& a, hipStream_t s);
// The host sees a launch complete without a runtime call: one lane stores `seq` into a host-coherent pinned flag
// once the stream reaches this point (a system-scope release store, so the stream's earlier downloads are
// visible first). The coalescer's completer polls the flags instead of querying events.
hipError_t launch_host_signal(uint32_t* flag, uint32_t seq, hipStream_t s);
// Strided row copies between HBM and mapped pinned host memory by a kernel on the caller's stream (a coalesced
// launch's uploads and downloads): no copy-engine command, so a lane's transfers never queue behind another
// lane's download that is waiting for that lane's kernels (measured: ~1-2 ms stalls). Region
// k copies `rows` rows of `width` bytes; 16-byte vectors when every address, stride and the width allow.
struct CopyRegion {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t dst_stride, src_stride, rows;
  uint64_t width;
};
constexpr uint32_t COPY_MAX_REGIONS = 12;
struct CopyArgs {
  CopyRegion r[COPY_MAX_REGIONS];
  uint32_t nr;
};
hipError_t launch_copy_regions(const CopyArgs& a, hipStream_t s);
hipError_t launch_combine(const Cfg& c, const uint8_t* parts, uint32_t nparts, uint8_t* out, uint32_t* err,
                          hipStream_t s);
// ns records of contiguous segment state (agg [ns][out_len], count [ns], checksum [ns][8])
hipError_t launch_record_export(const Cfg& c, const uint4* agg, const unsigned long long* count,
                                const uint32_t* checksum, uint8_t* dst, hipStream_t s, uint32_t ns = 1);
hipError_t launch_record_combine(const Cfg& c, const uint8_t* parts, uint32_t nparts, uint8_t* out, uint32_t* err,
                                 hipStream_t s);
hipError_t launch_transpose_out(const Cfg& c, const uint4* outs, uint64_t n, uint8_t* dst, hipStream_t s);
hipError_t launch_agg_encode(const Cfg& c, const uint4* agg, uint8_t* dst, hipStream_t s);
// one job of a coalesced launch: reports [first, first + n) go to the job's batch buffers
struct JobSlice {
  uint64_t first, n;
  uint4* outs;
  uint8_t* verdicts;
  uint8_t* msgs;
  uint8_t* nonces;
};
constexpr uint32_t MAX_JOBS_PER_LAUNCH = 4096;
hipError_t launch_scatter_jobs(const Cfg& c, const JobSlice* d_jobs, uint32_t njobs, uint64_t max_job_reports,
                               const uint4* outs, const uint8_t* verdicts, const uint8_t* msgs, const uint8_t* nonces,
                               hipStream_t s);
// ---- HPKE open inside a helper prepare launch (jx_hpke.hip; jx_helper_prep_encrypted_batch)
// A recipient keypair as the rows kernel reads it: clamped X25519 scalar and public key (LE words) and the
// RFC 9180 key_schedule_context of its application info (0x00 || psk_id_hash || info_hash, 65 bytes).
struct HpkeKeyRow {
  uint32_t sk[8];
  uint32_t pk[8];
  uint8_t ksc[68];
  uint8_t pad[4];
};
static_assert(sizeof(HpkeKeyRow) == 136, "HpkeKeyRow layout");
enum : uint8_t {
  ENC_ROW_ENCRYPTED = 1,         // the report's helper input share is inside `enc` / the ciphertext (else: uploaded)
  ENC_ROW_REQUIRE_TASKPROV = 2,  // the task is provisioned by taskprov (aggregator.rs:1869-1879)
  ENC_ROW_MALFORMED = 4,         // the encapsulated key is not 32 bytes: HpkeDecryptError without an open
};
// One report's encrypted input share: the HpkeCiphertext's encapsulated key and ciphertext (at ct_off of the
// launch's ciphertext bytes), what its InputShareAad needs besides the id and public share rows, and the
// keypairs to try (launch key-table rows; key0 JX_KEY_NONE: the config id is unknown).
struct EncRow {
  uint8_t enc[32];
  uint8_t task_id[32];
  uint8_t time_be[8];  // ReportMetadata.time, big-endian as encoded
  uint64_t ct_off;
  uint32_t ct_len;
  uint8_t key0, key1, flags, pad;
  uint8_t pad2[8];
};
static_assert(sizeof(EncRow) == 96, "EncRow layout");
constexpr uint32_t ENC_MAX_KEYS = 16;  // distinct keypairs in one launch's key table
struct HpkeRowsArgs {
  uint64_t n;
  const EncRow* rows;
  const uint8_t* cts;   // ciphertext bytes of the launch
  uint8_t* pts;         // plaintext scratch (same offsets as cts)
  const HpkeKeyRow* keys;
  uint32_t nkeys;
  const uint8_t* nonces;
  const uint8_t* ps;
  uint32_t ps_bytes;
  uint8_t* his;  // out: the helper input-share rows K1 reads
  uint32_t his_bytes;
  uint8_t* status;  // out: JX_OPEN_* per report
};

// multiproof Field64 SumVec (jx_mp64.hip)
uint64_t k1_round_reports(const Cfg& c, int device, uint32_t k1_split = 0);
// The helper reports [S, b.n) of a launch as Bufs of their own (S a multiple of 64: every staging array is
// interleaved by 64-report blocks), for a K1 launch over part of the reports.
Bufs bufs_tail(const Cfg& c, const Bufs& b, uint64_t S);
uint32_t lanes_lds_bytes(uint32_t wgs_per_cu);
uint64_t mp_k1_round_reports(int device);
hipError_t launch_mp_xof(const Cfg& c, const Bufs& b, hipStream_t s);
hipError_t launch_mp_slow(const Cfg& c, const Bufs& b, hipStream_t s);
hipError_t launch_mp_flp(const Cfg& c, const Bufs& b, hipStream_t s);

}  // namespace jx
