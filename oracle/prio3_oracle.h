/*
 * prio3_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Prio3 (draft-irtf-cfrg-vdaf-08 as implemented by the
 * `prio` crate v0.16.1, which Janus pins at /root/reference/Cargo.toml:50 and
 * Cargo.lock:3435-3438) for the helper prepare + aggregate hot path that
 * Janus drives from aggregator/src/aggregator.rs:1945-1967.
 *
 * Who may use this: tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg — as the CHECKER, never as the product. The product path
 * (janus_amd + libjanus_prio3.so) never links or calls it.
 *
 * Parity status:
 *   - TurboSHAKE128 / Keccak-p[1600,12]: pinned by the published TurboSHAKE
 *     KATs and by hashlib.shake_128 at 24 rounds (tests/test_oracle_xof.py).
 *   - Prio3 algorithm vs prio 0.16.1: UNPINNED. The reference tree holds no
 *     Prio3 test vectors and prio is not vendored; the
 *     restatement follows the VDAF-08 text from memory, cross-checked against
 *     an independent pure-Python restatement (oracle/pyref.py).
 */
#ifndef JANUS_PRIO3_ORACLE_H
#define JANUS_PRIO3_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Prio3 algorithm ids == taskprov VDAF type codes, messages/src/taskprov.rs:358-363.
 * JO_SUMVEC_F64_MULTIPROOF selects Prio3SumVecField64MultiproofHmacSha256Aes128
 * (core/src/vdaf.rs:173-199: Field64, proofs >= 2, XofHmacSha256Aes128, 32-byte seeds and
 * verify key, DST algorithm id 0xFFFF1003).
 * JO_FIXEDPOINT_L2 selects Prio3FixedPointBoundedL2VecSum{bitsize, length} (core/src/vdaf.rs:
 * 26-33,86-91; aggregator/src/aggregator.rs:916-932): bits = 16 (FixedI16<U15>) or 32
 * (FixedI32<U31>), length = entries, chunk ignored; DST algorithm id 0xFFFF0000. Measurements
 * are the entries' two's-complement bit patterns (FixedI{n}::to_bits as u{n}). */
enum { JO_COUNT = 0, JO_SUM = 1, JO_SUMVEC = 2, JO_HISTOGRAM = 3, JO_SUMVEC_F64_MULTIPROOF = 4,
       JO_FIXEDPOINT_L2 = 5 };

/* Verdicts, mirroring the PingPongError labels of aggregator/src/aggregator/error.rs:379-424 */
enum {
  JO_FINISHED = 0,
  JO_PREPARE_INIT_FAILURE = 1,
  JO_PREP_SHARE_DECODE_FAILURE = 2,
  JO_PREPARE_MESSAGE_FAILURE = 3,
  JO_PREPARE_NEXT_FAILURE = 4,
};

/* Size table. Index meanings (uint32 each):
 *  0 meas_len  1 output_len  2 joint_rand_len  3 proof_len  4 verifier_len
 *  5 public_share_bytes  6 leader_input_share_bytes  7 helper_input_share_bytes
 *  8 prep_share_bytes  9 prep_msg_bytes  10 field_bytes  11 client_rand_bytes
 *  12 gadget_arity  13 gadget_calls  14 P (wire poly length)  15 seed_size
 *  16 verify_key_size  17 gadget chunk_length
 *  18..20 second gadget (FixedPointBoundedL2VecSum's norm gadget): arity, calls, P (0 if none)
 * Indices 12-14 and 17 describe the first gadget.                         */
#define JO_NSIZES 21
int jo_sizes(int algo, int bits, int length, int chunk, int proofs, uint32_t out[JO_NSIZES]);

/* Client: shard one measurement. measurement: Count {0,1}; Sum integer;
 * SumVec `length` integers; Histogram bucket index. rand = client_rand_bytes. */
int jo_shard(int algo, int bits, int length, int chunk, int proofs,
             const uint64_t *measurement, const uint8_t nonce[16], const uint8_t *rand,
             uint8_t *public_share, uint8_t *leader_input_share, uint8_t *helper_input_share);

/* Prio3 prepare_init for one aggregator. Returns 0 or JO_PREPARE_INIT_FAILURE.
 * out_share: output_len*field_bytes; corrected_seed: seed_size bytes (unused w/o joint rand).
 * verify_key: verify_key_size bytes (16, or 32 for JO_SUMVEC_F64_MULTIPROOF). */
int jo_prep_init(int algo, int bits, int length, int chunk, int proofs,
                 const uint8_t *verify_key, int agg_id, const uint8_t nonce[16],
                 const uint8_t *public_share, const uint8_t *input_share,
                 uint8_t *prep_share, uint8_t *out_share, uint8_t *corrected_seed);

/* prepare_shares_to_prepare_message([leader, helper]). Returns 0, JO_PREP_SHARE_DECODE_FAILURE
 * (either share malformed) or JO_PREPARE_MESSAGE_FAILURE (decide false). */
int jo_prep_shares_to_prep(int algo, int bits, int length, int chunk, int proofs,
                           const uint8_t *leader_prep_share, size_t leader_len,
                           const uint8_t *helper_prep_share, size_t helper_len,
                           uint8_t *prep_msg);

/* Ping-pong helper step: helper_initialized(...).evaluate(). Returns the verdict;
 * on JO_FINISHED writes prep_msg (prep_msg_bytes) and out_share. */
int jo_helper_prep(int algo, int bits, int length, int chunk, int proofs,
                   const uint8_t *verify_key, const uint8_t nonce[16],
                   const uint8_t *public_share, const uint8_t *helper_input_share,
                   const uint8_t *leader_prep_share, size_t leader_len,
                   uint8_t *prep_msg, uint8_t *out_share);

/* Batched helper prep + aggregate (report-parallel over nthreads). Inputs are
 * fixed-stride arrays. agg_out (nullable) receives the sum of accepted output
 * shares; count_out (nullable) the accepted count; checksum_out (nullable) the XOR
 * of SHA-256(report id = nonce) over accepted reports. out_shares nullable. */
int jo_helper_prep_batch(int algo, int bits, int length, int chunk, int proofs,
                         const uint8_t *verify_key, uint64_t n, const uint8_t *nonces,
                         const uint8_t *public_shares, const uint8_t *helper_input_shares,
                         const uint8_t *leader_prep_shares, uint8_t *prep_msgs, uint8_t *verdicts,
                         uint8_t *out_shares, uint8_t *agg_out, uint64_t *count_out,
                         uint8_t *checksum_out, int nthreads);

/* Batched client shard + leader prep_init (input generation for tests/bench).
 * measurements: n * (SumVec: length; else 1) uint64; rands: n*client_rand_bytes. */
int jo_client_leader_batch(int algo, int bits, int length, int chunk, int proofs,
                           const uint8_t *verify_key, uint64_t n, const uint64_t *measurements,
                           const uint8_t *nonces, const uint8_t *rands, uint8_t *public_shares,
                           uint8_t *helper_input_shares, uint8_t *leader_prep_shares,
                           uint8_t *leader_out_shares, int nthreads);

/* aggregate: element-wise field sum of n output shares (out_len elements each). */
int jo_aggregate(int algo, int bits, int length, int chunk, int proofs, uint64_t n,
                 const uint8_t *out_shares, uint8_t *agg_out);

/* Building blocks exposed for the KAT / cross-check tests. */
void jo_keccak_p1600(uint64_t state[25], int rounds);
void jo_turboshake128(const uint8_t *msg, size_t len, uint8_t D, uint8_t *out, size_t outlen);
void jo_xof_expand(const uint8_t seed[16], const uint8_t *dst, size_t dst_len,
                   const uint8_t *binder, size_t binder_len, uint8_t *out, size_t outlen);
/* XofHmacSha256Aes128 stream: the first outlen bytes for (seed, dst, binder). */
void jo_xof_hmac_aes(const uint8_t seed[32], const uint8_t *dst, size_t dst_len,
                     const uint8_t *binder, size_t binder_len, uint8_t *out, size_t outlen);
void jo_aes128_encrypt(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]);
int jo_field_op(int field64, int op, const uint8_t *a, const uint8_t *b, uint8_t *out);
void jo_sha256(const uint8_t *msg, size_t len, uint8_t out[32]);

#ifdef __cplusplus
}
#endif
#endif
