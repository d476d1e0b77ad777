/*
 * jx_hpke.h — C ABI of batched HPKE open on the MI355X.
 *
 * Replaces the per-report HPKE open of the helper's aggregate-init loop,
 *   /root/reference/aggregator/src/aggregator.rs:1772-1832
 *     hpke::open(&hpke_keypair, &HpkeApplicationInfo::new(&Label::InputShare, &Role::Client,
 *                &Role::Helper), prepare_init.report_share().encrypted_input_share(), &aad)
 * (core/src/hpke.rs:200-230), for Janus's suite: RFC 9180 base mode, DHKEM(X25519, HKDF-SHA256)
 * (0x0020), HKDF-SHA256 (0x0001), AES-128-GCM (0x0001). Once prepare runs on the GPU this is the
 * next per-report CPU cost (X25519 + key schedule + AEAD per report).
 *
 * Conventions as in jx_prio3.h: int32 status (0 = OK), caller-owned buffers, one context per
 * (keypair, application info, GPU). Calls on one context from several threads are serialized (a mutex per
 * context); jx_hpke_last_error returns the calling thread's last failure. The host-buffer open takes its
 * device buffers from the device's arena (shared with the prepare engines) and synchronizes only the
 * context's stream. jx_helper_prep_encrypted_batch (jx_prio3.h) opens inside the prepare launch instead.
 *  - encs:        n x 32 bytes (HpkeCiphertext.encapsulated_key)
 *  - cts:         ciphertexts (payload || 16-byte tag) back to back; ct_offsets[n + 1], ciphertext i
 *                 is [ct_offsets[i], ct_offsets[i+1]) and at least 16 bytes
 *  - aads:        associated data back to back (the encoded InputShareAad), aad_offsets[n + 1]
 *  - plaintexts:  plaintext i (ct length - 16 bytes) at offset ct_offsets[i] - 16 * i
 *  - ok:          n bytes, 1 = opened, 0 = HpkeDecryptError (bad tag, bad length, all-zero DH)
 */
#ifndef JX_HPKE_H
#define JX_HPKE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JX_HPKE_OK 0
#define JX_HPKE_E_INVALID (-1)
#define JX_HPKE_E_HIP (-3)
#define JX_HPKE_E_NOMEM (-4)
#define JX_HPKE_E_NODEVICE (-6)

typedef struct jx_hpke jx_hpke;

/* sk/pk: the recipient's X25519 key pair (SerializePrivateKey / public key, 32 bytes each);
 * info: the HPKE application info (Janus: "dap-09 input share" || sender role || recipient role). */
int32_t jx_hpke_create(const uint8_t sk[32], const uint8_t pk[32], const uint8_t* info, uint32_t info_len,
                       int32_t device, jx_hpke** out);
void jx_hpke_destroy(jx_hpke* h);

/* Host buffers. */
int32_t jx_hpke_open_batch(jx_hpke* h, uint64_t n, const uint8_t* encs, const uint8_t* cts,
                           const uint64_t* ct_offsets, const uint8_t* aads, const uint64_t* aad_offsets,
                           uint8_t* out_plaintexts, uint8_t* out_ok);
/* Device buffers (asynchronous on the context's stream; e.g. chain into jx_helper_prep_*). */
int32_t jx_hpke_open_batch_device(jx_hpke* h, uint64_t n, const void* d_encs, const void* d_cts,
                                  const uint64_t* d_ct_offsets, const void* d_aads, const uint64_t* d_aad_offsets,
                                  void* d_out_plaintexts, void* d_out_ok);
const char* jx_hpke_last_error(const jx_hpke* h);

#ifdef __cplusplus
}
#endif
#endif /* JX_HPKE_H */
