/* hbx.h -- C ABI of the MI355X batch engine for hbbft's threshold-crypto hot path.
 *
 * Drop-in boundary.  The reference calls threshold_crypto / pairing 0.14 one
 * share at a time on the caller's thread; this ABI takes a whole epoch's worth in one call.  Each
 * entry point names the reference interface it replaces (file:line in jonnydubowsky/hbbft @ v0).
 *
 * Conventions
 *  - Plain pointers + sizes, caller-owned buffers, no torch types.
 *  - Functions without the `_d` suffix take HOST pointers, stage through device buffers owned
 *    by the context and block until results are back on the host.
 *  - Functions with the `_d` suffix take DEVICE pointers (hipMalloc'd on the context's device)
 *    and a hipStream_t passed as `void*` (NULL = the HIP null stream, i.e. what a framework's
 *    default stream hands over); they enqueue work on that stream, in stream order with the
 *    caller's own work on it, and return without synchronising.
 *  - Return value: HBX_OK (0) or a negative HBX_E_* code.  A failed verification is NOT an error:
 *    it is a 0 in the corresponding validity output, exactly as the reference returns `false`.
 *  - Validity outputs are byte-per-item (1 = valid) in the `_d` API and little-endian bitmaps
 *    (bit k of byte k/8) in the host API.
 *  - Point encodings are the zcash/pairing 0.14 formats: G1 compressed 48 B, G2 compressed
 *    96 B, G2 uncompressed 192 B (x.c1 || x.c0 || y.c1 || y.c0).
 *  - Share matrices are proposer-major: share[j][i] = the decryption share node i sent for
 *    proposer j's ciphertext, at offset (j * n + i) * 48.
 *  - One context per device.  Calls on one context must be serialised by the caller.
 */
#ifndef HBX_H
#define HBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HBX_OK 0
#define HBX_E_INVALID_ARG (-1)
#define HBX_E_DEVICE (-2)
#define HBX_E_NOT_ENOUGH_SHARES (-3) /* threshold_crypto Error::NotEnoughShares */
#define HBX_E_DUPLICATE_ENTRY (-4)   /* threshold_crypto Error::DuplicateEntry */
#define HBX_E_NO_KEYS (-5)           /* hbx_set_pk_shares not called / wrong n */
#define HBX_E_NO_CIPHERTEXTS (-6)    /* hbx_prepare_ciphertexts not called / wrong p */
#define HBX_E_INVALID_CIPHERTEXT (-7)/* Ciphertext::verify failed or undecodable (honey_badger.rs:366-373) */
#define HBX_E_OUT_OF_MEMORY (-8)
#define HBX_E_TOO_FEW_SHARDS (-9)    /* reed_solomon_erasure Error::TooFewShardsPresent */
#define HBX_E_ROOT_MISMATCH (-10)    /* decode_from_shards: rebuilt Merkle root != hash (broadcast.rs:686) */
#define HBX_E_NO_PAYLOAD (-11)       /* glue_shards: fewer than 4 bytes (broadcast.rs:702) */

/* per-point decode status (hbx_set_pk_shares / hbx_prepare_ciphertexts) */
#define HBX_PT_OK 0
#define HBX_PT_BAD_FLAGS 1
#define HBX_PT_NOT_IN_FIELD 2
#define HBX_PT_NOT_ON_CURVE 3
#define HBX_PT_INFINITY 4
#define HBX_PT_NOT_IN_SUBGROUP 5 /* on the curve but not in G1 / G2 (pairing's into_affine rejects it) */

/* Per-share status (one byte per share: the d_valid arrays of the _d API, hbx_get_share_status,
 * hbx_get_sig_share_status).  1 = valid and 0 = verified false, so "byte == 1" is "valid";
 * the other codes tell the caller which reference fault, if any, the share maps to:
 *   HBX_SHARE_INVALID        verify returned false: FaultKind::UnverifiedDecryptionShareSender
 *                            (honey_badger.rs:199, :437) / UnverifiedSignatureShareSender
 *                            (common_coin.rs:153); the share is dropped.
 *   HBX_SHARE_VALID          verified true.
 *   HBX_SHARE_ABSENT         present bit 0: no message, nothing to report.
 *   HBX_SHARE_UNDECODABLE    the 48/96 bytes are not a subgroup point: the reference never sees
 *                            such a share (serde/bincode rejects the message before
 *                            HoneyBadger/CommonCoin), so no fault kind of the algorithm applies.
 *   HBX_SHARE_SKIPPED_CT     not verified because the proposer's ciphertext failed to decode or
 *                            Ciphertext::verify: the reference skips that proposer
 *                            (honey_badger.rs:359-376) and never verifies its shares.
 *   HBX_SHARE_UNKNOWN_SENDER sender index >= n of hbx_set_pk_shares: the reference rejects the
 *                            message with Error UnknownSender (honey_badger.rs:64-66,
 *                            common_coin.rs:158).  (own-share mode: `me` is always checked.) */
#define HBX_SHARE_INVALID 0
#define HBX_SHARE_VALID 1
#define HBX_SHARE_ABSENT 2
#define HBX_SHARE_UNDECODABLE 3
#define HBX_SHARE_SKIPPED_CT 4
#define HBX_SHARE_UNKNOWN_SENDER 5

/* Per-ciphertext status (d_ct_valid of the _d API, hbx_get_ct_status):
 *   HBX_CT_INVALID      Ciphertext::verify returned false: FaultKind::ShareDecryptionFailed
 *                       (honey_badger.rs:371-375).
 *   HBX_CT_VALID        verified.
 *   HBX_CT_UNDECODABLE  U or W does not decode to a subgroup point: bincode::deserialize of the
 *                       ciphertext fails, FaultKind::InvalidCiphertext (honey_badger.rs:359-368). */
#define HBX_CT_INVALID 0
#define HBX_CT_VALID 1
#define HBX_CT_UNDECODABLE 3

/* Digest variants (hbx_set_digest, hbx_set_merkle_digest). */
#define HBX_DIGEST_SHA256 0   /* default: ring SHA-256 (reference Cargo.toml:32) */
#define HBX_DIGEST_SHA3_256 1 /* tiny-keccak SHA3-256 */
#define HBX_MERKLE_SHA256 0   /* default: merkle (afck fork) + ring SHA-256, leaf H(0x00||v),
                                 node H(0x01||l||r), odd node promoted (broadcast.rs:161, :381) */
#define HBX_MERKLE_SHA3 1     /* later hbbft's own tree (src/broadcast/merkle.rs, tiny-keccak):
                                 leaf SHA3(v), node SHA3(l||r), odd node promoted */

typedef struct hbx_ctx hbx_ctx;

/* Create / destroy a context bound to HIP device `device`. */
int hbx_ctx_create(int device, hbx_ctx** out);
int hbx_ctx_destroy(hbx_ctx* ctx);
/* Human-readable description of the last error on this context (never NULL). */
const char* hbx_last_error(const hbx_ctx* ctx);
/* Library version string, e.g. "hbx 0.1.0 gfx950". */
const char* hbx_version(void);
/* SHA-256 (hex) of the sources this library was built from (hbbft_amd/buildinfo.py source_hash,
 * set by tools/build.py); "unknown" for a build outside it.  Provenance only: no reference
 * counterpart. */
const char* hbx_build_id(void);

/* Kernel timing (instrumentation; no reference counterpart).  With timing on, the library
 * brackets each launch of the kernels below with HIP events recorded on the stream the kernel
 * runs on; hbx_kernel_time synchronizes those events and reports the summed duration and the
 * number of launches since the last hbx_set_timing call. */
#define HBX_K_PREPARE_CT 0      /* hash_g1_g2 + decode of U/W per proposer */
#define HBX_K_PREPARE_LINES 1   /* prepared Miller lines of H_j, W_j (and coin H) */
#define HBX_K_CT_CHECKS 2       /* Ciphertext::verify pairing checks (wide executor) */
#define HBX_K_VERIFY_SHARES 3   /* decryption-share pairing checks */
#define HBX_K_COMBINE 4         /* Lagrange combine + key derivation per proposer */
#define HBX_K_VERIFY_SIG 5      /* coin signature-share checks */
#define HBX_K_COMBINE_SIGS 6    /* coin G2 Lagrange combine + master-key check */
#define HBX_K_RS_CODE 7         /* Reed-Solomon encode / reconstruct passes */
#define HBX_K_MERKLE_LEAVES 8   /* SHA-256 leaf hashes */
#define HBX_K_HASH_NONCES 9     /* coin nonce hash_g2 */
#define HBX_K_DECODE_SIGS 10    /* coin signature-share decode (G2 decompression; the checks test G2 membership) */
#define HBX_K_COUNT 11
int hbx_set_timing(hbx_ctx* ctx, int on);
int hbx_kernel_time(hbx_ctx* ctx, int kernel, double* total_ms, uint32_t* launches);

/* ---------------------------------------------------------------------------------------------
 * DIGEST of threshold_crypto's hash_g2 / hash_g1_g2 / hash_bytes.  The
 * reference's threshold_crypto dependency is an unpinned git revision (Cargo.toml:35): revisions
 * hash with SHA-256 or with tiny-keccak's SHA3-256.  Per context, default HBX_DIGEST_SHA256;
 * switching voids the prepared ciphertexts / nonces.  Affects every H_j, W, plaintext keystream,
 * nonce hash and signature of this context.
 * hbx_set_merkle_digest -- the Merkle tree of the broadcast calls (HBX_MERKLE_*).
 * ------------------------------------------------------------------------------------------- */
int hbx_set_digest(hbx_ctx* ctx, int variant);
/* Lanes per decryption-share check (no reference counterpart; results identical): 1 = one lane
 * per check (the throughput path when a launch fills the chip: a Miller-loop kernel and the final
 * exponentiation as four step kernels over per-lane slots), 7 = one lane per check in a single
 * kernel (the final exponentiation through call frames; kept for comparison), 2 = a lane pair per
 * check (the
 * Fq12 state split in halves, no scratch), 3 = three cooperating lanes per check, 6 = six lanes per
 * check (the two Miller loops on two lane triplets side by side; lowest latency per check), 0 =
 * choose by launch size (default: 1 when one-lane checks fill >= 1024 waves, else 6 when six-lane
 * checks fit in 1024 waves, else 3). */
int hbx_set_verify_lanes(hbx_ctx* ctx, int lanes);
/* Lanes per check the last decryption-share launch used (1, 2, 3, 6 or 7; 0 before any launch). */
int hbx_get_verify_lanes_used(const hbx_ctx* ctx);
/* Tests only: in one-lane decryption-share checks and two-lane coin checks, treat the check of
 * every `every`-th sender (0 = none, the default) as if its compressed squarings had met a zero
 * denominator, so the fallback path decides it (the single-kernel one-lane check; for the coin, the
 * pair's Miller loop again and a final exponentiation without compressed runs).  Results are
 * unchanged.  (Real inputs reach that path only through an element with a zero Fq2 coefficient at
 * the end of a compressed run, ~2^-760 for values nobody chose; the one degenerate start a proposer
 * can choose -- a ciphertext with r = 3(x^2 - 1), for which every honest share's check is 1 after
 * the easy part -- is decided by the first step without a fallback.) */
int hbx_debug_force_fallback(hbx_ctx* ctx, uint32_t every);
/* Checks of the last share-check launch (decryption-share or coin, whichever came last) that the
 * fallback path decided: 0 unless hbx_debug_force_fallback is on, and 0 when that launch used a lane
 * count without a fallback path (decryption shares at lanes 2/3/6/7, coin at one lane).  The two
 * kinds count separately; "last" is host call order, so the value is meaningful when the caller
 * reads it after the launch it asks about (waits for the context's streams).  Diagnostics: no
 * reference counterpart. */
int64_t hbx_get_fallback_lanes(hbx_ctx* ctx);
/* Lanes per Lagrange term of hbx_combine_decrypt_d (no reference counterpart; results identical):
 * 1 = one lane per GLV term, one block per proposer (k_combine), 4 = a quad of lanes per term over
 * one-wave blocks (k_combine_q, t <= 128), 0 = by launch size (default: 4 when the quad blocks fit
 * in 1024 waves, else 1). */
int hbx_set_combine_lanes(hbx_ctx* ctx, int lanes);
int hbx_set_merkle_digest(hbx_ctx* ctx, int variant);

/* ---------------------------------------------------------------------------------------------
 * Key material (once per era).
 * Replaces: NetworkInfo::new's public_key_share derivation (src/messaging.rs:251-254) and the
 * per-call lookup NetworkInfo::public_key_share (src/messaging.rs:312) used by
 * HoneyBadger::verify_decryption_share (src/honey_badger/honey_badger.rs:228-232).
 * pk_comp: n x 48 B compressed pk_i (node index order = BTreeMap order, messaging.rs:246-250).
 * status (optional, n entries): HBX_PT_* per key.
 * A new key set clears this node's own share (hbx_set_own_share must be called again for the
 * new era) and every epoch result computed under the old keys.
 * ------------------------------------------------------------------------------------------- */
int hbx_set_pk_shares(hbx_ctx* ctx, const uint8_t* pk_comp, uint32_t n, int32_t* status);

/* ---------------------------------------------------------------------------------------------
 * This node's own secret key share (once per era; optional).
 * Replaces: the node's own share path -- SecretKeyShare::decrypt_share_no_verify in
 * send_decryption_share (src/honey_badger/honey_badger.rs:394-418), whose result the node feeds
 * back to itself as sender `me`.  With it set, hbx_prepare_ciphertexts* computes S_j,me = sk_me U_j
 * for every ciphertext, hbx_verify_dec_shares* uses it for sender `me` (that row of the share
 * input is ignored), and the check of that share doubles as Ciphertext::verify (:371): U_j, W_j are
 * decoded with subgroup checks and H_j is in G2, so e(sk U, H) e(-sk g1, W) = 1 exactly when
 * e(U, H) = e(g1, W) (sk != 0 mod r).  This removes the separate latency-bound ciphertext checks.
 * sk32: canonical big-endian scalar in [1, r) matching pk[me] of hbx_set_pk_shares
 * (HBX_E_INVALID_ARG otherwise); NULL clears the mode.
 * ------------------------------------------------------------------------------------------- */
int hbx_set_own_share(hbx_ctx* ctx, uint32_t me, const uint8_t* sk32);

/* ---------------------------------------------------------------------------------------------
 * Ciphertexts of one epoch (one per accepted proposer).
 * Replaces: threshold_crypto Ciphertext::verify (src/honey_badger/honey_badger.rs:371) and
 * hoists hash_g1_g2(U_j, V_j) -- recomputed by the reference inside every
 * verify_decryption_share call -- to once per ciphertext.
 * u_comp: p x 48 B; w_comp: p x 96 B; v_blob + v_off[p + 1]: the V byte strings.
 * ct_valid_bits: ceil(p/8) B out; bit j = Ciphertext::verify(ct_j) (0 also for undecodable
 * points, i.e. the reference's InvalidCiphertext / ShareDecryptionFailed faults).
 * ------------------------------------------------------------------------------------------- */
int hbx_prepare_ciphertexts(hbx_ctx* ctx, const uint8_t* u_comp, const uint8_t* v_blob,
                            const uint64_t* v_off, const uint8_t* w_comp, uint32_t p,
                            uint8_t* ct_valid_bits);

/* ---------------------------------------------------------------------------------------------
 * Decryption-share verification, whole epoch.
 * Replaces: PublicKeyShare::verify_decryption_share (src/honey_badger/honey_badger.rs:229) as
 * called from verify_pending_decryption_shares (:422-444) and handle_decryption_share_message
 * (:198).  valid[j][i] = e(S_ji, H_j) == e(pk_i, W_j).  Absent shares (present bit 0), unknown
 * senders (i >= n of hbx_set_pk_shares), undecodable encodings and shares of a ciphertext that
 * failed hbx_prepare_ciphertexts give 0; hbx_get_share_status tells these apart (HBX_SHARE_*),
 * so a caller raises UnverifiedDecryptionShareSender exactly for HBX_SHARE_INVALID.
 * shares: p x n x 48 B; present_bits: ceil(p*n/8) B (NULL = all present);
 * valid_bits: ceil(p*n/8) B out (bit j*n + i).
 * ------------------------------------------------------------------------------------------- */
int hbx_verify_dec_shares(hbx_ctx* ctx, const uint8_t* shares, const uint8_t* present_bits,
                          uint32_t n, uint32_t p, uint8_t* valid_bits);

/* Status bytes of the last share verification (p x n, HBX_SHARE_*) and of the last prepared
 * ciphertexts (p, HBX_CT_*), copied to the host (blocking).  count must equal p*n (resp. p). */
int hbx_get_share_status(hbx_ctx* ctx, uint8_t* status, size_t count);
int hbx_get_ct_status(hbx_ctx* ctx, uint8_t* status, size_t count);
/* The hoisted H_j = hash_g1_g2(U_j, V_j) of the last prepared ciphertexts (threshold_crypto,
 * recomputed by the reference inside every verify_decryption_share, honey_badger.rs:229),
 * compressed, p x 96 B; the identity for a ciphertext that does not decode. */
int hbx_get_ct_hashes(hbx_ctx* ctx, uint8_t* h96, size_t count);

/* ---------------------------------------------------------------------------------------------
 * Threshold decryption of every proposer's contribution.
 * Replaces: PublicKeySet::decrypt (src/honey_badger/honey_badger.rs:340) inside
 * try_decrypt_proposer_contribution (:315-349): for each proposer j takes the FIRST t valid
 * shares in node-index order, Lagrange-interpolates at 0 (x = index + 1) and XORs V_j with
 * hash_bytes(g, |V_j|).  Uses the shares and validity of the last hbx_verify_dec_shares call.
 * out_blob: sum |V_j| bytes at the v_off offsets of hbx_prepare_ciphertexts.
 * status: p entries, HBX_OK / HBX_E_NOT_ENOUGH_SHARES / HBX_E_INVALID_CIPHERTEXT.
 * ------------------------------------------------------------------------------------------- */
int hbx_combine_decrypt(hbx_ctx* ctx, uint32_t t, uint8_t* out_blob, int32_t* status);

/* ---------------------------------------------------------------------------------------------
 * Device-pointer / stream variants (inputs resident in HBM; nothing is copied to the host).
 *   d_present is a byte-per-share array (nonzero = present); d_valid receives one HBX_SHARE_*
 *   status byte per share and d_ct_valid one HBX_CT_* byte per ciphertext (1 = valid in both).
 *   A prepare invalidates the previous verification: combine needs a verify of the same p after
 *   the latest prepare (HBX_E_NO_CIPHERTEXTS otherwise).
 * hbx_prepare_ciphertexts_d with d_ct_valid == NULL DEFERS Ciphertext::verify: the checks then run
 * fused into the next hbx_verify_dec_shares_d launch (one more pairing check per proposer next
 * to its n share checks), and hbx_get_ct_valid_d copies the result out afterwards.
 * ------------------------------------------------------------------------------------------- */
int hbx_prepare_ciphertexts_d(hbx_ctx* ctx, const uint8_t* d_u_comp, const uint8_t* d_v_blob,
                              const uint64_t* d_v_off, const uint8_t* d_w_comp, uint32_t p,
                              uint64_t max_v_len, uint8_t* d_ct_valid, void* stream);
int hbx_verify_dec_shares_d(hbx_ctx* ctx, const uint8_t* d_shares, const uint8_t* d_present,
                            uint32_t n, uint32_t p, uint8_t* d_valid, void* stream);
int hbx_combine_decrypt_d(hbx_ctx* ctx, uint32_t t, uint8_t* d_out_blob, int32_t* d_status,
                          void* stream);
int hbx_get_ct_valid_d(hbx_ctx* ctx, uint8_t* d_ct_valid, void* stream);

/* One node-epoch of threshold decryption in ONE call: what honey_badger.rs does per epoch through
 * Ciphertext::verify (:371), verify_decryption_share (:229, :422-444) and PublicKeySet::decrypt
 * (:340), batched ("route whole epochs' worth of shares through one batched call").
 * Results and stream semantics are those of hbx_prepare_ciphertexts_d (Ciphertext::verify
 * deferred) + hbx_verify_dec_shares_d + hbx_get_ct_valid_d + hbx_combine_decrypt_d.
 * All outputs are device arrays, complete when `stream` reaches the end of the call's work. */
int hbx_decrypt_epoch_d(hbx_ctx* ctx, const uint8_t* d_u_comp, const uint8_t* d_v_blob, const uint64_t* d_v_off,
                        const uint8_t* d_w_comp, uint32_t p, uint64_t max_v_len, const uint8_t* d_shares,
                        const uint8_t* d_present, uint32_t n, uint32_t t, uint8_t* d_valid, uint8_t* d_ct_valid,
                        uint8_t* d_out_blob, int32_t* d_status, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Producer side.  Scalars are canonical Fr values as
 * 32-byte big-endian strings (< r; anything else is HBX_E_INVALID_ARG).
 *
 * hbx_public_keys -- threshold_crypto SecretKey::public_key, pk_i = g1 * sk_i, as used by the
 *   test key generation NetworkInfo::generate_map (src/messaging.rs:359-401).
 * hbx_encrypt -- PublicKey::encrypt (src/honey_badger/honey_badger.rs:116) with the randomness
 *   r_j passed in (threshold_crypto draws it from thread_rng):  U = g1 r, V = M xor
 *   hash_bytes(pk r, |M|), W = hash_g1_g2(U, V) r.  v_blob uses the msg_off offsets.
 * hbx_decrypt_shares -- SecretKeyShare::decrypt_share_no_verify
 *   (src/honey_badger/honey_badger.rs:403): shares[j][i] = sk_i * U_j, proposer-major p x n x 48.
 * ------------------------------------------------------------------------------------------- */
int hbx_public_keys(hbx_ctx* ctx, const uint8_t* sk32, uint32_t n, uint8_t* pk48);
int hbx_encrypt(hbx_ctx* ctx, const uint8_t* pk48, const uint8_t* msg_blob, const uint64_t* msg_off,
                uint32_t p, const uint8_t* r32, uint8_t* u48, uint8_t* v_blob, uint8_t* w96);
int hbx_decrypt_shares(hbx_ctx* ctx, const uint8_t* sk32, uint32_t n, const uint8_t* u48, uint32_t p,
                       uint8_t* shares48);

/* ---------------------------------------------------------------------------------------------
 * Common Coin, batched over `count` coin instances (concurrent
 * Agreement instances; the nonce of each is Nonce::new, src/agreement/mod.rs:155-165).
 * hbx_prepare_nonces -- hash_g2(nonce_i) once per instance (threshold_crypto, hoisted out of
 *   every share verification); h96 (optional) = the compressed points.  The call returns once the
 *   nonces are uploaded (with h96, once the hashes are in h96); later coin calls on any stream are
 *   ordered after the hashing, and only hbx_sign waits for the true H (the checks and the combine
 *   work on [m] H).
 * hbx_sign -- SecretKeyShare::sign (src/common_coin.rs:142): sig96[inst][i] = sk_i * hash_g2(nonce).
 * hbx_verify_sig_shares -- PublicKeyShare::verify (src/common_coin.rs:151) for a [count][n] matrix
 *   of compressed signature shares (present_bits NULL = all present); uses hbx_set_pk_shares keys.
 *   Bit inst*n+i = e(pk_i, H) == e(g1, sig_i); absent / undecodable / unknown sender -> 0.
 * hbx_combine_signatures -- PublicKeySet::combine_signatures over the first t valid shares in
 *   node-index order (src/common_coin.rs:190) + PublicKey::verify with the master key (:196) +
 *   Signature::parity (:173).  status[inst]: HBX_OK / HBX_E_NOT_ENOUGH_SHARES.
 * Device variants (torch-style HBM buffers, `stream` as in the threshold _d calls):
 * hbx_verify_sig_shares_d -- d_sig96 [count][n][96], d_present [count][n] bytes (NULL = all),
 *   d_status [count][n] = HBX_SHARE_* (NULL: keep them in the context only).
 * hbx_combine_signatures_d -- as hbx_combine_signatures over the last verification's valid shares,
 *   restricted to d_use[inst][i] != 0 when d_use is given (the shares a node held when try_output
 *   ran, common_coin.rs:163-190); outputs d_sig96 [I][96], d_status [I] int32, d_master_ok [I] and
 *   d_parity [I] bytes (each may be NULL).  The master key is a host pointer (48 bytes; decoded
 *   once per distinct value).
 * ------------------------------------------------------------------------------------------- */
int hbx_prepare_nonces(hbx_ctx* ctx, const uint8_t* nonce_blob, const uint64_t* nonce_off, uint32_t count,
                       uint8_t* h96);
int hbx_sign(hbx_ctx* ctx, const uint8_t* sk32, uint32_t n, uint8_t* sig96);
int hbx_verify_sig_shares(hbx_ctx* ctx, const uint8_t* sig96, const uint8_t* present_bits, uint32_t n,
                          uint32_t count, uint8_t* valid_bits);
/* HBX_SHARE_* status of every share of the last hbx_verify_sig_shares (count x n bytes). */
int hbx_get_sig_share_status(hbx_ctx* ctx, uint8_t* status, size_t count);
int hbx_combine_signatures(hbx_ctx* ctx, const uint8_t* master_pk48, uint32_t t, uint8_t* sig96,
                           int32_t* status, uint8_t* master_ok_bits, uint8_t* parity_bits);
int hbx_verify_sig_shares_d(hbx_ctx* ctx, const uint8_t* d_sig96, const uint8_t* d_present, uint32_t n,
                            uint32_t count, uint8_t* d_status, void* stream);
int hbx_combine_signatures_d(hbx_ctx* ctx, const uint8_t* master_pk48, uint32_t t, const uint8_t* d_use,
                             uint8_t* d_sig96, int32_t* d_status, uint8_t* d_master_ok, uint8_t* d_parity,
                             void* stream);
/* Lanes per check the last signature-share verification used (1 or 2; 0 before any): the coin
 * honours hbx_set_verify_lanes 1 and 2; 0, 3, 6 and 7 choose automatically (2 when one-lane checks
 * would fill fewer than 1024 waves, else 1). */
int hbx_get_coin_lanes_used(const hbx_ctx* ctx);

/* ---------------------------------------------------------------------------------------------
 * Dynamic HoneyBadger / key-generation signatures: threshold_crypto
 * PublicKey::verify(sig, msg) = e(pk, hash_g2(msg)) == e(g1, sig) for `count` independent items,
 * each with its own key, message and signature -- the signed votes of
 * src/dynamic_honey_badger/votes.rs:151-156 (msg = bincode(vote)) and the key-generation messages
 * of src/dynamic_honey_badger/dynamic_honey_badger.rs:395-410 (msg = bincode(kg_msg)).
 *   pk48[count][48], sig96[count][96] compressed; msg_off[count + 1] byte offsets into msg_blob.
 *   status[count] = HBX_SHARE_VALID (true), HBX_SHARE_INVALID (false), HBX_SHARE_UNDECODABLE (the
 *   key or the signature is not a subgroup point: the reference cannot deserialise it).
 *   hash_g2 uses the context's digest (hbx_set_digest).  Independent of the coin state.
 * ------------------------------------------------------------------------------------------- */
int hbx_verify_sigs(hbx_ctx* ctx, const uint8_t* pk48, const uint8_t* msg_blob, const uint64_t* msg_off,
                    const uint8_t* sig96, uint32_t count, uint8_t* status);
/* SyncKeyGen (src/sync_key_gen.rs) commitment checks over p Parts' BivarCommitments of degree t:
 *   commit48[p][(t+1)(t+2)/2][48], compressed, in threshold_crypto's coefficient order
 *   coeff_pos(i, j) = j (j + 1)/2 + i for i <= j (the symmetric matrix stored once).
 * hbx_bivar_rows -- BivarCommitment::row(x) (sync_key_gen.rs:313 `commit.row(idx + 1)`, :401):
 *   rows48[p][t + 1][48] = sum_i C_ij x^i; status[p] = HBX_SHARE_VALID, or HBX_SHARE_UNDECODABLE
 *   when a point of the commitment is not in G1 (the Part does not deserialise).
 * hbx_bivar_check_acks -- handle_ack's value check (sync_key_gen.rs:449):
 *   commit[ack_proposer[k]].evaluate(x, ack_y[k]) == g1 * val_k with val_k = vals32[k] (32-byte
 *   big-endian Fr; x = our_idx + 1, y = sender_idx + 1).  status[k] = HBX_SHARE_VALID (equal),
 *   HBX_SHARE_INVALID ("wrong value"), HBX_SHARE_UNDECODABLE (val >= r or the commitment does
 *   not decode). */
int hbx_bivar_rows(hbx_ctx* ctx, const uint8_t* commit48, uint32_t p, uint32_t t, uint64_t x, uint8_t* rows48,
                   uint8_t* status);
int hbx_bivar_check_acks(hbx_ctx* ctx, const uint8_t* commit48, uint32_t p, uint32_t t, uint64_t x,
                         const uint32_t* ack_proposer, const uint64_t* ack_y, const uint8_t* vals32, uint32_t count,
                         uint8_t* status);

/* ---------------------------------------------------------------------------------------------
 * Broadcast: Reed-Solomon erasure coding and the Merkle tree over shards (SURVEY.md §8 rows
 * C1-C5d), batched over `inst` broadcast instances.  Device pointers, stream-ordered.
 * Shards of one instance are contiguous: d_shards[inst][k + m][L]; leaf i of an instance is the
 * index byte i followed by shard i (src/broadcast.rs:373-377).  Requires k + m <= 256, k <= 128.
 *
 * hbx_rs_encode_d -- ReedSolomon::encode (reed-solomon-erasure 3.1.0) via Coding::encode
 *   (src/broadcast.rs:632-640, called at :365): fills the m parity shards of every instance.
 * hbx_rs_reconstruct_d -- ReedSolomon::reconstruct_shards via Coding::reconstruct_shards
 *   (src/broadcast.rs:643-657, called at :667): rebuilds every shard whose d_present byte is 0
 *   from the first k present shards.  d_status[inst]: HBX_OK or HBX_E_TOO_FEW_SHARDS.
 * hbx_merkle_roots_d -- MerkleTree::from_vec(&SHA256, leaves).root_hash() (src/broadcast.rs:381,
 *   :683-686) over the index-prefixed shards: d_roots[inst][32].
 * hbx_merkle_validate_d -- Broadcast::validate_proof (src/broadcast.rs:555-575):
 *   Proof::validate(&root_hash) && node_index(sender) == value[0] && Proof::index(count) == value[0],
 *   for nproofs flattened proofs: d_values[j][vlen] (the leaf: index byte + shard),
 *   d_node_hash[j][17][32] (lemma node hashes from the root down to the leaf hash),
 *   d_sib_hash[j][16][32], d_sides[j] (bit l: the level-l sibling is Positioned::Left),
 *   d_depth[j], d_root[j][32] (the proof's root_hash), d_sender[j]; d_valid[j] out.
 * hbx_broadcast_decode_d -- decode_from_shards + glue_shards (src/broadcast.rs:660-707):
 *   reconstruct, rebuild the tree, compare with d_root_expect[inst][32], glue the first k shards.
 *   d_out[inst][out_stride], d_out_len[inst], d_status[inst]: HBX_OK / HBX_E_TOO_FEW_SHARDS /
 *   HBX_E_ROOT_MISMATCH / HBX_E_NO_PAYLOAD.  With m == 0 (Coding::Trivial) any absent shard
 *   is HBX_E_TOO_FEW_SHARDS.
 * ------------------------------------------------------------------------------------------- */
int hbx_rs_encode_d(hbx_ctx* ctx, uint8_t* d_shards, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                    void* stream);
int hbx_rs_reconstruct_d(hbx_ctx* ctx, uint8_t* d_shards, const uint8_t* d_present, uint32_t inst, uint32_t k,
                         uint32_t m, uint32_t L, int32_t* d_status, void* stream);
int hbx_merkle_roots_d(hbx_ctx* ctx, const uint8_t* d_shards, uint32_t inst, uint32_t n, uint32_t L,
                       uint8_t* d_roots, void* stream);
int hbx_merkle_validate_d(hbx_ctx* ctx, const uint8_t* d_values, uint32_t vlen, const uint8_t* d_node_hash,
                          const uint8_t* d_sib_hash, const uint32_t* d_sides, const uint32_t* d_depth,
                          const uint8_t* d_root, const uint32_t* d_sender, uint32_t count, uint32_t nproofs,
                          uint8_t* d_valid, void* stream);
/* hbx_merkle_build_d -- MerkleTree::from_vec over the index-prefixed shards, keeping the whole
 *   tree (SURVEY.md §8(b) hbx_merkle_build): d_nodes[inst][hbx_merkle_node_count(n)][32], the
 *   levels from the n leaf digests up to the root (last), a promoted odd node repeated on the
 *   level it moves to; d_roots[inst][32] optional.
 * hbx_merkle_proofs_d -- MerkleTree::gen_proof (src/broadcast.rs:389-401: one Value proof per
 *   node) from such trees: proof q for leaf d_req[2q + 1] of instance d_req[2q] (the proof of the
 *   first leaf with an equal digest, as merkle.rs finds the first equal value), written in the
 *   format hbx_merkle_validate_d reads (d_node_hash[q][17][32] root first, d_sib_hash[q][16][32],
 *   d_sides[q], d_depth[q], d_root[q][32]). */
uint32_t hbx_merkle_node_count(uint32_t n);
int hbx_merkle_build_d(hbx_ctx* ctx, const uint8_t* d_shards, uint32_t inst, uint32_t n, uint32_t L,
                       uint8_t* d_nodes, uint8_t* d_roots, void* stream);
int hbx_merkle_proofs_d(hbx_ctx* ctx, const uint8_t* d_nodes, uint32_t n, const uint32_t* d_req, uint32_t count,
                        uint8_t* d_node_hash, uint8_t* d_sib_hash, uint32_t* d_sides, uint32_t* d_depth,
                        uint8_t* d_root, void* stream);
int hbx_broadcast_decode_d(hbx_ctx* ctx, uint8_t* d_shards, const uint8_t* d_present,
                           const uint8_t* d_root_expect, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                           uint8_t* d_out, uint64_t out_stride, uint64_t* d_out_len, int32_t* d_status,
                           void* stream);
/* hbx_broadcast_decode_leaves_d -- the same decode for Echo values that were validated
 *   (hbx_merkle_validate_d): d_leaf_hash[inst][k + m][32] holds, for every present shard, the leaf
 *   digest its Echo proof carries (the last lemma node, which validation proved equal to the digest
 *   of the value).  compute_output rebuilds the tree over those same bytes (broadcast.rs:530-544,
 *   :683), so only the reconstructed shards are hashed.  Same outputs as
 *   hbx_broadcast_decode_d when the digests are the values' own. */
int hbx_broadcast_decode_leaves_d(hbx_ctx* ctx, uint8_t* d_shards, const uint8_t* d_present,
                                  const uint8_t* d_leaf_hash, const uint8_t* d_root_expect, uint32_t inst,
                                  uint32_t k, uint32_t m, uint32_t L, uint8_t* d_out, uint64_t out_stride,
                                  uint64_t* d_out_len, int32_t* d_status, void* stream);

/* Host-pointer forms of the Broadcast calls: the same operations and layouts on HOST buffers,
 * staged through device buffers the context owns, on the context's own stream; they block until
 * the outputs are back (the stack-A/B convention above).  What a thin Rust FFI calls from
 * Vec<u8> / &[u8] without a HIP runtime binding of its own:
 *   hbx_rs_encode          Coding::encode / ReedSolomon::encode (src/broadcast.rs:632-640, called at
 *                          :366): shards[inst][k + m][L]; reads the k data rows, writes the m parity
 *                          rows of every instance.
 *   hbx_rs_reconstruct     Coding::reconstruct_shards (src/broadcast.rs:643-657, called at :667):
 *                          present[inst][k + m] bytes; shards rewritten in place, status[inst].
 *   hbx_merkle_roots       MerkleTree::from_vec(..).root_hash() (src/broadcast.rs:381): roots[inst][32].
 *   hbx_merkle_build       the whole tree (src/broadcast.rs:381): nodes[inst][hbx_merkle_node_count(n)][32],
 *                          roots optional.
 *   hbx_merkle_proofs      MerkleTree::gen_proof (src/broadcast.rs:389-401) from hbx_merkle_build's
 *                          nodes of `inst` instances: req[count][2] = (instance, leaf); outputs as
 *                          hbx_merkle_proofs_d, sides[count] and depth[count] as uint32.
 *   hbx_merkle_validate    Broadcast::validate_proof (src/broadcast.rs:555-575, called for Value at
 *                          :430 and Echo at :451); arrays as hbx_merkle_validate_d, valid[nproofs].
 *   hbx_broadcast_decode   decode_from_shards + glue_shards (src/broadcast.rs:660-707): shards
 *                          rewritten in place (reconstructed rows), out[inst][out_stride],
 *                          out_len[inst], status[inst].
 *   hbx_broadcast_decode_leaves  the same with the validated Echo proofs' leaf digests
 *                          (leaf_hash[inst][k + m][32]). */
int hbx_rs_encode(hbx_ctx* ctx, uint8_t* shards, uint32_t inst, uint32_t k, uint32_t m, uint32_t L);
int hbx_rs_reconstruct(hbx_ctx* ctx, uint8_t* shards, const uint8_t* present, uint32_t inst, uint32_t k, uint32_t m,
                       uint32_t L, int32_t* status);
int hbx_merkle_roots(hbx_ctx* ctx, const uint8_t* shards, uint32_t inst, uint32_t n, uint32_t L, uint8_t* roots);
int hbx_merkle_build(hbx_ctx* ctx, const uint8_t* shards, uint32_t inst, uint32_t n, uint32_t L, uint8_t* nodes,
                     uint8_t* roots);
int hbx_merkle_proofs(hbx_ctx* ctx, const uint8_t* nodes, uint32_t inst, uint32_t n, const uint32_t* req,
                      uint32_t count, uint8_t* node_hash, uint8_t* sib_hash, uint32_t* sides, uint32_t* depth,
                      uint8_t* root);
int hbx_merkle_validate(hbx_ctx* ctx, const uint8_t* values, uint32_t vlen, const uint8_t* node_hash,
                        const uint8_t* sib_hash, const uint32_t* sides, const uint32_t* depth, const uint8_t* root,
                        const uint32_t* sender, uint32_t count, uint32_t nproofs, uint8_t* valid);
int hbx_broadcast_decode(hbx_ctx* ctx, uint8_t* shards, const uint8_t* present, const uint8_t* root_expect,
                         uint32_t inst, uint32_t k, uint32_t m, uint32_t L, uint8_t* out, uint64_t out_stride,
                         uint64_t* out_len, int32_t* status);
int hbx_broadcast_decode_leaves(hbx_ctx* ctx, uint8_t* shards, const uint8_t* present, const uint8_t* leaf_hash,
                                const uint8_t* root_expect, uint32_t inst, uint32_t k, uint32_t m, uint32_t L,
                                uint8_t* out, uint64_t out_stride, uint64_t* out_len, int32_t* status);

#ifdef __cplusplus
}
#endif
#endif /* HBX_H */
