/*
 * rsgpu.h — C ABI of the MI355X-native Reed–Solomon GF(2^8) erasure engine.
 *
 * This is the drop-in boundary for the erasure hot path of rustfs
 * (crates/ecstore/src/erasure/).  Every entry point names the reference
 * interface it replaces; the Rust-side `extern "C"` binding a maintainer would
 * add is in INTEGRATION.md.  Plain pointers and sizes only; no torch types.
 *
 * Codec: GF(2^8) with polynomial 0x11D, generator 2, systematic matrix
 * V * inv(V[0..k]) with V[r][c] = r^c ("rs-vandermonde", the construction of
 * reed_solomon_erasure::galois_8::ReedSolomon used by rustfs and MinIO;
 * docs/architecture/erasure-coding.md:41-50).  Outputs are bit-exact with it.
 *
 * Threading: every function is thread-safe.  A context owns one device and
 * per-geometry coefficient caches.  Host-buffer calls (rsg_encode,
 * rsg_reconstruct, rsg_verify, rsg_hash) run on one of the context's 8 lanes
 * (own stream and device buffer), so up to 8 concurrent callers overlap and
 * further ones wait for a free lane (the reference calls encode from many
 * tokio workers concurrently, encode.rs:511-526).  Device-batch calls are
 * asynchronous on the caller's stream; every record-engine call (decode / heal /
 * bitrot_verify) takes its own scratch from the context's pool, so concurrent
 * calls overlap.  Tickets (host-batch PUT, asynchronous GET / heal) may be
 * polled or waited on from several threads.
 *
 * Errors: functions return an rsg_status; rsg_strerror() gives the message
 * fragment the reference uses for the same condition (erasure.rs:87-121,
 * 396-446, 505-594; bridge.rs:202-235; bitrot.rs:227-247).
 */
#ifndef RSGPU_H
#define RSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSG_ABI_VERSION 6
#define RSG_MAX_TOTAL_SHARDS 256 /* galois_8::Field::ORDER, erasure.rs:72 */
#define RSG_DIGEST_BYTES 32      /* HighwayHash-256 */

typedef enum rsg_status {
    RSG_OK = 0,
    RSG_ERR_INVALID_ARG = 1,           /* null pointer / bad flag */
    RSG_ERR_ZERO_DATA_SHARDS = 2,      /* ErasureConstructionError::ZeroDataShards, erasure.rs:90 */
    RSG_ERR_ZERO_PARITY_SHARDS = 3,    /* reed_solomon_erasure::Error::TooFewParityShards */
    RSG_ERR_TOO_MANY_SHARDS = 4,       /* UnsupportedModernShardCount, erasure.rs:102 */
    RSG_ERR_INVALID_SHARD_COUNT = 5,   /* "invalid shard count", erasure.rs:512 */
    RSG_ERR_INCONSISTENT_LENGTH = 6,   /* "inconsistent shard length", erasure.rs:536 */
    RSG_ERR_EMPTY_SHARD = 7,           /* reed_solomon_erasure::Error::EmptyShard */
    RSG_ERR_TOO_FEW_SHARDS = 8,        /* Error::TooFewShardsPresent -> "Reed-Solomon reconstruct failed" */
    RSG_ERR_NO_VALID_SHARDS = 9,       /* "No valid shards found", erasure.rs:521 */
    RSG_ERR_INCONSISTENT_SOURCES = 10, /* InvalidData "inconsistent read source shards", bridge.rs:231 */
    RSG_ERR_BITROT_MISMATCH = 11,      /* InvalidData "bitrot hash mismatch", bitrot.rs:241 */
    RSG_ERR_NO_DEVICE = 12,            /* no HIP device / bad ordinal */
    RSG_ERR_DEVICE = 13,               /* HIP runtime failure */
    RSG_ERR_OUT_OF_MEMORY = 14,
    RSG_ERR_UNSUPPORTED = 15,
    RSG_ERR_FILE_SIZE_MISMATCH = 16,   /* "bitrot shard file size mismatch", bitrot.rs:627 */
    RSG_ERR_UNEXPECTED_EOF = 17,       /* io::ErrorKind::UnexpectedEof from read_exact, bitrot.rs:631,639 */
    RSG_ERR_TRAILING_DATA = 18         /* "bitrot shard file has trailing data", bitrot.rs:651 */
} rsg_status;

/* Bitrot hash selector (crates/utils/src/hash.rs:52-68). */
typedef enum rsg_hash_algo {
    RSG_HASH_NONE = 0,
    RSG_HASH_HIGHWAY256S = 1,        /* HashAlgorithm::HighwayHash256S (default), pi-derived key */
    RSG_HASH_HIGHWAY256S_LEGACY = 2  /* HashAlgorithm::HighwayHash256SLegacy, key [3,4,2,1] */
} rsg_hash_algo;

/* Reconstruct modes. */
typedef enum rsg_reconstruct_mode {
    /* ReedSolomonEncoder::reconstruct_data (erasure.rs:411-422): rebuild missing
     * data shards only; missing parity buffers are left untouched. */
    RSG_RECONSTRUCT_DATA = 0,
    /* reconstruct_opt (bridge.rs:296): rebuild every missing shard, data and parity. */
    RSG_RECONSTRUCT_MISSING = 1,
    /* ReedSolomonEncoder::reconstruct (erasure.rs:425-428): rebuild missing data,
     * then re-encode ALL parity shards from the data (present ones are overwritten). */
    RSG_RECONSTRUCT_REENCODE_PARITY = 2
} rsg_reconstruct_mode;

typedef struct rsg_ctx rsg_ctx;

/* ---- library / context ---- */
int rsg_abi_version(void);
const char *rsg_strerror(int status);
int rsg_device_count(int *count);
/* Create a context bound to HIP device `device`. */
int rsg_create(int device, rsg_ctx **out);
void rsg_destroy(rsg_ctx *ctx);

/* Measurement hook (no reference counterpart; bench.py): with timing on, the
 * record engines (rsg_decode_records_dev, rsg_heal_records_dev,
 * rsg_bitrot_verify_dev) record HIP events around their kernel launches on
 * the call's stream;
 * rsg_last_kernel_ms returns the summed kernel time of the last such call
 * (-1 if none was timed).  Off by default. */
int rsg_set_kernel_timing(rsg_ctx *ctx, int on);
int rsg_last_kernel_ms(rsg_ctx *ctx, float *ms);

/* Record-engine path of rsg_decode_records_dev / rsg_heal_records_dev (no
 * reference counterpart; tests and A/B runs).  AUTO (default): the one-pass
 * kernel from 1024 stripes where the geometry has one, else the two-pass
 * path; ONE_PASS / TWO_PASS force a path where the geometry allows it.  Both
 * paths produce identical bytes and statuses. */
typedef enum rsg_record_engine {
    RSG_RECORD_ENGINE_AUTO = 0,
    RSG_RECORD_ENGINE_ONE_PASS = 1,
    RSG_RECORD_ENGINE_TWO_PASS = 2
} rsg_record_engine;
int rsg_set_record_engine(rsg_ctx *ctx, int engine);

/* Kernel-choice knobs (no reference counterpart; ABI 6: tests and A/B runs).
 * The library runs its defaults; nothing in the process environment changes
 * them (the RSG_* variables are read only by measurement builds compiled with
 * RSG_MEASUREMENT_BUILD).  rsg_set_tuning(name, value) sets one knob for the
 * whole process (every context): value NULL = that knob's default, name NULL
 * = every knob's default; an unknown name or a value the knob does not take is
 * RSG_ERR_INVALID_ARG and changes nothing.  Launches already queued keep the
 * setting they were made with.  Every setting produces identical bytes and
 * statuses; only the kernel (and its speed) differs.  rsg_get_tuning writes
 * the knob's current value (NUL-terminated, at most cap bytes).  Knobs (value
 * syntax): RSG_FUSED, RSG_LOST_DISK_FAST, RSG_ZERO_COPY, RSG_ROLLED,
 * RSG_HASH_COPY, RSG_FUSED_SPW1, RSG_DECODE_NET, RSG_HASH_UNAL, RSG_GET_CACHED
 * (0|1); RSG_VEC_BLOCK (0|64|256); RSG_VEC_OCC (-1..8); RSG_HASH_DEPTH (1..3);
 * RSG_FUSED_KIND (auto|packed|ring|dma|wide2|wide4|split2|split4|net|table);
 * RSG_ENC_PRIO, RSG_DMA_PRIO, RSG_DMA_NT (0..3); RSG_DMA_EW (2|4);
 * RSG_DMA_SPW (4|8); RSG_NET12_RD (2; 4 only in measurement builds, whose
 * library carries that A/B kernel form).  INTEGRATION.md lists what each
 * selects. */
int rsg_set_tuning(const char *name, const char *value);
int rsg_get_tuning(const char *name, char *out, size_t cap);

/* Fault injection, tests only (no reference counterpart; ABI 5): sub-batch
 * `index` of every later rsg_encode_batch_host_submit on this context fails
 * to enqueue with RSG_ERR_DEVICE (-1, the default: never).  Lets the tests
 * check that a failing submit drains the sub-batches it had queued.  Nothing
 * else (no environment variable) can trigger it. */
int rsg_test_fail_subbatch(rsg_ctx *ctx, int index);

/* Encoding matrix ((k+m) x k, row-major) as reed_solomon_erasure::ReedSolomon::new
 * builds it (erasure.rs:448-470 cached_modern_reed_solomon).  Host only. */
int rsg_matrix(int k, int m, uint8_t *out);
/* Validate a geometry like Erasure::try_new_with_options (erasure.rs:708-773):
 * k > 0, k+m <= 256.  m == 0 is valid (no codec; encode is a no-op). */
int rsg_check_geometry(int k, int m);

/* ---- host-buffer API: drop-in for ReedSolomonEncoder (erasure.rs:358-446) ----
 * `shards` holds k+m host pointers of shard_len bytes each: k data then m parity. */

/* ReedSolomonEncoder::encode (erasure.rs:396-408): overwrite shards[k..k+m). */
int rsg_encode(rsg_ctx *ctx, int k, int m, size_t shard_len, uint8_t *const *shards);

/* ReedSolomonEncoder::reconstruct_data / reconstruct and reconstruct_opt
 * (erasure.rs:411-428, bridge.rs:295-301).  present[i] != 0 marks shard i valid;
 * every pointer must be a writable shard_len buffer; rebuilt shards are written
 * in place.  Fewer than k present -> RSG_ERR_TOO_FEW_SHARDS. */
int rsg_reconstruct(rsg_ctx *ctx, int k, int m, size_t shard_len, uint8_t *const *shards,
                    const uint8_t *present, int mode);

/* ReedSolomonEncoder::verify (erasure.rs:430-441): *ok = 1 when every parity
 * shard equals the parity re-encoded from the data shards. */
int rsg_verify(rsg_ctx *ctx, int k, int m, size_t shard_len, const uint8_t *const *shards, int *ok);

/* HashAlgorithm::hash_encode for the Highway variants (hash.rs:114-141). */
int rsg_hash(rsg_ctx *ctx, int algo, const uint8_t *data, size_t len, uint8_t out[32]);

/* ---- device-batch API: the batched GPU path (encode.rs:795-919 dispatch point) ----
 * d_stripes: device memory holding n stripes.  Stripe s, shard i starts at
 *   d_stripes + s*stripe_stride + i*shard_pitch   (a3 layout: shard_pitch = shard_len,
 *   stripe_stride = (k+m)*shard_len, erasure.rs:848-887).
 * stream: a hipStream_t; NULL = the HIP null (default) stream.  Calls are
 * asynchronous and ordered with other work on that stream. */

/* Encode parity for n stripes; if d_digests != NULL and algo != NONE also write
 * the (k+m) per-shard bitrot digests of every stripe, [n][k+m][32] — identical to
 * BitrotWriter::write's prefix (bitrot.rs:496-502) — in the same pass. */
int rsg_encode_batch_dev(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                         uint8_t *d_stripes, size_t shard_pitch, size_t stripe_stride,
                         uint8_t *d_digests, int algo, void *stream);

/* Reconstruct n stripes that share one erasure pattern `present` (k+m host bytes). */
int rsg_reconstruct_batch_dev(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                              uint8_t *d_stripes, size_t shard_pitch, size_t stripe_stride,
                              const uint8_t *present, int mode, void *stream);

/* Per-stripe parity check of n complete stripes: d_ok[s] = 1 if consistent. */
int rsg_verify_batch_dev(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                         const uint8_t *d_stripes, size_t shard_pitch, size_t stripe_stride,
                         uint8_t *d_ok, void *stream);

/* Hash n messages of len bytes each (message j at d_data + j*stride) into
 * d_out[n][32] (HashAlgorithm::hash_encode, hash.rs:114). */
int rsg_hash_batch_dev(rsg_ctx *ctx, int algo, const uint8_t *d_data, size_t len, size_t stride,
                       size_t n, uint8_t *d_out, void *stream);

/* DEPRECATED since ABI 6 (kept so ABI-4 bindings stay valid; nothing in this
 * repository calls it): use rsg_decode_records_into_dev, the form the
 * reference's GET has — write_data_blocks writes from the per-shard buffers
 * (decode.rs:1390), so copying every present data shard into one block buffer
 * is work the reference does not do, and at RS(12,4) this form runs at a third
 * of the HBM roofline (records 2 mod 8 copied to 8-aligned rows).
 * GET-side engine, batched, gather form (RustfsCodecDecodeEngine::reconstruct_into,
 * bridge.rs:274-307, with BitrotReader's verify-before-use, bitrot.rs:227-247).
 * Shard i of n stripes is resident on the device in BitrotWriter layout:
 * record s at d_files[i] + s*(32+shard_len) = [32-byte digest][shard_len bytes]
 * (d_files[i] == NULL: shard unavailable).  Every available record is hashed
 * and compared with its digest; a mismatching record counts as missing for
 * that stripe only.  The k data shards of stripe s are written contiguously to
 * d_out + s*k*shard_len (present ones copied, missing ones rebuilt from the
 * first k valid shards).  With verify_surplus, stripes that rebuilt data while
 * holding more than k valid shards re-derive the surplus parity and compare
 * (decode_data_with_reconstruction_verification, erasure.rs:935-973).
 * h_status[s] (host array): RSG_OK, RSG_ERR_TOO_FEW_SHARDS or
 * RSG_ERR_INCONSISTENT_SOURCES.  Synchronous. */
int rsg_decode_records_dev(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                           const uint8_t *const *d_files, int algo, int verify_surplus,
                           uint8_t *d_out, int *h_status, void *stream);

/* GET-side engine, in-place form (ABI 5): RustfsCodecDecodeEngine::reconstruct_into
 * (bridge.rs:274-307) fills only the None slots of its shards slice and skips a
 * stripe whose data shards are all present (data_shards_complete ->
 * skip_data_complete, bridge.rs:52-54); write_data_blocks then writes straight
 * from the per-shard buffers (decode.rs:1390).  Same sources, verification and
 * statuses as rsg_decode_records_dev, but a data shard whose record verifies is
 * served from that record (its body at d_files[i] + s*(32+shard_len) + 32) and
 * nothing is copied; only the shards no verified record serves — file absent or
 * record rotten — are rebuilt, into d_targets[i] + s*target_stride.
 * d_targets: k device slots, one per data shard, each at least
 * (n-1)*target_stride + shard_len bytes (target_stride >= shard_len;
 * target_stride = k*shard_len with d_targets[i] = base + i*shard_len gives the
 * contiguous block layout); a slot range overlapping a source record file, or
 * two slots with a stripe window in common (some s, s' with
 * [d_targets[i] + s*target_stride, +shard_len) and [d_targets[j] +
 * s'*target_stride, +shard_len) sharing a byte), is RSG_ERR_INVALID_ARG.  With every data file present the call only verifies
 * the k data records of each stripe (parity is read for a stripe only if one of
 * its data records is rotten).  h_src (host, optional, k*n bytes, [shard][stripe]):
 * 1 where data shard i of stripe s is served from its record, 0 where it was
 * written to its slot (unspecified for a failed stripe).  Synchronous. */
int rsg_decode_records_into_dev(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                                const uint8_t *const *d_files, int algo, int verify_surplus,
                                uint8_t *const *d_targets, size_t target_stride, uint8_t *h_src,
                                int *h_status, void *stream);

/* Asynchronous GET (ABI 5): either form — d_out (gather, deprecated as
 * rsg_decode_records_dev) or d_targets + target_stride (in place), exactly one
 * non-NULL — queued on `stream` with a
 * ticket returned at once, so a caller decoding many batches (decode.rs's
 * pipeline, decode.rs:1702-1968) overlaps one batch's status handling with the
 * next batch's kernels.  rsg_poll / rsg_wait complete it (the same tickets as
 * the host-batch PUT); h_status and h_src are filled when the ticket completes,
 * and every buffer must stay alive and unmodified (sources) / unread (outputs)
 * until then.  Each call uses its own scratch: calls from several threads run
 * concurrently.  Completion normally needs no further device work; a batch with
 * a rotten record is redone for the affected stripes inside the wait/poll that
 * completes it. */
int rsg_decode_records_submit(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                              const uint8_t *const *d_files, int algo, int verify_surplus,
                              uint8_t *d_out, uint8_t *const *d_targets, size_t target_stride,
                              uint8_t *h_src, int *h_status, void *stream, uint64_t *ticket);

/* Heal, batched (Erasure::heal, heal.rs:112-206, which calls
 * decode_data_and_parity, erasure.rs:917, per block).  Sources as in
 * rsg_decode_records_dev (d_files[i] == NULL: no reader; every record is
 * verified before use).  d_targets[i] != NULL marks shard i as a heal target
 * (a writer; a target range overlapping any source or another target is
 * RSG_ERR_INVALID_ARG): it receives n BitrotWriter records
 * [HH256S][shard_len bytes] (stride 32+shard_len) of the rebuilt shard i (data
 * shards as read/rebuilt, parity re-encoded), computed in one pass over the
 * survivors.  Every verified source parity is compared with the parity
 * re-encoded from the data (heal.rs:180-196).  d_work: unused since ABI 3
 * (may be NULL; kept so existing bindings stay valid).
 * h_status[s]: RSG_OK, RSG_ERR_TOO_FEW_SHARDS (ErasureReadQuorum) or
 * RSG_ERR_INCONSISTENT_SOURCES ("inconsistent heal source shards"); target
 * records of a failed stripe carry an all-zero digest header (they never
 * verify) and unspecified bodies.  Synchronous. */
int rsg_heal_records_dev(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                         const uint8_t *const *d_files, uint8_t *const *d_targets, int algo,
                         uint8_t *d_work, int *h_status, void *stream);

/* Asynchronous heal (ABI 5): rsg_heal_records_dev queued with a ticket, as
 * rsg_decode_records_submit (heal.rs's per-block loop, heal.rs:112-206, batched
 * and overlapped). */
int rsg_heal_records_submit(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n,
                            const uint8_t *const *d_files, uint8_t *const *d_targets, int algo,
                            int *h_status, void *stream, uint64_t *ticket);

/* Whole-shard-file bitrot verification (bitrot_verify, bitrot.rs:616-655) of
 * n_files device-resident shard files of one part (file f: file_lens[f]
 * bytes at d_files[f]).  want_size must equal
 * bitrot_shard_file_size(part_size, shard_size, algo) (else every file gets
 * RSG_ERR_FILE_SIZE_MISMATCH); then records are checked in order like the
 * reference's read loop: h_status[f] = RSG_ERR_BITROT_MISMATCH at the first
 * bad digest, RSG_ERR_UNEXPECTED_EOF if the file ends early,
 * RSG_ERR_TRAILING_DATA if it is longer than want_size, else RSG_OK.
 * algo: HIGHWAY256S / LEGACY (streaming records) or NONE (sizes only);
 * whole-file algorithms are RSG_ERR_UNSUPPORTED, as in the reference.
 * Synchronous. */
int rsg_bitrot_verify_dev(rsg_ctx *ctx, int algo, size_t n_files, const uint8_t *const *d_files,
                          const size_t *file_lens, size_t want_size, size_t part_size, size_t shard_size,
                          int *h_status, void *stream);

/* Block until all work queued on `stream` (NULL = the null stream) is done. */
int rsg_sync(rsg_ctx *ctx, void *stream);

/* ---- host-batch API: the PUT path starts and ends in host memory ----
 * Encode n stripes held in HOST memory (same addressing as the device-batch
 * API): sub-batches are pipelined over the context's stream/staging slots
 * (H2D data -> encode + fused digests -> D2H parity + digests).  This is the
 * batched replacement for encode_batched's per-block encode_data_block calls
 * (encode.rs:795-919); pin the buffers (rsg_pin or a pinned allocation) for
 * full PCIe bandwidth and for the copies to run asynchronously.  With m == 0
 * only the digests are computed; an empty shard hashes as the empty message.
 *
 * Asynchronous form: rsg_encode_batch_host_submit queues the job and returns
 * a ticket at once; jobs run in submission order and the sub-batches of
 * consecutive jobs overlap, so a producer reads and submits batch i+1 (and
 * writes batch i-1's shards) while the GPU encodes batch i — the bounded
 * in-flight queue of encode_batched (RUSTFS_ERASURE_ENCODE_MAX_INFLIGHT_BYTES,
 * encode.rs:64-72) with the caller choosing the bound.  h_stripes / h_digests
 * must stay alive and untouched until the ticket completes.
 * rsg_poll sets *done = 1 (and releases the ticket) when the job has finished,
 * returning its status; rsg_wait blocks until then.  An unknown or already
 * released ticket is RSG_ERR_INVALID_ARG.  Several threads may poll or wait
 * on one ticket; all of them see it finish.  If submit returns an error, no
 * ticket is issued and none of the job's copies is still in flight: the
 * sub-batches it had already queued are drained before it returns, so the
 * caller may reuse or free h_stripes / h_digests at once (their contents are
 * then unspecified).  rsg_encode_batch_host = submit + wait. */
int rsg_encode_batch_host(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n, uint8_t *h_stripes,
                          size_t shard_pitch, size_t stripe_stride, uint8_t *h_digests, int algo);
int rsg_encode_batch_host_submit(rsg_ctx *ctx, int k, int m, size_t shard_len, size_t n, uint8_t *h_stripes,
                                 size_t shard_pitch, size_t stripe_stride, uint8_t *h_digests, int algo,
                                 uint64_t *ticket);
int rsg_poll(rsg_ctx *ctx, uint64_t ticket, int *done);
int rsg_wait(rsg_ctx *ctx, uint64_t ticket);

/* Page-lock / release host memory for DMA (hipHostRegister). */
int rsg_pin(void *ptr, size_t bytes);
int rsg_unpin(void *ptr);

#ifdef __cplusplus
}
#endif
#endif /* RSGPU_H */
