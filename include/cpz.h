/*
 * cpz.h -- C ABI of the MI355X-native Chaum-Pedersen / ristretto255 batch verifier.
 *
 * Drop-in boundary for the reference's `verifier::batch::BatchVerifier`
 * (kobby-pentangeli/chaum-pedersen-zkp, src/verifier/batch.rs).  Plain C: caller-owned
 * buffers, structure-of-arrays inputs, no callbacks, no torch/HIP types in signatures.
 * Every entry point returns an int status (CPZ_OK = 0, < 0 on error) and never aborts;
 * cpz_last_error() describes the most recent failure on the calling thread.
 *
 * Input layout (per proof i, each field a 32-byte little-endian encoding):
 *   y1[i], y2[i]  Statement (gadgets.rs:177-239), compressed ristretto255 points
 *   r1[i], r2[i]  Commitment (gadgets.rs:245-265), compressed ristretto255 points
 *   s[i]          Response (gadgets.rs:272-286), canonical scalar bytes
 * i.e. the bytes [5..37), [41..73), [77..109) of `Proof::to_bytes` (gadgets.rs:343-361)
 * plus the statement encodings.  Optional per-proof transcript contexts
 * (`add_with_context`, batch.rs:144-168) are given as one byte blob plus n + 1 offsets;
 * ctx_present distinguishes Some(b"") from None (NULL = every entry Some).
 *
 * Per-proof status codes (uint8):
 *   CPZ_STATUS_OK               Ok(())
 *   CPZ_STATUS_EQ_FAIL          Err(InvalidParams("Proof verification failed"))  batch.rs:224-228
 *   CPZ_STATUS_BAD_POINT        a point fails to decode (InvalidGroupElement)    ristretto.rs:120-138
 *   CPZ_STATUS_BAD_SCALAR       s is not canonical (InvalidScalar)                ristretto.rs:94-112
 *   CPZ_STATUS_IDENTITY         r1 or r2 is the identity (InvalidParams            gadgets.rs:474-478
 *                               "Commitment contains identity element")
 *   CPZ_STATUS_ZERO_S           s is zero (InvalidParams "Response scalar is zero")  gadgets.rs:480-482
 * Codes 2-5 are rejected by the reference before an entry can reach the batch
 * (`Proof::from_bytes`, service.rs:501-507); the bulk path reports them per entry.
 */
#ifndef CPZ_H_
#define CPZ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPZ_OK 0
#define CPZ_EINVAL (-1)     /* bad argument (null pointer, n == 0 where forbidden, misalignment) */
#define CPZ_EHIP (-2)       /* HIP runtime / kernel failure */
#define CPZ_ENOMEM (-3)     /* device or host allocation failed */
#define CPZ_EGENERATOR (-4) /* g or h does not decode to a valid, non-identity, distinct pair */
#define CPZ_EEMPTY (-5)     /* "Cannot verify empty batch" (batch.rs:172-176) */

#define CPZ_STATUS_OK 0
#define CPZ_STATUS_EQ_FAIL 1
#define CPZ_STATUS_BAD_POINT 2
#define CPZ_STATUS_BAD_SCALAR 3
#define CPZ_STATUS_IDENTITY 4
#define CPZ_STATUS_ZERO_S 5

/* ABI revision of this header (cpz_abi_version): bumped whenever an entry point's signature or
 * an array size it writes changes, so that callers built against another header can refuse
 * to run instead of passing wrongly sized buffers.  3: CPZ_NUM_STAGES = 16,
 * cpz_ctx_stage_times_n, cpz_ctx_set_commitment_checks.  4: per-call flags (the _ex entry
 * points, CPZ_CALL_EQUATIONS_ONLY), stage 7 (generator tables), density probe with contexts.
 * 5: CPZ_FALLBACK_STATS = 8 (the partitioned check's locate pass). */
#define CPZ_ABI_VERSION 5

typedef struct cpz_ctx cpz_ctx;

/* The CPZ_ABI_VERSION the library was built with. */
int cpz_abi_version(void);

/* Number of visible GPUs (0 when none / no HIP runtime). */
int cpz_device_count(void);

/* Create a verifier context bound to one GPU (one HIP stream, cached generator tables,
 * reusable device buffers).  Contexts serialise concurrent calls internally. */
int cpz_ctx_create(int device_ordinal, cpz_ctx **out);
void cpz_ctx_destroy(cpz_ctx *ctx);

/* Commitment checks (default on): statuses 4 (identity r1 / r2) and 5 (zero s) are the
 * rejections Proof::from_bytes applies (gadgets.rs:474-482) before a proof can reach the
 * service's batch (service.rs:501-507).  A Proof built with Proof::new(Commitment::new(..),
 * Response::new(..)) (gadgets.rs:252, 278, 317) skips them, and the reference's verify_one
 * (batch.rs:185-231) / verify_with_transcript (verifier/mod.rs:120-171) judge it by the two
 * equations alone -- e.g. a nonce k = 0 gives r1 = r2 = identity and an accepted proof.
 * enable = 0 gives exactly that: identity commitments and zero s are not reported, the
 * equations decide (and such entries keep their RLC weight).  Applies to every later call
 * on the context, from any thread: callers that share a context and need the equations-only
 * mode for their own calls pass CPZ_CALL_EQUATIONS_ONLY to the _ex entry points instead. */
int cpz_ctx_set_commitment_checks(cpz_ctx *ctx, int enable);

/* Per-call flags of the _ex entry points (cpz_verify_each_ex, cpz_verify_batch_ex,
 * cpz_verify_response_ex): each behaves as its plain form with these options for that call
 * alone -- the context's own mode and other threads' calls are unaffected.
 *   CPZ_CALL_EQUATIONS_ONLY  commitment checks off for this call (as
 *                            cpz_ctx_set_commitment_checks(ctx, 0)): what verify_one does
 *                            with a Proof value (the mirrors of BatchVerifier / Verifier). */
#define CPZ_CALL_EQUATIONS_ONLY 1u

/* Thread-local description of the last error returned on this thread. */
const char *cpz_last_error(void);

/* Encodings of the default generators: g = ristretto255 basepoint, h = hash-to-group of
 * SHA-512("chaum-pedersen-zkp-v1.0.0-generator-h")   (ristretto.rs:27, 79-91). */
void cpz_default_generators(uint8_t g[32], uint8_t h[32]);

/* Per-proof verification of n proofs under generators (g, h).
 * Replaces BatchVerifier::verify (batch.rs:171-183) / verify_one (batch.rs:185-231):
 * status_out[i] is the outcome the reference reports for entry i.  Host buffers.
 * n == 0 -> CPZ_EEMPTY. */
int cpz_verify_each(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                    const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                    const uint8_t *s, const uint8_t *ctx_bytes, const uint64_t *ctx_off,
                    const uint8_t *ctx_present, uint8_t *status_out);
int cpz_verify_each_ex(cpz_ctx *ctx, uint32_t flags, const uint8_t g[32], const uint8_t h[32], size_t n,
                       const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                       const uint8_t *s, const uint8_t *ctx_bytes, const uint64_t *ctx_off,
                       const uint8_t *ctx_present, uint8_t *status_out);

/* Same with device-resident, 16-byte aligned inputs/outputs, enqueued on `stream`
 * (a hipStream_t, or NULL for the context's own stream, which is a blocking stream and so
 * is ordered with the legacy default stream).  Does not synchronise.  Any later call on the
 * same context, on any stream, is ordered after this call's kernels (they read the context's
 * cached tables and work buffers). */
int cpz_verify_each_device(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                           const void *d_y1, const void *d_y2, const void *d_r1, const void *d_r2,
                           const void *d_s, const void *d_ctx_bytes, const uint64_t *d_ctx_off,
                           const uint8_t *d_ctx_present, void *d_status_out, void *stream);

/* Fiat-Shamir challenges c_i (32-byte canonical scalars), bit-exact with
 * Transcript::challenge_scalar (transcript.rs:67-71) as built by batch.rs:188-206. */
int cpz_challenges(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                   const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                   const uint8_t *ctx_bytes, const uint64_t *ctx_off, const uint8_t *ctx_present,
                   uint8_t *c_out);

/* Per-proof verification with caller-supplied challenges c_i (32-byte little-endian scalars):
 * Verifier::verify_response (verifier/mod.rs:144-171) -- g^s == r1 y1^c and h^s == r2 y2^c,
 * no transcript.  status_out[i] as for cpz_verify_each: the entry's decode-level checks first
 * (2, 3 for s, 4, 5), then CPZ_STATUS_BAD_SCALAR if c_i is not canonical (c_i >= l: what
 * scalar_from_bytes would reject, ristretto.rs:94-112), then 0 / 1.  n == 0 -> CPZ_EEMPTY. */
int cpz_verify_response(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                        const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                        const uint8_t *s, const uint8_t *c, uint8_t *status_out);
int cpz_verify_response_ex(cpz_ctx *ctx, uint32_t flags, const uint8_t g[32], const uint8_t h[32], size_t n,
                           const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                           const uint8_t *s, const uint8_t *c, uint8_t *status_out);
int cpz_verify_response_device(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                               const void *d_y1, const void *d_y2, const void *d_r1, const void *d_r2,
                               const void *d_s, const void *d_c, void *d_status_out, void *stream);

/* Batch prover from caller witnesses x_i and nonces k_i (32-byte little-endian scalars, taken
 * mod l): Prover::prove_with_transcript (prover/mod.rs:86-110) with commit's nonce supplied
 * (commit :115-121, respond :126-131) and the statement from the witness (gadgets.rs:217-221):
 *   y1 = x g, y2 = x h, r1 = k g, r2 = k h, c = the transcript challenge (optional per-proof
 *   contexts as in cpz_verify_each, appended first as the service does), s = k + c x.
 * Outputs are n x 32-byte encodings.  n == 0 -> CPZ_EEMPTY. */
int cpz_prove(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t *x,
              const uint8_t *k, const uint8_t *ctx_bytes, const uint64_t *ctx_off, const uint8_t *ctx_present,
              uint8_t *y1, uint8_t *y2, uint8_t *r1, uint8_t *r2, uint8_t *s);
int cpz_prove_device(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const void *d_x,
                     const void *d_k, const void *d_ctx_bytes, const uint64_t *d_ctx_off,
                     const uint8_t *d_ctx_present, void *d_y1, void *d_y2, void *d_r1, void *d_r2, void *d_s,
                     void *stream);

/* Synthetic input generator (Prover::prove_with_transcript, prover/mod.rs:86-131):
 * witness x_i and nonce k_i = from_bytes_mod_order_wide(ChaCha20(seed_x / seed_k, block
 * first_index + i)); writes y1 = x g, y2 = x h, r1 = k g, r2 = k h, s = k + c x. */
int cpz_prove_synthetic(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                        uint64_t first_index, const uint8_t seed_x[32], const uint8_t seed_k[32],
                        const uint8_t *ctx_bytes, const uint64_t *ctx_off, const uint8_t *ctx_present,
                        uint8_t *y1, uint8_t *y2, uint8_t *r1, uint8_t *r2, uint8_t *s);
int cpz_prove_synthetic_device(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                               uint64_t first_index, const uint8_t seed_x[32], const uint8_t seed_k[32],
                               const void *d_ctx_bytes, const uint64_t *d_ctx_off,
                               const uint8_t *d_ctx_present, void *d_y1, void *d_y2, void *d_r1,
                               void *d_r2, void *d_s, void *stream);

/* Random-linear-combination batch verification (configs C3-C5): one Pippenger MSM checks
 *   P = sum_i [a_i s_i] g - [a_i] r1_i - [a_i c_i] y1_i + [b_i s_i] h - [b_i] r2_i - [b_i c_i] y2_i == O
 * -- the reference's verify_batch_equations (batch.rs:271-312) with the equation corrected
 * (the reference omits alpha on y*c, batch.rs:297-300).  Weights replace random_scalar
 * (batch.rs:240): the (first_index + i)-th ChaCha20 keystream block of `seed` read as 32
 * little-endian int16 words w_k; a_i = sum_{k<8} w_k 2^(16k), b_i = sum_{k<8} w_(8+k) 2^(16k)
 * (mod l) -- 128-bit weights, uniform over 2^128 values each (error <= 2^-128 per forged
 * entry), whose MSM digits are the words themselves.
 *   partial_out  32-byte encoding of P for this batch / shard (identity = 32 zero bytes);
 *                shards with global first_index values sum to the single-GPU P.
 *   batch_ok     1 iff every entry decodes and P is the identity.
 *   status_out   optional (n): exact per-entry statuses.  When the batch fails, a fallback
 *                search (sub-range RLC partials, per-proof verification at the leaves)
 *                locates the invalid entries (verify_individually, batch.rs:314-318).
 *                With a fallback, a batch of >= 2^20 entries (with or without contexts) is
 *                first sampled (4096 entries verified per proof, beside the batch's challenges):
 *                if two or more sampled entries are invalid the batch cannot pass and
 *                bisection could not prune it.  2 to 20 sampled invalid entries (density
 *                up to ~0.5 %): the partitioned check -- every 128-proof block's own RLC
 *                partial, then for the failing blocks an index-weighted second partial that
 *                locates a block's single invalid entry, per-proof verification of the
 *                located entries and of the blocks holding more; partial_out is the batch's
 *                partial as usual.  More: nothing is prepared, every entry is verified per
 *                proof, batch_ok = 0 and partial_out is 32 bytes of 0xff (not an encoding:
 *                "no partial computed").
 *   seed         must be secret and unpredictable to whoever produced the proofs (a CSPRNG
 *                draw per call, as the reference's random_scalar(rng) is, batch.rs:240): the
 *                weights' 2^-128 bound per forged entry, and the locate pass's ~2^-121 per
 *                failing block (CPZ_FALLBACK_STATS out[7]), hold only for weights the prover
 *                could not predict.  A seed an adversary knows lets forgeries cancel.
 * The _device form takes device-resident inputs and always needs d_status_out (decode-level
 * statuses, or exact ones when fallback != 0); it synchronises `stream`. */
int cpz_verify_batch(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                     const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                     const uint8_t *s, const uint8_t *ctx_bytes, const uint64_t *ctx_off,
                     const uint8_t *ctx_present, const uint8_t seed[32], uint64_t first_index,
                     uint8_t partial_out[32], int *batch_ok, uint8_t *status_out);
int cpz_verify_batch_ex(cpz_ctx *ctx, uint32_t flags, const uint8_t g[32], const uint8_t h[32], size_t n,
                        const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                        const uint8_t *s, const uint8_t *ctx_bytes, const uint64_t *ctx_off,
                        const uint8_t *ctx_present, const uint8_t seed[32], uint64_t first_index,
                        uint8_t partial_out[32], int *batch_ok, uint8_t *status_out);
int cpz_verify_batch_device(cpz_ctx *ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                            const void *d_y1, const void *d_y2, const void *d_r1, const void *d_r2,
                            const void *d_s, const void *d_ctx_bytes, const uint64_t *d_ctx_off,
                            const uint8_t *d_ctx_present, const uint8_t seed[32], uint64_t first_index,
                            uint8_t partial_out[32], int *batch_ok, void *d_status_out, int fallback,
                            void *stream);

/* What the last cpz_verify_batch[_device] call on the context did to locate invalid entries
 * (fallback != 0), for tests and benchmarks:
 *   out[0]  path: CPZ_FALLBACK_NONE (the batch passed, or no fallback), _BISECTION (sub-range
 *           RLC partials, per-proof leaves: a failed batch below 2^19 proofs), _PARTITIONED
 *           (every 128-proof block's partial, the failing blocks' index-weighted partials,
 *           per-proof verification of the located entries and of the blocks not located: the
 *           density probe's moderate densities, and a failed batch of 2^19 proofs or more),
 *           _PER_PROOF (dense: everything)
 *   out[1]  invalid entries the density probe saw (0 without a probe)
 *   out[2]  blocks whose partial the partitioned check computed
 *   out[3]  blocks whose partial was not the identity
 *   out[4]  entries the fallback verified per proof
 *   out[5]  sub-range MSMs the bisection ran
 *   out[6]  failing blocks whose index-weighted partial the locate pass computed
 *   out[7]  of those, blocks whose one invalid entry it located (verified alone; the rest of
 *           such a block is accepted on P'_b = [j] P_b, error <= ~2^-121 per block for a seed
 *           the proofs' author could not predict -- see `seed` above; with a known seed an
 *           adversary could place two related forgeries in one block that pass as one) */
#define CPZ_FALLBACK_STATS 8
#define CPZ_FALLBACK_NONE 0
#define CPZ_FALLBACK_BISECTION 1
#define CPZ_FALLBACK_PARTITIONED 2
#define CPZ_FALLBACK_PER_PROOF 3
int cpz_ctx_fallback_stats(cpz_ctx *ctx, uint64_t out[CPZ_FALLBACK_STATS]);

/* Bulk Ristretto255::element_from_bytes (ristretto.rs:120-138) on the device: ok_out[i] = 1 iff
 * the 32-byte encoding points[i] decodes (RFC 9496), and, when reencoded_out is not NULL, the
 * element_to_bytes (ristretto.rs:141-143) encoding of the decoded point (32 zero bytes where
 * it does not decode).  Statement registration (service.rs:82-86) and parity checks use it. */
int cpz_decode_points(cpz_ctx *ctx, size_t n, const uint8_t *points, uint8_t *ok_out, uint8_t *reencoded_out);

/* Multi-scalar multiplication through the same Pippenger kernels: out = enc(sum_j [k_j] P_j)
 * for n encoded points and n scalars (little-endian, < 2^253), n <= 2^24 - 3 (CPZ_EINVAL above).
 * Exposed for testing the MSM against the oracle with adversarial digit patterns. */
int cpz_msm(cpz_ctx *ctx, size_t n, const uint8_t *points, const uint8_t *scalars, uint8_t out[32]);

/* Sum k 32-byte partials (per-GPU shards) on the device: out = encoding of the sum,
 * *is_identity = 1 iff the combined batch equation holds.  A partial of 32 x 0xff (a shard
 * whose fallback skipped its MSM, cpz_verify_batch) makes out 32 x 0xff and *is_identity 0:
 * the batch cannot pass.  CPZ_EINVAL if a partial does not decode. */
int cpz_combine_partials(cpz_ctx *ctx, size_t k, const uint8_t *partials, uint8_t out[32], int *is_identity);

/* Bulk wire-format ingestion: Proof::from_bytes (gadgets.rs:364-489) for n
 * 109-byte-format blobs at blob[off[i] .. off[i+1]), on the device.  Writes the r1, r2, s rows
 * (n x 32 B SoA, zero where not parsed) and one CPZ_PARSE_* code per blob -- the first check
 * the reference would fail, in its order (each field's structure, then its decode
 * element_from_bytes / scalar_from_bytes, before the next field; trailing bytes; identity
 * commitment; zero s).  aux_out (optional) holds the value the reference's message prints
 * (length, version or trailing-byte count).  Entries with a non-zero code are rejected before
 * batching, as the service does (service.rs:501-507). */
#define CPZ_PARSE_OK 0
#define CPZ_PARSE_TOO_SMALL 1        /* InvalidParams "Proof too small: {aux} bytes" */
#define CPZ_PARSE_BAD_VERSION 2      /* InvalidParams "Unsupported proof version: {aux}" */
#define CPZ_PARSE_R1_LEN_MISSING 3   /* InvalidParams "Truncated proof: missing r1 length" */
#define CPZ_PARSE_R1_LEN_INVALID 4   /* InvalidParams "Invalid r1 length: {aux}" */
#define CPZ_PARSE_R1_TRUNCATED 5     /* InvalidParams "Truncated proof: incomplete r1 data" */
#define CPZ_PARSE_R1_SIZE 6          /* InvalidGroupElement "Expected 32 bytes, got {aux}" */
#define CPZ_PARSE_R1_POINT 7         /* InvalidGroupElement "Bytes do not represent a valid Ristretto point" */
#define CPZ_PARSE_R2_LEN_MISSING 8   /* as 3..7 for r2 */
#define CPZ_PARSE_R2_LEN_INVALID 9
#define CPZ_PARSE_R2_TRUNCATED 10
#define CPZ_PARSE_R2_SIZE 11
#define CPZ_PARSE_R2_POINT 12
#define CPZ_PARSE_S_LEN_MISSING 13   /* InvalidParams "Truncated proof: missing s length" */
#define CPZ_PARSE_S_LEN_INVALID 14   /* InvalidParams "Invalid s length: {aux}" */
#define CPZ_PARSE_S_TRUNCATED 15     /* InvalidParams "Truncated proof: incomplete s data" */
#define CPZ_PARSE_S_SIZE 16          /* InvalidScalar "Expected 32 bytes, got {aux}" */
#define CPZ_PARSE_S_SCALAR 17        /* InvalidScalar "Bytes do not represent a valid scalar" */
#define CPZ_PARSE_TRAILING 18        /* InvalidParams "Proof has {aux} trailing bytes" */
#define CPZ_PARSE_IDENTITY 19        /* InvalidParams "Commitment contains identity element" */
#define CPZ_PARSE_ZERO_S 20          /* InvalidParams "Response scalar is zero" */
int cpz_parse_proofs(cpz_ctx *ctx, size_t n, const uint8_t *blob, const uint64_t *off, uint8_t *r1_out,
                     uint8_t *r2_out, uint8_t *s_out, uint8_t *code_out, uint32_t *aux_out);
int cpz_parse_proofs_device(cpz_ctx *ctx, size_t n, const void *d_blob, const uint64_t *d_off, void *d_r1,
                            void *d_r2, void *d_s, void *d_code, void *d_aux, void *stream);

/* Single-process multi-GPU forms: one context per GPU (e.g. the 8 GPUs of a node, or
 * several contexts on one GPU), the n proofs cut into nctx contiguous shards whose
 * boundaries are multiples of 256 proofs (the RLC weight-block granule), each shard
 * verified by its own context on its own host thread -- what a single host process behind
 * BatchVerifier::verify (batch.rs:171-183) uses instead of one process per GPU.
 *   cpz_verify_each_multi   per-proof statuses for all n (no data exchange).
 *   cpz_verify_batch_multi  per-shard RLC partials (weights keyed by the GLOBAL index, so
 *                           they sum to the single-GPU partial) -> partials_out (nctx x 32,
 *                           identity for an empty shard), combined on ctxs[0] ->
 *                           total_out; batch_ok = 1 iff every entry decodes and the sum is
 *                           the identity; status_out (optional, n) exact per entry, failing
 *                           shards running their own fallback search.
 * Contexts are given in shard order; the first failing shard's error is returned (its
 * message via cpz_last_error on the calling thread). */
int cpz_verify_each_multi(cpz_ctx *const *ctxs, int nctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                          const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                          const uint8_t *s, const uint8_t *ctx_bytes, const uint64_t *ctx_off,
                          const uint8_t *ctx_present, uint8_t *status_out);
int cpz_verify_batch_multi(cpz_ctx *const *ctxs, int nctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                           const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                           const uint8_t *s, const uint8_t *ctx_bytes, const uint64_t *ctx_off,
                           const uint8_t *ctx_present, const uint8_t seed[32], uint8_t *partials_out,
                           uint8_t total_out[32], int *batch_ok, uint8_t *status_out);

/* Per-kernel timing (HIP events recorded on the launch stream around every kernel).
 * Stages: 0 = k_challenge, 1 = k_verify_each, 2 = RLC decode/weights, 3 = RLC MSM,
 * 4 = fallback, 5 = the whole per-proof verify of one call (first to last k_verify_each,
 * whose launches overlap on several streams), 6 = prover (commitments / statements, then
 * challenges + responses), 7 = generator tables (a (g, h) pair's combs and transcript prefix
 * built: a cache miss, one launch each; a context keeps the tables of its 4 most recently used
 * pairs, or of CPZ_GEN_CACHE = 1..4 set in the environment when it is created, and frees the
 * others when a new pair's combs do not fit); phases of the RLC MSM (inside stage 3): 8 = bucket
 * sort, 9 = bucket accumulation (k_rlc_bucket), 10 = bucket fix-up, 11 = bucket reduction
 * (segment + window), 12 = window combine + encode (k_rlc_final16); 13 = variable-base generator
 * tables (a per-proof call of at most 16384 proofs on a pair other than the default one and
 * without combs in the cache builds only the pair's Niels tables and transcript prefix, ~0.5 ms
 * instead of ~3 ms, and verifies [s'] g, [s'] h from them; a context keeps 64 such pairs);
 * phases of the partitioned check (inside stage 3): 14 = every block's bucket walk
 * (k_part_acc), 15 = the locate pass's walk over the failing blocks.
 * cpz_ctx_stage_times synchronises, writes the summed milliseconds and launch counts per stage
 * since the last call, and resets them. */
#define CPZ_NUM_STAGES 16
int cpz_ctx_set_timing(cpz_ctx *ctx, int enable);
int cpz_ctx_stage_times(cpz_ctx *ctx, double ms_out[CPZ_NUM_STAGES], int launches_out[CPZ_NUM_STAGES]);
/* The same for the first nstages stages only (arrays of nstages entries; launches_out may be
 * NULL): callers built against a header with another CPZ_NUM_STAGES pass their own size. */
int cpz_ctx_stage_times_n(cpz_ctx *ctx, int nstages, double *ms_out, int *launches_out);

#ifdef __cplusplus
}
#endif

#endif /* CPZ_H_ */
