/* eg_hip.h — C ABI of the MI355X-native ElectionGuard group-operation library
 * (libeg_hip.so).  Plain pointers and sizes only; no torch / HIP types.
 *
 * This is the drop-in boundary for the batched 4096-bit modexp path of
 * JohnLCaron/electionguard-remote:
 *
 *   B1 — group layer.  The reference builds exactly one GroupContext, in
 *        KUtils.productionGroup()  (src/main/java/electionguard/util/KUtils.java:10-12),
 *        and moves elements across its wire boundary as fixed-width big-endian
 *        bytes: ElementModP = 512 B (src/main/proto/common.proto:6-10),
 *        ElementModQ = 32 B (common.proto:12-16), imported unchecked through
 *        new BigInteger(1, bytes) (src/main/java/electionguard/util/ConvertCommonProto.java:41-57)
 *        and exported with byteArray() (ConvertCommonProto.java:111-121).
 *        Every buffer here uses that layout: element i of a batch occupies bytes
 *        [512*i, 512*i+512) (or [32*i, 32*i+32) for exponents).
 *   B2 — trustee plugin.  DecryptingTrusteeIF.directDecrypt / compensatedDecrypt,
 *        implemented by RunRemoteDecryptingTrustee (:180-208, :217-247) and the
 *        client proxy RemoteDecryptingTrusteeProxy (:48-115): see eg_trustee_*.
 *
 * Semantics shared by all entry points (match java.math.BigInteger):
 *   - bases are reduced mod p (any 512-byte value is accepted, no subgroup check,
 *     as ConvertCommonProto.importElementModP does not check);
 *   - x^0 = 1 (including 0^0 = 1), 0^e = 0 for e > 0;
 *   - exponents are used as given (not reduced mod q);
 *   - outputs are canonical: 0 <= out < p, 512-byte big-endian.
 * Status: 0 = EG_OK; non-zero on error with a thread-local message from
 * eg_last_error().  No pointer is retained past a call except ctx / fixed-base
 * handles.  Calls on one ctx are serialised on the ctx's HIP stream (thread-safe
 * through an internal mutex); use one ctx per device.
 * Host-pointer entry points copy over PCIe; the *_dev variants take device
 * pointers (hipMalloc'd, e.g. torch CUDA tensors) and run asynchronously on the
 * ctx stream (eg_ctx_sync to wait).
 */
#ifndef EG_HIP_H
#define EG_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EG_OK 0
#define EG_ERR_ARG 1
#define EG_ERR_HIP 2
#define EG_ERR_NOMEM 3
#define EG_ERR_MODULUS 4
#define EG_ERR_STATE 5

#define EG_P_BYTES 512
#define EG_Q_BYTES 32

typedef struct eg_ctx eg_ctx;
typedef struct eg_fixed_base eg_fixed_base;

/* Thread-local description of the last error on this thread ("" if none). */
const char* eg_last_error(void);

/* Library / device info: writes a NUL-terminated string (arch, limb layout). */
int eg_version(char* buf, size_t len);

/* GroupContext construction — replaces productionGroup(LOW_MEMORY_USE, Mode4096)
 * (KUtils.java:10-12).  p must be odd, 2^4095 < p < 2^4096; q, g as in the group.
 * device = HIP device ordinal (one ctx per device; trustee processes pin one GPU). */
int eg_ctx_create(const uint8_t p_be[EG_P_BYTES], const uint8_t q_be[EG_Q_BYTES],
                  const uint8_t g_be[EG_P_BYTES], int device, eg_ctx** out);
int eg_ctx_destroy(eg_ctx* ctx);
int eg_ctx_sync(eg_ctx* ctx);
/* Kernel-level timing of the dominant kernel (k_pow, the windowed exponentiation):
 * between begin and end every k_pow launch on the ctx stream is bracketed by HIP
 * events; end synchronises and returns the summed device milliseconds, the
 * Montgomery operations those launches performed (multiplies + squarings), how
 * many of them were squarings (which use the symmetric-half schedule, 24,640
 * instead of 32,768 algorithmic 32-bit MACs), and the number of launches.
 * Any out pointer may be NULL. */
int eg_ctx_profile_begin(eg_ctx* ctx);
int eg_ctx_profile_end(eg_ctx* ctx, double* kernel_ms, double* mont_ops, double* squarings, int* launches);
/* Shader clock (GHz) the k_pow launches of the last profile_begin/end window ran at: the median
 * over workgroups of (s_memtime ticks / s_memrealtime ticks) x 100 MHz (eg_clock_median), with
 * the number of clock records used and dropped (unset, wrapped or out of range).  0 GHz when no
 * record was usable.  used / dropped may be NULL.  Instrumentation; no reference counterpart. */
int eg_ctx_profile_clock(eg_ctx* ctx, double* ghz, uint32_t* used, uint32_t* dropped);
/* The reduction behind it, a pure host function: recs = n pairs (shader ticks, 100 MHz real-time
 * ticks).  A record is dropped when a field is 0 or >= 2^62 (unset / wrapped), the real-time span
 * is under 10 us, or its ratio lies outside [0.5, 3.5] GHz; *ghz = median of the rest, or 0. */
int eg_clock_median(const uint64_t* recs, size_t n, double* ghz, uint32_t* used, uint32_t* dropped);
/* Fixed-base table for g (built at ctx creation) — accessor. */
eg_fixed_base* eg_ctx_g_table(eg_ctx* ctx);

/* Fiat-Shamir pre-image format of every hash this ctx computes (proof generation and
 * verification): "|" + "|".join(upper-case hex of each element) + "|", SHA-256, mod q.
 * The upstream format (electionguard-kotlin-multiplatform 1.0-SNAPSHOT hashElements) is not in
 * the container, so both candidate hex forms are offered:
 *   EG_HASH_FIXED_WIDTH (default): ElementModP as 1024 chars, ElementModQ as 64 (the wire widths,
 *                                  common.proto:6-16);
 *   EG_HASH_MINIMAL: the integer's even-length hex (leading zero bytes dropped, 0 -> "00"),
 *                    as electionguard-python 1.x's to_hex. */
#define EG_HASH_FIXED_WIDTH 0
#define EG_HASH_MINIMAL 1
int eg_ctx_set_hash_format(eg_ctx* ctx, int format);

/* The two other unpinned proof conventions (upstream 1.0-SNAPSHOT's are not in the container;
 * common.proto:23-28 pins only the field names "c" and "v"), switchable per context like the hex
 * form; every proof this ctx makes or checks (range, constant, trustee share) follows them:
 *   response: EG_RESPONSE_MINUS (default): v = u - c*x, checked as a = g^v X^c (eg_oracle.py);
 *             EG_RESPONSE_PLUS: v = u + c*x, checked as g^v = a X^c (ElectionGuard 1.0's spec form);
 *   preimage: the hashed elements after Q-bar --
 *     EG_PREIMAGE_MESSAGE_FIRST (default): (alpha, beta, a0, b0, a1, b1) / (A, B, a, b) / (pad, data, a, b, M);
 *     EG_PREIMAGE_COMMITMENTS_FIRST: (a0, b0, a1, b1, alpha, beta) / (a, b, A, B) / (a, b, pad, data, M);
 *     EG_PREIMAGE_WITH_KEY: the public key first, (K, alpha, beta, ...) / (K, A, B, a, b) /
 *                           (K_i, pad, data, a, b, M) with K_i = g^secret for a share.
 * tools/pin_format.py reports which combination (with the hex form) verifies a given record. */
#define EG_RESPONSE_MINUS 0
#define EG_RESPONSE_PLUS 1
#define EG_PREIMAGE_MESSAGE_FIRST 0
#define EG_PREIMAGE_COMMITMENTS_FIRST 1
#define EG_PREIMAGE_WITH_KEY 2
int eg_ctx_set_proof_format(eg_ctx* ctx, int response, int preimage);

/* Fixed-base radix table (PowRadix / acceleratePow; LOW_MEMORY_USE = 8-bit
 * windows).  window_bits in [4, 22]; table = ceil(256/w) * 2^w elements of 640 B
 * in HBM (w = 16: 671 MB, w = 22: 32 GB). */
int eg_fixed_base_create(eg_ctx* ctx, const uint8_t base_be[EG_P_BYTES], int window_bits,
                         eg_fixed_base** out);
int eg_fixed_base_destroy(eg_fixed_base* fb);

/* ElementModP.powP(ElementModQ), variable base: out[i] = base[i]^exp[i] mod p.  Up to one
 * element per SIMD (1,024 on MI355X) runs one element per wave, up to half a resident round
 * 16 lanes per element (latency shapes), larger batches on 8-lane groups. */
int eg_powp_batch(eg_ctx* ctx, const uint8_t* base_be, const uint8_t* exp_be,
                  uint8_t* out_be, size_t n);
/* Fixed-base powP (gPowP / accelerated K.powP): out[i] = base^exp[i] mod p. */
int eg_fb_pow_batch(eg_fixed_base* fb, const uint8_t* exp_be, uint8_t* out_be, size_t n);
/* Same two, device pointers (512 B / 32 B big-endian rows in HBM), asynchronous on
 * the ctx stream (eg_ctx_sync to wait): for callers that keep elements resident
 * across calls, e.g. the modexp-per-second microbenchmark. */
int eg_powp_batch_dev(eg_ctx* ctx, const uint8_t* d_base_be, const uint8_t* d_exp_be,
                      uint8_t* d_out_be, size_t n);
int eg_fb_pow_batch_dev(eg_fixed_base* fb, const uint8_t* d_exp_be, uint8_t* d_out_be, size_t n);
/* ElementModP.times: out[i] = a[i] * b[i] mod p. */
int eg_multp_batch(eg_ctx* ctx, const uint8_t* a_be, const uint8_t* b_be, uint8_t* out_be,
                   size_t n);
/* Iterable<ElementModP>.multP(): out[g] = prod_{k<len} elems[g*len + k] mod p
 * (tally accumulation, runAccumulateBallots — RunRemoteWorkflowTest.java:151). */
int eg_prod_reduce(eg_ctx* ctx, const uint8_t* elems_be, size_t groups, size_t len,
                   uint8_t* out_be);
/* ElementModP.multInv: out[i] = a[i]^-1 mod p (0 -> 0, as a^(p-2)). */
int eg_multinv_batch(eg_ctx* ctx, const uint8_t* a_be, uint8_t* out_be, size_t n);

/* ---- fused ballot verification + tally (Verifier(record, 11).verify() and
 * runAccumulateBallots — RunRemoteWorkflowTest.java:151,179-182) ----
 * Layout (all big-endian, ballot-major):
 *   cts    : nballots * nsel * 2 * 512   (pad alpha, data beta) per selection
 *   rproof : nballots * nsel * 4 * 32    (c0, v0, c1, v1)       per selection
 *   cproof : nballots * ncontest * 2 * 32 (c, v)                per contest
 * Selections are contest-major; contest k owns selections [k*spc, (k+1)*spc)
 * (placeholders last: the tally skips the last `placeholders` of each contest).
 * K_be = joint election key, qbar_be = extended base hash, limit = votesAllowed.
 * cast (may be NULL = every ballot cast): nballots bytes, 0 = spoiled.  Every ballot is
 * verified; only cast ballots enter the tally (runAccumulateBallots sums cast ballots, the
 * spoiled ones are decrypted individually, RunRemoteDecryptor.java:264-269).
 * Outputs: ok_sel[nballots*nsel], ok_contest[nballots*ncontest] (1 = valid),
 * tally_be[ncontest*(spc-placeholders)*2*512] (may be NULL; all ones for no cast ballot).
 * A contest's verdict includes the validity of its message (A, B) = (prod alpha, prod beta),
 * decided from its selections: every alpha and beta must be in range and a valid residue
 * (x^q = 1).  This is a deliberate, documented choice: a contest whose
 * selections hold two non-residue alphas with a residue product is REJECTED here, while a check
 * of A^q = 1 alone would accept its constant proof; the ballot's verdict is the same either way
 * (the selections fail), and the oracles apply the same rule (tests/test_gpu_golden.py,
 * test_gpu_rejects_contest_whose_selections_are_invalid).
 * The key is set under the ctx lock for the call (a matching table is reused; a different K
 * rebuilds it at the window width of the ctx's current table, see eg_set_election_key). */
int eg_verify_ballots(eg_ctx* ctx, const uint8_t K_be[EG_P_BYTES], const uint8_t qbar_be[EG_Q_BYTES],
                      size_t nballots, size_t ncontest, size_t spc, size_t placeholders,
                      uint32_t limit, const uint8_t* cts, const uint8_t* rproof,
                      const uint8_t* cproof, const uint8_t* cast, uint8_t* ok_sel, uint8_t* ok_contest,
                      uint8_t* tally_be);
/* Builds K's fixed-base radix table (window_bits in [4, 22]; g's table follows the width) once,
 * so later calls with the same K only compare it. */
int eg_set_election_key(eg_ctx* ctx, const uint8_t K_be[EG_P_BYTES], int window_bits);
/* Same as eg_verify_ballots, device pointers (d_cast may be NULL), asynchronous on the ctx stream. */
int eg_verify_ballots_dev(eg_ctx* ctx, const uint8_t K_be[EG_P_BYTES], const uint8_t qbar_be[EG_Q_BYTES],
                          size_t nballots, size_t ncontest, size_t spc, size_t placeholders, uint32_t limit,
                          const uint8_t* d_cts, const uint8_t* d_rproof, const uint8_t* d_cproof,
                          const uint8_t* d_cast, uint8_t* d_ok_sel, uint8_t* d_ok_contest,
                          uint8_t* d_tally_be);

/* ---- batched encryption (batchEncryption, RunRemoteWorkflowTest.java:140-141) ----
 * Per selection: plaintext m (0/1), nonces (R, u, c_fake, v_fake) as 4*32 B.
 * Per contest: constant-proof nonce u (32 B).  Outputs cts / rproof / cproof in
 * the eg_verify_ballots layout.  K_be is set for the call as in eg_verify_ballots. */
int eg_encrypt_ballots(eg_ctx* ctx, const uint8_t K_be[EG_P_BYTES], const uint8_t qbar_be[EG_Q_BYTES],
                       size_t nballots, size_t ncontest, size_t spc, const uint8_t* votes,
                       const uint8_t* sel_nonces, const uint8_t* contest_nonces,
                       uint8_t* cts, uint8_t* rproof, uint8_t* cproof);
/* Constant-time encryption (on != 0): the fixed-base terms of eg_encrypt_ballots[_dev] read the
 * 6-bit radix tables of g and K (1.76 MB each, built once per key) with masked scans of every
 * window's 64 entries instead of indexing 22-bit tables by nonce digits, so neither the schedule
 * nor any address depends on a nonce or a vote (the commitments of both proof branches are
 * computed and put in order with masks in either mode).  The bytes are identical; the rate is
 * lower.  The trustee's kernels are always constant-time. */
int eg_ctx_set_ct_encrypt(eg_ctx* ctx, int on);
/* Same, device pointers (inputs and outputs resident in HBM); returns when the outputs
 * are written.  The votes (1 byte per selection) are read back to the host to build the
 * job tables (except in constant-time mode, eg_ctx_set_ct_encrypt); nonces and outputs never
 * leave the device. */
int eg_encrypt_ballots_dev(eg_ctx* ctx, const uint8_t K_be[EG_P_BYTES], const uint8_t qbar_be[EG_Q_BYTES],
                           size_t nballots, size_t ncontest, size_t spc, const uint8_t* d_votes,
                           const uint8_t* d_sel_nonces, const uint8_t* d_contest_nonces,
                           uint8_t* d_cts, uint8_t* d_rproof, uint8_t* d_cproof);

/* ---- trustee partial decryption (DecryptingTrusteeIF) ----
 * directDecrypt (RunRemoteDecryptingTrustee.java:189-193): per text i,
 *   M_i = pad_i^secret, proof (c, v) with a = g^u_i, b = pad_i^u_i,
 *   c = H(qbar, pad_i, data_i, a, b, M_i), v = u_i - c*secret mod q.
 * texts: n * 2 * 512 (pad, data); nonces: n * 32; out_M: n * 512; out_proof: n * 64 (c, v).
 * compensatedDecrypt uses the same kernel with secret = P_l(x_i). */
int eg_trustee_decrypt_batch(eg_ctx* ctx, const uint8_t secret_be[EG_Q_BYTES],
                             const uint8_t qbar_be[EG_Q_BYTES], const uint8_t* texts,
                             const uint8_t* nonces, size_t n, uint8_t* out_M, uint8_t* out_proof);
/* Share-proof verification (mediator side of Decryption.decrypt,
 * RunRemoteDecryptor.java:261-262): a = g^v K_i^c, b = pad^v M^c, check c. */
int eg_verify_shares(eg_ctx* ctx, const uint8_t qbar_be[EG_Q_BYTES], const uint8_t* Ki_be,
                     const uint8_t* texts, const uint8_t* M_be, const uint8_t* proof, size_t n,
                     uint8_t* ok);

/* ---- per-element calls, coalesced (upstream ElementModP.powP / times, GroupContext.gPowP and the
 * accelerated election key's K.powP, called element by element from 11 threads:
 * RunRemoteWorkflowTest.java:140-141,179-181, on the group of KUtils.java:10-12) ----
 * Every per-element call is a JOB:
 *   out = (bases[0] * ... * bases[nbases-1])^exp * fb0^e0 * fb1^e1  mod p
 * (exp NULL: exponent 1, the product itself; fb NULL: no fixed-base term; nbases = 0 with an exponent:
 * 1; nbases <= 16, eg_prod_reduce for longer products; fb0 / fb1 tables of this ctx, kept alive until
 * the ticket is waited).  eg_*_submit queues one job on the ctx's open batch and returns a ticket at
 * once; a dispatcher thread runs the batch as ONE launch of the per-wave job kernel (every mix of
 * kinds side by side; large batches of one plain kind on the throughput layouts) once the GPU is
 * free and the oldest job has waited its window, or as many jobs are queued as the previous batch
 * took, or max_batch jobs are queued.  The window is ADAPTIVE by default (half as long as the
 * previous batch ran, within [20 us, 100 us]); eg_ctx_set_coalescing(ctx, max_batch, window_us)
 * with window_us > 0 fixes it at exactly window_us, window_us = 0 restores the adaptive default
 * (EG_COALESCE_WINDOW_US=n in the environment also fixes it).  A job records eg_ctx_set_ct_pow's
 * setting when it is SUBMITTED and runs in that mode; a batch never mixes modes (a job of the other
 * mode closes the open batch, which is dispatched first).  The caller's out
 * must stay valid until eg_ticket_wait, which blocks until the result is in out, frees the ticket
 * and returns the batch's status.  eg_ctx_destroy first runs every queued job, and a ticket stays
 * waitable after it (each ticket must still be waited once, to free it); submits racing destroy fail
 * with EG_ERR_STATE.  eg_*_one = submit + wait.  Defaults: max_batch 16384, adaptive window.
 *   eg_powp_submit   : base^exp                    (ElementModP.powP)
 *   eg_gpowp_submit  : g^exp, g's table            (GroupContext.gPowP)
 *   eg_fb_pow_submit : base^exp over fb's table    (an accelerated element's powP: acceleratePow(),
 *                                                    e.g. the election key K.powP(R))
 *   eg_multp_submit  : a * b                       (ElementModP.times)
 *   eg_mexp_submit   : the general job, e.g. g^v * alpha^c in one job (fb0 = g's table, e0 = v,
 *                      bases = {alpha}, exp = c), or the contest aggregate (alpha_1 ... alpha_k)^c */
typedef struct eg_ticket eg_ticket;
int eg_ctx_set_coalescing(eg_ctx* ctx, size_t max_batch, uint32_t window_us);
int eg_mexp_submit(eg_ctx* ctx, const uint8_t* bases_be, size_t nbases, const uint8_t* exp_be, eg_fixed_base* fb0,
                   const uint8_t* e0_be, eg_fixed_base* fb1, const uint8_t* e1_be, uint8_t out_be[EG_P_BYTES],
                   eg_ticket** ticket);
int eg_powp_submit(eg_ctx* ctx, const uint8_t base_be[EG_P_BYTES], const uint8_t exp_be[EG_Q_BYTES],
                   uint8_t out_be[EG_P_BYTES], eg_ticket** ticket);
int eg_gpowp_submit(eg_ctx* ctx, const uint8_t exp_be[EG_Q_BYTES], uint8_t out_be[EG_P_BYTES], eg_ticket** ticket);
int eg_fb_pow_submit(eg_fixed_base* fb, const uint8_t exp_be[EG_Q_BYTES], uint8_t out_be[EG_P_BYTES],
                     eg_ticket** ticket);
int eg_multp_submit(eg_ctx* ctx, const uint8_t a_be[EG_P_BYTES], const uint8_t b_be[EG_P_BYTES],
                    uint8_t out_be[EG_P_BYTES], eg_ticket** ticket);
int eg_ticket_wait(eg_ticket* ticket);
int eg_mexp_one(eg_ctx* ctx, const uint8_t* bases_be, size_t nbases, const uint8_t* exp_be, eg_fixed_base* fb0,
                const uint8_t* e0_be, eg_fixed_base* fb1, const uint8_t* e1_be, uint8_t out_be[EG_P_BYTES]);
int eg_powp_one(eg_ctx* ctx, const uint8_t base_be[EG_P_BYTES], const uint8_t exp_be[EG_Q_BYTES],
                uint8_t out_be[EG_P_BYTES]);
int eg_gpowp_one(eg_ctx* ctx, const uint8_t exp_be[EG_Q_BYTES], uint8_t out_be[EG_P_BYTES]);
int eg_fb_pow_one(eg_fixed_base* fb, const uint8_t exp_be[EG_Q_BYTES], uint8_t out_be[EG_P_BYTES]);
int eg_multp_one(eg_ctx* ctx, const uint8_t a_be[EG_P_BYTES], const uint8_t b_be[EG_P_BYTES],
                 uint8_t out_be[EG_P_BYTES]);

/* Constant-time exponentiation for secret exponents (on != 0), e.g. a trustee's share s_i or P_l(x_i)
 * through the per-element API (RunRemoteDecryptingTrustee.java:189-193,227-232, where the L1 group
 * context hands the trustee's powP to this library; SURVEY §7 "secret exponents"):
 *   - variable-base terms (eg_powp_batch[_dev], the per-element jobs) use a fixed 4-bit window,
 *     4 squarings + 1 multiply per nibble whatever its value, every window-table read a masked scan
 *     of all 16 entries (no sliding window, no early exit on leading zero bits);
 *   - fixed-base terms (eg_fb_pow_batch[_dev], gPowP, fb jobs) multiply in every radix window (no
 *     zero-digit skip), each entry a masked scan of the window's whole column; a table wider than
 *     8 bits gets a 6-bit companion table for this (built once per table, 1.76 MB).
 * The schedule and every address are then independent of the exponent; the results are identical.
 * eg_multinv_batch's public exponent p - 2 keeps the variable-time schedule.  The batch trustee
 * entry (eg_trustee_decrypt_batch) is always constant-time.  Default off. */
int eg_ctx_set_ct_pow(eg_ctx* ctx, int on);

/* ---- device memory on the ctx's device (no reference counterpart: it lets a caller keep ballots
 * resident in HBM through this library alone, so its process runs ONE HIP runtime; bench.py) ----
 * Copies are ordered after every call queued on the ctx before them and return when complete;
 * eg_dev_free waits for the ctx stream first.  eg_all_nonzero_dev: *all = 1 iff every one of the
 * n flags (e.g. eg_verify_ballots_dev's d_ok_sel) is non-zero. */
int eg_dev_alloc(eg_ctx* ctx, size_t bytes, void** d_out);
int eg_dev_free(eg_ctx* ctx, void* d);
int eg_memcpy_htod(eg_ctx* ctx, void* d_dst, const void* src, size_t bytes);
int eg_memcpy_dtoh(eg_ctx* ctx, void* dst, const void* d_src, size_t bytes);
int eg_memset_dev(eg_ctx* ctx, void* d, int value, size_t bytes);
int eg_all_nonzero_dev(eg_ctx* ctx, const uint8_t* d_flags, size_t n, int* all);

/* ---- multi-GPU tally exchange (ballots sharded over the node's GPUs, one process
 * per GPU, partial tallies all-gathered over RCCL/xGMI and folded mod p on one GPU; the
 * reference's RunRemoteWorkflowTest.java:151 accumulates the whole tally in one process) ----
 * RCCL (librccl.so.1, dlopen'd on first use) runs on the ctx's stream and HIP runtime.
 * eg_comm_unique_id: rank 0 makes the 128-byte id, the caller distributes it (any host channel);
 * eg_comm_init: every rank calls it with the same id (collective); one communicator per ctx.
 * eg_comm_all_valid: *all_ok = min over ranks of local_ok (the verdict all-reduce).
 * eg_tally_allgather_fold: every rank passes nparts partial tallies of n elements (d_parts_be,
 * nparts x n x 512 B big-endian in HBM); root receives out_be[k] = product over every rank and
 * part of element k mod p (n x 512 B, host; may be NULL on the other ranks).  One ncclAllGather
 * plus the k_prod tree on root's GPU.  Without eg_comm_init it folds the local parts alone.
 * Deadlines: the communicator is non-blocking; eg_comm_init, every collective's enqueue AND its
 * completion (a hipEvent behind it, polled with ncclCommGetAsyncError) wait at most EG_COMM_TIMEOUT_S
 * seconds (default 300).  On expiry or an asynchronous error the communicator is aborted
 * (ncclCommAbort), the call returns EG_ERR_HIP, and the context stays FAILED: eg_comm_all_valid and
 * eg_tally_allgather_fold then return EG_ERR_STATE (never a fold of the local parts alone) until
 * eg_comm_destroy or eg_comm_init resets it. */
#define EG_COMM_ID_BYTES 128
int eg_comm_unique_id(uint8_t id[EG_COMM_ID_BYTES]);
int eg_comm_init(eg_ctx* ctx, const uint8_t id[EG_COMM_ID_BYTES], int world, int rank);
int eg_comm_destroy(eg_ctx* ctx);
int eg_comm_all_valid(eg_ctx* ctx, int local_ok, int* all_ok);
/* What the communicator reports about itself (ncclCommCount / ncclCommUserRank): *nranks = ranks of
 * the ctx's RCCL communicator and *rank this one's; both 0 when eg_comm_init was never called (a world
 * of one folds locally, without RCCL).  Either pointer may be NULL. */
int eg_comm_info(eg_ctx* ctx, int* nranks, int* rank);
int eg_tally_allgather_fold(eg_ctx* ctx, const uint8_t* d_parts_be, size_t nparts, size_t n, int root,
                            uint8_t* out_be);

#ifdef __cplusplus
}
#endif
#endif /* EG_HIP_H */
