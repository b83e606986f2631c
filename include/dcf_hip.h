/*
 * dcf_hip.h — C ABI of the MI355X (gfx950) DCF evaluator.
 *
 * Drop-in boundary for the hot path of the `dcf` crate (xymeng16/dcf v0.2.2):
 * the `Dcf<N, LAMBDA>` operator (lib.rs:24-35) implemented by `DcfImpl`
 * (lib.rs:63-205) over the `Aes256HirosePrg` plugin (prg.rs:22-74).  Every
 * entry point is plain C: pointers, sizes, int status codes.  A Rust crate binds
 * it with `extern "C"` declarations (INTEGRATION.md shows the stub).
 *
 * Conventions
 *   n_bytes   `N` of `Dcf<N, LAMBDA>` / `CmpFn<N, LAMBDA>` (lib.rs:39): domain
 *             size in bytes; the tree has n = 8 * n_bytes levels (lib.rs:93).
 *   lambda    `LAMBDA` (lib.rs:40): seed and output size in bytes; must be a
 *             multiple of 16 (prg.rs:17-18).
 *   party     `b` of `Dcf::eval` (lib.rs:34): 0 = false, 1 = true.
 *   bound     `BoundState` (lib.rs:342-349): 0 = LtBeta, 1 = GtBeta.
 *   seeds     `Share::s0s` (lib.rs:278).  gen takes both; eval takes the one the
 *             reference reads, `k.s0s[0]` (lib.rs:168), as `s0`.
 *
 * Key layout ("correction-word block", CWB) for K keys, n = 8 * n_bytes
 * (replaces `Share { cws: Vec<Cw>, cw_np1 }`, lib.rs:208-214 and 275-283),
 * structure-of-arrays so a wave reads one level of 64 keys coalesced:
 *   offset 0                 cw_s  [n][K][lambda]   Cw::s
 *   offset n*K*lambda        cw_v  [n][K][lambda]   Cw::v
 *   offset 2*n*K*lambda      cw_t  [n][K]  u8       bit0 = Cw::tl, bit1 = Cw::tr
 *   offset dcf_cwb_np1_offset cw_np1[K][lambda]     Share::cw_np1
 * (the cw_np1 offset is 2*n*K*lambda + n*K rounded up to 16).  K = 1 is the
 * single-key layout.  Size: dcf_cwb_bytes().
 *
 * Errors: the reference panics where this ABI returns a code —
 *   DCF_ERR_KEY      assert_eq!(k.cws.len(), N * 8)           lib.rs:165
 *   DCF_ERR_CIPHER_N self.ciphers[i * 16 + j] out of range     prg.rs:51
 *   DCF_ERR_LEN      xs.len() != ys.len() (the reference silently truncates
 *                    via zip, lib.rs:196-198)
 * Nothing aborts the process.
 *
 * Memory: `*_device` entry points take device pointers and a hipStream_t (as
 * void*, NULL = the legacy default stream) and are asynchronous; the library
 * keeps no reference to caller buffers once the stream has passed the call.
 * Host entry points take host pointers and are synchronous: they run on three
 * streams the dcf_prg owns (copy-in, compute, copy-out) through pinned staging
 * buffers pooled on the dcf_prg, in chunks whose PCIe copies overlap the
 * kernels of neighbouring chunks, and they wait for those streams only (never
 * the whole device).  The GPU never reads or writes caller host memory.
 *
 * Threading (the reference's `Dcf::eval(&self, ...)` over a `Prg: Sync`, lib.rs:34,52):
 * every compute entry point may be called on ONE dcf_prg from any number of host
 * threads at once, and its device calls may be queued on different streams at once.
 * Each call leases a workspace (work counter, scratch, shared-prefix table, host
 * streams and staging) from a pool on the prg, so concurrent calls share no mutable
 * buffer; a workspace re-used on another stream first waits (on the device, with an
 * event) for the device work of its previous call, so a host call queued after a
 * *_device call on the same prg is ordered after it without any synchronization by the
 * caller.  The pool grows to the number of calls in flight at once and is freed with
 * the prg (dcf_prg_workspaces, dcf_prg_device_bytes, dcf_prg_host_pinned_bytes report
 * it).  The setters (dcf_prg_set_*) may race calls: a call reads each setting once.
 * Multi-GPU: one dcf_prg per device (all built from the same keys) and
 * dcf_eval_multi_gpu / _device below, or one process per device; the path shards by
 * points/keys with no collective.
 */
#ifndef DCF_HIP_H
#define DCF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCF_OK 0
#define DCF_ERR_ARG -1        /* null pointer, bad enum */
#define DCF_ERR_LAMBDA -2     /* lambda == 0 or lambda % 16 != 0 (prg.rs:17-18) */
#define DCF_ERR_CIPHER_N -3   /* too few ciphers for lambda (reference panics, prg.rs:51) */
#define DCF_ERR_N -4          /* n_bytes == 0 */
#define DCF_ERR_LEN -5        /* length mismatch (reference truncates, lib.rs:196) */
#define DCF_ERR_HIP -6        /* HIP runtime error; see dcf_last_error() */
#define DCF_ERR_UNSUPPORTED -7 /* shape not implemented by any kernel */
#define DCF_ERR_KEY -8        /* malformed key (lib.rs:165) */

#define DCF_BOUND_LT_BETA 0
#define DCF_BOUND_GT_BETA 1

/* AES engine for LAMBDA = 16 eval (dcf_prg_set_eval_mode); results are identical.  Values 2, 3
 * and 5 (bitsliced, hybrid and stream-hybrid engines, rounds 1-4) are retired: every A/B measured
 * them slower than the stream engine (profiles/AB_LOG.md), and setting them returns DCF_ERR_ARG. */
#define DCF_EVAL_AUTO 0      /* library's choice: STREAM for one key or N <= 32, TTABLE for many keys at N > 32 */
#define DCF_EVAL_TTABLE 1    /* LDS T-table AES, lockstep walk (A and B every level), one lane per point */
#define DCF_EVAL_STREAM 4    /* LDS T-table AES, per-lane block scheduling: a right step encrypts B only */

/* Opaque: an Aes256HirosePrg (prg.rs:22-24) whose AES-256 schedules live on one
 * device, i.e. `DcfImpl::new(Aes256HirosePrg::new(keys))` (lib.rs:74, prg.rs:27). */
typedef struct dcf_prg dcf_prg;

/* Version string of this library. */
const char* dcf_version(void);

/* Last error message of the calling thread ("" if none). */
const char* dcf_last_error(void);

/* Aes256HirosePrg::<LAMBDA, CIPHER_N>::new(keys) (prg.rs:27-33) on `device`.
 * keys: cipher_n * 32 bytes.  Needs cipher_n >= 1 for lambda == 16 and
 * cipher_n >= 18 for lambda >= 32 (the diagonal zip reads ciphers 0 and 17,
 * prg.rs:48-51). */
int dcf_hirose_prg_new(const uint8_t* keys, size_t cipher_n, size_t lambda, int device, dcf_prg** out);
/* Aes128MatyasMeyerOseasPrg::<LAMBDA, CIPHER_N>::new(keys) on `device` — the PRG
 * BASELINE.json's north_star names; the reference crate has no such PRG, so the
 * definition is ours (parity UNPINNED by the reference; DESIGN.md §4 "MMO"):
 *   out_b[j] = AES128_{keys[b * LAMBDA/16 + j]}(seed_j) ^ seed_j for b = s_L, v_L,
 *   s_R, v_R and every 16-byte block j (one key per output and block: "multi-block
 *   MMO" at LAMBDA >= 32), t_L / t_R = Lsb0 bit 0 of byte 0 of s_L / s_R, then bit 0
 *   of byte LAMBDA-1 cleared in all four outputs (the Hirose convention of prg.rs:63-68).
 * keys: cipher_n * 16 bytes, cipher_n >= 4 * lambda / 16 (else DCF_ERR_CIPHER_N).
 * Every gen / eval / prg entry point below accepts either PRG (LAMBDA >= 32: no
 * shared-prefix table). */
int dcf_mmo_prg_new(const uint8_t* keys, size_t cipher_n, size_t lambda, int device, dcf_prg** out);

/* 0 = Aes256HirosePrg, 1 = Aes128MatyasMeyerOseasPrg, -1 = null. */
int dcf_prg_kind(const dcf_prg* prg);

void dcf_prg_free(dcf_prg* prg);
size_t dcf_prg_lambda(const dcf_prg* prg);

/* Select the AES engine used by eval at LAMBDA = 16 (DCF_EVAL_AUTO / _TTABLE / _STREAM; the
 * LAMBDA >= 32 head and the MMO PRG have one engine each and ignore it).  Tuning and test knob
 * only: every engine returns identical bytes. */
int dcf_prg_set_eval_mode(dcf_prg* prg, int mode);

/* Shared prefix for single-key eval at LAMBDA = 16 (Hirose PRG: stream engine, and the
 * automatic engine's small-batch path; Aes128MatyasMeyerOseasPrg: every
 * engine setting) and, per key, for the LAMBDA >= 32
 * stream head (bytes [0,32) of the walk and the t-vector rows, 80 B per node).
 * Every point's walk (lib.rs:174-189) passes through the node of the key's GGM
 * tree named by its first D bits, and that node's (s, v, t) depends on nothing
 * else, so eval expands the top D levels once (2^(D+1) AES blocks, 33 B per node,
 * as the full-domain eval does) and starts each point at level D from its node:
 * D fewer levels per point, identical output bytes.
 *   levels = -1: automatic (the default): D = log2(points) (Aes128MatyasMeyerOseasPrg:
 *                log2(points) - 1), at most 27 (LAMBDA >= 32: log2(points) - 1, at most
 *                22), none below 8; Hirose small batches (32768 < points < 2^19 on the
 *                pair walk): 18 below 2^18 points, 19 above (1.7e7 / 3.4e7 B with the build buffers), at most
 *                8N - 1; none for Aes128MatyasMeyerOseasPrg small batches or up to 32768 points;
 *   levels =  0: off;  levels > 0: that depth (capped at 28 (LAMBDA >= 32: 30) and
 *                at 8N - 1).
 * The table and its build buffers are one allocation of the call's workspace; they stay
 * resident on the prg (sized by the largest D used) until dcf_prg_trim / dcf_prg_free, and
 * dcf_prg_device_bytes counts them.  Bytes at depth D:
 *   Hirose, LAMBDA = 16:  32 * 2^D (rows) + the one-launch build's two node buffers,
 *                         2 * 33 * 2^(D-H) with H = min(4, D - 18) levels built depth-first
 *                         (33 * 2^D when D <= 18) — 4.85e9 B at D = 27 (2^28 points, the auto
 *                         cap), 2.42e9 at 26, 0.61e9 at 24 (C2);
 *   MMO, LAMBDA = 16:     2 * 33 * 2^D (level-by-level build, rows packed into one half) —
 *                         8.86e9 B at D = 27;
 *   LAMBDA >= 32:         160 * 2^D (80-B rows + the build's two node buffers) — 0.34e9 at 21.
 * Multi-key stream eval (LAMBDA = 16, >= 32 points per key, 8N > 6 levels):
 * each key's own top tree of depth 5 (32 rows of 32 B per key, 36 PRG calls per key)
 * unless levels = 0; if its buffer cannot be allocated the points walk from the root. */
int dcf_prg_set_prefix_levels(dcf_prg* prg, int levels);
/* The prefix depth D a dcf_eval* call of this shape would use (0 = none). */
int dcf_eval_prefix_levels(const dcf_prg* prg, size_t n_bytes, size_t num_keys, size_t points_per_key);
/* Keys per kernel launch of a LAMBDA = 16 multi-key stream eval (dcf_eval_multikey_device and
 * the host entry points with several keys): min(2^24, 2^31 / points_per_key, 2^30 / 8N), at
 * least 1 — the engine's point, work and CW-digest-row indices are 32-bit, so a larger call runs
 * as consecutive launches over whole keys.  Pure arithmetic (no device access). */
size_t dcf_eval_keys_per_launch(size_t n_bytes, size_t points_per_key);
/* Cap on the device memory the AUTOMATIC prefix depth may allocate (table + build
 * buffers, which stay resident on the prg until dcf_prg_trim / dcf_prg_free; sizes above):
 * the auto depth is lowered until they fit, and no table is built below depth 8.  0 = no cap
 * (the default: 4.85e9 B at the auto cap D = 27, Hirose LAMBDA = 16).  Forced depths ignore
 * it.  Output bytes never change. */
int dcf_prg_set_prefix_max_bytes(dcf_prg* prg, size_t max_bytes);
/* Device memory this dcf_prg currently holds (tables, prefix tables, scratch, staging, over
 * all of its workspaces). */
size_t dcf_prg_device_bytes(const dcf_prg* prg);
/* Pinned host memory this dcf_prg holds for the host-pointer entry points (per workspace: up
 * to two 128 MiB x + y chunks of the eval pipeline, sized to the largest call, a 1 MiB mapped
 * buffer for tiny calls and a mapped buffer of up to 64 MiB for mid-size evals: ~321 MiB per
 * workspace at most, one workspace per call in flight), kept until dcf_prg_trim / dcf_prg_free. */
size_t dcf_prg_host_pinned_bytes(const dcf_prg* prg);
/* Number of workspaces in the prg's pool (the most calls that were in flight at once). */
int dcf_prg_workspaces(const dcf_prg* prg);
/* Free every workspace no call holds right now (their device scratch, prefix tables, pinned
 * staging); calls in flight keep theirs.  The next call allocates afresh.  Returns the number
 * of workspaces freed. */
int dcf_prg_trim(dcf_prg* prg);

/* AES blocks the last eval call on this prg (the last one to return, from any thread)
 * encrypted for live points (LAMBDA = 16: the DCF_EVAL_STREAM engine;
 * LAMBDA >= 32: the stream head over all of the call's keys and passes; not counting a
 * shared-prefix table build, except the multi-key per-key top trees, whose blocks are
 * included), counted on the device; 0 for engines that do not count.
 * Measurement hook for the bench; call after the eval's stream has been synchronized.  0
 * before any eval; DCF_ERR_ARG while that call's workspace is leased by another call (the
 * hook never reads a workspace in use). */
int dcf_prg_last_eval_blocks(dcf_prg* prg, uint64_t* blocks);

/* Phase timing of eval calls (measurement hook, off by default).  When on, every eval call
 * records HIP events on its stream at entry, before its walk kernel(s) (after any shared-
 * prefix table, per-key top trees or CW digest/rows were built) and at the end.
 * dcf_prg_last_eval_phases reads the last eval call's split (call after synchronizing its
 * stream): prep_ms = table / digest preparation, walk_ms = the walk kernels, prefix_levels =
 * the shared-prefix depth it used (0 = none).  DCF_ERR_ARG if no timed eval has run, or while
 * that call's workspace is leased by another call. */
int dcf_prg_set_phase_timing(dcf_prg* prg, int on);
int dcf_prg_last_eval_phases(dcf_prg* prg, float* prep_ms, float* walk_ms, int* prefix_levels);

/* CWB layout helpers (see above). */
size_t dcf_cwb_bytes(size_t n_bytes, size_t lambda, size_t num_keys);
size_t dcf_cwb_np1_offset(size_t n_bytes, size_t lambda, size_t num_keys);

/* ---- host-pointer, synchronous (mirror Dcf::gen / Dcf::eval) ---- */

/* Dcf::gen (lib.rs:26-31, impl lib.rs:86-161) for one key.
 * alpha: n_bytes, beta / s0_0 / s0_1: lambda, cwb_out: dcf_cwb_bytes(n_bytes, lambda, 1). */
int dcf_gen(dcf_prg* prg, size_t n_bytes, const uint8_t* alpha, const uint8_t* beta, const uint8_t* s0_0,
            const uint8_t* s0_1, int bound, uint8_t* cwb_out);

/* Dcf::eval (lib.rs:34, impl lib.rs:163-204).  xs: m * n_bytes (x_i contiguous),
 * ys: m * lambda (overwritten, lib.rs:171).  cwb: one key, s0: k.s0s[0]. */
int dcf_eval(dcf_prg* prg, size_t n_bytes, int party, const uint8_t* cwb, size_t cwb_len, const uint8_t* s0,
             const uint8_t* xs, size_t m, uint8_t* ys, size_t ys_len);

/* Aes256HirosePrg::gen (prg.rs:42-73) for m seeds (test hook for PRG vectors).
 * seeds: m * lambda; out: m * (4 * lambda + 2) = s_l | v_l | s_r | v_r | t_l | t_r. */
int dcf_prg_gen(dcf_prg* prg, const uint8_t* seeds, size_t m, uint8_t* out);

/* ---- device-pointer, asynchronous on `stream` ---- */

/* Batched Dcf::gen: K independent keys, one GPU lane per key.
 * alpha: K * n_bytes, beta / s0_0 / s0_1: K * lambda (row k = key k),
 * cwb_out: dcf_cwb_bytes(n_bytes, lambda, K). */
int dcf_gen_batch_device(dcf_prg* prg, size_t n_bytes, size_t num_keys, const uint8_t* alpha, const uint8_t* beta,
                         const uint8_t* s0_0, const uint8_t* s0_1, int bound, uint8_t* cwb_out, void* stream);

/* Dcf::eval of one key over m points (x_i contiguous, n_bytes each). */
int dcf_eval_device(dcf_prg* prg, size_t n_bytes, int party, const uint8_t* cwb, const uint8_t* s0,
                    const uint8_t* xs, size_t m, uint8_t* ys, void* stream);

/* Dcf::eval for K keys x P points each: point j of key k is xs[k*P + j],
 * its output ys[k*P + j]; s0s: K * lambda (k.s0s[0] of each key). */
int dcf_eval_multikey_device(dcf_prg* prg, size_t n_bytes, size_t num_keys, size_t points_per_key, int party,
                             const uint8_t* cwb, const uint8_t* s0s, const uint8_t* xs, uint8_t* ys, void* stream);

/* ---- multi-GPU (one call drives G devices) ----
 * The reference spreads Dcf::eval over every host core inside one call (rayon,
 * lib.rs:194-199); these spread it over G GPUs.  prgs[g] is a dcf_prg on the
 * device that evaluates slice g; all G must be built from the same keys (and
 * kind, lambda) — checked, DCF_ERR_ARG otherwise — and be distinct.  Points are
 * split into G contiguous slices, slice g = dcf_point_slice(m, G, g): the first
 * m % G slices hold one extra point.  Every (key, point) is independent, so no
 * collective runs during evaluation. */

/* Contiguous slice [start, start + count) of `total` items for slice g of G. */
void dcf_point_slice(size_t total, size_t G, size_t g, size_t* start, size_t* count);

/* Dcf::eval (lib.rs:163-204) of one key over host buffers on G devices: slice g
 * of xs goes to prgs[g]'s device (one host thread per device, each running the
 * pipelined host path above) and its outputs land directly in the matching rows
 * of ys.  Synchronous; same arguments and errors as dcf_eval. */
int dcf_eval_multi_gpu(dcf_prg* const* prgs, size_t G, size_t n_bytes, int party, const uint8_t* cwb,
                       size_t cwb_len, const uint8_t* s0, const uint8_t* xs, size_t m, uint8_t* ys, size_t ys_len);

/* Device-resident variant.  cwb (cwb_len bytes) and s0 are HOST pointers: the key
 * is copied to every device once per call (the broadcast; 4.2 KB at N = LAMBDA =
 * 16).  xs[g] / ys[g]: ms[g] points / outputs on prgs[g]'s device; streams[g]:
 * that device's stream (streams may be NULL = each device's default stream).
 * gather_ys: NULL, or a buffer on prgs[0]'s device of (sum of ms) * lambda bytes
 * that receives every slice's outputs in slice order (hipMemcpyPeerAsync over
 * xGMI, queued on streams[g] after slice g's eval).  Asynchronous: the caller
 * synchronizes every streams[g] before reading ys or gather_ys. */
int dcf_eval_multi_gpu_device(dcf_prg* const* prgs, size_t G, size_t n_bytes, int party, const uint8_t* cwb,
                              size_t cwb_len, const uint8_t* s0, const uint8_t* const* xs, const size_t* ms,
                              uint8_t* const* ys, void* const* streams, uint8_t* gather_ys);

/* ---- key wire format (host only, no GPU) ----
 * `Share` as serialised by serde + bincode 1.x `bincode::serialize` (lib.rs:217-340;
 * Cargo.toml:44): little-endian, u64 length before every Vec, fields in
 * declaration order, bool = one byte 0/1:
 *   u64 |s0s|, |s0s| x (u64 lambda, lambda bytes)
 *   u64 8N,    8N x (u64 lambda, Cw.s, u64 lambda, Cw.v, u8 tl, u8 tr)
 *   u64 lambda, cw_np1
 * from_bincode writes the single-key CWB and the seeds; a Vec of the wrong
 * length (the reference's copy_from_slice panics, lib.rs:251), a bool byte > 1,
 * cws.len() != 8N (lib.rs:165), truncation or trailing bytes -> DCF_ERR_KEY. */
size_t dcf_share_bincode_bytes(size_t n_bytes, size_t lambda, size_t num_s0s);
int dcf_share_to_bincode(size_t n_bytes, size_t lambda, const uint8_t* cwb, const uint8_t* s0s, size_t num_s0s,
                         uint8_t* out, size_t out_len);
int dcf_share_from_bincode(size_t n_bytes, size_t lambda, const uint8_t* in, size_t in_len, uint8_t* cwb_out,
                           uint8_t* s0s_out, size_t max_s0s, size_t* num_s0s);

/* Full-domain eval: ys[x] = Dcf::eval(party, k, x) for every x in
 * [0, 2^(8N)), x read big-endian (Msb0, lib.rs:181) — i.e. the output of
 * dcf_eval_device over all points in increasing order.  ys: 2^(8N) * lambda
 * bytes.  At lambda = 16 the tree is expanded breadth-first (2 AES blocks per
 * leaf instead of 16N per point); N <= 4. */
int dcf_eval_full_domain_device(dcf_prg* prg, size_t n_bytes, int party, const uint8_t* cwb, const uint8_t* s0,
                                uint8_t* ys, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DCF_HIP_H */
