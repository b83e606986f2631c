// dcf_hip.hip — MI355X (gfx950, CDNA4) DCF evaluator: HIP kernels + C ABI.
//
// Replaces the hot path of the `dcf` crate (xymeng16/dcf v0.2.2):
//   DcfImpl::eval  (lib.rs:163-204)   -> k_eval16 (one lane per (key, point))
//   DcfImpl::gen   (lib.rs:86-161)    -> k_gen16  (batched; a lane quad or one lane per key)
//   Aes256HirosePrg::gen (prg.rs:42-73) inlined into both (hirose16)
// The C ABI is declared in include/dcf_hip.h.  No CPU fallback: every compute
// entry point runs a kernel or returns an error.
//
// AES-256 on CDNA4 (no AES instructions): T-table rounds with the four 1 KiB
// tables replicated 32 ways in LDS so that lane l of every 32-lane half-wave
// always reads bank l (ds_read_b32 banks are (addr/4) mod 32 per half-wave,
// MI355X_MICROARCH.md §LDS) — conflict-free for any data.  Layout (128 KiB):
//   addr(T, b, lane) = (T>>1)*64K + b*256 + (T&1)*128 + (lane&31)*4
// so one v_perm_b32 builds the address from the state byte and a per-lane
// constant: byte0 = lane slot (T even: (l&31)*4, T odd: 128+(l&31)*4),
// byte1 = state byte b, byte2 = 64K half select.  One VALU op + one LDS read
// per lookup; 16 lookups per round.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <utility>
#include <vector>

#include "dcf_hip.h"

#define DCF_VERSION "dcf_amd 0.2.0 (gfx950)"

#include "aes_lds.h"
#include "kernels16.h"
#include "kernels_lat.h"
#include "kernels_wide.h"
#include "kernels_stream.h"
#include "kernels_mmo.h"
#include "kernels_mmo_wide.h"
#include "kernels_wide_stream.h"

namespace {

// ------------------------------------------------------------------------
// Host plumbing
// ------------------------------------------------------------------------
thread_local std::string t_err;

int fail(int code, const std::string& msg) {
  t_err = msg;
  return code;
}

// On failure the runtime's per-thread last error is cleared as well, so a later call on
// this thread does not report a stale error (e.g. an OOM) from its own launch check.
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      (void)hipGetLastError();                                                          \
      return fail(DCF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));        \
    }                                                                                   \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) return;
    ok = (prev == dev) || (hipSetDevice(dev) == hipSuccess);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (ok && hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

uint64_t grid_for(uint64_t work_items, int cus) {
  uint64_t blocks = (work_items + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)cus;  // one 128 KiB-LDS workgroup per CU, persistent loop
  if (blocks > cap) blocks = cap;
  return blocks ? blocks : 1;
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) { return hipMalloc(&p, n ? n : 1); }
};

}  // namespace

constexpr size_t kCtrBytes = 16;  // d_ctr: work counter (u32), then the stream engine's block count (u64)

// Per-call mutable state of a dcf_prg (the reference's `Dcf::eval(&self, ...)` is reentrant and
// its PRG is `Sync`, lib.rs:34,52: one DcfImpl may be shared by many threads).  Every compute
// entry point leases one workspace from the prg's pool for its duration, so concurrent calls
// on one prg — from several host threads, or device calls queued on different streams — never
// share a buffer.  The pool is LIFO, so a single caller keeps reusing one workspace whose
// buffers have already grown.  Device calls return before their kernels finish: the lease
// records `done` on the caller's stream, and the next lease of this workspace on another
// stream waits for that event on the device (hipStreamWaitEvent) before touching a buffer.
struct Workspace {
  uint32_t* d_ctr = nullptr;  // work counter / device-counted AES blocks (dcf_prg_last_eval_blocks)
  uint8_t* d_ws = nullptr;    // stream-ordered scratch (LAMBDA >= 32 paths, full domain)
  size_t ws_bytes = 0;
  uint8_t* d_dig = nullptr;   // LAMBDA >= 32 stream head: compact CW digest of the current key
  uint32_t dig_levels = 0;
  uint8_t* d_kdig = nullptr;  // LAMBDA = 16 multi-key stream eval: key-major CW digest
  size_t kdig_bytes = 0;
  uint8_t* d_pfx = nullptr;   // shared-prefix table + its build buffers / per-key top trees
  size_t pfx_bytes = 0;
  uint8_t* d_mkey = nullptr;  // dcf_eval_multi_gpu_device: this device's copy of the key (CWB + s0)
  size_t mkey_bytes = 0;
  uint32_t* d_tctr = nullptr; // LAMBDA >= 32 paired-slot tail with LDS-filling tables: per-workgroup block counters
  size_t tctr_bytes = 0;
  // Host-pointer entry points: three non-blocking streams (copy-in, compute, copy-out), their
  // events and staging (pinned host + device), grown on demand and kept.
  hipStream_t hs[3] = {nullptr, nullptr, nullptr};
  hipEvent_t hev[6] = {};     // in[2], kernel[2], out[2] (double-buffered chunks)
  uint8_t* h_stage = nullptr; // pinned
  size_t h_stage_bytes = 0;
  uint8_t* d_stage = nullptr;
  size_t d_stage_bytes = 0;
  uint8_t* h_tiny = nullptr;  // small host calls: pinned, device-mapped, coherent (read/written by the kernel)
  size_t tiny_bytes = 0;
  uint8_t* h_mid = nullptr;   // mid-size host evals: pinned, device-mapped, coarse-grained (x in, y out)
  size_t mid_bytes = 0;
  // Ordering of the device work of successive leases (see above).
  hipEvent_t done = nullptr;
  hipStream_t done_stream = nullptr;
  // Multi-key LAMBDA = 16 eval: a second stream for the per-key top trees, built while the
  // key-major digest is written on the call's stream (fork / join events).
  hipStream_t aux = nullptr;
  hipEvent_t aux_ev[2] = {};
  bool pending = false;
  uint32_t host_streams = 0;  // hs[] the current host call queued work on (bit i = hs[i])
  // dcf_prg_set_phase_timing: events around the last eval's preparation and walk kernels.
  hipEvent_t tev[3] = {};
  bool timed = false;
  uint32_t last_prefix = 0;
};

struct dcf_prg {
  int kind = 0;               // 0: Aes256HirosePrg (prg.rs), 1: Aes128MatyasMeyerOseasPrg (kernels_mmo.h)
  int device = 0;
  int cus = 256;
  size_t lambda = 0;
  size_t cipher_n = 0;
  std::vector<RoundKeys> rk;  // Aes256::new per key (prg.rs:28-31)
  uint4* d_rk128 = nullptr;   // MMO: AES-128 schedules (4 * LAMBDA/16 x 11 round keys)
  size_t rk128_count = 0;     // ... how many
  uint4* d_rk2 = nullptr;     // LAMBDA >= 32 stream head: AES-256 schedules of ciphers 0 and 17
  uint4* d_rk0 = nullptr;     // LAMBDA = 16 stream eval: AES-256 schedule of cipher 0 (15 x 16 B)
  uint32_t* d_tab = nullptr;  // T0..T3 (4 KiB) on the device
  std::vector<uint8_t> key_blob;  // the PRG keys as given (multi-GPU calls check every prg holds the same)
  // Settings (read once per call; atomics so a setter racing a call is not a data race).
  std::atomic<int> eval_mode{DCF_EVAL_AUTO};
  std::atomic<int> prefix_levels{-1};     // shared-prefix table depth: -1 auto, 0 off
  std::atomic<size_t> prefix_cap{0};      // dcf_prg_set_prefix_max_bytes (0 = none)
  std::atomic<int> timing{0};             // dcf_prg_set_phase_timing
  // Workspace pool (see Workspace).
  std::mutex pool_mu;
  std::vector<Workspace*> all_ws, free_ws;
  std::atomic<Workspace*> last_ws{nullptr};  // the workspace of the last eval call to return
};

namespace {

// The prg's settings as one call sees them: read once, when the call leases its workspace (the
// setters may race a call; no decision inside a call reads a setting twice).
struct Cfg {
  int mode, prefix_levels;
  size_t prefix_cap;
  bool timing;
};
Cfg snapshot(const dcf_prg* p) {
  return Cfg{p->eval_mode.load(), p->prefix_levels.load(), p->prefix_cap.load(), p->timing.load() != 0};
}

// A workspace leased for one call.  `st` is the stream the call's device work is queued on
// (for host entry points: the workspace's own compute stream, set by host_lease()).
struct Lease {
  dcf_prg* p;
  const Cfg c;  // the call's settings
  Workspace* w = nullptr;
  hipStream_t st = nullptr;
  bool ordered = false;
  bool drained = false;  // a host call synchronized its streams: nothing left to order after
  Lease(dcf_prg* prg) : p(prg), c(snapshot(prg)) {
    {
      std::lock_guard<std::mutex> g(p->pool_mu);
      if (!p->free_ws.empty()) {
        w = p->free_ws.back();
        p->free_ws.pop_back();
      }
    }
    if (!w) {
      w = new Workspace();
      std::lock_guard<std::mutex> g(p->pool_mu);
      p->all_ws.push_back(w);
    }
  }
  // Queue the call's device work on `stream`, after this workspace's previous device work.
  int order(hipStream_t stream) {
    st = stream;
    ordered = true;
    if (w->pending && w->done_stream != st) {
      const hipError_t e = hipStreamWaitEvent(st, w->done, 0);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(DCF_ERR_HIP, std::string("hipStreamWaitEvent: ") + hipGetErrorString(e));
      }
    }
    return DCF_OK;
  }
  ~Lease() {
    if (drained) {
      w->pending = false;
    } else if (ordered) {
      if (!w->done) (void)hipEventCreateWithFlags(&w->done, hipEventDisableTiming);
      if (w->done && hipEventRecord(w->done, st) == hipSuccess) {
        w->done_stream = st;
        w->pending = true;
      } else {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(st);  // cannot order the next user: drain instead
        w->pending = false;
      }
    }
    std::lock_guard<std::mutex> g(p->pool_mu);
    p->free_ws.push_back(w);
  }
  Lease(const Lease&) = delete;
  Lease& operator=(const Lease&) = delete;
};

constexpr int kPrefixNoMem = -100;            // build_prefix: table allocation failed (internal)
constexpr uint64_t kWideChunk = 1ull << 22;   // points per head/tail pass (t-vector scratch 256 MiB at N <= 31)
// Points per LAMBDA >= 32 head/tail pass for t-vectors of tw words: kWideChunk up to N = 31 (16
// words), fewer for longer t-sequences so the scratch stays ~256 MiB.
uint64_t wide_chunk_points(uint32_t tw) {
  return std::max<uint64_t>(16384, kWideChunk * 16 / std::max<uint32_t>(tw, 16u));
}
constexpr uint64_t kGenChunk = 4096;          // keys per wide-gen launch (scratch 3*LAMBDA per key)
constexpr uint32_t kTailPts = 4096;          // points per tail workgroup (one table build each)

// Grow a workspace buffer to `need` bytes (contents not kept).  The old buffer may still be
// read by this workspace's earlier work on `st`, so that drains first.
int grow(uint8_t** buf, size_t* have, size_t need, hipStream_t st) {
  if (*have >= need) return DCF_OK;
  if (*buf) {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipFree(*buf));
    *buf = nullptr;
    *have = 0;
  }
  HIP_TRY(hipMalloc(buf, need));
  *have = need;
  return DCF_OK;
}

int ensure_ws(Workspace* w, size_t bytes, hipStream_t st) { return grow(&w->d_ws, &w->ws_bytes, bytes, st); }

int ensure_ctr(Workspace* w) {
  if (!w->d_ctr) HIP_TRY(hipMalloc(&w->d_ctr, kCtrBytes));
  return DCF_OK;
}

// Phase timing (dcf_prg_set_phase_timing): event i of the lease's workspace on its stream.
void phase_mark(dcf_prg*, Lease& L, int i) {
  if (!L.c.timing) return;
  Workspace* w = L.w;
  if (!w->tev[i] && hipEventCreate(&w->tev[i]) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  if (hipEventRecord(w->tev[i], L.st) != hipSuccess) (void)hipGetLastError();
  if (i == 0) w->timed = false;
  if (i == 2) w->timed = true;
}

// Workgroups of the single-launch table builds (k_prefix_build16, k_wpfx_build): 2^S
// subtrees under level S, each expanded by one workgroup.
uint32_t prefix_split(uint32_t levels) { return levels > 18u ? 8u : (levels > 10u ? levels - 10u : 0u); }

// Depth-first tail of k_prefix_build16: the last H <= kPfxDfsMax levels, once the workgroup's
// level holds at least one node per thread (2^10 = kBlock).
// Full-domain eval: the last kFdTail levels in registers, depth-first (k_fd_dfs16; 5 levels:
// 128 VGPRs + scratch spills), the levels above by one k_prefix_build16 launch.
constexpr uint32_t kFdTail = 4;
uint32_t prefix_dfs_levels(uint32_t levels, uint32_t S) {
  const uint32_t cap = kPfxDfsMax;
  return levels >= S + 10u + 1u ? std::min<uint32_t>(cap, levels - S - 10u) : 0u;
}

// Shared-prefix depth for a single-key stream eval of `total` points (kernels_stream.h
// PrefixTable): the top tree has 2^D nodes (33 B each, built with 2^(D+1) AES blocks)
// and saves every point D levels.  Auto: D = log2(total) - 1 (table build < 1 block per
// point; Hirose: log2(total)), at most kPrefixMax = 27 (a 4.3 GB table of 32-B rows beside 0.55 GB of build
// buffers since r06; prefix_table_bytes), none below 8, always < 8N.  If the buffers cannot be
// allocated in auto mode, eval retries 2 levels shallower down to 8, then runs without a
// table (identical bytes; see try_prefix).  Measured (r01i, C2: 2^24 points, N = 4):
// D = 12 / 16 / 20 / 24 -> 2.00 / 2.29 / 2.62 / 2.83 G evals/s (1.44 without);
// C3 (2^28, N = 16): D = 16 / 24 / 26 -> 450 / 477 / ~482 M (397 M without; r01q/r).
// auto cap.  C3 sweeps (2^28 points): r01q 24 519, 25 521, 26 524, 27 524 M evals/s; r05y (today's
// walk, 2 runs, ms per step) 25 495.5 / 495.5, 26 491.6 / 492.0, 27 489.3 / 488.8, 28 488.9 / 488.8
constexpr uint32_t kPrefixMax = 27;
constexpr uint32_t kPrefixMaxForced = 28;  // dcf_prg_set_prefix_levels (Hirose 9.7 GB, MMO 2^28 x 33 B x 2 = 17.7 GB)
// Nodes per workgroup region of k_prefix_build16's two ping-pong buffers (log2): the widest
// level a workgroup writes there.  With a depth-first tail of H levels the breadth-first part
// stops at level D - H, so that is 2^(D-H-S) nodes (at D = 27: 553 MB of buffers beside the
// 4.3 GB table, r06; it was 2^(D-1-S), 4.4 GB); without one the last level goes straight to
// the table and the widest buffered level is D - 1.
uint32_t prefix_region_log2(uint32_t d, uint32_t S) {
  const uint32_t H = prefix_dfs_levels(d, S);
  return d - std::max<uint32_t>(H, 1u) - S;
}

// Device bytes of a shared-prefix table of depth d (table + build buffers, as build_prefix /
// build_wide_prefix allocate them).
size_t prefix_table_bytes(const dcf_prg* p, uint32_t d) {
  if (d == 0) return 0;
  const uint32_t S = prefix_split(d);
  if (p->lambda > 16) return (((size_t)80 << d) + 255) + 2 * ((size_t)80 << (d - 1u));
  if (p->kind == 1) return 2 * ((((size_t)33 << d) + 255) & ~(size_t)255) + 256;
  return ((((size_t)32 << d) + 255) & ~(size_t)255) +
         2 * ((size_t)1 << S) * ((((size_t)33 << prefix_region_log2(d, S)) + 255) & ~(size_t)255);
}

// Auto depth under the dcf_prg_set_prefix_max_bytes cap: shallower until it fits (none below 8).
uint32_t capped_depth(const dcf_prg* p, const Cfg& c, uint32_t d) {
  if (!c.prefix_cap) return d;
  while (d >= 8u && prefix_table_bytes(p, d) > c.prefix_cap) --d;
  return d >= 8u ? d : 0u;
}

uint32_t prefix_depth(const dcf_prg* p, const Cfg& c, size_t n_bytes, uint64_t num_keys, uint64_t total) {
  if (p->lambda != 16 || num_keys != 1 || c.prefix_levels == 0) return 0;
  uint32_t d;
  if (c.prefix_levels > 0) {
    d = std::min((uint32_t)c.prefix_levels, kPrefixMaxForced);
  } else {
    // Hirose (one-launch build, k_prefix_build16): D = log2(total), r02g sweep C2 (2^24
    // points) D = 22/23/24/25 -> 3.97/4.08/4.13/3.93 G evals/s; MMO (level kernels): log2 - 1
    const uint32_t lg = 63u - (uint32_t)__builtin_clzll(total | 1u);
    d = p->kind == 0 ? lg : (lg > 1u ? lg - 1u : 0u);
    if (d < 8u) return 0;
    d = std::min(d, kPrefixMax);
    d = capped_depth(p, c, std::min<uint32_t>(d, (uint32_t)(8 * n_bytes - 1)));
  }
  return std::min<uint32_t>(d, (uint32_t)(8 * n_bytes - 1));
}

// Tiny batches run the latency kernels of kernels_lat.h (thresholds below and at kEvalRowMax).
#ifndef DCF_EVAL_OCT_MAX
#define DCF_EVAL_OCT_MAX 32768
#endif
constexpr uint64_t kEvalOctMax = DCF_EVAL_OCT_MAX;  // points (one key) up to which auto-mode eval runs k_eval16_oct
                                         // (r03a, us per device call: 32768 oct 187 vs pair 273; 100k 623 vs 485)
bool oct_eval(const dcf_prg* p, const Cfg& c, size_t n_bytes, uint64_t num_keys, uint64_t total) {
  return p->kind == 0 && p->lambda == 16 && num_keys == 1 && total <= kEvalOctMax && 8 * n_bytes <= kColMaxLevels &&
         c.prefix_levels <= 0 && c.mode == DCF_EVAL_AUTO;
}

// Shared-prefix depth for the small-batch pair path (k_eval16_pair: one key, fewer points than
// two per lane of the GPU, more than the latency kernels take).  Forced: dcf_prg_set_prefix_levels.
// Auto: 18 below 2^18 points, 19 from there (at most 8N - 1; none below 8 or up to kEvalOctMax
// points) — the build is one
// launch of k_prefix_build16 (row-AES root path, depth-first tail) whose blocks cost far less than
// the walk's latency-bound levels they save.  r06 sweep (one key, both parties, ms per step;
// `scripts/c1_prefix_sweep.sh`, profiles/r06/r06v_*): N = 16 100k points 0.895 without a table,
// 0.851 / 0.850 / 0.860 at D = 17 / 18 / 19; 250k 1.878 vs 1.704 at 18; 500k 3.736 vs 3.299 at 19;
// N = 4 100k 0.249 vs 0.200 at 18, 400k 0.966 vs 0.530 at 19; N = 8 100k 0.464 vs 0.413 at 18.
// (Round 3 measured no gain at D = 14-16 on C1, before the build's row-AES root path and
// depth-first tail.)
uint32_t small_prefix_depth(const dcf_prg* p, const Cfg& c, size_t n_bytes, uint64_t total) {
  if (p->lambda != 16 || p->kind != 0 || c.prefix_levels == 0) return 0;
  const uint32_t cap = (uint32_t)(8 * n_bytes - 1);
  if (c.prefix_levels > 0) return std::min<uint32_t>(std::min((uint32_t)c.prefix_levels, kPrefixMaxForced), cap);
  // none up to kEvalOctMax points: the latency kernels walk from the root there, and at N > 32 (the
  // pair walk) a table's fixed build latency would cost more than a few thousand points save
  if (total <= kEvalOctMax) return 0;
  const uint32_t lg = 63u - (uint32_t)__builtin_clzll(total | 1u);
  const uint32_t d = capped_depth(p, c, std::min<uint32_t>(lg < 18u ? 18u : 19u, cap));
  return d >= 8u ? d : 0u;
}

// Shared-prefix depth for the LAMBDA >= 32 stream head over m points of one key
// (kernels_wide_stream.h WidePrefix): 80 B per node, 4 AES blocks per parent.
// Auto: log2(m) - 1, at most 22 (two 336 MB node buffers at 2^22), none below 8.
constexpr uint32_t kWidePrefixMax = 22;
uint32_t wide_prefix_depth(const dcf_prg* p, const Cfg& c, size_t n_bytes, uint64_t m) {
  if (p->lambda <= 16 || p->kind != 0 || c.prefix_levels == 0 || m == 0) return 0;
  uint32_t d;
  if (c.prefix_levels > 0) {
    d = std::min((uint32_t)c.prefix_levels, 30u);
  } else {
    const uint32_t lg = 63u - (uint32_t)__builtin_clzll(m | 1u);
    d = lg > 1u ? lg - 1u : 0u;
    if (d < 8u) return 0;
    d = std::min(d, kWidePrefixMax);
    d = capped_depth(p, c, std::min<uint32_t>(d, (uint32_t)(8 * n_bytes - 1)));
  }
  return std::min<uint32_t>(d, (uint32_t)(8 * n_bytes - 1));
}

// Expand the top `levels` levels of one key's tree for the wide stream head (the CW
// digest w->d_dig must hold this key) into WidePrefix rows in w->d_pfx, in one launch
// (k_wpfx_build): [table 2^D x 80 B | 2 x 2^S regions of 2^(D-1-S) nodes].
int build_wide_prefix(dcf_prg* p, Workspace* w, uint32_t nlev, int party, const uint8_t* s0, uint32_t levels,
                      WidePrefix* out, hipStream_t st) {
  const uint32_t S = prefix_split(levels);
  const uint32_t R = 1u << (levels - 1u - S);
  const size_t tab_bytes = (((size_t)80 << levels) + 255) & ~(size_t)255;
  const size_t region = (size_t)80 * R;
  const size_t need = tab_bytes + 2 * ((size_t)1 << S) * region;
  if (int rc = grow(&w->d_pfx, &w->pfx_bytes, need, st)) return rc;
  uint4* table = (uint4*)w->d_pfx;
  uint4* ba = (uint4*)(w->d_pfx + tab_bytes);
  uint4* bb = (uint4*)(w->d_pfx + tab_bytes + ((size_t)1 << S) * region);
  if (p->lambda == 32)
    hipLaunchKernelGGL(k_wpfx_build<true>, dim3(1u << S), dim3(kBlock), 0, st, p->d_tab, p->d_rk2,
                       (const uint4*)w->d_dig, w->d_dig + (size_t)nlev * 64, s0, (uint32_t)party, S, levels, ba, bb, R,
                       table);
  else
    hipLaunchKernelGGL(k_wpfx_build<false>, dim3(1u << S), dim3(kBlock), 0, st, p->d_tab, p->d_rk2,
                       (const uint4*)w->d_dig, w->d_dig + (size_t)nlev * 64, s0, (uint32_t)party, S, levels, ba, bb, R,
                       table);
  HIP_TRY(hipGetLastError());
  *out = WidePrefix{table, levels};
  return DCF_OK;
}


// Expand the top `levels` levels of the key's tree (s = s0, v = 0, t = party at the
// root; k_fd_level16 per level, as the full-domain eval does) into w->d_pfx.

int build_prefix(dcf_prg* p, Workspace* w, size_t n_bytes, int party, const uint4* cws, const uint4* cwv,
                 const uint8_t* cwt, const uint4* np1, const uint8_t* s0, uint32_t levels, PrefixTable* out,
                 hipStream_t st) {
  const uint64_t maxnodes = 1ull << levels;
  const size_t nodeb = 33, half = (maxnodes * nodeb + 255) & ~(size_t)255;
  // Hirose: [table 2^D x 32 B | 2 x 2^S regions of 2^(D-1-S) nodes]; MMO: two level buffers + counters
  const uint32_t S = prefix_split(levels);
  const uint32_t R = 1u << prefix_region_log2(levels, S);
  const size_t region = ((size_t)R * nodeb + 255) & ~(size_t)255;
  const size_t tab_bytes = (maxnodes * 32 + 255) & ~(size_t)255;
  const size_t need = p->kind == 0 ? tab_bytes + 2 * ((size_t)1 << S) * region : 2 * half + 64 * sizeof(uint32_t);
  if (w->pfx_bytes < need) {
    if (w->d_pfx) {
      HIP_TRY(hipStreamSynchronize(st));
      HIP_TRY(hipFree(w->d_pfx));
      w->d_pfx = nullptr;
      w->pfx_bytes = 0;
    }
    const hipError_t e = hipMalloc(&w->d_pfx, need);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      w->d_pfx = nullptr;
      return fail(kPrefixNoMem, std::string("prefix table: hipMalloc: ") + hipGetErrorString(e));
    }
    w->pfx_bytes = need;
  }
  if (p->kind == 0) {  // one launch: k_prefix_build16
    uint8_t* ba = w->d_pfx + tab_bytes;
    const uint32_t H = prefix_dfs_levels(levels, S);
    hipLaunchKernelGGL(k_prefix_build16, dim3(1u << S), dim3(kBlock), 0, st, p->d_tab, p->rk[0], cws, cwv, cwt,
                       (const uint4*)s0, (uint32_t)party, S, levels, H, ba, ba + ((size_t)1 << S) * region,
                       (uint64_t)region, R, (uint4*)w->d_pfx, p->d_rk0);
    HIP_TRY(hipGetLastError());
    *out = PrefixTable{(const uint4*)w->d_pfx, levels};
    return DCF_OK;
  }
  uint4* s_a = (uint4*)w->d_pfx;
  uint4* v_a = s_a + maxnodes;
  uint8_t* t_a = (uint8_t*)(v_a + maxnodes);
  uint4* s_b = (uint4*)(w->d_pfx + half);
  uint4* v_b = s_b + maxnodes;
  uint8_t* t_b = (uint8_t*)(v_b + maxnodes);
  uint32_t* ctrs = (uint32_t*)(w->d_pfx + 2 * half);
  HIP_TRY(hipMemsetAsync(ctrs, 0, 64 * sizeof(uint32_t), st));
  hipLaunchKernelGGL(k_fd_root16, dim3(1), dim3(64), 0, st, (const uint4*)s0, (uint32_t)party, s_a, v_a, t_a);
  HIP_TRY(hipGetLastError());
  const uint32_t nlev = (uint32_t)(8 * n_bytes);  // > levels: no level here is the last one
  for (uint32_t lev = 0; lev < levels; ++lev) {
    const uint64_t parents = 1ull << lev;
    if (p->kind == 1)
      hipLaunchKernelGGL(k_fd_level16_mmo, dim3((unsigned)grid_for(parents, p->cus)), dim3(kBlock), 0, st, p->d_tab,
                         p->d_rk128, cws, cwv, cwt, np1, lev, nlev, parents, s_a, v_a, t_a, s_b, v_b, t_b,
                         (uint4*)nullptr, ctrs + lev);
    else
      hipLaunchKernelGGL(k_fd_level16, dim3((unsigned)grid_for(parents, p->cus)), dim3(kBlock), 0, st, p->d_tab,
                         p->rk[0], cws, cwv, cwt, np1, lev, nlev, parents, s_a, v_a, t_a, s_b, v_b, t_b,
                         (uint4*)nullptr, ctrs + lev);
    HIP_TRY(hipGetLastError());
    std::swap(s_a, s_b);
    std::swap(v_a, v_b);
    std::swap(t_a, t_b);
  }
  // 32-byte rows (kernels16.h PrefixTable) into the other buffer: 2^D * 32 <= half.
  hipLaunchKernelGGL(k_prefix_pack, dim3((unsigned)std::min<uint64_t>((maxnodes + 255) / 256, 4096)), dim3(256), 0,
                     st, s_a, v_a, t_a, maxnodes, s_b);
  HIP_TRY(hipGetLastError());
  *out = PrefixTable{s_b, levels};
  return DCF_OK;
}

// build_prefix at depth d; in auto mode (prefix_levels < 0) an allocation failure retries
// two levels shallower, down to 8, and then evaluates without a table (same output bytes).
int try_prefix(dcf_prg* p, const Cfg& c, Workspace* w, size_t n_bytes, int party, const uint4* cws, const uint4* cwv,
               const uint8_t* cwt, const uint4* np1, const uint8_t* s0, uint32_t d, PrefixTable* out, hipStream_t st) {
  *out = PrefixTable{nullptr, 0u};
  while (d) {
    const int rc = build_prefix(p, w, n_bytes, party, cws, cwv, cwt, np1, s0, d, out, st);
    if (rc != kPrefixNoMem) return rc;
    if (c.prefix_levels >= 0) return fail(DCF_ERR_HIP, t_err);  // a forced depth must fit
    d = d >= 10u ? d - 2u : 0u;
  }
  *out = PrefixTable{nullptr, 0u};
  return DCF_OK;
}

// Tails over cnt points of cnt / ppk consecutive keys key, key + 1, ... (ppk points each, s0: their
// s0s back to back; one key: ppk = cnt); grid rows = keys x ranges per key.
template <int TW, int NCH = 0, bool ACC = false>
int launch_tail(const uint8_t* cws, const uint8_t* cwv, const uint8_t* np1, const uint8_t* s0, uint32_t nlev,
                uint32_t lam, uint64_t K, uint64_t key, const uint32_t* tvec, uint64_t cnt, uint8_t* ys,
                hipStream_t st, uint64_t ppk, uint32_t c0 = 0, uint32_t ncp = 0) {
  static_assert(TW == 32 || TW == 64 || TW == 128 || TW == 256, "tile width");
  if (ncp == 0) ncp = (nlev + 1 + 3) / 4;
  const size_t lds = (size_t)ncp * 16 * TW;
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_eval_wide_tail<TW, NCH, ACC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // Points per workgroup: each workgroup builds its tile's tables once, then streams its
  // kTailPts points (r02i A/B on C4: 41.1-41.3 ms vs 41.7-42.3 with ranges sized to 1, 2 or 4
  // workgroups per CU).
  const uint64_t tiles = (lam + TW - 1) / TW;
  const uint64_t rpk = (ppk + kTailPts - 1) / kTailPts;
  const dim3 grid((unsigned)tiles, (unsigned)((cnt / ppk) * rpk));
  hipLaunchKernelGGL((k_eval_wide_tail<TW, NCH, ACC>), grid, dim3(kBlock), lds, st, cws, cwv, np1, s0, nlev, lam, K,
                     key, tvec, cnt, kTailPts, ys, t_words(nlev), ppk, (uint32_t)rpk, c0, ncp);
  HIP_TRY(hipGetLastError());
  return DCF_OK;
}

// More chunks than one 32-byte-tile table set holds (N >= 160): passes of kTailPassChunks chunks,
// each after the first adding its rows' share to the y the previous pass wrote.
constexpr uint32_t kTailPassChunks = 320;  // 320 x 16 entries x 32 B = 160 KiB
int launch_tail_passes(const uint8_t* cws, const uint8_t* cwv, const uint8_t* np1, const uint8_t* s0, uint32_t nlev,
                       uint32_t lam, uint64_t K, uint64_t key, const uint32_t* tvec, uint64_t cnt, uint8_t* ys,
                       hipStream_t st, uint64_t ppk) {
  const uint32_t nch = (nlev + 1 + 3) / 4;
  for (uint32_t c0 = 0; c0 < nch; c0 += kTailPassChunks) {
    const uint32_t ncp = std::min(kTailPassChunks, nch - c0);
    const int rc = c0 == 0 ? launch_tail<32>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk, 0, ncp)
                           : launch_tail<32, 0, true>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk,
                                                      c0, ncp);
    if (rc) return rc;
  }
  return DCF_OK;
}

// Paired-slot tail (k_eval_wide_tail2, 128-byte tiles, 6/5-bit chunks in LDS): the t-vectors are
// repacked into chunk bytes in place, then the tail runs as launch_tail does.  (8-bit chunks in
// global memory beside the LDS tables, read through the vector L1 / L2, measured 11-24 % slower on
// C4: profiles/AB_LOG.md r04d.)
template <int R6, int R5, int ROW0>
int launch_tail2(const uint8_t* cws, const uint8_t* cwv, const uint8_t* np1, const uint8_t* s0, uint32_t nlev,
                 uint32_t lam, uint64_t K, uint64_t key, uint32_t* tvec, uint64_t cnt, uint8_t* ys, hipStream_t st,
                 int cus, uint64_t ppk, int party, Workspace* w) {
  using L = Tail2Layout<R6, R5, ROW0>;
  if (nlev + 1 > L::rows()) return fail(DCF_ERR_UNSUPPORTED, "tail2 layout too small");
  const uint64_t tiles = (lam + 127) / 128;
  hipLaunchKernelGGL((k_tvec_chunks<R6, R5, ROW0>), dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, tvec, nlev,
                     cnt);
  HIP_TRY(hipGetLastError());
  const size_t lds = L::lds_bytes();
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_eval_wide_tail2<R6, R5, ROW0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // One workgroup per CU at a time, kTail2Rounds rounds of them: the batch split into
  // rounds x cus / tiles ranges, so the tiles of a range build their tables once and walk its
  // points together (the rows being written at any time stay few), at least 32768 points per
  // workgroup.  Several rounds let the dispatcher even out the CUs' speeds (one round: the last
  // workgroup ended ~1 ms after the first, profiles/r04b_c4_timeline_dynamic_tail.json).  C4 A/B
  // (r04t / r04u, 3 alternating runs per box): rounds 1 / 2 / 4 / 8 32.33-32.53 / 32.46-32.73 /
  // 32.28-32.43 / 32.16-32.27 ms; on a second box 8 / 16 / 32 / 64 (= 32768-point ranges)
  // 33.08-33.12 / 33.12-33.41 / 33.24-33.28 / 33.69-33.99 ms.
  // Several keys (ppk < cnt): each key's points are ranges of their own (its own tables).
  constexpr uint64_t kTail2Rounds = 8;
  const uint64_t ranges = std::max<uint64_t>(1, (uint64_t)cus * kTail2Rounds / tiles);
  const uint64_t per = std::max<uint64_t>(32768, (((cnt + ranges - 1) / ranges) + 255) & ~(uint64_t)255);
  const uint64_t rpk = (ppk + per - 1) / per;
  const dim3 grid((unsigned)tiles, (unsigned)((cnt / ppk) * rpk));
  uint32_t* gctr = nullptr;
  if (L::GCTR) {  // one block counter per workgroup (each workgroup resets its own)
    uint8_t* b = reinterpret_cast<uint8_t*>(w->d_tctr);
    if (int rc = grow(&b, &w->tctr_bytes, (size_t)grid.x * grid.y * kT2CtrStride * sizeof(uint32_t), st)) return rc;
    w->d_tctr = reinterpret_cast<uint32_t*>(b);
    gctr = w->d_tctr;
  }
  hipLaunchKernelGGL((k_eval_wide_tail2<R6, R5, ROW0>), grid, dim3(kBlock), lds, st, cws, cwv, np1, s0, nlev, lam, K,
                     key, tvec, cnt, (uint32_t)per, ys, ppk, (uint32_t)rpk, (uint32_t)party, gctr);
  HIP_TRY(hipGetLastError());
  return DCF_OK;
}

// The tail for n = nlev levels: the paired-slot tail when one of its instances covers the
// n + 1 rows with fewer LDS reads than the 4-bit tail's ceil((n + 1) / 4), else the 4-bit one.
// ppk: points per key (= cnt for one key).
int run_tail(const uint8_t* cws, const uint8_t* cwv, const uint8_t* np1, const uint8_t* s0, uint32_t nlev,
             uint32_t lam, uint64_t K, uint64_t key, uint32_t* tvec, uint64_t cnt, uint8_t* ys, hipStream_t st,
             int cus, uint64_t ppk, int party, Workspace* w) {
  const uint32_t nrows = nlev + 1, nch = (nrows + 3) / 4;
  if (lam % 128 == 0) {
    // Paired-slot layouts with row 0 folded into the constant (t_0 = party): the first that covers
    // rows 1 .. n, in increasing reads per 16 bytes of y (2 (R6 + R5)), used when it beats the
    // 4-bit tail's ceil((n + 1) / 4).  (r04 layouts, row 0 in the tables: N = 16 took (5, 7), 24 reads.)
#define DCF_T2(A, B)                                                                               \
  if (nrows <= Tail2Layout<A, B, 1>::rows() && 2u * (A + B) < nch)                                 \
    return launch_tail2<A, B, 1>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, cus, ppk, party, w);
#ifndef DCF_T2_ROW0
#define DCF_T2_ROW0 1
#endif
    if (!DCF_T2_ROW0) {  // A/B knob: the r04 layouts (row 0 in the tables)
      if (nrows <= Tail2Layout<5, 7>::rows() && nrows > Tail2Layout<3, 3>::rows() && 24u < nch)
        return launch_tail2<5, 7, 0>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, cus, ppk, party, w);
    }
    DCF_T2(0, 1)   // N = 1: 8 rows, 2 reads (4-bit: 3)
    DCF_T2(2, 0)   // N = 2, 3: 16 / 24 rows, 4 reads (5 / 7)
    DCF_T2(1, 2)   // N = 4: 32 rows, 6 reads (9)
    DCF_T2(4, 0)   // N = 5, 6: 40 / 48 rows, 8 reads (11 / 13)
    DCF_T2(3, 2)   // N = 7: 56 rows, 10 reads (15)
    DCF_T2(6, 0)   // N = 8, 9: 64 / 72 rows, 12 reads (17 / 19)
    DCF_T2(5, 2)   // N = 10: 80 rows, 14 reads (21)
    DCF_T2(8, 0)   // N = 11, 12: 88 / 96 rows, 16 reads (23 / 25)
    DCF_T2(7, 2)   // N = 13: 104 rows, 18 reads (27)
    DCF_T2(10, 0)  // N = 14, 15: 112 / 120 rows, 20 reads (29 / 31), 160 KiB of tables
    DCF_T2(9, 2)   // N = 16: 128 rows, 22 reads (33), 160 KiB of tables
    DCF_T2(8, 4)   // N = 17: 136 rows, 24 reads (35), 160 KiB of tables
#undef DCF_T2
  }
  // 4-bit tail: the widest tile whose tables (nch x 16 entries x TW bytes) fit the LDS
  if (nch == 33) return launch_tail<256, 33>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk);
  if (nch <= 40) return launch_tail<256>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk);
  if (nch <= 80) return launch_tail<128>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk);
  if (nch <= 160) return launch_tail<64>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk);
  if (nch <= kTailPassChunks) return launch_tail<32>(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk);
  return launch_tail_passes(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys, st, ppk);
}

// Dcf::eval at LAMBDA >= 32 for key `key` of a K-key CWB (see kernels_wide.h).
// The caller (eval_launch) has zeroed the workspace's block count once for the whole call.
int eval_wide(dcf_prg* p, const Cfg& c, Workspace* w, size_t n_bytes, uint64_t K, uint64_t key, int party, const uint8_t* cwb,
              const uint8_t* s0, const uint8_t* xs, uint64_t m, uint8_t* ys, hipStream_t st) {
  const uint32_t lam = (uint32_t)p->lambda, nlev = (uint32_t)(8 * n_bytes);
  const size_t n = 8 * n_bytes;
  const uint8_t* cws = cwb;
  const uint8_t* cwv = cwb + n * K * lam;
  const uint8_t* cwt = cwb + 2 * n * K * lam;
  const uint8_t* np1 = cwb + dcf_cwb_np1_offset(n_bytes, lam, K);
  const uint32_t tw = t_words(nlev);  // t-vector words per point
  const uint64_t chunk = std::min<uint64_t>(m, wide_chunk_points(tw));
  // + 256 B: a multi-pass tail's t loads run up to 64 B past the last row (never used)
  const size_t tvb = ((chunk * tw * 4 + 255) & ~(size_t)255) + 256;
  int rc = ensure_ws(w, tvb, st);
  if (rc) return rc;
  uint32_t* tvec = reinterpret_cast<uint32_t*>(w->d_ws);
  WidePrefix wpf{nullptr, 0u};
  for (uint64_t off = 0; off < m; off += chunk) {
    const uint64_t cnt = (m - off < chunk) ? m - off : chunk;
    {  // stream head: 2.5 AES blocks per level instead of 4
      HIP_TRY(hipMemsetAsync(w->d_ctr, 0, 8, st));  // the pass's work counter (the block count stays)
      if (off == 0) {  // CW digest of this key (bytes [0,32) of each level's cw_s / cw_v, and cw_t)
        if (w->dig_levels < nlev) {
          size_t have = (size_t)w->dig_levels * 65;
          if (int rc2 = grow(&w->d_dig, &have, (size_t)nlev * 65, st)) return rc2;
          w->dig_levels = nlev;
        }
        hipLaunchKernelGGL(k_cw_digest, dim3((4 * nlev + 255) / 256), dim3(256), 0, st, cws, cwv, cwt, nlev, lam, K,
                           key, 1u, (uint4*)w->d_dig, w->d_dig + (size_t)nlev * 64);
        HIP_TRY(hipGetLastError());
        const uint32_t d = wide_prefix_depth(p, c, n_bytes, m);
        if (d) {
          rc = build_wide_prefix(p, w, nlev, party, s0, d, &wpf, st);
          if (rc) return rc;
        }
        w->last_prefix = d;
      }
      const uint64_t units = (cnt + kWideUnit - 1) / kWideUnit;
      uint64_t blocks = (units + 15) / 16;
      if (blocks > (uint64_t)p->cus) blocks = (uint64_t)p->cus;
      // one point per lane, one 1024-thread workgroup per CU (the T-tables fill the LDS)
#define DCF_WHS(MH, XR)                                                                                        \
  hipLaunchKernelGGL((k_eval_wide_head_stream<1, MH, XR, false, kBlock>), dim3((unsigned)blocks), dim3(kBlock), 0, st, p->d_tab, \
                     p->d_rk2, (const uint4*)w->d_dig, w->d_dig + (size_t)nlev * 64, np1, s0, (uint32_t)party, xs + off * n_bytes, (uint32_t)n_bytes,   \
                     lam, K, key, cnt, w->d_ctr, ys + off * lam, tvec, wpf, tw, (uint32_t)cnt)
      const bool xreg = n_bytes % 4 == 0 && n_bytes <= 16;
      if (lam == 32 && xreg) DCF_WHS(true, true);
      else if (lam == 32) DCF_WHS(true, false);
      else if (xreg) DCF_WHS(false, true);
      else DCF_WHS(false, false);
#undef DCF_WHS
    }
    HIP_TRY(hipGetLastError());
    if (lam > 32) {
      rc = run_tail(cws, cwv, np1, s0, nlev, lam, K, key, tvec, cnt, ys + off * lam, st, p->cus, cnt, party, w);
      if (rc) return rc;
    }
  }
  return DCF_OK;
}

// Dcf::eval at LAMBDA >= 32 for keys 0 .. K - 1, ppk points each (key-major xs / ys, s0s[K][LAMBDA]),
// several keys per pass: one key-major CW digest, one stream-head launch (each point's key =
// point / ppk) and one tail launch whose workgroups build the tables of their own key.  For
// ppk <= kWideBatchPpk (larger keys amortise their own launches: eval_wide per key).  No shared
// prefix; the MMO PRG keeps the per-key path.
constexpr uint64_t kWideBatchPpk = 32768;
constexpr uint64_t kWideBatchKeys = 4096;  // keys per pass: tail grid rows (keys x <= 8 ranges) <= 32768
// The multi-key shapes eval_wide_batch takes: several keys of few points each, Hirose PRG, and no
// forced prefix depth (a forced depth runs the per-key passes, which build one table per key).
bool wide_batched(const dcf_prg* p, const Cfg& c, uint64_t num_keys, uint64_t ppk) {
  return num_keys > 1 && ppk > 0 && p->kind == 0 && ppk <= kWideBatchPpk && c.prefix_levels <= 0;
}

int eval_wide_batch(dcf_prg* p, Workspace* w, size_t n_bytes, uint64_t K, uint64_t ppk, int party,
                    const uint8_t* cwb, const uint8_t* s0s, const uint8_t* xs, uint8_t* ys, hipStream_t st) {
  const uint32_t lam = (uint32_t)p->lambda, nlev = (uint32_t)(8 * n_bytes);
  const size_t n = 8 * n_bytes;
  const uint8_t* cws = cwb;
  const uint8_t* cwv = cwb + n * K * lam;
  const uint8_t* cwt = cwb + 2 * n * K * lam;
  const uint8_t* np1 = cwb + dcf_cwb_np1_offset(n_bytes, lam, K);
  const uint32_t tw = t_words(nlev);
  // keys per pass; the digest's uint4 index 4 * (key * nlev + level) and dig_levels are 32-bit
  const uint64_t kdig = std::max<uint64_t>(1, (0xFFFFFFFFull / 4u) / nlev);
  const uint64_t kp =
      std::max<uint64_t>(1, std::min<uint64_t>({K, wide_chunk_points(tw) / ppk, kWideBatchKeys, kdig}));
  const size_t tvb = ((kp * ppk * tw * 4 + 255) & ~(size_t)255) + 256;
  if (int rc = ensure_ws(w, tvb, st)) return rc;
  if (w->dig_levels < kp * nlev) {
    size_t have = (size_t)w->dig_levels * 65;
    if (int rc = grow(&w->d_dig, &have, (size_t)kp * nlev * 65, st)) return rc;
    w->dig_levels = (uint32_t)(kp * nlev);
  }
  uint32_t* tvec = reinterpret_cast<uint32_t*>(w->d_ws);
  const WidePrefix none{nullptr, 0u};
  const bool xreg = n_bytes % 4 == 0 && n_bytes <= 16;
  for (uint64_t k0 = 0; k0 < K; k0 += kp) {
    const uint64_t nk = std::min<uint64_t>(kp, K - k0), cnt = nk * ppk;
    HIP_TRY(hipMemsetAsync(w->d_ctr, 0, 8, st));  // the pass's work counter (the block count stays)
    uint4* dig = (uint4*)w->d_dig;
    uint8_t* dig_t = w->d_dig + (size_t)nk * nlev * 64;
    hipLaunchKernelGGL(k_cw_digest, dim3((unsigned)((4 * nlev * nk + 255) / 256)), dim3(256), 0, st, cws, cwv, cwt, nlev,
                       lam, K, k0, (uint32_t)nk, dig, dig_t);
    HIP_TRY(hipGetLastError());
    const uint64_t units = (cnt + kWideUnit - 1) / kWideUnit;
    const uint64_t blocks = std::min<uint64_t>((units + 15) / 16, (uint64_t)p->cus);
    const uint8_t* s0p = s0s + k0 * lam;
    const uint8_t* xp = xs + k0 * ppk * n_bytes;
    uint8_t* yp = ys + k0 * ppk * lam;
#define DCF_WHB(MH, XR)                                                                                           \
  hipLaunchKernelGGL((k_eval_wide_head_stream<1, MH, XR, true, kBlock>), dim3((unsigned)blocks), dim3(kBlock), 0, st, \
                     p->d_tab, p->d_rk2, (const uint4*)dig, dig_t, np1, s0p, (uint32_t)party, xp, (uint32_t)n_bytes,  \
                     lam, K, k0, cnt, w->d_ctr, yp, tvec, none, tw, (uint32_t)ppk)
    if (lam == 32 && xreg) DCF_WHB(true, true);
    else if (lam == 32) DCF_WHB(true, false);
    else if (xreg) DCF_WHB(false, true);
    else DCF_WHB(false, false);
#undef DCF_WHB
    HIP_TRY(hipGetLastError());
    if (lam > 32) {
      if (int rc = run_tail(cws, cwv, np1, s0p, nlev, lam, K, k0, tvec, cnt, yp, st, p->cus, ppk, party, w)) return rc;
    }
  }
  return DCF_OK;
}

// Dcf::eval with the MMO PRG at LAMBDA >= 32 for key `key` (kernels_mmo_wide.h): per pass
// of up to kWideChunk points, the head walks block 0 (y[0:16), t-vector), then the tail
// walks blocks 1..nb-1 given the t-vectors.
int eval_mmo_wide(dcf_prg* p, Workspace* w, size_t n_bytes, uint64_t K, uint64_t key, int party, const uint8_t* cwb,
                  const uint8_t* s0, const uint8_t* xs, uint64_t m, uint8_t* ys, hipStream_t st) {
  const uint32_t lam = (uint32_t)p->lambda, nb = lam / 16u;
  const size_t n = 8 * n_bytes;
  const uint8_t* cws = cwb;
  const uint8_t* cwv = cwb + n * K * lam;
  const uint8_t* cwt = cwb + 2 * n * K * lam;
  const uint8_t* np1 = cwb + dcf_cwb_np1_offset(n_bytes, lam, K);
  const uint32_t tw = mmo_t_words((uint32_t)n);
  const uint64_t chunk = std::min<uint64_t>(m, wide_chunk_points(2 * tw));
  if (int rc = ensure_ws(w, chunk * tw * 4, st)) return rc;
  uint32_t* tvec = reinterpret_cast<uint32_t*>(w->d_ws);
  for (uint64_t off = 0; off < m; off += chunk) {
    const uint64_t cnt = std::min<uint64_t>(chunk, m - off);
    const uint64_t groups = (cnt + 63) / 64;
    const dim3 gh((unsigned)std::min<uint64_t>((groups + 15) / 16, (uint64_t)p->cus));
    hipLaunchKernelGGL(k_mmo_wide_eval<true>, gh, dim3(kBlock), 0, st, p->d_tab, p->d_rk128, cws, cwv, cwt, np1, s0,
                       (uint32_t)party, xs + off * n_bytes, (uint32_t)n_bytes, lam, K, key, cnt, tvec, ys + off * lam);
    HIP_TRY(hipGetLastError());
    if (nb > 1) {
      const uint64_t items = groups * (nb - 1);
      const dim3 gt((unsigned)std::min<uint64_t>((items + 15) / 16, 4 * (uint64_t)p->cus));
      hipLaunchKernelGGL(k_mmo_wide_eval<false>, gt, dim3(kBlock), 0, st, p->d_tab, p->d_rk128, cws, cwv, cwt, np1,
                         s0, (uint32_t)party, xs + off * n_bytes, (uint32_t)n_bytes, lam, K, key, cnt, tvec,
                         ys + off * lam);
      HIP_TRY(hipGetLastError());
    }
  }
  return DCF_OK;
}

// Batched Dcf::gen with the MMO PRG at LAMBDA >= 32 (kernels_mmo_wide.h): per pass of keys,
// the head over block 0 of both parties (t-CWs, per-level t bits), then the tail.
int gen_mmo_wide(dcf_prg* p, Workspace* w, size_t n_bytes, uint64_t K, const uint8_t* alpha, const uint8_t* beta,
                 const uint8_t* s0_0, const uint8_t* s0_1, int bound, uint8_t* cws, uint8_t* cwv, uint8_t* cwt,
                 uint8_t* np1, hipStream_t st) {
  const uint32_t lam = (uint32_t)p->lambda, nb = lam / 16u, nlev = (uint32_t)(8 * n_bytes);
  if (int rc = ensure_ws(w, (size_t)K * nlev * 4, st)) return rc;
  uint32_t* tinfo = reinterpret_cast<uint32_t*>(w->d_ws);
  const uint64_t groups = (K + 63) / 64;
  const dim3 gh((unsigned)std::min<uint64_t>((groups + 15) / 16, (uint64_t)p->cus));
  hipLaunchKernelGGL(k_mmo_wide_gen<true>, gh, dim3(kBlock), 0, st, p->d_tab, p->d_rk128, alpha, beta, s0_0, s0_1,
                     (uint32_t)bound, (uint32_t)n_bytes, lam, K, cws, cwv, cwt, np1, tinfo);
  HIP_TRY(hipGetLastError());
  if (nb > 1) {
    const uint64_t items = groups * (nb - 1);
    const dim3 gt((unsigned)std::min<uint64_t>((items + 15) / 16, 4 * (uint64_t)p->cus));
    hipLaunchKernelGGL(k_mmo_wide_gen<false>, gt, dim3(kBlock), 0, st, p->d_tab, p->d_rk128, alpha, beta, s0_0,
                       s0_1, (uint32_t)bound, (uint32_t)n_bytes, lam, K, cws, cwv, cwt, np1, tinfo);
    HIP_TRY(hipGetLastError());
  }
  return DCF_OK;
}

}  // namespace

extern "C" {

const char* dcf_version(void) { return DCF_VERSION; }

const char* dcf_last_error(void) { return t_err.c_str(); }

size_t dcf_cwb_np1_offset(size_t n_bytes, size_t lambda, size_t num_keys) {
  const size_t n = 8 * n_bytes;
  return ((2 * n * num_keys * lambda + n * num_keys) + 15) & ~(size_t)15;
}

size_t dcf_cwb_bytes(size_t n_bytes, size_t lambda, size_t num_keys) {
  return dcf_cwb_np1_offset(n_bytes, lambda, num_keys) + num_keys * lambda;
}

int dcf_hirose_prg_new(const uint8_t* keys, size_t cipher_n, size_t lambda, int device, dcf_prg** out) {
  if (!keys || !out) return fail(DCF_ERR_ARG, "null argument");
  *out = nullptr;
  if (lambda == 0 || lambda % 16 != 0) return fail(DCF_ERR_LAMBDA, "lambda must be a positive multiple of 16");
  const size_t need = (lambda / 16 >= 2) ? 18 : 1;
  if (cipher_n < need)
    return fail(DCF_ERR_CIPHER_N, "cipher_n too small: the Hirose PRG reads ciphers[i*16+j] (prg.rs:51)");
  std::call_once(g_aes_once, aes_init_tables);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(DCF_ERR_ARG, "bad device ordinal");
  DeviceGuard dg(device);
  if (!dg.ok) return fail(DCF_ERR_HIP, "hipSetDevice failed");
  dcf_prg* p = new dcf_prg();
  p->device = device;
  p->lambda = lambda;
  p->cipher_n = cipher_n;
  p->rk.resize(cipher_n);
  for (size_t i = 0; i < cipher_n; i++) aes256_expand_words(keys + 32 * i, &p->rk[i]);
  p->key_blob.assign(keys, keys + 32 * cipher_n);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    p->cus = prop.multiProcessorCount;
  hipError_t e = hipMalloc(&p->d_tab, sizeof(g_tab));
  if (e == hipSuccess) e = hipMemcpy(p->d_tab, g_tab, sizeof(g_tab), hipMemcpyHostToDevice);
  // device copies of the schedules the kernels read per round: cipher 0 (LAMBDA = 16 stream /
  // pair / table-build kernels) and, at LAMBDA >= 32, ciphers 0 and 17 (the wide stream head)
  if (e == hipSuccess) e = hipMalloc(&p->d_rk0, sizeof(RoundKeys));
  if (e == hipSuccess) e = hipMemcpy(p->d_rk0, &p->rk[0], sizeof(RoundKeys), hipMemcpyHostToDevice);
  if (e == hipSuccess && lambda > 16) {
    e = hipMalloc(&p->d_rk2, 2 * sizeof(RoundKeys));
    if (e == hipSuccess) e = hipMemcpy(p->d_rk2, &p->rk[0], sizeof(RoundKeys), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_rk2 + 15, &p->rk[17], sizeof(RoundKeys), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    dcf_prg_free(p);
    return fail(DCF_ERR_HIP, std::string("table upload: ") + hipGetErrorString(e));
  }
  *out = p;
  return DCF_OK;
}

int dcf_mmo_prg_new(const uint8_t* keys, size_t cipher_n, size_t lambda, int device, dcf_prg** out) {
  if (!keys || !out) return fail(DCF_ERR_ARG, "null argument");
  *out = nullptr;
  if (lambda == 0 || lambda % 16 != 0) return fail(DCF_ERR_LAMBDA, "lambda must be a positive multiple of 16");
  if (cipher_n < 4 * (lambda / 16)) return fail(DCF_ERR_CIPHER_N, "MMO PRG needs 4 * lambda / 16 AES-128 keys");
  std::call_once(g_aes_once, aes_init_tables);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(DCF_ERR_ARG, "bad device ordinal");
  DeviceGuard dg(device);
  if (!dg.ok) return fail(DCF_ERR_HIP, "hipSetDevice failed");
  dcf_prg* p = new dcf_prg();
  p->kind = 1;
  p->device = device;
  p->lambda = lambda;
  p->cipher_n = cipher_n;
  p->eval_mode = DCF_EVAL_TTABLE;
  p->key_blob.assign(keys, keys + 16 * cipher_n);
  // schedule b * nb + j for output b (s_L, v_L, s_R, v_R) and 16-byte block j (kernels_mmo_wide.h)
  const size_t nsched = 4 * (lambda / 16);
  std::vector<uint32_t> w(nsched * 44);
  for (size_t i = 0; i < nsched; i++) aes128_expand_words(keys + 16 * i, w.data() + 44 * i);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    p->cus = prop.multiProcessorCount;
  hipError_t e = hipMalloc(&p->d_tab, sizeof(g_tab));
  if (e == hipSuccess) e = hipMemcpy(p->d_tab, g_tab, sizeof(g_tab), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&p->d_rk128, w.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(p->d_rk128, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) p->rk128_count = nsched;
  if (e != hipSuccess) {
    dcf_prg_free(p);
    return fail(DCF_ERR_HIP, std::string("table upload: ") + hipGetErrorString(e));
  }
  *out = p;
  return DCF_OK;
}

int dcf_prg_kind(const dcf_prg* p) { return p ? p->kind : -1; }

static void free_workspace(Workspace* w) {
  for (hipStream_t s : w->hs)  // host-path work still queued (an error return drains these too)
    if (s) (void)hipStreamSynchronize(s);
  if (w->aux) (void)hipStreamSynchronize(w->aux);
  if (w->pending) (void)hipEventSynchronize(w->done);  // the last device call's kernels
  for (void* b : {(void*)w->d_ctr, (void*)w->d_ws, (void*)w->d_dig, (void*)w->d_kdig, (void*)w->d_pfx,
                  (void*)w->d_mkey, (void*)w->d_stage, (void*)w->d_tctr})
    if (b) (void)hipFree(b);
  if (w->h_stage) (void)hipHostFree(w->h_stage);
  if (w->h_tiny) (void)hipHostFree(w->h_tiny);
  if (w->h_mid) (void)hipHostFree(w->h_mid);
  for (hipStream_t s : w->hs)
    if (s) (void)hipStreamDestroy(s);
  if (w->aux) (void)hipStreamDestroy(w->aux);
  for (hipEvent_t e : w->aux_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : w->hev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : w->tev)
    if (e) (void)hipEventDestroy(e);
  if (w->done) (void)hipEventDestroy(w->done);
  delete w;
}

void dcf_prg_free(dcf_prg* p) {
  if (!p) return;
  {
    DeviceGuard dg(p->device);
    for (Workspace* w : p->all_ws) free_workspace(w);
    for (void* b : {(void*)p->d_tab, (void*)p->d_rk128, (void*)p->d_rk2, (void*)p->d_rk0})
      if (b) (void)hipFree(b);
  }
  delete p;
}

size_t dcf_prg_lambda(const dcf_prg* p) { return p ? p->lambda : 0; }

int dcf_prg_set_eval_mode(dcf_prg* p, int mode) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (mode != DCF_EVAL_AUTO && mode != DCF_EVAL_TTABLE && mode != DCF_EVAL_STREAM)
    return fail(DCF_ERR_ARG, "bad eval mode (DCF_EVAL_AUTO, DCF_EVAL_TTABLE or DCF_EVAL_STREAM)");
  p->eval_mode = mode;
  return DCF_OK;
}

int dcf_prg_set_prefix_levels(dcf_prg* p, int levels) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (levels < -1) return fail(DCF_ERR_ARG, "prefix levels must be -1 (auto), 0 (off) or > 0");
  p->prefix_levels = levels;
  return DCF_OK;
}

int dcf_eval_prefix_levels(const dcf_prg* p, size_t n_bytes, size_t num_keys, size_t points_per_key) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  const uint64_t total = (uint64_t)num_keys * points_per_key;
  // the paths eval_launch takes without a table: small batches (MMO: at auto depth; Hirose: in
  // auto mode), Hirose engines other than the stream engine (MMO ignores the engine setting)
  const Cfg c = snapshot(p);
  const bool small = total < (uint64_t)p->cus * kBlock * 2;
  if (p->kind == 1 && p->lambda > 16) return 0;  // MMO at LAMBDA >= 32: no shared prefix (head/tail per block)
  if (p->kind == 1) return small && c.prefix_levels < 0 ? 0 : (int)prefix_depth(p, c, n_bytes, num_keys, total);
  if (p->lambda > 16)  // batched keys (eval_wide_batch) build no table; per-key passes do
    return wide_batched(p, c, num_keys, points_per_key) ? 0 : (int)wide_prefix_depth(p, c, n_bytes, points_per_key);
  if (c.mode == DCF_EVAL_AUTO && small) return num_keys == 1 ? (int)small_prefix_depth(p, c, n_bytes, total) : 0;
  if (c.mode != DCF_EVAL_AUTO && c.mode != DCF_EVAL_STREAM) return 0;
  return (int)prefix_depth(p, c, n_bytes, num_keys, total);
}

int dcf_prg_set_prefix_max_bytes(dcf_prg* p, size_t max_bytes) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  p->prefix_cap = max_bytes;
  return DCF_OK;
}

size_t dcf_prg_device_bytes(const dcf_prg* p) {
  if (!p) return 0;
  size_t b = 0;
  if (p->d_tab) b += sizeof(g_tab);
  if (p->d_rk128) b += p->rk128_count * 44 * 4;
  if (p->d_rk2) b += 2 * sizeof(RoundKeys);
  if (p->d_rk0) b += sizeof(RoundKeys);
  std::lock_guard<std::mutex> g(const_cast<dcf_prg*>(p)->pool_mu);
  for (const Workspace* w : p->all_ws) {
    if (w->d_ctr) b += kCtrBytes;
    b += (size_t)w->dig_levels * 65 + w->kdig_bytes + w->ws_bytes + w->pfx_bytes +
         w->d_stage_bytes + w->mkey_bytes + w->tctr_bytes;
  }
  return b;
}

size_t dcf_prg_host_pinned_bytes(const dcf_prg* p) {
  if (!p) return 0;
  size_t b = 0;
  std::lock_guard<std::mutex> g(const_cast<dcf_prg*>(p)->pool_mu);
  for (const Workspace* w : p->all_ws) b += w->h_stage_bytes + w->tiny_bytes + w->mid_bytes;
  return b;
}

int dcf_prg_workspaces(const dcf_prg* p) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  std::lock_guard<std::mutex> g(const_cast<dcf_prg*>(p)->pool_mu);
  return (int)p->all_ws.size();
}

// The measurement hooks read the last eval's workspace only while no call holds it: under the
// pool lock (a lease takes that lock to pop the workspace), after the workspace's last device
// work has finished.
static bool ws_idle(const dcf_prg* p, const Workspace* w) {
  return std::find(p->free_ws.begin(), p->free_ws.end(), w) != p->free_ws.end();
}

int dcf_prg_last_eval_blocks(dcf_prg* p, uint64_t* blocks) {
  if (!p || !blocks) return fail(DCF_ERR_ARG, "null argument");
  *blocks = 0;
  Workspace* w = nullptr;
  {  // take the workspace out of the pool (as a lease does), so the drain below holds no lock
    std::lock_guard<std::mutex> g(p->pool_mu);
    w = p->last_ws.load();
    if (!w || !w->d_ctr) return DCF_OK;
    auto it = std::find(p->free_ws.begin(), p->free_ws.end(), w);
    if (it == p->free_ws.end()) return fail(DCF_ERR_ARG, "the last eval's workspace is in use by another call");
    p->free_ws.erase(it);
  }
  int rc = DCF_OK;
  {
    DeviceGuard dg(p->device);
    hipError_t e = w->pending ? hipEventSynchronize(w->done) : hipSuccess;
    if (e == hipSuccess) e = hipMemcpy(blocks, w->d_ctr + 2, sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      rc = fail(DCF_ERR_HIP, std::string("dcf_prg_last_eval_blocks: ") + hipGetErrorString(e));
    } else {
      w->pending = false;  // drained
    }
  }
  std::lock_guard<std::mutex> g(p->pool_mu);
  p->free_ws.push_back(w);
  return rc;
}

int dcf_prg_set_phase_timing(dcf_prg* p, int on) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (on != 0 && on != 1) return fail(DCF_ERR_ARG, "on must be 0 or 1");
  p->timing = on;
  return DCF_OK;
}

int dcf_prg_last_eval_phases(dcf_prg* p, float* prep_ms, float* walk_ms, int* prefix_levels) {
  if (!p || !prep_ms || !walk_ms) return fail(DCF_ERR_ARG, "null argument");
  *prep_ms = *walk_ms = 0.f;
  if (prefix_levels) *prefix_levels = 0;
  std::lock_guard<std::mutex> g(p->pool_mu);
  Workspace* w = p->last_ws.load();
  if (!w || !w->timed) return fail(DCF_ERR_ARG, "no timed eval yet (dcf_prg_set_phase_timing)");
  if (!ws_idle(p, w)) return fail(DCF_ERR_ARG, "the last eval's workspace is in use by another call");
  DeviceGuard dg(p->device);
  HIP_TRY(hipEventElapsedTime(prep_ms, w->tev[0], w->tev[1]));
  HIP_TRY(hipEventElapsedTime(walk_ms, w->tev[1], w->tev[2]));
  if (prefix_levels) *prefix_levels = (int)w->last_prefix;
  return DCF_OK;
}

int dcf_prg_trim(dcf_prg* p) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  std::vector<Workspace*> idle;
  {
    std::lock_guard<std::mutex> g(p->pool_mu);
    idle.swap(p->free_ws);
    for (Workspace* w : idle) p->all_ws.erase(std::find(p->all_ws.begin(), p->all_ws.end(), w));
    Workspace* last = p->last_ws.load();
    if (std::find(idle.begin(), idle.end(), last) != idle.end()) p->last_ws.store(nullptr);
  }
  DeviceGuard dg(p->device);
  for (Workspace* w : idle) free_workspace(w);  // waits for each one's last device work
  return (int)idle.size();
}

// Tiny batches run the latency kernels of kernels_lat.h (one AES column per lane).  Thresholds:
// scripts/lat_sweep.py / row_threshold.py (DESIGN.md §4 "Latency kernels", profiles/AB_LOG.md).
constexpr uint64_t kEvalRowMax = 8192;   // points up to which auto-mode eval runs k_eval16_row (32 lanes per point)
#ifndef DCF_EVAL_ROW2_MAX
#define DCF_EVAL_ROW2_MAX 2048
#endif
constexpr uint64_t kEvalRow2Max = DCF_EVAL_ROW2_MAX;  // ... k_eval16_row2 (64 lanes per point, two levels per
// chain on right steps) up to this many points (r06i, us per device call, row2 vs row: 1 point 75.7 vs
// 97.6, 256 81.9 vs 108.1, 2048 87.4 vs 97.7, 4096 105.1 vs 100.3)
constexpr uint64_t kGenRowMax = 2048;    // keys up to which gen runs k_gen16_row (one wave per key; pipelined, r03t3:
                                         // 2048 keys 110 vs 148 us col, 4096 keys 149 vs 147, 8192 277 vs 165)
constexpr uint64_t kGenColMax = 16384;   // keys up to which gen runs k_gen16_col (r03a: 4096 keys 232 vs 562 us quads)
// Items per workgroup of the latency kernels: a small batch spread over the CUs (one wave per
// CU while it lasts), at most `cap` (a full 1024-thread workgroup).
static uint32_t per_wg(uint64_t items, int cus, uint32_t cap) {
  const uint64_t per = (items + (uint64_t)cus - 1) / (uint64_t)cus;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(cap, per));
}
static bool col_gen(const dcf_prg* p, size_t n_bytes, uint64_t num_keys) {
  return p->kind == 0 && p->lambda == 16 && num_keys <= kGenColMax && 8 * n_bytes <= kColMaxLevels;
}

static int gen_launch(dcf_prg* p, Lease& L, size_t n_bytes, size_t num_keys, const uint8_t* alpha,
                      const uint8_t* beta, const uint8_t* s0_0, const uint8_t* s0_1, int bound, uint8_t* cwb_out) {
  Workspace* w = L.w;
  hipStream_t st = L.st;
  const size_t n = 8 * n_bytes, lam = p->lambda;
  uint8_t* cws = cwb_out;
  uint8_t* cwv = cwb_out + n * num_keys * lam;
  uint8_t* cwt = cwb_out + 2 * n * num_keys * lam;
  uint8_t* np1 = cwb_out + dcf_cwb_np1_offset(n_bytes, lam, num_keys);
  if (p->kind == 1 && lam > 16) return gen_mmo_wide(p, w, n_bytes, num_keys, alpha, beta, s0_0, s0_1, bound, cws, cwv,
                                                    cwt, np1, st);
  if (p->kind == 1) {  // Aes128MatyasMeyerOseasPrg (LAMBDA = 16)
    hipLaunchKernelGGL(k_gen16_mmo, dim3((unsigned)grid_for(num_keys, p->cus)), dim3(kBlock), 0, st, p->d_tab,
                       p->d_rk128, alpha, (const uint4*)beta, (const uint4*)s0_0, (const uint4*)s0_1, (uint32_t)bound,
                       (uint32_t)n_bytes, (uint64_t)num_keys, (uint4*)cws, (uint4*)cwv, cwt, (uint4*)np1);
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  if (lam > 16) {  // one workgroup per key, keys in chunks (scratch 3*LAMBDA per key)
    const uint64_t chunk = num_keys < kGenChunk ? num_keys : kGenChunk;
    int rc = ensure_ws(w, chunk * 3 * lam, st);
    if (rc) return rc;
    for (uint64_t k0 = 0; k0 < num_keys; k0 += chunk) {
      const uint64_t cnt = (num_keys - k0 < chunk) ? num_keys - k0 : chunk;
      hipLaunchKernelGGL(k_gen_wide, dim3((unsigned)cnt), dim3(kBlock), 0, st, p->d_tab, p->d_rk2, alpha,
                         beta, s0_0, s0_1, (uint32_t)bound, (uint32_t)n_bytes, (uint64_t)num_keys, k0, (uint32_t)lam,
                         cws, cwv, cwt, np1, w->d_ws);
      HIP_TRY(hipGetLastError());
    }
    return DCF_OK;
  }
  if (col_gen(p, n_bytes, num_keys) && num_keys <= kGenRowMax) {
    // The smallest batches: one wave per key, one table lookup per lane and AES round
    // (k_gen16_row: a lone key's level is one 16-lane AES chain).
    const uint32_t kpw = per_wg(num_keys, p->cus, kBlock / 64);
    hipLaunchKernelGGL(k_gen16_row, dim3((unsigned)((num_keys + kpw - 1) / kpw)), dim3(kBlock), 0, st, p->d_tab,
                       p->rk[0], alpha, beta, s0_0, s0_1, (uint32_t)bound, (uint32_t)n_bytes, kpw,
                       (uint64_t)num_keys, cws, cwv, cwt, np1);
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  if (col_gen(p, n_bytes, num_keys)) {
    // Small batches (a single key through the C ABI: benches/dcf.rs bench_gen) are latency-
    // bound: 16 lanes per key, one AES column each (k_gen16_col).
    const uint32_t kpw = per_wg(num_keys, p->cus, kBlock / 16);
    hipLaunchKernelGGL(k_gen16_col, dim3((unsigned)((num_keys + kpw - 1) / kpw)), dim3(kBlock), 0, st, p->d_tab,
                       p->rk[0], alpha, beta, s0_0, s0_1, (uint32_t)bound, (uint32_t)n_bytes, kpw,
                       (uint64_t)num_keys, cws, cwv, cwt, np1);
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  // Large batches: 64-lane units from the work counter (waves drift apart, as in k_eval16).
  // Lanes per key: a quad while the batch leaves lanes idle (a key's 8N levels take a quarter of
  // the AES latency: single gen 826 -> 266 us), one lane per key for large batches (2^20 keys:
  // 7.5-7.6 ms with one lane, 8.0 with quads — the four lanes repeat the level update).
  const bool quad = (uint64_t)num_keys <= (uint64_t)p->cus * kBlock / 2;
  const uint64_t items = (uint64_t)num_keys * (quad ? 4u : 1u);
  uint32_t* ctr = nullptr;
  if (items >= (uint64_t)p->cus * kBlock * 2 && (items + 63) / 64 <= 0xFFFFFFFFull) {
    if (int rc = ensure_ctr(w)) return rc;
    HIP_TRY(hipMemsetAsync(w->d_ctr, 0, kCtrBytes, st));
    ctr = w->d_ctr;
  }
  // Round keys in SGPRs (22 / 26 SGPR spills into VGPR lanes in the one-lane / quad instances):
  // per-round keys from the device copy spill none but gen ran 1-1.5 % slower (C5 r05l).
#define DCF_GEN16(LN)                                                                                           \
  hipLaunchKernelGGL(k_gen16<LN>, dim3((unsigned)grid_for(items, p->cus)), dim3(kBlock), 0, st, p->d_tab, p->rk[0], \
                     alpha, (const uint4*)beta, (const uint4*)s0_0, (const uint4*)s0_1, (uint32_t)bound,          \
                     (uint32_t)n_bytes, (uint64_t)num_keys, (uint4*)cws, (uint4*)cwv, cwt, (uint4*)np1, ctr)
  if (quad) DCF_GEN16(4);
  else DCF_GEN16(1);
#undef DCF_GEN16
  HIP_TRY(hipGetLastError());
  return DCF_OK;
}

int dcf_gen_batch_device(dcf_prg* p, size_t n_bytes, size_t num_keys, const uint8_t* alpha, const uint8_t* beta,
                         const uint8_t* s0_0, const uint8_t* s0_1, int bound, uint8_t* cwb_out, void* stream) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (bound != DCF_BOUND_LT_BETA && bound != DCF_BOUND_GT_BETA) return fail(DCF_ERR_ARG, "bad bound");
  if (num_keys == 0) return DCF_OK;
  if (!alpha || !beta || !s0_0 || !s0_1 || !cwb_out) return fail(DCF_ERR_ARG, "null buffer");
  DeviceGuard dg(p->device);
  Lease L(p);
  if (int rc = L.order((hipStream_t)stream)) return rc;
  return gen_launch(p, L, n_bytes, num_keys, alpha, beta, s0_0, s0_1, bound, cwb_out);
}

// Dcf::eval of K keys x ppk points on the lease's stream (arguments checked by the caller).
// Phase marks (dcf_prg_set_phase_timing): 0 at entry, 1 before the walk kernel (after any
// table / digest preparation), 2 at the end.
static int eval_body(dcf_prg* p, Lease& L, size_t n_bytes, size_t num_keys, size_t ppk, int party, const uint8_t* cwb,
                     const uint8_t* s0s, const uint8_t* xs, uint8_t* ys);

#ifndef DCF_SK_PFX
#define DCF_SK_PFX 1
#endif
// Single key below a shared-prefix table (C2 / C3 shapes): the instance whose starts all take the
// table row (PFX), so the fresh-x-word path (4 selects per stream and step) is compiled out; 87 ->
// 74 SGPRs.  r05v A/B (same box, 3 alternating runs): C3 491.3-491.7 vs 493.1-493.9 ms, C2
// 3.354-3.360 vs 3.391-3.396 ms (round 2's attempt at this split lost to a register-allocation flip).
constexpr bool kSkPfx = DCF_SK_PFX;
#ifndef DCF_STG
#define DCF_STG 1
#endif
// N <= 4 single key below the table (C2): prefix rows staged two iterations ahead into LDS by DMA
// (kernels_stream.h STG) instead of gathered at each point start.
constexpr bool kStg = DCF_STG;
#ifndef DCF_MK_NBC16
#define DCF_MK_NBC16 1
#endif
constexpr bool kMkNbc16 = DCF_MK_NBC16;  // A/B knob: the N = 16 multi-key top-tree instance
#ifndef DCF_MK_PK2
#define DCF_MK_PK2 1
#endif
// ... and of it, for a power-of-two points per key (C5: 64), point -> key by a shift instead of
// the division sequence (65 fewer VALU in the kernel)
constexpr bool kMkPk2 = DCF_MK_PK2;
#ifndef DCF_MK_NBC4
#define DCF_MK_NBC4 1
#endif
constexpr bool kMkNbc4 = DCF_MK_NBC4;  // A/B knob: the N = 4 multi-key top-tree instance (C5 at N = 4)

static int eval_launch(dcf_prg* p, Lease& L, size_t n_bytes, size_t num_keys, size_t ppk, int party,
                       const uint8_t* cwb, const uint8_t* s0s, const uint8_t* xs, uint8_t* ys) {
  if (int rc = ensure_ctr(L.w)) return rc;
  // the block count (dcf_prg_last_eval_blocks) covers the whole call: zeroed once here (the
  // latency kernels zero it themselves: one command less on a ~100 us call).  The decision and
  // eval_body's engine choice read the same settings snapshot (L.c).
  if (!oct_eval(p, L.c, n_bytes, num_keys, (uint64_t)num_keys * ppk))
    HIP_TRY(hipMemsetAsync(L.w->d_ctr, 0, kCtrBytes, L.st));
  L.w->last_prefix = 0;
  phase_mark(p, L, 0);
  const int rc = eval_body(p, L, n_bytes, num_keys, ppk, party, cwb, s0s, xs, ys);
  phase_mark(p, L, 2);
  p->last_ws.store(L.w);
  return rc;
}

// Multi-key stream eval: keys per launch.  The kernel's work distribution, point and digest-row
// indices are 32-bit (kernels_stream.h StreamLane): a launch covers < 2^31 points, and its digest
// rows key * 8N + level index uint4 pairs (2 * row < 2^31), so at most 2^30 / 8N keys.
static uint64_t mk_keys_per_launch(size_t n_bytes, uint64_t ppk) {
  return std::max<uint64_t>(1, std::min<uint64_t>({1ull << 24, (1ull << 31) / ppk, (1ull << 30) / (8 * n_bytes)}));
}

size_t dcf_eval_keys_per_launch(size_t n_bytes, size_t points_per_key) {
  if (n_bytes == 0 || points_per_key == 0) return 0;
  return (size_t)mk_keys_per_launch(n_bytes, points_per_key);
}

static int eval_body(dcf_prg* p, Lease& L, size_t n_bytes, size_t num_keys, size_t ppk, int party, const uint8_t* cwb,
                     const uint8_t* s0s, const uint8_t* xs, uint8_t* ys) {
  Workspace* w = L.w;
  const Cfg& c = L.c;
  hipStream_t st = L.st;
  const uint64_t total = (uint64_t)num_keys * ppk;
  const size_t n = 8 * n_bytes, lam = p->lambda;
  if (lam > 16) {  // head/tail pipeline: keys with few points batched, else per key
    phase_mark(p, L, 1);
    if (wide_batched(p, c, num_keys, ppk))
      return eval_wide_batch(p, w, n_bytes, num_keys, ppk, party, cwb, s0s, xs, ys, st);
    for (uint64_t k = 0; k < num_keys; ++k) {
      int rc = p->kind == 1 ? eval_mmo_wide(p, w, n_bytes, num_keys, k, party, cwb, s0s + k * lam,
                                            xs + k * ppk * n_bytes, ppk, ys + k * ppk * lam, st)
                            : eval_wide(p, c, w, n_bytes, num_keys, k, party, cwb, s0s + k * lam,
                                        xs + k * ppk * n_bytes, ppk, ys + k * ppk * lam, st);
      if (rc) return rc;
    }
    return DCF_OK;
  }
  const uint4* cws = (const uint4*)cwb;
  const uint4* cwv = (const uint4*)(cwb + n * num_keys * lam);
  const uint8_t* cwt = cwb + 2 * n * num_keys * lam;
  const uint4* np1 = (const uint4*)(cwb + dcf_cwb_np1_offset(n_bytes, lam, num_keys));
  const dim3 grid((unsigned)grid_for(total, p->cus)), block(kBlock);
  if (p->kind == 1) {  // MMO: lockstep, two blocks per level (the side's s and v), any engine setting
#define DCF_MMO(MODE)                                                                                          \
  hipLaunchKernelGGL(k_eval16_mmo<MODE>, grid, block, 0, st, p->d_tab, p->d_rk128, cws, cwv, cwt, np1,            \
                     (const uint4*)s0s, (uint32_t)party, xs, (uint32_t)n_bytes, (uint64_t)num_keys, (uint64_t)ppk, \
                     (uint4*)ys, pf)
    PrefixTable pf{nullptr, 0u};
    // auto depth: none for small batches (latency-bound: the table's D launches cost what it saves)
    if (num_keys == 1 && (c.prefix_levels > 0 || total >= (uint64_t)p->cus * kBlock * 2)) {
      const uint32_t d = prefix_depth(p, c, n_bytes, num_keys, total);
      if (d) {
        int rc = try_prefix(p, c, w, n_bytes, party, cws, cwv, cwt, np1, s0s, d, &pf, st);
        if (rc) return rc;
        w->last_prefix = pf.levels;
      }
    }
    phase_mark(p, L, 1);
    if (num_keys == 1) DCF_MMO(0);
    else if (ppk % 64 == 0) DCF_MMO(1);
    else DCF_MMO(2);
#undef DCF_MMO
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  int mode = c.mode;
  if (oct_eval(p, c, n_bytes, num_keys, total) && total <= kEvalRow2Max) {
    // The very smallest batches: one wave per point, two levels per AES chain on right steps
    // (k_eval16_row2: rows 2 / 3 encrypt the right successor's blocks alongside the level's own).
    phase_mark(p, L, 1);
    const uint32_t ppw = per_wg(total, p->cus, kBlock / 64);
    hipLaunchKernelGGL(k_eval16_row2, dim3((unsigned)((total + ppw - 1) / ppw)), dim3(kBlock), 0, st, p->d_tab,
                       p->rk[0], cwb, s0s, (uint32_t)party, xs, (uint32_t)n_bytes, ppw, (uint64_t)total, ys, w->d_ctr);
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  if (oct_eval(p, c, n_bytes, num_keys, total) && total <= kEvalRowMax) {
    // The smallest batches: 32 lanes per point, one table lookup per lane and AES round
    // (k_eval16_row: a lone point's level is one 16-lane AES chain).
    phase_mark(p, L, 1);
    const uint32_t ppw = per_wg(total, p->cus, kBlock / 32);
    hipLaunchKernelGGL(k_eval16_row, dim3((unsigned)((total + ppw - 1) / ppw)), dim3(kBlock), 0, st, p->d_tab,
                       p->rk[0], cwb, s0s, (uint32_t)party, xs, (uint32_t)n_bytes, ppw, (uint64_t)total, ys, w->d_ctr);
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  if (oct_eval(p, c, n_bytes, num_keys, total)) {
    // Tiny batches (a single point through the C ABI: benches/dcf.rs bench_eval) are latency-
    // bound: 8 lanes per point, one AES column each, A and B side by side (k_eval16_oct).
    phase_mark(p, L, 1);
    const uint32_t ppw = per_wg(total, p->cus, kBlock / 8);
    hipLaunchKernelGGL(k_eval16_oct, dim3((unsigned)((total + ppw - 1) / ppw)), dim3(kBlock), 0, st, p->d_tab,
                       p->rk[0], cwb, s0s, (uint32_t)party, xs, (uint32_t)n_bytes, ppw, (uint64_t)total, ys, w->d_ctr);
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  // Auto: small batches (fewer points than two per lane of the GPU) are latency-bound: one
  // point's 8N levels run back to back, so the lockstep walk (A and B of a level in one AES
  // pass: 8N passes) beats the stream engine (~12N passes); it runs on a lane pair per point
  // (k_eval16_pair: the even lane encrypts A, the odd lane B), spread over every CU with
  // workgroups just big enough (C1).  Larger batches: the stream engine, single key or many
  // (C3 r01: 407 M evals/s vs 332 M lockstep T-table; C5 with the key-major digest).  DCF_EVAL_TTABLE
  // forces the lockstep walk (k_eval16: A and B every level), which auto takes for many keys at N > 32.
  if (mode == DCF_EVAL_AUTO && total < (uint64_t)p->cus * kBlock * 2) {
    PrefixTable spf{nullptr, 0u};
    if (num_keys == 1) {
      const uint32_t d = small_prefix_depth(p, c, n_bytes, total);
      if (d) {
        int rc = try_prefix(p, c, w, n_bytes, party, cws, cwv, cwt, np1, s0s, d, &spf, st);
        if (rc) return rc;
        w->last_prefix = spf.levels;
      }
    }
    phase_mark(p, L, 1);
    // Whole waves per workgroup.  r06c (C1, same box, 4 alternating runs): rounding the lanes to a
    // pair instead, so that all 256 CUs get a workgroup (782 lanes, the last wave partial) rather than
    // 241 (13 whole waves), ran 0.913-0.915 vs 0.894-0.895 ms per step.
    uint64_t threads = (total * 2 + p->cus - 1) / p->cus;
    threads = ((threads + 63) / 64) * 64;
    if (threads > (uint64_t)kBlock) threads = kBlock;
    const dim3 g2((unsigned)((total * 2 + threads - 1) / threads)), b2((unsigned)threads);
#define DCF_SMALL(MODE)                                                                                           \
  hipLaunchKernelGGL(k_eval16_pair<MODE>, g2, b2, 0, st, p->d_tab, p->rk[0], cws, cwv, cwt, np1,                  \
                     (const uint4*)s0s, (uint32_t)party, xs, (uint32_t)n_bytes, (uint64_t)num_keys, (uint64_t)ppk,  \
                     (uint4*)ys, p->d_rk0, MODE == 0 ? spf : PrefixTable{nullptr, 0u})
    // (r06i: a per-lane block schedule for one key, k_eval16_pair2 — ~100 instead of 128 AES passes
    // per wave by simulation — ran 31 % slower on C1 and was removed; AB_LOG round 6)
    if (num_keys == 1) DCF_SMALL(0);
    else if (ppk % 64 == 0) DCF_SMALL(1);
    else DCF_SMALL(2);
#undef DCF_SMALL
    HIP_TRY(hipGetLastError());
    return DCF_OK;
  }
  if (mode == DCF_EVAL_AUTO) mode = (num_keys == 1 || n_bytes <= 32) ? DCF_EVAL_STREAM : DCF_EVAL_TTABLE;
  if (mode == DCF_EVAL_STREAM && num_keys > 1 && n_bytes > 32)
    return fail(DCF_ERR_UNSUPPORTED, "multi-key stream eval: N <= 32");
  if (mode == DCF_EVAL_STREAM) {
    constexpr int NS = 2;  // streams per lane
    const bool xreg = n_bytes % 4 == 0 && n_bytes <= 16, multi = num_keys > 1;
    if (multi && ppk >= (1ull << 31)) return fail(DCF_ERR_UNSUPPORTED, "multi-key stream eval: 2^31 points per key or more");
    const uint4* scs = cws;
    const uint8_t* sct = cwt;
    PrefixTable pf{nullptr, 0u};
    if (multi && c.prefix_levels != 0 && n > kMkPfxLevels && ppk >= 32 && num_keys <= (1ull << (31 - kMkPfxLevels))) {
      // per-key top trees (k_mk_prefix16: 32 rows per key); no room -> walk from the root (same bytes)
      const size_t need = (size_t)num_keys * (32u << kMkPfxLevels);
      if (w->pfx_bytes < need) {
        if (w->d_pfx) {
          HIP_TRY(hipStreamSynchronize(st));
          HIP_TRY(hipFree(w->d_pfx));
          w->d_pfx = nullptr;
          w->pfx_bytes = 0;
        }
        if (hipMalloc(&w->d_pfx, need) != hipSuccess) {
          (void)hipGetLastError();
        } else {
          w->pfx_bytes = need;
        }
      }
      if (w->pfx_bytes >= need) {
        pf = PrefixTable{(const uint4*)w->d_pfx, kMkPfxLevels};
        w->last_prefix = kMkPfxLevels;
      }
    }
    if (multi) {
      // The top trees (k_mk_prefix16: LDS-bound AES, 128 KiB of LDS per workgroup) on the
      // workspace's second stream while the key-major digest (kernels_stream.h: memory-bound,
      // 17 KiB per workgroup, so one fits beside a top-tree workgroup on a CU) is written on the
      // call's stream; the walk waits for both.
      if (int rc = grow(&w->d_kdig, &w->kdig_bytes, (size_t)num_keys * n * 33, st)) return rc;
      const bool fork = pf.levels != 0;
      // Once the top trees are queued on aux, every exit from this block — the normal one and an
      // error return — joins aux into the call's stream (the walk and the lease's `done` event must
      // cover them: the next user of this workspace overwrites d_pfx / d_ctr); if the join cannot
      // be queued, aux is drained on the host instead.
      struct AuxJoin {
        Workspace* w;
        hipStream_t st;
        bool armed = false;
        ~AuxJoin() {
          if (!armed) return;
          if (hipEventRecord(w->aux_ev[1], w->aux) != hipSuccess || hipStreamWaitEvent(st, w->aux_ev[1], 0) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipStreamSynchronize(w->aux);
          }
        }
      } join{w, st};
      if (fork) {
        if (!w->aux) HIP_TRY(hipStreamCreateWithFlags(&w->aux, hipStreamNonBlocking));
        for (auto& e : w->aux_ev)
          if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(w->aux_ev[0], st));
        HIP_TRY(hipStreamWaitEvent(w->aux, w->aux_ev[0], 0));
        join.armed = true;
        hipLaunchKernelGGL(k_mk_prefix16<true>,
                           dim3((unsigned)(((num_keys << kMkPfxRoot) + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           w->aux, p->d_tab, p->rk[0], cws, cwv, cwt, (const uint4*)s0s, (uint32_t)party,
                           (uint64_t)num_keys, (uint4*)w->d_pfx, p->d_rk0, w->d_ctr);
        HIP_TRY(hipGetLastError());
      }
      hipLaunchKernelGGL(k_cw_keymajor, dim3((unsigned)((num_keys + kKmKeys - 1) / kKmKeys), (unsigned)((n + kKmLevs - 1) / kKmLevs)),
                         dim3(kKmThreads), 0, st, cws, cwv, cwt, (uint32_t)n, (uint64_t)num_keys, (uint4*)w->d_kdig,
                         w->d_kdig + (size_t)num_keys * n * 32);
      HIP_TRY(hipGetLastError());
      // (the join runs here, as `join` leaves scope: the walk below waits for the top trees)
      scs = (const uint4*)w->d_kdig;
      sct = w->d_kdig + (size_t)num_keys * n * 32;
    }
    if (!multi) {
      const uint32_t d = prefix_depth(p, c, n_bytes, num_keys, total);
      if (d) {
        int rc = try_prefix(p, c, w, n_bytes, party, cws, cwv, cwt, np1, s0s, d, &pf, st);
        if (rc) return rc;
        w->last_prefix = pf.levels;
      }
    }
    phase_mark(p, L, 1);
    // One launch covers < 2^31 points (multi-key: mk_keys_per_launch whole keys).  Larger
    // batches run as several launches over consecutive points / whole keys, sharing the table
    // and digest built above.
    const uint64_t kpl = multi ? mk_keys_per_launch(n_bytes, ppk) : 1;
    const uint64_t ppl = multi ? kpl * ppk : (1ull << 31);  // points per launch
    for (uint64_t c0 = 0; c0 < total; c0 += ppl) {
      const uint64_t cnt = std::min<uint64_t>(ppl, total - c0), k0 = multi ? c0 / ppk : 0, kc = multi ? cnt / ppk : 1;
      // each walk's work counter starts at 0 (the block count beside it keeps the per-key top
      // trees' blocks): eval_launch zeroed it for the first launch (the table builds and the
      // digest do not touch it), so a one-launch eval has no fill between the build and the walk
      if (c0 > 0) HIP_TRY(hipMemsetAsync(w->d_ctr, 0, 8, st));
      const uint64_t units = (cnt + kStreamUnit - 1) / kStreamUnit;
      uint64_t blocks = (units + 15) / 16;
      if (blocks > (uint64_t)p->cus) blocks = (uint64_t)p->cus;
      const uint4* lcs = multi ? scs + k0 * 2 * n : scs;
      const uint8_t* lct = multi ? sct + k0 * n : sct;
      const uint4* lnp1 = np1 + k0;
      const uint8_t* lxs = xs + c0 * n_bytes;
      uint8_t* lys = ys + c0 * lam;
      const uint8_t* ls0 = s0s + k0 * lam;
      const PrefixTable lpf = (multi && pf.levels) ? PrefixTable{pf.sv + 2 * (k0 << pf.levels), pf.levels} : pf;
#define DCF_STREAM(XR, MK, PF, NBC) DCF_STREAM7(XR, MK, PF, NBC, false, false)
#define DCF_STREAM6(XR, MK, PF, NBC, PK2) DCF_STREAM7(XR, MK, PF, NBC, PK2, false)
#define DCF_STREAM7(XR, MK, PF, NBC, PK2, STG)                                                                  \
  hipLaunchKernelGGL((k_eval16_stream<NS, XR, MK, PF, NBC, PK2, STG>), dim3((unsigned)blocks), block, 0, st, p->d_tab, \
                     p->rk[0],                                                                                 \
                     lcs, cwv, lct, lnp1, (const uint4*)ls0, (uint32_t)party, lxs, (uint32_t)n_bytes, (uint64_t)kc, \
                     (uint64_t)ppk, (uint64_t)cnt, w->d_ctr, (uint4*)lys, lpf, p->d_rk0)
      // multi-key: an instance for "per-key top trees present" (no root-seed start path: 48 -> 33
      // SGPR spills; C5 r03c A/B 414.6 / 413.7 vs 408.5 / 408.1 M evals/s), and of it one with the
      // x width fixed at N = 16 (C5: 33 -> 18 SGPR spills, 121 -> 119 VGPRs, r05k).  Single key, x in
      // registers: N = 16 (C1 / C3) and N = 4 (C2) with the x width fixed at compile time (a
      // point's start loads x without width branches: C2 starts a point every ~13 AES slots).
      if (multi && lpf.levels) {
        if (xreg && n_bytes == 16 && kMkNbc16 && kMkPk2 && (ppk & (ppk - 1)) == 0) DCF_STREAM6(true, true, true, 16, true);
        else if (xreg && n_bytes == 16 && kMkNbc16) DCF_STREAM(true, true, true, 16);
        else if (xreg && n_bytes == 4 && kMkNbc4 && (ppk & (ppk - 1)) == 0) DCF_STREAM6(true, true, true, 4, true);
        else if (xreg) DCF_STREAM(true, true, true, 0);
        else DCF_STREAM(false, true, true, 0);
      } else if (multi) {
        if (xreg) DCF_STREAM(true, true, false, 0);
        else DCF_STREAM(false, true, false, 0);
      } else if (xreg && n_bytes == 16 && lpf.levels && kSkPfx) {
        DCF_STREAM(true, false, true, 16);  // every start below the shared prefix: no fresh-x-word path
      } else if (xreg && n_bytes == 16) {
        DCF_STREAM(true, false, false, 16);
      } else if (xreg && n_bytes == 4 && lpf.levels && kSkPfx && kStg) {
        DCF_STREAM7(true, false, true, 4, false, true);  // rows staged two iterations ahead (C2)
      } else if (xreg && n_bytes == 4 && lpf.levels && kSkPfx) {
        DCF_STREAM(true, false, true, 4);
      } else if (xreg && n_bytes == 4) {
        DCF_STREAM(true, false, false, 4);
      } else if (xreg) {
        DCF_STREAM(true, false, false, 0);
      } else {
        DCF_STREAM(false, false, false, 0);
      }
#undef DCF_STREAM
#undef DCF_STREAM6
#undef DCF_STREAM7
      HIP_TRY(hipGetLastError());
    }
  } else {  // lockstep T-table, 64-point units from the work counter
    if ((total + 63) / 64 > 0xFFFFFFFFull) return fail(DCF_ERR_UNSUPPORTED, "more than 2^32 64-point units");
    phase_mark(p, L, 1);
#define DCF_TT(MODE)                                                                                         \
  hipLaunchKernelGGL(k_eval16<MODE>, grid, block, 0, st, p->d_tab, p->rk[0], cws, cwv, cwt, np1,               \
                     (const uint4*)s0s, (uint32_t)party, xs, (uint32_t)n_bytes, (uint64_t)num_keys, (uint64_t)ppk, \
                     (uint4*)ys, w->d_ctr)
    if (num_keys == 1) DCF_TT(0);
    else if (ppk % 64 == 0) DCF_TT(1);
    else DCF_TT(2);
#undef DCF_TT
  }
  HIP_TRY(hipGetLastError());
  return DCF_OK;
}

static int check_eval_args(dcf_prg* p, size_t n_bytes, int party, uint64_t total, const void* cwb, const void* s0s,
                           const void* xs, const void* ys) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (party != 0 && party != 1) return fail(DCF_ERR_ARG, "party must be 0 or 1");
  if (total && (!cwb || !s0s || !xs || !ys)) return fail(DCF_ERR_ARG, "null buffer");
  return DCF_OK;
}

int dcf_eval_device(dcf_prg* p, size_t n_bytes, int party, const uint8_t* cwb, const uint8_t* s0,
                    const uint8_t* xs, size_t m, uint8_t* ys, void* stream) {
  if (int rc = check_eval_args(p, n_bytes, party, m, cwb, s0, xs, ys)) return rc;
  if (m == 0) return DCF_OK;
  DeviceGuard dg(p->device);
  Lease L(p);
  if (int rc = L.order((hipStream_t)stream)) return rc;
  return eval_launch(p, L, n_bytes, 1, m, party, cwb, s0, xs, ys);
}

int dcf_eval_multikey_device(dcf_prg* p, size_t n_bytes, size_t num_keys, size_t points_per_key, int party,
                             const uint8_t* cwb, const uint8_t* s0s, const uint8_t* xs, uint8_t* ys,
                             void* stream) {
  const uint64_t total = (uint64_t)num_keys * points_per_key;
  if (int rc = check_eval_args(p, n_bytes, party, total, cwb, s0s, xs, ys)) return rc;
  if (total == 0) return DCF_OK;
  DeviceGuard dg(p->device);
  Lease L(p);
  if (int rc = L.order((hipStream_t)stream)) return rc;
  return eval_launch(p, L, n_bytes, num_keys, points_per_key, party, cwb, s0s, xs, ys);
}

// ---- host-pointer path: per-workspace streams and staging, chunked pipeline ----

static size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

// Points per chunk of the host eval pipeline: ~128 MiB of x + y per buffer (C3 shape: 4 Mi
// points, an 8 ms kernel against ~3 ms of PCIe each way, so the copies hide behind it).
constexpr size_t kHostChunkBytes = 128ull << 20;
// Tiny host calls (the latency kernels' batch sizes): inputs and outputs through one pinned,
// device-mapped buffer that the kernel reads and writes itself — one launch, no copy commands.
constexpr size_t kTinyBytes = 1ull << 20;
constexpr size_t kHostMidBytes = 64ull << 20;  // x + y of a mid-size host eval through the mapped buffer

static int ensure_host_path(Workspace* w) {
  if (w->hs[0]) return DCF_OK;
  hipStream_t hs[3] = {nullptr, nullptr, nullptr};
  for (auto& s : hs) HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (auto& e : w->hev)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (int i = 0; i < 3; ++i) w->hs[i] = hs[i];
  return DCF_OK;
}

static int ensure_stage(Workspace* w, size_t hbytes, size_t dbytes) {
  if (w->h_stage_bytes < hbytes) {
    if (w->h_stage) HIP_TRY(hipHostFree(w->h_stage));
    w->h_stage = nullptr;
    w->h_stage_bytes = 0;
    HIP_TRY(hipHostMalloc((void**)&w->h_stage, hbytes, hipHostMallocDefault));
    w->h_stage_bytes = hbytes;
  }
  if (w->d_stage_bytes < dbytes) {
    if (w->d_stage) HIP_TRY(hipFree(w->d_stage));
    w->d_stage = nullptr;
    w->d_stage_bytes = 0;
    HIP_TRY(hipMalloc(&w->d_stage, dbytes));
    w->d_stage_bytes = dbytes;
  }
  return DCF_OK;
}

// The tiny-call buffer: coherent (the kernel's stores are visible once the stream has passed
// it) and mapped into the device's address space.  Returns its device address.
static int ensure_tiny(Workspace* w, uint8_t** dptr) {
  if (!w->h_tiny) {
    HIP_TRY(hipHostMalloc((void**)&w->h_tiny, kTinyBytes, hipHostMallocMapped | hipHostMallocCoherent));
    w->tiny_bytes = kTinyBytes;
  }
  HIP_TRY(hipHostGetDevicePointer((void**)dptr, w->h_tiny, 0));
  return DCF_OK;
}

// The mid-size host buffer: mapped into the device's address space, coarse-grained (the GPU may
// cache it; the host reads the outputs only after the stream has passed the kernel; fine-grained
// measured the same, r03y2 C1 host path 143-148 vs 141-146 M evals/s).  Grown on demand and kept.
// Returns its device address.
static int ensure_mid(Workspace* w, size_t bytes, uint8_t** dptr) {
  if (w->mid_bytes < bytes) {
    if (w->h_mid) HIP_TRY(hipHostFree(w->h_mid));
    w->h_mid = nullptr;
    w->mid_bytes = 0;
    HIP_TRY(hipHostMalloc((void**)&w->h_mid, bytes,
                          hipHostMallocMapped | hipHostMallocNonCoherent));
    w->mid_bytes = bytes;
  }
  HIP_TRY(hipHostGetDevicePointer((void**)dptr, w->h_mid, 0));
  return DCF_OK;
}

// Every host entry point ends here: wait for the workspace's own streams only (never the
// whole device), also after an error, so no queued copy still targets the staging buffers.
static int host_finish(Lease& L, int rc) {
  Workspace* w = L.w;
  bool ok = true;
  for (int i = 0; i < 3; ++i) {
    if (!w->hs[i] || !((w->host_streams >> i) & 1u)) continue;
    const hipError_t e = hipStreamSynchronize(w->hs[i]);
    if (e != hipSuccess) {
      ok = false;
      (void)hipGetLastError();
      if (rc == DCF_OK) rc = fail(DCF_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
    }
  }
  w->host_streams = 0;
  L.drained = ok;
  return rc;
}

// A lease for a host entry point: its workspace's streams exist and the compute stream is
// ordered after the workspace's earlier device work (a *_device call on any stream).
static int host_lease(Lease& L) {
  if (int rc = ensure_host_path(L.w)) return rc;
  L.w->host_streams = 2u;  // the compute stream; the chunked eval pipeline adds copy-in / copy-out
  return L.order(L.w->hs[1]);
}

// Dcf::eval over host buffers (caller: DeviceGuard held, arguments checked, m > 0).
// Tiny batches: one launch of a latency kernel (k_eval16_row / k_eval16_oct) that reads the key and points from, and writes
// the outputs to, the workspace's mapped pinned buffer.  Otherwise chunks of `chunk` points
// flow through two staging slots on three streams: copy-in (pinned -> device), compute
// (eval_launch), copy-out (device -> pinned); the host copies chunk c's x into pinned memory
// and chunk c-1's y out of it while the GPU works on chunk c, so PCIe transfers overlap the
// kernels of neighbouring chunks.  The GPU never touches caller memory.
static int host_eval(dcf_prg* p, Lease& L, size_t nb, int party, const uint8_t* cwb, size_t cwb_len,
                     const uint8_t* s0, const uint8_t* xs, uint64_t m, uint8_t* ys) {
  Workspace* w = L.w;
  const size_t lam = p->lambda;
  const size_t ko = 0, so0 = align256(cwb_len), xo = so0 + 256, yo = xo + align256(m * nb);
  if (oct_eval(p, L.c, nb, 1, m) && yo + m * lam <= kTinyBytes) {
    uint8_t* d = nullptr;
    if (int rc = ensure_tiny(w, &d)) return rc;
    uint8_t* h = w->h_tiny;
    memcpy(h + ko, cwb, cwb_len);
    memcpy(h + so0, s0, lam);
    memcpy(h + xo, xs, m * nb);
    if (int rc = eval_launch(p, L, nb, 1, m, party, d + ko, d + so0, d + xo, d + yo)) return rc;
    HIP_TRY(hipStreamSynchronize(L.st));
    memcpy(ys, h + yo, m * lam);
    return DCF_OK;
  }
  // Mid-size batches (the small-batch kernels' range, LAMBDA = 16): the kernel reads x from and
  // writes y to a mapped pinned buffer, so the call is one host copy in, a 4 KiB key copy, one
  // launch, one stream sync and one host copy out — no staging DMAs or chunk events (a C1-size
  // call is one chunk, its copies cannot overlap its kernel anyway).  The key goes to device
  // memory first: the walk reads a correction word per level.
  if (lam == 16 && L.c.mode == DCF_EVAL_AUTO && m < (uint64_t)p->cus * kBlock * 2 &&
      m * (nb + lam) <= kHostMidBytes) {
    const size_t kb = align256(cwb_len) + align256(lam);
    const size_t mx = align256(m * nb), need = kb + mx + m * lam;
    uint8_t* d = nullptr;
    if (int rc = ensure_mid(w, need, &d)) return rc;
    if (int rc = ensure_stage(w, 0, kb)) return rc;
    uint8_t* h = w->h_mid;
    memcpy(h, cwb, cwb_len);
    memcpy(h + align256(cwb_len), s0, lam);
    memcpy(h + kb, xs, m * nb);
    HIP_TRY(hipMemcpyAsync(w->d_stage, h, kb, hipMemcpyHostToDevice, L.st));
    if (int rc = eval_launch(p, L, nb, 1, m, party, w->d_stage, w->d_stage + align256(cwb_len), d + kb, d + kb + mx))
      return rc;
    HIP_TRY(hipStreamSynchronize(L.st));
    memcpy(ys, h + kb + mx, m * lam);
    return DCF_OK;
  }
  w->host_streams = 7u;
  const uint64_t chunk = std::min<uint64_t>(m, std::max<uint64_t>(256, kHostChunkBytes / (nb + lam)));
  const int nbuf = m > chunk ? 2 : 1;
  const size_t kb = align256(cwb_len) + align256(lam);
  const size_t xb = align256(chunk * nb), yb = align256(chunk * lam);
  if (int rc = ensure_stage(w, nbuf * (xb + yb), kb + nbuf * (xb + yb))) return rc;
  uint8_t* dk = w->d_stage;
  uint8_t* ds0 = dk + align256(cwb_len);
  uint8_t *dx[2], *dy[2], *hx[2], *hy[2];
  for (int b = 0; b < nbuf; ++b) {
    dx[b] = dk + kb + b * xb;
    dy[b] = dk + kb + nbuf * xb + b * yb;
    hx[b] = w->h_stage + b * xb;
    hy[b] = w->h_stage + nbuf * xb + b * yb;
  }
  hipStream_t si = w->hs[0], sc = w->hs[1], so = w->hs[2];
  hipEvent_t *ev_in = w->hev, *ev_k = w->hev + 2, *ev_out = w->hev + 4;
  HIP_TRY(hipMemcpyAsync(dk, cwb, cwb_len, hipMemcpyHostToDevice, sc));
  HIP_TRY(hipMemcpyAsync(ds0, s0, lam, hipMemcpyHostToDevice, sc));
  const uint64_t nch = (m + chunk - 1) / chunk;
  for (uint64_t c = 0; c <= nch; ++c) {
    if (c < nch) {
      const int b = (int)(c & (nbuf - 1));
      const uint64_t off = c * chunk, cnt = std::min<uint64_t>(chunk, m - off);
      if (c >= 2) HIP_TRY(hipEventSynchronize(ev_in[b]));  // chunk c-2's H2D has read hx[b]
      memcpy(hx[b], xs + off * nb, cnt * nb);
      if (c >= 2) HIP_TRY(hipStreamWaitEvent(si, ev_k[b], 0));  // chunk c-2's kernel is done with dx[b]
      HIP_TRY(hipMemcpyAsync(dx[b], hx[b], cnt * nb, hipMemcpyHostToDevice, si));
      HIP_TRY(hipEventRecord(ev_in[b], si));
      HIP_TRY(hipStreamWaitEvent(sc, ev_in[b], 0));
      if (c >= 2) HIP_TRY(hipStreamWaitEvent(sc, ev_out[b], 0));  // chunk c-2's D2H is done with dy[b]
      if (int rc = eval_launch(p, L, nb, 1, cnt, party, dk, ds0, dx[b], dy[b])) return rc;
      HIP_TRY(hipEventRecord(ev_k[b], sc));
      HIP_TRY(hipStreamWaitEvent(so, ev_k[b], 0));
      HIP_TRY(hipMemcpyAsync(hy[b], dy[b], cnt * lam, hipMemcpyDeviceToHost, so));
      HIP_TRY(hipEventRecord(ev_out[b], so));
    }
    if (c >= 1) {  // drain chunk c-1 while chunk c is in flight
      const uint64_t pc = c - 1;
      const int b = (int)(pc & (nbuf - 1));
      const uint64_t off = pc * chunk, cnt = std::min<uint64_t>(chunk, m - off);
      HIP_TRY(hipEventSynchronize(ev_out[b]));
      memcpy(ys + off * lam, hy[b], cnt * lam);
    }
  }
  return DCF_OK;
}

// Dcf::gen for one key over host buffers, on the workspace's compute stream.  Tiny path (the
// column kernel): inputs and the CWB through the mapped pinned buffer, one launch.
static int host_gen(dcf_prg* p, Lease& L, size_t nb, const uint8_t* alpha, const uint8_t* beta, const uint8_t* s0_0,
                    const uint8_t* s0_1, int bound, uint8_t* cwb_out) {
  Workspace* w = L.w;
  const size_t lam = p->lambda, cwb_len = dcf_cwb_bytes(nb, lam, 1);
  const size_t oa = 0, ob = align256(nb), o0 = ob + align256(lam), o1 = o0 + align256(lam), ok = o1 + align256(lam);
  const size_t total = ok + align256(cwb_len);
  const bool tiny = col_gen(p, nb, 1) && total <= kTinyBytes;
  uint8_t *h = nullptr, *d = nullptr;
  if (tiny) {
    if (int rc = ensure_tiny(w, &d)) return rc;
    h = w->h_tiny;
  } else {
    if (int rc = ensure_stage(w, total, total)) return rc;
    h = w->h_stage;
    d = w->d_stage;
  }
  memcpy(h + oa, alpha, nb);
  memcpy(h + ob, beta, lam);
  memcpy(h + o0, s0_0, lam);
  memcpy(h + o1, s0_1, lam);
  hipStream_t sc = L.st;
  if (!tiny) HIP_TRY(hipMemcpyAsync(d, h, ok, hipMemcpyHostToDevice, sc));
  if (!tiny) HIP_TRY(hipMemsetAsync(d + ok, 0, cwb_len, sc));  // the CWB's padding bytes read 0
  int rc = gen_launch(p, L, nb, 1, d + oa, d + ob, d + o0, d + o1, bound, d + ok);
  if (rc) return rc;
  if (!tiny) HIP_TRY(hipMemcpyAsync(h + ok, d + ok, cwb_len, hipMemcpyDeviceToHost, sc));
  HIP_TRY(hipStreamSynchronize(sc));
  memcpy(cwb_out, h + ok, cwb_len);
  if (tiny)  // the CWB's padding bytes (between cw_t and cw_np1) read 0, as on the staged path
    memset(cwb_out + 2 * 8 * nb * lam + 8 * nb, 0, dcf_cwb_np1_offset(nb, lam, 1) - (2 * 8 * nb * lam + 8 * nb));
  return DCF_OK;
}

// Prg::gen for m seeds over host buffers (test hook), on the workspace's compute stream.
static int host_prg_gen(dcf_prg* p, Lease& L, const uint8_t* seeds, size_t m, uint8_t* out) {
  Workspace* w = L.w;
  const size_t lam = p->lambda, row = 4 * lam + 2;
  const size_t so = align256(m * lam), total = so + align256(m * row);
  if (int rc = ensure_stage(w, total, total)) return rc;
  uint8_t *h = w->h_stage, *d = w->d_stage;
  hipStream_t sc = L.st;
  memcpy(h, seeds, m * lam);
  HIP_TRY(hipMemcpyAsync(d, h, m * lam, hipMemcpyHostToDevice, sc));
  if (p->kind == 1 && lam > 16)
    hipLaunchKernelGGL(k_prg_mmo_wide, dim3((unsigned)grid_for(m * (lam / 16), p->cus)), dim3(kBlock), 0, sc,
                       p->d_tab, p->d_rk128, (const uint8_t*)d, (uint64_t)m, (uint32_t)lam, d + so);
  else if (p->kind == 1)
    hipLaunchKernelGGL(k_prg16_mmo, dim3((unsigned)grid_for(m, p->cus)), dim3(kBlock), 0, sc, p->d_tab, p->d_rk128,
                       (const uint4*)d, (uint64_t)m, d + so);
  else if (lam == 16)
    hipLaunchKernelGGL(k_prg16, dim3((unsigned)grid_for(m, p->cus)), dim3(kBlock), 0, sc, p->d_tab, p->rk[0],
                       (const uint4*)d, (uint64_t)m, d + so);
  else
    hipLaunchKernelGGL(k_prg_wide, dim3((unsigned)std::min<uint64_t>((m * (lam / 16) + 255) / 256, 65535)),
                       dim3(256), 0, sc, p->d_tab, p->d_rk2, (const uint8_t*)d, (uint64_t)m, (uint32_t)lam,
                       d + so);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(h + so, d + so, m * row, hipMemcpyDeviceToHost, sc));
  HIP_TRY(hipStreamSynchronize(sc));
  memcpy(out, h + so, m * row);
  return DCF_OK;
}

// ---- serde / bincode wire format of Share (lib.rs:217-340) ----
// bincode 1.x `serialize` (the crate's declared dep, Cargo.toml:44): little-endian,
// u64 length prefix per Vec, struct fields in declaration order, bool as one byte.

size_t dcf_share_bincode_bytes(size_t n_bytes, size_t lambda, size_t num_s0s) {
  const size_t n = 8 * n_bytes;
  return 8 + num_s0s * (8 + lambda) + 8 + n * (2 * (8 + lambda) + 2) + 8 + lambda;
}

static void put_u64(uint8_t*& o, uint64_t v) {
  for (int i = 0; i < 8; i++) *o++ = (uint8_t)(v >> (8 * i));
}

int dcf_share_to_bincode(size_t n_bytes, size_t lambda, const uint8_t* cwb, const uint8_t* s0s, size_t num_s0s,
                         uint8_t* out, size_t out_len) {
  if (!cwb || !out || (num_s0s && !s0s)) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (lambda == 0 || lambda % 16) return fail(DCF_ERR_LAMBDA, "lambda must be a positive multiple of 16");
  if (out_len != dcf_share_bincode_bytes(n_bytes, lambda, num_s0s)) return fail(DCF_ERR_LEN, "bad out_len");
  const size_t n = 8 * n_bytes;
  uint8_t* o = out;
  put_u64(o, num_s0s);  // s0s: Vec<Vec<u8>> (lib.rs:291-292)
  for (size_t i = 0; i < num_s0s; i++) {
    put_u64(o, lambda);
    memcpy(o, s0s + i * lambda, lambda);
    o += lambda;
  }
  put_u64(o, n);  // cws: Vec<Cw> (lib.rs:293), Cw = (s, v, tl, tr) (lib.rs:222-227)
  for (size_t i = 0; i < n; i++) {
    put_u64(o, lambda);
    memcpy(o, cwb + i * lambda, lambda);
    o += lambda;
    put_u64(o, lambda);
    memcpy(o, cwb + (n + i) * lambda, lambda);
    o += lambda;
    const uint8_t t = cwb[2 * n * lambda + i];
    *o++ = t & 1;
    *o++ = (t >> 1) & 1;
  }
  put_u64(o, lambda);  // cw_np1 (lib.rs:294)
  memcpy(o, cwb + dcf_cwb_np1_offset(n_bytes, lambda, 1), lambda);
  return DCF_OK;
}

int dcf_share_from_bincode(size_t n_bytes, size_t lambda, const uint8_t* in, size_t in_len, uint8_t* cwb_out,
                           uint8_t* s0s_out, size_t max_s0s, size_t* num_s0s) {
  if (!in || !cwb_out || !num_s0s) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (lambda == 0 || lambda % 16) return fail(DCF_ERR_LAMBDA, "lambda must be a positive multiple of 16");
  const size_t n = 8 * n_bytes;
  size_t pos = 0;
  auto u64 = [&](uint64_t* v) {
    if (in_len - pos < 8) return false;
    *v = 0;
    for (int i = 0; i < 8; i++) *v |= (uint64_t)in[pos + i] << (8 * i);
    pos += 8;
    return true;
  };
  auto arr = [&](uint8_t* dst) {  // Vec<u8> that must hold exactly lambda bytes (copy_from_slice, lib.rs:251)
    uint64_t len;
    if (!u64(&len) || len != lambda || in_len - pos < lambda) return false;
    if (dst) memcpy(dst, in + pos, lambda);
    pos += lambda;
    return true;
  };
  uint64_t ns;
  if (!u64(&ns)) return fail(DCF_ERR_KEY, "truncated Share (s0s length)");
  if (ns > max_s0s && s0s_out) return fail(DCF_ERR_LEN, "more seeds than s0s_out holds");
  for (uint64_t i = 0; i < ns; i++)
    if (!arr(s0s_out ? s0s_out + i * lambda : nullptr)) return fail(DCF_ERR_KEY, "bad seed in s0s");
  uint64_t ncw;
  if (!u64(&ncw)) return fail(DCF_ERR_KEY, "truncated Share (cws length)");
  if (ncw != n) return fail(DCF_ERR_KEY, "cws.len() != N * 8 (lib.rs:165)");
  memset(cwb_out, 0, dcf_cwb_bytes(n_bytes, lambda, 1));
  for (size_t i = 0; i < n; i++) {
    if (!arr(cwb_out + i * lambda) || !arr(cwb_out + (n + i) * lambda)) return fail(DCF_ERR_KEY, "bad Cw.s / Cw.v");
    if (in_len - pos < 2 || in[pos] > 1 || in[pos + 1] > 1) return fail(DCF_ERR_KEY, "bad Cw bool (bincode bool is 0/1)");
    cwb_out[2 * n * lambda + i] = (uint8_t)(in[pos] | (in[pos + 1] << 1));
    pos += 2;
  }
  if (!arr(cwb_out + dcf_cwb_np1_offset(n_bytes, lambda, 1))) return fail(DCF_ERR_KEY, "bad cw_np1");
  if (pos != in_len) return fail(DCF_ERR_KEY, "trailing bytes after Share");
  *num_s0s = (size_t)ns;
  return DCF_OK;
}

int dcf_eval_full_domain_device(dcf_prg* p, size_t n_bytes, int party, const uint8_t* cwb, const uint8_t* s0,
                                uint8_t* ys, void* stream) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (n_bytes > 4) return fail(DCF_ERR_UNSUPPORTED, "full-domain eval: N <= 4 (2^32 outputs)");
  if (party != 0 && party != 1) return fail(DCF_ERR_ARG, "party must be 0 or 1");
  if (!cwb || !s0 || !ys) return fail(DCF_ERR_ARG, "null buffer");
  DeviceGuard dg(p->device);
  Lease L(p);
  if (int rc = L.order((hipStream_t)stream)) return rc;
  hipStream_t st = L.st;
  const uint32_t nlev = (uint32_t)(8 * n_bytes);
  const uint64_t npts = 1ull << nlev;
  const size_t lam = p->lambda;
  if (lam != 16) {  // no tree sharing at LAMBDA >= 32: materialise the domain and run eval
    DevBuf xs;  // eval_wide owns the workspace, so the points get their own buffer
    HIP_TRY(xs.alloc(npts * n_bytes));
    hipLaunchKernelGGL(k_domain_points, dim3(1024), dim3(256), 0, st, (uint32_t)n_bytes, npts, (uint8_t*)xs.p);
    HIP_TRY(hipGetLastError());
    int rc = eval_launch(p, L, n_bytes, 1, npts, party, cwb, s0, (const uint8_t*)xs.p, ys);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(st));  // xs is freed on return
    return DCF_OK;
  }
  // Two ping-pong node buffers: s (16 B), v (16 B), t (1 B) per node.  With the
  // Hirose PRG the last kFdTail levels run in registers (k_fd_dfs16), so the widest
  // node level in HBM is 2^(n - kFdTail).
  const bool fused = p->kind == 0 && nlev > kFdTail;
  const size_t n = 8 * n_bytes;
  const uint4* cws = (const uint4*)cwb;
  const uint4* cwv = (const uint4*)(cwb + n * lam);
  const uint8_t* cwt = cwb + 2 * n * lam;
  const uint4* np1 = (const uint4*)(cwb + dcf_cwb_np1_offset(n_bytes, lam, 1));
  const uint32_t lev_end = fused ? nlev - kFdTail : nlev;
  // Hirose with the depth-first tail: levels 0 .. lev_end - 1 in ONE launch of the shared-prefix
  // table build (k_prefix_build16: workgroup subtrees, a depth-first register tail, 32-byte rows)
  // instead of one breadth-first level launch per level with 33-byte SoA nodes through HBM;
  // the tail then starts from the rows.  Falls back to the level kernels if the table and its
  // build buffers (~65 B per node of level lev_end) cannot be allocated.
  if (fused && lev_end >= 12) {
    PrefixTable pf{nullptr, 0u};
    const int brc = build_prefix(p, L.w, n_bytes, party, cws, cwv, cwt, np1, s0, lev_end, &pf, st);
    if (brc != DCF_OK && brc != kPrefixNoMem) return brc;
    if (brc == DCF_OK) {
      const uint64_t nodes = 1ull << lev_end;
      if (int rc2 = ensure_ctr(L.w)) return rc2;
      HIP_TRY(hipMemsetAsync(L.w->d_ctr, 0, kCtrBytes, st));
      hipLaunchKernelGGL((k_fd_dfs16<kFdTail, true>), dim3((unsigned)grid_for(nodes, p->cus)), dim3(kBlock), 0, st,
                         p->d_tab, p->rk[0], cws, cwv, cwt, np1, lev_end, nodes, pf.sv, (const uint4*)nullptr,
                         (const uint8_t*)nullptr, (uint4*)ys, L.w->d_ctr);
      HIP_TRY(hipGetLastError());
      return DCF_OK;
    }
  }
  const uint64_t maxnodes = fused ? (npts >> kFdTail) : npts / 2;
  const size_t nodeb = 33;
  // + one work counter per launch (64-node units, see next_wave_base) after the nodes
  const size_t ctr_off = (2 * maxnodes * nodeb + 64 + 255) & ~(size_t)255;
  int rc = ensure_ws(L.w, ctr_off + 64 * sizeof(uint32_t), st);
  if (rc) return rc;
  uint8_t* w = L.w->d_ws;
  uint32_t* ctrs = (uint32_t*)(w + ctr_off);
  HIP_TRY(hipMemsetAsync(ctrs, 0, 64 * sizeof(uint32_t), st));
  uint4* s_a = (uint4*)w;
  uint4* v_a = s_a + maxnodes;
  uint8_t* t_a = (uint8_t*)(v_a + maxnodes);
  uint4* s_b = (uint4*)(w + maxnodes * nodeb + 16 - (maxnodes * nodeb) % 16);
  uint4* v_b = s_b + maxnodes;
  uint8_t* t_b = (uint8_t*)(v_b + maxnodes);
  hipLaunchKernelGGL(k_fd_root16, dim3(1), dim3(64), 0, st, (const uint4*)s0, (uint32_t)party, s_a, v_a, t_a);
  HIP_TRY(hipGetLastError());
  for (uint32_t lev = 0; lev < lev_end; ++lev) {
    const uint64_t parents = 1ull << lev;
    if (p->kind == 1)
      hipLaunchKernelGGL(k_fd_level16_mmo, dim3((unsigned)grid_for(parents, p->cus)), dim3(kBlock), 0, st, p->d_tab,
                         p->d_rk128, cws, cwv, cwt, np1, lev, nlev, parents, s_a, v_a, t_a, s_b, v_b, t_b,
                         (uint4*)ys, ctrs + lev);
    else
      hipLaunchKernelGGL(k_fd_level16, dim3((unsigned)grid_for(parents, p->cus)), dim3(kBlock), 0, st, p->d_tab,
                         p->rk[0], cws, cwv, cwt, np1, lev, nlev, parents, s_a, v_a, t_a, s_b, v_b, t_b, (uint4*)ys,
                         ctrs + lev);
    HIP_TRY(hipGetLastError());
    std::swap(s_a, s_b);
    std::swap(v_a, v_b);
    std::swap(t_a, t_b);
  }
  if (fused) {
    const uint64_t nodes = 1ull << lev_end;
    hipLaunchKernelGGL(k_fd_dfs16<kFdTail>, dim3((unsigned)grid_for(nodes, p->cus)), dim3(kBlock), 0, st, p->d_tab,
                       p->rk[0], cws, cwv, cwt, np1, lev_end, nodes, s_a, v_a, t_a, (uint4*)ys, ctrs + 63);
    HIP_TRY(hipGetLastError());
  }
  return DCF_OK;
}

int dcf_gen(dcf_prg* p, size_t n_bytes, const uint8_t* alpha, const uint8_t* beta, const uint8_t* s0_0,
            const uint8_t* s0_1, int bound, uint8_t* cwb_out) {
  if (!p || !alpha || !beta || !s0_0 || !s0_1 || !cwb_out) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (bound != DCF_BOUND_LT_BETA && bound != DCF_BOUND_GT_BETA) return fail(DCF_ERR_ARG, "bad bound");
  DeviceGuard dg(p->device);
  if (!dg.ok) return fail(DCF_ERR_HIP, "hipSetDevice failed");
  Lease L(p);
  int rc = host_lease(L);
  if (rc == DCF_OK) rc = host_gen(p, L, n_bytes, alpha, beta, s0_0, s0_1, bound, cwb_out);
  return host_finish(L, rc);
}

int dcf_eval(dcf_prg* p, size_t n_bytes, int party, const uint8_t* cwb, size_t cwb_len, const uint8_t* s0,
             const uint8_t* xs, size_t m, uint8_t* ys, size_t ys_len) {
  if (!p || !cwb || !s0) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (party != 0 && party != 1) return fail(DCF_ERR_ARG, "party must be 0 or 1");
  const size_t lam = p->lambda;
  if (cwb_len != dcf_cwb_bytes(n_bytes, lam, 1))
    return fail(DCF_ERR_KEY, "key size does not match 8*N levels (lib.rs:165)");
  if (ys_len != m * lam) return fail(DCF_ERR_LEN, "ys length != m * lambda");
  if (m == 0) return DCF_OK;
  if (!xs || !ys) return fail(DCF_ERR_ARG, "null buffer");
  DeviceGuard dg(p->device);
  if (!dg.ok) return fail(DCF_ERR_HIP, "hipSetDevice failed");
  Lease L(p);
  int rc = host_lease(L);
  if (rc == DCF_OK) rc = host_eval(p, L, n_bytes, party, cwb, cwb_len, s0, xs, m, ys);
  return host_finish(L, rc);
}

int dcf_prg_gen(dcf_prg* p, const uint8_t* seeds, size_t m, uint8_t* out) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (m == 0) return DCF_OK;
  if (!seeds || !out) return fail(DCF_ERR_ARG, "null buffer");
  DeviceGuard dg(p->device);
  if (!dg.ok) return fail(DCF_ERR_HIP, "hipSetDevice failed");
  Lease L(p);
  int rc = host_lease(L);
  if (rc == DCF_OK) rc = host_prg_gen(p, L, seeds, m, out);
  return host_finish(L, rc);
}

// ---- multi-GPU (SURVEY §8(b) dcf_eval_multi_gpu; the reference spreads Dcf::eval over
// every host core inside one call, lib.rs:194-199) ----

static int check_group(dcf_prg* const* prgs, size_t G) {
  if (!prgs || G == 0) return fail(DCF_ERR_ARG, "prgs must hold at least one dcf_prg");
  for (size_t g = 0; g < G; ++g) {
    if (!prgs[g]) return fail(DCF_ERR_ARG, "null dcf_prg in prgs");
    for (size_t h = 0; h < g; ++h)
      if (prgs[h] == prgs[g]) return fail(DCF_ERR_ARG, "a dcf_prg appears twice in prgs (one thread per prg)");
    if (prgs[g]->kind != prgs[0]->kind || prgs[g]->lambda != prgs[0]->lambda ||
        prgs[g]->key_blob != prgs[0]->key_blob)
      return fail(DCF_ERR_ARG, "prgs disagree on the PRG (kind, lambda or keys)");
  }
  return DCF_OK;
}

int dcf_eval_multi_gpu(dcf_prg* const* prgs, size_t G, size_t n_bytes, int party, const uint8_t* cwb,
                       size_t cwb_len, const uint8_t* s0, const uint8_t* xs, size_t m, uint8_t* ys, size_t ys_len) {
  if (int rc = check_group(prgs, G)) return rc;
  if (!cwb || !s0) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (party != 0 && party != 1) return fail(DCF_ERR_ARG, "party must be 0 or 1");
  const size_t lam = prgs[0]->lambda;
  if (cwb_len != dcf_cwb_bytes(n_bytes, lam, 1))
    return fail(DCF_ERR_KEY, "key size does not match 8*N levels (lib.rs:165)");
  if (ys_len != m * lam) return fail(DCF_ERR_LEN, "ys length != m * lambda");
  if (m == 0) return DCF_OK;
  if (!xs || !ys) return fail(DCF_ERR_ARG, "null buffer");
  std::vector<int> rcs(G, DCF_OK);
  std::vector<std::string> errs(G);
  auto run = [&](size_t g) {
    size_t start, cnt;
    dcf_point_slice(m, G, g, &start, &cnt);
    if (cnt == 0) return;
    DeviceGuard dg(prgs[g]->device);
    if (!dg.ok) {
      rcs[g] = fail(DCF_ERR_HIP, "hipSetDevice failed");
    } else {
      Lease L(prgs[g]);
      int rc = host_lease(L);
      if (rc == DCF_OK)
        rc = host_eval(prgs[g], L, n_bytes, party, cwb, cwb_len, s0, xs + start * n_bytes, cnt, ys + start * lam);
      rcs[g] = host_finish(L, rc);
    }
    if (rcs[g]) errs[g] = t_err;
  };
  std::vector<std::thread> th;
  for (size_t g = 1; g < G; ++g) th.emplace_back(run, g);
  run(0);
  for (auto& t : th) t.join();
  for (size_t g = 0; g < G; ++g)
    if (rcs[g]) return fail(rcs[g], "device slice " + std::to_string(g) + ": " + errs[g]);
  return DCF_OK;
}

int dcf_eval_multi_gpu_device(dcf_prg* const* prgs, size_t G, size_t n_bytes, int party, const uint8_t* cwb,
                              size_t cwb_len, const uint8_t* s0, const uint8_t* const* xs, const size_t* ms,
                              uint8_t* const* ys, void* const* streams, uint8_t* gather_ys) {
  if (int rc = check_group(prgs, G)) return rc;
  if (!cwb || !s0 || !xs || !ms || !ys) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (party != 0 && party != 1) return fail(DCF_ERR_ARG, "party must be 0 or 1");
  const size_t lam = prgs[0]->lambda;
  if (cwb_len != dcf_cwb_bytes(n_bytes, lam, 1))
    return fail(DCF_ERR_KEY, "key size does not match 8*N levels (lib.rs:165)");
  const int dev0 = prgs[0]->device;
  size_t off = 0;
  for (size_t g = 0; g < G; ++g) {
    dcf_prg* p = prgs[g];
    DeviceGuard dg(p->device);
    if (!dg.ok) return fail(DCF_ERR_HIP, "hipSetDevice failed");
    Lease L(p);
    if (int rc = L.order(streams ? (hipStream_t)streams[g] : nullptr)) return rc;
    hipStream_t st = L.st;
    Workspace* w = L.w;
    // the key to this device, once per call (4.2 KB at N = LAMBDA = 16): the "broadcast"
    const size_t kb = align256(cwb_len) + align256(lam);
    if (int rc = grow(&w->d_mkey, &w->mkey_bytes, kb, st)) return rc;
    HIP_TRY(hipMemcpyAsync(w->d_mkey, cwb, cwb_len, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(w->d_mkey + align256(cwb_len), s0, lam, hipMemcpyHostToDevice, st));
    if (ms[g]) {
      if (!xs[g] || !ys[g]) return fail(DCF_ERR_ARG, "null slice buffer");
      int rc = eval_launch(p, L, n_bytes, 1, ms[g], party, w->d_mkey, w->d_mkey + align256(cwb_len), xs[g], ys[g]);
      if (rc) return rc;
      if (gather_ys) {  // slice g -> its rows of the gather buffer on prgs[0]'s device, over xGMI
        if (p->device != dev0) {
          // direct peer writes when the devices can map each other; hipMemcpyPeerAsync stages the
          // copy itself when they cannot, so a refused peer mapping is not an error
          const hipError_t e = hipDeviceEnablePeerAccess(dev0, 0);
          if (e != hipSuccess) (void)hipGetLastError();
          HIP_TRY(hipMemcpyPeerAsync(gather_ys + off * lam, dev0, ys[g], p->device, ms[g] * lam, st));
        } else {
          HIP_TRY(hipMemcpyAsync(gather_ys + off * lam, ys[g], ms[g] * lam, hipMemcpyDeviceToDevice, st));
        }
      }
    }
    off += ms[g];
  }
  return DCF_OK;
}

#ifdef DCF_CLOCK_STAMPS
// Diagnostic builds only (not in include/dcf_hip.h): the in-kernel clock stamps of slot `slot`
// (0 = k_eval_wide_tail2 main loop, 1 = k_eval_wide_head_stream walk, 2 = k_eval16_stream, 3 = k_eval16_oct,
// 4 = k_eval_wide_tail2 entry (phase 0 only), 5 = k_eval_wide_head_stream entry (phase 0 only)) of the last launch:
// per workgroup {memtime, realtime} at start and end, kClkGroups x 4 u64.
int dcf_debug_clock_stamps(int device, int slot, unsigned long long* out, size_t n) {
  if (!out || slot < 0 || slot >= (int)kClkSlots || n < (size_t)kClkGroups * 4) return fail(DCF_ERR_ARG, "bad argument");
  DeviceGuard dg(device);
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk_stamps), (size_t)kClkGroups * 4 * 8,
                              (size_t)slot * kClkGroups * 4 * 8, hipMemcpyDeviceToHost));
  return DCF_OK;
}
int dcf_debug_clock_reset(int device) {
  DeviceGuard dg(device);
  static std::vector<unsigned long long> z((size_t)kClkSlots * kClkGroups * 4, 0);
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_clk_stamps), z.data(), z.size() * 8, 0, hipMemcpyHostToDevice));
  return DCF_OK;
}
#endif

void dcf_point_slice(size_t total, size_t G, size_t g, size_t* start, size_t* count) {
  if (!start || !count) return;
  if (G == 0 || g >= G) {
    *start = total;
    *count = 0;
    return;
  }
  const size_t base = total / G, rem = total % G;
  *start = g * base + (g < rem ? g : rem);
  *count = base + (g < rem ? 1 : 0);
}

}  // extern "C"
