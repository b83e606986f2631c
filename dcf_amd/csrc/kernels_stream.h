// kernels_stream.h — LAMBDA = 16 eval with per-lane AES block scheduling.
// Included by dcf_hip.hip only.
//
// At LAMBDA = 16 one level of the GGM walk (lib.rs:174-189 over prg.rs:42-73)
// needs AES_K0(~s) = B on every step but AES_K0(s) = A only on a LEFT step:
//   right (x bit 1): s' = s&M ^ t*cw.s,  v ^= ~s&M ^ t*cw.v,  t' = lsb(B^~s) ^ t&tr
//   left  (x bit 0): s' = (A^s)&M ^ t*cw.s,  v ^= (B^~s)&M ^ t*cw.v,  t' = lsb(A^s) ^ t&tl
// A lockstep kernel computes A and B on every level (2 blocks); here each lane
// runs NS independent points ("streams") and every AES slot encrypts the NEXT
// block its stream needs — B, then A only if the step goes left — so every
// encrypted block is used: 1 + (zero bits of x)/8N blocks per level, 1.5 on
// average for uniform x instead of 2.  Outputs are bit-identical; the streams of
// one wave sit on different levels, so correction words are per-lane vector
// loads (L1/L2-resident: 4.2 KB per key) instead of scalar loads.
//
// Multi-key (MULTI): lanes on different levels of one key would each touch a
// different line of the level-major CWB (K * 16 B apart), so the host first
// builds a key-major digest — dig[key][level] = cw_s | cw_v (32 B), dig_t[key][level]
// — and the kernel reads a key's 4 KiB contiguously (k_cw_keymajor below).
//
// Work: each wave takes kStreamUnit consecutive points at a time from one
// global counter and hands them to its finished streams (wave-aggregated, in
// uniform control flow), so a wave's x reads and y writes stay within a few KiB;
// a stream with nothing left goes idle and the wave exits when all its streams
// are idle.  (A static strided assignment of points to streams measured 25 %
// slower: scattered 16-byte x reads and y writes.)  Multi-key (MULTI): point p
// belongs to key p / points_per_key; CW index = key * 8N + level into the digest.
#pragma once

#include "aes_lds.h"
#include "kernels16.h"

namespace {

// One work unit from a global counter (reset by the host before the launch), taken by lane 0
// of the wave and broadcast: the wave's streams (and the LAMBDA >= 32 head's) share it.
__device__ __forceinline__ uint32_t dequeue_unit(uint32_t* ctr) {
  uint32_t u = 0;
  if ((threadIdx.x & 63u) == 0) u = atomicAdd(ctr, 1u);
  return __builtin_amdgcn_readfirstlane(u);
}

constexpr uint32_t kStreamUnit = 256;  // points per refill of a wave
// Round keys: the single-key engine reads them per round from the device copy of the schedule
// (aes256_tt_gk, 3 rounds ahead: C3 +3.6 % over SGPR keys, r01o); the multi-key engine keeps
// them in SGPRs (global keys: C5 -14 %, their waits retire in order behind the CW digest loads;
// keys in LDS, by scalar loads or half in SGPRs measured slower too — profiles/AB_LOG.md).

// Lane's rank among the set bits of `mask` (bits below this lane).
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <int NS, bool XREG, bool MULTI>
struct StreamLane {
  uint32_t s[NS][4], v[NS][4], t[NS], ph[NS], lev[NS], cur[NS];
  uint32_t xw[NS][4];             // XREG: queue of the point's next x words, as loaded (byte-swapped on use)
  bool fresh[NS];                 // XREG: take cur from the queue head xw[0] before the next update
  const uint8_t* xp[NS];          // !XREG: the point's row in xs
  // MULTI: key-major digest row key * 8N + level (< 2^32: the host launches at most 2^24 keys
  // at a time); pt: the point's index in this launch (< 2^32: the host cuts larger batches).
  // The key itself is pt / points_per_key, needed once per point (its cw_np1), so it holds
  // no registers during the walk (r03: the C5 multi-key instance spilled at 128 VGPRs).
  uint32_t ci[NS], pt[NS];
  bool alive[NS];
};

// The point's x words into the stream's queue (as loaded; byte-swapped on use).
template <int NS, bool XREG, bool MULTI>
__device__ __forceinline__ void stream_load_x(StreamLane<NS, XREG, MULTI>& L, int i, const uint8_t* row,
                                              uint32_t nbytes) {
  if (nbytes == 16) {
    const uint4 x = *reinterpret_cast<const uint4*>(row);
    L.xw[i][0] = x.x; L.xw[i][1] = x.y; L.xw[i][2] = x.z; L.xw[i][3] = x.w;
  } else {
#pragma unroll
    for (int w = 0; w < 4; ++w) L.xw[i][w] = (4u * w < nbytes) ? reinterpret_cast<const uint32_t*>(row)[w] : 0u;
  }
}

// XLOADED: the caller has already loaded the point's x words into L.xw[i] (stream_load_x).
// PK2 (multi-key): points per key is a power of two (C5: 64), so point -> key is a shift.
template <int NS, bool XREG, bool MULTI, bool PFX = false, int NBC = 0, bool XLOADED = false, bool PK2 = false>
__device__ __forceinline__ void stream_start(StreamLane<NS, XREG, MULTI>& L, int i, uint64_t p,
                                             const uint4* __restrict__ s0s, const uint4 s0v, uint32_t party,
                                             const uint8_t* __restrict__ xs, uint32_t nbytes_rt, uint64_t ppk,
                                             const PrefixTable& pf) {
  const uint32_t nbytes = NBC ? (uint32_t)NBC : nbytes_rt;  // NBC: x width fixed at compile time
  const uint32_t k = !MULTI ? 0u : PK2 ? (uint32_t)p >> __builtin_ctz((uint32_t)ppk) : (uint32_t)p / (uint32_t)ppk;
  const uint8_t* row = xs + p * nbytes;
  uint32_t w0;  // first 32 x bits, Msb0 (lib.rs:181)
  if (XREG) {
    if (!XLOADED) stream_load_x(L, i, row, nbytes);
    w0 = bswap32(L.xw[i][0]);
  } else {
    L.xp[i] = row;
    w0 = load_bits32(row, 0, nbytes);
  }
  uint32_t lev0 = 0u;
  if (PFX || pf.levels) {  // start below the shared prefix: its row of the top-tree table
    lev0 = pf.levels;      // (MULTI: the key's own top tree, k_mk_prefix16, rows k * 2^levels + ...)
    uint4 sv, vv;
    const uint32_t top = w0 >> (32u - lev0);
    prefix_row(pf, MULTI ? (k << lev0) + top : top, sv, vv, L.t[i]);
    L.s[i][0] = sv.x; L.s[i][1] = sv.y; L.s[i][2] = sv.z; L.s[i][3] = sv.w;
    L.v[i][0] = vv.x; L.v[i][1] = vv.y; L.v[i][2] = vv.z; L.v[i][3] = vv.w;
  } else {
    const uint4 sv = MULTI ? s0s[k] : s0v;  // k.s0s[0] (lib.rs:168)
    L.s[i][0] = sv.x; L.s[i][1] = sv.y; L.s[i][2] = sv.z; L.s[i][3] = sv.w;
#pragma unroll
    for (int j = 0; j < 4; ++j) L.v[i][j] = 0u;
    L.t[i] = party;  // lib.rs:169
  }
  L.ph[i] = 0u;
  L.lev[i] = lev0;
  L.ci[i] = (uint32_t)k * (8u * nbytes) + lev0;  // key-major digest row (MULTI); the level of the single key otherwise
  L.pt[i] = (uint32_t)p;
  L.alive[i] = true;
  if (XREG) {
    if (PFX || lev0) {  // word 0 is consumed here, shifted past the prefix bits
      L.cur[i] = w0 << lev0;
      L.xw[i][0] = L.xw[i][1]; L.xw[i][1] = L.xw[i][2]; L.xw[i][2] = L.xw[i][3];
      L.fresh[i] = false;
    } else {
      L.fresh[i] = true;
    }
  } else {
    L.cur[i] = w0 << lev0;
  }
}

// Give every lane whose stream i is free (`mine`) a new point, or retire the
// stream when the counter is exhausted.  Called in wave-uniform control flow.
template <int NS, bool XREG, bool MULTI, uint32_t UNIT = kStreamUnit, bool PFX = false, int NBC = 0, bool PK2 = false>
__device__ __forceinline__ void stream_refill(StreamLane<NS, XREG, MULTI>& L, int i, bool mine, uint32_t& unext,
                                              uint32_t& uend, bool& exhausted, uint32_t* __restrict__ ctr,
                                              uint32_t nunits, uint32_t total, const uint4* __restrict__ s0s,
                                              const uint4 s0v, uint32_t party, const uint8_t* __restrict__ xs,
                                              uint32_t nbytes, uint64_t ppk, const PrefixTable& pf) {
  // Single key, x width fixed: the loop only hands out point indices and the stream state is
  // written once after it, so it is not a loop-carried value (no copies of it per pass; the
  // multi-key and runtime-width instances spill VGPRs that way and start streams in the loop).
  uint64_t need = __ballot(mine);
  constexpr bool ONCE = !MULTI && NBC != 0;
  if (ONCE) {
    uint32_t pnew = 0;
    bool got = false;
    while (need) {
      if (unext >= uend && !exhausted) {
        const uint32_t u = dequeue_unit(ctr);
        if (u >= nunits) {
          exhausted = true;
        } else {
          unext = u * UNIT;
          uend = min(unext + UNIT, total);
        }
      }
      if (exhausted && unext >= uend) break;
      const uint32_t rank = lane_rank(need);
      const bool take = mine && rank < uend - unext;
      pnew = take ? unext + rank : pnew;
      got = got || take;
      const uint64_t taken = __ballot(take);
      unext += (uint32_t)__popcll(taken);
      need &= ~taken;
      mine = mine && !take;
    }
    if (got) {
      stream_start<NS, XREG, MULTI, PFX, NBC, false, PK2>(L, i, pnew, s0s, s0v, party, xs, nbytes, ppk, pf);
    } else if (mine) {  // nothing left: the stream retires
      L.alive[i] = false;
      L.ci[i] = 0;  // keep the idle stream's CW loads in bounds
      L.lev[i] = 0;
    }
    return;
  }
  while (need) {
    if (unext >= uend && !exhausted) {
      const uint32_t u = dequeue_unit(ctr);
      if (u >= nunits) {
        exhausted = true;
      } else {
        unext = u * UNIT;
        uend = min(unext + UNIT, total);
      }
    }
    if (exhausted && unext >= uend) {
      if (mine) {
        L.alive[i] = false;
        L.ci[i] = 0;  // keep the idle stream's CW loads in bounds
        L.lev[i] = 0;
      }
      return;
    }
    const uint32_t rank = lane_rank(need);
    const bool take = mine && rank < uend - unext;
    if (take)
      stream_start<NS, XREG, MULTI, PFX, NBC, false, PK2>(L, i, unext + rank, s0s, s0v, party, xs, nbytes, ppk, pf);
    const uint64_t taken = __ballot(take);
    unext += (uint32_t)__popcll(taken);
    need &= ~taken;
    mine = mine && !take;
  }
}

// The stream's next 32 x bits at level nl (a multiple of 32): from the queue (XREG) or x.
template <int NS, bool XREG, bool MULTI>
__device__ __forceinline__ void stream_next_word(StreamLane<NS, XREG, MULTI>& L, int i, uint32_t nl, uint32_t nlev,
                                                 uint32_t nbytes) {
  if (XREG) {
    L.cur[i] = bswap32(L.xw[i][0]);
    L.xw[i][0] = L.xw[i][1];
    L.xw[i][1] = L.xw[i][2];
    L.xw[i][2] = L.xw[i][3];
  } else if (nl < nlev) {
    L.cur[i] = load_bits32(L.xp[i], nl >> 5, nbytes);
  }
}

// Key-major CW digest for the multi-key stream engine, tiled: a workgroup transposes KK keys x
// KL levels through LDS — per level KK x 16 B contiguous reads of cw_s and of cw_v, per key
// KL x 32 B contiguous writes of dig and KL bytes of dig_t.  Small enough to share a CU with a
// k_mk_prefix16 workgroup (128 KiB), which runs beside it on a second stream.  A key's LDS row is
// padded to 2 KL + 1 uint4 so the transposing writes spread over the banks.  Every thread's loads
// are issued before its first LDS store (compile-time trip counts, kKmThreads per workgroup).
// (C5 A/B r04y2: 2.55 vs 2.67 ms per launch for the previous runtime-strided loops; 64 x 8 and
// 128 x 4 tiles 0.5 % slower per C5 step.  The digest runs beside k_mk_prefix16, which is longer.)
constexpr uint32_t kKmKeys = 32, kKmLevs = 16, kKmThreads = 256;
__global__ __launch_bounds__(kKmThreads) void k_cw_keymajor(const uint4* __restrict__ cw_s,
                                                            const uint4* __restrict__ cw_v,
                                                            const uint8_t* __restrict__ cw_t, const uint32_t nlev,
                                                            const uint64_t num_keys, uint4* __restrict__ dig,
                                                            uint8_t* __restrict__ dig_t) {
  constexpr uint32_t RW = 2 * kKmLevs + 1;  // uint4 per key row
  constexpr uint32_t ITEMS = kKmKeys * kKmLevs, PER = (ITEMS + kKmThreads - 1) / kKmThreads;
  __shared__ uint4 sh[kKmKeys * RW];
  __shared__ uint8_t sht[kKmKeys * kKmLevs];
  const uint64_t k0 = (uint64_t)blockIdx.x * kKmKeys;
  const uint32_t l0 = blockIdx.y * kKmLevs;
  const uint32_t nk = (uint32_t)min<uint64_t>(kKmKeys, num_keys - k0), nl = min(kKmLevs, nlev - l0);
  uint4 vs[PER], vv[PER];
  uint32_t vt[PER];
#pragma unroll
  for (uint32_t j = 0; j < PER; ++j) {
    const uint32_t it = threadIdx.x + j * kKmThreads;
    const uint32_t l = it / kKmKeys, kk = it % kKmKeys;
    const bool ok = it < ITEMS && kk < nk && l < nl;
    const uint64_t src = ok ? (uint64_t)(l0 + l) * num_keys + k0 + kk : 0u;
    vs[j] = cw_s[src];
    vv[j] = cw_v[src];
    vt[j] = cw_t[src];
  }
#pragma unroll
  for (uint32_t j = 0; j < PER; ++j) {
    const uint32_t it = threadIdx.x + j * kKmThreads;
    if (it < ITEMS) {
      const uint32_t l = it / kKmKeys, kk = it % kKmKeys;
      sh[kk * RW + 2 * l] = vs[j];
      sh[kk * RW + 2 * l + 1] = vv[j];
      sht[kk * kKmLevs + l] = (uint8_t)vt[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < (2 * ITEMS + kKmThreads - 1) / kKmThreads; ++j) {
    const uint32_t it = threadIdx.x + j * kKmThreads;
    const uint32_t kk = it / (2 * kKmLevs), r = it % (2 * kKmLevs);
    if (it < 2 * ITEMS && kk < nk && r < 2 * nl) dig[(k0 + kk) * nlev * 2 + 2 * l0 + r] = sh[kk * RW + r];
  }
#pragma unroll
  for (uint32_t j = 0; j < PER; ++j) {
    const uint32_t it = threadIdx.x + j * kKmThreads;
    const uint32_t kk = it / kKmLevs, l = it % kKmLevs;
    if (it < ITEMS && kk < nk && l < nl) dig_t[(k0 + kk) * nlev + l0 + l] = sht[kk * kKmLevs + l];
  }
}

// B reuse over whole runs of right steps at t = 0 (A/B knob, see the reuse block in stream_run).
#ifndef DCF_REUSE_RUN
#define DCF_REUSE_RUN 0
#endif
// STG (staged rows; single key, prefix table, x in one word — C2): a wave claims its points in
// halves of kStgUnit (from its own 256-point counter claims: 32-point atomics on the one counter ran
// C2 2x slower) and stages each half ahead of use: the x words by an ordinary load (end of iteration
// k), the 32-B prefix rows by LDS DMA into the wave's 2 KiB area (k + 1, right after the CW wait:
// lanes 0-31 the s halves, 32-63 the v halves), read by the refills of k + 2 instead of a gather
// from HBM at every point start.  The DMA is inline asm, so hipcc adds no vmcnt(0) for it; the
// next iteration's CW wait retires it before any read of the staged rows, and the update and the
// refills lie between it and the next round-key wait (in-order VM counter).  C2 r05as (same box, 4
// alternating runs): 3.189-3.204 vs 3.237-3.258 ms with the DMA there and device-copy keys, 3.18-3.22
// with SGPR keys (SGPR keys alone: +3.9 %), 3.18-3.23 with the DMA at the iteration's end; the
// bound (rows from an L2-resident span, r05ar) is -6.8 %.
#ifndef DCF_STG_SLOTS
#define DCF_STG_SLOTS 2  // A/B: staging slots per wave (2 KiB of LDS split evenly)
#endif
constexpr int kStgH = DCF_STG_SLOTS;
// A slot's s halves are DMA'd by lanes [0, kStgUnit) and its v halves by [kStgUnit, 2 kStgUnit), so
// the wave covers both only if 2 kStgUnit <= 64 (kStgH >= 2); kStgUnit = 64 / kStgH must be exact
// and at least 2 (one slot silently staged the s halves only).
static_assert(kStgH >= 2 && kStgH <= 32 && 64 % kStgH == 0, "DCF_STG_SLOTS: 2, 4, 8, 16 or 32");
constexpr uint32_t kStgUnit = 64 / kStgH;          // points per slot
constexpr uint32_t kStgBytes = kStgUnit * 32u;     // LDS bytes per slot (s halves, then v halves)
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_dst)
               : "memory");
}

// s_waitcnt immediate (gfx9 encoding): vmcnt(0), expcnt and lgkmcnt at their maxima (no wait).
constexpr int kVmcnt0 = (0x7 << 4) | (0xF << 8);
#ifndef DCF_STG_PIN
#define DCF_STG_PIN 1  // A/B knob: the stream state pinned before the staging DMA (see stream_run)
#endif
#ifndef DCF_STG_EARLY
#define DCF_STG_EARLY 1  // the staging DMA right after the CW wait (state 4 until the next one; 0: at the end)
#endif
// Wave priority knob (see the AES call in stream_run).
#ifndef DCF_STREAM_PRIO
#define DCF_STREAM_PRIO 1
#endif
// The stream loop of one wave over the work counter's UNIT-point units (tables already in LDS).
// GK: round keys per round from the device copy rkg (aes256_tt_gk); otherwise from the kernel
// argument (SGPRs).  PFX: every stream starts below the per-key top trees (multi-key).
template <int NS, bool XREG, bool MULTI, uint32_t UNIT, bool GK, bool PFX = false, int NBC = 0, bool PK2 = false,
          bool STG = false>
__device__ __forceinline__ void stream_run(
    const uint32_t* lds, const uint4* rkl, const RoundKeys& rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes_rt,
    const uint64_t num_keys, const uint64_t ppk, const uint64_t total, uint32_t* __restrict__ ctr,
    uint4* __restrict__ ys, const PrefixTable& pf, const uint32_t stg_lds = 0u) {
  static_assert(!STG || (!MULTI && XREG && PFX && NBC > 0 && NBC <= 4),
                "staged rows: single key, prefix table, x in one word");
  const uint32_t nbytes = NBC ? (uint32_t)NBC : nbytes_rt;
  const uint32_t lc = lane_const();
  const uint32_t nlev = 8u * nbytes;
  // one launch covers < 2^32 points (the host cuts larger batches): 32-bit work distribution
  const uint32_t total32 = (uint32_t)total;
  const uint32_t nunits = (uint32_t)((total + UNIT - 1) / UNIT);
  uint32_t unext = 0, uend = 0;
  bool exhausted = false;
  const uint4 s0v = s0s[0];
  StreamLane<NS, XREG, MULTI> L;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    L.fresh[i] = false;
    L.alive[i] = false;
    L.ci[i] = 0;
    L.lev[i] = 0;
    L.ph[i] = 0u;
  }
  const uint4 np1v = cw_np1[0];  // single key: cw_np1 hoisted out of the loop
  // STG: per half h (wave-uniform) its first point, size, stage (0 free, 1 x loading, 2 rows
  // loading, 3 ready) and points handed out; xh[h]: lane r's raw x word of point base + (r & 31)
  uint32_t hb[kStgH], hn[kStgH], hs[kStgH], hu[kStgH], xh[kStgH], xr[kStgH];
#pragma unroll
  for (int h = 0; h < kStgH; ++h) hb[h] = hn[h] = hs[h] = hu[h] = xh[h] = xr[h] = 0u;
  auto staged = [&]() {  // a slot holds points not handed out yet
    bool any = false;
#pragma unroll
    for (int h = 0; h < kStgH; ++h) any = any || hs[h] != 0u;
    return any;
  };
  const uint32_t lane = threadIdx.x & 63u;
  auto claim = [&](int h) {  // the wave's next (up to) kStgUnit points into free half h, x loading
    if (unext >= uend && !exhausted) {  // the same UNIT-point claims as the direct path
      const uint32_t u = dequeue_unit(ctr);
      if (u >= nunits) {
        exhausted = true;
      } else {
        unext = u * UNIT;
        uend = min(unext + UNIT, total32);
      }
    }
    if (unext >= uend) return;
    hb[h] = unext;
    hn[h] = min(kStgUnit, uend - unext);
    unext += hn[h];
    hu[h] = 0u;
    const uint32_t pp = hb[h] + min(lane % kStgUnit, hn[h] - 1u);
    xh[h] = *reinterpret_cast<const uint32_t*>(xs + (size_t)pp * nbytes);
    hs[h] = 1u;
  };
  // At the end of an iteration (after its refills, so that no later wait in the iteration drains
  // the DMA): rows of the halves claimed an iteration ago (their x in by now) into LDS, ready for
  // the next iteration's refills; then new claims for free halves.  States: 0 free, 1 claimed now
  // (x loading), 2 x in (DMA due), 3 ready.
  auto stage = [&]() {
#pragma unroll
    for (int h = 0; h < kStgH; ++h)  // claims first: the counter atomic's wait would drain a DMA
      if (hs[h] == 0u) claim(h);
#pragma unroll
    for (int h = 0; h < kStgH; ++h) {
      if (!DCF_STG_EARLY && hs[h] == 2u) {  // xr[h]: copied by prep() this iteration
        const uint32_t top = bswap32(xr[h]) >> (32u - pf.levels);
        if (lane < 2u * kStgUnit) glds16(pf.sv + 2u * top + lane / kStgUnit, stg_lds + kStgBytes * h);
        hs[h] = 3u;
      }
    }
#pragma unroll
    for (int h = 0; h < kStgH; ++h)
      if (hs[h] == 1u) hs[h] = 2u;
  };
  // After the iteration's CW wait (which retired every load of the previous iteration): the x words
  // of halves due for their DMA, copied into registers no later load targets, so neither the DMA's
  // address nor the refills' ds_bpermute makes hipcc wait for the claims' fresh x loads.
  auto prep = [&]() {
    // Slots whose DMA (last iteration) is out: retired by now — every vmcnt wait since (this
    // iteration's round keys and CWs, issued after it) drained it, as vmcnt counts in order.  hipcc
    // does not see the asm DMA, so that is made explicit: one vmcnt(0) before the slots'
    // rows may be read, free here (the CW wait has retired every load in flight), and before this
    // call's own DMAs below, which it would otherwise drain.
    if (DCF_STG_EARLY) {
      bool out = false;
#pragma unroll
      for (int h = 0; h < kStgH; ++h) out = out || hs[h] == 4u;
      if (out) __builtin_amdgcn_s_waitcnt(kVmcnt0);
#pragma unroll
      for (int h = 0; h < kStgH; ++h)
        if (hs[h] == 4u) hs[h] = 3u;
    }
#pragma unroll
    for (int h = 0; h < kStgH; ++h) {
      if (hs[h] == 2u) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(xr[h]) : "v"(xh[h]));
        if (DCF_STG_EARLY) {  // the DMA here, an update and a refill ahead of the next key wait
          const uint32_t top = bswap32(xr[h]) >> (32u - pf.levels);
          if (lane < 2u * kStgUnit) glds16(pf.sv + 2u * top + lane / kStgUnit, stg_lds + kStgBytes * h);
          hs[h] = 4u;
        }
      }
    }
  };
  // Staged refill of the lanes whose stream i is free (`mine`) from the ready halves.
  auto refill_stg = [&](int i, bool mine) {
    uint64_t need = __ballot(mine);
    asm volatile("" ::: "memory");  // staged-row reads stay below the CW wait that retired their DMA
#pragma unroll
    for (int h = 0; h < kStgH; ++h) {
      if (need && hs[h] == 3u) {
        const uint32_t rank = lane_rank(need);
        const bool take = mine && rank < hn[h] - hu[h];
        const uint32_t r = min(hu[h] + rank, hn[h] - 1u);
        const uint32_t xw = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(r << 2), (int)xr[h]);
        const uint4 sv = lds_load16(stg_lds + kStgBytes * h + 16u * r);
        const uint4 vv = lds_load16(stg_lds + kStgBytes * h + 16u * (kStgUnit + r));
        if (take) {  // stream_start below the shared prefix, with the row and x in hand (prefix_row)
          const uint32_t lev0 = pf.levels;
          L.s[i][0] = sv.x; L.s[i][1] = sv.y; L.s[i][2] = sv.z; L.s[i][3] = sv.w & kMaskLast;
          L.v[i][0] = vv.x; L.v[i][1] = vv.y; L.v[i][2] = vv.z; L.v[i][3] = vv.w;
          L.t[i] = (sv.w >> 24) & 1u;
          L.ph[i] = 0u;
          L.lev[i] = lev0;
          L.ci[i] = lev0;
          L.pt[i] = hb[h] + r;
          L.alive[i] = true;
          L.cur[i] = bswap32(xw) << lev0;
          L.xw[i][0] = 0u; L.xw[i][1] = 0u; L.xw[i][2] = 0u;
          L.fresh[i] = false;
        }
        const uint64_t taken = __ballot(take);
        hu[h] += (uint32_t)__popcll(taken);
        need &= ~taken;
        mine = mine && !take;
        if (hu[h] == hn[h]) {  // used up: refill the half at once
          hs[h] = 0u;
          claim(h);
        }
      }
    }
    // the rest gathers directly (the direct path's claimed unit first); with the counter spent
    // it parks the stream, which retries while staged points remain (`want` below)
    if (need)
      stream_refill<NS, XREG, MULTI, UNIT, PFX, NBC, PK2>(L, i, mine, unext, uend, exhausted, ctr, nunits, total32,
                                                         s0s, s0v, party, xs, nbytes, ppk, pf);
  };
  if (STG) stage();
#pragma unroll
  for (int i = 0; i < NS; ++i)
    stream_refill<NS, XREG, MULTI, UNIT, PFX, NBC, PK2>(L, i, true, unext, uend, exhausted, ctr, nunits, total32,
                                                       s0s, s0v, party, xs, nbytes, ppk, pf);

  uint64_t nblk = 0;  // AES blocks this wave encrypts for live streams (wave-uniform)
  for (;;) {
    bool any = false;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      any = any || L.alive[i];
      nblk += (uint64_t)__popcll(__ballot(L.alive[i]));
    }
    const bool pend = STG && staged();  // staged points not handed out yet
    if (!__ballot(any) && !pend) break;
    // Correction words of each stream's current level (vector loads, issued before the AES),
    // and of the next level for a stream whose step may end with B still valid (a right
    // step at t = 0 keeps s: see "B reuse" below).
    uint4 cs[NS], cv[NS], cs2[NS], cv2[NS];
    uint32_t ct[NS], ct2[NS];
    bool maybe[NS];  // the next level's CWs were loaded
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      // CW row: the key-major digest row (MULTI: cw_s = digest, 2 uint4 per level, cw_t = its t
      // bytes); for one key the row is the level itself (a 32-bit index: ci only mirrors lev
      // there, and a retired stream's lev is reset to 0)
      const uint32_t cwi = MULTI ? L.ci[i] : L.lev[i];
      if (MULTI) {
        cs[i] = cw_s[2 * cwi];
        cv[i] = cw_s[2 * cwi + 1];
      } else {
        cs[i] = cw_s[cwi];
        cv[i] = cw_v[cwi];
      }
      ct[i] = cw_t[cwi];
      // XREG: a fresh stream's x word is still in the queue; its first step is a B step
      // at the root, whose seed may be unmasked, so no reuse follows it anyway.
      maybe[i] = L.alive[i] && L.ph[i] == 0u && L.t[i] == 0u && (!XREG || PFX || !L.fresh[i]) &&
                 (L.cur[i] >> 31) != 0u && L.lev[i] + 1u < nlev;
      // Loaded unconditionally (L1-resident): loads under a divergent branch made the
      // compiler wait for them before the AES.
      const uint32_t c2 = cwi + (L.lev[i] + 1u < nlev ? 1u : 0u);
      if (MULTI) {
        cs2[i] = cw_s[2 * c2];
        cv2[i] = cw_s[2 * c2 + 1];
      } else {
        cs2[i] = cw_s[c2];
        cv2[i] = cw_v[c2];
      }
      ct2[i] = cw_t[c2];
    }
    // Slot i encrypts ~s (B) in phase 0 and s (A) in phase 1.
    uint32_t st[NS][4];
    // GK: round key 0 is folded into the input XOR (one 3-input XOR per word)
    uint4 k0 = make_uint4(0u, 0u, 0u, 0u);
    if (GK) k0 = rkl[0];
    const uint32_t k0w[4] = {k0.x, k0.y, k0.z, k0.w};
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint32_t inv = L.ph[i] - 1u;
#pragma unroll
      for (int j = 0; j < 4; ++j) st[i][j] = GK ? xor3(L.s[i][j], inv, k0w[j]) : (L.s[i][j] ^ inv);
    }
    // Wave priority: the AES rounds run at s_setprio 1, the level update / refill at 0, so the
    // arbiter issues the LDS lookups of waves in their rounds ahead of other waves' update VALU
    // and the LDS stays fed.  r05ae (same box, 3 alternating runs): C3 479.1-480.4 vs 497.9-499.8
    // ms (-3.9 %), C2 3.325-3.391 vs 3.401-3.416, C5 319.2-319.8 vs 322.1-323.4; the update at
    // priority 1 instead (knob 2) lost 2-5 %; widening the priority-1 span to the CW loads (noise)
    // or to the stores and refill as well (C3 +2 %) did not help (r05aj).
    if (DCF_STREAM_PRIO == 1) __builtin_amdgcn_s_setprio(1);
    if (DCF_STREAM_PRIO == 2) __builtin_amdgcn_s_setprio(0);
    if (GK)
      aes256_tt_gk<NS, true>(st, rkl, lds, lc);
    else
      aes256_tt<NS>(st, rk, lds, lc);
    if (DCF_STREAM_PRIO == 1) __builtin_amdgcn_s_setprio(0);
    if (DCF_STREAM_PRIO == 2) __builtin_amdgcn_s_setprio(1);
    // Pin the CW loads above the update: without this the compiler sinks the
    // cw_t load into the (divergent) level-done path and waits on it there.
#pragma unroll
    for (int i = 0; i < NS; ++i)
      asm volatile("" : "+v"(cs[i].x), "+v"(cs[i].y), "+v"(cs[i].z), "+v"(cs[i].w), "+v"(cv[i].x), "+v"(cv[i].y),
                   "+v"(cv[i].z), "+v"(cv[i].w), "+v"(ct[i]));
#pragma unroll
    for (int i = 0; i < NS; ++i)
      asm volatile("" : "+v"(cs2[i].x), "+v"(cs2[i].y), "+v"(cs2[i].z), "+v"(cs2[i].w), "+v"(cv2[i].x),
                   "+v"(cv2[i].y), "+v"(cv2[i].z), "+v"(cv2[i].w), "+v"(ct2[i]));
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      if (XREG && !PFX) {  // next 32 x bits from the word queue (raw loads, byte-swapped here)
        const bool nw = L.fresh[i];
        L.cur[i] = nw ? bswap32(L.xw[i][0]) : L.cur[i];
        L.xw[i][0] = nw ? L.xw[i][1] : L.xw[i][0];
        L.xw[i][1] = nw ? L.xw[i][2] : L.xw[i][1];
        L.xw[i][2] = nw ? L.xw[i][3] : L.xw[i][2];
        L.fresh[i] = false;
      }
      const uint32_t p = L.ph[i], xb = L.cur[i] >> 31;  // Msb0 bit of x (lib.rs:181)
      const uint32_t adv = L.alive[i] ? (p | xb) : 0u;   // this step finishes the level
      const uint32_t inv = p - 1u;                        // all ones on a B step
      const uint32_t keepB = xb - 1u;                     // all ones when going left
      const uint32_t tm = 0u - L.t[i], am = 0u - adv, pm = 0u - p;
      const uint32_t csw[4] = {cs[i].x, cs[i].y, cs[i].z, cs[i].w};
      const uint32_t cvw[4] = {cv[i].x, cv[i].y, cv[i].z, cv[i].w};
      uint32_t d[4];  // (A^s) or (B^~s)
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = st[i][j] ^ L.s[i][j] ^ inv;
      const uint32_t d0 = d[0];
      // B reuse: a right step at t = 0 leaves s = s & M, which is s itself when s is
      // already masked (every seed below the root: side & M ^ t*cw.s, cw.s masked), so
      // the next level's PRG(s) is this one's and its B is d ^ ~s, already in hand.
      const bool reuse = maybe[i] && (L.s[i][3] & ~kMaskLast) == 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
        const uint32_t in = L.s[i][j] ^ inv;
        // B step: v ^= v_hat(side) ^ t*cw.v, v_hat = (~s ^ [left] B) & M   (lib.rs:182/186)
        const uint32_t vhat = (in ^ (st[i][j] & keepB)) & msk;
        L.v[i][j] ^= inv & (vhat ^ (tm & cvw[j]));
        // level done: s' = s(side) ^ t*cw.s, s(side) = (A^s)&M (left) or s&M (right)  (lib.rs:177-178)
        const uint32_t sx = L.s[i][j] ^ (st[i][j] & pm);  // p: A ^ s
        const uint32_t sn = (sx & msk) ^ (tm & csw[j]);
        L.s[i][j] = (am & sn) | (~am & L.s[i][j]);
      }
      // t' = lsb(side) ^ t & cw.t(side)   (lib.rs:179-180, 183/187)
      const uint32_t tb = (d0 ^ (L.t[i] & (ct[i] >> xb))) & 1u;
      L.t[i] = (am & tb) | (~am & L.t[i]);
      L.ph[i] = adv ^ 1u;
      uint32_t nl = L.lev[i] + adv;
      L.cur[i] <<= adv;
      // (x in one word, NBC <= 4: the only crossing ends the point, so no next word is taken)
      if (!(NBC && NBC <= 4) && adv && (nl & 31u) == 0u) stream_next_word<NS, XREG, MULTI>(L, i, nl, nlev, nbytes);
      L.ci[i] += adv;
      {  // reuse: level nl with B known: its B half now, without an AES slot (branch-free)
        const uint32_t xb2 = L.cur[i] >> 31, t1 = L.t[i], tm1 = 0u - t1;
        const uint32_t rm = 0u - (uint32_t)reuse, rr = rm & (0u - xb2);  // reuse / reuse and right
        const uint32_t cs2w[4] = {cs2[i].x, cs2[i].y, cs2[i].z, cs2[i].w};
        const uint32_t cv2w[4] = {cv2[i].x, cv2[i].y, cv2[i].z, cv2[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
          // v ^= v_hat(side) ^ t*cw.v: right ~s & M, left (B^~s) & M   (lib.rs:182/186)
          L.v[i][j] ^= rm & ((((xb2 ? ~L.s[i][j] : d[j]) & msk) ^ (tm1 & cv2w[j])));
          L.s[i][j] ^= rr & tm1 & cs2w[j];  // right: s' = s & M ^ t*cw.s   (lib.rs:178)
        }
        // right: the level ends, t' = lsb(B^~s) ^ t & cw.tr (lib.rs:180); left: A next
        L.t[i] = rr ? ((d0 ^ (t1 & (ct2[i] >> 1))) & 1u) : L.t[i];
        L.ph[i] = (reuse && !xb2) ? 1u : L.ph[i];
        nl += rr & 1u;
        L.cur[i] <<= (rr & 1u);
        L.ci[i] += rr & 1u;
        if (!(NBC && NBC <= 4) && rr && (nl & 31u) == 0u) stream_next_word<NS, XREG, MULTI>(L, i, nl, nlev, nbytes);
        if (DCF_REUSE_RUN) {
          // A reused right step that left t = 0 (t1 = 0) kept s, so the next level has the same
          // B again: a run of k further right steps keeps s and t = 0 and XORs ~s & M into v k
          // times (lib.rs:178-186 with t = 0: no CW enters); the left step that ends the run has
          // its B half too (v ^= (B ^ ~s) & M), leaving A for the next slot.  The run stops at the
          // x word's end (the next word's first step recomputes B).
          const bool go = rr && t1 == 0u && (nl & 31u) != 0u && nl < nlev;
          const uint32_t k = go ? min((uint32_t)__clz(~L.cur[i]), nlev - nl) : 0u;
          const uint32_t ko = 0u - (k & 1u);
          nl += k;
          L.cur[i] <<= k;
          L.ci[i] += k;
          const uint32_t lm = 0u - (uint32_t)(go && nl < nlev && (nl & 31u) != 0u);  // the left step after the run
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
            L.v[i][j] ^= ((ko & ~L.s[i][j]) ^ (lm & d[j])) & msk;
          }
          L.ph[i] = lm ? 1u : L.ph[i];
          if (!(NBC && NBC <= 4) && go && k && (nl & 31u) == 0u && nl < nlev)
            stream_next_word<NS, XREG, MULTI>(L, i, nl, nlev, nbytes);
        }
      }
      L.lev[i] = nl;
    }
    // Finished points: y = v ^ s_n ^ t_n*cw_np1 (lib.rs:192), then refill.  (vmcnt counts
    // stores too, so the refill's wait for its x word also waits for this store; issuing the
    // store after the refill's loads measured slower, AB_LOG r02.)
    if (STG) {
      // The level update (and so the AES's last round-key wait) before the staging DMA: else hipcc
      // sinks the last round's key XOR below the DMA and its vmcnt(0) drains the DMA at once.
      if (DCF_STG_PIN)
#pragma unroll
        for (int i = 0; i < NS; ++i)
          asm volatile("" : "+v"(L.s[i][0]), "+v"(L.s[i][1]), "+v"(L.s[i][2]), "+v"(L.s[i][3]), "+v"(L.v[i][0]),
                       "+v"(L.v[i][1]), "+v"(L.v[i][2]), "+v"(L.v[i][3]), "+v"(L.t[i]));
      prep();
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const bool done = L.alive[i] && L.lev[i] == nlev;
      if (done) {
        const uint32_t key = PK2 ? L.pt[i] >> __builtin_ctz((uint32_t)ppk) : L.pt[i] / (uint32_t)ppk;
        // (MULTI: cw_np1 loaded here; with the CWs before the AES instead it ran 0.5 % slower, r06f)
        const uint4 np = MULTI ? cw_np1[key] : np1v;
        const uint32_t tm = 0u - L.t[i];
        ys[L.pt[i]] = make_uint4(L.v[i][0] ^ L.s[i][0] ^ (tm & np.x), L.v[i][1] ^ L.s[i][1] ^ (tm & np.y),
                                 L.v[i][2] ^ L.s[i][2] ^ (tm & np.z), L.v[i][3] ^ L.s[i][3] ^ (tm & np.w));
      }
      if (STG) {
        const bool want = done || (!L.alive[i] && staged());
        if (__ballot(want)) refill_stg(i, want);
      } else if (__ballot(done)) {
        stream_refill<NS, XREG, MULTI, UNIT, PFX, NBC, PK2>(L, i, done, unext, uend, exhausted, ctr, nunits, total32,
                                                           s0s, s0v, party, xs, nbytes, ppk, pf);
      }
    }
    if (STG) stage();
  }
  // ctr[2..3]: the launch's AES block count (dcf_prg_last_eval_blocks)
  if ((threadIdx.x & 63u) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(ctr) + 1, (unsigned long long)nblk);
}

// One 1024-thread workgroup per CU (the replicated T-tables take 128 KiB of LDS).
template <int NS, bool XREG, bool MULTI, bool PFX = false, int NBC = 0, bool PK2 = false, bool STG = false>
__global__ __launch_bounds__(kBlock, 1) void k_eval16_stream(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t num_keys, const uint64_t ppk, const uint64_t total, uint32_t* __restrict__ ctr,
    uint4* __restrict__ ys, const PrefixTable pf, const uint4* __restrict__ rkg) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  DCF_CLK(2, 0);
  // Round keys: per round from the device copy (GK), except in the multi-key instances with per-key
  // top trees (C5), which keep them in SGPRs (device-copy keys cost C5 14 %, AB_LOG).  The multi-key
  // instance without top trees (fewer than 32 points per key, or prefix levels forced off) has the
  // root-seed start path as well and spilled 45 SGPRs with SGPR keys (r04 resource usage): with x in
  // registers it takes the device-copy keys (0 spills); with x loaded per word the key look-ahead
  // registers would spill 2 VGPRs to scratch instead, so it keeps SGPR keys (40 SGPR spills, to VGPR lanes).
#ifndef DCF_STG_GK
#define DCF_STG_GK 1  // the staged instance with device-copy round keys (0: SGPR keys, r05as)
#endif
  constexpr bool GK = (!STG || DCF_STG_GK) && (!MULTI || (!PFX && XREG));
  if constexpr (STG) {  // 2 KiB of staged rows per wave beside the 128 KiB of tables (160 KiB in all)
    __shared__ uint4 stg[kBlock / 64 * 128];
    const uint32_t stg_lds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)stg + (threadIdx.x >> 6) * 2048u);
    stream_run<NS, XREG, MULTI, kStreamUnit, GK, PFX, NBC, PK2, STG>(
        lds, rkg, rk, cw_s, cw_v, cw_t, cw_np1, s0s, party, xs, nbytes, num_keys, ppk, total, ctr, ys, pf, stg_lds);
  } else {
    stream_run<NS, XREG, MULTI, kStreamUnit, GK, PFX, NBC, PK2>(lds, rkg, rk, cw_s, cw_v, cw_t, cw_np1, s0s, party,
                                                               xs, nbytes, num_keys, ppk, total, ctr, ys, pf);
  }
  DCF_CLK(2, 1);
}

}  // namespace
