// kernels_wide_stream.h — LAMBDA >= 32 eval head with per-lane AES block
// scheduling.  Included by dcf_hip.hip only (after kernels_stream.h).
//
// The head walks bytes [0,32) of the state (kernels_wide.h).  Per level the PRG
// (prg.rs:42-73 at LAMBDA >= 32) encrypts four blocks, but a step needs only
//   left  (x bit 0): B = E0(~s[0:16]) (v_L) and A = E0(s[0:16]) (s_L, t_L)
//   right (x bit 1): B (t_R = lsb(B ^ ~s)[0]), D = E17(~s[16:32]) (v_R), C = E17(s[16:32]) (s_R)
// i.e. 2.5 blocks per level on average instead of 4.  As in kernels_stream.h
// each lane runs two points and each AES slot encrypts the next block its point
// needs, in the order B, A (left) or B, D, C (right).  A slot's cipher is chosen
// per lane: the schedules of ciphers 0 and 17 sit in LDS beside the T-tables and
// each round reads the lane's key with one ds_read_b128 (as kernels_mmo.h does;
// key words in SGPRs would need a v_mov per use for the per-lane select).
// Outputs: y[0:32) and the t-vector for the tail (kernels_wide.h).
#pragma once

#include "aes_lds.h"
#include "kernels_lat.h"     // dpp<>
#include "kernels_stream.h"  // dequeue_unit

// Wave priority for the head's AES rounds (r05af: C4 -2.0 % with DCF_TAIL_PRIO).
#ifndef DCF_HEAD_PRIO
#define DCF_HEAD_PRIO 1
#endif

namespace {

__device__ __forceinline__ uint32_t xand(uint32_t a, uint32_t m, uint32_t c) {  // a ^ (m & c)
  return __builtin_amdgcn_bitop3_b32(a, m, c, 0x78);
}
__device__ __forceinline__ uint32_t xandn(uint32_t a, uint32_t m, uint32_t c) {  // a ^ (m & ~c)
  return __builtin_amdgcn_bitop3_b32(a, m, c, 0xB4);
}
__device__ __forceinline__ uint32_t pick(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b, m = 0 or ~0
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}

// Shared prefix for the stream head (as kernels16.h PrefixTable at LAMBDA = 16): the
// key's top `levels` tree levels expanded once, one 80-byte node per prefix:
// rows[5 i .. 5 i + 5) = s[0:32) | v[0:32) | {t, t-vector word 0, partial t-vector word, 0}.
struct WidePrefix {
  const uint4* rows;
  uint32_t levels;  // < 31 and < 8N; 0 = none
};

template <int NS>
struct WideLane {
  uint32_t s[NS][8], v[NS][8];           // bytes [0,32) of the seed and of the v accumulator
  uint32_t dB[NS][4];                    // this level's B ^ ~s[0:16) (B reuse)
  uint32_t t[NS], ph[NS], lev[NS], cur[NS], tR[NS], tacc[NS];
  uint32_t xq[NS][3];                    // XREG: the point's next raw x words (byte-swapped on use)
  uint32_t pt[NS];                       // point index within this launch (<= 2^22); x row = xs + pt * N
  uint32_t kk[NS];                       // MK: the point's key within this launch (pt / points per key)
  bool alive[NS];
};

template <int NS, bool XREG, bool MK>
__device__ __forceinline__ void wide_start(WideLane<NS>& L, int i, uint32_t p, const uint8_t* __restrict__ s0p,
                                           uint32_t party, const uint8_t* __restrict__ xs, uint32_t nbytes,
                                           const WidePrefix& pf, uint32_t* __restrict__ tvec, uint32_t tw,
                                           uint32_t ppk, uint32_t lam) {
  const uint32_t kk = MK ? p / ppk : 0u;
  L.kk[i] = kk;
  // k.s0s[0] (lib.rs:168) of the point's key, L2-resident
  const uint4* s4 = reinterpret_cast<const uint4*>(s0p + (uint64_t)kk * lam);
  const uint4 a = s4[0], b = s4[1];
  L.s[i][0] = a.x; L.s[i][1] = a.y; L.s[i][2] = a.z; L.s[i][3] = a.w;
  L.s[i][4] = b.x; L.s[i][5] = b.y; L.s[i][6] = b.z; L.s[i][7] = b.w;
#pragma unroll
  for (int j = 0; j < 8; ++j) L.v[i][j] = 0u;
  L.t[i] = party;
  L.tacc[i] = party;  // row 0 of the t-vector is t_0 = party
  L.tR[i] = 0u;
  L.ph[i] = 0u;
  L.lev[i] = 0u;
  L.pt[i] = p;
  L.alive[i] = true;
  // x bits are needed before the next AES (they pick its block): one 32-bit word
  // per 32 levels.  XREG (N % 4 == 0, N <= 16): all of x now, queued, so a level
  // crossing 32 bits never waits on a load.
  const uint8_t* row = xs + (uint64_t)p * nbytes;
  if (XREG) {
    uint32_t w[4];
    if (nbytes == 16) {
      const uint4 x = *reinterpret_cast<const uint4*>(row);
      w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = (4u * k < nbytes) ? reinterpret_cast<const uint32_t*>(row)[k] : 0u;
    }
    L.cur[i] = bswap32(w[0]);
    L.xq[i][0] = w[1]; L.xq[i][1] = w[2]; L.xq[i][2] = w[3];
  } else {
    L.cur[i] = load_bits32(row, 0, nbytes);
  }
  if (pf.levels) {  // start at level D from the node named by x's first D bits (Msb0)
    const uint32_t D = pf.levels;
    const uint4* nd = pf.rows + 5u * (L.cur[i] >> (32u - D));
    const uint4 a0 = nd[0], a1 = nd[1], b0 = nd[2], b1 = nd[3], e = nd[4];
    L.s[i][0] = a0.x; L.s[i][1] = a0.y; L.s[i][2] = a0.z; L.s[i][3] = a0.w;
    L.s[i][4] = a1.x; L.s[i][5] = a1.y; L.s[i][6] = a1.z; L.s[i][7] = a1.w;
    L.v[i][0] = b0.x; L.v[i][1] = b0.y; L.v[i][2] = b0.z; L.v[i][3] = b0.w;
    L.v[i][4] = b1.x; L.v[i][5] = b1.y; L.v[i][6] = b1.z; L.v[i][7] = b1.w;
    L.t[i] = e.x;
    L.tacc[i] = e.z;  // rows 16 (D >> 4) .. D of the t-vector
    if (D >= 15u) tvec[(uint64_t)p * tw] = e.y;  // rows 0..15, complete (row 15 = t_15 of depth 15)
    L.lev[i] = D;
    L.cur[i] <<= D;
  }
}

// Points per refill of a wave.  A lane of C4 runs only ~16 points per launch (2^22 over 2^18
// lanes), so the last units decide when the grid drains: 256-point units (4 per lane) left
// ~11 % of the head's LDS instructions to lanes idling at the end (PMC: 265 per block vs 239).
constexpr uint32_t kWideUnit = 64;

template <int NS, bool XREG, bool MK>
__device__ __forceinline__ void wide_refill(WideLane<NS>& L, int i, bool mine, uint64_t& unext, uint64_t& uend,
                                            bool& exhausted, uint32_t* __restrict__ ctr, uint64_t nunits,
                                            uint64_t count, const uint8_t* __restrict__ s0p, uint32_t party,
                                            const uint8_t* __restrict__ xs, uint32_t nbytes, const WidePrefix& pf,
                                            uint32_t* __restrict__ tvec, uint32_t tw, uint32_t ppk, uint32_t lam) {
  uint64_t need = __ballot(mine);
  while (need) {
    if (unext >= uend && !exhausted) {
      const uint32_t u = dequeue_unit(ctr);
      if (u >= nunits) {
        exhausted = true;
      } else {
        unext = (uint64_t)u * kWideUnit;
        uend = min(unext + kWideUnit, count);
      }
    }
    if (exhausted && unext >= uend) {
      if (mine) {
        L.alive[i] = false;
        L.lev[i] = 0u;  // keep the idle stream's CW loads in bounds
      }
      return;
    }
    const uint32_t rank = lane_rank(need);
    const bool take = mine && (uint64_t)rank < uend - unext;
    if (take) wide_start<NS, XREG, MK>(L, i, (uint32_t)(unext + rank), s0p, party, xs, nbytes, pf, tvec, tw, ppk, lam);
    const uint64_t taken = __ballot(take);
    unext += (uint64_t)__popcll(taken);
    need &= ~taken;
    mine = mine && !take;
  }
}

// Compact CW digest of keys key0 .. key0 + nk - 1 for the stream head, key-major: for key kk of
// the range, dig[4 (kk nlev + l) .. + 4) = cw_s[l][0:32) | cw_v[l][0:32), dig_t[kk nlev + l] = cw_t[l].
__global__ void k_cw_digest(const uint8_t* __restrict__ cw_s, const uint8_t* __restrict__ cw_v,
                            const uint8_t* __restrict__ cw_t, const uint32_t nlev, const uint32_t lam,
                            const uint64_t num_keys, const uint64_t key0, const uint32_t nk, uint4* __restrict__ dig,
                            uint8_t* __restrict__ dig_t) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4ull * nlev * nk) return;
  const uint32_t kk = (uint32_t)(i / (4u * nlev)), r = (uint32_t)(i % (4u * nlev));
  const uint32_t l = r >> 2, q = r & 3u;
  const uint64_t ci = (uint64_t)l * num_keys + key0 + kk;
  const uint8_t* src = (q < 2 ? cw_s : cw_v) + ci * lam + 16u * (q & 1u);
  dig[i] = *reinterpret_cast<const uint4*>(src);
  if (q == 0) dig_t[(uint64_t)kk * nlev + l] = cw_t[ci];
}

// Round keys: the lane's schedule (cipher 0 or 17) from the LDS copy, one ds_read_b128 per round
// and block.  Through the vector L1 instead (per-lane buffer loads, or both schedules by uniform
// loads and a per-word pick) it measured 4-6 % slower on C4: the key waits retire in order behind
// the CW loads (AB_LOG r02z / r03f).  B reuse: the B block after a right step at t = 0 is skipped.
// Key `key` of a num_keys-key CWB; count <= 2^22 points per launch.  MK (batched keys): the
// launch's points are keys key .. key + count / ppk - 1, ppk points each (point p: key p / ppk),
// dig / dig_t / s0p hold those keys back to back, no shared prefix.
template <int NS, bool MASK_HEAD, bool XREG, bool MK, int WG = kBlock, int KR = 4>
__global__ __launch_bounds__(WG, 1) void k_eval_wide_head_stream(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk2, const uint4* __restrict__ dig,
    const uint8_t* __restrict__ dig_t, const uint8_t* __restrict__ cw_np1,
    const uint8_t* __restrict__ s0p, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint32_t lam, const uint64_t num_keys, const uint64_t key, const uint64_t count, uint32_t* __restrict__ ctr,
    uint8_t* __restrict__ ys, uint32_t* __restrict__ tvec, const WidePrefix pf, const uint32_t tw, const uint32_t ppk) {
  DCF_CLK(5, 0);  // (diagnostic builds) workgroup entry, before the table fill
  __shared__ uint32_t lds[kLdsWords];
  // Schedules of cipher 0 (slots 0..14) and cipher 17 (slots 23..37): 23 slots apart,
  // so lanes reading the two never share a ds_read_b128 bank group.
  __shared__ uint4 rks[23 + 15];
  if (threadIdx.x < 30) rks[threadIdx.x < 15 ? threadIdx.x : threadIdx.x + 8] = rk2[threadIdx.x];
  lds_fill_tables(lds, tab);  // its barrier also publishes rks
  DCF_CLK(1, 0);
  const uint32_t rks_a = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)rks;  // LDS byte address
  // Rounds 0 .. KR - 1 of both schedules in registers (8 VGPRs per round, lane-picked per block:
  // one 3-input pick per word), the rest read per lane from LDS.  C4 A/B r04j (2 runs each, same
  // box): KR = 4 33.99-34.15 ms vs 34.24-34.36 with every key from LDS, KR = 2 no change, KR = 6
  // spills.  More rounds at 8 waves per CU (512-thread workgroups, 2 streams per lane, up to all
  // 15 rounds in registers) ran 36.4-37.7 vs 31.8-32.0 ms (r04l): the head needs the 16 waves.
  uint32_t rkr[KR > 0 ? KR : 1][2][4];
#pragma unroll
  for (int r = 0; r < KR; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint4 k = rk2[c * 15 + r];
      rkr[r][c][0] = k.x; rkr[r][c][1] = k.y; rkr[r][c][2] = k.z; rkr[r][c][3] = k.w;
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(rkr[r][c][j]));
    }
  const uint32_t lc = lane_const();
  const uint32_t nlev = 8u * nbytes;
  const uint64_t nunits = (count + kWideUnit - 1) / kWideUnit;
  const uint32_t mlast = MASK_HEAD ? kMaskLast : 0xFFFFFFFFu;  // LAMBDA == 32: byte 31 is the cleared byte
  uint64_t unext = 0, uend = 0;
  bool exhausted = false;
  WideLane<NS> L;
  uint64_t nblk = 0;  // AES blocks this wave encrypts for live streams (wave-uniform)
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    L.alive[i] = false;
    L.lev[i] = 0u;
    L.ph[i] = 0u;
    L.kk[i] = 0u;  // an idle stream's CW loads stay in bounds
  }
#pragma unroll
  for (int i = 0; i < NS; ++i)
    wide_refill<NS, XREG, MK>(L, i, true, unext, uend, exhausted, ctr, nunits, count, s0p, party, xs, nbytes, pf,
                              tvec, tw, ppk, lam);

  for (;;) {
    bool any = false;
#pragma unroll
    for (int i = 0; i < NS; ++i) any = any || L.alive[i];
    if (!__ballot(any)) break;
#pragma unroll
    for (int i = 0; i < NS; ++i) nblk += (uint64_t)__popcll(__ballot(L.alive[i]));
    // Correction words, used only on the step that ends a level (the update masks them with
    // am): bytes [0,32) of cw_s / cw_v from the compact per-key digest (64 B per level,
    // 8 KiB, L1-resident; the CWB rows are LAMBDA bytes apart, one cache line per lane).
    // Loaded on every step (the level clamped for idle streams): under a branch they cost
    // 17 zeroing moves per step and the loads issued anyway.  Issued before the AES and
    // pinned after it, so they are waited on long after the last y / t-vector stores
    // (vmcnt is in order: a load issued after a store cannot be waited on alone).
    uint4 cs[NS][2], cv[NS][2];
    uint32_t ct[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint32_t lv = min(L.lev[i], nlev - 1u) + (MK ? L.kk[i] * nlev : 0u);
      const uint4* d4 = dig + 4u * lv;
      cs[i][0] = d4[0]; cs[i][1] = d4[1];
      cv[i][0] = d4[2]; cv[i][1] = d4[3];
      ct[i] = dig_t[lv];
    }
    // Block of this step: B (ph 0), then A (ph 1, left) or D (ph 1, right), C (ph 2).  The
    // lane's 16-byte half (sel) stays live: d = E(sel ^ inv) ^ sel ^ inv is one 3-input XOR.
    uint32_t st[NS][4], sel[NS][4], inv[NS];
    uint32_t ka[NS], hmk[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint32_t xb = L.cur[i] >> 31, ph = L.ph[i];
      const uint32_t hi = (ph != 0u) & xb;                            // D or C: bytes [16,32), cipher 17
      inv[i] = 0u - ((ph == 0u) | ((ph == 1u) & xb));                // B or D: ~s
      // cipher 17's schedule sits 23 slots on.  The empty asm keeps the compiler from
      // re-associating base + 16 r (rks_a is a link-time symbol: 14 materialised constants and
      // a v_mad per round); the mask proves the sign bit clear, so +16 r folds into ds_read
      uint32_t kb = rks_a + 368u * hi;
      asm volatile("" : "+v"(kb));
      ka[i] = kb & 0x3FFFFu;
      const uint32_t hm = 0u - hi;
      hmk[i] = hm;
      uint32_t k0w[4];
      if (KR > 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) k0w[j] = pick(hm, rkr[0][1][j], rkr[0][0][j]);
      } else {
        const uint4 k0 = lds_load16(ka[i]);
        k0w[0] = k0.x; k0w[1] = k0.y; k0w[2] = k0.z; k0w[3] = k0.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sel[i][j] = pick(hm, L.s[i][4 + j], L.s[i][j]);
        st[i][j] = xor3(sel[i][j], inv[i], k0w[j]);  // round key 0 folded in
      }
    }
    if (DCF_HEAD_PRIO) __builtin_amdgcn_s_setprio(1);  // A/B knob: the AES rounds at priority 1
    aes_tt_lka<14, NS, true, KR>(st, ka, lds, lc, rkr, hmk);
    if (DCF_HEAD_PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int i = 0; i < NS; ++i)
      asm volatile("" : "+v"(cs[i][0].x), "+v"(cs[i][0].y), "+v"(cs[i][0].z), "+v"(cs[i][0].w), "+v"(cs[i][1].x),
                   "+v"(cs[i][1].y), "+v"(cs[i][1].z), "+v"(cs[i][1].w), "+v"(cv[i][0].x), "+v"(cv[i][0].y),
                   "+v"(cv[i][0].z), "+v"(cv[i][0].w), "+v"(cv[i][1].x), "+v"(cv[i][1].y), "+v"(cv[i][1].z),
                   "+v"(cv[i][1].w), "+v"(ct[i]));
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint32_t xb = L.cur[i] >> 31, ph = L.ph[i];
      const bool live = L.alive[i];
      const uint32_t mB = 0u - (uint32_t)(live & (ph == 0u));
      const uint32_t mA = 0u - (uint32_t)(live & (ph == 1u) & (xb == 0u));
      const uint32_t mD = 0u - (uint32_t)(live & (ph == 1u) & (xb == 1u));
      const uint32_t mC = 0u - (uint32_t)(live & (ph == 2u));
      const uint32_t mBl = mB & (xb - 1u);  // B on a left step: v_L[0:16) = B ^ ~s
      const uint32_t adv = (mA | mC) & 1u;   // this step finishes the level
      const uint32_t am = 0u - adv, tm = 0u - L.t[i];
      // d = E(in) ^ in: the PRG output block (prg.rs:57-62)
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = xor3(st[i][j], sel[i][j], inv[i]);
      L.tR[i] = mB ? (d[0] & 1u) : L.tR[i];  // t_R = lsb(B ^ ~s)[0] (prg.rs:64)
#pragma unroll
      for (int j = 0; j < 4; ++j) L.dB[i][j] = pick(mB, d[j], L.dB[i][j]);
      // B reuse: a right step at t = 0 leaves s[0:16) as it is (s_R = s with only [16:32)
      // replaced, ^ 0 cw_s), so the next level's B = E0(~s[0:16)) is this level's
      const uint32_t ru = mC & (L.t[i] - 1u);
      const uint32_t tb = ((mA ? d[0] : L.tR[i]) & 1u) ^ (L.t[i] & (ct[i] >> xb) & 1u);  // lib.rs:179-180
      const uint32_t csw[8] = {cs[i][0].x, cs[i][0].y, cs[i][0].z, cs[i][0].w,
                               cs[i][1].x, cs[i][1].y, cs[i][1].z, cs[i][1].w};
      const uint32_t cvw[8] = {cv[i][0].x, cv[i][0].y, cv[i][0].z, cv[i][0].w,
                               cv[i][1].x, cv[i][1].y, cv[i][1].z, cv[i][1].w};
      // Three-input forms (one v_bitop3 each): xand(a, m, c) = a ^ (m & c),
      // xandn(a, m, c) = a ^ (m & ~c), pick(m, a, b) = m ? a : b (m all-ones or zero).
      const uint32_t amtm = am & tm;
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // bytes [0,16): AES on the left branch only
        // v ^= v_hat ^ t*cw.v: v_hat = B ^ ~s (left, at the B step) or ~s (right, at the C step)
        L.v[i][j] = xandn(xand(xand(L.v[i][j], amtm, cvw[j]), mBl, d[j]), mC, L.s[i][j]);
        // level end: s' = (A ^ s on the left, s on the right) ^ t*cw.s (lib.rs:177-178)
        L.s[i][j] = xand(pick(mA, d[j], L.s[i][j]), amtm, csw[j]);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {  // bytes [16,28): AES on the right branch only
        // v ^= v_hat ^ t*cw.v: v_hat = D ^ ~s (right, at the D step) or ~s (left, at the A step)
        L.v[i][4 + j] = xandn(xand(xand(L.v[i][4 + j], amtm, cvw[4 + j]), mD, d[j]), mA, L.s[i][4 + j]);
        // level end: s' = (C ^ s on the right, s on the left) ^ t*cw.s
        L.s[i][4 + j] = xand(pick(mC, d[j], L.s[i][4 + j]), amtm, csw[4 + j]);
      }
      {  // bytes [28,32): as above, with the cleared bit when LAMBDA == 32 (mlast)
        const uint32_t vh = xandn(mD & d[3], mA, L.s[i][7]) & mlast;
        L.v[i][7] = xand(L.v[i][7] ^ vh, amtm, cvw[7]);
        const uint32_t sn = xand(pick(mC, d[3], L.s[i][7]) & mlast, tm, csw[7]);
        L.s[i][7] = pick(am, sn, L.s[i][7]);  // an idle step keeps s (the root seed may be unmasked)
      }
      L.t[i] = adv ? tb : L.t[i];
      L.ph[i] = mB ? 1u : (mD ? 2u : 0u);
      const bool reuse = ru != 0u && L.lev[i] + adv != nlev;
      L.ph[i] = reuse ? 1u : L.ph[i];  // the next level starts at A / D
      // t-vector: row r = lev + 1 gets t_r (byte r >> 2, bit r & 3), the layout the tail reads
      const uint32_t r = L.lev[i] + adv;
      L.tacc[i] |= (am & L.t[i]) << (8u * ((r >> 2) & 3u) + (r & 3u));
      uint32_t* trow = tvec + (uint64_t)L.pt[i] * tw;
      const bool pdone = adv && r == nlev;
      if (adv && ((r & 15u) == 15u || pdone)) {
        trow[r >> 4] = L.tacc[i];
        L.tacc[i] = 0u;
      }
      L.cur[i] <<= adv;
      if (XREG) {  // next x word from the queue at a 32-level boundary
        const bool nw = adv && (r & 31u) == 0u;
        L.cur[i] = nw ? bswap32(L.xq[i][0]) : L.cur[i];
        L.xq[i][0] = nw ? L.xq[i][1] : L.xq[i][0];
        L.xq[i][1] = nw ? L.xq[i][2] : L.xq[i][1];
      } else if (adv && (r & 31u) == 0u && r < nlev) {
        L.cur[i] = load_bits32(xs + (uint64_t)L.pt[i] * nbytes, r >> 5, nbytes);
      }
      L.lev[i] = r;
      if (pdone) {  // y[0:32) = v ^ s ^ t * cw_np1 (lib.rs:192)
        const uint4* np4 = reinterpret_cast<const uint4*>(cw_np1 + (key + (MK ? L.kk[i] : 0u)) * lam);
        const uint4 n0 = np4[0], n1 = np4[1];
        const uint32_t nw[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
        const uint32_t tn = 0u - L.t[i];
        uint32_t y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = L.v[i][j] ^ L.s[i][j] ^ (tn & nw[j]);
        uint4* y4 = reinterpret_cast<uint4*>(ys + (uint64_t)L.pt[i] * lam);
        y4[0] = make_uint4(y[0], y[1], y[2], y[3]);
        y4[1] = make_uint4(y[4], y[5], y[6], y[7]);
      }
      {  // the skipped B step of the next level: v[0:16) ^= B ^ ~s when it goes left
        const uint32_t ml = 0u - (uint32_t)(reuse & ((L.cur[i] >> 31) == 0u));
#pragma unroll
        for (int j = 0; j < 4; ++j) L.v[i][j] = xand(L.v[i][j], ml, L.dB[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const bool done = L.alive[i] && L.lev[i] == nlev;
      if (__ballot(done))
        wide_refill<NS, XREG, MK>(L, i, done, unext, uend, exhausted, ctr, nunits, count, s0p, party, xs, nbytes,
                                  pf, tvec, tw, ppk, lam);
    }
  }
  // ctr[2..3]: the launch's AES block count (dcf_prg_last_eval_blocks), accumulated over passes
  if ((threadIdx.x & 63u) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(ctr) + 1, (unsigned long long)nblk);
  DCF_CLK(1, 1);
}

// One wide prefix node (80 B: s[0:32) | v[0:32) | {t, t-vector word 0, partial word, 0}) at depth
// `lev` -> its two children, bytes [0,32) of the walk exactly as k_eval_wide_head_stream updates
// them, on a lane QUAD: lane q encrypts one of the node's four blocks — A = E0(s_lo), B = E0(~s_lo),
// C = E17(s_hi), D = E17(~s_hi) for q = 0..3 — and writes the child pieces its block decides:
//   q = 0: left s_lo = A ^ s_lo ^ t cs_lo            right s_lo = s_lo ^ t cs_lo
//   q = 1: left v_lo = v_lo ^ B ^ ~s_lo ^ t cv_lo    right v_lo = v_lo ^ ~s_lo ^ t cv_lo
//   q = 2: right s_hi = (C ^ s_hi) & M ^ t cs_hi     left s_hi = s_hi & M ^ t cs_hi           + left's word 4
//   q = 3: right v_hi = v_hi ^ (D ^ ~s_hi) & M ^ t cv_hi   left v_hi = v_hi ^ ~s_hi & M ^ t cv_hi   + right's word 4
// (prg.rs:57-68 under the diagonal zip; M clears bit 0 of byte 31 when LAMBDA == 32), t_L = lsb(A ^ s)[0]
// ^ t cw.tl from lane 0 and t_R = lsb(B ^ ~s)[0] ^ t cw.tr from lane 1, broadcast over the quad
// (lib.rs:177-180).  One block per lane instead of four: a level's latency is one AES chain, and no
// lane holds more than a node piece (the four-block form held 2 x 5 uint4 of children and spilled
// to 176 B of scratch).  Must run in uniform control flow (DPP): whole waves, quads past the level's
// nodes compute a copy and skip the stores.  rks_a: LDS byte address of the schedules (cipher 0 at
// slot 0, cipher 17 at slot 23); node / piece pointers may be LDS or global.
struct WpfxQuad {
  uint32_t q, lo, in_piece, v_piece, cw_piece, ka;
  __device__ __forceinline__ void init(uint32_t rks_a) {
    q = threadIdx.x & 3u;
    lo = (q >> 1) == 0u;                 // bytes [0,16): blocks A, B (cipher 0)
    in_piece = q >> 1;                   // s_lo / s_hi
    v_piece = 2u + (q >> 1);             // v_lo / v_hi
    cw_piece = (q & 1u) ? 2u + (q >> 1) : (q >> 1);  // digest row: cs_lo, cs_hi, cv_lo, cv_hi = 0, 1, 2, 3
    ka = rks_a + (lo ? 0u : 368u);
  }
  // the pieces of node `n` (LDS or global) this lane reads: its AES input half, its v half, word 4
  __device__ __forceinline__ void load(const uint4* n, uint4& sp, uint4& vp, uint4& e) const {
    sp = n[in_piece];
    vp = n[v_piece];
    e = n[4];
  }
};

template <bool MASK_HEAD>
__device__ __forceinline__ void wpfx_quad_children(const uint32_t* lds, uint32_t lc, const WpfxQuad& Q,
                                                   const uint4* __restrict__ dig, const uint8_t* __restrict__ dig_t,
                                                   uint32_t lev, const uint4 sp, const uint4 vp, const uint4 e,
                                                   bool store, uint4* left, uint4* right) {
  const uint32_t q = Q.q;
  const uint4 cw = dig[4u * lev + Q.cw_piece];
  const uint32_t ct = dig_t[lev];
  const uint32_t inv = 0u - (q & 1u);
  const uint32_t s[4] = {sp.x, sp.y, sp.z, sp.w}, v[4] = {vp.x, vp.y, vp.z, vp.w};
  const uint32_t c[4] = {cw.x, cw.y, cw.z, cw.w};
  uint32_t st[1][4];
  const uint32_t ka[1] = {Q.ka};
#pragma unroll
  for (int j = 0; j < 4; ++j) st[0][j] = s[j] ^ inv;
  aes_tt_lka<14, 1, false>(st, ka, lds, lc);
  const uint32_t t = e.x, tm = 0u - t;
  // d = E(in) ^ in: the PRG output block (prg.rs:57-62); bit 0 of byte 31 masked (hi half, LAMBDA == 32)
  const uint32_t mlast = (MASK_HEAD && !Q.lo) ? kMaskLast : 0xFFFFFFFFu;
  uint32_t d[4], keep[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t m = (j == 3) ? mlast : 0xFFFFFFFFu;
    d[j] = (st[0][j] ^ s[j] ^ inv) & m;   // A ^ s, B ^ ~s, C ^ s, D ^ ~s
    keep[j] = (s[j] ^ inv) & m;           // the branch this block does not touch: s or ~s
  }
  // t_L (lane 0: lsb of A ^ s), t_R (lane 1: lsb of B ^ ~s), each ^ t & its cw.t bit
  const uint32_t tb = (d[0] ^ (t & (ct >> (q & 1u)))) & 1u;
  const uint32_t tl = dpp<kQpBcast0>(tb), tr = dpp<1 | (1 << 2) | (1 << 4) | (1 << 6)>(tb);
  if (!store) return;
  // AES'd piece (to the block's branch) and the pass-through piece (to the other branch); the v
  // lanes (q odd) add v, every piece adds t * its CW piece
  uint4 pa, pk;
  {
    uint32_t a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t base = (q & 1u) ? v[j] : 0u;
      a[j] = base ^ d[j] ^ (tm & c[j]);
      b[j] = base ^ keep[j] ^ (tm & c[j]);
    }
    pa = make_uint4(a[0], a[1], a[2], a[3]);
    pk = make_uint4(b[0], b[1], b[2], b[3]);
  }
  // A (q 0) and B (q 1) belong to the left child, C (q 2) and D (q 3) to the right one
  uint4* mine = Q.lo ? left : right;
  uint4* other = Q.lo ? right : left;
  const uint32_t piece = (q & 1u) ? Q.v_piece : Q.in_piece;
  mine[piece] = pa;
  other[piece] = pk;
  if (q >= 2u) {  // word 4: t, t-vector word 0, partial word (row r = lev + 1 at bit pos)
    const uint32_t r = lev + 1u, pos = 8u * ((r >> 2) & 3u) + (r & 3u);
    const uint32_t tc = (q == 2u) ? tl : tr;
    uint32_t acc = e.z | (tc << pos), w0 = e.y;
    if ((r & 15u) == 15u) {  // word r >> 4 of the t-vector is complete (r < 31: word 0)
      w0 = acc;
      acc = 0u;
    }
    ((q == 2u) ? left : right)[4] = make_uint4(tc, w0, acc, 0u);
  }
}

// The whole wide prefix tree of depth D in ONE launch (as k_prefix_build16 at LAMBDA = 16):
// workgroup w (2^S of them) owns the subtree under node w of level S.  One lane quad walks the
// root path (root = k.s0s[0][0:32), v = 0, t = party, t-vector row 0 = party: lib.rs:167-169);
// the workgroup then expands its subtree level by level (a quad per node, wpfx_quad_children):
// while a level has <= kWpfxLdsPar parents its children stay in an LDS node buffer (two barriers
// per level, no global round trip); wider levels go through the workgroup's regions (R =
// 2^(D-1-S) nodes of 80 B) of two global buffers, waves claiming 16 nodes at a time from an LDS
// counter (waves of a workgroup do not progress at one rate); the last level writes the
// workgroup's contiguous block of the table.  C4 (D = 21): the build went from 0.38 ms with a
// lone wave's four-block T-table calls on the root path and every level through global memory.
constexpr uint32_t kWpfxLdsNodes = 384;  // 30 KiB of 80-byte nodes beside the 128 KiB tables
constexpr uint32_t kWpfxLdsPar = 128;    // parents per level whose children stay in the LDS (256 <= 384)
template <bool MASK_HEAD>
__global__ __launch_bounds__(kBlock, 1) void k_wpfx_build(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk2, const uint4* __restrict__ dig,
    const uint8_t* __restrict__ dig_t, const uint8_t* __restrict__ s0p, const uint32_t party, const uint32_t S,
    const uint32_t D, uint4* __restrict__ buf_a, uint4* __restrict__ buf_b, const uint32_t region_nodes,
    uint4* __restrict__ table) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 rks[23 + 15];
  __shared__ uint4 nodes[5 * kWpfxLdsNodes];
  __shared__ uint32_t claim;
  if (threadIdx.x < 30) rks[threadIdx.x < 15 ? threadIdx.x : threadIdx.x + 8] = rk2[threadIdx.x];
  if (threadIdx.x < 5) {  // the root node (level 0) into LDS slot 0
    const uint4* s4 = reinterpret_cast<const uint4*>(s0p);
    nodes[threadIdx.x] = threadIdx.x < 2 ? s4[threadIdx.x]
                                          : (threadIdx.x < 4 ? make_uint4(0u, 0u, 0u, 0u)
                                                             : make_uint4(party, 0u, party, 0u));
  }
  lds_fill_tables(lds, tab);  // its barrier publishes rks and the root
  DCF_CLK(6, 0);  // (diagnostic builds; slots 6 / 7 are k_prefix_build16's at LAMBDA = 16) after the fill
  const uint32_t lc = lane_const();
  WpfxQuad Q;
  Q.init((uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)rks);
  const uint32_t w = blockIdx.x, g = threadIdx.x >> 2;  // quad g of 256
  const uint32_t nq = blockDim.x >> 2;
  if (threadIdx.x < 64) {  // wave 0, quad 0: root -> node w of level S (slot 0 -> slot 0)
    for (uint32_t lev = 0; lev < S; ++lev) {
      const bool right = (w >> (S - 1u - lev)) & 1u;
      // children to slots 1 / 2, then the chosen one back to slot 0 (one wave: LDS is in order)
      uint4 sp, vp, e;
      Q.load(nodes, sp, vp, e);
      wpfx_quad_children<MASK_HEAD>(lds, lc, Q, dig, dig_t, lev, sp, vp, e, g == 0u, nodes + 5, nodes + 10);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (threadIdx.x < 5) nodes[threadIdx.x] = nodes[(right ? 10 : 5) + threadIdx.x];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  }
  __syncthreads();
  DCF_CLK(6, 1);  // root path done
  const uint64_t R5 = 5ull * region_nodes;
  uint4* X = buf_a + (uint64_t)w * R5;
  uint4* Y = buf_b + (uint64_t)w * R5;
  uint32_t lev = S;
  // narrow levels in the LDS: parents in slots [0, np), children to [0, 2 np) after a barrier
  for (; lev < D && (1u << (lev - S)) <= kWpfxLdsPar; ++lev) {
    const uint32_t np = 1u << (lev - S);
    const bool last = lev + 1u == D;
    const uint32_t j = g < np ? g : np - 1u;
    uint4 sp, vp, e;
    Q.load(nodes + 5u * j, sp, vp, e);
    __syncthreads();  // every parent read before any child overwrites it
    uint4* out = last ? table + 5ull * ((uint64_t)w << (D - S)) : nodes;
    if (g - (g & 15u) < np)  // whole waves (uniform DPP); quads past np store nothing
      wpfx_quad_children<MASK_HEAD>(lds, lc, Q, dig, dig_t, lev, sp, vp, e, g < np, out + 10u * j, out + 10u * j + 5u);
    __syncthreads();
  }
  if (lev == D) return;
  // wide levels: parents from the LDS (first one) or X, children to Y or the table
  bool from_lds = true;
  for (; lev < D; ++lev) {
    const uint32_t np = 1u << (lev - S);
    const bool last = lev + 1u == D;
    uint4* out = last ? table + 5ull * ((uint64_t)w << (D - S)) : Y;
    const uint4* in = from_lds ? nodes : X;
    if (threadIdx.x == 0) claim = 0u;
    __syncthreads();
    for (;;) {  // 16 nodes per wave per claim (np is a multiple of 256 here)
      uint32_t base = 0u;
      if ((threadIdx.x & 63u) == 0)
        base = __hip_atomic_fetch_add(&claim, 16u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      base = __builtin_amdgcn_readfirstlane(base);
      if (base >= np) break;
      const uint32_t j = base + ((threadIdx.x & 63u) >> 2);
      uint4 sp, vp, e;
      Q.load(in + 5u * j, sp, vp, e);
      wpfx_quad_children<MASK_HEAD>(lds, lc, Q, dig, dig_t, lev, sp, vp, e, true, out + 10u * j, out + 10u * j + 5u);
    }
    __syncthreads();  // the workgroup's children are its next parents
    uint4* tmp = X;
    X = Y;
    Y = tmp;
    from_lds = false;
  }
  DCF_CLK(7, 1);
}

}  // namespace
