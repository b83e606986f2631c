// kernels16.h — LAMBDA = 16 kernels (eval, batched gen, PRG hook).
// Included by dcf_hip.hip only.
#pragma once

#include "aes_lds.h"
#include "kernels_lat.h"

// A/B knob: the pair walk's AES rounds (k_eval16_pair, k_eval16) at wave priority 1.
#ifndef DCF_PAIR_PRIO
#define DCF_PAIR_PRIO 1
#endif

namespace {


// ------------------------------------------------------------------------
// k_eval16: DcfImpl::eval (lib.rs:163-204) at LAMBDA = 16.
//   MODE 0: one key.  MODE 1: K keys, points_per_key % 64 == 0 (key is
//   wave-uniform -> scalar CW loads).  MODE 2: K keys, any points_per_key.
// The Hirose PRG at LAMBDA = 16 (prg.rs:42-73 with the diagonal zip):
//   A = AES_K0(s), B = AES_K0(~s), M = clear bit0 of byte 15
//   L = ((A^s)&M, (B^~s)&M, lsb(A^s)[0]),  R = (s&M, ~s&M, lsb(B^~s)[0])
// ------------------------------------------------------------------------
// One point, one lane: returns y for point gg of key `key` (the whole
// lib.rs:166-193 closure).  Used by k_eval16.
__device__ __forceinline__ uint4 tt_eval_one(const uint32_t* lds, uint32_t lc, const RoundKeys& rk,
                                             const uint4* __restrict__ cw_s, const uint4* __restrict__ cw_v,
                                             const uint8_t* __restrict__ cw_t, const uint4 np, const uint4 sv,
                                             uint32_t party, const uint8_t* __restrict__ x, uint32_t nbytes,
                                             uint64_t num_keys, uint64_t key) {
  const uint32_t nlev = 8u * nbytes;
  const uint32_t nchunk = (nbytes + 3u) >> 2;
  uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  uint32_t t = party;
  uint32_t lev = 0;
  for (uint32_t c = 0; c < nchunk; ++c) {
    uint32_t cur = load_bits32(x, c, nbytes);
    const uint32_t lend = min(32u, nlev - 32u * c);
    for (uint32_t b = 0; b < lend; ++b, ++lev) {
      uint32_t st[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        st[0][j] = s[j];
        st[1][j] = ~s[j];
      }
      if (DCF_PAIR_PRIO) __builtin_amdgcn_s_setprio(1);
      aes256_tt<2>(st, rk, lds, lc);  // st[0] = A, st[1] = B
      if (DCF_PAIR_PRIO) __builtin_amdgcn_s_setprio(0);
      const uint64_t ci = (uint64_t)lev * num_keys + key;
      const uint4 cs = cw_s[ci];
      const uint4 cv = cw_v[ci];
      const uint32_t ct = cw_t[ci];
      const uint32_t xb = cur >> 31;  // Msb0 bit of x (lib.rs:181)
      cur <<= 1;
      const uint32_t keepA = xb - 1u;  // all ones when going left
      const uint32_t tm = 0u - t;
      const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w};
      const uint32_t cvw[4] = {cv.x, cv.y, cv.z, cv.w};
      // t' (lib.rs:179-180, 183/187): left lsb(A^s)[0] ^ t&tl, right lsb(B^~s)[0] ^ t&tr
      const uint32_t tl = (st[0][0] ^ s[0]) & 1u;
      const uint32_t tr = (st[1][0] ^ ~s[0]) & 1u;
      const uint32_t tn = (xb ? tr : tl) ^ (t & (ct >> xb) & 1u);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
        // v ^= v_hat(side) ^ t*cw.v   (lib.rs:182/186)
        v[j] ^= (((~s[j]) ^ (st[1][j] & keepA)) & msk) ^ (tm & cvw[j]);
        // s' = s(side) ^ t*cw.s       (lib.rs:177-178, 183/187)
        s[j] = ((s[j] ^ (st[0][j] & keepA)) & msk) ^ (tm & csw[j]);
      }
      t = tn;
    }
  }
  // y = v ^ s_n ^ t_n*cw_np1 (lib.rs:192)
  const uint32_t tm = 0u - t;
  return make_uint4(v[0] ^ s[0] ^ (tm & np.x), v[1] ^ s[1] ^ (tm & np.y), v[2] ^ s[2] ^ (tm & np.z),
                    v[3] ^ s[3] ^ (tm & np.w));
}

// Work distribution: with ctr == nullptr a grid-stride loop (small batches: every
// wave runs once); otherwise waves take 64-point units from the counter, so the
// waves of a CU drift apart and their AES rounds do not hit the LDS in lockstep
// bursts (C5: see DESIGN.md).
__device__ __forceinline__ uint64_t next_wave_base(uint32_t* __restrict__ ctr, uint64_t base, uint64_t stride) {
  if (!ctr) return base + stride;
  uint32_t u = 0;
  if ((threadIdx.x & 63u) == 0) u = atomicAdd(ctr, 1u);
  return (uint64_t)__builtin_amdgcn_readfirstlane(u) * 64u;
}

// Units of 64 * U consecutive items for kernels with little work per item (the
// full-domain levels: one PRG call per node): a wave walks its unit 64 items at a
// time and takes the next unit from ctr, so one atomic covers U wave iterations.
// Start with base = ~0.
template <uint32_t U>
__device__ __forceinline__ uint64_t next_unit_base(uint32_t* __restrict__ ctr, uint64_t base) {
  if (base != ~0ull && ((base >> 6) + 1) % U != 0) return base + 64;
  uint32_t u = 0;
  if ((threadIdx.x & 63u) == 0) u = atomicAdd(ctr, 1u);
  return (uint64_t)__builtin_amdgcn_readfirstlane(u) * 64u * U;
}
constexpr uint32_t kFdUnit = 16;

// Runtime unit size for a grid over n items: kFdUnit wave iterations per unit when
// there is work for every wave that many times over, fewer (down to 1) otherwise,
// so a small level is spread over all the grid's waves instead of one wave walking
// a whole 1024-item unit (the shared-prefix tables' upper levels: 60-110 us each).
__device__ __forceinline__ uint32_t fd_unit(uint64_t n) {
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t per = n / (64u * waves);
  return per >= kFdUnit ? kFdUnit : (per ? (uint32_t)per : 1u);
}
__device__ __forceinline__ uint64_t next_unit_base_n(uint32_t* __restrict__ ctr, uint64_t base, uint32_t U) {
  if (base != ~0ull && ((base >> 6) + 1) % U != 0) return base + 64;
  uint32_t u = 0;
  if ((threadIdx.x & 63u) == 0) u = atomicAdd(ctr, 1u);
  return (uint64_t)__builtin_amdgcn_readfirstlane(u) * 64u * U;
}

template <int MODE>
__global__ __launch_bounds__(kBlock, 1) void k_eval16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t num_keys, const uint64_t points_per_key, uint4* __restrict__ ys, uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint64_t total = num_keys * points_per_key;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t first = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
  for (uint64_t base = ctr ? next_wave_base(ctr, 0, 0) : first; base < total;
       base = next_wave_base(ctr, base, stride)) {
    const uint64_t g = base + (threadIdx.x & 63u);
    const bool live = g < total;
    const uint64_t gg = live ? g : total - 1;
    uint64_t key = 0;
    if (MODE == 1) key = __builtin_amdgcn_readfirstlane((uint32_t)(gg / points_per_key));
    if (MODE == 2) key = gg / points_per_key;
    const uint4 y = tt_eval_one(lds, lc, rk, cw_s, cw_v, cw_t, cw_np1[key], s0s[key], party, xs + gg * nbytes,
                                nbytes, num_keys, key);
    if (live) ys[g] = y;
  }
}

// Shared prefix (single key): the walk's state after its first `levels` levels depends
// only on those bits of x, so the host expands that top tree once (the full-domain
// level kernels, k_fd_level16 / k_fd_level16_mmo) into a table indexed by the prefix, and a point
// starts at level `levels` from its table row.  levels = 0: no table.
// Row i is 32 contiguous bytes, sv[2i] = s and sv[2i+1] = v, with t in s's bit 0 of
// byte 15: below the root s is always masked there (s' = side & M ^ t*cw.s, and cw.s
// is a XOR of two masked seeds, lib.rs:119-121 / prg.rs:63-68), so a point's start
// is one 32-byte gather (one cache line) instead of three arrays' lines.
struct PrefixTable {
  const uint4* sv;
  uint32_t levels;  // < 32 and < 8N
};

__device__ __forceinline__ void prefix_row(const PrefixTable& pf, uint32_t idx, uint4& s, uint4& v, uint32_t& t) {
  s = pf.sv[2u * idx];
  v = pf.sv[2u * idx + 1u];
  t = (s.w >> 24) & 1u;
  s.w &= kMaskLast;
}

// Small batches, two lanes per point: lane 2k encrypts A = AES(s), lane 2k + 1
// B = AES(~s), they swap the result (DPP quad_perm 1,0,3,2) and both run the level
// update (lib.rs:174-189).  Twice the waves of k_eval16 for the same points, each
// with half the AES work per level: a small batch has too few waves per SIMD to
// overlap the LDS lookups with the rest (C1: 7 waves per CU with one lane per point).
constexpr int kQpSwap1 = 1 | (0 << 2) | (3 << 4) | (2 << 6);

__device__ __forceinline__ uint4 tt_eval_pair(const uint32_t* lds, uint32_t lc, const RoundKeys& rk,
                                              const uint4* __restrict__ cw_s, const uint4* __restrict__ cw_v,
                                              const uint8_t* __restrict__ cw_t, const uint4 np, const uint4 sv,
                                              uint32_t party, const uint8_t* __restrict__ x, uint32_t nbytes,
                                              uint64_t num_keys, uint64_t key, uint32_t odd,
                                              const uint4* __restrict__ rkg, const PrefixTable& pf) {
  const uint32_t nlev = 8u * nbytes;
  const uint32_t nchunk = (nbytes + 3u) >> 2;
  const uint32_t inv = 0u - odd;  // odd lane: ~s (B)
  uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  uint32_t t = party;
  uint32_t lev = 0;
  if (pf.levels) {  // start at level D from the row named by x's first D bits (Msb0)
    uint4 s4, v4;
    prefix_row(pf, load_bits32(x, 0, nbytes) >> (32u - pf.levels), s4, v4, t);
    s[0] = s4.x; s[1] = s4.y; s[2] = s4.z; s[3] = s4.w;
    v[0] = v4.x; v[1] = v4.y; v[2] = v4.z; v[3] = v4.w;
    lev = pf.levels;
  }
  for (uint32_t c = lev >> 5; c < nchunk; ++c) {
    const uint32_t b0 = (32u * c < lev) ? (lev & 31u) : 0u;
    uint32_t cur = load_bits32(x, c, nbytes) << b0;
    const uint32_t lend = min(32u, nlev - 32u * c);
    for (uint32_t b = b0; b < lend; ++b, ++lev) {
      uint32_t st[1][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) st[0][j] = s[j] ^ inv;
      if (DCF_PAIR_PRIO) __builtin_amdgcn_s_setprio(1);
      aes256_tt_gk<1>(st, rkg, lds, lc);  // round keys per round from global memory (SGPR keys spill)
      if (DCF_PAIR_PRIO) __builtin_amdgcn_s_setprio(0);
      uint32_t A[4], B[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t other = (uint32_t)__builtin_amdgcn_mov_dpp((int)st[0][j], kQpSwap1, 0xF, 0xF, true);
        A[j] = odd ? other : st[0][j];
        B[j] = odd ? st[0][j] : other;
      }
      const uint64_t ci = (uint64_t)lev * num_keys + key;
      const uint4 cs = cw_s[ci];
      const uint4 cv = cw_v[ci];
      const uint32_t ct = cw_t[ci];
      const uint32_t xb = cur >> 31;  // Msb0 bit of x (lib.rs:181)
      cur <<= 1;
      const uint32_t keepA = xb - 1u;  // all ones when going left
      const uint32_t tm = 0u - t;
      const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w};
      const uint32_t cvw[4] = {cv.x, cv.y, cv.z, cv.w};
      const uint32_t tl = (A[0] ^ s[0]) & 1u;
      const uint32_t tr = (B[0] ^ ~s[0]) & 1u;
      const uint32_t tn = (xb ? tr : tl) ^ (t & (ct >> xb) & 1u);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
        v[j] ^= (((~s[j]) ^ (B[j] & keepA)) & msk) ^ (tm & cvw[j]);  // lib.rs:182/186
        s[j] = ((s[j] ^ (A[j] & keepA)) & msk) ^ (tm & csw[j]);      // lib.rs:177-178, 183/187
      }
      t = tn;
    }
  }
  const uint32_t tm = 0u - t;  // y = v ^ s_n ^ t_n*cw_np1 (lib.rs:192)
  return make_uint4(v[0] ^ s[0] ^ (tm & np.x), v[1] ^ s[1] ^ (tm & np.y), v[2] ^ s[2] ^ (tm & np.z),
                    v[3] ^ s[3] ^ (tm & np.w));
}

template <int MODE>
__global__ __launch_bounds__(kBlock, 1) void k_eval16_pair(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t num_keys, const uint64_t points_per_key, uint4* __restrict__ ys,
    const uint4* __restrict__ rkg, const PrefixTable pf) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint64_t total = num_keys * points_per_key;
  const uint64_t stride = (uint64_t)gridDim.x * (blockDim.x >> 1);
  for (uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 1; g - ((threadIdx.x & 63u) >> 1) < total;
       g += stride) {
    const bool live = g < total;
    const uint64_t gg = live ? g : total - 1;
    uint64_t key = 0;
    if (MODE == 1) key = __builtin_amdgcn_readfirstlane((uint32_t)(gg / points_per_key));
    if (MODE == 2) key = gg / points_per_key;
    const uint32_t odd = threadIdx.x & 1u;
    const uint4 y = tt_eval_pair(lds, lc, rk, cw_s, cw_v, cw_t, cw_np1[key], s0s[key], party, xs + gg * nbytes,
                                 nbytes, num_keys, key, odd, rkg, pf);
    if (live && !odd) ys[g] = y;
  }
}

// ------------------------------------------------------------------------
// k_gen16: DcfImpl::gen (lib.rs:86-161) at LAMBDA = 16.  Four AES blocks per level
// (PRG on both parties' seeds, lib.rs:103-104): LANES = 1, one lane per key encrypts all
// four; LANES = 4, a lane quad per key, lane q encrypts block q (A0, B0, A1, B1) and a DPP
// broadcast per word hands every lane of the quad all four, which then run the same
// level update (a key's 8N levels take a quarter of the AES latency: single-key gen).
// ------------------------------------------------------------------------
template <int LANES>
__global__ __launch_bounds__(kBlock, 1) void k_gen16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint8_t* __restrict__ alpha,
    const uint4* __restrict__ beta, const uint4* __restrict__ s0_0, const uint4* __restrict__ s0_1,
    const uint32_t bound, const uint32_t nbytes, const uint64_t num_keys, uint4* __restrict__ cw_s,
    uint4* __restrict__ cw_v, uint8_t* __restrict__ cw_t, uint4* __restrict__ cw_np1, uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint32_t nlev = 8u * nbytes;
  const uint32_t nchunk = (nbytes + 3u) >> 2;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t first = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
  const uint64_t items = num_keys * LANES;
  for (uint64_t base = ctr ? next_wave_base(ctr, 0, 0) : first; base < items;
       base = next_wave_base(ctr, base, stride)) {
    const uint64_t g = base + (threadIdx.x & 63u);
    const bool live = g < items;
    const uint64_t k = (live ? g : items - 1) / LANES;
    const uint32_t q = (uint32_t)(g % LANES);  // LANES = 4: this lane's block (0 A0, 1 B0, 2 A1, 3 B1)
    uint32_t s[2][4], va[4] = {0u, 0u, 0u, 0u}, be[4];
    {
      const uint4 a0 = s0_0[k], a1 = s0_1[k], bb = beta[k];
      s[0][0] = a0.x; s[0][1] = a0.y; s[0][2] = a0.z; s[0][3] = a0.w;
      s[1][0] = a1.x; s[1][1] = a1.y; s[1][2] = a1.z; s[1][3] = a1.w;
      be[0] = bb.x; be[1] = bb.y; be[2] = bb.z; be[3] = bb.w;
    }
    uint32_t t0 = 0u, t1 = 1u;  // lib.rs:100
    const uint8_t* al = alpha + k * nbytes;
    uint32_t lev = 0;
    for (uint32_t c = 0; c < nchunk; ++c) {
      uint32_t cur = load_bits32(al, c, nbytes);
      const uint32_t lend = min(32u, nlev - 32u * c);
      for (uint32_t b = 0; b < lend; ++b, ++lev) {
        uint32_t st[4][4];
        if (LANES == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            st[0][j] = s[0][j];
            st[1][j] = ~s[0][j];
            st[2][j] = s[1][j];
            st[3][j] = ~s[1][j];
          }
          aes256_tt<4>(st, rk, lds, lc);  // A0, B0, A1, B1
        } else {
          uint32_t one[1][4];
          const uint32_t inv = 0u - (q & 1u);  // B blocks encrypt ~s
#pragma unroll
          for (int j = 0; j < 4; ++j) one[0][j] = ((q >> 1) ? s[1][j] : s[0][j]) ^ inv;
          aes256_tt<1>(one, rk, lds, lc);
#pragma unroll
          for (int j = 0; j < 4; ++j) {  // quad_perm broadcasts of lane b's block (b, b, b, b)
            st[0][j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)one[0][j], 0x00, 0xF, 0xF, true);
            st[1][j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)one[0][j], 0x55, 0xF, 0xF, true);
            st[2][j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)one[0][j], 0xAA, 0xF, 0xF, true);
            st[3][j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)one[0][j], 0xFF, 0xF, 0xF, true);
          }
        }
        const uint32_t a = cur >> 31;   // alpha_i, Msb0 (lib.rs:106)
        cur <<= 1;
        const uint32_t am = 0u - a;     // all ones when keep = R, lose = L
        // LtBeta: beta joins v_cw when lose == L (alpha_i = 1); GtBeta when lose == R (lib.rs:114-125)
        const uint32_t bm = (bound == 0) ? am : ~am;
        uint32_t scw[4], vcw[4];
        // PRG outputs per party p: L = ((A^s)&M, (B^~s)&M), R = (s&M, ~s&M)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
          const uint32_t sl0 = (st[0][j] ^ s[0][j]) & msk, vl0 = (st[1][j] ^ ~s[0][j]) & msk;
          const uint32_t sr0 = s[0][j] & msk, vr0 = ~s[0][j] & msk;
          const uint32_t sl1 = (st[2][j] ^ s[1][j]) & msk, vl1 = (st[3][j] ^ ~s[1][j]) & msk;
          const uint32_t sr1 = s[1][j] & msk, vr1 = ~s[1][j] & msk;
          const uint32_t slose0 = a ? sl0 : sr0, slose1 = a ? sl1 : sr1;
          const uint32_t vlose0 = a ? vl0 : vr0, vlose1 = a ? vl1 : vr1;
          const uint32_t vkeep0 = a ? vr0 : vl0, vkeep1 = a ? vr1 : vl1;
          scw[j] = slose0 ^ slose1;                                    // lib.rs:112
          vcw[j] = vlose0 ^ vlose1 ^ va[j] ^ (bm & be[j]);             // lib.rs:113-125
          va[j] ^= vkeep0 ^ vkeep1 ^ vcw[j];                           // lib.rs:126-129
        }
        const uint32_t tl0 = (st[0][0] ^ s[0][0]) & 1u, tr0 = (st[1][0] ^ ~s[0][0]) & 1u;
        const uint32_t tl1 = (st[2][0] ^ s[1][0]) & 1u, tr1 = (st[3][0] ^ ~s[1][0]) & 1u;
        const uint32_t tlcw = tl0 ^ tl1 ^ a ^ 1u;  // lib.rs:130
        const uint32_t trcw = tr0 ^ tr1 ^ a;       // lib.rs:131
        const uint32_t tkcw = a ? trcw : tlcw;
        const uint32_t m0 = 0u - t0, m1 = 0u - t1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // lib.rs:139-148
          const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
          const uint32_t sk0 = a ? (s[0][j] & msk) : ((st[0][j] ^ s[0][j]) & msk);
          const uint32_t sk1 = a ? (s[1][j] & msk) : ((st[2][j] ^ s[1][j]) & msk);
          s[0][j] = sk0 ^ (m0 & scw[j]);
          s[1][j] = sk1 ^ (m1 & scw[j]);
        }
        const uint32_t nt0 = (a ? tr0 : tl0) ^ (t0 & tkcw);  // lib.rs:149-152
        const uint32_t nt1 = (a ? tr1 : tl1) ^ (t1 & tkcw);
        t0 = nt0;
        t1 = nt1;
        if (live) {  // LANES = 4: the quad's lanes 0, 1, 2 store one output each
          const uint64_t ci = (uint64_t)lev * num_keys + k;
          if (LANES == 1 || q == 0) cw_s[ci] = make_uint4(scw[0], scw[1], scw[2], scw[3]);
          if (LANES == 1 || q == 1) cw_v[ci] = make_uint4(vcw[0], vcw[1], vcw[2], vcw[3]);
          if (LANES == 1 || q == 2) cw_t[ci] = (uint8_t)(tlcw | (trcw << 1));
        }
      }
    }
    if (live && (LANES == 1 || q == 0))  // lib.rs:155
      cw_np1[k] = make_uint4(s[0][0] ^ s[1][0] ^ va[0], s[0][1] ^ s[1][1] ^ va[1], s[0][2] ^ s[1][2] ^ va[2],
                             s[0][3] ^ s[1][3] ^ va[3]);
  }
}

// ------------------------------------------------------------------------
// k_prg16: Aes256HirosePrg::gen (prg.rs:42-73) at LAMBDA = 16 for m seeds.
// Output row per seed: s_l | v_l | s_r | v_r | t_l | t_r (66 bytes).
// ------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock, 1) void k_prg16(const uint32_t* __restrict__ tab, const RoundKeys rk,
                                                     const uint4* __restrict__ seeds, const uint64_t m,
                                                     uint8_t* __restrict__ out) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < m; g += stride) {
    const uint4 sv = seeds[g];
    const uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
    uint32_t st[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      st[0][j] = s[j];
      st[1][j] = ~s[j];
    }
    aes256_tt<2>(st, rk, lds, lc);
    uint32_t o[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
      o[0][j] = (st[0][j] ^ s[j]) & msk;
      o[1][j] = (st[1][j] ^ ~s[j]) & msk;
      o[2][j] = s[j] & msk;
      o[3][j] = ~s[j] & msk;
    }
    uint8_t* row = out + g * 66;
    for (int q = 0; q < 4; ++q)
      for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) row[16 * q + 4 * j + k] = (uint8_t)(o[q][j] >> (8 * k));
    row[64] = (uint8_t)((st[0][0] ^ s[0]) & 1u);
    row[65] = (uint8_t)((st[1][0] ^ ~s[0]) & 1u);
  }
}

}  // namespace

namespace {

// ------------------------------------------------------------------------
// Full-domain eval at LAMBDA = 16: y for every x in [0, 2^n),
// n = 8N, by breadth-first tree expansion.  One lane per parent node per
// level: one PRG call (A, B) yields BOTH children, so the whole domain costs
// 2 AES blocks per leaf instead of 2n per point.  Node state (s, v, t) lives in
// SoA buffers indexed by the big-endian x prefix; the last level writes y.
// Child rules are lib.rs:176-189 with x-bit 0 (left) / 1 (right).
// ------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock, 1) void k_fd_level16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint32_t lev, const uint32_t nlev, const uint64_t nparents, const uint4* __restrict__ s_in,
    const uint4* __restrict__ v_in, const uint8_t* __restrict__ t_in, uint4* __restrict__ s_out,
    uint4* __restrict__ v_out, uint8_t* __restrict__ t_out, uint4* __restrict__ ys, uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint4 cs = cw_s[lev], cv = cw_v[lev], np = cw_np1[0];
  const uint32_t ct = cw_t[lev];
  const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w}, cvw[4] = {cv.x, cv.y, cv.z, cv.w};
  const uint32_t npw[4] = {np.x, np.y, np.z, np.w};
  const bool last = lev + 1 == nlev;
  const uint32_t unit = fd_unit(nparents);
  for (uint64_t base = next_unit_base_n(ctr, ~0ull, unit); base < nparents;
       base = next_unit_base_n(ctr, base, unit)) {
    const uint64_t j = base + (threadIdx.x & 63u);
    const bool live = j < nparents;
    const uint64_t jj = live ? j : nparents - 1;
    const uint4 sv = s_in[jj], vv = v_in[jj];
    const uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w}, v[4] = {vv.x, vv.y, vv.z, vv.w};
    const uint32_t t = t_in[jj];
    uint32_t st[2][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      st[0][k] = s[k];
      st[1][k] = ~s[k];
    }
    aes256_tt<2>(st, rk, lds, lc);  // A, B
    const uint32_t tm = 0u - t;
    uint32_t sl[4], vl[4], sr[4], vr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t msk = (k == 3) ? kMaskLast : 0xFFFFFFFFu;
      sl[k] = ((st[0][k] ^ s[k]) & msk) ^ (tm & csw[k]);
      sr[k] = (s[k] & msk) ^ (tm & csw[k]);
      vl[k] = v[k] ^ ((st[1][k] ^ ~s[k]) & msk) ^ (tm & cvw[k]);
      vr[k] = v[k] ^ ((~s[k]) & msk) ^ (tm & cvw[k]);
    }
    const uint32_t tl = ((st[0][0] ^ s[0]) & 1u) ^ (t & ct & 1u);
    const uint32_t tr = ((st[1][0] ^ ~s[0]) & 1u) ^ (t & (ct >> 1) & 1u);
    if (!live) continue;
    if (last) {  // y = v ^ s ^ t * cw_np1 (lib.rs:192)
      const uint32_t ml = 0u - tl, mr = 0u - tr;
      ys[2 * j] = make_uint4(vl[0] ^ sl[0] ^ (ml & npw[0]), vl[1] ^ sl[1] ^ (ml & npw[1]),
                             vl[2] ^ sl[2] ^ (ml & npw[2]), vl[3] ^ sl[3] ^ (ml & npw[3]));
      ys[2 * j + 1] = make_uint4(vr[0] ^ sr[0] ^ (mr & npw[0]), vr[1] ^ sr[1] ^ (mr & npw[1]),
                                 vr[2] ^ sr[2] ^ (mr & npw[2]), vr[3] ^ sr[3] ^ (mr & npw[3]));
    } else {
      s_out[2 * j] = make_uint4(sl[0], sl[1], sl[2], sl[3]);
      s_out[2 * j + 1] = make_uint4(sr[0], sr[1], sr[2], sr[3]);
      v_out[2 * j] = make_uint4(vl[0], vl[1], vl[2], vl[3]);
      v_out[2 * j + 1] = make_uint4(vr[0], vr[1], vr[2], vr[3]);
      t_out[2 * j] = (uint8_t)tl;
      t_out[2 * j + 1] = (uint8_t)tr;
    }
  }
}

// Pack the prefix level's (s, v, t) arrays into PrefixTable rows.
__global__ void k_prefix_pack(const uint4* __restrict__ s, const uint4* __restrict__ v,
                              const uint8_t* __restrict__ t, const uint64_t n, uint4* __restrict__ sv) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 a = s[i];
    a.w = (a.w & kMaskLast) | ((uint32_t)(t[i] & 1u) << 24);
    sv[2 * i] = a;
    sv[2 * i + 1] = v[i];
  }
}

// One PRG call (A, B) on node (s, v, t) of level `lev` -> both children (lib.rs:176-189
// with x bit 0 / 1), as in k_fd_level16.
// GKB: round keys read per round from the device copy rkg (aes256_tt_gk) instead of SGPRs.
template <bool GKB = false>
__device__ __forceinline__ void fd_children(const uint32_t* lds, uint32_t lc, const RoundKeys& rk,
                                            const uint32_t (&csw)[4], const uint32_t (&cvw)[4], uint32_t ct,
                                            const uint32_t (&s)[4], const uint32_t (&v)[4], uint32_t t,
                                            uint32_t (&sl)[4], uint32_t (&vl)[4], uint32_t& tl, uint32_t (&sr)[4],
                                            uint32_t (&vr)[4], uint32_t& tr, const uint4* __restrict__ rkg = nullptr) {
  uint32_t st[2][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    st[0][k] = s[k];
    st[1][k] = ~s[k];
  }
  if (GKB)
    aes256_tt_gk<2>(st, rkg, lds, lc);  // A, B
  else
    aes256_tt<2>(st, rk, lds, lc);  // A, B
  const uint32_t tm = 0u - t;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t msk = (k == 3) ? kMaskLast : 0xFFFFFFFFu;
    sl[k] = ((st[0][k] ^ s[k]) & msk) ^ (tm & csw[k]);
    sr[k] = (s[k] & msk) ^ (tm & csw[k]);
    vl[k] = v[k] ^ ((st[1][k] ^ ~s[k]) & msk) ^ (tm & cvw[k]);
    vr[k] = v[k] ^ ((~s[k]) & msk) ^ (tm & cvw[k]);
  }
  tl = ((st[0][0] ^ s[0]) & 1u) ^ (t & ct & 1u);
  tr = ((st[1][0] ^ ~s[0]) & 1u) ^ (t & (ct >> 1) & 1u);
}

// Multi-key top trees: for each of K keys, its PrefixTable rows of depth D (2^D rows per
// key, row k * 2^D + the point's top D x bits), so a key's points start on level D instead of
// each walking levels 0..D-1 (C5: 64 points per key share the top of the tree).  Thread
// (key k, node j of level D - 3) walks root -> j (D - 3 PRG calls), then expands j's subtree
// depth-first to its 8 leaves (7 calls): D = 5: 36 PRG calls per key instead of 64 x 5 walks.
// Same node values as the lockstep / stream walks (fd_children: lib.rs:176-189).
// Multi-key stream eval (>= 32 points per key): per-key top trees of kMkPfxLevels levels.
// C5 A/B (same box, M evals/s): 6 levels 400.5-400.8, 5 402.0-402.6, 4 401.2-401.7.
constexpr uint32_t kMkPfxLevels = 5;  // 4..6
constexpr uint32_t kMkPfxRoot = kMkPfxLevels - 3u;     // levels walked from the root per thread
template <bool GKB = true>
__global__ __launch_bounds__(kBlock, 1) void k_mk_prefix16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ s0s,
    const uint32_t party, const uint64_t num_keys, uint4* __restrict__ table, const uint4* __restrict__ rkg,
    uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t k = g >> kMkPfxRoot;
  // the eval's AES block count (dcf_prg_last_eval_blocks) includes the trees: kMkPfxRoot + 7
  // PRG calls of 2 blocks per thread
  const uint64_t live = __ballot(k < num_keys);
  if ((threadIdx.x & 63u) == 0 && live)
    atomicAdd(reinterpret_cast<unsigned long long*>(ctr) + 1,
              2ull * (kMkPfxRoot + 7u) * (unsigned long long)__popcll(live));
  if (k >= num_keys) return;  // after the only barrier (lds_fill_tables)
  const uint32_t j = (uint32_t)g & ((1u << kMkPfxRoot) - 1u);
  auto cw = [&](uint32_t lev, uint32_t (&csw)[4], uint32_t (&cvw)[4]) {
    const uint4 cs = cw_s[(uint64_t)lev * num_keys + k], cv = cw_v[(uint64_t)lev * num_keys + k];
    csw[0] = cs.x; csw[1] = cs.y; csw[2] = cs.z; csw[3] = cs.w;
    cvw[0] = cv.x; cvw[1] = cv.y; cvw[2] = cv.z; cvw[3] = cv.w;
    return (uint32_t)cw_t[(uint64_t)lev * num_keys + k];
  };
  const uint4 sv = s0s[k];
  uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w}, v[4] = {0u, 0u, 0u, 0u}, t = party;
  for (uint32_t lev = 0; lev < kMkPfxRoot; ++lev) {
    uint32_t csw[4], cvw[4];
    const uint32_t ct = cw(lev, csw, cvw);
    uint32_t sl[4], vl[4], sr[4], vr[4], tl, tr;
    fd_children<GKB>(lds, lc, rk, csw, cvw, ct, s, v, t, sl, vl, tl, sr, vr, tr, rkg);
    const bool right = (j >> (kMkPfxRoot - 1u - lev)) & 1u;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      s[w] = right ? sr[w] : sl[w];
      v[w] = right ? vr[w] : vl[w];
    }
    t = right ? tr : tl;
  }
  uint32_t c3s[4], c3v[4], c4s[4], c4v[4], c5s[4], c5v[4];
  constexpr uint32_t A = kMkPfxRoot;
  const uint32_t c3t = cw(A, c3s, c3v), c4t = cw(A + 1, c4s, c4v), c5t = cw(A + 2, c5s, c5v);
  uint4* out = table + 2u * ((k << kMkPfxLevels) + 8u * j);
  auto put = [&](uint32_t leaf, const uint32_t (&ls)[4], const uint32_t (&lv)[4], uint32_t lt) {
    out[2u * leaf] = make_uint4(ls[0], ls[1], ls[2], (ls[3] & kMaskLast) | ((lt & 1u) << 24));
    out[2u * leaf + 1u] = make_uint4(lv[0], lv[1], lv[2], lv[3]);
  };
  uint32_t as[2][4], av[2][4], at[2];  // level 4
  fd_children<GKB>(lds, lc, rk, c3s, c3v, c3t, s, v, t, as[0], av[0], at[0], as[1], av[1], at[1], rkg);
#pragma unroll
  for (uint32_t b4 = 0; b4 < 2; ++b4) {
    uint32_t bs[2][4], bv[2][4], bt[2];  // level 5
    fd_children<GKB>(lds, lc, rk, c4s, c4v, c4t, as[b4], av[b4], at[b4], bs[0], bv[0], bt[0], bs[1], bv[1], bt[1], rkg);
#pragma unroll
    for (uint32_t b5 = 0; b5 < 2; ++b5) {
      uint32_t ls[4], lv[4], lt, rs[4], rv[4], rt;  // level 6
      fd_children<GKB>(lds, lc, rk, c5s, c5v, c5t, bs[b5], bv[b5], bt[b5], ls, lv, lt, rs, rv, rt, rkg);
      put(4u * b4 + 2u * b5, ls, lv, lt);
      put(4u * b4 + 2u * b5 + 1u, rs, rv, rt);
    }
  }
}

// Shared-prefix table (PrefixTable rows) of depth D in ONE launch, Hirose PRG.
// The level-by-level build (k_fd_level16, one launch per level) spends most of its time
// on the narrow upper levels (C2: 23 launches, ~1 ms of a 5 ms step).  Here workgroup w
// (2^S of them) owns the subtree under node w of level S: wave 0 walks the root path to
// it (S PRG calls, bits of w Msb-first), then the workgroup expands its subtree level
// by level with workgroup barriers only (no grid-wide sync), nodes ping-ponging through
// the workgroup's own regions of two buffers (SoA: s[R] | v[R] | t[R], R = 2^(D-1-S)),
// and the last level writes packed 32-B rows of the workgroup's contiguous block of the
// table directly (no pack pass).  Same bytes as the level kernels + k_prefix_pack.
// H > 0: the level-by-level part stops at level D - H (one node or more per thread) and
// each thread expands its nodes' last H levels depth-first (see the tail below).
// Round keys per round from the device copy (aes256_tt_gk: SGPR keys spill here).
constexpr uint32_t kPfxDfsMax = 4;  // H <= 4: a 3-slot stack of 9-word nodes (27 VGPRs; 5 slots spill to scratch)
__global__ __launch_bounds__(kBlock, 1) void k_prefix_build16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ s0,
    const uint32_t party, const uint32_t S, const uint32_t D, const uint32_t H, uint8_t* __restrict__ buf_a,
    uint8_t* __restrict__ buf_b, const uint64_t region_bytes, const uint32_t region_nodes,
    uint4* __restrict__ table, const uint4* __restrict__ rkg) {
  constexpr bool GKB = true;
  __shared__ uint32_t lds[kLdsWords];
  // the narrow levels below the root path: up to 1024 nodes of 32 B (s with t in bit 0 of byte 15 |
  // v); then the depth-first tail's work counter
  __shared__ uint4 nodes[2048];
  lds_fill_tables(lds, tab);
  DCF_CLK(6, 0);  // (diagnostic builds) after the table fill; (6, 1) after the breadth-first levels
  const uint32_t lc = lane_const();
  const uint32_t w = blockIdx.x;
  uint8_t* X = buf_a + (uint64_t)w * region_bytes;
  uint8_t* Y = buf_b + (uint64_t)w * region_bytes;
  const uint32_t R = region_nodes;
  // wave 0: the path root -> node w of level S on 16-lane rows (kernels_lat.h row_root_path);
  // thread 0 keeps it for the first expansion
  uint32_t rs[4] = {0u, 0u, 0u, 0u}, rv[4] = {0u, 0u, 0u, 0u}, rt = 0u;
  RowPrg rp;
  rp.init(rk);
  if (threadIdx.x < 64) row_root_path(lds, rp, cw_s, cw_v, cw_t, s0[0], party, S, w, rs, rv, rt);
  DCF_CLK(7, 0);  // (diagnostic builds) root path done; (7, 1) thread 0's depth-first tail done
  uint32_t L0 = S;  // first level whose parents come from the global buffers (or the root / LDS)
  // Levels whose children fit the LDS node buffer (<= 512 parents), expanded in place: a level
  // costs two workgroup barriers instead of a round trip through the global buffers (C2 A/B r04e:
  // table build 0.571-0.583 vs 0.574-0.599 ms, 4.766-4.772 vs 4.760-4.767 G evals/s).  At least one
  // level through the global buffers follows (it reads this loop's last level from the LDS).
  for (; L0 + 1u < D - H && L0 - S <= 9u; ++L0) {
    const uint32_t np = 1u << (L0 - S), j = threadIdx.x;
    const uint4 cs = cw_s[L0], cv = cw_v[L0];
    const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w}, cvw[4] = {cv.x, cv.y, cv.z, cv.w};
    const uint32_t ct = cw_t[L0];
    // A few nodes (<= 32): 32 lanes per node (RowPrg), node jr = thread / 32, column rp.a — one
    // 16-lane AES chain per level instead of a lone lane's (C2 A/B r04g: breadth-first levels done
    // at 56 vs 69 us, 4.792-4.822 vs 4.772-4.812 G evals/s)
    if (np <= 32u) {
      const uint32_t jr = j >> 5, a = rp.a;
      uint32_t sl, vl, tl = 0u, sr, vr, tr = 0u;
      if (jr < np) {
        uint32_t s, v, t;
        if (L0 == S) {  // wave 0: the root path's node
          s = (a & 2u) ? ((a & 1u) ? rs[3] : rs[2]) : ((a & 1u) ? rs[1] : rs[0]);
          v = (a & 2u) ? ((a & 1u) ? rv[3] : rv[2]) : ((a & 1u) ? rv[1] : rv[0]);
          t = rt;
        } else {
          const uint32_t* nw = reinterpret_cast<const uint32_t*>(nodes + 2 * jr);
          const uint32_t w3 = nw[3];
          s = a == 3u ? (w3 & kMaskLast) : nw[a];
          v = nw[4 + a];
          t = (w3 >> 24) & 1u;
        }
        rp.children(lds, s, v, t, reinterpret_cast<const uint32_t*>(cw_s + L0)[a],
                    reinterpret_cast<const uint32_t*>(cw_v + L0)[a], cw_t[L0], sl, vl, tl, sr, vr, tr);
      }
      __syncthreads();  // every parent read before any child overwrites it
      if (jr < np && (j & 31u) < 4u) {  // row 0, lanes 0..3: column a of both children
        uint32_t* o = reinterpret_cast<uint32_t*>(nodes + 4 * jr);
        o[a] = a == 3u ? ((sl & kMaskLast) | (tl << 24)) : sl;
        o[4 + a] = vl;
        o[8 + a] = a == 3u ? ((sr & kMaskLast) | (tr << 24)) : sr;
        o[12 + a] = vr;
      }
      __syncthreads();
      continue;
    }
    uint32_t sl[4], vl[4], sr[4], vr[4], tl = 0u, tr = 0u;
    if (j < np) {
      uint32_t s[4], v[4], t;
      if (L0 == S) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s[k] = rs[k];
          v[k] = rv[k];
        }
        t = rt;
      } else {
        const uint4 a = nodes[2 * j], b = nodes[2 * j + 1];
        s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w & kMaskLast;
        v[0] = b.x; v[1] = b.y; v[2] = b.z; v[3] = b.w;
        t = (a.w >> 24) & 1u;
      }
      fd_children<GKB>(lds, lc, rk, csw, cvw, ct, s, v, t, sl, vl, tl, sr, vr, tr, rkg);
    }
    __syncthreads();  // every parent read before any child overwrites it
    if (j < np) {
      nodes[4 * j] = make_uint4(sl[0], sl[1], sl[2], (sl[3] & kMaskLast) | (tl << 24));
      nodes[4 * j + 1] = make_uint4(vl[0], vl[1], vl[2], vl[3]);
      nodes[4 * j + 2] = make_uint4(sr[0], sr[1], sr[2], (sr[3] & kMaskLast) | (tr << 24));
      nodes[4 * j + 3] = make_uint4(vr[0], vr[1], vr[2], vr[3]);
    }
    __syncthreads();
  }
  for (uint32_t lev = L0; lev < D - H; ++lev) {
    const uint32_t np = 1u << (lev - S);  // this workgroup's parents at level lev
    const bool last = lev + 1u == D;
    const uint4 cs = cw_s[lev], cv = cw_v[lev];
    const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w}, cvw[4] = {cv.x, cv.y, cv.z, cv.w};
    const uint32_t ct = cw_t[lev];
    const uint4* xs_ = reinterpret_cast<const uint4*>(X);
    const uint4* xv_ = xs_ + R;
    const uint8_t* xt_ = X + (uint64_t)R * 32u;
    uint4* ys_ = reinterpret_cast<uint4*>(Y);
    uint4* yv_ = ys_ + R;
    uint8_t* yt_ = Y + (uint64_t)R * 32u;
    // parents of this thread: j, j + blockDim, ...; the next one's node is loaded before the
    // current one's PRG call so the load latency hides behind the AES
    uint4 nsv = make_uint4(0u, 0u, 0u, 0u), nvv = nsv;
    uint32_t nt = 0u;
    if (threadIdx.x < np) {
      if (lev == S) {  // np = 1: thread 0, the root path's node
        nsv = make_uint4(rs[0], rs[1], rs[2], rs[3]);
        nvv = make_uint4(rv[0], rv[1], rv[2], rv[3]);
        nt = rt;
      } else if (lev == L0) {  // the last LDS level (np <= 1024: one parent per thread)
        const uint4 a = nodes[2 * threadIdx.x], b = nodes[2 * threadIdx.x + 1];
        nsv = make_uint4(a.x, a.y, a.z, a.w & kMaskLast);
        nvv = b;
        nt = (a.w >> 24) & 1u;
      } else {
        nsv = xs_[threadIdx.x];
        nvv = xv_[threadIdx.x];
        nt = xt_[threadIdx.x];
      }
    }
    for (uint32_t j = threadIdx.x; j < np; j += blockDim.x) {
      const uint4 sv = nsv, vv = nvv;
      const uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w}, v[4] = {vv.x, vv.y, vv.z, vv.w};
      const uint32_t t = nt;
      const uint32_t jn = j + blockDim.x;
      if (jn < np) {
        nsv = xs_[jn];
        nvv = xv_[jn];
        nt = xt_[jn];
      }
      uint32_t sl[4], vl[4], sr[4], vr[4], tl, tr;
      fd_children<GKB>(lds, lc, rk, csw, cvw, ct, s, v, t, sl, vl, tl, sr, vr, tr, rkg);
      if (last) {  // PrefixTable rows: s with t in bit 0 of byte 15 (below the root s is masked there)
        uint4* row = table + 2ull * (((uint64_t)w << (D - S)) + 2u * j);
        row[0] = make_uint4(sl[0], sl[1], sl[2], (sl[3] & kMaskLast) | (tl << 24));
        row[1] = make_uint4(vl[0], vl[1], vl[2], vl[3]);
        row[2] = make_uint4(sr[0], sr[1], sr[2], (sr[3] & kMaskLast) | (tr << 24));
        row[3] = make_uint4(vr[0], vr[1], vr[2], vr[3]);
      } else {
        ys_[2 * j] = make_uint4(sl[0], sl[1], sl[2], sl[3]);
        ys_[2 * j + 1] = make_uint4(sr[0], sr[1], sr[2], sr[3]);
        yv_[2 * j] = make_uint4(vl[0], vl[1], vl[2], vl[3]);
        yv_[2 * j + 1] = make_uint4(vr[0], vr[1], vr[2], vr[3]);
        yt_[2 * j] = (uint8_t)tl;
        yt_[2 * j + 1] = (uint8_t)tr;
      }
    }
    __syncthreads();  // the workgroup's children are its next parents
    uint8_t* tmp = X;
    X = Y;
    Y = tmp;
  }
  DCF_CLK(6, 1);
  if (H == 0) return;
  // Depth-first tail: thread j expands node j (j + blockDim, ...) of level B = D - H H
  // levels down in registers — the right child of every expansion above the bottom waits
  // on a stack (one slot per depth), the bottom expansion writes two rows — so the last H
  // levels need neither barriers nor node traffic.  Leaf-parent i (0 .. 2^(H-1) - 1, bits
  // Msb-first = the choices at depths 0 .. H-2) starts from the right child saved at the
  // depth of i's lowest set bit, so every node is expanded exactly once.
  const uint32_t B = D - H, nb = 1u << (B - S), nleafp = 1u << (H - 1u);
  const uint4* xs_ = reinterpret_cast<const uint4*>(X);
  const uint4* xv_ = xs_ + R;
  const uint8_t* xt_ = X + (uint64_t)R * 32u;
  // Nodes are claimed 64 at a time per wave from an LDS counter (the node buffer is free by now):
  // the waves of a workgroup do not progress at one rate (issue goes to the older wave first), and
  // with a static split the oldest wave finished its nodes well before the youngest (in-kernel
  // stamps, C2: wave 0 at 0.39 ms of a ~0.58 ms build, profiles/r04d2_c2_timeline.json).
  uint32_t* dctr = reinterpret_cast<uint32_t*>(nodes);
  if (threadIdx.x == 0) *dctr = 0u;
  __syncthreads();
  for (;;) {  // nb is a multiple of 64 (B - S >= 10)
    uint32_t base = 0u;
    if ((threadIdx.x & 63u) == 0)
      base = __hip_atomic_fetch_add(dctr, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    base = __builtin_amdgcn_readfirstlane(base);
    if (base >= nb) break;
    const uint32_t j = base + (threadIdx.x & 63u);
    uint32_t stk[kPfxDfsMax - 1][9];  // pending right children: s[4] | v[4] | t, by depth
    uint32_t n[9];
    {
      const uint4 sv = xs_[j], vv = xv_[j];
      n[0] = sv.x; n[1] = sv.y; n[2] = sv.z; n[3] = sv.w;
      n[4] = vv.x; n[5] = vv.y; n[6] = vv.z; n[7] = vv.w;
      n[8] = xt_[j];
    }
    uint4* rows = table + 2ull * (((uint64_t)w << (D - S)) + ((uint64_t)j << H));
    for (uint32_t i = 0; i < nleafp; ++i) {
      uint32_t k = 0;
      if (i) {  // resume at the right child saved at depth H - 2 - ctz(i) (wave-uniform)
        const uint32_t d = H - 2u - (uint32_t)__builtin_ctz(i);
#pragma unroll
        for (uint32_t q = 0; q + 1 < kPfxDfsMax; ++q)
          if (q == d)
#pragma unroll
            for (int e = 0; e < 9; ++e) n[e] = stk[q][e];
        k = d + 1u;
      }
      for (;; ++k) {  // expand depth k (level B + k)
        const uint4 cs = cw_s[B + k], cv = cw_v[B + k];
        const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w}, cvw[4] = {cv.x, cv.y, cv.z, cv.w};
        const uint32_t s[4] = {n[0], n[1], n[2], n[3]}, v[4] = {n[4], n[5], n[6], n[7]};
        uint32_t sl[4], vl[4], sr[4], vr[4], tl, tr;
        fd_children<GKB>(lds, lc, rk, csw, cvw, cw_t[B + k], s, v, n[8], sl, vl, tl, sr, vr, tr, rkg);
        if (k + 1u == H) {  // bottom: leaves 2i, 2i + 1 of this node's block of rows
          uint4* row = rows + 4u * i;
          row[0] = make_uint4(sl[0], sl[1], sl[2], (sl[3] & kMaskLast) | (tl << 24));
          row[1] = make_uint4(vl[0], vl[1], vl[2], vl[3]);
          row[2] = make_uint4(sr[0], sr[1], sr[2], (sr[3] & kMaskLast) | (tr << 24));
          row[3] = make_uint4(vr[0], vr[1], vr[2], vr[3]);
          break;
        }
#pragma unroll
        for (uint32_t q = 0; q + 1 < kPfxDfsMax; ++q)
          if (q == k) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              stk[q][e] = sr[e];
              stk[q][4 + e] = vr[e];
            }
            stk[q][8] = tr;
          }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          n[e] = sl[e];
          n[4 + e] = vl[e];
        }
        n[8] = tl;
      }
    }
  }
#ifdef DCF_CLOCK_STAMPS
  __syncthreads();  // (diagnostic builds) stamp when the workgroup's last wave is done
#endif
  DCF_CLK(7, 1);
}

// Last H levels of the full-domain expansion depth-first (as k_prefix_build16's tail): one
// lane per node at level nlev - H expands its subtree with a register stack of pending right
// children (one 9-word slot per depth above the bottom), so the node state in registers grows
// with H, not 2^H as in k_fd_tail16, and H = 4..5 fits.  Leaf-parent i (bits Msb-first = the
// choices at depths 0 .. H-2) resumes from the slot at the depth of i's lowest set bit; its
// expansion writes y for leaves 2i, 2i + 1 of the node's 2^H contiguous outputs.
// ROWS: the nodes of level lev0 are PrefixTable rows (k_prefix_build16's output: s with t in bit 0
// of byte 15, then v) at s_in; v_in / t_in unused.
template <int H, bool ROWS = false>
__global__ __launch_bounds__(kBlock, 1) void k_fd_dfs16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint32_t lev0, const uint64_t nnodes, const uint4* __restrict__ s_in, const uint4* __restrict__ v_in,
    const uint8_t* __restrict__ t_in, uint4* __restrict__ ys, uint32_t* __restrict__ ctr) {
  static_assert(H >= 2 && H <= 6, "depth-first tail of 2..6 levels");
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint4 np = cw_np1[0];
  const uint32_t unit = fd_unit(nnodes);
  for (uint64_t base = next_unit_base_n(ctr, ~0ull, unit); base < nnodes;
       base = next_unit_base_n(ctr, base, unit)) {
    const uint64_t j = base + (threadIdx.x & 63u);
    const bool live = j < nnodes;
    const uint64_t jj = live ? j : nnodes - 1;
    uint32_t stk[H - 1][9];  // pending right children: s[4] | v[4] | t, by depth
    uint32_t n[9];
    if (ROWS) {
      const uint4 sv = s_in[2 * jj], vv = s_in[2 * jj + 1];
      n[0] = sv.x; n[1] = sv.y; n[2] = sv.z; n[3] = sv.w & kMaskLast;
      n[4] = vv.x; n[5] = vv.y; n[6] = vv.z; n[7] = vv.w;
      n[8] = (sv.w >> 24) & 1u;
    } else {
      const uint4 sv = s_in[jj], vv = v_in[jj];
      n[0] = sv.x; n[1] = sv.y; n[2] = sv.z; n[3] = sv.w;
      n[4] = vv.x; n[5] = vv.y; n[6] = vv.z; n[7] = vv.w;
      n[8] = t_in[jj];
    }
    uint4* y = ys + (jj << H);
    for (uint32_t i = 0; i < (1u << (H - 1)); ++i) {
      uint32_t k = 0;
      if (i) {  // resume at the right child saved at depth H - 2 - ctz(i) (wave-uniform)
        const uint32_t d = (uint32_t)(H - 2) - (uint32_t)__builtin_ctz(i);
#pragma unroll
        for (uint32_t q = 0; q + 1 < (uint32_t)H; ++q)
          if (q == d)
#pragma unroll
            for (int e = 0; e < 9; ++e) n[e] = stk[q][e];
        k = d + 1u;
      }
      for (;; ++k) {  // expand depth k (level lev0 + k)
        const uint4 cs = cw_s[lev0 + k], cv = cw_v[lev0 + k];
        const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w}, cvw[4] = {cv.x, cv.y, cv.z, cv.w};
        const uint32_t s[4] = {n[0], n[1], n[2], n[3]}, v[4] = {n[4], n[5], n[6], n[7]};
        uint32_t sl[4], vl[4], sr[4], vr[4], tl, tr;
        fd_children(lds, lc, rk, csw, cvw, cw_t[lev0 + k], s, v, n[8], sl, vl, tl, sr, vr, tr);
        if (k + 1u == (uint32_t)H) {  // leaves: y = v ^ s ^ t * cw_np1 (lib.rs:192)
          if (live) {
            const uint32_t ml = 0u - tl, mr = 0u - tr;
            y[2 * i] = make_uint4(vl[0] ^ sl[0] ^ (ml & np.x), vl[1] ^ sl[1] ^ (ml & np.y),
                                  vl[2] ^ sl[2] ^ (ml & np.z), vl[3] ^ sl[3] ^ (ml & np.w));
            y[2 * i + 1] = make_uint4(vr[0] ^ sr[0] ^ (mr & np.x), vr[1] ^ sr[1] ^ (mr & np.y),
                                      vr[2] ^ sr[2] ^ (mr & np.z), vr[3] ^ sr[3] ^ (mr & np.w));
          }
          break;
        }
#pragma unroll
        for (uint32_t q = 0; q + 1 < (uint32_t)H; ++q)
          if (q == k) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              stk[q][e] = sr[e];
              stk[q][4 + e] = vr[e];
            }
            stk[q][8] = tr;
          }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          n[e] = sl[e];
          n[4 + e] = vl[e];
        }
        n[8] = tl;
      }
    }
  }
}

// Root node for full-domain eval: s = s0 (k.s0s[0]), v = 0, t = party.
__global__ void k_fd_root16(const uint4* __restrict__ s0, const uint32_t party, uint4* __restrict__ s,
                            uint4* __restrict__ v, uint8_t* __restrict__ t) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    s[0] = s0[0];
    v[0] = make_uint4(0u, 0u, 0u, 0u);
    t[0] = (uint8_t)party;
  }
}

// All 2^n points of an n-bit domain as big-endian N-byte strings (LAMBDA >= 32 full domain).
__global__ void k_domain_points(const uint32_t nbytes, const uint64_t count, uint8_t* __restrict__ xs) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (uint64_t)gridDim.x * blockDim.x)
    for (uint32_t b = 0; b < nbytes; ++b) {
      const uint32_t sh = 8u * (nbytes - 1u - b);
      xs[i * nbytes + b] = sh < 64 ? (uint8_t)(i >> sh) : 0u;
    }
}

}  // namespace
