// kernels_bs.h — bitsliced AES-256 on the VALU (LAMBDA = 16).
// Included by dcf_hip.hip only.
//
// Layout: a quad of lanes (4q..4q+3) evaluates 32 points, one per bit.  Lane
// c = lane & 3 holds column c of the 16-byte AES state for all 32 points as 32
// registers st[8r + k] = bit k of the row-r byte (bit j of the register =
// point j).  SubBytes is the 115-gate Boyar-Peralta circuit on each row
// (bs_sbox.h); MixColumns and AddRoundKey are lane-local; ShiftRows moves
// rows 1..3 across the quad with DPP quad_perm (row r of column c comes from
// column c + r).  No LDS: this path runs on the VALU, which the T-table path
// (LDS-bound) leaves ~60 % idle — k_eval16_hybrid runs both side by side.
#pragma once

#include "aes_lds.h"
#include "bs_sbox.h"

namespace {

constexpr uint32_t kBsPoints = 32;   // points per quad
constexpr uint32_t kWavePoints = 512;  // points per wave (16 quads)

template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
  // mov_dpp (no `old` operand): quad_perm reads a valid lane for every lane, so no
  // v_mov of a fallback value is needed before each DPP move.
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

// 32 x 32 bit transpose (LSB convention): afterwards a[j] bit i = old a[i] bit j.
__device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
  uint32_t m = 0x0000FFFFu;
#pragma unroll
  for (int j = 16; j != 0; j >>= 1, m ^= (m << j)) {
#pragma unroll
    for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
      const uint32_t t = ((a[k] >> j) ^ a[k + j]) & m;
      a[k + j] ^= t;
      a[k] ^= t << j;
    }
  }
}

__device__ __forceinline__ void bs_subbytes(uint32_t (&st)[32]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint32_t row[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) row[k] = st[8 * r + k];
    bs_sbox(row);
#pragma unroll
    for (int k = 0; k < 8; ++k) st[8 * r + k] = row[k];
  }
}

__device__ __forceinline__ void bs_shiftrows(uint32_t (&st)[32]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    st[8 + k] = qperm<kQpRot1>(st[8 + k]);
    st[16 + k] = qperm<kQpRot2>(st[16 + k]);
    st[24 + k] = qperm<kQpRot3>(st[24 + k]);
  }
}

#define DCF_B3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))
// bitop3 immediates (imm = f(src0 = 0xF0, src1 = 0xCC, src2 = 0xAA)):
constexpr uint32_t kXor3 = 0x96;  // a ^ b ^ c

// Round-key masks of cipher 0 for the bitsliced engine: uint4 km[32 r + 8 c + q]
// holds, as four all-ones/zero words, bits 4q..4q+3 of column c of round key r
// (rounds 0..14; 7.5 KiB, built on the host from the key schedule, L1-resident).
__device__ __forceinline__ void bs_ark_tab(uint32_t (&st)[32], const uint4* __restrict__ km, bool inv) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 k = km[q];
    const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) st[4 * q + e] ^= inv ? ~kk[e] : kk[e];
  }
}

// MixColumns + AddRoundKey on this lane's column:
//   out_r = xtime(a_r ^ a_{r+1}) ^ (T ^ a_r ^ key_r),  T = a0 ^ a1 ^ a2 ^ a3.
__device__ __forceinline__ void bs_mixcolumns_ark(uint32_t (&st)[32], const uint4* __restrict__ km) {
  uint32_t T[8], a0[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a0[k] = st[k];
    T[k] = DCF_B3(st[k], st[8 + k], st[16 + k], kXor3) ^ st[24 + k];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint4 k0 = km[2 * r], k1 = km[2 * r + 1];
    const uint32_t key[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
    uint32_t d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = st[8 * r + k] ^ ((r == 3) ? a0[k] : st[8 * (r + 1) + k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t e = DCF_B3(T[k], st[8 * r + k], key[k], kXor3);
      if (k == 0)
        st[8 * r + k] = d[7] ^ e;
      else if (k == 1 || k == 3 || k == 4)
        st[8 * r + k] = DCF_B3(d[k - 1], d[7], e, kXor3);
      else
        st[8 * r + k] = d[k - 1] ^ e;
    }
  }
}

// AES-256 encryption of 32 blocks (quad-sliced).  `inv_in`: encrypt ~st instead.
// km: this lane's column of the round-key masks (km + 8 c; round r at + 32 r).
__device__ __forceinline__ void bs_aes256(uint32_t (&st)[32], const uint4* __restrict__ km, bool inv_in) {
  bs_ark_tab(st, km, inv_in);
#pragma unroll 1
  for (int r = 1; r < 14; ++r) {
    bs_subbytes(st);
    bs_shiftrows(st);
    bs_mixcolumns_ark(st, km + 32 * r);
  }
  bs_subbytes(st);
  bs_shiftrows(st);
  bs_ark_tab(st, km + 32 * 14, false);
}

#undef DCF_B3

// Broadcast a uniform 16-byte value's column c into bitsliced registers.
__device__ __forceinline__ void bs_splat(uint32_t (&st)[32], uint32_t w) {
#pragma unroll
  for (int i = 0; i < 32; ++i) st[i] = (uint32_t)__builtin_amdgcn_sbfe((int)w, i, 1);
}

__device__ __forceinline__ uint32_t sel4(uint4 v, uint32_t c) {
  return (c & 2u) ? ((c & 1u) ? v.w : v.z) : ((c & 1u) ? v.y : v.x);
}

// One wave's batch of 512 points (32 per quad), party `party`, single key.
// xl: this wave's 2 KiB of LDS holding 32 levels of transposed x, [level][quad].
template <bool XALIGNED>
__device__ __forceinline__ void bs_eval_batch(const uint4* __restrict__ km, const uint4* __restrict__ cw_s,
                                              const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                              const uint4 np1, const uint4 s0v, const uint32_t party,
                                              const uint8_t* __restrict__ xs, const uint32_t nbytes,
                                              const uint64_t m, const uint64_t p_base, uint32_t* xl,
                                              uint4* __restrict__ ys) {
  const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, quad = lane >> 2;
  const uint64_t p0 = p_base + (uint64_t)quad * kBsPoints;
  const uint32_t nlev = 8u * nbytes, nchunk = (nbytes + 3u) >> 2;
  const uint4* __restrict__ kmc = km + 8 * c;
  uint32_t s[32], v[32];
  bs_splat(s, sel4(s0v, c));
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = 0u;
  uint32_t T = party ? 0xFFFFFFFFu : 0u;                // t of the 32 points
  const uint32_t mlast = (c == 3u) ? 0u : 0xFFFFFFFFu;  // register 24 of column 3 = bit 0 of byte 15
  uint32_t lev = 0;
  for (uint32_t cc = 0; cc < nchunk; ++cc) {
    // Lane cc of each quad transposes the quad's 32 x words for levels [32cc, 32cc+32) into LDS.
    __builtin_amdgcn_wave_barrier();
    if (c == cc) {
      uint32_t w[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) {  // rows past m are clamped (their outputs are not stored)
        const uint64_t p = min(p0 + j, m - 1);
        if (XALIGNED)
          w[j] = bswap32(*reinterpret_cast<const uint32_t*>(xs + p * nbytes + 4 * cc));
        else
          w[j] = load_bits32(xs + p * nbytes, cc, nbytes);
      }
      transpose32(w);  // w[i] bit j = bit i of point j's Msb0-ordered word = level 32cc + 31 - i
#pragma unroll
      for (int i = 0; i < 32; ++i) xl[(31u - i) * 16u + quad] = w[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t lend = min(32u, nlev - 32u * cc);
    for (uint32_t b = 0; b < lend; ++b, ++lev) {
      const uint32_t X = xl[b * 16u + quad];  // bit j: x bit of point j (1 = right)
      const uint4 cs = cw_s[lev], cv = cw_v[lev];
      const uint32_t ct = cw_t[lev];
      const uint32_t csw = sel4(cs, c), cvw = sel4(cv, c);
      uint32_t st[32];
      // B = AES(~s): v ^= ((~s) ^ (B & ~X)) & M ^ (T & cw.v)   (lib.rs:182/186)
#pragma unroll
      for (int i = 0; i < 32; ++i) st[i] = s[i];
      bs_aes256(st, kmc, true);
      const uint32_t tR = qperm<kQpBcast0>(st[0] ^ ~s[0]);  // lsb(B ^ ~s)[0] of each point
      uint32_t cvo = cvw;
      asm volatile("" : "+v"(cvo));  // keep the 32 CW masks from being materialised before the AES
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        uint32_t hv = (~s[i]) ^ (st[i] & ~X);
        if (i == 24) hv &= mlast;
        v[i] ^= hv ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)cvo, i, 1));
      }
      // A = AES(s): s' = (s ^ (A & ~X)) & M ^ (T & cw.s)   (lib.rs:177-178, 183/187)
#pragma unroll
      for (int i = 0; i < 32; ++i) st[i] = s[i];
      bs_aes256(st, kmc, false);
      const uint32_t tL = qperm<kQpBcast0>(st[0] ^ s[0]);
      uint32_t cso = csw;
      asm volatile("" : "+v"(cso));
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        uint32_t hs = s[i] ^ (st[i] & ~X);
        if (i == 24) hs &= mlast;
        s[i] = hs ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)cso, i, 1));
      }
      // t' = side t ^ (t & side cw.t)   (lib.rs:179-180)
      const uint32_t ctl = 0u - (ct & 1u), ctr = 0u - ((ct >> 1) & 1u);
      T = ((X & tR) | (~X & tL)) ^ (T & ((X & ctr) | (~X & ctl)));
    }
  }
  // y = v ^ s ^ t * cw_np1   (lib.rs:192), then back to one dword per point
  const uint32_t npw = sel4(np1, c);
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] ^= s[i] ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)npw, i, 1));
  transpose32(v);  // v[j] = column-c dword of point j
  uint32_t* y32 = reinterpret_cast<uint32_t*>(ys);
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const uint64_t p = p0 + j;
    if (p < m) y32[p * 4 + c] = v[j];
  }
}

// Same batch with the 32-register v accumulator of each lane kept in a per-wave
// scratch slab ([v q0..q7][64 lanes] uint4, coalesced 1 KiB accesses) instead
// of registers, so the lane fits in 128 VGPRs and 4 waves share each SIMD to
// hide the S-box's dependency chains.  v is read and written once per level
// (256 B per lane against ~12.7K VALU ops).
template <bool XALIGNED>
__device__ __forceinline__ void bs_eval_batch_mem(const uint4* __restrict__ km, const uint4* __restrict__ cw_s,
                                                  const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                                  const uint4 np1, const uint4 s0v, const uint32_t party,
                                                  const uint8_t* __restrict__ xs, const uint32_t nbytes,
                                                  const uint64_t m, const uint64_t p_base, uint32_t* xl,
                                                  uint4* __restrict__ slab, uint4* __restrict__ ys) {
  const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, quad = lane >> 2;
  const uint64_t p0 = p_base + (uint64_t)quad * kBsPoints;
  const uint32_t nlev = 8u * nbytes, nchunk = (nbytes + 3u) >> 2;
  const uint4* __restrict__ kmc = km + 8 * c;
  uint4* __restrict__ vp = slab + lane;  // v quad q at vp[64 q]
  uint32_t s[32];
  bs_splat(s, sel4(s0v, c));
#pragma unroll
  for (int q = 0; q < 8; ++q) vp[64 * q] = make_uint4(0u, 0u, 0u, 0u);
  uint32_t T = party ? 0xFFFFFFFFu : 0u;
  const uint32_t mlast = (c == 3u) ? 0u : 0xFFFFFFFFu;
  uint32_t lev = 0;
  for (uint32_t cc = 0; cc < nchunk; ++cc) {
    __builtin_amdgcn_wave_barrier();
    if (c == cc) {
      uint32_t w[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint64_t p = min(p0 + j, m - 1);
        if (XALIGNED)
          w[j] = bswap32(*reinterpret_cast<const uint32_t*>(xs + p * nbytes + 4 * cc));
        else
          w[j] = load_bits32(xs + p * nbytes, cc, nbytes);
      }
      transpose32(w);
#pragma unroll
      for (int i = 0; i < 32; ++i) xl[(31u - i) * 16u + quad] = w[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t lend = min(32u, nlev - 32u * cc);
    for (uint32_t b = 0; b < lend; ++b, ++lev) {
      const uint32_t X = xl[b * 16u + quad];
      const uint4 cs = cw_s[lev], cv = cw_v[lev];
      const uint32_t ct = cw_t[lev];
      uint32_t csw = sel4(cs, c), cvw = sel4(cv, c);
      uint32_t st[32];
      // B = AES(~s); v ^= ((~s) ^ (B & ~X)) & M ^ (T & cw.v)   (v lives in the slab)
#pragma unroll
      for (int i = 0; i < 32; ++i) st[i] = s[i];
      bs_aes256(st, kmc, true);
      asm volatile("" : "+v"(cvw));
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint4 vv = vp[64 * q];
        uint32_t va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * q + e;
          uint32_t hv = (~s[i]) ^ (st[i] & ~X);
          if (i == 24) hv &= mlast;
          va[e] ^= hv ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)cvw, i, 1));
        }
        vp[64 * q] = make_uint4(va[0], va[1], va[2], va[3]);
      }
      const uint32_t tR = qperm<kQpBcast0>(st[0] ^ ~s[0]);
      // A = AES(s); s' = (s ^ (A & ~X)) & M ^ (T & cw.s)
#pragma unroll
      for (int i = 0; i < 32; ++i) st[i] = s[i];
      bs_aes256(st, kmc, false);
      const uint32_t tL = qperm<kQpBcast0>(st[0] ^ s[0]);
      asm volatile("" : "+v"(csw));
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        uint32_t hs = s[i] ^ (st[i] & ~X);
        if (i == 24) hs &= mlast;
        s[i] = hs ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)csw, i, 1));
      }
      const uint32_t ctl = 0u - (ct & 1u), ctr = 0u - ((ct >> 1) & 1u);
      T = ((X & tR) | (~X & tL)) ^ (T & ((X & ctr) | (~X & ctl)));
    }
  }
  const uint32_t npw = sel4(np1, c);
  uint32_t y[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 vv = vp[64 * q];
    const uint32_t va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * q + e;
      y[i] = va[e] ^ s[i] ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)npw, i, 1));
    }
  }
  transpose32(y);
  uint32_t* y32 = reinterpret_cast<uint32_t*>(ys);
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const uint64_t p = p0 + j;
    if (p < m) y32[p * 4 + c] = y[j];
  }
}

// Stand-alone bitsliced eval (single key, N <= 16), one wave per 512-point batch.
template <bool XALIGNED>
__global__ __launch_bounds__(256, 3) void k_eval16_bs(const uint4* __restrict__ km, const uint4* __restrict__ cw_s,
                                                   const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                                   const uint4* __restrict__ cw_np1, const uint4* __restrict__ s0,
                                                   const uint32_t party, const uint8_t* __restrict__ xs,
                                                   const uint32_t nbytes, const uint64_t m, uint4* __restrict__ ys) {
  __shared__ uint32_t xl_all[4][32 * 16];
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t gwave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint4 np1 = cw_np1[0], s0v = s0[0];
  for (uint64_t b = gwave; b * kWavePoints < m; b += nwaves)
    bs_eval_batch<XALIGNED>(km, cw_s, cw_v, cw_t, np1, s0v, party, xs, nbytes, m, b * kWavePoints, xl_all[wave],
                            ys);
}

}  // namespace

namespace {

// ------------------------------------------------------------------------
// k_eval16_hybrid: both AES engines in one launch, one 12-wave workgroup per
// CU.  Waves [0, n_tt) run the LDS T-table engine (LDS-bound), waves
// [n_tt, 12) the bitsliced engine (VALU-bound), so the CU's LDS and VALU are
// busy at the same time.  Work is dequeued in 512-point units from one global
// counter (reset by the host before each launch): each engine takes units at
// its own pace, so the split adapts to their relative speed.
// ------------------------------------------------------------------------
constexpr int kHybridWaves = 12;

__device__ __forceinline__ uint32_t dequeue_unit(uint32_t* ctr) {
  uint32_t u = 0;
  if ((threadIdx.x & 63u) == 0) u = atomicAdd(ctr, 1u);
  return __builtin_amdgcn_readfirstlane(u);
}

// MEM = false: s/v in registers (168 VGPRs, 12 waves per workgroup).
// MEM = true:  s/v in a per-wave scratch slab (<= 128 VGPRs, 16 waves), n_tt >= 1.
constexpr uint32_t kSlabUint4 = 8 * 64;  // per-wave slab: 8 KiB (v)

template <bool XALIGNED, bool MEM>
__global__ __launch_bounds__((MEM ? 16 : kHybridWaves) * 64) void k_eval16_hybrid(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t m, const uint32_t n_tt, uint32_t* __restrict__ ctr, uint4* __restrict__ slabs,
    const uint4* __restrict__ km, uint4* __restrict__ ys) {
  constexpr int kWaves = MEM ? 16 : kHybridWaves;
  constexpr int kXlSlots = MEM ? 15 : kHybridWaves;  // LDS budget: 128 KiB tables + 2 KiB per bitsliced wave
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint32_t xl_all[kXlSlots][32 * 16];
  lds_fill_tables(lds, tab);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t nunits = (m + kWavePoints - 1) / kWavePoints;
  const uint4 np1 = cw_np1[0], s0v = s0[0];
  if (wave < n_tt) {
    const uint32_t lc = lane_const();
    for (uint32_t u = dequeue_unit(ctr); u < nunits; u = dequeue_unit(ctr)) {
      const uint64_t base = (uint64_t)u * kWavePoints;
      for (uint32_t it = 0; it < kWavePoints / 64 && base + 64u * it < m; ++it) {
        const uint64_t g = base + 64u * it + lane;
        const uint64_t gg = g < m ? g : m - 1;
        const uint4 y = tt_eval_one(lds, lc, rk, cw_s, cw_v, cw_t, np1, s0v, party, xs + gg * nbytes, nbytes, 1, 0);
        if (g < m) ys[g] = y;
      }
    }
  } else {
    uint32_t* xl = xl_all[MEM ? wave - n_tt : wave];
    uint4* slab = slabs + ((uint64_t)blockIdx.x * kWaves + wave) * kSlabUint4;
    for (uint32_t u = dequeue_unit(ctr); u < nunits; u = dequeue_unit(ctr)) {
      if (MEM)
        bs_eval_batch_mem<XALIGNED>(km, cw_s, cw_v, cw_t, np1, s0v, party, xs, nbytes, m,
                                    (uint64_t)u * kWavePoints, xl, slab, ys);
      else
        bs_eval_batch<XALIGNED>(km, cw_s, cw_v, cw_t, np1, s0v, party, xs, nbytes, m, (uint64_t)u * kWavePoints,
                                xl, ys);
    }
  }
}

}  // namespace
