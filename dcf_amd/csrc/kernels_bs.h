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
// The key-mask loads sit behind zb, a zero an empty asm "redefines" from the state, so the
// compiler can neither hoist the first and last rounds' 64 masks out of the caller's level loop
// nor share them between a level's two encryptions (that alone spilled ~120 VGPRs).
__device__ __forceinline__ void bs_aes256(uint32_t (&st)[32], const uint4* __restrict__ km, bool inv_in) {
  uint32_t zb = 0u;
  asm volatile("" : "+v"(zb) : "v"(st[0]));
  bs_ark_tab(st, km + zb, inv_in);
#pragma unroll 1
  for (int r = 1; r < 14; ++r) {
    bs_subbytes(st);
    bs_shiftrows(st);
    asm volatile("" : "+v"(zb) : "v"(st[0]));
    bs_mixcolumns_ark(st, km + 32 * r + zb);
  }
  bs_subbytes(st);
  bs_shiftrows(st);
  asm volatile("" : "+v"(zb) : "v"(st[0]));
  bs_ark_tab(st, km + 32 * 14 + zb, false);
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

// ---- the bitsliced walk: s and v in the wave's slab, the AES state in registers ----
// A lane's 32 words of s and of v (this column, 32 points) live in the wave's scratch slab:
// v quad q at slab[64 q + lane], s quad q at slab[512 + 64 q + lane] (each access a coalesced
// 1 KiB, L1/L2-resident), and only the AES state is in registers.  Kept in registers beside the
// state (96 VGPRs for the AES alone) they pushed the engine to 336 spilled VGPRs (1.1 KiB of
// scratch per lane, r03 resource-usage build): the slab round trips cost ~10 KiB of traffic per
// wave and level against ~13 K VALU instructions.
constexpr uint32_t kSlabUint4 = 16 * 64;  // per-wave slab: 16 KiB (v, then s)

// (each helper "redefines" its slab pointer, so the compiler forms the 8 quad addresses where they
// are used instead of hoisting them out of the caller's loops: loop-invariant addresses of the
// wave's slab were ~32 live VGPRs, and spilled)
__device__ __forceinline__ void bs_load32(uint32_t (&a)[32], const uint4* __restrict__ p) {
  asm volatile("" : "+v"(p));
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 x = p[64 * q];
    a[4 * q] = x.x; a[4 * q + 1] = x.y; a[4 * q + 2] = x.z; a[4 * q + 3] = x.w;
  }
}
__device__ __forceinline__ void bs_store32(uint4* __restrict__ p, const uint32_t (&a)[32]) {
  asm volatile("" : "+v"(p));
#pragma unroll
  for (int q = 0; q < 8; ++q) p[64 * q] = make_uint4(a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]);
}

// One level of the GGM walk (lib.rs:174-189 over prg.rs:42-73) for the quad's 32 points: xw ->
// the quad's x word of this level in LDS (bit j = x bit of point j, 1 = right), T bit j = its t;
// cs / cv / ct: this level's correction word (uniform).  s and v in the slab (vp, sp), updated in
// place.  Everything but T and the AES state is read after the encryption that first needs it
// (the CW column select, the x word), so the AES runs with ~100 VGPRs live.
__device__ __forceinline__ void bs_level(const uint4* __restrict__ kmc, uint4* __restrict__ vp,
                                         uint4* __restrict__ sp, const uint32_t* xw, uint32_t& T, const uint4 cs,
                                         const uint4 cv, const uint32_t ct) {
  // the slab pointers are "redefined" here, so the 16 quad addresses are formed inside the level
  // instead of being hoisted out of the caller's loops (32 live VGPRs of addresses)
  asm volatile("" : "+v"(vp), "+v"(sp));
  const uint32_t c = threadIdx.x & 3u;
  uint32_t st[32];
  // B = AES(~s): v ^= ((~s) ^ (B & ~X)) & M ^ (T & cw.v)   (lib.rs:182/186)
  bs_load32(st, sp);
  bs_aes256(st, kmc, true);
  uint32_t cvw = sel4(cv, c), X = *xw;
  asm volatile("" : "+v"(cvw), "+v"(X) : "v"(st[0]));  // selected after the AES, masks made per use
  const uint32_t mlast = (c == 3u) ? 0u : 0xFFFFFFFFu;  // word 24 of column 3 = bit 0 of byte 15
  uint32_t tR = 0u;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 sq = sp[64 * q];
    const uint4 vq = vp[64 * q];
    const uint32_t sw[4] = {sq.x, sq.y, sq.z, sq.w};
    uint32_t vw[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * q + e;
      uint32_t hv = (~sw[e]) ^ (st[i] & ~X);
      if (i == 24) hv &= mlast;
      vw[e] ^= hv ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)cvw, i, 1));
    }
    if (q == 0) tR = qperm<kQpBcast0>(st[0] ^ ~sw[0]);  // lsb(B ^ ~s)[0] of each point
    vp[64 * q] = make_uint4(vw[0], vw[1], vw[2], vw[3]);
  }
  // A = AES(s): s' = (s ^ (A & ~X)) & M ^ (T & cw.s)   (lib.rs:177-178, 183/187)
  bs_load32(st, sp);
  bs_aes256(st, kmc, false);
  uint32_t csw = sel4(cs, c), X2 = *xw;
  asm volatile("" : "+v"(csw), "+v"(X2) : "v"(st[0]));
  const uint32_t mlast2 = (c == 3u) ? 0u : 0xFFFFFFFFu;
  uint32_t tL = 0u;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 sq = sp[64 * q];
    const uint32_t sw[4] = {sq.x, sq.y, sq.z, sq.w};
    uint32_t nw[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * q + e;
      uint32_t hs = sw[e] ^ (st[i] & ~X2);
      if (i == 24) hs &= mlast2;
      nw[e] = hs ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)csw, i, 1));
    }
    if (q == 0) tL = qperm<kQpBcast0>(st[0] ^ sw[0]);  // lsb(A ^ s)[0]
    sp[64 * q] = make_uint4(nw[0], nw[1], nw[2], nw[3]);
  }
  // t' = side t ^ (t & side cw.t)   (lib.rs:179-180)
  const uint32_t ctl = 0u - (ct & 1u), ctr = 0u - ((ct >> 1) & 1u);
  T = ((X2 & tR) | (~X2 & tL)) ^ (T & ((X2 & ctr) | (~X2 & ctl)));
}

// The quad's x bits for levels [32 cc, 32 cc + 32) into the wave's 2 KiB of LDS: byte c of word
// [level][quad] holds points 8c .. 8c + 7 of the quad (bit j = point 8c + j), written by lane c
// from its 8 points' x words (rows past m are clamped; their outputs are not stored).  No 32 x 32
// transpose: 8 words in registers, not 32 (a transposing lane pushed the engine into spills).
template <bool XALIGNED>
__device__ __forceinline__ void bs_stage_x(uint32_t* xl, const uint8_t* __restrict__ xs, uint32_t nbytes,
                                           uint64_t m, uint64_t p0, uint32_t cc) {
  const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, quad = lane >> 2;
  __builtin_amdgcn_wave_barrier();
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t p = min(p0 + 8u * c + j, m - 1);
    if (XALIGNED)
      w[j] = bswap32(*reinterpret_cast<const uint32_t*>(xs + p * nbytes + 4 * cc));
    else
      w[j] = load_bits32(xs + p * nbytes, cc, nbytes);  // Msb0 (lib.rs:181)
  }
  uint8_t* xb = reinterpret_cast<uint8_t*>(xl) + 4u * quad + c;
#pragma unroll
  for (int b = 0; b < 32; ++b) {
    uint32_t byte = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) byte |= ((w[j] >> (31 - b)) & 1u) << j;
    xb[64 * b] = (uint8_t)byte;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// y = v ^ s ^ t * cw_np1 (lib.rs:192) from the slab, back to one dword per point, stored.
__device__ __forceinline__ void bs_finish(const uint4* __restrict__ vp, const uint4* __restrict__ sp, uint32_t T,
                                          uint32_t npw, uint64_t m, uint64_t p0, uint4* __restrict__ ys) {
  const uint32_t c = threadIdx.x & 3u;
  asm volatile("" : "+v"(vp), "+v"(sp));
  uint32_t y[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 vq = vp[64 * q], sq = sp[64 * q];
    const uint32_t va[4] = {vq.x ^ sq.x, vq.y ^ sq.y, vq.z ^ sq.z, vq.w ^ sq.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) y[4 * q + e] = va[e] ^ (T & (uint32_t)__builtin_amdgcn_sbfe((int)npw, 4 * q + e, 1));
  }
  transpose32(y);  // y[j] = column-c dword of point j
  uint32_t* y32 = reinterpret_cast<uint32_t*>(ys);
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const uint64_t p = p0 + j;
    if (p < m) y32[p * 4 + c] = y[j];
  }
}

// One wave's batch of 512 points (32 per quad), party `party`, single key, from the root.
// xl: this wave's 2 KiB of LDS; slab: its kSlabUint4 uint4 of scratch.
template <bool XALIGNED>
__device__ __forceinline__ void bs_eval_batch(const uint4* __restrict__ km, const uint4* __restrict__ cw_s,
                                              const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                              const uint4 np1, const uint4 s0v, const uint32_t party,
                                              const uint8_t* __restrict__ xs, const uint32_t nbytes,
                                              const uint64_t m, const uint64_t p_base, uint32_t* xl,
                                              uint4* __restrict__ slab, uint4* __restrict__ ys) {
  const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, quad = lane >> 2;
  const uint64_t p0 = p_base + (uint64_t)quad * kBsPoints;
  const uint32_t nlev = 8u * nbytes, nchunk = (nbytes + 3u) >> 2;
  const uint4* __restrict__ kmc = km + 8 * c;
  uint4* __restrict__ vp = slab + lane;
  uint4* __restrict__ sp = slab + 512 + lane;
  {
    uint32_t s[32], w0 = sel4(s0v, c);
    asm volatile("" : "+v"(w0));  // not hoisted out of the batch loop (32 live masks)
    bs_splat(s, w0);  // k.s0s[0] (lib.rs:168)
    bs_store32(sp, s);
    for (int i = 0; i < 32; ++i) s[i] = 0u;
    bs_store32(vp, s);
  }
  uint32_t T = party ? 0xFFFFFFFFu : 0u;  // t of the 32 points (lib.rs:169)
  uint32_t lev = 0;
  for (uint32_t cc = 0; cc < nchunk; ++cc) {
    bs_stage_x<XALIGNED>(xl, xs, nbytes, m, p0, cc);
    const uint32_t lend = min(32u, nlev - 32u * cc);
    for (uint32_t b = 0; b < lend; ++b, ++lev)
      bs_level(kmc, vp, sp, xl + b * 16u + quad, T, cw_s[lev], cw_v[lev], cw_t[lev]);
  }
  bs_finish(vp, sp, T, sel4(np1, c), m, p0, ys);
}

// Stand-alone bitsliced eval (single key, N <= 16), one wave per 512-point batch; 4 waves per
// SIMD (<= 128 VGPRs), grid <= 4 workgroups per CU (one slab per resident wave).
template <bool XALIGNED>
__global__ __launch_bounds__(256, 4) void k_eval16_bs(const uint4* __restrict__ km, const uint4* __restrict__ cw_s,
                                                   const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                                   const uint4* __restrict__ cw_np1, const uint4* __restrict__ s0,
                                                   const uint32_t party, const uint8_t* __restrict__ xs,
                                                   const uint32_t nbytes, const uint64_t m, uint4* __restrict__ slabs,
                                                   uint4* __restrict__ ys) {
  __shared__ uint32_t xl_all[4][32 * 16];
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t gwave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint4 np1 = cw_np1[0], s0v = s0[0];
  uint4* slab = slabs + gwave * kSlabUint4;
  for (uint64_t b = gwave; b * kWavePoints < m; b += nwaves)
    bs_eval_batch<XALIGNED>(km, cw_s, cw_v, cw_t, np1, s0v, party, xs, nbytes, m, b * kWavePoints, xl_all[wave],
                            slab, ys);
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

// MEM = true: 16-wave workgroups (n_tt >= 1: 15 LDS x-slots); false: 12 waves.  Both keep the
// bitsliced s / v in per-wave slabs.

template <bool XALIGNED, bool MEM>
__global__ __launch_bounds__((MEM ? 16 : kHybridWaves) * 64) void k_eval16_hybrid(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t m, const uint32_t n_tt, uint32_t* __restrict__ ctr, uint4* __restrict__ slabs,
    const uint4* __restrict__ km, uint4* __restrict__ ys) {
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
    uint4* slab = slabs + ((uint64_t)blockIdx.x * 16 + wave) * kSlabUint4;
    for (uint32_t u = dequeue_unit(ctr); u < nunits; u = dequeue_unit(ctr))
      bs_eval_batch<XALIGNED>(km, cw_s, cw_v, cw_t, np1, s0v, party, xs, nbytes, m, (uint64_t)u * kWavePoints, xl,
                              slab, ys);
  }
}

}  // namespace
