// kernels_shybrid.h — single-key LAMBDA = 16 eval with both AES engines on
// every CU: stream T-table waves (LDS-bound, kernels_stream.h) and bitsliced
// waves (VALU-bound, kernels_bs.h) in one 16-wave workgroup, below the shared
// prefix table.  Included by dcf_hip.hip only (after kernels_stream.h).
//
// The stream engine keeps the LDS ~90 % busy but issues only ~2 VALU per LDS
// lookup, so about half of every SIMD's VALU cycles are idle.  Bitsliced AES
// needs no LDS at all.  Roles are per wave (`tt_mask` bit w: wave w runs the
// stream engine); a workgroup's waves land on the SIMDs in a fixed cyclic order,
// so waves w and w + 4 share a SIMD and a mask like 0x7777 gives one SIMD to
// the bitsliced engine and three to the stream engine.  Both roles take
// 512-point units from one work counter, so the split adapts to their speeds.
// `prio`: bit 0 raises the stream waves' issue priority (s_setprio), so the
// bitsliced waves only fill VALU slots the stream waves leave.
#pragma once

#include "aes_lds.h"
#include "kernels16.h"
#include "kernels_bs.h"
#include "kernels_stream.h"

namespace {

constexpr int kQpBcast3 = 3 | (3 << 2) | (3 << 4) | (3 << 6);  // c <- 3
constexpr int kShybridXlSlots = 12;  // LDS: 128 KiB tables + 2 KiB of transposed x per bitsliced wave

// One wave's 512 points (32 per quad) through the bitsliced engine, starting at
// level pf.levels from the points' rows of the shared-prefix table (or at the
// root when pf.levels = 0).  x rows are 4-byte aligned (nbytes % 4 == 0, <= 16).
// v is kept in the wave's scratch slab (as bs_eval_batch_mem) so a lane fits in
// 128 VGPRs next to 15 other waves.
__device__ __forceinline__ void bs_eval_batch_pf(const uint4* __restrict__ km, const uint4* __restrict__ cw_s,
                                                 const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                                 const uint4 np1, const uint4 s0v, const uint32_t party,
                                                 const uint8_t* __restrict__ xs, const uint32_t nbytes,
                                                 const uint64_t m, const uint64_t p_base, uint32_t* xl,
                                                 uint4* __restrict__ slab, uint4* __restrict__ ys,
                                                 const PrefixTable& pf) {
  const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, quad = lane >> 2;
  const uint64_t p0 = p_base + (uint64_t)quad * kBsPoints;
  const uint32_t nlev = 8u * nbytes, nchunk = nbytes >> 2, D = pf.levels;
  const uint4* __restrict__ kmc = km + 8 * c;
  uint4* __restrict__ vp = slab + lane;  // v quad q at vp[64 q]
  const uint32_t mlast = (c == 3u) ? 0u : 0xFFFFFFFFu;  // register 24 of column 3 = bit 0 of byte 15
  uint32_t s[32];
  uint32_t T;
  if (D) {
    // Row of the top-tree table named by each point's first D x bits (Msb0): this
    // lane's column of s and of v, transposed into bitsliced registers.
    uint32_t u[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint64_t p = min(p0 + j, m - 1);
      const uint32_t idx = bswap32(*reinterpret_cast<const uint32_t*>(xs + p * nbytes)) >> (32u - D);
      const uint32_t* row = reinterpret_cast<const uint32_t*>(pf.sv + 2u * idx);
      s[j] = row[c];
      u[j] = row[4u + c];
    }
    transpose32(s);
    transpose32(u);
#pragma unroll
    for (int q = 0; q < 8; ++q) vp[64 * q] = make_uint4(u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3]);
    T = qperm<kQpBcast3>(s[24]);  // t rides in s's masked bit (kernels16.h PrefixTable)
    s[24] &= mlast;
  } else {
    bs_splat(s, sel4(s0v, c));
#pragma unroll
    for (int q = 0; q < 8; ++q) vp[64 * q] = make_uint4(0u, 0u, 0u, 0u);
    T = party ? 0xFFFFFFFFu : 0u;
  }
  uint32_t lev = D;
  for (uint32_t cc = D >> 5; cc < nchunk; ++cc) {
    __builtin_amdgcn_wave_barrier();
    if (c == cc) {
      uint32_t w[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint64_t p = min(p0 + j, m - 1);
        w[j] = bswap32(*reinterpret_cast<const uint32_t*>(xs + p * nbytes + 4 * cc));
      }
      transpose32(w);
#pragma unroll
      for (int i = 0; i < 32; ++i) xl[(31u - i) * 16u + quad] = w[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t b = lev - 32u * cc; b < 32u; ++b, ++lev) {
      const uint32_t X = xl[b * 16u + quad];  // bit j: x bit of point j (1 = right)
      const uint4 cs = cw_s[lev], cv = cw_v[lev];
      const uint32_t ct = cw_t[lev];
      uint32_t csw = sel4(cs, c), cvw = sel4(cv, c);
      uint32_t st[32];
      // B = AES(~s); v ^= ((~s) ^ (B & ~X)) & M ^ (T & cw.v)   (lib.rs:182/186)
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
      // A = AES(s); s' = (s ^ (A & ~X)) & M ^ (T & cw.s)   (lib.rs:177-178, 183/187)
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
      // t' = side t ^ (t & side cw.t)   (lib.rs:179-180)
      const uint32_t ctl = 0u - (ct & 1u), ctr = 0u - ((ct >> 1) & 1u);
      T = ((X & tR) | (~X & tL)) ^ (T & ((X & ctr) | (~X & ctl)));
    }
  }
  // y = v ^ s ^ t * cw_np1   (lib.rs:192), then back to one dword per point
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

// Single key, nbytes % 4 == 0 and <= 16.  tt_mask: stream waves (bit w = wave w),
// at most kShybridXlSlots waves outside it; slabs: 16 x kSlabUint4 uint4 per workgroup.
__global__ __launch_bounds__(kBlock, 1) void k_eval16_shybrid(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t total, uint32_t* __restrict__ ctr, uint4* __restrict__ ys, const PrefixTable pf,
    const uint32_t tt_mask, const uint32_t prio, uint4* __restrict__ slabs, const uint4* __restrict__ km) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint32_t xl_all[kShybridXlSlots][32 * 16];
  lds_fill_tables(lds, tab);
  const uint32_t wave = threadIdx.x >> 6;
  if ((tt_mask >> wave) & 1u) {
    if (prio & 1u) __builtin_amdgcn_s_setprio(2);
    stream_run<2, true, false, kWavePoints, false>(lds, nullptr, rk, cw_s, cw_v, cw_t, cw_np1, s0s, party, xs, nbytes, 1,
                                                   total, total, ctr, ys, pf);
    return;
  }
  const uint32_t slot = (uint32_t)__popc(~tt_mask & ((1u << wave) - 1u) & 0xFFFFu);
  if (slot >= (uint32_t)kShybridXlSlots) return;
  uint32_t* xl = xl_all[slot];
  uint4* slab = slabs + ((uint64_t)blockIdx.x * 16 + wave) * kSlabUint4;
  const uint64_t nunits = (total + kWavePoints - 1) / kWavePoints;
  const uint4 np1 = cw_np1[0], s0v = s0s[0];
  for (uint32_t u = dequeue_unit(ctr); u < nunits; u = dequeue_unit(ctr))
    bs_eval_batch_pf(km, cw_s, cw_v, cw_t, np1, s0v, party, xs, nbytes, total, (uint64_t)u * kWavePoints, xl, slab,
                     ys, pf);
}

}  // namespace
