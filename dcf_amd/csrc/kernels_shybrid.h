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

// One wave's 512 points (32 per quad) through the bitsliced engine (kernels_bs.h bs_level: s
// and v in the wave's slab), starting at level pf.levels from the points' rows of the
// shared-prefix table (or at the root when pf.levels = 0).  x rows are 4-byte aligned
// (nbytes % 4 == 0, <= 16).
__device__ __forceinline__ void bs_eval_batch_pf(const uint4* __restrict__ km, const uint4* __restrict__ cw_s,
                                                 const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                                 const uint4 np1, const uint4 s0v, const uint32_t party,
                                                 const uint8_t* __restrict__ xs, const uint32_t nbytes,
                                                 const uint64_t m, const uint64_t p_base, uint32_t* xl,
                                                 uint4* __restrict__ slab, uint4* __restrict__ ys,
                                                 const PrefixTable& pf) {
  const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, quad = lane >> 2;
  const uint64_t p0 = p_base + (uint64_t)quad * kBsPoints;
  const uint32_t nchunk = nbytes >> 2, D = pf.levels;
  const uint4* __restrict__ kmc = km + 8 * c;
  uint4* __restrict__ vp = slab + lane;
  uint4* __restrict__ sp = slab + 512 + lane;
  const uint32_t mlast = (c == 3u) ? 0u : 0xFFFFFFFFu;  // register 24 of column 3 = bit 0 of byte 15
  uint32_t T;
  if (D) {
    // Row of the top-tree table named by each point's first D x bits (Msb0): this lane's
    // column of v, then of s, transposed into bitsliced words.  Gathered 8 rows per pass of a
    // loop that is not unrolled, shifted into place (a shift register of 32 words): 32
    // independent 64-bit gather addresses in flight spilled 128 VGPRs.
    uint32_t a[32];
    for (uint32_t half = 0; half < 2; ++half) {
#pragma unroll 1
      for (uint32_t g = 0; g < 4; ++g) {
        uint32_t t8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint64_t p = min(p0 + 8u * g + k, m - 1);
          const uint32_t idx = bswap32(*reinterpret_cast<const uint32_t*>(xs + p * nbytes)) >> (32u - D);
          t8[k] = reinterpret_cast<const uint32_t*>(pf.sv + 2u * idx)[(half ? 0u : 4u) + c];
        }
#pragma unroll
        for (int k = 0; k < 24; ++k) a[k] = a[k + 8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[24 + k] = t8[k];
      }
      transpose32(a);
      if (half == 0) bs_store32(vp, a);
    }
    T = qperm<kQpBcast3>(a[24]);  // t rides in s's masked bit (kernels16.h PrefixTable)
    a[24] &= mlast;
    bs_store32(sp, a);
  } else {
    uint32_t a[32], w0 = sel4(s0v, c);
    asm volatile("" : "+v"(w0));  // not hoisted out of the batch loop (32 live masks)
    bs_splat(a, w0);
    bs_store32(sp, a);
    for (int i = 0; i < 32; ++i) a[i] = 0u;
    bs_store32(vp, a);
    T = party ? 0xFFFFFFFFu : 0u;
  }
  uint32_t lev = D;
  for (uint32_t cc = D >> 5; cc < nchunk; ++cc) {
    bs_stage_x<true>(xl, xs, nbytes, m, p0, cc);
    for (uint32_t b = lev - 32u * cc; b < 32u; ++b, ++lev)
      bs_level(kmc, vp, sp, xl + b * 16u + quad, T, cw_s[lev], cw_v[lev], cw_t[lev]);
  }
  bs_finish(vp, sp, T, sel4(np1, c), m, p0, ys);
}

// Single key, nbytes % 4 == 0 and <= 16.  tt_mask: stream waves (bit w = wave w),
// at most kShybridXlSlots waves outside it; slabs: 16 x kSlabUint4 uint4 per workgroup.
__global__ __launch_bounds__(kBlock, 1) void k_eval16_shybrid(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t total, uint32_t* __restrict__ ctr, uint4* __restrict__ ys, const PrefixTable pf,
    const uint32_t tt_mask, const uint32_t prio, uint4* __restrict__ slabs, const uint4* __restrict__ km,
    const uint4* __restrict__ rkg) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint32_t xl_all[kShybridXlSlots][32 * 16];
  lds_fill_tables(lds, tab);
  const uint32_t wave = threadIdx.x >> 6;
  if ((tt_mask >> wave) & 1u) {
    if (prio & 1u) __builtin_amdgcn_s_setprio(2);
    // round keys per round from the device copy, as the stream kernel (SGPR keys spill)
    stream_run<2, true, false, kWavePoints, true>(lds, rkg, rk, cw_s, cw_v, cw_t, cw_np1, s0s, party, xs, nbytes, 1,
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
