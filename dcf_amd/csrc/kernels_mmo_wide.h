// kernels_mmo_wide.h — the Matyas-Meyer-Oseas AES-128 PRG at LAMBDA >= 32 (SURVEY §8 f3:
// BASELINE.json config 4 names "multi-block MMO PRG output per level").  Included by
// dcf_hip.hip only (after kernels_mmo.h).
//
// Definition (ours — the reference crate has no MMO PRG, so parity is UNPINNED by it;
// the same definition as the test suite's CPU restatement and the LAMBDA = 16 kernels):
//   out_b[j] = AES128_{k[b * nb + j]}(seed_j) ^ seed_j,  nb = LAMBDA / 16, 16-byte block j,
//   b = 0: s_L, 1: v_L, 2: s_R, 3: v_R;  t_L = lsb(s_L[0]), t_R = lsb(s_R[0]) (before the
//   clear); bit 0 of byte LAMBDA - 1 cleared in all four outputs (prg.rs:63-68 convention).
// Block j of every output depends only on block j of the seed, and the walk's t bits
// (lib.rs:179-180) only on block 0.  So, as the Hirose LAMBDA >= 32 path does, eval runs
//   head: block 0 of every point's walk -> y[0:16) and the point's t-vector (t_0..t_n);
//   tail: block j >= 1 of every point's walk, given the t-vector -> y[16j:16j+16);
// and gen runs a head over block 0 of both parties (t bits and t-CWs) and a tail over the
// other blocks.  A wave always holds 64 lanes on the same level of the same block j, so the
// correction words are wave-uniform loads and a lane's two round-key schedules (its side's
// s and v keys) are the wave's j-th schedules of outputs (0, 1) or (2, 3), read per round
// from the device copy (L1-resident).  Work per eval: 2 AES-128 blocks per level per block
// (the side's s and v), 2 * 8N * LAMBDA / 16 in all.
#pragma once

#include "aes_lds.h"
#include "kernels_mmo.h"

namespace {

// t-vector words per point: t_0 .. t_n (n = 8N) at bit r & 31 of word r >> 5
__host__ __device__ constexpr uint32_t mmo_t_words(uint32_t nlev) { return (nlev + 32u) / 32u; }

__device__ __forceinline__ uint32_t mmo_xbit(const uint8_t* __restrict__ x, uint32_t lev) {
  return (x[lev >> 3] >> (7u - (lev & 7u))) & 1u;  // Msb0 (lib.rs:181)
}

// Walk of block j over n levels for 64 points per wave (lane = point).  HEAD (j = 0):
// t comes from the AES output and the t-vector is written; otherwise t is read from it.
// rk: 4 * nb AES-128 schedules (11 round keys each), schedule b * nb + j.
template <bool HEAD>
__global__ __launch_bounds__(kBlock, 1) void k_mmo_wide_eval(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk, const uint8_t* __restrict__ cw_s,
    const uint8_t* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint8_t* __restrict__ cw_np1,
    const uint8_t* __restrict__ s0, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint32_t lam, const uint64_t num_keys, const uint64_t key, const uint64_t count,
    uint32_t* __restrict__ tvec, uint8_t* __restrict__ ys) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint32_t nb = lam / 16u, nlev = 8u * nbytes, lane = threadIdx.x & 63u;
  const uint32_t twn = mmo_t_words(nlev);
  const uint64_t groups = (count + 63) / 64;
  const uint64_t jn = HEAD ? 1 : nb - 1;  // blocks per point group handled by this kernel
  const uint64_t items = groups * jn;
  const uint64_t wstride = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t it = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); it < items; it += wstride) {
    const uint64_t g = it / jn;
    const uint32_t j = HEAD ? 0u : 1u + (uint32_t)(it % jn);
    const uint64_t p = g * 64 + lane;
    const bool live = p < count;
    const uint64_t pp = live ? p : count - 1;
    const uint8_t* x = xs + pp * nbytes;
    const uint4 sv = reinterpret_cast<const uint4*>(s0)[j];  // k.s0s[0] (lib.rs:168), block j
    uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w}, v[4] = {0u, 0u, 0u, 0u};
    // t-vector word of bits 32w..32w+31 (t_r at bit r & 31): HEAD accumulates and stores
    // each word when complete, the tail streams them in (wave-uniform level: L1 hits)
    uint32_t tw = HEAD ? party : tvec[pp * twn];  // t_0 (lib.rs:169)
    uint32_t t = party;
    const uint32_t mlast = (j == nb - 1) ? kMaskLast : 0xFFFFFFFFu;
    for (uint32_t lev = 0; lev < nlev; ++lev) {
      const uint32_t xb = mmo_xbit(x, lev);
      const uint4* rks = rk + (uint64_t)((2u * xb) * nb + j) * kMmoRk;       // s_side key
      const uint4* rkv = rk + (uint64_t)((2u * xb + 1u) * nb + j) * kMmoRk;  // v_side key
      uint32_t st[2][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) st[0][k] = st[1][k] = s[k];
      const uint4* const rkp[2] = {rks, rkv};
      aes_tt_lk<10, 2, true>(st, rkp, lds, lc);
      const uint64_t ci = ((uint64_t)lev * num_keys + key) * lam + 16ull * j;
      const uint4 cs = *reinterpret_cast<const uint4*>(cw_s + ci), cv = *reinterpret_cast<const uint4*>(cw_v + ci);
      const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w}, cvw[4] = {cv.x, cv.y, cv.z, cv.w};
      const uint32_t tm = 0u - t;
      uint32_t tn = 0u;
      if (HEAD) {
        const uint32_t ct = cw_t[(uint64_t)lev * num_keys + key];
        tn = ((st[0][0] ^ s[0]) & 1u) ^ (t & (ct >> xb) & 1u);  // t' = t_side ^ t & cw.t_side (lib.rs:179-180)
      } else {
        const uint32_t r = lev + 1u;
        if ((r & 31u) == 0u) tw = tvec[pp * twn + (r >> 5)];
        tn = (tw >> (r & 31u)) & 1u;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t msk = (k == 3) ? mlast : 0xFFFFFFFFu;
        v[k] ^= ((st[1][k] ^ s[k]) & msk) ^ (tm & cvw[k]);  // v ^= v_side ^ t*cw.v (lib.rs:182/186)
        s[k] = ((st[0][k] ^ s[k]) & msk) ^ (tm & csw[k]);   // s' = s_side ^ t*cw.s (lib.rs:177-178)
      }
      t = tn;
      if (HEAD) {
        const uint32_t r = lev + 1u;
        if ((r & 31u) == 0u) {  // word (r >> 5) - 1 complete
          if (live) tvec[p * twn + (r >> 5) - 1u] = tw;
          tw = 0u;
        }
        tw |= tn << (r & 31u);
      }
    }
    const uint4 np = *reinterpret_cast<const uint4*>(cw_np1 + key * lam + 16ull * j);
    const uint32_t tm = 0u - t;
    if (live) {
      *reinterpret_cast<uint4*>(ys + p * lam + 16ull * j) =  // y = v ^ s ^ t*cw_np1 (lib.rs:192)
          make_uint4(v[0] ^ s[0] ^ (tm & np.x), v[1] ^ s[1] ^ (tm & np.y), v[2] ^ s[2] ^ (tm & np.z),
                     v[3] ^ s[3] ^ (tm & np.w));
      if (HEAD) tvec[p * twn + (nlev >> 5)] = tw;  // the word holding t_n
    }
  }
}

// DcfImpl::gen (lib.rs:86-161) with the MMO PRG at LAMBDA >= 32, block j of K keys (lane =
// key).  HEAD (j = 0): the parties' t bits evolve from the AES outputs, the t-CWs are
// written to cw_t and the per-level (t0, t1) pairs to tinfo; otherwise they are read from
// tinfo.  All four outputs of both parties' seeds per level: 8 AES-128 blocks.
template <bool HEAD>
__global__ __launch_bounds__(kBlock, 1) void k_mmo_wide_gen(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk, const uint8_t* __restrict__ alpha,
    const uint8_t* __restrict__ beta, const uint8_t* __restrict__ s0_0, const uint8_t* __restrict__ s0_1,
    const uint32_t bound, const uint32_t nbytes, const uint32_t lam, const uint64_t num_keys,
    uint8_t* __restrict__ cw_s, uint8_t* __restrict__ cw_v, uint8_t* __restrict__ cw_t,
    uint8_t* __restrict__ cw_np1, uint32_t* __restrict__ tinfo) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint32_t nb = lam / 16u, nlev = 8u * nbytes, lane = threadIdx.x & 63u;
  const uint64_t groups = (num_keys + 63) / 64;
  const uint64_t jn = HEAD ? 1 : nb - 1;
  const uint64_t items = groups * jn;
  const uint64_t wstride = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t it = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); it < items; it += wstride) {
    const uint64_t g = it / jn;
    const uint32_t j = HEAD ? 0u : 1u + (uint32_t)(it % jn);
    const uint64_t k = g * 64 + lane;
    const bool live = k < num_keys;
    const uint64_t kk = live ? k : num_keys - 1;
    const uint8_t* al = alpha + kk * nbytes;
    const uint4 a0 = *reinterpret_cast<const uint4*>(s0_0 + kk * lam + 16ull * j);
    const uint4 a1 = *reinterpret_cast<const uint4*>(s0_1 + kk * lam + 16ull * j);
    const uint4 be = *reinterpret_cast<const uint4*>(beta + kk * lam + 16ull * j);
    uint32_t s[2][4] = {{a0.x, a0.y, a0.z, a0.w}, {a1.x, a1.y, a1.z, a1.w}};
    const uint32_t bw[4] = {be.x, be.y, be.z, be.w};
    uint32_t va[4] = {0u, 0u, 0u, 0u};
    uint32_t t0 = 0u, t1 = 1u;  // lib.rs:100
    const uint32_t mlast = (j == nb - 1) ? kMaskLast : 0xFFFFFFFFu;
    for (uint32_t lev = 0; lev < nlev; ++lev) {
      // o[p][b]: output b (s_L, v_L, s_R, v_R) of party p's seed, block j (masked)
      uint32_t o[2][4][4];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t st[2][4];
#pragma unroll
          for (int q = 0; q < 4; ++q) st[0][q] = st[1][q] = s[p][q];
          const uint4* const rkp[2] = {rk + (uint64_t)((2u * h) * nb + j) * kMmoRk,
                                       rk + (uint64_t)((2u * h + 1u) * nb + j) * kMmoRk};
          aes_tt_lk<10, 2, true>(st, rkp, lds, lc);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t msk = (q == 3) ? mlast : 0xFFFFFFFFu;
            o[p][2 * h][q] = (st[0][q] ^ s[p][q]) & msk;
            o[p][2 * h + 1][q] = (st[1][q] ^ s[p][q]) & msk;
          }
        }
      const uint32_t a = mmo_xbit(al, lev);  // alpha bit, Msb0 (lib.rs:106)
      const uint32_t am = 0u - a;
      const uint32_t bm = (bound == 0) ? am : ~am;  // LtBeta: beta when alpha_i = 1 (lib.rs:114-125)
      uint32_t tlcw, trcw, tl0, tr0, tl1, tr1;
      if (HEAD) {  // t from byte 0 of the s outputs, before the clear (byte 0 is never cleared here)
        tl0 = o[0][0][0] & 1u; tr0 = o[0][2][0] & 1u;
        tl1 = o[1][0][0] & 1u; tr1 = o[1][2][0] & 1u;
        tlcw = tl0 ^ tl1 ^ a ^ 1u;  // lib.rs:130
        trcw = tr0 ^ tr1 ^ a;       // lib.rs:131
      } else {
        const uint32_t w = tinfo[kk * nlev + lev];  // t0, t1 before this level, tlcw, trcw
        t0 = w & 1u; t1 = (w >> 1) & 1u; tlcw = (w >> 2) & 1u; trcw = (w >> 3) & 1u;
        tl0 = tr0 = tl1 = tr1 = 0u;
      }
      // the lose side is left (outputs 0, 1) when alpha_i = 1, right (2, 3) otherwise: picked by a
      // select per word (a runtime index into o[][][] would put the array on the stack)
      const uint32_t m0 = 0u - t0, m1 = 0u - t1;
      uint32_t scw[4], vcw[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t ls[2], lv[2], ks[2], kv[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          ls[p] = a ? o[p][0][q] : o[p][2][q];
          lv[p] = a ? o[p][1][q] : o[p][3][q];
          ks[p] = a ? o[p][2][q] : o[p][0][q];
          kv[p] = a ? o[p][3][q] : o[p][1][q];
        }
        scw[q] = ls[0] ^ ls[1];                             // lib.rs:112
        vcw[q] = lv[0] ^ lv[1] ^ va[q] ^ (bm & bw[q]);      // lib.rs:113-125
        va[q] ^= kv[0] ^ kv[1] ^ vcw[q];                    // lib.rs:126-129
        s[0][q] = ks[0] ^ (m0 & scw[q]);                    // lib.rs:139-148
        s[1][q] = ks[1] ^ (m1 & scw[q]);
      }
      if (live) {
        const uint64_t ci = ((uint64_t)lev * num_keys + k) * lam + 16ull * j;
        *reinterpret_cast<uint4*>(cw_s + ci) = make_uint4(scw[0], scw[1], scw[2], scw[3]);
        *reinterpret_cast<uint4*>(cw_v + ci) = make_uint4(vcw[0], vcw[1], vcw[2], vcw[3]);
      }
      if (HEAD) {
        if (live) {
          cw_t[(uint64_t)lev * num_keys + k] = (uint8_t)(tlcw | (trcw << 1));
          tinfo[k * nlev + lev] = t0 | (t1 << 1) | (tlcw << 2) | (trcw << 3);
        }
        const uint32_t tkcw = a ? trcw : tlcw;
        const uint32_t nt0 = (a ? tr0 : tl0) ^ (t0 & tkcw);  // lib.rs:149-152
        const uint32_t nt1 = (a ? tr1 : tl1) ^ (t1 & tkcw);
        t0 = nt0;
        t1 = nt1;
      }
    }
    if (live)  // cw_np1 = s_0 ^ s_1 ^ v_alpha (lib.rs:155)
      *reinterpret_cast<uint4*>(cw_np1 + k * lam + 16ull * j) =
          make_uint4(s[0][0] ^ s[1][0] ^ va[0], s[0][1] ^ s[1][1] ^ va[1], s[0][2] ^ s[1][2] ^ va[2],
                     s[0][3] ^ s[1][3] ^ va[3]);
  }
}

// Prg::gen test hook at LAMBDA >= 32: row per seed = s_l | v_l | s_r | v_r | t_l | t_r; one
// lane per (seed, block j), all four outputs of block j.
__global__ __launch_bounds__(kBlock, 1) void k_prg_mmo_wide(const uint32_t* __restrict__ tab,
                                                            const uint4* __restrict__ rk,
                                                            const uint8_t* __restrict__ seeds, const uint64_t m,
                                                            const uint32_t lam, uint8_t* __restrict__ out) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint32_t nb = lam / 16u;
  const uint64_t n = m * nb, row = 4ull * lam + 2;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    const uint64_t ii = i < n ? i : n - 1;
    const uint64_t sd = ii / nb;
    const uint32_t j = (uint32_t)(ii % nb);
    const uint4 sv = *reinterpret_cast<const uint4*>(seeds + sd * lam + 16ull * j);
    const uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
    const uint32_t mlast = (j == nb - 1) ? kMaskLast : 0xFFFFFFFFu;
    uint32_t o[4][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t st[2][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) st[0][q] = st[1][q] = s[q];
      const uint4* const rkp[2] = {rk + (uint64_t)((2u * h) * nb + j) * kMmoRk,
                                   rk + (uint64_t)((2u * h + 1u) * nb + j) * kMmoRk};
      aes_tt_lk<10, 2, true>(st, rkp, lds, lc);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[2 * h][q] = st[0][q] ^ s[q];
        o[2 * h + 1][q] = st[1][q] ^ s[q];
      }
    }
    if (i < n) {
      uint8_t* r = out + sd * row;
      if (j == 0) {  // t bits before the clear
        r[4ull * lam] = (uint8_t)(o[0][0] & 1u);
        r[4ull * lam + 1] = (uint8_t)(o[2][0] & 1u);
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        uint8_t* d = r + (uint64_t)b * lam + 16ull * j;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t w = o[b][q] & ((q == 3) ? mlast : 0xFFFFFFFFu);
#pragma unroll
          for (int y = 0; y < 4; ++y) d[4 * q + y] = (uint8_t)(w >> (8 * y));
        }
      }
    }
  }
}

}  // namespace
