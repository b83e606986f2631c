// kernels_mmo.h — DCF over the Matyas-Meyer-Oseas AES-128 PRG at LAMBDA = 16.
// Included by dcf_hip.hip only.
//
// Aes128MatyasMeyerOseasPrg (BASELINE.json north_star; absent from the
// reference crate, so its definition here is ours and parity is UNPINNED by the
// reference — see DESIGN.md §4 "MMO"):
//   out[b] = AES128_{k_b}(seed) ^ seed,  b = 0: s_L, 1: v_L, 2: s_R, 3: v_R
//   t_L = lsb(out[0])[0], t_R = lsb(out[2])[0]   (Lsb0 bit 0 of byte 0, read before the clear)
//   bit 0 of byte 15 cleared in all four outputs  (as prg.rs:63-68 does for Hirose)
// So a walk step needs exactly two blocks, (k0, k1) going left or (k2, k3)
// going right: each lane reads the round keys of its side from LDS.
#pragma once

// A/B knob: the MMO AES rounds at wave priority 1.
#ifndef DCF_MMO_PRIO
#define DCF_MMO_PRIO 1
#endif

#include "aes_lds.h"
#include "kernels16.h"

namespace {

constexpr int kMmoRk = 11;  // AES-128 round keys per schedule

// The 4 schedules in LDS, 11 uint4 apart: schedule i starts at 16-byte slot 11 i,
// so the two a lane may pick for one block (i and i + 2) sit 22 slots apart and
// ds_read_b128 from both halves of a wave never share a bank group.
__device__ __forceinline__ void lds_fill_rk128(uint4* rks, const uint4* __restrict__ rk128) {
  if (threadIdx.x < 4 * kMmoRk) rks[threadIdx.x] = rk128[threadIdx.x];
}

// One point (lib.rs:166-193) over the MMO PRG.
__device__ __forceinline__ uint4 mmo_eval_one(const uint32_t* lds, uint32_t lc, const uint4* rks,
                                              const uint4* __restrict__ cw_s, const uint4* __restrict__ cw_v,
                                              const uint8_t* __restrict__ cw_t, const uint4 np, const uint4 sv,
                                              uint32_t party, const uint8_t* __restrict__ x, uint32_t nbytes,
                                              uint64_t num_keys, uint64_t key, const PrefixTable& pf) {
  const uint32_t nlev = 8u * nbytes;
  const uint32_t nchunk = (nbytes + 3u) >> 2;
  uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  uint32_t t = party;
  uint32_t lev = 0;
  uint32_t w0 = load_bits32(x, 0, nbytes);
  if (pf.levels) {  // one key: start below the shared prefix (wave-uniform depth)
    lev = pf.levels;
    uint4 ps, pv;
    prefix_row(pf, w0 >> (32u - lev), ps, pv, t);
    s[0] = ps.x; s[1] = ps.y; s[2] = ps.z; s[3] = ps.w;
    v[0] = pv.x; v[1] = pv.y; v[2] = pv.z; v[3] = pv.w;
  }
  for (uint32_t c = 0; c < nchunk; ++c) {
    uint32_t cur = c ? load_bits32(x, c, nbytes) : w0 << lev;  // levels < 32: the prefix sits in word 0
    const uint32_t lend = min(32u, nlev - 32u * c);
    for (uint32_t b = c ? 0u : lev; b < lend; ++b, ++lev) {
      const uint32_t xb = cur >> 31;  // Msb0 bit of x (lib.rs:181)
      cur <<= 1;
      const uint4* const rk[2] = {rks + kMmoRk * (2u * xb), rks + kMmoRk * (2u * xb + 1u)};
      uint32_t st[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) st[0][j] = st[1][j] = s[j];
      if (DCF_MMO_PRIO) __builtin_amdgcn_s_setprio(1);
      aes128_tt<2>(st, rk, lds, lc);  // side's s and v blocks
      if (DCF_MMO_PRIO) __builtin_amdgcn_s_setprio(0);
      const uint64_t ci = (uint64_t)lev * num_keys + key;
      const uint4 cs = cw_s[ci], cv = cw_v[ci];
      const uint32_t ct = cw_t[ci];
      const uint32_t tm = 0u - t;
      const uint32_t csw[4] = {cs.x, cs.y, cs.z, cs.w}, cvw[4] = {cv.x, cv.y, cv.z, cv.w};
      const uint32_t tn = ((st[0][0] ^ s[0]) & 1u) ^ (t & (ct >> xb) & 1u);  // lib.rs:179-180
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t msk = (j == 3) ? kMaskLast : 0xFFFFFFFFu;
        v[j] ^= ((st[1][j] ^ s[j]) & msk) ^ (tm & cvw[j]);  // lib.rs:182/186
        s[j] = ((st[0][j] ^ s[j]) & msk) ^ (tm & csw[j]);   // lib.rs:177-178, 183/187
      }
      t = tn;
    }
  }
  const uint32_t tm = 0u - t;  // lib.rs:192
  return make_uint4(v[0] ^ s[0] ^ (tm & np.x), v[1] ^ s[1] ^ (tm & np.y), v[2] ^ s[2] ^ (tm & np.z),
                    v[3] ^ s[3] ^ (tm & np.w));
}

// DcfImpl::eval with the MMO PRG.  MODE as k_eval16 (0 one key, 1 wave-uniform key, 2 any).
template <int MODE>
__global__ __launch_bounds__(kBlock, 1) void k_eval16_mmo(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk128, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t num_keys, const uint64_t points_per_key, uint4* __restrict__ ys, const PrefixTable pf) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 rks[4 * kMmoRk];
  lds_fill_rk128(rks, rk128);
  lds_fill_tables(lds, tab);  // its barrier also publishes rks
  const uint32_t lc = lane_const();
  const uint64_t total = num_keys * points_per_key;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < total; base += stride) {
    const uint64_t g = base + (threadIdx.x & 63u);
    const bool live = g < total;
    const uint64_t gg = live ? g : total - 1;
    uint64_t key = 0;
    if (MODE == 1) key = __builtin_amdgcn_readfirstlane((uint32_t)(gg / points_per_key));
    if (MODE == 2) key = gg / points_per_key;
    const uint4 y = mmo_eval_one(lds, lc, rks, cw_s, cw_v, cw_t, cw_np1[key], s0s[key], party, xs + gg * nbytes,
                                 nbytes, num_keys, key, pf);
    if (live) ys[g] = y;
  }
}

// All four MMO outputs of one seed (masked) and the two t bits.
__device__ __forceinline__ void mmo_prg4(const uint32_t* lds, uint32_t lc, const uint4* rks, const uint32_t (&s)[4],
                                         uint32_t (&o)[4][4], uint32_t& tl, uint32_t& tr) {
  // Two blocks at a time.  A zero offset laundered through an empty asm keeps the
  // loop-invariant round-key reads from being hoisted out of the caller's level
  // loop (4 x 44 words would not fit in registers); the base stays the LDS array,
  // so the reads remain ds_read (a laundered generic pointer would not be).
  uint32_t off = 0u;
  asm volatile("" : "+v"(off));
  const uint4* r = rks + off;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint4* const rk[2] = {r + 2 * h * kMmoRk, r + (2 * h + 1) * kMmoRk};
    uint32_t st[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) st[0][j] = st[1][j] = s[j];
    if (DCF_MMO_PRIO) __builtin_amdgcn_s_setprio(1);
    aes128_tt<2>(st, rk, lds, lc);
    if (DCF_MMO_PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * h][j] = st[0][j];
      o[2 * h + 1][j] = st[1][j];
    }
  }
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) o[b][j] ^= s[j];  // Matyas-Meyer-Oseas: E_k(m) ^ m
  tl = o[0][0] & 1u;
  tr = o[2][0] & 1u;
#pragma unroll
  for (int b = 0; b < 4; ++b) o[b][3] &= kMaskLast;
}

// DcfImpl::gen (lib.rs:86-161) with the MMO PRG, one lane per key.
__global__ __launch_bounds__(kBlock, 1) void k_gen16_mmo(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk128, const uint8_t* __restrict__ alpha,
    const uint4* __restrict__ beta, const uint4* __restrict__ s0_0, const uint4* __restrict__ s0_1,
    const uint32_t bound, const uint32_t nbytes, const uint64_t num_keys, uint4* __restrict__ cw_s,
    uint4* __restrict__ cw_v, uint8_t* __restrict__ cw_t, uint4* __restrict__ cw_np1) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 rks[4 * kMmoRk];
  lds_fill_rk128(rks, rk128);
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint32_t nlev = 8u * nbytes;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < num_keys; base += stride) {
    const uint64_t g = base + (threadIdx.x & 63u);
    const bool live = g < num_keys;
    const uint64_t k = live ? g : num_keys - 1;
    uint32_t s[2][4], va[4] = {0u, 0u, 0u, 0u}, be[4];
    {
      const uint4 a0 = s0_0[k], a1 = s0_1[k], bb = beta[k];
      s[0][0] = a0.x; s[0][1] = a0.y; s[0][2] = a0.z; s[0][3] = a0.w;
      s[1][0] = a1.x; s[1][1] = a1.y; s[1][2] = a1.z; s[1][3] = a1.w;
      be[0] = bb.x; be[1] = bb.y; be[2] = bb.z; be[3] = bb.w;
    }
    uint32_t t0 = 0u, t1 = 1u;  // lib.rs:100
    const uint8_t* al = alpha + k * nbytes;
    for (uint32_t lev = 0; lev < nlev; ++lev) {
      uint32_t o0[4][4], o1[4][4], tl0, tr0, tl1, tr1;  // per party: s_L, v_L, s_R, v_R
      mmo_prg4(lds, lc, rks, s[0], o0, tl0, tr0);       // lib.rs:103
      mmo_prg4(lds, lc, rks, s[1], o1, tl1, tr1);       // lib.rs:104
      const uint32_t a = (al[lev >> 3] >> (7u - (lev & 7u))) & 1u;  // alpha_i, Msb0 (lib.rs:106)
      const uint32_t am = 0u - a;  // keep = R, lose = L when alpha_i = 1 (lib.rs:107-111)
      const uint32_t bm = (bound == 0) ? am : ~am;  // lib.rs:114-125: LtBeta when lose == L
      uint32_t scw[4], vcw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t sl = o0[0][j] ^ o1[0][j], sr = o0[2][j] ^ o1[2][j];
        const uint32_t vl = o0[1][j] ^ o1[1][j], vr = o0[3][j] ^ o1[3][j];
        scw[j] = a ? sl : sr;                                // lib.rs:112 (lose side)
        vcw[j] = (a ? vl : vr) ^ va[j] ^ (bm & be[j]);       // lib.rs:113-125
        va[j] ^= (a ? vr : vl) ^ vcw[j];                     // lib.rs:126-129 (keep side)
      }
      const uint32_t tlcw = tl0 ^ tl1 ^ a ^ 1u;  // lib.rs:130
      const uint32_t trcw = tr0 ^ tr1 ^ a;       // lib.rs:131
      const uint32_t tkcw = a ? trcw : tlcw;
      const uint32_t m0 = 0u - t0, m1 = 0u - t1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // lib.rs:139-148
        s[0][j] = (a ? o0[2][j] : o0[0][j]) ^ (m0 & scw[j]);
        s[1][j] = (a ? o1[2][j] : o1[0][j]) ^ (m1 & scw[j]);
      }
      const uint32_t nt0 = (a ? tr0 : tl0) ^ (t0 & tkcw);  // lib.rs:149-152
      const uint32_t nt1 = (a ? tr1 : tl1) ^ (t1 & tkcw);
      t0 = nt0;
      t1 = nt1;
      if (live) {
        const uint64_t ci = (uint64_t)lev * num_keys + k;
        cw_s[ci] = make_uint4(scw[0], scw[1], scw[2], scw[3]);
        cw_v[ci] = make_uint4(vcw[0], vcw[1], vcw[2], vcw[3]);
        cw_t[ci] = (uint8_t)(tlcw | (trcw << 1));
      }
    }
    if (live)  // lib.rs:155
      cw_np1[k] = make_uint4(s[0][0] ^ s[1][0] ^ va[0], s[0][1] ^ s[1][1] ^ va[1], s[0][2] ^ s[1][2] ^ va[2],
                             s[0][3] ^ s[1][3] ^ va[3]);
  }
}

// Prg::gen test hook: row per seed = s_l | v_l | s_r | v_r | t_l | t_r (66 bytes).
__global__ __launch_bounds__(kBlock, 1) void k_prg16_mmo(const uint32_t* __restrict__ tab,
                                                         const uint4* __restrict__ rk128,
                                                         const uint4* __restrict__ seeds, const uint64_t m,
                                                         uint8_t* __restrict__ out) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 rks[4 * kMmoRk];
  lds_fill_rk128(rks, rk128);
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x; g0 < m; g0 += stride) {
    const uint64_t g = g0 + threadIdx.x;
    const uint4 sv = seeds[g < m ? g : m - 1];
    const uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
    uint32_t o[4][4], tl, tr;
    mmo_prg4(lds, lc, rks, s, o, tl, tr);
    if (g >= m) continue;
    uint8_t* row = out + g * 66;
    for (int q = 0; q < 4; ++q)
      for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) row[16 * q + 4 * j + k] = (uint8_t)(o[q][j] >> (8 * k));
    row[64] = (uint8_t)tl;
    row[65] = (uint8_t)tr;
  }
}

// Full-domain level with the MMO PRG: one lane per parent, four blocks give both children.
__global__ __launch_bounds__(kBlock, 1) void k_fd_level16_mmo(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk128, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint32_t lev, const uint32_t nlev, const uint64_t nparents, const uint4* __restrict__ s_in,
    const uint4* __restrict__ v_in, const uint8_t* __restrict__ t_in, uint4* __restrict__ s_out,
    uint4* __restrict__ v_out, uint8_t* __restrict__ t_out, uint4* __restrict__ ys, uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 rks[4 * kMmoRk];
  lds_fill_rk128(rks, rk128);
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
    uint32_t o[4][4], tl0, tr0;
    mmo_prg4(lds, lc, rks, s, o, tl0, tr0);
    const uint32_t tm = 0u - t;
    uint32_t sl[4], vl[4], sr[4], vr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // lib.rs:177-189 with x bit 0 (L) and 1 (R)
      sl[k] = o[0][k] ^ (tm & csw[k]);
      vl[k] = v[k] ^ o[1][k] ^ (tm & cvw[k]);
      sr[k] = o[2][k] ^ (tm & csw[k]);
      vr[k] = v[k] ^ o[3][k] ^ (tm & cvw[k]);
    }
    const uint32_t tl = tl0 ^ (t & ct & 1u), tr = tr0 ^ (t & (ct >> 1) & 1u);
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

}  // namespace
