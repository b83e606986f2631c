// kernels_lat.h — latency kernels for tiny batches at LAMBDA = 16 (Hirose PRG):
// one AES-256 column per lane.  Included by dcf_hip.hip only (after kernels16.h).
//
// The crate's own benches time ONE gen and ONE single-point eval per call
// (benches/dcf.rs:7-43).  A lone point walks its 8N levels back to back, so what
// bounds the call is the latency of one level, not throughput: with a whole block
// per lane (k_eval16_pair) a round is 16 table lookups + 16 address VALUs + 8 XORs
// issued by one wave (~300 cycles per round).  Here the four columns of a block sit
// in a lane quad: lane j builds column j of the next state from byte 0 of its own
// column and bytes 1..3 of columns j+1..j+3, which DPP quad_perm rotations bring in
// (T-table round of FIPS-197 §5.1 as in aes256_tt: out_j = T0[s_j.b0] ^ T1[s_{j+1}.b1]
// ^ T2[s_{j+2}.b2] ^ T3[s_{j+3}.b3] ^ rk_j) — 4 lookups, 4 address VALUs, 3 DPP moves
// and 2 XORs per lane and round, a quarter of the dependent chain.
//   eval  (k_eval16_oct): 8 lanes per point, quad 0 = A = AES(s), quad 1 = B = AES(~s);
//         a DPP row rotation swaps the two quads' column, and every lane then runs the
//         level update (lib.rs:174-189) for its column; t comes from column 0's lanes.
//   gen   (k_gen16_col):  16 lanes per key, quad q = block q of the level (A0, B0, A1,
//         B1: prg.rs:42-73 on both parties' seeds, lib.rs:103-104); three DPP row
//         rotations give every lane its column of all four blocks (lib.rs:105-152).
// The key (eval) / alpha (gen) are staged in LDS beside the T-tables, so the kernels may
// read their inputs from, and write outputs to, host-mapped pinned memory (the C ABI's
// host entry points pass such buffers for tiny calls: no copy commands at all).
#pragma once

#include "aes_lds.h"

namespace {

constexpr uint32_t kColMaxLevels = 256;  // N <= 32 (the staged key / x rows)

// DPP: quad_perm rotations (aes_lds.h kQpRot*) and row rotations (lane i <- i - n mod 16).
constexpr int kRowRor4 = 0x124, kRowRor8 = 0x128, kRowRor12 = 0x12C;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

// Column j of AES-256(in) for the lane quad holding the block's four columns (lane j of the
// quad holds column j); kw[r] = word j of round key r.
__device__ __forceinline__ uint32_t aes256_col(uint32_t st, const uint32_t (&kw)[15], const uint32_t* lds,
                                               uint32_t lc) {
  st ^= kw[0];
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    // out_j = T0[s_j.b0] ^ T1[s_{j+1}.b1] ^ T2[s_{j+2}.b2] ^ T3[s_{j+3}.b3]: lane j looks up all
    // four bytes of ITS word (T1[s_j.b1] is lane j-1's term, ...) and the quad rotations move
    // the results instead of the inputs — the lookups start right after the previous round's
    // XOR (no DPP hazard wait, no moves in front of them) and the moves fold into the XORs.
    const uint32_t a = lk<0, 0>(lds, st, lc);
    const uint32_t c = lk<1, 1>(lds, st, lc);
    const uint32_t d = lk<2, 2>(lds, st, lc);
    const uint32_t e = lk<3, 3>(lds, st, lc);
    st = (a ^ kw[r]) ^ dpp<kQpRot1>(c) ^ dpp<kQpRot2>(d) ^ dpp<kQpRot3>(e);
  }
  // final round: SubBytes + ShiftRows + AddRoundKey (S(x) sits in byte r of T_{(r+2)&3})
  const uint32_t w1 = dpp<kQpRot1>(st), w2 = dpp<kQpRot2>(st), w3 = dpp<kQpRot3>(st);
  const uint32_t a = lk<2, 0>(lds, st, lc);
  const uint32_t c = lk<3, 1>(lds, w1, lc);
  const uint32_t d = lk<0, 2>(lds, w2, lc);
  const uint32_t e = lk<1, 3>(lds, w3, lc);
  return xor3(__builtin_amdgcn_perm(c, a, 0x0c0c0500u), __builtin_amdgcn_perm(e, d, 0x07020c0cu), kw[14]);
}

// AES-256 with a block on a 16-lane row, ONE table lookup per lane and round (k_eval16_row).
// Layout A: lane p of the row holds column p&3 of the state; layout B: column p>>2.  From A,
// lane p computes the term T_k[byte k of its column] of output column j = p>>2 (k = (p&3) - j):
// the XOR over its quad is column j, so one round leaves layout B (FIPS-197 §5.1 T-table form,
// out_j = T0[s_j.b0] ^ T1[s_{j+1}.b1] ^ T2[s_{j+2}.b2] ^ T3[s_{j+3}.b3] ^ rk_j); from B the
// roles transpose and a stride-4 XOR over the row (row_ror 4, 8) returns to layout A.  Per
// round: one v_perm address, one ds_read_b32, two DPP XORs and the round-key XOR — 7
// instructions in one lane's dependent chain against aes256_col's 18; a lone wave pays ~10
// cycles per dependent VALU and 64 per dependent LDS read on gfx950, so the block takes 1234
// instead of 1692 cycles (scripts/micro/lat_chain.hip, profiles/r03v_lat_chain.json).
// Fourteen lookup rounds leave layout A again; rkA[r] / rkB[r] = word p&3 / p>>2 of round key r.
__device__ __forceinline__ uint32_t col16_sel(uint32_t k, uint32_t tbl) {  // lk()'s selector, k per lane
  return ((tbl & 1u) ? 1u : 0u) | ((4u + k) << 8) | (((tbl >> 1) ? 2u : 0x0cu) << 16) | (0x0cu << 24);
}
__device__ __forceinline__ uint32_t aes256_col16(uint32_t st, const uint32_t (&rkA)[15], const uint32_t (&rkB)[15],
                                                 const uint32_t* lds, uint32_t lc, uint32_t selA, uint32_t selB,
                                                 uint32_t selF, uint32_t fmask) {
  st ^= rkA[0];
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    const bool fromA = r & 1;
    uint32_t x = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) +
                                                    __builtin_amdgcn_perm(st, lc, fromA ? selA : selB));
    if (fromA) {  // XOR over the quad: output column p>>2 (layout B)
      x ^= dpp<1 | (0 << 2) | (3 << 4) | (2 << 6)>(x);
      x ^= dpp<kQpRot2>(x);
      st = x ^ rkB[r];
    } else {      // XOR over lanes p, p-4, p-8, p-12: output column p&3 (layout A)
      x ^= dpp<kRowRor4>(x);
      x ^= dpp<kRowRor8>(x);
      st = x ^ rkA[r];
    }
  }
  // final round from layout B: SubBytes + ShiftRows (S(x) sits in byte k of T_{(k+2)&3}), the
  // lane keeps byte k of its lookup; the row XOR assembles the column
  uint32_t x = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + __builtin_amdgcn_perm(st, lc, selF)) & fmask;
  x ^= dpp<kRowRor4>(x);
  x ^= dpp<kRowRor8>(x);
  return x ^ rkA[14];
}

// One PRG call (prg.rs:42-73) on a 32-lane half-wave with k_eval16_row's layout: lane p of a
// 16-lane row holds column a = p & 3 of the state; row 0 encrypts A = AES(s), row 1 B = AES(~s)
// with aes256_col16, and v_permlane16_swap hands each row the other's block (rows 2 and 3 repeat
// rows 0 and 1).  A level costs one 16-lane AES chain (~1234 cycles) instead of a lone lane's
// T-table rounds.  Used where a few nodes are on the critical path: the root path and the first
// levels of k_prefix_build16 (kernels16.h).
struct RowPrg {
  uint32_t rkA[15], rkB[15], selA, selB, selF, fmask, lc, a, inv, msk;
  __device__ __forceinline__ void init(const RoundKeys& rk) {
    const uint32_t lane = threadIdx.x & 63u, p = lane & 15u, bq = p >> 2;
    a = p & 3u;
    lc = lane_const();
#pragma unroll
    for (int r = 0; r < 15; ++r) {
      const uint32_t w0 = rk.w[4 * r], w1 = rk.w[4 * r + 1], w2 = rk.w[4 * r + 2], w3 = rk.w[4 * r + 3];
      rkA[r] = (a & 2u) ? ((a & 1u) ? w3 : w2) : ((a & 1u) ? w1 : w0);
      rkB[r] = (bq & 2u) ? ((bq & 1u) ? w3 : w2) : ((bq & 1u) ? w1 : w0);
    }
    const uint32_t kA = (a - bq) & 3u, kB = (bq - a) & 3u;
    selA = col16_sel(kA, kA);
    selB = col16_sel(kB, kB);
    selF = col16_sel(kB, (kB + 2u) & 3u);
    fmask = 0xFFu << (8u * kB);
    inv = 0u - ((lane >> 4) & 1u);
    msk = (a == 3u) ? kMaskLast : 0xFFFFFFFFu;
  }
  // Column a of both children of node (s, v, t) given column a of the level's CW (lib.rs:174-189):
  // left s' = (A ^ s) & M ^ t cw.s, v' = v ^ (B ^ ~s) & M ^ t cw.v; right s' = s & M ^ t cw.s,
  // v' = v ^ ~s & M ^ t cw.v; tl / tr from column 0, broadcast over each quad.
  __device__ __forceinline__ void children(const uint32_t* lds, uint32_t s, uint32_t v, uint32_t t, uint32_t cs,
                                           uint32_t cv, uint32_t ct, uint32_t& sl, uint32_t& vl, uint32_t& tl,
                                           uint32_t& sr, uint32_t& vr, uint32_t& tr) const {
    const uint32_t mine = aes256_col16(s ^ inv, rkA, rkB, lds, lc, selA, selB, selF, fmask);
    const auto sw = __builtin_amdgcn_permlane16_swap(mine, mine, false, false);
    const uint32_t A = sw[0], B = sw[1], tm = 0u - t;
    sl = ((A ^ s) & msk) ^ (tm & cs);
    vl = v ^ ((B ^ ~s) & msk) ^ (tm & cv);
    sr = (s & msk) ^ (tm & cs);
    vr = v ^ (~s & msk) ^ (tm & cv);
    tl = dpp<kQpBcast0>(((A ^ s) & 1u) ^ (t & ct & 1u));          // lib.rs:179-180
    tr = dpp<kQpBcast0>(((B ^ ~s) & 1u) ^ (t & (ct >> 1) & 1u));
  }
};

// The root path of k_prefix_build16: the node of level S named by the bits of w (Msb-first), one
// wave, RowPrg per level (C2's 8 levels took 24 us as lone-lane T-table rounds,
// profiles/r04f_c2_timeline.json).  Returns the node (s, v, t) in every lane.
__device__ __forceinline__ void row_root_path(const uint32_t* lds, const RowPrg& rp, const uint4* __restrict__ cw_s,
                                              const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t,
                                              const uint4 s0, const uint32_t party, const uint32_t S,
                                              const uint32_t w, uint32_t (&rs)[4], uint32_t (&rv)[4], uint32_t& rt) {
  const uint32_t a = rp.a;
  const uint32_t s0w[4] = {s0.x, s0.y, s0.z, s0.w};
  uint32_t s = s0w[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) s = (a == (uint32_t)k) ? s0w[k] : s;
  uint32_t v = 0u, t = party;
  for (uint32_t lev = 0; lev < S; ++lev) {
    const uint32_t cs = reinterpret_cast<const uint32_t*>(cw_s + lev)[a];
    const uint32_t cv = reinterpret_cast<const uint32_t*>(cw_v + lev)[a], ct = cw_t[lev];
    uint32_t sl, vl, tl, sr, vr, tr;
    rp.children(lds, s, v, t, cs, cv, ct, sl, vl, tl, sr, vr, tr);
    const bool right = (w >> (S - 1u - lev)) & 1u;
    s = right ? sr : sl;
    v = right ? vr : vl;
    t = right ? tr : tl;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rs[k] = __builtin_amdgcn_readlane(s, k);
    rv[k] = __builtin_amdgcn_readlane(v, k);
  }
  rt = __builtin_amdgcn_readlane(t, 0);
}

// The 128 KiB replicated T-tables (lds_fill_tables' layout), every load of a thread issued
// before its stores: a latency kernel cannot afford 32 dependent load/store round trips.
constexpr int kFillPer = kLdsWords / kBlock;
__device__ __forceinline__ void lds_fill_load(uint32_t (&v)[kFillPer], const uint32_t* __restrict__ tab) {
#pragma unroll
  for (int i = 0; i < kFillPer; ++i) {
    const int idx = (int)threadIdx.x + i * kBlock;
    const int half = idx >> 14, rem = idx & 16383;
    v[i] = tab[(2 * half + ((rem & 63) >> 5)) * 256 + (rem >> 6)];
  }
}
__device__ __forceinline__ void lds_fill_store(uint32_t* lds, const uint32_t (&v)[kFillPer]) {
#pragma unroll
  for (int i = 0; i < kFillPer; ++i) lds[(int)threadIdx.x + i * kBlock] = v[i];
}
__device__ __forceinline__ void lds_fill_tables_fast(uint32_t* lds, const uint32_t* __restrict__ tab) {
  uint32_t v[kFillPer];
  lds_fill_load(v, tab);
  lds_fill_store(lds, v);
}

__device__ __forceinline__ void col_round_keys(const RoundKeys& rk, uint32_t j, uint32_t (&kw)[15]) {
#pragma unroll
  for (int r = 0; r < 15; ++r) {
    const uint32_t a = rk.w[4 * r], b = rk.w[4 * r + 1], c = rk.w[4 * r + 2], d = rk.w[4 * r + 3];
    kw[r] = (j & 2u) ? ((j & 1u) ? d : c) : ((j & 1u) ? b : a);
  }
}

// Dcf::eval (lib.rs:163-204) of one key at m points, 8 lanes per point: `ppw` points per
// workgroup of kBlock threads (every thread fills the LDS tables; the octets past ppw leave
// after that).  The host spreads a small batch over the CUs (ppw = ceil(m / CUs)): 16 active
// waves on one CU make each round LDS-throughput bound instead of latency bound.  ctr: the
// workspace counter, whose block count (dcf_prg_last_eval_blocks) this engine zeroes (it
// counts none).  cwb / s0 / xs / ys may be host-mapped.
__global__ __launch_bounds__(kBlock, 1) void k_eval16_oct(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint8_t* __restrict__ cwb,
    const uint8_t* __restrict__ s0, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint32_t ppw, const uint64_t m, uint8_t* __restrict__ ys, uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 key[2 * kColMaxLevels + kColMaxLevels / 16 + 2];  // cw_s | cw_v | cw_t | cw_np1
  __shared__ uint8_t xsh[(kBlock / 8) * (kColMaxLevels / 8)];
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<uint4*>(ctr) = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t n = 8u * nbytes;
  const uint64_t p0 = (uint64_t)blockIdx.x * ppw;
  const uint32_t np = (uint32_t)min<uint64_t>(ppw, m - p0);
  // stage the key (single-key CWB, include/dcf_hip.h: 16-byte multiple) and this group's x rows
  const uint32_t np1_off = (2u * n * 16u + n + 15u) & ~15u;
  const uint32_t kq = np1_off / 16u + 1u;
  // every load first (the T-tables from L2, the key and x rows possibly over PCIe from mapped
  // host memory), then every LDS store: one memory latency in the prologue, not three
  uint32_t tv[kFillPer];
  lds_fill_load(tv, tab);
  const bool kl = threadIdx.x < kq, xl = threadIdx.x < np * nbytes;
  const uint4 kv = kl ? reinterpret_cast<const uint4*>(cwb)[threadIdx.x] : make_uint4(0u, 0u, 0u, 0u);
  const uint8_t xv = xl ? xs[p0 * nbytes + threadIdx.x] : (uint8_t)0;
  lds_fill_store(lds, tv);
  if (kl) key[threadIdx.x] = kv;
  if (xl) xsh[threadIdx.x] = xv;
  for (uint32_t i = threadIdx.x + blockDim.x; i < kq; i += blockDim.x) key[i] = reinterpret_cast<const uint4*>(cwb)[i];
  for (uint32_t i = threadIdx.x + blockDim.x; i < np * nbytes; i += blockDim.x) xsh[i] = xs[p0 * nbytes + i];
  __syncthreads();
  DCF_CLK(3, 0);
  const uint32_t lc = lane_const();
  const uint32_t oct = threadIdx.x >> 3, b = (threadIdx.x >> 2) & 1u, j = threadIdx.x & 3u;
  if (oct >= np) return;  // whole octets (and whole quads) leave together: after the only barrier
  uint32_t kw[15];
  col_round_keys(rk, j, kw);
  const uint32_t* kcs = reinterpret_cast<const uint32_t*>(key);             // cw_s[l] word j: kcs[4l + j]
  const uint32_t* kcv = kcs + 4u * n;                                        // cw_v
  const uint8_t* kct = reinterpret_cast<const uint8_t*>(key) + 32u * n;     // cw_t[l]
  const uint32_t np1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(key) + np1_off)[j];
  const uint8_t* x = xsh + oct * nbytes;
  const uint32_t inv = 0u - b;                                      // quad 1 encrypts ~s (B)
  const uint32_t msk = (j == 3u) ? kMaskLast : 0xFFFFFFFFu;         // clear bit 0 of byte 15 (prg.rs:65-68)
  uint32_t s = reinterpret_cast<const uint32_t*>(s0)[j];            // k.s0s[0] (lib.rs:168)
  uint32_t v = 0u, t = party, cur = 0u;
  for (uint32_t lev = 0; lev < n; ++lev) {
    if ((lev & 31u) == 0u) {  // next 32 bits of x, Msb0 (lib.rs:181)
      const uint32_t c = lev >> 5;
      uint32_t wv = 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) wv = (wv << 8) | (4u * c + k < nbytes ? (uint32_t)x[4u * c + k] : 0u);
      cur = wv;
    }
    const uint32_t cs = kcs[4u * lev + j], cv = kcv[4u * lev + j], ct = kct[lev];
    const uint32_t mine = aes256_col(s ^ inv, kw, lds, lc);
    // The other quad's column j.  Both rotations run on every lane, then a bitwise select: a
    // DPP move reads its source lane through EXEC, so it must not sit under a per-lane branch
    // (the compiler turned `b ? dpp(4) : dpp(12)` into one — each side then read 0 from the
    // other quad's disabled lanes).
    uint32_t r4 = dpp<kRowRor4>(mine), r12 = dpp<kRowRor12>(mine);
    asm volatile("" : "+v"(r4), "+v"(r12));
    const uint32_t other = (r4 & inv) | (r12 & ~inv);
    const uint32_t A = (other & inv) | (mine & ~inv), B = (mine & inv) | (other & ~inv);
    const uint32_t xb = cur >> 31;
    cur <<= 1;
    const uint32_t keepA = xb - 1u, tm = 0u - t;
    // t' = lsb(side)[0] ^ t & cw.t(side): column 0 holds byte 0 (lib.rs:179-180, 183/187)
    const uint32_t tl = (A ^ s) & 1u, tr = (B ^ ~s) & 1u;
    const uint32_t tn = dpp<kQpBcast0>((xb ? tr : tl) ^ (t & (ct >> xb) & 1u));
    v ^= ((~s ^ (B & keepA)) & msk) ^ (tm & cv);   // v ^= v_hat(side) ^ t*cw.v   (lib.rs:182/186)
    s = ((s ^ (A & keepA)) & msk) ^ (tm & cs);      // s' = s(side) ^ t*cw.s      (lib.rs:177-178)
    t = tn;
  }
  if (b == 0u)  // y = v ^ s_n ^ t_n*cw_np1 (lib.rs:192), column j of point p0 + oct
    reinterpret_cast<uint32_t*>(ys)[(p0 + oct) * 4u + j] = v ^ s ^ ((0u - t) & np1);
  DCF_CLK(3, 1);
}

// Dcf::eval (lib.rs:163-204) of one key at m points, 32 lanes per point: row 0 (lanes 0-15)
// encrypts A = AES(s), row 1 B = AES(~s), each with aes256_col16; v_permlane16_swap hands
// each row the other's block (gfx950: odd rows of the first operand trade places with even
// rows of the second, so with x in both, the results hold row 0's and row 1's x in every
// lane); every lane then runs the level update for its column (p & 3), t comes from column 0.
// The tiny-batch kernel (auto mode, up to kEvalRowMax points): a lone point's level costs
// one 16-lane AES chain instead of aes256_col's.  `ppw` points per workgroup (<= 32), spread
// over the CUs like k_eval16_oct.  cwb / s0 / xs / ys may be host-mapped.
__global__ __launch_bounds__(kBlock, 1) void k_eval16_row(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint8_t* __restrict__ cwb,
    const uint8_t* __restrict__ s0, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint32_t ppw, const uint64_t m, uint8_t* __restrict__ ys, uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 key[2 * kColMaxLevels + kColMaxLevels / 16 + 2];  // cw_s | cw_v | cw_t | cw_np1
  __shared__ uint8_t xsh[(kBlock / 32) * (kColMaxLevels / 8)];
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<uint4*>(ctr) = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t n = 8u * nbytes;
  const uint64_t p0 = (uint64_t)blockIdx.x * ppw;
  const uint32_t np = (uint32_t)min<uint64_t>(ppw, m - p0);
  const uint32_t np1_off = (2u * n * 16u + n + 15u) & ~15u;
  const uint32_t kq = np1_off / 16u + 1u;
  // every load first, then every LDS store (k_eval16_oct's prologue)
  uint32_t tv[kFillPer];
  lds_fill_load(tv, tab);
  const bool kl = threadIdx.x < kq, xl = threadIdx.x < np * nbytes;
  const uint4 kv = kl ? reinterpret_cast<const uint4*>(cwb)[threadIdx.x] : make_uint4(0u, 0u, 0u, 0u);
  const uint8_t xv = xl ? xs[p0 * nbytes + threadIdx.x] : (uint8_t)0;
  lds_fill_store(lds, tv);
  if (kl) key[threadIdx.x] = kv;
  if (xl) xsh[threadIdx.x] = xv;
  for (uint32_t i = threadIdx.x + blockDim.x; i < kq; i += blockDim.x) key[i] = reinterpret_cast<const uint4*>(cwb)[i];
  __syncthreads();
  DCF_CLK(3, 0);
  const uint32_t lc = lane_const();
  const uint32_t pt = threadIdx.x >> 5, p = threadIdx.x & 15u, a = p & 3u, bq = p >> 2;
  if (pt >= np) return;  // whole points (two whole rows) leave together, after the only barrier
  const uint32_t row = (threadIdx.x >> 4) & 1u;
  // per-lane round-key words and lookup selectors (aes256_col16)
  uint32_t rkA[15], rkB[15];
#pragma unroll
  for (int r = 0; r < 15; ++r) {
    const uint32_t w0 = rk.w[4 * r], w1 = rk.w[4 * r + 1], w2 = rk.w[4 * r + 2], w3 = rk.w[4 * r + 3];
    rkA[r] = (a & 2u) ? ((a & 1u) ? w3 : w2) : ((a & 1u) ? w1 : w0);
    rkB[r] = (bq & 2u) ? ((bq & 1u) ? w3 : w2) : ((bq & 1u) ? w1 : w0);
  }
  const uint32_t kA = (a - bq) & 3u, kB = (bq - a) & 3u;
  const uint32_t selA = col16_sel(kA, kA), selB = col16_sel(kB, kB), selF = col16_sel(kB, (kB + 2u) & 3u);
  const uint32_t fmask = 0xFFu << (8u * kB);
  const uint32_t* kcs = reinterpret_cast<const uint32_t*>(key);             // cw_s[l] word a: kcs[4l + a]
  const uint32_t* kcv = kcs + 4u * n;                                        // cw_v
  const uint8_t* kct = reinterpret_cast<const uint8_t*>(key) + 32u * n;     // cw_t[l]
  const uint32_t np1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(key) + np1_off)[a];
  const uint8_t* x = xsh + pt * nbytes;
  const uint32_t inv = 0u - row;                                    // row 1 encrypts ~s (B)
  const uint32_t msk = (a == 3u) ? kMaskLast : 0xFFFFFFFFu;         // clear bit 0 of byte 15 (prg.rs:65-68)
  uint32_t s = reinterpret_cast<const uint32_t*>(s0)[a];            // k.s0s[0] (lib.rs:168)
  uint32_t v = 0u, t = party, cur = 0u;
  for (uint32_t lev = 0; lev < n; ++lev) {
    if ((lev & 31u) == 0u) {  // next 32 bits of x, Msb0 (lib.rs:181)
      const uint32_t c = lev >> 5;
      uint32_t wv = 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) wv = (wv << 8) | (4u * c + k < nbytes ? (uint32_t)x[4u * c + k] : 0u);
      cur = wv;
    }
    const uint32_t cs = kcs[4u * lev + a], cv = kcv[4u * lev + a], ct = kct[lev];
    const uint32_t mine = aes256_col16(s ^ inv, rkA, rkB, lds, lc, selA, selB, selF, fmask);
    const auto sw = __builtin_amdgcn_permlane16_swap(mine, mine, false, false);
    const uint32_t A = sw[0], B = sw[1];  // row 0's block (A) and row 1's (B), column a, in every lane
    const uint32_t xb = cur >> 31;
    cur <<= 1;
    const uint32_t keepA = xb - 1u, tm = 0u - t;
    // t' = lsb(side)[0] ^ t & cw.t(side): column 0 holds byte 0 (lib.rs:179-180, 183/187)
    const uint32_t tl = (A ^ s) & 1u, tr = (B ^ ~s) & 1u;
    const uint32_t tn = dpp<kQpBcast0>((xb ? tr : tl) ^ (t & (ct >> xb) & 1u));
    v ^= ((~s ^ (B & keepA)) & msk) ^ (tm & cv);   // v ^= v_hat(side) ^ t*cw.v   (lib.rs:182/186)
    s = ((s ^ (A & keepA)) & msk) ^ (tm & cs);      // s' = s(side) ^ t*cw.s      (lib.rs:177-178)
    t = tn;
  }
  if (row == 0u && p < 4u)  // y = v ^ s_n ^ t_n*cw_np1 (lib.rs:192), column a of point p0 + pt
    reinterpret_cast<uint32_t*>(ys)[(p0 + pt) * 4u + a] = v ^ s ^ ((0u - t) & np1);
  DCF_CLK(3, 1);
}

// Dcf::eval (lib.rs:163-204) of one key at m points, one wave (64 lanes) per point, two levels per
// AES chain whenever x goes right.  Rows 0 / 1 encrypt A = AES(s) and B = AES(~s) of level l as in
// k_eval16_row; rows 2 / 3 encrypt the same two blocks of the seed level l + 1 has if x goes right
// at l, s_R = s & M ^ t cw_s[l] (lib.rs:177-178: no AES needed to know it).  Going right, level l
// needs only B (t_R = lsb(B ^ ~s), lib.rs:180), so level l + 1 completes in the same pass from rows 2
// / 3; going left, rows 2 / 3 were speculation.  A lone point takes ~8N / 1.5 chains (~85 at N = 16)
// instead of 8N.  The walk is wave-uniform (one point per wave), so the two-level step is a plain
// branch; `ppw` points per workgroup (<= 16), spread over the CUs like k_eval16_row.
__global__ __launch_bounds__(kBlock, 1) void k_eval16_row2(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint8_t* __restrict__ cwb,
    const uint8_t* __restrict__ s0, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint32_t ppw, const uint64_t m, uint8_t* __restrict__ ys, uint32_t* __restrict__ ctr) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint4 key[2 * kColMaxLevels + kColMaxLevels / 16 + 2];  // cw_s | cw_v | cw_t | cw_np1
  __shared__ uint8_t xsh[(kBlock / 64) * (kColMaxLevels / 8)];
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<uint4*>(ctr) = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t n = 8u * nbytes;
  const uint64_t p0 = (uint64_t)blockIdx.x * ppw;
  const uint32_t np = (uint32_t)min<uint64_t>(ppw, m - p0);
  const uint32_t np1_off = (2u * n * 16u + n + 15u) & ~15u;
  const uint32_t kq = np1_off / 16u + 1u;
  // every load first, then every LDS store (k_eval16_oct's prologue)
  uint32_t tv[kFillPer];
  lds_fill_load(tv, tab);
  const bool kl = threadIdx.x < kq, xl = threadIdx.x < np * nbytes;
  const uint4 kv = kl ? reinterpret_cast<const uint4*>(cwb)[threadIdx.x] : make_uint4(0u, 0u, 0u, 0u);
  const uint8_t xv = xl ? xs[p0 * nbytes + threadIdx.x] : (uint8_t)0;
  lds_fill_store(lds, tv);
  if (kl) key[threadIdx.x] = kv;
  if (xl) xsh[threadIdx.x] = xv;
  for (uint32_t i = threadIdx.x + blockDim.x; i < kq; i += blockDim.x) key[i] = reinterpret_cast<const uint4*>(cwb)[i];
  __syncthreads();
  const uint32_t lc = lane_const();
  const uint32_t pt = threadIdx.x >> 6, p = threadIdx.x & 15u, a = p & 3u, bq = p >> 2;
  if (pt >= np) return;  // whole waves (whole points) leave together, after the only barrier
  const uint32_t q = (threadIdx.x >> 4) & 3u;  // row: 0 A(s), 1 B(~s), 2 A(s_R), 3 B(~s_R)
  uint32_t rkA[15], rkB[15];
#pragma unroll
  for (int r = 0; r < 15; ++r) {
    const uint32_t w0 = rk.w[4 * r], w1 = rk.w[4 * r + 1], w2 = rk.w[4 * r + 2], w3 = rk.w[4 * r + 3];
    rkA[r] = (a & 2u) ? ((a & 1u) ? w3 : w2) : ((a & 1u) ? w1 : w0);
    rkB[r] = (bq & 2u) ? ((bq & 1u) ? w3 : w2) : ((bq & 1u) ? w1 : w0);
  }
  const uint32_t kA = (a - bq) & 3u, kB = (bq - a) & 3u;
  const uint32_t selA = col16_sel(kA, kA), selB = col16_sel(kB, kB), selF = col16_sel(kB, (kB + 2u) & 3u);
  const uint32_t fmask = 0xFFu << (8u * kB);
  const uint32_t* kcs = reinterpret_cast<const uint32_t*>(key);             // cw_s[l] word a: kcs[4l + a]
  const uint32_t* kcv = kcs + 4u * n;                                        // cw_v
  const uint8_t* kct = reinterpret_cast<const uint8_t*>(key) + 32u * n;     // cw_t[l]
  const uint32_t np1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(key) + np1_off)[a];
  // bit l of x, Msb0 (lib.rs:181), from the staged row (wave-uniform: the point is the wave's); read
  // well ahead of its use after the AES chain
  const uint8_t* x = xsh + pt * nbytes;
  auto xbit = [&](uint32_t l) { return ((uint32_t)x[l >> 3] >> (7u - (l & 7u))) & 1u; };
  const uint32_t inv = 0u - (q & 1u);                               // odd rows encrypt ~seed (B)
  const bool spec = (q >> 1) != 0u;                                 // rows 2 / 3: the right successor
  const uint32_t msk = (a == 3u) ? kMaskLast : 0xFFFFFFFFu;         // clear bit 0 of byte 15 (prg.rs:65-68)
  uint32_t s = reinterpret_cast<const uint32_t*>(s0)[a];            // k.s0s[0] (lib.rs:168)
  uint32_t v = 0u, t = party;
  // one level's update from its blocks A, B (column a in every lane): lib.rs:174-189
  auto level = [&](uint32_t lv, uint32_t A, uint32_t B) {
    const uint32_t xb = xbit(lv), cs = kcs[4u * lv + a], cv = kcv[4u * lv + a], ct = kct[lv];
    const uint32_t keepA = xb - 1u, tm = 0u - t;
    const uint32_t tl = (A ^ s) & 1u, tr = (B ^ ~s) & 1u;            // t' = lsb(side)[0] ^ t & cw.t(side)
    const uint32_t tn = dpp<kQpBcast0>((xb ? tr : tl) ^ (t & (ct >> xb) & 1u));
    v ^= ((~s ^ (B & keepA)) & msk) ^ (tm & cv);                     // lib.rs:182/186
    s = ((s ^ (A & keepA)) & msk) ^ (tm & cs);                       // lib.rs:177-178
    t = tn;
  };
  for (uint32_t lev = 0; lev < n;) {
    const uint32_t sR = (s & msk) ^ ((0u - t) & kcs[4u * lev + a]);  // level lev + 1's seed going right
    const uint32_t mine = aes256_col16((spec ? sR : s) ^ inv, rkA, rkB, lds, lc, selA, selB, selF, fmask);
    // rows (0,1) and (2,3) trade, then the wave halves: column a of A, B, A_R, B_R in every lane
    const auto h = __builtin_amdgcn_permlane16_swap(mine, mine, false, false);
    const auto e0 = __builtin_amdgcn_permlane32_swap(h[0], h[0], false, false);  // {A, A_R}
    const auto e1 = __builtin_amdgcn_permlane32_swap(h[1], h[1], false, false);  // {B, B_R}
    const bool right = xbit(lev) != 0u;
    level(lev, e0[0], e1[0]);
    ++lev;
    if (right && lev < n) {  // wave-uniform: s is now s_R, whose blocks rows 2 / 3 encrypted
      level(lev, e0[1], e1[1]);
      ++lev;
    }
  }
  if (q == 0u && p < 4u)  // y = v ^ s_n ^ t_n*cw_np1 (lib.rs:192), column a of point p0 + pt
    reinterpret_cast<uint32_t*>(ys)[(p0 + pt) * 4u + a] = v ^ s ^ ((0u - t) & np1);
}

// Dcf::gen (lib.rs:86-161) of num_keys keys, 16 lanes per key: `kpw` keys per workgroup of
// kBlock threads (spread over the CUs as k_eval16_oct spreads points).  Inputs and the CWB
// output may be host-mapped.
__global__ __launch_bounds__(kBlock, 1) void k_gen16_col(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint8_t* __restrict__ alpha,
    const uint8_t* __restrict__ beta, const uint8_t* __restrict__ s0_0, const uint8_t* __restrict__ s0_1,
    const uint32_t bound, const uint32_t nbytes, const uint32_t kpw, const uint64_t num_keys,
    uint8_t* __restrict__ cw_s, uint8_t* __restrict__ cw_v, uint8_t* __restrict__ cw_t, uint8_t* __restrict__ cw_np1) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint8_t ash[(kBlock / 16) * (kColMaxLevels / 8)];
  const uint32_t n = 8u * nbytes;
  const uint64_t k0 = (uint64_t)blockIdx.x * kpw;
  const uint32_t nk = (uint32_t)min<uint64_t>(kpw, num_keys - k0);
  for (uint32_t i = threadIdx.x; i < nk * nbytes; i += blockDim.x) ash[i] = alpha[k0 * nbytes + i];
  lds_fill_tables_fast(lds, tab);
  __syncthreads();
  const uint32_t lc = lane_const();
  const uint32_t kk = threadIdx.x >> 4, q = (threadIdx.x >> 2) & 3u, j = threadIdx.x & 3u;
  if (kk >= nk) return;  // whole keys (whole DPP rows) leave together, after the only barrier
  const uint64_t k = k0 + kk;
  uint32_t kw[15];
  col_round_keys(rk, j, kw);
  const uint32_t msk = (j == 3u) ? kMaskLast : 0xFFFFFFFFu;
  uint32_t s0w = reinterpret_cast<const uint32_t*>(s0_0)[k * 4u + j];   // s0s[0] (lib.rs:98)
  uint32_t s1w = reinterpret_cast<const uint32_t*>(s0_1)[k * 4u + j];   // s0s[1]
  const uint32_t be = reinterpret_cast<const uint32_t*>(beta)[k * 4u + j];
  uint32_t va = 0u, t0 = 0u, t1 = 1u, cur = 0u;  // lib.rs:99-100
  const uint8_t* al = ash + kk * nbytes;
  const uint32_t inv = 0u - (q & 1u);                  // blocks 1 and 3 encrypt ~s
  const uint32_t rot = q;                               // block q's source lane offsets below
  for (uint32_t lev = 0; lev < n; ++lev) {
    if ((lev & 31u) == 0u) {  // next 32 bits of alpha, Msb0 (lib.rs:106)
      const uint32_t c = lev >> 5;
      uint32_t wv = 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) wv = (wv << 8) | (4u * c + e < nbytes ? (uint32_t)al[4u * c + e] : 0u);
      cur = wv;
    }
    const uint32_t mine = aes256_col(((q >> 1) ? s1w : s0w) ^ inv, kw, lds, lc);
    // column j of every block: row_ror:4n brings block (q - n) & 3
    const uint32_t r4 = dpp<kRowRor4>(mine), r8 = dpp<kRowRor8>(mine), r12 = dpp<kRowRor12>(mine);
    uint32_t X[4];
#pragma unroll
    for (uint32_t tb = 0; tb < 4; ++tb) {
      const uint32_t d = (rot - tb) & 3u;  // block tb sits in the value rotated by 4d lanes
      X[tb] = (d & 2u) ? ((d & 1u) ? r12 : r8) : ((d & 1u) ? r4 : mine);
    }
    const uint32_t A0 = X[0], B0 = X[1], A1 = X[2], B1 = X[3];
    const uint32_t a = cur >> 31;  // alpha_i (lib.rs:106)
    cur <<= 1;
    const uint32_t am = 0u - a;
    const uint32_t bm = (bound == 0u) ? am : ~am;  // LtBeta: beta joins v_cw when alpha_i = 1 (lib.rs:114-125)
    // PRG outputs per party: L = ((A^s)&M, (B^~s)&M), R = (s&M, ~s&M)
    const uint32_t sl0 = (A0 ^ s0w) & msk, vl0 = (B0 ^ ~s0w) & msk, sr0 = s0w & msk, vr0 = ~s0w & msk;
    const uint32_t sl1 = (A1 ^ s1w) & msk, vl1 = (B1 ^ ~s1w) & msk, sr1 = s1w & msk, vr1 = ~s1w & msk;
    const uint32_t scw = (a ? sl0 : sr0) ^ (a ? sl1 : sr1);                       // lib.rs:112
    const uint32_t vcw = (a ? vl0 : vr0) ^ (a ? vl1 : vr1) ^ va ^ (bm & be);      // lib.rs:113-125
    va ^= (a ? vr0 : vl0) ^ (a ? vr1 : vl1) ^ vcw;                                 // lib.rs:126-129
    // t bits from byte 0 (column 0 lanes), broadcast to the quad
    const uint32_t tl0 = (A0 ^ s0w) & 1u, tr0 = (B0 ^ ~s0w) & 1u, tl1 = (A1 ^ s1w) & 1u, tr1 = (B1 ^ ~s1w) & 1u;
    const uint32_t tlcw = tl0 ^ tl1 ^ a ^ 1u, trcw = tr0 ^ tr1 ^ a;  // lib.rs:130-131
    const uint32_t tkcw = a ? trcw : tlcw;
    const uint32_t nt0 = (a ? tr0 : tl0) ^ (t0 & tkcw), nt1 = (a ? tr1 : tl1) ^ (t1 & tkcw);  // lib.rs:149-152
    const uint32_t tp = dpp<kQpBcast0>(tlcw | (trcw << 1) | (nt0 << 2) | (nt1 << 3));
    const uint32_t m0 = 0u - t0, m1 = 0u - t1;
    s0w = (a ? sr0 : sl0) ^ (m0 & scw);  // lib.rs:139-148
    s1w = (a ? sr1 : sl1) ^ (m1 & scw);
    t0 = (tp >> 2) & 1u;
    t1 = (tp >> 3) & 1u;
    const uint64_t ci = (uint64_t)lev * num_keys + k;
    if (q == 0u) reinterpret_cast<uint32_t*>(cw_s)[ci * 4u + j] = scw;
    if (q == 1u) reinterpret_cast<uint32_t*>(cw_v)[ci * 4u + j] = vcw;
    if (q == 2u && j == 0u) cw_t[ci] = (uint8_t)(tp & 3u);
  }
  if (q == 0u) reinterpret_cast<uint32_t*>(cw_np1)[k * 4u + j] = s0w ^ s1w ^ va;  // lib.rs:155
}

// Dcf::gen (lib.rs:86-161) of num_keys keys, one wave per key: row q (16 lanes) encrypts block q
// of the level (A0, B0, A1, B1: prg.rs:42-73 on both parties' seeds, lib.rs:103-104) with
// aes256_col16; v_permlane16_swap then v_permlane32_swap put column p&3 of all four blocks in
// every lane, which runs k_gen16_col's level update (lib.rs:105-152) for its column.  The
// tiny-batch gen (up to kGenRowMax keys), `kpw` keys per workgroup (<= 16).  Inputs and
// the CWB output may be host-mapped.
__global__ __launch_bounds__(kBlock, 1) void k_gen16_row(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint8_t* __restrict__ alpha,
    const uint8_t* __restrict__ beta, const uint8_t* __restrict__ s0_0, const uint8_t* __restrict__ s0_1,
    const uint32_t bound, const uint32_t nbytes, const uint32_t kpw, const uint64_t num_keys,
    uint8_t* __restrict__ cw_s, uint8_t* __restrict__ cw_v, uint8_t* __restrict__ cw_t, uint8_t* __restrict__ cw_np1) {
  __shared__ uint32_t lds[kLdsWords];
  __shared__ uint8_t ash[(kBlock / 64) * (kColMaxLevels / 8)];
  const uint32_t n = 8u * nbytes;
  const uint64_t k0 = (uint64_t)blockIdx.x * kpw;
  const uint32_t nk = (uint32_t)min<uint64_t>(kpw, num_keys - k0);
  uint32_t tv[kFillPer];
  lds_fill_load(tv, tab);
  const bool al = threadIdx.x < nk * nbytes;
  const uint8_t av = al ? alpha[k0 * nbytes + threadIdx.x] : (uint8_t)0;
  lds_fill_store(lds, tv);
  if (al) ash[threadIdx.x] = av;
  __syncthreads();
  const uint32_t lc = lane_const();
  const uint32_t kk = threadIdx.x >> 6, q = (threadIdx.x >> 4) & 3u, p = threadIdx.x & 15u, a = p & 3u, bq = p >> 2;
  if (kk >= nk) return;  // whole keys (whole waves) leave together, after the only barrier
  const uint64_t k = k0 + kk;
  uint32_t rkA[15], rkB[15];
#pragma unroll
  for (int r = 0; r < 15; ++r) {
    const uint32_t w0 = rk.w[4 * r], w1 = rk.w[4 * r + 1], w2 = rk.w[4 * r + 2], w3 = rk.w[4 * r + 3];
    rkA[r] = (a & 2u) ? ((a & 1u) ? w3 : w2) : ((a & 1u) ? w1 : w0);
    rkB[r] = (bq & 2u) ? ((bq & 1u) ? w3 : w2) : ((bq & 1u) ? w1 : w0);
  }
  const uint32_t kA = (a - bq) & 3u, kB = (bq - a) & 3u;
  const uint32_t selA = col16_sel(kA, kA), selB = col16_sel(kB, kB), selF = col16_sel(kB, (kB + 2u) & 3u);
  const uint32_t fmask = 0xFFu << (8u * kB);
  const uint32_t msk = (a == 3u) ? kMaskLast : 0xFFFFFFFFu;
  uint32_t s0w = reinterpret_cast<const uint32_t*>(s0_0)[k * 4u + a];   // s0s[0] (lib.rs:98)
  uint32_t s1w = reinterpret_cast<const uint32_t*>(s0_1)[k * 4u + a];   // s0s[1]
  const uint32_t be = reinterpret_cast<const uint32_t*>(beta)[k * 4u + a];
  uint32_t va = 0u, t0 = 0u, t1 = 1u, cur = 0u;  // lib.rs:99-100
  const uint8_t* alk = ash + kk * nbytes;
  const uint32_t inv = 0u - (q & 1u);            // blocks 1 and 3 encrypt ~s
  // Software-pipelined: a level's AES results feed only s' through scw (lib.rs:112, 139-148);
  // the next level's AES starts right there, and this level's v / t / CW-store work (which the
  // next level needs only after its AES) sits in the same basic block, so the compiler issues it
  // in the lookups' LDS-latency gaps (a lone wave pays issue time for every instruction).  One
  // extra AES runs after the last level.  The CW stores go from every lane (lanes of one column
  // write the same word to the same address) so no branch splits the block.
  auto alpha_word = [&](uint32_t c) {  // 32 bits of alpha from byte 4c, Msb0 (lib.rs:106)
    uint32_t wv = 0u;
#pragma unroll
    for (int e = 0; e < 4; ++e) wv = (wv << 8) | (4u * c + e < nbytes ? (uint32_t)alk[4u * c + e] : 0u);
    return wv;
  };
  cur = alpha_word(0);
  uint32_t mine = aes256_col16(((q >> 1) ? s1w : s0w) ^ inv, rkA, rkB, lds, lc, selA, selB, selF, fmask);
  for (uint32_t lev = 0; lev < n; ++lev) {
    // rows (0,1) and (2,3) trade, then the wave halves: X[q] = column a of block q in every lane
    const auto h = __builtin_amdgcn_permlane16_swap(mine, mine, false, false);  // {even row, odd row} of the pair
    const auto e0 = __builtin_amdgcn_permlane32_swap(h[0], h[0], false, false);  // {A0, A1}
    const auto e1 = __builtin_amdgcn_permlane32_swap(h[1], h[1], false, false);  // {B0, B1}
    const uint32_t A0 = e0[0], A1 = e0[1], B0 = e1[0], B1 = e1[1];
    const uint32_t ab = cur >> 31;  // alpha_i (lib.rs:106)
    // PRG outputs per party: L = ((A^s)&M, (B^~s)&M), R = (s&M, ~s&M)
    const uint32_t sl0 = (A0 ^ s0w) & msk, sr0 = s0w & msk, sl1 = (A1 ^ s1w) & msk, sr1 = s1w & msk;
    const uint32_t scw = (ab ? sl0 : sr0) ^ (ab ? sl1 : sr1);                       // lib.rs:112
    const uint32_t m0 = 0u - t0, m1 = 0u - t1;
    const uint32_t ns0 = (ab ? sr0 : sl0) ^ (m0 & scw);  // lib.rs:139-148
    const uint32_t ns1 = (ab ? sr1 : sl1) ^ (m1 & scw);
    mine = aes256_col16(((q >> 1) ? ns1 : ns0) ^ inv, rkA, rkB, lds, lc, selA, selB, selF, fmask);  // level lev+1
    // --- the rest of level lev, off the chain
    const uint32_t am = 0u - ab;
    const uint32_t bm = (bound == 0u) ? am : ~am;  // LtBeta: beta joins v_cw when alpha_i = 1 (lib.rs:114-125)
    const uint32_t vl0 = (B0 ^ ~s0w) & msk, vr0 = ~s0w & msk, vl1 = (B1 ^ ~s1w) & msk, vr1 = ~s1w & msk;
    const uint32_t vcw = (ab ? vl0 : vr0) ^ (ab ? vl1 : vr1) ^ va ^ (bm & be);      // lib.rs:113-125
    va ^= (ab ? vr0 : vl0) ^ (ab ? vr1 : vl1) ^ vcw;                                 // lib.rs:126-129
    // t bits from byte 0 (column 0 lanes), broadcast to the quad
    const uint32_t tl0 = (A0 ^ s0w) & 1u, tr0 = (B0 ^ ~s0w) & 1u, tl1 = (A1 ^ s1w) & 1u, tr1 = (B1 ^ ~s1w) & 1u;
    const uint32_t tlcw = tl0 ^ tl1 ^ ab ^ 1u, trcw = tr0 ^ tr1 ^ ab;  // lib.rs:130-131
    const uint32_t tkcw = ab ? trcw : tlcw;
    const uint32_t nt0 = (ab ? tr0 : tl0) ^ (t0 & tkcw), nt1 = (ab ? tr1 : tl1) ^ (t1 & tkcw);  // lib.rs:149-152
    const uint32_t tp = dpp<kQpBcast0>(tlcw | (trcw << 1) | (nt0 << 2) | (nt1 << 3));
    t0 = (tp >> 2) & 1u;
    t1 = (tp >> 3) & 1u;
    s0w = ns0;
    s1w = ns1;
    const uint64_t ci = (uint64_t)lev * num_keys + k;
    reinterpret_cast<uint32_t*>(cw_s)[ci * 4u + a] = scw;
    reinterpret_cast<uint32_t*>(cw_v)[ci * 4u + a] = vcw;
    cw_t[ci] = (uint8_t)(tp & 3u);
    cur <<= 1;
    if (((lev + 1u) & 31u) == 0u) cur = alpha_word((lev + 1u) >> 5);
  }
  if (q == 0u && p < 4u) reinterpret_cast<uint32_t*>(cw_np1)[k * 4u + a] = s0w ^ s1w ^ va;  // lib.rs:155
}

}  // namespace
