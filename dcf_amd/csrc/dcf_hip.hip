// dcf_hip.hip — MI355X (gfx950, CDNA4) DCF evaluator: HIP kernels + C ABI.
//
// Replaces the hot path of the `dcf` crate (xymeng16/dcf v0.2.2):
//   DcfImpl::eval  (lib.rs:163-204)   -> k_eval16 (one lane per (key, point))
//   DcfImpl::gen   (lib.rs:86-161)    -> k_gen16  (one lane per key, batched)
//   Aes256HirosePrg::gen (prg.rs:42-73) inlined into both (hirose16)
// The C ABI is declared in include/dcf_hip.h.  No CPU fallback: every compute
// entry point runs a kernel or returns an error.
//
// AES-256 on CDNA4 (no AES instructions): T-table rounds with the four 1 KiB
// tables replicated 32 ways in LDS so that lane l of every 32-lane half-wave
// always reads bank l (ds_read_b32 banks are (addr/4) mod 32 per half-wave,
// MI355X_MICROARCH.md §LDS) — conflict-free for any data.  Layout (128 KiB):
//   addr(T, b, lane) = (T>>1)*64K + b*256 + (T&1)*128 + (lane&31)*4
// so one v_perm_b32 builds the address from the state byte and a per-lane
// constant: byte0 = lane slot (T even: (l&31)*4, T odd: 128+(l&31)*4),
// byte1 = state byte b, byte2 = 64K half select.  One VALU op + one LDS read
// per lookup; 16 lookups per round.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "dcf_hip.h"

#define DCF_VERSION "dcf_amd 0.1.0 (gfx950)"

namespace {

// ------------------------------------------------------------------------
// Host-side AES-256 material (key schedule + T-tables), derived from the
// GF(2^8) definition.  State words are little-endian columns: word j holds
// bytes 4j..4j+3 = rows 0..3 of column j.
// ------------------------------------------------------------------------
uint8_t g_sbox[256];
uint32_t g_tab[4 * 256];  // T0..T3, LE
std::once_flag g_aes_once;

uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  for (; b; b >>= 1) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
  }
  return r;
}

void aes_init_tables() {
  // log/antilog over generator 3 gives inverses without exponentiation.
  uint8_t exp_t[256], log_t[256] = {0};
  uint8_t x = 1;
  for (int i = 0; i < 255; i++) {
    exp_t[i] = x;
    log_t[x] = (uint8_t)i;
    x = gmul(x, 3);
  }
  for (int v = 0; v < 256; v++) {
    uint8_t inv = v ? exp_t[(255 - log_t[v]) % 255] : 0;
    uint8_t s = inv;
    for (int k = 1; k <= 4; k++) s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    g_sbox[v] = (uint8_t)(s ^ 0x63);
  }
  for (int v = 0; v < 256; v++) {
    uint32_t s = g_sbox[v], s2 = gmul((uint8_t)s, 2), s3 = gmul((uint8_t)s, 3);
    uint32_t t0 = s2 | (s << 8) | (s << 16) | (s3 << 24);  // MixColumns column (2,1,1,3)
    for (int t = 0; t < 4; t++) g_tab[t * 256 + v] = t ? ((t0 << (8 * t)) | (t0 >> (32 - 8 * t))) : t0;
  }
}

struct RoundKeys {
  uint32_t w[60];
};

void aes256_expand_words(const uint8_t key[32], RoundKeys* rk) {
  uint8_t b[240];
  memcpy(b, key, 32);
  uint8_t rcon = 1;
  for (int i = 8; i < 60; i++) {
    uint8_t t[4] = {b[4 * i - 4], b[4 * i - 3], b[4 * i - 2], b[4 * i - 1]};
    if (i % 8 == 0) {
      uint8_t t0 = t[0];
      t[0] = (uint8_t)(g_sbox[t[1]] ^ rcon);
      t[1] = g_sbox[t[2]];
      t[2] = g_sbox[t[3]];
      t[3] = g_sbox[t0];
      rcon = gmul(rcon, 2);
    } else if (i % 8 == 4) {
      for (auto& c : t) c = g_sbox[c];
    }
    for (int k = 0; k < 4; k++) b[4 * i + k] = (uint8_t)(b[4 * (i - 8) + k] ^ t[k]);
  }
  for (int i = 0; i < 60; i++)
    rk->w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
               ((uint32_t)b[4 * i + 3] << 24);
}

// ------------------------------------------------------------------------
// Device: LDS T-tables and AES-256
// ------------------------------------------------------------------------
constexpr int kLdsWords = 32768;  // 128 KiB
constexpr int kBlock = 1024;      // 16 waves; one workgroup per CU (LDS-limited)
constexpr uint32_t kMaskLast = 0xFEFFFFFFu;  // clear Lsb0 bit 0 of byte 15 (prg.rs:65-68)

__device__ __forceinline__ void lds_fill_tables(uint32_t* lds, const uint32_t* __restrict__ tab) {
  for (int idx = threadIdx.x; idx < kLdsWords; idx += blockDim.x) {
    const int half = idx >> 14, rem = idx & 16383;
    const int b = rem >> 6, slot = rem & 63;
    lds[idx] = tab[(2 * half + (slot >> 5)) * 256 + b];
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t lane_const() {
  const uint32_t l = (threadIdx.x & 31u) * 4u;
  return l | ((128u + l) << 8) | (1u << 16);
}

// perm selector: byte0 <- lane-const byte (T&1), byte1 <- state byte K,
// byte2 <- half select (T>>1) or zero, byte3 <- zero.
template <int T, int K>
struct Sel {
  static constexpr uint32_t v =
      ((T & 1) ? 1u : 0u) | ((4u + K) << 8) | (((T >> 1) ? 2u : 0x0cu) << 16) | (0x0cu << 24);
};

template <int T, int K>
__device__ __forceinline__ uint32_t lk(const uint32_t* lds, uint32_t w, uint32_t lc) {
  const uint32_t addr = __builtin_amdgcn_perm(w, lc, Sel<T, K>::v);
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + addr);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// NB independent AES-256 encryptions under one key schedule (FIPS-197),
// interleaved for ILP.  st holds LE column words.
template <int NB>
__device__ __forceinline__ void aes256_tt(uint32_t (&st)[NB][4], const RoundKeys& rk, const uint32_t* lds,
                                          uint32_t lc) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) st[b][j] ^= rk.w[j];
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    uint32_t o[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t a = lk<0, 0>(lds, st[b][j], lc);
        const uint32_t c = lk<1, 1>(lds, st[b][(j + 1) & 3], lc);
        const uint32_t d = lk<2, 2>(lds, st[b][(j + 2) & 3], lc);
        const uint32_t e = lk<3, 3>(lds, st[b][(j + 3) & 3], lc);
        o[b][j] = xor3(xor3(a, c, d), e, rk.w[4 * r + j]);
      }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
  }
  // Final round: SubBytes+ShiftRows+AddRoundKey.  S(x) sits in byte r of T_{(r+2)&3}.
  uint32_t o[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t a = lk<2, 0>(lds, st[b][j], lc);
      const uint32_t c = lk<3, 1>(lds, st[b][(j + 1) & 3], lc);
      const uint32_t d = lk<0, 2>(lds, st[b][(j + 2) & 3], lc);
      const uint32_t e = lk<1, 3>(lds, st[b][(j + 3) & 3], lc);
      const uint32_t lo = __builtin_amdgcn_perm(c, a, 0x0c0c0500u);
      const uint32_t hi = __builtin_amdgcn_perm(e, d, 0x07020c0cu);
      o[b][j] = xor3(lo, hi, rk.w[56 + j]);
    }
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }

// 32 bits of a byte string starting at byte 4c, Msb0 order (lib.rs:106,181),
// zero-padded past nbytes.
__device__ __forceinline__ uint32_t load_bits32(const uint8_t* __restrict__ p, uint32_t c, uint32_t nbytes) {
  if ((nbytes & 3u) == 0) return bswap32(*reinterpret_cast<const uint32_t*>(p + 4 * c));
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t idx = 4 * c + k;
    w = (w << 8) | (idx < nbytes ? (uint32_t)p[idx] : 0u);
  }
  return w;
}

// ------------------------------------------------------------------------
// k_eval16: DcfImpl::eval (lib.rs:163-204) at LAMBDA = 16.
//   MODE 0: one key.  MODE 1: K keys, points_per_key % 64 == 0 (key is
//   wave-uniform -> scalar CW loads).  MODE 2: K keys, any points_per_key.
// The Hirose PRG at LAMBDA = 16 (prg.rs:42-73 with the diagonal zip):
//   A = AES_K0(s), B = AES_K0(~s), M = clear bit0 of byte 15
//   L = ((A^s)&M, (B^~s)&M, lsb(A^s)[0]),  R = (s&M, ~s&M, lsb(B^~s)[0])
// ------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock, 1) void k_eval16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint4* __restrict__ cw_s,
    const uint4* __restrict__ cw_v, const uint8_t* __restrict__ cw_t, const uint4* __restrict__ cw_np1,
    const uint4* __restrict__ s0s, const uint32_t party, const uint8_t* __restrict__ xs, const uint32_t nbytes,
    const uint64_t num_keys, const uint64_t points_per_key, uint4* __restrict__ ys) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint64_t total = num_keys * points_per_key;
  const uint32_t nlev = 8u * nbytes;
  const uint32_t nchunk = (nbytes + 3u) >> 2;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < total; base += stride) {
    const uint64_t g = base + (threadIdx.x & 63u);
    const bool live = g < total;
    const uint64_t gg = live ? g : total - 1;
    uint64_t key = 0;
    if (MODE == 1) key = __builtin_amdgcn_readfirstlane((uint32_t)(gg / points_per_key));
    if (MODE == 2) key = gg / points_per_key;
    const uint4 sv = s0s[key];
    uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
    uint32_t v[4] = {0u, 0u, 0u, 0u};
    uint32_t t = party;
    const uint8_t* x = xs + gg * nbytes;
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
        aes256_tt<2>(st, rk, lds, lc);  // st[0] = A, st[1] = B
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
    const uint4 np = cw_np1[key];
    const uint32_t tm = 0u - t;
    if (live) {
      uint4 y;
      y.x = v[0] ^ s[0] ^ (tm & np.x);
      y.y = v[1] ^ s[1] ^ (tm & np.y);
      y.z = v[2] ^ s[2] ^ (tm & np.z);
      y.w = v[3] ^ s[3] ^ (tm & np.w);
      ys[g] = y;
    }
  }
}

// ------------------------------------------------------------------------
// k_gen16: DcfImpl::gen (lib.rs:86-161) at LAMBDA = 16, one lane per key.
// Four AES blocks per level (PRG on both parties' seeds, lib.rs:103-104).
// ------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock, 1) void k_gen16(
    const uint32_t* __restrict__ tab, const RoundKeys rk, const uint8_t* __restrict__ alpha,
    const uint4* __restrict__ beta, const uint4* __restrict__ s0_0, const uint4* __restrict__ s0_1,
    const uint32_t bound, const uint32_t nbytes, const uint64_t num_keys, uint4* __restrict__ cw_s,
    uint4* __restrict__ cw_v, uint8_t* __restrict__ cw_t, uint4* __restrict__ cw_np1) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint32_t nlev = 8u * nbytes;
  const uint32_t nchunk = (nbytes + 3u) >> 2;
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
    uint32_t lev = 0;
    for (uint32_t c = 0; c < nchunk; ++c) {
      uint32_t cur = load_bits32(al, c, nbytes);
      const uint32_t lend = min(32u, nlev - 32u * c);
      for (uint32_t b = 0; b < lend; ++b, ++lev) {
        uint32_t st[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          st[0][j] = s[0][j];
          st[1][j] = ~s[0][j];
          st[2][j] = s[1][j];
          st[3][j] = ~s[1][j];
        }
        aes256_tt<4>(st, rk, lds, lc);  // A0, B0, A1, B1
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
        if (live) {
          const uint64_t ci = (uint64_t)lev * num_keys + k;
          cw_s[ci] = make_uint4(scw[0], scw[1], scw[2], scw[3]);
          cw_v[ci] = make_uint4(vcw[0], vcw[1], vcw[2], vcw[3]);
          cw_t[ci] = (uint8_t)(tlcw | (trcw << 1));
        }
      }
    }
    if (live)  // lib.rs:155
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

// ------------------------------------------------------------------------
// Host plumbing
// ------------------------------------------------------------------------
thread_local std::string t_err;

int fail(int code, const std::string& msg) {
  t_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(DCF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) return;
    ok = (prev == dev) || (hipSetDevice(dev) == hipSuccess);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (ok && hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

uint64_t grid_for(uint64_t work_items, int cus) {
  uint64_t blocks = (work_items + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)cus;  // one 128 KiB-LDS workgroup per CU, persistent loop
  if (blocks > cap) blocks = cap;
  return blocks ? blocks : 1;
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) { return hipMalloc(&p, n ? n : 1); }
};

}  // namespace

struct dcf_prg {
  int device = 0;
  int cus = 256;
  size_t lambda = 0;
  size_t cipher_n = 0;
  std::vector<RoundKeys> rk;  // Aes256::new per key (prg.rs:28-31)
  uint32_t* d_tab = nullptr;  // T0..T3 (4 KiB) on the device
};

extern "C" {

const char* dcf_version(void) { return DCF_VERSION; }

const char* dcf_last_error(void) { return t_err.c_str(); }

size_t dcf_cwb_np1_offset(size_t n_bytes, size_t lambda, size_t num_keys) {
  const size_t n = 8 * n_bytes;
  return ((2 * n * num_keys * lambda + n * num_keys) + 15) & ~(size_t)15;
}

size_t dcf_cwb_bytes(size_t n_bytes, size_t lambda, size_t num_keys) {
  return dcf_cwb_np1_offset(n_bytes, lambda, num_keys) + num_keys * lambda;
}

int dcf_hirose_prg_new(const uint8_t* keys, size_t cipher_n, size_t lambda, int device, dcf_prg** out) {
  if (!keys || !out) return fail(DCF_ERR_ARG, "null argument");
  *out = nullptr;
  if (lambda == 0 || lambda % 16 != 0) return fail(DCF_ERR_LAMBDA, "lambda must be a positive multiple of 16");
  const size_t need = (lambda / 16 >= 2) ? 18 : 1;
  if (cipher_n < need)
    return fail(DCF_ERR_CIPHER_N, "cipher_n too small: the Hirose PRG reads ciphers[i*16+j] (prg.rs:51)");
  std::call_once(g_aes_once, aes_init_tables);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(DCF_ERR_ARG, "bad device ordinal");
  DeviceGuard dg(device);
  if (!dg.ok) return fail(DCF_ERR_HIP, "hipSetDevice failed");
  dcf_prg* p = new dcf_prg();
  p->device = device;
  p->lambda = lambda;
  p->cipher_n = cipher_n;
  p->rk.resize(cipher_n);
  for (size_t i = 0; i < cipher_n; i++) aes256_expand_words(keys + 32 * i, &p->rk[i]);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    p->cus = prop.multiProcessorCount;
  hipError_t e = hipMalloc(&p->d_tab, sizeof(g_tab));
  if (e == hipSuccess) e = hipMemcpy(p->d_tab, g_tab, sizeof(g_tab), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (p->d_tab) (void)hipFree(p->d_tab);
    delete p;
    return fail(DCF_ERR_HIP, std::string("table upload: ") + hipGetErrorString(e));
  }
  *out = p;
  return DCF_OK;
}

void dcf_prg_free(dcf_prg* p) {
  if (!p) return;
  {
    DeviceGuard dg(p->device);
    if (p->d_tab) (void)hipFree(p->d_tab);
  }
  delete p;
}

size_t dcf_prg_lambda(const dcf_prg* p) { return p ? p->lambda : 0; }

int dcf_gen_batch_device(dcf_prg* p, size_t n_bytes, size_t num_keys, const uint8_t* alpha, const uint8_t* beta,
                         const uint8_t* s0_0, const uint8_t* s0_1, int bound, uint8_t* cwb_out, void* stream) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (bound != DCF_BOUND_LT_BETA && bound != DCF_BOUND_GT_BETA) return fail(DCF_ERR_ARG, "bad bound");
  if (num_keys == 0) return DCF_OK;
  if (!alpha || !beta || !s0_0 || !s0_1 || !cwb_out) return fail(DCF_ERR_ARG, "null buffer");
  if (p->lambda != 16) return fail(DCF_ERR_UNSUPPORTED, "batched gen implemented for lambda = 16");
  DeviceGuard dg(p->device);
  const size_t n = 8 * n_bytes, lam = p->lambda;
  uint8_t* cws = cwb_out;
  uint8_t* cwv = cwb_out + n * num_keys * lam;
  uint8_t* cwt = cwb_out + 2 * n * num_keys * lam;
  uint8_t* np1 = cwb_out + dcf_cwb_np1_offset(n_bytes, lam, num_keys);
  hipLaunchKernelGGL(k_gen16, dim3((unsigned)grid_for(num_keys, p->cus)), dim3(kBlock), 0, (hipStream_t)stream,
                     p->d_tab, p->rk[0], alpha, (const uint4*)beta, (const uint4*)s0_0, (const uint4*)s0_1,
                     (uint32_t)bound, (uint32_t)n_bytes, (uint64_t)num_keys, (uint4*)cws, (uint4*)cwv, cwt,
                     (uint4*)np1);
  HIP_TRY(hipGetLastError());
  return DCF_OK;
}

static int eval_launch(dcf_prg* p, size_t n_bytes, size_t num_keys, size_t ppk, int party, const uint8_t* cwb,
                       const uint8_t* s0s, const uint8_t* xs, uint8_t* ys, void* stream) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  if (party != 0 && party != 1) return fail(DCF_ERR_ARG, "party must be 0 or 1");
  const uint64_t total = (uint64_t)num_keys * ppk;
  if (total == 0) return DCF_OK;
  if (!cwb || !s0s || !xs || !ys) return fail(DCF_ERR_ARG, "null buffer");
  if (p->lambda != 16) return fail(DCF_ERR_UNSUPPORTED, "eval kernels implemented for lambda = 16");
  DeviceGuard dg(p->device);
  const size_t n = 8 * n_bytes, lam = p->lambda;
  const uint4* cws = (const uint4*)cwb;
  const uint4* cwv = (const uint4*)(cwb + n * num_keys * lam);
  const uint8_t* cwt = cwb + 2 * n * num_keys * lam;
  const uint4* np1 = (const uint4*)(cwb + dcf_cwb_np1_offset(n_bytes, lam, num_keys));
  const dim3 grid((unsigned)grid_for(total, p->cus)), block(kBlock);
  hipStream_t st = (hipStream_t)stream;
  if (num_keys == 1)
    hipLaunchKernelGGL(k_eval16<0>, grid, block, 0, st, p->d_tab, p->rk[0], cws, cwv, cwt, np1,
                       (const uint4*)s0s, (uint32_t)party, xs, (uint32_t)n_bytes, (uint64_t)1, (uint64_t)ppk,
                       (uint4*)ys);
  else if (ppk % 64 == 0)
    hipLaunchKernelGGL(k_eval16<1>, grid, block, 0, st, p->d_tab, p->rk[0], cws, cwv, cwt, np1,
                       (const uint4*)s0s, (uint32_t)party, xs, (uint32_t)n_bytes, (uint64_t)num_keys,
                       (uint64_t)ppk, (uint4*)ys);
  else
    hipLaunchKernelGGL(k_eval16<2>, grid, block, 0, st, p->d_tab, p->rk[0], cws, cwv, cwt, np1,
                       (const uint4*)s0s, (uint32_t)party, xs, (uint32_t)n_bytes, (uint64_t)num_keys,
                       (uint64_t)ppk, (uint4*)ys);
  HIP_TRY(hipGetLastError());
  return DCF_OK;
}

int dcf_eval_device(dcf_prg* p, size_t n_bytes, int party, const uint8_t* cwb, const uint8_t* s0,
                    const uint8_t* xs, size_t m, uint8_t* ys, void* stream) {
  return eval_launch(p, n_bytes, 1, m, party, cwb, s0, xs, ys, stream);
}

int dcf_eval_multikey_device(dcf_prg* p, size_t n_bytes, size_t num_keys, size_t points_per_key, int party,
                             const uint8_t* cwb, const uint8_t* s0s, const uint8_t* xs, uint8_t* ys,
                             void* stream) {
  return eval_launch(p, n_bytes, num_keys, points_per_key, party, cwb, s0s, xs, ys, stream);
}

int dcf_gen(dcf_prg* p, size_t n_bytes, const uint8_t* alpha, const uint8_t* beta, const uint8_t* s0_0,
            const uint8_t* s0_1, int bound, uint8_t* cwb_out) {
  if (!p || !alpha || !beta || !s0_0 || !s0_1 || !cwb_out) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  const size_t lam = p->lambda, cwb_len = dcf_cwb_bytes(n_bytes, lam, 1);
  DeviceGuard dg(p->device);
  DevBuf a, b, s0, s1, out;
  HIP_TRY(a.alloc(n_bytes));
  HIP_TRY(b.alloc(lam));
  HIP_TRY(s0.alloc(lam));
  HIP_TRY(s1.alloc(lam));
  HIP_TRY(out.alloc(cwb_len));
  HIP_TRY(hipMemcpy(a.p, alpha, n_bytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(b.p, beta, lam, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s0.p, s0_0, lam, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s1.p, s0_1, lam, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(out.p, 0, cwb_len));
  int rc = dcf_gen_batch_device(p, n_bytes, 1, (const uint8_t*)a.p, (const uint8_t*)b.p, (const uint8_t*)s0.p,
                                (const uint8_t*)s1.p, bound, (uint8_t*)out.p, nullptr);
  if (rc) return rc;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(cwb_out, out.p, cwb_len, hipMemcpyDeviceToHost));
  return DCF_OK;
}

int dcf_eval(dcf_prg* p, size_t n_bytes, int party, const uint8_t* cwb, size_t cwb_len, const uint8_t* s0,
             const uint8_t* xs, size_t m, uint8_t* ys, size_t ys_len) {
  if (!p || !cwb || !s0) return fail(DCF_ERR_ARG, "null argument");
  if (n_bytes == 0) return fail(DCF_ERR_N, "n_bytes must be > 0");
  const size_t lam = p->lambda;
  if (cwb_len != dcf_cwb_bytes(n_bytes, lam, 1))
    return fail(DCF_ERR_KEY, "key size does not match 8*N levels (lib.rs:165)");
  if (ys_len != m * lam) return fail(DCF_ERR_LEN, "ys length != m * lambda");
  if (m == 0) return DCF_OK;
  if (!xs || !ys) return fail(DCF_ERR_ARG, "null buffer");
  DeviceGuard dg(p->device);
  DevBuf k, s, x, y;
  HIP_TRY(k.alloc(cwb_len));
  HIP_TRY(s.alloc(lam));
  HIP_TRY(x.alloc(m * n_bytes));
  HIP_TRY(y.alloc(m * lam));
  HIP_TRY(hipMemcpy(k.p, cwb, cwb_len, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.p, s0, lam, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(x.p, xs, m * n_bytes, hipMemcpyHostToDevice));
  int rc = dcf_eval_device(p, n_bytes, party, (const uint8_t*)k.p, (const uint8_t*)s.p, (const uint8_t*)x.p, m,
                           (uint8_t*)y.p, nullptr);
  if (rc) return rc;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(ys, y.p, m * lam, hipMemcpyDeviceToHost));
  return DCF_OK;
}

int dcf_prg_gen(dcf_prg* p, const uint8_t* seeds, size_t m, uint8_t* out) {
  if (!p) return fail(DCF_ERR_ARG, "null prg");
  if (m == 0) return DCF_OK;
  if (!seeds || !out) return fail(DCF_ERR_ARG, "null buffer");
  if (p->lambda != 16) return fail(DCF_ERR_UNSUPPORTED, "PRG test hook implemented for lambda = 16");
  DeviceGuard dg(p->device);
  const size_t lam = p->lambda, row = 4 * lam + 2;
  DevBuf s, o;
  HIP_TRY(s.alloc(m * lam));
  HIP_TRY(o.alloc(m * row));
  HIP_TRY(hipMemcpy(s.p, seeds, m * lam, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_prg16, dim3((unsigned)grid_for(m, p->cus)), dim3(kBlock), 0, nullptr, p->d_tab, p->rk[0],
                     (const uint4*)s.p, (uint64_t)m, (uint8_t*)o.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, o.p, m * row, hipMemcpyDeviceToHost));
  return DCF_OK;
}

}  // extern "C"
