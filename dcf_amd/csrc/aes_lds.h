// aes_lds.h — AES-256 for gfx950: host key schedule / T-tables and the
// LDS-replicated T-table device rounds.  Included by dcf_hip.hip only.
#pragma once

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

// AES-128 key expansion (FIPS-197 §5.2, Nk = 4): 44 words = 11 round keys.
void aes128_expand_words(const uint8_t key[16], uint32_t w[44]) {
  uint8_t b[176];
  memcpy(b, key, 16);
  uint8_t rcon = 1;
  for (int i = 4; i < 44; i++) {
    uint8_t t[4] = {b[4 * i - 4], b[4 * i - 3], b[4 * i - 2], b[4 * i - 1]};
    if (i % 4 == 0) {
      const uint8_t t0 = t[0];
      t[0] = (uint8_t)(g_sbox[t[1]] ^ rcon);
      t[1] = g_sbox[t[2]];
      t[2] = g_sbox[t[3]];
      t[3] = g_sbox[t0];
      rcon = gmul(rcon, 2);
    }
    for (int k = 0; k < 4; k++) b[4 * i + k] = (uint8_t)(b[4 * (i - 4) + k] ^ t[k]);
  }
  for (int i = 0; i < 44; i++)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
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

#ifndef DCF_T1_BITOP3
#define DCF_T1_BITOP3 1
#endif
// B1: T1 at state byte 1 through the v_bitop3.  Same-box A/Bs, 3 alternating runs (r05s, r05t): C5
// 317.2-317.8 vs 319.0-319.3 and 323.6-324.1 vs 325.3-325.5 ms, C3 492.8-494.5 vs 494.0-494.6 and
// 502.7-504.4 vs 504.1-504.5, C2 3.446-3.452 vs 3.456-3.457 — kept; the λ ≥ 32 head (aes_tt_lka)
// ran 31.21-31.23 vs 30.91-30.97 ms with it, so it keeps the v_perm.
template <int T, int K, bool B1 = true>
__device__ __forceinline__ uint32_t lk(const uint32_t* lds, uint32_t w, uint32_t lc) {
  uint32_t addr;
  if (DCF_T1_BITOP3 && B1 && T == 1 && K == 1) {
    // T1 at state byte 1: the byte already sits at address bits 8..15, so one 2-cycle v_bitop3
    // (w & 0xFF00) | slot builds the address instead of a 4-cycle v_perm (the slot byte is
    // loop-invariant: hoisted once)
    addr = __builtin_amdgcn_bitop3_b32(w, 0xFF00u, (lc >> 8) & 0xFFu, 0xEA);
  } else {
    addr = __builtin_amdgcn_perm(w, lc, Sel<T, K>::v);
  }
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + addr);
}

// DPP quad_perm encodings: lane c reads lane sel[c]; ctrl = sel0 | sel1<<2 | sel2<<4 | sel3<<6
constexpr int kQpRot1 = 1 | (2 << 2) | (3 << 4) | (0 << 6);  // c <- c+1
constexpr int kQpRot2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // c <- c+2
constexpr int kQpRot3 = 3 | (0 << 2) | (1 << 4) | (2 << 6);  // c <- c+3
constexpr int kQpBcast0 = 0;                                   // c <- 0

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

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// 16 bytes at an LDS byte address: ds_read takes the address as is (a generic
// pointer into an extern __shared__ array costs a v_add of the array base per read).
__device__ __forceinline__ uint4 lds_load16(uint32_t a) {
  const u32x4_t v = *(__attribute__((address_space(3))) const u32x4_t*)(size_t)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}

// NB independent AES-NR encryptions, each under the round keys at LDS byte address ka[b]
// (+16 per round: the offset rides in the ds_read_b128 immediate, no address VALU).
// PRE: the caller has XORed round key 0 into st already (into its own input XOR).
// KR > 0: rounds 1 .. KR - 1 take their key from registers instead (rkr[r][c][j]: word j of round r
// of cipher c, c = 1 where the lane's mask hm[b] is all ones), one 3-input pick per word instead of
// a ds_read_b128 (round 0 is the caller's, PRE).
template <int NR, int NB, bool PRE, int KR = 0>
__device__ __forceinline__ void aes_tt_lka(uint32_t (&st)[NB][4], const uint32_t (&ka)[NB], const uint32_t* lds,
                                           uint32_t lc, const uint32_t (*rkr)[2][4] = nullptr,
                                           const uint32_t* hm = nullptr) {
  if (!PRE) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const uint4 k = lds_load16(ka[b]);
      st[b][0] ^= k.x; st[b][1] ^= k.y; st[b][2] ^= k.z; st[b][3] ^= k.w;
    }
  }
#pragma unroll
  for (int r = 1; r <= NR; ++r) {
    uint32_t o[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      uint32_t kw[4];
      if (r < KR) {
#pragma unroll
        for (int j = 0; j < 4; ++j) kw[j] = __builtin_amdgcn_bitop3_b32(hm[b], rkr[r][1][j], rkr[r][0][j], 0xCA);
      } else {
        const uint4 k = lds_load16(ka[b] + 16u * r);
        kw[0] = k.x; kw[1] = k.y; kw[2] = k.z; kw[3] = k.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (r < NR) {
          const uint32_t a = lk<0, 0, false>(lds, st[b][j], lc);
          const uint32_t c = lk<1, 1, false>(lds, st[b][(j + 1) & 3], lc);
          const uint32_t d = lk<2, 2, false>(lds, st[b][(j + 2) & 3], lc);
          const uint32_t e = lk<3, 3, false>(lds, st[b][(j + 3) & 3], lc);
          o[b][j] = xor3(xor3(a, c, d), e, kw[j]);
        } else {  // final round: S(x) sits in byte r of T_{(r+2)&3}
          const uint32_t a = lk<2, 0>(lds, st[b][j], lc);
          const uint32_t c = lk<3, 1>(lds, st[b][(j + 1) & 3], lc);
          const uint32_t d = lk<0, 2>(lds, st[b][(j + 2) & 3], lc);
          const uint32_t e = lk<1, 3>(lds, st[b][(j + 3) & 3], lc);
          o[b][j] = xor3(__builtin_amdgcn_perm(c, a, 0x0c0c0500u), __builtin_amdgcn_perm(e, d, 0x07020c0cu), kw[j]);
        }
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
  }
}

// NB independent AES encryptions with NR rounds (10: AES-128, 14: AES-256), each
// under its own key schedule read from LDS: rk[b] points at NR + 1 uint4 round
// keys (per lane, so a lane may pick its schedule; lanes reading the same
// schedule broadcast).
// LATE_KEYS: each round's key read waits (through an empty asm) for the previous
// round's state, so the compiler cannot hoist all the key reads up front (for
// kernels that are short of VGPRs; costs one v_add per round and block).
template <int NR, int NB, bool LATE_KEYS = false>
__device__ __forceinline__ void aes_tt_lk(uint32_t (&st)[NB][4], const uint4* const (&rk)[NB], const uint32_t* lds,
                                          uint32_t lc) {
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint4 k = rk[b][0];
    st[b][0] ^= k.x; st[b][1] ^= k.y; st[b][2] ^= k.z; st[b][3] ^= k.w;
  }
#pragma unroll
  for (int r = 1; r < NR; ++r) {
    uint32_t o[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      uint32_t z = 0u;
      if (LATE_KEYS) asm volatile("" : "+v"(z) : "v"(st[b][0]));
      const uint4 k = rk[b][r + z];
      const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t a = lk<0, 0>(lds, st[b][j], lc);
        const uint32_t c = lk<1, 1>(lds, st[b][(j + 1) & 3], lc);
        const uint32_t d = lk<2, 2>(lds, st[b][(j + 2) & 3], lc);
        const uint32_t e = lk<3, 3>(lds, st[b][(j + 3) & 3], lc);
        o[b][j] = xor3(xor3(a, c, d), e, kw[j]);
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
  }
  uint32_t o[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint4 k = rk[b][NR];
    const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t a = lk<2, 0>(lds, st[b][j], lc);
      const uint32_t c = lk<3, 1>(lds, st[b][(j + 1) & 3], lc);
      const uint32_t d = lk<0, 2>(lds, st[b][(j + 2) & 3], lc);
      const uint32_t e = lk<1, 3>(lds, st[b][(j + 3) & 3], lc);
      const uint32_t lo = __builtin_amdgcn_perm(c, a, 0x0c0c0500u);
      const uint32_t hi = __builtin_amdgcn_perm(e, d, 0x07020c0cu);
      o[b][j] = xor3(lo, hi, kw[j]);
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
}

// AES-256 with round keys read per round from a device copy of the schedule (one
// uniform global_load_dwordx4 per round, shared by the NB blocks).  The load
// address is base + zb + 16 r, where zb is a zero that an empty asm "redefines"
// after the previous round's state, so the compiler can neither hoist the
// 15 loads into 60 live registers nor needs any VALU to form the address.
// PRE: the caller has already XORed round key 0 into st (folded into its own input XOR).
template <int NB, bool PRE = false>
__device__ __forceinline__ void aes256_tt_gk(uint32_t (&st)[NB][4], const uint4* __restrict__ rkg,
                                             const uint32_t* lds, uint32_t lc) {
  const char* base = reinterpret_cast<const char*>(rkg);
  uint32_t zb = 0u;
  if (!PRE) {
    const uint4 k = *reinterpret_cast<const uint4*>(base);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      st[b][0] ^= k.x; st[b][1] ^= k.y; st[b][2] ^= k.z; st[b][3] ^= k.w;
    }
  }
  // rounds between a key's load and its use (r01o A/B on C3: 1 -1.2 %, 2 +2.2 %, 3 +3.6 %, 4 +3.1 %,
  // 6 -12 % vs SGPR keys)
  constexpr int AH = 3;
  uint4 kq[AH];
#pragma unroll
  for (int q = 0; q < AH - 1; ++q) kq[q] = *reinterpret_cast<const uint4*>(base + 16 * (q + 1));
#pragma unroll
  for (int r = 1; r < 15; ++r) {
    asm volatile("" : "+v"(zb) : "v"(st[0][0]), "v"(st[NB - 1][0]));
    const int rn = r + AH - 1;  // the round whose key is loaded now
    if (rn < 15) kq[(rn - 1) % AH] = *reinterpret_cast<const uint4*>(base + zb + 16 * rn);
    const uint4 k = kq[(r - 1) % AH];
    const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
    uint32_t o[NB][4];
    if (r < 14) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t a = lk<0, 0>(lds, st[b][j], lc);
          const uint32_t c = lk<1, 1>(lds, st[b][(j + 1) & 3], lc);
          const uint32_t d = lk<2, 2>(lds, st[b][(j + 2) & 3], lc);
          const uint32_t e = lk<3, 3>(lds, st[b][(j + 3) & 3], lc);
          o[b][j] = xor3(xor3(a, c, d), e, kw[j]);
        }
    } else {
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
          o[b][j] = xor3(lo, hi, kw[j]);
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
  }
}

template <int NB>
__device__ __forceinline__ void aes128_tt(uint32_t (&st)[NB][4], const uint4* const (&rk)[NB], const uint32_t* lds,
                                          uint32_t lc) {
  aes_tt_lk<10, NB>(st, rk, lds, lc);
}

// In-kernel clock probe (diagnostic builds only, -DDCF_CLOCK_STAMPS; MI355X_MICROARCH.md "DVFS
// give-back" item 6): lane 0 of workgroup w stamps the shader-clock counter (s_memtime) and the
// 100 MHz real-time counter (s_memrealtime) when its work starts and ends; the engine clock is
// the ratio of the deltas x 100 MHz.  The stamps go to a buffer of their own by plain vector
// stores (dcf_debug_clock_stamps reads them back); no output is computed from them.
#ifdef DCF_CLOCK_STAMPS
constexpr uint32_t kClkSlots = 8, kClkGroups = 4096;
__device__ unsigned long long g_clk_stamps[kClkSlots * kClkGroups * 4];
__device__ __forceinline__ void clk_stamp(uint32_t slot, uint32_t phase) {
  const uint32_t wg = blockIdx.x + gridDim.x * blockIdx.y;
  if (threadIdx.x == 0 && wg < kClkGroups) {
    const unsigned long long t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o = g_clk_stamps + ((size_t)slot * kClkGroups + wg) * 4 + 2 * phase;
    __hip_atomic_store(o, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(o + 1, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
#define DCF_CLK(slot, phase) clk_stamp(slot, phase)
#else
#define DCF_CLK(slot, phase)
#endif

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

}  // namespace
