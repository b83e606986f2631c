// Micro-benchmark: dependent-chain latencies of ONE wave alone on a CU (the single-point
// eval's regime, kernels_lat.h): cycles per dependent ds_read_b32, per dependent VALU, per
// dependent DPP-xor, and per AES-256 block in the lane-quad column form (aes256_col) and in
// the whole-block-per-lane form (aes256_tt<1>).  s_memtime clocks around the chain.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/micro/lat_chain.hip -o scripts/micro/lat_chain
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include "../../dcf_amd/csrc/aes_lds.h"
#include "../../dcf_amd/csrc/kernels_lat.h"

// AES-256 with a block on 16 lanes, ONE lookup per lane and round: lane p (of its row) holds
// column p&3 (layout A) or p>>2 (layout B) of the state; from A, lane p computes the term
// T_k[byte k of its column] of output column j = p>>2 (k = (p&3) - j), the quad's XOR is
// column j (layout B); from B the roles transpose and a stride-4 XOR over the row (row_ror 4,
// 8) gives layout A.  7 instructions per round instead of 18.
__device__ __forceinline__ uint32_t sel_for(uint32_t k, uint32_t tbl) {
  return ((tbl & 1u) ? 1u : 0u) | ((4u + k) << 8) | (((tbl >> 1) ? 2u : 0x0cu) << 16) | (0x0cu << 24);
}
template <bool KEYXOR = true>
__device__ __forceinline__ uint32_t aes256_col16(uint32_t st, const RoundKeys& rk, const uint32_t* lds, uint32_t lc) {
  const uint32_t p = threadIdx.x & 15u, a = p & 3u, b = p >> 2;
  const uint32_t kA = (a - b) & 3u, kB = (b - a) & 3u;
  const uint32_t sA = sel_for(kA, kA), sB = sel_for(kB, kB), sF = sel_for(kB, (kB + 2u) & 3u);
  const uint32_t fm = 0xFFu << (8u * kB);
  st ^= rk.w[a];
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    const bool fromA = r & 1;
    uint32_t x = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) +
                                                    __builtin_amdgcn_perm(st, lc, fromA ? sA : sB));
    if (fromA) {
      x ^= dpp<1 | (0 << 2) | (3 << 4) | (2 << 6)>(x);
      x ^= dpp<2 | (3 << 2) | (0 << 4) | (1 << 6)>(x);
      st = KEYXOR ? x ^ rk.w[4 * r + b] : x;
    } else {
      x ^= dpp<kRowRor4>(x);
      x ^= dpp<kRowRor8>(x);
      st = KEYXOR ? x ^ rk.w[4 * r + a] : x;
    }
  }
  uint32_t x = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + __builtin_amdgcn_perm(st, lc, sF)) & fm;
  x ^= dpp<kRowRor4>(x);
  x ^= dpp<kRowRor8>(x);
  return x ^ rk.w[56 + a];
}

template <int MODE>
__global__ __launch_bounds__(64, 1) void k_chain(const uint32_t* __restrict__ tab, const RoundKeys rk, int iters,
                                                 uint32_t* out, unsigned long long* cyc) {
  __shared__ uint32_t lds[kLdsWords];
  for (int i = threadIdx.x; i < kLdsWords; i += 64) {
    const int half = i >> 14, rem = i & 16383;
    lds[i] = tab[(2 * half + ((rem & 63) >> 5)) * 256 + (rem >> 6)];
  }
  __syncthreads();
  const uint32_t lc = lane_const();
  uint32_t kw[15];
  col_round_keys(rk, threadIdx.x & 3u, kw);
  uint32_t x = (MODE >= 3) ? ((threadIdx.x & 3u) + 1u) * 0x9E3779B9u : threadIdx.x * 0x9E3779B9u, y = 0x1234567u + threadIdx.x;
  const bool on = (MODE == 0 || MODE == 5) ? threadIdx.x == 0 : (MODE == 3 ? threadIdx.x < 8 : ((MODE == 6 || MODE == 8) ? threadIdx.x < 16 : true));
  unsigned long long t0 = 0, t1 = 0;
  if (on) {
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
      if (MODE == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x = lds[(x & 1023u) * 4u + (threadIdx.x & 31u)];
      } else if (MODE == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "v"(y));
      } else if (MODE == 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x = dpp<kQpRot1>(x) ^ y;
      } else if (MODE == 3 || MODE == 4) {
        x = aes256_col(x, kw, lds, lc);
      } else if (MODE == 6 || MODE == 7) {
        x = aes256_col16(x, rk, lds, lc);
      } else if (MODE == 8) {
        x = aes256_col16<false>(x, rk, lds, lc);  // rounds 1-13 without the key XOR (not AES: timing only)
      } else {
        uint32_t st[1][4] = {{x, y, x ^ 1u, y ^ 2u}};
        aes256_tt<1>(st, rk, lds, lc);
        x = st[0][0] ^ st[0][1] ^ st[0][2] ^ st[0][3];
      }
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int MODE>
double run(const uint32_t* dtab, const RoundKeys& rk, uint32_t* out, unsigned long long* cyc, int iters, int per) {
  hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64), 0, 0, dtab, rk, iters, out, cyc);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64), 0, 0, dtab, rk, iters, out, cyc);
  unsigned long long c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  return (double)c / ((double)iters * per);
}

int main() {
  std::call_once(g_aes_once, aes_init_tables);
  uint8_t key[32];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
  RoundKeys rk;
  aes256_expand_words(key, &rk);
  uint32_t *dtab, *out;
  unsigned long long* cyc;
  hipMalloc(&dtab, sizeof(g_tab));
  hipMalloc(&out, 64 * 4);
  hipMalloc(&cyc, 8);
  hipMemcpy(dtab, g_tab, sizeof(g_tab), hipMemcpyHostToDevice);
  printf("{\"lds_read_dep_cycles\": %.2f, ", run<0>(dtab, rk, out, cyc, 2000, 8));
  printf("\"valu_dep_cycles\": %.2f, ", run<1>(dtab, rk, out, cyc, 2000, 8));
  printf("\"dpp_xor_dep_cycles\": %.2f, ", run<2>(dtab, rk, out, cyc, 2000, 8));
  printf("\"aes_col_8lanes_cycles\": %.1f, ", run<3>(dtab, rk, out, cyc, 2000, 1));
  printf("\"aes_col_64lanes_cycles\": %.1f, ", run<4>(dtab, rk, out, cyc, 2000, 1));
  printf("\"aes_block_per_lane_1lane_cycles\": %.1f, ", run<5>(dtab, rk, out, cyc, 2000, 1));
  uint32_t ref[64], got[64];
  run<3>(dtab, rk, out, cyc, 7, 1);
  hipMemcpy(ref, out, 256, hipMemcpyDeviceToHost);
  printf("\"aes_col16_16lanes_cycles\": %.1f, ", run<6>(dtab, rk, out, cyc, 2000, 1));
  run<6>(dtab, rk, out, cyc, 7, 1);
  hipMemcpy(got, out, 256, hipMemcpyDeviceToHost);
  bool same = true;
  for (int i = 0; i < 16; ++i) same &= got[i] == ref[i & 3];
  printf("\"aes_col16_matches_col\": %s, ", same ? "true" : "false");
  printf("\"col16_without_round_key_xor_16lanes_cycles\": %.1f, ", run<8>(dtab, rk, out, cyc, 2000, 1));
  printf("\"aes_col16_64lanes_cycles\": %.1f, \"unit\": \"s_memtime ticks (shader clock)\"}\n",
         run<7>(dtab, rk, out, cyc, 2000, 1));
  return 0;
}
