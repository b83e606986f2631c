// Micro-benchmark: AES-256 throughput of the LDS T-table rounds alone (no DCF walk), one
// 1024-thread workgroup per CU (as the eval kernels), NB independent chains per lane,
// round keys from SGPRs (aes256_tt) or per round from global memory (aes256_tt_gk).
// Tells how much of the stream kernel's gap to the LDS bound is the AES itself.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/micro/aes_rate.hip -o scripts/micro/aes_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>
#include "../../dcf_amd/csrc/aes_lds.h"

constexpr int kIters = 2048;

// T1 lookups of the middle rounds through one v_bitop3 ((w & 0xFF00) | lc1: the state byte
// already sits at address bits 8..15) instead of a v_perm.
template <int NB>
__device__ __forceinline__ void aes256_tt_b(uint32_t (&st)[NB][4], const RoundKeys& rk, const uint32_t* lds,
                                            uint32_t lc, uint32_t lc1) {
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
        const uint32_t ad = __builtin_amdgcn_bitop3_b32(st[b][(j + 1) & 3], 0xFF00u, lc1, 0xEA);
        const uint32_t c = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + ad);
        const uint32_t d = lk<2, 2>(lds, st[b][(j + 2) & 3], lc);
        const uint32_t e = lk<3, 3>(lds, st[b][(j + 3) & 3], lc);
        o[b][j] = xor3(xor3(a, c, d), e, rk.w[4 * r + j]);
      }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
  }
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

// Lookup of T_T at state byte K through the vector L1 instead of the LDS: the compact 4 KiB
// T0..T3 image in global memory (L1-resident), offset (byte << 2) by a shift and a mask.
template <int T, int K>
__device__ __forceinline__ uint32_t lkg(const uint32_t* __restrict__ gt, uint32_t w) {
  const uint32_t off = (K == 0 ? (w << 2) : (w >> (8 * K - 2))) & 0x3FCu;
  // buffer load: 32-bit VGPR offset, resource in SGPRs (no 64-bit address VALU)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(gt), 0, 4096, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b32(rs, off, T * 1024, 0);
}

// Middle rounds with GN of the 16 lookups per round through the vector L1 (column j's T3
// lookup for j < GN, then column j - 4's T2 lookup): LDS and L1 share the lookups.
template <int NB, int GN>
__device__ __forceinline__ void aes256_tt_mix(uint32_t (&st)[NB][4], const RoundKeys& rk, const uint32_t* lds,
                                              uint32_t lc, const uint32_t* __restrict__ gt) {
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
        const uint32_t d = (j + 4 < GN) ? lkg<2, 2>(gt, st[b][(j + 2) & 3]) : lk<2, 2>(lds, st[b][(j + 2) & 3], lc);
        const uint32_t e = (j < GN) ? lkg<3, 3>(gt, st[b][(j + 3) & 3]) : lk<3, 3>(lds, st[b][(j + 3) & 3], lc);
        o[b][j] = xor3(xor3(a, c, d), e, rk.w[4 * r + j]);
      }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[b][j] = o[b][j];
  }
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

template <int NB, int MODE>
__global__ __launch_bounds__(1024, 1) void k_aes(const uint32_t* __restrict__ tab, const RoundKeys rk,
                                                 const uint4* __restrict__ rkg, uint32_t* out) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  const uint32_t lc1 = (lc >> 8) & 0xFFu;  // T1's lane bits, state byte 1 goes to bits 8..15
  uint32_t st[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) st[b][j] = (blockIdx.x * 1024 + threadIdx.x) * 0x9E3779B9u + 77u * b + j;
  for (int it = 0; it < kIters; ++it) {
    if (MODE == 0) aes256_tt<NB>(st, rk, lds, lc);
    if (MODE == 1) aes256_tt_gk<NB>(st, rkg, lds, lc);
    if (MODE == 2) aes256_tt_b<NB>(st, rk, lds, lc, lc1);
    if (MODE >= 10) aes256_tt_mix<NB, MODE - 10>(st, rk, lds, lc, tab);
  }
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) r ^= st[b][j];
  if (out) out[blockIdx.x * 1024 + threadIdx.x] = r;
}

// ds_read_b32 alone: 16 independent conflict-free lookups per iteration at addresses an empty
// asm redefines (no address VALU, no dependency between iterations): the LDS issue ceiling.
__global__ __launch_bounds__(1024, 1) void k_lds_only(const uint32_t* __restrict__ tab, uint32_t* out) {
  __shared__ uint32_t lds[kLdsWords];
  lds_fill_tables(lds, tab);
  const uint32_t lc = lane_const();
  uint32_t a[16], acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    a[j] = __builtin_amdgcn_perm(threadIdx.x * 0x9E3779B9u + j, lc, 0x0c020501u);
    acc[j] = 0u;
  }
  for (int it = 0; it < kIters * 14 * 2 * 16 / 16 / 8; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(a[j]));
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] ^= *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + a[j]);
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) r ^= acc[j];
  if (out) out[blockIdx.x * 1024 + threadIdx.x] = r;
}

template <int NB, int MODE>
void run(const char* name, int cus, const uint32_t* dtab, const RoundKeys& rk, const uint4* rkg, uint32_t* out,
         int wgs_per_cu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = cus * wgs_per_cu;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_aes<NB, MODE>), dim3(grid), dim3(1024), 0, 0, dtab, rk, rkg, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep == 1) {
      const double blocks = (double)grid * 1024 * NB * kIters;
      printf("%-28s NB=%d %8.3f ms  %6.2f G blocks/s  (%.3f of the 87.8 LDS bound)\n", name, NB, ms,
             blocks / (ms * 1e-3) / 1e9, blocks / (ms * 1e-3) / 87.77e9);
    }
  }
}

// Occupancy sweep (C1's ceiling): one workgroup of `waves` waves per CU, one AES block per lane,
// round keys per round from global memory as the pair walk (k_eval16_pair) reads them; blocks / s
// per CU against the waves the CU holds (C1: 100k points x 2 lanes = 13 waves on 241 CUs).
void occupancy(int cus, const uint32_t* dtab, const RoundKeys& rk, const uint4* rkg, uint32_t* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // NB = 1 at 4 .. 16 waves; NB = 2 at half the waves (the same blocks in flight, twice the ILP)
  for (int cfg = 0; cfg < 9; ++cfg) {
    const int nb = cfg < 6 ? 1 : 2;
    const int waves = cfg < 6 ? (int[]){4, 8, 12, 13, 14, 16}[cfg] : (int[]){6, 7, 8}[cfg - 6];
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (nb == 1) hipLaunchKernelGGL((k_aes<1, 1>), dim3(cus), dim3(64 * waves), 0, 0, dtab, rk, rkg, out);
      else hipLaunchKernelGGL((k_aes<2, 1>), dim3(cus), dim3(64 * waves), 0, 0, dtab, rk, rkg, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) {
        const double blocks = (double)cus * 64 * waves * kIters * nb;
        printf("occupancy %2d waves/CU, %d block(s)/lane, global keys: %8.3f ms  %6.2f G blocks/s  (%.3f of the 87.8 "
               "LDS bound)\n", waves, nb, ms, blocks / (ms * 1e-3) / 1e9, blocks / (ms * 1e-3) / 87.77e9);
      }
    }
  }
}

int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::call_once(g_aes_once, aes_init_tables);
  uint8_t key[32];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
  RoundKeys rk;
  aes256_expand_words(key, &rk);
  uint32_t *dtab, *out;
  uint4* rkg;
  hipMalloc(&dtab, sizeof(g_tab));
  hipMalloc(&rkg, 240);
  hipMalloc(&out, (size_t)cus * 16 * 1024 * 4);
  hipMemcpy(dtab, g_tab, sizeof(g_tab), hipMemcpyHostToDevice);
  hipMemcpy(rkg, rk.w, 240, hipMemcpyHostToDevice);
  printf("CUs %d\n", cus);
  if (argc > 1 && !strcmp(argv[1], "occ")) {
    occupancy(cus, dtab, rk, rkg, out);
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "mix")) {
    // LDS + vector-L1 split of the lookups, and the outputs against the all-LDS rounds
    for (int w : {4, 16}) {
      printf("-- %d workgroups per CU\n", w);
      run<2, 0>("all LDS", cus, dtab, rk, rkg, out, w);
      run<2, 11>("1 of 16 via L1", cus, dtab, rk, rkg, out, w);
      run<2, 12>("2 of 16 via L1", cus, dtab, rk, rkg, out, w);
      run<2, 13>("3 of 16 via L1", cus, dtab, rk, rkg, out, w);
      run<2, 14>("4 of 16 via L1", cus, dtab, rk, rkg, out, w);
      run<2, 16>("6 of 16 via L1", cus, dtab, rk, rkg, out, w);
      run<2, 18>("8 of 16 via L1", cus, dtab, rk, rkg, out, w);
      run<3, 12>("2 of 16 via L1", cus, dtab, rk, rkg, out, w);
      run<3, 14>("4 of 16 via L1", cus, dtab, rk, rkg, out, w);
    }
    const int n = cus * 1024;
    uint32_t* o2;
    hipMalloc(&o2, n * 4);
    hipLaunchKernelGGL((k_aes<2, 0>), dim3(cus), dim3(1024), 0, 0, dtab, rk, rkg, out);
    hipLaunchKernelGGL((k_aes<2, 16>), dim3(cus), dim3(1024), 0, 0, dtab, rk, rkg, o2);
    std::vector<uint32_t> h1(n), h2(n);
    hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), o2, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += h1[i] != h2[i];
    printf("6-via-L1 outputs vs all-LDS rounds: %d of %d differ\n", bad, n);
    return 0;
  }
  for (int w : {4, 16}) {
    printf("-- %d workgroups per CU (work items in flight)\n", w);
    run<1, 0>("sgpr keys", cus, dtab, rk, rkg, out, w);
    run<2, 0>("sgpr keys", cus, dtab, rk, rkg, out, w);
    run<3, 0>("sgpr keys", cus, dtab, rk, rkg, out, w);
    run<4, 0>("sgpr keys", cus, dtab, rk, rkg, out, w);
    run<2, 1>("global keys (3 ahead)", cus, dtab, rk, rkg, out, w);
    run<3, 1>("global keys (3 ahead)", cus, dtab, rk, rkg, out, w);
    run<4, 1>("global keys (3 ahead)", cus, dtab, rk, rkg, out, w);
    run<2, 2>("sgpr keys, T1 by bitop3", cus, dtab, rk, rkg, out, w);
    run<3, 2>("sgpr keys, T1 by bitop3", cus, dtab, rk, rkg, out, w);
  }
  {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = kIters * 14 * 2 * 16 / 16 / 8;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_lds_only, dim3(cus * 4), dim3(1024), 0, 0, dtab, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double lookups = (double)cus * 4 * 1024 * iters * 16;
      if (rep) printf("ds_read_b32 only: %.3f ms, %.2f lookups/clk/CU at 2.4 GHz (%.3f of 32)\n", ms,
                      lookups / (ms * 1e-3) / 2.4e9 / cus, lookups / (ms * 1e-3) / 2.4e9 / cus / 32);
    }
  }
  // same outputs as the v_perm rounds?
  {
    const int n = cus * 1024;
    uint32_t* o2;
    hipMalloc(&o2, n * 4);
    hipLaunchKernelGGL((k_aes<2, 0>), dim3(cus), dim3(1024), 0, 0, dtab, rk, rkg, out);
    hipLaunchKernelGGL((k_aes<2, 2>), dim3(cus), dim3(1024), 0, 0, dtab, rk, rkg, o2);
    std::vector<uint32_t> h1(n), h2(n);
    hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), o2, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += h1[i] != h2[i];
    printf("T1-by-bitop3 outputs vs v_perm rounds: %d of %d differ\n", bad, n);
  }
  return 0;
}
