// Micro-benchmark: VALU issue rate of the ops the AES rounds use (v_perm_b32,
// v_bitop3_b32, v_xor_b32, v_add_u32), wave64, 16 waves per CU, 8 independent
// chains per lane; and ds_read_b32 (per-lane replicated, conflict-free) alone.
// Prints lane-ops per clock per CU at the measured kernel time and a nominal 2.4 GHz.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 65536;

template <int OP>
__global__ __launch_bounds__(1024, 1) void k_valu(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 7 * i + 1);
  uint32_t c = seed ^ threadIdx.x, c2 = seed + threadIdx.x;
  asm volatile("" : "+v"(c), "+v"(c2));
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = __builtin_amdgcn_perm(a[i], c, 0x05040100u + (uint32_t)i);
      if (OP == 1) a[i] = __builtin_amdgcn_bitop3_b32(a[i], c, c2, 0x96);
      if (OP == 2) a[i] ^= c;
      if (OP == 3) a[i] += c;
      if (OP == 4) a[i] = (a[i] & 1u) ? c : c2;
      if (OP == 5) a[i] = __builtin_amdgcn_perm(a[i], c, c2);  // selector in a VGPR
      if (OP == 6) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3"
                                : "+v"(a[i]) : "v"(c));
      if (OP == 7) a[i] = (a[i] & 0xFF00u) | c;   // v_and_or_b32
      if (OP == 8) a[i] = __builtin_amdgcn_ubfe(a[i], 8, 8);
      if (OP == 9) a[i] = (a[i] << 8) | c;        // v_lshl_or_b32
      asm volatile("" : "+v"(a[i]));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[threadIdx.x] = r;
}

__global__ __launch_bounds__(1024, 1) void k_lds(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t lds[32768];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = i * seed;
  __syncthreads();
  const uint32_t lane = (threadIdx.x & 31u) * 4u;
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (threadIdx.x * 16 + i) & 0xFF;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t addr = ((a[i] & 0xFFu) << 8) | lane;  // bank = lane: conflict-free
      a[i] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + addr);
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[threadIdx.x] = r;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out;
  hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v_perm_b32", "v_bitop3_b32", "v_xor_b32", "v_add_u32", "v_cndmask_b32",
                         "ds_read_b32+and_or", "v_perm (vgpr sel)", "v_mov_sdwa preserve", "v_and_or_b32",
                         "v_bfe_u32", "v_lshl_or_b32"};
  for (int op = 0; op < 11; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      switch (op) {
        case 0: hipLaunchKernelGGL(k_valu<0>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 1: hipLaunchKernelGGL(k_valu<1>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 2: hipLaunchKernelGGL(k_valu<2>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 3: hipLaunchKernelGGL(k_valu<3>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 4: hipLaunchKernelGGL(k_valu<4>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 5: hipLaunchKernelGGL(k_lds, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 6: hipLaunchKernelGGL(k_valu<5>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 7: hipLaunchKernelGGL(k_valu<6>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 8: hipLaunchKernelGGL(k_valu<7>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 9: hipLaunchKernelGGL(k_valu<8>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
        case 10: hipLaunchKernelGGL(k_valu<9>, dim3(cus), dim3(1024), 0, 0, out, 3u); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) {
        const double ops = (double)cus * 1024 * kIters * 8;  // lane-ops (or lane-lookups)
        printf("%-20s %8.3f ms  %7.2f lane-ops/clk/CU at 2.4 GHz\n", names[op], ms, ops / (ms * 1e-3) / 2.4e9 / cus);
      }
    }
  }
  return 0;
}
