// Micro-benchmark: HBM write bandwidth of the LAMBDA >= 32 tail's store pattern.
// 2^20 rows of 16 KiB; workgroup (tile, point block) writes TW bytes of each of its
// 4096 rows (16-byte stores, TW/16 lanes per row), as k_eval_wide_tail does.
// Build: hipcc --offload-arch=gfx950 -O3 tile_write_bw.hip -o tile_write_bw
#include <hip/hip_runtime.h>
#include <cstdio>

template <int TW>
__global__ __launch_bounds__(1024) void k_tiles(uint8_t* ys, uint32_t lam, uint64_t count, uint32_t pts) {
  constexpr int LP = TW / 16;
  const uint32_t q = threadIdx.x % LP;
  const uint32_t off = blockIdx.x * TW + 16 * q;
  const uint64_t p0 = (uint64_t)blockIdx.y * pts;
  const uint64_t p1 = p0 + pts < count ? p0 + pts : count;
  for (uint64_t p = p0 + threadIdx.x / LP; p < p1; p += blockDim.x / LP) {
    uint32_t* yo = reinterpret_cast<uint32_t*>(ys + p * lam + off);
    __builtin_nontemporal_store((uint32_t)p, yo);
    __builtin_nontemporal_store(off, yo + 1);
    __builtin_nontemporal_store(0u, yo + 2);
    __builtin_nontemporal_store(1u, yo + 3);
  }
}

template <int TW>
static void run(uint8_t* ys, uint32_t lam, uint64_t count, size_t lds = 0) {
  const uint32_t pts = 4096;
  dim3 g(lam / TW, (unsigned)((count + pts - 1) / pts));
  hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tiles<TW>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_tiles<TW><<<g, 1024, lds>>>(ys, lam, count, pts);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) k_tiles<TW><<<g, 1024, lds>>>(ys, lam, count, pts);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  printf("TW=%5d LDS=%6zu: %.3f ms per 2^20 rows, %.2f TB/s\n", TW, lds, ms, (double)count * lam / ms / 1e9);
}

int main() {
  const uint32_t lam = 16384;
  const uint64_t count = 1ull << 20;
  uint8_t* ys = nullptr;
  if (hipMalloc(&ys, count * lam) != hipSuccess) return 1;
  run<256>(ys, lam, count);
  run<32>(ys, lam, count, 135168);   // narrower tiles: partial 128-B lines per workgroup
  run<64>(ys, lam, count, 135168);
  run<128>(ys, lam, count, 135168);
  run<256>(ys, lam, count, 135168);  // the tail's LDS: one 1024-thread workgroup per CU
  run<256>(ys, lam, count, 66000);
  run<512>(ys, lam, count);
  run<1024>(ys, lam, count);
  run<4096>(ys, lam, count);
  run<16384>(ys, lam, count);
  hipFree(ys);
  return 0;
}
