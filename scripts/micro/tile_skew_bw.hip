// Micro-benchmark: does workgroup drift cost HBM write bandwidth in the paired-slot tail's
// store pattern?  2^21 rows of 16 KiB, 128-byte tiles, one round of workgroups (tiles x
// ranges = 256, as DCF_TAIL2_ONE_ROUND launches): workgroup (tile t, range r) writes its
// 128 bytes of each row of the range, starting `skew * t` rows into the range (wrapping), so
// skew 0 = all tiles in step, larger skews = tiles writing rows far apart at any time.
// Build: hipcc --offload-arch=gfx950 -O3 tile_skew_bw.hip -o tile_skew_bw
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(1024) void k_skew(uint8_t* ys, uint32_t lam, uint64_t pts, uint64_t skew) {
  constexpr int TW = 128, LP = TW / 16;
  const uint32_t q = threadIdx.x % LP;
  const uint32_t off = blockIdx.x * TW + 16 * q;
  const uint64_t p0 = (uint64_t)blockIdx.y * pts;
  const uint64_t start = (skew * blockIdx.x) % pts;
  for (uint64_t i = threadIdx.x / LP; i < pts; i += blockDim.x / LP) {
    uint64_t r = start + i;
    if (r >= pts) r -= pts;
    const uint64_t p = p0 + r;
    uint32_t* yo = reinterpret_cast<uint32_t*>(ys + p * lam + off);
    __builtin_nontemporal_store((uint32_t)p, yo);
    __builtin_nontemporal_store(off, yo + 1);
    __builtin_nontemporal_store(0u, yo + 2);
    __builtin_nontemporal_store(1u, yo + 3);
  }
}

int main() {
  const uint32_t lam = 16384;
  const uint64_t count = 1ull << 21;
  const int ranges = 2;
  const uint64_t pts = count / ranges;
  uint8_t* ys = nullptr;
  if (hipMalloc(&ys, count * lam) != hipSuccess) return 1;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&k_skew), hipFuncAttributeMaxDynamicSharedMemorySize, 139264);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const uint64_t skews[] = {0, 8, 64, 256, 1024, 4096, 16384, 65536, 8191};
  for (uint64_t s : skews) {
    dim3 g(lam / 128, ranges);
    k_skew<<<g, 1024, 139264>>>(ys, lam, pts, s);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) k_skew<<<g, 1024, 139264>>>(ys, lam, pts, s);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("skew %6llu rows per tile: %.3f ms per 2^21 rows, %.2f TB/s\n", (unsigned long long)s, ms,
           (double)count * lam / ms / 1e9);
  }
  hipFree(ys);
  return 0;
}
