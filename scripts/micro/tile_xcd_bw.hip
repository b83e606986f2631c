// Micro-benchmark: HBM write bandwidth of narrow (32 / 64-byte) output tiles when the
// workgroups that share a 128-byte line run on one XCD.  tile_write_bw.hip measured 0.71 TB/s
// for 32-byte tiles dealt tile-fastest (the four tiles of a line land on four XCDs, whose L2s
// each write back a partial line); here block b's siblings are b + 8, b + 16, ... (blocks are
// dealt round-robin over the 8 XCDs, MI355X_MICROARCH.md "Workgroup dispatch"), so one L2
// sees the whole line.  2^20 rows of 16 KiB; one 1024-thread workgroup per CU (LDS padding).
// Build: hipcc --offload-arch=gfx950 -O3 tile_xcd_bw.hip -o tile_xcd_bw
#include <hip/hip_runtime.h>
#include <cstdio>

template <int TW, bool XCD, bool NT>
__global__ __launch_bounds__(1024) void k_tiles(uint8_t* ys, uint32_t lam, uint64_t count, uint32_t pts) {
  constexpr int LP = TW / 16, SIB = 128 / TW;
  const uint32_t nt = lam / TW;  // tiles per row
  uint32_t tile, range;
  const uint32_t b = blockIdx.x;
  if (XCD && SIB > 1) {
    // unit u = (line, range); its SIB siblings are blocks 8 * (SIB * (u / 8) + s) + u % 8
    const uint32_t xcd = b & 7u, slot = b >> 3;
    const uint32_t u = (slot / SIB) * 8u + xcd, s = slot % SIB;
    const uint32_t nl = lam / 128;
    tile = (u % nl) * SIB + s;
    range = u / nl;
  } else {
    tile = b % nt;
    range = b / nt;
  }
  const uint32_t q = threadIdx.x % LP;
  const uint32_t off = tile * TW + 16 * q;
  const uint64_t p0 = (uint64_t)range * pts;
  const uint64_t p1 = p0 + pts < count ? p0 + pts : count;
  for (uint64_t p = p0 + threadIdx.x / LP; p < p1; p += blockDim.x / LP) {
    uint32_t* yo = reinterpret_cast<uint32_t*>(ys + p * lam + off);
    if (NT) {
      __builtin_nontemporal_store((uint32_t)p, yo);
      __builtin_nontemporal_store(off, yo + 1);
      __builtin_nontemporal_store(0u, yo + 2);
      __builtin_nontemporal_store(1u, yo + 3);
    } else {
      *reinterpret_cast<uint4*>(yo) = make_uint4((uint32_t)p, off, 0u, 1u);
    }
  }
}

template <int TW, bool XCD, bool NT>
static void run(uint8_t* ys, uint32_t lam, uint64_t count, uint32_t pts, size_t lds) {
  const uint64_t nblk = (uint64_t)(lam / TW) * ((count + pts - 1) / pts);
  hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tiles<TW, XCD, NT>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_tiles<TW, XCD, NT><<<(unsigned)nblk, 1024, lds>>>(ys, lam, count, pts);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) k_tiles<TW, XCD, NT><<<(unsigned)nblk, 1024, lds>>>(ys, lam, count, pts);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  printf("TW=%4d xcd_siblings=%d nt=%d pts=%6u: %.3f ms per 2^20 rows, %.2f TB/s\n", TW, (int)XCD, (int)NT, pts, ms,
         (double)count * lam / ms / 1e9);
  fflush(stdout);
}

int main() {
  const uint32_t lam = 16384;
  const uint64_t count = 1ull << 20;
  uint8_t* ys = nullptr;
  if (hipMalloc(&ys, count * lam) != hipSuccess) return 1;
  const size_t lds = 135168;
  run<128, false, true>(ys, lam, count, 4096, lds);   // the tail today
  run<32, false, true>(ys, lam, count, 16384, lds);   // tile-fastest: siblings on four XCDs
  run<32, true, true>(ys, lam, count, 16384, lds);
  run<32, true, false>(ys, lam, count, 16384, lds);
  run<32, true, true>(ys, lam, count, 4096, lds);
  run<64, true, true>(ys, lam, count, 8192, lds);
  run<64, true, false>(ys, lam, count, 8192, lds);
  run<128, false, true>(ys, lam, count, 4096, lds);
  hipFree(ys);
  return 0;
}
