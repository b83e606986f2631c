// kernels_wide.h — LAMBDA >= 32 kernels (eval head/tail, gen, PRG hook).
// Included by dcf_hip.hip only.
//
// At LAMBDA >= 32 the Hirose PRG (prg.rs:42-73, diagonal zip (0,0),(1,1))
// encrypts only bytes [0,16) under cipher 0 and bytes [16,32) under cipher 17;
// every other byte of the four outputs is the seed (or ~seed), and bit 0 of
// byte LAMBDA-1 is cleared.  So per level, with A = E0(s[0:16]),
// B = E0(~s[0:16]), C = E17(s[16:32]), D = E17(~s[16:32]):
//   s_L = s  with [0:16) := A ^ s[0:16]      v_L = ~s with [0:16)  := B ^ ~s[0:16]
//   s_R = s  with [16:32) := C ^ s[16:32]    v_R = ~s with [16:32) := D ^ ~s[16:32]
//   t_L = lsb(A ^ s)[0], t_R = lsb(B ^ ~s)[0]
// Bytes [32, LAMBDA) of eval's state therefore never see AES and evolve the
// same way on both branches: eval's output there is LINEAR in the point's
// t-sequence T = (t_0 .. t_n) (n = 8N even):
//   y[j] = c[j] ^ XOR_{l=1..n+1} t_{l-1} W_l[j]
//   W_l = cw_v[l] ^ (l even ? cw_s[l] : 0)   (l <= n),   W_{n+1} = cw_np1
//   c   = s0
// except bit 0 of byte LAMBDA-1, which the PRG clears every level:
//   W_l.bit = cw_v[l].bit ^ (l == n ? cw_s[l].bit : 0),  W_{n+1}.bit = np1.bit,  c.bit = 0.
// Eval = k_eval_wide_head_stream (kernels_wide_stream.h: AES walk over bytes [0,32),
// emits y[0:32) and T) + k_eval_wide_tail / k_eval_wide_tail2 (y[32:LAMBDA) as a GF(2)
// combination of W rows, four-Russians tables in LDS).
// tests/test_gpu_parity.py checks the result bit for bit against the oracle,
// which runs the reference algorithm literally.
#pragma once

#include "aes_lds.h"

// Wave priority for the tail2 table reads (r05af: C4 -2.0 % with DCF_HEAD_PRIO).
#ifndef DCF_TAIL_PRIO
#define DCF_TAIL_PRIO 1
#endif

namespace {

// Per-point t-vector (head -> tail), tw words (64 B for N <= 31): byte c holds rows 4c..4c+3
// of the t-sequence in bits 0..3 (bit k = t_{4c+k}), i.e. the four-Russians index of chunk c,
// ready for v_perm address building in the tail.  tw = t_words(nlev): 16 for n + 1 <= 256 rows,
// else ceil((n + 1) / 16) rounded up to whole uint4.
constexpr int kTWords = 16;
__host__ __device__ constexpr uint32_t t_words(uint32_t nlev) {
  return nlev + 1u <= 256u ? 16u : ((((nlev + 1u + 15u) / 16u) + 3u) & ~3u);
}

__device__ __forceinline__ void load_tab4(uint32_t* t4, const uint32_t* __restrict__ tab) {
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) t4[i] = tab[i];
  __syncthreads();
}

// The schedules of ciphers 0 and 17 (p->d_rk2: 2 x 15 round keys) into LDS, 60 words each: a
// lane picks its cipher by a pointer, not by selecting between two by-value kernel arguments (which
// put both 240-byte schedules on the stack: 484 B of scratch per lane, r04).
__device__ __forceinline__ void load_rk2(uint32_t (*rks)[60], const uint4* __restrict__ rk2) {
  if (threadIdx.x < 30) {
    const uint4 k = rk2[threadIdx.x];
    uint32_t* o = &rks[threadIdx.x / 15][4 * (threadIdx.x % 15)];
    o[0] = k.x; o[1] = k.y; o[2] = k.z; o[3] = k.w;
  }
}

// AES-256 for a few lanes: plain T-table reads from a 4 KiB LDS copy; rk: 60 round-key words (LDS).
__device__ __forceinline__ void aes256_small(uint32_t (&w)[4], const uint32_t* rk, const uint32_t* t4) {
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] ^= rk[j];
  for (int r = 1; r < 14; ++r) {
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = t4[w[j] & 0xff] ^ t4[256 + ((w[(j + 1) & 3] >> 8) & 0xff)] ^
             t4[512 + ((w[(j + 2) & 3] >> 16) & 0xff)] ^ t4[768 + (w[(j + 3) & 3] >> 24)] ^ rk[4 * r + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = o[j];
  }
  uint32_t o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    o[j] = (t4[512 + (w[j] & 0xff)] & 0xffu) ^ (t4[768 + ((w[(j + 1) & 3] >> 8) & 0xff)] & 0xff00u) ^
           (t4[(w[(j + 2) & 3] >> 16) & 0xff] & 0xff0000u) ^ (t4[256 + (w[(j + 3) & 3] >> 24)] & 0xff000000u) ^
           rk[56 + j];
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = o[j];
}

// The W-row formula (see file header), the one definition every user shares: row r < n is
// cw_v[r] ^ (r + 1 even ? cw_s[r] : 0), except bit 0 of byte LAMBDA - 1 (bit 24 of the last word
// of the last piece), where cw_s joins only at r + 1 == n; row n is cw_np1 (passed as cv).
__device__ __forceinline__ uint4 w_row_form(const uint4 cv, const uint4 cs, uint32_t r, uint32_t nlev,
                                            bool last_piece) {
  if (r >= nlev) return cv;
  const uint32_t l = r + 1u, even = (l & 1u) ? 0u : 0xFFFFFFFFu;
  uint4 w = make_uint4(cv.x ^ (cs.x & even), cv.y ^ (cs.y & even), cv.z ^ (cs.z & even), cv.w ^ (cs.w & even));
  if (last_piece) {
    const uint32_t bit = (cv.w ^ ((l == nlev) ? cs.w : 0u)) & 0x01000000u;
    w.w = (w.w & ~0x01000000u) | bit;
  }
  return w;
}

// W row r (coefficient t_r) of key `key`, 16 bytes at byte offset `off`; zero for an offset outside
// [32, LAMBDA) or r > n.
__device__ __forceinline__ uint4 w_row_piece(const uint8_t* __restrict__ cw_s, const uint8_t* __restrict__ cw_v,
                                             const uint8_t* __restrict__ cw_np1, uint32_t nlev, uint32_t lam,
                                             uint64_t num_keys, uint64_t key, uint32_t r, uint32_t off) {
  if (r > nlev || off >= lam || off < 32u) return make_uint4(0u, 0u, 0u, 0u);
  if (r == nlev) return *reinterpret_cast<const uint4*>(cw_np1 + key * lam + off);
  const uint64_t ro = ((uint64_t)r * num_keys + key) * lam + off;
  return w_row_form(*reinterpret_cast<const uint4*>(cw_v + ro), *reinterpret_cast<const uint4*>(cw_s + ro), r, nlev,
                    off + 16 == lam);
}


// The point's first 16 t-vector words (64 chunks); tw4 = uint4 per t-vector row.
__device__ __forceinline__ void tail_load_t(uint4 (&d)[4], const uint4* __restrict__ tv4, uint64_t pp, uint64_t p1,
                                            uint32_t tw4) {
  pp = min<uint64_t>(pp, p1 - 1);
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = tv4[tw4 * pp + k];
}

// One 16-byte piece of y for the point whose t-vector is t: cst ^ XOR over chunks c of
// G[c][t nibble c] (four-Russians, see k_eval_wide_tail).
// trow: the point's t-vector row, read directly for chunks past the first 64 (N >= 32).
template <int TW, int LP, int NCH>
__device__ __forceinline__ uint4 tail_piece(const uint4 (&t)[4], const uint4 cst, const char* gb, const uint4* G,
                                            uint32_t q, uint32_t nch16_rt, uint32_t nrem_rt,
                                            const uint4* __restrict__ trow) {
  // NCH > 0: chunk count fixed at compile time (fully unrolled; N = 16 has 33 chunks)
  const uint32_t nch16 = NCH > 0 ? (uint32_t)NCH / 16u : nch16_rt;
  const uint32_t nrem = NCH > 0 ? (uint32_t)NCH % 16u : nrem_rt;
  uint32_t acc[4] = {cst.x, cst.y, cst.z, cst.w};
  uint32_t tq[16] = {t[0].x, t[0].y, t[0].z, t[0].w, t[1].x, t[1].y, t[1].z, t[1].w,
                     t[2].x, t[2].y, t[2].z, t[2].w, t[3].x, t[3].y, t[3].z, t[3].w};
  // Row read of chunk c: G + c * 16 * TW + e * TW + q * 16 bytes.  At TW = 256 one
  // v_perm builds e * 256 + q * 16 (+ 64 KiB per group of 16 chunks) from the t byte
  // and a lane constant, and c * 4096 mod 64 KiB rides in the ds_read offset field.
  uint32_t qb = 16u * q;
  // BT reads are issued before their XORs (more LDS reads in flight per wave)
  constexpr uint32_t BT = 2;
  for (uint32_t g16 = 0; g16 < nch16; ++g16) {  // full groups of 16 chunks (4 t words)
    if (NCH == 0 && g16 >= 4) {  // past the 16 queued words
      const uint4 w = trow[g16];
      tq[0] = w.x; tq[1] = w.y; tq[2] = w.z; tq[3] = w.w;
    }
#pragma unroll
    for (uint32_t j = 0; j < 16; j += BT) {
      uint4 b[BT];
#pragma unroll
      for (uint32_t h = 0; h < BT; ++h) {
        const uint32_t cc = j + h;
        if (TW == 256) {
          const uint32_t a = __builtin_amdgcn_perm(tq[cc >> 2], qb, 0x0c020000u | ((4u + (cc & 3u)) << 8));
          b[h] = lds_load16(a + cc * 4096u);  // G sits at LDS address 0 (checked in the kernel)
        } else {
          const uint32_t e = (tq[cc >> 2] >> (8u * (cc & 3u))) & 15u;
          b[h] = G[((16u * g16 + cc) * 16u + e) * LP + q];
        }
      }
      // keep the batch's reads ahead of its XORs (the scheduler otherwise interleaves
      // them two at a time); LDS reads cannot move across a memory clobber
      if (BT > 2) asm volatile("" ::: "memory");
#pragma unroll
      for (uint32_t h = 0; h < BT; h += 2) {
        acc[0] = xor3(acc[0], b[h].x, b[h + 1].x);
        acc[1] = xor3(acc[1], b[h].y, b[h + 1].y);
        acc[2] = xor3(acc[2], b[h].z, b[h + 1].z);
        acc[3] = xor3(acc[3], b[h].w, b[h + 1].w);
      }
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) tq[k] = tq[k + 4];  // word queue: no dynamic register indexing
    qb += 0x10000u;
  }
  if (NCH == 0 && nch16 >= 4 && nrem) {
    const uint4 w = trow[nch16];
    tq[0] = w.x; tq[1] = w.y; tq[2] = w.z; tq[3] = w.w;
  }
#pragma unroll
  for (uint32_t cc = 0; cc < 15; ++cc) {  // remaining nch % 16 chunks
    if (cc < nrem) {
      const uint32_t e = (tq[cc >> 2] >> (8u * (cc & 3u))) & 15u;
      const uint4 b = G[((16u * nch16 + cc) * 16u + e) * LP + q];
      acc[0] ^= b.x; acc[1] ^= b.y; acc[2] ^= b.z; acc[3] ^= b.w;
    }
  }
  return make_uint4(acc[0], acc[1], acc[2], acc[3]);
}

// Non-temporal (written once, never re-read here; C4 A/B r02z: 36.0-36.2 ms vs 36.9-37.0 plain) buffer store of
// a y piece; `kill` != 0 puts the lane's offset past num_records, which drops it.
template <int LP>
__device__ __forceinline__ void tail_store(uint8_t* ys, uint64_t pw, uint32_t pin, uint32_t lam, uint32_t off,
                                           uint32_t kill, uint4 y) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t base = (uint64_t)(uintptr_t)(ys + pw * lam);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base), hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  uint8_t* wb = reinterpret_cast<uint8_t*>((uintptr_t)(((uint64_t)hi << 32) | lo));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(wb, (short)0, (int)((64 / LP) * lam), 0x00020000);
  const u32x4 v = {y.x, y.y, y.z, y.w};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (pin * lam + off) | kill, 0, 2 /* nt */);
}

// ------------------------------------------------------------------------
// Tail: y[32 + TW*tile .. +TW) for a range of points.  LP = TW/16 lanes per
// point, each owns one 16-byte piece.  LDS: G[chunk][nibble][LP] uint4,
// G[c][e] = XOR of W rows 4c+k over the set bits k of e.  All LP lanes of a
// point read one contiguous TW-byte entry -> conflict-free ds_read_b128.
// A launch covers chunks [c0, c0 + ncp) (ncp <= what the LDS holds; c0 % 16 == 0): when
// the t-sequence has more chunks than one table set holds (N >= 160 at 32-byte tiles), the
// host runs passes and ACC launches start from the y the previous pass wrote instead of s0.
// ------------------------------------------------------------------------
template <int TW, int NCH = 0, bool ACC = false>
__global__ __launch_bounds__(kBlock) void k_eval_wide_tail(const uint8_t* __restrict__ cw_s,
                                                            const uint8_t* __restrict__ cw_v,
                                                            const uint8_t* __restrict__ cw_np1,
                                                            const uint8_t* __restrict__ s0, const uint32_t nlev,
                                                            const uint32_t lam, const uint64_t num_keys,
                                                            const uint64_t key0, const uint32_t* __restrict__ tvec,
                                                            const uint64_t count, const uint32_t pts_per_block,
                                                            uint8_t* __restrict__ ys, const uint32_t tw,
                                                            const uint64_t ppk, const uint32_t rpk,
                                                            const uint32_t c0, const uint32_t ncp) {
  constexpr int LP = TW / 16;
  const uint32_t cb = ACC ? c0 : 0u;  // first chunk of this pass
  // Row blockIdx.y of the grid = range rr of key kk of the launch's keys (ppk points each, rpk
  // ranges per key; one key: ppk = count, rpk = gridDim.y)
  const uint32_t kk = blockIdx.y / rpk, rr = blockIdx.y % rpk;
  const uint64_t key = key0 + kk;
  extern __shared__ uint4 G[];
  if (TW == 256 && (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)G != 0u) __builtin_trap();
  const uint32_t nch = ncp;
  // Tiles are aligned to TW bytes of the output row (tile 0's first 32 bytes belong to
  // the head and are skipped): unaligned 256-byte pieces split cache lines between
  // neighbouring tiles and measured 20 % slower HBM writes.
  const uint32_t byte0 = (uint32_t)blockIdx.x * TW;
  // Tables: one thread per (chunk, piece) loads its chunk's 4 W-row pieces (all
  // loads in flight at once) and writes the 16 XOR combinations; one barrier.
  for (uint32_t it = threadIdx.x; it < nch * LP; it += blockDim.x) {
    const uint32_t qq = it % LP, c = it / LP;
    uint4 w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = w_row_piece(cw_s, cw_v, cw_np1, nlev, lam, num_keys, key, 4 * (cb + c) + k, byte0 + 16 * qq);
    uint4* dst = G + (c * 16) * LP + qq;
    uint4 e[16];
    e[0] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int x = 1; x < 16; ++x) {  // e[x] = e[x without its lowest bit] ^ w[lowest bit]
      const uint4 a0 = e[x & (x - 1)], b0 = w[__builtin_ctz(x)];
      e[x] = make_uint4(a0.x ^ b0.x, a0.y ^ b0.y, a0.z ^ b0.z, a0.w ^ b0.w);
    }
#pragma unroll
    for (int x = 0; x < 16; ++x) dst[x * LP] = e[x];
  }
  __syncthreads();
  const uint32_t q = threadIdx.x % LP;
  const uint32_t off = byte0 + 16 * q;
  const bool lane_live = off >= 32u && off < lam;
  uint4 cst = make_uint4(0u, 0u, 0u, 0u);
  if (lane_live) {
    cst = *reinterpret_cast<const uint4*>(s0 + (uint64_t)kk * lam + off);
    if (off + 16 == lam) cst.w &= kMaskLast;
  }
  const uint64_t kb = (uint64_t)kk * ppk;
  const uint64_t p0 = kb + (uint64_t)rr * pts_per_block;
  const uint64_t p1 = min<uint64_t>(min<uint64_t>(count, kb + ppk), p0 + pts_per_block);
  const uint32_t pstep = blockDim.x / LP;
  const uint32_t pin = (threadIdx.x & 63u) / LP;  // the lane's point among the wave's 64 / LP
  // t-vectors (their first 64 B) are loaded two points ahead into ping-pong registers,
  // clamped instead of guarded, and the y store below is unconditional too: with no
  // branch around any vector-memory instruction the compiler counts vmcnt exactly and
  // waits for the t-vector loads only, never for an older non-temporal y store.
  const uint4* tv4 = reinterpret_cast<const uint4*>(tvec) + cb / 16u;  // this pass's t words
  const uint32_t tw4 = tw / 4u;
  uint64_t p = p0 + threadIdx.x / LP;
  // ACC: the point's y piece so far (dead lanes and past-the-end points read a clamped, unused piece)
  auto ycur = [&](uint64_t pp) -> uint4 {
    if (!ACC) return cst;
    pp = min<uint64_t>(pp, p1 - 1);
    const uint4 v = *reinterpret_cast<const uint4*>(ys + pp * lam + (lane_live ? off : 32u));
    return lane_live ? v : make_uint4(0u, 0u, 0u, 0u);
  };
  uint4 ta[4], tb[4];
  tail_load_t(ta, tv4, p, p1, tw4);
  tail_load_t(tb, tv4, p + pstep, p1, tw4);
  const char* gb = reinterpret_cast<const char*>(G);
  const uint32_t nch16 = nch >> 4, nrem = nch & 15u;
  // Buffer store: base = the wave's first point row, dead lanes get an offset past
  // num_records (the store drops it).  4 points x LAMBDA bytes <= 4 GiB.
  const uint32_t dead = 0x80000000u;
  for (;;) {
    if (p >= p1) break;
    {
      const uint4 y = tail_piece<TW, LP, NCH>(ta, ycur(p), gb, G, q, nch16, nrem, tv4 + tw4 * min<uint64_t>(p, p1 - 1));
      tail_load_t(ta, tv4, p + 2 * pstep, p1, tw4);
      tail_store<LP>(ys, p - pin, pin, lam, off, lane_live ? 0u : dead, y);
    }
    p += pstep;
    if (p >= p1) break;
    {
      const uint4 y = tail_piece<TW, LP, NCH>(tb, ycur(p), gb, G, q, nch16, nrem, tv4 + tw4 * min<uint64_t>(p, p1 - 1));
      tail_load_t(tb, tv4, p + 2 * pstep, p1, tw4);
      tail_store<LP>(ys, p - pin, pin, lam, off, lane_live ? 0u : dead, y);
    }
    p += pstep;
  }
}

// ------------------------------------------------------------------------
// Tail with wide chunks ("paired-slot" four-Russians): 128-byte tiles, 6- and 5-bit chunks.
//
// The 4-bit tail above reads 33 table entries per 16 bytes of y (N = 16): its tables are
// 16 x 256 B per chunk and a chunk's entry must span all 64 banks for 16 lanes to read it
// conflict-free, so 160 KB of LDS cannot hold wider chunks.  Here a tile is 128 bytes (8
// lanes per point; 128-B tiles still write whole cache lines: 5.6 TB/s vs 3.75 at 64 B and
// 0.71 at 32 B, scripts/micro/tile_write_bw.hip) and two chunks share a 256-byte LDS row:
// region m holds chunks 2m and 2m+1, entry e of both in row e (chunk 2m in bytes [0,128),
// 2m+1 in [128,256)).  A 16-lane LDS pass holds two points (pi = 0, 1); at step i of region
// m the point pi reads chunk 2m + (i ^ pi), so the two points always sit in opposite halves
// of the bank span — conflict-free for any data.  With chunks of 6 bits (regions of 16 KiB)
// and 5 bits (8 KiB), N = 16's 129 rows take 5 + 7 regions = 24 reads per 16 bytes of y
// (136 KiB of LDS) instead of 33.
//
// t-vector ("chunk bytes", produced from the head's nibble format by k_tvec_chunks): byte k =
// the index of chunk k: chunks 0 .. 2 R6 - 1 are 6 rows each from row 0, then 5-row chunks.
// Rows past n + 1 are zero.  Kept in place in the head's 64-byte t-vector rows (first 32 B).
// ------------------------------------------------------------------------
// ROW0 = 1 ("party folded"): row 0's coefficient is t_0 = party (lib.rs:169), the same for every
// point of the call, so its W row joins the constant (s0 ^ party W_0) and the chunks cover rows
// 1 .. n only — at N = 16 that is 128 rows, which (R6, R5) = (9, 2) covers in 22 reads per 16 bytes
// of y instead of (5, 7)'s 24, in exactly 160 KiB of LDS: the workgroup's block counter then lives
// in global memory (GCTR).
constexpr uint32_t kLdsMaxBytes = 160u * 1024u;
#ifndef DCF_T2_CLAIM
#define DCF_T2_CLAIM 4
#endif
constexpr uint32_t kT2ClaimBlocks = DCF_T2_CLAIM;  // 16-point blocks per global-counter claim (GCTR layouts; r05e A/B
                                                   // on C4 with 128-B-line counters: 1 / 4 / 16 blocks 32.4-32.7 / 32.0 / 31.8 ms)
#ifndef DCF_T2_CTR_STRIDE
#define DCF_T2_CTR_STRIDE 1
#endif
constexpr uint32_t kT2CtrStride = DCF_T2_CTR_STRIDE;  // words between workgroups' counters (r05e A/B: packed 31.57 / 31.73 ms
                                                     // vs one 128-B line each 32.01 / 32.00 on C4)
template <int R6, int R5, int ROW0 = 0>
struct Tail2Layout {
  static constexpr int R = R6 + R5, NC = 2 * R;
  static_assert(NC <= 32, "t-vector holds 32 chunk bytes");
  static constexpr uint32_t width(int k) { return k < 2 * R6 ? 6u : 5u; }
  static constexpr uint32_t start(int k) { return (uint32_t)ROW0 + (k < 2 * R6 ? 6u * k : 12u * R6 + 5u * (k - 2 * R6)); }
  static constexpr uint32_t region(int m) { return m < R6 ? 16384u * m : 16384u * R6 + 8192u * (m - R6); }
  static constexpr uint32_t rows() { return (uint32_t)ROW0 + 12u * R6 + 10u * R5; }  // rows 0 .. rows() - 1 covered
  static constexpr bool GCTR = region(R) + 16u > kLdsMaxBytes;  // no LDS left for the block counter
  static constexpr uint32_t lds_bytes() { return GCTR ? region(R) : region(R) + 16u; }
};

// Old nibble t-vector (row r at byte r >> 2, bit r & 3; words 0 .. nlev >> 4 valid) -> chunk
// bytes of Tail2Layout<R6, R5>, in place (bytes [0, 32) of each 64-byte row).  One thread
// per point: the row's first 16-byte pieces the layout's rows need read whole (unwritten
// words hold rows past t_n, cleared below), 32 bytes written.
template <int R6, int R5, int ROW0 = 0>
__global__ void k_tvec_chunks(uint32_t* __restrict__ tvec, const uint32_t nlev, const uint64_t count) {
  using L = Tail2Layout<R6, R5, ROW0>;
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= count) return;
  uint32_t* row = tvec + p * kTWords;
  constexpr uint32_t NQ = (L::rows() + 63u) / 64u;  // 16-byte pieces holding rows 0 .. rows() - 1
  uint32_t wv[4 * NQ];
#pragma unroll
  for (uint32_t q = 0; q < NQ; ++q) {
    const uint4 t = reinterpret_cast<const uint4*>(row)[q];
    wv[4 * q] = t.x; wv[4 * q + 1] = t.y; wv[4 * q + 2] = t.z; wv[4 * q + 3] = t.w;
  }
  uint32_t pk[6] = {0u, 0u, 0u, 0u, 0u, 0u};  // rows as a plain bit string, row r = bit r
#pragma unroll
  for (uint32_t j = 0; j < 4 * NQ; ++j) {
    if (16u * j < L::rows()) {
      uint32_t x = wv[j] & 0x0F0F0F0Fu;
      x = (x | (x >> 4)) & 0x00FF00FFu;
      x = (x | (x >> 8)) & 0x0000FFFFu;
      pk[j >> 1] |= x << (16u * (j & 1u));
    }
  }
  const uint32_t nrows = nlev + 1u;  // clear rows past t_n (never written by the head)
#pragma unroll
  for (uint32_t w = 0; w < 6; ++w) {
    const uint32_t lo = 32u * w;
    pk[w] &= nrows >= lo + 32u ? 0xFFFFFFFFu : (nrows <= lo ? 0u : ((1u << (nrows - lo)) - 1u));
  }
  uint32_t out[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
  for (int k = 0; k < L::NC; ++k) {
    const uint32_t s = L::start(k), w = L::width(k);
    const uint32_t lo = pk[s >> 5], hi = (s >> 5) + 1 < 6 ? pk[(s >> 5) + 1] : 0u;
    const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31u)) & ((1u << w) - 1u);
    out[k >> 2] |= v << (8 * (k & 3));
  }
  uint4* o4 = reinterpret_cast<uint4*>(row);
  o4[0] = make_uint4(out[0], out[1], out[2], out[3]);
  o4[1] = make_uint4(out[4], out[5], out[6], out[7]);
}

template <int R6, int R5, int ROW0 = 0>
__global__ __launch_bounds__(kBlock) void k_eval_wide_tail2(const uint8_t* __restrict__ cw_s,
                                                             const uint8_t* __restrict__ cw_v,
                                                             const uint8_t* __restrict__ cw_np1,
                                                             const uint8_t* __restrict__ s0, const uint32_t nlev,
                                                             const uint32_t lam, const uint64_t num_keys,
                                                             const uint64_t key0, const uint32_t* __restrict__ tvec,
                                                             const uint64_t count, const uint32_t pts_per_block,
                                                             uint8_t* __restrict__ ys, const uint64_t ppk,
                                                             const uint32_t rpk, const uint32_t party,
                                                             uint32_t* __restrict__ gctr) {
  using L = Tail2Layout<R6, R5, ROW0>;
  constexpr int TW = 128, LP = 8;
  // Row blockIdx.y of the grid = range rr of key kk of the launch's keys (as k_eval_wide_tail)
  const uint32_t kk = blockIdx.y / rpk, rr = blockIdx.y % rpk;
  const uint64_t key = key0 + kk;
  DCF_CLK(4, 0);  // (diagnostic builds) workgroup entry, before the table build
  extern __shared__ uint4 G[];
  if ((uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)G != 0u) __builtin_trap();
  const uint32_t byte0 = (uint32_t)blockIdx.x * TW;
  // Tables: item (chunk k, piece q, group g of 8 entries): the group's base (rows of the
  // entry bits >= 3) then its 8 entries in Gray-code order, one XOR each.
  {
    constexpr uint32_t items6 = 2 * R6 * LP * 8, items = items6 + 2 * R5 * LP * 4;
    char* gb = reinterpret_cast<char*>(G);
    for (uint32_t it = threadIdx.x; it < items; it += blockDim.x) {
      uint32_t k, rest, w;
      if (it < items6) { k = it / (LP * 8); rest = it % (LP * 8); w = 6u; }
      else { k = 2 * R6 + (it - items6) / (LP * 4); rest = (it - items6) % (LP * 4); w = 5u; }
      const uint32_t q = rest % LP, g = rest / LP;
      const uint32_t st = (uint32_t)ROW0 + (k < 2u * R6 ? 6u * k : 12u * R6 + 5u * (k - 2u * R6));
      const uint32_t off = byte0 + 16u * q;
      // W rows st .. st + 5 (row st + b used if b < w): all 12 loads issued before any is
      // used (w_row_piece's branches would serialise them), addresses clamped, then masked.
      uint4 wr[6];
      {
        const bool offok = off >= 32u && off < lam;
        uint4 cv[6], cs[6];
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          const uint32_t r = st + b;
          const bool isn = r == nlev;  // row n: cw_np1
          const uint32_t rr = (r < nlev && offok) ? r : 0u;
          const uint32_t o = offok ? off : 32u;
          const uint64_t ro = ((uint64_t)rr * num_keys + key) * lam + o;
          cv[b] = *reinterpret_cast<const uint4*>((isn && offok ? cw_np1 + key * lam + o : cw_v + ro));
          cs[b] = *reinterpret_cast<const uint4*>(cw_s + ro);
        }
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          const uint32_t r = st + b;
          const bool valid = offok && (uint32_t)b < w && r <= nlev;
          const uint32_t vm = valid ? 0xFFFFFFFFu : 0u;
          const uint4 x = w_row_form(cv[b], cs[b], r, nlev, off + 16 == lam);
          wr[b] = make_uint4(x.x & vm, x.y & vm, x.z & vm, x.w & vm);
        }
      }
      uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int b = 3; b < 6; ++b)
        if ((g >> (b - 3)) & 1u) { acc.x ^= wr[b].x; acc.y ^= wr[b].y; acc.z ^= wr[b].z; acc.w ^= wr[b].w; }
      const uint32_t m = k >> 1;
      const uint32_t rbase = m < (uint32_t)R6 ? 16384u * m : 16384u * R6 + 8192u * (m - R6);
      char* dst = gb + rbase + (k & 1u) * 128u + 16u * q;
#pragma unroll
      for (uint32_t i = 0; i < 8; ++i) {
        if (i) {
          const uint4 x = wr[__builtin_ctz(i)];
          acc.x ^= x.x; acc.y ^= x.y; acc.z ^= x.z; acc.w ^= x.w;
        }
        const uint32_t e = 8u * g + (i ^ (i >> 1));
        *reinterpret_cast<uint4*>(dst + 256u * e) = acc;
      }
    }
  }
  // the workgroup's block counter: past the tables, or (GCTR: the tables fill the LDS) its own word
  // of gctr, reset here (an atomic store at L2, where the claims' atomics run; the barrier orders it)
  uint32_t* bctr = L::GCTR ? gctr + kT2CtrStride * ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x)
                           : reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(G) + L::region(L::R));
  if (threadIdx.x == 0) {
    if (L::GCTR) __hip_atomic_store(bctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *bctr = 0u;
  }
  __syncthreads();
  DCF_CLK(0, 0);
  const uint32_t q = threadIdx.x % LP;
  const uint32_t pi = (threadIdx.x >> 3) & 1u;   // the point's half of a 16-lane LDS pass
  const uint32_t off = byte0 + 16 * q;
  const bool lane_live = off >= 32u && off < lam;
  uint4 cst = make_uint4(0u, 0u, 0u, 0u);
  if (lane_live) {
    cst = *reinterpret_cast<const uint4*>(s0 + (uint64_t)kk * lam + off);
    if (off + 16 == lam) cst.w &= kMaskLast;
    if (ROW0 && party) {  // row 0 (t_0 = party for every point) folded into the constant
      const uint4 w0 = w_row_piece(cw_s, cw_v, cw_np1, nlev, lam, num_keys, key, 0u, off);
      cst = make_uint4(cst.x ^ w0.x, cst.y ^ w0.y, cst.z ^ w0.z, cst.w ^ w0.w);
    }
  }
  // lane constants (address byte 0 = slot, byte 2 = 64 KiB group): step i of a region reads
  // chunk 2m + (i ^ pi), whose entry sits in bytes [(i ^ pi) 128, +128) of the 256-B row
  const uint32_t lc0 = pi * 128u + 16u * q, lc1 = (pi ^ 1u) * 128u + 16u * q;
  // pi = 1: swap the chunk bytes of each region (stored pre-swapped by k_tvec_chunks instead, the
  // tail has 6 fewer v_perm per point: C4 A/B 34.8-35.1 vs 34.5-34.8 ms, no gain — kept here)
  const uint32_t rsel = pi ? 0x02030001u : 0x03020100u;
  const uint64_t kb = (uint64_t)kk * ppk;
  const uint64_t p0 = kb + (uint64_t)rr * pts_per_block;
  const uint64_t p1 = min<uint64_t>(min<uint64_t>(count, kb + ppk), p0 + pts_per_block);
  const uint32_t pin = (threadIdx.x & 63u) / LP;  // the lane's point among the wave's 8
  const uint4* tv4 = reinterpret_cast<const uint4*>(tvec);
  auto load_t = [&](uint4 (&d)[2], uint64_t pp) {
    pp = min<uint64_t>(pp, p1 - 1);
    d[0] = tv4[4 * pp];
    d[1] = tv4[4 * pp + 1];
  };
  constexpr int NW = (L::NC + 3) / 4;  // chunk-byte words
  auto rotate = [&](const uint4 (&t)[2], uint32_t (&tw)[NW]) {
    const uint32_t w[8] = {t[0].x, t[0].y, t[0].z, t[0].w, t[1].x, t[1].y, t[1].z, t[1].w};
#pragma unroll
    for (int j = 0; j < NW; ++j) tw[j] = __builtin_amdgcn_perm(w[j], w[j], rsel);
  };
  // entry read for step i of region m of the point whose rotated chunk words are tw
  auto rd = [&](const uint32_t (&tw)[NW], int m, int i) {
    const uint32_t rb = L::region(m);
    const uint32_t grp = (rb >> 16) << 16;  // compile-time per m: the 64 KiB group in address byte 2
    const int c = 2 * m + i;               // byte of the rotated chunk vector
    const uint32_t a = __builtin_amdgcn_perm(tw[c >> 2], (i ? lc1 : lc0) | grp, 0x0c020000u | ((4u + (c & 3)) << 8));
    // the rest of the region base rides in the offset field
    return *(__attribute__((address_space(3))) const u32x4_t*)(size_t)(a + (rb & 0xFFFFu));
  };
  // Work: 16-point blocks of the workgroup's range, claimed per wave from the LDS counter (A = the
  // block's first 8 points, B = the next 8; a lane owns one 16-byte piece of one point of each).
  // The waves of a workgroup do not progress at one rate (VALU / LDS issue goes to the older
  // wave first), so a static split left the younger waves working alone for the last third of
  // the launch (in-kernel stamps: wave 0 done at 11 ms of a 17.5 ms kernel).  A block is claimed
  // one iteration ahead so its t-vectors load behind the current block's work.  The loop
  // condition is wave-uniform: no branch around a vector-memory instruction, so the compiler
  // counts vmcnt exactly (the t-vectors, loaded at the end of an iteration, are waited on at the
  // end of the next one, past the two y stores).  Past-the-end lanes load a clamped row and their
  // stores are dropped (offset past num_records).
  const uint32_t nblk = p1 > p0 ? (uint32_t)((p1 - p0 + 15) / 16) : 0u;
  auto claim = [&]() -> uint32_t {
    uint32_t b = 0u;
    if ((threadIdx.x & 63u) == 0)
      b = L::GCTR ? __hip_atomic_fetch_add(bctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : __hip_atomic_fetch_add(bctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(b);
  };
  const uint32_t dead = 0x80000000u;
  const uint32_t kill = lane_live ? 0u : dead;
  // GCTR: the counter is a global atomic, so a claim takes kT2ClaimBlocks consecutive blocks
  constexpr uint32_t CB = L::GCTR ? kT2ClaimBlocks : 1u;
  auto next_block = [&](uint32_t b) -> uint32_t { return ((b + 1u) % CB) ? b + 1u : claim() * CB; };
  // BT regions (4 reads each) are issued before their XORs: the compiler otherwise waits after
  // every two reads, ~3 reads in flight per wave.  All R regions into the accumulators.
  auto regions = [&](const uint32_t (&twa)[NW], const uint32_t (&twb)[NW], uint32_t (&aa)[4], uint32_t (&ab)[4]) {
#ifndef DCF_T2_BT
#define DCF_T2_BT 2
#endif
    // regions per read batch (r05ad, C4 same box: 2 / 3 / 4 regions 32.22-32.63 / 32.17-32.45 /
    // 32.12-32.42 ms, within noise)
    constexpr int BT = DCF_T2_BT;
#pragma unroll
    for (int m0 = 0; m0 < L::R; m0 += BT) {
      u32x4_t rb[BT][4];
#pragma unroll
      for (int k = 0; k < BT; ++k)
        if (m0 + k < L::R) {
          rb[k][0] = rd(twa, m0 + k, 0); rb[k][1] = rd(twa, m0 + k, 1);
          rb[k][2] = rd(twb, m0 + k, 0); rb[k][3] = rd(twb, m0 + k, 1);
        }
      // the batch's reads are all issued before the first result is used: a memory clobber
      // keeps them above, and one empty asm per read (issued in order) makes each XOR wait
      // for its own read only (lgkmcnt counts down in order).  One 128-bit operand per read:
      // four 32-bit operands let the allocator copy the tuple apart (a per-lane 64-bit row
      // address in the loop then spilled ~120 VGPRs, r05j)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < BT; ++k)
        if (m0 + k < L::R)
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(rb[k][j]));
#pragma unroll
      for (int k = 0; k < BT; ++k)
        if (m0 + k < L::R) {
          const u32x4_t a0 = rb[k][0], a1 = rb[k][1], b0 = rb[k][2], b1 = rb[k][3];
          aa[0] = xor3(aa[0], a0.x, a1.x); aa[1] = xor3(aa[1], a0.y, a1.y);
          aa[2] = xor3(aa[2], a0.z, a1.z); aa[3] = xor3(aa[3], a0.w, a1.w);
          ab[0] = xor3(ab[0], b0.x, b1.x); ab[1] = xor3(ab[1], b0.y, b1.y);
          ab[2] = xor3(ab[2], b0.z, b1.z); ab[3] = xor3(ab[3], b0.w, b1.w);
        }
      // the accumulators are materialised here, before the next batch's reads (else the XORs
      // may sink below them and every read result stays live: the r05j sorted tail spilled)
      asm volatile("" : "+v"(aa[0]), "+v"(aa[1]), "+v"(aa[2]), "+v"(aa[3]), "+v"(ab[0]), "+v"(ab[1]), "+v"(ab[2]),
                   "+v"(ab[3]));
    }
  };
  uint4 ta[2], tb[2];
  uint32_t twa[NW], twb[NW];
  uint32_t bc = claim() * CB;
  load_t(ta, p0 + 16u * bc + pin);
  load_t(tb, p0 + 16u * bc + 8u + pin);
  rotate(ta, twa);
  rotate(tb, twb);
  uint32_t bn = next_block(bc);
  load_t(ta, p0 + 16u * bn + pin);
  load_t(tb, p0 + 16u * bn + 8u + pin);
  while (bc < nblk) {
    uint32_t aa[4] = {cst.x, cst.y, cst.z, cst.w}, ab[4] = {cst.x, cst.y, cst.z, cst.w};
    if (DCF_TAIL_PRIO) __builtin_amdgcn_s_setprio(1);  // A/B knob: the table reads at priority 1
    regions(twa, twb, aa, ab);
    if (DCF_TAIL_PRIO) __builtin_amdgcn_s_setprio(0);
    const uint64_t pw = p0 + 16u * bc, pa = pw + pin, pb = pa + 8u;
    tail_store<LP>(ys, pw, pin, lam, off, kill | (pa < p1 ? 0u : dead), make_uint4(aa[0], aa[1], aa[2], aa[3]));
    tail_store<LP>(ys, pw + 8u, pin, lam, off, kill | (pb < p1 ? 0u : dead), make_uint4(ab[0], ab[1], ab[2], ab[3]));
    // the next block's t-vectors (loaded one iteration ago, before these two stores)
    bc = bn;
    rotate(ta, twa);
    rotate(tb, twb);
    bn = next_block(bc);
    load_t(ta, p0 + 16u * bn + pin);
    load_t(tb, p0 + 16u * bn + 8u + pin);
  }
  DCF_CLK(0, 1);
}

// ------------------------------------------------------------------------
// Gen at LAMBDA >= 32: one workgroup per key; thread i owns 16-byte pieces
// i, i+blockDim, ... of s_0, s_1, v_alpha (kept in `ws`, 3*LAMBDA per key).
// Per level 8 AES blocks (E0/E17 on s_p and ~s_p, p = 0, 1) by lanes 0..7.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_gen_wide(
    const uint32_t* __restrict__ tab, const uint4* __restrict__ rk2, const uint8_t* __restrict__ alpha,
    const uint8_t* __restrict__ beta, const uint8_t* __restrict__ s0_0, const uint8_t* __restrict__ s0_1,
    const uint32_t bound, const uint32_t nbytes, const uint64_t num_keys, const uint64_t key_base, const uint32_t lam,
    uint8_t* __restrict__ cw_s, uint8_t* __restrict__ cw_v, uint8_t* __restrict__ cw_t, uint8_t* __restrict__ cw_np1,
    uint8_t* __restrict__ ws) {
  __shared__ uint32_t t4[1024];
  __shared__ uint32_t head[2][2][8];  // [buffer][party][word]: s_p bytes [0,32)
  __shared__ uint32_t eo[2][4][4];    // [party][A,B,C,D][word]
  __shared__ uint32_t rks[2][60];     // ciphers 0 and 17
  load_rk2(rks, rk2);
  load_tab4(t4, tab);  // its barrier publishes rks
  const uint64_t k = key_base + blockIdx.x;
  const uint32_t npieces = lam / 16, nlev = 8u * nbytes;
  uint4* w_s0 = reinterpret_cast<uint4*>(ws + (uint64_t)blockIdx.x * 3 * lam);
  uint4* w_s1 = w_s0 + npieces;
  uint4* w_va = w_s1 + npieces;
  const uint4* in0 = reinterpret_cast<const uint4*>(s0_0 + k * lam);
  const uint4* in1 = reinterpret_cast<const uint4*>(s0_1 + k * lam);
  const uint4* be = reinterpret_cast<const uint4*>(beta + k * lam);
  for (uint32_t q = threadIdx.x; q < npieces; q += blockDim.x) {
    w_s0[q] = in0[q];
    w_s1[q] = in1[q];
    w_va[q] = make_uint4(0u, 0u, 0u, 0u);
    if (q < 2) {
      const uint4 a = in0[q], b = in1[q];
      head[0][0][4 * q] = a.x; head[0][0][4 * q + 1] = a.y; head[0][0][4 * q + 2] = a.z; head[0][0][4 * q + 3] = a.w;
      head[0][1][4 * q] = b.x; head[0][1][4 * q + 1] = b.y; head[0][1][4 * q + 2] = b.z; head[0][1][4 * q + 3] = b.w;
    }
  }
  __syncthreads();
  uint32_t t0 = 0u, t1 = 1u;  // lib.rs:100
  const uint8_t* al = alpha + k * nbytes;
  for (uint32_t lev = 0; lev < nlev; ++lev) {
    const uint32_t buf = lev & 1u;
    if (threadIdx.x < 8) {
      const uint32_t p = threadIdx.x >> 2, which = threadIdx.x & 3u, hi = which >> 1;
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t sw = head[buf][p][4 * hi + j];
        w[j] = (which & 1u) ? ~sw : sw;
      }
      aes256_small(w, rks[hi], t4);
#pragma unroll
      for (int j = 0; j < 4; ++j) eo[p][which][j] = w[j];
    }
    __syncthreads();
    const uint32_t a = (al[lev >> 3] >> (7 - (lev & 7))) & 1u;  // Msb0 (lib.rs:106)
    const uint32_t am = 0u - a;
    const uint32_t bm = (bound == 0) ? am : ~am;
    const uint32_t h00 = head[buf][0][0], h10 = head[buf][1][0];
    const uint32_t tl0 = (eo[0][0][0] ^ h00) & 1u, tr0 = (eo[0][1][0] ^ ~h00) & 1u;
    const uint32_t tl1 = (eo[1][0][0] ^ h10) & 1u, tr1 = (eo[1][1][0] ^ ~h10) & 1u;
    const uint32_t tlcw = tl0 ^ tl1 ^ a ^ 1u, trcw = tr0 ^ tr1 ^ a;  // lib.rs:130-131
    const uint32_t tkcw = a ? trcw : tlcw;
    const uint32_t m0 = 0u - t0, m1 = 0u - t1;
    for (uint32_t q = threadIdx.x; q < npieces; q += blockDim.x) {
      const uint4 S0 = w_s0[q], S1 = w_s1[q], VA = w_va[q], BE = be[q];
      uint32_t s0w[4] = {S0.x, S0.y, S0.z, S0.w}, s1w[4] = {S1.x, S1.y, S1.z, S1.w};
      uint32_t vaw[4] = {VA.x, VA.y, VA.z, VA.w};
      const uint32_t bw[4] = {BE.x, BE.y, BE.z, BE.w};
      uint32_t scw[4], vcw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t msk = (q == npieces - 1 && j == 3) ? kMaskLast : 0xFFFFFFFFu;
        // PRG outputs for this piece (see file header)
        const uint32_t sl0 = ((q == 0) ? (eo[0][0][j] ^ s0w[j]) : s0w[j]) & msk;
        const uint32_t vl0 = ((q == 0) ? (eo[0][1][j] ^ ~s0w[j]) : ~s0w[j]) & msk;
        const uint32_t sr0 = ((q == 1) ? (eo[0][2][j] ^ s0w[j]) : s0w[j]) & msk;
        const uint32_t vr0 = ((q == 1) ? (eo[0][3][j] ^ ~s0w[j]) : ~s0w[j]) & msk;
        const uint32_t sl1 = ((q == 0) ? (eo[1][0][j] ^ s1w[j]) : s1w[j]) & msk;
        const uint32_t vl1 = ((q == 0) ? (eo[1][1][j] ^ ~s1w[j]) : ~s1w[j]) & msk;
        const uint32_t sr1 = ((q == 1) ? (eo[1][2][j] ^ s1w[j]) : s1w[j]) & msk;
        const uint32_t vr1 = ((q == 1) ? (eo[1][3][j] ^ ~s1w[j]) : ~s1w[j]) & msk;
        scw[j] = (a ? sl0 : sr0) ^ (a ? sl1 : sr1);                          // lib.rs:112
        vcw[j] = (a ? vl0 : vr0) ^ (a ? vl1 : vr1) ^ vaw[j] ^ (bm & bw[j]);  // lib.rs:113-125
        vaw[j] ^= (a ? vr0 : vl0) ^ (a ? vr1 : vl1) ^ vcw[j];                // lib.rs:126-129
        s0w[j] = (a ? sr0 : sl0) ^ (m0 & scw[j]);                            // lib.rs:139-148
        s1w[j] = (a ? sr1 : sl1) ^ (m1 & scw[j]);
      }
      const uint64_t ci = ((uint64_t)lev * num_keys + k) * lam + 16ull * q;
      *reinterpret_cast<uint4*>(cw_s + ci) = make_uint4(scw[0], scw[1], scw[2], scw[3]);
      *reinterpret_cast<uint4*>(cw_v + ci) = make_uint4(vcw[0], vcw[1], vcw[2], vcw[3]);
      w_s0[q] = make_uint4(s0w[0], s0w[1], s0w[2], s0w[3]);
      w_s1[q] = make_uint4(s1w[0], s1w[1], s1w[2], s1w[3]);
      w_va[q] = make_uint4(vaw[0], vaw[1], vaw[2], vaw[3]);
      if (q < 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          head[buf ^ 1u][0][4 * q + j] = s0w[j];
          head[buf ^ 1u][1][4 * q + j] = s1w[j];
        }
      }
    }
    if (threadIdx.x == 0) cw_t[(uint64_t)lev * num_keys + k] = (uint8_t)(tlcw | (trcw << 1));
    const uint32_t nt0 = (a ? tr0 : tl0) ^ (t0 & tkcw);  // lib.rs:149-152
    const uint32_t nt1 = (a ? tr1 : tl1) ^ (t1 & tkcw);
    t0 = nt0;
    t1 = nt1;
    __syncthreads();
  }
  for (uint32_t q = threadIdx.x; q < npieces; q += blockDim.x) {  // lib.rs:155
    const uint4 S0 = w_s0[q], S1 = w_s1[q], VA = w_va[q];
    *reinterpret_cast<uint4*>(cw_np1 + k * lam + 16ull * q) =
        make_uint4(S0.x ^ S1.x ^ VA.x, S0.y ^ S1.y ^ VA.y, S0.z ^ S1.z ^ VA.z, S0.w ^ S1.w ^ VA.w);
  }
}

// PRG test hook at LAMBDA >= 32: one thread per (seed, 16-byte piece).
__global__ __launch_bounds__(256) void k_prg_wide(const uint32_t* __restrict__ tab, const uint4* __restrict__ rk2,
                                                  const uint8_t* __restrict__ seeds,
                                                  const uint64_t m, const uint32_t lam, uint8_t* __restrict__ out) {
  __shared__ uint32_t t4[1024];
  __shared__ uint32_t rks[2][60];  // ciphers 0 and 17
  load_rk2(rks, rk2);
  load_tab4(t4, tab);
  const uint32_t npieces = lam / 16;
  const uint64_t total = m * npieces;
  const uint64_t row = 4ull * lam + 2;
  for (uint64_t it = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = it / npieces;
    const uint32_t q = (uint32_t)(it % npieces);
    const uint4 sv = *reinterpret_cast<const uint4*>(seeds + g * lam + 16ull * q);
    const uint32_t s[4] = {sv.x, sv.y, sv.z, sv.w};
    uint32_t e[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      e[0][j] = s[j];
      e[1][j] = ~s[j];
    }
    if (q < 2) {
      aes256_small(e[0], rks[q], t4);
      aes256_small(e[1], rks[q], t4);
    }
    uint32_t o[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t msk = (q == npieces - 1 && j == 3) ? kMaskLast : 0xFFFFFFFFu;
      o[0][j] = ((q == 0) ? (e[0][j] ^ s[j]) : s[j]) & msk;
      o[1][j] = ((q == 0) ? (e[1][j] ^ ~s[j]) : ~s[j]) & msk;
      o[2][j] = ((q == 1) ? (e[0][j] ^ s[j]) : s[j]) & msk;
      o[3][j] = ((q == 1) ? (e[1][j] ^ ~s[j]) : ~s[j]) & msk;
    }
    uint8_t* r = out + g * row;
    for (int b = 0; b < 4; ++b)  // rows are 4*LAMBDA+2 bytes: not 16-byte aligned
      for (int j = 0; j < 16; ++j) r[(uint64_t)b * lam + 16ull * q + j] = (uint8_t)(o[b][j >> 2] >> (8 * (j & 3)));
    if (q == 0) {
      r[4ull * lam] = (uint8_t)((e[0][0] ^ s[0]) & 1u);
      r[4ull * lam + 1] = (uint8_t)((e[1][0] ^ ~s[0]) & 1u);
    }
  }
}

}  // namespace
