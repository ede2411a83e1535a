// Shared pieces of the flash-attention kernels (attention.hip, attention_bwd_pipe.hip): operand
// types, the MFMA / LDS-image helpers, tile staging and the launch-order map.  See attention.hip
// for the layout and MFMA plan.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t bf16_t;
// native clang vectors (HIP's u32x4 is a struct: copies of it into arrays become memcpys that
// keep the staging arrays in scratch)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int D = 128;       // head dim (the 8B / 70B Llama-3 value)
constexpr int NDS = D / 16;  // k-steps of a d-contraction
constexpr int NDT = D / 32;  // 32-wide output tiles along d
constexpr int BM = 128;      // query rows per forward / dQ workgroup (32 per wave)
constexpr int BN = 64;       // keys per K/V tile
constexpr int BK = 128;      // keys per dK/dV workgroup (32 per wave)
constexpr int QT = 32;       // query rows per dK/dV tile
constexpr int NT = 256;
constexpr int CH = D / 8;    // 16-byte chunks per row (16)
constexpr int NT8 = 512;     // 8-wave workgroups (two waves per SIMD)
constexpr int BM8 = 256;     // query rows per 8-wave forward / dQ workgroup
constexpr float DEFER = 8.f; // deferred-rescale threshold of the 8-wave forward (log2 units)

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// XOR-swizzled image of a [rows][128] bf16 tile, in 16-byte units: chunk ch of row r.
// Row reads of 16 consecutive rows at one chunk and transposed 4-row x 16-column reads both
// hit 64 distinct banks.
__device__ __forceinline__ int xo(int r, int ch) { return r * CH + (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// registers 8s..8s+7 of an accumulator as a bf16 MFMA operand (k-step s)
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  u32x4 u;
  u.x = pk_bf16(a[8 * s + 0], a[8 * s + 1]);
  u.y = pk_bf16(a[8 * s + 2], a[8 * s + 3]);
  u.z = pk_bf16(a[8 * s + 4], a[8 * s + 5]);
  u.w = pk_bf16(a[8 * s + 6], a[8 * s + 7]);
  return __builtin_bit_cast(bf16x8, u);
}

// operand whose k runs along the tile's COLUMNS: element j <- [row][ch*8 + j]
__device__ __forceinline__ bf16x8 row_frag(const u32x4* tile, int row, int ch) {
  return __builtin_bit_cast(bf16x8, tile[xo(row, ch)]);
}

__device__ __forceinline__ s16x4 tr_read(const u32x4* tile, int row, int ch, int sub_bytes) {
  const char* p = reinterpret_cast<const char*>(tile + xo(row, ch)) + sub_bytes;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// operand whose k runs along the tile's ROWS, in the accumulator-as-operand order: element j
// of lane half h <- row rbase + 8*(j>>2) + 4h + (j&3), column cbase + (lane & 31).
__device__ __forceinline__ bf16x8 tr_frag(const u32x4* tile, int rbase, int cbase, int lane) {
  const int l16 = lane & 15, q = l16 >> 2, p = l16 & 3;
  const int col = cbase + 16 * ((lane >> 4) & 1) + 4 * p;
  const int r0 = rbase + 4 * (lane >> 5) + q;
  const s16x4 lo = tr_read(tile, r0, col >> 3, (col & 7) * 2);
  const s16x4 hi = tr_read(tile, r0 + 8, col >> 3, (col & 7) * 2);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v;
  v.lo = lo;
  v.hi = hi;
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// combine a lane's value with lane ^ 32's (v_permlane32_swap: one VALU op, no LDS round trip);
// both halves get the same result (lower half's value first)
__device__ __forceinline__ float half_max(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return max3(__uint_as_float(s[0]), __uint_as_float(s[1]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// key/query row index of accumulator register i in lane half h (C/D map of 32x32x16)
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }

// Stage a [ROWS][128] bf16 tile (rows ROWS apart in global by `stride` elements) into the
// XOR image: each thread moves ROWS*16/NT 16-byte chunks.
template <int ROWS, int NTH = NT>
struct Stage {
  static constexpr int N = ROWS * CH / NTH;
  u32x4 r[N];
  __device__ __forceinline__ void load(const bf16_t* base, size_t stride, int tid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int e = tid + NTH * i, row = e / CH, ch = e % CH;
      r[i] = *reinterpret_cast<const u32x4*>(base + (size_t)row * stride + ch * 8);
    }
  }
  __device__ __forceinline__ void store(u32x4* tile, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int e = tid + NTH * i, row = e / CH, ch = e % CH;
      tile[xo(row, ch)] = r[i];
    }
  }
};

// The same XOR image filled by LDS-DMA (global_load_lds_dwordx4: no staging registers).  A
// wave-instruction writes 64 consecutive 16-byte slots (wave-uniform base + 16 x lane), so the
// swizzle moves to the per-lane SOURCE address: slot j of row R holds chunk j ^ swz(R).  Wave w
// issues pieces w, w + NW, ...  The LDS writes count on vmcnt: __syncthreads() retires them.
template <int ROWS, int NTH>
__device__ __forceinline__ void glds_tile(const bf16_t* base, size_t stride, u32x4* tile, int tid) {
  constexpr int NP = ROWS * CH / 64, NW = NTH / 64;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  static_assert(NP % NW == 0, "whole pieces per wave");
#pragma unroll
  for (int i = 0; i < NP / NW; ++i) {
    const int p = w + NW * i;
    const int e = 64 * p + lane, row = e / CH, j = e % CH;
    const int ch = j ^ (((row & 3) << 2) | ((row >> 2) & 3));
    __builtin_amdgcn_global_load_lds(base + (size_t)row * stride + ch * 8,
                                     (__attribute__((address_space(3))) void*)(tile + 64 * p), 16, 0, 0);
  }
}

// glds_tile with the LDS-DMA issued from inline asm.  The compiler cannot see that these loads
// write LDS, so it no longer puts an `s_waitcnt vmcnt(0)` in front of the next LDS read (with the
// builtin it must assume any LDS read may alias the DMA target, so every tile waited for the
// NEXT tile's prefetch before computing: the prefetch never overlapped anything).  The caller
// owns the ordering: `s_waitcnt vmcnt(0)` before the barrier that publishes the tile.
template <int ROWS, int NTH>
__device__ __forceinline__ void glds_tile_asm(const bf16_t* base, size_t stride, u32x4* tile, int tid) {
  constexpr int NP = ROWS * CH / 64, NW = NTH / 64;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  static_assert(NP % NW == 0, "whole pieces per wave");
#pragma unroll
  for (int i = 0; i < NP / NW; ++i) {
    const int p = w + NW * i;
    const int e = 64 * p + lane, row = e / CH, j = e % CH;
    const int ch = j ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const bf16_t* src = base + (size_t)row * stride + ch * 8;
    const unsigned dst = (unsigned)(uintptr_t)(tile + 64 * p);  // LDS byte address, wave-uniform
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                 :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(src) : "memory", "m0");
  }
}
__device__ __forceinline__ void glds_dword_asm(const float* src, float* lds_dst) {
  const unsigned dst = (unsigned)(uintptr_t)lds_dst;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off"
               :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(src) : "memory", "m0");
}

// Write a wave's 32 x 128 transposed accumulator (acc[dt] reg i = [d = dt*32 + acc_row(i,h)]
// [col = lane & 31]) as rows [col][d] bf16 to global via the wave's LDS region (8 KB).
__device__ __forceinline__ void store_rows_T(const f32x16 (&acc)[NDT], float scale, u32x4* stage, int lane,
                                             bf16_t* out, size_t row_stride) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = dt * 32 + 8 * g + 4 * h;
      u32x2 w;
      w.x = pk_bf16(acc[dt][4 * g + 0] * scale, acc[dt][4 * g + 1] * scale);
      w.y = pk_bf16(acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale);
      *reinterpret_cast<u32x2*>(reinterpret_cast<char*>(stage + xo(c, d0 >> 3)) + (d0 & 7) * 2) = w;
    }
  __syncthreads();  // every wave calls this together (after its tile loop)
#pragma unroll
  for (int i = 0; i < 32 * CH / 64; ++i) {
    const int e = lane + 64 * i, row = e / CH, ch = e % CH;
    *reinterpret_cast<u32x4*>(out + (size_t)row * row_stride + ch * 8) = stage[xo(row, ch)];
  }
}

// store_rows_T for a wave whose staging region no other wave touches any more (after the last
// tile's barrier): the hand-off from this wave's LDS writes to its own reads needs no block
// barrier (one wave's LDS operations complete in order)
__device__ __forceinline__ void store_rows_T_wave(const f32x16 (&acc)[NDT], float scale, u32x4* stage, int lane,
                                                  bf16_t* out, size_t row_stride) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = dt * 32 + 8 * g + 4 * h;
      u32x2 w;
      w.x = pk_bf16(acc[dt][4 * g + 0] * scale, acc[dt][4 * g + 1] * scale);
      w.y = pk_bf16(acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale);
      *reinterpret_cast<u32x2*>(reinterpret_cast<char*>(stage + xo(c, d0 >> 3)) + (d0 & 7) * 2) = w;
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int i = 0; i < 32 * CH / 64; ++i) {
    const int e = lane + 64 * i, row = e / CH, ch = e % CH;
    *reinterpret_cast<u32x4*>(out + (size_t)row * row_stride + ch * 8) = stage[xo(row, ch)];
  }
}

// Forward / dQ workgroup -> (query block, batch, q head, kv head).  The query block is the
// slowest index of the launch order, heaviest (last) block first under the causal mask, so
// the light blocks fill in behind the heavy ones across the whole grid.
__device__ __forceinline__ void block_coords(int S, int B, int Hq, int Hkv, int causal, int& qblk, int& b, int& hq,
                                             int& hk) {
  const int nqb = S / BM, qi = (int)blockIdx.x / (B * Hq), bh = (int)blockIdx.x % (B * Hq);
  qblk = causal ? nqb - 1 - qi : qi;
  b = bh / Hq;
  hq = bh % Hq;
  hk = hq / (Hq / Hkv);
}

}  // namespace
