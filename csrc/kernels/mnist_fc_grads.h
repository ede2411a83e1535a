// The fully connected layers' weight gradients of the MNIST step as wave-level MFMA tiles, shared
// by the kernels that produce them: the world-1 tail (mnist_kernels.hip, SGD applied from the
// accumulators), the DDP gradient tail over RCCL, and the xGMI exchange (xgmi_allreduce.hip, the
// tiles pushed straight to their owners).  One definition, so every form produces the same bits
// (fc1_bwd's job 1 / 3 use the same lane mapping and summation order).
//
//   dW_fc1 [500][800] = dh^T . a2      (K = B)   tile (nt, kt): rows 16 nt.., columns 16 kt..
//   db_fc1 [500]      = column sums of dh          (the kt == 0 tiles)
//   dW_fc2 [10][500]  = d(logits)^T . h (K = B)   tile nt: columns 16 nt..
//   db_fc2 [10]       = column sums of d(logits)   (the nt == 0 tile)
#pragma once
#include "pto_common.h"

namespace pto {

// Sum over the 64 lanes, every lane the same bits: quad xor 1 and 2 and the row half-mirror /
// mirror (DPP on the add), then v_permlane16_swap / v_permlane32_swap pairs (each step adds
// two equal-size partial sums, a + b == b + a, so all lanes round identically).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_allsum_dpp(float x) {
  x += dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_f<0x141>(x);  // row_half_mirror
  x += dpp_f<0x140>(x);  // row_mirror
  {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(s[0]) + __uint_as_float(s[1]);
  }
  {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(s[0]) + __uint_as_float(s[1]);
  }
  return x;
}

// Sum over the four 16-lane rows at this lane's row position (= x + shfl_xor 16, then + shfl_xor
// 32, bit for bit): v_permlane16_swap / v_permlane32_swap pair sums instead of two ds_bpermute
// round trips.
__device__ __forceinline__ float sum_lane_rows(float x) {
  {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(s[0]) + __uint_as_float(s[1]);
  }
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// dW_fc1 tile (nt, kt) of this lane: returns dW_fc1[16 nt + (lane & 15)][16 kt + 4 (lane >> 4) + r]
// in register r (one 16-byte run of the row); dbsum = this lane's share of db_fc1[16 nt + (lane & 15)]
// (complete after sum_lane_rows; meaningful on the kt == 0 tiles).  n >= 500 lanes give zeros.
__device__ __forceinline__ f32x4 fc1_wgrad_tile(const float* __restrict__ dh, const float* __restrict__ a2, int B,
                                                 int nt, int kt, int lane, float& dbsum) {
  const int i = lane & 15, g = lane >> 4;
  const int n = nt * 16 + i, f = kt * 16 + i;
  const bool nv = n < 500;
  const int nc = nv ? n : 499;
  f32x4 c0 = zero4(), c1 = zero4();
  dbsum = 0.f;
  for (int base = 0; base < B; base += 64) {
    float av[16], fv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int bb = min(base + 4 * s + g, B - 1);
      av[s] = dh[(size_t)bb * 500 + nc];
      fv[s] = a2[(size_t)bb * 800 + f];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool bv = base + 4 * s + g < B;
      const float x = (bv && nv) ? av[s] : 0.f;
      dbsum += x;
      const float fb = bv ? fv[s] : 0.f;
      // transposed tile (A = a2 columns, B = dh columns): lane (i, g) ends with
      // dW_fc1[n = 16 nt + i][16 kt + 4 g + r], four consecutive columns -> one 16-B store
      if (s & 1) c1 = mfma16x16x4(fb, x, c1);
      else c0 = mfma16x16x4(fb, x, c0);
    }
  }
  return c0 + c1;
}

// dW_fc2 tile nt of this lane: register r = dW_fc2[4 (lane >> 4) + r][16 nt + (lane & 15)] (rows >= 10
// and columns >= 500 are zero / unused); dbsum = this lane's share of db_fc2[lane & 15] (nt == 0).
__device__ __forceinline__ f32x4 fc2_wgrad_tile(const float* __restrict__ dlog, const float* __restrict__ h, int B,
                                                 int nt, int lane, float& dbsum) {
  const int i = lane & 15, g = lane >> 4;
  const int jc = min(i, 9);
  const int ncl = min(nt * 16 + i, 499);
  f32x4 c0 = zero4(), c1 = zero4();
  dbsum = 0.f;
  for (int base = 0; base < B; base += 64) {
    float av[16], hv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int bb = min(base + 4 * s + g, B - 1);
      av[s] = dlog[(size_t)bb * 10 + jc];
      hv[s] = h[(size_t)bb * 500 + ncl];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool bv = base + 4 * s + g < B;
      const float x = (bv && i < 10) ? av[s] : 0.f;
      dbsum += x;
      const float hb = bv ? hv[s] : 0.f;
      if (s & 1) c1 = mfma16x16x4(x, hb, c1);
      else c0 = mfma16x16x4(x, hb, c0);
    }
  }
  return c0 + c1;
}

// The step's loss sum and correct count, (sum of per_sample[2 b], sum of per_sample[2 b + 1]) over the
// B samples, every lane the same bits: loss_stats_load issues the first 64 samples' loads (early, in
// flight with a tile's operand loads), loss_stats_finish adds the rest and sums over the wave.
__device__ __forceinline__ void loss_stats_load(const float* __restrict__ per_sample, int B, int lane, float& ls,
                                                float& cs) {
  ls = 0.f;
  cs = 0.f;
  if (lane < B) { ls = per_sample[2 * lane]; cs = per_sample[2 * lane + 1]; }
}
__device__ __forceinline__ void loss_stats_finish(const float* __restrict__ per_sample, int B, int lane, float& ls,
                                                  float& cs) {
  for (int bb = lane + 64; bb < B; bb += 64) { ls += per_sample[2 * bb]; cs += per_sample[2 * bb + 1]; }
  ls = wave_allsum_dpp(ls);
  cs = wave_allsum_dpp(cs);
}

}  // namespace pto
