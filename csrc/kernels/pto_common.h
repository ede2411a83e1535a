// Shared device helpers for the MI355X (gfx950 / CDNA4) data-plane kernels.
//
// Everything here is written for 64-lane wavefronts and the exact-fp32 MFMA
// (`v_mfma_f32_16x16x4_f32`): the reference workload (examples/mnist/mnist.py:17-43
// in jiaqianjing/pytorch-operator) trains in fp32, so the matrix cores are used at
// full fp32 precision (no bf16 down-cast, no TF32-like shortcut exists on gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pto {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// D = A*B + C for one 16x16 fp32 tile, K=4 per instruction.
// Lane maps (gfx950, verified by tests/test_kernels_gpu.py::test_mfma_layout):
//   A[i = lane & 15][k = lane >> 4]    B[k = lane >> 4][j = lane & 15]
//   C/D: col = lane & 15, row = (lane >> 4) * 4 + reg
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Where the training batch comes from.  The harness keeps the whole synthetic
// dataset resident in HBM as uint8 pixels (60000 x 784 B = 47 MB -- nothing on a
// 288 GB part) and a per-epoch permutation; the batch for step `cursor[0]` is a
// gather through that permutation, so a captured hipGraph replays successive
// batches without host involvement.  ToTensor()+Normalize((0.1307,),(0.3081,))
// (examples/mnist/mnist.py:122-123) is folded into the load as `px*scale+shift`.
struct BatchSrc {
  const void* x;        // [n_total, 784] uint8 or fp32
  const int* labels;    // [n_total] int32 (nullable when unused)
  const int* perm;      // [n_total] sample order (nullable: identity, batch = rows 0..B-1)
  const int* cursor;    // device step counter (nullable: use host_offset)
  int host_offset;      // first permutation slot of this batch when cursor == nullptr
  int n_total;          // dataset size (for wrap-around)
  int is_u8;            // 1: uint8 pixels, 0: fp32
  float scale, shift;   // x_norm = x * scale + shift
};

__device__ __forceinline__ int batch_row(const BatchSrc& s, int b, int B) {
  if (s.perm == nullptr) return b;
  long long base = s.cursor ? ((long long)s.cursor[0] * B) % s.n_total : s.host_offset;
  long long i = base + b;
  if (i >= s.n_total) i -= s.n_total;
  return s.perm[i];
}

__device__ __forceinline__ float load_px(const BatchSrc& s, int row, int e) {
  float v = s.is_u8 ? (float)((const uint8_t*)s.x)[(size_t)row * 784 + e]
                    : ((const float*)s.x)[(size_t)row * 784 + e];
  return v * s.scale + s.shift;
}

}  // namespace pto
