// 3x3 / stride 2 / pad 1 max-pool for channels-last (NHWC) bf16 activations -- the ResNet-50
// stem pool (B=256: a 411 MB input, the largest activation of the step).
//
// PyTorch-ROCm's max_pool2d_with_indices stores an int64 index per output element (411 MB at
// B=256, as large as the input) and reads it back in the backward.  Here the forward stores
// the winning tap of each output channel as one byte (kh * 3 + kw), and the backward is a
// gather: every input pixel sums the gradients of the <= 4 windows that cover it and chose
// it, in PyTorch's (oh, ow) order with an fp32 accumulator -- no atomics, no zero fill,
// deterministic.  Max semantics follow PyTorch's kernel: the first maximum in (kh, kw) scan
// order wins, a NaN replaces the running maximum (so the last NaN's tap is kept).
//
// Layout: x [N][H][W][C], C a multiple of 8; one thread per (pixel, 8 channels): 16-byte
// loads/stores of bf16, 8-byte stores of the tap bytes.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int P_NT = 256;

__device__ __forceinline__ void ld8(const uint16_t* p, float (&v)[8]) {
  const uint4 r = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint32_t rne16(float f) {  // fp32 -> bf16 bits, round to nearest even
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return 0x7fc0u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ void st8(uint16_t* p, const float (&v)[8]) {
  uint4 r;
  r.x = rne16(v[0]) | (rne16(v[1]) << 16);
  r.y = rne16(v[2]) | (rne16(v[3]) << 16);
  r.z = rne16(v[4]) | (rne16(v[5]) << 16);
  r.w = rne16(v[6]) | (rne16(v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = r;
}

// y[n, oh, ow, c] = max over the 3x3 window at (2oh - 1, 2ow - 1); tap[n, oh, ow, c] = argmax
__global__ __launch_bounds__(P_NT) void maxpool3s2_fwd_kernel(const uint16_t* __restrict__ x,
                                                              uint16_t* __restrict__ y,
                                                              uint8_t* __restrict__ tap, int N, int H, int W,
                                                              int C, int OH, int OW) {
  const int cg = C >> 3;
  const long total = (long)N * OH * OW * cg;
  for (long t = (long)blockIdx.x * P_NT + threadIdx.x; t < total; t += (long)gridDim.x * P_NT) {
    const int c8 = (int)(t % cg);
    long r = t / cg;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    const int h0 = 2 * oh - 1, w0 = 2 * ow - 1;
    // every in-bounds tap's load first (one memory round), then the scan
    float v[9][8];
    bool ok[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ih = h0 + kh, iw = w0 + kw, k = kh * 3 + kw;
        ok[k] = ih >= 0 && ih < H && iw >= 0 && iw < W;
        const int ihc = min(max(ih, 0), H - 1), iwc = min(max(iw, 0), W - 1);
        ld8(x + (((long)n * H + ihc) * W + iwc) * C + c8 * 8, v[k]);
      }
    float m[8];
    uint8_t a[8];
    int first = 0;
#pragma unroll
    for (int k = 8; k >= 0; --k)
      if (ok[k]) first = k;
#pragma unroll
    for (int j = 0; j < 8; ++j) { m[j] = -__builtin_inff(); a[j] = (uint8_t)first; }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (!ok[k]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[k][j] > m[j] || __builtin_isnan(v[k][j])) { m[j] = v[k][j]; a[j] = (uint8_t)k; }
    }
    const long o = (((long)n * OH + oh) * OW + ow) * C + c8 * 8;
    st8(y + o, m);
    uint2 pk;
    pk.x = a[0] | (a[1] << 8) | (a[2] << 16) | ((uint32_t)a[3] << 24);
    pk.y = a[4] | (a[5] << 8) | (a[6] << 16) | ((uint32_t)a[7] << 24);
    *reinterpret_cast<uint2*>(tap + o) = pk;
  }
}

// dx[n, ih, iw, c] = sum over windows (oh, ow) covering (ih, iw) whose tap chose it of dy
__global__ __launch_bounds__(P_NT) void maxpool3s2_bwd_kernel(const uint16_t* __restrict__ dy,
                                                              const uint8_t* __restrict__ tap,
                                                              uint16_t* __restrict__ dx, int N, int H, int W,
                                                              int C, int OH, int OW) {
  const int cg = C >> 3;
  const long total = (long)N * H * W * cg;
  for (long t = (long)blockIdx.x * P_NT + threadIdx.x; t < total; t += (long)gridDim.x * P_NT) {
    const int c8 = (int)(t % cg);
    long r = t / cg;
    const int iw = (int)(r % W);
    r /= W;
    const int ih = (int)(r % H);
    const int n = (int)(r / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // ih = 2 oh - 1 + kh: kh = 2, 1, 0 visits oh in increasing order (PyTorch's loop order)
#pragma unroll
    for (int kh = 2; kh >= 0; --kh) {
      const int th = ih + 1 - kh;
      if (th < 0 || (th & 1) || (th >> 1) >= OH) continue;
      const int oh = th >> 1;
#pragma unroll
      for (int kw = 2; kw >= 0; --kw) {
        const int tw = iw + 1 - kw;
        if (tw < 0 || (tw & 1) || (tw >> 1) >= OW) continue;
        const int ow = tw >> 1;
        const long o = (((long)n * OH + oh) * OW + ow) * C + c8 * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(tap + o);
        float g[8];
        ld8(dy + o, g);
        const uint8_t want = (uint8_t)(kh * 3 + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint8_t a = (uint8_t)(((j < 4 ? pk.x : pk.y) >> (8 * (j & 3))) & 0xffu);
          if (a == want) acc[j] += g[j];
        }
      }
    }
    st8(dx + (((long)n * H + ih) * W + iw) * C + c8 * 8, acc);
  }
}

int grid_for(long total) {
  long g = (total + P_NT - 1) / P_NT;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

// x [N][H][W][C] bf16 -> y [N][OH][OW][C] bf16 + tap bytes [N][OH][OW][C]; OH = (H - 1) / 2 + 1.
int pto_maxpool3s2_fwd(const void* x, void* y, void* tap, int N, int H, int W, int C, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || (C & 7) || !aligned16(x) || !aligned16(y) ||
      (reinterpret_cast<uintptr_t>(tap) & 7))
    return -2;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long total = (long)N * OH * OW * (C >> 3);
  hipLaunchKernelGGL(maxpool3s2_fwd_kernel, dim3(grid_for(total)), dim3(P_NT), 0, (hipStream_t)stream,
                     static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), static_cast<uint8_t*>(tap), N, H,
                     W, C, OH, OW);
  return (int)hipGetLastError();
}

int pto_maxpool3s2_bwd(const void* dy, const void* tap, void* dx, int N, int H, int W, int C, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || (C & 7) || !aligned16(dy) || !aligned16(dx) ||
      (reinterpret_cast<uintptr_t>(tap) & 7))
    return -2;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long total = (long)N * H * W * (C >> 3);
  hipLaunchKernelGGL(maxpool3s2_bwd_kernel, dim3(grid_for(total)), dim3(P_NT), 0, (hipStream_t)stream,
                     static_cast<const uint16_t*>(dy), static_cast<const uint8_t*>(tap), static_cast<uint16_t*>(dx),
                     N, H, W, C, OH, OW);
  return (int)hipGetLastError();
}

}  // extern "C"
