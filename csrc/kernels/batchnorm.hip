// Training-mode BatchNorm2d for channels-last (NHWC) activations with the ReLU and the
// residual add of a ResNet bottleneck fused in -- the ResNet-50 worker's memory-bound
// half.  PyTorch-ROCm runs this as MIOpen's mean/variance + normalise kernels plus separate
// clamp / add / threshold-backward passes (profiles/r2_resnet50_kernels.md: 58 % of the
// step in BN + elementwise); here the forward is 1 read (statistics) + 1 read/1 write
// (normalise + add + ReLU), the backward 2 reads (reductions) + 2 reads/1 write (dx), with
// the ReLU mask recomputed from x where no residual was added.
//
// Layout: x [M = N*H*W][C], C/8 threads per row each owning 8 consecutive channels
// (one 16-byte bf16 or two 16-byte fp32 accesses), C/8 a divisor of 256 (C = 8 .. 2048).
// Statistics are fp32: per-thread shifted sums (shift = the thread's first value), turned
// into (mean, M2) and merged with Chan's pairwise update inside the block and across blocks
// in a fixed order -- accurate for large means, deterministic.  Running stats follow
// PyTorch (momentum, unbiased variance).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>

namespace {

constexpr int BN_NT = 256;
constexpr int FIN_CH = 16;  // finalize blocks: 16 channels x 64 partial groups = 1024 threads
constexpr int FIN_G = 64;
constexpr int FIN_NT = FIN_CH * FIN_G;
#ifndef PTO_BN_FIN_BATCH
#define PTO_BN_FIN_BATCH 1  // finalize: all of a thread's partials loaded at once (0: one per loop trip)
#endif
constexpr int FIN_GMAX = 1024;               // pto_bn_plan's cap on the reduction grid
constexpr int FIN_IT = FIN_GMAX / FIN_G;     // partials per finalize thread, loaded together

typedef __hip_bfloat16 bf16;

template <typename T>
struct V8;
template <>
struct V8<float> {
  static __device__ __forceinline__ void ld(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void st(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};
__device__ __forceinline__ uint32_t rne16(float f) {  // fp32 -> bf16 bits, round to nearest even
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return 0x7fc0u;  // NaN stays NaN
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
template <>
struct V8<bf16> {
  static __device__ __forceinline__ void ld(const bf16* p, float (&v)[8]) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void st(bf16* p, const float (&v)[8]) {
    uint4 r;
    r.x = rne16(v[0]) | (rne16(v[1]) << 16);
    r.y = rne16(v[2]) | (rne16(v[3]) << 16);
    r.z = rne16(v[4]) | (rne16(v[5]) << 16);
    r.w = rne16(v[6]) | (rne16(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = r;
  }
};

// (n, mean, M2) += (nb, mb, m2b)   (Chan et al. pairwise update)
__device__ __forceinline__ void chan(float& n, float& m, float& m2, float nb, float mb, float m2b) {
  if (nb <= 0.f) return;
  const float nn = n + nb, d = mb - m, f = nb / nn;
  m += d * f;
  m2 += m2b + d * d * n * f;
  n = nn;
}

// ---- forward 1: per-block (mean, M2) of every channel over rows [blk*rpb, +rpb)
template <typename T>
__global__ __launch_bounds__(BN_NT) void bn_stats_kernel(const T* __restrict__ x, long M, int C, int rpb,
                                                         float* __restrict__ part, float* __restrict__ part_n) {
  __shared__ float s_m[BN_NT * 8], s_q[BN_NT * 8], s_n[BN_NT];
  const int tpr = C >> 3, rpi = BN_NT / tpr, tid = threadIdx.x;
  const int slot = tid / tpr, cv = tid - slot * tpr;
  const long r0 = (long)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  float k[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s1[8], s2[8];
  int n = 0;
  const long rf = r0 + slot;
  if (rf < r1) V8<T>::ld(x + rf * C + cv * 8, k);
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  long r = rf;
  for (; r + 3 * rpi < r1; r += 4 * rpi) {  // 4 rows in flight per thread
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) V8<T>::ld(x + (r + u * rpi) * C + cv * 8, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[u][j] - k[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    n += 4;
  }
  for (; r < r1; r += rpi) {
    float v[8];
    V8<T>::ld(x + r * C + cv * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[j] - k[j];
      s1[j] += d;
      s2[j] = fmaf(d, d, s2[j]);
    }
    ++n;
  }
  if (slot < rpi) {
    const float fn = (float)n;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float mean = n ? k[j] + s1[j] / fn : 0.f;
      const float m2 = n ? fmaxf(s2[j] - s1[j] * s1[j] / fn, 0.f) : 0.f;
      s_m[slot * C + cv * 8 + j] = mean;
      s_q[slot * C + cv * 8 + j] = m2;
    }
    if (cv == 0) s_n[slot] = fn;
  }
  __syncthreads();
  for (int c = tid; c < C; c += BN_NT) {
    float nn = 0.f, m = 0.f, q = 0.f;
    for (int s = 0; s < rpi; ++s) chan(nn, m, q, s_n[s], s_m[s * C + c], s_q[s * C + c]);
    part[(size_t)blockIdx.x * 2 * C + c] = m;
    part[(size_t)blockIdx.x * 2 * C + C + c] = q;
  }
  if (tid == 0) part_n[blockIdx.x] = (float)(r1 > r0 ? r1 - r0 : 0);
}

// ---- forward 2: merge the G partials; mean / rstd for the backward, scale/shift for the
// apply kernel, running statistics (and num_batches_tracked) updated in place
__global__ __launch_bounds__(FIN_NT) void bn_stats_finalize_kernel(
    const float* __restrict__ part, const float* __restrict__ part_n, int G, int C, float eps, float momentum,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, float* __restrict__ ss, float* __restrict__ run_mean,
    float* __restrict__ run_var, long long* __restrict__ nbt) {
  __shared__ float s_n[FIN_G][FIN_CH], s_m[FIN_G][FIN_CH], s_q[FIN_G][FIN_CH];
  const int pg = threadIdx.x / FIN_CH, cl = threadIdx.x % FIN_CH, c = blockIdx.x * FIN_CH + cl;
  float n = 0.f, m = 0.f, q = 0.f;
#if !PTO_BN_FIN_BATCH
  if (c < C)
    for (int g = pg; g < G; g += FIN_G) chan(n, m, q, part_n[g], part[(size_t)g * 2 * C + c], part[(size_t)g * 2 * C + C + c]);
#else
  {
    // every partial of this thread in flight at once (G <= FIN_GMAX), then merged in g order
    float pn[FIN_IT], pm[FIN_IT], pq[FIN_IT];
    const int cc = c < C ? c : 0;
#pragma unroll
    for (int i = 0; i < FIN_IT; ++i) {
      const int g = pg + FIN_G * i, gg = g < G ? g : 0;
      pn[i] = part_n[gg];
      pm[i] = part[(size_t)gg * 2 * C + cc];
      pq[i] = part[(size_t)gg * 2 * C + C + cc];
      if (g >= G || c >= C) pn[i] = 0.f;  // chan() skips empty partials
    }
#pragma unroll
    for (int i = 0; i < FIN_IT; ++i) chan(n, m, q, pn[i], pm[i], pq[i]);
  }
#endif
  s_n[pg][cl] = n; s_m[pg][cl] = m; s_q[pg][cl] = q;
  __syncthreads();
  for (int w = FIN_G / 2; w >= 1; w >>= 1) {  // fixed-shape tree: deterministic
    if (pg < w) {
      chan(n, m, q, s_n[pg + w][cl], s_m[pg + w][cl], s_q[pg + w][cl]);
      s_n[pg][cl] = n; s_m[pg][cl] = m; s_q[pg][cl] = q;
    }
    __syncthreads();
  }
  if (pg == 0 && c < C) {
    const float var = n > 0.f ? q / n : 0.f;
    const float rstd = rsqrtf(var + eps);
    const float sc = gamma[c] * rstd;
    mean_out[c] = m;
    rstd_out[c] = rstd;
    ss[c] = sc;
    ss[C + c] = beta[c];
    if (run_mean != nullptr) {
      const float unb = n > 1.f ? q / (n - 1.f) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * m;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
    }
  }
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

// ---- forward 3: y = (x - mean) * scale + beta [+ z] [ReLU] (centred first: no cancellation
// of x * scale against mean * scale near the ReLU boundary); the grid stride is a multiple
// of C/8, so a thread's channels (and its per-channel registers) never change
// MOUT: also write the ReLU mask as one byte per 8-channel vector (bit j: stored y > 0), which
// the backward reads instead of y (1/16 of its bytes)
template <typename T>
__device__ __forceinline__ uint32_t pos_bits(const float (&v)[8]) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // the value as stored (bf16: rounded) is > 0; v >= 0 after the ReLU
    const bool p = sizeof(T) == 2 ? (v[j] > 0.f && rne16(v[j]) != 0u) : v[j] > 0.f;
    b |= (uint32_t)p << j;
  }
  return b;
}

template <typename T, bool RELU, bool RES, bool MOUT = false>
__global__ __launch_bounds__(BN_NT) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ z,
                                                         const float* __restrict__ ss,
                                                         const float* __restrict__ mean, T* __restrict__ y,
                                                         long nvec, int C, uint8_t* __restrict__ mo) {
  const int tpr = C >> 3;
  const long i0 = (long)blockIdx.x * BN_NT + threadIdx.x, stride = (long)gridDim.x * BN_NT;
  const int cv = (int)(i0 % tpr);
  float sc[8], sh[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = ss[cv * 8 + j]; sh[j] = ss[C + cv * 8 + j]; mu[j] = mean[cv * 8 + j]; }
  long i = i0;
  for (; i + stride < nvec; i += 2 * stride) {
    float a[2][8], b[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      V8<T>::ld(x + (i + u * stride) * 8, a[u]);
      if (RES) V8<T>::ld(z + (i + u * stride) * 8, b[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = fmaf(a[u][j] - mu[j], sc[j], sh[j]);
        if (RES) v += b[u][j];
        a[u][j] = RELU ? fmaxf(v, 0.f) : v;
      }
      V8<T>::st(y + (i + u * stride) * 8, a[u]);
      if (MOUT) mo[i + u * stride] = (uint8_t)pos_bits<T>(a[u]);
    }
  }
  for (; i < nvec; i += stride) {
    float a[8], b[8];
    V8<T>::ld(x + i * 8, a);
    if (RES) V8<T>::ld(z + i * 8, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = fmaf(a[j] - mu[j], sc[j], sh[j]);
      if (RES) v += b[j];
      a[j] = RELU ? fmaxf(v, 0.f) : v;
    }
    V8<T>::st(y + i * 8, a);
    if (MOUT) mo[i] = (uint8_t)pos_bits<T>(a);
  }
}

// ReLU mask of the backward: MASK 0 = no ReLU, 1 = recompute (x-mean)*scale+beta > 0 (bitwise
// the forward's value), 2 = y > 0 (a residual was added before the ReLU), 3 = the same mask
// from the forward's bit image (one byte per 8-channel vector, passed in place of y).
// ADD2: the output has two consumers whose gradients arrive separately (a bottleneck's output
// feeds the next block's conv1 AND, as the identity, its residual add): g = dy + dy2, summed
// in fp32 here instead of by an extra elementwise pass over the activation.
template <typename T, int MASK, bool ADD2>
__device__ __forceinline__ void masked_grad(const T* dy, const T* dy2, const T* x, const T* y, long e,
                                            const float (&sc)[8], const float (&sh)[8], const float (&mu)[8],
                                            float (&g)[8], float (&xv)[8]) {
  V8<T>::ld(dy + e, g);
  if (ADD2) {
    float g2[8];
    V8<T>::ld(dy2 + e, g2);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] += g2[j];
  }
  V8<T>::ld(x + e, xv);
  if (MASK == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = fmaf(xv[j] - mu[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
  } else if (MASK == 2) {
    float yv[8];
    V8<T>::ld(y + e, yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
  } else if (MASK == 3) {
    const uint32_t bits = reinterpret_cast<const uint8_t*>(y)[e >> 3];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (bits >> j) & 1u ? g[j] : 0.f;
  }
}

#ifndef PTO_BN_GOUT
#define PTO_BN_GOUT 1  // residual BNs: the reduce pass writes g (= dz), the dx pass reads it back
#endif

// g as the activation dtype stores it (bf16: round to nearest even)
template <typename T>
__device__ __forceinline__ void round_t(float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(rne16(v[j]) << 16);
  }
}

// ---- backward 1: per-block sums of g and g * (x - mean) per channel.  GOUT (residual BNs,
// whose masked g is also the residual's gradient dz): g is rounded to T, summed as rounded and
// stored to gout, so the dx pass reads that one tensor instead of dy [+ dy2] and the mask again
template <typename T, int MASK, bool ADD2, bool GOUT = false>
__global__ __launch_bounds__(BN_NT) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                              const T* __restrict__ x,
                                                              const T* __restrict__ y, const float* __restrict__ ss,
                                                              const float* __restrict__ mean, long M, int C, int rpb,
                                                              float* __restrict__ part, T* __restrict__ gout) {
  __shared__ float s_a[BN_NT * 8], s_b[BN_NT * 8];
  const int tpr = C >> 3, rpi = BN_NT / tpr, tid = threadIdx.x;
  const int slot = tid / tpr, cv = tid - slot * tpr;
  const long r0 = (long)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  float sc[8], sh[8], mu[8], a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = ss[cv * 8 + j]; sh[j] = ss[C + cv * 8 + j]; mu[j] = mean[cv * 8 + j];
    a[j] = 0.f; b[j] = 0.f;
  }
  long r = r0 + slot;
  for (; r + rpi < r1; r += 2 * rpi) {
    float g[2][8], xv[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u)
      masked_grad<T, MASK, ADD2>(dy, dy2, x, y, (r + u * rpi) * C + cv * 8, sc, sh, mu, g[u], xv[u]);
    if (GOUT) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        round_t<T>(g[u]);
        V8<T>::st(gout + (r + u * rpi) * C + cv * 8, g[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] += g[u][j]; b[j] = fmaf(g[u][j], xv[u][j] - mu[j], b[j]); }
  }
  for (; r < r1; r += rpi) {
    float g[8], xv[8];
    masked_grad<T, MASK, ADD2>(dy, dy2, x, y, r * C + cv * 8, sc, sh, mu, g, xv);
    if (GOUT) {
      round_t<T>(g);
      V8<T>::st(gout + r * C + cv * 8, g);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] += g[j]; b[j] = fmaf(g[j], xv[j] - mu[j], b[j]); }
  }
  if (slot < rpi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { s_a[slot * C + cv * 8 + j] = a[j]; s_b[slot * C + cv * 8 + j] = b[j]; }
  }
  __syncthreads();
  for (int c = tid; c < C; c += BN_NT) {
    float sa = 0.f, sb = 0.f;
    for (int s = 0; s < rpi; ++s) { sa += s_a[s * C + c]; sb += s_b[s * C + c]; }
    part[(size_t)blockIdx.x * 2 * C + c] = sa;
    part[(size_t)blockIdx.x * 2 * C + C + c] = sb;
  }
}

// ---- backward 2: dgamma, dbeta and the per-channel dx = ca*g + cb*(x - mean) + cc coefficients
// (x - mean, not x: no cancellation against a large mean)
__global__ __launch_bounds__(FIN_NT) void bn_bwd_finalize_kernel(const float* __restrict__ part, int G, int C, long M,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                float* __restrict__ coef) {
  __shared__ float s_a[FIN_G][FIN_CH], s_b[FIN_G][FIN_CH];
  const int pg = threadIdx.x / FIN_CH, cl = threadIdx.x % FIN_CH, c = blockIdx.x * FIN_CH + cl;
  float a = 0.f, b = 0.f;
#if !PTO_BN_FIN_BATCH
  if (c < C)
    for (int g = pg; g < G; g += FIN_G) { a += part[(size_t)g * 2 * C + c]; b += part[(size_t)g * 2 * C + C + c]; }
#else
  {
    float pa[FIN_IT], pb[FIN_IT];
    const int cc = c < C ? c : 0;
#pragma unroll
    for (int i = 0; i < FIN_IT; ++i) {
      const int g = pg + FIN_G * i, gg = g < G ? g : 0;
      pa[i] = part[(size_t)gg * 2 * C + cc];
      pb[i] = part[(size_t)gg * 2 * C + C + cc];
    }
#pragma unroll
    for (int i = 0; i < FIN_IT; ++i)
      if (pg + FIN_G * i < G && c < C) { a += pa[i]; b += pb[i]; }
  }
#endif
  s_a[pg][cl] = a; s_b[pg][cl] = b;
  __syncthreads();
  for (int w = FIN_G / 2; w >= 1; w >>= 1) {
    if (pg < w) {
      a += s_a[pg + w][cl]; b += s_b[pg + w][cl];
      s_a[pg][cl] = a; s_b[pg][cl] = b;
    }
    __syncthreads();
  }
  if (pg == 0 && c < C) {
    const float rs = rstd[c], sc = gamma[c] * rs, inv = 1.f / (float)M;
    dgamma[c] = b * rs;
    dbeta[c] = a;
    coef[c] = sc;
    coef[C + c] = -sc * rs * rs * b * inv;
    coef[2 * C + c] = -sc * a * inv;
  }
}

// ---- backward 3: dx = ca*g + cb*(x - mean) + cc  (and dz = g for the residual branch)
template <typename T, int MASK, bool DZ, bool ADD2>
__global__ __launch_bounds__(BN_NT) void bn_bwd_dx_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                          const T* __restrict__ x,
                                                          const T* __restrict__ y, const float* __restrict__ ss,
                                                          const float* __restrict__ coef,
                                                          const float* __restrict__ mean, T* __restrict__ dx,
                                                          T* __restrict__ dz, long nvec, int C) {
  const int tpr = C >> 3;
  const long i0 = (long)blockIdx.x * BN_NT + threadIdx.x, stride = (long)gridDim.x * BN_NT;
  const int cv = (int)(i0 % tpr);
  float sc[8], sh[8], ca[8], cb[8], cc[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ch = cv * 8 + j;
    sc[j] = ss[ch]; sh[j] = ss[C + ch];
    ca[j] = coef[ch]; cb[j] = coef[C + ch]; cc[j] = coef[2 * C + ch]; mu[j] = mean[ch];
  }
  for (long i = i0; i < nvec; i += stride) {
    float g[8], xv[8];
    masked_grad<T, MASK, ADD2>(dy, dy2, x, y, i * 8, sc, sh, mu, g, xv);
    if (DZ) V8<T>::st(dz + i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = fmaf(ca[j], g[j], fmaf(cb[j], xv[j] - mu[j], cc[j]));
    V8<T>::st(dx + i * 8, xv);
  }
}

// ---- backward 3, GOUT form: dx = ca*g + cb*(x - mean) + cc from the reduce pass's stored g
template <typename T>
__global__ __launch_bounds__(BN_NT) void bn_bwd_dxg_kernel(const T* __restrict__ g_in, const T* __restrict__ x,
                                                           const float* __restrict__ coef,
                                                           const float* __restrict__ mean, T* __restrict__ dx,
                                                           long nvec, int C) {
  const int tpr = C >> 3;
  const long i0 = (long)blockIdx.x * BN_NT + threadIdx.x, stride = (long)gridDim.x * BN_NT;
  const int cv = (int)(i0 % tpr);
  float ca[8], cb[8], cc[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ch = cv * 8 + j;
    ca[j] = coef[ch]; cb[j] = coef[C + ch]; cc[j] = coef[2 * C + ch]; mu[j] = mean[ch];
  }
  long i = i0;
  for (; i + stride < nvec; i += 2 * stride) {  // two vectors in flight per thread
    float g[2][8], xv[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      V8<T>::ld(g_in + (i + u * stride) * 8, g[u]);
      V8<T>::ld(x + (i + u * stride) * 8, xv[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[u][j] = fmaf(ca[j], g[u][j], fmaf(cb[j], xv[u][j] - mu[j], cc[j]));
      V8<T>::st(dx + (i + u * stride) * 8, xv[u]);
    }
  }
  for (; i < nvec; i += stride) {
    float g[8], xv[8];
    V8<T>::ld(g_in + i * 8, g);
    V8<T>::ld(x + i * 8, xv);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = fmaf(ca[j], g[j], fmaf(cb[j], xv[j] - mu[j], cc[j]));
    V8<T>::st(dx + i * 8, xv);
  }
}

int grid_for(long nvec, int C) {
  // ~8 vectors per thread, at most 8 blocks per CU worth; a multiple of nothing in particular:
  // BN_NT is a multiple of C/8, so any grid keeps each thread on one channel group
  long g = (nvec + BN_NT * 8 - 1) / (BN_NT * 8);
  (void)C;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

template <typename T>
int fwd_t(const void* x, const void* z, void* y, const float* gamma, const float* beta, float* rm, float* rv,
          long long* nbt, float* mean, float* rstd, float* ss, float* part, long M, int C, int G, int rpb,
          float momentum, float eps, int relu, uint8_t* mo, hipStream_t s) {
  const T* xt = static_cast<const T*>(x);
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(G), dim3(BN_NT), 0, s, xt, M, C, rpb, part, part + (size_t)G * 2 * C);
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + FIN_CH - 1) / FIN_CH), dim3(FIN_NT), 0, s, part,
                     part + (size_t)G * 2 * C, G, C, eps, momentum, gamma, beta, mean, rstd, ss, rm, rv, nbt);
  const long nvec = M * (long)C / 8;
  const int gr = grid_for(nvec, C);
  const T* zt = static_cast<const T*>(z);
  T* yt = static_cast<T*>(y);
  if (z != nullptr) {
    if (relu && mo != nullptr)
      hipLaunchKernelGGL((bn_apply_kernel<T, true, true, true>), dim3(gr), dim3(BN_NT), 0, s, xt, zt, ss, mean, yt, nvec, C, mo);
    else if (relu) hipLaunchKernelGGL((bn_apply_kernel<T, true, true>), dim3(gr), dim3(BN_NT), 0, s, xt, zt, ss, mean, yt, nvec, C, mo);
    else hipLaunchKernelGGL((bn_apply_kernel<T, false, true>), dim3(gr), dim3(BN_NT), 0, s, xt, zt, ss, mean, yt, nvec, C, mo);
  } else {
    if (relu) hipLaunchKernelGGL((bn_apply_kernel<T, true, false>), dim3(gr), dim3(BN_NT), 0, s, xt, zt, ss, mean, yt, nvec, C, mo);
    else hipLaunchKernelGGL((bn_apply_kernel<T, false, false>), dim3(gr), dim3(BN_NT), 0, s, xt, zt, ss, mean, yt, nvec, C, mo);
  }
  return (int)hipGetLastError();
}

template <typename T, int MASK, bool ADD2>
void bwd_dx_launch(const T* dy, const T* dy2, const T* x, const T* y, const float* ss, const float* coef,
                   const float* mean, T* dx, T* dz, long nvec, int C, hipStream_t s) {
  const int gr = grid_for(nvec, C);
  if (dz != nullptr)
    hipLaunchKernelGGL((bn_bwd_dx_kernel<T, MASK, true, ADD2>), dim3(gr), dim3(BN_NT), 0, s, dy, dy2, x, y, ss, coef,
                       mean, dx, dz, nvec, C);
  else
    hipLaunchKernelGGL((bn_bwd_dx_kernel<T, MASK, false, ADD2>), dim3(gr), dim3(BN_NT), 0, s, dy, dy2, x, y, ss, coef,
                       mean, dx, dz, nvec, C);
}

template <typename T, int MASK, bool ADD2>
int bwd_t2(const T* dyt, const T* dy2t, const T* xt, const T* yt, const float* gamma, const float* mean,
           const float* rstd, const float* ss, float* dgamma, float* dbeta, void* dx, void* dz, float* part,
           float* coef, long M, int C, int G, int rpb, hipStream_t s) {
  T* dzt = static_cast<T*>(dz);
  const bool gout = PTO_BN_GOUT && dz != nullptr;
  if (gout)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, MASK, ADD2, true>), dim3(G), dim3(BN_NT), 0, s, dyt, dy2t, xt, yt, ss,
                       mean, M, C, rpb, part, dzt);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, MASK, ADD2>), dim3(G), dim3(BN_NT), 0, s, dyt, dy2t, xt, yt, ss, mean,
                       M, C, rpb, part, dzt);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + FIN_CH - 1) / FIN_CH), dim3(FIN_NT), 0, s, part, G, C, M, gamma,
                     mean, rstd, dgamma, dbeta, coef);
  const long nvec = M * (long)C / 8;
  if (gout)
    hipLaunchKernelGGL(bn_bwd_dxg_kernel<T>, dim3(grid_for(nvec, C)), dim3(BN_NT), 0, s, dzt, xt, coef, mean,
                       static_cast<T*>(dx), nvec, C);
  else
    bwd_dx_launch<T, MASK, ADD2>(dyt, dy2t, xt, yt, ss, coef, mean, static_cast<T*>(dx), dzt, nvec, C, s);
  return (int)hipGetLastError();
}

template <typename T, int MASK>
int bwd_t(const void* dy, const void* dy2, const void* x, const void* y, const float* gamma, const float* mean,
          const float* rstd, const float* ss, float* dgamma, float* dbeta, void* dx, void* dz, float* part,
          float* coef, long M, int C, int G, int rpb, hipStream_t s) {
  const T* dyt = static_cast<const T*>(dy);
  const T* dy2t = static_cast<const T*>(dy2);
  const T* xt = static_cast<const T*>(x);
  const T* yt = static_cast<const T*>(y);
  if (dy2 != nullptr)
    return bwd_t2<T, MASK, true>(dyt, dy2t, xt, yt, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G,
                                 rpb, s);
  return bwd_t2<T, MASK, false>(dyt, dy2t, xt, yt, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G,
                                rpb, s);
}

bool shape_ok(long M, int C, int G, int rpb) {
  if (M <= 0 || C < 8 || C > 2048 || (C & 7) || (BN_NT % (C >> 3)) || G < 1 || G > FIN_GMAX || rpb < 1) return false;
  const int rpi = BN_NT / (C >> 3);
  return rpb % rpi == 0 && (long)G * rpb >= M && (long)(G - 1) * rpb < M;
}

bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

// Plan of the reduction grid: G blocks of rows_per_block rows (a multiple of 256 / (C/8)),
// about 8 row-vectors per thread, at most 1024 blocks.  Returns G (0: unsupported C).
int pto_bn_plan(long M, int C, int* rows_per_block) {
  if (C < 8 || C > 2048 || (C & 7) || (BN_NT % (C >> 3)) || M <= 0) return 0;
  const long rpi = BN_NT / (C >> 3);
  long G = (M * (long)C / 8 + BN_NT * 8 - 1) / (BN_NT * 8);
  G = G < 1 ? 1 : (G > 1024 ? 1024 : G);
  long rpb = (M + G - 1) / G;
  rpb = (rpb + rpi - 1) / rpi * rpi;
  G = (M + rpb - 1) / rpb;
  *rows_per_block = (int)rpb;
  return (int)G;
}

// dtype: 0 fp32, 1 bf16.  part: fp32 workspace of G*(2C+1) floats.  z (residual) may be null;
// running stats / nbt may be null.  momentum as nn.BatchNorm2d (weight of the new value).
// mask_out (may be null; residual + ReLU only): M*C/8 bytes, the ReLU mask for mask_mode 3.
int pto_bn_fwd_train(const void* x, const void* z, void* y, const float* gamma, const float* beta, float* run_mean,
                     float* run_var, long long* nbt, float* mean, float* rstd, float* ss, float* part, long M, int C,
                     int G, int rows_per_block, float momentum, float eps, int dtype, int relu, void* mask_out,
                     void* stream) {
  if (!shape_ok(M, C, G, rows_per_block) || !aligned16(x) || !aligned16(z) || !aligned16(y)) return -2;
  if (mask_out != nullptr && (z == nullptr || !relu)) return -1;
  uint8_t* mo = static_cast<uint8_t*>(mask_out);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1)
    return fwd_t<bf16>(x, z, y, gamma, beta, run_mean, run_var, nbt, mean, rstd, ss, part, M, C, G, rows_per_block,
                       momentum, eps, relu, mo, s);
  if (dtype == 0)
    return fwd_t<float>(x, z, y, gamma, beta, run_mean, run_var, nbt, mean, rstd, ss, part, M, C, G, rows_per_block,
                        momentum, eps, relu, mo, s);
  return -1;
}

// mask_mode: 0 no ReLU, 1 ReLU (mask recomputed from x), 2 ReLU after a residual add (mask
// from y), 3 the same from the forward's mask_out bytes (passed as y).  dz (the residual's gradient = the masked dy) only with mask_mode 2 (may be null).
// dy2 (may be null): a second incoming gradient of the output, summed with dy in-kernel.
// coef: fp32 workspace of 3C floats.
int pto_bn_bwd(const void* dy, const void* dy2, const void* x, const void* y, const float* gamma, const float* mean,
               const float* rstd, const float* ss, float* dgamma, float* dbeta, void* dx, void* dz, float* part,
               float* coef, long M, int C, int G, int rows_per_block, int dtype, int mask_mode, void* stream) {
  if (!shape_ok(M, C, G, rows_per_block) || !aligned16(dy) || !aligned16(dy2) || !aligned16(x) || !aligned16(y) ||
      !aligned16(dx) || !aligned16(dz))
    return -2;
  if ((mask_mode == 2 || mask_mode == 3) && y == nullptr) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) {
    if (mask_mode == 0) return bwd_t<bf16, 0>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
    if (mask_mode == 1) return bwd_t<bf16, 1>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
    if (mask_mode == 2) return bwd_t<bf16, 2>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
    if (mask_mode == 3) return bwd_t<bf16, 3>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
  } else if (dtype == 0) {
    if (mask_mode == 0) return bwd_t<float, 0>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
    if (mask_mode == 1) return bwd_t<float, 1>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
    if (mask_mode == 2) return bwd_t<float, 2>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
    if (mask_mode == 3) return bwd_t<float, 3>(dy, dy2, x, y, gamma, mean, rstd, ss, dgamma, dbeta, dx, dz, part, coef, M, C, G, rows_per_block, s);
  }
  return -1;
}

}  // extern "C"
