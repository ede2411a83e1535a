// Fused RMSNorm forward/backward for the Llama path (fp32 or bf16 activations, fp32
// weight, fp32 statistics).  y = x * rsqrt(mean(x^2) + eps) * w.
//
// Forward: one workgroup per row, D/256 elements per lane held in registers, sum of
// squares reduced wave-then-LDS, rstd saved for the backward.
// Backward: a workgroup owns R consecutive rows; per row it recomputes the row dot
// product sum_j dy_j w_j x_j, writes dx, and accumulates dw_j += dy_j x_j rstd for its
// columns in registers; the per-workgroup dw partials are reduced column-wise by a
// second tiny launch in fixed order (deterministic, no atomics).
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <initializer_list>

namespace {

constexpr int kT = 256;
constexpr int kMaxPer = 32;  // D <= kT * kMaxPer = 8192

template <typename T>
__device__ __forceinline__ float ld(const T* p, long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<__hip_bfloat16>(const __hip_bfloat16* p, long i) {
  return __bfloat162float(p[i]);
}
template <typename T>
__device__ __forceinline__ void st(T* p, long i, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, long i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void st<__hip_bfloat16>(__hip_bfloat16* p, long i, float v) {
  p[i] = __float2bfloat16(v);
}

// 4 consecutive elements per access (16 B fp32 / 8 B bf16): the D % 4 == 0 fast path.
struct F4 {
  float v[4];
};
template <typename T>
__device__ __forceinline__ F4 ld4(const T* p);
template <>
__device__ __forceinline__ F4 ld4<float>(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  return F4{{a.x, a.y, a.z, a.w}};
}
template <>
__device__ __forceinline__ F4 ld4<__hip_bfloat16>(const __hip_bfloat16* p) {
  const uint2 q = *reinterpret_cast<const uint2*>(p);
  return F4{{__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u), __uint_as_float(q.y << 16),
             __uint_as_float(q.y & 0xffff0000u)}};
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const F4& r);
template <>
__device__ __forceinline__ void st4<float>(float* p, const F4& r) {
  *reinterpret_cast<float4*>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
}
__device__ __forceinline__ uint32_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
template <>
__device__ __forceinline__ void st4<__hip_bfloat16>(__hip_bfloat16* p, const F4& r) {
  *reinterpret_cast<uint2*>(p) = make_uint2(bf16_rne(r.v[0]) | (bf16_rne(r.v[1]) << 16),
                                            bf16_rne(r.v[2]) | (bf16_rne(r.v[3]) << 16));
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < kT / 64; ++k) t += sh[k];
  return t;
}

// TX: activation dtype of x / dx (the residual stream, fp32 or bf16).  TY: dtype of y / dy
// (bf16 when the norm feeds autocast bf16 matmuls: writing bf16 here removes the separate
// fp32->bf16 cast kernel in the forward and the bf16->fp32 dy cast in the backward).
template <typename TX, typename TY, int PER>
__global__ __launch_bounds__(kT) void rmsnorm_fwd_kernel(const TX* __restrict__ x, const float* __restrict__ w,
                                                         TY* __restrict__ y, float* __restrict__ rstd, int D,
                                                         float eps) {
  __shared__ float sh[kT / 64];
  const long row = blockIdx.x;
  const TX* xr = x + row * D;
  float v[PER];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = threadIdx.x + k * kT;
    v[k] = j < D ? ld(xr, j) : 0.f;
    ss += v[k] * v[k];
  }
  const float r = rsqrtf(block_sum(ss, sh) / (float)D + eps);
  if (threadIdx.x == 0) rstd[row] = r;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = threadIdx.x + k * kT;
    if (j < D) st(y + row * D, j, v[k] * r * w[j]);
  }
}

template <typename TX, typename TY, int PER>
__global__ __launch_bounds__(kT) void rmsnorm_bwd_kernel(const TY* __restrict__ dy, const TX* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ rstd, TX* __restrict__ dx,
                                                         float* __restrict__ dw_part, long rows, int D,
                                                         int rows_per_block) {
  __shared__ float sh[kT / 64];
  float wv[PER], dwa[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = threadIdx.x + k * kT;
    wv[k] = j < D ? w[j] : 0.f;
    dwa[k] = 0.f;
  }
  const long r0 = (long)blockIdx.x * rows_per_block;
  for (long row = r0; row < min(rows, r0 + rows_per_block); ++row) {
    float xv[PER], gv[PER];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int j = threadIdx.x + k * kT;
      const bool ok = j < D;
      xv[k] = ok ? ld(x + row * D, j) : 0.f;
      gv[k] = ok ? ld(dy + row * D, j) : 0.f;
      dot += gv[k] * wv[k] * xv[k];
    }
    const float r = rstd[row];
    const float c = block_sum(dot, sh) * r * r * r / (float)D;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int j = threadIdx.x + k * kT;
      if (j < D) {
        st(dx + row * D, j, r * wv[k] * gv[k] - xv[k] * c);
        dwa[k] += gv[k] * xv[k] * r;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = threadIdx.x + k * kT;
    if (j < D) dw_part[(long)blockIdx.x * D + j] = dwa[k];
  }
}

// ---- D % 4 == 0 fast path: lane owns column groups j = 4*(threadIdx.x + k*kT), k < P4.
// Fused residual form (delta != nullptr): s = x + delta is written to s_out (the residual
// stream, dtype TX) and normalised, so the block's residual add costs no separate pass.
template <typename TX, typename TY, int P4>
__global__ __launch_bounds__(kT) void rmsnorm_fwd_vec_kernel(const TX* __restrict__ x, const float* __restrict__ w,
                                                             TY* __restrict__ y, float* __restrict__ rstd, int D,
                                                             float eps, const TY* __restrict__ delta,
                                                             TX* __restrict__ s_out) {
  __shared__ float sh[kT / 64];
  const long row = blockIdx.x;
  F4 v[P4];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < P4; ++k) {
    const int j = 4 * (threadIdx.x + k * kT);
    v[k] = j < D ? ld4(x + row * D + j) : F4{{0.f, 0.f, 0.f, 0.f}};
    if (delta != nullptr && j < D) {
      const F4 dd = ld4(delta + row * D + j);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k].v[e] += dd.v[e];
      st4(s_out + row * D + j, v[k]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) ss += v[k].v[e] * v[k].v[e];
  }
  const float r = rsqrtf(block_sum(ss, sh) / (float)D + eps);
  if (threadIdx.x == 0) rstd[row] = r;
#pragma unroll
  for (int k = 0; k < P4; ++k) {
    const int j = 4 * (threadIdx.x + k * kT);
    if (j < D) {
      const float4 wv = *reinterpret_cast<const float4*>(w + j);
      st4(y + row * D + j, F4{{v[k].v[0] * r * wv.x, v[k].v[1] * r * wv.y, v[k].v[2] * r * wv.z,
                               v[k].v[3] * r * wv.w}});
    }
  }
}

// Backward, software-pipelined: the next row's x / dy loads are issued before this row's
// block reduction, so HBM latency overlaps the two LDS barriers of block_sum.
// Fused residual form (gres != nullptr): dx = gres + d(norm)/dx -- the residual stream's
// gradient is summed here instead of by a separate add; with dbranch != nullptr the same
// value is also written in the branch dtype TY (the gradient of the block's bf16 output).
template <typename TX, typename TY, int P4>
__global__ __launch_bounds__(kT) void rmsnorm_bwd_vec_kernel(const TY* __restrict__ dy, const TX* __restrict__ x,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ rstd, TX* __restrict__ dx,
                                                             float* __restrict__ dw_part, long rows, int D,
                                                             int rows_per_block, const TX* __restrict__ gres,
                                                             TY* __restrict__ dbranch) {
  __shared__ float sh[kT / 64];
  F4 wv[P4], dwa[P4], xv[P4], gv[P4];
#pragma unroll
  for (int k = 0; k < P4; ++k) {
    const int j = 4 * (threadIdx.x + k * kT);
    const F4 z{{0.f, 0.f, 0.f, 0.f}};
    wv[k] = j < D ? ld4(w + j) : z;
    dwa[k] = z;
  }
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  auto load_row = [&](long row, F4* xo, F4* go) {
#pragma unroll
    for (int k = 0; k < P4; ++k) {
      const int j = 4 * (threadIdx.x + k * kT);
      const F4 z{{0.f, 0.f, 0.f, 0.f}};
      xo[k] = j < D ? ld4(x + row * D + j) : z;
      go[k] = j < D ? ld4(dy + row * D + j) : z;
    }
  };
  if (r0 < r1) load_row(r0, xv, gv);
  for (long row = r0; row < r1; ++row) {
    F4 xn[P4], gn[P4];
    if (row + 1 < r1) load_row(row + 1, xn, gn);
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < P4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) dot += gv[k].v[e] * wv[k].v[e] * xv[k].v[e];
    const float r = rstd[row];
    const float c = block_sum(dot, sh) * r * r * r / (float)D;
#pragma unroll
    for (int k = 0; k < P4; ++k) {
      const int j = 4 * (threadIdx.x + k * kT);
      if (j < D) {
        F4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o.v[e] = r * wv[k].v[e] * gv[k].v[e] - xv[k].v[e] * c;
          dwa[k].v[e] += gv[k].v[e] * xv[k].v[e] * r;
        }
        if (gres != nullptr) {
          const F4 gr = ld4(gres + row * D + j);
#pragma unroll
          for (int e = 0; e < 4; ++e) o.v[e] += gr.v[e];
        }
        if (dbranch != nullptr) st4(dbranch + row * D + j, o);
        st4(dx + row * D + j, o);
      }
    }
    if (row + 1 < r1) {
#pragma unroll
      for (int k = 0; k < P4; ++k) {
        xv[k] = xn[k];
        gv[k] = gn[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < P4; ++k) {
    const int j = 4 * (threadIdx.x + k * kT);
    if (j < D) st4(dw_part + (long)blockIdx.x * D + j, dwa[k]);
  }
}

// Column sums of dw_part [nparts, D] in a fixed order (deterministic).  A workgroup owns
// kColsPerWg columns: kCLanes lanes per row slice read them as float4 and kSlices slices
// walk disjoint row ranges with all loads of a slice issued back to back, then the slices
// are added in slice order through LDS.  D=4096, 512 parts: 128 workgroups x 256 lanes
// with 32 float4 loads in flight each, instead of 16 workgroups each walking 512 rows one
// dependent load at a time (123 us -> a few us, see docs/kernels.md).
constexpr int kCLanes = 8;                   // float4 lanes per slice -> 32 columns
constexpr int kColsPerWg = kCLanes * 4;
constexpr int kSlices = kT / kCLanes;        // 32 row slices
__global__ __launch_bounds__(kT) void colsum_kernel(const float* __restrict__ part, int nparts, int D,
                                                    float* __restrict__ out) {
  __shared__ float4 sh[kSlices][kCLanes];
  const int lane = threadIdx.x % kCLanes, slice = threadIdx.x / kCLanes;
  const int j = blockIdx.x * kColsPerWg + lane * 4;
  const int per = (nparts + kSlices - 1) / kSlices;
  const int p0 = slice * per, p1 = min(nparts, p0 + per);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j + 3 < D && (D & 3) == 0) {
#pragma unroll 8
    for (int p = p0; p < p1; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(part + (long)p * D + j);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  } else {
    for (int p = p0; p < p1; ++p) {
      const float* r = part + (long)p * D;
      if (j < D) s.x += r[j];
      if (j + 1 < D) s.y += r[j + 1];
      if (j + 2 < D) s.z += r[j + 2];
      if (j + 3 < D) s.w += r[j + 3];
    }
  }
  sh[slice][lane] = s;
  __syncthreads();
  if (slice == 0) {
    float4 t = sh[0][lane];
    for (int k = 1; k < kSlices; ++k) {
      const float4 v = sh[k][lane];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    if (j < D) out[j] = t.x;
    if (j + 1 < D) out[j + 1] = t.y;
    if (j + 2 < D) out[j + 2] = t.z;
    if (j + 3 < D) out[j + 3] = t.w;
  }
}

template <typename TX, typename TY, int PER>
void fwd_launch(const void* x, const float* w, void* y, float* rstd, long rows, int D, float eps, void* stream) {
  hipLaunchKernelGGL((rmsnorm_fwd_kernel<TX, TY, PER>), dim3(rows), dim3(kT), 0, (hipStream_t)stream,
                     (const TX*)x, w, (TY*)y, rstd, D, eps);
}

template <typename TX, typename TY, int P4>
void fwd_vec_launch(const void* x, const float* w, void* y, float* rstd, long rows, int D, float eps,
                    void* stream, const void* delta = nullptr, void* s_out = nullptr) {
  hipLaunchKernelGGL((rmsnorm_fwd_vec_kernel<TX, TY, P4>), dim3(rows), dim3(kT), 0, (hipStream_t)stream,
                     (const TX*)x, w, (TY*)y, rstd, D, eps, (const TY*)delta, (TX*)s_out);
}

bool vec_ok(int D, std::initializer_list<const void*> ptrs) {
  if (D % 4) return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p & 15u) return false;
  return true;
}

template <typename TX, typename TY>
int fwd_dispatch(const void* x, const float* w, void* y, float* rstd, long rows, int D, float eps, void* stream,
                 const void* delta = nullptr, void* s_out = nullptr) {
  if (vec_ok(D, {x, w, y}) && (delta == nullptr || vec_ok(D, {delta, s_out}))) {
    const int p4 = (D + 4 * kT - 1) / (4 * kT);
    if (p4 <= 1) fwd_vec_launch<TX, TY, 1>(x, w, y, rstd, rows, D, eps, stream, delta, s_out);
    else if (p4 <= 2) fwd_vec_launch<TX, TY, 2>(x, w, y, rstd, rows, D, eps, stream, delta, s_out);
    else if (p4 <= 4) fwd_vec_launch<TX, TY, 4>(x, w, y, rstd, rows, D, eps, stream, delta, s_out);
    else fwd_vec_launch<TX, TY, 8>(x, w, y, rstd, rows, D, eps, stream, delta, s_out);
    return (int)hipGetLastError();
  }
  if (delta != nullptr) return -3;  // the fused residual form needs the vector path
  const int per = (D + kT - 1) / kT;
  if (per <= 1) fwd_launch<TX, TY, 1>(x, w, y, rstd, rows, D, eps, stream);
  else if (per <= 2) fwd_launch<TX, TY, 2>(x, w, y, rstd, rows, D, eps, stream);
  else if (per <= 4) fwd_launch<TX, TY, 4>(x, w, y, rstd, rows, D, eps, stream);
  else if (per <= 8) fwd_launch<TX, TY, 8>(x, w, y, rstd, rows, D, eps, stream);
  else if (per <= 16) fwd_launch<TX, TY, 16>(x, w, y, rstd, rows, D, eps, stream);
  else fwd_launch<TX, TY, 32>(x, w, y, rstd, rows, D, eps, stream);
  return (int)hipGetLastError();
}

template <typename TX, typename TY, int PER>
void bwd_launch(const void* dy, const void* x, const float* w, const float* rstd, void* dx, float* dw_part,
                long rows, int D, int rpb, long nb, void* stream) {
  hipLaunchKernelGGL((rmsnorm_bwd_kernel<TX, TY, PER>), dim3(nb), dim3(kT), 0, (hipStream_t)stream,
                     (const TY*)dy, (const TX*)x, w, rstd, (TX*)dx, dw_part, rows, D, rpb);
}

template <typename TX, typename TY, int P4>
void bwd_vec_launch(const void* dy, const void* x, const float* w, const float* rstd, void* dx, float* dw_part,
                    long rows, int D, int rpb, long nb, void* stream, const void* gres, void* dbranch) {
  hipLaunchKernelGGL((rmsnorm_bwd_vec_kernel<TX, TY, P4>), dim3(nb), dim3(kT), 0, (hipStream_t)stream,
                     (const TY*)dy, (const TX*)x, w, rstd, (TX*)dx, dw_part, rows, D, rpb, (const TX*)gres,
                     (TY*)dbranch);
}

template <typename TX, typename TY>
int bwd_dispatch(const void* dy, const void* x, const float* w, const float* rstd, void* dx, float* dw_part,
                 long rows, int D, int rpb, long nb, void* stream, const void* gres = nullptr,
                 void* dbranch = nullptr) {
  if (vec_ok(D, {dy, x, w, dx, dw_part}) && (gres == nullptr || vec_ok(D, {gres})) &&
      (dbranch == nullptr || vec_ok(D, {dbranch}))) {
    const int p4 = (D + 4 * kT - 1) / (4 * kT);
    if (p4 <= 1) bwd_vec_launch<TX, TY, 1>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream, gres, dbranch);
    else if (p4 <= 2)
      bwd_vec_launch<TX, TY, 2>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream, gres, dbranch);
    else if (p4 <= 4)
      bwd_vec_launch<TX, TY, 4>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream, gres, dbranch);
    else bwd_vec_launch<TX, TY, 8>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream, gres, dbranch);
    return 0;
  }
  if (gres != nullptr || dbranch != nullptr) return -3;
  const int per = (D + kT - 1) / kT;
  if (per <= 1) bwd_launch<TX, TY, 1>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream);
  else if (per <= 2) bwd_launch<TX, TY, 2>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream);
  else if (per <= 4) bwd_launch<TX, TY, 4>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream);
  else if (per <= 8) bwd_launch<TX, TY, 8>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream);
  else if (per <= 16) bwd_launch<TX, TY, 16>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream);
  else bwd_launch<TX, TY, 32>(dy, x, w, rstd, dx, dw_part, rows, D, rpb, nb, stream);
  return 0;
}

// dtype pair code: 0 = (x fp32, y fp32), 1 = (bf16, bf16), 2 = (x fp32, y bf16)
bool valid_pair(int code) { return code >= 0 && code <= 2; }

}  // namespace

extern "C" {

int pto_add_rmsnorm_bwd(const void* dy, const void* x, const float* w, const float* rstd, const void* gres,
                        void* dx, void* dbranch, float* dw, float* dw_part, long rows, int D, int rows_per_block,
                        int dtype, void* stream);

int pto_rmsnorm_fwd(const void* x, const float* w, void* y, float* rstd, long rows, int D, float eps, int dtype,
                    void* stream) {
  if (D <= 0 || D > kT * kMaxPer || rows <= 0 || !valid_pair(dtype)) return -1;
  if (dtype == 0) return fwd_dispatch<float, float>(x, w, y, rstd, rows, D, eps, stream);
  if (dtype == 1) return fwd_dispatch<__hip_bfloat16, __hip_bfloat16>(x, w, y, rstd, rows, D, eps, stream);
  return fwd_dispatch<float, __hip_bfloat16>(x, w, y, rstd, rows, D, eps, stream);
}

// Number of workgroups (= rows of dw_part) the backward uses for `rows` rows.
long pto_rmsnorm_bwd_parts(long rows, int rows_per_block) { return (rows + rows_per_block - 1) / rows_per_block; }

int pto_rmsnorm_bwd(const void* dy, const void* x, const float* w, const float* rstd, void* dx, float* dw,
                    float* dw_part, long rows, int D, int rows_per_block, int dtype, void* stream) {
  if (D <= 0 || D > kT * kMaxPer || rows <= 0 || rows_per_block <= 0 || !valid_pair(dtype)) return -1;
  const long nb = (rows + rows_per_block - 1) / rows_per_block;
  if (nb > (1L << 30)) return -1;
  return pto_add_rmsnorm_bwd(dy, x, w, rstd, nullptr, dx, nullptr, dw, dw_part, rows, D, rows_per_block, dtype,
                             stream);
}

// Residual-fused forms.  fwd: s = x + delta (written to s_out), y = rmsnorm(s).  bwd: x is s,
// gres the residual stream's incoming gradient; dx = gres + d(norm), dbranch = the same in
// the y dtype (nullable).  Vector path only (D % 4 == 0, 16-byte aligned): -3 otherwise.
int pto_add_rmsnorm_fwd(const void* x, const void* delta, const float* w, void* y, void* s_out, float* rstd,
                        long rows, int D, float eps, int dtype, void* stream) {
  if (D <= 0 || D > kT * kMaxPer || rows <= 0 || !valid_pair(dtype) || delta == nullptr || s_out == nullptr)
    return -1;
  if (dtype == 0) return fwd_dispatch<float, float>(x, w, y, rstd, rows, D, eps, stream, delta, s_out);
  if (dtype == 1)
    return fwd_dispatch<__hip_bfloat16, __hip_bfloat16>(x, w, y, rstd, rows, D, eps, stream, delta, s_out);
  return fwd_dispatch<float, __hip_bfloat16>(x, w, y, rstd, rows, D, eps, stream, delta, s_out);
}

int pto_add_rmsnorm_bwd(const void* dy, const void* x, const float* w, const float* rstd, const void* gres,
                        void* dx, void* dbranch, float* dw, float* dw_part, long rows, int D, int rows_per_block,
                        int dtype, void* stream) {
  if (D <= 0 || D > kT * kMaxPer || rows <= 0 || rows_per_block <= 0 || !valid_pair(dtype)) return -1;
  const long nb = (rows + rows_per_block - 1) / rows_per_block;
  if (nb > (1L << 30)) return -1;
  int rc;
  if (dtype == 0)
    rc = bwd_dispatch<float, float>(dy, x, w, rstd, dx, dw_part, rows, D, rows_per_block, nb, stream, gres, dbranch);
  else if (dtype == 1)
    rc = bwd_dispatch<__hip_bfloat16, __hip_bfloat16>(dy, x, w, rstd, dx, dw_part, rows, D, rows_per_block, nb,
                                                      stream, gres, dbranch);
  else
    rc = bwd_dispatch<float, __hip_bfloat16>(dy, x, w, rstd, dx, dw_part, rows, D, rows_per_block, nb, stream, gres,
                                             dbranch);
  if (rc != 0) return rc;
  hipLaunchKernelGGL(colsum_kernel, dim3((D + kColsPerWg - 1) / kColsPerWg), dim3(kT), 0, (hipStream_t)stream,
                     dw_part, (int)nb, D, dw);
  return (int)hipGetLastError();
}

}  // extern "C"
