// Fused elementwise kernels for the Llama DDP worker (BASELINE "Llama-3 8B DDP bf16").
//
// The eager PyTorch forms of these ops each expand into a chain of fp32 elementwise
// kernels over [tokens, hidden] tensors (RoPE: bf16->fp32 copy, 4 muls, add, sub, stack,
// fp32->bf16 copy; SwiGLU backward: silu_backward + 2 muls + the saved silu), which the
// rocprofv3 trace of the 8B step showed as ~15% of step time (profiles/
// r1_llama3_8b_kernel_stats.md).  Here each op is one pass over HBM: 16-byte vector
// loads/stores (8 bf16 or 2x4 fp32 per lane), fp32 math in registers.
//
//   rope:    x [rows = B*S*H, D] (adjacent pairs rotated, Meta's complex layout), position
//            of a row = (row / H) % S, tables cos/sin [S, D/2] fp32.  sign = +1 forward,
//            -1 backward (the adjoint of a rotation is the rotation by -theta).
//   swiglu:  y = silu(a) * b ; backward da = dy*b*sig(a)*(1 + a*(1-sig(a))), db = dy*silu(a)
//   rope_qkv: the fused QKV projection's output [rows = B*S, (Hq + 2 Hkv) * D] split into
//            contiguous q [B,S,Hq,D], k [B,S,Hkv,D] (both rotated) and v (copied) in one pass;
//            dir = 1 is its adjoint (dq, dk rotated by -theta, dv) -> packed d(qkv).
//   swiglu_packed: the fused W1|W3 projection's output x [rows, 2F]: y = silu(x[:, :F]) * x[:, F:],
//            backward writes the packed d(x) -- no gradient accumulation between two matmuls.
//   xent:    cross-entropy over the vocabulary straight from the lm-head's logits (bf16 or
//            fp32, [rows, V]): forward = one read of each row (per-lane online max / sum-exp,
//            one block reduction) -> per-row lse and loss; backward = one read + one write,
//            d(logits) = (exp(x - lse) - onehot(t)) * scale, written in place over the logits
//            (no fp32 copy of the 128k-wide logits, no separate softmax / NLL kernels).
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kT = 256;

struct V8 {
  float v[8];
};

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even (inputs are finite)
  const uint32_t u = __float_as_uint(f);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

template <typename T>
struct Vec;

template <>
struct Vec<float> {
  static __device__ __forceinline__ V8 load(const float* p) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    return V8{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
  }
  static __device__ __forceinline__ void store(float* p, const V8& r) {
    reinterpret_cast<float4*>(p)[0] = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(r.v[4], r.v[5], r.v[6], r.v[7]);
  }
  static __device__ __forceinline__ float load1(const float* p) { return *p; }
  static __device__ __forceinline__ void store1(float* p, float v) { *p = v; }
};

template <>
struct Vec<uint16_t> {  // bf16 bits
  static __device__ __forceinline__ V8 load(const uint16_t* p) {
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    V8 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r.v[2 * i] = __uint_as_float(w[i] << 16);
      r.v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
    return r;
  }
  static __device__ __forceinline__ void store(uint16_t* p, const V8& r) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(r.v[2 * i]) | ((uint32_t)f2bf(r.v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  static __device__ __forceinline__ float load1(const uint16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void store1(uint16_t* p, float v) { *p = f2bf(v); }
};

// ---------------------------------------------------------------------------------- rope
template <typename T>
__global__ __launch_bounds__(kT) void rope_kernel(const T* __restrict__ x, const float* __restrict__ cosb,
                                                  const float* __restrict__ sinb, T* __restrict__ y, long groups,
                                                  int H, int S, int D, float sign) {
  const int gpr = D / 8;  // 8-element groups per row (D % 8 == 0 checked on the host)
  for (long g = (long)blockIdx.x * kT + threadIdx.x; g < groups; g += (long)gridDim.x * kT) {
    const long row = g / gpr;
    const int c8 = (int)(g - row * gpr) * 8;
    const int s = (int)((row / H) % S);
    const V8 in = Vec<T>::load(x + row * D + c8);
    const float4 cv = *reinterpret_cast<const float4*>(cosb + (long)s * (D / 2) + c8 / 2);
    const float4 sv = *reinterpret_cast<const float4*>(sinb + (long)s * (D / 2) + c8 / 2);
    const float cs[4] = {cv.x, cv.y, cv.z, cv.w}, sn[4] = {sign * sv.x, sign * sv.y, sign * sv.z, sign * sv.w};
    V8 out;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x0 = in.v[2 * i], x1 = in.v[2 * i + 1];
      out.v[2 * i] = x0 * cs[i] - x1 * sn[i];
      out.v[2 * i + 1] = x0 * sn[i] + x1 * cs[i];
    }
    Vec<T>::store(y + row * D + c8, out);
  }
}

// One thread per 8-element group of the packed row; heads [0, Hq) -> q, [Hq, Hq+Hkv) -> k,
// the rest -> v.  dir 0: packed -> q/k/v (sign +1); dir 1: dq/dk/dv -> packed (sign -1).
template <typename T>
__global__ __launch_bounds__(kT) void rope_qkv_kernel(T* __restrict__ pk, T* __restrict__ q, T* __restrict__ k,
                                                      T* __restrict__ v, const float* __restrict__ cosb,
                                                      const float* __restrict__ sinb, long tokens, int S, int Hq,
                                                      int Hkv, int D, int dir) {
  const int W = (Hq + 2 * Hkv) * D, gpr = W / 8;
  const long groups = tokens * gpr;
  for (long gi = (long)blockIdx.x * kT + threadIdx.x; gi < groups; gi += (long)gridDim.x * kT) {
    const long tok = gi / gpr;
    const int c = (int)(gi - tok * gpr) * 8;
    const int hh = c / D, d0 = c - hh * D;
    T* other;
    bool rot = true;
    if (hh < Hq) {
      other = q + (tok * Hq + hh) * D + d0;
    } else if (hh < Hq + Hkv) {
      other = k + (tok * Hkv + (hh - Hq)) * D + d0;
    } else {
      other = v + (tok * Hkv + (hh - Hq - Hkv)) * D + d0;
      rot = false;
    }
    T* packed = pk + tok * W + c;
    const V8 in = dir == 0 ? Vec<T>::load(packed) : Vec<T>::load(other);
    V8 out = in;
    if (rot) {
      const int s = (int)(tok % S);
      const float sign = dir == 0 ? 1.f : -1.f;
      const float4 cv = *reinterpret_cast<const float4*>(cosb + (long)s * (D / 2) + d0 / 2);
      const float4 sv = *reinterpret_cast<const float4*>(sinb + (long)s * (D / 2) + d0 / 2);
      const float cs[4] = {cv.x, cv.y, cv.z, cv.w}, sn[4] = {sign * sv.x, sign * sv.y, sign * sv.z, sign * sv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x0 = in.v[2 * i], x1 = in.v[2 * i + 1];
        out.v[2 * i] = x0 * cs[i] - x1 * sn[i];
        out.v[2 * i + 1] = x0 * sn[i] + x1 * cs[i];
      }
    }
    Vec<T>::store(dir == 0 ? other : packed, out);
  }
}

// -------------------------------------------------------------------------------- swiglu
__device__ __forceinline__ float sigmoid(float a) { return 1.f / (1.f + __expf(-a)); }

// Packed form: x [rows, 2F] (a = x[:, :F], b = x[:, F:]), y / dy [rows, F].  F % 8 == 0.
template <typename T>
__global__ __launch_bounds__(kT) void swiglu_packed_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                               long rows, int F) {
  const int gpr = F / 8;
  const long groups = rows * gpr;
  for (long g = (long)blockIdx.x * kT + threadIdx.x; g < groups; g += (long)gridDim.x * kT) {
    const long r = g / gpr;
    const int c = (int)(g - r * gpr) * 8;
    const V8 av = Vec<T>::load(x + r * 2 * F + c), bv = Vec<T>::load(x + r * 2 * F + F + c);
    V8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.v[i] = av.v[i] * sigmoid(av.v[i]) * bv.v[i];
    Vec<T>::store(y + r * F + c, o);
  }
}

template <typename T>
__global__ __launch_bounds__(kT) void swiglu_packed_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               T* __restrict__ dx, long rows, int F) {
  const int gpr = F / 8;
  const long groups = rows * gpr;
  for (long g = (long)blockIdx.x * kT + threadIdx.x; g < groups; g += (long)gridDim.x * kT) {
    const long r = g / gpr;
    const int c = (int)(g - r * gpr) * 8;
    const V8 gv = Vec<T>::load(dy + r * F + c);
    const V8 av = Vec<T>::load(x + r * 2 * F + c), bv = Vec<T>::load(x + r * 2 * F + F + c);
    V8 oa, ob;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sg = sigmoid(av.v[i]);
      oa.v[i] = gv.v[i] * bv.v[i] * sg * (1.f + av.v[i] * (1.f - sg));
      ob.v[i] = gv.v[i] * av.v[i] * sg;
    }
    Vec<T>::store(dx + r * 2 * F + c, oa);
    Vec<T>::store(dx + r * 2 * F + F + c, ob);
  }
}

template <typename T>
__global__ __launch_bounds__(kT) void swiglu_fwd_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                        T* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long g = (long)blockIdx.x * kT + threadIdx.x; g <= n8; g += (long)gridDim.x * kT) {
    if (g < n8) {
      const V8 av = Vec<T>::load(a + g * 8), bv = Vec<T>::load(b + g * 8);
      V8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o.v[i] = av.v[i] * sigmoid(av.v[i]) * bv.v[i];
      Vec<T>::store(y + g * 8, o);
    } else {
      for (long i = n8 * 8; i < n; ++i) {
        const float av = Vec<T>::load1(a + i);
        Vec<T>::store1(y + i, av * sigmoid(av) * Vec<T>::load1(b + i));
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kT) void swiglu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ a,
                                                        const T* __restrict__ b, T* __restrict__ da,
                                                        T* __restrict__ db, long n) {
  const long n8 = n / 8;
  for (long g = (long)blockIdx.x * kT + threadIdx.x; g <= n8; g += (long)gridDim.x * kT) {
    if (g < n8) {
      const V8 gv = Vec<T>::load(dy + g * 8), av = Vec<T>::load(a + g * 8), bv = Vec<T>::load(b + g * 8);
      V8 oa, ob;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float sg = sigmoid(av.v[i]);
        oa.v[i] = gv.v[i] * bv.v[i] * sg * (1.f + av.v[i] * (1.f - sg));
        ob.v[i] = gv.v[i] * av.v[i] * sg;
      }
      Vec<T>::store(da + g * 8, oa);
      Vec<T>::store(db + g * 8, ob);
    } else {
      for (long i = n8 * 8; i < n; ++i) {
        const float gv = Vec<T>::load1(dy + i), av = Vec<T>::load1(a + i), bv = Vec<T>::load1(b + i);
        const float sg = sigmoid(av);
        Vec<T>::store1(da + i, gv * bv * sg * (1.f + av * (1.f - sg)));
        Vec<T>::store1(db + i, gv * av * sg);
      }
    }
  }
}

// ---------------------------------------------------------------------------- xent
// One workgroup per row (rows = tokens: thousands of workgroups), kX threads, 8 elements
// (one 16-byte bf16 / two 16-byte fp32 loads) per lane per iteration.  V % 8 == 0.
constexpr int kX = 512;

template <typename T>
__global__ __launch_bounds__(kX) void xent_fwd_kernel(const T* __restrict__ x, const long* __restrict__ tgt,
                                                      float* __restrict__ lse_out, float* __restrict__ loss_out,
                                                      int V, long ignore_index) {
  __shared__ float sm[kX / 64], ss[kX / 64];
  const long row = blockIdx.x;
  const T* xr = x + row * (long)V;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float m = -INFINITY, s = 0.f;
  const int n8 = V / 8;
  for (int g = tid; g < n8; g += kX) {
    const V8 v = Vec<T>::load(xr + (long)g * 8);
    float mx = v.v[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) mx = fmaxf(mx, v.v[i]);
    const float mn = fmaxf(m, mx);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += __expf(v.v[i] - mn);
    s = s * __expf(m - mn) + acc;  // m = -inf on the first group: exp(-inf) = 0
    m = mn;
  }
  // wave, then block: combine (m, s) pairs
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, mo);
    s = (mn == -INFINITY) ? 0.f : s * __expf(m - mn) + so * __expf(mo - mn);
    m = mn;
  }
  if (lane == 0) { sm[wv] = m; ss[wv] = s; }
  __syncthreads();
  if (tid == 0) {
    float M = sm[0], Ssum = ss[0];
#pragma unroll
    for (int q = 1; q < kX / 64; ++q) {
      const float mn = fmaxf(M, sm[q]);
      Ssum = Ssum * __expf(M - mn) + ss[q] * __expf(sm[q] - mn);
      M = mn;
    }
    const float lse = M + __logf(Ssum);
    const long t = tgt[row];
    lse_out[row] = lse;
    loss_out[row] = (t == ignore_index || t < 0 || t >= V) ? 0.f : lse - Vec<T>::load1(xr + t);
  }
}

// d(logits)[row] = (exp(x - lse) - onehot(t)) * scale[0]; rows whose target is ignored get 0.
// dx may alias x (each element is read, then written, by the same lane).
template <typename T>
__global__ __launch_bounds__(kX) void xent_bwd_kernel(const T* x, const long* __restrict__ tgt,
                                                      const float* __restrict__ lse_in,
                                                      const float* __restrict__ scale, T* dx, int V,
                                                      long ignore_index) {
  const long row = blockIdx.x;
  const T* xr = x + row * (long)V;
  T* dr = dx + row * (long)V;
  const long t = tgt[row];
  const bool ign = t == ignore_index || t < 0 || t >= V;
  const float lse = lse_in[row], sc = ign ? 0.f : scale[0];
  const int n8 = V / 8;
  for (int g = threadIdx.x; g < n8; g += kX) {
    V8 v = Vec<T>::load(xr + (long)g * 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float p = __expf(v.v[i] - lse);
      v.v[i] = (p - ((long)(g * 8 + i) == t ? 1.f : 0.f)) * sc;
    }
    Vec<T>::store(dr + (long)g * 8, v);
  }
}

// ------------------------------------------------------------------------------ transpose
// out[c][r] = in[r][c] for a [rows, cols] 16-bit matrix (bf16 bits), rows % 64 == cols % 64 == 0.
// One 64x64 tile per workgroup: 16-byte row loads into a padded LDS tile (row stride 66
// halfwords: the column reads of the store phase spread over the banks), 16-byte row
// stores of the transposed tile.  Used to give hipBLASLt K-contiguous operands (the "TN"
// form it runs fastest) for the Llama linears' backward GEMMs.
constexpr int kTT = 64;
__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ in,
                                                          uint16_t* __restrict__ out, long rows, long cols) {
  __shared__ uint16_t t[kTT][kTT + 2];
  const long r0 = (long)blockIdx.y * kTT, c0 = (long)blockIdx.x * kTT;
  const int tid = threadIdx.x, rr = tid >> 3, cc = (tid & 7) * 8;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = rr + 32 * p;
    const uint4 q = *reinterpret_cast<const uint4*>(in + (r0 + r) * cols + c0 + cc);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      t[r][cc + 2 * i] = (uint16_t)(w[i] & 0xffffu);
      t[r][cc + 2 * i + 1] = (uint16_t)(w[i] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int oc = rr + 32 * p;  // output row = input column
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)t[cc + 2 * i][oc] | ((uint32_t)t[cc + 2 * i + 1][oc] << 16);
    *reinterpret_cast<uint4*>(out + (c0 + oc) * rows + r0 + cc) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Enough workgroups to fill 256 CUs several times over; grid-stride beyond that.
unsigned grid_for(long work) {
  const long b = (work + kT - 1) / kT;
  return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

extern "C" {

// dtype: 0 = fp32, 1 = bf16.  All pointers 16-byte aligned, tensors contiguous.
int pto_rope(const void* x, const float* cosb, const float* sinb, void* y, long rows, int H, int S, int D,
             float sign, int dtype, void* stream) {
  if (rows <= 0 || H <= 0 || S <= 0 || D <= 0 || D % 8 || (rows % H) || dtype < 0 || dtype > 1) return -1;
  if (!aligned16(x) || !aligned16(y) || !aligned16(cosb) || !aligned16(sinb)) return -2;
  const long groups = rows * (D / 8);
  if (dtype == 0)
    hipLaunchKernelGGL(rope_kernel<float>, dim3(grid_for(groups)), dim3(kT), 0, (hipStream_t)stream,
                       (const float*)x, cosb, sinb, (float*)y, groups, H, S, D, sign);
  else
    hipLaunchKernelGGL(rope_kernel<uint16_t>, dim3(grid_for(groups)), dim3(kT), 0, (hipStream_t)stream,
                       (const uint16_t*)x, cosb, sinb, (uint16_t*)y, groups, H, S, D, sign);
  return (int)hipGetLastError();
}

int pto_swiglu_fwd(const void* a, const void* b, void* y, long n, int dtype, void* stream) {
  if (n <= 0 || dtype < 0 || dtype > 1) return -1;
  if (!aligned16(a) || !aligned16(b) || !aligned16(y)) return -2;
  const unsigned grid = grid_for(n / 8 + 1);
  if (dtype == 0)
    hipLaunchKernelGGL(swiglu_fwd_kernel<float>, dim3(grid), dim3(kT), 0, (hipStream_t)stream, (const float*)a,
                       (const float*)b, (float*)y, n);
  else
    hipLaunchKernelGGL(swiglu_fwd_kernel<uint16_t>, dim3(grid), dim3(kT), 0, (hipStream_t)stream,
                       (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)y, n);
  return (int)hipGetLastError();
}

int pto_swiglu_bwd(const void* dy, const void* a, const void* b, void* da, void* db, long n, int dtype,
                   void* stream) {
  if (n <= 0 || dtype < 0 || dtype > 1) return -1;
  if (!aligned16(dy) || !aligned16(a) || !aligned16(b) || !aligned16(da) || !aligned16(db)) return -2;
  const unsigned grid = grid_for(n / 8 + 1);
  if (dtype == 0)
    hipLaunchKernelGGL(swiglu_bwd_kernel<float>, dim3(grid), dim3(kT), 0, (hipStream_t)stream, (const float*)dy,
                       (const float*)a, (const float*)b, (float*)da, (float*)db, n);
  else
    hipLaunchKernelGGL(swiglu_bwd_kernel<uint16_t>, dim3(grid), dim3(kT), 0, (hipStream_t)stream,
                       (const uint16_t*)dy, (const uint16_t*)a, (const uint16_t*)b, (uint16_t*)da,
                       (uint16_t*)db, n);
  return (int)hipGetLastError();
}

// packed [tokens, (Hq + 2 Hkv) * D] <-> q [tokens, Hq, D], k / v [tokens, Hkv, D]; dir 0 / 1.
int pto_rope_qkv(void* packed, void* q, void* k, void* v, const float* cosb, const float* sinb, long tokens,
                 int S, int Hq, int Hkv, int D, int dir, int dtype, void* stream) {
  if (tokens <= 0 || S <= 0 || tokens % S || Hq <= 0 || Hkv <= 0 || D <= 0 || D % 8 || dir < 0 || dir > 1 ||
      dtype < 0 || dtype > 1)
    return -1;
  if (!aligned16(packed) || !aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(cosb) ||
      !aligned16(sinb))
    return -2;
  const long groups = tokens * ((Hq + 2 * Hkv) * D / 8);
  if (dtype == 0)
    hipLaunchKernelGGL(rope_qkv_kernel<float>, dim3(grid_for(groups)), dim3(kT), 0, (hipStream_t)stream,
                       (float*)packed, (float*)q, (float*)k, (float*)v, cosb, sinb, tokens, S, Hq, Hkv, D, dir);
  else
    hipLaunchKernelGGL(rope_qkv_kernel<uint16_t>, dim3(grid_for(groups)), dim3(kT), 0, (hipStream_t)stream,
                       (uint16_t*)packed, (uint16_t*)q, (uint16_t*)k, (uint16_t*)v, cosb, sinb, tokens, S, Hq,
                       Hkv, D, dir);
  return (int)hipGetLastError();
}

int pto_swiglu_packed_fwd(const void* x, void* y, long rows, int F, int dtype, void* stream) {
  if (rows <= 0 || F <= 0 || F % 8 || dtype < 0 || dtype > 1) return -1;
  if (!aligned16(x) || !aligned16(y)) return -2;
  const unsigned grid = grid_for(rows * (F / 8));
  if (dtype == 0)
    hipLaunchKernelGGL(swiglu_packed_fwd_kernel<float>, dim3(grid), dim3(kT), 0, (hipStream_t)stream,
                       (const float*)x, (float*)y, rows, F);
  else
    hipLaunchKernelGGL(swiglu_packed_fwd_kernel<uint16_t>, dim3(grid), dim3(kT), 0, (hipStream_t)stream,
                       (const uint16_t*)x, (uint16_t*)y, rows, F);
  return (int)hipGetLastError();
}

int pto_swiglu_packed_bwd(const void* dy, const void* x, void* dx, long rows, int F, int dtype, void* stream) {
  if (rows <= 0 || F <= 0 || F % 8 || dtype < 0 || dtype > 1) return -1;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(dx)) return -2;
  const unsigned grid = grid_for(rows * (F / 8));
  if (dtype == 0)
    hipLaunchKernelGGL(swiglu_packed_bwd_kernel<float>, dim3(grid), dim3(kT), 0, (hipStream_t)stream,
                       (const float*)dy, (const float*)x, (float*)dx, rows, F);
  else
    hipLaunchKernelGGL(swiglu_packed_bwd_kernel<uint16_t>, dim3(grid), dim3(kT), 0, (hipStream_t)stream,
                       (const uint16_t*)dy, (const uint16_t*)x, (uint16_t*)dx, rows, F);
  return (int)hipGetLastError();
}

// [rows, cols] 16-bit -> [cols, rows]; rows % 64 == cols % 64 == 0, 16-byte aligned.
int pto_transpose16(const void* in, void* out, long rows, long cols, void* stream) {
  if (rows <= 0 || cols <= 0 || rows % kTT || cols % kTT || rows / kTT > 65535 || cols / kTT > 0x7fffffffL) return -1;
  if (!aligned16(in) || !aligned16(out)) return -2;
  hipLaunchKernelGGL(transpose16_kernel, dim3((unsigned)(cols / kTT), (unsigned)(rows / kTT)), dim3(256), 0,
                     (hipStream_t)stream, (const uint16_t*)in, (uint16_t*)out, rows, cols);
  return (int)hipGetLastError();
}

// Cross-entropy over [rows, V] logits (dtype 0 = fp32, 1 = bf16), int64 targets.
int pto_xent_fwd(const void* x, const long* tgt, float* lse, float* loss, long rows, int V, long ignore_index,
                 int dtype, void* stream) {
  if (rows <= 0 || rows > 0x7fffffffL || V <= 0 || V % 8 || dtype < 0 || dtype > 1) return -1;
  if (!aligned16(x)) return -2;
  if (dtype == 0)
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3((unsigned)rows), dim3(kX), 0, (hipStream_t)stream,
                       (const float*)x, tgt, lse, loss, V, ignore_index);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<uint16_t>, dim3((unsigned)rows), dim3(kX), 0, (hipStream_t)stream,
                       (const uint16_t*)x, tgt, lse, loss, V, ignore_index);
  return (int)hipGetLastError();
}

int pto_xent_bwd(const void* x, const long* tgt, const float* lse, const float* scale, void* dx, long rows, int V,
                 long ignore_index, int dtype, void* stream) {
  if (rows <= 0 || rows > 0x7fffffffL || V <= 0 || V % 8 || dtype < 0 || dtype > 1) return -1;
  if (!aligned16(x) || !aligned16(dx)) return -2;
  if (dtype == 0)
    hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3((unsigned)rows), dim3(kX), 0, (hipStream_t)stream,
                       (const float*)x, tgt, lse, scale, (float*)dx, V, ignore_index);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<uint16_t>, dim3((unsigned)rows), dim3(kX), 0, (hipStream_t)stream,
                       (const uint16_t*)x, tgt, lse, scale, (uint16_t*)dx, V, ignore_index);
  return (int)hipGetLastError();
}

}  // extern "C"
