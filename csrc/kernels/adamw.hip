// Fused mixed-precision AdamW step for the Llama DDP worker (BASELINE "Llama-3 8B DDP bf16").
//
// The matmul weights live in bf16 (the tensors autocast matmuls read, so no per-step
// fp32->bf16 weight cast) and their gradients arrive in bf16 (no bf16->fp32 grad cast);
// the optimizer owns an fp32 master copy plus the fp32 moments.  One pass per parameter:
//
//   read  g (bf16 or fp32), master, m, v          write master, m, v, and the bf16 weight
//
// = 28 B per bf16-weight element, the same HBM traffic as torch's fused fp32 AdamW alone,
// with the two cast kernels (12 B/element) gone.  fp32 parameters (embedding, norm
// weights) use the same kernel with the parameter itself as the master and no bf16 copy.
// Semantics match torch.optim.AdamW (decoupled weight decay, bias-corrected moments):
//   p *= 1 - lr*wd;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p -= lr * (m / bc1) / (sqrt(v / bc2) + eps),   bc_i = 1 - b_i^t
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kT = 256;

struct AdamArgs {
  float lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, gscale;
};

__device__ __forceinline__ uint32_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ float adam1(float& p, float& m, float& v, float g, const AdamArgs& a) {
  g *= a.gscale;  // 1, or the data-parallel 1/W of an unscaled gradient sum (exact for W = 2^k)
  p *= 1.f - a.lr * a.wd;
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  // torch: denom = sqrt(v) / sqrt(bc2) + eps ; p -= (lr / bc1) * m / denom
  p -= a.lr * a.inv_bc1 * m / (sqrtf(v) * a.inv_sqrt_bc2 + a.eps);
  return p;
}

template <bool GBF16, bool OUTBF16>
__global__ __launch_bounds__(kT) void adamw_kernel(float* __restrict__ master, float* __restrict__ mom,
                                                   float* __restrict__ var, const void* __restrict__ grad,
                                                   uint16_t* __restrict__ out, long n, AdamArgs a) {
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * kT + threadIdx.x; i <= n4; i += (long)gridDim.x * kT) {
    if (i < n4) {
      float4 p = reinterpret_cast<float4*>(master)[i];
      float4 m = reinterpret_cast<float4*>(mom)[i];
      float4 v = reinterpret_cast<float4*>(var)[i];
      float g[4];
      if (GBF16) {
        const uint2 q = reinterpret_cast<const uint2*>(grad)[i];
        g[0] = __uint_as_float(q.x << 16);
        g[1] = __uint_as_float(q.x & 0xffff0000u);
        g[2] = __uint_as_float(q.y << 16);
        g[3] = __uint_as_float(q.y & 0xffff0000u);
      } else {
        const float4 q = reinterpret_cast<const float4*>(grad)[i];
        g[0] = q.x; g[1] = q.y; g[2] = q.z; g[3] = q.w;
      }
      adam1(p.x, m.x, v.x, g[0], a);
      adam1(p.y, m.y, v.y, g[1], a);
      adam1(p.z, m.z, v.z, g[2], a);
      adam1(p.w, m.w, v.w, g[3], a);
      reinterpret_cast<float4*>(master)[i] = p;
      reinterpret_cast<float4*>(mom)[i] = m;
      reinterpret_cast<float4*>(var)[i] = v;
      if (OUTBF16)
        reinterpret_cast<uint2*>(out)[i] =
            make_uint2(bf16_rne(p.x) | (bf16_rne(p.y) << 16), bf16_rne(p.z) | (bf16_rne(p.w) << 16));
    } else {
      for (long j = n4 * 4; j < n; ++j) {
        const float g = GBF16 ? __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(grad)[j] << 16)
                              : reinterpret_cast<const float*>(grad)[j];
        const float p = adam1(master[j], mom[j], var[j], g, a);
        if (OUTBF16) out[j] = (uint16_t)bf16_rne(p);
      }
    }
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

extern "C" {

// grad_bf16: gradient dtype (1 = bf16, 0 = fp32).  out: bf16 weight to refresh (nullptr for
// fp32 parameters, whose master IS the parameter).  step >= 1.  grad_scale multiplies the
// gradient first (ZeRO's gradient-view buckets hold the unscaled sum over ranks).
int pto_adamw_step_scaled(float* master, float* m, float* v, const void* grad, void* out, long n, int grad_bf16,
                          float lr, float b1, float b2, float eps, float wd, int step, float grad_scale,
                          void* stream) {
  if (n <= 0 || step < 1) return -1;
  if (!aligned16(master) || !aligned16(m) || !aligned16(v) || !aligned16(grad) || (out && !aligned16(out)))
    return -2;
  AdamArgs a;
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd; a.gscale = grad_scale;
  a.inv_bc1 = (float)(1.0 / (1.0 - pow((double)b1, step)));
  a.inv_sqrt_bc2 = (float)(1.0 / sqrt(1.0 - pow((double)b2, step)));
  const long work = n / 4 + 1;
  long blocks = (work + kT - 1) / kT;
  if (blocks > 8192) blocks = 8192;  // 32 waves per CU resident at most; grid-stride beyond
  const dim3 grid((unsigned)blocks), block(kT);
  hipStream_t s = (hipStream_t)stream;
  if (grad_bf16 && out) hipLaunchKernelGGL((adamw_kernel<true, true>), grid, block, 0, s, master, m, v, grad,
                                           (uint16_t*)out, n, a);
  else if (grad_bf16) hipLaunchKernelGGL((adamw_kernel<true, false>), grid, block, 0, s, master, m, v, grad,
                                         (uint16_t*)nullptr, n, a);
  else if (out) hipLaunchKernelGGL((adamw_kernel<false, true>), grid, block, 0, s, master, m, v, grad,
                                   (uint16_t*)out, n, a);
  else hipLaunchKernelGGL((adamw_kernel<false, false>), grid, block, 0, s, master, m, v, grad,
                          (uint16_t*)nullptr, n, a);
  return (int)hipGetLastError();
}

int pto_adamw_step(float* master, float* m, float* v, const void* grad, void* out, long n, int grad_bf16,
                   float lr, float b1, float b2, float eps, float wd, int step, void* stream) {
  return pto_adamw_step_scaled(master, m, v, grad, out, n, grad_bf16, lr, b1, b2, eps, wd, step, 1.f, stream);
}

}  // extern "C"
