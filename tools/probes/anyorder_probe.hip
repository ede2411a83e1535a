// Probe: can a kernel launched with hipExtAnyOrderLaunch start before its in-stream
// predecessor ends on gfx950 (AQL barrier bit cleared), and what does a device-side
// completion-counter hand-off between two such launches cost vs a plain dependent boundary?
//
//   hipcc --offload-arch=gfx950 -O3 -o build/anyorder_probe tools/probes/anyorder_probe.hip
//   ./build/anyorder_probe            (prints one JSON line per test)
//
// Every wait is bounded by the 100 MHz wall clock (err flag set, kernel exits): nothing can hang.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ unsigned ld_relaxed(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// block 0 lane 0 spins `ticks` (100 MHz) then raises the flag
__global__ void spin_kernel(long long ticks, unsigned* flag, u64* ts) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const u64 t0 = wall_clock64();
    ts[0] = t0;
    while ((long long)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(4);
    ts[1] = wall_clock64();
    __hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void probe_kernel(unsigned* flag, u64* ts) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ts[2] = wall_clock64();
    ts[3] = ld_relaxed(flag);
  }
}

// One hop of a chain: wait until cnt[k-1] == nblk (all blocks of the previous kernel done),
// then each block writes `words` floats write-through (relaxed agent atomic stores = sc1) and
// reads the previous kernel's words, then counts itself done.
__global__ void __launch_bounds__(256) hop_kernel(unsigned* cnt, int k, unsigned nblk, float* buf, int words,
                                                  unsigned* err, u64* ts, int wait) {
  __shared__ int ok;
  const int tid = threadIdx.x;
  if (tid == 0) {
    ok = 1;
    if (wait && k > 0) {
      const u64 t0 = wall_clock64();
      while (ld_relaxed(&cnt[k - 1]) < nblk) {
        if (wall_clock64() - t0 > 2000000ull) {  // 20 ms
          atomicOr(err, 1u);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    if (blockIdx.x == 0) ts[2 * k] = wall_clock64();
  }
  __syncthreads();
  if (!ok) return;
  float s = 0.f;
  const float* src = buf + (size_t)((k + 1) & 1) * nblk * words + (size_t)blockIdx.x * words;
  float* dst = buf + (size_t)(k & 1) * nblk * words + (size_t)blockIdx.x * words;
  for (int i = tid; i < words; i += 256) s += src[i];
  for (int i = tid; i < words; i += 256)
    __hip_atomic_store(&dst[i], s + (float)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_fetch_add(&cnt[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(reinterpret_cast<unsigned long long*>(&ts[2 * k + 1]), (unsigned long long)wall_clock64(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int main(int argc, char** argv) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned *flag, *cnt, *err;
  u64* ts;
  float* buf;
  const int KMAX = 64;
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&cnt, KMAX * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&ts, 4 * KMAX * 8));
  CK(hipMalloc(&buf, 2 * 1024 * 4096 * 4));
  CK(hipMemset(buf, 0, 2 * 1024 * 4096 * 4));
  u64 h[4 * KMAX];

  // ---- test 1: does an any-order launch overlap a 50 us predecessor?
  for (int flags = 0; flags <= 1; ++flags) {
    CK(hipMemset(flag, 0, 4));
    CK(hipMemset(ts, 0, 64));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, 5000LL, flag, ts);
    hipExtLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, s, nullptr, nullptr, (unsigned)flags, flag, ts);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h, ts, 32, hipMemcpyDeviceToHost));
    printf("{\"test\": \"overlap\", \"anyorder\": %d, \"probe_start_minus_spin_end_us\": %.2f, \"flag_seen\": %llu}\n",
           flags, ((double)(long long)(h[2] - h[1])) / 100.0, h[3]);
  }

  // ---- test 2: chain of K hops, 256 blocks each: plain launches vs any-order + counter waits
  const int K = 48;
  for (int words : {16, 1024}) {
    for (int mode = 0; mode <= 1; ++mode) {
      double best = 1e30;
      unsigned e_host = 0;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipMemset(cnt, 0, KMAX * 4));
        CK(hipMemset(err, 0, 4));
        CK(hipMemset(ts, 0, 4 * KMAX * 8));
        CK(hipDeviceSynchronize());
        for (int k = 0; k < K; ++k) {
          if (mode == 0)
            hipLaunchKernelGGL(hop_kernel, dim3(256), dim3(256), 0, s, cnt, k, 256u, buf, words, err, ts, 0);
          else
            hipExtLaunchKernelGGL(hop_kernel, dim3(256), dim3(256), 0, s, nullptr, nullptr, 1u, cnt, k, 256u, buf,
                                  words, err, ts, 1);
        }
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h, ts, 2 * K * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&e_host, err, 4, hipMemcpyDeviceToHost));
        // per hop: first block start of kernel k+1 minus last block end of kernel k, and the
        // whole chain first start -> last end
        const double chain = (double)(h[2 * (K - 1) + 1] - h[0]) / 100.0;
        if (chain < best) best = chain;
      }
      double gap = 0;
      for (int k = 0; k + 1 < K; ++k) gap += (double)(long long)(h[2 * (k + 1)] - h[2 * k + 1]) / 100.0;
      printf("{\"test\": \"chain\", \"mode\": \"%s\", \"words_per_block\": %d, \"hops\": %d, \"chain_us_best\": %.2f, "
             "\"us_per_hop\": %.3f, \"mean_gap_end_to_next_start_us\": %.3f, \"err\": %u}\n",
             mode ? "anyorder+counter" : "plain", words, K, best, best / K, gap / (K - 1), e_host);
    }
  }
  CK(hipStreamDestroy(s));
  return 0;
}
