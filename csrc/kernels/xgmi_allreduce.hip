// Single-node gradient all-reduce over xGMI peer memory, fused with the SGD update.
//
// Why: at B=64 the MNIST step is ~50 us of GPU time and the DDP gradient all-reduce is
// 1.7 MB (431k fp32).  RCCL launched from the host between graph replays adds its own
// launch/proxy latency and keeps the step out of a single hipGraph.  Every GPU of an
// 8x MI355X node has a direct xGMI link to every other, so a two-shot all-reduce done
// with ordinary stores into peer memory (IPC-mapped) moves only 2 x 1.7 MB x (W-1)/W per
// GPU, spread over all W-1 links, and is captured in the step's hipGraph like any other
// kernel.
//
// PUSH protocol (one launch per step, `nblk` workgroups per rank, all co-resident).
// Remote traffic is only posted stores (no remote loads, no remote polling: a remote load
// is a full xGMI round trip, a store is fire-and-forget); every wait polls LOCAL memory
// with one lane per flag, so W flags cost one local round trip, not W remote ones.
//
//   buffer (per rank, uncached device memory, IPC-exported):
//     [flag1[W][nblk] | flag2[W][nblk] | stepc[nblk] | pad | recv[W][shard] | gath[npad]]
//   shard = npad / W (rank q owns flat elements [q*shard, (q+1)*shard)),
//   chunk = shard / nblk (block b of every rank handles chunk b of each shard).
//   step s = ++stepc[b] (per block, local): flags hold step numbers, compared with >= s.
//
//   phase 1  produce + push: block b computes its balanced slice of the flat gradient
//            (the conv segment reduced from the per-sample slabs in fixed row order, the
//            rest copied) and stores every element into its OWNER's recv[my rank][.];
//            fence; flag1[my rank][b] := s on every rank.
//   phase 2  (owner) wait until flag1[q][j] >= s for every sender q and every sender block j
//            whose phase-1 slice lands in chunk b of my shard (push_sources; local, lanes in
//            parallel; a chunk fed only by the producer's pre-push waits on block b's flag);
//            chunk b of my shard = sum over senders in rank order (deterministic), scale 1/W; SGD on
//            it (mode 1, ZeRO-1: each parameter is updated by exactly one rank) or the mean
//            (mode 0); store the result locally and into every peer's gath[.]; fence;
//            flag2[my rank][b] := s on every rank.
//   phase 3  wait flag2[q][b] >= s for every q != me (local, one lane per owner), copy
//            chunk b of every other shard from gath into the output / parameters.
//
// Single buffering is safe: a rank writes step s+1 data into a peer only after its whole
// step-s launch finished, and that launch waited (phase 3) for every owner's flag2 of step
// s, which each owner raises only after it finished reading its step-s recv chunk; gath
// of step s+1 is written only after the owner saw flag1 of step s+1 from the receiver.
//
// Every wait is bounded (wall clock): on timeout the kernel sets an error word and goes
// on without waiting; later launches see the error and fall back to a rank-local SGD
// step (no remote traffic) instead of hanging.  The Python side self-tests the path
// against torch.distributed.all_reduce at start-up and falls back to RCCL when anything
// disagrees (parallel/xgmi.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>

#include "mnist_fc_grads.h"

namespace {

// clang vector type: element-wise arithmetic stays in VGPRs (HIP's f4 wrapper makes
// SROA give up on member references and spill to scratch)
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kMaxWorld = 8;
constexpr int kThreads = 256;  // threads per exchange workgroup (the one-GPU-per-rank kernel)
constexpr int kEmuThreads = 64;  // emulation of W x nblk > 1024 workgroups on one GPU: one wave each,
                                 // so every emulated rank's workgroups fit on the device at once
constexpr int kMaxBlocks = 256;
constexpr size_t kHdrBytes = 64 * 1024;  // flag1 + flag2 + stepc (<= 2*8*256*4 + 1 KB)

struct XarArgs {
  char* base[kMaxWorld];  // every rank's buffer (IPC-mapped; base[rank] is local)
  int rank, world, nblk, mode;
  long n4, npad4, shard4, chunk4;
  const float* in;
  float* out;            // mode 0
  float* p;              // mode 1: parameters (updated in place)
  float* mbuf;           // mode 1: momentum buffer
  float lr, momentum, dampening, wd, scale;
  int nesterov, first_step;
  int* step_counter;     // optional: advanced once per launch (the trainer's batch cursor)
  // optional fused slab reduction: the first conv4 f4s of the gradient are
  // sum_{r < slab_rows} slab[r * slab_stride + .] (the conv backward's per-sample partials)
  // (conv_bwd4: the columns [big_lo4, big_hi4) hold one row per 4-sample chunk and are
  // summed over slab_rows_big rows)
  const float* slab;
  int slab_rows, slab_rows_big;
  long slab_stride, conv4, big_lo4, big_hi4;
  // [skip_lo4, skip_hi4): gradient float4s an earlier launch of this step already pushed into
  // their owners' receive buffers (fc1_bwd's dW_fc1 tiles, mnist_kernels.hip XPush); phase 1
  // produces and pushes only the rest
  long skip_lo4, skip_hi4;
  int* err;
  long long timeout_ticks;  // wall_clock64 ticks (100 MHz)
  unsigned long long* stamps;  // optional: 4 wall_clock64 stamps per (rank, block)
  // stamp_ring > 0 (the one-rank-per-process exchange, diagnostics): stamps is a ring of
  // stamp_ring launches x nblk records of 8 words -- step, block start, flag1 raised, flag2
  // raised, end, error word at the end, first pending flag1 index (q * nblk + j) + 1 at a
  // phase-2 timeout; a launch that starts degraded writes none (the failing one is kept)
  int stamp_ring;
  int light_fence;  // exchange buffers are uncached: no L2 writeback / invalidate needed
  // fc_tiles (the fused DDP step, round 6): phase 1 also computes the fully connected layers'
  // gradients on MFMA from the step's activations (mnist_fc_grads.h: dW_fc1 / db_fc1 from dh and
  // a2, dW_fc2 / db_fc2 from d(logits) and h) and deposits them straight with their owners, and
  // writes the step's loss statistics -- no producer launch stores or pushes them.  The fc range is
  // the skip range [skip_lo4, n4); fc_*4: float4 offsets of fc1.weight / fc1.bias / fc2.weight /
  // fc2.bias in the flat gradient.  An owner then waits for every sender block (the tiles of a
  // chunk come from any block).
  int fc_tiles, fc_B;
  const float *fc_dh, *fc_a2, *fc_dlog, *fc_h, *fc_per_sample;
  float* fc_stats;
  float fc_loss_scale;
  long fc_w1_4, fc_b1_4, fc_w2_4, fc_b2_4;
};

// Release before raising a flag / acquire after seeing one.  The exchange buffers are
// allocated uncached (MTYPE UC), so their data never sits in any L2: draining this wave's
// outstanding memory operations (s_waitcnt) orders them.  A system-scope fence would also
// write back (buffer_wbl2) / invalidate (buffer_inv) the whole L2 of this XCD -- 10s of
// us when the step's tensors are dirty in it -- and is kept only for cached fallbacks.
__device__ __forceinline__ void release_fence(const XarArgs& a) {
  if (a.light_fence) {
    __builtin_amdgcn_s_waitcnt(0);  // every store of this wave acknowledged
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  } else {
    __threadfence_system();
  }
}
__device__ __forceinline__ void acquire_fence(const XarArgs& a) {
  if (a.light_fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  else __atomic_thread_fence(__ATOMIC_ACQUIRE);
}

__device__ __forceinline__ unsigned* flag1(char* b, int nblk, int q, int blk) {
  return reinterpret_cast<unsigned*>(b) + q * nblk + blk;
}
__device__ __forceinline__ unsigned* flag2(char* b, int nblk, int q, int blk) {
  return reinterpret_cast<unsigned*>(b) + (kMaxWorld + q) * nblk + blk;
}
__device__ __forceinline__ unsigned* stepc(char* b, int nblk, int blk) {
  return reinterpret_cast<unsigned*>(b) + 2 * kMaxWorld * nblk + blk;
}
// Pre-exchange rank barrier (XarCtx::prebarrier): pb_flag(b, q) = the last barrier step rank q
// arrived at, in rank b's buffer; pb_step = this rank's own barrier count.  Fixed offsets past the
// largest flag1 / flag2 / stepc layout (kMaxBlocks), inside the 64 KB header.
constexpr int kPbWord = 2 * kMaxWorld * kMaxBlocks + kMaxBlocks + 64;
__device__ __forceinline__ unsigned* pb_flag(char* b, int q) {
  return reinterpret_cast<unsigned*>(b) + kPbWord + q;
}
__device__ __forceinline__ unsigned* pb_step(char* b) {
  return reinterpret_cast<unsigned*>(b) + kPbWord + kMaxWorld;
}
static_assert((kPbWord + kMaxWorld + 1) * 4 <= (int)kHdrBytes, "pre-barrier words inside the header");

__device__ __forceinline__ f4* recv_buf(char* b) {
  return reinterpret_cast<f4*>(b + kHdrBytes);
}
__device__ __forceinline__ f4* gath_buf(char* b, long npad4) {
  return reinterpret_cast<f4*>(b + kHdrBytes) + npad4;
}

// Buffer of rank q: a select chain over the kernel arguments (SGPR selects when q is
// uniform) -- keeps the pointer in the global address space and `a` out of scratch.
__device__ __forceinline__ char* peer(const XarArgs& a, int q) {
  char* r = a.base[0];
#pragma unroll
  for (int k = 1; k < kMaxWorld; ++k) r = q == k ? a.base[k] : r;
  return r;
}

// Posted store into a peer's buffer, written through to memory (sc0 sc1 = system scope)
// whatever MTYPE the importing GPU's page tables give the IPC mapping of a REMOTE device's
// buffer: the light fence below (s_waitcnt only) is then enough on every fabric, not just
// for the uncached local allocation the 1-GPU tests exercise.  A 16-B write-through store
// costs about what a plain one does (MI355X_MICROARCH.md, hand-off price list).
__device__ __forceinline__ void push4(f4* p, f4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ unsigned load_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void store_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Error word bits: which bounded wait timed out first (host reads it with pto_xar_error)
constexpr int kErrPushWait = 1;    // phase 2: the senders' flag1 (their pushes to this owner)
constexpr int kErrGatherWait = 2;  // phase 3: an owner's flag2 (its updated shard)
constexpr int kErrPreBarrier = 4;  // the pre-exchange rank barrier

// Poll one local flag until >= target; false (error flagged) on timeout.
__device__ bool wait_flag(const unsigned* p, unsigned target, long long deadline, int* err, int code) {
  while (load_sys(p) < target) {
    if ((long long)wall_clock64() > deadline) {
      atomicOr(err, code);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// torch.optim.SGD (momentum, dampening, weight decay, nesterov) on four elements
// (explicit fmas in mnist_kernels.hip's sgd_elem order: bit-identical to the 1-GPU step)
__device__ __forceinline__ void sgd4(f4& p, f4 g, f4& m, const XarArgs& a, float scale) {
  const f4 wd = a.wd, mo = a.momentum, nlr = -a.lr;
  f4 d = __builtin_elementwise_fma(wd, p, g * scale);
  if (a.momentum != 0.f) {
    m = a.first_step ? d : __builtin_elementwise_fma(mo, m, (1.f - a.dampening) * d);
    d = a.nesterov ? __builtin_elementwise_fma(mo, m, d) : m;
  }
  p = __builtin_elementwise_fma(nlr, d, p);
}

// Element v (float4 units, v < npad4) of this rank's flat gradient outside the slab-reduced
// conv segment.  Padding reads as zero.
__device__ __forceinline__ f4 grad4(const XarArgs& a, long v) {
  return v < a.n4 ? reinterpret_cast<const f4*>(a.in)[v] : f4{0.f, 0.f, 0.f, 0.f};
}


// Deposit gradient element v with the rank that owns it (or apply a local SGD step when
// the exchange is degraded).
__device__ __forceinline__ void deposit(const XarArgs& a, long v, f4 g, bool degraded) {
  if (degraded) {
    if (v >= a.n4) return;
    if (a.mode == 0) {
      reinterpret_cast<f4*>(a.out)[v] = g;
    } else {
      f4 pp = reinterpret_cast<f4*>(a.p)[v];
      f4 bb = reinterpret_cast<f4*>(a.mbuf)[v];
      sgd4(pp, g, bb, a, 1.f);
      reinterpret_cast<f4*>(a.p)[v] = pp;
      reinterpret_cast<f4*>(a.mbuf)[v] = bb;
    }
    return;
  }
  const int q = (int)((unsigned)v / (unsigned)a.shard4);  // npad4 < 2^31 (host-checked)
  const long pos = v - (long)q * a.shard4;
  push4(recv_buf(peer(a, q)) + (long)a.rank * a.shard4 + pos, g);
}

// Wait until flag1[q][j] >= target for every sender q and every sender block j in the (at
// most 3) ranges [lo[k], hi[k]); flags are [q][nblk] contiguous.  All of a thread's flags are
// loaded back to back (one local round trip per poll), the block leaves together.  False (error
// flagged) on timeout.
template <int NT>
__device__ bool wait_flag_ranges(const unsigned* f, int nblk, int world, const int (&lo)[3], const int (&hi)[3],
                                 unsigned target, long long deadline, int* err, int code) {
  const int n0 = hi[0] - lo[0], n1 = hi[1] - lo[1], n = n0 + n1 + (hi[2] - lo[2]);
  for (;;) {
    int pending = 0;
    for (int i = threadIdx.x; i < world * n; i += NT) {
      const int q = i / n, j = i - q * n;
      const int blk = j < n0 ? lo[0] + j : (j < n0 + n1 ? lo[1] + j - n0 : lo[2] + j - n0 - n1);
      pending |= load_sys(f + q * nblk + blk) < target;
    }
    if (!__syncthreads_or(pending)) return true;
    if ((long long)wall_clock64() > deadline) {
      if (threadIdx.x == 0) atomicOr(err, code);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Sender blocks whose phase-1 pushes land in chunk b of my shard -- the same block indices on
// every sender (every rank partitions its gradient identically): the conv columns of the chunk
// (slab reduction, per_c columns per block) and its copied elements before / after the
// pre-pushed range (per logical elements per block).  A chunk wholly inside the pre-pushed
// range needs no phase-1 data; it waits on sender block b's flag alone, which proves that
// sender's exchange launch began, so its producer launch (and its pre-push) had finished.
__device__ __forceinline__ void push_sources(const XarArgs& a, int b, int (&lo)[3], int (&hi)[3]) {
  if (a.fc_tiles) {  // in-launch fc tiles: any sender block may feed any chunk
    lo[0] = 0;
    hi[0] = a.nblk;
    lo[1] = hi[1] = lo[2] = hi[2] = 0;
    return;
  }
  const long c4 = a.slab != nullptr ? a.conv4 : 0;
  const long skip = a.skip_hi4 - a.skip_lo4;
  const long rest = a.npad4 - c4 - skip;
  const long per = (rest + a.nblk - 1) / a.nblk;
  const long per_c = c4 > 0 ? (c4 + a.nblk - 1) / a.nblk : 1;
  const long f_lo = (long)a.rank * a.shard4 + (long)b * a.chunk4, f_hi = f_lo + a.chunk4;
  for (int k = 0; k < 3; ++k) lo[k] = hi[k] = 0;
  if (f_lo < c4) {  // conv columns
    lo[0] = (int)(f_lo / per_c);
    hi[0] = (int)((min(f_hi, c4) - 1) / per_c) + 1;
  }
  const long sk_lo = max(a.skip_lo4, c4), sk_hi = max(a.skip_hi4, c4);
  const long a_lo = max(f_lo, c4), a_hi = min(f_hi, sk_lo);  // before the pre-pushed range
  if (a_lo < a_hi) {
    lo[1] = (int)((a_lo - c4) / per);
    hi[1] = (int)((a_hi - 1 - c4) / per) + 1;
  }
  const long b_lo = max(f_lo, sk_hi), b_hi = f_hi;  // after it
  if (b_lo < b_hi) {
    lo[2] = (int)((b_lo - c4 - skip) / per);
    hi[2] = (int)((b_hi - 1 - c4 - skip) / per) + 1;
  }
  if (lo[0] == hi[0] && lo[1] == hi[1] && lo[2] == hi[2]) {
    lo[0] = b;
    hi[0] = b + 1;
  }
}

// Phase 1's fc gradient tiles (XarArgs::fc_tiles): tile t of the 1600 dW_fc1 tiles (row tile t / 50,
// column tile t % 50) then the 32 dW_fc2 tiles, one wave each, dealt round-robin over every wave of
// every block.  Each lane deposits its 16-byte run of dW_fc1 as computed; db_fc1, dW_fc2 and db_fc2
// run along rows whose four consecutive elements sit in lanes i .. i + 3, so lane i (i % 4 == 0)
// gathers them (ds_bpermute) and deposits one float4.
template <int NT>
__device__ __forceinline__ void fc_tiles_phase1(const XarArgs& a, int b, bool degraded) {
  constexpr int kWpb = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  if (b == a.nblk - 1) {
    // the padding float4s inside the fc range (between / after the four tensors): zero, deposited
    // like the rest -- an owner's receive slot keeps whatever was last written to it (the start-up
    // self-test's data), and the padding would otherwise take SGD steps with that
    const long gaps[4][2] = {{a.fc_w1_4 + 100000, a.fc_b1_4}, {a.fc_b1_4 + 125, a.fc_w2_4},
                             {a.fc_w2_4 + 1250, a.fc_b2_4}, {a.fc_b2_4 + 3, a.n4}};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      for (long v = gaps[k][0] + tid; v < gaps[k][1]; v += NT) deposit(a, v, f4{0.f, 0.f, 0.f, 0.f}, degraded);
  }
  for (int t = b * kWpb + wv; t < 1632; t += a.nblk * kWpb) {  // wave-uniform
    float dbsum;
    if (t < 1600) {
      const int nt = t / 50, kt = t - nt * 50;
      const f4 c = pto::fc1_wgrad_tile(a.fc_dh, a.fc_a2, a.fc_B, nt, kt, lane, dbsum);
      const int n = nt * 16 + i;
      if (n < 500) deposit(a, a.fc_w1_4 + (long)(n * 200 + kt * 4 + g), c, degraded);
      if (kt == 0) {
        dbsum = pto::sum_lane_rows(dbsum);
        const float d1 = __shfl_down(dbsum, 1, 64), d2 = __shfl_down(dbsum, 2, 64), d3 = __shfl_down(dbsum, 3, 64);
        if (g == 0 && (i & 3) == 0 && n < 500) deposit(a, a.fc_b1_4 + n / 4, f4{dbsum, d1, d2, d3}, degraded);
      }
    } else {
      const int nt = t - 1600;
      const bool do_stats = nt == 1 && a.fc_stats != nullptr;
      float ls = 0.f, cs = 0.f;
      if (do_stats) pto::loss_stats_load(a.fc_per_sample, a.fc_B, lane, ls, cs);
      const f4 c = pto::fc2_wgrad_tile(a.fc_dlog, a.fc_h, a.fc_B, nt, lane, dbsum);
      const int n = nt * 16 + i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = c[r];
        const float v1 = __shfl_down(v, 1, 64), v2 = __shfl_down(v, 2, 64), v3 = __shfl_down(v, 3, 64);
        const int j = 4 * g + r;
        if (j < 10 && (i & 3) == 0 && n < 500) deposit(a, a.fc_w2_4 + (long)(j * 500 + n) / 4, f4{v, v1, v2, v3}, degraded);
      }
      if (nt == 0) {
        dbsum = pto::sum_lane_rows(dbsum);  // zero for classes >= 10: the padding float4 stays zero
        const float d1 = __shfl_down(dbsum, 1, 64), d2 = __shfl_down(dbsum, 2, 64), d3 = __shfl_down(dbsum, 3, 64);
        if (g == 0 && (i & 3) == 0 && i < 12) deposit(a, a.fc_b2_4 + i / 4, f4{dbsum, d1, d2, d3}, degraded);
      }
      if (do_stats) {
        pto::loss_stats_finish(a.fc_per_sample, a.fc_B, lane, ls, cs);
        if (lane == 0) {
          a.fc_stats[0] = ls * a.fc_loss_scale;
          a.fc_stats[1] = cs;
        }
      }
    }
  }
}

constexpr int kP2 = 2;  // phase-2 elements per thread per batch (chunk4 > kThreads: xar_kernel_p2)
constexpr int kP3 = 4;  // phase-3 float4s per thread per batch

// FC: the fused DDP step's exchange (XarArgs::fc_tiles), a separate instantiation so the round-5
// exchange keeps its register allocation (the tiles' operands raise it from 112 to 152 VGPRs --
// what decides whether the step's kernels fit beside a spinning exchange when ranks share a GPU,
// tests/test_kernel_resources.py).  P2: phase-2 float4s per thread per batch.  A chunk of at most
// NT float4s (every chunk at 256 workgroups and world >= 2: 53 at world 8) needs one, and the
// 8 senders' operands of a second batch are what held the exchange at 112 VGPRs: P2 = 1 brings it
// under 96, so even the 4-wave fused conv12 forward (4 x 104) fits beside a spinning exchange wave.
template <int NT, bool FC = false, int P2 = kP2>
__device__ __forceinline__ void xar_body(const XarArgs& a, const int b) {
  constexpr int kThreads = NT;
  __shared__ unsigned s_step;
  __shared__ int s_degraded;
  __shared__ f4 part[kThreads];
  const int tid = threadIdx.x;
  char* mine = peer(a, a.rank);
  if (tid == 0) {
    s_step = load_sys(stepc(mine, a.nblk, b)) + 1u;
    s_degraded = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  }
  __syncthreads();
  const unsigned s = s_step;
  const bool degraded = s_degraded;
  const long long deadline = (long long)wall_clock64() + a.timeout_ticks;
  unsigned long long* st = nullptr;
  if (a.stamps != nullptr) {
    if (a.stamp_ring == 0) {
      st = a.stamps + ((long)a.rank * a.nblk + b) * 4;
    } else if (!degraded) {
      unsigned long long* r = a.stamps + ((long)(s % (unsigned)a.stamp_ring) * a.nblk + b) * 8;
      if (tid == 0) {
        r[0] = s;
        for (int k = 2; k < 8; ++k) r[k] = 0ull;
      }
      st = r + 1;
    }
  }
  if (st != nullptr && tid == 0) st[0] = wall_clock64();
  const f4 zero4 = f4{0.f, 0.f, 0.f, 0.f};

  // ---- phase 1: produce my gradient slice and push it to the owners
  {
    const long c4 = a.slab != nullptr ? a.conv4 : 0;
    // the copied segment: logical index L -> flat float4 v = c4 + L, stepping over the
    // pre-pushed range [skip_lo4, skip_hi4) (host-checked: skip_lo4 >= c4)
    const long skip = a.skip_hi4 - a.skip_lo4;
    const long rest = a.npad4 - c4 - skip;
    const long per = (rest + a.nblk - 1) / a.nblk;
    const long lo4 = (long)b * per, hi4 = min(lo4 + per, rest);
    auto vmap = [&](long L) {
      const long v = c4 + L;
      return v >= a.skip_lo4 ? v + skip : v;
    };
    // first batch of the copied segment: loads in flight while the slab rows are summed
    f4 g0, g1, g2, g3;
    // unconditional loads from clamped addresses, then selects (a predicated load becomes
    // a branch + a wait per element)
    const f4* gin = reinterpret_cast<const f4*>(a.in);
    const long vmax = a.n4 - 1;
    auto ld = [&](long L) {
      const long v = vmap(L);
      const f4 x = gin[v < vmax ? v : vmax];
      return (L < hi4 && v < a.n4) ? x : zero4;
    };
    auto load_batch = [&](long v0) {
      g0 = ld(v0);
      g1 = ld(v0 + kThreads);
      g2 = ld(v0 + 2 * kThreads);
      g3 = ld(v0 + 3 * kThreads);
    };
    load_batch(lo4 + tid);
    if constexpr (FC) fc_tiles_phase1<NT>(a, b, degraded);
    if (c4 > 0) {
      // conv segment: columns [b*per_c, (b+1)*per_c) reduced over the slab rows, split in
      // nsplit row groups (fixed order -> deterministic)
      const int per_c = (int)((c4 + a.nblk - 1) / a.nblk);  // <= kThreads (host-checked)
      int nsplit = kThreads / per_c;
      nsplit = nsplit < 1 ? 1 : (nsplit > 8 ? 8 : nsplit);
      const int grp = tid / per_c, ci = tid - grp * per_c;
      const long col = (long)b * per_c + ci;
      const int rows = (col >= a.big_lo4 && col < a.big_hi4) ? a.slab_rows_big : a.slab_rows;
      const int rows_per = (rows + nsplit - 1) / nsplit;
      f4 acc = zero4;
      if (grp < nsplit && col < c4) {
        const f4* sp = reinterpret_cast<const f4*>(a.slab) + col;
        const long s4 = a.slab_stride >> 2;
        const int r0 = grp * rows_per, r1 = min(rows, r0 + rows_per);
#pragma unroll 8
        for (int r = r0; r < r1; ++r) acc += sp[(long)r * s4];
      }
      part[tid] = acc;
      __syncthreads();
      if (tid < per_c && col < c4) {
        f4 gs = part[tid];
        for (int k = 1; k < nsplit; ++k) gs += part[k * per_c + tid];
        deposit(a, col, gs, degraded);
      }
    }
    for (long v0 = lo4 + tid; v0 < hi4; v0 += 4 * kThreads) {
      if (v0 != lo4 + tid) load_batch(v0);
      deposit(a, vmap(v0), g0, degraded);
      if (v0 + kThreads < hi4) deposit(a, vmap(v0 + kThreads), g1, degraded);
      if (v0 + 2 * kThreads < hi4) deposit(a, vmap(v0 + 2 * kThreads), g2, degraded);
      if (v0 + 3 * kThreads < hi4) deposit(a, vmap(v0 + 3 * kThreads), g3, degraded);
    }
    if (degraded && skip > 0 && !FC) {
      // rank-local fallback: the pre-pushed range still needs its local SGD step (the
      // pushing launch also stored it to `in`); block b takes its share of it
      const long sper = (skip + a.nblk - 1) / a.nblk;
      const long s0 = a.skip_lo4 + (long)b * sper, s1 = min(s0 + sper, a.skip_hi4);
      for (long v = s0 + tid; v < s1; v += kThreads) deposit(a, v, grad4(a, v), true);
    }
    if (degraded) {
      if (a.step_counter != nullptr && b == 0 && tid == 0) atomicAdd(a.step_counter, 1);
      if (tid == 0) store_sys(stepc(mine, a.nblk, b), s);
      return;
    }
    release_fence(a);
    __syncthreads();
    if (tid < a.world) store_sys(flag1(peer(a, tid), a.nblk, a.rank, b), s);
    if (st != nullptr && tid == 0) st[1] = wall_clock64();
  }

  // ---- phase 2: reduce chunk b of my shard (+ SGD), push the result to every rank
  {
    const long base4 = (long)a.rank * a.shard4 + (long)b * a.chunk4;
    const f4* rv = recv_buf(mine) + (long)b * a.chunk4;
    f4 pp[P2], bb[P2];
    auto load_pb = [&](long i0) {  // parameters / momentum: independent of the peers
#pragma unroll
      for (int k = 0; k < P2; ++k) {
        const long i = i0 + (long)k * kThreads, v = base4 + i;
        const bool in = a.mode == 1 && i < a.chunk4 && v < a.n4;
        pp[k] = in ? reinterpret_cast<const f4*>(a.p)[v] : zero4;
        bb[k] = in ? reinterpret_cast<const f4*>(a.mbuf)[v] : zero4;
      }
    };
    load_pb(tid);  // in flight while waiting
    // the flags of the sender blocks that feed this chunk (or timed out: go on, the error is
    // set); block-uniform.  Not every sender block's: chunks fed only by the producer's
    // pre-push start as soon as the matching sender block is in its exchange
    int src_lo[3], src_hi[3];
    push_sources(a, b, src_lo, src_hi);
    const bool got = wait_flag_ranges<NT>(reinterpret_cast<const unsigned*>(mine), a.nblk, a.world, src_lo,
                                          src_hi, s, deadline, a.err, kErrPushWait);
    if (!got && st != nullptr && a.stamp_ring > 0) {  // which sender block was missing
      const unsigned* f = reinterpret_cast<const unsigned*>(mine);
      for (int k = 0; k < 3; ++k)
        for (int j = src_lo[k] + tid; j < src_hi[k]; j += NT)
          for (int q = 0; q < a.world; ++q)
            if (load_sys(f + q * a.nblk + j) < s) atomicCAS(&st[5], 0ull, (unsigned long long)(q * a.nblk + j + 1));
    }
    acquire_fence(a);
    for (long i0 = tid;;) {  // no barrier inside: threads may leave at different times
      // every sender's contribution in flight at once (clamped addresses, no predicated
      // load: a runtime-bounded loop here waited a full memory round trip per sender)
      f4 rq[P2][kMaxWorld];
#pragma unroll
      for (int k = 0; k < P2; ++k) {
        const long i = min(i0 + (long)k * kThreads, a.chunk4 - 1);
#pragma unroll
        for (int q = 0; q < kMaxWorld; ++q) rq[k][q] = rv[(long)min(q, a.world - 1) * a.shard4 + i];
      }
      f4 acc[P2];
#pragma unroll
      for (int k = 0; k < P2; ++k) {
        acc[k] = rq[k][0];
#pragma unroll
        for (int q = 1; q < kMaxWorld; ++q)
          if (q < a.world) acc[k] += rq[k][q];  // rank order (deterministic)
      }
#pragma unroll
      for (int k = 0; k < P2; ++k) {
        const long i = i0 + (long)k * kThreads, v = base4 + i;
        if (i >= a.chunk4) continue;
        f4 res;
        if (a.mode == 0) {
          res = acc[k] * a.scale;
          if (v < a.n4) reinterpret_cast<f4*>(a.out)[v] = res;
        } else if (v < a.n4) {
          sgd4(pp[k], acc[k], bb[k], a, a.scale);
          reinterpret_cast<f4*>(a.p)[v] = pp[k];
          reinterpret_cast<f4*>(a.mbuf)[v] = bb[k];
          res = pp[k];
        } else {
          res = zero4;
        }
#pragma unroll
        for (int j = 1; j < kMaxWorld; ++j) {
          if (j >= a.world) break;
          const int q = a.rank + j < a.world ? a.rank + j : a.rank + j - a.world;
          push4(gath_buf(peer(a, q), a.npad4) + v, res);
        }
      }
      i0 += (long)P2 * kThreads;
      if (i0 >= a.chunk4) break;
      load_pb(i0);
    }
    release_fence(a);
    __syncthreads();
    if (tid < a.world && tid != a.rank) store_sys(flag2(peer(a, tid), a.nblk, a.rank, b), s);
    if (st != nullptr && tid == 0) st[2] = wall_clock64();
  }

  // ---- phase 3: collect chunk b of every other shard
  {
    int ok = 1;
    if (tid < a.world && tid != a.rank) ok = wait_flag(flag2(mine, a.nblk, tid, b), s, deadline, a.err, kErrGatherWait);
    (void)__syncthreads_and(ok);
    acquire_fence(a);
    f4* dst = reinterpret_cast<f4*>(a.mode == 0 ? a.out : a.p);
    const f4* gb = gath_buf(mine, a.npad4);
    const long tot = (long)(a.world - 1) * a.chunk4;
    for (long j0 = tid; j0 < tot; j0 += (long)kP3 * kThreads) {
      f4 x[kP3];
      long vv[kP3];
#pragma unroll
      for (int k = 0; k < kP3; ++k) {
        const long j = j0 + (long)k * kThreads;
        const long kk = j / a.chunk4, i = j - kk * a.chunk4;
        const int q = a.rank + 1 + (int)kk < a.world ? a.rank + 1 + (int)kk : a.rank + 1 + (int)kk - a.world;
        vv[k] = j < tot ? (long)q * a.shard4 + (long)b * a.chunk4 + i : a.n4;
        const f4 xg = gb[vv[k] < a.npad4 ? vv[k] : a.npad4 - 1];  // unconditional load
        x[k] = vv[k] < a.n4 ? xg : zero4;
      }
#pragma unroll
      for (int k = 0; k < kP3; ++k)
        if (vv[k] < a.n4) dst[vv[k]] = x[k];
    }
  }
  if (a.step_counter != nullptr && b == 0 && tid == 0) atomicAdd(a.step_counter, 1);
  if (tid == 0) store_sys(stepc(mine, a.nblk, b), s);
  if (st != nullptr && tid == 0) {
    st[3] = wall_clock64();
    if (a.stamp_ring > 0) st[4] = (unsigned long long)__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(kThreads) void xar_kernel(XarArgs a) { xar_body<kThreads, false, 1>(a, blockIdx.x); }
__global__ __launch_bounds__(kThreads) void xar_kernel_p2(XarArgs a) { xar_body<kThreads, false, 2>(a, blockIdx.x); }
__global__ __launch_bounds__(kThreads) void xar_kernel_fc(XarArgs a) { xar_body<kThreads, true, 1>(a, blockIdx.x); }
__global__ __launch_bounds__(kThreads) void xar_kernel_fc_p2(XarArgs a) { xar_body<kThreads, true, 2>(a, blockIdx.x); }

// Pre-exchange rank barrier (XarCtx::prebarrier; ranks sharing one GPU, the rehearsal of the
// one-GPU-per-rank geometry): ONE wave, no LDS, launched before the exchange on the same stream.
// An exchange's workgroups spin on the CUs until every peer's exchange joins; a peer still running
// its step kernels must then find room beside them -- and LDS / VGPR fragmentation around a
// spinning workgroup can leave none (conv_bwd4's 152 KB of LDS needs one contiguous range), which
// the exchange stamps showed as a peer starting only after the waiter's deadline.  With this
// barrier no rank's exchange starts before every rank has finished its step kernels: then only
// exchanges (and this one wave) share the CUs.  Bounded wait like the exchange's; a degraded
// exchange (error word set) skips it.
__global__ __launch_bounds__(64) void xar_prebarrier_kernel(XarArgs a) {
  const int lane = threadIdx.x;
  char* mine = peer(a, a.rank);
  if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;  // wave-uniform
  const unsigned s = load_sys(pb_step(mine)) + 1u;  // one writer (lane 0, below): every lane reads the same
  if (lane < a.world) store_sys(pb_flag(peer(a, lane), a.rank), s);
  const long long deadline = (long long)wall_clock64() + a.timeout_ticks;
  bool pending = lane < a.world;
  for (;;) {
    if (pending) pending = load_sys(pb_flag(mine, lane)) < s;
    if (!__any(pending)) break;  // before the deadline check: a barrier met as it expires is met
    if ((long long)wall_clock64() > deadline) {
      if (lane == 0) atomicOr(a.err, kErrPreBarrier);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (lane == 0) store_sys(pb_step(mine), s);
}

// Emulation of `world` ranks on ONE device in one launch (blockIdx.y = rank): all blocks
// of all ranks are co-resident, so the protocol (and its latency floor over local HBM)
// can be tested at any world size on a single GPU.  NT = kEmuThreads when the emulated
// grid (W x nblk workgroups) would not fit the device with 256-thread workgroups (W = 8 x
// 256: the production geometry); same chunking, flags and phases, fewer lanes per chunk.
// FC: the fused DDP step's exchange (xar_kernel_fc), e.g. at the W = 8 x 256 production geometry.
template <int NT, bool FC>
__global__ __launch_bounds__(NT) void xar_kernel_emu(const XarArgs* __restrict__ all) {
  xar_body<NT, FC>(all[blockIdx.y], blockIdx.x);
}

// Emulated producer push (what fc1_bwd does with XPush): every emulated rank (blockIdx.y)
// pushes its gradient float4s [skip_lo4, skip_hi4) into their owners' receive buffers, then
// waits for the stores (the exchange launch that follows skips that range).
__global__ __launch_bounds__(kThreads) void xar_emu_prepush(const XarArgs* __restrict__ all) {
  const XarArgs& a = all[blockIdx.y];
  for (long v = a.skip_lo4 + (long)blockIdx.x * kThreads + threadIdx.x; v < a.skip_hi4;
       v += (long)gridDim.x * kThreads)
    deposit(a, v, grad4(a, v), false);
  __builtin_amdgcn_s_waitcnt(0);
}

struct XarCtx {
  int rank, world, nblk, device;
  long n, npad;
  int alloc_kind;  // 3 = uncached, 1 = fine-grained, 0 = default
  char* base[kMaxWorld];
  int* err;
  long long timeout_ticks;
  unsigned long long* stamps;  // optional diagnostics ring (pto_xar_stamps)
  int stamp_ring;
  int prebarrier;  // launch xar_prebarrier_kernel before every exchange (pto_xar_prebarrier)
  int fence;       // -1: light fences iff the buffer is uncached; 0 / 1: forced (pto_xar_fence)
};

long round_up(long x, long m) { return (x + m - 1) / m * m; }

}  // namespace

extern "C" {

// Allocate this rank's exchange buffer; writes its 64-byte IPC handle to handle_out.
int pto_xar_create(int rank, int world, long n, int nblk, double timeout_s, void** ctx_out,
                   void* handle_out) {
  if (world < 2 || world > kMaxWorld || rank < 0 || rank >= world || n <= 0 || (n & 3) ||
      nblk < 1 || nblk > kMaxBlocks || n > (1L << 32))
    return -1;
  XarCtx* c = new XarCtx{};
  c->fence = -1;
  c->rank = rank;
  c->world = world;
  c->nblk = nblk;
  c->n = n;
  c->npad = round_up(n, (long)world * nblk * 4);
  if (hipGetDevice(&c->device) != hipSuccess) {
    delete c;
    return -2;
  }
  const size_t bytes = kHdrBytes + (size_t)2 * c->npad * sizeof(float);
  void* p = nullptr;
  const unsigned kinds[] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
  for (unsigned k : kinds) {
    if (hipExtMallocWithFlags(&p, bytes, k) == hipSuccess) {
      c->alloc_kind = (int)k;
      break;
    }
    p = nullptr;
    (void)hipGetLastError();
  }
  if (p == nullptr) {
    if (hipMalloc(&p, bytes) != hipSuccess) {
      delete c;
      return -2;
    }
    c->alloc_kind = 0;
  }
  c->base[rank] = static_cast<char*>(p);
  hipIpcMemHandle_t h;
  int rc = 0;
  if (hipMemset(p, 0, bytes) != hipSuccess || hipMalloc(&c->err, sizeof(int)) != hipSuccess ||
      hipMemset(c->err, 0, sizeof(int)) != hipSuccess)
    rc = -2;
  else if (hipIpcGetMemHandle(&h, p) != hipSuccess)
    rc = -3;
  else if (hipDeviceSynchronize() != hipSuccess)
    rc = -2;
  if (rc != 0) {
    (void)hipFree(c->err);
    (void)hipFree(p);
    delete c;
    return rc;
  }
  c->timeout_ticks = (long long)(timeout_s * 1e8);  // wall_clock64 runs at 100 MHz
  memcpy(handle_out, &h, sizeof(h));
  *ctx_out = c;
  return 0;
}

int pto_xar_alloc_kind(void* ctx) { return static_cast<XarCtx*>(ctx)->alloc_kind; }

// What a producer kernel needs to push gradient float4s straight into their owners' receive
// buffers (mnist_kernels.hip XPush): every rank's buffer base (world entries), this rank, the
// world size and the float4s per owner shard.
int pto_xar_push_info(void* ctx, void** bases, int* rank, int* world, long* shard4) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  for (int q = 0; q < c->world; ++q) bases[q] = c->base[q];
  *rank = c->rank;
  *world = c->world;
  *shard4 = (c->npad >> 2) / c->world;
  return 0;
}
long pto_xar_npad(void* ctx) { return static_cast<XarCtx*>(ctx)->npad; }
// Device address of the exchange's error word (non-zero after a bounded wait timed out): a
// producer that pushes into peers' receive buffers checks it and stops pushing (XPush::err).
void* pto_xar_err_ptr(void* ctx) { return static_cast<XarCtx*>(ctx)->err; }

// Diagnostics: per-block phase stamps of the last `ring` launches into buf (ring x nblk x 8
// uint64, see XarArgs::stamp_ring; wall_clock64 at 100 MHz, shared by every process on the GPU).
// Null buf turns them off.  Applies to launches made (or captured) afterwards.
int pto_xar_stamps(void* ctx, unsigned long long* buf, int ring) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  if (buf != nullptr && ring < 1) return -1;
  c->stamps = buf;
  c->stamp_ring = buf != nullptr ? ring : 0;
  return 0;
}

// Diagnostics: force the release / acquire fences light (1: s_waitcnt + workgroup fence) or full
// (0: system-scope fences with L2 writeback / invalidate); -1 restores the default (light iff the
// buffer is uncached).  Applies to launches made (or captured) afterwards.
int pto_xar_fence(void* ctx, int light) {
  if (light < -1 || light > 1) return -1;
  static_cast<XarCtx*>(ctx)->fence = light;
  return 0;
}

// Ranks sharing one GPU: a one-wave rank barrier before every later (or later-captured) exchange
// launch (xar_prebarrier_kernel).  Off by default: one rank per GPU never needs it.
int pto_xar_prebarrier(void* ctx, int on) {
  static_cast<XarCtx*>(ctx)->prebarrier = on != 0;
  return 0;
}

// Map every peer's buffer (handles: world x 64 bytes, in rank order).
int pto_xar_open(void* ctx, const void* handles) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank) continue;
    hipIpcMemHandle_t h;
    memcpy(&h, static_cast<const char*>(handles) + (size_t)q * sizeof(h), sizeof(h));
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return 100 + (int)e;
    c->base[q] = static_cast<char*>(p);
  }
  return 0;
}

// Restart the protocol after a failed exchange: zero this rank's header (flags, step counters,
// pre-barrier words) and error word.  Collective: every rank calls it with no exchange in flight
// on any rank (its caller synchronises and barriers before and after), so every rank's next
// exchange starts from step 1 against peers that also do.
int pto_xar_reset(void* ctx) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemset(c->base[c->rank], 0, kHdrBytes) != hipSuccess || hipMemset(c->err, 0, sizeof(int)) != hipSuccess)
    return -2;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}

// Workgroups of this rank's exchange kernel (the fused-form one with fc != 0) that the device holds
// at once, by the occupancy calculator: ranks sharing one GPU can only finish an exchange when
// all of their exchange workgroups are resident together.
int pto_xar_resident_blocks(void* ctx, int fc) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  const long shard4 = (c->npad >> 2) / c->world;
  const bool one = shard4 / c->nblk <= kThreads;
  const void* k = fc ? (one ? (const void*)xar_kernel_fc : (const void*)xar_kernel_fc_p2)
                     : (one ? (const void*)xar_kernel : (const void*)xar_kernel_p2);
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, 0) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) return -1;
  return per_cu * cus;
}

int pto_xar_error(void* ctx) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  int v = 0;
  if (hipMemcpy(&v, c->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}

static int launch(XarCtx* c, XarArgs& a, void* stream) {
  for (int q = 0; q < kMaxWorld; ++q) a.base[q] = q < c->world ? c->base[q] : nullptr;
  a.rank = c->rank;
  a.world = c->world;
  a.nblk = c->nblk;
  a.n4 = c->n >> 2;
  a.npad4 = c->npad >> 2;
  a.shard4 = a.npad4 / c->world;
  a.chunk4 = a.shard4 / c->nblk;
  a.err = c->err;
  a.timeout_ticks = c->timeout_ticks;
  a.stamps = c->stamps;
  a.stamp_ring = c->stamp_ring;
  a.light_fence = c->fence >= 0 ? c->fence : c->alloc_kind == (int)hipDeviceMallocUncached;
  if ((((uintptr_t)a.in) | ((uintptr_t)a.out) | ((uintptr_t)a.p) | ((uintptr_t)a.mbuf)) & 15) return -2;
  if (c->prebarrier) {
    hipLaunchKernelGGL(xar_prebarrier_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  const bool one = a.chunk4 <= kThreads;  // phase 2 in one batch per thread
  auto* k = a.fc_tiles ? (one ? xar_kernel_fc : xar_kernel_fc_p2) : (one ? xar_kernel : xar_kernel_p2);
  hipLaunchKernelGGL(k, dim3(c->nblk), dim3(kThreads), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// out = mean over ranks of in (n floats).
int pto_xar_allreduce(void* ctx, const float* in, float* out, float scale, void* stream) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  XarArgs a{};
  a.mode = 0;
  a.in = in;
  a.out = out;
  a.scale = scale;
  return launch(c, a, stream);
}

static int prep_sgd(XarCtx* c, XarArgs& a, const float* grads, float* p, float* mbuf, float lr, float momentum,
                    float dampening, float wd, float scale, int nesterov, int first_step, int* step_counter,
                    const float* slab, int slab_rows, long slab_stride, long conv_n, int slab_rows_big, long big_lo,
                    long big_hi, long skip_lo, long skip_hi) {
  a.mode = 1;
  if (skip_lo < 0 || skip_hi < skip_lo || skip_hi > c->n || (skip_lo & 3) || (skip_hi & 3) ||
      (skip_hi > skip_lo && skip_lo < (slab != nullptr ? conv_n : 0)))
    return -1;
  a.skip_lo4 = skip_lo >> 2;
  a.skip_hi4 = skip_hi >> 2;
  a.in = grads;
  a.p = p;
  a.mbuf = mbuf;
  a.lr = lr;
  a.momentum = momentum;
  a.dampening = dampening;
  a.wd = wd;
  a.scale = scale;
  a.nesterov = nesterov;
  a.first_step = first_step;
  a.step_counter = step_counter;
  if (slab != nullptr) {
    if (slab_rows <= 0 || (conv_n & 3) || (slab_stride & 3) || slab_stride < conv_n || conv_n > c->n ||
        ((uintptr_t)slab & 15))
      return -1;
    if (slab_rows_big <= 0 || slab_rows_big > slab_rows || big_lo < 0 || big_hi < big_lo || big_hi > conv_n ||
        (big_lo & 3) || (big_hi & 3))
      return -1;
    a.slab = slab;
    a.slab_rows = slab_rows;
    a.slab_rows_big = slab_rows_big;
    a.big_lo4 = big_lo >> 2;
    a.big_hi4 = big_hi >> 2;
    a.slab_stride = slab_stride;
    a.conv4 = conv_n >> 2;
    if ((a.conv4 + c->nblk - 1) / c->nblk > kThreads) return -1;  // one column per thread
  }
  return 0;
}

// p, mbuf <- SGD(p, mean over ranks of grads) -- each rank updates its shard, then all gather.
int pto_xar_allreduce_sgd(void* ctx, const float* grads, float* p, float* mbuf, float lr, float momentum,
                          float dampening, float wd, float scale, int nesterov, int first_step,
                          int* step_counter, const float* slab, int slab_rows, long slab_stride,
                          long conv_n, int slab_rows_big, long big_lo, long big_hi, long skip_lo, long skip_hi,
                          void* stream) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  XarArgs a{};
  const int rc = prep_sgd(c, a, grads, p, mbuf, lr, momentum, dampening, wd, scale, nesterov, first_step, step_counter,
                          slab, slab_rows, slab_stride, conv_n, slab_rows_big, big_lo, big_hi, skip_lo, skip_hi);
  return rc != 0 ? rc : launch(c, a, stream);
}

// The fused DDP step's exchange (round 6): as pto_xar_allreduce_sgd with the conv slab, plus the
// fully connected layers' gradients computed in phase 1 (XarArgs::fc_tiles) from dh [B][500], a2
// [B][800], dlog [B][10], h [B][500] and the loss statistics from per_sample [B][2] into stats.
// w1_off / b1_off / w2_off / b2_off: float offsets of fc1.weight, fc1.bias, fc2.weight, fc2.bias in the
// flat gradient (multiples of 4; [w1_off, n) is the fc range, nothing of it is read from grads).
int pto_xar_allreduce_sgd_fc(void* ctx, const float* grads, float* p, float* mbuf, float lr, float momentum,
                             float dampening, float wd, float scale, int nesterov, int first_step, int* step_counter,
                             const float* slab, int slab_rows, long slab_stride, long conv_n, int slab_rows_big,
                             long big_lo, long big_hi, const float* dh, const float* a2, const float* dlog,
                             const float* h, const float* per_sample, float* stats, float loss_scale, int B,
                             long w1_off, long b1_off, long w2_off, long b2_off, void* stream) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  if (slab == nullptr || dh == nullptr || a2 == nullptr || dlog == nullptr || h == nullptr || B < 1 ||
      ((w1_off | b1_off | w2_off | b2_off) & 3) || w1_off < conv_n || b1_off < w1_off + 400000 ||
      w2_off < b1_off + 500 || b2_off < w2_off + 5000 || b2_off + 12 > c->n)
    return -1;
  XarArgs a{};
  const int rc = prep_sgd(c, a, grads, p, mbuf, lr, momentum, dampening, wd, scale, nesterov, first_step, step_counter,
                          slab, slab_rows, slab_stride, conv_n, slab_rows_big, big_lo, big_hi, w1_off, c->n);
  if (rc != 0) return rc;
  a.fc_tiles = 1;
  a.fc_B = B;
  a.fc_dh = dh;
  a.fc_a2 = a2;
  a.fc_dlog = dlog;
  a.fc_h = h;
  a.fc_per_sample = per_sample;
  a.fc_stats = stats;
  a.fc_loss_scale = loss_scale;
  a.fc_w1_4 = w1_off >> 2;
  a.fc_b1_4 = b1_off >> 2;
  a.fc_w2_4 = w2_off >> 2;
  a.fc_b2_4 = b2_off >> 2;
  return launch(c, a, stream);
}

// ---- single-device emulation of `world` ranks (tests / latency floor) -------------------
// Emulated workgroup size: 256 threads while W x nblk <= 1024 (4 per CU: 4 waves of 104 VGPRs per
// SIMD), else one wave.  The fc form's 160-VGPR waves fit 3 per SIMD: 256 threads up to 768.
static int emu_threads(int world, int nblk, bool fc = false) {
  return world * nblk <= (fc ? 768 : 1024) ? kThreads : kEmuThreads;
}

struct XarEmu {
  int world, nblk;
  long n, npad;
  char* base[kMaxWorld];
  int* err;         // one word per emulated rank
  XarArgs* d_args;  // device copy of the per-rank arguments
  XarArgs h_args[kMaxWorld];  // host copy (pto_xar_emu_set_fc amends it)
  long long timeout_ticks;
  unsigned long long* stamps;
  int light_fence;
};

// alloc_kind: 0 = uncached (as the multi-process path), 1 = fine-grained, 2 = hipMalloc.
// fence: -1 = light iff uncached (as the multi-process path), 0 = system, 1 = light.
int pto_xar_emu_create(int world, long n, int nblk, double timeout_s, int alloc_kind, int fence,
                       void** ctx_out) {
  if (world < 2 || world > kMaxWorld || n <= 0 || (n & 3) || nblk < 1 || nblk > kMaxBlocks ||
      n > (1L << 32))
    return -1;
  XarEmu* e = new XarEmu{};
  e->world = world;
  e->nblk = nblk;
  e->n = n;
  e->npad = round_up(n, (long)world * nblk * 4);
  const size_t bytes = kHdrBytes + (size_t)2 * e->npad * sizeof(float);
  for (int q = 0; q < world; ++q) {
    void* p = nullptr;
    const hipError_t r = alloc_kind == 2 ? hipMalloc(&p, bytes)
                         : hipExtMallocWithFlags(&p, bytes, alloc_kind == 1 ? hipDeviceMallocFinegrained
                                                                            : hipDeviceMallocUncached);
    if (r != hipSuccess) return -2;
    if (hipMemset(p, 0, bytes) != hipSuccess) return -2;
    e->base[q] = static_cast<char*>(p);
  }
  if (hipMalloc(&e->err, kMaxWorld * sizeof(int)) != hipSuccess) return -2;
  if (hipMemset(e->err, 0, kMaxWorld * sizeof(int)) != hipSuccess) return -2;
  if (hipMalloc(&e->d_args, kMaxWorld * sizeof(XarArgs)) != hipSuccess) return -2;
  e->timeout_ticks = (long long)(timeout_s * 1e8);
  e->light_fence = fence < 0 ? alloc_kind == 0 : fence;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  *ctx_out = e;
  return 0;
}

long pto_xar_emu_npad(void* ctx) { return static_cast<XarEmu*>(ctx)->npad; }

// Phase stamps (world x nblk x 4 uint64, wall_clock64 at 100 MHz) for the next emu_set.
void pto_xar_emu_stamps(void* ctx, unsigned long long* buf) { static_cast<XarEmu*>(ctx)->stamps = buf; }

// Per-rank tensors as arrays of `world` device addresses.  mode 0: dst = out (mean);
// mode 1: dst = parameters, mbuf = momentum (SGD).  slab may be null.
int pto_xar_emu_set(void* ctx, int mode, const long long* in, const long long* dst, const long long* mbuf,
                    const long long* slab, int slab_rows, long slab_stride, long conv_n, int slab_rows_big,
                    long big_lo, long big_hi, float lr, float momentum, float dampening, float wd,
                    int nesterov, int first_step, long skip_lo, long skip_hi) {
  XarEmu* e = static_cast<XarEmu*>(ctx);
  XarArgs h[kMaxWorld];
  if (skip_lo < 0 || skip_hi < skip_lo || skip_hi > e->n || (skip_lo & 3) || (skip_hi & 3) ||
      (skip_hi > skip_lo && skip_lo < (slab != nullptr ? conv_n : 0)))
    return -1;
  for (int r = 0; r < e->world; ++r) {
    XarArgs a{};
    for (int q = 0; q < kMaxWorld; ++q) a.base[q] = q < e->world ? e->base[q] : nullptr;
    a.rank = r;
    a.world = e->world;
    a.nblk = e->nblk;
    a.mode = mode;
    a.n4 = e->n >> 2;
    a.npad4 = e->npad >> 2;
    a.shard4 = a.npad4 / e->world;
    a.chunk4 = a.shard4 / e->nblk;
    a.in = reinterpret_cast<const float*>(in[r]);
    if (mode == 0) {
      a.out = reinterpret_cast<float*>(dst[r]);
    } else {
      a.p = reinterpret_cast<float*>(dst[r]);
      a.mbuf = reinterpret_cast<float*>(mbuf[r]);
    }
    a.lr = lr;
    a.momentum = momentum;
    a.dampening = dampening;
    a.wd = wd;
    a.scale = 1.f / (float)e->world;
    a.nesterov = nesterov;
    a.first_step = first_step;
    if (slab != nullptr) {
      if (slab_rows <= 0 || (conv_n & 3) || (slab_stride & 3) || slab_stride < conv_n || conv_n > e->n)
        return -1;
      if (slab_rows_big <= 0 || slab_rows_big > slab_rows || big_lo < 0 || big_hi < big_lo || big_hi > conv_n ||
          (big_lo & 3) || (big_hi & 3))
        return -1;
      a.slab = reinterpret_cast<const float*>(slab[r]);
      a.slab_rows = slab_rows;
      a.slab_rows_big = slab_rows_big;
      a.big_lo4 = big_lo >> 2;
      a.big_hi4 = big_hi >> 2;
      a.slab_stride = slab_stride;
      a.conv4 = conv_n >> 2;
      if ((a.conv4 + e->nblk - 1) / e->nblk > emu_threads(e->world, e->nblk)) return -1;
    }
    a.skip_lo4 = skip_lo >> 2;
    a.skip_hi4 = skip_hi >> 2;
    a.err = e->err + r;
    a.timeout_ticks = e->timeout_ticks;
    a.stamps = e->stamps;
    a.light_fence = e->light_fence;
    h[r] = a;
  }
  for (int r = 0; r < e->world; ++r) e->h_args[r] = h[r];
  if (hipMemcpy(e->d_args, h, e->world * sizeof(XarArgs), hipMemcpyHostToDevice) != hipSuccess) return -2;
  return 0;
}

// The fused DDP step's exchange on top of the last pto_xar_emu_set (mode 1, skip = [w1_off, n) as
// pto_xar_allreduce_sgd_fc sets it): per emulated rank the step's activations, from which phase 1
// computes the fc gradients (XarArgs::fc_tiles).  Arrays of `world` device addresses.
int pto_xar_emu_set_fc(void* ctx, const long long* dh, const long long* a2, const long long* dlog,
                       const long long* hh, const long long* per_sample, const long long* stats, int B,
                       float loss_scale, long w1_off, long b1_off, long w2_off, long b2_off) {
  XarEmu* e = static_cast<XarEmu*>(ctx);
  if (B < 1 || ((w1_off | b1_off | w2_off | b2_off) & 3) || b1_off < w1_off + 400000 || w2_off < b1_off + 500 ||
      b2_off < w2_off + 5000 || b2_off + 12 > e->n)
    return -1;
  for (int r = 0; r < e->world; ++r) {
    XarArgs& a = e->h_args[r];
    if (a.mode != 1 || a.skip_lo4 != (w1_off >> 2) || a.skip_hi4 != (e->n >> 2) ||
        w1_off < (a.slab != nullptr ? a.conv4 * 4 : 0) ||
        (a.slab != nullptr && (a.conv4 + e->nblk - 1) / e->nblk > emu_threads(e->world, e->nblk, true)))
      return -1;
    a.fc_tiles = 1;
    a.fc_B = B;
    a.fc_dh = reinterpret_cast<const float*>(dh[r]);
    a.fc_a2 = reinterpret_cast<const float*>(a2[r]);
    a.fc_dlog = reinterpret_cast<const float*>(dlog[r]);
    a.fc_h = reinterpret_cast<const float*>(hh[r]);
    a.fc_per_sample = per_sample != nullptr ? reinterpret_cast<const float*>(per_sample[r]) : nullptr;
    a.fc_stats = stats != nullptr ? reinterpret_cast<float*>(stats[r]) : nullptr;
    a.fc_loss_scale = loss_scale;
    a.fc_w1_4 = w1_off >> 2;
    a.fc_b1_4 = b1_off >> 2;
    a.fc_w2_4 = w2_off >> 2;
    a.fc_b2_4 = b2_off >> 2;
  }
  if (hipMemcpy(e->d_args, e->h_args, e->world * sizeof(XarArgs), hipMemcpyHostToDevice) != hipSuccess) return -2;
  return 0;
}

int pto_xar_emu_threads(void* ctx) {
  XarEmu* e = static_cast<XarEmu*>(ctx);
  return emu_threads(e->world, e->nblk, e->h_args[0].fc_tiles != 0);
}

int pto_xar_emu_launch(void* ctx, void* stream) {
  XarEmu* e = static_cast<XarEmu*>(ctx);
  const bool fc = e->h_args[0].fc_tiles != 0;
  const bool wide = emu_threads(e->world, e->nblk, fc) == kThreads;
  void (*k)(const XarArgs*) = wide ? (fc ? xar_kernel_emu<kThreads, true> : xar_kernel_emu<kThreads, false>)
                                   : (fc ? xar_kernel_emu<kEmuThreads, true> : xar_kernel_emu<kEmuThreads, false>);
  hipLaunchKernelGGL(k, dim3(e->nblk, e->world), dim3(wide ? kThreads : kEmuThreads), 0, (hipStream_t)stream,
                     e->d_args);
  return (int)hipGetLastError();
}

// The emulated producer push of the configured skip range (call before pto_xar_emu_launch).
int pto_xar_emu_prepush(void* ctx, void* stream) {
  XarEmu* e = static_cast<XarEmu*>(ctx);
  hipLaunchKernelGGL(xar_emu_prepush, dim3(e->nblk, e->world), dim3(kThreads), 0, (hipStream_t)stream, e->d_args);
  return (int)hipGetLastError();
}

int pto_xar_emu_error(void* ctx) {
  XarEmu* e = static_cast<XarEmu*>(ctx);
  int v[kMaxWorld] = {};
  if (hipMemcpy(v, e->err, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -2;
  int acc = 0;
  for (int q = 0; q < e->world; ++q) acc |= v[q];
  return acc;
}

int pto_xar_emu_destroy(void* ctx) {
  XarEmu* e = static_cast<XarEmu*>(ctx);
  (void)hipDeviceSynchronize();
  for (int q = 0; q < e->world; ++q) (void)hipFree(e->base[q]);
  (void)hipFree(e->err);
  (void)hipFree(e->d_args);
  delete e;
  return 0;
}

int pto_xar_destroy(void* ctx) {
  XarCtx* c = static_cast<XarCtx*>(ctx);
  (void)hipDeviceSynchronize();
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank || c->base[q] == nullptr) continue;
    (void)hipIpcCloseMemHandle(c->base[q]);
  }
  (void)hipFree(c->base[c->rank]);
  (void)hipFree(c->err);
  delete c;
  return 0;
}

}  // extern "C"
