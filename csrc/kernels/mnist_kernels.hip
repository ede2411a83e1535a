// Hand-written CDNA4 (gfx950) kernels for the MNIST DDP training step of the
// reference workload (jiaqianjing/pytorch-operator examples/mnist/mnist.py:17-43):
//
//   conv1(1->20,k5) -> ReLU -> maxpool2 -> conv2(20->50,k5) -> ReLU -> maxpool2
//   -> fc1(800->500) -> ReLU -> fc2(500->10) -> log_softmax -> nll_loss(mean)
//
// The single-GPU training step is 5 launches (round 5).  World size > 1 (round 6) keeps the first
// four: over xGMI the exchange of xgmi_allreduce.hip replaces the tail and computes the fc
// gradient tiles itself (mnist_fc_grads.h, shared with the tail), over RCCL the tail runs
// gradient-only (pto_mnist_tail_grads) before ONE all-reduce and the SGD launch; the round-5
// forms (head + fc1_bwd, 6 launches) stay as start-up race candidates.  At B=64
// the step is ~0.84 GFLOP: it is latency-bound, so every kernel is shaped to (a) issue all of its
// global loads up front (no load -> use -> load chains, no predicated loads, at most the 63 loads
// vmcnt can track), (b) keep its MFMA chains short by splitting K across the waves of a workgroup,
// (c) keep the launch count low, and (d) keep bulk stores off the critical waves and out of the
// kernel's last moments (docs/kernels.md has the measured design log):
//
//   AB conv12_fwd      uint8 batch (staged by the previous step) + Normalize; conv1 channels 0-15
//                      on MFMA with the 2x2 pool in the accumulator registers, 16-19 as 4x4x1 MFMA
//                      chains; bias + ReLU + pool (argmax) into an LDS im2col image; conv2 as an
//                      implicit GEMM on v_mfma_f32_16x16x4_f32, bias + ReLU + pool in the epilogue;
//                      a1 / idx1 published per channel group by the waves conv2's epilogue idles
//   C  fc1_fwd<2>      split-K MFMA GEMM (256 workgroups), pre-activation halves (bias in the first)
//   E' fc1_bwd_head    per (16-sample, 16-feature) tile: the head recomputed on MFMA (h, logits,
//                      DPP log-softmax / NLL, d(logits), dh on 4x4x1 chains), then d(a2) =
//                      relu'(a2) . (dh W1) written pooled; next-batch staging blocks
//   F' conv_bwd4       per (4-sample chunk, 5-channel group): d(a2) un-pooled in LDS, dcol = W2^T
//                      dz2 (MFMA) -> col2im + ReLU mask (dz1 kept pooled) -> dW_conv1 through idx1
//                      on waves 0-7, dW_conv2 over the chunk (MFMA + VALU rows) on waves 8-15
//   G  slab_reduce_sgd the tail: dW_fc1 / db_fc1 and dW_fc2 / db_fc2 tiles (MFMA) with SGD from the
//                      accumulators, the deterministic conv-slab reduction + SGD(momentum), stats
// (D head + E fc1_bwd: the world > 1 / fallback form of E'; A conv1_fwd_pool, B conv2_fwd_pool,
// conv_bwd (per-sample slab rows), sgd_momentum: the unfused / eval / fallback building blocks.)
//
// All arithmetic is fp32 (the reference's dtype); matrix work uses the exact-fp32
// MFMA (one rounding per product, same as an fmaf chain).
//
// Every kernel takes an optional `dbg` pointer: when non-null, thread 0 of each
// block records wall_clock64() (100 MHz) at phase boundaries into
// dbg[block * 16 + phase] (tools/phase_profile.py, tools/step_timeline.py; null in
// production).  Each launch gets its own slot of the debug buffer (dbg_next()).
//
// Variants measured slower and removed from this file (round-3 A/B records in
// profiles/r3_*; source at commit f6f36d4): the 5-launch schedule (fc1_bwd_head, fc tiles in
// conv_bwd's idle waves, tail_sgd), fc SGD fused into fc1_bwd, fc SGD deferred into the next
// conv12, fc1 split-K 5, nontemporal hand-off stores, shuffle-butterfly head sums.
#include <atomic>

#include "pto_common.h"
#include "mnist_fc_grads.h"

using namespace pto;

// fc1 split-K factor of the training path: 256 workgroups of 5 waves (K = 800 = 2 x 400)
constexpr int FC1_KS = 2;


namespace {

typedef unsigned long long u64;

// diagnostic builds only (-DPTO_MNIST_STAMPW): a stamp from the thread `who` of the block
__device__ __forceinline__ void stamp_by(u64* dbg, int phase, int who) {
#ifdef PTO_MNIST_STAMPW
  if (dbg != nullptr && (int)threadIdx.x == who) {
    const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    dbg[blk * 16 + phase] = (u64)wall_clock64();
  }
#else
  (void)dbg; (void)phase; (void)who;
#endif
}
__device__ __forceinline__ void stamp(u64* dbg, int phase, int thread = 0) {
  if (dbg != nullptr && (int)threadIdx.x == thread) {
    const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    dbg[blk * 16 + phase] = (u64)wall_clock64();
    dbg[blk * 16 + 8 + phase] = (u64)clock64();  // shader clock -> effective GHz per phase
  }
}

// ---------------------------------------------------------------------------
// A: conv1 forward (+bias, ReLU, 2x2 max-pool with argmax).  One thread per
// pooled output (B*20*144 threads); a 256-thread block spans at most two
// samples, whose normalised images are staged in LDS.  The block that owns a
// sample's first output also publishes xn[b] (normalised image) and lab[b].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv1_fwd_pool_kernel(
    BatchSrc src, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ a1, uint8_t* __restrict__ idx1, int B,
    float* __restrict__ zero_ptr, int zero_n, float* __restrict__ xn_out,
    int* __restrict__ lab_out, u64* dbg) {
  __shared__ float img[2][784];
  __shared__ float ws[500];
  __shared__ float bs[20];
  const int tid = threadIdx.x;
  stamp(dbg, 0);
  const int item0 = blockIdx.x * 256;
  const int total = B * 2880;
  const int b0 = item0 / 2880;
  const int b1 = min((item0 + 255) / 2880, B - 1);
  const int nb = b1 - b0 + 1;
  const int row0 = batch_row(src, b0, B);
  const int row1 = batch_row(src, b1, B);
  if (zero_ptr != nullptr) {
    for (int i = blockIdx.x * 256 + tid; i < zero_n; i += gridDim.x * 256) zero_ptr[i] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int e = tid + k * 256;
    if (e < nb * 784) {
      const int s = e >= 784 ? 1 : 0;
      const int p = e - s * 784;
      const float v = load_px(src, s ? row1 : row0, p);
      img[s][p] = v;
      const int bb = b0 + s;
      if (xn_out != nullptr && bb * 2880 >= item0) xn_out[(size_t)bb * 784 + p] = v;
    }
  }
  if (lab_out != nullptr && src.labels != nullptr && tid < nb) {
    const int bb = b0 + tid;
    if (bb * 2880 >= item0) lab_out[bb] = src.labels[tid ? row1 : row0];
  }
  for (int e = tid; e < 500; e += 256) ws[e] = w[e];
  if (tid < 20) bs[tid] = bias[tid];
  __syncthreads();
  stamp(dbg, 1);

  const int item = item0 + tid;
  if (item >= total) return;
  const int b = item / 2880;
  const int rem = item - b * 2880;
  const int c = rem / 144;
  const int p = rem - c * 144;
  const int ph = p / 12, pw = p - ph * 12;
  const float* im = &img[b - b0][(2 * ph) * 28 + 2 * pw];
  float patch[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int q = 0; q < 6; ++q) patch[r][q] = im[r * 28 + q];
  const float* wc = ws + c * 25;
  float o00 = 0.f, o01 = 0.f, o10 = 0.f, o11 = 0.f;
#pragma unroll
  for (int kh = 0; kh < 5; ++kh)
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
      const float wv = wc[kh * 5 + kw];
      o00 = fmaf(patch[kh][kw], wv, o00);
      o01 = fmaf(patch[kh][kw + 1], wv, o01);
      o10 = fmaf(patch[kh + 1][kw], wv, o10);
      o11 = fmaf(patch[kh + 1][kw + 1], wv, o11);
    }
  const float bc = bs[c];
  o00 += bc; o01 += bc; o10 += bc; o11 += bc;
  // torch max_pool2d scans (0,0),(0,1),(1,0),(1,1) and keeps the first maximum.
  float m = o00; int am = 0;
  if (o01 > m) { m = o01; am = 1; }
  if (o10 > m) { m = o10; am = 2; }
  if (o11 > m) { m = o11; am = 3; }
  a1[item] = fmaxf(m, 0.f);
  idx1[item] = (uint8_t)am;
}

// ---------------------------------------------------------------------------
// B: conv2 forward as an implicit GEMM on fp32 MFMA.
//   grid = (4 output-channel groups of 16, B samples), 8 waves per block.
//   wave w: position tile pt = w & 3 (conv rows {2pt, 2pt+1} x 8 cols = 16
//   positions, M) x 16 channels (N); K half kh2 = w >> 2 walks (cj,kh) pairs
//   [0,13) or [13,25) x 5 kw = 65 / 60 MFMA steps.  Lane group g = lane>>4 owns
//   input channels {g, g+4, .., g+16}, so every LDS offset of the unrolled loop
//   is a compile-time immediate.  LDS strides give conflict-free ds_read_b32:
//     image: row stride 16, channel stride 200 (== 8 mod 32)
//     weights: row stride 514 (== 2 mod 32, lane groups differ by 25 -> odd banks)
//   The two K halves meet in LDS; the 2x2 pool window = 2 registers of this
//   lane x 2 registers of lane^32.
// ---------------------------------------------------------------------------
// wave_allsum_dpp / sum_lane_rows: mnist_fc_grads.h

// Value of lane l + 32 for lanes l < 32 (v_permlane32_swap: one VALU op; __shfl_xor(v, 32)
// lowers to an LDS ds_bpermute round trip).  Lanes >= 32 get an unspecified value.
__device__ __forceinline__ float from_upper_half(float v) {
  return __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false)[1]);
}
__device__ __forceinline__ int from_upper_half(int v) {
  return (int)__builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false)[1];
}

struct SgdHyper {
  float lr, momentum, dampening, wd, grad_scale;
  int nesterov, first_step;
};

// torch.optim.SGD on one element (buf = momentum*buf + (1-dampening)*d, or d on the first step).
// Explicit fmas: every kernel that inlines this (the tail, sgd_momentum, xgmi_allreduce.hip's
// sgd4) rounds identically, whatever the contraction choices.
__device__ __forceinline__ void sgd_elem(float& pv, float& mv, float gv, const SgdHyper& hy) {
  float d = __builtin_fmaf(hy.wd, pv, gv * hy.grad_scale);
  if (hy.momentum != 0.f) {
    mv = hy.first_step ? d : __builtin_fmaf(hy.momentum, mv, (1.f - hy.dampening) * d);
    d = hy.nesterov ? __builtin_fmaf(hy.momentum, mv, d) : mv;
  }
  pv = __builtin_fmaf(-hy.lr, d, pv);
}

__device__ __forceinline__ void sgd4(float4& p, float4& m, const float4& g, const SgdHyper& hy) {
  sgd_elem(p.x, m.x, g.x, hy);
  sgd_elem(p.y, m.y, g.y, hy);
  sgd_elem(p.z, m.z, g.z, hy);
  sgd_elem(p.w, m.w, g.w, hy);
}

constexpr int C2_RS = 16;
constexpr int C2_CS = 200;
constexpr int C2_WS = 514;
// conv2 im2col image: channel c starts at c * C2_CS + 2 (c >> 2) (round 6).  C2_CS == 8 (mod 32)
// puts the two channels of a conv2 A-operand read 8 banks apart (their 16 positions are two 8-wide
// runs 16 apart); the extra 2 (c >> 2) spreads the conv1 epilogue's 16 channels x 2 columns over 32
// distinct banks (with C2_CS alone: 4 channels per bank, 4-way store conflicts).  Model:
// tools/lds_banks_fwd.py.
constexpr int C2_IMG = 20 * C2_CS + 8;
__device__ __forceinline__ constexpr int c2_ch(int c) { return c * C2_CS + 2 * (c >> 2); }

template <int Q0, int Q1>
__device__ __forceinline__ f32x4 conv2_k_range(const float* Ab, const float* Bb) {
  f32x4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
  for (int q = Q0; q < Q1; ++q) {
    const int cj = q / 5, kh = q % 5;
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
      const float av = Ab[cj * (4 * C2_CS + 2) + kh * C2_RS + kw];  // channel 4 cj + g: c2_ch
      const float bv = Bb[cj * 100 + kh * 5 + kw];
      if (kw & 1) acc1 = mfma16x16x4(av, bv, acc1);
      else acc0 = mfma16x16x4(av, bv, acc0);
    }
  }
  return acc0 + acc1;
}

constexpr int AB_NT = 1024;  // conv forward blocks: 16 waves, 4 per SIMD keep the matrix pipe fed
// conv12's LDS image row stride: with 44 (== 12 mod 32) the conv1 MFMA operand reads (lane
// rows {r, r+1} x 8 columns, lane groups one tap apart) touch 32
// distinct banks per half-wave; the dense 28 gave 2-way conflicts (bank model: profiles/
// r2_lds_banks.md)
constexpr int AB_IRS = 44;
// conv1 weights in LDS: 20 rows of 25 taps, W1R floats apart (26 == 26 mod 32: a weight-fragment read's
// 16 channels x 2 taps on 32 distinct banks; the dense 25 gave 2-way conflicts), the 20 biases at W1B
constexpr int W1R = 26;
constexpr int W1B = 20 * W1R;
static_assert(W1R == 26, "the conv1 weight staging store computes row * W1R + tap as tid + tid / 25");

// conv2 implicit GEMM of one block: 4 position tiles x 4 K quarters (the 25
// (ci-group, kh) rows split 6/7/6/6) over 16 waves; the quarters meet in LDS in a fixed
// order (the standalone and the fused kernel produce bit-identical a2).  Returns the
// full sum in the kq == 0 waves.
__device__ __forceinline__ f32x4 conv2_block(const float* in_s, const float* w_s, f32x4 (*red)[4][64],
                                             int wv, int lane) {
  const int pt = wv & 3, kq = wv >> 2;
  const int i = lane & 15, g = lane >> 4;
  const int oh = 2 * pt + (i >> 3), ow = i & 7;
  const float* Ab = in_s + g * C2_CS + oh * C2_RS + ow;
  const float* Bb = w_s + i * C2_WS + g * 25;
  f32x4 acc;
  if (kq == 0) acc = conv2_k_range<0, 6>(Ab, Bb);
  else if (kq == 1) acc = conv2_k_range<6, 13>(Ab, Bb);
  else if (kq == 2) acc = conv2_k_range<13, 19>(Ab, Bb);
  else acc = conv2_k_range<19, 25>(Ab, Bb);
  if (kq > 0) red[kq - 1][pt][lane] = acc;
  __syncthreads();
  if (kq == 0) acc += red[0][pt][lane] + red[1][pt][lane] + red[2][pt][lane];
  return acc;
}

__global__ __launch_bounds__(AB_NT) void conv2_fwd_pool_kernel(
    const float* __restrict__ a1, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ a2, uint8_t* __restrict__ idx2, int B, u64* dbg) {
  __shared__ float in_s[C2_IMG];
  __shared__ float w_s[16 * C2_WS];
  __shared__ f32x4 red[3][4][64];
  const int cg = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  stamp(dbg, 0);
  const float* src = a1 + (size_t)b * 2880;
  // epilogue bias, loaded now so the tail after the last barrier has no memory round trip
  const int co_pre = cg * 16 + (tid & 15);
  const float bco = co_pre < 50 ? bias[co_pre] : 0.f;
#pragma unroll
  for (int k = 0; k < (2880 + AB_NT - 1) / AB_NT; ++k) {
    const int e = tid + k * AB_NT;
    if (e < 2880) {
      const int c = e / 144, p = e - c * 144;
      const int y = p / 12, x = p - y * 12;
      in_s[c2_ch(c) + y * C2_RS + x] = src[e];
    }
  }
#pragma unroll
  for (int k = 0; k < (2000 + AB_NT - 1) / AB_NT; ++k) {
    const int e = tid + k * AB_NT;
    if (e < 16 * 125) {
      const int j = e / 125, q = e - j * 125;
      const int co = cg * 16 + j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (co < 50) v = reinterpret_cast<const float4*>(w + (size_t)co * 500)[q];
      float2* d = reinterpret_cast<float2*>(w_s + j * C2_WS + q * 4);
      d[0] = make_float2(v.x, v.y);
      d[1] = make_float2(v.z, v.w);
    }
  }
  __syncthreads();
  stamp(dbg, 1);

  const int lane = tid & 63, wv = tid >> 6;
  const int pt = wv & 3, i = lane & 15, g = lane >> 4;
  f32x4 acc = conv2_block(in_s, w_s, red, wv, lane);
  stamp(dbg, 2);
  if (wv >= 4) return;
  const int co = cg * 16 + i;
  // reg r of this lane = conv position (oh = 2pt + (g>>1), ow = 4(g&1) + r)
  const float v0 = acc[0] + bco, v1 = acc[1] + bco, v2 = acc[2] + bco, v3 = acc[3] + bco;
  float mA = v0; int aA = 0;
  if (v1 > mA) { mA = v1; aA = 1; }
  float mB = v2; int aB = 0;
  if (v3 > mB) { mB = v3; aB = 1; }
  const float pA = from_upper_half(mA);
  const int paA = from_upper_half(aA);
  const float pB = from_upper_half(mB);
  const int paB = from_upper_half(aB);
  if (g < 2 && co < 50) {  // top row of the window; partner lane holds the bottom row
    if (pA > mA) { mA = pA; aA = 2 + paA; }
    if (pB > mB) { mB = pB; aB = 2 + paB; }
    const size_t o = (size_t)b * 800 + co * 16 + pt * 4 + 2 * (g & 1);  // even: one 8-B / 2-B store each
    *reinterpret_cast<float2*>(a2 + o) = make_float2(fmaxf(mA, 0.f), fmaxf(mB, 0.f));
    *reinterpret_cast<uint16_t*>(idx2 + o) = (uint16_t)(aA | (aB << 8));
  }
}

// ---------------------------------------------------------------------------
// AB: conv1 + conv2 forward fused (the training path).  grid = (4 conv2 output
//   channel groups, B samples), 16 waves.  Every block recomputes conv1 + ReLU +
//   pool for its sample on MFMA straight into the conv2 im2col image in LDS
//   (4x redundant, ~1 us, cheaper than a launch boundary + an HBM round trip);
//   block cg publishes a1/idx1 channels [5 cg, 5 cg + 5) (for the backward), cg == 0 also xn
//   and lab.
//   conv2 then runs exactly as conv2_fwd_pool_kernel.
// ---------------------------------------------------------------------------
// conv1 channels 0-15 on MFMA: position tiles t0, t0 + 16, .. (NU of them) as NU independent
// accumulator chains, then bias + ReLU + 2x2 max-pool into the conv2 im2col image (and a1/idx1
// if pub).  Tile t = pooled row py = t / 3, pooled columns 4 (t % 3) .. + 3; its 16 MFMA rows are
// those 4 pooling windows x their 4 elements (row 4 w + e, e = 2 di + dj), so a lane's four
// accumulator registers ARE one window: the pool is a max over registers (round 5: the
// rows x columns tile needed four v_permlane32_swap pairings per tile and ~2x the epilogue VALU
// work, which the conv1 phase is issue-bound on).  Same taps in the same MFMA K order per output:
// bit-identical.  Channels 16-19 would fill only a quarter of a second 16-wide channel tile:
// conv1_tiles2_group does them as 4x4x1 MFMA chains.
template <int NU, int TS = 16>
__device__ __forceinline__ void conv1_tasks(int t0, const float* img, const int (&toff)[7],
                                            const float (&bw)[7], float bc, float* in_s, uint8_t* id1_s,
                                            int i, int g) {
  f32x4 acc[NU];
  const float* ibs[NU];
  const int wi = i >> 2, e = i & 3;  // A row i: window wi, element e
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int pt1 = t0 + TS * u;
    const int py = pt1 / 3, pq = pt1 - py * 3;
    ibs[u] = img + (2 * py + (e >> 1)) * AB_IRS + 8 * pq + 2 * wi + (e & 1);
    acc[u] = zero4();
  }
  // every LDS operand read is issued before the first MFMA (the scheduler would otherwise
  // interleave them and stall each MFMA on its own read)
  float av[NU][7];
#pragma unroll
  for (int s = 0; s < 7; ++s)
#pragma unroll
    for (int u = 0; u < NU; ++u) av[u][s] = ibs[u][toff[s]];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < 7; ++s)
#pragma unroll
    for (int u = 0; u < NU; ++u) acc[u] = mfma16x16x4(av[u][s], bw[s], acc[u]);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    // lane (channel i, g): window g of tile pt1 -- pooled (py, 4 pq + g) -- elements in acc[u][0..3]
    const int pt1 = t0 + TS * u;
    const int py = pt1 / 3, px = 4 * (pt1 - py * 3) + g;
    const float o00 = acc[u][0] + bc, o01 = acc[u][1] + bc, o10 = acc[u][2] + bc, o11 = acc[u][3] + bc;
    // torch max_pool2d scans (0,0),(0,1),(1,0),(1,1) and keeps the first maximum
    float m = o00;
    int am = 0;
    if (o01 > m) { m = o01; am = 1; }
    if (o10 > m) { m = o10; am = 2; }
    if (o11 > m) { m = o11; am = 3; }
    const float v = fmaxf(m, 0.f);
    in_s[c2_ch(i) + py * C2_RS + px] = v;
    id1_s[i * 144 + py * 12 + px] = (uint8_t)am;
  }
}

// Waves 7-15: two channel 0-15 tiles (as conv1_tasks<2>) and one channel 16-19 group -- 16 pooled
// positions (two blocks of 4 rows x 2 columns, see below) on v_mfma_f32_4x4x1_16b_f32: block lane / 4 is one pooled position,
// its 4 rows the 2x2 window (row 2 di + dj), its 4 columns the channels; the 25 taps are 25 K = 1
// steps in tap order from zero, the fmaf chain of conv1_fwd_pool_kernel
// (bit-identical).  The group's dependent chain is interleaved with the tiles' MFMAs (3-4 after
// every tile k-step) so each chain's latency hides behind the others, on the matrix pipe instead
// of ~140 VALU instructions per lane.  D of the group: lane 4 b + j, register i = window element
// i of channel 16 + j.
__device__ __forceinline__ void conv1_tiles2_group(int t0, int G, const float* img, const float* w1s,
                                                   const int (&toff)[7], const float (&bw)[7], float bc,
                                                   float* in_s, uint8_t* id1_s, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int wi = i >> 2, e = i & 3;
  const float* ibs[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int pt1 = t0 + 16 * u;
    const int py = pt1 / 3, pq = pt1 - py * 3;
    ibs[u] = img + (2 * py + (e >> 1)) * AB_IRS + 8 * pq + 2 * wi + (e & 1);
  }
  const int q = lane & 3;
  // the 8 pooled positions of a half-wave: one block of 4 pooled rows x 2 columns (18 blocks = the
  // 12 x 12 positions; b = 2 G + half): their image windows then fall on 8 disjoint 4-bank runs for
  // every tap (round 6; a run of 8 consecutive positions put rows 2 py and 2 py + 1 of
  // neighbouring positions on the same banks -- 2-way conflicts on all 25 operand reads)
  const int blk_ = 2 * G + (lane >> 5), pp = (lane >> 2) & 7;
  const int ph4 = 4 * (blk_ / 6) + (pp >> 1), pw4 = 2 * (blk_ % 6) + (pp & 1);
  const float* ia = img + (2 * ph4 + (q >> 1)) * AB_IRS + 2 * pw4 + (q & 1);
  const float* wb = w1s + (16 + q) * W1R;
  float av[2][7], av4[25], bv4[25];
#pragma unroll
  for (int st = 0; st < 7; ++st)
#pragma unroll
    for (int u = 0; u < 2; ++u) av[u][st] = ibs[u][toff[st]];
#pragma unroll
  for (int k = 0; k < 25; ++k) {
    av4[k] = ia[(k / 5) * AB_IRS + k % 5];
    bv4[k] = wb[k];
  }
  const float bc4 = w1s[W1B + 16 + q];
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[2] = {zero4(), zero4()}, acc4 = zero4();
#pragma unroll
  for (int st = 0; st < 7; ++st) {
    acc[0] = mfma16x16x4(av[0][st], bw[st], acc[0]);
    acc[1] = mfma16x16x4(av[1][st], bw[st], acc[1]);
    const int k0 = st < 4 ? 4 * st : 16 + 3 * (st - 4), nk = st < 4 ? 4 : 3;  // 4 x 4 + 3 x 3 = 25
#pragma unroll
    for (int k = k0; k < k0 + nk; ++k) acc4 = __builtin_amdgcn_mfma_f32_4x4x1f32(av4[k], bv4[k], acc4, 0, 0, 0);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // the tiles' epilogue (conv1_tasks)
    const int pt1 = t0 + 16 * u;
    const int py = pt1 / 3, px = 4 * (pt1 - py * 3) + g;
    const float o00 = acc[u][0] + bc, o01 = acc[u][1] + bc, o10 = acc[u][2] + bc, o11 = acc[u][3] + bc;
    float m = o00;
    int am = 0;
    if (o01 > m) { m = o01; am = 1; }
    if (o10 > m) { m = o10; am = 2; }
    if (o11 > m) { m = o11; am = 3; }
    const float v = fmaxf(m, 0.f);
    in_s[c2_ch(i) + py * C2_RS + px] = v;
    id1_s[i * 144 + py * 12 + px] = (uint8_t)am;
  }
  {  // the group's epilogue
    const float o00 = acc4[0] + bc4, o01 = acc4[1] + bc4, o10 = acc4[2] + bc4, o11 = acc4[3] + bc4;
    float m = o00;
    int am = 0;
    if (o01 > m) { m = o01; am = 1; }
    if (o10 > m) { m = o10; am = 2; }
    if (o11 > m) { m = o11; am = 3; }
    const float v = fmaxf(m, 0.f);
    in_s[c2_ch(16 + q) + ph4 * C2_RS + pw4] = v;
    id1_s[(16 + q) * 144 + ph4 * 12 + pw4] = (uint8_t)am;
  }
}

// conv2 weight slice of output-channel group cg (16 rows of 500) from registers into LDS
__device__ __forceinline__ void conv12_store_w2(float* w_s, const float4 (&wq)[2], int cg, int tid) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = tid + k * AB_NT;
    if (e < 16 * 125) {
      const int j = e / 125, q = e - j * 125;
      float4 v = wq[k];
      if (cg * 16 + j >= 50) v = make_float4(0.f, 0.f, 0.f, 0.f);
      // lanes 8-15 of every 16 store their upper pair first: each ds_write_b64 of the 16 lanes then
      // covers 32 distinct banks (dwords 4q, 4q + 1 of lanes 0-7 and 4q + 2, 4q + 3 of lanes 8-15)
      float2* d = reinterpret_cast<float2*>(w_s + j * C2_WS + q * 4);
      const int sw = (tid >> 3) & 1;
      const float2 lo = make_float2(v.x, v.y), hi = make_float2(v.z, v.w);
      d[sw] = sw ? hi : lo;
      d[sw ^ 1] = sw ? lo : hi;
    }
  }
}

__global__ __launch_bounds__(AB_NT) void conv12_fwd_kernel(
    BatchSrc src, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w, const float* __restrict__ bias, float* __restrict__ a1,
    uint8_t* __restrict__ idx1, float* __restrict__ xn_out, int* __restrict__ lab_out,
    float* __restrict__ a2, uint8_t* __restrict__ idx2, int B, const uint8_t* __restrict__ stg_x,
    const int* __restrict__ stg_lab, const int* __restrict__ stg_tag, u64* dbg) {
  __shared__ float img[28 * AB_IRS];
  __shared__ float w1s[W1B + 20];
  __shared__ __align__(16) float in_s[C2_IMG];
  __shared__ float w_s[16 * C2_WS];
  __shared__ f32x4 red[3][4][64];
  __shared__ __align__(16) uint8_t id1_s[20 * 144];  // conv1 pool argmax (published per channel group)
  const int cg = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  stamp(dbg, 0);
  const bool pub = cg == 0;  // xn and lab
  // conv2 epilogue bias, loaded with the staging loads (no round trip after the last barrier)
  const int co_pre = cg * 16 + (tid & 15);
  const float bco = co_pre < 50 ? bias[co_pre] : 0.f;
  float4 wq[2];
  {
    // the batch: from the staging buffer the previous step's fc1_bwd filled (one load, no
    // cursor -> permutation -> pixel chain) when its tag is this step's cursor, else gathered
    float x0;
    int lab = 0;
    if (stg_x != nullptr) {
      x0 = (float)stg_x[(size_t)b * 784 + min(tid, 783)] * src.scale + src.shift;
      lab = stg_lab[b];
      if (stg_tag[0] != src.cursor[0]) {  // block-uniform
        const int row = batch_row(src, b, B);
        x0 = load_px(src, row, min(tid, 783));
        if (src.labels != nullptr) lab = src.labels[row];
      }
    } else {
      const int row = batch_row(src, b, B);
      x0 = load_px(src, row, min(tid, 783));
      if (src.labels != nullptr) lab = src.labels[row];
    }
    const float wv = w1[min(tid, 499)];
    const float bv1 = b1[min(tid, 19)];
    // conv2 weight slice of this output-channel group (measured: landing it after conv1
    // instead, with its loads in flight through conv1, was no faster -- profiles/r3_*)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = min(tid + k * AB_NT, 16 * 125 - 1);
      const int j = e / 125, q = e - j * 125;
      const int co = min(cg * 16 + j, 49);
      wq[k] = reinterpret_cast<const float4*>(w + (size_t)co * 500)[q];
    }
    if (tid < 784) img[(tid / 28) * AB_IRS + tid % 28] = x0;
    if (tid < 500) w1s[tid + tid / 25] = wv;  // (tid / 25) * W1R + tid % 25 with W1R = 26
    if (tid < 20) w1s[W1B + tid] = bv1;
    conv12_store_w2(w_s, wq, cg, tid);
    if (pub && tid < 784) {
      xn_out[(size_t)b * 784 + tid] = x0;
      if (tid == 0 && lab_out != nullptr) lab_out[b] = lab;
    }
  }
  __syncthreads();
  stamp(dbg, 1);
  // conv1 + bias + ReLU + 2x2 max-pool.  Channels 0-15: implicit GEMM on MFMA, 36
  // position tiles (4 pooling windows each, see conv1_tasks) x 7 K-steps (25 taps,
  // zero-padded to 28 through the weight fragments); wave w takes tiles w, w+16 (+ w+32
  // for w < 4): 9 tiles per SIMD.  The pool is a max over each lane's four accumulator
  // registers.  Channels 16-19: 4x4x1 MFMA chains interleaved with the tiles on waves 7-15
  // (conv1_tiles2_group; the round-4 VALU windows: profiles/r5_c1g/ab.txt).
  {
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i = lane & 15, g = lane >> 4;
    int toff[7];
    float bw[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int tap = 4 * s + g;
      const int tc = tap < 25 ? tap : 24;
      toff[s] = (tc / 5) * AB_IRS + (tc % 5);
      const float wv_ = w1s[i * W1R + tc];
      bw[s] = tap < 25 ? wv_ : 0.f;
    }
    const float bc = w1s[W1B + i];
    __builtin_amdgcn_sched_barrier(0);  // weight fragments in registers before the tasks
    if (wv >= 7) conv1_tiles2_group(wv, wv - 7, img, w1s, toff, bw, bc, in_s, id1_s, lane);
    else conv1_tasks<2>(wv, img, toff, bw, bc, in_s, id1_s, i, g);
    if (wv < 4) conv1_tasks<1>(wv + 32, img, toff, bw, bc, in_s, id1_s, i, g);
    stamp_by(dbg, 4, 0);             // wave 0: 3 MFMA tiles done
    stamp_by(dbg, 5, AB_NT - 64);    // last wave: 2 MFMA tiles + the 4x4x1 group done
    stamp_by(dbg, 7, 4 * 64);        // wave 4: 2 MFMA tiles
  }
  __syncthreads();
  stamp(dbg, 2);
  const int lane = tid & 63, wv = tid >> 6;
  const int pt = wv & 3, i = lane & 15, g = lane >> 4;
  f32x4 acc = conv2_block(in_s, w_s, red, wv, lane);
  stamp(dbg, 3);
  if (wv >= 4) {
    // a1 / idx1 for the backward, by the waves the conv2 epilogue does not need: block cg publishes
    // channels [5 cg, 5 cg + 5) (conv_bwd4's block (cg, b) reads exactly that slice) with 16-byte
    // stores from the LDS images -- instead of scattered 4- and 1-byte stores in the conv1
    // epilogues of one block per sample (round 5)
    const int e = tid - 256;
    if (e < 180) {  // 5 channels x 12 rows x 3 float4
      const int c = 5 * cg + e / 36, rem = e - (e / 36) * 36, py = rem / 3, k = rem - py * 3;
      const float2* s2 = reinterpret_cast<const float2*>(in_s + c2_ch(c) + py * C2_RS + 4 * k);  // 8-B aligned
      const float2 u0 = s2[0], u1 = s2[1];
      *reinterpret_cast<float4*>(a1 + (size_t)b * 2880 + c * 144 + py * 12 + 4 * k) = make_float4(u0.x, u0.y, u1.x, u1.y);
    } else if (e < 225) {
      reinterpret_cast<uint4*>(idx1 + (size_t)b * 2880 + 720 * cg)[e - 180] =
          reinterpret_cast<const uint4*>(id1_s + 720 * cg)[e - 180];
    }
    return;
  }
  const int co = cg * 16 + i;
  const float v0 = acc[0] + bco, v1 = acc[1] + bco, v2 = acc[2] + bco, v3 = acc[3] + bco;
  float mA = v0; int aA = 0;
  if (v1 > mA) { mA = v1; aA = 1; }
  float mB = v2; int aB = 0;
  if (v3 > mB) { mB = v3; aB = 1; }
  const float pA = from_upper_half(mA);
  const int paA = from_upper_half(aA);
  const float pB = from_upper_half(mB);
  const int paB = from_upper_half(aB);
  if (g < 2 && co < 50) {
    if (pA > mA) { mA = pA; aA = 2 + paA; }
    if (pB > mB) { mB = pB; aB = 2 + paB; }
    const size_t o = (size_t)b * 800 + co * 16 + pt * 4 + 2 * (g & 1);  // even: one 8-B / 2-B store each
    *reinterpret_cast<float2*>(a2 + o) = make_float2(fmaxf(mA, 0.f), fmaxf(mB, 0.f));
    *reinterpret_cast<uint16_t*>(idx2 + o) = (uint16_t)(aA | (aB << 8));
  }
}

// ---------------------------------------------------------------------------
// C: fc1 forward: h = relu(x[B,800] . W[500,800]^T + b).
//   grid = (32 N-tiles, ceil(B/16) M-tiles), 10 waves; wave w reduces K range
//   [80w, 80w+80); lane group g owns k = 80w + 16s + 4g + [0,4), s < 5 (5 float4
//   loads per operand, all issued before the first MFMA; the four lane groups of a
//   row read one contiguous 64 B segment per load); the ten partial tiles are summed
//   through LDS and the bias+ReLU epilogue is applied once.
// ---------------------------------------------------------------------------
// KS = 2 (training path): K split over two blocks (blockIdx.z) of 5 waves each, 256
// blocks on the 256 CUs with half the operand bytes per CU; each writes its pre-activation
// partial to h + z * B * 500, the z == 0 half with the bias added (round 6: the consumers --
// fc1_bwd_head's 216 tiles, head_kernel -- then form relu(part0 + part1) without reloading b1:
// 4 of every tile's 12 float4 staging loads), and the consumer adds the halves and the ReLU.
template <int KS>
__global__ __launch_bounds__(640 / KS) void fc1_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ h, int B, u64* dbg) {
  static_assert(KS == 1 || KS == 2, "fc1: 10 or 5 waves of 80 K each");
  constexpr int NW = 10 / KS;
  __shared__ f32x4 red[NW][64];
  const int nt = blockIdx.x, mt = blockIdx.y, kz = blockIdx.z, tid = threadIdx.x;
  stamp(dbg, 0);
  const int lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int row = mt * 16 + i, col = nt * 16 + i;
  const bool rv = row < B, cv = col < 500;
  const int k0 = (kz * NW + wv) * 80 + g * 4;
  const float4* xa = reinterpret_cast<const float4*>(x + (size_t)(rv ? row : B - 1) * 800 + k0);
  const float4* wb = reinterpret_cast<const float4*>(w + (size_t)(cv ? col : 499) * 800 + k0);
  float4 av[5], bv[5];
#pragma unroll
  for (int s = 0; s < 5; ++s) { av[s] = xa[4 * s]; bv[s] = wb[4 * s]; }
  // epilogue operands of thread tid < 256, in flight with the GEMM loads
  const int l_e = tid >> 2, r_e = tid & 3;
  const int orow = mt * 16 + (l_e >> 4) * 4 + r_e, ocol = nt * 16 + (l_e & 15);
  const float bo = (bias != nullptr && tid < 256 && ocol < 500) ? bias[ocol] : 0.f;
  f32x4 c0 = zero4(), c1 = zero4();
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const float* ae = &av[s].x;
    const float* be = &bv[s].x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = rv ? ae[e] : 0.f;
      const float bb = cv ? be[e] : 0.f;
      if (e & 1) c1 = mfma16x16x4(a, bb, c1);
      else c0 = mfma16x16x4(a, bb, c0);
    }
  }
  red[wv][lane] = c0 + c1;
  __syncthreads();
  stamp(dbg, 1);
  if (tid < 256) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += red[q][l_e][r_e];
    if (orow < B && ocol < 500) {
      if (KS == 1) h[(size_t)orow * 500 + ocol] = fmaxf(s + bo, 0.f);
      else h[((size_t)kz * B + orow) * 500 + ocol] = kz == 0 ? s + bo : s;
    }
  }
}

// ---------------------------------------------------------------------------
// D: head.  One wave per sample: logits = h.W2^T + b2, log_softmax, NLL,
// d(logits) = (softmax - onehot) * grad_scale, dh = (d(logits).W2) * (h > 0).
// All loads (label, h row, the 10x500 W2 slice this lane needs) are issued
// first.  Per-sample (loss, correct) go to per_sample[b] (reduced later by
// fc1_bwd, deterministic); eval callers may instead accumulate into `stats`
// (one atomic per block after an LDS reduction).
// WPB waves per block: the training path (B = 64) runs one wave per block so the
// 20 KB W2 stream of each sample lands on its own CU (4 waves per block put 80 KB of
// L2 traffic on each of 16 CUs); the eval path (B = 1000) keeps 4 to cut the atomics.
// ---------------------------------------------------------------------------
// With hp2 (the split-K fc1 path, the bias folded into the first partial h): h = relu(h + hp2)
// is formed here and written to h_out for the backward.
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void head_kernel(
    const float* __restrict__ h, const float* __restrict__ w2, const float* __restrict__ b2,
    const int* __restrict__ lab, int B, float grad_scale, float loss_scale,
    float* __restrict__ dlogits, float* __restrict__ dh, float* __restrict__ logp_out,
    float* __restrict__ per_sample, float* __restrict__ stats, const float* __restrict__ hp2,
    float* __restrict__ h_out, u64* dbg) {
  __shared__ float red[2][WPB];
  const int tid = threadIdx.x, lane = tid & 63, wq = tid >> 6;
  stamp(dbg, 0);
  const int b = blockIdx.x * WPB + wq;
  const bool bvalid = b < B;
  const int bc = bvalid ? b : B - 1;
  const int t = lab[bc];
  // lane owns k = 8 lane + [0, 8): two float4 per row (h, every W2 row), 22 loads per
  // lane, all in flight at once (lane 62 has half a chunk, lane 63 none)
  const int k0 = 8 * lane;
  const bool v0 = k0 < 500, v1 = k0 + 4 < 500;
  const int o0 = v0 ? k0 : 496, o1 = v1 ? k0 + 4 : 496;
  float hv[8], wv[10][8];
  {
    float4 h0 = *reinterpret_cast<const float4*>(h + (size_t)bc * 500 + o0);
    float4 h1 = *reinterpret_cast<const float4*>(h + (size_t)bc * 500 + o1);
    if (hp2 != nullptr) {
      // the second split-K fc1 partial (the first holds the bias)
      const float4 q0 = *reinterpret_cast<const float4*>(hp2 + (size_t)bc * 500 + o0);
      const float4 q1 = *reinterpret_cast<const float4*>(hp2 + (size_t)bc * 500 + o1);
      h0 = make_float4(fmaxf(h0.x + q0.x, 0.f), fmaxf(h0.y + q0.y, 0.f), fmaxf(h0.z + q0.z, 0.f),
                       fmaxf(h0.w + q0.w, 0.f));
      h1 = make_float4(fmaxf(h1.x + q1.x, 0.f), fmaxf(h1.y + q1.y, 0.f), fmaxf(h1.z + q1.z, 0.f),
                       fmaxf(h1.w + q1.w, 0.f));
      if (bvalid) {
        float4* ho = reinterpret_cast<float4*>(h_out + (size_t)b * 500);
        if (v0) ho[k0 >> 2] = h0;
        if (v1) ho[(k0 >> 2) + 1] = h1;
      }
    }
    float4 w0[10], w1v[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      w0[j] = *reinterpret_cast<const float4*>(w2 + j * 500 + o0);
      w1v[j] = *reinterpret_cast<const float4*>(w2 + j * 500 + o1);
    }
    hv[0] = v0 ? h0.x : 0.f; hv[1] = v0 ? h0.y : 0.f; hv[2] = v0 ? h0.z : 0.f; hv[3] = v0 ? h0.w : 0.f;
    hv[4] = v1 ? h1.x : 0.f; hv[5] = v1 ? h1.y : 0.f; hv[6] = v1 ? h1.z : 0.f; hv[7] = v1 ? h1.w : 0.f;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      wv[j][0] = w0[j].x; wv[j][1] = w0[j].y; wv[j][2] = w0[j].z; wv[j][3] = w0[j].w;
      wv[j][4] = w1v[j].x; wv[j][5] = w1v[j].y; wv[j][6] = w1v[j].z; wv[j][7] = w1v[j].w;
    }
  }
  float logit[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    float p = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) p = fmaf(hv[q], wv[j][q], p);
    logit[j] = p;
  }
  // DPP / permlane all-reduce: six VALU steps per sum, no LDS round trips (-0.3 to -0.5 us/step
  // against __shfl_xor butterflies, profiles/r3_mnist_ab_dpp_ks5.txt)
#pragma unroll
  for (int j = 0; j < 10; ++j) logit[j] = wave_allsum_dpp(logit[j]);
#pragma unroll
  for (int j = 0; j < 10; ++j) logit[j] += b2[j];
  float m = logit[0];
#pragma unroll
  for (int j = 1; j < 10; ++j) m = fmaxf(m, logit[j]);
  float se = 0.f;
#pragma unroll
  for (int j = 0; j < 10; ++j) se += __expf(logit[j] - m);
  const float lse = m + __logf(se);
  float lt = 0.f;
  int pred = 0;
  float best = logit[0];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    if (j == t) lt = logit[j];
    if (logit[j] > best) { best = logit[j]; pred = j; }
  }
  const float lossb = lse - lt;
  const float corr = pred == t ? 1.f : 0.f;
  if (bvalid && lane == 0 && per_sample != nullptr) {
    per_sample[2 * b] = lossb;
    per_sample[2 * b + 1] = corr;
  }
  if (stats != nullptr) {
    if (lane == 0) {
      red[0][wq] = bvalid ? lossb * loss_scale : 0.f;
      red[1][wq] = bvalid ? corr : 0.f;
    }
    __syncthreads();
    if (tid == 0) {
      float sl = 0.f, sc = 0.f;
#pragma unroll
      for (int q = 0; q < WPB; ++q) { sl += red[0][q]; sc += red[1][q]; }
      atomicAdd(&stats[0], sl);
      atomicAdd(&stats[1], sc);
    }
  }
  if (!bvalid) return;
  if (logp_out != nullptr) {
#pragma unroll
    for (int j = 0; j < 10; ++j)
      if (lane == j) logp_out[(size_t)b * 10 + j] = logit[j] - lse;
  }
  if (dh == nullptr) return;
  float dl[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) dl[j] = (__expf(logit[j] - lse) - (j == t ? 1.f : 0.f)) * grad_scale;
  if (dlogits != nullptr) {
#pragma unroll
    for (int j = 0; j < 10; ++j)
      if (lane == j) dlogits[(size_t)b * 10 + j] = dl[j];
  }
  float dv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 10; ++j) s = fmaf(dl[j], wv[j][q], s);
    dv[q] = hv[q] > 0.f ? s : 0.f;
  }
  float4* dr = reinterpret_cast<float4*>(dh + (size_t)b * 500 + k0);
  if (v0) dr[0] = make_float4(dv[0], dv[1], dv[2], dv[3]);
  if (v1) dr[1] = make_float4(dv[4], dv[5], dv[6], dv[7]);
  stamp(dbg, 1);
}

// ---------------------------------------------------------------------------
// E: fc1 backward, three independent jobs in one launch (blockDim 512 = 8 waves):
//   job 1 (200 blocks x 8 waves = 1600 tiles): dW_fc1[500,800] = dh^T . a2 (K = B,
//          64 samples per register-preloaded chunk), db_fc1 from the kt==0 tiles.
//          Written, not accumulated: no zeroing needed.
//   job 2 (ceil(B/16)*50 blocks): da2[B,800] = dh . W_fc1 (K = 500 split over 8
//          waves, 16 steps = 32 loads per lane: within the 63 outstanding loads vmcnt
//          can track, so every load is in flight at once; LDS reduce); the epilogue
//          un-pools through idx2 and applies the ReLU mask, writing dz2[B,50,8,8].
//          This job is the critical path into the conv backward.
//   job 3 (4 blocks): dW_fc2[10,500] = dlogits^T . h (MFMA, K = B), db_fc2, and
//          the step's loss statistics from the head's per-sample values.
// ---------------------------------------------------------------------------
constexpr int E_NT = 512;
constexpr int E_NW = E_NT / 64;
constexpr int E_NJ1 = 1600 / E_NW;  // job-1 blocks
constexpr int E_NJ3 = 32 / E_NW;    // job-3 blocks

// Row of sample b of the batch taken at step `step` (perm required).
__device__ __forceinline__ int batch_row_at(const BatchSrc& s, long long step, int b, int B) {
  long long i = (step * B) % s.n_total + b;
  if (i >= s.n_total) i -= s.n_total;
  return s.perm[i];
}

// DDP over xGMI (parallel/xgmi.py): fc1_bwd pushes each dW_fc1 tile straight into the receive
// buffer of the rank that owns it (xgmi_allreduce.hip layout: recv[sender][shard] behind a 64 KB
// header, element v of the flat gradient owned by rank v / shard4), so the exchange kernel's
// phase 1 no longer re-reads and re-sends 93.9 % of the gradient bytes.  Write-through system-
// scope stores (visible over the fabric whatever the IPC mapping's cache type), drained by every
// pushing wave before it ends; the exchange raises its flags in a later launch of this stream.
// Write-after-read invariant the push relies on: the owner reduces its receive slot in the
// exchange launch of step t and this launch (step t + 1) overwrites it; that is safe only because
// the step-t exchange waited for every owner's flag2 before it ended, i.e. every owner finished
// reading.  After a timed-out wait (the exchange's error word is set) that no longer holds, so a
// degraded rank stops pushing (err != 0): its replicas have diverged and the worker exits 138.
struct XPush {
  char* base[8];  // every rank's exchange buffer (IPC-mapped); null: no push
  int rank, world;
  long shard4;    // float4s per owner shard
  long w1_f4;     // flat float4 index of fc1.weight's first element
  const int* err; // the exchange's error word (pto_xar_err_ptr); nullable
};
constexpr long kXarHdrBytes = 64 * 1024;  // xgmi_allreduce.hip kHdrBytes

__device__ __forceinline__ void push_wt4(char* dst, float4 v) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v x = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(dst), "v"(x) : "memory");
}

struct Fc1Bwd {
  XPush xp;
  const float *dh, *a2;
  const uint8_t* idx2;
  const float *w1, *dlog, *h;
  float *gw1, *gb1, *gw2, *gb2, *dz2;
  float* dpool;  // non-null: the dz2 job writes d(a2) pooled [B][800] here instead of dense dz2
  const float* per_sample;
  float* stats;
  float loss_scale;
  int jobs, B;
  // next-batch staging (stage_x != null): ceil(B/4) extra blocks copy the uint8 pixels and
  // labels of the batch of step cursor + stage_adv into stage_x / stage_lab and write that
  // step number to stage_tag (conv12_fwd uses the staged batch when its tag matches)
  BatchSrc nsrc;
  int stage_adv;
  uint8_t* stage_x;
  int* stage_lab;
  int* stage_tag;
};

__global__ __launch_bounds__(E_NT) void fc1_bwd_kernel(Fc1Bwd a, u64* dbg) {
  __shared__ f32x4 red[E_NW][64];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int B = a.B;
  // jobs bit0: dW_fc1/db_fc1, bit1: dz2, bit2: dW_fc2/db_fc2/stats.  Block ids are
  // laid out job1 | job2 | job3 | staging with absent jobs taking no blocks.
  const int nJ1 = (a.jobs & 1) ? E_NJ1 : 0;
  const int nJ2 = (a.jobs & 2) ? ((B + 15) / 16) * 50 : 0;
  const int nJ3 = (a.jobs & 4) ? E_NJ3 : 0;
  int blk = blockIdx.x;
  stamp(dbg, 0);
  // Block layout (round-4 A/B, profiles/r4_fb_ab.txt: -0.8 us per step): physical ids
  // [0, nJ2) run the dz2 job -- the launch's critical path into the conv backward -- so it is
  // dispatched first onto idle CUs, ordered so the four sample tiles of one feature tile share an
  // XCD (round-robin placement: blocks b and b + 8 share one) and read that W1 column slab into
  // one L2; then [nJ2, nJ2 + nJ1) dW_fc1, then fc2 + staging
  if (blk < nJ2) {
    int t2x = blk;  // dz2 tile mt * 50 + kt
    if (nJ2 == 200) {
      const int s = (blk & 7) * 25 + (blk >> 3);  // blocks grouped by XCD: 25 per XCD
      t2x = (s & 3) * 50 + (s >> 2);              // 4 consecutive slots = the 4 mt of one kt
    }
    blk = nJ1 + t2x;
  } else if (blk < nJ2 + nJ1) {
    blk -= nJ2;
  }
  if (blk < nJ1) {
    const int tile = blk * E_NW + wv;
    const int nt = tile / 50, kt = tile - nt * 50;
    const int n = nt * 16 + i, f = kt * 16 + i;
    const bool nv = n < 500;
    const int nc = nv ? n : 499;
    f32x4 c0 = zero4(), c1 = zero4();
    float dbsum = 0.f;
    for (int base = 0; base < B; base += 64) {
      float av[16], fv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int bb = min(base + 4 * s + g, B - 1);
        av[s] = a.dh[(size_t)bb * 500 + nc];
        fv[s] = a.a2[(size_t)bb * 800 + f];
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
    const f32x4 c = c0 + c1;
    // DDP over xGMI: push unless the exchange has flagged an error (wave-uniform)
    const bool push = a.xp.base[0] != nullptr &&
                      (a.xp.err == nullptr || __hip_atomic_load(a.xp.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0);
    if (nv) {
      const unsigned e4 = (unsigned)(n * 200 + kt * 4 + g);  // float4 index of (n, 16 kt + 4 g)
      const float4 v4 = make_float4(c[0], c[1], c[2], c[3]);
      reinterpret_cast<float4*>(a.gw1)[e4] = v4;
      if (push) {  // also straight to the owner's receive buffer
        const long v = a.xp.w1_f4 + (long)e4;
        const int q = (int)(v / a.xp.shard4);
        char* b = a.xp.base[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) b = q == k ? a.xp.base[k] : b;
        push_wt4(b + kXarHdrBytes + (((long)a.xp.rank * a.xp.shard4 + (v - (long)q * a.xp.shard4)) << 4), v4);
      }
    }
    if (push) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (kt == 0) {
      dbsum = sum_lane_rows(dbsum);
      if (g == 0 && nv) a.gb1[n] = dbsum;
    }
  } else if (blk < nJ1 + nJ2) {
    const int t2 = blk - nJ1;
    const int mt = t2 / 50, kt = t2 - mt * 50;
    const int row = mt * 16 + i;
    const bool rv = row < B;
    const int rc = rv ? row : B - 1;
    const int f = kt * 16 + i;
    // K order: step s of wave wv, lane group g covers k = 64 wv + 16 g + s, so a lane's
    // 16 dh values are contiguous (4 float4 loads); k >= 500 (wave 7, g = 3, s >= 4) is 0
    const int kb = 64 * wv + 16 * g;
    float av[16], bv[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kq = kb + 4 * q;
      const float4 d4 = *reinterpret_cast<const float4*>(a.dh + (size_t)rc * 500 + min(kq, 496));
      const bool ok = rv && kq < 500;
      av[4 * q] = ok ? d4.x : 0.f;
      av[4 * q + 1] = ok ? d4.y : 0.f;
      av[4 * q + 2] = ok ? d4.z : 0.f;
      av[4 * q + 3] = ok ? d4.w : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) bv[s] = a.w1[(size_t)min(kb + s, 499) * 800 + f];
    // epilogue operands of threads tid < 256 (ReLU mask + pool argmax), in flight with
    // the GEMM loads
    const int l = (tid & 255) >> 2, r = tid & 3;
    const int bs = mt * 16 + (l >> 4) * 4 + r;
    const int ff = kt * 16 + (l & 15);
    const size_t o = (size_t)min(bs, B - 1) * 800 + ff;
    float a2o = a.a2[o];
    int p = a.idx2[o];
    f32x4 c0 = zero4(), c1 = zero4();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s & 1) c1 = mfma16x16x4(av[s], bv[s], c1);
      else c0 = mfma16x16x4(av[s], bv[s], c0);
    }
    asm volatile("" : "+v"(a2o), "+v"(p));  // keep the epilogue loads above the barrier
    red[wv][lane] = c0 + c1;
    __syncthreads();
    float v = red[0][l][r];
#pragma unroll
    for (int q = 1; q < E_NW; ++q) v += red[q][l][r];
    if (tid < 256 && bs < B) {
      const float d = a2o > 0.f ? v : 0.f;
      if (a.dpool != nullptr) {
        a.dpool[(size_t)bs * 800 + ff] = d;
      } else {
        const int co = ff >> 4, ph = (ff >> 2) & 3, pw = ff & 3;
        float* z = a.dz2 + (size_t)bs * 3200 + co * 64 + (2 * ph) * 8 + 2 * pw;
        z[0] = p == 0 ? d : 0.f;
        z[1] = p == 1 ? d : 0.f;
        z[8] = p == 2 ? d : 0.f;
        z[9] = p == 3 ? d : 0.f;
      }
    }
  } else if (blk < nJ1 + nJ2 + nJ3) {
    // dW_fc2[10,500] = dlogits^T . h : M = 10 (16), N = 500 (32 tiles), K = B
    const int nt = (blk - nJ1 - nJ2) * E_NW + wv;  // 0..31
    const int jc = min(i, 9);
    const int n = nt * 16 + i;
    const int ncl = min(n, 499);
    // loss statistics (wave nt == 1): the first 64 samples' values, in flight with the GEMM loads
    const bool do_stats = nt == 1 && a.per_sample != nullptr && a.stats != nullptr;
    float ls = 0.f, cs = 0.f;
    if (do_stats && lane < B) { ls = a.per_sample[2 * lane]; cs = a.per_sample[2 * lane + 1]; }
    f32x4 c0 = zero4(), c1 = zero4();
    float dbsum = 0.f;
    for (int base = 0; base < B; base += 64) {
      float av[16], hv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int bb = min(base + 4 * s + g, B - 1);
        av[s] = a.dlog[(size_t)bb * 10 + jc];
        hv[s] = a.h[(size_t)bb * 500 + ncl];
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
    const f32x4 c = c0 + c1;
    if (n < 500) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = g * 4 + r;
        if (j < 10) a.gw2[j * 500 + n] = c[r];
      }
    }
    if (nt == 0) {
      dbsum = sum_lane_rows(dbsum);
      if (g == 0 && i < 10) a.gb2[i] = dbsum;
    }
    if (do_stats) {
      for (int bb = lane + 64; bb < B; bb += 64) { ls += a.per_sample[2 * bb]; cs += a.per_sample[2 * bb + 1]; }
      ls = wave_allsum_dpp(ls);
      cs = wave_allsum_dpp(cs);
      if (lane == 0) { a.stats[0] = ls * a.loss_scale; a.stats[1] = cs; }
    }
  } else {
    // next-batch staging: samples 4 j4 .. 4 j4 + 3, 49 x 16 B of pixels each
    const int j4 = blk - nJ1 - nJ2 - nJ3;
    const long long step = (long long)a.nsrc.cursor[0] + a.stage_adv;
    if (tid < 196) {
      const int s = tid / 49, c = tid - s * 49, smp = 4 * j4 + s;
      if (smp < B) {
        const int row = batch_row_at(a.nsrc, step, smp, B);
        const uint4 v = reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(a.nsrc.x) + (size_t)row * 784)[c];
        reinterpret_cast<uint4*>(a.stage_x + (size_t)smp * 784)[c] = v;
        if (c == 0) a.stage_lab[smp] = a.nsrc.labels[row];
      }
    }
    if (j4 == 0 && tid == 0) a.stage_tag[0] = (int)step;
  }
  stamp(dbg, 1);
}

// ---------------------------------------------------------------------------
// E': fc1 backward with the head fused in (the world-1 step, round 5).  Replaces the head launch
// and its kernel boundary.  Every dz2 block (mt, kt) of fc1_bwd's layout recomputes the head of
// its 16 samples on MFMA, then runs the dz2 job on that dh:
//   h  = relu(p0 + p1)                           (the split-K fc1 partials, p0 with the bias; into LDS)
//   logits = h . W2^T + b2                       (M 16 samples, N 16 (10), K 512 over 8 waves)
//   log-softmax, NLL, d(logits) = (softmax - onehot) / B        (one thread per sample)
//   dh = (d(logits) . W2) * (h > 0)             (M 16, N 512, K 16; each wave its own 64 k)
//   dz2 = un-pool(relu'(a2) * (dh . W1))         (fc1_bwd's job 2, unchanged)
// The 50 kt blocks of a sample tile recompute the same head -- a few MFMAs next to the dz2 GEMM,
// against a launch + boundary -- and the kt == 0 block publishes h, d(logits) and the
// per-sample (loss, correct), the kt = 1..8 blocks one wave's dh columns each, for the tail
// (dW_fc1, dW_fc2, statistics).  Sums differ from
// head_kernel's lane-tree order by fp32 rounding (the DDP paths keep head + fc1_bwd).
struct Fc1BwdHead {
  const float *hp0, *hp1;       // fc1 split-K partials [B][500] x 2 (hp0 includes fc1.bias)
  const float *w2, *b2;         // fc2.weight [10][500], fc2.bias [10]
  const int* lab;               // [B]
  const float* a2;              // [B][800]
  const uint8_t* idx2;          // [B][800]
  const float* w1;              // fc1.weight [500][800]
  float* dz2;                   // [B][50][8][8] (dense), or
  float* dpool;                 // [B][800] pooled d(a2) (conv_bwd4 un-pools it through idx2)
  float *h_out, *dh_out, *dlog_out, *per_sample;  // published by the kt == 0 (dh: 1..8) blocks
  float grad_scale;             // 1 / B
  int B;
  BatchSrc nsrc;                // next-batch staging (stage_x != null), as fc1_bwd
  int stage_adv;
  uint8_t* stage_x;
  int* stage_lab;
  int* stage_tag;
};
// LDS layouts (round 6; bank model and the round-5 layouts' conflicts: tools/lds_banks_fwd.py):
//   hs / w2s  row r at r * H_RS, column c stored at c ^ (2 [r >= 8]).  H_RS == 4 (mod 32) puts rows
//             4 apart 16 banks apart (the ReLU-mask reads: 4 sample rows x 16 columns per half-wave)
//             and the XOR moves rows 8-15 two banks over (the logits operand reads: 16 rows x 2
//             adjacent columns); 16-byte rows: one ds_write_b128 per staged float4 (the XOR swaps its
//             halves).  Round 5 (514, no XOR): 2-way on the mask reads and the float2 stores.
//   dhs       row r at r * H_DS (16-byte rows).  The dz2 job's ds_read_b128 (lanes (i, g): row i,
//             chunks 16 wv + 4 g + q) stay 2-way (16 cycles per wave): no plain stride or row order
//             avoids it.  Measured and rejected (profiles/r6_banks/ab.md): the 16-byte chunk XOR the
//             row (conflict-free; per-lane address VALU on the 16 dh stores, +0.34 us in the phase)
//             and K chunks 64 columns apart per wave (conflict-free; +26 LDS instructions per wave
//             from lost read2/offset folding, +0.1 us).
constexpr int H_RS = 516;
constexpr int H_DS = 516;
__device__ __forceinline__ int hsx(int row, int col) { return row * H_RS + (col ^ ((row >> 3) << 1)); }
__device__ __forceinline__ int dsx(int row, int col) { return row * H_DS + col; }
// float4 entry of staging pass q (0-3) for thread tid: rows 0-7 in passes 0-1, rows 8-15 in 2-3
__device__ __forceinline__ int stage_e(int q, int tid) { return q < 2 ? tid + q * E_NT : 1000 + tid + (q - 2) * E_NT; }

__global__ __launch_bounds__(E_NT) void fc1_bwd_head_kernel(Fc1BwdHead a, u64* dbg) {
  __shared__ __align__(16) float hs[16 * H_RS];
  __shared__ __align__(16) float w2s[16 * H_RS];
  __shared__ __align__(16) float dhs[16 * H_DS];
  __shared__ f32x4 red[E_NW][64];
  __shared__ float dls[16][17];  // +1: the dh operand reads (8 sample rows per half-wave) hit 8 banks
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int B = a.B;
  const int nmt = (B + 15) / 16;
  const int nJ2 = nmt * 50;
  stamp(dbg, 0);
  if ((int)blockIdx.x >= nJ2) {  // next-batch staging (fc1_bwd's staging blocks)
    const int j4 = blockIdx.x - nJ2;
    const long long step = (long long)a.nsrc.cursor[0] + a.stage_adv;
    if (tid < 196) {
      const int s = tid / 49, c = tid - s * 49, smp = 4 * j4 + s;
      if (smp < B) {
        const int row = batch_row_at(a.nsrc, step, smp, B);
        const uint4 v = reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(a.nsrc.x) + (size_t)row * 784)[c];
        reinterpret_cast<uint4*>(a.stage_x + (size_t)smp * 784)[c] = v;
        if (c == 0) a.stage_lab[smp] = a.nsrc.labels[row];
      }
    }
    if (j4 == 0 && tid == 0) a.stage_tag[0] = (int)step;
    stamp(dbg, 1);
    return;
  }
  int t2x = blockIdx.x;  // dz2 tile mt * 50 + kt; grouped by XCD as fc1_bwd (4 mt of one kt together)
  if (nJ2 == 200) {
    const int s = (t2x & 7) * 25 + (t2x >> 3);
    t2x = (s & 3) * 50 + (s >> 2);
  }
  const int mt = t2x / 50, kt = t2x - mt * 50;
  const bool pub = kt == 0;

  // ---- loads, all issued before the first use: the 16 rows' fc1 partials and bias, W2, the W1
  // column slice of the dz2 job, its epilogue operands, labels and b2
  // staged float4 entries e of the 16 h rows / 10 W2 rows (125 per row): passes 0-1 take rows 0-7
  // (e < 1000), passes 2-3 rows 8-15, so hsx's swap of the float4 halves in rows 8-15 is a
  // compile-time choice per pass (no per-lane select)
  float4 hq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = min(stage_e(q, tid), 1999), row = e / 125, c4 = e - row * 125;
    const size_t o = (size_t)min(mt * 16 + row, B - 1) * 500 + 4 * c4;
    const float4 x0 = *reinterpret_cast<const float4*>(a.hp0 + o);
    const float4 x1 = *reinterpret_cast<const float4*>(a.hp1 + o);
    // head_kernel's h: relu(part0 + part1), the bias folded into part0 by fc1_fwd
    hq[q] = make_float4(fmaxf(x0.x + x1.x, 0.f), fmaxf(x0.y + x1.y, 0.f), fmaxf(x0.z + x1.z, 0.f),
                        fmaxf(x0.w + x1.w, 0.f));
  }
  float4 wq[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) wq[q] = reinterpret_cast<const float4*>(a.w2)[min(stage_e(q, tid), 1249)];
  const int kb = 64 * wv + 16 * g;  // the dz2 job's K range of this lane
  float bv[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) bv[s] = a.w1[(size_t)min(kb + s, 499) * 800 + kt * 16 + i];
  const int l_e = (tid & 255) >> 2, r_e = tid & 3;
  const int bs = mt * 16 + (l_e >> 4) * 4 + r_e;
  const int ff = kt * 16 + (l_e & 15);
  const size_t oe = (size_t)min(bs, B - 1) * 800 + ff;
  float a2o = a.a2[oe];
  int pidx = a.idx2[oe];
  // softmax lanes (waves 0-3): sample 4 wv + (lane >> 4), class lane & 15
  const int sm_s = 4 * wv + (lane >> 4), sm_j = lane & 15;
  int lab_t = 0;
  float b2v = 0.f;
  if (tid < 256) {
    lab_t = a.lab[min(mt * 16 + sm_s, B - 1)];
    b2v = a.b2[min(sm_j, 9)];
  }
  // ---- h and W2 into LDS (zero rows / columns pad K to 512 and N to 16)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = stage_e(q, tid);
    if (e < (q < 2 ? 1000 : 2000)) {
      const int row = e / 125, c4 = e - row * 125;
      const bool rv = mt * 16 + row < B;
      const float4 h4 = rv ? hq[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(hs + row * H_RS + 4 * c4) =
          q >= 2 ? make_float4(h4.z, h4.w, h4.x, h4.y) : h4;  // hsx: columns ^ 2 in rows 8-15
      if (pub && rv) reinterpret_cast<float4*>(a.h_out + (size_t)(mt * 16 + row) * 500)[c4] = h4;
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int e = stage_e(q, tid);
    if (e < (q < 2 ? 1000 : 1250)) {
      const int row = e / 125, c4 = e - row * 125;
      const float4 w4 = wq[q];
      *reinterpret_cast<float4*>(w2s + row * H_RS + 4 * c4) =
          q >= 2 ? make_float4(w4.z, w4.w, w4.x, w4.y) : w4;
    }
  }
  for (int e = tid; e < 16 * 12; e += E_NT) {  // columns 500..511 of every row (a set closed under the XOR)
    const int row = e / 12, c = 500 + e % 12;
    hs[row * H_RS + c] = 0.f;
    w2s[row * H_RS + c] = 0.f;
  }
  for (int e = tid; e < 6 * 512; e += E_NT) w2s[(10 + e / 512) * H_RS + (e & 511)] = 0.f;  // rows 10-15
  __syncthreads();
  stamp(dbg, 1);

  // ---- logits partials: wave wv sums k in [64 wv, 64 wv + 64)
  {
    const float* ha = hs + hsx(i, 64 * wv + g);   // + 4 s: the XOR touches only column bit 1
    const float* wb = w2s + hsx(i, 64 * wv + g);
    float av[16], wvv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) { av[s] = ha[4 * s]; wvv[s] = wb[4 * s]; }
    __builtin_amdgcn_sched_barrier(0);  // every operand read in flight before the first MFMA
    f32x4 c0 = zero4(), c1 = zero4();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s & 1) c1 = mfma16x16x4(av[s], wvv[s], c1);
      else c0 = mfma16x16x4(av[s], wvv[s], c0);
    }
    red[wv][lane] = c0 + c1;  // lane (i = j, g): logits of samples 4g + r
  }
  __syncthreads();
  // ---- log-softmax / NLL / d(logits), one 16-lane row per sample (waves 0-3): max, sums and
  // argmax over the row by quad / half-row / row-mirror DPP steps (every lane of the row ends
  // with the same bits)
  if (tid < 256) {
    const int smp = mt * 16 + sm_s;
    const bool jv = sm_j < 10, sv = smp < B;
    float part[E_NW];
#pragma unroll
    for (int q = 0; q < E_NW; ++q) part[q] = red[q][16 * wv + sm_j][lane >> 4];
    __builtin_amdgcn_sched_barrier(0);
    float v = part[0];
#pragma unroll
    for (int q = 1; q < E_NW; ++q) v += part[q];
    const float logit = v + b2v;
    float mx = jv ? logit : -INFINITY;
    mx = fmaxf(mx, dpp_f<0xB1>(mx));
    mx = fmaxf(mx, dpp_f<0x4E>(mx));
    mx = fmaxf(mx, dpp_f<0x141>(mx));
    mx = fmaxf(mx, dpp_f<0x140>(mx));
    float se = jv ? __expf(logit - mx) : 0.f;
    float lt = sm_j == lab_t ? logit : 0.f;  // one non-zero term: exact
    int pr = (jv && logit == mx) ? sm_j : 16;  // first maximum, as torch / head_kernel
#define PTO_ROW_STEP(CTRL)                                                                      \
    se += dpp_f<CTRL>(se);                                                                      \
    lt += dpp_f<CTRL>(lt);                                                                      \
    pr = min(pr, __builtin_amdgcn_mov_dpp(pr, CTRL, 0xF, 0xF, false));
    PTO_ROW_STEP(0xB1) PTO_ROW_STEP(0x4E) PTO_ROW_STEP(0x141) PTO_ROW_STEP(0x140)
#undef PTO_ROW_STEP
    const float lse = mx + __logf(se);
    const float dl = (jv && sv) ? (__expf(logit - lse) - (sm_j == lab_t ? 1.f : 0.f)) * a.grad_scale : 0.f;
    dls[sm_s][sm_j] = dl;
    if (pub && sv) {
      if (jv) a.dlog_out[(size_t)smp * 10 + sm_j] = dl;
      if (sm_j == 0) {
        a.per_sample[2 * smp] = lse - lt;
        a.per_sample[2 * smp + 1] = pr == lab_t ? 1.f : 0.f;
      }
    }
  }
  __syncthreads();
  stamp(dbg, 2);
  // ---- dh for this wave's 64 k (= its dz2 K range): four 16-column tiles, K = the 10 classes
  // exactly, as 10 K = 1 steps of v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4 x 4: block lane / 4 =
  // samples 4 (lane / 16) .. + 3 x columns 16 t + 4 ((lane / 4) % 4) .. + 3) -- the same D layout
  // as a 16x16x4 tile (lane (g, i): samples 4 g + r, column 16 t + i) without its 6 zero classes,
  // 80 instead of 128 matrix-pipe cycles per tile; the same k-ordered fmaf chain
  {
    float da[10], db[4][10], hm[4][4];
#pragma unroll
    for (int c = 0; c < 10; ++c) {
      da[c] = dls[4 * g + (lane & 3)][c];
#pragma unroll
      for (int t = 0; t < 4; ++t) db[t][c] = w2s[hsx(c, 64 * wv + 16 * t + i)];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) hm[t][r] = hs[hsx(4 * g + r, 64 * wv + 16 * t + i)];
    __builtin_amdgcn_sched_barrier(0);  // operands and ReLU masks in registers first
    float dv[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 c = zero4();
#pragma unroll
      for (int k = 0; k < 10; ++k) c = __builtin_amdgcn_mfma_f32_4x4x1f32(da[k], db[t][k], c, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dv[t][r] = hm[t][r] > 0.f ? c[r] : 0.f;
        dhs[dsx(4 * g + r, 64 * wv + 16 * t + i)] = dv[t][r];
      }
    }
  }
  // The dz2 job and the dh publication below read dhs columns [64 wv, 64 wv + 64) that OTHER lanes
  // of this wave just wrote.  LDS operations of one wave execute in order, so no s_barrier is
  // needed; the wave barrier and the wavefront-scope fences make that hand-off explicit to the
  // compiler (no LDS read may be scheduled above the stores) without emitting a wait.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // ---- dz2 job (fc1_bwd's job 2): K = 500 split over the waves; this wave reads only the dh it wrote
  {
    float av[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 d4 = *reinterpret_cast<const float4*>(dhs + dsx(i, kb + 4 * q));
      av[4 * q] = d4.x; av[4 * q + 1] = d4.y; av[4 * q + 2] = d4.z; av[4 * q + 3] = d4.w;
    }
    f32x4 c0 = zero4(), c1 = zero4();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s & 1) c1 = mfma16x16x4(av[s], bv[s], c1);
      else c0 = mfma16x16x4(av[s], bv[s], c0);
    }
    asm volatile("" : "+v"(a2o), "+v"(pidx));
    red[wv][lane] = c0 + c1;  // (the logits partials in red were consumed before the last barrier)
  }
  if (kt == 1 + wv) {  // dh for the tail: wave wv of tile kt = 1 + wv publishes its 64 columns of the
                       // 16 rows (every tile of the row block computes the same dh), 16-byte stores
                       // from its own LDS writes -- not all on the kt == 0 tiles, which then ended
                       // the kernel 0.3 us after the others (profiles/r5_dhs); one block-end copy of
                       // all 500 columns was slower still (profiles/r5_dhw)
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = lane + 64 * it, row = e >> 4, col = 64 * wv + 4 * (e & 15);
      if (col < 500 && mt * 16 + row < B)
        *reinterpret_cast<float4*>(a.dh_out + (size_t)(mt * 16 + row) * 500 + col) =
            *reinterpret_cast<const float4*>(dhs + dsx(row, col));
    }
  }
  __syncthreads();
  float v = red[0][l_e][r_e];
#pragma unroll
  for (int q = 1; q < E_NW; ++q) v += red[q][l_e][r_e];
  if (tid < 256 && bs < B) {
    const float d = a2o > 0.f ? v : 0.f;
    if (a.dpool != nullptr) {
      a.dpool[(size_t)bs * 800 + ff] = d;
    } else {
      const int co = ff >> 4, ph = (ff >> 2) & 3, pw = ff & 3;
      float* z = a.dz2 + (size_t)bs * 3200 + co * 64 + (2 * ph) * 8 + 2 * pw;
      z[0] = pidx == 0 ? d : 0.f;
      z[1] = pidx == 1 ? d : 0.f;
      z[8] = pidx == 2 ? d : 0.f;
      z[9] = pidx == 3 ? d : 0.f;
    }
  }
  stamp(dbg, 3);
}

// ---------------------------------------------------------------------------
// F: conv backward.  grid = (4 input-channel groups of 5, B samples), F_NT/64 waves.
//   phase 1   stage dz2[b] (two layouts), the W2 column slice, a1 slice, xn[b], idx1 slice
//   phase 2a  dcol[64 pos, 125 (ci,kh,kw)] = dz2[b]^T . W2[:, group]   (MFMA, K = 50)
//   phase 2b  dW_conv2[50, group] partial = dz2[b] . im2col(a1[b])      (MFMA, K = 64)
//   phase 3   da1 = col2im(dcol); un-pool via idx1 + ReLU mask -> dz1 (LDS)
//   phase 4   dW_conv1[group, 25] + db_conv1 partials = dz1 . im2col(xn[b]) (VALU)
//   The block's partial conv grads go to its sample's slab row (slab_stride > 0,
//   reduced deterministically later) or are added with fp32 atomics.
// ---------------------------------------------------------------------------
// LDS row strides (ds_read_b32/ds_write_b32 banks = word % 32, 32-lane groups):
constexpr int F_DS = 66;    // dz_s   [64 co][66]    A of 2b: lanes = co rows  (== 2 mod 32)
constexpr int F_D8 = 80;    // dz80_s [52 co][80]    B of 2a: lanes = pos cols, +row per g (== 16 mod 32)
constexpr int F_WS = 144;   // w_s    [52 co][144]   A of 2a: lanes = j cols, +row per g (== 16 mod 32)
constexpr int F_DC = 68;    // dcolT  [128 j][68]    2a C writes (4*68 == 16 mod 32); col2im reads
                            //                       walk pos with lanes -> conflict-free
constexpr int F_Z1 = 628;   // dz1_s [5][24 rows x F_Z1R] (+4 pad)
// strides picked with an LDS bank-conflict model so that the phase-2b im2col gathers,
// the phase-3 reads/stores and the phase-4 sliding windows are (nearly) conflict-free:
constexpr int F_Z1R = 26;   // dz1 row stride
constexpr int F_A1R = 13;   // a1 row stride
constexpr int F_A1C = 160;  // a1 channel stride (>= 12 rows x F_A1R)
constexpr int F_XR = 29;    // xn row stride
constexpr int F_OFF_DZ = 0;
constexpr int F_OFF_D8 = F_OFF_DZ + 64 * F_DS;
constexpr int F_OFF_W = F_OFF_D8 + 52 * F_D8;
constexpr int F_OFF_DCOL = F_OFF_W + 52 * F_WS;
constexpr int F_OFF_A1 = F_OFF_DCOL + 128 * F_DC;
constexpr int F_OFF_X = F_OFF_A1 + 4 * F_A1C + 12 * F_A1R;  // last channel ends at 12 rows
constexpr int F_OFF_IDX = F_OFF_X + 28 * F_XR;  // 720 uint8 (180 floats)
constexpr int F_LDS = F_OFF_IDX + 180;
// aliases of the (dead after phase 2a) weight region:
constexpr int F_OFF_DZ1 = F_OFF_W;
constexpr int F_OFF_RED = F_OFF_W + 5 * F_Z1;
constexpr int F_RED1 = 132;  // phase-4 partial row: 125 dW_conv1 taps + 5 bias sums
static_assert(5 * F_Z1 + 16 * F_RED1 <= 52 * F_WS, "alias region too small");
static_assert(F_A1C >= 12 * F_A1R && F_Z1 >= 24 * F_Z1R && F_Z1R >= 24 && F_A1R >= 12 && F_XR >= 28,
              "padded LDS rows/channels must not overlap");

constexpr int F_NT = 1024;          // 16 waves: 4 per SIMD hide the LDS latency of phase 2
constexpr int F_NW = F_NT / 64;
constexpr int F_TPW = 32 / F_NW;     // 16x16 tiles per wave in each of 2a / 2b (32 tiles each)
constexpr int F_NDZ = 4096 / F_NT;   // dz2 staging: 64 co (50 real) x 64 pos
constexpr int F_NW2 = (6656 + F_NT - 1) / F_NT;  // W2 slice staging: 52 co x 128 j
static_assert(F_NT >= 784 && 4096 % F_NT == 0 && 32 % F_NW == 0, "conv_bwd thread mapping");

__global__ __launch_bounds__(F_NT) void conv_bwd_kernel(
    const float* __restrict__ dz2, const float* __restrict__ w2, const float* __restrict__ a1,
    const uint8_t* __restrict__ idx1, const float* __restrict__ xn, float* __restrict__ gw2,
    float* __restrict__ gb2, float* __restrict__ gw1, float* __restrict__ gb1,
    float* __restrict__ dz1_out, int slab_stride, int B, u64* dbg) {
  extern __shared__ float lds[];
  float* dz_s = lds + F_OFF_DZ;
  float* dz80_s = lds + F_OFF_D8;
  float* w_s = lds + F_OFF_W;
  float* dcol_s = lds + F_OFF_DCOL;
  float* a1_s = lds + F_OFF_A1;
  float* x_s = lds + F_OFF_X;
  uint8_t* idx_s = reinterpret_cast<uint8_t*>(lds + F_OFF_IDX);
  float* dz1_s = lds + F_OFF_DZ1;
  float* red = lds + F_OFF_RED;

  const int cig = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  stamp(dbg, 0);

  // ---- phase 1: stage (all loads of a thread are independent and unrolled)
  {
    const float* dzb = dz2 + (size_t)b * 3200;
    // clamped addresses + register selects: no load is predicated (a predicated
    // load makes hipcc wait vmcnt(0) per element)
    float v[F_NDZ];
#pragma unroll
    for (int k = 0; k < F_NDZ; ++k) v[k] = dzb[min(tid + k * F_NT, 3199)];
    float wv_[F_NW2];
#pragma unroll
    for (int k = 0; k < F_NW2; ++k) {
      const int e = tid + k * F_NT;
      const int co = min(e >> 7, 49), j = min(e & 127, 124);
      wv_[k] = w2[(size_t)co * 500 + cig * 125 + j];
    }
    const int ec = min(tid, 719);
    const float av = a1[(size_t)b * 2880 + cig * 720 + ec];
    const uint8_t iv = idx1[(size_t)b * 2880 + cig * 720 + ec];
    const float xv = xn[(size_t)b * 784 + min(tid, 783)];
#pragma unroll
    for (int k = 0; k < F_NDZ; ++k)
      if (tid + k * F_NT >= 3200) v[k] = 0.f;  // co >= 50
#pragma unroll
    for (int k = 0; k < F_NW2; ++k) {
      const int e = tid + k * F_NT;
      if ((e >> 7) >= 50 || (e & 127) >= 125) wv_[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < F_NDZ; ++k) {
      const int e = tid + k * F_NT;
      const int co = e >> 6, pos = e & 63;
      dz_s[co * F_DS + pos] = v[k];
      if (co < 52) dz80_s[co * F_D8 + pos] = v[k];
    }
#pragma unroll
    for (int k = 0; k < F_NW2; ++k) {
      const int e = tid + k * F_NT;
      if (e < 6656) w_s[(e >> 7) * F_WS + (e & 127)] = wv_[k];
    }
    if (tid < 720) {
      const int c = tid / 144, pp = tid - c * 144, yy = pp / 12;
      a1_s[c * F_A1C + yy * F_A1R + (pp - yy * 12)] = av;
      idx_s[tid] = iv;
    }
    if (tid < 784) x_s[(tid / 28) * F_XR + tid % 28] = xv;
  }
  __syncthreads();
  stamp(dbg, 1);

  // ---- phase 2a: dcolT[j][pos] = W2 slice^T . dz2   (M = 128 j, N = 64 pos, K = 52)
  {
    const int pt = wv & 3, jt0 = (wv >> 2) * F_TPW;
    f32x4 acc[F_TPW];
#pragma unroll
    for (int n = 0; n < F_TPW; ++n) acc[n] = zero4();
    // all 39 LDS operands of the wave first, then the MFMA chains
    float bv[13], av[F_TPW][13];
#pragma unroll
    for (int s = 0; s < 13; ++s) {
      bv[s] = dz80_s[(4 * s + g) * F_D8 + pt * 16 + i];
#pragma unroll
      for (int n = 0; n < F_TPW; ++n) av[n][s] = w_s[(4 * s + g) * F_WS + (jt0 + n) * 16 + i];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 13; ++s)
#pragma unroll
      for (int n = 0; n < F_TPW; ++n) acc[n] = mfma16x16x4(av[n][s], bv[s], acc[n]);
#pragma unroll
    for (int n = 0; n < F_TPW; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        dcol_s[((jt0 + n) * 16 + g * 4 + r) * F_DC + pt * 16 + i] = acc[n][r];
  }
  // ---- phase 2b: dW_conv2 partial  (M = 48 co, N = 128 (ci,kh,kw), K = 64 pos)
  // MFMA tiles (mt, nt) for co 0..47: waves 0-3 take mt 0, nt {2w, 2w+1}; waves 4-7 mt 1,
  // nt {2w-8, 2w-7}; waves 8-15 mt 2, nt w-8 -- 6 tiles per SIMD, and one A fragment per
  // K-step for both tiles of a wave.  co 48 and 49 (a fourth 16-row tile would be 7/8
  // padding) are 250 VALU dot products in waves 8-11, one per SIMD, same pos order as the
  // MFMA chain.
  const int mt = wv < 4 ? 0 : (wv < 8 ? 1 : 2);
  const int ntw = wv < 8 ? 2 * (wv & 3) : wv - 8;
  const int nt2 = wv < 8 ? 2 : 1;  // tiles of this wave
  f32x4 gacc[2] = {zero4(), zero4()};
  float grow = 0.f;  // VALU rows: co 48 + item / 125, j = item % 125
  const int item = tid - 512;
  {
    // B columns j >= 125 read a clamped (valid, finite) address: they only feed output
    // columns the epilogue never stores, so no select/branch sits between load and MFMA
    int boff[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int jc = min(max((ntw + n) * 16 + i - cig, 0), 124);
      const int ci = jc / 25, t = jc - ci * 25;
      boff[n] = ci * F_A1C + (t / 5) * F_A1R + (t % 5);
    }
    const float* arow = dz_s + (mt * 16 + i) * F_DS + g;
    if (wv < 8) {
      float av[16], b0[16], b1[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int poff = (s2 >> 1) * F_A1R + 4 * (s2 & 1) + g;  // pos = 4s+g -> (oh, ow)
        av[s2] = arow[4 * s2];
        b0[s2] = a1_s[boff[0] + poff];
        b1[s2] = a1_s[boff[1] + poff];
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        gacc[0] = mfma16x16x4(b0[s2], av[s2], gacc[0]);
        gacc[1] = mfma16x16x4(b1[s2], av[s2], gacc[1]);
      }
    } else {
      float av[16], b0[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int poff = (s2 >> 1) * F_A1R + 4 * (s2 & 1) + g;
        av[s2] = arow[4 * s2];
        b0[s2] = a1_s[boff[0] + poff];
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) gacc[0] = mfma16x16x4(b0[s2], av[s2], gacc[0]);
    }
    // store the tiles now, so they drain under phases 3-4.  The tile is transposed
    // (A = im2col, B = dz2): lane (i, g) holds co = mt*16 + i and 4 consecutive
    // j = t*16 + g*4 - cig + r.  The -cig shift makes every full group start on a 16-byte
    // boundary of the slab row (544 + co*500 + cig*125 + j0 = 4 * (...)), so it is one
    // float4 store; groups cut by j < 0 or j > 124 store element-wise.
    const size_t so = slab_stride > 0 ? (size_t)b * slab_stride : 0;
    float* rowp = gw2 + so + (size_t)(mt * 16 + i) * 500 + cig * 125;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      if (n < nt2) {
        const int j0 = (ntw + n) * 16 + g * 4 - cig;
        if (slab_stride > 0 && j0 >= 0 && j0 + 3 < 125) {
          *reinterpret_cast<float4*>(rowp + j0) =
              make_float4(gacc[n][0], gacc[n][1], gacc[n][2], gacc[n][3]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = j0 + r;
            if (j >= 0 && j < 125) {
              if (slab_stride > 0) rowp[j] = gacc[n][r];
              else atomicAdd(rowp + j, gacc[n][r]);
            }
          }
        }
      }
    }
    if (item >= 0 && item < 250) {
      const int co = 48 + item / 125, j = item % 125;
      const int ci = j / 25, t = j - ci * 25;
      const float* ar = a1_s + ci * F_A1C + (t / 5) * F_A1R + (t % 5);
      const float* dr = dz_s + co * F_DS;
#pragma unroll 16
      for (int pos = 0; pos < 64; ++pos) grow = fmaf(dr[pos], ar[(pos >> 3) * F_A1R + (pos & 7)], grow);
    }
  }
  float b2sum = 0.f;
  if (cig == 0 && tid < 50) {
#pragma unroll 8
    for (int p = 0; p < 64; ++p) b2sum += dz_s[tid * F_DS + p];
  }
  __syncthreads();
  stamp(dbg, 2);

  // ---- phase 3: col2im + un-pool + ReLU mask -> dz1_s[5][24*24]
#pragma unroll
  for (int k = 0; k < (720 + F_NT - 1) / F_NT; ++k) {
    const int e = tid + k * F_NT;
    if (e < 720) {
      const int c = e / 144, p = e - c * 144;
      const int y = p / 12, x = p - y * 12;
      // tap (kh, kw) reads dcolT[(c*25 + kh*5 + kw)][(y-kh)*8 + (x-kw)] = one base address +
      // a compile-time offset (ds_read immediate).  Taps outside the 8x8 conv2 output read
      // a neighbouring in-bounds element and are dropped by the row / column masks, which
      // separate: 10 compares per output instead of 4 per tap.
      const float* base = dcol_s + c * 25 * F_DC + y * 8 + x;
      bool colok[5];
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) colok[kw] = (x - kw >= 0) & (x - kw <= 7);
      float da = 0.f;
#pragma unroll
      for (int kh = 0; kh < 5; ++kh) {
        float dr = 0.f;
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float v = base[kh * (5 * F_DC - 8) + kw * (F_DC - 1)];
          dr += colok[kw] ? v : 0.f;
        }
        da += ((y - kh >= 0) & (y - kh <= 7)) ? dr : 0.f;
      }
      const float d = a1_s[c * F_A1C + y * F_A1R + x] > 0.f ? da : 0.f;
      const int pidx = idx_s[e];
      float* z = dz1_s + c * F_Z1 + (2 * y) * F_Z1R + 2 * x;
      z[0] = pidx == 0 ? d : 0.f;
      z[1] = pidx == 1 ? d : 0.f;
      z[F_Z1R] = pidx == 2 ? d : 0.f;
      z[F_Z1R + 1] = pidx == 3 ? d : 0.f;
      if (dz1_out != nullptr) {
        float* zo = dz1_out + (size_t)b * 11520 + (cig * 5 + c) * 576 + (2 * y) * 24 + 2 * x;
        zo[0] = z[0]; zo[1] = z[1]; zo[24] = z[F_Z1R]; zo[25] = z[F_Z1R + 1];
      }
    }
  }
  __syncthreads();
  stamp(dbg, 3);

  // ---- phase 4: dW_conv1 partial + db_conv1 on the VALU.  As an MFMA GEMM this is
  // M = 5 channels padded to 16 (3/4 of every MFMA wasted, ~3 us); here 400 threads =
  // (channel c, 8 row-groups x 2 column-halves, kernel row kh) each slide a 16-wide
  // register window of the input row across 12 output columns: 5 FMAs per 2 LDS reads.
  // The kh == 0 threads also sum dz1 for the bias gradient.  16 partials meet in LDS.
  if (tid < 400) {
    const int c = tid / 80, rem = tid - c * 80;
    const int part = rem / 5, kh = rem - part * 5;
    const int ry = part & 7, cx = (part >> 3) * 12;
    const float* zr = dz1_s + c * F_Z1;
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    float bs = 0.f;
#pragma unroll
    for (int yy = 0; yy < 3; ++yy) {
      const int y = ry * 3 + yy;
      const float* xr = x_s + (y + kh) * F_XR + cx;
      float xw[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) xw[q] = xr[q];
#pragma unroll
      for (int x = 0; x < 12; ++x) {
        const float a = zr[y * F_Z1R + cx + x];
        bs += a;
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) acc[kw] = fmaf(a, xw[x + kw], acc[kw]);
      }
    }
    float* pr = red + part * F_RED1;
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) pr[c * 25 + kh * 5 + kw] = acc[kw];
    if (kh == 0) pr[125 + c] = bs;
  }
  __syncthreads();
  float w1sum = 0.f;
  if (tid < 130) {
#pragma unroll
    for (int q = 0; q < 16; ++q) w1sum += red[q * F_RED1 + tid];
  }
  stamp(dbg, 4);

  // ---- epilogue.  slab_stride > 0: plain stores of this block's partial grads into
  // the per-sample slab (reduced deterministically by conv_grad_reduce_kernel);
  // slab_stride == 0: fp32 atomics straight into the grads (standalone use).
  const bool slab = slab_stride > 0;
  const size_t so = slab ? (size_t)b * slab_stride : 0;
  if (item >= 0 && item < 250) {
    float* dst = gw2 + so + (size_t)(48 + item / 125) * 500 + cig * 125 + item % 125;
    if (slab) *dst = grow;
    else atomicAdd(dst, grow);
  }
  if (cig == 0 && tid < 50) {
    if (slab) gb2[so + tid] = b2sum;
    else atomicAdd(&gb2[tid], b2sum);
  }
  if (tid < 125) {  // tid = c * 25 + kh * 5 + kw
    float* dst = gw1 + so + cig * 125 + tid;
    if (slab) *dst = w1sum;
    else atomicAdd(dst, w1sum);
  } else if (tid < 130) {
    float* dst = gb1 + so + cig * 5 + (tid - 125);
    if (slab) *dst = w1sum;
    else atomicAdd(dst, w1sum);
  }
  stamp(dbg, 5);
}

// ---------------------------------------------------------------------------
// F4: conv backward with dW_conv2 summed over 4-sample chunks (the training path).
//   grid = (4 input-channel groups, 4 * ceil(B / 4)); block (cig, b): chunk q = b / 4,
//   quarter r = b % 4.  The per-sample input-gradient work of sample b < B is the same as
//   conv_bwd_kernel's (dcol = W2^T dz2[b] on MFMA, col2im + un-pool + ReLU mask -> dz1,
//   dW_conv1 / db_conv1 / db_conv2 partials into slab row b).  dW_conv2 instead sums the
//   chunk's FOUR samples (K = 256 positions) over one quarter of the group's 125 (ci, kh, kw)
//   columns: the same 384 MFMAs per block as the per-sample form, written to slab row q.  The
//   conv2.weight part of the slab the tail reduces shrinks 4x (B rows -> ceil(B/4): 6.4 -> 1.6
//   MB at B = 64), and so does this launch's dirty write-back at its boundary.  Deterministic:
//   every slab element has one writer, K halves and sample partials meet in a fixed order.
//   Blocks b >= B (B % 4 != 0) only compute their quarter of the last chunk.
// ---------------------------------------------------------------------------
constexpr int G_DZS = 82;             // dz row stride (== 18 mod 32: 2a reads 2-way on 2 banks, 2b free)
constexpr int G_DZR = 52;             // rows per sample: 50 co + 2 zero rows (2a's K padding to 52)
constexpr int G_DZN = G_DZR * G_DZS;  // 4264 floats per sample
constexpr int G_A1S = 2 * F_A1C;      // 2b im2col source per sample: the (at most) 2 channels touched
constexpr int G_OFF_DZ = 0;
constexpr int G_OFF_W = G_OFF_DZ + 4 * G_DZN;
constexpr int G_OFF_DCOL = G_OFF_W + 52 * F_WS;
constexpr int G_OFF_A1 = G_OFF_DCOL + 128 * F_DC;
constexpr int G_OFF_A1C = G_OFF_A1 + 4 * F_A1C + 12 * F_A1R;
constexpr int G_OFF_X = G_OFF_A1C + 4 * G_A1S;
// xn row stride of conv_bwd4 (round 6): phase 4 reads each lane's row 2 py + dy + kh at its own
// pooling argmax, so a half-wave touches ~17 rows x 2 column parities; 30 (== -2 mod 32) halves
// the conflicts of 29 (tools/lds_banks_fwd.py --only conv_bwd4: 99 -> 48 cycles per active wave)
constexpr int G_XR = 30;
constexpr int G_OFF_IDX = G_OFF_X + 28 * G_XR;
constexpr int G_OFF_PK = G_OFF_IDX + 180;     // 2b K-half-1 partial tiles: 6 x 64 lanes x f32x4
constexpr int G_OFF_PV = G_OFF_PK + 6 * 256;  // co 48/49 per-sample partials: 4 x 64
constexpr int G_LDS = G_OFF_PV + 4 * 64;
constexpr int G_OFF_DZ1 = G_OFF_W;            // aliases of the W2 slice (dead after phase 2a)
constexpr int G_OFF_RED = G_OFF_W + 5 * F_Z1;
static_assert(G_LDS * 4 <= 160 * 1024, "conv_bwd4 LDS budget");
static_assert(G_OFF_PK % 4 == 0 && G_OFF_DZ1 % 4 == 0 && G_OFF_DZ % 2 == 0 && G_DZN % 2 == 0 && G_DZS % 2 == 0, "LDS alignment");



// conv_bwd4's two wave groups synchronise through LDS arrival counters (one lane per wave adds,
// release; every lane polls, acquire)
__device__ __forceinline__ void wave_group_sync(unsigned* ctr, unsigned target) {
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
}

// conv_bwd4 phase 4 on the pooled dz1 (round 5), one item: channel c, pooled row py, tap row kh.
// dz1 is non-zero only at each pooling window's argmax (dy, dx) = idx1 (row-major 2 x 2), so
//   dW_conv1[c][kh][kw] += d[c][py][px] * x[2 py + dy + kh][2 px + dx + kw],  db_conv1[c] += d
// -- half the FMAs of the dense sliding window and one item per thread; partial rows red[py].
__device__ __forceinline__ void bwd4_dw1_item_pooled(int it, const float* dp1_s, const uint8_t* idx_s,
                                                     const float* x_s, float* red) {
  const int c = it / 60, rem = it - c * 60;
  const int py = rem / 5, kh = rem - py * 5;
  const float* dr = dp1_s + c * 144 + py * 12;
  const uint8_t* ir = idx_s + c * 144 + py * 12;
  float dv[12];
  int iv[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    dv[k] = dr[k];
    iv[k] = ir[k];
  }
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float bs = 0.f;
#pragma unroll
  for (int px = 0; px < 12; ++px) {
    const int p = iv[px];
    const float* xr = x_s + (2 * py + (p >> 1) + kh) * G_XR + 2 * px + (p & 1);
    const float a = dv[px];
    bs += a;
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) acc[kw] = fmaf(a, xr[kw], acc[kw]);
  }
  float* pr = red + py * F_RED1;
#pragma unroll
  for (int kw = 0; kw < 5; ++kw) pr[c * 25 + kh * 5 + kw] = acc[kw];
  if (kh == 0) pr[125 + c] = bs;
}

// 2a for wave w of 8: dcolT tiles jt0 .. jt0 + 3 (jt0 = 4 (w >> 2)) x position tile w & 3.
// Software-pipelined like 2b below: the LDS operand reads of k-chunk c + 1 are issued before
// the MFMAs of chunk c (sched_barrier groups keep the compiler from sinking each read to its
// use, which serialises one LDS round trip per MFMA pair).
__device__ __forceinline__ void bwd4_2a4(const float* dzc_s, const float* w_s, float* dcol_s, int r, int w,
                                         int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int pt = w & 3, jt0 = (w >> 2) * 4;
  const float* qa_b = dzc_s + r * G_DZN + g * G_DZS + pt * 16 + i;
  const float* qa_a = w_s + g * F_WS + jt0 * 16 + i;
  float ya[13], xa[4][13];
  f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#define A4_R(c)                                                 \
  _Pragma("unroll") for (int s = 4 * (c); s < 4 * (c) + 4; ++s) \
    if (s < 13) {                                               \
      ya[s] = qa_b[4 * s * G_DZS];                              \
      _Pragma("unroll") for (int t = 0; t < 4; ++t) xa[t][s] = qa_a[4 * s * F_WS + 16 * t]; \
    }
#define A4_M(c)                                                 \
  _Pragma("unroll") for (int s = 4 * (c); s < 4 * (c) + 4; ++s) \
    if (s < 13) {                                               \
      _Pragma("unroll") for (int t = 0; t < 4; ++t) acc[t] = mfma16x16x4(xa[t][s], ya[s], acc[t]); \
    }
#define A4_SB __builtin_amdgcn_sched_barrier(0);
  A4_R(0) A4_SB A4_R(1) A4_SB A4_M(0) A4_SB A4_R(2) A4_SB A4_M(1) A4_SB A4_R(3) A4_SB A4_M(2) A4_SB A4_M(3)
#undef A4_R
#undef A4_M
#undef A4_SB
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) dcol_s[((jt0 + t) * 16 + g * 4 + rr) * F_DC + pt * 16 + i] = acc[t][rr];
}

// 2b, one K half (samples 2 kh2, 2 kh2 + 1 of the chunk) of dW_conv2 tile pair tp, in four
// chunks of 8 k-steps, reads one chunk ahead of the MFMAs
__device__ __forceinline__ f32x4 bwd4_2b(const float* dzc_s, const float* a1c_s, int tp, int kh2, int lane,
                                         int jbase, int c0) {
  const int i = lane & 15, g = lane >> 4;
  const int ct = tp >> 1, jt = tp & 1;
  const int jc = min(max(jbase + jt * 16 + i, 0), 124);
  const int ci = jc / 25, t = jc - ci * 25;
  const float* qb_a = a1c_s + 2 * kh2 * G_A1S + (ci - c0) * F_A1C + (t / 5) * F_A1R + (t % 5) + g;
  const float* qb_b = dzc_s + 2 * kh2 * G_DZN + (ct * 16 + i) * G_DZS + g;
  float xb[32], yb[32];
  f32x4 e0 = zero4(), e1 = zero4();
#define B2_R(c)                                                   \
  _Pragma("unroll") for (int u = 8 * (c); u < 8 * (c) + 8; ++u) { \
    const int s_ = u >> 4, uu = u & 15;                           \
    xb[u] = qb_a[s_ * G_A1S + (uu >> 1) * F_A1R + 4 * (uu & 1)];  \
    yb[u] = qb_b[s_ * G_DZN + 4 * uu];                            \
  }
#define B2_M(c)                                                   \
  _Pragma("unroll") for (int u = 8 * (c); u < 8 * (c) + 8; ++u) { \
    if (u & 1) e1 = mfma16x16x4(xb[u], yb[u], e1);                \
    else e0 = mfma16x16x4(xb[u], yb[u], e0);                      \
  }
#define B2_SB __builtin_amdgcn_sched_barrier(0);
  B2_R(0) B2_SB B2_R(1) B2_SB B2_M(0) B2_SB B2_R(2) B2_SB B2_M(1) B2_SB B2_R(3) B2_SB B2_M(2) B2_SB B2_M(3)
#undef B2_R
#undef B2_M
#undef B2_SB
  return e0 + e1;
}

__global__ __launch_bounds__(F_NT) void conv_bwd4_kernel(
    const float* __restrict__ dp, const uint8_t* __restrict__ ip,
    const float* __restrict__ w2, const float* __restrict__ a1,
    const uint8_t* __restrict__ idx1, const float* __restrict__ xn, float* __restrict__ slab,
    int stride, int o_gw2, int o_gb2, int o_gw1, int o_gb1, int B, u64* dbg) {
  extern __shared__ float lds[];
  float* dzc_s = lds + G_OFF_DZ;
  float* w_s = lds + G_OFF_W;
  float* dcol_s = lds + G_OFF_DCOL;
  float* a1_s = lds + G_OFF_A1;
  float* a1c_s = lds + G_OFF_A1C;
  float* x_s = lds + G_OFF_X;
  uint8_t* idx_s = reinterpret_cast<uint8_t*>(lds + G_OFF_IDX);
  f32x4* pk_s = reinterpret_cast<f32x4*>(lds + G_OFF_PK);
  float* pv_s = lds + G_OFF_PV;
  float* dp1_s = lds + G_OFF_DZ1;  // pooled d(a1) [5][144]
  float* red = lds + G_OFF_RED;

  const int cig = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int q = b >> 2, r = b & 3;
  const bool own = b < B;  // block-uniform: this block also does sample b's input-gradient work
  const int bo = own ? b : B - 1;
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  // dW_conv2 columns of this block: j in [32r - cig, 32r - cig + 32) of the group's 125; the
  // -cig shift puts every whole 4-column group on a 16-byte slab boundary (epilogue float4s)
  const int jbase = 32 * r - cig;
  const int c0 = max(jbase, 0) / 25;  // first of the <= 2 input channels those columns touch
  stamp(dbg, 0);

  // ---- phase 1: stage.  dz2 arrives pooled -- d(a2) [B][800] (ReLU-masked) + conv12's pool
  // argmax idx2 [B][800] -- and is un-pooled into the LDS image of the chunk's 4 samples (3.2 KB
  // per sample instead of the 12.8 KB dense dz2); with it the W2 slice, the 2b im2col source, the
  // own a1 / idx1 / xn.  Every load is a 16-byte vector (4-byte for idx2), spread over the
  // waves (<= 6 per wave instead of 20 scalar ones), all issued before the first LDS write.
  // The W2 slice is staged as the aligned float4 window w2[co][124 cig .. 124 cig + 128) and read
  // at j + cig (2a's rows j >= 125 are garbage-in, never read by col2im).
  float4 pdv = make_float4(0.f, 0.f, 0.f, 0.f), wq1 = pdv, cvv = pdv, avv = pdv, xvv = pdv;
  uint32_t piv = 0u;
  uint4 ivv = make_uint4(0u, 0u, 0u, 0u);
  const int e_cv = tid - 736, e_av = tid - 640, e_x = tid - 800;  // 288 / 180 / 196 lanes
  if (tid < 800) {
    const int sq = tid / 200;
    const size_t o = (size_t)min(4 * q + sq, B - 1) * 200 + (tid - sq * 200);
    pdv = reinterpret_cast<const float4*>(dp)[o];
    piv = reinterpret_cast<const uint32_t*>(ip)[o];
  }
  const float4* w24 = reinterpret_cast<const float4*>(w2) + cig * 31;
  const float4 wq0 = w24[(tid >> 5) * 125 + (tid & 31)];
  if (tid < 640) wq1 = w24[min((tid + 1024) >> 5, 49) * 125 + (tid & 31)];
  if (e_cv >= 0) {
    const int s = e_cv / 72, rem = e_cv - s * 72, c = rem / 36;
    cvv = reinterpret_cast<const float4*>(a1)[(size_t)min(4 * q + s, B - 1) * 720 + (cig * 5 + c0 + c) * 36 +
                                              (rem - c * 36)];
  }
  if (e_av >= 0 && e_av < 180) avv = reinterpret_cast<const float4*>(a1)[(size_t)bo * 720 + cig * 180 + e_av];
  if (e_x >= 0 && e_x < 196) xvv = reinterpret_cast<const float4*>(xn)[(size_t)bo * 196 + e_x];
  if (tid < 45) ivv = reinterpret_cast<const uint4*>(idx1)[(size_t)bo * 180 + cig * 45 + tid];
  __shared__ unsigned s_grp[2];  // group arrival counters (waves 0-7, waves 8-15)
  if (tid == 0) {
    s_grp[0] = 0u;
    s_grp[1] = 0u;
  }
  if (tid < 800) {  // the lane's 4 pooled values (one co, pooled row ph, pw 0..3) -> 2 rows x 8
    const int sq = tid / 200, f4 = tid - sq * 200, co = f4 >> 2, ph = f4 & 3;
    const bool ok = 4 * q + sq < B;  // samples >= B of the chunk as 0
    const float v[4] = {pdv.x, pdv.y, pdv.z, pdv.w};
    float2* z0 = reinterpret_cast<float2*>(dzc_s + sq * G_DZN + co * G_DZS + 16 * ph);
    // lanes with ph 2, 3 store their second row first (round 6): their rows sit 32 floats after
    // ph 0, 1's, i.e. on the same banks, and each 16-lane group of the float2 stores is 2-way
    // otherwise (tools/lds_banks_fwd.py --only conv_bwd4: 25 -> 0 conflict cycles per wave)
    const int sw = (ph & 2) ? 4 : 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned pu = (piv >> (8 * u)) & 0xffu;
      const float vv = ok ? v[u] : 0.f;
      const float2 ra = make_float2(pu == 0u ? vv : 0.f, pu == 1u ? vv : 0.f);
      const float2 rb = make_float2(pu == 2u ? vv : 0.f, pu == 3u ? vv : 0.f);
      z0[u + sw] = sw ? rb : ra;
      z0[u + 4 - sw] = sw ? ra : rb;
    }
  }
  if (tid < 512) {  // zero rows 50, 51 of every sample (2a reads co up to 51)
    const int s = tid >> 7, rr = 50 + ((tid >> 6) & 1);
    dzc_s[s * G_DZN + rr * G_DZS + (tid & 63)] = 0.f;
  }
  reinterpret_cast<float4*>(w_s + (tid >> 5) * F_WS)[tid & 31] = wq0;
  if (tid < 640) {
    const int co = (tid + 1024) >> 5;
    reinterpret_cast<float4*>(w_s + co * F_WS)[tid & 31] = co < 50 ? wq1 : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (tid >= 960 && tid < 1012)  // window tail (j + cig reads up to m = 130)
    reinterpret_cast<float4*>(w_s + (tid - 960) * F_WS)[32] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e_cv >= 0) {
    const int s = e_cv / 72, rem = e_cv - s * 72, c = rem / 36, p4 = rem - c * 36, y = p4 / 3;
    const bool ok = 4 * q + s < B;
    float* d = a1c_s + s * G_A1S + c * F_A1C + y * F_A1R + 4 * (p4 - 3 * y);
    d[0] = ok ? cvv.x : 0.f;
    d[1] = ok ? cvv.y : 0.f;
    d[2] = ok ? cvv.z : 0.f;
    d[3] = ok ? cvv.w : 0.f;
  }
  if (e_av >= 0 && e_av < 180) {
    const int c = e_av / 36, p4 = e_av - c * 36, y = p4 / 3;
    float* d = a1_s + c * F_A1C + y * F_A1R + 4 * (p4 - 3 * y);
    d[0] = avv.x;
    d[1] = avv.y;
    d[2] = avv.z;
    d[3] = avv.w;
  }
  if (e_x >= 0 && e_x < 196) {
    const int y = e_x / 7;
    float* d = x_s + y * G_XR + 4 * (e_x - 7 * y);
    d[0] = xvv.x;
    d[1] = xvv.y;
    d[2] = xvv.z;
    d[3] = xvv.w;
  }
  if (tid < 45) {
    uint32_t* d = reinterpret_cast<uint32_t*>(idx_s) + 4 * tid;
    d[0] = ivv.x;
    d[1] = ivv.y;
    d[2] = ivv.z;
    d[3] = ivv.w;
  }
  __syncthreads();
  stamp(dbg, 1);

  // ---- phases 2-4 in two wave groups (round-4 A/B, profiles/r4_bwd4_split_ab.txt: -0.6 us per
  // step).  Waves w and w + 4 share a SIMD, so each SIMD runs two waves of each group:
  //   group B (waves 8-15): all of 2b -- dW_conv2[co, jbase + jl] over the chunk's 4 samples
  //     (K = 256 positions); waves 8-11 tile pairs 0-3 over both K halves, waves 12-15 tile
  //     pairs 4-5 one K half each + co 48 / 49 (a fourth 16-row tile would be 7/8 padding) as
  //     256 VALU dot products; then its slab rows.
  //   group A (waves 0-7): 2a -- dcolT[j][pos] = W2 slice^T . dz2[b] (M = 128 j, N = 64 pos,
  //     K = 52), four tiles per wave -- then col2im, dW_conv1 and the own sample's slab row:
  //     its VALU phases overlap group B's MFMAs instead of following them behind a barrier.
  // The groups synchronise through LDS arrival counters; per-tile operation order as the
  // one-barrier form: bit-identical.
  if (wv >= 8) {  // ---- group B: all of 2b, then its slab rows
    const int w8 = wv - 8;
    const int tpb = w8 < 4 ? w8 : 4 + ((w8 - 4) >> 1), khb = (w8 - 4) & 1;
    f32x4 gacc;
    if (w8 < 4) {
      const f32x4 h0 = bwd4_2b(dzc_s, a1c_s, tpb, 0, lane, jbase, c0);
      gacc = h0 + bwd4_2b(dzc_s, a1c_s, tpb, 1, lane, jbase, c0);  // K half 0 + K half 1
    } else {
      gacc = bwd4_2b(dzc_s, a1c_s, tpb, khb, lane, jbase, c0);
      if (khb) pk_s[tpb * 64 + lane] = gacc;
      const int item = tid - 768;  // co 48 / 49 on the VALU, as the barrier form
      const int sm = item >> 6, cr = (item >> 5) & 1, jl = item & 31;
      const int jc = min(max(jbase + jl, 0), 124);
      const int ci = jc / 25, t = jc - ci * 25;
      const float* ar = a1c_s + sm * G_A1S + (ci - c0) * F_A1C + (t / 5) * F_A1R + (t % 5);
      const float* dr = dzc_s + sm * G_DZN + (48 + cr) * G_DZS;
      float accv = 0.f;
#pragma unroll 16
      for (int pos = 0; pos < 64; ++pos) accv = fmaf(dr[pos], ar[(pos >> 3) * F_A1R + (pos & 7)], accv);
      pv_s[item] = accv;
    }
    wave_group_sync(&s_grp[1], 8u);
    stamp(dbg, 7, 512);  // diagnostics: 2b done (group B), read by tools/step_timeline.py (round 5:
                         // 4.66 us after the stage, when group A has just finished col2im)
    float* rowq = slab + (size_t)q * stride + o_gw2 + cig * 125;
    if (w8 < 4 || khb == 0) {
      if (w8 >= 4) gacc += pk_s[tpb * 64 + lane];
      const int ctb = tpb >> 1, jtb = tpb & 1;
      float* rp = rowq + (ctb * 16 + i) * 500;
      const int j0 = jbase + jtb * 16 + 4 * g;
      if (j0 >= 0 && j0 + 3 < 125) {
        *reinterpret_cast<float4*>(rp + j0) = make_float4(gacc[0], gacc[1], gacc[2], gacc[3]);
      } else {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          if (j0 + rr >= 0 && j0 + rr < 125) rp[j0 + rr] = gacc[rr];
      }
    } else if (w8 == 5) {
      const float v = ((pv_s[lane] + pv_s[64 + lane]) + pv_s[128 + lane]) + pv_s[192 + lane];
      const int j = jbase + (lane & 31);
      if (j >= 0 && j < 125) rowq[(48 + (lane >> 5)) * 500 + j] = v;
    } else if (cig == 0 && own && lane < 50) {  // wave 15: db_conv2 of the own sample, off group A's
      // critical path (on wave 0 of group A it made the cig == 0 blocks 0.5 us slower, profiles/r5_b2)
      const float* dzo = dzc_s + r * G_DZN + lane * G_DZS;
      float b2sum = 0.f;
#pragma unroll 8
      for (int p = 0; p < 64; ++p) b2sum += dzo[p];
      slab[(size_t)b * stride + o_gb2 + lane] = b2sum;
    }
    return;
  }
  // ---- group A (waves 0-7): 2a, col2im, dW_conv1, the own sample's slab row
  if (!own) return;
  bwd4_2a4(dzc_s, w_s + cig, dcol_s, r, wv, lane);
  wave_group_sync(&s_grp[0], 8u);
  stamp(dbg, 2);
  for (int it = tid; it < 720; it += 512) {  // phase 3 (as below)
    const int c = it / 144, p = it - c * 144;
    const int y = p / 12, x = p - y * 12;
    const float* base = dcol_s + c * 25 * F_DC + y * 8 + x;
    bool colok[5];
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) colok[kw] = (x - kw >= 0) & (x - kw <= 7);
    float da = 0.f;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh) {
      float dr = 0.f;
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        const float v = base[kh * (5 * F_DC - 8) + kw * (F_DC - 1)];
        dr += colok[kw] ? v : 0.f;
      }
      da += ((y - kh >= 0) & (y - kh <= 7)) ? dr : 0.f;
    }
    // the pooled d(a1), ReLU-masked: dz1 stays pooled (its un-pooled image is 3/4 zeros; phase 4
    // places each value through idx1)
    dp1_s[it] = a1_s[c * F_A1C + y * F_A1R + x] > 0.f ? da : 0.f;
  }
  wave_group_sync(&s_grp[0], 16u);
  stamp(dbg, 3);
  {
    constexpr int NPART = 12;
    // phase 4 on the pooled dz1: 300 items (c, pooled row py, tap row kh), one per thread
    if (tid < 300) bwd4_dw1_item_pooled(tid, dp1_s, idx_s, x_s, red);
    wave_group_sync(&s_grp[0], 24u);
    stamp(dbg, 4);
    float* rowb = slab + (size_t)b * stride;
    if (tid < 130) {
      float w1sum = 0.f;
#pragma unroll
      for (int qq = 0; qq < NPART; ++qq) w1sum += red[qq * F_RED1 + tid];
      if (tid < 125) rowb[o_gw1 + cig * 125 + tid] = w1sum;
      else rowb[o_gb1 + cig * 5 + (tid - 125)] = w1sum;
    }
    stamp(dbg, 5);
  }
}

// ---------------------------------------------------------------------------
// G: deterministic reduction of the conv-grad slabs:
//   out[c] = sum_{row < rows(c)} P[row * stride + c],  rows(c) = rows_big for the float4
//   columns [big_lo4, big_hi4) (conv2.weight: one row per 4-sample chunk, conv_bwd4_kernel)
//   and B elsewhere (the per-sample conv1 / bias partials).  Rows are summed in a fixed
//   order (slices of consecutive rows, then the slices in order): bit-reproducible.
// ---------------------------------------------------------------------------
// Slab reduction geometry: SR_COLS float4 columns per workgroup x SR_SL row slices, SR_CH
// loads in flight per thread.  32 columns (200 reduction workgroups at B = 64, 32 KB each)
// beat 64 (100 x 64 KB): 0.25 us off the load phase.
constexpr int SR_COLS = 32;
constexpr int SR_CH = 8;
constexpr int SR_SL = 256 / SR_COLS;

__device__ __forceinline__ void add4(float4& a, const float4& v) {
  a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
}

// Rows [slice * per, min(rows, (slice + 1) * per)) of float4 column cc summed in row order,
// per = ceil(rows / nsl).  Every load is issued before the first add (clamped addresses).
__device__ __forceinline__ float4 slab_col_sum(const float4* __restrict__ P4, long s4, int cc, int rows,
                                               int slice, int nsl) {
  const int per = (rows + nsl - 1) / nsl;
  const int b0 = slice * per, b1 = min(rows, b0 + per);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (per <= 2) {  // chunked conv2.weight rows: 16 rows / 8 slices at B = 64
    const float4 v0 = P4[(size_t)min(b0, rows - 1) * s4 + cc];
    const float4 v1 = P4[(size_t)min(b0 + 1, rows - 1) * s4 + cc];
    if (b0 < b1) add4(acc, v0);
    if (b0 + 1 < b1) add4(acc, v1);
    return acc;
  }
  for (int base = b0; base < b1; base += SR_CH) {
    float4 v[SR_CH];
#pragma unroll
    for (int k = 0; k < SR_CH; ++k) v[k] = P4[(size_t)min(base + k, rows - 1) * s4 + cc];
#pragma unroll
    for (int k = 0; k < SR_CH; ++k)
      if (base + k < b1) add4(acc, v[k]);
  }
  return acc;
}

struct SlabRows {
  int rows;      // rows of every column outside [big_lo4, big_hi4)
  int rows_big;  // rows of the columns inside
  int big_lo4, big_hi4;
  __device__ __forceinline__ int of(int c4) const { return (c4 >= big_lo4 && c4 < big_hi4) ? rows_big : rows; }
};

__global__ __launch_bounds__(256) void slab_reduce_kernel(
    const float* __restrict__ P, SlabRows sr, int n, int stride, float* __restrict__ out, u64* dbg) {
  __shared__ float4 red[SR_SL][SR_COLS];
  stamp(dbg, 0);
  const int tid = threadIdx.x;
  const int col = blockIdx.x * SR_COLS + (tid % SR_COLS);
  const int slice = tid / SR_COLS;
  const int n4 = n >> 2;
  const int cc = min(col, n4 - 1);
  red[slice][tid % SR_COLS] = slab_col_sum(reinterpret_cast<const float4*>(P), stride >> 2, cc, sr.of(cc),
                                           slice, SR_SL);
  __syncthreads();
  if (tid < SR_COLS && col < n4) {
    float4 r = red[0][tid];
#pragma unroll
    for (int q = 1; q < SR_SL; ++q) add4(r, red[q][tid]);
    reinterpret_cast<float4*>(out)[col] = r;
  }
  stamp(dbg, 1);
}

// ---------------------------------------------------------------------------
// G+H: slab reduction fused with the SGD(momentum) update of the same elements
//   (single-process path: the conv grads never make a round trip before the
//   update).  Also writes the reduced grads (inspection / grad-norm logging) and
//   advances the device batch cursor.  Blocks past the reduction: plain SGD over a
//   second, already-reduced range (p2/g2/buf2: the fc parameters).
// ---------------------------------------------------------------------------
// fc1.weight's gradient computed inside the tail (world-1 step, round 5): dW_fc1 = dh^T . a2
// (K = B) tile by tile on MFMA -- the same tiles, lane mapping and summation order as
// fc1_bwd's job 1, so the gradient bits are identical -- and SGD applied to the tile's float4s
// straight from the accumulators.  fc1_bwd then runs only the dz2 / fc2 / staging jobs (its
// span no longer waits for the dW_fc1 tiles), and the 1.6 MB gradient is neither stored by
// fc1_bwd nor re-read here.  db_fc1 (the kt == 0 tiles' dh column sums) gets its SGD here too.
struct TailW1 {
  const float *dh, *a2;  // head's dh [B][500], conv12's a2 [B][800]
  float *p, *m;          // fc1.weight then fc1.bias (p + 400000) params / momentum
  float* g;              // optional: also store the gradient (fc1.weight, then fc1.bias)
  int B, blocks;         // blocks: 400 (4 tiles of 16 x 16 per 256-thread block), +8 with fc2; 0 = off
  // fc2 (with the fused head, fc1_bwd's job 3 moves here too): dW_fc2 = d(logits)^T . h, db_fc2,
  // their SGD, and the step's loss statistics; fc2 == 0: off
  int fc2;
  const float *dlog, *h, *per_sample;
  float* stats;
  float loss_scale;
  float *p2, *m2, *g2;    // fc2.weight [10][500] params / momentum / optional gradient
  float *pb2, *mb2, *gb2; // fc2.bias [10]
  // grad_only (the DDP step over RCCL, round 6): store every gradient (g, g2, gb2, the slab
  // reduction's gout) and touch no parameter or momentum -- the all-reduced buckets then feed
  // one SGD launch
  int grad_only;
};
constexpr int T_W1_BLOCKS = 1600 / 4;
constexpr int T_FC2_BLOCKS = 32 / 4;

// fc1_bwd's job 3 as a tail tile (same tiles, operands and summation order: the same gradient
// bits) with SGD applied from the accumulators
__device__ __forceinline__ void tail_fc2_tile(const TailW1& tw, int nt, int lane, const SgdHyper& hy) {
  const int i = lane & 15, g = lane >> 4;
  const int B = tw.B;
  const int jc = min(i, 9);
  const int n = nt * 16 + i;
  const int ncl = min(n, 499);
  const bool do_stats = nt == 1 && tw.per_sample != nullptr && tw.stats != nullptr;
  float ls = 0.f, cs = 0.f;  // the first 64 samples' statistics, in flight with the GEMM loads
  if (do_stats) loss_stats_load(tw.per_sample, B, lane, ls, cs);
  const bool upd = !tw.grad_only;
  float pp[4] = {0.f, 0.f, 0.f, 0.f}, mm[4] = {0.f, 0.f, 0.f, 0.f};
  if (upd) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = min(g * 4 + r, 9);
      pp[r] = tw.p2[j * 500 + ncl];
      mm[r] = tw.m2[j * 500 + ncl];
    }
  }
  float bp = 0.f, bm = 0.f;
  if (upd && nt == 0 && g == 0) { bp = tw.pb2[jc]; bm = tw.mb2[jc]; }
  float dbsum;
  const f32x4 c = fc2_wgrad_tile(tw.dlog, tw.h, B, nt, lane, dbsum);
  if (n < 500) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = g * 4 + r;
      if (j < 10) {
        if (tw.g2 != nullptr) tw.g2[j * 500 + n] = c[r];
        if (upd) {
          sgd_elem(pp[r], mm[r], c[r], hy);
          tw.p2[j * 500 + n] = pp[r];
          tw.m2[j * 500 + n] = mm[r];
        }
      }
    }
  }
  if (nt == 0) {
    dbsum = sum_lane_rows(dbsum);
    if (g == 0 && i < 10) {
      if (tw.gb2 != nullptr) tw.gb2[i] = dbsum;
      if (upd) {
        sgd_elem(bp, bm, dbsum, hy);
        tw.pb2[i] = bp;
        tw.mb2[i] = bm;
      }
    }
  }
  if (do_stats) {
    loss_stats_finish(tw.per_sample, B, lane, ls, cs);
    if (lane == 0) { tw.stats[0] = ls * tw.loss_scale; tw.stats[1] = cs; }
  }
}

__device__ __forceinline__ void tail_w1_tile(const TailW1& tw, int tile, int lane, const SgdHyper& hy) {
  const int i = lane & 15, g = lane >> 4;
  const int nt = tile / 50, kt = tile - nt * 50;
  const int n = nt * 16 + i;
  const bool nv = n < 500;
  const int nc = nv ? n : 499;
  // parameters + momentum of this lane's four outputs, in flight with the GEMM operand loads
  const unsigned e4 = (unsigned)(nc * 200 + kt * 4 + g);
  const bool upd = !tw.grad_only;
  float4 pp = make_float4(0.f, 0.f, 0.f, 0.f), mm = pp;
  if (upd) {
    pp = reinterpret_cast<const float4*>(tw.p)[e4];
    mm = reinterpret_cast<const float4*>(tw.m)[e4];
  }
  const bool bl = kt == 0 && g == 0;  // this lane also updates fc1.bias[n]
  float bp = 0.f, bm = 0.f;
  if (upd && bl) { bp = tw.p[400000 + nc]; bm = tw.m[400000 + nc]; }
  float dbsum;
  const f32x4 c = fc1_wgrad_tile(tw.dh, tw.a2, tw.B, nt, kt, lane, dbsum);
  if (nv) {
    const float4 gg = make_float4(c[0], c[1], c[2], c[3]);
    if (tw.g != nullptr) reinterpret_cast<float4*>(tw.g)[e4] = gg;
    if (upd) {
      sgd4(pp, mm, gg, hy);
      reinterpret_cast<float4*>(tw.p)[e4] = pp;
      reinterpret_cast<float4*>(tw.m)[e4] = mm;
    }
  }
  if (kt == 0) {
    dbsum = sum_lane_rows(dbsum);
    if (bl && nv) {
      if (tw.g != nullptr) tw.g[400000 + n] = dbsum;
      if (upd) {
        sgd_elem(bp, bm, dbsum, hy);
        tw.p[400000 + n] = bp;
        tw.m[400000 + n] = bm;
      }
    }
  }
}

__global__ __launch_bounds__(256) void slab_reduce_sgd_kernel(
    const float* __restrict__ P, SlabRows sr, int n, int stride, float* __restrict__ gout,
    float* __restrict__ p, float* __restrict__ buf, SgdHyper hy, int* __restrict__ step_counter,
    float* __restrict__ p2, const float* __restrict__ g2, float* __restrict__ buf2, int n2,
    int red_blocks, TailW1 tw, u64* dbg) {
  __shared__ float4 red[SR_SL][SR_COLS];
  stamp(dbg, 0);
  const int tid = threadIdx.x;
  // logical block ids: [0, red_blocks) the slab reduction, [red_blocks, + tw.blocks) the
  // fc1.weight tiles, then the plain SGD range.  Dispatch order: the fc1.weight tiles first
  // (same-box A/B against reduction-first: 38.49-38.63 vs 38.60-38.77 us/step at K = 2000,
  // profiles/r5_tail/ab.txt)
  const int blk = (int)blockIdx.x < tw.blocks ? (int)blockIdx.x + red_blocks
                  : (int)blockIdx.x < tw.blocks + red_blocks ? (int)blockIdx.x - tw.blocks : (int)blockIdx.x;
  if (blk >= red_blocks && blk < red_blocks + tw.blocks) {
    const int tile = (blk - red_blocks) * 4 + (tid >> 6);
    if (tile < 1600) tail_w1_tile(tw, tile, tid & 63, hy);
    else tail_fc2_tile(tw, tile - 1600, tid & 63, hy);
    stamp(dbg, 1);
    return;
  }
  if (blk >= red_blocks) {
    // plain SGD over the second range (already-reduced grads, e.g. the fc bucket)
    const int v = (blk - red_blocks - tw.blocks) * 256 + tid;
    if (v < (n2 >> 2)) {
      float4 pp = reinterpret_cast<float4*>(p2)[v];
      const float4 gg = reinterpret_cast<const float4*>(g2)[v];
      float4 bb = reinterpret_cast<float4*>(buf2)[v];
      sgd4(pp, bb, gg, hy);
      reinterpret_cast<float4*>(p2)[v] = pp;
      reinterpret_cast<float4*>(buf2)[v] = bb;
    }
    stamp(dbg, 1);
    return;
  }
  const int col = blk * SR_COLS + (tid % SR_COLS);
  const int slice = tid / SR_COLS;
  const int n4 = n >> 2;
  const int cc = min(col, n4 - 1);
  float4 pp = make_float4(0.f, 0.f, 0.f, 0.f), bb = pp;
  if (tid < SR_COLS && !tw.grad_only) {  // prefetch the parameters + momentum this column updates
    pp = reinterpret_cast<const float4*>(p)[cc];
    bb = reinterpret_cast<const float4*>(buf)[cc];
  }
  red[slice][tid % SR_COLS] = slab_col_sum(reinterpret_cast<const float4*>(P), stride >> 2, cc, sr.of(cc),
                                           slice, SR_SL);
  __syncthreads();
  if (tid < SR_COLS && col < n4) {
    float4 r = red[0][tid];
#pragma unroll
    for (int q = 1; q < SR_SL; ++q) add4(r, red[q][tid]);
    if (gout != nullptr) reinterpret_cast<float4*>(gout)[col] = r;
    if (!tw.grad_only) {
      sgd4(pp, bb, r, hy);
      reinterpret_cast<float4*>(p)[col] = pp;
      reinterpret_cast<float4*>(buf)[col] = bb;
    }
  }
  if (step_counter != nullptr && blk == 0 && tid == 0) atomicAdd(step_counter, 1);
  stamp(dbg, 1);
}

// ---------------------------------------------------------------------------
// H: SGD with momentum over a flat fp32 buffer (torch.optim.SGD semantics:
// buf = momentum*buf + (1-dampening)*g (buf = g on the first step),
// p -= lr * (nesterov ? g + momentum*buf : buf)); grad_scale folds the DDP 1/world.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sgd_momentum_kernel(
    float* __restrict__ p, const float* __restrict__ gr, float* __restrict__ buf, long n, SgdHyper hy,
    int* __restrict__ step_counter) {
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < n4 + 4; v += stride) {
    // vector body + scalar tail (the last 4 "virtual" slots cover n % 4 elements)
    long lo, hi;
    if (v < n4) { lo = v * 4; hi = lo + 4; }
    else { lo = n4 * 4 + (v - n4); hi = lo + 1; if (lo >= n) continue; }
    if (hi - lo == 4) {
      float4 pp = reinterpret_cast<float4*>(p)[v];
      const float4 gg = reinterpret_cast<const float4*>(gr)[v];
      float4 bb = reinterpret_cast<float4*>(buf)[v];
      sgd4(pp, bb, gg, hy);
      reinterpret_cast<float4*>(p)[v] = pp;
      reinterpret_cast<float4*>(buf)[v] = bb;
    } else {
      float pv = p[lo], mv = buf[lo];
      sgd_elem(pv, mv, gr[lo], hy);
      p[lo] = pv;
      buf[lo] = mv;
    }
  }
  if (step_counter != nullptr && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(step_counter, 1);
}

inline BatchSrc make_src(const void* x, int is_u8, const int* labels, const int* perm,
                         const int* cursor, int host_offset, int n_total, float scale,
                         float shift) {
  BatchSrc s;
  s.x = x; s.labels = labels; s.perm = perm; s.cursor = cursor; s.host_offset = host_offset;
  s.n_total = n_total; s.is_u8 = is_u8; s.scale = scale; s.shift = shift;
  return s;
}

// Phase-timestamp buffer (tools/phase_profile.py, tools/step_timeline.py); null in production.
// Every launch takes the next of kDbgSlots slots of kDbgSlotU64 words (<= 1024 blocks x 16), so
// the kernels of one captured step stamp disjoint regions.
constexpr int kDbgSlots = 16;
constexpr long kDbgSlotU64 = 1024L * 16;
u64* g_dbg = nullptr;
int g_dbg_slot = 0;

u64* dbg_next() {
  if (g_dbg == nullptr) return nullptr;
  u64* p = g_dbg + (long)(g_dbg_slot % kDbgSlots) * kDbgSlotU64;
  ++g_dbg_slot;
  return p;
}

template <typename K>
int set_max_lds(K kernel, int bytes, std::atomic<unsigned>& done) {
  // > 64 KB of dynamic LDS must be opted into once per device and kernel (thread-safe: several
  // host threads may drive different GPUs through this library)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 32) return -1;
  if (!(done.load(std::memory_order_acquire) & (1u << dev))) {
    const hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return (int)e;
    done.fetch_or(1u << dev, std::memory_order_release);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// S: the learnable synthetic MNIST stand-in (data/synthetic.py's recipe) drawn on the device by
// one launch of this library -- the worker's start-up path: torch's own kernels for the same
// warps cost 0.4-0.8 s of first-use code-object loading there (profiles/r4_startup.md).  Image
// n: label = class template picked by a counter hash; sample = the template under a random
// isotropic scale (+-10 %) and shift (+-0.125 of the half-width) read bilinearly with zero
// padding (affine_grid / grid_sample, align_corners = False), times a random contrast in
// [0.6, 1), plus noise * u^3; clamped to [0, 1], rounded to uint8.  One thread per pixel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned hash3(unsigned a, unsigned b, unsigned c) {
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float unif(unsigned h) { return (float)(h >> 8) * (1.f / 16777216.f); }

__global__ __launch_bounds__(256) void synth_mnist_kernel(const float* __restrict__ tmpl, uint8_t* __restrict__ img,
                                                          int* __restrict__ lab, int n, unsigned seed,
                                                          float noise) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)n * 784) return;
  const int im = (int)(idx / 784), px = (int)(idx - (long)im * 784);
  const unsigned u = (unsigned)im;
  const int c = (int)(hash3(seed, u, 0u) % 10u);
  const float sc = 1.f + (unif(hash3(seed, u, 1u)) - 0.5f) * 0.2f;
  const float tx = (unif(hash3(seed, u, 2u)) - 0.5f) * 0.25f, ty = (unif(hash3(seed, u, 3u)) - 0.5f) * 0.25f;
  const float contrast = 0.6f + 0.4f * unif(hash3(seed, u, 4u));
  const int y = px / 28, x = px - y * 28;
  const float gx = sc * ((2 * x + 1) / 28.f - 1.f) + tx, gy = sc * ((2 * y + 1) / 28.f - 1.f) + ty;
  const float ix = ((gx + 1.f) * 28.f - 1.f) * 0.5f, iy = ((gy + 1.f) * 28.f - 1.f) * 0.5f;
  const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  const float fx = ix - x0, fy = iy - y0;
  const float* t = tmpl + c * 784;
  auto at = [&](int yy, int xx) { return (yy >= 0 && yy < 28 && xx >= 0 && xx < 28) ? t[yy * 28 + xx] : 0.f; };
  float v = (1.f - fy) * ((1.f - fx) * at(y0, x0) + fx * at(y0, x0 + 1)) +
            fy * ((1.f - fx) * at(y0 + 1, x0) + fx * at(y0 + 1, x0 + 1));
  const float un = unif(hash3(seed, u, 5u + (unsigned)px));
  v = v * contrast + noise * un * un * un;
  img[idx] = (uint8_t)__float2int_rn(fminf(fmaxf(v, 0.f), 1.f) * 255.f);
  if (px == 0) lab[im] = c;
}

}  // namespace

// ===========================================================================
// C ABI (loaded with ctypes by pytorch_operator_amd/ops/_native.py).  Every
// launcher validates the shapes its grid assumes before touching the GPU.
// Returns hipSuccess (0) or a hipError_t / -1 for a host-side shape error.
// ===========================================================================
#define PTO_CHECK_B(B) do { if ((B) <= 0 || (B) > (1 << 20)) return -1; } while (0)

extern "C" {

// Synthetic MNIST: n images [n][784] uint8 + int32 labels from the 10 class templates
// tmpl [10][28][28] fp32 (synth_mnist_kernel).
int pto_mnist_synth(const float* tmpl, void* img, int* lab, int n, unsigned seed, float noise, void* stream) {
  if (tmpl == nullptr || img == nullptr || lab == nullptr || n <= 0 || n > (1 << 24)) return -1;
  const long total = (long)n * 784;
  hipLaunchKernelGGL(synth_mnist_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     tmpl, (uint8_t*)img, lab, n, seed, noise);
  return (int)hipGetLastError();
}


void pto_set_debug_buffer(void* p) {
  g_dbg = reinterpret_cast<u64*>(p);
  g_dbg_slot = 0;
}

int pto_mnist_conv1_fwd(const void* x, int is_u8, const int* labels, const int* perm,
                        const int* cursor, int host_offset, int n_total, float scale,
                        float shift, const float* w, const float* bias, float* a1, uint8_t* idx1,
                        int B, float* zero_ptr, int zero_n, float* xn_out, int* lab_out,
                        void* stream) {
  PTO_CHECK_B(B);
  if (perm != nullptr && n_total <= 0) return -1;
  if (lab_out != nullptr && labels == nullptr) return -1;
  const BatchSrc src = make_src(x, is_u8, labels, perm, cursor, host_offset, n_total, scale, shift);
  const int blocks = (B * 2880 + 255) / 256;
  hipLaunchKernelGGL(conv1_fwd_pool_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     src, w, bias, a1, idx1, B, zero_ptr, zero_n, xn_out, lab_out, dbg_next());
  return (int)hipGetLastError();
}

int pto_mnist_conv2_fwd(const float* a1, const float* w, const float* bias, float* a2,
                        uint8_t* idx2, int B, void* stream) {
  PTO_CHECK_B(B);
  if ((((uintptr_t)a2) & 7) || (((uintptr_t)idx2) & 1)) return -2;  // 8-byte / 2-byte pair stores
  hipLaunchKernelGGL(conv2_fwd_pool_kernel, dim3(4, B), dim3(AB_NT), 0, (hipStream_t)stream,
                     a1, w, bias, a2, idx2, B, dbg_next());
  return (int)hipGetLastError();
}

int pto_mnist_conv12_fwd(const void* x, int is_u8, const int* labels, const int* perm,
                         const int* cursor, int host_offset, int n_total, float scale,
                         float shift, const float* w1, const float* b1, const float* w2,
                         const float* b2, float* a1, uint8_t* idx1, float* xn_out, int* lab_out,
                         float* a2, uint8_t* idx2, int B, const uint8_t* stg_x, const int* stg_lab,
                         const int* stg_tag, void* stream) {
  PTO_CHECK_B(B);
  if (B > 65535) return -1;  // grid y
  if (perm != nullptr && n_total <= 0) return -1;
  if (lab_out != nullptr && labels == nullptr) return -1;
  if ((((uintptr_t)w2) & 15) || (((uintptr_t)a1) & 15) || (((uintptr_t)idx1) & 15) || (((uintptr_t)a2) & 7) ||
      (((uintptr_t)idx2) & 1))
    return -2;  // a1 / idx1: 16-byte, a2: 8-byte, idx2: 2-byte stores
  // staged batches exist only for uint8 sources walked by a device cursor
  if (stg_x != nullptr && (stg_lab == nullptr || stg_tag == nullptr || cursor == nullptr || perm == nullptr ||
                           !is_u8 || labels == nullptr))
    return -1;
  const BatchSrc src = make_src(x, is_u8, labels, perm, cursor, host_offset, n_total, scale, shift);
  hipLaunchKernelGGL(conv12_fwd_kernel, dim3(4, B), dim3(AB_NT), 0, (hipStream_t)stream, src, w1, b1, w2, b2,
                     a1, idx1, xn_out, lab_out, a2, idx2, B, stg_x, stg_lab, stg_tag, dbg_next());
  return (int)hipGetLastError();
}

int pto_mnist_fc1_fwd(const float* x, const float* w, const float* bias, float* h, int B,
                      void* stream) {
  PTO_CHECK_B(B);
  if ((((uintptr_t)x) | ((uintptr_t)w)) & 15) return -2;  // float4 loads
  hipLaunchKernelGGL(fc1_fwd_kernel<1>, dim3(32, (B + 15) / 16), dim3(640), 0,
                     (hipStream_t)stream, x, w, bias, h, B, dbg_next());
  return (int)hipGetLastError();
}

int pto_mnist_fc1_ks() { return FC1_KS; }
// conv_bwd4's dynamic LDS (bytes): not in the code object's metadata (tests/test_kernel_resources.py)
int pto_mnist_conv_bwd4_lds() { return G_LDS * (int)sizeof(float); }

// Split-K fc1: pre-activation partials to parts[KS][B][500], the bias (may be null) added to
// parts[0] (head_kernel / fc1_bwd_head finish h = relu(parts[0] + parts[1])).
int pto_mnist_fc1_fwd_parts(const float* x, const float* w, const float* bias, float* parts, int B, void* stream) {
  PTO_CHECK_B(B);
  if ((((uintptr_t)x) | ((uintptr_t)w) | ((uintptr_t)parts)) & 15) return -2;
  hipLaunchKernelGGL(fc1_fwd_kernel<FC1_KS>, dim3(32, (B + 15) / 16, FC1_KS), dim3(640 / FC1_KS), 0,
                     (hipStream_t)stream, x, w, bias, parts, B, dbg_next());
  return (int)hipGetLastError();
}

int pto_mnist_head(const float* h, const float* w2, const float* b2, const int* lab, int B,
                   float grad_scale, float loss_scale, float* dlogits, float* dh, float* logp,
                   float* per_sample, float* stats, const float* hp2, float* h_out, void* stream) {
  PTO_CHECK_B(B);
  if (lab == nullptr) return -1;
  if (hp2 != nullptr && h_out == nullptr) return -1;
  if ((((uintptr_t)h) | ((uintptr_t)w2) | ((uintptr_t)dh) | ((uintptr_t)hp2) | ((uintptr_t)h_out)) & 15)
    return -2;  // float4 rows
  if (stats == nullptr)
    hipLaunchKernelGGL(head_kernel<1>, dim3(B), dim3(64), 0, (hipStream_t)stream, h, w2, b2, lab,
                       B, grad_scale, loss_scale, dlogits, dh, logp, per_sample, stats, hp2,
                       h_out, dbg_next());
  else
    hipLaunchKernelGGL(head_kernel<4>, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, h,
                       w2, b2, lab, B, grad_scale, loss_scale, dlogits, dh, logp, per_sample,
                       stats, hp2, h_out, dbg_next());
  return (int)hipGetLastError();
}

static int fc1_bwd_launch(const Fc1Bwd& a, void* stream) {
  const int B = a.B;
  PTO_CHECK_B(B);
  if (a.jobs <= 0 || a.jobs > 7) return -1;
  if (a.gw1 == nullptr || a.gb1 == nullptr || a.gw2 == nullptr || a.gb2 == nullptr) return -1;
  if ((a.jobs & 2) && a.dz2 == nullptr && a.dpool == nullptr) return -1;  // job 2 writes one of them
  if ((((uintptr_t)a.dh) | ((uintptr_t)a.gw1)) & 15) return -2;  // float4 dh rows (job 2), dW_fc1 stores
  if (a.xp.base[0] != nullptr) {
    if (a.xp.world < 2 || a.xp.world > 8 || a.xp.rank < 0 || a.xp.rank >= a.xp.world || a.xp.shard4 <= 0 ||
        a.xp.w1_f4 < 0 || a.xp.w1_f4 + 100000 > a.xp.shard4 * a.xp.world)
      return -1;
    for (int q = 0; q < a.xp.world; ++q)
      if (a.xp.base[q] == nullptr) return -1;
  }
  int nst = 0;
  if (a.stage_x != nullptr) {
    if (a.nsrc.perm == nullptr || a.nsrc.cursor == nullptr || a.nsrc.labels == nullptr || !a.nsrc.is_u8 ||
        a.stage_lab == nullptr || a.stage_tag == nullptr || a.nsrc.n_total <= 0 ||
        ((((uintptr_t)a.nsrc.x) | ((uintptr_t)a.stage_x)) & 15))
      return -1;
    nst = (B + 3) / 4;
  }
  const int blocks = ((a.jobs & 1) ? E_NJ1 : 0) + ((a.jobs & 2) ? ((B + 15) / 16) * 50 : 0) +
                     ((a.jobs & 4) ? E_NJ3 : 0) + nst;
  hipLaunchKernelGGL(fc1_bwd_kernel, dim3(blocks), dim3(E_NT), 0, (hipStream_t)stream, a, dbg_next());
  return (int)hipGetLastError();
}

// fc1_bwd that also pushes dW_fc1 into the xGMI owners' receive buffers (xp_bases: `world`
// device addresses in rank order, pto_xar_push_info), every job.
int pto_mnist_fc1_bwd_push(const float* dh, const float* a2, const uint8_t* idx2, const float* w1,
                           const float* dlog, const float* h, float* gw1, float* gb1, float* gw2,
                           float* gb2, float* dz2, const float* per_sample, float* stats,
                           float loss_scale, int B, void* const* xp_bases, int xp_rank, int xp_world,
                           long xp_shard4, long xp_w1_f4, const int* xp_err, float* dpool, void* stream) {
  Fc1Bwd a{};
  a.dpool = dpool;
  if (xp_bases == nullptr || xp_world < 2 || xp_world > 8) return -1;
  for (int q = 0; q < xp_world; ++q) a.xp.base[q] = static_cast<char*>(xp_bases[q]);
  a.xp.rank = xp_rank; a.xp.world = xp_world; a.xp.shard4 = xp_shard4; a.xp.w1_f4 = xp_w1_f4;
  a.xp.err = xp_err;
  a.dh = dh; a.a2 = a2; a.idx2 = idx2; a.w1 = w1; a.dlog = dlog; a.h = h;
  a.gw1 = gw1; a.gb1 = gb1; a.gw2 = gw2; a.gb2 = gb2; a.dz2 = dz2;
  a.per_sample = per_sample; a.stats = stats; a.loss_scale = loss_scale; a.jobs = 7; a.B = B;
  return fc1_bwd_launch(a, stream);
}

int pto_mnist_fc1_bwd(const float* dh, const float* a2, const uint8_t* idx2, const float* w1,
                      const float* dlog, const float* h, float* gw1, float* gb1, float* gw2,
                      float* gb2, float* dz2, const float* per_sample, float* stats,
                      float loss_scale, int jobs, int B, float* dpool, void* stream) {
  Fc1Bwd a{};
  a.dpool = dpool;
  a.dh = dh; a.a2 = a2; a.idx2 = idx2; a.w1 = w1; a.dlog = dlog; a.h = h;
  a.gw1 = gw1; a.gb1 = gb1; a.gw2 = gw2; a.gb2 = gb2; a.dz2 = dz2;
  a.per_sample = per_sample; a.stats = stats; a.loss_scale = loss_scale; a.jobs = jobs; a.B = B;
  return fc1_bwd_launch(a, stream);
}

// fc1_bwd (jobs: 7, or 6 when the tail computes dW_fc1) + next-batch staging blocks.
int pto_mnist_fc1_bwd_stage(const float* dh, const float* a2, const uint8_t* idx2, const float* w1,
                            const float* dlog, const float* h, float* gw1, float* gb1, float* gw2,
                            float* gb2, float* dz2, const float* per_sample, float* stats,
                            float loss_scale, int B, const void* nx, const int* nlabels, const int* nperm,
                            const int* ncursor, int n_total, int stage_adv, int jobs, uint8_t* stage_x,
                            int* stage_lab, int* stage_tag, float* dpool, void* stream) {
  Fc1Bwd a{};
  a.dpool = dpool;
  a.dh = dh; a.a2 = a2; a.idx2 = idx2; a.w1 = w1; a.dlog = dlog; a.h = h;
  a.gw1 = gw1; a.gb1 = gb1; a.gw2 = gw2; a.gb2 = gb2; a.dz2 = dz2;
  a.per_sample = per_sample; a.stats = stats; a.loss_scale = loss_scale; a.jobs = jobs; a.B = B;
  if ((jobs & 6) != 6) return -1;  // staging rides with the dz2 and fc2 jobs
  if (stage_x == nullptr) return -1;
  a.nsrc = make_src(nx, 1, nlabels, nperm, ncursor, 0, n_total, 1.f, 0.f);
  a.stage_adv = stage_adv;
  a.stage_x = stage_x;
  a.stage_lab = stage_lab;
  a.stage_tag = stage_tag;
  return fc1_bwd_launch(a, stream);
}

int pto_mnist_conv_bwd(const float* dz2, const float* w2, const float* a1, const uint8_t* idx1,
                       const float* xn, float* gw2, float* gb2, float* gw1, float* gb1,
                       float* dz1_out, int slab_stride, int B, void* stream) {
  PTO_CHECK_B(B);
  if (B > 65535 || slab_stride < 0) return -1;
  // the slab path writes dW_conv2 as float4: row starts and gw2 + 544-float offsets aligned
  if (slab_stride > 0 && (slab_stride % 4 != 0 || (reinterpret_cast<uintptr_t>(gw2) & 15) != 0)) return -2;
  static std::atomic<unsigned> attr_set{0};
  const int rc = set_max_lds(conv_bwd_kernel, F_LDS * (int)sizeof(float), attr_set);
  if (rc != 0) return rc;
  hipLaunchKernelGGL(conv_bwd_kernel, dim3(4, B), dim3(F_NT), F_LDS * sizeof(float), (hipStream_t)stream, dz2,
                     w2, a1, idx1, xn, gw2, gb2, gw1, gb1, dz1_out, slab_stride, B, dbg_next());
  return (int)hipGetLastError();
}

// Conv-grad slab reduction.  rows_big / [big_lo, big_hi) (floats, multiples of 4): the
// columns summed over rows_big rows (conv_bwd4's chunk rows); every other column over B.
static bool slab_rows_ok(int B, int n, int rows_big, int big_lo, int big_hi, SlabRows& sr) {
  if (rows_big <= 0 || rows_big > B || big_lo < 0 || big_hi < big_lo || big_hi > n || (big_lo & 3) || (big_hi & 3))
    return false;
  sr = SlabRows{B, rows_big, big_lo >> 2, big_hi >> 2};
  return true;
}

int pto_slab_reduce(const float* P, int B, int n, int stride, float* out, int rows_big, int big_lo,
                    int big_hi, void* stream) {
  PTO_CHECK_B(B);
  if (n <= 0 || (n & 3) || (stride & 3) || stride < n) return -1;
  if ((((uintptr_t)P) | ((uintptr_t)out)) & 15) return -2;
  SlabRows sr;
  if (!slab_rows_ok(B, n, rows_big, big_lo, big_hi, sr)) return -1;
  const int blocks = (n / 4 + SR_COLS - 1) / SR_COLS;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, P, sr, n,
                     stride, out, dbg_next());
  return (int)hipGetLastError();
}

int pto_sgd_momentum(float* p, const float* g, float* buf, long n, float lr, float momentum,
                     float dampening, float wd, float grad_scale, int nesterov, int first_step,
                     int* step_counter, void* stream) {
  if (n <= 0) return -1;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)buf) & 15) return -2;  // float4 path
  long v = (n >> 2) + 4;
  int blocks = (int)((v + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  const SgdHyper hy{lr, momentum, dampening, wd, grad_scale, nesterov, first_step};
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p, g,
                     buf, n, hy, step_counter);
  return (int)hipGetLastError();
}

int pto_slab_reduce_sgd(const float* P, int B, int n, int stride, float* gout, float* p,
                        float* buf, float lr, float momentum, float dampening, float wd,
                        float grad_scale, int nesterov, int first_step, int* step_counter,
                        float* p2, const float* g2, float* buf2, int n2, int rows_big, int big_lo,
                        int big_hi, void* stream) {
  PTO_CHECK_B(B);
  if (n <= 0 || (n & 3) || (stride & 3) || stride < n) return -1;
  if (n2 < 0 || (n2 & 3) || (n2 > 0 && (p2 == nullptr || g2 == nullptr || buf2 == nullptr)))
    return -1;
  if ((((uintptr_t)P) | ((uintptr_t)gout) | ((uintptr_t)p) | ((uintptr_t)buf) |
       ((uintptr_t)p2) | ((uintptr_t)g2) | ((uintptr_t)buf2)) & 15)
    return -2;
  SlabRows sr;
  if (!slab_rows_ok(B, n, rows_big, big_lo, big_hi, sr)) return -1;
  const int red_blocks = (n / 4 + SR_COLS - 1) / SR_COLS;
  const int blocks = red_blocks + (n2 / 4 + 255) / 256;
  const SgdHyper hy{lr, momentum, dampening, wd, grad_scale, nesterov, first_step};
  const TailW1 tw{};
  hipLaunchKernelGGL(slab_reduce_sgd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, P,
                     sr, n, stride, gout, p, buf, hy, step_counter, p2, g2, buf2, n2, red_blocks, tw, dbg_next());
  return (int)hipGetLastError();
}

// The tail with fc1.weight's gradient computed in it (TailW1): as pto_slab_reduce_sgd, plus
// dW_fc1 = dh^T . a2 (dh [B][500], a2 [B][800]) and SGD on w1p/w1m [400000 + 500: fc1.weight
// then fc1.bias] (w1g: optional gradient output of the same layout).  The plain SGD range
// p2/g2/buf2 then covers only the parameters after fc1.bias.
int pto_slab_reduce_sgd_w1(const float* P, int B, int n, int stride, float* gout, float* p,
                           float* buf, float lr, float momentum, float dampening, float wd,
                           float grad_scale, int nesterov, int first_step, int* step_counter,
                           float* p2, const float* g2, float* buf2, int n2, int rows_big, int big_lo,
                           int big_hi, const float* dh, const float* a2, float* w1p, float* w1m, float* w1g,
                           void* stream) {
  PTO_CHECK_B(B);
  if (n <= 0 || (n & 3) || (stride & 3) || stride < n) return -1;
  if (n2 < 0 || (n2 & 3) || (n2 > 0 && (p2 == nullptr || g2 == nullptr || buf2 == nullptr)))
    return -1;
  if (dh == nullptr || a2 == nullptr || w1p == nullptr || w1m == nullptr) return -1;
  if ((((uintptr_t)P) | ((uintptr_t)gout) | ((uintptr_t)p) | ((uintptr_t)buf) | ((uintptr_t)p2) |
       ((uintptr_t)g2) | ((uintptr_t)buf2) | ((uintptr_t)w1p) | ((uintptr_t)w1m) | ((uintptr_t)w1g)) & 15)
    return -2;
  SlabRows sr;
  if (!slab_rows_ok(B, n, rows_big, big_lo, big_hi, sr)) return -1;
  const int red_blocks = (n / 4 + SR_COLS - 1) / SR_COLS;
  const int blocks = T_W1_BLOCKS + red_blocks + (n2 / 4 + 255) / 256;
  const SgdHyper hy{lr, momentum, dampening, wd, grad_scale, nesterov, first_step};
  TailW1 tw{};
  tw.dh = dh; tw.a2 = a2; tw.p = w1p; tw.m = w1m; tw.g = w1g; tw.B = B; tw.blocks = T_W1_BLOCKS;
  hipLaunchKernelGGL(slab_reduce_sgd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, P,
                     sr, n, stride, gout, p, buf, hy, step_counter, p2, g2, buf2, n2, red_blocks, tw, dbg_next());
  return (int)hipGetLastError();
}

// The tail of the fused-head step: as pto_slab_reduce_sgd_w1 (no plain SGD range) plus fc1_bwd's
// job 3 -- dW_fc2 = dlog^T . h, db_fc2 and their SGD on fc2.weight (p2w/m2w, [10][500]) and
// fc2.bias (pb2/mb2), optional gradients g2w/gb2, and stats = (sum(loss) * loss_scale, #correct)
// from per_sample.
int pto_mnist_tail(const float* P, int B, int n, int stride, float* gout, float* p, float* buf, float lr,
                   float momentum, float dampening, float wd, float grad_scale, int nesterov, int first_step,
                   int* step_counter, int rows_big, int big_lo, int big_hi, const float* dh, const float* a2,
                   float* w1p, float* w1m, float* w1g, const float* dlog, const float* h, const float* per_sample,
                   float* stats, float loss_scale, float* p2w, float* m2w, float* g2w, float* pb2, float* mb2,
                   float* gb2, void* stream) {
  PTO_CHECK_B(B);
  if (n <= 0 || (n & 3) || (stride & 3) || stride < n) return -1;
  if (dh == nullptr || a2 == nullptr || w1p == nullptr || w1m == nullptr || dlog == nullptr || h == nullptr ||
      p2w == nullptr || m2w == nullptr || pb2 == nullptr || mb2 == nullptr || per_sample == nullptr || stats == nullptr)
    return -1;
  if ((((uintptr_t)P) | ((uintptr_t)gout) | ((uintptr_t)p) | ((uintptr_t)buf) | ((uintptr_t)w1p) |
       ((uintptr_t)w1m) | ((uintptr_t)w1g)) & 15)
    return -2;
  SlabRows sr;
  if (!slab_rows_ok(B, n, rows_big, big_lo, big_hi, sr)) return -1;
  const int red_blocks = (n / 4 + SR_COLS - 1) / SR_COLS;
  const int blocks = T_W1_BLOCKS + T_FC2_BLOCKS + red_blocks;
  const SgdHyper hy{lr, momentum, dampening, wd, grad_scale, nesterov, first_step};
  TailW1 tw{};
  tw.dh = dh; tw.a2 = a2; tw.p = w1p; tw.m = w1m; tw.g = w1g; tw.B = B; tw.blocks = T_W1_BLOCKS + T_FC2_BLOCKS;
  tw.fc2 = 1; tw.dlog = dlog; tw.h = h; tw.per_sample = per_sample; tw.stats = stats; tw.loss_scale = loss_scale;
  tw.p2 = p2w; tw.m2 = m2w; tw.g2 = g2w; tw.pb2 = pb2; tw.mb2 = mb2; tw.gb2 = gb2;
  hipLaunchKernelGGL(slab_reduce_sgd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, P,
                     sr, n, stride, gout, p, buf, hy, step_counter, nullptr, nullptr, nullptr, 0, red_blocks, tw,
                     dbg_next());
  return (int)hipGetLastError();
}

// The fused-head step's gradients for DDP over RCCL (round 6): pto_mnist_tail's tiles and slab
// reduction with every gradient stored and no parameter touched -- gout [n] (the conv bucket,
// reduced from the slab), w1g [400000 + 500] (fc1.weight, fc1.bias), g2w [10][500], gb2 [10] (fc2)
// and the loss statistics.  The step counter is left to the SGD launch after the all-reduces.
int pto_mnist_tail_grads(const float* P, int B, int n, int stride, float* gout, int rows_big, int big_lo,
                         int big_hi, const float* dh, const float* a2, float* w1g, const float* dlog,
                         const float* h, const float* per_sample, float* stats, float loss_scale, float* g2w,
                         float* gb2, void* stream) {
  PTO_CHECK_B(B);
  if (n <= 0 || (n & 3) || (stride & 3) || stride < n) return -1;
  if (gout == nullptr || dh == nullptr || a2 == nullptr || w1g == nullptr || dlog == nullptr || h == nullptr ||
      per_sample == nullptr || stats == nullptr || g2w == nullptr || gb2 == nullptr)
    return -1;
  if ((((uintptr_t)P) | ((uintptr_t)gout) | ((uintptr_t)w1g)) & 15) return -2;
  SlabRows sr;
  if (!slab_rows_ok(B, n, rows_big, big_lo, big_hi, sr)) return -1;
  const int red_blocks = (n / 4 + SR_COLS - 1) / SR_COLS;
  const int blocks = T_W1_BLOCKS + T_FC2_BLOCKS + red_blocks;
  const SgdHyper hy{};
  TailW1 tw{};
  tw.dh = dh; tw.a2 = a2; tw.g = w1g; tw.B = B; tw.blocks = T_W1_BLOCKS + T_FC2_BLOCKS;
  tw.fc2 = 1; tw.dlog = dlog; tw.h = h; tw.per_sample = per_sample; tw.stats = stats; tw.loss_scale = loss_scale;
  tw.g2 = g2w; tw.gb2 = gb2; tw.grad_only = 1;
  hipLaunchKernelGGL(slab_reduce_sgd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, P,
                     sr, n, stride, gout, nullptr, nullptr, hy, nullptr, nullptr, nullptr, nullptr, 0, red_blocks, tw,
                     dbg_next());
  return (int)hipGetLastError();
}

// fc1_bwd with the head fused in (fc1_bwd_head_kernel): dz2 from the split-K fc1 partials hp0/hp1;
// publishes h_out, dh_out [B][500], dlog_out [B][10], per_sample [B][2]; with stage_x, also the
// next-batch staging blocks (as pto_mnist_fc1_bwd_stage).
int pto_mnist_fc1_bwd_head(const float* hp0, const float* hp1, const float* w2, const float* b2,
                           const int* lab, const float* a2, const uint8_t* idx2, const float* w1, float* dz2,
                           float* h_out, float* dh_out, float* dlog_out, float* per_sample, float grad_scale, int B,
                           const void* nx, const int* nlabels, const int* nperm, const int* ncursor, int n_total,
                           int stage_adv, uint8_t* stage_x, int* stage_lab, int* stage_tag, float* dpool,
                           void* stream) {
  PTO_CHECK_B(B);
  if (hp0 == nullptr || hp1 == nullptr || w2 == nullptr || b2 == nullptr || lab == nullptr ||
      a2 == nullptr || idx2 == nullptr || w1 == nullptr || (dz2 == nullptr && dpool == nullptr) ||
      h_out == nullptr || dh_out == nullptr || dlog_out == nullptr || per_sample == nullptr)
    return -1;
  if ((((uintptr_t)hp0) | ((uintptr_t)hp1) | ((uintptr_t)w2) | ((uintptr_t)h_out) | ((uintptr_t)dh_out)) & 15)
    return -2;  // float4 rows
  Fc1BwdHead a{};
  a.hp0 = hp0; a.hp1 = hp1; a.w2 = w2; a.b2 = b2; a.lab = lab; a.a2 = a2; a.idx2 = idx2; a.w1 = w1;
  a.dz2 = dz2; a.dpool = dpool; a.h_out = h_out; a.dh_out = dh_out; a.dlog_out = dlog_out; a.per_sample = per_sample;
  a.grad_scale = grad_scale; a.B = B;
  int nst = 0;
  if (stage_x != nullptr) {
    if (nperm == nullptr || ncursor == nullptr || nlabels == nullptr || stage_lab == nullptr || stage_tag == nullptr ||
        n_total <= 0 || ((((uintptr_t)nx) | ((uintptr_t)stage_x)) & 15))
      return -1;
    a.nsrc = make_src(nx, 1, nlabels, nperm, ncursor, 0, n_total, 1.f, 0.f);
    a.stage_adv = stage_adv;
    a.stage_x = stage_x;
    a.stage_lab = stage_lab;
    a.stage_tag = stage_tag;
    nst = (B + 3) / 4;
  }
  const int blocks = ((B + 15) / 16) * 50 + nst;
  hipLaunchKernelGGL(fc1_bwd_head_kernel, dim3(blocks), dim3(E_NT), 0, (hipStream_t)stream, a, dbg_next());
  return (int)hipGetLastError();
}

// conv backward, dW_conv2 over 4-sample chunks (conv_bwd4_kernel): slab rows 0..ceil(B/4)-1
// get the chunk partials of conv2.weight at row offset o_gw2; rows 0..B-1 the per-sample
// conv1.weight / conv1.bias / conv2.bias partials at o_gw1 / o_gb1 / o_gb2.
int pto_mnist_conv_bwd4(const float* dpool, const uint8_t* idx2, const float* w2, const float* a1,
                        const uint8_t* idx1, const float* xn, float* slab, int stride, int o_gw2, int o_gb2,
                        int o_gw1, int o_gb1, int B, void* stream) {
  PTO_CHECK_B(B);
  if (4 * ((B + 3) / 4) > 65535) return -1;  // grid y
  if (dpool == nullptr || idx2 == nullptr || w2 == nullptr || a1 == nullptr || idx1 == nullptr || xn == nullptr)
    return -1;
  // 16-byte staging loads (idx2: 4-byte)
  if ((stride & 3) || (o_gw2 & 3) || ((((uintptr_t)slab) | ((uintptr_t)dpool) | ((uintptr_t)w2) | ((uintptr_t)a1) |
                                       ((uintptr_t)idx1) | ((uintptr_t)xn)) & 15) || (((uintptr_t)idx2) & 3))
    return -2;
  if (o_gw2 < 0 || o_gb2 < 0 || o_gw1 < 0 || o_gb1 < 0 || o_gw2 + 25000 > stride || o_gb2 + 50 > stride ||
      o_gw1 + 500 > stride || o_gb1 + 20 > stride)
    return -1;
  static std::atomic<unsigned> attr_set{0};
  const int rc = set_max_lds(conv_bwd4_kernel, G_LDS * (int)sizeof(float), attr_set);
  if (rc != 0) return rc;
  const int nb = 4 * ((B + 3) / 4);
  hipLaunchKernelGGL(conv_bwd4_kernel, dim3(4, nb), dim3(F_NT), G_LDS * sizeof(float), (hipStream_t)stream,
                     dpool, idx2, w2, a1, idx1, xn, slab, stride, o_gw2, o_gb2, o_gw1, o_gb1, B, dbg_next());
  return (int)hipGetLastError();
}

}  // extern "C"
