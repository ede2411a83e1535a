// Attention kernel variants measured and rejected in rounds 2-4 (profiles/r3_attn_*,
// r4_attn_*): NOT part of the default libpto_hip.so.  tools/build_exp.sh links this file into its
// experiment libraries (pytorch_operator_amd/_lib/exp/*.so, loaded through PTO_HIP_LIB), where
// attention.hip's dispatcher reaches them through the weak pto_attn_exp_* entry points below
// (PTO_ATTN_FWD / PTO_ATTN_DQ / PTO_ATTN_DKDV or pto_attn_set_*_variant select them):
//   forward 9   8-wave ping-pong forward (attn_fwd8p_kernel; bit-identical to the default, slower)
//   dQ 8        8-wave compiler-scheduled dQ pass (attn_bwd_dq8_kernel; the pipelined pass 9 matches it)
//   dK/dV 2     software-pipelined 4-wave (3-deep Q/dO ring)                 -- slower
//   dK/dV 3     8-wave workgroup (S % 256 == 0)                               -- slower
//   dK/dV 4, 7  lean-register 4-wave, builtin / inline-asm LDS-DMA staging     -- 429 vs 314 us
//   dK/dV 6     a dV pass and a dK pass, two waves per SIMD each              -- slower
// tools/attn_variant_check.py compares them with the default passes on a GPU.
#include "../attention_common.h"

namespace {

// ------------------------------------------------ forward, 8-wave ping-pong workgroup
// attn_fwd8_kernel's barrier per K/V tile re-aligns the two waves of every SIMD each tile, so
// both run their QK^T MFMAs, then both their softmax (matrix pipe idle), then both P.V.  Here
// the younger half (waves 4-7) runs its loop rotated by one phase -- softmax(t), P.V(t),
// QK^T(t+1) -- against the older half's QK^T(t), softmax(t), P.V(t) between the same two
// barriers, so one wave's softmax issues under the other's MFMAs.  The rotated half reads
// K(t+1) while tile t is current: K/V tiles cycle through a 3-deep LDS ring (96 KB), stored two
// tiles ahead.  Numerics are those of attn_fwd8_kernel (same per-row operation order).
__global__ __launch_bounds__(NT8, 1) void attn_fwd8p_kernel(const bf16_t* __restrict__ q,
                                                           const bf16_t* __restrict__ k,
                                                           const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                           float* __restrict__ lse2, int B, int S, int Hq, int Hkv,
                                                           float c, int causal) {
  __shared__ u32x4 smem[6 * BN * CH];  // (K, V) x 3 (96 KB); the O staging image after the loop
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const bool rot = __builtin_amdgcn_readfirstlane(tid) >= NT8 / 2;  // wave-uniform
  if (rot) __builtin_amdgcn_s_setprio(1);
  const int G = Hq / Hkv, nqb = S / BM8;
  int bi = (int)blockIdx.x;
  const int hk = bi % Hkv;
  bi /= Hkv;
  const int hq = hk * G + bi % G;
  bi /= G;
  const int b = bi % B, qi = bi / B;
  const int qblk = causal ? nqb - 1 - qi : qi;
  const int q0w = qblk * BM8 + w * 32, qme = q0w + r;
  const size_t qstride = (size_t)Hq * D, kvstride = (size_t)Hkv * D;

  bf16x8 qf[NDS];
  {
    const bf16_t* qrow = q + ((size_t)b * S + qme) * qstride + (size_t)hq * D + 8 * h;
#pragma unroll
    for (int s = 0; s < NDS; ++s) qf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(qrow + 16 * s));
  }
  const bf16_t* kb = k + (size_t)b * S * kvstride + (size_t)hk * D;
  const bf16_t* vb = v + (size_t)b * S * kvstride + (size_t)hk * D;
  const int ntiles = causal ? (qblk * BM8 + BM8) / BN : S / BN;
  const int wtiles = causal ? (q0w + 31) / BN + 1 : ntiles;
  // ring slot base, opaque to the optimiser: otherwise it hoists every (slot, operand address)
  // combination out of the loop and spills them
  auto kbuf = [&](int t) {
    int off = (t % 3) * 2 * BN * CH;
    asm volatile("" : "+s"(off));
    return smem + off;
  };

  // K/V by LDS-DMA (no staging registers: both halves' loops sit at the register cap)
  glds_tile<BN, NT8>(kb, kvstride, smem, tid);
  glds_tile<BN, NT8>(vb, kvstride, smem + BN * CH, tid);
  if (ntiles > 1) {
    glds_tile<BN, NT8>(kb + (size_t)BN * kvstride, kvstride, smem + 2 * BN * CH, tid);
    glds_tile<BN, NT8>(vb + (size_t)BN * kvstride, kvstride, smem + 3 * BN * CH, tid);
  }
  __syncthreads();

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16();
  float m2 = -INFINITY, l = 0.f;
  f32x16 sacc[2];

  auto qk = [&](const u32x4* Ks, int r, int h) {
    __builtin_amdgcn_sched_barrier(0);  // keep the operand reads out of the previous phase
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {  // one 32-key half at a time: 32 operand registers, not 64
      bf16x8 a0[NDS];
#pragma unroll
      for (int s = 0; s < NDS; ++s) a0[s] = row_frag(Ks, 32 * kt + r, 2 * s + h);
      __builtin_amdgcn_sched_barrier(0);
      sacc[kt] = zero16();
#pragma unroll
      for (int s = 0; s < NDS; ++s) sacc[kt] = mfma(a0[s], qf[s], sacc[kt]);
    }
  };
  auto softmax_pv = [&](int t, const u32x4* Vs, int lane, int r, int h) {
    __builtin_amdgcn_sched_barrier(0);
    const int kv0 = t * BN;
    if (causal && kv0 + BN - 1 > q0w) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const int lim = qme - kv0 - kt * 32 - 4 * h;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i & 3) + 8 * (i >> 2) > lim) sacc[kt][i] = -INFINITY;
      }
    }
    float mx = max3(sacc[0][0], sacc[0][1], sacc[0][2]);
#pragma unroll
    for (int i = 3; i < 15; i += 2) mx = max3(mx, sacc[0][i], sacc[0][i + 1]);
    mx = max3(mx, sacc[0][15], sacc[1][0]);
#pragma unroll
    for (int i = 1; i < 15; i += 2) mx = max3(mx, sacc[1][i], sacc[1][i + 1]);
    mx = max3(mx, sacc[1][15], sacc[1][15]);
    mx = half_max(mx);
    const float mt = mx * c;
    if (__builtin_amdgcn_ballot_w64(mt > m2 + DEFER) != 0) {
      const float mnew = fmaxf(m2, mt);
      const float alpha = __builtin_amdgcn_exp2f(m2 - mnew);
      m2 = mnew;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) oacc[dt] *= alpha;
    }
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sacc[kt][i], c, -m2));
        sacc[kt][i] = p;
        rs += p;
      }
    l += rs;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      bf16x8 pb[2], vv[2][NDT];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) vv[s2][dt] = tr_frag(Vs, kt * 32 + 16 * s2, dt * 32, lane);
      pb[0] = acc_frag(sacc[kt], 0);
      pb[1] = acc_frag(sacc[kt], 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) oacc[dt] = mfma(vv[s2][dt], pb[s2], oacc[dt]);
    }
  };

  auto stage_next = [&](int t) {  // tile t+2 into the slot tile t-1 left (nobody reads it this round)
    if (t + 2 < ntiles) {
      u32x4* nk = kbuf(t + 2);
      glds_tile<BN, NT8>(kb + (size_t)(t + 2) * BN * kvstride, kvstride, nk, tid);
      glds_tile<BN, NT8>(vb + (size_t)(t + 2) * BN * kvstride, kvstride, nk + BN * CH, tid);
    }
  };
  // one loop per half (same trip count, one barrier per trip each): loop-invariant operand
  // addresses of the two orders then live in separate loops instead of all at once
  // (lane indices re-derived per half behind an optimisation barrier, for the same reason)
  if (!rot) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int rr = ln & 31, hh = ln >> 5;
#pragma nounroll
    for (int t = 0; t < ntiles; ++t) {
      stage_next(t);
      if (t < wtiles) {  // wave-uniform
        const u32x4* Ks = kbuf(t);
        qk(Ks, rr, hh);
        softmax_pv(t, Ks + BN * CH, ln, rr, hh);
      }
      __syncthreads();
    }
  } else {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int rr = ln & 31, hh = ln >> 5;
    if (wtiles > 0) qk(kbuf(0), rr, hh);
#pragma nounroll
    for (int t = 0; t < ntiles; ++t) {
      stage_next(t);
      if (t < wtiles) softmax_pv(t, kbuf(t) + BN * CH, ln, rr, hh);
      if (t + 1 < wtiles) qk(kbuf(t + 1), rr, hh);
      __syncthreads();
    }
  }
  l = half_sum(l);
  const float inv = 1.f / l;
  store_rows_T(oacc, inv, smem + w * 32 * CH, lane, o + ((size_t)b * S + q0w) * qstride + (size_t)hq * D, qstride);
  if (h == 0) lse2[((size_t)b * Hq + hq) * S + qme] = m2 + log2f(l);
}

// ------------------------------------------------- backward pass 1, 8-wave workgroup
// The dQ pass in the forward's 8-wave shape (256 query rows share each K/V tile, two waves
// per SIMD, kv head fastest in the block order, causal per-wave tile skip, younger half at
// priority 1).  Registers: the S and dP operand reads are issued per 32-key half as two
// 8-fragment groups so Q, dO, dQ^T and both chains fit the 256 of two waves per SIMD.
__global__ __launch_bounds__(NT8, 1) void attn_bwd_dq8_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout, const float* __restrict__ lse2,
    float* __restrict__ delta, bf16_t* __restrict__ dq, int B, int S, int Hq, int Hkv, float c, float scale,
    int causal) {
  __shared__ u32x4 smem[4 * BN * CH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  if (__builtin_amdgcn_readfirstlane(tid) >= NT8 / 2) __builtin_amdgcn_s_setprio(1);
  const int G = Hq / Hkv, nqb = S / BM8;
  int bi = (int)blockIdx.x;
  const int hk = bi % Hkv;
  bi /= Hkv;
  const int hq = hk * G + bi % G;
  bi /= G;
  const int b = bi % B, qi = bi / B;
  const int qblk = causal ? nqb - 1 - qi : qi;
  const int q0w = qblk * BM8 + w * 32, qme = q0w + r;
  const size_t qstride = (size_t)Hq * D, kvstride = (size_t)Hkv * D;

  bf16x8 qf[NDS], df[NDS];
  float dl;
  {
    const size_t off = ((size_t)b * S + qme) * qstride + (size_t)hq * D + 8 * h;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < NDS; ++s) {
      const u32x4 qq = *reinterpret_cast<const u32x4*>(q + off + 16 * s);
      const u32x4 dd = *reinterpret_cast<const u32x4*>(dout + off + 16 * s);
      const u32x4 oo = *reinterpret_cast<const u32x4*>(o + off + 16 * s);
      qf[s] = __builtin_bit_cast(bf16x8, qq);
      df[s] = __builtin_bit_cast(bf16x8, dd);
      const uint32_t dw[4] = {dd.x, dd.y, dd.z, dd.w}, ow[4] = {oo.x, oo.y, oo.z, oo.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        part = fmaf(bf2f(dw[e] & 0xffffu), bf2f(ow[e] & 0xffffu), part);
        part = fmaf(bf2f(dw[e] >> 16), bf2f(ow[e] >> 16), part);
      }
    }
    dl = half_sum(part);
  }
  const size_t srow = ((size_t)b * Hq + hq) * S + qme;
  const float lq = lse2[srow];
  if (h == 0) delta[srow] = dl;

  const bf16_t* kb = k + (size_t)b * S * kvstride + (size_t)hk * D;
  const bf16_t* vb = v + (size_t)b * S * kvstride + (size_t)hk * D;
  const int ntiles = causal ? (qblk * BM8 + BM8) / BN : S / BN;
  const int wtiles = causal ? (q0w + 31) / BN + 1 : ntiles;
  // K/V tiles by LDS-DMA: no staging registers (the register-staged form spilled in the loop)
  glds_tile<BN, NT8>(kb, kvstride, smem, tid);
  glds_tile<BN, NT8>(vb, kvstride, smem + BN * CH, tid);
  __syncthreads();

  f32x16 dacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dacc[dt] = zero16();

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    int boff = cur * 2 * BN * CH;
    asm volatile("" : "+s"(boff));  // opaque: one set of operand addresses, not one per buffer
    const u32x4* Ks = smem + boff;
    const u32x4* Vs = Ks + BN * CH;
    const int kv0 = t * BN;
    const bool more = t + 1 < ntiles;
    if (more) {  // into the buffer tile t-1 left; lands under this tile's MFMAs
      u32x4* nk = smem + (cur ^ 1) * 2 * BN * CH;
      glds_tile<BN, NT8>(kb + (size_t)(t + 1) * BN * kvstride, kvstride, nk, tid);
      glds_tile<BN, NT8>(vb + (size_t)(t + 1) * BN * kvstride, kvstride, nk + BN * CH, tid);
    }
    if (t < wtiles) {  // wave-uniform
      const bool diag = causal && kv0 + BN - 1 > q0w;
      // this lane's row-read chunk XOR (xo: chunk 2s+h of row r sits at (2s) ^ cx), re-derived
      // per tile behind an optimisation barrier: hoisted, the eight per-k-step addresses were
      // spilled and their reloads' vmcnt(0) waited for the K/V staging loads every tile
      int cx = h ^ (((r & 3) << 2) | ((r >> 2) & 3));
      asm volatile("" : "+v"(cx));
      const u32x4* Kr = Ks + r * CH;
      const u32x4* Vr = Vs + r * CH;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f32x16 sa = zero16(), pa = zero16();
        {
          bf16x8 ka[NDS];
#pragma unroll
          for (int s = 0; s < NDS; ++s) ka[s] = __builtin_bit_cast(bf16x8, Kr[kt * 32 * CH + ((2 * s) ^ cx)]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s = 0; s < NDS; ++s) sa = mfma(ka[s], qf[s], sa);
        }
        {
          bf16x8 va[NDS];
#pragma unroll
          for (int s = 0; s < NDS; ++s) va[s] = __builtin_bit_cast(bf16x8, Vr[kt * 32 * CH + ((2 * s) ^ cx)]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s = 0; s < NDS; ++s) pa = mfma(va[s], df[s], pa);
        }
        const int lim = qme - kv0 - kt * 32 - 4 * h;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float p = __builtin_amdgcn_exp2f(fmaf(sa[i], c, -lq));
          if (diag && (i & 3) + 8 * (i >> 2) > lim) p = 0.f;
          sa[i] = p * (pa[i] - dl);
        }
        // dQ^T += K^T dS^T, one 16-key k-step at a time (16 operand registers, not 32: the
        // kernel is at the 256 of two waves per SIMD)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 kk[NDT];
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) kk[dt] = tr_frag(Ks, kt * 32 + 16 * s2, dt * 32, lane);
          const bf16x8 db = acc_frag(sa, s2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) dacc[dt] = mfma(kk[dt], db, dacc[dt]);
        }
      }
    }
    __syncthreads();
  }
  store_rows_T(dacc, scale, smem + w * 32 * CH, lane, dq + ((size_t)b * S + q0w) * qstride + (size_t)hq * D, qstride);
}

// ------------------------------------- backward pass 2, lean registers (dK, dV)
// attn_bwd_dkdv_kernel's loop needed more than the 256 architectural VGPRs (K/V fragments, both
// row-operand sets, both transposed-operand sets and the staging registers live at once), so the
// compiler parked values in AGPRs and moved them back every tile (64 v_accvgpr_read + 32
// v_accvgpr_write per 32 MFMAs, on a one-wave-per-SIMD kernel where every VALU slot is MFMA
// issue time).  Here the operand sets are read one chain at a time (S, dP, dV^T, dK^T), the
// Q / dO tiles arrive by LDS-DMA (no staging registers, no per-tile store address math), the
// causal mask is a uniform branch taken on diagonal tiles only, and waves skip the query
// tiles wholly above their keys.
template <bool ASM_DMA>
__global__ __launch_bounds__(NT, 1) void attn_bwd_dkdv2_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int B, int S, int Hq, int Hkv, float c, float scale,
    int causal) {
  __shared__ u32x4 qd[2][2 * QT * CH];               // [buf][Q | dO] (32 KB); dK/dV epilogue
  __shared__ __align__(16) float stat[2][2 * QT];    // [buf][lse2 | delta]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int kblk = (int)blockIdx.x / (B * Hkv), bh = (int)blockIdx.x % (B * Hkv);
  const int b = bh / Hkv, hk = bh % Hkv, G = Hq / Hkv;
  const int k0w = kblk * BK + w * 32, kme = k0w + r;
  const size_t qstride = (size_t)Hq * D, kvstride = (size_t)Hkv * D;

  bf16x8 kf[NDS], vf[NDS];
  {
    const size_t off = ((size_t)b * S + kme) * kvstride + (size_t)hk * D + 8 * h;
#pragma unroll
    for (int s = 0; s < NDS; ++s) {
      kf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(k + off + 16 * s));
      vf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(v + off + 16 * s));
    }
  }
  const int qt0 = causal ? (kblk * BK) / QT : 0;
  const int nqt = S / QT - qt0;
  const int ntiles = G * nqt;
  const int wskip = causal ? __builtin_amdgcn_readfirstlane(w) : 0;  // first live tile: qt0 + w

  auto fetch = [&](int t, int buf) {
    const int g = t / nqt, qt = qt0 + t % nqt, hq = hk * G + g;
    const size_t off = ((size_t)b * S + (size_t)qt * QT) * qstride + (size_t)hq * D;
    if constexpr (ASM_DMA) {
      glds_tile_asm<QT, NT>(q + off, qstride, qd[buf], tid);
      glds_tile_asm<QT, NT>(dout + off, qstride, qd[buf] + QT * CH, tid);
    } else {
      glds_tile<QT, NT>(q + off, qstride, qd[buf], tid);
      glds_tile<QT, NT>(dout + off, qstride, qd[buf] + QT * CH, tid);
    }
    if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0) {
      const size_t srow = ((size_t)b * Hq + hq) * S + (size_t)qt * QT;
      const float* src = (lane < 32 ? lse2 : delta) + srow + (lane & 31);
      if constexpr (ASM_DMA) glds_dword_asm(src, stat[buf]);
      else __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)stat[buf], 4, 0, 0);
    }
  };
  fetch(0, 0);
  if constexpr (ASM_DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x16 dka[NDT], dva[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    dka[dt] = zero16();
    dva[dt] = zero16();
  }
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) fetch(t + 1, cur ^ 1);  // lands under this tile's MFMAs
    const int qtl = t % nqt;
    if (qtl >= wskip) {  // wave-uniform
      int boff = cur * 2 * QT * CH;
      asm volatile("" : "+s"(boff));  // one set of operand addresses for both buffers
      const u32x4* Qs = &qd[0][0] + boff;
      const u32x4* Ds = Qs + QT * CH;
      const int q0 = (qt0 + qtl) * QT;
      f32x16 sa, pa;
      {
        bf16x8 qa[NDS];
#pragma unroll
        for (int s = 0; s < NDS; ++s) qa[s] = row_frag(Qs, r, 2 * s + h);
        __builtin_amdgcn_sched_barrier(0);
        sa = zero16();
#pragma unroll
        for (int s = 0; s < NDS; ++s) sa = mfma(qa[s], kf[s], sa);
      }
      {
        bf16x8 da[NDS];
#pragma unroll
        for (int s = 0; s < NDS; ++s) da[s] = row_frag(Ds, r, 2 * s + h);
        __builtin_amdgcn_sched_barrier(0);
        pa = zero16();
#pragma unroll
        for (int s = 0; s < NDS; ++s) pa = mfma(da[s], vf[s], pa);
      }
      const float* st = reinterpret_cast<const float*>(stat) + cur * 2 * QT;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 L4 = *reinterpret_cast<const float4*>(st + 8 * g4 + 4 * h);
        const float4 D4 = *reinterpret_cast<const float4*>(st + QT + 8 * g4 + 4 * h);
        const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g4 + e;
          const float p = __builtin_amdgcn_exp2f(fmaf(sa[i], c, -Lv[e]));
          sa[i] = p;
          pa[i] = p * (pa[i] - Dv[e]);
        }
      }
      if (causal && qtl == wskip) {  // the diagonal tile: keys after the query are masked
        const int lim = kme - q0 - 4 * h;  // key > query  <=>  (i&3) + 8(i>>2) < lim
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i & 3) + 8 * (i >> 2) < lim) {
            sa[i] = 0.f;
            pa[i] = 0.f;
          }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 td[NDT];
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) td[dt] = tr_frag(Ds, 16 * s2, dt * 32, lane);
        const bf16x8 pb = acc_frag(sa, s2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) dva[dt] = mfma(td[dt], pb, dva[dt]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 tq[NDT];
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) tq[dt] = tr_frag(Qs, 16 * s2, dt * 32, lane);
        const bf16x8 db = acc_frag(pa, s2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) dka[dt] = mfma(tq[dt], db, dka[dt]);
      }
    }
    if constexpr (ASM_DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t + 1 landed
    __syncthreads();
  }
  const size_t off = ((size_t)b * S + k0w) * kvstride + (size_t)hk * D;
  store_rows_T(dva, 1.f, &qd[0][0] + w * 32 * CH, lane, dv + off, kvstride);
  __syncthreads();
  store_rows_T(dka, scale, &qd[0][0] + w * 32 * CH, lane, dk + off, kvstride);
}

// ------------------------------------- backward pass 2 split in two (dV pass, dK pass)
// attn_bwd_dkdv2_kernel holds both 32-key x 128-d accumulators (128 registers) plus the K and V
// fragments: 394 registers, one wave per SIMD, nothing to hide its LDS / exp2 latencies under.
// Split, each pass holds one accumulator and fits 256 registers, so two workgroups share a CU
// (two waves per SIMD):
//   DK = false (dV pass): S = Q.K^T, P = exp2(S c - lse2), dV^T += dO^T.P
//   DK = true  (dK pass): S, dP = dO.V^T, dS = P (dP - delta), dK^T += Q^T.dS
// (S is computed twice: 40 MFMAs per tile instead of 32).  Same per-element operation order
// as attn_bwd_dkdv2_kernel: bit-identical dK, dV.  Block order pairs key blocks so the two
// resident on a CU sum to the same causal work: heavy ones first, then the light ones
// lightest-first (block j and j + grid/2 land on one CU).
template <bool DK>
__global__ __launch_bounds__(NT, 2) void attn_bwd_dkdv_split_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2, const float* __restrict__ delta,
    bf16_t* __restrict__ dkv, int B, int S, int Hq, int Hkv, float c, float scale, int causal) {
  __shared__ u32x4 qd[2][2 * QT * CH];               // [buf][Q | dO] (32 KB); epilogue staging
  __shared__ __align__(16) float stat[2][2 * QT];    // [buf][lse2 | delta]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int per = B * Hkv, nkb = S / BK;
  const int jb = (int)blockIdx.x / per, bh = (int)blockIdx.x % per;
  const int kblk = !causal || jb < nkb / 2 ? jb : nkb - 1 - (jb - nkb / 2);
  const int b = bh / Hkv, hk = bh % Hkv, G = Hq / Hkv;
  const int k0w = kblk * BK + w * 32, kme = k0w + r;
  const size_t qstride = (size_t)Hq * D, kvstride = (size_t)Hkv * D;

  bf16x8 kf[NDS], vf[DK ? NDS : 1];
  {
    const size_t off = ((size_t)b * S + kme) * kvstride + (size_t)hk * D + 8 * h;
#pragma unroll
    for (int s = 0; s < NDS; ++s) {
      kf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(k + off + 16 * s));
      if constexpr (DK) vf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(v + off + 16 * s));
    }
  }
  const int qt0 = causal ? (kblk * BK) / QT : 0;
  const int nqt = S / QT - qt0;
  const int ntiles = G * nqt;
  const int wskip = causal ? __builtin_amdgcn_readfirstlane(w) : 0;

  auto fetch = [&](int t, int buf) {
    const int g = t / nqt, qt = qt0 + t % nqt, hq = hk * G + g;
    const size_t off = ((size_t)b * S + (size_t)qt * QT) * qstride + (size_t)hq * D;
    glds_tile<QT, NT>(q + off, qstride, qd[buf], tid);
    glds_tile<QT, NT>(dout + off, qstride, qd[buf] + QT * CH, tid);
    if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0) {
      const size_t srow = ((size_t)b * Hq + hq) * S + (size_t)qt * QT;
      const float* src = (lane < 32 ? lse2 : delta) + srow + (lane & 31);
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)stat[buf], 4, 0, 0);
    }
  };
  fetch(0, 0);
  __syncthreads();

  f32x16 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = zero16();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) fetch(t + 1, cur ^ 1);  // lands under this tile's MFMAs
    const int qtl = t % nqt;
    if (qtl >= wskip) {  // wave-uniform
      int boff = cur * 2 * QT * CH;
      asm volatile("" : "+s"(boff));
      const u32x4* Qs = &qd[0][0] + boff;
      const u32x4* Ds = Qs + QT * CH;
      const int q0 = (qt0 + qtl) * QT;
      f32x16 sa, pa;
      {
        bf16x8 qa[NDS];
#pragma unroll
        for (int s = 0; s < NDS; ++s) qa[s] = row_frag(Qs, r, 2 * s + h);
        __builtin_amdgcn_sched_barrier(0);
        sa = zero16();
#pragma unroll
        for (int s = 0; s < NDS; ++s) sa = mfma(qa[s], kf[s], sa);
      }
      if constexpr (DK) {
        bf16x8 da[NDS];
#pragma unroll
        for (int s = 0; s < NDS; ++s) da[s] = row_frag(Ds, r, 2 * s + h);
        __builtin_amdgcn_sched_barrier(0);
        pa = zero16();
#pragma unroll
        for (int s = 0; s < NDS; ++s) pa = mfma(da[s], vf[s], pa);
      }
      const float* st = reinterpret_cast<const float*>(stat) + cur * 2 * QT;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 L4 = *reinterpret_cast<const float4*>(st + 8 * g4 + 4 * h);
        const float Lv[4] = {L4.x, L4.y, L4.z, L4.w};
        float Dv[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (DK) {
          const float4 D4 = *reinterpret_cast<const float4*>(st + QT + 8 * g4 + 4 * h);
          Dv[0] = D4.x; Dv[1] = D4.y; Dv[2] = D4.z; Dv[3] = D4.w;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g4 + e;
          const float p = __builtin_amdgcn_exp2f(fmaf(sa[i], c, -Lv[e]));
          if constexpr (DK) pa[i] = p * (pa[i] - Dv[e]);
          else sa[i] = p;
        }
      }
      f32x16& op = DK ? pa : sa;
      if (causal && qtl == wskip) {  // the diagonal tile: keys after the query are masked
        const int lim = kme - q0 - 4 * h;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i & 3) + 8 * (i >> 2) < lim) op[i] = 0.f;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 tf[NDT];
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) tf[dt] = tr_frag(DK ? Qs : Ds, 16 * s2, dt * 32, lane);
        const bf16x8 ob = acc_frag(op, s2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) acc[dt] = mfma(tf[dt], ob, acc[dt]);
      }
    }
    __syncthreads();
  }
  const size_t off = ((size_t)b * S + k0w) * kvstride + (size_t)hk * D;
  store_rows_T(acc, DK ? scale : 1.f, &qd[0][0] + w * 32 * CH, lane, dkv + off, kvstride);
}

// ----------------------------------------- backward pass 2, software-pipelined (dK, dV)
// Same work split as attn_bwd_dkdv_kernel (one wave per SIMD: dK^T / dV^T of 32 keys, K and V
// fragments in registers, 390 of the 512), with the free registers spent on a pipeline: the
// Q / dO tiles cycle through a 3-deep LDS ring, so the row operands of tile t+1 are read into
// registers while tile t's dV / dK MFMAs run, and tile t+1's S / dP chains start without an LDS
// round trip (a single wave per SIMD has no sibling to hide it).  Stored tile t+2 and the
// global loads of tile t+3 ride behind the same MFMAs.
__global__ __launch_bounds__(NT, 1) void attn_bwd_dkdv_p_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int B, int S, int Hq, int Hkv, float c, float scale,
    int causal) {
  __shared__ u32x4 smem[3 * 2 * QT * CH];  // 3 x (Q, dO) tiles (48 KB); the dK/dV epilogue
  __shared__ float4 stat[3][2][QT / 4];    // [buf][lse2 | delta][32 rows]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int kblk = (int)blockIdx.x / (B * Hkv), bh = (int)blockIdx.x % (B * Hkv);
  const int b = bh / Hkv, hk = bh % Hkv, G = Hq / Hkv;
  const int k0w = kblk * BK + w * 32, kme = k0w + r;
  const size_t qstride = (size_t)Hq * D, kvstride = (size_t)Hkv * D;

  bf16x8 kf[NDS], vf[NDS];
  {
    const size_t off = ((size_t)b * S + kme) * kvstride + (size_t)hk * D + 8 * h;
#pragma unroll
    for (int s = 0; s < NDS; ++s) {
      kf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(k + off + 16 * s));
      vf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(v + off + 16 * s));
    }
  }
  const int qt0 = causal ? (kblk * BK) / QT : 0;
  const int nqt = S / QT - qt0;
  const int ntiles = G * nqt;

  Stage<QT> qs, ds;
  float4 st = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load = [&](int t) {
    const int g = t / nqt, qt = qt0 + t % nqt, hq = hk * G + g;
    const size_t off = ((size_t)b * S + (size_t)qt * QT) * qstride + (size_t)hq * D;
    const size_t srow = ((size_t)b * Hq + hq) * S + (size_t)qt * QT;
    qs.load(q + off, qstride, tid);
    ds.load(dout + off, qstride, tid);
    if (tid < 16) st = reinterpret_cast<const float4*>((tid < 8 ? lse2 : delta) + srow)[tid & 7];
  };
  auto store = [&](int buf) {
    qs.store(smem + buf * 2 * QT * CH, tid);
    ds.store(smem + buf * 2 * QT * CH + QT * CH, tid);
    if (tid < 16) stat[buf][tid >> 3][tid & 7] = st;
  };
  load(0);
  store(0);
  if (ntiles > 1) {
    load(1);
    store(1);
  }
  if (ntiles > 2) load(2);
  __syncthreads();

  bf16x8 qa[NDS], da[NDS];
#pragma unroll
  for (int s = 0; s < NDS; ++s) {
    qa[s] = row_frag(smem, r, 2 * s + h);
    da[s] = row_frag(smem + QT * CH, r, 2 * s + h);
  }
  f32x16 dka[NDT], dva[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    dka[dt] = zero16();
    dva[dt] = zero16();
  }
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const u32x4* Qs = smem + cur * 2 * QT * CH;
    const u32x4* Ds = Qs + QT * CH;
    const int nxt = cur == 2 ? 0 : cur + 1, nn2 = nxt == 2 ? 0 : nxt + 1;
    const int q0 = (qt0 + t % nqt) * QT;
    f32x16 sa = zero16(), pa = zero16();
#pragma unroll
    for (int s = 0; s < NDS; ++s) {
      sa = mfma(qa[s], kf[s], sa);
      pa = mfma(da[s], vf[s], pa);
    }
    const bool diag = causal && k0w + 31 > q0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 L4 = stat[cur][0][2 * g + h];
      const float4 D4 = stat[cur][1][2 * g + h];
      const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        float p = __builtin_amdgcn_exp2f(fmaf(sa[i], c, -Lv[e]));
        if (diag && kme > q0 + 8 * g + 4 * h + e) p = 0.f;
        sa[i] = p;
        pa[i] = p * (pa[i] - Dv[e]);
      }
    }
    bf16x8 pb[2], db[2], td[2][NDT], tq[2][NDT];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        td[s2][dt] = tr_frag(Ds, 16 * s2, dt * 32, lane);
        tq[s2][dt] = tr_frag(Qs, 16 * s2, dt * 32, lane);
      }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      pb[s2] = acc_frag(sa, s2);
      db[s2] = acc_frag(pa, s2);
    }
    if (t + 1 < ntiles) {  // next tile's row operands: in flight under this tile's dV / dK MFMAs
      const u32x4* Qn = smem + nxt * 2 * QT * CH;
#pragma unroll
      for (int s = 0; s < NDS; ++s) {
        qa[s] = row_frag(Qn, r, 2 * s + h);
        da[s] = row_frag(Qn + QT * CH, r, 2 * s + h);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        dva[dt] = mfma(td[s2][dt], pb[s2], dva[dt]);
        dka[dt] = mfma(tq[s2][dt], db[s2], dka[dt]);
      }
    if (t + 2 < ntiles) {
      store(nn2);
      if (t + 3 < ntiles) load(t + 3);
    }
    __syncthreads();
    cur = nxt;
  }
  const size_t off = ((size_t)b * S + k0w) * kvstride + (size_t)hk * D;
  store_rows_T(dva, 1.f, smem + w * 32 * CH, lane, dv + off, kvstride);
  __syncthreads();
  store_rows_T(dka, scale, smem + w * 32 * CH, lane, dk + off, kvstride);
}

// ------------------------------------------- backward pass 2, 8-wave workgroup (dK, dV)
// Two waves per SIMD (the 4-wave pass runs one, 390 registers): 8 waves x 32 keys = 256 keys
// per workgroup share each staged Q / dO tile.  To fit 256 registers a wave keeps only K's
// fragments (the S = Q.K^T operand) in registers; V's (the dP = dO.V^T operand) are re-read
// per tile from an LDS-resident image of the workgroup's 256 V rows (64 KB, loaded once), and
// Q / dO / lse2 / delta arrive by LDS-DMA (no staging registers).  Waves skip the query tiles
// wholly above their keys.  Block order: key block slowest (heaviest first under the mask),
// kv head fastest (the blocks reading one (b, kv head)'s Q / dO rows share an XCD at Hkv = 8).
constexpr int BK8 = 256;

__global__ __launch_bounds__(NT8, 1) void attn_bwd_dkdv8_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int B, int S, int Hq, int Hkv, float c, float scale,
    int causal) {
  __shared__ u32x4 vall[BK8 * CH];           // V rows of the workgroup (64 KB); dK/dV epilogue
  __shared__ u32x4 qd[2][2 * QT * CH];       // [buf][Q | dO] (32 KB)
  __shared__ __align__(16) float stat[2][2 * QT];  // [buf][lse2 | delta]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  if (__builtin_amdgcn_readfirstlane(tid) >= NT8 / 2) __builtin_amdgcn_s_setprio(1);
  int bi = (int)blockIdx.x;
  const int hk = bi % Hkv;
  bi /= Hkv;
  const int b = bi % B, kblk = bi / B, G = Hq / Hkv;
  const int k0w = kblk * BK8 + w * 32, kme = k0w + r;
  const size_t qstride = (size_t)Hq * D, kvstride = (size_t)Hkv * D;

  bf16x8 kf[NDS];
  {
    const size_t off = ((size_t)b * S + kme) * kvstride + (size_t)hk * D + 8 * h;
#pragma unroll
    for (int s = 0; s < NDS; ++s) kf[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(k + off + 16 * s));
  }
  const int qt0 = causal ? (kblk * BK8) / QT : 0;
  const int nqt = S / QT - qt0;
  const int ntiles = G * nqt;
  // this wave's first live query tile of every head: qt0 + w (readfirstlane: provably uniform,
  // so the branches around the LDS-DMA issue stay scalar)
  const int wskip = causal ? __builtin_amdgcn_readfirstlane(w) : 0;

  auto fetch = [&](int t, int buf) {  // Q, dO rows + lse2 / delta of tile t by LDS-DMA
    const int g = t / nqt, qt = qt0 + t % nqt, hq = hk * G + g;
    const size_t off = ((size_t)b * S + (size_t)qt * QT) * qstride + (size_t)hq * D;
    glds_tile<QT, NT8>(q + off, qstride, qd[buf], tid);
    glds_tile<QT, NT8>(dout + off, qstride, qd[buf] + QT * CH, tid);
    if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0) {
      const size_t srow = ((size_t)b * Hq + hq) * S + (size_t)qt * QT;
      const float* src = (lane < 32 ? lse2 : delta) + srow + (lane & 31);
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)stat[buf], 4, 0, 0);
    }
  };
  glds_tile<BK8, NT8>(v + (size_t)b * S * kvstride + (size_t)kblk * BK8 * kvstride + (size_t)hk * D, kvstride,
                      vall, tid);
  fetch(0, 0);
  __syncthreads();

  f32x16 dka[NDT], dva[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    dka[dt] = zero16();
    dva[dt] = zero16();
  }
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) fetch(t + 1, cur ^ 1);  // lands under this tile's MFMAs
    const int qtl = t % nqt;
    if (qtl >= wskip) {  // wave-uniform
      int boff = cur * 2 * QT * CH;
      asm volatile("" : "+s"(boff));  // opaque: one set of operand addresses, not one per buffer
      const u32x4* Qs = &qd[0][0] + boff;
      const u32x4* Ds = Qs + QT * CH;
      const int q0 = (qt0 + qtl) * QT;
      // row-read chunk XOR of this lane's rows (r of the Q / dO tiles, 32w + r of V: the same
      // low bits), re-derived per tile behind an optimisation barrier so the eight per-k-step
      // addresses are not hoisted (and spilled) across the loop
      int cx = h ^ (((r & 3) << 2) | ((r >> 2) & 3));
      asm volatile("" : "+v"(cx));
      const u32x4* Qr = Qs + r * CH;
      const u32x4* Dr = Ds + r * CH;
      const u32x4* Vr = vall + (32 * w + r) * CH;
      f32x16 sa = zero16(), pa = zero16();
      {
        bf16x8 qa[NDS];
#pragma unroll
        for (int s = 0; s < NDS; ++s) qa[s] = __builtin_bit_cast(bf16x8, Qr[(2 * s) ^ cx]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < NDS; ++s) sa = mfma(qa[s], kf[s], sa);
      }
#pragma unroll
      for (int half = 0; half < 2; ++half) {  // dP in two k-halves: 32 operand registers
        bf16x8 da[NDS / 2], vf[NDS / 2];
#pragma unroll
        for (int s = 0; s < NDS / 2; ++s) {
          da[s] = __builtin_bit_cast(bf16x8, Dr[(2 * (4 * half + s)) ^ cx]);
          vf[s] = __builtin_bit_cast(bf16x8, Vr[(2 * (4 * half + s)) ^ cx]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < NDS / 2; ++s) pa = mfma(da[s], vf[s], pa);
      }
      const bool diag = causal && k0w + 31 > q0;
      const float* st = stat[cur];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 L4 = *reinterpret_cast<const float4*>(st + 8 * g4 + 4 * h);
        const float4 D4 = *reinterpret_cast<const float4*>(st + QT + 8 * g4 + 4 * h);
        const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g4 + e;
          float p = __builtin_amdgcn_exp2f(fmaf(sa[i], c, -Lv[e]));
          if (diag && kme > q0 + 8 * g4 + 4 * h + e) p = 0.f;
          sa[i] = p;
          pa[i] = p * (pa[i] - Dv[e]);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {  // one 16-query k-step at a time, dV^T += dO^T P then dK^T += Q^T dS
#pragma unroll
        for (int which = 0; which < 2; ++which) {
          const u32x4* src = which == 0 ? Ds : Qs;
          bf16x8 tf[NDT];
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) tf[dt] = tr_frag(src, 16 * s2, dt * 32, lane);
          const bf16x8 op = acc_frag(which == 0 ? sa : pa, s2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            if (which == 0) dva[dt] = mfma(tf[dt], op, dva[dt]);
            else dka[dt] = mfma(tf[dt], op, dka[dt]);
          }
        }
      }
    }
    __syncthreads();
  }
  const size_t off = ((size_t)b * S + k0w) * kvstride + (size_t)hk * D;
  store_rows_T(dva, 1.f, vall + w * 32 * CH, lane, dv + off, kvstride);
  __syncthreads();
  store_rows_T(dka, scale, vall + w * 32 * CH, lane, dk + off, kvstride);
}

}  // namespace

extern "C" {

int pto_attn_exp_fwd(int variant, const void* q, const void* k, const void* v, void* o, float* lse2, int B, int S,
                     int Hq, int Hkv, float c, int causal, void* stream) {
  if (variant != 9 || S % BM8 != 0) return -1;
  hipLaunchKernelGGL(attn_fwd8p_kernel, dim3((S / BM8) * B * Hq), dim3(NT8), 0, (hipStream_t)stream,
                     (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse2, B, S, Hq, Hkv, c, causal);
  return (int)hipGetLastError();
}

int pto_attn_exp_dq(int variant, const void* q, const void* k, const void* v, const void* o, const void* dout,
                    const float* lse2, float* delta, void* dq, int B, int S, int Hq, int Hkv, float c, float scale,
                    int causal, void* stream) {
  if (variant != 8 || S % BM8 != 0) return -1;
  hipLaunchKernelGGL(attn_bwd_dq8_kernel, dim3((S / BM8) * B * Hq), dim3(NT8), 0, (hipStream_t)stream,
                     (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)o, (const bf16_t*)dout,
                     lse2, delta, (bf16_t*)dq, B, S, Hq, Hkv, c, scale, causal);
  return (int)hipGetLastError();
}

int pto_attn_exp_dkdv(int variant, const void* q, const void* k, const void* v, const void* dout, const float* lse2,
                      const float* delta, void* dk, void* dv, int B, int S, int Hq, int Hkv, float c, float scale,
                      int causal, void* stream) {
  const bf16_t *Q = (const bf16_t*)q, *K = (const bf16_t*)k, *V = (const bf16_t*)v, *DO = (const bf16_t*)dout;
  if (variant == 3) {
    if (S % BK8 != 0) return -1;
    hipLaunchKernelGGL(attn_bwd_dkdv8_kernel, dim3((S / BK8) * B * Hkv), dim3(NT8), 0, (hipStream_t)stream, Q, K, V,
                       DO, lse2, delta, (bf16_t*)dk, (bf16_t*)dv, B, S, Hq, Hkv, c, scale, causal);
  } else if (variant == 6) {
    hipLaunchKernelGGL(attn_bwd_dkdv_split_kernel<false>, dim3((S / BK) * B * Hkv), dim3(NT), 0, (hipStream_t)stream,
                       Q, K, V, DO, lse2, delta, (bf16_t*)dv, B, S, Hq, Hkv, c, scale, causal);
    hipLaunchKernelGGL(attn_bwd_dkdv_split_kernel<true>, dim3((S / BK) * B * Hkv), dim3(NT), 0, (hipStream_t)stream,
                       Q, K, V, DO, lse2, delta, (bf16_t*)dk, B, S, Hq, Hkv, c, scale, causal);
  } else if (variant == 2 || variant == 4 || variant == 7) {
    hipLaunchKernelGGL(variant == 7 ? attn_bwd_dkdv2_kernel<true>
                       : variant == 4 ? attn_bwd_dkdv2_kernel<false>
                                      : attn_bwd_dkdv_p_kernel,
                       dim3((S / BK) * B * Hkv), dim3(NT), 0, (hipStream_t)stream, Q, K, V, DO, lse2, delta,
                       (bf16_t*)dk, (bf16_t*)dv, B, S, Hq, Hkv, c, scale, causal);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
