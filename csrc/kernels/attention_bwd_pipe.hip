// Flash-attention backward, dK/dV pass, software-pipelined across query tiles (the default dK/dV
// pass of attention.hip's pto_attn_bwd), and the dQ pass in the same form.  Its own translation unit: its dK / dV accumulators are
// pinned in AGPRs by hand-written MFMAs (below), and everything the compiler allocates fits the
// 256 architectural VGPRs.
#include "attention_common.h"

namespace {

// dK / dV accumulators pinned in AGPRs a0-a127 (dV^T tile dt in a[16dt..], dK^T tile dt in
// a[64 + 16dt..]): only these asm MFMAs touch them, so the compiler neither copies them between
// register files nor counts them against the 256 VGPRs its own values share.  Every statement
// clobbers all 128 so nothing of the compiler's is kept there (checked in the ISA: no compiler
// v_accvgpr_* in the kernel).  Hazards: the accumulate chains are MFMA -> MFMA (C = previous D:
// none); every VALU-written operand (the bf16-packed P and dS) is packed at least two gaps
// before the MFMA that reads it (the schedule below), so no `s_nop` pad is needed
// (tests/test_attention_isa.py checks the distance in the built code object); the epilogue
// waits out the last MFMA before reading (acc_read).
#define PTO_AGPR_CLOBBERS "a0","a1","a2","a3","a4","a5","a6","a7","a8","a9","a10","a11","a12","a13","a14","a15","a16","a17","a18","a19","a20","a21","a22","a23","a24","a25","a26","a27","a28","a29","a30","a31","a32","a33","a34","a35","a36","a37","a38","a39","a40","a41","a42","a43","a44","a45","a46","a47","a48","a49","a50","a51","a52","a53","a54","a55","a56","a57","a58","a59","a60","a61","a62","a63","a64","a65","a66","a67","a68","a69","a70","a71","a72","a73","a74","a75","a76","a77","a78","a79","a80","a81","a82","a83","a84","a85","a86","a87","a88","a89","a90","a91","a92","a93","a94","a95","a96","a97","a98","a99","a100","a101","a102","a103","a104","a105","a106","a107","a108","a109","a110","a111","a112","a113","a114","a115","a116","a117","a118","a119","a120","a121","a122","a123","a124","a125","a126","a127"
// Round-4 ablation and placement knobs (no dS / exp2 / DMA / barrier; lse2 staged per four tiles;
// DMA start gap and spacing; an s_nop pad before each k-step's first MFMA; barrier-staged
// epilogue) were measured and are recorded in profiles/r4_attn_dkdv_pipe_ablations.md and
// r4_attn_dkdv_pipe_knobs_ab.json; the source keeps only the chosen settings (git show 3eed2ef
// for the knobbed form).
constexpr int DMA0 = 8;  // gap of the first of a tile's five LDS-DMA pieces (one per gap after it)
#define PTO_AGPR_CLOBBERS_0_63 "a0","a1","a2","a3","a4","a5","a6","a7","a8","a9","a10","a11","a12","a13","a14","a15","a16","a17","a18","a19","a20","a21","a22","a23","a24","a25","a26","a27","a28","a29","a30","a31","a32","a33","a34","a35","a36","a37","a38","a39","a40","a41","a42","a43","a44","a45","a46","a47","a48","a49","a50","a51","a52","a53","a54","a55","a56","a57","a58","a59","a60","a61","a62","a63"
#define PTO_ZERO_0_63 "v_accvgpr_write_b32 a0, 0\n\tv_accvgpr_write_b32 a1, 0\n\tv_accvgpr_write_b32 a2, 0\n\tv_accvgpr_write_b32 a3, 0\n\tv_accvgpr_write_b32 a4, 0\n\tv_accvgpr_write_b32 a5, 0\n\tv_accvgpr_write_b32 a6, 0\n\tv_accvgpr_write_b32 a7, 0\n\tv_accvgpr_write_b32 a8, 0\n\tv_accvgpr_write_b32 a9, 0\n\tv_accvgpr_write_b32 a10, 0\n\tv_accvgpr_write_b32 a11, 0\n\tv_accvgpr_write_b32 a12, 0\n\tv_accvgpr_write_b32 a13, 0\n\tv_accvgpr_write_b32 a14, 0\n\tv_accvgpr_write_b32 a15, 0\n\tv_accvgpr_write_b32 a16, 0\n\tv_accvgpr_write_b32 a17, 0\n\tv_accvgpr_write_b32 a18, 0\n\tv_accvgpr_write_b32 a19, 0\n\tv_accvgpr_write_b32 a20, 0\n\tv_accvgpr_write_b32 a21, 0\n\tv_accvgpr_write_b32 a22, 0\n\tv_accvgpr_write_b32 a23, 0\n\tv_accvgpr_write_b32 a24, 0\n\tv_accvgpr_write_b32 a25, 0\n\tv_accvgpr_write_b32 a26, 0\n\tv_accvgpr_write_b32 a27, 0\n\tv_accvgpr_write_b32 a28, 0\n\tv_accvgpr_write_b32 a29, 0\n\tv_accvgpr_write_b32 a30, 0\n\tv_accvgpr_write_b32 a31, 0\n\tv_accvgpr_write_b32 a32, 0\n\tv_accvgpr_write_b32 a33, 0\n\tv_accvgpr_write_b32 a34, 0\n\tv_accvgpr_write_b32 a35, 0\n\tv_accvgpr_write_b32 a36, 0\n\tv_accvgpr_write_b32 a37, 0\n\tv_accvgpr_write_b32 a38, 0\n\tv_accvgpr_write_b32 a39, 0\n\tv_accvgpr_write_b32 a40, 0\n\tv_accvgpr_write_b32 a41, 0\n\tv_accvgpr_write_b32 a42, 0\n\tv_accvgpr_write_b32 a43, 0\n\tv_accvgpr_write_b32 a44, 0\n\tv_accvgpr_write_b32 a45, 0\n\tv_accvgpr_write_b32 a46, 0\n\tv_accvgpr_write_b32 a47, 0\n\tv_accvgpr_write_b32 a48, 0\n\tv_accvgpr_write_b32 a49, 0\n\tv_accvgpr_write_b32 a50, 0\n\tv_accvgpr_write_b32 a51, 0\n\tv_accvgpr_write_b32 a52, 0\n\tv_accvgpr_write_b32 a53, 0\n\tv_accvgpr_write_b32 a54, 0\n\tv_accvgpr_write_b32 a55, 0\n\tv_accvgpr_write_b32 a56, 0\n\tv_accvgpr_write_b32 a57, 0\n\tv_accvgpr_write_b32 a58, 0\n\tv_accvgpr_write_b32 a59, 0\n\tv_accvgpr_write_b32 a60, 0\n\tv_accvgpr_write_b32 a61, 0\n\tv_accvgpr_write_b32 a62, 0\n\tv_accvgpr_write_b32 a63, 0"
template <int A0>
__device__ __forceinline__ void mfma_acc(const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]"
               :: "v"(a), "v"(b), "i"(A0), "i"(A0 + 15) : PTO_AGPR_CLOBBERS);
}
// tile `slot` (0-3 dV^T, 4-7 dK^T); a constant after unrolling, so the switch folds away
__device__ __forceinline__ void mfma_acc_slot(int slot, const bf16x8& a, const bf16x8& b) {
  switch (slot) {
    case 0: mfma_acc<0>(a, b); break;
    case 1: mfma_acc<16>(a, b); break;
    case 2: mfma_acc<32>(a, b); break;
    case 3: mfma_acc<48>(a, b); break;
    case 4: mfma_acc<64>(a, b); break;
    case 5: mfma_acc<80>(a, b); break;
    case 6: mfma_acc<96>(a, b); break;
    default: mfma_acc<112>(a, b); break;
  }
}
__device__ __forceinline__ void acc_zero() {
  asm volatile("v_accvgpr_write_b32 a0, 0\n\tv_accvgpr_write_b32 a1, 0\n\tv_accvgpr_write_b32 a2, 0\n\tv_accvgpr_write_b32 a3, 0\n\tv_accvgpr_write_b32 a4, 0\n\tv_accvgpr_write_b32 a5, 0\n\tv_accvgpr_write_b32 a6, 0\n\tv_accvgpr_write_b32 a7, 0\n\tv_accvgpr_write_b32 a8, 0\n\tv_accvgpr_write_b32 a9, 0\n\tv_accvgpr_write_b32 a10, 0\n\tv_accvgpr_write_b32 a11, 0\n\tv_accvgpr_write_b32 a12, 0\n\tv_accvgpr_write_b32 a13, 0\n\tv_accvgpr_write_b32 a14, 0\n\tv_accvgpr_write_b32 a15, 0\n\tv_accvgpr_write_b32 a16, 0\n\tv_accvgpr_write_b32 a17, 0\n\tv_accvgpr_write_b32 a18, 0\n\tv_accvgpr_write_b32 a19, 0\n\tv_accvgpr_write_b32 a20, 0\n\tv_accvgpr_write_b32 a21, 0\n\tv_accvgpr_write_b32 a22, 0\n\tv_accvgpr_write_b32 a23, 0\n\tv_accvgpr_write_b32 a24, 0\n\tv_accvgpr_write_b32 a25, 0\n\tv_accvgpr_write_b32 a26, 0\n\tv_accvgpr_write_b32 a27, 0\n\tv_accvgpr_write_b32 a28, 0\n\tv_accvgpr_write_b32 a29, 0\n\tv_accvgpr_write_b32 a30, 0\n\tv_accvgpr_write_b32 a31, 0\n\tv_accvgpr_write_b32 a32, 0\n\tv_accvgpr_write_b32 a33, 0\n\tv_accvgpr_write_b32 a34, 0\n\tv_accvgpr_write_b32 a35, 0\n\tv_accvgpr_write_b32 a36, 0\n\tv_accvgpr_write_b32 a37, 0\n\tv_accvgpr_write_b32 a38, 0\n\tv_accvgpr_write_b32 a39, 0\n\tv_accvgpr_write_b32 a40, 0\n\tv_accvgpr_write_b32 a41, 0\n\tv_accvgpr_write_b32 a42, 0\n\tv_accvgpr_write_b32 a43, 0\n\tv_accvgpr_write_b32 a44, 0\n\tv_accvgpr_write_b32 a45, 0\n\tv_accvgpr_write_b32 a46, 0\n\tv_accvgpr_write_b32 a47, 0\n\tv_accvgpr_write_b32 a48, 0\n\tv_accvgpr_write_b32 a49, 0\n\tv_accvgpr_write_b32 a50, 0\n\tv_accvgpr_write_b32 a51, 0\n\tv_accvgpr_write_b32 a52, 0\n\tv_accvgpr_write_b32 a53, 0\n\tv_accvgpr_write_b32 a54, 0\n\tv_accvgpr_write_b32 a55, 0\n\tv_accvgpr_write_b32 a56, 0\n\tv_accvgpr_write_b32 a57, 0\n\tv_accvgpr_write_b32 a58, 0\n\tv_accvgpr_write_b32 a59, 0\n\tv_accvgpr_write_b32 a60, 0\n\tv_accvgpr_write_b32 a61, 0\n\tv_accvgpr_write_b32 a62, 0\n\tv_accvgpr_write_b32 a63, 0\n\tv_accvgpr_write_b32 a64, 0\n\tv_accvgpr_write_b32 a65, 0\n\tv_accvgpr_write_b32 a66, 0\n\tv_accvgpr_write_b32 a67, 0\n\tv_accvgpr_write_b32 a68, 0\n\tv_accvgpr_write_b32 a69, 0\n\tv_accvgpr_write_b32 a70, 0\n\tv_accvgpr_write_b32 a71, 0\n\tv_accvgpr_write_b32 a72, 0\n\tv_accvgpr_write_b32 a73, 0\n\tv_accvgpr_write_b32 a74, 0\n\tv_accvgpr_write_b32 a75, 0\n\tv_accvgpr_write_b32 a76, 0\n\tv_accvgpr_write_b32 a77, 0\n\tv_accvgpr_write_b32 a78, 0\n\tv_accvgpr_write_b32 a79, 0\n\tv_accvgpr_write_b32 a80, 0\n\tv_accvgpr_write_b32 a81, 0\n\tv_accvgpr_write_b32 a82, 0\n\tv_accvgpr_write_b32 a83, 0\n\tv_accvgpr_write_b32 a84, 0\n\tv_accvgpr_write_b32 a85, 0\n\tv_accvgpr_write_b32 a86, 0\n\tv_accvgpr_write_b32 a87, 0\n\tv_accvgpr_write_b32 a88, 0\n\tv_accvgpr_write_b32 a89, 0\n\tv_accvgpr_write_b32 a90, 0\n\tv_accvgpr_write_b32 a91, 0\n\tv_accvgpr_write_b32 a92, 0\n\tv_accvgpr_write_b32 a93, 0\n\tv_accvgpr_write_b32 a94, 0\n\tv_accvgpr_write_b32 a95, 0\n\tv_accvgpr_write_b32 a96, 0\n\tv_accvgpr_write_b32 a97, 0\n\tv_accvgpr_write_b32 a98, 0\n\tv_accvgpr_write_b32 a99, 0\n\tv_accvgpr_write_b32 a100, 0\n\tv_accvgpr_write_b32 a101, 0\n\tv_accvgpr_write_b32 a102, 0\n\tv_accvgpr_write_b32 a103, 0\n\tv_accvgpr_write_b32 a104, 0\n\tv_accvgpr_write_b32 a105, 0\n\tv_accvgpr_write_b32 a106, 0\n\tv_accvgpr_write_b32 a107, 0\n\tv_accvgpr_write_b32 a108, 0\n\tv_accvgpr_write_b32 a109, 0\n\tv_accvgpr_write_b32 a110, 0\n\tv_accvgpr_write_b32 a111, 0\n\tv_accvgpr_write_b32 a112, 0\n\tv_accvgpr_write_b32 a113, 0\n\tv_accvgpr_write_b32 a114, 0\n\tv_accvgpr_write_b32 a115, 0\n\tv_accvgpr_write_b32 a116, 0\n\tv_accvgpr_write_b32 a117, 0\n\tv_accvgpr_write_b32 a118, 0\n\tv_accvgpr_write_b32 a119, 0\n\tv_accvgpr_write_b32 a120, 0\n\tv_accvgpr_write_b32 a121, 0\n\tv_accvgpr_write_b32 a122, 0\n\tv_accvgpr_write_b32 a123, 0\n\tv_accvgpr_write_b32 a124, 0\n\tv_accvgpr_write_b32 a125, 0\n\tv_accvgpr_write_b32 a126, 0\n\tv_accvgpr_write_b32 a127, 0" ::: PTO_AGPR_CLOBBERS);
}
// two floats -> packed bf16 (v_cvt_pk_bf16_f32, RNE; compiler-visible, so no inline-asm pads)
__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const f32x2 v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
// accumulator tile A0 (16 AGPRs) -> registers, after the last MFMA into it has drained
template <int A0>
__device__ __forceinline__ f32x16 acc_read() {
  f32x16 x;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float f;
    asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(f) : "i"(A0 + i));
    x[i] = f;
  }
  return x;
}

// ------------------------------------- backward pass 2, software-pipelined across query tiles
// attn_bwd_dkdv2_kernel (attention.hip) runs one wave per SIMD and issues in order, so a tile's
// phases serialize: S MFMAs, dP MFMAs, ~100 VALU instructions (exp2, dS, bf16 packing) with the
// matrix pipe idle, then the dV / dK MFMAs -- and an MFMA chain holds the wave for its whole
// length, so nothing placed after it overlaps it (26.5 % MFMA busy, profiles/r3_pmc_digest.md).
// Here a tile is 32 MFMA gaps, each one MFMA plus about five independent fillers (at most one
// v_exp; MI355X_MICROARCH.md, constants table), and the iteration also computes S for the next
// tile (its Q tile is prefetched two ahead, three LDS buffers):
//   gaps  0-7   dP_t          P_t = exp2(S_t c - lse2), one element per gap; dO_t rows 4-7
//   gaps  8-15  S_{t+1}       the rest of P_t; Q_{t+1} rows read in gaps 4-7
//   gaps 16-23  dV_t          dS_t = P_t (dP_t - delta); dO_t^T transposed reads (gaps 12-19)
//   gaps 24-31  dK_t          Q_t^T reads (20-27); tile t+1's dO rows 0-3 and lse2
// Tile t+2's LDS-DMA goes out in gaps 8-12: iteration t+1 reads it (its S_{t+2} operands), so
// it has to land by this iteration's closing barrier.
// Every operand is read four gaps ahead of its MFMA; every gap ends in a sched_barrier.  The
// loop is unrolled over the three buffers, so each LDS read is a per-lane offset plus an
// immediate and S_t / S_{t+1} rotate through three register sets with no copies.  Per-element operations and their order match attn_bwd_dkdv2_kernel:
// bit-identical dK, dV.
#ifdef PTO_ATTN_STAMPS
// diagnostic build only (tools/build_exp.sh ... "-DPTO_ATTN_STAMPS"): per wave, s_memtime at
// kernel entry, loop entry, loop exit and kernel end, plus s_memrealtime at entry / end and the
// tile count; read back with pto_attn_pipe_stamps()
// slots 8-15: s_memtime at gaps 0, 8, 16, 24 of tile 9 and after its closing barrier
__device__ unsigned long long g_pipe_stamps[8192 * 16];
#define PTO_STAMP(k) \
  if (lane == 0 && blockIdx.x < 2048) g_pipe_stamps[((size_t)blockIdx.x * 4 + w) * 16 + (k)] = __builtin_amdgcn_s_memtime()
#define PTO_RSTAMP(k) \
  if (lane == 0 && blockIdx.x < 2048) g_pipe_stamps[((size_t)blockIdx.x * 4 + w) * 16 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define PTO_STAMP(k)
#define PTO_RSTAMP(k)
#endif
constexpr int TLEAD = 4;  // gaps between a transposed operand read and its MFMA
__global__ __launch_bounds__(NT, 1) void attn_bwd_dkdv_pipe_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2, const float* __restrict__ delta,
    bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int B, int S, int Hq, int Hkv, float c, float scale,
    int causal) {
  constexpr int NB = 3, TILE = 2 * QT * CH;
  __shared__ u32x4 qd[NB * TILE];                   // [buf][Q | dO] (48 KB); dK/dV epilogue
  __shared__ __align__(16) float stat[NB][2 * QT];  // [buf][lse2 | delta]
  constexpr int SDOFF = QT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int kblk = (int)blockIdx.x / (B * Hkv), bh = (int)blockIdx.x % (B * Hkv);
  const int b = bh / Hkv, hk = bh % Hkv, G = Hq / Hkv;
  const int k0w = kblk * BK + w * 32, kme = k0w + r;
  const size_t qstride = (size_t)Hq * D, kvstride = (size_t)Hkv * D;
  PTO_STAMP(0);
  PTO_RSTAMP(4);

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
  const int wskip = causal ? wu : 0;  // first live tile of a head: qt0 + w

  // LDS-DMA: piece k of a tile (k = 0, 1: Q rows; 2, 3: dO rows; 4: lse2 | delta).  Each wave
  // moves pieces w and w + 4 of the 8 per [QT][D] tile; every wave also issues the statistics
  // piece (the same 256 bytes), so all waves count the same five loads per tile.
  uint32_t doff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = 64 * (w + 4 * i) + lane, row = e / CH, j = e % CH;
    doff[i] = (uint32_t)(row * qstride) + 8 * (j ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  }
  const float* sbase = (lane < 32 ? lse2 : delta) + (lane & 31);
  auto tile_off = [&](int t, size_t& toff, size_t& soff) {  // scalar: tile t's Q/dO and stat offsets
    t = t < ntiles ? t : ntiles - 1;  // past the end: refetch the last tile into a dead buffer
    const int g = t / nqt, qt = qt0 + t % nqt, hq = hk * G + g;
    toff = ((size_t)b * S + (size_t)qt * QT) * qstride + (size_t)hq * D;
    soff = ((size_t)b * Hq + hq) * S + (size_t)qt * QT;
  };
  const unsigned lds_w = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(qd + 64 * wu));  // this wave's piece 0
  auto dma = [&](int buf, int piece, size_t toff, size_t soff) {
    if (piece < 4) {
      const int i = piece & 1;
      const bf16_t* src = (piece < 2 ? q : dout) + toff + doff[i];
      const unsigned dst = lds_w + 16u * (buf * TILE + (piece < 2 ? 0 : QT * CH) + 64 * 4 * i);
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                   :: "s"(dst), "v"(src) : "memory", "m0");
    } else {
      glds_dword_asm(sbase + soff, stat[buf]);
    }
  };

  // loop-carried: S of the current tile (one of three rotating sets), dO rows 0-3 and lse2 rows
  // 0-3 of the current tile
  f32x16 s0 = zero16(), s1 = zero16(), s2 = zero16();
  bf16x8 da[NDS];
  float4 L4[4], D4[4];

  acc_zero();

  // one tile in buffer CUR: consumes sin (S_t), produces sout (S_{t+1} from buffer CUR + 1),
  // DMAs tile t + 2 into buffer CUR + 2
  auto step = [&](auto curc, auto maskc, f32x16& sin, f32x16& sout, int lim, size_t toff2, size_t soff2, bool stamp,
                  int t) {
    constexpr int CUR = decltype(curc)::value, NXT = (CUR + 1) % NB, NN = (CUR + 2) % NB;
    constexpr bool MASK = decltype(maskc)::value;
    const u32x4* Qs = qd + CUR * TILE;
    const u32x4* Ds = Qs + QT * CH;
    const u32x4* Qn = qd + NXT * TILE;
    const u32x4* Dn = Qn + QT * CH;
    const float* st = stat[CUR];
    const float* stn = stat[NXT];
    (void)t;
    f32x16 pa = zero16();
    sout = zero16();
    bf16x8 qa[NDS], td[8], tq[8], pb[2], db[2];
    uint32_t pw[8], dw[8];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
#ifdef PTO_ATTN_STAMPS
      if ((j & 7) == 0 && stamp) PTO_STAMP(8 + (j >> 3));
#endif
      // ---- the gap's MFMA
      if (j < 8) {
        pa = mfma(da[j], vf[j], pa);
      } else if (j < 16) {
        sout = mfma(qa[j - 8], kf[j - 8], sout);
      } else if (j < 24) {  // dV^T tile (j & 3) += dO^T . P
        mfma_acc_slot(j & 3, td[j - 16], pb[(j - 16) >> 2]);
      } else {               // dK^T tile (j & 3) += Q^T . dS
        mfma_acc_slot(4 + (j & 3), tq[j - 24], db[(j - 24) >> 2]);
      }
      // ---- VALU, skewed so that no filler waits on another in the same gap (in-order issue:
      // a dependent VALU op stalls the wave, and the next MFMA with it):
      //   P_t:  fma of element j in gap j, its exp2 in gap j + 1, the pair's bf16 pack in the
      //         gap after the pair's second exp2 (gaps 0-17)
      //   dS_t: dP - delta of elements 2m, 2m+1 in gap 16 + m, times P in gap 17 + m, the pack
      //         in gap 18 + m (gaps 16-25)
      if (j < 16) {
        const float4 l4 = L4[j >> 2];
        const int e = j & 3;
        const float Lv = e == 0 ? l4.x : e == 1 ? l4.y : e == 2 ? l4.z : l4.w;
        sin[j] = fmaf(sin[j], c, -Lv);
      }
      if (j >= 1 && j <= 16) {
        const int i = j - 1;
        float p = __builtin_amdgcn_exp2f(sin[i]);
        if (MASK && (i & 3) + 8 * (i >> 2) < lim) p = 0.f;  // key > query
        sin[i] = p;
      }
      if (j >= 3 && j <= 17 && (j & 1)) {
        const int k2 = (j - 3) >> 1;  // pair k2 = elements 2 k2, 2 k2 + 1
        pw[k2] = pk2(sin[2 * k2], sin[2 * k2 + 1]);
        if (k2 == 3 || k2 == 7) {
          const int s = k2 >> 2;
          u32x4 u = {pw[4 * s], pw[4 * s + 1], pw[4 * s + 2], pw[4 * s + 3]};
          pb[s] = __builtin_bit_cast(bf16x8, u);
        }
      }
      if (j >= 16 && j < 24) {
        const int m = j - 16;
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          const int i = 2 * m + e2, ei = i & 3;
          const float4 d4 = D4[i >> 2];
          const float Dv = ei == 0 ? d4.x : ei == 1 ? d4.y : ei == 2 ? d4.z : d4.w;
          pa[i] = pa[i] - Dv;
        }
      }
      if (j >= 17 && j < 25) {
        const int m = j - 17;
        pa[2 * m] = sin[2 * m] * pa[2 * m];
        pa[2 * m + 1] = sin[2 * m + 1] * pa[2 * m + 1];
      }
      if (j >= 18 && j < 26) {
        const int m = j - 18;
        dw[m] = pk2(pa[2 * m], pa[2 * m + 1]);
        if (m == 3 || m == 7) {
          const int s = m >> 2;
          u32x4 u = {dw[4 * s], dw[4 * s + 1], dw[4 * s + 2], dw[4 * s + 3]};
          db[s] = __builtin_bit_cast(bf16x8, u);
        }
      }
      // ---- LDS reads, four gaps ahead of their consumer
      if (j < 4) da[4 + j] = row_frag(Ds, r, 2 * (4 + j) + h);
      if (j == 0 || j == 4 || j == 8) L4[(j >> 2) + 1] = *reinterpret_cast<const float4*>(st + 8 * ((j >> 2) + 1) + 4 * h);
      if (j >= 4 && j < 8) {
        qa[2 * (j - 4)] = row_frag(Qn, r, 4 * (j - 4) + h);
        qa[2 * (j - 4) + 1] = row_frag(Qn, r, 4 * (j - 4) + 2 + h);
      }
      if (j >= 16 - TLEAD && j < 24 - TLEAD)
        td[j - 16 + TLEAD] = tr_frag(Ds, 16 * ((j - 16 + TLEAD) >> 2), ((j - 16 + TLEAD) & 3) * 32, lane);
      if (j == 12 || j == 14 || j == 16 || j == 18)
        D4[(j - 12) >> 1] = *reinterpret_cast<const float4*>(st + SDOFF + 8 * ((j - 12) >> 1) + 4 * h);
      if (j >= 24 - TLEAD && j < 32 - TLEAD)
        tq[j - 24 + TLEAD] = tr_frag(Qs, 16 * ((j - 24 + TLEAD) >> 2), ((j - 24 + TLEAD) & 3) * 32, lane);
      if (j >= 28) {
        da[j - 28] = row_frag(Dn, r, 2 * (j - 28) + h);
        if (j == 28) L4[0] = *reinterpret_cast<const float4*>(stn + 4 * h);
      }
      // ---- tile t + 2 -> buffer NN (last read before this tile's opening barrier); it must
      // land by this tile's closing barrier (tile t + 1 reads it), so it goes out early
      if (j >= DMA0 && j < DMA0 + 5) dma(NN, j - DMA0, toff2, soff2);

      __builtin_amdgcn_sched_barrier(0);
    }
  };
  std::integral_constant<bool, true> MK;
  std::integral_constant<bool, false> NM;
  std::integral_constant<int, 0> B0;
  std::integral_constant<int, 1> B1;
  std::integral_constant<int, 2> B2;

  // prologue: tiles 0 and 1 in flight, then S_0 and the loop-carried operands of tile 0
  {
    size_t toff, soff;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      tile_off(t, toff, soff);
#pragma unroll
      for (int pc = 0; pc < 5; ++pc) dma(t, pc, toff, soff);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const u32x4* Qs = qd;
    bf16x8 qa[NDS];
#pragma unroll
    for (int s = 0; s < NDS; ++s) qa[s] = row_frag(Qs, r, 2 * s + h);
#pragma unroll
    for (int s = 0; s < 4; ++s) da[s] = row_frag(Qs + QT * CH, r, 2 * s + h);
    L4[0] = *reinterpret_cast<const float4*>(stat[0] + 4 * h);
#pragma unroll
    for (int s = 0; s < NDS; ++s) s0 = mfma(qa[s], kf[s], s0);
  }
  // causal: a wave's diagonal tile is masked per element, the tiles wholly above its keys
  // (t % nqt < wskip) are masked whole (they add exact zeros; wave 0, which has none, sets the
  // block's time); every other tile runs the unmasked step
  auto masked_of = [&](int t) { return causal && t % nqt <= wskip; };  // wave-uniform
  auto lim_of = [&](int t) {  // mask P where (i&3) + 8(i>>2) < lim
    const int qtl = t % nqt;
    return !causal || qtl > wskip ? 0 : qtl < wskip ? QT : kme - (qt0 + qtl) * QT - 4 * h;
  };

  auto tile_end = [&](int t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t + 2 landed (read from tile t + 1 on)
#ifdef PTO_ATTN_STAMPS
    if (t == 9) PTO_STAMP(12);
#endif
    __syncthreads();
#ifdef PTO_ATTN_STAMPS
    if (t == 9) PTO_STAMP(13);
#endif
    (void)t;
  };
  PTO_STAMP(1);
  for (int t = 0;;) {
    size_t toff, soff;
    tile_off(t + 2, toff, soff);
    if (masked_of(t))
      step(B0, MK, s0, s1, lim_of(t), toff, soff, t == 9, t);
    else
      step(B0, NM, s0, s1, 0, toff, soff, t == 9, t);
    tile_end(t);
    if (++t == ntiles) break;
    tile_off(t + 2, toff, soff);
    if (masked_of(t))
      step(B1, MK, s1, s2, lim_of(t), toff, soff, t == 9, t);
    else
      step(B1, NM, s1, s2, 0, toff, soff, t == 9, t);
    tile_end(t);
    if (++t == ntiles) break;
    tile_off(t + 2, toff, soff);
    if (masked_of(t))
      step(B2, MK, s2, s0, lim_of(t), toff, soff, t == 9, t);
    else
      step(B2, NM, s2, s0, 0, toff, soff, t == 9, t);
    tile_end(t);
    if (++t == ntiles) break;
  }
  PTO_STAMP(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped refetches, before the epilogue
  __syncthreads();                                   // reuses buffers 0-1
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");  // last MFMA drained
  f32x16 acc[NDT];
  acc[0] = acc_read<0>();
  acc[1] = acc_read<16>();
  acc[2] = acc_read<32>();
  acc[3] = acc_read<48>();
  const size_t off = ((size_t)b * S + k0w) * kvstride + (size_t)hk * D;
  // wave-local staging: the loop's closing barrier already retired every tile read
  store_rows_T_wave(acc, 1.f, qd + w * 32 * CH, lane, dv + off, kvstride);
  acc[0] = acc_read<64>();
  acc[1] = acc_read<80>();
  acc[2] = acc_read<96>();
  acc[3] = acc_read<112>();
  store_rows_T_wave(acc, scale, qd + w * 32 * CH, lane, dk + off, kvstride);
  PTO_STAMP(3);
  PTO_RSTAMP(5);
#ifdef PTO_ATTN_STAMPS
  if (lane == 0 && blockIdx.x < 2048) g_pipe_stamps[((size_t)blockIdx.x * 4 + w) * 16 + 6] = (unsigned long long)ntiles;
#endif
}

// ---------------------------------- backward pass 1 (dQ), software-pipelined across key tiles
// The dQ pass in the dK/dV pipeline's form.  NW waves x 32 queries per workgroup (the query on
// the lane): NW = 8 (default, S % 256 == 0: 256 query rows share each K/V tile, two waves per
// SIMD) or NW = 4 (one per SIMD).  Key tiles of KT = 32 keys (K | V, 16 KB) pass through three
// LDS buffers; the dQ^T accumulator is pinned in AGPRs a0-a63 and the wave's Q / dO operands
// (the B operands of S^T and dP^T) in a64-a127, so the compiler's VGPRs fit 128 (NW = 8).
// A tile is 24 MFMA gaps:
//   gaps  0-7   dP^T_t = V_t . dO^T      P_t = exp2(S^T_t c - lse2): fma gap i, exp2 gap i + 1
//   gaps  8-15  S^T_{t+1} = K_{t+1} . Q^T     dS_t = P (dP - delta): subtract gaps 9-16, multiply
//                                              10-17, bf16 pack 11-18
//   gaps 16-23  dQ^T += K_t^T . dS^T_t
// LDS reads LEAD gaps ahead (4 at NW = 4, 2 at NW = 8): V_t rows, K_{t+1} rows, K_t^T
// transposed.  Tile t+2's LDS-DMA goes out in gaps 4-7 and lands by the closing barrier (tile
// t+1 computes S^T_{t+2} from it).  lse2 and delta are per-lane scalars.  A wave past its
// causal diagonal only moves its DMA pieces.  Block order: kv head fastest (the G query heads
// sharing a K/V stream sit 8 blocks apart, on one XCD), heaviest causal query block first.
// Per-element operations and the key order of the dQ accumulation match attn_bwd_dq8_kernel:
// bit-identical dQ and delta.  NW = 8: 247 vs 274 us on the 8B shape
// (profiles/r4_attn_dq_pipe_ab.json); NW = 4 measured equal to attn_bwd_dq8_kernel.
constexpr int KT = 32;
// dQ^T accumulator tile `slot` (0-3) in a[16 slot..]: clobbers only a0-a63, so two waves per
// SIMD fit (NW = 8: 184 VGPRs + 64 AGPRs of the 256 each)
// qf / df (the MFMA B operands of S^T and dP^T, fixed per wave) in a64-a95 / a96-a127, so the
// compiler's VGPRs stay within 128 (two waves per SIMD at NW = 8); every asm statement of this
// kernel clobbers a0-a127 so the compiler keeps nothing of its own there
#define PTO_AGPR_CLOBBERS_64 PTO_AGPR_CLOBBERS
// acc (16 VGPRs) = A . a[B0..B0+3] (+ acc unless FIRST, which starts from 0).  The S^T / dP^T
// chains are read by VALU only gaps later (>= 12 wait states after the chain's last MFMA).
template <int B0, bool FIRST>
__device__ __forceinline__ void mfma_vb(f32x16& acc, const bf16x8& a) {
  if constexpr (FIRST)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, a[%c2:%c3], 0" : "=v"(acc) : "v"(a), "i"(B0), "i"(B0 + 3)
                 : PTO_AGPR_CLOBBERS_64);
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, a[%c2:%c3], %0" : "+v"(acc) : "v"(a), "i"(B0), "i"(B0 + 3)
                 : PTO_AGPR_CLOBBERS_64);
}
// k-step s (a constant after unrolling) of the chain whose B operands start at BASE
template <int BASE>
__device__ __forceinline__ void mfma_vb_step(int s, f32x16& acc, const bf16x8& a) {
  switch (s) {
    case 0: mfma_vb<BASE, true>(acc, a); break;
    case 1: mfma_vb<BASE + 4, false>(acc, a); break;
    case 2: mfma_vb<BASE + 8, false>(acc, a); break;
    case 3: mfma_vb<BASE + 12, false>(acc, a); break;
    case 4: mfma_vb<BASE + 16, false>(acc, a); break;
    case 5: mfma_vb<BASE + 20, false>(acc, a); break;
    case 6: mfma_vb<BASE + 24, false>(acc, a); break;
    default: mfma_vb<BASE + 28, false>(acc, a); break;
  }
}
__device__ __forceinline__ void mfma_dq_slot(int slot, const bf16x8& a, const bf16x8& b) {
  switch (slot) {
    case 0: asm volatile("v_mfma_f32_32x32x16_bf16 a[0:15], %0, %1, a[0:15]" :: "v"(a), "v"(b) : PTO_AGPR_CLOBBERS_64); break;
    case 1: asm volatile("v_mfma_f32_32x32x16_bf16 a[16:31], %0, %1, a[16:31]" :: "v"(a), "v"(b) : PTO_AGPR_CLOBBERS_64); break;
    case 2: asm volatile("v_mfma_f32_32x32x16_bf16 a[32:47], %0, %1, a[32:47]" :: "v"(a), "v"(b) : PTO_AGPR_CLOBBERS_64); break;
    default: asm volatile("v_mfma_f32_32x32x16_bf16 a[48:63], %0, %1, a[48:63]" :: "v"(a), "v"(b) : PTO_AGPR_CLOBBERS_64); break;
  }
}
template <int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_bwd_dq_pipe_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout, const float* __restrict__ lse2,
    float* __restrict__ delta, bf16_t* __restrict__ dq, int B, int S, int Hq, int Hkv, float c, float scale,
    int causal) {
  constexpr int NB = 3, TILE = 2 * KT * CH, BMW = 32 * NW;  // BMW query rows per workgroup
  constexpr int NPW = 8 / NW;  // pieces of one [KT][D] image per wave
  constexpr int LEAD = NW == 8 ? 2 : 4;
  __shared__ u32x4 kvs[NB * TILE > NW * 32 * CH ? NB * TILE : NW * 32 * CH];  // [buf][K | V]; dQ epilogue
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int G = Hq / Hkv, nqb = S / BMW;
  int bi = (int)blockIdx.x;
  const int hk = bi % Hkv;
  bi /= Hkv;
  const int hq = hk * G + bi % G;
  bi /= G;
  const int b = bi % B, qi = bi / B;
  const int qblk = causal ? nqb - 1 - qi : qi;
  const int q0w = qblk * BMW + w * 32, qme = q0w + r;
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
#pragma unroll
  for (int s = 0; s < NDS; ++s) {
    const u32x4 qq = __builtin_bit_cast(u32x4, qf[s]), dd = __builtin_bit_cast(u32x4, df[s]);
    asm volatile("v_accvgpr_write_b32 a[%c4], %0\n\tv_accvgpr_write_b32 a[%c5], %1\n\t"
                 "v_accvgpr_write_b32 a[%c6], %2\n\tv_accvgpr_write_b32 a[%c7], %3"
                 :: "v"(qq.x), "v"(qq.y), "v"(qq.z), "v"(qq.w), "i"(64 + 4 * s), "i"(65 + 4 * s), "i"(66 + 4 * s),
                    "i"(67 + 4 * s) : PTO_AGPR_CLOBBERS_64);
    asm volatile("v_accvgpr_write_b32 a[%c4], %0\n\tv_accvgpr_write_b32 a[%c5], %1\n\t"
                 "v_accvgpr_write_b32 a[%c6], %2\n\tv_accvgpr_write_b32 a[%c7], %3"
                 :: "v"(dd.x), "v"(dd.y), "v"(dd.z), "v"(dd.w), "i"(96 + 4 * s), "i"(97 + 4 * s), "i"(98 + 4 * s),
                    "i"(99 + 4 * s) : PTO_AGPR_CLOBBERS_64);
  }
  asm volatile("s_nop 4" ::: "memory");  // AGPR writes before the first MFMA reading them
  const size_t srow = ((size_t)b * Hq + hq) * S + qme;
  const float lq = lse2[srow];
  if (h == 0) delta[srow] = dl;

  const int ntiles = causal ? (qblk * BMW + BMW) / KT : S / KT;
  const int tdiag = q0w / KT;  // causal: this wave's diagonal tile; later tiles are masked whole

  // LDS-DMA: piece k of a tile (k < NPW: K rows, then V rows); wave w moves pieces w + NW i of
  // the 8 per [KT][D] image
  uint32_t doff[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int e = 64 * (w + NW * i) + lane, row = e / CH, j = e % CH;
    doff[i] = (uint32_t)(row * kvstride) + 8 * (j ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  }
  const bf16_t* kb = k + (size_t)b * S * kvstride + (size_t)hk * D;
  const bf16_t* vb = v + (size_t)b * S * kvstride + (size_t)hk * D;
  const unsigned lds_w = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(kvs + 64 * wu));
  auto dma = [&](int buf, int piece, int t) {
    t = t < ntiles ? t : ntiles - 1;  // past the end: refetch the last tile into a dead buffer
    const int i = piece % NPW;
    const bf16_t* src = (piece < NPW ? kb : vb) + (size_t)t * KT * kvstride + doff[i];
    const unsigned dst = lds_w + 16u * (buf * TILE + (piece < NPW ? 0 : KT * CH) + 64 * NW * i);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                 :: "s"(dst), "v"(src) : "memory", "m0");
  };

  // loop-carried: S^T of the current tile (rotating sets) and V rows 0-3 of the current tile
  f32x16 s0 = zero16(), s1 = zero16(), s2 = zero16();
  bf16x8 va[NDS];
  asm volatile(PTO_ZERO_0_63 ::: PTO_AGPR_CLOBBERS_64);

  auto step = [&](auto curc, auto maskc, f32x16& sin, f32x16& sout, int lim, int t2) {
    constexpr int CUR = decltype(curc)::value, NXT = (CUR + 1) % NB, NN = (CUR + 2) % NB;
    constexpr bool MASK = decltype(maskc)::value;
    const u32x4* Ks = kvs + CUR * TILE;
    const u32x4* Vs = Ks + KT * CH;
    const u32x4* Kn = kvs + NXT * TILE;
    const u32x4* Vn = Kn + KT * CH;
    f32x16 pa;
    bf16x8 ka[NDS], kt[8], db[2];
    uint32_t dw[8];
#pragma unroll
    for (int j = 0; j < 24; ++j) {
      // ---- the gap's MFMA
      if (j < 8) {
        mfma_vb_step<96>(j, pa, va[j]);  // dP^T = V . dO^T
      } else if (j < 16) {
        mfma_vb_step<64>(j - 8, sout, ka[j - 8]);  // S^T = K . Q^T
      } else {  // dQ^T tile (j & 3) += K^T . dS^T, k-step (j - 16) >> 2
        mfma_dq_slot(j & 3, kt[j - 16], db[(j - 16) >> 2]);
      }
      // ---- VALU (no filler depends on another in the same gap)
      if (j < 16) {  // (opaque first: lse2 is loop-invariant, and the compiler would otherwise
                     // hoist all 16 fma into the tile's first gap)
        asm volatile("" : "+v"(sin[j]));
        sin[j] = fmaf(sin[j], c, -lq);
      }
      if (j >= 1 && j <= 16) {
        const int i = j - 1;
        float p = __builtin_amdgcn_exp2f(sin[i]);
        if (MASK && (i & 3) + 8 * (i >> 2) > lim) p = 0.f;  // key > query
        sin[i] = p;
      }
      if (j >= 9 && j < 17) {
        const int m = j - 9;
        pa[2 * m] = pa[2 * m] - dl;
        pa[2 * m + 1] = pa[2 * m + 1] - dl;
      }
      if (j >= 10 && j < 18) {
        const int m = j - 10;
        pa[2 * m] = sin[2 * m] * pa[2 * m];
        pa[2 * m + 1] = sin[2 * m + 1] * pa[2 * m + 1];
      }
      if (j >= 11 && j < 19) {
        const int m = j - 11;
        dw[m] = pk2(pa[2 * m], pa[2 * m + 1]);
        if (m == 3 || m == 7) {
          const int s = m >> 2;
          u32x4 u = {dw[4 * s], dw[4 * s + 1], dw[4 * s + 2], dw[4 * s + 3]};
          db[s] = __builtin_bit_cast(bf16x8, u);
        }
      }
      // ---- LDS reads, LEAD gaps ahead of their MFMA (4 at one wave per SIMD; 2 at two, where
      // the partner wave covers the latency and the registers are scarcer)
      if (j < 8 - LEAD) va[LEAD + j] = row_frag(Vs, r, 2 * (LEAD + j) + h);
      if (j >= 8 - LEAD && j < 16 - LEAD) ka[j - 8 + LEAD] = row_frag(Kn, r, 2 * (j - 8 + LEAD) + h);
      if (j >= 16 - LEAD && j < 24 - LEAD)
        kt[j - 16 + LEAD] = tr_frag(Ks, 16 * ((j - 16 + LEAD) >> 2), ((j - 16 + LEAD) & 3) * 32, lane);
      if (j >= 24 - LEAD) va[j - 24 + LEAD] = row_frag(Vn, r, 2 * (j - 24 + LEAD) + h);
      // ---- tile t + 2 -> buffer NN
      if (j >= 4 && j < 4 + 2 * NPW) dma(NN, j - 4, t2);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  std::integral_constant<bool, true> MK;
  std::integral_constant<bool, false> NM;
  std::integral_constant<int, 0> B0;
  std::integral_constant<int, 1> B1;
  std::integral_constant<int, 2> B2;

  // prologue: tiles 0 and 1 in flight, then S^T_0 and V_0 rows 0-3
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int pc = 0; pc < 2 * NPW; ++pc) dma(t, pc, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  {
    bf16x8 ka[NDS];
#pragma unroll
    for (int s = 0; s < NDS; ++s) ka[s] = row_frag(kvs, r, 2 * s + h);
#pragma unroll
    for (int s = 0; s < LEAD; ++s) va[s] = row_frag(kvs + KT * CH, r, 2 * s + h);
#pragma unroll
    for (int s = 0; s < NDS; ++s) mfma_vb_step<64>(s, s0, ka[s]);
    asm volatile("s_nop 15" ::: "memory");  // S^T_0 complete before the first tile's VALU reads it
  }
  // causal: keys after the query are masked (the diagonal tile per element, later tiles whole)
  auto masked_of = [&](int t) { return causal && t >= tdiag; };  // wave-uniform
  auto lim_of = [&](int t) { return qme - t * KT - 4 * h; };  // t <= tdiag
  auto tile_end = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t + 2 landed
    __syncthreads();
  };
  // tiles after the wave's diagonal (causal) are all masked and come last: the wave only moves
  // its DMA pieces and keeps the barriers (its partner wave on the SIMD runs unslowed)
  auto idle = [&](int nn, int t2) {
#pragma unroll
    for (int pc = 0; pc < 2 * NPW; ++pc) dma(nn, pc, t2);
  };
  for (int t = 0;;) {
    if (causal && t > tdiag) idle(2, t + 2);
    else if (masked_of(t)) step(B0, MK, s0, s1, lim_of(t), t + 2);
    else step(B0, NM, s0, s1, 0, t + 2);
    tile_end();
    if (++t == ntiles) break;
    if (causal && t > tdiag) idle(0, t + 2);
    else if (masked_of(t)) step(B1, MK, s1, s2, lim_of(t), t + 2);
    else step(B1, NM, s1, s2, 0, t + 2);
    tile_end();
    if (++t == ntiles) break;
    if (causal && t > tdiag) idle(1, t + 2);
    else if (masked_of(t)) step(B2, MK, s2, s0, lim_of(t), t + 2);
    else step(B2, NM, s2, s0, 0, t + 2);
    tile_end();
    if (++t == ntiles) break;
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");  // last MFMA drained
  f32x16 acc[NDT];
  acc[0] = acc_read<0>();
  acc[1] = acc_read<16>();
  acc[2] = acc_read<32>();
  acc[3] = acc_read<48>();
  store_rows_T_wave(acc, scale, kvs + w * 32 * CH, lane, dq + ((size_t)b * S + q0w) * qstride + (size_t)hq * D,
                    qstride);
}

}  // namespace

extern "C" int pto_attn_dkdv_pipe(const void* q, const void* k, const void* v, const void* dout, const float* lse2,
                                  const float* delta, void* dk, void* dv, int B, int S, int Hq, int Hkv, float c,
                                  float scale, int causal, int variant, void* stream) {
  if (S % BK != 0 || S % QT != 0 || Hq % Hkv != 0) return -1;
  (void)variant;
  hipLaunchKernelGGL(attn_bwd_dkdv_pipe_kernel, dim3((S / BK) * B * Hkv), dim3(NT), 0, (hipStream_t)stream,
                     (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse2, delta,
                     (bf16_t*)dk, (bf16_t*)dv, B, S, Hq, Hkv, c, scale, causal);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

#ifdef PTO_ATTN_STAMPS
extern "C" int pto_attn_pipe_stamps(void* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pipe_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int pto_attn_dq_pipe(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                const float* lse2, float* delta, void* dq, int B, int S, int Hq, int Hkv, float c,
                                float scale, int causal, void* stream) {
  if (S % BM != 0 || Hq % Hkv != 0) return -1;
  if (S % (2 * BM) == 0)  // 8 waves (256 query rows share each K/V tile), two per SIMD
    hipLaunchKernelGGL(attn_bwd_dq_pipe_kernel<8>, dim3((S / (2 * BM)) * B * Hq), dim3(8 * 64), 0,
                       (hipStream_t)stream, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)o,
                       (const bf16_t*)dout, lse2, delta, (bf16_t*)dq, B, S, Hq, Hkv, c, scale, causal);
  else
    hipLaunchKernelGGL(attn_bwd_dq_pipe_kernel<4>, dim3((S / BM) * B * Hq), dim3(4 * 64), 0, (hipStream_t)stream,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)o, (const bf16_t*)dout,
                       lse2, delta, (bf16_t*)dq, B, S, Hq, Hkv, c, scale, causal);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
