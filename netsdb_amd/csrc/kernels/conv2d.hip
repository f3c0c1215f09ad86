// Fused conv2d (implicit GEMM) on CDNA4 matrix cores — the MI355X realisation of netsDB's
// conv2d_memory_fusion spatial rewriting (reference: src/conv2d_memory_fusion/*:
// ImageToChunks -> ImageChunksToBlock -> ImageBlockToMatrix -> FFTransposeMult -> FFAggMatrix, and
// KernelBiasJoin's "+1 bias column"). The reference materialises the im2col matrix
// (N*OH*OW x C*KH*KW+1) as FFMatrixBlocks in a set and then runs the block GEMM; here the
// im2col rows never exist in HBM: every lane gathers its own MFMA A fragment (8 consecutive
// k of one output pixel) straight from the L2/MALL-resident image, the filter panel sits in
// LDS, and bias (+ optional relu) is applied in the epilogue.
//
//   out[p][oc] = act( sum_k im2col(X)[p][k] * W[oc][k] + bias[oc] ),  p = (n, oh, ow)
//
// Block = 256 threads = 4 waves; tile = 128 pixels x 64 output channels; each wave owns
// 32 pixels x 64 channels = 2 x 4 mfma_f32_16x16x32_bf16 accumulators.
#include "common.h"
#include <algorithm>
#include <type_traits>

namespace nsdb {

constexpr int CV_BM = 128, CV_BN = 64, CV_KC = 256;      // K staged in LDS in chunks of 256 (36 KB LDS -> 4 blocks/CU)
constexpr int CV_WROW = CV_KC * 2 + 16;                   // padded LDS row (bytes) of the filter panel

struct ConvParams {
  const unsigned short* X;   // bf16 [N][C][H][W]
  const unsigned short* Wt;  // bf16 [OC][ldw]   (im2col column order: c, kh, kw)
  const float* bias;         // f32 [OC] or null
  void* out;                 // bf16/f32, NHWC-matrix [N*OH*OW][OC] or NCHW [N][OC][OH][OW]
  int N, C, H, W, OC, KH, KW, OH, OW;
  int stride, pad, dil;
  int K, ldw;
  int act, nchw_out, out_f32;
};

__global__ void __launch_bounds__(256, 4) conv2d_igemm_kernel(ConvParams p) {
  __shared__ __attribute__((aligned(16))) char smem[CV_BN * CV_WROW + CV_KC * 8];
  char* wpanel = smem;
  int* koff = reinterpret_cast<int*>(smem + CV_BN * CV_WROW);          // per-k image offset
  int* khw = koff + CV_KC;                                             // (kh*dil)<<16 | (kw*dil)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long P = (long long)p.N * p.OH * p.OW;
  const long long p0 = (long long)blockIdx.x * CV_BM;
  const int oc0 = blockIdx.y * CV_BN;
  const int HW = p.H * p.W, KHW = p.KH * p.KW;

  // per-lane pixel coordinates for the wave's two 16-pixel m-tiles
  int pix_base[2], ih0[2], iw0[2];
  bool pix_ok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long pp = p0 + wave * 32 + i * 16 + (lane & 15);
    pix_ok[i] = pp < P;
    const long long q = pix_ok[i] ? pp : 0;
    const int n = (int)(q / (p.OH * p.OW));
    const int rem = (int)(q % (p.OH * p.OW));
    const int oh = rem / p.OW, ow = rem % p.OW;
    ih0[i] = oh * p.stride - p.pad;
    iw0[i] = ow * p.stride - p.pad;
    pix_base[i] = n * p.C * HW;
  }

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(p.X), (short)0, (int)((long long)p.N * p.C * HW * 2), 0x00020000);

  for (int kc = 0; kc < p.K; kc += CV_KC) {
    const int klen = min(CV_KC, p.K - kc);
    const int klen32 = (klen + 31) & ~31;
    __syncthreads();
    // filter panel [64][klen32] -> LDS (16-B vector loads; zero past K / OC)
    const int chunks_per_row = klen32 / 8;
    for (int e = tid; e < CV_BN * chunks_per_row; e += 256) {
      const int r = e / chunks_per_row, ch = e % chunks_per_row;
      const int oc = oc0 + r, k = kc + ch * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (oc < p.OC && k < p.ldw) v = *reinterpret_cast<const uint4*>(p.Wt + (long long)oc * p.ldw + k);
      *reinterpret_cast<uint4*>(wpanel + r * CV_WROW + ch * 16) = v;
    }
    for (int k = tid; k < klen32; k += 256) {
      const int kg = kc + k;
      if (kg < p.K) {
        const int c = kg / KHW, r2 = kg % KHW, kh = r2 / p.KW, kw = r2 % p.KW;
        koff[k] = c * HW + kh * p.dil * p.W + kw * p.dil;
        khw[k] = ((kh * p.dil) << 16) | (kw * p.dil);
      } else {
        koff[k] = 0;
        khw[k] = 0x7fff7fff;   // always out of bounds -> contributes 0
      }
    }
    __syncthreads();

    // software-pipelined gather: the 16 loads of k-step t+1 are issued before step t's MFMAs and
    // only packed into the bf16x8 fragment after them (sched_barrier keeps the pack below)
    auto gather = [&](int ks, unsigned (&raw)[2][8]) {
      const int kb = ks + 8 * (lane >> 4);
      // (kh, kw) and image offsets of this lane's 8 k values: 4 x ds_read_b128 (16 lanes share them)
      const int4 ko0 = *reinterpret_cast<const int4*>(koff + kb), ko1 = *reinterpret_cast<const int4*>(koff + kb + 4);
      const int4 hw0 = *reinterpret_cast<const int4*>(khw + kb), hw1 = *reinterpret_cast<const int4*>(khw + kb + 4);
      const int ko[8] = {ko0.x, ko0.y, ko0.z, ko0.w, ko1.x, ko1.y, ko1.z, ko1.w};
      const int hw[8] = {hw0.x, hw0.y, hw0.z, hw0.w, hw1.x, hw1.y, hw1.z, hw1.w};
      // buffer loads: a masked lane gets an out-of-range offset and the descriptor's range check
      // returns 0 -> no select after the load and no branch around it
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int base = pix_base[i] + ih0[i] * p.W + iw0[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ih = ih0[i] + (hw[j] >> 16), iw = iw0[i] + (hw[j] & 0xffff);
          const bool ok = pix_ok[i] & ((unsigned)ih < (unsigned)p.H) & ((unsigned)iw < (unsigned)p.W);
          const int off = ok ? (base + ko[j]) * 2 : 0x7ffffff0;
          raw[i][j] = __builtin_amdgcn_raw_buffer_load_b16(xr, off, 0, 0);
        }
      }
    };
    auto pack = [&](const unsigned (&raw)[2][8], bf16x8 (&af)[2]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) af[i][j] = (short)raw[i][j];
    };
    unsigned raw[2][8];
    bf16x8 cur[2];
    gather(0, raw);
    pack(raw, cur);
    for (int ks = 0; ks < klen32; ks += 32) {
      const bool more = ks + 32 < klen32;
      if (more) gather(ks + 32, raw);
      __builtin_amdgcn_sched_barrier(0);
      const int kb = ks + 8 * (lane >> 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(wpanel + (j * 16 + (lane & 15)) * CV_WROW + kb * 2);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[i], bfr, acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (more) pack(raw, cur);
    }
  }

  // epilogue: col (oc) = lane&15, row (pixel) = (lane>>4)*4 + r. NCHW: the lane's 4 pixels are
  // consecutive in one output plane -> one 8-byte (bf16) / 16-byte (f32) store when they share an image.
  const long long OHW = (long long)p.OH * p.OW;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int oc = oc0 + j * 16 + (lane & 15);
    if (oc >= p.OC) continue;
    const float b = p.bias ? p.bias[oc] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long long pp0 = p0 + wave * 32 + i * 16 + (lane >> 4) * 4;
      float vv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) vv[r] = apply_act(acc[i][j][r] + b, p.act);
      if (p.nchw_out) {
        const long long n0 = pp0 / OHW, rem0 = pp0 % OHW;
        if (pp0 + 3 < P && rem0 + 3 < OHW) {
          const long long off = (n0 * p.OC + oc) * OHW + rem0;
          if (p.out_f32) {
            float* o = reinterpret_cast<float*>(p.out) + off;
            if ((off & 3) == 0) *reinterpret_cast<float4*>(o) = make_float4(vv[0], vv[1], vv[2], vv[3]);
            else { o[0] = vv[0]; o[1] = vv[1]; o[2] = vv[2]; o[3] = vv[3]; }
          } else {
            unsigned short* o = reinterpret_cast<unsigned short*>(p.out) + off;
            const unsigned lo = f32_to_bf16(vv[0]) | ((unsigned)f32_to_bf16(vv[1]) << 16);
            const unsigned hi = f32_to_bf16(vv[2]) | ((unsigned)f32_to_bf16(vv[3]) << 16);
            if ((off & 3) == 0) *reinterpret_cast<uint2*>(o) = make_uint2(lo, hi);
            else if ((off & 1) == 0) { reinterpret_cast<unsigned*>(o)[0] = lo; reinterpret_cast<unsigned*>(o)[1] = hi; }
            else { o[0] = (unsigned short)lo; o[1] = (unsigned short)(lo >> 16); o[2] = (unsigned short)hi; o[3] = (unsigned short)(hi >> 16); }
          }
          continue;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long pp = pp0 + r;
        if (pp >= P) continue;
        long long off;
        if (p.nchw_out) {
          const long long n = pp / OHW, rem = pp % OHW;
          off = (n * p.OC + oc) * OHW + rem;
        } else {
          off = pp * p.OC + oc;
        }
        if (p.out_f32) reinterpret_cast<float*>(p.out)[off] = vv[r];
        else reinterpret_cast<unsigned short*>(p.out)[off] = f32_to_bf16(vv[r]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Row-tiled direct conv for small-C / wide-image layers (the memfuse headline: 3 -> 64, 7x7,
// stride 1, pad 0 on 112x112). The generic kernel above gathers one bf16 per lane per k (TA-bound:
// ~2.8M scalar-gather wave instructions for the headline shape). Here:
//  * a block owns TR=4 consecutive output rows of one image (one per wave) and stages the
//    C x (TR+KH-1) input rows it needs into LDS ONCE, as 4 copies shifted by 0..3 elements, so the
//    8 taps (kw = 0..7, KW <= 8 zero-padded) of a (c, kh) filter row at any output column are one
//    8-byte-aligned pair of ds_read_b64 — the MFMA A fragment comes straight out of LDS;
//  * K is re-ordered to (c, kh, kw8): k-step = 4 (c, kh) rows x 8 taps = 32 = one
//    mfma_f32_16x16x32_bf16; the re-ordered filter (4 n-tiles x NKS k-steps) lives in VGPRs for the
//    whole (persistent) block;
//  * copy stride 288 B and the 4-copy interleave make a wave's ds_read_b64 bank-conflict free
//    (16 lanes of one (c,kh) row cover 128 B, the next row is +128 B mod 256);
//  * the block's [64 oc][4 rows][OW] bf16 output tile is staged through LDS segment-major and written as one
//    contiguous run per oc (the 4 output rows of a plane are adjacent in NCHW) with coalesced 8-byte stores
//    (the store tail is issue-bound: 8 B/lane halves the instructions of dword stores); per-lane
//    fragment stores into 64 different planes were the limit of the gather kernel (~1 TB/s).
// Preconditions (host-checked): stride 1, dil 1, pad 0, KW <= 8, W % 8 == 0, OW <= 112,
// C*KH <= 4*CVR_NKS, C*(4+KH-1) <= CVR_ROWS.
constexpr int CVR_TR = 4, CVR_NKS = 6, CVR_CP = 288;                 // rows/block, max k-steps, copy stride (B)
constexpr int CVR_ROWS = 30;                                           // max (c, r) input rows per group
constexpr int CVR_ZERO = CVR_ROWS * 4 * CVR_CP;                        // zero block (A source past C*KH)
constexpr int CVR_BUF = CVR_ZERO + 4 * CVR_CP;
constexpr int CVR_MAXT = 7;                                            // output tiles of 16 per row (OW <= 112)
constexpr int CVR_OSTAGE = 32 * CVR_TR * (16 * CVR_MAXT + 4) * 2;      // [TR][32 oc][OWS] bf16 (one half)
constexpr int CVR_WROW = CVR_NKS * 4 * 16 + 16;                       // staged filter row (B)
constexpr int CVR_TRASH = 64;                                          // sink for masked epilogue LDS writes

struct ConvRowParams {
  const unsigned short* X;
  const unsigned short* Wt;
  const float* bias;
  void* out;
  int N, C, H, W, OC, KH, KW, OH, OW, ldw;
  int rin, ckh, nks, ntiles, chunks, groups_per_img, ngroups;
  int act, nchw_out, out_f32;
  int segs, vec8;  // staged output: LDS run stride per oc (elements); 8-B output chunks allowed
  int contig;      // full-row kernel: each block walks a contiguous run of row groups (same image, consecutive
                   // rows: every plane's output grows as one sequential stream) instead of a grid stride
  const unsigned short* Wfrag;   // warp-specialised kernel: the filter pre-packed in MFMA B-fragment order
                                 // [OC/64][4 n-tiles][6 k-steps][64 lanes][8] bf16 (ops.conv_filter_fragments)
  int variant;   // diagnostics (bit flags, timing only): 1 no global stores, 2 no MFMA, 4 no LDS output
                 // staging, 8 prologue only, 16 no compute, 32 s_memtime stamps over the output
};

// STAGED (LDS-staged NCHW bf16 output) and the diagnostics switch are template parameters: a runtime
// flag here made hipcc wrap every MFMA of the inner loop in its own branch (+ s_nop padding).
// DIAG = false compiles every diagnostic test to a constant.
template <int ACT, bool STAGED, bool DIAG>
__global__ void __launch_bounds__(256, 2) conv2d_rows_kernel(ConvRowParams p) {
  const int var = DIAG ? p.variant : 0;
  __shared__ __attribute__((aligned(16))) char smem[CVR_BUF + CVR_OSTAGE + CVR_TRASH];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc0 = blockIdx.y * 64;

  // ---- filter -> VGPRs (B fragments in (c*KH+kh, kw8) k order): raw [64][ldw] rows staged into LDS with
  // independent 16-B loads (<= 6 per thread, all in flight together), then each lane picks its taps
  {
    const int cpr = p.ldw / 8, nch = 64 * cpr;
    uint4 v[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = tid + u * 256;
      const int r = e / cpr, ch = e - (e / cpr) * cpr;
      v[u] = make_uint4(0, 0, 0, 0);
      if (e < nch && oc0 + r < p.OC) v[u] = *reinterpret_cast<const uint4*>(p.Wt + (long long)(oc0 + r) * p.ldw + ch * 8);
    }
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = tid + u * 256;
      if (e < nch) reinterpret_cast<uint4*>(smem)[e] = v[u];
    }
  }
  __syncthreads();
  bf16x8 bw[4][CVR_NKS];
  {
    const unsigned short* raw = reinterpret_cast<const unsigned short*>(smem);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int ks = 0; ks < CVR_NKS; ++ks) {
        const int ocl = nt * 16 + (lane & 15), q = ks * 4 + (lane >> 4);
#pragma unroll
        for (int kw = 0; kw < 8; ++kw)
          bw[nt][ks][kw] = (q < p.ckh && kw < p.KW) ? (short)raw[ocl * p.ldw + q * p.KW + kw] : (short)0;
      }
  }
  float bias_v[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int oc = oc0 + nt * 16 + (lane & 15);
    bias_v[nt] = (p.bias && oc < p.OC) ? p.bias[oc] : 0.f;
  }
  __syncthreads();

  // zero block at the end of both buffers (the A source of k-steps past C*KH)
  for (int e = tid; e < 4 * CVR_CP / 16; e += 256)
    reinterpret_cast<uint4*>(smem + CVR_ZERO)[e] = make_uint4(0, 0, 0, 0);

  // per-lane A base offsets for each k-step (relative to a buffer), wave row folded in
  int abase[CVR_NKS];
#pragma unroll
  for (int ks = 0; ks < CVR_NKS; ++ks) {
    const int q = ks * 4 + (lane >> 4);
    if (q < p.ckh) {
      const int c = q / p.KH, kh = q % p.KH;
      abase[ks] = ((c * p.rin + wave + kh) * 4 + (lane & 3)) * CVR_CP + (lane & 12) * 2;
    } else {
      abase[ks] = CVR_ZERO + (lane & 3) * 16 + (lane & 12) * 2;   // inside the zero block
    }
  }

  // input staging work items: (c, r, chunk j); each thread handles <= 2 items per group
  const int items = p.C * p.rin * p.chunks;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(p.X), (short)0, (int)((long long)p.N * p.C * p.H * p.W * 2), 0x00020000);
  u32x4 lo[2];
  u32x2 hi[2];
  // per-thread staging items are the same for every group: precompute their image-relative byte offsets
  // and validity once (a per-group div/mod + 64-bit mad chain here sat between the prefetch loads and made
  // hipcc wait for them in place)
  int it_off[2], it_r[2];
  bool it_lo[2], it_hi[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int it = min(tid + u * 256, items - 1);
    const int j = it % p.chunks, cr = it / p.chunks, r = cr % p.rin, c = cr / p.rin;
    it_off[u] = ((c * p.H + r) * p.W + 8 * j) * 2;
    it_r[u] = r;
    it_lo[u] = 8 * j < p.W;
    it_hi[u] = 8 * (j + 1) < p.W;
  }
  // branch-free: an invalid chunk gets an out-of-range offset and the buffer range check returns
  // zeros (a branch around each load makes hipcc wait vmcnt(0) right after it — no prefetch)
  auto fetch = [&](int g) {
    const bool gok = g < p.ngroups;
    const int n = g / p.groups_per_img, oh0 = (g % p.groups_per_img) * CVR_TR;
    const int gbase = ((n * p.C * p.H) + oh0) * p.W * 2;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool rok = gok && oh0 + it_r[u] < p.H;
      const int o = gbase + it_off[u];
      lo[u] = __builtin_amdgcn_raw_buffer_load_b128(xr, (rok && it_lo[u]) ? o : 0x7ffffff0, 0, 0);
      hi[u] = __builtin_amdgcn_raw_buffer_load_b64(xr, (rok && it_hi[u]) ? o + 16 : 0x7ffffff0, 0, 0);
    }
  };
  auto store_rows = [&](char* buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = tid + u * 256;
      if (it >= items) continue;
      const int j = it % p.chunks, cr = it / p.chunks;
      char* row = buf + cr * 4 * CVR_CP + j * 16;
      const unsigned w[6] = {lo[u].x, lo[u].y, lo[u].z, lo[u].w, hi[u].x, hi[u].y};
      // shift s (elements) = 2s bytes: copy s holds in[e + s] at entry e
      *reinterpret_cast<u32x4*>(row) = lo[u];
      *reinterpret_cast<u32x4*>(row + CVR_CP) =
          u32x4{__builtin_amdgcn_alignbyte(w[1], w[0], 2), __builtin_amdgcn_alignbyte(w[2], w[1], 2),
                     __builtin_amdgcn_alignbyte(w[3], w[2], 2), __builtin_amdgcn_alignbyte(w[4], w[3], 2)};
      *reinterpret_cast<u32x4*>(row + 2 * CVR_CP) = u32x4{w[1], w[2], w[3], w[4]};
      *reinterpret_cast<u32x4*>(row + 3 * CVR_CP) =
          u32x4{__builtin_amdgcn_alignbyte(w[2], w[1], 2), __builtin_amdgcn_alignbyte(w[3], w[2], 2),
                     __builtin_amdgcn_alignbyte(w[4], w[3], 2), __builtin_amdgcn_alignbyte(w[5], w[4], 2)};
    }
  };

  const long long OHW = (long long)p.OH * p.OW;
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      p.out, (short)0, (int)std::min<long long>((long long)p.N * p.OC * OHW * (p.out_f32 ? 4 : 2), 0x7fffffffLL),
      0x00020000);
  unsigned short* ostage = reinterpret_cast<unsigned short*>(smem + CVR_BUF);   // [32 oc][segs] bf16
  constexpr bool staged = STAGED;
  // stage layout "segment-major" [32 oc][segs]: the TR output rows of one oc plane are adjacent in
  // NCHW, so each oc's rows_valid*OW outputs are ONE contiguous run both in LDS and in HBM and a
  // wave moves it with 8-B (4-pixel) loads/stores. segs = 4*OW rounded so that segs/2 dwords is
  // 2 mod 4: the 16 oc a ds_write lane group touches land on 16 distinct banks.
  const int segs = p.segs;
  int g = blockIdx.x;
  if (var & 8) return;          // diagnostics: prologue only
  // variant 7: s_memtime stamps (diagnostic build: written over the start of the output)
  unsigned long long st_t0 = 0, st_stage = 0, st_work = 0, st_tmp = 0, st_comp = 0, st_bar = 0;
  auto stamp = [&]() -> unsigned long long {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
  };
  if (var & 32) st_t0 = stamp();
  if (g < p.ngroups) {
    fetch(g);
    store_rows(smem);                                  // first group staged before the loop (one drain)
  }
  for (; g < p.ngroups; g += gridDim.x) {
    const int n = g / p.groups_per_img, oh0 = (g % p.groups_per_img) * CVR_TR, oh = oh0 + wave;
    if (var & 32) st_tmp = stamp();
    __syncthreads();                                   // this group's staged input rows are visible
    if (var & 32) { const unsigned long long t = stamp(); st_stage += t - st_tmp; st_tmp = t; }
    // next group's rows in flight during compute and the output stores; staged into LDS at the END of
    // this iteration. Issued unconditionally (past the last group every offset is out of range), so the
    // loads consumed in an iteration are always the ones issued at its top, followed by exactly the
    // group's output stores: hipcc waits vmcnt(<stores>) for them instead of draining the output stores
    fetch(g + gridDim.x);
    // two passes over the row, 32 output channels each: the [32 oc][TR][OWS] bf16 stage is 28 KB, so
    // two blocks fit a CU (the A fragments are re-read from LDS for the second half — cheap)
    const int rows_valid = min(CVR_TR, p.OH - oh0);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (!staged && half == 1) break;
      if (oh < p.OH && !(var & 16)) {
        auto load_a = [&](int t, bf16x8 (&af)[CVR_NKS]) {
#pragma unroll
          for (int ks = 0; ks < CVR_NKS; ++ks) {
            const uint2* a = reinterpret_cast<const uint2*>(__builtin_assume_aligned(smem + abase[ks] + t * 32, 8));
            const uint2 a0 = a[0], a1 = a[1];
            af[ks][0] = (short)a0.x; af[ks][1] = (short)(a0.x >> 16); af[ks][2] = (short)a0.y; af[ks][3] = (short)(a0.y >> 16);
            af[ks][4] = (short)a1.x; af[ks][5] = (short)(a1.x >> 16); af[ks][6] = (short)a1.y; af[ks][7] = (short)(a1.y >> 16);
          }
        };
        // A fragments of tile t+1 are read from LDS while tile t's MFMAs run (software pipeline; the
        // 16x16x32 MFMA issues back to back on one accumulator chain, so one chain per n-tile)
        bf16x8 af[CVR_NKS];
        load_a(0, af);
        for (int t = 0; t < p.ntiles; ++t) {
          f32x4 acc[4];
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (!(var & 2)) {
#pragma unroll
            for (int ks = 0; ks < CVR_NKS; ++ks)
#pragma unroll
              for (int nt = 0; nt < 4; ++nt)
                if (!staged || (nt >> 1) == half)
                  acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], bw[nt][ks], acc[nt], 0, 0, 0);
          } else {
#pragma unroll
            for (int ks = 0; ks < CVR_NKS; ++ks) acc[0][0] += (float)af[ks][0];
          }
          if (t + 1 < p.ntiles) load_a(t + 1, af);
          const int owb = t * 16 + (lane >> 4) * 4;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            if (staged && (nt >> 1) != half) continue;
            const int ocl = nt * 16 + (lane & 15);
            const int oc = oc0 + ocl;
            float vv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) vv[r] = act_t<ACT>(acc[nt][r] + bias_v[nt]);
            if (staged) {
              if (!(var & 4)) {   // [ocl - 32*half][row*OW + ow]: 2 dword writes (OW even -> 4-B aligned)
                // branch-free: a pixel pair past OW is written to the trash word (a branch per write made
                // hipcc split the tile epilogue into 8 exec-masked blocks)
                unsigned* dst = reinterpret_cast<unsigned*>(ostage + (ocl - 32 * half) * segs + wave * p.OW + owb);
                unsigned* trash = reinterpret_cast<unsigned*>(smem + CVR_BUF + CVR_OSTAGE);
                *(owb + 1 < p.OW ? dst : trash) = pack_bf16x2(vv[0], vv[1]);
                *(owb + 3 < p.OW ? dst + 1 : trash) = pack_bf16x2(vv[2], vv[3]);
              } else {
                acc[0][0] += vv[1];
              }
            } else if (oc < p.OC) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                if (owb + r >= p.OW) continue;
                const long long off = p.nchw_out ? ((long long)n * p.OC + oc) * OHW + (long long)oh * p.OW + owb + r
                                                 : (((long long)n * p.OH + oh) * p.OW + owb + r) * p.OC + oc;
                if (p.out_f32) reinterpret_cast<float*>(p.out)[off] = vv[r];
                else reinterpret_cast<unsigned short*>(p.out)[off] = f32_to_bf16(vv[r]);
              }
            }
          }
        }
      }
      if (!staged) break;
      if (var & 32) { const unsigned long long t = stamp(); st_comp += t - st_tmp; st_tmp = t; }
      __syncthreads();
      if (var & 32) { const unsigned long long t = stamp(); st_bar += t - st_tmp; st_tmp = t; }
      if (!(var & 1)) {
        // one contiguous run of seg = rows_valid*OW outputs per oc plane; wave w stores oc w, w+4, ..
        // (all LDS reads first, then the stores: a read->store pair per oc would expose the LDS latency)
        const int noc = min(32, p.OC - (oc0 + 32 * half));
        const int seg = rows_valid * p.OW;
        const int obase = (int)((((long long)n * p.OC + oc0 + 32 * half) * OHW + (long long)oh0 * p.OW) * 2);
        {
          // 8-B chunks (plane and row offsets are 8-B aligned and every run is a multiple of 4 pixels:
          // host checked OH*OW % 4 == 0 and (OH % 4) * OW % 4 == 0)
          const int n4 = seg >> 2;
          uint2 v[8][2];
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              v[j][h] = *reinterpret_cast<const uint2*>(ostage + (wave + 4 * j) * segs + 4 * min(lane + 64 * h, n4 - 1));
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int ocl = wave + 4 * j, q = lane + 64 * h;
              const int off = (ocl < noc && q < n4) ? obase + (int)(ocl * OHW * 2) + 8 * q : 0x7ffffff0;
              __builtin_amdgcn_raw_buffer_store_b64(u32x2{v[j][h].x, v[j][h].y}, orsrc, off, 0, 0);
            }
        }
      }
      __syncthreads();
    }
    if (!staged) __syncthreads();                      // (the staged half loop ends with a barrier)
    store_rows(smem);
    if (var & 32) st_work += stamp() - st_tmp;
  }
  if ((var & 32) && lane == 0) {
    unsigned long long* d = reinterpret_cast<unsigned long long*>(p.out) + (blockIdx.x * 4 + wave) * 4;
    d[0] = stamp() - st_t0; d[1] = st_stage; d[2] = st_comp; d[3] = st_bar;
  }
}

// ---------------------------------------------------------------------------------------------
// Full-row variant of the row-tiled conv (the headline 3 -> 64, 7x7 on 112^2: 7 pixel tiles per output row).
// conv2d_rows_kernel above computes each 16-pixel tile as two 6-deep dependent MFMA chains (32 oc per pass,
// two passes) with the epilogue right behind the last MFMA, at 2 waves/SIMD: its inner loop is latency-bound
// (~30 % MFMA issue). Here ONE wave per SIMD (1 block of 4 waves per CU, 512 registers per lane):
//  * a wave owns one output row x all 64 oc: 7 tiles x 4 n-tiles = 28 independent accumulator chains, so the
//    6 k-steps issue 28 back-to-back MFMAs each; the A fragments of k-step ks+1 (7 ds_read pairs) are read
//    while k-step ks's MFMAs run (register double buffer);
//  * epilogue (bias + act -> bf16) into ONE [64 oc][segs] LDS image of the block's 4 rows, then every oc's
//    4-row run (contiguous in NCHW) leaves as 8-B coalesced stores. The stores of group g drain while group
//    g+1's MFMAs run: the next group's input rows are fetched BEFORE them (the wait for that fetch never
//    waits for the stores), and only two barriers per group separate the LDS phases;
//  * segs = 2 x (64k + 36) bf16: the ds_write_b32 lane groups (16 oc rows x {+0, +2 dwords}) hit 32 distinct
//    banks.
// Input staging (4 shifted copies per (c, r) row) and the filter-in-VGPRs layout are the row kernel's.
constexpr int CVF_NT = 7;                                            // pixel tiles per row (OW 97..112)
constexpr int CVF_SEGS = 2 * (64 * 3 + 36);                          // 456 >= 4 * 112 - pad
constexpr int CVF_STAGE = 2 * 64 * CVF_SEGS * 2;                     // 2 x [64 oc][segs] bf16 (PIPE: double)
template <int ACT, bool DIAG, bool PIPE>
__global__ void __launch_bounds__(256, 1) conv2d_rowfull_kernel(ConvRowParams p) {
  // DIAG: s_memtime phase stamps per wave (timing build, written over the output): total, MFMA, epilogue,
  // mid barrier, stores, input staging
  unsigned long long tt[6] = {0, 0, 0, 0, 0, 0}, t_prev = 0;
  auto stamp = [&](int slot) {
    if constexpr (DIAG) {
      unsigned long long t;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      __builtin_amdgcn_sched_barrier(0);
      if (slot >= 0) tt[slot] += t - t_prev;
      t_prev = t;
    }
  };
  stamp(-1);
  const unsigned long long t_start = t_prev;
  __shared__ __attribute__((aligned(16))) char smem[CVR_BUF + CVF_STAGE + CVR_TRASH];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oc0 = blockIdx.y * 64;

  // ---- filter -> VGPRs (as conv2d_rows_kernel)
  {
    const int cpr = p.ldw / 8, nch = 64 * cpr;
    uint4 v[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = tid + u * 256;
      const int r = e / cpr, ch = e - (e / cpr) * cpr;
      v[u] = make_uint4(0, 0, 0, 0);
      if (e < nch && oc0 + r < p.OC) v[u] = *reinterpret_cast<const uint4*>(p.Wt + (long long)(oc0 + r) * p.ldw + ch * 8);
    }
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = tid + u * 256;
      if (e < nch) reinterpret_cast<uint4*>(smem)[e] = v[u];
    }
  }
  __syncthreads();
  bf16x8 bw[4][CVR_NKS];
  {
    const unsigned short* raw = reinterpret_cast<const unsigned short*>(smem);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int ks = 0; ks < CVR_NKS; ++ks) {
        const int ocl = nt * 16 + (lane & 15), q = ks * 4 + (lane >> 4);
#pragma unroll
        for (int kw = 0; kw < 8; ++kw)
          bw[nt][ks][kw] = (q < p.ckh && kw < p.KW) ? (short)raw[ocl * p.ldw + q * p.KW + kw] : (short)0;
      }
  }
  float bias_v[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int oc = oc0 + nt * 16 + (lane & 15);
    bias_v[nt] = (p.bias && oc < p.OC) ? p.bias[oc] : 0.f;
  }
  __syncthreads();
  for (int e = tid; e < 4 * CVR_CP / 16; e += 256)
    reinterpret_cast<uint4*>(smem + CVR_ZERO)[e] = make_uint4(0, 0, 0, 0);

  int abase[CVR_NKS];
#pragma unroll
  for (int ks = 0; ks < CVR_NKS; ++ks) {
    const int q = ks * 4 + (lane >> 4);
    if (q < p.ckh) {
      const int c = q / p.KH, kh = q % p.KH;
      abase[ks] = ((c * p.rin + wave + kh) * 4 + (lane & 3)) * CVR_CP + (lane & 12) * 2;
    } else {
      abase[ks] = CVR_ZERO + (lane & 3) * 16 + (lane & 12) * 2;
    }
  }

  // input staging work items (c, r, chunk j), <= 2 per thread, identical for every group
  const int items = p.C * p.rin * p.chunks;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(p.X), (short)0, (int)((long long)p.N * p.C * p.H * p.W * 2), 0x00020000);
  u32x4 lo[2][2];      // [fetch slot][item]: two groups' rows in flight (slot = group parity)
  u32x2 hi[2][2];
  int it_off[2], it_r[2];
  bool it_lo[2], it_hi[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int it = min(tid + u * 256, items - 1);
    const int j = it % p.chunks, cr = it / p.chunks, r = cr % p.rin, c = cr / p.rin;
    it_off[u] = ((c * p.H + r) * p.W + 8 * j) * 2;
    it_r[u] = r;
    it_lo[u] = 8 * j < p.W;
    it_hi[u] = 8 * (j + 1) < p.W;
  }
  // group walk: grid stride, or (contig) one contiguous run of row groups per block
  const int per = p.contig ? (p.ngroups + gridDim.x - 1) / gridDim.x : 0;
  int g0 = p.contig ? blockIdx.x * per : blockIdx.x;
  const int gstep = p.contig ? 1 : gridDim.x;
  const int gend = p.contig ? min(p.ngroups, g0 + per) : p.ngroups;
  auto fetch = [&](int g, auto SLOT) {
    constexpr int sl = decltype(SLOT)::value;
    const bool gok = g < gend;
    const int n = g / p.groups_per_img, oh0 = (g % p.groups_per_img) * CVR_TR;
    const int gbase = ((n * p.C * p.H) + oh0) * p.W * 2;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool rok = gok && oh0 + it_r[u] < p.H;
      const int o = gbase + it_off[u];
      lo[sl][u] = __builtin_amdgcn_raw_buffer_load_b128(xr, (rok && it_lo[u]) ? o : 0x7ffffff0, 0, 0);
      hi[sl][u] = __builtin_amdgcn_raw_buffer_load_b64(xr, (rok && it_hi[u]) ? o + 16 : 0x7ffffff0, 0, 0);
    }
  };
  auto store_rows = [&](auto SLOT) {
    constexpr int sl = decltype(SLOT)::value;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = tid + u * 256;
      if (it >= items) continue;
      const int j = it % p.chunks, cr = it / p.chunks;
      char* row = smem + cr * 4 * CVR_CP + j * 16;
      const unsigned w[6] = {lo[sl][u].x, lo[sl][u].y, lo[sl][u].z, lo[sl][u].w, hi[sl][u].x, hi[sl][u].y};
      *reinterpret_cast<u32x4*>(row) = lo[sl][u];
      *reinterpret_cast<u32x4*>(row + CVR_CP) =
          u32x4{__builtin_amdgcn_alignbyte(w[1], w[0], 2), __builtin_amdgcn_alignbyte(w[2], w[1], 2),
                __builtin_amdgcn_alignbyte(w[3], w[2], 2), __builtin_amdgcn_alignbyte(w[4], w[3], 2)};
      *reinterpret_cast<u32x4*>(row + 2 * CVR_CP) = u32x4{w[1], w[2], w[3], w[4]};
      *reinterpret_cast<u32x4*>(row + 3 * CVR_CP) =
          u32x4{__builtin_amdgcn_alignbyte(w[2], w[1], 2), __builtin_amdgcn_alignbyte(w[3], w[2], 2),
                __builtin_amdgcn_alignbyte(w[4], w[3], 2), __builtin_amdgcn_alignbyte(w[5], w[4], 2)};
    }
  };

  const long long OHW = (long long)p.OH * p.OW;
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      p.out, (short)0, (int)std::min<long long>((long long)p.N * p.OC * OHW * 2, 0x7fffffffLL), 0x00020000);
  unsigned short* ostage = reinterpret_cast<unsigned short*>(smem + CVR_BUF);
  unsigned* const trash = reinterpret_cast<unsigned*>(smem + CVR_BUF + CVF_STAGE);

  // one output chunk of the group held in stage `st`: oc (wave + 4 j), 8-byte piece q = lane + 64 h of its
  // rows_valid * OW run (c = 2 j + h); pieces past the run / oc past OC go to an out-of-range offset (dropped)
  auto chunk_read = [&](const unsigned short* st, int c, int n4) -> uint2 {
    const int j = c >> 1, h = c & 1;
    return *reinterpret_cast<const uint2*>(st + (wave + 4 * j) * CVF_SEGS + 4 * min(lane + 64 * h, n4 - 1));
  };
  auto chunk_store = [&](uint2 v, int c, int obase, int n4, int noc) {
    const int j = c >> 1, h = c & 1;
    const int ocl = wave + 4 * j, q = lane + 64 * h;
    const int off = (ocl < noc && q < n4) ? obase + (int)(ocl * OHW * 2) + 8 * q : 0x7ffffff0;
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, orsrc, off, 0, 0);
  };
  const int noc = min(64, p.OC - oc0);
  // the previous group's stores (PIPE: issued between this group's MFMA blocks; n4 = 0 before the first group)
  int prev_obase = 0, prev_n4 = 0;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  int g = g0;
  // input rows are fetched TWO groups ahead (slot = group parity): a load queues behind the stores issued
  // before it on the CU, so the rows consumed at the end of group g were requested before group g-1's stores
  // (one group ahead, the wait for them was a wait for the previous group's store drain)
  fetch(g, I0{});
  store_rows(I0{});
  fetch(g + gstep, I1{});
  // 32 dropped stores (out-of-range offset) after it, as after every loop body: the first group's wait for
  // slot 1 then counts past 32 stores like every later one (hipcc merges the entry path into the loop's count)
#pragma unroll
  for (int c = 0; c < 32; ++c) __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, orsrc, 0x7ffffff0, 0, 0);
  auto body = [&](auto PAR) {
    constexpr int par = decltype(PAR)::value;
    const int n = g / p.groups_per_img, oh0 = (g % p.groups_per_img) * CVR_TR, oh = oh0 + wave;
    __syncthreads();                                   // input rows of g visible; stage reads of g-1 done
    fetch(g + 2 * gstep, PAR);                     // into the slot group g's rows were staged from
    stamp(5);
    unsigned short* const st_cur = ostage + (PIPE ? par * (64 * CVF_SEGS) : 0);
    const unsigned short* const st_prev = ostage + (PIPE ? (par ^ 1) * (64 * CVF_SEGS) : 0);
    f32x4 acc[CVF_NT][4];          // the bias rides in as the accumulators' initial value
#pragma unroll
    for (int t = 0; t < CVF_NT; ++t)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[t][nt] = f32x4{bias_v[nt], bias_v[nt], bias_v[nt], bias_v[nt]};
    bf16x8 af[2][CVF_NT];
    auto load_a = [&](int ks, bf16x8 (&a)[CVF_NT]) {
#pragma unroll
      for (int t = 0; t < CVF_NT; ++t) {
        const uint2* src = reinterpret_cast<const uint2*>(__builtin_assume_aligned(smem + abase[ks] + t * 32, 8));
        const uint2 a0 = src[0], a1 = src[1];
        a[t] = __builtin_bit_cast(bf16x8, u32x4{a0.x, a0.y, a1.x, a1.y});
      }
    };
    // the order is pinned (sched_barrier): left to itself hipcc funnels every A fragment through one register
    // quad (read -> lgkmcnt(0) -> 4 MFMAs -> read ...), which exposes the LDS latency 42 times per group.
    // PIPE: each k-step also carries 6 of the previous group's 32 output chunks per wave (LDS read before the
    // MFMAs, global store after them), so the store stream drains under the MFMAs instead of after them
    constexpr int CPK = 6;
    load_a(0, af[0]);
#pragma unroll
    for (int ks = 0; ks < CVR_NKS; ++ks) {
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < CVR_NKS) load_a(ks + 1, af[(ks + 1) & 1]);
      uint2 sv[CPK];
      if constexpr (PIPE) {
#pragma unroll
        for (int i = 0; i < CPK; ++i)
          if (ks * CPK + i < 32) sv[i] = chunk_read(st_prev, ks * CPK + i, max(prev_n4, 1));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < CVF_NT; ++t)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][t], bw[nt][ks], acc[t][nt], 0, 0, 0);
      if constexpr (PIPE) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < CPK; ++i)
          if (ks * CPK + i < 32) chunk_store(sv[i], ks * CPK + i, prev_obase, prev_n4, noc);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    stamp(1);
    // epilogue -> [oc][row * OW + ow] bf16 (4 consecutive pixels per lane: two dword writes, branch-free:
    // pixel pairs past OW go to the trash word)
#pragma unroll
    for (int t = 0; t < CVF_NT; ++t) {
      const int owb = t * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        float vv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) vv[r] = act_t<ACT>(acc[t][nt][r]);
        unsigned* dst = reinterpret_cast<unsigned*>(st_cur + (nt * 16 + (lane & 15)) * CVF_SEGS + wave * p.OW + owb);
        if (t + 1 < CVF_NT) {        // tiles 0..5 lie inside every row (OW > 96): constant LDS offsets
          dst[0] = pack_bf16x2(vv[0], vv[1]);
          dst[1] = pack_bf16x2(vv[2], vv[3]);
        } else {
          *(owb + 1 < p.OW ? dst : trash) = pack_bf16x2(vv[0], vv[1]);
          *(owb + 3 < p.OW ? dst + 1 : trash) = pack_bf16x2(vv[2], vv[3]);
        }
      }
    }
    stamp(2);
    __syncthreads();                                   // stage complete; every input-row read of g retired
    stamp(3);
    const int rows_valid = min(CVR_TR, p.OH - oh0);
    prev_n4 = (rows_valid * p.OW) >> 2;
    prev_obase = (int)((((long long)n * p.OC + oc0) * OHW + (long long)oh0 * p.OW) * 2);
    if constexpr (!PIPE) {
      uint2 v[32];
#pragma unroll
      for (int c = 0; c < 32; ++c) v[c] = chunk_read(st_cur, c, prev_n4);
#pragma unroll
      for (int c = 0; c < 32; ++c) chunk_store(v[c], c, prev_obase, prev_n4, noc);
    }
    stamp(4);
    // rows of g + grid into the (now free) input buffer
    if constexpr (par == 0) store_rows(I1{});
    else store_rows(I0{});
    (void)oh;
  };
  int it = 0;
  while (g < gend) {
    body(I0{});
    g += gstep;
    ++it;
    if (g >= gend) break;
    body(I1{});
    g += gstep;
    ++it;
  }
  if constexpr (PIPE) {
    // the last group's chunks (its stage was completed before the loop's last barrier)
    if (it > 0) {
      const unsigned short* st_last = ostage + ((it + 1) & 1) * (64 * CVF_SEGS);
      uint2 v[32];
#pragma unroll
      for (int c = 0; c < 32; ++c) v[c] = chunk_read(st_last, c, prev_n4);
#pragma unroll
      for (int c = 0; c < 32; ++c) chunk_store(v[c], c, prev_obase, prev_n4, noc);
    }
  }
  if constexpr (DIAG) {
    stamp(5);
    tt[0] = t_prev - t_start;
    if (lane == 0) {
      unsigned long long* d = reinterpret_cast<unsigned long long*>(p.out) + (blockIdx.x * 4 + wave) * 8;
#pragma unroll
      for (int i = 0; i < 6; ++i) d[i] = tt[i];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Warp-specialised full-row conv (the default for the headline layer). The phase stamps of
// conv2d_rowfull_kernel (profiles/r2_s3, r2_write_bw) show its ONE wave per SIMD stalling the MFMAs queued
// behind a store that finds the CU's memory queue full: 25 K cycles of store issue + 27 K of waiting per wave,
// on top of 33 K of MFMA and 15 K of epilogue — serialised, not overlapped. Here 8 waves = 2 per SIMD in two roles:
//  * compute waves 0-3 (one output row x 64 oc each, filter in VGPRs as before) run the 7 pixel tiles one after
//    the other: 24 MFMAs per tile on 4 accumulator chains (a 16x16x32 bf16 chain issues every 16 cycles even on
//    one accumulator, so the 28-chain interleave is not needed). The 42 (tile, k-step) A fragments stream from
//    LDS through a 4-deep register ring, and tile t-2's epilogue (bias seeded in the accumulators, act, bf16
//    pack, LDS stage) is slotted between tile t's k-steps. 3 x 16 accumulator registers instead of 112: the
//    wave fits the 256 registers of 2 waves per SIMD;
//  * store waves 4-7 own every vector-memory instruction: they read the previous group's staged
//    [64 oc][4 rows x OW] image into registers, release the stage, send it as 8-B stores (each oc's 4-row run
//    is contiguous in NCHW), then write the next group's input rows (fetched one group earlier) into the other
//    row buffer as the 4 shifted copies. A store waiting for queue space stalls only its own wave; the MFMAs of
//    the compute wave on the same SIMD keep issuing.
// LDS: 2 input-row buffers (double-buffered, so row staging never sits between two compute phases) + ONE output
// stage. Two barriers per group: top (rows of g staged, stage of g-1 complete) and S (the store waves hold
// stage g-1 in registers; the compute waves reach it after tile 1, before their first epilogue write).
constexpr int CVW_STAGE = 64 * CVF_SEGS * 2;                          // [64 oc][segs] bf16
constexpr int CVW_LDS = 2 * CVR_BUF + CVW_STAGE + CVR_TRASH;
template <int ACT, bool DIAG>
__global__ void __launch_bounds__(512, 1) conv2d_ws_kernel(ConvRowParams p) {
  // DIAG: s_memtime phase stamps per wave (timing build, written over the output). Compute waves: [1] tiles 0-1,
  // [2] wait at S, [3] tiles 2-6 + epilogues, [4] -, [5] wait at the top barrier. Store waves: [1] stage reads,
  // [2] wait at S, [3] store issue, [4] row staging (incl. the wait for the fetched rows) + next fetch, [5] wait
  // at the top barrier.
  unsigned long long tt[6] = {0, 0, 0, 0, 0, 0}, t_prev = 0;
  auto stamp = [&](int slot) {
    if constexpr (DIAG) {
      unsigned long long t;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      __builtin_amdgcn_sched_barrier(0);
      if (slot >= 0) tt[slot] += t - t_prev;
      t_prev = t;
    }
  };
  stamp(-1);
  const unsigned long long t_start = t_prev;
  __shared__ __attribute__((aligned(16))) char smem[CVW_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool is_compute = wave < 4;
  const int oc0 = blockIdx.y * 64;

  // store waves: input staging work items (c, r, chunk j), <= 2 per store lane, identical for every group
  const int sl_id = tid - 256;
  const int items = p.C * p.rin * p.chunks;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(p.X), (short)0, (int)((long long)p.N * p.C * p.H * p.W * 2), 0x00020000);
  u32x4 lo[2];         // [item]: the next group's rows, fetched one group ahead
  u32x2 hi[2];
  int it_off[2], it_r[2];
  bool it_lo[2], it_hi[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int it = max(0, min(sl_id + u * 256, items - 1));
    const int j = it % p.chunks, cr = it / p.chunks, r = cr % p.rin, c = cr / p.rin;
    it_off[u] = ((c * p.H + r) * p.W + 8 * j) * 2;
    it_r[u] = r;
    it_lo[u] = 8 * j < p.W;
    it_hi[u] = 8 * (j + 1) < p.W;
  }
  const int gstep = gridDim.x, gend = p.ngroups;
  auto fetch = [&](int g) {
    const bool gok = g < gend;
    const int n = g / p.groups_per_img, oh0 = (g % p.groups_per_img) * CVR_TR;
    const int gbase = ((n * p.C * p.H) + oh0) * p.W * 2;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool rok = gok && oh0 + it_r[u] < p.H;
      const int o = gbase + it_off[u];
      lo[u] = __builtin_amdgcn_raw_buffer_load_b128(xr, (rok && it_lo[u]) ? o : 0x7ffffff0, 0, 0);
      hi[u] = __builtin_amdgcn_raw_buffer_load_b64(xr, (rok && it_hi[u]) ? o + 16 : 0x7ffffff0, 0, 0);
    }
  };
  auto store_rows = [&](char* rb) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = sl_id + u * 256;
      if (it >= items) continue;
      const int j = it % p.chunks, cr = it / p.chunks;
      char* row = rb + cr * 4 * CVR_CP + j * 16;
      const unsigned w[6] = {lo[u].x, lo[u].y, lo[u].z, lo[u].w, hi[u].x, hi[u].y};
      *reinterpret_cast<u32x4*>(row) = lo[u];
      *reinterpret_cast<u32x4*>(row + CVR_CP) =
          u32x4{__builtin_amdgcn_alignbyte(w[1], w[0], 2), __builtin_amdgcn_alignbyte(w[2], w[1], 2),
                __builtin_amdgcn_alignbyte(w[3], w[2], 2), __builtin_amdgcn_alignbyte(w[4], w[3], 2)};
      *reinterpret_cast<u32x4*>(row + 2 * CVR_CP) = u32x4{w[1], w[2], w[3], w[4]};
      *reinterpret_cast<u32x4*>(row + 3 * CVR_CP) =
          u32x4{__builtin_amdgcn_alignbyte(w[2], w[1], 2), __builtin_amdgcn_alignbyte(w[3], w[2], 2),
                __builtin_amdgcn_alignbyte(w[4], w[3], 2), __builtin_amdgcn_alignbyte(w[5], w[4], 2)};
    }
  };

  // ---- prologue. The store waves request group 0's input rows first and write them into row buffer 0 while the
  // compute waves load their filter fragments; the loop's first top barrier joins them.
  if (!is_compute) fetch(blockIdx.x);
  // filter fragments straight from the pre-packed tensor: one 16-B load per (n-tile, k-step) and lane (no LDS
  // staging, no per-element extraction: a few dozen instructions of prologue instead of ~700 — on a cold
  // instruction cache the prologue's code size, not its work, was its cost)
  bf16x8 bw[4][CVR_NKS];
  float bias_v[4];
  int abase[CVR_NKS];          // byte offset of k-step ks's A fragment (tile 0) inside a row buffer
  if (is_compute) {
    const uint4* wf = reinterpret_cast<const uint4*>(p.Wfrag) + (long long)blockIdx.y * 4 * CVR_NKS * 64 + lane;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int ks = 0; ks < CVR_NKS; ++ks) bw[nt][ks] = __builtin_bit_cast(bf16x8, wf[(nt * CVR_NKS + ks) * 64]);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int oc = oc0 + nt * 16 + (lane & 15);
      bias_v[nt] = (p.bias && oc < p.OC) ? p.bias[oc] : 0.f;
    }
#pragma unroll
    for (int ks = 0; ks < CVR_NKS; ++ks) {
      const int q = ks * 4 + (lane >> 4);
      if (q < p.ckh) {
        const int c = q / p.KH, kh = q % p.KH;
        abase[ks] = ((c * p.rin + wave + kh) * 4 + (lane & 3)) * CVR_CP + (lane & 12) * 2;
      } else {
        abase[ks] = CVR_ZERO + (lane & 3) * 16 + (lane & 12) * 2;
      }
    }
  }
  if (!is_compute) {
    for (int e = sl_id; e < 2 * (4 * CVR_CP / 16); e += 256) {
      const int b = e / (4 * CVR_CP / 16), i = e - b * (4 * CVR_CP / 16);
      reinterpret_cast<uint4*>(smem + b * CVR_BUF + CVR_ZERO)[i] = make_uint4(0, 0, 0, 0);
    }
    store_rows(smem);
    fetch(blockIdx.x + gstep);
  }

  const long long OHW = (long long)p.OH * p.OW;
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      p.out, (short)0, (int)std::min<long long>((long long)p.N * p.OC * OHW * 2, 0x7fffffffLL), 0x00020000);
  unsigned short* const stage = reinterpret_cast<unsigned short*>(smem + 2 * CVR_BUF);
  unsigned* const trash = reinterpret_cast<unsigned*>(smem + 2 * CVR_BUF + CVW_STAGE);
  const int sw = wave - 4;          // store wave index: oc rows sw + 4 j of the stage

  // one output chunk of the staged group: oc (sw + 4 j), 8-byte piece q = lane + 64 h of its rows_valid * OW
  // run (c = 2 j + h). The per-lane part of the LDS address / global offset is one register per h (rd[h] /
  // vo[h], set per group); the oc part is an immediate / a scalar offset. Pieces past the run / oc past OC go
  // to an out-of-range offset (dropped).
  auto chunk_read = [&](int c, const int (&rd)[2]) -> uint2 {
    const int j = c >> 1, h = c & 1;
    return *reinterpret_cast<const uint2*>(stage + (sw + 4 * j) * CVF_SEGS + rd[h]);
  };
  auto chunk_store = [&](uint2 v, int c, int obase, const int (&vo)[2], int noc) {
    const int j = c >> 1, h = c & 1;
    const int ocl = sw + 4 * j;
    const int soff = ocl < noc ? obase + (int)(ocl * OHW * 2) : 0x7ffffff0;
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, orsrc, vo[h], soff, 0);
  };
  auto lane_offsets = [&](int n4, int (&rd)[2], int (&vo)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = lane + 64 * h;
      rd[h] = 4 * min(q, max(n4, 1) - 1);
      vo[h] = q < n4 ? 8 * q : 0x7ffffff0;
    }
  };
  // tile t's epilogue for n-tile nt: act -> bf16 pairs -> [oc][row * OW + ow] of the stage (pixel pairs past
  // OW in the last tile go to the trash word)
  auto epi = [&](int t, int nt, const f32x4& a) {
    const int owb = t * 16 + (lane >> 4) * 4;
    float vv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) vv[r] = act_t<ACT>(a[r]);
    unsigned* dst = reinterpret_cast<unsigned*>(stage + (nt * 16 + (lane & 15)) * CVF_SEGS + wave * p.OW + owb);
    if (t + 1 < CVF_NT) {
      dst[0] = pack_bf16x2(vv[0], vv[1]);
      dst[1] = pack_bf16x2(vv[2], vv[3]);
    } else {
      *(owb + 1 < p.OW ? dst : trash) = pack_bf16x2(vv[0], vv[1]);
      *(owb + 3 < p.OW ? dst + 1 : trash) = pack_bf16x2(vv[2], vv[3]);
    }
  };
  auto load_frag = [&](const char* rb, int t, int ks) -> bf16x8 {
    const uint2* src = reinterpret_cast<const uint2*>(__builtin_assume_aligned(rb + abase[ks] + t * 32, 8));
    const uint2 a0 = src[0], a1 = src[1];
    return __builtin_bit_cast(bf16x8, u32x4{a0.x, a0.y, a1.x, a1.y});
  };

  const int noc = min(64, p.OC - oc0);
  // The two roles run separate loops with the same barrier sequence (top, S per group; one final barrier):
  // is_compute is wave-uniform, and one loop with role branches inside made hipcc merge the two roles' wait
  // counters at the joins (the store waves then waited for their own stores to drain before writing rows).
  if (is_compute) {
    int par = 0;
    for (int g = blockIdx.x; g < gend; g += gstep, par ^= 1) {
      stamp(4);
      __syncthreads();                                 // top: rows of g staged, stage of g-1 complete
      stamp(5);
      const char* const rb = smem + par * CVR_BUF;
      constexpr int NF = CVF_NT * CVR_NKS, AHEAD = 3, LAG = 2;
      f32x4 acc[LAG + 1][4];
      bf16x8 ring[4];
#pragma unroll
      for (int f = 0; f < AHEAD; ++f) ring[f] = load_frag(rb, f / CVR_NKS, f % CVR_NKS);
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int t = f / CVR_NKS, ks = f % CVR_NKS;
        __builtin_amdgcn_sched_barrier(0);
        if (f + AHEAD < NF) ring[(f + AHEAD) & 3] = load_frag(rb, (f + AHEAD) / CVR_NKS, (f + AHEAD) % CVR_NKS);
        if (ks == 0) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[t % (LAG + 1)][nt] = f32x4{bias_v[nt], bias_v[nt], bias_v[nt], bias_v[nt]};
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[t % (LAG + 1)][nt] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[f & 3], bw[nt][ks], acc[t % (LAG + 1)][nt], 0, 0, 0);
        if (f == LAG * CVR_NKS - 1) {
          __builtin_amdgcn_sched_barrier(0);
          stamp(1);
          __syncthreads();                             // S: the store waves hold stage g-1 in registers
          stamp(2);
        }
        if (t >= LAG && ks < 4) {
          __builtin_amdgcn_sched_barrier(0);
          epi(t - LAG, ks, acc[(t - LAG) % (LAG + 1)][ks]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = CVF_NT - LAG; t < CVF_NT; ++t)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) epi(t, nt, acc[t % (LAG + 1)][nt]);
      stamp(3);
    }
    __syncthreads();
  } else {
    int prev_obase = 0, prev_n4 = 0, par = 0;
    int g = blockIdx.x;
    for (; g < gend; g += gstep, par ^= 1) {
      stamp(4);
      __syncthreads();                                 // top
      stamp(5);
      int rd[2], vo[2];
      lane_offsets(prev_n4, rd, vo);                   // the stage holds g-1 (first group: every store dropped)
      uint2 v[32];
#pragma unroll
      for (int c = 0; c < 32; ++c) v[c] = chunk_read(c, rd);
      stamp(1);
      __syncthreads();                                 // S: stage free for g's epilogues
      stamp(2);
#pragma unroll
      for (int c = 0; c < 32; ++c) chunk_store(v[c], c, prev_obase, vo, noc);
      stamp(3);
      store_rows(smem + (par ^ 1) * CVR_BUF);          // rows of g + grid (fetched one group ago)
      fetch(g + 2 * gstep);                            // behind this group's stores: a whole group to arrive
      stamp(4);
      const int n = g / p.groups_per_img, oh0 = (g % p.groups_per_img) * CVR_TR;
      prev_n4 = (min(CVR_TR, p.OH - oh0) * p.OW) >> 2;
      prev_obase = (int)((((long long)n * p.OC + oc0) * OHW + (long long)oh0 * p.OW) * 2);
    }
    __syncthreads();                                   // the last group's stage is complete
    if (g != (int)blockIdx.x) {
      int rd[2], vo[2];
      lane_offsets(prev_n4, rd, vo);
      uint2 v[32];
#pragma unroll
      for (int c = 0; c < 32; ++c) v[c] = chunk_read(c, rd);
#pragma unroll
      for (int c = 0; c < 32; ++c) chunk_store(v[c], c, prev_obase, vo, noc);
    }
  }
  if constexpr (DIAG) {
    stamp(-1);
    tt[0] = t_prev - t_start;
    if (lane == 0) {
      unsigned long long* d = reinterpret_cast<unsigned long long*>(p.out) + (blockIdx.x * 8 + wave) * 8;
#pragma unroll
      for (int i = 0; i < 6; ++i) d[i] = tt[i];
    }
  }
}

// Explicit im2col (the reference's materialised ImageToChunks/ImageBlockToMatrix path, kept for the
// "materialise" plan and for testing). out[p][k] bf16 with ld = ldk (>= K, zero padded).
__global__ void im2col_kernel(const unsigned short* X, unsigned short* out, int N, int C, int H, int W,
                              int KH, int KW, int OH, int OW, int stride, int pad, int dil, int ldk) {
  const long long P = (long long)N * OH * OW;
  const int K = C * KH * KW;
  const long long total = P * ldk;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long pp = e / ldk;
    const int k = (int)(e % ldk);
    unsigned short v = 0;
    if (k < K) {
      const int n = (int)(pp / (OH * OW)), rem = (int)(pp % (OH * OW));
      const int oh = rem / OW, ow = rem % OW;
      const int c = k / (KH * KW), r2 = k % (KH * KW), kh = r2 / KW, kw = r2 % KW;
      const int ih = oh * stride - pad + kh * dil, iw = ow * stride - pad + kw * dil;
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        v = X[(((long long)n * C + c) * H + ih) * W + iw];
    }
    out[e] = v;
  }
}

}  // namespace nsdb

extern "C" {

// Per-call launch options (no process-wide state: a choice applies to exactly the call that passes it).
struct ConvOpts {
  int force_generic;   // 1: the generic gather kernel (A/B, tests)
  int variant;         // row-kernel diagnostics (timing only)
  // row kernel grid cap: > 0 persistent blocks (default 512 = 2 per CU: the filter prologue is paid once per block);
  // 0 = one block per row group (short-lived blocks that the dispatcher can interleave with higher-priority
  // kernels when the conv shares the GPU with another job, e.g. gated into a GEMM's tail)
  int max_blocks;
  // row-kernel choice for 97 <= OW <= 112: 5 = warp-specialised (default), 1 = full-row, 0 = two-pass; 2/3/4/6 are
  // diagnostics (phase stamps, unpipelined stores)
  int kernel;
  int contig;          // full-row kernel: contiguous row-group runs per block (A/B)
};

int nsdb_conv2d_igemm(const void* X, const void* Wt, const float* bias, void* out, int N, int C, int H,
                      int W, int OC, int KH, int KW, int stride, int pad, int dil, int ldw, int act,
                      int nchw_out, int out_f32, const void* wfrag, const ConvOpts* opts, hipStream_t stream) {
  const ConvOpts o = opts ? *opts : ConvOpts{0, 0, 512, 5, 0};
  nsdb::ConvParams p;
  p.X = (const unsigned short*)X; p.Wt = (const unsigned short*)Wt; p.bias = bias; p.out = out;
  p.N = N; p.C = C; p.H = H; p.W = W; p.OC = OC; p.KH = KH; p.KW = KW;
  p.stride = stride; p.pad = pad; p.dil = dil;
  p.OH = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  p.OW = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  p.K = C * KH * KW; p.ldw = ldw;
  if (ldw % 8 != 0 || ldw < p.K || p.OH <= 0 || p.OW <= 0) return -1;
  if ((long long)N * C * H * W >= 0x7fffffffLL) return -2;   // 32-bit image offsets
  p.act = act; p.nchw_out = nchw_out; p.out_f32 = out_f32;
  // row-tiled LDS kernel for small-C, wide-row layers (see conv2d_rows_kernel)
  const int rin = nsdb::CVR_TR + KH - 1;
  if (o.force_generic == 0 && stride == 1 && dil == 1 && pad == 0 && KW <= 8 && W % 8 == 0 &&
      C * KH <= 4 * nsdb::CVR_NKS && C * rin <= nsdb::CVR_ROWS && p.OW <= 16 * nsdb::CVR_MAXT) {
    nsdb::ConvRowParams q;
    q.X = p.X; q.Wt = p.Wt; q.bias = bias; q.out = out;
    q.N = N; q.C = C; q.H = H; q.W = W; q.OC = OC; q.KH = KH; q.KW = KW; q.OH = p.OH; q.OW = p.OW; q.ldw = ldw;
    q.rin = rin; q.ckh = C * KH; q.nks = (C * KH + 3) / 4;
    q.ntiles = (p.OW + 15) / 16;
    q.chunks = std::min((16 * q.ntiles + 4 + 7) / 8, nsdb::CVR_CP / 16);
    q.groups_per_img = (p.OH + nsdb::CVR_TR - 1) / nsdb::CVR_TR;
    q.ngroups = N * q.groups_per_img;
    q.act = act; q.nchw_out = nchw_out; q.out_f32 = out_f32; q.variant = o.variant;
    q.contig = o.contig;
    q.Wfrag = (const unsigned short*)wfrag;
    q.segs = (4 * p.OW + 3) & ~3;
    if ((q.segs / 2) % 4 == 0) q.segs += 4;
    q.vec8 = ((long long)p.OH * p.OW) % 4 == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0;
    if (32 * q.segs * 2 > nsdb::CVR_OSTAGE) goto generic;
    if ((long long)N * OC * p.OH * p.OW * 2 >= 0x7ffffff0LL) goto generic;    // 31-bit buffer offsets
    if (C * rin * q.chunks > 512 || 64 * ldw / 8 > 6 * 256 || 64 * ldw * 2 > nsdb::CVR_BUF) goto generic;
    {
      const int blocks = o.max_blocks > 0 ? std::min(q.ngroups, o.max_blocks) : q.ngroups;
      const dim3 grid(blocks, (OC + 63) / 64);
      const bool staged = nchw_out && !out_f32 && (p.OW & 1) == 0 && q.vec8 && ((p.OH % 4) * p.OW) % 4 == 0;
      if (staged && q.variant == 0 && o.kernel && q.ntiles == nsdb::CVF_NT && 4 * p.OW <= nsdb::CVF_SEGS) {
        // one block of 4 waves per CU (one wave per SIMD), persistent over the row groups
        const dim3 gridf(std::min(q.ngroups, o.max_blocks > 0 ? std::min(o.max_blocks, 256) : q.ngroups),
                         (OC + 63) / 64);
#define NSDB_CVF_LAUNCH(A) hipLaunchKernelGGL((nsdb::conv2d_rowfull_kernel<A, false, true>), gridf, dim3(256), 0, stream, q)
        if (o.kernel == 2 || o.kernel == 3) {   // phase-stamp timing builds (diagnostic)
          if (o.kernel == 2)
            hipLaunchKernelGGL((nsdb::conv2d_rowfull_kernel<nsdb::ACT_NONE, true, true>), gridf, dim3(256), 0, stream, q);
          else
            hipLaunchKernelGGL((nsdb::conv2d_rowfull_kernel<nsdb::ACT_NONE, true, false>), gridf, dim3(256), 0, stream, q);
          return (int)hipGetLastError();
        }
        if (o.kernel == 4) {   // unpipelined stores (A/B)
          hipLaunchKernelGGL((nsdb::conv2d_rowfull_kernel<nsdb::ACT_NONE, false, false>), gridf, dim3(256), 0, stream, q);
          return (int)hipGetLastError();
        }
        if (o.kernel == 6 && wfrag != nullptr) {   // warp-specialised, phase-stamp timing build (diagnostic)
          hipLaunchKernelGGL((nsdb::conv2d_ws_kernel<nsdb::ACT_NONE, true>), gridf, dim3(512), 0, stream, q);
          return (int)hipGetLastError();
        }
        if (o.kernel == 5 && wfrag != nullptr) {   // warp-specialised: 4 compute + 4 store waves per CU
#define NSDB_CVW_LAUNCH(A) hipLaunchKernelGGL((nsdb::conv2d_ws_kernel<A, false>), gridf, dim3(512), 0, stream, q)
          switch (act) {
            case nsdb::ACT_RELU: NSDB_CVW_LAUNCH(nsdb::ACT_RELU); break;
            case nsdb::ACT_SIGMOID: NSDB_CVW_LAUNCH(nsdb::ACT_SIGMOID); break;
            case nsdb::ACT_EXP: NSDB_CVW_LAUNCH(nsdb::ACT_EXP); break;
            case nsdb::ACT_TANH: NSDB_CVW_LAUNCH(nsdb::ACT_TANH); break;
            default: NSDB_CVW_LAUNCH(nsdb::ACT_NONE); break;
          }
#undef NSDB_CVW_LAUNCH
          return (int)hipGetLastError();
        }
        switch (act) {
          case nsdb::ACT_RELU: NSDB_CVF_LAUNCH(nsdb::ACT_RELU); break;
          case nsdb::ACT_SIGMOID: NSDB_CVF_LAUNCH(nsdb::ACT_SIGMOID); break;
          case nsdb::ACT_EXP: NSDB_CVF_LAUNCH(nsdb::ACT_EXP); break;
          case nsdb::ACT_TANH: NSDB_CVF_LAUNCH(nsdb::ACT_TANH); break;
          default: NSDB_CVF_LAUNCH(nsdb::ACT_NONE); break;
        }
#undef NSDB_CVF_LAUNCH
        return (int)hipGetLastError();
      }
      if (q.variant != 0) {   // diagnostics build (timing only): runtime variant bits, no activation
        if (staged) hipLaunchKernelGGL((nsdb::conv2d_rows_kernel<nsdb::ACT_NONE, true, true>), grid, dim3(256), 0, stream, q);
        else hipLaunchKernelGGL((nsdb::conv2d_rows_kernel<nsdb::ACT_NONE, false, true>), grid, dim3(256), 0, stream, q);
        return (int)hipGetLastError();
      }
#define NSDB_CVR_LAUNCH(A)                                                                                      \
  do {                                                                                                        \
    if (staged) hipLaunchKernelGGL((nsdb::conv2d_rows_kernel<A, true, false>), grid, dim3(256), 0, stream, q); \
    else hipLaunchKernelGGL((nsdb::conv2d_rows_kernel<A, false, false>), grid, dim3(256), 0, stream, q);       \
  } while (0)
      switch (act) {
        case nsdb::ACT_RELU: NSDB_CVR_LAUNCH(nsdb::ACT_RELU); break;
        case nsdb::ACT_SIGMOID: NSDB_CVR_LAUNCH(nsdb::ACT_SIGMOID); break;
        case nsdb::ACT_EXP: NSDB_CVR_LAUNCH(nsdb::ACT_EXP); break;
        case nsdb::ACT_TANH: NSDB_CVR_LAUNCH(nsdb::ACT_TANH); break;
        default: NSDB_CVR_LAUNCH(nsdb::ACT_NONE); break;
      }
#undef NSDB_CVR_LAUNCH
      return (int)hipGetLastError();
    }
  }
generic:
  const long long P = (long long)N * p.OH * p.OW;
  dim3 grid((unsigned)((P + nsdb::CV_BM - 1) / nsdb::CV_BM), (OC + nsdb::CV_BN - 1) / nsdb::CV_BN);
  hipLaunchKernelGGL(nsdb::conv2d_igemm_kernel, grid, dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

int nsdb_im2col(const void* X, void* out, int N, int C, int H, int W, int KH, int KW, int stride, int pad,
                int dil, int ldk, hipStream_t stream) {
  const int OH = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  const int OW = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  const long long total = (long long)N * OH * OW * ldk;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(nsdb::im2col_kernel, dim3(blocks), dim3(256), 0, stream, (const unsigned short*)X,
                     (unsigned short*)out, N, C, H, W, KH, KW, OH, OW, stride, pad, dil, ldk);
  return (int)hipGetLastError();
}

}  // extern "C"
