// Shared pieces of the block-GEMM kernels (gemm.hip, gemm_w4a.hip and the study build):
// launch parameters, tile walk, LDS-DMA staging helpers, the LDS-staged epilogue store and the
// split-K reducer epilogue. Reference pattern: src/FF/headers/FFTransposeMult.h + FFAggMatrix.h.
#pragma once
#include "common.h"
#include <algorithm>

namespace nsdb {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NTHREADS = 256;
constexpr int TILE_BYTES = BM * BK * 2;          // 16 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;      // A + B
constexpr int OOB = 0x7ffffff0;                  // voffset that the range check turns into zeros

struct GemmParams {
  const unsigned short* A;  // bf16 [batch][M][lda]
  const unsigned short* B;  // bf16 [batch][N][ldb]
  void* C;                  // bf16 or f32 [batch][M][ldc]
  float* ws;                // f32 [batch][splits][M][N] (split-K partial slabs)
  const float* bias;        // f32 [batch?][M] or [N]
  long long lda, ldb, ldc;
  long long sA, sB, sC, sBias;
  int M, N, K;
  int splits, kchunk;
  int act, bias_mode, out_f32, accumulate;
  float alpha, dropout;
  unsigned long long seed;
  int tiles_m, tiles_n;
  int vec_ws;               // N % 4 == 0: 4-column groups of the split-K slabs are 16-B aligned
  int vec_c;                // C rows/base aligned for 4-column vector stores (16 B f32, 8 B bf16)
  int diag;                 // timing diagnostics (wrong results): 1 no epilogue global stores, 2 no operand loads
  // K-segmented B (an all-gathered [S][N][seg_k] chunk consumed in place, no permute copy): the B rows of
  // K segment s start at B + s * seg_stride_b (elements) with k taken relative to s * seg_k; every split
  // lies inside one segment (host forces kchunk | seg_k). seg_k = 0: plain B.
  long long seg_k, seg_stride_b;
  // fused softmax epilogue (8-phase kernel, splits == 1): 1 = over the columns of C (per row), 2 = over the
  // rows of C (per column); per-tile (max, sum) partials, per row/column-block arrival counters (zero at
  // launch, re-zeroed by the fix-up kernel) and per-tile fallback flags
  int softmax;
  float2* sm_part;
  int* sm_cnt;
  int* sm_flag;
  int* sm_dep = nullptr;     // fused softmax: departures (low 16 bits) + timed-out tiles (high 16) per group
  unsigned* start_signal = nullptr;   // study build only (csrc/study): start-gate experiments
  const char* pf_ptr = nullptr;   // operand prefetch for the NEXT kernel (8-phase, EPI 0): bytes read into the
  long long pf_bytes = 0;         // Infinity Cache by the workgroups after their main loops
  unsigned long long* stamps;   // diagnostic variant 12: per-workgroup real-time stamps every 32 k-tiles
  struct AdaptState* adapt;     // split-K: launch-to-launch adaptive K partition (see AdaptState)
  // study build only (csrc/study, rejected in the product: profiles/r2_tail): a tail trigger raised by every
  // workgroup when its main loop is done
  unsigned* signal;
  unsigned signal_value;
  // K-tail stealing (variant 19, split-K): per-tile claim counters (zero at launch; the split-K reducer re-zeroes
  // them) for the steal_tq tail chunks of steal_ch k-tiles at the end of every split's K range
  int* steal_cnt;
  int steal_tq, steal_ch;       // tail chunks per split, k-tiles per chunk (nsdb_gemm_steal)
  // 8-phase kernel, unsplit launches: store C straight from the accumulator registers (no LDS round trip;
  // see store_direct_8ph in gemm.hip). 0: the LDS-staged store_tile_lds epilogue.
  int direct_epi;
  // 8-phase split-K launches: the reduction inside the launch (gemm.hip splitk_fixup_8ph). Slabs are written through
  // to the device-coherent level; the splits of a tile count in on fx_cnt[tile], wait for each other (bounded), and
  // each reduces 1/splits of the tile's rows; fx_dep[tile] counts departures (low 16 bits) and timed-out workgroups
  // (high 16): the last to leave re-zeroes both and, after a time-out, reduces the whole tile itself.
  int fixup = 0;
  int* fx_cnt = nullptr;
  int* fx_dep = nullptr;
};

// Adaptive split-K partition (8-phase kernel, split-K launches). The splits of one GEMM run on different XCDs
// (the bijective remap puts a split's tiles on one XCD) and the XCDs of one MI355X stream at persistently
// different rates: per-split finish times of the FF layer-1 GEMM rank-correlate 0.76-0.94 from one launch to
// the next and spread over ~40 k-tiles (~80 us) — a tail of idle CUs (profiles/r2_gemm1_study, drift and
// persistence logs). Each launch reads the K share of every split from this state (equal shares on the first
// launch), times its workgroups, and the last workgroup to finish turns the measured per-split rates
// (median workgroup of the split; EMA over launches, shares clamped to [0.6, 1.4] of equal) into the shares
// of the NEXT launch, which is stream-ordered after it. Every workgroup of a launch derives the same
// contiguous K ranges from the same floats, so any shares give an exact partition of K: only the speed
// depends on them. Release/acquire hand-off per cdna_hip_programming.md §6 G16.
struct AdaptState {
  float share[64];
  float rate[64];
  unsigned cnt;
  unsigned pad[15];
  unsigned long long t0[4096];
  unsigned long long t1[4096];
};
constexpr int ADAPT_MAX_SPLITS = 64, ADAPT_MAX_WG = 4096;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// Grouped tile walk: each XCD owns a contiguous run of tile ids (xcd_remap); walking them in groups of
// GROUP_M row-tiles makes the ~32 tiles an XCD runs at once a GROUP_M x 4 block, so every A row-panel is
// re-read by 4 column tiles and every B panel by GROUP_M row tiles out of that XCD's L2 (instead of one
// column of tiles pulling every A panel through each XCD).
constexpr int GROUP_M = 8;
__device__ __forceinline__ void grouped_tile(int tile, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = GROUP_M * tiles_n;
  const int g = tile / per_group;
  const int first_m = g * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int r = tile - g * per_group;
  tm = first_m + r % gsize;
  tn = r / gsize;
}

// Stage one ROWSx64 bf16 operand tile with NW waves: ROWS/(8*NW) wave-instructions of 1 KiB per wave.
template <int ROWS, int NW>
__device__ __forceinline__ void stage_tile(__amdgpu_buffer_rsrc_t rsrc, char* lds_tile, long long ld,
                                           int rows_valid, int k0, int K, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < ROWS / (8 * NW); ++i) {
    const int rbase = i * (8 * NW) + wave * 8;
    const int r = rbase + (lane >> 3);
    const int pc = lane & 7;
    const int c = pc ^ ((r >> 1) & 7);              // logical chunk held at physical slot pc
    const int k = k0 + c * 8;
    const bool ok = (r < rows_valid) && (k < K);
    const int voff = ok ? (int)(((long long)r * ld + k) * 2) : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_tile + rbase * 128), 16, voff, 0, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 read_frag(const char* lds_tile, int row, int chunk) {
  const int pc = chunk ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(lds_tile + row * 128 + pc * 16);
}

// ---- epilogue, staged through the (now free) LDS: each wave spills its accumulators with
// statically indexed ds_writes (keeps acc in registers: a heavy per-element epilogue unrolled
// 128x would push acc to scratch), then all threads run the epilogue over whole rows ->
// coalesced global stores (f32 split-K slabs or bf16/f32 C).
// C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + reg
// TSL: the accumulators hold TRANSPOSED 16x16 tiles (lane l: row l&15, 4 consecutive columns 4*(l>>4)..):
// each lane spills a tile with ONE 16-B ds_write into a [row][chunk ^ (row & 15)] image (conflict-free over
// the 8-lane write groups) instead of 4 dword writes.
template <int TBM, int TBN, int WGM, int WGN, bool TSL = false>
__device__ __forceinline__ void store_tile_lds(const f32x4 (&acc)[TBM / WGM / 16][TBN / WGN / 16], char* smem,
                                               int smem_bytes, const GemmParams& p, int batch, int split, int m0,
                                               int n0, int tid, int lane, int wave, float* lds_bias = nullptr) {
  constexpr int NW = WGM * WGN, TM = TBM / WGM / 16, TN = TBN / WGN / 16;
  constexpr int WR = TBM / WGM, WC = TBN / WGN, WTILE = WR * WC;
  static_assert(WC >= 32, "swizzle needs >= 32 columns per wave tile");
  const int per_pass = min(smem_bytes / (WTILE * 4), NW);
  float* st = reinterpret_cast<float*>(smem);
  const int col_l = lane & 15, row_q = (lane >> 4) * 4;
  const float* bias = p.bias ? p.bias + batch * p.sBias : nullptr;
  const float keep_scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  float* ws = p.splits > 1 ? p.ws + ((long long)batch * p.splits + split) * (long long)p.M * p.N : nullptr;
  // Per-row / per-column bias of the tile staged in LDS (lds_bias: >= max(TBM, TBN) floats, 16-B aligned) before
  // any store is issued. A global bias load inside the store loop waits on vmcnt, which also counts the stores
  // issued before it (in-order counter): the output stream then drained once per iteration.
  const bool lbias = lds_bias && bias && !ws && (p.bias_mode == 1 || p.bias_mode == 2);
  if (lbias) {
    const int nb = p.bias_mode == 1 ? TBM : TBN, base = p.bias_mode == 1 ? m0 : n0, lim = p.bias_mode == 1 ? p.M : p.N;
    for (int i = tid; i < nb; i += 64 * NW) lds_bias[i] = base + i < lim ? bias[base + i] : 0.f;
  }
  for (int g0 = 0; g0 < NW; g0 += per_pass) {
    __syncthreads();
    if (wave >= g0 && wave < g0 + per_pass) {
      float* w = st + (wave - g0) * WTILE;
      if constexpr (TSL) {
        static_assert(WC % 64 == 0, "TSL image: 16-chunk swizzle groups of 4 floats");
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int row = i * 16 + col_l, ch = j * 4 + (lane >> 4);
            *reinterpret_cast<f32x4*>(w + row * WC + ((ch ^ (row & 15)) << 2)) = acc[i][j];
          }
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = i * 16 + row_q + r, col = j * 16 + col_l;
              w[row * WC + (col ^ (((row >> 2) & 1) << 4))] = acc[i][j][r];
            }
      }
    }
    __syncthreads();
    const int nwv = min(per_pass, NW - g0);
    // 4 consecutive columns per thread: one 16-B LDS read and one 16-B (f32) / 8-B (bf16) global
    // store — the tail of a short-K tile is store-ISSUE bound, so 4x fewer store instructions than
    // an element per lane. Chunks of CH iterations: every LDS read and every global load the epilogue needs
    // (bias, accumulate input) is issued first, then the math + stores. A bias load inside the store loop
    // made every iteration wait vmcnt for it — and vmcnt counts the earlier STORES too, so the output
    // stream drained once per iteration (the 1000x14588 exp/bias layer: +11 us of tail).
    constexpr int STEP = 64 * NW * 4, CH = 4;
    const int total = nwv * WTILE;
    for (int e0 = tid * 4; e0 < total; e0 += STEP * CH) {
      f32x4 v4[CH], bb[CH], cc[CH];
      int rows[CH], cols[CH];
      bool okk[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int e = e0 + k * STEP;
        const int wl = e / WTILE, loc = e % WTILE, r = loc / WC, c = loc % WC;
        const int wv = g0 + wl;
        const int row = m0 + (wv / WGN) * WR + r, col = n0 + (wv % WGN) * WC + c;
        rows[k] = row;
        cols[k] = col;
        okk[k] = e < total && row < p.M && col < p.N && !(p.diag & 1);
        v4[k] = *reinterpret_cast<const f32x4*>(
            st + min(wl, per_pass - 1) * WTILE + r * WC + (TSL ? ((((c >> 2) ^ (r & 15)) << 2)) : (c ^ (((r >> 2) & 1) << 4))));
        bb[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        cc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (ws || !okk[k]) continue;
        const int nv = min(4, p.N - col);
        if (lbias) {
          if (p.bias_mode == 1) {
            const float b = lds_bias[(wv / WGN) * WR + r];
            bb[k] = f32x4{b, b, b, b};
          } else {
            bb[k] = *reinterpret_cast<const f32x4*>(lds_bias + (wv % WGN) * WC + c);
          }
        } else if (bias) {
          if (p.bias_mode == 1) {
            const float b = bias[row];
            bb[k] = f32x4{b, b, b, b};
          } else {
            const float* bp = p.bias_mode == 3 ? bias + (long long)row * p.N + col : bias + col;
            if (nv == 4 && ((reinterpret_cast<uintptr_t>(bp) & 15) == 0)) bb[k] = *reinterpret_cast<const f32x4*>(bp);
            else {
#pragma unroll
              for (int j = 0; j < 4; ++j) bb[k][j] = bp[min(j, nv - 1)];
            }
          }
        }
        if (p.accumulate) {
          const float* cf = reinterpret_cast<const float*>(p.C) + batch * p.sC + (long long)row * p.ldc + col;
          if (nv == 4 && p.vec_c) cc[k] = *reinterpret_cast<const f32x4*>(cf);
          else {
#pragma unroll
            for (int j = 0; j < 4; ++j) cc[k][j] = cf[min(j, nv - 1)];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        if (!okk[k]) continue;
        const int row = rows[k], col = cols[k];
        const int nv = min(4, p.N - col);
        if (ws) {
          float* d = ws + (long long)row * p.N + col;
          if (nv == 4 && p.vec_ws) {
            *reinterpret_cast<f32x4*>(d) = v4[k];
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (j < nv) d[j] = v4[k][j];
          }
          continue;
        }
        const long long off = batch * p.sC + (long long)row * p.ldc + col;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float x = v4[k][j] * p.alpha + bb[k][j];
          x = apply_act(x, p.act);
          if (p.dropout > 0.f) {
            const unsigned long long idx = ((unsigned long long)batch * p.M + row) * p.N + col + j;
            x = hash_uniform(p.seed, idx) < p.dropout ? 0.f : x * keep_scale;
          }
          v[j] = x + cc[k][j];
        }
        const bool vec = nv == 4 && p.vec_c;
        if (p.out_f32) {
          float* d = reinterpret_cast<float*>(p.C) + off;
          if (vec) {
            *reinterpret_cast<f32x4*>(d) = f32x4{v[0], v[1], v[2], v[3]};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (j < nv) d[j] = v[j];
          }
        } else {
          unsigned short* d = reinterpret_cast<unsigned short*>(p.C) + off;
          if (vec) {
            *reinterpret_cast<uint2*>(d) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (j < nv) d[j] = f32_to_bf16(v[j]);
          }
        }
      }
    }
  }
}

// Epilogue of 4 consecutive reduced columns of one row (alpha, bias, activation, dropout, accumulate,
// f32 / bf16 store) shared by the split-K reducers.
__device__ __forceinline__ void reduce_epilogue4(const GemmParams& p, int batch, long long MN, long long e, f32x4 s) {
  const float* bias = p.bias ? p.bias + batch * p.sBias : nullptr;
  const float keep_scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  const int row = (int)(e / p.N), col = (int)(e % p.N);
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x = s[j] * p.alpha;
    if (bias) x += (p.bias_mode == 1) ? bias[row] : (p.bias_mode == 3) ? bias[e + j] : bias[col + j];
    x = apply_act_compact(x, p.act);
    if (p.dropout > 0.f) {
      const unsigned long long idx = (unsigned long long)batch * MN + e + j;
      x = hash_uniform(p.seed, idx) < p.dropout ? 0.f : x * keep_scale;
    }
    v[j] = x;
  }
  const long long off = batch * p.sC + (long long)row * p.ldc + col;
  if (p.accumulate) {
    const float* cf = reinterpret_cast<const float*>(p.C) + off;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += cf[j];
  }
  if (p.out_f32) {
    float* d = reinterpret_cast<float*>(p.C) + off;
    if (p.vec_c) *reinterpret_cast<f32x4*>(d) = f32x4{v[0], v[1], v[2], v[3]};
    else { d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3]; }
  } else {
    unsigned short* d = reinterpret_cast<unsigned short*>(p.C) + off;
    if (p.vec_c) *reinterpret_cast<uint2*>(d) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    else { d[0] = f32_to_bf16(v[0]); d[1] = f32_to_bf16(v[1]); d[2] = f32_to_bf16(v[2]); d[3] = f32_to_bf16(v[3]); }
  }
}

}  // namespace nsdb
