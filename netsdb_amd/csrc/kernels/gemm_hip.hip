#include "hip/hip_runtime.h"
// Block GEMM on CDNA4 matrix cores — the MI355X realisation of netsDB's
// join(A.blockCol == B.blockCol) + ClusterAggregate(sum over k) matmul pattern
// (reference: src/FF/headers/FFTransposeMult.h + FFAggMatrix.h,
//  src/sharedLibraries/headers/LASillyMultiply1Join.h + LASillyMultiply2Aggregate.h).
//
//   C[b] = epilogue( alpha * A[b] (MxK) . B[b]^T (NxK) )          ("NT": both K-contiguous)
//   epilogue = (+ bias per row | per col) -> act (relu/sigmoid/exp/tanh) -> dropout -> bf16|f32
//
// The netsDB aggregate over k-blocks becomes split-K: each split is one
// "partial block product" and the slab reducer is the ClusterAggregate combiner.
//
// Kernel structure (cdna_hip_programming.md §5):
//  * 128x128x64 tile, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 x mfma_f32_16x16x32_bf16
//  * global -> LDS with buffer_load ... lds (16 B/lane, LDS-DMA, no VGPR round trip); the
//    buffer descriptor's range check zero-fills rows past M/N and k past K (no tail code)
//  * LDS image lane-linear per wave-instruction; bank-conflict-free ds_read_b128 fragment reads via
//    an XOR swizzle applied to the per-lane SOURCE address and to the read address (rule 21):
//    physical 16-B chunk = logical chunk ^ ((row >> 1) & 7)
//  * 2-stage LDS double buffer: the DMA for k-tile t+1 is in flight while tile t is on the MFMAs
//  * XCD-aware bijective workgroup remap (T1)
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
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
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

// TBM x TBN tile, WGM x WGN waves; each wave owns (TBM/WGM) x (TBN/WGN) = TM x TN 16x16 MFMA tiles.
//   <128,128,2,2>: 256 threads, 64 KiB LDS, 2 blocks/CU (general shapes)
//   <256,256,2,4>: 512 threads, 128 KiB LDS, 1 block/CU, 128x64 per wave = 32 MFMAs per k-substep:
//                  half the LDS/L2 bytes per FLOP of the 128^2 tile (large / split-K shapes)
template <int TBM, int TBN, int WGM, int WGN>
__global__ void __launch_bounds__(64 * WGM * WGN, (64 * WGM * WGN * ((64 * WGM * WGN) >= 512 ? 1 : 2)) / 256)
gemm_nt_tile_kernel(GemmParams p) {
  constexpr int NW = WGM * WGN;
  constexpr int TM = TBM / WGM / 16, TN = TBN / WGN / 16;
  constexpr int A_BYTES = TBM * BK * 2, B_BYTES = TBN * BK * 2, STG = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];

  // 1-D grid over (split, tile); the bijective XCD remap hands every XCD a contiguous run of
  // work ids, split-major: with splits a multiple of 8 each XCD owns whole K-slices, so the A and
  // B panels of a slice are re-read out of ONE XCD's L2 (the M=N=1000, K=600k FF layer-1 shape).
  const int ntiles = p.tiles_m * p.tiles_n;
  const int wg = xcd_remap(blockIdx.x, ntiles * p.splits);
  const int split = wg / ntiles, tile = wg % ntiles;
  // column-major tile walk: consecutive tiles (same XCD after the remap) share the B panel
  const int tm = tile % p.tiles_m, tn = tile / p.tiles_m;
  const int batch = blockIdx.z;
  const int m0 = tm * TBM, n0 = tn * TBN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;

  const int rows_a = min(TBM, p.M - m0), rows_b = min(TBN, p.N - n0);
  const unsigned short* Ab = p.A + batch * p.sA + (long long)m0 * p.lda;
  const unsigned short* Bb = p.B + batch * p.sB + (long long)n0 * p.ldb;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, (unsigned)((long long)rows_a * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, (unsigned)((long long)rows_b * p.ldb * 2));

  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = (kend - kbeg + BK - 1) / BK;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    stage_tile<TBM, NW>(ra, smem, p.lda, rows_a, kbeg, kend, wave, lane);
    stage_tile<TBN, NW>(rb, smem + A_BYTES, p.ldb, rows_b, kbeg, kend, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STG;
    if (t + 1 < nk) {
      char* nxt = smem + ((t + 1) & 1) * STG;
      const int k1 = kbeg + (t + 1) * BK;
      stage_tile<TBM, NW>(ra, nxt, p.lda, rows_a, k1, kend, wave, lane);
      stage_tile<TBN, NW>(rb, nxt + A_BYTES, p.ldb, rows_b, k1, kend, wave, lane);
    }
    const char* la = cur;
    const char* lb = cur + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag(la, wm * (TBM / WGM) + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag(lb, wn * (TBN / WGN) + j * 16 + (lane & 15), chunk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue, staged through the (now free) LDS: each wave spills its accumulators with
  // statically indexed ds_writes (keeps acc in registers: a heavy per-element epilogue unrolled
  // 128x would push acc to scratch), then all threads run the epilogue over whole rows ->
  // coalesced global stores (f32 split-K slabs or bf16/f32 C).
  // C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + reg
  constexpr int WR = TBM / WGM, WC = TBN / WGN, WTILE = WR * WC;
  constexpr int PER_PASS = (2 * STG) / (WTILE * 4) < NW ? (2 * STG) / (WTILE * 4) : NW;
  static_assert(WC >= 32, "swizzle needs >= 32 columns per wave tile");
  float* st = reinterpret_cast<float*>(smem);
  const int col_l = lane & 15, row_q = (lane >> 4) * 4;
  const float* bias = p.bias ? p.bias + batch * p.sBias : nullptr;
  const float keep_scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  float* ws = p.splits > 1 ? p.ws + ((long long)batch * p.splits + split) * (long long)p.M * p.N : nullptr;
  for (int g0 = 0; g0 < NW; g0 += PER_PASS) {
    __syncthreads();
    if (wave >= g0 && wave < g0 + PER_PASS) {
      float* w = st + (wave - g0) * WTILE;
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
    __syncthreads();
    const int nwv = min(PER_PASS, NW - g0);
    for (int e = tid; e < nwv * WTILE; e += 64 * NW) {
      const int wl = e / WTILE, loc = e % WTILE, r = loc / WC, c = loc % WC;
      const int wv = g0 + wl;
      const int row = m0 + (wv / WGN) * WR + r, col = n0 + (wv % WGN) * WC + c;
      if (row >= p.M || col >= p.N) continue;
      float v = st[wl * WTILE + r * WC + (c ^ (((r >> 2) & 1) << 4))];
      if (ws) {
        ws[(long long)row * p.N + col] = v;
        continue;
      }
      v *= p.alpha;
      if (bias) v += p.bias_mode == 1 ? bias[row] : bias[col];
      v = apply_act(v, p.act);
      if (p.dropout > 0.f) {
        const unsigned long long idx = ((unsigned long long)batch * p.M + row) * p.N + col;
        v = hash_uniform(p.seed, idx) < p.dropout ? 0.f : v * keep_scale;
      }
      const long long off = batch * p.sC + (long long)row * p.ldc + col;
      if (p.accumulate) v += reinterpret_cast<float*>(p.C)[off];
      if (p.out_f32) reinterpret_cast<float*>(p.C)[off] = v;
      else reinterpret_cast<unsigned short*>(p.C)[off] = f32_to_bf16(v);
    }
  }
}

// Split-K slab reducer + fused epilogue (the ClusterAggregate "combine" of the partial block products).
__global__ void __launch_bounds__(256) splitk_reduce_kernel(GemmParams p) {
  const long long MN = (long long)p.M * p.N;
  const long long total = MN * gridDim.y;
  const int batch = blockIdx.y;
  const float* bias = p.bias ? p.bias + batch * p.sBias : nullptr;
  const float keep_scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  (void)total;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < MN;
       e += (long long)gridDim.x * blockDim.x) {
    const float* w = p.ws + (long long)batch * p.splits * MN + e;
    float s = 0.f;
    for (int k = 0; k < p.splits; ++k) s += w[k * MN];
    const int row = (int)(e / p.N), col = (int)(e % p.N);
    float v = s * p.alpha;
    if (bias) v += (p.bias_mode == 1) ? bias[row] : bias[col];
    v = apply_act_compact(v, p.act);
    if (p.dropout > 0.f) {
      const unsigned long long idx = (unsigned long long)batch * MN + e;
      v = hash_uniform(p.seed, idx) < p.dropout ? 0.f : v * keep_scale;
    }
    const long long off = batch * p.sC + (long long)row * p.ldc + col;
    if (p.accumulate) v += reinterpret_cast<float*>(p.C)[off];
    if (p.out_f32) reinterpret_cast<float*>(p.C)[off] = v;
    else reinterpret_cast<unsigned short*>(p.C)[off] = f32_to_bf16(v);
  }
}

}  // namespace nsdb

// ---------------------------------------------------------------- host side
extern "C" {

static int g_force_cfg = -1;   // -1 auto, 0 = 128x128, 1 = 256x256 (A/B testing)

// Tile config: the 256x256 tile (1 block/CU) when both dims fill it and there is enough work.
static int pick_cfg(int M, int N, int K, int batch) {
  if (g_force_cfg >= 0) return g_force_cfg;
  const long long big_tiles = (long long)((M + 255) / 256) * ((N + 255) / 256) * batch;
  const bool fills = M >= 192 && N >= 192;
  const long long ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  return (fills && big_tiles * ksteps >= 256LL * 32) ? 1 : 0;
}

void nsdb_gemm_force_config(int cfg) { g_force_cfg = cfg; }

// Number of split-K slices the launcher will use; the caller sizes the workspace with it.
int nsdb_gemm_splits(int M, int N, int K, int batch) {
  const int cfg = pick_cfg(M, N, K, batch);
  const int tbm = cfg ? 256 : nsdb::BM, tbn = cfg ? 256 : nsdb::BN;
  const int tiles = ((M + tbm - 1) / tbm) * ((N + tbn - 1) / tbn) * batch;
  const int ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  // fill the chip: 256 CUs x (2 blocks of 128^2 | 1 block of 256^2); keep >= 8 k-steps per split
  const int target = cfg ? 256 : 512;
  int splits = 1;
  if (tiles < target) {
    splits = (target + tiles - 1) / tiles;
    splits = std::min(splits, std::max(1, ksteps / 8));
  }
  if (splits > 1) {
    const int kchunk_steps = (ksteps + splits - 1) / splits;
    splits = (ksteps + kchunk_steps - 1) / kchunk_steps;
  }
  return splits;
}

int nsdb_gemm_nt_bf16(const void* A, const void* B, void* C, float* ws, const float* bias,
                      int M, int N, int K, long long lda, long long ldb, long long ldc,
                      long long sA, long long sB, long long sC, long long sBias, int batch,
                      int splits, int act, int bias_mode, int out_f32, float alpha, float dropout,
                      unsigned long long seed, int accumulate, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (K % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0) return -1;        // 16-B rows for the LDS-DMA
  if (256LL * lda * 2 >= 0x7ffffff0LL || 256LL * ldb * 2 >= 0x7ffffff0LL)
    return -2;                                                         // per-tile buffer range
  if (splits > 1 && ws == nullptr) return -3;
  if (accumulate && !out_f32) return -4;                                // C += A.B^T only into f32
  nsdb::GemmParams p;
  p.A = (const unsigned short*)A; p.B = (const unsigned short*)B; p.C = C; p.ws = ws; p.bias = bias;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.sA = sA; p.sB = sB; p.sC = sC; p.sBias = sBias;
  p.M = M; p.N = N; p.K = K;
  const int ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  splits = std::max(1, splits);
  const int kchunk_steps = (ksteps + splits - 1) / splits;
  p.kchunk = std::max(1, kchunk_steps) * nsdb::BK;
  p.splits = (K + p.kchunk - 1) / p.kchunk;
  if (p.splits < 1) p.splits = 1;
  p.act = act; p.bias_mode = bias ? bias_mode : 0; p.out_f32 = out_f32; p.accumulate = accumulate;
  p.alpha = alpha; p.dropout = dropout; p.seed = seed;
  const int cfg = pick_cfg(M, N, K, batch);
  const int tbm = cfg ? 256 : nsdb::BM, tbn = cfg ? 256 : nsdb::BN;
  p.tiles_m = (M + tbm - 1) / tbm;
  p.tiles_n = (N + tbn - 1) / tbn;
  dim3 grid(p.tiles_m * p.tiles_n * p.splits, 1, batch);
  if (cfg)
    hipLaunchKernelGGL((nsdb::gemm_nt_tile_kernel<256, 256, 2, 4>), grid, dim3(512), 0, stream, p);
  else
    hipLaunchKernelGGL((nsdb::gemm_nt_tile_kernel<128, 128, 2, 2>), grid, dim3(256), 0, stream, p);
  if (p.splits > 1) {
    const long long MN = (long long)M * N;
    int blocks = (int)std::min<long long>((MN + 255) / 256, 4096);
    hipLaunchKernelGGL(nsdb::splitk_reduce_kernel, dim3(blocks, batch), dim3(256), 0, stream, p);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
