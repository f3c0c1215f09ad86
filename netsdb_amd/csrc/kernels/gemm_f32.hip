// FP32-input MFMA block GEMM for the analytics libraries (k-means distance GEMM, GMM responsibility
// statistics: src/sharedLibraries/headers/KMeansAggregate.h / GmmAggregate.h compute these on doubles with
// per-point loops). gfx950 has exact f32-in / f32-accumulate MFMA (v_mfma_f32_16x16x4_f32: one f32 per lane per
// operand, products and sums in f32 — cdna_hip_programming.md §3 'FP32-input MFMA'), so precision-sensitive
// statistics stay at fp32 instead of going through the bf16 matrix path.
//
//   C[M, N] (f32) = alpha * A[M, K] . B[N, K]^T  (+ C when accumulate)     A, B f32, K-contiguous rows
//
//  * 128x128 tile, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 MFMA tiles of 16x16; K step 16.
//  * Operand fragments: for each 16-deep k step every lane reads ONE 16-B chunk (4 consecutive k) per m / n
//    tile with ds_read_b128 and feeds element s to the s-th of 4 MFMAs — MFMA s then sums over
//    k = 4 * (lane >> 4) + s, the same permutation of k on A and B, so the product is unchanged and each
//    operand costs one LDS read per 4 MFMAs.
//  * LDS tiles [128 rows][16 f32] = 64-B rows, 16-B chunk h of row r stored at slot (h + 2*((r >> 2) & 3)) & 3:
//    conflict-free for the ds_read_b128 lane groups ({0-3,12-15,20-27}, ...) and for the 8-lane ds_write_b128
//    groups of the register-staged stores.
//  * Register-staged double buffer: the next k step's global loads are issued before the current step's
//    MFMAs, written to the other LDS buffer after them; one barrier per k step.
#include "common.h"

namespace nsdb {

namespace {

constexpr int F_BM = 128, F_BN = 128, F_BK = 16;
constexpr int F_TILE = F_BM * F_BK;             // floats per operand per stage

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int f_slot(int row, int h) { return row * F_BK + (((h + 2 * ((row >> 2) & 3)) & 3) << 2); }

struct F32Params {
  const float* A;
  const float* B;
  float* C;
  long long lda, ldb, ldc;
  int M, N, K;
  float alpha;
  int accumulate;
};

__global__ void __launch_bounds__(256, 2) gemm_nt_f32_kernel(F32Params p) {
  __shared__ __attribute__((aligned(16))) float smem[2][2][F_TILE];   // [buffer][A,B][tile]
  const int tm = blockIdx.y, tn = blockIdx.x;
  const int m0 = tm * F_BM, n0 = tn * F_BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // staging: thread t loads chunks (row = t/4 + 64*i, h = t%4), i = 0, 1, of A and of B
  const int srow = tid >> 2, sh = tid & 3;
  f32x4_t ga[2], gb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = srow + 64 * i;
      const int k = k0 + sh * 4;
      const int ra = m0 + r, rb = n0 + r;
      ga[i] = (ra < p.M && k < p.K) ? *reinterpret_cast<const f32x4_t*>(p.A + (long long)ra * p.lda + k)
                                     : f32x4_t{0.f, 0.f, 0.f, 0.f};
      gb[i] = (rb < p.N && k < p.K) ? *reinterpret_cast<const f32x4_t*>(p.B + (long long)rb * p.ldb + k)
                                     : f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = srow + 64 * i;
      *reinterpret_cast<f32x4_t*>(&smem[buf][0][f_slot(r, sh)]) = ga[i];
      *reinterpret_cast<f32x4_t*>(&smem[buf][1][f_slot(r, sh)]) = gb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + F_BK - 1) / F_BK;
  const int fr = lane & 15, fh = lane >> 4;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) gload((t + 1) * F_BK);
    f32x4_t a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const f32x4_t*>(&smem[cur][0][f_slot(wm * 64 + i * 16 + fr, fh)]);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const f32x4_t*>(&smem[cur][1][f_slot(wn * 64 + j * 16 + fr, fh)]);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    if (t + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }
  // C/D map of 16x16x4: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + j * 16 + fr;
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + fh * 4 + r;
        if (row >= p.M) continue;
        float* d = p.C + (long long)row * p.ldc + col;
        const float v = acc[i][j][r] * p.alpha;
        *d = p.accumulate ? *d + v : v;
      }
    }
}

}  // namespace

}  // namespace nsdb

extern "C" {

// C = alpha * A . B^T (+ C): A [M, K], B [N, K] f32 with 16-B aligned rows (lda, ldb % 4 == 0, K % 4 == 0).
int nsdb_gemm_nt_f32(const float* A, const float* B, float* C, int M, int N, int K, long long lda, long long ldb,
                     long long ldc, float alpha, int accumulate, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 4 != 0 || lda % 4 != 0 || ldb % 4 != 0) return -1;
  if ((reinterpret_cast<uintptr_t>(A) & 15) || (reinterpret_cast<uintptr_t>(B) & 15)) return -2;
  nsdb::F32Params p{A, B, C, lda, ldb, ldc, M, N, K, alpha, accumulate};
  dim3 grid((N + nsdb::F_BN - 1) / nsdb::F_BN, (M + nsdb::F_BM - 1) / nsdb::F_BM);
  if (grid.y > 65535) return -3;
  hipLaunchKernelGGL(nsdb::gemm_nt_f32_kernel, grid, dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

}  // extern "C"
