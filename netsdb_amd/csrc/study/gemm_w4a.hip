// "w4a": asm-scheduled 256x256x64 block GEMM for long-K split-K products (the FF layer-1 shape
// 1000 x 1000 x 597568 of src/FF/headers/FFTransposeMult.h + FFAggMatrix.h; the LA DSL's K-split
// %*% of src/sharedLibraries/headers/LASillyMultiply1Join.h + LASillyMultiply2Aggregate.h).
//
// Geometry: 4 waves (256 threads, ONE wave per SIMD), 2(M) x 2(N); each wave owns a 128x128 output block =
// 8x8 mfma_f32_16x16x32_bf16 tiles, 256 f32 accumulators per lane in AGPRs. Per k-tile a wave reads
// 16 + 16 fragments (ds_read_b128) for 128 MFMAs: 2/3 of the LDS bytes per MFMA of the 8-wave 8-phase kernel.
//
// Data path (the MT256x256x64 structure of hipBLASLt's Tensile kernel on gfx950, read from its code object,
// profiles/r2_gemm1_study/README.md): register-staged global loads (16 x buffer_load_dwordx4 per thread per
// k-tile, one tile ahead), ONE LDS buffer of 2 x 256 rows x 160 B (64 bf16 of k + 32 B pad: conflict-free
// ds_read_b128 fragment reads and ds_write_b128 stores without a swizzle), two barriers per k-tile.
//
// The main loop is written instruction by instruction: every MFMA, LDS read/write, global load, counted
// wait and barrier of a k-tile is an asm statement, emitted in a fixed order by scripts/gen_gemm_w4a.py
// (gemm_w4a_sched.inc), so hipcc cannot move a load, a wait or an MFMA (volatile asm keeps program order)
// and inserts no waits of its own (it issues no memory operation in the loop). Register-safety rules
// (cdna_hip_programming.md §5.7): every asynchronously written register (ds_read / buffer_load
// destinations) is named "+v" by the wait statement that retires it, so no compiler copy can read it
// early; the accumulators are "+a" operands of the MFMA statements only.
#include "../kernels/gemm_common.h"

namespace nsdb {

#define W4A_MFMA(mi, ni, FA, FB) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[mi][ni]) : "v"(FB[ni]), "v"(FA[mi]))
#define W4A_DSR(DST, ADDR, OFF) asm volatile("ds_read_b128 %0, %1 offset:" #OFF : "=v"(DST) : "v"(ADDR))
#define W4A_DSW(ADDR, SRC, OFF) asm volatile("ds_write_b128 %0, %1 offset:" #OFF ::"v"(ADDR), "v"(SRC) : "memory")
#define W4A_GL(DST, VOFF, SRD, SOFF) \
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(DST) : "v"(VOFF), "s"(SRD), "s"(SOFF) : "memory")
#define W4A_VMWAIT(N, REG) asm volatile("s_waitcnt vmcnt(" #N ")" : "+v"(REG)::"memory")
#define W4A_WAIT_FRAGS(FA, FB)                                                                              \
  asm volatile("s_waitcnt lgkmcnt(0)"                                                                       \
               : "+v"(FA[0]), "+v"(FA[1]), "+v"(FA[2]), "+v"(FA[3]), "+v"(FA[4]), "+v"(FA[5]), "+v"(FA[6]), \
                 "+v"(FA[7]), "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3]), "+v"(FB[4]), "+v"(FB[5]),   \
                 "+v"(FB[6]), "+v"(FB[7])::"memory")
#define W4A_WAIT_F1                    \
  do {                                 \
    W4A_WAIT_FRAGS(fa1, fb1);          \
    asm volatile("s_barrier" ::: "memory"); \
  } while (0)
#define W4A_WAIT_W asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
#define W4A_WAIT_F1_NB W4A_WAIT_FRAGS(fa1, fb1)
#define W4A_WAIT_W_NB asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define W4A_WAIT_F0 W4A_WAIT_FRAGS(fa0, fb0)

#include "gemm_w4a_sched.inc"

typedef int i32x4_t __attribute__((ext_vector_type(4)));

// 128-bit buffer descriptor in SGPRs (raw buffer, 32-bit range checked: offsets >= bytes read as zero)
__device__ __forceinline__ i32x4_t w4a_srd(const void* base, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32) & 0xffff);
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

template <int V>
__global__ void __launch_bounds__(256, 1) gemm_nt_256_w4a_kernel(GemmParams p) {
  constexpr int ROW = 160, B_BASE = 256 * ROW;
  __shared__ __attribute__((aligned(16))) char smem[2 * 256 * ROW];

  const int ntiles = p.tiles_m * p.tiles_n;
  const int wg = xcd_remap(blockIdx.x, ntiles * p.splits);
  const int split = wg / ntiles, tile = wg % ntiles;
  int tm, tn;
  grouped_tile(tile, p.tiles_m, p.tiles_n, tm, tn);
  const int batch = blockIdx.z;
  const int m0 = tm * 256, n0 = tn * 256;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  const int rows_a = min(256, p.M - m0), rows_b = min(256, p.N - n0);
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = max(0, (kend - kbeg) / BK);           // host guarantees K % 64 == 0 and kchunk % 64 == 0
  const i32x4_t srd_a = w4a_srd(p.A + batch * p.sA + (long long)m0 * p.lda + kbeg, (unsigned)((long long)rows_a * p.lda * 2));
  const i32x4_t srd_b = w4a_srd(p.B + batch * p.sB + (long long)n0 * p.ldb + kbeg, (unsigned)((long long)rows_b * p.ldb * 2));

  // staged chunk j of this thread: row (j & 7) * 32 + tid / 8 of A (j < 8) or B, 16-B chunk tid % 8
  const int lrow = tid >> 3, lch = tid & 7;
  int vo[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int r = (j & 7) * 32 + lrow;
    const bool isa = j < 8;
    const int rows = isa ? rows_a : rows_b;
    const long long ld = isa ? p.lda : p.ldb;
    vo[j] = r < rows ? (int)((long long)r * ld * 2 + lch * 16) : OOB;
  }
  const int wr_a = lrow * ROW + lch * 16;
  const int wr_b = B_BASE + wr_a;
  // fragment reads: row = w*128 + f*16 + (lane & 15), 16-B k-chunk (lane >> 4) (+4 for the second k-half)
  const int rd_a = (wr * 128 + (lane & 15)) * ROW + (lane >> 4) * 16;
  const int rd_b = B_BASE + (wc * 128 + (lane & 15)) * ROW + (lane >> 4) * 16;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  u32x4 sg[16];

  if (nk > 0) {
    // prologue: tile 0 -> LDS, tile 1 -> staging registers, F0 of tile 0
    int soff = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) W4A_GL(sg[j], vo[j], srd_a, soff);
#pragma unroll
    for (int j = 8; j < 16; ++j) W4A_GL(sg[j], vo[j], srd_b, soff);
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(sg[0]), "+v"(sg[1]), "+v"(sg[2]), "+v"(sg[3]), "+v"(sg[4]), "+v"(sg[5]), "+v"(sg[6]), "+v"(sg[7]),
                   "+v"(sg[8]), "+v"(sg[9]), "+v"(sg[10]), "+v"(sg[11]), "+v"(sg[12]), "+v"(sg[13]), "+v"(sg[14]),
                   "+v"(sg[15])::"memory");
    W4A_DSW(wr_a, sg[0], 0); W4A_DSW(wr_a, sg[1], 5120); W4A_DSW(wr_a, sg[2], 10240); W4A_DSW(wr_a, sg[3], 15360);
    W4A_DSW(wr_a, sg[4], 20480); W4A_DSW(wr_a, sg[5], 25600); W4A_DSW(wr_a, sg[6], 30720); W4A_DSW(wr_a, sg[7], 35840);
    W4A_DSW(wr_b, sg[8], 0); W4A_DSW(wr_b, sg[9], 5120); W4A_DSW(wr_b, sg[10], 10240); W4A_DSW(wr_b, sg[11], 15360);
    W4A_DSW(wr_b, sg[12], 20480); W4A_DSW(wr_b, sg[13], 25600); W4A_DSW(wr_b, sg[14], 30720); W4A_DSW(wr_b, sg[15], 35840);
    W4A_WAIT_W;
    soff = min(1, nk - 1) * (BK * 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) W4A_GL(sg[j], vo[j], srd_a, soff);
#pragma unroll
    for (int j = 8; j < 16; ++j) W4A_GL(sg[j], vo[j], srd_b, soff);
    W4A_DSR(fb0[0], rd_b, 0); W4A_DSR(fa0[0], rd_a, 0); W4A_DSR(fb0[1], rd_b, 2560); W4A_DSR(fa0[1], rd_a, 2560);
    W4A_DSR(fb0[2], rd_b, 5120); W4A_DSR(fa0[2], rd_a, 5120); W4A_DSR(fb0[3], rd_b, 7680); W4A_DSR(fa0[3], rd_a, 7680);
    W4A_DSR(fb0[4], rd_b, 10240); W4A_DSR(fa0[4], rd_a, 10240); W4A_DSR(fb0[5], rd_b, 12800); W4A_DSR(fa0[5], rd_a, 12800);
    W4A_DSR(fb0[6], rd_b, 15360); W4A_DSR(fa0[6], rd_a, 15360); W4A_DSR(fb0[7], rd_b, 17920); W4A_DSR(fa0[7], rd_a, 17920);
    W4A_WAIT_F0;
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");    // accumulator initialisation -> first MFMA srcC read

    for (int t = 0; t < nk; ++t) {
      // tile t+2 into the staging registers (clamped: the last iterations re-stage the last tile, unused)
      soff = min(t + 2, nk - 1) * (BK * 2);
      if constexpr (V == 0) { W4A_TILE_V0; }
      else if constexpr (V == 1) { W4A_TILE_V1; }
      else if constexpr (V == 2) { W4A_TILE_V2; }
      else if constexpr (V == 3) { W4A_TILE_V3; }     // diagnostics (timing only, wrong results): no loads
      else if constexpr (V == 4) { W4A_TILE_V4; }     // no LDS writes
      else if constexpr (V == 5) { W4A_TILE_V5; }     // no barriers
      else { W4A_TILE_V6; }                           // no fragment reads
    }
    // drain the trailing staging loads (they write registers the epilogue reuses) and let the last MFMAs
    // retire before the compiler's accumulator reads
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(sg[0]), "+v"(sg[1]), "+v"(sg[2]), "+v"(sg[3]), "+v"(sg[4]), "+v"(sg[5]), "+v"(sg[6]), "+v"(sg[7]),
                   "+v"(sg[8]), "+v"(sg[9]), "+v"(sg[10]), "+v"(sg[11]), "+v"(sg[12]), "+v"(sg[13]), "+v"(sg[14]),
                   "+v"(sg[15])::"memory");
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  }
  __syncthreads();
  store_tile_lds<256, 256, 2, 2, true>(acc, smem, (int)sizeof(smem), p, batch, split, m0, n0, tid, lane, wave);
}

}  // namespace nsdb

extern "C" {

// Launch the w4a kernel (variant v) for a split-K GEMM whose parameters the caller prepared (gemm.hip's
// launcher): K and every split's K range are multiples of 64; lda/ldb rows fit the 32-bit buffer range.
int nsdb_study_gemm_w4a_launch(const nsdb::GemmParams* p, int batch, int v, hipStream_t stream) {
  if (p->K % nsdb::BK != 0 || p->kchunk % nsdb::BK != 0) return -1;
  dim3 grid(p->tiles_m * p->tiles_n * p->splits, 1, batch);
  if (v == 1) hipLaunchKernelGGL(nsdb::gemm_nt_256_w4a_kernel<1>, grid, dim3(256), 0, stream, *p);
  else if (v == 2) hipLaunchKernelGGL(nsdb::gemm_nt_256_w4a_kernel<2>, grid, dim3(256), 0, stream, *p);
  else if (v == 3) hipLaunchKernelGGL(nsdb::gemm_nt_256_w4a_kernel<3>, grid, dim3(256), 0, stream, *p);
  else if (v == 4) hipLaunchKernelGGL(nsdb::gemm_nt_256_w4a_kernel<4>, grid, dim3(256), 0, stream, *p);
  else if (v == 5) hipLaunchKernelGGL(nsdb::gemm_nt_256_w4a_kernel<5>, grid, dim3(256), 0, stream, *p);
  else if (v == 6) hipLaunchKernelGGL(nsdb::gemm_nt_256_w4a_kernel<6>, grid, dim3(256), 0, stream, *p);
  else hipLaunchKernelGGL(nsdb::gemm_nt_256_w4a_kernel<0>, grid, dim3(256), 0, stream, *p);
  return (int)hipGetLastError();
}

}  // extern "C"
