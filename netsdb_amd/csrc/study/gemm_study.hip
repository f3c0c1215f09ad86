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
#include "../kernels/gemm_common.h"
#include <map>
#include <tuple>

namespace nsdb {


// (the fused softmax GEMM epilogue lives only in the product build, csrc/kernels/gemm.hip)

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
  int tm, tn;
  grouped_tile(tile, p.tiles_m, p.tiles_n, tm, tn);
  const int batch = blockIdx.z;
  const int m0 = tm * TBM, n0 = tn * TBN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;

  const int rows_a = min(TBM, p.M - m0), rows_b = min(TBN, p.N - n0);
  const unsigned short* Ab = p.A + batch * p.sA + (long long)m0 * p.lda;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = (kend - kbeg + BK - 1) / BK;
  const long long kseg = p.seg_k ? kbeg / p.seg_k : 0;
  const int kb0 = (int)(kseg * p.seg_k);      // B's k origin (segmented B)
  const unsigned short* Bb = p.B + batch * p.sB + (long long)n0 * p.ldb + kseg * p.seg_stride_b;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, (unsigned)((long long)rows_a * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, (unsigned)((long long)rows_b * p.ldb * 2));

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0 && !(p.diag & 2)) {
    stage_tile<TBM, NW>(ra, smem, p.lda, rows_a, kbeg, kend, wave, lane);
    stage_tile<TBN, NW>(rb, smem + A_BYTES, p.ldb, rows_b, kbeg - kb0, kend - kb0, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STG;
    if (t + 1 < nk && !(p.diag & 2)) {
      char* nxt = smem + ((t + 1) & 1) * STG;
      const int k1 = kbeg + (t + 1) * BK;
      stage_tile<TBM, NW>(ra, nxt, p.lda, rows_a, k1, kend, wave, lane);
      stage_tile<TBN, NW>(rb, nxt + A_BYTES, p.ldb, rows_b, k1 - kb0, kend - kb0, wave, lane);
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

  store_tile_lds<TBM, TBN, WGM, WGN>(acc, smem, 2 * STG, p, batch, split, m0, n0, tid, lane, wave);
}

// ---------------------------------------------------------------------------------------------
// 256x256x64 "8-phase" kernel for long-K / large shapes (cdna_hip_programming.md §5, the 256^2
// 8-phase template): 512 threads = 8 waves as 2(M) x 4(N), each wave 128x64 = 8x4 MFMA tiles.
//
//  * Each K-tile (64 KiB: A 256x64 + B 256x64) is held as four 16 KiB "half-tiles" in LDS:
//      A0 = rows {0..63, 128..191}, A1 = rows {64..127, 192..255}      (wave M-group wr: rows wr*128+qm*64..)
//      B0 = rows {wc*64 + 0..31},    B1 = rows {wc*64 + 32..63}           (wave N index wc)
//    so the C-quadrant (qm, qn) a wave computes in a phase reads exactly half-tiles A_qm and B_qn.
//  * 4 phases per K-tile, quadrant order (0,0) (0,1) (1,1) (1,0); 2 LDS buffers, 2 K-tiles/iteration.
//    Every phase: ds_read its fragments -> issue ONE half-tile LDS-DMA (2 x buffer_load...lds per
//    thread) -> raw s_barrier -> lgkmcnt(0) -> 16 MFMAs at high priority -> raw s_barrier.
//  * Wave group wr=1 runs one barrier behind wr=0 (one extra s_barrier up front): on every SIMD one
//    wave is on the MFMAs while the other issues its LDS reads and DMA (ping-pong).
//  * Staging schedule for the tile t in buffer b (phase j):
//      j0 -> A1 of t+1 (buffer b^1)   j1 -> B0 of t+2 (b)   j2 -> A0 of t+2 (b)   j3 -> B1 of t+2 (b)
//    WAR: a half-tile is restaged >= 2 phases after its last ds_read, or 1 phase after when a counted
//    lgkmcnt before the reading phase's first barrier retired those reads (B0: lgkmcnt(8) in j0 —
//    its 4 B reads are issued first, then 8 A reads, order pinned by sched_barrier).
//    RAW: s_waitcnt vmcnt(6) in j3 (3 half-tiles stay in flight across the barrier) retires all of
//    tile t+1, which is first read in the NEXT phase (never in the same phase as its wait).
//    vmcnt is never 0 inside the loop; beyond the last K-tile the DMA targets k >= kend, which the
//    buffer range check zero-fills, so every phase issues the same number of VMEM ops.
//  * All LDS is one __shared__ array (a second object makes hipcc drain vmcnt before ds_reads).
// ---------------------------------------------------------------------------------------------
#define NSDB_BARRIER()                          \
  do {                                          \
    __builtin_amdgcn_sched_barrier(0);          \
    asm volatile("s_barrier" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0);          \
  } while (0)

// V: diagnostic variants (0 = production). 1 no setprio, 2 stage before ds_reads, 3 no group stagger,
// 4 no DMA issued (load-free upper bound, wrong results), 5 no ds_reads after the first tile (wrong results),
// 6 no vmcnt wait in the loop (racy), 7 zero-record descriptors (DMA issued, no memory traffic),
// 8 vmcnt(2) instead of 6 (1 half-tile in flight: latency sensitivity)

template <int V>
__global__ void __launch_bounds__(512, 2) gemm_nt_256_8ph_kernel(GemmParams p) {
  constexpr int HALF = 128 * 128;            // bytes of one half-tile (128 rows x 64 bf16)
  constexpr int BUF = 4 * HALF;              // one K-tile
  // RING (variant 10): the 160 KiB LDS as a ring of 10 half-tile slots. Half-tile h = 4u + q (staging
  // order q: B0, A0, B1, A1 of k-tile u) lives in slot h % 10 and is staged at phase P = h - 9 (P = 4u' + j
  // counts phases), so 5 half-tiles (80 KiB) stay in flight across the barriers instead of 3: the
  // slot restaged at phase P held half-tile P - 1, the same WAR distance as the 2-buffer schedule.
  constexpr bool RING = (V == 10);
  // TS: the MFMA computes the TRANSPOSED 16x16 tile (B fragment as the A operand), so lane l holds
  // C[row = l & 15][4 consecutive columns 4*(l >> 4) ..] per accumulator: the epilogue spills each tile to LDS
  // with one 16-B write (store_tile_lds TSL). Variant 11 keeps the untransposed layout (A/B). (Storing those
  // 16 B straight from registers to global — 16 rows x 64 B per wave-instruction — measured 40 us of store
  // tail on the 1000x14588 f32 output vs 21 us through the LDS image and full-row 1 KiB stores.)
  constexpr bool TS = (V != 11);
  constexpr int NRING = 10;
  __shared__ __attribute__((aligned(16))) char smem[RING ? NRING * HALF : 2 * BUF];

  const int ntiles = p.tiles_m * p.tiles_n;
  const int wg = xcd_remap(blockIdx.x, ntiles * p.splits);
  const int split = wg / ntiles, tile = wg % ntiles;
  int tm, tn;
  grouped_tile(tile, p.tiles_m, p.tiles_n, tm, tn);
  const int batch = blockIdx.z;
  const int m0 = tm * 256, n0 = tn * 256;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int rows_a = min(256, p.M - m0), rows_b = min(256, p.N - n0);
  AdaptState* const ad = (V == 0 && p.adapt != nullptr) ? p.adapt : nullptr;
  int kbeg = split * p.kchunk;
  int kend = min(p.K, kbeg + p.kchunk);
  if (ad != nullptr) {
    // this split's K range from the shares (identical arithmetic in every workgroup)
    const int total = (p.K + BK - 1) / BK;
    float acc_s = 0.f, tot_s = 0.f;
    for (int g = 0; g < p.splits; ++g) {
      const float sh = ad->share[g];
      tot_s += sh;
      if (g < split) acc_s += sh;
    }
    const float my_s = ad->share[split];
    if (tot_s > 0.f) {
      const int b0 = (int)((float)total * (acc_s / tot_s) + 0.5f);
      const int b1 = split == p.splits - 1 ? total : (int)((float)total * ((acc_s + my_s) / tot_s) + 0.5f);
      kbeg = min(b0, total) * BK;
      kend = min(p.K, min(b1, total) * BK);
    }
  }
  // start time kept in a register and stored with the finish time: a vector store (or load) pending at the
  // loop entry would make the compiler's wait-count pass put vmcnt(0) waits into the counted-vmcnt loop
  const unsigned long long t_begin = ad != nullptr ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // V19: this workgroup's static part stops steal_tq * steal_ch k-tiles short of its split's end; those tail
  // chunks (of every split of the tile) are claimed afterwards by whichever workgroup of the tile is free first
  if constexpr (V == 19) kend = max(kbeg, min(kend, kbeg + p.kchunk - p.steal_tq * p.steal_ch * BK));
  if constexpr (V == 22) {   // pair range [2 * (split / 2) * kchunk, ...): this split takes every other k-tile
    kbeg = (split & ~1) * p.kchunk;
    kend = min(p.K, kbeg + 2 * p.kchunk);
  }
  int nk = V == 22 ? max(0, ((kend - kbeg + BK - 1) / BK - (split & 1) + 1) / 2) : max(0, (kend - kbeg + BK - 1) / BK);
  int niter = (nk + 1) >> 1;

  // KT (variant 9): K-tiled operands [K/64][ld rows][64] — every (tile, k-step) half-tile is one
  // contiguous 16 KiB run instead of 128 rows x 128 B strided by the row length (DRAM page locality
  // study). lda/ldb are then the padded row counts; the descriptor base sits at this split's first slab.
  constexpr bool KT = (V == 9);
  const unsigned short* Ab = KT ? p.A + batch * p.sA + ((long long)(kbeg / BK) * p.lda + m0) * BK
                                : p.A + batch * p.sA + (long long)m0 * p.lda;
  const long long kseg = (!KT && p.seg_k) ? kbeg / p.seg_k : 0;
  const int kb0 = (int)(kseg * p.seg_k);      // B's k origin (segmented B)
  const unsigned short* Bb = KT ? p.B + batch * p.sB + ((long long)(kbeg / BK) * p.ldb + n0) * BK
                                : p.B + batch * p.sB + (long long)n0 * p.ldb + kseg * p.seg_stride_b;
  const long long bytes_a = KT ? std::min<long long>(0x7fffffffLL, (long long)nk * p.lda * BK * 2) : (long long)rows_a * p.lda * 2;
  const long long bytes_b = KT ? std::min<long long>(0x7fffffffLL, (long long)nk * p.ldb * BK * 2) : (long long)rows_b * p.ldb * 2;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, V == 7 ? 0u : (unsigned)bytes_a);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, V == 7 ? 0u : (unsigned)bytes_b);
  const int slab_a = KT ? p.lda * BK * 2 : 0, slab_b = KT ? p.ldb * BK * 2 : 0;

  // Per-thread DMA source rows. Wave-instruction i of a half-tile fills LDS rows
  // hr = i*64 + wave*8 + (lane>>3) (1 KiB, lane-linear); the logical 16-B chunk at physical slot
  // lane&7 is chunk ^ ((hr>>1)&7) (same swizzle as read_frag), hence a per-lane k offset.
  const int lr = wave * 8 + (lane >> 3);
  const int kc = ((lane & 7) ^ ((lr >> 1) & 7)) * 8;
  int roff[4][2];      // [slot A0,A1,B0,B1][i] byte offset of the source row, or -1 if out of range
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ta = i * 128 + q * 64 + lr;
      const int tb = (2 * i + (lr >> 5)) * 64 + q * 32 + (lr & 31);
      roff[q][i] = ta < rows_a ? (KT ? ta * BK * 2 : (int)((long long)ta * p.lda * 2)) : -1;
      roff[2 + q][i] = tb < rows_b ? (KT ? tb * BK * 2 : (int)((long long)tb * p.ldb * 2)) : -1;
    }

  // cache-policy bits of the operand DMAs (gfx950 CPol: sc0 1, nt 2, sc1 16): V15 nt on both; V16 sc1 (L1
  // bypass) on both; V17 nt+sc1 on B only; V18 nt+sc1 on A only (hipBLASLt's MT256x256x64 streams one operand
  // with `nt sc1`)
  constexpr int AUX_A = V == 15 ? 2 : V == 16 ? 16 : V == 18 ? 18 : 0;
  constexpr int AUX_B = V == 15 ? 2 : V == 16 ? 16 : V == 17 ? 18 : 0;
  auto stage = [&](int buf, int slot, int u) {
    if constexpr (V == 4) return;
    const int k = kbeg + u * BK + kc;
    const bool kin = (V == 22 ? kbeg + (2 * u + (split & 1)) * BK + kc : k) < kend;
    // memory-side diagnostics (timing only, wrong results): 13 every split streams the SAME K window
    // [0, kchunk) (unique bytes / splits: Infinity-Cache resident); 14 every workgroup cycles over 2 k-tiles
    // (L2/L1 resident: the L2 -> CU path alone)
    // V22: the two splits an XCD runs interleave their k-tiles over the pair's joint K range (split parity p
    // takes k-tiles 2u + p), so both stream the same DRAM pages at the same time
    const int ks = V == 13 ? k - kbeg : V == 14 ? (u & 1) * BK + kc : V == 22 ? kbeg + (2 * u + (split & 1)) * BK + kc : k;
    char* dst = RING ? smem + buf * HALF : smem + buf * BUF + slot * HALF;   // RING: buf = ring slot
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ro = roff[slot][i];
      const int voff = (kin && ro >= 0) ? (KT ? u * (slot < 2 ? slab_a : slab_b) + ro + kc * 2
                                              : ro + (slot < 2 ? ks : ks - kb0) * 2) : OOB;
      // V15: non-temporal operand stream (aux nt): the once-streamed panels do not displace the split-K slabs
      // (and other resident sets) from the Infinity Cache
      if (slot < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(dst + (i * 64 + wave * 8) * 128), 16, voff, 0, 0, AUX_A);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst + (i * 64 + wave * 8) * 128), 16, voff, 0, 0, AUX_B);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], b0[2][2], b1[2][2];

  bool skip_reads = false;
  auto readA = [&](int buf, int q) {
    if constexpr (V == 5) { if (skip_reads) return; }
    const char* base = smem + buf * BUF + q * HALF;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kk] = read_frag(base, wr * 64 + mi * 16 + (lane & 15), kk * 4 + (lane >> 4));
  };
  auto readB = [&](int buf, int q, bf16x8 (&bq)[2][2]) {
    if constexpr (V == 5) { if (skip_reads) return; }
    const char* base = smem + buf * BUF + (2 + q) * HALF;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bq[ni][kk] = read_frag(base, wc * 32 + ni * 16 + (lane & 15), kk * 4 + (lane >> 4));
  };
  auto mma = [&](int qm, int qn, const bf16x8 (&bq)[2][2]) {
    NSDB_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (V != 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[qm * 4 + mi][qn * 2 + ni] = TS
              ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ni][kk], af[mi][kk], acc[qm * 4 + mi][qn * 2 + ni], 0, 0, 0)
              : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][kk], bq[ni][kk], acc[qm * 4 + mi][qn * 2 + ni], 0, 0, 0);
    if constexpr (V != 1) __builtin_amdgcn_s_setprio(0);
    NSDB_BARRIER();
  };
  // RING: half-tile h = 4u + q, q = 0 B0, 1 A0, 2 B1, 3 A1 (slot ids A0=0, A1=1, B0=2, B1=3)
  auto stage_h = [&](int h) {
    constexpr int slot_of[4] = {2, 0, 3, 1};
    stage(h % NRING, slot_of[h & 3], h >> 2);
  };
  auto ring_base = [&](int u, int q) { return smem + ((4 * u + q) % NRING) * HALF; };
  auto readA_r = [&](const char* base) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kk] = read_frag(base, wr * 64 + mi * 16 + (lane & 15), kk * 4 + (lane >> 4));
  };
  auto readB_r = [&](const char* base, bf16x8 (&bq)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bq[ni][kk] = read_frag(base, wc * 32 + ni * 16 + (lane & 15), kk * 4 + (lane >> 4));
  };
  auto ktile_ring = [&](int u) {
    // j0: (0,0) reads B0, A0 of u; stages h = 4u+9 (A0 of u+2)
    readB_r(ring_base(u, 0), b0);
    __builtin_amdgcn_sched_barrier(0);
    readA_r(ring_base(u, 1));
    stage_h(4 * u + 9);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");   // B0 reads retired before the barrier
    mma(0, 0, b0);
    // j1: (0,1) reads B1; stages B1 of u+2 (into B0(u)'s slot, read in j0)
    readB_r(ring_base(u, 2), b1);
    stage_h(4 * u + 10);
    mma(0, 1, b1);
    // j2: (1,1) reads A1; stages A1 of u+2
    readA_r(ring_base(u, 3));
    stage_h(4 * u + 11);
    mma(1, 1, b1);
    // j3: (1,0) from registers; stages B0 of u+3; retires k-tile u+1 (5 half-tiles stay in flight)
    stage_h(4 * u + 12);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    mma(1, 0, b0);
  };
  // one K-tile u held in buffer `cur` (u+1 in cur^1)
  auto ktile = [&](int cur, int u) {
    // j0: quadrant (0,0); reads B0 then A0; stages A1 of u+1
    if constexpr (V == 2) stage(cur ^ 1, 1, u + 1);
    readB(cur, 0, b0);
    __builtin_amdgcn_sched_barrier(0);
    readA(cur, 0);
    if constexpr (V != 2) stage(cur ^ 1, 1, u + 1);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");   // the 4 B0 reads (issued first) are done
    mma(0, 0, b0);
    // j1: quadrant (0,1); reads B1; stages B0 of u+2
    if constexpr (V == 2) stage(cur, 2, u + 2);
    readB(cur, 1, b1);
    if constexpr (V != 2) stage(cur, 2, u + 2);
    mma(0, 1, b1);
    // j2: quadrant (1,1); reads A1; stages A0 of u+2
    if constexpr (V == 2) stage(cur, 0, u + 2);
    readA(cur, 1);
    if constexpr (V != 2) stage(cur, 0, u + 2);
    mma(1, 1, b1);
    // j3: quadrant (1,0) from registers; stages B1 of u+2; retires tile u+1 (3 half-tiles stay in flight)
    stage(cur, 3, u + 2);
    if constexpr (V == 8) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (V != 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    mma(1, 0, b0);
  };

  if constexpr (RING) {
    // prologue: half-tiles 0..8 (tile 0, tile 1, B0 of tile 2); tile 0 complete when <= 10 ops remain
#pragma unroll
    for (int h = 0; h < 9; ++h) stage_h(h);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    NSDB_BARRIER();
    if (wr == 1) NSDB_BARRIER();
    for (int u = 0; u < nk; ++u) ktile_ring(u);
  } else {
  for (int seg = 0;; ++seg) {      // V19: the static part, then claimed tail chunks (one segment otherwise)
  // prologue: tile 0 (4 halves) + B0, A0, B1 of tile 1; tile 0 complete when <= 6 ops remain
  stage(0, 2, 0); stage(0, 0, 0); stage(0, 3, 0); stage(0, 1, 0);
  stage(1, 2, 1); stage(1, 0, 1); stage(1, 3, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  NSDB_BARRIER();
  if (V != 3 && wr == 1) NSDB_BARRIER();            // stagger the two wave groups by one barrier

  for (int it = 0; it < niter; ++it) {
    ktile(0, 2 * it);
    ktile(1, 2 * it + 1);
    if constexpr (V == 5) skip_reads = true;
    if constexpr (V == 12) {     // progress stamps (100 MHz real-time clock, comparable across CUs)
      if (tid == 0 && (it & 15) == 0) p.stamps[(long long)wg * 64 + min(it >> 4, 62)] = __builtin_amdgcn_s_memrealtime();
    }
  }
  if constexpr (V != 19) {
    break;
  } else {
    // segment done: re-align the wave groups, drain every wave's trailing DMAs, then claim the tile's next tail
    // chunk (one returning vector atomic by thread 0, broadcast through LDS between two full barriers)
    if (wr == 0) NSDB_BARRIER();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* slot = reinterpret_cast<int*>(smem);
    const int nchunks = p.splits * p.steal_tq;
    if (tid == 0) {
      int c = nchunks, kb = 0, ke = 0;
      while (true) {                                  // skip empty chunks (short last split); bounded by nchunks
        c = __hip_atomic_fetch_add(&p.steal_cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c >= nchunks) break;
        const int v = c % p.splits, j = c / p.splits;
        const int vend = min(p.K, (v + 1) * p.kchunk);
        const int tail0 = max(v * p.kchunk, v * p.kchunk + p.kchunk - p.steal_tq * p.steal_ch * BK);
        kb = tail0 + j * p.steal_ch * BK;
        ke = min(vend, kb + p.steal_ch * BK);
        if (kb < ke) break;
      }
      slot[0] = c < nchunks ? kb : -1;
      slot[1] = ke;
    }
    __syncthreads();
    const int nkb = slot[0], nke = slot[1];
    __syncthreads();                                  // slot read before the next prologue's DMAs land
    if (nkb < 0) break;
    kbeg = nkb;
    kend = nke;
    nk = (kend - kbeg + BK - 1) / BK;
    niter = (nk + 1) >> 1;
  }
  }
  }
  if constexpr (V == 12) {      // slot 63: the XCD this workgroup ran on (HW_REG_XCC_ID) and its CU id
    if (tid == 0) p.stamps[(long long)wg * 64 + 63] =
        ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) | (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 4);
  }
  if (V != 3 && V != 19 && wr == 0) NSDB_BARRIER();  // re-align the groups (V19 re-aligned per segment)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing zero-fill DMAs land before LDS reuse
  if ((V == 0 || V == 19) && p.signal != nullptr && tid == 0)   // tail trigger: this CU frees up soon
    __hip_atomic_fetch_max(p.signal, p.signal_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (ad != nullptr) {
    // finish time; the last workgroup of the launch derives the next launch's shares (the groups are
    // re-aligned here, so the block-wide barriers below pair up)
    // (the flag lives in the tile buffer, free here: a second __shared__ object makes the wait-count pass
    // assume the loop's LDS-DMA writes may alias its ds_reads and put vmcnt(0) before every one of them)
    int& adapt_last = reinterpret_cast<int*>(smem)[64 * 65];
    if (tid == 0) {
      ad->t0[wg] = t_begin;
      ad->t1[wg] = __builtin_amdgcn_s_memrealtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const unsigned c = __hip_atomic_fetch_add(&ad->cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      adapt_last = (c + 1 == (unsigned)(ntiles * p.splits)) ? 1 : 0;
    }
    __syncthreads();
    if (adapt_last && wave == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const int total = (p.K + BK - 1) / BK;
      float acc_s = 0.f, tot_s = 0.f, my_s = 0.f;
      for (int g = 0; g < p.splits; ++g) {
        const float sh = ad->share[g];
        tot_s += sh;
        if (g < lane) acc_s += sh;
        if (g == lane) my_s = sh;
      }
      float rate = 0.f;
      if (lane < p.splits) {
        int kt = (total + p.splits - 1) / p.splits;
        if (tot_s > 0.f) {
          const int b0 = (int)((float)total * (acc_s / tot_s) + 0.5f);
          const int b1 = lane == p.splits - 1 ? total : (int)((float)total * ((acc_s + my_s) / tot_s) + 0.5f);
          kt = b1 - b0;
        } else {
          kt = min(total, (lane + 1) * kt) - min(total, lane * kt);
        }
        // median duration of the split's workgroups: durations staged in LDS (row per split), rank select
        float* dl = reinterpret_cast<float*>(smem) + lane * 65;
        const int n = ntiles;          // <= 64 (host guard)
        for (int i = 0; i < n; ++i) {
          const int w = lane * ntiles + i;
          dl[i] = (float)(long long)(__hip_atomic_load(&ad->t1[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                                     __hip_atomic_load(&ad->t0[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        float med = 1.f;
        for (int i = 0; i < n; ++i) {
          const float di = dl[i];
          int rank = 0;
          for (int j = 0; j < n; ++j) {
            const float dj = dl[j];
            rank += (dj < di || (dj == di && j < i)) ? 1 : 0;
          }
          if (rank == n / 2) med = fmaxf(di, 1.f);
        }
        const float r = (float)max(kt, 1) / med;
        const float prev = ad->rate[lane];
        rate = prev > 0.f ? 0.5f * prev + 0.5f * r : r;
      }
      float sum = rate;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
      if (lane < p.splits && sum > 0.f) {
        const float eq = 1.f / (float)p.splits;
        ad->rate[lane] = rate;
        ad->share[lane] = fminf(fmaxf(rate / sum, 0.6f * eq), 1.4f * eq);   // readers renormalise
      }
      if (lane == 0) ad->cnt = 0u;     // ready for the next launch (stream-ordered after this one)
    }
    __syncthreads();                   // LDS scratch above is reused by the epilogue
  }
  store_tile_lds<256, 256, 2, 4, TS>(acc, smem, (int)sizeof(smem), p, batch, split, m0, n0, tid, lane, wave);
  if constexpr (V == 23) {
    // split-K fix-up in the GEMM launch (no reducer kernel): every workgroup releases its slab and counts itself
    // in on the tile's arrival counter; the last one to arrive sums the tile's slabs in split order (the
    // reducer's order: bit-identical results) and runs the reducer's epilogue, then re-zeroes the counter.
    // No workgroup waits on another (host guard: vec_ws, batch 1, no segmented B).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();                                   // every wave's slab stores released; LDS image consumed
    int* last = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      const int c = __hip_atomic_fetch_add(&p.steal_cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last[0] = (c == p.splits - 1) ? 1 : 0;
    }
    __syncthreads();
    if (last[0] == 0) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const long long MN = (long long)p.M * p.N;
    const int cq = tid & 63;                           // column quad of the tile (64 x 4 columns)
    const int col = n0 + cq * 4;
    if (col < p.N) {
      for (int r = tid >> 6; r < 256 && m0 + r < p.M; r += 8) {
        const long long e = (long long)(m0 + r) * p.N + col;
        const float* w = p.ws + e;
        f32x4 part[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k < p.splits) part[k] = *reinterpret_cast<const f32x4*>(w + k * MN);
        f32x4 s = part[0];
#pragma unroll
        for (int k = 1; k < 16; ++k)
          if (k < p.splits) s += part[k];
        for (int k = 16; k < p.splits; ++k) s += *reinterpret_cast<const f32x4*>(w + k * MN);
        reduce_epilogue4(p, 0, MN, e, s);
      }
    }
    if (tid == 0) p.steal_cnt[tile] = 0;               // next launch is stream-ordered after this one
  }
}

// ---------------------------------------------------------------------------------------------
// 256x256x64 "w4" kernel: 4 waves (256 threads, ONE wave per SIMD), 2(M) x 2(N), each wave owns a
// 128x128 output block = 8x8 mfma_f32_16x16x32_bf16 tiles, 256 f32 accumulators per lane (AGPRs;
// 512-register budget at one wave/SIMD).
//
//  * LDS per MFMA: each k32 sub-step a wave reads 8 A + 8 B fragments (16 ds_read_b128) for 64 MFMAs,
//    2/3 of the LDS bytes per FLOP of the 8-wave 128x64-per-wave 8-phase kernel (24 reads / 64 MFMAs).
//  * Register double buffer: fragment sets R0 (k32 sub-step s0) and R1 (s1). The reads of the next
//    sub-step are issued between the MFMAs of the current one (sched_group_barrier interleave), so the
//    MFMA stream never waits on an LDS round trip; one wave per SIMD hides its own latencies.
//  * LDS ring of 5 operand slots (32 KiB = 256 rows x 64 bf16 each; 160 KiB): k-tile u's A in slot
//    (2u)%5, its B in slot (2u+1)%5. One barrier per k-tile, between the two sub-steps' MFMA blocks:
//        [s0 MFMAs on R0 | ds_read s1 -> R1]  lgkmcnt(0) vmcnt(8) s_barrier  (tile t+1 landed, every
//        read of tile t retired)  stage B of t+2 and A of t+3 into tile t's two slots
//        [s1 MFMAs on R1 | ds_read s0 of tile t+1 -> R0 | 16 LDS-DMA issues]
//    so A is fetched 2 k-tiles ahead and B 1 k-tile ahead (64-96 KiB in flight per CU); vmcnt is never
//    0 inside the loop (the youngest half-tile, A of t+2, stays in flight across the barrier).
//  * DMA rows are 128 B (full cache lines); LDS image lane-linear per wave-instruction with the same
//    XOR swizzle as read_frag applied to the per-lane SOURCE k (rule 21). Rows past M/N are zero-filled
//    by the descriptor's range check; k past the split is redirected out of range.
// ---------------------------------------------------------------------------------------------
template <int V>
__global__ void __launch_bounds__(256, 1) gemm_nt_256_w4_kernel(GemmParams p) {
  constexpr int SLOT = 256 * 128;             // one operand's 256 rows x 64 bf16
  constexpr int NSLOT = 5;
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];

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
  const int nk = max(0, (kend - kbeg + BK - 1) / BK);
  const long long kseg = p.seg_k ? kbeg / p.seg_k : 0;
  const int kb0 = (int)(kseg * p.seg_k);
  const unsigned short* Ab = p.A + batch * p.sA + (long long)m0 * p.lda;
  const unsigned short* Bb = p.B + batch * p.sB + (long long)n0 * p.ldb + kseg * p.seg_stride_b;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, (unsigned)((long long)rows_a * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, (unsigned)((long long)rows_b * p.ldb * 2));

  // DMA: wave-instruction i (0..7) of a slot fills rows i*32 + wave*8 + (lane>>3); physical 16-B slot
  // lane&7 holds logical chunk (lane&7) ^ ((row>>1)&7), and (row>>1)&7 does not depend on i.
  const int hr0 = wave * 8 + (lane >> 3);
  const int kc = ((lane & 7) ^ ((hr0 >> 1) & 7)) * 8;
  const unsigned a_lane = (unsigned)(hr0 * p.lda * 2 + kc * 2), b_lane = (unsigned)(hr0 * p.ldb * 2 + kc * 2);
  const unsigned a_step = (unsigned)(32 * p.lda * 2), b_step = (unsigned)(32 * p.ldb * 2);

  auto stage = [&](int op, int u) {
    if constexpr (V == 4) return;
    const int slot = (2 * u + op) % NSLOT;
    char* dst = smem + slot * SLOT + wave * 8 * 128;
    const int k = kbeg + u * BK;                        // this k-tile's first k (absolute)
    const bool kin = k + kc < kend;
    const unsigned base = op == 0 ? a_lane + (unsigned)k * 2 : b_lane + (unsigned)(k - kb0) * 2;
    const unsigned step = op == 0 ? a_step : b_step;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned voff = kin ? base + i * step : (unsigned)OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(op == 0 ? ra : rb, (lds_void*)(dst + i * 32 * 128), 16, (int)voff, 0, 0, 0);
    }
  };

  auto stage_one = [&](int op, int u, int i) {
    if constexpr (V == 4) return;
    const int slot = (2 * u + op) % NSLOT;
    char* dst = smem + slot * SLOT + wave * 8 * 128 + i * 32 * 128;
    const int k = kbeg + u * BK;
    const bool kin = k + kc < kend;
    const unsigned voff = kin ? (op == 0 ? a_lane + (unsigned)k * 2 + i * a_step : b_lane + (unsigned)(k - kb0) * 2 + i * b_step)
                              : (unsigned)OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(op == 0 ? ra : rb, (lds_void*)dst, 16, (int)voff, 0, 0, 0);
  };

  // Fragment reads: row = w*128 + f*16 + (lane&15), (row>>1)&7 = ((lane&15)>>1); f adds 2 KiB (imm offset).
  const int rl = lane & 15, sw = (rl >> 1) & 7;
  const int off_s0 = rl * 128 + (((lane >> 4)) ^ sw) * 16;
  const int off_s1 = rl * 128 + ((4 + (lane >> 4)) ^ sw) * 16;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[8], a1[8], b1[8];

  auto read_set = [&](int u, int off, bf16x8 (&af)[8], bf16x8 (&bq)[8]) {
    const char* sa = smem + ((2 * u) % NSLOT) * SLOT + wr * 128 * 128 + off;
    const char* sb = smem + ((2 * u + 1) % NSLOT) * SLOT + wc * 128 * 128 + off;
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = *reinterpret_cast<const bf16x8*>(sa + f * 2048);
      bq[f] = *reinterpret_cast<const bf16x8*>(sb + f * 2048);
    }
  };
  // 64 MFMAs on (af, bq) with the 16 fragment reads of the next sub-step (B first: the next block's
  // first row of MFMAs needs every B fragment) interleaved 1 per 2 MFMAs over the first 32, and, with
  // DMA, 16 LDS-DMA issues interleaved 1 per 4 MFMAs. The MFMAs are inline asm with the accumulator pinned to AGPRs ("+a", in place): the
  // builtin's register-class heuristics at 512 registers copy every accumulator AGPR<->VGPR per
  // iteration. Source order is the issue order (the asm is volatile); hipcc still inserts the
  // counted lgkmcnt waits for the fragment registers the asm reads.
  auto mma_rd = [&](const bf16x8 (&af)[8], const bf16x8 (&bq)[8], int u_next, int off_next, bf16x8 (&an)[8],
                    bf16x8 (&bn)[8], bool dma, int t) {
    const char* sa = smem + ((2 * u_next) % NSLOT) * SLOT + wr * 128 * 128 + off_next;
    const char* sb = smem + ((2 * u_next + 1) % NSLOT) * SLOT + wc * 128 * 128 + off_next;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(af[i]), "v"(bq[j]));
        // reads in the first half of the block (1 per 2 MFMAs): they retire long before the next
        // block's first MFMA / the barrier's lgkmcnt(0)
        if (i < 4 && (j & 1) == 1) {
          const int r = i * 4 + (j >> 1);        // 0..15
          if (r < 8) bn[r] = *reinterpret_cast<const bf16x8*>(sb + r * 2048);
          else an[r - 8] = *reinterpret_cast<const bf16x8*>(sa + (r - 8) * 2048);
        }
        if (dma && (j & 3) == 3) {
          const int g = i * 2 + (j >> 2);        // 0..15
          if (g < 8) stage_one(1, t + 2, g);
          else stage_one(0, t + 3, g - 8);
        }
      }
  };

  // prologue: A0 B0 A1 B1 A2 in flight; tile 0 complete when <= 3 half-tiles (24 ops) remain
  stage(0, 0); stage(1, 0); stage(0, 1); stage(1, 1); stage(0, 2);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  NSDB_BARRIER();
  read_set(0, off_s0, a0, b0);

  for (int t = 0; t < nk; ++t) {
    // s0: 64 MFMAs on R0 | the s1 reads of tile t -> R1
    mma_rd(a0, b0, t, off_s1, a1, b1, false, t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (V != 6) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    NSDB_BARRIER();
    // s1: 64 MFMAs on R1 | tile t+1's s0 reads -> R0 | DMA of B(t+2), A(t+3) into tile t's slots
    mma_rd(a1, b1, t + 1, off_s0, a0, b0, true, t);
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // MFMA results -> AGPR reads (asm: no hazard padding)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing zero-fill DMAs land before LDS reuse
  __syncthreads();
  store_tile_lds<256, 256, 2, 2>(acc, smem, NSLOT * SLOT, p, batch, split, m0, n0, tid, lane, wave);
}

// ---------------------------------------------------------------------------------------------
// "w4r": the 4-wave / 128x128-per-wave 256x256x64 tile (one wave per SIMD, 256 AGPR accumulators — the
// structure hipBLASLt's Tensile kernel uses on gfx950: MT256x256x64, 256 threads, ~130 KiB LDS) with
// REGISTER-staged global loads instead of LDS-DMA. The LDS-DMA variant (w4 above) paid ~60+ issue cycles per
// buffer_load...lds (MI355X_MICROARCH 'LDS-DMA piece issue cost'): 16 per wave per k-tile next to 128 MFMAs
// left the MFMA pipe idle; a global_load_dwordx4 + ds_write_b128 pair costs a fraction of that.
//  * per k-tile t (k64 = sub-steps s0, s1, 64 MFMAs each on fragment sets R0 / R1):
//      [s0: MFMAs(R0) | ds_read (t,s1) -> R1 | ds_write G (= tile t+1) -> L[(t+1)&1] | global_load t+2 -> G]
//      lgkmcnt(0) + s_barrier   (tile t+1 in LDS; every read of tile t's s1 retired)
//      [s1: MFMAs(R1) | ds_read (t+1,s0) -> R0 from L[(t+1)&1]]
//    G = 16 x 16 B per thread (one k-tile of A and B: 512 rows x 128 B); its loads are issued one k-tile
//    before their ds_write; L = 2 LDS buffers x 64 KiB. (Splitting G into k-halves written in both blocks —
//    to spread the ~830 LDS write cycles — measured slower: 8192^3 1152 vs 1204 TF, FF layer 1 -20 %.)
//  * global loads: 8 consecutive lanes read one row's 128 B (full cache line); the ds_write puts chunk c of
//    row r at slot c ^ ((r >> 1) & 7) — the read_frag swizzle — so both the 8-lane write groups and the
//    fragment reads are bank-conflict free.
//  * MFMA operands swapped (transposed accumulator tiles, TSL store) — in-place asm MFMAs keep the
//    accumulators in AGPRs (see w4).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 1) gemm_nt_256_w4r_kernel(GemmParams p) {
  constexpr int OPB = 256 * 128;             // one operand's 256 rows x 64 bf16
  constexpr int BUFB = 2 * OPB;              // A + B of one k-tile
  __shared__ __attribute__((aligned(16))) char smem[2 * BUFB];

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
  const int nk = max(0, (kend - kbeg + BK - 1) / BK);
  const long long kseg = p.seg_k ? kbeg / p.seg_k : 0;
  const int kb0 = (int)(kseg * p.seg_k);
  const unsigned short* Ab = p.A + batch * p.sA + (long long)m0 * p.lda;
  const unsigned short* Bb = p.B + batch * p.sB + (long long)n0 * p.ldb + kseg * p.seg_stride_b;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, (unsigned)((long long)rows_a * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, (unsigned)((long long)rows_b * p.ldb * 2));

  // load i (0..15) of this thread: rows (i & 7) * 32 + tid / 8 of A (i < 8) or B, 16-B chunk tid % 8
  const int lrow = tid >> 3, lch = tid & 7;
  const unsigned a_off = (unsigned)(lrow * p.lda * 2 + lch * 16), b_off = (unsigned)(lrow * p.ldb * 2 + lch * 16);
  const unsigned a_step = (unsigned)(32 * p.lda * 2), b_step = (unsigned)(32 * p.ldb * 2);
  const int kcl = lch * 8;                   // this lane's k within the k-tile
  // LDS image byte offset of load i: row r = (i & 7) * 32 + lrow, chunk lch -> r*128 + (lch ^ ((r>>1)&7))*16
  const int w_off = lrow * 128 + ((lch ^ ((lrow >> 1) & 7)) * 16);    // (i & 7) * 32 rows add 4096 B, same swizzle

  u32x4 g[16];
  auto gload_one = [&](int u, int i) {
    const int k = kbeg + u * BK;
    const bool kin = k + kcl < kend;
    const bool isa = i < 8;
    const unsigned off = isa ? a_off + (unsigned)k * 2 + (i & 7) * a_step
                             : b_off + (unsigned)(k - kb0) * 2 + (i & 7) * b_step;
    g[i] = __builtin_amdgcn_raw_buffer_load_b128(isa ? ra : rb, kin ? (int)off : OOB, 0, 0);
  };
  auto gwrite_one = [&](int buf, int i) {
    char* base = smem + buf * BUFB + (i < 8 ? 0 : OPB) + (i & 7) * 4096 + w_off;
    *reinterpret_cast<u32x4*>(base) = g[i];
  };

  // fragment reads: row = w*128 + f*16 + (lane&15); (row>>1)&7 = ((lane&15)>>1)
  const int rl = lane & 15, sw = (rl >> 1) & 7;
  const int off_s0 = rl * 128 + (((lane >> 4)) ^ sw) * 16;
  const int off_s1 = rl * 128 + ((4 + (lane >> 4)) ^ sw) * 16;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[8], a1[8], b1[8];

  auto read_set = [&](int buf, int off, bf16x8 (&af)[8], bf16x8 (&bq)[8]) {
    const char* sa = smem + buf * BUFB + wr * 128 * 128 + off;
    const char* sb = smem + buf * BUFB + OPB + wc * 128 * 128 + off;
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = *reinterpret_cast<const bf16x8*>(sa + f * 2048);
      bq[f] = *reinterpret_cast<const bf16x8*>(sb + f * 2048);
    }
  };
  // 64 MFMAs (transposed tiles: B fragment first) with the next sub-step's 16 fragment reads (1 per 2 MFMAs
  // over the first 32) and, in s0 blocks, the 16 ds_writes of the staged tile each followed by its refill load
  auto block = [&](const bf16x8 (&af)[8], const bf16x8 (&bq)[8], int rbuf, int roff, bf16x8 (&an)[8], bf16x8 (&bn)[8],
                   bool stage, int wbuf, int u_load) {
    const char* sa = smem + rbuf * BUFB + wr * 128 * 128 + roff;
    const char* sb = smem + rbuf * BUFB + OPB + wc * 128 * 128 + roff;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(bq[j]), "v"(af[i]));
        if (i < 4 && (j & 1) == 1) {
          const int r = i * 4 + (j >> 1);
          if (r < 8) bn[r] = *reinterpret_cast<const bf16x8*>(sb + r * 2048);
          else an[r - 8] = *reinterpret_cast<const bf16x8*>(sa + (r - 8) * 2048);
        }
        if (stage && (j & 3) == 3) {
          const int q = i * 2 + (j >> 2);        // 0..15: write staged chunk q, then refill it
          gwrite_one(wbuf, q);
          gload_one(u_load, q);
        }
      }
  };

  // prologue: tile 0 -> L[0]; tile 1 in flight in G; tile 0's s0 fragments
#pragma unroll
  for (int i = 0; i < 16; ++i) gload_one(0, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) gwrite_one(0, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) gload_one(1, i);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  read_set(0, off_s0, a0, b0);

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    block(a0, b0, cur, off_s1, a1, b1, true, cur ^ 1, t + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    NSDB_BARRIER();
    block(a1, b1, cur ^ 1, off_s0, a0, b0, false, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __syncthreads();
  store_tile_lds<256, 256, 2, 2, true>(acc, smem, (int)sizeof(smem), p, batch, split, m0, n0, tid, lane, wave);
}


// Split-K slab reducer + fused epilogue (the ClusterAggregate "combine" of the partial block products).
// the K-tail stealing counters of the GEMM this reducer follows go back to zero for the next launch
__device__ __forceinline__ void reset_steal_counters(const GemmParams& p) {
  if (p.steal_cnt != nullptr && blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = threadIdx.x; i < p.tiles_m * p.tiles_n; i += blockDim.x) p.steal_cnt[i] = 0;
}

__global__ void __launch_bounds__(256) splitk_reduce_kernel(GemmParams p) {
  reset_steal_counters(p);
  const long long MN = (long long)p.M * p.N;
  const int batch = blockIdx.y;
  const float* bias = p.bias ? p.bias + batch * p.sBias : nullptr;
  const float keep_scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  if (p.vec_ws) {
    // N % 4 == 0: 4 consecutive columns of one row per thread, 16-B slab loads (splits in flight together)
    for (long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; e < MN;
         e += (long long)gridDim.x * blockDim.x * 4) {
      const float* w = p.ws + (long long)batch * p.splits * MN + e;
      // up to 16 slab loads in flight per thread (uniform predicates, one wait before the adds): the
      // reducer is HBM/MALL-latency bound with 4 outstanding loads
      f32x4 part[16];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < p.splits) part[k] = *reinterpret_cast<const f32x4*>(w + k * MN);
      f32x4 s = part[0];
#pragma unroll
      for (int k = 1; k < 16; ++k)
        if (k < p.splits) s += part[k];
      for (int k = 16; k < p.splits; ++k) s += *reinterpret_cast<const f32x4*>(w + k * MN);
      reduce_epilogue4(p, batch, MN, e, s);
    }
    return;
  }
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < MN;
       e += (long long)gridDim.x * blockDim.x) {
    const float* w = p.ws + (long long)batch * p.splits * MN + e;
    float s = 0.f;
    for (int k = 0; k < p.splits; ++k) s += w[k * MN];
    const int row = (int)(e / p.N), col = (int)(e % p.N);
    float v = s * p.alpha;
    if (bias) v += (p.bias_mode == 1) ? bias[row] : (p.bias_mode == 3) ? bias[e] : bias[col];
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

// Narrow outputs with many splits (M x N small, K huge: dedup / word2vec scoring 500 x 100 x 1e6): the
// plain reducer has too few workgroups and walks every slab serially per thread.  Here 8 groups of 64
// lanes share 64 output vec4s; group g sums slabs g, g+8, ... with 4 loads in flight, then the 8
// partials meet in LDS.  Deterministic (fixed summation tree).
__global__ void __launch_bounds__(512) splitk_reduce_wide_kernel(GemmParams p) {
  reset_steal_counters(p);
  const long long MN = (long long)p.M * p.N;
  const int batch = blockIdx.y;
  const int v = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long e = ((long long)blockIdx.x * 64 + v) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (e < MN) {
    const float* w = p.ws + (long long)batch * p.splits * MN + e;
    for (int k = g; k < p.splits; k += 32) {
      f32x4 a[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (k + 8 * q < p.splits) a[q] = *reinterpret_cast<const f32x4*>(w + (long long)(k + 8 * q) * MN);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (k + 8 * q < p.splits) s += a[q];
    }
  }
  __shared__ f32x4 red[8][64];
  red[g][v] = s;
  __syncthreads();
  if (g == 0 && e < MN) {
    f32x4 t = red[0][v];
#pragma unroll
    for (int q = 1; q < 8; ++q) t += red[q][v];
    reduce_epilogue4(p, batch, MN, e, t);
  }
}

}  // namespace nsdb

// ---------------------------------------------------------------- host side
extern "C" {


static int g_force_cfg = -1;  // -1 auto, 0 = 128x128, 1 = 256x256 2-stage, 2 = 256x256 8-phase (A/B testing)
static int g_diag = 0;        // force_config / 100: kernel timing diagnostics (GemmParams::diag)
static unsigned long long* g_stamps = nullptr;   // cfg 17 progress-stamp buffer ([wg][64] u64)
static int g_adapt = 0;   // adaptive split-K partition: opt-in (measured neutral, profiles/r2_gemm1_study)

void nsdb_study_gemm_set_adapt(int on) { g_adapt = on; }

// K-tail stealing geometry (cfg 24): tail chunks per split and k-tiles per chunk (even)
static int g_steal_tq = 4, g_steal_ch = 16;
static int g_steal_on = 0;   // opt-in: long split-K launches of cfg 2 take the stealing variant (not bit-reproducible)
void nsdb_study_gemm_set_steal(int on) { g_steal_on = on; }
void nsdb_study_gemm_steal(int tq, int ch) {
  g_steal_tq = tq < 1 ? 1 : tq;
  g_steal_ch = ch < 2 ? 2 : (ch & ~1);
}

// Tail trigger: start an independent job in the tail of the next long GEMM instead of after it.
// arm(flag, v): the next 8-phase launch with >= 128 workgroups and >= 64 k-tiles per workgroup makes each
// workgroup raise *flag to v when its main loop ends (the grid is one resident wave, so by then every
// workgroup of it has been dispatched and the CUs that finish first are idle until the launch drains).
// consumed() tells the caller whether a launch took it (only then may a stream wait on the flag: the value is
// written unconditionally by every workgroup of that launch, so the wait always ends).
static struct { unsigned* flag; unsigned value; int consumed; } g_trig = {nullptr, 0u, 0};

void nsdb_study_tail_trigger_arm(void* flag, unsigned value) {
  g_trig.flag = (unsigned*)flag;
  g_trig.value = value;
  g_trig.consumed = 0;
}

int nsdb_study_tail_trigger_consumed() {
  const int c = g_trig.flag != nullptr && g_trig.consumed;
  if (c) g_trig.flag = nullptr;         // one launch per arm
  return c;
}

void nsdb_study_tail_trigger_disarm() { g_trig.flag = nullptr; g_trig.consumed = 0; }

// Make `stream` wait (on the GPU command processor, no host involvement) until *flag >= value.
int nsdb_study_stream_wait_value(hipStream_t stream, void* flag, unsigned value) {
  return (int)hipStreamWaitValue32(stream, flag, value, hipStreamWaitValueGte, 0xffffffffu);
}

static std::map<std::tuple<int, void*, int, int, int, int>, nsdb::AdaptState*>& adapt_states() {
  static std::map<std::tuple<int, void*, int, int, int, int>, nsdb::AdaptState*> states;
  return states;
}

// Inspection: copy the learned shares and rates (splits floats each) of the first state matching
// (M, N, K) into out[0:2*64]; returns the split count, 0 if there is none. Synchronises the device.
int nsdb_study_gemm_adapt_state(int M, int N, int K, float* out) {
  for (auto& kv : adapt_states()) {
    if (std::get<2>(kv.first) == M && std::get<3>(kv.first) == N && std::get<4>(kv.first) == K && kv.second) {
      if (hipDeviceSynchronize() != hipSuccess) return -1;
      if (hipMemcpy(out, kv.second, 2 * 64 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return -1;
      return std::get<5>(kv.first);
    }
  }
  return 0;
}


void nsdb_study_gemm_set_stamps(void* ptr) { g_stamps = (unsigned long long*)ptr; }

// Tile config: the 256x256 tile (1 block/CU) when both dims fill it and there is enough work.
static int pick_cfg(int M, int N, int K, int batch) {
  if (g_force_cfg >= 0) return g_force_cfg;
  const long long big_tiles = (long long)((M + 255) / 256) * ((N + 255) / 256) * batch;
  const bool fills = M >= 192 && N >= 192;
  const long long ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  // 8-phase 256^2 when there is a long mainloop, or when >= 3/4 of the CUs get a tile and K spans at
  // least 16 k-tiles (the FF output layer 1000x14588x1000: 60 us vs 75 us for 128^2, kernel trace)
  return (fills && (big_tiles * ksteps >= 256LL * 32 || (big_tiles >= 192 && ksteps >= 16))) ? 2 : 0;
}

void nsdb_study_gemm_force_config(int cfg) {
  g_force_cfg = cfg < 0 ? cfg : cfg % 100;
  g_diag = cfg < 0 ? 0 : cfg / 100;
}

// Number of split-K slices the launcher will use; the caller sizes the workspace with it.
int nsdb_study_gemm_splits(int M, int N, int K, int batch) {
  const int cfg = pick_cfg(M, N, K, batch);
  const int tbm = cfg ? 256 : nsdb::BM, tbn = cfg ? 256 : nsdb::BN;
  const int tiles = ((M + tbm - 1) / tbm) * ((N + tbn - 1) / tbn) * batch;
  const int ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  // fill the chip: 256 CUs x (2 blocks of 128^2 | 1 block of 256^2); keep >= 8 k-steps per split
  const int target = cfg ? 256 : 512;
  int splits = 1;
  // >= 3/4 of the chip busy: a split's f32 slabs + reduce pass cost more than the idle CUs (1000x14588x1024:
  // 51 us + 24 us reduce with 2 splits vs 60 us unsplit)
  if (tiles < target && !(cfg && tiles >= 192)) {
    // round DOWN: tiles * splits stays within one wave of resident workgroups. Rounding up left a
    // handful of workgroups for a second, nearly empty wave (6000x100x100k: 47 tiles x 11 splits =
    // 517 WGs ran 456 us; x 10 = 470 WGs fit one wave)
    splits = std::max(1, target / tiles);
    splits = std::min(splits, std::max(1, ksteps / 8));
  }
  if (splits > 1) {
    const int kchunk_steps = (ksteps + splits - 1) / splits;
    splits = (ksteps + kchunk_steps - 1) / kchunk_steps;
  }
  return splits;
}


int nsdb_study_gemm_nt_bf16(const void* A, const void* B, void* C, float* ws, const float* bias,
                      int M, int N, int K, long long lda, long long ldb, long long ldc,
                      long long sA, long long sB, long long sC, long long sBias, int batch,
                      int splits, int act, int bias_mode, int out_f32, float alpha, float dropout,
                      unsigned long long seed, int accumulate, long long seg_k, long long seg_stride_b,
                      hipStream_t stream) {
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
  p.diag = g_diag;
  p.seg_k = seg_k;
  p.seg_stride_b = seg_stride_b;
  p.softmax = 0; p.sm_part = nullptr; p.sm_cnt = nullptr; p.sm_flag = nullptr;
  p.stamps = g_stamps;
  p.adapt = nullptr;
  p.signal = nullptr; p.signal_value = 0; p.steal_cnt = nullptr; p.steal_tq = 0; p.steal_ch = 2;
  if (g_force_cfg == 17 && g_stamps == nullptr) return -6;
  if (seg_k > 0 && (seg_k % p.kchunk != 0 || seg_k % nsdb::BK != 0)) return -5;   // a split must not cross a segment
  const int cfg = pick_cfg(M, N, K, batch);
  const int tbm = cfg ? 256 : nsdb::BM, tbn = cfg ? 256 : nsdb::BN;
  p.tiles_m = (M + tbm - 1) / tbm;
  p.tiles_n = (N + tbn - 1) / tbn;
  p.vec_ws = (N % 4 == 0) ? 1 : 0;
  p.vec_c = (ldc % 4 == 0 && sC % 4 == 0 &&
             (reinterpret_cast<uintptr_t>(C) & (out_f32 ? 15 : 7)) == 0) ? 1 : 0;
  dim3 grid(p.tiles_m * p.tiles_n * p.splits, 1, batch);
  // only long split-K GEMMs (>= 8 splits of >= 16 k-tiles: the XCD tail is worth it); the rest keep the
  // static partition, bit-reproducible from run to run (the adaptive one is exact but moves the summation
  // grouping between launches; nsdb_study_gemm_set_adapt(0) restores full reproducibility)
  if (cfg == 2 && g_adapt && p.splits >= 8 && (K / nsdb::BK) / p.splits >= 16 && batch == 1 && seg_k == 0 && p.splits <= nsdb::ADAPT_MAX_SPLITS &&
      (long long)p.tiles_m * p.tiles_n * p.splits <= nsdb::ADAPT_MAX_WG && p.tiles_m * p.tiles_n <= 64) {
    // one persistent state per (shape, splits) — the measured rates belong to that workload
    // (per stream: launches on one stream are ordered, so every workgroup of a launch reads the same shares)
    auto& states = adapt_states();
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(dev, (void*)stream, M, N, K, p.splits);
    auto it = states.find(key);
    nsdb::AdaptState* st = nullptr;
    if (it != states.end()) {
      st = it->second;
    } else if (hipMalloc((void**)&st, sizeof(nsdb::AdaptState)) == hipSuccess) {
      if (hipMemset(st, 0, sizeof(nsdb::AdaptState)) != hipSuccess) st = nullptr;
      states[key] = st;
    }
    p.adapt = st;
  }
  if (cfg == 2 && g_trig.flag != nullptr && !g_trig.consumed && (long long)grid.x * batch >= 128 &&
      (long long)((p.kchunk + nsdb::BK - 1) / nsdb::BK) >= 64) {
    p.signal = g_trig.flag;               // the armed tail trigger goes to this long GEMM
    p.signal_value = g_trig.value;
    g_trig.consumed = 1;
  }
  const bool steal = g_steal_on && cfg == 2 && p.splits > 1 && batch == 1 && seg_k == 0 &&
                     p.tiles_m * p.tiles_n <= 4096 && (K / nsdb::BK) / p.splits >= 4 * g_steal_tq * g_steal_ch;
  if (cfg == 2 && !steal)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<0>, grid, dim3(512), 0, stream, p);
  else if (cfg == 10)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<8>, grid, dim3(512), 0, stream, p);
  else if (cfg == 17)   // 8-phase with progress stamps (diagnostic: workgroup drift within a split)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<12>, grid, dim3(512), 0, stream, p);
  else if (cfg == 15)   // 8-phase, untransposed accumulators + LDS-staged epilogue store (A/B of the direct store)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<11>, grid, dim3(512), 0, stream, p);
  else if (cfg == 14)   // 8-phase with a 10-slot half-tile LDS ring (5 half-tiles in flight)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<10>, grid, dim3(512), 0, stream, p);
  else if (cfg == 12)   // 4-wave 128x128-per-wave kernel (one wave per SIMD)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_w4_kernel<0>, grid, dim3(256), 0, stream, p);
  else if (cfg == 16)   // w4r: 4-wave 128x128-per-wave kernel, register-staged global loads
    hipLaunchKernelGGL(nsdb::gemm_nt_256_w4r_kernel, grid, dim3(256), 0, stream, p);
  else if (cfg == 13)   // w4 diagnostic: no DMA issued (load-free upper bound, wrong results)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_w4_kernel<4>, grid, dim3(256), 0, stream, p);
  else if ((cfg == 24 || (cfg == 2 && g_steal_on && (K / nsdb::BK) / p.splits >= 4 * g_steal_tq * g_steal_ch)) &&
           p.splits > 1 && batch == 1 && seg_k == 0 && p.tiles_m * p.tiles_n <= 4096) {
    // 8-phase with K-tail stealing: per-(device, stream) claim counters, zeroed once here and re-zeroed by the
    // split-K reducer that follows every launch
    static std::map<std::pair<int, void*>, int*> bufs;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int*& cnt = bufs[{dev, (void*)stream}];
    if (cnt == nullptr) {
      if (hipMalloc((void**)&cnt, 4096 * sizeof(int)) != hipSuccess) return -7;
      if (hipMemset(cnt, 0, 4096 * sizeof(int)) != hipSuccess) return -7;
    }
    p.steal_cnt = cnt;
    p.steal_tq = g_steal_tq;
    p.steal_ch = g_steal_ch;
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<19>, grid, dim3(512), 0, stream, p);
  }
  else if (cfg == 26 && p.splits > 1 && batch == 1 && seg_k == 0 && p.vec_ws && p.tiles_m * p.tiles_n <= 4096) {
    // 8-phase with the split-K fix-up by each tile's last-arriving workgroup (no reducer launch below):
    // per-(device, stream) arrival counters, zeroed once here and re-zeroed by the fixing workgroup
    static std::map<std::pair<int, void*>, int*> fix_bufs;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int*& cnt = fix_bufs[{dev, (void*)stream}];
    if (cnt == nullptr) {
      if (hipMalloc((void**)&cnt, 4096 * sizeof(int)) != hipSuccess) return -7;
      if (hipMemset(cnt, 0, 4096 * sizeof(int)) != hipSuccess) return -7;
    }
    p.steal_cnt = cnt;
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<23>, grid, dim3(512), 0, stream, p);
    return (int)hipGetLastError();
  }
  else if (cfg == 25 && p.splits % 2 == 0)   // 8-phase, XCD split pairs interleave their k-tiles
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<22>, grid, dim3(512), 0, stream, p);
  else if (cfg == 20)   // 8-phase with non-temporal operand loads
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<15>, grid, dim3(512), 0, stream, p);
  else if (cfg == 21)   // 8-phase, sc1 (L1 bypass) operand loads
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<16>, grid, dim3(512), 0, stream, p);
  else if (cfg == 22)   // 8-phase, nt sc1 on B
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<17>, grid, dim3(512), 0, stream, p);
  else if (cfg == 23)   // 8-phase, nt sc1 on A
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<18>, grid, dim3(512), 0, stream, p);
  else if (cfg == 18)   // diagnostic: all splits stream one shared K window (MALL-resident operands)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<13>, grid, dim3(512), 0, stream, p);
  else if (cfg == 19)   // diagnostic: every workgroup cycles over 2 k-tiles (L2-resident operands)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<14>, grid, dim3(512), 0, stream, p);
  // (cfg 30-36, the asm-scheduled 4-wave "w4a" kernel, was removed after profiles/r3_w4a: 1139 vs 1379 TF)
  else if (cfg == 11)   // K-tiled operands (caller passes [K/64][ld][64] panels, lda/ldb = padded rows)
    hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<9>, grid, dim3(512), 0, stream, p);
  else if (cfg >= 3 && cfg <= 9) {   // diagnostic variants of the 8-phase kernel (timing only)
    auto kern = cfg == 3 ? nsdb::gemm_nt_256_8ph_kernel<1> : cfg == 4 ? nsdb::gemm_nt_256_8ph_kernel<2>
              : cfg == 5 ? nsdb::gemm_nt_256_8ph_kernel<3> : cfg == 6 ? nsdb::gemm_nt_256_8ph_kernel<4>
              : cfg == 7 ? nsdb::gemm_nt_256_8ph_kernel<5> : cfg == 8 ? nsdb::gemm_nt_256_8ph_kernel<6>
                         : nsdb::gemm_nt_256_8ph_kernel<7>;
    hipLaunchKernelGGL(kern, grid, dim3(512), 0, stream, p);
  }
  else if (cfg == 1)
    hipLaunchKernelGGL((nsdb::gemm_nt_tile_kernel<256, 256, 2, 4>), grid, dim3(512), 0, stream, p);
  else
    hipLaunchKernelGGL((nsdb::gemm_nt_tile_kernel<128, 128, 2, 2>), grid, dim3(256), 0, stream, p);
  if (p.splits > 1) {
    const long long MN = (long long)M * N;
    const long long plain_blocks = ((p.vec_ws ? MN / 4 : MN) + 255) / 256;
    if (p.vec_ws && p.splits >= 8 && plain_blocks * batch < 512) {
      hipLaunchKernelGGL(nsdb::splitk_reduce_wide_kernel, dim3((unsigned)((MN / 4 + 63) / 64), batch), dim3(512), 0,
                         stream, p);
    } else {
      int blocks = (int)std::min<long long>(plain_blocks, 4096);
      hipLaunchKernelGGL(nsdb::splitk_reduce_kernel, dim3(blocks, batch), dim3(256), 0, stream, p);
    }
  }
  return (int)hipGetLastError();
}

}  // extern "C"
