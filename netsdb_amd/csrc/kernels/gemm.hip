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
//  * the long-K / large-shape config is the 256x256 8-phase kernel below; the split-K reducers finish split
//    products. Production configs only: study kernels are built separately (csrc/study, _hip_study).
#include "gemm_common.h"

namespace nsdb {


// ---- fused, max-subtracted softmax epilogue of the 256x256 8-wave tile (FFOutputLayer: the reference's
// exp(x + b) / rowsum without its overflow at x > 88; src/FF/headers/FFOutputLayer.h + FFRowAggregate.h).
// The softmax row (AXIS 1) spans tiles_n workgroups, so the tile's logits stay in registers while the
// workgroups of one row-block exchange per-row (max, sum exp) partials through global memory:
//   logits -> per-row tile partial (wave shuffles + LDS across the 4 column waves) -> store partial ->
//   agent-scope release + arrival counter -> bounded poll until every tile of the row-block arrived ->
//   acquire -> combine all partials of the row -> exp(x - M) / S written once (no exp'd f32 round trip
//   through HBM and no separate row-normalise pass).
// Placement-independent (cdna_hip_programming.md §6 G16 release/acquire): correct on any XCD mapping. The
// poll is bounded (~200 us on the 100 MHz real-time clock): if the row-block's workgroups are not
// co-resident (the GPU shared with another job), a timed-out tile writes exp(x - m_tile), flags itself and
// the fix-up kernel rescales it by exp(m_tile - M) / S after the launch — slow but never wrong or hung.
// AXIS 2 is the same over the rows of C (the planner computed C^T).
__device__ __forceinline__ void sm_combine(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

// Cross-half wave reductions on the gfx950 lane-swap VALU ops (v_permlane32_swap / v_permlane16_swap: lanes l and
// l ^ 32 / l ^ 16 exchange in one instruction, no LDS round trip like ds_bpermute)
__device__ __forceinline__ float2 swap_pair32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return make_float2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float2 swap_pair16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return make_float2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor16_32(float x) {          // max over lanes {l, l^16, l^32, l^48}
  float2 a = swap_pair16(x);
  x = fmaxf(a.x, a.y);
  a = swap_pair32(x);
  return fmaxf(a.x, a.y);
}
__device__ __forceinline__ float sum_xor16_32(float x) {
  float2 a = swap_pair16(x);
  x = a.x + a.y;
  a = swap_pair32(x);
  return a.x + a.y;
}

// Partials of one softmax group (row-block for AXIS 1, column-block for AXIS 2): float2 (max, sum exp)
// [group][256 lines][need_pad] with need_pad = need rounded up to even, so the partials of one line are
// contiguous and 16-B aligned: the combine reads a line's partials with 16-B loads, all in flight at once.
__host__ __device__ __forceinline__ int sm_need_pad(int need) { return (need + 1) & ~1; }

// LDS map of the epilogue. Bytes [0, 128 KiB): the tile buffers, which the main loop no longer needs, become the
// landing zone of the group's partials (LDS-DMA, [256 lines][32 16-B slots], slot = pair ^ (line & 31)).
// From SM_ST = 128 KiB, floats:
//   [0, 2048)      per-wave line partials [8 waves][128 | 64][2]
//   [2048, 2560)   this tile's own partial per line [256][2]    (fallback scale)
//   [2560, 3072)   second half of the combine [256][2]
//   [3072, 3584)   final (max, 1/sum) per line [256][2]
//   [3584]         poll verdict
//   [SM_BIAS, +2 KiB)   the tile's column bias [256] and row bias [256], staged at launch (before the main loop's
//                       first barrier), so the epilogue does not wait on global loads
constexpr int SM_ST = 131072;
constexpr int SM_BIAS = SM_ST + 3600 * 4;
constexpr int SM_LDS = SM_BIAS + 2048;                // LDS bytes of a fused-softmax launch

// Final (max M, 1/sum S) per line of a softmax group into fin[256][2]: the group's partials ([256 lines][npad]
// float2, contiguous) come into LDS by LDS-DMA (no VGPRs: the tile's logits hold 128 of them), 64 partials per
// line per chunk, every wave-instruction moving 1 KiB and a whole chunk in flight at once (one round trip for up
// to 64 tiles per group). Device-scope (sc1) loads: never served from a stale line of this XCD's L2, so no
// acquire fence (which would invalidate the L2 under the tiles still in their main loops). Two threads per
// line then reduce from LDS: the max first, then the rescaled sums (independent exps, no serial chain).
// Every thread of the workgroup calls it (barriers inside).
__device__ __forceinline__ void sm_group_stats(const float2* part, int npad, char* smem, float* fin, float* h2,
                                               int tid, int lane, int wave) {
  const int e = tid & 255, half = tid >> 8;
  const int npairs = npad >> 1;
  const __amdgpu_buffer_rsrc_t rp = make_rsrc(part, (unsigned)(256 * npad * 8));
  float m = -INFINITY, s = 0.f;
  for (int c0 = 0; c0 < npairs; c0 += 32) {
#pragma unroll 4
    for (int w = wave; w < 128; w += 8) {              // 256 lines x 32 slots = 128 wave-instructions
      const int piece = w * 64 + lane;
      const int line = piece >> 5, pr = c0 + ((piece & 31) ^ (line & 31));
      const int voff = pr < npairs ? (line * npad + pr * 2) * 8 : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rp, (lds_void*)(smem + w * 1024), 16, voff, 0, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int q0 = half * 16, qe = min(min(32, npairs - c0), q0 + 16);
    const char* row = smem + e * 512;
    float cm = -INFINITY;
    for (int q = q0; q < qe; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(row + ((q ^ (e & 31)) * 16));
      cm = fmaxf(cm, fmaxf(v.x, v.z));
    }
    if (cm != -INFINITY) {
      float cs = 0.f;
      for (int q = q0; q < qe; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(row + ((q ^ (e & 31)) * 16));
        cs += v.y * __expf(v.x - cm) + v.w * __expf(v.z - cm);   // exp(-inf - cm) = 0 for empty partials
      }
      sm_combine(m, s, cm, cs);
    }
    __syncthreads();                                   // the zone is refilled by the next chunk
  }
  if (half == 1) { h2[e * 2] = m; h2[e * 2 + 1] = s; }
  __syncthreads();
  if (half == 0) {
    sm_combine(m, s, h2[e * 2], h2[e * 2 + 1]);
    fin[e * 2] = m;
    fin[e * 2 + 1] = s > 0.f ? 1.f / s : 0.f;
  }
  __syncthreads();
}

template <int AXIS>
__device__ __forceinline__ bool softmax_epilogue_8ph(f32x4 (&acc)[8][4], char* smem, int /*smem_bytes*/, const GemmParams& p,
                                                     int m0, int n0, int tm, int tn, int tid, int lane, int wave) {
  // transposed accumulator layout (TS): acc[i][j][r] = C[wr*128 + i*16 + rl][wc*64 + j*16 + cq + r]
  const int wr = wave >> 2, wc = wave & 3;
  const int rl = lane & 15, cq = (lane >> 4) * 4;
  const float* sbias = reinterpret_cast<const float*>(smem + SM_BIAS);   // [256 column | 256 row] bias of the tile
  // 1. logits in registers (invalid rows / columns -> -inf: they never win a max and exp to 0). Per-row or
  // per-column bias only (host-checked)
  float bcol[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = n0 + wc * 64 + j * 16 + cq + r;
      bcol[j][r] = sbias[wc * 64 + j * 16 + cq + r];     // staged in LDS at launch (0 without a column bias)
      if (col >= p.N) bcol[j][r] = -INFINITY;
    }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + rl;
    float brow = sbias[256 + wr * 128 + i * 16 + rl];
    if (row >= p.M) brow = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = acc[i][j][r] * p.alpha + brow + bcol[j][r];
  }
  // 2. per-wave line max m_w (registers + wave shuffles); acc becomes exp(x - m_w) — the ONLY exp per element:
  // the final value is that times exp(m_w - M) / S, one factor per line and wave; wave sums of the exps, then
  // across the waves of a line in LDS
  float* st = reinterpret_cast<float*>(smem + SM_ST);  // [8 waves][128 | 64][2]
  if constexpr (AXIS == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, acc[i][j][r]);
      m = max_xor16_32(m);
      float sum = 0.f;
      const float ms = m == -INFINITY ? 0.f : m;        // an all-invalid line: exp(-inf) = 0 everywhere
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(acc[i][j][r] - ms);
          acc[i][j][r] = e;
          sum += e;
        }
      sum = sum_xor16_32(sum);
      if (lane < 16) {
        const int idx = ((wr * 4 + wc) * 128 + i * 16 + rl) * 2;
        st[idx] = m;
        st[idx + 1] = sum;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float m = -INFINITY;
#pragma unroll
        for (int i = 0; i < 8; ++i) m = fmaxf(m, acc[i][j][r]);
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        float sum = 0.f;
        const float ms = m == -INFINITY ? 0.f : m;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float e = __expf(acc[i][j][r] - ms);
          acc[i][j][r] = e;
          sum += e;
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
        if (rl == 0) {
          const int idx = ((wc * 2 + wr) * 64 + j * 16 + cq + r) * 2;
          st[idx] = m;
          st[idx + 1] = sum;
        }
      }
  }
  __syncthreads();
  unsigned long long* stamp = p.stamps ? p.stamps + (long long)(tm * p.tiles_n + tn) * 8 : nullptr;
  const int grp = AXIS == 1 ? tm : tn, need = AXIS == 1 ? p.tiles_n : p.tiles_m;
  const int my = AXIS == 1 ? tn : tm;
  const int npad = sm_need_pad(need);
  float2* part = p.sm_part + (long long)grp * 256 * npad;
  float* tstat = st + 2048;                           // [256][2] this tile's own partial (fallback scale)
  if (tid < 256) {
    float m = -INFINITY, s = 0.f;
    if constexpr (AXIS == 1) {
      const int wrr = tid >> 7, rl = tid & 127;
#pragma unroll
      for (int w = 0; w < 4; ++w) sm_combine(m, s, st[((wrr * 4 + w) * 128 + rl) * 2], st[((wrr * 4 + w) * 128 + rl) * 2 + 1]);
    } else {
      const int wcc = tid >> 6, c2 = tid & 63;
#pragma unroll
      for (int w = 0; w < 2; ++w) sm_combine(m, s, st[((wcc * 2 + w) * 64 + c2) * 2], st[((wcc * 2 + w) * 64 + c2) * 2 + 1]);
    }
    // device-scope (sc1) stores: written through this XCD's L2, so no L2 write-back fence is needed before the
    // arrival (a release fence writes back the whole L2 and measured 5-14 us per tile)
    auto put = [&](int idx, float a, float b) {
      const unsigned long long v = ((unsigned long long)__float_as_uint(b) << 32) | __float_as_uint(a);
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(part + idx), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    put(tid * npad + my, m, s);
    if (npad != need && my == 0) put(tid * npad + need, -INFINITY, 0.f);   // the pad slot
    tstat[tid * 2] = m;
    tstat[tid * 2 + 1] = s;
  }
  // 3. publish the partial, arrive, poll (bounded) for the whole group
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* okslot = reinterpret_cast<int*>(st + 3584);
  if (tid == 0) {
    // every wave's partial stores were acknowledged (vmcnt(0) + barrier above) before the arrival
    int c = __hip_atomic_fetch_add(p.sm_cnt + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (stamp) stamp[2] = t0;                          // diagnostic stamps: partial published, arrived
    while (c < need) {
      __builtin_amdgcn_s_sleep(1);
      c = __hip_atomic_load(p.sm_cnt + grp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000ull) break;   // 200 us at 100 MHz
    }
    const bool ok = c >= need && !(p.diag & 4);        // diag 4: take the fallback path (tests)
    if (stamp) stamp[3] = __builtin_amdgcn_s_memrealtime();   // the group complete
    *okslot = ok ? 1 : 0;
  }
  __syncthreads();
  const bool ok = *okslot != 0;
  // 4. final (max, 1/sum) per line of the tile from the group's partials, or this tile's own on the fallback path
  float* fin = st + 3072;                              // [256][2]
  if (ok) {
    sm_group_stats(part, npad, smem, fin, st + 2560, tid, lane, wave);
  } else {
    if (tid < 256) {
      fin[tid * 2] = tstat[tid * 2];
      fin[tid * 2 + 1] = 1.f;
    }
    __syncthreads();
  }
  if (stamp && tid == 0) stamp[4] = __builtin_amdgcn_s_memrealtime();   // group statistics combined
  // 5. final values in place: acc (= exp(x - m_w)) times exp(m_w - M) / S, one factor per line of the wave
  // (the caller's store writes them)
  if constexpr (AXIS == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = wr * 128 + i * 16 + rl;
      const float mw = st[((wr * 4 + wc) * 128 + i * 16 + rl) * 2];
      const float M = fin[e * 2];
      const float f = mw == -INFINITY ? 0.f : __expf(mw - M) * fin[e * 2 + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] *= f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = wc * 64 + j * 16 + cq + r;
        const float mw = st[((wc * 2 + wr) * 64 + j * 16 + cq + r) * 2];
        const float M = fin[e * 2];
        const float f = mw == -INFINITY ? 0.f : __expf(mw - M) * fin[e * 2 + 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j][r] *= f;
      }
  }
  return ok;
}

// Late rescale (the rare fallback path): run by the last tile of a group to depart when some tiles of the group
// timed out. Every partial is published and every timed-out tile's exp(x - m_tile) is written back (they depart
// after their stores and an L2 write-back); each gets the factor exp(m_tile - M) / S per line.
template <int AXIS>
__device__ __forceinline__ void sm_late_rescale(const GemmParams& p, char* smem, int grp, int need, int tid, int lane,
                                             int wave) {
  const int npad = sm_need_pad(need);
  float* st = reinterpret_cast<float*>(smem + SM_ST);
  int* slot = reinterpret_cast<int*>(st + 3592);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const float2* part = p.sm_part + (long long)grp * 256 * npad;
  float* fin = st + 3072;
  sm_group_stats(part, npad, smem, fin, st + 2560, tid, lane, wave);
  float* fac = st + 2048;                             // [256]
  float* C = reinterpret_cast<float*>(p.C);
  for (int t = 0; t < need; ++t) {
    const int ttm = AXIS == 1 ? grp : t, ttn = AXIS == 1 ? t : grp;
    int* fl = p.sm_flag + ttm * p.tiles_n + ttn;
    if (tid == 0) *slot = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const bool flagged = *slot != 0;
    if (flagged && tid < 256) {
      const float mt = part[tid * npad + t].x;
      fac[tid] = (fin[tid * 2 + 1] > 0.f && mt != -INFINITY) ? __expf(mt - fin[tid * 2]) * fin[tid * 2 + 1] : 0.f;
    }
    __syncthreads();
    if (flagged) {
      const int m0 = ttm * 256, n0 = ttn * 256;
      for (int e = tid; e < 256 * 256; e += 512) {
        const int r = e >> 8, c = e & 255;
        const int row = m0 + r, col = n0 + c;
        if (row < p.M && col < p.N) C[(long long)row * p.ldc + col] *= fac[AXIS == 1 ? r : c];
      }
      if (tid == 0) __hip_atomic_store(fl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();                                   // slot / fac reused
  }
}

// Departure of a fused-softmax tile (no fix-up launch). One word per group counts departures (low 16 bits) and
// timed-out tiles (high 16 bits). A tile on the normal path departs as soon as it has the group's statistics
// (before its stores); a timed-out tile departs after its exp(x - m_tile) stores are complete and written back,
// with its flag set. The last tile to depart re-zeroes the group's counters for the next launch (every tile has
// passed its poll by then) and, if some tiles timed out, rescales them (sm_late_rescale). Every thread calls it.
template <int AXIS>
__device__ __forceinline__ void sm_depart(const GemmParams& p, char* smem, bool ok, int tm, int tn, int tid, int lane,
                                          int wave) {
  const int grp = AXIS == 1 ? tm : tn, need = AXIS == 1 ? p.tiles_n : p.tiles_m;
  int* slot = reinterpret_cast<int*>(smem + SM_ST) + 3588;
  if (!ok) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (tid == 0) {
    if (!ok) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // this tile's outputs written back from its L2
      __hip_atomic_store(p.sm_flag + tm * p.tiles_n + tn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int inc = ok ? 1 : 0x10001;
    const int d = __hip_atomic_fetch_add(p.sm_dep + grp, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + inc;
    int verdict = 0;
    if ((d & 0xffff) == need) {
      verdict = (d >> 16) > 0 ? 2 : 1;
      __hip_atomic_store(p.sm_cnt + grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.sm_dep + grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *slot = verdict;
  }
  __syncthreads();
  if (*slot == 2) sm_late_rescale<AXIS>(p, smem, grp, need, tid, lane, wave);
}

// ---- split-K reduction inside the launch (GemmParams::fixup; the layer-1 GEMM's 14.6 us reducer launch + gap).
// Every workgroup of a tile, after its slab is written through (store_direct_8ph) and acknowledged, counts in on the
// tile's arrival word and waits (bounded poll) for the tile's other splits; then split s reduces rows
// [s * R, s * R + R) of the tile (R = 256 / splits, 16 at 16 splits) over all slabs in split order — the separate
// reducer's summation order, so the result is bit-identical — with the reducer's epilogue (bias, activation,
// dropout, bf16 / f32 store). A single workgroup fixing a whole tile reads 4 MiB through one CU (~30 us; the
// rejected cfg-26 last-arriver design, profiles/r2_gemm1_study); split 16 ways it is 256 KiB per CU, a few us after
// the tile's last split lands. The wait relies on the tile's splits being co-resident (the launch is one workgroup
// per CU); if the poll times out (the GPU shared with another job), the workgroup skips its rows, flags itself on
// the departure word, and the tile's last workgroup to leave reduces the whole tile (slow, never wrong or hung).
// Slabs of other splits are read with device-scope loads (never a stale line of this XCD's L2).
__device__ __forceinline__ void fixup_rows_8ph(const GemmParams& p, int m0, int n0, int r0, int r1, int tid, int nthr) {
  const long long MN = (long long)p.M * p.N;
  const int cols = min(256, p.N - n0);
  const int q4 = (cols + 3) >> 2;                  // 4-column groups per row (N % 4 == 0: no partial group)
  const int rows = min(r1, p.M - m0) - r0;
  for (int e4 = tid; e4 < rows * q4; e4 += nthr) {
    const int r = r0 + e4 / q4, c = (e4 % q4) * 4;
    const long long e = (long long)(m0 + r) * p.N + n0 + c;
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(p.ws + e);
    const long long step = MN / 2;                 // one slab in 8-byte words
    unsigned long long lo[32], hi[32];
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k < p.splits) {
        lo[k] = __hip_atomic_load(w + k * step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hi[k] = __hip_atomic_load(w + k * step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    f32x4 s = f32x4{__uint_as_float((unsigned)lo[0]), __uint_as_float((unsigned)(lo[0] >> 32)),
                    __uint_as_float((unsigned)hi[0]), __uint_as_float((unsigned)(hi[0] >> 32))};
#pragma unroll
    for (int k = 1; k < 32; ++k)
      if (k < p.splits)
        s += f32x4{__uint_as_float((unsigned)lo[k]), __uint_as_float((unsigned)(lo[k] >> 32)),
                   __uint_as_float((unsigned)hi[k]), __uint_as_float((unsigned)(hi[k] >> 32))};
    reduce_epilogue4(p, 0, MN, e, s);
  }
}

__device__ __forceinline__ void splitk_fixup_8ph(const GemmParams& p, int* slot, int tile, int split, int m0, int n0,
                                              int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's slab stores acknowledged
  __syncthreads();
  if (tid == 0) {
    int c = __hip_atomic_fetch_add(p.fx_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (c < p.splits) {
      __builtin_amdgcn_s_sleep(2);
      c = __hip_atomic_load(p.fx_cnt + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000ull) break;   // 200 us at 100 MHz
    }
    slot[0] = c >= p.splits ? 1 : 0;
  }
  __syncthreads();
  const bool ok = slot[0] != 0;
  const int R = (256 + p.splits - 1) / p.splits;
  if (ok) fixup_rows_8ph(p, m0, n0, split * R, min(256, split * R + R), tid, 512);
  if (tid == 0) {
    const int inc = ok ? 1 : 0x10001;
    const int d = __hip_atomic_fetch_add(p.fx_dep + tile, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + inc;
    int verdict = 0;
    if ((d & 0xffff) == p.splits) {                // the last to leave: every split has passed its poll
      verdict = (d >> 16) > 0 ? 2 : 1;
      __hip_atomic_store(p.fx_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.fx_dep + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    slot[1] = verdict;
  }
  __syncthreads();
  if (slot[1] == 2) fixup_rows_8ph(p, m0, n0, 0, 256, tid, 512);   // some split timed out: the whole tile here
}

// Direct epilogue of the unsplit 8-phase tile: every lane stores its own accumulators, 4 consecutive columns
// of one row per (i, j) (the transposed TS layout: acc[i][j][r] = C[wr*128 + i*16 + rl][wc*64 + j*16 + cq + r]),
// i.e. one 16-B (f32) / 8-B (bf16) store per lane and a wave instruction of 16 rows x 64 B. No LDS image, no
// barrier, no per-pass wait: the store_tile_lds path spends two LDS passes (4 of the 8 waves' f32 tiles fit
// its 128 KiB) with a barrier and an LDS-read -> store dependency per iteration, and the FF output layer's
// all-at-once tail (228 tiles ending together) paid ~2x the bare store stream for it (scripts/native/
// store_gemm2: 10-12 us for the 58 MB stream either way). Bias (per row / per column) is loaded into
// registers before the first store (a load behind stores waits for them: vmcnt is in order).
// Split-K launches store their raw f32 slab the same way (the reducer applies the epilogue): no LDS image, so no
// compiler-inserted vmcnt drain before each LDS read of the staged store loop (which also made that loop wait for
// its own earlier stores and for anything else in flight, e.g. an operand prefetch).
template <bool WT = false>   // WT: split-K slabs written through to the device-coherent level (in-launch fix-up)
__device__ __forceinline__ void store_direct_8ph(const f32x4 (&acc)[8][4], const GemmParams& p, int batch, int split,
                                                 int m0, int n0, int lane, int wave) {
  const int wr = wave >> 2, wc = wave & 3;
  const int rl = lane & 15, cq = (lane >> 4) * 4;
  if (p.splits > 1) {
    float* ws = p.ws + ((long long)batch * p.splits + split) * (long long)p.M * p.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = m0 + wr * 128 + i * 16 + rl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + j * 16 + cq;
        if (row < p.M && col < p.N) {
          float* d = ws + (long long)row * p.N + col;
          if constexpr (WT) {   // in-launch reduction: written through to the device-coherent level (vec_ws)
            unsigned long long* d2 = reinterpret_cast<unsigned long long*>(d);
            const f32x4 a = acc[i][j];
            __hip_atomic_store(d2, ((unsigned long long)__float_as_uint(a[1]) << 32) | __float_as_uint(a[0]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(d2 + 1, ((unsigned long long)__float_as_uint(a[3]) << 32) | __float_as_uint(a[2]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else if (col + 4 <= p.N) *reinterpret_cast<f32x4*>(d) = acc[i][j];   // N % 4 == 0 (host: vec_ws)
          else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (col + r < p.N) d[r] = acc[i][j][r];
          }
        }
      }
    }
    return;
  }
  const float* bias = p.bias ? p.bias + batch * p.sBias : nullptr;
  const float keep_scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  f32x4 bc[4];
  float br[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int col = n0 + wc * 64 + j * 16 + cq;
    if (bias && p.bias_mode == 2 && col < p.N) {
      const float* bp = bias + col;
      if (col + 3 < p.N && ((reinterpret_cast<uintptr_t>(bp) & 15) == 0)) bc[j] = *reinterpret_cast<const f32x4*>(bp);
      else {
#pragma unroll
        for (int r = 0; r < 4; ++r) bc[j][r] = bp[min(r, p.N - 1 - col)];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + rl;
    br[i] = (bias && p.bias_mode == 1 && row < p.M) ? bias[row] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + rl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * 64 + j * 16 + cq;
      f32x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = apply_act_compact(acc[i][j][r] * p.alpha + br[i] + bc[j][r], p.act);
        if (p.dropout > 0.f) {
          const unsigned long long idx = ((unsigned long long)batch * p.M + row) * p.N + col + r;
          x = hash_uniform(p.seed, idx) < p.dropout ? 0.f : x * keep_scale;
        }
        w[r] = x;
      }
      if (row < p.M && col < p.N) {
        const long long off = batch * p.sC + (long long)row * p.ldc + col;
        const int nv = min(4, p.N - col);
        if (p.out_f32) {
          float* d = reinterpret_cast<float*>(p.C) + off;
          if (nv == 4) *reinterpret_cast<f32x4*>(d) = w;
          else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (r < nv) d[r] = w[r];
          }
        } else {
          unsigned short* d = reinterpret_cast<unsigned short*>(p.C) + off;
          if (nv == 4) *reinterpret_cast<uint2*>(d) = make_uint2(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]));
          else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (r < nv) d[r] = f32_to_bf16(w[r]);
          }
        }
      }
    }
  }
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
  __shared__ __attribute__((aligned(16))) char smem[2 * STG + 1024];   // + the epilogue's bias (store_tile_lds)

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

  store_tile_lds<TBM, TBN, WGM, WGN>(acc, smem, 2 * STG, p, batch, split, m0, n0, tid, lane, wave,
                                     reinterpret_cast<float*>(smem + 2 * STG));
}

#define NSDB_BARRIER()                          \
  do {                                          \
    __builtin_amdgcn_sched_barrier(0);          \
    asm volatile("s_barrier" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0);          \
  } while (0)

// Skinny long-K streaming tile (cfg 3: 256 x 128, cfg 4: 128 x 256): one operand has <= 128 rows and K is long, so
// the big operand streams from HBM exactly once and the GEMM is bound by that stream, not by the MFMAs (the dedup
// scoring GEMMs 500 x 100 x 900k and 12 x 500 x 100 x 100k; DedupModels / FFMatrixBlockScanner-style inference,
// reference src/FF/headers/FFTransposeMult.h:92). The 256x256 8-phase tile pads the 100-row operand to 256 rows,
// i.e. 2.5x the MFMA work, which at ~6 TB/s of operand bytes lands at the power-capped MFMA ceiling; this tile pads
// it to 128.
//  * 8 waves as WGM x WGN, 64 x 64 per wave (4 x 4 MFMA tiles of 16x16x32), plain C layout (store_tile_lds).
//  * An NS-slot LDS ring of whole k-tiles (TBM+TBN rows x 64 bf16, 48 KiB) with NS-1 tiles in flight: 96 KiB at
//    NS = 3, twice the 8-phase kernel's 3 half-tiles, for the HBM latency at one workgroup per CU.
//  * ONE barrier per k-tile: wait for this thread's DMAs of tile t (vmcnt = the DMAs of the NS-2 younger tiles) ->
//    raw s_barrier (every wave's DMAs of t have landed, every wave's reads of t-1's slot are consumed by its MFMAs)
//    -> DMA tile t+NS-1 into t-1's slot -> ds_read + MFMA tile t.
//  * Past the last k-tile the DMAs target k >= kend and the buffer range check zero-fills them, so every iteration
//    issues the same OPS VMEM instructions and the counted wait is a constant.
//  * KI (k-interleaved splits, unsegmented B only): split s takes k-tiles s, s + S, s + 2S, ... instead of one
//    contiguous chunk, so the S workgroups of a tile read S adjacent 128-B pieces of every operand row at about the
//    same time (whole DRAM pages instead of one 128-B piece per page visit).
template <int TBM, int TBN, int WGM, int WGN, int NS, bool KI>
__global__ void __launch_bounds__(64 * WGM * WGN, 2) gemm_nt_stream_kernel(GemmParams p) {
  constexpr int NW = WGM * WGN;
  constexpr int TM = TBM / WGM / 16, TN = TBN / WGN / 16;
  constexpr int A_BYTES = TBM * BK * 2, B_BYTES = TBN * BK * 2, STG = A_BYTES + B_BYTES;
  constexpr int OPS = (TBM + TBN) / (8 * NW);      // 1 KiB wave-instructions per thread per k-tile
  static_assert(TBM % (8 * NW) == 0 && TBN % (8 * NW) == 0 && NS >= 2, "stream tile geometry");
  __shared__ __attribute__((aligned(16))) char smem[NS * STG + 1024];   // + the epilogue's bias (store_tile_lds)

  const int ntiles = p.tiles_m * p.tiles_n;
  const int wg = xcd_remap(blockIdx.x, ntiles * p.splits);
  const int split = wg / ntiles, tile = wg % ntiles;
  int tm, tn;
  grouped_tile(tile, p.tiles_m, p.tiles_n, tm, tn);
  const int batch = blockIdx.z;
  const int m0 = tm * TBM, n0 = tn * TBN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;

  const int rows_a = min(TBM, p.M - m0), rows_b = min(TBN, p.N - n0);
  const unsigned short* Ab = p.A + batch * p.sA + (long long)m0 * p.lda;
  const int ksteps = (p.K + BK - 1) / BK;
  const int kbeg = KI ? split * BK : split * p.kchunk;
  const int kend = KI ? p.K : min(p.K, kbeg + p.kchunk);
  const int kstep = KI ? p.splits * BK : BK;            // k distance between consecutive k-tiles of this split
  const int nk = KI ? max(0, (ksteps - split + p.splits - 1) / p.splits) : max(0, (kend - kbeg + BK - 1) / BK);
  const long long kseg = (!KI && p.seg_k) ? kbeg / p.seg_k : 0;
  const int kb0 = (int)(kseg * p.seg_k);
  const unsigned short* Bb = p.B + batch * p.sB + (long long)n0 * p.ldb + kseg * p.seg_stride_b;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, (unsigned)((long long)rows_a * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, (unsigned)((long long)rows_b * p.ldb * 2));

  auto stage = [&](int slot, int t) {
    char* dst = smem + slot * STG;
    const int k = min(kbeg + t * kstep, kend);          // past the last k-tile: k = kend, zero-filled
    stage_tile<TBM, NW>(ra, dst, p.lda, rows_a, k, kend, wave, lane);
    stage_tile<TBN, NW>(rb, dst + A_BYTES, p.ldb, rows_b, k - kb0, kend - kb0, wave, lane);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NS - 1; ++t) stage(t, t);
  int slot = 0, wslot = NS - 1;
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS * (NS - 2)) : "memory");
    NSDB_BARRIER();
    stage(wslot, t + NS - 1);
    wslot = wslot + 1 == NS ? 0 : wslot + 1;
    const char* la = smem + slot * STG;
    const char* lb = la + A_BYTES;
    slot = slot + 1 == NS ? 0 : slot + 1;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag(la, wm * (TBM / WGM) + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag(lb, wn * (TBN / WGN) + j * 16 + (lane & 15), chunk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing zero-fill DMAs land before LDS reuse
  __syncthreads();
  store_tile_lds<TBM, TBN, WGM, WGN>(acc, smem, NS * STG, p, batch, split, m0, n0, tid, lane, wave,
                                     reinterpret_cast<float*>(smem + NS * STG));
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
//  * The MFMA computes the TRANSPOSED 16x16 tile (B fragment as the A operand): lane l holds
//    C[row = l & 15][4 consecutive columns 4*(l >> 4) ..], spilled to the LDS image with one 16-B write per
//    tile (store_tile_lds TSL) for full-row epilogue stores.
//  * EPI: 0 = the common epilogue (bias / activation / dropout / split-K slabs); 1 / 2 = fused max-subtracted
//    softmax over the columns / rows of C (one instantiation each: both in one kernel pushed the epilogue
//    past 256 VGPRs into scratch).
//  Studies of this loop (diagnostic variants, K-tail stealing, adaptive split-K, in-launch fix-up, ring
//  buffers, cache policies, the 4-wave structures) live in the separate study build (csrc/study).
// ---------------------------------------------------------------------------------------------
template <int EPI>
__global__ void __launch_bounds__(512, 2) gemm_nt_256_8ph_kernel(GemmParams p) {
  // fused-softmax launches may carry diagnostic phase stamps (p.stamps: [tile][8] on the 100 MHz real-time clock)
  constexpr bool SMX = EPI == 1 || EPI == 2;   // the fused-softmax instantiations (EPI 3: split-K, reduced in-launch)
  const unsigned long long t_entry = SMX ? __builtin_amdgcn_s_memrealtime() : 0ull;
  constexpr int HALF = 128 * 128;            // bytes of one half-tile (128 rows x 64 bf16)
  constexpr int BUF = 4 * HALF;              // one K-tile
  // + the epilogue's bias (store_tile_lds) and the operand-prefetch sink (1 KiB per wave), or the fused softmax's
  // line statistics (SM_LDS)
  __shared__ __attribute__((aligned(16))) char smem[SMX ? SM_LDS : 2 * BUF + 1024 + 8 * 1024];

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
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = max(0, (kend - kbeg + BK - 1) / BK);
  const int niter = (nk + 1) >> 1;

  const unsigned short* Ab = p.A + batch * p.sA + (long long)m0 * p.lda;
  const long long kseg = p.seg_k ? kbeg / p.seg_k : 0;
  const int kb0 = (int)(kseg * p.seg_k);      // B's k origin (segmented B)
  const unsigned short* Bb = p.B + batch * p.sB + (long long)n0 * p.ldb + kseg * p.seg_stride_b;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, (unsigned)((long long)rows_a * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, (unsigned)((long long)rows_b * p.ldb * 2));

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
      roff[q][i] = ta < rows_a ? (int)((long long)ta * p.lda * 2) : -1;
      roff[2 + q][i] = tb < rows_b ? (int)((long long)tb * p.ldb * 2) : -1;
    }

  // fused softmax: the tile's per-column (threads 0-255) / per-row (256-511) bias, loaded before the prologue's DMAs
  // and written to LDS after its wait (read by the epilogue, after the main loop's barriers)
  float bias_v = 0.f;
  if constexpr (SMX) {
    const int c = tid & 255;
    const int idx = tid < 256 ? n0 + c : m0 + c;
    const bool use = p.bias && (tid < 256 ? (p.bias_mode == 2 && idx < p.N) : (p.bias_mode == 1 && idx < p.M));
    if (use) bias_v = p.bias[idx];
  }
  auto stage = [&](int buf, int slot, int u) {
    const int k = kbeg + u * BK + kc;
    const bool kin = k < kend;
    char* dst = smem + buf * BUF + slot * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ro = roff[slot][i];
      const int voff = (kin && ro >= 0) ? ro + (slot < 2 ? k : k - kb0) * 2 : OOB;
      if (slot < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(dst + (i * 64 + wave * 8) * 128), 16, voff, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst + (i * 64 + wave * 8) * 128), 16, voff, 0, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], b0[2][2], b1[2][2];

  auto readA = [&](int buf, int q) {
    const char* base = smem + buf * BUF + q * HALF;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kk] = read_frag(base, wr * 64 + mi * 16 + (lane & 15), kk * 4 + (lane >> 4));
  };
  auto readB = [&](int buf, int q, bf16x8 (&bq)[2][2]) {
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
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[qm * 4 + mi][qn * 2 + ni] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ni][kk], af[mi][kk], acc[qm * 4 + mi][qn * 2 + ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    NSDB_BARRIER();
  };
  // one K-tile u held in buffer `cur` (u+1 in cur^1)
  auto ktile = [&](int cur, int u) {
    // j0: quadrant (0,0); reads B0 then A0; stages A1 of u+1
    readB(cur, 0, b0);
    __builtin_amdgcn_sched_barrier(0);
    readA(cur, 0);
    stage(cur ^ 1, 1, u + 1);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");   // the 4 B0 reads (issued first) are done
    mma(0, 0, b0);
    // j1: quadrant (0,1); reads B1; stages B0 of u+2
    readB(cur, 1, b1);
    stage(cur, 2, u + 2);
    mma(0, 1, b1);
    // j2: quadrant (1,1); reads A1; stages A0 of u+2
    readA(cur, 1);
    stage(cur, 0, u + 2);
    mma(1, 1, b1);
    // j3: quadrant (1,0) from registers; stages B1 of u+2; retires tile u+1 (3 half-tiles stay in flight)
    stage(cur, 3, u + 2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    mma(1, 0, b0);
  };

  // prologue: tile 0 (4 halves) + B0, A0, B1 of tile 1; tile 0 complete when <= 6 ops remain
  stage(0, 2, 0); stage(0, 0, 0); stage(0, 3, 0); stage(0, 1, 0);
  stage(1, 2, 1); stage(1, 0, 1); stage(1, 3, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  if constexpr (SMX) reinterpret_cast<float*>(smem + SM_BIAS)[tid] = bias_v;   // [256 col | 256 row]
  NSDB_BARRIER();
  if (wr == 1) NSDB_BARRIER();            // stagger the two wave groups by one barrier
  for (int it = 0; it < niter; ++it) {
    ktile(0, 2 * it);
    ktile(1, 2 * it + 1);
  }
  if (wr == 0) NSDB_BARRIER();            // re-align the groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing zero-fill DMAs land before LDS reuse
  if constexpr (!SMX) {
    // Operand prefetch (per launch, GemmParams::pf_ptr): the next kernel's operand (the FF output weight after
    // layer 1, whose 2.4 GB stream evicts it) is read into the Infinity Cache by this launch's workgroups as each
    // finishes its main loop, spread over the launch's tail. 1/nwg of the bytes per workgroup, LDS-DMA into a
    // 1 KiB sink per wave (no VGPRs; the sink is disjoint from the epilogue's LDS image); the loads stay in
    // flight under the epilogue's stores and retire before the wave ends.
    if (p.pf_ptr != nullptr) {
      const long long nwg = (long long)gridDim.x * gridDim.z;
      const long long wid = (long long)blockIdx.z * gridDim.x + blockIdx.x;
      const long long chunk = ((p.pf_bytes + nwg - 1) / nwg + 1023) & ~1023LL;
      const long long beg = wid * chunk;
      if (beg < p.pf_bytes) {
        const int len = (int)min(chunk, p.pf_bytes - beg);
        const __amdgpu_buffer_rsrc_t rf = make_rsrc(p.pf_ptr + beg, (unsigned)len);
        char* sink = smem + 2 * BUF + 1024 + wave * 1024;
        for (int off = wave * 1024; off < len; off += 8 * 1024)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rf, (lds_void*)sink, 16, off + lane * 16, 0, 0, 0);
      }
    }
  }
  if constexpr (SMX) {
    // the fused softmax turns acc into the final values in place; the common store then runs with a plain
    // (alpha 1, no bias/act/dropout, f32) epilogue
    unsigned long long* stamp = p.stamps ? p.stamps + (long long)(tm * p.tiles_n + tn) * 8 : nullptr;
    if (stamp && tid == 0) {
      stamp[0] = t_entry;
      stamp[1] = __builtin_amdgcn_s_memrealtime();     // main loop done
    }
    const bool ok = softmax_epilogue_8ph<EPI>(acc, smem, (int)sizeof(smem), p, m0, n0, tm, tn, tid, lane, wave);
    if (ok) sm_depart<EPI>(p, smem, true, tm, tn, tid, lane, wave);
    GemmParams q = p;
    q.alpha = 1.f; q.bias = nullptr; q.act = 0; q.dropout = 0.f; q.accumulate = 0; q.out_f32 = 1; q.splits = 1;
    if (p.direct_epi) store_direct_8ph(acc, q, 0, 0, m0, n0, lane, wave);
    else store_tile_lds<256, 256, 2, 4, true>(acc, smem, 2 * BUF, q, 0, 0, m0, n0, tid, lane, wave);
    if (!ok) sm_depart<EPI>(p, smem, false, tm, tn, tid, lane, wave);
    if (stamp) {
      if (tid == 0) stamp[5] = __builtin_amdgcn_s_memrealtime();   // stores issued (wave 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        stamp[6] = __builtin_amdgcn_s_memrealtime();                 // every wave's stores complete
        stamp[7] = ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) |
                   (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 4);   // XCC id, HW_ID (CU / SE)
      }
    }
    return;
  }
  if constexpr (EPI == 3) {
    // split-K reduced inside the launch (host: direct epilogue, batch 1): write-through slabs, then the tile's splits
    // meet; a separate instantiation, so the production EPI 0 kernel's registers are untouched by this code
    store_direct_8ph<true>(acc, p, batch, split, m0, n0, lane, wave);
    splitk_fixup_8ph(p, reinterpret_cast<int*>(smem + 2 * BUF), tm * p.tiles_n + tn, split, m0, n0, tid);
    return;
  }
  if (p.direct_epi) {
    store_direct_8ph(acc, p, batch, split, m0, n0, lane, wave);
  } else {
    store_tile_lds<256, 256, 2, 4, true>(acc, smem, 2 * BUF, p, batch, split, m0, n0, tid, lane, wave,
                                         reinterpret_cast<float*>(smem + 2 * BUF));
  }
  if (p.pf_ptr != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // prefetch DMAs retired
}

// ---------------------------------------------------------------------------------------------
// The same 8-phase loop on v_mfma_f32_32x32x16_bf16 (GemmOpts::mfma = 32; common epilogue only).
// Each MFMA does 2x the MACs of a 16x16x32 for the same 8 operand VGPRs, so the register-file operand reads per
// MAC halve: the lever the power-limited layer-1 GEMM was measured to want (profiles/r2_gemm1_study/
// mfma_power_waves.txt: 32x32x16 1,825-1,831 TF vs 16x16x32 1,672-1,753 TF at 2 waves/SIMD on random operands).
// Unchanged: the half-tile LDS map and its DMA schedule, the ping-pong wave groups, the barrier/vmcnt/lgkmcnt
// protocol (4 B reads, then 8 A reads, per phase — the same counts as the 16x16 loop). Changed:
//  * fragments: lane l reads row l & 31 of a 32-row block, 16-B chunk 2s + (l >> 5) for k-step s (k 16s..16s+15)
//    — the 32x32x16 operand map (A[row r][k = 8h + j]) with the same k permutation on both operands; the XOR
//    swizzle of read_frag keeps these reads conflict-free (per 16-lane group: 16 distinct (row & 1, chunk ^ ...)
//    slots);
//  * per phase 2 (m) x 1 (n) 32x32 tiles x 4 k-steps = 8 MFMAs (the same 256 MFMA cycles as 16 of 16x16x32);
//  * accumulators acc[mb][nb] (f32x16): the transposed product (B fragment as the A operand), so lane l holds
//    C[m = wr*128 + mb*32 + (l & 31)][n = wc*64 + nb*32 + 8g + 4(l >> 5) + r] in register 4g + r: four runs of 4
//    consecutive columns per lane, stored as 16-B (f32) / 8-B (bf16) pieces straight from the registers.
// ---------------------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ void store_direct_8ph32(const f32x16 (&acc)[4][2], const GemmParams& p, int batch, int split,
                                                   int m0, int n0, int lane, int wave) {
  const int wr = wave >> 2, wc = wave & 3;
  const int rl = lane & 31, ch = (lane >> 5) * 4;
  if (p.splits > 1) {
    float* ws = p.ws + ((long long)batch * p.splits + split) * (long long)p.M * p.N;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int row = m0 + wr * 128 + mb * 32 + rl;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = n0 + wc * 64 + nb * 32 + g * 8 + ch;
          if (row < p.M && col < p.N) {
            float* d = ws + (long long)row * p.N + col;
            const f32x4 v = {acc[mb][nb][4 * g], acc[mb][nb][4 * g + 1], acc[mb][nb][4 * g + 2], acc[mb][nb][4 * g + 3]};
            if (col + 4 <= p.N) *reinterpret_cast<f32x4*>(d) = v;          // N % 4 == 0 (host: vec_ws)
            else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (col + r < p.N) d[r] = v[r];
            }
          }
        }
    }
    return;
  }
  const float* bias = p.bias ? p.bias + batch * p.sBias : nullptr;
  const float keep_scale = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  float br[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int row = m0 + wr * 128 + mb * 32 + rl;
    br[mb] = (bias && p.bias_mode == 1 && row < p.M) ? bias[row] : 0.f;
  }
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = n0 + wc * 64 + nb * 32 + g * 8 + ch;
      f32x4 bc = {0.f, 0.f, 0.f, 0.f};
      if (bias && p.bias_mode == 2 && col < p.N) {
        const float* bp = bias + col;
        if (col + 3 < p.N && ((reinterpret_cast<uintptr_t>(bp) & 15) == 0)) bc = *reinterpret_cast<const f32x4*>(bp);
        else {
#pragma unroll
          for (int r = 0; r < 4; ++r) bc[r] = bp[min(r, p.N - 1 - col)];
        }
      }
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int row = m0 + wr * 128 + mb * 32 + rl;
        f32x4 w;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = apply_act_compact(acc[mb][nb][4 * g + r] * p.alpha + br[mb] + bc[r], p.act);
          if (p.dropout > 0.f) {
            const unsigned long long idx = ((unsigned long long)batch * p.M + row) * p.N + col + r;
            x = hash_uniform(p.seed, idx) < p.dropout ? 0.f : x * keep_scale;
          }
          w[r] = x;
        }
        if (row < p.M && col < p.N) {
          const long long off = batch * p.sC + (long long)row * p.ldc + col;
          const int nv = min(4, p.N - col);
          if (p.out_f32) {
            float* d = reinterpret_cast<float*>(p.C) + off;
            if (nv == 4) *reinterpret_cast<f32x4*>(d) = w;
            else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (r < nv) d[r] = w[r];
            }
          } else {
            unsigned short* d = reinterpret_cast<unsigned short*>(p.C) + off;
            if (nv == 4) *reinterpret_cast<uint2*>(d) = make_uint2(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]));
            else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (r < nv) d[r] = f32_to_bf16(w[r]);
            }
          }
        }
      }
    }
}

__global__ void __launch_bounds__(512, 2) gemm_nt_256_8ph32_kernel(GemmParams p) {
  constexpr int HALF = 128 * 128;
  constexpr int BUF = 4 * HALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 1024 + 8 * 1024];

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
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = max(0, (kend - kbeg + BK - 1) / BK);
  const int niter = (nk + 1) >> 1;

  const unsigned short* Ab = p.A + batch * p.sA + (long long)m0 * p.lda;
  const long long kseg = p.seg_k ? kbeg / p.seg_k : 0;
  const int kb0 = (int)(kseg * p.seg_k);
  const unsigned short* Bb = p.B + batch * p.sB + (long long)n0 * p.ldb + kseg * p.seg_stride_b;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, (unsigned)((long long)rows_a * p.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, (unsigned)((long long)rows_b * p.ldb * 2));

  // DMA source rows: identical half-tile map to gemm_nt_256_8ph_kernel
  const int lr = wave * 8 + (lane >> 3);
  const int kc = ((lane & 7) ^ ((lr >> 1) & 7)) * 8;
  int roff[4][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ta = i * 128 + q * 64 + lr;
      const int tb = (2 * i + (lr >> 5)) * 64 + q * 32 + (lr & 31);
      roff[q][i] = ta < rows_a ? (int)((long long)ta * p.lda * 2) : -1;
      roff[2 + q][i] = tb < rows_b ? (int)((long long)tb * p.ldb * 2) : -1;
    }
  auto stage = [&](int buf, int slot, int u) {
    const int k = kbeg + u * BK + kc;
    const bool kin = k < kend;
    char* dst = smem + buf * BUF + slot * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ro = roff[slot][i];
      const int voff = (kin && ro >= 0) ? ro + (slot < 2 ? k : k - kb0) * 2 : OOB;
      if (slot < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(dst + (i * 64 + wave * 8) * 128), 16, voff, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst + (i * 64 + wave * 8) * 128), 16, voff, 0, 0, 0);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  bf16x8 af[2][4], b0[4], b1[4];
  const int frow = lane & 31, fch = lane >> 5;

  auto readA = [&](int buf, int q) {
    const char* base = smem + buf * BUF + q * HALF;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) af[mi][s] = read_frag(base, wr * 64 + mi * 32 + frow, 2 * s + fch);
  };
  auto readB = [&](int buf, int q, bf16x8 (&bq)[4]) {
    const char* base = smem + buf * BUF + (2 + q) * HALF;
#pragma unroll
    for (int s = 0; s < 4; ++s) bq[s] = read_frag(base, wc * 32 + frow, 2 * s + fch);
  };
  auto mma = [&](int qm, int qn, const bf16x8 (&bq)[4]) {
    NSDB_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
        acc[qm * 2 + mi][qn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bq[s], af[mi][s], acc[qm * 2 + mi][qn], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    NSDB_BARRIER();
  };
  auto ktile = [&](int cur, int u) {
    readB(cur, 0, b0);
    __builtin_amdgcn_sched_barrier(0);
    readA(cur, 0);
    stage(cur ^ 1, 1, u + 1);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");   // the 4 B0 reads (issued first) are done
    mma(0, 0, b0);
    readB(cur, 1, b1);
    stage(cur, 2, u + 2);
    mma(0, 1, b1);
    readA(cur, 1);
    stage(cur, 0, u + 2);
    mma(1, 1, b1);
    stage(cur, 3, u + 2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    mma(1, 0, b0);
  };

  stage(0, 2, 0); stage(0, 0, 0); stage(0, 3, 0); stage(0, 1, 0);
  stage(1, 2, 1); stage(1, 0, 1); stage(1, 3, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  NSDB_BARRIER();
  if (wr == 1) NSDB_BARRIER();
  for (int it = 0; it < niter; ++it) {
    ktile(0, 2 * it);
    ktile(1, 2 * it + 1);
  }
  if (wr == 0) NSDB_BARRIER();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (p.pf_ptr != nullptr) {           // operand prefetch of the next kernel (see gemm_nt_256_8ph_kernel)
    const long long nwg = (long long)gridDim.x * gridDim.z;
    const long long wid = (long long)blockIdx.z * gridDim.x + blockIdx.x;
    const long long chunk = ((p.pf_bytes + nwg - 1) / nwg + 1023) & ~1023LL;
    const long long beg = wid * chunk;
    if (beg < p.pf_bytes) {
      const int len = (int)min(chunk, p.pf_bytes - beg);
      const __amdgpu_buffer_rsrc_t rf = make_rsrc(p.pf_ptr + beg, (unsigned)len);
      char* sink = smem + 2 * BUF + 1024 + wave * 1024;
      for (int off = wave * 1024; off < len; off += 8 * 1024)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rf, (lds_void*)sink, 16, off + lane * 16, 0, 0, 0);
    }
  }
  store_direct_8ph32(acc, p, batch, split, m0, n0, lane, wave);
  if (p.pf_ptr != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// Split-K slab reducer + fused epilogue (the ClusterAggregate "combine" of the partial block products).
__global__ void __launch_bounds__(256) splitk_reduce_kernel(GemmParams p) {
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
// Every launch decision is a per-call parameter (GemmOpts): a forced config or an operand prefetch applies to
// exactly the call that passes it — no process-wide state, so lanes on other streams / threads are never
// affected. The product build exports only the production configs; the study variants are in csrc/study.
struct GemmOpts {
  int cfg;                  // -1 auto, 0 = 128x128 tile, 2 = 256x256 8-phase, 3 / 4 = 256x128 / 128x256 stream
  int epi;                  // 8-phase unsplit epilogue: -1 auto (direct), 0 LDS-staged, 1 direct register stores
  const void* pf_ptr;       // operand prefetch of this launch (8-phase only): pf_bytes at pf_ptr, or nullptr
  long long pf_bytes;
  int kinter;               // stream tiles: 1 = k-interleaved splits (split s takes k-tiles s, s + S, ...)
  int mfma;                 // 8-phase main loop: 0 auto, 16 = 16x16x32, 32 = 32x32x16 (direct epilogue launches)
  int fixup;                // 8-phase split-K: 1 = reduce inside the launch (splitk_fixup_8ph), no reducer launch
  int* fx_state;            // its arrival / departure words ([2 * tiles] ints, zero between launches on a stream)
};

extern "C" {

// Tile config: the 256x256 8-phase tile (1 block/CU) when both dims fill it and there is enough work.
static int pick_cfg(int M, int N, int K, int batch) {
  const long long big_tiles = (long long)((M + 255) / 256) * ((N + 255) / 256) * batch;
  const bool fills = M >= 192 && N >= 192;
  const long long ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  // 8-phase 256^2 when there is a long mainloop, or when >= 3/4 of the CUs get a tile and K spans at
  // least 16 k-tiles (the FF output layer 1000x14588x1000: 60 us vs 75 us for 128^2, kernel trace)
  if (fills && (big_tiles * ksteps >= 256LL * 32 || (big_tiles >= 192 && ksteps >= 16))) return 2;
  // skinny, very long K (the dedup scoring GEMMs 500 x 100 x 900k and 12 x 500 x 100 x 100k): memory-bound; the
  // 8-phase kernel keeps three half-tiles of A in flight and zero-fills the missing B rows without reading them
  // (common panel 205 vs 222 us, batched private panels 263 vs 285 us, profiles/r4_dedup)
  // skinny (one side <= 128 rows) with a long K: the 256x128 / 128x256 stream tile (MFMA work padded to 128, not
  // 256 rows; 2 k-tiles in flight per CU): 500x100x900k 208.7 vs 213.9 us, 12x500x100x100k 290.5 vs 292.9,
  // 4096x128x16k 38.4 vs 40.7 (8-phase) / 43.8 (128^2) (profiles/r5_stream)
  if (std::max(M, N) >= 192 && std::min(M, N) <= 128 && ksteps >= 256) return M >= N ? 3 : 4;
  if ((M >= 192 || N >= 192) && std::min(M, N) >= 64 && ksteps >= 1024) return 2;
  return 0;
}

// Macro tile of a config: 0 = 128x128, 2 = 256x256 8-phase, 3 = 256x128 stream, 4 = 128x256 stream.
static void cfg_tile(int cfg, int& tbm, int& tbn) {
  tbm = cfg == 2 || cfg == 3 ? 256 : nsdb::BM;
  tbn = cfg == 2 || cfg == 4 ? 256 : nsdb::BN;
}

static int resolve_cfg(int cfg, int M, int N, int K, int batch) { return cfg < 0 ? pick_cfg(M, N, K, batch) : cfg; }

// Number of split-K slices the launcher will use for config `cfg` (-1 auto); the caller sizes the workspace.
int nsdb_gemm_splits(int M, int N, int K, int batch, int cfg) {
  cfg = resolve_cfg(cfg, M, N, K, batch);
  int tbm, tbn;
  cfg_tile(cfg, tbm, tbn);
  const int tiles = ((M + tbm - 1) / tbm) * ((N + tbn - 1) / tbn) * batch;
  const int ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  // fill the chip: 256 CUs x (2 blocks of 128^2 | 1 block of 256^2); keep >= 8 k-steps per split
  const int target = cfg ? 256 : 512;   // the 256^2 and stream tiles run one block per CU
  int splits = 1;
  // >= 3/4 of the chip busy: a split's f32 slabs + reduce pass cost more than the idle CUs (1000x14588x1024:
  // 51 us + 24 us reduce with 2 splits vs 60 us unsplit)
  if (tiles < target && !(cfg == 2 && tiles >= 192)) {
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

// Workgroups of the launch nsdb_gemm_nt_bf16 makes for this shape (splits <= 0: the launcher's own choice).
int nsdb_gemm_launch_wgs(int M, int N, int K, int batch, int splits, int cfg) {
  cfg = resolve_cfg(cfg, M, N, K, batch);
  int tbm, tbn;
  cfg_tile(cfg, tbm, tbn);
  const int ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  if (splits <= 0) splits = nsdb_gemm_splits(M, N, K, batch, cfg);
  splits = std::max(1, splits);
  const int kchunk_steps = std::max(1, (ksteps + splits - 1) / splits);
  const int s = std::max(1, (ksteps + kchunk_steps - 1) / kchunk_steps);
  return ((M + tbm - 1) / tbm) * ((N + tbn - 1) / tbn) * s * batch;
}

// Would a launch of this shape take an operand prefetch (an 8-phase launch of >= 128 workgroups with >= 64
// k-tiles per workgroup: a long, one-wave-resident GEMM whose finishing workgroups can warm the next operand)?
int nsdb_gemm_prefetch_eligible(int M, int N, int K, int batch, int splits, int cfg) {
  if (resolve_cfg(cfg, M, N, K, batch) != 2) return 0;
  const int ksteps = (K + nsdb::BK - 1) / nsdb::BK;
  if (splits <= 0) splits = nsdb_gemm_splits(M, N, K, batch, cfg);    // the launcher's own choice
  splits = std::max(1, splits);
  const int kchunk_steps = (ksteps + splits - 1) / splits;
  const long long wgs = (long long)((M + 255) / 256) * ((N + 255) / 256) * ((ksteps + kchunk_steps - 1) / kchunk_steps) * batch;
  return wgs >= 128 && kchunk_steps >= 64 ? 1 : 0;
}

// C (f32) = softmax(alpha * A . B^T + bias) along axis 1 (each row of C) or 2 (each column of C), fused into
// the 8-phase GEMM's epilogue (one launch + the fix-up). part: f32x2 [tiles][256]; cnt: int [max(tiles_m,
// tiles_n)] and flag: int [tiles], both zero on entry (the fix-up leaves them zero). force_fallback (tests):
// every tile takes the non-co-resident fallback path.
int nsdb_gemm_nt_softmax(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, long long lda,
                         long long ldb, long long ldc, int bias_mode, float alpha, int axis, void* part, int* cnt,
                         int* flag, int* dep, int force_fallback, int epi, unsigned long long* stamps,
                         hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || (axis != 1 && axis != 2)) return -1;
  if (256LL * lda * 2 >= 0x7ffffff0LL || 256LL * ldb * 2 >= 0x7ffffff0LL) return -2;
  nsdb::GemmParams p;
  p.A = (const unsigned short*)A; p.B = (const unsigned short*)B; p.C = C; p.ws = nullptr; p.bias = bias;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.sA = p.sB = p.sC = p.sBias = 0;
  p.M = M; p.N = N; p.K = K;
  p.kchunk = std::max(1, (K + nsdb::BK - 1) / nsdb::BK) * nsdb::BK;
  p.splits = 1;
  p.act = 0; p.bias_mode = bias ? bias_mode : 0; p.out_f32 = 1; p.accumulate = 0;
  p.alpha = alpha; p.dropout = 0.f; p.seed = 0; p.diag = force_fallback ? 4 : 0;
  p.seg_k = 0; p.seg_stride_b = 0;
  p.tiles_m = (M + 255) / 256;
  p.tiles_n = (N + 255) / 256;
  p.vec_ws = 0;
  p.vec_c = (ldc % 4 == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0) ? 1 : 0;
  p.softmax = axis; p.sm_part = (float2*)part; p.sm_cnt = cnt; p.sm_flag = flag; p.sm_dep = dep; p.stamps = stamps;
  p.adapt = nullptr;
  p.signal = nullptr; p.signal_value = 0; p.steal_cnt = nullptr; p.steal_tq = 0; p.steal_ch = 2;
  p.direct_epi = p.vec_c && epi != 0 ? 1 : 0;      // final values straight from registers (store_direct_8ph)
  const int tiles = p.tiles_m * p.tiles_n;
  if (axis == 1) hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<1>, dim3(tiles), dim3(512), 0, stream, p);
  else hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<2>, dim3(tiles), dim3(512), 0, stream, p);
  return (int)hipGetLastError();
}

int nsdb_gemm_nt_bf16(const void* A, const void* B, void* C, float* ws, const float* bias,
                      int M, int N, int K, long long lda, long long ldb, long long ldc,
                      long long sA, long long sB, long long sC, long long sBias, int batch,
                      int splits, int act, int bias_mode, int out_f32, float alpha, float dropout,
                      unsigned long long seed, int accumulate, long long seg_k, long long seg_stride_b,
                      const GemmOpts* opts, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (K % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0) return -1;        // 16-B rows for the LDS-DMA
  if (256LL * lda * 2 >= 0x7ffffff0LL || 256LL * ldb * 2 >= 0x7ffffff0LL)
    return -2;                                                         // per-tile buffer range
  if (splits > 1 && ws == nullptr) return -3;
  if (accumulate && !out_f32) return -4;                                // C += A.B^T only into f32
  const int cfg = resolve_cfg(opts ? opts->cfg : -1, M, N, K, batch);
  if (cfg < 0 || cfg > 4 || cfg == 1) return -8;                      // not a production config
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
  p.diag = 0;
  p.seg_k = seg_k;
  p.seg_stride_b = seg_stride_b;
  p.softmax = 0; p.sm_part = nullptr; p.sm_cnt = nullptr; p.sm_flag = nullptr;
  p.stamps = nullptr; p.adapt = nullptr;
  p.signal = nullptr; p.signal_value = 0; p.steal_cnt = nullptr; p.steal_tq = 0; p.steal_ch = 2;
  if (seg_k > 0 && (seg_k % p.kchunk != 0 || seg_k % nsdb::BK != 0)) return -5;   // a split must not cross a segment
  int tbm, tbn;
  cfg_tile(cfg, tbm, tbn);
  p.tiles_m = (M + tbm - 1) / tbm;
  p.tiles_n = (N + tbn - 1) / tbn;
  p.vec_ws = (N % 4 == 0) ? 1 : 0;
  p.vec_c = (ldc % 4 == 0 && sC % 4 == 0 &&
             (reinterpret_cast<uintptr_t>(C) & (out_f32 ? 15 : 7)) == 0) ? 1 : 0;
  // the direct register epilogue for unsplit 8-phase launches with aligned C rows and for split-K slabs (opts->epi:
  // -1 auto = direct, 0 = LDS-staged, 1 = direct); C += A.B^T and per-element bias keep the LDS-staged epilogue
  const int epi_pref = opts ? opts->epi : -1;
  // split-K slabs (N % 4 == 0) take the direct stores too
  p.direct_epi = (cfg == 2 && epi_pref != 0 &&
                  ((p.splits == 1 && !accumulate && p.vec_c && p.bias_mode != 3) || (p.splits > 1 && p.vec_ws))) ? 1 : 0;
  dim3 grid(p.tiles_m * p.tiles_n * p.splits, 1, batch);
  if (cfg == 2) {
    if (opts && opts->pf_ptr && opts->pf_bytes > 0) {   // this launch's operand prefetch
      p.pf_ptr = (const char*)opts->pf_ptr;
      p.pf_bytes = opts->pf_bytes;
    }
    // the 32x32x16 main loop stores from registers only (store_direct_8ph32): launches that need the LDS-staged
    // epilogue (C += A.B^T, a per-element bias, unaligned C) stay on the 16x16x32 loop
    const int mf = opts ? opts->mfma : 0;
    // only where the separate reducer would be the plain one (same summation order: bit-identical results); narrow
    // outputs with many splits keep splitk_reduce_wide_kernel
    const long long fx_blocks = ((long long)M * N / 4 + 255) / 256;
    if (opts && opts->fixup && opts->fx_state && p.splits > 1 && p.splits <= 32 && p.direct_epi && p.vec_ws &&
        batch == 1 && !(mf == 32) && !(p.splits >= 8 && fx_blocks < 512)) {
      p.fixup = 1;
      p.fx_cnt = opts->fx_state;
      p.fx_dep = opts->fx_state + p.tiles_m * p.tiles_n;
    }
    if (p.fixup)
      hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<3>, grid, dim3(512), 0, stream, p);
    else if (mf == 32 && p.direct_epi)
      hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph32_kernel, grid, dim3(512), 0, stream, p);
    else
      hipLaunchKernelGGL(nsdb::gemm_nt_256_8ph_kernel<0>, grid, dim3(512), 0, stream, p);
  } else if (cfg == 3 || cfg == 4) {
    // contiguous K chunks per split; k-interleaved splits on request (GemmOpts::kinter, unsegmented B only: a split
    // must stay inside one segment). A/B in profiles/r5_stream: interleaving wins 3 % at M = 1000, N <= 128 and
    // loses 4-5 % on the batched dedup panels, so it is not the default.
    const bool ki = seg_k == 0 && p.splits > 1 && opts && opts->kinter;
    if (cfg == 3) {
      if (ki) hipLaunchKernelGGL((nsdb::gemm_nt_stream_kernel<256, 128, 4, 2, 3, true>), grid, dim3(512), 0, stream, p);
      else hipLaunchKernelGGL((nsdb::gemm_nt_stream_kernel<256, 128, 4, 2, 3, false>), grid, dim3(512), 0, stream, p);
    } else {
      if (ki) hipLaunchKernelGGL((nsdb::gemm_nt_stream_kernel<128, 256, 2, 4, 3, true>), grid, dim3(512), 0, stream, p);
      else hipLaunchKernelGGL((nsdb::gemm_nt_stream_kernel<128, 256, 2, 4, 3, false>), grid, dim3(512), 0, stream, p);
    }
  } else {
    hipLaunchKernelGGL((nsdb::gemm_nt_tile_kernel<128, 128, 2, 2>), grid, dim3(256), 0, stream, p);
  }
  if (p.splits > 1 && !p.fixup) {
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
