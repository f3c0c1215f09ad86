// Memory-bound row/elementwise kernels (vectorised, one workgroup per row or grid-stride):
//  * row softmax          — netsDB FFRowAggregate (row sum of exp) + FFOutputLayer (divide), fused
//                           (reference: src/FF/headers/FFRowAggregate.h, FFOutputLayer.h)
//  * bias + activation    — FFReluBiasSum / FFTransposeBiasSum / FFTransposeBiasSumSigmoid as a
//                           standalone epilogue for tensors not produced by the GEMM kernel
//  * LSTM cell            — src/LSTM (LSTMThreeWaySum -> LSTMHiddenState gate math), fused
//  * embedding bag        — src/word2vec EmbeddingLookupSparse / EmbeddingSegment (gather + segment sum)
#include "common.h"
#include <algorithm>

namespace nsdb {

template <typename T> __device__ __forceinline__ float ld(const T* p, long long i);
template <> __device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <> __device__ __forceinline__ float ld<unsigned short>(const unsigned short* p, long long i) {
  return bf16_to_f32(p[i]);
}
__device__ __forceinline__ void st(float* p, long long i, float v) { p[i] = v; }
__device__ __forceinline__ void st(unsigned short* p, long long i, float v) { p[i] = f32_to_bf16(v); }

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_reduce_max(v) : wave_reduce_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < nw; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

// softmax over rows of X[R][N] (+ optional per-column bias), online max/sum in one read pass.
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) softmax_rows_kernel(const TI* X, const float* bias, TO* Y, int R, int N,
                                                           long long ldx, long long ldy, int log_out) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  if (row >= R) return;
  const TI* x = X + (long long)row * ldx;
  float m = -INFINITY, s = 0.f;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    const float v = ld(x, j) + (bias ? bias[j] : 0.f);
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
  }
  const float gm = block_reduce(m, red, true);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  const float gs = block_reduce(s, red, false);
  const float inv = 1.f / gs, lgs = logf(gs);
  TO* y = Y + (long long)row * ldy;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    const float v = ld(x, j) + (bias ? bias[j] : 0.f);
    st(y, j, log_out ? (v - gm - lgs) : __expf(v - gm) * inv);
  }
}

// y = x / rowsum(x): FFOutputLayer applied to exp'd scores (FFTransposeBiasSum wrote exp(z)).
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) row_normalize_kernel(const TI* X, TO* Y, int R, int N, long long ldx,
                                                            long long ldy) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  if (row >= R) return;
  const TI* x = X + (long long)row * ldx;
  float s = 0.f;
  for (int j = threadIdx.x; j < N; j += blockDim.x) s += ld(x, j);
  const float inv = 1.f / block_reduce(s, red, false);
  TO* y = Y + (long long)row * ldy;
  for (int j = threadIdx.x; j < N; j += blockDim.x) st(y, j, ld(x, j) * inv);
}

// Register-resident variant for f32 rows with 16-B aligned rows (the [batch, labels] exp'd scores of
// the FF output layer, 58 KB/row): 512 threads each hold NV float4 of the row, so the row is read
// from HBM once (the two-pass kernel above re-reads it) — 1 read + 1 write per element.
template <typename TO, int NV>
__global__ void __launch_bounds__(512) row_normalize_vec_kernel(const float* X, TO* Y, int R, int N, long long ldx,
                                                                long long ldy, int plain_loads) {
  // plain_loads: cache-allocating instead of non-temporal row loads (the rows were usually just written by the
  // producing GEMM and may still sit in the Infinity Cache; per-call option plain_loads)
  __shared__ float red[8];
  const int row = blockIdx.x;
  if (row >= R) return;
  const int n4 = N >> 2;
  const f32x4* x = reinterpret_cast<const f32x4*>(X + (long long)row * ldx);
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = threadIdx.x + i * 512;
    v[i] = j < n4 ? (plain_loads ? x[j] : __builtin_nontemporal_load(x + j)) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  }
  const float inv = 1.f / block_reduce(s, red, false);
  TO* y = Y + (long long)row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = threadIdx.x + i * 512;
    if (j >= n4) break;
    const f32x4 o = v[i] * inv;
    if constexpr (sizeof(TO) == 4) {
      __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(y) + j);
    } else {
      uint2 pk{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
      reinterpret_cast<uint2*>(y)[j] = pk;
    }
  }
}

// y = dropout(act(x + bias[row|col])) elementwise over [R][N]
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) bias_act_kernel(const TI* X, const float* bias, TO* Y, int R, int N,
                                                       int bias_mode, int act, float dropout,
                                                       unsigned long long seed) {
  const long long total = (long long)R * N;
  const float keep_scale = dropout > 0.f ? 1.f / (1.f - dropout) : 1.f;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    float v = ld(X, e);
    if (bias) v += bias_mode == 1 ? bias[e / N] : bias[e % N];
    v = apply_act(v, act);
    if (dropout > 0.f) v = hash_uniform(seed, e) < dropout ? 0.f : v * keep_scale;
    st(Y, e, v);
  }
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// gates[B][4H] laid out (i, f, g, o); c_prev f32 [B][H]; outputs h (bf16|f32) and c (f32)
template <typename TG, typename TH>
__global__ void __launch_bounds__(256) lstm_cell_kernel(const TG* gates, const float* c_prev, TH* h_out,
                                                        float* c_out, int B, int H) {
  const long long total = (long long)B * H;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long b = e / H, j = e % H;
    const TG* g = gates + b * 4 * H;
    const float ig = sigm(ld(g, j)), fg = sigm(ld(g, H + j)), gg = tanhf(ld(g, 2 * H + j)),
                og = sigm(ld(g, 3 * H + j));
    const float c = fg * (c_prev ? c_prev[e] : 0.f) + ig * gg;
    c_out[e] = c;
    st(h_out, e, og * tanhf(c));
  }
}

// LSTM cell elementwise steps over [n] f32 (row-major matrices of equal shape):
//   mode 0 (LSTMTwoSum):      out = a * b + c * d      (f * c_prev + i * g)
//   mode 1 (LSTMHiddenState): out = a * tanh(b)         (o * tanh(c))
// 16-B loads/stores (4 floats per thread), scalar tail
__global__ void __launch_bounds__(256) lstm_ew_kernel(int mode, const float* a, const float* b, const float* c,
                                                      const float* d, float* out, long long n) {
  const long long n4 = n / 4;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += (long long)gridDim.x * blockDim.x) {
    const f32x4 x = reinterpret_cast<const f32x4*>(a)[e], y = reinterpret_cast<const f32x4*>(b)[e];
    f32x4 r;
    if (mode == 0) {
      const f32x4 z = reinterpret_cast<const f32x4*>(c)[e], w = reinterpret_cast<const f32x4*>(d)[e];
      r = x * y + z * w;
    } else {
      r = f32x4{x[0] * tanhf(y[0]), x[1] * tanhf(y[1]), x[2] * tanhf(y[2]), x[3] * tanhf(y[3])};
    }
    reinterpret_cast<f32x4*>(out)[e] = r;
  }
  for (long long e = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    out[e] = mode == 0 ? a[e] * b[e] + c[e] * d[e] : a[e] * tanhf(b[e]);
}

// out[b][:] = reduce_{i in [offsets[b], offsets[b+1])} w_i * table[idx[i]][:]   (mode 0 sum, 1 mean)
template <typename TT>
__global__ void __launch_bounds__(256) embedding_bag_kernel(const TT* table, const long long* idx,
                                                            const long long* offsets, const float* weights,
                                                            float* out, int Bn, int D, int mode) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (wave >= Bn) return;
  const long long s = offsets[wave], e = offsets[wave + 1];
  for (int d0 = 0; d0 < D; d0 += 64 * 4) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    for (long long i = s; i < e; ++i) {
      const long long r = idx[i];
      const float w = weights ? weights[i] : 1.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = d0 + q * 64 + lane;
        if (d < D) a[q] += w * ld(table, r * D + d);
      }
    }
    const float sc = (mode == 1 && e > s) ? 1.f / (float)(e - s) : 1.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = d0 + q * 64 + lane;
      if (d < D) out[(long long)wave * D + d] = a[q] * sc;
    }
  }
}

}  // namespace nsdb

static int grid_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 8192); }

namespace nsdb {

// Cache warm-up read: every 128-B line of [base, base + bytes) is loaded once (16 B per lane, a 2 KiB stride
// per wave instruction keeps each load on its own line group) so a consumer launched later finds it in the
// Infinity Cache (MALL) instead of HBM. The loaded words are folded into one value that is stored to a scratch
// word only when it equals a host-chosen key (keeps the loads live; the store almost never happens and only
// touches the scratch word). Few workgroups: it runs in CUs another kernel's tail leaves idle.
__global__ void __launch_bounds__(256) prefetch_kernel(const char* base, long long bytes, unsigned* sink,
                                                       unsigned key) {
  const long long lines = bytes >> 7;
  unsigned acc = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long l = (long long)blockIdx.x * blockDim.x + threadIdx.x; l < lines; l += stride) {
    const uint4 v = *reinterpret_cast<const uint4*>(base + (l << 7));
    acc ^= v.x ^ v.w;
  }
  if (acc == key) sink[0] = acc;
}
}  // namespace nsdb

extern "C" {

// plain_loads (per call): row_normalize_vec_kernel's row load policy (0 = non-temporal, the default; 1 = plain)
int nsdb_softmax_rows(const void* X, int x_f32, const float* bias, void* Y, int y_f32, int R, int N,
                      long long ldx, long long ldy, int log_out, int plain_loads, hipStream_t st) {
  if (R <= 0) return 0;
  if (log_out == 2) {   // row normalise
    const bool vec = x_f32 && (N % 4 == 0) && (ldx % 4 == 0) && (ldy % 4 == 0) &&
                     ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Y)) & 15) == 0;
    if (vec && N <= 512 * 4 * 8) {
#define NSDB_RNV(TO, NV) \
  hipLaunchKernelGGL((nsdb::row_normalize_vec_kernel<TO, NV>), dim3(R), dim3(512), 0, st, (const float*)X, (TO*)Y, R, N, ldx, ldy, plain_loads)
      const int nv = (N / 4 + 511) / 512;
      if (y_f32) { if (nv <= 2) NSDB_RNV(float, 2); else if (nv <= 4) NSDB_RNV(float, 4); else NSDB_RNV(float, 8); }
      else { if (nv <= 2) NSDB_RNV(unsigned short, 2); else if (nv <= 4) NSDB_RNV(unsigned short, 4); else NSDB_RNV(unsigned short, 8); }
#undef NSDB_RNV
      return (int)hipGetLastError();
    }
#define NSDB_RN(TI, TO) \
  hipLaunchKernelGGL((nsdb::row_normalize_kernel<TI, TO>), dim3(R), dim3(256), 0, st, (const TI*)X, (TO*)Y, R, N, ldx, ldy)
    if (x_f32 && y_f32) NSDB_RN(float, float);
    else if (x_f32) NSDB_RN(float, unsigned short);
    else if (y_f32) NSDB_RN(unsigned short, float);
    else NSDB_RN(unsigned short, unsigned short);
#undef NSDB_RN
    return (int)hipGetLastError();
  }
#define NSDB_SM(TI, TO) \
  hipLaunchKernelGGL((nsdb::softmax_rows_kernel<TI, TO>), dim3(R), dim3(256), 0, st, (const TI*)X, bias, (TO*)Y, R, N, ldx, ldy, log_out)
  if (x_f32 && y_f32) NSDB_SM(float, float);
  else if (x_f32) NSDB_SM(float, unsigned short);
  else if (y_f32) NSDB_SM(unsigned short, float);
  else NSDB_SM(unsigned short, unsigned short);
#undef NSDB_SM
  return (int)hipGetLastError();
}

int nsdb_bias_act(const void* X, int x_f32, const float* bias, void* Y, int y_f32, int R, int N, int bias_mode,
                  int act, float dropout, unsigned long long seed, hipStream_t st) {
  const long long n = (long long)R * N;
  if (n <= 0) return 0;
#define NSDB_BA(TI, TO) \
  hipLaunchKernelGGL((nsdb::bias_act_kernel<TI, TO>), dim3(grid_for(n)), dim3(256), 0, st, (const TI*)X, bias, (TO*)Y, R, N, bias_mode, act, dropout, seed)
  if (x_f32 && y_f32) NSDB_BA(float, float);
  else if (x_f32) NSDB_BA(float, unsigned short);
  else if (y_f32) NSDB_BA(unsigned short, float);
  else NSDB_BA(unsigned short, unsigned short);
#undef NSDB_BA
  return (int)hipGetLastError();
}

int nsdb_lstm_ew(int mode, const float* a, const float* b, const float* c, const float* d, float* out, long long n,
                 hipStream_t st) {
  const long long n4 = (n + 3) / 4;
  const int grid = (int)std::min<long long>((n4 + 255) / 256, 4096);
  hipLaunchKernelGGL(nsdb::lstm_ew_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, st, mode, a, b, c, d, out, n);
  return (int)hipGetLastError();
}

int nsdb_lstm_cell(const void* gates, int g_f32, const float* c_prev, void* h_out, int h_f32, float* c_out, int B,
                   int H, hipStream_t st) {
  const long long n = (long long)B * H;
  if (n <= 0) return 0;
#define NSDB_LC(TG, TH) \
  hipLaunchKernelGGL((nsdb::lstm_cell_kernel<TG, TH>), dim3(grid_for(n)), dim3(256), 0, st, (const TG*)gates, c_prev, (TH*)h_out, c_out, B, H)
  if (g_f32 && h_f32) NSDB_LC(float, float);
  else if (g_f32) NSDB_LC(float, unsigned short);
  else if (h_f32) NSDB_LC(unsigned short, float);
  else NSDB_LC(unsigned short, unsigned short);
#undef NSDB_LC
  return (int)hipGetLastError();
}

int nsdb_embedding_bag(const void* table, int t_f32, const long long* idx, const long long* offsets,
                       const float* weights, float* out, int Bn, int D, int mode, hipStream_t st) {
  if (Bn <= 0) return 0;
  const int blocks = (Bn * 64 + 255) / 256;
  if (t_f32)
    hipLaunchKernelGGL((nsdb::embedding_bag_kernel<float>), dim3(blocks), dim3(256), 0, st, (const float*)table,
                       idx, offsets, weights, out, Bn, D, mode);
  else
    hipLaunchKernelGGL((nsdb::embedding_bag_kernel<unsigned short>), dim3(blocks), dim3(256), 0, st,
                       (const unsigned short*)table, idx, offsets, weights, out, Bn, D, mode);
  return (int)hipGetLastError();
}

// Warm the caches with a read of [ptr, ptr + bytes) (prefetch_kernel) on `stream`; blocks <= 0: 64.
int nsdb_prefetch(const void* ptr, long long bytes, unsigned* sink, int blocks, hipStream_t stream) {
  if (bytes <= 0) return 0;
  hipLaunchKernelGGL(nsdb::prefetch_kernel, dim3(blocks > 0 ? blocks : 64), dim3(256), 0, stream,
                     reinterpret_cast<const char*>(ptr), bytes, sink, 0x9e3779b9u);
  return (int)hipGetLastError();
}

}  // extern "C"
