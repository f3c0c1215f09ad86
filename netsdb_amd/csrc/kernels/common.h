// Shared CDNA4 (gfx950) helpers for the netsdb_amd HIP kernels.
// Wave = 64 lanes; MFMA operands are bf16x8 fragments, accumulators f32x4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nsdb {

typedef __attribute__((ext_vector_type(8))) short bf16x8;   // 4 VGPRs, one MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;    // 16x16 accumulator (4 regs)
typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));   // 16-B raw buffer load / LDS store
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_EXP = 3, ACT_TANH = 4 };

__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
  return __uint_as_float(((unsigned)h) << 16);
}

// Round-to-nearest-even f32 -> bf16 with NaN kept NaN: a plain conversion to __bf16 compiles to the
// hardware v_cvt_pk_bf16_f32 on gfx950 (MI355X_MICROARCH correctness table) — branch-free, unlike an
// integer-rounding version with a NaN test (a divergent branch per element in unrolled epilogues).
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  const __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

// Two f32 -> one packed bf16x2 dword in ONE v_cvt_pk_bf16_f32 (same RNE / NaN semantics as f32_to_bf16); the
// element-wise form compiled to two converts + shift + or per dword in every epilogue.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}

// Compile-time activation (kernels templated on ACT: no per-element switch in unrolled epilogues).
template <int ACT>
__device__ __forceinline__ float act_t(float v) {
  if constexpr (ACT == ACT_RELU) return v > 0.f ? v : 0.f;
  else if constexpr (ACT == ACT_SIGMOID) return 1.f / (1.f + __expf(-v));
  else if constexpr (ACT == ACT_EXP) return __expf(v);
  else if constexpr (ACT == ACT_TANH) return tanhf(v);
  else return v;
}

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    case ACT_EXP: return __expf(v);
    case ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// Compact activation for unrolled MFMA epilogues: exp / sigmoid / tanh share ONE __expf
// (t = exp(a*v): exp -> t, sigmoid -> 1/(1+t) with a=-1, tanh -> 2/(1+t)-1 with a=-2), so a
// 128-element unrolled epilogue stays small enough to be fully unrolled (no acc spill to scratch).
__device__ __forceinline__ float apply_act_compact(float v, int act) {
  if (act == ACT_NONE) return v;
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  const float a = act == ACT_EXP ? 1.f : (act == ACT_SIGMOID ? -1.f : -2.f);
  const float t = __expf(a * v);
  if (act == ACT_EXP) return t;
  const float s = __frcp_rn(1.f + t);
  return act == ACT_SIGMOID ? s : 2.f * s - 1.f;
}

// Counter-based hash RNG (stateless; identical on every launch for a given seed).
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 T1):
// blocks b and b+8 share an XCD under round-robin dispatch, so give each XCD a
// contiguous run of tile ids -> neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg <= 8) return bid;
  const int xcd = bid & 7, pos = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

__device__ __forceinline__ float wave_reduce_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_reduce_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace nsdb
