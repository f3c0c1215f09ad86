// Device-resident string columns (objects/strings.py StringColumn): UTF-8 bytes in one HBM buffer +
// int64 offsets[n+1]. The reference keeps pdb::String objects inside pages and runs string predicates
// and hash-map probes on the CPU per object (src/objectModel String.h, tpchBench Q12/Q13/Q14 selections,
// StringIntPair hash maps); here a whole column is one launch:
//
//  * nsdb_str_hash   — 64-bit hash per string (group-by / join keys, IN-lists),
//  * nsdb_str_like   — SQL LIKE with '%' and single-byte '_' (=, prefix, suffix, contains are the
//                      1-segment special cases), pattern in the kernarg segment (scalar loads),
//  * nsdb_str_gather — take(): copy selected strings into a new packed buffer.
//
// One lane per string: TPC-H / Reddit strings are 1-120 bytes, so 64 neighbouring strings of a wave
// are a few contiguous KB that the L1/L2 serve from a handful of lines. Bytes are read as aligned
// dwords from a buffer the host pads by >= 16 bytes, so an 8-byte chunk at any offset is two 64-bit
// halves funnel-shifted together (no byte loads, no unaligned access).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kPatBytes = 224;
constexpr int kPatSegs = 16;
constexpr uint8_t kAnyByte = 0xFF;   // '_' (never a byte of valid UTF-8)

struct LikePattern {               // passed by value: lives in the kernarg segment, read by s_load
  uint8_t bytes[kPatBytes];
  uint8_t seg_start[kPatSegs];
  uint8_t seg_len[kPatSegs];
  int nseg;
  int anchor_start;
  int anchor_end;
  int negate;
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

// 8 bytes starting at byte offset p (little endian), from a dword view of the padded buffer.
__device__ __forceinline__ uint64_t load8(const uint32_t* __restrict__ w, int64_t p) {
  const int64_t q = p >> 2;
  const uint32_t sh = (uint32_t)(p & 3) * 8u;
  const uint64_t a = (uint64_t)w[q] | ((uint64_t)w[q + 1] << 32);
  const uint64_t b = (uint64_t)w[q + 2];
  return sh ? (a >> sh) | (b << (64u - sh)) : a;
}

__device__ __forceinline__ uint32_t byte_at(const uint32_t* __restrict__ w, int64_t p) {
  return (w[p >> 2] >> ((uint32_t)(p & 3) * 8u)) & 0xFFu;
}

__global__ __launch_bounds__(256) void str_hash_kernel(const uint32_t* __restrict__ w,
                                                      const int64_t* __restrict__ st, const int64_t* __restrict__ en,
                                                      int64_t n, uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = st[i], e = en[i];
  const int64_t len = e - s;
  uint64_t h = mix64((uint64_t)len ^ 0x9E3779B97F4A7C15ull);
  for (int64_t p = s; p < e; p += 8) {
    uint64_t c = load8(w, p);
    const int64_t rem = e - p;
    if (rem < 8) c &= (1ull << (8 * rem)) - 1ull;
    h = mix64(h ^ c);
  }
  out[i] = h;
}

__device__ __forceinline__ bool seg_match_at(const uint32_t* __restrict__ w, int64_t p, const LikePattern& pt,
                                             int sg) {
  const int st = pt.seg_start[sg], ln = pt.seg_len[sg];
  for (int k = 0; k < ln; ++k) {
    const uint32_t pc = pt.bytes[st + k];
    if (pc != kAnyByte && byte_at(w, p + k) != pc) return false;
  }
  return true;
}

// 0x80 in every byte of v that is zero (exact: no borrow between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
  return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}

// Leftmost start p in [pos, e - ln] of segment sg, or -1. Segments whose first two bytes are literal scan a dword
// (4 candidate starts) per step: the starts whose first two bytes match are found with two SWAR byte compares over
// the dword and the next one, and only those are verified byte by byte (a contains-search over TPC-H comments was
// ~1 byte load + branch per position).
__device__ __forceinline__ int64_t find_seg(const uint32_t* __restrict__ w, int64_t pos, int64_t e, const LikePattern& pt,
                                            int sg) {
  const int ln = pt.seg_len[sg];
  const int64_t last = e - ln;                      // the last possible start
  if (last < pos) return -1;
  const uint32_t b0 = pt.bytes[pt.seg_start[sg]], b1 = ln >= 2 ? pt.bytes[pt.seg_start[sg] + 1] : kAnyByte;
  if (ln < 2 || b0 == kAnyByte || b1 == kAnyByte) {
    for (int64_t p = pos; p <= last; ++p)
      if (seg_match_at(w, p, pt, sg)) return p;
    return -1;
  }
  const uint32_t B0 = b0 * 0x01010101u, B1 = b1 * 0x01010101u;
  int64_t base = pos & ~(int64_t)3;
  uint32_t x = w[base >> 2];
  while (base <= last) {
    const uint32_t y = w[(base >> 2) + 1];            // padded buffer: one dword past any string is readable
    const uint32_t x1 = (x >> 8) | (y << 24);         // the bytes at base + 1 .. base + 4
    uint32_t cand = zero_bytes(x ^ B0) & zero_bytes(x1 ^ B1);
    while (cand) {
      const int o = (__builtin_ctz(cand) >> 3);
      cand &= cand - 1;
      const int64_t p = base + o;
      if (p < pos || p > last) continue;
      if (ln == 2 || seg_match_at(w, p, pt, sg)) return p;
    }
    base += 4;
    x = y;
  }
  return -1;
}

__global__ __launch_bounds__(256) void str_like_kernel(const uint32_t* __restrict__ w,
                                                      const int64_t* __restrict__ st, const int64_t* __restrict__ en,
                                                      int64_t n, LikePattern pt, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = st[i], e = en[i];
  bool ok = true;
  int64_t pos = s;
  for (int sg = 0; sg < pt.nseg && ok; ++sg) {
    const int ln = pt.seg_len[sg];
    const bool first = sg == 0, last = sg == pt.nseg - 1;
    if (first && pt.anchor_start) {
      ok = (e - pos >= ln) && seg_match_at(w, pos, pt, sg);
      pos += ln;
      if (ok && last && pt.anchor_end) ok = pos == e;
    } else if (last && pt.anchor_end) {
      const int64_t p = e - ln;
      ok = (p >= pos) && seg_match_at(w, p, pt, sg);
      pos = e;
    } else {   // leftmost occurrence at or after pos (greedy is exact for '%'-separated fixed segments)
      const int64_t p = find_seg(w, pos, e, pt, sg);
      ok = p >= 0;
      pos = p + ln;
    }
  }
  if (pt.nseg == 0 && pt.anchor_start && pt.anchor_end) ok = (e == s);   // pattern '' matches only ''
  out[i] = (uint8_t)(ok != (pt.negate != 0));
}

// LIKE with floating segments only ('%a%b%': no anchored end), by occurrence bitmaps instead of a per-row search.
// Pass 1 scans the WHOLE byte buffer once, buffer-parallel: thread t owns bytes [64 t, 64 t + 64) and writes, per
// segment, the 64-bit word whose bit o says "the segment matches at byte 64 t + o" (80-byte register window: 5
// aligned 16-B loads, candidates by the two-byte SWAR test, verified 8 bytes at a time under the '_' mask). Pass 2 is
// per row: the leftmost set bit of segment 0 in [s, e - len0], then of segment 1 after it, ... — a few bitmap words
// per row. Greedy leftmost placement is exact for '%'-separated fixed segments, and a bit only counts when the whole
// occurrence lies inside the row, so matches across row boundaries never leak. Every row is then the same few word
// reads, where the per-row search (str_like_kernel, and the compiled pipelines' matcher) costs a data-dependent
// scan of every string: TPC-H Q13's NOT LIKE '%special%requests%' over 15 M order comments.
constexpr int kOccSegs = 4;

__global__ __launch_bounds__(256) void like_occ_kernel(const uint32_t* __restrict__ w, int64_t nwords, int64_t ndw,
                                                       LikePattern pt, uint64_t* __restrict__ occ) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nwords) return;
  uint32_t win[20];
  const int64_t d0 = t * 16;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int64_t d = d0 + 4 * q;
    if (d + 4 <= ndw) {
      const uint4 v = *reinterpret_cast<const uint4*>(w + d);
      win[4 * q] = v.x;
      win[4 * q + 1] = v.y;
      win[4 * q + 2] = v.z;
      win[4 * q + 3] = v.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) win[4 * q + k] = d + k < ndw ? w[d + k] : 0u;
    }
  }
  for (int sg = 0; sg < pt.nseg; ++sg) {
    const int ss = pt.seg_start[sg], ln = pt.seg_len[sg];
    const uint32_t B0 = pt.bytes[ss] * 0x01010101u, B1 = pt.bytes[ss + 1] * 0x01010101u;
    uint64_t v0 = 0, m0 = 0, v1 = 0, m1 = 0;
    for (int k = 0; k < ln; ++k) {
      const uint64_t c = pt.bytes[ss + k];
      if (c == kAnyByte) continue;
      if (k < 8) {
        v0 |= c << (8 * k);
        m0 |= 0xFFull << (8 * k);
      } else {
        v1 |= c << (8 * (k - 8));
        m1 |= 0xFFull << (8 * (k - 8));
      }
    }
    uint64_t bits = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t x1 = (win[i] >> 8) | (win[i + 1] << 24);
      uint32_t z = zero_bytes(win[i] ^ B0) & zero_bytes(x1 ^ B1);
      while (z) {
        const uint32_t o = (uint32_t)__builtin_ctz(z) >> 3;
        z &= z - 1;
        const uint64_t lo = (uint64_t)win[i] | ((uint64_t)win[i + 1] << 32), hi = win[i + 2];
        const uint64_t a = o ? (lo >> (8 * o)) | (hi << (64 - 8 * o)) : lo;
        bool ok = ((a ^ v0) & m0) == 0;
        if (ok && ln > 8) {
          const uint64_t lo2 = (uint64_t)win[i + 2] | ((uint64_t)win[i + 3] << 32), hi2 = win[i + 4];
          const uint64_t b = o ? (lo2 >> (8 * o)) | (hi2 << (64 - 8 * o)) : lo2;
          ok = ((b ^ v1) & m1) == 0;
        }
        if (ok) bits |= 1ull << (4 * i + o);
      }
    }
    occ[(int64_t)sg * nwords + t] = bits;
  }
}

__global__ __launch_bounds__(256) void like_rows_kernel(const int64_t* __restrict__ st, const int64_t* __restrict__ en,
                                                        int64_t n, const uint64_t* __restrict__ occ, int64_t nwords,
                                                        LikePattern pt, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t e = en[i];
  int64_t pos = st[i];
  bool ok = true;
  for (int sg = 0; sg < pt.nseg && ok; ++sg) {
    const int ln = pt.seg_len[sg];
    const int64_t last = e - ln;
    if (last < pos) {
      ok = false;
      break;
    }
    const uint64_t* ob = occ + (int64_t)sg * nwords;
    int64_t wi = pos >> 6;
    uint64_t b = ob[wi] & (~0ull << (pos & 63));
    int64_t p = -1;
    while (true) {
      if (b) {
        p = wi * 64 + __builtin_ctzll(b);
        break;
      }
      if (++wi * 64 > last) break;
      b = ob[wi];
    }
    ok = p >= 0 && p <= last;
    pos = p + ln;
  }
  out[i] = (uint8_t)(ok != (pt.negate != 0));
}

// out_off[j] = exclusive prefix of the selected lengths (computed on the device by the caller).
__global__ __launch_bounds__(256) void str_gather_kernel(const uint8_t* __restrict__ src,
                                                        const int64_t* __restrict__ st,
                                                        const int64_t* __restrict__ en,
                                                        const int64_t* __restrict__ idx,
                                                        const int64_t* __restrict__ out_off, int64_t m,
                                                        uint8_t* __restrict__ dst) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int64_t r = idx ? idx[j] : j;
  const int64_t s = st[r], len = en[r] - s, d = out_off[j];
  for (int64_t k = 0; k < len; ++k) dst[d + k] = src[s + k];
}

// SUBSTRING: row j's bytes [start, start + len_j) (len_j = out_off[j+1] - out_off[j], computed on the device by the
// caller as clamp(row length - start, 0, length)) copied to out_off[j].
__global__ __launch_bounds__(256) void str_slice_kernel(const uint8_t* __restrict__ src,
                                                       const int64_t* __restrict__ st, int64_t start,
                                                       const int64_t* __restrict__ out_off, int64_t n,
                                                       uint8_t* __restrict__ dst) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t s = st[j] + start, d = out_off[j], len = out_off[j + 1] - d;
  for (int64_t k = 0; k < len; ++k) dst[d + k] = src[s + k];
}

inline int grid_for(int64_t n) { return (int)((n + 255) / 256); }

// Exact short-string code (every row <= L <= 7 bytes, L a bound the caller knows): the row's bytes big-endian in
// the low 8L bits, shifted left by 3, OR its length. Equal codes <=> equal strings, and code order is the bytes'
// lexicographic order, so short string keys (TPC-H flags, modes, priorities) group / sort as plain integers with
// no hash and no byte re-check.
__global__ __launch_bounds__(256) void str_pack_kernel(const uint32_t* __restrict__ w, const int64_t* __restrict__ st,
                                                      const int64_t* __restrict__ en, int64_t n, int L,
                                                      int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = st[i];
  const int64_t len = en[i] - s;
  uint64_t be = 0;
  if (len > 0 && L > 0) {
    uint64_t c = load8(w, s);
    c &= len < 8 ? (1ull << (8 * len)) - 1ull : ~0ull;
    be = __builtin_bswap64(c) >> (8 * (8 - L));   // byte 0 at bits [8(L-1), 8L)
  }
  out[i] = (int64_t)((be << 3) | (uint64_t)len);
}


// Exact equality of row pairs (a[ia[i]] == b[ib[i]]) for value-exact string keys: group-by / join / IN decide by
// 64-bit hash first, then every row is byte-compared with its group's or match's representative
// (reference pdb::String equality, src/objectModel/headers/PDBString.h:46-48).
__global__ __launch_bounds__(256) void str_eq_pairs_kernel(const uint32_t* __restrict__ wa, const int64_t* __restrict__ sta,
                                                           const int64_t* __restrict__ ena, const int64_t* __restrict__ ia,
                                                           const uint32_t* __restrict__ wb, const int64_t* __restrict__ stb,
                                                           const int64_t* __restrict__ enb, const int64_t* __restrict__ ib,
                                                           int64_t m, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int64_t ra = ia ? ia[i] : i, rb = ib ? ib[i] : i;
  const int64_t sa = sta[ra], la = ena[ra] - sa;
  const int64_t sb = stb[rb], lb = enb[rb] - sb;
  bool eq = la == lb;
  for (int64_t p = 0; eq && p < la; p += 8) {
    uint64_t x = load8(wa, sa + p) ^ load8(wb, sb + p);
    const int64_t rem = la - p;
    if (rem < 8) x &= (1ull << (8 * rem)) - 1ull;
    eq = x == 0;
  }
  out[i] = eq ? 1 : 0;
}

}  // namespace

extern "C" {


// Every string entry point takes row bounds as (starts [n], ends [n]): a packed column passes (off, off + 1) of its
// offsets[n+1]; a gathered view (StringColumn.take without a byte copy) passes its own starts / ends.
int nsdb_str_hash(const void* bytes, const int64_t* starts, const int64_t* ends, int64_t n, uint64_t* out,
                  hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_hash_kernel, dim3(grid_for(n)), dim3(256), 0, st, (const uint32_t*)bytes, starts, ends, n,
                     out);
  return (int)hipGetLastError();
}

int nsdb_str_pack(const void* bytes, const int64_t* starts, const int64_t* ends, int64_t n, int L, int64_t* out,
                  hipStream_t st) {
  if (L < 0 || L > 7) return -2;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_pack_kernel, dim3(grid_for(n)), dim3(256), 0, st, (const uint32_t*)bytes, starts, ends, n, L,
                     out);
  return (int)hipGetLastError();
}

int nsdb_str_like(const void* bytes, const int64_t* starts, const int64_t* ends, int64_t n, const uint8_t* pat,
                  int pat_len,
                  const int* seg_start, const int* seg_len, int nseg, int anchor_start, int anchor_end, int negate,
                  uint8_t* out, hipStream_t st) {
  if (pat_len > kPatBytes || nseg > kPatSegs || pat_len < 0 || nseg < 0) return -2;
  LikePattern pt{};
  for (int k = 0; k < pat_len; ++k) pt.bytes[k] = pat[k];
  for (int k = 0; k < nseg; ++k) {
    if (seg_start[k] < 0 || seg_len[k] < 0 || seg_start[k] + seg_len[k] > pat_len) return -3;
    pt.seg_start[k] = (uint8_t)seg_start[k];
    pt.seg_len[k] = (uint8_t)seg_len[k];
  }
  pt.nseg = nseg;
  pt.anchor_start = anchor_start;
  pt.anchor_end = anchor_end;
  pt.negate = negate;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_like_kernel, dim3(grid_for(n)), dim3(256), 0, st, (const uint32_t*)bytes, starts, ends, n, pt,
                     out);
  return (int)hipGetLastError();
}

// The bitmap form of nsdb_str_like: floating segments only (no anchors), 1..kOccSegs segments of 2..16 bytes whose
// first two bytes are literal (else -4: the caller takes nsdb_str_like). occ: nseg * ceil(payload_end / 64) words of
// scratch; nbytes: the readable buffer length (payload + pad).
int nsdb_str_like_occ(const void* bytes, int64_t nbytes, int64_t payload_end, const int64_t* starts, const int64_t* ends,
                      int64_t n, const uint8_t* pat, int pat_len, const int* seg_start, const int* seg_len, int nseg,
                      int negate, uint64_t* occ, uint8_t* out, hipStream_t st) {
  if (pat_len > kPatBytes || nseg < 1 || nseg > kOccSegs || pat_len < 0) return -4;
  LikePattern pt{};
  for (int k = 0; k < pat_len; ++k) pt.bytes[k] = pat[k];
  for (int k = 0; k < nseg; ++k) {
    if (seg_start[k] < 0 || seg_len[k] < 2 || seg_len[k] > 16 || seg_start[k] + seg_len[k] > pat_len) return -4;
    if (pat[seg_start[k]] == kAnyByte || pat[seg_start[k] + 1] == kAnyByte) return -4;
    pt.seg_start[k] = (uint8_t)seg_start[k];
    pt.seg_len[k] = (uint8_t)seg_len[k];
  }
  pt.nseg = nseg;
  pt.negate = negate;
  if (n <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(bytes) & 15) return -4;
  const int64_t nwords = (payload_end + 63) / 64;
  if (nwords > 0)
    hipLaunchKernelGGL(like_occ_kernel, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, st,
                       (const uint32_t*)bytes, nwords, nbytes / 4, pt, occ);
  hipLaunchKernelGGL(like_rows_kernel, dim3(grid_for(n)), dim3(256), 0, st, starts, ends, n, occ, nwords, pt, out);
  return (int)hipGetLastError();
}

int nsdb_str_gather(const void* src, const int64_t* starts, const int64_t* ends, const int64_t* idx,
                    const int64_t* out_off, int64_t m, void* dst, hipStream_t st) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(str_gather_kernel, dim3(grid_for(m)), dim3(256), 0, st, (const uint8_t*)src, starts, ends, idx,
                     out_off, m, (uint8_t*)dst);
  return (int)hipGetLastError();
}

int nsdb_str_slice(const void* src, const int64_t* starts, int64_t start, const int64_t* out_off, int64_t n,
                   void* dst, hipStream_t st) {
  if (n <= 0) return 0;
  if (start < 0) return -2;
  hipLaunchKernelGGL(str_slice_kernel, dim3(grid_for(n)), dim3(256), 0, st, (const uint8_t*)src, starts, start, out_off, n,
                     (uint8_t*)dst);
  return (int)hipGetLastError();
}

int nsdb_str_eq_pairs(const void* a, const int64_t* sta, const int64_t* ena, const int64_t* ia, const void* b,
                      const int64_t* stb, const int64_t* enb, const int64_t* ib, int64_t m, uint8_t* out,
                      hipStream_t st) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(str_eq_pairs_kernel, dim3(grid_for(m)), dim3(256), 0, st, (const uint32_t*)a, sta, ena, ia,
                     (const uint32_t*)b, stb, enb, ib, m, out);
  return (int)hipGetLastError();
}

}  // extern "C"
