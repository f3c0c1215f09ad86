// Shared definitions of the fused relational pipeline (pipeline.hip) and the bodies of its run-time compiled kernels.
//
// This header is compiled twice: into the ahead-of-time kernels (pipeline.hip, hipcc) and, as the only include of
// every run-time generated kernel source (execution/pipeline.py jit_source), by hiprtc inside the process. It
// therefore includes nothing and uses only HIP device built-ins.
//
// Run-time compiled kernels (jit_agg_body / jit_mask_body): the host turns a stage's register program into a
// program policy P whose loads, instructions, keep flag, key and values are straight-line C++ on compile-time
// register and column indices (immediates stay kernel arguments, so one compiled kernel serves every literal of a
// query shape). The interpreter's per-instruction dispatch (a scalar load, a branch and an indirect register access
// per instruction and row block: 32-45 us per instruction per 60 M rows, profiles/r5_tpch/pipe_micro_modes.log)
// disappears, and the compiler schedules every row load of an iteration ahead of its first use.
#pragma once

namespace nsdb_pipe {

constexpr int NREG = 16, MAXINS = 48, MAXCOL = 10, MAXSTR = 4, FMAX = 8, KSLOT = 4, CAP = 256, NTHR = 256;
constexpr int GCAP = 2048;             // global table slots (power of two)
constexpr int NREG_SMALL = 8;          // the 8-register x 4-row shape
constexpr long long EMPTY = (long long)0x8000000000000000ULL;
constexpr int IMM_REG = -2;            // operand register meaning "the instruction's immediate"
// tile-mode instruction flags (Ins.pad; the operand fields are then byte offsets of T-row register vectors)
constexpr int TF_AIMM = 1, TF_ANONE = 2, TF_BIMM = 4, TF_BNONE = 8, TF_C = 16;

enum Op : int {
  OP_NOP = 0, OP_CONST, OP_ADDF, OP_SUBF, OP_MULF, OP_DIVF, OP_ADDI, OP_SUBI, OP_MULI, OP_I2F,
  OP_LTF, OP_LEF, OP_GTF, OP_GEF, OP_EQF, OP_NEF, OP_LTI, OP_LEI, OP_GTI, OP_GEI, OP_EQI, OP_NEI,
  OP_AND, OP_OR, OP_NOT, OP_PACK, OP_SEQ, OP_SPRE, OP_SSUF, OP_SEL, OP_NEGF, OP_RNGF, OP_RNGI, OP_SLIKE
};
constexpr int KPOOL = 16;              // second immediates: range upper bounds
enum ColKind : int { C_F64 = 0, C_I64, C_I32, C_F32, C_U8, C_SCODE, C_SREF };

struct Ins {
  int op, dst, a, b;
  int c;                         // c >= 0: compares AND their result with register c
  int pad;                       // bits 0-7: tile-mode operand flags (TF_*); bits 8+: aux (range: kpool index | mode << 8)
  long long imm;
};
struct Col {
  const void* p;                 // numeric column
  const long long* st;           // string column: row starts / ends into dat
  const long long* en;
  const unsigned char* dat;
  int kind, late, L;
  int raw_off, aux_off;          // tile kernels: LDS byte offsets of the column's DMA image (string starts / ends)
  int contig;                    // strings: en == st + 1 (one offsets array): the tile DMAs the starts only
};
struct PipeArgs {
  Ins ins[MAXINS + 1];           // + a NOP sentinel (the dispatch prefetches one instruction ahead)
  Col col[MAXCOL];
  const unsigned char* lit;      // literal pool of the string ops
  long long n;
  int nins_a, nins, ncol, keep_reg, key_reg, nval, agg_op, nreg;
  int val_reg[FMAX];
  long long kpool[KPOOL];        // range ops' upper bounds
  int tile, lds_bytes;           // tile / hybrid kernels: rows per tile, dynamic LDS bytes
  int kmode, pad2;               // 0 register kernels, 1 LDS-tile kernels, 2 hybrid (LDS-DMA columns, VGPR registers)
  unsigned long long* table;     // [2 + GCAP + GCAP * FMAX]: status (overflow, kept rows), keys, values (f64 bits)
  // fused join probe (compiled kernels only, jit_join_agg_body): the build side's table of 16-byte slots
  // {join hash, extra rows | payload << 32} (relops.hip join_build: cap + 1 slots, slot cap = the kEmpty key's),
  // its CSR runs of repeated keys, cap - 1, and the build rows (columns with late == 2 are build-side columns)
  const unsigned long long* jtab;
  const long long* jperm;
  unsigned long long jmask;
  long long bn;
  // the table's probe filter (relops.hip join_bloom_kernel; null: none): one word per 2^jbshift home slots
  const unsigned long long* jbloom;
  long long jbshift;
};

typedef unsigned long long u64;
// The register file of one row slot: NR 64-bit registers as ONE vector value (NR VGPR pairs).
template <int NR>
struct RF {
  typedef unsigned long long vec __attribute__((ext_vector_type(NR)));
};

__device__ __forceinline__ double u2f(u64 x) { return __longlong_as_double((long long)x); }
__device__ __forceinline__ u64 f2u(double x) { return (u64)__double_as_longlong(x); }

// Short-string code exactly as StringColumn.short_codes / str_pack (bytes big-endian in the low 8L bits, << 3 | len)
__device__ __forceinline__ u64 short_code(const unsigned char* d, long long s, long long len, int L) {
  if (len > L) return (u64)-1;
  u64 c = 0;
  for (int b = 0; b < L; ++b) c |= (b < len ? (u64)d[s + b] : 0ull) << (8 * (L - 1 - b));
  return (c << 3) | (u64)len;
}

__device__ __forceinline__ bool str_match(const unsigned char* d, u64 ref, const unsigned char* lit, long long imm,
                                          int mode) {
  const long long s = (long long)(ref >> 24);
  const int len = (int)(ref & 0xFFFFFF);
  const unsigned char* l = lit + (imm >> 16);
  const int ll = (int)(imm & 0xFFFF);
  if (mode == 0 ? len != ll : len < ll) return false;
  const long long o = mode == 2 ? s + len - ll : s;     // suffix: compare the last ll bytes
  for (int b = 0; b < ll; ++b)
    if (d[o + b] != l[b]) return false;
  return true;
}

// General LIKE (OP_SLIKE: '%x%', '%a%b%', 'a%b', '_'): the literal is [flags: 1 anchored start, 2 anchored end]
// [nseg][len_0 .. len_{nseg-1}][segment bytes], '_' = 0xFF (never a byte of UTF-8). The string buffer is read as
// aligned dwords (StringColumn pads it by >= 16 bytes and keeps it a 4-byte multiple, as strings.hip str_like does);
// a floating segment is searched 4 candidate starts per dword (SWAR compare of its first two bytes), and only those
// candidates are verified byte by byte. Greedy leftmost matching is exact for '%'-separated fixed segments.
__device__ __forceinline__ unsigned lk_byte(const unsigned* w, long long p) {
  return (w[p >> 2] >> ((unsigned)(p & 3) * 8u)) & 0xFFu;
}
__device__ __forceinline__ bool lk_seg_at(const unsigned* w, long long p, const unsigned char* sb, int ln) {
  for (int k = 0; k < ln; ++k) {
    const unsigned c = sb[k];
    if (c != 0xFFu && lk_byte(w, p + k) != c) return false;
  }
  return true;
}
__device__ __forceinline__ unsigned lk_zero_bytes(unsigned v) {   // 0x80 in every zero byte of v (exact)
  return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}
__device__ __forceinline__ long long lk_find(const unsigned* w, long long pos, long long e, const unsigned char* sb,
                                             int ln) {
  const long long last = e - ln;
  if (last < pos) return -1;
  const unsigned b0 = sb[0], b1 = ln >= 2 ? sb[1] : 0xFFu;
  if (ln < 2 || b0 == 0xFFu || b1 == 0xFFu) {
    for (long long p = pos; p <= last; ++p)
      if (lk_seg_at(w, p, sb, ln)) return p;
    return -1;
  }
  const unsigned B0 = b0 * 0x01010101u, B1 = b1 * 0x01010101u;
  long long base = pos & ~3ll;
  unsigned x = w[base >> 2];
  while (base <= last) {
    const unsigned y = w[(base >> 2) + 1];
    const unsigned x1 = (x >> 8) | (y << 24);           // the bytes at base + 1 .. base + 4
    unsigned cand = lk_zero_bytes(x ^ B0) & lk_zero_bytes(x1 ^ B1);
    while (cand) {
      const long long p = base + (__builtin_ctz(cand) >> 3);
      cand &= cand - 1;
      if (p < pos || p > last) continue;
      if (ln == 2 || lk_seg_at(w, p, sb, ln)) return p;
    }
    base += 4;
    x = y;
  }
  return -1;
}
// The register-window form of str_like: the string's bytes come in as LKW16 16-byte loads from a 16-B aligned start
// (all issued before any use: one memory latency per string instead of one per dword of a data-dependent scan loop),
// then every segment is searched in registers — per dword, the SWAR test of the segment's first two bytes over its 4
// candidate starts, and a candidate verified by comparing the (up to 16) bytes at that start, funnel-shifted out of
// the window, against the segment under its '_' mask. All window indices are compile-time constants (no scratch).
constexpr int LKW16 = 7;                  // 112-byte window
constexpr int LKWD = LKW16 * 4;           // its dwords
__device__ __forceinline__ u64 lk_bytes8(const unsigned (&w)[LKWD], int i, int o) {   // bytes 4i + o .. 4i + o + 7
  const u64 lo = (u64)w[i] | ((u64)w[i + 1] << 32);
  const u64 hi = (u64)w[i + 2];
  return o ? (lo >> (8 * o)) | (hi << (64 - 8 * o)) : lo;
}
// pattern bytes [k, k + 8) of a segment (0xFF = any byte) as value / mask words
__device__ __forceinline__ void lk_pat8(const unsigned char* sb, int ln, int k, u64& v, u64& m) {
  v = 0;
  m = 0;
  for (int j = 0; j < 8 && k + j < ln; ++j) {
    const u64 c = sb[k + j];
    if (c != 0xFFu) {
      v |= c << (8 * j);
      m |= 0xFFull << (8 * j);
    }
  }
}
__device__ __forceinline__ bool lk_match_at(const unsigned (&w)[LKWD], int i, int o, int ln, u64 v0, u64 m0, u64 v1,
                                            u64 m1) {
  if (((lk_bytes8(w, i, o) ^ v0) & m0) != 0) return false;
  return ln <= 8 || ((lk_bytes8(w, i + 2, o) ^ v1) & m1) == 0;
}
// leftmost start in [pos, last] of a segment (ln <= 16) inside the window, or -1
__device__ __forceinline__ int lk_find_w(const unsigned (&w)[LKWD], int pos, int last, const unsigned char* sb, int ln) {
  if (last < pos) return -1;
  u64 v0, m0, v1 = 0, m1 = 0;
  lk_pat8(sb, ln, 0, v0, m0);
  if (ln > 8) lk_pat8(sb, ln, 8, v1, m1);
  const unsigned b0 = sb[0], b1 = ln >= 2 ? sb[1] : 0xFFu;
  const bool swar = ln >= 2 && b0 != 0xFFu && b1 != 0xFFu;
  const unsigned B0 = b0 * 0x01010101u, B1 = b1 * 0x01010101u;
  int found = -1;
#pragma unroll
  for (int i = 0; i < LKWD - 4; ++i) {
    if (found < 0 && 4 * i + 3 >= pos && 4 * i <= last) {
      unsigned cand = 0xFu;
      if (swar) {
        const unsigned x1 = (w[i] >> 8) | (w[i + 1] << 24);
        const unsigned z = lk_zero_bytes(w[i] ^ B0) & lk_zero_bytes(x1 ^ B1);   // 0x80 per candidate byte
        cand = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
      }
      while (cand) {
        const int o = __builtin_ctz(cand);
        cand &= cand - 1;
        const int p = 4 * i + o;
        if (p < pos || p > last) continue;
        if (lk_match_at(w, i, o, ln, v0, m0, v1, m1)) {
          found = p;
          break;
        }
      }
    }
  }
  return found;
}

// WIN false: the memory scan only (the run-time kernels choose per program: pipeline.py JIT_LIKE_WINDOW)
template <bool WIN = true>
__device__ __forceinline__ bool str_like(const unsigned char* d, u64 ref, const unsigned char* lit, long long imm) {
  const long long s = (long long)(ref >> 24), e = s + (long long)(ref & 0xFFFFFF);
  const unsigned char* l = lit + (imm >> 16);
  const int flags = l[0], nseg = l[1];
  const unsigned* w = reinterpret_cast<const unsigned*>(d);
  if constexpr (WIN) {
    // the register window: the string inside 112 bytes from a 16-B aligned start with >= 16 zero bytes after it (the
    // funnel shifts' look-ahead: a candidate start p <= e - ln never compares a byte past e), every segment at most
    // 16 bytes. Only the 16-B chunks holding the string are loaded: the last ends before e + 16, inside the buffer
    // (StringColumn pads it by 16 bytes).
    const long long a0 = s & ~15ll;
    bool short_segs = true;
    for (int sg = 0; sg < nseg; ++sg) short_segs &= l[2 + sg] <= 16;
    if (short_segs && e - a0 + 16 <= 4 * LKWD) {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      unsigned win[LKWD];
      const u32x4* src = reinterpret_cast<const u32x4*>(d + a0);
      const int nload = (int)((e - a0 + 15) >> 4);
#pragma unroll
      for (int q = 0; q < LKW16; ++q) {
        const u32x4 v = q < nload ? src[q] : u32x4{0u, 0u, 0u, 0u};
        win[4 * q] = v.x;
        win[4 * q + 1] = v.y;
        win[4 * q + 2] = v.z;
        win[4 * q + 3] = v.w;
      }
      const int ws = (int)(s - a0), we = (int)(e - a0);
      if (nseg == 0) return (flags & 3) == 3 ? we == ws : true;
      const unsigned char* sb = l + 2 + nseg;
      int pos = ws;
      for (int sg = 0; sg < nseg; ++sg) {
        const int ln = l[2 + sg];
        const bool last = sg == nseg - 1;
        int p;
        if (sg == 0 && (flags & 1)) {                  // anchored start: only at pos
          p = lk_find_w(win, pos, pos, sb, ln);
          if (p < 0 || we - pos < ln) return false;
          pos += ln;
          if (last && (flags & 2) && pos != we) return false;
        } else if (last && (flags & 2)) {              // anchored end: only at we - ln
          p = we - ln >= pos ? lk_find_w(win, we - ln, we - ln, sb, ln) : -1;
          if (p < 0) return false;
          pos = we;
        } else {
          p = lk_find_w(win, pos, we - ln, sb, ln);
          if (p < 0) return false;
          pos = p + ln;
        }
        sb += ln;
      }
      return true;
    }
  }
  const unsigned char* sb = l + 2 + nseg;
  if (nseg == 0) return (flags & 3) == 3 ? e == s : true;
  long long pos = s;
  for (int sg = 0; sg < nseg; ++sg) {
    const int ln = l[2 + sg];
    const bool last = sg == nseg - 1;
    if (sg == 0 && (flags & 1)) {
      if (e - pos < ln || !lk_seg_at(w, pos, sb, ln)) return false;
      pos += ln;
      if (last && (flags & 2) && pos != e) return false;
    } else if (last && (flags & 2)) {
      const long long p = e - ln;
      if (p < pos || !lk_seg_at(w, p, sb, ln)) return false;
      pos = e;
    } else {
      const long long p = lk_find(w, pos, e, sb, ln);
      if (p < 0) return false;
      pos = p + ln;
    }
    sb += ln;
  }
  return true;
}

__device__ __forceinline__ unsigned slot_hash(long long k) {
  u64 z = (u64)k * 0x9E3779B97F4A7C15ull;
  return (unsigned)(z >> 40);
}

__device__ __forceinline__ double acc_op(double a, double b, int op) {
  return op == 0 ? a + b : (op == 1 ? fmin(a, b) : fmax(a, b));
}

// *p = op(*p, v) atomically (LDS or global: the pointer's address space is known after inlining). Sums use the
// hardware f64 add atomic, min / max a 64-bit CAS loop.
__device__ __forceinline__ void atomic_acc(double* p, double v, int op) {
  if (op == 0) {
    atomicAdd(p, v);
    return;
  }
  u64* q = reinterpret_cast<u64*>(p);
  u64 old = *q;
  while (true) {
    const double cur = u2f(old);
    const double nv = acc_op(cur, v, op);
    if (nv == cur) return;
    const u64 got = atomicCAS(q, old, f2u(nv));
    if (got == old) return;
    old = got;
  }
}

// Linear-probing insert of (key, values) into a table of cap slots (LDS or global). False: no free or matching slot
// within maxp probes (the table counts as full: the stage then runs in the emitted form). The global table takes a
// window of GWIN probes: near its capacity every insert of every workgroup would walk hundreds of slots with global
// atomics (Q17's ~2,000 part groups in the 2,048-slot table measured 2 ms instead of ~0.3).
constexpr unsigned GWIN = 64;
template <int F, int STRIDE = FMAX>
__device__ __forceinline__ bool table_insert(long long* tk, double* tv, unsigned cap, long long key, const double (&v)[F],
                                             int nval, int op, unsigned maxp = 0xffffffffu) {
  unsigned h = slot_hash(key) & (cap - 1);
  const unsigned lim = cap < maxp ? cap : maxp;
  for (unsigned p = 0; p < lim; ++p) {
    const long long prev = (long long)atomicCAS(reinterpret_cast<u64*>(tk + h), (u64)EMPTY, (u64)key);
    if (prev == EMPTY || prev == key) {
#pragma unroll
      for (int f = 0; f < F; ++f)
        if (f < nval) atomic_acc(tv + (size_t)h * STRIDE + f, v[f], op);
      return true;
    }
    h = (h + 1) & (cap - 1);
  }
  return false;
}

__device__ __forceinline__ double wave_reduce(double v, int op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = acc_op(v, __shfl_xor(v, o), op);
  return v;
}


// Overflow of a fused aggregation (more groups than the tables hold): the launch's result is discarded and the host
// re-runs the batch in the emitted form, so the scan stops as soon as any workgroup has overflowed — its own flag
// every iteration (LDS), the launch's status word every 64 (a full LDS table otherwise costs every later row a probe
// of all CAP slots: a 60 M-row scan that overflowed early measured 67-77 ms instead of ~0.5).
__device__ __forceinline__ bool agg_overflowed(const PipeArgs& a, int* s_ovf, int it) {
  if (__hip_atomic_load(s_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return true;
  // the launch word (a device-scope load of one address by every thread) only every 64 iterations: a long scan
  // with few groups never pays it more than a handful of times
  return (it & 63) == 63 && (__hip_atomic_load(a.table, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1ull);
}
__device__ __forceinline__ void agg_mark_overflow(const PipeArgs& a, int* s_ovf) {
  __hip_atomic_store(s_ovf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_or(a.table, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- run-time compiled (JIT) kernel bodies
// P (generated): F, NR, ROWS; load<LATE, FULL>(a, row, m, R) (the columns of one pass into their registers, 0 where m
// is false; FULL: every row of the block is in range and unmasked, so the loads carry no per-row exec mask); run_a / run_b (the predicate / key-and-value segments); keep(r), key(r), vals(r, v). Registers are a
// plain u64 [ROWS][NR] array indexed by constants only, so every register lives in VGPRs.
//
// The aggregation is the register kernels' (pipe_agg_kernel): KSLOT register slots per thread, the workgroup's LDS
// table, one merge into the global table; status[0] = overflow, status[1] = kept rows.
template <typename P>
__device__ __forceinline__ void jit_agg_body(const PipeArgs& a) {
  constexpr int F = P::F, NR = P::NR, ROWS = P::ROWS;
  __shared__ long long tk[CAP];
  __shared__ double tv[CAP * FMAX];
  __shared__ int s_ovf;
  __shared__ unsigned long long s_kept;
  const int tid = threadIdx.x, lane = tid & 63;
  // the aggregation op as a compile-time constant when the generated program fixes it (P::OP >= 0): a run-time op made
  // every accumulate compute the sum, the min and the max and select (1,303 v_max / v_min_f64 in TPC-H Q01's kernel)
  const int op = P::OP >= 0 ? P::OP : a.agg_op;
  const double init = op == 0 ? 0.0 : (op == 1 ? __builtin_inf() : -__builtin_inf());
  for (int i = tid; i < CAP; i += NTHR) tk[i] = EMPTY;
  for (int i = tid; i < CAP * FMAX; i += NTHR) tv[i] = init;
  if (tid == 0) {
    s_ovf = 0;
    s_kept = 0;
  }
  __syncthreads();

  u64 R[ROWS][NR];
#pragma unroll
  for (int j = 0; j < ROWS; ++j)
#pragma unroll
    for (int r = 0; r < NR; ++r) R[j][r] = 0ull;
  long long sk[KSLOT];
  double sv[KSLOT][F];
  int used = 0;
  unsigned kept = 0;
  bool ovf = false;
#pragma unroll
  for (int s = 0; s < KSLOT; ++s) {
    sk[s] = EMPTY;
#pragma unroll
    for (int f = 0; f < F; ++f) sv[s][f] = init;
  }

  const long long step = (long long)gridDim.x * NTHR * ROWS;
  int it = 0;
  for (long long base = (long long)blockIdx.x * NTHR * ROWS; base < a.n; base += step, ++it) {
    if (agg_overflowed(a, &s_ovf, it)) break;                 // the launch's result is discarded: stop scanning
    long long row[ROWS];
    bool inr[ROWS], keep[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      row[j] = base + (long long)j * NTHR + tid;
      inr[j] = row[j] < a.n;
    }
    if (base + (long long)NTHR * ROWS <= a.n) P::template load<false, true>(a, row, inr, R);   // whole block: no masks
    else P::template load<false, false>(a, row, inr, R);
    P::run_a(a, R);
    bool any = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      keep[j] = inr[j] && P::keep(R[j]);
      any |= keep[j];
      kept += keep[j] ? 1u : 0u;
    }
    if (!__builtin_amdgcn_ballot_w64(any)) continue;           // no kept row in this wave
    P::template load<true, false>(a, row, keep, R);            // late columns: the kept rows only
    P::run_b(a, R);
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      if (!keep[j]) continue;
      const long long key = P::key(R[j]);
      double v[F];
      P::vals(R[j], v);
      bool done = false;
#pragma unroll
      for (int s = 0; s < KSLOT; ++s) {
        const bool hit = !done && s < used && sk[s] == key;   // selects (see the insert below)
#pragma unroll
        for (int f = 0; f < F; ++f) sv[s][f] = hit ? acc_op(sv[s][f], v[f], op) : sv[s][f];
        done = done || hit;
      }
      if (!done && used < KSLOT) {
#pragma unroll
        for (int s = 0; s < KSLOT; ++s) {
          const bool ins = !done && s == used;   // selects, not a store at [used]: that form went to scratch
          sk[s] = ins ? key : sk[s];
#pragma unroll
          for (int f = 0; f < F; ++f) sv[s][f] = ins ? v[f] : sv[s][f];
          done = done || ins;
        }
        ++used;
      }
      if (!done && !ovf) {
        ovf = (key == EMPTY) || !table_insert<F>(tk, tv, CAP, key, v, a.nval, op);
        if (ovf) agg_mark_overflow(a, &s_ovf);
      }
    }
  }
  __syncthreads();
  if (s_ovf) {                                               // no flush: the host re-runs the batch (emitted form)
    if (tid == 0) {
      atomicOr(a.table, 1ull);
      atomicAdd(a.table + 1, (unsigned long long)kept);
    }
    return;
  }
#pragma unroll
  for (int s = 0; s < KSLOT; ++s) {
    bool act = s < used;
    while (true) {
      const u64 bal = __builtin_amdgcn_ballot_w64(act);
      if (!bal) break;
      const int leader = __builtin_ctzll(bal);
      const long long kl = __shfl(sk[s], leader);
      const bool mine = act && sk[s] == kl;
      double v[F];
#pragma unroll
      for (int f = 0; f < F; ++f) v[f] = wave_reduce(mine ? sv[s][f] : init, op);
      if (lane == leader) ovf |= (kl == EMPTY) || !table_insert<F>(tk, tv, CAP, kl, v, a.nval, op);
      act = act && !mine;
    }
  }
  atomicAdd(&s_kept, (unsigned long long)kept);
  if (ovf) s_ovf = 1;
  __syncthreads();
  long long* gk = reinterpret_cast<long long*>(a.table + 2);
  double* gv = reinterpret_cast<double*>(a.table + 2 + GCAP);
  for (int i = tid; i < CAP; i += NTHR) {
    const long long k = tk[i];
    if (k == EMPTY) continue;
    double v[F];
#pragma unroll
    for (int f = 0; f < F; ++f) v[f] = tv[i * FMAX + f];
    if (!table_insert<F>(gk, gv, GCAP, k, v, a.nval, op, GWIN)) s_ovf = 1;
  }
  __syncthreads();
  if (tid == 0) {
    if (s_ovf) atomicOr(a.table, 1ull);
    atomicAdd(a.table + 1, s_kept);
  }
}

// ---------------------------------------------------------------- fused join probe (reference JoinProbe inside the
// pipeline chain: src/lambdas/headers/JoinTuple.h:434, Pipeline.h:194)
// The probe side's join hash is the engine's (kernels.hash_keys of one integer key column: splitmix64's finaliser of
// key + golden ratio), the slot the build's (relops.hip join_insert: the finaliser of the hash, masked; the kEmpty
// hash has the extra slot cap). A slot is ONE 16-byte read; a key with one build row keeps that row as its payload,
// a repeated key the start of its CSR run in jperm.
constexpr u64 JEMPTY = 0x8000000000000000ull, JGOLD = 0x9E3779B97F4A7C15ull;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u64 fin64(u64 x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

// build rows matching probe key k: cnt (0 = none) and the payload (the row when cnt == 1, else the run start)
// Join tables of more than JWHOLE slots probe linearly INSIDE aligned regions of JREGION slots (wrapping at the
// region's end, not the table's): relops.hip builds them region by region in LDS (kJRegion / kJWholeWrap there: the
// values must be equal). Smaller tables: plain linear probing over the whole table.
constexpr unsigned long long JREGION = 4096, JWHOLE = 1ull << 22;
__device__ __forceinline__ unsigned long long jnext(unsigned long long s, unsigned long long mask) {
  const unsigned long long rm = mask < JWHOLE ? mask : JREGION - 1;
  return (s & ~rm) | ((s + 1) & rm);
}

__device__ __forceinline__ void join_find(const PipeArgs& a, long long k, unsigned& cnt, unsigned& pay) {
  const u64 h = fin64((u64)k + JGOLD);
  u64 s = h == JEMPTY ? a.jmask + 1 : (fin64(h) & a.jmask);
  cnt = 0;
  pay = 0;
  for (u64 it = 0; it <= a.jmask; ++it) {       // >= 2 slots per build row: an empty slot ends every chain
    const u64x2 e = *reinterpret_cast<const u64x2*>(a.jtab + 2 * s);
    if (e[0] == h) {
      cnt = (unsigned)e[1] + (h != JEMPTY ? 1u : 0u);
      pay = (unsigned)(e[1] >> 32);
      return;
    }
    if (e[0] == JEMPTY || h == JEMPTY) return;
    s = jnext(s, a.jmask);
  }
}

// join_find for the ROWS rows of a thread at once: every kept row's first slot is read before any is compared (the
// rows' probe latencies overlap instead of adding up), then each row walks its own collision chain.
template <int ROWS>
__device__ __forceinline__ void join_find_rows(const PipeArgs& a, const long long (&k)[ROWS], const bool (&keep)[ROWS],
                                               unsigned (&cnt)[ROWS], unsigned (&pay)[ROWS]) {
  u64 h[ROWS], s[ROWS];
  u64x2 e[ROWS];
  bool may[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    cnt[j] = 0;
    pay[j] = 0;
    h[j] = fin64((u64)k[j] + JGOLD);
    const u64 f = fin64(h[j]);
    s[j] = h[j] == JEMPTY ? a.jmask + 1 : (f & a.jmask);
    may[j] = keep[j];
    if (a.jbloom && keep[j] && h[j] != JEMPTY) {    // the table's probe filter first (L2-resident)
      const u64 b = (1ull << ((f >> 40) & 63)) | (1ull << ((f >> 46) & 63));
      may[j] = (a.jbloom[s[j] >> a.jbshift] & b) == b;
    }
  }
#pragma unroll
  for (int j = 0; j < ROWS; ++j)
    if (may[j]) e[j] = *reinterpret_cast<const u64x2*>(a.jtab + 2 * s[j]);
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    if (!may[j]) continue;
    for (u64 it = 0; it <= a.jmask; ++it) {       // >= 2 slots per build row: an empty slot ends every chain
      if (e[j][0] == h[j]) {
        cnt[j] = (unsigned)e[j][1] + (h[j] != JEMPTY ? 1u : 0u);
        pay[j] = (unsigned)(e[j][1] >> 32);
        break;
      }
      if (e[j][0] == JEMPTY || h[j] == JEMPTY) break;
      s[j] = jnext(s[j], a.jmask);
      e[j] = *reinterpret_cast<const u64x2*>(a.jtab + 2 * s[j]);
    }
  }
}

// One kept (key, values) row into the thread's KSLOT register slots, else the workgroup's LDS table.
template <int F>
__device__ __forceinline__ void agg_row(const PipeArgs& a, long long key, const double (&v)[F], long long (&sk)[KSLOT],
                                        double (&sv)[KSLOT][F], int& used, bool& ovf, long long* tk, double* tv,
                                        int op) {
  bool done = false;
#pragma unroll
  for (int s = 0; s < KSLOT; ++s) {
    const bool hit = !done && s < used && sk[s] == key;   // selects (see the insert below)
#pragma unroll
    for (int f = 0; f < F; ++f) sv[s][f] = hit ? acc_op(sv[s][f], v[f], op) : sv[s][f];
    done = done || hit;
  }
  if (!done && used < KSLOT) {
#pragma unroll
    for (int s = 0; s < KSLOT; ++s) {
      const bool ins = !done && s == used;   // selects, not a store at [used]: that form went to scratch
      sk[s] = ins ? key : sk[s];
#pragma unroll
      for (int f = 0; f < F; ++f) sv[s][f] = ins ? v[f] : sv[s][f];
      done = done || ins;
    }
    ++used;
  }
  if (!done && !ovf) {
    ovf = (key == EMPTY) || !table_insert<F>(tk, tv, CAP, key, v, a.nval, op);
    if (ovf) __hip_atomic_fetch_or(a.table, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // seen by every loop
  }
}

// register slots -> LDS table (wave-combined per key) -> the global table; status words
template <int F>
__device__ __forceinline__ void agg_flush(const PipeArgs& a, long long (&sk)[KSLOT], double (&sv)[KSLOT][F], int used,
                                          bool ovf, unsigned long long kept, long long* tk, double* tv, int* s_ovf,
                                          unsigned long long* s_kept, double init, int op) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (ovf) *s_ovf = 1;
  __syncthreads();
  if (*s_ovf || (__hip_atomic_load(a.table, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1ull)) {
    atomicAdd(s_kept, kept);                       // the launch overflowed: no flush (the host re-runs the batch)
    __syncthreads();
    if (tid == 0) {
      atomicOr(a.table, 1ull);
      atomicAdd(a.table + 1, *s_kept);
    }
    return;
  }
#pragma unroll
  for (int s = 0; s < KSLOT; ++s) {
    bool act = s < used;
    while (true) {
      const u64 bal = __builtin_amdgcn_ballot_w64(act);
      if (!bal) break;
      const int leader = __builtin_ctzll(bal);
      const long long kl = __shfl(sk[s], leader);
      const bool mine = act && sk[s] == kl;
      double v[F];
#pragma unroll
      for (int f = 0; f < F; ++f) v[f] = wave_reduce(mine ? sv[s][f] : init, op);
      if (lane == leader) ovf |= (kl == EMPTY) || !table_insert<F>(tk, tv, CAP, kl, v, a.nval, op);
      act = act && !mine;
    }
  }
  atomicAdd(s_kept, kept);
  if (ovf) *s_ovf = 1;
  __syncthreads();
  long long* gk = reinterpret_cast<long long*>(a.table + 2);
  double* gv = reinterpret_cast<double*>(a.table + 2 + GCAP);
  for (int i = tid; i < CAP; i += NTHR) {
    const long long k = tk[i];
    if (k == EMPTY) continue;
    double v[F];
#pragma unroll
    for (int f = 0; f < F; ++f) v[f] = tv[i * FMAX + f];
    if (!table_insert<F>(gk, gv, GCAP, k, v, a.nval, op, GWIN)) *s_ovf = 1;
  }
  __syncthreads();
  if (tid == 0) {
    if (*s_ovf) atomicOr(a.table, 1ull);
    atomicAdd(a.table + 1, *s_kept);
  }
}

// scan -> predicate -> join probe -> [post-join predicate, key, values] per match -> aggregate, ONE launch. P adds to
// the jit_agg_body policy: JK (the probe key's register), loadb(a, brow, m, R) (the build-side columns of the matched
// build rows) and keep2(r) (the predicate after the join: the key re-check and any build-side condition). The
// matches of a probe row (several for a repeated build key) are walked in lock step over the wave's rows: every
// step loads one matched build row per active row and runs segment B on it. status[1] counts the rows that passed
// segment A (the stage's selectivity estimate, as in jit_agg_body).
template <typename P>
__device__ __forceinline__ void jit_join_agg_body(const PipeArgs& a) {
  constexpr int F = P::F, NR = P::NR, ROWS = P::ROWS;
  __shared__ long long tk[CAP];
  __shared__ double tv[CAP * FMAX];
  __shared__ int s_ovf;
  __shared__ unsigned long long s_kept;
  const int tid = threadIdx.x;
  const int op = P::OP >= 0 ? P::OP : a.agg_op;     // compile-time when the program fixes it (see jit_agg_body)
  const double init = op == 0 ? 0.0 : (op == 1 ? __builtin_inf() : -__builtin_inf());
  for (int i = tid; i < CAP; i += NTHR) tk[i] = EMPTY;
  for (int i = tid; i < CAP * FMAX; i += NTHR) tv[i] = init;
  if (tid == 0) {
    s_ovf = 0;
    s_kept = 0;
  }
  __syncthreads();

  u64 R[ROWS][NR];
#pragma unroll
  for (int j = 0; j < ROWS; ++j)
#pragma unroll
    for (int r = 0; r < NR; ++r) R[j][r] = 0ull;
  long long sk[KSLOT];
  double sv[KSLOT][F];
  int used = 0;
  unsigned kept = 0;
  bool ovf = false;
#pragma unroll
  for (int s = 0; s < KSLOT; ++s) {
    sk[s] = EMPTY;
#pragma unroll
    for (int f = 0; f < F; ++f) sv[s][f] = init;
  }

  const long long step = (long long)gridDim.x * NTHR * ROWS;
  int it = 0;
  for (long long base = (long long)blockIdx.x * NTHR * ROWS; base < a.n; base += step, ++it) {
    if (ovf || agg_overflowed(a, &s_ovf, it)) break;       // the launch's result is discarded: stop scanning
    long long row[ROWS], brow[ROWS];
    bool inr[ROWS], keep[ROWS], act[ROWS];
    unsigned cnt[ROWS], pay[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      row[j] = base + (long long)j * NTHR + tid;
      inr[j] = row[j] < a.n;
    }
    if (base + (long long)NTHR * ROWS <= a.n) P::template load<false, true>(a, row, inr, R);
    else P::template load<false, false>(a, row, inr, R);
    P::run_a(a, R);
    bool any = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      keep[j] = inr[j] && P::keep(R[j]);
      kept += keep[j] ? 1u : 0u;
    }
    // probe: every kept row's first slot read issued together
    {
      long long k[ROWS];
#pragma unroll
      for (int j = 0; j < ROWS; ++j) k[j] = (long long)R[j][P::JK];
      join_find_rows<ROWS>(a, k, keep, cnt, pay);
    }
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      keep[j] = keep[j] && cnt[j] != 0;
      any |= keep[j];
    }
    if (!__builtin_amdgcn_ballot_w64(any)) continue;
    P::template load<true, false>(a, row, keep, R);            // late probe-side columns: the matched rows only
    for (unsigned t = 0;; ++t) {
      bool more = false;
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        act[j] = keep[j] && t < cnt[j];
        brow[j] = !act[j] ? 0ll : (cnt[j] == 1u ? (long long)pay[j] : a.jperm[(long long)pay[j] + t]);
        more |= act[j];
      }
      if (!__builtin_amdgcn_ballot_w64(more)) break;
      P::loadb(a, brow, act, R);
      P::run_b(a, R);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        if (!act[j] || !P::keep2(R[j])) continue;
        const long long key = P::key(R[j]);
        double v[F];
        P::vals(R[j], v);
        agg_row<F>(a, key, v, sk, sv, used, ovf, tk, tv, op);
      }
    }
  }
  agg_flush<F>(a, sk, sv, used, ovf, (unsigned long long)kept, tk, tv, &s_ovf, &s_kept, init, op);
}

// ---------------------------------------------------------------- emit: (key parts, values) rows for the sink
// The high-cardinality form of a fused stage (more groups than GCAP): instead of pre-aggregating, every kept (and,
// with a join, matched) row writes its P::NE emitted registers (key parts, then values) straight from registers —
// no filter mask, compaction, key / value gathers or value-expression temporaries in HBM. The sink's device group-by
// (relops) then reduces them. Workgroup w owns the rows [w * tile_rows, (w + 1) * tile_rows) and writes its rows
// densely into ITS region [w * cap, (w + 1) * cap) of every output column (out + c * ostride): no global atomics,
// deterministic placement; tile_cnt[w] = rows written, status[0] |= 1 when a region overflowed (the host then runs
// the batch eagerly). Per block of NTHR * ROWS rows: a count pass, a workgroup exclusive scan in LDS, a write pass
// (segment B is re-run for the write only when some lane of the wave walked more than one match). P::emit also gets
// the row's index and its matched build row: the "pairs" form of a fused filter + join probe emits exactly those two.
template <typename P>
__device__ __forceinline__ void jit_emit_body(const PipeArgs& a, unsigned long long* __restrict__ out, long long tile_rows,
                                              long long cap, long long ostride, unsigned* __restrict__ tile_cnt) {
  constexpr int NR = P::NR, ROWS = P::ROWS, NE = P::NE;
  __shared__ unsigned s_scan[NTHR / 64];
  __shared__ unsigned s_jscan[ROWS][NTHR / 64];   // per row slot j: each wave's count of emitted rows
  __shared__ int s_multi[NTHR / 64];              // a wave walked more than one match for some row
  __shared__ unsigned long long s_kept;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long t0 = (long long)blockIdx.x * tile_rows;
  const long long t1 = t0 + tile_rows < a.n ? t0 + tile_rows : a.n;
  unsigned long long* region = out + (long long)blockIdx.x * cap;
  if (tid == 0) s_kept = 0;
  u64 R[ROWS][NR];
#pragma unroll
  for (int j = 0; j < ROWS; ++j)
#pragma unroll
    for (int r = 0; r < NR; ++r) R[j][r] = 0ull;
  long long written = 0;
  unsigned kept = 0;
  bool ovf = false;
  for (long long base = t0; base < t1; base += (long long)NTHR * ROWS) {
    long long row[ROWS], brow[ROWS];
    bool inr[ROWS], keep[ROWS], act[ROWS];
    unsigned cnt[ROWS], pay[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      row[j] = base + (long long)j * NTHR + tid;
      inr[j] = row[j] < t1;
    }
    if (base + (long long)NTHR * ROWS <= t1) P::template load<false, true>(a, row, inr, R);
    else P::template load<false, false>(a, row, inr, R);
    P::run_a(a, R);
    bool any = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      keep[j] = inr[j] && P::keep(R[j]);
      kept += keep[j] ? 1u : 0u;
      cnt[j] = keep[j] ? 1u : 0u;
      pay[j] = 0;
    }
    if constexpr (P::JOIN) {                       // every kept row's first slot read together
      long long k[ROWS];
#pragma unroll
      for (int j = 0; j < ROWS; ++j) k[j] = (long long)R[j][P::JK];
      join_find_rows<ROWS>(a, k, keep, cnt, pay);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) keep[j] = keep[j] && cnt[j] != 0;
    }
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      any |= keep[j];
    }
    const bool wave_any = __builtin_amdgcn_ballot_w64(any) != 0ull;
    if (wave_any) P::template load<true, false>(a, row, keep, R);
    // count pass
    unsigned e = 0, trips = 0;
    if (wave_any) {
      for (unsigned t = 0;; ++t) {
        bool more = false;
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
          act[j] = keep[j] && t < cnt[j];
          brow[j] = !act[j] ? 0ll : (!P::JOIN || cnt[j] == 1u ? (long long)pay[j] : a.jperm[(long long)pay[j] + t]);
          more |= act[j];
        }
        if (!__builtin_amdgcn_ballot_w64(more)) break;
        ++trips;
        if constexpr (P::JOIN) P::loadb(a, brow, act, R);
        P::run_b(a, R);
#pragma unroll
        for (int j = 0; j < ROWS; ++j) e += (act[j] && P::keep2(R[j])) ? 1u : 0u;
      }
    }
    // workgroup exclusive scan of e (thread-major placement), and per row slot j (row-order placement: with at most
    // one output per row the block's rows leave in row order — a scan of a table stored in key order then emits its
    // keys in order, which the sink's clustered-key group-by (relops run_aggregate) needs)
    unsigned x = e;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) s_scan[wave] = x;
    unsigned cj[ROWS], xj[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      cj[j] = (trips == 1 && keep[j] && P::keep2(R[j])) ? 1u : 0u;
      unsigned z = cj[j];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned y = __shfl_up(z, d, 64);
        if (lane >= d) z += y;
      }
      xj[j] = z;
      if (lane == 63) s_jscan[j][wave] = z;
    }
    if (lane == 0) s_multi[wave] = trips > 1 ? 1 : 0;
    __syncthreads();
    unsigned before = 0, total = 0;
    bool multi = false;
#pragma unroll
    for (int w = 0; w < NTHR / 64; ++w) {
      const unsigned v = s_scan[w];
      before += w < wave ? v : 0u;
      total += v;
      multi |= s_multi[w] != 0;
    }
    long long o = written + before + x - e;
    long long oj[ROWS];
    {
      unsigned long long acc = 0;
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        unsigned bj = 0, tj = 0;
#pragma unroll
        for (int w = 0; w < NTHR / 64; ++w) {
          const unsigned v = s_jscan[j][w];
          bj += w < wave ? v : 0u;
          tj += v;
        }
        oj[j] = written + (long long)acc + bj + xj[j] - cj[j];
        acc += tj;
      }
    }
    if (written + total > cap) ovf = true;
    // write pass
    if (e != 0 && !ovf) {
      if (trips <= 1) {              // the registers still hold the single match's segment B
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
          if (!keep[j] || !P::keep2(R[j])) continue;     // keep[j] => exactly one match (trips <= 1)
          u64 w[NE];
          P::emit(R[j], w, row[j], P::JOIN ? (long long)pay[j] : 0ll);
          const long long at = multi ? o : oj[j];
#pragma unroll
          for (int c = 0; c < NE; ++c) region[c * ostride + at] = w[c];
          ++o;
        }
      } else {
        for (unsigned t = 0;; ++t) {
          bool more = false;
#pragma unroll
          for (int j = 0; j < ROWS; ++j) {
            act[j] = keep[j] && t < cnt[j];
            brow[j] = !act[j] ? 0ll : (!P::JOIN || cnt[j] == 1u ? (long long)pay[j] : a.jperm[(long long)pay[j] + t]);
            more |= act[j];
          }
          if (!__builtin_amdgcn_ballot_w64(more)) break;
          if constexpr (P::JOIN) P::loadb(a, brow, act, R);
          P::run_b(a, R);
#pragma unroll
          for (int j = 0; j < ROWS; ++j) {
            if (!act[j] || !P::keep2(R[j])) continue;
            u64 w[NE];
            P::emit(R[j], w, row[j], brow[j]);
#pragma unroll
            for (int c = 0; c < NE; ++c) region[c * ostride + o] = w[c];
            ++o;
          }
        }
      }
    }
    written += total;
    __syncthreads();                 // s_scan is rewritten by the next block
  }
  atomicAdd(&s_kept, (unsigned long long)kept);
  __syncthreads();
  if (tid == 0) {
    tile_cnt[blockIdx.x] = ovf ? 0u : (unsigned)written;
    if (ovf) atomicOr(a.table, 1ull);
    atomicAdd(a.table + 1, s_kept);
  }
}

// Filter only: keep flag per row (every column early, the whole program in run_a).
template <typename P>
__device__ __forceinline__ void jit_mask_body(const PipeArgs& a, unsigned char* __restrict__ mask) {
  constexpr int NR = P::NR, ROWS = P::ROWS;
  u64 R[ROWS][NR];
#pragma unroll
  for (int j = 0; j < ROWS; ++j)
#pragma unroll
    for (int r = 0; r < NR; ++r) R[j][r] = 0ull;
  const int tid = threadIdx.x;
  const long long step = (long long)gridDim.x * NTHR * ROWS;
  for (long long base = (long long)blockIdx.x * NTHR * ROWS; base < a.n; base += step) {
    long long row[ROWS];
    bool inr[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      row[j] = base + (long long)j * NTHR + tid;
      inr[j] = row[j] < a.n;
    }
    if (base + (long long)NTHR * ROWS <= a.n) P::template load<false, true>(a, row, inr, R);
    else P::template load<false, false>(a, row, inr, R);
    P::run_a(a, R);
#pragma unroll
    for (int j = 0; j < ROWS; ++j)
      if (inr[j]) mask[row[j]] = P::keep(R[j]) ? 1 : 0;
  }
}

}  // namespace nsdb_pipe
