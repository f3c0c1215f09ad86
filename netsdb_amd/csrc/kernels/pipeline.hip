// Fused relational pipeline: scan -> filter -> project -> low-cardinality group-by + aggregate in ONE pass over the
// input columns (reference: src/lambdas/headers/Pipeline.h:57,194, which pushes each page through the whole chain
// of executors while it is cache-resident; the executors are FilterExecutor / ApplyExecutor / the aggregation
// HashSink, src/queryExecution/headers/AggregationProcessor.h:16).
//
// The stage's lambda trees (the selection predicate, the group key and the value row: makeLambdaFromMember, ==, <,
// &&, ||, +, -, *, /, IN, LIKE prefix/suffix, CASE) are compiled on the host (execution/pipeline.py) into a short
// register program that this kernel INTERPRETS per row in registers: no intermediate column (filter mask, value row,
// key) is ever materialised in HBM. The program is ahead-of-time code (no run-time compilation); its interpretation
// cost is amortised over ROWS rows per thread and the opcode / register indices are wave-uniform (kernel arguments,
// scalar branches only).
//
//  * Register file: NREG virtual 64-bit registers per row slot as ONE vector value in VGPRs; the wave-uniform register
//    number indexes it with indirect register addressing (s_set_gpr_idx_on + v_mov): no scratch, no per-register
//    branches.
//  * Columns are loaded straight into their registers: registers [0, ncol) hold the loaded columns. "Late" columns
//    (read only by the key / value row) are loaded after the predicate, for the kept rows only (a wave skips the
//    cache lines none of its kept rows needs).
//  * Column loads are unrolled over the MAXCOL column slots (compile-time register numbers): every row load of a pass
//    is issued before the first one is used (the 2nd round only fetches the bytes of short-string columns), so a
//    wave keeps all its columns' cache lines in flight instead of one column at a time.
//  * Aggregation: each thread keeps KSLOT (key, F values) slots in registers (few groups hit them every row); a row
//    whose key is in no slot goes to the workgroup's LDS hash table (CAP slots, 64-bit CAS + LDS float atomics). At
//    the end every wave reduces its lanes' slots per distinct key (cross-lane butterflies, one LDS update per key per
//    wave), and the workgroup merges its table into ONE global table of GCAP slots with device atomics: the host
//    reads back a few KB, no per-workgroup partials and no second merge pass. A table overflow raises status[0]:
//    the stage then runs the unfused path (more groups than this kernel is for). status[1] counts the kept rows
//    (the host's selectivity estimate decides whether value columns load late, after the predicate).
#include "common.h"

namespace nsdb_pipe {

constexpr int NREG = 16, ROWS = 2, MAXINS = 48, MAXCOL = 10, FMAX = 8, KSLOT = 4, CAP = 256, NTHR = 256;
constexpr int GCAP = 2048;             // global table slots (power of two)
constexpr long long EMPTY = (long long)0x8000000000000000ULL;
constexpr int IMM_REG = -2;            // operand register meaning "the instruction's immediate"

enum Op : int {
  OP_NOP = 0, OP_CONST, OP_ADDF, OP_SUBF, OP_MULF, OP_DIVF, OP_ADDI, OP_SUBI, OP_MULI, OP_I2F,
  OP_LTF, OP_LEF, OP_GTF, OP_GEF, OP_EQF, OP_NEF, OP_LTI, OP_LEI, OP_GTI, OP_GEI, OP_EQI, OP_NEI,
  OP_AND, OP_OR, OP_NOT, OP_PACK, OP_SEQ, OP_SPRE, OP_SSUF, OP_SEL, OP_NEGF
};
enum ColKind : int { C_F64 = 0, C_I64, C_I32, C_F32, C_U8, C_SCODE, C_SREF };

struct Ins {
  int op, dst, a, b;
  long long imm;
};
struct Col {
  const void* p;                 // numeric column
  const long long* st;           // string column: row starts / ends into dat
  const long long* en;
  const unsigned char* dat;
  int kind, late, L, pad;
};
struct PipeArgs {
  Ins ins[MAXINS];
  Col col[MAXCOL];
  const unsigned char* lit;      // literal pool of the string ops
  long long n;
  int nins_a, nins, ncol, keep_reg, key_reg, nval, agg_op, pad;
  int val_reg[FMAX];
  unsigned long long* table;     // [2 + GCAP + GCAP * FMAX]: status (overflow, kept rows), keys, values (f64 bits)
};

typedef unsigned long long u64;
// The register file of one row slot: NREG 64-bit registers as ONE vector value (NREG VGPR pairs).
typedef unsigned long long regfile __attribute__((ext_vector_type(NREG)));

__device__ __forceinline__ double u2f(u64 x) { return __longlong_as_double((long long)x); }
__device__ __forceinline__ u64 f2u(double x) { return (u64)__double_as_longlong(x); }

// Short-string code exactly as StringColumn.short_codes / str_pack (bytes big-endian in the low 8L bits, << 3 | len)
__device__ __forceinline__ u64 short_code(const unsigned char* d, long long s, long long e, int L) {
  const long long len = e - s;
  if (len > L) return (u64)-1;
  u64 c = 0;
  for (int b = 0; b < L; ++b) c |= (b < len ? (u64)d[s + b] : 0ull) << (8 * (L - 1 - b));
  return (c << 3) | (u64)len;
}

// Pass 1 of a column's load: the row's value (numeric kinds) or its string start (x) and the low word of its end (y).
__device__ __forceinline__ void fetch(const Col& c, const long long (&row)[ROWS], const bool (&m)[ROWS], u64 (&x)[ROWS],
                                      unsigned (&y)[ROWS]) {
#pragma unroll
  for (int j = 0; j < ROWS; ++j) {
    x[j] = 0;
    y[j] = 0;
    if (m[j]) {
      const long long i = row[j];
      switch (c.kind) {
        case C_F64:
        case C_I64: x[j] = reinterpret_cast<const u64*>(c.p)[i]; break;
        case C_I32: x[j] = (u64)(long long)reinterpret_cast<const int*>(c.p)[i]; break;
        case C_F32: x[j] = f2u((double)reinterpret_cast<const float*>(c.p)[i]); break;
        case C_U8: x[j] = (u64)reinterpret_cast<const unsigned char*>(c.p)[i]; break;
        default:
          x[j] = (u64)c.st[i];
          y[j] = (unsigned)c.en[i];
      }
    }
  }
}

// Pass 2: the register value (string kinds: the short code from the bytes / the (start << 24 | length) reference;
// lengths fit 32 bits, so the end's low word suffices).
__device__ __forceinline__ u64 finish(const Col& c, u64 x, unsigned y, bool m) {
  if (c.kind == C_SCODE) return m ? short_code(c.dat, (long long)x, (long long)x + (long long)(unsigned)(y - (unsigned)x), c.L) : 0;
  if (c.kind == C_SREF) return (x << 24) | (u64)min(y - (unsigned)x, 0xFFFFFFu);
  return x;
}

// Every column of the pass (LATE: the late columns; else the early ones) into its register, all loads in flight at once.
template <bool LATE>
__device__ __forceinline__ void load_cols(const PipeArgs& a, const long long (&row)[ROWS], const bool (&m)[ROWS],
                                          regfile (&R)[ROWS]) {
  u64 x[MAXCOL][ROWS];
  unsigned y[MAXCOL][ROWS];
#pragma unroll
  for (int c = 0; c < MAXCOL; ++c)
    if (c < a.ncol && (a.col[c].late != 0) == LATE) fetch(a.col[c], row, m, x[c], y[c]);
#pragma unroll
  for (int c = 0; c < MAXCOL; ++c)
    if (c < a.ncol && (a.col[c].late != 0) == LATE) {
#pragma unroll
      for (int j = 0; j < ROWS; ++j) R[j][c] = finish(a.col[c], x[c][j], y[c][j], m[j]);
    }
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

__device__ __forceinline__ u64 operand(const regfile& R, int k, long long imm) {
  return k == IMM_REG ? (u64)imm : (k >= 0 ? R[k] : 0ull);
}

// Instructions [lo, hi) of the program over every row slot. The opcode and register numbers are kernel arguments
// (SGPRs): one scalar dispatch per instruction, indirect register reads / writes.
__device__ __forceinline__ void run(const PipeArgs& a, regfile (&R)[ROWS], int lo, int hi) {
  for (int pc = lo; pc < hi; ++pc) {
    const int op = a.ins[pc].op, dst = a.ins[pc].dst, ia = a.ins[pc].a, ib = a.ins[pc].b;
    const long long imm = a.ins[pc].imm;
    u64 x[ROWS], y[ROWS], z[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      x[j] = operand(R[j], ia, imm);
      y[j] = operand(R[j], ib, imm);
    }
    switch (op) {
#define NSDB_EACH(E)                                          \
  _Pragma("unroll") for (int j = 0; j < ROWS; ++j) {          \
    const double fx = u2f(x[j]), fy = u2f(y[j]);              \
    const long long sx = (long long)x[j], sy = (long long)y[j]; \
    (void)fx; (void)fy; (void)sx; (void)sy;                   \
    z[j] = (E);                                               \
  }                                                           \
  break;
      case OP_CONST: NSDB_EACH((u64)imm)
      case OP_ADDF: NSDB_EACH(f2u(fx + fy))
      case OP_SUBF: NSDB_EACH(f2u(fx - fy))
      case OP_MULF: NSDB_EACH(f2u(fx * fy))
      case OP_DIVF: NSDB_EACH(f2u(fx / fy))
      case OP_NEGF: NSDB_EACH(f2u(-fx))
      case OP_ADDI: NSDB_EACH((u64)(sx + sy))
      case OP_SUBI: NSDB_EACH((u64)(sx - sy))
      case OP_MULI: NSDB_EACH((u64)(sx * sy))
      case OP_I2F: NSDB_EACH(f2u((double)sx))
      case OP_LTF: NSDB_EACH((u64)(fx < fy))
      case OP_LEF: NSDB_EACH((u64)(fx <= fy))
      case OP_GTF: NSDB_EACH((u64)(fx > fy))
      case OP_GEF: NSDB_EACH((u64)(fx >= fy))
      case OP_EQF: NSDB_EACH((u64)(fx == fy))
      case OP_NEF: NSDB_EACH((u64)(fx != fy))
      case OP_LTI: NSDB_EACH((u64)(sx < sy))
      case OP_LEI: NSDB_EACH((u64)(sx <= sy))
      case OP_GTI: NSDB_EACH((u64)(sx > sy))
      case OP_GEI: NSDB_EACH((u64)(sx >= sy))
      case OP_EQI: NSDB_EACH((u64)(sx == sy))
      case OP_NEI: NSDB_EACH((u64)(sx != sy))
      case OP_AND: NSDB_EACH((u64)((x[j] != 0) & (y[j] != 0)))
      case OP_OR: NSDB_EACH((u64)((x[j] != 0) | (y[j] != 0)))
      case OP_NOT: NSDB_EACH((u64)(x[j] == 0))
      case OP_PACK: NSDB_EACH((x[j] << (imm & 63)) | y[j])
      case OP_SEL: NSDB_EACH(x[j] ? y[j] : R[j][(int)imm])                // z = x ? y : r[imm]
      case OP_SEQ:
      case OP_SPRE:
      case OP_SSUF: {                                      // ib: the column whose bytes x refers to
        const unsigned char* d = a.col[ib].dat;
        const int mode = op == OP_SEQ ? 0 : (op == OP_SPRE ? 1 : 2);
#pragma unroll
        for (int j = 0; j < ROWS; ++j) z[j] = str_match(d, x[j], a.lit, imm, mode) ? 1ull : 0ull;
        break;
      }
      default:
#pragma unroll
        for (int j = 0; j < ROWS; ++j) z[j] = 0;
#undef NSDB_EACH
    }
#pragma unroll
    for (int j = 0; j < ROWS; ++j) R[j][dst] = z[j];
  }
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

// Linear-probing insert of (key, values) into a table of cap slots (LDS or global). False: the table is full.
template <int F>
__device__ __forceinline__ bool table_insert(long long* tk, double* tv, unsigned cap, long long key, const double (&v)[F],
                                             int nval, int op) {
  unsigned h = slot_hash(key) & (cap - 1);
  for (unsigned p = 0; p < cap; ++p) {
    const long long prev = (long long)atomicCAS(reinterpret_cast<u64*>(tk + h), (u64)EMPTY, (u64)key);
    if (prev == EMPTY || prev == key) {
#pragma unroll
      for (int f = 0; f < F; ++f)
        if (f < nval) atomic_acc(tv + (size_t)h * FMAX + f, v[f], op);
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

template <int F>
__global__ void __launch_bounds__(NTHR) pipe_agg_kernel(const PipeArgs a) {
  __shared__ long long tk[CAP];
  __shared__ double tv[CAP * FMAX];
  __shared__ int s_ovf;
  __shared__ unsigned long long s_kept;
  const int tid = threadIdx.x, lane = tid & 63;
  const double init = a.agg_op == 0 ? 0.0 : (a.agg_op == 1 ? __builtin_inf() : -__builtin_inf());
  for (int i = tid; i < CAP; i += NTHR) tk[i] = EMPTY;
  for (int i = tid; i < CAP * FMAX; i += NTHR) tv[i] = init;
  if (tid == 0) {
    s_ovf = 0;
    s_kept = 0;
  }
  __syncthreads();

  regfile R[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) R[j] = (regfile)0;
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
  for (long long base = (long long)blockIdx.x * NTHR * ROWS; base < a.n; base += step) {
    long long row[ROWS];
    bool inr[ROWS], keep[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      row[j] = base + (long long)j * NTHR + tid;
      inr[j] = row[j] < a.n;
    }
    load_cols<false>(a, row, inr, R);                          // the predicate's ("early") columns
    run(a, R, 0, a.nins_a);
    bool any = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      keep[j] = inr[j] && (a.keep_reg < 0 || R[j][a.keep_reg] != 0);
      any |= keep[j];
      kept += keep[j] ? 1u : 0u;
    }
    if (!__builtin_amdgcn_ballot_w64(any)) continue;           // no kept row in this wave
    load_cols<true>(a, row, keep, R);                          // late columns: the kept rows only
    run(a, R, a.nins_a, a.nins);
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      if (!keep[j]) continue;
      const long long key = a.key_reg < 0 ? 0 : (long long)R[j][a.key_reg];   // key_reg < 0: one global group
      double v[F];
#pragma unroll
      for (int f = 0; f < F; ++f) v[f] = f < a.nval ? u2f(R[j][a.val_reg[f]]) : 0.0;
      bool done = false;
#pragma unroll
      for (int s = 0; s < KSLOT; ++s) {
        if (!done && s < used && sk[s] == key) {
#pragma unroll
          for (int f = 0; f < F; ++f) sv[s][f] = acc_op(sv[s][f], v[f], a.agg_op);
          done = true;
        }
      }
      if (!done && used < KSLOT) {
#pragma unroll
        for (int s = 0; s < KSLOT; ++s) {
          if (!done && s == used) {
            sk[s] = key;
#pragma unroll
            for (int f = 0; f < F; ++f) sv[s][f] = v[f];
            done = true;
          }
        }
        ++used;
      }
      if (!done) ovf |= (key == EMPTY) || !table_insert<F>(tk, tv, CAP, key, v, a.nval, a.agg_op);
    }
  }
  // flush the register slots: per slot, the wave's lanes holding the leader's key are reduced across lanes and the
  // leader lane makes the one LDS update for that key (no 64-way atomic contention on a few hot entries)
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
      for (int f = 0; f < F; ++f) v[f] = wave_reduce(mine ? sv[s][f] : init, a.agg_op);
      if (lane == leader) ovf |= (kl == EMPTY) || !table_insert<F>(tk, tv, CAP, kl, v, a.nval, a.agg_op);
      act = act && !mine;
    }
  }
  atomicAdd(&s_kept, (unsigned long long)kept);
  if (ovf) s_ovf = 1;
  __syncthreads();
  // the workgroup's table into the global one
  long long* gk = reinterpret_cast<long long*>(a.table + 2);
  double* gv = reinterpret_cast<double*>(a.table + 2 + GCAP);
  for (int i = tid; i < CAP; i += NTHR) {
    const long long k = tk[i];
    if (k == EMPTY) continue;
    double v[F];
#pragma unroll
    for (int f = 0; f < F; ++f) v[f] = tv[i * FMAX + f];
    if (!table_insert<F>(gk, gv, GCAP, k, v, a.nval, a.agg_op)) s_ovf = 1;
  }
  __syncthreads();
  if (tid == 0) {
    if (s_ovf) atomicOr(a.table, 1ull);
    atomicAdd(a.table + 1, s_kept);
  }
}

// The global table's initial state (status 0, keys EMPTY, values the aggregation's identity), one launch.
__global__ void __launch_bounds__(NTHR) pipe_init_kernel(unsigned long long* table, int op) {
  const double init = op == 0 ? 0.0 : (op == 1 ? __builtin_inf() : -__builtin_inf());
  const int i = blockIdx.x * NTHR + threadIdx.x;
  if (i < 2) table[i] = 0;
  if (i < GCAP) table[2 + i] = (u64)EMPTY;
  for (int k = i; k < GCAP * FMAX; k += gridDim.x * NTHR) table[2 + GCAP + k] = f2u(init);
}

// Filter only: the predicate program over every row, the keep flag written as one byte per row (the FILTER of a
// scan-filter stage that feeds a join / materialisation: no comparison column, literal column or AND of two masks is
// materialised; the engine turns the mask into the stage's row selection).
__global__ void __launch_bounds__(NTHR) pipe_mask_kernel(const PipeArgs a, unsigned char* __restrict__ mask) {
  regfile R[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) R[j] = (regfile)0;
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
    load_cols<false>(a, row, inr, R);
    run(a, R, 0, a.nins);
#pragma unroll
    for (int j = 0; j < ROWS; ++j)
      if (inr[j]) mask[row[j]] = (unsigned char)(a.keep_reg < 0 ? 1 : (R[j][a.keep_reg] != 0));
  }
}

}  // namespace nsdb_pipe

extern "C" {

int nsdb_pipe_sizes(int* out) {
  out[0] = nsdb_pipe::MAXINS;
  out[1] = nsdb_pipe::MAXCOL;
  out[2] = nsdb_pipe::NREG;
  out[3] = nsdb_pipe::FMAX;
  out[4] = nsdb_pipe::CAP;
  out[5] = (int)sizeof(nsdb_pipe::PipeArgs);
  out[6] = nsdb_pipe::ROWS;
  out[7] = nsdb_pipe::NTHR;
  out[8] = nsdb_pipe::GCAP;
  return 0;
}

// args: a host PipeArgs image (the binding fills it field by field, the mask pass marks every column early);
// grid = number of workgroups. Initialises the global table, then the fused pass.
int nsdb_pipe_agg(const void* args, int grid, hipStream_t st) {
  if (grid <= 0) return -1;
  const nsdb_pipe::PipeArgs& a = *reinterpret_cast<const nsdb_pipe::PipeArgs*>(args);
  if (a.nins > nsdb_pipe::MAXINS || a.ncol > nsdb_pipe::MAXCOL || a.nval > nsdb_pipe::FMAX || a.nins_a > a.nins ||
      a.table == nullptr)
    return -2;
  hipLaunchKernelGGL(nsdb_pipe::pipe_init_kernel, dim3(nsdb_pipe::GCAP / nsdb_pipe::NTHR), dim3(nsdb_pipe::NTHR), 0, st,
                     a.table, a.agg_op);
  if (a.nval <= 2)
    hipLaunchKernelGGL(nsdb_pipe::pipe_agg_kernel<2>, dim3(grid), dim3(nsdb_pipe::NTHR), 0, st, a);
  else if (a.nval <= 4)
    hipLaunchKernelGGL(nsdb_pipe::pipe_agg_kernel<4>, dim3(grid), dim3(nsdb_pipe::NTHR), 0, st, a);
  else if (a.nval <= 6)
    hipLaunchKernelGGL(nsdb_pipe::pipe_agg_kernel<6>, dim3(grid), dim3(nsdb_pipe::NTHR), 0, st, a);
  else
    hipLaunchKernelGGL(nsdb_pipe::pipe_agg_kernel<nsdb_pipe::FMAX>, dim3(grid), dim3(nsdb_pipe::NTHR), 0, st, a);
  return (int)hipGetLastError();
}

int nsdb_pipe_mask(const void* args, unsigned char* mask, int grid, hipStream_t st) {
  if (grid <= 0) return -1;
  const nsdb_pipe::PipeArgs& a = *reinterpret_cast<const nsdb_pipe::PipeArgs*>(args);
  if (a.nins > nsdb_pipe::MAXINS || a.ncol > nsdb_pipe::MAXCOL) return -2;
  hipLaunchKernelGGL(nsdb_pipe::pipe_mask_kernel, dim3(grid), dim3(nsdb_pipe::NTHR), 0, st, a, mask);
  return (int)hipGetLastError();
}

}  // extern "C"
