// Fused relational pipeline: scan -> filter -> project -> low-cardinality group-by + aggregate in ONE pass over the
// input columns (reference: src/lambdas/headers/Pipeline.h:57,194, which pushes each page through the whole chain
// of executors while it is cache-resident; the executors are FilterExecutor / ApplyExecutor / the aggregation
// HashSink, src/queryExecution/headers/AggregationProcessor.h:16).
//
// The stage's lambda trees (the selection predicate, the group key and the value row: makeLambdaFromMember, ==, <,
// &&, ||, +, -, *, /, IN, LIKE prefix/suffix, CASE) are compiled on the host (execution/pipeline.py) into a short
// register program that this kernel INTERPRETS per row in registers: no intermediate column (filter mask, value row,
// key) is ever materialised in HBM. The program is ahead-of-time code (no run-time compilation); the opcode and
// register indices are wave-uniform (kernel arguments: scalar loads and scalar branches only).
//
//  * Register file: NR virtual 64-bit registers per row slot as ONE vector value in VGPRs; the wave-uniform register
//    number indexes it with indirect register addressing (s_set_gpr_idx_on + v_mov): no scratch, no per-register
//    branches. Each interpreted instruction runs over ROWS rows per thread, so its dispatch (one scalar load of the
//    next instruction, issued before the current one executes, and a scalar branch) is amortised over ROWS x 64
//    rows. Two shapes are instantiated, NR x ROWS = 16 x 2 and 8 x 4: a program that fits in 8 registers (most
//    predicates, Q06-like aggregates) runs twice as many rows per dispatch.
//  * Compares carry an AND-with register (the host folds `x CMP y && r` into one instruction), so a conjunction of
//    k range tests is k instructions, not 2k - 1.
//  * Columns are loaded straight into their (compile-time) registers [0, ncol): every row load of a pass is issued
//    before the first one is used (the 2nd round only fetches the bytes of short-string columns, which the host
//    places in the first MAXSTR column slots). "Late" columns (read only by the key / value row) are loaded after the
//    predicate, for the kept rows only, when the host's selectivity estimate says that saves bandwidth.
//  * Aggregation: each thread keeps KSLOT (key, F values) slots in registers (few groups hit them every row); a row
//    whose key is in no slot goes to the workgroup's LDS hash table (CAP slots, 64-bit CAS + LDS float atomics). At
//    the end every wave reduces its lanes' slots per distinct key (cross-lane butterflies, one LDS update per key per
//    wave), and the workgroup merges its table into ONE global table of GCAP slots with device atomics: the host
//    reads back a few KB, no per-workgroup partials and no second merge pass. A table overflow raises status[0]:
//    the stage then runs the unfused path (more groups than this kernel is for). status[1] counts the kept rows.
#include "common.h"
#include "pipeline_core.h"

namespace nsdb_pipe {

// Every column of the pass (LATE: the late columns; else the early ones) into its register. Round 1 issues every
// row load (numeric values; string starts and the low words of their ends) before any is used; round 2 turns the
// string columns (slots < MAXSTR) into their register form: the short code from the bytes (keys), or the
// (start << 24 | length) reference (byte comparisons). Lengths fit 32 bits, so the ends' low words suffice.
template <bool LATE, int NR, int ROWS>
__device__ __forceinline__ void load_cols(const PipeArgs& a, const long long (&row)[ROWS], const bool (&m)[ROWS],
                                          typename RF<NR>::vec (&R)[ROWS]) {
  unsigned y[MAXSTR][ROWS];
#pragma unroll
  for (int c = 0; c < (NR < MAXCOL ? NR : MAXCOL); ++c) {
    if (c >= a.ncol || (a.col[c].late != 0) != LATE) continue;
    const Col& C = a.col[c];
    const int kind = C.kind;
    if (kind == C_F64 || kind == C_I64) {
      const u64* p = reinterpret_cast<const u64*>(C.p);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) R[j][c] = m[j] ? p[row[j]] : 0ull;
    } else if (kind == C_I32) {
      const int* p = reinterpret_cast<const int*>(C.p);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) R[j][c] = m[j] ? (u64)(long long)p[row[j]] : 0ull;
    } else if (kind == C_F32) {
      const float* p = reinterpret_cast<const float*>(C.p);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) R[j][c] = m[j] ? f2u((double)p[row[j]]) : 0ull;
    } else if (kind == C_U8) {
      const unsigned char* p = reinterpret_cast<const unsigned char*>(C.p);
#pragma unroll
      for (int j = 0; j < ROWS; ++j) R[j][c] = m[j] ? (u64)p[row[j]] : 0ull;
    } else if (c < MAXSTR) {
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        R[j][c] = m[j] ? (u64)C.st[row[j]] : 0ull;
        y[c < MAXSTR ? c : 0][j] = m[j] ? (unsigned)C.en[row[j]] : 0u;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < MAXSTR; ++c) {
    if (c >= a.ncol || (a.col[c].late != 0) != LATE) continue;
    const Col& C = a.col[c];
    if (C.kind == C_SCODE) {
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        const u64 s = R[j][c];
        R[j][c] = m[j] ? short_code(C.dat, (long long)s, (long long)(unsigned)(y[c][j] - (unsigned)s), C.L) : 0ull;
      }
    } else if (C.kind == C_SREF) {
#pragma unroll
      for (int j = 0; j < ROWS; ++j) {
        const u64 s = R[j][c];
        R[j][c] = (s << 24) | (u64)min(y[c][j] - (unsigned)s, 0xFFFFFFu);
      }
    }
  }
}

extern __shared__ __attribute__((aligned(16))) unsigned char tile_smem[];

__device__ __forceinline__ int kind_width(int kind) {
  return (kind == C_F64 || kind == C_I64) ? 8 : ((kind == C_I32 || kind == C_F32) ? 4 : (kind == C_U8 ? 1 : 8));
}

// `bytes` of the tile image from g to LDS l, wave `wave`'s share of the wave-instructions. A full tile whose image
// is a multiple of 1 KiB uses 16-B DMA lanes; otherwise 4-byte elements use 4-B DMA lanes over exactly `valid` bytes
// of a bounds-checked buffer resource (lanes past the column's end read zeros, never out of the column), and byte
// columns are copied by the threads (a 1-byte DMA lane writes a whole LDS dword).
__device__ __forceinline__ void dma_tile(const void* g, long long valid, unsigned char* l, int bytes, int w, bool full,
                                         int wave, int lane) {
  constexpr int NW = NTHR / 64;
  const int nv = (int)(valid < (long long)bytes ? valid : (long long)bytes);
  if (w < 4 && !(full && (bytes & 1023) == 0)) {
    const unsigned char* src = reinterpret_cast<const unsigned char*>(g);
    for (int i = wave * 64 + lane; i < nv; i += NTHR) l[i] = src[i];
    return;
  }
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(g), (short)0, nv, 0x00020000);
  if (full && (bytes & 1023) == 0) {
    for (int ch = wave; ch < (bytes >> 10); ch += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (nsdb::lds_void*)(l + (ch << 10)), 16, (ch << 10) + lane * 16, 0, 0, 0);
  } else {
    for (int ch = wave; ch < (bytes >> 8); ch += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (nsdb::lds_void*)(l + (ch << 8)), 4, (ch << 8) + lane * 4, 0, 0, 0);
  }
}

// Hybrid kernels (HYB): the block's NTHR * ROWS rows of an iteration are first copied HBM -> LDS by LDS-DMA (every
// column at its native width: many KB in flight per workgroup, no VGPRs), then each thread moves its rows' values
// LDS -> its VGPR register file (one ds_read per column and row) and the register interpreter runs as usual. The
// interpreter's operands never touch LDS, so LDS carries each column byte once.
template <int NR, int ROWS>
__device__ __forceinline__ void hyb_dma(const PipeArgs& a, long long row0, long long nrow) {
  constexpr int T = NTHR * ROWS;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool full = nrow == T;
  for (int c = 0; c < a.ncol; ++c) {
    const Col& C = a.col[c];
    if (C.kind == C_SCODE || C.kind == C_SREF) {
      dma_tile(C.st + row0, nrow * 8, tile_smem + C.raw_off, T * 8, 8, full, wave, lane);
      if (!C.contig) dma_tile(C.en + row0, nrow * 8, tile_smem + C.aux_off, T * 8, 8, full, wave, lane);
    } else {
      const int w = kind_width(C.kind);
      dma_tile(reinterpret_cast<const unsigned char*>(C.p) + row0 * w, nrow * w, tile_smem + C.raw_off, T * w, w, full,
               wave, lane);
    }
  }
}

template <int NR, int ROWS>
__device__ __forceinline__ void hyb_load(const PipeArgs& a, long long row0, long long nrow, const bool (&m)[ROWS],
                                         typename RF<NR>::vec (&R)[ROWS]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int c = 0; c < (NR < MAXCOL ? NR : MAXCOL); ++c) {
    if (c >= a.ncol) break;
    const Col& C = a.col[c];
    const unsigned char* raw = tile_smem + C.raw_off;
    const int kind = C.kind;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      const int r = j * NTHR + tid;
      u64 v = 0;
      if (kind == C_F64 || kind == C_I64) v = reinterpret_cast<const u64*>(raw)[r];
      else if (kind == C_I32) v = (u64)(long long)reinterpret_cast<const int*>(raw)[r];
      else if (kind == C_F32) v = f2u((double)reinterpret_cast<const float*>(raw)[r]);
      else if (kind == C_U8) v = (u64)raw[r];
      else {
        const long long st = reinterpret_cast<const long long*>(raw)[r];
        const long long en = C.contig ? (r + 1 < nrow ? reinterpret_cast<const long long*>(raw)[r + 1]
                                                      : (m[j] ? C.en[row0 + r] : st))
                                      : reinterpret_cast<const long long*>(tile_smem + C.aux_off)[r];
        v = kind == C_SCODE ? (m[j] ? short_code(C.dat, st, en - st, C.L) : 0ull)
                            : (((u64)st << 24) | (u64)min(en - st, 0xFFFFFFll));
      }
      R[j][c] = m[j] ? v : 0ull;
    }
  }
}

template <int NR>
__device__ __forceinline__ u64 operand(const typename RF<NR>::vec& R, int k, long long imm) {
  return k == IMM_REG ? (u64)imm : (k >= 0 ? R[k] : 0ull);
}

// Instructions [lo, hi) of the program over every row slot. The opcode and register numbers are kernel arguments
// (SGPRs): one scalar dispatch per instruction (the next instruction's fields are loaded while this one runs),
// indirect register reads / writes.
template <int NR, int ROWS>
__device__ __forceinline__ void run(const PipeArgs& a, typename RF<NR>::vec (&R)[ROWS], int lo, int hi) {
  if (lo >= hi) return;
  Ins cur = a.ins[lo];
  for (int pc = lo; pc < hi; ++pc) {
    const Ins nxt = a.ins[pc + 1];                     // in bounds: ins has a sentinel after MAXINS
    const int op = cur.op, dst = cur.dst, ia = cur.a, ib = cur.b, ic = cur.c;
    const long long imm = cur.imm;
    u64 x[ROWS], y[ROWS], z[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      x[j] = operand<NR>(R[j], ia, imm);
      y[j] = operand<NR>(R[j], ib, imm);
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
      case OP_RNGF: {                                      // lo <(=) x <(=) hi: imm = lo, kpool[aux] = hi
        const int aux = cur.pad >> 8, mode = aux >> 8;
        const double lo = u2f((u64)imm), hi = u2f((u64)a.kpool[aux & 0xFF]);
        NSDB_EACH((u64)(((mode & 1) ? fx >= lo : fx > lo) && ((mode & 2) ? fx <= hi : fx < hi)))
      }
      case OP_RNGI: {
        const int aux = cur.pad >> 8, mode = aux >> 8;
        const long long lo = imm, hi = a.kpool[aux & 0xFF];
        NSDB_EACH((u64)(((mode & 1) ? sx >= lo : sx > lo) && ((mode & 2) ? sx <= hi : sx < hi)))
      }
      case OP_SEQ:
      case OP_SPRE:
      case OP_SSUF: {                                      // ib: the column whose bytes x refers to
        const unsigned char* d = a.col[ib].dat;
        const int mode = op == OP_SEQ ? 0 : (op == OP_SPRE ? 1 : 2);
#pragma unroll
        for (int j = 0; j < ROWS; ++j) z[j] = str_match(d, x[j], a.lit, imm, mode) ? 1ull : 0ull;
        break;
      }
      case OP_SLIKE: {
        const unsigned char* d = a.col[ib].dat;
#pragma unroll
        for (int j = 0; j < ROWS; ++j) z[j] = str_like(d, x[j], a.lit, imm) ? 1ull : 0ull;
        break;
      }
      default:
#pragma unroll
        for (int j = 0; j < ROWS; ++j) z[j] = 0;
#undef NSDB_EACH
    }
    if (ic >= 0) {                                     // compare folded with the AND of its conjunction
#pragma unroll
      for (int j = 0; j < ROWS; ++j) z[j] = (z[j] != 0 && R[j][ic] != 0) ? 1ull : 0ull;
    }
#pragma unroll
    for (int j = 0; j < ROWS; ++j) R[j][dst] = z[j];
    cur = nxt;
  }
}

template <int F, int NR, int ROWS, bool HYB>
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

  typename RF<NR>::vec R[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) R[j] = (typename RF<NR>::vec)0;
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
    if (HYB) {                                                 // the block's rows: HBM -> LDS -> registers
      const long long nrow = min((long long)NTHR * ROWS, a.n - base);
      __syncthreads();                                         // the previous rows' LDS reads are done
      hyb_dma<NR, ROWS>(a, base, nrow);
      __syncthreads();                                         // every wave's DMA has landed
      hyb_load<NR, ROWS>(a, base, nrow, inr, R);
    } else {
      load_cols<false, NR, ROWS>(a, row, inr, R);              // the predicate's ("early") columns
    }
    run<NR, ROWS>(a, R, 0, a.nins_a);
    bool any = false;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
      keep[j] = inr[j] && (a.keep_reg < 0 || R[j][a.keep_reg] != 0);
      any |= keep[j];
      kept += keep[j] ? 1u : 0u;
    }
    if (!__builtin_amdgcn_ballot_w64(any)) continue;           // no kept row in this wave
    if (!HYB) load_cols<true, NR, ROWS>(a, row, keep, R);     // late columns: the kept rows only
    run<NR, ROWS>(a, R, a.nins_a, a.nins);
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
          const bool ins = !done && s == used;   // selects, not a store at [used]: that form went to scratch
          sk[s] = ins ? key : sk[s];
#pragma unroll
          for (int f = 0; f < F; ++f) sv[s][f] = ins ? v[f] : sv[s][f];
          done = done || ins;
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
// materialised; the engine turns the mask into the stage's row selection). The binding marks every column early.
template <int NR, int ROWS, bool HYB>
__global__ void __launch_bounds__(NTHR) pipe_mask_kernel(const PipeArgs a, unsigned char* __restrict__ mask) {
  typename RF<NR>::vec R[ROWS];
#pragma unroll
  for (int j = 0; j < ROWS; ++j) R[j] = (typename RF<NR>::vec)0;
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
    if (HYB) {
      const long long nrow = min((long long)NTHR * ROWS, a.n - base);
      __syncthreads();
      hyb_dma<NR, ROWS>(a, base, nrow);
      __syncthreads();
      hyb_load<NR, ROWS>(a, base, nrow, inr, R);
    } else {
      load_cols<false, NR, ROWS>(a, row, inr, R);
    }
    run<NR, ROWS>(a, R, 0, a.nins);
#pragma unroll
    for (int j = 0; j < ROWS; ++j)
      if (inr[j]) mask[row[j]] = (unsigned char)(a.keep_reg < 0 ? 1 : (R[j][a.keep_reg] != 0));
  }
}

// ------------------------------------------------------------------------------------------------ tile kernels
// The same programs over LDS-resident column tiles. A workgroup owns tiles of T = 256 * RPT rows: every column's tile
// is copied HBM -> LDS by LDS-DMA (buffer_load ... lds, 16 B per lane, no VGPR staging), so a wave has T x (column
// bytes) in flight per tile instead of a few registers' worth, and the registers of the program live in LDS as
// T-row vectors (register r = rows [r*T, (r+1)*T) of the tile image; 8-byte columns are DMA'd straight into their
// register). Each thread owns rows tid + 256 i of the tile in every instruction, so the program runs with no barrier;
// its operands are ds_read_b64 at the thread's row offsets (conflict-free), its dispatch is amortised over RPT rows
// and it needs no indirect VGPR addressing. Narrow columns (i32 / f32 / u8) and strings are widened into their
// register by the thread that owns the row (string codes gather their bytes from HBM). Several workgroups per CU
// overlap one tile's DMA with another's interpretation.
// Every column's tile (rows [row0, row0 + T)) into its LDS image, then the widening into 8-byte registers for the
// rows this thread owns (after the barrier that makes every wave's DMA visible). A narrow column (i32 / f32 / u8) is
// DMA'd into the top of its own register vector and widened in place: every thread first reads its rows' narrow
// values, a barrier, then writes the widened words (a row's word may cover another row's narrow bytes). A string's
// starts are DMA'd into its register, its ends into an aux vector, or, when starts / ends are one offsets array,
// taken from the next row's start (the tile's last row reads its end from HBM).
template <int RPT>
__device__ __forceinline__ void tile_load(const PipeArgs& a, long long row0, long long nrow, u64* regs) {
  const int T = NTHR * RPT, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool full = nrow == T;
  unsigned char* sm = tile_smem;
  bool narrow = false;
  for (int c = 0; c < a.ncol; ++c) {
    const Col& C = a.col[c];
    if (C.kind == C_SCODE || C.kind == C_SREF) {
      dma_tile(C.st + row0, nrow * 8, sm + C.raw_off, T * 8, 8, full, wave, lane);
      if (!C.contig) dma_tile(C.en + row0, nrow * 8, sm + C.aux_off, T * 8, 8, full, wave, lane);
    } else {
      const int w = kind_width(C.kind);
      narrow |= w < 8;
      dma_tile(reinterpret_cast<const unsigned char*>(C.p) + row0 * w, nrow * w, sm + C.raw_off, T * w, w, full, wave,
               lane);
    }
  }
  __syncthreads();                                     // waits for this wave's DMA; the barrier for everyone's
  if (narrow) {
    for (int c = 0; c < a.ncol; ++c) {
      const int k = a.col[c].kind;
      if (k != C_I32 && k != C_F32 && k != C_U8) continue;
      const unsigned char* raw = sm + a.col[c].raw_off;
      u64 wide[RPT];
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int r = tid + i * NTHR;
        wide[i] = k == C_I32 ? (u64)(long long)reinterpret_cast<const int*>(raw)[r]
                : k == C_F32 ? f2u((double)reinterpret_cast<const float*>(raw)[r])
                : (u64)raw[r];
      }
      __syncthreads();                                 // every narrow value read before any word overwrites it
      u64* R = regs + (long long)c * T;
#pragma unroll
      for (int i = 0; i < RPT; ++i) R[tid + i * NTHR] = wide[i];
    }
  }
  for (int c = 0; c < a.ncol && c < MAXSTR; ++c) {
    const Col& C = a.col[c];
    if (C.kind != C_SCODE && C.kind != C_SREF) continue;
    u64* R = regs + (long long)c * T;
    const long long* en = reinterpret_cast<const long long*>(sm + C.aux_off);
    long long st[RPT], e[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = tid + i * NTHR;
      st[i] = (long long)R[r];
      if (!C.contig)
        e[i] = en[r];
      else
        e[i] = r + 1 < nrow ? (long long)R[r + 1] : (r < nrow ? C.en[row0 + r] : st[i]);
    }
    if (C.contig) __syncthreads();                     // every start read before any is overwritten by a code
    if (C.kind == C_SCODE) {
      u64 code[RPT];
#pragma unroll
      for (int i = 0; i < RPT; ++i)
        code[i] = (tid + i * NTHR < nrow) ? short_code(C.dat, st[i], e[i] - st[i], C.L) : 0ull;
#pragma unroll
      for (int i = 0; i < RPT; ++i) R[tid + i * NTHR] = code[i];
    } else {
#pragma unroll
      for (int i = 0; i < RPT; ++i) R[tid + i * NTHR] = ((u64)st[i] << 24) | (u64)min(e[i] - st[i], 0xFFFFFFll);
    }
  }
}

// The program over the thread's RPT rows of the tile; registers are T-row vectors in LDS.
template <int RPT>
__device__ __forceinline__ void tile_run(const PipeArgs& a, u64* regs, int lo, int hi) {
  const int T = NTHR * RPT, tid = threadIdx.x;
  if (lo >= hi) return;
  // tile mode: the binding pre-decodes every operand into a byte offset of its T-row vector and a flag word
  // (TF_*), so an instruction costs one scalar load of its record, its flag tests and the dispatch
  const unsigned char* base = reinterpret_cast<const unsigned char*>(regs) + tid * 8;
  (void)T;
  for (int pc = lo; pc < hi; ++pc) {
    const Ins cur = a.ins[pc];
    const int op = cur.op, fl = cur.pad;
    const long long imm = cur.imm;
    u64 x[RPT], y[RPT], z[RPT];
    if (fl & (TF_AIMM | TF_ANONE)) {
#pragma unroll
      for (int i = 0; i < RPT; ++i) x[i] = (fl & TF_AIMM) ? (u64)imm : 0ull;
    } else {
#pragma unroll
      for (int i = 0; i < RPT; ++i) x[i] = *reinterpret_cast<const u64*>(base + cur.a + i * NTHR * 8);
    }
    if (fl & (TF_BIMM | TF_BNONE)) {
#pragma unroll
      for (int i = 0; i < RPT; ++i) y[i] = (fl & TF_BIMM) ? (u64)imm : 0ull;
    } else {
#pragma unroll
      for (int i = 0; i < RPT; ++i) y[i] = *reinterpret_cast<const u64*>(base + cur.b + i * NTHR * 8);
    }
    switch (op) {
#define NSDB_EACH(E)                                          \
  _Pragma("unroll") for (int j = 0; j < RPT; ++j) {           \
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
      case OP_SEL: {                                   // imm: the byte offset of the "else" register
#pragma unroll
        for (int j = 0; j < RPT; ++j) z[j] = x[j] ? y[j] : *reinterpret_cast<const u64*>(base + imm + j * NTHR * 8);
        break;
      }
      case OP_RNGF: {
        const int aux = fl >> 8, mode = aux >> 8;
        const double lo = u2f((u64)imm), hi = u2f((u64)a.kpool[aux & 0xFF]);
        NSDB_EACH((u64)(((mode & 1) ? fx >= lo : fx > lo) && ((mode & 2) ? fx <= hi : fx < hi)))
      }
      case OP_RNGI: {
        const int aux = fl >> 8, mode = aux >> 8;
        const long long lo = imm, hi = a.kpool[aux & 0xFF];
        NSDB_EACH((u64)(((mode & 1) ? sx >= lo : sx > lo) && ((mode & 2) ? sx <= hi : sx < hi)))
      }
      case OP_SEQ:
      case OP_SPRE:
      case OP_SSUF: {                                  // b: the column whose bytes x refers to
        const unsigned char* d = a.col[cur.b].dat;
        const int mode = op == OP_SEQ ? 0 : (op == OP_SPRE ? 1 : 2);
#pragma unroll
        for (int j = 0; j < RPT; ++j) z[j] = str_match(d, x[j], a.lit, imm, mode) ? 1ull : 0ull;
        break;
      }
      case OP_SLIKE: {
        const unsigned char* d = a.col[cur.b].dat;
#pragma unroll
        for (int j = 0; j < RPT; ++j) z[j] = str_like(d, x[j], a.lit, imm) ? 1ull : 0ull;
        break;
      }
      default:
#pragma unroll
        for (int j = 0; j < RPT; ++j) z[j] = 0;
#undef NSDB_EACH
    }
    if (fl & TF_C) {
#pragma unroll
      for (int j = 0; j < RPT; ++j)
        z[j] = (z[j] != 0 && *reinterpret_cast<const u64*>(base + cur.c + j * NTHR * 8) != 0) ? 1ull : 0ull;
    }
#pragma unroll
    for (int j = 0; j < RPT; ++j) *reinterpret_cast<u64*>(const_cast<unsigned char*>(base) + cur.dst + j * NTHR * 8) = z[j];
  }
}

template <int F, int RPT>
__global__ void __launch_bounds__(NTHR) tile_agg_kernel(const PipeArgs a) {
  __shared__ long long tk[CAP];
  __shared__ double tv[CAP * F];                     // stride F: the table costs what the stage's values need
  __shared__ int s_ovf;
  __shared__ unsigned long long s_kept;
  constexpr int T = NTHR * RPT;
  constexpr int KS = F <= 6 ? 2 * KSLOT : KSLOT;   // no register file in VGPRs here: room for more register slots
  const int tid = threadIdx.x, lane = tid & 63;
  u64* regs = reinterpret_cast<u64*>(tile_smem);
  const double init = a.agg_op == 0 ? 0.0 : (a.agg_op == 1 ? __builtin_inf() : -__builtin_inf());
  for (int i = tid; i < CAP; i += NTHR) tk[i] = EMPTY;
  for (int i = tid; i < CAP * F; i += NTHR) tv[i] = init;
  if (tid == 0) {
    s_ovf = 0;
    s_kept = 0;
  }
  long long sk[KS];
  double sv[KS][F];
  int used = 0;
  unsigned kept = 0;
  bool ovf = false;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    sk[s] = EMPTY;
#pragma unroll
    for (int f = 0; f < F; ++f) sv[s][f] = init;
  }
  const long long ntiles = (a.n + T - 1) / T;
  for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long long row0 = t * T, nrow = min((long long)T, a.n - row0);
    __syncthreads();                                   // the previous tile's registers are no longer read
    tile_load<RPT>(a, row0, nrow, regs);
    tile_run<RPT>(a, regs, 0, a.nins);
    // every row's keep flag, key and values read first (all LDS reads in flight together), then the slots
    bool kp[RPT];
    long long kk[RPT];
    double vv[RPT][F];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = tid + i * NTHR;
      kp[i] = r < nrow && (a.keep_reg < 0 || regs[(long long)a.keep_reg * T + r] != 0);
      kk[i] = a.key_reg < 0 ? 0 : (long long)regs[(long long)a.key_reg * T + r];
#pragma unroll
      for (int f = 0; f < F; ++f) vv[i][f] = f < a.nval ? u2f(regs[(long long)a.val_reg[f] * T + r]) : 0.0;
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      if (!kp[i]) continue;
      ++kept;
      const long long key = kk[i];
      const double (&v)[F] = vv[i];
      bool done = false;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (!done && s < used && sk[s] == key) {
#pragma unroll
          for (int f = 0; f < F; ++f) sv[s][f] = acc_op(sv[s][f], v[f], a.agg_op);
          done = true;
        }
      }
      if (!done && used < KS) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const bool ins = !done && s == used;   // selects, not a store at [used]: that form went to scratch
          sk[s] = ins ? key : sk[s];
#pragma unroll
          for (int f = 0; f < F; ++f) sv[s][f] = ins ? v[f] : sv[s][f];
          done = done || ins;
        }
        ++used;
      }
      if (!done) ovf |= (key == EMPTY) || !table_insert<F, F>(tk, tv, CAP, key, v, a.nval, a.agg_op);
    }
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
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
      if (lane == leader) ovf |= (kl == EMPTY) || !table_insert<F, F>(tk, tv, CAP, kl, v, a.nval, a.agg_op);
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
    for (int f = 0; f < F; ++f) v[f] = tv[i * F + f];
    if (!table_insert<F>(gk, gv, GCAP, k, v, a.nval, a.agg_op)) s_ovf = 1;
  }
  __syncthreads();
  if (tid == 0) {
    if (s_ovf) atomicOr(a.table, 1ull);
    atomicAdd(a.table + 1, s_kept);
  }
}

template <int RPT>
__global__ void __launch_bounds__(NTHR) tile_mask_kernel(const PipeArgs a, unsigned char* __restrict__ mask) {
  constexpr int T = NTHR * RPT;
  const int tid = threadIdx.x;
  u64* regs = reinterpret_cast<u64*>(tile_smem);
  const long long ntiles = (a.n + T - 1) / T;
  for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long long row0 = t * T, nrow = min((long long)T, a.n - row0);
    __syncthreads();
    tile_load<RPT>(a, row0, nrow, regs);
    tile_run<RPT>(a, regs, 0, a.nins);
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = tid + i * NTHR;
      if (r < nrow) mask[row0 + r] = (unsigned char)(a.keep_reg < 0 ? 1 : (regs[(long long)a.keep_reg * T + r] != 0));
    }
  }
}

// Dynamic LDS above the 64 KiB default needs the kernel's attribute raised (once per shape is enough; it is cheap).
template <int F>
void launch_tile_agg(const PipeArgs& a, int grid, hipStream_t st) {
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              a.lds_bytes);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHR), a.lds_bytes, st, a);
  };
  if (a.tile == 2048)
    go(tile_agg_kernel<F, 8>);
  else if (a.tile == 1024)
    go(tile_agg_kernel<F, 4>);
  else if (a.tile == 768)
    go(tile_agg_kernel<F, 3>);
  else
    go(tile_agg_kernel<F, 2>);
}

void launch_tile_mask(const PipeArgs& a, unsigned char* mask, int grid, hipStream_t st) {
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              a.lds_bytes);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHR), a.lds_bytes, st, a, mask);
  };
  if (a.tile == 2048)
    go(tile_mask_kernel<8>);
  else if (a.tile == 1024)
    go(tile_mask_kernel<4>);
  else if (a.tile == 768)
    go(tile_mask_kernel<3>);
  else
    go(tile_mask_kernel<2>);
}


template <int F>
void launch_agg(const PipeArgs& a, int grid, hipStream_t st) {
  auto go = [&](auto kern) {
    if (a.lds_bytes > 0)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                a.lds_bytes);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHR), a.lds_bytes, st, a);
  };
  if (a.kmode == 2) {
    if (a.nreg <= NREG_SMALL)
      go(pipe_agg_kernel<F, NREG_SMALL, 4, true>);
    else
      go(pipe_agg_kernel<F, NREG, 2, true>);
  } else if (a.nreg <= NREG_SMALL) {
    go(pipe_agg_kernel<F, NREG_SMALL, 4, false>);
  } else {
    go(pipe_agg_kernel<F, NREG, 2, false>);
  }
}

}  // namespace nsdb_pipe

namespace nsdb_pipe {
// Emit regions (jit_emit_body) -> dense columns: workgroup w copies the cnt[w] rows its tile wrote, of every one of
// the ne columns, to dst at off[w] (the exclusive scan of cnt). Reads and writes only the emitted rows.
__global__ void __launch_bounds__(NTHR) emit_compact_kernel(const unsigned long long* __restrict__ src, int ne,
                                                            long long ostride, long long cap,
                                                            const unsigned* __restrict__ cnt,
                                                            const long long* __restrict__ off,
                                                            unsigned long long* __restrict__ dst, long long total) {
  const long long w = blockIdx.x;
  const long long c = cnt[w], o = off[w];
  for (int e = 0; e < ne; ++e)
    for (long long i = threadIdx.x; i < c; i += NTHR) dst[e * total + o + i] = src[e * ostride + w * cap + i];
}
}  // namespace nsdb_pipe

extern "C" {

int nsdb_pipe_emit_compact(const unsigned long long* src, int ne, long long ostride, long long cap, const unsigned* cnt,
                           const long long* off, long long tiles, unsigned long long* dst, long long total,
                           hipStream_t st) {
  if (tiles <= 0 || ne <= 0 || total < 0) return total == 0 ? 0 : -1;
  hipLaunchKernelGGL(nsdb_pipe::emit_compact_kernel, dim3((unsigned)tiles), dim3(nsdb_pipe::NTHR), 0, st, src, ne,
                     ostride, cap, cnt, off, dst, total);
  return (int)hipGetLastError();
}

int nsdb_pipe_sizes(int* out) {
  out[0] = nsdb_pipe::MAXINS;
  out[1] = nsdb_pipe::MAXCOL;
  out[2] = nsdb_pipe::NREG;
  out[3] = nsdb_pipe::FMAX;
  out[4] = nsdb_pipe::CAP;
  out[5] = (int)sizeof(nsdb_pipe::PipeArgs);
  out[6] = nsdb_pipe::MAXSTR;
  out[7] = nsdb_pipe::NTHR;
  out[8] = nsdb_pipe::GCAP;
  out[9] = nsdb_pipe::NREG_SMALL;
  return 0;
}

// args: a host PipeArgs image (the binding fills it field by field and sets nreg = 1 + the highest register the
// program touches, which picks the register-file shape); grid = number of workgroups. Initialises the global
// table, then the fused pass.
int nsdb_pipe_agg(const void* args, int grid, hipStream_t st) {
  if (grid <= 0) return -1;
  const nsdb_pipe::PipeArgs& a = *reinterpret_cast<const nsdb_pipe::PipeArgs*>(args);
  if (a.nins > nsdb_pipe::MAXINS || a.ncol > nsdb_pipe::MAXCOL || a.nval > nsdb_pipe::FMAX || a.nins_a > a.nins ||
      a.table == nullptr || a.nreg < 1 || a.nreg > nsdb_pipe::NREG)
    return -2;
  if (a.kmode == 1 && a.tile != 512 && a.tile != 768 && a.tile != 1024 && a.tile != 2048) return -3;
  if (a.kmode == 2 && a.tile != nsdb_pipe::NTHR * (a.nreg <= nsdb_pipe::NREG_SMALL ? 4 : 2)) return -3;
  hipLaunchKernelGGL(nsdb_pipe::pipe_init_kernel, dim3(nsdb_pipe::GCAP / nsdb_pipe::NTHR), dim3(nsdb_pipe::NTHR), 0, st,
                     a.table, a.agg_op);
  if (a.kmode == 1) {
    if (a.nval <= 2)
      nsdb_pipe::launch_tile_agg<2>(a, grid, st);
    else if (a.nval <= 4)
      nsdb_pipe::launch_tile_agg<4>(a, grid, st);
    else if (a.nval <= 6)
      nsdb_pipe::launch_tile_agg<6>(a, grid, st);
    else
      nsdb_pipe::launch_tile_agg<nsdb_pipe::FMAX>(a, grid, st);
  } else if (a.nval <= 2) {
    nsdb_pipe::launch_agg<2>(a, grid, st);
  } else if (a.nval <= 4) {
    nsdb_pipe::launch_agg<4>(a, grid, st);
  } else if (a.nval <= 6) {
    nsdb_pipe::launch_agg<6>(a, grid, st);
  } else {
    nsdb_pipe::launch_agg<nsdb_pipe::FMAX>(a, grid, st);
  }
  return (int)hipGetLastError();
}

// The global result table's initial state (the run-time compiled aggregation kernels are launched by the binding).
int nsdb_pipe_init(unsigned long long* table, int op, hipStream_t st) {
  if (table == nullptr || op < 0 || op > 2) return -1;
  hipLaunchKernelGGL(nsdb_pipe::pipe_init_kernel, dim3(nsdb_pipe::GCAP / nsdb_pipe::NTHR), dim3(nsdb_pipe::NTHR), 0, st,
                     table, op);
  return (int)hipGetLastError();
}

int nsdb_pipe_mask(const void* args, unsigned char* mask, int grid, hipStream_t st) {
  if (grid <= 0) return -1;
  const nsdb_pipe::PipeArgs& a = *reinterpret_cast<const nsdb_pipe::PipeArgs*>(args);
  if (a.nins > nsdb_pipe::MAXINS || a.ncol > nsdb_pipe::MAXCOL || a.nreg < 1 || a.nreg > nsdb_pipe::NREG) return -2;
  if (a.kmode == 1 && a.tile != 512 && a.tile != 768 && a.tile != 1024 && a.tile != 2048) return -3;
  if (a.kmode == 2 && a.tile != nsdb_pipe::NTHR * (a.nreg <= nsdb_pipe::NREG_SMALL ? 4 : 2)) return -3;
  auto go = [&](auto kern) {
    if (a.lds_bytes > 0)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                a.lds_bytes);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(nsdb_pipe::NTHR), a.lds_bytes, st, a, mask);
  };
  if (a.kmode == 1)
    nsdb_pipe::launch_tile_mask(a, mask, grid, st);
  else if (a.kmode == 2 && a.nreg <= nsdb_pipe::NREG_SMALL)
    go(nsdb_pipe::pipe_mask_kernel<nsdb_pipe::NREG_SMALL, 4, true>);
  else if (a.kmode == 2)
    go(nsdb_pipe::pipe_mask_kernel<nsdb_pipe::NREG, 2, true>);
  else if (a.nreg <= nsdb_pipe::NREG_SMALL)
    go(nsdb_pipe::pipe_mask_kernel<nsdb_pipe::NREG_SMALL, 4, false>);
  else
    go(nsdb_pipe::pipe_mask_kernel<nsdb_pipe::NREG, 2, false>);
  return (int)hipGetLastError();
}

}  // extern "C"
