// PyTorch binding of the fused relational pipeline kernel (pipeline.hip). The program, the column table and the
// aggregation are validated on the host — register / column / literal indices in range, every column on the
// device with at least n rows and the dtype its kind reads — before the argument image is built and launched on
// the current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

extern "C" {
int nsdb_pipe_sizes(int* out);
int nsdb_pipe_agg(const void* args, int grid, hipStream_t st);
int nsdb_pipe_mask(const void* args, unsigned char* mask, int grid, hipStream_t st);
int nsdb_pipe_init(unsigned long long* table, int op, hipStream_t st);
int nsdb_pipe_emit_compact(const unsigned long long* src, int ne, long long ostride, long long cap, const unsigned* cnt,
                           const long long* off, long long tiles, unsigned long long* dst, long long total,
                           hipStream_t st);
}

namespace {

// host mirror of nsdb_pipe::PipeArgs (layout checked against the kernel's sizeof at first use)
constexpr int MAXINS = 48, MAXCOL = 10, FMAX = 8, KPOOL = 16;
struct Ins {
  int op, dst, a, b;
  int c, pad;
  long long imm;
};
struct Col {
  const void* p;
  const long long* st;
  const long long* en;
  const unsigned char* dat;
  int kind, late, L;
  int raw_off, aux_off;
  int contig;
};
struct PipeArgs {
  Ins ins[MAXINS + 1];
  Col col[MAXCOL];
  const unsigned char* lit;
  long long n;
  int nins_a, nins, ncol, keep_reg, key_reg, nval, agg_op, nreg;
  int val_reg[FMAX];
  long long kpool[KPOOL];
  int tile, lds_bytes;
  int kmode, pad2;
  unsigned long long* table;
  const unsigned long long* jtab;
  const long long* jperm;
  unsigned long long jmask;
  long long bn;
  const unsigned long long* jbloom;
  long long jbshift;
};

enum ColKind : int { C_F64 = 0, C_I64, C_I32, C_F32, C_U8, C_SCODE, C_SREF };

// a join table's probe filter (relops join_build's third output; empty: none): W words, one per cap / W home slots
void set_bloom(PipeArgs& a, int64_t cap, const c10::optional<torch::Tensor>& jbloom, const torch::Tensor& tab) {
  a.jbloom = nullptr;
  a.jbshift = 0;
  if (!jbloom.has_value() || !jbloom->defined() || jbloom->numel() == 0) return;
  const int64_t W = jbloom->numel();
  TORCH_CHECK(jbloom->is_cuda() && jbloom->device() == tab.device() && jbloom->scalar_type() == torch::kInt64 &&
                  jbloom->is_contiguous() && W <= cap && (W & (W - 1)) == 0,
              "malformed join probe filter");
  int sh = 0;
  while ((W << sh) < cap) ++sh;
  a.jbloom = reinterpret_cast<const unsigned long long*>(jbloom->data_ptr<int64_t>());
  a.jbshift = sh;
}
enum : int { OP_LTF = 10, OP_NEI = 21, OP_SEQ = 26, OP_SPRE = 27, OP_SSUF = 28, OP_SEL = 29, OP_RNGF = 31, OP_RNGI = 32,
             OP_SLIKE = 33, OP_LAST = 33 };
inline bool is_str_op(int op) { return op == OP_SEQ || op == OP_SPRE || op == OP_SSUF || op == OP_SLIKE; }

int sizes(int i) {
  static int s[10] = {0};
  static bool init = false;
  if (!init) {
    nsdb_pipe_sizes(s);
    init = true;
  }
  return s[i];
}

void check_col(const torch::Tensor& t, int64_t n, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "pipe_agg: ", what, " must be a contiguous device tensor");
  TORCH_CHECK(t.numel() >= n, "pipe_agg: ", what, " has fewer than n rows");
}

// prog: int64 [nins, 6 | 7] (op, dst, a, b, c, imm[, aux]) on the CPU; c >= 0 only on compares (AND with register c);
// aux (range ops): kpool index | mode << 8.
// cols: per column (kind, late, L, data, starts, ends, bytes): data for numeric kinds, starts / ends / bytes for strings.
typedef std::vector<std::tuple<int64_t, int64_t, int64_t, c10::optional<torch::Tensor>, c10::optional<torch::Tensor>,
                               c10::optional<torch::Tensor>, c10::optional<torch::Tensor>>>
    ColList;

// Validate the program / columns / registers and fill the kernel's argument image.
// bn >= 0: a fused join (compiled kernels): columns with late == 2 are build-side columns of bn rows.
void fill_args(PipeArgs& a, const torch::Tensor& prog, int64_t nins_a, const ColList& cols, const torch::Tensor& lit,
               int64_t n, int64_t keep_reg, int64_t key_reg, const std::vector<int64_t>& val_regs, int64_t agg_op,
               const std::vector<int64_t>& kpool, int64_t bn = -1) {
  TORCH_CHECK(sizes(0) == MAXINS && sizes(1) == MAXCOL && sizes(3) == FMAX && sizes(5) == (int)sizeof(PipeArgs) &&
                  sizes(8) > 0 && (sizes(8) & (sizes(8) - 1)) == 0,
              "pipe_agg: host / kernel argument layout mismatch");
  const int NREG = sizes(2);
  TORCH_CHECK(prog.device().is_cpu() && prog.scalar_type() == torch::kInt64 && prog.dim() == 2 &&
                  (prog.size(1) == 6 || prog.size(1) == 7),
              "pipe_agg: prog must be a CPU int64 [nins, 6 | 7] tensor");
  TORCH_CHECK(kpool.size() <= (size_t)KPOOL, "pipe_agg: at most ", KPOOL, " range bounds");
  const int nins = (int)prog.size(0), ncol = (int)cols.size(), nval = (int)val_regs.size();
  TORCH_CHECK(nins <= MAXINS && ncol <= MAXCOL && ncol <= NREG && nval <= FMAX && nval >= 0, "pipe_agg: too large");
  const int MAXSTR = sizes(6);
  TORCH_CHECK(nins_a >= 0 && nins_a <= nins, "pipe_agg: bad nins_a");
  TORCH_CHECK(n >= 0, "pipe_agg: n < 0");
  TORCH_CHECK(agg_op >= 0 && agg_op <= 2, "pipe_agg: agg_op is 0 sum, 1 min, 2 max");
  TORCH_CHECK(keep_reg >= -1 && keep_reg < NREG && key_reg >= -1 && key_reg < NREG, "pipe_agg: bad keep/key reg");
  TORCH_CHECK(lit.is_cuda() && lit.scalar_type() == torch::kUInt8 && lit.is_contiguous(), "pipe_agg: lit");
  std::memset(&a, 0, sizeof(a));
  for (size_t i = 0; i < kpool.size(); ++i) a.kpool[i] = kpool[i];
  const bool has_aux = prog.size(1) == 7;
  auto P = prog.accessor<int64_t, 2>();
  for (int i = 0; i < nins; ++i) {
    Ins& I = a.ins[i];
    I.op = (int)P[i][0];
    I.dst = (int)P[i][1];
    I.a = (int)P[i][2];
    I.b = (int)P[i][3];
    I.c = (int)P[i][4];
    I.imm = P[i][5];
    const int64_t aux = has_aux ? P[i][6] : 0;
    TORCH_CHECK(aux >= 0 && aux < (int64_t(1) << 16), "pipe_agg: bad aux at ", i);
    I.pad = (int)(aux << 8);
    if (I.op == OP_RNGF || I.op == OP_RNGI)
      TORCH_CHECK(I.b == -1 && (aux & 0xFF) < (int64_t)kpool.size() && (aux >> 8) <= 3,
                  "pipe_agg: range op needs b = -1, a pool index and a mode, at ", i);
    TORCH_CHECK(I.op >= 0 && I.op <= OP_LAST, "pipe_agg: bad opcode at ", i);
    TORCH_CHECK(I.dst >= 0 && I.dst < NREG && I.a >= -2 && I.a < NREG && I.b >= -2 && I.b < NREG,
                "pipe_agg: register out of range at ", i);
    TORCH_CHECK(I.c == -1 || (I.c >= 0 && I.c < NREG && ((I.op >= OP_LTF && I.op <= OP_NEI) || I.op == OP_RNGF ||
                                                            I.op == OP_RNGI)),
                "pipe_agg: AND-with register only on compares, at ", i);
    if (I.op == OP_SEL) TORCH_CHECK(I.imm >= 0 && I.imm < NREG, "pipe_agg: select register at ", i);
    a.nreg = std::max({a.nreg, I.dst + 1, I.a + 1, I.b + 1, I.c + 1, I.op == OP_SEL ? (int)I.imm + 1 : 0});
    if (is_str_op(I.op)) {
      TORCH_CHECK(I.b >= 0 && I.b < ncol && std::get<0>(cols[I.b]) == C_SREF, "pipe_agg: string op column at ", i);
      const long long off = I.imm >> 16, len = I.imm & 0xFFFF;
      TORCH_CHECK(off >= 0 && off + len <= lit.numel(), "pipe_agg: literal out of the pool at ", i);
      // [flags][nseg][lens][bytes]: built and checked by the host compiler (pipeline.py Program.like_literal); the
      // pool lives on the device, so only its header size is checked here (no device read per launch)
      if (I.op == OP_SLIKE) TORCH_CHECK(len >= 2, "pipe_agg: LIKE literal header at ", i);
    }
  }
  a.nins = nins;
  a.nins_a = (int)nins_a;
  for (int c = 0; c < ncol; ++c) {
    const auto& t = cols[c];
    Col& C = a.col[c];
    C.kind = (int)std::get<0>(t);
    C.late = (int)std::get<1>(t);
    C.L = (int)std::get<2>(t);
    TORCH_CHECK(C.kind >= C_F64 && C.kind <= C_SREF, "pipe_agg: bad column kind");
    TORCH_CHECK(C.late >= 0 && C.late <= (bn >= 0 ? 2 : 1), "pipe_agg: bad column pass (2 = build side of a join)");
    const int64_t rows = C.late == 2 ? bn : n;       // the rows this column is indexed by
    if (C.kind == C_SCODE || C.kind == C_SREF) {
      TORCH_CHECK(c < MAXSTR, "pipe_agg: string columns must take the first ", MAXSTR, " column slots");
      TORCH_CHECK(std::get<4>(t).has_value() && std::get<5>(t).has_value() && std::get<6>(t).has_value(),
                  "pipe_agg: string column needs starts / ends / bytes");
      const auto &s = *std::get<4>(t), &e = *std::get<5>(t), &d = *std::get<6>(t);
      check_col(s, rows, "starts");
      check_col(e, rows, "ends");
      TORCH_CHECK(s.scalar_type() == torch::kInt64 && e.scalar_type() == torch::kInt64, "pipe_agg: starts/ends int64");
      TORCH_CHECK(d.is_cuda() && d.scalar_type() == torch::kUInt8, "pipe_agg: string bytes must be device uint8");
      TORCH_CHECK(C.kind != C_SCODE || (C.L >= 0 && C.L <= 7), "pipe_agg: short code length bound 0..7");
      C.st = reinterpret_cast<const long long*>(s.data_ptr<int64_t>());
      C.en = reinterpret_cast<const long long*>(e.data_ptr<int64_t>());
      C.contig = C.en == C.st + 1 ? 1 : 0;             // one offsets array: ends are the next rows' starts
      C.dat = d.data_ptr<uint8_t>();
      TORCH_CHECK((reinterpret_cast<uintptr_t>(C.dat) & 3) == 0, "pipe_agg: string bytes must be 4-byte aligned");
    } else {
      TORCH_CHECK(std::get<3>(t).has_value(), "pipe_agg: numeric column needs data");
      const auto& x = *std::get<3>(t);
      check_col(x, rows, "column");
      const auto st = x.scalar_type();
      const bool ok = (C.kind == C_F64 && st == torch::kFloat64) || (C.kind == C_I64 && st == torch::kInt64) ||
                      (C.kind == C_I32 && st == torch::kInt32) || (C.kind == C_F32 && st == torch::kFloat32) ||
                      (C.kind == C_U8 && (st == torch::kUInt8 || st == torch::kBool));
      TORCH_CHECK(ok, "pipe_agg: column dtype does not match its kind");
      C.p = x.data_ptr();
    }
  }
  a.ncol = ncol;
  a.nreg = std::max({a.nreg, ncol, (int)keep_reg + 1, (int)key_reg + 1, 1});
  a.lit = lit.data_ptr<uint8_t>();
  a.n = n;
  a.keep_reg = (int)keep_reg;
  a.key_reg = (int)key_reg;
  a.nval = nval;
  for (int f = 0; f < nval; ++f) {
    TORCH_CHECK(val_regs[f] >= 0 && val_regs[f] < NREG, "pipe_agg: bad value register");
    a.val_reg[f] = (int)val_regs[f];
    a.nreg = std::max(a.nreg, a.val_reg[f] + 1);
  }
  a.agg_op = (int)agg_op;
}

// LDS layout of the tile kernels for tile T: registers [0, nreg) as T x 8-byte vectors. 8-byte columns and string
// starts are DMA'd straight into their register, narrow columns into its top (widened in place), string ends (when
// not the next row's start) into an aux vector after the registers. Returns the dynamic LDS bytes.
int tile_bytes(PipeArgs& a, int T) {
  long long off = (long long)a.nreg * T * 8;
  for (int c = 0; c < a.ncol; ++c) {
    Col& C = a.col[c];
    const int w = (C.kind == C_I32 || C.kind == C_F32) ? 4 : (C.kind == C_U8 ? 1 : 8);
    C.raw_off = c * T * 8 + T * (8 - w);
    C.aux_off = 0;
    if ((C.kind == C_SCODE || C.kind == C_SREF) && !C.contig) {
      C.aux_off = (int)off;
      off += (long long)T * 8;
    }
  }
  return (int)off;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Tile kernels take pre-decoded instructions: every register operand as the byte offset of its T-row vector in
// LDS, immediates / absent operands as flags (pipeline.hip TF_*), the select's register as an offset too.
void predecode_tile(PipeArgs& a) {
  const long long T8 = (long long)a.tile * 8;
  for (int i = 0; i < a.nins; ++i) {
    Ins& I = a.ins[i];
    const bool str = is_str_op(I.op);
    int fl = 0;
    if (I.a == -2) fl |= 1; else if (I.a < 0) fl |= 2; else I.a = (int)(I.a * T8);
    if (str) fl |= 8;                                  // b: the column index of the bytes, not a register
    else if (I.b == -2) fl |= 4; else if (I.b < 0) fl |= 8; else I.b = (int)(I.b * T8);
    if (I.c >= 0) {
      fl |= 16;
      I.c = (int)(I.c * T8);
    }
    if (I.op == OP_SEL) I.imm = I.imm * T8;
    I.dst = (int)(I.dst * T8);
    I.pad = fl | (I.pad & ~0xFF);
  }
}

// Hybrid kernels: the block's NTHR * ROWS rows of every column DMA'd at native width (string ends only when they are
// not the next row's start); registers stay in VGPRs. Returns the dynamic LDS bytes.
int hyb_bytes(PipeArgs& a, int T) {
  long long off = 0;
  for (int c = 0; c < a.ncol; ++c) {
    Col& C = a.col[c];
    const int w = (C.kind == C_I32 || C.kind == C_F32) ? 4 : (C.kind == C_U8 ? 1 : 8);
    C.raw_off = (int)off;
    off += ((long long)T * w + 15) / 16 * 16;
    C.aux_off = 0;
    if ((C.kind == C_SCODE || C.kind == C_SREF) && !C.contig) {
      C.aux_off = (int)off;
      off += (long long)T * 8;
    }
  }
  return (int)off;
}

// Pick the tile kernels' tile size (0: the register kernels): the largest tile whose LDS lets several workgroups
// share a CU, every column 16-byte aligned (the DMA's 16-byte lanes). `force` >= 0 overrides (0 = register kernels).
// mode: -1 hybrid (the default), -2 LDS-tile auto, 0 register kernels, > 0 LDS-tile kernels of that tile size.
void choose_tile(PipeArgs& a, int static_bytes, int64_t force, int reg_static_bytes) {
  a.tile = 0;
  a.lds_bytes = 0;
  a.kmode = 0;
  if (force == 0) return;
  for (int c = 0; c < a.ncol; ++c) {
    const Col& C = a.col[c];
    if ((C.kind == C_SCODE || C.kind == C_SREF) ? !(aligned16(C.st) && (C.contig || aligned16(C.en))) : !aligned16(C.p))
      return;
  }
  if (force == -1) {
    const int T = 256 * (a.nreg <= sizes(9) ? 4 : 2);
    const int b = hyb_bytes(a, T);
    if ((long long)(b + reg_static_bytes) * 2 <= 160 * 1024) {
      a.tile = T;
      a.lds_bytes = b;
      a.kmode = 2;
      for (int c = 0; c < a.ncol; ++c) a.col[c].late = 0;   // every column arrives with the block's DMA
    }
    return;
  }
  const int LDS = 160 * 1024;
  // (tile, workgroups per CU): three workgroups per CU overlap one's DMA with the others' work; then the larger tile
  const int cand[7][2] = {{2048, 3}, {1024, 3}, {768, 3}, {1024, 2}, {768, 2}, {512, 2}, {512, 1}};
  for (const auto& tc : cand) {
    if (force > 0 && tc[0] != force) continue;
    const int b = tile_bytes(a, tc[0]);
    if ((long long)(b + static_bytes) * tc[1] <= LDS) {
      a.tile = tc[0];
      a.lds_bytes = b;
      a.kmode = 1;
      return;
    }
  }
}

// ---- run-time compiled kernels (pipeline_core.h jit_agg_body / jit_mask_body; sources from execution/pipeline.py)
// hiprtc compile of one generated source whose only include is pipeline_core.h (passed as text): the gfx950 code
// object, with the flags of the ahead-of-time kernels (-O3, hardware float atomics).
pybind11::bytes jit_compile(const std::string& src, const std::string& header) {
  hiprtcProgram prog;
  const char* hdr[1] = {header.c_str()};
  const char* names[1] = {"pipeline_core.h"};
  TORCH_CHECK(hiprtcCreateProgram(&prog, src.c_str(), "nsdb_jit.hip", 1, hdr, names) == HIPRTC_SUCCESS,
              "jit_compile: hiprtcCreateProgram failed");
  const char* env = std::getenv("PYTORCH_ROCM_ARCH");
  const std::string arch = std::string("--offload-arch=") + (env && *env ? env : "gfx950");
  const char* opts[] = {arch.c_str(), "-O3", "-std=c++17", "-munsafe-fp-atomics"};
  const hiprtcResult r = hiprtcCompileProgram(prog, 4, opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  std::string log(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    TORCH_CHECK(false, "jit_compile: ", hiprtcGetErrorString(r), "\n", log);
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  std::string code(n, '\0');
  hiprtcGetCode(prog, &code[0]);
  hiprtcDestroyProgram(&prog);
  return pybind11::bytes(code);
}

// hiprtc version ("major.minor"): part of the on-disk code-object cache key, so a toolchain upgrade recompiles.
std::string jit_version() {
  int major = 0, minor = 0;
  hiprtcVersion(&major, &minor);
  return std::to_string(major) + "." + std::to_string(minor);
}

// Load a code object and return the kernel `name` as an opaque handle (modules stay loaded for the process).
int64_t jit_load(const std::string& code, const std::string& name) {
  static std::mutex mu;
  static std::vector<hipModule_t> modules;
  hipModule_t m;
  TORCH_CHECK(hipModuleLoadData(&m, code.data()) == hipSuccess, "jit_load: hipModuleLoadData failed");
  hipFunction_t f;
  TORCH_CHECK(hipModuleGetFunction(&f, m, name.c_str()) == hipSuccess, "jit_load: no kernel ", name);
  std::lock_guard<std::mutex> g(mu);
  modules.push_back(m);
  return reinterpret_cast<int64_t>(f);
}

// Returns the global result table, int64 [2 + GCAP * (1 + FMAX)]: status (overflow flag, kept rows), GCAP keys
// (INT64_MIN = free slot), then GCAP x FMAX f64 values (bit patterns). The host reads it back in one copy.
torch::Tensor pipe_agg(torch::Tensor prog, int64_t nins_a, ColList cols, torch::Tensor lit, int64_t n, int64_t keep_reg,
                       int64_t key_reg, std::vector<int64_t> val_regs, int64_t agg_op, int64_t max_wg, int64_t tile,
                       std::vector<int64_t> kpool, int64_t jit, int64_t jit_nreg, int64_t jit_rows,
                       c10::optional<torch::Tensor> jtab, c10::optional<torch::Tensor> jperm, int64_t bn,
                       c10::optional<torch::Tensor> jbloom) {
  const int ROWS = 4, NTHR = sizes(7), GCAP = sizes(8), CAP = sizes(4);
  PipeArgs a;
  const bool join = jtab.has_value() && jtab->defined();
  fill_args(a, prog, nins_a, cols, lit, n, keep_reg, key_reg, val_regs, agg_op, kpool, join ? bn : -1);
  if (join) {
    // the fused join probe exists in the compiled kernels only; the table is relops join_build's
    TORCH_CHECK(jit != 0, "pipe_agg: a fused join needs its compiled kernel");
    const auto& T = *jtab;
    TORCH_CHECK(T.is_cuda() && T.scalar_type() == torch::kInt64 && T.dim() == 2 && T.size(1) == 2 && T.is_contiguous(),
                "pipe_agg: join table must be join_build's int64 [cap + 1, 2] device tensor");
    const int64_t cap = T.size(0) - 1;
    TORCH_CHECK(cap >= 1024 && (cap & (cap - 1)) == 0, "pipe_agg: malformed join table");
    TORCH_CHECK(jperm.has_value() && jperm->defined() && jperm->is_cuda() && jperm->scalar_type() == torch::kInt64 &&
                    jperm->is_contiguous() && jperm->numel() >= bn && bn >= 0 && bn < (int64_t(1) << 29),
                "pipe_agg: join permutation [build rows] int64 expected");
    TORCH_CHECK(T.device() == lit.device() && jperm->device() == lit.device(), "pipe_agg: join table on another device");
    a.jtab = reinterpret_cast<const unsigned long long*>(T.data_ptr<int64_t>());
    a.jperm = reinterpret_cast<const long long*>(jperm->data_ptr<int64_t>());
    a.jmask = (unsigned long long)(cap - 1);
    a.bn = bn;
    set_bloom(a, cap, jbloom, T);
  }
  if (jit != 0) {                                   // the run-time compiled kernel of exactly this program shape
    TORCH_CHECK(a.nreg == jit_nreg && jit_rows >= 1 && jit_rows <= 16,
                "pipe_agg: compiled kernel for ", jit_nreg, " registers, the program uses ", a.nreg);
    const long long per = (long long)NTHR * jit_rows * 4;
    const int nwg = (int)std::max<long long>(1, std::min<long long>(max_wg > 0 ? max_wg : 2048, (n + per - 1) / per));
    auto table = torch::empty({2 + (long long)GCAP * (1 + FMAX)}, lit.options().dtype(torch::kInt64));
    a.table = reinterpret_cast<unsigned long long*>(table.data_ptr<int64_t>());
    hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    TORCH_CHECK(nsdb_pipe_init(a.table, a.agg_op, st) == 0, "pipe_agg: table init failed");
    void* params[] = {&a};
    TORCH_CHECK(hipModuleLaunchKernel(reinterpret_cast<hipFunction_t>(jit), nwg, 1, 1, NTHR, 1, 1, 0, st, params,
                                      nullptr) == hipSuccess,
                "pipe_agg: compiled kernel launch failed");
    return table;
  }
  const int F = a.nval <= 2 ? 2 : (a.nval <= 4 ? 4 : (a.nval <= 6 ? 6 : FMAX));
  choose_tile(a, CAP * (8 + 8 * F) + 16, tile, CAP * (8 + 8 * FMAX) + 16);
  if (a.kmode == 1) predecode_tile(a);
  // enough workgroups to fill 256 CUs several times over, each still looping over a few tiles / row blocks
  const long long per = a.tile ? (long long)a.tile : (long long)NTHR * ROWS * 4;
  const int nwg = (int)std::max<long long>(1, std::min<long long>(max_wg > 0 ? max_wg : 2048, (n + per - 1) / per));
  auto table = torch::empty({2 + (long long)GCAP * (1 + FMAX)}, lit.options().dtype(torch::kInt64));
  a.table = reinterpret_cast<unsigned long long*>(table.data_ptr<int64_t>());
  const int rc = nsdb_pipe_agg(&a, nwg, c10::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(rc == 0, "pipe_agg launch failed: ", rc);
  return table;
}

// High-cardinality form of a fused stage (pipeline_core.h jit_emit_body, compiled kernels only): every kept (and
// matched) row's ne emitted registers. Workgroup w writes the rows of input tile w into its region of `cap` rows;
// the regions are then compacted into dense columns. Returns (dst int64 [ne, rows], status int64 [2] on the host:
// overflow flag, rows that passed segment A). One host read (the status and the row total together).
std::vector<torch::Tensor> pipe_emit(torch::Tensor prog, int64_t nins_a, ColList cols, torch::Tensor lit, int64_t n,
                                     int64_t keep_reg, int64_t key_reg, std::vector<int64_t> val_regs,
                                     std::vector<int64_t> kpool, int64_t jit, int64_t jit_nreg, int64_t jit_rows,
                                     int64_t ne, int64_t tile_rows, int64_t cap, c10::optional<torch::Tensor> jtab,
                                     c10::optional<torch::Tensor> jperm, int64_t bn, c10::optional<torch::Tensor> jbloom) {
  const int NTHR = sizes(7);
  PipeArgs a;
  const bool join = jtab.has_value() && jtab->defined();
  fill_args(a, prog, nins_a, cols, lit, n, keep_reg, key_reg, val_regs, 0, kpool, join ? bn : -1);
  TORCH_CHECK(jit != 0 && a.nreg == jit_nreg && jit_rows >= 1 && jit_rows <= 16,
              "pipe_emit: needs its compiled kernel (", jit_nreg, " registers, the program uses ", a.nreg, ")");
  TORCH_CHECK(ne >= 1 && ne <= 16, "pipe_emit: 1..16 emitted registers");
  TORCH_CHECK(tile_rows >= NTHR * jit_rows && tile_rows % (NTHR * jit_rows) == 0 && cap >= 1 && cap <= tile_rows * 64,
              "pipe_emit: tile rows must be whole row blocks, cap in [1, 64 * tile rows]");
  if (join) {
    const auto& T = *jtab;
    TORCH_CHECK(T.is_cuda() && T.scalar_type() == torch::kInt64 && T.dim() == 2 && T.size(1) == 2 && T.is_contiguous(),
                "pipe_emit: join table must be join_build's int64 [cap + 1, 2] device tensor");
    const int64_t jcap = T.size(0) - 1;
    TORCH_CHECK(jcap >= 1024 && (jcap & (jcap - 1)) == 0, "pipe_emit: malformed join table");
    TORCH_CHECK(jperm.has_value() && jperm->defined() && jperm->is_cuda() && jperm->scalar_type() == torch::kInt64 &&
                    jperm->is_contiguous() && jperm->numel() >= bn && bn >= 0 && bn < (int64_t(1) << 29),
                "pipe_emit: join permutation [build rows] int64 expected");
    a.jtab = reinterpret_cast<const unsigned long long*>(T.data_ptr<int64_t>());
    a.jperm = reinterpret_cast<const long long*>(jperm->data_ptr<int64_t>());
    a.jmask = (unsigned long long)(jcap - 1);
    a.bn = bn;
    set_bloom(a, jcap, jbloom, T);
  }
  auto i64 = lit.options().dtype(torch::kInt64);
  const int64_t tiles = std::max<int64_t>(1, (n + tile_rows - 1) / tile_rows);
  TORCH_CHECK(tiles < (int64_t(1) << 31), "pipe_emit: too many tiles");
  const int64_t ostride = tiles * cap;
  auto out = torch::empty({ne, ostride}, i64);
  auto cnt = torch::empty({tiles}, lit.options().dtype(torch::kInt32));
  auto status = torch::zeros({2}, i64);
  a.table = reinterpret_cast<unsigned long long*>(status.data_ptr<int64_t>());
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  unsigned long long* op = reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>());
  long long tr = tile_rows, cp = cap, os = ostride;
  unsigned* cp_cnt = reinterpret_cast<unsigned*>(cnt.data_ptr<int>());
  void* params[] = {&a, &op, &tr, &cp, &os, &cp_cnt};
  if (n > 0) {
    TORCH_CHECK(hipModuleLaunchKernel(reinterpret_cast<hipFunction_t>(jit), (unsigned)tiles, 1, 1, NTHR, 1, 1, 0, st,
                                      params, nullptr) == hipSuccess,
                "pipe_emit: compiled kernel launch failed");
  } else {
    cnt.zero_();
  }
  auto incl = torch::cumsum(cnt, 0, torch::kInt64);
  auto head = torch::cat({status, incl.narrow(0, tiles - 1, 1)}).to(torch::kCPU);   // the one host read
  auto hv = head.accessor<int64_t, 1>();
  const int64_t total = hv[2];
  if (hv[0] != 0) return {torch::empty({ne, 0}, i64), head.narrow(0, 0, 2)};
  auto off = incl.sub_(cnt.to(torch::kInt64));
  auto dst = torch::empty({ne, total}, i64);
  if (total > 0)
    TORCH_CHECK(nsdb_pipe_emit_compact(op, (int)ne, ostride, cap, cp_cnt,
                                       reinterpret_cast<const long long*>(off.data_ptr<int64_t>()), tiles,
                                       reinterpret_cast<unsigned long long*>(dst.data_ptr<int64_t>()), total, st) == 0,
                "pipe_emit: compaction launch failed");
  return {dst, head.narrow(0, 0, 2)};
}

// The predicate program's keep flag per row (uint8 [n]); key / values unused.
torch::Tensor pipe_mask(torch::Tensor prog, ColList cols, torch::Tensor lit, int64_t n, int64_t keep_reg, int64_t tile,
                        std::vector<int64_t> kpool, int64_t jit, int64_t jit_nreg, int64_t jit_rows) {
  const int ROWS = 4, NTHR = sizes(7);
  PipeArgs a;
  fill_args(a, prog, prog.size(0), cols, lit, n, keep_reg, -1, {}, 0, kpool);
  for (int c = 0; c < a.ncol; ++c) a.col[c].late = 0;      // the mask pass loads every column up front
  if (jit != 0) {
    TORCH_CHECK(a.nreg == jit_nreg && jit_rows >= 1 && jit_rows <= 16,
                "pipe_mask: compiled kernel for ", jit_nreg, " registers, the program uses ", a.nreg);
    auto mask = torch::empty({n}, lit.options().dtype(torch::kUInt8));
    if (n > 0) {
      const long long per = (long long)NTHR * jit_rows * 4;
      const int nwg = (int)std::max<long long>(1, std::min<long long>(4096, (n + per - 1) / per));
      unsigned char* mp = mask.data_ptr<uint8_t>();
      void* params[] = {&a, &mp};
      TORCH_CHECK(hipModuleLaunchKernel(reinterpret_cast<hipFunction_t>(jit), nwg, 1, 1, NTHR, 1, 1, 0,
                                        c10::hip::getCurrentHIPStream().stream(), params, nullptr) == hipSuccess,
                  "pipe_mask: compiled kernel launch failed");
    }
    return mask;
  }
  choose_tile(a, 0, tile, 0);
  if (a.kmode == 1) predecode_tile(a);
  auto mask = torch::empty({n}, lit.options().dtype(torch::kUInt8));
  if (n > 0) {
    const long long per = a.tile ? (long long)a.tile : (long long)NTHR * ROWS * 4;
    const int nwg = (int)std::max<long long>(1, std::min<long long>(a.tile ? 2048 : 4096, (n + per - 1) / per));
    const int rc = nsdb_pipe_mask(&a, mask.data_ptr<uint8_t>(), nwg, c10::hip::getCurrentHIPStream().stream());
    TORCH_CHECK(rc == 0, "pipe_mask launch failed: ", rc);
  }
  return mask;
}

}  // namespace

void register_pipeline(pybind11::module& m) {
  m.def("pipe_mask", &pipe_mask, "fused filter predicate (pipeline.hip): keep flag per row (uint8)",
        pybind11::arg("prog"), pybind11::arg("cols"), pybind11::arg("lit"), pybind11::arg("n"), pybind11::arg("keep_reg"),
        pybind11::arg("tile") = -1, pybind11::arg("kpool") = std::vector<int64_t>(), pybind11::arg("jit") = 0,
        pybind11::arg("jit_nreg") = 0, pybind11::arg("jit_rows") = 0);
  m.def("pipe_agg", &pipe_agg,
        "fused scan -> filter -> project -> low-cardinality aggregate (pipeline.hip): the global result table "
        "int64 [2 + GCAP * 9] = status (overflow, kept rows), keys, f64 values [GCAP, 8]",
        pybind11::arg("prog"), pybind11::arg("nins_a"), pybind11::arg("cols"), pybind11::arg("lit"), pybind11::arg("n"),
        pybind11::arg("keep_reg"), pybind11::arg("key_reg"), pybind11::arg("val_regs"), pybind11::arg("agg_op") = 0,
        pybind11::arg("max_wg") = 0, pybind11::arg("tile") = -1, pybind11::arg("kpool") = std::vector<int64_t>(),
        pybind11::arg("jit") = 0, pybind11::arg("jit_nreg") = 0, pybind11::arg("jit_rows") = 0,
        pybind11::arg("jtab") = pybind11::none(), pybind11::arg("jperm") = pybind11::none(), pybind11::arg("bn") = -1,
        pybind11::arg("jbloom") = pybind11::none());
  m.def("pipe_emit", &pipe_emit,
        "fused stage, high-cardinality form: every kept (matched) row's emitted registers as dense int64 columns "
        "[ne, rows], and the host status (overflow, rows through segment A)",
        pybind11::arg("prog"), pybind11::arg("nins_a"), pybind11::arg("cols"), pybind11::arg("lit"), pybind11::arg("n"),
        pybind11::arg("keep_reg"), pybind11::arg("key_reg"), pybind11::arg("val_regs"), pybind11::arg("kpool"),
        pybind11::arg("jit"), pybind11::arg("jit_nreg"), pybind11::arg("jit_rows"), pybind11::arg("ne"),
        pybind11::arg("tile_rows"), pybind11::arg("cap"), pybind11::arg("jtab") = pybind11::none(),
        pybind11::arg("jperm") = pybind11::none(), pybind11::arg("bn") = -1, pybind11::arg("jbloom") = pybind11::none());
  m.def("jit_compile", &jit_compile, "hiprtc compile of a generated pipeline kernel source (gfx950 code object)",
        pybind11::arg("src"), pybind11::arg("header"));
  m.def("jit_version", &jit_version, "hiprtc version of the run-time compiler (code-object cache key)");
  m.def("jit_load", &jit_load, "load a code object; the named kernel as an opaque handle for pipe_agg / pipe_mask(jit=)",
        pybind11::arg("code"), pybind11::arg("name"));
}
