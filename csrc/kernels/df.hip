// DataFrame / SQL kernels (gfx950) — the executor-side compute of the Spark workloads.
//
//   expr VM        fused evaluation of a Column expression tree per row (Catalyst codegen's role:
//                  filter predicates, withColumn(when/otherwise), isnan/isNull, arithmetic;
//                  k_means.py:23-51, spark_installation_check.py:37)
//   compaction     predicate mask -> row indices (wave ballot + block prefix) -> row gather (filter)
//   reduce_stats   sum/count/min/max with null and NaN skipping (count(), agg avg; k_means.py:47)
//   hash agg       groupBy().agg(): LDS-resident open-addressing tables with a global overflow
//                  table; radix-partitioned two-pass variant for high-cardinality keys (BASELINE
//                  1B-row groupBy; StringIndexer's label count, k_means.py:34)
//   partition      hash partition ids + counting scatter (shuffle write for RCCL all-to-all-v)
//   histogram      dictionary-code counts (StringIndexer fit)
//
// Tables are sized to powers of two; keys are int64 with EMPTY = INT64_MIN.
#include "common.h"
#include <cstring>
#include <type_traits>

#define EMPTY_KEY ((long long)0x8000000000000000ULL)

PTG_DEV unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

// ================================================================================================
// Expression VM. Program lives in the kernel argument block (wave-uniform -> scalar branches,
// registers stay in VGPRs: every register access is a compile-time-unrolled select).
// ================================================================================================
enum VmOp {
  OP_LDCOL = 1, OP_LDC, OP_LDNULL, OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_MOD, OP_NEG, OP_ABS, OP_SQRT, OP_LOG,
  OP_EXP, OP_POW, OP_FLOOR, OP_CEIL, OP_EQ, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE, OP_AND, OP_OR, OP_NOT,
  OP_ISNULL, OP_ISNOTNULL, OP_ISNAN, OP_SELECT, OP_COALESCE, OP_CAST_INT, OP_EQ_NULLSAFE, OP_MIN2, OP_MAX2,
  OP_ROUND
};
enum ColType { CT_F32 = 0, CT_F64 = 1, CT_I32 = 2, CT_I64 = 3, CT_U8 = 4, CT_CODE = 5 };
#define VM_INS 96
#define VM_COLS 12
#define VM_CONSTS 32
struct VmProg {
  int n_ins, out_reg, out_type, filter_mode;
  int ins[VM_INS];
  double consts[VM_CONSTS];
  const void* cols[VM_COLS];
  const uint8_t* valid[VM_COLS];
  int col_type[VM_COLS];
};

PTG_DEV double rreg(const double (&R)[8], int i) {
  double v = R[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) v = (i == j) ? R[j] : v;
  return v;
}
PTG_DEV void wreg(double (&R)[8], int i, double v) {
#pragma unroll
  for (int j = 0; j < 8; ++j) R[j] = (i == j) ? v : R[j];
}
PTG_DEV double load_col(const void* p, int t, long i, bool& valid) {
  switch (t) {
    case CT_F32: return (double)((const float*)p)[i];
    case CT_F64: return ((const double*)p)[i];
    case CT_I32: return (double)((const int*)p)[i];
    case CT_I64: return (double)((const long long*)p)[i];
    case CT_U8: return (double)((const uint8_t*)p)[i];
    default: { const int c = ((const int*)p)[i]; if (c < 0) valid = false; return (double)c; }
  }
}

__global__ __launch_bounds__(256) void expr_eval_k(VmProg P, long n, void* out, uint8_t* out_valid) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    double R[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned vm = 0;  // validity bit per register
    for (int pc = 0; pc < P.n_ins; ++pc) {
      const int w = P.ins[pc];
      const int op = w & 0xff, d = (w >> 8) & 0xf, a = (w >> 12) & 0xf, b = (w >> 16) & 0xf, c = (w >> 20) & 0xf;
      const int k = (w >> 24) & 0xff;
      const double x = rreg(R, a), y = rreg(R, b);
      const bool va = (vm >> a) & 1, vb = (vm >> b) & 1;
      double r = 0.0; bool v = true;
      switch (op) {
        case OP_LDCOL: { bool ok = true; r = load_col(P.cols[k], P.col_type[k], i, ok);
                         if (P.valid[k]) ok = ok && P.valid[k][i]; v = ok; break; }
        case OP_LDC: r = P.consts[k]; break;
        case OP_LDNULL: v = false; break;
        case OP_ADD: r = x + y; v = va && vb; break;
        case OP_SUB: r = x - y; v = va && vb; break;
        case OP_MUL: r = x * y; v = va && vb; break;
        case OP_DIV: r = x / y; v = va && vb && y != 0.0; break;
        case OP_MOD: r = fmod(x, y); v = va && vb && y != 0.0; break;
        case OP_NEG: r = -x; v = va; break;
        case OP_ABS: r = fabs(x); v = va; break;
        case OP_SQRT: r = sqrt(x); v = va; break;
        case OP_LOG: r = log(x); v = va && x > 0.0; break;
        case OP_EXP: r = exp(x); v = va; break;
        case OP_POW: r = pow(x, y); v = va && vb; break;
        case OP_FLOOR: r = floor(x); v = va; break;
        case OP_CEIL: r = ceil(x); v = va; break;
        case OP_ROUND: r = round(x); v = va; break;
        case OP_EQ: r = (x == y || (isnan(x) && isnan(y))) ? 1.0 : 0.0; v = va && vb; break;
        case OP_NE: r = (x == y || (isnan(x) && isnan(y))) ? 0.0 : 1.0; v = va && vb; break;
        case OP_LT: r = x < y ? 1.0 : 0.0; v = va && vb; break;
        case OP_LE: r = x <= y ? 1.0 : 0.0; v = va && vb; break;
        case OP_GT: r = x > y ? 1.0 : 0.0; v = va && vb; break;
        case OP_GE: r = x >= y ? 1.0 : 0.0; v = va && vb; break;
        case OP_AND: {  // SQL three-valued logic
          const bool fa = va && x == 0.0, fb = vb && y == 0.0;
          if (fa || fb) { r = 0.0; v = true; } else if (va && vb) { r = 1.0; v = true; } else { v = false; }
          break; }
        case OP_OR: {
          const bool ta = va && x != 0.0, tb = vb && y != 0.0;
          if (ta || tb) { r = 1.0; v = true; } else if (va && vb) { r = 0.0; v = true; } else { v = false; }
          break; }
        case OP_NOT: r = x == 0.0 ? 1.0 : 0.0; v = va; break;
        case OP_ISNULL: r = va ? 0.0 : 1.0; break;
        case OP_ISNOTNULL: r = va ? 1.0 : 0.0; break;
        case OP_ISNAN: r = (va && isnan(x)) ? 1.0 : 0.0; break;
        case OP_SELECT: {  // d = (cond a) ? b : c
          const double z = rreg(R, c); const bool vc = (vm >> c) & 1;
          const bool t = va && x != 0.0;
          r = t ? y : z; v = t ? vb : vc; break; }
        case OP_COALESCE: r = va ? x : y; v = va || vb; break;
        case OP_CAST_INT: r = trunc(x); v = va && !isnan(x); break;
        case OP_EQ_NULLSAFE: r = (va && vb) ? (x == y ? 1.0 : 0.0) : ((va == vb) ? 1.0 : 0.0); break;
        case OP_MIN2: r = fmin(x, y); v = va && vb; break;
        case OP_MAX2: r = fmax(x, y); v = va && vb; break;
        default: break;
      }
      wreg(R, d, r);
      vm = v ? (vm | (1u << d)) : (vm & ~(1u << d));
    }
    const double r = rreg(R, P.out_reg);
    const bool v = (vm >> P.out_reg) & 1;
    if (P.filter_mode) {
      ((uint8_t*)out)[i] = (v && r != 0.0) ? 1 : 0;
    } else {
      switch (P.out_type) {
        case CT_F32: ((float*)out)[i] = v ? (float)r : __builtin_nanf(""); break;
        case CT_F64: ((double*)out)[i] = v ? r : __builtin_nan(""); break;
        case CT_I32: ((int*)out)[i] = v ? (int)r : 0; break;
        case CT_I64: ((long long*)out)[i] = v ? (long long)r : 0; break;
        case CT_U8: ((uint8_t*)out)[i] = (v && r != 0.0) ? 1 : 0; break;
        default: ((int*)out)[i] = v ? (int)r : -1; break;
      }
      if (out_valid) out_valid[i] = v ? 1 : 0;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Specialised expression kernels.  The VM above pays a register-select and an opcode dispatch per
// instruction per row (~4 ms for `(v * 4).cast("int")` over 200M rows, far from the 0.5 ms the
// 2.4 GB of traffic needs).  The host matches the hot shapes of a program - one column, one
// constant, at most one arithmetic op, an optional cast to int, or a comparison - and runs them
// here: four rows per thread per iteration, wide loads and stores, the op / cast / comparison
// fixed per launch (uniform branches hoisted out of the element math).  Semantics are the VM's
// exactly (same double arithmetic, same validity rules: a NaN cast is null, x / 0 is never matched).
// ------------------------------------------------------------------------------------------------
enum { AF_NONE = 0, AF_ADD, AF_SUB, AF_MUL, AF_DIV };
enum { AC_NONE = 0, AC_LT, AC_LE, AC_GT, AC_GE, AC_EQ, AC_NE };
struct AffineSpec { int op, cl, cast, cmp, filter; double c; };

template <typename TO>
PTG_DEV TO affine_out(double r, bool v) {
  if constexpr (sizeof(TO) == 1) return (TO)((v && r != 0.0) ? 1 : 0);
  else if constexpr (std::is_same<TO, float>::value) return v ? (float)r : __builtin_nanf("");
  else if constexpr (std::is_same<TO, double>::value) return v ? r : __builtin_nan("");
  else return v ? (TO)r : (TO)0;
}

template <typename TI, typename TO, int OP, int CMP>
PTG_DEV void affine_run(const TI* __restrict__ in, long n, const AffineSpec S, TO* __restrict__ out,
                        uint8_t* __restrict__ valid) {
  auto one = [&](double x, TO& o, uint8_t& vo) {
    double r = x;
    if constexpr (OP == AF_ADD) r = x + S.c;
    else if constexpr (OP == AF_SUB) r = S.cl ? S.c - x : x - S.c;
    else if constexpr (OP == AF_MUL) r = x * S.c;
    else if constexpr (OP == AF_DIV) r = x / S.c;
    bool v = true;
    if (S.cast) { v = !isnan(r); r = trunc(r); }
    if constexpr (CMP != AC_NONE) {
      // (operands are (r, c) or (c, r): cl swaps them)
      const double a = S.cl ? S.c : r, b = S.cl ? r : S.c;
      bool t;
      if constexpr (CMP == AC_LT) t = a < b;
      else if constexpr (CMP == AC_LE) t = a <= b;
      else if constexpr (CMP == AC_GT) t = a > b;
      else if constexpr (CMP == AC_GE) t = a >= b;
      else if constexpr (CMP == AC_EQ) t = a == b || (isnan(a) && isnan(b));
      else t = !(a == b || (isnan(a) && isnan(b)));
      r = t ? 1.0 : 0.0;
    }
    o = affine_out<TO>(r, v);
    vo = v ? 1 : 0;
  };
  const long n4 = n / 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const TI* p = in + 4 * i;
    const TI x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
    TO o[4];
    uint8_t vo[4];
    one((double)x0, o[0], vo[0]);
    one((double)x1, o[1], vo[1]);
    one((double)x2, o[2], vo[2]);
    one((double)x3, o[3], vo[3]);
    TO* q = out + 4 * i;
    q[0] = o[0]; q[1] = o[1]; q[2] = o[2]; q[3] = o[3];
    if (valid) *(uint32_t*)(valid + 4 * i) = vo[0] | (vo[1] << 8) | (vo[2] << 16) | ((uint32_t)vo[3] << 24);
  }
  for (long i = 4 * n4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    TO o;
    uint8_t vo;
    one((double)in[i], o, vo);
    out[i] = o;
    if (valid) valid[i] = vo;
  }
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void expr_affine_k(const TI* __restrict__ in, long n, AffineSpec S,
                                                     TO* __restrict__ out, uint8_t* __restrict__ valid) {
  in = (const TI*)__builtin_assume_aligned(in, 4 * sizeof(TI));
  out = (TO*)__builtin_assume_aligned(out, 4 * sizeof(TO));
  if (S.cmp == AC_NONE) {
    switch (S.op) {
      case AF_ADD: affine_run<TI, TO, AF_ADD, AC_NONE>(in, n, S, out, valid); break;
      case AF_SUB: affine_run<TI, TO, AF_SUB, AC_NONE>(in, n, S, out, valid); break;
      case AF_MUL: affine_run<TI, TO, AF_MUL, AC_NONE>(in, n, S, out, valid); break;
      case AF_DIV: affine_run<TI, TO, AF_DIV, AC_NONE>(in, n, S, out, valid); break;
      default: affine_run<TI, TO, AF_NONE, AC_NONE>(in, n, S, out, valid); break;
    }
  } else {  // comparisons of the (uncast, unop'd) column with the constant
    switch (S.cmp) {
      case AC_LT: affine_run<TI, TO, AF_NONE, AC_LT>(in, n, S, out, valid); break;
      case AC_LE: affine_run<TI, TO, AF_NONE, AC_LE>(in, n, S, out, valid); break;
      case AC_GT: affine_run<TI, TO, AF_NONE, AC_GT>(in, n, S, out, valid); break;
      case AC_GE: affine_run<TI, TO, AF_NONE, AC_GE>(in, n, S, out, valid); break;
      case AC_EQ: affine_run<TI, TO, AF_NONE, AC_EQ>(in, n, S, out, valid); break;
      default: affine_run<TI, TO, AF_NONE, AC_NE>(in, n, S, out, valid); break;
    }
  }
}

// ================================================================================================
// Stream compaction: mask (u8) -> ascending indices of set rows.
// ================================================================================================
#define CPT_ITEMS 16
#define CPT_TILE (256 * CPT_ITEMS)

__global__ __launch_bounds__(256) void compact_count_k(const uint8_t* __restrict__ mask, long n,
                                                       int* __restrict__ block_counts) {
  __shared__ float scr[4];
  const long base = (long)blockIdx.x * CPT_TILE;
  int c = 0;
#pragma unroll
  for (int j = 0; j < CPT_ITEMS; ++j) {
    const long i = base + j * 256 + threadIdx.x;
    c += (i < n && mask[i]) ? 1 : 0;
  }
  const float s = block_sum256((float)c, scr);
  if (threadIdx.x == 0) block_counts[blockIdx.x] = (int)s;
}

// exclusive scan of block counts (single workgroup, any length); total -> total_out
__global__ __launch_bounds__(256) void scan_excl_k(const int* __restrict__ in, long long* __restrict__ out, int nb,
                                                   long long* __restrict__ total_out) {
  __shared__ long long part[256];
  const int per = (nb + 255) / 256;
  const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
  long long s = 0;
  for (int b = b0; b < b1; ++b) s += in[b];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long run = 0;
    for (int t = 0; t < 256; ++t) { const long long v = part[t]; part[t] = run; run += v; }
    *total_out = run;
  }
  __syncthreads();
  long long run = part[threadIdx.x];
  for (int b = b0; b < b1; ++b) { out[b] = run; run += in[b]; }
}

__global__ __launch_bounds__(256) void compact_write_k(const uint8_t* __restrict__ mask, long n,
                                                       const long long* __restrict__ block_off,
                                                       long long* __restrict__ idx_out) {
  __shared__ int wave_tot[4];
  __shared__ int wave_base[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long base = (long)blockIdx.x * CPT_TILE;
  long long run = block_off[blockIdx.x];
  for (int j = 0; j < CPT_ITEMS; ++j) {
    const long i = base + j * 256 + threadIdx.x;
    const bool f = i < n && mask[i];
    const unsigned long long bal = __ballot(f);
    const int pre = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wave_tot[w] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
      int r = 0;
      for (int q = 0; q < 4; ++q) { wave_base[q] = r; r += wave_tot[q]; }
      wave_tot[0] = r;  // reuse slot 0 as the chunk total after bases are read
    }
    __syncthreads();
    if (f) idx_out[run + wave_base[w] + pre] = i;
    run += wave_tot[0];
    __syncthreads();
  }
}

// rows gather: dst[r] = src[idx[r]] for rows of row_bytes (multiple of 4)
__global__ __launch_bounds__(256) void gather_rows_k(const uint8_t* __restrict__ src, const long long* __restrict__ idx,
                                                     long m, int row_words, long nsrc, uint8_t* __restrict__ dst) {
  const long total = m * row_words;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const long r = t / row_words; const int w = t - r * row_words;
    ((uint32_t*)dst)[t] = ((const uint32_t*)src)[PTG_CHECKED_IDX(idx[r], nsrc) * row_words + w];
  }
  (void)nsrc;
}
__global__ __launch_bounds__(256) void gather_bytes_k(const uint8_t* __restrict__ src, const long long* __restrict__ idx,
                                                      long m, int row_bytes, long nsrc, uint8_t* __restrict__ dst) {
  const long total = m * row_bytes;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const long r = t / row_bytes; const int b = t - r * row_bytes;
    dst[t] = src[PTG_CHECKED_IDX(idx[r], nsrc) * row_bytes + b];
  }
  (void)nsrc;
}

// ================================================================================================
// reduce_stats: out[0]=sum, out[1]=count(valid, non-NaN if skip_nan), out[2]=min, out[3]=max,
// out[4]=count of nulls (+NaN when skip_nan)
// ================================================================================================
__global__ __launch_bounds__(256) void reduce_stats_k(const void* __restrict__ col, int type,
                                                      const uint8_t* __restrict__ valid, long n, int skip_nan,
                                                      double* __restrict__ partial) {
  __shared__ double sh[5][256];
  double s = 0, c = 0, mn = INFINITY, mx = -INFINITY, nul = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    bool ok = true;
    const double v = load_col(col, type, i, ok);
    if (valid) ok = ok && valid[i];
    if (ok && skip_nan && isnan(v)) ok = false;
    if (ok) { s += v; c += 1; mn = fmin(mn, v); mx = fmax(mx, v); } else { nul += 1; }
  }
  sh[0][threadIdx.x] = s; sh[1][threadIdx.x] = c; sh[2][threadIdx.x] = mn; sh[3][threadIdx.x] = mx;
  sh[4][threadIdx.x] = nul;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + o]; sh[1][threadIdx.x] += sh[1][threadIdx.x + o];
      sh[2][threadIdx.x] = fmin(sh[2][threadIdx.x], sh[2][threadIdx.x + o]);
      sh[3][threadIdx.x] = fmax(sh[3][threadIdx.x], sh[3][threadIdx.x + o]);
      sh[4][threadIdx.x] += sh[4][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x < 5) partial[blockIdx.x * 5 + threadIdx.x] = sh[threadIdx.x][0];
}
__global__ void reduce_stats_final_k(const double* __restrict__ partial, int nb, double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0, c = 0, mn = INFINITY, mx = -INFINITY, nul = 0;
  for (int b = 0; b < nb; ++b) {
    s += partial[b * 5]; c += partial[b * 5 + 1]; mn = fmin(mn, partial[b * 5 + 2]);
    mx = fmax(mx, partial[b * 5 + 3]); nul += partial[b * 5 + 4];
  }
  out[0] = s; out[1] = c; out[2] = mn; out[3] = mx; out[4] = nul;
}

// ================================================================================================
// Hash aggregation.  Aggregates are "slots": for every input value column j we keep
// sum[j], cnt[j] (non-null count), min[j], max[j] (doubles) per group, plus rows (count(*)).
// Global table layout (capacity cap, power of two):
//   keys[cap] (i64), rows[cap] (f64), then per value column j: sum, cnt, min, max  [4*nv][cap] (f64)
// ================================================================================================
#define AGG_MAXV 4
struct AggIn {
  const void* vals[AGG_MAXV];
  const uint8_t* valid[AGG_MAXV];
  int types[AGG_MAXV];
  int nv;
  int minmax;  // also maintain min/max (global-table path for every row)
};

PTG_DEV void atomic_min_f64(double* p, double v) {
  unsigned long long* a = (unsigned long long*)p;
  unsigned long long old = *a;
  while (__longlong_as_double(old) > v) {
    const unsigned long long prev = atomicCAS(a, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}
PTG_DEV void atomic_max_f64(double* p, double v) {
  unsigned long long* a = (unsigned long long*)p;
  unsigned long long old = *a;
  while (__longlong_as_double(old) < v) {
    const unsigned long long prev = atomicCAS(a, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}

// find-or-insert slot in the global table; returns -1 if the table is full
PTG_DEV long gtable_slot(long long* keys, long cap, long long key) {
  long h = (long)(mix64((unsigned long long)key) & (unsigned long long)(cap - 1));
  for (long probe = 0; probe < cap; ++probe) {
    const long long cur = keys[h];
    if (cur == key) return h;
    if (cur == EMPTY_KEY) {
      const long long prev = (long long)atomicCAS((unsigned long long*)&keys[h], (unsigned long long)EMPTY_KEY,
                                                  (unsigned long long)key);
      if (prev == EMPTY_KEY || prev == key) return h;
    }
    h = (h + 1) & (cap - 1);
  }
  return -1;
}

PTG_DEV void gtable_add(double* tab, long cap, long slot, double rows, const double* s, const double* c,
                        const double* mn, const double* mx, int nv) {
  atomicAdd(&tab[slot], rows);
  for (int j = 0; j < nv; ++j) {
    double* base = tab + cap * (1 + 4 * j);
    if (c[j] > 0) {
      atomicAdd(&base[slot], s[j]);
      atomicAdd(&base[cap + slot], c[j]);
      atomic_min_f64(&base[2 * cap + slot], mn[j]);
      atomic_max_f64(&base[3 * cap + slot], mx[j]);
    }
  }
}

// LDS-first aggregation: each workgroup aggregates a contiguous chunk of rows into an LDS table
// (lcap slots, a power of two sized by the host to ~2x the expected keys: at 1K sparse keys the old
// fixed 1024-slot table ran at load ~1, its probe chains hit the limit and rows spilled to global
// atomics - 41.6 ms per 1B rows), overflowing rows go straight to the global table; the LDS table is
// flushed with one global update per distinct key per workgroup.  Low/moderate cardinality =>
// global atomics drop by the per-chunk reuse factor.  Dynamic LDS: keys i64[lcap], sums
// f64[nv][lcap], rows u32[lcap], non-null counts u32[nv][lcap] (rows_per_block < 2^32).
__global__ __launch_bounds__(256) void hash_agg_lds_k(const long long* __restrict__ keys, long n, AggIn in,
                                                      long long* __restrict__ gkeys, double* __restrict__ gtab,
                                                      long gcap, long rows_per_block, int* __restrict__ overflow,
                                                      int lcap) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const int nvl = in.nv;
  long long* lk = (long long*)lds_raw;
  double* lsum = (double*)(lk + lcap);                    // [nv][lcap]
  unsigned int* lrows = (unsigned int*)(lsum + (long)nvl * lcap);
  unsigned int* lcnt = lrows + lcap;                      // [nv][lcap]
  const int lmask = lcap - 1;
  for (int t = threadIdx.x; t < lcap; t += 256) {
    lk[t] = EMPTY_KEY; lrows[t] = 0;
    for (int j = 0; j < nvl; ++j) { lsum[j * lcap + t] = 0.0; lcnt[j * lcap + t] = 0; }
  }
  __syncthreads();
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(n, r0 + rows_per_block);
  const bool need_minmax = in.minmax != 0;
  auto load_row = [&](long i, long long& key, double* s, double* c) {
    key = keys[i];
    for (int j = 0; j < in.nv; ++j) {
      bool ok = true;
      const double v = load_col(in.vals[j], in.types[j], i, ok);
      if (in.valid[j]) ok = ok && in.valid[j][i];
      if (ok && isnan(v)) ok = false;
      s[j] = ok ? v : 0.0; c[j] = ok ? 1.0 : 0.0;
    }
  };
  auto add_row = [&](long long key, const double* s, const double* c) {
    int h = (int)(mix64((unsigned long long)key) & (unsigned long long)lmask);
    int slot = -1;
    for (int probe = 0; probe < 32; ++probe) {
      const long long cur = lk[h];
      if (cur == key) { slot = h; break; }
      if (cur == EMPTY_KEY) {
        const long long prev = (long long)atomicCAS((unsigned long long*)&lk[h], (unsigned long long)EMPTY_KEY,
                                                    (unsigned long long)key);
        if (prev == EMPTY_KEY || prev == key) { slot = h; break; }
      }
      h = (h + 1) & lmask;
    }
    if (slot >= 0) {
      atomicAdd(&lrows[slot], 1u);
      for (int j = 0; j < nvl; ++j) {
        if (c[j] > 0) { atomicAdd(&lsum[j * lcap + slot], s[j]); atomicAdd(&lcnt[j * lcap + slot], 1u); }
      }
    }
    if (slot < 0 || need_minmax) {
      const long gs = gtable_slot(gkeys, gcap, key);
      if (gs < 0) { atomicAdd(overflow, 1); return; }
      if (slot < 0) {
        gtable_add(gtab, gcap, gs, 1.0, s, c, s, s, in.nv);
      } else {
        for (int j = 0; j < in.nv; ++j)
          if (c[j] > 0) {
            double* base = gtab + gcap * (1 + 4 * j);
            atomic_min_f64(&base[2 * gcap + gs], s[j]);
            atomic_max_f64(&base[3 * gcap + gs], s[j]);
          }
      }
    }
  };
  // 4 rows' loads in flight per thread ahead of the LDS probes (one row at a time left every load
  // exposed: 51 ms per 1B rows at 1K keys)
  long i = r0 + threadIdx.x;
  for (; i + 3 * 256 < r1; i += 4 * 256) {
    long long k4[4];
    double s4[4][AGG_MAXV], c4[4][AGG_MAXV];
#pragma unroll
    for (int u = 0; u < 4; ++u) load_row(i + u * 256, k4[u], s4[u], c4[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) add_row(k4[u], s4[u], c4[u]);
  }
  for (; i < r1; i += 256) {
    long long key;
    double s1[AGG_MAXV], c1[AGG_MAXV];
    load_row(i, key, s1, c1);
    add_row(key, s1, c1);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < lcap; t += 256) {
    const long long key = lk[t];
    if (key == EMPTY_KEY) continue;
    const long gs = gtable_slot(gkeys, gcap, key);
    if (gs < 0) { atomicAdd(overflow, 1); continue; }
    atomicAdd(&gtab[gs], (double)lrows[t]);
    for (int j = 0; j < nvl; ++j) {
      double* base = gtab + gcap * (1 + 4 * j);
      if (lcnt[j * lcap + t] > 0) {
        atomicAdd(&base[gs], lsum[j * lcap + t]);
        atomicAdd(&base[gcap + gs], (double)lcnt[j * lcap + t]);
      }
    }
  }
}

// table init: keys EMPTY, rows/sum/cnt 0, min +inf, max -inf
__global__ __launch_bounds__(256) void hash_table_init_k(long long* keys, double* tab, long cap, int nv) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < cap; i += (long)gridDim.x * 256) {
    keys[i] = EMPTY_KEY;
    tab[i] = 0.0;
    for (int j = 0; j < nv; ++j) {
      double* base = tab + cap * (1 + 4 * j);
      base[i] = 0.0; base[cap + i] = 0.0; base[2 * cap + i] = INFINITY; base[3 * cap + i] = -INFINITY;
    }
  }
}

// extract occupied slots into dense outputs: out_keys[m], out_tab[(1+4nv)][m]; count -> *m_out
__global__ __launch_bounds__(256) void hash_extract_k(const long long* __restrict__ keys, const double* __restrict__ tab,
                                                      long cap, int nv, long long* __restrict__ out_keys,
                                                      double* __restrict__ out_tab, long out_cap,
                                                      unsigned long long* __restrict__ m_out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < cap; i += (long)gridDim.x * 256) {
    const long long k = keys[i];
    if (k == EMPTY_KEY) continue;
    const unsigned long long p = atomicAdd(m_out, 1ULL);
    if ((long)p >= out_cap) continue;
    out_keys[p] = k;
    for (int s = 0; s < 1 + 4 * nv; ++s) out_tab[s * out_cap + p] = tab[s * cap + i];
  }
}

// ---- radix-partitioned aggregation (high cardinality) -------------------------------------------
// Recursive hash partitioning (the classic out-of-cache aggregation plan), LDS-staged:
//   level l (l = 0, 1, ...) splits every segment by 6 more hash bits (mix64(key) >> (58 - 6l)):
//   a tile of RT rows is counting-sorted by digit in LDS and written as 64 contiguous runs
//   (element-granular scatter is uncoalesced, cdna_hip_programming.md App. B "Scatter"), run
//   offsets come from one exclusive scan over per-tile digit counts laid out [segment][digit][tile].
//   Rows carry their key and up to PAY_MAX value columns, converted to f64 on the first level with
//   null -> NaN (aggregates skip NaN and null alike, as hash_agg_lds_k does).
//   part_agg2_k then gives every partition one workgroup and one LDS open-addressing table; a
//   partition whose distinct keys do not fit its table SPILLS (emits nothing, is listed in
//   `spilled`) and the host re-partitions only the spilled segments one level deeper.  mix64 is a
//   bijection, so partitions shrink to single keys after at most 64/6 levels: the recursion is
//   exact at any cardinality, with no global overflow table and no lost rows.
#ifndef PTG_RT
#define PTG_RT 4096
#endif
#define RT PTG_RT  // max rows per tile; radix_scatter_k<NV> uses RT (NV <= 1) or RT/2 (LDS budget)
#define RB 64
#define PAY_MAX 4
struct PayIn {  // value columns of a partitioning pass (first level: any type + validity)
  const void* vals[PAY_MAX];
  const uint8_t* valid[PAY_MAX];
  int types[PAY_MAX];
};
struct PayOut {
  double* vals[PAY_MAX];
};
PTG_DEV double load_pay(const PayIn& in, int j, long i) {
  bool ok = true;
  const double v = load_col(in.vals[j], in.types[j], i, ok);
  if (in.valid[j]) ok = ok && in.valid[j][i];
  return ok ? v : __builtin_nan("");
}

// XCD-aware tile order for the scatter passes: the dispatcher deals consecutive workgroups round-
// robin to the 8 XCDs, each with its own L2.  A digit's runs from consecutive tiles are adjacent in
// the output, so a short run (16-32 rows at 256 bins) shares its first / last cache line with the
// neighbouring tiles' runs; mapping workgroup b to tile xcd_tile(b) gives every XCD a contiguous
// range of tiles, so those partial lines are completed in ONE L2 instead of being written partially
// from several (cdna_hip_programming.md: XCD-aware blockIdx mapping).  A bijection on [0, ntiles).
#ifndef PTG_XCD_TILES
#define PTG_XCD_TILES 1
#endif
PTG_DEV int xcd_tile(int b, int ntiles) {
#if PTG_XCD_TILES
  const int q = ntiles >> 3, r = ntiles & 7, x = b & 7, i = b >> 3;
  return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
#else
  (void)ntiles;
  return b;
#endif
}

// Keys travel as i64, or — when the first level finds max - min < 2^32 - 1 — as u32 offsets from
// kbase = min (12 instead of 16 bytes per row through every later pass; the 1B-row / 1M-key
// groupBy moves 21 % fewer bytes).  Digits always hash the ORIGINAL key, mix64(kbase + offset),
// so the partitioning does not depend on the storage width.
template <class KT>
PTG_DEV unsigned long long orig_key(KT k, long long kbase) {
  if constexpr (sizeof(KT) == 4) return (unsigned long long)(kbase + (long long)(unsigned int)k);
  else return (unsigned long long)k;
}

// range (level 1 only, optional): per-tile [min, max] of the i64 keys, [ntiles][2]
template <class KT>
__global__ __launch_bounds__(256) void radix_count_k(const KT* __restrict__ keys, long long kbase,
                                                     const long long* __restrict__ tstart,
                                                     const int* __restrict__ trows,
                                                     const long long* __restrict__ thbase,
                                                     const long long* __restrict__ thstride, int shift,
                                                     unsigned int* __restrict__ hist, long long* __restrict__ range) {
  // All RT/256 keys of a thread are loaded before the first LDS atomic (independent loads in
  // flight instead of a load->atomic chain per row), and each wave counts into its own 64-bin
  // histogram so the 4 waves never contend on a bin; trows <= RT by construction (_radix_level).
  constexpr int RPT = RT / 256;
  __shared__ unsigned int h[4][RB];
  const int tid = threadIdx.x, b = blockIdx.x, w = tid >> 6;
  h[w][tid & (RB - 1)] = 0;
  const long long s0 = tstart[b];
  const int nr = trows[b];
  unsigned long long k[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * 256;
    k[j] = i < nr ? orig_key<KT>(keys[s0 + i], kbase) : 0ull;
  }
  if (range) {  // per-tile [min, max] (no contended global atomics): the host reduces the tile pairs
    __shared__ long long rmn[4], rmx[4];
    long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000ULL;
#pragma unroll
    for (int j = 0; j < RPT; ++j)
      if (tid + j * 256 < nr) {
        const long long v = (long long)k[j];
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const long long a = __shfl_xor(mn, o, 64), c = __shfl_xor(mx, o, 64);
      mn = a < mn ? a : mn;
      mx = c > mx ? c : mx;
    }
    if ((tid & 63) == 0) { rmn[w] = mn; rmx[w] = mx; }
    __syncthreads();
    if (tid == 0) {
      long long a = rmn[0], c = rmx[0];
      for (int q = 1; q < 4; ++q) { a = rmn[q] < a ? rmn[q] : a; c = rmx[q] > c ? rmx[q] : c; }
      range[2 * b] = a;
      range[2 * b + 1] = c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (tid + j * 256 < nr) atomicAdd(&h[w][(unsigned)(mix64(k[j]) >> shift) & (RB - 1)], 1u);
  __syncthreads();
  if (tid < RB) hist[thbase[b] + (long long)tid * thstride[b]] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

#ifndef PTG_SCATTER_NT
#define PTG_SCATTER_NT 512
#endif
// NT threads per tile-workgroup (each holds RPT rows in registers): 512 threads keep the same
// waves per CU as two 256-thread tiles while each tile (and so each digit run) is twice as long.
template <int NV, class KIN, class KOUT, int NT = PTG_SCATTER_NT>
__global__ __launch_bounds__(NT) void radix_scatter_k(const KIN* __restrict__ keys, long long kbase_in, PayIn pin,
                                                       const long long* __restrict__ tstart,
                                                       const int* __restrict__ trows,
                                                       const long long* __restrict__ thbase,
                                                       const long long* __restrict__ thstride, int shift,
                                                       const long long* __restrict__ offs, long n_out,
                                                       KOUT* __restrict__ okeys, long long kbase_out, PayOut pout) {
  (void)n_out;
  constexpr int RTT = NV <= 1 ? RT : RT / 2;  // tile rows (ops/df.py radix_tile mirrors this)
  constexpr int RPT = RTT / NT;
  static_assert(RPT >= 1 && RTT % NT == 0, "tile rows must be a multiple of the thread count");
  constexpr int NVS = NV > 0 ? NV : 1;
  __shared__ KOUT sk[RTT];
  __shared__ double sv[NVS][RTT];
  __shared__ unsigned char sd[RTT];
  __shared__ unsigned int cnt[RB];
  __shared__ unsigned int lstart[RB];
  __shared__ long long goff[RB];
  const int tid = threadIdx.x, b = xcd_tile(blockIdx.x, gridDim.x);
  const long long s0 = tstart[b];
  const int nr = trows[b];
  if (tid < RB) {
    cnt[tid] = 0;
    goff[tid] = offs[thbase[b] + (long long)tid * thstride[b]];
  }
  __syncthreads();
  unsigned long long k[RPT];
  double v[NVS][RPT];
  int d[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * NT;
    d[j] = -1;
    if (i < nr) {
      k[j] = orig_key<KIN>(keys[s0 + i], kbase_in);
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q][j] = load_pay(pin, q, s0 + i);
      d[j] = (int)((mix64(k[j]) >> shift) & (RB - 1));
      atomicAdd(&cnt[d[j]], 1u);
    }
  }
  __syncthreads();
  if (tid < RB) {  // exclusive scan of the 64 digit counts within one wave
    const unsigned c = cnt[tid];
    unsigned incl = c;
#pragma unroll
    for (int o = 1; o < RB; o <<= 1) {
      const unsigned t = __shfl_up(incl, o, 64);
      if (tid >= o) incl += t;
    }
    lstart[tid] = incl - c;
    cnt[tid] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    if (d[j] < 0) continue;
    const unsigned pos = lstart[d[j]] + atomicAdd(&cnt[d[j]], 1u);
    if constexpr (sizeof(KOUT) == 4) sk[pos] = (KOUT)(unsigned int)((long long)k[j] - kbase_out);
    else sk[pos] = (KOUT)k[j];
#pragma unroll
    for (int q = 0; q < NV; ++q) sv[q][pos] = v[q][j];
    sd[pos] = (unsigned char)d[j];
  }
  __syncthreads();
  for (int i = tid; i < nr; i += NT) {  // consecutive rows of a digit run -> consecutive addresses
    const int dd = sd[i];
    const long long dst = PTG_CHECKED_IDX(goff[dd] + (i - (int)lstart[dd]), n_out);
#if PTG_NT_STORE  // streamed once, re-read only by the next pass
    __builtin_nontemporal_store(sk[i], &okeys[dst]);
#pragma unroll
    for (int q = 0; q < NV; ++q) __builtin_nontemporal_store(sv[q][i], &pout.vals[q][dst]);
#else
    okeys[dst] = sk[i];
#pragma unroll
    for (int q = 0; q < NV; ++q) pout.vals[q][dst] = sv[q][i];
#endif
  }
}

// Block-wide exclusive scan of one int per thread (256 threads); returns the total in *total.
PTG_DEV int block_excl_scan256(int c, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int base = 0;
  for (int q = 0; q < w; ++q) base += wsum[q];
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  return base + incl - c;
}

PTG_DEV void lds_min_f64(double* p, double v) {
  unsigned long long* a = (unsigned long long*)p;
  unsigned long long old = *a;
  while (__longlong_as_double(old) > v) {
    const unsigned long long prev = atomicCAS(a, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}
PTG_DEV void lds_max_f64(double* p, double v) {
  unsigned long long* a = (unsigned long long*)p;
  unsigned long long old = *a;
  while (__longlong_as_double(old) < v) {
    const unsigned long long prev = atomicCAS(a, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}

struct AggPay {
  const double* vals[PAY_MAX];
};

// One workgroup per partition (grid-stride over partitions), LDS table of `pcap` slots (power of
// two) laid out [keys i64][sum (, min, max) f64 per column][rows u32][cnt u32 per column] in dynamic
// LDS.  Output (non-spilled partitions): keys + table rows [rows, (sum, cnt, min, max) per column]
// in hash_extract_k's layout, one atomic per partition for the output base.  Every thread keeps 4
// rows' key + value loads in flight ahead of its LDS probes.
template <int NV, bool MINMAX, class KT>
__global__ __launch_bounds__(256) void part_agg2_k(const KT* __restrict__ okeys, long long kbase, AggPay pay,
                                                   const long long* __restrict__ pstart,
                                                   const long long* __restrict__ pend, int P, int pcap,
                                                   long long* __restrict__ out_keys, double* __restrict__ out_tab,
                                                   long out_cap, unsigned long long* __restrict__ m_out,
                                                   int* __restrict__ spilled, int* __restrict__ nspill) {
  constexpr int NACC = MINMAX ? 3 : 1;  // f64 accumulators per column
  constexpr int NVS = NV > 0 ? NV : 1;
  extern __shared__ __align__(16) unsigned char lds_raw[];
  __shared__ volatile int sflag;
  __shared__ int wsum[4];
  __shared__ unsigned long long obase;
  const int mask = pcap - 1;
  long long* lk = (long long*)lds_raw;
  double* lf = (double*)(lk + pcap);                       // [NV][NACC][pcap]
  unsigned int* lrows = (unsigned int*)(lf + (long)NV * NACC * pcap);
  unsigned int* lcnt = lrows + pcap;                        // [NV][pcap]
  auto insert = [&](long long key, const double* v) -> bool {
    int h = (int)(mix64((unsigned long long)key) & (unsigned long long)mask);
    int slot = -1;
    for (int probe = 0; probe < 64; ++probe) {
      const long long cur = lk[h];
      if (cur == key) { slot = h; break; }
      if (cur == EMPTY_KEY) {
        const long long prev = (long long)atomicCAS((unsigned long long*)&lk[h], (unsigned long long)EMPTY_KEY,
                                                    (unsigned long long)key);
        if (prev == EMPTY_KEY || prev == key) { slot = h; break; }
      }
      h = (h + 1) & mask;
    }
    if (slot < 0) return false;
    atomicAdd(&lrows[slot], 1u);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      if (v[j] != v[j]) continue;  // null / NaN
      atomicAdd(&lf[(j * NACC) * pcap + slot], v[j]);
      atomicAdd(&lcnt[j * pcap + slot], 1u);
      if (MINMAX) {
        lds_min_f64(&lf[(j * NACC + 1) * pcap + slot], v[j]);
        lds_max_f64(&lf[(j * NACC + 2) * pcap + slot], v[j]);
      }
    }
    return true;
  };
  for (int p = blockIdx.x; p < P; p += gridDim.x) {
    for (int t = threadIdx.x; t < pcap; t += 256) {
      lk[t] = EMPTY_KEY;
      lrows[t] = 0;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        lf[(j * NACC) * pcap + t] = 0.0;
        if (MINMAX) { lf[(j * NACC + 1) * pcap + t] = INFINITY; lf[(j * NACC + 2) * pcap + t] = -INFINITY; }
        lcnt[j * pcap + t] = 0;
      }
    }
    if (threadIdx.x == 0) sflag = 0;
    __syncthreads();
    const long long a = pstart[p], b = pend[p];
    long long i = a + threadIdx.x;
    bool ok = true;
    for (; ok && i + 3 * 256 < b; i += 4 * 256) {
      long long k4[4];
      double v4[4][NVS];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        k4[u] = (long long)orig_key<KT>(okeys[i + u * 256], kbase);
#pragma unroll
        for (int j = 0; j < NV; ++j) v4[u][j] = pay.vals[j][i + u * 256];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) ok = ok && insert(k4[u], v4[u]);
      if (sflag) ok = false;  // benign race: a spilled partition's rows are re-partitioned anyway
    }
    for (; ok && i < b; i += 256) {
      double v1[NVS];
#pragma unroll
      for (int j = 0; j < NV; ++j) v1[j] = pay.vals[j][i];
      ok = insert((long long)orig_key<KT>(okeys[i], kbase), v1);
    }
    if (!ok) sflag = 1;
    __syncthreads();
    if (sflag) {
      if (threadIdx.x == 0) spilled[atomicAdd(nspill, 1)] = p;
      __syncthreads();
      continue;
    }
    // compact the occupied slots: each thread owns pcap/256 consecutive slots
    const int per = pcap >> 8;
    const int s0 = threadIdx.x * per;
    int c = 0;
    for (int s = s0; s < s0 + per; ++s) c += lk[s] != EMPTY_KEY;
    int total;
    const int pre = block_excl_scan256(c, wsum, &total);
    if (threadIdx.x == 0) obase = total ? atomicAdd(m_out, (unsigned long long)total) : 0ull;
    __syncthreads();
    long long q = (long long)obase + pre;
    for (int s = s0; s < s0 + per; ++s) {
      const long long key = lk[s];
      if (key == EMPTY_KEY) continue;
      if (q < out_cap) {
        out_keys[q] = key;
        out_tab[q] = (double)lrows[s];
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          double* o = out_tab + out_cap * (1 + 4 * j);
          o[q] = lf[(j * NACC) * pcap + s];
          o[out_cap + q] = (double)lcnt[j * pcap + s];
          o[2 * out_cap + q] = MINMAX ? lf[(j * NACC + 1) * pcap + s] : INFINITY;
          o[3 * out_cap + q] = MINMAX ? lf[(j * NACC + 2) * pcap + s] : -INFINITY;
        }
      }
      ++q;
    }
    __syncthreads();
  }
}


// ---- dense small-range integer keys: one range level + direct-indexed LDS aggregation -----------
// When a groupBy key column spans R = max - min + 1 <= 2^20 values (ids, codes, bucketed keys), a
// partition by the top 8 bits of (key - lo) holds a contiguous window of W = 2^sh <= 4096 keys, so
// its aggregate table is a direct-indexed LDS array: no stored keys, no probing, no spill, and ONE
// partitioning pass instead of the two hash levels above (the 1B-row / 1M-key groupBy: count +
// scatter + aggregate, ~12 of its 21 ms were the second level).
//   range_count_k    per-tile 256-bin digit counts, tile-major [tile][digit], and per-tile [min, max]
//                    (the host checks that every key fell inside the sample-guessed window)
//   range_scatter_k  rows staged in LDS by digit, written as 256 contiguous runs; a key leaves as its
//                    u16 index inside its partition's window ((key - lo) & (W - 1): the partition
//                    is implied by the run), values as f64 (null -> NaN)
//   range_agg_k      (chunk, partition) workgroups: rows u32 / per-column sum f64 + count u32 over the
//                    partition's W-key window in LDS, written out as one dense partial table per chunk
//                    (plain coalesced stores, no global atomics; the host sums the chunks in a fixed order)
#define RGB 256
#ifndef PTG_RGT
#define PTG_RGT 4096  // range tile rows (nv <= 1; nv = 2 uses half); 8192: 62.7 vs 73.4G rows/s (1 workgroup per CU)
#endif
#define RGT PTG_RGT
PTG_DEV int range_digit(long long k, long long lo, int sh) {
  long long d = (k - lo) >> sh;
  return d < 0 ? 0 : (d > RGB - 1 ? RGB - 1 : (int)d);  // out-of-window keys are detected via range
}

__global__ __launch_bounds__(256) void range_count_k(const long long* __restrict__ keys, long n, long long lo, int sh,
                                                     int T, int ntiles, unsigned int* __restrict__ hist,
                                                     long long* __restrict__ range) {
  constexpr int RPT = RGT / 256;
  __shared__ unsigned int h[4][RGB];
  __shared__ long long rmn[4], rmx[4];
  const int tid = threadIdx.x, b = blockIdx.x, w = tid >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) h[q][tid] = 0;
  const long s0 = (long)b * T;
  const int nr = (int)min((long)T, n - s0);
  long long k[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * 256;
    k[j] = i < nr ? keys[s0 + i] : 0;
  }
  long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000ULL;
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (tid + j * 256 < nr) { mn = k[j] < mn ? k[j] : mn; mx = k[j] > mx ? k[j] : mx; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long a = __shfl_xor(mn, o, 64), c = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = c > mx ? c : mx;
  }
  if ((tid & 63) == 0) { rmn[w] = mn; rmx[w] = mx; }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (tid + j * 256 < nr) atomicAdd(&h[w][range_digit(k[j], lo, sh)], 1u);
  __syncthreads();
  hist[(long)b * RGB + tid] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
  (void)ntiles;
  if (tid == 0) {
    long long a = rmn[0], c = rmx[0];
    for (int q = 1; q < 4; ++q) { a = rmn[q] < a ? rmn[q] : a; c = rmx[q] > c ? rmx[q] : c; }
    range[2 * b] = a;
    range[2 * b + 1] = c;
  }
}

template <int NV, int RTT, int NT = 512, class OK = unsigned short>
__global__ __launch_bounds__(NT) void range_scatter_k(const long long* __restrict__ keys, PayIn pin, long n,
                                                       long long lo, int sh, int ntiles,
                                                       const long long* __restrict__ offs,
                                                       OK* __restrict__ okeys, PayOut pout) {
  constexpr int RPT = RTT / NT;
  static_assert(RPT >= 1 && RTT % NT == 0, "tile rows must be a multiple of the thread count");
  constexpr int NVS = NV > 0 ? NV : 1;
  __shared__ OK sk[RTT];
  __shared__ double sv[NVS][RTT];
  __shared__ unsigned char sd[RTT];
  __shared__ unsigned int cnt[RGB];
  __shared__ unsigned int lstart[RGB];
  __shared__ long long goff[RGB];
  const int tid = threadIdx.x, b = xcd_tile(blockIdx.x, ntiles);
  const long s0 = (long)b * RTT;
  const int nr = (int)min((long)RTT, n - s0);
  for (int d = tid; d < RGB; d += NT) {
    cnt[d] = 0;
    goff[d] = offs[(long)b * RGB + d];  // tile-major offsets (ptg_digit_offsets)
  }
  __syncthreads();
  long long k[RPT];
  double v[NVS][RPT];
  int d[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * NT;
    d[j] = -1;
    if (i < nr) {
      k[j] = keys[s0 + i];
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q][j] = load_pay(pin, q, s0 + i);
      d[j] = range_digit(k[j], lo, sh);
      atomicAdd(&cnt[d[j]], 1u);
    }
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 256 digit counts in one wave, 4 per lane
    unsigned c4[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { c4[q] = cnt[4 * tid + q]; sum += c4[q]; }
    unsigned incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned t = __shfl_up(incl, o, 64);
      if (tid >= o) incl += t;
    }
    unsigned run = incl - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) { lstart[4 * tid + q] = run; run += c4[q]; cnt[4 * tid + q] = 0; }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    if (d[j] < 0) continue;
    const unsigned pos = lstart[d[j]] + atomicAdd(&cnt[d[j]], 1u);
    sk[pos] = (OK)((unsigned long long)(k[j] - lo) & ((1ull << sh) - 1ull));
#pragma unroll
    for (int q = 0; q < NV; ++q) sv[q][pos] = v[q][j];
    sd[pos] = (unsigned char)d[j];
  }
  __syncthreads();
  for (int i = tid; i < nr; i += NT) {  // consecutive rows of a digit run -> consecutive addresses
    const int dd = sd[i];
    const long long dst = PTG_CHECKED_IDX(goff[dd] + (i - (int)lstart[dd]), n);
    okeys[dst] = sk[i];
#pragma unroll
    for (int q = 0; q < NV; ++q) pout.vals[q][dst] = sv[q][i];
  }
}

// grid (chunks, 256): partition p = blockIdx.y holds rows [offs[p], offs[p+1]) (tile 0's row of the
// tile-major offsets; offs[256*ntiles] = n closes the last partition), keys
// lo + p*W + okeys[i] (u16 window indices).  Output per chunk c (Rw = 256*W entries):
// prow[c][0][Rw] rows, prow[c][1+j][Rw] non-null count of column j, psum[c][j][Rw] sums and, with
// MINMAX, pmm[c][2j][Rw] / pmm[c][2j+1][Rw] min / max (+-inf where a key has no non-null value).
// LDS: W * (4 + NV * (12 + (MINMAX ? 16 : 0))) bytes (ops/df.py picks W to fit).
// One (partition, chunk) of a direct-indexed LDS aggregation: rows [a0, b0) of okeys (window
// indices < W = 2^sh) / pay, split C ways; the partition's dense partial table starts at column o of
// prow[c][1+NV][Rw] / psum[c][NV][Rw] (/ pmm[c][2NV][Rw] with MINMAX).
template <int NV, bool MINMAX, class OK>
PTG_DEV void range_agg_part(const OK* __restrict__ okeys, const AggPay& pay, long long a0, long long b0, int c, int C,
                            int sh, long Rw, long o, unsigned int* __restrict__ prow, double* __restrict__ psum,
                            double* __restrict__ pmm) {
  constexpr int NVS = NV > 0 ? NV : 1;
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const int W = 1 << sh;
  double* lsum = (double*)lds_raw;                                    // [NV][W]
  double* lmm = lsum + (long)NV * W;                                  // [NV][2][W] (MINMAX)
  unsigned int* lrow = (unsigned int*)(lmm + (MINMAX ? 2L * NV * W : 0L)); // [1 + NV][W]
  for (int t = threadIdx.x; t < W; t += 256) {
    lrow[t] = 0;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      lsum[j * W + t] = 0.0;
      lrow[(1 + j) * W + t] = 0;
      if (MINMAX) { lmm[(2 * j) * W + t] = INFINITY; lmm[(2 * j + 1) * W + t] = -INFINITY; }
    }
  }
  __syncthreads();
  const long long len = b0 - a0;
  const long long a = a0 + len * c / C, b = a0 + len * (c + 1) / C;
  auto add = [&](unsigned int i, const double* v) {  // i: index inside the window
    atomicAdd(&lrow[i], 1u);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      if (v[j] != v[j]) continue;  // null / NaN
      atomicAdd(&lsum[j * W + i], v[j]);
      atomicAdd(&lrow[(1 + j) * W + i], 1u);
      if (MINMAX) {
        lds_min_f64(&lmm[(2 * j) * W + i], v[j]);
        lds_max_f64(&lmm[(2 * j + 1) * W + i], v[j]);
      }
    }
  };
  long long i = a + threadIdx.x;
  for (; i + 3 * 256 < b; i += 4 * 256) {  // 4 rows' loads in flight ahead of the LDS atomics
    unsigned int k4[4];
    double v4[4][NVS];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      k4[u] = okeys[i + u * 256];
#pragma unroll
      for (int j = 0; j < NV; ++j) v4[u][j] = pay.vals[j][i + u * 256];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) add(k4[u], v4[u]);
  }
  for (; i < b; i += 256) {
    double v1[NVS];
#pragma unroll
    for (int j = 0; j < NV; ++j) v1[j] = pay.vals[j][i];
    add(okeys[i], v1);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < W; t += 256) {
    prow[((long)c * (1 + NV)) * Rw + o + t] = lrow[t];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      prow[((long)c * (1 + NV) + 1 + j) * Rw + o + t] = lrow[(1 + j) * W + t];
      psum[((long)c * NV + j) * Rw + o + t] = lsum[j * W + t];
      if (MINMAX) {
        pmm[((long)c * 2 * NV + 2 * j) * Rw + o + t] = lmm[(2 * j) * W + t];
        pmm[((long)c * 2 * NV + 2 * j + 1) * Rw + o + t] = lmm[(2 * j + 1) * W + t];
      }
    }
  }
}

// grid (chunks, 256): partition p = blockIdx.y holds rows [offs[p], offs[p+1]) (tile 0's row of the
// tile-major offsets; offs[256*ntiles] = n closes the last partition), keys
// lo + p*W + okeys[i] (u16 window indices).  Output per chunk c (Rw = 256*W entries):
// prow[c][0][Rw] rows, prow[c][1+j][Rw] non-null count of column j, psum[c][j][Rw] sums and, with
// MINMAX, pmm[c][2j][Rw] / pmm[c][2j+1][Rw] min / max (+-inf where a key has no non-null value).
// LDS: W * (4 + NV * (12 + (MINMAX ? 16 : 0))) bytes (ops/df.py picks W to fit).
template <int NV, bool MINMAX>
__global__ __launch_bounds__(256) void range_agg_k(const unsigned short* __restrict__ okeys, AggPay pay,
                                                   const long long* __restrict__ offs, int ntiles, int sh,
                                                   unsigned int* __restrict__ prow, double* __restrict__ psum,
                                                   double* __restrict__ pmm) {
  const int p = blockIdx.y;
  const long long a0 = offs[p], b0 = p + 1 < RGB ? offs[p + 1] : offs[(long)RGB * ntiles];
  range_agg_part<NV, MINMAX>(okeys, pay, a0, b0, (int)blockIdx.x, (int)gridDim.x, sh, (long)RGB << sh,
                             (long)p << sh, prow, psum, pmm);
}

// ---- dense key spans up to 2^28 (ids, dates x ids, ...): two 256-way range levels -----------------
// Level 1 (range_count_k + range_scatter_k<.., u32>): 256 coarse partitions of 2^(sh2+8) keys, keys
// leave as u32 offsets inside their coarse window.  Level 2 (range2_count_k / range2_scatter_k):
// every coarse partition is tiled on its own (ptg_seg_plan with 256 bins: histograms digit-major
// per segment, so ONE exclusive scan of all of them gives every (coarse, fine, tile) run its output
// position) and split 256 ways by off >> sh2; keys leave as u16 offsets inside 2^sh2-key fine windows.
// range2_agg_k: one workgroup (x chunks) per fine partition, the same direct-indexed LDS table as
// range_agg_k.  ~70 B of traffic per row, against ~100 for three hash radix levels + LDS hash tables.
template <int RTT>
__global__ __launch_bounds__(256) void range2_count_k(const unsigned int* __restrict__ okeys,
                                                      const long long* __restrict__ tstart,
                                                      const int* __restrict__ trows,
                                                      const long long* __restrict__ thbase,
                                                      const long long* __restrict__ thstride, int sh2,
                                                      unsigned int* __restrict__ hist) {
  constexpr int RPT = RTT / 256;
  __shared__ unsigned int h[4][RGB];
  const int tid = threadIdx.x, b = blockIdx.x, w = tid >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) h[q][tid] = 0;
  const long long s0 = tstart[b];
  const int nr = trows[b];
  unsigned int k[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * 256;
    k[j] = i < nr ? okeys[s0 + i] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (tid + j * 256 < nr) atomicAdd(&h[w][(k[j] >> sh2) & (RGB - 1)], 1u);
  __syncthreads();
  hist[thbase[b] + (long long)tid * thstride[b]] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

template <int NV, int RTT, int NT = 512>
__global__ __launch_bounds__(NT) void range2_scatter_k(const unsigned int* __restrict__ keys, AggPay pin,
                                                       const long long* __restrict__ tstart,
                                                       const int* __restrict__ trows,
                                                       const long long* __restrict__ thbase,
                                                       const long long* __restrict__ thstride, int sh2,
                                                       const long long* __restrict__ offs, long n,
                                                       unsigned short* __restrict__ okeys, PayOut pout) {
  constexpr int RPT = RTT / NT;
  static_assert(RPT >= 1 && RTT % NT == 0, "tile rows must be a multiple of the thread count");
  constexpr int NVS = NV > 0 ? NV : 1;
  __shared__ unsigned short sk[RTT];
  __shared__ double sv[NVS][RTT];
  __shared__ unsigned char sd[RTT];
  __shared__ unsigned int cnt[RGB];
  __shared__ unsigned int lstart[RGB];
  __shared__ long long goff[RGB];
  const int tid = threadIdx.x, b = xcd_tile(blockIdx.x, gridDim.x);
  const long long s0 = tstart[b];
  const int nr = trows[b];
  for (int d = tid; d < RGB; d += NT) {
    cnt[d] = 0;
    goff[d] = offs[thbase[b] + (long long)d * thstride[b]];
  }
  __syncthreads();
  unsigned int k[RPT];
  double v[NVS][RPT];
  int d[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * NT;
    d[j] = -1;
    if (i < nr) {
      k[j] = keys[s0 + i];
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q][j] = pin.vals[q][s0 + i];
      d[j] = (int)((k[j] >> sh2) & (RGB - 1));
      atomicAdd(&cnt[d[j]], 1u);
    }
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 256 digit counts in one wave, 4 per lane
    unsigned c4[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { c4[q] = cnt[4 * tid + q]; sum += c4[q]; }
    unsigned incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned t = __shfl_up(incl, o, 64);
      if (tid >= o) incl += t;
    }
    unsigned run = incl - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) { lstart[4 * tid + q] = run; run += c4[q]; cnt[4 * tid + q] = 0; }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    if (d[j] < 0) continue;
    const unsigned pos = lstart[d[j]] + atomicAdd(&cnt[d[j]], 1u);
    sk[pos] = (unsigned short)(k[j] & ((1u << sh2) - 1u));
#pragma unroll
    for (int q = 0; q < NV; ++q) sv[q][pos] = v[q][j];
    sd[pos] = (unsigned char)d[j];
  }
  __syncthreads();
  for (int i = tid; i < nr; i += NT) {
    const int dd = sd[i];
    const long long dst = PTG_CHECKED_IDX(goff[dd] + (i - (int)lstart[dd]), n);
    okeys[dst] = sk[i];
#pragma unroll
    for (int q = 0; q < NV; ++q) pout.vals[q][dst] = sv[q][i];
  }
}

// one workgroup per (fine partition p, chunk c): blockIdx.x = p * C + c; fine partition p holds rows
// [fstart[p], fend[p]) and keys lo + (p << sh2) + okeys[i]
template <int NV>
__global__ __launch_bounds__(256) void range2_agg_k(const unsigned short* __restrict__ okeys, AggPay pay,
                                                    const long long* __restrict__ fstart,
                                                    const long long* __restrict__ fend, int C, int sh2, long Rw,
                                                    unsigned int* __restrict__ prow, double* __restrict__ psum) {
  const int p = blockIdx.x / C, c = blockIdx.x - p * C;
  range_agg_part<NV, false>(okeys, pay, fstart[p], fend[p], c, C, sh2, Rw, (long)p << sh2, prow, psum, nullptr);
}

// ---- tiny key ranges (max - min < ~4K): no partitioning at all ---------------------------------
// Every workgroup holds the WHOLE key range as a direct-indexed LDS table (index = key - lo: no
// hashing, probing or CAS), aggregates a contiguous chunk of rows, and writes a dense partial table;
// dense_extract sums the partials.  One read of the data (the LDS hash table path, hash_agg_lds_k,
// ran 41-51 ms per 1B rows at 1K keys).
//  * the key window [lo, lo + W) comes from a strided sample, not a full min/max pass: a key outside
//    it sets *err and is skipped, and the host re-plans with the exact range (the sample costs 64K
//    loads instead of a second 8 GB read of the key column at 1B rows);
//  * per row: one u32 LDS atomic (row count) + one f64 LDS atomic per value column; the per-column
//    value count is rows - nulls, so the null-count atomic runs only for a null / NaN value;
//  * FAST (every value column plain f64 without a validity mask): rows go two per thread as 16-byte
//    loads of two keys and two values, UNR pairs in flight per thread, no per-element type switch
//    (the generic loader's switch serialised the unrolled loads behind vmcnt(0) waits).
template <int NV, bool FAST>
__global__ __launch_bounds__(256) void small_range_agg_k(const long long* __restrict__ keys, long n, long long lo, int W,
                                                         PayIn pin, long rows_per_block, unsigned int* __restrict__ prow,
                                                         double* __restrict__ psum, int* __restrict__ err) {
  constexpr int NVS = NV > 0 ? NV : 1;
  constexpr int UNR = 4;
  extern __shared__ __align__(16) unsigned char lds_raw[];
  double* lsum = (double*)lds_raw;                            // [NV][W]
  unsigned int* lrow = (unsigned int*)(lsum + (long)NV * W);  // [1 + NV][W]: rows, then nulls per column
  for (int t = threadIdx.x; t < W; t += 256) {
    lrow[t] = 0;
#pragma unroll
    for (int j = 0; j < NV; ++j) { lsum[j * W + t] = 0.0; lrow[(1 + j) * W + t] = 0; }
  }
  __syncthreads();
  bool bad = false;
  auto add = [&](long long k, const double* v) {
    const unsigned long long i = (unsigned long long)(k - lo);
    if (i >= (unsigned long long)W) { bad = true; return; }
    atomicAdd(&lrow[i], 1u);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      if (v[j] != v[j]) { atomicAdd(&lrow[(1 + j) * W + i], 1u); continue; }  // null / NaN
      atomicAdd(&lsum[j * W + i], v[j]);
    }
  };
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(n, r0 + rows_per_block);
  long i = r0;
  if (FAST) {
    // r0 is a multiple of 2 * 256 * UNR (host): pairs of rows are 16-byte aligned
    const double* const* vals = (const double* const*)pin.vals;
    for (; i + 2 * 256 * UNR <= r1; i += 2 * 256 * UNR) {
      longlong2 k2[UNR];
      double2 v2[UNR][NVS];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long e = i + 2 * (u * 256 + threadIdx.x);
        k2[u] = *(const longlong2*)(keys + e);
#pragma unroll
        for (int j = 0; j < NV; ++j) v2[u][j] = *(const double2*)(vals[j] + e);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        double a[NVS], b[NVS];
#pragma unroll
        for (int j = 0; j < NV; ++j) { a[j] = v2[u][j].x; b[j] = v2[u][j].y; }
        add(k2[u].x, a);
        add(k2[u].y, b);
      }
    }
    for (i += threadIdx.x; i < r1; i += 256) {
      double v1[NVS];
#pragma unroll
      for (int j = 0; j < NV; ++j) v1[j] = vals[j][i];
      add(keys[i], v1);
    }
  } else {
    for (i += threadIdx.x; i + 3 * 256 < r1; i += 4 * 256) {
      long long k4[4];
      double v4[4][NVS];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        k4[u] = keys[i + u * 256];
#pragma unroll
        for (int j = 0; j < NV; ++j) v4[u][j] = load_pay(pin, j, i + u * 256);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) add(k4[u], v4[u]);
    }
    for (; i < r1; i += 256) {
      double v1[NVS];
#pragma unroll
      for (int j = 0; j < NV; ++j) v1[j] = load_pay(pin, j, i);
      add(keys[i], v1);
    }
  }
  if (bad) atomicOr(err, 1);
  __syncthreads();
  const long b = blockIdx.x;
  for (int t = threadIdx.x; t < W; t += 256) {
    const unsigned int rows = lrow[t];
    prow[(b * (1 + NV)) * W + t] = rows;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      prow[(b * (1 + NV) + 1 + j) * W + t] = rows - lrow[(1 + j) * W + t];
      psum[(b * NV + j) * W + t] = lsum[j * W + t];
    }
  }
}

// ---- sparse keys at mid cardinality: ONE 512-way hash partition + LDS hash tables --------------
// The recursive radix path needs two 64-way levels for ~1M distinct keys (count + scatter twice:
// ~96 B moved per row with one f64 column).  Partitioned 512 ways by the top 9 bits of mix64(key),
// a partition holds K/512 keys (~2K at 1M groups), which fit one LDS hash table, so the data is
// counted, scattered and aggregated once (~56 B per row):
//   hash9_count_k    per-tile 512-bin histograms, tile-major [tile][512] (ptg_digit_offsets_b)
//   hash9_scatter_k  rows staged in LDS by digit, written as 512 contiguous runs (i64 key, f64
//                    values, null -> NaN); XCD-aware tile order as the other scatter passes
//   hash9_agg_k      (chunk, partition) workgroups of 1024 threads: an LDS hash table over the
//                    chunk's rows, occupied slots compacted into the (partition, chunk) region of a
//                    partial table (no global atomics on data)
//   hash9_merge_k    one workgroup per partition folds its chunks' partials into one table and
//                    appends the groups to the output in hash_extract_k's layout
// A table that overflows (far more keys than the estimate) sets the error word; the host then takes
// the recursive path, so a bad estimate costs time, never correctness.
#define H9B 512
#ifndef PTG_H9T
#define PTG_H9T 4096
#endif
#define H9T PTG_H9T  // tile rows for nv <= 1 (nv == 2: half, the LDS staging budget)
PTG_DEV int h9_digit(long long k) { return (int)(mix64((unsigned long long)k) >> (64 - 9)); }

__global__ __launch_bounds__(256) void hash9_count_k(const long long* __restrict__ keys, long n, int T,
                                                     unsigned int* __restrict__ hist) {
  constexpr int RPT = H9T / 256;
  __shared__ unsigned int h[4][H9B];
  const int tid = threadIdx.x, b = blockIdx.x, w = tid >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) { h[q][tid] = 0; h[q][tid + 256] = 0; }
  const long s0 = (long)b * T;
  const int nr = (int)min((long)T, n - s0);
  long long k[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * 256;
    k[j] = i < nr ? keys[s0 + i] : 0;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (tid + j * 256 < nr) atomicAdd(&h[w][h9_digit(k[j])], 1u);
  __syncthreads();
  for (int d = tid; d < H9B; d += 256) hist[(long)b * H9B + d] = h[0][d] + h[1][d] + h[2][d] + h[3][d];
}

template <int NV, int RTT, int NT = 512>
__global__ __launch_bounds__(NT) void hash9_scatter_k(const long long* __restrict__ keys, PayIn pin, long n,
                                                      int ntiles, const long long* __restrict__ offs,
                                                      long long* __restrict__ okeys, PayOut pout) {
  constexpr int RPT = RTT / NT;
  static_assert(RPT >= 1 && RTT % NT == 0, "tile rows must be a multiple of the thread count");
  constexpr int NVS = NV > 0 ? NV : 1;
  __shared__ long long sk[RTT];
  __shared__ double sv[NVS][NV > 0 ? RTT : 1];
  __shared__ unsigned short sd[RTT];
  __shared__ unsigned int cnt[H9B];
  __shared__ unsigned int lstart[H9B];
  __shared__ long long goff[H9B];
  const int tid = threadIdx.x, b = xcd_tile(blockIdx.x, ntiles);
  const long s0 = (long)b * RTT;
  const int nr = (int)min((long)RTT, n - s0);
  for (int d = tid; d < H9B; d += NT) {
    cnt[d] = 0;
    goff[d] = offs[(long)b * H9B + d];
  }
  __syncthreads();
  long long k[RPT];
  double v[NVS][RPT];
  int d[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = tid + j * NT;
    d[j] = -1;
    if (i < nr) {
      k[j] = keys[s0 + i];
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q][j] = load_pay(pin, q, s0 + i);
      d[j] = h9_digit(k[j]);
      atomicAdd(&cnt[d[j]], 1u);
    }
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 512 digit counts in one wave, 8 per lane
    unsigned c8[8], sum = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) { c8[q] = cnt[8 * tid + q]; sum += c8[q]; }
    unsigned incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned t = __shfl_up(incl, o, 64);
      if (tid >= o) incl += t;
    }
    unsigned run = incl - sum;
#pragma unroll
    for (int q = 0; q < 8; ++q) { lstart[8 * tid + q] = run; run += c8[q]; cnt[8 * tid + q] = 0; }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    if (d[j] < 0) continue;
    const unsigned pos = lstart[d[j]] + atomicAdd(&cnt[d[j]], 1u);
    sk[pos] = k[j];
#pragma unroll
    for (int q = 0; q < NV; ++q) sv[q][pos] = v[q][j];
    sd[pos] = (unsigned short)d[j];
  }
  __syncthreads();
  for (int i = tid; i < nr; i += NT) {  // consecutive rows of a digit run -> consecutive addresses
    const int dd = sd[i];
    const long long dst = PTG_CHECKED_IDX(goff[dd] + (i - (int)lstart[dd]), n);
    okeys[dst] = sk[i];
#pragma unroll
    for (int q = 0; q < NV; ++q) pout.vals[q][dst] = sv[q][i];
  }
}

// LDS hash table of TS slots (power of two, >= 1024): [keys i64][sum f64 per column][rows u32][cnt u32
// per column]; rows/sum/cnt added with LDS atomics.  Returns false when no slot was found in
// H9_PROBES probes (the table is too full: the host falls back).
#define H9_PROBES 256
template <int NV>
struct H9Table {
  long long* lk;
  double* lsum;
  unsigned int* lrow;
  unsigned int* lcnt;
  int TS;
  PTG_DEV H9Table(unsigned char* raw, int ts) : TS(ts) {
    lk = (long long*)raw;
    lsum = (double*)(lk + ts);
    lrow = (unsigned int*)(lsum + (long)NV * ts);
    lcnt = lrow + ts;
  }
  PTG_DEV void clear(int tid, int nt) {
    for (int t = tid; t < TS; t += nt) {
      lk[t] = EMPTY_KEY;
      lrow[t] = 0;
#pragma unroll
      for (int j = 0; j < NV; ++j) { lsum[j * TS + t] = 0.0; lcnt[j * TS + t] = 0; }
    }
  }
  PTG_DEV int slot(long long key) {
    const int mask = TS - 1;
    int h = (int)(mix64((unsigned long long)key) & (unsigned long long)mask);
    for (int probe = 0; probe < H9_PROBES; ++probe) {
      const long long cur = lk[h];
      if (cur == key) return h;
      if (cur == EMPTY_KEY) {
        const long long prev = (long long)atomicCAS((unsigned long long*)&lk[h], (unsigned long long)EMPTY_KEY,
                                                    (unsigned long long)key);
        if (prev == EMPTY_KEY || prev == key) return h;
      }
      h = (h + 1) & mask;
    }
    return -1;
  }
};

// Block-wide exclusive scan over 1024 threads (16 waves); *total = the sum.
PTG_DEV int block_excl_scan1024(int c, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int x = wsum[q];
    base += q < w ? x : 0;
    tot += x;
  }
  *total = tot;
  return base + incl - c;
}

// grid (chunks, 512): partition p = blockIdx.y holds rows [offs[p], offs[p+1]) of the scattered
// arrays (offs tile-major, offs[512*ntiles] = n); chunk c its c-th slice.  Partial region
// (p, c) = entries [(p*C + c)*TS, +pn[p*C + c]) of pkeys / prow / psum[j] / pcnt[j] (R = 512*C*TS each).
template <int NV>
__global__ __launch_bounds__(1024) void hash9_agg_k(const long long* __restrict__ okeys, AggPay pay,
                                                    const long long* __restrict__ offs, int ntiles, int TS,
                                                    long long* __restrict__ pkeys, unsigned int* __restrict__ prow,
                                                    double* __restrict__ psum, unsigned int* __restrict__ pcnt,
                                                    int* __restrict__ pn, unsigned long long* __restrict__ state) {
  constexpr int NVS = NV > 0 ? NV : 1;
  extern __shared__ __align__(16) unsigned char lds_raw[];
  __shared__ int wsum[16];
  __shared__ int sfail;
  const int p = blockIdx.y, c = blockIdx.x, C = gridDim.x, tid = threadIdx.x;
  H9Table<NV> tb(lds_raw, TS);
  tb.clear(tid, 1024);
  if (tid == 0) sfail = 0;
  __syncthreads();
  const long long a0 = offs[p], b0 = p + 1 < H9B ? offs[p + 1] : offs[(long)H9B * ntiles], len = b0 - a0;
  const long long a = a0 + len * c / C, b = a0 + len * (c + 1) / C;
  bool ok = true;
  auto add = [&](long long key, const double* v) {
    const int sl = tb.slot(key);
    if (sl < 0) { ok = false; return; }
    atomicAdd(&tb.lrow[sl], 1u);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      if (v[j] != v[j]) continue;  // null / NaN
      atomicAdd(&tb.lsum[j * TS + sl], v[j]);
      atomicAdd(&tb.lcnt[j * TS + sl], 1u);
    }
  };
  long long i = a + tid;
  for (; i + 3 * 1024 < b; i += 4 * 1024) {  // 4 rows' loads in flight ahead of the LDS probes
    long long k4[4];
    double v4[4][NVS];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      k4[u] = okeys[i + u * 1024];
#pragma unroll
      for (int j = 0; j < NV; ++j) v4[u][j] = pay.vals[j][i + u * 1024];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) add(k4[u], v4[u]);
  }
  for (; i < b; i += 1024) {
    double v1[NVS];
#pragma unroll
    for (int j = 0; j < NV; ++j) v1[j] = pay.vals[j][i];
    add(okeys[i], v1);
  }
  if (!ok) sfail = 1;
  __syncthreads();
  if (sfail) {
    if (tid == 0) { atomicOr(&state[1], 1ull); pn[p * C + c] = 0; }
    return;
  }
  // compact the occupied slots into the region: each thread owns TS/1024 consecutive slots
  const int per = TS >> 10, s0 = tid * per;
  int cn = 0;
  for (int t = s0; t < s0 + per; ++t) cn += tb.lk[t] != EMPTY_KEY;
  int total;
  int q = block_excl_scan1024(cn, wsum, &total);
  const long R = (long)H9B * C * TS, base = ((long)p * C + c) * TS;
  for (int t = s0; t < s0 + per; ++t) {
    const long long key = tb.lk[t];
    if (key == EMPTY_KEY) continue;
    pkeys[base + q] = key;
    prow[base + q] = tb.lrow[t];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      psum[j * R + base + q] = tb.lsum[j * TS + t];
      pcnt[j * R + base + q] = tb.lcnt[j * TS + t];
    }
    ++q;
  }
  if (tid == 0) pn[p * C + c] = total;
}

// grid 512: partition p folds its C partial regions into one LDS table, then appends its groups at
// state[0] (atomic base) to out_keys / out_tab ([1 + 4*NV][out_cap]: rows, then per column sum,
// non-null count, min, max as f64; min / max are +-inf: this path serves sum / count / avg).
template <int NV>
__global__ __launch_bounds__(1024) void hash9_merge_k(const long long* __restrict__ pkeys,
                                                      const unsigned int* __restrict__ prow,
                                                      const double* __restrict__ psum,
                                                      const unsigned int* __restrict__ pcnt,
                                                      const int* __restrict__ pn, int C, int TS,
                                                      long long* __restrict__ out_keys, double* __restrict__ out_tab,
                                                      long out_cap, unsigned long long* __restrict__ state) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  __shared__ int wsum[16];
  __shared__ int sfail;
  __shared__ unsigned long long obase;
  const int p = blockIdx.x, tid = threadIdx.x;
  H9Table<NV> tb(lds_raw, TS);
  tb.clear(tid, 1024);
  if (tid == 0) sfail = 0;
  __syncthreads();
  const long R = (long)H9B * C * TS;
  bool ok = true;
  for (int c = 0; c < C; ++c) {
    const long base = ((long)p * C + c) * TS;
    const int m = pn[p * C + c];
    for (int i = tid; i < m; i += 1024) {
      const int sl = tb.slot(pkeys[base + i]);
      if (sl < 0) { ok = false; continue; }
      atomicAdd(&tb.lrow[sl], prow[base + i]);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        atomicAdd(&tb.lsum[j * TS + sl], psum[j * R + base + i]);
        atomicAdd(&tb.lcnt[j * TS + sl], pcnt[j * R + base + i]);
      }
    }
  }
  if (!ok) sfail = 1;
  __syncthreads();
  if (sfail) {
    if (tid == 0) atomicOr(&state[1], 1ull);
    return;
  }
  const int per = TS >> 10, s0 = tid * per;
  int cn = 0;
  for (int t = s0; t < s0 + per; ++t) cn += tb.lk[t] != EMPTY_KEY;
  int total;
  const int pre = block_excl_scan1024(cn, wsum, &total);
  if (tid == 0) obase = total ? atomicAdd(&state[0], (unsigned long long)total) : 0ull;
  __syncthreads();
  long long q = (long long)obase + pre;
  for (int t = s0; t < s0 + per; ++t) {
    const long long key = tb.lk[t];
    if (key == EMPTY_KEY) continue;
    if (q < out_cap) {
      out_keys[q] = key;
      out_tab[q] = (double)tb.lrow[t];
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        double* o = out_tab + out_cap * (1 + 4 * j);
        o[q] = tb.lsum[j * TS + t];
        o[out_cap + q] = (double)tb.lcnt[j * TS + t];
        o[2 * out_cap + q] = INFINITY;
        o[3 * out_cap + q] = -INFINITY;
      }
    }
    ++q;
  }
}

// ================================================================================================
// Stable LSD radix sort of 64-bit keys with a 64-bit payload (DataFrame.orderBy / sort)
//   sort_key_prep_k  column -> unsigned-orderable u64 (asc or desc; NaN above +inf, -0 == +0) and
//                    the key range [min, max]: only the significant bits of (max - min) are sorted
//   sort_count_k     per-tile 256-bin digit histograms, tile-major [tile][digit] (one coalesced
//                    1 KB row per tile); dfutil.hip ptg_digit_offsets turns them into every
//                    (tile, digit)'s output run in stable (digit-major) order, also tile-major
//   sort_scatter_k   stable in-tile ranking (8-ballot match per wave, per-round wave prefix over
//                    LDS), rows staged in LDS by digit, written out as 256 contiguous runs
//   range_partition_k  destination rank = #splitters below the key (sample-based range shuffle)
// ================================================================================================
#ifndef PTG_ST
#define PTG_ST 4096
#endif
#define ST PTG_ST        // rows per sort tile
#define SB 256           // digit bins (8 bits per pass)
// threads per sort tile workgroup (A/B build: 512 with 8192-row tiles keeps 16 rows per thread and the
// same 8 waves per CU as two 256-thread 4096-row tiles, with digit runs twice as long)
#ifndef PTG_SORT_NTH
#define PTG_SORT_NTH 256
#endif
#define SNT PTG_SORT_NTH
#define SNW (SNT / 64)
#define SRPT (ST / SNT)

PTG_DEV unsigned long long orderable_key(const void* col, int type, long i, int desc) {
  unsigned long long u;
  switch (type) {
    case CT_F32:
    case CT_F64: {
      double x = type == CT_F32 ? (double)((const float*)col)[i] : ((const double*)col)[i];
      if (x != x) x = __builtin_nan("");
      x = x + 0.0;  // -0 -> +0
      const unsigned long long b = (unsigned long long)__double_as_longlong(x);
      u = (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
      break;
    }
    case CT_I32: u = (unsigned long long)(long long)((const int*)col)[i] ^ 0x8000000000000000ULL; break;
    case CT_U8: u = (unsigned long long)((const uint8_t*)col)[i]; break;
    default: u = (unsigned long long)((const long long*)col)[i] ^ 0x8000000000000000ULL; break;
  }
  return desc ? ~u : u;
}

PTG_DEV unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const unsigned long long t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
  return v;
}
PTG_DEV unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const unsigned long long t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
  return v;
}

// range[0] = min, range[1] = max (initialised to ~0 / 0 by the host)
__global__ __launch_bounds__(256) void sort_key_prep_k(const void* __restrict__ col, int type, long n, int desc,
                                                       unsigned long long* __restrict__ out,
                                                       unsigned long long* __restrict__ range) {
  unsigned long long mn = ~0ULL, mx = 0ULL;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const unsigned long long u = orderable_key(col, type, i, desc);
    if (out) out[i] = u;  // null: range only (the first radix pass applies the transform itself)
    mn = u < mn ? u : mn;
    mx = u > mx ? u : mx;
  }
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&range[0], mn);
    atomicMax(&range[1], mx);
  }
}

// xin: XOR mask applied to every key as it is read (int64 column -> orderable u64 in the first pass:
// sign bit for ascending, its complement for descending; 0 = keys already orderable)
__global__ __launch_bounds__(SNT) void sort_count_k(const unsigned long long* __restrict__ keys, long n,
                                                    unsigned long long base, int shift, int ntiles,
                                                    unsigned int* __restrict__ hist, unsigned long long xin) {
  __shared__ unsigned int h[SNW][SB];
  const int tid = threadIdx.x, w = tid >> 6, b = blockIdx.x;
  for (int t = tid; t < SNW * SB; t += SNT) (&h[0][0])[t] = 0;
  const long s0 = (long)b * ST;
  unsigned long long k[SRPT];
#pragma unroll
  for (int j = 0; j < SRPT; ++j) {
    const long i = s0 + j * SNT + tid;
    k[j] = i < n ? keys[i] ^ xin : 0ULL;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SRPT; ++j)
    if (s0 + j * SNT + tid < n) atomicAdd(&h[w][(unsigned)((k[j] - base) >> shift) & (SB - 1)], 1u);
  __syncthreads();
  if (tid < SB) {
    unsigned c = 0;
#pragma unroll
    for (int q = 0; q < SNW; ++q) c += h[q][tid];
    hist[(long)b * SB + tid] = c;
  }
  (void)ntiles;
}

// The key range and the first radix pass's histogram in ONE read of the keys (an int64 column read raw,
// XOR xin -> orderable): per tile the 256-bin histogram of the RAW low byte (the pass-0 digit
// (k - base) & 255 is that byte rotated by base & 255; ptg_digit_offsets rot) and the tile's
// min / max into tmm[2 * tile], reduced by sort_range_reduce_k.  Replaces sort_key_prep_k's range pass
// and pass 0's sort_count_k.
__global__ __launch_bounds__(SNT) void sort_range_count_k(const unsigned long long* __restrict__ keys, long n,
                                                          unsigned long long xin, unsigned int* __restrict__ hist,
                                                          unsigned long long* __restrict__ tmm) {
  __shared__ unsigned int h[SNW][SB];
  __shared__ unsigned long long wmn[SNW], wmx[SNW];
  const int tid = threadIdx.x, w = tid >> 6, b = blockIdx.x;
  for (int t = tid; t < SNW * SB; t += SNT) (&h[0][0])[t] = 0;
  const long s0 = (long)b * ST;
  unsigned long long k[SRPT];
  unsigned long long mn = ~0ULL, mx = 0ULL;
#pragma unroll
  for (int j = 0; j < SRPT; ++j) {
    const long i = s0 + j * SNT + tid;
    k[j] = i < n ? keys[i] ^ xin : 0ULL;
    if (i < n) { mn = k[j] < mn ? k[j] : mn; mx = k[j] > mx ? k[j] : mx; }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SRPT; ++j)
    if (s0 + j * SNT + tid < n) atomicAdd(&h[w][(unsigned)k[j] & (SB - 1)], 1u);
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  if ((tid & 63) == 0) { wmn[w] = mn; wmx[w] = mx; }
  __syncthreads();
  if (tid < SB) {
    unsigned c = 0;
#pragma unroll
    for (int q = 0; q < SNW; ++q) c += h[q][tid];
    hist[(long)b * SB + tid] = c;
  }
  if (tid == 0) {
#pragma unroll
    for (int q = 1; q < SNW; ++q) { mn = wmn[q] < mn ? wmn[q] : mn; mx = wmx[q] > mx ? wmx[q] : mx; }
    mn = wmn[0] < mn ? wmn[0] : mn;
    mx = wmx[0] > mx ? wmx[0] : mx;
    tmm[2L * b] = mn;
    tmm[2L * b + 1] = mx;
  }
}

// range[0] = min, range[1] = max over the tiles' (min, max) pairs (range initialised to ~0 / 0)
__global__ __launch_bounds__(256) void sort_range_reduce_k(const unsigned long long* __restrict__ tmm, int ntiles,
                                                           unsigned long long* __restrict__ range) {
  unsigned long long mn = ~0ULL, mx = 0ULL;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < ntiles; t += gridDim.x * 256) {
    const unsigned long long a = tmm[2L * t], c = tmm[2L * t + 1];
    mn = a < mn ? a : mn;
    mx = c > mx ? c : mx;
  }
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&range[0], mn);
    atomicMax(&range[1], mx);
  }
}

// vals_in == nullptr: payload = row index (first pass of a fresh sort).  VT = unsigned int when the
// row count fits 32 bits: 12 instead of 16 bytes per row read and written by every pass.
// offs holds every (tile, digit) run's output position (sort_count_k + ptg_digit_offsets).
template <typename VT>
__global__ __launch_bounds__(SNT) void sort_scatter_k(const unsigned long long* __restrict__ keys_in,
                                                      const VT* __restrict__ vals_in, long n,
                                                      unsigned long long base, int shift, int ntiles,
                                                      const long long* __restrict__ offs,
                                                      unsigned long long* __restrict__ keys_out,
                                                      VT* __restrict__ vals_out, unsigned long long xin,
                                                      unsigned long long xout) {
  // xin: XOR mask on the keys as read (sort_count_k); xout: on the keys as written (the last pass
  // writes the decoded column values: the same XOR mask undoes the orderable transform)
  __shared__ unsigned long long sk[ST];
  __shared__ VT sv[ST];
  __shared__ unsigned char sd[ST];
  __shared__ unsigned int wc[SNW][SB];
  __shared__ unsigned int woff[SNW][SB];
  __shared__ unsigned int lstart[SB];
  __shared__ long long goff[SB];
  __shared__ int wsum[SNW];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int b = xcd_tile(blockIdx.x, ntiles);
  if (tid < SB) goff[tid] = offs[(long)b * SB + tid];  // tile-major: one coalesced 2 KB row
  const long s0 = (long)b * ST;
  const int nr = (int)((n - s0) < ST ? (n - s0) : ST);
  for (int t = tid; t < SNW * SB; t += SNT) (&wc[0][0])[t] = 0;
  // Wave-contiguous rows: wave w owns tile rows [w*ST/4, (w+1)*ST/4), 64 consecutive rows per round
  // (coalesced loads), so the stable order inside the tile is (wave, round, lane).  Ranks come from
  // a wave-private running count per digit (wc[w]): no block barrier per round, only the one
  // cross-wave prefix per digit after the last round (the round-interleaved form needed 2 block
  // barriers per round to keep the order).
  unsigned long long k[SRPT];
  VT v[SRPT];
  int d[SRPT], r[SRPT];
#pragma unroll
  for (int j = 0; j < SRPT; ++j) {
    const int i = w * (ST / SNW) + j * 64 + lane;
    d[j] = -1;
    if (i < nr) {
      k[j] = keys_in[s0 + i] ^ xin;
      v[j] = vals_in ? vals_in[s0 + i] : (VT)(s0 + i);
      d[j] = (int)((k[j] - base) >> shift) & (SB - 1);
    }
  }
  __syncthreads();  // wc zeroed by every wave before any wave counts into it
  const unsigned long long lt = (1ULL << lane) - 1ULL;
#pragma unroll
  for (int j = 0; j < SRPT; ++j) {
    const bool valid = d[j] >= 0;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool set = valid && ((d[j] >> bit) & 1);
      const unsigned long long bb = __ballot(set);
      peers &= set ? bb : ~bb;
    }
    const int rank_w = __popcll(peers & lt);
    const unsigned old = valid ? wc[w][d[j]] : 0u;  // every lane reads before the leader writes
    __builtin_amdgcn_wave_barrier();
    if (valid && rank_w == 0) wc[w][d[j]] = old + (unsigned)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    r[j] = (int)old + rank_w;
  }
  __syncthreads();
  unsigned int running = 0;
  if (tid < SB) {  // thread tid owns digit tid: per-wave offsets inside the digit's run, and the tile total
#pragma unroll
    for (int q = 0; q < SNW; ++q) {
      woff[q][tid] = running;
      running += wc[q][tid];
    }
  }
  int total;
  const int ls = block_excl_scan256((int)running, wsum, &total);  // threads >= SB add 0 after digit 255
  if (tid < SB) lstart[tid] = (unsigned)ls;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SRPT; ++j) {
    if (d[j] < 0) continue;
    const int pos = (int)lstart[d[j]] + (int)woff[w][d[j]] + r[j];
    sk[pos] = k[j];
    sv[pos] = v[j];
    sd[pos] = (unsigned char)d[j];
  }
  __syncthreads();
  for (int i = tid; i < nr; i += SNT) {
    const int dd = sd[i];
    const long long dst = PTG_CHECKED_IDX(goff[dd] + (i - (int)lstart[dd]), n);
    keys_out[dst] = sk[i] ^ xout;
    vals_out[dst] = sv[i];
  }
}

// part[i] = number of splitters strictly below keys[i] (unsigned order); counts[dest] += 1
__global__ __launch_bounds__(256) void range_partition_k(const unsigned long long* __restrict__ keys, long n,
                                                         const unsigned long long* __restrict__ split, int nsplit,
                                                         int* __restrict__ part,
                                                         unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long sp[1024];
  __shared__ unsigned int h[1025];
  for (int t = threadIdx.x; t < nsplit; t += 256) sp[t] = split[t];
  for (int t = threadIdx.x; t <= nsplit; t += 256) h[t] = 0;
  __syncthreads();
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const unsigned long long k = keys[i];
    int lo = 0, hi = nsplit;  // first splitter >= k
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sp[mid] < k) lo = mid + 1; else hi = mid;
    }
    part[i] = lo;
    atomicAdd(&h[lo], 1u);
  }
  __syncthreads();
  for (int t = threadIdx.x; t <= nsplit; t += 256)
    if (h[t]) atomicAdd(&counts[t], (unsigned long long)h[t]);
}

// ================================================================================================
// histogram of int32 codes (StringIndexer fit); codes < 0 (null) counted in bin nbins
// ================================================================================================
__global__ __launch_bounds__(256) void histogram_k(const int* __restrict__ codes, long n, unsigned long long* __restrict__ out,
                                                   int nbins) {
  __shared__ unsigned int h[4097];
  const bool lds = nbins < 4096;
  if (lds)
    for (int t = threadIdx.x; t <= nbins; t += 256) h[t] = 0;
  __syncthreads();
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    int c = codes[i];
    if (c < 0 || c >= nbins) c = nbins;
    if (lds) atomicAdd(&h[c], 1u); else atomicAdd(&out[c], 1ULL);
  }
  __syncthreads();
  if (lds)
    for (int t = threadIdx.x; t <= nbins; t += 256)
      if (h[t]) atomicAdd(&out[t], (unsigned long long)h[t]);
}

// ================================================================================================
// hash partitioning for shuffles: part[i] = hash(key) % P, counts[P] (int64)
// ================================================================================================
__global__ __launch_bounds__(256) void hash_partition_k(const long long* __restrict__ keys, long n, int P,
                                                        int* __restrict__ part, unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[1024];
  for (int t = threadIdx.x; t < P; t += 256) h[t] = 0;
  __syncthreads();
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int p = (int)(mix64((unsigned long long)keys[i]) % (unsigned long long)P);
    part[i] = p;
    atomicAdd(&h[p], 1u);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < P; t += 256)
    if (h[t]) atomicAdd(&counts[t], (unsigned long long)h[t]);
}
// stable-by-block scatter of row indices into partition order (perm[dst] = i)
__global__ __launch_bounds__(256) void partition_perm_k(const int* __restrict__ part, long n, int P,
                                                        unsigned long long* __restrict__ cursor,
                                                        long long* __restrict__ perm, long rows_per_block) {
  __shared__ unsigned int lc[1024];
  __shared__ unsigned long long lb[1024];
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(n, r0 + rows_per_block);
  for (int t = threadIdx.x; t < P; t += 256) lc[t] = 0;
  __syncthreads();
  for (long i = r0 + threadIdx.x; i < r1; i += 256) atomicAdd(&lc[part[i]], 1u);
  __syncthreads();
  for (int t = threadIdx.x; t < P; t += 256) { lb[t] = lc[t] ? atomicAdd(&cursor[t], (unsigned long long)lc[t]) : 0; lc[t] = 0; }
  __syncthreads();
  for (long i = r0 + threadIdx.x; i < r1; i += 256) {
    const int p = part[i];
    perm[lb[p] + atomicAdd(&lc[p], 1u)] = i;
  }
}

// ================================================================================================
// synthetic (key, value) generator: key = hash(seed, row) % num_keys, value uniform [0,1)
// ================================================================================================
// sparse: the dense key k in [0, num_keys) is replaced by mix64(k + 1) (a bijection): the same
// number of distinct keys spread over the whole int64 range (the general hash path, not the range one)
__global__ __launch_bounds__(256) void fill_kv_k(long long* __restrict__ keys, double* __restrict__ vals, long n,
                                                 long offset, long num_keys, unsigned long long seed, int sparse) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const unsigned long long h = mix64((unsigned long long)(i + offset) * 0x9E3779B97F4A7C15ULL + seed);
    const unsigned long long k = h % (unsigned long long)num_keys;
    keys[i] = (long long)(sparse ? mix64(k + 1ULL) : k);
    vals[i] = (double)(mix64(h ^ 0x632BE59BD9B4E019ULL) >> 11) * (1.0 / 9007199254740992.0);
  }
}

static inline int grid_n(long n) {
  long g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

static long g_expr_spec_launches = 0;  // (tests: the specialised path really ran)

// Host-side match of the specialised shapes: [LDCOL x][LDC c] (either order) then one of
// ADD/SUB/MUL/DIV (x / c with c != 0 only) and an optional CAST_INT, or a single comparison; one
// non-nullable numeric column; numeric (or filter / boolean) output.  Returns 1 and fills S / col / tin.
static int match_affine(const VmProg& P, AffineSpec& S, int& kc) {
  if (P.n_ins < 2 || P.n_ins > 4) return 0;
  auto dec = [&](int pc, int& op, int& d, int& a, int& b, int& k) {
    const int w = P.ins[pc];
    op = w & 0xff; d = (w >> 8) & 0xf; a = (w >> 12) & 0xf; b = (w >> 16) & 0xf; k = (w >> 24) & 0xff;
  };
  int op, d, a, b, k;
  int rcol = -1, rc = -1;
  kc = -1;
  double cval = 0.0;
  int pc = 0;
  for (; pc < P.n_ins && pc < 2; ++pc) {
    dec(pc, op, d, a, b, k);
    if (op == OP_LDCOL && rcol < 0) { rcol = d; kc = k; }
    else if (op == OP_LDC && rc < 0) { rc = d; cval = P.consts[k]; }
    else break;
  }
  if (rcol < 0 || kc < 0 || kc >= VM_COLS || P.valid[kc]) return 0;
  const int ct = P.col_type[kc];
  if (ct != CT_F32 && ct != CT_F64 && ct != CT_I32 && ct != CT_I64) return 0;
  S = AffineSpec{AF_NONE, 0, 0, AC_NONE, P.filter_mode, cval};
  int cur = rcol;
  if (pc < P.n_ins) {
    dec(pc, op, d, a, b, k);
    const bool arith = op == OP_ADD || op == OP_SUB || op == OP_MUL || op == OP_DIV;
    const bool cmp = op == OP_LT || op == OP_LE || op == OP_GT || op == OP_GE || op == OP_EQ || op == OP_NE;
    if ((arith || cmp) && rc >= 0 && ((a == rcol && b == rc) || (a == rc && b == rcol))) {
      S.cl = a == rc ? 1 : 0;
      if (arith) {
        S.op = op == OP_ADD ? AF_ADD : op == OP_SUB ? AF_SUB : op == OP_MUL ? AF_MUL : AF_DIV;
        if (S.op == AF_DIV && (S.cl || cval == 0.0)) return 0;
        if ((S.op == AF_ADD || S.op == AF_MUL) && S.cl) S.cl = 0;  // commutative (same double result)
      } else {
        S.cmp = op == OP_LT ? AC_LT : op == OP_LE ? AC_LE : op == OP_GT ? AC_GT : op == OP_GE ? AC_GE
              : op == OP_EQ ? AC_EQ : AC_NE;
      }
      cur = d;
      ++pc;
    }
  }
  if (pc < P.n_ins && S.cmp == AC_NONE) {
    dec(pc, op, d, a, b, k);
    if (op == OP_CAST_INT && a == cur) { S.cast = 1; cur = d; ++pc; }
  }
  if (pc != P.n_ins || P.out_reg != cur) return 0;
  if (S.op == AF_NONE && S.cmp == AC_NONE && !S.cast) return 0;  // a bare column copy: leave it to the VM
  if (!S.filter && P.out_type != CT_F32 && P.out_type != CT_F64 && P.out_type != CT_I32 && P.out_type != CT_I64 &&
      P.out_type != CT_U8)
    return 0;
  return 1;
}

template <typename TI>
static int launch_affine(const VmProg& P, const AffineSpec& S, int kc, long n, void* out, void* out_valid,
                         hipStream_t s) {
  const TI* in = (const TI*)P.cols[kc];
  const int ot = S.filter ? CT_U8 : P.out_type;
  const size_t osz = ot == CT_F64 || ot == CT_I64 ? 8 : ot == CT_U8 ? 1 : 4;
  if ((uintptr_t)in % (4 * sizeof(TI)) || (uintptr_t)out % (4 * osz) || (out_valid && (uintptr_t)out_valid % 4))
    return -1;  // (a view at an odd offset: the VM handles it)
  const dim3 g(grid_n((n + 3) / 4)), b(256);
  uint8_t* v = (uint8_t*)out_valid;
  switch (ot) {
    case CT_F32: hipLaunchKernelGGL((expr_affine_k<TI, float>), g, b, 0, s, in, n, S, (float*)out, v); break;
    case CT_F64: hipLaunchKernelGGL((expr_affine_k<TI, double>), g, b, 0, s, in, n, S, (double*)out, v); break;
    case CT_I32: hipLaunchKernelGGL((expr_affine_k<TI, int>), g, b, 0, s, in, n, S, (int*)out, v); break;
    case CT_I64: hipLaunchKernelGGL((expr_affine_k<TI, long long>), g, b, 0, s, in, n, S, (long long*)out, v); break;
    default: hipLaunchKernelGGL((expr_affine_k<TI, uint8_t>), g, b, 0, s, in, n, S, (uint8_t*)out, v); break;
  }
  return (int)hipGetLastError();
}

extern "C" {

// prog: packed VmProg bytes (host-built, sizeof must match ptg_vm_prog_size)
int ptg_vm_prog_size() { return (int)sizeof(VmProg); }


int ptg_expr_spec_launches(long* out) {
  *out = g_expr_spec_launches;
  return 0;
}

int ptg_expr_eval(const void* prog, long n, void* out, void* out_valid, hipStream_t s) {
  VmProg P;
  memcpy(&P, prog, sizeof(VmProg));
  const char* se = getenv("PTG_EXPR_SPECIALIZE");  // A/B and tests: 0 = every program through the VM
  const bool spec = !(se && se[0] == '0');
  AffineSpec S;
  int kc;
  if (spec && n > 0 && match_affine(P, S, kc)) {
    int rc = -1;
    switch (P.col_type[kc]) {
      case CT_F32: rc = launch_affine<float>(P, S, kc, n, out, out_valid, s); break;
      case CT_F64: rc = launch_affine<double>(P, S, kc, n, out, out_valid, s); break;
      case CT_I32: rc = launch_affine<int>(P, S, kc, n, out, out_valid, s); break;
      default: rc = launch_affine<long long>(P, S, kc, n, out, out_valid, s); break;
    }
    if (rc >= 0) {
      ++g_expr_spec_launches;
      return rc;
    }
  }
  hipLaunchKernelGGL(expr_eval_k, dim3(grid_n(n)), dim3(256), 0, s, P, n, out, (uint8_t*)out_valid);
  PTG_RETURN_LAUNCH();
}

// indices of set mask rows; block_counts: int[ceil(n/4096)], block_off: i64[same], total: i64[1]
int ptg_compact(const void* mask, long n, void* block_counts, void* block_off, void* total, void* idx_out,
                hipStream_t s) {
  const int nb = (int)((n + CPT_TILE - 1) / CPT_TILE);
  if (nb == 0) return (int)hipMemsetAsync(total, 0, 8, s);
  hipLaunchKernelGGL(compact_count_k, dim3(nb), dim3(256), 0, s, (const uint8_t*)mask, n, (int*)block_counts);
  hipLaunchKernelGGL(scan_excl_k, dim3(1), dim3(256), 0, s, (const int*)block_counts, (long long*)block_off, nb,
                     (long long*)total);
  if (idx_out)
    hipLaunchKernelGGL(compact_write_k, dim3(nb), dim3(256), 0, s, (const uint8_t*)mask, n,
                       (const long long*)block_off, (long long*)idx_out);
  PTG_RETURN_LAUNCH();
}

// nsrc: rows of src (checked builds verify every idx against it)
int ptg_gather_rows(const void* src, const void* idx, long m, int row_bytes, long nsrc, void* dst, hipStream_t s) {
  if (m <= 0) return 0;
  if (row_bytes % 4 == 0) {
    const int rw = row_bytes / 4;
    hipLaunchKernelGGL(gather_rows_k, dim3(grid_n(m * rw)), dim3(256), 0, s, (const uint8_t*)src,
                       (const long long*)idx, m, rw, nsrc, (uint8_t*)dst);
  } else {
    hipLaunchKernelGGL(gather_bytes_k, dim3(grid_n(m * row_bytes)), dim3(256), 0, s, (const uint8_t*)src,
                       (const long long*)idx, m, row_bytes, nsrc, (uint8_t*)dst);
  }
  PTG_RETURN_LAUNCH();
}

// out: double[5] = {sum, count, min, max, nulls}; partial: double[5*1024]
int ptg_reduce_stats(const void* col, int type, const void* valid, long n, int skip_nan, void* partial, void* out,
                     hipStream_t s) {
  int g = grid_n(n);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(reduce_stats_k, dim3(g), dim3(256), 0, s, col, type, (const uint8_t*)valid, n, skip_nan,
                     (double*)partial);
  hipLaunchKernelGGL(reduce_stats_final_k, dim3(1), dim3(64), 0, s, (const double*)partial, g, (double*)out);
  PTG_RETURN_LAUNCH();
}

int ptg_hash_table_init(void* keys, void* tab, long cap, int nv, hipStream_t s) {
  hipLaunchKernelGGL(hash_table_init_k, dim3(grid_n(cap)), dim3(256), 0, s, (long long*)keys, (double*)tab, cap, nv);
  PTG_RETURN_LAUNCH();
}

// vals/valids/types: host arrays of nv entries (device pointers inside)
// est_keys: expected distinct keys (sizes the per-workgroup LDS table: ~2x, 1024..budget slots)
int ptg_hash_agg(const void* keys, long n, const void* const* vals, const void* const* valids, const int* types,
                 int nv, int minmax, void* gkeys, void* gtab, long gcap, void* overflow, long est_keys,
                 hipStream_t s) {
  if (nv > AGG_MAXV || nv < 0) return (int)hipErrorInvalidValue;
  const size_t per_slot = 12 + 12 * (size_t)nv;
  int lcap = 1024;
  while ((long)lcap < 2 * est_keys && (size_t)lcap * 2 * per_slot <= 64 * 1024) lcap *= 2;  // >= 2 workgroups/CU
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)hash_agg_lds_k, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr = true;
  }
  AggIn in;
  for (int j = 0; j < AGG_MAXV; ++j) {
    in.vals[j] = j < nv ? vals[j] : nullptr;
    in.valid[j] = j < nv ? (const uint8_t*)valids[j] : nullptr;
    in.types[j] = j < nv ? types[j] : 0;
  }
  in.nv = nv;
  in.minmax = minmax;
  long rpb = 65536;
  long nb = (n + rpb - 1) / rpb;
  if (nb < 512) { rpb = (n + 511) / 512; if (rpb < 256) rpb = 256; nb = (n + rpb - 1) / rpb; }
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(hash_agg_lds_k, dim3((unsigned)nb), dim3(256), (size_t)lcap * per_slot, s,
                     (const long long*)keys, n, in, (long long*)gkeys, (double*)gtab, gcap, rpb, (int*)overflow, lcap);
  PTG_RETURN_LAUNCH();
}

int ptg_hash_extract(const void* keys, const void* tab, long cap, int nv, void* out_keys, void* out_tab, long out_cap,
                     void* m_out, hipStream_t s) {
  hipLaunchKernelGGL(hash_extract_k, dim3(grid_n(cap)), dim3(256), 0, s, (const long long*)keys, (const double*)tab,
                     cap, nv, (long long*)out_keys, (double*)out_tab, out_cap, (unsigned long long*)m_out);
  PTG_RETURN_LAUNCH();
}

// One radix level (see radix_count_k / radix_scatter_k): tiles described by tstart/trows, digit
// counts at hist[thbase[t] + d*thstride[t]]; pin/pout: PayIn / PayOut structs (host-packed), nv <= 4.
// key32: keys are u32 offsets from kbase (else i64); range: optional per-tile [min, max] (i64 keys only)
int ptg_radix_count(const void* keys, int key32, long kbase, const void* tstart, const void* trows,
                    const void* thbase, const void* thstride, int ntiles, int shift, void* hist, void* range,
                    hipStream_t s) {
  if (ntiles <= 0) return 0;
  if (key32)
    hipLaunchKernelGGL(radix_count_k<unsigned int>, dim3(ntiles), dim3(256), 0, s, (const unsigned int*)keys,
                       (long long)kbase, (const long long*)tstart, (const int*)trows, (const long long*)thbase,
                       (const long long*)thstride, shift, (unsigned int*)hist, (long long*)nullptr);
  else
    hipLaunchKernelGGL(radix_count_k<long long>, dim3(ntiles), dim3(256), 0, s, (const long long*)keys,
                       (long long)kbase, (const long long*)tstart, (const int*)trows, (const long long*)thbase,
                       (const long long*)thstride, shift, (unsigned int*)hist, (long long*)range);
  PTG_RETURN_LAUNCH();
}
int ptg_pay_desc_size() { return (int)sizeof(PayIn); }
int ptg_radix_tile_rows() { return RT; }
// in32 / out32: input / output keys as u32 offsets from kbase_in / kbase_out (else i64); the
// (i64 -> u32) and (u32 -> u32) forms are the compressed-key levels
int ptg_radix_scatter(const void* keys, int in32, long kbase_in, const void* pin_p, int nv, const void* tstart,
                      const void* trows, const void* thbase, const void* thstride, int ntiles, int shift,
                      const void* offs, long n_out, void* okeys, int out32, long kbase_out, const void* pout_p,
                      hipStream_t s) {
  if (ntiles <= 0) return 0;
  if (in32 && !out32) return (int)hipErrorInvalidValue;
  PayIn pin;
  PayOut pout;
  memcpy(&pin, pin_p, sizeof(PayIn));
  memcpy(&pout, pout_p, sizeof(PayOut));
#define PTG_SCATTER3(NV, KI, KO)                                                                             \
  hipLaunchKernelGGL((radix_scatter_k<NV, KI, KO>), dim3(ntiles), dim3(PTG_SCATTER_NT), 0, s, (const KI*)keys, \
                     (long long)kbase_in, pin, (const long long*)tstart, (const int*)trows,                   \
                     (const long long*)thbase, (const long long*)thstride, shift, (const long long*)offs, n_out, \
                     (KO*)okeys, (long long)kbase_out, pout)
#define PTG_SCATTER(NV)                                                                                      \
  if (!out32) PTG_SCATTER3(NV, long long, long long);                                                        \
  else if (!in32) PTG_SCATTER3(NV, long long, unsigned int);                                                 \
  else PTG_SCATTER3(NV, unsigned int, unsigned int)
  switch (nv) {
    case 0: PTG_SCATTER(0); break;
    case 1: PTG_SCATTER(1); break;
    case 2: PTG_SCATTER(2); break;
    case 3: PTG_SCATTER(3); break;
    case 4: PTG_SCATTER(4); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef PTG_SCATTER
#undef PTG_SCATTER3
  PTG_RETURN_LAUNCH();
}
// vals: host array of nv f64 device pointers (payload columns in partition order)
int ptg_part_agg2(const void* okeys, int key32, long kbase, const void* const* vals, int nv, int minmax,
                  const void* pstart, const void* pend,
                  int P, int pcap, void* out_keys, void* out_tab, long out_cap, void* m_out, void* spilled,
                  void* nspill, hipStream_t s) {
  if (nv > PAY_MAX || pcap < 256 || (pcap & (pcap - 1)) || P <= 0) return (int)hipErrorInvalidValue;
  // dynamic LDS for a table of pcap slots (ops/df.py _part_agg_lds mirrors this)
  const long lds = (long)pcap * (8 + 4 + (long)nv * (4 + 8 * (minmax ? 3 : 1)));
  if (lds > 150 * 1024) return (int)hipErrorInvalidValue;
  AggPay pay;
  for (int j = 0; j < PAY_MAX; ++j) pay.vals[j] = j < nv ? (const double*)vals[j] : nullptr;
  const int g = P < 8192 ? P : 8192;
  (void)hipMemsetAsync(m_out, 0, 8, s);  // output / spill counters start at zero (no host fill)
  (void)hipMemsetAsync(nspill, 0, 4, s);
#define PTG_AGG(NV, MM) \
  if (key32) { PTG_AGGK(NV, MM, unsigned int) } else { PTG_AGGK(NV, MM, long long) }
#define PTG_AGGK(NV, MM, KT)                                                                                \
  {                                                                                                         \
    static bool attr = false;                                                                               \
    if (!attr) {                                                                                            \
      (void)hipFuncSetAttribute((const void*)part_agg2_k<NV, MM, KT>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                150 * 1024);                                                                \
      attr = true;                                                                                          \
    }                                                                                                       \
    hipLaunchKernelGGL((part_agg2_k<NV, MM, KT>), dim3(g), dim3(256), (size_t)lds, s, (const KT*)okeys,         \
                       (long long)kbase, pay,                                                              \
                       (const long long*)pstart, (const long long*)pend, P, pcap, (long long*)out_keys,     \
                       (double*)out_tab, out_cap, (unsigned long long*)m_out, (int*)spilled, (int*)nspill); \
  }
  if (minmax) {
    switch (nv) { case 0: PTG_AGG(0, true) break; case 1: PTG_AGG(1, true) break; case 2: PTG_AGG(2, true) break;
                  case 3: PTG_AGG(3, true) break; default: PTG_AGG(4, true) break; }
  } else {
    switch (nv) { case 0: PTG_AGG(0, false) break; case 1: PTG_AGG(1, false) break; case 2: PTG_AGG(2, false) break;
                  case 3: PTG_AGG(3, false) break; default: PTG_AGG(4, false) break; }
  }
#undef PTG_AGG
#undef PTG_AGGK
  PTG_RETURN_LAUNCH();
}

// dense small-range groupBy (range_count_k / range_scatter_k / range_agg_k).  Tiles are
// ptg_range_tile_rows(nv) rows; hist u32[256*ntiles] digit-major, range i64[ntiles][2];
// offs i64[256*ntiles + 1] = exclusive scan of hist with offs[last] = n.  sh <= 12, nv <= 4.
int ptg_range_tile_rows(int nv) { return nv <= 1 ? RGT : (nv == 2 ? RGT / 2 : RGT / 4); }
int ptg_range_count(const void* keys, long n, long lo, int sh, int T, int ntiles, void* hist, void* range,
                    hipStream_t s) {
  if (ntiles <= 0 || T > RGT || sh < 0 || sh > 24) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(range_count_k, dim3(ntiles), dim3(256), 0, s, (const long long*)keys, n, (long long)lo, sh, T,
                     ntiles, (unsigned int*)hist, (long long*)range);
  PTG_RETURN_LAUNCH();
}
int ptg_range_scatter(const void* keys, const void* pin_p, int nv, long n, long lo, int sh, int ntiles,
                      const void* offs, void* okeys, const void* pout_p, hipStream_t s) {
  if (ntiles <= 0 || sh < 0 || sh > 12) return (int)hipErrorInvalidValue;
  PayIn pin;
  PayOut pout;
  memcpy(&pin, pin_p, sizeof(PayIn));
  memcpy(&pout, pout_p, sizeof(PayOut));
#define PTG_RSC(NV, TR)                                                                                       \
  hipLaunchKernelGGL((range_scatter_k<NV, TR>), dim3(ntiles), dim3(512), 0, s, (const long long*)keys, pin, n,   \
                     (long long)lo, sh, ntiles, (const long long*)offs, (unsigned short*)okeys, pout)
  switch (nv) {
    case 0: PTG_RSC(0, RGT); break;
    case 1: PTG_RSC(1, RGT); break;
    case 2: PTG_RSC(2, RGT / 2); break;
    case 3: PTG_RSC(3, RGT / 4); break;
    case 4: PTG_RSC(4, RGT / 4); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef PTG_RSC
  PTG_RETURN_LAUNCH();
}
// coarse level of the two-level dense range groupBy: keys leave as u32 offsets inside 2^sh windows
int ptg_range_scatter32(const void* keys, const void* pin_p, int nv, long n, long lo, int sh, int ntiles,
                        const void* offs, void* okeys, const void* pout_p, hipStream_t s) {
  if (ntiles <= 0 || sh < 0 || sh > 24) return (int)hipErrorInvalidValue;
  PayIn pin;
  PayOut pout;
  memcpy(&pin, pin_p, sizeof(PayIn));
  memcpy(&pout, pout_p, sizeof(PayOut));
#define PTG_RSC(NV, TR)                                                                                       \
  hipLaunchKernelGGL((range_scatter_k<NV, TR, 512, unsigned int>), dim3(ntiles), dim3(512), 0, s,             \
                     (const long long*)keys, pin, n, (long long)lo, sh, ntiles, (const long long*)offs,       \
                     (unsigned int*)okeys, pout)
  switch (nv) {
    case 0: PTG_RSC(0, RGT); break;
    case 1: PTG_RSC(1, RGT); break;
    case 2: PTG_RSC(2, RGT / 2); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef PTG_RSC
  PTG_RETURN_LAUNCH();
}
// fine level: tiles from ptg_seg_plan(.., 256 bins) over the coarse partitions; T = ptg_range_tile_rows(nv)
int ptg_range2_count(const void* okeys, const void* tstart, const void* trows, const void* thbase,
                     const void* thstride, int ntiles, int nv, int sh2, void* hist, hipStream_t s) {
  if (ntiles <= 0) return 0;
  if (sh2 < 0 || sh2 > 12) return (int)hipErrorInvalidValue;
#define PTG_R2C(TR)                                                                                            \
  hipLaunchKernelGGL(range2_count_k<TR>, dim3(ntiles), dim3(256), 0, s, (const unsigned int*)okeys,            \
                     (const long long*)tstart, (const int*)trows, (const long long*)thbase,                    \
                     (const long long*)thstride, sh2, (unsigned int*)hist)
  if (nv <= 1) PTG_R2C(RGT); else PTG_R2C(RGT / 2);
#undef PTG_R2C
  PTG_RETURN_LAUNCH();
}
int ptg_range2_scatter(const void* okeys32, const void* const* vals, int nv, const void* tstart, const void* trows,
                       const void* thbase, const void* thstride, int ntiles, int sh2, const void* offs, long n,
                       void* okeys16, const void* pout_p, hipStream_t s) {
  if (ntiles <= 0) return 0;
  if (sh2 < 0 || sh2 > 12 || nv < 0 || nv > 2) return (int)hipErrorInvalidValue;
  AggPay pin;
  for (int j = 0; j < PAY_MAX; ++j) pin.vals[j] = j < nv ? (const double*)vals[j] : nullptr;
  PayOut pout;
  memcpy(&pout, pout_p, sizeof(PayOut));
#define PTG_R2S(NV, TR)                                                                                        \
  hipLaunchKernelGGL((range2_scatter_k<NV, TR>), dim3(ntiles), dim3(512), 0, s, (const unsigned int*)okeys32,  \
                     pin, (const long long*)tstart, (const int*)trows, (const long long*)thbase,               \
                     (const long long*)thstride, sh2, (const long long*)offs, n, (unsigned short*)okeys16, pout)
  switch (nv) {
    case 0: PTG_R2S(0, RGT); break;
    case 1: PTG_R2S(1, RGT); break;
    default: PTG_R2S(2, RGT / 2); break;
  }
#undef PTG_R2S
  PTG_RETURN_LAUNCH();
}
// nfine fine partitions x chunks workgroups; prow u32[chunks][1+nv][nfine<<sh2], psum f64[chunks][nv][nfine<<sh2]
int ptg_range2_agg(const void* okeys16, const void* const* vals, int nv, const void* fstart, const void* fend,
                   int nfine, int chunks, int sh2, void* prow, void* psum, hipStream_t s) {
  if (nv < 0 || nv > 2 || sh2 < 0 || sh2 > 12 || chunks <= 0 || nfine <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = ((size_t)1 << sh2) * (4 + (size_t)nv * 12);
  if (lds > 150 * 1024) return (int)hipErrorInvalidValue;
  AggPay pay;
  for (int j = 0; j < PAY_MAX; ++j) pay.vals[j] = j < nv ? (const double*)vals[j] : nullptr;
  const long Rw = (long)nfine << sh2;
#define PTG_R2A(NV)                                                                                            \
  {                                                                                                            \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      (void)hipFuncSetAttribute((const void*)range2_agg_k<NV>, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                150 * 1024);                                                                   \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL(range2_agg_k<NV>, dim3((unsigned)nfine * chunks), dim3(256), lds, s,                    \
                       (const unsigned short*)okeys16, pay, (const long long*)fstart, (const long long*)fend,  \
                       chunks, sh2, Rw, (unsigned int*)prow, (double*)psum);                                   \
  }
  switch (nv) { case 0: PTG_R2A(0) break; case 1: PTG_R2A(1) break; default: PTG_R2A(2) break; }
#undef PTG_R2A
  PTG_RETURN_LAUNCH();
}
// vals: host array of nv f64 device pointers (scattered payload); prow u32[chunks][1+nv][256<<sh],
// psum f64[chunks][nv][256<<sh], pmm f64[chunks][2*nv][256<<sh] (minmax only)
int ptg_range_agg(const void* okeys, const void* const* vals, int nv, int minmax, const void* offs, int ntiles,
                  int sh, int chunks, void* prow, void* psum, void* pmm, hipStream_t s) {
  if (nv < 0 || nv > PAY_MAX || sh < 0 || sh > 12 || chunks <= 0 || (minmax && !pmm)) return (int)hipErrorInvalidValue;
  const size_t lds = ((size_t)1 << sh) * (4 + (size_t)nv * (12 + (minmax ? 16 : 0)));
  if (lds > 150 * 1024) return (int)hipErrorInvalidValue;
  AggPay pay;
  for (int j = 0; j < PAY_MAX; ++j) pay.vals[j] = j < nv ? (const double*)vals[j] : nullptr;
#define PTG_RAG(NV, MM)                                                                                       \
  {                                                                                                           \
    static bool attr = false;                                                                                 \
    if (!attr) {                                                                                              \
      (void)hipFuncSetAttribute((const void*)range_agg_k<NV, MM>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                150 * 1024);                                                                  \
      attr = true;                                                                                            \
    }                                                                                                         \
    hipLaunchKernelGGL((range_agg_k<NV, MM>), dim3(chunks, RGB), dim3(256), lds, s, (const unsigned short*)okeys, \
                       pay, (const long long*)offs, ntiles, sh, (unsigned int*)prow, (double*)psum, (double*)pmm); \
  }
  if (minmax) {
    switch (nv) { case 0: PTG_RAG(0, true) break; case 1: PTG_RAG(1, true) break; case 2: PTG_RAG(2, true) break;
                  case 3: PTG_RAG(3, true) break; default: PTG_RAG(4, true) break; }
  } else {
    switch (nv) { case 0: PTG_RAG(0, false) break; case 1: PTG_RAG(1, false) break; case 2: PTG_RAG(2, false) break;
                  case 3: PTG_RAG(3, false) break; default: PTG_RAG(4, false) break; }
  }
#undef PTG_RAG
  PTG_RETURN_LAUNCH();
}
// tiny key range: prow u32[blocks][1+nv][W], psum f64[blocks][nv][W]; a key outside [lo, lo + W)
// sets *err (int, host-zeroed) and is left out.  fast: every value column plain f64 without a
// validity mask (rows_per_block then a multiple of 2048, see small_range_agg_k)
int ptg_small_range_agg(const void* keys, long n, long lo, int W, const void* pin_p, int nv, long rows_per_block,
                        int blocks, void* prow, void* psum, void* err, int fast, hipStream_t s) {
  const size_t lds = (size_t)W * (4 + (size_t)nv * 12);
  if (nv < 0 || nv > PAY_MAX || W <= 0 || blocks <= 0 || lds > 150 * 1024) return (int)hipErrorInvalidValue;
  if (fast && (rows_per_block % 2048 || ((uintptr_t)keys & 15))) return (int)hipErrorInvalidValue;
  PayIn pin;
  memcpy(&pin, pin_p, sizeof(PayIn));
#define PTG_SRA(NV, F)                                                                                       \
  {                                                                                                          \
    static bool attr = false;                                                                                \
    if (!attr) {                                                                                             \
      (void)hipFuncSetAttribute((const void*)small_range_agg_k<NV, F>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                150 * 1024);                                                                 \
      attr = true;                                                                                           \
    }                                                                                                        \
    hipLaunchKernelGGL((small_range_agg_k<NV, F>), dim3(blocks), dim3(256), lds, s, (const long long*)keys, n,  \
                       (long long)lo, W, pin, rows_per_block, (unsigned int*)prow, (double*)psum, (int*)err); \
  }
  if (fast) {
    switch (nv) { case 1: PTG_SRA(1, true) break; case 2: PTG_SRA(2, true) break;
                  case 3: PTG_SRA(3, true) break; case 4: PTG_SRA(4, true) break; default: PTG_SRA(0, false) break; }
  } else {
    switch (nv) { case 0: PTG_SRA(0, false) break; case 1: PTG_SRA(1, false) break; case 2: PTG_SRA(2, false) break;
                  case 3: PTG_SRA(3, false) break; default: PTG_SRA(4, false) break; }
  }
#undef PTG_SRA
  PTG_RETURN_LAUNCH();
}

// sort: keys u64[n] out, range u64[2] (host-initialised {~0, 0})
int ptg_sort_key_prep(const void* col, int type, long n, int desc, void* out, void* range, hipStream_t s) {
  int g = grid_n(n);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(sort_key_prep_k, dim3(g), dim3(256), 0, s, col, type, n, desc, (unsigned long long*)out,
                     (unsigned long long*)range);
  PTG_RETURN_LAUNCH();
}
int ptg_sort_tile_rows() { return ST; }
// hist u32[256 * ntiles] (raw low-byte counts per tile), tmm u64[2 * ntiles] scratch, range u64[2]
// (initialised to ~0 / 0 by the caller)
int ptg_sort_range_count(const void* keys, long n, long xin, void* hist, void* tmm, void* range, hipStream_t s) {
  const int ntiles = (int)((n + ST - 1) / ST);
  if (ntiles <= 0) return 0;
  hipLaunchKernelGGL(sort_range_count_k, dim3(ntiles), dim3(SNT), 0, s, (const unsigned long long*)keys, n,
                     (unsigned long long)xin, (unsigned int*)hist, (unsigned long long*)tmm);
  int g = (ntiles + 255) / 256;
  if (g > 256) g = 256;
  hipLaunchKernelGGL(sort_range_reduce_k, dim3(g), dim3(256), 0, s, (const unsigned long long*)tmm, ntiles,
                     (unsigned long long*)range);
  PTG_RETURN_LAUNCH();
}
// one LSD pass: hist u32[256*ntiles] (digit-major) -> offs i64[256*ntiles] (exclusive scan, host/torch)
int ptg_sort_count(const void* keys, long n, long base, int shift, void* hist, long xin, hipStream_t s) {
  const int ntiles = (int)((n + ST - 1) / ST);
  if (ntiles <= 0) return 0;
  hipLaunchKernelGGL(sort_count_k, dim3(ntiles), dim3(SNT), 0, s, (const unsigned long long*)keys, n,
                     (unsigned long long)base, shift, ntiles, (unsigned int*)hist, (unsigned long long)xin);
  PTG_RETURN_LAUNCH();
}
// v32: payload is u32 (requires n <= 2^32) instead of i64
int ptg_sort_scatter(const void* keys_in, const void* vals_in, long n, long base, int shift, const void* offs,
                     void* keys_out, void* vals_out, int v32, long xin, long xout, hipStream_t s) {
  const int ntiles = (int)((n + ST - 1) / ST);
  if (ntiles <= 0) return 0;
  if (v32 && n > 4294967296L) return (int)hipErrorInvalidValue;
  if (v32)
    hipLaunchKernelGGL((sort_scatter_k<unsigned int>), dim3(ntiles), dim3(SNT), 0, s,
                       (const unsigned long long*)keys_in, (const unsigned int*)vals_in, n, (unsigned long long)base,
                       shift, ntiles, (const long long*)offs, (unsigned long long*)keys_out, (unsigned int*)vals_out,
                       (unsigned long long)xin, (unsigned long long)xout);
  else
    hipLaunchKernelGGL((sort_scatter_k<long long>), dim3(ntiles), dim3(SNT), 0, s,
                       (const unsigned long long*)keys_in, (const long long*)vals_in, n, (unsigned long long)base,
                       shift, ntiles, (const long long*)offs, (unsigned long long*)keys_out, (long long*)vals_out,
                       (unsigned long long)xin, (unsigned long long)xout);
  PTG_RETURN_LAUNCH();
}
int ptg_range_partition(const void* keys, long n, const void* split, int nsplit, void* part, void* counts,
                        hipStream_t s) {
  if (nsplit > 1024 || nsplit < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(range_partition_k, dim3(grid_n(n)), dim3(256), 0, s, (const unsigned long long*)keys, n,
                     (const unsigned long long*)split, nsplit, (int*)part, (unsigned long long*)counts);
  PTG_RETURN_LAUNCH();
}

int ptg_histogram_i32(const void* codes, long n, void* out, int nbins, hipStream_t s) {
  hipLaunchKernelGGL(histogram_k, dim3(grid_n(n)), dim3(256), 0, s, (const int*)codes, n, (unsigned long long*)out,
                     nbins);
  PTG_RETURN_LAUNCH();
}

int ptg_hash_partition(const void* keys, long n, int P, void* part, void* counts, hipStream_t s) {
  if (P > 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(hash_partition_k, dim3(grid_n(n)), dim3(256), 0, s, (const long long*)keys, n, P, (int*)part,
                     (unsigned long long*)counts);
  PTG_RETURN_LAUNCH();
}
int ptg_partition_perm(const void* part, long n, int P, void* cursor, void* perm, hipStream_t s) {
  const long rpb = 16384;
  const long nb = (n + rpb - 1) / rpb;
  hipLaunchKernelGGL(partition_perm_k, dim3((unsigned)(nb < 1 ? 1 : nb)), dim3(256), 0, s, (const int*)part, n, P,
                     (unsigned long long*)cursor, (long long*)perm, rpb);
  PTG_RETURN_LAUNCH();
}

int ptg_fill_synthetic_kv(void* keys, void* vals, long n, long offset, long num_keys, long seed, int sparse,
                          hipStream_t s) {
  hipLaunchKernelGGL(fill_kv_k, dim3(grid_n(n)), dim3(256), 0, s, (long long*)keys, (double*)vals, n, offset, num_keys,
                     (unsigned long long)seed, sparse);
  PTG_RETURN_LAUNCH();
}


// sparse-key mid-cardinality groupBy (hash9_*_k).  Tiles: ptg_hash9_tile_rows(nv) rows, nv <= 2;
// hist u32[512*ntiles] tile-major; offs i64[512*ntiles + 1] from ptg_digit_offsets_b(bins = 512).
int ptg_hash9_tile_rows(int nv) { return nv <= 1 ? H9T : H9T / 2; }
int ptg_hash9_count(const void* keys, long n, int T, int ntiles, void* hist, hipStream_t s) {
  if (ntiles <= 0 || T > H9T || T <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(hash9_count_k, dim3(ntiles), dim3(256), 0, s, (const long long*)keys, n, T, (unsigned int*)hist);
  PTG_RETURN_LAUNCH();
}
int ptg_hash9_scatter(const void* keys, const void* pin_p, int nv, long n, int ntiles, const void* offs, void* okeys,
                      const void* pout_p, hipStream_t s) {
  if (ntiles <= 0) return (int)hipErrorInvalidValue;
  PayIn pin;
  PayOut pout;
  memcpy(&pin, pin_p, sizeof(PayIn));
  memcpy(&pout, pout_p, sizeof(PayOut));
#define PTG_H9S(NV, TR)                                                                                        \
  hipLaunchKernelGGL((hash9_scatter_k<NV, TR>), dim3(ntiles), dim3(512), 0, s, (const long long*)keys, pin, n,  \
                     ntiles, (const long long*)offs, (long long*)okeys, pout)
  switch (nv) {
    case 0: PTG_H9S(0, H9T); break;
    case 1: PTG_H9S(1, H9T); break;
    case 2: PTG_H9S(2, H9T / 2); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef PTG_H9S
  PTG_RETURN_LAUNCH();
}
static size_t h9_lds(int nv, int TS) { return (size_t)TS * (12 + 12 * (size_t)nv); }
// vals: host array of nv f64 device pointers (the scattered payload).  state u64[2] = {groups, error}:
// zeroed here; pkeys i64 / prow u32 / psum f64[nv] / pcnt u32[nv] regions of R = 512*chunks*TS
// entries, pn i32[512*chunks].
int ptg_hash9_agg(const void* okeys, const void* const* vals, int nv, const void* offs, int ntiles, int TS, int chunks,
                  void* pkeys, void* prow, void* psum, void* pcnt, void* pn, void* state, hipStream_t s) {
  if (nv < 0 || nv > 2 || chunks <= 0 || TS < 1024 || (TS & (TS - 1)) || h9_lds(nv, TS) > 150 * 1024)
    return (int)hipErrorInvalidValue;
  (void)hipMemsetAsync(state, 0, 16, s);
  AggPay pay;
  for (int j = 0; j < PAY_MAX; ++j) pay.vals[j] = j < nv ? (const double*)vals[j] : nullptr;
#define PTG_H9A(NV)                                                                                            \
  {                                                                                                            \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      (void)hipFuncSetAttribute((const void*)hash9_agg_k<NV>, hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                150 * 1024);                                                                   \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL((hash9_agg_k<NV>), dim3(chunks, H9B), dim3(1024), h9_lds(NV, TS), s,                    \
                       (const long long*)okeys, pay, (const long long*)offs, ntiles, TS, (long long*)pkeys,    \
                       (unsigned int*)prow, (double*)psum, (unsigned int*)pcnt, (int*)pn,                      \
                       (unsigned long long*)state);                                                            \
  }
  switch (nv) { case 0: PTG_H9A(0) break; case 1: PTG_H9A(1) break; default: PTG_H9A(2) break; }
#undef PTG_H9A
  PTG_RETURN_LAUNCH();
}
int ptg_hash9_merge(const void* pkeys, const void* prow, const void* psum, const void* pcnt, const void* pn, int nv,
                    int TS, int chunks, void* out_keys, void* out_tab, long out_cap, void* state, hipStream_t s) {
  if (nv < 0 || nv > 2 || chunks <= 0 || TS < 1024 || (TS & (TS - 1)) || h9_lds(nv, TS) > 150 * 1024)
    return (int)hipErrorInvalidValue;
#define PTG_H9M(NV)                                                                                            \
  {                                                                                                            \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      (void)hipFuncSetAttribute((const void*)hash9_merge_k<NV>, hipFuncAttributeMaxDynamicSharedMemorySize,    \
                                150 * 1024);                                                                   \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL((hash9_merge_k<NV>), dim3(H9B), dim3(1024), h9_lds(NV, TS), s, (const long long*)pkeys, \
                       (const unsigned int*)prow, (const double*)psum, (const unsigned int*)pcnt,              \
                       (const int*)pn, chunks, TS, (long long*)out_keys, (double*)out_tab, out_cap,            \
                       (unsigned long long*)state);                                                            \
  }
  switch (nv) { case 0: PTG_H9M(0) break; case 1: PTG_H9M(1) break; default: PTG_H9M(2) break; }
#undef PTG_H9M
  PTG_RETURN_LAUNCH();
}
}  // extern "C"

PTG_CHECK_STATUS(df)
