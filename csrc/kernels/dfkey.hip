// Group keys of any column types on the device (Spark groupBy / countDistinct / dropDuplicates over
// several columns or nullable columns: the health table's `subpopulation` has 1,508 empty values,
// infra/local/mysql-database/load_csv.py:49-63).
//
//   key_prep_k      one column -> orderable u64 key per row (the sort order of Spark: ints with the
//                   sign bit flipped, doubles by their ordered bit pattern with a canonical NaN and
//                   -0 -> +0, dictionary codes < 0 = null), a valid flag per row, and the column's
//                   (min, max, null count) over the rows (block reduce + one u64 atomic each)
//   key_pack_k      up to 8 columns -> ONE exact int64 key: each column contributes (key - min), or
//                   its rank in a sorted distinct-key table (`lut`, binary search) when its range is
//                   too wide, with one extra code for null, at a fixed bit offset.  No hashing, so no
//                   collisions: equal tuples <=> equal keys, and the groupBy hash paths take the
//                   combined key as they take a single column.
//   key_unpack_k    the inverse for the (few) result groups: typed values + validity per column
//   agg_finalize_k  the aggregation outputs (count / sum / avg / min / max with Spark's null rules
//                   and integral sums) straight from the f64 partial tables, no host-side tensor ops
//   iota_f64_k, f64_to_i64_k  row ids for representative-row queries (dropDuplicates)
#include "common.h"

namespace ptgk {

enum { KT_F32 = 0, KT_F64 = 1, KT_I32 = 2, KT_I64 = 3, KT_U8 = 4, KT_CODE = 5 };
constexpr int KMAX = 8;
constexpr unsigned long long SIGN = 0x8000000000000000ULL;

PTG_DEV unsigned long long okey(const void* col, int type, long i, bool& null) {
  null = false;
  switch (type) {
    case KT_F32:
    case KT_F64: {
      double x = type == KT_F32 ? (double)((const float*)col)[i] : ((const double*)col)[i];
      if (x != x) x = __builtin_nan("");
      x = x + 0.0;
      const unsigned long long b = (unsigned long long)__double_as_longlong(x);
      return (b >> 63) ? ~b : (b | SIGN);
    }
    case KT_I32: return (unsigned long long)(long long)((const int*)col)[i] ^ SIGN;
    case KT_CODE: {
      const int c = ((const int*)col)[i];
      null = c < 0;
      return null ? 0ULL : (unsigned long long)c;
    }
    case KT_U8: return (unsigned long long)((const uint8_t*)col)[i];
    default: return (unsigned long long)((const long long*)col)[i] ^ SIGN;
  }
}

PTG_DEV unsigned long long wmin(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const unsigned long long t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
  return v;
}
PTG_DEV unsigned long long wmax(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const unsigned long long t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
  return v;
}
PTG_DEV unsigned long long wsumu(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void key_stats_init_k(unsigned long long* st) {
  if (threadIdx.x == 0) { st[0] = ~0ULL; st[1] = 0ULL; st[2] = 0ULL; }
}

// The hash tables of df.hip reserve INT64_MIN as their empty key, and the orderable form maps int 0
// and +0.0 there.  Keys that feed a hash aggregation use the RAW canonical form instead: the int64
// value, the dictionary code, or the canonical double's bits (NaN canonical, -0 -> +0, so the bits
// are never INT64_MIN); mode 2 turns raw canonical keys of the column's type into the orderable form.
PTG_DEV unsigned long long raw_of_orderable(unsigned long long u, int type) {
  switch (type) {
    case KT_F32:
    case KT_F64: return (u >> 63) ? (u & ~SIGN) : ~u;
    case KT_CODE:
    case KT_U8: return u;
    default: return u ^ SIGN;
  }
}
PTG_DEV unsigned long long orderable_of_raw(unsigned long long r, int type) {
  switch (type) {
    case KT_F32:
    case KT_F64: return (r >> 63) ? ~r : (r | SIGN);
    case KT_CODE:
    case KT_U8: return r;
    default: return r ^ SIGN;
  }
}

// mode 0: orderable keys; 1: raw canonical keys; 2: `col` holds raw canonical int64 keys of `type`,
// out = their orderable form.  stats: [min, max, nulls] of the orderable keys (mode 0)
__global__ __launch_bounds__(256) void key_prep_k(const void* __restrict__ col, int type, int mode,
                                                  const uint8_t* __restrict__ valid, long n,
                                                  unsigned long long* __restrict__ out, uint8_t* __restrict__ oks,
                                                  unsigned long long* __restrict__ st) {
  unsigned long long mn = ~0ULL, mx = 0ULL, nn = 0ULL;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    bool null = false;
    unsigned long long u;
    if (mode == 2) u = orderable_of_raw(((const unsigned long long*)col)[i], type);
    else u = okey(col, type, i, null);
    if (valid && !valid[i]) null = true;
    if (null) { u = 0ULL; ++nn; }
    else { mn = u < mn ? u : mn; mx = u > mx ? u : mx; }
    out[i] = (mode == 1 && !null) ? raw_of_orderable(u, type) : u;
    if (oks) oks[i] = null ? 0 : 1;
  }
  __shared__ unsigned long long s[3][4];
  mn = wmin(mn); mx = wmax(mx); nn = wsumu(nn);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { s[0][w] = mn; s[1][w] = mx; s[2][w] = nn; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int j = 1; j < 4; ++j) {
      mn = s[0][j] < mn ? s[0][j] : mn;
      mx = s[1][j] > mx ? s[1][j] : mx;
    }
    nn = s[2][0] + s[2][1] + s[2][2] + s[2][3];
    if (mn != ~0ULL) atomicMin(st + 0, mn);
    if (mx) atomicMax(st + 1, mx);
    if (nn) atomicAdd(st + 2, nn);
  }
}

struct PackDesc {
  int ncols;
  const unsigned long long* u[KMAX];   // orderable keys (key_prep_k)
  const uint8_t* ok[KMAX];             // per-row valid flags (0 = null) or nullptr
  const unsigned long long* lut[KMAX]; // sorted distinct keys (rank coding) or nullptr
  long nlut[KMAX];
  unsigned long long lo[KMAX];         // min key (offset coding)
  unsigned long long nullcode[KMAX];   // code of null (= number of value codes)
  int shift[KMAX], bits[KMAX];
  int type[KMAX];                      // output type of unpack (KT_*)
};

PTG_DEV long lower_bound(const unsigned long long* a, long n, unsigned long long k) {
  long lo = 0, hi = n;
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    if (a[mid] < k) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void key_pack_k(const PackDesc D, long n, long long* __restrict__ out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned long long key = 0ULL;
#pragma unroll
    for (int c = 0; c < KMAX; ++c) {
      if (c >= D.ncols) break;
      const bool null = D.ok[c] && !D.ok[c][i];
      unsigned long long v;
      if (null) v = D.nullcode[c];
      else if (D.lut[c]) v = (unsigned long long)lower_bound(D.lut[c], D.nlut[c], D.u[c][i]);
      else v = D.u[c][i] - D.lo[c];
      key |= v << D.shift[c];
    }
    out[i] = (long long)key;
  }
}

PTG_DEV void store_typed(void* dst, int type, long i, unsigned long long u) {
  switch (type) {
    case KT_F32:
    case KT_F64: {
      const unsigned long long b = (u >> 63) ? (u & ~SIGN) : ~u;
      const double x = __longlong_as_double((long long)b);
      if (type == KT_F32) ((float*)dst)[i] = (float)x; else ((double*)dst)[i] = x;
      break;
    }
    case KT_I32: ((int*)dst)[i] = (int)(long long)(u ^ SIGN); break;
    case KT_CODE: ((int*)dst)[i] = (int)u; break;
    case KT_U8: ((uint8_t*)dst)[i] = (uint8_t)u; break;
    default: ((long long*)dst)[i] = (long long)(u ^ SIGN); break;
  }
}

struct UnpackOut { void* data[KMAX]; uint8_t* valid[KMAX]; };

__global__ __launch_bounds__(256) void key_unpack_k(const long long* __restrict__ keys, long m, const PackDesc D,
                                                    const UnpackOut O) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < m; i += (long)gridDim.x * 256) {
    const unsigned long long key = (unsigned long long)keys[i];
    for (int c = 0; c < D.ncols; ++c) {
      const unsigned long long mask = D.bits[c] >= 64 ? ~0ULL : ((1ULL << D.bits[c]) - 1ULL);
      const unsigned long long v = (key >> D.shift[c]) & mask;
      const bool null = D.ok[c] != nullptr && v == D.nullcode[c];
      unsigned long long u = 0ULL;
      if (!null) u = D.lut[c] ? D.lut[c][v] : v + D.lo[c];
      if (null) {  // the type's zero (a dictionary column's null code is -1)
        switch (D.type[c]) {
          case KT_F32: ((float*)O.data[c])[i] = 0.f; break;
          case KT_F64: ((double*)O.data[c])[i] = 0.0; break;
          case KT_I32: ((int*)O.data[c])[i] = 0; break;
          case KT_CODE: ((int*)O.data[c])[i] = -1; break;
          case KT_U8: ((uint8_t*)O.data[c])[i] = 0; break;
          default: ((long long*)O.data[c])[i] = 0; break;
        }
      } else {
        store_typed(O.data[c], D.type[c], i, u);
      }
      if (O.valid[c]) O.valid[c][i] = null ? 0 : 1;
    }
  }
}

// ---- aggregation outputs --------------------------------------------------------------------------
enum { AF_ROWS = 0, AF_COUNT = 1, AF_SUM_INT = 2, AF_SUM = 3, AF_AVG = 4, AF_MIN = 5, AF_MAX = 6 };
constexpr int AMAX = 16;
struct FinDesc {
  int nout;
  int fn[AMAX], type[AMAX];          // type: output KT_* (min / max of integral sources keep their type)
  const double* s[AMAX];
  const double* c[AMAX];
  const double* mn[AMAX];
  const double* mx[AMAX];
  void* out[AMAX];
  uint8_t* valid[AMAX];
};

__global__ __launch_bounds__(256) void agg_finalize_k(const double* __restrict__ rows, long m, const FinDesc F) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < m; i += (long)gridDim.x * 256) {
    for (int j = 0; j < F.nout; ++j) {
      const int fn = F.fn[j];
      if (fn == AF_ROWS) { ((long long*)F.out[j])[i] = __double2ll_rn(rows[i]); continue; }
      const double c = F.c[j][i];
      const bool has = c > 0.0;
      if (F.valid[j]) F.valid[j][i] = has ? 1 : 0;
      switch (fn) {
        case AF_COUNT: ((long long*)F.out[j])[i] = __double2ll_rn(c); break;
        case AF_SUM_INT: ((long long*)F.out[j])[i] = __double2ll_rn(F.s[j][i]); break;
        case AF_SUM: ((double*)F.out[j])[i] = F.s[j][i]; break;
        case AF_AVG: ((double*)F.out[j])[i] = F.s[j][i] / (c > 1.0 ? c : 1.0); break;
        default: {
          const double v = has ? (fn == AF_MIN ? F.mn[j][i] : F.mx[j][i]) : 0.0;
          switch (F.type[j]) {
            case KT_I32: ((int*)F.out[j])[i] = (int)v; break;
            case KT_I64: ((long long*)F.out[j])[i] = (long long)v; break;
            case KT_F32: ((float*)F.out[j])[i] = (float)v; break;
            default: ((double*)F.out[j])[i] = v; break;
          }
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void iota_f64_k(double* __restrict__ out, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = (double)i;
}
__global__ __launch_bounds__(256) void f64_to_i64_k(const double* __restrict__ in, long long* __restrict__ out,
                                                    long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = (long long)in[i];
}

static unsigned grid_for_n(long n) {
  long g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : g > 4096 ? 4096 : g);
}

}  // namespace ptgk

extern "C" {

int ptg_key_desc_size() { return (int)sizeof(ptgk::PackDesc); }
int ptg_unpack_out_size() { return (int)sizeof(ptgk::UnpackOut); }
int ptg_fin_desc_size() { return (int)sizeof(ptgk::FinDesc); }

int ptg_key_prep(const void* col, int type, int mode, const void* valid, long n, void* out, void* oks, void* stats,
                 hipStream_t s) {
  if (mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ptgk::key_stats_init_k, dim3(1), dim3(64), 0, s, (unsigned long long*)stats);
  if (n > 0)
    hipLaunchKernelGGL(ptgk::key_prep_k, dim3(ptgk::grid_for_n(n)), dim3(256), 0, s, col, type, mode, (const uint8_t*)valid, n,
                       (unsigned long long*)out, (uint8_t*)oks, (unsigned long long*)stats);
  PTG_RETURN_LAUNCH();
}

int ptg_key_pack(const void* desc, long n, void* out, hipStream_t s) {
  const ptgk::PackDesc D = *(const ptgk::PackDesc*)desc;
  if (D.ncols < 1 || D.ncols > ptgk::KMAX) return (int)hipErrorInvalidValue;
  if (n > 0)
    hipLaunchKernelGGL(ptgk::key_pack_k, dim3(ptgk::grid_for_n(n)), dim3(256), 0, s, D, n, (long long*)out);
  PTG_RETURN_LAUNCH();
}

int ptg_key_unpack(const void* keys, long m, const void* desc, const void* outs, hipStream_t s) {
  const ptgk::PackDesc D = *(const ptgk::PackDesc*)desc;
  const ptgk::UnpackOut O = *(const ptgk::UnpackOut*)outs;
  if (D.ncols < 1 || D.ncols > ptgk::KMAX) return (int)hipErrorInvalidValue;
  if (m > 0)
    hipLaunchKernelGGL(ptgk::key_unpack_k, dim3(ptgk::grid_for_n(m)), dim3(256), 0, s, (const long long*)keys, m, D,
                       O);
  PTG_RETURN_LAUNCH();
}

int ptg_agg_finalize(const void* rows, long m, const void* desc, hipStream_t s) {
  const ptgk::FinDesc F = *(const ptgk::FinDesc*)desc;
  if (F.nout < 1 || F.nout > ptgk::AMAX) return (int)hipErrorInvalidValue;
  if (m > 0)
    hipLaunchKernelGGL(ptgk::agg_finalize_k, dim3(ptgk::grid_for_n(m)), dim3(256), 0, s, (const double*)rows, m, F);
  PTG_RETURN_LAUNCH();
}

int ptg_iota_f64(void* out, long n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(ptgk::iota_f64_k, dim3(ptgk::grid_for_n(n)), dim3(256), 0, s, (double*)out, n);
  PTG_RETURN_LAUNCH();
}

int ptg_f64_to_i64(const void* in, void* out, long n, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(ptgk::f64_to_i64_k, dim3(ptgk::grid_for_n(n)), dim3(256), 0, s, (const double*)in,
                       (long long*)out, n);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"

// ---- partition helpers of the shuffle (no torch elementwise kernels on these paths) ---------------
namespace ptgk {
// repartition(n) without columns: row i of rank r goes to (i + r) % world
__global__ __launch_bounds__(256) void rr_part_k(long n, int rank, int world, int* __restrict__ part) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    part[i] = (int)((i + rank) % world);
}
// rows whose flag is set go to partition `value` (orderBy: nulls to the first / last rank)
__global__ __launch_bounds__(256) void part_override_k(int* __restrict__ part, const uint8_t* __restrict__ flag, long n,
                                                       int value) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    if (flag[i]) part[i] = value;
}
}  // namespace ptgk

extern "C" {
int ptg_rr_part(long n, int rank, int world, void* part, hipStream_t s) {
  if (world < 1) return (int)hipErrorInvalidValue;
  if (n > 0) hipLaunchKernelGGL(ptgk::rr_part_k, dim3(ptgk::grid_for_n(n)), dim3(256), 0, s, n, rank, world, (int*)part);
  PTG_RETURN_LAUNCH();
}
int ptg_part_override(void* part, const void* flag, long n, int value, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(ptgk::part_override_k, dim3(ptgk::grid_for_n(n)), dim3(256), 0, s, (int*)part,
                       (const uint8_t*)flag, n, value);
  PTG_RETURN_LAUNCH();
}
}  // extern "C"
