// Small device utilities of the DataFrame engine (gfx950), so that the groupBy / sort / shuffle
// hot paths run only hand-written kernels between their big passes (no rocprim / at::native
// launches): exclusive scans of histograms, int64 min/max, the dense-key extraction that sums the
// per-chunk partial tables and compacts the occupied keys in one go, radix-level tile planning,
// strided sampling and widening / u32-index gathers.
//
// Scans are reduce-then-scan in three launches (block sums -> one-workgroup scan of the block sums
// -> block-local scan + offset): no inter-workgroup waiting, so no launch can hang on a workgroup
// that was never scheduled.
#include "common.h"

namespace {

constexpr int SC_ITEMS = 16;
constexpr int SC_TILE = 256 * SC_ITEMS;

template <typename T>
PTG_DEV long long as_ll(const T* p, long i) { return (long long)p[i]; }

PTG_DEV long long wave_incl_scan(long long v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

PTG_DEV long long wave_sum(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block sums of SC_TILE-element tiles
template <typename T>
__global__ __launch_bounds__(256) void scan_reduce_k(const T* __restrict__ in, long n, long long* __restrict__ bsum) {
  __shared__ long long ws[4];
  const long base = (long)blockIdx.x * SC_TILE;
  long long s = 0;
#pragma unroll
  for (int j = 0; j < SC_ITEMS; ++j) {
    const long i = base + j * 256 + threadIdx.x;
    if (i < n) s += as_ll(in, i);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// exclusive scan of nb block sums in place (one workgroup), total -> *total
__global__ __launch_bounds__(256) void scan_top_k(long long* __restrict__ bsum, int nb, long long* __restrict__ total) {
  __shared__ long long part[256];
  const int per = (nb + 255) / 256;
  const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
  long long s = 0;
  for (int b = b0; b < b1; ++b) s += bsum[b];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long run = 0;
    for (int t = 0; t < 256; ++t) { const long long v = part[t]; part[t] = run; run += v; }
    if (total) *total = run;
  }
  __syncthreads();
  long long run = part[threadIdx.x];
  for (int b = b0; b < b1; ++b) { const long long v = bsum[b]; bsum[b] = run; run += v; }
}

// out[i] = sum_{j<i} in[j] (block offset from the scanned block sums)
template <typename T>
__global__ __launch_bounds__(256) void scan_apply_k(const T* __restrict__ in, long n, const long long* __restrict__ boff,
                                                    long long* __restrict__ out) {
  __shared__ long long wtot[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long base = (long)blockIdx.x * SC_TILE;
  long long run = boff[blockIdx.x];
  for (int j = 0; j < SC_ITEMS; ++j) {
    const long i = base + j * 256 + threadIdx.x;
    const long long v = i < n ? as_ll(in, i) : 0;
    const long long incl = wave_incl_scan(v, lane);
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    long long wb = 0;
    for (int q = 0; q < w; ++q) wb += wtot[q];
    if (i < n) out[i] = run + wb + incl - v;
    run += wtot[0] + wtot[1] + wtot[2] + wtot[3];
    __syncthreads();
  }
}

// ---- int64 min / max over a strided view: elements p[i * stride + off_min] and p[i * stride + off_max]
__global__ __launch_bounds__(256) void minmax_i64_k(const long long* __restrict__ p, long n, long stride, int off_min,
                                                    int off_max, long long* __restrict__ out) {
  long long mn = 0x7fffffffffffffffLL, mx = -0x7fffffffffffffffLL - 1;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    mn = min(mn, p[i * stride + off_min]);
    mx = max(mx, p[i * stride + off_max]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (long long)__shfl_xor(mn, o, 64));
    mx = max(mx, (long long)__shfl_xor(mx, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(out, mn);
    atomicMax(out + 1, mx);
  }
}

__global__ void minmax_init_k(long long* out) {
  if (threadIdx.x == 0) { out[0] = 0x7fffffffffffffffLL; out[1] = -0x7fffffffffffffffLL - 1; }
}

// ---- dense-key extraction: partial tables of C chunks -> compacted groups
// prow: int32 [C][1 + nv][W] (row count, then non-null counts per value column)
// psum: f64  [C][nv][W]; pmm: f64 [C][2 nv][W] (min, max interleaved) or null
struct DenseOut {
  long long* keys;
  double* rows;
  double* sum[4];
  double* cnt[4];
  double* mn[4];
  double* mx[4];
};

PTG_DEV long long dense_rows(const int* __restrict__ prow, int C, int nv, long W, long w) {
  long long c = 0;
  for (int k = 0; k < C; ++k) c += prow[((long)k * (1 + nv)) * W + w];
  return c;
}

__global__ __launch_bounds__(256) void dense_count_k(const int* __restrict__ prow, int C, int nv, long W,
                                                     int* __restrict__ bcount) {
  __shared__ int ws[4];
  const long base = (long)blockIdx.x * SC_TILE;
  int c = 0;
#pragma unroll
  for (int j = 0; j < SC_ITEMS; ++j) {
    const long w = base + j * 256 + threadIdx.x;
    if (w < W && dense_rows(prow, C, nv, W, w) > 0) ++c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcount[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void dense_write_k(const int* __restrict__ prow, const double* __restrict__ psum,
                                                     const double* __restrict__ pmm, int C, int nv, long W,
                                                     long long lo, const long long* __restrict__ boff, DenseOut o) {
  __shared__ int wtot[4];
  const int lane = threadIdx.x & 63, w8 = threadIdx.x >> 6;
  const long base = (long)blockIdx.x * SC_TILE;
  long long run = boff[blockIdx.x];
  for (int j = 0; j < SC_ITEMS; ++j) {
    const long w = base + j * 256 + threadIdx.x;
    const long long rows = w < W ? dense_rows(prow, C, nv, W, w) : 0;
    const bool f = rows > 0;
    const unsigned long long bal = __ballot(f);
    const int pre = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wtot[w8] = __popcll(bal);
    __syncthreads();
    int wb = 0;
    for (int q = 0; q < w8; ++q) wb += wtot[q];
    if (f) {
      const long long d = run + wb + pre;
      o.keys[d] = lo + w;
      o.rows[d] = (double)rows;
      for (int v = 0; v < nv; ++v) {
        long long cn = 0;
        double s = 0.0, mn = INFINITY, mx = -INFINITY;
        for (int k = 0; k < C; ++k) {
          cn += prow[((long)k * (1 + nv) + 1 + v) * W + w];
          s += psum[((long)k * nv + v) * W + w];
          if (pmm) {
            mn = fmin(mn, pmm[((long)k * 2 * nv + 2 * v) * W + w]);
            mx = fmax(mx, pmm[((long)k * 2 * nv + 2 * v + 1) * W + w]);
          }
        }
        o.sum[v][d] = s;
        o.cnt[v][d] = (double)cn;
        o.mn[v][d] = mn;
        o.mx[v][d] = mx;
      }
    }
    run += wtot[0] + wtot[1] + wtot[2] + wtot[3];
    __syncthreads();
  }
}

// ---- radix level planning (ops/df.py _radix_level): per segment its tile count; per tile its
// segment (binary search over the exclusive tile prefix), start row, rows, histogram base/stride
__global__ __launch_bounds__(256) void radix_ntiles_k(const long long* __restrict__ seg_len, int nseg, long long T,
                                                      long long* __restrict__ ntiles) {
  for (int s = blockIdx.x * 256 + threadIdx.x; s < nseg; s += gridDim.x * 256) ntiles[s] = (seg_len[s] + T - 1) / T;
}

__global__ __launch_bounds__(256) void radix_tiles_k(const long long* __restrict__ seg_start,
                                                     const long long* __restrict__ seg_len,
                                                     const long long* __restrict__ ntiles,
                                                     const long long* __restrict__ first, int nseg, long long total,
                                                     long long T, long long* __restrict__ tstart, int* __restrict__ trows,
                                                     long long* __restrict__ thbase, long long* __restrict__ thstride,
                                                     int bins) {
  for (long long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    int lo = 0, hi = nseg - 1;  // last segment with first[s] <= t (and at least one tile)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (first[mid] <= t) lo = mid; else hi = mid - 1;
    }
    int s = lo;
    while (s > 0 && ntiles[s] == 0) --s;  // (empty segments share their successor's first)
    const long long tl = t - first[s];
    const long long st = seg_start[s] + tl * T;
    tstart[t] = st;
    trows[t] = (int)min(T, seg_start[s] + seg_len[s] - st);
    thbase[t] = (long long)bins * first[s] + tl;
    thstride[t] = ntiles[s];
  }
}

// sub-segment (s, d) starts at offs[bins first[s] + d ntiles[s]]; ends where the next one starts
__global__ __launch_bounds__(256) void radix_bounds_k(const long long* __restrict__ offs,
                                                      const long long* __restrict__ first,
                                                      const long long* __restrict__ ntiles, int nseg, long long n_out,
                                                      long long* __restrict__ new_start, long long* __restrict__ new_end,
                                                      long long* __restrict__ new_len, int bins) {
  const long total = (long)nseg * bins;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int s = (int)(i / bins), d = (int)(i - (long)s * bins);
    new_start[i] = offs[(long long)bins * first[s] + d * ntiles[s]];
    long long e = n_out;
    if (i + 1 < total) {
      const int s2 = (int)((i + 1) / bins), d2 = (int)((i + 1) - (long)s2 * bins);
      e = offs[(long long)bins * first[s2] + d2 * ntiles[s2]];
    }
    new_end[i] = e;
    new_len[i] = e - new_start[i];
  }
}

// ---- strided sample copy and u32 -> i64 widening
__global__ __launch_bounds__(256) void strided_copy_i64_k(const long long* __restrict__ src, long stride, long m,
                                                          long long* __restrict__ dst) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < m; i += (long)gridDim.x * 256) dst[i] = src[i * stride];
}

__global__ __launch_bounds__(256) void widen_u32_k(const uint32_t* __restrict__ src, long n, long long* __restrict__ dst) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = (long long)src[i];
}

// ---- gathers of 4- / 8-byte rows by an int64 or u32 row index: one thread per output row, 4 rows
// in flight per thread (the random source reads dominate; no per-element division)
template <typename ROW, typename IDX>
__global__ __launch_bounds__(256) void gather_fixed_k(const ROW* __restrict__ src, const IDX* __restrict__ idx, long m,
                                                      ROW* __restrict__ dst) {
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + 3 * stride < m; i += 4 * stride) {
    const long long a = (long long)idx[i], b = (long long)idx[i + stride], c = (long long)idx[i + 2 * stride],
                    d = (long long)idx[i + 3 * stride];
    const ROW va = src[a], vb = src[b], vc = src[c], vd = src[d];
    dst[i] = va; dst[i + stride] = vb; dst[i + 2 * stride] = vc; dst[i + 3 * stride] = vd;
  }
  for (; i < m; i += stride) dst[i] = src[(long long)idx[i]];
}

// out[0] = sum_i min(x[i], cap)  (the output capacity of the partition aggregation)
__global__ __launch_bounds__(256) void sum_clamp_k(const long long* __restrict__ x, long n, long long cap,
                                                   unsigned long long* __restrict__ out) {
  long long s = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += min(x[i], cap);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)s);
}

inline int grid_for(long n, int cap = 4096) {
  long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

// ---- tile-major digit offsets (radix sort / range groupBy) -------------------------------------
// The count kernels write per-tile 256-bin histograms as one contiguous row per tile, [tile][digit];
// the scatter kernels read their tile's 256 run offsets as one contiguous row.  (Digit-major
// [digit][tile] arrays, which a plain 1-D scan orders correctly, cost every tile 256 partial cache
// lines on both sides: ~8 B of line traffic per sorted row.)  The digit-major exclusive scan over a
// tile-major array is a column scan: colsum_k reduces chunks of TPC tiles per digit into
// csum[digit][chunk], one 1-D exclusive scan of csum (digit-major = the global order) gives every
// (digit, chunk) its base, and colapply_k walks the chunk's tiles again writing running offsets.
constexpr int DO_BINS = 256;

// blockDim.x = number of digits (256, or 512 for the 9-bit hash partition of ptg_hash9_*)
// rot: digit c's counts sit in column (c + rot) % bins of hist (a histogram of raw low key bytes when
// the radix digit is (key - base) & 255: sort_range_count_k)
__global__ __launch_bounds__(512) void colsum_k(const unsigned int* __restrict__ hist, int ntiles, int tpc,
                                                long long* __restrict__ csum, int nch, int rot) {
  const int c = threadIdx.x, ch = blockIdx.x, bins = blockDim.x;
  const int hc = (c + rot) & (bins - 1);
  const int t0 = ch * tpc, t1 = min(ntiles, t0 + tpc);
  long long s = 0;
#pragma unroll 8
  for (int t = t0; t < t1; ++t) s += hist[(long)t * bins + hc];
  csum[(long)c * nch + ch] = s;
}

__global__ __launch_bounds__(512) void colapply_k(const unsigned int* __restrict__ hist, int ntiles, int tpc,
                                                  const long long* __restrict__ cbase, int nch,
                                                  long long* __restrict__ offs, int rot) {
  const int c = threadIdx.x, ch = blockIdx.x, bins = blockDim.x;
  const int hc = (c + rot) & (bins - 1);
  const int t0 = ch * tpc, t1 = min(ntiles, t0 + tpc);
  long long run = cbase[(long)c * nch + ch];
  for (int t0b = t0; t0b < t1; t0b += 8) {  // 8 loads in flight, then the dependent running sum
    unsigned int h[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) h[u] = t0b + u < t1 ? hist[(long)(t0b + u) * bins + hc] : 0u;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (t0b + u < t1) offs[(long)(t0b + u) * bins + c] = run;
      run += h[u];
    }
  }
}


// Small device utilities the DataFrame operators use instead of torch's fill / arange / bitwise
// kernels (the operator profile carries only framework kernels): a typed fill, an int64 iota and the
// inverse of the orderable sort-key transform.
__global__ __launch_bounds__(256) void fill_bytes_k(void* __restrict__ p, long n, int esize, unsigned long long pat) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    switch (esize) {
      case 1: ((uint8_t*)p)[i] = (uint8_t)pat; break;
      case 2: ((uint16_t*)p)[i] = (uint16_t)pat; break;
      case 4: ((uint32_t*)p)[i] = (uint32_t)pat; break;
      default: ((unsigned long long*)p)[i] = pat; break;
    }
  }
}
__global__ __launch_bounds__(256) void iota_i64_k(long long* __restrict__ out, long n, long long start) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = start + i;
}
// orderable u64 (sort_key) -> signed integer value: flip (descending), then the sign bit back
__global__ __launch_bounds__(256) void sort_key_decode_k(const long long* __restrict__ sk, long n, int desc, int out32,
                                                         void* __restrict__ out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const unsigned long long u = (unsigned long long)sk[i];
    const long long x = (long long)((desc ? ~u : u) ^ 0x8000000000000000ULL);
    if (out32) ((int*)out)[i] = (int)x;
    else ((long long*)out)[i] = x;
  }
}

extern "C" {

// out[0..n) = exclusive prefix sum of in (int32 when in64 == 0, else int64); total (optional) =
// the sum.  bsum: int64 workspace of ceil(n / 4096) entries.
// offs i64[256*ntiles] (tile-major) from hist u32[256*ntiles] (tile-major): the digit-major exclusive
// scan.  Three launches with a caller-provided ptg_scan_excl in between (see ops/df.py digit_offsets):
// phase 0 = colsum (csum i64[256*nch]), phase 1 = colapply (cbase = scanned csum).  tpc = tiles per chunk.
// bins: 256 (radix / range passes) or 512 (ptg_hash9_*); hist / offs rows are `bins` wide.
int ptg_digit_offsets_b(int phase, const void* hist, int ntiles, int tpc, void* csum_or_cbase, int nch, void* offs,
                        int bins, int rot, hipStream_t s) {
  if (ntiles <= 0 || tpc <= 0 || nch != (ntiles + tpc - 1) / tpc || (bins != DO_BINS && bins != 2 * DO_BINS))
    return (int)hipErrorInvalidValue;
  if (phase == 0)
    hipLaunchKernelGGL(colsum_k, dim3(nch), dim3(bins), 0, s, (const unsigned int*)hist, ntiles, tpc,
                       (long long*)csum_or_cbase, nch, rot);
  else
    hipLaunchKernelGGL(colapply_k, dim3(nch), dim3(bins), 0, s, (const unsigned int*)hist, ntiles, tpc,
                       (const long long*)csum_or_cbase, nch, (long long*)offs, rot);
  PTG_RETURN_LAUNCH();
}
int ptg_digit_offsets(int phase, const void* hist, int ntiles, int tpc, void* csum_or_cbase, int nch, void* offs,
                      int rot, hipStream_t s) {
  return ptg_digit_offsets_b(phase, hist, ntiles, tpc, csum_or_cbase, nch, offs, DO_BINS, rot, s);
}

int ptg_scan_excl(const void* in, int in64, long n, void* out, void* total, void* bsum, hipStream_t s) {
  if (n <= 0) {
    if (total) return (int)hipMemsetAsync(total, 0, 8, s);
    return 0;
  }
  const int nb = (int)((n + SC_TILE - 1) / SC_TILE);
  if (in64) hipLaunchKernelGGL(scan_reduce_k<long long>, dim3(nb), dim3(256), 0, s, (const long long*)in, n, (long long*)bsum);
  else hipLaunchKernelGGL(scan_reduce_k<int>, dim3(nb), dim3(256), 0, s, (const int*)in, n, (long long*)bsum);
  hipLaunchKernelGGL(scan_top_k, dim3(1), dim3(256), 0, s, (long long*)bsum, nb, (long long*)total);
  if (in64)
    hipLaunchKernelGGL(scan_apply_k<long long>, dim3(nb), dim3(256), 0, s, (const long long*)in, n,
                       (const long long*)bsum, (long long*)out);
  else
    hipLaunchKernelGGL(scan_apply_k<int>, dim3(nb), dim3(256), 0, s, (const int*)in, n, (const long long*)bsum,
                       (long long*)out);
  PTG_RETURN_LAUNCH();
}

int ptg_scan_ws_elems(long n) { return (int)((n + SC_TILE - 1) / SC_TILE); }

// out[0] = min over p[i*stride + off_min], out[1] = max over p[i*stride + off_max], i < n
int ptg_minmax_i64(const void* p, long n, long stride, int off_min, int off_max, void* out, hipStream_t s) {
  hipLaunchKernelGGL(minmax_init_k, dim3(1), dim3(64), 0, s, (long long*)out);
  if (n > 0)
    hipLaunchKernelGGL(minmax_i64_k, dim3(grid_for(n, 1024)), dim3(256), 0, s, (const long long*)p, n, stride, off_min,
                       off_max, (long long*)out);
  PTG_RETURN_LAUNCH();
}

// fold the C partial tables of a direct-indexed aggregation into ceil(C / F) tables (sums of F
// consecutive chunks, in chunk order): dense_count_k / dense_write_k parallelise over keys only, so
// with a narrow key range (W ~ 1K: one workgroup) and many chunks (small_range_agg_k: one per
// workgroup of the pass) their per-key loop over C partials was a latency-bound serial tail.
// grid (ceil(W / 256), ceil(C / F)); prow u32[C][1+nv][W], psum f64[C][nv][W] -> orow / osum.
__global__ __launch_bounds__(256) void dense_fold_k(const unsigned int* __restrict__ prow, const double* __restrict__ psum,
                                                    int C, int nv, long W, int F, unsigned int* __restrict__ orow,
                                                    double* __restrict__ osum) {
  const long w = (long)blockIdx.x * 256 + threadIdx.x;
  if (w >= W) return;
  const int c2 = blockIdx.y, k0 = c2 * F, k1 = min(C, k0 + F);
  for (int q = 0; q <= nv; ++q) {
    unsigned int acc[4] = {0u, 0u, 0u, 0u};
    int k = k0;
    for (; k + 4 <= k1; k += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += prow[((long)(k + u) * (1 + nv) + q) * W + w];
    }
    for (; k < k1; ++k) acc[0] += prow[((long)k * (1 + nv) + q) * W + w];
    orow[((long)c2 * (1 + nv) + q) * W + w] = acc[0] + acc[1] + acc[2] + acc[3];
  }
  for (int v = 0; v < nv; ++v) {
    double acc = 0.0;  // one accumulator in chunk order: the same sum as the unfolded extract
    for (int k = k0; k < k1; ++k) acc += psum[((long)k * nv + v) * W + w];
    osum[((long)c2 * nv + v) * W + w] = acc;
  }
}

int ptg_dense_fold(const void* prow, const void* psum, int C, int nv, long W, int F, void* orow, void* osum,
                   hipStream_t s) {
  if (nv < 0 || nv > 4 || C < 1 || F < 1 || W <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((W + 255) / 256), (unsigned)((C + F - 1) / F));
  hipLaunchKernelGGL(dense_fold_k, grid, dim3(256), 0, s, (const unsigned int*)prow, (const double*)psum, C, nv, W, F,
                     (unsigned int*)orow, (double*)osum);
  PTG_RETURN_LAUNCH();
}

// dense-key groups: see DenseOut.  Pass 1 (counts=1): block counts of occupied keys -> bcount
// (int32[nb]), boff (int64[nb]) scanned, total (int64[1]).  Pass 2 (counts=0): writes the outputs
// (capacity = total; the host allocates after reading total).  outs: host array of 2 + 4 * 4 device
// pointers {keys, rows, sum0..3, cnt0..3, min0..3, max0..3}.
int ptg_dense_extract(const void* prow, const void* psum, const void* pmm, int C, int nv, long W, long lo,
                      void* bcount, void* boff, void* total, const void* outs, int pass, hipStream_t s) {
  if (nv < 0 || nv > 4 || C < 1) return (int)hipErrorInvalidValue;
  const int nb = (int)((W + SC_TILE - 1) / SC_TILE);
  if (nb == 0) return (int)hipMemsetAsync(total, 0, 8, s);
  if (pass == 0) {  // block counts only (the caller scans them: any W)
    hipLaunchKernelGGL(dense_count_k, dim3(nb), dim3(256), 0, s, (const int*)prow, C, nv, W, (int*)bcount);
    PTG_RETURN_LAUNCH();
  }
  if (pass == 1 && nb > SC_TILE) return (int)hipErrorInvalidValue;  // one workgroup tile scans the block counts
  if (pass == 1) {
    hipLaunchKernelGGL(dense_count_k, dim3(nb), dim3(256), 0, s, (const int*)prow, C, nv, W, (int*)bcount);
    hipLaunchKernelGGL(scan_reduce_k<int>, dim3(1), dim3(256), 0, s, (const int*)bcount, (long)nb, (long long*)total);
    // boff = exclusive scan of the block counts (nb < 2^31 / 4096: one reduce tile holds them)
    (void)hipMemsetAsync(boff, 0, 8, s);
    hipLaunchKernelGGL(scan_apply_k<int>, dim3((nb + SC_TILE - 1) / SC_TILE), dim3(256), 0, s, (const int*)bcount,
                       (long)nb, (const long long*)boff, (long long*)boff);
    PTG_RETURN_LAUNCH();
  }
  const unsigned long long* o = (const unsigned long long*)outs;
  DenseOut d;
  d.keys = (long long*)o[0];
  d.rows = (double*)o[1];
  for (int v = 0; v < 4; ++v) {
    d.sum[v] = (double*)o[2 + v];
    d.cnt[v] = (double*)o[6 + v];
    d.mn[v] = (double*)o[10 + v];
    d.mx[v] = (double*)o[14 + v];
  }
  hipLaunchKernelGGL(dense_write_k, dim3(nb), dim3(256), 0, s, (const int*)prow, (const double*)psum,
                     (const double*)pmm, C, nv, W, (long long)lo, (const long long*)boff, d);
  PTG_RETURN_LAUNCH();
}

// radix level planning.  step 0: ntiles[s] = ceil(seg_len[s] / T); the caller then scans ntiles ->
// first (+ total) and seg_len -> n_out.  step 1: per-tile arrays for `total` tiles.
static int seg_plan(const void* seg_start, const void* seg_len, int nseg, long T, void* ntiles, const void* first,
                    long total, void* tstart, void* trows, void* thbase, void* thstride, int step, int bins,
                    hipStream_t s) {
  if (step == 0) {
    if (nseg > 0)
      hipLaunchKernelGGL(radix_ntiles_k, dim3(grid_for(nseg)), dim3(256), 0, s, (const long long*)seg_len, nseg,
                         (long long)T, (long long*)ntiles);
  } else if (total > 0) {
    hipLaunchKernelGGL(radix_tiles_k, dim3(grid_for(total)), dim3(256), 0, s, (const long long*)seg_start,
                       (const long long*)seg_len, (const long long*)ntiles, (const long long*)first, nseg,
                       (long long)total, (long long)T, (long long*)tstart, (int*)trows, (long long*)thbase,
                       (long long*)thstride, bins);
  }
  PTG_RETURN_LAUNCH();
}
int ptg_radix_plan(const void* seg_start, const void* seg_len, int nseg, long T, void* ntiles, const void* first,
                   long total, void* tstart, void* trows, void* thbase, void* thstride, int step, hipStream_t s) {
  return seg_plan(seg_start, seg_len, nseg, T, ntiles, first, total, tstart, trows, thbase, thstride, step, 64, s);
}
// the same tile plan for `bins`-way segmented passes (the 256-way level of the dense range groupBy)
int ptg_seg_plan(const void* seg_start, const void* seg_len, int nseg, long T, void* ntiles, const void* first,
                 long total, void* tstart, void* trows, void* thbase, void* thstride, int step, int bins,
                 hipStream_t s) {
  return seg_plan(seg_start, seg_len, nseg, T, ntiles, first, total, tstart, trows, thbase, thstride, step, bins, s);
}

static int seg_bounds(const void* offs, const void* first, const void* ntiles, int nseg, long n_out, void* new_start,
                      void* new_end, void* new_len, int bins, hipStream_t s) {
  if (nseg > 0)
    hipLaunchKernelGGL(radix_bounds_k, dim3(grid_for((long)nseg * bins)), dim3(256), 0, s, (const long long*)offs,
                       (const long long*)first, (const long long*)ntiles, nseg, (long long)n_out,
                       (long long*)new_start, (long long*)new_end, (long long*)new_len, bins);
  PTG_RETURN_LAUNCH();
}
int ptg_radix_bounds(const void* offs, const void* first, const void* ntiles, int nseg, long n_out, void* new_start,
                     void* new_end, void* new_len, hipStream_t s) {
  return seg_bounds(offs, first, ntiles, nseg, n_out, new_start, new_end, new_len, 64, s);
}
int ptg_seg_bounds(const void* offs, const void* first, const void* ntiles, int nseg, long n_out, void* new_start,
                   void* new_end, void* new_len, int bins, hipStream_t s) {
  return seg_bounds(offs, first, ntiles, nseg, n_out, new_start, new_end, new_len, bins, s);
}

int ptg_sum_clamp_i64(const void* x, long n, long cap, void* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, 8, s);
  if (n > 0)
    hipLaunchKernelGGL(sum_clamp_k, dim3(grid_for(n, 1024)), dim3(256), 0, s, (const long long*)x, n, (long long)cap,
                       (unsigned long long*)out);
  PTG_RETURN_LAUNCH();
}

int ptg_strided_copy_i64(const void* src, long stride, long m, void* dst, hipStream_t s) {
  if (m > 0)
    hipLaunchKernelGGL(strided_copy_i64_k, dim3(grid_for(m)), dim3(256), 0, s, (const long long*)src, stride, m,
                       (long long*)dst);
  PTG_RETURN_LAUNCH();
}

int ptg_widen_u32(const void* src, long n, void* dst, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(widen_u32_k, dim3(grid_for(n)), dim3(256), 0, s, (const uint32_t*)src, n, (long long*)dst);
  PTG_RETURN_LAUNCH();
}

// dst[i] = src[idx[i]] for 4- or 8-byte rows; idx int64 (idx32 == 0) or u32 (idx32 == 1)
int ptg_gather_fixed(const void* src, const void* idx, int idx32, long m, int row_bytes, void* dst, hipStream_t s) {
  if (m <= 0) return 0;
  const int g = grid_for(m, 8192);
  if (row_bytes == 8) {
    if (idx32) hipLaunchKernelGGL((gather_fixed_k<unsigned long long, uint32_t>), dim3(g), dim3(256), 0, s,
                                  (const unsigned long long*)src, (const uint32_t*)idx, m, (unsigned long long*)dst);
    else hipLaunchKernelGGL((gather_fixed_k<unsigned long long, long long>), dim3(g), dim3(256), 0, s,
                            (const unsigned long long*)src, (const long long*)idx, m, (unsigned long long*)dst);
  } else if (row_bytes == 4) {
    if (idx32) hipLaunchKernelGGL((gather_fixed_k<uint32_t, uint32_t>), dim3(g), dim3(256), 0, s, (const uint32_t*)src,
                                  (const uint32_t*)idx, m, (uint32_t*)dst);
    else hipLaunchKernelGGL((gather_fixed_k<uint32_t, long long>), dim3(g), dim3(256), 0, s, (const uint32_t*)src,
                            (const long long*)idx, m, (uint32_t*)dst);
  } else {
    return (int)hipErrorInvalidValue;
  }
  PTG_RETURN_LAUNCH();
}


int ptg_fill_bytes(void* p, long n, int esize, long pat, hipStream_t s) {
  if (n <= 0) return 0;
  if (esize != 1 && esize != 2 && esize != 4 && esize != 8) return (int)hipErrorInvalidValue;
  const long g = std::min<long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(fill_bytes_k, dim3((unsigned)g), dim3(256), 0, s, p, n, esize, (unsigned long long)pat);
  PTG_RETURN_LAUNCH();
}

int ptg_iota_i64(void* out, long n, long start, hipStream_t s) {
  if (n <= 0) return 0;
  const long g = std::min<long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(iota_i64_k, dim3((unsigned)g), dim3(256), 0, s, (long long*)out, n, (long long)start);
  PTG_RETURN_LAUNCH();
}

int ptg_sort_key_decode(const void* sk, long n, int desc, int out32, void* out, hipStream_t s) {
  if (n <= 0) return 0;
  const long g = std::min<long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(sort_key_decode_k, dim3((unsigned)g), dim3(256), 0, s, (const long long*)sk, n, desc, out32, out);
  PTG_RETURN_LAUNCH();
}
}  // extern "C"
