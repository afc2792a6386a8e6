// Spark-ML kernels (gfx950): feature assembly, k-means Lloyd iteration, silhouette.
//
//   assemble_features   StringIndexer code -> OneHotEncoder vector (repeated R times, the
//                       MEASURE_NAME_WEIGHT trick of k_means.py:56-64) + numeric columns ->
//                       row-major fp32 feature matrix (VectorAssembler, k_means.py:64-68)
//   kmeans_assign_accum fused assignment (argmin ||x-c||^2) + per-cluster sum/count/cost
//                       accumulation; centers staged in LDS; per-workgroup partial sums in LDS,
//                       one global atomic per (cluster, feature) per workgroup (KMeans.fit,
//                       k_means.py:83-87; Spark's treeAggregate becomes LDS+atomics, then one RCCL
//                       all-reduce of k*d+k floats across ranks)
//   kmeans_update       centers = sums / counts (empty clusters keep their center)
//   silhouette          Spark ClusteringEvaluator (squared Euclidean) closed form from per-cluster
//                       count / sum vector / sum of squared norms (spark_workload_to_cloud_k8s.py:141-144)
#include "common.h"
#include <cstring>

// one-hot segment: out[row][off + r*V + code] = 1 for r < R (code in [0, V); code == V or < 0 -> no hot)
// numeric segment:  out[row][off] = val (f64 or f32)
struct AsmDesc {
  int nseg;
  int kind[8];     // 0 = onehot(i32 codes), 1 = f64 scalar, 2 = f32 scalar
  const void* src[8];
  int off[8];
  int V[8];
  int R[8];
};

__global__ __launch_bounds__(256) void assemble_k(AsmDesc d, long n, int D, float* __restrict__ out) {
  const long total = n * (long)D;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) out[t] = 0.f;
}
__global__ __launch_bounds__(256) void assemble_fill_k(AsmDesc d, long n, int D, float* __restrict__ out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float* row = out + i * (long)D;
    for (int s = 0; s < d.nseg; ++s) {
      if (d.kind[s] == 0) {
        const int c = ((const int*)d.src[s])[i];
        if (c >= 0 && c < d.V[s])
          for (int r = 0; r < d.R[s]; ++r) row[d.off[s] + r * d.V[s] + c] = 1.f;
      } else if (d.kind[s] == 1) {
        row[d.off[s]] = (float)((const double*)d.src[s])[i];
      } else {
        row[d.off[s]] = ((const float*)d.src[s])[i];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// K-means Lloyd step on the matrix cores.  argmin_c ||x - c||^2 = argmin_c (||c||^2 - 2 x.c): the
// x.c products of a 64-row tile against every center are exact-f32 MFMA (v_mfma_f32_16x16x4_f32,
// bit-for-bit an fmaf chain, cdna_hip_programming.md 'FP32-input MFMA'): each wave owns 16 rows,
// the 4 waves share each 16-center block (B operand read straight from L1/L2, k*D floats), two
// independent accumulators hide the 40-cycle MFMA latency.  The 16 candidate distances of a row
// live on 16 lanes and are min-reduced with xor shuffles (ties -> lower center, as the scalar
// loop).  Per-cluster sums/counts accumulate in LDS when k*D fits, else with global atomics;
// zero features (one-hot blocks) are skipped either way.  No k or k*D limit; D > KM_DMAX takes the
// chunked variant below.
// `done` (device flag) turns every launch of a converged fit into a no-op, so the host can queue
// several iterations without reading the convergence test back (ml/clustering.py).
// ------------------------------------------------------------------------------------------------
#define KM_ROWS 64
#define KM_DMAX 576
typedef float km_f4 __attribute__((ext_vector_type(4)));

template <bool ACC_LDS>
__global__ __launch_bounds__(256) void kmeans_mfma_k(const float* __restrict__ X, long n, int D, int DP,
                                                     const float* __restrict__ C, const float* __restrict__ cn, int k,
                                                     int* __restrict__ assign, float* __restrict__ mind,
                                                     float* __restrict__ sums, float* __restrict__ counts,
                                                     double* __restrict__ cost, const float* __restrict__ weights,
                                                     const int* __restrict__ done) {
  if (done && *done) return;
  extern __shared__ __align__(16) float km_lds[];
  const int S = DP + 1;  // odd row stride: the 16 rows of an A fragment hit 16 different banks
  float* xs = km_lds;                   // [KM_ROWS][S]
  float* sacc = xs + KM_ROWS * S;       // [k][D] (ACC_LDS)
  float* scnt = sacc + (ACC_LDS ? (long)k * D : 0);  // [k] (ACC_LDS)
  __shared__ int sarg[KM_ROWS];
  __shared__ float sw[KM_ROWS];
  __shared__ float scost[4];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, c16 = l & 15;
  if (ACC_LDS && sums) {
    for (long t = tid; t < (long)k * D; t += 256) sacc[t] = 0.f;
    for (int t = tid; t < k; t += 256) scnt[t] = 0.f;
  }
  double mycost = 0.0;
  const long ntile = (n + KM_ROWS - 1) / KM_ROWS;
  for (long tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const long r0 = tile * KM_ROWS;
    __syncthreads();
    for (int t = tid; t < KM_ROWS * DP; t += 256) {
      const int r = t / DP, d = t - r * DP;
      xs[r * S + d] = (r0 + r < n && d < D) ? X[(r0 + r) * D + d] : 0.f;
    }
    __syncthreads();
    const float* xa = xs + (16 * w + c16) * S + g;
    float best[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    int arg[4] = {0, 0, 0, 0};
    for (int cb = 0; cb < k; cb += 16) {
      const int col = cb + c16;
      const bool cv = col < k;
      const float* cp = C + (long)(cv ? col : 0) * D + g;
      km_f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int d0 = 0; d0 < DP; d0 += 8) {
        const float b0 = (cv && d0 + g < D) ? cp[d0] : 0.f;
        const float b1 = (cv && d0 + 4 + g < D) ? cp[d0 + 4] : 0.f;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[d0], b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[d0 + 4], b1, acc1, 0, 0, 0);
      }
      const float cc = cv ? cn[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // C/D map: row 4g+i, column c16
        float v = cv ? cc - 2.f * (acc0[i] + acc1[i]) : INFINITY;
        int a = col;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const float ov = __shfl_xor(v, o, 64);
          const int oa = __shfl_xor(a, o, 64);
          if (ov < v || (ov == v && oa < a)) { v = ov; a = oa; }
        }
        if (v < best[i]) { best[i] = v; arg[i] = a; }
      }
    }
    // lanes with c16 < 4 finish row 4g + c16 of this wave
    if (c16 < 4) {
      const int r = 16 * w + 4 * g + c16;
      float bsel = best[0];
      int asel = arg[0];
#pragma unroll
      for (int i = 1; i < 4; ++i)
        if (c16 == i) { bsel = best[i]; asel = arg[i]; }
      const long row = r0 + r;
      float wt = 0.f;
      if (row < n) {
        float xn = 0.f;
        for (int d = 0; d < D; ++d) xn = fmaf(xs[r * S + d], xs[r * S + d], xn);
        const float dist = fmaxf(xn + bsel, 0.f);
        wt = weights ? weights[row] : 1.f;
        if (assign) assign[row] = asel;
        if (mind) mind[row] = dist;
        mycost += (double)dist * wt;
      }
      sarg[r] = asel;
      sw[r] = wt;
    }
    __syncthreads();
    if (sums) {  // each wave adds its 16 rows: lanes stride over the features (coalesced)
      for (int rr = 0; rr < 16; ++rr) {
        const int r = 16 * w + rr;
        const float wt = sw[r];
        if (wt == 0.f) continue;
        const int a = sarg[r];
        for (int d = l; d < D; d += 64) {
          const float v = xs[r * S + d] * wt;
          if (v != 0.f) {
            if (ACC_LDS) atomicAdd(&sacc[a * D + d], v);
            else atomicAdd(&sums[(long)a * D + d], v);
          }
        }
        if (l == 0) {
          if (ACC_LDS) atomicAdd(&scnt[a], wt);
          else atomicAdd(&counts[a], wt);
        }
      }
    }
  }
  const float c32 = block_sum256((float)mycost, scost);
  if (tid == 0 && cost) atomicAdd(cost, (double)c32);
  if (ACC_LDS && sums) {
    __syncthreads();
    for (long t = tid; t < (long)k * D; t += 256)
      if (sacc[t] != 0.f) atomicAdd(&sums[t], sacc[t]);
    for (int t = tid; t < k; t += 256)
      if (scnt[t] != 0.f) atomicAdd(&counts[t], scnt[t]);
  }
}

// new centers + their squared norms; moved[0] = max squared center shift (Spark's tol test);
// sums/counts are re-zeroed for the next iteration once read.
__global__ __launch_bounds__(256) void kmeans_update_k(float* __restrict__ sums, float* __restrict__ counts,
                                                       float* __restrict__ C, float* __restrict__ cn, int k, int D,
                                                       float* __restrict__ moved, const int* __restrict__ done) {
  if (done && *done) return;
  __shared__ float sh[2][256];
  const int c = blockIdx.x;
  float s2 = 0.f, nn = 0.f;
  const float cnt = counts[c];
  for (int j = threadIdx.x; j < D; j += 256) {
    const float old = C[(long)c * D + j];
    const float nw = cnt > 0.f ? sums[(long)c * D + j] / cnt : old;
    C[(long)c * D + j] = nw;
    sums[(long)c * D + j] = 0.f;
    s2 += (nw - old) * (nw - old);
    nn = fmaf(nw, nw, nn);
  }
  sh[0][threadIdx.x] = s2;
  sh[1][threadIdx.x] = nn;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) { sh[0][threadIdx.x] += sh[0][threadIdx.x + o]; sh[1][threadIdx.x] += sh[1][threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    atomicMax((unsigned int*)moved, __float_as_uint(sh[0][0]));  // non-negative floats order as uints
    if (cn) cn[c] = sh[1][0];
    counts[c] = 0.f;
  }
}

// convergence test on the device: state[0] = done, state[1] = iterations run
__global__ void kmeans_check_k(float* __restrict__ moved, float tol2, int* __restrict__ state) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || state[0]) return;
  state[1] += 1;
  if (*moved <= tol2) state[0] = 1;
  *moved = 0.f;
}

__global__ __launch_bounds__(256) void center_norms_k(const float* __restrict__ C, int k, int D, float* __restrict__ cn) {
  for (int c = blockIdx.x * 256 + threadIdx.x; c < k; c += gridDim.x * 256) {
    float nn = 0.f;
    for (int j = 0; j < D; ++j) nn = fmaf(C[(long)c * D + j], C[(long)c * D + j], nn);
    cn[c] = nn;
  }
}

// Silhouette (Spark ClusteringEvaluator, squared Euclidean) summed over points, on the matrix cores:
// sum_j ||x - x_j||^2 over cluster c = n_c ||x||^2 - 2 x.S_c + Q_c, so every point needs x.S_c for
// all clusters — the same MFMA tile product as kmeans_mfma_k with the centers replaced by the
// cluster sum vectors S.  a = own-cluster mean distance, b = min over the other non-empty clusters.
__global__ __launch_bounds__(256) void silhouette_mfma_k(const float* __restrict__ X, const int* __restrict__ assign,
                                                         const float* __restrict__ Sv, const float* __restrict__ Q,
                                                         const float* __restrict__ cnt, long n, int D, int DP, int k,
                                                         double* __restrict__ out) {
  extern __shared__ __align__(16) float km_lds[];
  const int S = DP + 1;
  float* xs = km_lds;
  __shared__ float sxn[KM_ROWS];
  __shared__ float scr[4];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, c16 = l & 15;
  double acc = 0.0;
  const long ntile = (n + KM_ROWS - 1) / KM_ROWS;
  for (long tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const long r0 = tile * KM_ROWS;
    __syncthreads();
    for (int t = tid; t < KM_ROWS * DP; t += 256) {
      const int r = t / DP, d = t - r * DP;
      xs[r * S + d] = (r0 + r < n && d < D) ? X[(r0 + r) * D + d] : 0.f;
    }
    __syncthreads();
    if (tid < KM_ROWS) {
      float xn = 0.f;
      for (int d = 0; d < D; ++d) xn = fmaf(xs[tid * S + d], xs[tid * S + d], xn);
      sxn[tid] = xn;
    }
    __syncthreads();
    const float* xa = xs + (16 * w + c16) * S + g;
    float xn[4], a_own[4], bmin[4];
    int own[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * w + 4 * g + i;
      xn[i] = sxn[r];
      own[i] = r0 + r < n ? assign[r0 + r] : -1;
      a_own[i] = 0.f;
      bmin[i] = INFINITY;
    }
    for (int cb = 0; cb < k; cb += 16) {
      const int col = cb + c16;
      const bool cv = col < k;
      const float* sp = Sv + (long)(cv ? col : 0) * D + g;
      km_f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int d0 = 0; d0 < DP; d0 += 8) {
        const float b0 = (cv && d0 + g < D) ? sp[d0] : 0.f;
        const float b1 = (cv && d0 + 4 + g < D) ? sp[d0 + 4] : 0.f;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[d0], b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[d0 + 4], b1, acc1, 0, 0, 0);
      }
      const float nc = cv ? cnt[col] : 0.f;
      const float qc = cv ? Q[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float total = nc * xn[i] - 2.f * (acc0[i] + acc1[i]) + qc;
        float v = INFINITY;
        if (cv && nc > 0.f) {
          if (col == own[i]) a_own[i] = nc > 1.f ? total / (nc - 1.f) : 0.f;
          else v = total / nc;
        }
        // the own-cluster term lives on one lane: broadcast it with a max over the 16 lanes
        float ao = (cv && col == own[i]) ? a_own[i] : -INFINITY;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          v = fminf(v, __shfl_xor(v, o, 64));
          ao = fmaxf(ao, __shfl_xor(ao, o, 64));
        }
        bmin[i] = fminf(bmin[i], v);
        if (ao != -INFINITY) a_own[i] = ao;
      }
    }
    if (c16 < 4) {
      float a = a_own[0], b = bmin[0];
      int o = own[0];
#pragma unroll
      for (int i = 1; i < 4; ++i)
        if (c16 == i) { a = a_own[i]; b = bmin[i]; o = own[i]; }
      if (o >= 0 && cnt[o] > 1.f && b < INFINITY) {
        const float m = fmaxf(a, b);
        acc += m > 0.f ? (double)((b - a) / m) : 0.0;
      }
    }
  }
  const float r = block_sum256((float)acc, scr);
  if (threadIdx.x == 0) atomicAdd(out, (double)r);
}

// per-cluster sum vectors and squared-norm sums for the silhouette
__global__ __launch_bounds__(256) void cluster_stats_k(const float* __restrict__ X, const int* __restrict__ assign,
                                                       long n, int D, float* __restrict__ S, float* __restrict__ Q,
                                                       float* __restrict__ cnt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float* x = X + i * (long)D;
    const int c = assign[i];
    float xn = 0.f;
    for (int j = 0; j < D; ++j) {
      xn = fmaf(x[j], x[j], xn);
      if (x[j] != 0.f) atomicAdd(&S[c * D + j], x[j]);
    }
    atomicAdd(&Q[c], xn);
    atomicAdd(&cnt[c], 1.f);
  }
}

// ------------------------------------------------------------------------------------------------
// D > KM_DMAX (e.g. MEASURE_NAME_WEIGHT = 20 -> D = 623 in k_means.py:56-64, or wide assembled
// vectors): the same exact-f32 MFMA assignment with the feature dimension tiled through LDS in
// KM_DT-wide chunks.  Loop order per 64-row tile: for every 16-center block, the X tile is staged
// chunk by chunk (from L2) and the x.c partial products accumulate in the two MFMA accumulators
// across chunks, so the argmin sees complete dot products; ||x||^2 is accumulated during the first
// block's pass.  Cluster sums take one more chunked pass with device atomics (k*D is large here).
// ------------------------------------------------------------------------------------------------
#define KM_DT 512

PTG_DEV void km_stage_chunk(float* xs, int S, const float* __restrict__ X, long n, int D, long r0, int d0, int DPc,
                            int dc) {
  for (int t = threadIdx.x; t < KM_ROWS * DPc; t += 256) {
    const int r = t / DPc, d = t - r * DPc;
    xs[r * S + d] = (r0 + r < n && d < dc) ? X[(r0 + r) * D + d0 + d] : 0.f;
  }
}

__global__ __launch_bounds__(256) void kmeans_chunk_k(const float* __restrict__ X, long n, int D,
                                                      const float* __restrict__ C, const float* __restrict__ cn, int k,
                                                      int* __restrict__ assign, float* __restrict__ mind,
                                                      float* __restrict__ sums, float* __restrict__ counts,
                                                      double* __restrict__ cost, const float* __restrict__ weights,
                                                      const int* __restrict__ done) {
  if (done && *done) return;
  constexpr int S = KM_DT + 1;
  __shared__ __align__(16) float xs[KM_ROWS * S];
  __shared__ float sxn[KM_ROWS];
  __shared__ int sarg[KM_ROWS];
  __shared__ float sw[KM_ROWS];
  __shared__ float scost[4];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, c16 = l & 15;
  double mycost = 0.0;
  const long ntile = (n + KM_ROWS - 1) / KM_ROWS;
  for (long tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const long r0 = tile * KM_ROWS;
    if (tid < KM_ROWS) sxn[tid] = 0.f;
    float best[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    int arg[4] = {0, 0, 0, 0};
    const float* xa = xs + (16 * w + c16) * S + g;
    for (int cb = 0; cb < k; cb += 16) {
      const int col = cb + c16;
      const bool cv = col < k;
      km_f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int d0 = 0; d0 < D; d0 += KM_DT) {
        const int dc = min(KM_DT, D - d0), DPc = (dc + 7) / 8 * 8;
        __syncthreads();
        km_stage_chunk(xs, S, X, n, D, r0, d0, DPc, dc);
        __syncthreads();
        if (cb == 0 && tid < KM_ROWS) {
          float xn = sxn[tid];
          for (int d = 0; d < dc; ++d) xn = fmaf(xs[tid * S + d], xs[tid * S + d], xn);
          sxn[tid] = xn;
        }
        const float* cp = C + (long)(cv ? col : 0) * D + d0 + g;
        for (int e = 0; e < DPc; e += 8) {
          const float b0 = (cv && e + g < dc) ? cp[e] : 0.f;
          const float b1 = (cv && e + 4 + g < dc) ? cp[e + 4] : 0.f;
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], b0, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e + 4], b1, acc1, 0, 0, 0);
        }
      }
      const float cc = cv ? cn[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = cv ? cc - 2.f * (acc0[i] + acc1[i]) : INFINITY;
        int a = col;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const float ov = __shfl_xor(v, o, 64);
          const int oa = __shfl_xor(a, o, 64);
          if (ov < v || (ov == v && oa < a)) { v = ov; a = oa; }
        }
        if (v < best[i]) { best[i] = v; arg[i] = a; }
      }
    }
    __syncthreads();  // sxn complete
    if (c16 < 4) {
      const int r = 16 * w + 4 * g + c16;
      float bsel = best[0];
      int asel = arg[0];
#pragma unroll
      for (int i = 1; i < 4; ++i)
        if (c16 == i) { bsel = best[i]; asel = arg[i]; }
      const long row = r0 + r;
      float wt = 0.f;
      if (row < n) {
        const float dist = fmaxf(sxn[r] + bsel, 0.f);
        wt = weights ? weights[row] : 1.f;
        if (assign) assign[row] = asel;
        if (mind) mind[row] = dist;
        mycost += (double)dist * wt;
      }
      sarg[r] = asel;
      sw[r] = wt;
    }
    if (sums) {
      for (int d0 = 0; d0 < D; d0 += KM_DT) {
        const int dc = min(KM_DT, D - d0), DPc = (dc + 7) / 8 * 8;
        __syncthreads();
        km_stage_chunk(xs, S, X, n, D, r0, d0, DPc, dc);
        __syncthreads();
        for (int rr = 0; rr < 16; ++rr) {
          const int r = 16 * w + rr;
          const float wt = sw[r];
          if (wt == 0.f) continue;
          const int a = sarg[r];
          for (int d = l; d < dc; d += 64) {
            const float v = xs[r * S + d] * wt;
            if (v != 0.f) atomicAdd(&sums[(long)a * D + d0 + d], v);
          }
          if (l == 0 && d0 == 0) atomicAdd(&counts[a], wt);
        }
      }
    }
    __syncthreads();
  }
  const float c32 = block_sum256((float)mycost, scost);
  if (tid == 0 && cost) atomicAdd(cost, (double)c32);
}

__global__ __launch_bounds__(256) void silhouette_chunk_k(const float* __restrict__ X, const int* __restrict__ assign,
                                                          const float* __restrict__ Sv, const float* __restrict__ Q,
                                                          const float* __restrict__ cnt, long n, int D, int k,
                                                          double* __restrict__ out) {
  constexpr int S = KM_DT + 1;
  __shared__ __align__(16) float xs[KM_ROWS * S];
  __shared__ float sxn[KM_ROWS];
  __shared__ float scr[4];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, c16 = l & 15;
  double acc = 0.0;
  const long ntile = (n + KM_ROWS - 1) / KM_ROWS;
  for (long tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const long r0 = tile * KM_ROWS;
    if (tid < KM_ROWS) sxn[tid] = 0.f;
    const float* xa = xs + (16 * w + c16) * S + g;
    float a_own[4], bmin[4];
    int own[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * w + 4 * g + i;
      own[i] = r0 + r < n ? assign[r0 + r] : -1;
      a_own[i] = 0.f;
      bmin[i] = INFINITY;
    }
    // pass 0 computes ||x||^2 only (the distances need it for every center block)
    for (int d0 = 0; d0 < D; d0 += KM_DT) {
      const int dc = min(KM_DT, D - d0), DPc = (dc + 7) / 8 * 8;
      __syncthreads();
      km_stage_chunk(xs, S, X, n, D, r0, d0, DPc, dc);
      __syncthreads();
      if (tid < KM_ROWS) {
        float xn = sxn[tid];
        for (int d = 0; d < dc; ++d) xn = fmaf(xs[tid * S + d], xs[tid * S + d], xn);
        sxn[tid] = xn;
      }
    }
    __syncthreads();
    float xn[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xn[i] = sxn[16 * w + 4 * g + i];
    for (int cb = 0; cb < k; cb += 16) {
      const int col = cb + c16;
      const bool cv = col < k;
      km_f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int d0 = 0; d0 < D; d0 += KM_DT) {
        const int dc = min(KM_DT, D - d0), DPc = (dc + 7) / 8 * 8;
        __syncthreads();
        km_stage_chunk(xs, S, X, n, D, r0, d0, DPc, dc);
        __syncthreads();
        const float* sp = Sv + (long)(cv ? col : 0) * D + d0 + g;
        for (int e = 0; e < DPc; e += 8) {
          const float b0 = (cv && e + g < dc) ? sp[e] : 0.f;
          const float b1 = (cv && e + 4 + g < dc) ? sp[e + 4] : 0.f;
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], b0, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e + 4], b1, acc1, 0, 0, 0);
        }
      }
      const float nc = cv ? cnt[col] : 0.f;
      const float qc = cv ? Q[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float total = nc * xn[i] - 2.f * (acc0[i] + acc1[i]) + qc;
        float v = INFINITY;
        if (cv && nc > 0.f) {
          if (col == own[i]) a_own[i] = nc > 1.f ? total / (nc - 1.f) : 0.f;
          else v = total / nc;
        }
        float ao = (cv && col == own[i]) ? a_own[i] : -INFINITY;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          v = fminf(v, __shfl_xor(v, o, 64));
          ao = fmaxf(ao, __shfl_xor(ao, o, 64));
        }
        bmin[i] = fminf(bmin[i], v);
        if (ao != -INFINITY) a_own[i] = ao;
      }
    }
    if (c16 < 4) {
      float a = a_own[0], b = bmin[0];
      int o = own[0];
#pragma unroll
      for (int i = 1; i < 4; ++i)
        if (c16 == i) { a = a_own[i]; b = bmin[i]; o = own[i]; }
      if (o >= 0 && cnt[o] > 1.f && b < INFINITY) {
        const float m = fmaxf(a, b);
        acc += m > 0.f ? (double)((b - a) / m) : 0.0;
      }
    }
  }
  const float r = block_sum256((float)acc, scr);
  if (threadIdx.x == 0) atomicAdd(out, (double)r);
}

static inline int grid_m(long n) {
  long g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return (int)g;
}

extern "C" {

int ptg_asm_desc_size() { return (int)sizeof(AsmDesc); }

int ptg_assemble_features(const void* desc, long n, int D, void* out, hipStream_t s) {
  AsmDesc d;
  memcpy(&d, desc, sizeof(AsmDesc));
  hipLaunchKernelGGL(assemble_k, dim3(grid_m(n * D)), dim3(256), 0, s, d, n, D, (float*)out);
  hipLaunchKernelGGL(assemble_fill_k, dim3(grid_m(n)), dim3(256), 0, s, d, n, D, (float*)out);
  PTG_RETURN_LAUNCH();
}

// cn: k squared center norms (ptg_center_norms); done: optional device flag (skip when set)
int ptg_kmeans_assign_accum(const void* X, const void* C, const void* cn, long n, int D, int k, void* assign,
                            void* sums, void* counts, void* cost, const void* weights, void* mind, const void* done,
                            hipStream_t s) {
  if (D <= 0 || k <= 0) return (int)hipErrorInvalidValue;
  if (D > KM_DMAX) {  // feature dimension tiled through LDS
    const long tiles = (n + KM_ROWS - 1) / KM_ROWS;
    const int g = (int)(tiles < 1 ? 1 : (tiles > 4096 ? 4096 : tiles));
    hipLaunchKernelGGL(kmeans_chunk_k, dim3(g), dim3(256), 0, s, (const float*)X, n, D, (const float*)C,
                       (const float*)cn, k, (int*)assign, (float*)mind, (float*)sums, (float*)counts, (double*)cost,
                       (const float*)weights, (const int*)done);
    PTG_RETURN_LAUNCH();
  }
  const int DP = (D + 7) / 8 * 8;
  const long xs_bytes = (long)KM_ROWS * (DP + 1) * 4;
  const long acc_bytes = ((long)k * D + k) * 4;
  const bool acc_lds = sums != nullptr && xs_bytes + acc_bytes <= 150 * 1024;
  const size_t lds = (size_t)(xs_bytes + (acc_lds ? acc_bytes : 0));
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kmeans_mfma_k<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    (void)hipFuncSetAttribute((const void*)kmeans_mfma_k<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr = true;
  }
  long tiles = (n + KM_ROWS - 1) / KM_ROWS;
  // LDS accumulation amortises its k*D flush over many tiles: fewer, longer-lived workgroups
  const long cap = acc_lds ? 512 : 4096;
  const int g = (int)(tiles < 1 ? 1 : (tiles > cap ? cap : tiles));
  if (acc_lds)
    hipLaunchKernelGGL(kmeans_mfma_k<true>, dim3(g), dim3(256), lds, s, (const float*)X, n, D, DP, (const float*)C,
                       (const float*)cn, k, (int*)assign, (float*)mind, (float*)sums, (float*)counts, (double*)cost,
                       (const float*)weights, (const int*)done);
  else
    hipLaunchKernelGGL(kmeans_mfma_k<false>, dim3(g), dim3(256), lds, s, (const float*)X, n, D, DP, (const float*)C,
                       (const float*)cn, k, (int*)assign, (float*)mind, (float*)sums, (float*)counts, (double*)cost,
                       (const float*)weights, (const int*)done);
  PTG_RETURN_LAUNCH();
}

int ptg_center_norms(const void* C, int k, int D, void* cn, hipStream_t s) {
  hipLaunchKernelGGL(center_norms_k, dim3((k + 255) / 256), dim3(256), 0, s, (const float*)C, k, D, (float*)cn);
  PTG_RETURN_LAUNCH();
}

int ptg_kmeans_update(void* sums, void* counts, void* C, void* cn, int k, int D, void* moved, const void* done,
                      hipStream_t s) {
  hipLaunchKernelGGL(kmeans_update_k, dim3(k), dim3(256), 0, s, (float*)sums, (float*)counts, (float*)C, (float*)cn, k,
                     D, (float*)moved, (const int*)done);
  PTG_RETURN_LAUNCH();
}

int ptg_kmeans_check(void* moved, float tol2, void* state, hipStream_t s) {
  hipLaunchKernelGGL(kmeans_check_k, dim3(1), dim3(64), 0, s, (float*)moved, tol2, (int*)state);
  PTG_RETURN_LAUNCH();
}

int ptg_cluster_stats(const void* X, const void* assign, long n, int D, void* S, void* Q, void* cnt, hipStream_t s) {
  hipLaunchKernelGGL(cluster_stats_k, dim3(grid_m(n)), dim3(256), 0, s, (const float*)X, (const int*)assign, n, D,
                     (float*)S, (float*)Q, (float*)cnt);
  PTG_RETURN_LAUNCH();
}

int ptg_silhouette(const void* X, const void* assign, const void* S, const void* Q, const void* cnt, long n, int D,
                   int k, void* out, hipStream_t s) {
  if (D <= 0 || k <= 0) return (int)hipErrorInvalidValue;
  if (D > KM_DMAX) {
    const long tiles = (n + KM_ROWS - 1) / KM_ROWS;
    const int g = (int)(tiles < 1 ? 1 : (tiles > 4096 ? 4096 : tiles));
    hipLaunchKernelGGL(silhouette_chunk_k, dim3(g), dim3(256), 0, s, (const float*)X, (const int*)assign,
                       (const float*)S, (const float*)Q, (const float*)cnt, n, D, k, (double*)out);
    PTG_RETURN_LAUNCH();
  }
  const int DP = (D + 7) / 8 * 8;
  const size_t lds = (size_t)KM_ROWS * (DP + 1) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)silhouette_mfma_k, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr = true;
  }
  long tiles = (n + KM_ROWS - 1) / KM_ROWS;
  const int g = (int)(tiles < 1 ? 1 : (tiles > 4096 ? 4096 : tiles));
  hipLaunchKernelGGL(silhouette_mfma_k, dim3(g), dim3(256), lds, s, (const float*)X, (const int*)assign,
                     (const float*)S, (const float*)Q, (const float*)cnt, n, D, DP, k, (double*)out);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"

PTG_CHECK_STATUS(ml)
