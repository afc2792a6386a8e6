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

// X [n][D] fp32, C [k][D] fp32 (k*D <= 8192), sums [k][D] f32 (zeroed), counts [k] f32, cost double[1]
#define KM_MAX 8192
__global__ __launch_bounds__(256) void kmeans_assign_k(const float* __restrict__ X, const float* __restrict__ C, long n,
                                                       int D, int k, int* __restrict__ assign, float* __restrict__ sums,
                                                       float* __restrict__ counts, double* __restrict__ cost,
                                                       const float* __restrict__ weights, float* __restrict__ mind) {
  __shared__ float sc[KM_MAX];
  __shared__ float ss[KM_MAX];
  __shared__ float scnt[256];
  __shared__ float scost[4];
  const int kd = k * D;
  for (int t = threadIdx.x; t < kd; t += 256) { sc[t] = C[t]; ss[t] = 0.f; }
  if (threadIdx.x < k) scnt[threadIdx.x] = 0.f;
  __syncthreads();
  double mycost = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float* x = X + i * (long)D;
    float best = INFINITY; int arg = 0;
    for (int c = 0; c < k; ++c) {
      const float* cc = sc + c * D;
      float dist = 0.f;
      for (int j = 0; j < D; ++j) { const float df = x[j] - cc[j]; dist = fmaf(df, df, dist); }
      if (dist < best) { best = dist; arg = c; }
    }
    const float w = weights ? weights[i] : 1.f;
    if (assign) assign[i] = arg;
    if (mind) mind[i] = best;
    mycost += (double)best * w;
    if (sums) {
      atomicAdd(&scnt[arg], w);
      for (int j = 0; j < D; ++j) {
        const float v = x[j];
        if (v != 0.f) atomicAdd(&ss[arg * D + j], v * w);
      }
    }
  }
  const float c32 = block_sum256((float)mycost, scost);
  __syncthreads();
  if (threadIdx.x == 0 && cost) atomicAdd(cost, (double)c32);
  if (sums) {
    for (int t = threadIdx.x; t < kd; t += 256)
      if (ss[t] != 0.f) atomicAdd(&sums[t], ss[t]);
    if (threadIdx.x < k && scnt[threadIdx.x] != 0.f) atomicAdd(&counts[threadIdx.x], scnt[threadIdx.x]);
  }
}

// new centers; moved[0] = max squared center shift (for Spark's tol convergence check)
__global__ __launch_bounds__(256) void kmeans_update_k(const float* __restrict__ sums, const float* __restrict__ counts,
                                                       float* __restrict__ C, int k, int D, float* __restrict__ moved) {
  __shared__ float shift[256];
  const int c = blockIdx.x;
  float s2 = 0.f;
  const float cnt = counts[c];
  for (int j = threadIdx.x; j < D; j += 256) {
    const float old = C[c * D + j];
    const float nw = cnt > 0.f ? sums[c * D + j] / cnt : old;
    C[c * D + j] = nw;
    s2 += (nw - old) * (nw - old);
  }
  shift[threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) shift[threadIdx.x] += shift[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    unsigned int* m = (unsigned int*)moved;  // non-negative floats order as unsigned ints
    atomicMax(m, __float_as_uint(shift[0]));
  }
}

// per-point silhouette, summed: S [k][D] cluster sums, Q[k] sum of squared norms, cnt[k]
__global__ __launch_bounds__(256) void silhouette_k(const float* __restrict__ X, const int* __restrict__ assign,
                                                    const float* __restrict__ S, const float* __restrict__ Q,
                                                    const float* __restrict__ cnt, long n, int D, int k,
                                                    double* __restrict__ out) {
  __shared__ float sS[KM_MAX];
  __shared__ float sQ[256], sN[256];
  __shared__ float scr[4];
  for (int t = threadIdx.x; t < k * D; t += 256) sS[t] = S[t];
  if (threadIdx.x < k) { sQ[threadIdx.x] = Q[threadIdx.x]; sN[threadIdx.x] = cnt[threadIdx.x]; }
  __syncthreads();
  double acc = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float* x = X + i * (long)D;
    float xn = 0.f;
    for (int j = 0; j < D; ++j) xn = fmaf(x[j], x[j], xn);
    const int own = assign[i];
    float a = 0.f, b = INFINITY;
    for (int c = 0; c < k; ++c) {
      const float nc = sN[c];
      if (nc <= 0.f) continue;
      float dot = 0.f;
      for (int j = 0; j < D; ++j) dot = fmaf(x[j], sS[c * D + j], dot);
      const float total = nc * xn - 2.f * dot + sQ[c];  // sum_j ||x - x_j||^2 over cluster c
      if (c == own) a = nc > 1.f ? total / (nc - 1.f) : 0.f;
      else b = fminf(b, total / nc);
    }
    float s = 0.f;
    if (sN[own] > 1.f && b < INFINITY) {
      const float m = fmaxf(a, b);
      s = m > 0.f ? (b - a) / m : 0.f;
    }
    acc += s;
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

int ptg_kmeans_assign_accum(const void* X, const void* C, long n, int D, int k, void* assign, void* sums, void* counts,
                            void* cost, const void* weights, void* mind, hipStream_t s) {
  if ((long)k * D > KM_MAX || k > 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_assign_k, dim3(grid_m(n)), dim3(256), 0, s, (const float*)X, (const float*)C, n, D, k,
                     (int*)assign, (float*)sums, (float*)counts, (double*)cost, (const float*)weights, (float*)mind);
  PTG_RETURN_LAUNCH();
}

int ptg_kmeans_update(const void* sums, const void* counts, void* C, int k, int D, void* moved, hipStream_t s) {
  hipLaunchKernelGGL(kmeans_update_k, dim3(k), dim3(256), 0, s, (const float*)sums, (const float*)counts, (float*)C, k,
                     D, (float*)moved);
  PTG_RETURN_LAUNCH();
}

int ptg_cluster_stats(const void* X, const void* assign, long n, int D, void* S, void* Q, void* cnt, hipStream_t s) {
  hipLaunchKernelGGL(cluster_stats_k, dim3(grid_m(n)), dim3(256), 0, s, (const float*)X, (const int*)assign, n, D,
                     (float*)S, (float*)Q, (float*)cnt);
  PTG_RETURN_LAUNCH();
}

int ptg_silhouette(const void* X, const void* assign, const void* S, const void* Q, const void* cnt, long n, int D,
                   int k, void* out, hipStream_t s) {
  if ((long)k * D > KM_MAX || k > 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(silhouette_k, dim3(grid_m(n)), dim3(256), 0, s, (const float*)X, (const int*)assign,
                     (const float*)S, (const float*)Q, (const float*)cnt, n, D, k, (double*)out);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"

PTG_CHECK_STATUS(ml)
