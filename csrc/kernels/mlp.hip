// Whole training step of a small MLP in ONE launch: the reference's CSV classifier
// (train_tf_ps.py:328-343, Input(3) -> Dense16 relu -> Dense32 relu -> Dense64 relu -> Dense(C)
// softmax, Adam, SparseCategoricalCrossentropy; 3,695 parameters) at the batch sizes the reference
// trains it with (32, train_tf_ps.py:831; 64, run_tf_training_from_bastion.sh:17).
//
// At those sizes the step is launch- and barrier-bound, not FLOP-bound (~1.4 MFLOP at batch 64),
// so one 512-thread workgroup keeps everything in LDS:
//   * every layer's weights and bias (fp32, read once from the flat master store), with odd row
//     strides so threads of one wave that read different rows hit different banks;
//   * every layer's activation for the batch (kept for the backward) and two ping-pong gradient
//     buffers.
// Per step: forward, fused softmax + cross-entropy (or MSE) producing dlogits, then per layer from
// the top: dX for the layer below (with the ReLU mask) from the pre-update LDS weights, a barrier,
// then each parameter's gradient followed immediately by its Adam update straight into the flat
// master / m / v / bf16 copy in HBM and into the LDS weights (no gradient buffer is written).  Every
// matrix product runs on the matrix cores (v_mfma_f32_16x16x4_f32: fp32 products and sums, one LDS
// float per lane per operand) - the register-tiled FMA form before it moved 8x the LDS bytes and
// made the step LDS-bound; the bias gradient is one more column of the weight-gradient GEMM (each
// activation row carries a constant 1), and the barriers only wait for LDS (tools/mlp_phases.py
// times the phases of the PTG_MLP_PROF build).  ``steps`` > 1 runs consecutive
// batches of a device-resident dataset in the same launch (Keras' steps_per_execution): each step
// is still a full forward / backward / Adam step.  Metric sums are kept in registers and added to
// `stats` once (the layouts of softmax_xent_k / mse_k).
#include <cstdlib>

#include "common.h"

namespace ptgm {

typedef __attribute__((address_space(3))) void lds_t;

#ifdef PTG_MLP_PROF  // phase timestamps of the first step (A/B build: tools/mlp_phases.py)
__device__ long long g_mlp_prof[32];
#define MLP_T(i) \
  if (threadIdx.x == 0 && st == 0) g_mlp_prof[i] = wall_clock64();
#else
#define MLP_T(i)
#endif

constexpr int MAXL = 6;
#ifndef PTG_MLP_NT
#define PTG_MLP_NT 512
#endif
constexpr int NT = PTG_MLP_NT;  // threads of the one workgroup (A/B builds: 256 / 1024)

struct MlpDesc {
  int L, B, steps, loss;        // loss 0: softmax + sparse categorical cross-entropy, 1: MSE
  int d[MAXL + 1];              // d[0] input features, d[l + 1] units of layer l
  int act[MAXL];                // hidden activation of layer l: 0 linear, 1 relu (last: from loss)
  long woff[MAXL], boff[MAXL];  // element offsets of W_l ([d[l+1]][d[l]]) and b_l in the flat store
  int lw[MAXL], lb[MAXL];       // LDS float offsets of W_l (row stride ws[l]) and b_l (copy 0)
  int wtot, dbl;                // floats of one weight copy; dbl: a second copy follows (LDS permitting)
  int ws[MAXL];                 // LDS row stride of W_l (odd)
  int la[MAXL + 1], as[MAXL + 1];  // LDS offset / row stride (odd) of activation l
  int lg0, lg1, gs;             // the two gradient buffers (row stride gs, odd) and red scratch
  int lred;
  int lg;                       // lanes per row of the softmax loss (16 / 32 / 64; 0: one thread per row)
  int ly;                       // LDS float offset of the step's labels / targets
  float lr, b1, b2, eps;
  int t0;                       // optimizer steps taken before this launch
  // LDS-resident Adam state (res): the flat span [lo, lo + rn) of p / m / v covering every layer is
  // copied into LDS by the prologue's LDS-DMA loads (p staged at lps, m / v live at lpm / lpv)
  int res, rn, lps, lpm, lpv;
  long lo;
};

// Workgroup barrier for LDS only.  __syncthreads() also waits for this wave's outstanding GLOBAL
// stores (its release fence covers global memory): after every dW+Adam phase that is a full HBM
// write round trip (~2.5 us of a 3.3 us phase, tools/mlp_phases.py).  Nothing in the step reads back
// the p / m / v / bf16 values it stores (the next launch is ordered by the kernel boundary), so the
// step's barriers only wait for LDS traffic.
PTG_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

PTG_DEV float sum_block(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  return r;
}

// out(i, j) = sum_k P[i*pi + k*pk] * Q[j*qj + k*qk] for i < M, j < N, all operands in LDS, on the
// matrix cores: each wave takes 16 x 16 output tiles and runs v_mfma_f32_16x16x4_f32 (fp32 products,
// fp32 sums) over K in steps of 4, every operand one LDS float per lane (lane l: A row l % 16 / B column
// l % 16 at k = l / 16).  The scalar register-tiled form this replaced moved 8x the LDS bytes per FMA
// and made the step LDS-bound (25 us of a 30 us step at batch 32).  Two accumulators split the k
// steps (even / odd) so consecutive MFMAs do not wait on each other.  Out-of-range rows / columns read
// the last valid one and are dropped at the epilogue; k >= K reads zero.
PTG_DEV f32x4_t mfma_dot(int K, const float* pa, int pk, const float* qb, int qk, int kq) {
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  int k0 = 0;
  for (; k0 + 8 <= K; k0 += 8) {
    const float a0 = pa[(k0 + kq) * pk], b0 = qb[(k0 + kq) * qk];
    const float a1 = pa[(k0 + 4 + kq) * pk], b1 = qb[(k0 + 4 + kq) * qk];
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc1, 0, 0, 0);
  }
  for (; k0 < K; k0 += 4) {
    const int k = k0 + kq;
    const float a = k < K ? pa[k * pk] : 0.f, b = k < K ? qb[k * qk] : 0.f;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
  }
  return acc0 + acc1;
}

template <class Epi>
PTG_DEV void gemm(int M, int N, int K, const float* P, int pi, int pk, const float* Q, int qj, int qk, Epi epi) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int tm = (M + 15) / 16, tn = (N + 15) / 16;
  for (int t = wid; t < tm * tn; t += NT / 64) {
    const int i0 = (t / tn) * 16, j0 = (t - (t / tn) * tn) * 16;
    const f32x4_t acc = mfma_dot(K, P + min(i0 + r16, M - 1) * pi, pk, Q + min(j0 + r16, N - 1) * qj, qk, kq);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * kq + r, j = j0 + r16;
      if (i < M && j < N) epi(i, j, acc[r]);
    }
  }
}

// tstep (nullable): the optimizer step counter on the device (read for Adam's bias correction and
// advanced by `steps` at the end), so a cached launch needs no per-step host argument
struct AdamArgs {
  float* p;
  float* m;
  float* v;
  bf16_t* pbf;
  float lr_t, b1, b2, eps;
};

// Adam on one element; m0 / v0 come back updated.  The HBM copies are written when `store`: every
// step, or only the launch's last step when the moments live in LDS.
PTG_DEV float adam_update(const AdamArgs& o, long idx, float g, float p0, float& m0, float& v0, bool store) {
  const float mm = o.b1 * m0 + (1.f - o.b1) * g;
  const float vv = o.b2 * v0 + (1.f - o.b2) * g * g;
  // v_sqrt_f32 / v_rcp_f32 (1 ulp) instead of the IEEE sequences: ~25 fewer dependent VALU ops per
  // element on this latency-bound single-workgroup step
  const float pp = p0 - o.lr_t * mm * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vv) + o.eps);
  m0 = mm;
  v0 = vv;
  if (store) {
    o.m[idx] = mm;
    o.v[idx] = vv;
    o.p[idx] = pp;
    if (o.pbf) o.pbf[idx] = f2bf(pp);
  }
  return pp;
}

// dW[i][j] = sum_k P[i*pi + k*pk] Q[j*qj + k*qk] (i < M output units, j < Nw inputs) with Adam on
// element wo + i*Nw + j, on the matrix cores as gemm().  With a bias (bo >= 0) the GEMM has one more
// column j = Nw whose Q entries are the constant-1 column every activation row carries at index Nw, so
// the same MFMAs produce db[i] = sum_k P[i][k] (Adam on element bo + i, LDS copy Bl / Bc) - no serial
// per-unit reduction over the batch.  A lane's four outputs have their p / m / v read BEFORE the MFMAs
// (the weight itself from its current LDS copy Wc / Bc; the moments from the LDS-resident copies
// Ml / Vl at element - lo, or else from HBM, whose latency then partly hides under the k loop); the
// updated value also goes to the LDS copy Wl / Bl.
// RES is a template argument so that the resident form has no global load at all: a run-time select
// between the LDS and HBM pointers compiles to FLAT loads, whose vmcnt waits then also wait for every
// earlier global store of the phase.
template <bool RES>
PTG_DEV void dw_adam(int M, int Nw, int K, const float* P, int pi, int pk, const float* Q, int qj, int qk,
                     const AdamArgs& o, long wo, long bo, float* Wl, int S, const float* Wc, float* Bl,
                     const float* Bc, float* Ml, float* Vl, long lo, bool store) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int N = Nw + (bo >= 0 ? 1 : 0);
  const int tm = (M + 15) / 16, tn = (N + 15) / 16;
  for (int t = wid; t < tm * tn; t += NT / 64) {
    const int i0 = (t / tn) * 16, j0 = (t - (t / tn) * tn) * 16;
    float p0[4], m0[4], v0[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = min(i0 + 4 * kq + r, M - 1), j = min(j0 + r16, N - 1);
      const bool isb = j == Nw;
      const long idx = isb ? bo + i : wo + (long)i * Nw + j;
      p0[r] = isb ? Bc[i] : Wc[i * S + j];
      if constexpr (RES) {
        m0[r] = Ml[idx - lo];
        v0[r] = Vl[idx - lo];
      } else {
        m0[r] = o.m[idx];
        v0[r] = o.v[idx];
      }
    }
    const f32x4_t acc = mfma_dot(K, P + min(i0 + r16, M - 1) * pi, pk, Q + min(j0 + r16, N - 1) * qj, qk, kq);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * kq + r, j = j0 + r16;
      if (i < M && j < N) {
        const long idx = j == Nw ? bo + i : wo + (long)i * Nw + j;
        const float pp = adam_update(o, idx, acc[r], p0[r], m0[r], v0[r], store);
        if (j == Nw) Bl[i] = pp;
        else Wl[i * S + j] = pp;
        if constexpr (RES) { Ml[idx - lo] = m0[r]; Vl[idx - lo] = v0[r]; }
      }
    }
  }
}

// max / first-argmax / sum over the `g` lanes of a row group (g = 16 / 32 / 64, aligned in the wave)
PTG_DEV void group_max_arg(float& v, int& i, int g) {
  for (int o = 1; o < g; o <<= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}
PTG_DEV float group_sum(float v, int g) {
  for (int o = 1; o < g; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(NT) void mlp_train_k(const float* __restrict__ x, const void* __restrict__ y,
                                                  float* __restrict__ p, float* __restrict__ m,
                                                  float* __restrict__ v, bf16_t* __restrict__ pbf,
                                                  float* __restrict__ stats, float* __restrict__ tstep,
                                                  const MlpDesc D) {
  extern __shared__ __align__(16) float sm[];
  const int tid = threadIdx.x;
  const int L = D.L, B = D.B;
#ifdef PTG_MLP_PROF
  if (tid == 0) g_mlp_prof[31] = wall_clock64();
#endif
  const int t0 = tstep ? (int)tstep[0] : D.t0;
  // step 0's inputs and labels: loads issued first, stored to LDS after the weight loads (one HBM
  // round trip for the whole prologue instead of two)
  const int K0 = D.d[0], C = D.d[L];
  const int nx = B * K0, ny = D.loss == 0 ? B : B * C;
  constexpr int PX = 2;
  float xr[PX], yr[PX];
  const bool xpre = nx <= PX * NT && ny <= PX * NT;
  if (xpre) {
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int i = tid + u * NT;
      xr[u] = i < nx ? x[i] : 0.f;
      yr[u] = i < ny ? (D.loss == 0 ? __int_as_float(((const int*)y)[i]) : ((const float*)y)[i]) : 0.f;
    }
  }
  // weights + biases -> LDS (the Adam epilogues keep them current in place).  res: one LDS-DMA
  // burst brings the p / m / v span (1 KB per wave instruction, all in flight together), then p is
  // spread into the padded weight layout LDS -> LDS; otherwise per-element loads.
  if (D.res) {
    const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t bytes = (uint32_t)D.rn * 4u;
    const Rsrc rp = make_rsrc(p + D.lo, bytes), rm = make_rsrc(m + D.lo, bytes), rv = make_rsrc(v + D.lo, bytes);
    unsigned char* sb = (unsigned char*)sm;
    for (int c = wid; c * 256 < D.rn; c += NT / 64) {
      const uint32_t off = (uint32_t)c * 1024u + (uint32_t)lane * 16u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rp, (lds_t*)(sb + D.lps * 4 + c * 1024), 16, off, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (lds_t*)(sb + D.lpm * 4 + c * 1024), 16, off, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_t*)(sb + D.lpv * 4 + c * 1024), 16, off, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* ps = sm + D.lps - D.lo;
    for (int l = 0; l < L; ++l) {
      const int K = D.d[l], N = D.d[l + 1], S = D.ws[l];
      for (int i = tid; i < N * K; i += NT) sm[D.lw[l] + (i / K) * S + i % K] = ps[D.woff[l] + i];
      for (int n = tid; n < N; n += NT) {
        sm[D.lb[l] + n] = D.boff[l] >= 0 ? ps[D.boff[l] + n] : 0.f;
        if (D.dbl && D.boff[l] < 0) sm[D.wtot + D.lb[l] + n] = 0.f;
      }
    }
  } else {
    for (int l = 0; l < L; ++l) {
      const int K = D.d[l], N = D.d[l + 1], S = D.ws[l];
      for (int i = tid; i < N * K; i += NT) sm[D.lw[l] + (i / K) * S + i % K] = p[D.woff[l] + i];
      for (int n = tid; n < N; n += NT) {
        sm[D.lb[l] + n] = D.boff[l] >= 0 ? p[D.boff[l] + n] : 0.f;
        if (D.dbl && D.boff[l] < 0) sm[D.wtot + D.lb[l] + n] = 0.f;  // bias-less: zeros in both copies
      }
    }
  }
  if (xpre) {
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int i = tid + u * NT;
      if (i < nx) sm[D.la[0] + (i / K0) * D.as[0] + i % K0] = xr[u];
      if (i < ny) sm[D.ly + i] = yr[u];
    }
  }
  float s_loss = 0.f, s_a = 0.f, s_b = 0.f;
#ifdef PTG_MLP_PROF
  if (tid == 0) g_mlp_prof[0] = wall_clock64();
#endif
  // with two weight copies a step reads one and its Adam epilogues write the other, so a layer's dX
  // and its weight update share one phase; otherwise the update is in place after a barrier
  // every activation row carries a constant 1 at column d[l] (its row stride leaves room): the
  // weight-gradient GEMM's extra column that yields the bias gradient
  for (int l = 0; l < L; ++l)
    for (int r = tid; r < B; r += NT) sm[D.la[l] + r * D.as[l] + D.d[l]] = 1.f;
  int wcur = 0;
  for (int st = 0; st < D.steps; ++st) {
    const int wnxt = D.dbl ? D.wtot - wcur : wcur;
    // ---- input batch, with its labels / targets (their HBM latency is paid once, not again in the
    // loss phase); step 0's came with the prologue
    if (st > 0 || !xpre) {
      const float* xs = x + (long)st * nx;
      for (int i = tid; i < nx; i += NT) sm[D.la[0] + (i / K0) * D.as[0] + i % K0] = xs[i];
      for (int i = tid; i < ny; i += NT)
        sm[D.ly + i] = D.loss == 0 ? __int_as_float(((const int*)y)[(long)st * B + i]) : ((const float*)y)[(long)st * ny + i];
    }
    lds_barrier();
    MLP_T(1)
    // ---- forward: O[r][n] = act(b[n] + A[r] . W[n])
    for (int l = 0; l < L; ++l) {
      const int K = D.d[l], N = D.d[l + 1], SO = D.as[l + 1];
      const float* bias = sm + wcur + D.lb[l];
      float* O = sm + D.la[l + 1];
      const bool relu = l < L - 1 && D.act[l] == 1;
      gemm(B, N, K, sm + D.la[l], D.as[l], 1, sm + wcur + D.lw[l], D.ws[l], 1, [&](int r, int n, float acc) {
        acc += bias[n];
        O[r * SO + n] = relu ? fmaxf(acc, 0.f) : acc;
      });
      lds_barrier();
      MLP_T(2 + l)
    }
    // ---- loss: dlogits into gradient buffer 0
    float* G = sm + D.lg0;
    const float* Z = sm + D.la[L];
    const int SZ = D.as[L];
    if (D.loss == 0 && D.lg) {
      // D.lg lanes per row: lane c holds logit c; max / argmax / sum by lane shuffles
      const int* lab = (const int*)(sm + D.ly);
      const float scale = 1.f / (float)B;
      const int g = D.lg, c = tid & (g - 1), rpp = NT / g;
      for (int r0 = 0; r0 < B; r0 += rpp) {  // uniform trip count: every lane joins the shuffles
        const int r = r0 + tid / g;
        const bool ok = r < B;
        const int t = ok ? lab[r] : 0;  // (issued first: its latency hides under the reductions)
        const float* z = Z + (ok ? r : 0) * SZ;
        const float zc = c < C ? z[c] : -__builtin_inff();
        float mx = zc;
        int am = c < C ? c : C;
        group_max_arg(mx, am, g);
        const float e = c < C ? __expf(zc - mx) : 0.f;
        const float inv = 1.f / group_sum(e, g);
        if (ok && c < C) {
          G[r * D.gs + c] = (e * inv - (c == t ? 1.f : 0.f)) * scale;
          if (c == t) {
            s_loss += -__logf(fminf(fmaxf(e * inv, 1e-7f), 1.f - 1e-7f));
            s_a += am == t ? 1.f : 0.f;
          }
        }
      }
    } else if (D.loss == 0) {
      const int* lab = (const int*)(sm + D.ly);
      const float scale = 1.f / (float)B;
      for (int r = tid; r < B; r += NT) {
        const float* z = Z + r * SZ;
        float mx = z[0];
        int am = 0;
        for (int c = 1; c < C; ++c)
          if (z[c] > mx) { mx = z[c]; am = c; }
        float s = 0.f;
        for (int c = 0; c < C; ++c) s += __expf(z[c] - mx);
        const float inv = 1.f / s;
        const int t = lab[r];
        for (int c = 0; c < C; ++c) G[r * D.gs + c] = (__expf(z[c] - mx) * inv - (c == t ? 1.f : 0.f)) * scale;
        const float pl = fminf(fmaxf(__expf(z[t] - mx) * inv, 1e-7f), 1.f - 1e-7f);
        s_loss += -__logf(pl);
        s_a += am == t ? 1.f : 0.f;
      }
    } else {
      const float* tg = sm + D.ly;
      const float inv = 1.f / (float)(B * C);
      for (int i = tid; i < B * C; i += NT) {
        const int r = i / C, c = i - r * C;
        const float d = Z[r * SZ + c] - tg[i];
        G[r * D.gs + c] = 2.f * d * inv;
        s_loss += d * d * inv * (float)B;
        s_a += fabsf(d);
        s_b += d * d;
      }
    }
    lds_barrier();
    MLP_T(9)
    // ---- backward, per layer: dX for the layer below from the pre-update LDS weights, a barrier,
    // then each weight gradient with its Adam update into HBM and into the LDS weights in place
    const float t = (float)(t0 + st + 1);
    const float lr_t = D.lr * sqrtf(1.f - powf(D.b2, t)) / (1.f - powf(D.b1, t));
    const AdamArgs ad{p, m, v, pbf, lr_t, D.b1, D.b2, D.eps};
    const bool store = !D.res || st == D.steps - 1;  // LDS-resident state: HBM copies at the end only
    int cur = D.lg0, nxt = D.lg1;
    for (int l = L - 1; l >= 0; --l) {
      const int K = D.d[l], N = D.d[l + 1], S = D.ws[l], SA = D.as[l];
      const float* Gc = sm + cur;
      const float* A = sm + D.la[l];
      if (l > 0) {
        const bool mask = D.act[l - 1] == 1;
        float* Gn = sm + nxt;
        const int gs = D.gs;
        // Gn[r][k] = (G[r] . W[:, k]) * relu'(A[r][k])
        gemm(B, K, N, Gc, gs, 1, sm + wcur + D.lw[l], 1, S, [&](int r, int k, float s) {
          if (mask && !(A[r * SA + k] > 0.f)) s = 0.f;
          Gn[r * gs + k] = s;
        });
        if (!D.dbl) lds_barrier();  // every dX read of W_l before the in-place update below
      }
      MLP_T(10 + 2 * (L - 1 - l))
      // dW[n][k] = sum_r G[r][n] A[r][k] and db[n] = sum_r G[r][n] (A's constant-1 column), Adam
      // straight from the register
      if (D.res)
        dw_adam<true>(N, K, B, Gc, 1, D.gs, A, 1, SA, ad, D.woff[l], D.boff[l], sm + wnxt + D.lw[l], S,
                      sm + wcur + D.lw[l], sm + wnxt + D.lb[l], sm + wcur + D.lb[l], sm + D.lpm, sm + D.lpv, D.lo, store);
      else
        dw_adam<false>(N, K, B, Gc, 1, D.gs, A, 1, SA, ad, D.woff[l], D.boff[l], sm + wnxt + D.lw[l], S,
                       sm + wcur + D.lw[l], sm + wnxt + D.lb[l], sm + wcur + D.lb[l], nullptr, nullptr, 0, true);
      lds_barrier();
      MLP_T(11 + 2 * (L - 1 - l))
      const int tmp = cur; cur = nxt; nxt = tmp;
    }
    wcur = wnxt;  // (the next step's input barrier orders the new copy before any forward read)
  }
  float* red = sm + D.lred;
#ifdef PTG_MLP_PROF
  if (tid == 0) g_mlp_prof[30] = wall_clock64();
#endif
  const float tl = sum_block(s_loss, red);
  const float ta = sum_block(s_a, red);
  const float tb = sum_block(s_b, red);
  if (tid == 0) {
    if (tstep) tstep[0] = (float)(t0 + D.steps);  // every thread read it before the barriers above
    const float nb = (float)(B * D.steps);
    if (D.loss == 0) {
      stats[0] += tl;
      stats[1] += ta;
      stats[4] += nb;
    } else {
      stats[0] += tl;
      stats[1] += ta;
      stats[2] += tb;
      stats[3] += nb * (float)C;
      stats[4] += nb;
    }
  }
}

}  // namespace ptgm

static int odd(int n) { return n | 1; }

// LDS bytes of the fused step (0: shape not supported).  hdesc (host, int64):
// [d0 .. dL][act0 .. act_{L-1}][woff0 .. woff_{L-1}][boff0 .. boff_{L-1}]
static long mlp_plan(const long* hdesc, int L, int B, ptgm::MlpDesc* D) {
  if (L < 1 || L > ptgm::MAXL || B < 1) return 0;
  D->L = L; D->B = B;
  int dmax = 0;
  for (int i = 0; i <= L; ++i) {
    D->d[i] = (int)hdesc[i];
    if (D->d[i] < 1 || D->d[i] > 1024) return 0;
    if (i > 0) dmax = dmax > D->d[i] ? dmax : D->d[i];
  }
  int off = 0;
  for (int l = 0; l < L; ++l) {
    D->act[l] = (int)hdesc[L + 1 + l];
    D->woff[l] = hdesc[2 * L + 1 + l];
    D->boff[l] = hdesc[3 * L + 1 + l];
    D->ws[l] = odd(D->d[l]);
    D->lw[l] = off; off += D->d[l + 1] * D->ws[l];
    D->lb[l] = off; off += D->d[l + 1];
  }
  for (int l = 0; l <= L; ++l) {
    D->as[l] = odd(D->d[l] + 1);  // room for the constant-1 bias column at d[l]
    D->la[l] = off; off += B * D->as[l];
  }
  D->gs = odd(dmax);
  D->lg0 = off; off += B * D->gs;
  D->lg1 = off; off += B * D->gs;
  D->lred = off; off += 16;
  D->ly = off; off += B * D->d[L];  // labels (B ints) or MSE targets (B x C)
  D->wtot = D->la[0];
  D->dbl = (long)(off + D->wtot) * 4 <= 160 * 1024;
  if (D->dbl) {  // the second weight copy goes right after the first: shift everything behind it
    for (int l = 0; l <= L; ++l) D->la[l] += D->wtot;
    D->lg0 += D->wtot; D->lg1 += D->wtot; D->lred += D->wtot; D->ly += D->wtot;
    off += D->wtot;
  }
  // LDS-resident Adam state: the 16-B aligned span of every W / b, three copies (p staging, m, v) in
  // whole 1 KB DMA chunks, when it fits next to the rest (PTG_MLP_RES=0: per-element HBM moments)
  D->res = 0;
  {
    long lo = D->woff[0], hi = 0, used = 0;
    for (int l = 0; l < L; ++l) {
      const long nw = (long)D->d[l] * D->d[l + 1];
      lo = lo < D->woff[l] ? lo : D->woff[l];
      hi = hi > D->woff[l] + nw ? hi : D->woff[l] + nw;
      used += nw;
      if (D->boff[l] >= 0) {
        lo = lo < D->boff[l] ? lo : D->boff[l];
        hi = hi > D->boff[l] + D->d[l + 1] ? hi : D->boff[l] + D->d[l + 1];
        used += D->d[l + 1];
      }
    }
    lo &= ~3L;
    const long rn = hi - lo, rpad = (rn + 255) / 256 * 256;
    const char* re = getenv("PTG_MLP_RES");
    const bool want = !(re && re[0] == '0');
    int o4 = (off + 3) & ~3;  // 16-B aligned regions
    if (want && rn <= 4 * used + 256 && (long)(o4 + 3 * rpad) * 4 <= 160 * 1024) {
      D->res = 1; D->lo = lo; D->rn = (int)rn;
      D->lps = o4; D->lpm = o4 + (int)rpad; D->lpv = o4 + 2 * (int)rpad;
      off = o4 + 3 * (int)rpad;
    }
  }
  // softmax loss with one row per lane group (PTG_MLP_LOSS_LANES=0: one thread per row)
  const char* lz = getenv("PTG_MLP_LOSS_LANES");
  const int C = D->d[L];
  D->lg = (lz && lz[0] == '0') ? 0 : C <= 16 ? 16 : C <= 32 ? 32 : C <= 64 ? 64 : 0;
  return (long)off * 4;
}

extern "C" {

// Bytes of LDS the fused step needs for this shape (the Python side checks it against the
// 160 KiB per CU before choosing the fused path); 0 = unsupported.
int ptg_mlp_lds_bytes(const long* hdesc, int L, int B, long* out) {
  ptgm::MlpDesc D;
  *out = mlp_plan(hdesc, L, B, &D);
  return 0;
}

int ptg_mlp_train(const void* x, const void* y, float* p, float* m, float* v, void* pbf, float* stats,
                  const long* hdesc, int L, int B, int steps, int loss, float lr, float b1, float b2, float eps,
                  int t0, hipStream_t s) {
  ptgm::MlpDesc D;
  const long bytes = mlp_plan(hdesc, L, B, &D);
  if (bytes <= 0 || bytes > 160 * 1024 || steps < 1 || (loss != 0 && loss != 1)) return (int)hipErrorInvalidValue;
  D.steps = steps; D.loss = loss;
  D.lr = lr; D.b1 = b1; D.b2 = b2; D.eps = eps; D.t0 = t0;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ptgm::mlp_train_k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(ptgm::mlp_train_k, dim3(1), dim3(ptgm::NT), (size_t)bytes, s, (const float*)x, y, p, m, v,
                     (bf16_t*)pbf, stats, (float*)nullptr, D);
  return (int)hipGetLastError();
}

// Cached launch state of one model's fused step (ops/nn.py MlpStep): every pointer, the LDS plan and
// the hyper-parameters are fixed at creation; a step passes only the batch and the stream, and the
// step counter lives on the device (tstep), so the per-step host cost is one short call.
struct MlpCtx {
  ptgm::MlpDesc D;
  long bytes;
  float *p, *m, *v, *stats, *tstep;
  bf16_t* pbf;
};

int ptg_mlp_ctx_create(float* p, float* m, float* v, void* pbf, float* stats, float* tstep, const long* hdesc, int L,
                       int B, int loss, float lr, float b1, float b2, float eps, void** out) {
  MlpCtx* c = new MlpCtx();
  c->bytes = mlp_plan(hdesc, L, B, &c->D);
  if (c->bytes <= 0 || c->bytes > 160 * 1024 || (loss != 0 && loss != 1) || !tstep) {
    delete c;
    return (int)hipErrorInvalidValue;
  }
  c->D.loss = loss; c->D.steps = 1;
  c->D.lr = lr; c->D.b1 = b1; c->D.b2 = b2; c->D.eps = eps; c->D.t0 = 0;
  c->p = p; c->m = m; c->v = v; c->pbf = (bf16_t*)pbf; c->stats = stats; c->tstep = tstep;
  (void)hipFuncSetAttribute((const void*)ptgm::mlp_train_k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  *out = c;
  return 0;
}

int ptg_mlp_ctx_run(void* ctx, const void* x, const void* y, int steps, hipStream_t s) {
  MlpCtx* c = (MlpCtx*)ctx;
  if (!c || steps < 1) return (int)hipErrorInvalidValue;
  ptgm::MlpDesc D = c->D;
  D.steps = steps;
  hipLaunchKernelGGL(ptgm::mlp_train_k, dim3(1), dim3(ptgm::NT), (size_t)c->bytes, s, (const float*)x, y, c->p, c->m,
                     c->v, c->pbf, c->stats, c->tstep, D);
  return (int)hipGetLastError();
}

#ifdef PTG_MLP_PROF
int ptg_mlp_prof_read(long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ptgm::g_mlp_prof), sizeof(long long) * 32);
}
#endif

int ptg_mlp_ctx_free(void* ctx) {
  delete (MlpCtx*)ctx;
  return 0;
}

}  // extern "C"
