// Memory-bound kernels of the training runtime (gfx950): PReLU (+ fused 2x2 max-pool) forward and
// backward, bias/activation epilogues, skinny dense layers, losses + metrics, fused flat Adam,
// image resize/normalise.  Reference semantics (TF/Keras inside train_tf_ps.py):
//   PReLU with per-element alpha (Keras default shared_axes=None)      train_tf_ps.py:352-364
//   MaxPooling2D(2x2, stride 2, valid)                                  train_tf_ps.py:353-362
//   Dense(relu/linear/softmax)                                          train_tf_ps.py:332-335,366-367
//   MeanSquaredError + MAE/MSE metrics                                  train_tf_ps.py:375-376,729-731
//   SparseCategoricalCrossentropy + accuracy                            train_tf_ps.py:340-341,607-608
//   Adam (epsilon 1e-7, Keras bias-corrected form)                      train_tf_ps.py:339,374,606,728
//   tf.image.resize bilinear (half-pixel centres) then /255             train_tf_ps.py:301-306
// All bf16 traffic is 16 B per lane (8 channels); channel counts are multiples of 8 except the
// 4-channel padded image.
#include "common.h"

#include <type_traits>

// ----------------------------------------------------------------------------------------------
// PReLU + 2x2 max-pool forward: p[n][ph][pw][c] = max_{2x2} prelu(z), prelu(z) = z>0 ? z : a*z.
// ----------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prelu_pool_fwd_k(const bf16_t* __restrict__ z,
                                                        const float* __restrict__ alpha,
                                                        bf16_t* __restrict__ p, int N, int H, int W,
                                                        int C) {
  const int PH = H >> 1, PW = W >> 1, C8 = C >> 3;
  const long total = (long)N * PH * PW * C8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c8 = i % C8;
    long t = i / C8;
    const int pw = t % PW; t /= PW;
    const int ph = t % PH; const int n = t / PH;
    float best[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) best[j] = -INFINITY;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = 2 * ph + (q >> 1), w = 2 * pw + (q & 1);
      const long off = (((long)n * H + h) * W + w) * C + c8 * 8;
      const long aoff = ((long)h * W + w) * C + c8 * 8;
      float zv[8];
      unpack8(*(const U4*)(z + off), zv);
      const float4 a0 = *(const float4*)(alpha + aoff), a1 = *(const float4*)(alpha + aoff + 4);
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float y = zv[j] > 0.f ? zv[j] : av[j] * zv[j];
        best[j] = fmaxf(best[j], y);
      }
    }
    *(U4*)(p + i * 8) = pack8(best);
  }
}

// Per-channel reduction of db[8] (channels c8*8..+7) over a 256-thread block whose threads hold
// channel group (tid % C8): xor-shuffles over the lanes that share a channel group (strides >= C8),
// then one LDS slot per (wave, channel) and one global atomic per channel per block.
PTG_DEV void bias_reduce_atomic(float db[8], int c8, int C8, float* sred, float* dbias) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, C = C8 * 8;
  if (C8 & (C8 - 1)) {  // channel groups not a power of two: LDS atomics
    if ((int)threadIdx.x < C) sred[threadIdx.x] = 0.f;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&sred[c8 * 8 + j], db[j]);
    __syncthreads();
    if ((int)threadIdx.x < C) atomicAdd(dbias + threadIdx.x, sred[threadIdx.x]);
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
    for (int o = 32; o >= C8; o >>= 1) db[j] += __shfl_xor(db[j], o, 64);
  if (lane < C8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) sred[wid * 256 + lane * 8 + j] = db[j];
  }
  __syncthreads();
  if ((int)threadIdx.x < C)
    atomicAdd(dbias + threadIdx.x,
              sred[threadIdx.x] + sred[256 + threadIdx.x] + sred[512 + threadIdx.x] + sred[768 + threadIdx.x]);
}

// Backward of prelu+pool, sample-parallel inside the block: 256 threads = 16 pooled positions x 16
// sample groups, so a block owns its 16 positions over a whole batch chunk and reduces dalpha over
// the sample groups in LDS.  Large layers run one chunk (dalpha += without atomics: no other block
// touches those elements); small layers split the batch over a few chunks and add with atomics.
// (the rejected per-block variant added every block's dalpha partial with fp32 atomics: ~17M per
// layer at batch 256.)
// dword w of a 2- or 4-dword vector (w a compile-time constant after unrolling): keeps the vectors
// in registers - indexing them through a uint32_t* put them in scratch memory
PTG_DEV uint32_t vword(const U2& v, int w) { return w == 0 ? v.x : v.y; }
PTG_DEV uint32_t vword(const U4& v, int w) { return w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w; }
PTG_DEV void vset(U2& v, int w, uint32_t x) { if (w == 0) v.x = x; else v.y = x; }
PTG_DEV void vset(U4& v, int w, uint32_t x) {
  if (w == 0) v.x = x; else if (w == 1) v.y = x; else if (w == 2) v.z = x; else v.w = x;
}

// STORE = false: dalpha / dbias only (dz already produced by the dgrad epilogue of the layer above,
// conv.hip EPI_PPB): the same loads and arithmetic, no dz stores.
template <int CH, bool STORE = true>
__global__ __launch_bounds__(256, 4) void prelu_pool_bwd_sg_k(const bf16_t* __restrict__ dp,
                                                           const bf16_t* __restrict__ z,
                                                           const float* __restrict__ alpha,
                                                           bf16_t* __restrict__ dz, float* __restrict__ dalpha,
                                                           float* __restrict__ dbias, int N, int H, int W,
                                                           int C, int nper) {
  // CH channels per thread (4: every per-thread array halves - 4 window positions x CH alphas and
  // dalpha sums - so the kernel runs 4 waves per SIMD instead of 2 at CH = 8 with 255 VGPRs)
  constexpr int PB = 16, SG = 16, NV = 4 * CH, RP = NV + 1;
  using V = typename std::conditional<CH == 8, U4, U2>::type;
  __shared__ float sda[SG * PB * RP];
  __shared__ float sdb[256];
  const int PH = H >> 1, PW = W >> 1, CG = C / CH;
  const int npos = PH * PW * CG;
  const int pl = threadIdx.x & (PB - 1), sg = threadIdx.x / PB;
  const int i = blockIdx.x * PB + pl;
  const int n0 = blockIdx.y * nper, n1 = min(N, n0 + nper);
  const bool active = i < npos;
  const int cg = active ? i % CG : 0;
  const int t = active ? i / CG : 0;
  const int pw = t % PW, ph = t / PW;
  // window position q = 2*dh + dw sits at zbase + dh*W*C + dw*C (the row/column steps are uniform,
  // so only zbase lives in a vector register)
  const uint32_t zbase = (uint32_t)((2 * ph * W + 2 * pw) * C + cg * CH), rowC = (uint32_t)(W * C);
  auto zoff = [&](int q) { return zbase + (uint32_t)(q >> 1) * rowC + (uint32_t)(q & 1) * (uint32_t)C; };
  const uint32_t HWC = (uint32_t)(H * W * C), PHWC = (uint32_t)(PH * PW * C);
  const uint32_t poff = (uint32_t)((ph * PW + pw) * C + cg * CH);
  float da[4][CH], db[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) db[j] = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < CH; ++j) da[q][j] = 0.f;
  if ((int)threadIdx.x < C) sdb[threadIdx.x] = 0.f;
  auto bload = [](Rsrc r, uint32_t off) -> V {
    if constexpr (CH == 8) return bload16(r, off); else return bload8(r, off);
  };
  if (active) {
    float av[4][CH];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < CH; j += 4) {
        const float4 a4 = *(const float4*)(alpha + zoff(q) + j);
        av[q][j] = a4.x; av[q][j + 1] = a4.y; av[q][j + 2] = a4.z; av[q][j + 3] = a4.w;
      }
    const bool lastw = (W & 1) && pw == PW - 1, lasth = (H & 1) && ph == PH - 1;
    const Rsrc dpr = make_rsrc(dp, (uint32_t)N * PHWC * 2u), zr = make_rsrc(z, (uint32_t)N * HWC * 2u);
    // one sample per iteration with the next sample's 5 loads in flight during this one's math
    V gc, zc[4];
    auto ld = [&](int nn, V& gq, V* zq) {
      gq = bload(dpr, ((uint32_t)nn * PHWC + poff) * 2u);
#pragma unroll
      for (int q = 0; q < 4; ++q) zq[q] = bload(zr, ((uint32_t)nn * HWC + zoff(q)) * 2u);
    };
    if (n0 + sg < n1) ld(n0 + sg, gc, zc);
    for (int n = n0 + sg; n < n1; n += SG) {
      V gn, zn[4];
      ld(min(n + SG, n1 - 1), gn, zn);
      uint32_t ow[4][CH / 2];
#pragma unroll
      for (int w = 0; w < CH / 2; ++w) {
        float ov[2][4];
        const uint32_t gww = vword(gc, w);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int jj = 2 * w + h;
          const float gj = h ? hi_bf(gww) : lo_bf(gww);
          float zq[4], yq[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t word = vword(zc[q], w);
            zq[q] = h ? hi_bf(word) : lo_bf(word);
            yq[q] = zq[q] > 0.f ? zq[q] : av[q][jj] * zq[q];
          }
          int a = 0;
          float b = yq[0];
#pragma unroll
          for (int q = 1; q < 4; ++q)
            if (yq[q] > b) { b = yq[q]; a = q; }  // first maximum in q order, as the forward's pool
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float gq = a == q ? gj : 0.f;
            const bool pos = zq[q] > 0.f;
            ov[h][q] = pos ? gq : gq * av[q][jj];
            da[q][jj] += pos ? 0.f : gq * zq[q];
            db[jj] += ov[h][q];
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) ow[q][w] = pack_bf(ov[0][q], ov[1][q]);
      }
      const long nb = (long)n * HWC;
      if constexpr (STORE) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          V o;
#pragma unroll
          for (int w = 0; w < CH / 2; ++w) vset(o, w, ow[q][w]);
          *(V*)(dz + nb + zoff(q)) = o;
        }
      } else {
        (void)ow;
      }
      gc = gn;
#pragma unroll
      for (int q = 0; q < 4; ++q) zc[q] = zn[q];
      if (STORE && (lastw || lasth)) {  // odd H / W: the row / column outside every window gets zero gradient
        V zz;
#pragma unroll
        for (int w = 0; w < CH / 2; ++w) vset(zz, w, 0u);
        bf16_t* d = dz + nb + cg * CH;
        if (lastw) {
          *(V*)(d + ((long)(2 * ph) * W + W - 1) * C) = zz;
          *(V*)(d + ((long)(2 * ph + 1) * W + W - 1) * C) = zz;
        }
        if (lasth) {
          *(V*)(d + ((long)(H - 1) * W + 2 * pw) * C) = zz;
          *(V*)(d + ((long)(H - 1) * W + 2 * pw + 1) * C) = zz;
        }
        if (lastw && lasth) *(V*)(d + ((long)(H - 1) * W + W - 1) * C) = zz;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < CH; ++j) sda[(sg * PB + pl) * RP + q * CH + j] = da[q][j];
  __syncthreads();
  if (active) {  // bias: LDS atomics per channel, then one global atomic per channel and block
#pragma unroll
    for (int j = 0; j < CH; ++j) atomicAdd(&sdb[cg * CH + j], db[j]);
  }
  // dalpha: PB positions x NV values per block, summed over the sample groups
  for (int o = threadIdx.x; o < PB * NV; o += 256) {
    const int p = o / NV, k = o % NV, q = k / CH, j = k % CH;
    float sum = 0.f;
#pragma unroll
    for (int gsg = 0; gsg < SG; ++gsg) sum += sda[(gsg * PB + p) * RP + k];
    const int ii = blockIdx.x * PB + p;
    if (ii < npos) {
      const int cc = ii % CG, tq = ii / CG, pww = tq % PW, phh = tq / PW;
      float* dst = dalpha + ((long)(2 * phh + (q >> 1)) * W + 2 * pww + (q & 1)) * C + cc * CH + j;
      if (gridDim.y == 1) *dst += sum;
      else atomicAdd(dst, sum);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < C) atomicAdd(dbias + threadIdx.x, sdb[threadIdx.x]);
}

// Backward of prelu+pool from the sparse forward record (conv.hip EPI_POOLS): per pooled element the
// argmax position q (uint8) and the z there (bf16).  dz is dense (zero off the argmax), dalpha and
// dbias as in prelu_pool_bwd_sg_k.  Reads dp + zsel + arg (2.5 B per pooled element) instead of the
// four z values of each window (8 B).
__global__ __launch_bounds__(256) void prelu_pool_bwd_sparse_k(const bf16_t* __restrict__ dp,
                                                               const bf16_t* __restrict__ zs,
                                                               const uint8_t* __restrict__ arg,
                                                               const float* __restrict__ alpha,
                                                               bf16_t* __restrict__ dz, float* __restrict__ dalpha,
                                                               float* __restrict__ dbias, int N, int H, int W, int C,
                                                               int nper) {
  __shared__ float sred[4 * 256];
  __shared__ float sda[256 * 32];
  const int PH = H >> 1, PW = W >> 1, C8 = C >> 3;
  const int npos = PH * PW * C8;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n0 = blockIdx.y * nper, n1 = min(N, n0 + nper);
  float db[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool active = i < npos;
  const int c8 = active ? i % C8 : 0;
  const int t = active ? i / C8 : 0;
  const int pw = t % PW, ph = t / PW;
  long zoff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) zoff[q] = ((long)(2 * ph + (q >> 1)) * W + 2 * pw + (q & 1)) * C + c8 * 8;
  const long HWC = (long)H * W * C, PHWC = (long)PH * PW * C;
  const long poff = ((long)ph * PW + pw) * C + c8 * 8;
  if (active) {
    float da[4][8], av[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a0 = *(const float4*)(alpha + zoff[q]), a1 = *(const float4*)(alpha + zoff[q] + 4);
      av[q][0] = a0.x; av[q][1] = a0.y; av[q][2] = a0.z; av[q][3] = a0.w;
      av[q][4] = a1.x; av[q][5] = a1.y; av[q][6] = a1.z; av[q][7] = a1.w;
#pragma unroll
      for (int j = 0; j < 8; ++j) da[q][j] = 0.f;
    }
    for (int n = n0; n < n1; n += 4) {  // 4 samples in flight: 12 independent loads per lane
      U4 graw[4], zraw[4];
      U2 araw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int nn = min(n + u, n1 - 1);
        graw[u] = *(const U4*)(dp + nn * PHWC + poff);
        zraw[u] = *(const U4*)(zs + nn * PHWC + poff);
        araw[u] = *(const U2*)(arg + nn * PHWC + poff);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (n + u >= n1) break;
        const long nb = (long)(n + u) * HWC;
        float g[8], zv[8];
        unpack8(graw[u], g);
        unpack8(zraw[u], zv);
        const uint8_t* ab = (const uint8_t*)&araw[u];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const bool hit = ab[j] == q;
            const float gq = hit ? g[j] : 0.f;
            o[j] = zv[j] > 0.f ? gq : gq * av[q][j];
            da[q][j] += (hit && !(zv[j] > 0.f)) ? gq * zv[j] : 0.f;
            db[j] += o[j];
          }
          *(U4*)(dz + nb + zoff[q]) = pack8(o);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) sda[(((q >> 1) * 256 + threadIdx.x) * 2 + (q & 1)) * 8 + j] = da[q][j];
  }
  __syncthreads();
  for (int k = 0; k < 32; ++k) {
    const int L = k * 256 + threadIdx.x;
    const int j = L & 7, qw = (L >> 3) & 1, tt = (L >> 4) & 255, qh = L >> 12;
    const int ii = blockIdx.x * 256 + tt;
    if (ii >= npos) continue;
    const int cc = ii % C8, tq = ii / C8, pww = tq % PW, phh = tq / PW;
    atomicAdd(dalpha + ((long)(2 * phh + qh) * W + 2 * pww + qw) * C + cc * 8 + j, sda[L]);
  }
  bias_reduce_atomic(db, c8, C8, sred, dbias);
}

// Sparse in, sparse out (the first conv layer, whose dZ only feeds the sparse-dZ weight gradient):
// from the forward's record (zsel = z at each window's argmax, arg = its position q) it writes
// dzsel = d(prelu)/dz at the argmax, i.e. dZ's only non-zero of the window, in the pooled layout.
// Sample-parallel like prelu_pool_bwd_sg_k (16 pooled positions x 16 sample groups per block,
// dalpha reduced over the sample groups in LDS); per pooled element of 8 channels it moves
// dp + zsel + arg + dzsel = 56 bytes instead of the dense backward's 144.
__global__ __launch_bounds__(256) void prelu_pool_bwd_sel_k(const bf16_t* __restrict__ dp,
                                                            const bf16_t* __restrict__ zs,
                                                            const uint8_t* __restrict__ arg,
                                                            const float* __restrict__ alpha,
                                                            bf16_t* __restrict__ dzs, float* __restrict__ dalpha,
                                                            float* __restrict__ dbias, int N, int H, int W,
                                                            int C, int nper) {
  constexpr int PB = 16, SG = 16, RP = 33;
  __shared__ float sda[SG * PB * RP];
  __shared__ float sdb[256];
  const int PH = H >> 1, PW = W >> 1, C8 = C >> 3;
  const int npos = PH * PW * C8;
  const int pl = threadIdx.x & (PB - 1), sg = threadIdx.x / PB;
  const int i = blockIdx.x * PB + pl;
  const int n0 = blockIdx.y * nper, n1 = min(N, n0 + nper);
  const bool active = i < npos;
  const int c8 = active ? i % C8 : 0;
  const int t = active ? i / C8 : 0;
  const int pw = t % PW, ph = t / PW;
  long zoff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) zoff[q] = ((long)(2 * ph + (q >> 1)) * W + 2 * pw + (q & 1)) * C + c8 * 8;
  const long PHWC = (long)PH * PW * C;
  const long poff = ((long)ph * PW + pw) * C + c8 * 8;
  float da[4][8], db[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) db[j] = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) da[q][j] = 0.f;
  if ((int)threadIdx.x < C) sdb[threadIdx.x] = 0.f;
  if (active) {
    float av[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a0 = *(const float4*)(alpha + zoff[q]), a1 = *(const float4*)(alpha + zoff[q] + 4);
      av[q][0] = a0.x; av[q][1] = a0.y; av[q][2] = a0.z; av[q][3] = a0.w;
      av[q][4] = a1.x; av[q][5] = a1.y; av[q][6] = a1.z; av[q][7] = a1.w;
    }
    constexpr int U = 4;  // samples in flight per thread: 12 independent loads
    for (int n = n0 + sg; n < n1; n += U * SG) {
      U4 graw[U], zraw[U];
      U2 araw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int nn = n + u * SG < n1 ? n + u * SG : n;
        const long o = (long)nn * PHWC + poff;
        graw[u] = *(const U4*)(dp + o);
        zraw[u] = *(const U4*)(zs + o);
        araw[u] = *(const U2*)(arg + o);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (n + u * SG >= n1) break;
        float g[8], zv[8], o[8];
        unpack8(graw[u], g);
        unpack8(zraw[u], zv);
        const uint32_t aw[2] = {araw[u].x, araw[u].y};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int q = (aw[j >> 2] >> (8 * (j & 3))) & 3;
          const float a = q == 0 ? av[0][j] : q == 1 ? av[1][j] : q == 2 ? av[2][j] : av[3][j];
          const bool pos = zv[j] > 0.f;
          o[j] = pos ? g[j] : g[j] * a;
          const float d = pos ? 0.f : g[j] * zv[j];
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) da[qq][j] += q == qq ? d : 0.f;
          db[j] += o[j];
        }
        *(U4*)(dzs + PTG_CHECKED_IDX((long)(n + u * SG) * PHWC + poff, (long)N * PHWC)) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) sda[(sg * PB + pl) * RP + q * 8 + j] = da[q][j];
  __syncthreads();
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&sdb[c8 * 8 + j], db[j]);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int o = h * 256 + threadIdx.x;
    const int p = o >> 5, k = o & 31, q = k >> 3, j = k & 7;
    float sum = 0.f;
#pragma unroll
    for (int gsg = 0; gsg < SG; ++gsg) sum += sda[(gsg * PB + p) * RP + k];
    const int ii = blockIdx.x * PB + p;
    if (ii < npos) {
      const int cc = ii % C8, tq = ii / C8, pww = tq % PW, phh = tq / PW;
      float* dst = dalpha + ((long)(2 * phh + (q >> 1)) * W + 2 * pww + (q & 1)) * C + cc * 8 + j;
      if (gridDim.y == 1) *dst += sum;
      else atomicAdd(dst, sum);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < C) atomicAdd(dbias + threadIdx.x, sdb[threadIdx.x]);
}

// Plain PReLU forward (no pool): a = z>0 ? z : alpha[hwc]*z ; HWC = per-sample element count.
__global__ __launch_bounds__(256) void prelu_fwd_k(const bf16_t* __restrict__ z,
                                                   const float* __restrict__ alpha,
                                                   bf16_t* __restrict__ a, long total8, int HWC8) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total8; i += (long)gridDim.x * 256) {
    const long e = (i % HWC8) * 8;
    float zv[8];
    unpack8(*(const U4*)(z + i * 8), zv);
    const float4 a0 = *(const float4*)(alpha + e), a1 = *(const float4*)(alpha + e + 4);
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) zv[j] = zv[j] > 0.f ? zv[j] : av[j] * zv[j];
    *(U4*)(a + i * 8) = pack8(zv);
  }
}

// PReLU backward, sample-parallel (the prelu_pool_bwd_sg_k layout without the pool): a block owns
// 16 8-element positions over a batch chunk split into 16 sample groups and reduces dalpha over the
// groups in LDS - one dalpha add per element and chunk instead of one fp32 atomic per element and
// sample pair (the rejected per-pair variant: 2.6M contended atomics for CNN-B1's last conv layer at batch 256).
template <bool STORE = true>  // false: dalpha / dbias only (dz made by the Dense dX epilogue, gemm.hip out2)
__global__ __launch_bounds__(256) void prelu_bwd_sg_k(const bf16_t* __restrict__ da, const bf16_t* __restrict__ z,
                                                      const float* __restrict__ alpha, bf16_t* __restrict__ dz,
                                                      float* __restrict__ dalpha, float* __restrict__ dbias, int N,
                                                      int HWC, int C, int nper) {
  constexpr int PB = 16, SG = 16, RP = 9, U = 4;
  __shared__ float sda[SG * PB * RP];
  __shared__ float sdb[256];
  const int HWC8 = HWC >> 3, C8 = C >> 3;
  const int pl = threadIdx.x & (PB - 1), sg = threadIdx.x / PB;
  const int i = blockIdx.x * PB + pl;
  const int n0 = blockIdx.y * nper, n1 = min(N, n0 + nper);
  const bool active = i < HWC8;
  const long e = (long)(active ? i : 0) * 8;
  float dal[8], db[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { dal[j] = 0.f; db[j] = 0.f; }
  if ((int)threadIdx.x < C) sdb[threadIdx.x] = 0.f;
  if (active) {
    const float4 a0 = *(const float4*)(alpha + e), a1 = *(const float4*)(alpha + e + 4);
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    for (int n = n0 + sg; n < n1; n += U * SG) {
      U4 graw[U], zraw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long o = (long)(n + u * SG < n1 ? n + u * SG : n) * HWC + e;
        graw[u] = *(const U4*)(da + o);
        zraw[u] = *(const U4*)(z + o);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (n + u * SG >= n1) break;
        float g[8], zv[8], o[8];
        unpack8(graw[u], g);
        unpack8(zraw[u], zv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool pos = zv[j] > 0.f;
          o[j] = pos ? g[j] : g[j] * av[j];
          dal[j] += pos ? 0.f : g[j] * zv[j];
          db[j] += o[j];
        }
        if constexpr (STORE) *(U4*)(dz + (long)(n + u * SG) * HWC + e) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) sda[(sg * PB + pl) * RP + j] = dal[j];
  __syncthreads();
  if (active) {
    const int c8 = i % C8;
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&sdb[c8 * 8 + j], db[j]);
  }
  if (threadIdx.x < PB * 8) {
    const int p = threadIdx.x >> 3, j = threadIdx.x & 7;
    float sum = 0.f;
#pragma unroll
    for (int gsg = 0; gsg < SG; ++gsg) sum += sda[(gsg * PB + p) * RP + j];
    const int ii = blockIdx.x * PB + p;
    if (ii < HWC8) {
      float* dst = dalpha + (long)ii * 8 + j;
      if (gridDim.y == 1) *dst += sum;
      else atomicAdd(dst, sum);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < C) atomicAdd(dbias + threadIdx.x, sdb[threadIdx.x]);
}

// out_bf16[m][n] = act(acc[m][n] + bias[n])   (split-K GEMM finishing pass)
// clear: zero the accumulator after reading it, so the next split-K GEMM into it needs no fill
__global__ __launch_bounds__(256) void bias_act_k(float* __restrict__ acc,
                                                  const float* __restrict__ bias, bf16_t* __restrict__ out,
                                                  float* __restrict__ out32, long total, int N, int act, int clear) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    float v = acc[i] + (bias ? bias[i % N] : 0.f);
    if (clear) acc[i] = 0.f;
    if (act == 1) v = fmaxf(v, 0.f);
    if (out) out[i] = f2bf(v);
    if (out32) out32[i] = v;
  }
}

// db[n] += sum_m g[m][n] (g bf16 or f32). One thread per column, coalesced across n.
template <typename T>
__global__ __launch_bounds__(256) void col_sum_k(const T* __restrict__ g, float* __restrict__ db, int M,
                                                 int N, int mper) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int m0 = blockIdx.y * mper, m1 = min(M, m0 + mper);
  float s = 0.f;
  for (int m = m0; m < m1; ++m) {
    if constexpr (sizeof(T) == 2) s += bf2f(g[(long)m * N + n]);
    else s += g[(long)m * N + n];
  }
  atomicAdd(db + n, s);
}

template <typename T> PTG_DEV float ldf(const T* p, long i) {
  if constexpr (sizeof(T) == 2) return bf2f(p[i]); else return p[i];
}

// ----------------------------------------------------------------------------------------------
// Skinny dense layers (N <= 64 outputs or tiny K): fp32 math, VALU.  Used by the CSV-MLP
// (3->16->32->64->15, 3,695 params: launch-bound, not FLOP-bound) and the CNN's Dense(2) head.
// ----------------------------------------------------------------------------------------------
// act: 0 none, 1 relu, 2 softmax (row-wise over N)
template <typename TX>
__global__ __launch_bounds__(256) void dense_small_fwd_k(const TX* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, float* __restrict__ y,
                                                         bf16_t* __restrict__ ybf, int M, int K, int N, int act) {
  // one wave per row; lanes stride K; N accumulators reduced across the wave
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float out_keep = 0.f;
  float rowmax = -INFINITY;
  for (int n = 0; n < N; ++n) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += ldf(x, (long)m * K + k) * w[(long)n * K + k];
    s = wave_sum(s) + (b ? b[n] : 0.f);
    if (act == 1) s = fmaxf(s, 0.f);
    if (lane == n) out_keep = s;
    rowmax = fmaxf(rowmax, s);
  }
  if (act == 2) {
    const float e = lane < N ? __expf(out_keep - rowmax) : 0.f;
    const float tot = wave_sum(e);
    out_keep = e / tot;
  }
  if (lane < N) {
    y[(long)m * N + lane] = out_keep;
    if (ybf) ybf[(long)m * N + lane] = f2bf(out_keep);
  }
}

// Narrow-K forward (K <= 64, e.g. the CSV MLP's 3 -> 16 -> 32 -> 64 layers at large batch): one
// thread per output element, no softmax (act 0/1).
template <typename TX>
__global__ __launch_bounds__(256) void dense_small_fwd_t_k(const TX* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ b, float* __restrict__ y,
                                                           bf16_t* __restrict__ ybf, int M, int K, int N, int act) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= (long)M * N) return;
  const int m = i / N, n = i - (long)m * N;
  float s = b ? b[n] : 0.f;
  for (int k = 0; k < K; ++k) s += ldf(x, (long)m * K + k) * w[(long)n * K + k];
  if (act == 1) s = fmaxf(s, 0.f);
  y[i] = s;
  if (ybf) ybf[i] = f2bf(s);
}

// dx[m][k] = (sum_n dy[m][n] w[n][k]) * (mask ? (mask[m][k] > 0) : 1)
template <typename TM, typename TO>
__global__ __launch_bounds__(256) void dense_small_dx_k(const float* __restrict__ dy, const float* __restrict__ w,
                                                        const TM* __restrict__ mask, TO* __restrict__ dx, int M,
                                                        int K, int N) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= (long)M * K) return;
  const int m = i / K, k = i - (long)m * K;
  float s = 0.f;
  for (int n = 0; n < N; ++n) s += dy[(long)m * N + n] * w[(long)n * K + k];
  if (mask && !(ldf(mask, i) > 0.f)) s = 0.f;
  if constexpr (sizeof(TO) == 2) dx[i] = f2bf(s); else dx[i] = s;
}

// dw[n][k] += sum_m dy[m][n] x[m][k];  db[n] += sum_m dy[m][n]
template <typename TX>
// dW[N][K] += dy^T x, db[N] += colsum(dy): thread per output, blockIdx.y = slice of the M rows
// (split-M with fp32 atomics, so a large batch - the joint pipeline's 8192-row MLP batches - is not
// a serial loop per thread).
__global__ __launch_bounds__(256) void dense_small_dw_k(const float* __restrict__ dy, const TX* __restrict__ x,
                                                        float* __restrict__ dw, float* __restrict__ db, int M,
                                                        int K, int N, int rows_per_slice) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  const int m0 = blockIdx.y * rows_per_slice, m1 = min(M, m0 + rows_per_slice);
  const bool single = gridDim.y == 1;
  if (i < (long)N * K) {
    const int n = i / K, k = i - (long)n * K;
    float s = 0.f;
    for (int m = m0; m < m1; ++m) s += dy[(long)m * N + n] * ldf(x, (long)m * K + k);
    if (single) dw[i] += s; else atomicAdd(dw + i, s);
  }
  if (db && i < N) {
    float s = 0.f;
    for (int m = m0; m < m1; ++m) s += dy[(long)m * N + i];
    if (single) db[i] += s; else atomicAdd(db + i, s);
  }
}

// ----------------------------------------------------------------------------------------------
// Losses. Single workgroup (B*D is tiny). stats: [loss_sum, abs_sum, sq_sum, count] accumulate.
// ----------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mse_k(const float* __restrict__ pred, const float* __restrict__ y,
                                             float* __restrict__ dpred, float* __restrict__ stats, int total,
                                             int B, float gscale) {
  __shared__ float scr[4];
  float se = 0.f, ae = 0.f;
  const float inv = 1.f / (float)total;
  for (int i = threadIdx.x; i < total; i += 256) {
    const float d = pred[i] - y[i];
    se += d * d; ae += fabsf(d);
    dpred[i] = 2.f * d * inv * gscale;
  }
  const float sse = block_sum256(se, scr);
  __syncthreads();
  const float sae = block_sum256(ae, scr);
  if (threadIdx.x == 0) {
    // Keras Mean tracker of per-batch loss (mean over batch of per-sample mean over D)
    stats[0] += sse * inv * (float)B;   // loss_sum weighted by batch count
    stats[1] += sae;                    // abs error sum (MAE metric numerator)
    stats[2] += sse;                    // squared error sum (MSE metric numerator)
    stats[3] += (float)total;           // element count
    stats[4] += (float)B;               // sample count
  }
}

// ----------------------------------------------------------------------------------------------
// Fused regression head (CNN-B1's Dense(2048, relu) -> Dense(2) -> MSE, train_tf_ps.py:366-378):
// two launches instead of bias_act / dense_small_fwd / mse / dense_small_dw / dense_small_dx /
// col_sum / the split-K accumulator fill.
//   head_row_k  one workgroup per sample row: h = relu(acc + b1) (fp32), pred = h.W2 + b2, the
//               row's squared / absolute error and dpred (mse_k's formulas), then
//               dz1 = (dpred.W2) * [h > 0] as bf16 for Dense1's dX / dW GEMMs
//   head_col_k  one thread per hidden unit (x 4 row groups): dW2 += dpred^T h, db1 += sum dz1,
//               re-zeroes acc for the next step's split-K atomics; workgroup (0, 0) also reduces the
//               per-row errors into the metric stats and dpred into db2
// ----------------------------------------------------------------------------------------------
#define HEAD_RG 4
template <int N2>
// nparts > 0: acc holds nparts split-K partial slices [nparts][B][K1] (dense.hip plain-store
// forward); the row pass sums them, and leaves h = relu(sum + b1) in slice 0 for head_col_k.
// nparts == 0: acc holds the summed split-K sums (atomic forward) and head_col_k re-zeroes it.
__global__ __launch_bounds__(256) void head_row_k(float* __restrict__ acc, const float* __restrict__ b1,
                                                  const float* __restrict__ w2, const float* __restrict__ b2,
                                                  const float* __restrict__ tgt, bf16_t* __restrict__ dz1,
                                                  float* __restrict__ dpred, float* __restrict__ rowerr,
                                                  float* __restrict__ pred_out, int B, int K1, float gscale,
                                                  int nparts) {
  __shared__ float red[4][N2];
  __shared__ float sdp[N2];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float* arow = acc + (long)m * K1;
  const long pstride = (long)B * K1;
  float dot[N2];
#pragma unroll
  for (int n = 0; n < N2; ++n) dot[n] = 0.f;
  for (int k = tid; k < K1; k += 256) {
    float a = arow[k];
    for (int p = 1; p < nparts; ++p) a += arow[p * pstride + k];
    const float h = fmaxf(a + b1[k], 0.f);
    if (nparts) arow[k] = h;
#pragma unroll
    for (int n = 0; n < N2; ++n) dot[n] = fmaf(h, w2[(long)n * K1 + k], dot[n]);
  }
#pragma unroll
  for (int n = 0; n < N2; ++n) {
    const float v = wave_sum(dot[n]);
    if (lane == 0) red[w][n] = v;
  }
  __syncthreads();
  if (tid == 0) {
    const float inv = 1.f / (float)(B * N2);
    float se = 0.f, ae = 0.f;
#pragma unroll
    for (int n = 0; n < N2; ++n) {
      const float p = red[0][n] + red[1][n] + red[2][n] + red[3][n] + b2[n];
      const float d = p - tgt[(long)m * N2 + n];
      se += d * d;
      ae += fabsf(d);
      sdp[n] = 2.f * d * inv * gscale;
      dpred[(long)m * N2 + n] = sdp[n];
      if (pred_out) pred_out[(long)m * N2 + n] = p;
    }
    rowerr[2 * m] = se;
    rowerr[2 * m + 1] = ae;
  }
  __syncthreads();
  float dp[N2];
#pragma unroll
  for (int n = 0; n < N2; ++n) dp[n] = sdp[n];
  for (int k = tid; k < K1; k += 256) {
    const float h = nparts ? arow[k] : fmaxf(arow[k] + b1[k], 0.f);  // (this thread's own store above)
    float g = 0.f;
#pragma unroll
    for (int n = 0; n < N2; ++n) g = fmaf(dp[n], w2[(long)n * K1 + k], g);
    dz1[(long)m * K1 + k] = f2bf(h > 0.f ? g : 0.f);
  }
}

// head_row_k for split-K partial slices (dense.hip forward), K1 % 4 == 0 and K1 <= 4 * 512: one
// workgroup per row, one float4 column group per thread, all NP slice loads of a thread issued
// before the first add (the slices are HBM / Infinity-Cache reads: a load-add-load loop exposes
// their latency NP times).  Leaves h = relu(sum + b1) in slice 0 for head_col_k.
template <int N2, int NP>
__global__ __launch_bounds__(512) void head_row_parts_k(float* __restrict__ acc, const float* __restrict__ b1,
                                                        const float* __restrict__ w2, const float* __restrict__ b2,
                                                        const float* __restrict__ tgt, bf16_t* __restrict__ dz1,
                                                        float* __restrict__ dpred, float* __restrict__ rowerr,
                                                        float* __restrict__ pred_out, int B, int K1, float gscale,
                                                        int nparts) {
  __shared__ float red[8][N2];
  __shared__ float sdp[N2];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int k = tid * 4;
  const bool on = k < K1;
  float4* arow = (float4*)(acc + (long)m * K1);
  const long ps4 = (long)B * K1 / 4;
  float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
  float dot[N2];
#pragma unroll
  for (int n = 0; n < N2; ++n) dot[n] = 0.f;
  if (on) {
    float4 u[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) u[p] = p < nparts ? arow[p * ps4 + tid] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = NP; p < nparts; ++p) {  // (more slices than the template holds)
      const float4 v = arow[p * ps4 + tid];
      u[0].x += v.x; u[0].y += v.y; u[0].z += v.z; u[0].w += v.w;
    }
    float4 a = u[0];
#pragma unroll
    for (int p = 1; p < NP; ++p) { a.x += u[p].x; a.y += u[p].y; a.z += u[p].z; a.w += u[p].w; }
    h.x = fmaxf(a.x + b1[k], 0.f); h.y = fmaxf(a.y + b1[k + 1], 0.f);
    h.z = fmaxf(a.z + b1[k + 2], 0.f); h.w = fmaxf(a.w + b1[k + 3], 0.f);
    arow[tid] = h;
#pragma unroll
    for (int n = 0; n < N2; ++n) {
      const float* wn = w2 + (long)n * K1 + k;
      dot[n] = h.x * wn[0] + h.y * wn[1] + h.z * wn[2] + h.w * wn[3];
    }
  }
#pragma unroll
  for (int n = 0; n < N2; ++n) {
    const float v = wave_sum(dot[n]);
    if (lane == 0) red[w][n] = v;
  }
  __syncthreads();
  if (tid == 0) {
    const float inv = 1.f / (float)(B * N2);
    float se = 0.f, ae = 0.f;
#pragma unroll
    for (int n = 0; n < N2; ++n) {
      float p = b2[n];
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) p += red[ww][n];
      const float d = p - tgt[(long)m * N2 + n];
      se += d * d;
      ae += fabsf(d);
      sdp[n] = 2.f * d * inv * gscale;
      dpred[(long)m * N2 + n] = sdp[n];
      if (pred_out) pred_out[(long)m * N2 + n] = p;
    }
    rowerr[2 * m] = se;
    rowerr[2 * m + 1] = ae;
  }
  __syncthreads();
  if (on) {
    float g[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < N2; ++n) {
      const float d = sdp[n];
      const float* wn = w2 + (long)n * K1 + k;
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = fmaf(d, wn[j], g[j]);
    }
    const float hv[4] = {h.x, h.y, h.z, h.w};
    uint2 o;
    o.x = pack_bf(hv[0] > 0.f ? g[0] : 0.f, hv[1] > 0.f ? g[1] : 0.f);
    o.y = pack_bf(hv[2] > 0.f ? g[2] : 0.f, hv[3] > 0.f ? g[3] : 0.f);
    *(uint2*)(dz1 + (long)m * K1 + k) = o;
  }
}

template <int N2>
__global__ __launch_bounds__(256) void head_col_k(float* __restrict__ acc, const float* __restrict__ b1,
                                                  const float* __restrict__ w2, const float* __restrict__ dpred,
                                                  const float* __restrict__ rowerr, float* __restrict__ dw2,
                                                  float* __restrict__ db2, float* __restrict__ db1,
                                                  float* __restrict__ stats, int B, int K1, int nparts) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int rows = (B + HEAD_RG - 1) / HEAD_RG, m0 = blockIdx.y * rows, m1 = min(B, m0 + rows);
  if (k < K1) {
    const float bk = b1[k];
    float wk[N2], sw[N2];
#pragma unroll
    for (int n = 0; n < N2; ++n) { wk[n] = w2[(long)n * K1 + k]; sw[n] = 0.f; }
    float sb = 0.f;
    for (int m = m0; m < m1; ++m) {
      float* ap = acc + (long)m * K1 + k;
      float h;
      if (nparts) {
        h = *ap;  // head_row_k left relu(sum + b1) here
      } else {
        h = fmaxf(*ap + bk, 0.f);
        *ap = 0.f;
      }
      float g = 0.f;
#pragma unroll
      for (int n = 0; n < N2; ++n) {
        const float d = dpred[(long)m * N2 + n];
        g = fmaf(d, wk[n], g);
        sw[n] = fmaf(d, h, sw[n]);
      }
      sb += h > 0.f ? g : 0.f;
    }
#pragma unroll
    for (int n = 0; n < N2; ++n) atomicAdd(dw2 + (long)n * K1 + k, sw[n]);
    atomicAdd(db1 + k, sb);
  }
  if (blockIdx.x == 0 && blockIdx.y == 0) {
    __shared__ float scr[4];
    float se = 0.f, ae = 0.f, dsum[N2];
#pragma unroll
    for (int n = 0; n < N2; ++n) dsum[n] = 0.f;
    for (int m = threadIdx.x; m < B; m += 256) {
      se += rowerr[2 * m];
      ae += rowerr[2 * m + 1];
#pragma unroll
      for (int n = 0; n < N2; ++n) dsum[n] += dpred[(long)m * N2 + n];
    }
    const float tse = block_sum256(se, scr);
    __syncthreads();
    const float tae = block_sum256(ae, scr);
    float td[N2];
#pragma unroll
    for (int n = 0; n < N2; ++n) {
      __syncthreads();
      td[n] = block_sum256(dsum[n], scr);
    }
    if (threadIdx.x == 0) {
      const float inv = 1.f / (float)(B * N2);
      stats[0] += tse * inv * (float)B;
      stats[1] += tae;
      stats[2] += tse;
      stats[3] += (float)(B * N2);
      stats[4] += (float)B;
#pragma unroll
      for (int n = 0; n < N2; ++n) db2[n] += td[n];
    }
  }
}

// softmax + sparse categorical cross-entropy on logits (row per thread, C <= 64).
// probs clipped to [1e-7, 1-1e-7] like Keras' backend.  dlogits = (p - onehot) / B * gscale.
// stats: [loss_sum, correct, -, -, count]
// One wave per row (ResNet-50's 1000-class head: B rows x 1000 logits); lanes stride the classes.
__global__ __launch_bounds__(256) void softmax_xent_k(const float* __restrict__ logits,
                                                      const int* __restrict__ labels,
                                                      float* __restrict__ dlogits, float* __restrict__ stats,
                                                      int B, int C, float gscale) {
  // one wave per row, grid-strided; the loss / correct / count sums go through LDS to ONE set of
  // three atomics per workgroup (one per row contended on the same three words: 23 us at B = 512)
  __shared__ float red[4][3];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float loss = 0.f, hit = 0.f, cnt = 0.f;
  for (int b = blockIdx.x * 4 + w; b < B; b += gridDim.x * 4) {
    const float* r = logits + (long)b * C;
    float mx = -INFINITY;
    int am = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      const float v = r[c];
      if (v > mx) { mx = v; am = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // arg-max, lowest index on ties
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += __expf(r[c] - mx);
    s = wave_sum(s);
    const int lab = labels[b];
    const float inv = 1.f / s, scale = gscale / (float)B;
    for (int c = lane; c < C; c += 64) {
      const float pr = __expf(r[c] - mx) * inv;
      dlogits[(long)b * C + c] = (pr - (c == lab ? 1.f : 0.f)) * scale;
    }
    const float pl = fminf(fmaxf(__expf(r[lab] - mx) * inv, 1e-7f), 1.f - 1e-7f);
    loss += -__logf(pl);
    hit += am == lab ? 1.f : 0.f;
    cnt += 1.f;
  }
  if (lane == 0) { red[w][0] = loss; red[w][1] = hit; red[w][2] = cnt; }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (t != 0.f) atomicAdd(stats + (threadIdx.x == 2 ? 4 : threadIdx.x), t);
  }
}

// ----------------------------------------------------------------------------------------------
// Fused flat Adam over the whole parameter buffer (one launch per step, float4 vectorised).
// Writes the fp32 master weights and their bf16 compute copy.  gscale folds in the 1/world
// averaging of all-reduced gradients.
// ----------------------------------------------------------------------------------------------
// Device-resident optimizer step state (HIP-graph capturable update): st[0] = step count t (as
// float), st[1] = lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t) for the step about to run.
__global__ void adam_step_k(float* st, float lr, float b1, float b2) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float t = st[0] + 1.f;
    st[0] = t;
    st[1] = lr * sqrtf(1.f - powf(b2, t)) / (1.f - powf(b1, t));
  }
}

// clear: the gradient is consumed here, so store zeros back (4 B/parameter, no separate fill pass
// before the next backward: the store skips its per-step zero_grad after a clearing update)
__global__ __launch_bounds__(256) void adam_k(float* __restrict__ p, float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              bf16_t* __restrict__ pbf, long n4, float lr_t, float b1,
                                              float b2, float eps, float gscale, const float* __restrict__ lr_dev,
                                              int clear) {
  if (lr_dev) lr_t = lr_dev[1];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 pp = ((float4*)p)[i];
    const float4 gg = ((const float4*)g)[i];
    if (clear) ((float4*)g)[i] = float4{0.f, 0.f, 0.f, 0.f};
    float4 mm = ((float4*)m)[i], vv = ((float4*)v)[i];
    float* P = &pp.x; const float* G = &gg.x; float* Mm = &mm.x; float* V = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = G[j] * gscale;
      Mm[j] = b1 * Mm[j] + (1.f - b1) * gj;
      V[j] = b2 * V[j] + (1.f - b2) * gj * gj;
      P[j] -= lr_t * Mm[j] / (sqrtf(V[j]) + eps);
    }
    ((float4*)p)[i] = pp; ((float4*)m)[i] = mm; ((float4*)v)[i] = vv;
    if (pbf) {
      U2 o; o.x = pack_bf(pp.x, pp.y); o.y = pack_bf(pp.z, pp.w);
      ((U2*)pbf)[i] = o;
    }
  }
}

// Adam over up to 4 disjoint [lo, hi) ranges of the flat store in ONE launch (the ranges a fused
// step's gradient producers did not update: the conv / PReLU block before a big Dense and the
// tail after it), optionally writing the flipped bf16 dgrad filters of up to 4 conv kernels that lie
// inside those ranges: wf[ci][KS-1-kh][KS-1-kw][co] = bf16(new W[co][kh][kw][ci]).  The next
// backward's halo dgrad then reads them as they are (no conv_flip4_k launch on its critical path).
struct AdamRanges { long lo[4]; long pre[5]; int nr; };
struct AdamFlips { bf16_t* wf[4]; long off[4]; int n[4], Cout[4], KS[4], Cin[4]; int nf; };
__global__ __launch_bounds__(256) void adam_multi_k(float* __restrict__ p, float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16_t* __restrict__ pbf, AdamRanges R, AdamFlips F, float lr_t,
                                                    float b1, float b2, float eps, float gscale,
                                                    const float* __restrict__ lr_dev, int clear) {
  if (lr_dev) lr_t = lr_dev[1];
  const long tot = R.pre[R.nr];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    int r = 0;
    while (r + 1 < R.nr && i >= R.pre[r + 1]) ++r;
    const long e = R.lo[r] + 4 * (i - R.pre[r]);  // first element of this float4
    const long q = e >> 2;
    float4 pp = ((float4*)p)[q];
    const float4 gg = ((const float4*)g)[q];
    if (clear) ((float4*)g)[q] = float4{0.f, 0.f, 0.f, 0.f};
    float4 mm = ((float4*)m)[q], vv = ((float4*)v)[q];
    float* P = &pp.x; const float* G = &gg.x; float* Mm = &mm.x; float* V = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = G[j] * gscale;
      Mm[j] = b1 * Mm[j] + (1.f - b1) * gj;
      V[j] = b2 * V[j] + (1.f - b2) * gj * gj;
      P[j] -= lr_t * Mm[j] / (sqrtf(V[j]) + eps);
    }
    ((float4*)p)[q] = pp; ((float4*)m)[q] = mm; ((float4*)v)[q] = vv;
    if (pbf) {
      U2 o; o.x = pack_bf(pp.x, pp.y); o.y = pack_bf(pp.z, pp.w);
      ((U2*)pbf)[q] = o;
    }
    for (int j = 0; j < F.nf; ++j) {
      const long d0 = e - F.off[j];
      if (d0 < 0 || d0 >= F.n[j]) continue;
      const int Cin = F.Cin[j], KS = F.KS[j], Cout = F.Cout[j];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int d = (int)d0 + t;
        const int ci = d % Cin;
        int rest = d / Cin;
        const int kw = rest % KS;
        rest /= KS;
        const int kh = rest % KS, co = rest / KS;
        F.wf[j][((ci * KS + (KS - 1 - kh)) * KS + (KS - 1 - kw)) * Cout + co] = f2bf(P[t]);
      }
    }
  }
}

// Fused flat SGD (+momentum, optional Nesterov), Keras convention:
//   v = momentum*v - lr*g ; p += v            (nesterov: p += momentum*v - lr*g)
__global__ __launch_bounds__(256) void sgd_k(float* __restrict__ p, float* __restrict__ g,
                                             float* __restrict__ vel, bf16_t* __restrict__ pbf, long n4, float lr,
                                             float momentum, int nesterov, float gscale, int clear) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 pp = ((float4*)p)[i];
    const float4 gg = ((const float4*)g)[i];
    if (clear) ((float4*)g)[i] = float4{0.f, 0.f, 0.f, 0.f};
    float4 vv = vel ? ((float4*)vel)[i] : float4{0.f, 0.f, 0.f, 0.f};
    float* P = &pp.x; const float* G = &gg.x; float* V = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = G[j] * gscale;
      V[j] = momentum * V[j] - lr * gj;
      P[j] += nesterov ? momentum * V[j] - lr * gj : V[j];
    }
    ((float4*)p)[i] = pp;
    if (vel) ((float4*)vel)[i] = vv;
    if (pbf) {
      U2 o; o.x = pack_bf(pp.x, pp.y); o.y = pack_bf(pp.z, pp.w);
      ((U2*)pbf)[i] = o;
    }
  }
}

__global__ __launch_bounds__(256) void cast_f32_bf16_k(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                       long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = f2bf(x[i]);
}
// Bilinear resize (tf.image.resize: half-pixel centres, no antialias) of uint8 NHWC (3 ch) images,
// scaled by 1/255, written as 4-channel NHWC bf16 (4th channel 0 = MFMA-friendly padding).
__global__ __launch_bounds__(256) void resize_norm_k(const uint8_t* __restrict__ in, bf16_t* __restrict__ out,
                                                     int N, int Hin, int Win, int H, int W) {
  const long total = (long)N * H * W;
  const float sy = (float)Hin / H, sx = (float)Win / W;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int x = i % W; long t = i / W; const int y = t % H; const int n = t / H;
    float fy = (y + 0.5f) * sy - 0.5f, fx = (x + 0.5f) * sx - 0.5f;
    fy = fmaxf(fy, 0.f); fx = fmaxf(fx, 0.f);
    int y0 = min((int)fy, Hin - 1), x0 = min((int)fx, Win - 1);
    const int y1 = min(y0 + 1, Hin - 1), x1 = min(x0 + 1, Win - 1);
    const float wy = fy - y0, wx = fx - x0;
    const uint8_t* b = in + (long)n * Hin * Win * 3;
    float o[4];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v00 = b[((long)y0 * Win + x0) * 3 + c], v01 = b[((long)y0 * Win + x1) * 3 + c];
      const float v10 = b[((long)y1 * Win + x0) * 3 + c], v11 = b[((long)y1 * Win + x1) * 3 + c];
      const float top = v00 + (v01 - v00) * wx, bot = v10 + (v11 - v10) * wx;
      o[c] = (top + (bot - top) * wy) * (1.f / 255.f);
    }
    o[3] = 0.f;
    U2 r; r.x = pack_bf(o[0], o[1]); r.y = pack_bf(o[2], o[3]);
    *(U2*)(out + i * 4) = r;
  }
}

// Same-size uint8 images [N][H][W][3] -> bf16 [N][H][W][4] / 255 (the decoded-image input pipeline
// when no resize is needed): 4 pixels per thread = three 4-byte loads in, two 16-byte stores out.
__global__ __launch_bounds__(256) void pack_u8rgb4_k(const uint32_t* __restrict__ in, U4* __restrict__ out,
                                                     long nquad) {
  constexpr float s = 1.f / 255.f;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < nquad; q += (long)gridDim.x * 256) {
    const uint32_t a = in[q * 3], b = in[q * 3 + 1], c = in[q * 3 + 2];
    const uint32_t by[12] = {a & 255, (a >> 8) & 255, (a >> 16) & 255, a >> 24,
                             b & 255, (b >> 8) & 255, (b >> 16) & 255, b >> 24,
                             c & 255, (c >> 8) & 255, (c >> 16) & 255, c >> 24};
    U4 o0, o1;
    o0.x = pack_bf(by[0] * s, by[1] * s); o0.y = pack_bf(by[2] * s, 0.f);
    o0.z = pack_bf(by[3] * s, by[4] * s); o0.w = pack_bf(by[5] * s, 0.f);
    o1.x = pack_bf(by[6] * s, by[7] * s); o1.y = pack_bf(by[8] * s, 0.f);
    o1.z = pack_bf(by[9] * s, by[10] * s); o1.w = pack_bf(by[11] * s, 0.f);
    out[q * 2] = o0;
    out[q * 2 + 1] = o1;
  }
}

// float images [N][H][W][3] in [0,1] -> 4-channel bf16
__global__ __launch_bounds__(256) void pack_rgb4_k(const float* __restrict__ in, bf16_t* __restrict__ out,
                                                   long npix) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < npix; i += (long)gridDim.x * 256) {
    U2 r; r.x = pack_bf(in[i * 3], in[i * 3 + 1]); r.y = pack_bf(in[i * 3 + 2], 0.f);
    *(U2*)(out + i * 4) = r;
  }
}

// Global average pool: out[n][c] = mean_hw x[n][hw][c] (fp32 out); backward broadcasts dy/HW.
// Global average pool, NHWC bf16 -> [N][C] fp32.  Block = (sample, pixel chunk); each thread reads
// 8 channels (16 B) of a pixel, rows of the chunk are spread over 256/(C/8) row slots with 4 loads
// in flight, the slots are combined in LDS and the chunk's mean contribution is added (fp32 atomic,
// `out` zeroed by the host) - coalesced 16-B loads instead of one 2-byte load per thread and pixel.
__global__ __launch_bounds__(256) void gap_fwd_k(const bf16_t* __restrict__ x, float* __restrict__ out, int N,
                                                 int HW, int C, int pchunk) {
  __shared__ float red[256 * 8];
  const int n = blockIdx.x, cpt = C >> 3, rpi = 256 / cpt;
  const int tid = threadIdx.x, slot = tid % cpt, rsub = tid / cpt;
  const int p0 = blockIdx.y * pchunk, p1 = min(HW, p0 + pchunk);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (rsub < rpi) {
    const bf16_t* base = x + (long)n * HW * C + slot * 8;
    int p = p0 + rsub;
    for (; p + 3 * rpi < p1; p += 4 * rpi) {
      U4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const U4*)(base + (long)(p + u * rpi) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    }
    for (; p < p1; p += rpi) {
      float f[8];
      unpack8(*(const U4*)(base + (long)p * C), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = s[j];
  __syncthreads();
  const float inv = 1.f / (float)HW;
  for (int c = tid; c < C; c += 256) {
    const int sl = c >> 3, j = c & 7;
    float t = 0.f;
    for (int r = 0; r < rpi; ++r) t += red[(r * cpt + sl) * 8 + j];
    atomicAdd(out + (long)n * C + c, t * inv);
  }
}
__global__ __launch_bounds__(256) void gap_bwd_k(const float* __restrict__ dy, bf16_t* __restrict__ out, int N,
                                                 int HW, int C) {
  const int C8 = C >> 3;
  const long total8 = (long)N * HW * C8;
  const float inv = 1.f / (float)HW;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total8; i += (long)gridDim.x * 256) {
    const int c8 = (int)(i % C8);
    const long n = i / ((long)HW * C8);
    const float4 a = *(const float4*)(dy + n * C + c8 * 8), b = *(const float4*)(dy + n * C + c8 * 8 + 4);
    const float f[8] = {a.x * inv, a.y * inv, a.z * inv, a.w * inv, b.x * inv, b.y * inv, b.z * inv, b.w * inv};
    *(U4*)(out + i * 8) = pack8(f);
  }
}

// ReLU backward: dz = (y > 0) ? dy : 0   (dy fp32 or bf16, y bf16 or fp32, dz bf16 or fp32)
template <typename TD, typename TY, typename TO>
__global__ __launch_bounds__(256) void relu_bwd_k(const TD* __restrict__ dy, const TY* __restrict__ y,
                                                  TO* __restrict__ dz, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float g = ldf(dy, i);
    const float v = ldf(y, i) > 0.f ? g : 0.f;
    if constexpr (sizeof(TO) == 2) dz[i] = f2bf(v); else dz[i] = v;
  }
}

static inline int grid_for(long n, int per = 1) {
  long g = (n / per + 255) / 256;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return (int)g;
}

extern "C" {

int ptg_prelu_pool_fwd(const void* z, const float* alpha, void* p, int N, int H, int W, int C,
                       hipStream_t s) {
  if (C % 8 || H < 2 || W < 2) return (int)hipErrorInvalidValue;
  const long total = (long)N * (H / 2) * (W / 2) * (C / 8);
  hipLaunchKernelGGL(prelu_pool_fwd_k, dim3(grid_for(total)), dim3(256), 0, s, (const bf16_t*)z, alpha,
                     (bf16_t*)p, N, H, W, C);
  PTG_RETURN_LAUNCH();
}

int ptg_prelu_pool_bwd2(const void* dp, const void* z, const float* alpha, void* dz, float* dalpha,
                        float* dbias, int N, int H, int W, int C, int nper, hipStream_t s) {
  if (C % 8 || C > 256 || H < 2 || W < 2 || !ptg_fits_2g((long)N * H * W * C * 2)) return (int)hipErrorInvalidValue;
  const int npos = (H / 2) * (W / 2) * (C / 4);
  const int bx = (npos + 15) / 16;
  if (nper <= 0) {  // >= ~1024 blocks, but at least 64 samples (4 per sample group) per chunk
    int chunks = (1024 + bx - 1) / bx;
    chunks = std::max(1, std::min(chunks, N / 64));
    nper = (N + chunks - 1) / chunks;
  }
  dim3 grid(bx, (N + nper - 1) / nper);
  if (dz)
    hipLaunchKernelGGL(prelu_pool_bwd_sg_k<4>, grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)z, alpha,
                       (bf16_t*)dz, dalpha, dbias, N, H, W, C, nper);
  else  // dalpha / dbias only (dz == nullptr)
    hipLaunchKernelGGL((prelu_pool_bwd_sg_k<4, false>), grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)z,
                       alpha, (bf16_t*)nullptr, dalpha, dbias, N, H, W, C, nper);
  PTG_RETURN_LAUNCH();
}

int ptg_prelu_pool_bwd_sparse(const void* dp, const void* zs, const void* arg, const float* alpha, void* dz,
                              float* dalpha, float* dbias, int N, int H, int W, int C, int nper, hipStream_t s) {
  if (C % 8 || C > 256 || (H & 1) || (W & 1) || H < 2 || W < 2) return (int)hipErrorInvalidValue;
  const int npos = (H / 2) * (W / 2) * (C / 8);
  if (nper <= 0) {
    const int bx = (npos + 255) / 256;
    int chunks = (2048 + bx - 1) / bx;
    if (chunks > N) chunks = N;
    nper = (N + chunks - 1) / chunks;
  }
  dim3 grid((npos + 255) / 256, (N + nper - 1) / nper);
  hipLaunchKernelGGL(prelu_pool_bwd_sparse_k, grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)zs,
                     (const uint8_t*)arg, alpha, (bf16_t*)dz, dalpha, dbias, N, H, W, C, nper);
  PTG_RETURN_LAUNCH();
}

int ptg_prelu_pool_bwd_sel(const void* dp, const void* zs, const void* arg, const float* alpha, void* dzs,
                           float* dalpha, float* dbias, int N, int H, int W, int C, int nper, hipStream_t s) {
  if (C % 8 || C > 256 || (H & 1) || (W & 1) || H < 2 || W < 2) return (int)hipErrorInvalidValue;
  const int npos = (H / 2) * (W / 2) * (C / 8);
  const int bx = (npos + 15) / 16;
  if (nper <= 0) {  // samples per chunk: a block's fixed cost (alpha loads, the dalpha reduction over
    //                 its sample groups, one RMW / atomic per (position, channel, q)) is amortised over
    //                 nper samples, so few chunks - ~400 blocks - beat filling the device
    //                 (tools/sel_bench.py, b256, us by nper: layer 2 64: 101.5, 128: 88.6, 256: 67.1;
    //                 layer 3 64: 59.8, 128: 43.1, 256: 45.9; layer 4 64: 38.6, 128: 31.2, 256: 41.6),
    //                 and >= 64 samples per chunk (the first layer: 173 vs 134 us at 4 chunks of 64)
    int chunks = std::max(1, 400 / bx);
    chunks = std::max(1, std::min(chunks, N / 64));
    nper = (N + chunks - 1) / chunks;
  }
  dim3 grid(bx, (N + nper - 1) / nper);
  hipLaunchKernelGGL(prelu_pool_bwd_sel_k, grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)zs,
                     (const uint8_t*)arg, alpha, (bf16_t*)dzs, dalpha, dbias, N, H, W, C, nper);
  PTG_RETURN_LAUNCH();
}

int ptg_prelu_fwd(const void* z, const float* alpha, void* a, int N, int HWC, hipStream_t s) {
  if (HWC % 8) return (int)hipErrorInvalidValue;
  const long total8 = (long)N * HWC / 8;
  hipLaunchKernelGGL(prelu_fwd_k, dim3(grid_for(total8)), dim3(256), 0, s, (const bf16_t*)z, alpha,
                     (bf16_t*)a, total8, HWC / 8);
  PTG_RETURN_LAUNCH();
}

int ptg_prelu_bwd2(const void* da, const void* z, const float* alpha, void* dz, float* dalpha,
                   float* dbias, int N, int HWC, int C, int nper, hipStream_t s) {
  if (HWC % 8 || C % 8 || C > 256) return (int)hipErrorInvalidValue;
  const int bx = (HWC / 8 + 15) / 16;
  if (nper <= 0) {  // >= ~512 blocks, >= 32 samples per chunk
    int chunks = (512 + bx - 1) / bx;
    chunks = std::max(1, std::min(chunks, N / 32));
    nper = (N + chunks - 1) / chunks;
  }
  dim3 grid(bx, (N + nper - 1) / nper);
  if (dz)
    hipLaunchKernelGGL(prelu_bwd_sg_k<true>, grid, dim3(256), 0, s, (const bf16_t*)da, (const bf16_t*)z, alpha,
                       (bf16_t*)dz, dalpha, dbias, N, HWC, C, nper);
  else  // dalpha / dbias only
    hipLaunchKernelGGL(prelu_bwd_sg_k<false>, grid, dim3(256), 0, s, (const bf16_t*)da, (const bf16_t*)z, alpha,
                       (bf16_t*)nullptr, dalpha, dbias, N, HWC, C, nper);
  PTG_RETURN_LAUNCH();
}

// fused Dense(relu) -> Dense(N2 <= 4, linear) -> MSE head (head_row_k + head_col_k); acc is zeroed
// on exit.  scratch: fp32 [B * (N2 + 2)] (dpred and per-row errors).
int ptg_head_mse(void* acc, const float* b1, const float* w2, const float* b2, const float* tgt, void* dz1,
                 float* dw2, float* db2, float* db1, float* stats, float* pred_out, float* scratch, int B, int K1,
                 int N2, float gscale, int nparts, hipStream_t s) {
  if (N2 < 1 || N2 > 4 || B <= 0 || K1 <= 0 || nparts < 0) return (int)hipErrorInvalidValue;
  float* dpred = scratch;
  float* rowerr = scratch + (long)B * N2;
  const dim3 gc((K1 + 255) / 256, HEAD_RG);
  const bool vec = nparts > 0 && K1 % 4 == 0 && K1 <= 4 * 512;
#define PTG_HEAD(NN)                                                                                          \
  if (vec && nparts <= 8)                                                                                     \
    hipLaunchKernelGGL((head_row_parts_k<NN, 8>), dim3(B), dim3(512), 0, s, (float*)acc, b1, w2, b2, tgt,     \
                       (bf16_t*)dz1, dpred, rowerr, pred_out, B, K1, gscale, nparts);                         \
  else if (vec)                                                                                               \
    hipLaunchKernelGGL((head_row_parts_k<NN, 16>), dim3(B), dim3(512), 0, s, (float*)acc, b1, w2, b2, tgt,    \
                       (bf16_t*)dz1, dpred, rowerr, pred_out, B, K1, gscale, nparts);                         \
  else                                                                                                        \
    hipLaunchKernelGGL(head_row_k<NN>, dim3(B), dim3(256), 0, s, (float*)acc, b1, w2, b2, tgt, (bf16_t*)dz1,     \
                       dpred, rowerr, pred_out, B, K1, gscale, nparts);                                       \
  hipLaunchKernelGGL(head_col_k<NN>, gc, dim3(256), 0, s, (float*)acc, b1, w2, dpred, rowerr, dw2, db2, db1,    \
                     stats, B, K1, nparts)
  switch (N2) {
    case 1: PTG_HEAD(1); break;
    case 2: PTG_HEAD(2); break;
    case 3: PTG_HEAD(3); break;
    default: PTG_HEAD(4); break;
  }
#undef PTG_HEAD
  PTG_RETURN_LAUNCH();
}

// out = act(sum over nparts slices [nparts][M][N] of part + bias[n]) (dense.hip split-K partials);
// N % 4 == 0, 16-B vectors
__global__ __launch_bounds__(256) void bias_act_parts_k(const float4* __restrict__ part, const float* __restrict__ bias,
                                                        uint2* __restrict__ out, float4* __restrict__ out32,
                                                        long total4, int N, int act, int nparts) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total4; i += (long)gridDim.x * 256) {
    float4 v = part[i];
    for (int p = 1; p < nparts; ++p) {
      const float4 u = part[p * total4 + i];
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    if (bias) {  // (a parameter view of the flat store: not necessarily 16-B aligned)
      const float* b = bias + (i * 4) % N;
      v.x += b[0]; v.y += b[1]; v.z += b[2]; v.w += b[3];
    }
    if (act == 1) {
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    }
    if (out) out[i] = make_uint2(pack_bf(v.x, v.y), pack_bf(v.z, v.w));
    if (out32) out32[i] = v;
  }
}

int ptg_bias_act_parts(const float* part, int nparts, const float* bias, void* out_bf16, float* out32, long M, int N,
                       int act, hipStream_t s) {
  if (nparts < 1 || N % 4 || M <= 0) return (int)hipErrorInvalidValue;
  const long total4 = M * N / 4;
  hipLaunchKernelGGL(bias_act_parts_k, dim3(grid_for(total4)), dim3(256), 0, s, (const float4*)part, bias,
                     (uint2*)out_bf16, (float4*)out32, total4, N, act, nparts);
  PTG_RETURN_LAUNCH();
}

int ptg_bias_act(float* acc, const float* bias, void* out_bf16, float* out32, long M, int N, int act, int clear,
                 hipStream_t s) {
  const long total = M * N;
  hipLaunchKernelGGL(bias_act_k, dim3(grid_for(total)), dim3(256), 0, s, acc, bias, (bf16_t*)out_bf16, out32,
                     total, N, act, clear);
  PTG_RETURN_LAUNCH();
}

int ptg_col_sum(const void* g, int g_is_bf16, float* db, int M, int N, hipStream_t s) {
  const int bx = (N + 255) / 256;
  int chunks = (512 + bx - 1) / bx;
  if (chunks > M) chunks = M;
  if (chunks < 1) chunks = 1;
  const int mper = (M + chunks - 1) / chunks;
  dim3 grid(bx, (M + mper - 1) / mper);
  if (g_is_bf16)
    hipLaunchKernelGGL(col_sum_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)g, db, M, N, mper);
  else
    hipLaunchKernelGGL(col_sum_k<float>, grid, dim3(256), 0, s, (const float*)g, db, M, N, mper);
  PTG_RETURN_LAUNCH();
}

int ptg_dense_small_fwd(const void* x, int x_is_bf16, const float* w, const float* b, float* y, void* ybf,
                        int M, int K, int N, int act, hipStream_t s) {
  if (N > 64) return (int)hipErrorInvalidValue;
  if (K <= 64 && act != 2 && M >= 256) {
    const dim3 g(ptg_ceil_div((long)M * N, 256));
    if (x_is_bf16)
      hipLaunchKernelGGL(dense_small_fwd_t_k<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, w, b, y, (bf16_t*)ybf, M,
                         K, N, act);
    else
      hipLaunchKernelGGL(dense_small_fwd_t_k<float>, g, dim3(256), 0, s, (const float*)x, w, b, y, (bf16_t*)ybf, M,
                         K, N, act);
    PTG_RETURN_LAUNCH();
  }
  dim3 grid((M + 3) / 4);
  if (x_is_bf16)
    hipLaunchKernelGGL(dense_small_fwd_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, w, b, y,
                       (bf16_t*)ybf, M, K, N, act);
  else
    hipLaunchKernelGGL(dense_small_fwd_k<float>, grid, dim3(256), 0, s, (const float*)x, w, b, y,
                       (bf16_t*)ybf, M, K, N, act);
  PTG_RETURN_LAUNCH();
}

// mask_kind: 0 none, 1 f32 mask, 2 bf16 mask. out_is_bf16 selects dx dtype.
int ptg_dense_small_dx(const float* dy, const float* w, const void* mask, int mask_kind, void* dx,
                       int out_is_bf16, int M, int K, int N, hipStream_t s) {
  const long total = (long)M * K;
  dim3 grid((total + 255) / 256);
  if (mask_kind == 2) {
    if (out_is_bf16)
      hipLaunchKernelGGL((dense_small_dx_k<bf16_t, bf16_t>), grid, dim3(256), 0, s, dy, w,
                         (const bf16_t*)mask, (bf16_t*)dx, M, K, N);
    else
      hipLaunchKernelGGL((dense_small_dx_k<bf16_t, float>), grid, dim3(256), 0, s, dy, w,
                         (const bf16_t*)mask, (float*)dx, M, K, N);
  } else {
    const float* mk = mask_kind == 1 ? (const float*)mask : nullptr;
    if (out_is_bf16)
      hipLaunchKernelGGL((dense_small_dx_k<float, bf16_t>), grid, dim3(256), 0, s, dy, w, mk, (bf16_t*)dx,
                         M, K, N);
    else
      hipLaunchKernelGGL((dense_small_dx_k<float, float>), grid, dim3(256), 0, s, dy, w, mk, (float*)dx, M,
                         K, N);
  }
  PTG_RETURN_LAUNCH();
}

int ptg_dense_small_dw(const float* dy, const void* x, int x_is_bf16, float* dw, float* db, int M, int K,
                       int N, hipStream_t s) {
  long total = (long)N * K;
  if (total < N) total = N;
  const int bx = (int)((total + 255) / 256);
  // split the rows so the grid has >= ~512 blocks, each slice >= 64 rows
  int slices = 1;
  while (bx * slices < 512 && M / (slices * 2) >= 64) slices *= 2;
  const int rps = ptg_ceil_div(M, slices);
  dim3 grid(bx, slices);
  if (x_is_bf16)
    hipLaunchKernelGGL(dense_small_dw_k<bf16_t>, grid, dim3(256), 0, s, dy, (const bf16_t*)x, dw, db, M, K, N, rps);
  else
    hipLaunchKernelGGL(dense_small_dw_k<float>, grid, dim3(256), 0, s, dy, (const float*)x, dw, db, M, K, N, rps);
  PTG_RETURN_LAUNCH();
}

int ptg_mse(const float* pred, const float* y, float* dpred, float* stats, int B, int D, float gscale,
            hipStream_t s) {
  hipLaunchKernelGGL(mse_k, dim3(1), dim3(256), 0, s, pred, y, dpred, stats, B * D, B, gscale);
  PTG_RETURN_LAUNCH();
}

int ptg_softmax_xent(const float* logits, const int* labels, float* dlogits, float* stats, int B, int C,
                     float gscale, hipStream_t s) {
  const int g = ptg_ceil_div(B, 16) < 256 ? ptg_ceil_div(B, 16) : 256;  // ~4 rows per wave, <= 256 workgroups
  hipLaunchKernelGGL(softmax_xent_k, dim3(g > 0 ? g : 1), dim3(256), 0, s, logits, labels, dlogits, stats, B, C,
                     gscale);
  PTG_RETURN_LAUNCH();
}

int ptg_adam(float* p, float* g, float* m, float* v, void* pbf, long n, float lr_t, float b1, float b2,
             float eps, float gscale, const float* lr_dev, int clear, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  const long n4 = n / 4;
  hipLaunchKernelGGL(adam_k, dim3(grid_for(n4)), dim3(256), 0, s, p, g, m, v, (bf16_t*)pbf, n4, lr_t, b1, b2,
                     eps, gscale, lr_dev, clear);
  PTG_RETURN_LAUNCH();
}

// ranges: nr (<= 4) pairs (lo, hi) of element offsets from p (multiples of 4, disjoint); flips: nf
// (<= 4) records (wf pointer, element offset of the conv kernel from p, Cout, KS, Cin), each kernel
// wholly inside one range.
int ptg_adam_multi(float* p, float* g, float* m, float* v, void* pbf, int nr, const long* ranges, float lr_t,
                   float b1, float b2, float eps, float gscale, const float* lr_dev, int clear, int nf,
                   const long* flips, hipStream_t s) {
  if (nr < 1 || nr > 4 || nf < 0 || nf > 4) return (int)hipErrorInvalidValue;
  AdamRanges R{};
  R.nr = nr;
  R.pre[0] = 0;
  for (int r = 0; r < nr; ++r) {
    const long lo = ranges[2 * r], hi = ranges[2 * r + 1];
    if (lo < 0 || hi < lo || lo % 4 || hi % 4) return (int)hipErrorInvalidValue;
    R.lo[r] = lo;
    R.pre[r + 1] = R.pre[r] + (hi - lo) / 4;
  }
  AdamFlips F{};
  F.nf = nf;
  for (int j = 0; j < nf; ++j) {
    const long* f = flips + 5 * j;
    F.wf[j] = (bf16_t*)f[0];
    F.off[j] = f[1]; F.Cout[j] = (int)f[2]; F.KS[j] = (int)f[3]; F.Cin[j] = (int)f[4];
    const long n = f[2] * f[3] * f[3] * f[4];
    if (!F.wf[j] || F.off[j] % 4 || n % 4 || n >= (1L << 31)) return (int)hipErrorInvalidValue;
    F.n[j] = (int)n;
    bool inside = false;
    for (int r = 0; r < nr; ++r) inside |= F.off[j] >= ranges[2 * r] && F.off[j] + n <= ranges[2 * r + 1];
    if (!inside) return (int)hipErrorInvalidValue;
  }
  if (R.pre[nr] == 0) return 0;
  hipLaunchKernelGGL(adam_multi_k, dim3(grid_for(R.pre[nr])), dim3(256), 0, s, p, g, m, v, (bf16_t*)pbf, R, F, lr_t,
                     b1, b2, eps, gscale, lr_dev, clear);
  PTG_RETURN_LAUNCH();
}

int ptg_adam_step(float* st, float lr, float b1, float b2, hipStream_t s) {
  hipLaunchKernelGGL(adam_step_k, dim3(1), dim3(64), 0, s, st, lr, b1, b2);
  PTG_RETURN_LAUNCH();
}

int ptg_sgd(float* p, float* g, float* vel, void* pbf, long n, float lr, float momentum, int nesterov,
            float gscale, int clear, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  const long n4 = n / 4;
  hipLaunchKernelGGL(sgd_k, dim3(grid_for(n4)), dim3(256), 0, s, p, g, vel, (bf16_t*)pbf, n4, lr, momentum,
                     nesterov, gscale, clear);
  PTG_RETURN_LAUNCH();
}

// p[0 .. nwords) = value (32-bit words): the runtime's buffer fills (zeroed workspaces, optimizer
// state, gradient buffers) without a framework fill kernel
__global__ __launch_bounds__(256) void fill_u32_k(uint32_t* __restrict__ p, long n4, long nwords, uint32_t value) {
  const U4 v = U4{value, value, value, value};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) *(U4*)(p + 4 * i) = v;
  const long tail = nwords - 4 * n4;  // < 4 words
  if (blockIdx.x == 0 && threadIdx.x < tail) p[4 * n4 + threadIdx.x] = value;
}

int ptg_fill_u32(void* p, long nwords, unsigned int value, hipStream_t s) {
  if (nwords <= 0) return 0;
  if (((uintptr_t)p & 15) != 0) return (int)hipErrorInvalidValue;
  const long n4 = nwords / 4;
  hipLaunchKernelGGL(fill_u32_k, dim3(grid_for(n4 > 0 ? n4 : 1)), dim3(256), 0, s, (uint32_t*)p, n4, nwords, value);
  PTG_RETURN_LAUNCH();
}

int ptg_cast_f32_bf16(const float* x, void* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_k, dim3(grid_for(n)), dim3(256), 0, s, x, (bf16_t*)y, n);
  PTG_RETURN_LAUNCH();
}
int ptg_resize_norm(const void* in_u8, void* out, int N, int Hin, int Win, int H, int W, hipStream_t s) {
  hipLaunchKernelGGL(resize_norm_k, dim3(grid_for((long)N * H * W)), dim3(256), 0, s, (const uint8_t*)in_u8,
                     (bf16_t*)out, N, Hin, Win, H, W);
  PTG_RETURN_LAUNCH();
}
int ptg_pack_u8rgb4(const void* in_u8, void* out, long npix, hipStream_t s) {
  if (npix % 4 || ((uintptr_t)in_u8 & 3) || ((uintptr_t)out & 15)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_u8rgb4_k, dim3(grid_for(npix / 4)), dim3(256), 0, s, (const uint32_t*)in_u8, (U4*)out,
                     npix / 4);
  PTG_RETURN_LAUNCH();
}
int ptg_pack_rgb4(const float* in, void* out, long npix, hipStream_t s) {
  hipLaunchKernelGGL(pack_rgb4_k, dim3(grid_for(npix)), dim3(256), 0, s, in, (bf16_t*)out, npix);
  PTG_RETURN_LAUNCH();
}

// flags: bit0 dy is bf16, bit1 y is bf16, bit2 dz is bf16
int ptg_relu_bwd(const void* dy, const void* y, void* dz, long n, int flags, hipStream_t s) {
  dim3 g(grid_for(n)), b(256);
#define PTG_RB(A, B, C) hipLaunchKernelGGL((relu_bwd_k<A, B, C>), g, b, 0, s, (const A*)dy, (const B*)y, (C*)dz, n)
  switch (flags & 7) {
    case 0: PTG_RB(float, float, float); break;
    case 1: PTG_RB(bf16_t, float, float); break;
    case 2: PTG_RB(float, bf16_t, float); break;
    case 3: PTG_RB(bf16_t, bf16_t, float); break;
    case 4: PTG_RB(float, float, bf16_t); break;
    case 5: PTG_RB(bf16_t, float, bf16_t); break;
    case 6: PTG_RB(float, bf16_t, bf16_t); break;
    default: PTG_RB(bf16_t, bf16_t, bf16_t); break;
  }
#undef PTG_RB
  PTG_RETURN_LAUNCH();
}

int ptg_gap_fwd(const void* x, float* out, int N, int HW, int C, hipStream_t s) {
  if (C % 8 || C > 2048 || N <= 0 || HW <= 0) return (int)hipErrorInvalidValue;
  // ~2048 workgroups over (sample, pixel chunk), at least 64 pixels per chunk
  int chunks = std::max(1, std::min((2048 + N - 1) / N, (HW + 63) / 64));
  const int pchunk = (HW + chunks - 1) / chunks;
  chunks = (HW + pchunk - 1) / pchunk;
  hipError_t e = hipMemsetAsync(out, 0, (size_t)N * C * sizeof(float), s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(gap_fwd_k, dim3(N, chunks), dim3(256), 0, s, (const bf16_t*)x, out, N, HW, C, pchunk);
  PTG_RETURN_LAUNCH();
}
int ptg_gap_bwd(const float* dy, void* out, int N, int HW, int C, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gap_bwd_k, dim3(grid_for((long)N * HW * C / 8)), dim3(256), 0, s, dy, (bf16_t*)out, N, HW, C);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"

PTG_CHECK_STATUS(nn_eltwise)

// ----------------------------------------------------------------------------------------------
// Streaming metric update in ONE launch (nn/metrics.py): state f64[2] = (total, count) += (the
// batch's sum, `count`).  kind 0 Mean(values), 1 MeanAbsoluteError, 2 MeanSquaredError (yp - yt
// elementwise, n elements), 3 SparseCategoricalAccuracy (yp [n][C] scores, yt [n] labels).  The
// Keras metric objects of the reference's custom loops (train_tf_ps.py:608-609,627-628) update every
// step; as torch ops each update was 4-7 small launches.  Types: 0 f32, 1 f64, 2 bf16, 3 i32, 4 i64.
// ----------------------------------------------------------------------------------------------
PTG_DEV double metric_ld(const void* p, int t, long i) {
  switch (t) {
    case 0: return (double)((const float*)p)[i];
    case 1: return ((const double*)p)[i];
    case 2: return (double)bf2f(((const bf16_t*)p)[i]);
    case 3: return (double)((const int*)p)[i];
    default: return (double)((const long long*)p)[i];
  }
}

__global__ __launch_bounds__(256) void metric_update_k(int kind, const void* __restrict__ yp, int tp,
                                                       const void* __restrict__ yt, int tt, long n, int C,
                                                       double count, double* __restrict__ state) {
  __shared__ double red[4];
  double s = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    if (kind == 0) {
      s += metric_ld(yp, tp, i);
    } else if (kind == 3) {
      double best = metric_ld(yp, tp, i * C);
      int am = 0;
      for (int c = 1; c < C; ++c) {
        const double v = metric_ld(yp, tp, i * C + c);
        if (v > best) { best = v; am = c; }
      }
      s += (long long)metric_ld(yt, tt, i) == (long long)am ? 1.0 : 0.0;
    } else {
      const double d = metric_ld(yp, tp, i) - metric_ld(yt, tt, i);
      s += kind == 1 ? fabs(d) : d * d;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = red[0] + red[1] + red[2] + red[3];
    if (gridDim.x == 1) {
      state[0] += t;
      state[1] += count;
    } else {
      atomicAdd(state, t);
      if (blockIdx.x == 0) atomicAdd(state + 1, count);
    }
  }
}

extern "C" {
int ptg_metric_update(int kind, const void* yp, int tp, const void* yt, int tt, long n, int C, double count,
                      void* state, hipStream_t s) {
  if (kind < 0 || kind > 3 || (kind == 3 && C < 1) || n < 0) return (int)hipErrorInvalidValue;
  long work = kind == 3 ? n * (long)C : n;
  int g = (int)((work + 8191) / 8192);
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  hipLaunchKernelGGL(metric_update_k, dim3(g), dim3(256), 0, s, kind, yp, tp, yt, tt, n, C, count, (double*)state);
  return (int)hipGetLastError();
}
}  // extern "C"
