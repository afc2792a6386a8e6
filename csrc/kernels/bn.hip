// BatchNormalization (training batch statistics and inference moving statistics), the
// MaxPooling2D k x k / stride s / zero-padding pair of ResNet's stem, and bf16 tensor add.
//
// Keras ResNet-50 (BASELINE.json "raw-tf ResNet-50 MultiWorkerMirroredStrategy") is a chain of
// Conv2D -> BatchNormalization -> ReLU blocks with a residual Add before the last ReLU of each
// bottleneck.  The conv itself is an MFMA GEMM (gemm.hip); everything here is bandwidth-bound and
// written for HBM3E: 16-byte bf16x8 vectors, per-channel coefficients computed ONCE by a tiny
// finalize kernel so the big passes are a single FMA per element, and batch statistics reduced
// block-locally (LDS) before a few spread-out fp32 atomics ([BN_G groups][C] partial sums) so no
// channel address sees more than ~M/(rows_per_block * BN_G) atomics.
//
//   bn_stats_k        part[g][0|1][c] += sum z, sum z^2      (z = conv output, [M][C] bf16)
//   bn_finalize_k     mean/var (or moving stats) -> scale = gamma*rstd, shift = beta - mean*scale;
//                     moving-average update (Keras momentum convention, biased batch variance)
//   bn_apply_k        y = act(z*scale + shift (+ residual))                      (bf16 out)
//   bn_bwd_reduce_k   part[g][0|1][c] += sum g, sum g*z with g = dy * relu'(y)
//   bn_bwd_finalize_k dgamma, dbeta (+= into the fp32 gradient buffer) and the per-channel affine
//                     form dz = a*g + c1*z + c0 of the BN input gradient
//   bn_bwd_apply_k    dz (bf16) and, for a fused residual Add, d(residual) = g
//   maxpool_fwd_k     out = max over the k x k window of the zero-padded input; stores the argmax
//                     window position (uint8) for the backward
//   maxpool_bwd_k     gather form (each input pixel sums the dy of the <= ceil(k/s)^2 windows
//                     whose argmax it is): deterministic, no atomics
//   add_bf16_k        out = a + b
#include "common.h"

namespace {

constexpr int BN_G = 64;

// Channel slices: a workgroup reduces BN_CS channels (8 threads x 8 channels) over 32 rows at a time,
// and grid.y walks the C / BN_CS slices.  With whole-C rows per workgroup, the C = 1024 / 2048 layers
// (a few thousand rows) ran ~100-400 workgroups of 1 row per pass: too few bytes in flight for HBM
// (0.7-2 TB/s measured).  Rows per workgroup: ~1024 workgroups in total, at least 8 rows per thread
// so the 2*BN_CS partial-sum atomics a workgroup flushes stay small next to the bytes it reads.
constexpr int BN_CS = 64;
inline int bn_slice(int C) { return (C <= BN_CS || C % BN_CS) ? C : BN_CS; }
inline int bn_rows_per_block(long M, int rpi, int slices) {
  long per_thread = (M * slices + 1024L * rpi - 1) / (1024L * rpi);
  if (per_thread < 8) per_thread = 8;
  return (int)(per_thread * rpi);
}

// Shared LDS reduction of per-thread [8] partials over the `rpi` row slots of each channel slot,
// then one atomic per (channel, array) into the block's partial group.
PTG_DEV void bn_flush(float (*red)[256][8], const float* s, const float* q, int tid, int cpt, int rpi,
                      float* part, int C, int cbase) {
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][tid][j] = s[j]; red[1][tid][j] = q[j]; }
  __syncthreads();
  if (tid < cpt) {
    float as[8], aq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { as[j] = 0.f; aq[j] = 0.f; }
    for (int r = 0; r < rpi; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { as[j] += red[0][r * cpt + tid][j]; aq[j] += red[1][r * cpt + tid][j]; }
    }
    float* p = part + (long)(blockIdx.x % BN_G) * 2 * C + cbase;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(p + tid * 8 + j, as[j]);
      atomicAdd(p + C + tid * 8 + j, aq[j]);
    }
  }
}

// Totals over the BN_G partial groups of channel c, read and re-zeroed (the buffer is reused).  All
// 2*BN_G loads are issued before any store: the finalize kernels are one or a few workgroups, so
// their time is the number of dependent memory round trips (stores interleaved with the loads
// serialised every load (possible aliasing); 8 batches of 8 groups still measured ~9 us per launch,
// 106 launches per ResNet-50 step).
PTG_DEV void bn_part_sums(float* part, int C, int c, double& s, double& q) {
  s = 0.0; q = 0.0;
  float a[BN_G], b[BN_G];
#pragma unroll
  for (int g = 0; g < BN_G; ++g) {
    const float* p = part + (long)g * 2 * C;
    a[g] = p[c];
    b[g] = p[C + c];
  }
#pragma unroll
  for (int g = 0; g < BN_G; ++g) { s += a[g]; q += b[g]; }
#pragma unroll
  for (int g = 0; g < BN_G; ++g) {
    float* p = part + (long)g * 2 * C;
    p[c] = 0.f; p[C + c] = 0.f;
  }
}

// ReLU masks as bits (residual BNs): bit j of byte i = (y[8i + j] > 0), written by bn_apply_k from
// the stored bf16 outputs, so the backward passes read 1 bit instead of the 16-bit y per element.
// relu mode 3 of the backward kernels: the mask byte expands to a bf16x8 vector of 1.0 / 0.0 that
// takes y's place in the mode-1 code path.
PTG_DEV unsigned relu_bits(const U4& y) {
  const uint32_t w[4] = {y.x, y.y, y.z, y.w};
  unsigned b = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t lo = w[k] & 0xFFFFu, hi = w[k] >> 16;
    b |= (unsigned)(lo != 0u && lo <= 0x7F80u) << (2 * k);  // > 0: positive, nonzero (+inf included)
    b |= (unsigned)(hi != 0u && hi <= 0x7F80u) << (2 * k + 1);
  }
  return b;
}
PTG_DEV U4 mask_u4(unsigned b) {
  U4 v;
  v.x = ((b & 1u) ? 0x3F80u : 0u) | ((b & 2u) ? 0x3F800000u : 0u);
  v.y = ((b & 4u) ? 0x3F80u : 0u) | ((b & 8u) ? 0x3F800000u : 0u);
  v.z = ((b & 16u) ? 0x3F80u : 0u) | ((b & 32u) ? 0x3F800000u : 0u);
  v.w = ((b & 64u) ? 0x3F80u : 0u) | ((b & 128u) ? 0x3F800000u : 0u);
  return v;
}

}  // namespace

__global__ __launch_bounds__(256) void bn_stats_k(const bf16_t* __restrict__ z, long M, int C, int rpb, int cs,
                                                  float* __restrict__ part) {
  __shared__ float red[2][256][8];
  const int tid = threadIdx.x, cpt = cs >> 3, rpi = 256 / cpt, cbase = blockIdx.y * cs;
  const int slot = tid % cpt, rsub = tid / cpt;
  z += cbase;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
  const long r0 = (long)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  if (rsub < rpi) {
    long r = r0 + rsub;
    for (; r + 3L * rpi < r1; r += 4L * rpi) {  // 4 independent 16-B loads in flight per thread
      U4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const U4*)(z + (r + (long)u * rpi) * C + slot * 8);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] = fmaf(f[j], f[j], q[j]); }
      }
    }
    for (; r < r1; r += rpi) {
      float f[8];
      unpack8(*(const U4*)(z + r * C + slot * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] = fmaf(f[j], f[j], q[j]); }
    }
  }
  bn_flush(red, s, q, tid, cpt, rpi, part, C, cbase);
}

__global__ __launch_bounds__(256) void bn_finalize_k(float* __restrict__ part, int C, long M,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps, float momentum,
                                                     float* __restrict__ mmean, float* __restrict__ mvar,
                                                     float* __restrict__ scale, float* __restrict__ shift,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int training) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  // every per-channel operand is loaded up front, in the same round trip as the partial sums
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const float mm0 = mmean ? mmean[c] : 0.f, mv0 = mmean ? mvar[c] : 0.f;
  float mean, var;
  if (training) {
    double s, q;
    bn_part_sums(part, C, c, s, q);
    const double invM = 1.0 / (double)M;
    const double m = s * invM;
    double v = q * invM - m * m;
    mean = (float)m; var = (float)(v > 0.0 ? v : 0.0);
    if (momentum >= 0.f && mmean) {
      mmean[c] = mm0 * momentum + mean * (1.f - momentum);
      mvar[c] = mv0 * momentum + var * (1.f - momentum);
    }
  } else {
    mean = mm0; var = mv0;
  }
  const float rstd = rsqrtf(var + eps);
  const float sc = gm * rstd;
  scale[c] = sc;
  shift[c] = bt - mean * sc;
  if (mean_out) { mean_out[c] = mean; rstd_out[c] = rstd; }
}

__global__ __launch_bounds__(256) void bn_apply_k(const bf16_t* __restrict__ z, const float* __restrict__ scale,
                                                  const float* __restrict__ shift, const bf16_t* __restrict__ res,
                                                  int relu, bf16_t* __restrict__ y, long n8, int C,
                                                  uint8_t* __restrict__ mask) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
    const int c0 = (int)((i * 8) % C);
    float f[8], r[8];
    unpack8(*(const U4*)(z + i * 8), f);
    const float4 s0 = *(const float4*)(scale + c0), s1 = *(const float4*)(scale + c0 + 4);
    const float4 h0 = *(const float4*)(shift + c0), h1 = *(const float4*)(shift + c0 + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    if (res) unpack8(*(const U4*)(res + i * 8), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = fmaf(f[j], sc[j], sh[j]);
      if (res) v += r[j];
      f[j] = relu ? fmaxf(v, 0.f) : v;
    }
    const U4 yv = pack8(f);
    *(U4*)(y + i * 8) = yv;
    if (mask) mask[i] = (uint8_t)relu_bits(yv);
  }
}

// relu: 0 = none, 1 = ReLU mask from the stored output y, 2 = mask recomputed from z as
// fmaf(z, scale, shift) > 0 - exactly the forward's pre-activation when no residual was added, so
// the y tensor is not read at all (a third less traffic for those BatchNormalizations); 3 = mask
// from the bit mask bn_apply_k wrote (residual BNs: 1 bit instead of 16 per element).
__global__ __launch_bounds__(256) void bn_bwd_reduce_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                       const bf16_t* __restrict__ z, long M, int C, int rpb, int cs,
                                                       int relu, float* __restrict__ part,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       const uint8_t* __restrict__ mask) {
  __shared__ float red[2][256][8];
  const int tid = threadIdx.x, cpt = cs >> 3, rpi = 256 / cpt, cbase = blockIdx.y * cs;
  const int slot = tid % cpt, rsub = tid / cpt;
  dy += cbase;
  z += cbase;
  if (y) y += cbase;
  if (mask) mask += cbase >> 3;
  float s[8], q[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; sc[j] = 0.f; sh[j] = 0.f; }
  if (relu == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = scale[cbase + slot * 8 + j]; sh[j] = shift[cbase + slot * 8 + j]; }
  }
  const long r0 = (long)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  auto acc_row = [&](const U4& vd, const U4& vz, const U4& vy) {
    float g[8], zz[8];
    unpack8(vd, g);
    unpack8(vz, zz);
    if (relu == 1 || relu == 3) {
      float yy[8];
      unpack8(vy, yy);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
    } else if (relu == 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(zz[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] += g[j]; q[j] = fmaf(g[j], zz[j], q[j]); }
  };
  if (rsub < rpi) {
    long r = r0 + rsub;
    for (; r + 3L * rpi < r1; r += 4L * rpi) {  // 8-12 independent 16-B loads in flight per thread
      U4 vd[4], vz[4], vy[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long off = (r + (long)u * rpi) * C + slot * 8;
        vd[u] = *(const U4*)(dy + off);
        vz[u] = *(const U4*)(z + off);
        vy[u] = relu == 1 ? *(const U4*)(y + off) : relu == 3 ? mask_u4(mask[off >> 3]) : vd[u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc_row(vd[u], vz[u], vy[u]);
    }
    for (; r < r1; r += rpi) {
      const long off = r * C + slot * 8;
      const U4 vd = *(const U4*)(dy + off);
      acc_row(vd, *(const U4*)(z + off),
              relu == 1 ? *(const U4*)(y + off) : relu == 3 ? mask_u4(mask[off >> 3]) : vd);
    }
  }
  bn_flush(red, s, q, tid, cpt, rpi, part, C, cbase);
}

// dz = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) = a*g + c1*z + c0.
// The preceding conv's bias gradient, sum(dz) = a*dbeta + M*(c1*mean + c0), is identically zero.
__global__ __launch_bounds__(256) void bn_bwd_finalize_k(float* __restrict__ part, int C, long M,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                         float* __restrict__ coef) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float m = mean[c], rs = rstd[c], gm = gamma ? gamma[c] : 1.f;  // loaded with the partials
  const float dg0 = dgamma ? dgamma[c] : 0.f, db0 = dbeta ? dbeta[c] : 0.f;
  double sg, sgz;
  bn_part_sums(part, C, c, sg, sgz);
  const float db = (float)sg;
  const float dg = (float)((sgz - (double)m * sg) * rs);
  if (dgamma) dgamma[c] = dg0 + dg;
  if (dbeta) dbeta[c] = db0 + db;
  const float a = gm * rs;
  const float invM = 1.f / (float)M;
  const float c1 = -a * dg * rs * invM;
  const float c0 = -a * db * invM - c1 * m;
  coef[c] = a; coef[C + c] = c1; coef[2 * C + c] = c0;
}

PTG_DEV void load8f(const float* p, float* f) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

__global__ __launch_bounds__(256) void bn_bwd_apply_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                      const bf16_t* __restrict__ z, const float* __restrict__ coef,
                                                      int relu, bf16_t* __restrict__ dz, bf16_t* __restrict__ dres,
                                                      long n8, int C, const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      const uint8_t* __restrict__ mask) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
    const int c0 = (int)((i * 8) % C);
    const U4 vd = *(const U4*)(dy + i * 8), vz = *(const U4*)(z + i * 8);
    const U4 vy = relu == 1 ? *(const U4*)(y + i * 8) : relu == 3 ? mask_u4(mask[i]) : vd;
    float g[8], zz[8], a[8], c1[8], c0v[8];
    unpack8(vd, g);
    unpack8(vz, zz);
    load8f(coef + c0, a);
    load8f(coef + C + c0, c1);
    load8f(coef + 2 * C + c0, c0v);
    if (relu == 1 || relu == 3) {
      float yy[8];
      unpack8(vy, yy);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
    } else if (relu == 2) {  // mask recomputed from z (see bn_bwd_reduce_k)
      float sc[8], sh[8];
      load8f(scale + c0, sc);
      load8f(shift + c0, sh);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(zz[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
    }
    if (dres) *(U4*)(dres + i * 8) = pack8(g);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(a[j], g[j], fmaf(c1[j], zz[j], c0v[j]));
    *(U4*)(dz + i * 8) = pack8(o);
  }
}

// -------------------------------------------------------------------------------------------------
// MaxPooling2D(k, stride s) on a zero-padded (pad p each side) NHWC input; C % 8 == 0.
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void maxpool_fwd_k(const bf16_t* __restrict__ x, bf16_t* __restrict__ out,
                                                     uint8_t* __restrict__ arg, int N, int H, int W, int C, int OH,
                                                     int OW, int k, int s, int p) {
  const int cv = C >> 3;
  const long total = (long)N * OH * OW * cv;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c8 = (int)(i % cv);
    long t = i / cv;
    const int ow = (int)(t % OW); t /= OW;
    const int oh = (int)(t % OH);
    const int n = (int)(t / OH);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * s - p + kh;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * s - p + kw;
        float f[8];
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
          unpack8(*(const U4*)(x + (((long)n * H + ih) * W + iw) * C + c8 * 8), f);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = 0.f;  // ZeroPadding2D semantics
        }
        const int pos = kh * k + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > best[j]) { best[j] = f[j]; bi[j] = pos; }
      }
    }
    const long o = (((long)n * OH + oh) * OW + ow) * C + c8 * 8;
    *(U4*)(out + o) = pack8(best);
    if (arg) {
      uint32_t lo = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
      uint32_t hi = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
      *(U2*)(arg + o) = U2{lo, hi};
    }
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_k(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                     bf16_t* __restrict__ dx, int N, int H, int W, int C, int OH,
                                                     int OW, int k, int s, int p, int accum) {
  const int cv = C >> 3;
  const long total = (long)N * H * W * cv;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c8 = (int)(i % cv);
    long t = i / cv;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    int oh_lo = h + p - k + 1; oh_lo = oh_lo <= 0 ? 0 : (oh_lo + s - 1) / s;
    int oh_hi = (h + p) / s; if (oh_hi > OH - 1) oh_hi = OH - 1;
    int ow_lo = w + p - k + 1; ow_lo = ow_lo <= 0 ? 0 : (ow_lo + s - 1) / s;
    int ow_hi = (w + p) / s; if (ow_hi > OW - 1) ow_hi = OW - 1;
    for (int oh = oh_lo; oh <= oh_hi; ++oh)
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int pos = (h + p - oh * s) * k + (w + p - ow * s);
        const long o = (((long)n * OH + oh) * OW + ow) * C + c8 * 8;
        const U2 a = *(const U2*)(arg + o);
        float g[8];
        unpack8(*(const U4*)(dy + o), g);
        const uint8_t* ab = (const uint8_t*)&a;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (ab[j] == pos) acc[j] += g[j];
      }
    const long xo = (((long)n * H + h) * W + w) * C + c8 * 8;
    if (accum) {
      float e[8];
      unpack8(*(const U4*)(dx + xo), e);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += e[j];
    }
    *(U4*)(dx + xo) = pack8(acc);
  }
}

__global__ __launch_bounds__(256) void add_bf16_k(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                  bf16_t* __restrict__ out, long n8) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float fa[8], fb[8];
    unpack8(*(const U4*)(a + i * 8), fa);
    unpack8(*(const U4*)(b + i * 8), fb);
#pragma unroll
    for (int j = 0; j < 8; ++j) fa[j] += fb[j];
    *(U4*)(out + i * 8) = pack8(fa);
  }
}

static inline int ew_grid(long n8) {
  long g = (n8 + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

// part: fp32 [BN_G][2][C], zero on entry (the finalize kernels re-zero it after reading).  C % 8 == 0 and C <= 2048.
int ptg_bn_stats(const void* z, long M, int C, float* part, hipStream_t s) {
  if (C % 8 || C > 2048 || M <= 0) return (int)hipErrorInvalidValue;
  const int cs = bn_slice(C), rpi = 256 / (cs / 8);
  const int rpb = bn_rows_per_block(M, rpi, C / cs);
  hipLaunchKernelGGL(bn_stats_k, dim3(ptg_ceil_div(M, rpb), C / cs), dim3(256), 0, s, (const bf16_t*)z, M, C, rpb,
                     cs, part);
  PTG_RETURN_LAUNCH();
}

int ptg_bn_finalize(float* part, int C, long M, const float* gamma, const float* beta, float eps,
                    float momentum, float* mmean, float* mvar, float* scale, float* shift, float* mean_out,
                    float* rstd_out, int training, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_k, dim3(ptg_ceil_div(C, 256)), dim3(256), 0, s, part, C, M, gamma, beta, eps,
                     momentum, mmean, mvar, scale, shift, mean_out, rstd_out, training);
  PTG_RETURN_LAUNCH();
}

// mask (nullable, u8[M*C/8]): the ReLU bit mask of y for the backward's relu mode 3
int ptg_bn_apply(const void* z, const float* scale, const float* shift, const void* res, int relu, void* y,
                 long M, int C, void* mask, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const long n8 = M * C / 8;
  hipLaunchKernelGGL(bn_apply_k, dim3(ew_grid(n8)), dim3(256), 0, s, (const bf16_t*)z, scale, shift,
                     (const bf16_t*)res, relu, (bf16_t*)y, n8, C, (uint8_t*)mask);
  PTG_RETURN_LAUNCH();
}

int ptg_bn_bwd_reduce(const void* dy, const void* y, const void* z, long M, int C, int relu, float* part,
                      const float* scale, const float* shift, const void* mask, hipStream_t s) {
  if (relu == 2 && (!scale || !shift)) return (int)hipErrorInvalidValue;
  if (relu == 3 && !mask) return (int)hipErrorInvalidValue;
  if (C % 8 || C > 2048 || M <= 0) return (int)hipErrorInvalidValue;
  const int cs = bn_slice(C), rpi = 256 / (cs / 8);
  const int rpb = bn_rows_per_block(M, rpi, C / cs);
  hipLaunchKernelGGL(bn_bwd_reduce_k, dim3(ptg_ceil_div(M, rpb), C / cs), dim3(256), 0, s, (const bf16_t*)dy,
                     (const bf16_t*)y, (const bf16_t*)z, M, C, rpb, cs, relu, part, scale, shift,
                     (const uint8_t*)mask);
  PTG_RETURN_LAUNCH();
}

int ptg_bn_bwd_finalize(float* part, int C, long M, const float* gamma, const float* mean, const float* rstd,
                        float* dgamma, float* dbeta, float* coef, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_k, dim3(ptg_ceil_div(C, 256)), dim3(256), 0, s, part, C, M, gamma, mean, rstd,
                     dgamma, dbeta, coef);
  PTG_RETURN_LAUNCH();
}

int ptg_bn_bwd_apply(const void* dy, const void* y, const void* z, const float* coef, int relu, void* dz, void* dres,
                     long M, int C, const float* scale, const float* shift, const void* mask, hipStream_t s) {
  if (relu == 2 && (!scale || !shift)) return (int)hipErrorInvalidValue;
  if (relu == 3 && !mask) return (int)hipErrorInvalidValue;
  if (C % 8) return (int)hipErrorInvalidValue;
  const long n8 = M * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_k, dim3(ew_grid(n8)), dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)y,
                     (const bf16_t*)z, coef, relu, (bf16_t*)dz, (bf16_t*)dres, n8, C, scale, shift,
                     (const uint8_t*)mask);
  PTG_RETURN_LAUNCH();
}

int ptg_maxpool_fwd(const void* x, void* out, void* arg, int N, int H, int W, int C, int OH, int OW, int k, int st,
                    int p, hipStream_t s) {
  if (C % 8 || k > 15) return (int)hipErrorInvalidValue;
  const long n8 = (long)N * OH * OW * C / 8;
  hipLaunchKernelGGL(maxpool_fwd_k, dim3(ew_grid(n8)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)out,
                     (uint8_t*)arg, N, H, W, C, OH, OW, k, st, p);
  PTG_RETURN_LAUNCH();
}

int ptg_maxpool_bwd(const void* dy, const void* arg, void* dx, int N, int H, int W, int C, int OH, int OW, int k,
                    int st, int p, int accum, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const long n8 = (long)N * H * W * C / 8;
  hipLaunchKernelGGL(maxpool_bwd_k, dim3(ew_grid(n8)), dim3(256), 0, s, (const bf16_t*)dy, (const uint8_t*)arg,
                     (bf16_t*)dx, N, H, W, C, OH, OW, k, st, p, accum);
  PTG_RETURN_LAUNCH();
}

int ptg_add_bf16(const void* a, const void* b, void* out, long n, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(add_bf16_k, dim3(ew_grid(n / 8)), dim3(256), 0, s, (const bf16_t*)a, (const bf16_t*)b,
                     (bf16_t*)out, n / 8);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"

PTG_CHECK_STATUS(bn)
