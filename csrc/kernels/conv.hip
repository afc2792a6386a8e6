// Halo-tiled direct convolution on MFMA (gfx950) — the CNN's hot path.
//
// The generic implicit-GEMM loaders of gemm.hip gather the im2col matrix element-by-element from
// global memory (one global load per 8 k-values per pixel).  With the reference CNN's tiny
// channel counts (Conv2D 3->8->16->32->64->64, 5x5, train_tf_ps.py:351-363) that is load-
// instruction bound.  Here a workgroup owns an output tile of TH x TW pixels and stages the input
// halo tile [TH+KS-1][TW+KWP-1][C] in LDS ONCE; every MFMA A-fragment (16 pixels x 8 k) is then a
// 16-byte LDS read, because for a fixed kernel row kh the K run (kw, ci) of one output pixel is a
// contiguous run of the halo row (ci fastest).  The K dimension is flattened over (kh, kw', ci)
// with kw' padded to KWP so every 8-wide K group stays inside one kernel row.
//
//   conv_fwd_halo_k   fwd (and dgrad, with flipped weights): z = conv(x) + bias, staged through
//                     LDS and written with 16-byte stores; optional fused epilogue
//                     EPI_POOL  -> also writes maxpool2x2(prelu(z, alpha))  (PReLU + MaxPooling2D)
//                     EPI_PRELU -> also writes prelu(z, alpha)                (last conv block)
//   conv_wgrad_halo_k dW[co][kh][kw][ci] = sum_pixels dZ[pix][co] * x[pix + (kh,kw)][ci]:
//                     M = Cout, N = 128-wide slice of (kh,kw,ci), K = pixels; dZ tile and x halo
//                     staged in LDS, both MFMA operands read with ds_read_b64_tr_b16 (gfx950
//                     transposed LDS read, cdna_hip_programming.md T10), partial sums of a whole
//                     chunk of tiles kept in registers, one fp32 atomic per output per workgroup.
//   conv_flip_k       W'[ci][kh][kw][co] = W[co][KS-1-kh][KS-1-kw][ci] (dgrad weights), bf16.
#include "common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

namespace ptgc {

enum { EPI_Z = 0, EPI_POOL = 1, EPI_PRELU = 2 };

template <int C> struct PixPitch { static constexpr int v = C >= 16 ? C + 8 : C; };  // bank-conflict pad
template <int C, int KS> struct Kwp { static constexpr int v = (KS * C) % 8 == 0 ? KS : ((KS + 1) * C) % 8 == 0 ? KS + 1 : KS + 3; };

// ------------------------------------------------------------------------------------------------
// halo staging: rows ih0 .. ih0+HR-1, cols iw0 .. iw0+HC-1, channels C, zero outside the image.
// ------------------------------------------------------------------------------------------------
template <int C, int PIX>
PTG_DEV void stage_halo(bf16_t* __restrict__ hs, const bf16_t* __restrict__ img, int H, int W, int ih0, int iw0,
                        int HR, int HC) {
  if constexpr (C == 4) {
    // 8 bytes per pixel
    const int total = HR * HC;
    for (int t = threadIdx.x; t < total; t += 256) {
      const int r = t / HC, c = t - r * HC;
      const int ih = ih0 + r, iw = iw0 + c;
      U2 v = U2{0u, 0u};
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) v = *(const U2*)(img + ((long)ih * W + iw) * 4);
      *(U2*)(hs + t * 4) = v;
    }
  } else {
    constexpr int V = C / 8;  // 16-byte vectors per pixel
    const int total = HR * HC * V;
    for (int t = threadIdx.x; t < total; t += 256) {
      const int pix = t / V, v = t - pix * V;
      const int r = pix / HC, c = pix - r * HC;
      const int ih = ih0 + r, iw = iw0 + c;
      U4 val = zero4();
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        val = *(const U4*)(img + ((long)ih * W + iw) * C + v * 8);
      *(U4*)(hs + pix * PIX + v * 8) = val;
    }
  }
}

// ================================================================================================
// forward / dgrad
// ================================================================================================
template <int C, int KS, int NF, int TW, int TH, int EPI>
__global__ __launch_bounds__(256) void conv_fwd_halo_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                       const float* __restrict__ bias, const float* __restrict__ alpha,
                                                       bf16_t* __restrict__ z, bf16_t* __restrict__ aux, int H, int W,
                                                       int Cout, int pad, int tiles_h, int tiles_w) {
  constexpr int KWP = Kwp<C, KS>::v;
  constexpr int PIX = PixPitch<C>::v;
  constexpr int HR = TH + KS - 1, HC = TW + KWP - 1;
  constexpr int KROW = KWP * C;         // flattened k per kernel row
  constexpr int KTOT = KS * KROW;
  constexpr int KSTEPS = (KTOT + 31) / 32;
  constexpr int M = TH * TW;
  constexpr int MFR = M / 16;           // 16-pixel fragments per tile
  constexpr int FM = MFR / 4;           // fragments per wave
  static_assert(MFR % 4 == 0, "tile must give 4 waves equal work");
  constexpr int HALO_ELEMS = HR * HC * PIX;
  constexpr int ZPITCH = NF * 16 + 8;   // staged output pixel pitch (bf16), padded
  constexpr int ZELEMS = M * ZPITCH;
  constexpr int LDS_ELEMS = (HALO_ELEMS + 8 > ZELEMS ? HALO_ELEMS + 8 : ZELEMS);
  __shared__ __attribute__((aligned(16))) bf16_t smem[LDS_ELEMS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int t = blockIdx.x;
  const int tw_i = t % tiles_w; t /= tiles_w;
  const int th_i = t % tiles_h; const int n = t / tiles_h;
  const int oh0 = th_i * TH, ow0 = tw_i * TW;
  const bf16_t* img = x + (long)n * H * W * C;

  stage_halo<C, PIX>(smem, img, H, W, oh0 - pad, ow0 - pad, HR, HC);
  // zero guard pixel used by padded K groups (k >= KTOT)
  if (tid < 8) smem[HALO_ELEMS + tid] = 0;
  __syncthreads();

  // per-lane fragment rows (pixels)
  const int frow = lane & 15, g = lane >> 4;
  int pbase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = (wid * FM + i) * 16 + frow;
    const int r = m / TW, c = m % TW;
    pbase[i] = (r * HC + c) * PIX;
  }
  f32x4_t acc[FM][NF];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int co_l = lane & 15;
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int kf = ks * 32 + 8 * g;   // this lane group's first k
    const bool kval = kf < KTOT;
    const int kh = kf / KROW, rem = kf - kh * KROW;
    const int kw = rem / C, ci = rem - kw * C;
    // B fragments (weights, from global / L1): w layout [Cout][KS][KS][C]
    bf16x8_t bf[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int co = j * 16 + co_l;
      U4 v = zero4();
      if (kval && co < Cout) {
        const bf16_t* wp = w + ((long)co * KS * KS + kh * KS) * C;
        if constexpr (C >= 8) {
          if (kw < KS) v = *(const U4*)(wp + kw * C + ci);
        } else {  // C == 4: two pixels (kw, kw+1), pad columns are zero
          U2 a = U2{0u, 0u}, b = U2{0u, 0u};
          if (kw < KS) a = *(const U2*)(wp + kw * 4);
          if (kw + 1 < KS) b = *(const U2*)(wp + (kw + 1) * 4);
          v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
        }
      }
      bf[j] = __builtin_bit_cast(bf16x8_t, v);
    }
    // A fragments from the halo: pixel (r + kh, c + kw), channels ci..ci+7
    const int koff = (kh * HC + kw) * PIX + ci;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      bf16x8_t af;
      if constexpr (C >= 8) {
        const int off = kval ? pbase[i] + koff : HALO_ELEMS;
        af = *(const bf16x8_t*)(smem + off);
      } else {
        const int off = kval ? pbase[i] + koff : HALO_ELEMS;
        U2 lo = *(const U2*)(smem + off);
        U2 hi = kval ? *(const U2*)(smem + off + 4) : U2{0u, 0u};
        U4 v; v.x = lo.x; v.y = lo.y; v.z = hi.x; v.w = hi.y;
        af = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // halo no longer needed: reuse LDS for the output tile

  // epilogue: + bias -> bf16 -> staged [pixel][co] tile
  bf16_t* zs = smem;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int co = j * 16 + co_l;
      const float b = (bias && co < Cout) ? bias[co] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (wid * FM + i) * 16 + g * 4 + r;
        zs[m * ZPITCH + co] = f2bf(acc[i][j][r] + b);
      }
    }
  __syncthreads();
  // z: 16-byte vectors, channels fastest
  const int CV = Cout / 8;
  for (int v = tid; v < M * CV; v += 256) {
    const int m = v / CV, cv = v - m * CV;
    const int oh = oh0 + m / TW, ow = ow0 + m % TW;
    if (oh < H && ow < W)
      *(U4*)(z + (((long)n * H + oh) * W + ow) * Cout + cv * 8) = *(const U4*)(zs + m * ZPITCH + cv * 8);
  }
  if constexpr (EPI == EPI_PRELU) {
    for (int v = tid; v < M * CV; v += 256) {
      const int m = v / CV, cv = v - m * CV;
      const int oh = oh0 + m / TW, ow = ow0 + m % TW;
      if (oh >= H || ow >= W) continue;
      float zf[8];
      unpack8(*(const U4*)(zs + m * ZPITCH + cv * 8), zf);
      const float* al = alpha + ((long)oh * W + ow) * Cout + cv * 8;
      const float4 a0 = *(const float4*)al, a1 = *(const float4*)(al + 4);
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int q = 0; q < 8; ++q) zf[q] = zf[q] > 0.f ? zf[q] : av[q] * zf[q];
      *(U4*)(aux + (((long)n * H + oh) * W + ow) * Cout + cv * 8) = pack8(zf);
    }
  }
  if constexpr (EPI == EPI_POOL) {
    const int PH = H >> 1, PW = W >> 1;
    constexpr int PM = (TH / 2) * (TW / 2);
    for (int v = tid; v < PM * CV; v += 256) {
      const int pm = v / CV, cv = v - pm * CV;
      const int pr = pm / (TW / 2), pc = pm - pr * (TW / 2);
      const int ph = (oh0 >> 1) + pr, pw = (ow0 >> 1) + pc;
      if (ph >= PH || pw >= PW) continue;
      float best[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) best[q] = -INFINITY;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int lr = 2 * pr + (qq >> 1), lc = 2 * pc + (qq & 1);
        float zf[8];
        unpack8(*(const U4*)(zs + (lr * TW + lc) * ZPITCH + cv * 8), zf);
        const float* al = alpha + ((long)(oh0 + lr) * W + (ow0 + lc)) * Cout + cv * 8;
        const float4 a0 = *(const float4*)al, a1 = *(const float4*)(al + 4);
        const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) best[q] = fmaxf(best[q], zf[q] > 0.f ? zf[q] : av[q] * zf[q]);
      }
      *(U4*)(aux + (((long)n * PH + ph) * PW + pw) * Cout + cv * 8) = pack8(best);
    }
  }
}

// ================================================================================================
// weight gradient
// ================================================================================================
// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group supplies the address of row q, 4 columns;
// lane i of the group receives column i of the 4 rows (row q in element q).
PTG_DEV s16x4_t tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p));
}

template <int C, int KS, int TW, int TH, int MF>
__global__ __launch_bounds__(256) void conv_wgrad_halo_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dz,
                                                         float* __restrict__ dw, int N, int H, int W, int Cout, int pad,
                                                         int tiles_h, int tiles_w, int tiles_per_block, int nslices) {
  constexpr int PIX = PixPitch<C>::v;
  constexpr int HR = TH + KS - 1, HC = TW + KS - 1;
  constexpr int M = TH * TW;              // pixels per tile (K of this GEMM)
  static_assert(M % 32 == 0 && TW % 4 == 0, "tile shape");
  constexpr int KF = KS * KS * C;         // output columns (kh, kw, ci)
  constexpr int DPITCH = MF * 16 + 4;     // dz tile pixel pitch (bf16): 8-byte aligned, bank-shifted
  constexpr int HALO_ELEMS = HR * HC * PIX;
  constexpr int DZ_ELEMS = M * DPITCH;
  __shared__ __attribute__((aligned(16))) bf16_t smem[HALO_ELEMS + DZ_ELEMS + 8];
  bf16_t* hs = smem;
  bf16_t* ds = smem + HALO_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int slice = blockIdx.x % nslices;
  const int chunk = blockIdx.x / nslices;
  const int total_tiles = N * tiles_h * tiles_w;
  const int t0 = chunk * tiles_per_block, t1 = min(total_tiles, t0 + tiles_per_block);
  if (t0 >= t1) return;

  // each wave owns 2 of the slice's 8 column fragments (16 kflat each)
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  int bcol[2];   // per-lane column base (kflat) for the B tr-read, or -1 if out of range
  int boff[2];   // halo offset of that kflat for pixel (0,0)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kf = slice * 128 + (wid * 2 + j) * 16 + 4 * p;
    bcol[j] = kf < KF ? kf : -1;
    const int kk = kf < KF ? kf : 0;
    const int kh = kk / (KS * C), rem = kk - kh * KS * C, kw = rem / C, ci = rem - kw * C;
    boff[j] = (kh * HC + kw) * PIX + ci;
  }
  f32x4_t acc[MF][2];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int t = t0; t < t1; ++t) {
    int tt = t;
    const int tw_i = tt % tiles_w; tt /= tiles_w;
    const int th_i = tt % tiles_h; const int n = tt / tiles_h;
    const int oh0 = th_i * TH, ow0 = tw_i * TW;
    __syncthreads();  // previous tile's reads done
    stage_halo<C, PIX>(hs, x + (long)n * H * W * C, H, W, oh0 - pad, ow0 - pad, HR, HC);
    // dz tile [M][Cout] (zero for pixels outside the image)
    {
      const int CV = Cout / 4;  // 8-byte vectors
      for (int v = tid; v < M * CV; v += 256) {
        const int m = v / CV, cv = v - m * CV;
        const int oh = oh0 + m / TW, ow = ow0 + m % TW;
        U2 val = U2{0u, 0u};
        if (oh < H && ow < W) val = *(const U2*)(dz + (((long)n * H + oh) * W + ow) * Cout + cv * 4);
        *(U2*)(ds + m * DPITCH + cv * 4) = val;
      }
    }
    __syncthreads();
    for (int k0 = 0; k0 < M; k0 += 32) {
      // rows of the two tr-reads of this lane group: pixels k0 + 8g + q and k0 + 8g + 4 + q
      const int m0 = k0 + 8 * g + q, m1 = m0 + 4;
      const int r0 = m0 / TW, c0 = m0 % TW, r1 = m1 / TW, c1 = m1 % TW;
      bf16x8_t af[MF];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int co = i * 16 + 4 * p;
        const s16x4_t lo = tr_read(ds + m0 * DPITCH + co);
        const s16x4_t hi = tr_read(ds + m1 * DPITCH + co);
        const U2 a = __builtin_bit_cast(U2, lo), b = __builtin_bit_cast(U2, hi);
        U4 v; v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
        af[i] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o0 = bcol[j] >= 0 ? (r0 * HC + c0) * PIX + boff[j] : HALO_ELEMS + DZ_ELEMS;
        const int o1 = bcol[j] >= 0 ? (r1 * HC + c1) * PIX + boff[j] : HALO_ELEMS + DZ_ELEMS;
        const s16x4_t lo = tr_read(smem + o0);
        const s16x4_t hi = tr_read(smem + o1);
        const U2 a = __builtin_bit_cast(U2, lo), b = __builtin_bit_cast(U2, hi);
        U4 v; v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
        const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
        for (int i = 0; i < MF; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
      }
    }
  }
  // epilogue: rows = co ((lane>>4)*4 + r), cols = kflat (lane & 15)
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kf = slice * 128 + (wid * 2 + j) * 16 + li;
      if (kf >= KF) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = i * 16 + g * 4 + r;
        if (co < Cout) atomicAdd(dw + (long)co * KF + kf, acc[i][j][r]);
      }
    }
}

// W'[ci][kh][kw][co] = W[co][KS-1-kh][KS-1-kw][ci]
__global__ __launch_bounds__(256) void conv_flip_k(const bf16_t* __restrict__ w, bf16_t* __restrict__ wf, int Cout, int KS,
                                                   int Cin) {
  const int total = Cout * KS * KS * Cin;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int co = i % Cout;
    int t = i / Cout;
    const int kw = t % KS; t /= KS;
    const int kh = t % KS; const int ci = t / KS;
    wf[i] = w[(((long)co * KS + (KS - 1 - kh)) * KS + (KS - 1 - kw)) * Cin + ci];
  }
}

// ------------------------------------------------------------------------------------------------
// host dispatch
// ------------------------------------------------------------------------------------------------
template <int C, int KS, int NF, int TW, int TH>
static int launch_fwd(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N,
                      int H, int W, int Cout, int pad, int epi, hipStream_t s) {
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  dim3 grid(N * th * tw);
#define PTG_FWD(E)                                                                                               \
  hipLaunchKernelGGL((conv_fwd_halo_k<C, KS, NF, TW, TH, E>), grid, dim3(256), 0, s, (const bf16_t*)x,          \
                     (const bf16_t*)w, bias, alpha, (bf16_t*)z, (bf16_t*)aux, H, W, Cout, pad, th, tw)
  if (epi == EPI_POOL) PTG_FWD(EPI_POOL);
  else if (epi == EPI_PRELU) PTG_FWD(EPI_PRELU);
  else PTG_FWD(EPI_Z);
#undef PTG_FWD
  PTG_RETURN_LAUNCH();
}

template <int C, int KS, int NF>
static int fwd_by_c(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N,
                    int H, int W, int Cout, int pad, int epi, hipStream_t s) {
  // tile shapes: TH x TW pixels, halo fits LDS, 4 waves with equal fragment counts
  if constexpr (C == 4) return launch_fwd<C, KS, NF, 64, 4>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
  else if constexpr (C == 8) return launch_fwd<C, KS, NF, 32, 8>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
  else if constexpr (C == 16) return launch_fwd<C, KS, NF, 16, 8>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
  else if constexpr (C == 32) return launch_fwd<C, KS, NF, 8, 16>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
  else return launch_fwd<C, KS, NF, 4, 16>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
}

template <int C, int KS>
static int fwd_by_nf(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N,
                     int H, int W, int Cout, int pad, int epi, hipStream_t s) {
  if (Cout <= 16) return fwd_by_c<C, KS, 1>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
  if (Cout <= 32) return fwd_by_c<C, KS, 2>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
  if (Cout <= 64) return fwd_by_c<C, KS, 4>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
  return (int)hipErrorInvalidValue;
}

template <int KS>
static int fwd_by_cin(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N,
                      int H, int W, int C, int Cout, int pad, int epi, hipStream_t s) {
  switch (C) {
    case 4: return fwd_by_nf<4, KS>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
    case 8: return fwd_by_nf<8, KS>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
    case 16: return fwd_by_nf<16, KS>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
    case 32: return fwd_by_nf<32, KS>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
    case 64: return fwd_by_nf<64, KS>(x, w, bias, alpha, z, aux, N, H, W, Cout, pad, epi, s);
    default: return (int)hipErrorInvalidValue;
  }
}

template <int C, int KS, int TW, int TH, int MF>
static int launch_wgrad(const void* x, const void* dz, float* dw, int N, int H, int W, int Cout, int pad, hipStream_t s) {
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const int tiles = N * th * tw;
  const int KF = KS * KS * C;
  const int nslices = (KF + 127) / 128;
  int chunks = (1024 + nslices - 1) / nslices;
  if (chunks > tiles) chunks = tiles;
  const int tpb = (tiles + chunks - 1) / chunks;
  chunks = (tiles + tpb - 1) / tpb;
  hipLaunchKernelGGL((conv_wgrad_halo_k<C, KS, TW, TH, MF>), dim3(chunks * nslices), dim3(256), 0, s,
                     (const bf16_t*)x, (const bf16_t*)dz, dw, N, H, W, Cout, pad, th, tw, tpb, nslices);
  PTG_RETURN_LAUNCH();
}

template <int C, int KS, int MF>
static int wgrad_by_c(const void* x, const void* dz, float* dw, int N, int H, int W, int Cout, int pad, hipStream_t s) {
  if constexpr (C == 4) return launch_wgrad<C, KS, 64, 4, MF>(x, dz, dw, N, H, W, Cout, pad, s);
  else if constexpr (C == 8) return launch_wgrad<C, KS, 32, 8, MF>(x, dz, dw, N, H, W, Cout, pad, s);
  else if constexpr (C == 16) return launch_wgrad<C, KS, 16, 8, MF>(x, dz, dw, N, H, W, Cout, pad, s);
  else if constexpr (C == 32) return launch_wgrad<C, KS, 8, 8, MF>(x, dz, dw, N, H, W, Cout, pad, s);
  else return launch_wgrad<C, KS, 4, 16, MF>(x, dz, dw, N, H, W, Cout, pad, s);
}

template <int KS, int MF>
static int wgrad_by_cin(const void* x, const void* dz, float* dw, int N, int H, int W, int C, int Cout, int pad,
                        hipStream_t s) {
  switch (C) {
    case 4: return wgrad_by_c<4, KS, MF>(x, dz, dw, N, H, W, Cout, pad, s);
    case 8: return wgrad_by_c<8, KS, MF>(x, dz, dw, N, H, W, Cout, pad, s);
    case 16: return wgrad_by_c<16, KS, MF>(x, dz, dw, N, H, W, Cout, pad, s);
    case 32: return wgrad_by_c<32, KS, MF>(x, dz, dw, N, H, W, Cout, pad, s);
    case 64: return wgrad_by_c<64, KS, MF>(x, dz, dw, N, H, W, Cout, pad, s);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace ptgc

using namespace ptgc;

extern "C" {

// stride-1 'same'-style conv with halo tiling. C in {4,8,16,32,64}, Cout % 8 == 0 and <= 64, KS in {3,5}.
// epi: 0 = z only, 1 = z + maxpool2x2(prelu(z)) into aux (H, W even), 2 = z + prelu(z) into aux.
int ptg_conv2d_fwd_halo(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N,
                        int H, int W, int C, int Cout, int KS, int pad, int epi, hipStream_t s) {
  if (Cout % 8 || Cout > 64) return (int)hipErrorInvalidValue;
  if (epi == EPI_POOL && ((H & 1) || (W & 1))) return (int)hipErrorInvalidValue;
  if (KS == 5) return fwd_by_cin<5>(x, w, bias, alpha, z, aux, N, H, W, C, Cout, pad, epi, s);
  if (KS == 3) return fwd_by_cin<3>(x, w, bias, alpha, z, aux, N, H, W, C, Cout, pad, epi, s);
  return (int)hipErrorInvalidValue;
}

// dw (fp32, [Cout][KS][KS][C]) += weight gradient; caller zeroes dw.
int ptg_conv2d_wgrad_halo(const void* x, const void* dz, float* dw, int N, int H, int W, int C, int Cout, int KS,
                          int pad, hipStream_t s) {
  if (Cout % 8 || Cout > 64) return (int)hipErrorInvalidValue;
  const int MF = Cout <= 16 ? 1 : (Cout <= 32 ? 2 : 4);
#define PTG_WG(KSV, MFV) return wgrad_by_cin<KSV, MFV>(x, dz, dw, N, H, W, C, Cout, pad, s)
  if (KS == 5) { if (MF == 1) PTG_WG(5, 1); if (MF == 2) PTG_WG(5, 2); PTG_WG(5, 4); }
  if (KS == 3) { if (MF == 1) PTG_WG(3, 1); if (MF == 2) PTG_WG(3, 2); PTG_WG(3, 4); }
#undef PTG_WG
  return (int)hipErrorInvalidValue;
}

int ptg_conv_flip_weights(const void* w, void* wf, int Cout, int KS, int Cin, hipStream_t s) {
  const int total = Cout * KS * KS * Cin;
  hipLaunchKernelGGL(conv_flip_k, dim3((total + 255) / 256), dim3(256), 0, s, (const bf16_t*)w, (bf16_t*)wf, Cout, KS,
                     Cin);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"
