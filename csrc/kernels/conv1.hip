// First conv layer of the reference CNN (train_tf_ps.py:351-353: Conv2D(8, 5x5, 'same') on the
// 3-channel image, PReLU, MaxPooling2D) as two position-major kernels with nothing but the pooled
// output in between:
//
//   conv1_fwd_pm_k   pooled = maxpool2x2(prelu(conv(x) + bias, alpha))       (writes 2 B/pooled elt)
//   conv1_bwd_pm_k   recomputes z, the PReLU and the window argmax from x in registers, turns the
//                    pooled gradient dp into dZ (non-zero only at each window's argmax), and in the
//                    same pass accumulates dW (MFMA over the tile's pixels), dalpha and dbias.
//
// The previous pipeline (conv.hip conv1_pair_pool_k EPI_POOLS -> prelu_pool_bwd_sel_k ->
// conv_wgrad_strip_k SPARSE) wrote a z-at-argmax + argmax record in the forward (126 MB at batch
// 256, 256x320), read it back and wrote/read a dZ record in between (210 MB more): three kernels
// and ~0.6 GB of traffic for a layer whose math is 25 GFLOP.  Recomputing the 5x5x4 -> 8 conv in
// the backward costs 8 MFMAs per wave and tile, far less than moving those records.
//
// Work decomposition (both kernels): a workgroup owns one 64x4-pixel output tile POSITION and a
// contiguous chunk of samples, and walks the samples.  Per-position operands (alpha, and in the
// backward the dalpha partial sums) stay in registers for the whole chunk; the next sample's halo
// (and pooled gradient) is prefetched into registers while this sample computes, into a second LDS
// halo buffer.  Items are laid out th-fastest and handed to XCDs in contiguous ranges (xcd_remap),
// so the two tiles sharing halo rows run at the same pace on the same L2.
//
// MFMA layout of the conv (shared with conv1_pair_pool_k): A rows 0-7 = the 8 filters, rows 8-15 the
// same filters shifted one column right (they fit the spare kw' = 5 column of the KWP = 6 padded K),
// B columns = 16 even pixels, so one v_mfma_f32_16x16x32_bf16 yields all 8 channels of 32 pixels;
// lane (px, g) ends with pixel 2*px + (g >> 1), channels 4*(g & 1) .. +3; the horizontal pool
// partner is lane ^ 32, the vertical one the wave's other fragment.
//
// The weight gradient is the conv_wgrad_strip_k GEMM (M = Cout, N = (kh, kw, ci) = 100, K = the
// tile's 256 pixels) with both operands read by ds_read_b64_tr_b16: dZ from a [pixel][co] LDS tile,
// x from the same halo buffer the recompute used.
#include "common.h"
#include "conv_common.h"

namespace ptgc1 {
using namespace ptgc;

constexpr int KS = 5, C = 4, TW = 64, TH = 4, KWP = KS + 1, PAD = 2, COUT = 8;
constexpr int HR = TH + KS - 1;                 // halo rows
constexpr int HC = TW + KWP - 1;                // halo columns
constexpr int HP = (HC + 1) / 2;                // 16-byte pixel pairs per halo row
constexpr int ROWE = HP * 8;                    // halo row pitch (elements)
constexpr int HBUF = HR * ROWE;                 // one halo buffer (elements)
constexpr int KROW = KWP * C, KTOT = KS * KROW, KSTEPS = (KTOT + 31) / 32;
constexpr int PFN = (HR * HP + 255) / 256;      // halo pair slots per thread
constexpr int MPIX = TH * TW;                   // pixels per tile (K of the weight-gradient GEMM)
constexpr int DPITCH = 20;                      // dZ tile pixel pitch (bf16): 16 MFMA rows + bank shift
constexpr int KF = KS * KS * C;                 // weight-gradient columns (kh, kw, ci)
constexpr int NB = 2;                           // 16-column B fragments per wave (4 waves x 32 >= KF)
constexpr int ZSLOT = 2 * HBUF;                 // 8 zero elements: reads of K past KTOT / KF
static_assert(4 * NB * 16 >= KF, "weight-gradient columns");

struct Item { int oh0, ow0, n0, n1; };

// item = chunk-major, position th-fastest; xcd_remap gives every XCD a contiguous item range
PTG_DEV Item work_item(int N, int tiles_h, int tiles_w, int nchunks) {
  const int npos = tiles_h * tiles_w;
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = item / npos, pos = item - chunk * npos;
  const int twi = pos / tiles_h, thi = pos - twi * tiles_h;
  Item it;
  it.oh0 = thi * TH;
  it.ow0 = twi * TW;
  it.n0 = (int)((long)N * chunk / nchunks);
  it.n1 = (int)((long)N * (chunk + 1) / nchunks);
  return it;
}

// A operand: row px = filter (px & 7), shifted one column right when px >= 8
PTG_DEV void load_wreg(const bf16_t* __restrict__ w, int px, int g, bf16x8_t* wreg) {
  const int co = px & 7, sh = px >> 3;
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int kf = ks * 32 + 8 * g;
    U4 v = zero4();
    if (kf < KTOT) {
      const int kh = kf / KROW, kw = (kf - kh * KROW) / C;  // kw even
      const bf16_t* wp = w + ((long)co * KS + kh) * KS * C;
      const int a = kw - sh, b = kw + 1 - sh;
      if (a >= 0 && a < KS) { const U2 t = *(const U2*)(wp + a * C); v.x = t.x; v.y = t.y; }
      if (b >= 0 && b < KS) { const U2 t = *(const U2*)(wp + b * C); v.z = t.x; v.w = t.y; }
    }
    wreg[ks] = __builtin_bit_cast(bf16x8_t, v);
  }
}

// One sample's halo: HR rows x HP pixel pairs, zero outside the image (buffer-load range check).
template <bool U8>
struct Halo {
  U4 pf[U8 ? 1 : PFN];
  U8Pair pu[U8 ? PFN : 1];
  // slot p of this thread: halo row idx / HP, pair idx % HP with idx = tid + 256 p (recomputed at
  // each use: cheaper than 2 * PFN live registers across the sample loop)
  PTG_DEV void load(const Rsrc& xr, int n, int H, int W, int oh0, int ow0) {
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      const int idx = (int)threadIdx.x + p * 256, r = idx / HP, c = idx - r * HP;
      const int ih = oh0 - PAD + r, iw = ow0 - PAD + 2 * c;
      const bool ok = r < HR && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      if constexpr (U8) {  // iw even, W even: the pair's second pixel is in the row too
        pu[p] = u8pair_load(xr, (uint32_t)((n * H + ih) * W + iw) * 3u, ok);
      } else {
        pf[p] = bload16(xr, ok ? (uint32_t)(((n * H + ih) * W + iw) * C) * 2u : PTG_OOB);
      }
    }
  }
  PTG_DEV void store(bf16_t* buf) const {
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      const int idx = (int)threadIdx.x + p * 256, r = idx / HP, c = idx - r * HP;
      if (r < HR) {
        U4 v;
        if constexpr (U8) v = u8pair_to_bf16x8(pu[p]);
        else v = pf[p];
        *(U4*)(buf + r * ROWE + c * 8) = v;
      }
    }
  }
};

template <bool U8>
PTG_DEV Rsrc x_rsrc(const void* x, int N, int H, int W) {
  return make_rsrc(x, U8 ? u8_rsrc_bytes((long)N * H * W * 3) : (uint32_t)((long)N * H * W * C * 2));
}

// z (fp32 accumulators, 2 row fragments x 4 channels) of this wave's 32 x 2 pixels from halo `hb`
PTG_DEV void conv_tile(const bf16_t* hb, const bf16_t* smem, const bf16x8_t* wreg, int rp, int hf, int px, int g,
                       f32x4_t* acc) {
  acc[0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int kf = ks * 32 + 8 * g;
    const int kh = kf / KROW, kw = (kf - kh * KROW) / C;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16_t* src = kf < KTOT ? hb + (2 * rp + i + kh) * ROWE + (hf * 32 + 2 * px + kw) * C : smem + ZSLOT;
      const bf16x8_t xf = *(const bf16x8_t*)src;
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[ks], xf, acc[i], 0, 0, 0);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// forward: pooled output only
// ------------------------------------------------------------------------------------------------
template <bool U8>
__global__ __launch_bounds__(256) void conv1_fwd_pm_k(const void* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const float* __restrict__ bias, const float* __restrict__ alpha,
                                                      bf16_t* __restrict__ pooled, int N, int H, int W, int tiles_h,
                                                      int tiles_w, int nchunks) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * HBUF + 8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int px = lane & 15, g = lane >> 4, hf = wid & 1, rp = wid >> 1;
  if (tid < 8) smem[ZSLOT + tid] = 0;
  const Item it = work_item(N, tiles_h, tiles_w, nchunks);
  if (it.n0 >= it.n1) return;  // whole workgroup
  bf16x8_t wreg[KSTEPS];
  load_wreg(w, px, g, wreg);
  const int cc = 4 * (g & 1);
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias) { const float4 b4 = *(const float4*)(bias + cc); bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w; }
  const int ow = it.ow0 + hf * 32 + 2 * px + (g >> 1);
  float al[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oh = it.oh0 + 2 * rp + i;
    const float4 a = (oh < H && ow < W) ? *(const float4*)(alpha + ((long)oh * W + ow) * COUT + cc)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
    al[i][0] = a.x; al[i][1] = a.y; al[i][2] = a.z; al[i][3] = a.w;
  }
  const int PH = H >> 1, PW = W >> 1;
  const int ph = (it.oh0 >> 1) + rp, pw = (it.ow0 >> 1) + hf * 16 + px;
  const bool store_lane = g < 2 && ph < PH && pw < PW;
  const Rsrc xr = x_rsrc<U8>(x, N, H, W);
  Halo<U8> hl;
  hl.load(xr, it.n0, H, W, it.oh0, it.ow0);
  hl.store(smem);
  __syncthreads();
  for (int n = it.n0; n < it.n1; ++n) {
    const int b = (n - it.n0) & 1;
    const bool has_next = n + 1 < it.n1;
    if (has_next) hl.load(xr, n + 1, H, W, it.oh0, it.ow0);
    f32x4_t acc[2];
    conv_tile(smem + b * HBUF, smem, wreg, rp, hf, px, g, acc);
    float pm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float y[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float zr = bf2f(f2bf(acc[i][r] + bv[r]));  // PReLU of the bf16-rounded z (as the backward)
        y[i] = zr > 0.f ? zr : al[i][r] * zr;
      }
      const float v = fmaxf(y[0], y[1]);
      pm[r] = fmaxf(v, __shfl_xor(v, 32, 64));
    }
    if (store_lane)
      *(U2*)(pooled + (((long)n * PH + ph) * PW + pw) * COUT + cc) = U2{pack_bf(pm[0], pm[1]), pack_bf(pm[2], pm[3])};
    if (has_next) hl.store(smem + (b ^ 1) * HBUF);  // buffer b^1 was last read before the previous barrier
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// backward: recompute + PReLU/pool backward + weight gradient, one pass
// ------------------------------------------------------------------------------------------------
template <bool U8>
__global__ __launch_bounds__(256, 4) void conv1_bwd_pm_k(const void* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const float* __restrict__ bias, const float* __restrict__ alpha,
                                                      const bf16_t* __restrict__ dp, float* __restrict__ dw,
                                                      float* __restrict__ dalpha, float* __restrict__ dbias, int N,
                                                      int H, int W, int tiles_h, int tiles_w, int nchunks) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * HBUF + 8 + MPIX * DPITCH + 8];
  __shared__ float sdb[4][COUT];
  bf16_t* const ds = smem + 2 * HBUF + 8;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int px = lane & 15, g = lane >> 4, hf = wid & 1, rp = wid >> 1;
  if (tid < 8) smem[ZSLOT + tid] = 0;
  for (int i = tid; i < (MPIX * DPITCH + 8) / 8; i += 256) *(U4*)(ds + 8 * i) = zero4();  // MFMA rows 8-15: 0
  const Item it = work_item(N, tiles_h, tiles_w, nchunks);
  if (it.n0 >= it.n1) return;  // whole workgroup
  bf16x8_t wreg[KSTEPS];
  load_wreg(w, px, g, wreg);
  const int cc = 4 * (g & 1), dwo = g >> 1;
  // the 8 biases in LDS, read per sample (a register array indexed by a lane-dependent select
  // is lowered to scratch memory)
  __shared__ float4 sbias[2];
  if (tid < 2) sbias[tid] = bias ? *(const float4*)(bias + 4 * tid) : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const int ow = it.ow0 + hf * 32 + 2 * px + dwo;
  float al[2][4], da[2][4], db[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oh = it.oh0 + 2 * rp + i;
    const float4 a = (oh < H && ow < W) ? *(const float4*)(alpha + ((long)oh * W + ow) * COUT + cc)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
    al[i][0] = a.x; al[i][1] = a.y; al[i][2] = a.z; al[i][3] = a.w;
#pragma unroll
    for (int r = 0; r < 4; ++r) da[i][r] = 0.f;
  }
  const int PH = H >> 1, PW = W >> 1;
  const int ph = (it.oh0 >> 1) + rp, pw = (it.ow0 >> 1) + hf * 16 + px;
  const bool pin = ph < PH && pw < PW;
  const Rsrc xr = x_rsrc<U8>(x, N, H, W);
  const Rsrc dr = make_rsrc(dp, (uint32_t)((long)N * PH * PW * COUT * 2));
  auto dp_off = [&](int n) { return pin ? (uint32_t)((((n * PH + ph) * PW + pw) * COUT + cc) * 2) : PTG_OOB; };
  const int li = lane & 15;
  f32x4_t wacc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) wacc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // this lane's two dZ pixels in the tile (row 2*rp + i, column hf*32 + 2*px + dwo)
  const int m_lane = (2 * rp) * TW + hf * 32 + 2 * px + dwo;

  Halo<U8> hl;
  hl.load(xr, it.n0, H, W, it.oh0, it.ow0);
  U2 dpr = bload8(dr, dp_off(it.n0));
  hl.store(smem);
  __syncthreads();
  for (int n = it.n0; n < it.n1; ++n) {
    const int b = (n - it.n0) & 1;
    const bf16_t* hb = smem + b * HBUF;
    const bool has_next = n + 1 < it.n1;
    const U2 dcur = dpr;
    // lane-derived LDS offsets are recomputed per sample from an opaque copy of the lane id:
    // hoisted out of the sample loop they would pin ~50 address registers and spill
    int ol = lane;
    asm volatile("" : "+v"(ol));
    const int opx = ol & 15, og = ol >> 4, oq = (ol & 15) >> 2, op = ol & 3;
    if (has_next) {
      hl.load(xr, n + 1, H, W, it.oh0, it.ow0);
      dpr = bload8(dr, dp_off(n + 1));
    }
    f32x4_t acc[2];
    conv_tile(hb, smem, wreg, rp, hf, opx, og, acc);
    const float gv[4] = {lo_bf(dcur.x), hi_bf(dcur.x), lo_bf(dcur.y), hi_bf(dcur.y)};
    const float4 bq = sbias[og & 1];
    const float bsel[4] = {bq.x, bq.y, bq.z, bq.w};
    float dz[2][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float zr[2], y[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        zr[i] = bf2f(f2bf(acc[i][r] + bsel[r]));
        y[i] = zr[i] > 0.f ? zr[i] : al[i][r] * zr[i];
      }
      // window (dh, dw) in q = 2*dh + dw order; this lane holds dw = dwo, the partner lane ^ 32 the other
      const float p0 = __shfl_xor(y[0], 32, 64), p1 = __shfl_xor(y[1], 32, 64);
      const float yq[4] = {dwo ? p0 : y[0], dwo ? y[0] : p0, dwo ? p1 : y[1], dwo ? y[1] : p1};
      float best = yq[0];
      int a = 0;
#pragma unroll
      for (int qq = 1; qq < 4; ++qq)
        if (yq[qq] > best) { best = yq[qq]; a = qq; }  // first maximum wins (as the forward record)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool hit = a == 2 * i + dwo;
        const bool pos = zr[i] > 0.f;
        const float gq = hit ? gv[r] : 0.f;
        dz[i][r] = pos ? gq : gq * al[i][r];
        da[i][r] += pos ? 0.f : gq * zr[i];
        db[r] += dz[i][r];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *(U2*)(ds + (m_lane + i * TW) * DPITCH + cc) = U2{pack_bf(dz[i][0], dz[i][1]), pack_bf(dz[i][2], dz[i][3])};
    __syncthreads();  // dZ tile complete
#pragma unroll 2
    for (int k0 = 0; k0 < MPIX; k0 += 32) {
      const int m0 = k0 + 8 * og + oq, m1 = m0 + 4;
      const s16x4_t alo = tr_read(ds + m0 * DPITCH + 4 * op);
      const s16x4_t ahi = tr_read(ds + m1 * DPITCH + 4 * op);
      U2 ua = __builtin_bit_cast(U2, alo), ub = __builtin_bit_cast(U2, ahi);
      const bf16x8_t af = __builtin_bit_cast(bf16x8_t, U4{ua.x, ua.y, ub.x, ub.y});
      const int h0 = (m0 / TW) * ROWE + (m0 % TW) * C, h1 = (m1 / TW) * ROWE + (m1 % TW) * C;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        // B column (kflat) base of this lane: (kh, kw) of kf = (wid*NB + j)*16 + 4*op, ci = 0..3
        const int kf = (wid * NB + j) * 16 + 4 * op;
        const int kh = kf / (KS * C), kw = (kf - kh * KS * C) / C;
        const bool bv_ok = kf < KF;
        const bf16_t* s0 = bv_ok ? hb + h0 + kh * ROWE + kw * C : smem + ZSLOT;
        const bf16_t* s1 = bv_ok ? hb + h1 + kh * ROWE + kw * C : smem + ZSLOT;
        const s16x4_t blo = tr_read(s0), bhi = tr_read(s1);
        ua = __builtin_bit_cast(U2, blo);
        ub = __builtin_bit_cast(U2, bhi);
        const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, U4{ua.x, ua.y, ub.x, ub.y});
        wacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, wacc[j], 0, 0, 0);
      }
    }
    if (has_next) hl.store(smem + (b ^ 1) * HBUF);
    __syncthreads();  // next halo visible; this dZ tile fully read before it is rewritten
  }
  // flush: dW rows co = g*4 + r (< 8), columns kf = (wid*NB + j)*16 + li
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int kf = (wid * NB + j) * 16 + li;
    if (kf < KF && g < 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(dw + (g * 4 + r) * KF + kf, wacc[j][r]);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oh = it.oh0 + 2 * rp + i;
    if (oh < H && ow < W) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (da[i][r] != 0.f) atomicAdd(dalpha + ((long)oh * W + ow) * COUT + cc + r, da[i][r]);
    }
  }
  // dbias: sum over the 16 px lanes and the two pixel halves (lane ^ 32), then over the waves
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = db[r];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 32, 64);
    db[r] = v;
  }
  if (px == 0 && g < 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sdb[wid][cc + r] = db[r];
  }
  __syncthreads();
  if (tid < COUT) atomicAdd(dbias + tid, sdb[0][tid] + sdb[1][tid] + sdb[2][tid] + sdb[3][tid]);
}

// ================================================================================================
// Wave-independent variants (default): each of the block's 4 waves owns its 32x2-pixel quarter of
// the tile (hf = columns, rp = row pair) with a PRIVATE LDS halo (6 rows x 36 pixels, double
// buffered) and dZ tile, and walks the chunk's samples on its own - no block barrier inside the
// sample loop.  The block-synchronised loop above stalled every sample on the slowest wave's
// halo load (measured 474 us for the b256 backward, 114 us forward): with independent waves the
// 16 waves of a CU keep their loads in flight while others compute.  Waves rp = 0 / 1 re-read 4 of
// their 6 halo rows from L2.
// ================================================================================================
constexpr int WTW = 32, WHR = 2 + KS - 1;         // wave tile: 32 x 2 pixels, 6 halo rows
constexpr int WHP = (2 * 15 + (KWP - 2) + 2) / 2;  // pixel pairs per halo row (36 pixels)
constexpr int WROWE = WHP * 8;                     // wave halo row pitch (elements)
constexpr int WHB = WHR * WROWE;                   // one wave halo buffer
constexpr int WPIX = 2 * WTW;                      // dZ pixels per wave (K of its weight-gradient GEMM)
constexpr int WDZ = WPIX * DPITCH;
constexpr int WREG = 2 * WHB + WDZ;                // LDS elements per wave
constexpr int WZS = 4 * WREG;                      // zero slot
constexpr int WPF = (WHR * WHP + 63) / 64;         // halo pair slots per lane
constexpr int WNB = (KF + 15) / 16;                // 16-column B fragments of the wave's dW
static_assert(WREG % 8 == 0 && WHP == 18, "wave halo layout");

PTG_DEV void wave_lds_sync() {  // this wave's LDS stores visible to its other lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool U8>
struct WaveHalo {
  U4 pf[U8 ? 1 : WPF];
  U8Pair pu[U8 ? WPF : 1];
  PTG_DEV void load(const Rsrc& xr, int n, int H, int W, int ih0, int iw0, int lane) {
#pragma unroll
    for (int p = 0; p < WPF; ++p) {
      const int idx = lane + p * 64, r = idx / WHP, c = idx - r * WHP;
      const int ih = ih0 + r, iw = iw0 + 2 * c;
      const bool ok = r < WHR && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      if constexpr (U8) pu[p] = u8pair_load(xr, (uint32_t)((n * H + ih) * W + iw) * 3u, ok);
      else pf[p] = bload16(xr, ok ? (uint32_t)(((n * H + ih) * W + iw) * C) * 2u : PTG_OOB);
    }
  }
  PTG_DEV void store(bf16_t* buf, int lane) const {
#pragma unroll
    for (int p = 0; p < WPF; ++p) {
      const int idx = lane + p * 64, r = idx / WHP, c = idx - r * WHP;
      if (r < WHR) {
        U4 v;
        if constexpr (U8) v = u8pair_to_bf16x8(pu[p]);
        else v = pf[p];
        *(U4*)(buf + r * WROWE + c * 8) = v;
      }
    }
  }
};

// z accumulators of the wave's 32 x 2 pixels from its halo `hb` (rows i + kh, columns 2*px + kw)
PTG_DEV void conv_tile_w(const bf16_t* hb, const bf16_t* zs, const bf16x8_t* wreg, int px, int g, f32x4_t* acc) {
  acc[0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int kf = ks * 32 + 8 * g;
    const int kh = kf / KROW, kw = (kf - kh * KROW) / C;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16_t* src = kf < KTOT ? hb + (i + kh) * WROWE + (2 * px + kw) * C : zs;
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[ks], *(const bf16x8_t*)src, acc[i], 0, 0, 0);
    }
  }
}

template <bool U8>
__global__ __launch_bounds__(256) void conv1_fwd_wv_k(const void* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const float* __restrict__ bias, const float* __restrict__ alpha,
                                                      bf16_t* __restrict__ pooled, int N, int H, int W, int tiles_h,
                                                      int tiles_w, int nchunks) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[WZS + 8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int px = lane & 15, g = lane >> 4, hf = wid & 1, rp = wid >> 1;
  if (tid < 8) smem[WZS + tid] = 0;
  __syncthreads();  // zero slot visible (the only block barrier)
  const Item it = work_item(N, tiles_h, tiles_w, nchunks);
  if (it.n0 >= it.n1) return;
  bf16_t* const wr = smem + wid * WREG;
  bf16x8_t wreg[KSTEPS];
  load_wreg(w, px, g, wreg);
  const int cc = 4 * (g & 1), dwo = g >> 1;
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias) { const float4 b4 = *(const float4*)(bias + cc); bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w; }
  const int ow = it.ow0 + hf * WTW + 2 * px + dwo;
  float al[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oh = it.oh0 + 2 * rp + i;
    const float4 a = (oh < H && ow < W) ? *(const float4*)(alpha + ((long)oh * W + ow) * COUT + cc)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
    al[i][0] = a.x; al[i][1] = a.y; al[i][2] = a.z; al[i][3] = a.w;
  }
  const int PH = H >> 1, PW = W >> 1;
  const int ph = (it.oh0 >> 1) + rp, pw = (it.ow0 >> 1) + hf * 16 + px;
  const bool store_lane = g < 2 && ph < PH && pw < PW;
  const int ih0 = it.oh0 + 2 * rp - PAD, iw0 = it.ow0 + hf * WTW - PAD;
  const Rsrc xr = x_rsrc<U8>(x, N, H, W);
  WaveHalo<U8> hl;
  hl.load(xr, it.n0, H, W, ih0, iw0, lane);
  hl.store(wr, lane);
  wave_lds_sync();
  for (int n = it.n0; n < it.n1; ++n) {
    const int b = (n - it.n0) & 1;
    const bool has_next = n + 1 < it.n1;
    if (has_next) hl.load(xr, n + 1, H, W, ih0, iw0, lane);
    f32x4_t acc[2];
    conv_tile_w(wr + b * WHB, smem + WZS, wreg, px, g, acc);
    float pm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float y[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float zr = bf2f(f2bf(acc[i][r] + bv[r]));
        y[i] = zr > 0.f ? zr : al[i][r] * zr;
      }
      const float v = fmaxf(y[0], y[1]);
      pm[r] = fmaxf(v, __shfl_xor(v, 32, 64));
    }
    if (store_lane)
      *(U2*)(pooled + (((long)n * PH + ph) * PW + pw) * COUT + cc) = U2{pack_bf(pm[0], pm[1]), pack_bf(pm[2], pm[3])};
    if (has_next) {
      hl.store(wr + (b ^ 1) * WHB, lane);
      wave_lds_sync();
    }
  }
}

template <bool U8>
__global__ __launch_bounds__(256, 4) void conv1_bwd_wv_k(const void* __restrict__ x, const bf16_t* __restrict__ w,
                                                         const float* __restrict__ bias, const float* __restrict__ alpha,
                                                         const bf16_t* __restrict__ dp, float* __restrict__ dw,
                                                         float* __restrict__ dalpha, float* __restrict__ dbias, int N,
                                                         int H, int W, int tiles_h, int tiles_w, int nchunks) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[WZS + 8];
  __shared__ float sdb[4][COUT];
  __shared__ float4 sda[4][2][64];  // dalpha partial sums: [wave][pixel row i][lane]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int px = lane & 15, g = lane >> 4, hf = wid & 1, rp = wid >> 1;
  if (tid < 8) smem[WZS + tid] = 0;
  bf16_t* const wr = smem + wid * WREG;
  bf16_t* const ds = wr + 2 * WHB;
  for (int i = lane; i < WDZ / 8; i += 64) *(U4*)(ds + 8 * i) = zero4();  // MFMA rows 8-15 read 0
  __syncthreads();
  const Item it = work_item(N, tiles_h, tiles_w, nchunks);
  if (it.n0 >= it.n1) return;
  bf16x8_t wreg[KSTEPS];
  load_wreg(w, px, g, wreg);
  const int cc = 4 * (g & 1), dwo = g >> 1;
  // the 8 biases in LDS, read per sample (a register array indexed by a lane-dependent select
  // is lowered to scratch memory)
  __shared__ float4 sbias[2];
  if (tid < 2) sbias[tid] = bias ? *(const float4*)(bias + 4 * tid) : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const int ow = it.ow0 + hf * WTW + 2 * px + dwo;
  float db[4] = {0.f, 0.f, 0.f, 0.f};
  // dalpha partial sums live in LDS (lane-private slots), not in 8 registers across the loop
  sda[wid][0][lane] = sda[wid][1][lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  // alpha of this lane's 2 x 4 (pixel, channel) elements: re-read per sample (an L1 / L2 hit)
  // rather than held in 8 registers across the loop
  const bool ain0 = it.oh0 + 2 * rp < H && ow < W, ain1 = it.oh0 + 2 * rp + 1 < H && ow < W;
  const long aoff = ((long)(it.oh0 + 2 * rp) * W + ow) * COUT + cc;
  const int PH = H >> 1, PW = W >> 1;
  const int ph = (it.oh0 >> 1) + rp, pw = (it.ow0 >> 1) + hf * 16 + px;
  const bool pin = ph < PH && pw < PW;
  const int ih0 = it.oh0 + 2 * rp - PAD, iw0 = it.ow0 + hf * WTW - PAD;
  const Rsrc xr = x_rsrc<U8>(x, N, H, W);
  const Rsrc dr = make_rsrc(dp, (uint32_t)((long)N * PH * PW * COUT * 2));
  auto dp_off = [&](int n) { return pin ? (uint32_t)((((n * PH + ph) * PW + pw) * COUT + cc) * 2) : PTG_OOB; };
  f32x4_t wacc[WNB];
#pragma unroll
  for (int j = 0; j < WNB; ++j) wacc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15;

  WaveHalo<U8> hl;
  hl.load(xr, it.n0, H, W, ih0, iw0, lane);
  U2 dpr = bload8(dr, dp_off(it.n0));
  hl.store(wr, lane);
  wave_lds_sync();
  for (int n = it.n0; n < it.n1; ++n) {
    const int b = (n - it.n0) & 1;
    const bf16_t* hb = wr + b * WHB;
    const bool has_next = n + 1 < it.n1;
    const U2 dcur = dpr;
    if (has_next) {
      hl.load(xr, n + 1, H, W, ih0, iw0, lane);
      dpr = bload8(dr, dp_off(n + 1));
    }
    // lane-derived offsets from an opaque lane id (hoisted out of the loop they would spill)
    int ol = lane;
    asm volatile("" : "+v"(ol));
    const int opx = ol & 15, og = ol >> 4, oq = (ol & 15) >> 2, op = ol & 3;
    f32x4_t acc[2];
    conv_tile_w(hb, smem + WZS, wreg, opx, og, acc);
    const float gv[4] = {lo_bf(dcur.x), hi_bf(dcur.x), lo_bf(dcur.y), hi_bf(dcur.y)};
    const float4 bq = sbias[og & 1];
    const float bsel[4] = {bq.x, bq.y, bq.z, bq.w};
    float al[2][4];
    {
      const long ao = aoff + (ol - lane);  // == aoff: keeps the loads inside the loop
      const float4 a0 = ain0 ? *(const float4*)(alpha + ao) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 a1 = ain1 ? *(const float4*)(alpha + ao + (long)W * COUT) : make_float4(0.f, 0.f, 0.f, 0.f);
      al[0][0] = a0.x; al[0][1] = a0.y; al[0][2] = a0.z; al[0][3] = a0.w;
      al[1][0] = a1.x; al[1][1] = a1.y; al[1][2] = a1.z; al[1][3] = a1.w;
    }
    float dz[2][4], da[2][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float zr[2], y[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        zr[i] = bf2f(f2bf(acc[i][r] + bsel[r]));
        y[i] = zr[i] > 0.f ? zr[i] : al[i][r] * zr[i];
      }
      const float p0 = __shfl_xor(y[0], 32, 64), p1 = __shfl_xor(y[1], 32, 64);
      const float yq[4] = {dwo ? p0 : y[0], dwo ? y[0] : p0, dwo ? p1 : y[1], dwo ? y[1] : p1};
      float best = yq[0];
      int a = 0;
#pragma unroll
      for (int qq = 1; qq < 4; ++qq)
        if (yq[qq] > best) { best = yq[qq]; a = qq; }  // first maximum wins (as the forward)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool hit = a == 2 * i + dwo;
        const bool pos = zr[i] > 0.f;
        const float gq = hit ? gv[r] : 0.f;
        dz[i][r] = pos ? gq : gq * al[i][r];
        da[i][r] = pos ? 0.f : gq * zr[i];
        db[r] += dz[i][r];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float4 t = sda[wid][i][lane];
      t.x += da[i][0]; t.y += da[i][1]; t.z += da[i][2]; t.w += da[i][3];
      sda[wid][i][lane] = t;
    }
    const int m_lane = 2 * opx + (og >> 1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *(U2*)(ds + (m_lane + i * WTW) * DPITCH + 4 * (og & 1)) =
          U2{pack_bf(dz[i][0], dz[i][1]), pack_bf(dz[i][2], dz[i][3])};
    wave_lds_sync();
    // dW[co][kf] += sum over the wave's 64 pixels of dZ[pix][co] * x[pix + (kh, kw)][ci]
#pragma unroll 1
    for (int k0 = 0; k0 < WPIX; k0 += 32) {
      const int m0 = k0 + 8 * og + oq, m1 = m0 + 4;
      const s16x4_t alo = tr_read(ds + m0 * DPITCH + 4 * op);
      const s16x4_t ahi = tr_read(ds + m1 * DPITCH + 4 * op);
      U2 ua = __builtin_bit_cast(U2, alo), ub = __builtin_bit_cast(U2, ahi);
      const bf16x8_t af = __builtin_bit_cast(bf16x8_t, U4{ua.x, ua.y, ub.x, ub.y});
      const int h0 = (m0 / WTW) * WROWE + (m0 % WTW) * C, h1 = (m1 / WTW) * WROWE + (m1 % WTW) * C;
#pragma unroll
      for (int j = 0; j < WNB; ++j) {
        const int kf = j * 16 + 4 * op;
        const int kh = kf / (KS * C), kw = (kf - kh * KS * C) / C;
        const bool ok = kf < KF;
        const bf16_t* s0 = ok ? hb + h0 + kh * WROWE + kw * C : smem + WZS;
        const bf16_t* s1 = ok ? hb + h1 + kh * WROWE + kw * C : smem + WZS;
        const s16x4_t blo = tr_read(s0), bhi = tr_read(s1);
        ua = __builtin_bit_cast(U2, blo);
        ub = __builtin_bit_cast(U2, bhi);
        wacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8_t, U4{ua.x, ua.y, ub.x, ub.y}),
                                                          wacc[j], 0, 0, 0);
      }
    }
    if (has_next) hl.store(wr + (b ^ 1) * WHB, lane);
    wave_lds_sync();  // next halo visible; this dZ tile read before it is rewritten
  }
  // dalpha: every (pixel, channel) of the tile belongs to exactly one lane
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oh = it.oh0 + 2 * rp + i;
    const float4 t = sda[wid][i][lane];
    const float dv[4] = {t.x, t.y, t.z, t.w};
    if (oh < H && ow < W) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (dv[r] != 0.f) atomicAdd(dalpha + ((long)oh * W + ow) * COUT + cc + r, dv[r]);
    }
  }
  // dbias: lanes sharing a channel group, then the waves
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = db[r];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 32, 64);
    db[r] = v;
  }
  if (px == 0 && g < 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sdb[wid][cc + r] = db[r];
  }
  // dW: the 4 waves' partial tiles summed in LDS (the halo area is free now), one atomic per output
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4][COUT * KF] floats = 12.8 KB < the wave regions
  if (g < 2) {
#pragma unroll
    for (int j = 0; j < WNB; ++j) {
      const int kf = j * 16 + li;
      if (kf < KF) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wid * COUT * KF + (g * 4 + r) * KF + kf] = wacc[j][r];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < COUT * KF; i += 256)
    atomicAdd(dw + i, red[i] + red[COUT * KF + i] + red[2 * COUT * KF + i] + red[3 * COUT * KF + i]);
  if (tid < COUT) atomicAdd(dbias + tid, sdb[0][tid] + sdb[1][tid] + sdb[2][tid] + sdb[3][tid]);
}
static_assert(4 * COUT * KF * 4 <= WZS * 2, "dW reduction scratch fits the wave regions");

// ================================================================================================
// Record pipeline (default): the forward keeps, per pooled element, z at the window's argmax (bf16)
// and the argmax q = 2*dh + dw (uint8) - 3 bytes next to the pooled output's 2 - and the backward
// turns (dp, zsel, q) into dZ directly: no conv recompute, and the PReLU/pool backward math runs
// once per POOLED element instead of once per pixel with an argmax search.  The recomputing backward
// above was VALU-bound (PMC: ~73% of VALU issue, 20 VALU instructions per MFMA).
// u8 images enter the MFMA as exact bf16 integers 0..255 (v_cvt_f32_ubyteN + the float's top half),
// the 1/255 is applied to the fp32 accumulators (forward) and to the weight gradient (backward).
// ================================================================================================
PTG_DEV U4 u8pair_to_bf16x8_int(const U8Pair& p) {
  const unsigned long long v = (((unsigned long long)p.w1 << 32) | p.w0) >> p.sh;
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  auto f = [](uint32_t w, int b) { return __float_as_uint((float)((w >> (8 * b)) & 255u)); };
  U4 o;
  o.x = (f(lo, 0) >> 16) | (f(lo, 1) & 0xffff0000u);
  o.y = f(lo, 2) >> 16;
  o.z = (f(lo, 3) >> 16) | (f(hi, 0) & 0xffff0000u);
  o.w = f(hi, 1) >> 16;
  return o;
}

// Per-lane B-fragment offsets of the conv MFMA (sample-invariant, computed once): k-step ks reads
// halo element (i + kh) * WROWE + (2*px + kw) * C; past KTOT the A fragment is zero, so any finite
// halo element will do (offset 0) and no zero-slot select is needed per read.
PTG_DEV void conv_boffs(int px, int g, int* boff) {
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int kf = ks * 32 + 8 * g;
    const int kh = kf / KROW, kw = (kf - kh * KROW) / C;
    boff[ks] = kf < KTOT ? kh * WROWE + (2 * px + kw) * C : 0;
  }
}
PTG_DEV void conv_tile_r(const bf16_t* hb, const int* boff, const bf16x8_t* wreg, f32x4_t* acc) {
  acc[0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[ks], *(const bf16x8_t*)(hb + boff[ks] + i * WROWE), acc[i], 0, 0, 0);
  }
}

// One sample's wave halo with the per-slot offsets precomputed (the bounds do not depend on the
// sample): goff = byte offset of the pixel pair inside one image (~0u: padding), loff = LDS element
// offset (~0u: slot past the halo).
template <bool U8>
struct HaloSlot {  // one sample's halo in registers (a prefetch ring entry)
  U4 pf[U8 ? 1 : WPF];
  U8Pair pu[U8 ? WPF : 1];
};
template <bool U8>
struct WaveHaloR {
  uint32_t goff[WPF], loff[WPF];
  U4 pf[U8 ? 1 : WPF];
  U8Pair pu[U8 ? WPF : 1];
  PTG_DEV void load_to(HaloSlot<U8>& s, const Rsrc& xr, uint32_t img_bytes, int n) const {
    const uint32_t base = (uint32_t)n * img_bytes;
#pragma unroll
    for (int p = 0; p < WPF; ++p) {
      const bool ok = goff[p] != ~0u;
      if constexpr (U8) s.pu[p] = u8pair_load(xr, base + goff[p], ok);
      else s.pf[p] = bload16(xr, ok ? base + goff[p] : PTG_OOB);
    }
  }
  PTG_DEV void store_from(const HaloSlot<U8>& s, bf16_t* buf) const {
#pragma unroll
    for (int p = 0; p < WPF; ++p) {
      if (loff[p] != ~0u) {
        U4 v;
        if constexpr (U8) v = u8pair_to_bf16x8_int(s.pu[p]);
        else v = s.pf[p];
        *(U4*)(buf + loff[p]) = v;
      }
    }
  }
  PTG_DEV void init(int H, int W, int ih0, int iw0, int lane) {
#pragma unroll
    for (int p = 0; p < WPF; ++p) {
      const int idx = lane + p * 64, r = idx / WHP, c = idx - r * WHP;
      const int ih = ih0 + r, iw = iw0 + 2 * c;
      const bool ok = r < WHR && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      goff[p] = ok ? (uint32_t)(ih * W + iw) * (U8 ? 3u : 8u) : ~0u;
      loff[p] = r < WHR ? (uint32_t)(r * WROWE + c * 8) : ~0u;
    }
  }
  PTG_DEV void load(const Rsrc& xr, uint32_t img_bytes, int n) {
    const uint32_t base = (uint32_t)n * img_bytes;
#pragma unroll
    for (int p = 0; p < WPF; ++p) {
      const bool ok = goff[p] != ~0u;
      if constexpr (U8) pu[p] = u8pair_load(xr, base + goff[p], ok);
      else pf[p] = bload16(xr, ok ? base + goff[p] : PTG_OOB);
    }
  }
  PTG_DEV void store(bf16_t* buf) const {
#pragma unroll
    for (int p = 0; p < WPF; ++p) {
      if (loff[p] != ~0u) {
        U4 v;
        if constexpr (U8) v = u8pair_to_bf16x8_int(pu[p]);
        else v = pf[p];
        *(U4*)(buf + loff[p]) = v;
      }
    }
  }
};

// lanes 0-31: the value of lane + 32 (v_permlane32_swap, one VALU op instead of an LDS-routed
// ds_bpermute per __shfl_xor(v, 32)); lanes 32-63 keep their own value
PTG_DEV float hi_half(float v) {
  return __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false)[1]);
}
// v_permlane32_swap(a, b): lanes 32-63 of a trade places with lanes 0-31 of b, so
//   lo = lanes < 32: own a,           lanes >= 32: b of lane - 32
//   hi = lanes < 32: a of lane + 32,  lanes >= 32: own b
PTG_DEV void swap32(float a, float b, float& lo, float& hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  lo = __uint_as_float(r[0]);
  hi = __uint_as_float(r[1]);
}

template <bool U8, int PD>
__global__ __launch_bounds__(256, PD == 1 ? 5 : 4) void conv1_fwd_rec_k(const void* __restrict__ x, const bf16_t* __restrict__ w,
                                                       const float* __restrict__ bias, const float* __restrict__ alpha,
                                                       bf16_t* __restrict__ pooled, bf16_t* __restrict__ zsel,
                                                       uint8_t* __restrict__ argq, int N, int H, int W, int tiles_h,
                                                       int tiles_w, int nchunks) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[WZS + 8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int px = lane & 15, g = lane >> 4, hf = wid & 1, rp = wid >> 1;
  if (tid < 8) smem[WZS + tid] = 0;
  __syncthreads();
  const Item it = work_item(N, tiles_h, tiles_w, nchunks);
  if (it.n0 >= it.n1) return;
  bf16_t* const wr = smem + wid * WREG;
  bf16x8_t wreg[KSTEPS];
  load_wreg(w, px, g, wreg);
  const int cc = 4 * (g & 1), dwo = g >> 1;
  constexpr float XS = U8 ? 1.f / 255.f : 1.f;  // integer pixels: z = acc / 255 + bias
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias) { const float4 b4 = *(const float4*)(bias + cc); bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w; }
  const int ow = it.ow0 + hf * WTW + 2 * px + dwo;
  float al[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oh = it.oh0 + 2 * rp + i;
    const float4 a = (oh < H && ow < W) ? *(const float4*)(alpha + ((long)oh * W + ow) * COUT + cc)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
    al[i][0] = a.x; al[i][1] = a.y; al[i][2] = a.z; al[i][3] = a.w;
  }
  const int PH = H >> 1, PW = W >> 1;
  const int ph = (it.oh0 >> 1) + rp, pw = (it.ow0 >> 1) + hf * 16 + px;
  const bool store_lane = ph < PH && pw < PW;
  // the lane's 2 pooled channels after the window exchange: 4 * (g & 1) + 2 * (g >> 1) + {0, 1}
  const long pstep = (long)PH * PW * COUT, pbase = ((long)ph * PW + pw) * COUT + cc + 2 * (g >> 1);
  const Rsrc xr = x_rsrc<U8>(x, N, H, W);
  const uint32_t img_bytes = (uint32_t)(H * W) * (U8 ? 3u : 8u);
  int boff[KSTEPS];
  conv_boffs(px, g, boff);
  WaveHaloR<U8> hl;
  hl.init(H, W, it.oh0 + 2 * rp - PAD, it.ow0 + hf * WTW - PAD, lane);
  // register prefetch ring: sample s lives in ring[(s - n0) % PD] from its load until it is copied
  // to the LDS double buffer, so PD samples' halos are in flight while one computes (the step is
  // bound by loads in flight per CU, not by the MFMAs: 4 waves x 864 B per SIMD at PD = 1)
  HaloSlot<U8> ring[PD];
#pragma unroll
  for (int u = 0; u < PD; ++u)
    if (it.n0 + u < it.n1) hl.load_to(ring[u], xr, img_bytes, it.n0 + u);
  hl.store_from(ring[0], wr);
  wave_lds_sync();
  if (it.n0 + PD < it.n1) hl.load_to(ring[0], xr, img_bytes, it.n0 + PD);
  for (int nb = it.n0; nb < it.n1; nb += PD)
#pragma unroll
  for (int u = 0; u < PD; ++u) {
    const int n = nb + u;
    if (n >= it.n1) break;
    const int b = (n - it.n0) & 1;
    const bool has_next = n + 1 < it.n1;
    f32x4_t acc[2];
    conv_tile_r(wr + b * WHB, boff, wreg, acc);
    float zv[2][4], yv[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        zv[i][r] = bf2f(f2bf(fmaf(acc[i][r], XS, bv[r])));
        yv[i][r] = zv[i][r] > 0.f ? zv[i][r] : al[i][r] * zv[i][r];
      }
    // 2x2 windows: lane l < 32 holds the dw = 0 pixel, lane l + 32 the dw = 1 pixel of the same
    // pooled column, 4 channels each.  One v_permlane32_swap per (r, r + 2) pair leaves every lane
    // with BOTH columns of 2 channels - lanes < 32 channels r = 0, 1, lanes >= 32 channels 2, 3 - in
    // (dw 0, dw 1) order, so all 64 lanes pool 2 windows (no half-wave of discarded pool math)
    float pm[2], zs[2];
    uint32_t qs = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float y0[2], y1[2], z0[2], z1[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        swap32(yv[i][k], yv[i][k + 2], y0[i], y1[i]);
        swap32(zv[i][k], zv[i][k + 2], z0[i], z1[i]);
      }
      const float yq[4] = {y0[0], y1[0], y0[1], y1[1]};  // q = 2*dh + dw
      const float zq[4] = {z0[0], z1[0], z0[1], z1[1]};
      float bm = yq[0], bz = zq[0];
      uint32_t a = 0;
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (yq[q] > bm) { bm = yq[q]; bz = zq[q]; a = q; }  // first maximum in q order
      pm[k] = bm;
      zs[k] = bz;
      qs |= a << (8 * k);
    }
    // the next halo goes to LDS BEFORE this sample's global stores: vmcnt counts loads and stores
    // in issue order, so waiting for the prefetch behind (conditional) stores waited for their
    // write acknowledgements too (s_waitcnt vmcnt(0) each sample)
    if (has_next) {
      hl.store_from(ring[(u + 1) % PD], wr + (b ^ 1) * WHB);
      wave_lds_sync();
      if (n + 1 + PD < it.n1) hl.load_to(ring[(u + 1) % PD], xr, img_bytes, n + 1 + PD);
    }
    if (store_lane) {
      const long po = (long)n * pstep + pbase;
      *(uint32_t*)(pooled + po) = pack_bf(pm[0], pm[1]);
      *(uint32_t*)(zsel + po) = pack_bf(zs[0], zs[1]);
      *(uint16_t*)(argq + po) = (uint16_t)qs;
    }
  }
}

template <bool U8>
__global__ __launch_bounds__(256, 4) void conv1_bwd_rec_k(const void* __restrict__ x, const float* __restrict__ alpha,
                                                       const bf16_t* __restrict__ dp, const bf16_t* __restrict__ zsel,
                                                       const uint8_t* __restrict__ argq, float* __restrict__ dw,
                                                       float* __restrict__ dalpha, float* __restrict__ dbias, int N,
                                                       int H, int W, int tiles_h, int tiles_w, int nchunks) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[WZS + 8];
  __shared__ float2 sda[4][4][64];  // dalpha partials: [wave][window position q][lane] (2 channels)
  __shared__ float sdb[4][COUT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hf = wid & 1, rp = wid >> 1;
  const int g = lane >> 4, li = lane & 15;
  // record lane: pooled column pc of the wave's 16, channels 2*c2, 2*c2 + 1
  const int pc = lane & 15, c2 = lane >> 4;
  if (tid < 8) smem[WZS + tid] = 0;
  bf16_t* const wr = smem + wid * WREG;
  bf16_t* const ds = wr + 2 * WHB;
  for (int i = lane; i < WDZ / 8; i += 64) *(U4*)(ds + 8 * i) = zero4();  // MFMA rows 8-15 read 0
#pragma unroll
  for (int q = 0; q < 4; ++q) sda[wid][q][lane] = make_float2(0.f, 0.f);
  __syncthreads();
  const Item it = work_item(N, tiles_h, tiles_w, nchunks);
  if (it.n0 >= it.n1) return;
  const int PH = H >> 1, PW = W >> 1;
  const int ph = (it.oh0 >> 1) + rp, pw = (it.ow0 >> 1) + hf * 16 + pc;
  const bool pin = ph < PH && pw < PW;
  // alpha of the lane's 2 channels at the 4 window pixels
  float2 al[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int oh = 2 * ph + (q >> 1), ow = 2 * pw + (q & 1);
    al[q] = pin ? *(const float2*)(alpha + ((long)oh * W + ow) * COUT + 2 * c2) : make_float2(0.f, 0.f);
  }
  const Rsrc xr = x_rsrc<U8>(x, N, H, W);
  const uint32_t img_bytes = (uint32_t)(H * W) * (U8 ? 3u : 8u);
  const uint32_t rec_elems = (uint32_t)(N * PH * PW * COUT);
  const Rsrc dr = make_rsrc(dp, rec_elems * 2u), zr_ = make_rsrc(zsel, rec_elems * 2u), qr = make_rsrc(argq, rec_elems);
  const uint32_t roff = (uint32_t)((ph * PW + pw) * COUT + 2 * c2), rstep = (uint32_t)(PH * PW * COUT);
  auto rec_load = [&](int n, uint32_t& gw, uint32_t& zw, uint32_t& qw) {
    const uint32_t o = pin ? (uint32_t)n * rstep + roff : PTG_OOB / 2;  // element index (PTG_OOB/2 * 2 = OOB bytes)
    gw = bload4(dr, pin ? 2u * o : PTG_OOB);
    zw = bload4(zr_, pin ? 2u * o : PTG_OOB);
    qw = __builtin_amdgcn_raw_buffer_load_b16(qr, pin ? o : PTG_OOB, 0, 0);
  };
  f32x4_t wacc[WNB];
#pragma unroll
  for (int j = 0; j < WNB; ++j) wacc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float db[2] = {0.f, 0.f};
  // weight-gradient operand offsets (sample-invariant): the A (dZ) rows of the lane's two pixels per
  // k-step, the halo pixel of those rows, and the B column base (kh, kw) of each 16-column fragment
  // (columns past KF read any finite halo element: their outputs are never flushed)
  const int q4 = (lane & 15) >> 2, p4 = lane & 3;
  int aoff[2][2], hoff[2][2], bcol[WNB];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = k * 32 + 8 * g + q4 + 4 * h;
      aoff[k][h] = m * DPITCH + 4 * p4;
      hoff[k][h] = (m / WTW) * WROWE + (m % WTW) * C;
    }
#pragma unroll
  for (int jj = 0; jj < WNB; ++jj) {
    const int kf = jj * 16 + 4 * p4;
    const int kh = kf / (KS * C), kw = (kf - kh * KS * C) / C;
    bcol[jj] = kf < KF ? kh * WROWE + kw * C : 0;
  }
  WaveHaloR<U8> hl;
  hl.init(H, W, it.oh0 + 2 * rp - PAD, it.ow0 + hf * WTW - PAD, lane);
  hl.load(xr, img_bytes, it.n0);
  uint32_t gn, zn, qn;
  rec_load(it.n0, gn, zn, qn);
  hl.store(wr);
  wave_lds_sync();
  for (int n = it.n0; n < it.n1; ++n) {
    const int b = (n - it.n0) & 1;
    const bf16_t* hb = wr + b * WHB;
    const bool has_next = n + 1 < it.n1;
    const uint32_t gw = gn, zw = zn, qw = qn;
    if (has_next) {
      hl.load(xr, img_bytes, n + 1);
      rec_load(n + 1, gn, zn, qn);
    }
    // dZ at each window's argmax for the lane's 2 channels, zero at the other 3 pixels
    uint32_t dzw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      const float gv = ch ? hi_bf(gw) : lo_bf(gw);
      const float zv = ch ? hi_bf(zw) : lo_bf(zw);
      const int q = (qw >> (8 * ch)) & 3;
      const float a = q == 0 ? (ch ? al[0].y : al[0].x) : q == 1 ? (ch ? al[1].y : al[1].x)
                    : q == 2 ? (ch ? al[2].y : al[2].x) : (ch ? al[3].y : al[3].x);
      const bool pos = zv > 0.f;
      const float d = pos ? gv : gv * a;
      db[ch] += d;
      if (!pos && gv != 0.f) {  // dalpha at the argmax pixel (lane-private LDS slot)
        float2* sp = &sda[wid][q][lane];
        if (ch) sp->y += gv * zv; else sp->x += gv * zv;
      }
      const uint32_t dbits = (uint32_t)f2bf(d) << (16 * ch);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) dzw[qq] |= q == qq ? dbits : 0u;
    }
    // pixel (dh, dw) of pooled column pc is wave pixel m = dh*32 + 2*pc + dw
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
      *(uint32_t*)(ds + ((qq >> 1) * WTW + 2 * pc + (qq & 1)) * DPITCH + 2 * c2) = dzw[qq];
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const s16x4_t alo = tr_read(ds + aoff[k][0]);
      const s16x4_t ahi = tr_read(ds + aoff[k][1]);
      U2 ua = __builtin_bit_cast(U2, alo), ub = __builtin_bit_cast(U2, ahi);
      const bf16x8_t af = __builtin_bit_cast(bf16x8_t, U4{ua.x, ua.y, ub.x, ub.y});
      const bf16_t* h0 = hb + hoff[k][0];
      const bf16_t* h1 = hb + hoff[k][1];
#pragma unroll
      for (int jj = 0; jj < WNB; ++jj) {
        const s16x4_t blo = tr_read(h0 + bcol[jj]), bhi = tr_read(h1 + bcol[jj]);
        ua = __builtin_bit_cast(U2, blo);
        ub = __builtin_bit_cast(U2, bhi);
        wacc[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8_t, U4{ua.x, ua.y, ub.x, ub.y}),
                                                           wacc[jj], 0, 0, 0);
      }
    }
    if (has_next) hl.store(wr + (b ^ 1) * WHB);
    wave_lds_sync();  // next halo visible; this dZ tile read before it is rewritten
  }
  // dalpha (each (pixel, channel) of the tile belongs to exactly one lane and window position)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float2 t = sda[wid][q][lane];
    const long o = ((long)(2 * ph + (q >> 1)) * W + 2 * pw + (q & 1)) * COUT + 2 * c2;
    if (pin) {
      if (t.x != 0.f) atomicAdd(dalpha + o, t.x);
      if (t.y != 0.f) atomicAdd(dalpha + o + 1, t.y);
    }
  }
  // dbias: the 16 pooled columns of a channel pair, then the waves
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    float v = db[ch];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    db[ch] = v;
  }
  if (pc == 0) { sdb[wid][2 * c2] = db[0]; sdb[wid][2 * c2 + 1] = db[1]; }
  __syncthreads();
  constexpr float XS = U8 ? 1.f / 255.f : 1.f;  // integer pixels in the halo: dW = sum / 255
  float* red = reinterpret_cast<float*>(smem);
  if (g < 2) {
#pragma unroll
    for (int j = 0; j < WNB; ++j) {
      const int kf = j * 16 + li;
      if (kf < KF) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wid * COUT * KF + (g * 4 + r) * KF + kf] = wacc[j][r];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < COUT * KF; i += 256)
    atomicAdd(dw + i, XS * (red[i] + red[COUT * KF + i] + red[2 * COUT * KF + i] + red[3 * COUT * KF + i]));
  if (tid < COUT) atomicAdd(dbias + tid, sdb[0][tid] + sdb[1][tid] + sdb[2][tid] + sdb[3][tid]);
}

// sample chunks per tile position: as many work items as fit the device at once (one wave of
// workgroups, no tail), or PTG_CONV1_*_PER_CU workgroups per CU when set
// PTG_CONV1_WAVE=0: the block-synchronised sample loop (A/B)
static bool conv1_wave() {
  static const bool on = [] {
    const char* e = getenv("PTG_CONV1_WAVE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// samples in flight per wave in the record forward (PTG_CONV1_PD = 1 or 2).  Measured at b256
// (rocprof, kernel us in the step): PD 1 148.5, 2 146.7, 3 167.6, 4 167.6 - the extra ring registers
// cost occupancy (3 waves per SIMD at PD >= 3) and the kernel is issue-bound, not load-latency-bound,
// so PD 1 at 5 waves per SIMD (launch bounds) is the default.
static int conv1_pd() {
  static const int pd = [] {
    const char* e = getenv("PTG_CONV1_PD");
    const int v = e ? atoi(e) : 1;
    return v < 1 ? 1 : v > 2 ? 2 : v;
  }();
  return pd;
}

static int conv1_chunks(int N, long npos, const void* kern, const char* env) {
  long slots = ptg_resident_blocks(kern);
  if (const char* e = getenv(env)) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (cus <= 0) cus = 256;
    }
    if (atoi(e) > 0) slots = (long)cus * atoi(e);
  }
  long c = slots / npos;
  if (c > N) c = N;
  return (int)(c < 1 ? 1 : c);
}

}  // namespace ptgc1

using namespace ptgc1;

extern "C" {

// pooled [N][H/2][W/2][8] = maxpool2x2(prelu(conv5x5(x) + bias, alpha)); x is the raw uint8
// [N][H][W][3] image batch (u8 = 1) or bf16 [N][H][W][4]; w bf16 [8][5][5][4]; alpha fp32 [H][W][8].
int ptg_conv1_fwd_pm(const void* x, int u8, const void* w, const float* bias, const float* alpha, void* pooled, int N,
                     int H, int W, hipStream_t s) {
  if ((H & 1) || (W & 1) || N <= 0 || !ptg_fits_2g((long)N * H * W * (u8 ? 3 : 8)) ||
      !ptg_fits_2g((long)N * H * W * 4))
    return (int)hipErrorInvalidValue;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const auto kern = conv1_wave() ? (u8 ? conv1_fwd_wv_k<true> : conv1_fwd_wv_k<false>)
                                  : (u8 ? conv1_fwd_pm_k<true> : conv1_fwd_pm_k<false>);
  const int nch = conv1_chunks(N, (long)th * tw, (const void*)kern, "PTG_CONV1_FWD_PER_CU");
  const long items = (long)th * tw * nch;
  if (items > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(256), 0, s, x, (const bf16_t*)w, bias, alpha, (bf16_t*)pooled,
                     N, H, W, th, tw, nch);
  PTG_RETURN_LAUNCH();
}

// Backward of ptg_conv1_fwd_pm from the pooled gradient dp [N][H/2][W/2][8] (bf16): accumulates
// (atomically, onto zeroed buffers) dw fp32 [8][5][5][4], dalpha fp32 [H][W][8], dbias fp32 [8].
int ptg_conv1_bwd_pm(const void* x, int u8, const void* w, const float* bias, const float* alpha, const void* dp,
                     float* dw, float* dalpha, float* dbias, int N, int H, int W, hipStream_t s) {
  if ((H & 1) || (W & 1) || N <= 0 || !ptg_fits_2g((long)N * H * W * (u8 ? 3 : 8)) ||
      !ptg_fits_2g((long)N * H * W * 4))
    return (int)hipErrorInvalidValue;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const auto kern = conv1_wave() ? (u8 ? conv1_bwd_wv_k<true> : conv1_bwd_wv_k<false>)
                                  : (u8 ? conv1_bwd_pm_k<true> : conv1_bwd_pm_k<false>);
  const int nch = conv1_chunks(N, (long)th * tw, (const void*)kern, "PTG_CONV1_BWD_PER_CU");
  const long items = (long)th * tw * nch;
  if (items > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(256), 0, s, x, (const bf16_t*)w, bias, alpha,
                     (const bf16_t*)dp, dw, dalpha, dbias, N, H, W, th, tw, nch);
  PTG_RETURN_LAUNCH();
}

// Record pipeline: forward writes pooled, zsel (bf16 z at each window's argmax) and argq (uint8
// argmax q = 2*dh + dw), all [N][H/2][W/2][8]; the backward reads them with x and the pooled gradient.
int ptg_conv1_fwd_rec(const void* x, int u8, const void* w, const float* bias, const float* alpha, void* pooled,
                      void* zsel, void* argq, int N, int H, int W, hipStream_t s) {
  if ((H & 1) || (W & 1) || N <= 0 || !ptg_fits_2g((long)N * H * W * (u8 ? 3 : 8)) ||
      !ptg_fits_2g((long)N * H * W * 4))
    return (int)hipErrorInvalidValue;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const int pd = conv1_pd();
  const auto kern = pd >= 2 ? (u8 ? conv1_fwd_rec_k<true, 2> : conv1_fwd_rec_k<false, 2>)
                            : (u8 ? conv1_fwd_rec_k<true, 1> : conv1_fwd_rec_k<false, 1>);
  const int nch = conv1_chunks(N, (long)th * tw, (const void*)kern, "PTG_CONV1_FWD_PER_CU");
  const long items = (long)th * tw * nch;
  if (items > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(256), 0, s, x, (const bf16_t*)w, bias, alpha, (bf16_t*)pooled,
                     (bf16_t*)zsel, (uint8_t*)argq, N, H, W, th, tw, nch);
  PTG_RETURN_LAUNCH();
}

int ptg_conv1_bwd_rec(const void* x, int u8, const float* alpha, const void* dp, const void* zsel, const void* argq,
                      float* dw, float* dalpha, float* dbias, int N, int H, int W, hipStream_t s) {
  if ((H & 1) || (W & 1) || N <= 0 || !ptg_fits_2g((long)N * H * W * (u8 ? 3 : 8)) ||
      !ptg_fits_2g((long)N * H * W * 4))
    return (int)hipErrorInvalidValue;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const auto kern = u8 ? conv1_bwd_rec_k<true> : conv1_bwd_rec_k<false>;
  const int nch = conv1_chunks(N, (long)th * tw, (const void*)kern, "PTG_CONV1_BWD_PER_CU");
  const long items = (long)th * tw * nch;
  if (items > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(256), 0, s, x, alpha, (const bf16_t*)dp, (const bf16_t*)zsel,
                     (const uint8_t*)argq, dw, dalpha, dbias, N, H, W, th, tw, nch);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"

PTG_CHECK_STATUS(conv1)
