// 5x5 'same' convolution (stride 1) as an implicit GEMM on v_mfma_f32_32x32x16_bf16, for the
// channel-rich CNN-B1 layers (train_tf_ps.py:357-364: Conv2D 16->32 @64x80, 32->64 @32x40,
// 64->64 @16x20, and their data gradients 32->16, 64->32, 64->64).
//
// Why a second conv kernel: the halo strip kernels of conv.hip run these layers at 7-19 % of the
// MFMA peak (profiles/r4_cnn_b1_roofline_overlapped_start.txt).  Their 16x16x32 fragments read
// 1 KB of LDS per 16 KFLOP MFMA and the C=64 variants wait on per-k-step weight loads from L2.
// Here every wave owns a 32x32 MFMA tile pair: a 32x32x16 MFMA does 32 KFLOP per 1 KB fragment
// read, each pixel fragment (LDS) feeds every output-channel block and each weight fragment
// (registers, prefetched PF k-steps ahead) feeds both pixel blocks.
//
// Tiling: a workgroup owns TR full image rows of one sample (TR * W = 320 pixels = 10 blocks of 32)
// and all output channels (CO = 32 or 64, one or two 32-row blocks); 5 waves x 2 pixel blocks.
// D[co][px] orientation: A = filter rows (32 co x 16 k from W[co][kh][kw][ci..]), B = the halo
// (16 k = 16 channels of the input pixel shifted by (kh, kw)), so the K loop is (kh, kw, 16-channel
// block) with no im2col and no padding waste for C % 16 == 0.  The input rows [r0-2, r0+TR+2) of the
// sample are staged in LDS once (zeros outside the image) with a pixel pitch of C + 8 elements: 16-byte
// reads of 32 consecutive pixels then spread over the banks.
//
// Epilogue through LDS (the halo buffer is free after the K loop): the accumulators are rounded to
// bf16 (+ bias) into a [pixel][channel] tile, then 16-byte chunks are written coalesced:
//   EPI_Z     z                         (data gradient / plain conv)
//   EPI_POOL  z, and maxpool2x2(prelu(z)) with per-element alphas    (conv + PReLU + MaxPool)
//   EPI_PRELU z, and prelu(z)                                          (conv + PReLU, last block)
// PReLU is applied to the bf16-rounded z, as the backward recomputes it.
#include "common.h"

namespace ptgm32 {

constexpr int NW = 5, NT = NW * 64, KS = 5, PAD = 2;
// PTG_C32_WLDS=1: the filter taps are staged in LDS once per workgroup, one (kh, kw) slice of
// [CO][CHP] at a time (double-buffered, the next slice's global loads in flight while this one
// computes), instead of every wave fetching its weight fragments from L2 each k-step (5x the L2
// traffic of the taps: ~1 MB per 320-pixel tile at C = CO = 64).  On by default since round 4 for
// the big slices (see launch()): CNN-B1 b256 1.650 -> 1.601 ms per step (profiles/r4_ab_conv32_wlds.txt);
// =0 for the A/B.
#ifndef PTG_C32_WLDS
#define PTG_C32_WLDS 1
#endif
constexpr bool WLDS = PTG_C32_WLDS != 0;
template <int CHP, int CO>
constexpr int wslice_elems() { return CO * (CHP + 8); }  // one (kh, kw) slice, row pitch CHP + 8
enum { EPI_Z = 0, EPI_POOL = 1, EPI_PRELU = 2 };

// Occupancy knobs (round 6).  With the whole C = 64 halo of a 320-pixel tile in LDS (76-87 KB) the
// C = 64 layers ran ONE 5-wave workgroup per CU, and the 16x20 layer only 256 workgroups in all:
//  * CHP (channels per halo pass): the K loop runs in C / CHP passes over channel slices, the halo
//    restaged per pass (pitch CHP + 8), so a C = 64 tile needs ~40 KB and three workgroups share a CU;
//  * PB (32-pixel blocks per wave): 2 = 320-pixel tiles (as before), 1 = 160-pixel tiles, twice the
//    workgroups (L5's 16x20 images then split into two 8-row tiles).
template <int C, int CO, int EPI, bool WL, int CHP, int PB>
__global__ __launch_bounds__(NT) void conv32_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                               const float* __restrict__ bias, const float* __restrict__ alpha,
                                               bf16_t* __restrict__ z, bf16_t* __restrict__ aux, int H, int W,
                                               int TR, int Cout) {
  static_assert(C % CHP == 0 && CHP % 16 == 0, "channel passes of 16-channel blocks");
  constexpr int PX = NW * 32 * PB;      // pixels per tile
  constexpr int NPASS = C / CHP;
  constexpr int CP = CHP + 8;           // LDS pixel pitch (elements): an odd multiple of 16 bytes
  constexpr int NCO = CO / 32;          // output-channel blocks
  constexpr int CB = CHP / 16;          // 16-channel K blocks per (kh, kw) and pass
  constexpr int KSTEPS = KS * KS * CB;  // per pass
  constexpr int PF = 4;                 // weight fragments prefetched ahead (k-steps)
  constexpr int SP = CO + 8;            // epilogue staging pitch (elements)
  extern __shared__ __align__(16) bf16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tiles_per_img = H / TR;
  const int n = blockIdx.x / tiles_per_img, r0 = (blockIdx.x - n * tiles_per_img) * TR;
  const int HR = TR + KS - 1, HC = W + KS - 1;
  const bf16_t* img = x + (long)n * H * W * C;
  // ---- stage the halo rows [r0-2, r0+TR+2) x [-2, W+2) x channels [c0, c0 + CHP) ----
  auto stage_halo = [&](int c0) {
    constexpr int V = CHP / 8;  // 16-byte vectors per pixel
    const int total = HR * HC * V;
    for (int t = tid; t < total; t += NT) {
      const int pix = t / V, v = t - pix * V;
      const int hr = pix / HC, hc = pix - hr * HC;
      const int ih = r0 - PAD + hr, iw = hc - PAD;
      U4 val = zero4();
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        val = *(const U4*)(img + ((long)ih * W + iw) * C + c0 + v * 8);
      *(U4*)(lds + pix * CP + v * 8) = val;
    }
  };
  // this lane's pixel in each of its PB blocks: tile pixel p = 32*PB*wv + 32*b + r, (row, col) in the tile
  int hbase[PB];
#pragma unroll
  for (int b = 0; b < PB; ++b) {
    const int p = 32 * PB * wv + 32 * b + r;
    const int pr = p / W, pc = p - pr * W;
    hbase[b] = (pr * HC + pc) * CP + 8 * h;
  }
  f32x16_t acc[NCO][PB];
#pragma unroll
  for (int j = 0; j < NCO; ++j)
#pragma unroll
    for (int b = 0; b < PB; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[j][b][i] = 0.f;
  for (int cp = 0; cp < NPASS; ++cp) {
    const int c0 = cp * CHP;
    if (cp > 0) __syncthreads();  // every wave is done reading the previous pass's halo / taps
    stage_halo(c0);
    if constexpr (WL) {
      // ---- taps from LDS: slice khw = W[0..CO)[kh][kw][c0..c0+CHP) at lds + halo_elems + (khw & 1) * WSL ----
      constexpr int WP = CHP + 8, WSL = wslice_elems<CHP, CO>(), WV = CO * CHP / 8;  // 16-byte vectors per slice
      constexpr int WPT = (WV + NT - 1) / NT;
      bf16_t* wbuf = lds + HR * HC * CP;
      U4 wreg[WPT];
      auto wfetch = [&](int khw) {  // this thread's part of slice khw into registers (zeros past Cout)
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
          const int t = tid + q * NT;
          U4 v = zero4();
          if (t < WV) {
            const int co = t / (CHP / 8), cv = t - co * (CHP / 8);
            if (co < Cout) v = *(const U4*)(w + ((long)co * KS * KS + khw) * C + c0 + cv * 8);
          }
          wreg[q] = v;
        }
      };
      auto wstore = [&](int khw) {
        bf16_t* dst = wbuf + (khw & 1) * WSL;
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
          const int t = tid + q * NT;
          if (t < WV) {
            const int co = t / (CHP / 8), cv = t - co * (CHP / 8);
            *(U4*)(dst + co * WP + cv * 8) = wreg[q];
          }
        }
      };
      wfetch(0);
      wstore(0);
      __syncthreads();  // halo + slice 0 staged
      for (int khw = 0; khw < KS * KS; ++khw) {
        if (khw + 1 < KS * KS) wfetch(khw + 1);  // global loads in flight under this slice's MFMAs
        const int kh = khw / KS, kw = khw - kh * KS;
        const bf16_t* ws = wbuf + (khw & 1) * WSL;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          const int koff = (kh * HC + kw) * CP + cb * 16;
          bf16x8_t wa[NCO];
#pragma unroll
          for (int j = 0; j < NCO; ++j) wa[j] = *(const bf16x8_t*)(ws + (32 * j + r) * WP + cb * 16 + 8 * h);
#pragma unroll
          for (int b = 0; b < PB; ++b) {
            const bf16x8_t xb = *(const bf16x8_t*)(lds + hbase[b] + koff);
#pragma unroll
            for (int j = 0; j < NCO; ++j)
              acc[j][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[j], xb, acc[j][b], 0, 0, 0);
          }
        }
        if (khw + 1 < KS * KS) {
          wstore(khw + 1);  // the other buffer: last read in iteration khw - 1, before the barrier below
          __syncthreads();
        }
      }
    } else {
      // weight fragments: W[co][kh][kw][C], lane (co = r (+32), k = 8h..8h+7 of the 16-channel block)
      const bf16_t* wl[NCO];
#pragma unroll
      for (int j = 0; j < NCO; ++j) {
        const int co = 32 * j + r;
        wl[j] = w + (long)(co < Cout ? co : 0) * KS * KS * C + c0 + 8 * h;
      }
      const bool co_ok0 = r < Cout, co_ok1 = 32 + r < Cout;
      auto wload = [&](int ks, int j) -> bf16x8_t {
        const int khw = ks / CB, cb = ks - khw * CB;
        const bool ok = j == 0 ? co_ok0 : co_ok1;
        U4 v = zero4();
        if (ok) v = *(const U4*)(wl[j] + khw * C + cb * 16);
        return __builtin_bit_cast(bf16x8_t, v);
      };
      bf16x8_t wq[PF][NCO];
#pragma unroll
      for (int s = 0; s < PF; ++s)
#pragma unroll
        for (int j = 0; j < NCO; ++j) wq[s][j] = wload(s, j);
      __syncthreads();
      // ---- K loop: (kh, kw, 16-channel block) ----
#pragma unroll PF
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const int slot = ks % PF;
        bf16x8_t wa[NCO];
#pragma unroll
        for (int j = 0; j < NCO; ++j) wa[j] = wq[slot][j];
        if (ks + PF < KSTEPS) {
#pragma unroll
          for (int j = 0; j < NCO; ++j) wq[slot][j] = wload(ks + PF, j);
        }
        const int khw = ks / CB, cb = ks - khw * CB;
        const int kh = khw / KS, kw = khw - kh * KS;
        const int koff = (kh * HC + kw) * CP + cb * 16;
#pragma unroll
        for (int b = 0; b < PB; ++b) {
          const bf16x8_t xb = *(const bf16x8_t*)(lds + hbase[b] + koff);
#pragma unroll
          for (int j = 0; j < NCO; ++j) acc[j][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[j], xb, acc[j][b], 0, 0, 0);
        }
      }
    }
  }
  __syncthreads();  // halo reads done: the buffer becomes the epilogue staging tile
  // ---- stage bf16(acc + bias) as [pixel][channel] ----
#pragma unroll
  for (int j = 0; j < NCO; ++j) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int co = 32 * j + 8 * g + 4 * h;
      float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bias && co < Cout) bb = *(const float4*)(bias + co);
#pragma unroll
      for (int b = 0; b < PB; ++b) {
        const int p = 32 * PB * wv + 32 * b + r;
        U2 v;
        v.x = pack_bf(acc[j][b][4 * g + 0] + bb.x, acc[j][b][4 * g + 1] + bb.y);
        v.y = pack_bf(acc[j][b][4 * g + 2] + bb.z, acc[j][b][4 * g + 3] + bb.w);
        *(U2*)(lds + p * SP + co) = v;
      }
    }
  }
  __syncthreads();
  // ---- coalesced stores: 16-byte chunks of 8 channels ----
  const int cv_n = Cout / 8;
  const long zimg = ((long)n * H + r0) * W * Cout;
  if constexpr (EPI != EPI_POOL) {
    for (int t = tid; t < PX * cv_n; t += NT) {
      const int p = t / cv_n, v = t - p * cv_n;
      const U4 val = *(const U4*)(lds + p * SP + v * 8);
      *(U4*)(z + zimg + (long)p * Cout + v * 8) = val;
      if constexpr (EPI == EPI_PRELU) {
        const long ae = ((long)r0 * W + p) * Cout + v * 8;
        const float4 a0 = *(const float4*)(alpha + ae), a1 = *(const float4*)(alpha + ae + 4);
        float f[8];
        unpack8(val, f);
        const float al[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) f[q] = f[q] > 0.f ? f[q] : al[q] * f[q];
        *(U4*)(aux + zimg + (long)p * Cout + v * 8) = pack8(f);
      }
    }
  } else {
    // z for every pixel, and one pooled pixel per (2x2 window, 8 channels)
    for (int t = tid; t < PX * cv_n; t += NT) {
      const int p = t / cv_n, v = t - p * cv_n;
      *(U4*)(z + zimg + (long)p * Cout + v * 8) = *(const U4*)(lds + p * SP + v * 8);
    }
    const int PW = W / 2, npool = (TR / 2) * PW;
    for (int t = tid; t < npool * cv_n; t += NT) {
      const int q = t / cv_n, v = t - q * cv_n;
      const int pr = q / PW, pc = q - pr * PW;
      float best[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) best[k] = -INFINITY;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int rr = 2 * pr + (d >> 1), cc = 2 * pc + (d & 1);
        const int p = rr * W + cc;
        float f[8];
        unpack8(*(const U4*)(lds + p * SP + v * 8), f);
        const long ae = ((long)(r0 + rr) * W + cc) * Cout + v * 8;
        const float4 a0 = *(const float4*)(alpha + ae), a1 = *(const float4*)(alpha + ae + 4);
        const float al[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float y = f[k] > 0.f ? f[k] : al[k] * f[k];
          best[k] = fmaxf(best[k], y);
        }
      }
      const long po = (((long)n * (H / 2) + r0 / 2 + pr) * PW + pc) * Cout + v * 8;
      *(U4*)(aux + po) = pack8(best);
    }
  }
}

template <int C, int CO, int EPI, bool WL, int CHP, int PB>
static int launch_k(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N,
                    int H, int W, int Cout, long bytes, hipStream_t s) {
  const int TR = NW * 32 * PB / W;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv32_k<C, CO, EPI, WL, CHP, PB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((conv32_k<C, CO, EPI, WL, CHP, PB>), dim3(N * (H / TR)), dim3(NT), (size_t)bytes, s,
                     (const bf16_t*)x, (const bf16_t*)w, bias, alpha, (bf16_t*)z, (bf16_t*)aux, H, W, TR, Cout);
  return (int)hipGetLastError();
}

template <int C, int CO, int EPI, int CHP, int PB>
static long lds_bytes(int W) {
  constexpr bool wl = WLDS && C * CO >= 2048;
  const int TR = NW * 32 * PB / W;
  constexpr int CP = CHP + 8, SP = CO + 8;
  const long halo = (long)(TR + KS - 1) * (W + KS - 1) * CP * 2 + (wl ? 2L * wslice_elems<CHP, CO>() * 2 : 0L);
  const long stage = (long)NW * 32 * PB * SP * 2;
  return halo > stage ? halo : stage;
}

// The LDS-staged taps pay where a (kh, kw) slice is big (C * CO >= 2048: L4 / L5 of CNN-B1, fwd 69 ->
// 61 and 40 -> 30 us, dgrad 74 -> 68 and 36 -> 26 us); with smaller slices the L2 fragment loads are
// cheap and the extra LDS / barriers lost (fwd 64 -> 72, dgrads 92 -> 98 and 175 -> 208 us).
template <int C, int CO, int EPI, int CHP, int PB>
static int launch_t(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N,
                    int H, int W, int Cout, hipStream_t s) {
  constexpr bool wl = WLDS && C * CO >= 2048;
  const long bytes = lds_bytes<C, CO, EPI, CHP, PB>(W);
  if (bytes > 160 * 1024) return (int)hipErrorInvalidValue;
  return launch_k<C, CO, EPI, wl, CHP, PB>(x, w, bias, alpha, z, aux, N, H, W, Cout, bytes, s);
}

// tile choice: PTG_C32_SPLIT (env, read once) = 0 keeps the round-5 tiles (whole-C halo, 320 pixels);
// 1 (default) takes half-channel passes for C = 64 and 160-pixel tiles where 320-pixel tiles leave
// the GPU with at most one workgroup per CU
static int c32_mode() {
  static int m = -1;
  if (m < 0) {
    const char* e = getenv("PTG_C32_SPLIT");
    m = e && *e ? atoi(e) : 1;
  }
  return m;
}

template <int C, int CO, int EPI>
static int launch(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N, int H,
                  int W, int Cout, hipStream_t s) {
  const int mode = c32_mode();
  constexpr int CH2 = C >= 64 ? C / 2 : C;
  // 160-pixel tiles when the 320-pixel grid would not give every CU two workgroups
  // (PTG_C32_SPLIT=2: 160-pixel tiles at every grid size, A/B)
  const bool small = mode != 0 && (320 / (W > 0 ? W : 1)) > 0 && (mode == 2 || (long)N * (H / (320 / W)) < 512) &&
                     W <= 160 && 160 % W == 0 && H % (160 / W) == 0 && (EPI != EPI_POOL || ((160 / W) % 2 == 0));
  if (mode == 0) return launch_t<C, CO, EPI, C, 2>(x, w, bias, alpha, z, aux, N, H, W, Cout, s);
  if (small) return launch_t<C, CO, EPI, CH2, 1>(x, w, bias, alpha, z, aux, N, H, W, Cout, s);
  return launch_t<C, CO, EPI, CH2, 2>(x, w, bias, alpha, z, aux, N, H, W, Cout, s);
}

template <int C, int EPI>
static int by_cout(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N, int H,
                   int W, int Cout, hipStream_t s) {
  if (Cout <= 32) return launch<C, 32, EPI>(x, w, bias, alpha, z, aux, N, H, W, Cout, s);
  return launch<C, 64, EPI>(x, w, bias, alpha, z, aux, N, H, W, Cout, s);
}

}  // namespace ptgm32

extern "C" {

// 1 when the shape is covered: 5x5 'same' stride 1, C in {16, 32, 64}, Cout % 8 == 0 and <= 64, W divides
// 320 with 320 / W rows dividing H (even for pooling).
int ptg_conv32_supported(int H, int W, int C, int Cout, int KS, int pad, int epi) {
  if (KS != 5 || pad != 2 || (C != 16 && C != 32 && C != 64) || Cout % 8 || Cout > 64 || Cout < 8) return 0;
  if (W <= 0 || 320 % W) return 0;
  const int TR = 320 / W;
  if (H % TR) return 0;
  if (epi == 1 && ((TR & 1) || (W & 1))) return 0;
  return 1;
}

// z [N][H][W][Cout] = conv(x [N][H][W][C], w [Cout][5][5][C]) + bias; epi 0: z only, 1: + aux = pooled
// maxpool2x2(prelu(z, alpha)) [N][H/2][W/2][Cout], 2: + aux = prelu(z, alpha) [N][H][W][Cout]
int ptg_conv32(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, int N, int H,
               int W, int C, int Cout, int epi, hipStream_t s) {
  if (!ptg_conv32_supported(H, W, C, Cout, 5, 2, epi) || !ptg_fits_2g((long)N * H * W * (C > Cout ? C : Cout) * 2))
    return (int)hipErrorInvalidValue;
  if (epi != 0 && !alpha) return (int)hipErrorInvalidValue;
#define PTG_C32(CV)                                                                                          \
  if (C == CV) {                                                                                             \
    if (epi == 0) return ptgm32::by_cout<CV, ptgm32::EPI_Z>(x, w, bias, alpha, z, aux, N, H, W, Cout, s);    \
    if (epi == 1) return ptgm32::by_cout<CV, ptgm32::EPI_POOL>(x, w, bias, alpha, z, aux, N, H, W, Cout, s); \
    return ptgm32::by_cout<CV, ptgm32::EPI_PRELU>(x, w, bias, alpha, z, aux, N, H, W, Cout, s);             \
  }
  PTG_C32(16)
  PTG_C32(32)
  PTG_C32(64)
#undef PTG_C32
  return (int)hipErrorInvalidValue;
}

}  // extern "C"
