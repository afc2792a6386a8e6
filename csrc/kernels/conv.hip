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
//   conv_wgrad_strip_k dW[co][kh][kw][ci] = sum_pixels dZ[pix][co] * x[pix + (kh,kw)][ci]:
//                     M = Cout, N = 128-wide slice of (kh,kw,ci), K = pixels; dZ tile and x halo
//                     staged in LDS, both MFMA operands read with ds_read_b64_tr_b16 (gfx950
//                     transposed LDS read, cdna_hip_programming.md T10), partial sums of a whole
//                     chunk of tiles kept in registers, one fp32 atomic per output per workgroup.
//   conv_flip_k       W'[ci][kh][kw][co] = W[co][KS-1-kh][KS-1-kw][ci] (dgrad weights), bf16.
#include "common.h"
#include "conv_common.h"

#include <algorithm>

namespace ptgc {

// EPI_POOLS ("sparse pool"): like EPI_POOL but instead of the full-resolution z it stores, per
// pooled output and channel, only what the backward needs: the z of the window's argmax (bf16, into
// `z`, shaped like the pooled output) and the argmax position q = 2*dh + dw (uint8, `argout`) -
// 2.5 bytes per pooled element instead of 8 bytes of z (the first conv layer writes 335 MB less per
// step at batch 256 and its backward reads 335 MB less).
enum { EPI_Z = 0, EPI_POOL = 1, EPI_PRELU = 2, EPI_POOLS = 3 };

template <int C> struct PixPitch { static constexpr int v = C >= 16 ? C + 8 : C; };  // bank-conflict pad (wgrad)
// forward halo: pixel pitch and per-row pad (elements) chosen with tools/lds_bank_sim.py so the
// ds_read_b128 A-fragment reads of every (fragment, k-step) are conflict-free on gfx950's lane
// groups (4 LDS cycles per read; C=16 was 7.9, C=32 12, C=64 8 with the uniform C+8 pitch).
template <int C> struct FwdPitch { static constexpr int pix = C == 64 ? 96 : C, rowpad = (C == 32 || C == 64) ? 16 : 0; };
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
// forward / dgrad: persistent column-strip kernel, transposed MFMA (D = W * X^T)
// ================================================================================================
// A workgroup owns a contiguous range of TH x TW output tiles, strip-major: it walks a vertical
// strip (n, tw) top to bottom.
//  * RING: the halo lives in a mirrored ring of 2*HR LDS rows; moving down one tile only loads the
//    TH new input rows.  Without RING (TH >= 2*(KS-1)) each tile reloads its HR rows.
//  * the next tile's rows are prefetched into registers before this tile's MFMAs and written to
//    LDS after them, so HBM latency hides behind compute.
//  * MFMA computes D[co][pixel] (weights are the A operand, the halo the B operand), so every lane
//    ends with 4 consecutive output channels of one pixel: bias, bf16 rounding, per-element PReLU
//    (one float4 alpha load) and 8-byte stores straight from registers - no LDS staging.
//  * the 2x2 max-pool runs in registers: horizontal neighbours are adjacent lanes (xor 1); vertical
//    neighbours are the paired fragment of the same wave (TW >= 16) or lanes xor TW (TW < 16).
//  * PReLU is applied to the bf16-rounded z, exactly what the backward recomputes.
typedef __attribute__((ext_vector_type(4))) unsigned int vu4_t;   // register-friendly (SROA-able)
typedef __attribute__((ext_vector_type(2))) unsigned int vu2_t;
template <int C> struct HVec { using T = vu4_t; static constexpr int per_pix = C / 8; };
template <> struct HVec<4> { using T = vu2_t; static constexpr int per_pix = 1; };

// Work queue of the persistent kernels: round 0 takes chunk `b` (the workgroup's own, no atomic: a
// launch-wide burst of claims on one address serialises for tens of us), later rounds claim chunk
// nb + counter++ once the previous chunk is done.  Every workgroup claims until it draws a chunk
// >= nch: (nch - nb) successful claims + one failing claim per workgroup that owns a chunk = nch
// claims in total, so the workgroup drawing the value nch - 1 re-arms the counter to 0 for the next
// launch (graph replays included).  Returns the chunk (>= nch: done).
PTG_DEV long wq_next(int* cnt, int round, int b, int nb, int nch, int* s_slot) {
  if (round == 0) return b;
  if (b >= nch) return nch;  // no own chunk: never claimed (keeps the claim count at nch)
  __syncthreads();
  if (threadIdx.x == 0) {
    const int v = atomicAdd(cnt, 1);
    if (v == nch - 1) atomicExch(cnt, 0);
    *s_slot = v;
  }
  __syncthreads();
  const long c = (long)nb + *s_slot;
  __syncthreads();
  return c;
}

template <class VT> PTG_DEV VT bload_vt(Rsrc r, uint32_t off);
template <> PTG_DEV vu4_t bload_vt<vu4_t>(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(vu4_t, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
template <> PTG_DEV vu2_t bload_vt<vu2_t>(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(vu2_t, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// dpp row_shl:n - lane l receives lane l+n of its 16-lane row (others keep their own value)
template <int NSH>
PTG_DEV float row_shl(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x100 | NSH, 0xF, 0xF, false));
}

// 8 bf16 channels of a sparse pool record, kept where their argmax byte (a) equals the pixel's window
// position q, zero elsewhere: x ^ (q * 0x01010101) has a zero byte exactly at the matching channels
PTG_DEV vu4_t sparse_select(vu4_t v, U2 a, uint32_t q) {
  const uint32_t rep = q * 0x01010101u, x0 = a.x ^ rep, x1 = a.y ^ rep;
  auto m = [](uint32_t x, int sh) -> uint32_t {
    return (((x >> sh) & 0xffu) == 0u ? 0x0000ffffu : 0u) | (((x >> (sh + 8)) & 0xffu) == 0u ? 0xffff0000u : 0u);
  };
  vu4_t o;
  o.x = v.x & m(x0, 0);
  o.y = v.y & m(x0, 16);
  o.z = v.z & m(x1, 0);
  o.w = v.w & m(x1, 16);
  return o;
}
PTG_DEV vu2_t sparse_select(vu2_t v, U2, uint32_t) { return v; }  // (C == 4: never instantiated with SPIN)

// WLDS: the block's weight slice [NF*16 co][KSTEPS*32 k] is staged in LDS once (persistent
// workgroup) and every A fragment is an LDS read instead of a per-wave global load per k-step
// (for C >= 16 those loads were L2-latency bound).  COS > 1 splits Cout over COS workgroup groups
// (blockIdx % COS), each holding NF*16 channels, when the whole filter does not fit LDS.
// SPIN (data gradients of a pooled layer, EPI_Z only): the input is the layer's sparse dZ record -
// x = dzsel [N][H/2][W/2][C] (dZ at each 2x2 window's argmax) and argout = argq (the argmax q = 2*dh
// + dw per channel, same shape) - and the halo loader expands it: halo pixel (ih, iw) keeps channel
// c of its window's dzsel where argq == 2*(ih & 1) + (iw & 1), zero elsewhere.  The full-resolution
// dZ is never written or read (4x fewer bytes than the dense dZ, plus the argq byte).
template <int C, int KS, int NF, int TW, int TH, int EPI, bool RING, bool KSPLIT, bool WLDS = false, int COS = 1,
          bool SPIN = false>
__global__ __launch_bounds__(256) void conv_fwd_strip_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                        const float* __restrict__ bias, const float* __restrict__ alpha,
                                                        bf16_t* __restrict__ z, bf16_t* __restrict__ aux,
                                                        uint8_t* __restrict__ argout, int N, int H,
                                                        int W, int Cout, int pad, int tiles_h, int tiles_w,
                                                        int* __restrict__ wq, int wchunk) {
  using VT = typename HVec<C>::T;
  constexpr int VPP = HVec<C>::per_pix;      // vectors per pixel
  constexpr int VE = C == 4 ? 4 : 8;          // elements per vector
  constexpr int KWP = Kwp<C, KS>::v;
  constexpr int PIX = FwdPitch<C>::pix;
  constexpr int HR = TH + KS - 1, HC = TW + KWP - 1;
  constexpr int ROWE = HC * PIX + FwdPitch<C>::rowpad;
  constexpr int NROWS = RING ? 2 * HR : HR;
  constexpr int KROW = KWP * C;
  constexpr int KTOT = KS * KROW;
  constexpr int KSTEPS = (KTOT + 31) / 32;
  constexpr int M = TH * TW;
  constexpr int MFR = M / 16;
  constexpr int FM = MFR / 4;
  constexpr bool WIDE = TW >= 16;             // fragment = 16 pixels of one row
  static_assert(MFR % 4 == 0 && TH % 2 == 0, "tile shape");
  static_assert(WIDE ? (TW % 16 == 0 && (FM % 2 == 0 || (EPI != EPI_POOL && EPI != EPI_POOLS))) : (TW == 4 || TW == 8),
                "pool pairing");
  constexpr int SEG = WIDE ? TW / 16 : 1;
  constexpr int HALO_ELEMS = NROWS * ROWE;
  constexpr int PFN = (HR * HC * VPP + 255) / 256;   // prefetch vectors per thread (worst case: HR rows)
  constexpr bool WREG = !KSPLIT && KSTEPS * NF <= 8;   // all weight fragments resident in VGPRs
  // KSPLIT: each wave runs every pixel fragment of the tile over a quarter of the K-steps, then
  // the partial sums are reduce-scattered through LDS (more MFMAs per weight fetch when FM is small)
  constexpr int AF = KSPLIT ? MFR : FM;                // fragments a wave accumulates
  constexpr int RED_F4 = KSPLIT ? 4 * 3 * FM * NF * 64 : 1;
  constexpr int WP = KSTEPS * 32 + 8;                  // LDS weight row pitch: odd multiple of 16 B
  constexpr int WL_ELEMS = WLDS ? NF * 16 * WP : 8;
  static_assert(!WLDS || (C >= 8 && !KSPLIT), "WLDS: contiguous filter rows, no k-split");
  static_assert(!SPIN || (EPI == EPI_Z && C >= 8), "sparse-record input: data gradient (EPI_Z), 8-channel vectors");
  __shared__ __attribute__((aligned(16))) bf16_t smem[HALO_ELEMS + 8];
  __shared__ __attribute__((aligned(16))) float4 sred[RED_F4];
  __shared__ __attribute__((aligned(16))) bf16_t wlds[WL_ELEMS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int px = lane & 15, g = lane >> 4;
  const int S = N * tiles_w;
  const int cb = COS > 1 ? (int)(blockIdx.x % COS) * NF * 16 : 0;   // first output channel of this block
  const int bid = COS > 1 ? (int)(blockIdx.x / COS) : (int)blockIdx.x;
  const int nblk = COS > 1 ? (int)(gridDim.x / COS) : (int)gridDim.x;
  if (tid < 8) smem[HALO_ELEMS + tid] = 0;  // zero guard for padded K groups
  if constexpr (WLDS) {
    constexpr int VR = KSTEPS * 4;  // 16-byte vectors per weight row
    for (int idx = tid; idx < NF * 16 * VR; idx += 256) {
      const int r = idx / VR, v = idx - r * VR, co = cb + r, kf = v * 8;
      U4 val = zero4();
      if (co < Cout && kf < KTOT) val = *(const U4*)(w + (long)co * KTOT + kf);
      *(U4*)(wlds + r * WP + kf) = val;
    }
  }

  // ---- weight fragments (MFMA A operand: row = co, 8 k per lane group): w [Cout][KS][KS][C] ----
  auto load_w = [&](int ks, int j) -> bf16x8_t {
    const int kf = ks * 32 + 8 * g;
    const int kh = kf / KROW, rem = kf - kh * KROW;
    const int kw = rem / C, ci = rem - kw * C;
    const int co = cb + j * 16 + px;
    U4 v = zero4();
    if constexpr (WLDS) {
      (void)kh; (void)kw; (void)ci; (void)co;
      return *(const bf16x8_t*)(wlds + (j * 16 + px) * WP + kf);
    } else if constexpr (C >= 8) {  // KWP == KS: flattened K is the memory order of a filter
      (void)kh; (void)kw; (void)ci;
      if (kf < KTOT && co < Cout) v = *(const U4*)(w + (long)co * KTOT + kf);
    } else if (kf < KTOT && co < Cout) {
      const bf16_t* wp = w + ((long)co * KS * KS + kh * KS) * C;
      {
        U2 a = U2{0u, 0u}, b = U2{0u, 0u};
        if (kw < KS) a = *(const U2*)(wp + kw * 4);
        if (kw + 1 < KS) b = *(const U2*)(wp + (kw + 1) * 4);
        v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
      }
    }
    return __builtin_bit_cast(bf16x8_t, v);
  };
  bf16x8_t wreg[WREG ? KSTEPS : 1][NF];
  if constexpr (WREG) {
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
      for (int j = 0; j < NF; ++j) wreg[ks][j] = load_w(ks, j);
  }
  // bias for this lane's 4 channels of each co fragment
  float bv[NF][4];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int co0 = cb + j * 16 + g * 4;
    float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias && co0 < Cout) b4 = *(const float4*)(bias + co0);
    bv[j][0] = b4.x; bv[j][1] = b4.y; bv[j][2] = b4.z; bv[j][3] = b4.w;
  }

  // ---- halo rows: per-thread fixed (row, col, vector) slots, global -> registers -> LDS ring ----
  int pr_r[PFN], pr_c[PFN], pr_l[PFN];
#pragma unroll
  for (int p = 0; p < PFN; ++p) {
    const int idx = tid + p * 256;
    const int pix = idx / VPP, vv = idx - pix * VPP;
    pr_r[p] = pix / HC;
    pr_c[p] = pix - pr_r[p] * HC;
    pr_l[p] = pr_c[p] * PIX + vv * VE;   // LDS offset inside a halo row
  }
  VT pf[PFN];
  U2 pa[SPIN ? PFN : 1];        // SPIN: the argq bytes of each slot's 8 channels
  uint32_t pq[SPIN ? PFN : 1];  // SPIN: the slot pixel's window position q
  // halo loads: buffer loads, the zero padding / rows past the image come back as 0 (PTG_OOB)
  const int SPH = H >> 1, SPW = W >> 1;
  const Rsrc xr = make_rsrc(x, SPIN ? (uint32_t)((long)N * SPH * SPW * C * 2) : (uint32_t)((long)N * H * W * C * 2));
  const Rsrc ar = make_rsrc(argout, SPIN ? (uint32_t)((long)N * SPH * SPW * C) : 0u);
  auto load_rows = [&](int n, int iw0, int ih_first, int nrows) {
    if constexpr (SPIN) {
      const uint32_t img = (uint32_t)(n * SPH * SPW * C);
#pragma unroll
      for (int p = 0; p < PFN; ++p) {
        const int ih = ih_first + pr_r[p], iw = iw0 + pr_c[p];
        const bool ok = pr_r[p] < nrows && (unsigned)ih < (unsigned)(2 * SPH) && (unsigned)iw < (unsigned)(2 * SPW);
        const uint32_t e = img + (uint32_t)(((ih >> 1) * SPW + (iw >> 1)) * C + (pr_l[p] - pr_c[p] * PIX));
        pf[p] = bload_vt<VT>(xr, ok ? 2u * e : PTG_OOB);
        pa[p] = bload8(ar, ok ? e : PTG_OOB);
        pq[p] = (uint32_t)(((ih & 1) << 1) | (iw & 1));
      }
    } else {
      const uint32_t img = (uint32_t)(n * H * W * C) * 2u;
#pragma unroll
      for (int p = 0; p < PFN; ++p) {
        const int ih = ih_first + pr_r[p], iw = iw0 + pr_c[p];
        const bool ok = pr_r[p] < nrows && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        pf[p] = bload_vt<VT>(xr, ok ? img + (uint32_t)((ih * W + iw) * C + (pr_l[p] - pr_c[p] * PIX)) * 2u : PTG_OOB);
      }
    }
  };
  auto store_rows = [&](int nrows, int slot_first) {
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      if (pr_r[p] < nrows) {
        int slot = slot_first + pr_r[p];
        if constexpr (RING) slot = slot >= HR ? slot - HR : slot;
        bf16_t* dst = smem + slot * ROWE + pr_l[p];
        VT v = pf[p];
        if constexpr (SPIN) v = sparse_select(v, pa[p], pq[p]);
        *(VT*)dst = v;
        if constexpr (RING) *(VT*)(dst + HR * ROWE) = v;
      }
    }
  };

  // ---- this lane's pixel of each fragment (tile coordinates): owned fragments first ----
  auto frag_rc = [&](int f, int& rr, int& cc) {
    if constexpr (WIDE) {
      const int pi = f >> 1, sub = f & 1;
      rr = 2 * (pi / SEG) + sub;
      cc = (pi % SEG) * 16 + px;
    } else {
      rr = (f * 16 + px) / TW;
      cc = (f * 16 + px) % TW;
    }
  };
  int f_r[FM], f_c[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int f = wid * FM + i;
    if constexpr (WIDE) {
      const int pi = f >> 1, sub = f & 1;  // fragment pairs = vertically adjacent rows
      f_r[i] = 2 * (pi / SEG) + sub;
      f_c[i] = (pi % SEG) * 16 + px;
    } else {
      f_r[i] = (f * 16 + px) / TW;
      f_c[i] = (f * 16 + px) % TW;
    }
  }

  // KUNROLL: the K loop fully unrolled with each lane's halo offset per k-step precomputed here
  // (tile-invariant; -1: k group past KTOT).  Rolled, every k-step spent ~14 VALU ops on the
  // (kh, kw, ci) division and waited for its LDS read right before its MFMA.
  constexpr bool KUNROLL = !WREG && !KSPLIT && KSTEPS <= 32;
  int koffs[KUNROLL ? KSTEPS : 1];
  if constexpr (KUNROLL) {
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int kf = ks * 32 + 8 * g;
      const int kh = kf / KROW, rem = kf - kh * KROW, kw = rem / C, ci = rem - kw * C;
      koffs[ks] = kf < KTOT ? kh * ROWE + kw * PIX + ci : -1;
    }
  }
  // tile-invariant parts of each fragment's output offsets (elements): full-resolution planes (lf)
  // and, for the pool-window leaders (even row and column), the pooled planes (lp; others ~0u)
  uint32_t lf[FM], lp[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    lf[i] = (uint32_t)(f_r[i] * W + f_c[i]) * (uint32_t)Cout + (uint32_t)(cb + g * 4);
    const bool lead = ((f_r[i] | f_c[i]) & 1) == 0;
    lp[i] = lead ? (uint32_t)((f_r[i] >> 1) * (W >> 1) + (f_c[i] >> 1)) * (uint32_t)Cout + (uint32_t)(cb + g * 4) : ~0u;
  }
  // pooled-plane element offset of fragment i's window for co fragment j, or PTG_OOB / 2 (dropped)
  // when the lane does not lead a window or the window / channel is outside the output
  auto pool_off = [&](int i, int j, bool cval, uint32_t tpool, uint32_t ppl, int oh0_, int ow0_) -> uint32_t {
    const int ph = (oh0_ + f_r[i]) >> 1, pw = (ow0_ + f_c[i]) >> 1;
    const bool ok = cval && lp[i] != ~0u && ph < (H >> 1) && pw < (W >> 1);
    return ok ? (uint32_t)PTG_CHECKED_IDX(tpool + lp[i] + j * 16, (long)ppl) : PTG_OOB / 2;
  };

  // Tile ranges, strip-major: static (this workgroup's contiguous 1/nblk of the tiles) or, with a
  // work queue `wq`, chunks of `wchunk` tiles claimed until none is left - a workgroup that starts
  // late (CUs held by a concurrent RCCL kernel) then takes less work instead of a full range.
  const long T = (long)S * tiles_h;
  // SMAJ (no halo ring, PReLU epilogue): tiles are ordered position-major, sample-minor, so the
  // consecutive tiles of a workgroup share one output position and the per-element PReLU alphas
  // (for CNN-B1 layer 2 16 KB per tile, more than its halo) stay in registers across samples
  constexpr bool SMAJ = !RING && EPI != EPI_Z;
  // tile t -> (sample n, column strip twi, row tile th); divisions only for a range's first tile,
  // then the next tile is stepped incrementally (each runtime 32-bit division is ~40 scalar and
  // vector instructions, and the tile loop did six of them per tile)
  auto decode = [&](int tt, int& n_, int& twi_, int& th_) {
    if constexpr (SMAJ) {
      const int pos = tt / N;
      n_ = tt - pos * N;
      twi_ = pos / tiles_h;
      th_ = pos - twi_ * tiles_h;
    } else {
      const int s_ = tt / tiles_h;
      th_ = tt - s_ * tiles_h;
      n_ = s_ / tiles_w;
      twi_ = s_ - n_ * tiles_w;
    }
  };
  auto step = [&](int& n_, int& twi_, int& th_) {
    if constexpr (SMAJ) {  // sample fastest, then row tile, then column strip
      if (++n_ == N) { n_ = 0; if (++th_ == tiles_h) { th_ = 0; ++twi_; } }
    } else {               // row tile fastest (down a strip), then strip, then sample
      if (++th_ == tiles_h) { th_ = 0; if (++twi_ == tiles_w) { twi_ = 0; ++n_; } }
    }
  };
  float4 al[EPI != EPI_Z ? FM : 1][NF];
  __shared__ int s_wq;
  for (int round = 0;; ++round) {
  int t0, t1;
  if (wq) {
    const long c = wq_next(wq + (COS > 1 ? (int)(blockIdx.x % COS) : 0), round, bid, nblk, (int)((T + wchunk - 1) / wchunk),
                           &s_wq);
    t0 = (int)min(T, c * wchunk);
    t1 = (int)min(T, (c + 1) * wchunk);
  } else {
    if (round) break;
    t0 = (int)(T * bid / nblk);
    t1 = (int)(T * (bid + 1) / nblk);
  }
  if (t0 >= t1) break;
  int n, twi, th;
  decode(t0, n, twi, th);
  int apos = -1;  // output position whose alphas are in al (SMAJ)
  {  // first tile: synchronous fill of its HR rows
    load_rows(n, twi * TW - pad, th * TH - pad, HR);
    store_rows(HR, RING ? (th * TH) % HR : 0);
  }
  __syncthreads();

  const int PH = H >> 1, PW = W >> 1;
  for (int t = t0; t < t1; ++t) {
    const int ow0 = twi * TW, oh0 = th * TH;
    // next tile of the range and the rows it needs that are not resident
    int n2 = n, twi2 = twi, th2 = th;
    step(n2, twi2, th2);
    const bool has_next = t + 1 < t1;
    const bool same_strip = !SMAJ && n2 == n && twi2 == twi;
    const int ow02 = twi2 * TW;
    const int nrows2 = (RING && same_strip) ? TH : HR;
    const int ih2 = (RING && same_strip) ? th2 * TH - pad + HR - TH : th2 * TH - pad;
    const int slot2 = !RING ? 0 : same_strip ? (th2 * TH + HR - TH) % HR : (th2 * TH) % HR;
    if (has_next) load_rows(n2, ow02 - pad, ih2, nrows2);

    // alpha for this lane's (pixel, 4 channels) of every fragment, needed after the MFMAs
    const int pos = twi * tiles_h + th;
    if constexpr (EPI != EPI_Z) {
      if (pos != apos) {
        apos = pos;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j) {
            const int oh = oh0 + f_r[i], ow = ow0 + f_c[i], co0 = cb + j * 16 + g * 4;
            al[i][j] = (co0 < Cout && oh < H && ow < W) ? *(const float4*)(alpha + ((long)oh * W + ow) * Cout + co0)
                                                        : make_float4(0.f, 0.f, 0.f, 0.f);
          }
      }
    }

    // ---- MFMA main loop over the flattened K = (kh, kw', ci) ----
    const int wstart = RING ? (oh0 % HR) : 0;
    int pbase[AF];
#pragma unroll
    for (int i = 0; i < AF; ++i) {
      int rr, cc;
      if constexpr (KSPLIT) frag_rc(i, rr, cc);
      else { rr = f_r[i]; cc = f_c[i]; }
      pbase[i] = (wstart + rr) * ROWE + cc * PIX;
    }
    f32x4_t acc[AF][NF];
#pragma unroll
    for (int i = 0; i < AF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    constexpr int KS0 = 0, KSTEP = KSPLIT ? 4 : 1;
    const int ks_begin = KSPLIT ? wid : KS0;
    bf16x8_t wnext[NF];
    if constexpr (!WREG) {
#pragma unroll
      for (int j = 0; j < NF; ++j) wnext[j] = load_w(ks_begin, j);
    }
#pragma unroll((WREG || KUNROLL) ? KSTEPS : 1)
    for (int ks = ks_begin; ks < KSTEPS; ks += KSTEP) {
      bf16x8_t wf[NF];
      if constexpr (WREG) {
#pragma unroll
        for (int j = 0; j < NF; ++j) wf[j] = wreg[WREG ? ks : 0][j];
      } else {
#pragma unroll
        for (int j = 0; j < NF; ++j) wf[j] = wnext[j];
        if (ks + KSTEP < KSTEPS) {
#pragma unroll
          for (int j = 0; j < NF; ++j) wnext[j] = load_w(ks + KSTEP, j);
        }
      }
      int koff;
      bool kval;
      if constexpr (KUNROLL) {
        koff = koffs[KUNROLL ? ks : 0];
        kval = koff >= 0;
      } else {
        const int kf = ks * 32 + 8 * g;
        kval = kf < KTOT;
        const int kh = kf / KROW, rem = kf - kh * KROW;
        const int kw = rem / C, ci = rem - kw * C;
        koff = kh * ROWE + kw * PIX + ci;
      }
#pragma unroll
      for (int i = 0; i < AF; ++i) {
        bf16x8_t xf;
        const int off = kval ? pbase[i] + koff : HALO_ELEMS;
        if constexpr (C >= 8) {
          xf = *(const bf16x8_t*)(smem + off);
        } else {
          const U2 lo = *(const U2*)(smem + off);
          const U2 hi = kval ? *(const U2*)(smem + off + 4) : U2{0u, 0u};
          U4 v; v.x = lo.x; v.y = lo.y; v.z = hi.x; v.w = hi.y;
          xf = __builtin_bit_cast(bf16x8_t, v);
        }
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf, acc[i][j], 0, 0, 0);
      }
    }
    f32x4_t res[FM][NF];
    if constexpr (KSPLIT) {
      // reduce-scatter: fragment f belongs to wave f / FM; partials go to that owner's slots
#pragma unroll
      for (int f = 0; f < MFR; ++f) {
        const int o = f / FM, q = f % FM;
        if (o != wid) {
          const int src = wid < o ? wid : wid - 1;  // 0..2 among the non-owners
#pragma unroll
          for (int j = 0; j < NF; ++j)
            sred[(((o * 3 + src) * FM + q) * NF + j) * 64 + lane] =
                make_float4(acc[f][j][0], acc[f][j][1], acc[f][j][2], acc[f][j][3]);
        }
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < FM; ++q)
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          f32x4_t a = acc[0][j];
          // own partial (static index: select among fragments)
#pragma unroll
          for (int f = 0; f < MFR; ++f)
            if (f == wid * FM + q) a = acc[f][j];
#pragma unroll
          for (int src = 0; src < 3; ++src) {
            const float4 v = sred[(((wid * 3 + src) * FM + q) * NF + j) * 64 + lane];
            a[0] += v.x; a[1] += v.y; a[2] += v.z; a[3] += v.w;
          }
          res[q][j] = a;
        }
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) res[i][j] = acc[i][j];
    }
    __syncthreads();  // every wave is done reading the halo window
    if (has_next) store_rows(nrows2, slot2);

    // ---- epilogue from registers ----
    // Stores go through per-tile buffer descriptors over sample n's output planes: the 64-bit plane
    // base is uniform (scalar math once per tile) and each lane adds a 32-bit offset = the tile's
    // uniform offset + its precomputed fragment offset (lf / lp), instead of 64-bit per-fragment
    // index arithmetic (v_mul_lo_u32 / v_mad_u64_u32: ~100 VALU ops of a ~360-op tile on layer 2).
    // Lanes outside the image / channel range or not leading a pool window store at PTG_OOB, which
    // the descriptor's range check drops - no exec-mask branches.
    const uint32_t zpl = (uint32_t)(EPI == EPI_POOLS ? PH * PW : H * W) * (uint32_t)Cout;  // elements
    const uint32_t ppl = (uint32_t)(PH * PW) * (uint32_t)Cout;
    const Rsrc rz = make_rsrc(z + (long)n * zpl, zpl * 2u);
    const Rsrc ra = make_rsrc(aux + (long)n * (EPI == EPI_PRELU ? zpl : ppl), (EPI == EPI_PRELU ? zpl : ppl) * 2u);
    const uint32_t tfull = (uint32_t)(oh0 * W + ow0) * (uint32_t)Cout;
    const uint32_t tpool = (uint32_t)((oh0 >> 1) * PW + (ow0 >> 1)) * (uint32_t)Cout;
    if constexpr (EPI == EPI_POOLS) {
      // sparse pool record, one vertical fragment pair (WIDE) / one fragment at a time to keep the
      // live register set small; the first maximum in q order (0,1,2,3) wins, as in the dense
      // backward
      const Rsrc rq = make_rsrc(argout + (long)n * ppl, ppl);
      constexpr int STEP = WIDE ? 2 : 1;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int co0 = cb + j * 16 + g * 4;
        const bool cval = co0 < Cout;
#pragma unroll
        for (int i = 0; i < FM; i += STEP) {
          float yy[STEP][4], zz[STEP][4], qq[STEP][4];
#pragma unroll
          for (int u = 0; u < STEP; ++u) {
            const float a4[4] = {al[i + u][j].x, al[i + u][j].y, al[i + u][j].z, al[i + u][j].w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float zr = bf2f(f2bf(res[i + u][j][r] + bv[j][r]));
              const float yv = zr > 0.f ? zr : a4[r] * zr;
              const float yn = row_shl<1>(yv), zn = row_shl<1>(zr);
              const bool right = yn > yv;
              yy[u][r] = right ? yn : yv;
              zz[u][r] = right ? zn : zr;
              qq[u][r] = right ? 1.f : 0.f;
            }
          }
          float pm[4], pz[4], pq[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float yb, zb, qb;
            if constexpr (WIDE) { yb = yy[STEP - 1][r]; zb = zz[STEP - 1][r]; qb = qq[STEP - 1][r]; }
            else {
              yb = row_shl<(WIDE ? 1 : TW)>(yy[0][r]);
              zb = row_shl<(WIDE ? 1 : TW)>(zz[0][r]);
              qb = row_shl<(WIDE ? 1 : TW)>(qq[0][r]);
            }
            const bool down = yb > yy[0][r];
            pm[r] = down ? yb : yy[0][r];
            pz[r] = down ? zb : zz[0][r];
            pq[r] = down ? qb + 2.f : qq[0][r];
          }
          const uint32_t po = pool_off(i, j, cval, tpool, ppl, oh0, ow0);
          bstore8(ra, 2u * po, U2{pack_bf(pm[0], pm[1]), pack_bf(pm[2], pm[3])});
          bstore8(rz, 2u * po, U2{pack_bf(pz[0], pz[1]), pack_bf(pz[2], pz[3])});
          bstore4(rq, po, (uint32_t)pq[0] | ((uint32_t)pq[1] << 8) | ((uint32_t)pq[2] << 16) | ((uint32_t)pq[3] << 24));
        }
      }
    } else
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int co0 = cb + j * 16 + g * 4;
      const bool cval = co0 < Cout;
      float y[FM][4];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        float zr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) zr[r] = bf2f(f2bf(res[i][j][r] + bv[j][r]));
        const bool in = cval && oh0 + f_r[i] < H && ow0 + f_c[i] < W;
        const uint32_t o = in ? (uint32_t)PTG_CHECKED_IDX(tfull + lf[i] + j * 16, (long)zpl) : PTG_OOB / 2;
        bstore8(rz, 2u * o, U2{pack_bf(zr[0], zr[1]), pack_bf(zr[2], zr[3])});
        if constexpr (EPI != EPI_Z) {
          const float a4[4] = {al[i][j].x, al[i][j].y, al[i][j].z, al[i][j].w};
#pragma unroll
          for (int r = 0; r < 4; ++r) y[i][r] = zr[r] > 0.f ? zr[r] : a4[r] * zr[r];
          if constexpr (EPI == EPI_PRELU) bstore8(ra, 2u * o, U2{pack_bf(y[i][0], y[i][1]), pack_bf(y[i][2], y[i][3])});
        }
      }
      if constexpr (EPI == EPI_POOL) {
        // horizontal pair: lanes px, px^1; vertical pair: fragment i^1 (WIDE) or lanes px^TW
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) y[i][r] = fmaxf(y[i][r], row_shl<1>(y[i][r]));  // lead lanes: even column
#pragma unroll
        for (int i = 0; i < FM; i += (WIDE ? 2 : 1)) {
          float pm[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if constexpr (WIDE) pm[r] = fmaxf(y[i][r], y[i + 1][r]);
            else pm[r] = fmaxf(y[i][r], row_shl<(WIDE ? 1 : TW)>(y[i][r]));
          }
          bstore8(ra, 2u * pool_off(i, j, cval, tpool, ppl, oh0, ow0), U2{pack_bf(pm[0], pm[1]), pack_bf(pm[2], pm[3])});
        }
      }
    }
    if (!has_next) break;
    __syncthreads();  // next tile's halo rows visible
    n = n2;
    twi = twi2;
    th = th2;
  }
  }  // work rounds
}

// ================================================================================================
// weight gradient
// ================================================================================================

// Persistent: a workgroup owns one 64*NB-wide kflat slice and a contiguous strip-major range of
// tiles; the next tile's halo rows (RING: only the TH new ones) and dZ tile are prefetched into
// registers during this tile's MFMAs.  Partial sums stay in registers for the whole range and are
// flushed with one fp32 atomic per output.
//
// SPARSE: dZ comes as the sparse pool record of its prelu+pool backward (dzsel [N][H/2][W/2][Cout]
// = dZ at each window's argmax, argq = the argmax position q = 2*dh + dw; dZ is zero elsewhere in
// the window): each thread loads 4 channels of one pooled pixel (8 + 4 bytes instead of the 32
// bytes of the dense 2x2 window) and expands them into the same dense LDS dZ tile.
// U8 (C == 4 only): x is uint8 [N][H][W][3]; each halo pixel is three byte loads, converted to the
// 4-channel bf16 pixel (/255, zero 4th channel) in registers before the LDS store.
template <int C, int KS, int TW, int TH, int MF, int NB, bool RING, bool SPARSE = false, bool U8 = false>
__global__ __launch_bounds__(256) void conv_wgrad_strip_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dz,
                                                          float* __restrict__ dw, int N, int H, int W, int Cout, int pad,
                                                          int tiles_h, int tiles_w, int nslices,
                                                          const uint8_t* __restrict__ argq, int* __restrict__ wq,
                                                          int wchunk) {
  using VT = typename HVec<C>::T;
  constexpr int VPP = HVec<C>::per_pix, VE = C == 4 ? 4 : 8;
  constexpr int PIX = PixPitch<C>::v;
  constexpr int HR = TH + KS - 1, HC = TW + KS - 1;
  constexpr int ROWE = HC * PIX;
  constexpr int NROWS = RING ? 2 * HR : HR;
  constexpr int M = TH * TW;              // pixels per tile (K of this GEMM)
  static_assert(M % 32 == 0 && TW % 4 == 0, "tile shape");
  constexpr int KF = KS * KS * C;         // output columns (kh, kw, ci)
  constexpr int SLICE = 64 * NB;
  constexpr int DPITCH = MF * 16 + 4;     // dZ tile pixel pitch (bf16): 8-byte aligned, bank-shifted
  constexpr int HALO_ELEMS = NROWS * ROWE;
  constexpr int DZ_ELEMS = M * DPITCH;
  static_assert(!U8 || HC % 2 == 0, "uint8 halo rows are loaded as pixel pairs");
  // U8: one slot = a pixel PAIR (16 bytes of bf16 in LDS); otherwise one 16-/8-byte vector
  constexpr int PFN = U8 ? (HR * (HC / 2) + 255) / 256 : (HR * HC * VPP + 255) / 256;
  constexpr int DV = (SPARSE ? M / 4 : M) * MF * 4;  // 8-byte dZ vectors per tile (upper bound: Cout <= MF*16)
  constexpr int PFD = (DV + 255) / 256;
  static_assert(!SPARSE || (TH % 2 == 0 && TW % 2 == 0), "sparse dZ needs whole 2x2 windows per tile");
  __shared__ __attribute__((aligned(16))) bf16_t smem[HALO_ELEMS + DZ_ELEMS + 8];
  bf16_t* const ds = smem + HALO_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int slice = blockIdx.x % nslices, chunk = blockIdx.x / nslices, nchunks = gridDim.x / nslices;
  const long T = (long)N * tiles_w * tiles_h;

  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  // per-lane B column (kflat) base of each of this wave's NB fragments
  int boff[NB];
  bool bval[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int kf = slice * SLICE + (wid * NB + j) * 16 + 4 * p;
    bval[j] = kf < KF;
    const int kk = bval[j] ? kf : 0;
    const int kh = kk / (KS * C), rem = kk - kh * KS * C, kw = rem / C, ci = rem - kw * C;
    boff[j] = (kh * HC + kw) * PIX + ci;
  }
  f32x4_t acc[MF][NB];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // KSEP (32 % TW == 0): a k0 block of 32 pixels starts a tile row, so the pixel of a lane's
  // tr-read rows splits into k0's rows (compile-time) + the lane's own (row, column) below
  constexpr bool KSEP = 32 % TW == 0;
  const int lp0 = 8 * g + q, lp1 = lp0 + 4;
  const int hl0 = ((lp0 / TW) * HC + lp0 % TW) * PIX, hl1 = ((lp1 / TW) * HC + lp1 % TW) * PIX;
  const int dl0 = lp0 * DPITCH, dl1 = lp1 * DPITCH;

  // halo slots of this thread
  int pr_r[PFN], pr_c[PFN], pr_l[PFN];
#pragma unroll
  for (int k = 0; k < PFN; ++k) {
    const int idx = tid + k * 256;
    if constexpr (U8) {
      pr_r[k] = idx / (HC / 2);
      pr_c[k] = 2 * (idx - pr_r[k] * (HC / 2));
      pr_l[k] = pr_c[k] * PIX;
    } else {
      const int pix = idx / VPP, vv = idx - pix * VPP;
      pr_r[k] = pix / HC;
      pr_c[k] = pix - pr_r[k] * HC;
      pr_l[k] = pr_c[k] * PIX + vv * VE;
    }
  }
  static_assert(!U8 || (C == 4 && PIX == 4), "uint8 input is the 3-channel image (C padded to 4, unpadded pixels)");
  VT pf[U8 ? 1 : PFN];
  U8Pair pu[U8 ? PFN : 1];
  U2 pd[PFD];
  uint32_t pq[SPARSE ? PFD : 1];
  const int CV = Cout / 4;
  const int PH = H >> 1, PW = W >> 1;
  // buffer loads: halo padding, pixels past the image and unused slots read as 0 (PTG_OOB)
  const Rsrc xr = make_rsrc(x, U8 ? u8_rsrc_bytes((long)N * H * W * 3) : (uint32_t)((long)N * H * W * C * 2));
  const Rsrc dr = make_rsrc(dz, (uint32_t)(SPARSE ? (long)N * PH * PW * Cout * 2 : (long)N * H * W * Cout * 2));
  const Rsrc qr = make_rsrc(argq, SPARSE ? (uint32_t)((long)N * PH * PW * Cout) : 0u);
  auto load_tile = [&](int n, int twi_, int th_, int nrows, int ih_first) {
    const int ow0 = twi_ * TW, oh0 = th_ * TH;
    const uint32_t img = (uint32_t)(n * H * W * C) * 2u;
#pragma unroll
    for (int k = 0; k < PFN; ++k) {
      const int ih = ih_first + pr_r[k], iw = ow0 - pad + pr_c[k];
      const bool ok = pr_r[k] < nrows && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      if constexpr (U8) {  // iw even, W even: both pixels of the pair are in the row or both are padding
        pu[k] = u8pair_load(xr, (uint32_t)((n * H + ih) * W + iw) * 3u, ok && pr_r[k] < HR);
      } else {
        pf[k] = bload_vt<VT>(xr, ok ? img + (uint32_t)((ih * W + iw) * C + (pr_l[k] - pr_c[k] * PIX)) * 2u : PTG_OOB);
      }
    }
#pragma unroll
    for (int k = 0; k < PFD; ++k) {
      const int v = tid + k * 256;
      if constexpr (SPARSE) {
        const int m = v / CV, cv = v - m * CV;
        const int ph = (oh0 >> 1) + m / (TW / 2), pw = (ow0 >> 1) + m % (TW / 2);
        const bool ok = v < (M / 4) * CV && ph < PH && pw < PW;
        const uint32_t o = (uint32_t)(((n * PH + ph) * PW + pw) * Cout + cv * 4);
        pd[k] = bload8(dr, ok ? 2u * o : PTG_OOB);
        pq[k] = bload4(qr, ok ? o : PTG_OOB);
      } else {
        const int m = v / CV, cv = v - m * CV;
        const int oh = oh0 + m / TW, ow = ow0 + m % TW;
        const bool ok = v < M * CV && oh < H && ow < W;
        pd[k] = bload8(dr, ok ? (uint32_t)((((n * H + oh) * W + ow) * Cout + cv * 4) * 2) : PTG_OOB);
      }
    }
  };
  auto store_tile = [&](int nrows, int slot_first) {
#pragma unroll
    for (int k = 0; k < PFN; ++k) {
      if (pr_r[k] < nrows) {
        int slot = slot_first + pr_r[k];
        if constexpr (RING) slot = slot >= HR ? slot - HR : slot;
        bf16_t* dst = smem + slot * ROWE + pr_l[k];
        if constexpr (U8) {
          const U4 v = u8pair_to_bf16x8(pu[k]);
          *(U4*)dst = v;
          if constexpr (RING) *(U4*)(dst + HR * ROWE) = v;
        } else {
          *(VT*)dst = pf[k];
          if constexpr (RING) *(VT*)(dst + HR * ROWE) = pf[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < PFD; ++k) {
      const int v = tid + k * 256;
      if constexpr (SPARSE) {
        if (v < (M / 4) * CV) {
          const int m = v / CV, cv = v - m * CV;
          const int m00 = (2 * (m / (TW / 2))) * TW + 2 * (m % (TW / 2));
          const uint32_t lo = pd[k].x, hi = pd[k].y, qv = pq[k];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            // keep channel c's bf16 where its argmax byte equals q
            const uint32_t h0 = ((qv & 0xffu) == (uint32_t)q ? 0x0000ffffu : 0u) |
                                (((qv >> 8) & 0xffu) == (uint32_t)q ? 0xffff0000u : 0u);
            const uint32_t h1 = (((qv >> 16) & 0xffu) == (uint32_t)q ? 0x0000ffffu : 0u) |
                                (((qv >> 24) & 0xffu) == (uint32_t)q ? 0xffff0000u : 0u);
            *(U2*)(ds + (m00 + (q >> 1) * TW + (q & 1)) * DPITCH + cv * 4) = U2{lo & h0, hi & h1};
          }
        }
      } else if (v < M * CV) {
        const int m = v / CV, cv = v - m * CV;
        *(U2*)(ds + m * DPITCH + cv * 4) = pd[k];
      }
    }
  };

  // static range or work-queue chunks (see conv_fwd_strip_k); partial sums stay in registers across
  // every chunk this workgroup claims and are flushed once
  __shared__ int s_wq;
  for (int round = 0;; ++round) {
  int t0, t1;
  if (wq) {
    __syncthreads();  // the previous chunk's LDS reads are done before its refill
    const long c = wq_next(wq + slice, round, chunk, nchunks, (int)((T + wchunk - 1) / wchunk), &s_wq);
    t0 = (int)min(T, c * wchunk);
    t1 = (int)min(T, (c + 1) * wchunk);
  } else {
    if (round) break;
    t0 = (int)(T * chunk / nchunks);
    t1 = (int)(T * (chunk + 1) / nchunks);
  }
  if (t0 >= t1) break;
  // (sample, column strip, row tile) of t0; later tiles are stepped without divisions
  int th, twi, n;
  {
    const int s = t0 / tiles_h;
    th = t0 - s * tiles_h;
    n = s / tiles_w;
    twi = s - n * tiles_w;
  }
  load_tile(n, twi, th, HR, th * TH - pad);
  store_tile(HR, RING ? (th * TH) % HR : 0);
  __syncthreads();
  for (int t = t0; t < t1; ++t) {
    int n2 = n, twi2 = twi, th2 = th + 1;
    if (th2 >= tiles_h) { th2 = 0; if (++twi2 == tiles_w) { twi2 = 0; ++n2; } }
    const bool has_next = t + 1 < t1;
    const bool same_strip = th2 != 0;
    const int nrows2 = (RING && same_strip) ? TH : HR;
    const int ih2 = (RING && same_strip) ? th2 * TH - pad + HR - TH : th2 * TH - pad;
    const int slot2 = !RING ? 0 : same_strip ? (th2 * TH + HR - TH) % HR : (th2 * TH) % HR;
    if (has_next) load_tile(n2, twi2, th2, nrows2, ih2);

    const int wrow = RING ? (th * TH) % HR : 0;
    if constexpr (KSEP) {
      // fully unrolled: every read address = a per-tile base (lane + ring row) + a compile-time
      // offset of k0, so the loop is tr-reads and MFMAs only (the rolled form spent ~40 VALU ops per
      // 4 MFMAs on addresses and selects, and rotated the accumulators through AGPR moves)
      const int hw = wrow * HC * PIX;
      const bf16_t* hb0[NB];
      const bf16_t* hb1[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        hb0[j] = smem + hw + hl0 + boff[j];
        hb1[j] = smem + hw + hl1 + boff[j];
      }
#pragma unroll
      for (int k0 = 0; k0 < M; k0 += 32) {
        const int kr = (k0 / TW) * HC * PIX;  // compile-time after unrolling
        // (columns past KF read real halo data through boff's kk = 0 fallback: their outputs are
        // never flushed, see the epilogue)
        bf16x8_t af[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int co = i * 16 + 4 * p;
          const s16x4_t lo = tr_read(ds + dl0 + k0 * DPITCH + co);
          const s16x4_t hi = tr_read(ds + dl1 + k0 * DPITCH + co);
          const U2 a = __builtin_bit_cast(U2, lo), b = __builtin_bit_cast(U2, hi);
          U4 v; v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
          af[i] = __builtin_bit_cast(bf16x8_t, v);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const s16x4_t lo = tr_read(hb0[j] + kr);
          const s16x4_t hi = tr_read(hb1[j] + kr);
          const U2 a = __builtin_bit_cast(U2, lo), b = __builtin_bit_cast(U2, hi);
          U4 v; v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
          const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
          for (int i = 0; i < MF; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
        }
      }
    } else
#pragma unroll 2
    for (int k0 = 0; k0 < M; k0 += 32) {
      // rows of the two tr-reads of this lane group: pixels k0 + 8g + q and k0 + 8g + 4 + q
      const int m0 = k0 + 8 * g + q, m1 = m0 + 4;
      const int r0 = m0 / TW + wrow, c0 = m0 % TW, r1 = m1 / TW + wrow, c1 = m1 % TW;
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
      const int h0 = (r0 * HC + c0) * PIX, h1 = (r1 * HC + c1) * PIX;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int o0 = bval[j] ? h0 + boff[j] : HALO_ELEMS + DZ_ELEMS;
        const int o1 = bval[j] ? h1 + boff[j] : HALO_ELEMS + DZ_ELEMS;
        const s16x4_t lo = tr_read(smem + o0);
        const s16x4_t hi = tr_read(smem + o1);
        const U2 a = __builtin_bit_cast(U2, lo), b = __builtin_bit_cast(U2, hi);
        U4 v; v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
        const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
        for (int i = 0; i < MF; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
      }
    }
    if (!has_next) break;
    __syncthreads();  // all reads of this tile done
    store_tile(nrows2, slot2);
    __syncthreads();
    n = n2;
    twi = twi2;
    th = th2;
  }
  }  // work rounds
  // epilogue: rows = co ((lane>>4)*4 + r), cols = kflat (lane & 15)
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int kf = slice * SLICE + (wid * NB + j) * 16 + li;
      if (kf >= KF) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = i * 16 + g * 4 + r;
        if (co < Cout) atomicAdd(dw + (long)co * KF + kf, acc[i][j][r]);
      }
    }
}

// ================================================================================================
// first layer: C=4 (packed RGB), Cout=8, fused bias + PReLU + 2x2 max-pool, pixel-pair MFMA
// ================================================================================================
// With Cout=8 the generic kernel wastes half of every 16-row MFMA (and half of the epilogue lanes).
// Here the A operand's rows 0-7 are the 8 filters and rows 8-15 the same filters shifted one
// column right - they fit the spare kw'=KS column of the KWP=KS+1 padded K for free - so with the
// B columns at even pixels p, one v_mfma_f32_16x16x32_bf16 yields all 8 channels of pixels p and
// p+1: 32 output pixels per MFMA, every lane busy in the epilogue, and each B fragment is one
// aligned 16-byte LDS read (the pair (p+kw, p+kw+1) starts on an even pixel).  Lane (px, g) owns
// pixel 2*px + (g>>1) of its 32-pixel fragment, channels 4*(g&1)..+3: z stores cover 512
// contiguous bytes per wave instruction; the horizontal pool partner is lane ^ 32, the vertical one
// the wave's other fragment (rows 2*rp, 2*rp+1).
// Layout: 256x4-pixel... tiles of TW=64 x TH=4 pixels, mirrored ring of 2*HR halo rows walked
// down a column strip, next rows prefetched into registers during the MFMAs (as conv_fwd_strip_k).
// SPARSE: the sparse pool record (EPI_POOLS) instead of the full-resolution z: `z` receives, per
// pooled element, the z of the window's argmax ([N][H/2][W/2][8]) and `argout` its position
// q = 2*dh + dw (first maximum in q order wins, as in the dense backward).
// U8: x is the raw decoded image batch, uint8 [N][H][W][3]: a pixel pair is three 2-byte buffer
// loads (6 bytes instead of 16), and the /255 + zero 4th channel of pack_u8rgb4_k happens in
// registers before the LDS store (same rounding), so no packed bf16 copy of the input is written.

template <int KS, bool SPARSE, bool U8 = false>
__global__ __launch_bounds__(256, 5) void conv1_pair_pool_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                         const float* __restrict__ bias, const float* __restrict__ alpha,
                                                         bf16_t* __restrict__ z, bf16_t* __restrict__ pooled,
                                                         uint8_t* __restrict__ argout, int N, int H,
                                                         int W, int pad, int tiles_h, int tiles_w,
                                                         int* __restrict__ wq, int wchunk) {
  constexpr int C = 4, TW = 64, TH = 4;
  constexpr int KWP = KS + 1;
  static_assert((KWP * C) % 8 == 0 && TH < 2 * (KS - 1), "pair layout needs KS odd >= 5");
  constexpr int HR = TH + KS - 1, HC = TW + KWP - 1;
  constexpr int HP = (HC + 1) / 2;      // 16-byte pixel pairs per halo row
  constexpr int ROWE = HP * 8;          // halo row pitch (elements), 16-byte aligned
  constexpr int KROW = KWP * C, KTOT = KS * KROW, KSTEPS = (KTOT + 31) / 32;
  constexpr int HALO = 2 * HR * ROWE;   // mirrored ring
  constexpr int PFN = (HR * HP + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t smem[HALO + 8];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int px = lane & 15, g = lane >> 4;
  if (tid < 8) smem[HALO + tid] = 0;

  // A operand: row px = filter (px & 7), shifted one column right when px >= 8
  bf16x8_t wreg[KSTEPS];
  {
    const int co = px & 7, sh = px >> 3;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int kf = ks * 32 + 8 * g;
      U4 v = zero4();
      if (kf < KTOT) {
        const int kh = kf / KROW, kw = (kf - kh * KROW) / C;   // kw even
        const bf16_t* wp = w + ((long)co * KS + kh) * KS * C;
        const int a = kw - sh, b = kw + 1 - sh;
        if (a >= 0 && a < KS) { const U2 t = *(const U2*)(wp + a * C); v.x = t.x; v.y = t.y; }
        if (b >= 0 && b < KS) { const U2 t = *(const U2*)(wp + b * C); v.z = t.x; v.w = t.y; }
      }
      wreg[ks] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  const int cc = 4 * (g & 1);
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias) { const float4 b4 = *(const float4*)(bias + cc); bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w; }

  // halo slots: (row, pixel pair) per thread
  int pr_r[PFN], pr_c[PFN];
#pragma unroll
  for (int p = 0; p < PFN; ++p) {
    const int idx = tid + p * 256;
    pr_r[p] = idx / HP;
    pr_c[p] = idx - pr_r[p] * HP;
  }
  U4 pf[PFN];
  U8Pair pu[U8 ? PFN : 1];
  const Rsrc xr = make_rsrc(x, U8 ? u8_rsrc_bytes((long)N * H * W * 3) : (uint32_t)((long)N * H * W * C * 2));
  auto load_rows = [&](int n, int iw0, int ih_first, int nrows) {  // padding reads 0 (PTG_OOB)
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      const int ih = ih_first + pr_r[p], iw = iw0 + 2 * pr_c[p];
      const bool ok = pr_r[p] < nrows && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      if constexpr (U8) {  // iw is even and W is even: the pair's second pixel is in the row too
        pu[p] = u8pair_load(xr, (uint32_t)((n * H + ih) * W + iw) * 3u, ok);
      } else {
        const uint32_t img = (uint32_t)(n * H * W * C) * 2u;
        pf[p] = bload16(xr, ok ? img + (uint32_t)((ih * W + iw) * C) * 2u : PTG_OOB);
      }
    }
  };
  auto store_rows = [&](int nrows, int slot_first) {
#pragma unroll
    for (int p = 0; p < PFN; ++p) {
      if (pr_r[p] < nrows) {
        int slot = slot_first + pr_r[p];
        slot = slot >= HR ? slot - HR : slot;
        bf16_t* dst = smem + slot * ROWE + pr_c[p] * 8;
        U4 v = pf[p];
        if constexpr (U8) v = u8pair_to_bf16x8(pu[p]);
        *(U4*)dst = v;
        *(U4*)(dst + HR * ROWE) = v;
      }
    }
  };

  const int hf = wid & 1, rp = wid >> 1;   // this wave: columns hf*32.., rows 2*rp, 2*rp+1
  const int S = N * tiles_w;
  const long T = (long)S * tiles_h;
  __shared__ int s_wq;
  for (int round = 0;; ++round) {  // static range, or work-queue chunks (see conv_fwd_strip_k)
  int t0, t1;
  if (wq) {
    const long c = wq_next(wq, round, blockIdx.x, gridDim.x, (int)((T + wchunk - 1) / wchunk), &s_wq);
    t0 = (int)min(T, c * wchunk);
    t1 = (int)min(T, (c + 1) * wchunk);
  } else {
    if (round) break;
    t0 = (int)(T * blockIdx.x / gridDim.x);
    t1 = (int)(T * (blockIdx.x + 1) / gridDim.x);
  }
  if (t0 >= t1) break;
  int s = t0 / tiles_h, th = t0 - s * tiles_h;
  {
    const int n = s / tiles_w, ow0 = (s - n * tiles_w) * TW;
    load_rows(n, ow0 - pad, th * TH - pad, HR);
    store_rows(HR, (th * TH) % HR);
  }
  __syncthreads();
  const int PH = H >> 1, PW = W >> 1;
  for (int t = t0; t < t1; ++t) {
    const int n = s / tiles_w, ow0 = (s - n * tiles_w) * TW, oh0 = th * TH;
    int s2 = s, th2 = th + 1;
    if (th2 >= tiles_h) { s2 = s + 1; th2 = 0; }
    const bool has_next = t + 1 < t1;
    const bool same_strip = s2 == s;
    const int n2 = s2 / tiles_w, ow02 = (s2 - n2 * tiles_w) * TW;
    const int nrows2 = same_strip ? TH : HR;
    const int ih2 = same_strip ? th2 * TH - pad + HR - TH : th2 * TH - pad;
    const int slot2 = same_strip ? (th2 * TH + HR - TH) % HR : (th2 * TH) % HR;
    if (has_next) load_rows(n2, ow02 - pad, ih2, nrows2);

    const int ow = ow0 + hf * 32 + 2 * px + (g >> 1);
    float4 al[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int oh = oh0 + 2 * rp + i;
      al[i] = (oh < H && ow < W) ? *(const float4*)(alpha + ((long)oh * W + ow) * 8 + cc) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int wstart = oh0 % HR;
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int kf = ks * 32 + 8 * g;
      const int kh = kf / KROW, kw = (kf - kh * KROW) / C;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int off = kf < KTOT ? (wstart + 2 * rp + i + kh) * ROWE + (hf * 32 + 2 * px + kw) * C : HALO;
        const bf16x8_t xf = *(const bf16x8_t*)(smem + off);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[ks], xf, acc[i], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done reading the halo window
    if (has_next) store_rows(nrows2, slot2);

    float y[2][4], zr[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int oh = oh0 + 2 * rp + i;
      const float a4[4] = {al[i].x, al[i].y, al[i].z, al[i].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        zr[i][r] = bf2f(f2bf(acc[i][r] + bv[r]));
        y[i][r] = zr[i][r] > 0.f ? zr[i][r] : a4[r] * zr[i][r];
      }
      if (!SPARSE && oh < H && ow < W)
        *(U2*)(z + (((long)n * H + oh) * W + ow) * 8 + cc) =
            U2{pack_bf(zr[i][0], zr[i][1]), pack_bf(zr[i][2], zr[i][3])};
    }
    const int ph = (oh0 >> 1) + rp, pw = (ow0 >> 1) + hf * 16 + px;
    float pm[4];
    if constexpr (SPARSE) {
      // window (dh, dw): this lane holds dw = g >> 1 for dh = 0, 1; the partner lane ^ 32 the other dw
      float zs[4];
      uint32_t qs = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float py0 = __shfl_xor(y[0][r], 32, 64), py1 = __shfl_xor(y[1][r], 32, 64);
        const float pz0 = __shfl_xor(zr[0][r], 32, 64), pz1 = __shfl_xor(zr[1][r], 32, 64);
        const bool odd = g >= 2;
        const float yq[4] = {odd ? py0 : y[0][r], odd ? y[0][r] : py0, odd ? py1 : y[1][r], odd ? y[1][r] : py1};
        const float zq[4] = {odd ? pz0 : zr[0][r], odd ? zr[0][r] : pz0, odd ? pz1 : zr[1][r], odd ? zr[1][r] : pz1};
        float b = yq[0], bz = zq[0];
        uint32_t a = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q)
          if (yq[q] > b) { b = yq[q]; bz = zq[q]; a = q; }
        pm[r] = b;
        zs[r] = bz;
        qs |= a << (8 * r);
      }
      if (g < 2 && ph < PH && pw < PW) {
        const long po = (((long)n * PH + ph) * PW + pw) * 8 + cc;
        *(U2*)(pooled + po) = U2{pack_bf(pm[0], pm[1]), pack_bf(pm[2], pm[3])};
        *(U2*)(z + po) = U2{pack_bf(zs[0], zs[1]), pack_bf(zs[2], zs[3])};
        *(uint32_t*)(argout + po) = qs;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = fmaxf(y[0][r], y[1][r]);
        pm[r] = fmaxf(v, __shfl_xor(v, 32, 64));
      }
      if (g < 2 && ph < PH && pw < PW)
        *(U2*)(pooled + (((long)n * PH + ph) * PW + pw) * 8 + cc) = U2{pack_bf(pm[0], pm[1]), pack_bf(pm[2], pm[3])};
    }
    if (!has_next) break;
    __syncthreads();  // next tile's halo rows visible
    s = s2;
    th = th2;
  }
  }  // work rounds
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

// Up to four flips in one launch: job j covers elements [off[j], off[j+1]) of the concatenated range.
struct FlipJobs { const bf16_t* w[4]; bf16_t* wf[4]; int Cout[4], KS[4], Cin[4], off[5]; };
__global__ __launch_bounds__(256) void conv_flip4_k(FlipJobs J) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < J.off[4]; i += gridDim.x * 256) {
    const int j = i < J.off[1] ? 0 : i < J.off[2] ? 1 : i < J.off[3] ? 2 : 3;
    const int e = i - J.off[j], Cout = J.Cout[j], KS = J.KS[j], Cin = J.Cin[j];
    const int co = e % Cout;
    int t = e / Cout;
    const int kw = t % KS; t /= KS;
    const int kh = t % KS; const int ci = t / KS;
    J.wf[j][e] = J.w[j][(((long)co * KS + (KS - 1 - kh)) * KS + (KS - 1 - kw)) * Cin + ci];
  }
}

// ------------------------------------------------------------------------------------------------
// host dispatch
// ------------------------------------------------------------------------------------------------
// workgroups of `kernel` (256 threads) that fit on the device at once (cached per kernel)
// Persistent grids are sized to OVERSUB x the resident workgroups: when another stream's kernel (an
// RCCL collective overlapping the backward on a multi-GPU node) holds some CUs, the workgroups that
// cannot start until a slot frees carry 1/OVERSUB of a full range instead of a whole one, bounding
// the tail.  PTG_PERSIST_OVERSUB (default 1: measured 122.7k vs 117.3k samples/s at 2 on an idle GPU) sets it.
static int persist_oversub() {
  static const int v = [] {
    const char* e = getenv("PTG_PERSIST_OVERSUB");
    const int k = e ? atoi(e) : 1;
    return k < 1 ? 1 : (k > 8 ? 8 : k);
  }();
  return v;
}

// Work-queue mode of the persistent kernels (off: static ranges; on: the data-parallel strategies
// switch it on when RCCL collectives overlap the backward).  The queue counters live in one small
// device buffer allocated and zeroed on the first (eager) launch; kernels re-arm them (wq_next).
static int g_persist_dynamic = -1;
static bool persist_dynamic() {
  if (g_persist_dynamic < 0) {
    const char* e = getenv("PTG_PERSIST_DYNAMIC");
    g_persist_dynamic = (e && e[0] == '1') ? 1 : 0;
  }
  return g_persist_dynamic == 1;
}
// queue counters (one per channel group / weight slice), zeroed once; every launch leaves them at 0.
// One counter block PER STREAM: kernels of one stream run in order, but a dgrad on the step's stream
// and a wgrad on the side stream run at the same time and must never draw from the same counter
// (each would skip the chunks the other claimed).  Up to 16 streams; beyond that -> static ranges.
static int* work_queue(int slots, hipStream_t s) {
  constexpr int NSTREAM = 16, SLOTS = 64;
  static int* buf = nullptr;
  static hipStream_t owner[NSTREAM];
  static int used = 0;
  if (!buf) {
    if (hipMalloc(&buf, NSTREAM * SLOTS * sizeof(int)) != hipSuccess ||
        hipMemset(buf, 0, NSTREAM * SLOTS * sizeof(int)) != hipSuccess) {
      buf = nullptr;
      return nullptr;
    }
  }
  if (slots > SLOTS) return nullptr;
  for (int i = 0; i < used; ++i)
    if (owner[i] == s) return buf + i * SLOTS;
  if (used == NSTREAM) return nullptr;
  owner[used] = s;
  return buf + (used++) * SLOTS;
}
// tiles per claimed chunk: ~4 chunks per workgroup, at least 4 tiles (each chunk restarts the halo;
// 8 per workgroup cost 14% on CNN-B1 with the claim not yet prefetched)
static int wq_chunk(long tiles, int groups) {
  long c = tiles / ((long)groups * 4);
  return (int)(c < 4 ? 4 : c);
}

template <int C, int KS, int NF, int TW, int TH, int E, bool WLDS, int COS, bool SPIN = false>
static int launch_fwd_k(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, void* arg,
                        int N, int H, int W, int Cout, int pad, hipStream_t s) {
  constexpr bool RING = TH < 2 * (KS - 1);
  constexpr int KTOT = KS * Kwp<C, KS>::v * C, KSTEPS = (KTOT + 31) / 32, MFR = TH * TW / 16;
  constexpr bool WREG = KSTEPS * NF <= 8;
  constexpr bool KSPLIT = !WLDS && !WREG && MFR / 4 <= 2 && MFR * NF <= 16;
  const auto kern = conv_fwd_strip_k<C, KS, NF, TW, TH, E, RING, KSPLIT, WLDS, COS, SPIN>;
  static const int resident = ptg_resident_blocks((const void*)kern);
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const long tiles = (long)N * tw * th;
  // persistent: one wave of resident workgroups, each walking a contiguous range of tiles
  // (COS groups of workgroups each cover all tiles for their slice of output channels)
  const int grid = (int)std::min<long>(tiles * COS, (long)resident * persist_oversub() / COS * COS);
  int* wq = persist_dynamic() ? work_queue(COS, s) : nullptr;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)w, bias, alpha, (bf16_t*)z,
                     (bf16_t*)aux, (uint8_t*)arg, N, H, W, Cout, pad, th, tw, wq, wq_chunk(tiles, grid / COS));
  PTG_RETURN_LAUNCH();
}

// PTG_CONV1_PAIR=0 routes the first layer (C=4, Cout=8) through the generic strip kernel
static bool conv1_pair_enabled() {
  static const bool on = [] {
    const char* e = getenv("PTG_CONV1_PAIR");
    return !(e && e[0] == '0');
  }();
  return on;
}

// PTG_CONV_WLDS=0 keeps the per-wave global weight loads (A/B switch for the LDS-resident path)
static bool conv_wlds_enabled() {
  static const bool on = [] {
    const char* e = getenv("PTG_CONV_WLDS");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int C, int KS, int NF, int TW, int TH, int E, bool SPIN = false>
static int launch_fwd_e(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, void* arg, int N,
                        int H, int W, int Cout, int pad, hipStream_t s) {
  constexpr int KTOT = KS * Kwp<C, KS>::v * C, KSTEPS = (KTOT + 31) / 32;
  constexpr bool WREG = KSTEPS * NF <= 8;
  // measured on CNN-B1 shapes: C=16/32 gain 10-37 %; C=64 (4x16 tiles, one fragment per wave) is
  // LDS-read bound at one workgroup per CU and loses to the k-split global-weight path
  if constexpr (C >= 8 && C <= 32 && !WREG) {
    // LDS budget: halo rows + weight slice must leave the block resident (160 KiB per CU)
    constexpr int HR = TH + KS - 1, HC = TW + Kwp<C, KS>::v - 1;
    constexpr int HALO_B = (HR < 2 * (KS - 1) ? 2 : 1) * HR * (HC * FwdPitch<C>::pix + FwdPitch<C>::rowpad) * 2;
    constexpr int WB = NF * 16 * (KSTEPS * 32 + 8) * 2;
    if (conv_wlds_enabled()) {
      if constexpr (HALO_B + WB <= 150 * 1024)
        return launch_fwd_k<C, KS, NF, TW, TH, E, true, 1, SPIN>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, s);
      else if constexpr (NF % 2 == 0 && HALO_B + WB / 2 <= 150 * 1024)
        return launch_fwd_k<C, KS, NF / 2, TW, TH, E, true, 2, SPIN>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, s);
    }
  }
  return launch_fwd_k<C, KS, NF, TW, TH, E, false, 1, SPIN>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, s);
}

template <int C, int KS, int NF, int TW, int TH>
static int launch_fwd(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, void* arg, int N,
                      int H, int W, int Cout, int pad, int epi, hipStream_t s) {
  if (epi == EPI_POOL) return launch_fwd_e<C, KS, NF, TW, TH, EPI_POOL>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, s);
  if (epi == EPI_POOLS) return launch_fwd_e<C, KS, NF, TW, TH, EPI_POOLS>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, s);
  if (epi == EPI_PRELU) return launch_fwd_e<C, KS, NF, TW, TH, EPI_PRELU>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, s);
  return launch_fwd_e<C, KS, NF, TW, TH, EPI_Z>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, s);
}

template <int C, int KS, int NF>
static int fwd_by_c(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, void* arg, int N,
                    int H, int W, int Cout, int pad, int epi, hipStream_t s) {
  // tile shapes: TH x TW pixels, halo fits LDS, 4 waves with equal fragment counts
  if constexpr (C == 4) return launch_fwd<C, KS, NF, 64, 4>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
  else if constexpr (C == 8) return launch_fwd<C, KS, NF, 32, 8>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
  else if constexpr (C == 16) return launch_fwd<C, KS, NF, 16, 8>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
  else if constexpr (C == 32) return launch_fwd<C, KS, NF, 8, 16>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
  else return launch_fwd<C, KS, NF, 4, 16>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
}

template <int C, int KS>
static int fwd_by_nf(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, void* arg, int N,
                     int H, int W, int Cout, int pad, int epi, hipStream_t s) {
  if (Cout <= 16) return fwd_by_c<C, KS, 1>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
  if (Cout <= 32) return fwd_by_c<C, KS, 2>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
  if (Cout <= 64) return fwd_by_c<C, KS, 4>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
  return (int)hipErrorInvalidValue;
}

template <int KS>
static int fwd_by_cin(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, void* arg, int N,
                      int H, int W, int C, int Cout, int pad, int epi, hipStream_t s) {
  switch (C) {
    case 4: return fwd_by_nf<4, KS>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
    case 8: return fwd_by_nf<8, KS>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
    case 16: return fwd_by_nf<16, KS>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
    case 32: return fwd_by_nf<32, KS>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
    case 64: return fwd_by_nf<64, KS>(x, w, bias, alpha, z, aux, arg, N, H, W, Cout, pad, epi, s);
    default: return (int)hipErrorInvalidValue;
  }
}

template <int C, int KS, int TW, int TH, int MF, bool SPARSE = false>
static int launch_wgrad(const void* x, const void* dz, float* dw, int N, int H, int W, int Cout, int pad, hipStream_t s,
                        const void* argq = nullptr) {
  constexpr bool RING = TH < 2 * (KS - 1);
  constexpr int KF = KS * KS * C;
  constexpr int NB = KF > 512 ? 4 : 2;
  const auto kern = conv_wgrad_strip_k<C, KS, TW, TH, MF, NB, RING, SPARSE>;
  static const int resident = ptg_resident_blocks((const void*)kern);
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const long tiles = (long)N * tw * th;
  const int nslices = (KF + 64 * NB - 1) / (64 * NB);
  int chunks = (resident * persist_oversub() + nslices - 1) / nslices;
  if (chunks > tiles) chunks = (int)tiles;
  int* wq = persist_dynamic() ? work_queue(nslices, s) : nullptr;
  hipLaunchKernelGGL(kern, dim3(chunks * nslices), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)dz, dw, N, H, W,
                     Cout, pad, th, tw, nslices, (const uint8_t*)argq, wq, wq_chunk(tiles, chunks));
  PTG_RETURN_LAUNCH();
}

// C = 32 / 64 weight gradients at small batch (<= WG_SMALL_N samples): wider tiles (16 x 8 and 20 x 16
// pixels instead of 8 x 8 and 4 x 16).  Every workgroup flushes its 64 x (64 * NB) partial sums with
// one fp32 atomic each, and with few samples a workgroup owns ~one small tile, so the flush dominated:
// CNN-B1 b32 L4 / L5 wgrad 37.2 / 37.6 -> 30.5 / 23.3 us; at b256 the small tiles stay faster
// (82.8 / 71.8 vs 111.6 / 91.3 us, profiles/r6_ab_wgrad_tiles.txt).
static int wg_small_n() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PTG_WG_SMALL_N");
    v = e && *e ? atoi(e) : 0;  // 0 since the unrolled (KSEP) loop: the large-batch tiles win at
    //                              b32 / b64 too (profiles/r6_ab_wgrad_small_tiles_after_unroll.txt)
  }
  return v;
}
template <int C, int KS, int MF, bool SPARSE>
static int wgrad_by_c(const void* x, const void* dz, float* dw, int N, int H, int W, int Cout, int pad, hipStream_t s,
                      const void* argq) {
  const bool small = N <= wg_small_n();
  if constexpr (C == 4) return launch_wgrad<C, KS, 64, 4, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
  else if constexpr (C == 8) return launch_wgrad<C, KS, 32, 8, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
  else if constexpr (C == 16) return launch_wgrad<C, KS, 16, 8, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
  else if constexpr (C == 32) {
    if (small) return launch_wgrad<C, KS, 16, 8, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
    return launch_wgrad<C, KS, 8, 8, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
  } else {
    if (small) return launch_wgrad<C, KS, 20, 16, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
    return launch_wgrad<C, KS, 4, 16, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
  }
}

template <int KS, int MF, bool SPARSE = false>
static int wgrad_by_cin(const void* x, const void* dz, float* dw, int N, int H, int W, int C, int Cout, int pad,
                        hipStream_t s, const void* argq = nullptr) {
  switch (C) {
    case 4: return wgrad_by_c<4, KS, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
    case 8: return wgrad_by_c<8, KS, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
    case 16: return wgrad_by_c<16, KS, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
    case 32: return wgrad_by_c<32, KS, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
    case 64: return wgrad_by_c<64, KS, MF, SPARSE>(x, dz, dw, N, H, W, Cout, pad, s, argq);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace ptgc

using namespace ptgc;

extern "C" {

// stride-1 'same'-style conv with halo tiling. C in {4,8,16,32,64}, Cout % 8 == 0 and <= 64, KS in {3,5}.
// epi: 0 = z only, 1 = z + maxpool2x2(prelu(z)) into aux (H, W even), 2 = z + prelu(z) into aux,
// 3 = maxpool2x2(prelu(z)) into aux + argmax z into z ([N][H/2][W/2][Cout]) + argmax q into arg.
int ptg_conv2d_fwd_halo(const void* x, const void* w, const float* bias, const float* alpha, void* z, void* aux, void* arg, int N,
                        int H, int W, int C, int Cout, int KS, int pad, int epi, hipStream_t s) {
  if (Cout % 8 || Cout > 64 || !ptg_fits_2g((long)N * H * W * C * 2)) return (int)hipErrorInvalidValue;
  if ((epi == EPI_POOL || epi == EPI_POOLS) && ((H & 1) || (W & 1))) return (int)hipErrorInvalidValue;
  if (epi < EPI_Z || epi > EPI_POOLS) return (int)hipErrorInvalidValue;
  if (C == 4 && Cout == 8 && KS == 5 && (epi == EPI_POOL || epi == EPI_POOLS) && pad == 2 && conv1_pair_enabled()) {
    const auto kern = epi == EPI_POOLS ? conv1_pair_pool_k<5, true> : conv1_pair_pool_k<5, false>;
    static const int res_dense = ptg_resident_blocks((const void*)conv1_pair_pool_k<5, false>);
    static const int res_sparse = ptg_resident_blocks((const void*)conv1_pair_pool_k<5, true>);
    const int resident = epi == EPI_POOLS ? res_sparse : res_dense;
    const int th = (H + 3) / 4, tw = (W + 63) / 64;
    const long tiles = (long)N * th * tw;
    const int grid = (int)std::min<long>(tiles, (long)resident * persist_oversub());
    int* wq = persist_dynamic() ? work_queue(1, s) : nullptr;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)w, bias, alpha, (bf16_t*)z,
                       (bf16_t*)aux, (uint8_t*)arg, N, H, W, pad, th, tw, wq, wq_chunk(tiles, grid));
    PTG_RETURN_LAUNCH();
  }
  if (KS == 5) return fwd_by_cin<5>(x, w, bias, alpha, z, aux, arg, N, H, W, C, Cout, pad, epi, s);
  if (KS == 3) return fwd_by_cin<3>(x, w, bias, alpha, z, aux, arg, N, H, W, C, Cout, pad, epi, s);
  return (int)hipErrorInvalidValue;
}

// Data gradient of a 5x5 'same' conv whose output was 2x2-pooled, from its SPARSE dZ record:
// dzsel / argq [N][H/2][W/2][C] (dZ at each window's argmax, the argmax q); wf = the flipped filter
// [Cout][5][5][C]; dx [N][H][W][Cout] (bf16).  C in {16, 32} (CNN-B1 layers 2 / 3), Cout <= 64.
int ptg_conv2d_dgrad_halo_sparse(const void* dzsel, const void* argq, const void* wf, void* dx, int N, int H, int W,
                                 int C, int Cout, int KS, int pad, hipStream_t s) {
  if (KS != 5 || (H & 1) || (W & 1) || Cout % 8 || Cout > 64 || !ptg_fits_2g((long)N * H * W * Cout * 2))
    return (int)hipErrorInvalidValue;
  const int NF = Cout <= 16 ? 1 : (Cout <= 32 ? 2 : 4);
#define PTG_SPD(CV, TWV, THV)                                                                                        \
  {                                                                                                                  \
    if (NF == 1) return launch_fwd_e<CV, 5, 1, TWV, THV, EPI_Z, true>(dzsel, wf, nullptr, nullptr, dx, nullptr,       \
                                                                      (void*)argq, N, H, W, Cout, pad, s);          \
    if (NF == 2) return launch_fwd_e<CV, 5, 2, TWV, THV, EPI_Z, true>(dzsel, wf, nullptr, nullptr, dx, nullptr,       \
                                                                      (void*)argq, N, H, W, Cout, pad, s);          \
    return launch_fwd_e<CV, 5, 4, TWV, THV, EPI_Z, true>(dzsel, wf, nullptr, nullptr, dx, nullptr, (void*)argq, N, H, \
                                                         W, Cout, pad, s);                                          \
  }
  if (C == 16) PTG_SPD(16, 16, 8)
  if (C == 32) PTG_SPD(32, 8, 16)
#undef PTG_SPD
  return (int)hipErrorInvalidValue;
}

// dw (fp32, [Cout][KS][KS][C]) += weight gradient; caller zeroes dw.
int ptg_conv2d_wgrad_halo(const void* x, const void* dz, float* dw, int N, int H, int W, int C, int Cout, int KS,
                          int pad, hipStream_t s) {
  if (Cout % 8 || Cout > 64 || !ptg_fits_2g((long)N * H * W * C * 2) || !ptg_fits_2g((long)N * H * W * Cout * 2))
    return (int)hipErrorInvalidValue;
  const int MF = Cout <= 16 ? 1 : (Cout <= 32 ? 2 : 4);
#define PTG_WG(KSV, MFV) return wgrad_by_cin<KSV, MFV>(x, dz, dw, N, H, W, C, Cout, pad, s)
  if (KS == 5) { if (MF == 1) PTG_WG(5, 1); if (MF == 2) PTG_WG(5, 2); PTG_WG(5, 4); }
  if (KS == 3) { if (MF == 1) PTG_WG(3, 1); if (MF == 2) PTG_WG(3, 2); PTG_WG(3, 4); }
#undef PTG_WG
  return (int)hipErrorInvalidValue;
}

// Weight gradient from the sparse pool record of dZ: dzsel / argq are [N][H/2][W/2][Cout] (H, W even);
// only the 5x5 layers of the reference CNN (first layer: no dgrad needs a dense dZ) are instantiated.
int ptg_conv2d_wgrad_halo_sparse(const void* x, const void* dzsel, const void* argq, float* dw, int N, int H, int W,
                                 int C, int Cout, int KS, int pad, hipStream_t s) {
  if (Cout % 8 || Cout > 64 || KS != 5 || (H & 1) || (W & 1) || !ptg_fits_2g((long)N * H * W * C * 2))
    return (int)hipErrorInvalidValue;
  const int MF = Cout <= 16 ? 1 : (Cout <= 32 ? 2 : 4);
  if (MF == 1) return wgrad_by_cin<5, 1, true>(x, dzsel, dw, N, H, W, C, Cout, pad, s, argq);
  if (MF == 2) return wgrad_by_cin<5, 2, true>(x, dzsel, dw, N, H, W, C, Cout, pad, s, argq);
  return wgrad_by_cin<5, 4, true>(x, dzsel, dw, N, H, W, C, Cout, pad, s, argq);
}

// First layer straight from the raw uint8 [N][H][W][3] image batch (no packed bf16 copy): the
// 5x5 Cout=8 conv + bias + PReLU + 2x2 max-pool with the sparse pool record (epi 3 of
// ptg_conv2d_fwd_halo), and its weight gradient from the sparse dZ record.  H, W even, pad 2.
int ptg_conv1_pool_sparse_u8(const void* x_u8, const void* w, const float* bias, const float* alpha, void* zsel,
                             void* pooled, void* arg, int N, int H, int W, hipStream_t s) {
  if ((H & 1) || (W & 1) || !ptg_fits_2g((long)N * H * W * 3)) return (int)hipErrorInvalidValue;
  const auto kern = conv1_pair_pool_k<5, true, true>;
  static const int resident = ptg_resident_blocks((const void*)kern);
  const int th = (H + 3) / 4, tw = (W + 63) / 64;
  const long tiles = (long)N * th * tw;
  const int grid = (int)std::min<long>(tiles, (long)resident * persist_oversub());
  int* wq = persist_dynamic() ? work_queue(1, s) : nullptr;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, (const bf16_t*)x_u8, (const bf16_t*)w, bias, alpha,
                     (bf16_t*)zsel, (bf16_t*)pooled, (uint8_t*)arg, N, H, W, 2, th, tw, wq, wq_chunk(tiles, grid));
  PTG_RETURN_LAUNCH();
}

int ptg_conv1_wgrad_sparse_u8(const void* x_u8, const void* dzsel, const void* argq, float* dw, int N, int H, int W,
                              int Cout, hipStream_t s) {
  if (Cout != 8 || (H & 1) || (W & 1) || !ptg_fits_2g((long)N * H * W * 3)) return (int)hipErrorInvalidValue;
  constexpr int C = 4, KS = 5, TW = 64, TH = 4, MF = 1;
  constexpr bool RING = TH < 2 * (KS - 1);
  constexpr int KF = KS * KS * C;
  constexpr int NB = KF > 512 ? 4 : 2;
  const auto kern = conv_wgrad_strip_k<C, KS, TW, TH, MF, NB, RING, true, true>;
  static const int resident = ptg_resident_blocks((const void*)kern);
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const long tiles = (long)N * tw * th;
  const int nslices = (KF + 64 * NB - 1) / (64 * NB);
  int chunks = (resident * persist_oversub() + nslices - 1) / nslices;
  if (chunks > tiles) chunks = (int)tiles;
  int* wq = persist_dynamic() ? work_queue(nslices, s) : nullptr;
  hipLaunchKernelGGL(kern, dim3(chunks * nslices), dim3(256), 0, s, (const bf16_t*)x_u8, (const bf16_t*)dzsel, dw, N,
                     H, W, Cout, 2, th, tw, nslices, (const uint8_t*)argq, wq, wq_chunk(tiles, chunks));
  PTG_RETURN_LAUNCH();
}

// dynamic: 1 = persistent conv kernels claim tile chunks from a work queue, 0 = static ranges,
// -1 = PTG_PERSIST_DYNAMIC (default static).
int ptg_set_persist_mode(int dynamic, hipStream_t s) {
  (void)s;
  g_persist_dynamic = dynamic < 0 ? -1 : (dynamic ? 1 : 0);
  return 0;
}

int ptg_conv_flip_weights4(int n, const void* w0, void* wf0, int Cout0, int KS0, int Cin0, const void* w1, void* wf1,
                           int Cout1, int KS1, int Cin1, const void* w2, void* wf2, int Cout2, int KS2, int Cin2,
                           const void* w3, void* wf3, int Cout3, int KS3, int Cin3, hipStream_t s) {
  if (n < 1 || n > 4) return (int)hipErrorInvalidValue;
  FlipJobs J{};
  const void* ws[4] = {w0, w1, w2, w3};
  void* wfs[4] = {wf0, wf1, wf2, wf3};
  const int co[4] = {Cout0, Cout1, Cout2, Cout3}, ks[4] = {KS0, KS1, KS2, KS3}, ci[4] = {Cin0, Cin1, Cin2, Cin3};
  J.off[0] = 0;
  for (int j = 0; j < 4; ++j) {
    const bool on = j < n;
    J.w[j] = (const bf16_t*)ws[j]; J.wf[j] = (bf16_t*)wfs[j];
    J.Cout[j] = on ? co[j] : 1; J.KS[j] = on ? ks[j] : 1; J.Cin[j] = on ? ci[j] : 1;
    J.off[j + 1] = J.off[j] + (on ? co[j] * ks[j] * ks[j] * ci[j] : 0);
  }
  const int blocks = std::min(1024, (J.off[4] + 255) / 256);
  hipLaunchKernelGGL(conv_flip4_k, dim3(std::max(blocks, 1)), dim3(256), 0, s, J);
  PTG_RETURN_LAUNCH();
}

int ptg_conv_flip_weights(const void* w, void* wf, int Cout, int KS, int Cin, hipStream_t s) {
  const int total = Cout * KS * KS * Cin;
  hipLaunchKernelGGL(conv_flip_k, dim3((total + 255) / 256), dim3(256), 0, s, (const bf16_t*)w, (bf16_t*)wf, Cout, KS,
                     Cin);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"

PTG_CHECK_STATUS(conv)
