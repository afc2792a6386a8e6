// MFMA GEMM engine for gfx950 + implicit-GEMM 2-D convolution (fwd / dgrad / wgrad).
//
// One templated main loop serves every matmul-shaped op of the training runtime:
//   Dense fwd / dX / dW (TF `Dense`, reference train_tf_ps.py:332-335, :366-367) and
//   Conv2D fwd / dgrad / wgrad (TF `Conv2D(k, 5, padding="same")`, train_tf_ps.py:351-363).
// The reference gets these from cuBLAS/cuDNN inside TensorFlow; here they are hand-written
// around v_mfma_f32_16x16x32_bf16 (bf16 in, fp32 accumulate).
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"):
//   * 256 threads = 4 waves arranged WM x WN; each wave owns a (BM/WM) x (BN/WN) sub-tile made
//     of 16x16 MFMA fragments; accumulators indexed by fragment repeat only.
//   * BK = 64 K-step, two LDS buffers; the next tile's global loads are issued into registers
//     before the MFMAs of the current tile and written to the other LDS buffer after them,
//     one barrier per K-step.
//   * Operands whose source memory is k-contiguous are staged as [rows][BK] images (fragment =
//     one 16-byte ds_read); operands whose source is row-contiguous (transposed use of a matrix,
//     the im2col^T of wgrad, the dgrad filter) are staged k-major exactly as they sit in memory
//     and read with the transposed LDS read ds_read_b64_tr_b16 - every LDS store is a 16-byte
//     vector in both cases.
//   * Operand "loaders" turn (row, k) into a 16-byte vector: plain matrices, the implicit im2col
//     gather of a NHWC activation, the flipped/transposed filter of dgrad, the im2col^T of wgrad.
//     The convolution therefore never materialises its im2col matrix.
//   * blockIdx.x is remapped XCD-aware (T1) so tiles that share operand panels share an L2;
//     blockIdx.y indexes split-K slices (fp32 atomic epilogue).
#include "common.h"

// nontemporal loads/stores of the fused Adam epilogue (on: CNN-B1 b256 1.608 -> 1.600 ms,
// profiles/r4_ab_adam_nt.txt); -DPTG_ADAM_NT=0 for the A/B
#ifndef PTG_ADAM_NT
#define PTG_ADAM_NT 1
#endif

// p/m/v groups of 8 whose loads the fused-Adam epilogue issues before its first update (per thread)
#ifndef PTG_ADAM_V4
#define PTG_ADAM_V4 1
#endif
#ifndef PTG_ADAM_PRE4
#define PTG_ADAM_PRE4 8
#endif
#ifndef PTG_ADAM_PRE
#define PTG_ADAM_PRE 4
#endif

#include <cstdlib>
#include <type_traits>
#include <utility>

namespace ptg {

constexpr int BK = 64;

// ------------------------------------------------------------------------------------------
// Operand loaders. K_CONTIG loaders return elements (r, k..k+7); the others return
// elements (r..r+7, k).  Ctx caches the per-row decode so the K loop only does k-math.
//
// Every operand is read with buffer loads (cdna_hip_programming.md T8) through a descriptor built
// once per workgroup from the kernel arguments: a 32-bit byte offset per lane, and every element
// the GEMM must see as zero (rows past M/N, k past K, the convolution's zero padding) gets the
// offset OOB, which the hardware range check returns as 0 - no branch per load, no 64-bit address
// arithmetic.  Operands must be smaller than 2 GiB (checked on the host).
// ------------------------------------------------------------------------------------------
constexpr uint32_t OOB = PTG_OOB;
PTG_DEV U4 join(U2 a, U2 b) { U4 v; v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y; return v; }

template <int VEC>
struct MatK {  // element(r,k) = p[r*ld + k]; ld % VEC == 0, K % 8 == 0 or zero-padded rows
  static constexpr bool K_CONTIG = true;
  static constexpr bool DMA16 = VEC == 8;  // 8 consecutive k = one aligned 16-B chunk (off())
  const bf16_t* p; long ld; int R; int K; uint32_t bytes;
  struct Ctx { uint32_t row; };
  PTG_DEV Rsrc rsrc() const { return make_rsrc(p, bytes); }
  PTG_DEV Ctx ctx(int r) const { Ctx c; c.row = r < R ? (uint32_t)(r * ld) * 2u : OOB; return c; }
  // byte offset of elements (r, k..k+7) for the LDS-DMA path (VEC == 8 only)
  PTG_DEV uint32_t off(const Ctx& c, int k) const { return (k < K && c.row != OOB) ? c.row + 2u * k : OOB; }
  PTG_DEV U4 load(Rsrc rs, const Ctx& c, int k) const {
    const uint32_t off = k < K ? c.row + 2u * k : OOB;
    if constexpr (VEC == 8) {
      return bload16(rs, off);
    } else {
      return join(bload8(rs, off), bload8(rs, k + 4 < K ? off + 8u : OOB));
    }
  }
};

struct MatMN {  // element(r,k) = p[k*ld + r]; R % 8 == 0, ld % 8 == 0
  static constexpr bool K_CONTIG = false;
  const bf16_t* p; long ld; int R; int K; uint32_t bytes;
  struct Ctx { uint32_t col; };
  PTG_DEV Rsrc rsrc() const { return make_rsrc(p, bytes); }
  PTG_DEV Ctx ctx(int r0) const { Ctx c; c.col = r0 < R ? 2u * r0 : OOB; return c; }
  PTG_DEV U4 load(Rsrc rs, const Ctx& c, int k) const {
    return bload16(rs, k < K ? c.col + (uint32_t)(k * ld) * 2u : OOB);
  }
};

// Implicit im2col of an NHWC activation: row m = output pixel (n, oh, ow); k = (kh, kw, ci).
// C is a power of two; CVEC = 8 (C % 8 == 0, one 16-B load) or 4 (C == 4, two 8-B loads).
template <int CVEC>
struct ConvFwdA {
  static constexpr bool K_CONTIG = true;
  static constexpr bool DMA16 = CVEC == 8;
  const bf16_t* x; int H, W, C, logC, OH, OW, KW, stride, pad, M, Kc; uint32_t bytes;
  FastDiv fKW, fOHW, fOW;  // set by init(): the per-load (kh, kw) and per-row pixel decodes without idiv
  ConvFwdA& init() {
    fKW = fastdiv(KW); fOHW = fastdiv(OH * OW); fOW = fastdiv(OW);
    bytes = (uint32_t)((long)(M / (OH * OW)) * H * W * C * 2);
    return *this;
  }
  struct Ctx { uint32_t img; int ih0, iw0; };
  PTG_DEV Rsrc rsrc() const { return make_rsrc(x, bytes); }
  PTG_DEV Ctx ctx(int m) const {
    Ctx c;
    const bool ok = m < M;
    if (!ok) m = 0;
    const int ohw = OH * OW;
    const int n = (int)fOHW.div(m), rem = m - n * ohw, oh = (int)fOW.div(rem), ow = rem - oh * OW;
    c.img = ok ? (uint32_t)(n * H * W * C) * 2u : OOB;
    c.ih0 = oh * stride - pad; c.iw0 = ow * stride - pad;
    return c;
  }
  PTG_DEV uint32_t at(const Ctx& c, int k) const {
    const int pos = k >> logC, ci = k & (C - 1);
    const int kh = (int)fKW.div(pos), kw = pos - kh * KW;
    const int ih = c.ih0 + kh, iw = c.iw0 + kw;
    const bool ok = (k < Kc) && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    return ok ? c.img + (uint32_t)((ih * W + iw) * C + ci) * 2u : OOB;
  }
  PTG_DEV uint32_t off(const Ctx& c, int k) const { return c.img == OOB ? OOB : at(c, k); }
  PTG_DEV U4 load(Rsrc rs, const Ctx& c, int k) const {
    if constexpr (CVEC == 8) return bload16(rs, at(c, k));
    else return join(bload8(rs, at(c, k)), bload8(rs, at(c, k + 4)));
  }
};

// dgrad filter: rows = input channel ci (8 at a time), k = (kh', kw', co) of the flipped filter
// W'[ci][kh'][kw'][co] = W[co][KH-1-kh'][KW-1-kw'][ci]. W is stored [Cout][KH][KW][Cin].
struct ConvDgradB {
  static constexpr bool K_CONTIG = false;
  const bf16_t* w; int Cin, Cout, logCout, KH, KW, Kc2; uint32_t bytes;
  FastDiv fKW;
  ConvDgradB& init() { fKW = fastdiv(KW); bytes = (uint32_t)((long)Cout * KH * KW * Cin * 2); return *this; }
  struct Ctx { uint32_t ci0; };
  PTG_DEV Rsrc rsrc() const { return make_rsrc(w, bytes); }
  PTG_DEV Ctx ctx(int r0) const { Ctx c; c.ci0 = r0 < Cin ? 2u * r0 : OOB; return c; }
  PTG_DEV U4 load(Rsrc rs, const Ctx& c, int k) const {
    const int pos = k >> logCout, co = k & (Cout - 1);
    const int kh = (int)fKW.div(pos), kw = pos - kh * KW;
    const uint32_t off = c.ci0 + (uint32_t)((co * KH * KW + (KH - 1 - kh) * KW + (KW - 1 - kw)) * Cin) * 2u;
    return bload16(rs, k < Kc2 ? off : OOB);
  }
};

// wgrad im2col^T: rows = kc = (kh, kw, ci) (8 at a time), k = output pixel (n, oh, ow).
template <int CVEC>
struct ConvWgradB {
  static constexpr bool K_CONTIG = false;
  const bf16_t* x; int H, W, C, logC, OH, OW, KW, stride, pad, P, Kc; uint32_t bytes;
  FastDiv fKW, fOHW, fOW;  // the per-load pixel decode (k -> n, oh, ow) is the loader's hot path
  ConvWgradB& init() {
    fKW = fastdiv(KW); fOHW = fastdiv(OH * OW); fOW = fastdiv(OW);
    bytes = (uint32_t)((long)(P / (OH * OW)) * H * W * C * 2);
    return *this;
  }
  struct Ctx { int dh0, dw0, dh1, dw1; uint32_t ci0, ci1; };
  PTG_DEV Rsrc rsrc() const { return make_rsrc(x, bytes); }
  PTG_DEV Ctx ctx(int r0) const {
    Ctx c;
    int pos = r0 >> logC;
    int q = (int)fKW.div(pos);
    c.dh0 = q - pad; c.dw0 = pos - q * KW - pad; c.ci0 = r0 < Kc ? 2u * (r0 & (C - 1)) : OOB;
    const int r1 = r0 + 4;
    pos = r1 >> logC;
    q = (int)fKW.div(pos);
    c.dh1 = q - pad; c.dw1 = pos - q * KW - pad; c.ci1 = r1 < Kc ? 2u * (r1 & (C - 1)) : OOB;
    return c;
  }
  PTG_DEV uint32_t at(int k, int n, int oh, int ow, int dh, int dw, uint32_t ci) const {
    const int ih = oh * stride + dh, iw = ow * stride + dw;
    const bool ok = k < P && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    return ok ? ci + (uint32_t)(((n * H + ih) * W + iw) * C) * 2u : OOB;
  }
  PTG_DEV U4 load(Rsrc rs, const Ctx& c, int k) const {
    const int ohw = OH * OW;
    const int n = (int)fOHW.div(k), rem = k - n * ohw, oh = (int)fOW.div(rem), ow = rem - oh * OW;
    if constexpr (CVEC == 8) {
      return bload16(rs, at(k, n, oh, ow, c.dh0, c.dw0, c.ci0));
    } else {
      return join(bload8(rs, at(k, n, oh, ow, c.dh0, c.dw0, c.ci0)), bload8(rs, at(k, n, oh, ow, c.dh1, c.dw1, c.ci1)));
    }
  }
};

// ------------------------------------------------------------------------------------------
// Epilogues: called per accumulator element (m, n) inside bounds.
// ------------------------------------------------------------------------------------------
enum { ACT_NONE = 0, ACT_RELU = 1 };

// Every epilogue has a per-element operator() and vec8(m, n, v, cnt) for the 8 consecutive
// columns n..n+cnt-1 of row m (the kernel stages the tile through LDS so each lane owns 8
// consecutive outputs: 16-byte stores instead of 2-byte ones).
PTG_DEV bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// PTG_EPI_NT: the bf16 epilogue outputs (conv / GEMM activations, read back only by a later kernel)
// written with nontemporal stores: ResNet-50 b128 14.02 / 13.99 -> 13.93 / 13.87 ms, CNN-B1 b256
// 1.546 / 1.531 -> 1.536 / 1.530 ms (profiles/r5_ab_epi_nt.txt); -DPTG_EPI_NT=0 for the A/B
#ifndef PTG_EPI_NT
#define PTG_EPI_NT 1
#endif
PTG_DEV void bf16_store8(bf16_t* p, float* v, int cnt, bool accum) {
  if (cnt == 8 && al16(p)) {
    if (accum) {
      float e[8];
      unpack8(*(const U4*)p, e);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += e[j];
    }
#if PTG_EPI_NT
    typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
    const U4 w = pack8(v);
    __builtin_nontemporal_store(u4nt{w.x, w.y, w.z, w.w}, (u4nt*)p);
#else
    *(U4*)p = pack8(v);
#endif
    return;
  }
  for (int j = 0; j < cnt; ++j) p[j] = f2bf(accum ? v[j] + bf2f(p[j]) : v[j]);
}

// stats (optional, [BN_G][2][N] fp32): the following BatchNormalization's batch statistics - sum and
// sum of squares of the STORED (bf16-rounded) outputs per column - reduced per tile in LDS and added
// into partial group (tile row % BN_G), the layout bn_finalize_k reads; the separate bn_stats pass
// over z disappears.
constexpr int EPI_BN_G = 64;  // == bn.hip BN_G
// Backward form (bz != nullptr, with stats): the GEMM is the data gradient feeding a Conv -> BN -> ReLU
// block whose forward z is bz ([M][ldc] bf16): each output is first masked by that block's ReLU,
// g = (z*bsc + bsh > 0) ? v : 0 (no mask when bsc is null), stored as g, and the statistics are the
// BN backward's sums - sum g and sum g*z per column, bn_bwd_reduce_k's partial layout - so that
// reduction pass over dy and z disappears (graph_ops.ConvBNOp.bwd_bn_op).
struct EpiBf16 {  // out[m*ldc+n] = act(acc + bias[n]) (+ out if accum) as bf16 (optionally also fp32)
  static constexpr bool VEC = true;
  static constexpr bool STATS = true;
  bf16_t* out; long ldc; const float* bias; int act; float* out32; int accum; float* stats = nullptr;
  const bf16_t* bz = nullptr; const float* bsc = nullptr; const float* bsh = nullptr;
  // backward form: mask v in place with the block's ReLU and return its z values in zz
  PTG_DEV void bwd_prep(int m, int n, float* v, int cnt, float* zz) const {
    const bf16_t* zp = bz + (long)m * ldc + n;
    if (cnt == 8 && al16(zp)) {
      unpack8(*(const U4*)zp, zz);
    } else {
      for (int j = 0; j < 8; ++j) zz[j] = j < cnt ? bf2f(zp[j]) : 0.f;
    }
    if (bsc) {
      for (int j = 0; j < cnt; ++j) v[j] = fmaf(zz[j], bsc[n + j], bsh[n + j]) > 0.f ? v[j] : 0.f;
    }
  }
  PTG_DEV void operator()(int m, int n, float v) const {
    if (bias) v += bias[n];
    if (act == ACT_RELU) v = fmaxf(v, 0.f);
    bf16_t* p = out + (long)m * ldc + n;
    if (accum) v += bf2f(*p);
    *p = f2bf(v);
    if (out32) out32[(long)m * ldc + n] = v;
  }
  PTG_DEV void vec8(int m, int n, float* v, int cnt) const {
    if (bias && cnt == 8 && al16(bias + n)) {
      const float4 b0 = *(const float4*)(bias + n), b1 = *(const float4*)(bias + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    } else if (bias) {
      for (int j = 0; j < cnt; ++j) v[j] += bias[n + j];
    }
    if (act == ACT_RELU)
      for (int j = 0; j < cnt; ++j) v[j] = fmaxf(v[j], 0.f);
    if (out32) {
      for (int j = 0; j < cnt; ++j) out32[(long)m * ldc + n + j] = accum ? v[j] + bf2f(out[(long)m * ldc + n + j]) : v[j];
    }
    bf16_store8(out + (long)m * ldc + n, v, cnt, accum);
  }
};
// Strided scatter (dgrad of a 1x1 stride-s conv): GEMM row m = output pixel (n, oh, ow) lands on
// input pixel (n, oh*s, ow*s) of an [N][H][W][ldc] tensor; the other input pixels are untouched.
struct EpiBf16Remap {
  static constexpr bool VEC = true;
  bf16_t* out; long ldc; int OH, OW, H, W, s, accum;
  PTG_DEV void operator()(int m, int n, float v) const {
    const int ohw = OH * OW, b = m / ohw, rem = m - b * ohw, oh = rem / OW, ow = rem - oh * OW;
    bf16_t* p = out + (((long)b * H + oh * s) * W + ow * s) * ldc + n;
    if (accum) v += bf2f(*p);
    *p = f2bf(v);
  }
  PTG_DEV void vec8(int m, int n, float* v, int cnt) const {
    const int ohw = OH * OW, b = m / ohw, rem = m - b * ohw, oh = rem / OW, ow = rem - oh * OW;
    bf16_store8(out + (((long)b * H + oh * s) * W + ow * s) * ldc + n, v, cnt, accum);
  }
};
struct EpiF32 {  // out[m*ldc+n] (=|+=) act(acc + bias)
  static constexpr bool VEC = true;  // staged through LDS: each lane stores 8 consecutive fp32 (2 x 16 B)
  float* out; long ldc; const float* bias; int act; int accumulate;
  PTG_DEV void operator()(int m, int n, float v) const {
    if (bias) v += bias[n];
    if (act == ACT_RELU) v = fmaxf(v, 0.f);
    float* p = out + (long)m * ldc + n;
    if (accumulate) *p += v; else *p = v;
  }
  PTG_DEV void vec8(int m, int n, float* v, int cnt) const {
    float* p = out + (long)m * ldc + n;
    if (cnt == 8 && al16(p) && (!bias || al16(bias + n))) {
      float4 a = make_float4(v[0], v[1], v[2], v[3]), b = make_float4(v[4], v[5], v[6], v[7]);
      if (bias) {
        const float4 b0 = *(const float4*)(bias + n), b1 = *(const float4*)(bias + n + 4);
        a.x += b0.x; a.y += b0.y; a.z += b0.z; a.w += b0.w; b.x += b1.x; b.y += b1.y; b.z += b1.z; b.w += b1.w;
      }
      if (act == ACT_RELU) {
        a.x = fmaxf(a.x, 0.f); a.y = fmaxf(a.y, 0.f); a.z = fmaxf(a.z, 0.f); a.w = fmaxf(a.w, 0.f);
        b.x = fmaxf(b.x, 0.f); b.y = fmaxf(b.y, 0.f); b.z = fmaxf(b.z, 0.f); b.w = fmaxf(b.w, 0.f);
      }
      if (accumulate) {
        const float4 e0 = *(const float4*)p, e1 = *(const float4*)(p + 4);
        a.x += e0.x; a.y += e0.y; a.z += e0.z; a.w += e0.w; b.x += e1.x; b.y += e1.y; b.z += e1.z; b.w += e1.w;
      }
      *(float4*)p = a;
      *(float4*)(p + 4) = b;
      return;
    }
    for (int j = 0; j < cnt; ++j) (*this)(m, n + j, v[j]);
  }
};
// Adam applied in the epilogue of the weight-gradient GEMM (1-GPU training): the gradient tile
// never goes to HBM - each lane reads its 8 parameters' p/m/v, updates them and writes p, m, v and
// the bf16 mirror (26 bytes per parameter instead of the 4-byte gradient store + the 30-byte
// adam_k pass).  Same arithmetic as adam_k (nn_eltwise.hip); lr_dev[1] (device step state, HIP
// graphs) overrides lr_t.
struct EpiAdam {
  static constexpr bool VEC = true;
  // the kernel issues PRE lanes' worth of p/m/v loads before any update is stored (the epilogue's
  // stores could alias later loads, so the compiler would otherwise serialise 8 HBM round trips)
  static constexpr int PRE = PTG_ADAM_PRE;
  struct Pre { float4 P[2], Mm[2], V[2]; };
  float* p; float* mo; float* ve; bf16_t* pbf; long ldc; float lr_t, b1, b2, eps, gscale; const float* lr_dev;
  PTG_DEV float lr() const { return lr_dev ? lr_dev[1] : lr_t; }
  PTG_DEV static bool fast(long i, int cnt) { return cnt == 8 && (i & 7) == 0; }
  PTG_DEV void upd(float& pp, float& mm, float& vv, float g, float l) const {
    const float gj = g * gscale;
    mm = b1 * mm + (1.f - b1) * gj;
    vv = b2 * vv + (1.f - b2) * gj * gj;
    pp -= l * mm / (sqrtf(vv) + eps);
  }
  PTG_DEV void operator()(int m, int n, float v) const {
    const long i = (long)m * ldc + n;
    float pp = p[i], mm = mo[i], vv = ve[i];
    upd(pp, mm, vv, v, lr());
    p[i] = pp; mo[i] = mm; ve[i] = vv;
    pbf[i] = f2bf(pp);
  }
#if PTG_ADAM_NT
  // streaming hints: the 1.1 GB of CNN-B1's Dense state is touched once per step
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  PTG_DEV static float4 ld4(const float* a) {
    const f4v v = __builtin_nontemporal_load((const f4v*)a);
    return make_float4(v.x, v.y, v.z, v.w);
  }
  PTG_DEV static void st4(float* a, float4 v) {
    const f4v w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (f4v*)a);
  }
  PTG_DEV static void st16(bf16_t* a, U4 v) {
    const u4v w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (u4v*)a);
  }
#else
  PTG_DEV static float4 ld4(const float* a) { return *(const float4*)a; }
  PTG_DEV static void st4(float* a, float4 v) { *(float4*)a = v; }
  PTG_DEV static void st16(bf16_t* a, U4 v) { *(U4*)a = v; }
#endif
  PTG_DEV void preload(int m, int n, int cnt, Pre& r) const {
    const long i = (long)m * ldc + n;
    if (!fast(i, cnt)) return;
    r.P[0] = ld4(p + i); r.P[1] = ld4(p + i + 4);
    r.Mm[0] = ld4(mo + i); r.Mm[1] = ld4(mo + i + 4);
    r.V[0] = ld4(ve + i); r.V[1] = ld4(ve + i + 4);
  }
  PTG_DEV void vec8_pre(int m, int n, float* v, int cnt, Pre& r) const {
    const long i = (long)m * ldc + n;
    if (!fast(i, cnt)) {
      for (int j = 0; j < cnt; ++j) (*this)(m, n + j, v[j]);
      return;
    }
    const float l = lr();
    float o[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float* pp = &r.P[h].x; float* mm = &r.Mm[h].x; float* vv = &r.V[h].x;
#pragma unroll
      for (int j = 0; j < 4; ++j) { upd(pp[j], mm[j], vv[j], v[4 * h + j], l); o[4 * h + j] = pp[j]; }
    }
    st4(p + i, r.P[0]); st4(p + i + 4, r.P[1]);
    st4(mo + i, r.Mm[0]); st4(mo + i + 4, r.Mm[1]);
    st4(ve + i, r.V[0]); st4(ve + i + 4, r.V[1]);
    st16(pbf + i, pack8(o));
  }
#if PTG_ADAM_V4
  // 4 columns per lane (PTG_ADAM_V4, default): 32 lanes cover a 128-column row, so every load /
  // store instruction of a wave is two fully contiguous 512-byte runs (the 8-column form issues each
  // instruction as 64 16-byte pieces at a 32-byte stride, every line touched by two instructions).
  // CNN-B1 step: b256 1.555 -> 1.527 ms, b32 0.619 -> 0.600 ms (profiles/r6_ab_adam_v4.txt); an
  // 8-deep preload batch (PTG_ADAM_PRE4) beat 4.  A one-stage / half-tile-staging low-LDS form of
  // this GEMM lost at b256 (profiles/r6_ab_adam_lowlds_rejected.txt) and was removed.
  static constexpr int PRE4 = PTG_ADAM_PRE4;
  struct Pre4 { float4 P, Mm, V; };
  PTG_DEV void preload4(int m, int n, int cnt, Pre4& r) const {
    const long i = (long)m * ldc + n;
    if (cnt != 4 || (i & 3)) return;
    r.P = ld4(p + i); r.Mm = ld4(mo + i); r.V = ld4(ve + i);
  }
  PTG_DEV void vec4_pre(int m, int n, const float* v, int cnt, Pre4& r) const {
    const long i = (long)m * ldc + n;
    if (cnt != 4 || (i & 3)) {
      for (int j = 0; j < cnt; ++j) (*this)(m, n + j, v[j]);
      return;
    }
    const float l = lr();
    float* pp = &r.P.x; float* mm = &r.Mm.x; float* vv = &r.V.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) upd(pp[j], mm[j], vv[j], v[j], l);
    st4(p + i, r.P); st4(mo + i, r.Mm); st4(ve + i, r.V);
    U2 b;
    b.x = pack_bf(pp[0], pp[1]);
    b.y = pack_bf(pp[2], pp[3]);
    *(U2*)(pbf + i) = b;
  }
#endif
  PTG_DEV void vec8(int m, int n, float* v, int cnt) const {
    Pre r;
    preload(m, n, cnt, r);
    vec8_pre(m, n, v, cnt, r);
  }
};
template <class E, class = void> struct EpiPre { static constexpr int v = 0; };
template <class E> struct EpiPre<E, std::void_t<decltype(E::PRE)>> { static constexpr int v = E::PRE; };
template <class E, class = void> struct EpiPre4 { static constexpr int v = 0; };
template <class E> struct EpiPre4<E, std::void_t<decltype(E::PRE4)>> { static constexpr int v = E::PRE4; };
struct EpiAtomic {  // split-K: out[m*ldc+n] += acc  (device-scope fp32 atomic, no return)
  static constexpr bool VEC = false;  // lane-consecutive atomics coalesce; 8-per-lane runs do not
  float* out; long ldc;
  PTG_DEV void operator()(int m, int n, float v) const { atomicAdd(out + (long)m * ldc + n, v); }
  PTG_DEV void vec8(int m, int n, float* v, int cnt) const {
    float* p = out + (long)m * ldc + n;
    for (int j = 0; j < cnt; ++j) atomicAdd(p + j, v[j]);
  }
};

template <class E, class = void> struct EpiStats { static constexpr bool v = false; };
template <class E> struct EpiStats<E, std::void_t<decltype(E::STATS)>> { static constexpr bool v = E::STATS; };

// backward form: sums of the stored (bf16-rounded, masked) gradient g and of g*z
PTG_DEV void stats_acc8_bwd(const float* v, const float* zz, int cnt, float* s, float* q) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float r = j < cnt ? bf2f(f2bf(v[j])) : 0.f;
    s[j] += r;
    q[j] = fmaf(r, zz[j], q[j]);
  }
}
// per-thread column sums of the stored (bf16-rounded) values
PTG_DEV void stats_acc8(const float* v, int cnt, float* s, float* q) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float r = j < cnt ? bf2f(f2bf(v[j])) : 0.f;
    s[j] += r;
    q[j] = fmaf(r, r, q[j]);
  }
}
// Block reduction of the per-thread sums into the tile's TN columns: thread tid always owns column
// group tid % (TN/8) in the epilogue loops, so the lanes of a wave that share a group are reduced
// with xor shuffles, each wave writes its TN partial sums to LDS (no LDS atomics: 16-way contended
// ds_add_f32 made this flush cost more than the bn_stats pass it replaces), and TN threads add the
// waves' rows into partial group tm % EPI_BN_G with 2 * TN global atomics.  `scratch` (>= 2 * TN *
// NT/64 floats) is the epilogue's LDS staging area.
template <int TN, int NT>
PTG_DEV void stats_flush(float* stats, int N, int tm, int n0, float* s, float* q, float* scratch) {
  constexpr int G = TN / 8, NW = NT / 64;
  static_assert(G <= 64, "column groups per wave");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int o = G; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += __shfl_xor(s[j], o, 64);
      q[j] += __shfl_xor(q[j], o, 64);
    }
  }
  __syncthreads();  // every thread is done reading the staged C tile
  if (lane < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      scratch[(w * 2) * TN + lane * 8 + j] = s[j];
      scratch[(w * 2 + 1) * TN + lane * 8 + j] = q[j];
    }
  }
  __syncthreads();
  float* g = stats + (long)(tm % EPI_BN_G) * 2 * N;
  for (int i = tid; i < TN; i += NT) {
    if (n0 + i < N) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) { a += scratch[(ww * 2) * TN + i]; b += scratch[(ww * 2 + 1) * TN + i]; }
      atomicAdd(g + n0 + i, a);
      atomicAdd(g + N + n0 + i, b);
    }
  }
}

// ------------------------------------------------------------------------------------------
// The main loop.
// ------------------------------------------------------------------------------------------
// LDS images (one __shared__ array, two stages):
//   K_CONTIG operand: [rows][LDK] (k contiguous, 16-B padded rows): 16-B vector stores, fragment
//     reads of 8 (or 2 x 4) consecutive k.
//   row-contiguous operand: [BK][rows + 16] (k-major, exactly the global layout of a transposed
//     use): 16-B vector stores of 8 consecutive rows, fragments read with the gfx950 transposed
//     LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md T10).  The +16 row padding makes the
//     8 k-rows a half-wave touches land on distinct 8-dword bank groups.
// When either operand is row-contiguous both use the k order in which lane group g holds
// k = {4g..4g+3, 16+4g..16+4g+3} of each 32-wide MFMA step (any k permutation shared by A and B
// leaves the product unchanged); the tr-read half-wave then reads 8 consecutive k-rows.
typedef __attribute__((ext_vector_type(4))) short gs16x4_t;
typedef __attribute__((address_space(3))) gs16x4_t glds_s16x4_t;

PTG_DEV U2 gtr_read(const bf16_t* p) {
  return __builtin_bit_cast(U2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((glds_s16x4_t*)(p)));
}

template <class L, int R>
struct LdsImg {
  static constexpr int LD = L::K_CONTIG ? BK + 8 : R + 16;
  static constexpr int ELEMS = L::K_CONTIG ? R * LD : BK * LD;
};

// PF: how many K-steps ahead the global loads run (register slots; 1 = the next step only).  With one
// 4-wave workgroup per CU (256-row skinny tiles) one K-step of MFMAs is shorter than an HBM round
// trip, so those tiles load 2 steps ahead.
// Work item of a split-K GEMM workgroup.  kchunk > 0: tile = XCD-remapped blockIdx.x (tiles sharing
// a panel share an L2), split = blockIdx.y.  kchunk < 0 (split-major, the host's choice when there
// are >= 8 splits): every XCD takes whole K-splits - all tiles of a split run on one XCD, so both
// operands' K-range panels of that split are fetched into its L2 once and shared by every tile
// (the Dense forward, M = 256, N = 2048, 16 splits: the tile mapping fetched each weight panel on two
// XCDs and each activation panel on all eight).  Workgroups go to XCDs round-robin by linear id.
PTG_DEV void split_xcd_map(int& t, int& split, int& kchunk) {
  if (kchunk > 0) {
    t = xcd_remap(blockIdx.x, gridDim.x);
    split = blockIdx.y;
    return;
  }
  kchunk = -kchunk;
  const int tiles = gridDim.x, total = tiles * gridDim.y;
  const int lin = blockIdx.y * tiles + blockIdx.x;
  const int item = (lin % 8) * (total / 8) + lin / 8;  // host guarantees total % 8 == 0
  split = item / tiles;
  t = item - split * tiles;
}

template <int BM, int BN, int WM, int WN, class LA, class LB, class EPI, int PF = 1>
__global__ __launch_bounds__(256) void gemm_kernel(LA la, LB lb, EPI epi, int M, int N, int K,
                                                   int kchunk) {
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(FM >= 1 && FN >= 1, "wave tile >= 16x16");
  constexpr bool PERM = !LA::K_CONTIG || !LB::K_CONTIG;
  using IA = LdsImg<LA, BM>;
  using IB = LdsImg<LB, BN>;
  constexpr int AV = BM * BK / 8, BV = BN * BK / 8;  // 16-B vectors per operand tile
  constexpr int AI = (AV + 255) / 256, BI = (BV + 255) / 256;
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (N + BN - 1) / BN;
  int t, split;
  split_xcd_map(t, split, kchunk);
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = split * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke) return;
  const int nk = (ke - kb + BK - 1) / BK;

  typename LA::Ctx ca[AI]; int akk[AI], aoff[AI]; bool aon[AI];
  typename LB::Ctx cb[BI]; int bkk[BI], boff[BI]; bool bon[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int v = tid + i * 256;
    aon[i] = v < AV;
    if constexpr (LA::K_CONTIG) {
      const int r = v / (BK / 8), kv = v % (BK / 8);
      ca[i] = la.ctx(m0 + r); akk[i] = kv * 8; aoff[i] = r * IA::LD + kv * 8;
    } else {
      const int kk = v / (BM / 8), rv = v % (BM / 8);
      ca[i] = la.ctx(m0 + rv * 8); akk[i] = kk; aoff[i] = kk * IA::LD + rv * 8;
    }
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int v = tid + i * 256;
    bon[i] = v < BV;
    if constexpr (LB::K_CONTIG) {
      const int r = v / (BK / 8), kv = v % (BK / 8);
      cb[i] = lb.ctx(n0 + r); bkk[i] = kv * 8; boff[i] = r * IB::LD + kv * 8;
    } else {
      const int kk = v / (BN / 8), rv = v % (BN / 8);
      cb[i] = lb.ctx(n0 + rv * 8); bkk[i] = kk; boff[i] = kk * IB::LD + rv * 8;
    }
  }

  static_assert(PF >= 1 && PF <= 3, "register prefetch depth");
  U4 ra[PF][AI], rb[PF][BI];
  const Rsrc rsA = la.rsrc(), rsB = lb.rsrc();
  // slots past the tile (AV or BV not a multiple of 256) exist only in the last unrolled slot
  constexpr bool AFULL = AV % 256 == 0, BFULL = BV % 256 == 0;
  auto gload = [&](auto slot, int k0) {
    constexpr int sl = decltype(slot)::value;
#pragma unroll
    for (int i = 0; i < AI; ++i) ra[sl][i] = la.load(rsA, ca[i], k0 + akk[i]);
#pragma unroll
    for (int i = 0; i < BI; ++i) rb[sl][i] = lb.load(rsB, cb[i], k0 + bkk[i]);
  };
  auto sstore = [&](auto slot, int stage) {
    constexpr int sl = decltype(slot)::value;
    bf16_t* sA = smem + stage * STAGE;
    bf16_t* sB = sA + IA::ELEMS;
#pragma unroll
    for (int i = 0; i < AI; ++i)
      if (AFULL || aon[i]) *(U4*)(sA + aoff[i]) = ra[sl][i];
#pragma unroll
    for (int i = 0; i < BI; ++i)
      if (BFULL || bon[i]) *(U4*)(sB + boff[i]) = rb[sl][i];
  };
  // fragment (16 rows x 32 k at k-offset kk) of an LDS image; rows start at `row0`
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = (li & 3) * 4;
  auto frag_k = [&](const bf16_t* img, int ld, int row0, int kk) -> bf16x8_t {  // [rows][k] image
    const bf16_t* r = img + (row0 + li) * ld + kk;
    U4 v;
    if constexpr (PERM) {
      const U2 a = *(const U2*)(r + 4 * g), b = *(const U2*)(r + 16 + 4 * g);
      v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
    } else {
      v = *(const U4*)(r + 8 * g);
    }
    return __builtin_bit_cast(bf16x8_t, v);
  };
  auto frag_t = [&](const bf16_t* img, int ld, int row0, int kk) -> bf16x8_t {  // [k][rows] image
    const U2 a = gtr_read(img + (kk + 4 * g + q) * ld + row0 + p4);
    const U2 b = gtr_read(img + (kk + 16 + 4 * g + q) * ld + row0 + p4);
    U4 v; v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
    return __builtin_bit_cast(bf16x8_t, v);
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int cur) {
    const bf16_t* sA = smem + cur * STAGE;
    const bf16_t* sB = sA + IA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8_t af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (LA::K_CONTIG) af[i] = frag_k(sA, IA::LD, wm * WTM + i * 16, kk);
        else af[i] = frag_t(sA, IA::LD, wm * WTM + i * 16, kk);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (LB::K_CONTIG) bfr[j] = frag_k(sB, IB::LD, wn * WTN + j * 16, kk);
        else bfr[j] = frag_t(sB, IB::LD, wn * WTN + j * 16, kk);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // K-step t's tile sits in register slot t % PF from its load (PF steps ahead) until it is written to
  // LDS stage t & 1 at the end of step t-1; step t then refills slot t % PF with tile t + PF.
  gload(std::integral_constant<int, 0>{}, kb);
  sstore(std::integral_constant<int, 0>{}, 0);
  if constexpr (PF >= 2) { if (1 < nk) gload(std::integral_constant<int, 1>{}, kb + BK); }
  if constexpr (PF >= 3) { if (2 < nk) gload(std::integral_constant<int, 2>{}, kb + 2 * BK); }
  __syncthreads();
  for (int it = 0; it < nk; it += PF) {
    auto step = [&](auto u) {
      constexpr int U = decltype(u)::value;
      const int t = it + U;
      if (t >= nk) return;
      if constexpr (PF == 1) {
        if (t + 1 < nk) gload(std::integral_constant<int, 0>{}, kb + (t + 1) * BK);
      } else {
        if (t + PF < nk) gload(std::integral_constant<int, U>{}, kb + (t + PF) * BK);
      }
      compute(t & 1);
      // the other stage was last read in step t-1, which ended with a barrier
      if (t + 1 < nk) sstore(std::integral_constant<int, (U + 1) % PF>{}, (t + 1) & 1);
      __syncthreads();
    };
    step(std::integral_constant<int, 0>{});
    if constexpr (PF >= 2) step(std::integral_constant<int, 1>{});
    if constexpr (PF >= 3) step(std::integral_constant<int, 2>{});
  }

  // C/D map of mfma_f32_16x16x32: col = lane&15, row = (lane>>4)*4 + r
  if constexpr (!EPI::VEC) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WTN + j * 16 + (lane & 15);
          if (m < M && n < N) epi(m, n, acc[i][j][r]);
        }
    return;
  }
  // bf16 outputs: stage the fp32 tile through LDS, then every thread hands 8 consecutive columns
  // of a row to the epilogue (one 16-byte store instead of eight 2-byte ones).
  constexpr int CP = BN + 4;
  static_assert(!EPI::VEC || BM * CP * 4 <= 2 * STAGE * 2, "C tile must fit in the staging LDS");
  float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wm * WTM + i * 16 + (lane >> 4) * 4 + r) * CP + wn * WTN + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  constexpr int NV = BM * BN / 8;
  if constexpr (EpiPre4<EPI>::v > 0 && (BM * BN / 4) % 256 == 0) {
    // read-modify-write epilogue, 4 consecutive columns per lane (EpiAdam with PTG_ADAM_V4)
    constexpr int NIT = BM * BN / 4 / 256, B = EpiPre4<EPI>::v < NIT ? EpiPre4<EPI>::v : NIT;
#pragma unroll
    for (int b0 = 0; b0 < NIT; b0 += B) {
      typename EPI::Pre4 pre[B];
      int mm[B], nn[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int v = (b0 + u) * 256 + tid;
        const int row = v / (BN / 4), c4 = v - row * (BN / 4);
        mm[u] = m0 + row; nn[u] = n0 + c4 * 4;
        if (mm[u] < M && nn[u] < N) epi.preload4(mm[u], nn[u], min(4, N - nn[u]), pre[u]);
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        if (mm[u] >= M || nn[u] >= N) continue;
        const int v = (b0 + u) * 256 + tid;
        const int row = v / (BN / 4), c4 = v - row * (BN / 4);
        const float4 a = *(const float4*)(cs + row * CP + c4 * 4);
        const float vals[4] = {a.x, a.y, a.z, a.w};
        epi.vec4_pre(mm[u], nn[u], vals, min(4, N - nn[u]), pre[u]);
      }
    }
    return;
  } else if constexpr (EpiPre<EPI>::v > 0 && NV % 256 == 0) {
    // read-modify-write epilogue: a batch of lanes' operand loads first, then the updates
    constexpr int NIT = NV / 256, B = EpiPre<EPI>::v < NIT ? EpiPre<EPI>::v : NIT;
#pragma unroll
    for (int b0 = 0; b0 < NIT; b0 += B) {
      typename EPI::Pre pre[B];
      int mm[B], nn[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int v = (b0 + u) * 256 + tid;
        const int row = v / (BN / 8), c8 = v - row * (BN / 8);
        mm[u] = m0 + row; nn[u] = n0 + c8 * 8;
        if (mm[u] < M && nn[u] < N) epi.preload(mm[u], nn[u], min(8, N - nn[u]), pre[u]);
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        if (mm[u] >= M || nn[u] >= N) continue;
        const int v = (b0 + u) * 256 + tid;
        const int row = v / (BN / 8), c8 = v - row * (BN / 8);
        const float4 a = *(const float4*)(cs + row * CP + c8 * 8), b = *(const float4*)(cs + row * CP + c8 * 8 + 4);
        float vals[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        epi.vec8_pre(mm[u], nn[u], vals, min(8, N - nn[u]), pre[u]);
      }
    }
    return;
  }
  float st_s[8], st_q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
  if constexpr (EpiStats<EPI>::v && NV % 256 == 0 && 256 % (BN / 8) == 0) {
    if (epi.stats && epi.bz) {
      // backward BN form: every z vector of this thread's NV/256 output groups is loaded up front
      // (independent 16-B loads in flight instead of one exposed load per group), and the block's
      // ReLU coefficients once (this thread's column group is fixed), then mask, store, sum
      constexpr int NIT = NV / 256;
      const int c8 = tid % (BN / 8), n = n0 + c8 * 8;
      U4 zv[NIT];
#pragma unroll
      for (int u = 0; u < NIT; ++u) {
        const int m = m0 + (u * 256 + tid) / (BN / 8);
        zv[u] = (m < M && n + 8 <= N) ? *(const U4*)(epi.bz + (long)m * epi.ldc + n) : zero4();
      }
      float sc[8], sh[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { sc[j] = 0.f; sh[j] = 1.f; }
      if (epi.bsc && n + 8 <= N) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { sc[j] = epi.bsc[n + j]; sh[j] = epi.bsh[n + j]; }
      }
#pragma unroll
      for (int u = 0; u < NIT; ++u) {
        const int row = (u * 256 + tid) / (BN / 8), m = m0 + row;
        if (m >= M || n >= N) continue;
        const float4 a = *(const float4*)(cs + row * CP + c8 * 8), b = *(const float4*)(cs + row * CP + c8 * 8 + 4);
        float vals[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        float zz[8];
        unpack8(zv[u], zz);
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[j] = fmaf(zz[j], sc[j], sh[j]) > 0.f ? vals[j] : 0.f;
        epi.vec8(m, n, vals, min(8, N - n));
        stats_acc8_bwd(vals, zz, min(8, N - n), st_s, st_q);
      }
      stats_flush<BN, 256>(epi.stats, N, tm, n0, st_s, st_q, cs);
      return;
    }
  }
#pragma unroll
  for (int v0 = 0; v0 < NV; v0 += 256) {
    const int v = v0 + tid;
    if (NV % 256 != 0 && v >= NV) break;
    const int row = v / (BN / 8), c8 = v - row * (BN / 8);
    const int m = m0 + row, n = n0 + c8 * 8;
    if (m >= M || n >= N) continue;
    const float4 a = *(const float4*)(cs + row * CP + c8 * 8), b = *(const float4*)(cs + row * CP + c8 * 8 + 4);
    float vals[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    if constexpr (EpiStats<EPI>::v) {
      if (epi.stats && epi.bz) {
        float zz[8];
        epi.bwd_prep(m, n, vals, min(8, N - n), zz);
        epi.vec8(m, n, vals, min(8, N - n));
        stats_acc8_bwd(vals, zz, min(8, N - n), st_s, st_q);
        continue;
      }
    }
    epi.vec8(m, n, vals, min(8, N - n));
    if constexpr (EpiStats<EPI>::v) {
      if (epi.stats) stats_acc8(vals, min(8, N - n), st_s, st_q);
    }
  }
  if constexpr (EpiStats<EPI>::v) {
    // (the host requests statistics only for N < 4096: never the skinny 80-wide tiles, whose
    // column group per thread is not fixed)
    if constexpr (256 % (BN / 8) == 0) {
      if (epi.stats) stats_flush<BN, 256>(epi.stats, N, tm, n0, st_s, st_q, cs);
    }
  }
}

// ------------------------------------------------------------------------------------------
// 256x256 tile, 8 waves (2 in M x 4 in N, 128x64 outputs = 8x4 MFMA fragments per wave), operands
// staged by LDS-DMA (buffer_load ... lds, 16 B per lane: no VGPR round trip, the hardware range
// check zero-fills padding / tails) into a two-stage ring (2 x 64 KiB): the DMA of K-tile t+1 is
// in flight during the 64 MFMAs per wave of tile t (cdna_hip_programming.md "The 256^2 template";
// 4x the MFMA work per barrier of the 128x128 kernel).  A DMA wave-instruction writes 1 KiB
// lane-linearly = 8 rows x 8 16-B k-chunks, so the bank swizzle is applied on the SOURCE side:
// lane l of a block fetches chunk (l&7) ^ ((row>>1)&7) and the fragment read un-XORs it — 16
// consecutive rows of one k-chunk then hit 16 distinct 16-B bank slots (conflict-free ds_read_b128).
// Both operands must be k-contiguous loaders with a 16-B off() (plain matrices, conv im2col).
// ------------------------------------------------------------------------------------------
template <class L, class = void> struct HasOff : std::false_type {};
// (detected from the DMA16 constant, not from off() itself: a __device__ member in an unevaluated
// host-side expression resolves differently in the host and device compilation passes)
template <class L> struct HasOff<L, std::void_t<decltype(L::DMA16)>> : std::integral_constant<bool, L::DMA16> {};

typedef __attribute__((address_space(3))) void g256_lds_t;

template <class LA, class LB, class EPI>
__global__ __launch_bounds__(512) void gemm256_kernel(LA la, LB lb, EPI epi, int M, int N, int K, int kchunk) {
  constexpr int TM = 256, TN = 256, WTM = 128, WTN = 64, FM = 8, FN = 4;
  constexpr int OPB = TM * BK * 2;          // bytes of one operand tile (32 KiB)
  constexpr int STB = 2 * OPB;              // stage bytes (A + B)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int tiles_n = (N + TN - 1) / TN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  const int kb = blockIdx.y * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke) return;
  const int nk = (ke - kb + BK - 1) / BK;

  // this lane's 4 DMA rows per operand: block b = wid*4 + j covers rows 8b..8b+7
  typename LA::Ctx ca[4];
  typename LB::Ctx cb[4];
  int kcA[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (wid * 4 + j) * 8 + (lane >> 3);
    ca[j] = la.ctx(m0 + row);
    cb[j] = lb.ctx(n0 + row);
    kcA[j] = ((lane & 7) ^ ((row >> 1) & 7)) * 8;  // source-side swizzle
  }
  const Rsrc rsA = la.rsrc(), rsB = lb.rsrc();
  // one K-tile of both operands: 4 LDS-DMA wave-instructions per operand per wave, written inline
  // (a lambda or template helper around the device-only builtin breaks the host compilation pass
  // and with it the kernel's host stub)
#define G256_DMA(stage, k0)                                                                                  \
  _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_) {                                                         \
    unsigned char* b_ = smem + (stage) * STB + (wid * 4 + j_) * 1024;                                        \
    const uint32_t oa_ = la.off(ca[j_], (k0) + kcA[j_]), ob_ = lb.off(cb[j_], (k0) + kcA[j_]);               \
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (g256_lds_t*)b_, 16, oa_, 0, 0, 0);                        \
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (g256_lds_t*)(b_ + OPB), 16, ob_, 0, 0, 0);                \
  }
  // fragment: rows row0..row0+15, k-chunk cbase + (lane>>4): one ds_read_b128
  const int fr = lane & 15, fc = lane >> 4;
  auto frag = [&](const unsigned char* img, int row0, int cbase) -> bf16x8_t {
    const int r = row0 + fr;
    const int pos = (cbase + fc) ^ ((r >> 1) & 7);
    return __builtin_bit_cast(bf16x8_t, *(const U4*)(img + r * 128 + pos * 16));
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  { G256_DMA(0, kb) }
  __syncthreads();  // waits vmcnt(0): this wave's DMA landed; the barrier publishes every wave's
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nk) {  // stage cur^1 was last read in step it-1
      G256_DMA(cur ^ 1, kb + (it + 1) * BK)
    }
    const unsigned char* sA = smem + cur * STB;
    const unsigned char* sB = sA + OPB;
#pragma unroll
    for (int kc = 0; kc < 8; kc += 4) {
      bf16x8_t af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag(sB, wn * WTN + j * 16, kc);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag(sA, wm * WTM + i * 16, kc);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

#undef G256_DMA
  // C/D map of mfma_f32_16x16x32: col = lane&15, row = (lane>>4)*4 + r
  if constexpr (!EPI::VEC) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WTN + j * 16 + (lane & 15);
          if (m < M && n < N) epi(m, n, acc[i][j][r]);
        }
    return;
  } else {
    // 4 passes of 64 rows through LDS: each thread then hands 8 consecutive columns to the epilogue
    constexpr int CP = TN + 4;
    float* cs = reinterpret_cast<float*>(smem);
    float st_s[8], st_q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
    // backward BN form (EpiBf16 bz): this thread's column group is fixed (512 % (TN/8) == 0), so its
    // ReLU coefficients load once, and each pass's 4 z vectors are issued together before the pass
    constexpr int G256 = 64 * TN / 8 / 512;
    bool bwd = false;
    float bsc8[8], bsh8[8];
    const int bc8 = tid % (TN / 8), bn8 = n0 + bc8 * 8;
    if constexpr (EpiStats<EPI>::v) {
      bwd = epi.stats && epi.bz;
#pragma unroll
      for (int j = 0; j < 8; ++j) { bsc8[j] = 0.f; bsh8[j] = 1.f; }
      if (bwd && epi.bsc && bn8 + 8 <= N) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { bsc8[j] = epi.bsc[bn8 + j]; bsh8[j] = epi.bsh[bn8 + j]; }
      }
    }
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      U4 zv[G256];
      if constexpr (EpiStats<EPI>::v) {
        if (bwd) {
#pragma unroll
          for (int u = 0; u < G256; ++u) {
            const int m = m0 + pass * 64 + (u * 512 + tid) / (TN / 8);
            zv[u] = (m < M && bn8 + 8 <= N) ? *(const U4*)(epi.bz + (long)m * epi.ldc + bn8) : zero4();
          }
        }
      }
      if (wm == (pass >> 1)) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int i = (pass & 1) * 4 + ii;
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              cs[(ii * 16 + (lane >> 4) * 4 + r) * CP + wn * WTN + j * 16 + (lane & 15)] = acc[i][j][r];
        }
      }
      __syncthreads();
#pragma unroll
      for (int v0 = 0; v0 < 64 * TN / 8; v0 += 512) {
        const int v = v0 + tid;
        const int row = v / (TN / 8), c8 = v - row * (TN / 8);
        const int m = m0 + pass * 64 + row, n = n0 + c8 * 8;
        if (m < M && n < N) {
          const float4 a = *(const float4*)(cs + row * CP + c8 * 8), b = *(const float4*)(cs + row * CP + c8 * 8 + 4);
          float vals[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          bool done = false;
          if constexpr (EpiStats<EPI>::v) {
            if (bwd) {
              float zz[8];
              unpack8(zv[v0 / 512], zz);
#pragma unroll
              for (int j = 0; j < 8; ++j) vals[j] = fmaf(zz[j], bsc8[j], bsh8[j]) > 0.f ? vals[j] : 0.f;
              epi.vec8(m, n, vals, min(8, N - n));
              stats_acc8_bwd(vals, zz, min(8, N - n), st_s, st_q);
              done = true;
            }
          }
          if (!done) {
            epi.vec8(m, n, vals, min(8, N - n));
            if constexpr (EpiStats<EPI>::v) {
              if (epi.stats) stats_acc8(vals, min(8, N - n), st_s, st_q);
            }
          }
        }
      }
      __syncthreads();
    }
    if constexpr (EpiStats<EPI>::v) {
      if (epi.stats) stats_flush<TN, 512>(epi.stats, N, tm, n0, st_s, st_q, cs);
    }
  }
}

template <class LA, class LB, class EPI>
static int launch_gemm256(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, int splits, hipStream_t s) {
  const int tiles = ptg_ceil_div(M, 256) * ptg_ceil_div(N, 256);
  if (splits < 1) splits = 1;
  int kchunk = ptg_ceil_div(ptg_ceil_div(K, splits), BK) * BK;
  if (kchunk < BK) kchunk = BK;
  splits = ptg_ceil_div(K, kchunk);
  hipLaunchKernelGGL((gemm256_kernel<LA, LB, EPI>), dim3(tiles, splits), dim3(512), 0, s, la, lb, epi, M, N, K,
                     kchunk);
  PTG_RETURN_LAUNCH();
}

// PTG_GEMM256=0 (or ptg_gemm256_set(0)) disables the 256x256 LDS-DMA kernel (A/B runs)
static int g_gemm256 = -1;
static bool gemm256_enabled() {
  if (g_gemm256 < 0) {
    const char* e = getenv("PTG_GEMM256");
    g_gemm256 = (e && e[0] == '0') ? 0 : 1;  // measured: 1040 / 1124 TF/s vs 677 / 870 (4096^3 / 8192^3)
  }
  return g_gemm256 == 1;
}

// split-major XCD mapping for split-K launches with >= 8 splits (split_xcd_map); PTG_GEMM_SPLIT_XCD=0
// keeps the tile mapping.  Measured: ResNet-50 b128 8.83k -> 8.88k img/s, CNN-B1 b256 within noise
// (profiles/r4_ab_gemm_split_xcd.txt)
static int g_split_xcd = -1;
static bool split_xcd_on() {
  if (g_split_xcd < 0) {
    const char* e = getenv("PTG_GEMM_SPLIT_XCD");
    g_split_xcd = !(e && e[0] == '0');
  }
  return g_split_xcd == 1;
}

template <int BM, int BN, int WM, int WN, class LA, class LB, class EPI, int PF = 1>
static int launch_gemm(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, int splits,
                       hipStream_t s) {
  const int tiles = ptg_ceil_div(M, BM) * ptg_ceil_div(N, BN);
  if (splits < 1) splits = 1;
  int kchunk = ptg_ceil_div(ptg_ceil_div(K, splits), BK) * BK;
  if (kchunk < BK) kchunk = BK;
  splits = ptg_ceil_div(K, kchunk);
  dim3 grid(tiles, splits);
  if (split_xcd_on() && splits >= 8 && ((long)tiles * splits) % 8 == 0) kchunk = -kchunk;  // split-major
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, LA, LB, EPI, PF>), grid, dim3(256), 0, s, la, lb, epi, M,
                     N, K, kchunk);
  PTG_RETURN_LAUNCH();
}

// Skinny-M, wide-N GEMMs (the Dense layers' dX: M = batch <= 256, N = 20480, K = 2048): one 256-row
// tile covers all of M, so every column panel of B is streamed from HBM exactly once (the 128x128
// tiling read the 84 MB weight twice), and BN is picked so the grid is ~one workgroup per CU
// (N = 20480: 256 x 80 tiles = 256 workgroups).  PTG_SKINNY_BN=0 disables it, =64/80 forces a width.
static int g_skinny_bn = -2;
int skinny_bn_choice(int M, int N) {
  if (g_skinny_bn == -2) {
    const char* e = getenv("PTG_SKINNY_BN");
    g_skinny_bn = e ? atoi(e) : -1;
  }
  if (g_skinny_bn == 0 || M <= 128 || M > 256) return 0;
  if (g_skinny_bn > 0) return g_skinny_bn;
  const int cands[2] = {80, 64};
  for (int bn : cands)
    if (N % bn == 0 && N / bn >= 192 && N / bn <= 320) return bn;
  return N >= 64 * 192 ? 64 : 0;
}

// Tile-shape choice. N is the narrow dimension for convolutions (output channels).
template <class LA, class LB, class EPI>
static int dispatch_gemm(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, int splits,
                         hipStream_t s) {
  if (splits == 1 && N >= 4096) {
    switch (skinny_bn_choice(M, N)) {
      case 64: return launch_gemm<256, 64, 4, 1, LA, LB, EPI, 2>(la, lb, epi, M, N, K, 1, s);
      case 80: return launch_gemm<256, 80, 4, 1, LA, LB, EPI, 2>(la, lb, epi, M, N, K, 1, s);
      case 81: return launch_gemm<256, 80, 4, 1, LA, LB, EPI, 3>(la, lb, epi, M, N, K, 1, s);
      case 82: return launch_gemm<256, 80, 4, 1, LA, LB, EPI, 1>(la, lb, epi, M, N, K, 1, s);
      default: break;
    }
  }
  if constexpr (HasOff<LA>::value && HasOff<LB>::value && EpiPre<EPI>::v == 0) {
    // big problems: >= one 256x256 tile per CU and K deep enough to amortise the 2-stage ring
    if (gemm256_enabled() && N >= 256 && M >= 256 && K >= 256 &&
        (long)ptg_ceil_div(M, 256) * ptg_ceil_div(N, 256) * splits >= 200)
      return launch_gemm256(la, lb, epi, M, N, K, splits, s);
  }
  if (N <= 16) return launch_gemm<256, 16, 4, 1>(la, lb, epi, M, N, K, splits, s);
  if (N <= 32) return launch_gemm<256, 32, 4, 1>(la, lb, epi, M, N, K, splits, s);
  if (N <= 64) return launch_gemm<128, 64, 2, 2>(la, lb, epi, M, N, K, splits, s);
  if (M <= 64) return launch_gemm<64, 128, 1, 4>(la, lb, epi, M, N, K, splits, s);
  // fewer 128x128 tiles than CUs (late ResNet stages: M = batch*7*7): halve the M tile so the grid
  // covers the 256 CUs (measured: helps below one tile per CU, hurts at 1.5 per CU)
  if ((long)ptg_ceil_div(M, 128) * ptg_ceil_div(N, 128) * splits < 256)
    return launch_gemm<64, 128, 1, 4>(la, lb, epi, M, N, K, splits, s);
  return launch_gemm<128, 128, 2, 2>(la, lb, epi, M, N, K, splits, s);
}

// Narrow-M variant (wgrad: M = output channels).
template <class LA, class LB, class EPI>
static int dispatch_gemm_narrow_m(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K,
                                  int splits, hipStream_t s) {
  if (M <= 16) return launch_gemm<16, 128, 1, 4>(la, lb, epi, M, N, K, splits, s);
  if (M <= 32) return launch_gemm<32, 128, 1, 4>(la, lb, epi, M, N, K, splits, s);
  if (M <= 64) return launch_gemm<64, 128, 1, 4>(la, lb, epi, M, N, K, splits, s);
  return launch_gemm<128, 128, 2, 2>(la, lb, epi, M, N, K, splits, s);
}

static int ilog2(int v) { int l = 0; while ((1 << l) < v) ++l; return l; }
// byte extents of the operand views (the buffer descriptors' range); the engine's operands are far
// below the 2 GiB the 32-bit offsets (and the OOB sentinel above them) allow
static long matk_bytes(long ld, int R, int K) { return ((long)(R - 1) * ld + K) * 2; }
static long matmn_bytes(long ld, int R, int K) { return ((long)(K - 1) * ld + R) * 2; }
static bool fits(long bytes) { return bytes > 0 && bytes < (long)OOB; }
static bool is_pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

}  // namespace ptg

using namespace ptg;

extern "C" {

// PTG_GEMM_SPLIT_XCD at run time (tests / A/B): 1 split-major split-K mapping, 0 the tile mapping
int ptg_gemm_set_split_xcd(int on) {
  ptg::g_split_xcd = on ? 1 : 0;
  return 0;
}

int ptg_gemm256_set(int on) {
  g_gemm256 = on ? 1 : 0;
  return 0;
}

// A/B switch for the skinny-M tiles: 0 = off, -1 = automatic, 64 / 80 = forced tile width
int ptg_gemm_skinny_set(int bn) {
  g_skinny_bn = bn;
  return 0;
}

// Generic bf16 GEMM: C[M][N] = sum_k A(m,k) B(k,n).
//   a_kcontig: A(m,k) = A[m*lda + k]  else A(m,k) = A[k*lda + m]
//   b_kcontig: B(k,n) = B[n*ldb + k]  else B(k,n) = B[k*ldb + n]
//   epi: 0 = bf16 store (+bias, act); 1 = fp32 store (+bias, act); 2 = fp32 accumulate (+=);
//        3 = fp32 atomic add (split-K; caller zeroes C); 4 = bf16 accumulate (C += A.B)
int ptg_gemm_bf16(int M, int N, int K, const void* A, long lda, int a_kcontig, const void* B, long ldb,
                  int b_kcontig, int epi, void* C, long ldc, const float* bias, int act, int splits,
                  hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (!fits(a_kcontig ? matk_bytes(lda, M, K) : matmn_bytes(lda, M, K)) ||
      !fits(b_kcontig ? matk_bytes(ldb, N, K) : matmn_bytes(ldb, N, K)))
    return (int)hipErrorInvalidValue;
  if (epi != 3) splits = 1;
  const bf16_t* a = (const bf16_t*)A; const bf16_t* b = (const bf16_t*)B;
#define PTG_EPI_SWITCH(LAX, LBX)                                                                 \
  switch (epi) {                                                                                 \
    case 0: return dispatch_gemm(LAX, LBX, EpiBf16{(bf16_t*)C, ldc, bias, act, nullptr, 0}, M, N, \
                                 K, 1, s);                                                       \
    case 4: return dispatch_gemm(LAX, LBX, EpiBf16{(bf16_t*)C, ldc, bias, act, nullptr, 1}, M, N, \
                                 K, 1, s);                                                       \
    case 1: return dispatch_gemm(LAX, LBX, EpiF32{(float*)C, ldc, bias, act, 0}, M, N, K, 1, s); \
    case 2: return dispatch_gemm(LAX, LBX, EpiF32{(float*)C, ldc, bias, act, 1}, M, N, K, 1, s); \
    case 3: return dispatch_gemm(LAX, LBX, EpiAtomic{(float*)C, ldc}, M, N, K, splits, s);       \
    default: return (int)hipErrorInvalidValue;                                                   \
  }
  if (a_kcontig && b_kcontig) {
    if (lda % 8 || ldb % 8 || K % 8) return (int)hipErrorInvalidValue;
    MatK<8> la{a, lda, M, K, (uint32_t)matk_bytes(lda, M, K)}; MatK<8> lb{b, ldb, N, K, (uint32_t)matk_bytes(ldb, N, K)};
    PTG_EPI_SWITCH(la, lb)
  } else if (a_kcontig && !b_kcontig) {
    if (lda % 8 || ldb % 8 || K % 8 || N % 8) return (int)hipErrorInvalidValue;
    MatK<8> la{a, lda, M, K, (uint32_t)matk_bytes(lda, M, K)}; MatMN lb{b, ldb, N, K, (uint32_t)matmn_bytes(ldb, N, K)};
    PTG_EPI_SWITCH(la, lb)
  } else if (!a_kcontig && !b_kcontig) {
    if (lda % 8 || ldb % 8 || M % 8 || N % 8) return (int)hipErrorInvalidValue;
    MatMN la{a, lda, M, K, (uint32_t)matmn_bytes(lda, M, K)}; MatMN lb{b, ldb, N, K, (uint32_t)matmn_bytes(ldb, N, K)};
    PTG_EPI_SWITCH(la, lb)
  } else {
    if (lda % 8 || ldb % 8 || M % 8 || K % 8) return (int)hipErrorInvalidValue;
    MatMN la{a, lda, M, K, (uint32_t)matmn_bytes(lda, M, K)}; MatK<8> lb{b, ldb, N, K, (uint32_t)matk_bytes(ldb, N, K)};
    PTG_EPI_SWITCH(la, lb)
  }
#undef PTG_EPI_SWITCH
}

// Weight gradient with Adam fused into the epilogue (EpiAdam): G[M][N] = A^T-style product as in
// ptg_gemm_bf16 (same operand conventions, no split-K), then p/m/v/pbf[m*ldc+n] updated in place.
int ptg_gemm_adam(int M, int N, int K, const void* A, long lda, int a_kcontig, const void* B, long ldb,
                  int b_kcontig, float* p, float* m, float* v, void* pbf, long ldc, float lr_t, float b1,
                  float b2, float eps, float gscale, const float* lr_dev, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (a_kcontig || b_kcontig || lda % 8 || ldb % 8 || M % 8 || N % 8 || ldc % 8) return (int)hipErrorInvalidValue;
  if (!fits(matmn_bytes(lda, M, K)) || !fits(matmn_bytes(ldb, N, K))) return (int)hipErrorInvalidValue;
  const bf16_t* a = (const bf16_t*)A; const bf16_t* b = (const bf16_t*)B;
  MatMN la{a, lda, M, K, (uint32_t)matmn_bytes(lda, M, K)}; MatMN lb{b, ldb, N, K, (uint32_t)matmn_bytes(ldb, N, K)};
  return dispatch_gemm(la, lb, EpiAdam{p, m, v, (bf16_t*)pbf, ldc, lr_t, b1, b2, eps, gscale, lr_dev}, M, N, K, 1, s);
}

// Conv2D forward, NHWC bf16: z[n][oh][ow][co] = bias[co] + sum_{kh,kw,ci} x[..] w[co][kh][kw][ci]
// w is [Cout][KH*KW*C] bf16. C must be a power of two >= 4.
int ptg_conv2d_fwd(const void* x, const void* w, const float* bias, void* z, int N, int H, int W, int C,
                   int Cout, int KH, int KW, int stride, int pad, int OH, int OW, int act,
                   hipStream_t s) {
  if (!is_pow2(C) || C < 4) return (int)hipErrorInvalidValue;
  const int M = N * OH * OW, Kc = KH * KW * C;
  if (!fits((long)N * H * W * C * 2) || !fits((long)Cout * Kc * 2)) return (int)hipErrorInvalidValue;
  EpiBf16 epi{(bf16_t*)z, Cout, bias, act, nullptr, 0};
  if (C % 8 == 0) {
    ConvFwdA<8> la{(const bf16_t*)x, H, W, C, ilog2(C), OH, OW, KW, stride, pad, M, Kc};
    la.init();
    MatK<8> lb{(const bf16_t*)w, Kc, Cout, Kc, (uint32_t)matk_bytes(Kc, Cout, Kc)};
    return dispatch_gemm(la, lb, epi, M, Cout, Kc, 1, s);
  } else {
    ConvFwdA<4> la{(const bf16_t*)x, H, W, C, ilog2(C), OH, OW, KW, stride, pad, M, Kc};
    la.init();
    MatK<4> lb{(const bf16_t*)w, Kc, Cout, Kc, (uint32_t)matk_bytes(Kc, Cout, Kc)};
    return dispatch_gemm(la, lb, epi, M, Cout, Kc, 1, s);
  }
}

// Conv2D data gradient for stride-1 convolutions: dx = conv(dz, flip(w)^T, pad' = K-1-pad).
// dz [N][H][W][Cout] (Cout power of two >= 8), dx [N][H][W][Cin] (Cin % 8 == 0).
int ptg_conv2d_dgrad(const void* dz, const void* w, void* dx, int N, int H, int W, int Cin, int Cout,
                     int KH, int KW, int pad, int accum, hipStream_t s) {
  if (!is_pow2(Cout) || Cout < 8 || Cin % 8) return (int)hipErrorInvalidValue;
  const int M = N * H * W, Kc2 = KH * KW * Cout;
  if (!fits((long)M * Cout * 2) || !fits((long)Kc2 * Cin * 2)) return (int)hipErrorInvalidValue;
  ConvFwdA<8> la{(const bf16_t*)dz, H, W, Cout, ilog2(Cout), H, W, KW, 1, KH - 1 - pad, M, Kc2};
  ConvDgradB lb{(const bf16_t*)w, Cin, Cout, ilog2(Cout), KH, KW, Kc2};
  la.init();
  lb.init();
  EpiBf16 epi{(bf16_t*)dx, Cin, nullptr, ACT_NONE, nullptr, accum};
  return dispatch_gemm(la, lb, epi, M, Cin, Kc2, 1, s);
}

// Data gradients feeding a Conv -> BN -> ReLU block (EpiBf16 backward form): dx = g (masked by the
// block's ReLU via bsc / bsh, may be null), and stats ([64][2][Cin] fp32, accumulated into) += the
// block's BN backward sums over (g, g*bz).  Stride 1, no accumulation, Cin < 4096.
int ptg_conv2d_dgrad_bnstats(const void* dz, const void* w, void* dx, int N, int H, int W, int Cin, int Cout, int KH,
                             int KW, int pad, float* stats, const void* bz, const float* bsc, const float* bsh,
                             hipStream_t s) {
  if (!is_pow2(Cout) || Cout < 8 || Cin % 8 || Cin >= 4096 || !stats || !bz) return (int)hipErrorInvalidValue;
  const int M = N * H * W, Kc2 = KH * KW * Cout;
  if (!fits((long)M * Cout * 2) || !fits((long)Kc2 * Cin * 2) || !fits((long)M * Cin * 2))
    return (int)hipErrorInvalidValue;
  ConvFwdA<8> la{(const bf16_t*)dz, H, W, Cout, ilog2(Cout), H, W, KW, 1, KH - 1 - pad, M, Kc2};
  ConvDgradB lb{(const bf16_t*)w, Cin, Cout, ilog2(Cout), KH, KW, Kc2};
  la.init();
  lb.init();
  EpiBf16 epi{(bf16_t*)dx, Cin, nullptr, ACT_NONE, nullptr, 0, stats, (const bf16_t*)bz, bsc, bsh};
  return dispatch_gemm(la, lb, epi, M, Cin, Kc2, 1, s);
}
int ptg_conv1x1_dgrad_bnstats(const void* dz, const void* w, void* dx, int N, int H, int W, int Cin, int Cout,
                              float* stats, const void* bz, const float* bsc, const float* bsh, hipStream_t s) {
  if (Cin % 8 || Cout % 8 || Cin >= 4096 || !stats || !bz) return (int)hipErrorInvalidValue;
  const int M = N * H * W;
  if (!fits((long)M * Cout * 2) || !fits((long)M * Cin * 2)) return (int)hipErrorInvalidValue;
  MatK<8> la{(const bf16_t*)dz, Cout, M, Cout, (uint32_t)matk_bytes(Cout, M, Cout)};
  MatMN lb{(const bf16_t*)w, Cin, Cin, Cout, (uint32_t)matmn_bytes(Cin, Cin, Cout)};
  EpiBf16 epi{(bf16_t*)dx, Cin, nullptr, ACT_NONE, nullptr, 0, stats, (const bf16_t*)bz, bsc, bsh};
  return dispatch_gemm(la, lb, epi, M, Cin, Cout, 1, s);
}

// Data gradient of a 1x1 convolution with stride s (pad 0): dx[n][oh*s][ow*s][ci] (+)= sum_co
// dz[n][oh][ow][co] w[co][ci]; input pixels off the stride lattice get no contribution (the caller
// zeroes dx once when s > 1 and this is the first gradient written into it).
int ptg_conv1x1_dgrad(const void* dz, const void* w, void* dx, int N, int OH, int OW, int H, int W, int Cin,
                      int Cout, int stride, int accum, hipStream_t s) {
  if (Cin % 8 || Cout % 8) return (int)hipErrorInvalidValue;
  const int M = N * OH * OW;
  if (!fits((long)M * Cout * 2)) return (int)hipErrorInvalidValue;
  MatK<8> la{(const bf16_t*)dz, Cout, M, Cout, (uint32_t)matk_bytes(Cout, M, Cout)};
  MatMN lb{(const bf16_t*)w, Cin, Cin, Cout, (uint32_t)matmn_bytes(Cin, Cin, Cout)};
  if (stride == 1) {
    EpiBf16 epi{(bf16_t*)dx, Cin, nullptr, ACT_NONE, nullptr, accum};
    return dispatch_gemm(la, lb, epi, M, Cin, Cout, 1, s);
  }
  EpiBf16Remap epi{(bf16_t*)dx, Cin, OH, OW, H, W, stride, accum};
  return dispatch_gemm(la, lb, epi, M, Cin, Cout, 1, s);
}

// Conv2D weight gradient: dw[co][kc] (+)= sum_pixels dz[p][co] * im2col(x)[p][kc], fp32.
// Split-K over output pixels with fp32 atomics; dw must be zeroed (or hold a sum to add to).
int ptg_conv2d_wgrad(const void* x, const void* dz, float* dw, int N, int H, int W, int C, int Cout,
                     int KH, int KW, int stride, int pad, int OH, int OW, int splits, hipStream_t s) {
  if (!is_pow2(C) || C < 4 || Cout % 8) return (int)hipErrorInvalidValue;
  const int P = N * OH * OW, Kc = KH * KW * C;
  if (!fits((long)N * H * W * C * 2) || !fits((long)P * Cout * 2)) return (int)hipErrorInvalidValue;
  MatMN la{(const bf16_t*)dz, Cout, Cout, P, (uint32_t)matmn_bytes(Cout, Cout, P)};
  EpiAtomic epi{dw, Kc};
  if (splits <= 0) {
    const int tiles = ptg_ceil_div(Cout, Cout <= 16 ? 16 : (Cout <= 32 ? 32 : 64)) * ptg_ceil_div(Kc, 128);
    // ~2 blocks per CU: more K slices only add fp32 atomic traffic (which runs at ~1.3 TB/s of
    // added bytes, MI355X_MICROARCH.md "Global float atomics") without adding useful overlap
    splits = ptg_ceil_div(512, tiles);
    const int max_splits = ptg_ceil_div(P, 4 * BK);
    if (splits > max_splits) splits = max_splits;
  }
  if (C % 8 == 0) {
    ConvWgradB<8> lb{(const bf16_t*)x, H, W, C, ilog2(C), OH, OW, KW, stride, pad, P, Kc};
    lb.init();
    return dispatch_gemm_narrow_m(la, lb, epi, Cout, Kc, P, splits, s);
  } else {
    ConvWgradB<4> lb{(const bf16_t*)x, H, W, C, ilog2(C), OH, OW, KW, stride, pad, P, Kc};
    lb.init();
    return dispatch_gemm_narrow_m(la, lb, epi, Cout, Kc, P, splits, s);
  }
}

// ---- BatchNormalization statistics from the conv GEMMs (ResNet, graph_ops.ConvBNOp) --------------
// stats (fp32 [64][2][Cout], accumulated into): batch statistics of the bf16 output z for the
// following BatchNormalization, produced in the epilogue.
int ptg_conv_bn_fwd(const void* x, const void* w, const float* bias, void* z, int N, int H, int W, int C, int Cout,
                    int KH, int KW, int stride, int pad, int OH, int OW, float* stats, hipStream_t s) {
  if (!is_pow2(C) || C < 4 || Cout % 8 || (stats && Cout >= 4096)) return (int)hipErrorInvalidValue;
  const int M = N * OH * OW, Kc = KH * KW * C;
  if (!fits((long)N * H * W * C * 2) || !fits((long)M * Cout * 2) || !fits((long)Cout * Kc * 2))
    return (int)hipErrorInvalidValue;
  EpiBf16 epi{(bf16_t*)z, Cout, bias, ACT_NONE, nullptr, 0, stats};
  const bf16_t* xb = (const bf16_t*)x;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {  // plain GEMM over the NHWC pixel rows
    if (C % 8) return (int)hipErrorInvalidValue;
    MatK<8> la{xb, C, M, C, (uint32_t)matk_bytes(C, M, C)};
    MatK<8> lb{(const bf16_t*)w, C, Cout, C, (uint32_t)matk_bytes(C, Cout, C)};
    return dispatch_gemm(la, lb, epi, M, Cout, C, 1, s);
  }
  if (C % 8 == 0) {
    ConvFwdA<8> la{xb, H, W, C, ilog2(C), OH, OW, KW, stride, pad, M, Kc};
    la.init();
    MatK<8> lb{(const bf16_t*)w, Kc, Cout, Kc, (uint32_t)matk_bytes(Kc, Cout, Kc)};
    return dispatch_gemm(la, lb, epi, M, Cout, Kc, 1, s);
  }
  ConvFwdA<4> la{xb, H, W, C, ilog2(C), OH, OW, KW, stride, pad, M, Kc};
  la.init();
  MatK<4> lb{(const bf16_t*)w, Kc, Cout, Kc, (uint32_t)matk_bytes(Kc, Cout, Kc)};
  return dispatch_gemm(la, lb, epi, M, Cout, Kc, 1, s);
}

}  // extern "C"

PTG_CHECK_STATUS(gemm)
