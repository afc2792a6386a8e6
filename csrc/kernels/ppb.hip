// Backward of PReLU + MaxPooling2D(2x2) (train_tf_ps.py:352-362, CNN-B1 layers 2-4), row-pair
// layout: HBM-bound (z read, dz written at full resolution), so every access is a coalesced
// 16-byte vector.
//
// A thread owns one 16-byte chunk (8 channels) of one pixel column p in BOTH rows of a pooled row
// (2ph, 2ph+1) and walks a chunk of samples.  The horizontal window partner (pixel p ^ 1, same
// channels) is lane ^ CPX (CPX = C / 8 chunks per pixel) of the same wave, reached with
// ds_swizzle (no LDS traffic); both lanes evaluate the window's four PReLU values in the same
// q = 2*dh + dw order, so they agree on the argmax (first maximum, as the forward's pool).  The
// pooled gradient chunk is one 16-byte load shared by the pair.  Alphas (own and partner's) and the
// dalpha sums stay in registers across the samples; the next sample's loads are issued before this
// one's math.
//
// dalpha = sum over the batch: each sample chunk writes its partial sums for its positions (no
// atomics) and ppb_reduce_k adds the chunk partials into dalpha; dbias partials are one row of C
// floats per workgroup, reduced by the same kernel's last workgroup row.  Exactly prelu_pool_bwd_sg_k's
// arithmetic (nn_eltwise.hip), so the dz bits are identical.
#include "common.h"

namespace ptgp {

template <int CPX>
PTG_DEV uint32_t partner(uint32_t v) {
  // bit-mode swizzle within 32 lanes: and_mask 0x1F, xor_mask CPX
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (CPX << 10));
}

template <int CPX>
__global__ __launch_bounds__(256) void ppb_rows_k(const bf16_t* __restrict__ dp, const bf16_t* __restrict__ z,
                                                  const float* __restrict__ alpha, bf16_t* __restrict__ dz,
                                                  float* __restrict__ part, float* __restrict__ dbpart, int N, int H,
                                                  int W, int nper) {
  constexpr int C = CPX * 8;
  const int RW = W * CPX;  // chunks per full-resolution row
  const int PH = H >> 1, PW = W >> 1;
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const bool active = t < (long)PH * RW;
  const int ph = active ? (int)(t / RW) : 0;
  const int j = active ? (int)(t - (long)ph * RW) : 0;
  const int p = j / CPX, c = j - p * CPX;
  const int dw = p & 1;
  const int n0 = blockIdx.y * nper, n1 = min(N, n0 + nper);
  __shared__ float sdb[4][C];
  float da[2][8], db[8], aa[2][8], ap[2][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { da[0][k] = da[1][k] = 0.f; db[k] = 0.f; }
  // own and partner alphas: [row][channel], rows 2ph / 2ph+1
  const long a0 = ((long)(2 * ph) * W + p) * C + c * 8, a1 = a0 + (long)W * C;
  const long pa0 = ((long)(2 * ph) * W + (p ^ 1)) * C + c * 8, pa1 = pa0 + (long)W * C;
  if (active) {
#pragma unroll
    for (int k = 0; k < 8; k += 4) {
      const float4 x0 = *(const float4*)(alpha + a0 + k), x1 = *(const float4*)(alpha + a1 + k);
      const float4 y0 = *(const float4*)(alpha + pa0 + k), y1 = *(const float4*)(alpha + pa1 + k);
      aa[0][k] = x0.x; aa[0][k + 1] = x0.y; aa[0][k + 2] = x0.z; aa[0][k + 3] = x0.w;
      aa[1][k] = x1.x; aa[1][k + 1] = x1.y; aa[1][k + 2] = x1.z; aa[1][k + 3] = x1.w;
      ap[0][k] = y0.x; ap[0][k + 1] = y0.y; ap[0][k + 2] = y0.z; ap[0][k + 3] = y0.w;
      ap[1][k] = y1.x; ap[1][k + 1] = y1.y; ap[1][k + 2] = y1.z; ap[1][k + 3] = y1.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) aa[0][k] = aa[1][k] = ap[0][k] = ap[1][k] = 0.f;
  }
  const uint32_t HWC = (uint32_t)(H * W * C), PHWC = (uint32_t)(PH * PW * C);
  const uint32_t zo = (uint32_t)(((2 * ph) * W + p) * C + c * 8) * 2u;   // byte offset, row 2ph
  const uint32_t zrow = (uint32_t)(W * C) * 2u;
  const uint32_t po = (uint32_t)((ph * PW + (p >> 1)) * C + c * 8) * 2u;
  const Rsrc zr = make_rsrc(z, (uint32_t)((long)N * HWC * 2)), dpr = make_rsrc(dp, (uint32_t)((long)N * PHWC * 2));
  U4 za, zb, g;
  auto ld = [&](int n, U4& a, U4& b, U4& gg) {
    const bool ok = active && n < n1;
    const uint32_t zn = (uint32_t)n * HWC * 2u, pn = (uint32_t)n * PHWC * 2u;
    a = bload16(zr, ok ? zn + zo : PTG_OOB);
    b = bload16(zr, ok ? zn + zo + zrow : PTG_OOB);
    gg = bload16(dpr, ok ? pn + po : PTG_OOB);
  };
  ld(n0, za, zb, g);
  for (int n = n0; n < n1; ++n) {
    U4 za2, zb2, g2;
    ld(n + 1, za2, zb2, g2);
    U4 oa, ob;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t wa = w == 0 ? za.x : w == 1 ? za.y : w == 2 ? za.z : za.w;
      const uint32_t wb = w == 0 ? zb.x : w == 1 ? zb.y : w == 2 ? zb.z : zb.w;
      const uint32_t wg = w == 0 ? g.x : w == 1 ? g.y : w == 2 ? g.z : g.w;
      const uint32_t pwa = partner<CPX>(wa), pwb = partner<CPX>(wb);
      uint32_t outa = 0u, outb = 0u;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * w + h;
        const float zA = h ? hi_bf(wa) : lo_bf(wa), zB = h ? hi_bf(wb) : lo_bf(wb);
        const float qA = h ? hi_bf(pwa) : lo_bf(pwa), qB = h ? hi_bf(pwb) : lo_bf(pwb);
        const float yA = zA > 0.f ? zA : aa[0][k] * zA, yB = zB > 0.f ? zB : aa[1][k] * zB;
        const float rA = qA > 0.f ? qA : ap[0][k] * qA, rB = qB > 0.f ? qB : ap[1][k] * qB;
        // the window in q order: q0 = (row a, dw 0), q1 = (a, 1), q2 = (b, 0), q3 = (b, 1)
        const float y0 = dw ? rA : yA, y1 = dw ? yA : rA, y2 = dw ? rB : yB, y3 = dw ? yB : rB;
        int am = 0;
        float b = y0;
        if (y1 > b) { b = y1; am = 1; }
        if (y2 > b) { b = y2; am = 2; }
        if (y3 > b) { b = y3; am = 3; }
        const float gj = h ? hi_bf(wg) : lo_bf(wg);
        const bool hitA = am == dw, hitB = am == 2 + dw;
        const float dA = hitA ? (zA > 0.f ? gj : gj * aa[0][k]) : 0.f;
        const float dB = hitB ? (zB > 0.f ? gj : gj * aa[1][k]) : 0.f;
        da[0][k] += (hitA && !(zA > 0.f)) ? gj * zA : 0.f;
        da[1][k] += (hitB && !(zB > 0.f)) ? gj * zB : 0.f;
        db[k] += dA + dB;
        outa |= (uint32_t)f2bf(dA) << (16 * h);
        outb |= (uint32_t)f2bf(dB) << (16 * h);
      }
      if (w == 0) { oa.x = outa; ob.x = outb; }
      else if (w == 1) { oa.y = outa; ob.y = outb; }
      else if (w == 2) { oa.z = outa; ob.z = outb; }
      else { oa.w = outa; ob.w = outb; }
    }
    if (active) {
      bf16_t* d = dz + (long)n * HWC + zo / 2;
      *(U4*)d = oa;
      *(U4*)(d + W * C) = ob;
    }
    za = za2; zb = zb2; g = g2;
  }
  // dalpha partials of this sample chunk: part[chunk][row][col][ch]
  if (active) {
    float* pp = part + (long)blockIdx.y * H * W * C;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float* q = pp + (r ? a1 : a0);
      *(float4*)q = make_float4(da[r][0], da[r][1], da[r][2], da[r][3]);
      *(float4*)(q + 4) = make_float4(da[r][4], da[r][5], da[r][6], da[r][7]);
    }
  }
  // dbias: lanes with the same chunk index c hold the same 8 channels
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float v = db[k];
    for (int o = 32; o >= CPX; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane < CPX) sdb[wv][lane * 8 + k] = v;
  }
  __syncthreads();
  if ((int)threadIdx.x < C) {
    const long row = (long)blockIdx.y * gridDim.x + blockIdx.x;
    dbpart[row * C + threadIdx.x] = sdb[0][threadIdx.x] + sdb[1][threadIdx.x] + sdb[2][threadIdx.x] +
                                    sdb[3][threadIdx.x];
  }
}

// dalpha[e] += sum_c part[c][e] (float4 per thread); blockIdx.x == gridDim.x - 1: dbias[ch] +=
// sum of the dbias partial rows
__global__ __launch_bounds__(256) void ppb_reduce_k(const float* __restrict__ part, int nchunks, long e4,
                                                    float* __restrict__ dalpha, const float* __restrict__ dbpart,
                                                    int nrows, int C, float* __restrict__ dbias) {
  if (blockIdx.x == gridDim.x - 1) {
    __shared__ float s[256];
    const int ch = threadIdx.x % C, grp = threadIdx.x / C, ng = 256 / C;
    float v = 0.f;
    if (grp < ng)
      for (int r = grp; r < nrows; r += ng) v += dbpart[(long)r * C + ch];
    s[threadIdx.x] = grp < ng ? v : 0.f;
    __syncthreads();
    if ((int)threadIdx.x < C) {
      float tot = 0.f;
      for (int q = 0; q < ng; ++q) tot += s[q * C + threadIdx.x];
      dbias[threadIdx.x] += tot;
    }
    return;
  }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < e4; i += (long)(gridDim.x - 1) * 256) {
    float4 acc = ((float4*)dalpha)[i];
    for (int c = 0; c < nchunks; ++c) {
      const float4 v = ((const float4*)part)[(long)c * e4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    ((float4*)dalpha)[i] = acc;
  }
}

}  // namespace ptgp

extern "C" {

// Workspace: part [nchunks][H][W][C] fp32 + dbpart [nchunks * ceil(PH*W*C/8 / 256)][C] fp32.
int ptg_ppb_rows_ws_floats(int N, int H, int W, int C, int nchunks, long* out) {
  const long bx = ((long)(H / 2) * W * (C / 8) + 255) / 256;
  *out = (long)nchunks * H * W * C + (long)nchunks * bx * C;
  return 0;
}

int ptg_prelu_pool_bwd_rows(const void* dp, const void* z, const float* alpha, void* dz, float* dalpha, float* dbias,
                            int N, int H, int W, int C, int nchunks, float* ws, hipStream_t s) {
  if ((H & 1) || (W & 1) || H < 2 || W < 2 || (C != 8 && C != 16 && C != 32 && C != 64) || nchunks < 1 ||
      nchunks > N || !ptg_fits_2g((long)N * H * W * C * 2))
    return (int)hipErrorInvalidValue;
  const int CPX = C / 8;
  const long pos = (long)(H / 2) * W * CPX;
  const int bx = (int)((pos + 255) / 256);
  const int nper = (N + nchunks - 1) / nchunks;
  const int ny = (N + nper - 1) / nper;
  float* part = ws;
  float* dbpart = ws + (long)nchunks * H * W * C;
  dim3 grid(bx, ny);
  switch (CPX) {
    case 1: hipLaunchKernelGGL(ptgp::ppb_rows_k<1>, grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)z, alpha,
                               (bf16_t*)dz, part, dbpart, N, H, W, nper); break;
    case 2: hipLaunchKernelGGL(ptgp::ppb_rows_k<2>, grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)z, alpha,
                               (bf16_t*)dz, part, dbpart, N, H, W, nper); break;
    case 4: hipLaunchKernelGGL(ptgp::ppb_rows_k<4>, grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)z, alpha,
                               (bf16_t*)dz, part, dbpart, N, H, W, nper); break;
    default: hipLaunchKernelGGL(ptgp::ppb_rows_k<8>, grid, dim3(256), 0, s, (const bf16_t*)dp, (const bf16_t*)z, alpha,
                                (bf16_t*)dz, part, dbpart, N, H, W, nper); break;
  }
  const long e4 = (long)H * W * C / 4;
  const int rb = (int)((e4 + 255) / 256 < 1024 ? (e4 + 255) / 256 : 1024);
  hipLaunchKernelGGL(ptgp::ppb_reduce_k, dim3(rb + 1), dim3(256), 0, s, part, ny, e4, dalpha, dbpart, ny * bx, C,
                     dbias);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"
