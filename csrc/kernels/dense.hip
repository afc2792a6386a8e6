// Weight-streaming GEMMs of the big Dense layer (CNN-B1: Flatten(20480) -> Dense(2048, relu),
// reference train_tf_ps.py:366-367; any Dense whose weight is tens of MB and whose M is a batch).
//
// Shape: M = batch <= 256 rows, the [N][K] bf16 weight (84 MB for CNN-B1) read from HBM once per
// pass.  The MFMA work (21.5 GFLOP at b256) is ~9 us at the dense bf16 peak and the weight stream
// ~13 us at 6.3 TB/s, so the kernel has to keep both the matrix cores and HBM busy at once:
//
//   * One 512-thread workgroup per CU (grid = N/128 column tiles x S K-splits = 256), each owning
//     ALL M rows of a 128-column tile over one K range, so every weight byte is read exactly once.
//   * Both operands are staged with LDS-DMA (buffer_load ... lds, 16 B per lane, source-side XOR
//     swizzle for conflict-free ds_read_b128) into an NS-deep LDS ring.  Waits are COUNTED
//     (s_waitcnt vmcnt(L*(NS-2))): NS-1 K-steps of loads stay in flight across the barriers, which
//     covers the HBM latency of the weight stream (the 2-stage drain-to-zero form exposes it
//     every step).  cdna_hip_programming.md T3/T4, T8.
//   * Split-major XCD mapping: the workgroups of one K-split land on one XCD, so that split's
//     activation panel (M x kchunk, <= 655 KB) is fetched into one L2 and shared by its 16 tiles.
//   * Split-K partials leave with PLAIN stores into part[S][M][N] (fp32).  Device float atomics run
//     at the memory side (~1.3 TB/s chip-wide, MI355X_MICROARCH.md "Global float atomics"): the
//     old atomic epilogue spent ~25 us of the 58 us forward adding 32 MB.  The consumer (the fused
//     regression head, or bias_act) sums the S slices in its own pass, so no fill and no atomics.
#include "common.h"

namespace ptgd {

constexpr int BK = 64;   // K per stage (one 128-B row per operand row)
constexpr int NT = 128;  // output columns per workgroup

typedef __attribute__((address_space(3))) void lds_t;

template <int MT>
struct FwdCfg {
  static constexpr int WM = MT >= 256 ? 4 : MT >= 128 ? 2 : 1;  // waves along M
  static constexpr int WN = 8 / WM;                            // waves along N
  static constexpr int WTM = MT / WM, WTN = NT / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int ROWS = MT + NT;                          // operand rows per stage
  static constexpr int STAGE = ROWS * BK * 2;                   // bytes per stage
  static constexpr int BLK = ROWS / 8;                          // 1-KB DMA blocks per stage
  static constexpr int L = (BLK + 7) / 8;                       // DMA instructions per wave per stage
  static constexpr int NS = (152 * 1024) / STAGE < 8 ? (152 * 1024) / STAGE : 8;  // ring depth
  static_assert(FM >= 1 && FN >= 1 && NS >= 3, "tile");
};

// vmcnt(n) for a compile-time n (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[15:14])
template <int N>
PTG_DEV void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// part[s][m][n] = sum_{k in split s} x[m][k] * w[n][k]
// DBG (measurement variants, tools/dense_bench.py): bit 0 skips the MFMAs, bit 1 the partial stores;
// WAUX: cache policy bits of the weight-stream loads (2 = nt)
template <int MT, int DBG = 0, int WAUX = 0>
__global__ __launch_bounds__(512) void dense_fwd_sk_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      float* __restrict__ part, int M, int N, int K, int kchunk,
                                                      uint32_t xbytes, uint32_t wbytes) {
  using C = FwdCfg<MT>;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): no waterfall loops
  const int wm = wid / C::WN, wn = wid % C::WN;
  // split-major XCD mapping (host: gridDim.x % 8 == 0): consecutive items of one XCD share a split
  const int tiles = N / NT, total = gridDim.x;
  const int item = (blockIdx.x % 8) * (total / 8) + blockIdx.x / 8;
  const int split = item / tiles, tn = item - split * tiles;
  const int n0 = tn * NT, kb = split * kchunk;
  const int nk = min(kchunk, K - kb) / BK;

  // this wave's DMA blocks: block b = rows 8b..8b+7 of [A rows (MT) | B rows (NT)]; lanes 8 per row
  const Rsrc rsA = make_rsrc(x, xbytes), rsB = make_rsrc(w, wbytes);
  uint32_t goff[C::L];  // byte offset of this lane's 16-B chunk at k = 0 (OOB for rows past M)
  bool isA[C::L];
  int lds_off[C::L];
#pragma unroll
  for (int j = 0; j < C::L; ++j) {
    int b = wid + 8 * j;
    b = b < C::BLK ? b : C::BLK - 1;  // waves with fewer blocks repeat their last one (same bytes)
    const int row = b * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);  // source-side swizzle of the 16-B chunk
    isA[j] = b < MT / 8;  // whole 8-row blocks belong to one operand (MT % 8 == 0): wave-uniform
    if (isA[j]) {
      goff[j] = row < M ? (uint32_t)row * (uint32_t)K * 2u + (uint32_t)(kb + chunk * 8) * 2u : PTG_OOB;
    } else if constexpr ((DBG & 4) != 0) {
      // measurement only: the weight as if stored tile-contiguous ([tile][split][stage][128][64]): each
      // stage's 16 KB of B is one contiguous run (the numbers are garbage, the timing is the point)
      goff[j] = (uint32_t)((tn * (K / kchunk) + split) * (kchunk / BK)) * 16384u + (uint32_t)(row - MT) * 128u +
                (uint32_t)chunk * 16u;
    } else {
      goff[j] = (uint32_t)(n0 + row - MT) * (uint32_t)K * 2u + (uint32_t)(kb + chunk * 8) * 2u;
    }
    lds_off[j] = b * 1024;
  }
  auto issue = [&](int t) {  // stage t -> ring slot t % NS
    unsigned char* base = smem + (t % C::NS) * C::STAGE;
    const uint32_t dk = (uint32_t)t * BK * 2u;
#pragma unroll
    for (int j = 0; j < C::L; ++j) {
      const uint32_t step = ((DBG & 4) != 0 && !isA[j]) ? (uint32_t)t * 16384u : dk;
      const uint32_t o = goff[j] == PTG_OOB ? PTG_OOB : goff[j] + step;
      if (isA[j])
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t*)(base + lds_off[j]), 16, o, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t*)(base + lds_off[j]), 16, o, 0, 0, WAUX);
    }
  };

  // fragment: rows row0..row0+15, 16-B chunk (cbase + lane>>4) of the 128-B row, swizzled
  const int fr = lane & 15, fc = lane >> 4;
  auto frag = [&](const unsigned char* img, int row0, int cbase) -> bf16x8_t {
    const int r = row0 + fr;
    const int pos = (cbase + fc) ^ ((r >> 1) & 7);
    return __builtin_bit_cast(bf16x8_t, *(const U4*)(img + r * 128 + pos * 16));
  };

  f32x4_t acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < C::NS - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    // stage t landed (this wave's part): the younger stages t+1..t+NS-2 may still be in flight
    if (t + C::NS - 2 < nk) wait_vm<C::L * (C::NS - 2)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // ... and every other wave's part; slot (t-1) % NS is free
    if (t + C::NS - 1 < nk) issue(t + C::NS - 1);
    const unsigned char* sA = smem + (t % C::NS) * C::STAGE;
    const unsigned char* sB = sA + MT * 128;
    if constexpr (DBG & 1) continue;
#pragma unroll
    for (int kc = 0; kc < 8; kc += 4) {
      bf16x8_t af[C::FM], bfr[C::FN];
#pragma unroll
      for (int j = 0; j < C::FN; ++j) bfr[j] = frag(sB, wn * C::WTN + j * 16, kc);
#pragma unroll
      for (int i = 0; i < C::FM; ++i) af[i] = frag(sA, wm * C::WTM + i * 16, kc);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // C/D map of mfma_f32_16x16x32: col = lane&15, row = (lane>>4)*4 + r.  Plain stores: each store
  // instruction writes 4 rows x 64 contiguous bytes; the neighbouring fragment completes the lines.
  if constexpr ((DBG & 2) != 0) return;
  float* out = part + (long)split * M * N;
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = wm * C::WTM + i * 16 + (lane >> 4) * 4 + r;
      if (m < M) {
#pragma unroll
        for (int j = 0; j < C::FN; ++j) out[(long)m * N + n0 + wn * C::WTN + j * 16 + (lane & 15)] = acc[i][j][r];
      }
    }
}

template <int MT, int DBG = 0, int WAUX = 0>
static int launch_fwd(const bf16_t* x, const bf16_t* w, float* part, int M, int N, int K, int splits,
                      hipStream_t s) {
  using C = FwdCfg<MT>;
  const int kchunk = K / splits;
  const int grid = (N / NT) * splits;
  const int lds = C::NS * C::STAGE;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)dense_fwd_sk_k<MT, DBG, WAUX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    attr = true;
  }
  hipLaunchKernelGGL((dense_fwd_sk_k<MT, DBG, WAUX>), dim3(grid), dim3(512), lds, s, x, w, part, M, N, K, kchunk,
                     (uint32_t)((long)M * K * 2), (uint32_t)((long)N * K * 2));
  PTG_RETURN_LAUNCH();
}

}  // namespace ptgd

using namespace ptgd;

extern "C" {

// Split count the forward uses for (M, N, K): ~one workgroup per CU, K-splits of >= 4 stages.
int ptg_dense_fwd_splits(int M, int N, int K) {
  if (M <= 0 || M > 256 || N <= 0 || N % NT || K % BK) return 0;
  const int tiles = N / NT;
  int best = 0;
  for (int s = 1; s <= 64; ++s) {
    if (K % (s * BK) || (tiles * s) % 8 || K / s < 4 * BK) continue;
    if (tiles * s <= 256) best = s;  // the largest grid that is still one workgroup per CU
  }
  return best;
}

// part[s][m][n] (fp32, S = splits slices) = x[M][K] . w[N][K]^T restricted to K-split s.
// Requirements (checked): M <= 256, N % 128 == 0, K % (64 * splits) == 0, (N/128 * splits) % 8 == 0,
// operands < 2 GiB.  Every element of part[0..S) is written (no fill needed).
int ptg_dense_fwd_sk(const void* x, const void* w, float* part, int M, int N, int K, int splits, hipStream_t s) {
  if (M <= 0 || M > 256 || N <= 0 || N % NT || K <= 0 || splits <= 0 || K % (BK * splits) ||
      ((N / NT) * splits) % 8 || K / splits < 2 * BK)
    return (int)hipErrorInvalidValue;
  if (!ptg_fits_2g((long)N * K * 2) || !ptg_fits_2g((long)M * K * 2)) return (int)hipErrorInvalidValue;
  const bf16_t* xb = (const bf16_t*)x;
  const bf16_t* wb = (const bf16_t*)w;
  if (M > 128) return launch_fwd<256>(xb, wb, part, M, N, K, splits, s);
  if (M > 64) return launch_fwd<128>(xb, wb, part, M, N, K, splits, s);
  if (M > 32) return launch_fwd<64>(xb, wb, part, M, N, K, splits, s);
  return launch_fwd<32>(xb, wb, part, M, N, K, splits, s);
}

// measurement variants of the forward at M in (128, 256] (tools/dense_bench.py): mode 1 no MFMA, 2 no
// partial stores, 3 neither, 4 nt weight loads
int ptg_dense_fwd_sk_dbg(const void* x, const void* w, float* part, int M, int N, int K, int splits, int mode,
                         hipStream_t s) {
  if (M > 256 || N % NT || K % (BK * splits) || ((N / NT) * splits) % 8) return (int)hipErrorInvalidValue;
  if (M <= 128 && mode < 8) return (int)hipErrorInvalidValue;
  const bf16_t* xb = (const bf16_t*)x;
  const bf16_t* wb = (const bf16_t*)w;
  switch (mode) {
    case 1: return launch_fwd<256, 1>(xb, wb, part, M, N, K, splits, s);
    case 2: return launch_fwd<256, 2>(xb, wb, part, M, N, K, splits, s);
    case 3: return launch_fwd<256, 3>(xb, wb, part, M, N, K, splits, s);
    case 4: return launch_fwd<256, 0, 2>(xb, wb, part, M, N, K, splits, s);
    case 5: return launch_fwd<256, 4>(xb, wb, part, M, N, K, splits, s);  // tiled-B addressing
    case 7: return launch_fwd<256, 7>(xb, wb, part, M, N, K, splits, s);  // tiled-B, DMA only
    case 8: return launch_fwd<32, 7>(xb, wb, part, M, N, K, splits, s);   // M=32 tile, tiled-B, DMA only
    case 9: return launch_fwd<32, 3>(xb, wb, part, M, N, K, splits, s);   // M=32 tile, DMA only
    default: return launch_fwd<256>(xb, wb, part, M, N, K, splits, s);
  }
}

}  // extern "C"
