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

#include <cstdlib>

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


// ------------------------------------------------------------------------------------------------
// dX of the big Dense layer: out[M][Kc] (bf16) = dy[M][Nr] . W[Nr][Kc]  (CNN-B1: Nr = 2048 units,
// Kc = 20480 inputs).  The weight is k-major for this product (W[n][k] with the reduction index n
// in the rows), the MFMA B operand needs 8 consecutive n per lane: W tiles go through LDS and are
// read with the transposed LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md T10).
//   * grid = Kc / 80 workgroups (256 for CNN-B1), each all M rows x 80 output columns over the
//     whole reduction: every weight byte is read once, no split-K partials.
//   * 8 waves x 32 rows.  A wave's dy rows are private to it, so its A fragments come straight
//     from global memory into registers (16 B per lane = one 16x16x32 fragment row, L2 hits: dy is
//     1 MB), prefetched P K-steps ahead in a register ring; only the shared W tiles use LDS.
//   * W stage = 64 rows x 80 cols (10 KB) by LDS-DMA, 10 wave-instructions per stage (2 per wave;
//     the 6 spare ones land OOB zeros in a scratch KB).  Inside each 16-row group the rows are
//     stored interleaved (global row 8h+r -> LDS row 2r+h) so that the two 4-row blocks a 32-lane
//     half reads in one transposed read fall on disjoint banks (row stride 160 B = 40 banks).
//   * per stage per wave 4 A loads + 2 DMA = 6 vector-memory ops in issue order: one counted
//     s_waitcnt vmcnt(6 (P-1)) + a barrier retires stage t for everyone.
// ------------------------------------------------------------------------------------------------
constexpr int DX_KT = 80, DX_BK = 64;
constexpr int DX_IMG = DX_BK * DX_KT * 2;  // 10 KB
constexpr int DX_SLOT = DX_IMG + 1024;     // + DMA scratch

// Row placement inside a 64-row W stage (an involution): bit 2 flips with bit 4.  LDS rows 160 B
// apart start 40 banks apart, so any 8 rows with distinct (row mod 8) start on the 8 distinct 8-bank
// groups; each transposed read of a 32-lane half covers rows {16g+8s+4h+q} for the half's two lane
// groups g = 2c, 2c+1 (q = 0..3), which this placement maps to 8 distinct residues mod 8.
PTG_DEV int dx_lds_row(int k) { return k ^ (((k >> 4) & 1) << 2); }
PTG_DEV int dx_glb_row(int kk) { return kk ^ (((kk >> 4) & 1) << 2); }

// ds_read_b64_tr_b16 as inline asm: the builtin form carries no alias information, so hipcc
// drains every LDS-DMA in flight (s_waitcnt vmcnt(0)) before each one, which serialises the
// weight stream.  The asm result is only valid after an lgkmcnt wait: dx_lgkm_fence() below, whose
// "+v" operands order every consumer (the MFMAs) after it.
typedef __attribute__((ext_vector_type(2))) unsigned dx_u2_t;
PTG_DEV dx_u2_t dx_tr_read(uint32_t lds_addr) {
  dx_u2_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr));
  return r;
}
PTG_DEV void dx_lgkm_fence(dx_u2_t (&r)[10]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]),
                 "+v"(r[8]), "+v"(r[9]));
}
PTG_DEV uint32_t dx_lds_addr(const unsigned char* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
}

template <int P>
__global__ __launch_bounds__(512) void dense_dx_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ w,
                                                  bf16_t* __restrict__ out, int M, int Nr, int Kc, uint32_t dybytes,
                                                  uint32_t wbytes) {
  constexpr int NS = P + 1;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col0 = blockIdx.x * DX_KT;
  const int nk = Nr / DX_BK;
  const bool live = wid * 32 < M;  // waves whose rows are all past M only move bytes
  const uint32_t lds0 = dx_lds_addr(smem);

  const Rsrc rsA = make_rsrc(dy, dybytes), rsB = make_rsrc(w, wbytes);
  uint32_t aoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = wid * 32 + i * 16 + (lane & 15);
    // lane group g holds k = 16g + 8s .. +7 of a 64-deep stage (s = the 32-deep MFMA step): its two
    // fragments are 32 contiguous bytes of the dy row
    aoff[i] = r < M ? (uint32_t)r * (uint32_t)Nr * 2u + 32u * (uint32_t)(lane >> 4) : PTG_OOB;
  }
  uint32_t boff[2];
  int bdst[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int b = wid + 8 * j;
    if (b < 10) {
      const int f = b * 64 + lane, kk = f / 10, c8 = f - kk * 10;
      boff[j] = (uint32_t)dx_glb_row(kk) * (uint32_t)Kc * 2u + (uint32_t)(col0 + c8 * 8) * 2u;
      bdst[j] = b * 1024;
    } else {
      boff[j] = PTG_OOB;
      bdst[j] = DX_IMG;
    }
  }
  const uint32_t bstep = (uint32_t)DX_BK * (uint32_t)Kc * 2u;

  bf16x8_t areg[NS][2][2];  // [slot][k32 half][row fragment]
  f32x4_t acc[2][5];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // tr-read geometry: lane group g = lane>>4 takes k rows 16g+8s .. +7 of MFMA step s (the order of
  // its A fragment); within the group lane 4q+p addresses row q, columns 4p..4p+3 of the 16-column block
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  int trow[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) trow[s][h] = dx_lds_row(16 * g + 8 * s + 4 * h + q) * (DX_KT * 2) + pq * 8;

#define DX_ISSUE(T, SL)                                                                                         \
  {                                                                                                             \
    const int t_ = (T);                                                                                         \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                                            \
      _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_)                                                          \
        areg[SL][s_][i_] = __builtin_bit_cast(bf16x8_t, bload16(rsA, (aoff[i_] == PTG_OOB || t_ >= nk) ? PTG_OOB  \
                                                                       : aoff[i_] + (uint32_t)(t_ * DX_BK + s_ * 8) * 2u)); \
    unsigned char* base_ = smem + (SL) * DX_SLOT;                                                               \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                                            \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t*)(base_ + bdst[j_]), 16,                             \
                                               boff[j_] == PTG_OOB ? PTG_OOB : boff[j_] + (uint32_t)t_ * bstep, \
                                               0, 0, 0);                                                        \
  }
// Every step issues its 6 loads unconditionally (stages past the end read OOB zeros, steps past the
// end add zeros): uniform control flow lets hipcc track the register ring's loads exactly; a
// conditional issue made it wait for the newest loads before every MFMA group.
#define DX_STEP(T, SL)                                                                                          \
  {                                                                                                             \
    wait_vm<6 * (P - 1)>();                                                                                     \
    __builtin_amdgcn_s_barrier();                                                                               \
    DX_ISSUE((T) + P, ((SL) + P) % NS)                                                                          \
    if (live) {                                                                                                 \
      const uint32_t img_ = lds0 + (SL) * DX_SLOT;                                                              \
      _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                                        \
        dx_u2_t tr_[10];                                                                                        \
        _Pragma("unroll") for (int j_ = 0; j_ < 5; ++j_) {                                                      \
          tr_[2 * j_] = dx_tr_read(img_ + trow[s_][0] + j_ * 32);                                               \
          tr_[2 * j_ + 1] = dx_tr_read(img_ + trow[s_][1] + j_ * 32);                                           \
        }                                                                                                       \
        dx_lgkm_fence(tr_);                                                                                     \
        bf16x8_t bf_[5];                                                                                        \
        _Pragma("unroll") for (int j_ = 0; j_ < 5; ++j_) {                                                      \
          U4 v_;                                                                                                \
          v_.x = tr_[2 * j_].x; v_.y = tr_[2 * j_].y; v_.z = tr_[2 * j_ + 1].x; v_.w = tr_[2 * j_ + 1].y;       \
          bf_[j_] = __builtin_bit_cast(bf16x8_t, v_);                                                           \
        }                                                                                                       \
        _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_)                                                        \
          _Pragma("unroll") for (int j_ = 0; j_ < 5; ++j_)                                                      \
            acc[i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(areg[SL][s_][i_], bf_[j_], acc[i_][j_], 0, 0, 0); \
      }                                                                                                         \
    }                                                                                                           \
  }

#pragma unroll
  for (int t = 0; t < P; ++t) DX_ISSUE(t, t)
  for (int t0 = 0; t0 < nk; t0 += NS) {
    DX_STEP(t0 + 0, 0)
    if constexpr (NS > 1) { DX_STEP(t0 + 1, 1 % NS) }
    if constexpr (NS > 2) { DX_STEP(t0 + 2, 2 % NS) }
    if constexpr (NS > 3) { DX_STEP(t0 + 3, 3 % NS) }
    if constexpr (NS > 4) { DX_STEP(t0 + 4, 4 % NS) }
    if constexpr (NS > 5) { DX_STEP(t0 + 5, 5 % NS) }
  }
#undef DX_STEP
#undef DX_ISSUE

  // epilogue: the tile through LDS as bf16 [256][80] (160-B rows), then 16-B coalesced row stores
  wait_vm<0>();
  __syncthreads();
  bf16_t* stile = (bf16_t*)smem;
  if (live) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          stile[(wid * 32 + i * 16 + (lane >> 4) * 4 + r) * DX_KT + j * 16 + (lane & 15)] = f2bf(acc[i][j][r]);
  }
  __syncthreads();
  const int rows = min(M, 256);
  for (int c = tid; c < rows * 10; c += 512) {
    const int r = c / 10, c8 = c - r * 10;
    *(U4*)(out + (long)r * Kc + col0 + c8 * 8) = *(const U4*)(stile + r * DX_KT + c8 * 8);
  }
}

// dX, all-LDS form: both operands by LDS-DMA.  Measured on the dense_dx_k form above (dy fragments
// loaded straight into registers): its 16-rows-x-64-B loads cost the texture addresser two line
// lookups per 128 B (TA busy 78 %, stalled by the L1 15.8 M cycles, 4.0 M L2 requests for 352 MB,
// 52 us), so here dy goes through LDS as whole 128-B rows like the forward's activations, and the
// 80-column W tiles of neighbouring workgroups (which share 128-B lines) run on one XCD.
//   stage = dy [256 rows][64 k] (32 KB, the forward's swizzled row image, 4 DMA per wave) + W [64 n][80]
//   (10 KB + 1 KB DMA scratch, 2 DMA per wave); 3-deep ring (129 KB), counted vmcnt(6) per stage.
PTG_DEV int dx2_lds_row(int k) { return (k & ~15) | ((k & 7) << 1) | ((k >> 3) & 1); }
PTG_DEV int dx2_glb_row(int kk) { return (kk & ~15) | ((kk & 1) << 3) | ((kk >> 1) & 7); }
constexpr int DX2_A = 256 * 128;              // dy image bytes per stage
constexpr int DX2_SLOT = DX2_A + DX_SLOT;      // + W image + scratch
constexpr int DX2_NS = 3;

__global__ __launch_bounds__(512) void dense_dx2_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ w,
                                                   bf16_t* __restrict__ out, int M, int Nr, int Kc, uint32_t dybytes,
                                                   uint32_t wbytes) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col0 = xcd_remap(blockIdx.x, gridDim.x) * DX_KT;  // neighbouring tiles share an L2
  const int nk = Nr / DX_BK;
  const bool live = wid * 32 < M;
  const uint32_t lds0 = dx_lds_addr(smem);
  const Rsrc rsA = make_rsrc(dy, dybytes), rsB = make_rsrc(w, wbytes);

  // 6 DMA per wave per stage: j = 0..3 the dy blocks wid + 8j (rows 8b..8b+7), j = 4, 5 the W blocks
  uint32_t goff[6];
  int dst[6];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = wid + 8 * j, row = b * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    goff[j] = row < M ? (uint32_t)row * (uint32_t)Nr * 2u + (uint32_t)chunk * 16u : PTG_OOB;
    dst[j] = b * 1024;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int b = wid + 8 * j;
    if (b < 10) {
      const int f = b * 64 + lane, kk = f / 10, c8 = f - kk * 10;
      goff[4 + j] = (uint32_t)dx2_glb_row(kk) * (uint32_t)Kc * 2u + (uint32_t)(col0 + c8 * 8) * 2u;
      dst[4 + j] = DX2_A + b * 1024;
    } else {
      goff[4 + j] = PTG_OOB;
      dst[4 + j] = DX2_A + DX_IMG;
    }
  }
  const uint32_t astep = DX_BK * 2u, bstep = (uint32_t)DX_BK * (uint32_t)Kc * 2u;
  auto issue = [&](int t) {
    unsigned char* base = smem + (t % DX2_NS) * DX2_SLOT;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t*)(base + dst[j]), 16,
                                               goff[j] == PTG_OOB ? PTG_OOB : goff[j] + (uint32_t)t * astep, 0, 0, 0);
#pragma unroll
    for (int j = 4; j < 6; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t*)(base + dst[j]), 16,
                                               goff[j] == PTG_OOB ? PTG_OOB : goff[j] + (uint32_t)t * bstep, 0, 0, 0);
  };

  // A fragment (16 rows, 16-B chunk cbase + lane>>4 of the swizzled 128-B row): lane group g holds
  // k = 8g..8g+7 of MFMA step s (cbase = 4s); B: the same k through two transposed reads
  const int fr = lane & 15, fc = lane >> 4;
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  int trow[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) trow[s][h] = DX2_A + dx2_lds_row(s * 32 + 8 * g + 4 * h + q) * (DX_KT * 2) + pq * 8;

  f32x4_t acc[2][5];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < DX2_NS - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    if (t + DX2_NS - 2 < nk) wait_vm<6 * (DX2_NS - 2)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (t + DX2_NS - 1 < nk) issue(t + DX2_NS - 1);
    if (!live) continue;
    const int slot = (t % DX2_NS) * DX2_SLOT;
    const unsigned char* sA = smem + slot;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      dx_u2_t tr[10];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        tr[2 * j] = dx_tr_read(lds0 + slot + trow[s][0] + j * 32);
        tr[2 * j + 1] = dx_tr_read(lds0 + slot + trow[s][1] + j * 32);
      }
      bf16x8_t af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wid * 32 + i * 16 + fr;
        const int pos = (4 * s + fc) ^ ((r >> 1) & 7);
        af[i] = __builtin_bit_cast(bf16x8_t, *(const U4*)(sA + r * 128 + pos * 16));
      }
      dx_lgkm_fence(tr);
      bf16x8_t bf[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        U4 v;
        v.x = tr[2 * j].x; v.y = tr[2 * j].y; v.z = tr[2 * j + 1].x; v.w = tr[2 * j + 1].y;
        bf[j] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }

  wait_vm<0>();
  __syncthreads();
  bf16_t* stile = (bf16_t*)smem;
  if (live) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          stile[(wid * 32 + i * 16 + (lane >> 4) * 4 + r) * DX_KT + j * 16 + (lane & 15)] = f2bf(acc[i][j][r]);
  }
  __syncthreads();
  const int rows = min(M, 256);
  for (int c = tid; c < rows * 10; c += 512) {
    const int r = c / 10, c8 = c - r * 10;
    *(U4*)(out + (long)r * Kc + col0 + c8 * 8) = *(const U4*)(stile + r * DX_KT + c8 * 8);
  }
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


// dX of a big Dense layer: out[M][Kc] bf16 = dy[M][Nr] . w[Nr][Kc] (w row-major [Nr][Kc], the layer's
// [units][fan_in] weight).  Requirements (checked): M <= 256, Nr % 64 == 0, Kc % 80 == 0, operands
// < 2 GiB; `out` rows are Kc apart (16-B aligned rows).
int ptg_dense_dx(const void* dy, const void* w, void* out, int M, int Nr, int Kc, hipStream_t s) {
  if (M <= 0 || M > 256 || Nr <= 0 || Nr % DX_BK || Kc <= 0 || Kc % DX_KT) return (int)hipErrorInvalidValue;
  if (!ptg_fits_2g((long)Nr * Kc * 2) || !ptg_fits_2g((long)M * Nr * 2)) return (int)hipErrorInvalidValue;
  static int variant = -1;
  if (variant < 0) {
    const char* e = getenv("PTG_DENSE_DX_REG");  // A/B: 1 = dy fragments straight into registers
    variant = e && e[0] == '1' ? 1 : 0;
    (void)hipFuncSetAttribute((const void*)dense_dx2_k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              DX2_NS * DX2_SLOT);
  }
  if (variant == 1) {
    constexpr int P = 4;
    hipLaunchKernelGGL((dense_dx_k<P>), dim3(Kc / DX_KT), dim3(512), (P + 1) * DX_SLOT, s, (const bf16_t*)dy,
                       (const bf16_t*)w, (bf16_t*)out, M, Nr, Kc, (uint32_t)((long)M * Nr * 2),
                       (uint32_t)((long)Nr * Kc * 2));
  } else {
    hipLaunchKernelGGL(dense_dx2_k, dim3(Kc / DX_KT), dim3(512), DX2_NS * DX2_SLOT, s, (const bf16_t*)dy,
                       (const bf16_t*)w, (bf16_t*)out, M, Nr, Kc, (uint32_t)((long)M * Nr * 2),
                       (uint32_t)((long)Nr * Kc * 2));
  }
  PTG_RETURN_LAUNCH();
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
