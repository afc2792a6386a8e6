// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of pyspark_tf_gke_amd.
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 tensors are carried as raw uint16_t storage (bf16_t) and converted with
//     bf2f / f2bf (f2bf lowers to v_cvt_pk_bf16_f32, round-to-nearest-even, NaN-preserving).
//   * wave64: lane = threadIdx.x & 63, wave = threadIdx.x >> 6. Never 32.
//   * every host entry point is `extern "C" int ptg_*(..., hipStream_t)` returning the
//     hipError_t of the launch, so the Python side can fail loudly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;   // MFMA A/B fragment (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) float f32x4_t;     // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16_t;   // 32x32 MFMA accumulator

struct alignas(16) U4 { uint32_t x, y, z, w; };
struct alignas(8) U2 { uint32_t x, y; };

#define PTG_DEV __device__ __forceinline__

PTG_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
PTG_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
PTG_DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
PTG_DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
PTG_DEV uint32_t pack_bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
// unpack a 16-byte vector of 8 bf16 into floats
PTG_DEV void unpack8(const U4& v, float* f) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z); f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}
PTG_DEV U4 pack8(const float* f) {
  U4 v;
  v.x = pack_bf(f[0], f[1]); v.y = pack_bf(f[2], f[3]);
  v.z = pack_bf(f[4], f[5]); v.w = pack_bf(f[6], f[7]);
  return v;
}
PTG_DEV U4 zero4() { U4 z; z.x = z.y = z.z = z.w = 0u; return z; }

PTG_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
PTG_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == 256 (4 waves). `scratch` must hold >= 4 floats.
PTG_DEV float block_sum256(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float r = scratch[0] + scratch[1] + scratch[2] + scratch[3];
  return r;
}

// XCD-aware, bijective remap of a linear workgroup id (cdna_hip_programming.md §5, T1):
// blocks b and b+8 share an XCD under round-robin dispatch; give each XCD a contiguous
// chunk of the tile space so neighbouring tiles share that XCD's L2.
PTG_DEV int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Buffer loads (cdna_hip_programming.md T8): 32-bit byte offsets against a descriptor built once
// from kernel arguments; every offset >= the descriptor's byte count (use PTG_OOB) reads as zero
// through the hardware range check, so zero padding / tails need no branch.  Operands < 2 GiB.
constexpr uint32_t PTG_OOB = 0x80000000u;
typedef __amdgpu_buffer_rsrc_t Rsrc;
PTG_DEV Rsrc make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
PTG_DEV U4 bload16(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
PTG_DEV U2 bload8(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(U2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
PTG_DEV uint32_t bload4(Rsrc r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0); }
// vector buffer stores (offsets >= the descriptor's byte count are dropped by the range check)
typedef __attribute__((ext_vector_type(2))) unsigned int ptg_vu2_t;
PTG_DEV void bstore8(Rsrc r, uint32_t off, U2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(ptg_vu2_t{v.x, v.y}, r, off, 0, 0);
}
PTG_DEV void bstore4(Rsrc r, uint32_t off, uint32_t v) { __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 0); }
static inline bool ptg_fits_2g(long bytes) { return bytes > 0 && bytes < (long)PTG_OOB; }

static inline int ptg_ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Division by a runtime-invariant divisor without the ~30-instruction integer division sequence:
// round-up multiply-high (Granlund-Montgomery / libdivide "branchfree" u32), exact for every 32-bit
// dividend: q = (t + ((n - t) >> 1)) >> s with t = mulhi(n, m).  d == 1 is selected explicitly (its
// magic would need 33 bits).  Built on the host with fastdiv(d).
struct FastDiv {
  uint32_t d, m, s;
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint32_t t = __umulhi(n, m);
    const uint32_t q = (t + ((n - t) >> 1)) >> s;
    return d == 1u ? n : q;
  }
};
static inline FastDiv fastdiv(uint32_t d) {
  FastDiv f{d, 0u, 0u};
  if (d <= 1) return f;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;  // l = ceil(log2 d) >= 1
  f.m = (uint32_t)(((((unsigned __int128)1) << 32) * ((1ull << l) - d)) / d + 1);
  f.s = l - 1;
  return f;
}

#define PTG_RETURN_LAUNCH() return (int)hipGetLastError()

// Workgroups of `kernel` (256 threads) resident at once on the whole device: the grid of a
// persistent kernel (more would queue behind workgroups that only exit at the end).
static inline int ptg_resident_blocks(const void* kernel) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0) per_cu = 2;
  return cus * per_cu;
}

// ---- checked builds (-DPTG_CHECKED -> libptg_hip_checked.so, selected with PTG_CHECKED=1) ----
// PTG_CHECKED_IDX(i, n) is i when 0 <= i < n.  Otherwise it records the source line in this
// translation unit's ptg_check_line (first failure wins) and yields 0, so the access stays in
// bounds and the kernel never faults; the host reads and clears the line after every launch
// (PTG_CHECK_STATUS -> ptg_check_status_<tu>, polled by pyspark_tf_gke_amd._native).  Unchecked
// builds compile the macro to plain i.
#ifdef PTG_CHECKED
static __device__ unsigned int ptg_check_line;
PTG_DEV long long ptg_checked_idx(long long i, long long n, int line) {
  if ((unsigned long long)i < (unsigned long long)n) return i;
  atomicCAS(&ptg_check_line, 0u, (unsigned)line);
  return 0;
}
#define PTG_CHECKED_IDX(i, n) ptg_checked_idx((long long)(i), (long long)(n), __LINE__)
#define PTG_CHECK_STATUS(tu)                                                      \
  extern "C" int ptg_check_status_##tu() {                                        \
    unsigned int v = 0, z = 0;                                                    \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(ptg_check_line), sizeof(v)) != hipSuccess) return -1; \
    if (v) hipMemcpyToSymbol(HIP_SYMBOL(ptg_check_line), &z, sizeof(z));          \
    return (int)v;                                                                \
  }
#else
#define PTG_CHECKED_IDX(i, n) (i)
#define PTG_CHECK_STATUS(tu)
#endif
