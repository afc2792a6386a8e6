// Helpers shared by the halo-tiled convolution kernels (conv.hip, conv1.hip).
#pragma once
#include "common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

namespace ptgc {

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group supplies the address of row q, 4 columns;
// lane i of the group receives column i of the 4 rows (row q in element q).
PTG_DEV s16x4_t tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p));
}

// The 6 bytes of an RGB pixel pair at byte offset o (o even) as two ALIGNED dword loads covering
// [o & ~3, +8); sh = 8 * (o & 3) selects them.  The rsrc size is rounded up to 4 bytes, so the last
// pair's window stays in range (the caching allocator's 512-byte rounding backs the 2 extra bytes).
struct U8Pair { uint32_t w0, w1, sh; };
PTG_DEV U8Pair u8pair_load(Rsrc r, uint32_t o, bool ok) {
  const uint32_t a = o & ~3u;
  return U8Pair{bload4(r, ok ? a : PTG_OOB), bload4(r, ok ? a + 4u : PTG_OOB), (o & 3u) * 8u};
}
PTG_DEV U4 u8pair_to_bf16x8(const U8Pair& p) {
  constexpr float s = 1.f / 255.f;
  const unsigned long long v = (((unsigned long long)p.w1 << 32) | p.w0) >> p.sh;
  auto c = [&](int i) { return (float)((uint32_t)(v >> (8 * i)) & 255u) * s; };
  U4 o;
  o.x = pack_bf(c(0), c(1));
  o.y = pack_bf(c(2), 0.f);
  o.z = pack_bf(c(3), c(4));
  o.w = pack_bf(c(5), 0.f);
  return o;
}
PTG_DEV uint32_t u8_rsrc_bytes(long n_bytes) { return (uint32_t)((n_bytes + 3) & ~3L); }


}  // namespace ptgc
