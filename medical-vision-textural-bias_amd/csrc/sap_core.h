// sap_core.h -- salt-and-pepper per-voxel logic (filters_and_operators.py:465-482), Philox RNG,
// and the order-preserving float<->uint32 keys used for the per-sample MIN/MAX.
// Shared by the gfx950 kernels and the host test emulator.
#pragma once

#include <stdint.h>

#include "fft_core.h"

namespace tb {

// order-preserving key: a < b  <=>  key(a) < key(b)  (for non-NaN floats)
TB_HD uint32_t f2key(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
TB_HD float key2f(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}

// Philox4x32-10 (Salmon et al., SC'11): counter (c0..c3), key (k0,k1) -> 4 x uint32
struct u32x4 { uint32_t v[4]; };
TB_HD void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}
TB_HD u32x4 philox(uint64_t ctr, uint64_t stream, uint64_t seed) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = (uint32_t)stream, c3 = (uint32_t)(stream >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo(0xD2511F53u, c0, hi0, lo0);
    mulhilo(0xCD9E8D57u, c2, hi1, lo1);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  u32x4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}
// uniform in [0,1) with 24 random bits (exact in float32, like torch.rand's float path)
TB_HD float u01(uint32_t r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

// classification of SaltAndPepper.salt_and_pepper (:478-479): 1 = MIN, 2 = MAX, 0 = keep
TB_HD int sap_class(float u, float lo, float hi) { return u <= lo ? 1 : (u <= hi ? 2 : 0); }

}  // namespace tb
