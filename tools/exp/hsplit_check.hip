// h3 split check: hsplit2 (multiply + fma_mix form, mfma.h) against the
// ldexp form it replaced, over random bit patterns of every exponent and every
// shift the scale selection can produce; prints the mismatch count.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/hsplit_check.hip -o tools/exp/hsplit_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../molclr_amd/csrc/common.h"
#include "../../molclr_amd/csrc/mfma.h"
using namespace molclr;

__device__ __forceinline__ void ref2(float a, float b, int sh, uint32_t& h, uint32_t& l) {
  a = __builtin_ldexpf(a, sh);
  b = __builtin_ldexpf(b, sh);
  const f16x2 hh = {(_Float16)a, (_Float16)b};
  const f16x2 ll = {(_Float16)(a - (float)hh[0]), (_Float16)(b - (float)hh[1])};
  h = __builtin_bit_cast(uint32_t, hh);
  l = __builtin_bit_cast(uint32_t, ll);
}

__device__ uint32_t mix32(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(x ^ (x >> 31));
}

// thread t: shift sh = -113 + (t % 241) (h3_shift_of's range [-113, 127]); two
// values whose magnitude lies within 2^15 of 2^-sh (what the shift is chosen
// for) or anywhere (random bit patterns, NaN / inf excluded)
__global__ void k_check(uint64_t n, uint32_t* bad, uint32_t* first) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int sh = -113 + (int)(t % 241);
  uint32_t ua = mix32(2 * t), ub = mix32(2 * t + 1);
  if (t & 1) {  // near the scale: exponent e with e + sh in [-40, 15]
    const int ea = (int)(mix32(3 * t) % 56) - 40 - sh + 127;
    const int eb = (int)(mix32(5 * t) % 56) - 40 - sh + 127;
    ua = (ua & 0x807FFFFFu) | ((uint32_t)(ea < 0 ? 0 : ea > 254 ? 254 : ea) << 23);
    ub = (ub & 0x807FFFFFu) | ((uint32_t)(eb < 0 ? 0 : eb > 254 ? 254 : eb) << 23);
  }
  if (((ua >> 23) & 0xFF) == 0xFF) ua &= 0xBFFFFFFFu;
  if (((ub >> 23) & 0xFF) == 0xFF) ub &= 0xBFFFFFFFu;
  const float a = __builtin_bit_cast(float, ua), b = __builtin_bit_cast(float, ub);
  // the contract: a shift chosen from the max puts every |x 2^sh| below 2^15
  // (beyond fp16's range the two forms differ only in which of inf / NaN lo
  // gets: the fma never overflows its product)
  if (!(fabsf(__builtin_ldexpf(a, sh)) < 32768.f) || !(fabsf(__builtin_ldexpf(b, sh)) < 32768.f))
    return;
  uint32_t h0, l0, h1, l1;
  ref2(a, b, sh, h0, l0);
  hsplit2(a, b, sh, h1, l1);
  // halves equal, or both zeros: where x 2^sh is below fp16's range the old
  // form's lo is (x 2^sh rounded to f32) - hi = +0 while the fma keeps the
  // sign of the exact residual (-0); an MFMA sum from +0 cannot tell them apart
  auto same = [](uint32_t x, uint32_t y) {
    const uint32_t d = x ^ y;
    const bool lo_ok = (d & 0xFFFFu) == 0 || (((x | y) & 0x7FFFu) == 0);
    const bool hi_ok = (d >> 16) == 0 || ((((x | y) >> 16) & 0x7FFFu) == 0);
    return lo_ok && hi_ok;
  };
  if (!same(h0, h1) || !same(l0, l1)) {
    if (atomicAdd(bad, 1u) == 0) {
      first[0] = ua; first[1] = ub; first[2] = (uint32_t)sh;
      first[3] = h0; first[4] = l0; first[5] = h1; first[6] = l1;
    }
  }
}

int main() {
  const uint64_t n = 1ull << 30;
  uint32_t *bad, *first;
  if (hipMalloc(&bad, 4) || hipMalloc(&first, 32)) return 2;
  hipMemset(bad, 0, 4);
  k_check<<<(unsigned)(n / 256), 256>>>(n, bad, first);
  uint32_t hb = 0, hf[8] = {};
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  hipMemcpy(hf, first, 28, hipMemcpyDeviceToHost);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  printf("hsplit2 vs ldexp form: %llu pairs, %u mismatches\n", (unsigned long long)n, hb);
  if (hb)
    printf("first: a %08x b %08x sh %d ref (%08x, %08x) new (%08x, %08x)\n", hf[0], hf[1],
           (int)hf[2], hf[3], hf[4], hf[5], hf[6]);
  return hb ? 1 : 0;
}
