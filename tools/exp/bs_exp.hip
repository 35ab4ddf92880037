// B-stationary h3 GEMM experiment (NOT part of the product library; built by
// tools/exp/build_bs_exp.sh, driven by tools/bs_exp.py).
//
// k_gemm_pp (gemm.hip) stages B (the weight's fp16 planes) through LDS once
// per 32-deep K step behind block barriers, and its waves stall ~half their
// lifetime (profiles/r5_pmc_h3_lin1).  For K <= 320 a whole 128-column tile of
// B fits the 160 KB LDS: here each block loads its tile ONCE, then every wave
// streams its own 32-row slabs of A (global -> registers, split, MFMA) with
// no barrier at all; the same fragments, the same three products in the same
// order as the pp kernel's swapped form, so C is bit-identical.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "molclr.h"
#include "../../molclr_amd/csrc/mfma.h"

using namespace molclr;

namespace {

constexpr int kBN = 128;  // columns per tile (TN = 4)
constexpr int kTN = 4;
constexpr int kFullImg = 2 * kBN * XK;  // fp16 elements of one full K step (both planes)
constexpr int kHalfImg = 2 * kBN * 16;  // ... of a last step holding k0 .. k0+15 only

// offset (fp16 units) of chunk c (0 or 1) of row `row` in a half-step plane:
// 32 B per row, the two chunks swapped on alternate row quads
__device__ __forceinline__ int hoff(int row, int c) { return row * 16 + ((c ^ ((row >> 2) & 1)) << 3); }

// S full steps of 32 k, the last of which holds only its first 16 k when
// HALF (K - 32 (S - 1) <= 16: the lane half lh = 1 of the last step is all
// k >= K, whose A is zero, so its B fragment is replaced by zeros)
// ABL (ablations; results then differ): 1 no MFMA, 2 A rows folded onto the
// first slab (cache-hot), 4 no C stores
template <int EPI, int H3, int S, bool HALF, int W = 8, int DEP = 2, int ABL = 0>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(W / 4))) void k_gemm_bs(
    const float* __restrict__ A, const uint16_t* __restrict__ Bp, float* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux, int accumulate,
    const float* __restrict__ amax, const float* __restrict__ bmax, float* __restrict__ cmax,
    float* __restrict__ crow, float* __restrict__ amax_out, int arow_parts,
    uint32_t* __restrict__ bits_out, const uint32_t* __restrict__ bits_in, int64_t bits_ld,
    int ntn, int groups) {
  constexpr int NFULL = HALF ? S - 1 : S;
  constexpr int IMG = NFULL * kFullImg + (HALF ? kHalfImg : 0);
  __shared__ __attribute__((aligned(16))) uint16_t img[IMG];
  __shared__ __attribute__((aligned(16))) float bsh[kBN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  // logical block: XCD-contiguous, the ntn column tiles of one row group adjacent
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = L % ntn, grp = L / ntn;
  const int64_t n0 = (int64_t)tile * kBN;
  const int64_t slabs = (M + 31) / 32;
  const int64_t s_beg = slabs * grp / groups, s_end = slabs * (grp + 1) / groups;

  // ---- the tile's B planes into LDS, once (LDS-DMA), and its bias ----------
  const __amdgpu_buffer_rsrc_t brsrc = make_rsrc(Bp, (int64_t)2 * npad * kp * 2);
  {
    // full steps: chunk q = (step, plane, 16-row group) of 1 KB; lane l writes
    // physical chunk l % 4 of image row l / 4 (source swizzled as xoff)
    constexpr int CHF = NFULL * 2 * (kBN / 16);
    for (int q = w; q < CHF; q += W) {
      const int st = q / (2 * (kBN / 16)), rem = q % (2 * (kBN / 16));
      const int pl = rem / (kBN / 16), r0 = (rem % (kBN / 16)) * 16;
      const int row = r0 + (lane >> 2), c = lane & 3;
      int64_t gr = n0 + row;
      gr = gr < npad ? gr : npad - 1;
      const uint32_t voff = (uint32_t)(((pl * npad + gr) * kp + 32 * st + 8 * (c ^ ((row >> 2) & 3))) * 2);
      buf_lds16(brsrc, img + st * kFullImg + pl * kBN * XK + r0 * XK, voff, 0);
    }
    if constexpr (HALF) {
      // the last step's first 16 k: 512 B chunks of 32 rows x 32 B
      constexpr int CHH = 2 * (kBN / 32);
      for (int q = w; q < CHH; q += W) {
        const int pl = q / (kBN / 32), r0 = (q % (kBN / 32)) * 32;
        const int row = r0 + (lane >> 1), c = lane & 1;
        int64_t gr = n0 + row;
        gr = gr < npad ? gr : npad - 1;
        const uint32_t voff =
            (uint32_t)(((pl * npad + gr) * kp + 32 * (S - 1) + 8 * (c ^ ((row >> 2) & 1))) * 2);
        buf_lds16(brsrc, img + NFULL * kFullImg + pl * kBN * 16 + r0 * 16, voff, 0);
      }
    }
    constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;
    if constexpr (HAS_BIAS) {
      if (tid < kBN) bsh[tid] = n0 + tid < N ? bias[n0 + tid] : 0.f;
    }
    vm_wait<0>();
    __syncthreads();
  }

  const int shb = h3_shift(bmax);
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(A, M * lda * 4);
  float cm = 0.f;   // max |C| of this lane's stores (cmax)
  float ain = 0.f;  // max |A| of its loads (amax_out)

  // this wave's slabs: s_beg + w, + 8, ...
  for (int64_t slab = s_beg + w; slab < s_end; slab += W) {
    const int64_t mw = slab * 32;
    int64_t arow_i = mw + li;
    arow_i = arow_i < M ? arow_i : M - 1;
    const uint32_t avoff = (uint32_t)((((ABL & 2) ? (arow_i & 31) : arow_i) * lda + 16 * lh) * 4);
    auto load_a = [&](int r, float4(&v)[4]) {
      const uint32_t soff = (uint32_t)(r * BK * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = buf_ld4(arsrc, avoff + 16 * j, soff);
    };
    int sha = 0;
    if constexpr (H3 == 1) sha = h3_shift(amax);
    if constexpr (H3 == 2) {
      float m = 0.f;
      if (arow_parts < 0)
        m = row_max_of_waves(reinterpret_cast<const float2*>(amax), arow_i, -arow_parts);
      else
        for (int p = 0; p < arow_parts; ++p) m = fmaxf(m, amax[(int64_t)p * M + arow_i]);
      sha = h3_shift_of(m);
    }
    uint32_t mws[kTN];
    if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
#pragma unroll
      for (int b = 0; b < kTN; ++b) {
        int64_t nb = n0 + 32 * b;
        nb = nb < N ? nb : 0;
        mws[b] = bits_in[(nb >> 5) * bits_ld + arow_i];
      }
    }
    f32x16 acc[kTN];
#pragma unroll
    for (int b = 0; b < kTN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

    // A two steps ahead in two register sets: step r consumes set r & 1 into
    // its fragments, then reloads that set with step r + 2
    float4 ar[DEP][4];
#pragma unroll
    for (int d = 0; d < DEP; ++d)
      if (d < S) load_a(d, ar[d]);
    u32x4 fr[2][2];  // this step's A fragments [sub-step][hi / lo]
    // the step's 2 x kTN MFMA blocks; block k + 1's B fragments read from LDS
    // under block k's MFMAs (pinned by sched_group_barrier, as k_gemm_pp)
    auto compute = [&](const uint16_t* base) {
      constexpr int NB = 2 * kTN;
      auto rd = [&](int k, u32x4(&f)[2]) {
        const int s1 = k / kTN, b1 = k % kTN;
        const int row = 32 * b1 + li;
        f[0] = *reinterpret_cast<const u32x4*>(base + xoff(row, 2 * lh + s1));
        f[1] = *reinterpret_cast<const u32x4*>(base + kBN * XK + xoff(row, 2 * lh + s1));
      };
      u32x4 q[2][2];
      rd(0, q[0]);
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int s = k / kTN, b = k % kTN;
        if (k + 1 < NB) rd(k + 1, q[(k + 1) & 1]);
        if constexpr ((ABL & 1) != 0) {
          acc[b][0] += __builtin_bit_cast(float, q[k & 1][0].x ^ fr[s][0].x);
          continue;
        }
        acc[b] = mfma_h3_t(__builtin_bit_cast(f16x8, fr[s][0]), __builtin_bit_cast(f16x8, fr[s][1]),
                           __builtin_bit_cast(f16x8, q[k & 1][0]),
                           __builtin_bit_cast(f16x8, q[k & 1][1]), acc[b]);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int k = 0; k < NB; ++k) {
#pragma unroll
        for (int mm = 0; mm < 3; ++mm) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (k + 1 < NB && mm < 2) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    };
    // the last step with only k0 .. k0 + 15 staged: lane half 1 multiplies zeros
    auto compute_half = [&]() {
      const uint16_t* base = img + NFULL * kFullImg;
      const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < 2 * kTN; ++k) {
        const int s = k / kTN, b = k % kTN;
        const int row = 32 * b + li;
        const u32x4 h = *reinterpret_cast<const u32x4*>(base + hoff(row, s));
        const u32x4 l = *reinterpret_cast<const u32x4*>(base + kBN * 16 + hoff(row, s));
        acc[b] = mfma_h3_t(__builtin_bit_cast(f16x8, fr[s][0]), __builtin_bit_cast(f16x8, fr[s][1]),
                           __builtin_bit_cast(f16x8, lh ? z : h), __builtin_bit_cast(f16x8, lh ? z : l),
                           acc[b]);
      }
    };
    auto step = [&](auto P, int r) {
      float4(&a)[4] = ar[decltype(P)::value];
      // A(r) landed; the DEP - 1 steps after it may still be in flight
      if (DEP == 3 && r + 2 < S) vm_wait<8>();
      else if (r + 1 < S) vm_wait<4>();
      else vm_wait<0>();
      if (amax_out != nullptr) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          ain = fmaxf(ain, fmaxf(fmaxf(fabsf(a[j].x), fabsf(a[j].y)), fmaxf(fabsf(a[j].z), fabsf(a[j].w))));
      }
      if (r == S - 1) {  // k >= K of the last step: zero (wave-uniform branch)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if ((int64_t)r * BK + 16 * lh + 4 * j >= K) a[j] = f4zero();
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) hsplit8(a[2 * s], a[2 * s + 1], sha, fr[s][0], fr[s][1]);
      if (r + DEP < S) load_a(r + DEP, a);
      if (HALF && r == S - 1) compute_half();
      else compute(img + r * kFullImg);
    };
#pragma unroll 1
    for (int r = 0; r < S; r += DEP) {
      step(std::integral_constant<int, 0>{}, r);
      if (r + 1 < S) step(std::integral_constant<int, 1>{}, r + 1);
      if constexpr (DEP == 3)
        if (r + 2 < S) step(std::integral_constant<int, DEP == 3 ? 2 : 0>{}, r + 2);
    }

    // ---- epilogue: lane (li, lh) holds row mw + li, columns nb + 8 q + 4 lh ..
    const int64_t m = mw + li;
    const float sc = __builtin_ldexpf(1.f, -(sha + shb));
    float rmax = 0.f;
#pragma unroll
    for (int b = 0; b < kTN; ++b) {
      const int64_t nb = n0 + 32 * b;
      if (nb >= N) break;
      uint32_t pos = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cb = 8 * q + 4 * lh;
        const int64_t n = nb + cb;
        if (m < M && n < N) {
          float* o = C + m * ldc + n;
          float4 v = make_float4(acc[b][4 * q] * sc, acc[b][4 * q + 1] * sc, acc[b][4 * q + 2] * sc,
                                 acc[b][4 * q + 3] * sc);
          if constexpr (EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU) {
            v = f4add(v, *reinterpret_cast<const float4*>(bsh + 32 * b + cb));
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
            const uint32_t mk = (mws[b] >> cb) & 15u;
            v = make_float4(mk & 1u ? v.x : 0.f, mk & 2u ? v.y : 0.f, mk & 4u ? v.z : 0.f,
                            mk & 8u ? v.w : 0.f);
          }
          if (accumulate) v = f4add(v, *reinterpret_cast<const float4*>(o));
          if (!(ABL & 4) || v.x == 1.2345f) *reinterpret_cast<float4*>(o) = v;
          rmax = fmaxf(rmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          pos |= ((v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
                  (v.w > 0.f ? 8u : 0u)) << cb;
        }
      }
      if (bits_out != nullptr) {
        pos |= __shfl_xor(pos, 32, 64);
        if (lh == 0 && m < M) bits_out[(nb >> 5) * bits_ld + m] = pos;
      }
    }
    if (crow != nullptr) {
      const float v = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
      if (lh == 0 && m < M) crow[(int64_t)tile * M + m] = v;
    }
    cm = fmaxf(cm, rmax);
  }
  if (cmax != nullptr) absmax_publish(cm, cmax);
  if (amax_out != nullptr) absmax_publish(ain, amax_out);
}


// bs2: the same products, pipelined across slabs.  A wave's next slab --
// its row maxima, ReLU-mask words and first two A steps -- is issued during
// the current slab's last two steps and waited for BEFORE the current
// slab's C stores, so the next slab's first two steps run without a memory
// wait; the stores then drain under those steps' MFMAs (any wait for a load
// while stores are pending is a full drain on this target).  The first
// slab's loads go out with the B image's LDS-DMA: one latency for both.
template <int EPI, int H3, int S, bool HALF, int W = 8, int DEP = 2>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(W / 4))) void k_gemm_bs2(
    const float* __restrict__ A, const uint16_t* __restrict__ Bp, float* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux, int accumulate,
    const float* __restrict__ amax, const float* __restrict__ bmax, float* __restrict__ cmax,
    float* __restrict__ crow, float* __restrict__ amax_out, int arow_parts,
    uint32_t* __restrict__ bits_out, const uint32_t* __restrict__ bits_in, int64_t bits_ld,
    int ntn, int groups) {
  static_assert(S % 2 == 0 && S >= 4, "two A register sets, steps in pairs");
  constexpr int NFULL = HALF ? S - 1 : S;
  constexpr int IMG = NFULL * kFullImg + (HALF ? kHalfImg : 0);
  __shared__ __attribute__((aligned(16))) uint16_t img[IMG];
  __shared__ __attribute__((aligned(16))) float bsh[kBN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = L % ntn, grp = L / ntn;
  const int64_t n0 = (int64_t)tile * kBN;
  const int64_t slabs = (M + 31) / 32;
  const int64_t s_beg = slabs * grp / groups, s_end = slabs * (grp + 1) / groups;
  constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;

  const __amdgpu_buffer_rsrc_t brsrc = make_rsrc(Bp, (int64_t)2 * npad * kp * 2);
  {
    constexpr int CHF = NFULL * 2 * (kBN / 16);
    for (int q = w; q < CHF; q += W) {
      const int st = q / (2 * (kBN / 16)), rem = q % (2 * (kBN / 16));
      const int pl = rem / (kBN / 16), r0 = (rem % (kBN / 16)) * 16;
      const int row = r0 + (lane >> 2), c = lane & 3;
      int64_t gr = n0 + row;
      gr = gr < npad ? gr : npad - 1;
      const uint32_t voff = (uint32_t)(((pl * npad + gr) * kp + 32 * st + 8 * (c ^ ((row >> 2) & 3))) * 2);
      buf_lds16(brsrc, img + st * kFullImg + pl * kBN * XK + r0 * XK, voff, 0);
    }
    if constexpr (HALF) {
      constexpr int CHH = 2 * (kBN / 32);
      for (int q = w; q < CHH; q += W) {
        const int pl = q / (kBN / 32), r0 = (q % (kBN / 32)) * 32;
        const int row = r0 + (lane >> 1), c = lane & 1;
        int64_t gr = n0 + row;
        gr = gr < npad ? gr : npad - 1;
        const uint32_t voff =
            (uint32_t)(((pl * npad + gr) * kp + 32 * (S - 1) + 8 * (c ^ ((row >> 2) & 1))) * 2);
        buf_lds16(brsrc, img + NFULL * kFullImg + pl * kBN * 16 + r0 * 16, voff, 0);
      }
    }
    if constexpr (HAS_BIAS) {
      if (tid < kBN) bsh[tid] = n0 + tid < N ? bias[n0 + tid] : 0.f;
    }
  }
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(A, M * lda * 4);
  float cm = 0.f, ain = 0.f;

  // per-slab state: the lane's A row, its raw row-maximum words (folded when
  // the slab starts), the ReLU-mask words
  int64_t arow = 0;
  uint32_t avoff = 0;
  float rw[8];
  uint32_t mws[kTN];
  auto meta_issue = [&](int64_t slab) {
    arow = slab * 32 + li;
    arow = arow < M ? arow : M - 1;
    avoff = (uint32_t)((arow * lda + 16 * lh) * 4);
    if constexpr (H3 == 2) {
      if (arow_parts < 0) {  // per-wave pairs: <= 3 float2 words of the producer
        const int d4 = -arow_parts;
        const int64_t s0 = arow * d4, e0 = s0 + d4 - 1;
        const float2* wm = reinterpret_cast<const float2*>(amax);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int64_t wi = (s0 >> 6) + q;
          const float2 v = wm[wi <= (e0 >> 6) ? wi : (s0 >> 6)];
          rw[2 * q] = v.x;
          rw[2 * q + 1] = v.y;
        }
      } else {
#pragma unroll
        for (int p = 0; p < 8; ++p) rw[p] = amax[(int64_t)(p < arow_parts ? p : 0) * M + arow];
      }
    }
    if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
#pragma unroll
      for (int b = 0; b < kTN; ++b) {
        int64_t nb = n0 + 32 * b;
        nb = nb < N ? nb : 0;
        mws[b] = bits_in[(nb >> 5) * bits_ld + arow];
      }
    }
  };
  auto row_shift = [&]() -> int {
    if constexpr (H3 == 1) return h3_shift(amax);
    float m = 0.f;
    if (arow_parts < 0) {
      const int d4 = -arow_parts;
      const int64_t s0 = arow * d4, e0 = s0 + d4 - 1;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int64_t wi = (s0 >> 6) + q;
        if (wi <= (e0 >> 6)) m = fmaxf(m, (wi << 6) / d4 == arow ? rw[2 * q] : rw[2 * q + 1]);
      }
    } else {
#pragma unroll
      for (int p = 0; p < 8; ++p)
        if (p < arow_parts) m = fmaxf(m, rw[p]);
    }
    return h3_shift_of(m);
  };
  auto load_a = [&](int r, float4(&v)[4]) {
    const uint32_t soff = (uint32_t)(r * BK * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = buf_ld4(arsrc, avoff + 16 * j, soff);
  };

  float4 ar0[4], ar1[4], ar2[4];
  u32x4 fr[2][2];
  f32x16 acc[kTN];
  auto compute = [&](const uint16_t* base) {
    constexpr int NB = 2 * kTN;
    auto rd = [&](int k, u32x4(&f)[2]) {
      const int s1 = k / kTN, b1 = k % kTN;
      const int row = 32 * b1 + li;
      f[0] = *reinterpret_cast<const u32x4*>(base + xoff(row, 2 * lh + s1));
      f[1] = *reinterpret_cast<const u32x4*>(base + kBN * XK + xoff(row, 2 * lh + s1));
    };
    u32x4 q[2][2];
    rd(0, q[0]);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int s = k / kTN, b = k % kTN;
      if (k + 1 < NB) rd(k + 1, q[(k + 1) & 1]);
      acc[b] = mfma_h3_t(__builtin_bit_cast(f16x8, fr[s][0]), __builtin_bit_cast(f16x8, fr[s][1]),
                         __builtin_bit_cast(f16x8, q[k & 1][0]), __builtin_bit_cast(f16x8, q[k & 1][1]),
                         acc[b]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
#pragma unroll
      for (int mm = 0; mm < 3; ++mm) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (k + 1 < NB && mm < 2) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
  };
  auto compute_half = [&]() {
    const uint16_t* base = img + NFULL * kFullImg;
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 2 * kTN; ++k) {
      const int s = k / kTN, b = k % kTN;
      const int row = 32 * b + li;
      const u32x4 h = *reinterpret_cast<const u32x4*>(base + hoff(row, s));
      const u32x4 l = *reinterpret_cast<const u32x4*>(base + kBN * 16 + hoff(row, s));
      acc[b] = mfma_h3_t(__builtin_bit_cast(f16x8, fr[s][0]), __builtin_bit_cast(f16x8, fr[s][1]),
                         __builtin_bit_cast(f16x8, lh ? z : h), __builtin_bit_cast(f16x8, lh ? z : l),
                         acc[b]);
    }
  };
  auto split = [&](float4(&a)[4], int r, int sha) {
    if (amax_out != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ain = fmaxf(ain, fmaxf(fmaxf(fabsf(a[j].x), fabsf(a[j].y)), fmaxf(fabsf(a[j].z), fabsf(a[j].w))));
    }
    if (r == S - 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((int64_t)r * BK + 16 * lh + 4 * j >= K) a[j] = f4zero();
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) hsplit8(a[2 * s], a[2 * s + 1], sha, fr[s][0], fr[s][1]);
  };

  int64_t slab = s_beg + w;
  if (slab < s_end) {
    meta_issue(slab);
    load_a(0, ar0);
    load_a(1, ar1);
  }
  vm_wait<0>();  // B image, the first slab's row maxima and two A steps
  __syncthreads();
  const int shb = h3_shift(bmax);
  int sha = slab < s_end ? row_shift() : 0;
  int64_t mw = slab * 32;

  for (; slab < s_end; slab += W) {
    const int64_t next = slab + W;
    const bool more = next < s_end;
#pragma unroll
    for (int b = 0; b < kTN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
    uint32_t mcur[kTN];
#pragma unroll
    for (int b = 0; b < kTN; ++b) mcur[b] = mws[b];
    // steps 0 .. S-3: A(r) waited for (steps 0 and 1: already landed), A(r+DEP) issued
    if constexpr (DEP == 2) {
#pragma unroll 1
      for (int r = 0; r < S - 2; r += 2) {
        if (r > 0) vm_wait<4>();
        split(ar0, r, sha);
        load_a(r + 2, ar0);
        compute(img + r * kFullImg);
        if (r > 0) vm_wait<4>();
        split(ar1, r + 1, sha);
        load_a(r + 3, ar1);
        compute(img + (r + 1) * kFullImg);
      }
    } else {
      // three sets: set r % 3 holds A(r); A(2) issued here, A(r + 3) after step r
      load_a(2, ar2);
#pragma unroll
      for (int r = 0; r < S - 2; ++r) {
        float4(&a)[4] = r % 3 == 0 ? ar0 : r % 3 == 1 ? ar1 : ar2;
        if (r >= 2) vm_wait<8>();
        split(a, r, sha);
        if (r + 3 < S) load_a(r + 3, a);
        compute(img + r * kFullImg);
      }
    }
    // steps S-2, S-1: the next slab's state and first two A steps go out
    const int sha_cur = sha;
    const int64_t mw_cur = mw;
    {
      float4(&a8)[4] = DEP == 2 ? ar0 : ((S - 2) % 3 == 0 ? ar0 : (S - 2) % 3 == 1 ? ar1 : ar2);
      float4(&a9)[4] = DEP == 2 ? ar1 : ((S - 1) % 3 == 0 ? ar0 : (S - 1) % 3 == 1 ? ar1 : ar2);
      vm_wait<4>();
      split(a8, S - 2, sha_cur);
      if (more) {
        meta_issue(next);
        load_a(0, ar0);
      }
      compute(img + (S - 2) * kFullImg);
      if (more) vm_wait<8>();  // A(S-1) landed; the next slab's loads may be in flight
      else vm_wait<0>();
      split(a9, S - 1, sha_cur);
      if (more) load_a(1, ar1);
      if (HALF) compute_half();
      else compute(img + (S - 1) * kFullImg);
    }
    // the next slab's loads landed before any store is issued
    vm_wait<0>();
    if (more) {
      sha = row_shift();
      mw = next * 32;
    }

    // ---- epilogue of this slab
    const int64_t m = mw_cur + li;
    const float sc = __builtin_ldexpf(1.f, -(sha_cur + shb));
    float rmax = 0.f;
#pragma unroll
    for (int b = 0; b < kTN; ++b) {
      const int64_t nb = n0 + 32 * b;
      if (nb >= N) break;
      uint32_t pos = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cb = 8 * q + 4 * lh;
        const int64_t n = nb + cb;
        if (m < M && n < N) {
          float* o = C + m * ldc + n;
          float4 v = make_float4(acc[b][4 * q] * sc, acc[b][4 * q + 1] * sc, acc[b][4 * q + 2] * sc,
                                 acc[b][4 * q + 3] * sc);
          if constexpr (HAS_BIAS) {
            v = f4add(v, *reinterpret_cast<const float4*>(bsh + 32 * b + cb));
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
            const uint32_t mk = (mcur[b] >> cb) & 15u;
            v = make_float4(mk & 1u ? v.x : 0.f, mk & 2u ? v.y : 0.f, mk & 4u ? v.z : 0.f,
                            mk & 8u ? v.w : 0.f);
          }
          if (accumulate) v = f4add(v, *reinterpret_cast<const float4*>(o));
          *reinterpret_cast<float4*>(o) = v;
          rmax = fmaxf(rmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          pos |= ((v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
                  (v.w > 0.f ? 8u : 0u)) << cb;
        }
      }
      if (bits_out != nullptr) {
        pos |= __shfl_xor(pos, 32, 64);
        if (lh == 0 && m < M) bits_out[(nb >> 5) * bits_ld + m] = pos;
      }
    }
    if (crow != nullptr) {
      const float v = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
      if (lh == 0 && m < M) crow[(int64_t)tile * M + m] = v;
    }
    cm = fmaxf(cm, rmax);
  }
  if (cmax != nullptr) absmax_publish(cm, cmax);
  if (amax_out != nullptr) absmax_publish(ain, amax_out);
}
}  // namespace

// epi: MOLCLR_EPI_*; h3: 1 per-tensor / 2 row-wise A scales; K in (288, 300]
// (S = 10 steps, half last step) -- the c2 lin1 / dz1 shapes
extern "C" int bs_exp(int epi, int h3, const float* A, const uint16_t* Bp, float* C, int64_t M,
                      int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
                      const float* bias, const float* aux, int64_t ldaux, const float* amax,
                      const float* bmax, float* cmax, float* crow, float* amax_out,
                      int arow_parts, uint32_t* bits_out, const uint32_t* bits_in, int64_t bits_ld,
                      int groups, int variant, hipStream_t s) {
  if (K <= 288 || K > 304 || kp != 320 || h3 != 2) return -3;
  const int ntn = (int)((N + kBN - 1) / kBN);
  const dim3 grid((unsigned)(ntn * groups));
#define BS_L(E, WV, DP)                                                                          \
  hipLaunchKernelGGL((k_gemm_bs<E, 2, 10, true, WV, DP>), grid, dim3(64 * WV), 0, s, A, Bp, C, M, \
                     N, K, lda, kp, npad, ldc, bias, aux, ldaux, 0, amax, bmax, cmax, crow,      \
                     amax_out, arow_parts, bits_out, bits_in, bits_ld, ntn, groups)
#define BS_LA(E, AB)                                                                          \
  hipLaunchKernelGGL((k_gemm_bs<E, 2, 10, true, 8, 2, AB>), grid, dim3(512), 0, s, A, Bp, C, M, N, \
                     K, lda, kp, npad, ldc, bias, aux, ldaux, 0, amax, bmax, cmax, crow, amax_out, \
                     arow_parts, bits_out, bits_in, bits_ld, ntn, groups)
#define BS_L2(E, DP)                                                                              \
  hipLaunchKernelGGL((k_gemm_bs2<E, 2, 10, true, 8, DP>), grid, dim3(512), 0, s, A, Bp, C, M, N, K,   \
                     lda, kp, npad, ldc, bias, aux, ldaux, 0, amax, bmax, cmax, crow, amax_out,  \
                     arow_parts, bits_out, bits_in, bits_ld, ntn, groups)
#define BS_V(E)                          \
  switch (variant) {                     \
    case 0: BS_L(E, 8, 2); break;        \
    case 1: BS_L(E, 8, 3); break;        \
    case 11: BS_LA(E, 1); break;         \
    case 12: BS_LA(E, 2); break;         \
    case 13: BS_LA(E, 3); break;         \
    case 14: BS_LA(E, 4); break;         \
    case 16: BS_LA(E, 6); break;         \
    case 20: BS_L2(E, 2); break;         \
    case 21: BS_L2(E, 3); break;         \
    default: return -4;                  \
  }
  switch (epi) {
    case MOLCLR_EPI_BIAS_RELU: BS_V(MOLCLR_EPI_BIAS_RELU); break;
    case MOLCLR_EPI_RELU_MASK: BS_V(MOLCLR_EPI_RELU_MASK); break;
    default: return -1;
  }
#undef BS_V
#undef BS_LA
#undef BS_L2
#undef BS_L
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
