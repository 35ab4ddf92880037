// q6 main-loop experiments (tools/q6x.py): the product's k_gemm_q6 (one K
// group) with compile-time variants V, timed and compared bit for bit against
// the product kernel on the c2 step's shapes.  Not part of the product build.
//   V & 1: buffer-resource addressing -- A loads (raw_buffer_load) and the B
//          LDS-DMA (raw_ptr_buffer_load_lds) from per-lane 32-bit offsets
//          fixed for the whole tile plus a scalar K offset per step: no 64-bit
//          address arithmetic and no clamps in the loop (loads past the
//          matrix return zeros)
//   V & 2: the A tail mask only in the last round (the others run unmasked)
//   V & 4: B fragments of the next column block read under the current
//          block's MFMAs (register double buffer)
#include "../../molclr_amd/csrc/mfma.h"

#include <type_traits>

namespace {
using namespace molclr;

constexpr int kW = 4;          // waves
constexpr int kBM = 32 * kW;   // rows per block
constexpr unsigned kRsrc3 = 0x00020000u;


template <int TN, int EPI, bool MASK, int H3, int V>
__global__ __launch_bounds__(64 * kW) __attribute__((amdgpu_waves_per_eu(2))) void k_q6x(
    const float* __restrict__ A, const uint16_t* __restrict__ Bp, float* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux,
    const float* __restrict__ amax, const float* __restrict__ bmax, float* __restrict__ cmax,
    float* __restrict__ crow, float* __restrict__ amax_out, int arow_parts,
    uint32_t* __restrict__ bits_out, const uint32_t* __restrict__ bits_in, int64_t bits_ld) {
  constexpr bool BUF = (V & 1) != 0, TAILMASK = (V & 2) != 0, RDA = (V & 4) != 0;
  constexpr int BN = 32 * TN;
  constexpr int NP = H3 ? 2 : 3;
  constexpr int BI = NP * BN * XK;
  constexpr int EPI_ELEMS = kW * 32 * 32 * 2;
  constexpr int L0 = BI > EPI_ELEMS ? BI : EPI_ELEMS;
  __shared__ __attribute__((aligned(16))) uint16_t lds[L0];
  __shared__ __attribute__((aligned(16))) uint16_t lds_b1[BI];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wm = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;

  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + kBM - 1) / kBM);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int64_t m0 = (int64_t)(tile / ntn) * kBM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;

  constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;
  constexpr int BVN = HAS_BIAS ? TN : 1, MWN = EPI == MOLCLR_EPI_RELU_MASK ? TN : 1;
  float4 bvq[BVN];
  uint32_t mwq[MWN][4];
  {
    const int c4l = lane & 7;
    if constexpr (HAS_BIAS) {
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int64_t n = n0 + 32 * b + 4 * c4l;
        bvq[b] = (n + 4 <= N && (reinterpret_cast<uintptr_t>(bias) & 15) == 0)
                     ? *reinterpret_cast<const float4*>(bias + n) : f4zero();
      }
    }
    if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
      if (bits_in != nullptr) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            int64_t m = m0 + 32 * wm + 8 * it + (lane >> 3);
            m = m < M ? m : M - 1;
            int64_t nb = n0 + 32 * b;
            nb = nb < N ? nb : 0;
            mwq[b][it] = bits_in[(nb >> 5) * bits_ld + m];
          }
      }
    }
  }

  int64_t arow_i = m0 + 32 * wm + li;
  arow_i = arow_i < M ? arow_i : M - 1;
  const float* __restrict__ arow = A + arow_i * lda;
  const int nsteps = (int)(kp / BK);
  const int rounds = nsteps;
  // buffer addressing: per-lane byte offsets fixed for the tile
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(A, (M * lda) * 4);
  const __amdgpu_buffer_rsrc_t brsrc = make_rsrc(Bp, (int64_t)NP * npad * kp * 2);
  const uint32_t avoff = (uint32_t)((arow_i * lda + 16 * lh) * 4);
  auto load_a = [&](int r, float4(&v)[4]) {
    r = r < rounds ? r : rounds - 1;
    const int64_t k = (int64_t)r * BK + 16 * lh;
    if constexpr (BUF) {
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(r * BK * 4));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = buf_ld4(arsrc, avoff + 16 * j, soff);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int64_t kj = k + 4 * j;
        if constexpr (MASK) kj = kj < K - 4 ? kj : K - 4;
        v[j] = *reinterpret_cast<const float4*>(arow + kj);
      }
    }
  };
  // B DMA: per-lane offsets of this wave's chunks (fixed for the tile)
  constexpr int RPB = BN / 16, CH = NP * RPB, PERW = (CH + kW - 1) / kW;
  uint32_t bvoff[PERW];
#pragma unroll
  for (int qq = 0; qq < PERW; ++qq) {
    const int q = wm + kW * qq;
    const int qc = q < CH ? q : CH - 1;
    const int pl = qc / RPB, row = (qc % RPB) * 16 + (lane >> 2), c = lane & 3;
    int64_t gr = n0 + row;
    gr = gr < npad ? gr : npad - 1;
    bvoff[qq] = (uint32_t)(((pl * npad + gr) * kp + 8 * (c ^ ((row >> 2) & 3))) * 2);
  }
  auto dma_b = [&](int r, uint16_t* img) {
    r = r < nsteps ? r : nsteps - 1;
    const int64_t k0 = (int64_t)r * BK;
    if constexpr (BUF) {
#pragma unroll
      for (int qq = 0; qq < PERW; ++qq) {
        const int q = wm + kW * qq;
        if (CH % kW && q >= CH) break;
        buf_lds16(brsrc, img + ((q / RPB) * BN + (q % RPB) * 16) * XK, bvoff[qq],
                  __builtin_amdgcn_readfirstlane((uint32_t)(k0 * 2)));
      }
    } else {
#pragma unroll
      for (int qq = 0; qq < PERW; ++qq) {
        const int q = wm + kW * qq;
        if (CH % kW && q >= CH) break;
        const int pl = q / RPB, row = (q % RPB) * 16 + (lane >> 2), c = lane & 3;
        int64_t gr = n0 + row;
        gr = gr < npad ? gr : npad - 1;
        __builtin_amdgcn_global_load_lds(
            (gbl_as_ptr)(Bp + (pl * npad + gr) * kp + k0 + 8 * (c ^ ((row >> 2) & 3))),
            (lds_as_ptr)(img + (pl * BN + (q % RPB) * 16) * XK), 16, 0, 0);
      }
    }
  };

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  int sha = 0;
  if constexpr (H3 == 1) sha = h3_shift(amax);
  if constexpr (H3 == 2) {
    float m = 0.f;
    for (int p = 0; p < arow_parts; ++p) m = fmaxf(m, amax[(int64_t)p * M + arow_i]);
    sha = h3_shift_of(m);
  }
  const int shb = H3 ? h3_shift(bmax) : 0;
  float ain = 0.f;
  auto compute = [&](const uint16_t* Bs, const float4(&a)[4], int r, bool masked) {
    if (amax_out != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ain = fmaxf(ain, fmaxf(fmaxf(fabsf(a[j].x), fabsf(a[j].y)), fmaxf(fabsf(a[j].z), fabsf(a[j].w))));
    }
    float4 am4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      am4[j] = a[j];
      if (MASK && masked) {
        const int64_t kj = (int64_t)r * BK + 16 * lh + 4 * j;
        if (kj >= K) am4[j] = f4zero();
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 2 * lh + s;
      if constexpr (H3) {
        u32x4 h, l;
        hsplit8(am4[2 * s], am4[2 * s + 1], sha, h, l);
        const f16x8 ah = __builtin_bit_cast(f16x8, h);
        const f16x8 al = __builtin_bit_cast(f16x8, l);
        if constexpr (RDA) {
          u32x4 f0 = *reinterpret_cast<const u32x4*>(Bs + xoff(li, ch));
          u32x4 f1 = *reinterpret_cast<const u32x4*>(Bs + BN * XK + xoff(li, ch));
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            u32x4 g0 = f0, g1 = f1;
            if (b + 1 < TN) {
              f0 = *reinterpret_cast<const u32x4*>(Bs + xoff(32 * (b + 1) + li, ch));
              f1 = *reinterpret_cast<const u32x4*>(Bs + BN * XK + xoff(32 * (b + 1) + li, ch));
            }
            acc[b] = mfma_h3(ah, al, __builtin_bit_cast(f16x8, g0), __builtin_bit_cast(f16x8, g1),
                             acc[b]);
          }
        } else {
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const int row = 32 * b + li;
            const f16x8 bh = __builtin_bit_cast(f16x8, xfrag(Bs, row, ch));
            const f16x8 bl = __builtin_bit_cast(f16x8, xfrag(Bs + BN * XK, row, ch));
            acc[b] = mfma_h3(ah, al, bh, bl, acc[b]);
          }
        }
        continue;
      }
      u32x4 h, m, l;
      split8(am4[2 * s], am4[2 * s + 1], h, m, l);
      const bf16x8 ah = __builtin_bit_cast(bf16x8, h);
      const bf16x8 amm = __builtin_bit_cast(bf16x8, m);
      const bf16x8 al = __builtin_bit_cast(bf16x8, l);
      auto six = [&](int b, bf16x8 bh, bf16x8 bm, bf16x8 bl) {
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(amm, bm, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(amm, bh, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[b], 0, 0, 0);
      };
      if constexpr (RDA) {
        bf16x8 f0 = xfrag(Bs, li, ch), f1 = xfrag(Bs + BN * XK, li, ch),
               f2 = xfrag(Bs + 2 * BN * XK, li, ch);
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const bf16x8 g0 = f0, g1 = f1, g2 = f2;
          if (b + 1 < TN) {
            const int row = 32 * (b + 1) + li;
            f0 = xfrag(Bs, row, ch);
            f1 = xfrag(Bs + BN * XK, row, ch);
            f2 = xfrag(Bs + 2 * BN * XK, row, ch);
          }
          six(b, g0, g1, g2);
        }
      } else {
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int row = 32 * b + li;
          six(b, xfrag(Bs, row, ch), xfrag(Bs + BN * XK, row, ch), xfrag(Bs + 2 * BN * XK, row, ch));
        }
      }
    }
  };

  uint16_t* buf0 = lds;
  uint16_t* buf1 = lds_b1;
  float4 a0[4], a1[4];
  dma_b(0, buf0);
  load_a(0, a0);
  __syncthreads();
  // unmasked rounds: all but the last when TAILMASK (and MASK) is set
  const int full = (TAILMASK && MASK) ? rounds - 1 : rounds;
  const bool mask_all = MASK && !TAILMASK;
  int i = 0;
  for (; i + 2 <= full; i += 2) {
    dma_b(i + 1, buf1);
    load_a(i + 1, a1);
    compute(buf0, a0, i, mask_all);
    __syncthreads();
    dma_b(i + 2, buf0);
    load_a(i + 2, a0);
    compute(buf1, a1, i + 1, mask_all);
    __syncthreads();
  }
  // at most two rounds left: [full odd: round i unmasked], [the masked last]
  if (i < full) {  // one unmasked round in buf0, and (TAILMASK) the last round next
    if (i + 1 < rounds) {
      dma_b(i + 1, buf1);
      load_a(i + 1, a1);
    }
    compute(buf0, a0, i, mask_all);
    __syncthreads();
    if (i + 1 < rounds) compute(buf1, a1, i + 1, true);
  } else if (i < rounds) {
    compute(buf0, a0, i, true);
  }
  __syncthreads();

  const bool vec = ((ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                   (EPI != MOLCLR_EPI_RELU_MASK || bits_in != nullptr ||
                    (((ldaux & 3) == 0) && (reinterpret_cast<uintptr_t>(aux) & 15) == 0)) &&
                   ((EPI != MOLCLR_EPI_BIAS && EPI != MOLCLR_EPI_BIAS_RELU) ||
                    (reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  float* tw = reinterpret_cast<float*>(lds) + wm * 32 * 32;
  const int64_t mw = m0 + 32 * wm;
  float rm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int sr = H3 == 2 ? __shfl(sha, row, 64) : sha;
      tw[row * 32 + li] = H3 ? __builtin_ldexpf(acc[b][r], -(sr + shb)) : acc[b][r];
    }
    wave_lds_sync();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, c4 = idx & 7;
      const int64_t m = mw + row, n = nb + 4 * c4;
      uint32_t pos = 0;
      if (m < M && n < N) {
        const float4 v4 = *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
        float* o = C + m * ldc + n;
        uint32_t mk = 15u;
        if constexpr (EPI == MOLCLR_EPI_RELU_MASK)
          if (bits_in != nullptr) mk = (mwq[b][it] >> (4 * c4)) & 15u;
        if (vec && n + 4 <= N) {
          float4 v = v4;
          if constexpr (HAS_BIAS) {
            v = f4add(v, bvq[b]);
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if (EPI == MOLCLR_EPI_RELU_MASK) {
            if (bits_in != nullptr) {
              v = make_float4(mk & 1u ? v.x : 0.f, mk & 2u ? v.y : 0.f, mk & 4u ? v.z : 0.f,
                              mk & 8u ? v.w : 0.f);
            } else {
              const float4 x = *reinterpret_cast<const float4*>(aux + m * ldaux + n);
              v = make_float4(x.x > 0.f ? v.x : 0.f, x.y > 0.f ? v.y : 0.f,
                              x.z > 0.f ? v.z : 0.f, x.w > 0.f ? v.w : 0.f);
            }
          }
          *reinterpret_cast<float4*>(o) = v;
          rm[it] = fmaxf(rm[it], fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          pos = (v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
                (v.w > 0.f ? 8u : 0u);
        } else {
          const float e[4] = {v4.x, v4.y, v4.z, v4.w};
          for (int j = 0; j < 4 && n + j < N; ++j) {
            float x = e[j];
            if (EPI == MOLCLR_EPI_BIAS) x = x + bias[n + j];
            if (EPI == MOLCLR_EPI_BIAS_RELU) x = fmaxf(x + bias[n + j], 0.f);
            if (EPI == MOLCLR_EPI_RELU_MASK)
              x = (bits_in != nullptr ? ((mk >> j) & 1u) != 0u : aux[m * ldaux + n + j] > 0.f)
                      ? x : 0.f;
            o[j] = x;
            rm[it] = fmaxf(rm[it], fabsf(x));
            pos |= (x > 0.f ? 1u : 0u) << j;
          }
        }
      }
      if (bits_out != nullptr) {
        const uint64_t bj[4] = {__ballot((pos & 1u) != 0u), __ballot((pos & 2u) != 0u),
                                __ballot((pos & 4u) != 0u), __ballot((pos & 8u) != 0u)};
        if (c4 == 0 && m < M) {
          uint32_t w = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t x = (uint32_t)(bj[j] >> (8 * (lane >> 3))) & 0xFFu;
            x = (x | (x << 12)) & 0x000F000Fu;
            x = (x | (x << 6)) & 0x03030303u;
            x = (x | (x << 3)) & 0x11111111u;
            w |= x << j;
          }
          bits_out[(nb >> 5) * bits_ld + m] = w;
        }
      }
    }
    wave_lds_sync();
  }
  if (crow != nullptr) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      float v = rm[it];
      v = fmaxf(v, __shfl_xor(v, 1, 64));
      v = fmaxf(v, __shfl_xor(v, 2, 64));
      v = fmaxf(v, __shfl_xor(v, 4, 64));
      const int64_t m = mw + 8 * it + (lane >> 3);
      if ((lane & 7) == 0 && m < M) crow[(n0 / BN) * M + m] = v;
    }
  }
  if (cmax != nullptr) absmax_publish(fmaxf(fmaxf(rm[0], rm[1]), fmaxf(rm[2], rm[3])), cmax);
  if (amax_out != nullptr) absmax_publish(ain, amax_out);
}

// ---------------------------------------------------------------------------
// "pp": ping-pong.  8 waves per block in two groups of 4 (waves 0-3 rows
// m0 .. m0+127, waves 4-7 rows m0+128 .. m0+255; every SIMD holds one wave of
// each group), sharing one B image per K step.  Group 1 runs one phase behind
// group 0, so between two block barriers one group issues its step's MFMAs
// (B fragments read from LDS under them) while the other splits its next A
// step into bf16 / fp16 fragments, issues the following A loads and (group 1)
// the LDS-DMA of the B image two steps ahead:
//   phase 2i+1: group 0 computes step i      | group 1 splits step i (+ loads)
//   phase 2i+2: group 0 splits step i+1      | group 1 computes step i
// The MFMA and VALU pipes of a SIMD run the two waves' phases side by side.
// ---------------------------------------------------------------------------
// ABL (ablations, results then differ): 32 = timeline stamps (s_memtime at
// every phase boundary, lane 0 of every wave, into bits_out as uint64
// [block][wave][64]; results unchanged), 1 A rows folded into 64 (L2-hot),
// 2 no B DMA after the first two steps, 4 no MFMA, 8 no split (raw bits as
// fragments), 16 no epilogue stores
template <int TN, int EPI, int H3, int ABL = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_q6pp(
    const float* __restrict__ A, const uint16_t* __restrict__ Bp, float* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux,
    const float* __restrict__ amax, const float* __restrict__ bmax, float* __restrict__ cmax,
    float* __restrict__ crow, float* __restrict__ amax_out, int arow_parts,
    uint32_t* bits_out, const uint32_t* __restrict__ bits_in, int64_t bits_ld) {
  constexpr int BN = 32 * TN;
  constexpr int NP = H3 ? 2 : 3;
  constexpr int BI = NP * BN * XK;
  constexpr int BMR = 256;  // rows per block
  __shared__ __attribute__((aligned(16))) uint16_t bimg0[BI];
  __shared__ __attribute__((aligned(16))) uint16_t bimg1[BI];
  __shared__ __attribute__((aligned(16))) float ep[8 * 32 * 32];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, wm = w & 3;
  const int li = lane & 31, lh = lane >> 5;
  int nst = 0;
  uint32_t* const stamps = bits_out;
  if constexpr ((ABL & 32) != 0) bits_out = nullptr;  // the buffer holds the stamps
  auto stamp = [&]() {
    if constexpr ((ABL & 32) != 0) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      if (lane == 0 && nst < 64)
        reinterpret_cast<uint64_t*>(stamps)[((int64_t)blockIdx.x * 8 + w) * 64 + nst] = t;
      ++nst;
    }
  };

  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BMR - 1) / BMR);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int64_t m0 = (int64_t)(tile / ntn) * BMR;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;
  const int64_t mw = m0 + 128 * grp + 32 * wm;  // this wave's first row

  constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;
  constexpr int BVN = HAS_BIAS ? TN : 1, MWN = EPI == MOLCLR_EPI_RELU_MASK ? TN : 1;
  float4 bvq[BVN];
  uint32_t mwq[MWN][4];
  {
    const int c4l = lane & 7;
    if constexpr (HAS_BIAS) {
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int64_t n = n0 + 32 * b + 4 * c4l;
        bvq[b] = (n + 4 <= N && (reinterpret_cast<uintptr_t>(bias) & 15) == 0)
                     ? *reinterpret_cast<const float4*>(bias + n) : f4zero();
      }
    }
    if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
      if (bits_in != nullptr) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            int64_t m = mw + 8 * it + (lane >> 3);
            m = m < M ? m : M - 1;
            int64_t nb = n0 + 32 * b;
            nb = nb < N ? nb : 0;
            mwq[b][it] = bits_in[(nb >> 5) * bits_ld + m];
          }
      }
    }
  }

  int64_t arow_i = mw + li;
  arow_i = arow_i < M ? arow_i : M - 1;
  const int S = (int)(kp / BK);
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(A, (M * lda) * 4);
  const __amdgpu_buffer_rsrc_t brsrc = make_rsrc(Bp, (int64_t)NP * npad * kp * 2);
  const uint32_t avoff = (uint32_t)((((ABL & 1) ? (arow_i & 63) : arow_i) * lda + 16 * lh) * 4);
  auto load_a = [&](int r, float4(&v)[4]) {
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(r * BK * 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = buf_ld4(arsrc, avoff + 16 * j, soff);
  };
  // B image of a step: CH chunks of 1 KB, issued by group 1's four waves
  constexpr int RPB = BN / 16, CH = NP * RPB, PERW = (CH + 3) / 4;
  uint32_t bvoff[PERW];
#pragma unroll
  for (int qq = 0; qq < PERW; ++qq) {
    const int q = wm + 4 * qq;
    const int qc = q < CH ? q : CH - 1;
    const int pl = qc / RPB, row = (qc % RPB) * 16 + (lane >> 2), c = lane & 3;
    int64_t gr = n0 + row;
    gr = gr < npad ? gr : npad - 1;
    bvoff[qq] = (uint32_t)(((pl * npad + gr) * kp + 8 * (c ^ ((row >> 2) & 3))) * 2);
  }
  auto dma_b = [&](int r, uint16_t* img) {
    if ((ABL & 2) && r >= 2) return;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(r * BK * 2));
#pragma unroll
    for (int qq = 0; qq < PERW; ++qq) {
      const int q = wm + 4 * qq;
      if (CH % 4 && q >= CH) break;
      buf_lds16(brsrc, img + ((q / RPB) * BN + (q % RPB) * 16) * XK, bvoff[qq], soff);
    }
  };

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  int sha = 0;
  if constexpr (H3 == 1) sha = h3_shift(amax);
  if constexpr (H3 == 2) {
    float m = 0.f;
    for (int p = 0; p < arow_parts; ++p) m = fmaxf(m, amax[(int64_t)p * M + arow_i]);
    sha = h3_shift_of(m);
  }
  const int shb = H3 ? h3_shift(bmax) : 0;
  float ain = 0.f;

  // this step's A fragments: [s][plane]
  u32x4 fr[2][NP];
  auto split = [&](float4(&a)[4], int r) {
    if (amax_out != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ain = fmaxf(ain, fmaxf(fmaxf(fabsf(a[j].x), fabsf(a[j].y)), fmaxf(fabsf(a[j].z), fabsf(a[j].w))));
    }
    if (r == S - 1) {  // the last step may run past K: zero those k (uniform branch)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((int64_t)r * BK + 16 * lh + 4 * j >= K) a[j] = f4zero();
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr ((ABL & 8) != 0) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
          fr[s][p] = __builtin_bit_cast(u32x4, (p & 1) ? a[2 * s + 1] : a[2 * s]);
      } else if constexpr (H3) {
        hsplit8(a[2 * s], a[2 * s + 1], sha, fr[s][0], fr[s][1]);
      } else {
        split8(a[2 * s], a[2 * s + 1], fr[s][0], fr[s][1], fr[s][2]);
      }
    }
  };
  // The compute phase: 2 TN blocks of MFMAs (block k: sub-step s = k / TN,
  // column block b = k % TN), the B fragments of block k + 1 read from LDS
  // under block k's MFMAs; sched_group_barrier pins that interleave (left
  // alone, the compiler moves each read down to its use and waits on it).
  auto compute = [&](const uint16_t* Bs) {
    constexpr int NB = 2 * TN;
    constexpr int AH = (ABL & 128) ? 2 : 1;  // blocks read ahead
    auto rd = [&](int k, u32x4(&f)[NP]) {
      const int s1 = k / TN, b1 = k % TN;
#pragma unroll
      for (int p = 0; p < NP; ++p)
        f[p] = *reinterpret_cast<const u32x4*>(Bs + p * BN * XK + xoff(32 * b1 + li, 2 * lh + s1));
    };
    u32x4 q[AH + 1][NP];  // ring of fragment sets
#pragma unroll
    for (int k = 0; k < AH; ++k) rd(k, q[k]);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int s = k / TN, b = k % TN;
      if (k + AH < NB) rd(k + AH, q[(k + AH) % (AH + 1)]);
      const u32x4* cb = q[k % (AH + 1)];
      if constexpr ((ABL & 4) != 0) {
        acc[b][0] += __builtin_bit_cast(float, cb[0][0] ^ fr[s][0][0]);
      } else if constexpr (H3) {
        acc[b] = mfma_h3(__builtin_bit_cast(f16x8, fr[s][0]), __builtin_bit_cast(f16x8, fr[s][1]),
                         __builtin_bit_cast(f16x8, cb[0]), __builtin_bit_cast(f16x8, cb[1]), acc[b]);
      } else {
        const bf16x8 ah = __builtin_bit_cast(bf16x8, fr[s][0]);
        const bf16x8 am = __builtin_bit_cast(bf16x8, fr[s][1]);
        const bf16x8 al = __builtin_bit_cast(bf16x8, fr[s][2]);
        const bf16x8 bh = __builtin_bit_cast(bf16x8, cb[0]);
        const bf16x8 bm = __builtin_bit_cast(bf16x8, cb[1]);
        const bf16x8 bl = __builtin_bit_cast(bf16x8, cb[2]);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[b], 0, 0, 0);
      }
    }
    if constexpr ((ABL & 64) == 0 && (ABL & 4) == 0) {
      constexpr int NM = H3 ? 3 : 6;  // MFMAs per block
      __builtin_amdgcn_sched_group_barrier(0x100, AH * NP, 0);  // the first blocks' reads
#pragma unroll
      for (int k = 0; k < NB; ++k) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (k + AH < NB && m < NP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    }
  };

  // prologue: B(0), A(0) landed; A(1) in flight.  A runs two steps ahead
  // (two register sets), B one step (two LDS images); the loop is unrolled
  // by two so every register set and image is chosen at compile time.
  float4 ar0[4], ar1[4];
  if (grp == 1) dma_b(0, bimg0);
  load_a(0, ar0);
  if (S > 1) {
    load_a(1, ar1);
    vm_wait<4>();
  } else {
    vm_wait<0>();
  }
  __syncthreads();
  split(ar0, 0);
  if (S > 1 && grp == 1) dma_b(1, bimg1);
  if (S > 2) load_a(2, ar0);
  stamp();
  if (grp == 1) __syncthreads();  // group 1 runs one phase behind
  if (grp == 1) stamp();
  if constexpr ((ABL & 256) != 0) {
    if (grp == 1) __builtin_amdgcn_s_setprio(1);  // the younger half: static priority
  }
  // step i (parity P): compute from image P, then the load phase of step
  // i+1: its A is in set 1-P (issued two load phases ago), B(i+1) in image
  // 1-P (issued one load phase ago, before A(i+2): vmcnt(4) covers it)
  auto body = [&](auto P, int i) -> bool {
    constexpr int par = decltype(P)::value;
    compute(par ? bimg1 : bimg0);
    stamp();  // compute issued
    if (i + 1 >= S) return false;
    if (i + 2 < S) vm_wait<4>();
    else vm_wait<0>();
    stamp();  // loads waited
    __syncthreads();
    stamp();  // barrier passed
    float4(&an)[4] = par ? ar0 : ar1;  // step i+1's A
    split(an, i + 1);
    if (i + 2 < S && grp == 1) dma_b(i + 2, par ? bimg1 : bimg0);
    if (i + 3 < S) load_a(i + 3, an);
    stamp();  // load phase issued
    __syncthreads();
    stamp();  // barrier passed
    return true;
  };
  for (int i = 0;; i += 2) {
    if (!body(std::integral_constant<int, 0>{}, i)) break;
    if (!body(std::integral_constant<int, 1>{}, i + 1)) break;
  }
  if (grp == 0) __syncthreads();
  stamp();  // epilogue start
  if constexpr ((ABL & 512) != 0) {
    // direct epilogue: register r of block b holds row acc_row(r, lh) (the
    // 32 lanes of a half share it) and column nb + li; no LDS round trip
    int srow[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) srow[r] = H3 == 2 ? __shfl(sha, acc_row(r, lh), 64) + shb : sha + shb;
    float rmx[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) rmx[r] = 0.f;
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int64_t nb = n0 + 32 * b;
      if (nb >= N) break;  // block-uniform
      const int64_t n = nb + li;
      const bool nok = n < N;
      float bv = 0.f;
      if constexpr (HAS_BIAS) bv = nok ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = mw + acc_row(r, lh);
        const bool ok = nok && m < M;
        float v = acc[b][r];
        if constexpr (H3) v = __builtin_ldexpf(v, -srow[r]);
        if constexpr (HAS_BIAS) {
          v = v + bv;
          if (EPI == MOLCLR_EPI_BIAS_RELU) v = fmaxf(v, 0.f);
        }
        if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
          const int64_t mc = m < M ? m : M - 1;
          bool keep;
          if (bits_in != nullptr) keep = ((bits_in[(nb >> 5) * bits_ld + mc] >> li) & 1u) != 0u;
          else keep = ok && aux[mc * ldaux + n] > 0.f;
          v = keep ? v : 0.f;
        }
        float* o = C + m * ldc + n;
        if (ok) {
          // accumulate (the product's EPI_ACCUMULATE) is not taken by these shapes
          if (!(ABL & 16) || v == 1.2345f) *o = v;
          rmx[r] = fmaxf(rmx[r], fabsf(v));
        }
        if (bits_out != nullptr) {
          const uint64_t bal = __ballot(ok && v > 0.f);
          if (li == 0 && m < M) bits_out[(nb >> 5) * bits_ld + m] = (uint32_t)(bal >> (32 * lh));
        }
      }
    }
    float cm = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = rmx[r];
      v = fmaxf(v, __shfl_xor(v, 1, 64));
      v = fmaxf(v, __shfl_xor(v, 2, 64));
      v = fmaxf(v, __shfl_xor(v, 4, 64));
      v = fmaxf(v, __shfl_xor(v, 8, 64));
      v = fmaxf(v, __shfl_xor(v, 16, 64));
      cm = fmaxf(cm, v);
      const int64_t m = mw + acc_row(r, lh);
      if (crow != nullptr && li == 0 && m < M) crow[(n0 / BN) * M + m] = v;
    }
    if (cmax != nullptr) absmax_publish(cm, cmax);
    if (amax_out != nullptr) absmax_publish(ain, amax_out);
    stamp();  // end
    return;
  }
  const bool vec = ((ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                   (EPI != MOLCLR_EPI_RELU_MASK || bits_in != nullptr ||
                    (((ldaux & 3) == 0) && (reinterpret_cast<uintptr_t>(aux) & 15) == 0)) &&
                   ((EPI != MOLCLR_EPI_BIAS && EPI != MOLCLR_EPI_BIAS_RELU) ||
                    (reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  float* tw = ep + w * 32 * 32;
  float rm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int sr = H3 == 2 ? __shfl(sha, row, 64) : sha;
      tw[row * 32 + li] = H3 ? __builtin_ldexpf(acc[b][r], -(sr + shb)) : acc[b][r];
    }
    wave_lds_sync();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, c4 = idx & 7;
      const int64_t m = mw + row, n = nb + 4 * c4;
      uint32_t pos = 0;
      if (m < M && n < N) {
        const float4 v4 = *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
        float* o = C + m * ldc + n;
        uint32_t mk = 15u;
        if constexpr (EPI == MOLCLR_EPI_RELU_MASK)
          if (bits_in != nullptr) mk = (mwq[b][it] >> (4 * c4)) & 15u;
        if (vec && n + 4 <= N) {
          float4 v = v4;
          if constexpr (HAS_BIAS) {
            v = f4add(v, bvq[b]);
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if (EPI == MOLCLR_EPI_RELU_MASK) {
            if (bits_in != nullptr) {
              v = make_float4(mk & 1u ? v.x : 0.f, mk & 2u ? v.y : 0.f, mk & 4u ? v.z : 0.f,
                              mk & 8u ? v.w : 0.f);
            } else {
              const float4 x = *reinterpret_cast<const float4*>(aux + m * ldaux + n);
              v = make_float4(x.x > 0.f ? v.x : 0.f, x.y > 0.f ? v.y : 0.f,
                              x.z > 0.f ? v.z : 0.f, x.w > 0.f ? v.w : 0.f);
            }
          }
          if (!(ABL & 16) || v.x == 1.2345f) *reinterpret_cast<float4*>(o) = v;
          rm[it] = fmaxf(rm[it], fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          pos = (v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
                (v.w > 0.f ? 8u : 0u);
        } else {
          const float e[4] = {v4.x, v4.y, v4.z, v4.w};
          for (int j = 0; j < 4 && n + j < N; ++j) {
            float x = e[j];
            if (EPI == MOLCLR_EPI_BIAS) x = x + bias[n + j];
            if (EPI == MOLCLR_EPI_BIAS_RELU) x = fmaxf(x + bias[n + j], 0.f);
            if (EPI == MOLCLR_EPI_RELU_MASK)
              x = (bits_in != nullptr ? ((mk >> j) & 1u) != 0u : aux[m * ldaux + n + j] > 0.f)
                      ? x : 0.f;
            o[j] = x;
            rm[it] = fmaxf(rm[it], fabsf(x));
            pos |= (x > 0.f ? 1u : 0u) << j;
          }
        }
      }
      if (bits_out != nullptr) {
        const uint64_t bj[4] = {__ballot((pos & 1u) != 0u), __ballot((pos & 2u) != 0u),
                                __ballot((pos & 4u) != 0u), __ballot((pos & 8u) != 0u)};
        if (c4 == 0 && m < M) {
          uint32_t wd = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t x = (uint32_t)(bj[j] >> (8 * (lane >> 3))) & 0xFFu;
            x = (x | (x << 12)) & 0x000F000Fu;
            x = (x | (x << 6)) & 0x03030303u;
            x = (x | (x << 3)) & 0x11111111u;
            wd |= x << j;
          }
          bits_out[(nb >> 5) * bits_ld + m] = wd;
        }
      }
    }
    wave_lds_sync();
  }
  if (crow != nullptr) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      float v = rm[it];
      v = fmaxf(v, __shfl_xor(v, 1, 64));
      v = fmaxf(v, __shfl_xor(v, 2, 64));
      v = fmaxf(v, __shfl_xor(v, 4, 64));
      const int64_t m = mw + 8 * it + (lane >> 3);
      if ((lane & 7) == 0 && m < M) crow[(n0 / BN) * M + m] = v;
    }
  }
  if (cmax != nullptr) absmax_publish(fmaxf(fmaxf(rm[0], rm[1]), fmaxf(rm[2], rm[3])), cmax);
  if (amax_out != nullptr) absmax_publish(ain, amax_out);
  stamp();  // end
}

template <int EPI, int H3, int ABL = 0>
void launch_pp(const float* A, const uint16_t* Bp, float* C, int64_t M, int64_t N, int64_t K,
               int64_t lda, int64_t kp, int64_t npad, int64_t ldc, const float* bias,
               const float* aux, int64_t ldaux, const float* amax, const float* bmax, float* cmax,
               float* crow, float* amax_out, int arow_parts, uint32_t* bits_out,
               const uint32_t* bits_in, int64_t bits_ld, hipStream_t s) {
  constexpr int TN = 5;
  const int64_t blocks = ((M + 255) / 256) * ((N + 32 * TN - 1) / (32 * TN));
  hipLaunchKernelGGL((k_q6pp<TN, EPI, H3, ABL>), dim3((unsigned)blocks), dim3(512), 0, s, A, Bp, C, M,
                     N, K, lda, kp, npad, ldc, bias, aux, ldaux, amax, bmax, cmax, crow, amax_out,
                     arow_parts, bits_out, bits_in, bits_ld);
}

template <int EPI, int H3, int V>
void launch(const float* A, const uint16_t* Bp, float* C, int64_t M, int64_t N, int64_t K,
            int64_t lda, int64_t kp, int64_t npad, int64_t ldc, const float* bias, const float* aux,
            int64_t ldaux, const float* amax, const float* bmax, float* cmax, float* crow,
            float* amax_out, int arow_parts, uint32_t* bits_out, const uint32_t* bits_in,
            int64_t bits_ld, hipStream_t s) {
  constexpr int TN = 5;
  const int64_t blocks = ((M + kBM - 1) / kBM) * ((N + 32 * TN - 1) / (32 * TN));
  hipLaunchKernelGGL((k_q6x<TN, EPI, true, H3, V>), dim3((unsigned)blocks), dim3(64 * kW), 0, s, A,
                     Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, amax, bmax, cmax, crow,
                     amax_out, arow_parts, bits_out, bits_in, bits_ld);
}

template <int V>
int dispatch(int epi, int h3, const float* A, const uint16_t* Bp, float* C, int64_t M, int64_t N,
             int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc, const float* bias,
             const float* aux, int64_t ldaux, const float* amax, const float* bmax, float* cmax,
             float* crow, float* amax_out, int arow_parts, uint32_t* bits_out,
             const uint32_t* bits_in, int64_t bits_ld, hipStream_t s) {
#define Q6X_L(E, H)                                                                             \
  launch<E, H, V>(A, Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, amax, bmax, cmax, crow, \
                  amax_out, arow_parts, bits_out, bits_in, bits_ld, s)
  if (h3 == 0 && epi == MOLCLR_EPI_BIAS_RELU) Q6X_L(MOLCLR_EPI_BIAS_RELU, 0);
  else if (h3 == 0 && epi == MOLCLR_EPI_BIAS) Q6X_L(MOLCLR_EPI_BIAS, 0);
  else if (h3 == 2 && epi == MOLCLR_EPI_RELU_MASK) Q6X_L(MOLCLR_EPI_RELU_MASK, 2);
  else if (h3 == 2 && epi == MOLCLR_EPI_NONE) Q6X_L(MOLCLR_EPI_NONE, 2);
  else return -1;
#undef Q6X_L
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
}  // namespace

extern "C" int q6x(int variant, int epi, int h3, const float* A, const uint16_t* Bp, float* C,
                   int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad,
                   int64_t ldc, const float* bias, const float* aux, int64_t ldaux,
                   const float* amax, const float* bmax, float* cmax, float* crow,
                   float* amax_out, int arow_parts, uint32_t* bits_out, const uint32_t* bits_in,
                   int64_t bits_ld, hipStream_t s) {
#define Q6X_V(VV)                                                                                  \
  case VV:                                                                                         \
    return dispatch<VV>(epi, h3, A, Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, amax, bmax, \
                        cmax, crow, amax_out, arow_parts, bits_out, bits_in, bits_ld, s);
  if (variant >= 100 && variant < 1000) {
#define Q6PP_A(E, H, AB)                                                                         \
  launch_pp<E, H, AB>(A, Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, amax, bmax, cmax,  \
                      crow, amax_out, arow_parts, bits_out, bits_in, bits_ld, s)
#define Q6PP_L(E, H)                                   \
  switch (variant - 100) {                             \
    case 0: Q6PP_A(E, H, 0); break;                    \
    case 1: Q6PP_A(E, H, 1); break;                    \
    case 2: Q6PP_A(E, H, 2); break;                    \
    case 3: Q6PP_A(E, H, 3); break;                    \
    case 4: Q6PP_A(E, H, 4); break;                    \
    case 8: Q6PP_A(E, H, 8); break;                    \
    case 12: Q6PP_A(E, H, 12); break;                  \
    case 16: Q6PP_A(E, H, 16); break;                  \
    case 15: Q6PP_A(E, H, 15); break;                  \
    case 32: Q6PP_A(E, H, 32); break;                  \
    case 36: Q6PP_A(E, H, 36); break;                  \
    case 64: Q6PP_A(E, H, 64); break;                  \
    case 96: Q6PP_A(E, H, 96); break;                  \
    case 48: Q6PP_A(E, H, 48); break;                  \
    case 128: Q6PP_A(E, H, 128); break;                \
    case 160: Q6PP_A(E, H, 160); break;                \
    case 256: Q6PP_A(E, H, 256); break;                \
    case 384: Q6PP_A(E, H, 384); break;                \
    case 416: Q6PP_A(E, H, 416); break;                \
    case 512: Q6PP_A(E, H, 512); break;                \
    case 544: Q6PP_A(E, H, 544); break;                \
    default: return -4;                                \
  }
    if (h3 == 0 && epi == MOLCLR_EPI_BIAS_RELU) { Q6PP_L(MOLCLR_EPI_BIAS_RELU, 0) }
    else if (h3 == 0 && epi == MOLCLR_EPI_BIAS) { Q6PP_L(MOLCLR_EPI_BIAS, 0) }
    else if (h3 == 2 && epi == MOLCLR_EPI_RELU_MASK) { Q6PP_L(MOLCLR_EPI_RELU_MASK, 2) }
    else if (h3 == 2 && epi == MOLCLR_EPI_NONE) { Q6PP_L(MOLCLR_EPI_NONE, 2) }
    else return -1;
#undef Q6PP_L
#undef Q6PP_A
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  switch (variant) {
    Q6X_V(0)
    Q6X_V(1)
    Q6X_V(2)
    Q6X_V(3)
    Q6X_V(4)
    Q6X_V(7)
    default:
      return -3;
  }
#undef Q6X_V
}
