// Native bf16 GEMMs of the c5 configuration (BASELINE.json configs[4]: GIN
// 5 x 512, bf16, batch 1024 / GPU): node features are stored in bf16 and every
// product is ONE v_mfma_f32_32x32x16_bf16 with fp32 accumulation (the fp32
// path's split-bf16 kernels issue six).  The weights' bf16 operand is plane 0
// of the pre-split images molclr_bplanes_make already caches per optimizer
// step (the round-to-nearest bf16 of the fp32 master weight).
//
//   k_gemm_qb  C[M,N] = A[M,K] B(k,n) (+ bias / bias + ReLU / ReLU mask), bf16
//              out: the Linear forward (x W^T) and data gradient (dy W) of the
//              GIN MLP, A row-major bf16, B the weight plane.
//   k_gemm_wb  the weight gradient dW = dY^T X (both bf16, K = rows) with the
//              bias gradient Σ_rows dY from the staged tiles, fp32 split-K
//              partials summed in a fixed order (molclr_splitk_reduce_none).
//
// Reference: models/ginet_molclr.py:19-23,46-47 (GINEConv.mlp) at emb_dim 512,
// trained under the reference's mixed-precision switch (fp16_precision,
// molclr.py:16-24,93-96,121-123: apex O2 -- half-precision activations, fp32
// master weights and BatchNorm).
#include "mfma.h"

#include <stdlib.h>

namespace {

using namespace molclr;

// LDS written by a wave and read back by other lanes of the SAME wave: wait
// for the wave's LDS operations, no workgroup barrier

// One K step of B: a [BN][32] image (xoff swizzle) of the weight plane,
// rows clamped into the padded planes (columns >= N are never stored).
template <int BN, int T>
struct QbStageB {
  static constexpr int UNITS = BN * 4;  // 16-byte chunks per step
  static constexpr int PER = (UNITS + T - 1) / T;
  u32x4 r[PER];
  int64_t goff[PER];
  __device__ __forceinline__ void init(int64_t n0, int64_t npad, int64_t kp, int t) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      int64_t row = n0 + (u >> 2);
      row = row < npad ? row : npad - 1;
      goff[j] = (UNITS % T && u >= UNITS) ? 0 : row * kp + 8 * (u & 3);
    }
  }
  __device__ __forceinline__ void load(const uint16_t* __restrict__ Bp, int64_t k0, int t) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (j == PER - 1 && UNITS % T && t + j * T >= UNITS) continue;
      r[j] = *reinterpret_cast<const u32x4*>(Bp + goff[j] + k0);
    }
  }
  __device__ __forceinline__ void store(uint16_t* __restrict__ img, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (j == PER - 1 && UNITS % T && u >= UNITS) continue;
      *reinterpret_cast<u32x4*>(img + xoff(u >> 2, u & 3)) = r[j];
    }
  }
};

__device__ __forceinline__ float4 bf16x4_to_f4(uint2 u) {
  return make_float4(bf16_to_f32(u.x & 0xFFFFu), bf16_to_f32(u.x >> 16), bf16_to_f32(u.y & 0xFFFFu),
                     bf16_to_f32(u.y >> 16));
}
__device__ __forceinline__ uint2 f4_to_bf16x4(float4 v) {
  return make_uint2(f32x2_to_bf16x2(v.x, v.y), f32x2_to_bf16x2(v.z, v.w));
}


// ---------------------------------------------------------------------------
// k_gemm_qb: WM x WN waves; wave (wm, wn) owns rows m0 + 32 wm .. +31 and
// columns n0 + 32 TN wn .. + 32 TN - 1, the block a BM = 32 WM by BN =
// 32 TN WN tile.  A goes global -> registers -> MFMA operand: per K step of
// 32 a lane loads the two 16-byte pieces of its row it needs (lane half h:
// MFMA step s uses k0 + 16s + 8h .. +7, and the B fragment is image chunk
// 2s + h, the same k -- the k pairing of hipBLASLt's bf16 GEMM, whose results
// this kernel reproduces bit for bit on the epilogue-free products).  With BN = N every A row is
// fetched by one block only; the WN waves of a row slab read it at the same
// time, from L2.  B (the weight plane) is staged per K step into a [BN][32]
// image, double-buffered, one barrier per step.
// The main loop has no branch: every load comes from a clamped in-bounds
// address (MASK: the last K step is partial, its A values at k >= K are
// zeroed where they are consumed), so the compiler keeps counted vmcnt waits
// and the next steps' loads stay in flight across the MFMAs -- a conditional
// load made it drain every outstanding load at the top of each step.
// The epilogue goes through the wave's 4 KB of LDS so rows leave as 8-byte
// (4 x bf16) pieces.
// ---------------------------------------------------------------------------
template <int WM, int WN, int TN, int D, int EPI, bool MASK>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_qb(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bp, uint16_t* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const uint16_t* __restrict__ aux, int64_t ldaux) {
  constexpr int T = 64 * WM * WN;
  constexpr int BM = 32 * WM, WC = 32 * TN, BN = WC * WN;
  constexpr int BI = BN * XK;  // bf16 elements per B image
  static_assert(WM * WN * 32 * 32 * (int)sizeof(float) <= 2 * BI * (int)sizeof(uint16_t),
                "epilogue tiles exceed the LDS images");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BI];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BM - 1) / BM);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);  // a row slab's column tiles share an XCD
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;

  int64_t arow_i = m0 + 32 * wm + li;
  arow_i = arow_i < M ? arow_i : M - 1;
  const uint16_t* __restrict__ arow = A + arow_i * lda;
  const int ns = (int)(kp / BK);  // K steps (the planes' K is padded to BK)
  auto kstep = [&](int i) { return i < ns ? i : ns - 1; };
  // this lane's 16 k of step i (K % 8 == 0: an 8-element chunk is all in or out)
  auto load_a = [&](int i, u32x4(&r)[2]) {
    const int64_t k = (int64_t)kstep(i) * BK + 8 * lh;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      int64_t kc = k + 16 * c;
      if constexpr (MASK) kc = kc < K - 8 ? kc : K - 8;
      r[c] = *reinterpret_cast<const u32x4*>(arow + kc);
    }
  };

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  // All 2 TN B fragments of the step are read before the first MFMA (the
  // reads retire in order, so each MFMA waits only for its own fragment with
  // a counted lgkmcnt and the LDS latency hides behind the earlier MFMAs).
  auto compute = [&](const uint16_t* Bs, const u32x4(&a)[2], int i) {
    bf16x8 f[2][TN];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < TN; ++b) f[s][b] = xfrag(Bs, wn * WC + 32 * b + li, 2 * s + lh);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 as = a[s];
      if constexpr (MASK) {
        const u32x4 z = {0u, 0u, 0u, 0u};
        if ((int64_t)i * BK + 16 * s + 8 * lh >= K) as = z;
      }
      const bf16x8 av = __builtin_bit_cast(bf16x8, as);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, f[s][b], acc[b], 0, 0, 0);
    }
  };

  static_assert(D % 2 == 0, "the A ring spans whole B double-buffer periods");
  QbStageB<BN, T> sb;
  sb.init(n0, npad, kp, tid);
  uint16_t* buf[2] = {lds, lds + BI};
  auto kof = [&](int i) { return (int64_t)kstep(i) * BK; };
  u32x4 a[D][2];  // ring: slot j holds A of the steps i with i % D == j
  sb.load(Bp, kof(0), tid);
#pragma unroll
  for (int j = 0; j < D; ++j) load_a(j, a[j]);
  sb.store(buf[0], tid);
  sb.load(Bp, kof(1), tid);
  __syncthreads();
  // step i: buf[i & 1] holds B(i), sb holds B(i+1) in flight, A(i) .. A(i+D-1)
  // in flight in the ring.  B(i+1) is written right after the barrier into
  // the buffer the previous step read; A(i+D) is issued into the slot step i
  // has just consumed, so D steps of A (the streamed operand) are in flight.
  // Loads past the last step re-read it (never consumed).
  int i = 0;
  for (; i + D <= ns; i += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      sb.store(buf[(j + 1) & 1], tid);
      sb.load(Bp, kof(i + j + 2), tid);
      compute(buf[j & 1], a[j], i + j);
      load_a(i + j + D, a[j]);
      __syncthreads();
    }
  }
#pragma unroll
  for (int j = 0; j < D - 1; ++j) {  // the last ns % D steps (i is a multiple of D)
    if (i + j < ns) {
      sb.store(buf[(j + 1) & 1], tid);
      compute(buf[j & 1], a[j], i + j);
      __syncthreads();
    }
  }
  __syncthreads();  // the images are reused below

  float* tw = reinterpret_cast<float*>(lds) + wave * 32 * 32;
  const int64_t mw = m0 + 32 * wm;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + wn * WC + 32 * b;
    if (nb >= N) break;  // wave-uniform
#pragma unroll
    for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[b][r];
    wave_lds_sync();  // the tile is this wave's own: no block barrier
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, c4 = idx & 7;
      const int64_t m = mw + row, n = nb + 4 * c4;
      if (m >= M || n >= N) continue;
      float4 v = *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
      if (n + 4 <= N) {
        if (EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU) {
          v = f4add(v, *reinterpret_cast<const float4*>(bias + n));
          if (EPI == MOLCLR_EPI_BIAS_RELU)
            v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
        }
        if (EPI == MOLCLR_EPI_RELU_MASK) {
          const float4 x = bf16x4_to_f4(*reinterpret_cast<const uint2*>(aux + m * ldaux + n));
          v = make_float4(x.x > 0.f ? v.x : 0.f, x.y > 0.f ? v.y : 0.f, x.z > 0.f ? v.z : 0.f,
                          x.w > 0.f ? v.w : 0.f);
        }
        *reinterpret_cast<uint2*>(C + m * ldc + n) = f4_to_bf16x4(v);
      } else {
        const float e[4] = {v.x, v.y, v.z, v.w};
        for (int j = 0; j < 4 && n + j < N; ++j) {
          float x = e[j];
          if (EPI == MOLCLR_EPI_BIAS) x = x + bias[n + j];
          if (EPI == MOLCLR_EPI_BIAS_RELU) x = fmaxf(x + bias[n + j], 0.f);
          if (EPI == MOLCLR_EPI_RELU_MASK) x = bf16_to_f32(aux[m * ldaux + n + j]) > 0.f ? x : 0.f;
          C[m * ldc + n + j] = (uint16_t)(f32x2_to_bf16x2(x, 0.f) & 0xFFFFu);
        }
      }
    }
    wave_lds_sync();  // the wave's tile is rewritten by the next block
  }
}

// ---------------------------------------------------------------------------
// k_gemm_tb: the same product on 256 x 256 output tiles, both operands staged
// in LDS by global_load_lds (the LDS-DMA path: no VGPR round trip, no
// ds_write), 64-deep K steps, two stages.  8 waves as 4 (M) x 2 (N), each a
// 64 x 128 sub-tile (2 x 4 MFMA blocks: 6 fragment reads per 8 MFMAs).  Per
// stage and operand the image is [256 rows][128 B]; one wave-instruction of
// the DMA writes 1 KB (8 rows) linearly, so the bank swizzle -- chunk c of
// row r stored at chunk c ^ ((r >> 1) & 7) -- is applied on the SOURCE
// address (lane L of a piece fetches the logical chunk its slot holds) and
// again on the fragment read; every 16-lane group of a ds_read_b128 then
// hits 16 distinct 16-byte slots.  Requires K % 64 == 0 (the host falls back
// to k_gemm_qb otherwise).
// ---------------------------------------------------------------------------

__device__ __forceinline__ int t128(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }

template <int EPI>
__global__ __launch_bounds__(512) void k_gemm_tb(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bp, uint16_t* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const uint16_t* __restrict__ aux, int64_t ldaux) {
  constexpr int BM = 256, BN = 256, KT = 64;
  constexpr int SI = BM * KT * 2;  // bytes per operand image per stage (32 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * SI];  // [stage][A, B]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BM - 1) / BM);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);  // a row slab's column tiles share an XCD
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;

  // DMA sources: wave w fills pieces 4w .. 4w+3 (8 rows each) of both images
  const uint16_t* asrc[4];
  const uint16_t* bsrc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 8 * (4 * wave + q) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int64_t gm = m0 + r < M ? m0 + r : M - 1;
    const int64_t gn = n0 + r < npad ? n0 + r : npad - 1;
    asrc[q] = A + gm * lda + 8 * c;
    bsrc[q] = Bp + gn * kp + 8 * c;
  }
  const int nt = (int)(K / KT);
  auto stage = [&](int buf, int t) {
    const int64_t k0 = (int64_t)(t < nt ? t : nt - 1) * KT;
    uint8_t* ia = lds + buf * 2 * SI + wave * 4096;
    uint8_t* ib = ia + SI;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(asrc[q] + k0), (lds_as_ptr)(ia + 1024 * q), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(bsrc[q] + k0), (lds_as_ptr)(ib + 1024 * q), 16, 0, 0);
    }
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ra = 64 * wm + li, rb = 128 * wn + li;  // this lane's fragment rows
  // 16-deep substeps; substep q+1's six fragments are read before substep q's
  // eight MFMAs issue, so the LDS latency hides behind them
  auto compute = [&](int buf) {
    const uint8_t* ia = lds + buf * 2 * SI;
    const uint8_t* ib = ia + SI;
    bf16x8 fa[2][2], fb[2][4];
    auto read = [&](int q, bf16x8(&a)[2], bf16x8(&b)[4]) {
      const int c = 2 * q + lh;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ia + t128(ra + 32 * i, c)));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ib + t128(rb + 32 * j, c)));
    };
    read(0, fa[0], fb[0]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < 3) read(q + 1, fa[(q + 1) & 1], fb[(q + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q & 1][i], fb[q & 1][j], acc[i][j], 0,
                                                               0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  stage(0, 0);
  __syncthreads();  // (waits for the DMA: vmcnt(0))
  for (int t = 0; t < nt; ++t) {
    stage((t + 1) & 1, t + 1);  // past the last step: re-reads it into the idle buffer
    compute(t & 1);
    __syncthreads();
  }

  // epilogue: per 32 x 32 block through the wave's 4 KB of LDS, rows leave as
  // 8-byte (4 x bf16) pieces
  float* tw = reinterpret_cast<float*>(lds) + wave * 32 * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t mb = m0 + 64 * wm + 32 * i, nb = n0 + 128 * wn + 32 * j;
      if (nb >= N) continue;  // wave-uniform
#pragma unroll
      for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[i][j][r];
      wave_lds_sync();
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = it * 64 + lane;
        const int row = idx >> 3, c4 = idx & 7;
        const int64_t m = mb + row, n = nb + 4 * c4;
        if (m >= M || n >= N) continue;
        float4 v = *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
        if (n + 4 <= N) {
          if (EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU) {
            v = f4add(v, *reinterpret_cast<const float4*>(bias + n));
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if (EPI == MOLCLR_EPI_RELU_MASK) {
            const float4 x = bf16x4_to_f4(*reinterpret_cast<const uint2*>(aux + m * ldaux + n));
            v = make_float4(x.x > 0.f ? v.x : 0.f, x.y > 0.f ? v.y : 0.f, x.z > 0.f ? v.z : 0.f,
                            x.w > 0.f ? v.w : 0.f);
          }
          *reinterpret_cast<uint2*>(C + m * ldc + n) = f4_to_bf16x4(v);
        } else {
          const float e[4] = {v.x, v.y, v.z, v.w};
          for (int jj = 0; jj < 4 && n + jj < N; ++jj) {
            float x = e[jj];
            if (EPI == MOLCLR_EPI_BIAS) x = x + bias[n + jj];
            if (EPI == MOLCLR_EPI_BIAS_RELU) x = fmaxf(x + bias[n + jj], 0.f);
            if (EPI == MOLCLR_EPI_RELU_MASK) x = bf16_to_f32(aux[m * ldaux + n + jj]) > 0.f ? x : 0.f;
            C[m * ldc + n + jj] = (uint16_t)(f32x2_to_bf16x2(x, 0.f) & 0xFFFFu);
          }
        }
      }
      wave_lds_sync();
    }
  }
}

// bf16 bit pattern h (low 16 bits) > 0: +denormal .. +inf, not +0, NaN or negative
__device__ __forceinline__ bool bf16_pos(uint32_t h) { return h - 1u < 0x7F80u; }

// ---------------------------------------------------------------------------
// k_gemm_tp: k_gemm_tb as a persistent kernel.  One block per CU walks its
// share of the output tiles; the first K step of the NEXT tile is DMA-staged
// during the current tile's last step, and the epilogue (a separate 32 KB LDS
// region, 160 KB in all) runs while that DMA lands, so a tile's output
// stores and ReLU-mask / bias loads overlap the next tile's staging instead
// of idling the CU between blocks.  The mask operand is fetched before the
// last K step's MFMAs (its latency hides behind them).
// Tiles: XCD x's blocks own a contiguous range of logical tiles (row slab
// major), in proportion to their number; block p of the XCD takes every P-th.
// Results are identical to k_gemm_tb (same fragments, same MFMA order).
// BITS: the ReLU mask as bits, column-block-major words [n / 32][m] (bits_ld
// = M; k_gemm_q6's layout): a BIAS_RELU product writes bit (n % 32) = (C > 0)
// to bits_out, a RELU_MASK product reads its mask from bits_in instead of aux
// (1/16 of the bytes).  Everything the epilogue reads -- bias, mask words --
// is loaded at the start of the tile, ahead of the K loop: CDNA4's vmcnt
// counts stores too, so a load issued among the epilogue's stores would wait
// for them all.
// ---------------------------------------------------------------------------
// SW: the MFMAs take the operands swapped (B fragment first), so a lane's
// accumulators are one ROW of the 32 x 32 block (row li, columns in four runs
// of four): the epilogue stores straight from registers -- no LDS transpose,
// no wave syncs -- the bias comes from a 1 KB LDS copy of the tile's columns,
// and a row's ReLU bits are one word from two lanes.  Same products in the
// same k order: results identical to the unswapped form.  Needs the ReLU mask
// (if any) as bits.
template <int EPI, int NW, bool BITS = false, bool SW = false>
__global__ __launch_bounds__(64 * NW) void k_gemm_tp(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bp, uint16_t* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const uint16_t* __restrict__ aux, int64_t ldaux,
    uint32_t* __restrict__ bits_out, const uint32_t* __restrict__ bits_in, int64_t bits_ld) {
  constexpr bool MASK_BITS = BITS && EPI == MOLCLR_EPI_RELU_MASK;
  constexpr bool OUT_BITS = BITS && EPI == MOLCLR_EPI_BIAS_RELU;
  constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;
  static_assert(!SW || EPI != MOLCLR_EPI_RELU_MASK || BITS,
                "the swapped epilogue takes its ReLU mask as bits");
  constexpr int BM = 256, BN = 256, KT = 64;
  constexpr int SI = BM * KT * 2;       // bytes per operand image per stage (32 KB)
  constexpr int WMW = NW == 8 ? 4 : 2;  // waves along M (8 waves: 4 x 2, 4 waves: 2 x 2)
  constexpr int TI = BM / 32 / WMW, TJ = BN / 32 / (NW / WMW);  // a wave's 32 x 32 blocks
  constexpr int PQ = 32 / NW;           // 1 KB DMA pieces per wave and operand
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * SI + NW * 4096];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WMW, wn = wave / WMW;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntiles = (int)((M + BM - 1) / BM) * ntn;
  const int G = gridDim.x, x = blockIdx.x & 7, pos = blockIdx.x >> 3;
  const int q8 = G >> 3, r8 = G & 7;
  const int P = q8 + (x < r8 ? 1 : 0);                                  // blocks on XCD x
  const int base = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;  // their first rank
  const int hi = (int)((int64_t)(base + P) * ntiles / G);
  int t = (int)((int64_t)base * ntiles / G) + pos;
  if (t >= hi) return;

  auto tile_src = [&](int tt, const uint16_t* (&as)[PQ], const uint16_t* (&bs)[PQ]) {
    const int64_t m0 = (int64_t)(tt / ntn) * BM, n0 = (int64_t)(tt % ntn) * BN;
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int r = 8 * (PQ * wave + q) + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int64_t gm = m0 + r < M ? m0 + r : M - 1;
      const int64_t gn = n0 + r < npad ? n0 + r : npad - 1;
      as[q] = A + gm * lda + 8 * c;
      bs[q] = Bp + gn * kp + 8 * c;
    }
  };
  const int nt = (int)(K / KT);
  auto stage = [&](int buf, const uint16_t* const (&as)[PQ], const uint16_t* const (&bs)[PQ], int s) {
    const int64_t k0 = (int64_t)s * KT;
    uint8_t* ia = lds + buf * 2 * SI + wave * (PQ * 1024);
    uint8_t* ib = ia + SI;
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(as[q] + k0), (lds_as_ptr)(ia + 1024 * q), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(bs[q] + k0), (lds_as_ptr)(ib + 1024 * q), 16, 0, 0);
    }
  };

  const int ra = 32 * TI * wm + li, rb = 32 * TJ * wn + li;  // this lane's fragment rows
  f32x16 acc[TI][TJ];
  auto compute = [&](int buf) {
    const uint8_t* ia = lds + buf * 2 * SI;
    const uint8_t* ib = ia + SI;
    bf16x8 fa[2][TI], fb[2][TJ];
    auto read = [&](int q, bf16x8(&a)[TI], bf16x8(&b)[TJ]) {
      const int c = 2 * q + lh;
#pragma unroll
      for (int i = 0; i < TI; ++i)
        a[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ia + t128(ra + 32 * i, c)));
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        b[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ib + t128(rb + 32 * j, c)));
    };
    read(0, fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[q & 1][j], fa[q & 1][i],
                                                                    acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q & 1][i], fb[q & 1][j],
                                                                    acc[i][j], 0, 0, 0);
      if (q < 3) {
        read(q + 1, fa[(q + 1) & 1], fb[(q + 1) & 1]);
        interleave_mfma_reads<TI * TJ, TI + TJ>();
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // this lane's epilogue pieces of a 32 x 32 block: rows (lane >> 3) + 8 it,
  // columns 4 (lane & 7) .. +3
  const int erow = lane >> 3, ec4 = lane & 7;
  constexpr bool AUX_MASK = EPI == MOLCLR_EPI_RELU_MASK && !MASK_BITS;
  constexpr int AMI = AUX_MASK ? 2 : 1, AMJ = AUX_MASK ? TJ : 1;
  uint2 am[AMI][AMJ][4];  // ReLU-mask operand of one row of blocks, one row ahead
  auto fetch_mask = [&](int64_t m0, int64_t n0, int i, uint2(&dst)[AMJ][4]) {
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        int64_t m = m0 + 32 * TI * wm + 32 * i + erow + 8 * it;
        int64_t n = n0 + 32 * TJ * wn + 32 * j + 4 * ec4;
        m = m < M ? m : M - 1;
        n = n + 4 <= N ? n : 0;  // partial / outside pieces re-read below or skipped
        dst[j][it] = *reinterpret_cast<const uint2*>(aux + m * ldaux + n);
      }
  };

  float* tw = reinterpret_cast<float*>(lds + 4 * SI) + wave * 32 * 32;
  // SW: the tile's bias columns, one 1 KB copy per tile parity (the epilogue
  // region is free: no transposes)
  float* const bias_lds = reinterpret_cast<float*>(lds + 4 * SI);
  const uint16_t* asrc[PQ];
  const uint16_t* bsrc[PQ];
  tile_src(t, asrc, bsrc);
  stage(0, asrc, bsrc, 0);
  __syncthreads();
  int buf = 0;
  int parity = 0;
  constexpr int BVJ = HAS_BIAS && !SW ? TJ : 1, MWI = MASK_BITS ? TI : 1, MWJ = MASK_BITS ? TJ : 1;
  float4 bv[BVJ];           // this lane's bias columns of the tile
  uint32_t mw[MWI][MWJ][4];  // this lane's mask words of the tile (MASK_BITS)
  for (;;) {
    const int64_t m0 = (int64_t)(t / ntn) * BM, n0 = (int64_t)(t % ntn) * BN;
    const int tn = t + P;
    const bool more = tn < hi;
    float* const bl = bias_lds + 256 * parity;
    float4 breg = f4zero();  // SW: lanes 0..63's chunk of the tile's bias
    if constexpr (SW && HAS_BIAS) {
      if (tid < 64) {
        int64_t n = n0 + 4 * tid;
        n = n + 4 <= N ? n : N - 4;  // clamped chunks are never read (full path only)
        breg = *reinterpret_cast<const float4*>(bias + n);
      }
    } else if constexpr (HAS_BIAS) {
      // unconditional loads from a clamped column (bv[j] is used only where
      // n + 4 <= N): a zero-initialised conditional load wrote its registers
      // by VALU, which made the compiler drain the previous tile's stores
      // (vmcnt(0)) at the tile head
      // (N >= 4: launch_tp)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        int64_t n = n0 + 32 * TJ * wn + 32 * j + 4 * ec4;
        n = n + 4 <= N ? n : N - 4;
        bv[j] = *reinterpret_cast<const float4*>(bias + n);
      }
    }

#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int s = 0; s < nt; ++s) {
      if (s + 1 < nt) {
        stage(buf ^ 1, asrc, bsrc, s + 1);
      } else if (more) {
        const uint16_t* an[PQ];
        const uint16_t* bn[PQ];
        tile_src(tn, an, bn);
        stage(buf ^ 1, an, bn, 0);
      }
      if constexpr (SW && HAS_BIAS) {
        // visible to every wave after this step's barrier; the copy of the
        // other parity may still be read by the previous tile's epilogue
        if (s == nt - 1 && tid < 64) *reinterpret_cast<float4*>(bl + 4 * tid) = breg;
      }
      compute(buf);
      __syncthreads();  // step s + 1 (or the next tile's step 0) has landed; buf is free
      buf ^= 1;
    }

    if constexpr (SW) {
      // rows from registers: lane (li, lh) of block (i, j) holds row mb + li,
      // columns nb + 8 q + 4 lh .. +3 in acc[i][j][4 q .. 4 q + 3]
      uint32_t mws[MWI][MWJ];  // the row's mask word per block (MASK_BITS)
      if constexpr (MASK_BITS) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            int64_t m = m0 + 32 * TI * wm + 32 * i + li;
            m = m < M ? m : M - 1;
            int64_t nb = n0 + 32 * TJ * wn + 32 * j;
            nb = nb < N ? nb : 0;
            mws[i][j] = bits_in[(nb >> 5) * bits_ld + m];
          }
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int64_t mb = m0 + 32 * TI * wm + 32 * i, nb = n0 + 32 * TJ * wn + 32 * j;
          if (nb >= N) continue;  // wave-uniform
          const int64_t m = mb + li;
          uint32_t pos = 0;  // OUT_BITS: the row's bits of C > 0 in this lane's columns
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cb = 8 * q + 4 * lh;  // column within the block
            const int64_t n = nb + cb;
            float4 v = make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2],
                                   acc[i][j][4 * q + 3]);
            uint32_t mk = 15u;
            if constexpr (MASK_BITS) mk = (mws[i][j] >> cb) & 15u;
            if (m < M && n < N) {
              if (n + 4 <= N) {
                if constexpr (HAS_BIAS) {
                  v = f4add(v, *reinterpret_cast<const float4*>(bl + (nb - n0) + cb));
                  if (EPI == MOLCLR_EPI_BIAS_RELU)
                    v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
                }
                if constexpr (MASK_BITS)
                  v = make_float4(mk & 1u ? v.x : 0.f, mk & 2u ? v.y : 0.f, mk & 4u ? v.z : 0.f,
                                  mk & 8u ? v.w : 0.f);
                const uint2 o = f4_to_bf16x4(v);
                *reinterpret_cast<uint2*>(C + m * ldc + n) = o;
                if constexpr (OUT_BITS)
                  pos |= ((bf16_pos(o.x & 0xFFFFu) ? 1u : 0u) | (bf16_pos(o.x >> 16) ? 2u : 0u) |
                          (bf16_pos(o.y & 0xFFFFu) ? 4u : 0u) | (bf16_pos(o.y >> 16) ? 8u : 0u))
                         << cb;
              } else {
                const float e[4] = {v.x, v.y, v.z, v.w};
                for (int jj = 0; jj < 4 && n + jj < N; ++jj) {
                  float xv = e[jj];
                  if (EPI == MOLCLR_EPI_BIAS) xv = xv + bias[n + jj];
                  if (EPI == MOLCLR_EPI_BIAS_RELU) xv = fmaxf(xv + bias[n + jj], 0.f);
                  if constexpr (MASK_BITS) xv = ((mk >> jj) & 1u) ? xv : 0.f;
                  const uint16_t h = (uint16_t)(f32x2_to_bf16x2(xv, 0.f) & 0xFFFFu);
                  C[m * ldc + n + jj] = h;
                  if constexpr (OUT_BITS) pos |= (bf16_pos(h) ? 1u : 0u) << (cb + jj);
                }
              }
            }
          }
          if constexpr (OUT_BITS) {
            pos |= __shfl_xor(pos, 32, 64);  // the row's other 16 columns (lane half lh ^ 1)
            if (lh == 0 && m < M) bits_out[(nb >> 5) * bits_ld + m] = pos;
          }
        }
      }
      parity ^= 1;
      if (!more) break;
      t = tn;
      tile_src(t, asrc, bsrc);
      continue;
    }
    if constexpr (MASK_BITS) {
      // the tile's mask words, all loaded before the first store (then one
      // latency per tile); held through the K loop they would spill
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            int64_t m = m0 + 32 * TI * wm + 32 * i + erow + 8 * it;
            m = m < M ? m : M - 1;
            int64_t nb = n0 + 32 * TJ * wn + 32 * j;
            nb = nb < N ? nb : 0;
            mw[i][j][it] = bits_in[(nb >> 5) * bits_ld + m];
          }
    }
    if constexpr (AUX_MASK) fetch_mask(m0, n0, 0, am[0]);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      if constexpr (AUX_MASK)
        if (i + 1 < TI) fetch_mask(m0, n0, i + 1, am[(i + 1) & (AMI - 1)]);
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int64_t mb = m0 + 32 * TI * wm + 32 * i, nb = n0 + 32 * TJ * wn + 32 * j;
        if (nb >= N) continue;  // wave-uniform
#pragma unroll
        for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[i][j][r];
        wave_lds_sync();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const int row = erow + 8 * it;
          const int64_t m = mb + row, n = nb + 4 * ec4;
          uint32_t pos = 0;  // OUT_BITS: this lane's nibble of C > 0
          if (m < M && n < N) {
            float4 v = *reinterpret_cast<const float4*>(tw + row * 32 + 4 * ec4);
            uint32_t mk = 15u;  // MASK_BITS: this lane's mask nibble
            if constexpr (MASK_BITS) mk = (mw[i][j][it] >> (4 * ec4)) & 15u;
            if (n + 4 <= N) {
              if constexpr (HAS_BIAS) {
                v = f4add(v, bv[j]);
                if (EPI == MOLCLR_EPI_BIAS_RELU)
                  v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
              }
              if constexpr (MASK_BITS) {
                v = make_float4(mk & 1u ? v.x : 0.f, mk & 2u ? v.y : 0.f, mk & 4u ? v.z : 0.f,
                                mk & 8u ? v.w : 0.f);
              } else if constexpr (AUX_MASK) {
                const float4 xm = bf16x4_to_f4(am[i & (AMI - 1)][j][it]);
                v = make_float4(xm.x > 0.f ? v.x : 0.f, xm.y > 0.f ? v.y : 0.f,
                                xm.z > 0.f ? v.z : 0.f, xm.w > 0.f ? v.w : 0.f);
              }
              const uint2 o = f4_to_bf16x4(v);
              *reinterpret_cast<uint2*>(C + m * ldc + n) = o;
              if constexpr (OUT_BITS)  // the stored bf16 values > 0 (what the aux mask tests)
                pos = (bf16_pos(o.x & 0xFFFFu) ? 1u : 0u) | (bf16_pos(o.x >> 16) ? 2u : 0u) |
                      (bf16_pos(o.y & 0xFFFFu) ? 4u : 0u) | (bf16_pos(o.y >> 16) ? 8u : 0u);
            } else {
              const float e[4] = {v.x, v.y, v.z, v.w};
              for (int jj = 0; jj < 4 && n + jj < N; ++jj) {
                float xv = e[jj];
                if (EPI == MOLCLR_EPI_BIAS) xv = xv + bias[n + jj];
                if (EPI == MOLCLR_EPI_BIAS_RELU) xv = fmaxf(xv + bias[n + jj], 0.f);
                if constexpr (MASK_BITS) xv = ((mk >> jj) & 1u) ? xv : 0.f;
                if constexpr (AUX_MASK)
                  xv = bf16_to_f32(aux[m * ldaux + n + jj]) > 0.f ? xv : 0.f;
                const uint16_t h = (uint16_t)(f32x2_to_bf16x2(xv, 0.f) & 0xFFFFu);
                C[m * ldc + n + jj] = h;
                if constexpr (OUT_BITS) pos |= (bf16_pos(h) ? 1u : 0u) << jj;
              }
            }
          }
          if constexpr (OUT_BITS) {
            // a row's 8 lanes (lane / 8) hold its 32 columns as nibbles: one
            // ballot per nibble bit, interleaved into the row's word
            const uint64_t bj[4] = {__ballot((pos & 1u) != 0u), __ballot((pos & 2u) != 0u),
                                    __ballot((pos & 4u) != 0u), __ballot((pos & 8u) != 0u)};
            if (ec4 == 0 && m < M && nb < N) {
              uint32_t w = 0;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                uint32_t x = (uint32_t)(bj[q] >> (8 * erow)) & 0xFFu;  // bit c -> bit 4 c
                x = (x | (x << 12)) & 0x000F000Fu;
                x = (x | (x << 6)) & 0x03030303u;
                x = (x | (x << 3)) & 0x11111111u;
                w |= x << q;
              }
              bits_out[(nb >> 5) * bits_ld + m] = w;
            }
          }
        }
        wave_lds_sync();
      }
    }
    if (!more) break;
    t = tn;
    tile_src(t, asrc, bsrc);
  }
}

// ---------------------------------------------------------------------------
// k_gemm_tc: k_gemm_tb's tile and wave layout with 32-deep K steps in a ring
// of four LDS stages (32 KB each: [256 rows][64 B] per operand, the xoff
// swizzle applied on the DMA source address and on the read).  Three steps
// are in flight while one is consumed; a step is waited for with a counted
// vmcnt (the two younger steps' DMAs stay outstanding) and a raw s_barrier,
// never a full drain, so the loads span the barriers.
// ---------------------------------------------------------------------------
template <int EPI>
__global__ __launch_bounds__(512) void k_gemm_tc(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bp, uint16_t* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const uint16_t* __restrict__ aux, int64_t ldaux) {
  constexpr int BM = 256, BN = 256, NS = 4;
  constexpr int SI = BM * BK * 2;  // bytes per operand image per stage (16 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[NS * 2 * SI];  // [stage][A, B]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BM - 1) / BM);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;

  // DMA sources: wave w fills pieces 2w, 2w+1 (16 rows x 64 B each) of both
  // images; lane L of a piece: row 16p + L/4, slot L%4 holds chunk
  // (L%4) ^ ((row >> 2) & 3)
  const uint16_t* asrc[2];
  const uint16_t* bsrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 16 * (2 * wave + q) + (lane >> 2);
    const int c = (lane & 3) ^ ((r >> 2) & 3);
    const int64_t gm = m0 + r < M ? m0 + r : M - 1;
    const int64_t gn = n0 + r < npad ? n0 + r : npad - 1;
    asrc[q] = A + gm * lda + 8 * c;
    bsrc[q] = Bp + gn * kp + 8 * c;
  }
  const int nt = (int)(kp / BK);  // K % 32 == 0 (host)
  auto issue = [&](int t) {
    const int64_t k0 = (int64_t)(t < nt ? t : nt - 1) * BK;
    uint8_t* ia = lds + (t % NS) * 2 * SI + wave * 2048;
    uint8_t* ib = ia + SI;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(asrc[q] + k0), (lds_as_ptr)(ia + 1024 * q), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(bsrc[q] + k0), (lds_as_ptr)(ib + 1024 * q), 16, 0, 0);
    }
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ra = 64 * wm + li, rb = 128 * wn + li;
  bf16x8 fa[2][2], fb[2][4];
  auto read = [&](int t) {
    const uint16_t* ia = reinterpret_cast<const uint16_t*>(lds + (t % NS) * 2 * SI);
    const uint16_t* ib = ia + SI / 2;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[s][i] = xfrag(ia, ra + 32 * i, 2 * s + lh);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[s][j] = xfrag(ib, rb + 32 * j, 2 * s + lh);
    }
  };
  auto mfma = [&]() {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // Two wave groups, one wave of each per SIMD, run a barrier apart: while
  // one group issues MFMAs the other reads its fragments, so a SIMD's MFMA
  // pipe alternates between its two waves instead of both idling in the
  // read phase.  Group g's step t: X (barrier) -> DMA of step t+3 -> reads ->
  // Y (barrier) -> MFMAs.  Global barrier b_k: group 0's X_t = b_2t,
  // Y_t = b_2t+1; group 1's X_t = b_2t+1, Y_t = b_2t+2 (one extra barrier
  // first).  Step t is read after b_2t (group 0) / b_2t+1 (group 1), so every
  // wave retires its own DMA of step t before b_2t: group 0 before X_t,
  // group 1 before Y_t-1, each with steps t+1 and t+2 still in flight
  // (vmcnt(8)).  Step t+3 reuses step t-1's buffer, whose last reads (group
  // 1's, before b_2t) precede both groups' issue points.
  const bool g1 = wave >= 4;  // wave-uniform (scalar)
  issue(0);
  issue(1);
  issue(2);
  if (g1) {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // step 0 (before b_0)
    barrier();                                         // b_0
  }
  for (int t = 0; t < nt; ++t) {
    if (!g1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    barrier();  // X_t
    issue(t + 3);  // past the last step: re-reads it (never consumed)
    read(t);
    if (g1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // step t+1, before b_2t+2
    barrier();  // Y_t
    mfma();
  }
  if (!g1) barrier();  // group 0's partner of group 1's last Y
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  float* tw = reinterpret_cast<float*>(lds) + wave * 32 * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t mb = m0 + 64 * wm + 32 * i, nb = n0 + 128 * wn + 32 * j;
      if (nb >= N) continue;  // wave-uniform
#pragma unroll
      for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[i][j][r];
      wave_lds_sync();
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = it * 64 + lane;
        const int row = idx >> 3, c4 = idx & 7;
        const int64_t m = mb + row, n = nb + 4 * c4;
        if (m >= M || n >= N) continue;
        float4 v = *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
        if (n + 4 <= N) {
          if (EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU) {
            v = f4add(v, *reinterpret_cast<const float4*>(bias + n));
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if (EPI == MOLCLR_EPI_RELU_MASK) {
            const float4 x = bf16x4_to_f4(*reinterpret_cast<const uint2*>(aux + m * ldaux + n));
            v = make_float4(x.x > 0.f ? v.x : 0.f, x.y > 0.f ? v.y : 0.f, x.z > 0.f ? v.z : 0.f,
                            x.w > 0.f ? v.w : 0.f);
          }
          *reinterpret_cast<uint2*>(C + m * ldc + n) = f4_to_bf16x4(v);
        } else {
          const float e[4] = {v.x, v.y, v.z, v.w};
          for (int jj = 0; jj < 4 && n + jj < N; ++jj) {
            float x = e[jj];
            if (EPI == MOLCLR_EPI_BIAS) x = x + bias[n + jj];
            if (EPI == MOLCLR_EPI_BIAS_RELU) x = fmaxf(x + bias[n + jj], 0.f);
            if (EPI == MOLCLR_EPI_RELU_MASK) x = bf16_to_f32(aux[m * ldaux + n + jj]) > 0.f ? x : 0.f;
            C[m * ldc + n + jj] = (uint16_t)(f32x2_to_bf16x2(x, 0.f) & 0xFFFFu);
          }
        }
      }
      wave_lds_sync();
    }
  }
}

// ---------------------------------------------------------------------------
// k_gemm_wb: part[split][m][n] = Σ_{k in split} A[k][m] B[k][n] (A = dY, B = X,
// both row-major [rows][*] bf16, i.e. K-major operands), WM waves stacked
// along M (32 rows each, BM = 32 WM) over BN = 32 TN columns.  Both operands
// are staged as K-major [k][rows] bf16 images (kswz XOR) read with the
// transposed LDS read (kmfrag); staging is a 16-byte copy of 8 consecutive
// rows at one k.  CS: the column sums Σ_k A[k][m] (the bias gradient) of the
// staged A tiles go to cs_part[split][m].  Double-buffered, one barrier per K
// step, no branch in the main loop (loads from clamped rows; MASK: K % 32 !=
// 0, rows at or past K are zeroed when staged).
// ---------------------------------------------------------------------------
template <int ROWS, int T, bool MASK>
struct WbStage {
  static constexpr int UNITS = BK * (ROWS / 8);  // (k, 8-row group) per step
  static constexpr int PER = (UNITS + T - 1) / T;
  const uint16_t* p[PER];
  int64_t ld;
  u32x4 r[PER];
  __device__ __forceinline__ void init(const uint16_t* __restrict__ src, int64_t ld_, int64_t row0,
                                       int64_t rows, int t) {
    ld = ld_;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      const int rb = u % (ROWS / 8), k = u / (ROWS / 8);
      const int64_t gr = row0 + 8 * rb;
      p[j] = src + (int64_t)(k < BK ? k : 0) * ld + (gr < rows ? gr : rows - 8);
    }
  }
  // rows k0 .. k0 + 31; MASK: rows past kmax (= K - 1) read row kmax instead
  __device__ __forceinline__ void load(int64_t k0, int64_t kmax, int t) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (j == PER - 1 && UNITS % T && u >= UNITS) continue;
      int64_t base = k0;
      if constexpr (MASK) {
        const int k = u / (ROWS / 8);
        base = k0 + k <= kmax ? k0 : kmax - k;
      }
      r[j] = *reinterpret_cast<const u32x4*>(p[j] + base * ld);
    }
  }
  // zero the rows at or past kend (MASK only)
  __device__ __forceinline__ void mask(int64_t k0, int64_t kend, int t) {
    if constexpr (MASK) {
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int k = (t + j * T) / (ROWS / 8);
        const u32x4 z = {0u, 0u, 0u, 0u};
        if (k0 + k >= kend) r[j] = z;
      }
    }
  }
  __device__ __forceinline__ void store(uint16_t* __restrict__ img, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (j == PER - 1 && UNITS % T && u >= UNITS) continue;
      const int rb = u % (ROWS / 8), k = u / (ROWS / 8);
      *reinterpret_cast<u32x4*>(img + k * ROWS + ((8 * rb) ^ kswz<ROWS>(k))) = r[j];
    }
  }
  // column sums over k of this thread's 8 rows (fixed rows per thread: T is a
  // multiple of ROWS / 8); `valid` false adds nothing (a re-read step)
  __device__ __forceinline__ void colsum_add(float (&cs)[8], bool valid, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (j == PER - 1 && UNITS % T && t + j * T >= UNITS) continue;
      const uint32_t w[4] = {r[j][0], r[j][1], r[j][2], r[j][3]};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cs[2 * e] += valid ? bf16_to_f32(w[e] & 0xFFFFu) : 0.f;
        cs[2 * e + 1] += valid ? bf16_to_f32(w[e] >> 16) : 0.f;
      }
    }
  }
};

template <int WM, int TN, bool CS, bool MASK>
__global__ __launch_bounds__(64 * WM) void k_gemm_wb(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, float* __restrict__ part,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int ktiles_per_split, int splits,
    float* __restrict__ cs_part) {
  constexpr int T = 64 * WM;
  constexpr int BM = 32 * WM, BN = 32 * TN;
  constexpr int AI = BK * BM, BI = BK * BN;  // bf16 elements per step image
  static_assert(WM * 32 * 32 * (int)sizeof(float) <= 2 * (AI + BI) * (int)sizeof(uint16_t),
                "epilogue tiles exceed the LDS images");
  static_assert(T % (BM / 8) == 0, "colsum rows per thread");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * (AI + BI)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BM - 1) / BM);
  const int ntiles = ntm * ntn;
  const int id = xcd_remap(blockIdx.x, ntiles * splits);  // a K slice's tiles share an XCD
  const int split = id / ntiles, tile = id - split * ntiles;
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;
  const int nk_total = (int)((K + BK - 1) / BK);
  const int kt_beg = split * ktiles_per_split;
  int kt_end = kt_beg + ktiles_per_split;
  if (kt_end > nk_total) kt_end = nk_total;
  const int ns = kt_end - kt_beg;  // >= 1 (the host's split plan)
  const int64_t kend = (int64_t)kt_end * BK < K ? (int64_t)kt_end * BK : K;

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  WbStage<BM, T, MASK> sa;
  WbStage<BN, T, MASK> sb;
  sa.init(A, lda, m0, M, tid);
  sb.init(B, ldb, n0, N, tid);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto kof = [&](int i) { return (int64_t)(kt_beg + (i < ns ? i : ns - 1)) * BK; };
  uint16_t* buf0 = lds;
  uint16_t* buf1 = lds + (AI + BI);
  auto compute = [&](const uint16_t* img) {
    const uint16_t* As = img;
    const uint16_t* Bs = img + AI;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 av = kmfrag<BM>(As, 32 * wave, ks, lane);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, kmfrag<BN>(Bs, 32 * b, ks, lane), acc[b],
                                                          0, 0, 0);
    }
  };
  auto load = [&](int i) {
    sa.load(kof(i), K - 1, tid);
    sb.load(kof(i), K - 1, tid);
  };
  // step i's registers -> image (a step past the last is stored, never read,
  // and adds nothing to the column sums)
  auto stage = [&](uint16_t* img, int i) {
    sa.mask(kof(i), kend, tid);
    sb.mask(kof(i), kend, tid);
    if constexpr (CS) sa.colsum_add(cs, i < ns, tid);
    sa.store(img, tid);
    sb.store(img + AI, tid);
  };
  load(0);
  stage(buf0, 0);
  load(1);
  __syncthreads();
  int i = 0;
  for (; i + 2 <= ns; i += 2) {
    stage(buf1, i + 1);
    load(i + 2);
    compute(buf0);
    __syncthreads();
    stage(buf0, i + 2);
    load(i + 3);
    compute(buf1);
    __syncthreads();
  }
  if (i < ns) compute(buf0);  // odd count: step i is in buf0
  __syncthreads();

  if constexpr (CS) {
    if (n0 == 0 && cs_part != nullptr) {  // block-uniform
      // thread t owns rows 8 (t % G) .. +7 of the tile: T / G threads per row
      // group, folded in a fixed order through LDS
      constexpr int G = BM / 8;
      float* red = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int e = 0; e < 8; ++e) red[e * T + tid] = cs[e];
      __syncthreads();
      if (tid < BM) {
        const int g = tid / 8, e = tid % 8;
        float v = 0.f;
        for (int q = 0; q < T / G; ++q) v += red[e * T + g + q * G];
        const int64_t m = m0 + tid;
        if (m < M) cs_part[(int64_t)split * M + m] = v;
      }
      __syncthreads();
    }
  }

  // partial tile, per 32 x 32 block through the wave's own 4 KB of LDS, 16-byte stores
  float* tw = reinterpret_cast<float*>(lds) + wave * 32 * 32;
  float* P = part + (int64_t)split * M * N;
  const int64_t mw = m0 + 32 * wave;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;  // block-uniform
#pragma unroll
    for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[b][r];
    wave_lds_sync();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, c4 = idx & 7;
      const int64_t m = mw + row, n = nb + 4 * c4;
      if (m < M && n < N)
        *reinterpret_cast<float4*>(P + m * N + n) =
            *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
    }
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------
// k_gemm_tw: the weight gradient part[split][m][n] = Σ_{k in split} A[k][m]
// B[k][n] on 256 x 256 tiles with both K-major operands DMA-staged
// (global_load_lds) into [64 k][256] images, two stages, the transposed LDS
// read (kmfrag) building the MFMA fragments; 8 waves as 4 (M) x 2 (N), each a
// 64 x 128 sub-tile -- k_gemm_tp's wave layout, with the k pairing of every
// other bf16 kernel.  One image k-row is 512 B; the kswz XOR of its 16-byte
// chunks is applied on the DMA source address and again by kmfrag.  A split's
// last step may run past K: its rows at or past K are zeroed in LDS once the
// DMA has landed.  CS: the column sums Σ_k A[k][m] (the bias gradient) are
// taken from the A images, k-rows ≡ tn (mod ntn) by the block of column tile
// tn, into cs_part[split * ntn + tn][m] (fixed order).
// ---------------------------------------------------------------------------
template <bool CS>
__global__ __launch_bounds__(512) void k_gemm_tw(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, float* __restrict__ part,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int steps_per_split, int splits,
    float* __restrict__ cs_part) {
  constexpr int TM = 256, KT = 64;
  constexpr int SI = KT * TM * 2;  // bytes per operand image per stage (32 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * SI];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + TM - 1) / TM);
  const int ntiles = (int)((M + TM - 1) / TM) * ntn;
  const int id = xcd_remap(blockIdx.x, ntiles * splits);  // a K slice's tiles share an XCD
  const int split = id / ntiles, tile = id - split * ntiles;
  const int tn = tile % ntn;
  const int64_t m0 = (int64_t)(tile / ntn) * TM, n0 = (int64_t)tn * TM;
  const int nk = (int)((K + KT - 1) / KT);
  const int s_beg = split * steps_per_split;
  const int ns = (s_beg + steps_per_split < nk ? s_beg + steps_per_split : nk) - s_beg;  // >= 1

  // DMA: wave w fills 1 KB pieces 4w .. 4w+3 (k-rows 2p, 2p+1) of both images;
  // lane L: k-row 2p + (L >> 5), slot L & 31 holds logical chunk slot ^ kswz
  const uint16_t* asrc[4];
  const uint16_t* bsrc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 2 * (4 * wave + q) + (lane >> 5);
    const int c = (lane & 31) ^ (kswz<TM>(k) >> 3);
    const int64_t am = m0 + 8 * c < M ? m0 + 8 * c : M - 8;
    const int64_t bn = n0 + 8 * c < N ? n0 + 8 * c : N - 8;
    asrc[q] = A + (int64_t)k * lda + am;
    bsrc[q] = B + (int64_t)k * ldb + bn;
  }
  const int kq0 = 2 * 4 * wave + (lane >> 5);  // k-row of piece q: kq0 + 2q
  auto stage = [&](int buf, int st) {
    const int64_t k0 = (int64_t)(s_beg + st) * KT;
    uint8_t* ia = lds + buf * 2 * SI + wave * 4096;
    uint8_t* ib = ia + SI;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // rows past K re-read row K - 1 (zeroed in LDS before use)
      const int64_t kk = k0 + kq0 + 2 * q < K ? k0 : K - 1 - (kq0 + 2 * q);
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(asrc[q] + kk * lda), (lds_as_ptr)(ia + 1024 * q), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_as_ptr)(bsrc[q] + kk * ldb), (lds_as_ptr)(ib + 1024 * q), 16, 0, 0);
    }
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int buf) {
    const uint16_t* ia = reinterpret_cast<const uint16_t*>(lds + buf * 2 * SI);
    const uint16_t* ib = reinterpret_cast<const uint16_t*>(lds + buf * 2 * SI + SI);
    bf16x8 fa[2][2], fb[2][4];
    auto read = [&](int q, bf16x8(&a)[2], bf16x8(&b)[4]) {
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = kmfrag<TM>(ia, 64 * wm + 32 * i, q, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = kmfrag<TM>(ib, 128 * wn + 32 * j, q, lane);
    };
    read(0, fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q & 1][i], fb[q & 1][j], acc[i][j], 0,
                                                               0, 0);
      if (q < 3) {
        read(q + 1, fa[(q + 1) & 1], fb[(q + 1) & 1]);
        interleave_mfma_reads<8, 12>();  // kmfrag: two transposed reads per fragment
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // CS: thread t sums logical chunk (t & 31) (8 columns m) over the k-rows
  // (t >> 5) + 16 j of every step that are ≡ tn (mod ntn)
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto colsum = [&](int buf) {
    const uint8_t* ia = lds + buf * 2 * SI;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = (tid >> 5) + 16 * j;
      if (k % ntn != tn) continue;
      const int slot = (tid & 31) ^ (kswz<TM>(k) >> 3);
      const u32x4 w = *reinterpret_cast<const u32x4*>(ia + k * (TM * 2) + 16 * slot);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cs[2 * e] += bf16_to_f32(w[e] & 0xFFFFu);
        cs[2 * e + 1] += bf16_to_f32(w[e] >> 16);
      }
    }
  };

  stage(0, 0);
  __syncthreads();
  int buf = 0;
  for (int st = 0; st < ns; ++st) {
    if (st + 1 < ns) stage(buf ^ 1, st + 1);
    const int64_t k0 = (int64_t)(s_beg + st) * KT;
    if (k0 + KT > K) {  // block-uniform: the last step of the last split
      const int kv = (int)(K - k0);
      uint8_t* ia = lds + buf * 2 * SI;
      for (int u = tid; u < 2 * KT * 32; u += 512) {  // 16-byte slots of both images
        const int img = u / (KT * 32), k = (u % (KT * 32)) / 32, sl = u % 32;
        if (k >= kv) *reinterpret_cast<u32x4*>(ia + img * SI + k * (TM * 2) + 16 * sl) = u32x4{0u, 0u, 0u, 0u};
      }
      __syncthreads();
    }
    if constexpr (CS) colsum(buf);
    compute(buf);
    __syncthreads();  // step st + 1 has landed; buf is free
    buf ^= 1;
  }

  if constexpr (CS) {
    if (cs_part != nullptr) {
      // fold the 16 k-row groups of each chunk in a fixed order through LDS
      float* red = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int e = 0; e < 8; ++e) red[e * 512 + tid] = cs[e];
      __syncthreads();
      if (tid < TM) {
        const int c = tid >> 3, e = tid & 7;  // column m0 + tid = chunk c, element e
        float v = 0.f;
        for (int g = 0; g < 16; ++g) v += red[e * 512 + 32 * g + c];
        const int64_t m = m0 + tid;
        if (m < M) cs_part[((int64_t)split * ntn + tn) * M + m] = v;
      }
      __syncthreads();
    }
  }

  // partial tile, per 32 x 32 block through the wave's own 4 KB of LDS, 16-byte stores
  float* tw = reinterpret_cast<float*>(lds) + wave * 32 * 32;
  float* P = part + (int64_t)split * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t mb = m0 + 64 * wm + 32 * i, nb = n0 + 128 * wn + 32 * j;
      if (mb >= M || nb >= N) continue;  // wave-uniform
#pragma unroll
      for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[i][j][r];
      wave_lds_sync();
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = it * 64 + lane;
        const int row = idx >> 3, c4 = idx & 7;
        const int64_t m = mb + row, n = nb + 4 * c4;
        if (m < M && n < N)
          *reinterpret_cast<float4*>(P + m * N + n) =
              *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
      }
      wave_lds_sync();
    }
  }
}

// --------------------------------------------------------------------------- host side
template <int WM, int WN, int TN, int D, bool MASK>
int launch_qb(int epi, const uint16_t* A, const uint16_t* Bp, uint16_t* C, int64_t M, int64_t N,
              int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc, const float* bias,
              const uint16_t* aux, int64_t ldaux, hipStream_t s) {
  constexpr int BM = 32 * WM, BN = 32 * TN * WN;
  const int64_t blocks = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  MOLCLR_REQUIRE(blocks < (1ll << 31), "gemm_bf16: too many tiles");
  const dim3 g((unsigned)blocks), b(64 * WM * WN);
#define MOLCLR_QB(EPV)                                                                            \
  molclr::launch_timed(molclr::kTimeGemm, k_gemm_qb<WM, WN, TN, D, EPV, MASK>, g, b, 0, s, A, Bp, C, M, \
                       N, K, lda, kp, npad, ldc, bias, aux, ldaux)
  switch (epi) {
    case MOLCLR_EPI_NONE: MOLCLR_QB(MOLCLR_EPI_NONE); return MOLCLR_OK;
    case MOLCLR_EPI_BIAS: MOLCLR_QB(MOLCLR_EPI_BIAS); return MOLCLR_OK;
    case MOLCLR_EPI_BIAS_RELU: MOLCLR_QB(MOLCLR_EPI_BIAS_RELU); return MOLCLR_OK;
    case MOLCLR_EPI_RELU_MASK: MOLCLR_QB(MOLCLR_EPI_RELU_MASK); return MOLCLR_OK;
    default:
      molclr::set_error("gemm_bf16: bad epilogue %d", epi);
      return MOLCLR_ERR_ARG;
  }
#undef MOLCLR_QB
}

template <bool RING>
int launch_tb(int epi, const uint16_t* A, const uint16_t* Bp, uint16_t* C, int64_t M, int64_t N,
              int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc, const float* bias,
              const uint16_t* aux, int64_t ldaux, hipStream_t s) {
  const int64_t blocks = ((M + 255) / 256) * ((N + 255) / 256);
  MOLCLR_REQUIRE(blocks < (1ll << 31), "gemm_bf16: too many tiles");
  const dim3 g((unsigned)blocks), b(512);
#define MOLCLR_TB(EPV)                                                                          \
  molclr::launch_timed(molclr::kTimeGemm, RING ? k_gemm_tc<EPV> : k_gemm_tb<EPV>, g, b, 0, s, A, Bp, \
                       C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux)
  switch (epi) {
    case MOLCLR_EPI_NONE: MOLCLR_TB(MOLCLR_EPI_NONE); return MOLCLR_OK;
    case MOLCLR_EPI_BIAS: MOLCLR_TB(MOLCLR_EPI_BIAS); return MOLCLR_OK;
    case MOLCLR_EPI_BIAS_RELU: MOLCLR_TB(MOLCLR_EPI_BIAS_RELU); return MOLCLR_OK;
    case MOLCLR_EPI_RELU_MASK: MOLCLR_TB(MOLCLR_EPI_RELU_MASK); return MOLCLR_OK;
    default:
      molclr::set_error("gemm_bf16: bad epilogue %d", epi);
      return MOLCLR_ERR_ARG;
  }
#undef MOLCLR_TB
}

// one persistent k_gemm_tp block per CU (160 KB of LDS: one block fits):
// molclr::cu_count()
using molclr::cu_count;

// k_gemm_tp's swapped-operand register epilogue: taken by the bias+ReLU
// product that writes ReLU bits (c5 lin1: 115.5 -> 98.9 us, the four ballots
// per row group gone); measured slower on the others (mask-bits consumer
// 97.8 -> 99.7, plain 71.6 -> 74.0 us: four times the cache lines per store
// instruction), which keep the LDS transpose.  MOLCLR_TP_SWAP=0 disables it.
static bool tp_swap() {
  static const bool on = [] {
    const char* e = getenv("MOLCLR_TP_SWAP");
    return !(e != nullptr && e[0] == '0');
  }();
  return on;
}

template <int NW>
int launch_tp(int epi, const uint16_t* A, const uint16_t* Bp, uint16_t* C, int64_t M, int64_t N,
              int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc, const float* bias,
              const uint16_t* aux, int64_t ldaux, hipStream_t s, uint32_t* bits_out = nullptr,
              const uint32_t* bits_in = nullptr) {
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  MOLCLR_REQUIRE(tiles < (1ll << 31) / 256, "gemm_bf16: too many tiles");
  // k_gemm_tp reads its bias columns as float4s from a column clamped to N - 4
  MOLCLR_REQUIRE(N >= 4 || (epi != MOLCLR_EPI_BIAS && epi != MOLCLR_EPI_BIAS_RELU),
                 "gemm_bf16: the persistent tile kernel needs N >= 4 with a bias (N = %lld)",
                 (long long)N);
  const int64_t cus = cu_count();
  const dim3 g((unsigned)(tiles < cus ? tiles : cus)), b(64 * NW);
  if (bits_out || bits_in) {
    MOLCLR_REQUIRE(bits_out ? epi == MOLCLR_EPI_BIAS_RELU : epi == MOLCLR_EPI_RELU_MASK,
                   "gemm_bf16: ReLU bits go out of a bias+ReLU product / into a ReLU-mask one");
    const bool sw = NW == 8 && tp_swap();  // 4 waves: 256 accumulators each, the swap spills
    if (bits_out)
      molclr::launch_timed(molclr::kTimeGemm,
                           sw ? k_gemm_tp<MOLCLR_EPI_BIAS_RELU, NW, true, NW == 8>
                              : k_gemm_tp<MOLCLR_EPI_BIAS_RELU, NW, true, false>,
                           g, b, 0, s, A, Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux,
                           bits_out, bits_in, M);
    else
      molclr::launch_timed(molclr::kTimeGemm, k_gemm_tp<MOLCLR_EPI_RELU_MASK, NW, true>, g, b, 0, s,
                           A, Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, bits_out,
                           bits_in, M);
    return MOLCLR_OK;
  }
  uint32_t* no_out = nullptr;
  const uint32_t* no_in = nullptr;
#define MOLCLR_TP(EPV)                                                                          \
  molclr::launch_timed(molclr::kTimeGemm, k_gemm_tp<EPV, NW>, g, b, 0, s, A, Bp, C, M, N, K, lda, kp, \
                       npad, ldc, bias, aux, ldaux, no_out, no_in, (int64_t)0)
  switch (epi) {
    case MOLCLR_EPI_NONE: MOLCLR_TP(MOLCLR_EPI_NONE); return MOLCLR_OK;
    case MOLCLR_EPI_BIAS: MOLCLR_TP(MOLCLR_EPI_BIAS); return MOLCLR_OK;
    case MOLCLR_EPI_BIAS_RELU: MOLCLR_TP(MOLCLR_EPI_BIAS_RELU); return MOLCLR_OK;
    case MOLCLR_EPI_RELU_MASK: MOLCLR_TP(MOLCLR_EPI_RELU_MASK); return MOLCLR_OK;
    default:
      molclr::set_error("gemm_bf16: bad epilogue %d", epi);
      return MOLCLR_ERR_ARG;
  }
#undef MOLCLR_TP
}

template <int WM, int WN, int TN, int D>
int launch_qb_m(bool mask, int epi, const uint16_t* A, const uint16_t* Bp, uint16_t* C, int64_t M,
                int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
                const float* bias, const uint16_t* aux, int64_t ldaux, hipStream_t s) {
  return mask ? launch_qb<WM, WN, TN, D, true>(epi, A, Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux,
                                            ldaux, s)
              : launch_qb<WM, WN, TN, D, false>(epi, A, Bp, C, M, N, K, lda, kp, npad, ldc, bias, aux,
                                             ldaux, s);
}

// k_gemm_qb tile shapes (molclr_gemm_bf16_impl) and A ring depths:
// 0 = 128 x 128 (4 waves, 4 steps of A in flight), 1 = 128 x 256 (4 waves, 2),
// 2 = 128 x 512 (8 waves, 2), 3 = 64 x 512 (8 waves, 4), 4 = 128 x 256 (8
// waves, 4), 5 = 128 x 128 (4 waves, 2); 6 = k_gemm_tb (256 x 256, LDS-DMA
// staging of both operands; K % 64 == 0, else 2), 7 = k_gemm_tc (256 x 256,
// four-stage LDS-DMA ring; K % 32 == 0, else 2), 8 = k_gemm_tp (k_gemm_tb
// persistent, epilogue overlapped with the next tile's staging; K % 64 == 0,
// else 2), 9 = k_gemm_tp with 4 waves of 128 x 128 (fewer LDS fragment reads
// per MFMA; K % 64 == 0, else 2)
constexpr int kQbImpls = 10;
// measured at the c5 shapes (55k rows, tools/gemm_bf16_bench.py); k_gemm_qb:
// 128 x 512 for N <= 512, 128 x 128 above
// the persistent k_gemm_tp whenever K % 64 == 0 (k_gemm_tb was 10-15 %
// faster than the best k_gemm_qb shape on all four c5 products; k_gemm_tp is
// 2-5 % faster than k_gemm_tb on the plain products and ~20 % on the ReLU-mask
// one; its 4-wave 128 x 128 form, 9, is 10-25 % slower), k_gemm_tc for K % 32 == 0
int qb_default(int64_t N, int64_t K) {
  if (K % 64 == 0 && N >= 4) return 8;
  if (K % 32 == 0) return 7;
  return N > 512 ? 5 : 2;
}

struct WbPlan {
  int splits, kps;
  int64_t ntiles;
};
// bm x bn tiles, `slots` co-resident blocks on the chip, >= 8 K steps per split
WbPlan wb_plan(int64_t M, int64_t N, int64_t K, int64_t bm, int64_t bn, int64_t slots) {
  WbPlan p;
  p.ntiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int64_t nk = (K + BK - 1) / BK;
  int64_t s = slots / p.ntiles;
  if (s > nk / 8) s = nk / 8;
  if (s < 1) s = 1;
  p.kps = (int)((nk + s - 1) / s);
  p.splits = (int)((nk + p.kps - 1) / p.kps);  // every split has >= 1 step
  return p;
}
// k_gemm_tw: 256 x 256 tiles over 64-row K steps, >= 4 steps per split
WbPlan tw_plan(int64_t M, int64_t N, int64_t K) {
  WbPlan p;
  p.ntiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int64_t nk = (K + 63) / 64;
  int64_t s = 256 / p.ntiles;
  if (s > nk / 4) s = nk / 4;
  if (s < 1) s = 1;
  p.kps = (int)((nk + s - 1) / s);
  p.splits = (int)((nk + p.kps - 1) / p.kps);
  return p;
}
// weight-gradient kernels (molclr_linear_wgrad_bf16_impl): k_gemm_wb with
// 0 = 128 x 128 (4 waves), 1 = 256 x 256 (8 waves), 2 = 128 x 256 (4 waves);
// 3 = k_gemm_tw (256 x 256, LDS-DMA staging)
constexpr int kWbImpls = 4;
WbPlan wb_plan_impl(int impl, int64_t M, int64_t N, int64_t K) {
  if (impl == 3) return tw_plan(M, N, K);
  if (impl == 1) return wb_plan(M, N, K, 256, 256, 256);
  if (impl == 2) return wb_plan(M, N, K, 128, 256, 256);
  return wb_plan(M, N, K, 128, 128, 512);
}
// k_gemm_tw for the large c5 products (2-10 % faster than k_gemm_wb's 256 x 256 shape)
int wb_default(int64_t M, int64_t N) { return M * N >= 512 * 512 ? 3 : 0; }

template <int WM, int TN, bool MASK>
void launch_wb(const WbPlan& p, bool cs, hipStream_t s, const uint16_t* dy, const uint16_t* x,
               float* part, int64_t M, int64_t N, int64_t K, int64_t ld_dy, int64_t ld_x,
               float* cs_part) {
  const dim3 g((unsigned)(p.ntiles * p.splits)), b(64 * WM);
  if (cs)
    molclr::launch_timed(molclr::kTimeGemm, k_gemm_wb<WM, TN, true, MASK>, g, b, 0, s, dy, x, part, M,
                         N, K, ld_dy, ld_x, p.kps, p.splits, cs_part);
  else
    molclr::launch_timed(molclr::kTimeGemm, k_gemm_wb<WM, TN, false, MASK>, g, b, 0, s, dy, x, part,
                         M, N, K, ld_dy, ld_x, p.kps, p.splits, cs_part);
}
template <int WM, int TN>
void launch_wb_m(bool mask, const WbPlan& p, bool cs, hipStream_t s, const uint16_t* dy,
                 const uint16_t* x, float* part, int64_t M, int64_t N, int64_t K, int64_t ld_dy,
                 int64_t ld_x, float* cs_part) {
  if (mask) launch_wb<WM, TN, true>(p, cs, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
  else launch_wb<WM, TN, false>(p, cs, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
}

}  // namespace

MOLCLR_API int molclr_gemm_bf16_impl(const uint16_t* A, const uint16_t* planes, uint16_t* C,
                                     int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldc,
                                     int epilogue, const float* bias, const uint16_t* aux,
                                     int64_t ldaux, molclr_stream_t stream, int impl) {
  MOLCLR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_bf16: negative size");
  MOLCLR_REQUIRE(impl >= -1 && impl < kQbImpls, "gemm_bf16: bad impl %d", impl);
  MOLCLR_REQUIRE(epilogue >= MOLCLR_EPI_NONE && epilogue <= MOLCLR_EPI_RELU_MASK,
                 "gemm_bf16: bad epilogue %d (no accumulate into bf16)", epilogue);
  MOLCLR_REQUIRE((epilogue != MOLCLR_EPI_BIAS && epilogue != MOLCLR_EPI_BIAS_RELU) || bias,
                 "gemm_bf16: bias epilogue needs bias");
  MOLCLR_REQUIRE(epilogue != MOLCLR_EPI_RELU_MASK || (aux && ldaux % 4 == 0),
                 "gemm_bf16: relu-mask epilogue needs aux with ldaux %% 4 == 0");
  MOLCLR_REQUIRE(K % 8 == 0 && lda % 8 == 0 && lda >= K,
                 "gemm_bf16: A needs K (%lld) and lda multiples of 8", (long long)K);
  MOLCLR_REQUIRE(ldc >= N && ldc % 4 == 0, "gemm_bf16: ldc must be >= N and a multiple of 4");
  if (M == 0 || N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(K > 0 && A && planes && C, "gemm_bf16: null operand or K == 0");
  // the planes of molclr_bplanes_make(B, N, K, ...): plane 0 = bf16(B), [Npad][Kp]
  const int64_t npad = (N + 127) / 128 * 128, kp = (K + BK - 1) / BK * BK;
  hipStream_t s = molclr::as_stream(stream);
  const bool mask = K % BK != 0;
  const int v = impl < 0 ? qb_default(N, K) : impl;
  int rc;
#define MOLCLR_QBM(WMV, WNV, TNV, DV)                                                            \
  launch_qb_m<WMV, WNV, TNV, DV>(mask, epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, \
                                 aux, ldaux, s)
  const int vv = (((v == 6 || v == 8 || v == 9) && K % 64 != 0) || (v == 7 && K % 32 != 0)) ? 2 : v;
  switch (vv) {
    case 9:
      rc = launch_tp<4>(epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, s);
      break;
    case 8:
      rc = launch_tp<8>(epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, s);
      break;
    case 6:
      rc = launch_tb<false>(epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, s);
      break;
    case 7:
      rc = launch_tb<true>(epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux, s);
      break;
    case 1: rc = MOLCLR_QBM(4, 1, 8, 2); break;
    case 2: rc = MOLCLR_QBM(4, 2, 8, 2); break;
    case 3: rc = MOLCLR_QBM(2, 4, 4, 4); break;
    case 4: rc = MOLCLR_QBM(4, 2, 4, 4); break;
    case 5: rc = MOLCLR_QBM(4, 1, 4, 2); break;
    default: rc = MOLCLR_QBM(4, 1, 4, 4); break;
  }
#undef MOLCLR_QBM
  if (rc) return rc;
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_gemm_bf16(const uint16_t* A, const uint16_t* planes, uint16_t* C, int64_t M,
                                int64_t N, int64_t K, int64_t lda, int64_t ldc, int epilogue,
                                const float* bias, const uint16_t* aux, int64_t ldaux,
                                molclr_stream_t stream) {
  return molclr_gemm_bf16_impl(A, planes, C, M, N, K, lda, ldc, epilogue, bias, aux, ldaux, stream,
                               -1);
}

MOLCLR_API int molclr_gemm_bf16_bits(const uint16_t* A, const uint16_t* planes, uint16_t* C,
                                     int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldc,
                                     int epilogue, const float* bias, uint32_t* bits_out,
                                     const uint32_t* bits_in, molclr_stream_t stream) {
  MOLCLR_REQUIRE(M >= 0 && N >= 0 && K > 0 && A && planes && C, "gemm_bf16_bits: bad operands");
  MOLCLR_REQUIRE((epilogue == MOLCLR_EPI_BIAS_RELU && bias && bits_out && !bits_in) ||
                     (epilogue == MOLCLR_EPI_RELU_MASK && bits_in && !bits_out),
                 "gemm_bf16_bits: bias+ReLU with bits_out, or ReLU-mask with bits_in");
  MOLCLR_REQUIRE(K % 64 == 0 && lda % 8 == 0 && lda >= K && ldc >= N && ldc % 4 == 0,
                 "gemm_bf16_bits: K %% 64 == 0, lda %% 8 == 0, ldc %% 4 == 0 (%lld, %lld, %lld)",
                 (long long)K, (long long)lda, (long long)ldc);
  if (M == 0 || N == 0) return MOLCLR_OK;
  const int64_t npad = (N + 127) / 128 * 128, kp = (K + BK - 1) / BK * BK;
  const int rc = launch_tp<8>(epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, nullptr, 0,
                              molclr::as_stream(stream), bits_out, bits_in);
  if (rc) return rc;
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API size_t molclr_linear_wgrad_bf16_workspace_bytes(int64_t rows, int64_t n_out,
                                                           int64_t n_in) {
  size_t need = 0;
  for (int impl = 0; impl < kWbImpls; ++impl) {
    const WbPlan p = wb_plan_impl(impl, n_out, n_in, rows);
    const int64_t cs_rows = impl == 3 ? (n_in + 255) / 256 : 1;  // tw: per column tile
    const size_t b = (size_t)p.splits * (n_out * n_in + cs_rows * n_out) * sizeof(float) + 256;
    need = b > need ? b : need;
  }
  return need;
}

MOLCLR_API int molclr_linear_wgrad_bf16_impl(const uint16_t* dy, const uint16_t* x, float* dW,
                                             float* db, int64_t rows, int64_t n_out, int64_t n_in,
                                             int64_t ld_dy, int64_t ld_x, int accumulate,
                                             void* workspace, size_t workspace_bytes,
                                             molclr_stream_t stream, int impl) {
  MOLCLR_REQUIRE(rows >= 0 && n_out > 0 && n_in > 0, "linear_wgrad_bf16: bad sizes");
  MOLCLR_REQUIRE(impl >= -1 && impl < kWbImpls, "linear_wgrad_bf16: bad impl %d", impl);
  MOLCLR_REQUIRE(dy && x && dW, "linear_wgrad_bf16: null pointer");
  MOLCLR_REQUIRE(n_out % 8 == 0 && n_in % 8 == 0 && ld_dy % 8 == 0 && ld_x % 8 == 0 &&
                     ld_dy >= n_out && ld_x >= n_in,
                 "linear_wgrad_bf16: n_out, n_in and the leading dimensions must be multiples of 8");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_linear_wgrad_bf16_workspace_bytes(rows, n_out, n_in));
  hipStream_t s = molclr::as_stream(stream);
  if (rows == 0) {
    if (!accumulate) {
      (void)molclr::zero_async(dW, (size_t)n_out * n_in * sizeof(float), s);
      if (db) (void)molclr::zero_async(db, (size_t)n_out * sizeof(float), s);
    }
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  const int64_t M = n_out, N = n_in, K = rows;
  const int v = impl < 0 ? wb_default(M, N) : impl;
  const WbPlan p = wb_plan_impl(v, M, N, K);
  float* part = static_cast<float*>(workspace);
  float* cs_part = db ? part + (size_t)p.splits * M * N : nullptr;
  const bool mask = K % BK != 0;
  if (v == 3) {
    const int ntn = (int)((N + 255) / 256);
    const dim3 g((unsigned)(p.ntiles * p.splits)), b(512);
    if (db)
      molclr::launch_timed(molclr::kTimeGemm, k_gemm_tw<true>, g, b, 0, s, dy, x, part, M, N, K, ld_dy,
                           ld_x, p.kps, p.splits, cs_part);
    else
      molclr::launch_timed(molclr::kTimeGemm, k_gemm_tw<false>, g, b, 0, s, dy, x, part, M, N, K, ld_dy,
                           ld_x, p.kps, p.splits, cs_part);
    molclr_splitk_reduce_none(part, p.splits, M, N, dW, N, accumulate, cs_part, p.splits * ntn, db, s);
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  if (v == 1) launch_wb_m<8, 8>(mask, p, db != nullptr, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
  else if (v == 2) launch_wb_m<4, 8>(mask, p, db != nullptr, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
  else launch_wb_m<4, 4>(mask, p, db != nullptr, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
  molclr_splitk_reduce_none(part, p.splits, M, N, dW, N, accumulate, cs_part, p.splits, db, s);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_linear_wgrad_bf16(const uint16_t* dy, const uint16_t* x, float* dW, float* db,
                                        int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy,
                                        int64_t ld_x, int accumulate, void* workspace,
                                        size_t workspace_bytes, molclr_stream_t stream) {
  return molclr_linear_wgrad_bf16_impl(dy, x, dW, db, rows, n_out, n_in, ld_dy, ld_x, accumulate,
                                       workspace, workspace_bytes, stream, -1);
}
