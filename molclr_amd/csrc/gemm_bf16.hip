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

namespace {

using namespace molclr;

// ---------------------------------------------------------------------------
// k_gemm_qb: 4 waves stacked along M (32 rows each, 128 per block) over BN =
// 32 TN columns.  A goes global -> registers -> MFMA operand: a lane loads the
// 16 consecutive k (32 bytes) of its row it needs for one K step (lane half h:
// k0 + 16h .. +15; MFMA step s uses k0 + 16h + 8s .. +7, and the B fragment is
// image chunk 2h + s, the same k).  B (the weight plane) is staged per K step
// into a [BN][32] bf16 image (xoff swizzle), double-buffered, one barrier per
// K step.  The epilogue goes through the wave's 4 KB of LDS so rows leave as
// 8-byte (4 x bf16) pieces.
// ---------------------------------------------------------------------------
constexpr int kQbWaves = 4;
constexpr int kQbBM = 32 * kQbWaves;

template <int BN, int T>
struct QbStageB {
  static constexpr int UNITS = BN * 4;  // 16-byte chunks per K step
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
      if (UNITS % T && t + j * T >= UNITS) continue;
      r[j] = *reinterpret_cast<const u32x4*>(Bp + goff[j] + k0);
    }
  }
  __device__ __forceinline__ void store(uint16_t* __restrict__ img, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (UNITS % T && u >= UNITS) continue;
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

template <int TN, int EPI>
__global__ __launch_bounds__(64 * kQbWaves) __attribute__((amdgpu_waves_per_eu(2))) void k_gemm_qb(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bp, uint16_t* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const uint16_t* __restrict__ aux, int64_t ldaux) {
  constexpr int T = 64 * kQbWaves;
  constexpr int BN = 32 * TN;
  constexpr int BI = BN * XK;  // bf16 elements per B image
  static_assert(kQbWaves * 32 * 32 * (int)sizeof(float) <= 2 * BI * (int)sizeof(uint16_t),
                "epilogue tiles exceed the LDS images");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BI];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wm = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + kQbBM - 1) / kQbBM);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);  // a row slab's column tiles share an XCD
  const int64_t m0 = (int64_t)(tile / ntn) * kQbBM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;

  int64_t arow_i = m0 + 32 * wm + li;
  arow_i = arow_i < M ? arow_i : M - 1;
  const uint16_t* __restrict__ arow = A + arow_i * lda + 16 * lh;
  // this lane's 16 k of K step k0 (K % 8 == 0: an 8-element chunk is all in or out)
  auto load_a = [&](int64_t k0, u32x4(&r)[2]) {
    const uint16_t* q = arow + k0;
    if (k0 + BK <= K) {
      r[0] = *reinterpret_cast<const u32x4*>(q);
      r[1] = *reinterpret_cast<const u32x4*>(q + 8);
    } else {
      const u32x4 z = {0u, 0u, 0u, 0u};
      r[0] = k0 + 16 * lh < K ? *reinterpret_cast<const u32x4*>(q) : z;
      r[1] = k0 + 16 * lh + 8 < K ? *reinterpret_cast<const u32x4*>(q + 8) : z;
    }
  };

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  auto compute = [&](const uint16_t* Bs, const u32x4(&a)[2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 av = __builtin_bit_cast(bf16x8, a[s]);
      const int ch = 2 * lh + s;
#pragma unroll
      for (int b = 0; b < TN; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, xfrag(Bs, 32 * b + li, ch), acc[b],
                                                          0, 0, 0);
    }
  };

  QbStageB<BN, T> sb;
  sb.init(n0, npad, kp, tid);
  uint16_t* buf0 = lds;
  uint16_t* buf1 = lds + BI;
  const int ns = (int)((K + BK - 1) / BK);
  auto kof = [&](int i) { return (int64_t)i * BK; };
  u32x4 a0[2], a1[2];
  if (ns > 0) {
    sb.load(Bp, kof(0), tid);
    load_a(kof(0), a0);
    sb.store(buf0, tid);
  }
  if (ns > 1) {
    sb.load(Bp, kof(1), tid);
    load_a(kof(1), a1);
  }
  __syncthreads();
  // top of an iteration (i even): buf0 holds B(i), sb holds B(i+1) in flight,
  // a0 = A(i), a1 = A(i+1) in flight; B(i+1) is written right after the
  // barrier into the buffer the previous step read.
  int i = 0;
  for (; i + 2 <= ns; i += 2) {
    if (i + 1 < ns) sb.store(buf1, tid);
    if (i + 2 < ns) sb.load(Bp, kof(i + 2), tid);
    compute(buf0, a0);
    if (i + 2 < ns) load_a(kof(i + 2), a0);
    __syncthreads();
    if (i + 2 < ns) {
      sb.store(buf0, tid);
      if (i + 3 < ns) sb.load(Bp, kof(i + 3), tid);
    }
    compute(buf1, a1);
    if (i + 3 < ns) load_a(kof(i + 3), a1);
    __syncthreads();
  }
  if (i < ns) {
    compute(buf0, a0);
    __syncthreads();  // the images are reused below
  }

  float* tw = reinterpret_cast<float*>(lds) + wm * 32 * 32;
  const int64_t mw = m0 + 32 * wm;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;  // block-uniform
#pragma unroll
    for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[b][r];
    __syncthreads();
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
    __syncthreads();  // the wave's tile is rewritten by the next block
  }
}

// ---------------------------------------------------------------------------
// k_gemm_wb: part[split][m][n] = Σ_{k in split} A[k][m] B[k][n] (A = dY, B = X,
// both row-major [rows][*] bf16, i.e. K-major operands), 4 waves stacked along
// M (32 rows each, BM = 128) over BN = 32 TN columns.  Both operands are staged
// as K-major [k][rows] bf16 images (kswz XOR) read with the transposed LDS read
// (kmfrag); staging is a 16-byte copy of 8 consecutive rows at one k.  CS: the
// column sums Σ_k A[k][m] (the bias gradient) of the staged A tiles go to
// cs_part[split][m].  Double-buffered, one barrier per K step.
// ---------------------------------------------------------------------------
constexpr int kWbBM = 128;

template <int ROWS, int T>
struct WbStage {
  static constexpr int UNITS = BK * (ROWS / 8);  // (k, 8-row group) per K step
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
      p[j] = src + (int64_t)k * ld + (gr < rows ? gr : rows - 8);
    }
  }
  __device__ __forceinline__ void load(int64_t k0, int64_t K, int t) {
    const int64_t base = k0 * ld;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (UNITS % T && u >= UNITS) continue;
      const bool in = k0 + u / (ROWS / 8) < K;
      const u32x4 z = {0u, 0u, 0u, 0u};
      r[j] = in ? *reinterpret_cast<const u32x4*>(p[j] + base) : z;
    }
  }
  __device__ __forceinline__ void store(uint16_t* __restrict__ img, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (UNITS % T && u >= UNITS) continue;
      const int rb = u % (ROWS / 8), k = u / (ROWS / 8);
      *reinterpret_cast<u32x4*>(img + k * ROWS + ((8 * rb) ^ kswz<ROWS>(k))) = r[j];
    }
  }
  // column sums over k of this thread's 8 rows (fixed rows per thread: T is a
  // multiple of ROWS / 8)
  __device__ __forceinline__ void colsum_add(float (&cs)[8], int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (UNITS % T && t + j * T >= UNITS) continue;
      const uint32_t w[4] = {r[j][0], r[j][1], r[j][2], r[j][3]};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cs[2 * e] += bf16_to_f32(w[e] & 0xFFFFu);
        cs[2 * e + 1] += bf16_to_f32(w[e] >> 16);
      }
    }
  }
};

template <int TN, bool CS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_gemm_wb(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, float* __restrict__ part,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int ktiles_per_split, int splits,
    float* __restrict__ cs_part) {
  constexpr int T = 256;
  constexpr int BM = kWbBM, BN = 32 * TN;
  constexpr int AI = BK * BM, BI = BK * BN;  // bf16 elements per image
  static_assert(4 * 32 * 32 * (int)sizeof(float) <= 2 * (AI + BI) * (int)sizeof(uint16_t),
                "epilogue tiles exceed the LDS images");
  static_assert(T % (BM / 8) == 0, "colsum rows per thread");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * (AI + BI)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
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
  const int ns = kt_end > kt_beg ? kt_end - kt_beg : 0;

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  WbStage<BM, T> sa;
  WbStage<BN, T> sb;
  sa.init(A, lda, m0, M, tid);
  sb.init(B, ldb, n0, N, tid);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto kof = [&](int i) { return (int64_t)(kt_beg + i) * BK; };
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
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, kmfrag<BN>(Bs, 32 * b, ks, lane),
                                                          acc[b], 0, 0, 0);
    }
  };
  auto stage = [&](uint16_t* img) {
    if constexpr (CS) sa.colsum_add(cs, tid);
    sa.store(img, tid);
    sb.store(img + AI, tid);
  };
  if (ns > 0) {
    sa.load(kof(0), K, tid);
    sb.load(kof(0), K, tid);
    stage(buf0);
    if (ns > 1) {
      sa.load(kof(1), K, tid);
      sb.load(kof(1), K, tid);
    }
  }
  __syncthreads();
  int i = 0;
  for (; i + 2 <= ns; i += 2) {
    if (i + 1 < ns) stage(buf1);
    if (i + 2 < ns) {
      sa.load(kof(i + 2), K, tid);
      sb.load(kof(i + 2), K, tid);
    }
    compute(buf0);
    __syncthreads();
    if (i + 2 < ns) {
      stage(buf0);
      if (i + 3 < ns) {
        sa.load(kof(i + 3), K, tid);
        sb.load(kof(i + 3), K, tid);
      }
    }
    compute(buf1);
    __syncthreads();
  }
  if (i < ns) {
    compute(buf0);
    __syncthreads();
  }

  if constexpr (CS) {
    if (n0 == 0 && cs_part != nullptr) {  // block-uniform
      // thread t owns rows 8 (t % 16) .. +7 of the tile: 16 threads per row
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

  // partial tile, per 32 x 32 block through the wave's 4 KB of LDS, 16-byte stores
  float* tw = reinterpret_cast<float*>(lds) + wave * 32 * 32;
  float* P = part + (int64_t)split * M * N;
  const int64_t mw = m0 + 32 * wave;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;  // block-uniform
#pragma unroll
    for (int r = 0; r < 16; ++r) tw[acc_row(r, lh) * 32 + li] = acc[b][r];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, c4 = idx & 7;
      const int64_t m = mw + row, n = nb + 4 * c4;
      if (m < M && n < N)
        *reinterpret_cast<float4*>(P + m * N + n) =
            *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
    }
    __syncthreads();
  }
}

// column-tile width of k_gemm_qb: 256 for wide outputs, 128 otherwise
int qb_tn(int64_t N) { return N >= 1024 ? 8 : 4; }

template <int TN>
int launch_qb(int epi, const uint16_t* A, const uint16_t* Bp, uint16_t* C, int64_t M, int64_t N,
              int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc, const float* bias,
              const uint16_t* aux, int64_t ldaux, hipStream_t s) {
  const int64_t blocks = ((M + kQbBM - 1) / kQbBM) * ((N + 32 * TN - 1) / (32 * TN));
  MOLCLR_REQUIRE(blocks < (1ll << 31), "gemm_bf16: too many tiles");
  const dim3 g((unsigned)blocks), b(64 * kQbWaves);
  switch (epi) {
    case MOLCLR_EPI_NONE:
      molclr::launch_timed(molclr::kTimeGemm, k_gemm_qb<TN, MOLCLR_EPI_NONE>, g, b, 0, s, A, Bp, C,
                           M, N, K, lda, kp, npad, ldc, bias, aux, ldaux);
      return MOLCLR_OK;
    case MOLCLR_EPI_BIAS:
      molclr::launch_timed(molclr::kTimeGemm, k_gemm_qb<TN, MOLCLR_EPI_BIAS>, g, b, 0, s, A, Bp, C,
                           M, N, K, lda, kp, npad, ldc, bias, aux, ldaux);
      return MOLCLR_OK;
    case MOLCLR_EPI_BIAS_RELU:
      molclr::launch_timed(molclr::kTimeGemm, k_gemm_qb<TN, MOLCLR_EPI_BIAS_RELU>, g, b, 0, s, A, Bp,
                           C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux);
      return MOLCLR_OK;
    case MOLCLR_EPI_RELU_MASK:
      molclr::launch_timed(molclr::kTimeGemm, k_gemm_qb<TN, MOLCLR_EPI_RELU_MASK>, g, b, 0, s, A, Bp,
                           C, M, N, K, lda, kp, npad, ldc, bias, aux, ldaux);
      return MOLCLR_OK;
    default:
      molclr::set_error("gemm_bf16: bad epilogue %d", epi);
      return MOLCLR_ERR_ARG;
  }
}

struct WbPlan {
  int tn, splits, kps;
  int64_t ntiles;
};
WbPlan wb_plan(int64_t M, int64_t N, int64_t K) {
  WbPlan p;
  p.tn = 4;
  p.ntiles = ((M + kWbBM - 1) / kWbBM) * ((N + 32 * p.tn - 1) / (32 * p.tn));
  const int64_t nk = (K + BK - 1) / BK;
  int64_t s = 512 / p.ntiles;  // ~two blocks per CU
  if (s > nk / 8) s = nk / 8;  // >= 8 K steps per split
  if (s < 1) s = 1;
  p.kps = (int)((nk + s - 1) / s);
  p.splits = (int)((nk + p.kps - 1) / p.kps);
  return p;
}

}  // namespace

MOLCLR_API int molclr_gemm_bf16(const uint16_t* A, const uint16_t* planes, uint16_t* C, int64_t M,
                                int64_t N, int64_t K, int64_t lda, int64_t ldc, int epilogue,
                                const float* bias, const uint16_t* aux, int64_t ldaux,
                                molclr_stream_t stream) {
  MOLCLR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_bf16: negative size");
  MOLCLR_REQUIRE(epilogue >= MOLCLR_EPI_NONE && epilogue <= MOLCLR_EPI_RELU_MASK,
                 "gemm_bf16: bad epilogue %d (no accumulate into bf16)", epilogue);
  MOLCLR_REQUIRE((epilogue != MOLCLR_EPI_BIAS && epilogue != MOLCLR_EPI_BIAS_RELU) || bias,
                 "gemm_bf16: bias epilogue needs bias");
  MOLCLR_REQUIRE(epilogue != MOLCLR_EPI_RELU_MASK || (aux && ldaux % 4 == 0),
                 "gemm_bf16: relu-mask epilogue needs aux with ldaux % 4 == 0");
  MOLCLR_REQUIRE(K % 8 == 0 && lda % 8 == 0 && lda >= K,
                 "gemm_bf16: A needs K (%lld) and lda multiples of 8", (long long)K);
  MOLCLR_REQUIRE(ldc >= N && ldc % 4 == 0, "gemm_bf16: ldc must be >= N and a multiple of 4");
  if (M == 0 || N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(K > 0 && A && planes && C, "gemm_bf16: null operand or K == 0");
  // the planes of molclr_bplanes_make(B, N, K, ...): plane 0 = bf16(B), [Npad][Kp]
  const int64_t npad = (N + 127) / 128 * 128, kp = (K + BK - 1) / BK * BK;
  hipStream_t s = molclr::as_stream(stream);
  const int rc = qb_tn(N) == 8
                     ? launch_qb<8>(epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, aux,
                                    ldaux, s)
                     : launch_qb<4>(epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, aux,
                                    ldaux, s);
  if (rc) return rc;
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API size_t molclr_linear_wgrad_bf16_workspace_bytes(int64_t rows, int64_t n_out,
                                                           int64_t n_in) {
  const WbPlan p = wb_plan(n_out, n_in, rows);
  return (size_t)p.splits * (n_out * n_in + n_out) * sizeof(float) + 256;
}

MOLCLR_API int molclr_linear_wgrad_bf16(const uint16_t* dy, const uint16_t* x, float* dW, float* db,
                                        int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy,
                                        int64_t ld_x, int accumulate, void* workspace,
                                        size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_REQUIRE(rows >= 0 && n_out > 0 && n_in > 0, "linear_wgrad_bf16: bad sizes");
  MOLCLR_REQUIRE(dy && x && dW, "linear_wgrad_bf16: null pointer");
  MOLCLR_REQUIRE(n_out % 8 == 0 && n_in % 8 == 0 && ld_dy % 8 == 0 && ld_x % 8 == 0 &&
                     ld_dy >= n_out && ld_x >= n_in,
                 "linear_wgrad_bf16: n_out, n_in and the leading dimensions must be multiples of 8");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_linear_wgrad_bf16_workspace_bytes(rows, n_out, n_in));
  hipStream_t s = molclr::as_stream(stream);
  if (rows == 0) {
    if (!accumulate) {
      (void)hipMemsetAsync(dW, 0, (size_t)n_out * n_in * sizeof(float), s);
      if (db) (void)hipMemsetAsync(db, 0, (size_t)n_out * sizeof(float), s);
    }
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  const int64_t M = n_out, N = n_in, K = rows;
  const WbPlan p = wb_plan(M, N, K);
  float* part = static_cast<float*>(workspace);
  float* cs_part = db ? part + (size_t)p.splits * M * N : nullptr;
  const dim3 g((unsigned)(p.ntiles * p.splits)), b(256);
  if (db)
    molclr::launch_timed(molclr::kTimeGemm, k_gemm_wb<4, true>, g, b, 0, s, dy, x, part, M, N, K,
                         ld_dy, ld_x, p.kps, p.splits, cs_part);
  else
    molclr::launch_timed(molclr::kTimeGemm, k_gemm_wb<4, false>, g, b, 0, s, dy, x, part, M, N, K,
                         ld_dy, ld_x, p.kps, p.splits, cs_part);
  molclr_splitk_reduce_none(part, p.splits, M, N, dW, N, accumulate, cs_part, db, s);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
