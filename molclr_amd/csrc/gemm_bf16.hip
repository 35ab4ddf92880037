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

// LDS written by a wave and read back by other lanes of the SAME wave: wait
// for the wave's LDS operations, no workgroup barrier
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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
// 32 a lane loads the 16 consecutive k (32 bytes) of its row it needs (lane
// half h: k0 + 16h .. +15; MFMA step s uses k0 + 16h + 8s .. +7, and the B
// fragment is image chunk 2h + s, the same k).  With BN = N every A row is
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
    const int64_t k = (int64_t)kstep(i) * BK + 16 * lh;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      int64_t kc = k + 8 * c;
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
      for (int b = 0; b < TN; ++b) f[s][b] = xfrag(Bs, wn * WC + 32 * b + li, 2 * lh + s);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 as = a[s];
      if constexpr (MASK) {
        const u32x4 z = {0u, 0u, 0u, 0u};
        if ((int64_t)i * BK + 16 * lh + 8 * s >= K) as = z;
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
// waves, 4), 5 = 128 x 128 (4 waves, 2)
constexpr int kQbImpls = 6;
// measured at the c5 shapes (55k rows, tools/gemm_bf16_bench.py): 128 x 512
// for N <= 512, 128 x 128 above
int qb_default(int64_t N) { return N > 512 ? 5 : 2; }

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
// k_gemm_wb tile shapes (molclr_linear_wgrad_bf16_impl): 0 = 128 x 128 (4
// waves), 1 = 256 x 256 (8 waves), 2 = 128 x 256 (4 waves)
constexpr int kWbImpls = 3;
WbPlan wb_plan_impl(int impl, int64_t M, int64_t N, int64_t K) {
  if (impl == 1) return wb_plan(M, N, K, 256, 256, 256);
  if (impl == 2) return wb_plan(M, N, K, 128, 256, 256);
  return wb_plan(M, N, K, 128, 128, 512);
}
int wb_default(int64_t M, int64_t N) { return M * N >= 512 * 512 ? 1 : 0; }

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
  const int v = impl < 0 ? qb_default(N) : impl;
  int rc;
#define MOLCLR_QBM(WMV, WNV, TNV, DV)                                                            \
  launch_qb_m<WMV, WNV, TNV, DV>(mask, epilogue, A, planes, C, M, N, K, lda, kp, npad, ldc, bias, \
                                 aux, ldaux, s)
  switch (v) {
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

MOLCLR_API size_t molclr_linear_wgrad_bf16_workspace_bytes(int64_t rows, int64_t n_out,
                                                           int64_t n_in) {
  size_t need = 0;
  for (int impl = 0; impl < kWbImpls; ++impl) {
    const WbPlan p = wb_plan_impl(impl, n_out, n_in, rows);
    const size_t b = (size_t)p.splits * (n_out * n_in + n_out) * sizeof(float) + 256;
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
      (void)hipMemsetAsync(dW, 0, (size_t)n_out * n_in * sizeof(float), s);
      if (db) (void)hipMemsetAsync(db, 0, (size_t)n_out * sizeof(float), s);
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
  if (v == 1) launch_wb_m<8, 8>(mask, p, db != nullptr, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
  else if (v == 2) launch_wb_m<4, 8>(mask, p, db != nullptr, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
  else launch_wb_m<4, 4>(mask, p, db != nullptr, s, dy, x, part, M, N, K, ld_dy, ld_x, cs_part);
  molclr_splitk_reduce_none(part, p.splits, M, N, dW, N, accumulate, cs_part, db, s);
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
