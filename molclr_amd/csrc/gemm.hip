// FP32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32).
//
// Serves every dense product of the pre-training step:
//   GIN MLP  Linear(D,2D) -> ReLU -> Linear(2D,D)   models/ginet_molclr.py:19-23
//   heads    feat_lin / out_lin                     models/ginet_molclr.py:90-96
//   GCN      x @ W                                  models/gcn_molclr.py:76
// and their backward products (dX = dY W, dW = dY^T X).  The f32 MFMA is an
// exact f32 FMA chain (no TF32-style rounding), so results stay within the
// fp32 tolerance of the reference CPU path.
//
// Structure: a workgroup of WM x WN waves owns a BM x BN output tile
// (BM = WM*TM*32, BN = WN*TN*32); each wave owns TM x TN 32x32 MFMA tiles.
// A and B K-slices (BK = 32) are staged in LDS as [row][k] images with a
// 36-float row pitch; the next slice is prefetched into registers while the
// current one is consumed.  The K order inside a slice is permuted so that a
// lane half h consumes k = 16h .. 16h+15: one ds_read_b128 then feeds four
// MFMAs and the image stays conflict-free (pitch 36 -> distinct 4-bank groups
// across a 16-lane read group).  A K-major operand (X^T / dY^T of a weight
// gradient) is transposed while staging: 4 coalesced scalar loads per lane
// (64 consecutive m per wave instruction) then one ds_write_b128.
//
// Workgroups are remapped so that the tiles sharing an A row-slab land on the
// same XCD (blocks b and b+8 share an L2): the A slab is then read from HBM
// once per XCD rather than once per column tile.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDK = BK + 4;  // [row][k] image pitch (floats): conflict-free ds_read_b128
constexpr int RPAD = 4;      // [k][row] image pad (floats)

// One operand's K-slice in LDS.
//  K contiguous in memory ([rows][K]): image [row][LDK]; a lane reads 4
//    consecutive k of one row with one ds_read_b128.
//  rows contiguous ([K][rows], e.g. dY^T of a weight gradient): image
//    [k][ROWS+RPAD]; a lane reads one element per k with ds_read_b32
//    (32 consecutive rows per half-wave: conflict-free).
// Both are filled from float4 global loads (16 B per lane, coalesced).
template <bool KMAJOR, int ROWS>
struct Image {
  static constexpr int FLOATS = KMAJOR ? BK * (ROWS + RPAD) : ROWS * LDK;
};

template <bool KMAJOR, int ROWS, int T>
struct Stager {
  static constexpr int ITEMS = ROWS * BK / 4;  // float4 items per slice
  static constexpr int PER_THREAD = (ITEMS + T - 1) / T;
  float4 r[PER_THREAD];
  uint32_t ok;  // bit j: item j in range (applied at store time, so the loads
                // are never waited on until the LDS write that consumes them)

  // Branch-free: out-of-range items load from a clamped (valid) address.
  __device__ __forceinline__ void load(const float* __restrict__ src, int64_t ld, int64_t row0,
                                       int64_t rows, int64_t k0, int64_t K, int tid, bool vec) {
    ok = 0;
#pragma unroll
    for (int j = 0; j < PER_THREAD; ++j) {
      const int idx = tid + j * T;
      if (!KMAJOR) {
        const int row = idx / (BK / 4), k4 = idx % (BK / 4);
        const int64_t gr = row0 + row, gk = k0 + 4 * k4;
        const bool in = idx < ITEMS && gr < rows && gk < K;
        const int64_t cr = gr < rows ? gr : rows - 1, ck = gk < K ? gk : 0;
        r[j] = *reinterpret_cast<const float4*>(src + cr * ld + ck);
        ok |= (uint32_t)in << j;
      } else {
        const int k = idx / (ROWS / 4), r4 = idx % (ROWS / 4);
        const int64_t gk = k0 + k, gr = row0 + 4 * r4;
        const bool kin = idx < ITEMS && gk < K;
        const int64_t ck = gk < K ? gk : K - 1;
        if (vec) {
          const bool in = kin && gr + 3 < rows;
          const int64_t cr = gr + 3 < rows ? gr : 0;
          r[j] = *reinterpret_cast<const float4*>(src + ck * ld + cr);
          ok |= (uint32_t)in << j;
        } else {  // unaligned rows: per-element guards (rare path)
          const float* p = src + ck * ld;
          float4 v;
          v.x = (kin && gr + 0 < rows) ? p[gr + 0 < rows ? gr + 0 : 0] : 0.f;
          v.y = (kin && gr + 1 < rows) ? p[gr + 1 < rows ? gr + 1 : 0] : 0.f;
          v.z = (kin && gr + 2 < rows) ? p[gr + 2 < rows ? gr + 2 : 0] : 0.f;
          v.w = (kin && gr + 3 < rows) ? p[gr + 3 < rows ? gr + 3 : 0] : 0.f;
          r[j] = v;
          ok |= 1u << j;
        }
      }
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ lds, int tid) const {
#pragma unroll
    for (int j = 0; j < PER_THREAD; ++j) {
      const int idx = tid + j * T;
      if (idx < ITEMS) {
        const float4 v = ((ok >> j) & 1u) ? r[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        if (!KMAJOR) {
          const int row = idx / (BK / 4), k4 = idx % (BK / 4);
          *reinterpret_cast<float4*>(lds + row * LDK + 4 * k4) = v;
        } else {
          const int k = idx / (ROWS / 4), r4 = idx % (ROWS / 4);
          *reinterpret_cast<float4*>(lds + k * (ROWS + RPAD) + 4 * r4) = v;
        }
      }
    }
  }
};

// Fragment for MFMA k-steps 4q..4q+3 of lane half lh (k = 16 lh + 4q + j), row `row`.
template <bool KMAJOR, int ROWS>
__device__ __forceinline__ float4 frag(const float* __restrict__ lds, int row, int lh, int q) {
  if (!KMAJOR) return *reinterpret_cast<const float4*>(lds + row * LDK + lh * 16 + 4 * q);
  const float* p = lds + (lh * 16 + 4 * q) * (ROWS + RPAD) + row;
  return make_float4(p[0], p[ROWS + RPAD], p[2 * (ROWS + RPAD)], p[3 * (ROWS + RPAD)]);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: XCD x (= bid % 8) receives a contiguous range of tile ids
  int q = nwg / 8, r = nwg % 8;
  int x = bid % 8, pos = bid / 8;
  int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + pos;
}

template <int WM, int WN, int TM, int TN, bool AK, bool BKM, int EPI, bool SPLIT>
__global__ __launch_bounds__(WM* WN * 64) void k_gemm_f32(
    const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C, int64_t M,
    int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, const float* __restrict__ bias,
    const float* __restrict__ aux, int64_t ldaux, int ktiles_per_split, int accumulate) {
  constexpr int T = WM * WN * 64;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int AF = Image<AK, BM>::FLOATS, BF = Image<BKM, BN>::FLOATS;
  __shared__ __attribute__((aligned(16))) float lds[2 * (AF + BF)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, lh = lane >> 5;

  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BM - 1) / BM);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;

  const int nk_total = (int)((K + BK - 1) / BK);
  const int kt_beg = SPLIT ? blockIdx.y * ktiles_per_split : 0;
  int kt_end = SPLIT ? kt_beg + ktiles_per_split : nk_total;
  if (kt_end > nk_total) kt_end = nk_total;
  const bool avec = (lda % 4 == 0) && (M % 4 == 0);
  const bool bvec = (ldb % 4 == 0) && (N % 4 == 0);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // 3-stage pipeline: the global loads of slice k+2 are issued before slice k
  // is computed and written to LDS after slice k+1 is computed, so every load
  // has two compute phases to land; LDS is double-buffered (one barrier per
  // slice).  Two named register sets (no runtime-indexed arrays).
  Stager<AK, BM, T> sa0, sa1;
  Stager<BKM, BN, T> sb0, sb1;
  float* buf0 = lds;
  float* buf1 = lds + (AF + BF);

  auto compute = [&](const float* As) {
    const float* Bs = As + AF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = frag<AK, BM>(As, wm * TM * 32 + a * 32 + li, lh, q);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = frag<BKM, BN>(Bs, wn * TN * 32 + b * 32 + li, lh, q);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].x, bf[b].x, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].y, bf[b].y, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].z, bf[b].z, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].w, bf[b].w, acc[a][b], 0, 0, 0);
        }
    }
  };

  const int nsteps = kt_end - kt_beg;
  if (nsteps > 0) {
    sa0.load(A, lda, m0, M, (int64_t)kt_beg * BK, K, tid, avec);
    sb0.load(B, ldb, n0, N, (int64_t)kt_beg * BK, K, tid, bvec);
    if (nsteps > 1) {
      sa1.load(A, lda, m0, M, (int64_t)(kt_beg + 1) * BK, K, tid, avec);
      sb1.load(B, ldb, n0, N, (int64_t)(kt_beg + 1) * BK, K, tid, bvec);
    }
    sa0.store(buf0, tid);
    sb0.store(buf0 + AF, tid);
    __syncthreads();
  }
  // Straight-line body: loads past the last slice re-read a clamped (valid)
  // slice and their LDS writes land in the buffer nobody reads any more.
  int i = 0;
  for (; i + 2 <= nsteps; i += 2) {
    // slice i in buf0; slice i+1 in set 1; set 0 free
    sa0.load(A, lda, m0, M, (int64_t)(kt_beg + i + 2) * BK, K, tid, avec);
    sb0.load(B, ldb, n0, N, (int64_t)(kt_beg + i + 2) * BK, K, tid, bvec);
    compute(buf0);
    sa1.store(buf1, tid);
    sb1.store(buf1 + AF, tid);
    __syncthreads();
    // slice i+1 in buf1; slice i+2 in set 0; set 1 free
    sa1.load(A, lda, m0, M, (int64_t)(kt_beg + i + 3) * BK, K, tid, avec);
    sb1.load(B, ldb, n0, N, (int64_t)(kt_beg + i + 3) * BK, K, tid, bvec);
    compute(buf1);
    sa0.store(buf0, tid);
    sb0.store(buf0 + AF, tid);
    __syncthreads();
  }
  if (i < nsteps) compute(buf0);  // odd slice count: the last slice is in buf0

  // epilogue: acc register r of lane (li, lh) -> row (r&3) + 8*(r>>2) + 4*lh, col li
  float* Cout = SPLIT ? C + (int64_t)blockIdx.y * M * N : C;
  const int64_t ldo = SPLIT ? N : ldc;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t n = n0 + wn * TN * 32 + b * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (!SPLIT && (EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU)) bv = bias[n];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm * TM * 32 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m >= M) continue;
        float v = acc[a][b][r];
        if (!SPLIT) {
          if (EPI == MOLCLR_EPI_BIAS) v = v + bv;
          if (EPI == MOLCLR_EPI_BIAS_RELU) v = fmaxf(v + bv, 0.f);
          if (EPI == MOLCLR_EPI_RELU_MASK) v = aux[m * ldaux + n] > 0.f ? v : 0.f;
          if (accumulate) v += Cout[m * ldo + n];
        }
        Cout[m * ldo + n] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Register-direct variant.  One wave owns a (32 TM) x (32 TN) tile; each
// K-slice's A and B fragments are loaded straight from global memory into the
// MFMA operand layout (lane (li, lh) holds row li, k = 16 lh .. 16 lh + 15:
// four float4 loads of 64 contiguous bytes for a K-contiguous operand, 16
// coalesced 128-byte rows for a K-major one), double-buffered by K-slice.  No
// LDS and no barriers: fp32 MFMA needs only ~16 FLOP per byte from L2 at
// 64 x 64 per wave, so the reuse LDS would provide across waves is not needed.
// Out-of-range rows read a clamped row (their results are never stored); K
// past the end is zeroed at use time (the mask select sits next to the MFMA,
// so no load is waited on early).
template <bool KMAJOR, int TT>
struct DFrag {
  float4 v[TT][4];
  uint32_t kmask;  // bit (4*q + j): k = 16 lh + 4 q + j in range

  __device__ __forceinline__ void load(const float* __restrict__ X, int64_t ld, int64_t r0,
                                       int64_t rows, int64_t k0, int64_t K, int li, int lh) {
    const int64_t kb = k0 + 16 * lh;
    kmask = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) kmask |= (uint32_t)(kb + j < K) << j;
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      int64_t r = r0 + t * 32 + li;
      r = r < rows ? r : rows - 1;
      if (!KMAJOR) {
        const float* p = X + r * ld;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t k = kb + 4 * q;
          v[t][q] = *reinterpret_cast<const float4*>(p + (k < K ? k : 0));
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t k = kb + 4 * q + j;
            e[j] = X[(k < K ? k : K - 1) * ld + r];
          }
          v[t][q] = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    }
  }
  __device__ __forceinline__ float get(int t, int q, int j) const {
    const float4 x = v[t][q];
    const float e = j == 0 ? x.x : (j == 1 ? x.y : (j == 2 ? x.z : x.w));
    return ((kmask >> (4 * q + j)) & 1u) ? e : 0.f;
  }
};

template <int TM, int TN, bool AK, bool BKM, int EPI, bool SPLIT>
__global__ __launch_bounds__(256) void k_gemm_f32_direct(
    const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C, int64_t M,
    int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, const float* __restrict__ bias,
    const float* __restrict__ aux, int64_t ldaux, int ktiles_per_split, int accumulate) {
  constexpr int BM = TM * 32, BN = TN * 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BM - 1) / BM);
  const int nt = ntm * ntn;
  const int nwg = (nt + 3) / 4;
  const int tile = xcd_remap(blockIdx.x, nwg) * 4 + wave;  // 4 neighbouring tiles per WG
  if (tile >= nt) return;  // whole wave
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;
  const int nk_total = (int)((K + BK - 1) / BK);
  const int kt_beg = SPLIT ? blockIdx.y * ktiles_per_split : 0;
  int kt_end = SPLIT ? kt_beg + ktiles_per_split : nk_total;
  if (kt_end > nk_total) kt_end = nk_total;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  DFrag<AK, TM> fa0, fa1;
  DFrag<BKM, TN> fb0, fb1;
  auto compute = [&](const DFrag<AK, TM>& fa, const DFrag<BKM, TN>& fb) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.get(a, q, j), fb.get(b, q, j),
                                                             acc[a][b], 0, 0, 0);
  };
  const int nsteps = kt_end - kt_beg;
  if (nsteps > 0) {
    fa0.load(A, lda, m0, M, (int64_t)kt_beg * BK, K, li, lh);
    fb0.load(B, ldb, n0, N, (int64_t)kt_beg * BK, K, li, lh);
  }
  int i = 0;
  for (; i + 2 <= nsteps; i += 2) {
    fa1.load(A, lda, m0, M, (int64_t)(kt_beg + i + 1) * BK, K, li, lh);
    fb1.load(B, ldb, n0, N, (int64_t)(kt_beg + i + 1) * BK, K, li, lh);
    compute(fa0, fb0);
    fa0.load(A, lda, m0, M, (int64_t)(kt_beg + i + 2) * BK, K, li, lh);
    fb0.load(B, ldb, n0, N, (int64_t)(kt_beg + i + 2) * BK, K, li, lh);
    compute(fa1, fb1);
  }
  if (i < nsteps) compute(fa0, fb0);

  float* Cout = SPLIT ? C + (int64_t)blockIdx.y * M * N : C;
  const int64_t ldo = SPLIT ? N : ldc;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t n = n0 + b * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (!SPLIT && (EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU)) bv = bias[n];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m >= M) continue;
        float v = acc[a][b][r];
        if (!SPLIT) {
          if (EPI == MOLCLR_EPI_BIAS) v = v + bv;
          if (EPI == MOLCLR_EPI_BIAS_RELU) v = fmaxf(v + bv, 0.f);
          if (EPI == MOLCLR_EPI_RELU_MASK) v = aux[m * ldaux + n] > 0.f ? v : 0.f;
          if (accumulate) v += Cout[m * ldo + n];
        }
        Cout[m * ldo + n] = v;
      }
    }
  }
}

// C = epilogue(Σ_z partial[z])  (fixed order -> deterministic)
template <int EPI>
__global__ void k_splitk_reduce(const float* __restrict__ partial, int splits, int64_t M, int64_t N,
                                float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                const float* __restrict__ aux, int64_t ldaux, int accumulate) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * N) return;
  int64_t m = t / N, n = t - m * N;
  float v = 0.f;
  for (int z = 0; z < splits; ++z) v += partial[(int64_t)z * M * N + t];
  if (EPI == MOLCLR_EPI_BIAS) v = v + bias[n];
  if (EPI == MOLCLR_EPI_BIAS_RELU) v = fmaxf(v + bias[n], 0.f);
  if (EPI == MOLCLR_EPI_RELU_MASK) v = aux[m * ldaux + n] > 0.f ? v : 0.f;
  if (accumulate) v += C[m * ldc + n];
  C[m * ldc + n] = v;
}

struct Cfg {
  int wm, wn, tm, tn;
  int bm() const { return wm * tm * 32; }
  int bn() const { return wn * tn * 32; }
};

// 64 x 64 tiles (4 waves x one 32x32 MFMA tile): many small workgroups keep
// every CU's matrix pipe fed to the end of the grid (at M ~ 15k rows a 128 x 128
// tiling leaves 600 tiles for 512 resident slots: a 17%-full second wave).
Cfg pick_cfg(int64_t, int64_t) { return {2, 2, 1, 1}; }

// 0 = LDS-staged 64x64 (default), 1 = register-direct 64x64 per wave,
// 2 = register-direct 32x64 per wave (tuning knob, molclr_gemm_set_impl)
int g_impl = 0;
int tiles_for(int impl, int64_t M, int64_t N) {
  if (impl == 1) return (int)((((M + 63) / 64) * ((N + 63) / 64) + 3) / 4);
  if (impl == 2) return (int)((((M + 31) / 32) * ((N + 63) / 64) + 3) / 4);
  return (int)(((M + 63) / 64) * ((N + 63) / 64));
}

int pick_splits(const Cfg& c, int64_t M, int64_t N, int64_t K) {
  (void)c;
  int64_t tiles = tiles_for(g_impl, M, N) * (g_impl ? 4 : 1);
  int64_t nk = (K + BK - 1) / BK;
  if (tiles >= 512 || nk < 16) return 1;
  int64_t s = (1024 + tiles - 1) / tiles;
  if (s > nk / 8) s = nk / 8;  // keep >= 8 K-slices per split
  if (s > 64) s = 64;
  return s < 1 ? 1 : (int)s;
}

struct Args {
  const float *A, *B;
  float* C;
  int64_t M, N, K, lda, ldb, ldc;
  const float *bias, *aux;
  int64_t ldaux;
  int kps, accumulate;
};

template <int WM, int WN, int TM, int TN, bool AK, bool BKM, int EPI, bool SPLIT>
void launch_t(dim3 grid, hipStream_t s, const Args& a) {
  if (g_impl == 1) {
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_f32_direct<2, 2, AK, BKM, EPI, SPLIT>), grid, dim3(256), 0, s, a.A,
                       a.B, a.C, a.M, a.N, a.K, a.lda, a.ldb, a.ldc, a.bias, a.aux, a.ldaux, a.kps,
                       a.accumulate);
    return;
  }
  if (g_impl == 2) {
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_f32_direct<1, 2, AK, BKM, EPI, SPLIT>), grid, dim3(256), 0, s, a.A,
                       a.B, a.C, a.M, a.N, a.K, a.lda, a.ldb, a.ldc, a.bias, a.aux, a.ldaux, a.kps,
                       a.accumulate);
    return;
  }
  molclr::launch_timed(molclr::kTimeGemm, (k_gemm_f32<WM, WN, TM, TN, AK, BKM, EPI, SPLIT>), grid, dim3(WM * WN * 64),
                     0, s, a.A, a.B, a.C, a.M, a.N, a.K, a.lda, a.ldb, a.ldc, a.bias, a.aux,
                     a.ldaux, a.kps, a.accumulate);
}

template <int WM, int WN, int TM, int TN, bool SPLIT>
int dispatch_layout(int ak, int bk, int epi, dim3 grid, hipStream_t s, const Args& a) {
#define MOLCLR_GEMM_CASE(AKV, BKV, EPV)                                                   \
  if (ak == AKV && bk == BKV && (SPLIT || epi == EPV)) {                                  \
    launch_t<WM, WN, TM, TN, AKV, BKV, SPLIT ? MOLCLR_EPI_NONE : EPV, SPLIT>(grid, s, a); \
    return 0;                                                                             \
  }
#define MOLCLR_GEMM_EPIS(AKV, BKV)                \
  MOLCLR_GEMM_CASE(AKV, BKV, MOLCLR_EPI_NONE)      \
  MOLCLR_GEMM_CASE(AKV, BKV, MOLCLR_EPI_BIAS)      \
  MOLCLR_GEMM_CASE(AKV, BKV, MOLCLR_EPI_BIAS_RELU) \
  MOLCLR_GEMM_CASE(AKV, BKV, MOLCLR_EPI_RELU_MASK)
  if (SPLIT) {
    MOLCLR_GEMM_CASE(false, false, MOLCLR_EPI_NONE)
    MOLCLR_GEMM_CASE(false, true, MOLCLR_EPI_NONE)
    MOLCLR_GEMM_CASE(true, false, MOLCLR_EPI_NONE)
    MOLCLR_GEMM_CASE(true, true, MOLCLR_EPI_NONE)
  } else {
    MOLCLR_GEMM_EPIS(false, false)
    MOLCLR_GEMM_EPIS(false, true)
    MOLCLR_GEMM_EPIS(true, false)
    MOLCLR_GEMM_EPIS(true, true)
  }
#undef MOLCLR_GEMM_EPIS
#undef MOLCLR_GEMM_CASE
  return -1;
}

template <bool SPLIT>
int dispatch_cfg(const Cfg& c, int ak, int bk, int epi, dim3 grid, hipStream_t s, const Args& a) {
  (void)c;
  return dispatch_layout<2, 2, 1, 1, SPLIT>(ak, bk, epi, grid, s, a);
}

}  // namespace

MOLCLR_API size_t molclr_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  Cfg c = pick_cfg(M, N);
  int sp = pick_splits(c, M, N, K);
  return sp > 1 ? (size_t)sp * M * N * sizeof(float) + 256 : 0;
}

MOLCLR_API int molclr_gemm_f32(const float* A, const float* B, float* C, int64_t M, int64_t N,
                               int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor,
                               int b_kmajor, int epilogue_flags, const float* bias, const float* aux,
                               int64_t ldaux, void* workspace, size_t workspace_bytes,
                               molclr_stream_t stream) {
  const int accumulate = (epilogue_flags & MOLCLR_EPI_ACCUMULATE) ? 1 : 0;
  const int epilogue = epilogue_flags & ~MOLCLR_EPI_ACCUMULATE;
  MOLCLR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_f32: negative size");
  MOLCLR_REQUIRE(epilogue >= MOLCLR_EPI_NONE && epilogue <= MOLCLR_EPI_RELU_MASK,
                 "gemm_f32: bad epilogue %d", epilogue);
  MOLCLR_REQUIRE((epilogue != MOLCLR_EPI_BIAS && epilogue != MOLCLR_EPI_BIAS_RELU) || bias,
                 "gemm_f32: bias epilogue needs bias");
  MOLCLR_REQUIRE(epilogue != MOLCLR_EPI_RELU_MASK || aux, "gemm_f32: relu-mask epilogue needs aux");
  // float4 loads along K for the operands stored with K contiguous
  MOLCLR_REQUIRE(a_kmajor || (K % 4 == 0 && lda % 4 == 0),
                 "gemm_f32: A with K contiguous needs K (%lld) and lda multiples of 4", (long long)K);
  MOLCLR_REQUIRE(b_kmajor || (K % 4 == 0 && ldb % 4 == 0),
                 "gemm_f32: B with K contiguous needs K (%lld) and ldb multiples of 4", (long long)K);
  MOLCLR_REQUIRE(ldc >= N && (a_kmajor ? lda >= M : lda >= K) && (b_kmajor ? ldb >= N : ldb >= K),
                 "gemm_f32: leading dimension too small");
  if (M == 0 || N == 0) return MOLCLR_OK;
  hipStream_t s = molclr::as_stream(stream);
  if (K == 0) {
    molclr::set_error("gemm_f32: K == 0 unsupported");
    return MOLCLR_ERR_UNSUPPORTED;
  }
  Cfg c = pick_cfg(M, N);
  int64_t tiles = tiles_for(g_impl, M, N);  // workgroups along x
  MOLCLR_REQUIRE(tiles < (1ll << 31), "gemm_f32: too many tiles");
  int sp = pick_splits(c, M, N, K);
  if (sp > 1 && workspace_bytes < (size_t)sp * M * N * sizeof(float)) sp = 1;
  Args a{A, B, C, M, N, K, lda, ldb, ldc, bias, aux, ldaux, 0, accumulate};
  int rc;
  if (sp == 1) {
    rc = dispatch_cfg<false>(c, a_kmajor != 0, b_kmajor != 0, epilogue, dim3((unsigned)tiles), s, a);
  } else {
    int64_t nk = (K + BK - 1) / BK;
    int kps = (int)((nk + sp - 1) / sp);
    sp = (int)((nk + kps - 1) / kps);
    float* partial = (float*)workspace;
    Args ap{A, B, partial, M, N, K, lda, ldb, N, nullptr, nullptr, 0, kps, 0};
    rc = dispatch_cfg<true>(c, a_kmajor != 0, b_kmajor != 0, MOLCLR_EPI_NONE,
                            dim3((unsigned)tiles, sp), s, ap);
    if (rc == 0) {
      dim3 g((unsigned)molclr::ceil_div(M * N, 256));
      switch (epilogue) {
        case MOLCLR_EPI_NONE:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_NONE>, g, dim3(256), 0, s, partial, sp, M,
                             N, C, ldc, bias, aux, ldaux, accumulate);
          break;
        case MOLCLR_EPI_BIAS:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_BIAS>, g, dim3(256), 0, s, partial, sp, M,
                             N, C, ldc, bias, aux, ldaux, accumulate);
          break;
        case MOLCLR_EPI_BIAS_RELU:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_BIAS_RELU>, g, dim3(256), 0, s, partial, sp,
                             M, N, C, ldc, bias, aux, ldaux, accumulate);
          break;
        default:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_RELU_MASK>, g, dim3(256), 0, s, partial, sp,
                             M, N, C, ldc, bias, aux, ldaux, accumulate);
      }
    }
  }
  if (rc != 0) {
    molclr::set_error("gemm_f32: no kernel for this layout");
    return MOLCLR_ERR_UNSUPPORTED;
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_gemm_set_impl(int impl) {
  MOLCLR_REQUIRE(impl >= 0 && impl <= 2, "gemm_set_impl: impl must be 0, 1 or 2");
  g_impl = impl;
  return MOLCLR_OK;
}
