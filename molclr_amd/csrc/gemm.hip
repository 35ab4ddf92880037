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
#include "mfma.h"

#include <stdlib.h>

#include <type_traits>

namespace {

using namespace molclr;

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
// Split-bf16 fp32 GEMM on v_mfma_f32_32x32x16_bf16.
//
// Every fp32 operand element is split into three bf16 parts, each the
// round-to-nearest bf16 of what is left (mfma.h split2):
//   x = hi + mid + lo + t,  |mid| <= 2^-8 |x|,  |lo| <= 2^-16 |x|,  |t| <= 2^-24 |x|
// and C = Σ_k a b is accumulated in fp32 from the six products down to order
// 2^-16: hi·lo + lo·hi + mid·mid + hi·mid + mid·hi + hi·hi.  What is left out
// (mid·lo, lo·mid, lo·lo and the tails t) is below 4·2^-24 |a b| per product,
// of random sign: the order of one fp32 rounding of the product.  Every
// bf16 x bf16 product is exact in the fp32 accumulator.  The result has fp32
// GEMM accuracy (tests/test_gpu_kernels.py compares against float64 and the
// f32-input MFMA kernel above).  bf16 MFMA runs at 16x the f32-input MFMA
// rate, so six of them cost 3/8 of one f32 MFMA chain.  (Inputs beyond the
// bf16 range, |x| > 3.39e38, are not supported.)
//
// "p6": a 64 x 64 (or 128 x 64 / 64 x 128) tile of 2 x 2 waves with both
// operands staged as split [plane][row][k] images (xoff swizzle).  The first
// version split both operands while staging 4 x 4 blocks and was bound by it
// (rocprofv3: ~20 VALU instructions per MFMA, MFMA busy 22 %); here:
//  * Operand sources (template AMODE / BMODE):
//      0 fp32, K contiguous ([rows][K]): a thread stages 8 consecutive k of
//        one row (two float4 loads) and writes one 16-byte chunk per plane;
//      1 fp32, K-major ([K][rows], the dY^T / X^T of a weight gradient): a
//        thread stages a 4-row x 4-k block and transposes it in registers;
//      2 pre-split bf16 planes ([3][Npad][Kp], molclr_bplanes_make): the
//        weights of a Linear layer, split once per optimizer step instead of
//        once per row tile — staging is a plain 16-byte copy.
//  * Row pointers are fixed per thread (rows clamped once; rows beyond M / N
//    only feed output rows the epilogue never stores); K advances by pointer
//    offsets, and only the last, partial K tile takes the masked path.
// ---------------------------------------------------------------------------
constexpr int kPlanesRowPad = 128;  // Npad multiple (covers every BN)

// fp32, K contiguous: unit = (row, 8-k chunk); ROWS*4 units over T threads.
template <int ROWS, int T>
struct PStageK {
  static constexpr int UNITS = ROWS * 4;
  static constexpr int PER = (UNITS + T - 1) / T;
  const float* p[PER];
  float4 r[PER][2];
  __device__ __forceinline__ void init(const float* __restrict__ src, int64_t ld, int64_t row0,
                                       int64_t rows, int t) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      const int64_t gr = row0 + (u >> 2);
      p[j] = src + (gr < rows ? gr : rows - 1) * ld + 8 * (u & 3);
    }
  }
  __device__ __forceinline__ void load(int64_t k0, int64_t K, int t) {
    const bool full = k0 + BK <= K;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (j == PER - 1 && UNITS % T && t + j * T >= UNITS) continue;
      const float* q = p[j] + k0;
      if (full) {
        r[j][0] = *reinterpret_cast<const float4*>(q);
        r[j][1] = *reinterpret_cast<const float4*>(q + 4);
      } else {  // last K tile: K % 4 == 0, so each float4 is all in or all out
        const int64_t k = k0 + 8 * ((t + j * T) & 3);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        r[j][0] = k < K ? *reinterpret_cast<const float4*>(q) : z;
        r[j][1] = k + 4 < K ? *reinterpret_cast<const float4*>(q + 4) : z;
      }
    }
  }
  __device__ __forceinline__ void store(uint16_t* __restrict__ img, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (j == PER - 1 && UNITS % T && u >= UNITS) continue;
      u32x4 hi, mid, lo;
      split8(r[j][0], r[j][1], hi, mid, lo);
      const int o = xoff(u >> 2, u & 3);
      *reinterpret_cast<u32x4*>(img + o) = hi;
      *reinterpret_cast<u32x4*>(img + ROWS * XK + o) = mid;
      *reinterpret_cast<u32x4*>(img + 2 * ROWS * XK + o) = lo;
    }
  }
};

// fp32, K-major ([K][rows]: the dY^T / X^T of a weight gradient): the image
// is kept K-major too, [k][ROWS] bf16 per plane, and the MFMA fragments are
// read with the gfx950 transposed LDS read (ds_read_b64_tr_b16, kmfrag).  A
// thread stages single float4s (4 consecutive rows at one k): split, one
// 8-byte write per plane, no register transpose.  16 lanes write 128
// contiguous bytes of one k-row (conflict-free); the transposed reads are
// conflict-free through the 32-element XOR of kswz.  (The previous form,
// 4 x 4 blocks transposed in registers into the [row][k] image, spent 60 % of
// its LDS cycles in bank conflicts: rows 4 apart share banks.)
// Needs ROWS == 64, rows % 4 == 0 and ld % 4 == 0.
template <int ROWS, int T, bool H3 = false>
struct PStageM {
  static_assert(ROWS == 64 || ROWS == 128 || ROWS == 160,
                "K-major staging is laid out for 64/128/160-row tiles");
  static constexpr int UNITS = BK * (ROWS / 4);
  static constexpr int PER = (UNITS + T - 1) / T;
  const float* p[PER];
  int64_t ld;
  float4 r[PER];
  __device__ __forceinline__ void init(const float* __restrict__ src, int64_t ld_, int64_t row0,
                                       int64_t rows, int t) {
    ld = ld_;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      const int rb = u % (ROWS / 4), k = u / (ROWS / 4);
      const int64_t gr = row0 + 4 * rb;
      p[j] = src + (int64_t)k * ld + (gr < rows ? gr : rows - 4);
    }
  }
  __device__ __forceinline__ void load(int64_t k0, int64_t K, int t) {
    const bool full = k0 + BK <= K;
    const int64_t base = k0 * ld;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (j == PER - 1 && UNITS % T && u >= UNITS) continue;
      const float* q = p[j] + base;
      if (full) {
        r[j] = *reinterpret_cast<const float4*>(q);
      } else {
        r[j] = k0 + u / (ROWS / 4) < K ? *reinterpret_cast<const float4*>(q)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  // column sums over K of this thread's rows (the bias gradient of a Linear)
  __device__ __forceinline__ void colsum_add(float4* cs, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (j == PER - 1 && UNITS % T && t + j * T >= UNITS) continue;
      cs[j] = f4add(cs[j], r[j]);
    }
  }
  // H3: two fp16 planes of the values scaled by 2^sh; else three bf16 planes
  __device__ __forceinline__ void store(uint16_t* __restrict__ img, int t, int sh = 0) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      if (j == PER - 1 && UNITS % T && u >= UNITS) continue;
      const int rb = u % (ROWS / 4), k = u / (ROWS / 4);
      const int o = k * ROWS + ((4 * rb) ^ kswz<ROWS>(k));
      if constexpr (H3) {
        uint2 hi, lo;
        hsplit4(r[j], sh, hi, lo);
        *reinterpret_cast<uint2*>(img + o) = hi;
        *reinterpret_cast<uint2*>(img + ROWS * XK + o) = lo;
      } else {
        uint2 hi, mid, lo;
        split4(r[j], hi, mid, lo);
        *reinterpret_cast<uint2*>(img + o) = hi;
        *reinterpret_cast<uint2*>(img + ROWS * XK + o) = mid;
        *reinterpret_cast<uint2*>(img + 2 * ROWS * XK + o) = lo;
      }
    }
  }
};

// pre-split planes [3][Npad][Kp] bf16: unit = (plane, row, 16-byte chunk)
template <int ROWS, int T>
struct PStageP {
  static constexpr int UNITS = 3 * ROWS * 4;
  static constexpr int PER = (UNITS + T - 1) / T;
  const uint16_t* p[PER];
  int off[PER];
  u32x4 r[PER];
  __device__ __forceinline__ void init(const uint16_t* __restrict__ planes, int64_t kp,
                                       int64_t plane_stride, int64_t row0, int t) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      const int pl = u / (ROWS * 4), rem = u % (ROWS * 4);
      p[j] = planes + pl * plane_stride + (row0 + (rem >> 2)) * kp + 8 * (rem & 3);
      off[j] = pl * ROWS * XK + xoff(rem >> 2, rem & 3);
    }
  }
  __device__ __forceinline__ void load(int64_t k0, int64_t, int t) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (j == PER - 1 && UNITS % T && t + j * T >= UNITS) continue;
      r[j] = *reinterpret_cast<const u32x4*>(p[j] + k0);
    }
  }
  __device__ __forceinline__ void store(uint16_t* __restrict__ img, int t) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (j == PER - 1 && UNITS % T && t + j * T >= UNITS) continue;
      *reinterpret_cast<u32x4*>(img + off[j]) = r[j];
    }
  }
};

template <int MODE, int ROWS, int T>
struct PStageSel;
template <int ROWS, int T>
struct PStageSel<0, ROWS, T> { using type = PStageK<ROWS, T>; };
template <int ROWS, int T>
struct PStageSel<1, ROWS, T> { using type = PStageM<ROWS, T>; };
template <int ROWS, int T>
struct PStageSel<2, ROWS, T> { using type = PStageP<ROWS, T>; };

// CS: also the column sums of A over K (A K-major: the bias gradient Σ_rows dY
// of a Linear's weight-gradient product), written by the n-tile-0 blocks to
// colsum[m] (or, split-K, to colsum[split * M + m] for k_splitk_reduce).
template <int TM, int TN, int AMODE, int BMODE, int EPI, bool SPLIT, bool CS = false>
__global__ __launch_bounds__(256) void k_gemm_p6(
    const float* __restrict__ A, const float* __restrict__ Bf, const uint16_t* __restrict__ Bp,
    float* __restrict__ C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
    int64_t bplane_stride, int64_t ldc, const float* __restrict__ bias,
    const float* __restrict__ aux, int64_t ldaux, int ktiles_per_split, int accumulate,
    float* __restrict__ colsum) {
  static_assert(!CS || AMODE == 1, "column sums are taken over a K-major A");
  constexpr int T = 256;
  constexpr int BM = 64 * TM, BN = 64 * TN;
  constexpr int AI = 3 * BM * XK, BI = 3 * BN * XK;  // bf16 elements per image
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * (AI + BI)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
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

  f32x16 acc[TM][TN], acl[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = acl[a][b][r] = 0.f;

  using SA = typename PStageSel<AMODE, BM, T>::type;
  using SB = typename PStageSel<BMODE, BN, T>::type;
  // a K-major operand with fewer units than threads leaves threads idle: give
  // the other operand's units to those threads
  const int ta = tid;
  const int tb = (AMODE == 1 && SA::UNITS < T) ? (tid + SA::UNITS) % T : tid;
  SA sa0, sa1;
  SB sb0, sb1;
  sa0.init(A, lda, m0, M, ta);
  if constexpr (BMODE == 2) sb0.init(Bp, ldb, bplane_stride, n0, tb);
  else sb0.init(Bf, ldb, n0, N, tb);
  sa1 = sa0;
  sb1 = sb0;
  uint16_t* buf0 = lds;
  uint16_t* buf1 = lds + (AI + BI);

  // fragment of rows r0 .. r0+31 of an image plane: [row][k] images are read
  // by row (xfrag), K-major [k][row] images by the transposed read (kmfrag)
  auto afrag = [&](const uint16_t* plane, int r0, int ks) {
    if constexpr (AMODE == 1) return kmfrag<BM>(plane, r0, ks, lane);
    else return xfrag(plane, r0 + li, ks * 2 + lh);
  };
  auto bfrag = [&](const uint16_t* plane, int r0, int ks) {
    if constexpr (BMODE == 1) return kmfrag<BN>(plane, r0, ks, lane);
    else return xfrag(plane, r0 + li, ks * 2 + lh);
  };
  auto compute = [&](const uint16_t* As) {
    const uint16_t* Bs = As + AI;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bh[TN], bm[TN], bl[TN];
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int bro = wn * TN * 32 + b * 32;
        bh[b] = bfrag(Bs, bro, ks);
        bm[b] = bfrag(Bs + BN * XK, bro, ks);
        bl[b] = bfrag(Bs + 2 * BN * XK, bro, ks);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int aro = wm * TM * 32 + a * 32;
        const bf16x8 ah = afrag(As, aro, ks);
        const bf16x8 am = afrag(As + BM * XK, aro, ks);
        const bf16x8 al = afrag(As + 2 * BM * XK, aro, ks);
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acl[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[b], acl[a][b], 0, 0, 0);
          acl[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[b], acl[a][b], 0, 0, 0);
          acl[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm[b], acl[a][b], 0, 0, 0);
          acl[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm[b], acl[a][b], 0, 0, 0);
          acl[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh[b], acl[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[b], acc[a][b], 0, 0, 0);
        }
      }
    }
  };

  const int nsteps = kt_end - kt_beg;
  auto kof = [&](int step) { return (int64_t)(kt_beg + step) * BK; };
  constexpr int CSN = CS == 1 ? SA::PER : CS == 2 ? SB::PER : 1;
  float4 cs[CSN];
#pragma unroll
  for (int j = 0; j < CSN; ++j) cs[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (nsteps > 0) {
    sa0.load(kof(0), K, ta);
    sb0.load(kof(0), K, tb);
    if (nsteps > 1) {
      sa1.load(kof(1), K, ta);
      sb1.load(kof(1), K, tb);
    }
    if constexpr (CS) sa0.colsum_add(cs, ta);
    sa0.store(buf0, ta);
    sb0.store(buf0 + AI, tb);
    __syncthreads();
  }
  int i = 0;
  for (; i + 2 <= nsteps; i += 2) {
    if (i + 2 < nsteps) {
      sa0.load(kof(i + 2), K, ta);
      sb0.load(kof(i + 2), K, tb);
    }
    compute(buf0);
    if constexpr (CS) sa1.colsum_add(cs, ta);  // K step i + 1
    sa1.store(buf1, ta);
    sb1.store(buf1 + AI, tb);
    __syncthreads();
    if (i + 3 < nsteps) {
      sa1.load(kof(i + 3), K, ta);
      sb1.load(kof(i + 3), K, tb);
    }
    compute(buf1);
    if constexpr (CS) {
      if (i + 2 < nsteps) sa0.colsum_add(cs, ta);  // K step i + 2
    }
    // unconditional: when i + 2 >= nsteps the image is never read again
    sa0.store(buf0, ta);
    sb0.store(buf0 + AI, tb);
    __syncthreads();
  }
  if (i < nsteps) compute(buf0);

  if constexpr (CS) {
    if (n0 == 0 && colsum != nullptr) {  // block-uniform
      // a thread's units all share one 4-row group rb = tid % (BM/4); fold them,
      // then the T/(BM/4) threads of each group in a fixed order
      constexpr int RB = BM / 4;
      float4 v = cs[0];
#pragma unroll
      for (int j = 1; j < CSN; ++j) v = f4add(v, cs[j]);
      __syncthreads();  // K images no longer read
      float4* red = reinterpret_cast<float4*>(lds);
      red[tid] = v;
      __syncthreads();
      if (tid < RB) {
        float4 t4 = red[tid];
        for (int q = 1; q < T / RB; ++q) t4 = f4add(t4, red[tid + q * RB]);
        const float e[4] = {t4.x, t4.y, t4.z, t4.w};
        float* o = SPLIT ? colsum + (int64_t)blockIdx.y * M : colsum;
        for (int j = 0; j < 4; ++j) {
          const int64_t m = m0 + 4 * tid + j;
          if (m < M) o[m] = (!SPLIT && accumulate) ? o[m] + e[j] : e[j];
        }
      }
    }
  }

  float* Cout = SPLIT ? C + (int64_t)blockIdx.y * M * N : C;
  const int64_t ldo = SPLIT ? N : ldc;
  // Epilogue through LDS: each wave writes its accumulators as a row-major
  // [32 TM][32 TN] fp32 tile, then stores 16-byte row pieces (4 store
  // instructions per 32 x 32 instead of 16 dword stores: the store tail is
  // issue-bound).  Needs 16-byte aligned rows; otherwise the dword path.
  constexpr int WR = 32 * TM, WC = 32 * TN;
  static_assert(4 * WR * WC * (int)sizeof(float) <= (int)sizeof(lds), "epilogue tile > LDS");
  const bool vec = ((ldo & 3) == 0) && ((reinterpret_cast<uintptr_t>(Cout) & 15) == 0) &&
                   (SPLIT || EPI != MOLCLR_EPI_RELU_MASK ||
                    (((ldaux & 3) == 0) && (reinterpret_cast<uintptr_t>(aux) & 15) == 0)) &&
                   (SPLIT || (EPI != MOLCLR_EPI_BIAS && EPI != MOLCLR_EPI_BIAS_RELU) ||
                    (reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  if (vec) {
    __syncthreads();  // every wave is done reading the K images
    float* tw = reinterpret_cast<float*>(lds) + wave * WR * WC;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          tw[(a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * WC + b * 32 + li] =
              acc[a][b][r] + acl[a][b][r];
    __syncthreads();
    constexpr int C4 = WC / 4;
    const int64_t mw = m0 + wm * WR, nw = n0 + wn * WC;
#pragma unroll
    for (int it = 0; it < WR * C4 / 64; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx / C4, c4 = idx - row * C4;
      const int64_t m = mw + row, n = nw + 4 * c4;
      if (m >= M || n >= N) continue;
      float4 v = *reinterpret_cast<const float4*>(tw + row * WC + 4 * c4);
      float* o = Cout + m * ldo + n;
      if (n + 4 <= N) {
        if (!SPLIT) {
          if (EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU) {
            const float4 bv = *reinterpret_cast<const float4*>(bias + n);
            v = f4add(v, bv);
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if (EPI == MOLCLR_EPI_RELU_MASK) {
            const float4 x = *reinterpret_cast<const float4*>(aux + m * ldaux + n);
            v = make_float4(x.x > 0.f ? v.x : 0.f, x.y > 0.f ? v.y : 0.f, x.z > 0.f ? v.z : 0.f,
                            x.w > 0.f ? v.w : 0.f);
          }
          if (accumulate) v = f4add(v, *reinterpret_cast<const float4*>(o));
        }
        *reinterpret_cast<float4*>(o) = v;
      } else {  // the last, partial piece of a row (N % 4 != 0)
        const float e[4] = {v.x, v.y, v.z, v.w};
        for (int j = 0; j < 4 && n + j < N; ++j) {
          float x = e[j];
          if (!SPLIT) {
            if (EPI == MOLCLR_EPI_BIAS) x = x + bias[n + j];
            if (EPI == MOLCLR_EPI_BIAS_RELU) x = fmaxf(x + bias[n + j], 0.f);
            if (EPI == MOLCLR_EPI_RELU_MASK) x = aux[m * ldaux + n + j] > 0.f ? x : 0.f;
            if (accumulate) x += o[j];
          }
          o[j] = x;
        }
      }
    }
    return;
  }
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
        float v = acc[a][b][r] + acl[a][b][r];
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
// "q6": split-bf16 GEMM of a row-major fp32 A with pre-split weight planes
// (molclr_gemm_f32_bplanes with a_kmajor = 0): the forward and data-gradient
// products of every Linear.  On these shapes k_gemm_p6 is bound by staging,
// not by the MFMA: each K step of a 64 x 64 tile writes 24 KB of images to
// LDS (a ds_write_b128 moves ~80 B/clk/CU) and splits 8 A elements per
// thread, all for 12 MFMAs per wave and a barrier.  q6 decomposes differently:
//  * the block's 4 waves are stacked along M: wave w owns rows m0 + 32w .. +31
//    and all BN = 32 TN columns of the block, so no A element is needed by two
//    waves.  A goes global -> registers -> split -> MFMA operand: no A image,
//    no A ds_write, no redundant split;
//  * only B (the pre-split planes: a 16-byte copy per unit) is staged,
//    double-buffered and shared by the 4 waves: 30 KB per K step for
//    4 x 60 MFMAs at TN = 5 (against 24 KB for 4 x 12 in p6).  The stage is
//    written right after the barrier and the next one issued before the
//    MFMAs, so LDS writes and load latency overlap the compute;
//  * one accumulator: the six products of an element pair go into the same
//    fp32 sum, which keeps the registers at two waves per SIMD (p6's separate
//    correction sum would cost 80 more).  Over the K of a Linear's forward /
//    data gradient (K <= 1024: 64 MFMA accumulations per sum) the error stays
//    at p6's (tests/test_gpu_kernels.py); a 1000-step chain (K = 15700, all
//    products positive) measured 5x p6's, so longer K go to p6 / split-K.
// K order: for K step k0 and MFMA step s, lane half h of both operands holds
// the actual k = k0 + 16h + 8s .. +7, so an A lane loads its row's 64
// contiguous bytes k0 + 16h .. +15 once per K step, and the B fragment is
// image chunk 2h + s.
// ---------------------------------------------------------------------------
constexpr int kQ6Waves = 4;
constexpr int kQ6BM = 32 * kQ6Waves;
constexpr int64_t kQ6MaxK = 1024;  // longer chains of one fp32 sum: see above

// pre-split planes [3][npad][kp] -> LDS image [3][BN][XK]; unit = (plane, row,
// 16-byte chunk), rows clamped into the planes (columns >= N are never stored)
template <int BN, int T, int NP = 3>
struct QStageB {
  static constexpr int UNITS = NP * BN * 4;
  static constexpr int PER = (UNITS + T - 1) / T;
  u32x4 r[PER];
  int goff[PER];
  __device__ __forceinline__ void init(int64_t n0, int64_t npad, int64_t kp, int t) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = t + j * T;
      const int pl = u / (BN * 4), rem = u % (BN * 4);
      int64_t row = n0 + (rem >> 2);
      row = row < npad ? row : npad - 1;
      goff[j] = (UNITS % T && u >= UNITS) ? 0 : (int)((pl * npad + row) * kp + 8 * (rem & 3));
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
      const int pl = u / (BN * 4), rem = u % (BN * 4);
      *reinterpret_cast<u32x4*>(img + pl * BN * XK + xoff(rem >> 2, rem & 3)) = r[j];
    }
  }
};

// B by LDS-DMA (global_load_lds): the pre-split planes need no conversion, so
// a K step's image is copied straight into LDS -- no staging registers, no
// ds_write (measured: the register round trip and its LDS stores were 25-35 %
// of the kernel, tools/q6_abl.py).  One K step = NP x BN / 16 chunks of 1 KB
// (16 image rows of 64 B); wave w of the group issues chunks w, w + 4, ...;
// lane l writes physical chunk l % 4 of its image row, which xoff() gives
// the logical chunk (l % 4) ^ ((row >> 2) & 3) -- the swizzle is applied to
// the source address.  Rows past the planes are clamped (never stored).
template <int BN, int NP>
__device__ __forceinline__ void q6_dma_b(const uint16_t* __restrict__ Bp, int64_t n0, int64_t npad,
                                         int64_t kp, int64_t k0, uint16_t* img, int wm, int lane) {
  constexpr int RPB = BN / 16, CH = NP * RPB, PERW = (CH + kQ6Waves - 1) / kQ6Waves;
  static_assert(BN % 16 == 0, "q6 DMA: 16-row chunks");
#pragma unroll
  for (int qq = 0; qq < PERW; ++qq) {
    const int q = wm + kQ6Waves * qq;
    if (CH % kQ6Waves && q >= CH) break;  // wave-uniform
    const int pl = q / RPB, row = (q % RPB) * 16 + (lane >> 2), c = lane & 3;
    int64_t gr = n0 + row;
    gr = gr < npad ? gr : npad - 1;
    __builtin_amdgcn_global_load_lds(
        (gbl_as_ptr)(Bp + (pl * npad + gr) * kp + k0 + 8 * (c ^ ((row >> 2) & 3))),
        (lds_as_ptr)(img + (pl * BN + (q % RPB) * 16) * XK), 16, 0, 0);
  }
}

// KG > 1 splits K inside the block: KG groups of 4 waves take the K steps
// g, g + KG, ... of the same tile, each with its own B ring, and group 0 adds
// the other groups' sums (in group order, through LDS) before the epilogue.
// For the narrow products (N = 300: ~960 waves of 32 x 160 for 1024 SIMDs)
// this puts two waves on every SIMD instead of one.
// MASK: some K steps of this launch are partial or (KG > 1) beyond the last
// one; their A values at k >= K are zeroed where they are consumed.  The
// main loop has no branch: every load is issued from a clamped, in-bounds
// address, so the compiler keeps counted vmcnt waits and the next steps'
// loads stay in flight across the MFMAs (a conditional load makes it drain
// every outstanding load at the top of each step).
// H3 != 0: the fp16 two-part form (mfma.h "h3"): the planes are 2 fp16 parts
// of B scaled by its max slot `bmax`; A is scaled by its max slot `amax`
// (H3 == 1) or row by row (H3 == 2) by its row maxima, given as `arow_parts`
// partial arrays amax[p][M] (each lane splits one row of A, so a row of small
// values -- a node with a small gradient -- keeps its precision however large
// other rows are); three fp16 MFMAs per product; the sums are scaled back in
// the epilogue.  Any mode: the epilogue folds max |C| into the slot `cmax`
// (atomic maxima, the caller zeroes it) and stores the row maxima of C over
// this block's columns into crow[column tile][M] (plain stores: the column
// tiles' partial row maxima), and `amax_out` (zeroed) receives max |A| over
// the loaded rows -- the scales an h3 consumer of A or C needs, with no pass
// of their own.  Each is optional.  ReLU as bits: `bits_out` (optional)
// receives bit (n % 32) of word [n / 32][m] (column-block major, bits_ld =
// M: a wave's 8 rows of one block are 32 contiguous bytes) = C > 0 after the
// epilogue; a RELU_MASK epilogue given `bits_in` takes its mask from such bits
// instead of reading aux (32x fewer bytes than the fp32 a1).
template <int TN, int EPI, int KG, bool MASK, int H3 = 0>
__global__ __launch_bounds__(64 * kQ6Waves * KG) __attribute__((amdgpu_waves_per_eu(2))) void k_gemm_q6(
    const float* __restrict__ A, const uint16_t* __restrict__ Bp, float* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux,
    int accumulate, const float* __restrict__ amax, const float* __restrict__ bmax,
    float* __restrict__ cmax, float* __restrict__ crow, float* __restrict__ amax_out,
    int arow_parts, uint32_t* __restrict__ bits_out, const uint32_t* __restrict__ bits_in,
    int64_t bits_ld) {
  constexpr int T = 64 * kQ6Waves;  // threads of one K group
  constexpr int BN = 32 * TN;
  constexpr int NP = H3 ? 2 : 3;    // B planes
  constexpr int BI = NP * BN * XK;  // 16-bit elements per B image
  constexpr int EPI_ELEMS = kQ6Waves * 32 * 32 * 2;  // the epilogue's wave tiles (fp32)
  constexpr int L0 = KG == 1 ? (BI > EPI_ELEMS ? BI : EPI_ELEMS) : KG * 2 * BI;
  static_assert(KG == 1 || (kQ6Waves * 32 * BN * (int)sizeof(float) <=
                            KG * 2 * BI * (int)sizeof(uint16_t)),
                "group sums exceed the LDS images");
  // One K group: the two B buffers are separate __shared__ arrays, so the
  // compiler sees that the LDS-DMA in flight into one does not alias the
  // fragment reads of the other (one array: it waited vmcnt(0) -- the whole
  // prefetch of the next step -- before the first read of every step).
  // K groups: one array (their group sums need it contiguous).
  __shared__ __attribute__((aligned(16))) uint16_t lds[L0];
  __shared__ __attribute__((aligned(16))) uint16_t lds_b1[KG == 1 ? BI : 8];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar
  const int grp = wave / kQ6Waves, wm = wave % kQ6Waves, gt = tid - grp * T;
  const int li = lane & 31, lh = lane >> 5;

  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + kQ6BM - 1) / kQ6BM);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);  // a row slab's column tiles share an XCD
  const int64_t m0 = (int64_t)(tile / ntn) * kQ6BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;

  // What the epilogue reads -- bias columns, ReLU-mask words -- is loaded
  // here, ahead of the main loop: CDNA4's vmcnt counts stores too, so a load
  // issued among the epilogue's stores waits for all of them.  Epilogue lane
  // (row, c4): columns nb + 4 c4 .. +3 of rows mw + 8 it + lane / 8.
  constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;
  constexpr int BVN = HAS_BIAS ? TN : 1, MWN = EPI == MOLCLR_EPI_RELU_MASK ? TN : 1;
  float4 bvq[BVN];
  uint32_t mwq[MWN][4];
  if (grp == 0) {
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
      if (bits_in != nullptr) {  // block-uniform
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
  const int nsteps = (int)(kp / BK);             // K steps of the planes (K rounded up)
  const int rounds = (nsteps + KG - 1) / KG;     // every group runs as many
  // this group's round r is K step grp + KG r; B is read from a clamped step
  // (a step past the last is zeroed through A), A from clamped addresses
  auto kb = [&](int r) {
    const int st = grp + KG * r;
    return (int64_t)(st < nsteps ? st : nsteps - 1) * BK;
  };
  // this lane's 16 k of round r: float4 j holds k0 + 16 lh + 4 j .. +3 (K % 4 == 0)
  auto load_a = [&](int r, float4(&v)[4]) {
    r = r < rounds ? r : rounds - 1;  // prefetch past the end: never consumed
    const int64_t k = (int64_t)(grp + KG * r) * BK + 16 * lh;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t kj = k + 4 * j;
      if constexpr (MASK) kj = kj < K - 4 ? kj : K - 4;
      v[j] = *reinterpret_cast<const float4*>(arow + kj);
    }
  };

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  // this lane's A shift (its row's with H3 == 2), the planes' shift
  int sha = 0;
  if constexpr (H3 == 1) sha = h3_shift(amax);
  if constexpr (H3 == 2) {
    float m = 0.f;
    if (arow_parts < 0)  // per-wave pairs of a producer with D / 4 = -arow_parts
      m = row_max_of_waves(reinterpret_cast<const float2*>(amax), arow_i, -arow_parts);
    else
      for (int p = 0; p < arow_parts; ++p) m = fmaxf(m, amax[(int64_t)p * M + arow_i]);
    sha = h3_shift_of(m);
  }
  const int shb = H3 ? h3_shift(bmax) : 0;
  float ain = 0.f;  // max |A| of this lane's loads (amax_out)
  auto compute = [&](const uint16_t* Bs, const float4(&a)[4], int r) {
    if (amax_out != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ain = fmaxf(ain, fmaxf(fmaxf(fabsf(a[j].x), fabsf(a[j].y)), fmaxf(fabsf(a[j].z), fabsf(a[j].w))));
    }
    float4 am4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      am4[j] = a[j];
      if constexpr (MASK) {
        const int64_t kj = (int64_t)(grp + KG * r) * BK + 16 * lh + 4 * j;
        if (kj >= K) am4[j] = f4zero();
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (H3) {
        u32x4 h, l;
        hsplit8(am4[2 * s], am4[2 * s + 1], sha, h, l);
        const f16x8 ah = __builtin_bit_cast(f16x8, h);
        const f16x8 al = __builtin_bit_cast(f16x8, l);
        const int ch = 2 * lh + s;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int row = 32 * b + li;
          const f16x8 bh = __builtin_bit_cast(f16x8, xfrag(Bs, row, ch));
          const f16x8 bl = __builtin_bit_cast(f16x8, xfrag(Bs + BN * XK, row, ch));
          acc[b] = mfma_h3(ah, al, bh, bl, acc[b]);
        }
        continue;
      }
      u32x4 h, m, l;
      split8(am4[2 * s], am4[2 * s + 1], h, m, l);
      const bf16x8 ah = __builtin_bit_cast(bf16x8, h);
      const bf16x8 am = __builtin_bit_cast(bf16x8, m);
      const bf16x8 al = __builtin_bit_cast(bf16x8, l);
      const int ch = 2 * lh + s;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int row = 32 * b + li;
        const bf16x8 bh = xfrag(Bs, row, ch);
        const bf16x8 bm = xfrag(Bs + BN * XK, row, ch);
        const bf16x8 bl = xfrag(Bs + 2 * BN * XK, row, ch);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[b], 0, 0, 0);
      }
    }
  };

  uint16_t* buf0 = KG == 1 ? lds : lds + grp * 2 * BI;
  uint16_t* buf1 = KG == 1 ? lds_b1 : buf0 + BI;
  float4 a0[4], a1[4];
  (void)gt;
  q6_dma_b<BN, NP>(Bp, n0, npad, kp, kb(0), buf0, wm, lane);
  load_a(0, a0);
  __syncthreads();
  // Step i: its top issues every load it leaves for step i + 1 -- the DMA of
  // B(i + 1) into the other buffer and A(i + 1) into the other register set
  // -- then the MFMAs of step i, then the barrier (whose vmcnt(0) the compute
  // phase has already covered).  One barrier per K step.  Loads past the
  // last round re-read a clamped step.
  int i = 0;
  for (; i + 2 <= rounds; i += 2) {
    q6_dma_b<BN, NP>(Bp, n0, npad, kp, kb(i + 1), buf1, wm, lane);
    load_a(i + 1, a1);
    compute(buf0, a0, i);
    __syncthreads();
    q6_dma_b<BN, NP>(Bp, n0, npad, kp, kb(i + 2), buf0, wm, lane);
    load_a(i + 2, a0);
    compute(buf1, a1, i + 1);
    __syncthreads();
  }
  if (i < rounds) compute(buf0, a0, i);  // odd count: B(i) is in buf0
  __syncthreads();                       // the images are reused below

  if constexpr (KG > 1) {
    // the other groups' sums, added to group 0's in group order
    float* gw = reinterpret_cast<float*>(lds) + wm * 32 * BN;
#pragma unroll 1
    for (int g = 1; g < KG; ++g) {
      if (grp == g) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) gw[(b * 16 + r) * 64 + lane] = acc[b][r];
      }
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[b][r] += gw[(b * 16 + r) * 64 + lane];
      }
      __syncthreads();
    }
  }

  // Epilogue (group 0): per 32 x 32 block, the wave's accumulator goes through
  // its own 4 KB of LDS so that rows leave as 16-byte pieces (8 rows x 128 B
  // per store instruction).
  const bool vec = ((ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                   (EPI != MOLCLR_EPI_RELU_MASK || bits_in != nullptr ||
                    (((ldaux & 3) == 0) && (reinterpret_cast<uintptr_t>(aux) & 15) == 0)) &&
                   ((EPI != MOLCLR_EPI_BIAS && EPI != MOLCLR_EPI_BIAS_RELU) ||
                    (reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  float* tw = reinterpret_cast<float*>(lds) + wm * 32 * 32;
  const int64_t mw = m0 + 32 * wm;
  // max |C| of this lane's stores per epilogue row group it (row 8 it +
  // lane / 8 of the wave's 32): for cmax and crow
  float rm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;  // block-uniform
    if (grp == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
        // scale back by the row's shift (held by lane `row`) and the planes'
        const int sr = H3 == 2 ? __shfl(sha, row, 64) : sha;
        tw[row * 32 + li] = H3 ? __builtin_ldexpf(acc[b][r], -(sr + shb)) : acc[b][r];
      }
    }
    wave_lds_sync();  // tw is this wave's own 4 KB: no block barrier
    if (grp == 0) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = it * 64 + lane;
        const int row = idx >> 3, c4 = idx & 7;
        const int64_t m = mw + row, n = nb + 4 * c4;
        uint32_t pos = 0;  // bits of C > 0 for this lane's 4 columns (bits_out)
        if (m < M && n < N) {
          const float4 v4 = *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
          float* o = C + m * ldc + n;
          // the mask nibble of this lane's columns (RELU_MASK with bits_in)
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
            if (accumulate) v = f4add(v, *reinterpret_cast<const float4*>(o));
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
              if (accumulate) x += o[j];
              o[j] = x;
              rm[it] = fmaxf(rm[it], fabsf(x));
              pos |= (x > 0.f ? 1u : 0u) << j;
            }
          }
        }
        if (bits_out != nullptr) {
          // one ballot per column slot j (bit 8 row + c4 of the wave); a row's
          // word interleaves the 8 bits of its lanes: bit 4 c4 + j
          const uint64_t bj[4] = {__ballot((pos & 1u) != 0u), __ballot((pos & 2u) != 0u),
                                  __ballot((pos & 4u) != 0u), __ballot((pos & 8u) != 0u)};
          if (c4 == 0 && m < M) {
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              uint32_t x = (uint32_t)(bj[j] >> (8 * (lane >> 3))) & 0xFFu;  // bit c -> bit 4 c
              x = (x | (x << 12)) & 0x000F000Fu;
              x = (x | (x << 6)) & 0x03030303u;
              x = (x | (x << 3)) & 0x11111111u;
              w |= x << j;
            }
            bits_out[(nb >> 5) * bits_ld + m] = w;
          }
        }
      }
    }
    wave_lds_sync();  // the wave's tile is rewritten by the next block
  }
  {
    if (crow != nullptr && grp == 0) {
      // the 8 lanes of a row (lane / 8) fold their maxima, then one atomic per row
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
    if (cmax != nullptr)
      absmax_publish(grp == 0 ? fmaxf(fmaxf(rm[0], rm[1]), fmaxf(rm[2], rm[3])) : 0.f, cmax);
    if (amax_out != nullptr) absmax_publish(ain, amax_out);
  }
}

// ---------------------------------------------------------------------------
// "pp": the q6 product (one K group) as a ping-pong over two wave groups.
// A block of 8 waves owns 256 rows x BN columns: waves 0-3 (group 0) rows
// m0 .. m0+127 and waves 4-7 (group 1) rows m0+128 .. m0+255, 32 rows each,
// every SIMD holding one wave of each group; both groups read one shared B
// image per K step.  Group 1 runs one phase behind group 0, so between two
// block barriers one group issues its step's MFMAs -- the B fragments of the
// next column block read from LDS under the current block's MFMAs, pinned by
// sched_group_barrier -- while the other splits its next A step into bf16 /
// fp16 fragments, issues the A loads two steps ahead and (group 1) the
// LDS-DMA of the next B image:
//   phase 2i+1: group 0 computes step i      | group 1 splits step i, loads
//   phase 2i+2: group 0 splits step i+1      | group 1 computes step i
// The matrix and vector pipes of a SIMD run the two waves' phases side by
// side (q6: every wave splits and multiplies in turn, each K step behind a
// barrier of its own group).  Loads use buffer addressing: fixed per-lane
// offsets, one scalar offset per step.  The products, their order and the
// epilogue are q6's: results are bit-identical to k_gemm_q6<TN, EPI, 1, *, H3>
// (tests/test_gpu_kernels.py).  Measured at the c2 shapes in isolation
// (tools/q6x.py): lin1 80 -> 72 us, lin2 69 -> 63, dz1 61 -> 57, dagg 50 -> 46;
// in the step (rocprofv3, same box): lin1 88.1 -> 84.5, lin2 69.9 -> 67.5,
// dz1 79.6 -> 75.0, dagg 53.0 -> 57.9 (so narrow h3 products stay on q6).
// ---------------------------------------------------------------------------
constexpr int kPPRows = 256;

// SW (h3 only): the MFMAs take the operands swapped, so a lane's accumulators
// are one ROW of each 32 x 32 block (row li, columns in four runs of four):
// the epilogue unscales by the lane's own row shift, stores float4s straight
// from registers (no LDS transpose), keeps the row max in one register (crow:
// one shuffle per tile) and builds a row's ReLU bits from two lanes.  Same
// products in the same order: results identical to the unswapped form.
template <int TN, int EPI, int H3, bool SW = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_gemm_pp(
    const float* __restrict__ A, const uint16_t* __restrict__ Bp, float* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux,
    int accumulate, const float* __restrict__ amax, const float* __restrict__ bmax,
    float* __restrict__ cmax, float* __restrict__ crow, float* __restrict__ amax_out,
    int arow_parts, uint32_t* __restrict__ bits_out, const uint32_t* __restrict__ bits_in,
    int64_t bits_ld) {
  constexpr int BN = 32 * TN;
  constexpr int NP = H3 ? 2 : 3;
  constexpr int BI = NP * BN * XK;
  static_assert(!SW || H3, "the swapped form is the h3 kernel's");
  // two B images (separate arrays: the LDS-DMA into one must not look like it
  // aliases the fragment reads of the other) and the epilogue's wave tiles
  __shared__ __attribute__((aligned(16))) uint16_t bimg0[BI];
  __shared__ __attribute__((aligned(16))) uint16_t bimg1[BI];
  __shared__ __attribute__((aligned(16))) float ep[8 * 32 * 32];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, wm = w & 3;
  const int li = lane & 31, lh = lane >> 5;

  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + kPPRows - 1) / kPPRows);
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);  // a row slab's column tiles share an XCD
  const int64_t m0 = (int64_t)(tile / ntn) * kPPRows;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;
  const int64_t mw = m0 + 128 * grp + 32 * wm;  // this wave's first row

  // epilogue operands ahead of the main loop (vmcnt counts stores too)
  constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;
  constexpr int BVN = HAS_BIAS && !SW ? TN : 1, MWN = EPI == MOLCLR_EPI_RELU_MASK && !SW ? TN : 1;
  constexpr int MSN = EPI == MOLCLR_EPI_RELU_MASK && SW ? TN : 1;
  float4 bvq[BVN];
  uint32_t mwq[MWN][4];
  uint32_t mws[MSN];  // SW: the lane's row's mask word per column block
  float4 breg = f4zero();  // SW: lanes 0 .. BN/4-1's chunk of the tile's bias
  if constexpr (SW) {
    // the tile's bias columns go to the (then unused) epilogue LDS in the
    // prologue, once the load has landed
    if constexpr (HAS_BIAS) {
      const int64_t n = n0 + 4 * (tid < BN / 4 ? tid : 0);
      if (n + 4 <= N && (reinterpret_cast<uintptr_t>(bias) & 15) == 0)
        breg = *reinterpret_cast<const float4*>(bias + n);
    }
    if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
      if (bits_in != nullptr) {
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          int64_t m = mw + li;
          m = m < M ? m : M - 1;
          int64_t nb = n0 + 32 * b;
          nb = nb < N ? nb : 0;
          mws[b] = bits_in[(nb >> 5) * bits_ld + m];
        }
      }
    }
  } else {
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
  const int S = (int)(kp / BK);  // K steps (the last may run past K: zeroed)
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(A, M * lda * 4);
  const __amdgpu_buffer_rsrc_t brsrc = make_rsrc(Bp, (int64_t)NP * npad * kp * 2);
  const uint32_t avoff = (uint32_t)((arow_i * lda + 16 * lh) * 4);
  // this lane's 16 k of step r: float4 j holds k = 32 r + 16 lh + 4 j .. +3
  auto load_a = [&](int r, float4(&v)[4]) {
    const uint32_t soff = (uint32_t)(r * BK * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = buf_ld4(arsrc, avoff + 16 * j, soff);
  };
  // a step's B image: CH chunks of 1 KB (16 image rows of 64 B), issued by
  // group 1; lane l writes physical chunk l % 4 of its image row, the source
  // address carries the xoff swizzle (as q6_dma_b)
  constexpr int RPB = BN / 16, CH = NP * RPB, PERW = (CH + 3) / 4;
  uint32_t bvoff[PERW];
#pragma unroll
  for (int qq = 0; qq < PERW; ++qq) {
    const int q = wm + 4 * qq;
    const int qc = q < CH ? q : CH - 1;
    const int pl = qc / RPB, row = (qc % RPB) * 16 + (lane >> 2), c = lane & 3;
    int64_t gr = n0 + row;
    gr = gr < npad ? gr : npad - 1;  // rows past the planes: never stored
    bvoff[qq] = (uint32_t)(((pl * npad + gr) * kp + 8 * (c ^ ((row >> 2) & 3))) * 2);
  }
  auto dma_b = [&](int r, uint16_t* img) {
    const uint32_t soff = (uint32_t)(r * BK * 2);
#pragma unroll
    for (int qq = 0; qq < PERW; ++qq) {
      const int q = wm + 4 * qq;
      if (CH % 4 && q >= CH) break;  // wave-uniform
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
    if (arow_parts < 0)  // per-wave pairs of a producer with D / 4 = -arow_parts
      m = row_max_of_waves(reinterpret_cast<const float2*>(amax), arow_i, -arow_parts);
    else
      for (int p = 0; p < arow_parts; ++p) m = fmaxf(m, amax[(int64_t)p * M + arow_i]);
    sha = h3_shift_of(m);
  }
  const int shb = H3 ? h3_shift(bmax) : 0;
  float ain = 0.f;  // max |A| of this lane's loads (amax_out)

  u32x4 fr[2][NP];  // this step's A fragments [sub-step][plane]
  auto split = [&](float4(&a)[4], int r) {
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
    for (int s = 0; s < 2; ++s) {
      if constexpr (H3) hsplit8(a[2 * s], a[2 * s + 1], sha, fr[s][0], fr[s][1]);
      else split8(a[2 * s], a[2 * s + 1], fr[s][0], fr[s][1], fr[s][2]);
    }
  };
  // the compute phase: 2 TN blocks of MFMAs (block k: sub-step k / TN, column
  // block k % TN), block k + 1's B fragments read under block k's MFMAs
  auto compute = [&](const uint16_t* Bs) {
    constexpr int NB = 2 * TN;
    auto rd = [&](int k, u32x4(&f)[NP]) {
      const int s1 = k / TN, b1 = k % TN;
#pragma unroll
      for (int p = 0; p < NP; ++p)
        f[p] = *reinterpret_cast<const u32x4*>(Bs + p * BN * XK + xoff(32 * b1 + li, 2 * lh + s1));
    };
    u32x4 q[2][NP];
    rd(0, q[0]);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int s = k / TN, b = k % TN;
      if (k + 1 < NB) rd(k + 1, q[(k + 1) & 1]);
      const u32x4* cb = q[k & 1];
      if constexpr (H3 && SW) {
        acc[b] = mfma_h3_t(__builtin_bit_cast(f16x8, fr[s][0]), __builtin_bit_cast(f16x8, fr[s][1]),
                           __builtin_bit_cast(f16x8, cb[0]), __builtin_bit_cast(f16x8, cb[1]), acc[b]);
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
    constexpr int NM = H3 ? 3 : 6;  // MFMAs per block
    __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);  // block 0's reads
#pragma unroll
    for (int k = 0; k < NB; ++k) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        if (k + 1 < NB && m < NP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one read
      }
    }
  };

  // prologue: B(0), A(0) landed, A(1) in flight; A runs two steps ahead (two
  // register sets), B one step (two images); the loop is unrolled by two so
  // every register set and image is chosen at compile time
  float4 ar0[4], ar1[4];
  if (grp == 1) dma_b(0, bimg0);
  load_a(0, ar0);
  if (S > 1) {
    load_a(1, ar1);
    vm_wait<4>();
  } else {
    vm_wait<0>();
  }
  if constexpr (SW && HAS_BIAS)
    if (tid < BN / 4) *reinterpret_cast<float4*>(ep + 4 * tid) = breg;
  __syncthreads();
  split(ar0, 0);
  if (S > 1 && grp == 1) dma_b(1, bimg1);
  if (S > 2) load_a(2, ar0);
  if (grp == 1) __syncthreads();  // group 1 runs one phase behind
  // step i (parity P): compute from image P, then the load phase of step
  // i + 1: its A is in set 1 - P (issued two load phases ago), B(i + 1) in
  // image 1 - P (issued one load phase ago, before A(i + 2): vmcnt(4) covers it)
  auto body = [&](auto P, int i) -> bool {
    constexpr int par = decltype(P)::value;
    compute(par ? bimg1 : bimg0);
    if (i + 1 >= S) return false;
    if (i + 2 < S) vm_wait<4>();
    else vm_wait<0>();
    __syncthreads();
    float4(&an)[4] = par ? ar0 : ar1;  // step i + 1's A
    split(an, i + 1);
    if (i + 2 < S && grp == 1) dma_b(i + 2, par ? bimg1 : bimg0);
    if (i + 3 < S) load_a(i + 3, an);
    __syncthreads();
    return true;
  };
  for (int i = 0;; i += 2) {
    if (!body(std::integral_constant<int, 0>{}, i)) break;
    if (!body(std::integral_constant<int, 1>{}, i + 1)) break;
  }
  if (grp == 0) __syncthreads();  // the barrier count of both groups: 2 S

  const bool vec = ((ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                   (EPI != MOLCLR_EPI_RELU_MASK || bits_in != nullptr ||
                    (((ldaux & 3) == 0) && (reinterpret_cast<uintptr_t>(aux) & 15) == 0)) &&
                   ((EPI != MOLCLR_EPI_BIAS && EPI != MOLCLR_EPI_BIAS_RELU) ||
                    (reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  if constexpr (SW) {
    // rows from registers: lane (li, lh) holds row m = mw + li of block b at
    // columns nb + 8 q + 4 lh .. +3 in acc[b][4 q .. 4 q + 3]
    const int64_t m = mw + li;
    const float sc = __builtin_ldexpf(1.f, -(sha + shb));  // exact: a power of two
    float rmax = 0.f;
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int64_t nb = n0 + 32 * b;
      if (nb >= N) break;  // block-uniform
      uint32_t pos = 0;  // bits of C > 0 in this lane's columns of the row
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cb = 8 * q + 4 * lh;
        const int64_t n = nb + cb;
        if (m < M && n < N) {
          float* o = C + m * ldc + n;
          const float4 v4 = make_float4(acc[b][4 * q] * sc, acc[b][4 * q + 1] * sc,
                                        acc[b][4 * q + 2] * sc, acc[b][4 * q + 3] * sc);
          uint32_t mk = 15u;
          if constexpr (EPI == MOLCLR_EPI_RELU_MASK)
            if (bits_in != nullptr) mk = (mws[b] >> cb) & 15u;
          if (vec && n + 4 <= N) {
            float4 v = v4;
            if constexpr (HAS_BIAS) {
              v = f4add(v, *reinterpret_cast<const float4*>(ep + 32 * b + cb));
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
            if (accumulate) v = f4add(v, *reinterpret_cast<const float4*>(o));
            *reinterpret_cast<float4*>(o) = v;
            rmax = fmaxf(rmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            pos |= ((v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
                    (v.w > 0.f ? 8u : 0u)) << cb;
          } else {
            const float e[4] = {v4.x, v4.y, v4.z, v4.w};
            for (int j = 0; j < 4 && n + j < N; ++j) {
              float x = e[j];
              if (EPI == MOLCLR_EPI_BIAS) x = x + bias[n + j];
              if (EPI == MOLCLR_EPI_BIAS_RELU) x = fmaxf(x + bias[n + j], 0.f);
              if (EPI == MOLCLR_EPI_RELU_MASK)
                x = (bits_in != nullptr ? ((mk >> j) & 1u) != 0u : aux[m * ldaux + n + j] > 0.f)
                        ? x : 0.f;
              if (accumulate) x += o[j];
              o[j] = x;
              rmax = fmaxf(rmax, fabsf(x));
              pos |= (x > 0.f ? 1u : 0u) << (cb + j);
            }
          }
        }
      }
      if (bits_out != nullptr) {
        pos |= __shfl_xor(pos, 32, 64);  // the row's other 16 columns
        if (lh == 0 && m < M) bits_out[(nb >> 5) * bits_ld + m] = pos;
      }
    }
    if (crow != nullptr) {
      const float v = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
      if (lh == 0 && m < M) crow[(n0 / BN) * M + m] = v;
    }
    if (cmax != nullptr) absmax_publish(rmax, cmax);
    if (amax_out != nullptr) absmax_publish(ain, amax_out);
    return;
  }
  // Epilogue (q6's): per 32 x 32 block, the wave's accumulator goes through
  // its own 4 KB of LDS so that rows leave as 16-byte pieces
  float* tw = ep + w * 32 * 32;
  float rm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;  // block-uniform
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
          if (accumulate) v = f4add(v, *reinterpret_cast<const float4*>(o));
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
            if (accumulate) x += o[j];
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
}

// ---------------------------------------------------------------------------
// "bs": B-stationary h3 product for K in (288, 304] (the c2 / c3 width 300:
// lin1 = agg W1^T and dz1 = dz W2, 600 columns).  A 128-column tile of the
// weight's fp16 planes for the WHOLE K (9 full 32-deep steps and the first 16
// k of the last: 152 KB) is copied into LDS once per block by LDS-DMA; the
// block (one per CU, 8 waves) then streams its row slabs of A through
// registers -- load two steps ahead, split, MFMA against B fragments read from
// LDS -- with no barrier after the prologue (k_gemm_pp stages B per K step
// behind two barriers and its waves stalled half their lifetime,
// profiles/r5_pmc_h3_lin1).  Same fragments, the same three products in the
// same order as k_gemm_pp's swapped form: C, the ReLU bits, max |C|, max |A|
// and the row maxima are bit-identical to it (tests/test_gpu_kernels.py);
// the row maxima come as ceil(N / 128) partial arrays (molclr_gemm_row_parts).
// Blocks: ceil(N / 128) column tiles x (CUs / tiles) row groups, the tiles of
// a row group adjacent on one XCD (they read the same A rows).
// ---------------------------------------------------------------------------
constexpr int kBN = 128;  // columns per tile (TN = 4)
constexpr int kTN = 4;
constexpr int kFullImg = 2 * kBN * XK;  // fp16 elements of one full K step (both planes)
constexpr int kHalfImg = 2 * kBN * 16;  // ... of a last step holding k0 .. k0+15 only

// offset (fp16 units) of chunk c (0 or 1) of row `row` in a half-step plane:
// 32 B per row, the two chunks swapped on alternate row quads
__device__ __forceinline__ int hoff(int row, int c) { return row * 16 + ((c ^ ((row >> 2) & 1)) << 3); }

// Pipelined across slabs:  A wave's next slab --
// its row maxima, ReLU-mask words and first two A steps -- is issued during
// the current slab's last two steps and waited for BEFORE the current
// slab's C stores, so the next slab's first two steps run without a memory
// wait; the stores then drain under those steps' MFMAs (any wait for a load
// while stores are pending is a full drain on this target).  The first
// slab's loads go out with the B image's LDS-DMA: one latency for both.
template <int EPI, int H3, int S, bool HALF, int W = 8>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(W / 4))) void k_gemm_bs(
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
        // wave wi's first row is arow iff it starts inside the row (no division)
        if (wi <= (e0 >> 6)) m = fmaxf(m, (wi << 6) >= s0 ? rw[2 * q] : rw[2 * q + 1]);
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

  float4 ar0[4], ar1[4];
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
    // steps 0 .. S-3: A(r) waited for (steps 0 and 1: already landed), A(r+2) issued
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
    // steps S-2, S-1: the next slab's state and first two A steps go out
    const int sha_cur = sha;
    const int64_t mw_cur = mw;
    {
      float4(&a8)[4] = ar0;
      float4(&a9)[4] = ar1;
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
    int rmaxi = 0;  // the ReLU epilogue's maxima, as bits
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
          if (EPI == MOLCLR_EPI_BIAS_RELU && !accumulate) {
            // v = max(., 0) >= 0 or -0: the maxima as integer maxima of the
            // bits (no |.| and no NaN canonicalisation; -0 reads as < 0)
            rmaxi = max(rmaxi, max(max(__float_as_int(v.x), __float_as_int(v.y)),
                                   max(__float_as_int(v.z), __float_as_int(v.w))));
          } else {
            rmax = fmaxf(rmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          }
          pos |= ((v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
                  (v.w > 0.f ? 8u : 0u)) << cb;
        }
      }
      if (bits_out != nullptr) {
        pos |= __shfl_xor(pos, 32, 64);
        if (lh == 0 && m < M) bits_out[(nb >> 5) * bits_ld + m] = pos;
      }
    }
    rmax = fmaxf(rmax, __int_as_float(rmaxi));
    if (crow != nullptr) {
      const float v = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
      if (lh == 0 && m < M) crow[(int64_t)tile * M + m] = v;
    }
    cm = fmaxf(cm, rmax);
  }
  if (cmax != nullptr) absmax_publish(cm, cmax);
  if (amax_out != nullptr) absmax_publish(ain, amax_out);
}

// "bs16": k_gemm_bs on the 16 x 16 x 32 fp16 MFMA.  The same B image and the
// same pipeline, over 16-row slabs: a lane holds 8 consecutive k of its row
// (one fragment per 32-k step) and, after the MFMAs, 4 consecutive columns of
// its row per 16-column block, so an epilogue store instruction writes 16
// rows x 64 B (k_gemm_bs: 32 rows x 32 B), a block's slabs split over its 8
// waves in twice as many, finer rounds (c2: 4.7 slabs per wave against 2.3),
// and half the accumulator registers.  The k order inside an MFMA differs
// from the 32 x 32 x 16 form: results equal k_gemm_bs's to fp32 rounding,
// not bit for bit.
__device__ __forceinline__ f32x4 mfma16_h3_t(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, al, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, ah, acc, 0, 0, 0);
}
// k_gemm_bsn: the same kernel for any tile width BNT (128: the K = 300
// products; 64: the K = 600 products lin2 and dagg, N = 300, whose whole-K
// image of a 64-column tile is 19 full steps, 152 KB) and an odd step count.
// bsn's image swizzle: chunk c of row r sits in 16-byte slot c ^ F[(r >> 2) & 3]
// with F = {0, 2, 3, 1}.  A 16 x 16 x 32 fragment read (lane: row r16 of the
// block, chunk lane >> 4) then touches 16 distinct 16-byte bank slots in each
// of ds_read_b128's four lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31},
// and the same + 32); xoff's F = {0, 1, 2, 3}, right for the 32 x 32 x 16
// reads, gives these reads 2-way conflicts (PMC: SQ_LDS_BANK_CONFLICT 45 % of
// the LDS cycles).
__device__ __forceinline__ int bsn_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ int bsn_off(int row, int chunk) {
  return row * XK + ((chunk ^ bsn_swz(row)) << 3);
}
template <int EPI, int H3, int S, bool HALF, int W = 8, int BNT = kBN>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(W / 4))) void k_gemm_bsn(
    const float* __restrict__ A, const uint16_t* __restrict__ Bp, float* __restrict__ C,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t kp, int64_t npad, int64_t ldc,
    const float* __restrict__ bias, const float* __restrict__ aux, int64_t ldaux, int accumulate,
    const float* __restrict__ amax, const float* __restrict__ bmax, float* __restrict__ cmax,
    float* __restrict__ crow, float* __restrict__ amax_out, int arow_parts,
    uint32_t* __restrict__ bits_out, const uint32_t* __restrict__ bits_in, int64_t bits_ld,
    int ntn, int groups) {
  static_assert(S >= 4 && (S % 2 == 0 || !HALF), "steps in pairs, or an odd count of full steps");
  constexpr int kBN = BNT, kTN = BNT / 32;  // this tile (k_gemm_bs's constants shadowed)
  constexpr int kFullImg = 2 * kBN * XK, kHalfImg = 2 * kBN * 16;
  constexpr int NFULL = HALF ? S - 1 : S;
  constexpr int IMG = NFULL * kFullImg + (HALF ? kHalfImg : 0);
  constexpr int NB = kBN / 16;  // 16-column blocks of the tile
  __shared__ __attribute__((aligned(16))) uint16_t img[IMG];
  __shared__ __attribute__((aligned(16))) float bsh[kBN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q4 = lane >> 4;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = L % ntn, grp = L / ntn;
  const int64_t n0 = (int64_t)tile * kBN;
  const int64_t slabs = (M + 15) / 16;
  const int64_t s_beg = slabs * grp / groups, s_end = slabs * (grp + 1) / groups;
  constexpr bool HAS_BIAS = EPI == MOLCLR_EPI_BIAS || EPI == MOLCLR_EPI_BIAS_RELU;

  // the B image: as k_gemm_bs
  const __amdgpu_buffer_rsrc_t brsrc = make_rsrc(Bp, (int64_t)2 * npad * kp * 2);
  {
    constexpr int CHF = NFULL * 2 * (kBN / 16);
    for (int q = w; q < CHF; q += W) {
      const int st = q / (2 * (kBN / 16)), rem = q % (2 * (kBN / 16));
      const int pl = rem / (kBN / 16), r0 = (rem % (kBN / 16)) * 16;
      const int row = r0 + (lane >> 2), c = lane & 3;
      int64_t gr = n0 + row;
      gr = gr < npad ? gr : npad - 1;
      const uint32_t voff = (uint32_t)(((pl * npad + gr) * kp + 32 * st + 8 * (c ^ bsn_swz(row))) * 2);
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

  int64_t arow = 0;
  uint32_t avoff = 0;
  float rw[8];
  uint32_t mws[kTN];
  auto meta_issue = [&](int64_t slab) {
    arow = slab * 16 + r16;
    arow = arow < M ? arow : M - 1;
    avoff = (uint32_t)((arow * lda + 8 * q4) * 4);
    if constexpr (H3 == 2) {
      if (arow_parts < 0) {
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
      for (int g = 0; g < kTN; ++g) {
        int64_t nb = n0 + 32 * g;
        nb = nb < N ? nb : 0;
        mws[g] = bits_in[(nb >> 5) * bits_ld + arow];
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
        if (wi <= (e0 >> 6)) m = fmaxf(m, (wi << 6) >= s0 ? rw[2 * q] : rw[2 * q + 1]);
      }
    } else {
#pragma unroll
      for (int p = 0; p < 8; ++p)
        if (p < arow_parts) m = fmaxf(m, rw[p]);
    }
    return h3_shift_of(m);
  };
  auto load_a = [&](int r, float4(&v)[2]) {
    const uint32_t soff = (uint32_t)(r * BK * 4);
    v[0] = buf_ld4(arsrc, avoff, soff);
    v[1] = buf_ld4(arsrc, avoff + 16, soff);
  };

  float4 ar0[2], ar1[2];
  u32x4 frh, frl;
  f32x4 acc[NB];
  auto compute = [&](const uint16_t* base) {
    auto rd = [&](int b, u32x4(&f)[2]) {
      const int row = 16 * b + r16;
      f[0] = *reinterpret_cast<const u32x4*>(base + bsn_off(row, q4));
      f[1] = *reinterpret_cast<const u32x4*>(base + kBN * XK + bsn_off(row, q4));
    };
    u32x4 q[2][2];
    rd(0, q[0]);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b + 1 < NB) rd(b + 1, q[(b + 1) & 1]);
      acc[b] = mfma16_h3_t(__builtin_bit_cast(f16x8, frh), __builtin_bit_cast(f16x8, frl),
                           __builtin_bit_cast(f16x8, q[b & 1][0]),
                           __builtin_bit_cast(f16x8, q[b & 1][1]), acc[b]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int mm = 0; mm < 3; ++mm) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (b + 1 < NB && mm < 2) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
  };
  // the last step holds k0 .. k0+15 only: lanes q4 >= 2 (k0+16 ..) take zeros
  auto compute_half = [&]() {
    const uint16_t* base = img + NFULL * kFullImg;
    const u32x4 z = {0u, 0u, 0u, 0u};
    const int c = q4 & 1;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int row = 16 * b + r16;
      const u32x4 h = *reinterpret_cast<const u32x4*>(base + hoff(row, c));
      const u32x4 l = *reinterpret_cast<const u32x4*>(base + kBN * 16 + hoff(row, c));
      acc[b] = mfma16_h3_t(__builtin_bit_cast(f16x8, frh), __builtin_bit_cast(f16x8, frl),
                           __builtin_bit_cast(f16x8, q4 >= 2 ? z : h),
                           __builtin_bit_cast(f16x8, q4 >= 2 ? z : l), acc[b]);
    }
  };
  auto split = [&](float4(&a)[2], int r, int sha) {
    if (amax_out != nullptr) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        ain = fmaxf(ain, fmaxf(fmaxf(fabsf(a[j].x), fabsf(a[j].y)), fmaxf(fabsf(a[j].z), fabsf(a[j].w))));
    }
    if (r == S - 1) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if ((int64_t)r * BK + 8 * q4 + 4 * j >= K) a[j] = f4zero();
    }
    hsplit8(a[0], a[1], sha, frh, frl);
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
  int64_t mw = slab * 16;

  for (; slab < s_end; slab += W) {
    const int64_t next = slab + W;
    const bool more = next < s_end;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[b][r] = 0.f;
    uint32_t mcur[kTN];
#pragma unroll
    for (int g = 0; g < kTN; ++g) mcur[g] = mws[g];
    constexpr int SP = S % 2 ? S - 3 : S - 2;  // steps taken in pairs
#pragma unroll 1
    for (int r = 0; r < SP; r += 2) {
      if (r > 0) vm_wait<2>();
      split(ar0, r, sha);
      load_a(r + 2, ar0);
      compute(img + r * kFullImg);
      if (r > 0) vm_wait<2>();
      split(ar1, r + 1, sha);
      load_a(r + 3, ar1);
      compute(img + (r + 1) * kFullImg);
    }
    const int sha_cur = sha;
    const int64_t mw_cur = mw;
    if constexpr (S % 2) {
      // three last steps (ar0, ar1, ar0); the next slab's A(0), A(1) land in
      // ar1, ar0 and are swapped back
      vm_wait<2>();
      split(ar0, S - 3, sha_cur);
      load_a(S - 1, ar0);
      compute(img + (S - 3) * kFullImg);
      vm_wait<2>();
      split(ar1, S - 2, sha_cur);
      if (more) {
        meta_issue(next);
        load_a(0, ar1);
      }
      compute(img + (S - 2) * kFullImg);
      if (more) vm_wait<4>();
      else vm_wait<0>();
      split(ar0, S - 1, sha_cur);
      if (more) load_a(1, ar0);  // split consumed ar0
      compute(img + (S - 1) * kFullImg);
      if (more) {
        const float4 x0 = ar0[0], x1 = ar0[1];
        ar0[0] = ar1[0];
        ar0[1] = ar1[1];
        ar1[0] = x0;
        ar1[1] = x1;
      }
    } else {
      vm_wait<2>();
      split(ar0, S - 2, sha_cur);
      if (more) {
        meta_issue(next);
        load_a(0, ar0);
      }
      compute(img + (S - 2) * kFullImg);
      if (more) vm_wait<4>();
      else vm_wait<0>();
      split(ar1, S - 1, sha_cur);
      if (more) load_a(1, ar1);
      if (HALF) compute_half();
      else compute(img + (S - 1) * kFullImg);
    }
    vm_wait<0>();  // the next slab's loads landed before any store is issued
    if (more) {
      sha = row_shift();
      mw = next * 16;
    }

    // ---- epilogue: lane (r16, q4) holds columns 16 b + 4 q4 .. +3 of row r16
    const int64_t m = mw_cur + r16;
    const float sc = __builtin_ldexpf(1.f, -(sha_cur + shb));
    float rmax = 0.f;
    int rmaxi = 0;
#pragma unroll
    for (int g = 0; g < kTN; ++g) {  // 32-column groups (a ReLU-bit word each)
      const int64_t ng = n0 + 32 * g;
      if (ng >= N) break;
      uint32_t pos = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int b = 2 * g + h;
        const int cb = 16 * h + 4 * q4;  // column within the group
        const int64_t n = ng + cb;
        if (m < M && n < N) {
          float* o = C + m * ldc + n;
          float4 v = make_float4(acc[b][0] * sc, acc[b][1] * sc, acc[b][2] * sc, acc[b][3] * sc);
          if constexpr (HAS_BIAS) {
            v = f4add(v, *reinterpret_cast<const float4*>(bsh + 32 * g + cb));
            if (EPI == MOLCLR_EPI_BIAS_RELU)
              v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          }
          if constexpr (EPI == MOLCLR_EPI_RELU_MASK) {
            const uint32_t mk = (mcur[g] >> cb) & 15u;
            v = make_float4(mk & 1u ? v.x : 0.f, mk & 2u ? v.y : 0.f, mk & 4u ? v.z : 0.f,
                            mk & 8u ? v.w : 0.f);
          }
          if (accumulate) v = f4add(v, *reinterpret_cast<const float4*>(o));
          *reinterpret_cast<float4*>(o) = v;
          if (EPI == MOLCLR_EPI_BIAS_RELU && !accumulate) {
            rmaxi = max(rmaxi, max(max(__float_as_int(v.x), __float_as_int(v.y)),
                                   max(__float_as_int(v.z), __float_as_int(v.w))));
          } else {
            rmax = fmaxf(rmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          }
          pos |= ((v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
                  (v.w > 0.f ? 8u : 0u)) << cb;
        }
      }
      if (bits_out != nullptr) {
        pos |= __shfl_xor(pos, 16, 64);
        pos |= __shfl_xor(pos, 32, 64);
        if (q4 == 0 && m < M) bits_out[(ng >> 5) * bits_ld + m] = pos;
      }
    }
    rmax = fmaxf(rmax, __int_as_float(rmaxi));
    if (crow != nullptr) {
      float v = fmaxf(rmax, __shfl_xor(rmax, 16, 64));
      v = fmaxf(v, __shfl_xor(v, 32, 64));
      if (q4 == 0 && m < M) crow[(int64_t)tile * M + m] = v;
    }
    cm = fmaxf(cm, rmax);
  }
  if (cmax != nullptr) absmax_publish(cm, cmax);
  if (amax_out != nullptr) absmax_publish(ain, amax_out);
}

// ---------------------------------------------------------------------------
// "w6": the weight gradient of a Linear, C[m][n] = Σ_k A[k][m] B[k][n] with
// both operands K-major (K = rows: dW = dY^T X), optionally with the column
// sums Σ_k A[k][m] (the bias gradient, A = dY) taken from the staged tiles.
// The q6 decomposition with both operands staged: the 4 waves are stacked
// along M (32 rows each) over BN = 32 TN columns, so a wave issues TN x 6
// MFMAs per 16 k from one A fragment (p6's 128 x 64 tile: 2 x 6).  Both
// operands are split while staging into K-major [3][BK][rows] images read with
// the transposed LDS read (kmfrag).  One image (54 KB at TN = 5) and one
// accumulator per output block keep two blocks on a CU, so one block's
// split-and-stage phase runs beside the other's MFMAs.  Split-K over the rows
// keeps every fp32 sum short (<= ~40 MFMA accumulations); the partial tiles
// are summed in a fixed order by k_splitk_reduce (deterministic, no atomics).
//
// KG = 2 puts two such 4-wave groups in one block, each with its own image,
// taking the K steps g, g + 2, ... of the split; group 1 runs one phase behind
// group 0, so at every barrier one group splits and stages while the other
// issues MFMAs (the overlap two co-resident blocks gave), and group 0 adds
// group 1's sums through LDS before the store.  Each split then covers twice
// the K, so the partial tiles -- written here and read back by
// k_splitk_reduce -- are half as many.
// ---------------------------------------------------------------------------
constexpr int kW6BM = 128;

// H3: both operands scaled by their max slots and split into two fp16 parts
// (mfma.h "h3"), three fp16 MFMAs per product, partials scaled back.
// CS: column sums of nothing (0), of A (1: the bias gradient when A = dY), or
// of B (2: when the product runs transposed, B = dY -- w6_transposed).
template <int TN, int CS, int KG, bool H3 = false>
__global__ __launch_bounds__(256 * KG) __attribute__((amdgpu_waves_per_eu(2))) void k_gemm_w6(
    const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ part,
    int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int ktiles_per_split, int splits,
    float* __restrict__ cs_part, const float* __restrict__ amax, const float* __restrict__ bmax) {
  constexpr int T = 256;  // threads of one K group
  constexpr int BM = kW6BM, BN = 32 * TN;
  constexpr int NP = H3 ? 2 : 3;                       // planes per operand
  constexpr int AI = NP * BM * XK, BI = NP * BN * XK;  // 16-bit elements per image
  static_assert(4 * 32 * 32 * (int)sizeof(float) <= (AI + BI) * (int)sizeof(uint16_t),
                "epilogue tiles exceed the LDS image");
  // the images, or the group sums (4 waves x 32 x BN fp32) when those are larger
  constexpr int GS = KG > 1 ? 4 * 32 * BN * 2 : 0;
  constexpr int LDS_ELEMS = KG * (AI + BI) > GS ? KG * (AI + BI) : GS;
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_ELEMS];

  const int tid = threadIdx.x;
  const int grp = tid / T, gt = tid - grp * T;
  const int lane = tid & 63, wave = gt >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (int)((N + BN - 1) / BN);
  const int ntm = (int)((M + BM - 1) / BM);
  const int ntiles = ntm * ntn;
  // the blocks of one K slice are consecutive ids, so xcd_remap keeps them --
  // and the rows they all read -- on one XCD
  const int id = xcd_remap(blockIdx.x, ntiles * splits);
  const int split = id / ntiles, tile = id - split * ntiles;
  const int64_t m0 = (int64_t)(tile / ntn) * BM;
  const int64_t n0 = (int64_t)(tile % ntn) * BN;
  const int nk_total = (int)((K + BK - 1) / BK);
  const int kt_beg = split * ktiles_per_split;
  int kt_end = kt_beg + ktiles_per_split;
  if (kt_end > nk_total) kt_end = nk_total;
  const int nsteps = kt_end > kt_beg ? kt_end - kt_beg : 0;

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  using SA = PStageM<BM, T, H3>;
  using SB = PStageM<BN, T, H3>;
  const int sha = H3 ? h3_shift(amax) : 0, shb = H3 ? h3_shift(bmax) : 0;
  SA sa;
  SB sb;
  sa.init(A, lda, m0, M, gt);
  sb.init(B, ldb, n0, N, gt);
  constexpr int CSN = CS == 1 ? SA::PER : CS == 2 ? SB::PER : 1;
  float4 cs[CSN];
#pragma unroll
  for (int j = 0; j < CSN; ++j) cs[j] = f4zero();
  // this group's K steps: grp, grp + KG, ... of the split
  auto kof = [&](int step) { return (int64_t)(kt_beg + grp + KG * step) * BK; };
  uint16_t* img = lds + grp * (AI + BI);
  const uint16_t* As = img;
  const uint16_t* Bs = img + AI;
  // MFMA groups g = (ks, b) in order, 2 TN of them; the fragments of group
  // g + 2 are read while group g's MFMAs run (interleaved by
  // sched_group_barrier).  Left to itself the compiler front-loaded reads in
  // bursts and waited on them between MFMA runs; measured in the c2 step:
  // 60.5 -> 59.1 us per h3 weight gradient.  A's ks = 1 fragments come with
  // group TN's.
  auto compute = [&]() {
    constexpr int NG = 2 * TN, NM = H3 ? 3 : 6;
    bf16x8 fa[2][NP], fb[3][NP];
    auto read_a = [&](int ks) {
#pragma unroll
      for (int p = 0; p < NP; ++p) fa[ks][p] = kmfrag<BM>(As + p * BM * XK, 32 * wave, ks, lane);
    };
    auto read_b = [&](int g) {
#pragma unroll
      for (int p = 0; p < NP; ++p)
        fb[g % 3][p] = kmfrag<BN>(Bs + p * BN * XK, 32 * (g % TN), g / TN, lane);
    };
    read_a(0);
    read_b(0);
    read_b(1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int ks = g / TN, b = g % TN;
      const bf16x8* a = fa[ks];
      const bf16x8* f = fb[g % 3];
      if constexpr (H3) {
        acc[b] = mfma_h3(__builtin_bit_cast(f16x8, a[0]), __builtin_bit_cast(f16x8, a[1]),
                         __builtin_bit_cast(f16x8, f[0]), __builtin_bit_cast(f16x8, f[1]), acc[b]);
      } else {  // (hi, mid, lo) = 0, 1, 2; small terms first
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], f[2], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], f[0], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], f[1], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], f[1], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], f[0], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], f[0], acc[b], 0, 0, 0);
      }
      if (g + 2 < NG) {
        read_b(g + 2);
        if (g + 2 == TN) read_a(1);
        if (g + 2 == TN) interleave_mfma_reads<NM, 4 * NP>();
        else interleave_mfma_reads<NM, 2 * NP>();
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // per K step, two phases: (even) split + stage the registers loaded one
  // step earlier; (odd) issue the next step's loads, MFMAs.  A barrier after
  // every phase; group g runs g phases behind group 0.
  const int ns = (nsteps - grp + KG - 1) / KG;  // this group's steps
  const int ns0 = (nsteps + KG - 1) / KG;       // group 0's
  if (ns > 0) {
    sa.load(kof(0), K, gt);
    sb.load(kof(0), K, gt);
  }
  for (int p = 0; p < 2 * ns0 + KG - 1; ++p) {
    const int q = p - grp;
    if (q >= 0 && q < 2 * ns) {
      const int i = q >> 1;
      if ((q & 1) == 0) {
        if constexpr (CS == 1) sa.colsum_add(cs, gt);
        if constexpr (CS == 2) sb.colsum_add(cs, gt);
        sa.store(img, gt, sha);
        sb.store(img + AI, gt, shb);
      } else {
        if (i + 1 < ns) {
          sa.load(kof(i + 1), K, gt);
          sb.load(kof(i + 1), K, gt);
        }
        compute();
      }
    }
    __syncthreads();
  }

  if constexpr (CS == 2) {
    if (m0 == 0 && cs_part != nullptr) {  // block-uniform
      // B's column sums: every (group, unit u = k (BN/4) + rb) float4 through
      // LDS, then thread rb < BN/4 adds its units in (group, k) order
      constexpr int RB = BN / 4;
      float4* red = reinterpret_cast<float4*>(lds);
#pragma unroll
      for (int j = 0; j < CSN; ++j) {
        const int u = gt + j * T;
        if (u < SB::UNITS) red[grp * SB::UNITS + u] = cs[j];
      }
      __syncthreads();
      if (tid < RB) {
        float4 t4 = f4zero();
        for (int q = 0; q < KG * BK; ++q) t4 = f4add(t4, red[q * RB + tid]);
        const float e[4] = {t4.x, t4.y, t4.z, t4.w};
        for (int j = 0; j < 4; ++j) {
          const int64_t n = n0 + 4 * tid + j;
          if (n < N) cs_part[(int64_t)split * N + n] = e[j];
        }
      }
      __syncthreads();
    }
  }
  if constexpr (CS == 1) {
    if (n0 == 0 && cs_part != nullptr) {  // block-uniform
      // a thread's units all share one 4-row group rb = tid % (BM/4): fold
      // them, then the KG*T/(BM/4) threads of each group in a fixed order
      constexpr int RB = BM / 4;
      float4 v = cs[0];
#pragma unroll
      for (int j = 1; j < CSN; ++j) v = f4add(v, cs[j]);
      float4* red = reinterpret_cast<float4*>(lds);
      red[tid] = v;
      __syncthreads();
      if (tid < RB) {
        float4 t4 = red[tid];
        for (int q = 1; q < KG * T / RB; ++q) t4 = f4add(t4, red[tid + q * RB]);
        const float e[4] = {t4.x, t4.y, t4.z, t4.w};
        for (int j = 0; j < 4; ++j) {
          const int64_t m = m0 + 4 * tid + j;
          if (m < M) cs_part[(int64_t)split * M + m] = e[j];
        }
      }
      __syncthreads();
    }
  }

  if constexpr (KG > 1) {
    // the other groups' sums, added to group 0's in group order
    float* gw = reinterpret_cast<float*>(lds) + wave * 32 * BN;
#pragma unroll 1
    for (int g = 1; g < KG; ++g) {
      if (grp == g) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) gw[(b * 16 + r) * 64 + lane] = acc[b][r];
      }
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[b][r] += gw[(b * 16 + r) * 64 + lane];
      }
      __syncthreads();
    }
  }

  // partial tile (group 0), per 32 x 32 block through the wave's 4 KB of LDS,
  // 16-byte stores
  float* tw = reinterpret_cast<float*>(lds) + wave * 32 * 32;
  float* P = part + (int64_t)split * M * N;
  const int64_t mw = m0 + 32 * wave;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int64_t nb = n0 + 32 * b;
    if (nb >= N) break;  // block-uniform
    if (grp == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        tw[((r & 3) + 8 * (r >> 2) + 4 * lh) * 32 + li] =
            H3 ? __builtin_ldexpf(acc[b][r], -(sha + shb)) : acc[b][r];
    }
    wave_lds_sync();  // tw is this wave's own 4 KB: no block barrier
    if (grp == 0) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = it * 64 + lane;
        const int row = idx >> 3, c4 = idx & 7;
        const int64_t m = mw + row, n = nb + 4 * c4;
        if (m < M && n < N)
          *reinterpret_cast<float4*>(P + m * N + n) =
              *reinterpret_cast<const float4*>(tw + row * 32 + 4 * c4);
      }
    }
    wave_lds_sync();
  }
}

// Batched images (k_planes_make_tiled below): blockIdx.y = job.
struct PlanesJob {
  const float* B;
  uint16_t* planes;
  int64_t N, K, ldb, npad, kp;
  int kmajor;
  float* slot2 = nullptr;  // max pass: a second image of the same matrix takes the same slot
};
constexpr int kPlanesBatch = 32;
struct PlanesJobs {
  PlanesJob j[kPlanesBatch];
};
// h3 planes: [2][Npad][Kp] fp16 (hi, lo of B(k, n) 2^sh), zero beyond (N, K),
// then the max |B| slot (kMaxSlotParts floats), which sets sh.  The max kernel
// gives each job one block per slot entry, each storing its partial (plain
// stores: no zeroing, no atomics).
constexpr int kHMaxParts = kMaxSlotParts;
__global__ __launch_bounds__(1024) void k_hplanes_max_batch(PlanesJobs jobs) {
  const PlanesJob& jb = jobs.j[blockIdx.y];
  // B stored [rows][cols]: rows = N (kmajor 0) or K (kmajor 1)
  const int64_t rows = jb.kmajor ? jb.K : jb.N, cols = jb.kmajor ? jb.N : jb.K;
  float m = 0.f;
  if (jb.ldb == cols && cols % 4 == 0 && (reinterpret_cast<uintptr_t>(jb.B) & 15) == 0) {
    // dense: one flat float4 range (a large image -- e.g. NT-Xent's gathered
    // columns, 8192 x 256 -- is not 64 blocks of row-serial loops)
    m = absmax4_range(reinterpret_cast<const float4*>(jb.B),
                      (int64_t)blockIdx.x * blockDim.x + threadIdx.x, rows * cols / 4,
                      (int64_t)gridDim.x * blockDim.x);
  } else {
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x)
      for (int64_t c = threadIdx.x; c < cols; c += blockDim.x)
        m = fmaxf(m, fabsf(jb.B[r * jb.ldb + c]));
  }
  m = block_max(m);
  if (threadIdx.x == 0) {
    reinterpret_cast<float*>(jb.planes + 2 * jb.npad * jb.kp)[blockIdx.x * kMaxSlotStride] = m;
    if (jb.slot2 != nullptr) jb.slot2[blockIdx.x * kMaxSlotStride] = m;
  }
}
// Weight images of both kinds in one launch per batch, 8 consecutive k of one
// n per item (16-byte stores per plane).  A K-major job (B stored [K][N]: the
// data-gradient orientation) goes through a 64 (k) x 64 (n) LDS tile, read
// as float4 runs along n and written as runs along k; a row-major one reads
// its 8 k directly.  The per-job work is block-uniform (blockIdx.y = job).
// The per-element kernels this replaces read K-major weights one cache line
// per lane (c5's images took 44.9 us a step, c2's 7.3 + 15.1); the images are
// bit-identical to torch's round-to-nearest splits of the same values
// (tests/test_gpu_kernels.py::test_weight_images_bit_exact).
constexpr int kPT = 64;  // tile edge
template <bool H3>
__device__ __forceinline__ void planes_store8(const PlanesJob& jb, int sh, int64_t n, int64_t k0,
                                              const float v[8]) {
  const int64_t ps = jb.npad * jb.kp;
  const float4 a = make_float4(v[0], v[1], v[2], v[3]), b = make_float4(v[4], v[5], v[6], v[7]);
  if constexpr (H3) {
    u32x4 h, l;
    hsplit8(a, b, sh, h, l);
    *reinterpret_cast<u32x4*>(jb.planes + n * jb.kp + k0) = h;
    *reinterpret_cast<u32x4*>(jb.planes + ps + n * jb.kp + k0) = l;
  } else {
    u32x4 h, m, l;
    split8(a, b, h, m, l);
    *reinterpret_cast<u32x4*>(jb.planes + n * jb.kp + k0) = h;
    *reinterpret_cast<u32x4*>(jb.planes + ps + n * jb.kp + k0) = m;
    *reinterpret_cast<u32x4*>(jb.planes + 2 * ps + n * jb.kp + k0) = l;
  }
}
template <bool H3>
__global__ __launch_bounds__(256) void k_planes_make_tiled(PlanesJobs jobs) {
  const PlanesJob& jb = jobs.j[blockIdx.y];
  // every lane reads the slot (a wave reduction) before any lane returns
  const int sh = H3 ? h3_shift(reinterpret_cast<const float*>(jb.planes + 2 * jb.npad * jb.kp)) : 0;
  const int tid = threadIdx.x;
  const int kc = (int)(jb.kp >> 3);  // 8-k chunks per row
  if (!jb.kmajor) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + tid;
    if (t >= jb.npad * kc) return;
    const int64_t n = t / kc, k0 = 8 * (t - n * kc);
    float v[8];
    const float* src = jb.B + n * jb.ldb + k0;
    if (n < jb.N && k0 + 8 <= jb.K && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
      const float4 a = reinterpret_cast<const float4*>(src)[0];
      const float4 b = reinterpret_cast<const float4*>(src)[1];
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t k = k0 + j;
        v[j] = (n < jb.N && k < jb.K) ? jb.B[n * jb.ldb + k] : 0.f;
      }
    }
    planes_store8<H3>(jb, sh, n, k0, v);
    return;
  }
  const int64_t tn = (jb.npad + kPT - 1) / kPT, tk = (jb.kp + kPT - 1) / kPT;
  if ((int64_t)blockIdx.x >= tn * tk) return;  // block-uniform
  const int64_t n0 = ((int64_t)blockIdx.x % tn) * kPT, k0t = ((int64_t)blockIdx.x / tn) * kPT;
  __shared__ float tile[kPT][kPT + 1];  // [k][n]
  // load: 64 k-rows x 16 float4 along n, 4 per thread
  const bool vec = (jb.ldb & 3) == 0 && (reinterpret_cast<uintptr_t>(jb.B) & 15) == 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = tid + 256 * q;
    const int kr = idx >> 4, nc = 4 * (idx & 15);
    const int64_t k = k0t + kr, n = n0 + nc;
    float e[4] = {0.f, 0.f, 0.f, 0.f};
    if (k < jb.K) {
      if (vec && n + 3 < jb.N) {
        const float4 x = *reinterpret_cast<const float4*>(jb.B + k * jb.ldb + n);
        e[0] = x.x;
        e[1] = x.y;
        e[2] = x.z;
        e[3] = x.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n + j < jb.N) e[j] = jb.B[k * jb.ldb + n + j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) tile[kr][nc + j] = e[j];
  }
  __syncthreads();
  // store: 64 n x 8 chunks of 8 k, 2 per thread
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = tid + 256 * q;
    const int nr = idx >> 3, kq = 8 * (idx & 7);
    const int64_t n = n0 + nr, k0 = k0t + kq;
    if (n >= jb.npad || k0 >= jb.kp) continue;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[kq + j][nr];
    planes_store8<H3>(jb, sh, n, k0, v);
  }
}

// blocks one launch needs for a job of k_planes_make_tiled
int64_t planes_tiled_blocks(const PlanesJob& j) {
  return j.kmajor ? ((j.npad + kPT - 1) / kPT) * ((j.kp + kPT - 1) / kPT)
                  : molclr::ceil_div(j.npad * (j.kp >> 3), 256);
}

// max |x| over a [rows][cols] (ld) fp32 matrix, folded into *slot.  A dense
// matrix (ld == cols) is one flat range, float4 when aligned; else one block
// row at a time.  No 64-bit division per element.
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ x, int64_t rows,
                                                int64_t cols, int64_t ld, float* __restrict__ slot) {
  float m = 0.f;
  if (ld == cols) {
    const int64_t n = rows * cols;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
      const int64_t n4 = n >> 2;
      m = absmax4_range(reinterpret_cast<const float4*>(x), t, n4, stride);
      for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        m = fmaxf(m, fabsf(x[i]));
    } else {
      for (; t < n; t += stride) m = fmaxf(m, fabsf(x[t]));
    }
  } else {
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x)
      for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) m = fmaxf(m, fabsf(x[r * ld + c]));
  }
  absmax_publish(m, slot);
}

// bits[w][m] bit j = (C[m][32 w + j] > 0): thread per word
__global__ __launch_bounds__(256) void k_relu_bits(const float* __restrict__ C, int64_t M,
                                                   int64_t N, int64_t ldc,
                                                   uint32_t* __restrict__ bits, int64_t words) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * words) return;
  const int64_t w = t / M, m = t - w * M;
  uint32_t b = 0;
  for (int j = 0; j < 32 && 32 * w + j < N; ++j) b |= (C[m * ldc + 32 * w + j] > 0.f ? 1u : 0u) << j;
  bits[t] = b;
}

// row maxima rowmax[r] = max_c |x[r][c]| (plain stores) and the matrix max
// folded into *slot: a wave per row, float4 columns when aligned
__global__ __launch_bounds__(256) void k_absmax_rows(const float* __restrict__ x, int64_t rows,
                                                     int64_t cols, int64_t ld,
                                                     float* __restrict__ rowmax,
                                                     float* __restrict__ slot) {
  const int lane = threadIdx.x & 63;
  const bool v4 = (cols & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  float all = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const float* xr = x + r * ld;
    float m = 0.f;
    if (v4) {
      for (int64_t c = lane; c < (cols >> 2); c += 64) {
        const float4 v = reinterpret_cast<const float4*>(xr)[c];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    } else {
      for (int64_t c = lane; c < cols; c += 64) m = fmaxf(m, fabsf(xr[c]));
    }
    m = wave_max(m);
    if (lane == 0) rowmax[r] = m;
    all = fmaxf(all, m);
  }
  if (slot != nullptr) absmax_publish(all, slot);
}

// C = epilogue(Σ_z partial[z])  (fixed order -> deterministic)
// (and colsum[m] = Σ_{z < cs_splits} cs_partial[z][m] for t < M when cs_partial is given)
template <int EPI>
__global__ void k_splitk_reduce(const float* __restrict__ partial, int splits, int64_t M, int64_t N,
                                float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                const float* __restrict__ aux, int64_t ldaux, int accumulate,
                                const float* __restrict__ cs_partial, int cs_splits,
                                float* __restrict__ colsum) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // Σ_z p[z * stride] for z < splits in order, sixteen partials in flight per round trip
  auto ordered_sum = [](const float* __restrict__ p, int64_t stride, int splits) {
    float v = 0.f;
    int z = 0;
    for (; z + 16 <= splits; z += 16) {
      float buf[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) buf[j] = p[(int64_t)(z + j) * stride];
#pragma unroll
      for (int j = 0; j < 16; ++j) v += buf[j];
    }
    float buf[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) buf[j] = z + j < splits ? p[(int64_t)(z + j) * stride] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (z + j < splits) v += buf[j];
    return v;
  };
  if (cs_partial && t < M) {
    const float c = ordered_sum(cs_partial + t, M, cs_splits);
    colsum[t] = accumulate ? colsum[t] + c : c;
  }
  if (t >= M * N) return;
  int64_t m = t / N, n = t - m * N;
  float v = ordered_sum(partial + t, M * N, splits);
  if (EPI == MOLCLR_EPI_BIAS) v = v + bias[n];
  if (EPI == MOLCLR_EPI_BIAS_RELU) v = fmaxf(v + bias[n], 0.f);
  if (EPI == MOLCLR_EPI_RELU_MASK) v = aux[m * ldaux + n] > 0.f ? v : 0.f;
  if (accumulate) v += C[m * ldc + n];
  C[m * ldc + n] = v;
}

// Two weight gradients' ordered split-K reductions in ONE launch (the GIN
// layer's dW2 and dW1: molclr_linear_wgrad_h3_pair).  Threads [0, M_a N_a)
// reduce job a, the rest job b, each exactly as k_splitk_reduce<EPI_NONE>.
// A transposed job (trans = 1: partials of C^T, [split][N][M]; N % 4 == 0,
// ldc % 4 == 0) gives a thread four columns n0..n0+3 of one row m: it reads
// each column's partials along their rows (consecutive threads, consecutive
// m) and stores the four sums as one float4 of C's row m.
struct ReduceJob {
  const float* partial;
  int splits;
  int64_t M, N;
  float* C;
  int64_t ldc;
  const float* cs_partial;
  float* colsum;
  int trans = 0;
  __host__ __device__ int64_t threads() const { return trans ? M * N / 4 : M * N; }
};
__global__ void k_splitk_reduce_pair(ReduceJob ja, ReduceJob jb, int accumulate) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool second = t >= ja.threads();
  const ReduceJob& j = second ? jb : ja;
  if (second) t -= ja.threads();
  auto ordered_sum = [](const float* __restrict__ p, int64_t stride, int splits) {
    float v = 0.f;
    int z = 0;
    for (; z + 16 <= splits; z += 16) {
      float buf[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) buf[q] = p[(int64_t)(z + q) * stride];
#pragma unroll
      for (int q = 0; q < 16; ++q) v += buf[q];
    }
    float buf[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) buf[q] = z + q < splits ? p[(int64_t)(z + q) * stride] : 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (z + q < splits) v += buf[q];
    return v;
  };
  if (j.cs_partial && t < j.M) {
    const float c = ordered_sum(j.cs_partial + t, j.M, j.splits);
    j.colsum[t] = accumulate ? j.colsum[t] + c : c;
  }
  if (t >= j.threads()) return;
  if (j.trans) {
    const int64_t n0 = 4 * (t / j.M), m = t - (n0 / 4) * j.M;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = ordered_sum(j.partial + (n0 + q) * j.M + m, j.M * j.N, j.splits);
    float4* o = reinterpret_cast<float4*>(j.C + m * j.ldc + n0);
    float4 r = make_float4(v[0], v[1], v[2], v[3]);
    if (accumulate) r = f4add(r, *o);
    *o = r;
    return;
  }
  const int64_t m = t / j.N, n = t - m * j.N;
  float v = ordered_sum(j.partial + t, j.M * j.N, j.splits);
  if (accumulate) v += j.C[m * j.ldc + n];
  j.C[m * j.ldc + n] = v;
}

// Implementations of molclr_gemm_f32 (per call, molclr_gemm_f32_impl):
// 0 = f32-input MFMA, 64 x 64 tiles; 5 (automatic) / 6 = split-bf16 "p6",
// 64 x 64 / 128 x 64.  The split-bf16 kernels stage K-major operands 4 rows
// at a time, so they need rows % 4 == 0 and ld % 4 == 0 there; other shapes
// take impl 0.
int impl_for(int64_t M, int64_t N, int64_t lda, int64_t ldb, int ak, int bk, int want) {
  if (want < 0) want = 5;
  if (want == 0) return 0;
  if (ak && (M % 4 || lda % 4)) return 0;
  if (bk && (N % 4 || ldb % 4)) return 0;
  if (want == 6 && ak) return 5;  // the K-major image is laid out for 64-row tiles
  return want;
}
// p6 tiles of a weight-gradient product (both operands K-major): 128 along the
// longer of M / N (8.9 -> ~6 VALU per MFMA: half the B or A split work)
bool p6_wide(int impl, int ak, int bk) { return impl == 5 && ak && bk; }
int tiles_for(int impl, int64_t M, int64_t N, int ak = 0, int bk = 0) {
  int64_t bm = (impl == 6 || impl == 8) ? 128 : 64, bn = (impl == 7 || impl == 8) ? 128 : 64;
  if (p6_wide(impl, ak, bk)) {
    bm = M >= N ? 128 : 64;
    bn = M >= N ? 64 : 128;
  }
  return (int)(((M + bm - 1) / bm) * ((N + bn - 1) / bn));
}

int pick_splits(int impl, int64_t M, int64_t N, int64_t K, int ak = 0, int bk = 0) {
  int64_t tiles = tiles_for(impl, M, N, ak, bk);
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
  int impl;
  const uint16_t* Bp = nullptr;  // pre-split planes (molclr_gemm_f32_bplanes)
  int64_t bps = 0;               // their plane stride
  float* colsum = nullptr;       // Σ_k A(m, k) out (molclr_linear_wgrad; K-major A, p6)
  const float* amax = nullptr;   // h3: max |A| slot (or row maxima), max |B| slot,
  const float* bmax = nullptr;   // max |C| slot and row maxima out (may be null)
  float* cmax = nullptr;
  float* crow = nullptr;
  float* amax_out = nullptr;     // q6: max |A| of the loaded rows out (may be null)
  int arow_parts = 0;            // h3 row-wise: partial row-max arrays in amax
  uint32_t* bits_out = nullptr;  // q6: C > 0 as bits out / RELU_MASK bits in
  const uint32_t* bits_in = nullptr;
  int64_t bits_ld = 0;           // words per row of both
};

template <int TM, int AMODE, int BMODE, int EPI, bool SPLIT, int TN = 1, bool CS = false>
void launch_p6(dim3 grid, hipStream_t s, const Args& a) {
  molclr::launch_timed(molclr::kTimeGemm, (k_gemm_p6<TM, TN, AMODE, BMODE, EPI, SPLIT, CS>), grid,
                       dim3(256), 0, s, a.A, a.B, a.Bp, a.C, a.M, a.N, a.K, a.lda, a.ldb, a.bps,
                       a.ldc, a.bias, a.aux, a.ldaux, a.kps, a.accumulate, a.colsum);
}

template <int WM, int WN, int TM, int TN, bool AK, bool BKM, int EPI, bool SPLIT>
void launch_t(dim3 grid, hipStream_t s, const Args& a) {
  if (a.impl == 5) {
    if constexpr (AK && BKM) {
      if (a.colsum) {
        if constexpr (EPI == MOLCLR_EPI_NONE) {
          if (a.M >= a.N) launch_p6<2, 1, 1, EPI, SPLIT, 1, true>(grid, s, a);
          else launch_p6<1, 1, 1, EPI, SPLIT, 2, true>(grid, s, a);
        }
      } else if (a.M >= a.N) {
        launch_p6<2, 1, 1, EPI, SPLIT>(grid, s, a);
      } else {
        launch_p6<1, 1, 1, EPI, SPLIT, 2>(grid, s, a);
      }
    } else {
      launch_p6<1, AK ? 1 : 0, BKM ? 1 : 0, EPI, SPLIT>(grid, s, a);
    }
    return;
  }
  if (a.impl == 6) {
    launch_p6<(AK ? 1 : 2), AK ? 1 : 0, BKM ? 1 : 0, EPI, SPLIT>(grid, s, a);
    return;
  }
  molclr::launch_timed(molclr::kTimeGemm, (k_gemm_f32<WM, WN, TM, TN, AK, BKM, EPI, SPLIT>), grid,
                       dim3(WM * WN * 64), 0, s, a.A, a.B, a.C, a.M, a.N, a.K, a.lda, a.ldb, a.ldc,
                       a.bias, a.aux, a.ldaux, a.kps, a.accumulate);
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
int dispatch(int ak, int bk, int epi, dim3 grid, hipStream_t s, const Args& a) {
  return dispatch_layout<2, 2, 1, 1, SPLIT>(ak, bk, epi, grid, s, a);
}

template <int TM, bool SPLIT, int TN = 1>
int dispatch_bplanes_t(int ak, int epi, dim3 grid, hipStream_t s, const Args& a) {
#define MOLCLR_BP_CASE(AKV, EPV)                                                               \
  if (ak == AKV && (SPLIT || epi == EPV)) {                                                    \
    launch_p6<(AKV ? 1 : TM), AKV, 2, SPLIT ? MOLCLR_EPI_NONE : EPV, SPLIT, TN>(grid, s, a); \
    return 0;                                                                                  \
  }
  if (SPLIT) {
    MOLCLR_BP_CASE(0, MOLCLR_EPI_NONE)
    MOLCLR_BP_CASE(1, MOLCLR_EPI_NONE)
  } else {
    MOLCLR_BP_CASE(0, MOLCLR_EPI_NONE)
    MOLCLR_BP_CASE(0, MOLCLR_EPI_BIAS)
    MOLCLR_BP_CASE(0, MOLCLR_EPI_BIAS_RELU)
    MOLCLR_BP_CASE(0, MOLCLR_EPI_RELU_MASK)
    MOLCLR_BP_CASE(1, MOLCLR_EPI_NONE)
    MOLCLR_BP_CASE(1, MOLCLR_EPI_BIAS)
    MOLCLR_BP_CASE(1, MOLCLR_EPI_BIAS_RELU)
    MOLCLR_BP_CASE(1, MOLCLR_EPI_RELU_MASK)
  }
#undef MOLCLR_BP_CASE
  return -1;
}

template <bool SPLIT>
int dispatch_bplanes(int impl, int ak, int epi, dim3 grid, hipStream_t s, const Args& a) {
  if (impl == 7) return dispatch_bplanes_t<1, SPLIT, 2>(ak, epi, grid, s, a);
  if (impl == 8) return dispatch_bplanes_t<2, SPLIT, 2>(ak, epi, grid, s, a);
  return impl == 6 ? dispatch_bplanes_t<2, SPLIT>(ak, epi, grid, s, a)
                   : dispatch_bplanes_t<1, SPLIT>(ak, epi, grid, s, a);
}

// Column-tile width 32 TN of the q6 / w6 kernels: the least padding of N
// (ties: the wider tile), 64 for narrow outputs.
int wide_tn(int64_t N) {
  if (N <= 64) return 2;
  const int64_t p4 = (N + 127) / 128 * 128, p5 = (N + 159) / 160 * 160;
  return p5 <= p4 ? 5 : 4;
}
int64_t q6_col_tiles(int64_t N) {
  const int64_t bn = 32 * wide_tn(N);
  return (N + bn - 1) / bn;
}
int64_t q6_blocks(int64_t M, int64_t N) {
  const int64_t bn = 32 * wide_tn(N);
  return ((M + kQ6BM - 1) / kQ6BM) * ((N + bn - 1) / bn);
}

// in-block K groups: two for narrow products (fewer than 1.5 blocks per CU)
// with at least 8 K steps, else one.  MOLCLR_Q6_GROUPS = 1 / 2 forces the
// count for products of at least 8 K steps (a diagnostic: the K-chain length
// of the fp32 sums, tools/order_spread.py).
int q6_groups(int64_t M, int64_t N, int64_t K) {
  static const int forced = [] {
    const char* e = getenv("MOLCLR_Q6_GROUPS");
    return e ? atoi(e) : 0;
  }();
  if ((K + BK - 1) / BK < 8) return 1;
  if (forced == 1 || forced == 2) return forced;
  return q6_blocks(M, N) < 384 ? 2 : 1;
}

template <int TN, int EPI, int KG, bool MASK, int H3>
void launch_q6_t(const Args& a, int64_t npad, hipStream_t s) {
  molclr::launch_timed(molclr::kTimeGemm, (k_gemm_q6<TN, EPI, KG, MASK, H3>),
                       dim3((unsigned)q6_blocks(a.M, a.N)), dim3(KG * 64 * kQ6Waves), 0, s, a.A,
                       a.Bp, a.C, a.M, a.N, a.K, a.lda, a.ldb, npad, a.ldc, a.bias, a.aux, a.ldaux,
                       a.accumulate, a.amax, a.bmax, a.cmax, a.crow, a.amax_out, a.arow_parts,
                       a.bits_out, a.bits_in, a.bits_ld);
}
// the ping-pong form: one K group, five-block tiles, byte ranges within the
// buffer descriptors' 31-bit records (MOLCLR_Q6_PP=0 keeps k_gemm_q6)
bool q6_pp_ok(const Args& a, int64_t npad, int tn, int kg, int h3) {
  static const int off = [] {
    const char* e = getenv("MOLCLR_Q6_PP");
    return e && e[0] == '0';
  }();
  const int64_t kp = (a.K + BK - 1) / BK * BK;
  // narrow h3 products (<= 2 column tiles: 30 MFMAs per phase over 19 steps
  // at K = 600) measured slower in the step (dagg 53.0 -> 57.9 us): q6
  static const bool narrow = [] {
    const char* e = getenv("MOLCLR_PP_NARROW");
    return e != nullptr && e[0] == '1';
  }();
  if (h3 && a.N <= 320 && !narrow) return false;
  return !off && kg == 1 && tn == 5 && a.M * a.lda * 4 < (1ll << 31) &&
         (int64_t)(h3 ? 2 : 3) * npad * kp * 2 < (1ll << 31) && a.lda % 4 == 0;
}
// the h3 products take k_gemm_pp's swapped register epilogue; MOLCLR_PP_SWAP=0
// keeps the LDS-transpose epilogue
bool pp_swap() {
  static const bool on = [] {
    const char* e = getenv("MOLCLR_PP_SWAP");
    return !(e != nullptr && e[0] == '0');
  }();
  return on;
}
template <int TN, int EPI, int H3>
void launch_pp(const Args& a, int64_t npad, hipStream_t s) {
  const int64_t bn = 32 * TN;
  const int64_t blocks = ((a.M + kPPRows - 1) / kPPRows) * ((a.N + bn - 1) / bn);
  auto kern = (H3 != 0 && pp_swap()) ? k_gemm_pp<TN, EPI, H3, H3 != 0> : k_gemm_pp<TN, EPI, H3, false>;
  molclr::launch_timed(molclr::kTimeGemm, kern, dim3((unsigned)blocks),
                       dim3(512), 0, s, a.A, a.Bp, a.C, a.M, a.N, a.K, a.lda, a.ldb, npad, a.ldc,
                       a.bias, a.aux, a.ldaux, a.accumulate, a.amax, a.bmax, a.cmax, a.crow,
                       a.amax_out, a.arow_parts, a.bits_out, a.bits_in, a.bits_ld);
}
template <int TN, int EPI, int H3>
void launch_q6(const Args& a, int64_t npad, hipStream_t s) {
  const int64_t nsteps = (a.K + BK - 1) / BK;
  const int kg = q6_groups(a.M, a.N, a.K);
  if constexpr (TN == 5) {
    if (q6_pp_ok(a, npad, TN, kg, H3)) {
      launch_pp<TN, EPI, H3>(a, npad, s);
      return;
    }
  }
  // steps that need their A tail zeroed: a partial last step, or rounds past
  // the end for some K groups
  const bool mask = a.K % BK != 0 || nsteps % kg != 0;
  if (kg == 2) {
    if (mask) launch_q6_t<TN, EPI, 2, true, H3>(a, npad, s);
    else launch_q6_t<TN, EPI, 2, false, H3>(a, npad, s);
  } else {
    if (mask) launch_q6_t<TN, EPI, 1, true, H3>(a, npad, s);
    else launch_q6_t<TN, EPI, 1, false, H3>(a, npad, s);
  }
}

template <int TN, int H3>
int dispatch_q6(int epi, const Args& a, int64_t npad, hipStream_t s) {
  switch (epi) {
    case MOLCLR_EPI_NONE: launch_q6<TN, MOLCLR_EPI_NONE, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_BIAS: launch_q6<TN, MOLCLR_EPI_BIAS, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_BIAS_RELU: launch_q6<TN, MOLCLR_EPI_BIAS_RELU, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_RELU_MASK: launch_q6<TN, MOLCLR_EPI_RELU_MASK, H3>(a, npad, s); return 0;
    default: return -1;
  }
}

// a.ldb = kp (the planes' row pitch), a.Bp = the planes; h3 1 / 2: fp16
// two-part planes, a.amax (a slot / row maxima) and a.bmax set
template <int H3>
int dispatch_q6_tn(int epi, const Args& a, int64_t npad, hipStream_t s) {
  const int tn = wide_tn(a.N);
  return tn == 5 ? dispatch_q6<5, H3>(epi, a, npad, s)
         : tn == 4 ? dispatch_q6<4, H3>(epi, a, npad, s)
                   : dispatch_q6<2, H3>(epi, a, npad, s);
}
// The h3 products k_gemm_bs takes: K in (288, 304] (its LDS image), wide
// (> 320 columns), float4-aligned C, ReLU masks as bits, row maxima as a slot,
// <= 8 partial arrays or per-wave pairs.  MOLCLR_GEMM_BS=0 keeps pp / q6;
// g_bs_force (molclr_gemm_f32_h3_impl): 1 never, 2 bs, 3 bs16.
int g_bs_force = 0;
bool bs_shape_ok(const Args& a, int64_t npad, int epi, int h3) {
  if (h3 == 0 || a.N <= 320 || a.K <= 288 || a.K > 304 || a.ldb != 320) return false;
  if (a.lda % 4 || a.ldc % 4 || a.N % 4 || (reinterpret_cast<uintptr_t>(a.C) & 15)) return false;
  if (a.M * a.lda * 4 >= (1ll << 31) || 2 * npad * a.ldb * 2 >= (1ll << 31)) return false;
  if (epi == MOLCLR_EPI_RELU_MASK && a.bits_in == nullptr) return false;
  if (h3 == 2 && (a.arow_parts > 8 || (a.arow_parts < 0 && -a.arow_parts < 64))) return false;
  return true;
}
bool use_bs(const Args& a, int64_t npad, int epi, int h3) {
  static const bool off = [] {
    const char* e = getenv("MOLCLR_GEMM_BS");
    return e != nullptr && e[0] == '0';
  }();
  if (g_bs_force == 1 || (off && g_bs_force < 2)) return false;
  return bs_shape_ok(a, npad, epi, h3);
}
// k_gemm_bs16 (default) or k_gemm_bs: MOLCLR_GEMM_BS16=0 or g_bs_force 2
// (molclr_gemm_f32_h3_impl 2) takes the 32 x 32 x 16 form, g_bs_force 3 bs16
bool use_bs16() {
  static const bool off = [] {
    const char* e = getenv("MOLCLR_GEMM_BS16");
    return e != nullptr && e[0] == '0';
  }();
  return g_bs_force == 3 || (g_bs_force != 2 && !off);
}
template <int EPI, int H3>
void launch_bs(const Args& a, int64_t npad, hipStream_t s) {
  const int ntn = (int)((a.N + kBN - 1) / kBN);
  int groups = molclr::cu_count() / ntn;
  groups = groups < 1 ? 1 : groups;
  // three waves per SIMD (<= 168 VGPRs): the c2 step 187.1k molecules/s
  // against 186.1k at two (MOLCLR_BS16_WAVES=8) and 180.8k on k_gemm_bs
  // (same box, round 6)
  static const int w16 = [] {
    const char* e = getenv("MOLCLR_BS16_WAVES");
    return e != nullptr && atoi(e) == 8 ? 8 : 12;
  }();
  if (use_bs16() && w16 == 12)
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_bsn<EPI, H3, 10, true, 12>),
                         dim3((unsigned)(ntn * groups)), dim3(768), 0, s, a.A, a.Bp, a.C, a.M, a.N,
                         a.K, a.lda, a.ldb, npad, a.ldc, a.bias, a.aux, a.ldaux, a.accumulate, a.amax,
                         a.bmax, a.cmax, a.crow, a.amax_out, a.arow_parts, a.bits_out, a.bits_in,
                         a.bits_ld, ntn, groups);
  else if (use_bs16())
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_bsn<EPI, H3, 10, true>),
                         dim3((unsigned)(ntn * groups)), dim3(512), 0, s, a.A, a.Bp, a.C, a.M, a.N,
                         a.K, a.lda, a.ldb, npad, a.ldc, a.bias, a.aux, a.ldaux, a.accumulate, a.amax,
                         a.bmax, a.cmax, a.crow, a.amax_out, a.arow_parts, a.bits_out, a.bits_in,
                         a.bits_ld, ntn, groups);
  else
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_bs<EPI, H3, 10, true>),
                         dim3((unsigned)(ntn * groups)), dim3(512), 0, s, a.A, a.Bp, a.C, a.M, a.N,
                         a.K, a.lda, a.ldb, npad, a.ldc, a.bias, a.aux, a.ldaux, a.accumulate, a.amax,
                         a.bmax, a.cmax, a.crow, a.amax_out, a.arow_parts, a.bits_out, a.bits_in,
                         a.bits_ld, ntn, groups);
}
template <int H3>
int dispatch_bs(int epi, const Args& a, int64_t npad, hipStream_t s) {
  switch (epi) {
    case MOLCLR_EPI_NONE: launch_bs<MOLCLR_EPI_NONE, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_BIAS: launch_bs<MOLCLR_EPI_BIAS, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_BIAS_RELU: launch_bs<MOLCLR_EPI_BIAS_RELU, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_RELU_MASK: launch_bs<MOLCLR_EPI_RELU_MASK, H3>(a, npad, s); return 0;
    default: return -1;
  }
}
// The K = 600 products (lin2 = a1 W2^T and dagg = dz1 W1 of the c2 layer,
// N = 300) on k_gemm_bsn with 64-column tiles: K in (576, 608], N <= 320, no
// row maxima or ReLU bits out (their partial layouts are q6's), the rest as
// bs_shape_ok.  c2 step, same box, round 6: k_gemm_q6 185.1k / 185.2k
// molecules/s, bsn-64 at 12 waves 185.4k / 185.6k, at 8 waves 186.2k / 186.0k
// (16 waves measured slower on another box), so 8 waves is the default;
// MOLCLR_GEMM_BS64=0 keeps q6.
bool use_bs64(const Args& a, int64_t npad, int epi, int h3) {
  static const bool off = [] {
    const char* e = getenv("MOLCLR_GEMM_BS64");
    return e != nullptr && e[0] == '0';
  }();
  if (g_bs_force == 1 || g_bs_force == 2 || (off && g_bs_force != 3)) return false;
  if (h3 == 0 || a.N > 320 || a.N <= 192 || a.K <= 576 || a.K > 608 || a.ldb != 608) return false;
  if (a.crow != nullptr || a.bits_out != nullptr) return false;
  if (a.lda % 4 || a.ldc % 4 || a.N % 4 || (reinterpret_cast<uintptr_t>(a.C) & 15)) return false;
  if (a.M * a.lda * 4 >= (1ll << 31) || 2 * npad * a.ldb * 2 >= (1ll << 31)) return false;
  if (epi == MOLCLR_EPI_RELU_MASK && a.bits_in == nullptr) return false;
  if (h3 == 2 && (a.arow_parts > 8 || (a.arow_parts < 0 && -a.arow_parts < 64))) return false;
  return true;
}
template <int EPI, int H3>
void launch_bs64(const Args& a, int64_t npad, hipStream_t s) {
  const int ntn = (int)((a.N + 63) / 64);
  int groups = molclr::cu_count() / ntn;
  groups = groups < 1 ? 1 : groups;
  // MOLCLR_BS64_WAVES=12 / 16: three / four waves per SIMD (<= 128 VGPRs)
  static const int wv = [] {
    const char* e = getenv("MOLCLR_BS64_WAVES");
    const int v = e != nullptr ? atoi(e) : 8;
    return v == 16 || v == 12 ? v : 8;
  }();
  if (wv == 8)
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_bsn<EPI, H3, 19, false, 8, 64>),
                         dim3((unsigned)(ntn * groups)), dim3(512), 0, s, a.A, a.Bp, a.C, a.M, a.N,
                         a.K, a.lda, a.ldb, npad, a.ldc, a.bias, a.aux, a.ldaux, a.accumulate,
                         a.amax, a.bmax, a.cmax, a.crow, a.amax_out, a.arow_parts, a.bits_out,
                         a.bits_in, a.bits_ld, ntn, groups);
  else if (wv == 16)
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_bsn<EPI, H3, 19, false, 16, 64>),
                         dim3((unsigned)(ntn * groups)), dim3(1024), 0, s, a.A, a.Bp, a.C, a.M, a.N,
                         a.K, a.lda, a.ldb, npad, a.ldc, a.bias, a.aux, a.ldaux, a.accumulate,
                         a.amax, a.bmax, a.cmax, a.crow, a.amax_out, a.arow_parts, a.bits_out,
                         a.bits_in, a.bits_ld, ntn, groups);
  else
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_bsn<EPI, H3, 19, false, 12, 64>),
                         dim3((unsigned)(ntn * groups)), dim3(768), 0, s, a.A, a.Bp, a.C, a.M, a.N,
                         a.K, a.lda, a.ldb, npad, a.ldc, a.bias, a.aux, a.ldaux, a.accumulate,
                         a.amax, a.bmax, a.cmax, a.crow, a.amax_out, a.arow_parts, a.bits_out,
                         a.bits_in, a.bits_ld, ntn, groups);
}
template <int H3>
int dispatch_bs64(int epi, const Args& a, int64_t npad, hipStream_t s) {
  switch (epi) {
    case MOLCLR_EPI_NONE: launch_bs64<MOLCLR_EPI_NONE, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_BIAS: launch_bs64<MOLCLR_EPI_BIAS, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_BIAS_RELU: launch_bs64<MOLCLR_EPI_BIAS_RELU, H3>(a, npad, s); return 0;
    case MOLCLR_EPI_RELU_MASK: launch_bs64<MOLCLR_EPI_RELU_MASK, H3>(a, npad, s); return 0;
    default: return -1;
  }
}
// partial row-max arrays of an h3 product's C (crow): one per 128 columns for
// the wide products (k_gemm_bs's tiles); pp / q6, whose tiles may be 160
// wide, zero the arrays they do not write
int64_t crow_parts(int64_t N) { return N > 320 ? (N + kBN - 1) / kBN : q6_col_tiles(N); }

int run_q6(const Args& a, int64_t npad, int epi, hipStream_t s, int h3 = 0) {
  if (h3 != 0 && use_bs(a, npad, epi, h3)) {
    const int rc = h3 == 2 ? dispatch_bs<2>(epi, a, npad, s) : dispatch_bs<1>(epi, a, npad, s);
    if (rc) {
      molclr::set_error("gemm_f32_h3: no bs kernel for epilogue %d", epi);
      return MOLCLR_ERR_UNSUPPORTED;
    }
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  if (h3 != 0 && use_bs64(a, npad, epi, h3)) {
    const int rc = h3 == 2 ? dispatch_bs64<2>(epi, a, npad, s) : dispatch_bs64<1>(epi, a, npad, s);
    if (rc) {
      molclr::set_error("gemm_f32_h3: no bs64 kernel for epilogue %d", epi);
      return MOLCLR_ERR_UNSUPPORTED;
    }
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  if (g_bs_force >= 2) {
    molclr::set_error("gemm_f32_h3_impl: the bs kernel does not take this product");
    return MOLCLR_ERR_UNSUPPORTED;
  }
  if (a.crow != nullptr && crow_parts(a.N) > q6_col_tiles(a.N)) {
    const int64_t w = q6_col_tiles(a.N);
    const hipError_t e = molclr::zero_async(a.crow + w * a.M,
                                            (size_t)(crow_parts(a.N) - w) * a.M * sizeof(float), s);
    if (e != hipSuccess) return (int)e;
  }
  const int rc = h3 == 2   ? dispatch_q6_tn<2>(epi, a, npad, s)
                 : h3 == 1 ? dispatch_q6_tn<1>(epi, a, npad, s)
                           : dispatch_q6_tn<0>(epi, a, npad, s);
  if (rc) {
    molclr::set_error("gemm_f32_bplanes: no q6 kernel for epilogue %d", epi);
    return MOLCLR_ERR_UNSUPPORTED;
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

// w6: tile width as q6, K split over <= 512 4-wave groups (two per CU; 384 / 256
// single-group blocks measured 8 % / 40 % slower with the partial reduction
// included), each group at least 4 K tiles deep.  kg = 2 (default): two
// groups per block, ~256 blocks; kg = 1: ~512 one-group blocks.
struct W6Plan {
  int tn, splits, kps, kg;
  int64_t ntiles;
};
W6Plan w6_plan(int64_t M, int64_t N, int64_t K, int kg) {
  W6Plan p;
  p.tn = wide_tn(N);
  p.kg = kg;
  p.ntiles = ((M + kW6BM - 1) / kW6BM) * ((N + 32 * p.tn - 1) / (32 * p.tn));
  const int64_t nk = (K + BK - 1) / BK;
  // whole waves of blocks only: a block past 512 / kg (one per CU at kg = 2)
  // would run alone after the rest
  int64_t s = (512 / p.kg) / p.ntiles;
  if (s > nk / (4 * p.kg)) s = nk / (4 * p.kg);
  if (s < 1) s = 1;
  p.kps = (int)((nk + s - 1) / s);
  p.splits = (int)((nk + p.kps - 1) / p.kps);
  return p;
}
// shapes w6 takes: 4-aligned rows (float4 staging of K-major operands, float4
// partial stores) and a long K (the weight-gradient shape)
bool w6_shape_ok(int64_t M, int64_t N, int64_t K) {
  return M % 4 == 0 && N % 4 == 0 && K >= 1024 && M * N < (1ll << 28);
}
// sized for the larger of the two group settings (molclr_linear_wgrad_groups
// takes either with the same workspace query)
size_t w6_ws_bytes(int64_t M, int64_t N, int64_t K, bool colsum) {
  size_t need = 0;
  for (int kg = 1; kg <= 2; ++kg)
    for (int tr = 0; tr < 2; ++tr) {  // and the transposed plan (w6_transposed)
      const W6Plan p = tr ? w6_plan(N, M, K, kg) : w6_plan(M, N, K, kg);
      const size_t b = (size_t)p.splits * (M * N + (colsum ? M : 0)) * sizeof(float) + 256;
      need = b > need ? b : need;
    }
  return need;
}

template <int TN, int KG, bool H3>
void launch_w6_kg(const W6Plan& p, hipStream_t s, const float* A, const float* B, float* part,
                  int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, float* cs_part,
                  const float* amax, const float* bmax, bool cs_b) {
  const dim3 grid((unsigned)(p.ntiles * p.splits));
  if (cs_part && cs_b)
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_w6<TN, 2, KG, H3>), grid, dim3(256 * KG), 0,
                         s, A, B, part, M, N, K, lda, ldb, p.kps, p.splits, cs_part, amax, bmax);
  else if (cs_part)
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_w6<TN, 1, KG, H3>), grid, dim3(256 * KG), 0,
                         s, A, B, part, M, N, K, lda, ldb, p.kps, p.splits, cs_part, amax, bmax);
  else
    molclr::launch_timed(molclr::kTimeGemm, (k_gemm_w6<TN, 0, KG, H3>), grid, dim3(256 * KG),
                         0, s, A, B, part, M, N, K, lda, ldb, p.kps, p.splits, cs_part, amax, bmax);
}
template <int TN, bool H3>
void launch_w6(const W6Plan& p, hipStream_t s, const float* A, const float* B, float* part,
               int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, float* cs_part,
               const float* amax, const float* bmax, bool cs_b = false) {
  if (p.kg == 2)
    launch_w6_kg<TN, 2, H3>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax, cs_b);
  else
    launch_w6_kg<TN, 1, H3>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax, cs_b);
}

// C (+)= A^T B over K-major A [K][M] (lda) and B [K][N] (ldb); colsum (+)= Σ_k A
// when non-null.  Partial tiles in the workspace, then the fixed-order reduce.
// amax / bmax given: the h3 form (both max slots needed).
int run_w6(const float* A, const float* B, float* C, float* colsum, int64_t M, int64_t N,
           int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int accumulate, void* ws,
           size_t ws_bytes, hipStream_t s, int kg = 2, const float* amax = nullptr,
           const float* bmax = nullptr) {
  const W6Plan p = w6_plan(M, N, K, kg);
  MOLCLR_REQUIRE_WS(ws_bytes, w6_ws_bytes(M, N, K, colsum != nullptr));
  float* part = static_cast<float*>(ws);
  float* cs_part = colsum ? part + (size_t)p.splits * M * N : nullptr;
  if (amax) {
    if (p.tn == 5) launch_w6<5, true>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax);
    else if (p.tn == 4) launch_w6<4, true>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax);
    else launch_w6<2, true>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax);
  } else {
    if (p.tn == 5) launch_w6<5, false>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax);
    else if (p.tn == 4) launch_w6<4, false>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax);
    else launch_w6<2, false>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax);
  }
  const float* no_f = nullptr;
  molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_NONE>,
                       dim3((unsigned)molclr::ceil_div(M * N, 256)), dim3(256), 0, s,
                       static_cast<const float*>(part), p.splits, M, N, C, ldc, no_f, no_f,
                       (int64_t)0, accumulate, static_cast<const float*>(cs_part), p.splits, colsum);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

int64_t planes_npad(int64_t N) { return (N + kPlanesRowPad - 1) / kPlanesRowPad * kPlanesRowPad; }
int64_t planes_kp(int64_t K) { return (K + BK - 1) / BK * BK; }

// Launches the main GEMM (split-K when it pays) and the split-K reduction.
// `bp` selects the pre-split-B kernels.
int run_gemm(const Args& a0, int impl, bool bp, int a_kmajor, int b_kmajor, int epilogue,
             void* workspace, size_t workspace_bytes, hipStream_t s) {
  const int64_t M = a0.M, N = a0.N, K = a0.K;
  int64_t tiles = tiles_for(impl, M, N, a_kmajor, b_kmajor);  // workgroups along x
  MOLCLR_REQUIRE(tiles < (1ll << 31), "gemm_f32: too many tiles");
  int sp = pick_splits(impl, M, N, K, a_kmajor, b_kmajor);
  const size_t cs_floats = a0.colsum ? (size_t)M : 0;  // per split
  if (sp > 1 && workspace_bytes < (size_t)sp * (M * N + cs_floats) * sizeof(float)) sp = 1;
  Args a = a0;
  a.impl = impl;
  int rc;
  if (sp == 1) {
    rc = bp ? dispatch_bplanes<false>(impl, a_kmajor, epilogue, dim3((unsigned)tiles), s, a)
            : dispatch<false>(a_kmajor != 0, b_kmajor != 0, epilogue, dim3((unsigned)tiles), s, a);
  } else {
    int64_t nk = (K + BK - 1) / BK;
    int kps = (int)((nk + sp - 1) / sp);
    sp = (int)((nk + kps - 1) / kps);
    float* partial = (float*)workspace;
    float* cs_partial = a.colsum ? partial + (size_t)sp * M * N : nullptr;
    Args ap = a;
    ap.C = partial;
    ap.colsum = cs_partial;
    ap.ldc = N;
    ap.bias = nullptr;
    ap.aux = nullptr;
    ap.ldaux = 0;
    ap.kps = kps;
    ap.accumulate = 0;
    rc = bp ? dispatch_bplanes<true>(impl, a_kmajor, MOLCLR_EPI_NONE, dim3((unsigned)tiles, sp), s, ap)
            : dispatch<true>(a_kmajor != 0, b_kmajor != 0, MOLCLR_EPI_NONE,
                             dim3((unsigned)tiles, sp), s, ap);
    if (rc == 0) {
      dim3 g((unsigned)molclr::ceil_div(M * N, 256));
      float* C = a.C;
      const int64_t ldc = a.ldc, ldaux = a.ldaux;
      const float *bias = a.bias, *aux = a.aux;
      const int accumulate = a.accumulate;
      switch (epilogue) {
        case MOLCLR_EPI_NONE:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_NONE>, g, dim3(256), 0, s,
                               partial, sp, M, N, C, ldc, bias, aux, ldaux, accumulate, cs_partial, sp, a.colsum);
          break;
        case MOLCLR_EPI_BIAS:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_BIAS>, g, dim3(256), 0, s,
                               partial, sp, M, N, C, ldc, bias, aux, ldaux, accumulate, cs_partial, sp, a.colsum);
          break;
        case MOLCLR_EPI_BIAS_RELU:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_BIAS_RELU>, g, dim3(256), 0,
                               s, partial, sp, M, N, C, ldc, bias, aux, ldaux, accumulate, cs_partial, sp, a.colsum);
          break;
        default:
          molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_RELU_MASK>, g, dim3(256), 0,
                               s, partial, sp, M, N, C, ldc, bias, aux, ldaux, accumulate, cs_partial, sp, a.colsum);
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

}  // namespace

void molclr_splitk_reduce_none(const float* partial, int splits, int64_t M, int64_t N, float* C,
                               int64_t ldc, int accumulate, const float* cs_partial,
                               int cs_splits, float* colsum, hipStream_t s) {
  const float* no_f = nullptr;
  molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce<MOLCLR_EPI_NONE>,
                       dim3((unsigned)molclr::ceil_div(M * N > M ? M * N : M, 256)), dim3(256), 0,
                       s, partial, splits, M, N, C, ldc, no_f, no_f, (int64_t)0, accumulate,
                       cs_partial, cs_splits, colsum);
}

MOLCLR_API size_t molclr_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  // sized for the largest split count any implementation would pick
  int sp = pick_splits(0, M, N, K);
  for (int impl = 5; impl <= 8; ++impl) {
    const int s2 = pick_splits(impl, M, N, K);
    sp = s2 > sp ? s2 : sp;
  }
  const int s3 = pick_splits(5, M, N, K, 1, 1);  // the 128-wide weight-gradient tiles
  sp = s3 > sp ? s3 : sp;
  size_t need = sp > 1 ? (size_t)sp * M * N * sizeof(float) + 256 : 0;
  if (w6_shape_ok(M, N, K)) {  // both operands K-major: k_gemm_w6 partials
    const size_t w6 = w6_ws_bytes(M, N, K, false);
    need = w6 > need ? w6 : need;
  }
  return need;
}

MOLCLR_API int molclr_gemm_f32_impl(const float* A, const float* B, float* C, int64_t M, int64_t N,
                                    int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor,
                                    int b_kmajor, int epilogue_flags, const float* bias,
                                    const float* aux, int64_t ldaux, void* workspace,
                                    size_t workspace_bytes, molclr_stream_t stream, int impl_req) {
  const int accumulate = (epilogue_flags & MOLCLR_EPI_ACCUMULATE) ? 1 : 0;
  const int epilogue = epilogue_flags & ~MOLCLR_EPI_ACCUMULATE;
  MOLCLR_REQUIRE(impl_req == -1 || impl_req == 0 || impl_req == 5 || impl_req == 6,
                 "gemm_f32: impl %d (-1 automatic, 0, 5, 6)", impl_req);
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
  const int impl = impl_for(M, N, lda, ldb, a_kmajor, b_kmajor, impl_req);
  // a weight-gradient product (both operands K-major, long K): k_gemm_w6
  if (impl_req == -1 && impl == 5 && a_kmajor && b_kmajor && epilogue == MOLCLR_EPI_NONE &&
      w6_shape_ok(M, N, K) && lda % 4 == 0 && ldb % 4 == 0 &&
      workspace_bytes >= w6_ws_bytes(M, N, K, false))
    return run_w6(A, B, C, nullptr, M, N, K, lda, ldb, ldc, accumulate, workspace,
                  workspace_bytes, s);
  Args a{A, B, C, M, N, K, lda, ldb, ldc, bias, aux, ldaux, 0, accumulate, impl};
  return run_gemm(a, impl, false, a_kmajor, b_kmajor, epilogue, workspace, workspace_bytes, s);
}

MOLCLR_API int molclr_gemm_f32(const float* A, const float* B, float* C, int64_t M, int64_t N,
                               int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor,
                               int b_kmajor, int epilogue_flags, const float* bias, const float* aux,
                               int64_t ldaux, void* workspace, size_t workspace_bytes,
                               molclr_stream_t stream) {
  return molclr_gemm_f32_impl(A, B, C, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor, epilogue_flags,
                              bias, aux, ldaux, workspace, workspace_bytes, stream, -1);
}

MOLCLR_API size_t molclr_bplanes_bytes(int64_t N, int64_t K) {
  return (size_t)3 * planes_npad(N) * planes_kp(K) * sizeof(uint16_t);
}

MOLCLR_API int molclr_bplanes_make(const float* B, int64_t N, int64_t K, int64_t ldb, int b_kmajor,
                                   uint16_t* planes, molclr_stream_t stream) {
  MOLCLR_REQUIRE(N > 0 && K > 0 && B && planes, "bplanes_make: empty or null operand");
  MOLCLR_REQUIRE(b_kmajor ? ldb >= N : ldb >= K, "bplanes_make: leading dimension too small");
  PlanesJobs jobs{};
  jobs.j[0] = PlanesJob{B, planes, N, K, ldb, planes_npad(N), planes_kp(K), b_kmajor};
  hipLaunchKernelGGL(k_planes_make_tiled<false>, dim3((unsigned)planes_tiled_blocks(jobs.j[0]), 1),
                     dim3(256), 0, molclr::as_stream(stream), jobs);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_bplanes_make_batch(int count, const float* const* B, const int64_t* N,
                                         const int64_t* K, const int64_t* ldb,
                                         const int* b_kmajor, uint16_t* const* planes,
                                         molclr_stream_t stream) {
  MOLCLR_REQUIRE(count >= 0 && (count == 0 || (B && N && K && ldb && b_kmajor && planes)),
                 "bplanes_make_batch: null arrays");
  for (int base = 0; base < count; base += kPlanesBatch) {
    PlanesJobs jobs{};
    const int n = count - base < kPlanesBatch ? count - base : kPlanesBatch;
    int64_t most = 0;
    for (int i = 0; i < n; ++i) {
      const int q = base + i;
      MOLCLR_REQUIRE(N[q] > 0 && K[q] > 0 && B[q] && planes[q],
                     "bplanes_make_batch: job %d empty or null", q);
      MOLCLR_REQUIRE(b_kmajor[q] ? ldb[q] >= N[q] : ldb[q] >= K[q],
                     "bplanes_make_batch: job %d leading dimension too small", q);
      jobs.j[i] = PlanesJob{B[q], planes[q], N[q], K[q], ldb[q], planes_npad(N[q]), planes_kp(K[q]),
                            b_kmajor[q]};
      const int64_t e = planes_tiled_blocks(jobs.j[i]);
      most = e > most ? e : most;
    }
    hipLaunchKernelGGL(k_planes_make_tiled<false>, dim3((unsigned)most, (unsigned)n), dim3(256), 0,
                       molclr::as_stream(stream), jobs);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_gemm_f32_bplanes_tile(const float* A, const uint16_t* planes, float* C,
                                            int64_t M, int64_t N, int64_t K, int64_t lda,
                                            int64_t ldc, int a_kmajor, int epilogue_flags,
                                            const float* bias, const float* aux, int64_t ldaux,
                                            void* workspace, size_t workspace_bytes,
                                            molclr_stream_t stream, int tile) {
  const int accumulate = (epilogue_flags & MOLCLR_EPI_ACCUMULATE) ? 1 : 0;
  const int epilogue = epilogue_flags & ~MOLCLR_EPI_ACCUMULATE;
  MOLCLR_REQUIRE(tile == 0 || (tile >= 5 && tile <= 9),
                 "gemm_f32_bplanes: tile %d (0 automatic, 5..9)", tile);
  MOLCLR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_f32_bplanes: negative size");
  MOLCLR_REQUIRE(epilogue >= MOLCLR_EPI_NONE && epilogue <= MOLCLR_EPI_RELU_MASK,
                 "gemm_f32_bplanes: bad epilogue %d", epilogue);
  MOLCLR_REQUIRE((epilogue != MOLCLR_EPI_BIAS && epilogue != MOLCLR_EPI_BIAS_RELU) || bias,
                 "gemm_f32_bplanes: bias epilogue needs bias");
  MOLCLR_REQUIRE(epilogue != MOLCLR_EPI_RELU_MASK || aux,
                 "gemm_f32_bplanes: relu-mask epilogue needs aux");
  MOLCLR_REQUIRE(a_kmajor ? (M % 4 == 0 && lda % 4 == 0 && lda >= M)
                          : (K % 4 == 0 && lda % 4 == 0 && lda >= K),
                 "gemm_f32_bplanes: A needs 4-aligned rows (K-major) or K (K contiguous)");
  MOLCLR_REQUIRE(ldc >= N, "gemm_f32_bplanes: ldc < N");
  if (M == 0 || N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(K > 0 && A && planes && C, "gemm_f32_bplanes: null operand or K == 0");
  const int64_t npad = planes_npad(N), kp = planes_kp(K);
  // automatic: q6 for a row-major A whose row tiles fill the chip, else p6
  // (64 x 128 for N >= 512, else 64 x 64; split-K when it pays)
  int impl = tile;
  if (impl == 0) impl = (!a_kmajor && q6_blocks(M, N) >= 128) ? 9 : (N >= 512 ? 7 : 5);
  if (impl == 9 && (a_kmajor || K > kQ6MaxK || 3 * npad * kp >= (1ll << 31) ||
                    q6_blocks(M, N) >= (1ll << 31)))
    impl = N >= 512 ? 7 : 5;
  if ((impl == 6 || impl == 8) && a_kmajor) impl = 5;
  Args a{A, nullptr, C, M, N, K, lda, kp, ldc, bias, aux, ldaux, 0, accumulate, impl};
  a.Bp = planes;
  a.bps = npad * kp;
  if (impl == 9) return run_q6(a, npad, epilogue, molclr::as_stream(stream));
  return run_gemm(a, impl, true, a_kmajor, 0, epilogue, workspace, workspace_bytes,
                  molclr::as_stream(stream));
}

MOLCLR_API int molclr_gemm_f32_bplanes_max(const float* A, const uint16_t* planes, float* C,
                                           int64_t M, int64_t N, int64_t K, int64_t lda,
                                           int64_t ldc, int epilogue_flags, const float* bias,
                                           const float* aux, int64_t ldaux, float* amax_out,
                                           float* cmax, float* crow, uint32_t* relu_bits,
                                           void* workspace, size_t workspace_bytes,
                                           molclr_stream_t stream) {
  const int accumulate = (epilogue_flags & MOLCLR_EPI_ACCUMULATE) ? 1 : 0;
  const int epilogue = epilogue_flags & ~MOLCLR_EPI_ACCUMULATE;
  MOLCLR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_f32_bplanes_max: negative size");
  MOLCLR_REQUIRE(epilogue >= MOLCLR_EPI_NONE && epilogue <= MOLCLR_EPI_RELU_MASK,
                 "gemm_f32_bplanes_max: bad epilogue %d", epilogue);
  MOLCLR_REQUIRE((epilogue != MOLCLR_EPI_BIAS && epilogue != MOLCLR_EPI_BIAS_RELU) || bias,
                 "gemm_f32_bplanes_max: bias epilogue needs bias");
  MOLCLR_REQUIRE(epilogue != MOLCLR_EPI_RELU_MASK || aux,
                 "gemm_f32_bplanes_max: relu-mask epilogue needs aux");
  MOLCLR_REQUIRE(K % 4 == 0 && lda % 4 == 0 && lda >= K && ldc >= N && K <= kQ6MaxK,
                 "gemm_f32_bplanes_max: K (<= %lld) and lda multiples of 4, lda >= K, ldc >= N",
                 (long long)kQ6MaxK);
  if (M == 0 || N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(K > 0 && A && planes && C, "gemm_f32_bplanes_max: null operand or K == 0");
  const int64_t npad = planes_npad(N), kp = planes_kp(K);
  MOLCLR_REQUIRE(3 * npad * kp < (1ll << 31) && q6_blocks(M, N) < (1ll << 31),
                 "gemm_f32_bplanes_max: too large");
  hipStream_t s = molclr::as_stream(stream);
  if (q6_blocks(M, N) < 128) {
    // molclr_gemm_f32_bplanes' automatic tile is not q6 here: run it (same
    // kernel, same result as the plain call), then the max passes; crow's
    // parts all get the full row maxima
    MOLCLR_TRY_RC(molclr_gemm_f32_bplanes(A, planes, C, M, N, K, lda, ldc, 0, epilogue_flags, bias,
                                          aux, ldaux, workspace, workspace_bytes, stream));
    if (amax_out) MOLCLR_TRY_RC(molclr_absmax_f32(A, M, K, lda, amax_out, 1, stream));
    if (relu_bits) {
      const int64_t words = (N + 31) / 32;
      hipLaunchKernelGGL(k_relu_bits, dim3((unsigned)molclr::ceil_div(M * words, 256)), dim3(256),
                         0, s, C, M, N, ldc, relu_bits, words);
    }
    if (crow || cmax) {
      float* rows = crow;
      if (!rows) {  // cmax only
        MOLCLR_TRY_RC(molclr_absmax_f32(C, M, N, ldc, cmax, 1, stream));
        return MOLCLR_OK;
      }
      int64_t blocks = molclr::ceil_div(M, 32);
      blocks = blocks < 1 ? 1 : blocks > 2048 ? 2048 : blocks;
      hipLaunchKernelGGL(k_absmax_rows, dim3((unsigned)blocks), dim3(256), 0, s, C, M, N, ldc, rows,
                         cmax);
      for (int64_t p = 1; p < crow_parts(N); ++p)
        (void)molclr::copy_async(rows + p * M, rows, (size_t)M * sizeof(float), s);
    }
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  Args a{A, nullptr, C, M, N, K, lda, kp, ldc, bias, aux, ldaux, 0, accumulate, 9};
  a.Bp = planes;
  a.bps = npad * kp;
  a.cmax = cmax;
  a.crow = crow;
  a.amax_out = amax_out;
  a.bits_out = relu_bits;
  a.bits_ld = M;
  return run_q6(a, npad, epilogue, s, 0);
}

MOLCLR_API int64_t molclr_gemm_row_parts(int64_t N) { return crow_parts(N); }

MOLCLR_API int molclr_gemm_f32_bplanes(const float* A, const uint16_t* planes, float* C, int64_t M,
                                       int64_t N, int64_t K, int64_t lda, int64_t ldc,
                                       int a_kmajor, int epilogue_flags, const float* bias,
                                       const float* aux, int64_t ldaux, void* workspace,
                                       size_t workspace_bytes, molclr_stream_t stream) {
  return molclr_gemm_f32_bplanes_tile(A, planes, C, M, N, K, lda, ldc, a_kmajor, epilogue_flags,
                                      bias, aux, ldaux, workspace, workspace_bytes, stream, 0);
}

size_t molclr_colsum_ws(int64_t rows, int64_t cols);  // norm.hip

MOLCLR_API size_t molclr_linear_wgrad_workspace_bytes(int64_t rows, int64_t n_out, int64_t n_in) {
  const int64_t M = n_out, N = n_in, K = rows;
  size_t need = molclr_gemm_f32_workspace_bytes(M, N, K);
  const int sp = pick_splits(5, M, N, K, 1, 1);
  const size_t fused = sp > 1 ? (size_t)sp * (M * N + M) * sizeof(float) + 256 : 0;
  const size_t cs = molclr_colsum_ws(rows, n_out);
  need = fused > need ? fused : need;
  if (M % 4 == 0 && N % 4 == 0 && M * N < (1ll << 28)) {  // w6 (and its h3 form at any K)
    const size_t w6 = w6_ws_bytes(M, N, K, true);
    need = w6 > need ? w6 : need;
  }
  return cs > need ? cs : need;
}

MOLCLR_API int molclr_linear_wgrad_groups(const float* dy, const float* x, float* dW, float* db,
                                          int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy,
                                          int64_t ld_x, int accumulate, void* workspace,
                                          size_t workspace_bytes, molclr_stream_t stream,
                                          int groups) {
  MOLCLR_REQUIRE(groups == 1 || groups == 2, "linear_wgrad: groups must be 1 or 2");
  MOLCLR_REQUIRE(rows >= 0 && n_out > 0 && n_in > 0, "linear_wgrad: bad sizes");
  MOLCLR_REQUIRE(dy && x && dW, "linear_wgrad: null pointer");
  MOLCLR_REQUIRE(ld_dy >= n_out && ld_x >= n_in, "linear_wgrad: leading dimension too small");
  MOLCLR_REQUIRE(!db || (n_out % 4 == 0 && ld_dy % 4 == 0),
                 "linear_wgrad: db needs n_out and ld_dy multiples of 4");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_linear_wgrad_workspace_bytes(rows, n_out, n_in));
  const int flags = accumulate ? MOLCLR_EPI_ACCUMULATE : 0;
  if (rows == 0) {  // an empty batch contributes nothing: dW = 0 (or unchanged)
    if (!accumulate) {
      (void)molclr::zero_async(dW, (size_t)n_out * n_in * sizeof(float), molclr::as_stream(stream));
      if (db) (void)molclr::zero_async(db, (size_t)n_out * sizeof(float), molclr::as_stream(stream));
    }
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  // dW = dy^T x: A = dy (K-major, lda = ld_dy), B = x (K-major, ldb = ld_x)
  if (w6_shape_ok(n_out, n_in, rows) && ld_dy % 4 == 0 && ld_x % 4 == 0)
    return run_w6(dy, x, dW, db, n_out, n_in, rows, ld_dy, ld_x, n_in, accumulate, workspace,
                  workspace_bytes, molclr::as_stream(stream), groups);
  if (!db || impl_for(n_out, n_in, ld_dy, ld_x, 1, 1, -1) != 5) {
    int rc = molclr_gemm_f32(dy, x, dW, n_out, n_in, rows, ld_dy, ld_x, n_in, 1, 1, flags,
                             nullptr, nullptr, 0, workspace, workspace_bytes, stream);
    if (rc || !db) return rc;
    return molclr_colsum_f32(dy, db, rows, n_out, ld_dy, accumulate, workspace, workspace_bytes,
                             stream);
  }
  Args a{dy, x, dW, n_out, n_in, rows, ld_dy, ld_x, n_in, nullptr, nullptr, 0, 0, accumulate, 5};
  a.colsum = db;
  return run_gemm(a, 5, false, 1, 1, MOLCLR_EPI_NONE, workspace, workspace_bytes,
                  molclr::as_stream(stream));
}

MOLCLR_API int molclr_linear_wgrad(const float* dy, const float* x, float* dW, float* db,
                                   int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy,
                                   int64_t ld_x, int accumulate, void* workspace,
                                   size_t workspace_bytes, molclr_stream_t stream) {
  return molclr_linear_wgrad_groups(dy, x, dW, db, rows, n_out, n_in, ld_dy, ld_x, accumulate,
                                    workspace, workspace_bytes, stream, 2);
}

// ---------------------------------------------------------------------------
// h3 entry points (mfma.h "h3": three fp16 MFMAs per product with per-tensor
// power-of-two scaling; see include/molclr.h)
// ---------------------------------------------------------------------------
MOLCLR_API int molclr_absmax_f32(const float* x, int64_t rows, int64_t cols, int64_t ld,
                                 float* slot, int accumulate, molclr_stream_t stream) {
  MOLCLR_REQUIRE(rows >= 0 && cols >= 0 && ld >= cols && slot, "absmax_f32: bad arguments");
  hipStream_t s = molclr::as_stream(stream);
  if (!accumulate) (void)molclr::zero_async(slot, kMaxSlotFloats * sizeof(float), s);
  if (rows > 0 && cols > 0) {
    MOLCLR_REQUIRE(x, "absmax_f32: null x");
    int64_t blocks = ld == cols ? molclr::ceil_div(rows * cols, 256 * 16) : rows;
    blocks = blocks < 1 ? 1 : blocks > 1024 ? 1024 : blocks;
    hipLaunchKernelGGL(k_absmax, dim3((unsigned)blocks), dim3(256), 0, s, x, rows, cols, ld, slot);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_absmax_rows_f32(const float* x, int64_t rows, int64_t cols, int64_t ld,
                                      float* rowmax, float* slot, int accumulate,
                                      molclr_stream_t stream) {
  MOLCLR_REQUIRE(rows >= 0 && cols >= 0 && ld >= cols && rowmax && slot,
                 "absmax_rows_f32: bad arguments");
  hipStream_t s = molclr::as_stream(stream);
  if (!accumulate) (void)molclr::zero_async(slot, kMaxSlotFloats * sizeof(float), s);
  if (rows > 0) {
    MOLCLR_REQUIRE(x || cols == 0, "absmax_rows_f32: null x");
    int64_t blocks = molclr::ceil_div(rows, 4 * 8);
    blocks = blocks < 1 ? 1 : blocks > 2048 ? 2048 : blocks;
    hipLaunchKernelGGL(k_absmax_rows, dim3((unsigned)blocks), dim3(256), 0, s, x, rows, cols, ld,
                       rowmax, slot);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API size_t molclr_hplanes_bytes(int64_t N, int64_t K) {
  return (size_t)2 * planes_npad(N) * planes_kp(K) * sizeof(uint16_t) + kMaxSlotFloats * sizeof(float);
}

MOLCLR_API int molclr_hplanes_make_batch(int count, const float* const* B, const int64_t* N,
                                         const int64_t* K, const int64_t* ldb,
                                         const int* b_kmajor, uint16_t* const* planes,
                                         molclr_stream_t stream) {
  MOLCLR_REQUIRE(count >= 0 && (count == 0 || (B && N && K && ldb && b_kmajor && planes)),
                 "hplanes_make_batch: null arrays");
  for (int base = 0; base < count; base += kPlanesBatch) {
    PlanesJobs jobs{};
    const int n = count - base < kPlanesBatch ? count - base : kPlanesBatch;
    int64_t most = 0;
    for (int i = 0; i < n; ++i) {
      const int q = base + i;
      MOLCLR_REQUIRE(N[q] > 0 && K[q] > 0 && B[q] && planes[q],
                     "hplanes_make_batch: job %d empty or null", q);
      MOLCLR_REQUIRE(b_kmajor[q] ? ldb[q] >= N[q] : ldb[q] >= K[q],
                     "hplanes_make_batch: job %d leading dimension too small", q);
      jobs.j[i] = PlanesJob{B[q], planes[q], N[q], K[q], ldb[q], planes_npad(N[q]), planes_kp(K[q]),
                            b_kmajor[q]};
      const int64_t e = planes_tiled_blocks(jobs.j[i]);
      most = e > most ? e : most;
    }
    hipStream_t s = molclr::as_stream(stream);
    // the max pass once per matrix: both orientations of one weight (the
    // forward's and the data gradient's image) read the same values, so the
    // second takes the first's max (its slot written by the same block)
    PlanesJobs mj{};
    int nm = 0;
    for (int i = 0; i < n; ++i) {
      const PlanesJob& a = jobs.j[i];
      const int64_t ra = a.kmajor ? a.K : a.N, ca = a.kmajor ? a.N : a.K;
      int twin = -1;
      for (int q = 0; q < nm && twin < 0; ++q) {
        const PlanesJob& b = mj.j[q];
        const int64_t rb = b.kmajor ? b.K : b.N, cb = b.kmajor ? b.N : b.K;
        if (b.B == a.B && b.ldb == a.ldb && rb == ra && cb == ca && b.slot2 == nullptr) twin = q;
      }
      if (twin >= 0)
        mj.j[twin].slot2 = reinterpret_cast<float*>(a.planes + 2 * a.npad * a.kp);
      else
        mj.j[nm++] = a;
    }
    hipLaunchKernelGGL(k_hplanes_max_batch, dim3(kHMaxParts, (unsigned)nm), dim3(1024), 0, s, mj);
    hipLaunchKernelGGL(k_planes_make_tiled<true>, dim3((unsigned)most, (unsigned)n), dim3(256), 0, s,
                       jobs);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

namespace molclr {
int hplanes_make_and_max(const float* B, int64_t N, int64_t K, uint16_t* planes, const float* x,
                         int64_t x_rows, int64_t x_cols, float* x_slot, hipStream_t s) {
  MOLCLR_REQUIRE(N > 0 && K > 0 && B && planes && x && x_slot && x_rows > 0 && x_cols > 0,
                 "hplanes_make_and_max: empty or null operand");
  PlanesJobs jobs{};
  jobs.j[0] = PlanesJob{B, planes, N, K, K, planes_npad(N), planes_kp(K), 0};
  // job 1: x's max only -- no image (npad = kp = 0 puts its slot at x_slot)
  jobs.j[1] = PlanesJob{x, reinterpret_cast<uint16_t*>(x_slot), x_rows, x_cols, x_cols, 0, 0, 0};
  hipLaunchKernelGGL(k_hplanes_max_batch, dim3(kHMaxParts, 2), dim3(1024), 0, s, jobs);
  hipLaunchKernelGGL(k_planes_make_tiled<true>, dim3((unsigned)planes_tiled_blocks(jobs.j[0]), 1),
                     dim3(256), 0, s, jobs);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
}  // namespace molclr

MOLCLR_API int molclr_gemm_f32_h3_bits(const float* A, const float* amax, int a_row_parts,
                                       const uint16_t* hplanes, float* C, int64_t M, int64_t N,
                                       int64_t K, int64_t lda, int64_t ldc, int epilogue_flags,
                                       const float* bias, const float* aux, int64_t ldaux,
                                       const uint32_t* mask_bits, float* cmax, float* crow,
                                       float* amax_out, uint32_t* relu_bits,
                                       molclr_stream_t stream) {
  const int accumulate = (epilogue_flags & MOLCLR_EPI_ACCUMULATE) ? 1 : 0;
  const int epilogue = epilogue_flags & ~MOLCLR_EPI_ACCUMULATE;
  MOLCLR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_f32_h3: negative size");
  MOLCLR_REQUIRE(epilogue >= MOLCLR_EPI_NONE && epilogue <= MOLCLR_EPI_RELU_MASK,
                 "gemm_f32_h3: bad epilogue %d", epilogue);
  MOLCLR_REQUIRE((epilogue != MOLCLR_EPI_BIAS && epilogue != MOLCLR_EPI_BIAS_RELU) || bias,
                 "gemm_f32_h3: bias epilogue needs bias");
  MOLCLR_REQUIRE(epilogue != MOLCLR_EPI_RELU_MASK || aux || mask_bits,
                 "gemm_f32_h3: relu-mask epilogue needs aux or mask bits");
  MOLCLR_REQUIRE(K % 4 == 0 && lda % 4 == 0 && lda >= K && ldc >= N,
                 "gemm_f32_h3: K and lda multiples of 4, lda >= K, ldc >= N");
  MOLCLR_REQUIRE(K <= kQ6MaxK, "gemm_f32_h3: K %lld > %lld", (long long)K, (long long)kQ6MaxK);
  if (M == 0 || N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(K > 0 && A && amax && hplanes && C, "gemm_f32_h3: null operand or K == 0");
  const int64_t npad = planes_npad(N), kp = planes_kp(K);
  MOLCLR_REQUIRE(2 * npad * kp < (1ll << 31) && q6_blocks(M, N) < (1ll << 31),
                 "gemm_f32_h3: too large");
  Args a{A, nullptr, C, M, N, K, lda, kp, ldc, bias, aux, ldaux, 0, accumulate, 9};
  a.Bp = hplanes;
  a.bps = npad * kp;
  a.amax = amax;
  a.bmax = reinterpret_cast<const float*>(hplanes + 2 * npad * kp);
  a.cmax = cmax;
  a.crow = crow;
  a.amax_out = amax_out;
  MOLCLR_REQUIRE(a_row_parts >= 0 || (-a_row_parts == K / 4 && K / 4 >= 64 && lda == K),
                 "gemm_f32_h3: per-wave row maxima (a_row_parts %d) need a dense A of K / 4 "
                 "= %d >= 64 float4s per row", a_row_parts, (int)(K / 4));
  a.arow_parts = a_row_parts;
  a.bits_in = epilogue == MOLCLR_EPI_RELU_MASK ? mask_bits : nullptr;
  a.bits_out = epilogue == MOLCLR_EPI_BIAS_RELU ? relu_bits : nullptr;
  a.bits_ld = M;
  return run_q6(a, npad, epilogue, molclr::as_stream(stream), a_row_parts != 0 ? 2 : 1);
}

MOLCLR_API int molclr_gemm_f32_h3(const float* A, const float* amax, int a_row_parts,
                                  const uint16_t* hplanes, float* C, int64_t M, int64_t N,
                                  int64_t K, int64_t lda, int64_t ldc, int epilogue_flags,
                                  const float* bias, const float* aux, int64_t ldaux,
                                  const uint32_t* mask_bits, float* cmax, float* crow,
                                  float* amax_out, molclr_stream_t stream) {
  return molclr_gemm_f32_h3_bits(A, amax, a_row_parts, hplanes, C, M, N, K, lda, ldc,
                                 epilogue_flags, bias, aux, ldaux, mask_bits, cmax, crow, amax_out,
                                 nullptr, stream);
}

MOLCLR_API int molclr_gemm_f32_h3_impl(const float* A, const float* amax, int a_row_parts,
                                       const uint16_t* hplanes, float* C, int64_t M, int64_t N,
                                       int64_t K, int64_t lda, int64_t ldc, int epilogue_flags,
                                       const float* bias, const float* aux, int64_t ldaux,
                                       const uint32_t* mask_bits, float* cmax, float* crow,
                                       float* amax_out, uint32_t* relu_bits,
                                       molclr_stream_t stream, int impl) {
  MOLCLR_REQUIRE(impl >= 0 && impl <= 3,
                 "gemm_f32_h3_impl: impl %d (0 auto, 1 pp / q6, 2 bs, 3 bs16)", impl);
  g_bs_force = impl;
  const int rc = molclr_gemm_f32_h3_bits(A, amax, a_row_parts, hplanes, C, M, N, K, lda, ldc,
                                         epilogue_flags, bias, aux, ldaux, mask_bits, cmax, crow,
                                         amax_out, relu_bits, stream);
  g_bs_force = 0;
  return rc;
}

namespace {
// the w6 launch of run_w6 without its reduction: partials (and the bias
// partials) into `part`; returns the plan
// cs_b: the column sums are B's (a transposed launch, B = dY)
W6Plan launch_w6_h3(const float* A, const float* B, float* part, bool colsum, int64_t M, int64_t N,
                    int64_t K, int64_t lda, int64_t ldb, hipStream_t s, const float* amax,
                    const float* bmax, bool cs_b = false) {
  const W6Plan p = w6_plan(M, N, K, 2);
  float* cs_part = colsum ? part + (size_t)p.splits * M * N : nullptr;
  if (p.tn == 5) launch_w6<5, true>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax, cs_b);
  else if (p.tn == 4)
    launch_w6<4, true>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax, cs_b);
  else launch_w6<2, true>(p, s, A, B, part, M, N, K, lda, ldb, cs_part, amax, bmax, cs_b);
  return p;
}
// dW = dY^T X as (X^T dY)^T when that pads less: w6 tiles are 128 along M and
// 32 TN along N, so dW2 of the c2 layer (300 x 600) covers 384 x 640 and its
// transpose 640 x 320 (0.73 -> 0.88 of the MFMA work useful; measured in
// the c2 step 59.9 us against dW1's 52.3 us at the same FLOPs).
// MOLCLR_W6_TRANSPOSE=0 keeps every product in its own orientation.
int64_t w6_area(int64_t M, int64_t N) {
  const int64_t bn = 32 * wide_tn(N);
  return ((M + kW6BM - 1) / kW6BM * kW6BM) * ((N + bn - 1) / bn * bn);
}
bool w6_transposed(int64_t n_out, int64_t n_in) {
  static const bool off = [] {
    const char* e = getenv("MOLCLR_W6_TRANSPOSE");
    return e != nullptr && e[0] == '0';
  }();
  return !off && w6_area(n_in, n_out) < w6_area(n_out, n_in);
}
// the w6 partial bytes of dW [n_out][n_in] (its chosen orientation)
size_t w6_part_bytes(int64_t n_out, int64_t n_in, int64_t K, bool colsum) {
  // either orientation (launch_wgrad_job keeps dW's own for an unaligned dW)
  const W6Plan p = w6_plan(n_out, n_in, K, 2), q = w6_plan(n_in, n_out, K, 2);
  const int splits = p.splits > q.splits ? p.splits : q.splits;
  return molclr::align_up((size_t)splits * (n_out * n_in + (colsum ? n_out : 0)) * sizeof(float),
                          256);
}
// one job of the pair: dW = dY^T X (+ db = Σ dY) as partials, in the
// orientation w6_transposed picks; returns its reduce job
ReduceJob launch_wgrad_job(const float* dy, const float* dymax, const float* x, const float* xmax,
                           float* dW, float* db, int64_t n_out, int64_t n_in, int64_t rows,
                           int64_t ld_dy, int64_t ld_x, float* part, hipStream_t s) {
  // the transposed reduction stores float4 rows of dW
  const bool tr = w6_transposed(n_out, n_in) && (reinterpret_cast<uintptr_t>(dW) & 15) == 0;
  const W6Plan q = tr ? launch_w6_h3(x, dy, part, db != nullptr, n_in, n_out, rows, ld_x, ld_dy, s,
                                     xmax, dymax, true)
                      : launch_w6_h3(dy, x, part, db != nullptr, n_out, n_in, rows, ld_dy, ld_x, s,
                                     dymax, xmax);
  ReduceJob j{part, q.splits, n_out, n_in, dW, n_in,
              db ? part + (size_t)q.splits * n_out * n_in : nullptr, db};
  j.trans = tr ? 1 : 0;
  return j;
}
}  // namespace

MOLCLR_API int molclr_linear_wgrad_h3_groups(const float* dy, const float* dymax, const float* x,
                                             const float* xmax, float* dW, float* db, int64_t rows,
                                             int64_t n_out, int64_t n_in, int64_t ld_dy,
                                             int64_t ld_x, int accumulate, void* workspace,
                                             size_t workspace_bytes, molclr_stream_t stream,
                                             int groups) {
  MOLCLR_REQUIRE(groups == 1 || groups == 2, "linear_wgrad_h3: groups must be 1 or 2");
  MOLCLR_REQUIRE(rows >= 0 && n_out > 0 && n_in > 0, "linear_wgrad_h3: bad sizes");
  MOLCLR_REQUIRE(dy && dymax && x && xmax && dW, "linear_wgrad_h3: null pointer");
  MOLCLR_REQUIRE(ld_dy >= n_out && ld_x >= n_in, "linear_wgrad_h3: leading dimension too small");
  MOLCLR_REQUIRE(n_out % 4 == 0 && n_in % 4 == 0 && ld_dy % 4 == 0 && ld_x % 4 == 0 &&
                     n_out * n_in < (1ll << 28),
                 "linear_wgrad_h3: sizes and leading dimensions must be multiples of 4");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_linear_wgrad_workspace_bytes(rows, n_out, n_in));
  hipStream_t s = molclr::as_stream(stream);
  if (rows == 0) {
    if (!accumulate) {
      (void)molclr::zero_async(dW, (size_t)n_out * n_in * sizeof(float), s);
      if (db) (void)molclr::zero_async(db, (size_t)n_out * sizeof(float), s);
    }
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  MOLCLR_REQUIRE_WS(workspace_bytes, w6_ws_bytes(n_out, n_in, rows, db != nullptr));
  if (groups == 2 && w6_transposed(n_out, n_in)) {
    // the orientation the pair takes (bit-identical to it)
    const ReduceJob j = launch_wgrad_job(dy, dymax, x, xmax, dW, db, n_out, n_in, rows, ld_dy, ld_x,
                                         static_cast<float*>(workspace), s);
    ReduceJob none{nullptr, 0, 0, 0, nullptr, 0, nullptr, nullptr};
    molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce_pair,
                         dim3((unsigned)molclr::ceil_div(j.threads(), 256)), dim3(256), 0, s, j,
                         none, accumulate);
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  return run_w6(dy, x, dW, db, n_out, n_in, rows, ld_dy, ld_x, n_in, accumulate, workspace,
                workspace_bytes, s, groups, dymax, xmax);
}


MOLCLR_API size_t molclr_linear_wgrad_h3_pair_workspace_bytes(int64_t rows, int64_t n_out_a,
                                                              int64_t n_in_a, int64_t n_out_b,
                                                              int64_t n_in_b) {
  return w6_part_bytes(n_out_a, n_in_a, rows, true) + w6_part_bytes(n_out_b, n_in_b, rows, true) +
         256;
}

MOLCLR_API int molclr_linear_wgrad_h3_pair(
    const float* dy_a, const float* dymax_a, const float* x_a, const float* xmax_a, float* dW_a,
    float* db_a, int64_t n_out_a, int64_t n_in_a, int64_t ld_dy_a, int64_t ld_x_a,
    const float* dy_b, const float* dymax_b, const float* x_b, const float* xmax_b, float* dW_b,
    float* db_b, int64_t n_out_b, int64_t n_in_b, int64_t ld_dy_b, int64_t ld_x_b, int64_t rows,
    int accumulate, void* workspace, size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_REQUIRE(rows >= 1024, "linear_wgrad_h3_pair: rows %lld < 1024 (use linear_wgrad_h3)",
                 (long long)rows);
  MOLCLR_REQUIRE(dy_a && dymax_a && x_a && xmax_a && dW_a && dy_b && dymax_b && x_b && xmax_b &&
                     dW_b,
                 "linear_wgrad_h3_pair: null pointer");
  for (int q = 0; q < 2; ++q) {
    const int64_t no = q ? n_out_b : n_out_a, ni = q ? n_in_b : n_in_a;
    const int64_t ld1 = q ? ld_dy_b : ld_dy_a, ld2 = q ? ld_x_b : ld_x_a;
    MOLCLR_REQUIRE(no > 0 && ni > 0 && no % 4 == 0 && ni % 4 == 0 && ld1 % 4 == 0 &&
                       ld2 % 4 == 0 && ld1 >= no && ld2 >= ni && no * ni < (1ll << 28),
                   "linear_wgrad_h3_pair: job %d sizes must be multiples of 4", q);
  }
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_linear_wgrad_h3_pair_workspace_bytes(
                                         rows, n_out_a, n_in_a, n_out_b, n_in_b));
  hipStream_t s = molclr::as_stream(stream);
  float* pa = static_cast<float*>(workspace);
  float* pb = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                       w6_part_bytes(n_out_a, n_in_a, rows, true));
  const ReduceJob ja = launch_wgrad_job(dy_a, dymax_a, x_a, xmax_a, dW_a, db_a, n_out_a, n_in_a,
                                        rows, ld_dy_a, ld_x_a, pa, s);
  const ReduceJob jb = launch_wgrad_job(dy_b, dymax_b, x_b, xmax_b, dW_b, db_b, n_out_b, n_in_b,
                                        rows, ld_dy_b, ld_x_b, pb, s);
  const int64_t total = ja.threads() + jb.threads();
  molclr::launch_timed(molclr::kTimeGemm, k_splitk_reduce_pair,
                       dim3((unsigned)molclr::ceil_div(total, 256)), dim3(256), 0, s, ja, jb,
                       accumulate);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_linear_wgrad_h3(const float* dy, const float* dymax, const float* x,
                                      const float* xmax, float* dW, float* db, int64_t rows,
                                      int64_t n_out, int64_t n_in, int64_t ld_dy, int64_t ld_x,
                                      int accumulate, void* workspace, size_t workspace_bytes,
                                      molclr_stream_t stream) {
  return molclr_linear_wgrad_h3_groups(dy, dymax, x, xmax, dW, db, rows, n_out, n_in, ld_dy, ld_x,
                                       accumulate, workspace, workspace_bytes, stream, 2);
}
