// Fused NT-Xent (utils/nt_xent.py:47-65) on the f32 MFMA.
//
// The reference materialises the cosine broadcast (2B,2B,C), the mask gather
// and the cross entropy.  Here, with R = [zj; zi] (nt_xent.py:48) scaled to
// unit rows (CosineSimilarity, eps 1e-8; nt_xent.py:40-45):
//   S      = R R^T, logits S/T
//   lse_r  = log Σ_{c≠r} exp(S_rc/T)           (positive + masked negatives)
//   loss   = (1/2B) Σ_r (lse_r − S_{r,p(r)}/T),  p(r) = (r + B) mod 2B
// and the gradient is dR = W R with the SYMMETRIC
//   W_rc = g/(2B·T) · (P_rc + P_cr − 2·[c = p(r)]),  c ≠ r,  P_rc = exp(S_rc/T − lse_r)
// (S_rc enters loss rows r and c).  A rank that owns a subset of the rows only
// needs the gathered R and the gathered lse to produce the exact gradient of
// its rows: no reduce-scatter of column gradients is required.
//
// Tiles are computed transposed, S'[c][r] (rows c in registers, r on the lane):
// the per-row online logsumexp is then a register loop plus one lane-half
// shuffle, and in the backward the W' accumulator is directly the A operand
// of the second MFMA (dR[r][k] = Σ_c W'[c][r] R[c][k]) — no LDS round trip.
// One wave per (32-row block, column split[, k group]); partials are merged
// in a fixed order.
#include "common.h"

#include <math.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int crow(int reg, int lh) { return (reg & 3) + 8 * (reg >> 2) + 4 * lh; }

// S'[c][r] for c in [c0, c0+32), r in [r0, r0+32)
__device__ __forceinline__ f32x16 sim_tile(const float* __restrict__ rows, int64_t nrows, int64_t r0,
                                           const float* __restrict__ cols, int64_t ncols, int64_t c0,
                                           int64_t C, int li, int lh) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int64_t half = C / 2;
  const bool cv = c0 + li < ncols, rv = r0 + li < nrows;
  // out-of-range rows / columns read row 0 and are zeroed: loads stay unconditional
  const float4* ap = reinterpret_cast<const float4*>(cols + (cv ? (c0 + li) : 0) * C + lh * half);
  const float4* bp = reinterpret_cast<const float4*>(rows + (rv ? (r0 + li) : 0) * C + lh * half);
  const float am = cv ? 1.f : 0.f, bm = rv ? 1.f : 0.f;
  const int64_t n4 = half / 4;
  int64_t g = 0;
  // four float4 pairs in flight per step (C % 32 == 0 in practice; tail below)
  for (; g + 4 <= n4; g += 4) {
    float4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = ap[g + u];
      b[u] = bp[g + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].x * am, b[u].x * bm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].y * am, b[u].y * bm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].z * am, b[u].z * bm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].w * am, b[u].w * bm, acc, 0, 0, 0);
    }
  }
  for (; g < n4; ++g) {
    const float4 a = ap[g], b = bp[g];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x * am, b.x * bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y * am, b.y * bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z * am, b.z * bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w * am, b.w * bm, acc, 0, 0, 0);
  }
  return acc;
}

// The wave's 32 rows stay in registers for all its column chunks (NQ float4
// per lane: C = 8 NQ): only the column operand is re-read per chunk.
template <int NQ>
struct RowRegs {
  float4 v[NQ];
  __device__ __forceinline__ void load(const float* __restrict__ rows, int64_t nrows, int64_t r0,
                                       int li, int lh) {
    const bool rv = r0 + li < nrows;
    const float4* bp =
        reinterpret_cast<const float4*>(rows + (rv ? (r0 + li) : 0) * (8 * NQ) + lh * 4 * NQ);
    const float bm = rv ? 1.f : 0.f;
#pragma unroll
    for (int g = 0; g < NQ; ++g) {
      const float4 b = bp[g];
      v[g] = make_float4(b.x * bm, b.y * bm, b.z * bm, b.w * bm);
    }
  }
};

template <int NQ>
__device__ __forceinline__ f32x16 sim_tile_r(const RowRegs<NQ>& rr, const float* __restrict__ cols,
                                             int64_t ncols, int64_t c0, int li, int lh) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const bool cv = c0 + li < ncols;
  const float4* ap =
      reinterpret_cast<const float4*>(cols + (cv ? (c0 + li) : 0) * (8 * NQ) + lh * 4 * NQ);
  const float am = cv ? 1.f : 0.f;
#pragma unroll
  for (int g = 0; g < NQ; g += 4) {
    float4 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = ap[g + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 b = rr.v[g + u];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].x * am, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].y * am, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].z * am, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].w * am, b.w, acc, 0, 0, 0);
    }
  }
  return acc;
}

// partial layout: pm [splits][nrows], ps [splits][nrows]; pos [nrows]
template <int NQ>  // NQ > 0: rows in registers (C == 8 NQ); 0: any C
__global__ __launch_bounds__(64) void k_ntxent_fwd_partial(
    const float* __restrict__ rows, const int32_t* __restrict__ gidx, const float* __restrict__ cols,
    int64_t nrows, int64_t ncols, int64_t C, int64_t B, float inv_t, int64_t chunks_per_split,
    float* __restrict__ pm, float* __restrict__ ps, float* __restrict__ pos) {
  const int lane = threadIdx.x, li = lane & 31, lh = lane >> 5;
  const int64_t r0 = (int64_t)blockIdx.x * 32;
  const int64_t rl = r0 + li;
  const int64_t rg = rl < nrows ? gidx[rl] : -1;
  const int64_t pg = rg >= 0 ? (rg + B) % (2 * B) : -1;
  float m = -INFINITY, s = 0.f;
  const int64_t nchunks = (ncols + 31) / 32;
  int64_t ch = (int64_t)blockIdx.y * chunks_per_split;
  int64_t ch_end = ch + chunks_per_split < nchunks ? ch + chunks_per_split : nchunks;
  RowRegs<(NQ > 0 ? NQ : 4)> rr;
  if constexpr (NQ > 0) rr.load(rows, nrows, r0, li, lh);
  for (; ch < ch_end; ++ch) {
    const int64_t c0 = ch * 32;
    f32x16 st;
    if constexpr (NQ > 0) st = sim_tile_r<NQ>(rr, cols, ncols, c0, li, lh);
    else st = sim_tile(rows, nrows, r0, cols, ncols, c0, C, li, lh);
    float tmax = -INFINITY;
    float lg[16];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      int64_t cg = c0 + crow(reg, lh);
      bool ok = rg >= 0 && cg < ncols && cg != rg;
      lg[reg] = ok ? st[reg] * inv_t : -INFINITY;
      if (ok && cg == pg) pos[rl] = lg[reg];
      tmax = fmaxf(tmax, lg[reg]);
    }
    if (tmax > -INFINITY) {
      float nm = fmaxf(m, tmax);
      float acc = s * expf(m - nm);
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) acc += expf(lg[reg] - nm);
      m = nm;
      s = acc;
    }
  }
  // merge the two lane halves (same row r, different columns)
  float mo = __shfl_xor(m, 32, 64), so = __shfl_xor(s, 32, 64);
  float nm = fmaxf(m, mo);
  float tot = (nm == -INFINITY) ? 0.f : s * expf(m - nm) + so * expf(mo - nm);
  if (lh == 0 && rl < nrows) {
    pm[(int64_t)blockIdx.y * nrows + rl] = nm;
    ps[(int64_t)blockIdx.y * nrows + rl] = tot;
  }
}

__global__ void k_ntxent_fwd_final(const float* __restrict__ pm, const float* __restrict__ ps,
                                   const float* __restrict__ pos, int64_t splits, int64_t nrows,
                                   float inv_2b, float* __restrict__ lse, float* __restrict__ loss) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  float m = -INFINITY;
  for (int64_t z = 0; z < splits; ++z) m = fmaxf(m, pm[z * nrows + r]);
  float s = 0.f;
  for (int64_t z = 0; z < splits; ++z) {
    float mz = pm[z * nrows + r];
    if (mz > -INFINITY) s += ps[z * nrows + r] * expf(mz - m);
  }
  float l = m + logf(s);
  lse[r] = l;
  loss[r] = (l - pos[r]) * inv_2b;
}

// partial [splits][nrows][C]; grid (row blocks, splits, k groups of KT tiles)
template <int KT, int NQ>
__global__ __launch_bounds__(64) void k_ntxent_bwd_partial(
    const float* __restrict__ rows, const int32_t* __restrict__ gidx, const float* __restrict__ cols,
    const float* __restrict__ lse_cols, const float* __restrict__ grad_loss, int64_t nrows,
    int64_t ncols, int64_t C, int64_t B, float inv_t, int64_t chunks_per_split,
    float* __restrict__ partial) {
  const int lane = threadIdx.x, li = lane & 31, lh = lane >> 5;
  const int64_t r0 = (int64_t)blockIdx.x * 32;
  const int64_t rl = r0 + li;
  const int64_t rg = rl < nrows ? gidx[rl] : -1;
  const int64_t pg = rg >= 0 ? (rg + B) % (2 * B) : -1;
  const float lse_r = rg >= 0 ? lse_cols[rg] : 0.f;
  const float coef = (*grad_loss) * inv_t / (float)(2 * B);
  const int64_t kbase = (int64_t)blockIdx.z * KT * 32;
  const int nkt = (int)((C - kbase) / 32 < KT ? (C - kbase) / 32 : KT);

  f32x16 out[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) out[t][r] = 0.f;

  const int64_t nchunks = (ncols + 31) / 32;
  int64_t ch = (int64_t)blockIdx.y * chunks_per_split;
  int64_t ch_end = ch + chunks_per_split < nchunks ? ch + chunks_per_split : nchunks;
  RowRegs<(NQ > 0 ? NQ : 4)> rr;
  if constexpr (NQ > 0) rr.load(rows, nrows, r0, li, lh);
  for (; ch < ch_end; ++ch) {
    const int64_t c0 = ch * 32;
    f32x16 st;
    if constexpr (NQ > 0) st = sim_tile_r<NQ>(rr, cols, ncols, c0, li, lh);
    else st = sim_tile(rows, nrows, r0, cols, ncols, c0, C, li, lh);
    // W'[c][r] in place
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      int64_t cg = c0 + crow(reg, lh);
      float w = 0.f;
      if (rg >= 0 && cg < ncols && cg != rg) {
        float lg = st[reg] * inv_t;
        w = expf(lg - lse_r) + expf(lg - lse_cols[cg]);
        if (cg == pg) w -= 2.f;
        w *= coef;
      }
      st[reg] = w;
    }
    // out[r][k] += Σ_c W'[c][r] R[c][k]: A operand = W' register s (k-index c = crow(s, lh))
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      int64_t cg = c0 + crow(reg, lh);
      const float* crow_ptr = cols + (cg < ncols ? cg : 0) * C + kbase + li;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        if (t < nkt) {
          float b = cg < ncols ? crow_ptr[t * 32] : 0.f;
          out[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(st[reg], b, out[t], 0, 0, 0);
        }
      }
    }
  }
  // out[t] register reg of lane (li, lh): row r = crow(reg, lh), col k = kbase + 32 t + li
  float* base = partial + (int64_t)blockIdx.y * nrows * C;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    if (t >= nkt) continue;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      int64_t r = r0 + crow(reg, lh);
      if (r < nrows) base[r * C + kbase + t * 32 + li] = out[t][reg];
    }
  }
}

__global__ void k_reduce_splits(const float* __restrict__ partial, int64_t splits, int64_t n,
                                float* __restrict__ out) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  float acc = 0.f;
#pragma unroll 4
  for (int64_t z = 0; z < splits; ++z) acc += partial[z * n + t];
  out[t] = acc;
}

// ---- GEMM formulation (impl 1) ------------------------------------------------
// S = R_rows R_cols^T is one split-bf16 GEMM (molclr_gemm_f32_bplanes: six
// bf16 MFMA products per element pair, fp32 accuracy, at the bf16 MFMA rate)
// into an [nrows][ncols] fp32 buffer; the masked row logsumexp, and in the
// backward the symmetric weight W, are then elementwise passes over it, and
// dR = W R_cols a second GEMM.  At the c4 row shard (1024 x 8192 x 256) the
// buffer is 32 MB.

// four waves per row: lse_r = log Σ_{c != r} exp(S_rc / T), loss_r =
// (lse_r - S_{r,p(r)} / T) / 2B.  Wave w takes the float4 columns
// 4 lane + 256 w + 1024 j; each lane folds eight float4 loads (issued together)
// at a time into its running (max, sum) with one rescale per batch; the lanes
// and then the four waves merge in a fixed order.  (One wave per row with a
// rescale per float4 left one wave per SIMD in a serial exp chain: 12.1 us on
// c4's 1024 x 8192.)
constexpr int kLseWaves = 4;
__global__ __launch_bounds__(64 * kLseWaves) void k_ntxent_row_lse(
    const float* __restrict__ S, int64_t nrows, int64_t ncols, const int32_t* __restrict__ gidx,
    int64_t B, float inv_t, float inv_2b, float* __restrict__ lse, float* __restrict__ loss) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r = blockIdx.x;  // block-uniform: no early exit inside the block
  const int64_t rg = gidx[r];
  const float* row = S + r * ncols;
  float m = -INFINITY, s = 0.f;
  // n float4 of logits (columns c[u] .. c[u] + 3) into the running (max, sum)
  auto fold = [&](const float4* v, const int64_t* c, int n) {
    float x[32], bm = -INFINITY;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[4 * u + j] = (u < n && c[u] + j != rg) ? e[j] * inv_t : -INFINITY;
        bm = fmaxf(bm, x[4 * u + j]);
      }
    }
    if (bm > -INFINITY) {
      const float nm = fmaxf(m, bm);
      float acc = s * expf(m - nm);
#pragma unroll
      for (int i = 0; i < 32; ++i) acc += expf(x[i] - nm);
      m = nm;
      s = acc;
    }
  };
  constexpr int64_t kStep = 256 * kLseWaves;  // columns per float4 round of the block
  int64_t c0 = 4 * lane + 256 * wave;         // ncols % 4 == 0 (host)
  while (c0 < ncols) {
    float4 v[8];
    int64_t c[8];
    int n = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      c[u] = c0 + kStep * u;
      if (c[u] < ncols) {
        v[u] = *reinterpret_cast<const float4*>(row + c[u]);
        n = u + 1;
      } else {
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    fold(v, c, n);
    c0 += 8 * kStep;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, mo);
    s = nm == -INFINITY ? 0.f : s * expf(m - nm) + so * expf(mo - nm);
    m = nm;
  }
  __shared__ float wm[kLseWaves], ws[kLseWaves];
  if (lane == 0) {
    wm[wave] = m;
    ws[wave] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    m = wm[0];
    s = ws[0];
    for (int w = 1; w < kLseWaves; ++w) {
      const float nm = fmaxf(m, wm[w]);
      s = nm == -INFINITY ? 0.f : s * expf(m - nm) + ws[w] * expf(wm[w] - nm);
      m = nm;
    }
    const float l = m + logf(s);
    const int64_t pg = (rg + B) % (2 * B);
    lse[r] = l;
    loss[r] = (l - row[pg] * inv_t) * inv_2b;
  }
}

// W_rc = g/(2B T) (exp(S_rc/T - lse_r) + exp(S_rc/T - lse_c) - 2 [c = p(r)]), 0 on the
// diagonal c = r (W may be S itself)
__global__ __launch_bounds__(256) void k_ntxent_weights(const float* S, float* W, int64_t nrows,
                                                        int64_t ncols, const int32_t* __restrict__ gidx,
                                                        const float* __restrict__ lse_cols,
                                                        const float* __restrict__ grad_loss, int64_t B,
                                                        float inv_t) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // float4 index
  const int64_t per_row = ncols / 4;
  if (q >= nrows * per_row) return;
  const int64_t r = q / per_row, c0 = 4 * (q - r * per_row);
  const int64_t rg = gidx[r];
  const int64_t pg = (rg + B) % (2 * B);
  const float lse_r = lse_cols[rg];
  const float coef = (*grad_loss) * inv_t / (float)(2 * B);
  float4 v = *reinterpret_cast<const float4*>(S + r * ncols + c0);
  const float4 lc = *reinterpret_cast<const float4*>(lse_cols + c0);
  float e[4] = {v.x, v.y, v.z, v.w};
  const float l[4] = {lc.x, lc.y, lc.z, lc.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t c = c0 + j;
    float w = 0.f;
    if (c != rg) {
      const float lg = e[j] * inv_t;
      w = expf(lg - lse_r) + expf(lg - l[j]);
      if (c == pg) w -= 2.f;
      w *= coef;
    }
    e[j] = w;
  }
  *reinterpret_cast<float4*>(W + r * ncols + c0) = make_float4(e[0], e[1], e[2], e[3]);
}

// ---- h3 formulation (impl 2) ----------------------------------------------------
// S = R_rows R_cols^T by the h3 GEMM (three fp16 MFMAs per product,
// per-tensor power-of-two scales; the rows are unit vectors after
// F.normalize / the cosine's own normalisation), the row logsumexp as in
// impl 1; in the backward W^T = f(S) through an LDS transpose, and
// dR = W R_cols as the h3 weight-gradient product (dR = (W^T)^T R_cols:
// K = ncols, a long K split into ordered partials).

// max |x| of a dense [rows][cols] matrix into a max slot with plain stores
// (block b writes entry b of kMaxSlotParts: no zeroing, no atomics); block 0
// also zeroes `zero_slot` (the atomic slot the next kernel folds into)
__global__ __launch_bounds__(1024) void k_ntxent_absmax_plain(const float* __restrict__ x,
                                                              int64_t n4, float* __restrict__ slot,
                                                              float* __restrict__ zero_slot) {
  float m = absmax4_range(reinterpret_cast<const float4*>(x),
                          (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n4,
                          (int64_t)gridDim.x * blockDim.x);
  m = block_max(m);
  if (threadIdx.x == 0) slot[blockIdx.x * kMaxSlotStride] = m;
  if (zero_slot != nullptr && blockIdx.x == 0)
    for (int i = threadIdx.x; i < kMaxSlotFloats; i += blockDim.x) zero_slot[i] = 0.f;
}

// W^T[c][r] = g/(2B T) (exp(S_rc/T - lse_r) + exp(S_rc/T - lse_c) - 2 [c = p(r)]),
// 0 at c = r, from the row-major S through an LDS transpose: a block of 256
// threads takes a 64 (r) x 64 (c) tile, reads S rows as float4 runs along c and
// writes W^T rows as float4 runs along r; max |W| into `wmax` (zeroed before)
constexpr int kWT = 64;
__global__ __launch_bounds__(256) void k_ntxent_weights_tt(
    const float* __restrict__ S, float* __restrict__ Wt, int64_t nrows, int64_t ncols,
    const int32_t* __restrict__ gidx, const float* __restrict__ lse_cols,
    const float* __restrict__ grad_loss, int64_t B, float inv_t, float* __restrict__ wmax) {
  __shared__ float tile[kWT][kWT + 1];  // [c][r]
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * kWT, c0 = (int64_t)blockIdx.x * kWT;
  const float coef = (*grad_loss) * inv_t / (float)(2 * B);
  float mx = 0.f;
  // read: 64 rows x 16 float4 = 1024 float4, 4 per thread (16 threads per
  // row; a thread's column run cc is the same for its four rows).  All loads
  // are issued before any use (clamped indices, masked after): the chain
  // gidx -> lse_cols[rg] and the four S loads overlap instead of serialising.
  const int cc = 4 * (tid & 15), rr0 = tid >> 4;
  const int64_t c = c0 + cc;
  const bool cv = c < ncols;  // ncols % 4 == 0 (host)
  const int64_t cl = cv ? c : 0;
  const float4 lc = *reinterpret_cast<const float4*>(lse_cols + cl);
  float4 v[4];
  int64_t rg[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t r = r0 + rr0 + 16 * q;
    const int64_t rl = r < nrows ? r : nrows - 1;
    v[q] = *reinterpret_cast<const float4*>(S + rl * ncols + cl);
    rg[q] = gidx[rl];
  }
  float lr[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) lr[q] = lse_cols[rg[q]];
  const float lcv[4] = {lc.x, lc.y, lc.z, lc.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = rr0 + 16 * q;
    const bool ok = cv && r0 + rr < nrows;
    const int64_t pg = rg[q] + B < 2 * B ? rg[q] + B : rg[q] - B;
    const float sv[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float w = 0.f;
      if (ok && c + j != rg[q]) {
        const float lg = sv[j] * inv_t;
        w = expf(lg - lr[q]) + expf(lg - lcv[j]);
        if (c + j == pg) w -= 2.f;
        w *= coef;
      }
      mx = fmaxf(mx, fabsf(w));
      tile[cc + j][rr] = w;
    }
  }
  __syncthreads();
  // write: 64 W^T rows (c) x 16 float4 along r
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = tid + 256 * q;
    const int cc = idx >> 4, rr = 4 * (idx & 15);
    const int64_t c = c0 + cc, r = r0 + rr;
    if (c < ncols && r < nrows)  // nrows % 4 == 0 (host)
      *reinterpret_cast<float4*>(Wt + c * nrows + r) =
          make_float4(tile[cc][rr], tile[cc][rr + 1], tile[cc][rr + 2], tile[cc][rr + 3]);
  }
  absmax_publish(mx, wmax);
}

// ---- transposed h3 formulation (impl 3) ------------------------------------------
// S^T = R_cols R_rows^T [ncols][nrows] by the h3 GEMM (the columns as its A
// operand, split in registers with their per-tensor scale; the rows' h3
// image as B), so that the backward's W^T is elementwise in S^T's own layout
// (no LDS transpose) and feeds the h3 weight-gradient product dR = (W^T)^T
// R_cols directly.  The row logsumexp becomes a reduction down S^T's columns:
// partial (max, sum) per block of kColLseC columns of S (rows of S^T), merged
// in a fixed order by a second launch.
constexpr int64_t kColLseC = 128;  // S columns (S^T rows) per partial
// block: 256 consecutive r (a lane holds 4, one float4 per S^T row) x kColLseC
// S^T rows, the 4 waves striding them; partial[split][r] = (max, sum)
__global__ __launch_bounds__(256) void k_ntxent_col_lse_partial(
    const float* __restrict__ St, int64_t nrows, int64_t ncols, const int32_t* __restrict__ gidx,
    float inv_t, float2* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 256 + 4 * lane;  // nrows % 4 == 0 (host)
  const bool live = r0 < nrows;
  const int64_t rl = live ? r0 : 0;
  const int4 g4 = *reinterpret_cast<const int4*>(gidx + rl);
  const int64_t rg[4] = {g4.x, g4.y, g4.z, g4.w};
  const int64_t c0 = (int64_t)blockIdx.y * kColLseC;
  const int64_t c1 = c0 + kColLseC < ncols ? c0 + kColLseC : ncols;
  float m[4], sum[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = -INFINITY;
    sum[j] = 0.f;
  }
  // eight S^T rows per round in flight, each one float4 per lane
  for (int64_t c = c0 + wave; c < c1; c += 32) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t cc = c + 4 * u;
      v[u] = *reinterpret_cast<const float4*>(St + (cc < c1 ? cc : c0) * nrows + rl);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x[8], bm = -INFINITY;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t cc = c + 4 * u;
        const float e = j == 0 ? v[u].x : j == 1 ? v[u].y : j == 2 ? v[u].z : v[u].w;
        x[u] = (cc < c1 && cc != rg[j]) ? e * inv_t : -INFINITY;
        bm = fmaxf(bm, x[u]);
      }
      if (bm > -INFINITY) {
        const float nm = fmaxf(m[j], bm);
        float acc = sum[j] * expf(m[j] - nm);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += expf(x[u] - nm);
        m[j] = nm;
        sum[j] = acc;
      }
    }
  }
  __shared__ float4 wm[4][64], ws[4][64];
  wm[wave][lane] = make_float4(m[0], m[1], m[2], m[3]);
  ws[wave][lane] = make_float4(sum[0], sum[1], sum[2], sum[3]);
  __syncthreads();
  if (wave != 0 || !live) return;
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    const float4 mo4 = wm[w][lane], so4 = ws[w][lane];
    const float mo[4] = {mo4.x, mo4.y, mo4.z, mo4.w}, so[4] = {so4.x, so4.y, so4.z, so4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float nm = fmaxf(m[j], mo[j]);
      sum[j] = nm == -INFINITY ? 0.f : sum[j] * expf(m[j] - nm) + so[j] * expf(mo[j] - nm);
      m[j] = nm;
    }
  }
  float2* o = part + (int64_t)blockIdx.y * nrows + r0;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = make_float2(m[j], sum[j]);
}

// lse_r over the splits in order; the loss row (lse_r - S_{r,p(r)} / T) / 2B
__global__ __launch_bounds__(256) void k_ntxent_col_lse_final(
    const float2* __restrict__ part, int64_t splits, const float* __restrict__ St, int64_t nrows,
    const int32_t* __restrict__ gidx, int64_t B, float inv_t, float inv_2b, float* __restrict__ lse,
    float* __restrict__ loss) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  const int64_t rg = gidx[r];
  const int64_t pg = (rg + B) % (2 * B);
  const float pos = St[pg * nrows + r];
  float m = -INFINITY, sum = 0.f;
  for (int64_t q = 0; q < splits; q += 8) {
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = q + u < splits ? part[(q + u) * nrows + r] : make_float2(-INFINITY, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float nm = fmaxf(m, v[u].x);
      sum = nm == -INFINITY ? 0.f : sum * expf(m - nm) + v[u].y * expf(v[u].x - nm);
      m = nm;
    }
  }
  const float l = m + logf(sum);
  lse[r] = l;
  loss[r] = (l - pos * inv_t) * inv_2b;
}

// W^T[c][r] = g/(2B T) (exp(S_rc/T - lse_r) + exp(S_rc/T - lse_c) - 2 [c = p(r)]),
// 0 at c = r, elementwise from S^T (float4 runs along r)
__global__ __launch_bounds__(256) void k_ntxent_weights_t(
    const float* __restrict__ St, float* __restrict__ Wt, int64_t nrows, int64_t ncols,
    const int32_t* __restrict__ gidx, const float* __restrict__ lse_cols,
    const float* __restrict__ grad_loss, int64_t B, float inv_t) {
  const int64_t per = nrows / 4;  // nrows % 4 == 0 (host)
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < ncols * per) {
    const int64_t c = q / per, r0 = 4 * (q - c * per);
    const float coef = (*grad_loss) * inv_t / (float)(2 * B);
    const float4 v = *reinterpret_cast<const float4*>(St + c * nrows + r0);
    const int4 g4 = *reinterpret_cast<const int4*>(gidx + r0);
    const int64_t rg[4] = {g4.x, g4.y, g4.z, g4.w};
    const float lc = lse_cols[c];
    float lr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) lr[j] = lse_cols[rg[j]];
    const float sv[4] = {v.x, v.y, v.z, v.w};
    float w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w[j] = 0.f;
      if (c != rg[j]) {
        const float lg = sv[j] * inv_t;
        float e = expf(lg - lr[j]) + expf(lg - lc);
        const int64_t pg = rg[j] + B < 2 * B ? rg[j] + B : rg[j] - B;
        if (c == pg) e -= 2.f;
        w[j] = e * coef;
      }
    }
    *reinterpret_cast<float4*>(Wt + c * nrows + r0) = make_float4(w[0], w[1], w[2], w[3]);
  }
}

// impl 3's scales: the columns' max slot (plain stores, as k_ntxent_absmax_plain)
// and W's slot set to its bound, |W| <= 2 |g| / (2B T): the positive pair's
// -2 dominates every row, so max |W| is within a factor (1 - P) of the bound
// and the h3 scale (a power of two) is the one the measured max would give
// but for rows whose positive probability P exceeds 1/2
__global__ __launch_bounds__(1024) void k_ntxent_absmax_bound(const float* __restrict__ x,
                                                             int64_t n4, float* __restrict__ slot,
                                                             float* __restrict__ wslot,
                                                             const float* __restrict__ grad_loss,
                                                             int64_t B, float inv_t) {
  float m = absmax4_range(reinterpret_cast<const float4*>(x),
                          (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n4,
                          (int64_t)gridDim.x * blockDim.x);
  m = block_max(m);
  if (threadIdx.x == 0) {
    slot[blockIdx.x * kMaxSlotStride] = m;
    wslot[blockIdx.x * kMaxSlotStride] = 2.f * fabsf(*grad_loss) * inv_t / (float)(2 * B);
  }
}

// rhat = r / max(||r||, 1e-8) (cosine) or r (dot); norm saved for the backward
__global__ __launch_bounds__(256) void k_ntxent_prep(const float* __restrict__ r,
                                                     float* __restrict__ rhat,
                                                     float* __restrict__ norm, int64_t n,
                                                     int64_t C, int cosine) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= n) return;
  const float* x = r + row * C;
  float den = 1.f;
  if (cosine) {
    float ss = 0.f;
    for (int64_t c = lane; c < C; c += 64) ss += x[c] * x[c];
    ss = wave_sum(ss);
    den = fmaxf(sqrtf(ss), 1e-8f);
  }
  if (lane == 0) norm[row] = den;
  for (int64_t c = lane; c < C; c += 64) rhat[row * C + c] = cosine ? x[c] / den : x[c];
}

__global__ __launch_bounds__(256) void k_ntxent_prep_bwd(const float* __restrict__ drhat,
                                                         const float* __restrict__ rhat,
                                                         const float* __restrict__ norm,
                                                         float* __restrict__ dr, int64_t n,
                                                         int64_t C, int cosine) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= n) return;
  const float* g = drhat + row * C;
  if (!cosine) {
    for (int64_t c = lane; c < C; c += 64) dr[row * C + c] = g[c];
    return;
  }
  float den = norm[row];
  const float* y = rhat + row * C;
  float dot = 0.f;
  for (int64_t c = lane; c < C; c += 64) dot += g[c] * y[c];
  dot = wave_sum(dot);
  // norm clamped at eps: rhat = r / eps is linear in r
  bool clamped = !(den > 1e-8f);
  for (int64_t c = lane; c < C; c += 64)
    dr[row * C + c] = clamped ? g[c] / den : (g[c] - dot * y[c]) / den;
}

// The paired step's two row scalings in one pass (molclr.py:63-64 then
// nt_xent.py:40-45): z = [zis; zjs] ([2 Bl, C], GINet.forward_pair), R =
// [zjs; zis] (nt_xent.py:48) by a row swap, y = F.normalize(R row) (eps1), rhat =
// y / max(|y|, 1e-8) (cosine) or y.  Same per-lane loops and wave sums as
// k_l2norm_fwd followed by k_ntxent_prep: bit-identical results, one launch,
// no torch.cat.  y, |z| (n1) and the clamped |y| (n2) are kept for the backward.
__device__ __forceinline__ int64_t pair_src(int64_t r, int64_t Bl) { return r < Bl ? r + Bl : r - Bl; }

__global__ __launch_bounds__(256) void k_ntxent_prep_pair(const float* __restrict__ z,
                                                          float* __restrict__ y,
                                                          float* __restrict__ rhat,
                                                          float* __restrict__ n1,
                                                          float* __restrict__ n2, int64_t Bl,
                                                          int64_t C, float eps1, int cosine) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= 2 * Bl) return;
  const float* zr = z + pair_src(r, Bl) * C;
  float ss = 0.f;
  for (int64_t c = lane; c < C; c += 64) ss += zr[c] * zr[c];
  ss = wave_sum(ss);
  const float nrm = sqrtf(ss);
  const float d1 = fmaxf(nrm, eps1);
  float* yr = y + r * C;
  float ss2 = 0.f;
  for (int64_t c = lane; c < C; c += 64) {
    const float v = zr[c] / d1;
    yr[c] = v;
    ss2 += v * v;
  }
  float d2 = 1.f;
  if (cosine) {
    ss2 = wave_sum(ss2);
    d2 = fmaxf(sqrtf(ss2), 1e-8f);
  }
  if (lane == 0) {
    n1[r] = nrm;
    n2[r] = d2;
  }
  for (int64_t c = lane; c < C; c += 64) rhat[r * C + c] = cosine ? yr[c] / d2 : yr[c];
}

// dz (rows of z, un-swapped) from drhat: k_ntxent_prep_bwd then k_l2norm_bwd,
// the same arithmetic per element (dy staged in dz's row)
__global__ __launch_bounds__(256) void k_ntxent_prep_pair_bwd(
    const float* __restrict__ drhat, const float* __restrict__ rhat, const float* __restrict__ n2,
    const float* __restrict__ y, const float* __restrict__ n1, float* __restrict__ dz, int64_t Bl,
    int64_t C, float eps1, int cosine) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= 2 * Bl) return;
  const float* g = drhat + r * C;
  float* out = dz + pair_src(r, Bl) * C;
  if (!cosine) {
    for (int64_t c = lane; c < C; c += 64) out[c] = g[c];
  } else {
    const float den = n2[r];
    const float* rh = rhat + r * C;
    float dot = 0.f;
    for (int64_t c = lane; c < C; c += 64) dot += g[c] * rh[c];
    dot = wave_sum(dot);
    const bool clamped = !(den > 1e-8f);
    for (int64_t c = lane; c < C; c += 64) out[c] = clamped ? g[c] / den : (g[c] - dot * rh[c]) / den;
  }
  const float nrm = n1[r];
  const float* yr = y + r * C;
  if (nrm > eps1) {
    float dot = 0.f;
    for (int64_t c = lane; c < C; c += 64) dot += out[c] * yr[c];
    dot = wave_sum(dot);
    for (int64_t c = lane; c < C; c += 64) out[c] = (out[c] - dot * yr[c]) / nrm;
  } else {
    for (int64_t c = lane; c < C; c += 64) out[c] = out[c] / eps1;
  }
}

// column splits: single-wave workgroups per (32-row block, split); measured
// best at ~512 waves for the forward and ~1024 for the backward
// (tools/ntxent_scale.py; the backward's partials are [nrows][C] each)
int64_t ntx_splits(int64_t nrows, int64_t ncols, int64_t target = 512) {
  int64_t rb = (nrows + 31) / 32, nch = (ncols + 31) / 32;
  int64_t s = (target + rb - 1) / rb;
  if (s > nch) s = nch;
  if (s < 1) s = 1;
  return s;
}

}  // namespace

MOLCLR_API int molclr_ntxent_prep(const float* r, float* rhat, float* norm, int64_t n, int64_t C,
                                  int cosine, molclr_stream_t stream) {
  MOLCLR_REQUIRE(C > 0 && n >= 0, "ntxent_prep: bad sizes");
  if (n == 0) return MOLCLR_OK;
  hipLaunchKernelGGL(k_ntxent_prep, dim3(molclr::ceil_div(n * 64, 256)), dim3(256), 0,
                     molclr::as_stream(stream), r, rhat, norm, n, C, cosine);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ntxent_prep_bwd(const float* drhat, const float* rhat, const float* norm,
                                      float* dr, int64_t n, int64_t C, int cosine,
                                      molclr_stream_t stream) {
  MOLCLR_REQUIRE(C > 0 && n >= 0, "ntxent_prep_bwd: bad sizes");
  if (n == 0) return MOLCLR_OK;
  hipLaunchKernelGGL(k_ntxent_prep_bwd, dim3(molclr::ceil_div(n * 64, 256)), dim3(256), 0,
                     molclr::as_stream(stream), drhat, rhat, norm, dr, n, C, cosine);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ntxent_prep_pair(const float* z, float* y, float* rhat, float* n1, float* n2,
                                       int64_t batch_local, int64_t C, double eps, int cosine,
                                       molclr_stream_t stream) {
  MOLCLR_REQUIRE(C > 0 && batch_local >= 0 && (batch_local == 0 || (z && y && rhat && n1 && n2)),
                 "ntxent_prep_pair: bad arguments");
  if (batch_local == 0) return MOLCLR_OK;
  hipLaunchKernelGGL(k_ntxent_prep_pair, dim3(molclr::ceil_div(2 * batch_local * 64, 256)),
                     dim3(256), 0, molclr::as_stream(stream), z, y, rhat, n1, n2, batch_local, C,
                     (float)eps, cosine);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ntxent_prep_pair_bwd(const float* drhat, const float* rhat, const float* n2,
                                           const float* y, const float* n1, float* dz,
                                           int64_t batch_local, int64_t C, double eps, int cosine,
                                           molclr_stream_t stream) {
  MOLCLR_REQUIRE(C > 0 && batch_local >= 0, "ntxent_prep_pair_bwd: bad arguments");
  if (batch_local == 0) return MOLCLR_OK;
  hipLaunchKernelGGL(k_ntxent_prep_pair_bwd, dim3(molclr::ceil_div(2 * batch_local * 64, 256)),
                     dim3(256), 0, molclr::as_stream(stream), drhat, rhat, n2, y, n1, dz,
                     batch_local, C, (float)eps, cosine);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

constexpr int64_t kBwdWaves = 1024;

namespace {

// workspace of the GEMM formulation: the column planes, S / W, and both
// GEMMs' split-K space side by side (the backward without a kept S takes the
// similarity GEMM's and then the dR GEMM's from one workspace)
size_t ntx_gemm_ws(int64_t nrows, int64_t ncols, int64_t C) {
  size_t g1 = molclr_gemm_f32_workspace_bytes(nrows, ncols, C);
  size_t g2 = molclr_gemm_f32_workspace_bytes(nrows, C, ncols);
  return molclr_bplanes_bytes(ncols, C) + (size_t)nrows * ncols * sizeof(float) + g1 + g2 +
         4 * 256;
}
// shapes the h3 formulation takes: the h3 GEMM's K = C <= 1024, float4 rows
// of the row-major S, the weight-gradient kernel's long K (ncols >= 1024)
bool ntx_h3_ok(int64_t nrows, int64_t ncols, int64_t C) {
  return nrows % 4 == 0 && ncols % 4 == 0 && C % 4 == 0 && C <= 1024 && ncols >= 1024;
}
// workspace of the h3 formulation: W^T (and S when not kept), the rows' h3 image, the max
// slots of the columns and of W, the lse partials, the weight-gradient space
size_t ntx_h3_ws(int64_t nrows, int64_t ncols, int64_t C) {
  // W^T, and S when the backward recomputes it; the columns' image (impl 2)
  // or the rows' (impl 3) and impl 3's logsumexp partials
  const int64_t splits = (ncols + kColLseC - 1) / kColLseC;
  return 2 * (size_t)nrows * ncols * sizeof(float) + molclr_hplanes_bytes(ncols, C) +
         molclr_hplanes_bytes(nrows, C) + (size_t)splits * nrows * sizeof(float2) +
         3 * (size_t)kMaxSlotFloats * sizeof(float) +
         molclr_linear_wgrad_workspace_bytes(ncols, nrows, C) + 10 * 256;
}
// automatic choice: the fused kernels below 2^20 elements of S; the x6 GEMM
// formulation up to 2^22 (c2's 1024 x 1024: 41 us per step against 52 for
// h3, whose fixed costs -- max slots, the columns' image -- dominate there);
// the h3 formulation from 2^22 where its shapes allow (the c4 rank shard
// 1024 x 8192 x 256: 117.6 us against 128.6, tools/ntxent_c4.py)
int ntx_impl(int64_t nrows, int64_t ncols, int64_t C, int impl) {
  if (impl >= 0) return impl;
  if (nrows * ncols < (1 << 20) || ncols % 4 || C % 4) return 0;
  return nrows * ncols >= (1 << 22) && ntx_h3_ok(nrows, ncols, C) ? 2 : 1;
}

// S = rows cols^T into `sim` (or, when null, the workspace; planes of the
// columns made first); returns the GEMM's error code
int ntx_similarity(const float* rows, const float* cols, int64_t nrows, int64_t ncols, int64_t C,
                   molclr::Workspace& w, float* sim, float** S_out, hipStream_t s) {
  molclr::TimerKindScope timed_as(molclr::kTimeNtxent);
  uint16_t* planes = reinterpret_cast<uint16_t*>(w.take<char>(molclr_bplanes_bytes(ncols, C)));
  float* S = w.take<float>((size_t)nrows * ncols);
  if (sim) S = sim;
  const size_t gws = molclr_gemm_f32_workspace_bytes(nrows, ncols, C);
  void* g = w.take<char>(gws);
  if (!w.ok()) {
    molclr::set_error("ntxent: workspace too small");
    return MOLCLR_ERR_WORKSPACE;
  }
  int rc = molclr_bplanes_make(cols, ncols, C, C, 0, planes, s);
  if (rc) return rc;
  rc = molclr_gemm_f32_bplanes(rows, planes, S, nrows, ncols, C, C, ncols, 0, MOLCLR_EPI_NONE,
                               nullptr, nullptr, 0, g, gws, s);
  *S_out = S;
  return rc;
}

// S = rows cols^T into S (h3, row-major [nrows][ncols]): the rows' max slot
// (plain stores), the columns' h3 image (its own max slot included)
int ntx_similarity_h3(const float* rows, const float* cols, int64_t nrows, int64_t ncols, int64_t C,
                      float* S, uint16_t* planes, float* rmax, hipStream_t s) {
  molclr::TimerKindScope timed_as(molclr::kTimeNtxent);
  // the columns' image and both max slots (rows', columns') in two launches
  int rc = molclr::hplanes_make_and_max(cols, ncols, C, planes, rows, nrows, C, rmax, s);
  if (rc) return rc;
  return molclr_gemm_f32_h3(rows, rmax, 0, planes, S, nrows, ncols, C, C, ncols,
                            MOLCLR_EPI_NONE, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                            nullptr, s);
}

// S^T = cols rows^T into St (h3, row-major [ncols][nrows]): the rows' h3
// image with its max slot and the columns' max slot (cmax) in two launches
int ntx_similarity_t(const float* rows, const float* cols, int64_t nrows, int64_t ncols, int64_t C,
                     float* St, uint16_t* rplanes, float* cmax, hipStream_t s) {
  molclr::TimerKindScope timed_as(molclr::kTimeNtxent);
  int rc = molclr::hplanes_make_and_max(rows, nrows, C, rplanes, cols, ncols, C, cmax, s);
  if (rc) return rc;
  return molclr_gemm_f32_h3(cols, cmax, 0, rplanes, St, ncols, nrows, C, C, nrows,
                            MOLCLR_EPI_NONE, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                            nullptr, s);
}

}  // namespace

MOLCLR_API size_t molclr_ntxent_workspace_bytes(int64_t nrows, int64_t ncols, int64_t C) {
  int64_t sp = ntx_splits(nrows, ncols);
  size_t fwd = (size_t)(2 * sp + 1) * nrows * sizeof(float);
  size_t bwd = (size_t)ntx_splits(nrows, ncols, kBwdWaves) * nrows * C * sizeof(float);
  size_t fused = (fwd > bwd ? fwd : bwd) + 256;
  size_t gemm = ntx_gemm_ws(nrows, ncols, C);
  size_t h3 = ntx_h3_ok(nrows, ncols, C) ? ntx_h3_ws(nrows, ncols, C) : 0;
  size_t m = fused > gemm ? fused : gemm;
  return m > h3 ? m : h3;
}

MOLCLR_API size_t molclr_ntxent_sim_bytes(int64_t nrows, int64_t ncols, int64_t C, int impl) {
  if (nrows <= 0 || ncols <= 0 || C <= 0 || ntx_impl(nrows, ncols, C, impl) == 0) return 0;
  // row-major S [nrows][ncols] for both GEMM formulations (impl 1 and 2): the
  // forward writes it, the backward reads it back
  return (size_t)nrows * ncols * sizeof(float);
}

MOLCLR_API int molclr_ntxent_fwd_impl(const float* rows, const int32_t* gidx, const float* cols,
                                      int64_t nrows, int64_t ncols, int64_t C, int64_t B, double T,
                                      float* lse, float* loss, float* sim, void* workspace,
                                      size_t ws_bytes, molclr_stream_t stream, int impl) {
  MOLCLR_REQUIRE(C > 0 && C % 8 == 0, "ntxent_fwd: C=%lld must be a multiple of 8", (long long)C);
  MOLCLR_REQUIRE(B > 0 && ncols == 2 * B, "ntxent_fwd: ncols must equal 2*batch_size");
  MOLCLR_REQUIRE(nrows > 0 && nrows <= ncols, "ntxent_fwd: bad nrows");
  MOLCLR_REQUIRE(T > 0, "ntxent_fwd: temperature must be > 0");
  MOLCLR_REQUIRE(impl >= -1 && impl <= 3, "ntxent_fwd: bad impl %d", impl);
  MOLCLR_REQUIRE_WS(ws_bytes, molclr_ntxent_workspace_bytes(nrows, ncols, C));
  hipStream_t s = molclr::as_stream(stream);
  const float inv_t = (float)(1.0 / T);
  molclr::Workspace w(workspace, ws_bytes);
  const int which = ntx_impl(nrows, ncols, C, impl);
  if (which == 3) {
    MOLCLR_REQUIRE(ntx_h3_ok(nrows, ncols, C),
                   "ntxent_fwd: the h3 formulations need nrows, ncols, C multiples of 4, "
                   "C <= 1024, ncols >= 1024");
    float* St = w.take<float>((size_t)nrows * ncols);
    if (sim) St = sim;
    uint16_t* rplanes = reinterpret_cast<uint16_t*>(w.take<char>(molclr_hplanes_bytes(nrows, C)));
    float* cmax = w.take<float>(kMaxSlotFloats);
    const int64_t splits = (ncols + kColLseC - 1) / kColLseC;
    float2* part = w.take<float2>((size_t)splits * nrows);
    if (!w.ok()) {
      molclr::set_error("ntxent_fwd: workspace too small");
      return MOLCLR_ERR_WORKSPACE;
    }
    const int rc = ntx_similarity_t(rows, cols, nrows, ncols, C, St, rplanes, cmax, s);
    if (rc) return rc;
    molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_col_lse_partial,
                         dim3((unsigned)molclr::ceil_div(nrows, 256), (unsigned)splits), dim3(256), 0,
                         s, St, nrows, ncols, gidx, inv_t, part);
    molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_col_lse_final,
                         dim3((unsigned)molclr::ceil_div(nrows, 256)), dim3(256), 0, s, part, splits,
                         St, nrows, gidx, B, inv_t, (float)(1.0 / (2.0 * B)), lse, loss);
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  if (which == 2) {
    MOLCLR_REQUIRE(ntx_h3_ok(nrows, ncols, C),
                   "ntxent_fwd: the h3 formulation needs nrows, ncols, C multiples of 4, "
                   "C <= 1024, ncols >= 1024");
    float* S = w.take<float>((size_t)nrows * ncols);
    if (sim) S = sim;
    uint16_t* planes = reinterpret_cast<uint16_t*>(w.take<char>(molclr_hplanes_bytes(ncols, C)));
    float* rmax = w.take<float>(kMaxSlotFloats);
    if (!w.ok()) {
      molclr::set_error("ntxent_fwd: workspace too small");
      return MOLCLR_ERR_WORKSPACE;
    }
    const int rc = ntx_similarity_h3(rows, cols, nrows, ncols, C, S, planes, rmax, s);
    if (rc) return rc;
    molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_row_lse,
                         dim3((unsigned)nrows), dim3(64 * kLseWaves), 0, s, S,
                         nrows, ncols, gidx, B, inv_t, (float)(1.0 / (2.0 * B)), lse, loss);
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  if (which == 1) {
    MOLCLR_REQUIRE(ncols % 4 == 0, "ntxent_fwd: the GEMM formulation needs ncols %% 4 == 0");
    float* S = nullptr;
    const int rc = ntx_similarity(rows, cols, nrows, ncols, C, w, sim, &S, s);
    if (rc) return rc;
    molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_row_lse,
                         dim3((unsigned)nrows), dim3(64 * kLseWaves), 0, s, S,
                         nrows, ncols, gidx, B, inv_t, (float)(1.0 / (2.0 * B)), lse, loss);
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  int64_t sp = ntx_splits(nrows, ncols);
  int64_t nch = (ncols + 31) / 32;
  int64_t cps = (nch + sp - 1) / sp;
  sp = (nch + cps - 1) / cps;
  float* pm = w.take<float>(sp * nrows);
  float* ps = w.take<float>(sp * nrows);
  float* pos = w.take<float>(nrows);
  const dim3 grid((unsigned)((nrows + 31) / 32), (unsigned)sp);
#define MOLCLR_NXF(NQ)                                                                           \
  molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_fwd_partial<NQ>, grid, dim3(64), 0, s, rows, \
                       gidx, cols, nrows, ncols, C, B, inv_t, cps, pm, ps, pos)
  if (C == 256) MOLCLR_NXF(32);
  else if (C == 128) MOLCLR_NXF(16);
  else MOLCLR_NXF(0);
#undef MOLCLR_NXF
  hipLaunchKernelGGL(k_ntxent_fwd_final, dim3(molclr::ceil_div(nrows, 256)), dim3(256), 0, s, pm,
                     ps, pos, sp, nrows, (float)(1.0 / (2.0 * B)), lse, loss);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ntxent_fwd(const float* rows, const int32_t* gidx, const float* cols,
                                 int64_t nrows, int64_t ncols, int64_t C, int64_t B, double T,
                                 float* lse, float* loss, void* workspace, size_t ws_bytes,
                                 molclr_stream_t stream) {
  return molclr_ntxent_fwd_impl(rows, gidx, cols, nrows, ncols, C, B, T, lse, loss, nullptr,
                                workspace, ws_bytes, stream, -1);
}

MOLCLR_API int molclr_ntxent_bwd_impl(const float* rows, const int32_t* gidx, const float* cols,
                                      const float* lse_cols, const float* grad_loss, int64_t nrows,
                                      int64_t ncols, int64_t C, int64_t B, double T, const float* sim,
                                      float* drows, void* workspace, size_t ws_bytes,
                                      molclr_stream_t stream, int impl) {
  MOLCLR_REQUIRE(C > 0 && C % 32 == 0, "ntxent_bwd: C=%lld must be a multiple of 32", (long long)C);
  MOLCLR_REQUIRE(B > 0 && ncols == 2 * B, "ntxent_bwd: ncols must equal 2*batch_size");
  MOLCLR_REQUIRE(nrows > 0 && nrows <= ncols, "ntxent_bwd: bad nrows");
  MOLCLR_REQUIRE(impl >= -1 && impl <= 3, "ntxent_bwd: bad impl %d", impl);
  MOLCLR_REQUIRE_WS(ws_bytes, molclr_ntxent_workspace_bytes(nrows, ncols, C));
  hipStream_t s = molclr::as_stream(stream);
  const float inv_t = (float)(1.0 / T);
  const int which = ntx_impl(nrows, ncols, C, impl);
  if (which == 3) {
    MOLCLR_REQUIRE(ntx_h3_ok(nrows, ncols, C),
                   "ntxent_bwd: the h3 formulations need nrows, ncols, C multiples of 4, "
                   "C <= 1024, ncols >= 1024");
    molclr::Workspace w(workspace, ws_bytes);
    float* Wt = w.take<float>((size_t)nrows * ncols);
    uint16_t* rplanes = reinterpret_cast<uint16_t*>(w.take<char>(molclr_hplanes_bytes(nrows, C)));
    float* cmax = w.take<float>(kMaxSlotFloats);
    float* wmax = w.take<float>(kMaxSlotFloats);
    float* Sw = sim ? nullptr : w.take<float>((size_t)nrows * ncols);
    const size_t gws = molclr_linear_wgrad_workspace_bytes(ncols, nrows, C);
    void* g = w.take<char>(gws);
    if (!w.ok()) {
      molclr::set_error("ntxent_bwd: workspace too small");
      return MOLCLR_ERR_WORKSPACE;
    }
    int rc = 0;
    const float* St = sim;  // the forward's S^T, or recomputed here
    if (!sim) {
      rc = ntx_similarity_t(rows, cols, nrows, ncols, C, Sw, rplanes, cmax, s);
      if (rc) return rc;
      St = Sw;
    }
    {
      molclr::TimerKindScope timed_as(molclr::kTimeNtxent);
      // the columns' max slot and W's bound slot in one launch
      hipLaunchKernelGGL(k_ntxent_absmax_bound, dim3(kMaxSlotParts), dim3(1024), 0, s, cols,
                         ncols * C / 4, cmax, wmax, grad_loss, B, inv_t);
      molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_weights_t,
                           dim3((unsigned)molclr::ceil_div(ncols * nrows / 4, 256)), dim3(256), 0, s,
                           St, Wt, nrows, ncols, gidx, lse_cols, grad_loss, B, inv_t);
      // dR[r][k] = Σ_c W^T[c][r] cols[c][k]: the weight-gradient product
      rc = molclr_linear_wgrad_h3(Wt, wmax, cols, cmax, drows, nullptr, ncols, nrows, C, nrows, C,
                                  0, g, gws, s);
    }
    if (rc) return rc;
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  if (which == 2) {
    MOLCLR_REQUIRE(ntx_h3_ok(nrows, ncols, C),
                   "ntxent_bwd: the h3 formulation needs nrows, ncols, C multiples of 4, "
                   "C <= 1024, ncols >= 1024");
    molclr::Workspace w(workspace, ws_bytes);
    float* Wt = w.take<float>((size_t)nrows * ncols);
    uint16_t* planes = reinterpret_cast<uint16_t*>(w.take<char>(molclr_hplanes_bytes(ncols, C)));
    float* cmax = w.take<float>(kMaxSlotFloats);
    float* wmax = w.take<float>(kMaxSlotFloats);
    float* rmax = w.take<float>(kMaxSlotFloats);
    float* Sw = sim ? nullptr : w.take<float>((size_t)nrows * ncols);
    const size_t gws = molclr_linear_wgrad_workspace_bytes(ncols, nrows, C);
    void* g = w.take<char>(gws);
    if (!w.ok()) {
      molclr::set_error("ntxent_bwd: workspace too small");
      return MOLCLR_ERR_WORKSPACE;
    }
    int rc = 0;
    const float* S = sim;  // the forward's S, or recomputed here
    if (!sim) {
      rc = ntx_similarity_h3(rows, cols, nrows, ncols, C, Sw, planes, rmax, s);
      if (rc) return rc;
      S = Sw;
    }
    {
      molclr::TimerKindScope timed_as(molclr::kTimeNtxent);
      // the columns' max slot and W's zeroed slot in one launch
      hipLaunchKernelGGL(k_ntxent_absmax_plain, dim3(kMaxSlotParts), dim3(1024), 0, s, cols,
                         ncols * C / 4, cmax, wmax);
      molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_weights_tt,
                           dim3((unsigned)molclr::ceil_div(ncols, kWT),
                                (unsigned)molclr::ceil_div(nrows, kWT)),
                           dim3(256), 0, s, S, Wt, nrows, ncols, gidx, lse_cols, grad_loss, B,
                           inv_t, wmax);
      // dR[r][k] = Σ_c W^T[c][r] cols[c][k]: the weight-gradient product
      rc = molclr_linear_wgrad_h3(Wt, wmax, cols, cmax, drows, nullptr, ncols, nrows, C, nrows, C,
                                  0, g, gws, s);
    }
    if (rc) return rc;
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  if (which == 1) {
    MOLCLR_REQUIRE(ncols % 4 == 0, "ntxent_bwd: the GEMM formulation needs ncols %% 4 == 0");
    molclr::Workspace w(workspace, ws_bytes);
    int rc;
    const float* S = sim;  // the forward's similarities, or recomputed here
    float* W;
    if (sim) {
      W = w.take<float>((size_t)nrows * ncols);
    } else {
      float* Sw = nullptr;
      rc = ntx_similarity(rows, cols, nrows, ncols, C, w, nullptr, &Sw, s);
      if (rc) return rc;
      S = W = Sw;  // in place
    }
    molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_weights,
                         dim3((unsigned)molclr::ceil_div(nrows * ncols / 4, 256)), dim3(256), 0, s,
                         S, W, nrows, ncols, gidx, lse_cols, grad_loss, B, inv_t);
    // dR[r][k] = Σ_c W[r][c] cols[c][k]: A = W (row-major, K = ncols), B = cols ([K][N])
    const size_t gws = molclr_gemm_f32_workspace_bytes(nrows, C, ncols);
    void* g = w.take<char>(gws);
    if (!w.ok()) {
      molclr::set_error("ntxent_bwd: workspace too small");
      return MOLCLR_ERR_WORKSPACE;
    }
    {
      molclr::TimerKindScope timed_as(molclr::kTimeNtxent);
      rc = molclr_gemm_f32(W, cols, drows, nrows, C, ncols, ncols, C, C, 0, 1, MOLCLR_EPI_NONE,
                           nullptr, nullptr, 0, g, gws, s);
    }
    if (rc) return rc;
    MOLCLR_LAUNCHED();
    return MOLCLR_OK;
  }
  int64_t sp = ntx_splits(nrows, ncols, kBwdWaves);
  int64_t nch = (ncols + 31) / 32;
  int64_t cps = (nch + sp - 1) / sp;
  sp = (nch + cps - 1) / cps;
  constexpr int KT = 8;
  int64_t kgroups = (C / 32 + KT - 1) / KT;
  float* partial = (float*)workspace;
  const dim3 grid((unsigned)((nrows + 31) / 32), (unsigned)sp, (unsigned)kgroups);
#define MOLCLR_NXB(NQ)                                                                       \
  molclr::launch_timed(molclr::kTimeNtxent, k_ntxent_bwd_partial<KT, NQ>, grid, dim3(64), 0, s, \
                       rows, gidx, cols, lse_cols, grad_loss, nrows, ncols, C, B, inv_t, cps,   \
                       partial)
  if (C == 256) MOLCLR_NXB(32);
  else if (C == 128) MOLCLR_NXB(16);
  else MOLCLR_NXB(0);
#undef MOLCLR_NXB
  hipLaunchKernelGGL(k_reduce_splits, dim3(molclr::ceil_div(nrows * C, 256)), dim3(256), 0, s,
                     partial, sp, nrows * C, drows);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ntxent_bwd(const float* rows, const int32_t* gidx, const float* cols,
                                 const float* lse_cols, const float* grad_loss, int64_t nrows,
                                 int64_t ncols, int64_t C, int64_t B, double T, float* drows,
                                 void* workspace, size_t ws_bytes, molclr_stream_t stream) {
  return molclr_ntxent_bwd_impl(rows, gidx, cols, lse_cols, grad_loss, nrows, ncols, C, B, T,
                                nullptr, drows, workspace, ws_bytes, stream, -1);
}
