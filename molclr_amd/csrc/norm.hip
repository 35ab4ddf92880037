// Row-band reductions and normalisations: column sums (bias gradients),
// BatchNorm1d(+ReLU) forward/backward, segment mean/add pooling, F.normalize.
//
// Reference: models/ginet_molclr.py:107-113 (BatchNorm1d in train mode, ReLU on
// all but the last layer, dropout p = drop_ratio = 0, global_mean_pool),
// molclr.py:63-64 (F.normalize).  Column statistics are reduced in a fixed
// order (per-thread Welford -> per-block Chan merge -> per-column merge over
// blocks), so every result is run-to-run deterministic.
//
// Band layout (molclr::make_band): a block covers `band` consecutive rows x all
// D/4 float4 columns, each wave reading 1 KiB of contiguous memory.
#include "common.h"

#include <math.h>

namespace {

constexpr int kT = 256;

__host__ __device__ __forceinline__ int64_t band_parts(int64_t rows, int band) {
  // ~16 row-iterations per thread: many blocks keep enough loads in flight;
  // the final merge over the partitions is parallel (k_*_final)
  const int64_t unit = (int64_t)band * 16;
  int64_t P = (rows + unit - 1) / unit;
  if (P > 1024) P = 1024;
  if (P < 1) P = 1;
  return P;
}

// an upper bound of sum_s band_parts(n_s) over any split of `rows` rows into
// nseg segments: ceil(a / u) + ceil(b / u) <= ceil((a + b) / u) + 1, and an
// empty segment still takes one partition.  The per-segment cap (1024) applies
// to each segment, so the uncapped total is bounded first and only then
// capped at nseg * 1024 (capping the total at 1024 first undercounts: two
// segments of 865 partitions each need 1730).
int64_t band_parts_bound(int64_t rows, int band, int nseg) {
  const int64_t unit = (int64_t)band * 16;
  int64_t P = (rows + unit - 1) / unit + nseg;
  if (P > (int64_t)nseg * 1024) P = (int64_t)nseg * 1024;
  return P;
}

// ---------------------------------------------------------------------------
// column sums
// ---------------------------------------------------------------------------
__global__ void k_colsum_partial(const float4* __restrict__ X, int64_t rows, int d4, int64_t ld4,
                                 int band, int64_t rows_per_part, float4* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float4 red[];  // [band][d4]
  const int tid = threadIdx.x;
  const bool live = tid < band * d4;
  const int r = live ? tid / d4 : 0, c = live ? tid - r * d4 : 0;
  const int64_t beg = (int64_t)blockIdx.x * rows_per_part;
  int64_t end = beg + rows_per_part;
  if (end > rows) end = rows;
  float4 acc = f4zero();
  if (live) {
#pragma unroll 4
    for (int64_t i = beg + r; i < end; i += band) acc = f4add(acc, X[i * ld4 + c]);
  }
  if (live) red[r * d4 + c] = acc;
  __syncthreads();
  if (live && r == 0) {
    float4 s = red[c];
    for (int q = 1; q < band; ++q) s = f4add(s, red[q * d4 + c]);
    partial[(int64_t)blockIdx.x * d4 + c] = s;
  }
}

// Final column reductions over P partial rows: a block owns kRedCols columns
// with kRedLanes lanes each; a lane folds the partials p = lane (mod
// kRedLanes), four loads in flight per step, then the lanes are combined by
// a fixed-order tree through LDS (deterministic, no long serial chain: the
// previous 16-lane form spent 8-19 us waiting on one dependent load at a time).
constexpr int kRedCols = 4, kRedLanes = 256;

// sum-tree over the lanes of red[kRedLanes][kRedCols]; lane 0 ends with the total
template <typename T>
__device__ __forceinline__ T lane_tree_sum(T (*red)[kRedCols], int rl, int cl, T v) {
  red[rl][cl] = v;
  __syncthreads();
#pragma unroll
  for (int stride = kRedLanes / 2; stride > 0; stride >>= 1) {
    if (rl < stride) red[rl][cl] = v = v + red[rl + stride][cl];
    __syncthreads();
  }
  return v;
}

// Σ_p partial[p][c] for the block's columns, per lane (strided, 4 loads in flight)
__device__ __forceinline__ float lane_fold(const float* __restrict__ partial, int64_t P,
                                           int64_t cols, int64_t c, int rl) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int64_t p = rl;
  for (; p + 3 * kRedLanes < P; p += 4 * kRedLanes) {
    a0 += partial[p * cols + c];
    a1 += partial[(p + kRedLanes) * cols + c];
    a2 += partial[(p + 2 * kRedLanes) * cols + c];
    a3 += partial[(p + 3 * kRedLanes) * cols + c];
  }
  for (; p < P; p += kRedLanes) a0 += partial[p * cols + c];
  return (a0 + a1) + (a2 + a3);
}

__global__ __launch_bounds__(kRedCols* kRedLanes) void k_colsum_final(
    const float* __restrict__ partial, int64_t P, int64_t cols, float* __restrict__ out,
    int accumulate) {
  __shared__ float red[kRedLanes][kRedCols];
  const int cl = threadIdx.x % kRedCols, rl = threadIdx.x / kRedCols;
  const int64_t c = (int64_t)blockIdx.x * kRedCols + cl;
  const float acc = c < cols ? lane_fold(partial, P, cols, c, rl) : 0.f;
  const float s = lane_tree_sum(red, rl, cl, acc);
  if (rl == 0 && c < cols) out[c] = accumulate ? out[c] + s : s;
}

// ---------------------------------------------------------------------------
// BatchNorm
//
// Segmented: the rows are `nseg` consecutive segments (the two contrastive
// views of a step run through one encoder pass), each normalised with its
// OWN batch statistics -- exactly as the reference's two separate forward
// calls (molclr.py:57,60) -- and the running statistics are updated once per
// segment, in segment order.  A segment is partitioned exactly as a
// one-segment call over its rows would be, so every per-segment result is
// bit-identical to that call.  Storage of z / y / dy / dz is fp32 or bf16
// (StF32 / StBF16); the statistics are always fp32.
// ---------------------------------------------------------------------------
struct Segs {
  int n;     // segments
  int band;  // the partition plan's row unit (make_band(D).band)
  int64_t rows[MOLCLR_MAX_SEGMENTS];  // host-sized: rows of every segment
  // device-sized (a captured step over padded buffers): the rows of every
  // segment live on the device and rows[] is unused; rows past the last
  // segment are padding -- zero output, zero gradient, no statistics
  const int64_t* drows;
};

__device__ __forceinline__ int64_t seg_n(const Segs& sg, int s) {
  return sg.drows ? sg.drows[s] : sg.rows[s];
}

// Segment s's rows [row0, row1) and partitions [part0, part0 + P), each
// partition rpp rows: exactly a one-segment call's plan over its rows.  s = -1
// for a spare partition / padding row of a device-sized plan.
struct SegAt {
  int s;
  int64_t row0, row1, part0, P, rpp;
};
__device__ __forceinline__ SegAt seg_info(const Segs& sg, int s) {
  int64_t r = 0, p = 0;
  for (int q = 0; q < s; ++q) {
    const int64_t n = seg_n(sg, q);
    r += n;
    p += band_parts(n, sg.band);
  }
  const int64_t n = seg_n(sg, s), P = band_parts(n, sg.band);
  return {s, r, r + n, p, P, (n > 0 ? n + P - 1 : P) / P};
}
__device__ __forceinline__ SegAt seg_of_part(const Segs& sg, int64_t b) {
  int64_t r = 0, p = 0;
  for (int s = 0; s < sg.n; ++s) {
    const int64_t n = seg_n(sg, s), P = band_parts(n, sg.band);
    if (b < p + P) return {s, r, r + n, p, P, (n > 0 ? n + P - 1 : P) / P};
    r += n;
    p += P;
  }
  return {-1, r, r, p, 0, 1};
}
// t / d4 in 32 bits when the whole index range fits (uniform branch)
__device__ __forceinline__ int64_t row_of(int64_t t, int d4, int64_t total4) {
  return total4 <= 0x7FFFFFFF ? (int64_t)((uint32_t)t / (uint32_t)d4) : t / d4;
}
__device__ __forceinline__ int seg_of_row(const Segs& sg, int64_t i) {
  int64_t r = 0;
  for (int s = 0; s < sg.n; ++s) {
    r += seg_n(sg, s);
    if (i < r) return s;
  }
  return -1;
}

struct Welford4 {
  float n;
  float4 mean, m2;
};

__device__ __forceinline__ void chan_merge(float& na, float4& ma, float4& qa, float nb, float4 mb,
                                           float4 qb) {
  if (nb == 0.f) return;
  if (na == 0.f) {
    na = nb;
    ma = mb;
    qa = qb;
    return;
  }
  float n = na + nb;
  float wb = nb / n, wab = na * nb / n;
  float4 d = make_float4(mb.x - ma.x, mb.y - ma.y, mb.z - ma.z, mb.w - ma.w);
  ma = make_float4(ma.x + d.x * wb, ma.y + d.y * wb, ma.z + d.z * wb, ma.w + d.w * wb);
  qa = make_float4(qa.x + qb.x + d.x * d.x * wab, qa.y + qb.y + d.y * d.y * wab,
                   qa.z + qb.z + d.z * d.z * wab, qa.w + qb.w + d.w * d.w * wab);
  na = n;
}

// partial layout: mean [P][d4] float4, m2 [P][d4] float4, n [P]
template <typename St>
__global__ void k_bn_stats_partial(const typename St::T* __restrict__ z, int d4, int band, Segs sg,
                                   float4* __restrict__ pmean, float4* __restrict__ pm2,
                                   float* __restrict__ pn) {
  extern __shared__ __attribute__((aligned(16))) float4 red[];  // [2][band][d4]
  const int tid = threadIdx.x;
  const bool live = tid < band * d4;
  const int r = live ? tid / d4 : 0, c = live ? tid - r * d4 : 0;
  const SegAt at = seg_of_part(sg, blockIdx.x);
  if (at.s < 0) return;  // spare partition of a device-sized plan (block-uniform)
  const int64_t beg = at.row0 + (blockIdx.x - at.part0) * at.rpp;
  int64_t end = beg + at.rpp;
  if (end > at.row1) end = at.row1;
  float n = 0.f;
  float4 mean = f4zero(), m2 = f4zero();
  if (live) {
#pragma unroll 4
    for (int64_t i = beg + r; i < end; i += band) {
      float4 x = St::ld(z, i * d4 + c);
      n += 1.f;
      float inv = 1.f / n;
      float4 d = make_float4(x.x - mean.x, x.y - mean.y, x.z - mean.z, x.w - mean.w);
      mean = make_float4(mean.x + d.x * inv, mean.y + d.y * inv, mean.z + d.z * inv,
                         mean.w + d.w * inv);
      m2 = make_float4(m2.x + d.x * (x.x - mean.x), m2.y + d.y * (x.y - mean.y),
                       m2.z + d.z * (x.z - mean.z), m2.w + d.w * (x.w - mean.w));
    }
    red[r * d4 + c] = mean;
    red[(band + r) * d4 + c] = m2;
  }
  __syncthreads();
  if (live && r == 0) {
    // rows handled by lane-row q: ceil((cnt - q) / band)
    int64_t cnt = end > beg ? end - beg : 0;
    float na = (float)(cnt > 0 ? (cnt + band - 1) / band : 0);
    float4 ma = red[c], qa = red[band * d4 + c];
    for (int q = 1; q < band; ++q) {
      float nb = (float)(cnt > q ? (cnt - q + band - 1) / band : 0);
      chan_merge(na, ma, qa, nb, red[q * d4 + c], red[(band + q) * d4 + c]);
    }
    pmean[(int64_t)blockIdx.x * d4 + c] = ma;
    pm2[(int64_t)blockIdx.x * d4 + c] = qa;
    if (c == 0) pn[blockIdx.x] = (float)cnt;
  }
}

__device__ __forceinline__ void bn_coeffs(float gamma, float beta, float mean, float invstd,
                                          float& scale, float& shift) {
  scale = gamma * invstd;
  shift = __fmaf_rn(-mean, scale, beta);
}

__device__ __forceinline__ void chan1(float& n, float& mean, float& m2, float nb, float mb, float qb) {
  if (nb == 0.f) return;
  if (n == 0.f) {
    n = nb;
    mean = mb;
    m2 = qb;
    return;
  }
  float nn = n + nb;
  float d = mb - mean;
  mean = mean + d * (nb / nn);
  m2 = m2 + qb + d * d * (n * nb / nn);
  n = nn;
}

// Per segment and column: Chan-merge the segment's partials, update the
// running stats (segments in order), write save_mean / save_invstd and the
// apply coefficients [seg][D].  Segments are reduced two at a time side by
// side: lanes [0, kSegLanes) of a column take segment s0, the others s0 + 1;
// a lane folds the partials p = lane (mod kSegLanes), four in flight, then
// each half is combined by a fixed-order tree (a one-segment call reduces
// its segment exactly as a pair does: every result bit-identical).
// grid = ceil(D/kRedCols), block = kRedCols * kRedLanes.
constexpr int kSegLanes = kRedLanes / 2;

__global__ __launch_bounds__(kRedCols* kRedLanes) void k_bn_stats_final(
    const float* __restrict__ pmean, const float* __restrict__ pm2, const float* __restrict__ pn,
    Segs sg, int64_t D, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ running_mean, float* __restrict__ running_var,
    float* __restrict__ save_mean, float* __restrict__ save_invstd, float* __restrict__ scale,
    float* __restrict__ shift, float momentum, float eps, int64_t* __restrict__ nbt) {
  __shared__ float rn[kRedLanes][kRedCols], rm[kRedLanes][kRedCols], rq[kRedLanes][kRedCols];
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += sg.n;  // num_batches_tracked
  const int cl = threadIdx.x % kRedCols, rl = threadIdx.x / kRedCols;
  const int half = rl / kSegLanes, sl = rl % kSegLanes;
  const int64_t c = (int64_t)blockIdx.x * kRedCols + cl;
  for (int s0 = 0; s0 < sg.n; s0 += 2) {
    const int s = s0 + half;
    float n = 0.f, mean = 0.f, m2 = 0.f;
    if (s < sg.n && c < D) {
      const SegAt at = seg_info(sg, s);
      const int64_t P = at.P;
      const float* sm = pmean + at.part0 * D;
      const float* sq = pm2 + at.part0 * D;
      const float* sn = pn + at.part0;
      // four partials per lane in flight, the ragged last round included (a
      // missing one merges as n = 0, which chan1 skips): one dependent round
      // trip for P <= 4 kSegLanes; merge order = increasing p, as before
      for (int64_t p = sl; p < P; p += 4 * kSegLanes) {
        float bn[4], bm[4], bq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t q = p + u * kSegLanes;
          const bool in = q < P;
          bn[u] = in ? sn[q] : 0.f;
          bm[u] = in ? sm[q * D + c] : 0.f;
          bq[u] = in ? sq[q * D + c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) chan1(n, mean, m2, bn[u], bm[u], bq[u]);
      }
    }
    __syncthreads();  // the previous pair's trees are done with the arrays
    rn[rl][cl] = n;
    rm[rl][cl] = mean;
    rq[rl][cl] = m2;
    __syncthreads();
#pragma unroll
    for (int stride = kSegLanes / 2; stride > 0; stride >>= 1) {
      if (sl < stride) {
        chan1(n, mean, m2, rn[rl + stride][cl], rm[rl + stride][cl], rq[rl + stride][cl]);
        rn[rl][cl] = n;
        rm[rl][cl] = mean;
        rq[rl][cl] = m2;
      }
      __syncthreads();
    }
    if (rl == 0 && c < D) {
      for (int h = 0; h < 2 && s0 + h < sg.n; ++h) {  // segment order
        const int ss = s0 + h;
        const float nn = rn[h * kSegLanes][cl], mu = rm[h * kSegLanes][cl];
        const float q2 = rq[h * kSegLanes][cl];
        const float var = q2 / nn;
        const float invstd = 1.0f / sqrtf(var + eps);
        save_mean[ss * D + c] = mu;
        save_invstd[ss * D + c] = invstd;
        if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
        if (running_var) {
          const float unbiased = nn > 1.f ? q2 / (nn - 1.f) : var;
          running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
        }
        float sc, sh;
        bn_coeffs(gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f, mu, invstd, sc, sh);
        scale[ss * D + c] = sc;
        shift[ss * D + c] = sh;
      }
    }
  }
}

// eval: running statistics, the same coefficients for every segment
__global__ void k_bn_eval_coeffs(const float* __restrict__ gamma, const float* __restrict__ beta,
                                 const float* __restrict__ running_mean,
                                 const float* __restrict__ running_var, int64_t D, int nseg,
                                 float eps, float* __restrict__ save_mean,
                                 float* __restrict__ save_invstd, float* __restrict__ scale,
                                 float* __restrict__ shift) {
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float mean = running_mean[c];
  float invstd = 1.0f / sqrtf(running_var[c] + eps);
  float sc, sh;
  bn_coeffs(gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f, mean, invstd, sc, sh);
  for (int s = 0; s < nseg; ++s) {
    if (save_mean) save_mean[s * D + c] = mean;
    if (save_invstd) save_invstd[s * D + c] = invstd;
    scale[s * D + c] = sc;
    shift[s * D + c] = sh;
  }
}

__device__ __forceinline__ float bn_apply1(float z, float sc, float sh) { return __fmaf_rn(z, sc, sh); }

// U = 2 (bf16 storage): two column units per thread, one 16-byte access each
// way (8-byte bf16 accesses ran at half the HBM rate of the fp32 form); the
// same per-element arithmetic.  d4 % U == 0 (host).
template <typename St, int U = 1>
__global__ __launch_bounds__(kT) void k_bn_apply(const typename St::T* __restrict__ z,
                                                 const float4* __restrict__ scale,
                                                 const float4* __restrict__ shift,
                                                 typename St::T* __restrict__ y, int64_t total4,
                                                 int d4, int relu, Segs sg) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total4 / U) return;
  const int64_t u0 = t * U;
  const int64_t i = row_of(u0, d4, total4);
  const int c = (int)(u0 - i * d4);
  const int s = seg_of_row(sg, i);
  float4 v[U];
  if (s < 0) {  // padding row of a device-sized plan
    if constexpr (U == 2) St::st2(y, t, f4zero(), f4zero());
    else St::st(y, t, f4zero());
    return;
  }
  if constexpr (U == 2) St::ld2(z, t, v[0], v[1]);
  else v[0] = St::ld(z, t);
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const float4 sc = scale[s * d4 + c + j], sh = shift[s * d4 + c + j];
    float4 o = make_float4(bn_apply1(v[j].x, sc.x, sh.x), bn_apply1(v[j].y, sc.y, sh.y),
                           bn_apply1(v[j].z, sc.z, sh.z), bn_apply1(v[j].w, sc.w, sh.w));
    if (relu) o = make_float4(fmaxf(o.x, 0.f), fmaxf(o.y, 0.f), fmaxf(o.z, 0.f), fmaxf(o.w, 0.f));
    v[j] = o;
  }
  if constexpr (U == 2) St::st2(y, t, v[0], v[1]);
  else St::st(y, t, v[0]);
}

// BN backward pass 1: per-column Σ dyr and Σ dyr * xhat (fixed order).
__device__ __forceinline__ void bn_coeffs4(const float* gamma, const float* beta, float4 mu,
                                           float4 is, int c, float4& sc, float4& sh) {
  float4 g = gamma ? reinterpret_cast<const float4*>(gamma)[c] : make_float4(1.f, 1.f, 1.f, 1.f);
  float4 b = beta ? reinterpret_cast<const float4*>(beta)[c] : f4zero();
  bn_coeffs(g.x, b.x, mu.x, is.x, sc.x, sh.x);
  bn_coeffs(g.y, b.y, mu.y, is.y, sc.y, sh.y);
  bn_coeffs(g.z, b.z, mu.z, is.z, sc.z, sh.z);
  bn_coeffs(g.w, b.w, mu.w, is.w, sc.w, sh.w);
}

template <typename St>
__global__ void k_bn_bwd_partial(const typename St::T* __restrict__ dy,
                                 const typename St::T* __restrict__ z,
                                 const float4* __restrict__ mean, const float4* __restrict__ invstd,
                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                 int d4, int band, Segs sg, int relu, float4* __restrict__ p1,
                                 float4* __restrict__ p2) {
  extern __shared__ __attribute__((aligned(16))) float4 red[];  // [2][band][d4]
  const int tid = threadIdx.x;
  const bool live = tid < band * d4;
  const int r = live ? tid / d4 : 0, c = live ? tid - r * d4 : 0;
  const SegAt at = seg_of_part(sg, blockIdx.x);
  if (at.s < 0) return;  // spare partition of a device-sized plan (block-uniform)
  const int s = at.s;
  const int64_t beg = at.row0 + (blockIdx.x - at.part0) * at.rpp;
  int64_t end = beg + at.rpp;
  if (end > at.row1) end = at.row1;
  float4 s1 = f4zero(), s2 = f4zero();
  if (live) {
    float4 mu = mean[s * d4 + c], is = invstd[s * d4 + c], sc, sh;
    bn_coeffs4(gamma, beta, mu, is, c, sc, sh);
    // eight rows' loads in flight per round trip (few waves per CU here);
    // the sums stay in row order
    constexpr int U = 8;
    for (int64_t i0 = beg + r; i0 < end; i0 += U * (int64_t)band) {
      float4 gv[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * band;
        const int64_t ii = i < end ? i : i0;
        gv[u] = St::ld(dy, ii * d4 + c);
        xv[u] = St::ld(z, ii * d4 + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + (int64_t)u * band >= end) break;
        float4 g = gv[u];
        const float4 x = xv[u];
        if (relu) {
          g.x = bn_apply1(x.x, sc.x, sh.x) > 0.f ? g.x : 0.f;
          g.y = bn_apply1(x.y, sc.y, sh.y) > 0.f ? g.y : 0.f;
          g.z = bn_apply1(x.z, sc.z, sh.z) > 0.f ? g.z : 0.f;
          g.w = bn_apply1(x.w, sc.w, sh.w) > 0.f ? g.w : 0.f;
        }
        s1 = f4add(s1, g);
        s2.x += g.x * ((x.x - mu.x) * is.x);
        s2.y += g.y * ((x.y - mu.y) * is.y);
        s2.z += g.z * ((x.z - mu.z) * is.z);
        s2.w += g.w * ((x.w - mu.w) * is.w);
      }
    }
    red[r * d4 + c] = s1;
    red[(band + r) * d4 + c] = s2;
  }
  __syncthreads();
  if (live && r == 0) {
    float4 a = red[c], b = red[band * d4 + c];
    for (int q = 1; q < band; ++q) {
      a = f4add(a, red[q * d4 + c]);
      b = f4add(b, red[(band + q) * d4 + c]);
    }
    p1[(int64_t)blockIdx.x * d4 + c] = a;
    p2[(int64_t)blockIdx.x * d4 + c] = b;
  }
}

// dgamma / dbeta: Σ over segments in segment order (added to the existing
// value when accumulate); k1 / k2 [seg][D] per segment.  Segment pairs side
// by side as in k_bn_stats_final.
__global__ __launch_bounds__(kRedCols* kRedLanes) void k_bn_bwd_final(
    const float* __restrict__ p1, const float* __restrict__ p2, Segs sg, int64_t D,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ k1,
    float* __restrict__ k2, int accumulate) {
  __shared__ float ra[kRedLanes][kRedCols], rb[kRedLanes][kRedCols];
  const int cl = threadIdx.x % kRedCols, rl = threadIdx.x / kRedCols;
  const int half = rl / kSegLanes, sl = rl % kSegLanes;
  const int64_t c = (int64_t)blockIdx.x * kRedCols + cl;
  for (int s0 = 0; s0 < sg.n; s0 += 2) {
    const int s = s0 + half;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
    if (s < sg.n && c < D) {
      const SegAt at = seg_info(sg, s);
      const int64_t P = at.P;
      const float* q1 = p1 + at.part0 * D;
      const float* q2 = p2 + at.part0 * D;
      // four partials per lane in flight, the ragged last round included
      for (int64_t p = sl; p < P; p += 4 * kSegLanes) {
        float x1[4], x2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t q = p + u * kSegLanes;
          x1[u] = q < P ? q1[q * D + c] : 0.f;
          x2[u] = q < P ? q2[q * D + c] : 0.f;
        }
        a0 += x1[0];
        a1 += x1[1];
        a2 += x1[2];
        a3 += x1[3];
        b0 += x2[0];
        b1 += x2[1];
        b2 += x2[2];
        b3 += x2[3];
      }
    }
    float a = (a0 + a1) + (a2 + a3), b = (b0 + b1) + (b2 + b3);
    __syncthreads();  // the previous pair's trees are done with the arrays
    ra[rl][cl] = a;
    rb[rl][cl] = b;
    __syncthreads();
#pragma unroll
    for (int stride = kSegLanes / 2; stride > 0; stride >>= 1) {
      if (sl < stride) {
        ra[rl][cl] = a = a + ra[rl + stride][cl];
        rb[rl][cl] = b = b + rb[rl + stride][cl];
      }
      __syncthreads();
    }
    if (rl == 0 && c < D) {
      for (int h = 0; h < 2 && s0 + h < sg.n; ++h) {  // segment order
        const int ss = s0 + h;
        const float sa = ra[h * kSegLanes][cl], sb = rb[h * kSegLanes][cl];
        const float inv_rows = 1.0f / (float)seg_n(sg, ss);
        const bool add = accumulate || ss > 0;
        if (dbeta) dbeta[c] = add ? dbeta[c] + sa : sa;
        if (dgamma) dgamma[c] = add ? dgamma[c] + sb : sb;
        k1[ss * D + c] = sa * inv_rows;
        k2[ss * D + c] = sb * inv_rows;
      }
    }
  }
}

// one float4 of dz from its dy / z units (segment s, column unit c)
__device__ __forceinline__ float4 bn_bwd_math(float4 g, float4 x, const float4* __restrict__ mean,
                                              const float4* __restrict__ invstd,
                                              const float* __restrict__ gamma,
                                              const float* __restrict__ beta,
                                              const float4* __restrict__ k1,
                                              const float4* __restrict__ k2, int s, int c, int d4,
                                              int relu) {
  float4 mu = mean[s * d4 + c], is = invstd[s * d4 + c], sc, sh;
  bn_coeffs4(gamma, beta, mu, is, c, sc, sh);
  float4 a = k1[s * d4 + c], b = k2[s * d4 + c];
  if (relu) {
    g.x = bn_apply1(x.x, sc.x, sh.x) > 0.f ? g.x : 0.f;
    g.y = bn_apply1(x.y, sc.y, sh.y) > 0.f ? g.y : 0.f;
    g.z = bn_apply1(x.z, sc.z, sh.z) > 0.f ? g.z : 0.f;
    g.w = bn_apply1(x.w, sc.w, sh.w) > 0.f ? g.w : 0.f;
  }
  // dz = gamma*invstd * (g - mean(g) - xhat * mean(g*xhat))  (torch CPU BN backward)
  float4 o;
  o.x = (g.x - a.x - ((x.x - mu.x) * is.x) * b.x) * sc.x;
  o.y = (g.y - a.y - ((x.y - mu.y) * is.y) * b.y) * sc.y;
  o.z = (g.z - a.z - ((x.z - mu.z) * is.z) * b.z) * sc.z;
  o.w = (g.w - a.w - ((x.w - mu.w) * is.w) * b.w) * sc.w;
  return o;
}

// one float4 of dz (k_bn_bwd_apply), stored and returned
template <typename St>
__device__ __forceinline__ float4 bn_bwd_elem(
    const typename St::T* __restrict__ dy, const typename St::T* __restrict__ z,
    const float4* __restrict__ mean, const float4* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float4* __restrict__ k1,
    const float4* __restrict__ k2, typename St::T* __restrict__ dz, int64_t t, int d4, int relu,
    Segs sg, int64_t total4) {
  const int64_t i = row_of(t, d4, total4);
  const int c = (int)(t - i * d4);
  const int s = seg_of_row(sg, i);
  if (s < 0) {  // padding row of a device-sized plan: no gradient
    St::st(dz, t, f4zero());
    return f4zero();
  }
  const float4 o = bn_bwd_math(St::ld(dy, t), St::ld(z, t), mean, invstd, gamma, beta, k1, k2, s,
                               c, d4, relu);
  St::st(dz, t, o);
  return o;
}

// two column units per thread, 16-byte accesses (bf16 storage, no row maxima)
template <typename St>
__global__ __launch_bounds__(kT) void k_bn_bwd_apply2(
    const typename St::T* __restrict__ dy, const typename St::T* __restrict__ z,
    const float4* __restrict__ mean, const float4* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float4* __restrict__ k1,
    const float4* __restrict__ k2, typename St::T* __restrict__ dz, int64_t total4, int d4,
    int relu, Segs sg) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total4 / 2) return;
  const int64_t u0 = 2 * t;
  const int64_t i = row_of(u0, d4, total4);
  const int c = (int)(u0 - i * d4);
  const int s = seg_of_row(sg, i);
  if (s < 0) {
    St::st2(dz, t, f4zero(), f4zero());
    return;
  }
  float4 g0, g1, x0, x1;
  St::ld2(dy, t, g0, g1);
  St::ld2(z, t, x0, x1);
  St::st2(dz, t, bn_bwd_math(g0, x0, mean, invstd, gamma, beta, k1, k2, s, c, d4, relu),
          bn_bwd_math(g1, x1, mean, invstd, gamma, beta, k1, k2, s, c + 1, d4, relu));
}

template <typename St>
__global__ __launch_bounds__(kT) void k_bn_bwd_apply(
    const typename St::T* __restrict__ dy, const typename St::T* __restrict__ z,
    const float4* __restrict__ mean, const float4* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float4* __restrict__ k1,
    const float4* __restrict__ k2, typename St::T* __restrict__ dz, int64_t total4, int d4,
    int relu, Segs sg, float* __restrict__ rowparts, int nparts, float* __restrict__ slot) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (rowparts != nullptr) {  // block-uniform: every thread reaches the reductions
    // dz's row maxima as row parts (row_max_parts) and its max
    const int64_t rows = total4 / d4;
    float m = 0.f;
    int row = -1;
    if (t < total4) {
      const float4 o = bn_bwd_elem<St>(dy, z, mean, invstd, gamma, beta, k1, k2, dz, t, d4, relu,
                                       sg, total4);
      m = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w)));
      row = (int)row_of(t, d4, total4);
    }
    row_max_parts(m, row, t, rows, d4, rowparts, nparts);
    if (slot != nullptr) absmax_publish(m, slot);
    return;
  }
  if (t >= total4) return;
  bn_bwd_elem<St>(dy, z, mean, invstd, gamma, beta, k1, k2, dz, t, d4, relu, sg, total4);
}


// ---------------------------------------------------------------------------
// segment pooling over graph_ptr
// ---------------------------------------------------------------------------
template <typename St = StF32>
__global__ void k_pool_fwd(const typename St::T* __restrict__ h, const int32_t* __restrict__ ptr,
                           float4* __restrict__ out, int64_t G, int d4, int mode) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= G * d4) return;
  int64_t g = t / d4;
  int c = (int)(t - g * d4);
  int32_t beg = ptr[g], end = ptr[g + 1];
  float4 acc = f4zero();
  // eight rows' loads in flight (a graph's ~30 rows were a serial load chain);
  // the adds stay in row order
  int32_t i = beg;
  for (; i + 8 <= end; i += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = St::ld(h, (int64_t)(i + u) * d4 + c);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = f4add(acc, v[u]);
  }
  for (; i < end; ++i) acc = f4add(acc, St::ld(h, (int64_t)i * d4 + c));
  if (mode == 0) {
    float cnt = (float)(end - beg > 1 ? end - beg : 1);
    acc = make_float4(acc.x / cnt, acc.y / cnt, acc.z / cnt, acc.w / cnt);
  }
  out[t] = acc;
}

// Rows outside every segment ([0, ptr[0]) and [ptr[G], N): the padding rows
// of a captured step's capacity) get zero gradient from the same grid, no
// separate memset of all N rows.
template <typename St = StF32>
__global__ void k_pool_bwd(const float4* __restrict__ dout, const int32_t* __restrict__ ptr,
                           typename St::T* __restrict__ dh, int64_t G, int d4, int mode, int64_t N) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t lo = (int64_t)ptr[0] * d4, hi0 = (int64_t)ptr[G] * d4, n4 = N * d4;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t q = t; q < lo; q += stride) St::st(dh, q, z);
    for (int64_t q = hi0 + t; q < n4; q += stride) St::st(dh, q, z);
  }
  if (t >= G * d4) return;
  int64_t g = t / d4;
  int c = (int)(t - g * d4);
  int32_t beg = ptr[g], end = ptr[g + 1];
  float4 v = dout[t];
  if (mode == 0) {
    float cnt = (float)(end - beg > 1 ? end - beg : 1);
    v = make_float4(v.x / cnt, v.y / cnt, v.z / cnt, v.w / cnt);
  }
  for (int32_t i = beg; i < end; ++i) St::st(dh, (int64_t)i * d4 + c, v);
}

// global_max_pool (PyG 1.6.3 -> torch_scatter 2.0.6 scatter_max): per graph
// and column the largest value and the node holding it (the first in node
// order among equal values, as torch_scatter's CPU loop keeps it: strict >);
// a graph without nodes pools to 0 with no arg (-1).  The backward routes
// dout to that node only.
template <typename St = StF32>
__global__ void k_pool_max_fwd(const typename St::T* __restrict__ h, const int32_t* __restrict__ ptr,
                               float4* __restrict__ out, int4* __restrict__ arg, int64_t G, int d4) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= G * d4) return;
  int64_t g = t / d4;
  int c = (int)(t - g * d4);
  int32_t beg = ptr[g], end = ptr[g + 1];
  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int a[4] = {-1, -1, -1, -1};
  for (int32_t i = beg; i < end; ++i) {
    const float4 v = St::ld(h, (int64_t)i * d4 + c);
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (a[j] < 0 || e[j] > m[j]) {
        m[j] = e[j];
        a[j] = i;
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (a[j] < 0) m[j] = 0.f;
  out[t] = make_float4(m[0], m[1], m[2], m[3]);
  arg[t] = make_int4(a[0], a[1], a[2], a[3]);
}

template <typename St = StF32>
__global__ void k_pool_max_bwd(const float4* __restrict__ dout, const int4* __restrict__ arg,
                               typename St::T* __restrict__ dh, int64_t G, int d4) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= G * d4) return;
  const int c = (int)(t % d4);
  const float4 v = dout[t];
  const int4 a = arg[t];
  const float e[4] = {v.x, v.y, v.z, v.w};
  const int ai[4] = {a.x, a.y, a.z, a.w};
  // the other elements of each row stay zero (memset); a node is the arg of
  // at most one graph, so no two threads write one element
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (ai[j] >= 0) St::st1(dh, (int64_t)ai[j] * (4 * d4) + 4 * c + j, e[j]);
}

// ---------------------------------------------------------------------------
// F.normalize (one wave per row)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_l2norm_fwd(const float* __restrict__ z,
                                                    float* __restrict__ y,
                                                    float* __restrict__ norm, int64_t rows,
                                                    int64_t D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= rows) return;
  const float* zr = z + r * D;
  float ss = 0.f;
  for (int64_t c = lane; c < D; c += 64) ss += zr[c] * zr[c];
  ss = wave_sum(ss);
  float nrm = sqrtf(ss);
  float den = fmaxf(nrm, eps);
  if (lane == 0) norm[r] = nrm;
  for (int64_t c = lane; c < D; c += 64) y[r * D + c] = zr[c] / den;
}

__global__ __launch_bounds__(256) void k_l2norm_bwd(const float* __restrict__ dy,
                                                    const float* __restrict__ y,
                                                    const float* __restrict__ norm,
                                                    float* __restrict__ dz, int64_t rows,
                                                    int64_t D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= rows) return;
  float nrm = norm[r];
  if (nrm > eps) {
    float dot = 0.f;
    for (int64_t c = lane; c < D; c += 64) dot += dy[r * D + c] * y[r * D + c];
    dot = wave_sum(dot);
    for (int64_t c = lane; c < D; c += 64)
      dz[r * D + c] = (dy[r * D + c] - dot * y[r * D + c]) / nrm;
  } else {
    for (int64_t c = lane; c < D; c += 64) dz[r * D + c] = dy[r * D + c] / eps;
  }
}

__global__ __launch_bounds__(1024) void k_sum(const float* __restrict__ x, float* __restrict__ out,
                                              int64_t n) {
  __shared__ float ws[16];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) acc += x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += ws[w];
    *out = s;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// shared with aggregate.hip
// ---------------------------------------------------------------------------
size_t molclr_colsum_ws(int64_t rows, int64_t cols) {
  molclr::Band b = molclr::make_band(cols);
  return (size_t)band_parts(rows, b.band) * cols * sizeof(float) + 256;
}

int molclr_colsum_impl(const float* X, float* out, int64_t rows, int64_t cols, int64_t ld,
                       int accumulate, molclr::Workspace& w, hipStream_t s) {
  MOLCLR_REQUIRE(cols > 0 && cols % 4 == 0 && ld % 4 == 0, "colsum: cols/ld must be multiples of 4");
  molclr::Band b = molclr::make_band(cols);
  int64_t P = band_parts(rows, b.band);
  float* partial = w.take<float>(P * cols);
  if (!w.ok()) {
    molclr::set_error("colsum: workspace too small");
    return MOLCLR_ERR_WORKSPACE;
  }
  int64_t rpp = molclr::ceil_div(rows > 0 ? rows : 1, P);
  size_t lds = (size_t)b.band * b.d4 * sizeof(float4);
  hipLaunchKernelGGL(k_colsum_partial, dim3(P), dim3(b.threads), lds, s, (const float4*)X, rows,
                     b.d4, ld / 4, b.band, rpp, (float4*)partial);
  hipLaunchKernelGGL(k_colsum_final, dim3(molclr::ceil_div(cols, kRedCols)), dim3(kRedCols * kRedLanes), 0, s, partial, P,
                     cols, out, accumulate);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API size_t molclr_colsum_f32_workspace_bytes(int64_t rows, int64_t cols) {
  return molclr_colsum_ws(rows, cols);
}

MOLCLR_API int molclr_colsum_f32(const float* X, float* out, int64_t rows, int64_t cols,
                                 int64_t ld, int accumulate, void* workspace,
                                 size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_colsum_ws(rows, cols));
  molclr::Workspace w(workspace, workspace_bytes);
  return molclr_colsum_impl(X, out, rows, cols, ld, accumulate, w, molclr::as_stream(stream));
}

namespace {

// host-side segment plan: partitions of every segment exactly as a one-segment
// call over its rows would have them.  Device-sized (drows != NULL): the
// segments' rows are read on the device, `cap` rows in all; P covers any
// split of cap rows into nseg segments (spare partitions exit at once).
int make_segs(int nseg, const int64_t* seg_rows, const int64_t* drows, int64_t cap, int64_t D,
              Segs& sg, int64_t& P, int64_t& rows) {
  MOLCLR_REQUIRE(nseg >= 1 && nseg <= MOLCLR_MAX_SEGMENTS && (seg_rows || drows),
                 "batchnorm: %d segments (1..%d)", nseg, MOLCLR_MAX_SEGMENTS);
  const molclr::Band b = molclr::make_band(D);
  sg.n = nseg;
  sg.band = b.band;
  sg.drows = drows;
  P = 0;
  rows = 0;
  for (int s = 0; s < MOLCLR_MAX_SEGMENTS; ++s) sg.rows[s] = 0;
  if (drows) {
    MOLCLR_REQUIRE(cap >= 0, "batchnorm: negative row capacity");
    P = band_parts_bound(cap, b.band, nseg);
    rows = cap;
    return MOLCLR_OK;
  }
  for (int s = 0; s < nseg; ++s) {
    MOLCLR_REQUIRE(seg_rows[s] >= 0, "batchnorm: negative segment rows");
    sg.rows[s] = seg_rows[s];
    P += band_parts(seg_rows[s], b.band);
    rows += seg_rows[s];
  }
  return MOLCLR_OK;
}

size_t bn_ws_bytes(int64_t P, int64_t D, int nseg) {
  molclr::Workspace w(nullptr, 0);
  w.take<float>(P * D);     // partial mean / s1
  w.take<float>(P * D);     // partial m2 / s2
  w.take<float>(P);         // partial n
  w.take<float>(nseg * D);  // scale
  w.take<float>(nseg * D);  // shift
  w.take<float>(nseg * D);  // k1
  w.take<float>(nseg * D);  // k2
  return w.used + 256;
}

template <typename St>
int bn_fwd(const void* zv, const float* gamma, const float* beta, float* running_mean,
           float* running_var, int64_t* nbt, void* yv, float* save_mean, float* save_invstd,
           int nseg, const int64_t* seg_rows, int64_t D, double momentum, double eps, int training,
           int relu, void* workspace, size_t workspace_bytes, hipStream_t s,
           const int64_t* drows = nullptr, int64_t cap = 0) {
  Segs sg;
  int64_t P = 0, rows = 0;
  if (int rc = make_segs(nseg, seg_rows, drows, cap, D, sg, P, rows)) return rc;
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "batchnorm_fwd: dim must be a multiple of 4");
  for (int q = 0; q < nseg && !drows; ++q)  // device-sized: the caller's contract
    MOLCLR_REQUIRE(!training || seg_rows[q] > 1,
                   "batchnorm_fwd: need more than 1 row per segment when training");
  MOLCLR_REQUIRE(training || (running_mean && running_var), "batchnorm_fwd: eval needs running stats");
  MOLCLR_REQUIRE(save_mean && save_invstd && (rows == 0 || zv), "batchnorm_fwd: null pointer");
  MOLCLR_REQUIRE_WS(workspace_bytes, bn_ws_bytes(P, D, nseg));
  const auto* z = static_cast<const typename St::T*>(zv);
  auto* y = static_cast<typename St::T*>(yv);
  const molclr::Band b = molclr::make_band(D);
  molclr::Workspace w(workspace, workspace_bytes);
  float* pmean = w.take<float>(P * D);
  float* pm2 = w.take<float>(P * D);
  float* pn = w.take<float>(P);
  float* scale = w.take<float>(nseg * D);
  float* shift = w.take<float>(nseg * D);
  if (training) {
    const size_t lds = 2 * (size_t)b.band * b.d4 * sizeof(float4);
    hipLaunchKernelGGL(k_bn_stats_partial<St>, dim3((unsigned)P), dim3(b.threads), lds, s, z, b.d4,
                       b.band, sg, (float4*)pmean, (float4*)pm2, pn);
    hipLaunchKernelGGL(k_bn_stats_final, dim3(molclr::ceil_div(D, kRedCols)),
                       dim3(kRedCols * kRedLanes), 0, s, pmean, pm2, pn, sg, D, gamma, beta,
                       running_mean, running_var, save_mean, save_invstd, scale, shift,
                       (float)momentum, (float)eps, nbt);
  } else {
    hipLaunchKernelGGL(k_bn_eval_coeffs, dim3(molclr::ceil_div(D, kT)), dim3(kT), 0, s, gamma,
                       beta, running_mean, running_var, D, nseg, (float)eps, save_mean,
                       save_invstd, scale, shift);
  }
  const int64_t total4 = rows * (D / 4);
  if (total4 > 0 && y) {  // y == NULL: statistics only (the consumer applies them)
    if (St::kBytes == 2 && D % 8 == 0)
      hipLaunchKernelGGL((k_bn_apply<St, 2>), dim3(molclr::ceil_div(total4 / 2, kT)), dim3(kT), 0,
                         s, z, (const float4*)scale, (const float4*)shift, y, total4, (int)(D / 4),
                         relu, sg);
    else
      hipLaunchKernelGGL((k_bn_apply<St, 1>), dim3(molclr::ceil_div(total4, kT)), dim3(kT), 0, s,
                         z, (const float4*)scale, (const float4*)shift, y, total4, (int)(D / 4),
                         relu, sg);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

// waves a row of D / 4 float4s can touch (k_bn_bwd_apply's row parts)
int bn_row_parts(int64_t D) { return (int)((D / 4 + 62) / 64) + 1; }

template <typename St>
int bn_bwd(const void* dyv, const void* zv, const float* gamma, const float* beta,
           const float* save_mean, const float* save_invstd, void* dzv, float* dgamma,
           float* dbeta, int nseg, const int64_t* seg_rows, int64_t D, int relu, int accumulate,
           void* workspace, size_t workspace_bytes, hipStream_t s, float* rowparts = nullptr,
           float* slot = nullptr, const int64_t* drows = nullptr, int64_t cap = 0) {
  Segs sg;
  int64_t P = 0, rows = 0;
  if (int rc = make_segs(nseg, seg_rows, drows, cap, D, sg, P, rows)) return rc;
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "batchnorm_bwd: dim must be a multiple of 4");
  MOLCLR_REQUIRE(rows > 0 && dyv && zv && save_mean && save_invstd && dzv, "batchnorm_bwd: bad args");
  for (int q = 0; q < nseg && !drows; ++q)
    MOLCLR_REQUIRE(seg_rows[q] > 0, "batchnorm_bwd: empty segment");
  MOLCLR_REQUIRE_WS(workspace_bytes, bn_ws_bytes(P, D, nseg));
  const auto* dy = static_cast<const typename St::T*>(dyv);
  const auto* z = static_cast<const typename St::T*>(zv);
  auto* dz = static_cast<typename St::T*>(dzv);
  const molclr::Band b = molclr::make_band(D);
  molclr::Workspace w(workspace, workspace_bytes);
  float* p1 = w.take<float>(P * D);
  float* p2 = w.take<float>(P * D);
  w.take<float>(P);
  w.take<float>(nseg * D);  // scale
  w.take<float>(nseg * D);  // shift
  float* k1 = w.take<float>(nseg * D);
  float* k2 = w.take<float>(nseg * D);
  // the forward's coefficient expression is recomputed in-kernel (same ReLU mask)
  const size_t lds = 2 * (size_t)b.band * b.d4 * sizeof(float4);
  hipLaunchKernelGGL(k_bn_bwd_partial<St>, dim3((unsigned)P), dim3(b.threads), lds, s, dy, z,
                     (const float4*)save_mean, (const float4*)save_invstd, gamma, beta, b.d4,
                     b.band, sg, relu, (float4*)p1, (float4*)p2);
  hipLaunchKernelGGL(k_bn_bwd_final, dim3(molclr::ceil_div(D, kRedCols)), dim3(kRedCols * kRedLanes),
                     0, s, p1, p2, sg, D, dgamma, dbeta, k1, k2, accumulate);
  const int64_t total4 = rows * (D / 4);
  static_assert(kT % 64 == 0, "row parts follow the waves");
  MOLCLR_REQUIRE(!rowparts || rows < (1ll << 31), "batchnorm_seg_bwd_max: too many rows");
  if (St::kBytes == 2 && D % 8 == 0 && !rowparts && !slot)
    hipLaunchKernelGGL(k_bn_bwd_apply2<St>, dim3(molclr::ceil_div(total4 / 2, kT)), dim3(kT), 0, s,
                       dy, z, (const float4*)save_mean, (const float4*)save_invstd, gamma, beta,
                       (const float4*)k1, (const float4*)k2, dz, total4, (int)(D / 4), relu, sg);
  else
    hipLaunchKernelGGL(k_bn_bwd_apply<St>, dim3(molclr::ceil_div(total4, kT)), dim3(kT), 0, s, dy,
                       z, (const float4*)save_mean, (const float4*)save_invstd, gamma, beta,
                       (const float4*)k1, (const float4*)k2, dz, total4, (int)(D / 4), relu, sg,
                       rowparts, bn_row_parts(D), slot);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

}  // namespace

// Workspace that covers any split of `rows` rows into <= MOLCLR_MAX_SEGMENTS
// segments (the encoder executors size their scratch before knowing it).
size_t molclr_batchnorm_ws_bound(int64_t rows, int64_t D) {
  const molclr::Band b = molclr::make_band(D > 0 ? D : 4);
  return bn_ws_bytes(band_parts_bound(rows, b.band, MOLCLR_MAX_SEGMENTS), D, MOLCLR_MAX_SEGMENTS);
}

MOLCLR_API size_t molclr_batchnorm_seg_workspace_bytes(int nseg, const int64_t* seg_rows,
                                                       int64_t D) {
  Segs sg;
  int64_t P = 0, rows = 0;
  if (make_segs(nseg, seg_rows, nullptr, 0, D > 0 ? D : 4, sg, P, rows)) return 0;
  return bn_ws_bytes(P, D, nseg);
}

MOLCLR_API size_t molclr_batchnorm_workspace_bytes(int64_t rows, int64_t D) {
  return molclr_batchnorm_seg_workspace_bytes(1, &rows, D);
}

MOLCLR_API int molclr_batchnorm_seg_fwd(const void* z, const float* gamma, const float* beta,
                                        float* running_mean, float* running_var,
                                        int64_t* num_batches_tracked, void* y, float* save_mean,
                                        float* save_invstd, int nseg, const int64_t* seg_rows,
                                        int64_t D, int dtype, double momentum, double eps,
                                        int training, int relu, void* workspace,
                                        size_t workspace_bytes, molclr_stream_t stream) {
  hipStream_t s = molclr::as_stream(stream);
  if (dtype == MOLCLR_DTYPE_F32)
    return bn_fwd<StF32>(z, gamma, beta, running_mean, running_var, num_batches_tracked, y,
                         save_mean, save_invstd, nseg, seg_rows, D, momentum, eps, training, relu,
                         workspace, workspace_bytes, s);
  MOLCLR_REQUIRE(dtype == MOLCLR_DTYPE_BF16, "batchnorm_seg_fwd: dtype %d", dtype);
  return bn_fwd<StBF16>(z, gamma, beta, running_mean, running_var, num_batches_tracked, y,
                        save_mean, save_invstd, nseg, seg_rows, D, momentum, eps, training, relu,
                        workspace, workspace_bytes, s);
}

MOLCLR_API int molclr_batchnorm_seg_bwd(const void* dy, const void* z, const float* gamma,
                                        const float* beta, const float* save_mean,
                                        const float* save_invstd, void* dz, float* dgamma,
                                        float* dbeta, int nseg, const int64_t* seg_rows, int64_t D,
                                        int dtype, int relu, int accumulate, void* workspace,
                                        size_t workspace_bytes, molclr_stream_t stream) {
  hipStream_t s = molclr::as_stream(stream);
  if (dtype == MOLCLR_DTYPE_F32)
    return bn_bwd<StF32>(dy, z, gamma, beta, save_mean, save_invstd, dz, dgamma, dbeta, nseg,
                         seg_rows, D, relu, accumulate, workspace, workspace_bytes, s);
  MOLCLR_REQUIRE(dtype == MOLCLR_DTYPE_BF16, "batchnorm_seg_bwd: dtype %d", dtype);
  return bn_bwd<StBF16>(dy, z, gamma, beta, save_mean, save_invstd, dz, dgamma, dbeta, nseg,
                        seg_rows, D, relu, accumulate, workspace, workspace_bytes, s);
}

MOLCLR_API int molclr_bn_row_parts(int64_t dim) { return bn_row_parts(dim); }

MOLCLR_API int molclr_batchnorm_seg_bwd_max(const float* dy, const float* z, const float* gamma,
                                            const float* beta, const float* save_mean,
                                            const float* save_invstd, float* dz, float* dgamma,
                                            float* dbeta, int nseg, const int64_t* seg_rows,
                                            int64_t D, int relu, int accumulate, float* rowmax,
                                            float* slot, void* workspace, size_t workspace_bytes,
                                            molclr_stream_t stream) {
  MOLCLR_REQUIRE(rowmax, "batchnorm_seg_bwd_max: null rowmax");
  return bn_bwd<StF32>(dy, z, gamma, beta, save_mean, save_invstd, dz, dgamma, dbeta, nseg,
                       seg_rows, D, relu, accumulate, workspace, workspace_bytes,
                       molclr::as_stream(stream), rowmax, slot);
}

// Device-sized segments (a captured training step over padded buffers):
// seg_rows_dev [nseg] on the device, rows_cap rows in z / y / dy / dz; rows
// past the segments' sum are padding (zero output and gradient).  Same plan
// per segment as the host-sized calls, so the results are bit-identical to
// them on the real rows.  Workspace: molclr_batchnorm_seg_dev_workspace_bytes.
MOLCLR_API size_t molclr_batchnorm_seg_dev_workspace_bytes(int nseg, int64_t rows_cap, int64_t D) {
  if (nseg < 1 || nseg > MOLCLR_MAX_SEGMENTS) return 0;
  const molclr::Band b = molclr::make_band(D > 0 ? D : 4);
  return bn_ws_bytes(band_parts_bound(rows_cap, b.band, nseg), D, nseg);
}

MOLCLR_API int molclr_batchnorm_seg_fwd_dev(const void* z, const float* gamma, const float* beta,
                                            float* running_mean, float* running_var,
                                            int64_t* num_batches_tracked, void* y, float* save_mean,
                                            float* save_invstd, int nseg,
                                            const int64_t* seg_rows_dev, int64_t rows_cap,
                                            int64_t D, int dtype, double momentum, double eps,
                                            int training, int relu, void* workspace,
                                            size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_REQUIRE(seg_rows_dev, "batchnorm_seg_fwd_dev: null seg_rows_dev");
  hipStream_t s = molclr::as_stream(stream);
  if (dtype == MOLCLR_DTYPE_F32)
    return bn_fwd<StF32>(z, gamma, beta, running_mean, running_var, num_batches_tracked, y,
                         save_mean, save_invstd, nseg, nullptr, D, momentum, eps, training, relu,
                         workspace, workspace_bytes, s, seg_rows_dev, rows_cap);
  MOLCLR_REQUIRE(dtype == MOLCLR_DTYPE_BF16, "batchnorm_seg_fwd_dev: dtype %d", dtype);
  return bn_fwd<StBF16>(z, gamma, beta, running_mean, running_var, num_batches_tracked, y,
                        save_mean, save_invstd, nseg, nullptr, D, momentum, eps, training, relu,
                        workspace, workspace_bytes, s, seg_rows_dev, rows_cap);
}

MOLCLR_API int molclr_batchnorm_seg_bwd_dev(const void* dy, const void* z, const float* gamma,
                                            const float* beta, const float* save_mean,
                                            const float* save_invstd, void* dz, float* dgamma,
                                            float* dbeta, int nseg, const int64_t* seg_rows_dev,
                                            int64_t rows_cap, int64_t D, int dtype, int relu,
                                            int accumulate, float* rowmax, float* slot,
                                            void* workspace, size_t workspace_bytes,
                                            molclr_stream_t stream) {
  MOLCLR_REQUIRE(seg_rows_dev, "batchnorm_seg_bwd_dev: null seg_rows_dev");
  MOLCLR_REQUIRE(!rowmax || dtype == MOLCLR_DTYPE_F32, "batchnorm_seg_bwd_dev: row maxima are fp32 only");
  hipStream_t s = molclr::as_stream(stream);
  if (dtype == MOLCLR_DTYPE_F32)
    return bn_bwd<StF32>(dy, z, gamma, beta, save_mean, save_invstd, dz, dgamma, dbeta, nseg,
                         nullptr, D, relu, accumulate, workspace, workspace_bytes, s, rowmax, slot,
                         seg_rows_dev, rows_cap);
  MOLCLR_REQUIRE(dtype == MOLCLR_DTYPE_BF16, "batchnorm_seg_bwd_dev: dtype %d", dtype);
  return bn_bwd<StBF16>(dy, z, gamma, beta, save_mean, save_invstd, dz, dgamma, dbeta, nseg,
                        nullptr, D, relu, accumulate, workspace, workspace_bytes, s, nullptr,
                        nullptr, seg_rows_dev, rows_cap);
}

MOLCLR_API int molclr_batchnorm_fwd(const float* z, const float* gamma, const float* beta,
                                    float* running_mean, float* running_var,
                                    int64_t* num_batches_tracked, float* y,
                                    float* save_mean, float* save_invstd, int64_t rows,
                                    int64_t D, double momentum, double eps, int training,
                                    int relu, void* workspace, size_t workspace_bytes,
                                    molclr_stream_t stream) {
  return molclr_batchnorm_seg_fwd(z, gamma, beta, running_mean, running_var, num_batches_tracked,
                                  y, save_mean, save_invstd, 1, &rows, D, MOLCLR_DTYPE_F32,
                                  momentum, eps, training, relu, workspace, workspace_bytes, stream);
}

MOLCLR_API int molclr_batchnorm_bwd(const float* dy, const float* z, const float* gamma,
                                    const float* beta, const float* save_mean,
                                    const float* save_invstd, float* dz, float* dgamma,
                                    float* dbeta, int64_t rows, int64_t D, int relu,
                                    int accumulate, void* workspace, size_t workspace_bytes,
                                    molclr_stream_t stream) {
  return molclr_batchnorm_seg_bwd(dy, z, gamma, beta, save_mean, save_invstd, dz, dgamma, dbeta,
                                  1, &rows, D, MOLCLR_DTYPE_F32, relu, accumulate, workspace,
                                  workspace_bytes, stream);
}

MOLCLR_API int molclr_segment_pool_fwd(const float* h, const int32_t* graph_ptr, float* out,
                                       int64_t G, int64_t D, int mode, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "segment_pool_fwd: dim must be a multiple of 4");
  if (mode != 0 && mode != 1) {
    molclr::set_error("segment_pool_fwd: mode %d unsupported (0 mean, 1 add)", mode);
    return MOLCLR_ERR_UNSUPPORTED;
  }
  if (G == 0) return MOLCLR_OK;
  int d4 = (int)(D / 4);
  hipLaunchKernelGGL(k_pool_fwd<StF32>, dim3(molclr::ceil_div(G * d4, kT)), dim3(kT), 0,
                     molclr::as_stream(stream), h, graph_ptr, (float4*)out, G, d4, mode);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_segment_pool_bwd(const float* dout, const int32_t* graph_ptr, float* dh,
                                       int64_t N, int64_t G, int64_t D, int mode,
                                       molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "segment_pool_bwd: dim must be a multiple of 4");
  if (mode != 0 && mode != 1) {
    molclr::set_error("segment_pool_bwd: mode %d unsupported (0 mean, 1 add)", mode);
    return MOLCLR_ERR_UNSUPPORTED;
  }
  hipStream_t s = molclr::as_stream(stream);
  if (N == 0) return MOLCLR_OK;
  int d4 = (int)(D / 4);
  // nodes outside every segment get zero gradient (inside the kernel)
  const int64_t work = G * d4 > 0 ? G * d4 : 1;
  hipLaunchKernelGGL(k_pool_bwd<StF32>, dim3(molclr::ceil_div(work, kT)), dim3(kT), 0, s,
                     (const float4*)dout, graph_ptr, dh, G, d4, mode, N);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_segment_pool_fwd_bf16(const uint16_t* h, const int32_t* graph_ptr,
                                            float* out, int64_t G, int64_t D, int mode,
                                            molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "segment_pool_fwd_bf16: dim must be a multiple of 4");
  MOLCLR_REQUIRE(mode == 0 || mode == 1, "segment_pool_fwd_bf16: mode %d (0 mean, 1 add)", mode);
  if (G == 0) return MOLCLR_OK;
  const int d4 = (int)(D / 4);
  hipLaunchKernelGGL(k_pool_fwd<StBF16>, dim3(molclr::ceil_div(G * d4, kT)), dim3(kT), 0,
                     molclr::as_stream(stream), h, graph_ptr, (float4*)out, G, d4, mode);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_segment_pool_bwd_bf16(const float* dout, const int32_t* graph_ptr,
                                            uint16_t* dh, int64_t N, int64_t G, int64_t D, int mode,
                                            molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "segment_pool_bwd_bf16: dim must be a multiple of 4");
  MOLCLR_REQUIRE(mode == 0 || mode == 1, "segment_pool_bwd_bf16: mode %d (0 mean, 1 add)", mode);
  hipStream_t s = molclr::as_stream(stream);
  if (N == 0) return MOLCLR_OK;
  const int d4 = (int)(D / 4);
  const int64_t work = G * d4 > 0 ? G * d4 : 1;  // rows outside every segment: zeroed inside
  hipLaunchKernelGGL(k_pool_bwd<StBF16>, dim3(molclr::ceil_div(work, kT)), dim3(kT), 0, s,
                     (const float4*)dout, graph_ptr, dh, G, d4, mode, N);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

// dtype: MOLCLR_DTYPE_F32 / _BF16 node embeddings h (out and dout stay fp32)
MOLCLR_API int molclr_segment_max_fwd(const void* h, const int32_t* graph_ptr, float* out,
                                      int32_t* argmax, int64_t G, int64_t D, int dtype,
                                      molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "segment_max_fwd: dim must be a multiple of 4");
  MOLCLR_REQUIRE(dtype == MOLCLR_DTYPE_F32 || dtype == MOLCLR_DTYPE_BF16,
                 "segment_max_fwd: bad dtype %d", dtype);
  MOLCLR_REQUIRE(G >= 0, "segment_max_fwd: bad graph count");
  if (G == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(h && graph_ptr && out && argmax, "segment_max_fwd: null pointer");
  const int d4 = (int)(D / 4);
  const dim3 g(molclr::ceil_div(G * d4, kT)), b(kT);
  hipStream_t s = molclr::as_stream(stream);
  if (dtype == MOLCLR_DTYPE_BF16)
    hipLaunchKernelGGL(k_pool_max_fwd<StBF16>, g, b, 0, s, static_cast<const uint16_t*>(h),
                       graph_ptr, (float4*)out, (int4*)argmax, G, d4);
  else
    hipLaunchKernelGGL(k_pool_max_fwd<StF32>, g, b, 0, s, static_cast<const float*>(h), graph_ptr,
                       (float4*)out, (int4*)argmax, G, d4);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_segment_max_bwd(const float* dout, const int32_t* argmax, void* dh,
                                      int64_t N, int64_t G, int64_t D, int dtype,
                                      molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "segment_max_bwd: dim must be a multiple of 4");
  MOLCLR_REQUIRE(dtype == MOLCLR_DTYPE_F32 || dtype == MOLCLR_DTYPE_BF16,
                 "segment_max_bwd: bad dtype %d", dtype);
  MOLCLR_REQUIRE(N >= 0 && G >= 0, "segment_max_bwd: bad sizes");
  hipStream_t s = molclr::as_stream(stream);
  const size_t esz = dtype == MOLCLR_DTYPE_BF16 ? sizeof(uint16_t) : sizeof(float);
  if (N > 0 && molclr::zero_async(dh, (size_t)N * D * esz, s) != hipSuccess) {
    molclr::set_error("segment_max_bwd: memset failed");
    return MOLCLR_ERR_ARG;
  }
  if (G == 0) return MOLCLR_OK;
  const int d4 = (int)(D / 4);
  const dim3 g(molclr::ceil_div(G * d4, kT)), b(kT);
  if (dtype == MOLCLR_DTYPE_BF16)
    hipLaunchKernelGGL(k_pool_max_bwd<StBF16>, g, b, 0, s, (const float4*)dout,
                       (const int4*)argmax, static_cast<uint16_t*>(dh), G, d4);
  else
    hipLaunchKernelGGL(k_pool_max_bwd<StF32>, g, b, 0, s, (const float4*)dout, (const int4*)argmax,
                       static_cast<float*>(dh), G, d4);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_l2norm_fwd(const float* z, float* y, float* norm, int64_t rows, int64_t D,
                                 double eps, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0, "l2norm_fwd: bad dim");
  if (rows == 0) return MOLCLR_OK;
  hipLaunchKernelGGL(k_l2norm_fwd, dim3(molclr::ceil_div(rows * 64, 256)), dim3(256), 0,
                     molclr::as_stream(stream), z, y, norm, rows, D, (float)eps);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_l2norm_bwd(const float* dy, const float* y, const float* norm, float* dz,
                                 int64_t rows, int64_t D, double eps, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0, "l2norm_bwd: bad dim");
  if (rows == 0) return MOLCLR_OK;
  hipLaunchKernelGGL(k_l2norm_bwd, dim3(molclr::ceil_div(rows * 64, 256)), dim3(256), 0,
                     molclr::as_stream(stream), dy, y, norm, dz, rows, D, (float)eps);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_sum_f32(const float* x, float* out, int64_t n, molclr_stream_t stream) {
  MOLCLR_REQUIRE(out && (n == 0 || x), "sum_f32: null pointer");
  hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, molclr::as_stream(stream), x, out, n);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
