// Neighbour aggregation kernels: atom embedding, GINE and GCN message passing.
//
// Reference semantics (CameronDiao/MolCLR):
//   atom embedding   models/ginet_molclr.py:103  h = X1[x0] + X2[x1]
//   GINEConv         models/ginet_molclr.py:29-47 with PyG 1.6.3 propagate
//                    (aggr='add', flow source_to_target): message x_j + e_k,
//                    e_k = E1[bt_k] + E2[bd_k], scatter-add at edge_index[1],
//                    self loop (bt=4, bd=0) appended after the real edges.
//   GCNConv          models/gcn_molclr.py:62-91: message e_k + (xW)_j with a
//                    scalar e_k, then `out += bias`.
//
// Layout: node features are row-major [N, D] fp32, D % 4 == 0.  One thread
// owns one float4 column of one destination row; consecutive threads cover a
// row and then the next, so every neighbour-row gather is a contiguous
// 16*D-byte read by D/4 consecutive lanes, and the output write is fully
// coalesced.  The per-row neighbour loop is a segmented reduction over the
// CSR built by graph.hip — no atomics, deterministic, and in the reference's
// accumulation order (in-edges in edge order, self loop last), so the sums
// are bit-identical to the reference CPU path.
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int kT = 256;

// ---------------------------------------------------------------------------
// atom embedding
// ---------------------------------------------------------------------------
// An atom type or chirality outside the tables (the reference's
// nn.Embedding raises an IndexError on it) makes the row NaN and sets bit 3 of
// *status (MOLCLR_STATUS_ATOM_RANGE) instead of being clamped to a valid row.
// U = 2 (bf16 storage, d4 even): two column units per thread, one 16-byte
// store (as k_bn_apply<StBF16, 2>).
template <typename St, int U = 1>
__global__ void k_atom_embed_fwd(const int64_t* __restrict__ x, const float4* __restrict__ X1,
                                 const float4* __restrict__ X2, typename St::T* __restrict__ h,
                                 int64_t N, int d4, int64_t n1, int64_t n2,
                                 int32_t* __restrict__ status) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * d4 / U) return;
  const int64_t u0 = t * U;
  int64_t i = N * d4 < (1ll << 32) ? (int64_t)((uint32_t)u0 / (uint32_t)d4) : u0 / d4;
  int c = (int)(u0 - i * d4);
  const int64_t a = x[2 * i], b = x[2 * i + 1];
  float4 v[U];
  if (a < 0 || a >= n1 || b < 0 || b >= n2) {
    const float q = __builtin_nanf("");
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = make_float4(q, q, q, q);
    if (c == 0 && status != nullptr) atomicOr(status, MOLCLR_STATUS_ATOM_RANGE);
  } else {
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = f4add(X1[a * d4 + c + j], X2[b * d4 + c + j]);
  }
  if constexpr (U == 2) St::st2(h, t, v[0], v[1]);
  else St::st(h, t, v[0]);
}

// ---------------------------------------------------------------------------
// Atom-embedding gradient by type-sorted segments.  dX1[a] = Σ_{i: x[i,0]=a}
// dh[i] and dX2[b] = Σ_{i: x[i,1]=b} dh[i] are segmented column sums over
// the 2N (node, key) items, key = x[i,0] or n1 + x[i,1].  A stable counting
// sort groups them (item order within a key = node order); the segments are
// cut into chunks of kEmbChunk items, each chunk summed in fp32 by one wave
// (4 columns per lane, whole rows gathered: no LDS read-modify-write chain),
// and the chunk sums of a key are added in fp64 in a fixed order (chunks
// strided over 8 waves, then the waves in order; deterministic: the small
// tables' gradients are sums of ~10^4-10^6 nearly cancelling terms).
// ---------------------------------------------------------------------------
constexpr int kEmbBlock = 256;  // items per sort block
constexpr int kEmbChunk = 128;  // items per fp32 chunk sum

// Out-of-range indices were reported by the forward (NaN rows, status bit 3);
// they are clamped here only to keep the sort's keys in bounds.
__device__ __forceinline__ int emb_key(const int64_t* __restrict__ x, int64_t item, int64_t N,
                                       int64_t n1, int64_t n2) {
  if (item < N) {
    const int64_t a = x[2 * item];
    return (int)(a < 0 ? 0 : (a >= n1 ? n1 - 1 : a));
  }
  const int64_t b = x[2 * (item - N) + 1];
  return (int)(n1 + (b < 0 ? 0 : (b >= n2 ? n2 - 1 : b)));
}

// per sort block: counts of every key
__global__ __launch_bounds__(kEmbBlock) void k_emb_hist(const int64_t* __restrict__ x, int64_t N,
                                                        int64_t n1, int64_t n2,
                                                        int32_t* __restrict__ hist) {
  extern __shared__ int32_t h[];
  const int nk = (int)(n1 + n2);
  for (int k = threadIdx.x; k < nk; k += kEmbBlock) h[k] = 0;
  __syncthreads();
  const int64_t item = (int64_t)blockIdx.x * kEmbBlock + threadIdx.x;
  if (item < 2 * N) atomicAdd(&h[emb_key(x, item, N, n1, n2)], 1);
  __syncthreads();
  for (int k = threadIdx.x; k < nk; k += kEmbBlock) hist[(int64_t)k * gridDim.x + blockIdx.x] = h[k];
}

// one wave per key: exclusive scan of the key's per-block counts (in place,
// hist[k][blk] -> offset within the key's segment) and the key's total
__global__ __launch_bounds__(64) void k_emb_keyscan(int32_t* __restrict__ hist, int nblk,
                                                    int32_t* __restrict__ total) {
  const int64_t k = blockIdx.x;
  const int lane = threadIdx.x;
  int32_t* row = hist + k * nblk;
  int32_t carry = 0;
  for (int base = 0; base < nblk; base += 64) {
    const int b = base + lane;
    const int32_t v = b < nblk ? row[b] : 0;
    int32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (b < nblk) row[b] = carry + incl - v;
    carry += __shfl(incl, 63, 64);
  }
  if (lane == 0) total[k] = carry;
}

// one block: key starts, each key's first chunk, and the chunk table
// (chunk c: items [cbeg[c], cend[c]) of one key); nchunks[0] = count
__global__ __launch_bounds__(1024) void k_emb_plan(const int32_t* __restrict__ total, int nk,
                                                   int32_t* __restrict__ kstart,
                                                   int32_t* __restrict__ cbeg,
                                                   int32_t* __restrict__ cend,
                                                   int32_t* __restrict__ kchunk0,
                                                   int32_t* __restrict__ nchunks, int max_chunks) {
  __shared__ int32_t tot[1024], ks[1025], kc[1025];
  const int t = threadIdx.x;
  tot[t] = t < nk ? total[t] : 0;
  __syncthreads();
  if (t == 0) {
    int32_t run = 0, ch = 0;
    for (int k = 0; k < nk; ++k) {
      ks[k] = run;
      kc[k] = ch;
      run += tot[k];
      ch += (tot[k] + kEmbChunk - 1) / kEmbChunk;
    }
    ks[nk] = run;
    kc[nk] = ch;
    *nchunks = ch;
  }
  __syncthreads();
  for (int k = t; k <= nk; k += 1024) {
    kstart[k] = ks[k];
    kchunk0[k] = kc[k];
  }
  const int nch = kc[nk];
  for (int c = t; c < max_chunks; c += 1024) {
    if (c >= nch) break;
    int lo = 0, hi = nk - 1;  // the key whose chunk range holds c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (kc[mid] <= c) lo = mid;
      else hi = mid - 1;
    }
    const int32_t q = (c - kc[lo]) * kEmbChunk;
    cbeg[c] = ks[lo] + q;
    cend[c] = ks[lo] + (q + kEmbChunk < tot[lo] ? q + kEmbChunk : tot[lo]);
  }
}

// stable scatter: item -> its slot in key order (rank among the block's
// earlier items of the same key)
__global__ __launch_bounds__(kEmbBlock) void k_emb_scatter(const int64_t* __restrict__ x,
                                                           int64_t N, int64_t n1, int64_t n2,
                                                           const int32_t* __restrict__ off,
                                                           const int32_t* __restrict__ kstart,
                                                           int32_t* __restrict__ perm) {
  __shared__ int32_t keys[kEmbBlock];
  const int nk = (int)(n1 + n2);
  const int64_t item = (int64_t)blockIdx.x * kEmbBlock + threadIdx.x;
  const bool live = item < 2 * N;
  const int k = live ? emb_key(x, item, N, n1, n2) : -1;
  keys[threadIdx.x] = k;
  __syncthreads();
  if (!live) return;
  int rank = 0;
  for (int j = 0; j < (int)threadIdx.x; ++j) rank += keys[j] == k;
  (void)nk;
  perm[kstart[k] + off[(int64_t)k * gridDim.x + blockIdx.x] + rank] =
      (int32_t)(item < N ? item : item - N);
}

// one wave per (chunk, 256-column block): fp32 sum of the chunk's rows
template <typename St>
__global__ __launch_bounds__(64) void k_emb_chunk_sum(const typename St::T* __restrict__ dh,
                                                      const int32_t* __restrict__ perm,
                                                      const int32_t* __restrict__ cbeg,
                                                      const int32_t* __restrict__ cend,
                                                      const int32_t* __restrict__ nchunks,
                                                      int64_t d4, double* __restrict__ csum) {
  const int64_t ch = blockIdx.x;
  if (ch >= *nchunks) return;  // the grid is sized for the most chunks possible
  const int64_t c = (int64_t)blockIdx.y * 64 + threadIdx.x;  // float4 column
  if (c >= d4) return;
  const int32_t beg = cbeg[ch], end = cend[ch];
  float4 acc = f4zero();
  int32_t i = beg;
  // sixteen rows in flight (four left a 128-item chunk 32 round trips long);
  // adds in item order
  for (; i + 16 <= end; i += 16) {
    float4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = St::ld(dh, (int64_t)perm[i + u] * d4 + c);
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = f4add(acc, v[u]);
  }
  for (; i + 4 <= end; i += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = St::ld(dh, (int64_t)perm[i + u] * d4 + c);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = f4add(acc, v[u]);
  }
  for (; i < end; ++i) acc = f4add(acc, St::ld(dh, (int64_t)perm[i] * d4 + c));
  double* o = csum + ch * 4 * d4 + 4 * c;
  o[0] = acc.x;
  o[1] = acc.y;
  o[2] = acc.z;
  o[3] = acc.w;
}

// dX[key][col] (+)= Σ over the key's chunks in fp64.  A block per (key, 64
// columns): wave w folds the chunks w, w + kEmbFinW, ... of the key (eight in
// flight), then the waves' sums are added in wave order -- a common atom type
// has ~N / 128 chunks, which one thread per element took as ~30 dependent
// round trips.  Fixed order: deterministic.
constexpr int kEmbFinW = 8;
__global__ __launch_bounds__(64 * kEmbFinW) void k_emb_finish(
    const double* __restrict__ csum, const int32_t* __restrict__ kchunk0, int64_t n1, int64_t n2,
    int64_t D, float* __restrict__ dX1, float* __restrict__ dX2, int accumulate) {
  __shared__ double red[kEmbFinW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t k = blockIdx.x;
  const int64_t col = (int64_t)blockIdx.y * 64 + lane;
  double acc = 0.0;
  if (col < D) {
    int32_t ch = kchunk0[k] + w;
    const int32_t ce = kchunk0[k + 1];
    for (; ch + 7 * kEmbFinW < ce; ch += 8 * kEmbFinW) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = csum[(int64_t)(ch + u * kEmbFinW) * D + col];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; ch < ce; ch += kEmbFinW) acc += csum[(int64_t)ch * D + col];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w != 0 || col >= D) return;
  double t = red[0][lane];
#pragma unroll
  for (int q = 1; q < kEmbFinW; ++q) t += red[q][lane];
  float* o = k < n1 ? dX1 + k * D + col : dX2 + (k - n1) * D + col;
  *o = accumulate ? *o + (float)t : (float)t;
}

// out[r][c] = Σ_p partial[p][r][c], rows [0,n1) -> dX1, [n1,n1+n2) -> dX2.
// The small embedding-table gradients are sums of ~10^4-10^6 nearly cancelling
// terms (ill-conditioned): they are accumulated in fp64 and rounded once.
// A block owns 16 consecutive elements; 64 lanes fold strided partials (four
// loads in flight), then a fixed-order tree through LDS (deterministic).
__global__ __launch_bounds__(1024) void k_reduce_partials_split(
    const double* __restrict__ partial, int64_t P, int64_t rows, int64_t D, int64_t split,
    float* __restrict__ outA, float* __restrict__ outB, int accumulate) {
  constexpr int EL = 16, LANES = 64;
  __shared__ double red[LANES][EL];
  const int cl = threadIdx.x % EL, rl = threadIdx.x / EL;
  const int64_t t = (int64_t)blockIdx.x * EL + cl;
  const int64_t n = rows * D;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (t < n) {
    int64_t p = rl;
    for (; p + 3 * LANES < P; p += 4 * LANES) {
      a0 += partial[p * n + t];
      a1 += partial[(p + LANES) * n + t];
      a2 += partial[(p + 2 * LANES) * n + t];
      a3 += partial[(p + 3 * LANES) * n + t];
    }
    for (; p < P; p += LANES) a0 += partial[p * n + t];
  }
  double acc = (a0 + a1) + (a2 + a3);
  red[rl][cl] = acc;
  __syncthreads();
#pragma unroll
  for (int stride = LANES / 2; stride > 0; stride >>= 1) {
    if (rl < stride) red[rl][cl] = acc = acc + red[rl + stride][cl];
    __syncthreads();
  }
  if (rl != 0 || t >= n) return;
  int64_t r = t / D;
  float* o = r < split ? (outA ? outA + t : nullptr) : (outB ? outB + (t - split * D) : nullptr);
  if (o) *o = accumulate ? *o + (float)acc : (float)acc;
}

// ---------------------------------------------------------------------------
// GINE aggregation
// ---------------------------------------------------------------------------
// Ec[l][r][c] = E1_l[r / 3][c] + E2_l[r % 3][c]: the per-edge embedding of the
// reference (one fp32 add), tabulated once per forward for all layers.
struct TablePtrs {
  const float* e1[MOLCLR_MAX_LAYERS];
  const float* e2[MOLCLR_MAX_LAYERS];
};
__global__ void k_edge_tables_combine(TablePtrs p, float* __restrict__ Ec, int layers, int64_t D,
                                      float* __restrict__ zero, int64_t n_zero) {
  const int64_t per = (int64_t)MOLCLR_NUM_ECOMB * D;
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n_zero) zero[t] = 0.f;  // a caller's slots, zeroed by the same launch
  if (t >= layers * per) return;
  const int l = (int)(t / per);
  const int64_t rc = t - l * per;
  const int r = (int)(rc / D);
  const int64_t c = rc - (int64_t)r * D;
  Ec[t] = p.e1[l][(r / 3) * D + c] + p.e2[l][(r % 3) * D + c];
}

__device__ __forceinline__ uint32_t nbr_degree(uint32_t w0) { return w0 >> 29; }
__device__ __forceinline__ int32_t nbr_node(uint32_t w) { return (int32_t)(w & 0xFFFFFFu); }
__device__ __forceinline__ int nbr_ecomb(uint32_t w) { return (int)((w >> 24) & 15u); }

// message x[src] + Ec[type] of a packed slot
__device__ __forceinline__ float4 gine_msg(const float4* __restrict__ x, const float4* __restrict__ Ec,
                                           uint32_t w, int d4, int c) {
  return f4add(x[(int64_t)nbr_node(w) * d4 + c], Ec[nbr_ecomb(w) * d4 + c]);
}

// Row i's neighbour entry is one 16-byte load shared by the row's D/4 lanes;
// for degree <= 4 every gather is issued before the ordered adds, so the row
// costs two dependent memory latencies (slots, then features).  Rows of
// higher degree walk the CSR.  Order of the adds: in-edges in edge order,
// self loop last — the reference's, so the sums are bit-identical.  One
// float4 of the aggregation, stored and returned.
template <typename St, bool NT = false>
__device__ __forceinline__ float4 gine_agg_elem(
    const typename St::T* __restrict__ x, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
    const uint4* __restrict__ nbr, const float4* __restrict__ Ec, typename St::T* __restrict__ out,
    int64_t t, int64_t i, int c, int d4) {
  auto X = [&](int64_t idx) { return St::ld(x, idx); };
  auto msg = [&](uint32_t w) {
    return f4add(X((int64_t)nbr_node(w) * d4 + c), Ec[nbr_ecomb(w) * d4 + c]);
  };
  const uint4 s = nbr[i];
  const float4 self = X(t);
  const float4 es = Ec[MOLCLR_SELF_LOOP_ECOMB * d4 + c];
  const uint32_t deg = nbr_degree(s.x);
  float4 acc = f4zero();
  if (deg <= MOLCLR_NBR_SLOTS) {
    const float4 m0 = deg > 0 ? msg(s.x) : acc;
    const float4 m1 = deg > 1 ? msg(s.y) : acc;
    const float4 m2 = deg > 2 ? msg(s.z) : acc;
    const float4 m3 = deg > 3 ? msg(s.w) : acc;
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) acc = f4add(acc, m2);
    if (deg > 3) acc = f4add(acc, m3);
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k)
      acc = f4add(acc, f4add(X((int64_t)col[k] * d4 + c), Ec[MOLCLR_ECOMB(ecode[k]) * d4 + c]));
  }
  acc = f4add(acc, f4add(self, es));
  if constexpr (NT) {  // fp32 only
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{acc.x, acc.y, acc.z, acc.w}, reinterpret_cast<f4v*>(out) + t);
  } else {
    St::st(out, t, acc);
  }
  return acc;
}

// ROWMAX: also the output's row maxima as row parts (row_max_parts) and, when
// `slot` is given, its max -- the row scales of the h3 product that consumes it.
// NT: non-temporal output stores (fp32; MOLCLR_AGG_NT=1, an A/B switch).
template <typename St, bool ROWMAX, bool NT = false>
__global__ __launch_bounds__(kT) void k_gine_agg_fwd(
    const typename St::T* __restrict__ x, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
    const uint4* __restrict__ nbr, const float4* __restrict__ Ec, typename St::T* __restrict__ out,
    int64_t N, int d4, float* __restrict__ rowparts, int nparts, float* __restrict__ slot) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  // (row, float4 column) of this lane: 32-bit division when the grid allows
  int64_t i;
  int c;
  if (N * d4 < (1ll << 32)) {
    const uint32_t q = (uint32_t)t / (uint32_t)d4;
    i = q;
    c = (int)((uint32_t)t - q * (uint32_t)d4);
  } else {
    i = t / d4;
    c = (int)(t - i * d4);
  }
  if constexpr (ROWMAX) {
    // every lane reaches the wave reductions (and the slot's block barrier)
    float m = 0.f;
    int row = -1;
    if (t < N * d4) {
      const float4 v = gine_agg_elem<St, NT>(x, rowptr, col, ecode, nbr, Ec, out, t, i, c, d4);
      m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
      row = (int)i;
    }
    if (nparts < 0)  // d4 >= 64: per-wave pairs (molclr_rowmax_layout)
      row_max_waves(m, row, t, N, d4, reinterpret_cast<float2*>(rowparts));
    else
      row_max_parts(m, row, t, N, d4, rowparts, nparts);
    // the tensor max costs a block barrier (waves of one block then retire
    // together): callers whose consumer can fold it (a GEMM's amax_out) pass
    // no slot
    if (slot != nullptr) absmax_publish(m, slot);
    return;
  }
  if (t >= N * d4) return;
  gine_agg_elem<St, NT>(x, rowptr, col, ecode, nbr, Ec, out, t, i, c, d4);
}

// dx[j] = Σ_{out-edges of j in edge order} g[dst] + g[j]  (neighbour slots of the CSC).
// Unlike the forward, the self row is read last and the gathers stay in
// branches: measured 14.0 us against 17.3 us for the forward's structure here
// (round 1, unpaired c2 launch).
template <typename St = StF32>
__global__ __launch_bounds__(kT) void k_transpose_gather(const typename St::T* __restrict__ g,
                                                         const int32_t* __restrict__ rowptr_t,
                                                         const int32_t* __restrict__ col_t,
                                                         const uint4* __restrict__ nbr_t,
                                                         typename St::T* __restrict__ dx, int64_t N,
                                                         int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  // 32-bit division when the grid allows (uniform branch)
  int64_t j = N * d4 < (1ll << 32) ? (int64_t)((uint32_t)t / (uint32_t)d4) : t / d4;
  int c = (int)(t - j * d4);
  const uint4 s = nbr_t[j];
  const uint32_t deg = nbr_degree(s.x);
  float4 acc = f4zero();
  if (deg <= MOLCLR_NBR_SLOTS) {
    if (deg > 0) acc = f4add(acc, St::ld(g, (int64_t)nbr_node(s.x) * d4 + c));
    if (deg > 1) acc = f4add(acc, St::ld(g, (int64_t)nbr_node(s.y) * d4 + c));
    if (deg > 2) acc = f4add(acc, St::ld(g, (int64_t)nbr_node(s.z) * d4 + c));
    if (deg > 3) acc = f4add(acc, St::ld(g, (int64_t)nbr_node(s.w) * d4 + c));
  } else {
    for (int32_t k = rowptr_t[j], e = rowptr_t[j + 1]; k < e; ++k)
      acc = f4add(acc, St::ld(g, (int64_t)col_t[k] * d4 + c));
  }
  St::st(dx, t, f4add(acc, St::ld(g, t)));
}

// Edge-table gradient partials: partial[p][s][c] = Σ_{i in part p} ecount[i][s] * g[i][c].
// Band layout (a block covers `band` rows x all D/4 float4 columns, 1 KiB
// contiguous per wave); fp32 within a partition, fp64 partials across.
template <typename St = StF32>
__global__ void k_ecount_weighted_partial(const typename St::T* __restrict__ g,
                                          const int32_t* __restrict__ ecount, int64_t N, int d4,
                                          int band, int64_t rows_per_part,
                                          double* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float4 red[];  // [band][8][d4]
  const int tid = threadIdx.x;
  const bool live = tid < band * d4;
  const int r = live ? tid / d4 : 0, c = live ? tid - r * d4 : 0;
  const int64_t beg = (int64_t)blockIdx.x * rows_per_part;
  int64_t end = beg + rows_per_part;
  if (end > N) end = N;
  float4 acc[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) acc[s] = f4zero();
  if (live) {
    // a partition is band x 8 rows (ecount_parts), so a thread's eight rows
    // of it are ONE round trip with all eight loads in flight; past 1024
    // partitions (N > 1024 band 8: the c2 paired pass) the cap makes the
    // partitions longer and the loop takes a second, ragged trip.  The adds
    // stay in row order
    constexpr int U = 8;
    for (int64_t i0 = beg + r; i0 < end; i0 += U * (int64_t)band) {
      int4 lo[U], hi[U];
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * band;
        const bool in = i < end;
        const int4* ec = reinterpret_cast<const int4*>(ecount + (in ? i : beg) * 8);
        lo[u] = ec[0];
        hi[u] = ec[1];
        v[u] = St::ld(g, (in ? i : beg) * d4 + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + (int64_t)u * band >= end) break;
        const int cnt[8] = {lo[u].x, lo[u].y, lo[u].z, lo[u].w, hi[u].x, hi[u].y, hi[u].z, hi[u].w};
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const float w = (float)cnt[s];
          acc[s].x += w * v[u].x;
          acc[s].y += w * v[u].y;
          acc[s].z += w * v[u].z;
          acc[s].w += w * v[u].w;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) red[(r * 8 + s) * d4 + c] = acc[s];
  }
  __syncthreads();
  if (!live || r != 0) return;
  double* out = partial + (int64_t)blockIdx.x * 8 * (4 * d4);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    double x = 0.0, y = 0.0, z = 0.0, w = 0.0;
    for (int q = 0; q < band; ++q) {
      const float4 v = red[(q * 8 + s) * d4 + c];
      x += v.x;
      y += v.y;
      z += v.z;
      w += v.w;
    }
    double* o = out + s * 4 * d4 + 4 * c;
    o[0] = x;
    o[1] = y;
    o[2] = z;
    o[3] = w;
  }
}

// ---------------------------------------------------------------------------
// GCN aggregation (scalar edge embedding, bias)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float4 gcn_msg(const float4* __restrict__ xw, const float* __restrict__ E1,
                                          const float* __restrict__ E2, int32_t j, int q, int d4,
                                          int c) {
  const float e = E1[q / 3] + E2[q % 3];
  const float4 v = xw[(int64_t)j * d4 + c];
  return make_float4(e + v.x, e + v.y, e + v.z, e + v.w);
}

__global__ __launch_bounds__(kT) void k_gcn_agg_fwd(
    const float4* __restrict__ xw, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
    const uint4* __restrict__ nbr, const float* __restrict__ E1, const float* __restrict__ E2,
    const float4* __restrict__ bias, float4* __restrict__ out, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t i = N * d4 < (1ll << 32) ? (int64_t)((uint32_t)t / (uint32_t)d4) : t / d4;
  int c = (int)(t - i * d4);
  const uint4 s = nbr[i];
  const float4 self = xw[t];
  const uint32_t deg = nbr_degree(s.x);
  float4 acc = f4zero();
  if (deg <= MOLCLR_NBR_SLOTS) {
    const float4 m0 = deg > 0 ? gcn_msg(xw, E1, E2, nbr_node(s.x), nbr_ecomb(s.x), d4, c) : acc;
    const float4 m1 = deg > 1 ? gcn_msg(xw, E1, E2, nbr_node(s.y), nbr_ecomb(s.y), d4, c) : acc;
    const float4 m2 = deg > 2 ? gcn_msg(xw, E1, E2, nbr_node(s.z), nbr_ecomb(s.z), d4, c) : acc;
    const float4 m3 = deg > 3 ? gcn_msg(xw, E1, E2, nbr_node(s.w), nbr_ecomb(s.w), d4, c) : acc;
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) acc = f4add(acc, m2);
    if (deg > 3) acc = f4add(acc, m3);
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k)
      acc = f4add(acc, gcn_msg(xw, E1, E2, col[k], MOLCLR_ECOMB(ecode[k]), d4, c));
  }
  const float es = E1[MOLCLR_SELF_LOOP_BOND_TYPE] + E2[0];
  acc = f4add(acc, make_float4(es + self.x, es + self.y, es + self.z, es + self.w));
  out[t] = f4add(acc, bias[c]);
}

// One wave per row: rowsum(g_i) weighted by ecount[i][0..8); per-wave fp64 partials.
__global__ __launch_bounds__(256) void k_rowsum_ecount_partial(const float4* __restrict__ g,
                                                               const int32_t* __restrict__ ecount,
                                                               int64_t N, int d4,
                                                               double* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  // two rows per trip: both rows' loads are issued before either reduction
  for (int64_t i = wave; i < N; i += 2 * nwaves) {
    const int64_t i2 = i + nwaves;
    double s = 0.0, s2 = 0.0;
    for (int c = lane; c < d4; c += 64) {
      const float4 v = g[i * d4 + c];
      const float4 v2 = i2 < N ? g[i2 * d4 + c] : f4zero();
      s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
      s2 += ((double)v2.x + (double)v2.y) + ((double)v2.z + (double)v2.w);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_xor(s, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += (double)ecount[i * 8 + q] * s;
    if (i2 < N) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += (double)ecount[i2 * 8 + q] * s2;
    }
  }
  if (lane < 8) {
    double v = acc[0];
#pragma unroll
    for (int q = 1; q < 8; ++q)
      if (lane == q) v = acc[q];
    partial[wave * 8 + lane] = v;
  }
}

// 64 groups of 8 lanes (one per table entry) fold strided partials with four
// in flight, then a fixed-order tree through LDS (deterministic).
__global__ __launch_bounds__(512) void k_reduce_rowsum_partial(
    const double* __restrict__ partial, int64_t nparts, float* __restrict__ dE1,
    float* __restrict__ dE2, int accumulate) {
  constexpr int G = 64;
  __shared__ double red[G][8];
  const int q = threadIdx.x & 7, r = threadIdx.x >> 3;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int64_t p = r;
  for (; p + 3 * G < nparts; p += 4 * G) {
    a0 += partial[p * 8 + q];
    a1 += partial[(p + G) * 8 + q];
    a2 += partial[(p + 2 * G) * 8 + q];
    a3 += partial[(p + 3 * G) * 8 + q];
  }
  for (; p < nparts; p += G) a0 += partial[p * 8 + q];
  double acc = (a0 + a1) + (a2 + a3);
  red[r][q] = acc;
  __syncthreads();
#pragma unroll
  for (int stride = G / 2; stride > 0; stride >>= 1) {
    if (r < stride) red[r][q] = acc = acc + red[r + stride][q];
    __syncthreads();
  }
  if (r != 0) return;
  float* o = q < 5 ? (dE1 ? dE1 + q : nullptr) : (dE2 ? dE2 + (q - 5) : nullptr);
  if (o) *o = accumulate ? *o + (float)acc : (float)acc;
}

// bf16 storage with 16-byte units: a thread owns 8 consecutive columns (one
// uint4 of a bf16 row), so a wave moves the same 1 KiB per load instruction as
// the fp32 kernels' float4 units.  Per element the adds are the fp32 kernels'
// (same order), rounded once to bf16 at the store.
struct F8 {
  float4 a, b;
};
__device__ __forceinline__ F8 ld8(const uint16_t* __restrict__ p, int64_t unit) {
  const uint4 u = reinterpret_cast<const uint4*>(p)[unit];
  return {make_float4(bf16_to_f32(u.x & 0xFFFFu), bf16_to_f32(u.x >> 16), bf16_to_f32(u.y & 0xFFFFu),
                      bf16_to_f32(u.y >> 16)),
          make_float4(bf16_to_f32(u.z & 0xFFFFu), bf16_to_f32(u.z >> 16), bf16_to_f32(u.w & 0xFFFFu),
                      bf16_to_f32(u.w >> 16))};
}
__device__ __forceinline__ void st8(uint16_t* __restrict__ p, int64_t unit, F8 v) {
  reinterpret_cast<uint4*>(p)[unit] =
      make_uint4(f32x2_to_bf16x2(v.a.x, v.a.y), f32x2_to_bf16x2(v.a.z, v.a.w),
                 f32x2_to_bf16x2(v.b.x, v.b.y), f32x2_to_bf16x2(v.b.z, v.b.w));
}
__device__ __forceinline__ F8 f8add(F8 x, F8 y) { return {f4add(x.a, y.a), f4add(x.b, y.b)}; }
__device__ __forceinline__ F8 ec8(const float4* __restrict__ Ec, int comb, int d8, int c) {
  const float4* e = Ec + (int64_t)comb * 2 * d8 + 2 * c;
  return {e[0], e[1]};
}

__global__ __launch_bounds__(kT) void k_gine_agg_fwd_b8(
    const uint16_t* __restrict__ x, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
    const uint4* __restrict__ nbr, const float4* __restrict__ Ec, uint16_t* __restrict__ out,
    int64_t N, int d8) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d8) return;
  const int64_t i = t / d8;
  const int c = (int)(t - i * d8);
  auto msg = [&](uint32_t w) {
    return f8add(ld8(x, (int64_t)nbr_node(w) * d8 + c), ec8(Ec, nbr_ecomb(w), d8, c));
  };
  const uint4 s = nbr[i];
  const F8 self = ld8(x, t);
  const F8 es = ec8(Ec, MOLCLR_SELF_LOOP_ECOMB, d8, c);
  const uint32_t deg = nbr_degree(s.x);
  F8 acc = {f4zero(), f4zero()};
  if (deg <= MOLCLR_NBR_SLOTS) {
    const F8 m0 = deg > 0 ? msg(s.x) : acc;
    const F8 m1 = deg > 1 ? msg(s.y) : acc;
    const F8 m2 = deg > 2 ? msg(s.z) : acc;
    const F8 m3 = deg > 3 ? msg(s.w) : acc;
    if (deg > 0) acc = f8add(acc, m0);
    if (deg > 1) acc = f8add(acc, m1);
    if (deg > 2) acc = f8add(acc, m2);
    if (deg > 3) acc = f8add(acc, m3);
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k)
      acc = f8add(acc, f8add(ld8(x, (int64_t)col[k] * d8 + c), ec8(Ec, MOLCLR_ECOMB(ecode[k]), d8, c)));
  }
  st8(out, t, f8add(acc, f8add(self, es)));
}

__global__ __launch_bounds__(kT) void k_transpose_gather_b8(const uint16_t* __restrict__ g,
                                                            const int32_t* __restrict__ rowptr_t,
                                                            const int32_t* __restrict__ col_t,
                                                            const uint4* __restrict__ nbr_t,
                                                            uint16_t* __restrict__ dx, int64_t N,
                                                            int d8) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d8) return;
  const int64_t j = t / d8;
  const int c = (int)(t - j * d8);
  const uint4 s = nbr_t[j];
  const uint32_t deg = nbr_degree(s.x);
  F8 acc = {f4zero(), f4zero()};
  if (deg <= MOLCLR_NBR_SLOTS) {
    if (deg > 0) acc = f8add(acc, ld8(g, (int64_t)nbr_node(s.x) * d8 + c));
    if (deg > 1) acc = f8add(acc, ld8(g, (int64_t)nbr_node(s.y) * d8 + c));
    if (deg > 2) acc = f8add(acc, ld8(g, (int64_t)nbr_node(s.z) * d8 + c));
    if (deg > 3) acc = f8add(acc, ld8(g, (int64_t)nbr_node(s.w) * d8 + c));
  } else {
    for (int32_t k = rowptr_t[j], e = rowptr_t[j + 1]; k < e; ++k)
      acc = f8add(acc, ld8(g, (int64_t)col_t[k] * d8 + c));
  }
  st8(dx, t, f8add(acc, ld8(g, t)));
}

int64_t ecount_parts(int64_t N, int band) {
  int64_t P = molclr::ceil_div(N, (int64_t)band * 8);
  if (P > 1024) P = 1024;
  if (P < 1) P = 1;
  return P;
}
constexpr int64_t kRowsumBlocks = 1024;  // 4096 waves, ~2 trips of two rows each at c3

}  // namespace

// Column sums shared with norm.hip (declared there).
int molclr_colsum_impl(const float* X, float* out, int64_t rows, int64_t cols, int64_t ld,
                       int accumulate, molclr::Workspace& w, hipStream_t s);
size_t molclr_colsum_ws(int64_t rows, int64_t cols);

MOLCLR_API int molclr_atom_embed_fwd(const int64_t* x, const float* X1, const float* X2,
                                     float* h, int64_t N, int64_t D, int64_t n1, int64_t n2,
                                     int32_t* status, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "atom_embed_fwd: dim %lld must be a positive multiple of 4",
                 (long long)D);
  MOLCLR_REQUIRE(n1 > 0 && n2 > 0, "atom_embed_fwd: empty table");
  if (N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(x && X1 && X2 && h, "atom_embed_fwd: null pointer");
  int d4 = (int)(D / 4);
  hipLaunchKernelGGL(k_atom_embed_fwd<StF32>, dim3(molclr::ceil_div(N * d4, kT)), dim3(kT), 0,
                     molclr::as_stream(stream), x, (const float4*)X1, (const float4*)X2, h, N, d4,
                     n1, n2, status);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

namespace {
struct EmbWs {
  int32_t *hist, *total, *kstart, *cbeg, *cend, *kchunk0, *nchunks, *perm;
  double* csum;
  int64_t nblk, max_chunks;
};
EmbWs emb_ws(void* w, size_t bytes, int64_t N, int64_t D, int64_t n1, int64_t n2) {
  molclr::Workspace ws(w, bytes);
  EmbWs e;
  const int64_t nk = n1 + n2;
  e.nblk = molclr::ceil_div(2 * N > 0 ? 2 * N : 1, (int64_t)kEmbBlock);
  e.max_chunks = molclr::ceil_div(2 * N, (int64_t)kEmbChunk) + nk;  // every key may end ragged
  e.hist = ws.take<int32_t>(e.nblk * nk);
  e.total = ws.take<int32_t>(nk);
  e.kstart = ws.take<int32_t>(nk + 1);
  e.kchunk0 = ws.take<int32_t>(nk + 1);
  e.cbeg = ws.take<int32_t>(e.max_chunks);
  e.cend = ws.take<int32_t>(e.max_chunks);
  e.nchunks = ws.take<int32_t>(1);
  e.perm = ws.take<int32_t>(2 * N > 0 ? 2 * N : 1);
  e.csum = ws.take<double>(e.max_chunks * D);
  return e;
}

template <typename St>
int emb_bwd(const int64_t* x, const typename St::T* dh, float* dX1, float* dX2, int64_t N,
            int64_t D, int64_t n1, int64_t n2, int accumulate, void* workspace,
            size_t workspace_bytes, hipStream_t s) {
  const int64_t nk = n1 + n2;
  const EmbWs e = emb_ws(workspace, workspace_bytes, N, D, n1, n2);
  const int64_t d4 = D / 4;
  if (N > 0) {
    hipLaunchKernelGGL(k_emb_hist, dim3((unsigned)e.nblk), dim3(kEmbBlock), nk * sizeof(int32_t), s,
                       x, N, n1, n2, e.hist);
  } else {
    (void)molclr::zero_async(e.hist, (size_t)e.nblk * nk * sizeof(int32_t), s);
  }
  hipLaunchKernelGGL(k_emb_keyscan, dim3((unsigned)nk), dim3(64), 0, s, e.hist, (int)e.nblk,
                     e.total);
  hipLaunchKernelGGL(k_emb_plan, dim3(1), dim3(1024), 0, s, static_cast<const int32_t*>(e.total),
                     (int)nk, e.kstart, e.cbeg, e.cend, e.kchunk0, e.nchunks, (int)e.max_chunks);
  if (N > 0) {
    hipLaunchKernelGGL(k_emb_scatter, dim3((unsigned)e.nblk), dim3(kEmbBlock), 0, s, x, N, n1, n2,
                       static_cast<const int32_t*>(e.hist), static_cast<const int32_t*>(e.kstart),
                       e.perm);
    hipLaunchKernelGGL(k_emb_chunk_sum<St>, dim3((unsigned)e.max_chunks,
                                                 (unsigned)molclr::ceil_div(d4, 64)),
                       dim3(64), 0, s, dh, static_cast<const int32_t*>(e.perm),
                       static_cast<const int32_t*>(e.cbeg), static_cast<const int32_t*>(e.cend),
                       static_cast<const int32_t*>(e.nchunks), d4, e.csum);
  }
  hipLaunchKernelGGL(k_emb_finish, dim3((unsigned)nk, (unsigned)molclr::ceil_div(D, 64)),
                     dim3(64 * kEmbFinW), 0, s,
                     static_cast<const double*>(e.csum), static_cast<const int32_t*>(e.kchunk0), n1,
                     n2, D, dX1, dX2, accumulate);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
}  // namespace

MOLCLR_API size_t molclr_atom_embed_bwd_workspace_bytes(int64_t N, int64_t D, int64_t n1,
                                                        int64_t n2) {
  const int64_t nk = n1 + n2;
  const int64_t nblk = molclr::ceil_div(2 * N > 0 ? 2 * N : 1, (int64_t)kEmbBlock);
  const int64_t max_chunks = molclr::ceil_div(2 * N, (int64_t)kEmbChunk) + nk;
  return (size_t)(nblk * nk + nk + 2 * (nk + 1) + 2 * max_chunks + 1 + 2 * N) * sizeof(int32_t) +
         (size_t)max_chunks * D * sizeof(double) + 10 * 256;
}

MOLCLR_API int molclr_atom_embed_bwd(const int64_t* x, const float* dh, float* dX1, float* dX2,
                                     int64_t N, int64_t D, int64_t n1, int64_t n2, int accumulate,
                                     void* workspace, size_t workspace_bytes,
                                     molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0 && n1 > 0 && n2 > 0 && N >= 0,
                 "atom_embed_bwd: bad sizes (dim a multiple of 4)");
  MOLCLR_REQUIRE(n1 + n2 <= 1024, "atom_embed_bwd: tables too large");
  MOLCLR_REQUIRE(2 * N < (1ll << 31), "atom_embed_bwd: too many nodes");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_atom_embed_bwd_workspace_bytes(N, D, n1, n2));
  return emb_bwd<StF32>(x, dh, dX1, dX2, N, D, n1, n2, accumulate, workspace, workspace_bytes,
                        molclr::as_stream(stream));
}

MOLCLR_API int molclr_edge_tables_combine(int layers, const float* const* E1s,
                                          const float* const* E2s, float* Ec, int64_t D,
                                          molclr_stream_t stream) {
  return molclr::edge_tables_combine_zero(layers, E1s, E2s, Ec, D, nullptr, 0, stream);
}

int molclr::edge_tables_combine_zero(int layers, const float* const* E1s, const float* const* E2s,
                                     float* Ec, int64_t D, float* zero, int64_t n_zero,
                                     molclr_stream_t stream) {
  MOLCLR_REQUIRE(layers >= 0 && layers <= MOLCLR_MAX_LAYERS && D > 0,
                 "edge_tables_combine: %d layers (max %d), dim %lld", layers, MOLCLR_MAX_LAYERS,
                 (long long)D);
  if (layers == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(E1s && E2s && Ec, "edge_tables_combine: null pointer");
  TablePtrs p{};
  for (int l = 0; l < layers; ++l) {
    MOLCLR_REQUIRE(E1s[l] && E2s[l], "edge_tables_combine: null table of layer %d", l);
    p.e1[l] = E1s[l];
    p.e2[l] = E2s[l];
  }
  const int64_t n = (int64_t)layers * MOLCLR_NUM_ECOMB * D;
  const int64_t work = n > n_zero ? n : n_zero;
  hipLaunchKernelGGL(k_edge_tables_combine, dim3(molclr::ceil_div(work, kT)), dim3(kT), 0,
                     molclr::as_stream(stream), p, Ec, layers, D, zero, n_zero);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

static bool agg_nt() {
  static const bool on = [] {
    const char* e = getenv("MOLCLR_AGG_NT");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

MOLCLR_API int molclr_gine_aggregate_fwd(const float* x, const int32_t* rowptr,
                                         const int32_t* col, const uint8_t* ecode,
                                         const uint32_t* nbr, const float* Ec, float* out,
                                         int64_t N, int64_t D, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "gine_aggregate_fwd: dim %lld must be a multiple of 4",
                 (long long)D);
  if (N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(x && rowptr && nbr && Ec && out, "gine_aggregate_fwd: null pointer");
  int d4 = (int)(D / 4);
  molclr::launch_timed(molclr::kTimeGineAgg, agg_nt() ? k_gine_agg_fwd<StF32, false, true>
                                                      : k_gine_agg_fwd<StF32, false, false>,
                       dim3(molclr::ceil_div(N * d4, kT)), dim3(kT), 0, molclr::as_stream(stream),
                       x, rowptr, col, ecode, (const uint4*)nbr, (const float4*)Ec, out, N, d4,
                       nullptr, 0, nullptr);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int64_t molclr_rowmax_layout(int64_t D) {
  const int64_t d4 = D / 4;
  return d4 >= 64 ? -d4 : (int64_t)molclr_bn_row_parts(D);
}
MOLCLR_API size_t molclr_rowmax_bytes(int64_t N, int64_t D) {
  const int64_t code = molclr_rowmax_layout(D);
  return code < 0 ? (size_t)((N * (D / 4) + 63) / 64) * 2 * sizeof(float)
                  : (size_t)code * N * sizeof(float);
}

MOLCLR_API int molclr_gine_aggregate_fwd_rowmax(const float* x, const int32_t* rowptr,
                                                const int32_t* col, const uint8_t* ecode,
                                                const uint32_t* nbr, const float* Ec, float* out,
                                                int64_t N, int64_t D, float* rowparts, float* slot,
                                                molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "gine_aggregate_fwd_rowmax: dim %lld must be a multiple of 4",
                 (long long)D);
  MOLCLR_REQUIRE(N < (1ll << 31), "gine_aggregate_fwd_rowmax: too many rows");
  if (N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(x && rowptr && nbr && Ec && out && rowparts,
                 "gine_aggregate_fwd_rowmax: null pointer");
  const int d4 = (int)(D / 4);
  static_assert(kT % 64 == 0, "row parts follow the waves");
  molclr::launch_timed(molclr::kTimeGineAgg, agg_nt() ? k_gine_agg_fwd<StF32, true, true>
                                                      : k_gine_agg_fwd<StF32, true, false>,
                       dim3(molclr::ceil_div(N * d4, kT)), dim3(kT), 0, molclr::as_stream(stream),
                       x, rowptr, col, ecode, (const uint4*)nbr, (const float4*)Ec, out, N, d4,
                       rowparts, (int)molclr_rowmax_layout(D), slot);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API size_t molclr_gine_aggregate_bwd_workspace_bytes(int64_t N, int64_t D) {
  return (size_t)ecount_parts(N, molclr::make_band(D).band) * 8 * D * sizeof(double) + 256;
}

MOLCLR_API int molclr_gine_aggregate_bwd(const float* g, const int32_t* rowptr_t,
                                         const int32_t* col_t, const uint32_t* nbr_t,
                                         const int32_t* ecount, float* dx,
                                         float* dE1, float* dE2, int64_t N, int64_t D,
                                         int accumulate, void* workspace, size_t workspace_bytes,
                                         molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "gine_aggregate_bwd: dim must be a multiple of 4");
  hipStream_t s = molclr::as_stream(stream);
  int d4 = (int)(D / 4);
  if (dx && N > 0) {
    MOLCLR_REQUIRE(g && rowptr_t && nbr_t, "gine_aggregate_bwd: null pointer");
    hipLaunchKernelGGL(k_transpose_gather<StF32>, dim3(molclr::ceil_div(N * d4, kT)), dim3(kT), 0,
                       s, g, rowptr_t, col_t, (const uint4*)nbr_t, dx, N, d4);
  }
  if (dE1 || dE2) {
    MOLCLR_REQUIRE_WS(workspace_bytes, molclr_gine_aggregate_bwd_workspace_bytes(N, D));
    molclr::Band b = molclr::make_band(D);
    int64_t P = ecount_parts(N, b.band);
    int64_t rpp = molclr::ceil_div(N > 0 ? N : 1, P);
    double* partial = (double*)workspace;
    size_t lds = (size_t)b.band * 8 * b.d4 * sizeof(float4);
    MOLCLR_REQUIRE(lds <= 65536, "gine_aggregate_bwd: dim too large for the edge-table reduction");
    hipLaunchKernelGGL(k_ecount_weighted_partial<StF32>, dim3(P), dim3(b.threads), lds, s, g,
                       ecount, N, d4, b.band, rpp, partial);
    hipLaunchKernelGGL(k_reduce_partials_split, dim3(molclr::ceil_div(8 * D, 16)), dim3(1024), 0, s,
                       partial, P, (int64_t)8, D, (int64_t)5, dE1, dE2, accumulate);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_gcn_aggregate_fwd(const float* xw, const int32_t* rowptr,
                                        const int32_t* col, const uint8_t* ecode,
                                        const uint32_t* nbr, const float* E1, const float* E2,
                                        const float* bias,
                                        float* out, int64_t N, int64_t D,
                                        molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "gcn_aggregate_fwd: dim must be a multiple of 4");
  if (N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(xw && rowptr && nbr && E1 && E2 && bias && out, "gcn_aggregate_fwd: null pointer");
  int d4 = (int)(D / 4);
  molclr::launch_timed(molclr::kTimeGcnAgg, k_gcn_agg_fwd,
                       dim3(molclr::ceil_div(N * d4, kT)), dim3(kT), 0, molclr::as_stream(stream),
                       (const float4*)xw, rowptr, col, ecode, (const uint4*)nbr, E1, E2,
                       (const float4*)bias, (float4*)out, N, d4);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API size_t molclr_gcn_aggregate_bwd_workspace_bytes(int64_t N, int64_t D) {
  size_t a = (size_t)kRowsumBlocks * 4 * 8 * sizeof(double) + 256;
  return a + molclr_colsum_ws(N, D);
}

MOLCLR_API int molclr_gcn_aggregate_bwd(const float* g, const int32_t* rowptr_t,
                                        const int32_t* col_t, const uint32_t* nbr_t,
                                        const int32_t* ecount, float* dxw,
                                        float* dE1, float* dE2, float* dbias, int64_t N,
                                        int64_t D, int accumulate, void* workspace,
                                        size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "gcn_aggregate_bwd: dim must be a multiple of 4");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_gcn_aggregate_bwd_workspace_bytes(N, D));
  hipStream_t s = molclr::as_stream(stream);
  int d4 = (int)(D / 4);
  if (dxw && N > 0) {
    MOLCLR_REQUIRE(g && rowptr_t && nbr_t, "gcn_aggregate_bwd: null pointer");
    hipLaunchKernelGGL(k_transpose_gather<StF32>, dim3(molclr::ceil_div(N * d4, kT)), dim3(kT), 0,
                       s, g, rowptr_t, col_t, (const uint4*)nbr_t, dxw, N, d4);
  }
  molclr::Workspace w(workspace, workspace_bytes);
  double* partial = w.take<double>(kRowsumBlocks * 4 * 8);
  if (dE1 || dE2) {
    hipLaunchKernelGGL(k_rowsum_ecount_partial, dim3(kRowsumBlocks), dim3(256), 0, s,
                       (const float4*)g, ecount, N, d4, partial);
    hipLaunchKernelGGL(k_reduce_rowsum_partial, dim3(1), dim3(512), 0, s, partial,
                       kRowsumBlocks * 4, dE1, dE2, accumulate);
  }
  MOLCLR_LAUNCHED();
  if (dbias) {
    int rc = molclr_colsum_impl(g, dbias, N, D, D, accumulate, w, s);
    if (rc) return rc;
  }
  return MOLCLR_OK;
}

// ---------------------------------------------------------------------------
// bf16 storage (the c5 configuration): the same kernels over bf16 node
// features, fp32 arithmetic, fp32 tables and table gradients.
// ---------------------------------------------------------------------------
MOLCLR_API int molclr_atom_embed_fwd_bf16(const int64_t* x, const float* X1, const float* X2,
                                          uint16_t* h, int64_t N, int64_t D, int64_t n1,
                                          int64_t n2, int32_t* status, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "atom_embed_fwd_bf16: dim must be a multiple of 4");
  MOLCLR_REQUIRE(n1 > 0 && n2 > 0, "atom_embed_fwd_bf16: empty table");
  if (N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(x && X1 && X2 && h, "atom_embed_fwd_bf16: null pointer");
  const int d4 = (int)(D / 4);
  if (d4 % 2 == 0)
    hipLaunchKernelGGL((k_atom_embed_fwd<StBF16, 2>), dim3(molclr::ceil_div(N * d4 / 2, kT)),
                       dim3(kT), 0, molclr::as_stream(stream), x, (const float4*)X1,
                       (const float4*)X2, h, N, d4, n1, n2, status);
  else
    hipLaunchKernelGGL((k_atom_embed_fwd<StBF16, 1>), dim3(molclr::ceil_div(N * d4, kT)), dim3(kT),
                       0, molclr::as_stream(stream), x, (const float4*)X1, (const float4*)X2, h, N,
                       d4, n1, n2, status);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_atom_embed_bwd_bf16(const int64_t* x, const uint16_t* dh, float* dX1,
                                          float* dX2, int64_t N, int64_t D, int64_t n1, int64_t n2,
                                          int accumulate, void* workspace, size_t workspace_bytes,
                                          molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0 && n1 > 0 && n2 > 0 && N >= 0,
                 "atom_embed_bwd_bf16: bad sizes (dim a multiple of 4)");
  MOLCLR_REQUIRE(n1 + n2 <= 1024, "atom_embed_bwd_bf16: tables too large");
  MOLCLR_REQUIRE(2 * N < (1ll << 31), "atom_embed_bwd_bf16: too many nodes");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_atom_embed_bwd_workspace_bytes(N, D, n1, n2));
  return emb_bwd<StBF16>(x, dh, dX1, dX2, N, D, n1, n2, accumulate, workspace, workspace_bytes,
                         molclr::as_stream(stream));
}

MOLCLR_API int molclr_gine_aggregate_fwd_bf16(const uint16_t* x, const int32_t* rowptr,
                                              const int32_t* col, const uint8_t* ecode,
                                              const uint32_t* nbr, const float* Ec, uint16_t* out,
                                              int64_t N, int64_t D, molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "gine_aggregate_fwd_bf16: dim must be a multiple of 4");
  if (N == 0) return MOLCLR_OK;
  MOLCLR_REQUIRE(x && rowptr && nbr && Ec && out, "gine_aggregate_fwd_bf16: null pointer");
  if (D % 8 == 0) {
    const int d8 = (int)(D / 8);
    molclr::launch_timed(molclr::kTimeGineAgg, k_gine_agg_fwd_b8, dim3(molclr::ceil_div(N * d8, kT)),
                         dim3(kT), 0, molclr::as_stream(stream), x, rowptr, col, ecode,
                         (const uint4*)nbr, (const float4*)Ec, out, N, d8);
  } else {
    const int d4 = (int)(D / 4);
    molclr::launch_timed(molclr::kTimeGineAgg, k_gine_agg_fwd<StBF16, false>,
                         dim3(molclr::ceil_div(N * d4, kT)), dim3(kT), 0, molclr::as_stream(stream),
                         x, rowptr, col, ecode, (const uint4*)nbr, (const float4*)Ec, out, N, d4,
                         nullptr, 0, nullptr);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_gine_aggregate_bwd_bf16(const uint16_t* g, const int32_t* rowptr_t,
                                              const int32_t* col_t, const uint32_t* nbr_t,
                                              const int32_t* ecount, uint16_t* dx, float* dE1,
                                              float* dE2, int64_t N, int64_t D, int accumulate,
                                              void* workspace, size_t workspace_bytes,
                                              molclr_stream_t stream) {
  MOLCLR_REQUIRE(D > 0 && D % 4 == 0, "gine_aggregate_bwd_bf16: dim must be a multiple of 4");
  hipStream_t s = molclr::as_stream(stream);
  const int d4 = (int)(D / 4);
  if (dx && N > 0) {
    MOLCLR_REQUIRE(g && rowptr_t && nbr_t, "gine_aggregate_bwd_bf16: null pointer");
    if (D % 8 == 0)
      hipLaunchKernelGGL(k_transpose_gather_b8, dim3(molclr::ceil_div(N * (D / 8), kT)), dim3(kT), 0,
                         s, g, rowptr_t, col_t, (const uint4*)nbr_t, dx, N, (int)(D / 8));
    else
      hipLaunchKernelGGL(k_transpose_gather<StBF16>, dim3(molclr::ceil_div(N * d4, kT)), dim3(kT),
                         0, s, g, rowptr_t, col_t, (const uint4*)nbr_t, dx, N, d4);
  }
  if (dE1 || dE2) {
    MOLCLR_REQUIRE_WS(workspace_bytes, molclr_gine_aggregate_bwd_workspace_bytes(N, D));
    const molclr::Band b = molclr::make_band(D);
    const int64_t P = ecount_parts(N, b.band);
    const int64_t rpp = molclr::ceil_div(N > 0 ? N : 1, P);
    double* partial = (double*)workspace;
    const size_t lds = (size_t)b.band * 8 * b.d4 * sizeof(float4);
    MOLCLR_REQUIRE(lds <= 65536, "gine_aggregate_bwd_bf16: dim too large for the edge-table reduction");
    hipLaunchKernelGGL(k_ecount_weighted_partial<StBF16>, dim3(P), dim3(b.threads), lds, s, g,
                       ecount, N, d4, b.band, rpp, partial);
    hipLaunchKernelGGL(k_reduce_partials_split, dim3(molclr::ceil_div(8 * D, 16)), dim3(1024), 0, s,
                       partial, P, (int64_t)8, D, (int64_t)5, dE1, dE2, accumulate);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
