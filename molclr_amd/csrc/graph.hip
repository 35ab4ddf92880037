// Graph build: PyG Batch (edge_index / edge_attr / batch) -> destination CSR,
// source CSC, per-node bond-type counts and graph offsets.
//
// Replaces the per-layer `add_self_loops` + host-built self-loop attribute of
// the reference (models/ginet_molclr.py:31-37, models/gcn_molclr.py:64-70):
// here it is done once per batch and the self loop (bond type 4, dir 0,
// appended LAST by PyG) is implicit in the aggregation kernels.
//
// The CSR keeps, inside every destination row, the original edge order — the
// order in which PyG's scatter-add (torch_scatter 2.0.6 on CPU) accumulates
// messages — so the aggregation reproduces the reference's rounding exactly.
// Slots are claimed with integer atomics and each (short) row is then sorted by
// edge id, so the result is deterministic.
#include "common.h"

namespace {

constexpr int kScanThreads = 1024;

// The inputs as up to MOLCLR_MAX_SEGMENTS concatenated PyG batches (the two
// contrastive views of a step built as one graph): segment s's nodes, edges
// and graphs follow those of segments 0..s-1.
// Device-sized (molclr_graph_build_dev, a captured step): the node and edge
// counts of every segment are read on the device (dcount), the outputs have a
// fixed capacity and segment s's edge_index rows are eld[s] apart.
struct GSegs {
  int n;
  const int64_t* ei[MOLCLR_MAX_SEGMENTS];
  const int64_t* ea[MOLCLR_MAX_SEGMENTS];
  const int64_t* batch[MOLCLR_MAX_SEGMENTS];
  int64_t n0[MOLCLR_MAX_SEGMENTS + 1], e0[MOLCLR_MAX_SEGMENTS + 1], g0[MOLCLR_MAX_SEGMENTS + 1];
  int64_t eld[MOLCLR_MAX_SEGMENTS];
  const int64_t* dcount;  // [nseg] nodes, then [nseg] edges; NULL = host-sized
};

__device__ __forceinline__ int gseg(const int64_t* off, int n, int64_t k) {
  int s = 0;
  while (s + 1 < n && k >= off[s + 1]) ++s;
  return s;
}

// count of segment s: which = 0 nodes, 1 edges
__device__ __forceinline__ int64_t gcount(const GSegs& sg, int which, int s) {
  if (sg.dcount) return sg.dcount[which * sg.n + s];
  return which ? sg.e0[s + 1] - sg.e0[s] : sg.n0[s + 1] - sg.n0[s];
}
__device__ __forceinline__ int64_t gbase(const GSegs& sg, int which, int s) {
  if (!sg.dcount) return which ? sg.e0[s] : sg.n0[s];
  int64_t b = 0;
  for (int q = 0; q < s; ++q) b += sg.dcount[which * sg.n + q];
  return b;
}
struct GLoc {
  int s;  // -1: past the last segment
  int64_t base, cnt;
};
__device__ __forceinline__ GLoc glocate(const GSegs& sg, int which, int64_t k) {
  int64_t b = 0;
  for (int s = 0; s < sg.n; ++s) {
    const int64_t c = gcount(sg, which, s);
    if (k < b + c) return {s, b, c};
    b += c;
  }
  return {-1, b, 0};
}

__global__ void k_graph_init(int32_t* __restrict__ ecount, int32_t* __restrict__ counters,
                             int64_t n_counters, int64_t N, int32_t* __restrict__ status) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) *status = 0;
  if (t < n_counters) counters[t] = 0;
  if (t < N * MOLCLR_ECOUNT_STRIDE) {
    int j = (int)(t % MOLCLR_ECOUNT_STRIDE);
    // implicit self loop: bond type 4 (slot 4) and bond dir 0 (slot 5)
    ecount[t] = (j == MOLCLR_SELF_LOOP_BOND_TYPE || j == 5) ? 1 : 0;
  }
}

__device__ void graph_ptr_item(const GSegs& sg, int64_t t, int64_t N, int64_t G,
                               int32_t* __restrict__ graph_ptr, int32_t* __restrict__ status);

// blockIdx.y == 0: the edges (below); == 1: graph_ptr and the batch checks
// (independent work, one launch)
__global__ void k_graph_count(GSegs sg, int64_t E, int32_t* __restrict__ src32,
                              int32_t* __restrict__ dst32, uint8_t* __restrict__ code8,
                              int32_t* __restrict__ indeg, int32_t* __restrict__ outdeg,
                              int32_t* __restrict__ ecount, int32_t* __restrict__ status, int64_t N,
                              int64_t G, int32_t* __restrict__ graph_ptr) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.y == 1) {
    if (k < (N > G + 1 ? N : G + 1)) graph_ptr_item(sg, k, N, G, graph_ptr, status);
    return;
  }
  if (k >= E) return;
  const GLoc le = glocate(sg, 1, k);
  if (le.s < 0) return;  // past the real edges of a device-sized build
  const int g = le.s;
  const int64_t kk = k - le.base, Eg = le.cnt;
  const int64_t Ng = gcount(sg, 0, g), nb = gbase(sg, 0, g);
  const int64_t* ei = sg.ei[g];
  const int64_t* ea = sg.ea[g];
  int64_t s = ei[kk], d = ei[(sg.dcount ? sg.eld[g] : Eg) + kk];
  int64_t bt = ea[2 * kk], bd = ea[2 * kk + 1];
  int bad = 0;
  if (s < 0 || s >= Ng || d < 0 || d >= Ng) {
    bad |= 1;
    s = s < 0 ? 0 : (s >= Ng ? Ng - 1 : s);
    d = d < 0 ? 0 : (d >= Ng ? Ng - 1 : d);
  }
  if (bt < 0 || bt >= MOLCLR_NUM_BOND_TYPE || bd < 0 || bd >= MOLCLR_NUM_BOND_DIR) {
    bad |= 2;
    bt = bt < 0 ? 0 : (bt >= MOLCLR_NUM_BOND_TYPE ? MOLCLR_NUM_BOND_TYPE - 1 : bt);
    bd = bd < 0 ? 0 : (bd >= MOLCLR_NUM_BOND_DIR ? MOLCLR_NUM_BOND_DIR - 1 : bd);
  }
  if (bad) atomicOr(status, bad);
  s += nb;
  d += nb;
  src32[k] = (int32_t)s;
  dst32[k] = (int32_t)d;
  code8[k] = (uint8_t)(bt | (bd << 3));
  atomicAdd(&indeg[d], 1);
  atomicAdd(&outdeg[s], 1);
  atomicAdd(&ecount[d * MOLCLR_ECOUNT_STRIDE + bt], 1);
  atomicAdd(&ecount[d * MOLCLR_ECOUNT_STRIDE + 5 + bd], 1);
}

// Exclusive scan of deg[0..n) into ptr[0..n]; blockIdx.y selects one of two
// arrays, blockIdx.x a tile of 1024 x 8 elements.  Every tile's block first
// sums the degrees before its tile itself (a coalesced block reduction: the
// tiles need no carry from each other, so they run side by side instead of
// one block walking the tiles in turn -- 19.3 us at c2's 30.6k rows), then
// loads its tile coalesced into LDS; each thread sums 8 consecutive
// elements, one block-wide scan of the 1024 thread sums (wave scans + a scan
// of the 16 wave totals), and each thread writes its 8 prefixes.  Integer
// sums: the result is the sequential scan's.
constexpr int kScanPer = 8;
__global__ __launch_bounds__(kScanThreads) void k_scan2(const int32_t* __restrict__ degA,
                                                        int32_t* __restrict__ ptrA,
                                                        const int32_t* __restrict__ degB,
                                                        int32_t* __restrict__ ptrB, int64_t n) {
  constexpr int TILE = kScanPer * kScanThreads;
  const int32_t* deg = blockIdx.y == 0 ? degA : degB;
  int32_t* ptr = blockIdx.y == 0 ? ptrA : ptrB;
  __shared__ int32_t tile[TILE];
  __shared__ int32_t wsum[kScanThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * TILE;
  // this tile's loads first (their latency overlaps the prefix reduction)
  int32_t nx[kScanPer];
#pragma unroll
  for (int c = 0; c < kScanPer; ++c) {
    const int64_t idx = base + (int64_t)c * kScanThreads + tid;
    nx[c] = idx < n ? deg[idx] : 0;
  }
  // carry = Σ deg[0, base): eight loads in flight per thread
  int32_t pre = 0;
  for (int64_t i0 = tid; i0 < base; i0 += (int64_t)kScanPer * kScanThreads) {
    int32_t q[kScanPer];
#pragma unroll
    for (int c = 0; c < kScanPer; ++c) {
      const int64_t i = i0 + (int64_t)c * kScanThreads;
      q[c] = i < base ? deg[i] : 0;
    }
#pragma unroll
    for (int c = 0; c < kScanPer; ++c) pre += q[c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (lane == 0) wsum[wid] = pre;
#pragma unroll
  for (int c = 0; c < kScanPer; ++c) tile[c * kScanThreads + tid] = nx[c];
  __syncthreads();
  int32_t carry = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) carry += wsum[w];
  int32_t v[kScanPer], x = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    v[j] = tile[kScanPer * tid + j];
    x += v[j];
  }
  const int32_t own = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t u = __shfl_up(x, o, 64);
    if (lane >= o) x += u;
  }
  __syncthreads();  // every thread has read the prefix's wave sums
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (wid == 0) {
    int32_t w = lane < kScanThreads / 64 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t u = __shfl_up(w, o, 64);
      if (lane >= o) w += u;
    }
    if (lane < kScanThreads / 64) wsum[lane] = w;
  }
  __syncthreads();
  int32_t run = carry + (wid > 0 ? wsum[wid - 1] : 0) + x - own;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    const int64_t idx = base + (int64_t)kScanPer * tid + j;
    if (idx < n) ptr[idx] = run;
    run += v[j];
  }
  if (tid == 0 && base + TILE >= n) ptr[n] = carry + wsum[kScanThreads / 64 - 1];
}

__global__ void k_graph_fill(GSegs sg, const int32_t* __restrict__ src32,
                             const int32_t* __restrict__ dst32, int64_t E,
                             const int32_t* __restrict__ rowptr,
                             const int32_t* __restrict__ rowptr_t, int32_t* __restrict__ cur,
                             int32_t* __restrict__ cur_t, int32_t* __restrict__ perm,
                             int32_t* __restrict__ perm_t) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= E || (sg.dcount && k >= gbase(sg, 1, sg.n))) return;
  int32_t s = src32[k], d = dst32[k];
  perm[rowptr[d] + atomicAdd(&cur[d], 1)] = (int32_t)k;
  perm_t[rowptr_t[s] + atomicAdd(&cur_t[s], 1)] = (int32_t)k;
}

// Threads [0,N) finish CSR row i, threads [N,2N) finish CSC row i: sort the
// row's edge ids (insertion sort; molecular degrees are tiny), gather, and
// write the row's neighbour-slot entry (uint4, see molclr.h): the first four
// in-edges packed with their combined edge-table index, and the degree.
__global__ void k_graph_rows(int64_t N, const int32_t* __restrict__ src32,
                             const int32_t* __restrict__ dst32, const uint8_t* __restrict__ code8,
                             const int32_t* __restrict__ rowptr, const int32_t* __restrict__ rowptr_t,
                             int32_t* __restrict__ perm, int32_t* __restrict__ perm_t,
                             int32_t* __restrict__ col, uint8_t* __restrict__ ecode,
                             int32_t* __restrict__ col_t, uint4* __restrict__ nbr,
                             uint4* __restrict__ nbr_t) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * N) return;
  bool csc = t >= N;
  int64_t i = csc ? t - N : t;
  const int32_t* ptr = csc ? rowptr_t : rowptr;
  int32_t* p = csc ? perm_t : perm;
  int32_t beg = ptr[i], end = ptr[i + 1];
  for (int32_t a = beg + 1; a < end; ++a) {
    int32_t key = p[a];
    int32_t b = a - 1;
    while (b >= beg && p[b] > key) {
      p[b + 1] = p[b];
      --b;
    }
    p[b + 1] = key;
  }
  uint32_t slot[MOLCLR_NBR_SLOTS] = {0u, 0u, 0u, 0u};
  if (!csc) {
    for (int32_t a = beg; a < end; ++a) {
      int32_t k = p[a];
      col[a] = src32[k];
      ecode[a] = code8[k];
      if (a - beg < MOLCLR_NBR_SLOTS)
        slot[a - beg] = (uint32_t)src32[k] | ((uint32_t)MOLCLR_ECOMB(code8[k]) << 24);
    }
  } else {
    for (int32_t a = beg; a < end; ++a) {
      col_t[a] = dst32[p[a]];
      if (a - beg < MOLCLR_NBR_SLOTS) slot[a - beg] = (uint32_t)dst32[p[a]];
    }
  }
  const int32_t deg = end - beg;
  slot[0] |= (uint32_t)(deg > MOLCLR_NBR_SLOTS ? MOLCLR_NBR_OVERFLOW : deg) << 29;
  (csc ? nbr_t : nbr)[i] = make_uint4(slot[0], slot[1], slot[2], slot[3]);
}

__device__ void graph_ptr_item(const GSegs& sg, int64_t t, int64_t N, int64_t G,
                               int32_t* __restrict__ graph_ptr, int32_t* __restrict__ status) {
  if (t < N) {
    const GLoc ln = glocate(sg, 0, t);
    if (ln.s >= 0) {  // (padding rows of a device-sized build have no batch entry)
      const int g = ln.s;
      const int64_t* batch = sg.batch[g];
      const int64_t i = t - ln.base, Gg = sg.g0[g + 1] - sg.g0[g];
      const int64_t b = batch[i];
      if (b < 0 || b >= Gg || (i > 0 && batch[i - 1] > b)) atomicOr(status, 4);
    }
  }
  if (t <= G) {
    if (t == G) {
      graph_ptr[t] = (int32_t)gbase(sg, 0, sg.n);  // the real node count
    } else {
      // lower_bound(batch of t's segment, local graph id) + the segment's first node
      const int g = gseg(sg.g0, sg.n, t);
      const int64_t* batch = sg.batch[g];
      const int64_t want = t - sg.g0[g];
      int64_t lo = 0, hi = gcount(sg, 0, g);
      while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (batch[mid] < want) lo = mid + 1;
        else hi = mid;
      }
      graph_ptr[t] = (int32_t)(gbase(sg, 0, g) + lo);
    }
  }
}

// The kernels of a build over N rows / E edge slots (host-sized: the real
// counts; device-sized: the capacities, the kernels read the real counts).
int build_launch(const GSegs& sg, int64_t N, int64_t E, int64_t G, int32_t* rowptr, int32_t* col,
                 uint8_t* ecode, int32_t* rowptr_t, int32_t* col_t, uint32_t* nbr, uint32_t* nbr_t,
                 int32_t* ecount, int32_t* graph_ptr, int32_t* status, void* workspace,
                 size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_REQUIRE(rowptr && rowptr_t && ecount && graph_ptr && status && (N == 0 || (nbr && nbr_t)),
                 "graph_build: null output");
  MOLCLR_REQUIRE(E == 0 || (col && ecode && col_t), "graph_build: null edge buffer");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_graph_build_workspace_bytes(N, E));
  hipStream_t s = molclr::as_stream(stream);
  molclr::Workspace w(workspace, workspace_bytes);
  int32_t* src32 = w.take<int32_t>(E);
  int32_t* dst32 = w.take<int32_t>(E);
  uint8_t* code8 = w.take<uint8_t>(E);
  int32_t* counters = w.take<int32_t>(4 * N);
  int32_t* indeg = counters;
  int32_t* outdeg = counters + N;
  int32_t* cur = counters + 2 * N;
  int32_t* cur_t = counters + 3 * N;
  int32_t* perm = w.take<int32_t>(E);
  int32_t* perm_t = w.take<int32_t>(E);

  const int T = 256;
  int64_t n_init = 8 * N > 4 * N ? 8 * N : 4 * N;
  if (n_init < 1) n_init = 1;
  hipLaunchKernelGGL(k_graph_init, dim3(molclr::ceil_div(n_init, T)), dim3(T), 0, s, ecount,
                     counters, 4 * N, N, status);
  const int64_t n_ptr = N > G + 1 ? N : G + 1;
  const int64_t bx = molclr::ceil_div(E > n_ptr ? E : n_ptr, T);
  hipLaunchKernelGGL(k_graph_count, dim3((unsigned)bx, 2), dim3(T), 0, s, sg, E, src32, dst32,
                     code8, indeg, outdeg, ecount, status, N, G, graph_ptr);
  hipLaunchKernelGGL(k_scan2,
                     dim3((unsigned)(N > 0 ? molclr::ceil_div(N, kScanPer * kScanThreads) : 1), 2),
                     dim3(kScanThreads), 0, s, indeg, rowptr, outdeg, rowptr_t, N);
  if (E > 0) {
    hipLaunchKernelGGL(k_graph_fill, dim3(molclr::ceil_div(E, T)), dim3(T), 0, s, sg, src32, dst32,
                       E, rowptr, rowptr_t, cur, cur_t, perm, perm_t);
  }
  if (N > 0) {
    hipLaunchKernelGGL(k_graph_rows, dim3(molclr::ceil_div(2 * N, T)), dim3(T), 0, s, N, src32,
                       dst32, code8, rowptr, rowptr_t, perm, perm_t, col, ecode, col_t,
                       (uint4*)nbr, (uint4*)nbr_t);
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

}  // namespace

MOLCLR_API size_t molclr_graph_build_workspace_bytes(int64_t N, int64_t E) {
  molclr::Workspace w(nullptr, 0);
  w.take<int32_t>(E);      // src32
  w.take<int32_t>(E);      // dst32
  w.take<uint8_t>(E);      // code8
  w.take<int32_t>(4 * N);  // indeg, outdeg, cur, cur_t
  w.take<int32_t>(E);      // perm
  w.take<int32_t>(E);      // perm_t
  return w.used + 256;
}

MOLCLR_API int molclr_graph_build_multi(int nseg, const molclr_graph_segment* segs,
                                        int32_t* rowptr, int32_t* col, uint8_t* ecode,
                                        int32_t* rowptr_t, int32_t* col_t, uint32_t* nbr,
                                        uint32_t* nbr_t, int32_t* ecount, int32_t* graph_ptr,
                                        int32_t* status, void* workspace, size_t workspace_bytes,
                                        molclr_stream_t stream) {
  MOLCLR_REQUIRE(nseg >= 1 && nseg <= MOLCLR_MAX_SEGMENTS && segs,
                 "graph_build: %d segments (1..%d)", nseg, MOLCLR_MAX_SEGMENTS);
  GSegs sg{};
  sg.n = nseg;
  for (int g = 0; g < nseg; ++g) {
    const molclr_graph_segment& q = segs[g];
    MOLCLR_REQUIRE(q.num_nodes >= 0 && q.num_edges >= 0 && q.num_graphs >= 0,
                   "graph_build: negative size in segment %d", g);
    sg.ei[g] = q.edge_index;
    sg.ea[g] = q.edge_attr;
    sg.batch[g] = q.batch;
    sg.n0[g + 1] = sg.n0[g] + q.num_nodes;
    sg.e0[g + 1] = sg.e0[g] + q.num_edges;
    sg.g0[g + 1] = sg.g0[g] + q.num_graphs;
  }
  for (int g = nseg; g < MOLCLR_MAX_SEGMENTS; ++g) {
    sg.n0[g + 1] = sg.n0[nseg];
    sg.e0[g + 1] = sg.e0[nseg];
    sg.g0[g + 1] = sg.g0[nseg];
  }
  const int64_t N = sg.n0[nseg], E = sg.e0[nseg], G = sg.g0[nseg];
  MOLCLR_REQUIRE(N <= MOLCLR_NBR_MAX_NODES && E < (int64_t)1 << 31,
                 "graph_build: %lld nodes exceed the neighbour-slot limit %d (or E > int32)",
                 (long long)N, MOLCLR_NBR_MAX_NODES);
  for (int g = 0; g < nseg; ++g) {
    MOLCLR_REQUIRE(segs[g].num_edges == 0 || (segs[g].edge_index && segs[g].edge_attr),
                   "graph_build: null edge input in segment %d", g);
    MOLCLR_REQUIRE(segs[g].num_nodes == 0 || segs[g].batch, "graph_build: null batch in segment %d",
                   g);
  }
  return build_launch(sg, N, E, G, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount,
                      graph_ptr, status, workspace, workspace_bytes, stream);
}

MOLCLR_API int molclr_graph_build(const int64_t* edge_index, const int64_t* edge_attr,
                                  const int64_t* batch, int64_t N, int64_t E, int64_t G,
                                  int32_t* rowptr, int32_t* col, uint8_t* ecode,
                                  int32_t* rowptr_t, int32_t* col_t, uint32_t* nbr,
                                  uint32_t* nbr_t, int32_t* ecount, int32_t* graph_ptr,
                                  int32_t* status, void* workspace,
                                  size_t workspace_bytes, molclr_stream_t stream) {
  const molclr_graph_segment seg{edge_index, edge_attr, batch, N, E, G};
  return molclr_graph_build_multi(1, &seg, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount,
                                  graph_ptr, status, workspace, workspace_bytes, stream);
}

// ---------------------------------------------------------------------------
// Device-sized build (a captured training step, molclr_amd/graph_step.py):
// the batch arrives in fixed-capacity staging buffers and the kernels read
// the real counts on the device, so one launch sequence serves every batch
// whose sizes fit the capacities.
// ---------------------------------------------------------------------------
namespace {

constexpr int kStageJobs = 5 * MOLCLR_MAX_SEGMENTS + 1;
struct StageJob {
  const int64_t* src;  // NULL: fill with 0
  int64_t* dst;
  int64_t count;
};
struct StageJobs {
  StageJob j[kStageJobs];
  int64_t counts[2 * MOLCLR_MAX_SEGMENTS];
  int64_t* counts_dst;
  int ncounts;
};

// blockIdx.y: the job; grid-stride over its elements
__global__ void k_stage(StageJobs jb) {
  const StageJob& j = jb.j[blockIdx.y];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < j.count;
       i += (int64_t)gridDim.x * blockDim.x)
    j.dst[i] = j.src ? j.src[i] : 0;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < jb.ncounts)
    jb.counts_dst[threadIdx.x] = jb.counts[threadIdx.x];
}

}  // namespace

MOLCLR_API int molclr_stage_segments(int nseg, const molclr_stage_source* src,
                                     const molclr_graph_staged_segment* dst, int64_t* x_all,
                                     int64_t num_nodes_cap, int64_t num_edges_cap,
                                     int64_t* counts, molclr_stream_t stream) {
  MOLCLR_REQUIRE(nseg >= 1 && nseg <= MOLCLR_MAX_SEGMENTS && src && dst && x_all && counts,
                 "stage_segments: %d segments (1..%d) / null pointer", nseg, MOLCLR_MAX_SEGMENTS);
  StageJobs jb{};
  int nj = 0;
  int64_t row = 0, edges = 0, most = 1;
  auto job = [&](const int64_t* from, int64_t* to, int64_t n) {
    jb.j[nj++] = {from, to, n};
    if (n > most) most = n;
  };
  for (int s = 0; s < nseg; ++s) {
    const molclr_stage_source& a = src[s];
    const molclr_graph_staged_segment& b = dst[s];
    MOLCLR_REQUIRE(a.num_nodes >= 0 && a.num_edges >= 0 && a.num_nodes <= b.node_cap &&
                       a.num_edges <= b.edge_cap,
                   "stage_segments: segment %d has %lld nodes / %lld edges, capacity %lld / %lld", s,
                   (long long)a.num_nodes, (long long)a.num_edges, (long long)b.node_cap,
                   (long long)b.edge_cap);
    MOLCLR_REQUIRE((a.num_nodes == 0 || (a.x && a.batch && b.batch)) &&
                       (a.num_edges == 0 || (a.edge_index && a.edge_attr && b.edge_index &&
                                             b.edge_attr)),
                   "stage_segments: null buffer in segment %d", s);
    job(a.x, x_all + 2 * row, 2 * a.num_nodes);
    job(a.edge_index, const_cast<int64_t*>(b.edge_index), a.num_edges);
    job(a.edge_index + a.num_edges, const_cast<int64_t*>(b.edge_index) + b.edge_cap, a.num_edges);
    job(a.edge_attr, const_cast<int64_t*>(b.edge_attr), 2 * a.num_edges);
    job(a.batch, const_cast<int64_t*>(b.batch), a.num_nodes);
    jb.counts[s] = a.num_nodes;
    jb.counts[nseg + s] = a.num_edges;
    row += a.num_nodes;
    edges += a.num_edges;
  }
  MOLCLR_REQUIRE(edges <= num_edges_cap, "stage_segments: %lld edges exceed the capacity %lld",
                 (long long)edges, (long long)num_edges_cap);
  MOLCLR_REQUIRE(row <= num_nodes_cap, "stage_segments: %lld nodes exceed the capacity %lld",
                 (long long)row, (long long)num_nodes_cap);
  job(nullptr, x_all + 2 * row, 2 * (num_nodes_cap - row));  // padding atoms: type 0, chirality 0
  jb.counts_dst = counts;
  jb.ncounts = 2 * nseg;
  const int T = 256;
  int64_t bx = molclr::ceil_div(most, T);
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(k_stage, dim3((unsigned)bx, nj), dim3(T), 0, molclr::as_stream(stream), jb);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_graph_build_dev(int nseg, const molclr_graph_staged_segment* segs,
                                      const int64_t* counts, int64_t num_nodes_cap,
                                      int64_t num_edges_cap, int32_t* rowptr, int32_t* col,
                                      uint8_t* ecode, int32_t* rowptr_t, int32_t* col_t,
                                      uint32_t* nbr, uint32_t* nbr_t, int32_t* ecount,
                                      int32_t* graph_ptr, int32_t* status, void* workspace,
                                      size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_REQUIRE(nseg >= 1 && nseg <= MOLCLR_MAX_SEGMENTS && segs && counts,
                 "graph_build_dev: %d segments (1..%d)", nseg, MOLCLR_MAX_SEGMENTS);
  GSegs sg{};
  sg.n = nseg;
  sg.dcount = counts;
  int64_t ecap = 0;
  for (int g = 0; g < nseg; ++g) {
    const molclr_graph_staged_segment& q = segs[g];
    MOLCLR_REQUIRE(q.node_cap >= 0 && q.edge_cap >= 0 && q.num_graphs >= 0 &&
                       q.edge_index && q.edge_attr && q.batch,
                   "graph_build_dev: bad segment %d", g);
    sg.ei[g] = q.edge_index;
    sg.ea[g] = q.edge_attr;
    sg.batch[g] = q.batch;
    sg.eld[g] = q.edge_cap;
    sg.g0[g + 1] = sg.g0[g] + q.num_graphs;
    ecap += q.edge_cap;
  }
  for (int g = nseg; g < MOLCLR_MAX_SEGMENTS; ++g) sg.g0[g + 1] = sg.g0[nseg];
  const int64_t N = num_nodes_cap, E = num_edges_cap, G = sg.g0[nseg];
  MOLCLR_REQUIRE(E >= 1 && E <= ecap,
                 "graph_build_dev: num_edges_cap %lld must be in [1, sum of edge_cap %lld]",
                 (long long)E, (long long)ecap);
  MOLCLR_REQUIRE(N >= 1 && N <= MOLCLR_NBR_MAX_NODES && E < (int64_t)1 << 31,
                 "graph_build_dev: %lld nodes exceed the neighbour-slot limit %d (or E > int32)",
                 (long long)N, MOLCLR_NBR_MAX_NODES);
  return build_launch(sg, N, E, G, rowptr, col, ecode, rowptr_t, col_t, nbr, nbr_t, ecount,
                      graph_ptr, status, workspace, workspace_bytes, stream);
}
