// Microbenchmark: variants of the GINE forward aggregation (k_gine_agg_fwd)
// on real batch CSRs.  Tuning tool only — not part of the library.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/aggvar.hip -o tools/libaggvar.so
//   python tools/agg_bench.py
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace {

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  int q = nwg / 8, r = nwg % 8;
  int x = bid % 8, pos = bid / 8;
  int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + pos;
}

// V0: the library kernel
__global__ __launch_bounds__(256) void v0(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                          const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                          const uint32_t* __restrict__, const float4* __restrict__ E1,
                                          const float4* __restrict__ E2, float4* __restrict__ out,
                                          int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t i = t / d4;
  int c = (int)(t - i * d4);
  int32_t k = rowptr[i];
  const int32_t end = rowptr[i + 1];
  float4 acc = make_float4(0, 0, 0, 0);
  for (; k + 2 <= end; k += 2) {
    int32_t j0 = col[k], j1 = col[k + 1];
    uint8_t q0 = ecode[k], q1 = ecode[k + 1];
    float4 x0 = x[(int64_t)j0 * d4 + c];
    float4 x1 = x[(int64_t)j1 * d4 + c];
    float4 e0 = f4add(E1[(q0 & 7) * d4 + c], E2[(q0 >> 3) * d4 + c]);
    float4 e1 = f4add(E1[(q1 & 7) * d4 + c], E2[(q1 >> 3) * d4 + c]);
    acc = f4add(acc, f4add(x0, e0));
    acc = f4add(acc, f4add(x1, e1));
  }
  if (k < end) {
    int32_t j0 = col[k];
    uint8_t q0 = ecode[k];
    float4 e0 = f4add(E1[(q0 & 7) * d4 + c], E2[(q0 >> 3) * d4 + c]);
    acc = f4add(acc, f4add(x[(int64_t)j0 * d4 + c], e0));
  }
  float4 es = f4add(E1[4 * d4 + c], E2[c]);
  acc = f4add(acc, f4add(x[t], es));
  out[t] = acc;
}

// ELL slot: col | code << 24; slot 0 bits 29..31 = degree (7 = overflow -> CSR)
__device__ __forceinline__ float4 msg(const float4* __restrict__ x, const float4* __restrict__ E1,
                                      const float4* __restrict__ E2, uint32_t p, int d4, int c) {
  const int32_t j = (int32_t)(p & 0xFFFFFF);
  const uint32_t q = (p >> 24) & 31;
  return f4add(x[(int64_t)j * d4 + c], f4add(E1[(q & 7) * d4 + c], E2[(q >> 3) * d4 + c]));
}

template <bool REMAP, bool NT>
__device__ __forceinline__ void ell_row(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                        const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                        const uint4* __restrict__ ell, const float4* __restrict__ E1,
                                        const float4* __restrict__ E2, float4* __restrict__ out,
                                        int64_t t, int d4) {
  int64_t i = t / d4;
  int c = (int)(t - i * d4);
  const uint4 s = ell[i];
  const float4 self = x[t];
  const float4 es = f4add(E1[4 * d4 + c], E2[c]);
  const uint32_t deg = s.x >> 29;
  float4 acc = make_float4(0, 0, 0, 0);
  if (deg <= 4) {
    // predicated: issue all gathers first, add in order
    float4 m0 = deg > 0 ? msg(x, E1, E2, s.x, d4, c) : acc;
    float4 m1 = deg > 1 ? msg(x, E1, E2, s.y, d4, c) : acc;
    float4 m2 = deg > 2 ? msg(x, E1, E2, s.z, d4, c) : acc;
    float4 m3 = deg > 3 ? msg(x, E1, E2, s.w, d4, c) : acc;
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) acc = f4add(acc, m2);
    if (deg > 3) acc = f4add(acc, m3);
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k) {
      const uint8_t q = ecode[k];
      acc = f4add(acc, f4add(x[(int64_t)col[k] * d4 + c], f4add(E1[(q & 7) * d4 + c], E2[(q >> 3) * d4 + c])));
    }
  }
  acc = f4add(acc, f4add(self, es));
  if (NT)
  {
    typedef float v4f __attribute__((ext_vector_type(4)));
    v4f a = {acc.x, acc.y, acc.z, acc.w};
    __builtin_nontemporal_store(a, reinterpret_cast<v4f*>(out) + t);
  }
  else
    out[t] = acc;
}

template <bool REMAP, bool NT>
__global__ void v_ell(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                      const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                      const uint32_t* __restrict__ ell, const float4* __restrict__ E1,
                      const float4* __restrict__ E2, float4* __restrict__ out, int64_t N, int d4) {
  const int b = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  int64_t t = (int64_t)b * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  ell_row<REMAP, NT>(x, rowptr, col, ecode, reinterpret_cast<const uint4*>(ell), E1, E2, out, t, d4);
}

// ELL + combined edge table Ec[bt*3+bd] = E1[bt]+E2[bd] (same single rounding)
__global__ void v_ellc(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                       const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                       const uint32_t* __restrict__ ell, const float4* __restrict__ Ec,
                       const float4* __restrict__ E2, float4* __restrict__ out, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t i = t / d4;
  int c = (int)(t - i * d4);
  const uint4 s = reinterpret_cast<const uint4*>(ell)[i];
  const float4 self = x[t];
  const float4 es = Ec[12 * d4 + c];
  const uint32_t deg = s.x >> 29;
  float4 acc = make_float4(0, 0, 0, 0);
#define MSGC(p) f4add(x[(int64_t)((p) & 0xFFFFFF) * d4 + c], Ec[((((p) >> 24) & 7) * 3 + (((p) >> 27) & 3)) * d4 + c])
  if (deg <= 4) {
    float4 m0 = deg > 0 ? MSGC(s.x) : acc;
    float4 m1 = deg > 1 ? MSGC(s.y) : acc;
    float4 m2 = deg > 2 ? MSGC(s.z) : acc;
    float4 m3 = deg > 3 ? MSGC(s.w) : acc;
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) acc = f4add(acc, m2);
    if (deg > 3) acc = f4add(acc, m3);
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k) {
      const uint32_t p = (uint32_t)col[k] | ((uint32_t)ecode[k] << 24);
      acc = f4add(acc, MSGC(p));
    }
  }
#undef MSGC
  acc = f4add(acc, f4add(self, es));
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f a = {acc.x, acc.y, acc.z, acc.w};
  __builtin_nontemporal_store(a, reinterpret_cast<v4f*>(out) + t);
}

// v_ellc with the self row loaded last and a plain store
__global__ void v_ellc2(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                        const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                        const uint32_t* __restrict__ ell, const float4* __restrict__ Ec,
                        const float4* __restrict__ E2, float4* __restrict__ out, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t i = t / d4;
  int c = (int)(t - i * d4);
  const uint4 s = reinterpret_cast<const uint4*>(ell)[i];
  const uint32_t deg = s.x >> 29;
  float4 acc = make_float4(0, 0, 0, 0);
#define MSGC(p) f4add(x[(int64_t)((p) & 0xFFFFFF) * d4 + c], Ec[((((p) >> 24) & 7) * 3 + (((p) >> 27) & 3)) * d4 + c])
  if (deg <= 4) {
    if (deg > 0) acc = f4add(acc, MSGC(s.x));
    if (deg > 1) acc = f4add(acc, MSGC(s.y));
    if (deg > 2) acc = f4add(acc, MSGC(s.z));
    if (deg > 3) acc = f4add(acc, MSGC(s.w));
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k) {
      const uint32_t p = (uint32_t)col[k] | ((uint32_t)ecode[k] << 24);
      acc = f4add(acc, MSGC(p));
    }
  }
#undef MSGC
  out[t] = f4add(acc, f4add(x[t], Ec[12 * d4 + c]));
}

// 8 neighbour slots (two uint4 per row; degree in bits 29..31 of word 0 of the
// first uint4 as 0..7, with 7 meaning >= 7 -> CSR walk)
__global__ void v_ellc8(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                        const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                        const uint32_t* __restrict__ ell, const float4* __restrict__ Ec,
                        const float4* __restrict__ E2, float4* __restrict__ out, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t i = t / d4;
  int c = (int)(t - i * d4);
  const uint4 s = reinterpret_cast<const uint4*>(ell)[2 * i];
  const uint4 s2 = reinterpret_cast<const uint4*>(ell)[2 * i + 1];
  const float4 self = x[t];
  const float4 es = Ec[12 * d4 + c];
  const uint32_t deg = s.x >> 29;
  float4 acc = make_float4(0, 0, 0, 0);
#define MSGC(p) f4add(x[(int64_t)((p) & 0xFFFFFF) * d4 + c], Ec[((((p) >> 24) & 7) * 3 + (((p) >> 27) & 3)) * d4 + c])
  if (deg < 7) {
    float4 m0 = deg > 0 ? MSGC(s.x) : acc;
    float4 m1 = deg > 1 ? MSGC(s.y) : acc;
    float4 m2 = deg > 2 ? MSGC(s.z) : acc;
    float4 m3 = deg > 3 ? MSGC(s.w) : acc;
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) acc = f4add(acc, m2);
    if (deg > 3) acc = f4add(acc, m3);
    if (deg > 4) {
      float4 m4 = MSGC(s2.x);
      float4 m5 = deg > 5 ? MSGC(s2.y) : acc;
      acc = f4add(acc, m4);
      if (deg > 5) acc = f4add(acc, m5);
    }
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k) {
      const uint32_t p = (uint32_t)col[k] | ((uint32_t)ecode[k] << 24);
      acc = f4add(acc, MSGC(p));
    }
  }
#undef MSGC
  out[t] = f4add(acc, f4add(self, es));
}

__global__ void k_make_ell8(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                            const uint8_t* __restrict__ ecode, uint32_t* __restrict__ ell, int64_t N) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int32_t b = rowptr[i], e = rowptr[i + 1], deg = e - b;
  uint32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < 8 && k < deg; ++k) s[k] = (uint32_t)col[b + k] | ((uint32_t)ecode[b + k] << 24);
  s[0] = (s[0] & 0x1FFFFFFF) | ((uint32_t)(deg >= 7 ? 7 : deg) << 29);
  reinterpret_cast<uint4*>(ell)[2 * i] = make_uint4(s[0], s[1], s[2], s[3]);
  reinterpret_cast<uint4*>(ell)[2 * i + 1] = make_uint4(s[4], s[5], s[6], s[7]);
}

__global__ void k_make_ec(const float* E1, const float* E2, float* Ec, int D) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 15 * D) return;
  int r = t / D, c = t % D;
  Ec[t] = E1[(r / 3) * D + c] + E2[(r % 3) * D + c];
}

// LDS-staged molecule tiles.  Block t owns rows [s_t, s_{t+1}) where s_t is the
// first molecule start >= t*R (so tiles are unions of whole molecules and their
// edges are tile-internal).  The tile is processed in chunks of at most CAP
// rows: stage x rows + neighbour slots (coalesced, all loads in flight), sync,
// then every output float4 gathers its neighbours from LDS (global memory for
// neighbours outside the chunk), in the reference's order.
__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* __restrict__ a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <int R, int CAP>
__global__ __launch_bounds__(256) void v_tile(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                              const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                              const uint32_t* __restrict__ ell, const float4* __restrict__ Ec,
                                              const int32_t* __restrict__ gptr, int64_t G,
                                              float4* __restrict__ out, int64_t N, int d4) {
  extern __shared__ float4 xs[];  // [CAP * d4]
  __shared__ uint4 sl[CAP];
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  // tile bounds: molecule starts
  int64_t a = (int64_t)t * R, b = a + R;
  int64_t s0 = a >= N ? N : gptr[lower_bound_i32(gptr, G + 1, a)];
  int64_t s1 = b >= N ? N : gptr[lower_bound_i32(gptr, G + 1, b)];
  if (t == 0) s0 = 0;
  const uint4* nbr = reinterpret_cast<const uint4*>(ell);
  for (int64_t c0 = s0; c0 < s1; c0 += CAP) {
    const int rows = (int)min((int64_t)CAP, s1 - c0);
    const int n = rows * d4;
    const float4* src = x + c0 * d4;
    for (int k = threadIdx.x; k < n; k += blockDim.x) xs[k] = src[k];
    for (int k = threadIdx.x; k < rows; k += blockDim.x) sl[k] = nbr[c0 + k];
    __syncthreads();
    float4* dst = out + c0 * d4;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const int r = k / d4, c = k - r * d4;
      const uint4 s = sl[r];
      const uint32_t deg = s.x >> 29;
      float4 acc = make_float4(0, 0, 0, 0);
#define XJ(j) (((j) >= c0 && (j) < c0 + rows) ? xs[((j) - c0) * d4 + c] : x[(int64_t)(j) * d4 + c])
#define MSG(p) f4add(XJ((int64_t)((p) & 0xFFFFFF)), Ec[((((p) >> 24) & 7) * 3 + (((p) >> 27) & 3)) * d4 + c])
      if (deg <= 4) {
        float4 m0 = deg > 0 ? MSG(s.x) : acc;
        float4 m1 = deg > 1 ? MSG(s.y) : acc;
        float4 m2 = deg > 2 ? MSG(s.z) : acc;
        float4 m3 = deg > 3 ? MSG(s.w) : acc;
        if (deg > 0) acc = f4add(acc, m0);
        if (deg > 1) acc = f4add(acc, m1);
        if (deg > 2) acc = f4add(acc, m2);
        if (deg > 3) acc = f4add(acc, m3);
      } else {
        for (int32_t q = rowptr[c0 + r], e = rowptr[c0 + r + 1]; q < e; ++q) {
          const uint32_t p = (uint32_t)col[q] | ((uint32_t)ecode[q] << 24);
          acc = f4add(acc, MSG(p));
        }
      }
#undef MSG
#undef XJ
      acc = f4add(acc, f4add(xs[k], Ec[12 * d4 + c]));
      dst[k] = acc;
    }
    __syncthreads();
  }
}

// v_tile2: same tiling, 512 threads, all staging loads issued before any LDS
// store (U per thread), edge table in LDS, self value kept in registers.
template <int R, int CAP, int U>
__global__ __launch_bounds__(512) void v_tile2(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                               const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                               const uint32_t* __restrict__ ell, const float4* __restrict__ Ec,
                                               const int32_t* __restrict__ gptr, int64_t G,
                                               float4* __restrict__ out, int64_t N, int d4) {
  extern __shared__ float4 lds[];  // [15 * d4] edge table, then [CAP * d4] rows
  float4* es = lds;
  float4* xs = lds + 15 * d4;
  __shared__ uint4 sl[CAP];
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t s0 = gptr[t], s1 = gptr[t + 1];  // precomputed tile_ptr
  if (s0 >= s1) return;
  for (int k = threadIdx.x; k < 15 * d4; k += 512) es[k] = Ec[k];
  const uint4* nbr = reinterpret_cast<const uint4*>(ell);
  for (int64_t c0 = s0; c0 < s1; c0 += CAP) {
    const int rows = (int)min((int64_t)CAP, s1 - c0);
    const int n = rows * d4;
    const float4* src = x + c0 * d4;
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = threadIdx.x + u * 512;
      if (k < n) v[u] = src[k];
    }
    if (threadIdx.x < rows) sl[threadIdx.x] = nbr[c0 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = threadIdx.x + u * 512;
      if (k < n) xs[k] = v[u];
    }
    __syncthreads();
    float4* dst = out + c0 * d4;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = threadIdx.x + u * 512;
      if (k >= n) break;
      const int r = k / d4, c = k - r * d4;
      const uint4 s = sl[r];
      const uint32_t deg = s.x >> 29;
      float4 acc = make_float4(0, 0, 0, 0);
#define XJ(j) (((j) >= c0 && (j) < c0 + rows) ? xs[((j) - c0) * d4 + c] : x[(int64_t)(j) * d4 + c])
#define MSG(p) f4add(XJ((int64_t)((p) & 0xFFFFFF)), es[((((p) >> 24) & 7) * 3 + (((p) >> 27) & 3)) * d4 + c])
      if (deg <= 4) {
        float4 m0 = deg > 0 ? MSG(s.x) : acc;
        float4 m1 = deg > 1 ? MSG(s.y) : acc;
        float4 m2 = deg > 2 ? MSG(s.z) : acc;
        float4 m3 = deg > 3 ? MSG(s.w) : acc;
        if (deg > 0) acc = f4add(acc, m0);
        if (deg > 1) acc = f4add(acc, m1);
        if (deg > 2) acc = f4add(acc, m2);
        if (deg > 3) acc = f4add(acc, m3);
      } else {
        for (int32_t q = rowptr[c0 + r], e = rowptr[c0 + r + 1]; q < e; ++q) {
          const uint32_t p = (uint32_t)col[q] | ((uint32_t)ecode[q] << 24);
          acc = f4add(acc, MSG(p));
        }
      }
#undef MSG
#undef XJ
      acc = f4add(acc, f4add(v[u], es[12 * d4 + c]));
      dst[k] = acc;
    }
    __syncthreads();
  }
}

// two elements per thread, half the grid apart
__global__ void v_ell2(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                       const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                       const uint32_t* __restrict__ ell, const float4* __restrict__ E1,
                       const float4* __restrict__ E2, float4* __restrict__ out, int64_t N, int d4) {
  const int64_t total = N * d4, half = (total + 1) / 2;
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= half) return;
  ell_row<true, false>(x, rowptr, col, ecode, reinterpret_cast<const uint4*>(ell), E1, E2, out, t, d4);
  if (t + half < total)
    ell_row<true, false>(x, rowptr, col, ecode, reinterpret_cast<const uint4*>(ell), E1, E2, out, t + half, d4);
}

// bandwidth floor: out = x + self-loop embedding (same bytes, no gather)
__global__ void v_copy(const float4* __restrict__ x, const int32_t* __restrict__, const int32_t* __restrict__,
                       const uint8_t* __restrict__, const uint32_t* __restrict__, const float4* __restrict__ E1,
                       const float4* __restrict__ E2, float4* __restrict__ out, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int c = (int)(t % d4);
  out[t] = f4add(x[t], f4add(E1[4 * d4 + c], E2[c]));
}

__global__ void k_make_ell(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                           const uint8_t* __restrict__ ecode, uint32_t* __restrict__ ell, int64_t N) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int32_t b = rowptr[i], e = rowptr[i + 1], deg = e - b;
  uint32_t s[4] = {0, 0, 0, 0};
  for (int k = 0; k < 4 && k < deg; ++k) s[k] = (uint32_t)col[b + k] | ((uint32_t)ecode[b + k] << 24);
  s[0] = (s[0] & 0x1FFFFFFF) | ((uint32_t)(deg > 4 ? 7 : deg) << 29);
  reinterpret_cast<uint4*>(ell)[i] = make_uint4(s[0], s[1], s[2], s[3]);
}

// transpose gather, CSR (pre-slot library version) and slot versions
__global__ __launch_bounds__(256) void t_csr(const float4* __restrict__ g, const int32_t* __restrict__ rowptr_t,
                                             const int32_t* __restrict__ col_t, const uint4* __restrict__,
                                             float4* __restrict__ dx, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t j = t / d4;
  int c = (int)(t - j * d4);
  int32_t k = rowptr_t[j];
  const int32_t end = rowptr_t[j + 1];
  float4 acc = make_float4(0, 0, 0, 0);
  for (; k + 2 <= end; k += 2) {
    int32_t i0 = col_t[k], i1 = col_t[k + 1];
    float4 g0 = g[(int64_t)i0 * d4 + c];
    float4 g1 = g[(int64_t)i1 * d4 + c];
    acc = f4add(acc, g0);
    acc = f4add(acc, g1);
  }
  if (k < end) acc = f4add(acc, g[(int64_t)col_t[k] * d4 + c]);
  acc = f4add(acc, g[t]);
  dx[t] = acc;
}
template <bool REMAP>
__global__ __launch_bounds__(256) void t_slot(const float4* __restrict__ g, const int32_t* __restrict__ rowptr_t,
                                              const int32_t* __restrict__ col_t, const uint4* __restrict__ nbr_t,
                                              float4* __restrict__ dx, int64_t N, int d4) {
  int64_t t = (int64_t)(REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t j = t / d4;
  int c = (int)(t - j * d4);
  const uint4 s = nbr_t[j];
  const float4 self = g[t];
  const uint32_t deg = s.x >> 29;
  float4 acc = make_float4(0, 0, 0, 0);
  if (deg <= 4) {
    const float4 m0 = deg > 0 ? g[(int64_t)(s.x & 0xFFFFFF) * d4 + c] : acc;
    const float4 m1 = deg > 1 ? g[(int64_t)(s.y & 0xFFFFFF) * d4 + c] : acc;
    const float4 m2 = deg > 2 ? g[(int64_t)(s.z & 0xFFFFFF) * d4 + c] : acc;
    const float4 m3 = deg > 3 ? g[(int64_t)(s.w & 0xFFFFFF) * d4 + c] : acc;
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) acc = f4add(acc, m2);
    if (deg > 3) acc = f4add(acc, m3);
  } else {
    for (int32_t k = rowptr_t[j], e = rowptr_t[j + 1]; k < e; ++k) acc = f4add(acc, g[(int64_t)col_t[k] * d4 + c]);
  }
  dx[t] = f4add(acc, self);
}
__global__ void k_rewrite_t(const float4* __restrict__ src, float4* __restrict__ dst, int64_t n) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) dst[t] = src[t];
}
// slot variants: (3) self loaded last, (4) pairs like the CSR loop
__global__ __launch_bounds__(256) void t_slot3(const float4* __restrict__ g, const int32_t* __restrict__ rowptr_t,
                                               const int32_t* __restrict__ col_t, const uint4* __restrict__ nbr_t,
                                               float4* __restrict__ dx, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t j = t / d4;
  int c = (int)(t - j * d4);
  const uint4 s = nbr_t[j];
  const uint32_t deg = s.x >> 29;
  float4 acc = make_float4(0, 0, 0, 0);
  if (deg <= 4) {
    if (deg > 0) acc = f4add(acc, g[(int64_t)(s.x & 0xFFFFFF) * d4 + c]);
    if (deg > 1) acc = f4add(acc, g[(int64_t)(s.y & 0xFFFFFF) * d4 + c]);
    if (deg > 2) acc = f4add(acc, g[(int64_t)(s.z & 0xFFFFFF) * d4 + c]);
    if (deg > 3) acc = f4add(acc, g[(int64_t)(s.w & 0xFFFFFF) * d4 + c]);
  } else {
    for (int32_t k = rowptr_t[j], e = rowptr_t[j + 1]; k < e; ++k) acc = f4add(acc, g[(int64_t)col_t[k] * d4 + c]);
  }
  dx[t] = f4add(acc, g[t]);
}
__global__ __launch_bounds__(256) void t_slot4(const float4* __restrict__ g, const int32_t* __restrict__ rowptr_t,
                                               const int32_t* __restrict__ col_t, const uint4* __restrict__ nbr_t,
                                               float4* __restrict__ dx, int64_t N, int d4) {
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= N * d4) return;
  int64_t j = t / d4;
  int c = (int)(t - j * d4);
  const uint4 s = nbr_t[j];
  const uint32_t deg = s.x >> 29;
  float4 acc = make_float4(0, 0, 0, 0);
  if (deg <= 4) {
    // unconditional loads of valid rows (empty slots hold node 0, bits masked): no exec masking
    const float4 m0 = g[(int64_t)(s.x & 0xFFFFFF) * d4 + c];
    const float4 m1 = g[(int64_t)(s.y & 0xFFFFFF) * d4 + c];
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) {
      const float4 m2 = g[(int64_t)(s.z & 0xFFFFFF) * d4 + c];
      const float4 m3 = g[(int64_t)(s.w & 0xFFFFFF) * d4 + c];
      acc = f4add(acc, m2);
      if (deg > 3) acc = f4add(acc, m3);
    }
  } else {
    for (int32_t k = rowptr_t[j], e = rowptr_t[j + 1]; k < e; ++k) acc = f4add(acc, g[(int64_t)col_t[k] * d4 + c]);
  }
  dx[t] = f4add(acc, g[t]);
}
typedef void (*tgfn)(const float4*, const int32_t*, const int32_t*, const uint4*, float4*, int64_t, int);

typedef void (*kfn)(const float4*, const int32_t*, const int32_t*, const uint8_t*, const uint32_t*,
                    const float4*, const float4*, float4*, int64_t, int);

}  // namespace

extern "C" double aggvar_transpose(int variant, int nb, int reps, const float** gs, const int32_t** rowptrs,
                                   const int32_t** cols, const uint32_t** nbrs, const int64_t* Ns, float** outs,
                                   int d4, const float* warm_src, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  tgfn f = variant == 0 ? t_csr : variant == 1 ? t_slot<true> : variant == 2 ? t_slot<false>
          : variant == 3 ? t_slot3 : t_slot4;
  std::vector<hipEvent_t> ev(2 * nb * reps);
  for (auto& e : ev) (void)hipEventCreate(&e);
  int n = 0;
  for (int r = 0; r < reps; ++r)
    for (int g = 0; g < nb; ++g) {
      int64_t total = Ns[g] * d4;
      if (warm_src)
        hipLaunchKernelGGL(k_rewrite_t, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                           (const float4*)warm_src, (float4*)gs[g], total);
      hipExtLaunchKernelGGL(f, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, ev[2 * n], ev[2 * n + 1], 0u,
                            (const float4*)gs[g], rowptrs[g], cols[g], (const uint4*)nbrs[g], (float4*)outs[g], Ns[g], d4);
      ++n;
    }
  (void)hipStreamSynchronize(s);
  double tot = 0;
  for (int k = 0; k < n; ++k) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]);
    tot += ms;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return tot / n * 1e3;
}

extern "C" int aggvar_make_ell8(const int32_t* rowptr, const int32_t* col, const uint8_t* ecode,
                                uint32_t* ell, int64_t N, void* stream) {
  hipLaunchKernelGGL(k_make_ell8, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, rowptr, col, ecode,
                     ell, N);
  return (int)hipGetLastError();
}

extern "C" int aggvar_make_ell(const int32_t* rowptr, const int32_t* col, const uint8_t* ecode,
                               uint32_t* ell, int64_t N, void* stream) {
  hipLaunchKernelGGL(k_make_ell, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, rowptr, col, ecode,
                     ell, N);
  return (int)hipGetLastError();
}

// Runs `variant` over nb graphs (arrays of device pointers), `reps` rounds;
// returns the mean per-launch kernel time in microseconds (dispatch events).
__global__ void k_rewrite(const float4* __restrict__ src, float4* __restrict__ dst, int64_t n, int remap) {
  int64_t t = (int64_t)(remap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x) * blockDim.x + threadIdx.x;
  if (t < n) dst[t] = src[t];
}

static const float* g_warm_src = nullptr;  // non-null: rewrite x from here before each launch
static int g_warm_remap = 0;
extern "C" void aggvar_set_warm(const float* src, int remap) { g_warm_src = src; g_warm_remap = remap; }

static const int32_t** g_gptrs = nullptr;
static const int64_t* g_Gs = nullptr;
extern "C" void aggvar_set_graphs(const int32_t** gptrs, const int64_t* Gs) { g_gptrs = gptrs; g_Gs = Gs; }

typedef void (*tfn)(const float4*, const int32_t*, const int32_t*, const uint8_t*, const uint32_t*,
                    const float4*, const int32_t*, int64_t, float4*, int64_t, int);

extern "C" double aggvar_run(int variant, int block, int nb, int reps, const float** xs,
                             const int32_t** rowptrs, const int32_t** cols, const uint8_t** ecodes,
                             const uint32_t** ells, const int64_t* Ns, const float* E1, const float* E2,
                             float** outs, int d4, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  kfn f = nullptr;
  int per_thread = 1;
  switch (variant) {
    case 0: f = v0; break;
    case 1: f = v_ell<true, false>; break;
    case 2: f = v_ell<false, false>; break;
    case 3: f = v_ell<true, true>; break;
    case 4: f = v_ell2; per_thread = 2; break;
    case 5: f = v_copy; break;
    case 6: f = v_ellc; break;
    case 12: f = v_ellc2; break;
    case 13: f = v_ellc8; break;
    case 7: case 8: case 9: case 10: case 11: break;
    default: return -1;
  }
  float* Ec = nullptr;
  if (variant >= 6 && variant != 7 && variant != 8 && variant != 9 && variant != 10 && variant != 11) {
    (void)hipMalloc(&Ec, 15 * d4 * 16);
    hipLaunchKernelGGL(k_make_ec, dim3((15 * d4 * 4 + 255) / 256), dim3(256), 0, s, E1, E2, Ec, d4 * 4);
    E1 = Ec;
  }
  std::vector<hipEvent_t> ev(2 * nb * reps);
  for (auto& e : ev) (void)hipEventCreate(&e);
  int n = 0;
  for (int r = 0; r < reps; ++r)
    for (int g = 0; g < nb; ++g) {
      int64_t total = Ns[g] * d4;
      int64_t th = (total + per_thread - 1) / per_thread;
      dim3 grid((unsigned)((th + block - 1) / block));
      if (g_warm_src)
        hipLaunchKernelGGL(k_rewrite, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                           (const float4*)g_warm_src, (float4*)xs[g], total, g_warm_remap);
      if (variant == 10 || variant == 11) {
        tfn tf = variant == 10 ? v_tile2<32, 48, 8> : v_tile2<16, 32, 5>;
        int R = variant == 10 ? 32 : 16;
        int cap = variant == 10 ? 48 : 32;
        dim3 tg((unsigned)((Ns[g] + R - 1) / R));
        hipExtLaunchKernelGGL(tf, tg, dim3(512), (uint32_t)((cap + 15) * d4 * 16), s, ev[2 * n], ev[2 * n + 1], 0u,
                              (const float4*)xs[g], rowptrs[g], cols[g], ecodes[g], ells[g],
                              (const float4*)E1, g_gptrs[g], g_Gs[g], (float4*)outs[g], Ns[g], d4);
      } else if (variant >= 7 && variant <= 9) {
        tfn tf = variant == 7 ? v_tile<32, 56> : variant == 8 ? v_tile<16, 40> : v_tile<64, 96>;
        int R = variant == 7 ? 32 : variant == 8 ? 16 : 64;
        int cap = variant == 7 ? 56 : variant == 8 ? 40 : 96;
        dim3 tg((unsigned)((Ns[g] + R - 1) / R));
        hipExtLaunchKernelGGL(tf, tg, dim3(block), (uint32_t)(cap * d4 * 16), s, ev[2 * n], ev[2 * n + 1], 0u,
                              (const float4*)xs[g], rowptrs[g], cols[g], ecodes[g], ells[g],
                              (const float4*)E1, g_gptrs[g], g_Gs[g], (float4*)outs[g], Ns[g], d4);
      } else
      hipExtLaunchKernelGGL(f, grid, dim3(block), 0, s, ev[2 * n], ev[2 * n + 1], 0u,
                            (const float4*)xs[g], rowptrs[g], cols[g], ecodes[g], ells[g],
                            (const float4*)E1, (const float4*)E2, (float4*)outs[g], Ns[g], d4);
      ++n;
    }
  (void)hipStreamSynchronize(s);
  double tot = 0;
  for (int k = 0; k < n; ++k) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]);
    tot += ms;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  if (Ec) (void)hipFree(Ec);
  return tot / n * 1e3;
}
