// Scatter-add (GINE aggregation) layout experiments -- NOT part of the
// product library.  Built by tools/exp/build_agg_exp.sh into
// tools/exp/libagg_exp.so and driven by tools/scatter_cold.py --exp.
// Variants of k_gine_agg_fwd (molclr_amd/csrc/aggregate.hip) to find what
// bounds it on cold inputs: the copy floor, more units in flight per thread,
// non-temporal output stores, a persistent grid with the next slot prefetched.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "molclr.h"
#include "../../molclr_amd/csrc/common.h"

namespace {
constexpr int kT = 256;
__device__ __forceinline__ uint32_t deg_of(uint32_t w0) { return w0 >> 29; }
__device__ __forceinline__ int32_t node_of(uint32_t w) { return (int32_t)(w & 0xFFFFFFu); }
__device__ __forceinline__ int ec_of(uint32_t w) { return (int)((w >> 24) & 15u); }

template <bool NT>
__device__ __forceinline__ void store4(float4* p, float4 v) {
  if constexpr (NT) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
  } else {
    *p = v;
  }
}

__device__ __forceinline__ float4 agg_unit(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                           const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                           const float4* __restrict__ Ec, uint4 s, int64_t t, int64_t i,
                                           int c, int d4) {
  auto msg = [&](uint32_t w) { return f4add(x[(int64_t)node_of(w) * d4 + c], Ec[ec_of(w) * d4 + c]); };
  const float4 self = x[t];
  const float4 es = Ec[12 * d4 + c];
  const uint32_t deg = deg_of(s.x);
  float4 acc = f4zero();
  if (deg <= 4) {
    const float4 m0 = deg > 0 ? msg(s.x) : acc;
    const float4 m1 = deg > 1 ? msg(s.y) : acc;
    const float4 m2 = deg > 2 ? msg(s.z) : acc;
    const float4 m3 = deg > 3 ? msg(s.w) : acc;
    if (deg > 0) acc = f4add(acc, m0);
    if (deg > 1) acc = f4add(acc, m1);
    if (deg > 2) acc = f4add(acc, m2);
    if (deg > 3) acc = f4add(acc, m3);
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k) {
      const int code = ecode[k];
      acc = f4add(acc, f4add(x[(int64_t)col[k] * d4 + c], Ec[MOLCLR_ECOMB(code) * d4 + c]));
    }
  }
  return f4add(acc, f4add(self, es));
}

// Branch-free common path: the four slot gathers are issued unconditionally
// (an empty slot reads the node's own row, already being loaded) and their
// adds are selected, so the loads of several units can overlap; degree > 4
// rows take the CSR loop.  Same adds in the same order: bit-identical.
__device__ __forceinline__ float4 agg_unit_bf(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                              const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                              const float4* __restrict__ Ec, uint4 s, int64_t t, int64_t i,
                                              int c, int d4) {
  const uint32_t deg = deg_of(s.x);
  const float4 self = x[t];
  const float4 es = Ec[MOLCLR_SELF_LOOP_ECOMB * d4 + c];
  float4 acc = f4zero();
  if (deg <= 4) {
    auto node = [&](uint32_t w, uint32_t k) { return deg > k ? (int64_t)node_of(w) : i; };
    auto ec = [&](uint32_t w, uint32_t k) { return deg > k ? ec_of(w) : MOLCLR_SELF_LOOP_ECOMB; };
    const float4 x0 = x[node(s.x, 0) * d4 + c], x1 = x[node(s.y, 1) * d4 + c];
    const float4 x2 = x[node(s.z, 2) * d4 + c], x3 = x[node(s.w, 3) * d4 + c];
    const float4 e0 = Ec[ec(s.x, 0) * d4 + c], e1 = Ec[ec(s.y, 1) * d4 + c];
    const float4 e2 = Ec[ec(s.z, 2) * d4 + c], e3 = Ec[ec(s.w, 3) * d4 + c];
    const float4 a0 = f4add(acc, f4add(x0, e0));
    acc = deg > 0 ? a0 : acc;
    const float4 a1 = f4add(acc, f4add(x1, e1));
    acc = deg > 1 ? a1 : acc;
    const float4 a2 = f4add(acc, f4add(x2, e2));
    acc = deg > 2 ? a2 : acc;
    const float4 a3 = f4add(acc, f4add(x3, e3));
    acc = deg > 3 ? a3 : acc;
  } else {
    for (int32_t k = rowptr[i], e = rowptr[i + 1]; k < e; ++k) {
      const int code = ecode[k];
      acc = f4add(acc, f4add(x[(int64_t)col[k] * d4 + c], Ec[MOLCLR_ECOMB(code) * d4 + c]));
    }
  }
  return f4add(acc, f4add(self, es));
}

template <int U, bool NT>
__global__ __launch_bounds__(kT) void k_agg_bf(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                              const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                              const uint4* __restrict__ nbr, const float4* __restrict__ Ec,
                                              float4* __restrict__ out, int64_t N, int d4) {
  const int64_t total = N * d4;
  const int64_t base = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * kT * U + threadIdx.x;
  uint4 s[U];
  int64_t tt[U], ii[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    tt[u] = base + u * kT;
    const int64_t tc = tt[u] < total ? tt[u] : total - 1;
    ii[u] = tc / d4;
    s[u] = nbr[ii[u]];
  }
  float4 r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t tc = tt[u] < total ? tt[u] : total - 1;
    r[u] = agg_unit_bf(x, rowptr, col, ecode, Ec, s[u], tc, ii[u], (int)(tc - ii[u] * d4), d4);
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (tt[u] < total) store4<NT>(out + tt[u], r[u]);
}

// V: 0 product structure, 1 copy floor, 2 two units per thread, 3 product +
// non-temporal store, 5 product without the XCD remap, 6 empty (launch floor)
template <int V, int BS = kT>
__global__ __launch_bounds__(BS) void k_agg_v(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                             const uint4* __restrict__ nbr, const float4* __restrict__ Ec,
                                             float4* __restrict__ out, int64_t N, int d4) {
  const int bid = V == 5 ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int64_t total = N * d4;
  if constexpr (V == 6) {
    return;
  } else if constexpr (V == 2) {
    const int64_t half = (total + 1) / 2;
    const int64_t t0 = (int64_t)bid * BS + threadIdx.x;
    if (t0 >= half) return;
    const int64_t t1 = t0 + half;
    const bool has1 = t1 < total;
    const int64_t i0 = t0 / d4, i1 = has1 ? t1 / d4 : i0;
    const uint4 s0 = nbr[i0], s1 = nbr[i1];
    const float4 a0 = agg_unit(x, rowptr, col, ecode, Ec, s0, t0, i0, (int)(t0 - i0 * d4), d4);
    if (has1) {
      const float4 a1 = agg_unit(x, rowptr, col, ecode, Ec, s1, t1, i1, (int)(t1 - i1 * d4), d4);
      out[t1] = a1;
    }
    out[t0] = a0;
  } else {
    const int64_t t = (int64_t)bid * BS + threadIdx.x;
    if (t >= total) return;
    if constexpr (V == 1) {
      out[t] = x[t];
    } else {
      const int64_t i = t / d4;
      const int c = (int)(t - i * d4);
      const float4 a = agg_unit(x, rowptr, col, ecode, Ec, nbr[i], t, i, c, d4);
      store4<V == 3>(out + t, a);
    }
  }
}

// persistent: each thread walks units t, t + G, ... with the next unit's
// slot word loaded before the current unit's gathers
__global__ __launch_bounds__(kT) void k_agg_persist(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                                   const uint4* __restrict__ nbr, const float4* __restrict__ Ec,
                                                   float4* __restrict__ out, int64_t N, int d4) {
  const int64_t total = N * d4;
  const int64_t G = (int64_t)gridDim.x * kT;
  int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * kT + threadIdx.x;
  if (t >= total) return;
  int64_t i = t / d4;
  uint4 s = nbr[i];
  while (t < total) {
    const int64_t tn = t + G;
    const int64_t in = tn < total ? tn / d4 : i;
    const uint4 sn = nbr[in];
    out[t] = agg_unit(x, rowptr, col, ecode, Ec, s, t, i, (int)(t - i * d4), d4);
    t = tn;
    i = in;
    s = sn;
  }
}
// chunked persistent: block b (XCD-remapped) owns the contiguous unit range
// [b * per, (b + 1) * per); its threads walk it in strides of kT with the
// next unit's slot word (and, COPY: the next unit) loaded before the current
// unit's gathers.  COPY: the copy floor of the same structure.
template <bool COPY, bool NT>
__global__ __launch_bounds__(kT) void k_agg_chunk(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ col, const uint8_t* __restrict__ ecode,
                                                 const uint4* __restrict__ nbr, const float4* __restrict__ Ec,
                                                 float4* __restrict__ out, int64_t N, int d4) {
  const int64_t total = N * d4;
  const int64_t per = (total + gridDim.x - 1) / gridDim.x;
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t beg = b * per;
  int64_t end = beg + per;
  if (end > total) end = total;
  int64_t t = beg + threadIdx.x;
  if (t >= end) return;
  if constexpr (COPY) {
    float4 v = x[t];
    while (t < end) {
      const int64_t tn = t + kT;
      const float4 vn = tn < end ? x[tn] : v;
      store4<NT>(out + t, v);
      v = vn;
      t = tn;
    }
  } else {
    int64_t i = t / d4;
    uint4 s = nbr[i];
    while (t < end) {
      const int64_t tn = t + kT;
      const int64_t in = tn < end ? tn / d4 : i;
      const uint4 sn = nbr[in];
      store4<NT>(out + t, agg_unit(x, rowptr, col, ecode, Ec, s, t, i, (int)(t - i * d4), d4));
      t = tn;
      i = in;
      s = sn;
    }
  }
}
}  // namespace

extern "C" int agg_exp(int v, const float* x, const int32_t* rowptr, const int32_t* col, const uint8_t* ecode,
                       const uint32_t* nbr, const float* Ec, float* out, int64_t N, int64_t D, int blocks_per_cu,
                       hipStream_t stream) {
  const int d4 = (int)(D / 4);
  const int64_t total = N * d4;
  const int grid = (int)((total + kT - 1) / kT);
  auto args = [&](auto k, int g, int bs = kT) {
    hipLaunchKernelGGL(k, dim3(g), dim3(bs), 0, stream, (const float4*)x, rowptr, col, ecode, (const uint4*)nbr,
                       (const float4*)Ec, (float4*)out, N, d4);
  };
  switch (v) {
    case 0: args(k_agg_v<0>, grid); break;
    case 1: args(k_agg_v<1>, grid); break;
    case 2: args(k_agg_v<2>, (int)(((total + 1) / 2 + kT - 1) / kT)); break;
    case 3: args(k_agg_v<3>, grid); break;
    case 4: {
      const int g = 256 * blocks_per_cu;
      args(k_agg_persist, g < grid ? g : grid);
      break;
    }
    case 5: args(k_agg_v<5>, grid); break;
    case 6: args(k_agg_v<6>, grid); break;
    case 7: args(k_agg_bf<1, false>, grid); break;
    case 8: args(k_agg_bf<2, false>, (int)((total + 2 * kT - 1) / (2 * kT))); break;
    case 9: args(k_agg_bf<1, true>, grid); break;
    case 40: args(k_agg_bf<2, true>, (int)((total + 2 * kT - 1) / (2 * kT))); break;
    case 41: args(k_agg_bf<4, true>, (int)((total + 4 * kT - 1) / (4 * kT))); break;
    // block-size variants: 10 + V (512 threads), 20 + V (1024 threads)
    case 10: args(k_agg_v<0, 512>, (int)((total + 511) / 512), 512); break;
    case 11: args(k_agg_v<1, 512>, (int)((total + 511) / 512), 512); break;
    case 13: args(k_agg_v<3, 512>, (int)((total + 511) / 512), 512); break;
    case 16: args(k_agg_v<6, 512>, (int)((total + 511) / 512), 512); break;
    case 20: args(k_agg_v<0, 1024>, (int)((total + 1023) / 1024), 1024); break;
    case 21: args(k_agg_v<1, 1024>, (int)((total + 1023) / 1024), 1024); break;
    case 23: args(k_agg_v<3, 1024>, (int)((total + 1023) / 1024), 1024); break;
    case 26: args(k_agg_v<6, 1024>, (int)((total + 1023) / 1024), 1024); break;
    case 30: args(k_agg_v<0, 128>, (int)((total + 127) / 128), 128); break;
    case 50: args(k_agg_chunk<false, false>, 256 * blocks_per_cu); break;
    case 51: args(k_agg_chunk<true, false>, 256 * blocks_per_cu); break;
    case 52: args(k_agg_chunk<false, true>, 256 * blocks_per_cu); break;
    case 53: args(k_agg_chunk<true, true>, 256 * blocks_per_cu); break;
    case 33: args(k_agg_v<3, 128>, (int)((total + 127) / 128), 128); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
