// Shared helpers for the MolCLR gfx950 kernels (see include/molclr.h for the ABI).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>
#include <stddef.h>

#include "../../include/molclr.h"

#define MOLCLR_API extern "C" __attribute__((visibility("default")))

namespace molclr {

// Thread-local error text for molclr_last_error().
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

inline hipStream_t as_stream(molclr_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// molclr_edge_tables_combine that also zeroes n_zero floats at `zero` in the
// same launch (the encoder executor's h3 max slots)
int edge_tables_combine_zero(int layers, const float* const* E1s, const float* const* E2s,
                             float* Ec, int64_t D, float* zero, int64_t n_zero,
                             molclr_stream_t stream);

// molclr_hplanes_make_batch of one image (B: N x K row-major, ldb = K) whose
// max launch also writes the per-tensor max slot of a second dense fp32
// matrix x (n4 float4s) into `x_slot` (NT-Xent's rows and columns, one launch)
int hplanes_make_and_max(const float* B, int64_t N, int64_t K, uint16_t* planes, const float* x,
                         int64_t x_rows, int64_t x_cols, float* x_slot, hipStream_t stream);

// Compute units of the current device (cached per device): the grid of a
// persistent kernel.
inline int cu_count() {
  static int cached[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Carves sub-buffers out of a caller-provided workspace, 256-byte aligned.
struct Workspace {
  char* base;
  size_t size;
  size_t used = 0;
  Workspace(void* p, size_t n) : base(static_cast<char*>(p)), size(n) {}
  template <typename T>
  T* take(size_t count) {
    used = align_up(used, 256);
    T* p = reinterpret_cast<T*>(base + used);
    used += count * sizeof(T);
    return p;
  }
  bool ok() const { return used <= size && (used == 0 || base != nullptr); }
};

// Row-band geometry for [rows, D] kernels that own one float4 column per thread:
// a block covers `band` consecutive rows x all D/4 float4 columns, so each
// wave reads contiguous 1 KiB of the row-major matrix (rows are contiguous).
struct Band {
  int d4;       // float4 columns
  int band;     // rows per block iteration
  int threads;  // band * d4, rounded up to a multiple of 64
};
inline Band make_band(int64_t dim) {
  Band b;
  b.d4 = (int)(dim / 4);
  int band = 256 / b.d4;
  if (band < 1) band = 1;
  if (band * b.d4 < 192 && (band + 1) * b.d4 <= 1024) band += 1;
  while (band * b.d4 > 1024) band--;
  b.band = band;
  b.threads = (band * b.d4 + 63) / 64 * 64;
  return b;
}

// Opt-in per-launch kernel timer (molclr_ktimer_*; benchmarks only).  A timed
// launch goes through hipExtLaunchKernelGGL, whose start/stop events are
// written by the kernel dispatch itself: the elapsed time is the kernel's own
// execution window (what rocprofv3's kernel trace reports), not a bracket of
// separately queued event packets.
enum {
  kTimeGineAgg = MOLCLR_KTIMER_GINE_AGG,
  kTimeGemm = MOLCLR_KTIMER_GEMM,
  kTimeNtxent = MOLCLR_KTIMER_NTXENT,
  kTimeGcnAgg = MOLCLR_KTIMER_GCN_AGG
};
bool timer_wants(int kind);
void timer_record(int kind, hipEvent_t start, hipEvent_t stop);
// Launches made while a TimerKindScope is alive on the calling thread are
// attributed to its kind (NT-Xent's internal GEMMs count as NT-Xent time).
int& timer_kind_override();
struct TimerKindScope {
  int prev;
  explicit TimerKindScope(int kind) : prev(timer_kind_override()) { timer_kind_override() = kind; }
  ~TimerKindScope() { timer_kind_override() = prev; }
};

template <typename... Args, typename F = void (*)(Args...)>
void launch_timed(int kind, F kernel, dim3 grid, dim3 block, uint32_t shmem,
                  hipStream_t stream, Args... args) {
  if (timer_kind_override()) kind = timer_kind_override();
  if (timer_wants(kind)) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, e0, e1, 0u, args...);
      timer_record(kind, e0, e1);
      return;
    }
  }
  hipLaunchKernelGGL(kernel, grid, block, shmem, stream, args...);
}

// Zeroing and device-to-device copies as KERNELS, never hipMemsetAsync /
// hipMemcpyAsync: the library's steps are captured into HIP graphs, and a
// memset node that follows a kernel node in a captured graph was measured
// not to take effect on replays (tools/capture_memset_probe3.py: the region
// kept the value written before the replay in 299 of 300 replays, on this
// ROCm 7.0 runtime) -- which left the h3 max slots holding stale values and,
// on fresh pool memory, HBM garbage (zero MLP weight gradients).
namespace detail {
__global__ __launch_bounds__(256) static void k_fill_bytes(uint8_t* __restrict__ p, size_t n,
                                                           uint8_t v) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n16 = (reinterpret_cast<uintptr_t>(p) & 15) == 0 ? n / 16 : 0;
  const uint32_t w = 0x01010101u * v;
  for (size_t i = t; i < n16; i += stride)
    reinterpret_cast<uint4*>(p)[i] = make_uint4(w, w, w, w);
  for (size_t i = 16 * n16 + t; i < n; i += stride) p[i] = v;
}
__global__ __launch_bounds__(256) static void k_copy_bytes(uint8_t* __restrict__ d,
                                                           const uint8_t* __restrict__ s,
                                                           size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool al = ((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 15) == 0;
  const size_t n16 = al ? n / 16 : 0;
  for (size_t i = t; i < n16; i += stride)
    reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
  for (size_t i = 16 * n16 + t; i < n; i += stride) d[i] = s[i];
}
inline unsigned fill_blocks(size_t n) {
  const size_t b = (n / 16 + 255) / 256;
  return (unsigned)(b < 1 ? 1 : b > 2048 ? 2048 : b);
}
}  // namespace detail

// memset(p, v, bytes) on `s` as a kernel (capturable); hipSuccess or the launch error
inline hipError_t fill_async(void* p, int v, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  hipLaunchKernelGGL(detail::k_fill_bytes, dim3(detail::fill_blocks(bytes)), dim3(256), 0, s,
                     static_cast<uint8_t*>(p), bytes, (uint8_t)v);
  return hipGetLastError();
}
inline hipError_t zero_async(void* p, size_t bytes, hipStream_t s) {
  return fill_async(p, 0, bytes, s);
}
// device-to-device memcpy on `s` as a kernel (capturable)
inline hipError_t copy_async(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  hipLaunchKernelGGL(detail::k_copy_bytes, dim3(detail::fill_blocks(bytes)), dim3(256), 0, s,
                     static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), bytes);
  return hipGetLastError();
}

}  // namespace molclr

// norm.hip: BatchNorm workspace for any split of `rows` into segments
size_t molclr_batchnorm_ws_bound(int64_t rows, int64_t D);

#define MOLCLR_REQUIRE(cond, ...)        \
  do {                                   \
    if (!(cond)) {                       \
      molclr::set_error(__VA_ARGS__);    \
      return MOLCLR_ERR_ARG;             \
    }                                    \
  } while (0)

#define MOLCLR_REQUIRE_WS(ws, need)                                                   \
  do {                                                                                \
    if ((ws) < (need)) {                                                              \
      molclr::set_error("%s: workspace %zu bytes < required %zu", __func__,           \
                        (size_t)(ws), (size_t)(need));                                \
      return MOLCLR_ERR_WORKSPACE;                                                    \
    }                                                                                 \
  } while (0)

// return a non-zero status of a nested entry-point call
#define MOLCLR_TRY_RC(expr)   \
  do {                        \
    int rc_ = (expr);         \
    if (rc_) return rc_;      \
  } while (0)

#define MOLCLR_LAUNCHED()                                                             \
  do {                                                                                \
    hipError_t e_ = hipGetLastError();                                                \
    if (e_ != hipSuccess) {                                                           \
      molclr::set_error("%s: launch failed: %s", __func__, hipGetErrorString(e_));    \
      return (int)e_;                                                                 \
    }                                                                                 \
  } while (0)

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
// Workgroups are dealt round-robin to the 8 XCDs (bid % 8), each with its own
// L2.  Remapping so XCD x runs a contiguous range of logical blocks keeps
// neighbouring rows -- e.g. the atoms of one molecule that gather each other's
// features -- inside one L2 instead of fetching every row into several.
// Bijective for any nwg.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  int q = nwg / 8, r = nwg % 8;
  int x = bid % 8, pos = bid / 8;
  int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + pos;
}

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// LDS written by this wave, then read back by it (a wave-private tile): order
// the wave's own accesses, no block barrier
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------
// Storage types of node-feature matrices.  Kernels over [rows, D] matrices are
// templated on one of these: a "column unit" is 4 consecutive elements, read
// and written as a float4 of fp32 values (fp32 storage: one 16-byte access;
// bf16 storage: one 8-byte access, widened / rounded to nearest even).  All
// arithmetic stays fp32 (the c5 configuration's bf16 storage, fp32 math).
// ---------------------------------------------------------------------------
struct StF32 {
  typedef float T;
  static constexpr int kBytes = 4;
  __device__ __forceinline__ static float4 ld(const T* __restrict__ p, int64_t unit) {
    return reinterpret_cast<const float4*>(p)[unit];
  }
  __device__ __forceinline__ static void st(T* __restrict__ p, int64_t unit, float4 v) {
    reinterpret_cast<float4*>(p)[unit] = v;
  }
  __device__ __forceinline__ static void ld2(const T* __restrict__ p, int64_t u2, float4& a,
                                             float4& b) {
    a = reinterpret_cast<const float4*>(p)[2 * u2];
    b = reinterpret_cast<const float4*>(p)[2 * u2 + 1];
  }
  __device__ __forceinline__ static void st2(T* __restrict__ p, int64_t u2, float4 a, float4 b) {
    reinterpret_cast<float4*>(p)[2 * u2] = a;
    reinterpret_cast<float4*>(p)[2 * u2 + 1] = b;
  }
  __device__ __forceinline__ static float ld1(const T* __restrict__ p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void st1(T* __restrict__ p, int64_t i, float v) { p[i] = v; }
};

__device__ __forceinline__ float bf16_to_f32(uint32_t bits16) {
  return __uint_as_float(bits16 << 16);
}
// round to nearest even (v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ uint32_t f32x2_to_bf16x2(float a, float b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const bf2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

struct StBF16 {
  typedef uint16_t T;
  static constexpr int kBytes = 2;
  __device__ __forceinline__ static float4 ld(const T* __restrict__ p, int64_t unit) {
    const uint2 u = reinterpret_cast<const uint2*>(p)[unit];
    return make_float4(bf16_to_f32(u.x & 0xFFFFu), bf16_to_f32(u.x >> 16),
                       bf16_to_f32(u.y & 0xFFFFu), bf16_to_f32(u.y >> 16));
  }
  __device__ __forceinline__ static void st(T* __restrict__ p, int64_t unit, float4 v) {
    reinterpret_cast<uint2*>(p)[unit] = make_uint2(f32x2_to_bf16x2(v.x, v.y), f32x2_to_bf16x2(v.z, v.w));
  }
  // units 2 u2 and 2 u2 + 1 as one 16-byte access
  __device__ __forceinline__ static void ld2(const T* __restrict__ p, int64_t u2, float4& a,
                                             float4& b) {
    const uint4 q = reinterpret_cast<const uint4*>(p)[u2];
    a = make_float4(bf16_to_f32(q.x & 0xFFFFu), bf16_to_f32(q.x >> 16), bf16_to_f32(q.y & 0xFFFFu),
                    bf16_to_f32(q.y >> 16));
    b = make_float4(bf16_to_f32(q.z & 0xFFFFu), bf16_to_f32(q.z >> 16), bf16_to_f32(q.w & 0xFFFFu),
                    bf16_to_f32(q.w >> 16));
  }
  __device__ __forceinline__ static void st2(T* __restrict__ p, int64_t u2, float4 a, float4 b) {
    reinterpret_cast<uint4*>(p)[u2] = make_uint4(f32x2_to_bf16x2(a.x, a.y), f32x2_to_bf16x2(a.z, a.w),
                                                 f32x2_to_bf16x2(b.x, b.y), f32x2_to_bf16x2(b.z, b.w));
  }
  __device__ __forceinline__ static float ld1(const T* __restrict__ p, int64_t i) {
    return bf16_to_f32(p[i]);
  }
  __device__ __forceinline__ static void st1(T* __restrict__ p, int64_t i, float v) {
    p[i] = (uint16_t)(f32x2_to_bf16x2(v, 0.f) & 0xFFFFu);
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// max over the wave of v >= 0 by DPP within rows of 16 and four lane reads
// (no LDS crossbar traffic; every lane gets the result)
__device__ __forceinline__ float wave_max_dpp(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value,
                                                      0xF, 0xF, false));
  };
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0xB1>{}));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x4E>{}));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x140>{}));  // row_mirror
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(a, b), fmaxf(c, d));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Row maxima of a row-major [rows][d4] float4 tensor written by one thread per
// float4 (t = row * d4 + c, blocks of whole waves): a row's float4s are
// contiguous lanes spread over at most `nparts` waves; each wave's piece of a
// row is reduced by a segmented shuffle and its first lane stores the piece's
// max as rowparts[part][row], part = its wave - the row's first wave (plain
// stores, no atomics; the row max is the max over parts).  The writer of part
// 0 zeroes the parts the row does not reach.  m = this lane's max |.|, row =
// -1 for a lane past the end.  Every lane of the wave must call it.
__device__ __forceinline__ void row_max_parts(float m, int row, int64_t t, int64_t rows, int d4,
                                              float* __restrict__ rowparts, int nparts) {
  const int lane = threadIdx.x & 63;
  if (d4 >= 64) {
    // a wave holds pieces of at most two rows, r0 (its first lane's) and r0 + 1:
    // two plain wave maxima instead of the segmented scan
    const int64_t t0 = t - lane;
    const int64_t r0 = rows * d4 < (1ll << 32) ? (int64_t)((uint32_t)t0 / (uint32_t)d4) : t0 / d4;
    const bool second = row >= 0 && row != r0;
    const float m0 = wave_max_dpp(second ? 0.f : m), m1 = wave_max_dpp(second ? m : 0.f);
    if (lane == 0 && r0 < rows) {
      const int64_t rs = r0 * d4;
      const int part = (int)((t0 >> 6) - (rs >> 6));
      rowparts[part * rows + r0] = m0;
      if (part == 0)
        for (int q = (int)(((rs + d4 - 1) >> 6) - (rs >> 6)) + 1; q < nparts; ++q)
          rowparts[q * rows + r0] = 0.f;
    }
    const int64_t r1 = r0 + 1, rs1 = r1 * d4;
    if (lane == 1 && r1 < rows && rs1 < t0 + 64) {  // r1 starts in this wave: part 0
      rowparts[r1] = m1;
      for (int q = (int)(((rs1 + d4 - 1) >> 6) - (rs1 >> 6)) + 1; q < nparts; ++q)
        rowparts[q * rows + r1] = 0.f;
    }
    return;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float mv = __shfl_down(m, off, 64);
    const int rv = __shfl_down(row, off, 64);
    if (lane + off < 64 && rv == row) m = fmaxf(m, mv);
  }
  const int rp = __shfl_up(row, 1, 64);
  if (row >= 0 && (lane == 0 || rp != row)) {
    const int64_t rs = (int64_t)row * d4;  // the row's first float4
    const int part = (int)((t >> 6) - (rs >> 6));
    rowparts[part * rows + row] = m;
    if (part == 0)  // parts this row does not reach
      for (int q = (int)(((rs + d4 - 1) >> 6) - (rs >> 6)) + 1; q < nparts; ++q)
        rowparts[q * rows + row] = 0.f;
  }
}

// Row maxima as per-wave pairs (rows of d4 >= 64 float4s, one thread per
// float4 as row_max_parts): a wave holds pieces of at most two rows, r0 (its
// first lane's) and r0 + 1, and its lane 0 stores the two pieces' maxima as
// one float2 wm[wave] -- one 8-byte store per wave, consecutive across waves
// (row_max_parts' scattered 4-byte stores and zero fills cost the
// aggregation ~2 us).  row_max_of_waves folds a row's pieces back.
__device__ __forceinline__ void row_max_waves(float m, int row, int64_t t, int64_t rows, int d4,
                                              float2* __restrict__ wm) {
  const int lane = threadIdx.x & 63;
  const int64_t t0 = t - lane;
  const int64_t r0 = rows * d4 < (1ll << 32) ? (int64_t)((uint32_t)t0 / (uint32_t)d4) : t0 / d4;
  const bool second = row >= 0 && row != r0;
  const float m0 = wave_max_dpp(second ? 0.f : m), m1 = wave_max_dpp(second ? m : 0.f);
  if (lane == 0 && t0 < rows * d4) wm[t0 >> 6] = make_float2(m0, m1);
}
__device__ __forceinline__ float row_max_of_waves(const float2* __restrict__ wm, int64_t row,
                                                  int d4) {
  const int64_t s = row * d4, e = s + d4 - 1;
  float m = 0.f;
  for (int64_t w = s >> 6; w <= (e >> 6); ++w) {
    const float2 v = wm[w];
    // w's first row is `row` iff the wave starts inside it: w's units begin at
    // 64 w <= e (w <= e >> 6), so floor(64 w / d4) == row iff 64 w >= s
    m = fmaxf(m, (w << 6) >= s ? v.x : v.y);
  }
  return m;
}

// A tensor's max |x| "slot" (molclr_absmax_f32) is kMaxSlotParts entries, each
// on its own 128-byte line, whose max is the value: producers spread their
// atomics over the entries (atomics on one line serialise: thousands of them
// on one or two lines cost tens of microseconds), consumers fold all entries.
constexpr int kMaxSlotParts = 64;
constexpr int kMaxSlotStride = 32;  // floats: each entry on its own 128-byte line
constexpr int kMaxSlotFloats = kMaxSlotParts * kMaxSlotStride;

// Folds a lane's max |x| (v >= 0) into a slot: block max through LDS, then one
// global atomic max on the float's bits (ordered like the values for v >= 0)
// into entry blockIdx.x % 64.  Every thread of the block must call it (a
// block barrier inside).
// max |x| over float4 elements t, t + stride, ... < n4 with eight independent
// loads in flight per lane (a dependent one-load loop over a few blocks is
// latency-bound: 8 MB took 48 us)
__device__ __forceinline__ float absmax4_range(const float4* __restrict__ x, int64_t t, int64_t n4,
                                               int64_t stride) {
  auto amax4 = [](float4 v) {
    return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
  };
  float m = 0.f;
  for (; t + 7 * stride < n4; t += 8 * stride) {
    float4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[t + j * stride];
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, amax4(v[j]));
  }
  for (; t < n4; t += stride) m = fmaxf(m, amax4(x[t]));
  return m;
}

// block max of v (blockDim a multiple of 64, <= 1024), valid in thread 0
__device__ __forceinline__ float block_max(float v) {
  __shared__ float red_b[16];
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red_b[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) v = fmaxf(v, red_b[w]);
  return v;
}

__device__ __forceinline__ void absmax_publish(float v, float* slot) {
  __shared__ float red_[16];
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red_[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)((blockDim.x + 63) >> 6); ++w) v = fmaxf(v, red_[w]);
    atomicMax(reinterpret_cast<unsigned int*>(slot + (blockIdx.x % kMaxSlotParts) * kMaxSlotStride),
              __float_as_uint(v));
  }
  __syncthreads();  // red_ is reused by the block's next call
}
