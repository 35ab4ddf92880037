// Per-CU load throughput for L2-resident data: every block streams the same
// `bytes`-sized buffer `reps` times with 16-byte loads (mode 0: to VGPRs,
// mode 1: LDS-DMA).  Prints aggregate GB/s.  Development probe, not product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
typedef __attribute__((address_space(3))) void* lds_as_ptr;
typedef const __attribute__((address_space(1))) void* gbl_as_ptr;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ src, int64_t n16, int reps,
                                                uint32_t* out) {
  __shared__ __attribute__((aligned(16))) u32x4 lds[4 * 256];
  u32x4 acc = {0, 0, 0, 0};
  const int t = threadIdx.x, w = t >> 6;
  int64_t start = ((int64_t)blockIdx.x * 4096) & (n16 - 1);
  for (int r = 0; r < reps; ++r) {
    for (int64_t i = t; i < n16; i += 4 * 256) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        int64_t j = (start + i + u * 256) & (n16 - 1);  // n16: a power of two
        if (MODE == 0) {
          acc ^= src[j];
        } else {
          __builtin_amdgcn_global_load_lds((gbl_as_ptr)(src + j), (lds_as_ptr)(lds + u * 256 + w * 64), 16, 0, 0);
        }
      }
    }
  }
  if (MODE == 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc = lds[t];
  }
  if (acc[0] == 0x12345678u) out[0] = acc[1];
}

int main(int argc, char** argv) {
  const int64_t bytes = argc > 1 ? atoll(argv[1]) : (1 << 20);
  const int blocks = argc > 2 ? atoi(argv[2]) : 1024;
  const int reps = argc > 3 ? atoi(argv[3]) : 50;
  const int64_t n16 = bytes / 16;
  u32x4* src;
  uint32_t* out;
  hipMalloc(&src, bytes);
  hipMalloc(&out, 64);
  hipMemset(src, 1, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 2; ++mode) {
    for (int it = 0; it < 3; ++it) {
      hipEventRecord(e0);
      if (mode == 0) k_stream<0><<<blocks, 256>>>(src, n16, reps, out);
      else k_stream<1><<<blocks, 256>>>(src, n16, reps, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double tot = (double)bytes * reps * blocks;
      printf("mode %d bytes %lld blocks %d: %.3f ms, %.1f GB/s aggregate, %.1f B/clk/CU @2.4GHz\n", mode,
             (long long)bytes, blocks, ms, tot / ms / 1e6, tot / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
