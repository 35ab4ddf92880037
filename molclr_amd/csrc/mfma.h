// MFMA operand helpers shared by the GEMM kernels (gemm.hip: split-bf16 fp32
// GEMMs; gemm_bf16.hip: the native bf16 GEMMs of the c5 configuration).
//
// v_mfma_f32_32x32x16_bf16: lane l (r = l & 31, h = l >> 5) holds A[row r][k =
// 8h + j] and B[k = 8h + j][col r] in element j = 0..7 of its fragment; the
// 32 x 32 fp32 result has its column on the lane and rows (reg & 3) +
// 8 (reg >> 2) + 4 h in the 16 registers.
#pragma once

#include "common.h"

namespace molclr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// LDS-DMA operands of __builtin_amdgcn_global_load_lds
typedef __attribute__((address_space(3))) void* lds_as_ptr;
typedef const __attribute__((address_space(1))) void* gbl_as_ptr;

constexpr int BK = 32;  // K per staged slice
constexpr int XK = 32;  // bf16 per [row][k] image row (64 B, unpadded, chunk-swizzled)

// [row][k] images: bf16 offset of k = 8 * chunk in image row `row`; the four
// 16-byte chunks of a row are XOR-swizzled by (row >> 2) & 3, so a lane's
// 8 consecutive k of one row (one MFMA fragment) are one ds_read_b128,
// conflict-free over every 16-lane group, with no padding.
__device__ __forceinline__ int xoff(int row, int chunk) {
  return row * XK + ((chunk ^ ((row >> 2) & 3)) << 3);
}

__device__ __forceinline__ bf16x8 xfrag(const uint16_t* __restrict__ img, int row, int chunk) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(img + xoff(row, chunk)));
}

// Two floats -> packed hi / mid / lo bf16 pairs, each part the round-to-nearest
// bf16 of the remaining residual (v_cvt_pk_bf16_f32); both subtractions are
// exact (Sterbenz), so a = hi + mid + lo + t with |t| <= 2^-24 |a|.
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  const bf16x2 hh = {(__bf16)a, (__bf16)b};
  const float ra = a - (float)hh[0], rb = b - (float)hh[1];
  const bf16x2 mm = {(__bf16)ra, (__bf16)rb};
  const float sa = ra - (float)mm[0], sb = rb - (float)mm[1];
  const bf16x2 ll = {(__bf16)sa, (__bf16)sb};
  h = __builtin_bit_cast(uint32_t, hh);
  m = __builtin_bit_cast(uint32_t, mm);
  l = __builtin_bit_cast(uint32_t, ll);
}

__device__ __forceinline__ void split4(float4 v, uint2& hi, uint2& mid, uint2& lo) {
  split2(v.x, v.y, hi.x, mid.x, lo.x);
  split2(v.z, v.w, hi.y, mid.y, lo.y);
}

__device__ __forceinline__ void split8(const float4 a, const float4 b, u32x4& hi, u32x4& mid,
                                       u32x4& lo) {
  uint32_t h[4], m[4], l[4];
  split2(a.x, a.y, h[0], m[0], l[0]);
  split2(a.z, a.w, h[1], m[1], l[1]);
  split2(b.x, b.y, h[2], m[2], l[2]);
  split2(b.z, b.w, h[3], m[3], l[3]);
  hi = u32x4{h[0], h[1], h[2], h[3]};
  mid = u32x4{m[0], m[1], m[2], m[3]};
  lo = u32x4{l[0], l[1], l[2], l[3]};
}

// ---------------------------------------------------------------------------
// "h3": fp32 products from THREE fp16 MFMAs instead of six bf16 ones.
// An operand is scaled by a power of two 2^sh chosen from its tensor-wide
// max |x| (so the scaled max lies in [2^14, 2^15), below fp16's 65504) and
// split into hi = fp16(x 2^sh) and lo = fp16(x 2^sh - hi) (round to nearest,
// the subtraction is exact): x 2^sh = hi + lo + t with |t| <= 2^-22 |x 2^sh|
// while lo is an fp16 normal, i.e. for every element within 2^-17 of the
// tensor's max (smaller ones keep an absolute error below 2^-38 max |x|).
// hi_a hi_b + hi_a lo_b + lo_a hi_b then reproduces a b to ~3 2^-22, and the
// fp32 sums are scaled back by 2^-(sh_a + sh_b) (exact).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// Scale exponent for values of max |x| = m: 0 for a zero / NaN / infinite m
// (NaN and inf then propagate as in fp32).
// Capped at 127 (m < 2^-112: such a tensor / row keeps fewer lo bits) so that
// 2^sh is an fp32 normal and the split scales by a multiply (h3_scale).
__device__ __forceinline__ int h3_shift_of(float m) {
  if (!(m > 0.f) || !(m <= 3.402823466e38f)) return 0;
  const int sh = 15 - __builtin_amdgcn_frexp_expf(m);  // m = f 2^e, f in [0.5, 1)
  return sh < 127 ? sh : 127;
}
// 2^sh for sh in [-126, 127] (h3_shift_of's range: e <= 128 gives sh >= -113)
__device__ __forceinline__ float h3_scale(int sh) {
  return __builtin_bit_cast(float, (uint32_t)(sh + 127) << 23);
}
// ... of a tensor from its max slot (kMaxSlotParts entries, molclr_absmax_f32).
// Every lane of the wave must call it.
__device__ __forceinline__ int h3_shift(const float* __restrict__ slot) {
  return h3_shift_of(wave_max(slot[(threadIdx.x & (kMaxSlotParts - 1)) * kMaxSlotStride]));
}

// x 2^sh as a multiply by the exact power of two (the same value as ldexp),
// hi by the packed conversion, and lo = fp16(x 2^sh - hi) by one fma_mix per
// element reading hi's f16 half straight from the packed word (op_sel): the
// fma forms x 2^sh - hi exactly (a power-of-two product, an f32-exact
// difference) and rounds once to fp16 -- the value of the C expression
// (_Float16)(x 2^sh - (float)hi).  Written out because the compiler re-derives
// hi per element instead of reading the packed word: 4-5 VALU per pair
// against 7 (multiply form) and 10 (ldexp form).
__device__ __forceinline__ void hsplit2(float a, float b, int sh, uint32_t& h, uint32_t& l) {
#ifdef MOLCLR_HSPLIT_LDEXP  // the previous form, for A/B checks
  a = __builtin_ldexpf(a, sh);
  b = __builtin_ldexpf(b, sh);
  const f16x2 h2 = {(_Float16)a, (_Float16)b};
  const f16x2 l2 = {(_Float16)(a - (float)h2[0]), (_Float16)(b - (float)h2[1])};
  h = __builtin_bit_cast(uint32_t, h2);
  l = __builtin_bit_cast(uint32_t, l2);
  return;
#endif
  const float s = h3_scale(sh);
  const f16x2 hh = {(_Float16)(a * s), (_Float16)(b * s)};
  h = __builtin_bit_cast(uint32_t, hh);
  uint32_t lo;
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(lo) : "v"(a), "v"(s), "v"(h));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(lo) : "v"(b), "v"(s), "v"(h));
  l = lo;
}

__device__ __forceinline__ void hsplit4(float4 v, int sh, uint2& hi, uint2& lo) {
  hsplit2(v.x, v.y, sh, hi.x, lo.x);
  hsplit2(v.z, v.w, sh, hi.y, lo.y);
}

__device__ __forceinline__ void hsplit8(const float4 a, const float4 b, int sh, u32x4& hi,
                                        u32x4& lo) {
  uint32_t h[4], l[4];
  hsplit2(a.x, a.y, sh, h[0], l[0]);
  hsplit2(a.z, a.w, sh, h[1], l[1]);
  hsplit2(b.x, b.y, sh, h[2], l[2]);
  hsplit2(b.z, b.w, sh, h[3], l[3]);
  hi = u32x4{h[0], h[1], h[2], h[3]};
  lo = u32x4{l[0], l[1], l[2], l[3]};
}

// the three fp16 products of an (a, b) element pair, small terms first
__device__ __forceinline__ f32x16 mfma_h3(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
}
// the same three products in the same order with the operands swapped: the
// accumulator holds the transposed 32 x 32 block (lane li = row of A)
__device__ __forceinline__ f32x16 mfma_h3_t(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh, al, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(bh, ah, acc, 0, 0, 0);
}

// K-major [k][ROWS] image planes (the dY^T / X^T operands of a weight
// gradient), read with the gfx950 transposed LDS read.  32-element XOR of
// k-row k: separates the 4 k-rows one transposed read touches (64-row rows
// are 32 dwords: rows k and k+2 share banks; 128-row rows are 64 dwords: all
// four do, as on any multiple of 128 rows); 160-row rows are 80 dwords
// (16 mod 64 banks apart): no XOR.
template <int ROWS>
__device__ __forceinline__ int kswz(int k) {
  return ROWS == 64 ? ((k >> 1) & 1) << 5 : (ROWS % 128 == 0) ? (k & 3) << 5 : 0;
}

// MFMA 32x32x16 operand fragment of rows row0 .. row0+31 (lane: row row0 + li,
// k = 16 ks + 8 lh .. +7) from a [k][ROWS] K-major image plane: two transposed
// reads, each giving 4 consecutive k of one row.  Lane 4q+p of a 16-lane group
// addresses k-row q, rows 4p .. 4p+3 of the group's 16 (ISA ds_read_b64_tr_b16).
template <int ROWS>
__device__ __forceinline__ bf16x8 kmfrag(const uint16_t* __restrict__ plane, int row0, int ks,
                                         int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int m = row0 + (g & 1) * 16 + 4 * pp;
  const int k = 16 * ks + 8 * (g >> 1) + q;
  const uint16_t* a0 = plane + k * ROWS + (m ^ kswz<ROWS>(k));
  const uint16_t* a1 = plane + (k + 4) * ROWS + (m ^ kswz<ROWS>(k + 4));
  const v4i16 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a0);
  const v4i16 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a1);
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// Scheduling of one group of MFMAs: NM MFMAs with the NEXT group's NR LDS
// fragment reads threaded between them (one MFMA, then ceil(NR / NM) reads,
// ...).  The group's first MFMA then waits only for reads issued a whole
// group earlier, and the new reads' latency hides under the MFMAs -- left
// to itself the compiler issued every read of two substeps first and waited
// for all of them (s_waitcnt lgkmcnt(0)) before the first MFMA.
template <int NM, int NR, int K = 0>
__device__ __forceinline__ void interleave_mfma_reads() {
  if constexpr (K < NM) {
    constexpr int per = (NR + NM - 1) / NM;
    constexpr int left = NR - K * per;
    constexpr int n = left < per ? left : per;
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
    if constexpr (n > 0) __builtin_amdgcn_sched_group_barrier(0x100, n, 0);  // then DS reads
    interleave_mfma_reads<NM, NR, K + 1>();
  }
}

// ---------------------------------------------------------------------------
// Buffer-resource addressing (gfx9 descriptor word 3 = 0x00020000): a
// per-lane 32-bit byte offset fixed for a whole tile plus a wave-uniform
// (SGPR) offset per K step, so a main loop advances its loads with no 64-bit
// address arithmetic; reads past num_records return zeros.  Device pass only
// (the host pass compiles the launch stubs and has no AMDGPU builtins).
// ---------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int n = bytes > 0x7fffffffll ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, n, 0x00020000);
#else
  __builtin_unreachable();
#endif
}
// 16 bytes at voff + soff (soff made wave-uniform: a divergent soffset would
// turn every load into a readfirstlane loop)
__device__ __forceinline__ float4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(
      float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, __builtin_amdgcn_readfirstlane(soff), 0));
#else
  return make_float4(0.f, 0.f, 0.f, 0.f);
#endif
}
// LDS-DMA of 16 bytes per lane (buffer_load_dwordx4 ... lds) into the
// wave-uniform LDS address `lds` (+ 16 lane)
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff,
                                          uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_as_ptr)lds, 16, voff,
                                           __builtin_amdgcn_readfirstlane(soff), 0, 0);
#endif
}
// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt left at their maxima; gfx9 encoding)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// row of register r of a 32x32 MFMA accumulator, lane half lh
__device__ __forceinline__ int acc_row(int r, int lh) { return (r & 3) + 8 * (r >> 2) + 4 * lh; }

}  // namespace molclr

// split-K partial reduction of the fp32 GEMMs (gemm.hip), shared with the bf16
// weight-gradient GEMM: C (+)= Σ_{z < splits} partial[z] (fixed order), colsum
// (+)= Σ_{z < cs_splits} cs_partial[z] when cs_partial is given.
void molclr_splitk_reduce_none(const float* partial, int splits, int64_t M, int64_t N, float* C,
                               int64_t ldc, int accumulate, const float* cs_partial,
                               int cs_splits, float* colsum, hipStream_t s);
