// Shared device helpers for the fmdiff gfx950 (MI355X / CDNA4) kernels.
// Activations are NHWC bf16 ("pixel rows, channels contiguous"), statistics and
// accumulators fp32.  Wave = 64 lanes; MFMA = v_mfma_f32_16x16x32_bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FMD_DEV __device__ __forceinline__
#define FMD_HD __host__ __device__ __forceinline__

typedef uint16_t bf16r;                                           // raw bf16 bits in memory
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;        // MFMA A/B fragment (4 VGPR)
typedef __attribute__((ext_vector_type(4))) float f32x4;          // MFMA 16x16 accumulator
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;   // 16-byte vector
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;   // 8-byte vector
typedef __attribute__((ext_vector_type(4))) short s16x4;          // ds_read_tr16_b64 result

FMD_DEV float bf2f(unsigned int raw16) { return __uint_as_float(raw16 << 16); }
FMD_DEV float bf_lo(unsigned int w) { return __uint_as_float(w << 16); }
FMD_DEV float bf_hi(unsigned int w) { return __uint_as_float(w & 0xffff0000u); }

// round-to-nearest-even fp32 -> bf16 (hipcc emits v_cvt_pk_bf16_f32; keeps NaN a NaN)
FMD_DEV unsigned int f2bf(float f) {
  __bf16 b = (__bf16)f;
  return (unsigned int)__builtin_bit_cast(unsigned short, b);
}
// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (the f2bf(lo) | f2bf(hi) << 16 form compiles to two
// single-operand converts + shift + or)
typedef __attribute__((ext_vector_type(2))) float f32x2_;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_;
FMD_DEV unsigned int pack2(float lo, float hi) {
  return __builtin_bit_cast(unsigned int, __builtin_convertvector(f32x2_{lo, hi}, bf16x2_));
}

// v_exp_f32 + v_rcp_f32 (1 ulp): no IEEE division sequence in the hot prologues
FMD_DEV float sigmoidf_(float z) { return __builtin_amdgcn_rcpf(1.0f + __expf(-z)); }
FMD_DEV float siluf_(float z) { return z * sigmoidf_(z); }
// d silu / dz
FMD_DEV float silu_grad(float z) {
  float s = sigmoidf_(z);
  return s * (1.0f + z * (1.0f - s));
}

FMD_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
// gfx950 ds_read_b64_tr_b16: 16-lane group reads a 4-row x 16-col bf16 block;
// lane 4q+p supplies &T[row q][col 4p], lane i receives column i (rows 0..3).
FMD_DEV s16x4 ds_read_tr16(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_ptr));
}

// Sum over each 16-lane row with DPP row shifts (VALU, no LDS crossbar): lane 15 of every row
// receives the row's total (other lanes hold partial prefix sums).
FMD_DEV float row16_sum_to_last(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

FMD_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// XCD-aware bijective block remap: blocks b, b+8, ... share one XCD's L2; give
// each XCD a contiguous range of the logical grid (cdna_hip_programming.md T1).
FMD_DEV int xcd_remap(int b, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = b & 7, k = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// 16-byte LDS-DMA (global_load_lds_dwordx4) issued through inline asm: hipcc neither counts it nor
// makes later ds_reads wait for it (its builtin form drains vmcnt before every following LDS read),
// so the pipeline's own counted waits in step_barrier() are the only ones.  lds_dst: wave-uniform
// LDS byte address; lane i lands at lds_dst + 16 i.
// Scalar-base form: lane address = sbase + voff (a fixed 32-bit per-lane byte offset, "saddr" addressing), so
// a stream whose lanes always fetch the same offsets of consecutive blocks needs no per-DMA vector arithmetic.
FMD_DEV void glds16s(const void* sbase_, unsigned voff, unsigned lds_dst) {
  const unsigned long long sb = (unsigned long long)sbase_;   // wave-uniform: pinned to SGPRs for the "s" operand
  const void* sbase = (const void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(sb >> 32)) << 32) |
                                    (unsigned)__builtin_amdgcn_readfirstlane((unsigned)sb));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_dst) : "memory");
}
FMD_DEV void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
// The 4-byte form (lane i lands at lds_dst + 4 i): 4-byte-aligned sources such as parameter views.
FMD_DEV void glds4(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

