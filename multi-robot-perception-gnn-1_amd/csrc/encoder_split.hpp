#pragma once
// encoder_split.hpp — the split-bf16 arithmetic and packed weight image of the edge encoder
// (encoder_split.hip), kept apart from its kernels so kernel-lab variants can include them.
//
// Reference (xjh19971/multi-robot-perception-gnn-1, dgl/model/models.py:146-149):
//     z = Linear(C, 2C)(ReLU(Linear(9, C)(pose)))          pose (E, 9) -> z (E, 2C)
// Arithmetic: encoder_split.hip's header.

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mrp_x6 {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

constexpr int kNin = 9;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));

// two fp32 -> two bf16 (round to nearest even) in one dword: v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t cvt2(f2 x) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf2)); }
// ... and back to fp32 (exact)
__device__ __forceinline__ f2 widen2(uint32_t p) {
  f2 r;
  r.x = __uint_as_float(p << 16);
  r.y = __uint_as_float(p & 0xffff0000u);
  return r;
}

// The three bf16 parts of 8 fp32 values (exact split, see above), pairwise: one v_cvt_pk_bf16_f32 and
// one v_pk_add_f32 per pair and part, element j of a part in half j & 1 of dword j >> 1 (the MFMA's
// operand order).
__device__ __forceinline__ void split8(const float (&v)[8], bf8 (&p)[3]) {
  u4 a, b, c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f2 x;
    x.x = v[2 * i];
    x.y = v[2 * i + 1];
    a[i] = cvt2(x);
    const f2 r1 = x - widen2(a[i]);
    b[i] = cvt2(r1);
    const f2 r2 = r1 - widen2(b[i]);
    c[i] = cvt2(r2);
  }
  p[0] = __builtin_bit_cast(bf8, a);
  p[1] = __builtin_bit_cast(bf8, b);
  p[2] = __builtin_bit_cast(bf8, c);
}

// max(x, 0) on the bit pattern (negative floats, -0 included, are negative integers): one v_max_i32
__device__ __forceinline__ float relu(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

__device__ __forceinline__ bf8 as_bf8(u4 v) { return __builtin_bit_cast(bf8, v); }
__device__ __forceinline__ u4 as_u4(bf8 v) { return __builtin_bit_cast(u4, v); }

// The z accumulation (K = C, up to 128 16-k steps at C = 2048) keeps a0 b0 in its own accumulator
// and the five small products (at most 2^-8 of the product) in a second one, summed once in the
// epilogue: the long accumulation then sees a sixth of the additions into the large sum, as in the
// compress GEMMs (compress_split.hip, Acc2), whose pixel sums drifted 6x the fp32 GEMM's error with
// one accumulator (tests/test_gpu_encoder.py checks the column sums of z at C = 2048).
__device__ __forceinline__ void mma6_2(const bf8 (&a)[3], const bf8 (&b)[3], f16v& hi, f16v& lo) {
  lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], lo, 0, 0, 0);
  hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], hi, 0, 0, 0);
}

// acc += a b over the split parts: the six products with i + j <= 2, smallest first (one 16-k step:
// the hidden layer, K = 9 + bias)
__device__ __forceinline__ f16v mma6(const bf8 (&a)[3], const bf8 (&b)[3], f16v acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// Packed image, in 16-byte units (8 bf16 = one lane's fragment of one part):
//   W1 block hb, part p, lane l:        (hb * 3 + p) * 64 + l
//       unit u = 32 hb + (l & 31), k = 8 (l >> 5) + j: W1[u][k] (k < 9), b1[u] (k = 9), 0 (k > 9)
//   W2 column block cb, hidden block hb, 16-k step s, part p, lane l:
//       w2_base + (((cb * HB + hb) * 2 + s) * 3 + p) * 64 + l
//       column 32 cb + (l & 31), element j: hidden unit 32 hb + 16 s + 8 (j >> 2) + 4 (l >> 5) + (j & 3)
//       — the row of X that element j of the A operand built from X's registers 8 s .. 8 s + 7 holds
__host__ __device__ inline int64_t w1_units(int C) { return (int64_t)(C / 32) * 3 * 64; }
__host__ __device__ inline int64_t w2_units(int C) { return (int64_t)(2 * C / 32) * (C / 32) * 2 * 3 * 64; }

}  // namespace mrp_x6
