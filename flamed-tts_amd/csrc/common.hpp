// Common types, error plumbing and small device helpers for the Flamed MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

namespace fl {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // SROA-friendly (HIP uint4 is a union struct)

// ---- error reporting (thread-local last error, C-ABI flamed_last_error) ----
void set_error(const char* fmt, ...);
const char* last_error();

enum Status : int {
  kOk = 0,
  kBadArg = 1001,      // invalid dims / null pointers / unsupported config
  kNoWorkspace = 1002, // workspace too small
  kHip = 1003,         // HIP runtime failure (message has details)
};

#define FL_HIP(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      ::fl::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return ::fl::kHip;                                                                 \
    }                                                                                    \
  } while (0)

#define FL_REQUIRE(cond, ...)        \
  do {                               \
    if (!(cond)) {                   \
      ::fl::set_error(__VA_ARGS__);  \
      return ::fl::kBadArg;          \
    }                                \
  } while (0)

#define FL_LAUNCH_CHECK()                                                                  \
  do {                                                                                     \
    hipError_t e_ = hipGetLastError();                                                     \
    if (e_ != hipSuccess) {                                                                \
      ::fl::set_error("%s:%d kernel launch -> %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return ::fl::kHip;                                                                   \
    }                                                                                      \
  } while (0)

// ---- device helpers ----
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// erf by Abramowitz & Stegun 7.1.26 (|err| <= 4.7e-7 in fp32 with v_rcp_f32 / v_exp_f32, measured over
// [-6, 6]); ~15 VALU ops against ocml erff's branchy ~40 (the GELU epilogue of the B = 64 conv_2 GEMM
// spent 13.7 us per workgroup in erff).  Used only where the result is rounded to bf16 next.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  const float p = ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t + 0.254829592f) * t;
  return copysignf(1.0f - p * __expf(-ax * ax), x);
}
__device__ __forceinline__ float gelu_fast(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

__device__ __forceinline__ float wave_sum16(float v) {  // sum over the 16 lanes sharing lane>>4
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Chan et al. parallel combine of (count, mean, M2) partials.
__device__ __forceinline__ void chan_combine(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  float nn = n + nb;
  if (nn <= 0.f) return;
  float d = meanb - mean;
  mean += d * (nb / nn);
  m2 += m2b + d * d * (n * nb / nn);
  n = nn;
}

template <typename DT> struct DTraits;
template <> struct DTraits<bf16> {
  static constexpr int EPC = 8;  // elements per 16-byte chunk
  static constexpr int kCode = 1;
};
template <> struct DTraits<float> {
  static constexpr int EPC = 4;
  static constexpr int kCode = 0;
};

// 16-byte chunk of DT built from EPC floats.
template <typename DT> __device__ __forceinline__ u32x4 pack_chunk(const float* v);
template <> __device__ __forceinline__ u32x4 pack_chunk<float>(const float* v) {
  return u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
}
template <> __device__ __forceinline__ u32x4 pack_chunk<bf16>(const float* v) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (bf16)v[j];
  return __builtin_bit_cast(u32x4, b);
}

template <typename DT> __device__ __forceinline__ void store_val(DT* p, float v) { *p = (DT)v; }
// four consecutive values (16-B fp32 / 8-B bf16 store; p aligned accordingly)
template <typename DT> __device__ __forceinline__ void store_val4(DT* p, const float* v);
template <> __device__ __forceinline__ void store_val4<float>(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void store_val4<bf16>(bf16* p, const float* v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 b;
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = (bf16)v[j];
  *reinterpret_cast<uint2*>(p) = __builtin_bit_cast(uint2, b);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ---- phase stamps (diagnostic build only: -DFL_STAMPS, libflamed_hip_stamps.so) ----
// Thread 0 of every block writes s_memtime at numbered checkpoints into fl_stamp_buf[block][8]
// when the host has pointed fl_stamp_buf at a buffer (one chosen kernel class per step).
#ifdef FL_STAMPS
static __device__ unsigned long long* fl_stamp_buf = nullptr;  // per translation unit (no -fgpu-rdc)
__device__ __forceinline__ void fl_stamp(int i) {
  if (threadIdx.x == 0 && fl_stamp_buf) {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    const size_t blk = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
    fl_stamp_buf[blk * 8 + i] = t;
  }
}
#define FL_STAMP(i) ::fl::fl_stamp(i)
#else
#define FL_STAMP(i) ((void)0)
#endif

}  // namespace fl
