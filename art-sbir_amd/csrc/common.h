// Shared device/host helpers for libartsbir_hip (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this library:
//   * activations are NHWC, channel innermost; C % 8 == 0 (the stem input is
//     zero-padded from 3 to 8 channels by artsbir_pack_input);
//   * "T" is the activation/weight compute type: float (parity mode, exact
//     f32 MFMA) or __bf16 (throughput mode, bf16 MFMA with f32 accumulate);
//   * all statistics, optimizer state and gradients of parameters are f32;
//   * every entry point takes a hipStream_t and never synchronises.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define ARTSBIR_DT_F32 0
#define ARTSBIR_DT_BF16 1

// number of replica slots the per-channel statistics atomics are spread over
// (every workgroup adding into one 256-B row is ~14x slower than spreading)
#define ARTSBIR_NSLOT 32

namespace artsbir {

// error reporting (defined in capi.cpp)
void set_error(const char* fmt, ...);
// name of the GEMM kernel the last conv / gemm entry point launched (profiling)
void set_last_kernel(const char* name);

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// 16-byte vector of T: 8 x bf16 or 4 x f32
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  float v[4];
};
template <> struct Vec16<bf16> {
  static constexpr int N = 8;
  bf16 v[8];
};

template <typename T>
__device__ __forceinline__ Vec16<T> ld16(const T* p) {
  Vec16<T> r;
  *reinterpret_cast<uint4*>(&r) = *reinterpret_cast<const uint4*>(p);
  return r;
}
template <typename T>
__device__ __forceinline__ void st16(T* p, const Vec16<T>& r) {
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(&r);
}
template <typename T>
__device__ __forceinline__ Vec16<T> zero16() {
  Vec16<T> r;
  *reinterpret_cast<uint4*>(&r) = make_uint4(0, 0, 0, 0);
  return r;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace artsbir

#define ARTSBIR_CHECK_LAUNCH(name)                                   \
  do {                                                               \
    hipError_t e_ = hipGetLastError();                               \
    if (e_ != hipSuccess) {                                          \
      artsbir::set_error("%s: launch failed: %s", name,              \
                         hipGetErrorString(e_));                     \
      return -2;                                                     \
    }                                                                \
  } while (0)
