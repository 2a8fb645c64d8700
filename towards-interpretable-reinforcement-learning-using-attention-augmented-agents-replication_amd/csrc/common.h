// Shared device/host definitions for the gfx950 attention-agent kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace aaa {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

// Accurate versions for the recurrent gate math (parity 1e-4 over 20 steps).
__device__ __forceinline__ float sigm_acc(float x) { return 1.0f / (1.0f + expf(-x)); }

template <typename T> struct is_f32 { static constexpr bool value = false; };
template <> struct is_f32<float> { static constexpr bool value = true; };

// Convert a 16-byte global chunk of G elements to T and store into LDS.
template <typename G, typename T>
__device__ __forceinline__ void lds_store_chunk(T* dst, const u32x4& raw) {
  if constexpr (sizeof(G) == sizeof(T)) {
    *reinterpret_cast<u32x4*>(dst) = raw;
  } else {
    // float -> bf16 (4 elements, 8 bytes)
    f32x4 f = __builtin_bit_cast(f32x4, raw);
    bf16x4 b;
    b[0] = (__bf16)f[0]; b[1] = (__bf16)f[1]; b[2] = (__bf16)f[2]; b[3] = (__bf16)f[3];
    *reinterpret_cast<bf16x4*>(dst) = b;
  }
}

template <typename T> __device__ __forceinline__ T to_t(float x) { return (T)x; }

}  // namespace aaa
