// Shared device/host definitions for the gfx950 attention-agent kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>
#include <mutex>
#include <vector>

namespace aaa {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N).
template <int I0, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I0 < N) {
    f(std::integral_constant<int, I0>{});
    static_for<I0 + 1, N>(f);
  }
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

// Accurate versions for the recurrent gate math (parity 1e-4 over 20 steps).
__device__ __forceinline__ float sigm_acc(float x) { return 1.0f / (1.0f + expf(-x)); }

// bf16 -> fp32 (exact) of the low / high half of a dword holding two bf16
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ f32x4 bf4_f32(const u32x2& u) { return f32x4{bf_lo(u.x), bf_hi(u.x), bf_lo(u.y), bf_hi(u.y)}; }

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

// Host-side log of every divisor the runtime builds (aaa_debug_divisors): the
// tests re-check each one over the whole dividend range of FastDiv.
struct DivisorLog {
  std::mutex mu;
  bool on = false;
  std::vector<uint32_t> seen;
};
inline DivisorLog& divisor_log() {
  static DivisorLog g;
  return g;
}
inline void note_divisor(uint32_t d) {
  DivisorLog& g = divisor_log();
  std::lock_guard<std::mutex> lk(g.mu);
  if (g.on && std::find(g.seen.begin(), g.seen.end(), d) == g.seen.end()) g.seen.push_back(d);
}

// Division by a runtime constant d in [1, 2^31), exact for EVERY dividend
// 0 <= n < 2^31 (all indices here are non-negative ints): with l = ceil(log2 d),
// s = 31 + l and m = ceil(2^s / d), 2^s <= m*d < 2^s + 2^l, so n*m / 2^s
// exceeds n/d by less than 1/d and floor(n*m / 2^s) = floor(n/d)
// (Granlund & Montgomery 1994, Thm 4.2 with N = 31).  m < 2^32 and
// n*m < 2^63: one 32x32->64 multiply and a shift.  (The round-1 divider,
// m = ceil(2^32/d) >> 32, was exact only while n*d < 2^32 -- false for conv1's
// 5.38 M pixel rows at 168x168.)
struct FastDiv {
  uint32_t d, m, s;
  __host__ __device__ FastDiv() : d(1), m(1u << 31), s(31) {}
  __host__ explicit FastDiv(uint32_t dd) : d(dd ? dd : 1) {
    uint32_t l = 0;
    while (l < 31 && (1ull << l) < d) ++l;
    s = 31 + l;
    m = (uint32_t)(((1ull << s) + d - 1) / d);
    note_divisor(d);
  }
  __host__ __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (uint32_t)(((uint64_t)n * m) >> s);
  }
};


// Bounded wait of one lane for a partner workgroup's published step count
// (the multi-workgroup frame-resident kernels, recur*.h).  The bound is a
// deadline on the 100-MHz real-time counter: ``budget`` ticks after this
// workgroup's first wait that had to poll (``dl`` = 0 until then; the kernel
// keeps it in one variable for all its waits).  Past the deadline the lane
// adds 1 to ``report`` -- a word of pinned host memory mapped into the device
// (rt_core.hip pair_report), so the host reads it with no copy -- and returns;
// every later wait of that workgroup that is not satisfied at once returns
// after one poll, so a kernel whose partner never arrives ends within about
// ``budget`` ticks whatever its step count.  The host turns the report into
// AAA_E_STRANDED at the next API call (or aaa_pair_status), and a guarded
// optimizer step (aaa_pair_flag + aaa_adam_step_guarded) skips the update.
__device__ __forceinline__ bool wait_expired(uint64_t& dl, int budget) {
  const uint64_t now = __builtin_amdgcn_s_memrealtime();
  if (!dl) dl = now + (uint64_t)(budget > 0 ? budget : 1);
  return now >= dl;
}

__device__ __forceinline__ void pair_wait(const int* flag, int target, int* report, int budget, uint64_t& dl) {
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (wait_expired(dl, budget)) {
      __hip_atomic_fetch_add(report, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Start-time offset of half the frames of a frame-resident kernel: a wave
// waits ``ticks`` of the 100-MHz real-time counter.  All frames of such a
// kernel run their steps in lock step, so their epilogues' HBM traffic comes in
// one chip-wide burst per step while the memory system idles under the GEMMs;
// offsetting half of them by about half a step interleaves the bursts with
// the other half's GEMMs.
__device__ __forceinline__ void stagger_wait(int ticks) {
  if (ticks <= 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(8);
}

// The same for several partners at once, by one wave: lane j polls flags[j]
// for every bit j of ``mask`` (j < 64), all in one round trip per poll (a loop
// of pair_wait calls pays one L2 round trip per partner, in sequence).  Past
// the deadline one lane adds 1 to ``report`` and the wave returns.
__device__ __forceinline__ void wave_wait_flags(const int* flags, unsigned long long mask, int target, int* report,
                                                int budget, uint64_t& dl) {
  const int lane = (int)(threadIdx.x & 63);
  const bool mine = (mask >> lane) & 1ull;
  for (;;) {
    const int v = mine ? __hip_atomic_load(flags + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : target;
    if (__all(v >= target)) return;
    if (wait_expired(dl, budget)) {
      if (lane == 0) __hip_atomic_fetch_add(report, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Launch a paired kernel (two cooperating workgroups per frame) as an ordinary
// dispatch whose whole grid fits one residency wave of the device: every
// workgroup is placed at once on an idle chip, and the bounded partner waits
// (pair_wait) report instead of hanging if a pair is ever not co-resident
// (another kernel holding CUs: Learner.step never overlaps a collective with
// these launches).
// Not hipLaunchCooperativeKernel: ANY cooperative launch makes a process that
// rocprofv3 profiles crash in exit() after the tool's finalisation -- a trivial
// 256-workgroup kernel with no libaaa.so loaded reproduces it
// (tools/ubench/coop_exit.hip, profiles/r03/coop/) -- which cost every C4 PMC
// pass its own call in round 2.
template <class KP>
inline hipError_t launch_resident(const void* kernel, int grid, int block, KP& params, hipStream_t st) {
  int dev = 0, cus = 0, per_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0);
  if (e != hipSuccess) return e;
  if ((long)per_cu * cus < grid) return hipErrorCooperativeLaunchTooLarge;
  void* args[] = {&params};
  return hipLaunchKernel(kernel, dim3(grid), dim3(block), args, 0, st);
}

}  // namespace aaa
