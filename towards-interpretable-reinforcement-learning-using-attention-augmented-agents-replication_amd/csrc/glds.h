// LDS-DMA pipelined variant of the MFMA GEMM (k-contiguous operands, and
// row-contiguous ones whose k runs over pixels: GRowsT / GIm2colT).
//
// Operands go global -> LDS with `buffer_load_dwordx4 ... lds` (no VGPR
// staging, no ds_write pass).  NBUF LDS stages form a ring: at K tile kt the
// waves wait (counted vmcnt) until their own DMA for tile kt has landed,
// barrier, re-issue the DMA for tile kt+NBUF-1 into the stage that every wave
// finished reading before that barrier, then run the MFMAs of tile kt.  With
// NBUF = 3 one tile stays in flight across every barrier, so a tile's global
// latency is covered by two tiles of MFMA work instead of one.
//
// LDS image: one DMA wave-instruction writes 64 lanes x 16 B contiguously, so
// the image is lane-linear: 16-B slot s of the stage holds chunk s, i.e. row
// s / RS, physical column s % RS (RS = 16-B slots per row).  The XOR swizzle
// that makes the fragment reads (ds_read_b128 over 32 rows at one logical
// column) bank-conflict-free is applied on the SOURCE side: physical slot pc
// of row r holds logical column pc ^ lds_swz(r), and the reader applies the
// same XOR.  Masked lanes (conv zero padding, rows past the end) read through
// the buffer descriptor's range check and land as zeros.
//
// Preconditions (host-checked): G == T (no conversion while staging), each
// loader's chunk count is a multiple of the thread count (every wave issues
// the same number of DMA instructions per tile, which the counted vmcnt
// relies on), and the K slice is a multiple of BK.
#pragma once
#include <type_traits>
#include "loaders_b.h"

namespace aaa {

typedef __attribute__((address_space(3))) void* lds_vptr;

// 16-B slot XOR for a row of RS slots: rows that share a 256-B bank line
// (16/RS of them) keep their natural offset; successive lines rotate.
template <int RS>
__device__ __forceinline__ int lds_swz(int row) {
  constexpr int RPL = RS >= 16 ? 1 : 16 / RS;
  return (row / RPL) & (RS - 1);
}

// soff: wave-uniform byte offset added by the address unit (an SGPR, no VALU);
// the range check applies to voff + soff, so kOOB lanes stay out of range
// for any soff < 2^31.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const void* lds, uint32_t voff, int soff = 0) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr)(const_cast<void*>(lds)), 16, (int)voff, soff, 0, 0);
}
// the same with the sc1 cache policy (bytes another workgroup published with sc1 stores)
__device__ __forceinline__ void dma16_sc1(__amdgpu_buffer_rsrc_t r, const void* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr)(const_cast<void*>(lds)), 16, (int)voff, 0, 0, 16);
}

// The same issued from inline asm, for loaders whose consumer waits with its
// own counted vmcnt (gemm_pipe_kernel): the compiler does not see the LDS
// write, so it cannot insert the vmcnt(0) it otherwise places before the
// first LDS read after an LDS-DMA (which drains every tile still in flight
// and reduces the ring to one stage of latency cover).  M0 carries the
// wave-uniform LDS destination (an M0 operand, so the compiler sets it);
// s_nop 0 covers the M0 -> LDS-DMA hazard.
__device__ __forceinline__ void dma16a(__amdgpu_buffer_rsrc_t r, const void* lds, uint32_t voff, int soff = 0) {
  __builtin_assume(lds != nullptr);   // no generic-null select on the address-space cast
  const int m = __builtin_amdgcn_readfirstlane((int)(size_t)(lds_vptr)(const_cast<void*>(lds)));
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(r), "s"(soff), "{m0}"(m)
               : "memory");
}

// Epilogues with a split prefetch()/finish() (EP::Pre) have their global
// inputs loaded before the K loop, so the loads' latency hides under it.
template <class EP, class = void> struct has_pre : std::false_type {};
template <class EP> struct has_pre<EP, std::void_t<typename EP::Pre>> : std::true_type {};
template <class EP, bool> struct pre_of { using type = int; };
template <class EP> struct pre_of<EP, true> { using type = typename EP::Pre; };
// Epilogues with a per-thread accumulator (EP::Acc) get it passed to finish()
// and reduced by EP::flush<G4, NT>() after the epilogue (e.g. bias partials).
// Epilogues marked kDirect (split-K weight-gradient atomics) run straight from
// the accumulators: lanes of a 32-lane half own 32 consecutive columns of one
// row, so each atomic instruction covers a contiguous 128-B run of the output.
template <class EP, class = void> struct is_direct : std::false_type {};
template <class EP> struct is_direct<EP, std::enable_if_t<EP::kDirect>> : std::true_type {};
template <class EP, class = void> struct has_acc : std::false_type {};
template <class EP> struct has_acc<EP, std::void_t<typename EP::Acc>> : std::true_type {};
template <class EP, bool> struct acc_of { using type = int; };
template <class EP> struct acc_of<EP, true> { using type = typename EP::Acc; };
// Epilogues that store one partial per K slice (EpiSliceT): the kernel hands
// them the workgroup's slice index before any use (set_z on a local copy).
// EpiSliceT with the tile finished in the kernel (stream-K fixup): every K
// slice stores its partial, and the workgroup whose slice arrives last at the
// tile's counter (cnt[ti * ntj + tj], zeroed once, reset by that workgroup)
// sums the nz partials in slice order and runs the inner epilogue ``in`` on
// them (gemm_pipe_kernel calls fixup<C> after the staged epilogue): one launch
// per split-K step instead of a GEMM and a separate summing kernel.  Hand-off
// without fences (an agent-scope release would write back the whole L2):
// write-through (sc1) partial stores, every wave's vmcnt(0), a workgroup
// barrier, ONE lane's agent-scope add to the tile's counter, and the last
// workgroup -- told by the value its add returned -- takes one agent acquire
// and reads the partials with sc1 loads behind a barrier (MI355X_MICROARCH.md
// consumer rule; the hand-off table's row 1 without the acquire would do for
// fresh buffers, but these are rewritten every step).
template <class IN>
struct EpiSliceFix {
  static constexpr bool kFixup = true;
  static constexpr int kSc1 = 16;   // buffer cache policy: sc1
  float* out;        // slice 0 of the partials; slice s at out + s * sls (floats)
  int ld, Mi, Nj;
  size_t sls;
  int nz, ntj;
  int* cnt;
  IN in;
  int z = 0;
  __device__ __forceinline__ void set_z(int z_) { z = z_; }
  __device__ __forceinline__ void operator()(int i, int j, float v0, float v1, float v2, float v3) const {
    if (j >= Nj || i >= Mi) return;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(out, (uint32_t)((size_t)nz * sls * 4));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v0, v1, v2, v3}), rs,
                                           (uint32_t)(((size_t)z * sls + (size_t)j * ld + i) * 4), 0, kSc1);
  }
  template <class C>
  __device__ __forceinline__ void fixup(void* lds, int i0, int j0, int ti, int tj) const {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's partial stores retired
    __syncthreads();
    int* last = reinterpret_cast<int*>(lds);
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(cnt + ti * ntj + tj, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == nz - 1) {
        __hip_atomic_store(cnt + ti * ntj + tj, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the partial buffers are reused every step: drop this CU's / XCD's stale copies (one
        // agent acquire by the last workgroup; the barrier below holds the others until it completes)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *last = old == nz - 1;
    }
    __syncthreads();
    if (!*last) return;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(out, (uint32_t)((size_t)nz * sls * 4));
    constexpr int G4 = C::BI / 4;
    for (int c = (int)threadIdx.x; c < G4 * C::BJ; c += C::NT) {
      const int i = i0 + 4 * (c % G4), j = j0 + c / G4;
      if (j >= Nj || i >= Mi) continue;
      const uint32_t o = (uint32_t)(((size_t)j * ld + i) * 4);
      f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, kSc1));
      for (int k = 1; k < nz; ++k) {
        const f32x4 u = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + (uint32_t)((size_t)k * sls * 4), 0, kSc1));
        v[0] += u[0]; v[1] += u[1]; v[2] += u[2]; v[3] += u[3];
      }
      in(i, j, v[0], v[1], v[2], v[3]);
    }
  }
};

template <class EP, class = void> struct has_fixup : std::false_type {};
template <class EP> struct has_fixup<EP, std::enable_if_t<EP::kFixup>> : std::true_type {};
template <class EP, class = void> struct has_set_z : std::false_type {};
template <class EP>
struct has_set_z<EP, std::void_t<decltype(std::declval<EP&>().set_z(0))>> : std::true_type {};
template <class EP>
__device__ __forceinline__ EP with_z(const EP& ep, int tz) {
  if constexpr (has_set_z<EP>::value) {
    EP e = ep;
    e.set_z(tz);
    return e;
  } else {
    return ep;
  }
}

#ifdef AAA_STAMPS
// Diagnostic builds only (tools/ubench): per-workgroup phase timestamps
// (s_memrealtime, 100 MHz): [wg][0] entry, [1] K loop start, [2] K loop end, [3] exit.
__device__ uint64_t aaa_stamps[8192 * 4];
#define AAA_STAMP(k)                                                                                  \
  do {                                                                                                \
    if (threadIdx.x == 0)                                                                             \
      aaa_stamps[(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 4 + (k)] =        \
          __builtin_amdgcn_s_memrealtime();                                                           \
  } while (0)
#else
#define AAA_STAMP(k) do {} while (0)
#endif

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Barrier that does NOT drain the VM counter (an LDS-DMA in flight survives it).
__device__ __forceinline__ void barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Plain rows (weights): element (row, k) at src[row*ld + k].
template <typename T, int R, int BK, int NT>
struct GRowsB {
  static constexpr bool KC = true;
  static constexpr int VG = 16 / (int)sizeof(T);
  static constexpr int RS = BK / VG;
  static constexpr int NCH = R * RS;
  static constexpr int PER = NCH / NT;
  static constexpr int ELEMS = R * BK;
  static_assert(NCH % NT == 0, "every wave must issue the same number of DMA pieces");
  struct Params { const T* src; int ld; int nrows; };
  __amdgpu_buffer_rsrc_t rs;
  uint32_t voff[PER];
  int wofs;
  __device__ __forceinline__ GRowsB(const Params& p, int row0) {
    rs = make_rsrc(p.src, (uint32_t)((size_t)p.nrows * p.ld * sizeof(T)));
    wofs = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u) * VG);
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      const int lr = ch / RS, lc = (ch % RS) ^ lds_swz<RS>(lr), row = row0 + lr;
      voff[c] = row < p.nrows ? (uint32_t)((row * p.ld + lc * VG) * (int)sizeof(T)) : kOOB;
    }
  }
  __device__ __forceinline__ void issue(T* lds, int k0) {
    const int ko = __builtin_amdgcn_readfirstlane(k0 * (int)sizeof(T));
#pragma unroll
    for (int c = 0; c < PER; ++c) dma16a(rs, lds + c * NT * VG + wofs, voff[c], ko);
  }
};

// A operand of the split-product (SPLIT6) ring pre-split into three bf16
// planes (hi, mid, lo: split_planes) -- fp32 weights whose split the kernel
// would otherwise redo per fragment read: three GRowsB<bf16> stages side by
// side in the fp32 stage's place (ELEMS in float units: 1.5 x BI x BK).
template <int R, int BK, int NT>
struct GRows3B {
  using P1 = GRowsB<__bf16, R, BK, NT>;
  static constexpr bool KC = true, PRESPLIT = true;
  static constexpr int PER = 3 * P1::PER;
  static constexpr int ELEMS = 3 * R * BK / 2;
  struct Params { const __bf16* src; int ld; int nrows; size_t plane; };   // plane p at src + p * plane
  P1 pl[3];
  __device__ __forceinline__ GRows3B(const Params& p, int row0)
      : pl{P1(typename P1::Params{p.src, p.ld, p.nrows}, row0),
           P1(typename P1::Params{p.src + p.plane, p.ld, p.nrows}, row0),
           P1(typename P1::Params{p.src + 2 * p.plane, p.ld, p.nrows}, row0)} {}
  __device__ __forceinline__ void issue(float* lds, int k0) {
#pragma unroll
    for (int q = 0; q < 3; ++q) pl[q].issue(reinterpret_cast<__bf16*>(lds) + q * R * BK, k0);
  }
};
// B operand of the split-product ring as an implicit-GEMM gather over three
// bf16 planes of the fp32 source (split_planes): each element is split once
// instead of once per tap its window reads it.
template <int R, int BK, int NT>
struct GIm2colB3;
template <class LD, class = void> struct presplit_of : std::false_type {};
template <class LD> struct presplit_of<LD, std::enable_if_t<LD::PRESPLIT>> : std::true_type {};

// Implicit-GEMM gather (rows = output pixels, k = (tap, ci)); same geometry
// rules as LdIm2colB, whose per-pixel setup it shares.
template <typename T, int R, int BK, int NT>
struct GIm2colB {
  static constexpr bool KC = true;
  static constexpr int VG = 16 / (int)sizeof(T);
  static constexpr int RS = BK / VG;
  static constexpr int NCH = R * RS;
  static constexpr int PER = NCH / NT;
  static constexpr int ELEMS = R * BK;
  static_assert(NCH % NT == 0, "every wave must issue the same number of DMA pieces");
  struct Params { const T* src; ConvGeo g; int nrows; uint32_t src_bytes; };
  __amdgpu_buffer_rsrc_t rs;
  ConvGeo g;
  int base[PER], dt[PER];
  uint64_t vmask[PER];
  uint32_t vo[PER];     // whole-tap path: byte offset of this piece at tap ``cur`` (or kOOB)
  int cur;              // tap vo[] holds, -1 none
  bool whole;           // every K tile lies inside one tap (Cin % BK == 0): dt == 0
  int wofs;
  __device__ static bool ok_shape(const ConvGeo& g) { return LdIm2colB<T, T, R, BK, NT>::ok_shape(g); }
  __device__ __forceinline__ GIm2colB(const Params& p, int row0) : g(p.g) {
    rs = make_rsrc(p.src, p.src_bytes);
    wofs = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u) * VG);
    whole = g.Cin % BK == 0;
    cur = -1;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      const int lr = ch / RS, kc = ((ch % RS) ^ lds_swz<RS>(lr)) * VG, m = row0 + lr;
      im2col_setup(g, BK, m < p.nrows, m, kc, base[c], dt[c], vmask[c]);
      vo[c] = kOOB;
    }
  }
  // Whole-tap tiles: the per-lane offsets change only when the tap does (every
  // Cin / BK tiles); the channel offset ci0 is wave-uniform and goes in soff.
  // The tap's own offset is negative for the transposed gather, so vo carries
  // it (kOOB lanes stay kOOB), and soff = ci0 >= 0 only.
  __device__ __forceinline__ void issue(T* lds, int k0) {
    int tap, ci0;
    if (g.cmaj) {   // channel-chunk-major K (ConvGeo::cmaj == BK, whole taps)
      const int blk = k0 / BK, q = __builtin_amdgcn_readfirstlane((int)g.dTaps.div(blk));
      tap = blk - q * (int)g.dTaps.d;
      ci0 = q * BK;
    } else {
      tap = __builtin_amdgcn_readfirstlane((int)g.dCin.div(k0));
      ci0 = k0 - tap * g.Cin;
    }
    const int ky = __builtin_amdgcn_readfirstlane((int)g.dKW.div(tap));
    const int kx = tap - ky * g.KW;
    const int tv = (g.transposed ? -(ky * g.Win + kx) : (ky * g.Win + kx)) * g.cs;
    if (whole) {
      if (tap != cur) {
        cur = tap;
#pragma unroll
        for (int c = 0; c < PER; ++c) {
          const bool v = ((uint32_t)vmask[c] >> tap) & 1u;
          vo[c] = v ? (uint32_t)((base[c] + tv) * (int)sizeof(T)) : kOOB;
        }
      }
      const int so = __builtin_amdgcn_readfirstlane(ci0 * (int)sizeof(T));
#pragma unroll
      for (int c = 0; c < PER; ++c) dma16a(rs, lds + c * NT * VG + wofs, vo[c], so);
      return;
    }
    const int toff = tv + ci0;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const bool v = (vmask[c] >> (tap + dt[c])) & 1ull;
      dma16a(rs, lds + c * NT * VG + wofs, v ? (uint32_t)((base[c] + toff) * (int)sizeof(T)) : kOOB);
    }
  }
};

template <int R, int BK, int NT>
struct GIm2colB3 {
  using P1 = GIm2colB<__bf16, R, BK, NT>;
  static constexpr bool KC = true, PRESPLIT = true;
  static constexpr int PER = 3 * P1::PER;
  static constexpr int ELEMS = 3 * R * BK / 2;
  struct Params { const __bf16* src; ConvGeo g; int nrows; uint32_t src_bytes; size_t plane; };   // plane p at src + p * plane
  P1 pl[3];
  __device__ static bool ok_shape(const ConvGeo& g) { return P1::ok_shape(g); }
  __device__ __forceinline__ GIm2colB3(const Params& p, int row0)
      : pl{P1(typename P1::Params{p.src, p.g, p.nrows, p.src_bytes}, row0),
           P1(typename P1::Params{p.src + p.plane, p.g, p.nrows, p.src_bytes}, row0),
           P1(typename P1::Params{p.src + 2 * p.plane, p.g, p.nrows, p.src_bytes}, row0)} {}
  __device__ __forceinline__ void issue(float* lds, int k0) {
#pragma unroll
    for (int q = 0; q < 3; ++q) pl[q].issue(reinterpret_cast<__bf16*>(lds) + q * R * BK, k0);
  }
};

// Fragment of 8 consecutive logical k at row r from a swizzled KC stage.
template <int BK>
__device__ __forceinline__ void frag_sw(const float* t, int r, int kofs, float (&a)[8]) {
  constexpr int RS = BK / 4;
  const int g = lds_swz<RS>(r), c0 = kofs >> 2;
  const f32x4 x = *reinterpret_cast<const f32x4*>(t + r * BK + ((c0 ^ g) << 2));
  const f32x4 y = *reinterpret_cast<const f32x4*>(t + r * BK + (((c0 + 1) ^ g) << 2));
  a[0] = x[0]; a[1] = x[1]; a[2] = x[2]; a[3] = x[3];
  a[4] = y[0]; a[5] = y[1]; a[6] = y[2]; a[7] = y[3];
}
template <int BK>
__device__ __forceinline__ bf16x8 frag_sw(const __bf16* t, int r, int kofs) {
  constexpr int RS = BK / 8;
  const int g = lds_swz<RS>(r);
  return *reinterpret_cast<const bf16x8*>(t + r * BK + (((kofs >> 3) ^ g) << 3));
}

// Row-contiguous (RC) stages: k-rows of R elements, [BK][R], for operands whose
// k runs over pixels (weight gradients).  The fragment reads are transposed
// (bf16: ds_read_b64_tr_b16, a 32-lane half reading 4 k-rows x 4 slots; f32:
// ds_read_b32 down a column), so the slot XOR spreads each aligned 4-row
// group over the 256-B bank line: rows sharing a line (16/RS of them) keep
// their offset, the next 4 groups of lines rotate by 4 slots.
template <int RS>
__device__ __forceinline__ int lds_swz_rc(int k) {
  if constexpr (RS < 8) {
    return 0;
  } else {
    constexpr int RPL = RS >= 16 ? 1 : 16 / RS;
    return 4 * ((k / RPL) & (RS / 4 - 1));
  }
}

// Transposed rows: element (row, k) at src[k*ld + row] (activation gradients,
// k = pixel), staged RC.  Rows >= nrows and k >= ktotal land as zeros.
template <typename T, int R, int BK, int NT>
struct GRowsT {
  static constexpr bool KC = false;
  static constexpr int VG = 16 / (int)sizeof(T);
  static constexpr int RS = R / VG;
  static constexpr int NCH = BK * RS;
  static constexpr int PER = NCH / NT;
  static constexpr int ELEMS = R * BK;
  static_assert(NCH % NT == 0, "every wave must issue the same number of DMA pieces");
  struct Params { const T* src; int ld; int nrows; int ktotal; };
  __amdgpu_buffer_rsrc_t rs;
  uint32_t voff[PER];
  int wofs, rowbytes;
  __device__ __forceinline__ GRowsT(const Params& p, int row0) {
    rs = make_rsrc(p.src, (uint32_t)((size_t)p.ktotal * p.ld * sizeof(T)));
    rowbytes = p.ld * (int)sizeof(T);
    wofs = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u) * VG);
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      const int kr = ch / RS, row = row0 + ((ch % RS) ^ lds_swz_rc<RS>(kr)) * VG;
      voff[c] = row < p.nrows ? (uint32_t)((kr * p.ld + row) * (int)sizeof(T)) : kOOB;
    }
  }
  __device__ __forceinline__ void issue(T* lds, int k0) { issue_part(lds, k0, 0, 1); }
  // pieces c with c % nparts == part (part, nparts compile-time after unrolling)
  __device__ __forceinline__ void issue_part(T* lds, int k0, int part, int nparts) {
    const int ko = __builtin_amdgcn_readfirstlane(k0 * rowbytes);
#pragma unroll
    for (int c = 0; c < PER; ++c)
      if (c % nparts == part) dma16a(rs, lds + c * NT * VG + wofs, voff[c], ko);
  }
};

// Weight-gradient gather, staged RC: row = (tap, ci) fixed per piece, k =
// output pixel (forward geometry, as LdIm2colTB).  Cin % VG == 0.  Pixels
// past the source's frames fall outside src_bytes and land as zeros.
// Consecutive issues advance k by BK (the pipe kernel's ring order), so each
// piece carries its pixel's window origin (iy0, ix0) and source offset from
// tile to tile with two carries (x wraps the row, y wraps the frame) instead
// of decoding the pixel index with FastDivs every tile; start(k) seeds them.
template <typename T, int R, int BK, int NT>
struct GIm2colT {
  static constexpr bool KC = false;
  static constexpr int VG = 16 / (int)sizeof(T);
  static constexpr int RS = R / VG;
  static constexpr int NCH = BK * RS;
  static constexpr int PER = NCH / NT;
  static constexpr int ELEMS = R * BK;
  static_assert(NCH % NT == 0, "every wave must issue the same number of DMA pieces");
  struct Params { const T* src; ConvGeo g; int nrows; uint32_t src_bytes; };
  __amdgpu_buffer_rsrc_t rs;
  ConvGeo g;
  int kr[PER], ky[PER], kx[PER], toff[PER];
  int iy0[PER], ix0[PER], off[PER];   // per piece: window origin and source element offset of its current pixel
  // per-tile advance: BK = fq*HW + yq*Wout + xq (xq < Wout, yq < Hout), and the
  // offset / origin steps of one x wrap and one y wrap
  int dix, diy, doff, xlim, xw, xwoff, ylim, yw, ywoff;
  int wofs;
  // The pieces' pixel state advances by BK per issue instead of being derived
  // from k0, so callers must call start(kb) once and then issue every K tile
  // exactly once, in order (every pipe kernel of this file does).  Builds with
  // -DAAA_DEBUG_LOADERS check that contract: a k0 out of sequence traps.
#ifdef AAA_DEBUG_LOADERS
  int knext = 0;
#endif
  __device__ static bool ok_shape(const ConvGeo& g) { return g.Cin % VG == 0 && !g.transposed; }
  __device__ __forceinline__ GIm2colT(const Params& p, int row0) : g(p.g) {
    rs = make_rsrc(p.src, p.src_bytes);
    wofs = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u) * VG);
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int ch = threadIdx.x + c * NT;
      kr[c] = ch / RS;
      const int kp = row0 + ((ch % RS) ^ lds_swz_rc<RS>(kr[c])) * VG;
      const bool ok = kp < p.nrows;
      const int kq = ok ? kp : 0;
      const int tap = (int)g.dCin.div(kq), ci = kq - tap * g.Cin;
      ky[c] = ok ? (int)g.dKW.div(tap) : -100000;   // invalid rows never pass the bounds test
      kx[c] = tap - (int)g.dKW.div(tap) * g.KW;
      toff[c] = (ky[c] * g.Win + kx[c]) * g.cs + ci + g.coff;
    }
    const int hw = g.Hout * g.Wout;
    const int fq = BK / hw, rem = BK - fq * hw, yq = rem / g.Wout, xq = rem - yq * g.Wout;
    const int xs = g.stride * g.cs, ys = g.stride * g.Win * g.cs, fs = g.Hin * g.Win * g.cs;
    dix = xq * g.stride;
    diy = yq * g.stride;
    doff = fq * fs + yq * ys + xq * xs;
    xlim = g.Wout * g.stride - g.pad;   // ix0 >= xlim: x wrapped
    xw = g.Wout * g.stride;
    xwoff = ys - g.Wout * xs;
    ylim = g.Hout * g.stride - g.pad;
    yw = g.Hout * g.stride;
    ywoff = fs - g.Hout * ys;
  }
  __device__ __forceinline__ void start(int k0) {
    const int hw = g.Hout * g.Wout;
#ifdef AAA_DEBUG_LOADERS
    knext = k0;
#endif
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int m = k0 + kr[c];
      const int f = (int)g.dHW.div(m), pix = m - f * hw;
      const int oy = (int)g.dWout.div(pix), ox = pix - oy * g.Wout;
      iy0[c] = oy * g.stride - g.pad;
      ix0[c] = ox * g.stride - g.pad;
      off[c] = ((f * g.Hin + iy0[c]) * g.Win + ix0[c]) * g.cs + toff[c];
    }
  }
  __device__ __forceinline__ void issue(T* lds, int k0) { issue_part(lds, k0, 0, 1); }
  __device__ __forceinline__ void issue_part(T* lds, int k0, int part, int nparts) {
#ifdef AAA_DEBUG_LOADERS
    if (k0 != knext) __builtin_trap();   // out-of-order issue: the incremental gather would read wrong pixels
    if (part == nparts - 1) knext += BK;
#else
    (void)k0;
#endif
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      if (c % nparts != part) continue;
      const int iy = iy0[c] + ky[c], ix = ix0[c] + kx[c];
      const bool v = (unsigned)iy < (unsigned)g.Hin && (unsigned)ix < (unsigned)g.Win;
      dma16a(rs, lds + c * NT * VG + wofs, v ? (uint32_t)(off[c] * (int)sizeof(T)) : kOOB);
      // next tile: k += BK
      int nx = ix0[c] + dix, ny = iy0[c] + diy, no = off[c] + doff;
      if (nx >= xlim) { nx -= xw; ny += g.stride; no += xwoff; }
      if (ny >= ylim) { ny -= yw; no += ywoff; }
      ix0[c] = nx; iy0[c] = ny; off[c] = no;
    }
  }
};

// Loaders whose per-piece state follows the k order seed it here (GIm2colT).
template <class LD, class = void> struct has_start : std::false_type {};
template <class LD> struct has_start<LD, std::void_t<decltype(std::declval<LD&>().start(0))>> : std::true_type {};

// Fragments from an RC stage (same lane -> (row, k) map as frag_sw).
template <int R>
__device__ __forceinline__ void frag_rc(const float* t, int r, int kofs, float (&a)[8]) {
  constexpr int RS = R / 4;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = kofs + kk;
    a[kk] = t[k * R + (((r >> 2) ^ lds_swz_rc<RS>(k)) << 2) + (r & 3)];
  }
}
template <int R>
__device__ __forceinline__ bf16x8 frag_rc(const __bf16* t, int r, int kofs) {
  // two transpose reads: in each 16-lane group (rows c0..c0+15 of one h) lane
  // 4q+p addresses k-row kofs+q (+4), rows c0+4p..+3, and receives row
  // c0 + (lane & 15) of the 4 k-rows
  constexpr int RS = R / 8;
  const int li = (int)(threadIdx.x & 15), q = li >> 2, p = li & 3;
  const int lc = (r - li + 4 * p) >> 3, e = 4 * (p & 1);
  const int k0 = kofs + q, k1 = k0 + 4;
  const __bf16* a0 = t + k0 * R + ((lc ^ lds_swz_rc<RS>(k0)) << 3) + e;
  const __bf16* a1 = t + k1 * R + ((lc ^ lds_swz_rc<RS>(k1)) << 3) + e;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<__bf16*>(a0)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<__bf16*>(a1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// The same read with the lane's offsets precomputed: for a k offset kl + 16 j
// (kl = the lane/wave part, j uniform) the XOR key lds_swz_rc depends on kl
// only, so the two offsets are lane constants and the uniform 16 j R goes in
// the address base (the reads' immediate offsets), not per-read VALU.
struct RcOff { int o0, o1; };
template <int R>
__device__ __forceinline__ RcOff rc_off(int r, int kl) {
  constexpr int RS = R / 8;
  static_assert(RS < 8 || (RS >= 16 ? 1 : 16 / RS) <= 2, "swizzle key must not depend on the 16-k step");
  const int li = (int)(threadIdx.x & 15), q = li >> 2, p = li & 3;
  const int lc = (r - li + 4 * p) >> 3, e = 4 * (p & 1);
  const int k0 = kl + q, k1 = k0 + 4;
  return {k0 * R + ((lc ^ lds_swz_rc<RS>(k0)) << 3) + e, k1 * R + ((lc ^ lds_swz_rc<RS>(k1)) << 3) + e};
}
__device__ __forceinline__ bf16x8 frag_rc_at(const __bf16* t, const RcOff& o) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<__bf16*>(t + o.o0)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<__bf16*>(t + o.o1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Dispatch on the loader's stage layout.
template <class LD, int R, int BK>
__device__ __forceinline__ void frag_any(const float* t, int r, int kofs, float (&a)[8]) {
  if constexpr (LD::KC) frag_sw<BK>(t, r, kofs, a);
  else frag_rc<R>(t, r, kofs, a);
}
template <class LD, int R, int BK>
__device__ __forceinline__ bf16x8 frag_any(const __bf16* t, int r, int kofs) {
  if constexpr (LD::KC) return frag_sw<BK>(t, r, kofs);
  else return frag_rc<R>(t, r, kofs);
}

// Epilogue work split: the tile's (4-row group, column) items, G4 row groups
// per column, NPT items per thread.  Items with a split prefetch() (EP::Pre)
// keep at most PD of them in registers: the first PD are requested before the
// K loop, and each later one right after the item PD places before it is
// finished, so the loads of a wide tile (e.g. the BPTT gate backward, 32 floats
// per item) overlap the epilogue's own math instead of spilling.
template <class C, class EP, bool PRE_>
struct EpiPlan {
  static constexpr bool PRE = PRE_;
  using PreT = typename pre_of<EP, PRE>::type;
  static constexpr int G4 = C::BI / 4, NG = G4 * C::BJ, NPT = (NG + C::NT - 1) / C::NT;
  static constexpr int PRE_FLOATS = 64;         // register budget for prefetched epilogue inputs
  static constexpr int PW = (int)(sizeof(PreT) / 4) > 0 ? (int)(sizeof(PreT) / 4) : 1;
  static constexpr int PD0 = PRE_FLOATS / PW < 1 ? 1 : PRE_FLOATS / PW;
  static constexpr int PD = PD0 < NPT ? PD0 : NPT;
};

// Request the epilogue inputs of item q (slot q % PD).  ``jn`` = valid tile columns.
template <class C, class EP, class PL>
__device__ __forceinline__ void epilogue_load(const EP& ep, int i0, int j0, int jn, int q,
                                              typename PL::PreT (&pre)[PL::PD]) {
  if constexpr (PL::PRE) {
    const int c = q * C::NT + (int)threadIdx.x;
    if ((PL::NG % C::NT == 0 || c < PL::NG) && c / PL::G4 < jn)
      pre[q % PL::PD] = ep.prefetch(i0 + 4 * (c % PL::G4), j0 + c / PL::G4);
  }
}

// Epilogue inputs of this thread's first PD items, requested before the K loop
// (vmcnt retires in issue order; the compiler waits for these ordinary loads
// only at their use after the loop).
template <class C, class EP, class PL>
__device__ __forceinline__ void epilogue_prefetch(const EP& ep, int i0, int j0, int jn,
                                                  typename PL::PreT (&pre)[PL::PD]) {
#pragma unroll
  for (int q = 0; q < PL::PD; ++q) epilogue_load<C, EP, PL>(ep, i0, j0, jn, q, pre);
}

// Epilogue through LDS, shared by the ring GEMM and the halo conv (halo.h).
// Every wave (all WK groups) stores its partial tile pixel-major, E[wk][j][i];
// then the whole workgroup walks the tile in 4-row groups with consecutive
// lanes on consecutive row groups of ONE column, so the epilogue's global
// loads/stores (gate activations, cell state, outputs: all [pixel][channel])
// are contiguous per column instead of one 16-B access per lane at a 2 KB
// stride, and all waves share it.  Tiles too wide for LDS (the fp32 image of a
// 256x256 tile is 266 KB) go through in EC column chunks of BJ/EC columns: the
// waves owning a chunk's columns store them, all threads process the chunk's
// items (item order is column-major, so a chunk is a contiguous run of q).
// ``smem`` must hold WK*(BJ/EC)*(BI+4) floats.  Tile columns >= jn are skipped
// (the halo conv's tiles end at a frame edge).
template <class C>
constexpr int epi_chunks() {
  constexpr long full = (long)C::WK * C::BJ * (C::BI + 4) * 4;
  return full <= 160L * 1024 ? 1 : (full / 2 <= 160L * 1024 ? 2 : 4);
}

template <class C, class EP, class PL, typename T, int MI, int MJ>
__device__ __forceinline__ void staged_epilogue(const EP& ep, T* smem, const f32x16 (&acc)[MI][MJ], int i0, int j0,
                                                int jn, int tj, typename PL::PreT (&pre)[PL::PD]) {
  constexpr int BI = C::BI, BJ = C::BJ, WI = C::WI, WJ = C::WJ, WK = C::WK;
  constexpr int WTI = BI / WI, WTJ = BJ / WJ;
  constexpr int ELD = BI + 4;                 // epilogue tile pitch (pad: conflict-free b128 writes)
  constexpr int G4 = PL::G4, NG = PL::NG, NPT = PL::NPT, PD = PL::PD;
  constexpr int EC = epi_chunks<C>(), BJC = BJ / EC, QC = NPT / EC;
  static_assert(EC == 1 || (BJC % 32 == 0 && (G4 * BJC) % C::NT == 0), "column chunks: whole items per thread");
  constexpr bool PRE = PL::PRE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wk = wave / (WI * WJ), wr = wave - wk * (WI * WJ);
  const int wi = wr / WJ, wj = wr - (wr / WJ) * WJ;
  const int r32 = lane & 31, h = lane >> 5;
  float* E = reinterpret_cast<float*>(smem);
  constexpr bool ACC = has_acc<EP>::value && PRE && C::NT % G4 == 0;
  typename acc_of<EP, ACC>::type eacc{};
#pragma unroll
  for (int ec = 0; ec < EC; ++ec) {
    if (ec == 0) barrier_lds();                 // every wave is done reading the last stage
    else __syncthreads();                       // every thread is done reading the last chunk
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
      for (int b = 0; b < MJ; ++b) {
        const int jb = wj * WTJ + b * 32;       // the fragment's first column (chunk-uniform)
        if (EC > 1 && jb / BJC != ec) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int i = wi * WTI + a * 32 + 8 * g + 4 * h;
          const int j = jb - ec * BJC + r32;
          *reinterpret_cast<f32x4*>(E + (wk * BJC + j) * ELD + i) =
              f32x4{acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]};
        }
      }
    __syncthreads();
#pragma unroll
    for (int q = ec * QC; q < (ec + 1) * QC; ++q) {
      const int c = q * C::NT + (int)threadIdx.x;
      if ((NG % C::NT == 0 || c < NG) && c / G4 < jn) {
        const int r4 = c % G4, j = c / G4, jl = j - ec * BJC;
        f32x4 v = *reinterpret_cast<const f32x4*>(E + jl * ELD + 4 * r4);
#pragma unroll
        for (int w = 1; w < WK; ++w) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(E + (w * BJC + jl) * ELD + 4 * r4);
          v[0] += u[0]; v[1] += u[1]; v[2] += u[2]; v[3] += u[3];
        }
        if constexpr (ACC) ep.finish(i0 + 4 * r4, j0 + j, v[0], v[1], v[2], v[3], pre[q % PD], &eacc);
        else if constexpr (PRE) ep.finish(i0 + 4 * r4, j0 + j, v[0], v[1], v[2], v[3], pre[q % PD]);
        else ep(i0 + 4 * r4, j0 + j, v[0], v[1], v[2], v[3]);
      }
      if (q + PD < NPT) epilogue_load<C, EP, PL>(ep, i0, j0, jn, q + PD, pre);
    }
  }
  if constexpr (ACC) {
    __syncthreads();                          // every thread is done reading E
    ep.template flush<G4, C::NT>(eacc, E, i0, tj);
  }
}

// ABL (diagnostic builds only, tools/ubench): bit 0 = no in-loop DMA, bit 1 =
// no MFMA, bit 2 = no epilogue.  Production launches use ABL = 0.
// ILV: issue the next tile's DMA between the MFMA groups of this tile instead
// of all at once after the barrier, so the DMA issue overlaps MFMA execution:
// 1 = A pieces after the first 16-deep k step, B after the last; 2 = every
// loader's pieces spread evenly over the k steps (loaders with issue_part).
template <class C, class LA, class LB, class EP, int NBUF, int ABL = 0, int ILV = 0>
__global__ void __launch_bounds__(C::NT)
gemm_pipe_kernel(typename LA::Params pa, typename LB::Params pb, EP ep_, int K, int kchunk, TileMap tm) {
  using T = typename C::type;
  constexpr int BI = C::BI, BJ = C::BJ, BK = C::BK, WI = C::WI, WJ = C::WJ, WK = C::WK;
  constexpr int WTI = BI / WI, WTJ = BJ / WJ, MI = WTI / 32, MJ = WTJ / 32;
  static_assert(MI >= 1 && MJ >= 1 && BK % (16 * WK) == 0, "tile shape");
  static_assert(NBUF >= 2, "ring depth");
  constexpr int AEL = LA::ELEMS, STG = LA::ELEMS + LB::ELEMS;
  constexpr int PIECES = LA::PER + LB::PER;   // DMA instructions per wave per K tile
  // ONE shared array for everything (a second __shared__ object can make the
  // compiler drain vmcnt before the fragment reads).
  constexpr int ELD = BI + 4;                 // epilogue tile pitch (pad: conflict-free b128 writes)
  constexpr bool DIRECT = is_direct<EP>::value;
  static_assert(!DIRECT || WK == 1, "direct epilogue: no in-WG split-K");
  constexpr int EPI_T =
      DIRECT ? 0 : (int)((WK * (BJ / epi_chunks<C>()) * ELD * sizeof(float) + sizeof(T) - 1) / sizeof(T));
  __shared__ __attribute__((aligned(16))) T smem[NBUF * STG > EPI_T ? NBUF * STG : EPI_T];
  static_assert(!has_acc<EP>::value || C::NT * 16 * sizeof(float) <= sizeof(smem),
                "accumulator reduction does not fit in LDS");
  AAA_STAMP(0);

  int ti, tj, tz;
  tile_of(tm, ti, tj, tz);
  const int i0 = ti * BI, j0 = tj * BJ;
  const int kb = tz * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke) return;
  const EP ep = with_z(ep_, tz);

  LA la(pa, i0);
  LB lb(pb, j0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wk = wave / (WI * WJ), wr = wave - wk * (WI * WJ);
  const int wi = wr / WJ, wj = wr - (wr / WJ) * WJ;
  const int r32 = lane & 31, h = lane >> 5;

  f32x16 acc[MI][MJ];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < MJ; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int nk = (ke - kb) / BK;
  // Epilogue groups of this thread (see the epilogue below) and, when the
  // epilogue supports it, their inputs, requested first (vmcnt retires in issue order) and consumed after the
  // K loop (ordinary loads: the compiler waits for them only at their use).
  using PL = EpiPlan<C, EP, has_pre<EP>::value && (ABL & 4) == 0>;
  typename PL::PreT pre[PL::PD];
  epilogue_prefetch<C, EP, PL>(ep, i0, j0, BJ, pre);

  if constexpr (has_start<LA>::value) la.start(kb);
  if constexpr (has_start<LB>::value) lb.start(kb);
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nk) {
      la.issue(smem + s * STG, kb + s * BK);
      lb.issue(smem + s * STG + AEL, kb + s * BK);
    }

  // lane offsets of the RC-stage fragment reads (rc_off; unused for KC stages)
  RcOff ofa[MI], ofb[MJ];
#pragma unroll
  for (int a = 0; a < MI; ++a) ofa[a] = LA::KC ? RcOff{0, 0} : rc_off<BI>(wi * WTI + a * 32 + r32, 16 * wk + 8 * h);
#pragma unroll
  for (int b = 0; b < MJ; ++b) ofb[b] = LB::KC ? RcOff{0, 0} : rc_off<BJ>(wj * WTJ + b * 32 + r32, 16 * wk + 8 * h);
  AAA_STAMP(1);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt is the oldest of the (up to NBUF-1) tiles in flight
    if (kt + NBUF - 2 < nk) wait_vmcnt<PIECES * (NBUF - 2)>();
    else wait_vmcnt<0>();
    barrier_lds();
    const bool pf = !(ABL & 1) && kt + NBUF - 1 < nk;
    T* const st = smem + ((kt + NBUF - 1) % NBUF) * STG;
    const int kn = kb + (kt + NBUF - 1) * BK;
    if (!ILV && pf) {
      la.issue(st, kn);
      lb.issue(st + AEL, kn);
    }
    const T* Ac = smem + (kt % NBUF) * STG;
    const T* Bc = Ac + AEL;
    constexpr int S2 = BK / 16 / WK;
    constexpr bool MF = (ABL & 2) == 0;   // fragment reads + MFMAs
    if constexpr (is_f32<T>::value) {
#pragma unroll
      for (int s2 = 0; s2 < S2; ++s2) {
        const int kofs = 16 * (s2 * WK + wk) + 8 * h;
        float af[MI][8], bfr[MJ][8];
        if constexpr (MF) {
        if constexpr (!presplit_of<LA>::value) {
#pragma unroll
          for (int a = 0; a < MI; ++a) frag_any<LA, BI, BK>(Ac, wi * WTI + a * 32 + r32, kofs, af[a]);
        }
        if constexpr (!presplit_of<LB>::value) {
#pragma unroll
          for (int b = 0; b < MJ; ++b) frag_any<LB, BJ, BK>(Bc, wj * WTJ + b * 32 + r32, kofs, bfr[b]);
        }
        if constexpr (split6_of<C>::value) {   // fp32 at fp32 accuracy on the bf16 MFMA (gemm.h SPLIT6)
          bf16x8 ah[MI], am[MI], al[MI], bh[MJ], bm[MJ], bl[MJ];
          if constexpr (presplit_of<LA>::value) {   // A's parts straight from its three bf16 planes
            const __bf16* Ab = reinterpret_cast<const __bf16*>(Ac);
#pragma unroll
            for (int a = 0; a < MI; ++a) {
              const int r = wi * WTI + a * 32 + r32;
              ah[a] = frag_sw<BK>(Ab, r, kofs);
              am[a] = frag_sw<BK>(Ab + BI * BK, r, kofs);
              al[a] = frag_sw<BK>(Ab + 2 * BI * BK, r, kofs);
            }
          } else {
#pragma unroll
            for (int a = 0; a < MI; ++a) split3_bf16(af[a], ah[a], am[a], al[a]);
          }
          if constexpr (presplit_of<LB>::value) {   // B's parts straight from its three bf16 planes
            const __bf16* Bb = reinterpret_cast<const __bf16*>(Bc);
#pragma unroll
            for (int b = 0; b < MJ; ++b) {
              const int r = wj * WTJ + b * 32 + r32;
              bh[b] = frag_sw<BK>(Bb, r, kofs);
              bm[b] = frag_sw<BK>(Bb + BJ * BK, r, kofs);
              bl[b] = frag_sw<BK>(Bb + 2 * BJ * BK, r, kofs);
            }
          } else if constexpr (bexact_of<C>::value) {   // B exact in bf16: converted, its parts zero
#pragma unroll
            for (int b = 0; b < MJ; ++b) bh[b] = to_bf16x8(bfr[b]);
          } else {
#pragma unroll
            for (int b = 0; b < MJ; ++b) split3_bf16(bfr[b], bh[b], bm[b], bl[b]);
          }
#pragma unroll
          for (int a = 0; a < MI; ++a)
#pragma unroll
            for (int b = 0; b < MJ; ++b) {
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
              if constexpr (!bexact_of<C>::value) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[a], bm[b], acc[a][b], 0, 0, 0);
              }
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[a], bh[b], acc[a][b], 0, 0, 0);
              if constexpr (!bexact_of<C>::value)
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bm[b], acc[a][b], 0, 0, 0);
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
            }
        } else {
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int a = 0; a < MI; ++a)
#pragma unroll
              for (int b = 0; b < MJ; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][kk], bfr[b][kk], acc[a][b], 0, 0, 0);
        }
        }
        if constexpr (ILV == 1) {
          if (pf && s2 == 0) la.issue(st, kn);
          if (pf && s2 == S2 - 1) lb.issue(st + AEL, kn);
        } else if constexpr (ILV == 2) {
          if (pf) {
            la.issue_part(st, kn, s2, S2);
            lb.issue_part(st + AEL, kn, s2, S2);
          }
        }
      }
    } else {
      // Fragments run NS-1 sub-steps ahead of the MFMAs (NS register slots,
      // <= 32 VGPRs), so an MFMA waits only for its own reads (counted
      // lgkmcnt) instead of a full LDS round trip per sub-step; the sched
      // barriers stop the scheduler from sinking the reads back behind the MFMAs.
      constexpr int NS0 = 32 / ((MI + MJ) * 4), NS = NS0 < 2 ? 2 : (NS0 > S2 ? (S2 > 0 ? S2 : 1) : NS0);
      bf16x8 fa[NS][MI], fb[NS][MJ];
      auto ld = [&](int s2, int slot) {
        const int kofs = 16 * (s2 * WK + wk) + 8 * h;
#pragma unroll
        for (int a = 0; a < MI; ++a)
          fa[slot][a] = LA::KC ? frag_sw<BK>(Ac, wi * WTI + a * 32 + r32, kofs)
                               : frag_rc_at(Ac + 16 * s2 * WK * BI, ofa[a]);
#pragma unroll
        for (int b = 0; b < MJ; ++b)
          fb[slot][b] = LB::KC ? frag_sw<BK>(Bc, wj * WTJ + b * 32 + r32, kofs)
                               : frag_rc_at(Bc + 16 * s2 * WK * BJ, ofb[b]);
      };
#pragma unroll
      for (int s2 = 0; s2 < NS - 1; ++s2)
        if (MF && s2 < S2) ld(s2, s2);
#pragma unroll
      for (int s2 = 0; s2 < S2; ++s2) {
        if (MF && s2 + NS - 1 < S2) ld(s2 + NS - 1, (s2 + NS - 1) % NS);
        __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of these MFMAs
        if constexpr (MF) {
#pragma unroll
          for (int a = 0; a < MI; ++a)
#pragma unroll
            for (int b = 0; b < MJ; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s2 % NS][a], fb[s2 % NS][b], acc[a][b], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (ILV == 1) {
          if (pf && s2 == 0) la.issue(st, kn);
          if (pf && s2 == S2 - 1) lb.issue(st + AEL, kn);
        } else if constexpr (ILV == 2) {
          if (pf) {
            la.issue_part(st, kn, s2, S2);
            lb.issue_part(st + AEL, kn, s2, S2);
          }
        }
      }
    }
  }

  if constexpr ((ABL & 4) != 0) {   // keep every accumulator alive without the epilogue's memory traffic
    float sum = 0.f;
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
      for (int b = 0; b < MJ; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) sum += acc[a][b][e];
    if (sum == 1234.5f) ep(i0, j0, sum, 0.f, 0.f, 0.f);
    AAA_STAMP(2);
    AAA_STAMP(3);
    return;
  }
  AAA_STAMP(2);
  if constexpr (DIRECT) {
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
      for (int b = 0; b < MJ; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          ep(i0 + wi * WTI + a * 32 + 8 * g + 4 * h, j0 + wj * WTJ + b * 32 + r32, acc[a][b][4 * g],
             acc[a][b][4 * g + 1], acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]);
    AAA_STAMP(3);
    return;
  }
  staged_epilogue<C, EP, PL>(ep, smem, acc, i0, j0, BJ, tj, pre);
  if constexpr (has_fixup<EP>::value) ep.template fixup<C>(smem, i0, j0, ti, tj);
  AAA_STAMP(3);
}

// Read-ahead ring (bf16): the fragments of tile kt+1 are read from LDS into a
// second register set right after the barrier of iteration kt, while the
// MFMAs of tile kt run on the set read one iteration earlier, so no LDS read
// latency is exposed behind the per-tile barrier (in gemm_pipe_kernel every
// wave reads its fragments right after the barrier and the MFMA pipe idles
// until they return).  The barrier of iteration kt needs tile kt+1 landed
// (every wave's own pieces: counted vmcnt), so NBUF-2 tiles stay in flight
// across it; the DMA of tile kt+NBUF-1 refills the stage of tile kt-1, whose
// reads completed before the MFMAs of iteration kt-1.  The lgkmcnt(0) before
// each barrier is a builtin the compiler sees, so it does not add waits for
// the current set behind the reads of the next one.  ABL (diagnostic builds):
// bit 0 = no in-loop DMA, bit 2 = no epilogue.
template <class C, class LA, class LB, class EP, int NBUF, int ABL = 0, int PRIO = 1>
__global__ void __launch_bounds__(C::NT)
gemm_pipe_ra_kernel(typename LA::Params pa, typename LB::Params pb, EP ep, int K, int kchunk, TileMap tm) {
  using T = typename C::type;
  static_assert(std::is_same<T, __bf16>::value, "bf16 only");
  constexpr int BI = C::BI, BJ = C::BJ, BK = C::BK, WI = C::WI, WJ = C::WJ, WK = C::WK;
  constexpr int WTI = BI / WI, WTJ = BJ / WJ, MI = WTI / 32, MJ = WTJ / 32, S2 = BK / 16;
  static_assert(MI >= 1 && MJ >= 1 && WK == 1 && BK % 16 == 0, "tile shape");
  static_assert(NBUF >= 3, "ring depth: tile kt+1 landed while kt+2.. stay in flight");
  constexpr int AEL = LA::ELEMS, STG = LA::ELEMS + LB::ELEMS;
  constexpr int PIECES = LA::PER + LB::PER;
  constexpr int ELD = BI + 4;
  constexpr bool DIRECT = is_direct<EP>::value;
  constexpr int EPI_T =
      DIRECT ? 0 : (int)((WK * (BJ / epi_chunks<C>()) * ELD * sizeof(float) + sizeof(T) - 1) / sizeof(T));
  __shared__ __attribute__((aligned(16))) T smem[NBUF * STG > EPI_T ? NBUF * STG : EPI_T];
  AAA_STAMP(0);

  int ti, tj, tz;
  tile_of(tm, ti, tj, tz);
  const int i0 = ti * BI, j0 = tj * BJ;
  const int kb = tz * kchunk;
  const int ke = min(K, kb + kchunk);
  if (kb >= ke) return;

  LA la(pa, i0);
  LB lb(pb, j0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wi = wave / WJ, wj = wave - (wave / WJ) * WJ;
  const int r32 = lane & 31, h = lane >> 5;

  f32x16 acc[MI][MJ];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < MJ; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int nk = (ke - kb) / BK;
  using PL = EpiPlan<C, EP, has_pre<EP>::value && (ABL & 4) == 0>;
  typename PL::PreT pre[PL::PD];
  epilogue_prefetch<C, EP, PL>(ep, i0, j0, BJ, pre);

  if constexpr (has_start<LA>::value) la.start(kb);
  if constexpr (has_start<LB>::value) lb.start(kb);
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nk) {
      la.issue(smem + s * STG, kb + s * BK);
      lb.issue(smem + s * STG + AEL, kb + s * BK);
    }
  RcOff ofa[MI], ofb[MJ];
#pragma unroll
  for (int a = 0; a < MI; ++a) ofa[a] = LA::KC ? RcOff{0, 0} : rc_off<BI>(wi * WTI + a * 32 + r32, 8 * h);
#pragma unroll
  for (int b = 0; b < MJ; ++b) ofb[b] = LB::KC ? RcOff{0, 0} : rc_off<BJ>(wj * WTJ + b * 32 + r32, 8 * h);

  bf16x8 fa[2][S2][MI], fb[2][S2][MJ];
  auto rd = [&](int tile, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    const T* Ac = smem + (tile % NBUF) * STG;
    const T* Bc = Ac + AEL;
#pragma unroll
    for (int s2 = 0; s2 < S2; ++s2) {
#pragma unroll
      for (int b = 0; b < MJ; ++b)
        fb[buf][s2][b] = LB::KC ? frag_sw<BK>(Bc, wj * WTJ + b * 32 + r32, 16 * s2 + 8 * h)
                                : frag_rc_at(Bc + 16 * s2 * BJ, ofb[b]);
#pragma unroll
      for (int a = 0; a < MI; ++a)
        fa[buf][s2][a] = LA::KC ? frag_sw<BK>(Ac, wi * WTI + a * 32 + r32, 16 * s2 + 8 * h)
                                : frag_rc_at(Ac + 16 * s2 * BI, ofa[a]);
    }
  };
  auto lds_sync = [] {
    __builtin_amdgcn_s_waitcnt((7 << 4) | (0 << 8) | 15 | (3 << 14));   // lgkmcnt(0) only
    asm volatile("s_barrier" ::: "memory");                           // (no LDS access moves across it)
  };
  // iteration kt: tile kt+1 landed everywhere -> barrier -> read tile kt+1 ->
  // MFMAs of tile kt (DMA of tile kt+NBUF-1 issued between them)
  auto step = [&](int kt, auto curc) {
    constexpr int cur = decltype(curc)::value;
    const bool nx = kt + 1 < nk;
    if (nx) {
      if (kt + NBUF - 2 < nk) wait_vmcnt<PIECES * (NBUF - 3)>();
      else wait_vmcnt<0>();
    }
    lds_sync();
    if (nx) rd(kt + 1, std::integral_constant<int, cur ^ 1>{});
    const bool pf = !(ABL & 1) && kt + NBUF - 1 < nk;
    T* const st = smem + ((kt + NBUF - 1) % NBUF) * STG;
    const int kn = kb + (kt + NBUF - 1) * BK;
    __builtin_amdgcn_sched_barrier(0);
    // raised issue priority over the MFMA cluster (two waves per SIMD: the other wave's reads and DMA
    // issue wait; C3 wgrad 1012-1014 -> 976-988 us, profiles/r06/ab/s6l_prio/)
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < S2; ++s2) {
#pragma unroll
      for (int a = 0; a < MI; ++a) {
#pragma unroll
        for (int b = 0; b < MJ; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][s2][a], fb[cur][s2][b], acc[a][b], 0, 0, 0);
        if (s2 == S2 - 1 && a == (MI + 1) / 2 - 1) {   // DMA issue between the MFMAs (after the first half)
          __builtin_amdgcn_sched_barrier(0);
          if (pf) la.issue(st, kn);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (pf) lb.issue(st + AEL, kn);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  if (NBUF - 2 < nk) wait_vmcnt<PIECES * (NBUF - 2)>();
  else wait_vmcnt<0>();
  lds_sync();
  rd(0, std::integral_constant<int, 0>{});
  AAA_STAMP(1);
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nk) step(kt + 1, std::integral_constant<int, 1>{});
  }

  if constexpr ((ABL & 4) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
      for (int b = 0; b < MJ; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) sum += acc[a][b][e];
    if (sum == 1234.5f) ep(i0, j0, sum, 0.f, 0.f, 0.f);
    AAA_STAMP(2);
    AAA_STAMP(3);
    return;
  }
  AAA_STAMP(2);
  if constexpr (DIRECT) {
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
      for (int b = 0; b < MJ; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          ep(i0 + wi * WTI + a * 32 + 8 * g + 4 * h, j0 + wj * WTJ + b * 32 + r32, acc[a][b][4 * g],
             acc[a][b][4 * g + 1], acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]);
    AAA_STAMP(3);
    return;
  }
  staged_epilogue<C, EP, PL>(ep, smem, acc, i0, j0, BJ, tj, pre);
  AAA_STAMP(3);
}

template <class C, class LA, class LB, class EP, int NBUF>
inline hipError_t launch_pipe_ra(const typename LA::Params& pa, const typename LB::Params& pb, const EP& ep, int Mi,
                                 int Nj, int K, int nsplit, hipStream_t st) {
  if (Mi <= 0 || Nj <= 0 || K <= 0) return hipSuccess;
  if (K % C::BK) return hipErrorInvalidValue;
  if (nsplit < 1) nsplit = 1;
  int kchunk = (K + nsplit - 1) / nsplit;
  kchunk = (kchunk + C::BK - 1) / C::BK * C::BK;
  nsplit = (K + kchunk - 1) / kchunk;
  dim3 grid((Nj + C::BJ - 1) / C::BJ, (Mi + C::BI - 1) / C::BI, nsplit);
  hipLaunchKernelGGL((gemm_pipe_ra_kernel<C, LA, LB, EP, NBUF>), grid, dim3(C::NT), 0, st, pa, pb, ep, K, kchunk,
                     tile_map(grid));
  return hipGetLastError();
}

template <class C, class LA, class LB, class EP, int NBUF = 2, int ILV = 0>
inline hipError_t launch_pipe(const typename LA::Params& pa, const typename LB::Params& pb, const EP& ep, int Mi,
                              int Nj, int K, int nsplit, hipStream_t st) {
  if (Mi <= 0 || Nj <= 0 || K <= 0) return hipSuccess;
  if (K % C::BK) return hipErrorInvalidValue;
  if (nsplit < 1) nsplit = 1;
  int kchunk = (K + nsplit - 1) / nsplit;
  kchunk = (kchunk + C::BK - 1) / C::BK * C::BK;
  nsplit = (K + kchunk - 1) / kchunk;
  dim3 grid((Nj + C::BJ - 1) / C::BJ, (Mi + C::BI - 1) / C::BI, nsplit);
  hipLaunchKernelGGL((gemm_pipe_kernel<C, LA, LB, EP, NBUF, 0, ILV>), grid, dim3(C::NT), 0, st, pa, pb, ep, K, kchunk,
                     tile_map(grid));
  return hipGetLastError();
}

}  // namespace aaa
