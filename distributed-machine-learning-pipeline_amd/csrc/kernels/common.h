// Shared device-side helpers for the hipdsml CDNA4 (gfx950) kernels.
//
// Everything here is written for a 64-lane wavefront and the gfx950 MFMA
// operand/accumulator lane maps (see cdna_hip_programming.md §3):
//   v_mfma_f32_16x16x4_f32 : lane l supplies A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]
//                            and holds D[row=(l>>4)*4+r][col=l&15], r=0..3.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

// Measurement-only knobs (drop a phase's memory traffic, grow a grid, ...) exist
// only in a measurement build (`python -m hipdsml._build --measure` adds
// -DHIPDSML_MEASURE; tools/ profiles them).  A production build -- every build
// _build.py and __graft_entry__ make by default -- folds them to constant 0,
// so no environment variable can change what a training kernel computes.
#ifdef HIPDSML_MEASURE
#define DSML_MEASURE_KNOB(x) (x)
#else
#define DSML_MEASURE_KNOB(x) 0
#endif

namespace dsml {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

__device__ __forceinline__ f32x4 mfma_f32_16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float4 sel4(bool p, float4 v) {
  return p ? v : zero4();
}

// bf16 <-> f32 (round-to-nearest-even on the way down; NaN kept quiet).
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Workgroup barrier that orders LDS traffic only.  __syncthreads() is a
// workgroup release fence + s_barrier, and on gfx950 hipcc lowers that fence to
// s_waitcnt vmcnt(0): every barrier would also wait for the global STORES the
// waves issued before it (a full memory round trip each).  Nothing in the
// row-chain kernels reads its own global stores back, so LDS ordering is all
// that is needed.  The asm "memory" clobber keeps the compiler from moving
// memory operations across it.  Must NOT be used while LDS-DMA
// (global_load_lds) writes are in flight: those count on vmcnt.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// Barrier that also retires every outstanding vector-memory op (LDS-DMA included).
__device__ __forceinline__ void full_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- Cross-device (xGMI) release / acquire: why no fence instruction -------
// Every peer-exchange protocol here (pk in mlp_persist.hip, xact, xgmi, the
// standalone all-reduce in xchg.hip) follows ONE pattern, and it is a complete
// system-scope release/acquire without buffer_wbl2 / buffer_inv:
//  * memory: exchange buffers are hipExtMallocWithFlags(hipDeviceMallocUncached)
//    (runtime/peer_exchange.cpp), i.e. MTYPE UC -- no L1/L2 ever holds a line;
//  * producer: payload stored with sc0 sc1 (system scope, write-through) ->
//    `s_waitcnt vmcnt(0)` by EVERY storing wave (a store retires from vmcnt
//    only when the owning device's memory has acknowledged it, across xGMI
//    too) -> flag store (system-scope relaxed atomic) by a lane of that wave,
//    or by one lane behind a workgroup barrier that follows every wave's wait.
//    A system-scope release fence would add `buffer_wbl2 sc0 sc1`: it writes
//    back DIRTY L2 lines, and the payload never makes any (UC, write-through),
//    so the only thing it would order -- the payload before the flag -- is
//    already ordered by the vmcnt wait (measured cost of the wbl2 instead:
//    ~1.7 us per issuing wave, MI355X_MICROARCH price list);
//  * consumer: flag polled with system-scope relaxed loads (sc0 sc1, from
//    memory), the payload then read with sc0 sc1 loads issued only after the
//    poll's value returned (control dependency behind its s_waitcnt): nothing
//    can be served from a stale cache line, so `buffer_inv` (the acquire
//    fence) would invalidate nothing these loads could hit.
// What the pattern does NOT cover, and so never appears: plain (cached)
// payload stores or loads on exchange memory, and flags raised by a lane for
// other waves without the barrier.  The data-tagged 8-B granules of the
// on-device hand-offs (one sc1 store carries value + tag) need no ordering.
//
// Spin until the peer flag *f reaches `want` (system-scope relaxed polls).
// Gives up after `timeout` s_memrealtime ticks (100 MHz) and sets *err — and
// also stops as soon as *err is already set: once any wait of the exchange has
// timed out, the peer is gone, and every later wait (other blocks, later
// calls) returning at once keeps a dead peer from costing one full timeout per
// wait.  Returns true when the flag arrived.
template <int kSleep>
__device__ __forceinline__ bool poll_flag_ge(const uint64_t* f, uint64_t want, uint32_t* err,
                                             uint64_t timeout) {
  typedef __attribute__((address_space(1))) uint64_t g64;
  typedef __attribute__((address_space(1))) uint32_t g32;
  const g64* gf = (const g64*)f;
  const g32* ge = (const g32*)err;
  if (__hip_atomic_load(gf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= want) return true;
  if (__hip_atomic_load(ge, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return false;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t it = 0;
  while (__hip_atomic_load(gf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    if ((++it & 255u) == 0u &&
        __hip_atomic_load(ge, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
      return false;
    __builtin_amdgcn_s_sleep(kSleep);
  }
  return true;
}

// DPP lane permutations (no LDS round trip, unlike __shfl_* = ds_bpermute).
constexpr int kDppQuadXor1 = 0xB1;      // quad_perm:[1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;      // quad_perm:[2,3,0,1]
constexpr int kDppRowMirror = 0x140;    // lane i <-> 15-i within a row of 16
constexpr int kDppRowHalfMirror = 0x141;  // lane i <-> 7-i within a half row
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
// Sum over the 4 lanes of each quad (every lane gets its quad's sum).
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_f<kDppQuadXor1>(v);
  v += dpp_f<kDppQuadXor2>(v);
  return v;
}
// Full-wave (64-lane) sum, wave-uniform result: quad DPP, half-row and row
// mirrors (row sums), then 4 v_readlane.
__device__ __forceinline__ float wave_sum(float v) {
  v = quad_sum(v);
  v += dpp_f<kDppRowHalfMirror>(v);
  v += dpp_f<kDppRowMirror>(v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
}
// Sum over each row of 16 lanes (every lane gets its row's sum).
__device__ __forceinline__ float row16_sum(float v) {
  v = quad_sum(v);
  v += dpp_f<kDppRowHalfMirror>(v);
  v += dpp_f<kDppRowMirror>(v);
  return v;
}
__device__ __forceinline__ void argmax_combine(float& mx, int& amax, float om, int oa) {
  if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
}
// (max, first argmax) over each row of 16 lanes.
__device__ __forceinline__ void row16_argmax(float& mx, int& amax) {
  argmax_combine(mx, amax, dpp_f<kDppQuadXor1>(mx), dpp_i<kDppQuadXor1>(amax));
  argmax_combine(mx, amax, dpp_f<kDppQuadXor2>(mx), dpp_i<kDppQuadXor2>(amax));
  argmax_combine(mx, amax, dpp_f<kDppRowHalfMirror>(mx), dpp_i<kDppRowHalfMirror>(amax));
  argmax_combine(mx, amax, dpp_f<kDppRowMirror>(mx), dpp_i<kDppRowMirror>(amax));
}
// (max, argmax-first) over the 4 lanes of each quad.
__device__ __forceinline__ void quad_argmax(float& mx, int& amax) {
  {
    const float om = dpp_f<kDppQuadXor1>(mx);
    const int oa = dpp_i<kDppQuadXor1>(amax);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  {
    const float om = dpp_f<kDppQuadXor2>(mx);
    const int oa = dpp_i<kDppQuadXor2>(amax);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
}

}  // namespace dsml
