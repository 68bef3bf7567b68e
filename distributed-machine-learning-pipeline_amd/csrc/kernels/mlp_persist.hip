// Persistent fused training kernel for the flagship MLP 784-128-64-10 (fp32,
// batch 64 per replica): ONE launch runs S consecutive SGD steps with every
// weight resident on chip, replacing the three launches per step of
// mlp_f32.hip (K_A split-K layer 1, K_B row chain, K_C weight gradients).
//
// Reference hot loop replaced: client.go:596-647 (forwardPass :112-141,
// backwardPass :143-202, updateWeights :254-267), 937 x 10 times on the CPU.
//
// Why: at B = 64 a step is ~29 MFLOP, i.e. well under a microsecond of MFMA
// work spread over tens of CUs; the three-launch step costs ~18-21 us, almost
// all of it kernel boundaries, per-launch weight reloads and dependent memory
// round trips.  Here a step is two on-chip hand-offs between resident roles.
//
// Roles (36 workgroups x 256 threads, one per CU; residency is trivially met):
//
//  * 32 layer-1 blocks (gn, gk), gn < 8, gk < 4, own W1[16 gn .. +16][196 gk
//    .. +196] (and b1[16 gn ..] when gk == 0) in LDS for the whole launch.
//    Per step: Z1 partial [64 x 16] = X[:, k slice] . W1 tile^T (MFMA
//    16x16x4 f32), published as tagged granules; then, once the chain blocks
//    have published dZ1, dW1 tile = dZ1[:, n slice]^T . X[:, k slice] and the
//    SGD update in LDS.  The next step's X slice is prefetched into registers
//    while the block waits.
//  * 4 chain blocks c own batch rows 16c .. 16c+15 and a full copy of W2, b2,
//    W3, b3 in LDS.  Per step: H1 = relu(sum of the 4 k-partials), layer 2 and
//    3 forward, softmax + cross-entropy (eps 1e-10, client.go:151), dZ3 =
//    (p - y)/B, dZ2 = dZ3 W3 * (H2 > 0), dZ1 = dZ2 W2 * (H1 > 0) published to
//    the layer-1 blocks (the critical path ends here).  Off the critical path
//    the chains exchange their rows of H1, H2, dZ2, dZ3, and every chain
//    computes the full-batch dW2, db2, dW3, db3 in the same order, so the four
//    copies of W2 / W3 stay bit-identical without a broadcast.
//
// Hand-offs are data-tagged 8-byte granules {fp32 value, step tag} written by
// single write-through (sc1) stores and read with sc1 loads until every tag
// matches: no flags, no fences, no barriers across workgroups (MI355X
// microarch: an 8-B granule is never torn; sc1 loads/stores keep the hand-off
// coherent across XCDs).  Tags are the global step number + 1, so buffers
// need zeroing only when the step counter is rewound (host side).
//
// Every wait is bounded (timeout -> error word, checked by the host after the
// launch) and gives up at once when another block already timed out, so a
// fault ends the launch instead of hanging the GPU.
#include "common.h"
#include "../dsml.h"
#include <cstdlib>

namespace dsml {

namespace {

constexpr int kD0 = 784, kD1 = 128, kD2 = 64, kD3 = 10, kB = 64;
constexpr int kGN = 8, kGK = 4, kKC = kD0 / kGK;  // 196 k per layer-1 block
constexpr int kNL1 = kGN * kGK;                   // 32 layer-1 blocks
constexpr int kNCH = 4;                           // chain blocks (16 rows each)
constexpr int kThreads = 256;
static_assert(kKC % 4 == 0, "k slice must hold whole MFMA k-steps");

// ---- LDS layouts (floats) ----------------------------------------------------
constexpr int kXS = kKC + 16;              // W1 tile row stride (2-way conflicts at most)
// X tiles are [64][196] unpadded: LDS-DMA (global_load_lds) writes each wave
// instruction's 1 KiB lane-linearly, so the image must be contiguous; the
// 196-float stride costs at most 2-way bank conflicts on the MFMA operand reads.
struct L1Lay {
  static constexpr int X0 = 0;                       // X tile, buffer 0 [64][196]
  static constexpr int X1 = X0 + kB * kKC;           // buffer 1
  static constexpr int W = X1 + kB * kKC;            // W1 tile [16][kXS]
  static constexpr int DZ = W + 16 * kXS;            // dZ1 tile [64][17]
  static constexpr int B1 = DZ + kB * 17;            // b1 slice [16]
  static constexpr int TOTAL = B1 + 16;
};
constexpr int kS1 = kD1 + 4, kS2 = kD2 + 4, kS3 = 16 + 4;
struct ChLay {
  static constexpr int W2 = 0;                       // [64][kS1]
  static constexpr int W3 = W2 + kD2 * kS1;          // [16][kS2] rows >= 10 zero
  static constexpr int B2 = W3 + 16 * kS2;           // [64]
  static constexpr int B3 = B2 + kD2;                // [16]
  static constexpr int H1 = B3 + 16;                 // all rows [64][kS1]
  static constexpr int H2 = H1 + kB * kS1;           // [64][kS2]
  static constexpr int DZ2 = H2 + kB * kS2;          // [64][kS2]
  static constexpr int DZ3 = DZ2 + kB * kS2;         // [64][kS3] cols >= 10 zero
  static constexpr int RED = DZ3 + kB * kS3;         // [4][16][16] layer-3 partials
  static constexpr int TOTAL = RED + 4 * 256;
};
constexpr int kLdsFloats = L1Lay::TOTAL > ChLay::TOTAL ? L1Lay::TOTAL : ChLay::TOTAL;
static_assert(kLdsFloats * 4 <= 160 * 1024, "LDS budget");

// ---- exchange buffer layout (8-byte granules) -----------------------------------
// PART[32][16][64]   layer-1 partials, PLAIN fp32 column-major per block (b1
//                    added by gk == 0 blocks), published by one flag per block
//                    and step (PF): the chain reads 32 KiB of values instead of
//                    64 KiB of granules and checks 32 tags instead of 8192
// DZ1 [64][128]      activation gradient of layer 1
// CX  [2][4][kCXG]   chain exchange (parity by step), PLAIN fp32 (no tags):
//                    H1 rows [16][128], H2 rows [16][64], dZ2 rows [16][64],
//                    dZ3 rows [16][16]; published by one flag per chain and
//                    step (CXF), i.e. the flag form of the hand-off: half the
//                    bytes of granules and one bulk read once the flag is seen.
constexpr int kPartG = kNL1 * kB * 16;
constexpr int kDz1G = kB * kD1;
constexpr int kCXG = 16 * kD1 + 16 * kD2 + 16 * kD2 + 16 * 16;  // 4352
constexpr int64_t kOffPart = 0, kOffDz1 = kOffPart + kPartG, kOffCx = kOffDz1 + kDz1G;
constexpr int64_t kOffCxf = kOffCx + 2 * kNCH * kCXG / 2;  // CX holds floats: 2 per granule
constexpr int64_t kOffPf = kOffCxf + 2 * kNCH;                // PF[32]: partial flags
constexpr int64_t kTotalG = kOffPf + kNL1;
static_assert(kCXG % 4 == 0, "exchange rows travel as 16-B vectors");

constexpr int kSc1 = 16;  // buffer aux: sc1 (write-through store / L1-bypassing load)
typedef uint32_t nu4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ uint2 gran(float v, uint32_t tag) {
  return make_uint2(__float_as_uint(v), tag);
}
// One granule, one 8-byte write-through store.
__device__ __forceinline__ void st_gran(__amdgpu_buffer_rsrc_t r, int64_t g, float v, uint32_t tag) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  const uint2 x = gran(v, tag);
  u2 w = {x.x, x.y};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)(g * 8), 0, kSc1);
}
// Two adjacent granules (16 B, 16-B aligned), one load.
__device__ __forceinline__ uint4 ld_gran2(__amdgpu_buffer_rsrc_t r, int64_t g) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(g * 8), 0, kSc1);
  return make_uint4(v.x, v.y, v.z, v.w);
}

struct Poll {
  uint32_t* err;
  uint64_t timeout;
  uint64_t t0;
  uint32_t spins;
  __device__ __forceinline__ void start() { t0 = __builtin_amdgcn_s_memrealtime(); spins = 0; }
  // true: keep waiting; false: give up (timeout, or another block gave up)
  __device__ __forceinline__ bool again() {
    if ((++spins & 31u) == 0u &&
        __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
      return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
    return true;
  }
};

__device__ __forceinline__ uint64_t ld_ctr64(const int64_t* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// ---- replica exchange (nrep > 1): 16-B vector accesses at system scope
// (sc0 sc1) through a buffer descriptor on the wave-uniform slot base, so a
// wave's slot moves as coalesced 1 KiB instructions.  (Two 8-B system atomics
// per float4, the xchg.hip idiom, are one fabric transaction per lane each:
// measured 13 us for a chain wave's 40-float slot.) ----
typedef __attribute__((address_space(1))) uint64_t px_g64;
constexpr int kScSys = 17;  // buffer aux: sc0 | sc1 (system scope)
__device__ __forceinline__ void px_st4(const __amdgpu_buffer_rsrc_t& r, int off_bytes, float4 v) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4v, x), r, off_bytes, 0, kScSys);
}
__device__ __forceinline__ float4 px_ld4(const __amdgpu_buffer_rsrc_t& r, int off_bytes) {
  const nu4v v = __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, kScSys);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}

}  // namespace

// Phase stamps (s_memrealtime, 100 MHz) of layer-1 block 0 and chain block 0
// (and layer-2 gradient block 0) for steps 8..15 of a launch, profiling only
// (tools/pk_stamps.py): [role][step - 8][phase], role 0 = layer-1, 1 = chain,
// 2 = layer-2 gradients.
__device__ uint64_t g_pk_stamps[3][8][8];
__device__ int g_pk_stamp_on;
// Role 2, row 0 holds launch-level stamps: [0] layer-1 block 0 entry, [1] its
// prologue done, [2] its exit; [3] chain 0 entry, [4] prologue done, [5] exit.
#define PK_EDGE(ph)                                                                   \
  do {                                                                                \
    if (g_pk_stamp_on && threadIdx.x == 0)                                            \
      g_pk_stamps[2][0][(ph)] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
#define PK_STAMP(role, ph)                                                            \
  do {                                                                                \
    if (stamp_on && threadIdx.x == 0 && it >= 8 && it < 16)                            \
      g_pk_stamps[(role)][it - 8][(ph)] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)

struct PersistArgs {
  const float* X;
  int64_t ldx;
  const int32_t* labels;
  float* P;
  int64_t w_off[3], b_off[3];
  int64_t* ctr;
  int32_t nbatches;
  int32_t steps;
  float lr;
  float inv_batch;
  uint64_t* xb;  // exchange granules (kTotalG)
  float* stats;
  uint32_t* err;
  uint32_t* herr;  // host-mapped mirror of err (nullable): read without a copy
  uint64_t timeout_ticks;
  int32_t place;  // block -> role map: 1 = chains at b % 8 == 0 (one XCD, default), 0 = chains last
  // Data parallelism over nrep replicas (nrep > 1): every step, each weight
  // gradient slot is pushed into every peer's receive buffer (xt.buf[d], this
  // replica's slot; parity by step), flagged (xt.flags[d]), and summed over
  // the replicas in rank order from the local buffer -- identical bytes and
  // order on every replica, so the weights stay bit-identical.  lr is already
  // lr / nrep.
  XchgTab xt;
  int32_t nrep, rep;
  int64_t xhalf;   // floats per parity half of a receive buffer (>= px_half)
  uint32_t* xerr;  // the exchange's error word (a peer that did not arrive)
};

// Receive-buffer layout per parity half: [src][layer-1 block][wave] slots of
// 64 lanes x 16 floats (the wave's dW1 fragments, db1 included), then
// [src][chain wave] slots of 64 lanes x 40 floats (dW2 h-tile fragments, dW3,
// db2, db3).  Flags: [src][block][wave], then [src][wave].
constexpr int kPxL1 = 64 * 16, kPxCh = 64 * 40;
int64_t px_half(int n) { return (int64_t)n * (kNL1 * 4 * kPxL1 + 4 * kPxCh); }
int px_ntiles(int n) { return n * (kNL1 * 4 + 4); }

// One wave's slot, push half: v (this replica's) into every peer d with
// d % mod == sel, then raise their flags.
template <int NV>
__device__ __forceinline__ void px_push_wave(const PersistArgs& a, uint64_t s, const float4 (&v)[NV],
                                             int64_t base, int64_t per_src, int flag_base,
                                             int flag_per_src, int mod, int sel) {
  const int lane = threadIdx.x & 63;
  const int64_t poff = (int64_t)(s & 1) * a.xhalf;
  const uint64_t tag = s + 1;
  for (int d = 0; d < a.nrep; ++d) {
    if (d == a.rep || d % mod != sel) continue;
    const __amdgpu_buffer_rsrc_t r = rsrc(a.xt.buf[d] + poff + base + (int64_t)a.rep * per_src);
#pragma unroll
    for (int j = 0; j < NV; ++j) px_st4(r, (lane * (4 * NV) + 4 * j) * 4, v[j]);
  }
  // the slot landed (acknowledged by every peer's memory) before its flag: the
  // system-scope release of this protocol (common.h, "Cross-device release")
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0)
    for (int d = 0; d < a.nrep; ++d)
      if (d != a.rep && d % mod == sel)
        __hip_atomic_store((px_g64*)(a.xt.flags[d] + flag_base + a.rep * flag_per_src), tag,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pull half: wait for every peer's slot of step s here, then v (this
// replica's own values on entry) = the rank-ordered sum over all replicas.
// false: a peer did not arrive in time.
template <int NV>
__device__ __forceinline__ bool px_pull_wave(const PersistArgs& a, uint64_t s, float4 (&v)[NV],
                                             int64_t base, int64_t per_src, int flag_base,
                                             int flag_per_src) {
  const int lane = threadIdx.x & 63;
  const int64_t poff = (int64_t)(s & 1) * a.xhalf;
  const uint64_t tag = s + 1;
  bool ok = true;
  if (lane < a.nrep && lane != a.rep)
    ok = poll_flag_ge<1>(a.xt.flags[a.rep] + flag_base + lane * flag_per_src, tag, a.xerr,
                         a.timeout_ticks);
  ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
  asm volatile("" ::: "memory");
  if (!ok) return false;
  const float* mine = a.xt.buf[a.rep] + poff + base;
  float4 acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int src = 0; src < a.nrep; ++src) {
    const __amdgpu_buffer_rsrc_t r = rsrc(mine + src * per_src);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float4 x = src == a.rep ? v[j] : px_ld4(r, (lane * (4 * NV) + 4 * j) * 4);
      acc[j].x += x.x; acc[j].y += x.y; acc[j].z += x.z; acc[j].w += x.w;
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = acc[j];
  return true;
}

// Both halves back to back (the layer-1 blocks: their update is needed at once).
template <int NV>
__device__ __forceinline__ bool px_allreduce_wave(const PersistArgs& a, uint64_t s, float4 (&v)[NV],
                                                  int64_t base, int64_t per_src, int flag_base,
                                                  int flag_per_src, int mod, int sel) {
  px_push_wave<NV>(a, s, v, base, per_src, flag_base, flag_per_src, mod, sel);
  return px_pull_wave<NV>(a, s, v, base, per_src, flag_base, flag_per_src);
}


// A block that gave up leaves a mark in host memory on its way out, so the
// host learns the launch failed without a device->host copy.
__device__ __forceinline__ void pk_report(const PersistArgs& a, bool ok) {
  if (!ok && threadIdx.x == 0 && a.herr != nullptr)
    __hip_atomic_store(a.herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// -----------------------------------------------------------------------------
// Layer-1 block
// -----------------------------------------------------------------------------
constexpr int kXF4 = kB * (kKC / 4);  // float4 of one X tile (3136 = 49 KiB-chunks of 64)
static_assert(kXF4 % 64 == 0, "X tile must be whole 1 KiB LDS-DMA chunks");
typedef __attribute__((address_space(1))) void* pk_gptr;
typedef __attribute__((address_space(3))) void* pk_lptr;

// X tile of step s -> LDS buffer by LDS-DMA (16 B per lane, no registers):
// wave w issues chunks w, w+4, ...; completion is waited by the next
// __syncthreads (its vmcnt(0)).
__device__ __forceinline__ void pk_glds_x(const PersistArgs& a, float* lds, int buf, uint64_t s,
                                          int lane, int w, int k0) {
  const int64_t r0 = (int64_t)(s % (uint64_t)a.nbatches) * kB;
  float* xl = lds + (buf ? L1Lay::X1 : L1Lay::X0);
  for (int ch = w; ch < kXF4 / 64; ch += 4) {
    const int e = ch * 64 + lane;
    const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);
    __builtin_amdgcn_global_load_lds((pk_gptr)(a.X + (r0 + r) * a.ldx + k0 + 4 * c4),
                                     (pk_lptr)(xl + ch * 256), 16, 0, 0);
  }
}

template <bool DP>
__device__ __forceinline__ void pk_layer1(const PersistArgs& a, float* lds, int lb) {
  const int gn = lb % kGN, gk = lb / kGN;
  const int n0 = gn * 16, k0 = gk * kKC;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  float* Wl = lds + L1Lay::W;
  float* Dz = lds + L1Lay::DZ;
  float* B1 = lds + L1Lay::B1;

  if (lb == 0) PK_EDGE(0);
  // ---- prologue: W1 tile, b1 slice, X of the first step ----
  // every load of the tile in one batch (one memory round trip), then the LDS stores
  const float* W1g = a.P + a.w_off[0];
  constexpr int kW1F4 = 16 * (kKC / 4), kW1Per = (kW1F4 + kThreads - 1) / kThreads;
  float4 w1v[kW1Per];
#pragma unroll
  for (int j = 0; j < kW1Per; ++j) {
    const int e = min(tid + j * kThreads, kW1F4 - 1);
    const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);
    w1v[j] = *reinterpret_cast<const float4*>(W1g + (int64_t)(n0 + r) * kD0 + k0 + 4 * c4);
  }
  const float b1v = (tid < 16 && gk == 0) ? a.P[a.b_off[0] + n0 + tid] : 0.f;
#pragma unroll
  for (int j = 0; j < kW1Per; ++j) {
    const int e = tid + j * kThreads;
    if (e < kW1F4) {
      const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);
      *reinterpret_cast<float4*>(Wl + r * kXS + 4 * c4) = w1v[j];
    }
  }
  if (tid < 16) B1[tid] = b1v;
  constexpr int kXF4 = kB * (kKC / 4);                 // float4 of one X tile (3136)
  constexpr int kXPer = (kXF4 + kThreads - 1) / kThreads;  // 13
  pk_glds_x(a, lds, 0, s0, lane, w, k0);
  __syncthreads();
  if (lb == 0) PK_EDGE(1);

  bool ok = true;
  const int stamp_on = g_pk_stamp_on && lb == 0;
  for (int it = 0; it < a.steps && ok; ++it) {
    PK_STAMP(0, 0);
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    const int buf = it & 1;
    const float* Xl = lds + (buf ? L1Lay::X1 : L1Lay::X0);

    // ---- forward partial: wave w -> rows 16w..16w+15, all 16 n of the tile ----
    {
      // 49 k-steps in batches of 7: a batch's 14 LDS operands are read ahead
      // of its MFMAs (two accumulators hide the MFMA dependency latency)
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const float* xa = Xl + (16 * w + i) * kKC + q;
      const float* wa = Wl + i * kXS + q;
#pragma unroll
      for (int kb = 0; kb < kKC / 4; kb += 7) {
        float xv[7], wv[7];
#pragma unroll
        for (int u = 0; u < 7; ++u) {
          xv[u] = xa[4 * (kb + u)];
          wv[u] = wa[4 * (kb + u)];
        }
#pragma unroll
        for (int u = 0; u < 7; ++u) {
          if (u & 1) acc1 = mfma_f32_16x16x4(xv[u], wv[u], acc1);
          else acc0 = mfma_f32_16x16x4(xv[u], wv[u], acc0);
        }
      }
      // column i, rows 16w + 4q .. +3: one 16-B write-through store per lane
      const float bn = B1[i];
      const f32x4 z = {acc0[0] + acc1[0] + bn, acc0[1] + acc1[1] + bn, acc0[2] + acc1[2] + bn,
                       acc0[3] + acc1[3] + bn};
      const int off = (int)(((kOffPart * 2 + ((int64_t)lb * 16 + i) * kB + 16 * w + 4 * q)) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4v, z), rb, off, 0, kSc1);
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) st_gran(rb, kOffPf + lb, __uint_as_float(tag), tag);
    PK_STAMP(0, 1);
    // next step's X into the other buffer (its last reader, the previous
    // step's backward, finished before the barrier that ended that step)
    if (it + 1 < a.steps) pk_glds_x(a, lds, buf ^ 1, s + 1, lane, w, k0);

    // ---- wait for dZ1[:, n0 .. n0+15] of this step (4 chain blocks) ----
    {
      const int m = tid >> 2, qq = tid & 3;
      const int64_t g = kOffDz1 + (int64_t)m * kD1 + n0 + 4 * qq;
      uint4 v0, v1;
      poll.start();
      for (;;) {
        v0 = ld_gran2(rb, g);
        v1 = ld_gran2(rb, g + 2);
        if (v0.y == tag && v0.w == tag && v1.y == tag && v1.w == tag) break;
        if (!poll.again()) { ok = false; break; }
      }
      Dz[m * 17 + 4 * qq + 0] = __uint_as_float(v0.x);
      Dz[m * 17 + 4 * qq + 1] = __uint_as_float(v0.z);
      Dz[m * 17 + 4 * qq + 2] = __uint_as_float(v1.x);
      Dz[m * 17 + 4 * qq + 3] = __uint_as_float(v1.z);
    }
    if (lb == 0 && it + 1 == a.steps && tid == 0) {
      // every block has started (all chains published this step's dZ1, which
      // needed every layer-1 block's partial): hand the step counter on
      const uint64_t e = s0 + (uint64_t)a.steps;
      __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ctr), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ctr + 1), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    PK_STAMP(0, 2);

    // ---- backward: dW1 tile [16 n][196 k] = dZ1^T . X, SGD in LDS ----
    // wave w: k tiles kt = w, w + 4, w + 8, w + 12 (13 tiles of 16, the last 4 wide)
    f32x4 g[4];
    // The last k tile (kt = 12, wave 0) is 4 columns wide; its column k = 196
    // multiplies dZ1 by ones instead, so the MFMA also yields db1 = colsum(dZ1).
    float dv[kB / 4];  // A operand (dZ1 column i of rows 4ms + q), shared by the tiles
#pragma unroll
    for (int ms = 0; ms < kB / 4; ++ms) dv[ms] = Dz[(4 * ms + q) * 17 + i];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kt = w + 4 * t;
      if (kt * 16 < kKC) {
        const int kc = kt * 16 + i;
        const int kcc = kc < kKC ? kc : kKC - 1;
        const float pad = kc == kKC ? 1.f : 0.f;
        float xv[kB / 4];
#pragma unroll
        for (int ms = 0; ms < kB / 4; ++ms) xv[ms] = Xl[(4 * ms + q) * kKC + kcc];
#pragma unroll
        for (int ms = 0; ms < kB / 4; ++ms)
          g[t] = mfma_f32_16x16x4(dv[ms], kc < kKC ? xv[ms] : pad, g[t]);
      }
    }
    if (DP) {  // data parallel: sum this wave's fragments over the replicas
      // (waves 1-3 own 3 k tiles, wave 0 four: only real tiles travel)
      bool xok;
      const int64_t slot = (int64_t)(lb * 4 + w) * kPxL1, per = (int64_t)kNL1 * 4 * kPxL1;
      if (w == 0) {
        float4 v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = make_float4(g[t][0], g[t][1], g[t][2], g[t][3]);
        xok = px_allreduce_wave<4>(a, s, v, slot, per, lb * 4 + w, kNL1 * 4, 1, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t) g[t] = f32x4{v[t].x, v[t].y, v[t].z, v[t].w};
      } else {
        float4 v[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) v[t] = make_float4(g[t][0], g[t][1], g[t][2], g[t][3]);
        xok = px_allreduce_wave<3>(a, s, v, slot, per, lb * 4 + w, kNL1 * 4, 1, 0);
#pragma unroll
        for (int t = 0; t < 3; ++t) g[t] = f32x4{v[t].x, v[t].y, v[t].z, v[t].w};
      }
      ok = __syncthreads_and(xok ? 1 : 0) != 0;
      if (!ok) break;
    }
    // every wave read this step's W1 tile in the forward, before the barrier above
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kt = w + 4 * t;
      const int kc = kt * 16 + i;
      if (kt * 16 < kKC && kc < kKC) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Wl[(4 * q + r) * kXS + kc] -= a.lr * g[t][r];
      }
    }
    if (gk == 0 && w == 0 && i == kKC - 192) {  // wave 0, tile 12, column k = 196: db1
#pragma unroll
      for (int r = 0; r < 4; ++r) B1[4 * q + r] -= a.lr * g[3][r];
    }
    __syncthreads();
    PK_STAMP(0, 3);
  }

  // ---- epilogue: the resident weights back to HBM ----
  float* W1w = a.P + a.w_off[0];
  for (int e = tid; e < 16 * (kKC / 4); e += kThreads) {
    const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);
    *reinterpret_cast<float4*>(W1w + (int64_t)(n0 + r) * kD0 + k0 + 4 * c4) =
        *reinterpret_cast<const float4*>(Wl + r * kXS + 4 * c4);
  }
  if (gk == 0 && tid < 16) a.P[a.b_off[0] + n0 + tid] = B1[tid];
  pk_report(a, ok);
  if (lb == 0) PK_EDGE(2);
}

// -----------------------------------------------------------------------------
// Chain block
// -----------------------------------------------------------------------------
// A chain wave's SGD step on its LDS copies: W2 rows of h tile w, W3 columns
// of h tile w, b2 of h tile w, b3 (wave 0).  Every wave is past its reads of
// the old values (a barrier separates them): all old values read first, then
// all the updated ones written.
__device__ __forceinline__ void pk_chain_update(const PersistArgs& a, float* lds, int w, int q, int i,
                                                const f32x4 (&g)[8], const f32x4& g3, float sb2,
                                                float sb3) {
  float* W2 = lds + ChLay::W2;
  float* W3 = lds + ChLay::W3;
  float* B2 = lds + ChLay::B2;
  float* B3 = lds + ChLay::B3;
  float w2o[8][4], w3o[4];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) w2o[t][r] = W2[(16 * w + 4 * q + r) * kS1 + 16 * t + i];
#pragma unroll
  for (int r = 0; r < 4; ++r) w3o[r] = W3[(4 * q + r) * kS2 + 16 * w + i];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      W2[(16 * w + 4 * q + r) * kS1 + 16 * t + i] = w2o[t][r] - a.lr * g[t][r];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (4 * q + r < kD3) W3[(4 * q + r) * kS2 + 16 * w + i] = w3o[r] - a.lr * g3[r];
  if (q == 0) {
    B2[16 * w + i] -= a.lr * sb2;                     // h = 16 w + i
    if (w == 0 && i < kD3) B3[i] -= a.lr * sb3;       // class i
  }
}

// Pull the step s_pend slot of every replica (rank-ordered sum into v) and
// apply it.  false: a peer did not arrive in time.
__device__ __forceinline__ bool pk_chain_pull_apply(const PersistArgs& a, float* lds, uint64_t s_pend,
                                                    const float4 (&pend)[10], int64_t chb, int w,
                                                    int q, int i) {
  float4 v[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) v[j] = pend[j];
  if (!px_pull_wave<10>(a, s_pend, v, chb + (int64_t)w * kPxCh, 4 * kPxCh, a.nrep * kNL1 * 4 + w, 4))
    return false;
  f32x4 g[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) g[t] = f32x4{v[t].x, v[t].y, v[t].z, v[t].w};
  pk_chain_update(a, lds, w, q, i, g, f32x4{v[8].x, v[8].y, v[8].z, v[8].w}, v[9].x, v[9].y);
  return true;
}

template <bool DP>
__device__ __forceinline__ void pk_chain(const PersistArgs& a, float* lds, int c) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int rb0 = 16 * c;  // first batch row of this chain
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  float* W2 = lds + ChLay::W2;
  float* W3 = lds + ChLay::W3;
  float* B2 = lds + ChLay::B2;
  float* B3 = lds + ChLay::B3;
  float* H1 = lds + ChLay::H1;
  float* H2 = lds + ChLay::H2;
  float* DZ2 = lds + ChLay::DZ2;
  float* DZ3 = lds + ChLay::DZ3;
  float* RED = lds + ChLay::RED;

  if (c == 0) PK_EDGE(3);
  // ---- prologue: W2, W3 (rows padded to 16 with zeros), b2, b3 ----
  // every load in one batch (one memory round trip), then the LDS stores
  constexpr int kW2Per = kD2 * (kD1 / 4) / kThreads;  // 8 float4 per thread
  constexpr int kW3Per = 16 * kD2 / kThreads;          // 4 floats per thread
  static_assert(kW2Per * kThreads == kD2 * (kD1 / 4) && kW3Per * kThreads == 16 * kD2, "prologue split");
  float4 w2v[kW2Per];
  float w3v[kW3Per];
#pragma unroll
  for (int j = 0; j < kW2Per; ++j) {
    const int e = tid + j * kThreads, r = e / (kD1 / 4), c4 = e - r * (kD1 / 4);
    w2v[j] = *reinterpret_cast<const float4*>(a.P + a.w_off[1] + (int64_t)r * kD1 + 4 * c4);
  }
#pragma unroll
  for (int j = 0; j < kW3Per; ++j) {
    const int e = tid + j * kThreads, r = e / kD2, col = e - r * kD2;
    w3v[j] = r < kD3 ? a.P[a.w_off[2] + (int64_t)min(r, kD3 - 1) * kD2 + col] : 0.f;
  }
  const float b2v = tid < kD2 ? a.P[a.b_off[1] + tid] : 0.f;
  const float b3v = tid < kD3 ? a.P[a.b_off[2] + tid] : 0.f;
#pragma unroll
  for (int j = 0; j < kW2Per; ++j) {
    const int e = tid + j * kThreads, r = e / (kD1 / 4), c4 = e - r * (kD1 / 4);
    *reinterpret_cast<float4*>(W2 + r * kS1 + 4 * c4) = w2v[j];
  }
#pragma unroll
  for (int j = 0; j < kW3Per; ++j) {
    const int e = tid + j * kThreads, r = e / kD2, col = e - r * kD2;
    W3[r * kS2 + col] = w3v[j];
  }
  if (tid < kD2) B2[tid] = b2v;
  if (tid < 16) B3[tid] = b3v;
  for (int e = tid; e < kB * kS3; e += kThreads) DZ3[e] = 0.f;
  float loss_acc = 0.f, corr_acc = 0.f, cnt_acc = 0.f;
  __syncthreads();
  if (c == 0) PK_EDGE(4);

  bool ok = true;
  const int stamp_on = g_pk_stamp_on && c == 0;
  float4 pend[10];  // DP: this wave's last pushed gradient slot, applied after the next partials
  bool have_pend = false;
  uint64_t s_pend = 0;
  const int64_t chb = (int64_t)a.nrep * kNL1 * 4 * kPxL1;  // chain slots' base
  for (int it = 0; it < a.steps && ok; ++it) {
    PK_STAMP(1, 0);
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    const int par = (int)(s & 1);
    const int64_t r0 = (int64_t)(s % (uint64_t)a.nbatches) * kB;

    // ---- H1 rows = relu(sum of the 4 k-partials) ----
    // the 32 layer-1 blocks' flags (one lane each), then this chain's 16 rows of
    // every partial in one bulk read: thread -> (gn, column n, 8 rows), 4 gk
    {
      if (tid < kNL1) {
        poll.start();
        for (;;) {
          const uint4 f = ld_gran2(rb, (kOffPf + tid) & ~(int64_t)1);
          const uint32_t ft = ((kOffPf + tid) & 1) ? f.w : f.y;
          if (ft == tag) break;
          if (!poll.again()) { ok = false; break; }
        }
      }
      ok = __syncthreads_and(ok ? 1 : 0) != 0;
      if (!ok) break;
      const int gn = tid >> 5, n = (tid >> 1) & 15, half = tid & 1;
      nu4v v[kGK][2];
#pragma unroll
      for (int gk = 0; gk < kGK; ++gk) {
        const int lb = gn + kGN * gk;
        const int off = (int)(((kOffPart * 2 + ((int64_t)lb * 16 + n) * kB + rb0 + 8 * half)) * 4);
        v[gk][0] = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, kSc1);
        v[gk][1] = __builtin_amdgcn_raw_buffer_load_b128(rb, off + 16, 0, kSc1);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float z = 0.f;
#pragma unroll
        for (int gk = 0; gk < kGK; ++gk) z += __uint_as_float(v[gk][e >> 2][e & 3]);
        H1[(rb0 + 8 * half + e) * kS1 + 16 * gn + n] = fmaxf(z, 0.f);
      }
    }
    int y = -1;
    const int srow = w * 4 + (lane >> 4);  // softmax: 16 lanes per row, 4 rows per wave
    y = a.labels[r0 + rb0 + srow];
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    if (DP && have_pend) {  // the previous step's gradient summed over the replicas, applied
      ok = __syncthreads_and(pk_chain_pull_apply(a, lds, s_pend, pend, chb, w, q, i) ? 1 : 0) != 0;
      if (!ok) break;
      have_pend = false;
      __syncthreads();  // W2 / W3 / b updated before layer 2 reads them
    }
    PK_STAMP(1, 1);

    // ---- layer 2: H2 = relu(H1 W2^T + b2), wave w -> 16 output columns ----
    {
      // four interleaved accumulator chains (a dependent MFMA waits out the
      // previous one's latency), summed in a fixed order
      f32x4 ac[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f},
                     {0.f, 0.f, 0.f, 0.f}};
      const float* ha = H1 + (rb0 + i) * kS1 + q;
      const float* wb = W2 + (16 * w + i) * kS1 + q;
#pragma unroll
      for (int ks = 0; ks < kD1 / 4; ks += 4) {
        float hv[4], wv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          hv[u] = ha[4 * (ks + u)];
          wv[u] = wb[4 * (ks + u)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) ac[u] = mfma_f32_16x16x4(hv[u], wv[u], ac[u]);
      }
      const int n = 16 * w + i;
      const float bn = B2[n];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        H2[(rb0 + 4 * q + r) * kS2 + n] = fmaxf((ac[0][r] + ac[1][r]) + (ac[2][r] + ac[3][r]) + bn, 0.f);
    }
    __syncthreads();
    // ---- layer 3 partial logits: K = 64 split over the 4 waves ----
    {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* ha = H2 + (rb0 + i) * kS2 + q;
      const float* wb = W3 + i * kS2 + q;
#pragma unroll
      for (int ks = 4 * w; ks < 4 * w + 4; ++ks) acc = mfma_f32_16x16x4(ha[4 * ks], wb[4 * ks], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) RED[w * 256 + (4 * q + r) * 16 + i] = acc[r];
    }
    __syncthreads();
    // ---- softmax + CE + dLogits ----
    {
      const int col = lane & 15;
      const bool cv = col < kD3;
      float z = -3.402823466e38f;
      if (cv) {
        z = B3[col];
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) z += RED[ww * 256 + srow * 16 + col];
      }
      float mx = z;
      int amax = cv ? col : 0x7fffffff;
      row16_argmax(mx, amax);
      const float e = cv ? expf(z - mx) : 0.f;
      const float se = row16_sum(e);
      const float p = e / se;
      float g = 0.f;
      if (cv) {
        g = (p - (col == y ? 1.f : 0.f)) * a.inv_batch;
        if (col == y) loss_acc += -logf(p + 1e-10f);
      }
      DZ3[(rb0 + srow) * kS3 + col] = g;
      if (col == 0) {
        corr_acc += amax == y ? 1.f : 0.f;
        cnt_acc += 1.f;
      }
    }
    __syncthreads();
    PK_STAMP(1, 2);
    // ---- dZ2 = (dZ3 W3) * (H2 > 0), wave w -> 16 columns ----
    {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int h = 16 * w + i;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        acc = mfma_f32_16x16x4(DZ3[(rb0 + i) * kS3 + 4 * ks + q], W3[(4 * ks + q) * kS2 + h], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = rb0 + 4 * q + r;
        DZ2[m * kS2 + h] = H2[m * kS2 + h] > 0.f ? acc[r] : 0.f;
      }
    }
    __syncthreads();
    // ---- dZ1 = (dZ2 W2) * (H1 > 0), published to the layer-1 blocks ----
    // wave w: n tiles w and w + 4, their four accumulator chains interleaved
    {
      f32x4 a0[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      f32x4 a1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < kD2 / 4; ks += 2) {
        const float d0 = DZ2[(rb0 + i) * kS2 + 4 * ks + q];
        const float d1 = DZ2[(rb0 + i) * kS2 + 4 * ks + 4 + q];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int n = 16 * (w + 4 * tt) + i;
          a0[tt] = mfma_f32_16x16x4(d0, W2[(4 * ks + q) * kS1 + n], a0[tt]);
          a1[tt] = mfma_f32_16x16x4(d1, W2[(4 * ks + 4 + q) * kS1 + n], a1[tt]);
        }
      }
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int n = 16 * (w + 4 * tt) + i;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rb0 + 4 * q + r;
          const float v = H1[m * kS1 + n] > 0.f ? a0[tt][r] + a1[tt][r] : 0.f;
          st_gran(rb, kOffDz1 + (int64_t)m * kD1 + n, v, tag);
        }
      }
    }

    PK_STAMP(1, 3);
    // ---- off the critical path: exchange rows, full-batch dW2 / dW3 ----
    {
      // own rows -> CX[par][c] as 16-B write-through vectors; every storing
      // wave drains its stores, then one lane raises the chain's flag
      typedef float f4v __attribute__((ext_vector_type(4)));
      const int mine = (int)((kOffCx * 2 + ((int64_t)par * kNCH + c) * kCXG) * 4);  // bytes
      for (int e = tid * 4; e < kCXG; e += 4 * kThreads) {
        const float* src;
        if (e < 2048) src = H1 + (rb0 + (e >> 7)) * kS1 + (e & 127);
        else if (e < 3072) src = H2 + (rb0 + ((e - 2048) >> 6)) * kS2 + ((e - 2048) & 63);
        else if (e < 4096) src = DZ2 + (rb0 + ((e - 3072) >> 6)) * kS2 + ((e - 3072) & 63);
        else src = DZ3 + (rb0 + ((e - 4096) >> 4)) * kS3 + ((e - 4096) & 15);
        const f4v v = {src[0], src[1], src[2], src[3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4v, v), rb, mine + e * 4, 0, kSc1);
      }
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) st_gran(rb, kOffCxf + (int64_t)par * kNCH + c, __uint_as_float(tag), tag);
      // the peers' flags (one lane each), then their rows in one bulk read
      if (tid < kNCH - 1) {
        const int src = (c + 1 + tid) % kNCH;
        poll.start();
        for (;;) {
          const uint4 f = ld_gran2(rb, (kOffCxf + (int64_t)par * kNCH + src) & ~(int64_t)1);
          const uint32_t ft = ((kOffCxf + par * kNCH + src) & 1) ? f.w : f.y;
          if (ft == tag) break;
          if (!poll.again()) { ok = false; break; }
        }
      }
      ok = __syncthreads_and(ok ? 1 : 0) != 0;
      if (ok) {
        constexpr int kV = kCXG / 4;                          // 1088 vectors per peer
        constexpr int kPer = ((kNCH - 1) * kV + kThreads - 1) / kThreads;  // 13
        nu4v v[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const int x = tid + j * kThreads;
          const int xc = x < (kNCH - 1) * kV ? x : 0;
          const int cs = xc / kV, e = (xc - cs * kV) * 4;
          const int src = (c + 1 + cs) % kNCH;
          const int off = (int)((kOffCx * 2 + ((int64_t)par * kNCH + src) * kCXG + e) * 4);
          v[j] = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, kSc1);
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const int x = tid + j * kThreads;
          if (x >= (kNCH - 1) * kV) continue;
          const int cs = x / kV, e = (x - cs * kV) * 4;
          const int sr0 = 16 * ((c + 1 + cs) % kNCH);
          float* dst;
          if (e < 2048) dst = H1 + (sr0 + (e >> 7)) * kS1 + (e & 127);
          else if (e < 3072) dst = H2 + (sr0 + ((e - 2048) >> 6)) * kS2 + ((e - 2048) & 63);
          else if (e < 4096) dst = DZ2 + (sr0 + ((e - 3072) >> 6)) * kS2 + ((e - 3072) & 63);
          else dst = DZ3 + (sr0 + ((e - 4096) >> 4)) * kS3 + ((e - 4096) & 15);
          const f4v f = __builtin_bit_cast(f4v, v[j]);
          dst[0] = f[0]; dst[1] = f[1]; dst[2] = f[2]; dst[3] = f[3];
        }
      }
    }
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    PK_STAMP(1, 4);
    // dW2 [64 h][128 n] = dZ2^T H1 over the 64 batch rows; wave w: h tile w, 8 n
    // tiles.  Operands are read from LDS in batches ahead of their MFMAs (one
    // read per MFMA, issued just before it, would serialise on LDS latency).
    {
      // dW3 [16 o][64 h] = dZ3^T H2 (o >= 10 rows are zero, wave w -> h tile w)
      // rides along in the same batches: its single-accumulator chain gets
      // eight independent dW2 MFMAs between consecutive steps instead of
      // stalling on the MFMA latency.  The bias gradients (column sums of dZ2,
      // dZ3) are VALU sums of the same operands.  Every accumulation runs over
      // the rows in a fixed order, identical in the four chains.
      f32x4 g[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 g3 = {0.f, 0.f, 0.f, 0.f};
      float sb2 = 0.f, sb3 = 0.f;  // bias-gradient partial sums (VALU, rows m = q mod 4)
#pragma unroll
      for (int mb = 0; mb < kB / 4; mb += 4) {
        float av[4], bv[4][8], a3[4], b3[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = 4 * (mb + u) + q;
          av[u] = DZ2[m * kS2 + 16 * w + i];
#pragma unroll
          for (int t = 0; t < 8; ++t) bv[u][t] = H1[m * kS1 + 16 * t + i];
          a3[u] = DZ3[m * kS3 + i];
          b3[u] = H2[m * kS2 + 16 * w + i];
        }
        // keep the batch's LDS reads ahead of its MFMAs (one exposed LDS
        // latency per batch instead of one per MFMA pair)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            g[t] = mfma_f32_16x16x4(av[u], bv[u][t], g[t]);
            if (t == 1) g3 = mfma_f32_16x16x4(a3[u], b3[u], g3);
          }
          sb2 += av[u];
          sb3 += a3[u];
        }
      }
      // column sums over the 4 row phases q (lanes 16 apart), fixed order
      sb2 += __shfl_xor(sb2, 16, 64);
      sb2 += __shfl_xor(sb2, 32, 64);
      sb3 += __shfl_xor(sb3, 16, 64);
      sb3 += __shfl_xor(sb3, 32, 64);
      if (DP) {
        // data parallel: push this wave's h tile to the peers now (chain c to
        // the peers d with d % 4 == c; every chain reads all), sum and apply it
        // after the next step's partials arrived -- the exchange latency hides
        // behind that wait.  Nothing reads W2 / W3 / b before then.
        pend[8] = make_float4(g3[0], g3[1], g3[2], g3[3]);
        pend[9] = make_float4(sb2, sb3, 0.f, 0.f);
#pragma unroll
        for (int t = 0; t < 8; ++t) pend[t] = make_float4(g[t][0], g[t][1], g[t][2], g[t][3]);
        px_push_wave<10>(a, s, pend, chb + (int64_t)w * kPxCh, 4 * kPxCh, a.nrep * kNL1 * 4 + w, 4,
                         kNCH, c);
        have_pend = true;
        s_pend = s;
      } else {
        PK_STAMP(1, 6);
        pk_chain_update(a, lds, w, q, i, g, g3, sb2, sb3);
        PK_STAMP(1, 7);
      }
    }
    __syncthreads();
    PK_STAMP(1, 5);
  }
  if (DP && have_pend && ok) {  // the last step's summed gradient, before the write-back
    ok = __syncthreads_and(pk_chain_pull_apply(a, lds, s_pend, pend, chb, w, q, i) ? 1 : 0) != 0;
    __syncthreads();
  }

  // ---- epilogue: stats; chain 0 writes W2, b2, W3, b3 back ----
  const float l = wave_sum(loss_acc), cr = wave_sum(corr_acc), cn = wave_sum(cnt_acc);
  if (lane == 0 && a.stats != nullptr && cn > 0.f) {
    atomicAdd(a.stats + 0, l);
    atomicAdd(a.stats + 1, cr);
    atomicAdd(a.stats + 2, cn);
  }
  if (c == 0) {
    for (int e = tid; e < kD2 * (kD1 / 4); e += kThreads) {
      const int r = e / (kD1 / 4), c4 = e - r * (kD1 / 4);
      *reinterpret_cast<float4*>(a.P + a.w_off[1] + (int64_t)r * kD1 + 4 * c4) =
          *reinterpret_cast<const float4*>(W2 + r * kS1 + 4 * c4);
    }
    for (int e = tid; e < kD3 * kD2; e += kThreads) {
      const int r = e / kD2, col = e - r * kD2;
      a.P[a.w_off[2] + (int64_t)r * kD2 + col] = W3[r * kS2 + col];
    }
    if (tid < kD2) a.P[a.b_off[1] + tid] = B2[tid];
    if (tid < kD3) a.P[a.b_off[2] + tid] = B3[tid];
  }
  pk_report(a, ok);
  if (c == 0) PK_EDGE(5);
}

// DP: the data-parallel form (replica exchange compiled in); the single-replica
// launch runs the exchange-free code.
template <bool DP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1)))
void mlp_persist_k(PersistArgs a) {
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int b = blockIdx.x;
  if (a.place == 1) {
    // the 4 chain blocks exchange rows every step: blocks 0, 8, 16, 24 share
    // one XCD under round-robin placement (speed only, the hand-offs are
    // placement-independent)
    if (b < 8 * kNCH && (b & 7) == 0)
      pk_chain<DP>(a, lds, b >> 3);
    else
      pk_layer1<DP>(a, lds, b < 8 * kNCH ? b - (b >> 3) - 1 : b - kNCH);
    return;
  }
  if (b < kNL1)
    pk_layer1<DP>(a, lds, b);
  else
    pk_chain<DP>(a, lds, b - kNL1);
}

hipError_t mlp_persist_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_pk_stamps), sizeof(uint64_t) * 3 * 8 * 8, 0,
                             hipMemcpyDeviceToHost);
}
void mlp_persist_set_stamping(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pk_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}

bool mlp_persist_supported(const MlpDesc& d) {
  return d.nlayers == 3 && d.batch == kB && d.dims[0] == kD0 && d.dims[1] == kD1 &&
         d.dims[2] == kD2 && d.dims[3] == kD3;
}

int64_t mlp_persist_xbuf_granules() { return kTotalG; }

hipError_t mlp_persist_steps(const float* X, int64_t ldx, const int32_t* labels, float* P,
                             int64_t* ctr, const MlpDesc& d, float lr, int steps, uint64_t* xb,
                             float* stats, uint32_t* err, uint32_t* herr, uint64_t timeout_ticks,
                             hipStream_t s, const XchgArgs* xa, const XchgTab* tab) {
  if (!mlp_persist_supported(d) || steps < 1 || xb == nullptr || err == nullptr || ctr == nullptr ||
      (ldx % 4) != 0)
    return hipErrorInvalidValue;
  PersistArgs a{};
  a.X = X;
  a.ldx = ldx;
  a.labels = labels;
  a.P = P;
  for (int l = 0; l < 3; ++l) {
    a.w_off[l] = d.w_off[l];
    a.b_off[l] = d.b_off[l];
  }
  a.ctr = ctr;
  a.nbatches = d.nbatches;
  a.steps = steps;
  a.lr = lr;
  a.inv_batch = 1.0f / (float)kB;
  a.xb = xb;
  a.stats = stats;
  a.err = err;
  a.herr = herr;
  a.timeout_ticks = timeout_ticks;
  a.nrep = 1;
  if (xa != nullptr && xa->nranks > 1) {
    if (tab == nullptr || xa->nranks > kMaxPeers || xa->half < px_half(xa->nranks) ||
        xa->err == nullptr)
      return hipErrorInvalidValue;
    a.xt = *tab;
    a.nrep = xa->nranks;
    a.rep = xa->rank;
    a.xhalf = xa->half;
    a.xerr = xa->err;
  }
  a.place = 1;
  const size_t lds = (size_t)kLdsFloats * sizeof(float);
  static bool attr = false;
  if (!attr) {
    for (const void* f : {reinterpret_cast<const void*>(mlp_persist_k<false>),
                          reinterpret_cast<const void*>(mlp_persist_k<true>)}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  if (a.nrep > 1)
    hipLaunchKernelGGL(mlp_persist_k<true>, dim3(kNL1 + kNCH), dim3(kThreads), lds, s, a);
  else
    hipLaunchKernelGGL(mlp_persist_k<false>, dim3(kNL1 + kNCH), dim3(kThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace dsml
