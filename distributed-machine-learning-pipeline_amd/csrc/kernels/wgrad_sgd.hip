// Weight gradient + SGD of the wide-MLP step, straight from the row-major
// activations (BASELINE config 4):
//
//   G[n][k] = alpha * sum_m Z[m][n] X[m][k]        (Z = dZ_{l+1}, X = H_l; m = batch)
//   W[n][k] -= lr * G   (fp32 master, float4 RMW)  ;  Wb[n][k] = bf16(W)   (next GEMMs' copy)
//   b[n]    -= lr * alpha * sum_m Z[m][n]          (or G / db written out for an all-reduce)
//
// The reduction runs over the batch rows, which are the STRIDED dimension of
// both stored activations: the 64 x 64 tiles of Z and X are staged row-major
// by LDS-DMA and turned into MFMA operands by ds_read_b64_tr_b16 (gfx950's
// transposing LDS read; cdna_hip_programming.md T10) — so no producer has to
// write transposed activation copies (dZ^T, H^T) any more.
//
// The kernel is bound by the fp32 master read-modify-write (+ the bf16 copy):
// every workgroup issues its W-tile loads FIRST, so that HBM round trip
// overlaps the operand staging and the MFMAs instead of following them.
// Reference hot loop replaced: the per-sample weight update of client.go:112-202.
#include <algorithm>
#include <type_traits>

#include <cstdlib>
#include "common.h"
#include "../dsml.h"

namespace dsml {
namespace {

typedef __bf16 wg_bf16x8 __attribute__((ext_vector_type(8)));
typedef short wg_i16x4 __attribute__((ext_vector_type(4)));
typedef float wg_f4 __attribute__((ext_vector_type(4)));
typedef uint32_t wg_u2 __attribute__((ext_vector_type(2)));
typedef uint32_t wg_u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void* wg_gptr;
typedef __attribute__((address_space(3))) void* wg_lptr;
typedef __attribute__((address_space(3))) wg_i16x4* wg_lv4;

constexpr int kWgImg = 64 * 128;  // one 64-row x 64-column bf16 image, 128-B rows
constexpr int kWgPitch = 68;      // floats per row of the fp32 epilogue tile

__device__ __forceinline__ int wg_swz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

typedef WgLayer WgArgs;  // dsml.h: one layer's operands, targets and step

// Split fp32 master ("hi/lo" form, WgLayer::Wl): w's bit pattern = (hi << 16)
// + lo, hi = bf16(w) rounded half away from zero in magnitude, lo = the signed
// 16-bit remainder (in [-0x8000, 0x7fff]: exactly representable, so the split
// loses nothing).  hi IS the bf16 copy the GEMMs read; the update reads and
// writes 4 B per weight (hi + lo) instead of fp32 W + the bf16 copy (4 + 4 +
// 2 B): 20 % fewer bytes in this HBM-bound kernel.
__device__ __forceinline__ float hl_join(uint32_t h, uint32_t l) {
  return __uint_as_float((h << 16) + (uint32_t)(int32_t)(int16_t)l);
}
__device__ __forceinline__ uint32_t hl_hi(float v) { return (__float_as_uint(v) + 0x8000u) >> 16; }
__device__ __forceinline__ uint32_t hl_lo(float v, uint32_t h) { return (__float_as_uint(v) - (h << 16)) & 0xffffu; }
// 8 consecutive weights of the split master: hi and lo as one 16-B word each
// (a lane's accesses stay 16 B wide: the 8-B form halved the bytes per
// vector-memory instruction and ran no faster than the fp32 form)
__device__ __forceinline__ void hl_join8(uint4 h, uint4 l, float (&w)[8]) {
  const uint32_t hw[4] = {h.x, h.y, h.z, h.w}, lw[4] = {l.x, l.y, l.z, l.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[2 * i] = hl_join(hw[i] & 0xffffu, lw[i] & 0xffffu);
    w[2 * i + 1] = hl_join(hw[i] >> 16, lw[i] >> 16);
  }
}
__device__ __forceinline__ void hl_pack8(const float (&w)[8], uint32_t (&hw)[4], uint32_t (&lw)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t h0 = hl_hi(w[2 * i]), h1 = hl_hi(w[2 * i + 1]);
    hw[i] = h0 | (h1 << 16);
    lw[i] = hl_lo(w[2 * i], h0) | (hl_lo(w[2 * i + 1], h1) << 16);
  }
}
__device__ __forceinline__ void hl_put8(const WgArgs& a, int nr, int kc, const uint32_t (&hw)[4],
                                        const uint32_t (&lw)[4]) {
  __builtin_nontemporal_store(wg_u4{hw[0], hw[1], hw[2], hw[3]},
                              reinterpret_cast<wg_u4*>(a.Wb + (int64_t)nr * a.ldwb + kc));
  __builtin_nontemporal_store(wg_u4{lw[0], lw[1], lw[2], lw[3]},
                              reinterpret_cast<wg_u4*>(a.Wl + (int64_t)nr * a.ldwl + kc));
}
__device__ __forceinline__ void hl_store8(const WgArgs& a, int nr, int kc, const float (&w)[8]) {
  uint32_t hw[4], lw[4];
  hl_pack8(w, hw, lw);
  hl_put8(a, nr, kc, hw, lw);
}

// Several layers' weight gradients in ONE launch (flattened tile grid): the
// step's last kernel updates every layer, one launch ramp and tail instead of
// one per layer.
constexpr int kWgMaxLayers = 4;
struct WgMulti {
  WgArgs l[kWgMaxLayers];
  int start[kWgMaxLayers + 1];  // first tile of each layer (prefix sums)
  int ktiles[kWgMaxLayers];
  int n;
};

// Operand fragment of the 16 x 16 x 32 MFMA: lane (i, g) gets image column
// c0 + i at rows m0 + 8g .. +7 (two transposing reads of 4 rows each).
__device__ __forceinline__ uint4 wg_frag(const char* img, int m0, int c0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int chunk = (c0 >> 3) + (p >> 1);
  const int r0 = m0 + 8 * g + q, r1 = r0 + 4;
  const wg_i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (wg_lv4)(img + r0 * 128 + 16 * (chunk ^ wg_swz(r0)) + 8 * (p & 1)));
  const wg_i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (wg_lv4)(img + r1 * 128 + 16 * (chunk ^ wg_swz(r1)) + 8 * (p & 1)));
  const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
  return make_uint4(l2.x, l2.y, h2.x, h2.y);
}

constexpr int kWgOob = 0x7ffffff0;  // byte offset of a dropped store: past every bound (host check)
constexpr int kWgLds = 64 * kWgPitch * 4;  // two operand images (16 KiB), later the fp32 tile (17 KiB)
static_assert(kWgLds >= 2 * kWgImg, "LDS carve");
// + the bias gradient's 4 row-group partials per column ([4][64] floats)
constexpr int kWgLdsTot = kWgLds + 4 * 64 * 4;

// 1. a tile's W loads (rows rl + 16j, columns cl..cl+3), issued before anything else
__device__ __forceinline__ void wg_load_w(const WgArgs& a, int kt, int nt, float4 (&wold)[4]) {
  const int tid = threadIdx.x, rl = tid >> 4, kc = kt * 64 + 4 * (tid & 15);
  const bool kv = kc < a.K;  // K % 4 == 0: a 4-column group is whole or absent
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nr = min(nt * 64 + rl + 16 * j, a.N - 1);
    wold[j] = (kv && a.W) ? *reinterpret_cast<const float4*>(a.W + (int64_t)nr * a.ldw + kc)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
// 1'. split master: rows (tid >> 3) + 32 j, columns 8 (tid & 7) .. +7 (one 16-B hi
// and one 16-B lo word per row: 8 lanes cover a tile row's 128 B)
__device__ __forceinline__ void wg_load_hl(const WgArgs& a, int kt, int nt, uint4 (&w)[4]) {
  const int tid = threadIdx.x, kc = kt * 64 + 8 * (tid & 7);
  const bool kv = kc < a.K;  // K % 8 == 0 in this form
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nr = min(nt * 64 + (tid >> 3) + 32 * j, a.N - 1);
    w[2 * j] = kv ? *reinterpret_cast<const uint4*>(a.Wh + (int64_t)nr * a.ldwh + kc) : make_uint4(0u, 0u, 0u, 0u);
    w[2 * j + 1] = kv ? *reinterpret_cast<const uint4*>(a.Wl + (int64_t)nr * a.ldwl + kc) : make_uint4(0u, 0u, 0u, 0u);
  }
}

// 2. Z[mb.., n0..] and X[mb.., k0..] as row-major images: 2 LDS-DMA pieces per wave each
// (zpre: the Z image is already in LDS -- a hand-off written by this launch)
__device__ __forceinline__ void wg_stage(const WgArgs& a, int k0, int n0, int mb, char* lds,
                                         bool zpre = false) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* imz = lds;
  char* imx = lds + kWgImg;
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) {
    const int piece = 2 * w + pc;  // 8 rows x 128 B
    const int r = 8 * piece + (lane >> 3), p = lane & 7;
    const int m = min(mb + r, a.M - 1);
    const int zc = min(n0 + 8 * (p ^ wg_swz(r)), (int)((a.N + 7) & ~7) - 8);
    const int xc = min(k0 + 8 * (p ^ wg_swz(r)), (int)((a.K + 7) & ~7) - 8);
    if (!zpre)
      __builtin_amdgcn_global_load_lds((wg_gptr)(a.Z + (int64_t)m * a.ldz + zc),
                                       (wg_lptr)(imz + piece * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((wg_gptr)(a.X + (int64_t)m * a.ldx + xc),
                                     (wg_lptr)(imx + piece * 1024), 16, 0, 0);
  }
}

// 2-4. One 64 (n) x 64 (k) tile of layer `a` (k tile kt, n tile nt) whose W
// loads are already in flight in `wold`.
__device__ __forceinline__ void wgrad_tile_body(const WgArgs& a, int kt, int nt, char* lds,
                                                const uint4 (&wr)[4], bool zpre = false) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int k0 = kt * 64, n0 = nt * 64;
  char* imz = lds;
  char* imx = lds + kWgImg;
  const int rl = tid >> 4, cl = 4 * (tid & 15);
  const int kc = k0 + cl;
  const bool kv = kc < a.K;

  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};
  float dbias = 0.f;
  const int wn = (w >> 1) * 32, wk = (w & 1) * 32;

  for (int mb = 0; mb < a.M; mb += 64) {
    // ---- 2. Z[mb.., n0..] and X[mb.., k0..] row-major images ----
    wg_stage(a, k0, n0, mb, lds, zpre);
    full_barrier();  // every piece landed (vmcnt(0) also retires the W loads: issued earlier)

    // ---- 3. MFMAs: wave tile 32 n x 32 k, reduction over the batch rows ----
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint4 fz[2], fx[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) fz[x] = wg_frag(imz, 32 * h, wn + 16 * x, lane);
#pragma unroll
      for (int y = 0; y < 2; ++y) fx[y] = wg_frag(imx, 32 * h, wk + 16 * y, lane);
      if (mb + 32 * h + 32 > a.M) {  // batch tail: rows >= M (clamped copies) contribute 0
        const int g = lane >> 4;
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          uint32_t* e = reinterpret_cast<uint32_t*>(&fz[x]);
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (mb + 32 * h + 8 * g + t >= a.M) e[t >> 1] &= (t & 1) ? 0x0000ffffu : 0xffff0000u;
        }
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wg_bf16x8, fz[x]),
                                                              __builtin_bit_cast(wg_bf16x8, fx[y]),
                                                              acc[x][y], 0, 0, 0);
    }
    // bias gradient (k-tile 0 only): column sums of the Z image, all 256
    // threads (column tid & 63, rows 16 (tid >> 6) .. +15): a quarter of the
    // serial LDS reads of one 64-thread loop, which made these tiles the grid's
    // stragglers
    if (kt == 0) {
      const int c = tid & 63, ch = c >> 3, e = c & 7, r0 = 16 * (tid >> 6);
#pragma unroll 1  // (unrolled, the loads raise VGPRs past occupancy 5)
      for (int r = r0; r < r0 + 16 && mb + r < a.M; ++r) {
        const uint16_t v = *reinterpret_cast<const uint16_t*>(imz + r * 128 + 16 * (ch ^ wg_swz(r)) + 2 * e);
        dbias += bf16_to_f32(v);
      }
    }
    lds_barrier();  // images free for the next batch block / the epilogue tile (no DMA in flight here)
  }

  // ---- 4. epilogue: acc -> LDS tile [64 n][64 k] -> float4 RMW of W + bf16 copy ----
  float* tile = reinterpret_cast<float*>(lds);
  {
    const int i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tile[(wn + 16 * x + 4 * g + r) * kWgPitch + wk + 16 * y + i] = acc[x][y][r] * a.alpha;
  }
  float* bsum = reinterpret_cast<float*>(lds + kWgLds);
  if (kt == 0) bsum[tid] = dbias;  // [row group][column]
  __syncthreads();
  if (kv) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nr = n0 + rl + 16 * j;
      if (nr >= a.N) continue;
      const float4 gv = *reinterpret_cast<const float4*>(tile + (rl + 16 * j) * kWgPitch + cl);
      if (a.W) {
        float4 v = __builtin_bit_cast(float4, wr[j]);
        v.x -= a.lr * gv.x; v.y -= a.lr * gv.y; v.z -= a.lr * gv.z; v.w -= a.lr * gv.w;
        __builtin_nontemporal_store(wg_f4{v.x, v.y, v.z, v.w},
                                    reinterpret_cast<wg_f4*>(a.W + (int64_t)nr * a.ldw + kc));
        if (a.Wb) {
          const uint32_t lo = f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16);
          const uint32_t hi = f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16);
          __builtin_nontemporal_store(wg_u2{lo, hi},
                                      reinterpret_cast<wg_u2*>(a.Wb + (int64_t)nr * a.ldwb + kc));
        }
      } else if (a.G) {
        *reinterpret_cast<float4*>(a.G + (int64_t)nr * a.ldg + kc) = gv;
      }
    }
  }
  if (a.Wl) {  // split master: 8 consecutive weights per 16-B word
    const int kc8 = k0 + 8 * (tid & 7);
    if (kc8 < a.K) {
      // both row halves packed first, the four stores issued together at the
      // end: a store between them made the compiler wait vmcnt(0) (its data
      // registers reused by the second half) -- a store round trip per tile
      uint32_t hw[2][4], lw[2][4];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rr = (tid >> 3) + 32 * j;
        const float4 g0 = *reinterpret_cast<const float4*>(tile + rr * kWgPitch + 8 * (tid & 7));
        const float4 g1 = *reinterpret_cast<const float4*>(tile + rr * kWgPitch + 8 * (tid & 7) + 4);
        float w[8];
        hl_join8(wr[2 * j], wr[2 * j + 1], w);
        w[0] -= a.lr * g0.x; w[1] -= a.lr * g0.y; w[2] -= a.lr * g0.z; w[3] -= a.lr * g0.w;
        w[4] -= a.lr * g1.x; w[5] -= a.lr * g1.y; w[6] -= a.lr * g1.z; w[7] -= a.lr * g1.w;
        hl_pack8(w, hw[j], lw[j]);
      }
      // unpredicated buffer stores (rows past N: an offset past the bound,
      // dropped) -- a predicated store let the compiler sink the second
      // half's arithmetic behind the first store again
      const __amdgpu_buffer_rsrc_t rwb = __builtin_amdgcn_make_buffer_rsrc(a.Wb, (short)0, (int)(a.N * a.ldwb * 2), 0x00020000);
      const __amdgpu_buffer_rsrc_t rwl = __builtin_amdgcn_make_buffer_rsrc(a.Wl, (short)0, (int)(a.N * a.ldwl * 2), 0x00020000);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int nr = n0 + (tid >> 3) + 32 * j;
        const bool ok = nr < a.N;
        __builtin_amdgcn_raw_buffer_store_b128(wg_u4{hw[j][0], hw[j][1], hw[j][2], hw[j][3]}, rwb,
                                               ok ? (int)((nr * a.ldwb + kc8) * 2) : kWgOob, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(wg_u4{lw[j][0], lw[j][1], lw[j][2], lw[j][3]}, rwl,
                                               ok ? (int)((nr * a.ldwl + kc8) * 2) : kWgOob, 0, 0);
      }
    }
  }
  if (kt == 0 && tid < 64 && n0 + tid < a.N) {
    const float db = a.alpha * (((bsum[tid] + bsum[64 + tid]) + bsum[128 + tid]) + bsum[192 + tid]);
    if (a.bias) a.bias[n0 + tid] -= a.lr * db;
    if (a.bgrad) a.bgrad[n0 + tid] = db;
  }
}

__device__ __forceinline__ void wgrad_tile(const WgArgs& a, int kt, int nt, char* lds) {
  // the tile's W words in one register set: fp32 W (4 float4), or for the
  // split master {hi, lo} of rows (tid >> 3) and (tid >> 3) + 32
  uint4 wr[4];
  if (a.Wl) {
    wg_load_hl(a, kt, nt, wr);
  } else {
    float4 wold[4];
    wg_load_w(a, kt, nt, wold);
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[j] = __builtin_bit_cast(uint4, wold[j]);
  }
  wgrad_tile_body(a, kt, nt, lds, wr);
}

__global__ __launch_bounds__(256) void wgrad_sgd_k(WgArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[kWgLdsTot];
  wgrad_tile(a, blockIdx.x, blockIdx.y, lds);
}

// XCD-aware tile order (speed only): blocks b and b + 8 share an XCD under
// round-robin dispatch, and each XCD has its own 4 MiB L2.  At M = 64 N rows
// a layer's operands (Z: M x N, X: M x K bf16) outgrow one L2 for N >= 4
// (8 MB at N = 8 for 4096 x 4096), and every 64 x 64 W tile reads its M-row
// column blocks of both.  So the 8 XCDs take a 2 (n) x 4 (k) grid of tile
// blocks: each XCD's tiles read 1/2 of Z's columns and 1/4 of X's (3 MB at
// N = 8), which its L2 then serves, instead of every XCD cycling through all
// of both from the shared last-level cache.  Layers whose tile grid does not
// split that way keep the row-major order.
__device__ __forceinline__ void wg_tile_xcd(int t, int kts, int nts, int& kt, int& nt) {
  const int T = kts * nts;
  if ((T & 7) == 0 && (nts & 1) == 0 && (kts & 3) == 0) {
    const int x = t & 7, r = t >> 3;
    const int bn = nts >> 1, bk = kts >> 2;  // tile block of one XCD: bn x bk tiles
    nt = (x >> 2) * bn + r / bk;
    kt = (x & 3) * bk + r % bk;
  } else {
    kt = t % kts;
    nt = t / kts;
  }
}

__global__ __launch_bounds__(256) void wgrad_multi_k(WgMulti m) {
  __shared__ __attribute__((aligned(16))) char lds[kWgLdsTot];
  const int b = blockIdx.x;
  int j = 0;
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (q < m.n && b >= m.start[q]) j = q;
  const int t = b - m.start[j];
  // layers are few: select the operands with uniform branches, no dynamic
  // indexing of the kernel-argument array
  WgArgs a = m.l[0];
  int kts = m.ktiles[0];
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (j == q) { a = m.l[q]; kts = m.ktiles[q]; }
  int kt, nt;
  // a layer's first block must sit at a multiple of 8 for its XCD map to hold
  if ((m.start[j] & 7) == 0) wg_tile_xcd(t, kts, (a.N + 63) / 64, kt, nt);
  else { kt = t % kts; nt = t / kts; }
  wgrad_tile(a, kt, nt, lds);
}

// ---------------------------------------------------------------------------
// Large-tile form: one 128 (n) x 128 (k) tile per workgroup.  Against the
// 64 x 64 tiles above it reads the activation operands once per 128 x 128 W
// elements instead of once per 64 x 64 -- half the operand bytes per W byte,
// which is what the global-batch update (xact: M = 64 N rows) pays for: 0.4 M
// / T operand bytes per W byte at tile T.  The batch streams through a 4-slot
// LDS ring of 32-row blocks (Z and X images, 16 KiB a slot) with three
// blocks in flight at every wait, so a tile's chain is about one DMA latency
// plus the MFMAs, not M / 64 dependent rounds; the fp32 W tile's loads are
// issued right after the first blocks' DMA and retire under the batch loop.
//
// The block waits are counted: the wave knows how many vector-memory loads
// it issued after the block it needs (4 LDS-DMA per block, the 16 (+1) W /
// bias loads; loads return in order; the tile has no stores before its
// epilogue) and waits with vmcnt(that).  Every LDS access of the loop is
// inline asm: the compiler cannot see which LDS bytes a DMA writes, and its
// own waits before LDS accesses would be vmcnt(0), draining the ring.
// ---------------------------------------------------------------------------
constexpr int kBgT = 128;
constexpr int kBgR = 4;                          // ring slots: 32-row batch blocks
constexpr int kBgSlot = 2 * 32 * 256;            // Z + X images of one block (256-B rows): 16 KiB
constexpr int kBgPitch = 132;                    // floats per row of the fp32 epilogue tile
constexpr int kBgTile = kBgT * kBgPitch * 4;     // 67,584 B, aliasing the ring after the loop
constexpr int kBgLds = kBgTile + 4 * kBgT * 4;   // + the bias partials [4][128]
static_assert(kBgTile >= kBgR * kBgSlot, "LDS carve");

// 16-B chunk swizzle of a 256-B image row: the 8 rows one half-wave of a
// transposing read touches (r & 3 and bit 3 vary) land in 8 different 32-B
// bank groups.
__device__ __forceinline__ int bg_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

__device__ __forceinline__ wg_u2 bg_dstr(uint32_t addr) {
  wg_u2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ uint32_t bg_dsr_u16(uint32_t addr) {
  uint32_t v;
  asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
// s_waitcnt vmcnt(n) for a wave-uniform n, rounded down to a multiple of 4
// (waiting for more is always safe); n >= 64: nothing to wait for (a wave
// never has more than 63 vector-memory instructions outstanding).
__device__ __forceinline__ void bg_vm_wait(int n) {
  switch (n < 0 ? 0 : n >> 2) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(52)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
    default: break;
  }
}

// LDS-DMA of batch block s (rows 32 s ..) of the tile: Z[.., n0 ..+127] and
// X[.., k0 ..+127]; wave w stages rows 8w .. 8w+7 of both (4 instructions).
__device__ __forceinline__ void bg_stage(const WgArgs& a, int k0, int n0, int s, char* slot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nmax = (int)((a.N + 7) & ~7) - 8, kmax = (int)((a.K + 7) & ~7) - 8;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 8 * w + 4 * j + (lane >> 4), pc = lane & 15;
    const int m = min(32 * s + r, a.M - 1);
    const int c = 8 * (pc ^ bg_swz(r));
    __builtin_amdgcn_global_load_lds((wg_gptr)(a.Z + (int64_t)m * a.ldz + min(n0 + c, nmax)),
                                     (wg_lptr)(slot + (8 * w + 4 * j) * 256), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((wg_gptr)(a.X + (int64_t)m * a.ldx + min(k0 + c, kmax)),
                                     (wg_lptr)(slot + 8192 + (8 * w + 4 * j) * 256), 16, 0, 0);
  }
}

// One 32-row block's MFMAs: wave (wn, wk) owns a 64 x 64 quadrant, 4 x 4
// tiles of 16 x 16, one 32-row reduction step.
__device__ __forceinline__ void bg_compute(uint32_t iz, int mrow0, int M, int wn, int wk, int lane,
                                           f32x4 (&acc)[4][4]) {
  const uint32_t ix = iz + 8192;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = 8 * g + q, r1 = r0 + 4;
  wg_u2 zl[4], zh[4], xl[4], xh[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const int ch = ((wn + 16 * x) >> 3) + (p >> 1);
    zl[x] = bg_dstr(iz + r0 * 256 + 16 * (ch ^ bg_swz(r0)) + 8 * (p & 1));
    zh[x] = bg_dstr(iz + r1 * 256 + 16 * (ch ^ bg_swz(r1)) + 8 * (p & 1));
  }
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    const int ch = ((wk + 16 * y) >> 3) + (p >> 1);
    xl[y] = bg_dstr(ix + r0 * 256 + 16 * (ch ^ bg_swz(r0)) + 8 * (p & 1));
    xh[y] = bg_dstr(ix + r1 * 256 + 16 * (ch ^ bg_swz(r1)) + 8 * (p & 1));
  }
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(zl[0]), "+v"(zl[1]), "+v"(zl[2]), "+v"(zl[3]), "+v"(zh[0]), "+v"(zh[1]),
                 "+v"(zh[2]), "+v"(zh[3]), "+v"(xl[0]), "+v"(xl[1]), "+v"(xl[2]), "+v"(xl[3]),
                 "+v"(xh[0]), "+v"(xh[1]), "+v"(xh[2]), "+v"(xh[3])::"memory");
  uint4 fz[4], fx[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    fz[x] = make_uint4(zl[x].x, zl[x].y, zh[x].x, zh[x].y);
    fx[x] = make_uint4(xl[x].x, xl[x].y, xh[x].x, xh[x].y);
  }
  if (mrow0 + 32 > M) {  // batch tail: rows >= M (clamped copies) contribute 0
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      uint32_t* e = reinterpret_cast<uint32_t*>(&fz[x]);
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (mrow0 + 8 * g + t >= M) e[t >> 1] &= (t & 1) ? 0x0000ffffu : 0xffff0000u;
    }
  }
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
      acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wg_bf16x8, fz[x]),
                                                          __builtin_bit_cast(wg_bf16x8, fx[y]),
                                                          acc[x][y], 0, 0, 0);
}

__device__ __forceinline__ void wgrad_big_tile(const WgArgs& a, int kt, int nt, char* lds) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int k0 = kt * kBgT, n0 = nt * kBgT;
  const int wn = (w >> 1) * 64, wk = (w & 1) * 64;
  const int nb = (a.M + 31) / 32;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(wg_lptr)lds;
  // epilogue map: float4 column group c4, rows r8 + 8j (two full 512-B rows per wave instruction)
  const int c4 = tid & 31, r8 = tid >> 5;
  const int kc = k0 + 4 * c4;
  const bool kv = kc < a.K;  // K % 4 == 0: a 4-column group is whole or absent
  // blocks 0 .. R-2 first, then the W loads; e[] = loads issued up to each block in flight
  int issued = 0, e[kBgR - 1];
#pragma unroll
  for (int q = 0; q < kBgR - 1; ++q) {
    if (q < nb) { bg_stage(a, k0, n0, q, lds + q * kBgSlot); issued += 4; }
    e[q] = issued;
  }
  asm volatile("" ::: "memory");  // the W loads follow the DMA in issue order
  // the W tile's raw words: fp32 W (rows r8 + 8j, 4 columns at kc), or for the
  // split master 8 hi + 8 lo words (rows (tid >> 4) + 16 j', 8 columns at kc8)
  uint4 wraw[16];
  const int kc8 = k0 + 8 * (tid & 15);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (a.W) {
      const int nr = min(n0 + r8 + 8 * j, a.N - 1);
      wraw[j] = *reinterpret_cast<const uint4*>(a.W + (int64_t)nr * a.ldw + min(kc, a.K - 4));
    } else if (a.Wl) {
      const int nr = min(n0 + (tid >> 4) + 16 * (j >> 1), a.N - 1), k8 = min(kc8, a.K - 8);
      wraw[j] = (j & 1) ? *reinterpret_cast<const uint4*>(a.Wl + (int64_t)nr * a.ldwl + k8)
                        : *reinterpret_cast<const uint4*>(a.Wh + (int64_t)nr * a.ldwh + k8);
    } else {
      wraw[j] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  if (a.W || a.Wl) issued += 16;
  asm volatile("" ::: "memory");
  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};
  // bias column sums, in the 64 x 64 body's order (16-row groups of every
  // 64-row block summed over the blocks, then group 0 + 1 + 2 + 3): column
  // bc; this thread's groups: bh in even 32-row blocks, 2 + bh in odd ones
  float dA = 0.f, dB = 0.f;
  const int bc = tid & 127, bh = tid >> 7;
  for (int s = 0; s < nb; ++s) {
    bg_vm_wait(issued - e[0]);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // block s landed for every wave; slot (s-1) % R free
#pragma unroll
    for (int k = 0; k < kBgR - 2; ++k) e[k] = e[k + 1];
    if (s + kBgR - 1 < nb) { bg_stage(a, k0, n0, s + kBgR - 1, lds + ((s + kBgR - 1) % kBgR) * kBgSlot); issued += 4; }
    e[kBgR - 2] = issued;
    const uint32_t slot = lds0 + (s % kBgR) * kBgSlot;
    bg_compute(slot, 32 * s, a.M, wn, wk, lane, acc);
    if (kt == 0) {
      const int ch = bc >> 3, el = bc & 7;
      uint32_t v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = 16 * bh + r;
        v[r] = bg_dsr_u16(slot + rr * 256 + 16 * (ch ^ bg_swz(rr)) + 2 * el);
      }
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                     "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]),
                     "+v"(v[13]), "+v"(v[14]), "+v"(v[15])::"memory");
      if (s & 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (32 * s + 16 * bh + r < a.M) dB += __uint_as_float(v[r] << 16);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (32 * s + 16 * bh + r < a.M) dA += __uint_as_float(v[r] << 16);
      }
    }
  }
  // every wave out of the ring (and every load retired) before the tile overwrites it
  full_barrier();
  float* tile = reinterpret_cast<float*>(lds);
  {
    const int i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tile[(wn + 16 * x + 4 * g + r) * kBgPitch + wk + 16 * y + i] = acc[x][y][r] * a.alpha;
  }
  float* bsum = reinterpret_cast<float*>(lds + kBgTile);
  if (kt == 0) { bsum[bh * kBgT + bc] = dA; bsum[(2 + bh) * kBgT + bc] = dB; }
  lds_barrier();
  if (kv) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int nr = n0 + r8 + 8 * j;
      if (nr >= a.N) continue;
      const float4 gv = *reinterpret_cast<const float4*>(tile + (r8 + 8 * j) * kBgPitch + 4 * c4);
      if (a.W) {
        float4 v = __builtin_bit_cast(float4, wraw[j]);
        v.x -= a.lr * gv.x; v.y -= a.lr * gv.y; v.z -= a.lr * gv.z; v.w -= a.lr * gv.w;
        __builtin_nontemporal_store(wg_f4{v.x, v.y, v.z, v.w},
                                    reinterpret_cast<wg_f4*>(a.W + (int64_t)nr * a.ldw + kc));
        if (a.Wb) {
          const uint32_t lo = f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16);
          const uint32_t hi = f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16);
          __builtin_nontemporal_store(wg_u2{lo, hi},
                                      reinterpret_cast<wg_u2*>(a.Wb + (int64_t)nr * a.ldwb + kc));
        }
      } else if (a.G) {
        *reinterpret_cast<float4*>(a.G + (int64_t)nr * a.ldg + kc) = gv;
      }
    }
  }
  if (a.Wl && kc8 < a.K) {  // split master: 8 consecutive weights per 16-B word
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int rr = (tid >> 4) + 16 * j, nr = n0 + rr;
      if (nr >= a.N) continue;
      const float4 g0 = *reinterpret_cast<const float4*>(tile + rr * kBgPitch + 8 * (tid & 15));
      const float4 g1 = *reinterpret_cast<const float4*>(tile + rr * kBgPitch + 8 * (tid & 15) + 4);
      float w[8];
      hl_join8(wraw[2 * j], wraw[2 * j + 1], w);
      w[0] -= a.lr * g0.x; w[1] -= a.lr * g0.y; w[2] -= a.lr * g0.z; w[3] -= a.lr * g0.w;
      w[4] -= a.lr * g1.x; w[5] -= a.lr * g1.y; w[6] -= a.lr * g1.z; w[7] -= a.lr * g1.w;
      hl_store8(a, nr, kc8, w);
    }
  }
  if (kt == 0 && tid < kBgT && n0 + tid < a.N) {
    const float db = a.alpha * (((bsum[tid] + bsum[kBgT + tid]) + bsum[2 * kBgT + tid]) + bsum[3 * kBgT + tid]);
    if (a.bias) a.bias[n0 + tid] -= a.lr * db;
    if (a.bgrad) a.bgrad[n0 + tid] = db;
  }
}

// Flattened grid over the layers; big[j] selects the 128 x 128 tile for layer j
// (the 64 x 64 body otherwise: a 10-row classifier layer is one tile row).
struct WgMultiBig {
  WgMulti m;
  int big[kWgMaxLayers];
};

__global__ __launch_bounds__(256) void wgrad_multi_big_k(WgMultiBig mb) {
  __shared__ __attribute__((aligned(16))) char lds[kBgLds];
  const WgMulti& m = mb.m;
  const int b = blockIdx.x;
  int j = 0;
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (q < m.n && b >= m.start[q]) j = q;
  const int t = b - m.start[j];
  WgArgs a = m.l[0];
  int kts = m.ktiles[0], big = mb.big[0];
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (j == q) { a = m.l[q]; kts = m.ktiles[q]; big = mb.big[q]; }
  const int nts = big ? (a.N + kBgT - 1) / kBgT : (a.N + 63) / 64;
  int kt, nt;
  if ((m.start[j] & 7) == 0) wg_tile_xcd(t, kts, nts, kt, nt);
  else { kt = t % kts; nt = t / kts; }
  if (big) wgrad_big_tile(a, kt, nt, lds);
  else wgrad_tile(a, kt, nt, lds);
}

// ---------------------------------------------------------------------------
// Row-block form for a long batch: the global-batch update of sync=xact (M =
// 64 N rows, up to 512).  At M = 512 the 64 x 64 tiles above re-read the
// activation blocks 64 x 64 KiB per tile -- 537 MB of L2 traffic for the
// 4096 x 4096 layer -- in M / 64 dependent rounds, and the 128 x 128 tiles run
// two workgroups a CU: both 74 us (profiles/r4_wide_xact_cost.json).
//
// Here a workgroup owns a run of UNITS (a unit = 128 W rows x 64 k columns;
// units in (layer, n block, k tile) order, G = #CU contiguous runs, one
// workgroup a CU).  For each n block of its run it loads the Z^T operand of
// those 128 rows ONCE into registers (MFMA A fragments for every 32-row batch
// step: wave w keeps rows 32 w .. +31, M / 32 x 2 fragments), then streams the
// X column blocks of its k tiles through an LDS ring that holds one k tile
// (M / 32 blocks of 32 rows x 64 columns, 4 KiB each, one LDS-DMA per wave per
// block).  Block b's slot is refilled with the NEXT tile's block b as soon as
// every wave has read it, so a whole k tile of X stays in flight behind the
// MFMAs; the W words of a tile (split master: hi + lo, 16 B each) are loaded
// at the tile's start and the update is stored at its end.  Every wait is an
// exact vmcnt (the issue order per wave is fixed: the ring's DMA, the W loads,
// the stores -- all unpredicated buffer ops, out-of-range words dropped by
// the descriptor), every LDS access of the loop is inline asm (the compiler's
// own waits before an LDS access would be vmcnt(0) and drain the ring).
// Activation traffic for the 4096 x 4096 layer at M = 512: X 128 MB + Z 32 MB
// (vs 537 MB), and no dependent rounds.
// ---------------------------------------------------------------------------
constexpr int kRbN = 128;                      // W rows of an n block
constexpr int kRbRing = 16 * 4096;             // one k tile of X: <= 16 blocks of 32 rows, 4 KiB each
constexpr int kRbPitch = 68;                   // floats per row of the fp32 epilogue tile [128][68]
constexpr int kRbLds = kRbRing + kRbN * kRbPitch * 4;
constexpr int kRbMaxM = 512;
constexpr int kRbMaxGroups = 256;              // workgroups of a launch (one a CU)
constexpr bool kRbAuto = true;                 // auto dispatch (tile 0) picks it at M >= 256
#if defined(HIPDSML_MEASURE) && defined(HIPDSML_RB_PAIR)
constexpr bool kRbPair = HIPDSML_RB_PAIR != 0;  // measurement builds: the single-block A/B
#else
constexpr bool kRbPair = true;
#endif
  // two ring blocks per wait / barrier (NBLK >= 4)
constexpr int kRbOob = 0x7ffffff0;             // offset of a dropped word: past every bound (host check)

struct WgRowBlk {
  WgArgs l[kWgMaxLayers];
  int ustart[kWgMaxLayers + 1];  // first unit of each layer (prefix sums); ustart[n] = all units
  int ktiles[kWgMaxLayers];
  int n;
  int groups;  // workgroups: g owns units [gstart[g], gstart[g + 1])
  int dbg;     // measurement builds only (HIPDSML_RB_DBG): bit 0/1/2 drop the W / Z / X traffic
  int gstart[kRbMaxGroups + 1];  // cost-balanced runs (wgrad_rowblk_launch)
};

// s_waitcnt vmcnt(N) with every other counter left alone (gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt[5:4] << 14).  N is a
// compile-time constant: a runtime count became a 48-way branch tree, ~50
// scalar branches per block of the ring (round 5, first cut: 83.8 us at M = 512).
template <int N>
__device__ __forceinline__ void rb_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// f(integral_constant<int, B>) for B = B0 .. N - 1 (compile-time block indices)
template <int B0, int N, class F>
__device__ __forceinline__ void rb_for(F& f) {
  if constexpr (B0 < N) {
    f(std::integral_constant<int, B0>{});
    rb_for<B0 + 1, N>(f);
  }
}
// the wait in iteration B for block B + 1 of a k tile (B = -1: block 0, before
// the loop): ops issued after it are this tile's later blocks, the last tile's
// 8 stores (tile > 0), this tile's 8 W loads and the refills of iterations
// 0 .. B - 1 (slot b takes the next tile's block b in iteration b)
template <int NBLK, int B, bool LATER, bool MORE, int NW = 8>
__device__ __forceinline__ void rb_vm_block() {
  rb_vm<(NBLK - 2 - B) + (LATER ? NW : 0) + NW + ((MORE && B > 0) ? B : 0)>();
}
__device__ __forceinline__ void rb_dsw32(uint32_t addr, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ wg_u4 rb_dsr128(uint32_t addr) {
  wg_u4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
// The same LDS accesses with a compile-time byte offset in the instruction's
// 16-bit offset field: the lane-dependent part of an address is computed once
// (per segment / tile), each block / register then costs no address VALU.
// The profiled launch issued ~5.6 VALU per MFMA, much of it address adds
// (profiles/r6_rowblk_pmc.json).
template <int OFF>
__device__ __forceinline__ void rb_dsw32_o(uint32_t addr, float v) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ wg_u4 rb_dsr128_o(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  wg_u4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ wg_u2 rb_dstr_o(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  wg_u2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
// Lane addresses (block 0 of the X ring) of the 8 transposing reads a wave
// issues per 32-row block: [y][lo, hi], y = the 16-column group; block b adds
// b * 4096 (immediate).
__device__ __forceinline__ void rb_frag_addrs(uint32_t ring, int lane, uint32_t (&fa)[4][2]) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    const int c0 = 16 * y;
    const int r0 = 8 * g + q, r1 = r0 + 4;
    const int ch = (c0 >> 3) + (p >> 1);
    fa[y][0] = ring + r0 * 128 + 16 * (ch ^ wg_swz(r0)) + 8 * (p & 1);
    fa[y][1] = ring + r1 * 128 + 16 * (ch ^ wg_swz(r1)) + 8 * (p & 1);
  }
}
__device__ __forceinline__ void rb_barrier() { asm volatile("s_barrier" ::: "memory"); }
// A or B fragment (16 x 16 x 32 bf16) from a row-major image: lane (i, g) gets
// image column c0 + i at rows 8 g .. +7 of the 32-row block (two transposing
// 8-B reads).  pitch: 128 (X blocks, wg_swz) or 256 (Z chunks, bg_swz).
template <int PITCH>
__device__ __forceinline__ void rb_frag_issue(uint32_t img, int c0, int lane, wg_u2& lo, wg_u2& hi) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int ch = (c0 >> 3) + (p >> 1);
  const int r0 = 8 * g + q, r1 = r0 + 4;
  const int s0 = PITCH == 128 ? wg_swz(r0) : bg_swz(r0), s1 = PITCH == 128 ? wg_swz(r1) : bg_swz(r1);
  lo = bg_dstr(img + r0 * PITCH + 16 * (ch ^ s0) + 8 * (p & 1));
  hi = bg_dstr(img + r1 * PITCH + 16 * (ch ^ s1) + 8 * (p & 1));
}

// WAVES: 4 (wave w owns W rows 32 w .. +31 of the 128-row unit: two 16-row
// MFMA A fragments, one wave a SIMD) or 8 (rows 16 w .. +15, one fragment, two
// waves a SIMD; bit-identical).  Only the 4-wave form is instantiated: with
// cost-balanced runs the 8-wave one measured slower (profiles/r6_rowblk_balance.json).
#ifdef HIPDSML_MEASURE
// measurement builds: per workgroup s_memrealtime at entry, the first
// segment's Z^T in registers, the end of each of its first 12 k tiles, exit
__device__ uint64_t g_rb_stamps[256][16];
__device__ int g_rb_stamp_on;
#define RB_STAMP(k)                                                                                    \
  do {                                                                                                 \
    if (g_rb_stamp_on && threadIdx.x == 0 && blockIdx.x < 256 && (k) < 16)                              \
      g_rb_stamps[blockIdx.x][(k)] = __builtin_amdgcn_s_memrealtime();                                  \
  } while (0)
#else
#define RB_STAMP(k) \
  do {              \
  } while (0)
#endif

template <int NBLK, int WAVES>
__device__ __forceinline__ void wgrad_rowblk_body(const WgRowBlk& rb) {
  static_assert(WAVES == 4 || WAVES == 8, "4 or 8 waves");
  constexpr int RW = kRbN / WAVES;       // W rows of a wave
  constexpr int XM = RW / 16;            // its 16-row MFMA A fragments
  constexpr int JJ = kRbN / (8 * WAVES);  // epilogue rows of a thread (er + 8 WAVES jj)
  constexpr int NW = 2 * JJ;             // W loads (hi + lo) and stores of a thread a tile
  constexpr int ZJ = 8 / WAVES;          // Z chunk pieces (4 rows x 256 B) a wave DMAs a chunk
  extern __shared__ __attribute__((aligned(16))) char rb_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i = lane & 15;
  const uint32_t ring = (uint32_t)(uintptr_t)(wg_lptr)rb_lds;
  const uint32_t tileb = ring + kRbRing;
  uint32_t fa[4][2];  // the 8 transposing reads' lane addresses in ring block 0
  rb_frag_addrs(ring, lane, fa);
  const int U = rb.ustart[rb.n];
  const int u0 = rb.gstart[blockIdx.x], u1 = rb.gstart[blockIdx.x + 1];
  (void)U;
  RB_STAMP(0);
  int stile = 2;  // measurement builds: the next tile stamp
  for (int u = u0; u < u1;) {
    // ---- segment: units u .. of one n block of one layer ----
    int j = 0;
#pragma unroll
    for (int q = 1; q < kWgMaxLayers; ++q)
      if (q < rb.n && u >= rb.ustart[q]) j = q;
    WgArgs a = rb.l[0];
    int kts = rb.ktiles[0];
#pragma unroll
    for (int q = 1; q < kWgMaxLayers; ++q)
      if (j == q) { a = rb.l[q]; kts = rb.ktiles[q]; }
    const int lu = u - rb.ustart[j];
    const int nb = lu / kts, kt0 = lu - nb * kts;
    const int ntl = min(u1, rb.ustart[j] + (nb + 1) * kts) - u;  // k tiles of this segment
    u += ntl;
    const int n0 = nb * kRbN;
    constexpr int nblk = NBLK;  // M = 32 NBLK (the host picks the instance)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the previous segment's stores
    rb_barrier();                                      // and every wave out of the LDS

    // Buffer-addressed LDS-DMA (32-bit per-lane offsets; 64-bit global_load_lds
    // addresses had the compiler hoist an address pair per unrolled block and
    // spill them).  Every offset is clamped inside its tensor (columns past N /
    // K re-read the row's last 8 words, as the 64 x 64 form does: they only feed
    // outputs that are never stored), so no access relies on the bounds check.
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(a.Z), (short)0, (int)(a.M * a.ldz * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(a.X), (short)0, (int)(a.M * a.ldx * 2), 0x00020000);
    const int nmax = (int)((a.N + 7) & ~7) - 8, kmax = (int)((a.K + 7) & ~7) - 8;
    int zv[ZJ];  // this lane's Z chunk offset (row r of the chunk, clamped column), bytes
#pragma unroll
    for (int jj = 0; jj < ZJ; ++jj) {
      const int r = 4 * (ZJ * w + jj) + (lane >> 4), pc = lane & 15;
      zv[jj] = (int)((r * a.ldz + min(n0 + 8 * (pc ^ bg_swz(r)), nmax)) * 2);
    }
    // X ring pieces: 4 waves send 8 rows (1 KiB) of a block each, 8 waves 4 rows (lanes 0-31)
    const int xr = (32 / WAVES) * w + (lane >> 3), xc = 8 * ((lane & 7) ^ wg_swz(xr & 31));

    // ---- Z^T fragments into registers: 32-row chunks [32][128] (256-B rows), 8 per phase ----
    wg_u4 zf[16][XM];
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      if (8 * ph < nblk) {
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
          const int c = 8 * ph + cc;
          if (c < nblk) {
#pragma unroll
            for (int jj = 0; jj < ZJ; ++jj)
              __builtin_amdgcn_raw_ptr_buffer_load_lds(rz, (wg_lptr)(rb_lds + cc * 8192 + 4 * (ZJ * w + jj) * 256), 16,
                                                      (DSML_MEASURE_KNOB(rb.dbg) & 2) ? kRbOob : zv[jj] + (int)(32 * c * a.ldz * 2), 0, 0, 0);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        rb_barrier();
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
          const int c = 8 * ph + cc;
          if (c < nblk) {
            // [c][xm]: W rows RW w + 16 xm + l % 16, batch rows 32 c + 8 (l / 16) ..
            if constexpr (XM == 2) {
              wg_u2 lo0, hi0, lo1, hi1;
              rb_frag_issue<256>(ring + cc * 8192, RW * w, lane, lo0, hi0);
              rb_frag_issue<256>(ring + cc * 8192, RW * w + 16, lane, lo1, hi1);
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo0), "+v"(hi0), "+v"(lo1), "+v"(hi1)::"memory");
              zf[c][0] = wg_u4{lo0.x, lo0.y, hi0.x, hi0.y};
              zf[c][XM - 1] = wg_u4{lo1.x, lo1.y, hi1.x, hi1.y};
            } else {
              wg_u2 lo0, hi0;
              rb_frag_issue<256>(ring + cc * 8192, RW * w, lane, lo0, hi0);
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo0), "+v"(hi0)::"memory");
              zf[c][0] = wg_u4{lo0.x, lo0.y, hi0.x, hi0.y};
            }
          }
        }
        rb_barrier();  // the chunks' slots are free again
        if (ph == 1 || 8 * (ph + 1) >= nblk) RB_STAMP(stile == 2 ? 1 : 15);
      }
    }

    // ---- bias gradient (the segment holding k tile 0): column sums of Z, from the fragments ----
    if (kt0 == 0 && (a.bias || a.bgrad)) {
      float sm[XM];
#pragma unroll
      for (int xm = 0; xm < XM; ++xm) sm[xm] = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (c < nblk) {
#pragma unroll
          for (int xm = 0; xm < XM; ++xm) {
            const wg_u4 v = zf[c][xm];
            sm[xm] += ((bf16_to_f32(v.x & 0xffffu) + bf16_to_f32(v.x >> 16)) +
                       (bf16_to_f32(v.y & 0xffffu) + bf16_to_f32(v.y >> 16))) +
                      ((bf16_to_f32(v.z & 0xffffu) + bf16_to_f32(v.z >> 16)) +
                       (bf16_to_f32(v.w & 0xffffu) + bf16_to_f32(v.w >> 16)));
          }
        }
      }
#pragma unroll
      for (int xm = 0; xm < XM; ++xm) {
        sm[xm] += __shfl_xor(sm[xm], 16, 64);
        sm[xm] += __shfl_xor(sm[xm], 32, 64);
        const int n = n0 + RW * w + 16 * xm + i;
        if (lane < 16 && n < a.N) {
          const float db = a.alpha * sm[xm];
          if (a.bias) a.bias[n] -= a.lr * db;
          if (a.bgrad) a.bgrad[n] = db;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's count starts from zero
    }

    // ---- X ring: block b of local k tile lt -> slot b (wave w: rows 8 w .. +7) ----
    auto xdma = [&](int lt, int b) __attribute__((always_inline)) {
      // 8 waves: lanes 0-31 only (a lane's LDS word is base + 16 lane: lanes
      // 32-63 would land in the next wave's rows); still one op a wave a
      // block, so the counts below are the same for every wave
      const int off = (int)(((32 * b + xr) * a.ldx + min((kt0 + lt) * 64 + xc, kmax)) * 2);
      if (WAVES == 4 || lane < 32)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (wg_lptr)(rb_lds + b * 4096 + w * (4096 / WAVES)), 16,
                                                 (DSML_MEASURE_KNOB(rb.dbg) & 4) ? kRbOob : off, 0, 0, 0);
    };
#pragma unroll
    for (int b = 0; b < 16; ++b)
      if (b < nblk) xdma(0, b);

    // bounds = the matrices' exact byte sizes: the out-of-range words' offset
    // kRbOob lies past every one of them, so those loads return 0 and those
    // stores are dropped (a bound of 0x7fffffff would have let them through)
    const int bh = (int)(a.N * a.ldwh * 2), bl = (int)(a.N * a.ldwl * 2), bw = (int)(a.N * a.ldwb * 2);
    const __amdgpu_buffer_rsrc_t rh =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.Wh), (short)0, bh, 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(a.Wl, (short)0, bl, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(a.Wb, (short)0, bw, 0x00020000);
    const int er = tid >> 3, ec = 8 * (tid & 7);  // epilogue: rows er + 8 WAVES jj, columns ec .. +7
    for (int lt = 0; lt < ntl; ++lt) {
      const int k0 = (kt0 + lt) * 64;
      const bool more = lt + 1 < ntl;
      // W words of this tile: JJ hi + JJ lo loads, always issued (out of range -> 0)
      wg_u4 whv[JJ], wlv[JJ];
#pragma unroll
      for (int jj = 0; jj < JJ; ++jj) {
        const int nr = n0 + er + 8 * WAVES * jj, kc = k0 + ec;
        const bool ok = nr < a.N && kc < a.K && !(DSML_MEASURE_KNOB(rb.dbg) & 1);
        whv[jj] = __builtin_amdgcn_raw_buffer_load_b128(rh, ok ? (int)((nr * a.ldwh + kc) * 2) : kRbOob, 0, 0);
        wlv[jj] = __builtin_amdgcn_raw_buffer_load_b128(rl, ok ? (int)((nr * a.ldwl + kc) * 2) : kRbOob, 0, 0);
      }
      f32x4 acc[XM][4];
#pragma unroll
      for (int xm = 0; xm < XM; ++xm)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[xm][y] = {0.f, 0.f, 0.f, 0.f};
      // The ring, software-pipelined: block b + 1's X fragments are read while
      // block b's MFMAs run (b: a compile-time index -- the waits' counts and the
      // Z^T fragment registers are static).  Block b was read (and its reads
      // retired) one iteration earlier, so after iteration b's barrier its slot
      // takes the next tile's block b.
      if constexpr (kRbPair && NBLK >= 4) {
        // Two blocks per wait and barrier: blocks 2j + 2 and 2j + 3 are read
        // while blocks 2j and 2j + 1 run their MFMAs -- half the waits,
        // barriers and wait-select branches of the one-block form (the launch
        // is issue-bound: 52 of 64 us at M = 512 with every byte dropped).
        // Refills stay one DMA op a block, in block order, so the counts keep
        // the one-block form's rule: waiting for block k of this tile, the ops
        // issued after it are blocks k + 1 .. NBLK - 1, the last tile's 8
        // stores, this tile's 8 W loads and this tile's refills so far.
        wg_u2 lo[2][2][4], hi[2][2][4];
        auto reads2 = [&](auto b0c, int buf) __attribute__((always_inline)) {
          constexpr int b0 = decltype(b0c)::value;
#pragma unroll
          for (int y = 0; y < 4; ++y) {  // y: the 16-column group
            lo[buf][0][y] = rb_dstr_o<b0 * 4096>(fa[y][0]);
            hi[buf][0][y] = rb_dstr_o<b0 * 4096>(fa[y][1]);
            lo[buf][1][y] = rb_dstr_o<(b0 + 1) * 4096>(fa[y][0]);
            hi[buf][1][y] = rb_dstr_o<(b0 + 1) * 4096>(fa[y][1]);
          }
        };
        auto lgkm2 = [&](int buf) __attribute__((always_inline)) {
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(lo[buf][0][0]), "+v"(lo[buf][0][1]), "+v"(lo[buf][0][2]), "+v"(lo[buf][0][3]),
                         "+v"(hi[buf][0][0]), "+v"(hi[buf][0][1]), "+v"(hi[buf][0][2]), "+v"(hi[buf][0][3]),
                         "+v"(lo[buf][1][0]), "+v"(lo[buf][1][1]), "+v"(lo[buf][1][2]), "+v"(lo[buf][1][3]),
                         "+v"(hi[buf][1][0]), "+v"(hi[buf][1][1]), "+v"(hi[buf][1][2]), "+v"(hi[buf][1][3])::"memory");
        };
        // blocks 0 and 1 (nothing of this loop issued yet)
        if (lt > 0) rb_vm<(NBLK - 2) + NW + NW>();
        else rb_vm<(NBLK - 2) + NW>();
        rb_barrier();
        reads2(std::integral_constant<int, 0>{}, 0);
        lgkm2(0);
        auto pair = [&](auto jc) __attribute__((always_inline)) {
          constexpr int j = decltype(jc)::value;
          constexpr int cur = j & 1, nxt = cur ^ 1;
          if constexpr (2 * j + 3 < NBLK) {
            // block 2j + 3 landed: refills so far 2j (this tile's slots 0 .. 2j - 1)
            constexpr int later = NBLK - 1 - (2 * j + 3);
            if (lt > 0) {
              if (more) rb_vm<later + NW + NW + 2 * j>();
              else rb_vm<later + NW + NW>();
            } else {
              if (more) rb_vm<later + NW + 2 * j>();
              else rb_vm<later + NW>();
            }
            rb_barrier();  // blocks 2j + 2, 2j + 3 landed everywhere; 2j, 2j + 1 read by all
            if (more) {
              xdma(lt + 1, 2 * j);
              xdma(lt + 1, 2 * j + 1);
            }
            reads2(std::integral_constant<int, 2 * j + 2>{}, nxt);
          }
#pragma unroll
          for (int sb = 0; sb < 2; ++sb)
#pragma unroll
            for (int y = 0; y < 4; ++y) {
              const wg_u4 fx = {lo[cur][sb][y].x, lo[cur][sb][y].y, hi[cur][sb][y].x, hi[cur][sb][y].y};
#pragma unroll
              for (int xm = 0; xm < XM; ++xm)
                acc[xm][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(wg_bf16x8, zf[2 * j + sb][xm]), __builtin_bit_cast(wg_bf16x8, fx), acc[xm][y],
                    0, 0, 0);
            }
          if constexpr (2 * j + 3 < NBLK) lgkm2(nxt);
        };
        rb_for<0, NBLK / 2>(pair);
        // this tile's W words: only the refills of slots 0 .. NBLK - 3 are younger
        if (more) rb_vm<NBLK - 2>();
        else rb_vm<0>();
      } else {
      wg_u2 lo[2][4], hi[2][4];
      auto reads = [&](auto bc, int buf) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          lo[buf][y] = rb_dstr_o<b * 4096>(fa[y][0]);
          hi[buf][y] = rb_dstr_o<b * 4096>(fa[y][1]);
        }
      };
      auto lgkm = [&](int buf) __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(lo[buf][0]), "+v"(lo[buf][1]), "+v"(lo[buf][2]), "+v"(lo[buf][3]), "+v"(hi[buf][0]),
                       "+v"(hi[buf][1]), "+v"(hi[buf][2]), "+v"(hi[buf][3])::"memory");
      };
      if (lt > 0) rb_vm_block<NBLK, -1, true, false, NW>();  // block 0 (nothing of this loop issued yet)
      else rb_vm_block<NBLK, -1, false, false, NW>();
      rb_barrier();
      reads(std::integral_constant<int, 0>{}, 0);
      lgkm(0);
      auto block = [&](auto bc) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        constexpr int cur = b & 1, nxt = cur ^ 1;
        if constexpr (b + 1 < NBLK) {
          if (lt > 0) {
            if (more) rb_vm_block<NBLK, b, true, true, NW>();
            else rb_vm_block<NBLK, b, true, false, NW>();
          } else {
            if (more) rb_vm_block<NBLK, b, false, true, NW>();
            else rb_vm_block<NBLK, b, false, false, NW>();
          }
          rb_barrier();  // block b + 1 landed everywhere; block b read by all
          if (more) xdma(lt + 1, b);
          reads(std::integral_constant<int, b + 1>{}, nxt);
        }
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const wg_u4 fx = {lo[cur][y].x, lo[cur][y].y, hi[cur][y].x, hi[cur][y].y};
#pragma unroll
          for (int xm = 0; xm < XM; ++xm)
            acc[xm][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wg_bf16x8, zf[b][xm]),
                                                                __builtin_bit_cast(wg_bf16x8, fx), acc[xm][y],
                                                                0, 0, 0);
        }
        if constexpr (b + 1 < NBLK) lgkm(nxt);
      };
      rb_for<0, NBLK>(block);
      if (more) rb_vm<NBLK - 1>();  // this tile's W words (only the refills are younger)
      else rb_vm<0>();
      }
      // ---- epilogue: alpha * G -> LDS tile [128 n][64 k] -> split-master RMW ----
      {
        const uint32_t tb = tileb + ((RW * w + 4 * g) * kRbPitch + i) * 4;
        auto st = [&](auto kc) __attribute__((always_inline)) {  // k = 16 xm + 4 y + r
          constexpr int k = decltype(kc)::value;
          constexpr int xm = k >> 4, y = (k >> 2) & 3, rr = k & 3;
          rb_dsw32_o<((16 * xm + rr) * kRbPitch + 16 * y) * 4>(tb, acc[xm][y][rr] * a.alpha);
        };
        rb_for<0, 16 * XM>(st);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      rb_barrier();  // the tile is whole; every wave has read the last block(s)
      if (more) {
        if constexpr (kRbPair && NBLK >= 4) xdma(lt + 1, nblk - 2);
        xdma(lt + 1, nblk - 1);
      }
      wg_u4 gv[JJ][2];
      {
        const uint32_t tr = tileb + (er * kRbPitch + ec) * 4;
        auto rd = [&](auto jc) __attribute__((always_inline)) {
          constexpr int jj = decltype(jc)::value;
          gv[jj][0] = rb_dsr128_o<8 * WAVES * jj * kRbPitch * 4>(tr);
          gv[jj][1] = rb_dsr128_o<8 * WAVES * jj * kRbPitch * 4 + 16>(tr);
        };
        rb_for<0, JJ>(rd);
      }
      if constexpr (JJ == 4)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(gv[0][0]), "+v"(gv[0][1]), "+v"(gv[JJ - 3][0]), "+v"(gv[JJ - 3][1]), "+v"(gv[JJ - 2][0]),
                       "+v"(gv[JJ - 2][1]), "+v"(gv[JJ - 1][0]), "+v"(gv[JJ - 1][1])::"memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(gv[0][0]), "+v"(gv[0][1]), "+v"(gv[JJ - 1][0]), "+v"(gv[JJ - 1][1])::"memory");
#pragma unroll
      for (int jj = 0; jj < JJ; ++jj) {
        const int nr = n0 + er + 8 * WAVES * jj, kc = k0 + ec;
        const bool ok = nr < a.N && kc < a.K && !(DSML_MEASURE_KNOB(rb.dbg) & 1);
        float wv[8];
        hl_join8(make_uint4(whv[jj].x, whv[jj].y, whv[jj].z, whv[jj].w),
                 make_uint4(wlv[jj].x, wlv[jj].y, wlv[jj].z, wlv[jj].w), wv);
        const float gg[8] = {__uint_as_float(gv[jj][0].x), __uint_as_float(gv[jj][0].y),
                             __uint_as_float(gv[jj][0].z), __uint_as_float(gv[jj][0].w),
                             __uint_as_float(gv[jj][1].x), __uint_as_float(gv[jj][1].y),
                             __uint_as_float(gv[jj][1].z), __uint_as_float(gv[jj][1].w)};
        uint32_t hw[4], lw[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v0 = wv[2 * e] - a.lr * gg[2 * e], v1 = wv[2 * e + 1] - a.lr * gg[2 * e + 1];
          const uint32_t h0 = hl_hi(v0), h1 = hl_hi(v1);
          hw[e] = h0 | (h1 << 16);
          lw[e] = hl_lo(v0, h0) | (hl_lo(v1, h1) << 16);
        }
        // always issued (the ring's counts assume NW stores a tile): out of range -> dropped
        __builtin_amdgcn_raw_buffer_store_b128(wg_u4{hw[0], hw[1], hw[2], hw[3]}, rw,
                                               ok ? (int)((nr * a.ldwb + kc) * 2) : kRbOob, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(wg_u4{lw[0], lw[1], lw[2], lw[3]}, rl,
                                               ok ? (int)((nr * a.ldwl + kc) * 2) : kRbOob, 0, 0);
      }
      RB_STAMP(stile);
      ++stile;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  RB_STAMP(14);
}

template <int NBLK>
__global__ __launch_bounds__(256, 1) void wgrad_rowblk_k(WgRowBlk rb) {
  wgrad_rowblk_body<NBLK, 4>(rb);
}

bool wg_valid(const WgArgs& a) {
  if (a.M < 1 || a.N < 1 || a.K < 8 || (a.K & 3) || (a.ldz & 7) || (a.ldx & 7) ||
      a.ldz < ((a.N + 7) & ~7) || a.ldx < ((a.K + 7) & ~7) || (((uintptr_t)a.Z | (uintptr_t)a.X) & 15))
    return false;
  if (a.W == nullptr && a.Wl == nullptr && a.G == nullptr && a.bias == nullptr && a.bgrad == nullptr)
    return false;
  // split master: the current hi words in, the next step's hi copy and lo (in place) out
  if (a.Wl && (a.W || a.Wh == nullptr || a.Wb == nullptr || (a.K & 7) ||
               (((uintptr_t)a.Wh | (uintptr_t)a.Wl | (uintptr_t)a.Wb) & 15) || (a.ldwh & 7) || (a.ldwl & 7) ||
               (a.ldwb & 7) || (int64_t)a.N * a.ldwb * 2 + 16 > kWgOob || (int64_t)a.N * a.ldwl * 2 + 16 > kWgOob))
    return false;  // (the tile epilogue's buffer stores: dropped rows sit past both bounds)
  if ((a.W && (((uintptr_t)a.W & 15) || (a.ldw & 3))) || (a.Wb && (((uintptr_t)a.Wb & 7) || (a.ldwb & 3))) ||
      (a.G && (((uintptr_t)a.G & 15) || (a.ldg & 3))))
    return false;
  return true;
}

}  // namespace

hipError_t wgrad_sgd(const uint16_t* Z, int64_t ldz, const uint16_t* X, int64_t ldx, int M, int N,
                     int K, float alpha, float lr, float* W, int64_t ldw, uint16_t* Wb, int64_t ldwb,
                     float* G, int64_t ldg, float* bias, float* bgrad, hipStream_t s) {
  WgArgs a{Z, ldz, X, ldx, M, N, K, alpha, lr, W, ldw, Wb, ldwb, G, ldg, bias, bgrad};
  if (!wg_valid(a)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wgrad_sgd_k, dim3((K + 63) / 64, (N + 63) / 64), dim3(256), 0, s, a);
  return hipGetLastError();
}

// The row-block form's launch (see wgrad_rowblk_k); false: a layer does not fit it.
static bool rowblk_fits(const WgLayer& L) {
  return L.Wl != nullptr && L.W == nullptr && L.G == nullptr &&
         (L.M == 64 || L.M == 128 || L.M == 256 || L.M == kRbMaxM) &&
         (int64_t)L.M * L.ldz * 2 < 0x7fffffff && (int64_t)L.M * L.ldx * 2 < 0x7fffffff &&
         (int64_t)L.N * L.ldwb * 2 + 16 <= kRbOob && (int64_t)L.N * L.ldwl * 2 + 16 <= kRbOob &&
         (int64_t)L.N * L.ldwh * 2 + 16 <= kRbOob;
}
// Workgroup runs of the row-block form's units (layer j, 128-row n block, 64-deep
// k tile; launch order), balanced by cost, not unit count: every segment a
// workgroup starts (a new n block) pays its Z^T load and a cold X ring first
// -- ~2.3 k tiles' worth at M = 512 (profiles/r6_rowblk_balance.json) -- so an
// equal split of units left the workgroups whose run crossed an n block ~10 us
// behind the median.  Greedy fill against a target, the target bisected to the
// smallest that fits `groups` runs.  The segment overhead in k tiles: the
// stamps price it at ~2.3 at M = 512, but a sweep of the model's constant put
// the launch's end earliest at 1.5 (M = 512: 1.0 60.2 us, 1.5 48.7, 2.0 50.3,
// 2.3 50.5).  Writes starts[0 .. runs] and returns the number of runs.
int wgrad_rowblk_plan(const int* N, const int* K, int n, int groups, int* starts) {
  int u = 0;
  for (int j = 0; j < n; ++j) u += ((K[j] + 63) / 64) * ((N[j] + kRbN - 1) / kRbN);
  const double ov = 1.5;
  auto fill = [&](double T, int* st) -> int {
    int g = 0;
    double cur = 0.0;
    int prev_seg = -1;
    if (st) st[0] = 0;
    for (int j = 0, uu = 0, us = 0; j < n; ++j) {
      const int kts = (K[j] + 63) / 64, nbs = (N[j] + kRbN - 1) / kRbN;
      for (int nbk = 0; nbk < nbs; ++nbk) {
        for (int kt = 0; kt < kts; ++kt, ++uu) {
          const int seg = us + nbk * kts;  // the unit's segment id (first unit of its n block)
          double c = 1.0 + ((cur == 0.0 || seg != prev_seg) ? ov : 0.0);
          if (cur > 0.0 && cur + c > T) {  // close this workgroup's run
            ++g;
            if (st) st[g] = uu;
            cur = 0.0;
            c = 1.0 + ov;
          }
          cur += c;
          prev_seg = seg;
        }
      }
      us += kts * nbs;
    }
    ++g;
    if (st) st[g] = u;
    return g;
  };
  double lo = 1.0, hi = (double)u * (1.0 + ov) + 1.0;
  for (int it = 0; it < 40; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (fill(mid, nullptr) <= groups) hi = mid;
    else lo = mid;
  }
  return fill(hi, starts);
}
static hipError_t wgrad_rowblk_launch(const WgLayer* layers, int n, hipStream_t s) {
  WgRowBlk rb{};
  rb.n = n;
  int u = 0;
  for (int j = 0; j < n; ++j) {
    rb.l[j] = layers[j];
    rb.ustart[j] = u;
    rb.ktiles[j] = (layers[j].K + 63) / 64;
    u += rb.ktiles[j] * ((layers[j].N + kRbN - 1) / kRbN);
  }
  for (int j = n; j <= kWgMaxLayers; ++j) rb.ustart[j] = u;
  for (int j = n; j < kWgMaxLayers; ++j) { rb.l[j] = layers[0]; rb.ktiles[j] = rb.ktiles[0]; }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const void* fs[4] = {reinterpret_cast<const void*>(wgrad_rowblk_k<2>), reinterpret_cast<const void*>(wgrad_rowblk_k<4>),
                         reinterpret_cast<const void*>(wgrad_rowblk_k<8>), reinterpret_cast<const void*>(wgrad_rowblk_k<16>)};
    for (const void* f : fs) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kRbLds);
      if (e != hipSuccess) { cus = 0; return e; }
    }
  }
  // (wgrad_rowblk_plan: runs balanced by a cost model)
  const int G = std::min(std::min(cus, u), kRbMaxGroups);
  // the split depends only on the shapes: computed once per shape set (a host
  // bisection per launch cost ~90 us of launch rate in an eager loop)
  struct Plan {
    int key[2 + 2 * kWgMaxLayers];
    int groups;
    int gstart[kRbMaxGroups + 1];
  };
  static Plan cache[8];
  static int ncache = 0;
  int key[2 + 2 * kWgMaxLayers] = {n, layers[0].M};
  for (int j = 0; j < n; ++j) { key[2 + 2 * j] = layers[j].N; key[3 + 2 * j] = layers[j].K; }
  const Plan* hit = nullptr;
  for (int c = 0; c < ncache && !hit; ++c)
    if (std::equal(key, key + 2 + 2 * kWgMaxLayers, cache[c].key)) hit = &cache[c];
  if (hit == nullptr) {
    int Ns[kWgMaxLayers], Ks[kWgMaxLayers];
    for (int j = 0; j < n; ++j) { Ns[j] = layers[j].N; Ks[j] = layers[j].K; }
    Plan& pl = cache[ncache < 8 ? ncache++ : 7];
    std::copy(key, key + 2 + 2 * kWgMaxLayers, pl.key);
    pl.groups = wgrad_rowblk_plan(Ns, Ks, n, G, pl.gstart);
    hit = &pl;
  }
  rb.groups = hit->groups;
  std::copy(hit->gstart, hit->gstart + hit->groups + 1, rb.gstart);
#ifdef HIPDSML_MEASURE
  static const int rb_dbg = getenv("HIPDSML_RB_DBG") ? atoi(getenv("HIPDSML_RB_DBG")) : 0;
  rb.dbg = rb_dbg;
#else
  rb.dbg = 0;
#endif
  switch (layers[0].M) {
    case 64: hipLaunchKernelGGL(wgrad_rowblk_k<2>, dim3(rb.groups), dim3(256), kRbLds, s, rb); break;
    case 128: hipLaunchKernelGGL(wgrad_rowblk_k<4>, dim3(rb.groups), dim3(256), kRbLds, s, rb); break;
    case 256: hipLaunchKernelGGL(wgrad_rowblk_k<8>, dim3(rb.groups), dim3(256), kRbLds, s, rb); break;
    default: hipLaunchKernelGGL(wgrad_rowblk_k<16>, dim3(rb.groups), dim3(256), kRbLds, s, rb); break;
  }
  return hipGetLastError();
}

#ifdef HIPDSML_MEASURE
hipError_t wgrad_rowblk_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_rb_stamps), sizeof(uint64_t) * 256 * 16, 0, hipMemcpyDeviceToHost);
}
void wgrad_rowblk_set_stamping(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rb_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
#endif
namespace {
// ---------------------------------------------------------------------------
// The wide step's input layer as strips inside the update launch (one replica,
// batch 64): the work of kernels/wide_input.hip -- dZ_1 from the last dgrad's
// raw slices, the W_0 / b_0 step, the NEXT step's H_1 -- re-cut for this
// launch's 256-thread, <= 96-register, <= 32 KiB workgroups, so that 256
// strip workgroups (16 rows of W_0 each, first in the grid) run beside the
// 64 x 64 tiles of the layers above: their load / store phases, which left HBM
// idle between them in a launch of their own (profiles/r6_wide_fused_input.json),
// overlap the tiles' weight stream.  Same arithmetic and orders as wide_input.hip
// (bit-identical): wave w takes input chunks w and w + 4 of gemm_rows64_k's
// 8-chunk split one after the other, its chunk-w forward partial goes to LDS,
// the chunk-(w + 4) one stays in registers until the first four are summed.
constexpr int kWsZp = 72;                                // bf16 a row of the dZ_1^T image [16][64 + 8]
constexpr int kWsScP = 36;                               // floats a row of a wave's gradient tile [16][32 + 4]
constexpr int kWsRedP = 17;                              // floats a row of a chunk's forward partial [64][16 + 1]
constexpr int kWsOffSc = 16 * kWsZp * 2;                 // 2,304
constexpr int kWsOffP = kWsOffSc + 4 * 16 * kWsScP * 4;  // + 9,216
constexpr int kWsLds = kWsOffP + 4 * 64 * kWsRedP * 4;   // + 17,408 = 28,928: still 5 workgroups a CU
static_assert(kWsLds >= kWgLdsTot && kWsLds <= 32 * 1024, "LDS carve");

struct WgMultiIn {
  WgMulti m;
  WideInArgs in;
  int strips;  // in.N / 16 strip workgroups, then m's tiles
};

__device__ __forceinline__ uint4 ws_zero() { return make_uint4(0u, 0u, 0u, 0u); }
__device__ __forceinline__ f32x4 ws_mfma(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wg_bf16x8, a), __builtin_bit_cast(wg_bf16x8, b),
                                                  c, 0, 0, 0);
}

template <int S>
__device__ __forceinline__ void wide_strip(const WideInArgs& a, int sb, char* lds) {
  uint16_t* zt = reinterpret_cast<uint16_t*>(lds);
  float* sc = reinterpret_cast<float*>(lds + kWsOffSc);
  float* P = reinterpret_cast<float*>(lds + kWsOffP);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 15, g = lane >> 4;
  const int n0 = sb * 16, K = a.K;

  // ---- A. dZ_1 [64 m][16 n]: thread -> row tid >> 2, columns 4 (tid & 3) .. +3 ----
  {
    const int zm = tid >> 2, zn = 4 * (tid & 3);
    const int tile = n0 >> 6, nl = (n0 & 63) + zn;
    float4 sl[S];
#pragma unroll
    for (int z = 0; z < S; ++z)
      sl[z] = *reinterpret_cast<const float4*>(a.slabs + ((int64_t)z * a.tiles + tile) * 4096 + zm * 64 + nl);
    const uint2 mk = *reinterpret_cast<const uint2*>(a.H1 + (int64_t)zm * a.ldh1 + n0 + zn);
    float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);  // the split-K combine's order
#pragma unroll
    for (int z = 0; z < S; ++z) {
      sm.x += sl[z].x; sm.y += sl[z].y; sm.z += sl[z].z; sm.w += sl[z].w;
    }
    float x[4] = {sm.x * a.zalpha + a.zbias, sm.y * a.zalpha + a.zbias, sm.z * a.zalpha + a.zbias,
                  sm.w * a.zalpha + a.zbias};
    const uint32_t mw[4] = {mk.x << 16, mk.x & 0xffff0000u, mk.y << 16, mk.y & 0xffff0000u};
    uint16_t q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (!(__uint_as_float(mw[e]) > 0.f)) x[e] = 0.f;
      q[e] = f32_to_bf16(x[e]);
      zt[(zn + e) * kWsZp + zm] = q[e];
    }
    if (a.dzo)
      *reinterpret_cast<uint2*>(a.dzo + (int64_t)zm * a.lddz + n0 + zn) =
          make_uint2(q[0] | ((uint32_t)q[1] << 16), q[2] | ((uint32_t)q[3] << 16));
  }
  const float bold = a.bias[n0 + (tid & 15)];
  lds_barrier();
  uint4 zf[2];  // A fragments: dZ_1 column n0 + i, batch rows 32h + 8g .. +7
#pragma unroll
  for (int h = 0; h < 2; ++h) zf[h] = *reinterpret_cast<const uint4*>(zt + i * kWsZp + 32 * h + 8 * g);
  if (w == 0) {  // the bias gradient's four 16-row partial column sums
    const int c = lane & 15, qq = lane >> 4;
    float d = 0.f;
#pragma unroll
    for (int r = 16 * qq; r < 16 * qq + 16; ++r) d += bf16_to_f32(zt[c * kWsZp + r]);
    sc[qq * 16 + c] = d;
  }
  lds_barrier();
  if (tid < 16) {
    const float db = a.alpha * (((sc[tid] + sc[16 + tid]) + sc[32 + tid]) + sc[48 + tid]);
    float b = bold;
    b -= a.lr * db;
    a.bias[n0 + tid] = b;
    sc[64 + tid] = b;
  }
  lds_barrier();
  const float bnv = sc[64 + (tid & 15)];  // the updated bias of this thread's output column
  lds_barrier();                          // sc is the gradient tile from here on

  // ---- B. chunks w, then w + 4: per 32-column step the gradient MFMAs, the
  // update (new hi words = the forward's B fragments), the forward MFMAs ----
  float* mysc = sc + w * 16 * kWsScP;
  // buffer-addressed (32-bit lane offsets: 64-bit pointers per stream spilled)
  const __amdgpu_buffer_rsrc_t rwh = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.Wh), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwl = __builtin_amdgcn_make_buffer_rsrc(a.Wl, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwb = __builtin_amdgcn_make_buffer_rsrc(a.Wb, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rxg = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.XG), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rxf = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.XF), (short)0, 0x7fffffff, 0x00020000);
  const int owh = (int)((n0 + i) * a.ldwh * 2), owl = (int)((n0 + i) * a.ldwl * 2), owb = (int)((n0 + i) * a.ldwb * 2);
  const int oxg = 64 * i + 16 * g, oxf = 64 * i + 16 * g;
  f32x4 af2[4];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    const int c = w + 4 * cc;
    const int kb = a.kq * c, ke = min(K, kb + a.kq);
    f32x4 af[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) af[t] = {0.f, 0.f, 0.f, 0.f};
    if (kb < ke) {  // wave-uniform (chunk 7 of 784 inputs is empty)
#pragma unroll 1
      for (int u = 0; u < 4; ++u) {
        const int ks = kb + 32 * u;
        const int k = ks + 8 * g;
        const bool kvl = k < ke;
        const int kc = kvl ? k : 0;
        // the step's loads in one batch (W from HBM first)
        const uint4 wh = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rwh, owh + 2 * kc, 0, 0));
        const uint4 wl = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rwl, owl + 2 * kc, 0, 0));
        uint4 xf[2][2];
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          const int ky = ks + 16 * y;
          const int kg = ky < ke ? ky >> 4 : 0;
#pragma unroll
          for (int h = 0; h < 2; ++h)
            xf[y][h] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rxg, oxg + kg * 2048 + 1024 * h, 0, 0));
        }
        const int kx = ks < ke ? ks : 0;
        uint4 fa[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          fa[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rxf, oxf + (kx >> 5) * 4096 + 1024 * t, 0, 0));
        uint4 bw = ws_zero();
        if (ks < ke) {  // wave-uniform
          f32x4 acc[2];
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            acc[y] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[y] = ws_mfma(zf[h], xf[y][h], acc[y]);
          }
#pragma unroll
          for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r) mysc[(4 * g + r) * kWsScP + 16 * y + i] = acc[y][r] * a.alpha;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const float4 g0 = *reinterpret_cast<const float4*>(mysc + i * kWsScP + 8 * g);
          const float4 g1 = *reinterpret_cast<const float4*>(mysc + i * kWsScP + 8 * g + 4);
          if (kvl) {
            float wv[8];
            hl_join8(wh, wl, wv);
            wv[0] -= a.lr * g0.x; wv[1] -= a.lr * g0.y; wv[2] -= a.lr * g0.z; wv[3] -= a.lr * g0.w;
            wv[4] -= a.lr * g1.x; wv[5] -= a.lr * g1.y; wv[6] -= a.lr * g1.z; wv[7] -= a.lr * g1.w;
            uint32_t nh[4], nlw[4];
            hl_pack8(wv, nh, nlw);
            __builtin_amdgcn_raw_buffer_store_b128(wg_u4{nh[0], nh[1], nh[2], nh[3]}, rwb, owb + 2 * k, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(wg_u4{nlw[0], nlw[1], nlw[2], nlw[3]}, rwl, owl + 2 * k, 0, 0);
            bw = make_uint4(nh[0], nh[1], nh[2], nh[3]);
          }
          __builtin_amdgcn_wave_barrier();  // the tile's reads done before the next step rewrites it
        }
        // gemm_rows64_k's step: zero operands past the chunk (it issues them too)
#pragma unroll
        for (int t = 0; t < 4; ++t) af[t] = ws_mfma(kvl ? fa[t] : ws_zero(), kvl ? bw : ws_zero(), af[t]);
      }
    }
    if (cc == 0) {
      float* mine = P + w * 64 * kWsRedP;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mine[(16 * t + 4 * g + r) * kWsRedP + i] = af[t][r];
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) af2[t] = af[t];
    }
  }
  lds_barrier();
  // ---- C. the chunk partials in chunk order, the updated bias, ReLU -> bf16 ----
  const int on = tid & 15;
  float xs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = ((tid >> 4) + 16 * j) * kWsRedP + on;
    float x = P[o];
#pragma unroll
    for (int qq = 1; qq < 4; ++qq) x += P[qq * 64 * kWsRedP + o];
    xs[j] = x;
  }
  lds_barrier();
  {
    float* mine = P + w * 64 * kWsRedP;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mine[(16 * t + 4 * g + r) * kWsRedP + i] = af2[t][r];
  }
  lds_barrier();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = (tid >> 4) + 16 * j;
    const int o = m * kWsRedP + on;
    float x = xs[j];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) x += P[qq * 64 * kWsRedP + o];
    x *= a.falpha;
    x += bnv;
    x = fmaxf(x, 0.f);
    a.Hn[(int64_t)m * a.ldhn + n0 + on] = f32_to_bf16(x);
  }
}

template <int S>
__global__ __launch_bounds__(256, 5) void wgrad_multi_in_k(WgMultiIn mi) {
  __shared__ __attribute__((aligned(16))) char lds[kWsLds];
  const int b0 = blockIdx.x;
  if (b0 < mi.strips) {
    wide_strip<S>(mi.in, b0, lds);
    return;
  }
  const WgMulti& m = mi.m;
  const int b = b0 - mi.strips;
  int j = 0;
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (q < m.n && b >= m.start[q]) j = q;
  const int t = b - m.start[j];
  WgArgs a = m.l[0];
  int kts = m.ktiles[0];
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (j == q) { a = m.l[q]; kts = m.ktiles[q]; }
  int kt, nt;
  if ((m.start[j] & 7) == 0) wg_tile_xcd(t, kts, (a.N + 63) / 64, kt, nt);
  else { kt = t % kts; nt = t / kts; }
  wgrad_tile(a, kt, nt, lds);
}
}  // namespace

hipError_t wgrad_sgd_multi_in(const WgLayer* layers, int n, const WideInArgs& in, hipStream_t s) {
  if (n < 1 || n > kWgMaxLayers || wide_input_check(in) != hipSuccess) return hipErrorInvalidValue;
  WgMultiIn mi{};
  WgMulti& m = mi.m;
  m.n = n;
  int t = 0;
  for (int j = 0; j < n; ++j) {
    const WgLayer& L = layers[j];
    if (!wg_valid(L) || L.M != 64) return hipErrorInvalidValue;
    m.l[j] = L;
    m.start[j] = t;
    m.ktiles[j] = (L.K + 63) / 64;
    t += m.ktiles[j] * ((L.N + 63) / 64);
  }
  for (int j = n; j <= kWgMaxLayers; ++j) m.start[j] = t;
  for (int j = n; j < kWgMaxLayers; ++j) { m.l[j] = layers[0]; m.ktiles[j] = m.ktiles[0]; }
  mi.in = in;
  mi.strips = in.N / 16;  // a multiple of 8 keeps the tiles' XCD map (block b % 8)
  if (mi.strips & 7) return hipErrorInvalidValue;
  const dim3 grid(mi.strips + t);
  switch (in.S) {
    case 1: hipLaunchKernelGGL(wgrad_multi_in_k<1>, grid, dim3(256), 0, s, mi); break;
    case 2: hipLaunchKernelGGL(wgrad_multi_in_k<2>, grid, dim3(256), 0, s, mi); break;
    case 4: hipLaunchKernelGGL(wgrad_multi_in_k<4>, grid, dim3(256), 0, s, mi); break;
    default: hipLaunchKernelGGL(wgrad_multi_in_k<8>, grid, dim3(256), 0, s, mi); break;
  }
  return hipGetLastError();
}

hipError_t wgrad_sgd_multi(const WgLayer* layers, int n, hipStream_t s, int tile) {
  if (n < 1 || n > kWgMaxLayers || (tile != 0 && tile != 64 && tile != kBgT && tile != kWgRowBlkTile))
    return hipErrorInvalidValue;
  // the row-block form when asked for (tile kWgRowBlkTile) or, auto, at M >= 256
  // (M = 256 / 512: 47.3 / 64.7 us against 48.0 / 73.5 for the 64 x 64 tiles,
  // profiles/r5_wide_xact_cost.json; below 256 the square tiles are faster)
  bool rows = tile == kWgRowBlkTile || (tile == 0 && kRbAuto);
  for (int j = 0; j < n && rows; ++j)
    rows = wg_valid(layers[j]) && rowblk_fits(layers[j]) && layers[j].M == layers[0].M &&
           (tile == kWgRowBlkTile || layers[j].M >= 256);
  if (tile == kWgRowBlkTile && !rows) return hipErrorInvalidValue;
  if (rows) return wgrad_rowblk_launch(layers, n, s);
  WgMultiBig mb{};
  WgMulti& m = mb.m;
  m.n = n;
  int t = 0, any_big = 0;
  for (int j = 0; j < n; ++j) {
    const WgLayer& L = layers[j];
    if (!wg_valid(L)) return hipErrorInvalidValue;
    // 128 x 128 tiles where the layer fills them (a 10-row classifier does
    // not) and, by default, only for the fp32-master form at a long batch: the
    // 64 x 64 body's 5 workgroups per CU hide the W round trip better
    // (MI355X, 784-4096-4096-10 shapes, us at M = 64 / 128 / 256 / 512: fp32
    // form 34.9 / 40.2 / 54.7 / 78.6 against 39.7 / 45.5 / 55.6 / 74.9; split
    // master 31.3 / 36.7 / 48.9 / 72.8 against 38.2 / 43.4 / 53.6 / 74.7 --
    // profiles/r3_wide_xact_cost.json)
    const int big = L.N >= kBgT && L.K >= kBgT &&
                    (tile == kBgT || (tile == 0 && L.M >= 512 && L.W != nullptr));
    const int T = big ? kBgT : 64;
    mb.big[j] = big;
    any_big |= big;
    m.l[j] = L;
    m.start[j] = t;
    m.ktiles[j] = (L.K + T - 1) / T;
    t += m.ktiles[j] * ((L.N + T - 1) / T);
  }
  for (int j = n; j <= kWgMaxLayers; ++j) m.start[j] = t;
  for (int j = n; j < kWgMaxLayers; ++j) { m.l[j] = layers[0]; m.ktiles[j] = m.ktiles[0]; mb.big[j] = mb.big[0]; }
  if (any_big)
    hipLaunchKernelGGL(wgrad_multi_big_k, dim3(t), dim3(256), 0, s, mb);
  else
    hipLaunchKernelGGL(wgrad_multi_k, dim3(t), dim3(256), 0, s, m);
  return hipGetLastError();
}



namespace {
__global__ void hilo_split_k(const float* __restrict__ W, int N, int K, int64_t ldw, uint16_t* __restrict__ hi,
                             int64_t ldh, uint16_t* __restrict__ lo, int64_t ldl) {
  const int64_t total = (int64_t)N * K;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = e / K, k = e - n * K;
    const float v = W[n * ldw + k];
    const uint32_t h = hl_hi(v);
    hi[n * ldh + k] = (uint16_t)h;
    lo[n * ldl + k] = (uint16_t)hl_lo(v, h);
  }
}
__global__ void hilo_join_k(const uint16_t* __restrict__ hi, int64_t ldh, const uint16_t* __restrict__ lo,
                            int64_t ldl, int N, int K, float* __restrict__ W, int64_t ldw) {
  const int64_t total = (int64_t)N * K;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = e / K, k = e - n * K;
    W[n * ldw + k] = hl_join(hi[n * ldh + k], lo[n * ldl + k]);
  }
}
__global__ void hilo_sgd_k(const uint16_t* __restrict__ hic, int64_t ldc, uint16_t* __restrict__ lo, int64_t ldl,
                           const float* __restrict__ G, int64_t ldg, int N, int K, float lr,
                           uint16_t* __restrict__ hin, int64_t ldn) {
  const int64_t total = (int64_t)N * K;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = e / K, k = e - n * K;
    float w = hl_join(hic[n * ldc + k], lo[n * ldl + k]);
    if (G) w -= lr * G[n * ldg + k];
    const uint32_t h = hl_hi(w);
    hin[n * ldn + k] = (uint16_t)h;
    lo[n * ldl + k] = (uint16_t)hl_lo(w, h);
  }
}
}  // namespace

hipError_t hilo_sgd(const uint16_t* hic, int64_t ldc, uint16_t* lo, int64_t ldl, const float* G, int64_t ldg,
                    int N, int K, float lr, uint16_t* hin, int64_t ldn, hipStream_t s) {
  if (N <= 0 || K <= 0) return hipSuccess;
  const int64_t total = (int64_t)N * K;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(hilo_sgd_k, dim3(grid), dim3(256), 0, s, hic, ldc, lo, ldl, G, ldg, N, K, lr, hin, ldn);
  return hipGetLastError();
}

hipError_t hilo_split(const float* W, int N, int K, int64_t ldw, uint16_t* hi, int64_t ldh, uint16_t* lo,
                      int64_t ldl, hipStream_t s) {
  if (N <= 0 || K <= 0) return hipSuccess;
  const int64_t total = (int64_t)N * K;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(hilo_split_k, dim3(grid), dim3(256), 0, s, W, N, K, ldw, hi, ldh, lo, ldl);
  return hipGetLastError();
}
hipError_t hilo_join(const uint16_t* hi, int64_t ldh, const uint16_t* lo, int64_t ldl, int N, int K, float* W,
                     int64_t ldw, hipStream_t s) {
  if (N <= 0 || K <= 0) return hipSuccess;
  const int64_t total = (int64_t)N * K;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(hilo_join_k, dim3(grid), dim3(256), 0, s, hi, ldh, lo, ldl, N, K, W, ldw);
  return hipGetLastError();
}

}  // namespace dsml
