// Activation-exchange data parallelism for the fused fp32 MLP step ("xact").
//
// The gradient all-reduce the reference performs every step
// (gpu_coordinator_server.go:272-566, client.go:614-640) moves
// the whole 437 KB weight gradient of 784-128-64-10.  With a 64-row batch per
// GPU that is the wrong thing to put on an xGMI link: every weight gradient is
// dW_l = dZ_l^T . H_{l-1} over the batch rows, and the factors are far smaller
// than the product (dZ_1 is 64 x 128, dW_1 is 128 x 784).  So instead of
// reducing dW, every replica PUSHES its activations and activation gradients
// (H_1, dZ_1, H_2, dZ_2, dZ_3: the workspace image written by K_B, 100 KB) into
// every peer's receive buffer, and every replica then computes the weight
// gradients of the WHOLE global batch itself:
//
//     dW_l = sum_r dZ_{l,r}^T . H_{l-1,r}       (r = 0..N-1 in rank order)
//
// with H_0 = X read from the replicated dataset shard of rank r (MNIST-scale
// data fits every GPU's HBM many times over).  Per step each xGMI link carries
// 100 KB instead of 437 KB (one-shot) and no reduction crosses a link; the
// price is N x the (tiny) weight-gradient FLOPs on every GPU, which MFMA
// absorbs.  Sums run in the same order on every rank, so replicas stay
// bit-identical, and the result equals the all-reduced gradient up to fp32
// summation order.
//
// One launch replaces K_C:
//   blocks [0, S x G)       pushers: block (s, g) loads 16-column strip s of
//                           this rank's H_l / dZ_l from the workspace
//                           (coalesced), transposes it through LDS into
//                           fragment order and writes it into this rank's
//                           receive slot of the ranks of destination group g
//                           (G = 1 group with 4-wave blocks; with 8-wave blocks
//                           G = N/2 groups of 2 ranks, one per 256-thread half,
//                           so no CU issues more than one remote store per
//                           thread); all groups cover every rank, itself
//                           included, so tile blocks read all N images the same
//                           way.  16 B system-scope stores (sc0 sc1) over xGMI,
//                           drained, then flag (me, s) in each destination's
//                           memory.  Pushers never wait.
//   blocks [S x G, ...)     one 16(n) x 32(k) tile of some dW_l per block,
//                           4 (or 8) waves splitting the N x B/4 k-steps; they
//                           poll only LOCAL flags, and only those of the <= 3
//                           strips they read, load the N images from local HBM
//                           with sc0 sc1 16 B loads, reduce the 4 wave partials
//                           through LDS in wave order, apply SGD (lr / N).
// Pushers have the lowest block ids, so they are dispatched before any tile
// block can occupy a CU: a GPU never waits on work it has not started.
// Receive slots alternate by step parity (a peer is at most one step ahead).
//
// Fragment-order images.  A replica's image is not the workspace layout: the
// pushers gather it into the MFMA operand order of v_mfma_f32_16x16x4_f32, so
// a tile wave fetches its 4 k-steps of a 16-column strip with ONE 16 B load
// per lane.  For an activation matrix M [B x D] (B <= 64 rows, zero-padded),
// strip t (columns 16t..16t+15) is 1024 floats laid out [w][lane][j]:
//     img[t][w][lane = 16q + i][j] = M[row = 4w + 16j + q][col = 16t + i]
// i.e. wave w's k-steps are s = w + 4j (rows 4s + q), lane (i, q) holds the
// operand value of k-step s.  The input batch X is kept in the same order on
// the host side (parallel/xchg.py swizzle_inputs), shard by shard.
#include "common.h"
#include "../dsml.h"

namespace dsml {

namespace {

typedef __attribute__((address_space(1))) uint64_t xa_u64;
typedef float xa_f4 __attribute__((ext_vector_type(4)));
constexpr int kSys = 1 | 16;  // buffer aux: sc0 | sc1 = system scope

__device__ __forceinline__ void xa_st_flag(uint64_t* p, uint64_t v) {
  __hip_atomic_store((xa_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t xa_ctr(const int64_t* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t xa_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}

// Waves per block: 4, or 8 from N = 4 ranks on (the wave halves then split the
// ranks, halving each wave's loads and MFMA chain; pushers split the ranks).
constexpr int kStrip = 1024;  // floats of one 16-column strip of an image matrix

// a[k] for a runtime k from a kernel-argument array, by selects (a dynamic
// index would copy the array to scratch memory first)
template <typename T>
__device__ __forceinline__ T xa_pick(const T (&a)[kMaxPeers], int k) {
  T r = a[0];
#pragma unroll
  for (int j = 1; j < kMaxPeers; ++j) r = k == j ? a[j] : r;
  return r;
}

// Phase stamps (s_memrealtime, 100 MHz) of pusher block 0 ([0, 8)) and of the
// first tile block ([8, 16)), profiling only (tools/xact_stamps.py).
__device__ uint64_t g_xact_stamps[kMaxStamps];
__device__ int g_xact_stamp_on;
#define XA_STAMP(i)                                                                     \
  do {                                                                                  \
    if (stamp_on && threadIdx.x == 0) g_xact_stamps[(i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

__host__ __device__ inline int xa_strips(int D) { return (D + 15) >> 4; }

// Image segment of layer l's matrix: which = 0 -> H_l (1 <= l < L), 1 -> dZ_l (1 <= l <= L).
// Returns its float offset; segments follow ws order (H_1, dZ_1, H_2, dZ_2, ..., dZ_L).
__host__ __device__ inline int64_t xa_seg_off(const MlpDesc& d, int l, int which) {
  int64_t off = 0;
  for (int m = 1; m <= d.nlayers; ++m) {
    const int64_t sz = (int64_t)xa_strips(d.dims[m]) * kStrip;
    if (m < d.nlayers) {
      if (m == l && which == 0) return off;
      off += sz;
    }
    if (m == l && which == 1) return off;
    off += sz;
  }
  return off;  // total
}

// Segment of image strip s: layer m's H (which 0) or dZ (which 1), strip t of it.
__device__ __forceinline__ void xa_strip_seg(const MlpDesc& d, int s, int& m, int& which,
                                             int& t) {
  int base = 0;
  for (m = 1; m <= d.nlayers; ++m) {
    const int n = xa_strips(d.dims[m]);
    if (m < d.nlayers) {
      if (s < base + n) { which = 0; t = s - base; return; }
      base += n;
    }
    if (s < base + n) { which = 1; t = s - base; return; }
    base += n;
  }
  m = d.nlayers; which = 1; t = 0;  // unreachable for s < nstrips
}

template <int WV>
__global__ __launch_bounds__(64 * WV) void mlp_f32_wgrad_xact_k(
    const float* __restrict__ Xswz, int64_t xstride, float* __restrict__ P,
    const float* __restrict__ ws, int64_t* __restrict__ ctr, MlpDesc d, float lr, XchgArgs xa,
    XchgTab tab, int nstrips) {
  constexpr int NH = WV / 4;  // rank phases: wave w serves ranks r with r % NH == w / 4
  __shared__ float red[WV][9][64];  // pushers reuse it as the 64 x 17 transpose tile
  __shared__ int flag_ok;
  const uint64_t step = xa_ctr(ctr) - 1;  // K_A advanced A to step + 1
  const uint64_t want = step + 1;
  const int N = xa.nranks, me = xa.rank;
  // the peer pointer table arrives by value in the kernel arguments: no
  // dependent load before the first store or poll address is known
  const int64_t par = (int64_t)(step & 1) * xa.half;
  const int64_t payload = (int64_t)nstrips * kStrip;
  const int tid = threadIdx.x;
  const int B = d.batch;
  // pusher blocks: (strip, destination group); each writes its strip to <= NH
  // ranks (one per 256-thread half), so no CU issues more than NH remote stores
  // per thread (the store issue rate, not the links, bounded one block per strip)
  const int G = NH == 2 ? (N + 1) / 2 : 1;  // destination groups (= pusher blocks per strip)
  const int per = (N + G - 1) / G;          // destinations per pusher block
  const int npush = nstrips * G;
  const int stamp_on = g_xact_stamp_on && (blockIdx.x == 0 || (int)blockIdx.x == npush);

  if ((int)blockIdx.x < npush) {
    XA_STAMP(0);
    // ------------------------------------------------------------- pusher --
    // Block (s, grp): strip s of this rank's image -> ranks grp + G * half.
    const int s = blockIdx.x % nstrips, grp = blockIdx.x / nstrips;
    int m, which, t;
    xa_strip_seg(d, s, m, which, t);
    const int D = d.dims[m];
    const float* src = ws + (which ? d.dz_off[m] : d.act_off[m]);
    float* tile = &red[0][0][0];
    const int t2 = tid & 255, half = tid >> 8;
    if (half == 0) {  // 64 rows x 16 columns, one float4 per thread, zero-padded
      const int row = tid >> 2, c0 = 16 * t + 4 * (tid & 3);
      float v[4];
      if (row < B && (D & 3) == 0 && c0 + 3 < D) {
        const float4 x = *reinterpret_cast<const float4*>(src + (int64_t)row * D + c0);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] = (row < B && c0 + k < D) ? src[(int64_t)row * D + c0 + k] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) tile[row * 17 + 4 * (tid & 3) + k] = v[k];
    }
    __syncthreads();
    XA_STAMP(1);
    const int w = t2 >> 6, ln = t2 & 63, i = ln & 15, q = ln >> 4;
    xa_f4 f;
#pragma unroll
    for (int j = 0; j < 4; ++j) f[j] = tile[(4 * w + 16 * j + q) * 17 + i];
    const int64_t off = (int64_t)me * payload + (int64_t)s * kStrip + t2 * 4;  // floats
    for (int h = half; h < per; h += NH) {
      const int dst = grp + G * h;
      if (dst < N)
        __builtin_amdgcn_raw_buffer_store_b128(f, xa_rsrc(xa_pick(tab.buf, dst) + par),
                                               (int)(off * 4), 0, kSys);
    }
    XA_STAMP(2);
    // every storing wave drains its stores, then one lane per rank raises the flag
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    XA_STAMP(3);
    if (tid < per && grp + G * tid < N)
      xa_st_flag(xa_pick(tab.flags, grp + G * tid) + me * nstrips + s, want);
    if (blockIdx.x == 0 && tid == 0) {
      // step-counter hand-off B = A (the tile blocks never read B)
      __hip_atomic_store(reinterpret_cast<uint64_t*>(ctr + 1), xa_ctr(ctr), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }

  // ------------------------------------------------------------------ tile --
  XA_STAMP(8);
  int bid = blockIdx.x - npush;
  int l = 0;
  for (; l < d.nlayers - 1; ++l) {
    const int nt = ((d.dims[l + 1] + 15) >> 4) * ((d.dims[l] + 31) >> 5);
    if (bid < nt) break;
    bid -= nt;
  }
  const int Nn = d.dims[l + 1], K = d.dims[l];
  const int ntk = (K + 31) >> 5;
  const int tn = bid / ntk, tk = bid - tn * ntk;
  const int lane = tid & 63, w = tid >> 6, i = lane & 15, q = lane >> 4;
  const int wq = w & 3, hr = w >> 2;  // fragment row group; rank phase
  const int n = tn * 16 + i;
  const int k0 = tk * 32 + i, k1 = k0 + 16;
  const bool nv = n < Nn, k0v = k0 < K, k1v = k1 < K;
  const bool s1v = 32 * tk + 16 < K;  // second 16-column strip of the tile exists
  const int nc = nv ? n : Nn - 1, k0c = k0v ? k0 : K - 1, k1c = k1v ? k1 : K - 1;
  const int64_t woff = d.w_off[l];

  // old weights of this tile (wave 0 applies the update) — issued early
  float wold[4][2] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
  float bold = 0.f;
  if (w == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = tn * 16 + 4 * q + r;
      const float* wr = P + woff + (int64_t)(row < Nn ? row : Nn - 1) * K;
      wold[r][0] = wr[k0c];
      wold[r][1] = wr[k1c];
    }
    bold = P[d.b_off[l] + nc];
  }

  // Layer 0's B operand is this step's input rows of every rank, read from the
  // local replicated shards: no peer involved, so those loads go out BEFORE the
  // flag poll and land while it waits.
  const int64_t frag = (int64_t)wq * 256 + lane * 4;  // floats within a strip
  const int64_t s0 = (int64_t)(2 * tk) * kStrip + frag, s1 = s0 + kStrip;
  xa_f4 av[kMaxPeers], b0[kMaxPeers], b1[kMaxPeers];
  if (l == 0) {
    const int64_t bat = (int64_t)(step % (uint64_t)d.nbatches) * xa_strips(K) * kStrip;
#pragma unroll
    for (int r = 0; r < kMaxPeers; ++r) {
      if (r < N && r % NH == hr) {
        const float* xr = Xswz + (int64_t)r * xstride + bat;
        b0[r] = *reinterpret_cast<const xa_f4*>(xr + s0);
        b1[r] = s1v ? *reinterpret_cast<const xa_f4*>(xr + s1) : xa_f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }

  XA_STAMP(9);
  // wait for the strips this tile reads, from every rank (local flags):
  // threads [0,64) poll dZ_{l+1} strip tn, [64,128) H_l strip 2tk, [128,192) 2tk+1
  const int sdz = (int)(xa_seg_off(d, l + 1, 1) / kStrip) + tn;
  const int sh = l == 0 ? -1 : (int)(xa_seg_off(d, l, 0) / kStrip) + 2 * tk;
  // LDS-only barriers around the poll: __syncthreads() would also wait for the
  // input-fragment and old-weight loads above (s_waitcnt vmcnt(0)), serialising
  // their memory round trip with the poll's instead of overlapping the two.
  if (tid == 0) flag_ok = 1;
  lds_barrier();
  {
    const int part = tid >> 6, src = tid & 63;
    const int strip = part == 0 ? sdz : (sh < 0 || (part == 2 && !s1v) ? -1 : sh + part - 1);
    if (part < 3 && src < N && strip >= 0) {
      if (!poll_flag_ge<1>(xa_pick(tab.flags, me) + src * nstrips + strip, want, xa.err,
                           xa.timeout_ticks))
        flag_ok = 0;
    }
  }
  lds_barrier();  // every poller is done; flag_ok (LDS) is final
  XA_STAMP(10);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below the poll

  // The exchanged operands: one 16 B fragment load per matrix strip and lane.
  const __amdgpu_buffer_rsrc_t rv = xa_rsrc(xa_pick(tab.buf, me) + par);
  const int64_t dzo = (int64_t)sdz * kStrip + frag;
  const int64_t ao = l == 0 ? 0 : (int64_t)sh * kStrip - (int64_t)(2 * tk) * kStrip;
#pragma unroll
  for (int r = 0; r < kMaxPeers; ++r) {
    if (r < N && r % NH == hr) {
      const int64_t img = (int64_t)r * payload;
      av[r] = __builtin_amdgcn_raw_buffer_load_b128(rv, (int)((img + dzo) * 4), 0, kSys);
      if (l != 0) {
        b0[r] = __builtin_amdgcn_raw_buffer_load_b128(rv, (int)((img + ao + s0) * 4), 0, kSys);
        b1[r] = s1v ? __builtin_amdgcn_raw_buffer_load_b128(rv, (int)((img + ao + s1) * 4), 0, kSys)
                    : xa_f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
#pragma unroll
  for (int r = 0; r < kMaxPeers; ++r) {
    if (r < N && r % NH == hr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // zero padding rows/columns contribute 0
        dbacc += av[r][j];
        acc0 = mfma_f32_16x16x4(av[r][j], b0[r][j], acc0);
        acc1 = mfma_f32_16x16x4(av[r][j], b1[r][j], acc1);
      }
    }
  }
  XA_STAMP(11);
  dbacc += __shfl_xor(dbacc, 16, 64);
  dbacc += __shfl_xor(dbacc, 32, 64);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[w][r][lane] = acc0[r];
    red[w][4 + r][lane] = acc1[r];
  }
  red[w][8][lane] = dbacc;
  __syncthreads();
  XA_STAMP(12);
  if (w != 0 || !flag_ok) return;  // a timed-out peer: leave the weights alone
  float s0v[4], s1v4[4], sb = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) s0v[r] = s1v4[r] = 0.f;
#pragma unroll
  for (int v = 0; v < WV; ++v) {  // wave order: identical on every rank
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s0v[r] += red[v][r][lane];
      s1v4[r] += red[v][4 + r][lane];
    }
    sb += red[v][8][lane];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = tn * 16 + 4 * q + r;
    if (row < Nn) {
      float* wr = P + woff + (int64_t)row * K;
      if (k0v) wr[k0] = wold[r][0] - lr * s0v[r];
      if (k1v) wr[k1] = wold[r][1] - lr * s1v4[r];
    }
  }
  if (tk == 0 && q == 0 && nv) P[d.b_off[l] + n] = bold - lr * sb;
  if (stamp_on) {
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    XA_STAMP(13);
  }
}

}  // namespace

hipError_t mlp_read_stamps_xact(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_xact_stamps), sizeof(uint64_t) * kMaxStamps, 0,
                             hipMemcpyDeviceToHost);
}

void mlp_set_stamping_xact(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_xact_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}

int mlp_xact_payload(const MlpDesc& d) { return (int)xa_seg_off(d, d.nlayers + 1, 0); }

bool mlp_xact_supported(const MlpDesc& d) {
  if (d.batch > 64) return false;
  for (int l = 0; l < d.nlayers; ++l)
    if (d.dims[l] % 16) return false;  // K of every weight gradient: whole 16-column strips
  return true;
}

hipError_t mlp_f32_wgrad_xact(const float* Xswz, int64_t xstride, float* P, const float* ws,
                              int64_t* ctr, const MlpDesc& d, float lr_over_n, const XchgArgs& x,
                              const XchgTab& tab, int waves, hipStream_t s) {
  const int payload = mlp_xact_payload(d);
  const int nstrips = payload / kStrip;
  if (ctr == nullptr || x.tab == nullptr || x.err == nullptr || x.nranks < 1 ||
      x.nranks > kMaxPeers || x.rank < 0 || x.rank >= x.nranks || !mlp_xact_supported(d) ||
      x.half < (int64_t)x.nranks * payload || (int64_t)2 * x.half * 4 > 0x7fffffffLL ||
      xstride < (int64_t)d.nbatches * xa_strips(d.dims[0]) * kStrip ||
      (waves != 0 && waves != 4 && waves != 8))
    return hipErrorInvalidValue;
  const bool eight = waves == 8 || (waves == 0 && x.nranks >= 4);
  const int G = eight ? (x.nranks + 1) / 2 : 1;  // pusher blocks per strip
  dim3 grid(nstrips * G + mlp_wgrad_tiles(d));
  if (eight)
    hipLaunchKernelGGL(mlp_f32_wgrad_xact_k<8>, grid, dim3(512), 0, s, Xswz, xstride, P, ws, ctr,
                       d, lr_over_n, x, tab, nstrips);
  else
    hipLaunchKernelGGL(mlp_f32_wgrad_xact_k<4>, grid, dim3(256), 0, s, Xswz, xstride, P, ws, ctr,
                       d, lr_over_n, x, tab, nstrips);
  return hipGetLastError();
}

}  // namespace dsml
