// The wide classifier head's row work (kernels/gemm_bf16.hip head_softmax_xent_k;
// a header so another kernel can host the row work -- the dgrad-hosted form was
// measured slower, profiles/r5_head_dgrad_fusion_ab.json): logits[m][c] =
// H[m] . W[c] + b[c] for C <= 16 classes, softmax-CE, dLogits, and the next
// activation gradient dZ_prev[m] = (sum_c dZ[m][c] W[c]) * (H[m] > 0), for one
// row per 256-thread workgroup.  Both products run on packed-bf16 dot
// instructions (v_dot2c_f32_bf16: two bf16 MACs per lane per issue, straight
// from the loaded bf16 pairs, no unpacking): the logits pair k-neighbours, the
// activation gradient pairs class neighbours (one v_perm per output pair).
// The per-class block sum is a DPP row sum per class + 16 row partials through
// LDS (no bank conflicts: the r4 LDS transpose read 16 consecutive floats per
// lane, 71 % conflicted).  Every load of a thread goes out in one unpredicated
// batch (a predicated load compiled to a branch whose copy-out waited vmcnt(0):
// three serialised L2 round trips in the r4 ISA).
// Reference: the client's softmax and loss gradient (DSML/client/client.go:76-90
// softmax, :143-165 backwardPass: loss and dLogits), one batch row per workgroup here.
#pragma once
#include "common.h"

namespace dsml {

struct HeadRow {
  const uint16_t* H;  // [B][ldh] bf16 activations of the last hidden layer
  int64_t ldh;
  const uint16_t* W;  // [C][ldw] bf16 classifier weights
  int64_t ldw;
  const float* bias;
  int K, C, Cp;
  const int32_t* labels;
  float inv_batch;
  float* logits;  // nullable, [B][ldl]
  int64_t ldl;
  uint16_t* dz;  // [B][ldz] bf16 dLogits (Cp columns)
  int64_t ldz;
  uint16_t* dzT;  // nullable
  int64_t ldt;
  float* stats;  // nullable: loss / correct / count (row_stats: [B][4] per row)
  uint16_t* dzp;  // nullable: [B][ldzp] bf16 activation gradient of the layer below
  int64_t ldzp;
  uint16_t* dzpT;  // nullable
  int64_t ldpt;
  int row_stats;
  int dbg;  // measurement builds only: bit 0 skips the stats, bit 1 the dzp phase
  // H from a raw split-K GEMM instead (head_row<MAXC, SL>, SL slices): H[m][k] =
  // bf16(relu(hs_alpha * sum_z hs[z * hs_stride + (k / 64) * 4096 + m * 64 + k % 64]
  // + hs_bias[k])), summed in slice order like gemm_skinny's own combine, and
  // stored to hout (rows <= 64: one 64-row tile block)
  const float* hs;
  int64_t hs_stride;
  float hs_alpha;
  const float* hs_bias;
  int hs_relu;
  uint16_t* hout;
  int64_t ldho;
};
constexpr int kHeadMaxC = 16;  // classes the head supports (instantiated for <= 10 and <= 16)
constexpr int kHeadMaxK8 = 2;  // 16 B chunks of the row per thread: K <= 256 * 8 * 2 = 4096

typedef __bf16 hbf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float hdot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(hbf2, a), __builtin_bit_cast(hbf2, b), c, false);
}
__device__ __forceinline__ float hdot8(const uint4& a, const uint4& b, float c) {
  return hdot2(a.w, b.w, hdot2(a.z, b.z, hdot2(a.y, b.y, hdot2(a.x, b.x, c))));
}
#define HR_STAMP(k)                                                             \
  do {                                                                          \
    if (stamps && t == 0) stamps[(k)] = __builtin_amdgcn_s_memrealtime();       \
  } while (0)

// Row m; part: LDS [MAXC][17] floats, gz2: LDS [MAXC / 2] words; stamps:
// nullable [6] (profiling).  Ends with an LDS-only barrier after its LDS use.
// SL > 0: H comes as SL raw split-K slices (HeadRow::hs), combined on load.
template <int MAXC, int SL = 0>
__device__ __forceinline__ void head_row(const HeadRow& h, int m, float (*part)[17], uint32_t* gz2,
                                         uint64_t* stamps) {
  static_assert(MAXC % 2 == 0 && MAXC <= 16, "class pairs, one 16-lane row");
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint16_t* H = h.H;
  const int64_t ldh = h.ldh, ldw = h.ldw, ldl = h.ldl, ldz = h.ldz, ldt = h.ldt, ldzp = h.ldzp, ldpt = h.ldpt;
  const uint16_t* W = h.W;
  const float* bias = h.bias;
  const int K = h.K, C = h.C, Cp = h.Cp, row_stats = h.row_stats, dbg = DSML_MEASURE_KNOB(h.dbg);
  const int32_t* labels = h.labels;
  const float inv_batch = h.inv_batch;
  float* logits = h.logits;
  float* stats = h.stats;
  uint16_t* dz = h.dz;
  uint16_t* dzT = h.dzT;
  uint16_t* dzp = h.dzp;
  uint16_t* dzpT = h.dzpT;
  const uint16_t* hr = H + (int64_t)m * ldh;
  // the softmax's own operands go out with the first loads (not after the reduction)
  HR_STAMP(0);
  const int y = labels[m];
  const float bc = bias ? bias[min(lane, C - 1)] : 0.f;  // lanes >= C: unused
  // this row's own loss / correct / count accumulators (row_stats: only this
  // workgroup touches them): read now, under the operand loads, and written
  // back with one plain store after the softmax -- a read-modify-write with
  // no round trip of its own (device atomics there kept the kernel's tail
  // waiting 1.8 us for their completion: head_bench dbg1)
  // (a wave-uniform condition: a scalar load; under a per-lane one it was a
  // branch whose copy-out waited for the load before the operand batch)
  // Unconditional (absent: H's first words, dropped at the use): a load under
  // even a uniform condition became a branch whose copy-out waited for it.
  const bool rst = row_stats && stats;
  float4 racc = *reinterpret_cast<const float4*>(rst ? stats + 4 * (int64_t)m : reinterpret_cast<const float*>(H));
  // every load of the thread in one batch, unpredicated (clamped addresses,
  // out-of-range chunks zeroed after): its H chunks and the same chunks of all
  // C rows of W.  A predicated load is a branch around it, and the compiler
  // waited for each branch's load before the next (three serialised L2 round
  // trips in the r4 head's ISA).  Rows past C load row C - 1: their logits are
  // never read and their dLogits are 0.
  uint4 hv[kHeadMaxK8], wv[kHeadMaxK8][MAXC];
  // raw split-K slices (SL > 0): 8 consecutive floats of every slice per chunk,
  // plus the chunk's bias (absent: the slice's own words, dropped at the use)
  float4 sv[SL > 0 ? SL : 1][kHeadMaxK8][2], bv[kHeadMaxK8][2];
#pragma unroll
  for (int j = 0; j < kHeadMaxK8; ++j) {
    const int k = min((t + 256 * j) * 8, K - 8);
    if constexpr (SL == 0) {
      hv[j] = *reinterpret_cast<const uint4*>(hr + k);
    } else {
      const float* sb = h.hs + (int64_t)(k >> 6) * 4096 + m * 64 + (k & 63);
#pragma unroll
      for (int z = 0; z < SL; ++z) {
        sv[z][j][0] = *reinterpret_cast<const float4*>(sb + z * h.hs_stride);
        sv[z][j][1] = *reinterpret_cast<const float4*>(sb + z * h.hs_stride + 4);
      }
      const float* bp = h.hs_bias ? h.hs_bias + k : sb;
      bv[j][0] = *reinterpret_cast<const float4*>(bp);
      bv[j][1] = *reinterpret_cast<const float4*>(bp + 4);
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      wv[j][c] = *reinterpret_cast<const uint4*>(W + (int64_t)min(c, C - 1) * ldw + k);
  }
  if constexpr (SL > 0) {
    // gemm_skinny's combine order (0 + slice 0 + slice 1 + ...), then its
    // epilogue (alpha, bias, ReLU, bf16): the same bits as the combined GEMM
#pragma unroll
    for (int j = 0; j < kHeadMaxK8; ++j) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = 0.f;
#pragma unroll
      for (int z = 0; z < SL; ++z) {
        x[0] += sv[z][j][0].x; x[1] += sv[z][j][0].y; x[2] += sv[z][j][0].z; x[3] += sv[z][j][0].w;
        x[4] += sv[z][j][1].x; x[5] += sv[z][j][1].y; x[6] += sv[z][j][1].z; x[7] += sv[z][j][1].w;
      }
      const float b8[8] = {bv[j][0].x, bv[j][0].y, bv[j][0].z, bv[j][0].w,
                           bv[j][1].x, bv[j][1].y, bv[j][1].z, bv[j][1].w};
      uint32_t q[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float y = x[e] * h.hs_alpha + (h.hs_bias ? b8[e] : 0.f);
        if (h.hs_relu) y = fmaxf(y, 0.f);
        q[e] = f32_to_bf16(y);
      }
      hv[j] = make_uint4(q[0] | (q[1] << 16), q[2] | (q[3] << 16), q[4] | (q[5] << 16), q[6] | (q[7] << 16));
      const int k = (t + 256 * j) * 8;
      if (k < K && h.hout) *reinterpret_cast<uint4*>(h.hout + (int64_t)m * h.ldho + k) = hv[j];
    }
  }
#pragma unroll
  for (int j = 0; j < kHeadMaxK8; ++j)
    if ((t + 256 * j) * 8 >= K) hv[j] = make_uint4(0u, 0u, 0u, 0u);  // zero H: zero products
  float acc[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    acc[c] = 0.f;
#pragma unroll
    for (int j = 0; j < kHeadMaxK8; ++j) acc[c] = hdot8(hv[j], wv[j][c], acc[c]);
  }
  HR_STAMP(1);
  // block reduction per class: DPP sum over each 16-lane row, 16 row partials via LDS
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const float v = row16_sum(acc[c]);
    if ((lane & 15) == 0) part[c][4 * w + (lane >> 4)] = v;
  }
  lds_barrier();  // LDS only: no wait for this block's global stores
  HR_STAMP(2);
  if (w == 0) {
    const int c = lane;
    const bool cv = c < C;
    float z = -3.402823466e38f;
    if (cv) {
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) v += part[c][r];
      z = v + bc;
    }
    if (cv && logits) logits[(int64_t)m * ldl + c] = z;
    // every class sits in lanes 0-15 (C <= 16): 16-lane DPP reductions
    // instead of 64-lane shuffles (each an LDS-path ds_bpermute round trip)
    float mx = z;
    int am = cv ? c : 0x7fffffff;
    row16_argmax(mx, am);
    const float e = cv ? expf(z - mx) : 0.f;
    const float se = row16_sum(e);
    const float p = e / se;
    const float gr = cv ? (p - (c == y ? 1.f : 0.f)) * inv_batch : 0.f;
    const uint16_t hq = f32_to_bf16(gr);
    if (c < Cp) {
      dz[(int64_t)m * ldz + c] = hq;
      if (dzT) dzT[(int64_t)c * ldt + m] = hq;
    }
    // class pairs for the packed dZ pass: lane 2i packs (its, lane 2i+1's)
    const uint32_t hi = (uint32_t)__shfl_xor((int)hq, 1);
    if (c < MAXC && !(c & 1)) gz2[c >> 1] = (uint32_t)hq | (hi << 16);
    if (c == y && stats && !(dbg & 1)) {
      if (row_stats) {
        if (!rst) racc = make_float4(0.f, 0.f, 0.f, 0.f);
        racc.x += -logf(p + 1e-10f);
        racc.y += am == y ? 1.f : 0.f;
        racc.z += 1.f;
        *reinterpret_cast<float4*>(stats + 4 * (int64_t)m) = racc;
      } else {
        atomicAdd(stats + 0, -logf(p + 1e-10f));
        atomicAdd(stats + 1, am == y ? 1.f : 0.f);
        atomicAdd(stats + 2, 1.f);
      }
    }
  }
  HR_STAMP(3);
  if (dzp == nullptr || (dbg & 2)) return;
  // ---- fused activation gradient of the layer below (the NEXT backward GEMM):
  // dZ_prev[m][k] = (sum_c dZ[m][c] W[c][k]) * (H[m][k] > 0), from the W and H
  // chunks this thread already holds; bf16 row store + transposed copy.
  lds_barrier();  // LDS only: no wait for this block's global stores
  uint32_t g2[MAXC / 2];
#pragma unroll
  for (int i = 0; i < MAXC / 2; ++i) g2[i] = gz2[i];
#pragma unroll
  for (int j = 0; j < kHeadMaxK8; ++j) {
    const int k = (t + 256 * j) * 8;
    if (k >= K) continue;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MAXC / 2; ++i) {
      if (2 * i >= C) break;  // zero pairs past the classes (W rows not loaded)
      const uint32_t x0[4] = {wv[j][2 * i].x, wv[j][2 * i].y, wv[j][2 * i].z, wv[j][2 * i].w};
      const uint32_t x1[4] = {wv[j][2 * i + 1].x, wv[j][2 * i + 1].y, wv[j][2 * i + 1].z,
                              wv[j][2 * i + 1].w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        // (W[2i][k'], W[2i+1][k']) for the even and the odd k' of this dword
        a[2 * d] = hdot2(__builtin_amdgcn_perm(x1[d], x0[d], 0x05040100u), g2[i], a[2 * d]);
        a[2 * d + 1] = hdot2(__builtin_amdgcn_perm(x1[d], x0[d], 0x07060302u), g2[i], a[2 * d + 1]);
      }
    }
    const uint32_t hw[4] = {hv[j].x, hv[j].y, hv[j].z, hv[j].w};
    uint16_t q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int16_t hb = (int16_t)(e & 1 ? hw[e >> 1] >> 16 : hw[e >> 1] & 0xffffu);
      q[e] = hb > 0 ? f32_to_bf16(a[e]) : (uint16_t)0;  // bf16 bits > 0 <=> value > 0
    }
    const uint4 qv = make_uint4(q[0] | ((uint32_t)q[1] << 16), q[2] | ((uint32_t)q[3] << 16),
                                q[4] | ((uint32_t)q[5] << 16), q[6] | ((uint32_t)q[7] << 16));
    *reinterpret_cast<uint4*>(dzp + (int64_t)m * ldzp + k) = qv;
    if (dzpT) {
#pragma unroll
      for (int e = 0; e < 8; ++e) dzpT[(int64_t)(k + e) * ldpt + m] = q[e];
    }
  }
  HR_STAMP(4);
}

}  // namespace dsml
