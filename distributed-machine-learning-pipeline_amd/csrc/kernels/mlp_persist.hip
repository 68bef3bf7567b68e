// Persistent fused training kernel for the reference's MLP family on MNIST
// input: 784-128-64-10 (BASELINE / README model) and 784-128-10 (the model the
// reference client actually codes, client.go:22-33), fp32, batch <= 64 rows
// per replica and step.  ONE launch runs S consecutive SGD steps with every
// weight resident on chip, replacing the three launches per step of
// mlp_f32.hip (K_A split-K layer 1, K_B row chain, K_C weight gradients).
//
// Reference hot loop replaced: client.go:596-647 (forwardPass :112-141,
// backwardPass :143-202, updateWeights :254-267), 937 x 10 times on the CPU.
//
// Why: at B = 64 a step is ~29 MFLOP, well under a microsecond of MFMA work
// spread over tens of CUs; a three-launch step costs ~18-21 us, almost all of
// it kernel boundaries, weight reloads and dependent memory round trips.
//
// Two families of roles share this file.
//
// GRAM FORM (single replica, and the data-parallel pkg / pkg2 / pkx): one
// launch of 160 workgroups x 256 threads (one per CU), of which 76 work (132
// with pkx's helpers) and the rest exit at once; placement by blockIdx under
// round-robin dispatch (block b on XCD b % 8):
//
//  * 56 layer-1 blocks (gn < 8, gk < 7) at blockIdx 8 gn + gk + 1 own
//    W1[16 gn ..][112 gk ..] (b1 slice in gk == 0) in LDS.  SGD gives
//    Z1(s+1) = P(s+1) + C(s+1) with P(s+1) = X(s+1) W1(s)^T + b1(s) and the
//    correction C(s+1) = -lr (X(s+1) X(s)^T + 1) dZ1(s) over a per-batch Gram
//    block tabulated at init (engine/gram.py).  Per step each block publishes
//    its k-partial of P(s+1) BEFORE dZ1(s) exists; the four blocks gk = c < 4
//    are the gatherers of chain c: once dZ1(s) arrives they contract the
//    correction for chain c's 16 rows (K split over the 4 waves), add the 7
//    partials and publish Z1(s+1) as {value, step-tag} granules.  Then every
//    block forms its dW1 tile and updates W1 in LDS.
//  * 4 chain blocks (blockIdx 8 c) hold only the critical path: poll Z1, ReLU,
//    layers 2 (and 3), softmax-CE (eps 1e-10, client.go:151), backward to
//    dZ1, published as tagged granules.  Their activation rows go to the
//    gradient tiles.
//  * 16 (3 layers) / 8 (2 layers) gradient tiles (blockIdx 8 (4 + g)): the
//    upper weights' full-batch dW / db and SGD per tile, published back to the
//    chains.  Chains and tiles share XCD 0.
//
//  Data parallel (N replicas): every chain also pushes its dZ1 rows into every
//  peer's receive buffer (DZR), each correction sums over every replica with
//  cross-replica Gram blocks [N][64][64], and the upper tiles' gradients are
//  summed over the replicas inside the launch (one- / two-shot slot exchange).
//  The layer-1 gradient: pkg / pkg2 sum each wave's dW1 slot over xGMI; pkx
//  (exchange-free) forms the global-batch dW1 = sum_r dZ1_r^T X_r itself from
//  the peers' dZ1 rows and the all-gathered, swizzled input shards, with a
//  helper block per layer-1 tile on an idle CU from 4 replicas on.
//
// DIRECT FORM (data-parallel pk / pk2, 64 workgroups): 56 layer-1 blocks
// publish their k-partials of Z1 = X W1^T + b1, 4 chain blocks sum them and
// run the upper layers, 4 gradient blocks own a quarter of the upper weights;
// every wave's weight-gradient fragments are summed over the replicas.
//
// Hand-offs (placement-independent, kernels/common.h for the cross-device
// ones): tagged 8-byte granules {fp32, step tag} written by single
// write-through (sc1) stores and read with sc1 loads until the tags match;
// plain fp32 payloads stored sc1 by every wave, drained (s_waitcnt vmcnt(0)),
// then flagged by one lane behind a workgroup barrier, and read with sc1 loads
// after the flag (MI355X_MICROARCH "Valid forms", row 1).  Tags are the global
// step number + 1, so buffers need zeroing only when the step counter is
// rewound (host side).
//
// Every wait is bounded (timeout -> error word, checked by the host after the
// launch) and gives up at once when another block already timed out, so a
// fault ends the launch instead of hanging the GPU.
#include <cstdlib>

#include "common.h"
#include "../dsml.h"

namespace dsml {

namespace {

constexpr int kD0 = 784, kD1 = 128, kB = 64, kNC = 10;  // input, hidden 1, rows per step, classes
constexpr int kH2 = 64;                                 // hidden 2 (3-layer model)
constexpr int kGN = 8, kGK = 7, kKC = kD0 / kGK;        // 112 k per layer-1 block
constexpr int kNL1 = kGN * kGK;                         // 56 layer-1 blocks
constexpr int kNCH = 4, kNG = 4;                        // chains (16 rows each), gradient blocks
constexpr int kNBlk = kNL1 + kNCH + kNG;                // 64
constexpr int kNPart = kNL1;                            // partial slots per parity
// Single replica: the upper weights' full-batch gradients + SGD run in
// gradient TILES (W2 [16 h x 32 n] tiles of the 3-layer model, [16 o x 16 n]
// tiles of the 2-layer one) -- each loads only its operand columns and
// publishes only its tile, so the weights the chains wait for come back after
// ~16 MFMAs instead of a quarter of the update.  All upper blocks (chains +
// tiles) sit at blockIdx 8 k; layer-1 block (gn, gk) at blockIdx 8 gn + gk + 1.
template <int NL> struct GTile { static constexpr int kN = NL == 3 ? 16 : 8; };
constexpr int cmax0(int a, int b) { return a > b ? a : b; }
// pkx: up to 3 dW1 helper blocks per layer-1 block (helper h = 1..3 of block
// (gn, gk) at blockIdx 8 (8 h + gn) + gk + 1, on its owner's XCD: with 3 the
// layer-1 roles fill XCDs 1-7, 32 CUs each).
constexpr int kMaxHelpers = 3;
// Data-parallel Gram forms with the tagged one-shot tile sums: kPushers(NL)
// pusher blocks push the gradient tiles' slots to the peers (pk_pusher).  With
// 3 helpers the grid has 256 blocks and spare rows on XCD 0: pusher p at
// blockIdx 8 (4 + kN + p), beside its tiles.  Otherwise the grid keeps its
// size: pusher p at row (1 + helpers) kGN + p / 7 of XCD p % 7 + 1, in the
// layer-1 XCDs' spare CUs (the tiles then stage their slots write-through).
template <int NL> constexpr int kPushers() { return GTile<NL>::kN / 2; }
__host__ __device__ constexpr bool pk_push_xcd0(int helpers) { return helpers >= 3; }
template <int NL> constexpr int pk_grid(bool dp, int helpers = 0, bool pushers = false) {
  return dp ? kNBlk
            : 8 * cmax0(kNCH + GTile<NL>::kN + (pushers && pk_push_xcd0(helpers) ? kPushers<NL>() : 0),
                        (1 + helpers) * kGN + (pushers && !pk_push_xcd0(helpers) ? (kPushers<NL>() + 6) / 7 : 0));
}
// Pusher index of blockIdx b, or -1.
template <int NL> __device__ __forceinline__ int pk_pusher_of(int b, int helpers, bool pushers) {
  if (!pushers) return -1;
  const int x = b & 7, y = b >> 3;
  if (pk_push_xcd0(helpers)) {
    const int y0 = kNCH + GTile<NL>::kN;
    return x == 0 && y >= y0 && y < y0 + kPushers<NL>() ? y - y0 : -1;
  }
  const int y0 = (1 + helpers) * kGN;
  const int p = (y - y0) * 7 + (x - 1);
  return x != 0 && y >= y0 && p < kPushers<NL>() ? p : -1;
}
// Whether blockIdx b does work in the Gram-form grid (the rest exit).
template <int NL> __device__ __forceinline__ bool pk_sr_active(int b, int helpers = 0, bool pushers = false) {
  if (pk_pusher_of<NL>(b, helpers, pushers) >= 0) return true;
  return (b & 7) == 0 ? (b >> 3) < kNCH + GTile<NL>::kN : (b >> 3) < (1 + helpers) * kGN;
}
// Replicas [pk_hlo(N, H, k), pk_hlo(N, H, k + 1)) of the global-batch dW1 go to
// part k of a layer-1 tile (k = 0: the owner, k = h: helper h), rank order.
// gsplit (gatherer tiles, gk < 4): the owner, which first contracts the Z1
// correction on the chains' critical path, takes no replica; its helpers split
// all N (part k = helper k: [(k - 1) N / H, k N / H)).
__host__ __device__ constexpr int pk_hlo(int n, int helpers, int k, bool gsplit = false) {
  return (gsplit && helpers > 0) ? (k == 0 ? 0 : (k - 1) * n / helpers) : k * n / (1 + helpers);
}
constexpr int kThreads = 256;
static_assert(kKC % 16 == 0, "k slice must hold whole 16-wide k groups / k tiles");

// ---- LDS layouts (floats) ----------------------------------------------------
// W1 tile row stride: 120 floats puts the forward's 16 rows (+ the q offsets)
// of each ds_read_b128 lane group on 16 distinct 16-B bank slots (116 left 5
// slots 2-way); the once-a-step b32 update pass goes 2-way instead (bank model,
// MI355X_MICROARCH §LDS: 176 vs 256 LDS cycles a block-step)
constexpr int kXS = kKC + 8;
// X tiles are [64][112] unpadded: LDS-DMA (global_load_lds) writes each wave
// instruction's 1 KiB lane-linearly, so the image must be contiguous.
struct L1Lay {
  static constexpr int X0 = 0;                       // X tile, buffer 0 [64][112]
  static constexpr int X1 = X0 + kB * kKC;           // buffer 1
  static constexpr int W = X1 + kB * kKC;            // W1 tile [16][kXS]
  static constexpr int DZ = W + 16 * kXS;            // dZ1 tile [64][17]
  static constexpr int B1 = DZ + kB * 17;            // b1 slice [16]
  static constexpr int TOTAL = B1 + 16;
};
constexpr int kS1 = kD1 + 4, kS2 = kH2 + 4, kS3 = 16 + 4, kSG = 17, kSW = 36;
template <int NL> struct ChLay;
template <> struct ChLay<3> {
  static constexpr int W2 = 0;                       // [64][kS1]
  static constexpr int W3 = W2 + kH2 * kS1;          // [16][kS2] rows >= 10 zero
  static constexpr int B2 = W3 + 16 * kS2;           // [64]
  static constexpr int B3 = B2 + kH2;                // [16]
  static constexpr int H1 = B3 + 16;                 // own rows [16][kS1]
  static constexpr int H2 = H1 + 16 * kS1;           // [16][kS2]
  static constexpr int DZ2 = H2 + 16 * kS2;          // [16][kS2]
  static constexpr int DZ3 = DZ2 + 16 * kS2;         // [16][kS3] cols >= 10 zero
  static constexpr int RED = DZ3 + 16 * kS3;         // [4][16][16] logit partials
  static constexpr int TOTAL = RED + 4 * 256;
};
template <> struct ChLay<2> {
  static constexpr int W2 = 0;                       // [16][kS1] rows >= 10 zero
  static constexpr int B2 = W2 + 16 * kS1;           // [16]
  static constexpr int H1 = B2 + 16;                 // own rows [16][kS1]
  static constexpr int DZ2 = H1 + 16 * kS1;          // [16][kS3] cols >= 10 zero
  static constexpr int RED = DZ2 + 16 * kS3;         // [4][16][16] logit partials
  static constexpr int TOTAL = RED + 4 * 256;
};
// Gradient blocks keep the batch rows as the CONTIGUOUS dimension (operands
// transposed on their way into LDS): every MFMA operand pair then comes from
// one 16-B LDS read per lane feeding 4 MFMAs (k = 16 g + 4 q + j).
constexpr int kST = kB + 4;                          // 68: [feature][64 rows] stride
template <int NL> struct GLay;
template <> struct GLay<3> {
  static constexpr int H1T = 0;                      // [128 n][kST]
  static constexpr int DZ2T = H1T + kD1 * kST;       // [16 h of the slice][kST]
  static constexpr int H2T = DZ2T + 16 * kST;        // [16 h][kST]
  static constexpr int DZ3T = H2T + 16 * kST;        // [16 o][kST] (o >= 10 zero)
  static constexpr int W2 = DZ3T + 16 * kST;         // own W2 rows [16][kS1]
  static constexpr int W3 = W2 + 16 * kS1;           // own W3 columns [16 o][kSG]
  static constexpr int B2 = W3 + 16 * kSG;           // [16]
  static constexpr int B3 = B2 + 16;                 // [16]
  static constexpr int RED = B3 + 16;                // [4][256] dW3 partials
  static constexpr int TOTAL = RED + 4 * 256;
};
template <> struct GLay<2> {
  static constexpr int H1T = 0;                      // [32 n of the slice][kST]
  static constexpr int DZ2T = H1T + 32 * kST;        // [16 o][kST] (o >= 10 zero)
  static constexpr int W2 = DZ2T + 16 * kST;         // own W2 columns [16 o][kSW]
  static constexpr int B2 = W2 + 16 * kSW;           // [16]
  static constexpr int TOTAL = B2 + 16;
};
constexpr int cmax_(int a, int b) { return a > b ? a : b; }
// Layer-1 block of the single-replica (Gram-corrected) step: three X tiles
// (X(s) for the backward, X(s+1) for the next forward, X(s+2) in flight), and
// in the gk == 0 blocks the Gram block G1^T(s+1) = (X(s) X(s+1)^T + 1) [64][64].
struct L1GLay {
  static constexpr int X0 = 0;
  static constexpr int W = X0 + 3 * kB * kKC;         // W1 tile [16][kXS]
  static constexpr int DZ = W + 16 * kXS;             // dZ1 tile [64][17]
  static constexpr int B1 = DZ + kB * 17;             // b1 slice [16]
  static constexpr int G = B1 + 16;                   // data-parallel forms: the other replicas'
                                                      // dZ1 tiles [kMaxPeers - 1][64][17]
  static constexpr int RED = G + (kMaxPeers - 1) * kB * 17;  // correction partials [4 waves][64 lanes][4]
  static constexpr int FLG = RED + 4 * 256;                  // lds_and's per-wave words [4]
  static constexpr int TOTAL = FLG + 4;
};
// Workgroup AND of `ok` that orders LDS only: unlike __syncthreads_and it does
// not wait for the waves' outstanding global stores (the dZ1 rows a layer-1
// block just pushed to a peer, acknowledged only after a round trip).  One
// barrier; the words are rewritten only at the next call, behind the other
// barriers of a step.
__device__ __forceinline__ bool lds_and(bool ok, int* words) {
  const bool bad = __builtin_amdgcn_ballot_w64(!ok) != 0;
  if ((threadIdx.x & 63) == 0) words[threadIdx.x >> 6] = bad ? 1 : 0;
  lds_barrier();
  return (words[0] | words[1] | words[2] | words[3]) == 0;
}
static_assert(L1GLay::G % 4 == 0, "LDS-DMA image must be 16-B aligned");
constexpr int cmax(int a, int b) { return a > b ? a : b; }
template <int NL>
constexpr int lds_floats() {
  return cmax(cmax(L1Lay::TOTAL, L1GLay::TOTAL), cmax(ChLay<NL>::TOTAL, GLay<NL>::TOTAL));  // >= GTLay
}
static_assert(lds_floats<3>() * 4 <= 160 * 1024 && lds_floats<2>() * 4 <= 160 * 1024, "LDS budget");

// ---- hand-off buffer layout (8-byte granules) --------------------------------
// PART[2][56][4][16][16] partials [parity][slot][chain][n][row], plain fp32:
//                   the layer-1 blocks' k-partials of Z1 (b1 added by gk == 0);
//                   one flag per slot and step (PF[64]); the direct form (pk /
//                   pk2, read by the chains).  The Gram forms' partials are PG.
// SF[64]            started flags (tag = first step + 1): the step counter is
//                   handed on only once every block has read it
// DZ1[64][128]      activation gradient of layer 1, tagged granules
// CX[2][4][kCX]     chain rows for the gradient blocks, plain fp32, parity by
//                   step; 3 layers: H1 [16][128], H2 [16][64], dZ2 [16][64],
//                   dZ3 [16][16]; 2 layers: H1 [16][128], dZ2 [16][16]; CXF flags
//                   (H1 rows flagged as soon as they exist, the rest at the end)
// WX[2][4][kWX]     updated weight slices of the gradient blocks, parity by
//                   step; 3 layers: W2 rows [16][128], W3 columns [16 o][16],
//                   b2 slice [16], b3 [16]; 2 layers: W2 columns [16 o][32],
//                   b2 [16]; WF flags
constexpr int kCX = 16 * kD1 + 16 * kH2 + 16 * kH2 + 16 * 16;  // 4352 floats
constexpr int kWX = 16 * kD1 + 16 * 16 + 16 + 16;              // 2336 floats
constexpr int64_t kOffPart = 0;
constexpr int64_t kOffPf = kOffPart + 2 * kNPart * 16 * kB / 2;
constexpr int64_t kOffSf = kOffPf + 2 * 64;
constexpr int64_t kOffDz1 = kOffSf + 256;  // SF[256]: indexed by blockIdx
// DZ1[2][64][128]: parity by step in the single-replica step (there the
// chains' next step does not wait for the gk >= 1 layer-1 blocks to have read
// this step's dZ1, so it must not overwrite it); the data-parallel step (where
// it does wait, through every block's partials) uses parity 0
constexpr int64_t kOffCx = kOffDz1 + 2 * kB * kD1;
constexpr int64_t kOffCxf = kOffCx + 2 * kNCH * kCX / 2;
constexpr int64_t kOffWx = kOffCxf + 16;  // CXF: [part 0 = H1, part 1 = the rest][2][4]
constexpr int64_t kOffWf = kOffWx + 2 * kNG * kWX / 2;
// CG[64][128]: single replica, the layer-1 correction C(s) of step s as tagged
// granules (tag s + 1), written by the gk == 0 layer-1 blocks, polled directly
// by the chains (no drain, no flag: one hop).
constexpr int64_t kOffCg = kOffWf + 8;
// WXS[2][kWXS]: single replica, the gradient tiles' updated upper weights,
// parity by step, in the chains' order: 3 layers W2 [64][128], W3 [16 o][64]
// (o >= 10 zero), b2 [64], b3 [16]; 2 layers W2 [16 o][128], b2 [16].  WFS[2][16]
// flags, one per tile.
constexpr int kWXS = kH2 * kD1 + 16 * kH2 + kH2 + 16;   // 9296 floats
constexpr int64_t kOffWxs = kOffCg + kB * kD1;
constexpr int64_t kOffWfs = kOffWxs + 2 * kWXS / 2;
// HX[2][3][56][4 waves][64 lanes][8]: pkx with helpers, helper h's share of
// every layer-1 tile's dW1 (and db1) at [parity][h - 1], plain fp32;
// HF[2][3][64] flags, one per tile and helper.
constexpr int64_t kOffHx = kOffWfs + 32;
constexpr int64_t kOffHf = kOffHx + 2 * kMaxHelpers * kNL1 * 4 * 64 * 8 / 2;
constexpr int64_t kTotalG = kOffHf + 2 * kMaxHelpers * 64;
__device__ __forceinline__ int64_t pk_hx_off(uint64_t s, int h, int lb, int w, int lane) {  // floats
  return kOffHx * 2 + (((((int64_t)(s & 1) * kMaxHelpers + (h - 1)) * kNL1 + lb) * 4 + w) * 64 + lane) * 8;
}
__device__ __forceinline__ int64_t pk_hf(uint64_t s, int h, int lb) {
  return kOffHf + ((int64_t)(s & 1) * kMaxHelpers + (h - 1)) * 64 + lb;
}
// XS[2][16][3][64 lanes][4 granules]: data-parallel Gram forms (tagged sums),
// every gradient tile's slot values staged for its pusher block as {value,
// step tag} granules (no drain, no flag: the pusher polls the data itself).
constexpr int64_t kOffXs = kTotalG;
constexpr int64_t kTotalX = kOffXs + 2 * 16 * 3 * 64 * 4;
// PG[2][56][4][16][16] Gram forms: the layer-1 blocks' k-partials of Z1 as
// tagged granules [parity][slot][chain][n][row] (tag = step + 1), polled by the
// gatherer directly -- no store drain and flag by the producer, no flag round
// before the data by the gatherer (PART / PF above stay the direct form's)
constexpr int64_t kOffPg = kTotalX;
constexpr int64_t kTotalP = kOffPg + 2 * kNPart * kNCH * 256;
__device__ __forceinline__ int64_t pk_xs_g(uint64_t s, int g, int k, int lane) {  // granules
  return kOffXs + ((((int64_t)(s & 1) * 16 + g) * 3 + k) * 64 + lane) * 4;
}

static_assert(kCX % 4 == 0 && kWX % 4 == 0 && (kOffCx % 2) == 0 && (kOffWx % 2) == 0,
              "exchange rows travel as 16-B vectors");

constexpr int kSc1 = 16;  // buffer aux: sc1 (write-through store / L1-bypassing load)
typedef uint32_t nu4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}
// One granule {value, tag}, one 8-byte write-through store.
__device__ __forceinline__ void st_gran(__amdgpu_buffer_rsrc_t r, int64_t g, float v, uint32_t tag) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  u2 w = {__float_as_uint(v), tag};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)(g * 8), 0, kSc1);
}
// Two adjacent granules (16 B, 16-B aligned), one load.
__device__ __forceinline__ uint4 ld_gran2(__amdgpu_buffer_rsrc_t r, int64_t g) {
  const nu4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(g * 8), 0, kSc1);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_f4(__amdgpu_buffer_rsrc_t r, int64_t float_off, f4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4v, v), r, (int)(float_off * 4), 0, kSc1);
}
// Store of an upper-group hand-off (chains <-> gradient blocks): write-through
// (sc1) in general, PLAIN when the whole group was seen on one XCD (`local`):
// the line then stays in that XCD's L2, where the consumer's sc1 loads (L1
// bypass) find it -- coherent inside one XCD, ~1.6x the hand-off bandwidth
// (MI355X_MICROARCH "handoff-payload").  The flag stays an sc1 granule.
__device__ __forceinline__ void st_up4(__amdgpu_buffer_rsrc_t r, int64_t float_off, f4v v, bool local) {
  if (local)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4v, v), r, (int)(float_off * 4), 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4v, v), r, (int)(float_off * 4), 0, kSc1);
}
// Stage one slot value as two 16-B granule pairs (plain stores when the
// consumer shares the XCD: st_up4's rule).
__device__ __forceinline__ void pk_xs_put(__amdgpu_buffer_rsrc_t rb, int64_t g, float4 v, uint32_t tag, bool local) {
  const nu4v lo = {__float_as_uint(v.x), tag, __float_as_uint(v.y), tag};
  const nu4v hi = {__float_as_uint(v.z), tag, __float_as_uint(v.w), tag};
  if (local) {
    __builtin_amdgcn_raw_buffer_store_b128(lo, rb, (int)(g * 8), 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(hi, rb, (int)(g * 8 + 16), 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(lo, rb, (int)(g * 8), 0, kSc1);
    __builtin_amdgcn_raw_buffer_store_b128(hi, rb, (int)(g * 8 + 16), 0, kSc1);
  }
}
__device__ __forceinline__ f4v ld_f4(__amdgpu_buffer_rsrc_t r, int64_t float_off) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(float_off * 4), 0, kSc1));
}
__device__ __forceinline__ uint32_t flag_tag(__amdgpu_buffer_rsrc_t r, int64_t g) {
  const uint4 f = ld_gran2(r, g & ~(int64_t)1);
  return (g & 1) ? f.w : f.y;
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
// Spin (one lane) until flag granule g carries `tag`; false on give-up.
__device__ __forceinline__ bool wait_flag(__amdgpu_buffer_rsrc_t r, int64_t g, uint32_t tag, Poll& p) {
  p.start();
  while (flag_tag(r, g) != tag)
    if (!p.again()) return false;
  return true;
}

// The wave's index in its workgroup, provably wave-uniform (threadIdx.x >> 6 is
// uniform per wave, but the compiler's divergence analysis cannot see it):
// slot numbers and descriptors derived from it then stay in SGPRs.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
// The launch's first step, made wave-uniform: every lane loads the same word,
// and a value the compiler can prove uniform keeps every step-derived offset
// (parity halves, DZR slots, tags) in SGPRs -- otherwise each buffer access
// through a descriptor built from it runs in a readfirstlane waterfall loop
// (r5: the pkx exchange loads and pushes, 0.2-0.3 us apiece).
__device__ __forceinline__ uint64_t ld_ctr64(const int64_t* p) {
  const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// ---- replica exchange (nrep > 1): 16-B vector accesses at system scope
// (sc0 sc1) through a buffer descriptor on the wave-uniform slot base, so a
// wave's slot moves as coalesced 1 KiB instructions. ----
typedef __attribute__((address_space(1))) uint64_t px_g64;
constexpr int kScSys = 17;  // buffer aux: sc0 | sc1 (system scope)
__device__ __forceinline__ void px_st4(const __amdgpu_buffer_rsrc_t& r, int off_bytes, float4 v) {
  const f4v x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4v, x), r, off_bytes, 0, kScSys);
}
__device__ __forceinline__ float4 px_ld4(const __amdgpu_buffer_rsrc_t& r, int off_bytes) {
  const nu4v v = __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, kScSys);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}

}  // namespace

// Phase stamps (s_memrealtime, 100 MHz) of layer-1 block 0, chain 0 and
// gradient block 0 for steps 8..15 of a launch, profiling only
// (tools/pk_stamps.py): [role][step - 8][phase], role 0 = layer-1, 1 = chain,
// 2 = gradient block; role 3, row 0: launch edges ([0] layer-1 block 0 entry,
// [1] its prologue done, [2] its exit, [3] chain 0 entry, [4] prologue done,
// [5] exit).
__device__ uint64_t g_pk_stamps[4][8][8];
__device__ int g_pk_stamp_on;
// Testing only: uneven-load injection.  With g_pk_jitter = J > 0 every block
// of the single-replica step sleeps a pseudo-random 0..J x 64 cycles before
// its hand-off waits and publications, so producers and consumers drift
// apart by microseconds -- the results must stay bit-identical
// (tests/test_gpu_persist.py).  0 in production: one scalar load per block.
__device__ int g_pk_jitter;
// Testing only (tools/pk_probe.py, the lone-replica probe): peers' dZ1 rows are
// taken as arrived whatever their tags, so ONE replica can run the N-rank Gram
// forms with no peer (its flags preset).  0 in production.
__device__ int g_pk_probe;
// Testing only, host side: 0 off, 1 the probe above, 2 MIRROR -- a lone replica
// sends every "peer" push into its OWN receive buffer, in that peer's source
// slot (dZ1 rows and gradient slots alike, flags included), so it runs the
// N-replica data-parallel step against N - 1 exact copies of itself: the
// result must equal single-replica SGD at the same lr (tests/test_gpu_persist.py
// covers pkx and its helper blocks at N = 4 and 8 on one GPU this way).
static int g_pk_probe_mode = 0;
// pkx helper count override (-1: the default by replica count; set from
// HIPDSML_PKX_HELPERS at the first data-parallel launch)
static int g_pkx_helpers = -2;
// pkx dZ1 row pushes from the layer-1 owner blocks (1) or the chains (0): the
// default, and the HIPDSML_PKX_L1PUSH override (-2: not read yet, -1: none)
// (1: mirror-mode N = 8 step 17.5 -> 15.4 us, N = 4 13.3 -> 12.3 us; the
// lone-replica probe, which never waits for the rows, 10.9 -> 11.4 us at N = 8:
// profiles/r6_pkx_l1push_ab.json)
constexpr int kPkxL1PushDefault = 1;
static int g_pkx_l1push = -2;
// pkx: the gatherer tiles' owners take no dW1 replica (their helpers take all):
// lone-replica probe N = 8 11.57 -> 10.7 us, N = 4 9.96 -> 9.58, mirror mode
// unchanged; every owner taking none was slower (profiles/r6_pkx_gather_split_ab.json)
constexpr int kPkxGsplitDefault = 1;  // (HIPDSML_PKX_GSPLIT overrides)
static int g_pkx_gsplit = -2;
__device__ __forceinline__ void pk_jit(int jit, int blk, uint64_t it, int salt) {
  if (jit <= 0) return;
  uint32_t h = (uint32_t)blk * 2654435761u ^ (uint32_t)(it + 1) * 40503u ^ (uint32_t)salt * 0x9E3779B9u;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  const int n = (int)(h % (uint32_t)(jit + 1));
  for (int k = 0; k < n; ++k) __builtin_amdgcn_s_sleep(1);
}
#define PK_EDGE(ph)                                                                   \
  do {                                                                                \
    if (g_pk_stamp_on && threadIdx.x == 0)                                            \
      g_pk_stamps[3][0][(ph)] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
// g_pk_stamp_on = first stamped step + 1 (mlp_persist_set_stamp_window; the
// default window is steps 8-15)
#define PK_STAMP(role, ph)                                                            \
  do {                                                                                \
    if (stamp_on && threadIdx.x == 0 && it >= stamp_on - 1 && it < stamp_on + 7)          \
      g_pk_stamps[(role)][it - (stamp_on - 1)][(ph)] = __builtin_amdgcn_s_memrealtime();  \
  } while (0)

struct PersistArgs {
  const float* X;
  int64_t ldx;
  const int32_t* labels;
  float* P;
  int64_t w_off[3], b_off[3];
  int64_t* ctr;
  int32_t nbatches;
  int32_t batch;  // valid rows per step (<= 64; rows beyond are padding)
  int32_t steps;
  float lr;
  float inv_batch;
  uint64_t* xb;  // hand-off granules (kTotalG)
  float* stats;
  uint32_t* err;
  uint32_t* herr;  // host-mapped mirror of err (nullable): read without a copy
  uint64_t timeout_ticks;
  // Single replica: G1^T of every batch, [nbatches][64 m'][64 m] =
  // X_{b-1}[m'] . X_b[m] + 1 (padding rows repeat the batch's last row), and
  // whether the hand-off buffer carries the pipeline state of the previous
  // launch (its last step's next partials and correction, step tags s0 + 1).
  const float* gram;
  int32_t carry;
  // Data parallelism over nrep replicas (nrep > 1): every step, each wave's
  // weight-gradient slot is pushed into every peer's receive buffer (xt.buf[d],
  // this replica's slot; parity by step), flagged (xt.flags[d]), and summed
  // over the replicas in rank order from the local buffer -- identical bytes
  // and order on every replica, so the weights stay bit-identical.  lr is
  // already lr / nrep.
  XchgTab xt;
  int32_t nrep, rep;
  int32_t algo;    // 0: one-shot (every slot to every peer), 1: two-shot (reduce-scatter + all-gather)
  int64_t xhalf;   // floats per parity half of a receive buffer (>= px_half)
  uint32_t* xerr;  // the exchange's error word (a peer that did not arrive)
  int32_t pxslots;  // wave slots per source (kPxSlots; kPxSlotsG in the Gram form)
  int64_t dzr_off;  // Gram form: floats from a parity half's start to its dZ1 receive region
                    // (dzr3: from the buffer's start to the 3-slot region)
  // Exchange-free layer 1 (algo 4, sync 'pkx'): every replica's input shard in
  // MFMA fragment order (parallel/xchg.py swizzle_inputs), replica r's
  // [nbatches][49][4 w][64 lanes][4 j] at xsw + r * xsw_stride, so each replica
  // forms the global-batch dW1 = sum_r dZ1_r^T X_r itself from the peers' dZ1
  // rows it already receives for the Gram correction; those rows then rotate
  // over 3 slots (dzr3) -- every layer-1 block reads them, and a peer can be
  // two steps ahead of the slowest one (see pk_dzr_base).
  const float* xsw;
  int64_t xsw_stride;
  int32_t dzr3;
  int32_t helpers;  // pkx: dW1 helper blocks per layer-1 block (0..3); part k sums replicas
                    // [pk_hlo(nrep, helpers, k), pk_hlo(.., k + 1))
  int32_t mirror;   // testing only (g_pk_probe_mode 2): pushes loop back into this replica's buffer
  int32_t probe;    // testing only (g_pk_probe_mode 1): peers' tagged data taken as arrived
  int32_t pushers;  // Gram forms, tagged tile sums: the tiles' slots pushed by pusher blocks
  int32_t l1push;   // pkx: the replica's dZ1 rows go to the peers from the layer-1 owner blocks
                    // (block (gn, gk) sends column tile gn to peer rep + 1 + gk), not the chains
  int32_t gsplit;   // pkx: the gatherer tiles' owners leave every dW1 replica to their helpers
};

// Receive-buffer layout per parity half: [src][slot][64 lanes][16 floats],
// slots 0..223 = layer-1 block lb, wave w at 4 lb + w, slots 224..239 =
// gradient block g, wave w at 224 + 4 g + w.  Flags [src][slot].
constexpr int kPxSlot = 64 * 16, kPxSlots = kNL1 * 4 + kNG * 4;
// Two-shot adds an all-gather region [slot][64 lanes][16 floats] per parity
// half and its flags [owner][slot].
// Data-parallel Gram form (algo 2 / 3 = one- / two-shot slot sums): slots
// 0..223 the layer-1 waves as above, 224..287 gradient tile g, wave w at
// 224 + 4 g + w; after the slot regions of a parity half, every source's dZ1
// rows as tagged granules DZR[src][64][128] (2 floats a granule).
constexpr int kPxSlotsG = kNL1 * 4 + 16 * 4;
constexpr int64_t kDzrFloats = (int64_t)kB * kD1 * 2;
static int64_t px_slots_half(int n, int algo, int slots) {
  return (int64_t)(n + ((algo & 1) ? 1 : 0)) * slots * kPxSlot;
}
// Exchange-free form (algo 4): the gradient tiles' slots (one-shot) in both
// parity halves, then DZR[3][src][64][128] granules after the second half.
int64_t px_half(int n, int algo) {
  if (algo == 4) return px_slots_half(n, 0, kPxSlotsG) + (3 * n * kDzrFloats + 1) / 2;
  if (algo >= 2) return px_slots_half(n, algo, kPxSlotsG) + n * kDzrFloats;
  return px_slots_half(n, algo, kPxSlots);
}
int px_ntiles(int n, int algo) {
  if (algo == 4) return n * kPxSlotsG;
  return ((algo & 1) ? 2 : 1) * n * (algo >= 2 ? kPxSlotsG : kPxSlots);
}
// Floats from the start of a receive buffer to source `src`'s dZ1 rows of step
// s.  Gram form (pkg / pkg2): one region per parity half -- only the gk == 0
// blocks read it, before they publish Z1(s+1), and a peer's dZ1(s+2) needs
// that Z1 (through this replica's dZ1(s+1)).  Exchange-free (pkx): every
// layer-1 block reads it for dW1, possibly after Z1(s+1) is out; a peer's
// dZ1(s+3) needs this replica's P(s+2), which each block publishes only after
// its dW1(s) -- so three slots never overwrite rows still being read.
__device__ __forceinline__ int64_t pk_dzr_base(const PersistArgs& a, uint64_t s, int src) {
  if (a.dzr3) return a.dzr_off + (int64_t)(s % 3u) * a.nrep * kDzrFloats + (int64_t)src * kDzrFloats;
  return (int64_t)(s & 1) * a.xhalf + a.dzr_off + (int64_t)src * kDzrFloats;
}

// Measurement builds only (-DHIPDSML_MEASURE; tools/pk_probe.py --hop-us): an
// extra one-way latency on every cross-replica hop of the MIRROR test mode.
// Each push of peer data (a chain wave's dZ1 rows, a slot's values or flag)
// first stamps its publish time as a tagged granule {time, step tag} per item
// (dZ1: chain c, wave w -> item 4 c + w; slot k -> item 16 + k); a reader
// that has found the peers' data of an item also waits until g_pk_hop ticks
// (100 MHz) have passed since that stamp.  So the data becomes usable exactly
// T after its publication -- hidden when it arrived early, on the critical
// path when it did not: the cost of the xGMI hop a one-GPU run lacks.
#ifdef HIPDSML_MEASURE
__device__ int g_pk_hop;
constexpr int kHopItems = 16 + kPxSlotsG;
__device__ uint64_t g_pk_hop_st[4][kHopItems];
__device__ __forceinline__ void hop_stamp(const PersistArgs& a, uint64_t s, int item) {
  if (!a.mirror || g_pk_hop == 0 || (threadIdx.x & 63) != 0) return;
  const uint64_t v = ((uint64_t)(uint32_t)(s + 1) << 32) | (uint32_t)__builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(&g_pk_hop_st[s & 3][item], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void hop_wait(const PersistArgs& a, uint64_t s, int item) {
  const int hop = g_pk_hop;
  if (!a.mirror || hop == 0) return;
  uint64_t v;
  const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + a.timeout_ticks;
  do {
    v = __hip_atomic_load(&g_pk_hop_st[s & 3][item], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } while ((uint32_t)(v >> 32) != (uint32_t)(s + 1) && __builtin_amdgcn_s_memrealtime() < t_end);
  while ((uint32_t)__builtin_amdgcn_s_memrealtime() - (uint32_t)v < (uint32_t)hop &&
         __builtin_amdgcn_s_memrealtime() < t_end)
    __builtin_amdgcn_s_sleep(1);
}
#else
__device__ __forceinline__ void hop_stamp(const PersistArgs&, uint64_t, int) {}
__device__ __forceinline__ void hop_wait(const PersistArgs&, uint64_t, int) {}
#endif

// One wave's slot: push v into every peer, raise their flags, wait for every
// peer's slot of step s here, then v = the rank-ordered sum over all
// replicas.  false: a peer did not arrive in time.
template <int NV>
__device__ __forceinline__ bool px_allreduce_wave(const PersistArgs& a, uint64_t s, float4 (&v)[NV],
                                                  int slot) {
  const int lane = threadIdx.x & 63;
  const int64_t poff = (int64_t)(s & 1) * a.xhalf;
  const int64_t per_src = (int64_t)a.pxslots * kPxSlot;
  const uint64_t tag = s + 1;
  hop_stamp(a, s, 16 + slot);  // measurement builds only
  // peers unrolled to compile-time indices: a.xt.buf[d] is then a kernarg
  // (scalar) load, not a vector load + vmcnt(0) (which would wait for the
  // previous peer's pushes) + a readfirstlane waterfall per store
#pragma unroll
  for (int d = 0; d < kMaxPeers; ++d) {
    if (d >= a.nrep || d == a.rep) continue;
    const __amdgpu_buffer_rsrc_t r =
        rsrc(a.mirror ? a.xt.buf[a.rep] + poff + (int64_t)slot * kPxSlot + (int64_t)d * per_src
                      : a.xt.buf[d] + poff + (int64_t)slot * kPxSlot + (int64_t)a.rep * per_src);
#pragma unroll
    for (int j = 0; j < NV; ++j) px_st4(r, (lane * 16 + 4 * j) * 4, v[j]);
  }
  // every peer's memory acknowledged the slot before its flag: the
  // system-scope release of this protocol (common.h, "Cross-device release")
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < kMaxPeers; ++d)
      if (d < a.nrep && d != a.rep)
        __hip_atomic_store((px_g64*)(a.mirror ? a.xt.flags[a.rep] + slot + d * a.pxslots
                                              : a.xt.flags[d] + slot + a.rep * a.pxslots),
                           tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  bool ok = true;
  if (lane < a.nrep && lane != a.rep)
    ok = poll_flag_ge<1>(a.xt.flags[a.rep] + slot + lane * a.pxslots, tag, a.xerr, a.timeout_ticks);
  ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
  asm volatile("" ::: "memory");
  if (!ok) return false;
  hop_wait(a, s, 16 + slot);  // measurement builds only
  const float* mine = a.xt.buf[a.rep] + poff + (int64_t)slot * kPxSlot;
  // every source's slot loaded first (all in flight together), then summed in
  // rank order
  float4 x[kMaxPeers][NV];
#pragma unroll
  for (int src = 0; src < kMaxPeers; ++src) {
    if (src < a.nrep && src != a.rep) {
      const __amdgpu_buffer_rsrc_t r = rsrc(mine + src * per_src);
#pragma unroll
      for (int j = 0; j < NV; ++j) x[src][j] = px_ld4(r, (lane * 16 + 4 * j) * 4);
    }
  }
  float4 acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int src = 0; src < kMaxPeers; ++src) {
    if (src < a.nrep) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const float4 y = src == a.rep ? v[j] : x[src][j];
        acc[j].x += y.x; acc[j].y += y.y; acc[j].z += y.z; acc[j].w += y.w;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = acc[j];
  return true;
}

// Two-shot form of the same sum (sync 'pk2'): lane l's values are owned by
// replica l % n.  Reduce-scatter: each lane sends its values to their owner
// only; the owner sums all n in rank order.  All-gather: the owner sends the
// sum to every peer.  Per wave and step 2 (n-1)/n of the slot leaves each
// replica instead of (n-1) slots (n = 8: 4x fewer bytes per link), for one
// more flag round trip.  Every replica ends with the owner's bits.
template <int NV>
__device__ __forceinline__ bool px_allreduce2_wave(const PersistArgs& a, uint64_t s, float4 (&v)[NV],
                                                   int slot) {
  const int lane = threadIdx.x & 63;
  const int n = a.nrep, me = a.rep;
  const int own = lane % n;
  const int64_t poff = (int64_t)(s & 1) * a.xhalf;
  const int64_t per_src = (int64_t)a.pxslots * kPxSlot;
  const int64_t ag = (int64_t)n * per_src;  // all-gather region of a parity half
  const uint64_t tag = s + 1;
  // ---- reduce-scatter: values to their owner (peers unrolled: scalar buf[d]) ----
#pragma unroll
  for (int d = 0; d < kMaxPeers; ++d) {
    if (d >= n || d == me) continue;
    const __amdgpu_buffer_rsrc_t r =
        rsrc(a.xt.buf[d] + poff + (int64_t)slot * kPxSlot + (int64_t)me * per_src);
    if (own == d) {
#pragma unroll
      for (int j = 0; j < NV; ++j) px_st4(r, (lane * 16 + 4 * j) * 4, v[j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // system-scope release (common.h)
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < kMaxPeers; ++d)
      if (d < n && d != me)
        __hip_atomic_store((px_g64*)(a.xt.flags[d] + slot + me * a.pxslots), tag,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  bool ok = true;
  if (lane < n && lane != me)
    ok = poll_flag_ge<1>(a.xt.flags[me] + slot + lane * a.pxslots, tag, a.xerr, a.timeout_ticks);
  ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
  asm volatile("" ::: "memory");
  if (!ok) return false;
  if (own == me) {
    const float* mine = a.xt.buf[me] + poff + (int64_t)slot * kPxSlot;
    float4 acc[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int src = 0; src < n; ++src) {
      const __amdgpu_buffer_rsrc_t r = rsrc(mine + src * per_src);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const float4 x = src == me ? v[j] : px_ld4(r, (lane * 16 + 4 * j) * 4);
        acc[j].x += x.x; acc[j].y += x.y; acc[j].z += x.z; acc[j].w += x.w;
      }
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = acc[j];
  }
  // ---- all-gather: the owner's sums to every peer ----
#pragma unroll
  for (int d = 0; d < kMaxPeers; ++d) {
    if (d >= n || d == me) continue;
    const __amdgpu_buffer_rsrc_t r = rsrc(a.xt.buf[d] + poff + ag + (int64_t)slot * kPxSlot);
    if (own == me) {
#pragma unroll
      for (int j = 0; j < NV; ++j) px_st4(r, (lane * 16 + 4 * j) * 4, v[j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < kMaxPeers; ++d)
      if (d < n && d != me)
        __hip_atomic_store((px_g64*)(a.xt.flags[d] + n * a.pxslots + me * a.pxslots + slot), tag,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  ok = true;
  if (lane < n && lane != me)
    ok = poll_flag_ge<1>(a.xt.flags[me] + n * a.pxslots + lane * a.pxslots + slot, tag, a.xerr,
                         a.timeout_ticks);
  ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
  asm volatile("" ::: "memory");
  if (!ok) return false;
  if (own != me) {
    const __amdgpu_buffer_rsrc_t r = rsrc(a.xt.buf[me] + poff + ag + (int64_t)slot * kPxSlot);
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = px_ld4(r, (lane * 16 + 4 * j) * 4);
  }
  return true;
}

// Tagged one-shot form (the Gram forms' one-shot sums, NV <= 2): every value
// travels as an 8-B {value, step tag} granule (two per 16-B store), so the
// sender neither drains its stores (no write-acknowledge round trip over
// xGMI) nor raises a flag, and the receiver polls the data itself: one
// one-way hop instead of ack + flag + load.  Stale granules of step s - 2 (the
// same parity half) carry another tag.  Values are summed in rank order as in
// px_allreduce_wave (bit-identical replicas).
template <int NV>
__device__ __forceinline__ bool px_allreduce_tagged_wave(const PersistArgs& a, uint64_t s, float4 (&v)[NV],
                                                         int slot) {
  static_assert(NV == 1, "the gradient tiles' slots: one float4 a lane, as 4 granules");
  const int lane = threadIdx.x & 63;
  const int64_t poff = (int64_t)(s & 1) * a.xhalf;
  const int64_t per_src = (int64_t)a.pxslots * kPxSlot;
  const uint32_t tag = (uint32_t)(s + 1);
  hop_stamp(a, s, 16 + slot);  // measurement builds only
#pragma unroll
  for (int d = 0; d < kMaxPeers; ++d) {
    if (d >= a.nrep || d == a.rep) continue;
    const __amdgpu_buffer_rsrc_t r =
        rsrc(a.mirror ? a.xt.buf[a.rep] + poff + (int64_t)slot * kPxSlot + (int64_t)d * per_src
                      : a.xt.buf[d] + poff + (int64_t)slot * kPxSlot + (int64_t)a.rep * per_src);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const nu4v lo = {__float_as_uint(v[j].x), tag, __float_as_uint(v[j].y), tag};
      const nu4v hi = {__float_as_uint(v[j].z), tag, __float_as_uint(v[j].w), tag};
      __builtin_amdgcn_raw_buffer_store_b128(lo, r, (lane * 16 + 8 * j) * 4, 0, kScSys);
      __builtin_amdgcn_raw_buffer_store_b128(hi, r, (lane * 16 + 8 * j + 4) * 4, 0, kScSys);
    }
  }
  // every source's granules of this slot, all loads of a round in flight together
  const float* mine = a.xt.buf[a.rep] + poff + (int64_t)slot * kPxSlot;
  nu4v g[kMaxPeers][2 * NV];  // a source's granules, kept once its tags match
  uint32_t need = 0;
#pragma unroll
  for (int src = 0; src < kMaxPeers; ++src)
    if (src < a.nrep && src != a.rep) need |= 1u << src;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t spins = 0;
  bool ok = true;
  while (need != 0u) {
#pragma unroll
    for (int src = 0; src < kMaxPeers; ++src) {
      if (need & (1u << src)) {
        const __amdgpu_buffer_rsrc_t r = rsrc(mine + src * per_src);
#pragma unroll
        for (int h = 0; h < 2 * NV; ++h) g[src][h] = __builtin_amdgcn_raw_buffer_load_b128(r, (lane * 16 + 4 * h) * 4, 0, kScSys);
      }
    }
#pragma unroll
    for (int src = 0; src < kMaxPeers; ++src) {
      if (need & (1u << src)) {
        bool all = true;
#pragma unroll
        for (int h = 0; h < 2 * NV; ++h) all = all && g[src][h].y == tag && g[src][h].w == tag;
        if (all || a.probe) need &= ~(1u << src);
      }
    }
    if (need == 0u) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
      __hip_atomic_fetch_or(a.xerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ok = false;
      break;
    }
    if ((++spins & 63u) == 0u &&
        __hip_atomic_load(a.xerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
  if (!ok) return false;
  hop_wait(a, s, 16 + slot);  // measurement builds only
  float4 acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int src = 0; src < kMaxPeers; ++src) {
    if (src < a.nrep) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const float4 y = src == a.rep ? v[j]
                                      : make_float4(__uint_as_float(g[src][2 * j].x), __uint_as_float(g[src][2 * j].z),
                                                    __uint_as_float(g[src][2 * j + 1].x),
                                                    __uint_as_float(g[src][2 * j + 1].z));
        acc[j].x += y.x; acc[j].y += y.y; acc[j].z += y.z; acc[j].w += y.w;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = acc[j];
  return true;
}

// The same tagged one-shot sum split over waves (the Gram forms' gradient
// tiles): vmcnt retires loads and stores in issue order, so a wave that polls
// after pushing waits for every push's write acknowledgement -- a round trip
// to the peers' (uncached) memory per poll.  Pusher waves push (px_tagged_push,
// never drained here), other waves poll and sum (px_tagged_gather) with no
// store outstanding.  A CU's vector-memory pipe issues a 1 KiB system-scope
// store only every 30-120 ns (box-dependent), and a gathering wave's loads
// queue behind the stores of its CU: the pushes run on separate pusher blocks
// (pk_pusher), two waves per tile, each half the peers (profiles/r5_uc_bench*.jsonl,
// r5_pkx_stamps_*.jsonl).
// v[k] (this replica's value of slot slot0 + k, k < NS) <- the rank-ordered
// sum of every replica's; every source's loads of a round in flight together.
// false: a source did not arrive in time (error word raised).
template <int NS>
__device__ __forceinline__ bool px_tagged_gather(const PersistArgs& a, uint64_t s, float4 (&v)[NS], int slot0,
                                                 int dbg_row = -1) {
  const int lane = threadIdx.x & 63;
  // profiling (tools/pk_stamps.py grad_gather): entry / loads issued / data in / exit
  const bool dbg = dbg_row >= 0 && dbg_row < 6 && threadIdx.x == 0;
  if (dbg) g_pk_stamps[3][2 + dbg_row][0] = __builtin_amdgcn_s_memrealtime();
  const int64_t poff = (int64_t)(s & 1) * a.xhalf;
  const int64_t per_src = (int64_t)a.pxslots * kPxSlot;
  const uint32_t tag = (uint32_t)(s + 1);
  const float* mine = a.xt.buf[a.rep] + poff + (int64_t)slot0 * kPxSlot;
  nu4v g[kMaxPeers][NS][2];
  uint32_t need = 0;
#pragma unroll
  for (int src = 0; src < kMaxPeers; ++src)
    if (src < a.nrep && src != a.rep) need |= 1u << src;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t spins = 0;
  bool ok = true, first = true;
  while (need != 0u) {
#pragma unroll
    for (int src = 0; src < kMaxPeers; ++src) {
      if (need & (1u << src)) {
        const __amdgpu_buffer_rsrc_t r = rsrc(mine + src * per_src);
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          g[src][k][0] = __builtin_amdgcn_raw_buffer_load_b128(r, (k * kPxSlot + lane * 16) * 4, 0, kScSys);
          g[src][k][1] = __builtin_amdgcn_raw_buffer_load_b128(r, (k * kPxSlot + lane * 16 + 4) * 4, 0, kScSys);
        }
      }
    }
    if (dbg && first) g_pk_stamps[3][2 + dbg_row][1] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int src = 0; src < kMaxPeers; ++src) {
      if (need & (1u << src)) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < NS; ++k)
          all = all && g[src][k][0].y == tag && g[src][k][0].w == tag && g[src][k][1].y == tag &&
                g[src][k][1].w == tag;
        if (all || a.probe) need &= ~(1u << src);
      }
    }
    if (dbg && first) g_pk_stamps[3][2 + dbg_row][2] = __builtin_amdgcn_s_memrealtime();
    first = false;
    if (__builtin_amdgcn_ballot_w64(need != 0u) == 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
      __hip_atomic_fetch_or(a.xerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ok = false;
      break;
    }
    if ((++spins & 63u) == 0u &&
        __hip_atomic_load(a.xerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  ok = __builtin_amdgcn_ballot_w64(!ok) == 0;
  if (!ok) return false;
#pragma unroll
  for (int k = 0; k < NS; ++k) hop_wait(a, s, 16 + slot0 + k);  // measurement builds only
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int src = 0; src < kMaxPeers; ++src) {
      if (src < a.nrep) {
        const float4 y = src == a.rep ? v[k]
                                      : make_float4(__uint_as_float(g[src][k][0].x), __uint_as_float(g[src][k][0].z),
                                                    __uint_as_float(g[src][k][1].x), __uint_as_float(g[src][k][1].z));
        acc.x += y.x; acc.y += y.y; acc.z += y.z; acc.w += y.w;
      }
    }
    v[k] = acc;
  }
  if (dbg) g_pk_stamps[3][2 + dbg_row][3] = __builtin_amdgcn_s_memrealtime();
  return true;
}
// Pusher wave pw of npw: every npw-th peer, all `ns` slots (values in
// registers, v[k] = slot slot0 + k).
__device__ __forceinline__ void px_tagged_push_part(const PersistArgs& a, uint64_t s, const float4 (&v)[3], int ns,
                                                    int slot0, int pw, int npw) {
  const int lane = threadIdx.x & 63;
  const int64_t poff = (int64_t)(s & 1) * a.xhalf;
  const int64_t per_src = (int64_t)a.pxslots * kPxSlot;
  const uint32_t tag = (uint32_t)(s + 1);
  nu4v lo[3], hi[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (k < ns) hop_stamp(a, s, 16 + slot0 + k);  // measurement builds only
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    lo[k] = nu4v{__float_as_uint(v[k].x), tag, __float_as_uint(v[k].y), tag};
    hi[k] = nu4v{__float_as_uint(v[k].z), tag, __float_as_uint(v[k].w), tag};
  }
  int j = 0;
#pragma unroll
  for (int d = 0; d < kMaxPeers; ++d) {
    if (d >= a.nrep || d == a.rep) continue;
    if ((j++ % npw) != pw) continue;
    const __amdgpu_buffer_rsrc_t r =
        rsrc(a.mirror ? a.xt.buf[a.rep] + poff + (int64_t)slot0 * kPxSlot + (int64_t)d * per_src
                      : a.xt.buf[d] + poff + (int64_t)slot0 * kPxSlot + (int64_t)a.rep * per_src);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < ns) {
        __builtin_amdgcn_raw_buffer_store_b128(lo[k], r, (k * kPxSlot + lane * 16) * 4, 0, kScSys);
        __builtin_amdgcn_raw_buffer_store_b128(hi[k], r, (k * kPxSlot + lane * 16 + 4) * 4, 0, kScSys);
      }
    }
  }
}

template <int NV>
__device__ __forceinline__ bool px_sum_wave(const PersistArgs& a, uint64_t s, float4 (&v)[NV], int slot) {
  return a.algo ? px_allreduce2_wave<NV>(a, s, v, slot) : px_allreduce_wave<NV>(a, s, v, slot);
}
// The Gram forms' sums: tagged one-shot, or the flagged two-shot (pkg2).
template <int NV>
__device__ __forceinline__ bool px_sum_wave_g(const PersistArgs& a, uint64_t s, float4 (&v)[NV], int slot) {
  return a.algo ? px_allreduce2_wave<NV>(a, s, v, slot) : px_allreduce_tagged_wave<NV>(a, s, v, slot);
}

// A block that gave up leaves a mark in host memory on its way out, so the
// host learns the launch failed without a device->host copy.
__device__ __forceinline__ void pk_report(const PersistArgs& a, bool ok) {
  if (!ok && threadIdx.x == 0 && a.herr != nullptr)
    __hip_atomic_store(a.herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Every block announces the first step it read from the counter (SF granule;
// the value carries the XCD it runs on: hwreg XCC_ID, 0-7).
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}
__device__ __forceinline__ void pk_started(const PersistArgs& a, int blk, uint64_t s0) {
  if (threadIdx.x == 0) st_gran(rsrc(a.xb), kOffSf + blk, __uint_as_float(xcc_id()), (uint32_t)(s0 + 1));
}
// The upper group (4 chains + 4 gradient blocks, blocks 8 k): whether all of
// it runs on ONE XCD, read from their SF granules (same answer in every
// member).  false on a timeout (the caller's ok flag is cleared).
__device__ __forceinline__ bool pk_upper_local(const PersistArgs& a, uint64_t s0, Poll& poll, bool& ok,
                                               int count = kNCH + kNG) {
  __shared__ uint32_t xs[32];
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  const int tid = threadIdx.x;
  if (tid < count) {
    const int64_t g = kOffSf + 8 * tid;
    poll.start();
    uint4 f;
    for (;;) {
      f = ld_gran2(rb, g & ~(int64_t)1);
      if (((g & 1) ? f.w : f.y) == (uint32_t)(s0 + 1)) break;
      if (!poll.again()) { ok = false; break; }
    }
    xs[tid] = (g & 1) ? f.z : f.x;
  }
  ok = __syncthreads_and(ok ? 1 : 0) != 0;
  bool same = true;
  for (int k = 1; k < count; ++k) same = same && xs[k] == xs[0];
  return ok && same;
}

// -----------------------------------------------------------------------------
// Layer-1 block
// -----------------------------------------------------------------------------
constexpr int kXF4 = kB * (kKC / 4);  // float4 of one X tile (1792 = 28 LDS-DMA chunks of 64)
static_assert(kXF4 % 256 == 0, "X tile must be whole 1 KiB LDS-DMA chunks, 7 per wave");
typedef __attribute__((address_space(1))) void* pk_gptr;
typedef __attribute__((address_space(3))) void* pk_lptr;

// X tile of step s -> LDS buffer by LDS-DMA (16 B per lane, no registers):
// wave w issues chunks w, w+4, ...; completion is waited by the next
// __syncthreads (its vmcnt(0)).  Rows past the batch repeat its last row
// (their activation gradients are zero, so they add nothing).
__device__ __forceinline__ void pk_glds_x(const PersistArgs& a, float* lds, int buf, uint64_t s,
                                          int lane, int w, int k0) {
  const int64_t r0 = (int64_t)(s % (uint64_t)a.nbatches) * a.batch;
  float* xl = lds + (buf ? L1Lay::X1 : L1Lay::X0);
#pragma unroll
  for (int ch = w; ch < kXF4 / 64; ch += 4) {
    const int e = ch * 64 + lane;
    const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);
    const int64_t row = r0 + min(r, a.batch - 1);
    __builtin_amdgcn_global_load_lds((pk_gptr)(a.X + row * a.ldx + k0 + 4 * c4),
                                     (pk_lptr)(xl + ch * 256), 16, 0, 0);
  }
}

template <bool DP>
__device__ __forceinline__ void pk_layer1(const PersistArgs& a, float* lds, int lb, int blk) {
  const int gn = lb % kGN, gk = lb / kGN;
  const int n0 = gn * 16, k0 = gk * kKC;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int i = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  pk_started(a, blk, s0);
  float* Wl = lds + L1Lay::W;
  float* Dz = lds + L1Lay::DZ;
  float* B1 = lds + L1Lay::B1;

  if (lb == 0) PK_EDGE(0);
  // ---- prologue: W1 tile, b1 slice, X of the first step ----
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
  pk_glds_x(a, lds, 0, s0, lane, w, k0);
  __syncthreads();
  if (lb == 0) PK_EDGE(1);

  bool ok = true;
  const int stamp_on = lb == 0 ? g_pk_stamp_on : 0;
  for (int it = 0; it < a.steps && ok; ++it) {
    PK_STAMP(0, 0);
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    const int buf = it & 1;
    const float* Xl = lds + (buf ? L1Lay::X1 : L1Lay::X0);

    // ---- forward partial: wave w -> rows 16w .. +15, the tile's 16 n ----
    // Each lane reads 4 consecutive k of its row (X) and column (W) as one
    // 16-B LDS read and feeds them to 4 MFMAs: within every 16-wide k group,
    // MFMA j contracts k = 16 g + 4 q + j (a permutation of the group's k),
    // over 4 independent accumulator chains summed in a fixed order.
    {
      f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f},
                      {0.f, 0.f, 0.f, 0.f}};
      const float* xa = Xl + (16 * w + i) * kKC + 4 * q;
      const float* wa = Wl + i * kXS + 4 * q;
#pragma unroll
      for (int gq = 0; gq < kKC / 16; ++gq) {
        const float4 xv = *reinterpret_cast<const float4*>(xa + 16 * gq);
        const float4 wv = *reinterpret_cast<const float4*>(wa + 16 * gq);
        acc[0] = mfma_f32_16x16x4(xv.x, wv.x, acc[0]);
        acc[1] = mfma_f32_16x16x4(xv.y, wv.y, acc[1]);
        acc[2] = mfma_f32_16x16x4(xv.z, wv.z, acc[2]);
        acc[3] = mfma_f32_16x16x4(xv.w, wv.w, acc[3]);
      }
      // column i, rows 16w + 4q .. +3: one 16-B write-through store per lane
      const float bn = B1[i];
      f4v z;
#pragma unroll
      for (int r = 0; r < 4; ++r) z[r] = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]) + bn;
      // PART[lb][chain w][n][16 rows]: wave w's tile is exactly chain w's rows,
      // so each chain reads one contiguous 1 KiB run per block
      st_f4(rb, kOffPart * 2 + (((int64_t)lb * kNCH + w) * 16 + i) * 16 + 4 * q, z);
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
    if (lb == 0 && it + 1 == a.steps && tid < kNBlk && ok) {
      // hand the step counter on once every block has read it (SF tags)
      const uint32_t t0 = (uint32_t)(s0 + 1);
      poll.start();
      while (flag_tag(rb, kOffSf + tid) != t0)
        if (!poll.again()) { ok = false; break; }
    }
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    if (lb == 0 && it + 1 == a.steps && tid == 0) {
      const uint64_t e = s0 + (uint64_t)a.steps;
      __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ctr), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ctr + 1), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    PK_STAMP(0, 2);

    // ---- backward: dW1 tile [16 n][112 k] = dZ1^T . X, SGD in LDS ----
    // wave w: k tiles w and w + 4 (waves 0-2 two tiles, wave 3 one); wave 3
    // also sums db1 = colsum dZ1 (gk == 0 applies it)
    float dv[kB / 4];  // A operand (dZ1 column i of rows 4 ms + q), shared by the tiles
#pragma unroll
    for (int ms = 0; ms < kB / 4; ++ms) dv[ms] = Dz[(4 * ms + q) * 17 + i];
    f32x4 g[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float db = 0.f;
    if (w < 3) {
      const float* xb0 = Xl + q * kKC + 16 * w + i;
      const float* xb1 = xb0 + 64;
#pragma unroll
      for (int ms = 0; ms < kB / 4; ++ms) {
        g[0] = mfma_f32_16x16x4(dv[ms], xb0[4 * ms * kKC], g[0]);
        g[1] = mfma_f32_16x16x4(dv[ms], xb1[4 * ms * kKC], g[1]);
      }
    } else {
      const float* xb0 = Xl + q * kKC + 48 + i;
#pragma unroll
      for (int ms = 0; ms < kB / 4; ms += 2) {  // two chains over the row phases
        g[0] = mfma_f32_16x16x4(dv[ms], xb0[4 * ms * kKC], g[0]);
        g[1] = mfma_f32_16x16x4(dv[ms + 1], xb0[4 * (ms + 1) * kKC], g[1]);
      }
      g[0] = g[0] + g[1];
#pragma unroll
      for (int ms = 0; ms < kB / 4; ++ms) db += dv[ms];
      db += __shfl_xor(db, 16, 64);
      db += __shfl_xor(db, 32, 64);
    }
    if (DP) {  // data parallel: sum this wave's fragments over the replicas
      float4 v[2];
      v[0] = make_float4(g[0][0], g[0][1], g[0][2], g[0][3]);
      v[1] = w < 3 ? make_float4(g[1][0], g[1][1], g[1][2], g[1][3]) : make_float4(db, 0.f, 0.f, 0.f);
      const bool xok = px_sum_wave<2>(a, s, v, lb * 4 + w);
      g[0] = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
      if (w < 3) g[1] = f32x4{v[1].x, v[1].y, v[1].z, v[1].w};
      else db = v[1].x;
      ok = __syncthreads_and(xok ? 1 : 0) != 0;
      if (!ok) break;
    }
    // every wave read this step's W1 tile in the forward, before the barrier above
    const int kc0 = 16 * w + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) Wl[(4 * q + r) * kXS + kc0] -= a.lr * g[0][r];
    if (w < 3) {
#pragma unroll
      for (int r = 0; r < 4; ++r) Wl[(4 * q + r) * kXS + kc0 + 64] -= a.lr * g[1][r];
    } else if (gk == 0 && q == 0) {
      B1[i] -= a.lr * db;
    }
    __syncthreads();
    PK_STAMP(0, 3);
  }

  // ---- epilogue: the resident weights back to HBM ----
  float* W1w = a.P + a.w_off[0];
  for (int e = tid; e < kW1F4; e += kThreads) {
    const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);
    *reinterpret_cast<float4*>(W1w + (int64_t)(n0 + r) * kD0 + k0 + 4 * c4) =
        *reinterpret_cast<const float4*>(Wl + r * kXS + 4 * c4);
  }
  if (gk == 0 && tid < 16) a.P[a.b_off[0] + n0 + tid] = B1[tid];
  pk_report(a, ok);
  if (lb == 0) PK_EDGE(2);
}


// ---- single replica: the layer-1 blocks off the critical path (Gram form) ----
// W1(s+1) = W1(s) - lr dZ1(s)^T X(s) and b1(s+1) = b1(s) - lr colsum dZ1(s), so
//   Z1(s+1) = X(s+1) W1(s+1)^T + b1(s+1)
//           = [X(s+1) W1(s)^T + b1(s)] - lr (X(s+1) X(s)^T + 1) dZ1(s)
//           = P(s+1) + C(s+1).
// P(s+1) needs only W1(s): the layer-1 blocks compute and publish it BEFORE
// dZ1(s) exists, while the chains still work on step s.  The correction
// C(s+1) is a [64 x 64] . [64 x 128] product over the Gram block G1 (data
// only: precomputed per batch on the host): once dZ1(s) arrives, the gk == 0
// block of each column tile computes its [64 x 16] part (16 MFMAs a wave) and
// publishes it as an 8th partial.  The chain's critical path becomes chain ->
// dZ1 -> correction -> chain, instead of chain -> dZ1 -> dW1 + update ->
// forward -> 57 KB of partials -> chain (r3: 6.3 us of the 9.2 us step).
// Replicas of a data-parallel job keep the direct form (their W1 update sums
// every replica's dZ1^T X).

__device__ __forceinline__ int64_t pk_pg(int par, int slot, int c) {  // granules
  return kOffPg + (((int64_t)par * kNPart + slot) * kNCH + c) * 256;
}
// One lane's 4 partial values as 4 tagged granules (two 16-B stores, no drain)
__device__ __forceinline__ void st_part_g(__amdgpu_buffer_rsrc_t r, int64_t g, f4v z, uint32_t tag) {
  __builtin_amdgcn_raw_buffer_store_b128(nu4v{__float_as_uint(z[0]), tag, __float_as_uint(z[1]), tag}, r,
                                         (int)(g * 8), 0, kSc1);
  __builtin_amdgcn_raw_buffer_store_b128(nu4v{__float_as_uint(z[2]), tag, __float_as_uint(z[3]), tag}, r,
                                         (int)(g * 8 + 16), 0, kSc1);
}

// Gram-form X tile image: row r's 16-B chunks are XOR-swizzled within each
// 16-float group by ((r >> 1) & 3): the forward's ds_read_b128 of 16 rows at one
// k (row stride 112 floats puts rows r and r + 4 on one 16-B bank slot: 2-way in
// every lane group) is then conflict-free, and the backward's ds_read_b32 down a
// column stays conflict-free (bank model of MI355X_MICROARCH §LDS, both passes).
// The LDS-DMA writes the swizzled image by permuting its SOURCE chunks.
__device__ __forceinline__ int pk_xswz(int r) { return ((r >> 1) & 3) << 2; }  // float XOR
// X tile of step s -> the LDS image at xl (LDS-DMA, swizzled as pk_xswz).
__device__ __forceinline__ void pk_glds_x_to(const PersistArgs& a, float* xl, uint64_t s, int lane,
                                             int w, int k0) {
  const int64_t r0 = (int64_t)(s % (uint64_t)a.nbatches) * a.batch;
#pragma unroll
  for (int ch = w; ch < kXF4 / 64; ch += 4) {
    const int e = ch * 64 + lane;
    const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);  // LDS chunk c4 of row r holds
    const int64_t row = r0 + min(r, a.batch - 1);          // logical chunk c4 ^ ((r >> 1) & 3)
    __builtin_amdgcn_global_load_lds((pk_gptr)(a.X + row * a.ldx + k0 + ((4 * c4) ^ pk_xswz(r))),
                                     (pk_lptr)(xl + ch * 256), 16, 0, 0);
  }
}
// One wave's [16 rows x 16 n] of X . W1_tile^T (+ b1): lane (i, q) holds rows
// 16 w + 4 q .. +3 of column i.
__device__ __forceinline__ f4v pk_l1_fwd(const float* Xl, const float* Wl, const float* B1, int w, int i,
                                         int q) {
  f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f},
                  {0.f, 0.f, 0.f, 0.f}};
  const float* xa = Xl + (16 * w + i) * kKC + ((4 * q) ^ pk_xswz(16 * w + i));
  const float* wa = Wl + i * kXS + 4 * q;
#pragma unroll
  for (int gq = 0; gq < kKC / 16; ++gq) {
    const float4 xv = *reinterpret_cast<const float4*>(xa + 16 * gq);
    const float4 wv = *reinterpret_cast<const float4*>(wa + 16 * gq);
    acc[0] = mfma_f32_16x16x4(xv.x, wv.x, acc[0]);
    acc[1] = mfma_f32_16x16x4(xv.y, wv.y, acc[1]);
    acc[2] = mfma_f32_16x16x4(xv.z, wv.z, acc[2]);
    acc[3] = mfma_f32_16x16x4(xv.w, wv.w, acc[3]);
  }
  const float bn = B1[i];
  f4v z;
#pragma unroll
  for (int r = 0; r < 4; ++r) z[r] = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]) + bn;
  return z;
}
// Wave c of gatherer block (gn, gk = c): its own k-partial z of chain c's rows
// plus the 6 other k-partials of its column tile (slots gn + 8 gk'), summed in
// gk' order -- the partial sum of Z1 the correction completes.  Wave-local (the
// flags are polled by lanes 0-6 and agreed by a ballot); false: a wait gave up.
__device__ __forceinline__ bool pk_l1_gather_rows(__amdgpu_buffer_rsrc_t rb, f4v& z, int par, int gn, int c,
                                                  uint32_t tag, Poll& poll, int lane, int i, int q) {
  // the 6 others' granules polled together (PG: one round of loads per
  // attempt, each lane re-reading only the partials still behind)
  f4v v[kGK];
  uint32_t need = ((1u << kGK) - 1u) & ~(1u << c);
  poll.start();
  while (need != 0u) {
    nu4v u0[kGK], u1[kGK];
#pragma unroll
    for (int g2 = 0; g2 < kGK; ++g2) {
      if (need & (1u << g2)) {
        const int off = (int)((pk_pg(par, gn + kGN * g2, c) + i * 16 + 4 * q) * 8);
        u0[g2] = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, kSc1);
        u1[g2] = __builtin_amdgcn_raw_buffer_load_b128(rb, off + 16, 0, kSc1);
      }
    }
#pragma unroll
    for (int g2 = 0; g2 < kGK; ++g2) {
      if ((need & (1u << g2)) && u0[g2].y == tag && u0[g2].w == tag && u1[g2].y == tag && u1[g2].w == tag) {
        v[g2] = f4v{__uint_as_float(u0[g2].x), __uint_as_float(u0[g2].z), __uint_as_float(u1[g2].x),
                    __uint_as_float(u1[g2].z)};
        need &= ~(1u << g2);
      }
    }
    if (need != 0u && !poll.again()) return false;
  }
  f4v sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g2 = 0; g2 < kGK; ++g2) sum += g2 == c ? z : v[g2];
  z = sum;
  return true;
}

// XM: the data-parallel Gram form.  Each replica r's correction then sums over
// every replica r': C_r(s+1) = -(lr/N) sum_r' (X_r(s+1) X_r'(s)^T + 1) dZ1_r'(s),
// with every peer's dZ1 rows pushed by its chains into this replica's DZR
// region (tagged granules) and the cross-replica Gram blocks from the table
// [nbatches][N][64 m'][64 m]; the W1 update sums each wave's dW1 fragments
// over the replicas (the pk slot exchange) -- off the critical path here.
// XMODE 0: single replica; 1: data parallel, Gram form with the dW1 slot
// exchange (pkg / pkg2); 2: data parallel, exchange-free layer 1 (pkx): every
// layer-1 block reads the peers' dZ1 rows and forms the global-batch dW1 tile
// itself from the swizzled input shards, so no layer-1 gradient crosses xGMI.
constexpr int kKT = kD0 / 16;  // 49 k tiles of the swizzled shards
template <int NL, int XMODE>
__device__ __forceinline__ void pk_layer1_gram(const PersistArgs& a, float* lds, int lb, int blk) {
  constexpr bool XM = XMODE >= 1, XL = XMODE == 2;
  const int gn = lb % kGN, gk = lb / kGN;
  const int n0 = gn * 16, k0 = gk * kKC;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int i = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  pk_started(a, blk, s0);
  float* Wl = lds + L1GLay::W;
  float* Dz = lds + L1GLay::DZ;
  float* B1 = lds + L1GLay::B1;
  float* Gl = lds + L1GLay::G;
  auto xbuf = [&](uint64_t s) { return lds + L1GLay::X0 + (int)(s % 3u) * (kB * kKC); };
  const int jit = g_pk_jitter;
  const int probe = XM ? g_pk_probe : 0;
  // pkx, wave w's k tiles of the slice (waves 0-2: w and w + 4; wave 3: tile 3)
  const int kt0 = kKC / 16 * gk + w, kt1 = kKC / 16 * gk + (w < 3 ? w + 4 : w);
  // B operands of replica r's dW1 pass: the swizzled shard's [4 w'][lane][4 j]
  // fragments of the wave's k tiles (one 16-B load per w' and tile)
  auto xl_load = [&](float4 (&B)[2][4], int r, uint64_t s) __attribute__((always_inline)) {
    const float* xr = a.xsw + (int64_t)r * a.xsw_stride +
                      (int64_t)(s % (uint64_t)a.nbatches) * (kKT * 1024) + lane * 4;
#pragma unroll
    for (int wq = 0; wq < 4; ++wq) {
      B[0][wq] = *reinterpret_cast<const float4*>(xr + kt0 * 1024 + wq * 256);
      B[1][wq] = *reinterpret_cast<const float4*>(xr + kt1 * 1024 + wq * 256);  // wave 3: unused copy
    }
  };

  if (lb == 0) PK_EDGE(0);
  // ---- prologue: W1 tile, b1 slice, X of the first two steps ----
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
  pk_glds_x_to(a, xbuf(s0), s0, lane, w, k0);
  pk_glds_x_to(a, xbuf(s0 + 1), s0 + 1, lane, w, k0);
  __syncthreads();  // W1 / b1 stores and both X tiles (LDS-DMA, vmcnt) landed
  if (lb == 0) PK_EDGE(1);
  // Row-split correction: block (gn, gk < 4) gathers and publishes Z1 for
  // chain c = gk's 16 rows of column tile gn.  Its wave c keeps its own k-partial
  // of those rows and sums the 6 others (pk_l1_gather_rows); all 4 waves split
  // the correction's K (wave w: rows m' = 16 w .. +15 of every replica), and
  // wave c adds their partials.  gk >= 4 blocks only publish partials.
  const bool gat = gk < kNCH;
  const int c = gk;
  float* Red = lds + L1GLay::RED;
  int* Flg = reinterpret_cast<int*>(lds + L1GLay::FLG);
  if (!a.carry) {
    // no state from a previous launch: step s0's Z1 directly, correction 0
    const uint32_t t0 = (uint32_t)(s0 + 1);
    const int par0 = (int)(s0 & 1);
    f4v z = pk_l1_fwd(xbuf(s0), Wl, B1, w, i, q);
    st_part_g(rb, pk_pg(par0, lb, w) + i * 16 + 4 * q, z, t0);
    if (gat && w == c) {
      if (!pk_l1_gather_rows(rb, z, par0, gn, c, t0, poll, lane, i, q)) {
        pk_report(a, false);
        return;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) st_gran(rb, kOffCg + (int64_t)(16 * c + 4 * q + r) * kD1 + n0 + i, z[r], t0);
    }
  }

  bool ok = true;
  const int stamp_on = lb == 0 ? g_pk_stamp_on : 0;
  for (int it = 0; it < a.steps && ok; ++it) {
    PK_STAMP(0, 0);
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);       // step s
    const uint32_t tagn = tag + 1;                 // step s + 1
    const int parn = (int)((s + 1) & 1);
    pk_jit(jit, blk, s, 1);

    // ---- P(s+1) = X(s+1) W1(s)^T + b1(s), before dZ1(s) exists: every block
    // publishes its k-partial; wave c of a gatherer keeps its own and sums the
    // six others of chain c's rows ----
    f4v zs = pk_l1_fwd(xbuf(s + 1), Wl, B1, w, i, q);
    st_part_g(rb, pk_pg(parn, lb, w) + i * 16 + 4 * q, zs, tagn);
    // X(s+2) into the third buffer (its last reader, step s-1's backward,
    // finished before the barrier that ended that step)
    pk_glds_x_to(a, xbuf(s + 2), s + 2, lane, w, k0);
    // the Gram fragments of step s+1 go straight into registers (data only: in
    // flight during the waits): lane (i, q) holds G_r'[m = 16 c + i][m' =
    // 16 w + 4 kk + q] = T[r'][m'][m] for kk = 0..3
    float gv[XM ? kMaxPeers : 1][4];
    if (gat) {
      const int64_t bb = (int64_t)((s + 1) % (uint64_t)a.nbatches) * (XM ? a.nrep : 1);
#pragma unroll
      for (int r2 = 0; r2 < (XM ? kMaxPeers : 1); ++r2) {
        if (r2 < (XM ? a.nrep : 1)) {
          const float* gb = a.gram + (bb + r2) * (kB * kB) + 16 * c + i;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) gv[r2][kk] = gb[(16 * w + 4 * kk + q) * kB];
        }
      }
    }
    // pkx: the dW1 operands of this block's first (up to 3) replicas are data
    // only -- all in flight during the waits, so the dW1 passes find them in
    // registers instead of waiting one load latency per replica
    float4 xP[3][2][4];
    const int own_hi = XL ? pk_hlo(a.nrep, a.helpers, 1, a.gsplit && gat) : 0;
    if constexpr (XL) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (j < own_hi) xl_load(xP[j], j, s);
    }
    if (gat && w == c && !pk_l1_gather_rows(rb, zs, parn, gn, c, tagn, poll, lane, i, q)) ok = false;
    PK_STAMP(0, 1);
    pk_jit(jit, blk, s, 2);

    // ---- wait for dZ1[:, n0 .. n0+15] of step s (4 chain blocks) ----
    // (data parallel, gatherers and pkx owners: polled together with the
    // peers' rows below -- one round of loads instead of the local rows'
    // round trip and then the peers')
    const bool dz_merged = XM && (XL || gat);
    if (!dz_merged) {
      const int m = tid >> 2, qq = tid & 3;
      const int64_t g = kOffDz1 + (int64_t)(s & 1) * (kB * kD1) + (int64_t)m * kD1 + n0 + 4 * qq;
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
    if (lb == 0 && it + 1 == a.steps && tid < pk_grid<NL>(false, a.helpers, a.pushers) &&
        pk_sr_active<NL>(tid, a.helpers, a.pushers) &&
        ok) {
      // hand the step counter on once every block has read it (SF tags)
      const uint32_t t0 = (uint32_t)(s0 + 1);
      poll.start();
      while (flag_tag(rb, kOffSf + tid) != t0)
        if (!poll.again()) { ok = false; break; }
    }
    ok = __syncthreads_and(ok ? 1 : 0) != 0;  // also retires the X LDS-DMA
    if (!ok) break;
    // the Gram fragments are in (the barrier waited for every load): said to
    // the compiler, which otherwise cannot prove it across the poll loop below
    // and waits vmcnt(0) -- the pushed rows' acknowledgement -- inside the
    // correction's MFMA chain
    // (unconditional: a path around it would merge the loads back in)
#pragma unroll
    for (int r2 = 0; r2 < (XM ? kMaxPeers : 1); ++r2)
      asm volatile("" : "+v"(gv[r2][0]), "+v"(gv[r2][1]), "+v"(gv[r2][2]), "+v"(gv[r2][3]));
    if (lb == 0 && it + 1 == a.steps && tid == 0) {
      const uint64_t e = s0 + (uint64_t)a.steps;
      __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ctr), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<uint64_t*>(a.ctr + 1), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    PK_STAMP(0, 2);

    // ---- every other replica's dZ1[:, tile] (pushed by its chains), in rank
    // order: for the correction (gatherers) and, in pkx, every block's dW1 ----
    float* DzX = Gl;
    if (dz_merged) {
      // every replica's granules loaded together (one round of loads in
      // flight, not one poll per replica in turn), this replica's own rows
      // (its local DZ1 region, never a probe preset) among them; replicas not
      // yet complete are re-read
      const int m = tid >> 2, qq = tid & 3;
      const int off = (m * kD1 + n0 + 4 * qq) * 8;
      const int64_t gl = kOffDz1 + (int64_t)(s & 1) * (kB * kD1) + (int64_t)m * kD1 + n0 + 4 * qq;
      // this step's DZR slots and the push target, computed once (inside the
      // rounds the compiler reloaded the pointers from the kernel arguments
      // and waited for them per replica, the poll's memory clobbers aside)
      const float* rstep = a.xt.buf[a.rep] + pk_dzr_base(a, s, 0);
      // pkx l1push: this block sends the replica's own rows of column tile gn
      // to ONE peer as soon as they are here -- the 7 gk blocks of a tile
      // cover up to 7 peers, so a replica's 64 KB a peer leave from 56 CUs
      // instead of queueing behind each other in the 4 chains' CUs
      int push_d = -1;
      if constexpr (XL) {
        if (a.l1push && gk < a.nrep - 1) push_d = __builtin_amdgcn_readfirstlane((a.rep + 1 + gk) % a.nrep);
      }
      __amdgpu_buffer_rsrc_t rp = rb;
      if (XL && push_d >= 0)
        rp = rsrc(a.mirror ? a.xt.buf[a.rep] + pk_dzr_base(a, s, push_d) : a.xt.buf[push_d] + pk_dzr_base(a, s, a.rep));
      uint32_t need = 1u << a.rep;  // replicas whose rows this thread still waits for
      // gatherers: every replica (the correction); other pkx owners: only the
      // replicas of their own dW1 part (the helpers read theirs) -- the exchange
      // memory is uncached, and every redundant poll is HBM traffic
      const int rhi = gat ? a.nrep : own_hi;
#pragma unroll
      for (int r2 = 0; r2 < kMaxPeers; ++r2)
        if (r2 < rhi && r2 != a.rep) need |= 1u << r2;
      bool pok = true, peer_rows = false;
      poll.start();
      while (need != 0u) {
        nu4v v0[kMaxPeers], v1[kMaxPeers], o0, o1;
        const bool own = (need >> a.rep) & 1u;
        if (own) {
          o0 = __builtin_amdgcn_raw_buffer_load_b128(rb, (int)(gl * 8), 0, kSc1);
          o1 = __builtin_amdgcn_raw_buffer_load_b128(rb, (int)((gl + 2) * 8), 0, kSc1);
        }
#pragma unroll
        for (int r2 = 0; r2 < kMaxPeers; ++r2) {
          if ((need & (1u << r2)) && r2 != a.rep) {
            const __amdgpu_buffer_rsrc_t rr = rsrc(rstep + r2 * kDzrFloats);
            v0[r2] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, kScSys);
            v1[r2] = __builtin_amdgcn_raw_buffer_load_b128(rr, off + 16, 0, kScSys);
          }
        }
#pragma unroll
        for (int r2 = 0; r2 < kMaxPeers; ++r2) {
          if ((need & (1u << r2)) && r2 != a.rep &&
              (probe || (v0[r2].y == tag && v0[r2].w == tag && v1[r2].y == tag && v1[r2].w == tag))) {
            float* d = DzX + (r2 < a.rep ? r2 : r2 - 1) * (kB * 17) + m * 17 + 4 * qq;
            d[0] = __uint_as_float(v0[r2].x); d[1] = __uint_as_float(v0[r2].z);
            d[2] = __uint_as_float(v1[r2].x); d[3] = __uint_as_float(v1[r2].z);
            need &= ~(1u << r2);
            peer_rows = true;
          }
        }
        if (own && o0.y == tag && o0.w == tag && o1.y == tag && o1.w == tag) {
          float* d = Dz + m * 17 + 4 * qq;
          d[0] = __uint_as_float(o0.x); d[1] = __uint_as_float(o0.z);
          d[2] = __uint_as_float(o1.x); d[3] = __uint_as_float(o1.z);
          if (XL && push_d >= 0) {
            hop_stamp(a, s, 4 * w + (gn & 3));  // measurement builds only
            __builtin_amdgcn_raw_buffer_store_b128(o0, rp, off, 0, kScSys);
            __builtin_amdgcn_raw_buffer_store_b128(o1, rp, off + 16, 0, kScSys);
          }
          need &= ~(1u << a.rep);
        }
        if (need != 0u && !poll.again()) { pok = false; break; }
      }
      // every load of the poll is in: at most this thread's two push stores
      // are still in flight -- said explicitly, so that the compiler's own
      // waits below (the Gram fragments, loaded before the poll) are not a
      // vmcnt(0) that would wait for the pushes' acknowledgement
      __builtin_amdgcn_s_waitcnt(2 | (7 << 4) | (15 << 8));
      if (pok && peer_rows) hop_wait(a, s, 4 * (m >> 4) + (gn & 3));  // measurement builds only
      // (the pushed rows' acknowledgement is not waited for here: the peers
      // poll the granules' tags, and the chains' Z1 does not depend on it)
      ok = lds_and(pok, Flg);
      if (!ok) break;
      PK_STAMP(0, 6);  // every replica's dZ1 rows of the tile in LDS
    }
    // ---- gatherers: C(s+1)[chain c's 16 rows x 16 n] = -lr sum_r' G_r'
    // dZ1_r'(s)[:, tile]; wave w contracts m' = 16 w .. +15 of every replica,
    // wave c adds the four partials in a fixed order and publishes Z1 ----
    if (gat) {
      f32x4 cw = {0.f, 0.f, 0.f, 0.f};
      // every replica's B operands read up front, then one uninterrupted MFMA
      // chain (same order): read per replica, the chain paid an LDS round trip
      // every two MFMAs (1.1 us at N = 8)
      float dzv[XM ? kMaxPeers : 1][4];
#pragma unroll
      for (int r2 = 0; r2 < (XM ? kMaxPeers : 1); ++r2) {
        if (r2 < (XM ? a.nrep : 1)) {
          const float* Dr = (!XM || r2 == a.rep) ? Dz : DzX + (r2 < a.rep ? r2 : r2 - 1) * (kB * 17);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) dzv[r2][kk] = Dr[(16 * w + 4 * kk + q) * 17 + i];
        }
      }
#pragma unroll
      for (int r2 = 0; r2 < (XM ? kMaxPeers : 1); ++r2) {
        if (r2 < (XM ? a.nrep : 1)) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) cw = mfma_f32_16x16x4(gv[r2][kk], dzv[r2][kk], cw);
        }
      }
      *reinterpret_cast<f4v*>(Red + w * 256 + lane * 4) = f4v{cw[0], cw[1], cw[2], cw[3]};
      PK_STAMP(0, 5);  // wave 0's contraction done
      lds_barrier();   // (LDS only: the pushes above stay in flight)
      PK_STAMP(0, 7);  // every wave's
      if (w == c) {
        const f4v c0 = *reinterpret_cast<const f4v*>(Red + lane * 4);
        const f4v c1 = *reinterpret_cast<const f4v*>(Red + 256 + lane * 4);
        const f4v c2 = *reinterpret_cast<const f4v*>(Red + 512 + lane * 4);
        const f4v c3 = *reinterpret_cast<const f4v*>(Red + 768 + lane * 4);
        // Z1(s+1) = P(s+1) + C(s+1), one tagged granule per value: the chains
        // poll the data itself
#pragma unroll
        for (int r = 0; r < 4; ++r)
          st_gran(rb, kOffCg + (int64_t)(16 * c + 4 * q + r) * kD1 + n0 + i,
                  zs[r] + -a.lr * ((c0[r] + c1[r]) + (c2[r] + c3[r])), tagn);
      }
      PK_STAMP(0, 4);
    }

    // ---- backward: dW1 tile [16 n][112 k] = dZ1^T . X(s), SGD in LDS ----
    f32x4 g[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float db = 0.f;
    if constexpr (XL) {
      // global batch: sum over the replicas in rank order, every operand from
      // the swizzled shards (the SAME instruction sequence on every replica:
      // identical W1 bits); row m = 4 w' + 16 j + q of MFMA (w', j)
      // two named operand sets in ping-pong: replica r + 1's loads fly during
      // replica r's MFMAs (no dynamically indexed register array)
      auto pass = [&](const float4 (&cB)[2][4], int r) __attribute__((always_inline)) {
        const float* Dr = r == a.rep ? Dz : DzX + (r < a.rep ? r : r - 1) * (kB * 17);
#pragma unroll
        for (int wq = 0; wq < 4; ++wq) {
          const float d0 = Dr[(4 * wq + q) * 17 + i], d1 = Dr[(4 * wq + 16 + q) * 17 + i];
          const float d2 = Dr[(4 * wq + 32 + q) * 17 + i], d3 = Dr[(4 * wq + 48 + q) * 17 + i];
          if (w < 3) {
            g[0] = mfma_f32_16x16x4(d0, cB[0][wq].x, g[0]);
            g[1] = mfma_f32_16x16x4(d0, cB[1][wq].x, g[1]);
            g[0] = mfma_f32_16x16x4(d1, cB[0][wq].y, g[0]);
            g[1] = mfma_f32_16x16x4(d1, cB[1][wq].y, g[1]);
            g[0] = mfma_f32_16x16x4(d2, cB[0][wq].z, g[0]);
            g[1] = mfma_f32_16x16x4(d2, cB[1][wq].z, g[1]);
            g[0] = mfma_f32_16x16x4(d3, cB[0][wq].w, g[0]);
            g[1] = mfma_f32_16x16x4(d3, cB[1][wq].w, g[1]);
          } else {  // one tile, two chains over the row phases
            g[0] = mfma_f32_16x16x4(d0, cB[0][wq].x, g[0]);
            g[1] = mfma_f32_16x16x4(d1, cB[0][wq].y, g[1]);
            g[0] = mfma_f32_16x16x4(d2, cB[0][wq].z, g[0]);
            g[1] = mfma_f32_16x16x4(d3, cB[0][wq].w, g[1]);
            db += (d0 + d1) + (d2 + d3);
          }
        }
      };
      // replicas [0, own_hi) here, rank order; a set is reloaded for replica
      // j + 3 once pass j has consumed it (only with fewer helpers than the default)
#pragma unroll
      for (int j = 0; j < kMaxPeers; ++j) {
        if (j < own_hi) {
          pass(xP[j % 3], j);
          if (j + 3 < own_hi) xl_load(xP[j % 3], j + 3, s);
        }
      }
      if (w == 3) {
        g[0] = g[0] + g[1];
        db += __shfl_xor(db, 16, 64);
        db += __shfl_xor(db, 32, 64);
      }
      if (a.helpers) {
        // the helpers' parts (same fragment layout), added in helper order
        bool hok = true;
        if (lane < a.helpers) hok = wait_flag(rb, pk_hf(s, lane + 1, lb), tag, poll);
        hok = __builtin_amdgcn_ballot_w64(!hok) == 0;
        asm volatile("" ::: "memory");
        f4v hv[kMaxHelpers][2];
#pragma unroll
        for (int h = 0; h < kMaxHelpers; ++h) {
          if (h < a.helpers) {
            const int64_t ho = pk_hx_off(s, h + 1, lb, w, lane);
            hv[h][0] = ld_f4(rb, ho);
            hv[h][1] = ld_f4(rb, ho + 4);
          }
        }
        if (hok) {
#pragma unroll
          for (int h = 0; h < kMaxHelpers; ++h) {
            if (h < a.helpers) {
              g[0] = g[0] + f32x4{hv[h][0][0], hv[h][0][1], hv[h][0][2], hv[h][0][3]};
              if (w < 3) g[1] = g[1] + f32x4{hv[h][1][0], hv[h][1][1], hv[h][1][2], hv[h][1][3]};
              else db += hv[h][1][0];
            }
          }
        }
        ok = __syncthreads_and(hok ? 1 : 0) != 0;
        if (!ok) break;
      }
    } else {
    const float* Xl = xbuf(s);
    float dv[kB / 4];
#pragma unroll
    for (int ms = 0; ms < kB / 4; ++ms) dv[ms] = Dz[(4 * ms + q) * 17 + i];
    // row 4 ms + q's swizzle (pk_xswz) alternates with ms's parity: two bases
    const int ie = i ^ pk_xswz(q), io = i ^ pk_xswz(4 + q);
    if (w < 3) {
      const float* xe = Xl + q * kKC + 16 * w + ie;
      const float* xo = Xl + q * kKC + 16 * w + io;
#pragma unroll
      for (int ms = 0; ms < kB / 4; ++ms) {
        const float* xb0 = ms & 1 ? xo : xe;
        g[0] = mfma_f32_16x16x4(dv[ms], xb0[4 * ms * kKC], g[0]);
        g[1] = mfma_f32_16x16x4(dv[ms], xb0[4 * ms * kKC + 64], g[1]);
      }
    } else {
      const float* xe = Xl + q * kKC + 48 + ie;
      const float* xo = Xl + q * kKC + 48 + io;
#pragma unroll
      for (int ms = 0; ms < kB / 4; ms += 2) {
        g[0] = mfma_f32_16x16x4(dv[ms], xe[4 * ms * kKC], g[0]);
        g[1] = mfma_f32_16x16x4(dv[ms + 1], xo[4 * (ms + 1) * kKC], g[1]);
      }
      g[0] = g[0] + g[1];
#pragma unroll
      for (int ms = 0; ms < kB / 4; ++ms) db += dv[ms];
      db += __shfl_xor(db, 16, 64);
      db += __shfl_xor(db, 32, 64);
    }
    }
    if constexpr (XMODE == 1) {  // data parallel: this wave's fragments summed over the replicas
      float4 v[2];
      v[0] = make_float4(g[0][0], g[0][1], g[0][2], g[0][3]);
      v[1] = w < 3 ? make_float4(g[1][0], g[1][1], g[1][2], g[1][3]) : make_float4(db, 0.f, 0.f, 0.f);
      const bool xok = px_sum_wave<2>(a, s, v, lb * 4 + w);
      g[0] = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
      if (w < 3) g[1] = f32x4{v[1].x, v[1].y, v[1].z, v[1].w};
      else db = v[1].x;
      ok = __syncthreads_and(xok ? 1 : 0) != 0;
      if (!ok) break;
    }
    // every wave read this step's W1 tile in the P(s+1) forward, before the
    // barrier that followed it
    const int kc0 = 16 * w + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) Wl[(4 * q + r) * kXS + kc0] -= a.lr * g[0][r];
    if (w < 3) {
#pragma unroll
      for (int r = 0; r < 4; ++r) Wl[(4 * q + r) * kXS + kc0 + 64] -= a.lr * g[1][r];
    } else if (gk == 0 && q == 0) {
      B1[i] -= a.lr * db;
    }
    __syncthreads();
    PK_STAMP(0, 3);
  }

  // ---- epilogue: the resident weights back to HBM ----
  float* W1w = a.P + a.w_off[0];
  for (int e = tid; e < kW1F4; e += kThreads) {
    const int r = e / (kKC / 4), c4 = e - r * (kKC / 4);
    *reinterpret_cast<float4*>(W1w + (int64_t)(n0 + r) * kD0 + k0 + 4 * c4) =
        *reinterpret_cast<const float4*>(Wl + r * kXS + 4 * c4);
  }
  if (gk == 0 && tid < 16) a.P[a.b_off[0] + n0 + tid] = B1[tid];
  pk_report(a, ok);
  if (lb == 0) PK_EDGE(2);
}

// pkx helper block h (1..a.helpers) of layer-1 block lb: replicas
// [pk_hlo(N, H, h), pk_hlo(N, H, h + 1)) of the tile's dW1 (and db1), computed
// exactly as the owner computes its part, operands prefetched at step start,
// and handed over through HX[parity][h - 1] + one flag; the owner adds the
// helpers' parts in helper order.  Same XCD as the owner, so the shared X
// slices and the hand-off stay in that XCD's L2.
__device__ __forceinline__ void pk_l1_helper(const PersistArgs& a, float* lds, int lb, int h, int blk) {
  const int gn = lb % kGN, gk = lb / kGN;
  const int n0 = gn * 16;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int i = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  pk_started(a, blk, s0);
  float* Dh = lds;  // dZ1 tiles of replicas h0 .. h1 - 1: [h1 - h0][64][17]
  const int probe = g_pk_probe;
  const bool gsp = a.gsplit && gk < kNCH;
  const int h0 = pk_hlo(a.nrep, a.helpers, h, gsp), h1 = pk_hlo(a.nrep, a.helpers, h + 1, gsp);
  const int cnt = h1 - h0;
  const int kt0 = kKC / 16 * gk + w, kt1 = kKC / 16 * gk + (w < 3 ? w + 4 : w);
  auto xl_load = [&](float4 (&B)[2][4], int r, uint64_t s) __attribute__((always_inline)) {
    const float* xr = a.xsw + (int64_t)r * a.xsw_stride +
                      (int64_t)(s % (uint64_t)a.nbatches) * (kKT * 1024) + lane * 4;
#pragma unroll
    for (int wq = 0; wq < 4; ++wq) {
      B[0][wq] = *reinterpret_cast<const float4*>(xr + kt0 * 1024 + wq * 256);
      B[1][wq] = *reinterpret_cast<const float4*>(xr + kt1 * 1024 + wq * 256);
    }
  };
  bool ok = true;
  for (int it = 0; it < a.steps && ok; ++it) {
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    float4 xP[3][2][4];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < cnt) xl_load(xP[j], h0 + j, s);  // data only: in flight during the waits
    {
      // this part's dZ1 tiles: own rows from the local DZ1 region, the peers'
      // from their DZR slots, every load of a round in flight together.
      // Lone-replica probe: the peers' rows are taken as arrived, so the own
      // rows are polled in the same rounds (by their tags, whether or not
      // they are in this part) to pace the block on this replica's dZ1, as
      // the peers' tags pace it in a real run, instead of running ahead
      const int m = tid >> 2, qq = tid & 3;
      uint32_t need = probe ? 1u << a.rep : 0u;
#pragma unroll
      for (int r2 = 0; r2 < kMaxPeers; ++r2)
        if (r2 >= h0 && r2 < h1) need |= 1u << r2;
      const bool peer_rows = h1 - h0 > 1 || h0 != a.rep;
      const float* rstep = a.xt.buf[a.rep] + pk_dzr_base(a, s, 0);  // once, not per replica and round
      poll.start();
      while (need != 0u) {
        nu4v v0[kMaxPeers], v1[kMaxPeers];
#pragma unroll
        for (int r2 = 0; r2 < kMaxPeers; ++r2) {
          if (need & (1u << r2)) {
            if (r2 == a.rep) {
              const int64_t gg = kOffDz1 + (int64_t)(s & 1) * (kB * kD1) + (int64_t)m * kD1 + n0 + 4 * qq;
              const uint4 u0 = ld_gran2(rb, gg), u1 = ld_gran2(rb, gg + 2);
              v0[r2] = nu4v{u0.x, u0.y, u0.z, u0.w};
              v1[r2] = nu4v{u1.x, u1.y, u1.z, u1.w};
            } else {
              const __amdgpu_buffer_rsrc_t rr = rsrc(rstep + r2 * kDzrFloats);
              const int off = (m * kD1 + n0 + 4 * qq) * 8;
              v0[r2] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, kScSys);
              v1[r2] = __builtin_amdgcn_raw_buffer_load_b128(rr, off + 16, 0, kScSys);
            }
          }
        }
#pragma unroll
        for (int r2 = 0; r2 < kMaxPeers; ++r2) {
          if ((need & (1u << r2)) && ((probe && r2 != a.rep) ||
                                      (v0[r2].y == tag && v0[r2].w == tag && v1[r2].y == tag && v1[r2].w == tag))) {
            if (r2 >= h0 && r2 < h1) {
              float* d = Dh + (r2 - h0) * (kB * 17) + m * 17 + 4 * qq;
              d[0] = __uint_as_float(v0[r2].x); d[1] = __uint_as_float(v0[r2].z);
              d[2] = __uint_as_float(v1[r2].x); d[3] = __uint_as_float(v1[r2].z);
            }
            need &= ~(1u << r2);
          }
        }
        if (need != 0u && !poll.again()) { ok = false; break; }
      }
      if (ok && peer_rows) hop_wait(a, s, 4 * (m >> 4) + (gn & 3));  // measurement builds only
      ok = __syncthreads_and(ok ? 1 : 0) != 0;
      if (!ok) break;
    }
    f32x4 g[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float db = 0.f;
    auto pass = [&](const float4 (&cB)[2][4], int r) __attribute__((always_inline)) {
      const float* Dr = Dh + (r - h0) * (kB * 17);
#pragma unroll
      for (int wq = 0; wq < 4; ++wq) {
        const float d0 = Dr[(4 * wq + q) * 17 + i], d1 = Dr[(4 * wq + 16 + q) * 17 + i];
        const float d2 = Dr[(4 * wq + 32 + q) * 17 + i], d3 = Dr[(4 * wq + 48 + q) * 17 + i];
        if (w < 3) {
          g[0] = mfma_f32_16x16x4(d0, cB[0][wq].x, g[0]);
          g[1] = mfma_f32_16x16x4(d0, cB[1][wq].x, g[1]);
          g[0] = mfma_f32_16x16x4(d1, cB[0][wq].y, g[0]);
          g[1] = mfma_f32_16x16x4(d1, cB[1][wq].y, g[1]);
          g[0] = mfma_f32_16x16x4(d2, cB[0][wq].z, g[0]);
          g[1] = mfma_f32_16x16x4(d2, cB[1][wq].z, g[1]);
          g[0] = mfma_f32_16x16x4(d3, cB[0][wq].w, g[0]);
          g[1] = mfma_f32_16x16x4(d3, cB[1][wq].w, g[1]);
        } else {
          g[0] = mfma_f32_16x16x4(d0, cB[0][wq].x, g[0]);
          g[1] = mfma_f32_16x16x4(d1, cB[0][wq].y, g[1]);
          g[0] = mfma_f32_16x16x4(d2, cB[0][wq].z, g[0]);
          g[1] = mfma_f32_16x16x4(d3, cB[0][wq].w, g[1]);
          db += (d0 + d1) + (d2 + d3);
        }
      }
    };
#pragma unroll
    for (int j = 0; j < kMaxPeers; ++j) {
      if (j < cnt) {
        pass(xP[j % 3], h0 + j);
        if (j + 3 < cnt) xl_load(xP[j % 3], h0 + j + 3, s);
      }
    }
    if (w == 3) {
      g[0] = g[0] + g[1];
      db += __shfl_xor(db, 16, 64);
      db += __shfl_xor(db, 32, 64);
    }
    // hand the part over: the owner's fragment layout, plain fp32 drained by
    // every wave, then one flag
    const int64_t ho = pk_hx_off(s, h, lb, w, lane);
    st_f4(rb, ho, f4v{g[0][0], g[0][1], g[0][2], g[0][3]});
    st_f4(rb, ho + 4, w < 3 ? f4v{g[1][0], g[1][1], g[1][2], g[1][3]} : f4v{db, 0.f, 0.f, 0.f});
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_gran(rb, pk_hf(s, h, lb), __uint_as_float(tag), tag);
  }
  pk_report(a, ok);
}

// -----------------------------------------------------------------------------
// Chain block: the critical path of the upper layers for 16 batch rows
// -----------------------------------------------------------------------------
// Upper weights from HBM (launch prologue) or from the gradient blocks'
// published slices (every later step), in two halves: pk_w_fetch issues the
// loads into registers (in flight while the chain waits for the partials),
// pk_w_commit writes them to LDS.
// 3 layers, per slice g: W2 rows 512 f4, W3 columns 64 f4, b2 slice 4 f4, b3 4 f4
// (g = 0); 2 layers: W2 columns 32 g .. +32 of 16 class rows (128 f4), b2 4 f4.
template <int NL> struct WSlices {
  static constexpr int kPer = NL == 3 ? 584 : 132, kTot = kNG * kPer;
  static constexpr int kIt = (kTot + kThreads - 1) / kThreads;
};
template <int NL>
__device__ __forceinline__ void pk_w_fetch(const PersistArgs& a, f4v (&v)[WSlices<NL>::kIt],
                                           bool from_wx, int par) {
  using WS = WSlices<NL>;
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  const int boff = NL == 3 ? 2 : 1;  // bias of the output layer
#pragma unroll
  for (int j = 0; j < WS::kIt; ++j) {
    const int x = min(tid + j * kThreads, WS::kTot - 1);
    const int g = x / WS::kPer, e = x - g * WS::kPer;
    if (from_wx) {
      v[j] = ld_f4(rb, kOffWx * 2 + ((int64_t)par * kNG + g) * kWX + 4 * e);
      continue;
    }
    const int ebias = WS::kPer - 4;  // the output bias: last 4 f4 of a slice
    if (e >= ebias) {
      const int o = 4 * (e - ebias);
      const float* bp = a.P + a.b_off[boff];
      v[j] = f4v{o < kNC ? bp[o] : 0.f, o + 1 < kNC ? bp[o + 1] : 0.f,
                 o + 2 < kNC ? bp[o + 2] : 0.f, o + 3 < kNC ? bp[o + 3] : 0.f};
    } else if (NL == 3 && e < 512) {  // W2 row 16 g + e / 32
      v[j] = *reinterpret_cast<const f4v*>(a.P + a.w_off[1] + (int64_t)(16 * g + (e >> 5)) * kD1 + 4 * (e & 31));
    } else if (NL == 3 && e < 576) {  // W3[o][16 g + 4 c ..]
      const int o = (e - 512) >> 2, c = (e - 512) & 3;
      v[j] = o < kNC ? *reinterpret_cast<const f4v*>(a.P + a.w_off[2] + (int64_t)o * kH2 + 16 * g + 4 * c)
                     : f4v{0.f, 0.f, 0.f, 0.f};
    } else if (NL == 3) {             // b2 slice
      v[j] = *reinterpret_cast<const f4v*>(a.P + a.b_off[1] + 16 * g + 4 * (e - 576));
    } else {                          // 2 layers: W2[o][32 g + 4 c ..]
      const int o = e >> 3, c = e & 7;
      v[j] = o < kNC ? *reinterpret_cast<const f4v*>(a.P + a.w_off[1] + (int64_t)o * kD1 + 32 * g + 4 * c)
                     : f4v{0.f, 0.f, 0.f, 0.f};
    }
  }
}
template <int NL>
__device__ __forceinline__ void pk_w_commit(float* lds, const f4v (&v)[WSlices<NL>::kIt]) {
  using WS = WSlices<NL>;
  using L = ChLay<NL>;
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < WS::kIt; ++j) {
    const int x = tid + j * kThreads;
    if (x >= WS::kTot) continue;
    const int g = x / WS::kPer, e = x - g * WS::kPer;
    float* dst;
    if constexpr (NL == 3) {
      if (e < 512) dst = lds + L::W2 + (16 * g + (e >> 5)) * kS1 + 4 * (e & 31);
      else if (e < 576) dst = lds + ChLay<3>::W3 + ((e - 512) >> 2) * kS2 + 16 * g + 4 * ((e - 512) & 3);
      else if (e < 580) dst = lds + L::B2 + 16 * g + 4 * (e - 576);
      else if (g == 0) dst = lds + ChLay<3>::B3 + 4 * (e - 580);
      else continue;
    } else {
      if (e < 128) dst = lds + L::W2 + (e >> 3) * kS1 + 32 * g + 4 * (e & 7);
      else if (g == 0) dst = lds + L::B2 + 4 * (e - 128);
      else continue;
    }
    dst[0] = v[j][0]; dst[1] = v[j][1]; dst[2] = v[j][2]; dst[3] = v[j][3];
  }
}


// Single replica: the upper weights in the chains' order (WXS layout) from the
// gradient tiles' parity-`par` publication (from_wx) or, at the launch start,
// from P; pk_w_commit_sr writes them into the chain's LDS.
template <int NL> struct WSr { static constexpr int kTot = NL == 3 ? 2324 : 516,
                                                    kIt = (kTot + kThreads - 1) / kThreads; };
static_assert(WSr<3>::kIt == WSlices<3>::kIt && WSr<2>::kIt == WSlices<2>::kIt, "register budget");
template <int NL>
__device__ __forceinline__ void pk_w_fetch_sr(const PersistArgs& a, f4v (&v)[WSr<NL>::kIt], bool from_wx,
                                              int par) {
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  const int64_t base = kOffWxs * 2 + (int64_t)par * kWXS;
  auto bias = [&](int boff, int o0) {
    const float* bp = a.P + a.b_off[boff];
    return f4v{o0 < kNC ? bp[o0] : 0.f, o0 + 1 < kNC ? bp[o0 + 1] : 0.f, o0 + 2 < kNC ? bp[o0 + 2] : 0.f,
               o0 + 3 < kNC ? bp[o0 + 3] : 0.f};
  };
#pragma unroll
  for (int j = 0; j < WSr<NL>::kIt; ++j) {
    const int e = min(tid + j * kThreads, WSr<NL>::kTot - 1);
    if (from_wx) {
      v[j] = ld_f4(rb, base + 4 * e);  // the WXS order IS the fetch order
      continue;
    }
    if constexpr (NL == 3) {
      if (e < 2048) {
        v[j] = *reinterpret_cast<const f4v*>(a.P + a.w_off[1] + 4 * e);
      } else if (e < 2304) {
        const int o = (e - 2048) >> 4, c4 = (e - 2048) & 15;
        v[j] = o < kNC ? *reinterpret_cast<const f4v*>(a.P + a.w_off[2] + o * kH2 + 4 * c4)
                       : f4v{0.f, 0.f, 0.f, 0.f};
      } else if (e < 2320) {
        v[j] = *reinterpret_cast<const f4v*>(a.P + a.b_off[1] + 4 * (e - 2304));
      } else {
        v[j] = bias(2, 4 * (e - 2320));
      }
    } else {
      if (e < 512) {
        const int o = e >> 5, c4 = e & 31;
        v[j] = o < kNC ? *reinterpret_cast<const f4v*>(a.P + a.w_off[1] + o * kD1 + 4 * c4)
                       : f4v{0.f, 0.f, 0.f, 0.f};
      } else {
        v[j] = bias(1, 4 * (e - 512));
      }
    }
  }
}
template <int NL>
__device__ __forceinline__ void pk_w_commit_sr(float* lds, const f4v (&v)[WSr<NL>::kIt]) {
  using L = ChLay<NL>;
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < WSr<NL>::kIt; ++j) {
    const int e = tid + j * kThreads;
    if (e >= WSr<NL>::kTot) continue;
    float* dst;
    if constexpr (NL == 3) {
      if (e < 2048) dst = lds + L::W2 + (e >> 5) * kS1 + 4 * (e & 31);
      else if (e < 2304) dst = lds + ChLay<3>::W3 + ((e - 2048) >> 4) * kS2 + 4 * ((e - 2048) & 15);
      else if (e < 2320) dst = lds + L::B2 + 4 * (e - 2304);
      else dst = lds + ChLay<3>::B3 + 4 * (e - 2320);
    } else {
      if (e < 512) dst = lds + L::W2 + (e >> 5) * kS1 + 4 * (e & 31);
      else dst = lds + L::B2 + 4 * (e - 512);
    }
    dst[0] = v[j][0]; dst[1] = v[j][1]; dst[2] = v[j][2]; dst[3] = v[j][3];
  }
}

// The chain's rows after H1 -> CX (3 layers: H2 [16][64], dZ2 [16][64], dZ3
// [16][16]; 2 layers: dZ2 [16][16]), stored but not drained.
template <int NL>
__device__ __forceinline__ void pk_chain_rows_out(__amdgpu_buffer_rsrc_t rb, const float* lds, int par,
                                                  int c, bool local) {
  using L = ChLay<NL>;
  const int64_t cx = kOffCx * 2 + ((int64_t)par * kNCH + c) * kCX;
  constexpr int kRow = NL == 3 ? kCX : 16 * kD1 + 16 * 16;
  for (int e = 2048 + (int)threadIdx.x * 4; e < kRow; e += 4 * kThreads) {
    const float* src;
    if constexpr (NL == 3) {
      if (e < 3072) src = lds + L::H2 + ((e - 2048) >> 6) * kS2 + ((e - 2048) & 63);
      else if (e < 4096) src = lds + L::DZ2 + ((e - 3072) >> 6) * kS2 + ((e - 3072) & 63);
      else src = lds + L::DZ3 + ((e - 4096) >> 4) * kS3 + ((e - 4096) & 15);
    } else {
      src = lds + L::DZ2 + ((e - 2048) >> 4) * kS3 + ((e - 2048) & 15);
    }
    st_up4(rb, cx + e, f4v{src[0], src[1], src[2], src[3]}, local);
  }
}

// A chain's dZ1 rows as {value, step tag} granule PAIRS: lane (i, q) computes
// rows 4 q .. +3 of columns 16 (w + 4 tt) + i; lanes i and i ^ 1 swap halves
// (one DPP swap per value), so each lane owns two rows of an adjacent column
// pair and publishes each row as ONE 16-B store -- 4 stores a lane instead of
// 8 single granules, to the local DZ1 region (g0: its granule base) and, in the
// data-parallel Gram forms (XM), to every peer's DZR slot (system scope).
// Readers check both tags of a pair as before.
template <bool XM>
__device__ __forceinline__ void pk_publish_dz1(const PersistArgs& a, __amdgpu_buffer_rsrc_t rb, int64_t g0,
                                               uint64_t s, int rb0, int q, int w, int i, const float (&dzv)[2][4],
                                               uint32_t tag) {
  const bool odd = (i & 1) != 0;
  nu4v pr[2][2];
  int off[2][2];  // granule index in the [64][128] image
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    // each lane sends what its partner keeps (odd -> rows 0, 1; even -> rows
    // 2, 3) by one quad_perm [1, 0, 3, 2] DPP move apiece, no indexing by lane
    const float s0 = odd ? dzv[tt][0] : dzv[tt][2], s1 = odd ? dzv[tt][1] : dzv[tt][3];
    const float x0 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s0), 0xB1, 0xF, 0xF, false));
    const float x1 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s1), 0xB1, 0xF, 0xF, false));
    const int nb = 16 * (w + 4 * tt) + (i & ~1);
    const float lo0 = odd ? x0 : dzv[tt][0], hi0 = odd ? dzv[tt][2] : x0;
    const float lo1 = odd ? x1 : dzv[tt][1], hi1 = odd ? dzv[tt][3] : x1;
    pr[tt][0] = nu4v{__float_as_uint(lo0), tag, __float_as_uint(hi0), tag};
    pr[tt][1] = nu4v{__float_as_uint(lo1), tag, __float_as_uint(hi1), tag};
    off[tt][0] = (rb0 + 4 * q + (odd ? 2 : 0)) * kD1 + nb;
    off[tt][1] = (rb0 + 4 * q + (odd ? 3 : 1)) * kD1 + nb;
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      __builtin_amdgcn_raw_buffer_store_b128(pr[tt][k], rb, (int)((g0 + off[tt][k]) * 8), 0, kSc1);
  if constexpr (XM) {
    if (a.l1push) return;  // the layer-1 owner blocks send the rows on (pk_l1_gram)
    const int64_t base = pk_dzr_base(a, s, a.rep);
    hop_stamp(a, s, 4 * (rb0 >> 4) + w);  // measurement builds: the rows' publish time
#pragma unroll
    for (int d = 0; d < kMaxPeers; ++d) {
      if (d >= a.nrep || d == a.rep) continue;
      const __amdgpu_buffer_rsrc_t r = rsrc(a.mirror ? a.xt.buf[a.rep] + pk_dzr_base(a, s, d) : a.xt.buf[d] + base);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int k = 0; k < 2; ++k) __builtin_amdgcn_raw_buffer_store_b128(pr[tt][k], r, off[tt][k] * 8, 0, kScSys);
    }
  }
}

// Data-parallel Gram forms: the chain's last vector-memory ops of a step are its
// 4 local dZ1 pair stores and 4 pushed to each peer (pk_publish_dz1); only the
// rows stored BEFORE them must land before the rows flag.  vmcnt retires in
// issue order, so waiting down to those 4 n outstanding ops drains the rows
// without waiting for the peers' write acknowledgements (an xGMI round trip)
// on the tiles' path.
__device__ __forceinline__ void pk_drain_rows(int nrep) {
  switch (nrep) {
    case 1: __asm__ volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;  // local dZ1 stores only
    case 2: __asm__ volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: __asm__ volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 4: __asm__ volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 5: __asm__ volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 6: __asm__ volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 7: __asm__ volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 8: __asm__ volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    default: __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int NL, bool DP, bool XM = false>
__device__ __forceinline__ void pk_chain(const PersistArgs& a, float* lds, int c, int blk) {
  using L = ChLay<NL>;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int i = lane & 15, q = lane >> 4;
  const int rb0 = 16 * c;  // first batch row of this chain
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  pk_started(a, blk, s0);
  float* W2 = lds + L::W2;
  float* B2 = lds + L::B2;
  float* H1 = lds + L::H1;
  float* DZ2 = lds + L::DZ2;
  float* RED = lds + L::RED;

  if (c == 0) PK_EDGE(3);
  {
    f4v wv[WSlices<NL>::kIt];
    if constexpr (DP) {
      pk_w_fetch<NL>(a, wv, false, 0);
      pk_w_commit<NL>(lds, wv);
    } else {
      pk_w_fetch_sr<NL>(a, wv, false, 0);
      pk_w_commit_sr<NL>(lds, wv);
    }
  }
  if constexpr (NL == 3) {
    float* DZ3 = lds + L::DZ3;
    for (int e = tid; e < 16 * kS3; e += kThreads) DZ3[e] = 0.f;
  } else {
    for (int e = tid; e < 16 * kS3; e += kThreads) DZ2[e] = 0.f;
  }
  float loss_acc = 0.f, corr_acc = 0.f, cnt_acc = 0.f;
  __shared__ uint32_t s_fail;  // a wave saw a wait give up (set once: the loop then ends)
  if (tid == 0) s_fail = 0u;
  __syncthreads();
  bool ok = true;
  const bool local = pk_upper_local(a, s0, poll, ok, DP ? kNCH + kNG : kNCH + GTile<NL>::kN);
  if (c == 0) PK_EDGE(4);
  if (c == 0 && g_pk_stamp_on && tid == 0) g_pk_stamps[3][1][0] = local ? 1u : 0u;

  const int stamp_on = c == 0 ? g_pk_stamp_on : 0;
  const int jit = DP ? 0 : g_pk_jitter;
  // thread -> (column tile gn, column n, 8 rows) of this chain's H1 block
  const int pgn = tid >> 5, pn = (tid >> 1) & 15, phalf = tid & 1;
  for (int it = 0; ok && it < a.steps; ++it) {
    PK_STAMP(1, 0);
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    const int par = (int)(s & 1);
    const int64_t r0 = (int64_t)(s % (uint64_t)a.nbatches) * a.batch;
    if constexpr (!DP) pk_jit(jit, blk, s, 3);

    // this step's labels first: their memory round trip hides under the waits
    const int srow = w * 4 + (lane >> 4);  // softmax: 16 lanes per row, 4 rows per wave
    const bool rvalid = rb0 + srow < a.batch;
    const int y = rvalid ? a.labels[r0 + rb0 + srow] : -1;
    f4v wv[WSlices<NL>::kIt];
    // The previous step's updated upper weights (gradient blocks): every wave
    // checks their 4 flags itself (lanes 0-3, then a wave vote), so no
    // workgroup barrier -- which would drain the first load batch -- sits
    // between the two load batches.  Order, measured (r3 stamps): 2 layers,
    // whose 5 KB of weights are published ~1.8 us before the partials
    // complete, fetch them FIRST, in flight during the partials wait (step
    // 7.24 -> 6.96 us); 3 layers, whose 37 KB arrive about when the last
    // partial does, fetch them after the partials (weights first: 9.56 ->
    // 10.04 us).
    auto fetch_w = [&]() {
      if (it > 0) {
        bool wok = true;
        if constexpr (DP) {
          if (lane < kNG) wok = wait_flag(rb, kOffWf + (par ^ 1) * kNG + lane, tag - 1, poll);
        } else {
          if (lane < GTile<NL>::kN) wok = wait_flag(rb, kOffWfs + (par ^ 1) * 16 + lane, tag - 1, poll);
        }
        wok = __builtin_amdgcn_ballot_w64(!wok) == 0;
        asm volatile("" ::: "memory");
        if (!wok) ok = false;
        else if constexpr (DP) pk_w_fetch<NL>(a, wv, true, par ^ 1);
        else pk_w_fetch_sr<NL>(a, wv, true, par ^ 1);
      }
    };
    constexpr bool kWFirst = DP && NL == 2;  // single replica: Z1 before the weights (weights first: 7.16 -> 9.0 us)
    if (kWFirst) fetch_w();
    if constexpr (!DP) {
      // ---- H1 rows = relu(Z1(s)): the gk == 0 layer-1 blocks publish Z1 =
      // P + C as tagged granules; polled directly (one hop, no flag) ----
      bool cok = true;
      PK_STAMP(1, 6);
      {
        // thread -> row rr, columns cc .. cc + 7 (four 16-B granule pairs)
        const int rr = tid >> 4, cc = 8 * (tid & 15);
        const int64_t g0 = kOffCg + (int64_t)(rb0 + rr) * kD1 + cc;
        uint4 cv[4];
        // light polling: one lane per row spins on one 16-B pair (the payload
        // lines stay quiet while their writers store them); once all four rows
        // of the wave show it, every lane reads its four pairs and every tag
        // is checked (the writing lanes are unordered)
        poll.start();
        for (;;) {
          bool ready = true;
          if ((tid & 15) == 0) {
            const uint4 f = ld_gran2(rb, g0 + 6);
            ready = f.y == tag && f.w == tag;
          }
          if (__builtin_amdgcn_ballot_w64(!ready) == 0) {
            bool all = true;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              cv[j] = ld_gran2(rb, g0 + 2 * j);
              all = all && cv[j].y == tag && cv[j].w == tag;
            }
            if (__builtin_amdgcn_ballot_w64(!all) == 0) break;
          }
          if (!poll.again()) { cok = false; break; }
        }
        PK_STAMP(1, 1);
        if (cok) {
          float* hr = H1 + rr * kS1 + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            hr[2 * j] = fmaxf(__uint_as_float(cv[j].x), 0.f);
            hr[2 * j + 1] = fmaxf(__uint_as_float(cv[j].z), 0.f);
          }
        }
      }
      if (!cok) ok = false;
      if (!kWFirst) fetch_w();
      // every wave's waits agreed on (drains the weight loads, consumed next)
      ok = __syncthreads_and(ok ? 1 : 0) != 0;
      if (!ok) break;
      if (it > 0) pk_w_commit_sr<NL>(lds, wv);
    } else {
      // ---- H1 rows = relu(sum of the 7 k-partials) ----
      // this chain's 16 rows of every partial in one bulk read: thread -> (gn,
      // column n, 8 rows), 7 gk
      {
        if (tid < kNL1 && !wait_flag(rb, kOffPf + tid, tag, poll)) ok = false;
        if (!ok) s_fail = 1u;
        lds_barrier();
        ok = s_fail == 0u;
        if (!ok) break;
        PK_STAMP(1, 1);
        f4v v[kGK][2];
#pragma unroll
        for (int gk = 0; gk < kGK; ++gk) {
          const int lb = pgn + kGN * gk;
          const int64_t off = kOffPart * 2 + (((int64_t)lb * kNCH + c) * 16 + pn) * 16 + 8 * phalf;
          v[gk][0] = ld_f4(rb, off);
          v[gk][1] = ld_f4(rb, off + 4);
        }
        if (!kWFirst) fetch_w();
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float z = 0.f;
#pragma unroll
          for (int gk = 0; gk < kGK; ++gk) z += v[gk][e >> 2][e & 3];
          H1[(8 * phalf + e) * kS1 + 16 * pgn + pn] = fmaxf(z, 0.f);
        }
      }
      if (it > 0) {
        ok = __syncthreads_and(ok ? 1 : 0) != 0;
        if (!ok) break;
        pk_w_commit<NL>(lds, wv);
      }
    }
    lds_barrier();
    // the H1 rows go to the gradient blocks now; drained and flagged after the
    // forward, whose barriers order LDS only (lds_barrier: a __syncthreads
    // would wait for these stores), so their latency stays off this path
    {
      const int64_t cx = kOffCx * 2 + ((int64_t)par * kNCH + c) * kCX;
      for (int e = tid * 4; e < 16 * kD1; e += 4 * kThreads) {
        const float* src = H1 + (e >> 7) * kS1 + (e & 127);
        st_up4(rb, cx + e, f4v{src[0], src[1], src[2], src[3]}, local);
      }
    }
    PK_STAMP(1, 2);

    if constexpr (NL == 3) {
      float* W3 = lds + L::W3;
      float* B3 = lds + L::B3;
      float* H2 = lds + L::H2;
      float* DZ3 = lds + L::DZ3;
      // ---- layer 2: H2 = relu(H1 W2^T + b2), wave w -> 16 output columns ----
      {
        f32x4 ac[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f},
                       {0.f, 0.f, 0.f, 0.f}};
        const float* ha = H1 + i * kS1 + 4 * q;
        const float* wb = W2 + (16 * w + i) * kS1 + 4 * q;
#pragma unroll
        for (int gq = 0; gq < kD1 / 16; ++gq) {
          const float4 hv = *reinterpret_cast<const float4*>(ha + 16 * gq);
          const float4 wv = *reinterpret_cast<const float4*>(wb + 16 * gq);
          ac[0] = mfma_f32_16x16x4(hv.x, wv.x, ac[0]);
          ac[1] = mfma_f32_16x16x4(hv.y, wv.y, ac[1]);
          ac[2] = mfma_f32_16x16x4(hv.z, wv.z, ac[2]);
          ac[3] = mfma_f32_16x16x4(hv.w, wv.w, ac[3]);
        }
        const int n = 16 * w + i;
        const float bn = B2[n];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          H2[(4 * q + r) * kS2 + n] = fmaxf((ac[0][r] + ac[1][r]) + (ac[2][r] + ac[3][r]) + bn, 0.f);
      }
      lds_barrier();
      // ---- layer 3 partial logits: K = 64 split over the 4 waves ----
      {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const float* ha = H2 + i * kS2 + q;
        const float* wb = W3 + i * kS2 + q;
#pragma unroll
        for (int ks = 4 * w; ks < 4 * w + 4; ++ks) acc = mfma_f32_16x16x4(ha[4 * ks], wb[4 * ks], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) RED[w * 256 + (4 * q + r) * 16 + i] = acc[r];
      }
      lds_barrier();
      // ---- softmax + CE + dLogits ----
      {
        const int col = lane & 15;
        const bool cv = col < kNC;
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
        if (cv && rvalid) {
          g = (p - (col == y ? 1.f : 0.f)) * a.inv_batch;
          if (col == y) loss_acc += -logf(p + 1e-10f);
        }
        DZ3[srow * kS3 + col] = g;
        if (col == 0 && rvalid) {
          corr_acc += amax == y ? 1.f : 0.f;
          cnt_acc += 1.f;
        }
      }
      // the H1 rows stored before the forward have landed long since: every
      // wave drains its stores, then one lane flags them behind the barrier
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      if (tid == 0) st_gran(rb, kOffCxf + par * kNCH + c, __uint_as_float(tag), tag);
      PK_STAMP(1, 3);
      // ---- dZ2 = (dZ3 W3) * (H2 > 0), wave w -> 16 columns ----
      {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const int h = 16 * w + i;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          acc = mfma_f32_16x16x4(DZ3[i * kS3 + 4 * ks + q], W3[(4 * ks + q) * kS2 + h], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 4 * q + r;
          DZ2[m * kS2 + h] = H2[m * kS2 + h] > 0.f ? acc[r] : 0.f;
        }
      }
      lds_barrier();
      // the rest of the rows (H2, dZ2, dZ3) go to the gradient blocks now, ahead
      // of the dZ1 stage; drained and flagged at the end of the step
      pk_chain_rows_out<NL>(rb, lds, par, c, local);
      asm volatile("" ::: "memory");  // the rows' stores stay ahead of the dZ1 stage's (pk_drain_rows)
      // ---- dZ1 = (dZ2 W2) * (H1 > 0), published to the layer-1 blocks ----
      // wave w: n tiles w and w + 4, four accumulator chains interleaved
      {
        f32x4 a0[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        f32x4 a1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < kH2 / 4; ks += 2) {
          const float d0 = DZ2[i * kS2 + 4 * ks + q];
          const float d1 = DZ2[i * kS2 + 4 * ks + 4 + q];
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) {
            const int n = 16 * (w + 4 * tt) + i;
            a0[tt] = mfma_f32_16x16x4(d0, W2[(4 * ks + q) * kS1 + n], a0[tt]);
            a1[tt] = mfma_f32_16x16x4(d1, W2[(4 * ks + 4 + q) * kS1 + n], a1[tt]);
          }
        }
        float dzv[2][4];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int n = 16 * (w + 4 * tt) + i;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = 4 * q + r;
            const float v = H1[m * kS1 + n] > 0.f ? a0[tt][r] + a1[tt][r] : 0.f;
            dzv[tt][r] = v;
          }
        }
        pk_publish_dz1<XM>(a, rb, kOffDz1 + (DP ? 0 : (int64_t)par * (kB * kD1)), s, rb0, q, w, i, dzv, tag);
      }
    } else {
      // ---- logits = H1 W2^T + b2: K = 128 split over the 4 waves ----
      {
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        const float* ha = H1 + i * kS1 + q;
        const float* wb = W2 + i * kS1 + q;
#pragma unroll
        for (int ks = 8 * w; ks < 8 * w + 8; ks += 2) {
          acc0 = mfma_f32_16x16x4(ha[4 * ks], wb[4 * ks], acc0);
          acc1 = mfma_f32_16x16x4(ha[4 * ks + 4], wb[4 * ks + 4], acc1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) RED[w * 256 + (4 * q + r) * 16 + i] = acc0[r] + acc1[r];
      }
      lds_barrier();
      // ---- softmax + CE + dLogits -> DZ2 ----
      {
        const int col = lane & 15;
        const bool cv = col < kNC;
        float z = -3.402823466e38f;
        if (cv) {
          z = B2[col];
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
        if (cv && rvalid) {
          g = (p - (col == y ? 1.f : 0.f)) * a.inv_batch;
          if (col == y) loss_acc += -logf(p + 1e-10f);
        }
        DZ2[srow * kS3 + col] = g;
        if (col == 0 && rvalid) {
          corr_acc += amax == y ? 1.f : 0.f;
          cnt_acc += 1.f;
        }
      }
      // the H1 rows stored before the forward have landed long since: every
      // wave drains its stores, then one lane flags them behind the barrier
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      if (tid == 0) st_gran(rb, kOffCxf + par * kNCH + c, __uint_as_float(tag), tag);
      PK_STAMP(1, 3);
      pk_chain_rows_out<NL>(rb, lds, par, c, local);  // dZ2 (the logits' gradient)
      asm volatile("" ::: "memory");  // the rows' stores stay ahead of the dZ1 stage's (pk_drain_rows)
      // ---- dZ1 = (dZ2 W2) * (H1 > 0), published; wave w: n tiles w, w + 4 ----
      {
        f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const float d = DZ2[i * kS3 + 4 * ks + q];
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
            acc[tt] = mfma_f32_16x16x4(d, W2[(4 * ks + q) * kS1 + 16 * (w + 4 * tt) + i], acc[tt]);
        }
        float dzv[2][4];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int n = 16 * (w + 4 * tt) + i;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = 4 * q + r;
            const float v = H1[m * kS1 + n] > 0.f ? acc[tt][r] : 0.f;
            dzv[tt][r] = v;
          }
        }
        pk_publish_dz1<XM>(a, rb, kOffDz1 + (DP ? 0 : (int64_t)par * (kB * kD1)), s, rb0, q, w, i, dzv, tag);
      }
    }
    PK_STAMP(1, 4);

    // ---- the rest of the rows (stored before the dZ1 stage): drained by every
    // wave, then flagged behind the barrier ----
    if constexpr (XM) pk_drain_rows(a.l1push ? 1 : a.nrep);  // l1push: no peer pushes here
    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (tid == 0) st_gran(rb, kOffCxf + 8 + par * kNCH + c, __uint_as_float(tag), tag);
    PK_STAMP(1, 5);
  }

  // ---- epilogue: stats (the gradient blocks write the upper weights back) ----
  const float l = wave_sum(loss_acc), cr = wave_sum(corr_acc), cn = wave_sum(cnt_acc);
  if (lane == 0 && a.stats != nullptr && cn > 0.f) {
    atomicAdd(a.stats + 0, l);
    atomicAdd(a.stats + 1, cr);
    atomicAdd(a.stats + 2, cn);
  }
  pk_report(a, ok);
  if (c == 0) PK_EDGE(5);
}

// -----------------------------------------------------------------------------
// Gradient block: full-batch weight gradients + SGD of a quarter of the upper
// weights
// -----------------------------------------------------------------------------
template <int NL, bool DP>
__device__ __forceinline__ void pk_grad(const PersistArgs& a, float* lds, int g, int blk) {
  using L = GLay<NL>;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int i = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  pk_started(a, blk, s0);
  float* H1T = lds + L::H1T;
  float* DZ2T = lds + L::DZ2T;
  float* W2 = lds + L::W2;
  float* B2 = lds + L::B2;

  // ---- prologue: this block's slice of the upper weights ----
  if constexpr (NL == 3) {
    float* W3 = lds + L::W3;
    float* B3 = lds + L::B3;
    for (int e = tid; e < 16 * (kD1 / 4); e += kThreads) {
      const int r = e >> 5, c4 = e & 31;
      *reinterpret_cast<float4*>(W2 + r * kS1 + 4 * c4) =
          *reinterpret_cast<const float4*>(a.P + a.w_off[1] + (int64_t)(16 * g + r) * kD1 + 4 * c4);
    }
    {
      const int o = tid >> 4, j = tid & 15;  // 256 threads = [16 o][16 h]
      W3[o * kSG + j] = o < kNC ? a.P[a.w_off[2] + (int64_t)o * kH2 + 16 * g + j] : 0.f;
    }
    if (tid < 16) B2[tid] = a.P[a.b_off[1] + 16 * g + tid];
    if (tid < 16) B3[tid] = tid < kNC ? a.P[a.b_off[2] + tid] : 0.f;
  } else {
    for (int e = tid; e < 16 * 32; e += kThreads) {
      const int o = e >> 5, j = e & 31;
      W2[o * kSW + j] = o < kNC ? a.P[a.w_off[1] + (int64_t)o * kD1 + 32 * g + j] : 0.f;
    }
    if (tid < 16) B2[tid] = tid < kNC ? a.P[a.b_off[1] + tid] : 0.f;
  }
  __syncthreads();
  bool ok = true;
  const bool local = pk_upper_local(a, s0, poll, ok);
  const int stamp_on = g == 0 ? g_pk_stamp_on : 0;
  for (int it = 0; it < a.steps && ok; ++it) {
    PK_STAMP(2, 0);
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    const int par = (int)(s & 1);

    // ---- part 0: the chains' H1 rows (flagged while they run the forward) ----
    if (tid < kNCH && !wait_flag(rb, kOffCxf + par * kNCH + tid, tag, poll)) ok = false;
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    {
      // 3 layers: all 128 columns (8 f4 per thread); 2 layers: the slice's 32
      constexpr int kCols4 = NL == 3 ? 32 : 8, kIt = kNCH * 16 * kCols4 / kThreads;
      f4v v[kIt];
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int x = tid + j * kThreads;
        const int c4 = x % kCols4, r = x / kCols4;  // r = 16 chain + row
        const int c = r >> 4;
        v[j] = ld_f4(rb, kOffCx * 2 + ((int64_t)par * kNCH + c) * kCX + (r & 15) * kD1 +
                             (NL == 3 ? 0 : 32 * g) + 4 * c4);
      }
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int x = tid + j * kThreads;
        const int c4 = x % kCols4, r = x / kCols4;
#pragma unroll
        for (int e = 0; e < 4; ++e) H1T[(4 * c4 + e) * kST + r] = v[j][e];
      }
    }
    // ---- part 1: the rest of the rows (flagged at the end of the chains' step) ----
    if (tid < kNCH && !wait_flag(rb, kOffCxf + 8 + par * kNCH + tid, tag, poll)) ok = false;
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    {
      // 3 layers, per chain: H2 slice, dZ2 slice, dZ3 (16 rows x 4 f4 each);
      // 2 layers: dZ2 (16 rows x 4 f4)
      constexpr int kParts = NL == 3 ? 3 : 1, kIt = kParts * kNCH * 64 / kThreads;
      f4v v[kIt];
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int x = tid + j * kThreads;
        const int part = x >> 8, c = (x >> 6) & 3, r = (x >> 2) & 15, c4 = x & 3;
        int64_t off;
        if (NL == 3 && part == 0) off = 2048 + r * kH2 + 16 * g + 4 * c4;        // H2 slice
        else if (NL == 3 && part == 1) off = 3072 + r * kH2 + 16 * g + 4 * c4;   // dZ2 slice
        else off = (NL == 3 ? 4096 : 2048) + r * 16 + 4 * c4;                    // dZ of the logits
        v[j] = ld_f4(rb, kOffCx * 2 + ((int64_t)par * kNCH + c) * kCX + off);
      }
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int x = tid + j * kThreads;
        const int part = x >> 8, c = (x >> 6) & 3, r = (x >> 2) & 15, c4 = x & 3;
        float* dst;
        if constexpr (NL == 3) dst = lds + (part == 0 ? GLay<3>::H2T : part == 1 ? GLay<3>::DZ2T : GLay<3>::DZ3T);
        else dst = DZ2T;
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[(4 * c4 + e) * kST + 16 * c + r] = v[j][e];
      }
    }
    __syncthreads();
    PK_STAMP(2, 1);

    if constexpr (NL == 3) {
      float* W3 = lds + L::W3;
      float* B3 = lds + L::B3;
      float* H2T = lds + L::H2T;
      float* DZ3T = lds + L::DZ3T;
      float* RED = lds + L::RED;
      // dW2 rows [16 h of the slice][128 n] = dZ2^T H1; wave w: n tiles 2w, 2w+1,
      // two accumulator chains per tile; dW3 columns [16 o][16 h] = dZ3^T H2 over
      // the wave's 16-row quarter; bias gradients = row sums of the transposed
      // operands (db2 slice: wave 0, db3: wave 1), all in a fixed order
      f32x4 c0[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      f32x4 c1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      f32x4 g3 = {0.f, 0.f, 0.f, 0.f};
      float4 av[4], b0[4], b1[4];
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        av[gq] = *reinterpret_cast<const float4*>(DZ2T + i * kST + 16 * gq + 4 * q);
        b0[gq] = *reinterpret_cast<const float4*>(H1T + (32 * w + i) * kST + 16 * gq + 4 * q);
        b1[gq] = *reinterpret_cast<const float4*>(H1T + (32 * w + 16 + i) * kST + 16 * gq + 4 * q);
      }
      const float4 a3 = *reinterpret_cast<const float4*>(DZ3T + i * kST + 16 * w + 4 * q);
      const float4 h3 = *reinterpret_cast<const float4*>(H2T + i * kST + 16 * w + 4 * q);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        c0[0] = mfma_f32_16x16x4(av[gq].x, b0[gq].x, c0[0]);
        c0[1] = mfma_f32_16x16x4(av[gq].x, b1[gq].x, c0[1]);
        c1[0] = mfma_f32_16x16x4(av[gq].y, b0[gq].y, c1[0]);
        c1[1] = mfma_f32_16x16x4(av[gq].y, b1[gq].y, c1[1]);
        c0[0] = mfma_f32_16x16x4(av[gq].z, b0[gq].z, c0[0]);
        c0[1] = mfma_f32_16x16x4(av[gq].z, b1[gq].z, c0[1]);
        c1[0] = mfma_f32_16x16x4(av[gq].w, b0[gq].w, c1[0]);
        c1[1] = mfma_f32_16x16x4(av[gq].w, b1[gq].w, c1[1]);
      }
      g3 = mfma_f32_16x16x4(a3.x, h3.x, g3);
      g3 = mfma_f32_16x16x4(a3.y, h3.y, g3);
      g3 = mfma_f32_16x16x4(a3.z, h3.z, g3);
      g3 = mfma_f32_16x16x4(a3.w, h3.w, g3);
      f32x4 gw[2] = {c0[0] + c1[0], c0[1] + c1[1]};
#pragma unroll
      for (int r = 0; r < 4; ++r) RED[w * 256 + (4 * q + r) * 16 + i] = g3[r];
      float sb = 0.f;
      if (w < 2) {
        const float* rowp = (w == 0 ? DZ2T : DZ3T) + i * kST + 4 * q;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const float4 x = *reinterpret_cast<const float4*>(rowp + 16 * gq);
          sb += (x.x + x.y) + (x.z + x.w);
        }
        sb += __shfl_xor(sb, 16, 64);
        sb += __shfl_xor(sb, 32, 64);
      }
      __syncthreads();
      if (w == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = (4 * q + r) * 16 + i;
          g3[r] = (RED[e] + RED[256 + e]) + (RED[512 + e] + RED[768 + e]);
        }
      }
      // wave 1's db3 to wave 0 through LDS (RED row 0 is free again after the barrier)
      __syncthreads();
      if (w == 1 && q == 0) RED[i] = sb;
      __syncthreads();
      float sb3 = RED[i];
      PK_STAMP(2, 2);
      if (DP) {
        bool xok;
        if (w == 0) {
          float4 v[4] = {make_float4(gw[0][0], gw[0][1], gw[0][2], gw[0][3]),
                         make_float4(gw[1][0], gw[1][1], gw[1][2], gw[1][3]),
                         make_float4(g3[0], g3[1], g3[2], g3[3]), make_float4(sb, sb3, 0.f, 0.f)};
          xok = px_sum_wave<4>(a, s, v, kNL1 * 4 + g * 4 + w);
          gw[0] = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
          gw[1] = f32x4{v[1].x, v[1].y, v[1].z, v[1].w};
          g3 = f32x4{v[2].x, v[2].y, v[2].z, v[2].w};
          sb = v[3].x;
          sb3 = v[3].y;
        } else {
          float4 v[2] = {make_float4(gw[0][0], gw[0][1], gw[0][2], gw[0][3]),
                         make_float4(gw[1][0], gw[1][1], gw[1][2], gw[1][3])};
          xok = px_sum_wave<2>(a, s, v, kNL1 * 4 + g * 4 + w);
          gw[0] = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
          gw[1] = f32x4{v[1].x, v[1].y, v[1].z, v[1].w};
        }
        ok = __syncthreads_and(xok ? 1 : 0) != 0;
        if (!ok) break;
      }
      // SGD on the resident slice
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) W2[(4 * q + r) * kS1 + 32 * w + 16 * tt + i] -= a.lr * gw[tt][r];
      if (w == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * q + r < kNC) W3[(4 * q + r) * kSG + i] -= a.lr * g3[r];
        if (q == 0) {
          B2[i] -= a.lr * sb;
          if (i < kNC) B3[i] -= a.lr * sb3;
        }
      }
      __syncthreads();
      PK_STAMP(2, 3);
      // ---- publish the slice: W2 rows 512 f4, W3 columns 64 f4, b2 4, b3 4 ----
      const int64_t dst = kOffWx * 2 + ((int64_t)par * kNG + g) * kWX;
      for (int e = tid; e < 584; e += kThreads) {
        const float* src;
        if (e < 512) src = W2 + (e >> 5) * kS1 + 4 * (e & 31);
        else if (e < 576) src = W3 + ((e - 512) >> 2) * kSG + 4 * ((e - 512) & 3);
        else if (e < 580) src = B2 + 4 * (e - 576);
        else src = B3 + 4 * (e - 580);
        st_up4(rb, dst + 4 * e, f4v{src[0], src[1], src[2], src[3]}, local);
      }
    } else {
      // dW2 columns [16 o][32 n of the slice] = dZ2^T H1: waves 0, 1 one n tile
      // each (two chains); db2 (wave 2, row sums) applied by block 0
      f32x4 gw = {0.f, 0.f, 0.f, 0.f}, gx = {0.f, 0.f, 0.f, 0.f};
      float sb = 0.f;
      if (w < 2) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const float4 av = *reinterpret_cast<const float4*>(DZ2T + i * kST + 16 * gq + 4 * q);
          const float4 bv = *reinterpret_cast<const float4*>(H1T + (16 * w + i) * kST + 16 * gq + 4 * q);
          gw = mfma_f32_16x16x4(av.x, bv.x, gw);
          gx = mfma_f32_16x16x4(av.y, bv.y, gx);
          gw = mfma_f32_16x16x4(av.z, bv.z, gw);
          gx = mfma_f32_16x16x4(av.w, bv.w, gx);
        }
        gw = gw + gx;
      } else if (w == 2) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const float4 x = *reinterpret_cast<const float4*>(DZ2T + i * kST + 16 * gq + 4 * q);
          sb += (x.x + x.y) + (x.z + x.w);
        }
        sb += __shfl_xor(sb, 16, 64);
        sb += __shfl_xor(sb, 32, 64);
      }
      PK_STAMP(2, 2);
      if (DP) {
        bool xok = true;
        if (w < 3) {
          float4 v[1] = {w < 2 ? make_float4(gw[0], gw[1], gw[2], gw[3]) : make_float4(sb, 0.f, 0.f, 0.f)};
          xok = px_sum_wave<1>(a, s, v, kNL1 * 4 + g * 4 + w);
          if (w < 2) gw = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
          else sb = v[0].x;
        }
        ok = __syncthreads_and(xok ? 1 : 0) != 0;
        if (!ok) break;
      }
      if (w < 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * q + r < kNC) W2[(4 * q + r) * kSW + 16 * w + i] -= a.lr * gw[r];
      } else if (w == 2 && q == 0 && i < kNC && g == 0) {
        B2[i] -= a.lr * sb;
      }
      __syncthreads();
      PK_STAMP(2, 3);
      // ---- publish: W2 columns [16 o][32] (128 f4), b2 (4 f4) ----
      const int64_t dst = kOffWx * 2 + ((int64_t)par * kNG + g) * kWX;
      for (int e = tid; e < 132; e += kThreads) {
        const float* src = e < 128 ? W2 + (e >> 3) * kSW + 4 * (e & 7) : B2 + 4 * (e - 128);
        st_up4(rb, dst + 4 * e, f4v{src[0], src[1], src[2], src[3]}, local);
      }
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_gran(rb, kOffWf + par * kNG + g, __uint_as_float(tag), tag);
    PK_STAMP(2, 4);
  }

  // ---- epilogue: the slice back to HBM ----
  if constexpr (NL == 3) {
    float* W3 = lds + L::W3;
    float* B3 = lds + L::B3;
    for (int e = tid; e < 16 * (kD1 / 4); e += kThreads) {
      const int r = e >> 5, c4 = e & 31;
      *reinterpret_cast<float4*>(a.P + a.w_off[1] + (int64_t)(16 * g + r) * kD1 + 4 * c4) =
          *reinterpret_cast<const float4*>(W2 + r * kS1 + 4 * c4);
    }
    {
      const int o = tid >> 4, j = tid & 15;
      if (o < kNC) a.P[a.w_off[2] + (int64_t)o * kH2 + 16 * g + j] = W3[o * kSG + j];
    }
    if (tid < 16) a.P[a.b_off[1] + 16 * g + tid] = B2[tid];
    if (g == 0 && tid < kNC) a.P[a.b_off[2] + tid] = B3[tid];
  } else {
    for (int e = tid; e < kNC * 32; e += kThreads) {
      const int o = e >> 5, j = e & 31;
      a.P[a.w_off[1] + (int64_t)o * kD1 + 32 * g + j] = W2[o * kSW + j];
    }
    if (g == 0 && tid < kNC) a.P[a.b_off[1] + tid] = B2[tid];
  }
  pk_report(a, ok);
}


// -----------------------------------------------------------------------------
// Gradient tile (single replica): full-batch dW / db + SGD of one tile of the
// upper weights.  3 layers, tile g: W2 rows 16 gh .. +15 x columns 32 gn .. +31
// (gh = g / 4, gn = g % 4); the gn == 0 tiles also own W3 columns 16 gh .. +15
// and b2[16 gh ..], tile 0 b3.  2 layers, tile g: W2 columns 16 g .. +15 (all
// class rows); tile 0 b2.
// -----------------------------------------------------------------------------
struct GTLay {
  static constexpr int H1T = 0;                 // [32 n][kST] (rows contiguous)
  static constexpr int DZ2T = H1T + 32 * kST;   // [16][kST]
  static constexpr int H2T = DZ2T + 16 * kST;   // [16][kST]
  static constexpr int DZ3T = H2T + 16 * kST;   // [16][kST]
  static constexpr int W2 = DZ3T + 16 * kST;    // tile [16][33]
  static constexpr int W3 = W2 + 16 * 33;       // [16 o][17]
  static constexpr int B = W3 + 16 * 17;        // b2 slice [16], b3 [16]
  static constexpr int STG = B + 32;            // data parallel: the slots' values [3][64 lanes] f4
  static constexpr int BST = STG + 3 * 256;     // data parallel: bias partials [2][16]
  static constexpr int TOTAL = BST + 32;
};
static_assert(GTLay::STG % 4 == 0, "slot stage: 16-B aligned");

template <int NL, bool XM>
__device__ __forceinline__ void pk_gtile(const PersistArgs& a, float* lds, int g, int blk) {
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int i = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  pk_started(a, blk, s0);
  float* H1T = lds + GTLay::H1T;
  float* DZ2T = lds + GTLay::DZ2T;
  float* H2T = lds + GTLay::H2T;
  float* DZ3T = lds + GTLay::DZ3T;
  float* W2 = lds + GTLay::W2;
  float* W3 = lds + GTLay::W3;
  float* Bs = lds + GTLay::B;
  float4* Stg = reinterpret_cast<float4*>(lds + GTLay::STG);
  float* Bst = lds + GTLay::BST;
  __shared__ uint32_t s_xfail;  // a wave's exchange gave up (set once: the loop then ends)
  if (tid == 0) s_xfail = 0u;
  // tile geometry: W2 rows r0 .. r0 + 15 (3 layers: h; 2 layers: class o),
  // columns n0 .. n0 + nw - 1
  constexpr int nw = NL == 3 ? 32 : 16;
  const int gh = NL == 3 ? g >> 2 : 0;
  const int n0 = NL == 3 ? 32 * (g & 3) : 16 * g;
  const bool own3 = NL == 3 && (g & 3) == 0;  // W3 columns + b2 slice (3 layers)
  const int r0 = 16 * gh;

  // ---- prologue: the tile (and its extras) from P ----
  for (int e = tid; e < 16 * nw; e += kThreads) {
    const int r = e / nw, c = e - r * nw;
    W2[r * 33 + c] = (NL == 3 || r < kNC) ? a.P[a.w_off[1] + (int64_t)(r0 + r) * kD1 + n0 + c] : 0.f;
  }
  if (own3) {
    const int o = tid >> 4, j = tid & 15;
    W3[o * 17 + j] = o < kNC ? a.P[a.w_off[2] + (int64_t)o * kH2 + r0 + j] : 0.f;
    if (tid < 16) Bs[tid] = a.P[a.b_off[1] + r0 + tid];
  }
  if (g == 0 && tid < 16) {
    if constexpr (NL == 3) Bs[16 + tid] = tid < kNC ? a.P[a.b_off[2] + tid] : 0.f;
    else Bs[tid] = tid < kNC ? a.P[a.b_off[1] + tid] : 0.f;
  }
  __syncthreads();
  bool ok = true;
  const bool local = pk_upper_local(a, s0, poll, ok, kNCH + GTile<NL>::kN);
  // the staged slots stay in the L2 only when the pushers share the upper
  // group's XCD (3 helpers: pushers on XCD 0), else they are written through
  const int hl = XM && a.pushers && pk_push_xcd0(a.helpers) ? kPushers<NL>() : 0;
  const bool xs_local = hl ? pk_upper_local(a, s0, poll, ok, kNCH + GTile<NL>::kN + hl) : false;
  const int stamp_on = g == 0 ? g_pk_stamp_on : 0;
  const int jit = g_pk_jitter;
  for (int it = 0; it < a.steps && ok; ++it) {
    PK_STAMP(2, 0);
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    const int par = (int)(s & 1);
    pk_jit(jit, blk, s, 4);
    // ---- part 0: the tile's H1 columns of the 64 rows (flagged in the chains' forward) ----
    if (tid < kNCH && !wait_flag(rb, kOffCxf + par * kNCH + tid, tag, poll)) ok = false;
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    {
      constexpr int kC4 = nw / 4, kIt = 64 * kC4 / kThreads;  // f4 per row, per thread
      f4v v[kIt];
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int x = tid + j * kThreads, r = x / kC4, c4 = x - r * kC4;
        v[j] = ld_f4(rb, kOffCx * 2 + ((int64_t)par * kNCH + (r >> 4)) * kCX + (r & 15) * kD1 + n0 + 4 * c4);
      }
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int x = tid + j * kThreads, r = x / kC4, c4 = x - r * kC4;
#pragma unroll
        for (int e = 0; e < 4; ++e) H1T[(4 * c4 + e) * kST + r] = v[j][e];
      }
    }
    // ---- part 1: the rest of the rows (flagged at the end of the chains' step) ----
    if (tid < kNCH && !wait_flag(rb, kOffCxf + 8 + par * kNCH + tid, tag, poll)) ok = false;
    ok = __syncthreads_and(ok ? 1 : 0) != 0;
    if (!ok) break;
    {
      // thread -> row r = tid / 4, 4 columns 4 (tid % 4); 3 layers: dZ2 slice
      // (and H2 slice + dZ3 for the W3 owners); 2 layers: the logits' gradient
      const int r = tid >> 2, c4 = tid & 3;
      const int64_t rowb = kOffCx * 2 + ((int64_t)par * kNCH + (r >> 4)) * kCX + (r & 15) * (NL == 3 ? kH2 : 16);
      f4v vd, vh = {0.f, 0.f, 0.f, 0.f}, v3 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (NL == 3) {
        vd = ld_f4(rb, rowb + 3072 + r0 + 4 * c4);    // dZ2 [16][64] at 3072 of the chain's run
        if (own3) {
          vh = ld_f4(rb, rowb + 2048 + r0 + 4 * c4);  // H2 [16][64] at 2048
          v3 = ld_f4(rb, kOffCx * 2 + ((int64_t)par * kNCH + (r >> 4)) * kCX + 4096 + (r & 15) * 16 + 4 * c4);
        }
      } else {
        vd = ld_f4(rb, rowb + 2048 + 4 * c4);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        DZ2T[(4 * c4 + e) * kST + r] = vd[e];
        if (own3) {
          H2T[(4 * c4 + e) * kST + r] = vh[e];
          DZ3T[(4 * c4 + e) * kST + r] = v3[e];
        }
      }
    }
    __syncthreads();
    PK_STAMP(2, 1);

    // ---- gradients: 16 MFMAs per 16 x 16 output tile (K = the 64 rows), each
    // lane's 16-B LDS reads feeding 4 MFMAs (k = 16 gq + 4 q + j) ----
    f32x4 gw = {0.f, 0.f, 0.f, 0.f};
    float sb = 0.f;
    auto tile16 = [&](const float* A, const float* Bm) {
      f32x4 c[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const float4 av = *reinterpret_cast<const float4*>(A + i * kST + 16 * gq + 4 * q);
        const float4 bv = *reinterpret_cast<const float4*>(Bm + i * kST + 16 * gq + 4 * q);
        c[0] = mfma_f32_16x16x4(av.x, bv.x, c[0]);
        c[1] = mfma_f32_16x16x4(av.y, bv.y, c[1]);
        c[2] = mfma_f32_16x16x4(av.z, bv.z, c[2]);
        c[3] = mfma_f32_16x16x4(av.w, bv.w, c[3]);
      }
      return (c[0] + c[1]) + (c[2] + c[3]);
    };
    auto rowsum = [&](const float* A) {  // sum over the 64 rows of feature i (16 lanes x 4 q)
      float t = 0.f;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const float4 x = *reinterpret_cast<const float4*>(A + i * kST + 16 * gq + 4 * q);
        t += (x.x + x.y) + (x.z + x.w);
      }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      return t;
    };
    if constexpr (NL == 3) {
      if (w < 2) gw = tile16(DZ2T, H1T + 16 * w * kST);          // dW2 [16 h][16 n]
      else if (w == 2 && own3) gw = tile16(DZ3T, H2T);           // dW3 [16 o][16 h]
      else if (w == 3 && own3) sb = rowsum(DZ2T);                // db2 slice
      float sb3 = 0.f;
      if (w == 3 && g == 0) sb3 = rowsum(DZ3T);                  // db3
      PK_STAMP(2, 2);
      if constexpr (XM) {  // data parallel: this wave's gradients summed over the replicas
        bool xok = true;
        if (a.algo == 0) {
          // tagged one-shot: the bias partials ride in the dW3 slot's padding
          // rows o = 12, 13 (q == 3), so a tile has 2 slots (3 with W3).  The
          // slots are staged for this tile's pusher block (XS + flag, raised by
          // wave 3, which has no store of its own outstanding), and waves
          // 0 .. nslot-1 gather with no push on this CU's memory pipe
          if (w == 3 && q == 0) { Bst[i] = sb; Bst[16 + i] = sb3; }
          lds_barrier();
          const int nslot = own3 ? 3 : 2;
          if (w == 2 && own3 && q == 3) { gw[0] = Bst[i]; gw[1] = Bst[16 + i]; }
          if (w < nslot) Stg[w * 64 + lane] = make_float4(gw[0], gw[1], gw[2], gw[3]);
          lds_barrier();
          if (w == 3) {
            if (a.pushers) {  // stage every slot as tagged granules for the pusher block (no drain)
              for (int k = 0; k < nslot; ++k) pk_xs_put(rb, pk_xs_g(s, g, k, lane), Stg[k * 64 + lane], tag, xs_local);
            } else {  // few peers: wave 3 pushes every slot itself
              float4 v3[3];
#pragma unroll
              for (int k = 0; k < 3; ++k) v3[k] = k < nslot ? Stg[k * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
              px_tagged_push_part(a, s, v3, nslot, kNL1 * 4 + 4 * g, 0, 1);
            }
          }
          PK_STAMP(2, 5);
          const int dbg = stamp_on && it >= stamp_on - 1 ? it - (stamp_on - 1) : -1;
          if (w < nslot) {
            float4 v[1] = {make_float4(gw[0], gw[1], gw[2], gw[3])};
            xok = px_tagged_gather<1>(a, s, v, kNL1 * 4 + 4 * g + w, w == 0 ? dbg : -1);
            gw = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
            if (w == 2 && q == 3) { sb = gw[0]; sb3 = gw[1]; }
          }
          PK_STAMP(2, 6);
          // agreed without a vector-memory drain (wave 3's staging stores stay in flight)
          if (!xok) s_xfail = 1u;
          lds_barrier();
          PK_STAMP(2, 7);
          if (s_xfail != 0u) { ok = false; break; }
        } else {
          float4 v[1];
          if (w < 2 || (w == 2 && own3)) {
            v[0] = make_float4(gw[0], gw[1], gw[2], gw[3]);
            xok = px_sum_wave_g<1>(a, s, v, kNL1 * 4 + 4 * g + w);
            gw = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
          } else if (w == 3 && (own3 || g == 0)) {
            v[0] = make_float4(sb, sb3, 0.f, 0.f);
            xok = px_sum_wave_g<1>(a, s, v, kNL1 * 4 + 4 * g + w);
            sb = v[0].x;
            sb3 = v[0].y;
          }
          ok = __syncthreads_and(xok ? 1 : 0) != 0;
          if (!ok) break;
        }
      }
      // ---- SGD on the resident tile ----
      if (w < 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) W2[(4 * q + r) * 33 + 16 * w + i] -= a.lr * gw[r];
      }
      if (w == 2 && own3) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * q + r < kNC) W3[(4 * q + r) * 17 + i] -= a.lr * gw[r];
        if (XM && a.algo == 0 && q == 3) {  // the summed bias partials (packed rows 12, 13)
          Bs[i] -= a.lr * sb;
          if (g == 0 && i < kNC) Bs[16 + i] -= a.lr * sb3;
        }
      } else if (w == 3 && q == 0 && !(XM && a.algo == 0)) {
        if (own3) Bs[i] -= a.lr * sb;
        if (g == 0 && i < kNC) Bs[16 + i] -= a.lr * sb3;
      }
    } else {
      if (w == 0) gw = tile16(DZ2T, H1T);                         // dW2 [16 o][16 n]
      else if (w == 1 && g == 0) sb = rowsum(DZ2T);               // db2
      PK_STAMP(2, 2);
      if constexpr (XM) {
        bool xok = true;
        if (a.algo == 0) {
          // tagged one-shot: the b2 partial rides in the dW2 slot's padding
          // row o = 12 (q == 3); the slot is staged for the pusher block
          if (w == 1 && q == 0) Bst[i] = sb;
          lds_barrier();
          if (w == 0 && q == 3) gw[0] = Bst[i];
          if (w == 0) Stg[lane] = make_float4(gw[0], gw[1], gw[2], gw[3]);
          lds_barrier();
          if (w == 3) {
            if (a.pushers) {
              pk_xs_put(rb, pk_xs_g(s, g, 0, lane), Stg[lane], tag, xs_local);
            } else {
              const float4 v3[3] = {Stg[lane], make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
              px_tagged_push_part(a, s, v3, 1, kNL1 * 4 + 4 * g, 0, 1);
            }
          }
          if (w == 0) {
            float4 v[1] = {make_float4(gw[0], gw[1], gw[2], gw[3])};
            xok = px_tagged_gather<1>(a, s, v, kNL1 * 4 + 4 * g);
            gw = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
            if (q == 3) sb = gw[0];
          }
          if (!xok) s_xfail = 1u;
          lds_barrier();
          if (s_xfail != 0u) { ok = false; break; }
        } else {
          float4 v[1];
          if (w == 0) {
            v[0] = make_float4(gw[0], gw[1], gw[2], gw[3]);
            xok = px_sum_wave_g<1>(a, s, v, kNL1 * 4 + 4 * g + w);
            gw = f32x4{v[0].x, v[0].y, v[0].z, v[0].w};
          } else if (w == 1 && g == 0) {
            v[0] = make_float4(sb, 0.f, 0.f, 0.f);
            xok = px_sum_wave_g<1>(a, s, v, kNL1 * 4 + 4 * g + w);
            sb = v[0].x;
          }
          ok = __syncthreads_and(xok ? 1 : 0) != 0;
          if (!ok) break;
        }
      }
      if (w == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * q + r < kNC) W2[(4 * q + r) * 33 + i] -= a.lr * gw[r];
        if (XM && a.algo == 0 && q == 3 && g == 0 && i < kNC) Bs[i] -= a.lr * sb;
      } else if (w == 1 && g == 0 && q == 0 && i < kNC && !(XM && a.algo == 0)) {
        Bs[i] -= a.lr * sb;
      }
    }
    lds_barrier();  // no vector-memory drain: wave 3's pushes (data parallel) stay in flight
    PK_STAMP(2, 3);
    pk_jit(jit, blk, s, 5);
    // ---- publish the tile into WXS[par] (the chains' order), by waves 0-2:
    // W2 tile f4 0 .. kT4-1, then (W3 owners) 64 W3 f4 and 4 b2 f4, then (tile 0) 4 b3 f4 ----
    if (w < 3) {
      const int64_t base = kOffWxs * 2 + (int64_t)par * kWXS;
      constexpr int kT4 = 16 * nw / 4;  // f4 of the W2 tile
      const int nitem = kT4 + (NL == 3 && own3 ? 68 : 0) + (g == 0 ? 4 : 0);
      for (int x = tid; x < nitem; x += 192) {
        if (x < kT4) {
          const int r = x / (nw / 4), c4 = x - r * (nw / 4);
          const float* src = W2 + r * 33 + 4 * c4;
          st_up4(rb, base + (int64_t)(r0 + r) * kD1 + n0 + 4 * c4, f4v{src[0], src[1], src[2], src[3]}, local);
        } else if (NL == 3 && own3 && x < kT4 + 64) {
          const int y = x - kT4, o = y >> 2, c4 = y & 3;
          const float* src = W3 + o * 17 + 4 * c4;
          st_up4(rb, base + kH2 * kD1 + o * kH2 + r0 + 4 * c4, f4v{src[0], src[1], src[2], src[3]}, local);
        } else if (NL == 3 && own3 && x < kT4 + 68) {
          const int c4 = x - kT4 - 64;
          st_up4(rb, base + kH2 * kD1 + 16 * kH2 + r0 + 4 * c4,
                 f4v{Bs[4 * c4], Bs[4 * c4 + 1], Bs[4 * c4 + 2], Bs[4 * c4 + 3]}, local);
        } else {  // tile 0: b3 (3 layers) / b2 (2 layers)
          const int c4 = x - (nitem - 4);
          const float* src = Bs + (NL == 3 ? 16 : 0) + 4 * c4;
          st_up4(rb, base + (NL == 3 ? kH2 * kD1 + 16 * kH2 + kH2 : 16 * kD1) + 4 * c4,
                 f4v{src[0], src[1], src[2], src[3]}, local);
        }
      }
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    if (tid == 0) st_gran(rb, kOffWfs + par * 16 + g, __uint_as_float(tag), tag);
    PK_STAMP(2, 4);
  }

  // ---- epilogue: the tile back to HBM ----
  for (int e = tid; e < 16 * nw; e += kThreads) {
    const int r = e / nw, c = e - r * nw;
    if (NL == 3 || r < kNC) a.P[a.w_off[1] + (int64_t)(r0 + r) * kD1 + n0 + c] = W2[r * 33 + c];
  }
  if (own3) {
    const int o = tid >> 4, j = tid & 15;
    if (o < kNC) a.P[a.w_off[2] + (int64_t)o * kH2 + r0 + j] = W3[o * 17 + j];
    if (tid < 16) a.P[a.b_off[1] + r0 + tid] = Bs[tid];
  }
  if (g == 0 && tid < kNC) {
    if constexpr (NL == 3) a.P[a.b_off[2] + tid] = Bs[16 + tid];
    else a.P[a.b_off[1] + tid] = Bs[tid];
  }
  pk_report(a, ok);
}

// Pusher block p (data-parallel Gram forms, tagged tile sums): pushes the
// staged slots of gradient tiles p and p + kPushers to every peer -- waves
// 0, 1 tile p, waves 2, 3 tile p + kPushers, each wave half the peers -- so the
// tiles' gathers never queue behind their own pushes.  Same XCD as the tiles
// (blockIdx 8 k): the staged slots stay in that L2.
#ifdef HIPDSML_MEASURE
// measurement builds (tools/pk_probe.py --push-stamps): pusher 0 wave 0 per stamped
// step: poll entry, tile 0's staged slots seen, pushes issued, pushes acknowledged
__device__ uint64_t g_pk_push_st[8][4];
#define PUSH_STAMP(k)                                                                          \
  do {                                                                                         \
    if (p == 0 && tid == 0 && stamp_on && it >= stamp_on - 1 && it < stamp_on + 7)             \
      g_pk_push_st[it - (stamp_on - 1)][(k)] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
#else
#define PUSH_STAMP(k) do {} while (0)
#endif
template <int NL>
__device__ __forceinline__ void pk_pusher(const PersistArgs& a, int p, int blk) {
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
#ifdef HIPDSML_MEASURE
  const int stamp_on = g_pk_stamp_on;
#endif
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.xb);
  Poll poll{a.err, a.timeout_ticks, 0, 0};
  const uint64_t s0 = ld_ctr64(a.ctr + 1);
  pk_started(a, blk, s0);
  const int g = p + (w >> 1) * kPushers<NL>();
  const int nslot = NL == 3 ? ((g & 3) == 0 ? 3 : 2) : 1;
  bool ok = true;
  for (int it = 0; it < a.steps && ok; ++it) {
    const uint64_t s = s0 + (uint64_t)it;
    const uint32_t tag = (uint32_t)(s + 1);
    const int par = (int)(s & 1);
    // the tile's staged slots, polled by their tags (every load of a round in flight)
    uint4 u[3][2];
    PUSH_STAMP(0);
    poll.start();
    for (;;) {
      bool all = true;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k < nslot) {
          u[k][0] = ld_gran2(rb, pk_xs_g(s, g, k, lane));
          u[k][1] = ld_gran2(rb, pk_xs_g(s, g, k, lane) + 2);
          all = all && u[k][0].y == tag && u[k][0].w == tag && u[k][1].y == tag && u[k][1].w == tag;
        }
      }
      if (__builtin_amdgcn_ballot_w64(!all) == 0) break;
      if (!poll.again()) { ok = false; break; }
    }
    if (!ok) break;
    (void)par;
    float4 v[3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
      v[k] = k < nslot ? make_float4(__uint_as_float(u[k][0].x), __uint_as_float(u[k][0].z),
                                     __uint_as_float(u[k][1].x), __uint_as_float(u[k][1].z))
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    PUSH_STAMP(1);
    px_tagged_push_part(a, s, v, nslot, kNL1 * 4 + 4 * g, w & 1, 2);
    PUSH_STAMP(2);
#ifdef HIPDSML_MEASURE
    if (p == 0 && stamp_on) {
      __builtin_amdgcn_s_waitcnt(0);  // measurement only: when the pushes landed
      PUSH_STAMP(3);
    }
#endif
  }
  pk_report(a, ok);
}

// DP: the data-parallel form (replica exchange compiled in); the single-replica
// launch runs the exchange-free code.  Placement (speed only, every hand-off is
// placement-independent): under round-robin dispatch blocks b and b + 8 share
// an XCD, so the chains and gradient blocks (b % 8 == 0) share one XCD and the
// 8 layer-1 blocks of one k slice (b % 8 == gk + 1) share another, whose L2
// then serves their common X slice once.
// MODE 0: single replica (Gram form); 1: data parallel, direct form (pk /
// pk2); 2: data parallel, Gram form (pkg / pkg2); 3: data parallel,
// exchange-free layer 1 (pkx).
template <int NL, int MODE>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1)))
void mlp_persist_k(PersistArgs a) {
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int b = blockIdx.x;
  const int x = b & 7, y = b >> 3;
  if constexpr (MODE == 1) {
    if (x == 0) {
      if (y < kNCH) pk_chain<NL, true>(a, lds, y, b);
      else pk_grad<NL, true>(a, lds, y - kNCH, b);
    } else {
      pk_layer1<true>(a, lds, y + kGN * (x - 1), b);
    }
  } else {
    // 4 chains + the gradient tiles at blockIdx 8 k (one XCD under
    // round-robin dispatch), layer-1 block (gn, gk) at 8 gn + gk + 1; the
    // grid's other blocks exit at once
    constexpr bool XM = MODE >= 2;
    const int hl = MODE == 3 ? a.helpers : 0;
    if (!pk_sr_active<NL>(b, hl, a.pushers != 0)) return;
    if constexpr (XM) {
      const int pu = pk_pusher_of<NL>(b, hl, a.pushers != 0);
      if (pu >= 0) {
        pk_pusher<NL>(a, pu, b);
        return;
      }
    }
    if (x == 0) {
      if (y < kNCH) pk_chain<NL, false, XM>(a, lds, y, b);
      else pk_gtile<NL, XM>(a, lds, y - kNCH, b);
    } else if (y < kGN) {
      pk_layer1_gram<NL, MODE == 3 ? 2 : MODE == 2 ? 1 : 0>(a, lds, y + kGN * (x - 1), b);
    } else if constexpr (MODE == 3) {
      pk_l1_helper(a, lds, y % kGN + kGN * (x - 1), y / kGN, b);
    }
  }
}

hipError_t mlp_persist_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_pk_stamps), sizeof(uint64_t) * 4 * 8 * 8, 0,
                             hipMemcpyDeviceToHost);
}
void mlp_persist_set_jitter(int ticks) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pk_jitter), &ticks, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
#ifdef HIPDSML_MEASURE
hipError_t mlp_persist_read_push_stamps(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pk_push_st), sizeof(g_pk_push_st), 0, hipMemcpyDeviceToHost);
}
void mlp_persist_set_hop(int ticks) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pk_hop), &ticks, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
#endif
void mlp_persist_set_probe(int mode) {
  g_pk_probe_mode = mode;
  const int v = mode == 1 ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pk_probe), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
void mlp_persist_set_pkx_helpers(int helpers) { g_pkx_helpers = helpers < 0 ? -1 : helpers; }
void mlp_persist_set_pkx_l1push(int mode) { g_pkx_l1push = mode < 0 ? -1 : (mode ? 1 : 0); }
void mlp_persist_set_stamp_window(int first_step) {
  const int v = first_step < 0 ? 0 : first_step + 1;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pk_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
void mlp_persist_set_stamping(bool on) {
  const int v = on ? 9 : 0;  // steps 8-15
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pk_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}

bool mlp_persist_supported(const MlpDesc& d) {
  if (d.batch < 1 || d.batch > kB || d.nbatches < 1 || d.dims[0] != kD0 || d.dims[1] != kD1)
    return false;
  if (d.nlayers == 3) return d.dims[2] == kH2 && d.dims[3] == kNC;
  if (d.nlayers == 2) return d.dims[2] == kNC;
  return false;
}

int64_t mlp_persist_xbuf_granules() { return kTotalP; }

template <int NL, int MODE>
static hipError_t pk_launch(const PersistArgs& a, hipStream_t s) {
  const size_t lds = (size_t)lds_floats<NL>() * sizeof(float);
  static bool attr = false;
  static int slots = 0;  // co-resident workgroups (occupancy x CUs)
  if (!attr) {
    const void* f = reinterpret_cast<const void*>(mlp_persist_k<NL, MODE>);
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // Every block waits on others: the whole grid must be co-resident.  This
    // is the check a cooperative launch makes per launch (host wall +15-19 us
    // each, MI355X_MICROARCH "coop-launch"), made once here instead.
    int per_cu = 0, dev = 0, cus = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, kThreads, lds);
    if (e != hipSuccess) return e;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
      return e;
    if (per_cu < 1) return hipErrorCooperativeLaunchTooLarge;
    slots = per_cu * cus;
    attr = true;
  }
  // HIPDSML_PK_GRID_EXTRA (measurement builds only): that many more idle
  // workgroups (rounded to whole rows of 8, so the XCD map holds) -- prices the
  // idle blocks the round-robin XCD placement forces on the single-replica grid
#ifdef HIPDSML_MEASURE
  static const int extra = [] {
    const char* e = std::getenv("HIPDSML_PK_GRID_EXTRA");
    return e ? std::max(0, std::atoi(e)) / 8 * 8 : 0;
  }();
#else
  constexpr int extra = 0;
#endif
  const int grid = pk_grid<NL>(MODE == 1, MODE == 3 ? a.helpers : 0, a.pushers != 0) + (MODE == 0 ? extra : 0);
  if (slots < grid) return hipErrorCooperativeLaunchTooLarge;
  hipLaunchKernelGGL((mlp_persist_k<NL, MODE>), dim3(grid), dim3(kThreads), lds, s, a);
  return hipGetLastError();
}

hipError_t mlp_persist_steps(const float* X, int64_t ldx, const int32_t* labels, float* P,
                             int64_t* ctr, const MlpDesc& d, float lr, int steps, uint64_t* xb,
                             float* stats, uint32_t* err, uint32_t* herr, uint64_t timeout_ticks,
                             hipStream_t s, const XchgArgs* xa, const XchgTab* tab, int algo,
                             const float* gram, int carry, const float* xsw, int64_t xsw_stride) {
  if (!mlp_persist_supported(d) || steps < 1 || xb == nullptr || err == nullptr || ctr == nullptr ||
      (ldx % 4) != 0 || ldx < kD0 || (((uintptr_t)X) & 15) != 0)
    return hipErrorInvalidValue;
  PersistArgs a{};
  a.X = X;
  a.ldx = ldx;
  a.labels = labels;
  a.P = P;
  for (int l = 0; l < d.nlayers; ++l) {
    a.w_off[l] = d.w_off[l];
    a.b_off[l] = d.b_off[l];
    if ((d.w_off[l] % 4) != 0 || (d.b_off[l] % 4) != 0) return hipErrorInvalidValue;  // 16-B rows
  }
  a.ctr = ctr;
  a.nbatches = d.nbatches;
  a.batch = d.batch;
  a.steps = steps;
  a.lr = lr;
  a.inv_batch = 1.0f / (float)d.batch;
  a.xb = xb;
  a.stats = stats;
  a.err = err;
  a.herr = herr;
  a.timeout_ticks = timeout_ticks;
  a.nrep = 1;
  a.gram = gram;
  a.carry = carry ? 1 : 0;
  if (xa != nullptr && xa->nranks > 1) {
    if (tab == nullptr || xa->nranks > kMaxPeers || xa->half < px_half(xa->nranks, algo) ||
        xa->err == nullptr)
      return hipErrorInvalidValue;
    if (algo < 0 || algo > 4) return hipErrorInvalidValue;
    if (algo == 4 && (xsw == nullptr || ((uintptr_t)xsw & 15) != 0 ||
                      xsw_stride < (int64_t)d.nbatches * kKT * 1024 || (xsw_stride % 4) != 0))
      return hipErrorInvalidValue;
    a.xt = *tab;
    a.nrep = xa->nranks;
    a.rep = xa->rank;
    a.xhalf = xa->half;
    a.xerr = xa->err;
    a.algo = algo == 4 ? 0 : (algo & 1);
    a.pxslots = algo >= 2 ? kPxSlotsG : kPxSlots;
    a.dzr_off = px_slots_half(a.nrep, algo, kPxSlotsG);
    a.mirror = g_pk_probe_mode == 2 ? 1 : 0;
    a.probe = g_pk_probe_mode == 1 ? 1 : 0;
    if (a.mirror && (algo & 1) == 1 && algo != 4) return hipErrorInvalidValue;  // one-shot sums only
    if (algo == 4) {
      // the slot regions' parity halves are back to back ([2][slots_half], the
      // parity offset is slots_half, not the buffer's half), then the 3
      // rotating dZ1 slots: no slot region overlaps them
      a.dzr3 = 1;
      a.xhalf = px_slots_half(a.nrep, 0, kPxSlotsG);
      a.dzr_off = 2 * a.xhalf;
      a.xsw = xsw;
      a.xsw_stride = xsw_stride;
      // the dW1 sum over the replicas split with helper blocks on idle CUs
      // (pk_hlo): 3 from 4 replicas on, none below (HIPDSML_PKX_HELPERS overrides,
      // testing / tuning: 0, 1 or 3)
      if (g_pkx_helpers == -2) {
        const char* e = getenv("HIPDSML_PKX_HELPERS");
        g_pkx_helpers = e != nullptr && *e ? atoi(e) : -1;
      }
      int h = g_pkx_helpers >= 0 ? g_pkx_helpers : a.nrep >= 4 ? 3 : 0;
      if (h >= 3 && a.nrep >= 4) h = 3;        // every part gets >= 1 replica
      else if (h >= 1 && a.nrep >= 2) h = 1;
      else h = 0;
      a.helpers = h;
    }
    // the tagged one-shot tile sums (pkg, pkx): from 4 replicas on the slots
    // (2-3 per tile x N-1 peers) go out through pusher blocks, so a tile's
    // gather never queues behind its own pushes; with fewer peers the tile's
    // spare wave pushes them itself (a staging hop would cost more)
    a.pushers = ((algo == 2 || algo == 4) && a.nrep >= 4) ? 1 : 0;
    // pkx: the dZ1 rows leave from the layer-1 owner blocks (HIPDSML_PKX_L1PUSH
    // overrides: 0 the chains push them, 1 the owners)
    if (g_pkx_l1push == -2) {
      const char* e = getenv("HIPDSML_PKX_L1PUSH");
      g_pkx_l1push = e != nullptr && *e ? atoi(e) : -1;
    }
    a.l1push = algo == 4 ? (g_pkx_l1push >= 0 ? (g_pkx_l1push ? 1 : 0) : kPkxL1PushDefault) : 0;
    if (g_pkx_gsplit == -2) {
      const char* e = getenv("HIPDSML_PKX_GSPLIT");
      g_pkx_gsplit = e != nullptr && *e ? atoi(e) : -1;
    }
    a.gsplit = (algo == 4 && a.helpers > 0) ? (g_pkx_gsplit >= 0 ? (g_pkx_gsplit ? 1 : 0) : kPkxGsplitDefault) : 0;
    // Gram form: the previous launch's last Z1 carries over as in the single
    // replica (every replica launches the same sequence, so all agree)
    if (algo < 2) a.carry = 0;
  }
  const int mode = a.nrep == 1 ? 0 : (algo == 4 ? 3 : algo >= 2 ? 2 : 1);
  if (mode != 1 && (gram == nullptr || ((uintptr_t)gram & 15) != 0)) return hipErrorInvalidValue;
  if (d.nlayers == 3)
    return mode == 0 ? pk_launch<3, 0>(a, s) : mode == 1 ? pk_launch<3, 1>(a, s)
         : mode == 2 ? pk_launch<3, 2>(a, s) : pk_launch<3, 3>(a, s);
  return mode == 0 ? pk_launch<2, 0>(a, s) : mode == 1 ? pk_launch<2, 1>(a, s)
       : mode == 2 ? pk_launch<2, 2>(a, s) : pk_launch<2, 3>(a, s);
}

}  // namespace dsml
