// Host-side interface of the hipdsml native library (kernels + runtime).
//
// The kernels are plain HIP launchers over raw device pointers and a
// hipStream_t, so the device runtime (arena / copy engine / stream table /
// RCCL comm) and the PyTorch binding layer can both drive them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsml {

constexpr int kMaxLayers = 8;

// Descriptor of one data-parallel replica's MLP training state.
// Parameter layout (flat fp32 buffer, PyTorch Linear convention):
//   layer l (0-based): W_l [dims[l+1] x dims[l]] row-major at w_off[l],
//                      b_l [dims[l+1]]               at b_off[l].
// Every segment starts on a 16-float (64 B) boundary so float4 loads are legal.
// Workspace layout (flat fp32):
//   act_off[l]  l=1..L-1 : H_l  = relu(Z_l)   [batch x dims[l]]
//   dz_off[l]   l=1..L   : dZ_l = dLoss/dZ_l  [batch x dims[l]]
// The reference keeps W1 as [in x out] (client.go:118); conversion helpers in
// models/mlp.py map between the two layouts.
struct MlpDesc {
  int32_t nlayers;
  int32_t batch;     // rows handled per step by this replica
  int32_t nbatches;  // batches in the resident dataset (step counter wraps)
  int32_t w_in_lds;  // row chain stages W_l (l >= 2) in LDS (else reads them from HBM/L2)
  int32_t dims[kMaxLayers + 1];
  int32_t lds_act[kMaxLayers + 1];  // float offsets of the LDS activation tiles
  int32_t lds_dz[kMaxLayers + 1];   // float offsets of the LDS gradient tiles
  int32_t lds_stride[kMaxLayers + 1];
  int32_t lds_w[kMaxLayers + 1];    // LDS-staged W_l (l >= 2), row stride dims[l-1] + 4
  int32_t lds_b[kMaxLayers + 1];    // LDS-staged b_l (l >= 2)
  int32_t lds_floats;               // total LDS floats of the row-chain kernel
  int32_t pad1;
  int64_t w_off[kMaxLayers];
  int64_t b_off[kMaxLayers];
  int64_t act_off[kMaxLayers + 1];
  int64_t dz_off[kMaxLayers + 1];
  int64_t lab_off;  // ws offset (in 4-byte words) of the staged labels of the current batch
};

// ---- fused fp32 MLP step (kernels/mlp_f32.hip) -------------------------------
// Row tile of the row-chain kernel.
constexpr int kRowTile = 16;

struct MlpLaunchCfg {
  int kchunk;   // K elements per split of the first-layer GEMM (multiple of 16, <= 128)
  int nsplit;   // number of K splits (slabs)
};
MlpLaunchCfg mlp_plan_first_layer(const MlpDesc& d);
int mlp_wgrad_tiles(const MlpDesc& d);
bool mlp_rowchain_fits(const MlpDesc& d);

// Forward of layer 1 as a split-K MFMA GEMM into per-split slabs.
hipError_t mlp_f32_first_layer(const float* X, int64_t ldx, const float* P, float* slab,
                               int64_t* ctr, int64_t row0, const MlpDesc& d,
                               const MlpLaunchCfg& c, const int32_t* labels, float* ws,
                               hipStream_t s);
// Row-local chain: layer-1 epilogue, layers 2..L forward, softmax-xent,
// activation gradients down to dZ_1.  train=0 => forward + stats only;
// train=2 => forward + stats, logits written to ws + dz_off[L] ([batch x C]).
hipError_t mlp_f32_rowchain(const float* P, const float* slab, int nsplit, float* ws,
                            const int32_t* labels, int64_t* ctr, int64_t row0,
                            const MlpDesc& d, float* stats, int train, float inv_batch,
                            hipStream_t s);
// Shape-specialised row chain for 3-layer MLPs (mlp_f32_fast.hip); returns
// hipErrorNotSupported when no instantiation matches.
hipError_t mlp_f32_rowchain_fast(const float* P, const float* slab, int nsplit, float* ws,
                                 const int32_t* labels, int64_t* ctr, int64_t row0,
                                 const MlpDesc& d, float* stats, int train, float inv_batch,
                                 hipStream_t s);
// Weight/bias gradients of every layer; fused SGD (P -= lr*g) when fused_sgd,
// else gradients are written to G.
//
// Step counters (no atomics): ctr[0] = A, ctr[1] = B.  Step s starts with
// A = B = s.  K_A reads B, and its block 0 writes A = s + 1 and stages the
// batch's labels at ws + lab_off; K_B needs no counter; K_C reads A - 1 and its
// block 0 writes B = A.  No kernel writes a slot it also reads, so there is no
// intra-launch race and kernel boundaries order the rest.
hipError_t mlp_f32_wgrad(const float* X, int64_t ldx, float* P, float* G, const float* ws,
                         int64_t* ctr, int64_t row0, const MlpDesc& d, float lr, int fused_sgd,
                         hipStream_t s);

// ---- persistent fused step (kernels/mlp_persist.hip) -------------------------
// One launch runs `steps` SGD steps of the 784-128-64-10 or 784-128-10 MLP at
// batch <= 64 with the weights resident on chip (64 workgroups: 56 layer-1
// tiles, 4 row chains, 4 upper-layer gradient blocks; flag / tagged-granule
// hand-offs).  `xb` holds mlp_persist_xbuf_granules()
// uint64 granules, zeroed whenever the step counter is rewound; `err` is set
// when a hand-off timed out (the launch then ends early).
bool mlp_persist_supported(const MlpDesc& d);
hipError_t mlp_persist_read_stamps(uint64_t* host_out);  // [4][8][8] (role, step, phase)
void mlp_persist_set_stamping(bool on);
void mlp_persist_set_stamp_window(int first_step);  // stamp steps first..first+7 (< 0: off)
void mlp_persist_set_jitter(int ticks);  // testing only: uneven-load injection (0 = off)
int64_t mlp_persist_xbuf_granules();
// Gram tables of the persistent step's Gram form (kernels/gram.hip):
// T[b][r][m'][m] = Xs_r(b-1)[m'] . Xc(b)[m] + 1 over K features, fp64
// accumulation rounded to fp32; source r at Xs + r * src_stride floats, rows
// of ld_src / ldc floats (multiples of 4, 16-B aligned bases); batches of B
// <= 64 rows padded to 64 by repeating the last row; T [nb][nsrc][64][64].
hipError_t gram_table(const float* Xs, int64_t src_stride, int64_t ld_src, const float* Xc, int64_t ldc, int nb,
                      int B, int K, int nsrc, float* T, hipStream_t s);
hipError_t mlp_persist_steps(const float* X, int64_t ldx, const int32_t* labels, float* P,
                             int64_t* ctr, const MlpDesc& d, float lr, int steps, uint64_t* xb,
                             float* stats, uint32_t* err, uint32_t* herr, uint64_t timeout_ticks,
                             hipStream_t s, const struct XchgArgs* xa = nullptr,
                             const struct XchgTab* tab = nullptr, int algo = 0,
                             const float* gram = nullptr, int carry = 0,
                             const float* xsw = nullptr, int64_t xsw_stride = 0);
void mlp_persist_set_probe(int mode);  // testing only: 0 off, 1 lone-replica probe, 2 mirror
#ifdef HIPDSML_MEASURE
hipError_t mlp_persist_read_push_stamps(uint64_t* out);  // measurement builds: [8][4]
void mlp_persist_set_hop(int ticks);  // measurement builds: extra hop latency in mirror mode (100 MHz ticks)
#endif
// pkx dW1 helper blocks per layer-1 block: -1 the default (3 from 4 replicas on,
// else 0; HIPDSML_PKX_HELPERS overrides it), 0, 1 or 3 (tuning / testing)
void mlp_persist_set_pkx_helpers(int helpers);
// pkx: the dZ1 rows leave from the layer-1 owner blocks (1) or the chains (0); -1 the default
void mlp_persist_set_pkx_l1push(int mode);
// Single replica: the Gram table the persistent step reads, float[nbatches][64][64]
// with G1T[b][m'][m] = X_{b-1}[m'] . X_b[m] + 1 (rows past the batch repeat its
// last row; b - 1 wraps), and `carry` = 1 when the hand-off buffer still holds
// the state the previous launch left (nothing rewound or rewrote P since).
// Data-parallel form (xa->nranks > 1): the receive buffers / flags each replica
// needs (PeerExchange half >= px_half(n, algo), ntiles >= px_ntiles(n, algo));
// lr is passed as lr / n.  algo 0: one-shot sum (sync 'pk'), 1: two-shot
// reduce-scatter + all-gather per wave slot (sync 'pk2'); 2 / 3: the Gram form
// with the same sums (pkg / pkg2); 4: the Gram form with an exchange-free layer
// 1 (pkx): `xsw` = every replica's input shard in MFMA fragment order
// (float[n][nbatches][49][4][64][4], replica r at xsw + r * xsw_stride).
int64_t px_half(int n, int algo = 0);
int px_ntiles(int n, int algo = 0);

// ---- peer exchange: gradient all-reduce fused into K_C over xGMI -------------
// Every replica's K_C publishes each weight-gradient tile into its own
// exchange buffer (IPC-shared with the peers, uncached), raises a per-tile
// flag (= step + 1), waits for the same tile's flag of every peer, reads the
// peers' tiles over xGMI, sums all N in rank order (bit-identical replicas)
// and applies SGD with lr / N in place.  Buffers alternate by step parity, so
// a peer that is one step ahead never overwrites data still being read.
constexpr int kMaxPeers = 8;
struct XchgTab {                 // device-resident pointer table (as mapped in this process)
  float* buf[kMaxPeers];         // rank r's exchange buffer: [2][half] floats
  uint64_t* flags[kMaxPeers];    // rank r's per-tile flags
};
struct XchgArgs {
  const XchgTab* tab = nullptr;
  int32_t nranks = 1, rank = 0;
  int64_t half = 0;              // floats per parity half (>= nparams)
  uint32_t* err = nullptr;       // set to 1 when a peer did not arrive in time
  uint64_t timeout_ticks = 0;    // s_memrealtime ticks (100 MHz)
};
int mlp_wgrad_tiles(const MlpDesc& d);
// Standalone one-shot all-reduce (sum) of n fp32 (n % 4 == 0, n <= x.half)
// through the exchange buffers (kernels/xchg.hip).  `seq` >= 1 numbers the
// calls (monotonic per exchange; parity selects the buffer half).
int xchg_allreduce_blocks(int64_t n, int max_blocks, int* unroll);
hipError_t xchg_allreduce_f32(const float* in, float* out, int64_t n, const XchgArgs& x,
                              int max_blocks, uint64_t seq, hipStream_t s);
// Two-shot (reduce-scatter + all-gather) over the same buffers: 2n/N bytes per
// link.  Needs x.half >= n + ceil(n / N) and uses max_blocks / 2 flags per phase.
hipError_t xchg_allreduce2_f32(const float* in, float* out, int64_t n, const XchgArgs& x,
                               int max_blocks, uint64_t seq, hipStream_t s);
// Activation exchange (kernels/mlp_f32_xact.hip): K_C variant that pushes this
// replica's activations and activation gradients (H_l, dZ_l, in MFMA fragment
// order: mlp_xact_payload floats) to every rank and computes the global-batch
// weight gradients from all N images, SGD with lr / N.  Xswz holds every
// rank's input shard in fragment order (rank r at Xswz + r * xstride; see
// parallel/xchg.py swizzle_inputs).  Exchange buffers: half >= nranks *
// payload, ntiles = nranks * payload / 1024 (one flag per rank and strip).
// Needs batch <= 64 and every layer input dim a multiple of 16
// (mlp_xact_supported).
int mlp_xact_payload(const MlpDesc& d);
bool mlp_xact_supported(const MlpDesc& d);
// waves: 4 or 8 per tile block, 0 = 8 from 4 ranks on.
hipError_t mlp_f32_wgrad_xact(const float* Xswz, int64_t xstride, float* P, const float* ws,
                              int64_t* ctr, const MlpDesc& d, float lr_over_n, const XchgArgs& x,
                              const XchgTab& tab, int waves, hipStream_t s);
hipError_t mlp_f32_wgrad_xchg(const float* X, int64_t ldx, float* P, const float* ws, int64_t* ctr,
                              const MlpDesc& d, float lr_over_n, const XchgArgs& x,
                              const XchgTab& tab, hipStream_t s);

// ---- elementwise / reduction (kernels/elementwise.hip) -----------------------
enum DType : int32_t { kF32 = 0, kBF16 = 1, kF16 = 2, kU8 = 3, kI32 = 4 };
enum ReduceOp : int32_t { kSum = 0, kProd = 1, kMin = 2, kMax = 3 };

// In-kernel phase stamps (s_memrealtime, 100 MHz) of block 0, for profiling.
constexpr int kMaxStamps = 32;
hipError_t mlp_read_stamps(uint64_t* host_out);  // kMaxStamps entries
void mlp_set_stamping(bool on);
hipError_t mlp_read_stamps_fast(uint64_t* host_out);
void mlp_set_stamping_fast(bool on);
hipError_t mlp_read_stamps_xact(uint64_t* host_out);
void mlp_set_stamping_xact(bool on);

hipError_t sgd_update_f32(float* P, const float* G, int64_t n, float scale, hipStream_t s);
hipError_t sgd_momentum_f32(float* P, const float* G, float* V, int64_t n, float lr,
                            float momentum, float weight_decay, float gscale, hipStream_t s);
// dst = op(dst, src) elementwise; n in elements.
hipError_t reduce_inplace(void* dst, const void* src, int64_t n, int32_t dtype, int32_t op,
                          hipStream_t s);
// Up to kMaxReduceSegs in-place reductions dst_k = op(dst_k, src_k) in ONE
// launch (the in-house ring reduces every directed ring's segment of a step).
constexpr int kMaxReduceSegs = 8;
struct ReduceSeg {
  void* dst;
  const void* src;
  int64_t n;  // elements
};
struct ReduceSegs {
  ReduceSeg seg[kMaxReduceSegs];
  int32_t count;
};
hipError_t reduce_multi_inplace(const ReduceSegs& m, int32_t dtype, int32_t op, hipStream_t s);
// dst = op(a, b)
hipError_t reduce_into(void* dst, const void* a, const void* b, int64_t n, int32_t dtype,
                       int32_t op, hipStream_t s);
hipError_t scale_inplace(void* x, int64_t n, int32_t dtype, float alpha, hipStream_t s);
hipError_t u8_to_f32_scaled(float* dst, const uint8_t* src, int64_t n, float scale,
                            hipStream_t s);
hipError_t f32_to_bf16(uint16_t* dst, const float* src, int64_t n, hipStream_t s);
hipError_t bf16_to_f32(float* dst, const uint16_t* src, int64_t n, hipStream_t s);

// ---- bf16 MFMA GEMM with fused epilogues (kernels/gemm_bf16.hip) -------------
// Cp[s][M][N] (fp32 split-K slabs) = A[M x K] . B[N x K]^T, bf16 operands with
// K-contiguous rows (lda, ldb, K multiples of 8; 16 B aligned base pointers).
struct GemmEpi {
  float alpha;
  const float* bias;
  int relu;
  const uint16_t* mask;
  int64_t ldm;
  float* of32;
  int64_t ldo;
  uint16_t* obf;
  int64_t ldb;
  uint16_t* obfT;
  int64_t ldt;
  float* sgdW;  // fused SGD target (fp32 [M x N], ld ldw): W -= lr * acc
  int64_t ldw;
  float lr;
  float* bgrad;  // single split only: row sums of A over K (bias gradient of a dW GEMM)
  float* bsgd;   // single split only: bias SGD with those row sums (b -= lr * rowsum)
};
// epi == nullptr: fp32 partial slabs Cp[split] (finish with gemm_epilogue).
// epi != nullptr: epilogue applied in-kernel; with > 1 K split the last split
// of each tile reduces the slabs (Cp) and applies it — `tile_ctr` must hold one
// zero int per 64x64 output tile (the kernel leaves them zero again).
hipError_t gemm_bf16_nt(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, float* Cp,
                        int M, int N, int K, int splits, hipStream_t s,
                        const GemmEpi* epi = nullptr, int* tile_ctr = nullptr);
int gemm_bf16_num_splits(int K, int splits);
// Batch-row GEMM (C = A . B^T with <= 64 rows per block, 16 columns per block,
// full K per block split across its 4 waves) with the whole epilogue fused
// (alpha, bias, ReLU, ReLU'-mask, fp32 / bf16 / transposed bf16 outputs).
// a_blk: A stored k-blocked, element (m, k) at A[(k / 32) * lda + 32 m + k % 32]
// (one 16-row fragment load = 1 KiB contiguous instead of 16 half lines).
hipError_t gemm_bf16_rows64(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int M,
                            int N, int K, const GemmEpi& epi, hipStream_t s, bool a_blk = false);
// out = epi(alpha * sum_s Cp[s] + bias): relu, ReLU'-mask (bf16 mask > 0), fp32 / bf16 /
// transposed-bf16 outputs (each nullable).
hipError_t gemm_epilogue(const float* Cp, int S, int M, int N, float alpha, const float* bias,
                         int relu, const uint16_t* mask, int64_t ldm, float* of32, int64_t ldo,
                         uint16_t* obf, int64_t ldb, uint16_t* obfT, int64_t ldt, hipStream_t s);
hipError_t cast_transpose(const float* X, int64_t ldi, int M, int K, int Kp, uint16_t* Y,
                          int64_t ldo, uint16_t* YT, int64_t ldt, hipStream_t s);
hipError_t softmax_xent(const float* logits, int64_t ldl, const int32_t* labels, int B, int C,
                        int Cp, float inv_batch, uint16_t* dz, int64_t ldz, uint16_t* dzT,
                        int64_t ldt, float* stats, hipStream_t s);
// The head's H from a raw split-K skinny GEMM (gemm_skinny raw_slabs): H[m][k]
// = bf16(relu(alpha * sum_{z < S} slabs[z][k / 64][m][k % 64] + bias[k])),
// slices summed in slice order -- bit-identical to the skinny GEMM's own
// combine + epilogue -- and written to Hout (the weight update reads it).
struct HeadSlabs {
  const float* slabs;
  int S;              // 2, 4 or 8 slices
  int64_t stride;     // floats per slice (tiles * 4096)
  float alpha;
  const float* bias;  // [K] (nullable)
  int relu;
  uint16_t* Hout;     // [B][ldo] bf16
  int64_t ldo;
};
// Classifier head fused with softmax-CE (C <= 16, K <= 4096): logits = H . W^T
// (row_stats: loss / correct / count accumulate in stats[4m ..] per row m,
// summed by the reader, instead of atomics on stats[0..2])
// + b per row, then the softmax_xent outputs.  `logits` may be null.  With
// `dzp`, also the next backward product: dzp = (dz . W) * (H > 0) in bf16
// (+ the transposed copy dzpT), from operands the kernel already holds.
hipError_t head_softmax_xent(const uint16_t* H, int64_t ldh, const uint16_t* W, int64_t ldw,
                             const float* bias, int B, int K, int C, const int32_t* labels,
                             float inv_batch, float* logits, int64_t ldl, uint16_t* dz, int64_t ldz,
                             uint16_t* dzT, int64_t ldt, int Cp, float* stats, hipStream_t s,
                             uint16_t* dzp = nullptr, int64_t ldzp = 0, uint16_t* dzpT = nullptr,
                             int64_t ldpt = 0, int row_stats = 0, const HeadSlabs* hs = nullptr);
// Skinny GEMMs (kernels/gemm_skinny.hip): C[M x N] = A[M x K] . B^T for
// B [N x K] (nn = false) or A . B for B [K x N] (nn = true: W read in its
// stored layout through transposing LDS reads), 64 x 64 tiles, K split S ways
// (splits <= 0: auto, >= 256 workgroups) with the last-arriving slice reducing
// and applying `epi` (no sgdW / bgrad / bsgd).  slabs: S * tiles * 4096 fp32,
// tile_ctr: one zeroed int per 64 x 64 tile (left zero).  K, N multiples of 8.
int gemm_skinny_splits(int M, int N, int K, int splits);
// split-K workspace of one launch: fp32 words of `slabs`, int32 words of `tile_ctr`
// (zeroed once; every launch leaves its tickets at 0)
void gemm_skinny_ws(int M, int N, int K, int splits, int64_t* ws_words, int64_t* ctr_words);
hipError_t gemm_skinny_read_stamps(uint64_t* host_out);  // [1024][5], profiling only
void gemm_skinny_set_stamping(bool on);
// raw_slabs: every slice stores its fp32 partial tile into slabs[slice][tile]
// ([64 rows][64 cols] each, tile = m block * N tiles + n block) and the launch
// applies no epilogue: the consumer sums the slices (head_softmax_xent's Hs).
hipError_t gemm_skinny(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int M, int N,
                       int K, bool nn, int splits, float* slabs, int* tile_ctr, const GemmEpi& epi,
                       hipStream_t s, bool raw_slabs = false);
// Weight gradient from row-major activations (kernels/wgrad_sgd.hip):
// G = alpha * Z^T X (Z [M x N], X [M x K] bf16, rows padded to 8 columns), then
// W -= lr * G (+ bf16 copy Wb) when W is given, else G written out; bias -= lr
// * alpha * colsum(Z) and/or bgrad = alpha * colsum(Z).  K % 4 == 0.
hipError_t wgrad_sgd(const uint16_t* Z, int64_t ldz, const uint16_t* X, int64_t ldx, int M, int N,
                     int K, float alpha, float lr, float* W, int64_t ldw, uint16_t* Wb, int64_t ldwb,
                     float* G, int64_t ldg, float* bias, float* bgrad, hipStream_t s);
struct WgLayer {
  const uint16_t* Z;  // [M x >= N] bf16, ldz
  int64_t ldz;
  const uint16_t* X;  // [M x >= K] bf16, ldx
  int64_t ldx;
  int M, N, K;
  float alpha, lr;
  float* W;  // [N x K] fp32, ldw (SGD target), or null with G
  int64_t ldw;
  uint16_t* Wb;  // bf16 copy of the updated W (nullable), ldwb
  int64_t ldwb;
  float* G;  // alpha * gradient out (nullable), ldg
  int64_t ldg;
  float* bias;   // b -= lr * alpha * colsum(Z) (nullable)
  float* bgrad;  // alpha * colsum(Z) out (nullable)
  // split fp32 master instead of W (W == nullptr): bits = (hi << 16) + lo.
  // Wh: this step's hi words (= its bf16 GEMM copy), ldwh; Wl: the int16
  // remainders, updated in place, ldwl; the updated hi words go to Wb.
  const uint16_t* Wh;
  int64_t ldwh;
  uint16_t* Wl;
  int64_t ldwl;
};
// fp32 <-> split master (hi: bf16 rounded half away from zero, lo: int16 remainder)
hipError_t hilo_split(const float* W, int N, int K, int64_t ldw, uint16_t* hi, int64_t ldh, uint16_t* lo,
                      int64_t ldl, hipStream_t s);
hipError_t hilo_join(const uint16_t* hi, int64_t ldh, const uint16_t* lo, int64_t ldl, int N, int K, float* W,
                     int64_t ldw, hipStream_t s);
// split master SGD step: w = join(hic, lo) - lr * G (G nullable: a re-split);
// hin <- hi(w) (the next step's bf16 copy), lo <- lo(w) in place
hipError_t hilo_sgd(const uint16_t* hic, int64_t ldc, uint16_t* lo, int64_t ldl, const float* G, int64_t ldg,
                    int N, int K, float lr, uint16_t* hin, int64_t ldn, hipStream_t s);
// Up to 4 layers' wgrad_sgd in one launch (one flattened tile grid).  tile 128:
// 128 x 128 tiles for every layer with N, K >= 128, 64 x 64 for the rest; 64:
// 64 x 64 everywhere; 0 (auto): 128 for fp32-master layers at M >= 512 rows,
// else 64.
// tile: 0 auto, 64 / 128 square tiles, kWgRowBlkTile the row-block form (split
// master, one M of 64 / 128 / 256 / 512 for every layer; auto picks it from M >= 256)
constexpr int kWgRowBlkTile = 256;
hipError_t wgrad_sgd_multi(const WgLayer* layers, int n, hipStream_t s, int tile = 0);
// The wide step's input layer in one launch (kernels/wide_input.hip): dZ_1 from
// the last dgrad's raw split-K slices (+ ReLU' mask), the W_0 / b_0 SGD step on
// the split master, and the NEXT step's H_1 = relu(X' W_0'^T + b_0').  M = 64.
struct WideInArgs {
  const float* slabs;  // raw slices: slabs[(z * tiles + n / 64) * 4096 + m * 64 + n % 64]
  int S, tiles;
  float zalpha, zbias;   // the dgrad epilogue (alpha, + 0)
  const uint16_t* H1;    // this step's H_1 (the mask), ldh1
  int64_t ldh1;
  uint16_t* dzo;         // dZ_1 out (nullable), lddz
  int64_t lddz;
  const uint16_t* XG;    // this step's 64 input rows in gradient-fragment order [K/16][2][16][32]
  const uint16_t* XF;    // the next step's 64 input rows k-blocked [K/32][64][32]
  const uint16_t* Wh;    // this step's hi words, ldwh
  int64_t ldwh;
  uint16_t* Wl;          // int16 remainders (in place), ldwl
  int64_t ldwl;
  uint16_t* Wb;          // the updated hi words, ldwb
  int64_t ldwb;
  float* bias;           // b_0 (updated in place)
  float alpha, lr, falpha;
  uint16_t* Hn;          // the next step's H_1, ldhn
  int64_t ldhn;
  int M, N, K, kq;       // kq: columns per wave, gemm_rows64_k's split ((ceil(K/8) + 31) / 32 * 32)
};
hipError_t wide_input_step(const WideInArgs& a, hipStream_t s);
hipError_t wide_input_check(const WideInArgs& a);  // the shapes / alignment both forms assume
// The same input-layer work as 16-row strip workgroups at the FRONT of the
// update launch of the layers above (kernels/wgrad_sgd.hip wgrad_multi_in_k):
// the strips' HBM phases overlap the 64 x 64 tiles' weight stream.  layers:
// every layer but the input one, batch 64 (square tiles); bit-identical.
hipError_t wgrad_sgd_multi_in(const WgLayer* layers, int n, const WideInArgs& in, hipStream_t s);
#ifdef HIPDSML_MEASURE
hipError_t wide_input_read_stamps(uint64_t* host_out);  // [1024][8], measurement builds
void wide_input_set_stamping(bool on);
void wide_input_set_dbg(int bits);
hipError_t wgrad_rowblk_read_stamps(uint64_t* host_out);  // [256][16], measurement builds
void wgrad_rowblk_set_stamping(bool on);
#endif
// Row-block form (global-batch update): cost-balanced workgroup runs over the
// units of layers (N[j], K[j]) in launch order; starts[0 .. runs], returns runs
// (<= groups).  Host only.
int wgrad_rowblk_plan(const int* N, const int* K, int n, int groups, int* starts);
hipError_t head_read_stamps(uint64_t* host_out);  // [64][6], profiling only
void head_set_stamping(bool on);
#ifdef HIPDSML_MEASURE
void head_set_debug(int v);
#endif
hipError_t rowsum_bf16(const uint16_t* X, int64_t ld, int N, int cols, float* out, float* bias,
                       float lr, hipStream_t s);
hipError_t sgd_cast(float* W, const float* G, int N, int K, float lr, uint16_t* Wb, int64_t ldw,
                    uint16_t* WbT, int64_t ldt, hipStream_t s);

}  // namespace dsml
