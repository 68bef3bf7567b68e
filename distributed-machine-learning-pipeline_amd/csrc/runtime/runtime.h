// hipdsml native device runtime: the MI355X-native replacement of the
// reference's simulated GPU device (DSML/gpu_device_service/gpu_device_server.go).
//
//   DeviceArena  : linear HBM arena behind the reference's MemAddr space
//                  [0x1000, 0x1000+size)  (replaces map[uint64][]byte, :31,:204)
//   CopyEngine   : pinned host staging + hipMemcpyAsync on side streams
//                  (replaces Memcpy H2D/D2H blob copies, :195-230)
//   StreamTable  : BeginSend / BeginReceive / StreamSend / GetStreamStatus state
//                  machine with hipEvent completion (replaces :14-24,64-193)
//   RcclComm     : RCCL communicator + ring all-reduce over ncclSend/ncclRecv,
//                  ncclAllReduce reference path, abort / async-error (replaces the
//                  coordinator's gRPC "ring", gpu_coordinator_server.go:272-566)
//   MlpRunner    : one DP replica's fused train step, hipGraph-captured.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../dsml.h"
#include "ring_plan.h"

namespace dsml {

std::string hip_error_string(hipError_t e);
#define DSML_HIP_CHECK(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      throw std::runtime_error(std::string("HIP error at " __FILE__ ":") +            \
                               std::to_string(__LINE__) + " " #expr ": " +            \
                               ::dsml::hip_error_string(_e));                          \
  } while (0)

// ---------------------------------------------------------------------------
class DeviceArena {
 public:
  static constexpr uint64_t kBaseAddr = 0x1000;  // reference minMemAddr
  DeviceArena(int device, uint64_t size_bytes, uint64_t base_addr = kBaseAddr);
  ~DeviceArena();
  DeviceArena(const DeviceArena&) = delete;
  DeviceArena& operator=(const DeviceArena&) = delete;

  int device() const { return device_; }
  uint64_t min_addr() const { return base_; }
  uint64_t max_addr() const { return base_ + size_; }
  uint64_t size() const { return size_; }
  void* base_ptr() const { return ptr_; }
  // Bounds-checked MemAddr -> device pointer (throws std::out_of_range).
  void* translate(uint64_t addr, uint64_t nbytes) const;
  bool contains(uint64_t addr, uint64_t nbytes) const;
  // Extent bookkeeping for reference-compatible D2H with numBytes == 0
  // ("return the whole blob", gpu_device_server.go:217-226).
  void record_extent(uint64_t addr, uint64_t nbytes);
  uint64_t extent(uint64_t addr) const;

 private:
  int device_;
  uint64_t base_, size_;
  void* ptr_ = nullptr;
  mutable std::mutex mu_;
  std::map<uint64_t, uint64_t> extents_;
};

// ---------------------------------------------------------------------------
class CopyEngine {
 public:
  // staging_bytes is split into 2 ping-pong pinned buffers per direction.
  CopyEngine(int device, size_t staging_bytes = 16u << 20);
  ~CopyEngine();
  CopyEngine(const CopyEngine&) = delete;
  CopyEngine& operator=(const CopyEngine&) = delete;

  // Host (pageable) -> device: chunks are memcpy'd into pinned staging and
  // DMA'd with hipMemcpyAsync on the H2D side stream; the host memcpy of chunk
  // c+1 overlaps the DMA of chunk c.  Returns after the data is in HBM.
  void h2d(void* dst_dev, const void* src_host, size_t n);
  // Device -> host (pageable), same double-buffered pipeline in reverse.
  void d2h(void* dst_host, const void* src_dev, size_t n);
  // Device -> device on the D2D side stream.
  void d2d(void* dst_dev, const void* src_dev, size_t n);
  hipStream_t h2d_stream() const { return s_h2d_; }
  hipStream_t d2h_stream() const { return s_d2h_; }
  uint64_t bytes_h2d() const { return bytes_h2d_; }
  uint64_t bytes_d2h() const { return bytes_d2h_; }

 private:
  int device_;
  size_t half_;
  void* pin_up_[2] = {nullptr, nullptr};
  void* pin_dn_[2] = {nullptr, nullptr};
  hipEvent_t ev_up_[2], ev_dn_[2];
  hipStream_t s_h2d_, s_d2h_, s_d2d_;
  std::mutex mu_up_, mu_dn_, mu_dd_;
  uint64_t bytes_h2d_ = 0, bytes_d2h_ = 0;
};

// ---------------------------------------------------------------------------
enum class XferStatus : int { kInProgress = 0, kSuccess = 1, kFailed = 2 };

struct StreamState {
  uint64_t send_addr = 0, recv_addr = 0, num_bytes = 0;
  uint32_t src_rank = 0, dst_rank = 0;
  bool initiated_send = false, initiated_recv = false;
  XferStatus status = XferStatus::kInProgress;
  uint64_t received = 0;
  hipEvent_t done = nullptr;  // recorded after the last chunk's H2D
};

class StreamTable {
 public:
  StreamTable(DeviceArena* arena, CopyEngine* ce);
  ~StreamTable();
  // BeginSend: allocate a stream id (>= 1) recording the request (:64-88).
  uint64_t begin_send(uint64_t send_addr, uint64_t num_bytes, uint32_t dst_rank);
  // BeginReceive: bind the receive buffer (:90-110).  Throws std::out_of_range
  // for an OOB address and std::invalid_argument for an unknown stream id.
  void begin_receive(uint64_t stream_id, uint64_t recv_addr, uint64_t num_bytes,
                     uint32_t src_rank);
  // One StreamSend chunk: written at recv_addr + received.  Returns false if
  // the stream is unknown / not bound / overflowing (stream marked FAILED).
  bool push_chunk(uint64_t stream_id, const void* data, uint64_t n);
  // End of the client stream: SUCCESS iff received == num_bytes (:150-181).
  bool finish(uint64_t stream_id);
  XferStatus status(uint64_t stream_id);  // unknown id -> FAILED (:183-193)
  // Read the send buffer of a stream (device -> host) for forwarding.
  std::vector<uint8_t> read_send_buffer(uint64_t stream_id);
  void erase(uint64_t stream_id);
  size_t size() const;

 private:
  DeviceArena* arena_;
  CopyEngine* ce_;
  mutable std::mutex mu_;
  uint64_t next_id_ = 1;
  std::map<uint64_t, StreamState> streams_;
};

// ---------------------------------------------------------------------------
std::vector<uint8_t> rccl_unique_id();

class RcclComm {
 public:
  RcclComm(const std::vector<uint8_t>& uid, int rank, int nranks, int device, bool blocking);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  // RCCL's own all-reduce (multi-channel ring / LL protocols).
  void allreduce(void* buf, int64_t count, int32_t dtype, int32_t op, hipStream_t s);
  // In-house multi-ring all-reduce (ring_plan.h): one slice per directed
  // Hamiltonian ring (up to 6 at n = 8, each on its own xGMI links),
  // reduce-scatter + all-gather, every ring's ncclSend/ncclRecv of a step in
  // one ncclGroup, segment reductions by dsml::reduce_inplace, `chunk_bytes`
  // rounds.  max_rings = 0: all rings; 1: the classic single ring.
  // pipe: 1 the pipelined schedule (ring_plan.h ring_pipeline), 0 the
  // single-stream one, -1 this communicator's default (set_ring_pipeline;
  // until set, HIPDSML_RING_PIPELINE=1 selects the pipelined one).
  void ring_allreduce(void* buf, int64_t count, int32_t dtype, int32_t op, int64_t chunk_bytes,
                      hipStream_t s, int max_rings = 0, int pipe = -1);
  // The default schedule of ring_allreduce (parallel/ring_tune.py measures both
  // and keeps the faster): -1 env, 0 single-stream, 1 pipelined.
  void set_ring_pipeline(int mode) { pipe_default_ = mode; }
  int pipeline_mode() const;
  // Size the ring's reduce scratch for `count` elements once, up front (the
  // largest bucket): no hipMalloc / hipFree between buckets, and none inside a
  // stream capture (ring_allreduce refuses to grow it while capturing).
  void reserve_ring(int64_t count, int32_t dtype, int64_t chunk_bytes, int max_rings = 0);
  void broadcast(void* buf, int64_t count, int32_t dtype, int root, hipStream_t s);
  // in-place all-gather: rank r's `count` elements sit at buf + r * count
  void allgather(void* buf, int64_t count, int32_t dtype, hipStream_t s);
  void send(const void* buf, int64_t count, int32_t dtype, int peer, hipStream_t s);
  void recv(void* buf, int64_t count, int32_t dtype, int peer, hipStream_t s);
  void barrier(hipStream_t s);
  // Fault handling: abort in-flight collectives so no rank hangs.
  void abort();
  std::string async_error();
  bool aborted() const { return aborted_; }

 private:
  void check(ncclResult_t r, const char* what);
  void ensure_tmp(size_t bytes);
  size_t ring_tmp_bytes(int64_t count, int32_t dtype, int64_t chunk_bytes, int max_rings) const;
  ncclComm_t comm_ = nullptr;
  int rank_, nranks_, device_;
  bool blocking_;
  bool aborted_ = false;
  int pipe_default_ = -1;
  void* tmp_ = nullptr;
  size_t tmp_bytes_ = 0;
  void* one_ = nullptr;  // scratch for barrier
  // Pipelined ring (ring_plan.h ring_pipeline): the reduce-scatter's reduces run
  // on their own stream, ordered by events, so chunk c's reduce overlaps chunk
  // c+1's transfer; scratch is double buffered per ring.
  void ensure_pipe(size_t groups);
  hipStream_t red_ = nullptr;
  hipEvent_t fork_ = nullptr, join_ = nullptr;
  std::vector<hipEvent_t> ev_xfer_, ev_red_;
};

// ---------------------------------------------------------------------------
// Peer exchange buffers for the xGMI-fused gradient all-reduce (dsml.h
// XchgArgs).  One per replica: [2 x half floats][ntiles flags] in uncached HBM,
// exported by IPC handle; peers' buffers are opened from their handles (or, for
// replicas living in one process, referenced directly).
class PeerExchange {
 public:
  PeerExchange(int device, int64_t half_floats, int ntiles);
  ~PeerExchange();
  PeerExchange(const PeerExchange&) = delete;
  PeerExchange& operator=(const PeerExchange&) = delete;

  std::vector<uint8_t> ipc_handle() const;
  // handles[r] = rank r's ipc_handle() (own entry ignored).
  void connect_ipc(int rank, const std::vector<std::vector<uint8_t>>& handles);
  // Replicas of one process (same or peer-accessible devices).
  void connect_local(int rank, const std::vector<PeerExchange*>& peers);
  // Zero own flags and the error word (stream-ordered).  Collective in effect:
  // every rank resets, then all ranks barrier before the next exchange.
  void reset(hipStream_t s);
  uint32_t error(hipStream_t s);
  void set_timeout_ms(double ms);
  // One-shot all-reduce (sum) of n fp32 through the exchange (not graph-safe:
  // the call number is a kernel argument).  out may alias in.
  // algo 0: one-shot (every rank reads every peer's whole buffer); 1: two-shot
  // (reduce-scatter + all-gather, 2n/N bytes per link).
  void allreduce(const float* in, float* out, int64_t n, hipStream_t s, int algo = 0);
  bool connected() const { return args_.tab != nullptr; }
  const XchgArgs& args() const { return args_; }
  // Host copy of the pointer table (kernels that take it by value, as kernel
  // arguments, skip the dependent load of the device-resident copy).
  const XchgTab& table() const { return tab_host_; }
  int nranks() const { return args_.nranks; }
  int rank() const { return args_.rank; }
  int ntiles() const { return ntiles_; }
  int64_t half() const { return half_; }
  const char* memory_kind() const { return kind_; }
  float* buf() const { return static_cast<float*>(base_); }
  uint64_t* flags() const { return reinterpret_cast<uint64_t*>(static_cast<char*>(base_) + flag_off_); }

 private:
  void publish_table(const XchgTab& t, int rank, int n);
  int device_;
  int64_t half_;
  int ntiles_;
  size_t flag_off_ = 0, bytes_ = 0;
  void* base_ = nullptr;
  const char* kind_ = "";
  std::vector<void*> opened_;
  XchgTab* dtab_ = nullptr;
  uint32_t* err_ = nullptr;
  XchgArgs args_;
  XchgTab tab_host_{};
  uint64_t seq_ = 0;
};

// ---------------------------------------------------------------------------
// One data-parallel replica's training step.  Buffers are owned by the caller
// (PyTorch tensors); the runner only records pointers and launch plans.
struct MlpBuffers {
  const float* X = nullptr;  // [nsamples x ldx]
  int64_t ldx = 0;
  const int32_t* labels = nullptr;
  float* P = nullptr;     // params (flat)
  float* G = nullptr;     // grads  (flat)
  float* V = nullptr;     // momentum (flat, optional)
  float* ws = nullptr;    // activations / activation-grads
  float* slab = nullptr;  // split-K partials of layer 1
  int64_t* ctr = nullptr; // [step, ticket]
  float* stats = nullptr; // [loss_sum, correct, count]
  int64_t nparams = 0;    // floats in P / G (incl. alignment padding)
};

class MlpRunner {
 public:
  MlpRunner(const MlpDesc& d, const MlpBuffers& b, float lr, float momentum, float weight_decay);
  ~MlpRunner();
  void set_comm(RcclComm* c, int algo /*0 = rccl allreduce, 1 = in-house ring*/,
                int64_t chunk_bytes);
  // Gradient all-reduce fused into the weight-gradient kernel over xGMI
  // (plain SGD only).  Takes precedence over the RCCL communicator.
  void set_exchange(PeerExchange* x);
  // Activation exchange (kernels/mlp_f32_xact.hip): K_C pushes this replica's
  // activations to every rank and computes the global-batch weight gradients;
  // Xall holds every rank's input shard in MFMA fragment order (rank r at
  // Xall + r * xstride).  Replaces set_exchange's mode while set.
  void set_act_exchange(PeerExchange* x, const float* Xall, int64_t xstride, int waves = 0);
  // Persistent fused step (kernels/mlp_persist.hip): every enqueue of n steps
  // is ONE launch.  Single replica, plain SGD, the flagship shape only.
  // With `x` (>= 2 ranks): the data-parallel persistent step, every weight
  // gradient summed over the replicas inside the launch through x's buffers.
  void set_persist(uint64_t* xbuf, uint32_t* err, double timeout_ms, PeerExchange* x = nullptr,
                   int algo = 0);
  bool persist_active() const { return pk_xb_ != nullptr; }
  // Single replica: the Gram table of the batches (float[nbatches][64][64],
  // kernels/mlp_persist.hip), set once; and whether the hand-off buffer carries
  // the previous launch's pipeline state -- set by every single-replica
  // launch, cleared by set_persist / clear_persist_error and by the owner
  // whenever it rewrites the parameters or the buffer.
  // `numel` floats: enqueue_steps checks it against nbatches * 4096 (times the
  // replica count in the data-parallel Gram forms, which read [b][N][64][64]).
  void set_persist_gram(const float* g, int64_t numel) {
    pk_gram_ = g;
    pk_gram_numel_ = numel;
    pk_carry_ = false;
  }
  void set_persist_carry(bool c) { pk_carry_ = c; }
  // Exchange-free data-parallel form (algo 4): every replica's input shard in
  // MFMA fragment order, replica r at xsw + r * stride floats (numel checked
  // against the replica count at enqueue).
  void set_persist_xall(const float* xsw, int64_t stride, int64_t numel) {
    pk_xsw_ = xsw;
    pk_xsw_stride_ = stride;
    pk_xsw_numel_ = numel;
  }
  bool persist_carry() const { return pk_carry_; }
  // Whether a persistent launch gave up on a hand-off (read from host-mapped
  // memory the kernel marks on the way out: valid after a stream sync, no copy).
  bool persist_failed() const;
  void clear_persist_error();
  // Enqueue n full steps (one launch in persistent mode).
  void enqueue_steps(int n, hipStream_t s);
  bool exchange_active() const { return xchg_ != nullptr; }
  int exchange_mode() const { return xchg_ == nullptr ? 0 : (xact_ ? 2 : 1); }
  // Enqueue one full step on stream s (no host sync).
  void enqueue_step(hipStream_t s);
  // Enqueue only fwd/bwd (grads -> G, no update) — used by the DP engine when
  // the gradient all-reduce is driven from Python.
  void enqueue_fwd_bwd(hipStream_t s);
  void enqueue_update(hipStream_t s);
  // Capture `steps` steps into a hipGraph on stream s (the RCCL collective of a
  // multi-rank step included: it is recorded as graph nodes like any kernel).
  // Graphs are kept per step count, so a run of n = q * G + r steps replays a
  // G-step and an r-step graph instead of falling back to eager launches.
  void capture(int steps, bool capture_comm, hipStream_t s);
  // Replay the graph of `steps` steps (0: the most recently captured one).
  void replay(hipStream_t s, int steps = 0);
  bool captured(int steps = 0) const;
  int graph_steps() const { return graph_steps_; }
  void reset_graph();
  const MlpDesc& desc() const { return d_; }
  MlpLaunchCfg cfg() const { return cfg_; }
  void set_lr(float lr);
  // Replicas averaging gradients outside the runner (torch.distributed path);
  // the update then applies lr / world.  Defaults to the comm's size.
  void set_world_size(int n);

 private:
  MlpDesc d_;
  MlpBuffers b_;
  MlpLaunchCfg cfg_;
  float lr_, mom_, wd_;
  RcclComm* comm_ = nullptr;
  PeerExchange* xchg_ = nullptr;
  bool xact_ = false;
  const float* xall_ = nullptr;
  int64_t xstride_ = 0;
  int xact_waves_ = 0;
  uint64_t* pk_xb_ = nullptr;
  PeerExchange* pk_x_ = nullptr;  // replica exchange of the persistent step (nranks > 1)
  int pk_algo_ = 0;               // its sum: 0 one-shot, 1 two-shot
  uint32_t* pk_err_ = nullptr;
  uint32_t* pk_herr_ = nullptr;  // hipHostMalloc'd, device-visible
  uint64_t pk_timeout_ = 0;
  const float* pk_gram_ = nullptr;
  int64_t pk_gram_numel_ = 0;
  const float* pk_xsw_ = nullptr;
  int64_t pk_xsw_stride_ = 0, pk_xsw_numel_ = 0;
  bool pk_carry_ = false;
  int algo_ = 0;
  int world_ = 1;
  int64_t chunk_bytes_ = 1 << 20;
  struct Captured {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
  };
  std::map<int, Captured> graphs_;  // by step count
  int graph_steps_ = 0;             // step count of the last capture
  bool capture_comm_ = true;
};

// Forward-only evaluation over `rows` resident rows (one launch pair).
// logits != 0: also writes the logits to ws + dz_off[L] (ws sized for d).
void mlp_eval(const MlpDesc& d, const float* X, int64_t ldx, const int32_t* labels,
              int64_t row0, const float* P, float* ws, float* slab, float* stats, hipStream_t s,
              bool logits = false);

}  // namespace dsml
