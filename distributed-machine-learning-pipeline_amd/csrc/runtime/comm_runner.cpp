// RCCL communicator (ring all-reduce over ncclSend/ncclRecv, RCCL all-reduce
// reference path, abort / async error) and the hipGraph-captured MLP replica
// step.
//
// Reference behaviour being replaced: the coordinator-driven "ring"
// (gpu_coordinator_server.go:272-566) that moved bytes over gRPC to each rank's
// OWN device and reduced them as uint8.  Here each device
// process owns one GPU and a real ring moves segments GPU->GPU over xGMI.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "runtime.h"

namespace dsml {

static ncclDataType_t to_nccl(int32_t dt) {
  switch (dt) {
    case kF32: return ncclFloat32;
    case kBF16: return ncclBfloat16;
    case kF16: return ncclFloat16;
    case kU8: return ncclUint8;
    case kI32: return ncclInt32;
    default: throw std::invalid_argument("unsupported dtype " + std::to_string(dt));
  }
}
static size_t dtype_size(int32_t dt) {
  switch (dt) {
    case kF32: case kI32: return 4;
    case kBF16: case kF16: return 2;
    case kU8: return 1;
    default: throw std::invalid_argument("unsupported dtype " + std::to_string(dt));
  }
}
static ncclRedOp_t to_nccl_op(int32_t op) {
  switch (op) {
    case kSum: return ncclSum;
    case kProd: return ncclProd;
    case kMin: return ncclMin;
    case kMax: return ncclMax;
    default: throw std::invalid_argument("unsupported reduce op " + std::to_string(op));
  }
}

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  return std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id),
                              reinterpret_cast<uint8_t*>(&id) + sizeof(id));
}

RcclComm::RcclComm(const std::vector<uint8_t>& uid, int rank, int nranks, int device,
                   bool blocking)
    : rank_(rank), nranks_(nranks), device_(device), blocking_(blocking) {
  if (uid.size() != sizeof(ncclUniqueId))
    throw std::invalid_argument("unique id must be " + std::to_string(sizeof(ncclUniqueId)) +
                                " bytes");
  if (rank < 0 || rank >= nranks) throw std::invalid_argument("rank out of range");
  DSML_HIP_CHECK(hipSetDevice(device_));
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = blocking ? 1 : 0;
  check(ncclCommInitRankConfig(&comm_, nranks_, id, rank_, &cfg), "ncclCommInitRankConfig");
  DSML_HIP_CHECK(hipMalloc(&one_, 64));
  DSML_HIP_CHECK(hipMemset(one_, 0, 64));
}

RcclComm::~RcclComm() {
  (void)hipSetDevice(device_);
  if (comm_) {
    if (aborted_) {
      // already torn down by abort()
    } else {
      (void)ncclCommDestroy(comm_);
    }
  }
  if (tmp_) (void)hipFree(tmp_);
  if (one_) (void)hipFree(one_);
  for (hipEvent_t e : ev_xfer_) (void)hipEventDestroy(e);
  for (hipEvent_t e : ev_red_) (void)hipEventDestroy(e);
  if (fork_) (void)hipEventDestroy(fork_);
  if (join_) (void)hipEventDestroy(join_);
  if (red_) (void)hipStreamDestroy(red_);
}

void RcclComm::ensure_pipe(size_t groups) {
  if (red_ == nullptr) {
    DSML_HIP_CHECK(hipStreamCreateWithFlags(&red_, hipStreamNonBlocking));
    DSML_HIP_CHECK(hipEventCreateWithFlags(&fork_, hipEventDisableTiming));
    DSML_HIP_CHECK(hipEventCreateWithFlags(&join_, hipEventDisableTiming));
  }
  while (ev_red_.size() < groups) {
    hipEvent_t a, b;
    DSML_HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    DSML_HIP_CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    ev_xfer_.push_back(a);
    ev_red_.push_back(b);
  }
}

void RcclComm::check(ncclResult_t r, const char* what) {
  if (r == ncclInProgress) {
    // Non-blocking communicator: wait for the call to be enqueued, bounded so a
    // dead peer cannot wedge the caller forever (the health monitor aborts).
    const auto t0 = std::chrono::steady_clock::now();
    ncclResult_t st = ncclInProgress;
    while (st == ncclInProgress) {
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) break;
      if (st != ncclInProgress) break;
      if (aborted_) throw std::runtime_error(std::string(what) + ": communicator aborted");
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(300))
        throw std::runtime_error(std::string(what) + ": timed out waiting for RCCL");
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    r = st;
  }
  if (r != ncclSuccess)
    throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

void RcclComm::ensure_tmp(size_t bytes) {
  if (bytes <= tmp_bytes_) return;
  if (tmp_) DSML_HIP_CHECK(hipFree(tmp_));
  tmp_bytes_ = (bytes + 255) & ~size_t(255);
  DSML_HIP_CHECK(hipMalloc(&tmp_, tmp_bytes_));
}

size_t RcclComm::ring_tmp_bytes(int64_t count, int32_t dtype, int64_t chunk_bytes,
                                int max_rings) const {
  const int n = nranks_;
  if (n < 2 || count <= 0) return 0;
  const size_t es = dtype_size(dtype);
  const int64_t align = std::max<int64_t>(1, 16 / (int64_t)es);
  const int64_t chunk = chunk_bytes > 0 ? chunk_bytes / (int64_t)es : count;
  const auto plan = ring_schedule(n, rank_, count, align, chunk, max_rings);
  const int R = (int)directed_rings(n, max_rings).size();
  int64_t maxr = 0;
  for (const auto& g : plan)
    for (const auto& x : g)
      if (x.reduce) maxr = std::max(maxr, x.recv_len);
  const size_t slot = std::max<size_t>(((size_t)maxr * es + 255) & ~(size_t)255, 256);
  return slot * (size_t)R * 2;  // double buffered (the pipelined form alternates)
}

void RcclComm::reserve_ring(int64_t count, int32_t dtype, int64_t chunk_bytes, int max_rings) {
  ensure_tmp(ring_tmp_bytes(count, dtype, chunk_bytes, max_rings));
}

void RcclComm::allreduce(void* buf, int64_t count, int32_t dtype, int32_t op, hipStream_t s) {
  if (aborted_) throw std::runtime_error("allreduce on aborted communicator");
  check(ncclAllReduce(buf, buf, (size_t)count, to_nccl(dtype), to_nccl_op(op), comm_, s),
        "ncclAllReduce");
}

int RcclComm::pipeline_mode() const {
  static const bool kPipeEnv = [] {
    const char* e = std::getenv("HIPDSML_RING_PIPELINE");
    return e != nullptr && e[0] == '1';
  }();
  return pipe_default_ >= 0 ? pipe_default_ : (kPipeEnv ? 1 : 0);
}

void RcclComm::ring_allreduce(void* buf, int64_t count, int32_t dtype, int32_t op,
                              int64_t chunk_bytes, hipStream_t s, int max_rings, int pipe_mode) {
  if (aborted_) throw std::runtime_error("ring_allreduce on aborted communicator");
  const int n = nranks_;
  if (n < 2 || count == 0) return;
  const size_t es = dtype_size(dtype);
  // Slices / segments start on 16 B boundaries (vector reduce kernel); the
  // reference padded the whole buffer to a multiple of n instead
  // (gpu_coordinator_server.go:299-334).
  const int64_t align = std::max<int64_t>(1, 16 / (int64_t)es);
  const int64_t chunk = chunk_bytes > 0 ? chunk_bytes / (int64_t)es : count;
  const auto plan = ring_schedule(n, rank_, count, align, chunk, max_rings);
  const size_t need = ring_tmp_bytes(count, dtype, chunk_bytes, max_rings);
  const int R = (int)directed_rings(n, max_rings).size();
  const size_t slot = need / (size_t)(2 * R);
  if (need > tmp_bytes_) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &cs);
    if (cs != hipStreamCaptureStatusNone)
      throw std::runtime_error("ring_allreduce: reduce scratch must be reserved before a graph "
                               "capture (RcclComm::reserve_ring)");
    ensure_tmp(need);
  }
  uint8_t* b = static_cast<uint8_t*>(buf);
  uint8_t* tmp = static_cast<uint8_t*>(tmp_);
  const ncclDataType_t t = to_nccl(dtype);
  // Pipelined when the schedule has chunk rounds (ring_plan.h ring_pipeline):
  // the reduces run on red_, each transfer group waits only for the reduce of
  // the chunk it sends (and of the scratch slot it receives into), so chunk
  // c's reduce overlaps chunk c+1's transfer.  One round per step leaves
  // nothing to overlap: the single-stream order is kept (no event overhead).
  // Which schedule runs: the caller's choice, else the communicator's default
  // -- set by parallel/ring_tune.py after it timed both (the pipelined one
  // first validated on a throwaway communicator with a bounded wait, so a
  // hang there can never take down this one), else HIPDSML_RING_PIPELINE.
  const bool want = pipe_mode >= 0 ? pipe_mode == 1 : pipeline_mode() == 1;
  bool pipe = false;
  for (const auto& g : plan)
    if (want && !g.empty() && g[0].round > 0) pipe = true;
  const auto deps = pipe ? ring_pipeline(plan) : std::vector<RingDeps>(plan.size());
  if (pipe) {
    ensure_pipe(plan.size());
    DSML_HIP_CHECK(hipEventRecord(fork_, s));
    DSML_HIP_CHECK(hipStreamWaitEvent(red_, fork_, 0));
  }
  for (size_t i = 0; i < plan.size(); ++i) {
    const auto& g = plan[i];
    const bool rs = !g.empty() && g[0].reduce;
    if (pipe) {
      if (deps[i].wait_reduce >= 0) DSML_HIP_CHECK(hipStreamWaitEvent(s, ev_red_[deps[i].wait_reduce], 0));
      if (rs && deps[i].slot_free >= 0) DSML_HIP_CHECK(hipStreamWaitEvent(s, ev_red_[deps[i].slot_free], 0));
    }
    uint8_t* scr = tmp + slot * (size_t)R * (size_t)deps[i].slot;
    check(ncclGroupStart(), "ncclGroupStart");
    for (const auto& x : g) {
      if (x.send_len > 0)
        check(ncclSend(b + x.send_off * es, x.send_len, t, x.send_peer, comm_, s), "ncclSend");
      if (x.recv_len > 0) {
        void* dst = x.reduce ? (void*)(scr + slot * x.ring) : (void*)(b + x.recv_off * es);
        check(ncclRecv(dst, x.recv_len, t, x.recv_peer, comm_, s), "ncclRecv");
      }
    }
    check(ncclGroupEnd(), "ncclGroupEnd");
    if (!rs) continue;
    hipStream_t rs_s = s;
    if (pipe) {
      DSML_HIP_CHECK(hipEventRecord(ev_xfer_[i], s));
      DSML_HIP_CHECK(hipStreamWaitEvent(red_, ev_xfer_[i], 0));
      rs_s = red_;
    }
    // every ring's received segment of this step reduced by ONE launch
    ReduceSegs m{};
    for (const auto& x : g) {
      if (!x.reduce || x.recv_len <= 0) continue;
      if (m.count == kMaxReduceSegs) {
        DSML_HIP_CHECK(reduce_multi_inplace(m, dtype, op, rs_s));
        m.count = 0;
      }
      m.seg[m.count++] = ReduceSeg{b + x.recv_off * es, scr + slot * x.ring, x.recv_len};
    }
    if (m.count > 0) DSML_HIP_CHECK(reduce_multi_inplace(m, dtype, op, rs_s));
    if (pipe) DSML_HIP_CHECK(hipEventRecord(ev_red_[i], red_));
  }
  if (pipe) {  // every reduce done before the caller's next op on s
    DSML_HIP_CHECK(hipEventRecord(join_, red_));
    DSML_HIP_CHECK(hipStreamWaitEvent(s, join_, 0));
  }
}

void RcclComm::broadcast(void* buf, int64_t count, int32_t dtype, int root, hipStream_t s) {
  check(ncclBroadcast(buf, buf, (size_t)count, to_nccl(dtype), root, comm_, s), "ncclBroadcast");
}

void RcclComm::allgather(void* buf, int64_t count, int32_t dtype, hipStream_t s) {
  if (aborted_) throw std::runtime_error("allgather on aborted communicator");
  uint8_t* b = static_cast<uint8_t*>(buf);
  check(ncclAllGather(b + (size_t)rank_ * (size_t)count * dtype_size(dtype), b, (size_t)count,
                      to_nccl(dtype), comm_, s),
        "ncclAllGather");
}

void RcclComm::send(const void* buf, int64_t count, int32_t dtype, int peer, hipStream_t s) {
  check(ncclSend(buf, (size_t)count, to_nccl(dtype), peer, comm_, s), "ncclSend");
}

void RcclComm::recv(void* buf, int64_t count, int32_t dtype, int peer, hipStream_t s) {
  check(ncclRecv(buf, (size_t)count, to_nccl(dtype), peer, comm_, s), "ncclRecv");
}

void RcclComm::barrier(hipStream_t s) {
  check(ncclAllReduce(one_, one_, 1, ncclInt32, ncclSum, comm_, s), "barrier");
  DSML_HIP_CHECK(hipStreamSynchronize(s));
}

void RcclComm::abort() {
  if (aborted_ || !comm_) return;
  aborted_ = true;
  (void)ncclCommAbort(comm_);
}

std::string RcclComm::async_error() {
  if (aborted_) return "aborted";
  ncclResult_t st = ncclSuccess;
  const ncclResult_t r = ncclCommGetAsyncError(comm_, &st);
  if (r != ncclSuccess) return ncclGetErrorString(r);
  if (st == ncclSuccess) return "";
  if (st == ncclInProgress) return "in-progress";
  return ncclGetErrorString(st);
}

// ---------------------------------------------------------------------------
// MlpRunner
// ---------------------------------------------------------------------------
MlpRunner::MlpRunner(const MlpDesc& d, const MlpBuffers& b, float lr, float momentum,
                     float weight_decay)
    : d_(d), b_(b), lr_(lr), mom_(momentum), wd_(weight_decay) {
  if (d_.nlayers < 1 || d_.nlayers > kMaxLayers) throw std::invalid_argument("bad nlayers");
  if (!mlp_rowchain_fits(d_)) throw std::invalid_argument("MLP too wide for the fused row chain");
  if (b_.ctr == nullptr) throw std::invalid_argument("MlpRunner needs the step counters");
  cfg_ = mlp_plan_first_layer(d_);
  if (cfg_.nsplit > 8) throw std::invalid_argument("first layer needs > 8 K splits");
  if ((mom_ != 0.f || wd_ != 0.f) && b_.V == nullptr)
    throw std::invalid_argument("momentum/weight decay need a velocity buffer");
}

MlpRunner::~MlpRunner() {
  reset_graph();
  if (pk_herr_ != nullptr) (void)hipHostFree(pk_herr_);
}

bool MlpRunner::persist_failed() const {
  return pk_herr_ != nullptr && __atomic_load_n(pk_herr_, __ATOMIC_ACQUIRE) != 0u;
}

void MlpRunner::clear_persist_error() {
  if (pk_herr_ != nullptr) __atomic_store_n(pk_herr_, 0u, __ATOMIC_RELEASE);
  pk_carry_ = false;  // called when the buffer is rewound: nothing carries over
}

void MlpRunner::reset_graph() {
  for (auto& kv : graphs_) {
    if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    if (kv.second.graph) (void)hipGraphDestroy(kv.second.graph);
  }
  graphs_.clear();
  graph_steps_ = 0;
}

bool MlpRunner::captured(int steps) const {
  if (steps == 0) return graph_steps_ != 0;
  return graphs_.count(steps) != 0;
}

void MlpRunner::set_comm(RcclComm* c, int algo, int64_t chunk_bytes) {
  if (c != nullptr && c->nranks() > 1) pk_xb_ = nullptr, pk_x_ = nullptr;  // leaves the persistent step
  comm_ = c;
  algo_ = algo;
  chunk_bytes_ = chunk_bytes;
  reset_graph();
}

void MlpRunner::set_exchange(PeerExchange* x) {
  if (x != nullptr) {
    if (!x->connected()) throw std::invalid_argument("set_exchange: exchange not connected");
    if (mom_ != 0.f || wd_ != 0.f)
      throw std::invalid_argument("the fused xGMI exchange implements plain SGD only");
    if (x->ntiles() != mlp_wgrad_tiles(d_) || x->half() < b_.nparams)
      throw std::invalid_argument("set_exchange: exchange buffers sized for another model");
  }
  if (x != nullptr) pk_xb_ = nullptr, pk_x_ = nullptr;  // leaves the persistent step
  xchg_ = x;
  xact_ = false;
  reset_graph();
}

void MlpRunner::set_act_exchange(PeerExchange* x, const float* Xall, int64_t xstride, int waves) {
  if (x == nullptr) {
    set_exchange(nullptr);
    return;
  }
  if (!x->connected()) throw std::invalid_argument("set_act_exchange: exchange not connected");
  if (mom_ != 0.f || wd_ != 0.f)
    throw std::invalid_argument("the activation exchange implements plain SGD only");
  const int n = x->nranks();
  if (n < 2) throw std::invalid_argument("set_act_exchange: needs >= 2 ranks");
  if (!mlp_xact_supported(d_))
    throw std::invalid_argument("set_act_exchange: needs batch <= 64 and layer inputs % 16 == 0");
  if (x->ntiles() != n * (mlp_xact_payload(d_) / 1024) ||
      x->half() < (int64_t)n * mlp_xact_payload(d_))
    throw std::invalid_argument("set_act_exchange: exchange buffers sized for another model");
  if (Xall == nullptr || xstride < (int64_t)d_.nbatches * 64 * d_.dims[0])
    throw std::invalid_argument("set_act_exchange: replicated input shards too small");
  pk_xb_ = nullptr;  // leaves the persistent step
  pk_x_ = nullptr;
  xchg_ = x;
  xact_ = true;
  if (waves != 0 && waves != 4 && waves != 8)
    throw std::invalid_argument("set_act_exchange: waves must be 0 (auto), 4 or 8");
  xall_ = Xall;
  xstride_ = xstride;
  xact_waves_ = waves;
  reset_graph();
}

void MlpRunner::set_world_size(int n) {
  if (n < 1) throw std::invalid_argument("world size must be >= 1");
  world_ = n;
  reset_graph();
}

void MlpRunner::set_lr(float lr) {
  lr_ = lr;
  reset_graph();  // lr is a baked kernel argument
}

void MlpRunner::enqueue_fwd_bwd(hipStream_t s) {
  DSML_HIP_CHECK(mlp_f32_first_layer(b_.X, b_.ldx, b_.P, b_.slab, b_.ctr, 0, d_, cfg_, b_.labels, b_.ws, s));
  DSML_HIP_CHECK(mlp_f32_rowchain(b_.P, b_.slab, cfg_.nsplit, b_.ws, b_.labels, b_.ctr, 0, d_,
                                  b_.stats, 1, 1.0f / (float)d_.batch, s));
  DSML_HIP_CHECK(mlp_f32_wgrad(b_.X, b_.ldx, b_.P, b_.G, b_.ws, b_.ctr, 0, d_, lr_, 0, s));
}

void MlpRunner::enqueue_update(hipStream_t s) {
  const int n = comm_ ? comm_->nranks() : world_;
  const float gscale = 1.0f / (float)n;
  if (mom_ != 0.f || wd_ != 0.f)
    DSML_HIP_CHECK(sgd_momentum_f32(b_.P, b_.G, b_.V, b_.nparams, lr_, mom_, wd_, gscale, s));
  else
    DSML_HIP_CHECK(sgd_update_f32(b_.P, b_.G, b_.nparams, lr_ * gscale, s));
}

void MlpRunner::set_persist(uint64_t* xbuf, uint32_t* err, double timeout_ms, PeerExchange* x,
                            int algo) {
  if (xbuf == nullptr) {
    pk_xb_ = nullptr;
    pk_err_ = nullptr;
    pk_x_ = nullptr;
    reset_graph();
    return;
  }
  if (!mlp_persist_supported(d_))
    throw std::invalid_argument("set_persist: the persistent step covers 784-128-64-10 and "
                                "784-128-10 at batch <= 64");
  if (mom_ != 0.f || wd_ != 0.f) throw std::invalid_argument("set_persist: plain SGD only");
  if (x != nullptr) {
    const int n = x->nranks();
    if (!x->connected() || n < 2 || n != world_)
      throw std::invalid_argument("set_persist: the replica exchange must connect world_size >= 2 ranks");
    if (algo < 0 || algo > 4)
      throw std::invalid_argument("set_persist: algo must be 0 / 1 (pk / pk2), 2 / 3 (pkg / pkg2) "
                                  "or 4 (pkx)");
    if (x->ntiles() < px_ntiles(n, algo) || x->half() < px_half(n, algo))
      throw std::invalid_argument("set_persist: exchange buffers too small for the persistent step");
    xchg_ = nullptr;  // the three-launch exchanges are off while the persistent step runs
  } else if (comm_ != nullptr || xchg_ != nullptr || world_ != 1) {
    throw std::invalid_argument("set_persist: single replica only (or pass the replica exchange)");
  }
  pk_x_ = x;
  pk_algo_ = x != nullptr ? algo : 0;
  if (err == nullptr) throw std::invalid_argument("set_persist: needs an error word");
  if (pk_herr_ == nullptr) {
    void* h = nullptr;
    DSML_HIP_CHECK(hipHostMalloc(&h, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
    pk_herr_ = static_cast<uint32_t*>(h);
    *pk_herr_ = 0u;
  }
  pk_xb_ = xbuf;
  pk_err_ = err;
  pk_timeout_ = (uint64_t)(timeout_ms * 1e5);  // s_memrealtime: 100 MHz
  pk_carry_ = false;
  reset_graph();
}

void MlpRunner::enqueue_steps(int n, hipStream_t s) {
  if (n <= 0) return;
  if (pk_xb_ != nullptr) {
    const bool gram = pk_x_ == nullptr || pk_algo_ >= 2;
    if (gram && pk_gram_ == nullptr)
      throw std::invalid_argument("persistent step: set_persist_gram first (the Gram form's table)");
    if (gram) {
      // the data-parallel Gram forms read [nbatches][nrep][64][64]
      const int64_t reps = pk_x_ != nullptr ? pk_x_->nranks() : 1;
      if (pk_gram_numel_ < (int64_t)d_.nbatches * reps * 64 * 64)
        throw std::invalid_argument("persistent step: the Gram table is smaller than nbatches x "
                                    "replicas x 64 x 64 (a table built for another world size?)");
    }
    // a launch that gave up left a half-written pipeline: never carry it over
    if (persist_failed()) pk_carry_ = false;
    if (pk_x_ != nullptr && pk_algo_ == 4) {
      const int64_t per = (int64_t)d_.nbatches * (d_.dims[0] / 16) * 1024;
      if (pk_xsw_ == nullptr || pk_xsw_stride_ < per ||
          pk_xsw_numel_ < (int64_t)(pk_x_->nranks() - 1) * pk_xsw_stride_ + per)
        throw std::invalid_argument("persistent step (pkx): set_persist_xall with every replica's "
                                    "swizzled shard first");
    }
    if (gram && !pk_carry_) {
      // A launch without carried state recomputes the first step's Z1 in its
      // prologue under the SAME hand-off tags the previous launch's last step
      // published (partials and Z1 of step s0): clear them so no block can
      // take a stale granule for this launch's.
      DSML_HIP_CHECK(hipMemsetAsync(pk_xb_, 0, (size_t)mlp_persist_xbuf_granules() * sizeof(uint64_t), s));
    }
    if (pk_x_ != nullptr)
      DSML_HIP_CHECK(mlp_persist_steps(b_.X, b_.ldx, b_.labels, b_.P, b_.ctr, d_,
                                       lr_ / (float)pk_x_->nranks(), n, pk_xb_, b_.stats, pk_err_,
                                       pk_herr_, pk_timeout_, s, &pk_x_->args(), &pk_x_->table(),
                                       pk_algo_, gram ? pk_gram_ : nullptr, pk_carry_ ? 1 : 0,
                                       pk_xsw_, pk_xsw_stride_));
    else
      DSML_HIP_CHECK(mlp_persist_steps(b_.X, b_.ldx, b_.labels, b_.P, b_.ctr, d_, lr_, n, pk_xb_,
                                       b_.stats, pk_err_, pk_herr_, pk_timeout_, s, nullptr, nullptr,
                                       0, pk_gram_, pk_carry_ ? 1 : 0));
    if (gram) pk_carry_ = true;  // the next launch, in stream order, finds this one's state
    return;
  }
  for (int i = 0; i < n; ++i) enqueue_step(s);
}

void MlpRunner::enqueue_step(hipStream_t s) {
  if (pk_xb_ != nullptr) {
    enqueue_steps(1, s);
    return;
  }
  if (xchg_ != nullptr) {
    DSML_HIP_CHECK(mlp_f32_first_layer(b_.X, b_.ldx, b_.P, b_.slab, b_.ctr, 0, d_, cfg_, b_.labels, b_.ws, s));
    DSML_HIP_CHECK(mlp_f32_rowchain(b_.P, b_.slab, cfg_.nsplit, b_.ws, b_.labels, b_.ctr, 0, d_,
                                    b_.stats, 1, 1.0f / (float)d_.batch, s));
    if (xact_)
      DSML_HIP_CHECK(mlp_f32_wgrad_xact(xall_, xstride_, b_.P, b_.ws, b_.ctr, d_,
                                        lr_ / (float)xchg_->nranks(), xchg_->args(),
                                        xchg_->table(), xact_waves_, s));
    else
      DSML_HIP_CHECK(mlp_f32_wgrad_xchg(b_.X, b_.ldx, b_.P, b_.ws, b_.ctr, d_,
                                        lr_ / (float)xchg_->nranks(), xchg_->args(),
                                        xchg_->table(), s));
    return;
  }
  const bool multi = comm_ != nullptr && comm_->nranks() > 1;
  const bool plain = mom_ == 0.f && wd_ == 0.f;
  if (!multi && plain) {
    // Single replica, plain SGD: the update is fused into the weight-grad kernel.
    DSML_HIP_CHECK(mlp_f32_first_layer(b_.X, b_.ldx, b_.P, b_.slab, b_.ctr, 0, d_, cfg_, b_.labels, b_.ws, s));
    DSML_HIP_CHECK(mlp_f32_rowchain(b_.P, b_.slab, cfg_.nsplit, b_.ws, b_.labels, b_.ctr, 0, d_,
                                    b_.stats, 1, 1.0f / (float)d_.batch, s));
    DSML_HIP_CHECK(mlp_f32_wgrad(b_.X, b_.ldx, b_.P, b_.G, b_.ws, b_.ctr, 0, d_, lr_, 1, s));
    return;
  }
  enqueue_fwd_bwd(s);
  if (multi) {
    if (algo_ == 1)
      comm_->ring_allreduce(b_.G, b_.nparams, kF32, kSum, chunk_bytes_, s);
    else
      comm_->allreduce(b_.G, b_.nparams, kF32, kSum, s);
  }
  enqueue_update(s);
}

void MlpRunner::capture(int steps, bool capture_comm, hipStream_t s) {
  if (steps < 1) throw std::invalid_argument("capture: steps must be >= 1");
  if (capture_comm != capture_comm_) reset_graph();
  capture_comm_ = capture_comm;
  auto it = graphs_.find(steps);
  if (it != graphs_.end()) {  // recapture (buffers or plan may have changed)
    if (it->second.exec) (void)hipGraphExecDestroy(it->second.exec);
    if (it->second.graph) (void)hipGraphDestroy(it->second.graph);
    graphs_.erase(it);
  }
  Captured c;
  DSML_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  try {
    enqueue_steps(steps, s);
  } catch (...) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(s, &g);
    if (g) (void)hipGraphDestroy(g);
    throw;
  }
  DSML_HIP_CHECK(hipStreamEndCapture(s, &c.graph));
  const hipError_t e = hipGraphInstantiate(&c.exec, c.graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(c.graph);
    DSML_HIP_CHECK(e);
  }
  graphs_[steps] = c;
  graph_steps_ = steps;
}

void MlpRunner::replay(hipStream_t s, int steps) {
  if (steps == 0) steps = graph_steps_;
  auto it = graphs_.find(steps);
  if (it == graphs_.end()) throw std::runtime_error("replay: no captured graph of that size");
  DSML_HIP_CHECK(hipGraphLaunch(it->second.exec, s));
}

void mlp_eval(const MlpDesc& d, const float* X, int64_t ldx, const int32_t* labels, int64_t row0,
              const float* P, float* ws, float* slab, float* stats, hipStream_t s, bool logits) {
  const MlpLaunchCfg c = mlp_plan_first_layer(d);
  DSML_HIP_CHECK(mlp_f32_first_layer(X, ldx, P, slab, nullptr, row0, d, c, labels, ws, s));
  DSML_HIP_CHECK(mlp_f32_rowchain(P, slab, c.nsplit, ws, labels, nullptr, row0, d, stats,
                                  logits ? 2 : 0, 1.0f, s));
}

}  // namespace dsml
