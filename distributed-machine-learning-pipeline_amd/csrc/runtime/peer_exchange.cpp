// Peer exchange buffers for the xGMI-fused gradient all-reduce.
//
// Replaces, for the training step, the reference's coordinator "ring"
// (gpu_coordinator_server.go:272-566: 2(n-1) rounds of BeginSend / BeginReceive /
// StreamSend / 50 ms status polling / Memcpy per rank and step).
// On MI355X every GPU reaches every other over a direct xGMI link, so for the
// 437 KB gradient of the flagship MLP the latency-optimal all-reduce is one-shot:
// each replica publishes its gradient tiles in its own HBM, and the weight-gradient
// kernel of every peer reads them directly (kernels/mlp_f32.hip, XCHG path).
// This file only owns memory: allocation (uncached, IPC-exportable), handle
// export/import, the device-side pointer table and the error word.
#include <cstring>

#include "runtime.h"

namespace dsml {

PeerExchange::PeerExchange(int device, int64_t half_floats, int ntiles)
    : device_(device), half_(half_floats), ntiles_(ntiles) {
  if (half_floats <= 0 || ntiles <= 0) throw std::invalid_argument("PeerExchange: empty");
  DSML_HIP_CHECK(hipSetDevice(device));
  flag_off_ = ((size_t)(2 * half_floats) * sizeof(float) + 255) & ~(size_t)255;
  bytes_ = flag_off_ + (size_t)ntiles * sizeof(uint64_t);
  // Uncached HBM: peers' reads/writes over xGMI never see stale cache lines.
  if (hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocUncached) == hipSuccess) {
    kind_ = "uncached";
  } else {
    (void)hipGetLastError();
    if (hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocFinegrained) == hipSuccess) {
      kind_ = "finegrained";
    } else {
      (void)hipGetLastError();
      DSML_HIP_CHECK(hipMalloc(&base_, bytes_));
      kind_ = "coarse";
    }
  }
  DSML_HIP_CHECK(hipMemset(base_, 0, bytes_));
  DSML_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&dtab_), sizeof(XchgTab)));
  DSML_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&err_), 256));
  DSML_HIP_CHECK(hipMemset(err_, 0, 256));
  DSML_HIP_CHECK(hipDeviceSynchronize());
  args_.half = half_;
  args_.err = err_;
  set_timeout_ms(10000.0);
}

PeerExchange::~PeerExchange() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
  if (dtab_) (void)hipFree(dtab_);
  if (err_) (void)hipFree(err_);
  if (base_) (void)hipFree(base_);
}

std::vector<uint8_t> PeerExchange::ipc_handle() const {
  hipIpcMemHandle_t h;
  DSML_HIP_CHECK(hipSetDevice(device_));
  DSML_HIP_CHECK(hipIpcGetMemHandle(&h, base_));
  std::vector<uint8_t> out(sizeof(h));
  std::memcpy(out.data(), &h, sizeof(h));
  return out;
}

void PeerExchange::publish_table(const XchgTab& t, int rank, int n) {
  DSML_HIP_CHECK(hipMemcpy(dtab_, &t, sizeof(t), hipMemcpyHostToDevice));
  tab_host_ = t;
  args_.tab = dtab_;
  args_.rank = rank;
  args_.nranks = n;
}

void PeerExchange::connect_ipc(int rank, const std::vector<std::vector<uint8_t>>& handles) {
  const int n = (int)handles.size();
  if (n < 1 || n > kMaxPeers || rank < 0 || rank >= n)
    throw std::invalid_argument("connect_ipc: bad rank / group size");
  if (!opened_.empty()) throw std::runtime_error("connect_ipc: already connected");
  DSML_HIP_CHECK(hipSetDevice(device_));
  XchgTab t{};
  for (int r = 0; r < n; ++r) {
    char* b;
    if (r == rank) {
      b = static_cast<char*>(base_);
    } else {
      if (handles[r].size() != sizeof(hipIpcMemHandle_t))
        throw std::invalid_argument("connect_ipc: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      DSML_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(p);
      b = static_cast<char*>(p);
    }
    t.buf[r] = reinterpret_cast<float*>(b);
    t.flags[r] = reinterpret_cast<uint64_t*>(b + flag_off_);
  }
  publish_table(t, rank, n);
}

void PeerExchange::connect_local(int rank, const std::vector<PeerExchange*>& peers) {
  const int n = (int)peers.size();
  if (n < 1 || n > kMaxPeers || rank < 0 || rank >= n || peers[rank] != this)
    throw std::invalid_argument("connect_local: bad rank / group");
  DSML_HIP_CHECK(hipSetDevice(device_));
  XchgTab t{};
  for (int r = 0; r < n; ++r) {
    if (peers[r]->half_ != half_ || peers[r]->ntiles_ != ntiles_)
      throw std::invalid_argument("connect_local: peers sized differently");
    if (peers[r]->device_ != device_) {
      int ok = 0;
      DSML_HIP_CHECK(hipDeviceCanAccessPeer(&ok, device_, peers[r]->device_));
      if (!ok) throw std::runtime_error("connect_local: no peer access");
      const hipError_t e = hipDeviceEnablePeerAccess(peers[r]->device_, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) DSML_HIP_CHECK(e);
      (void)hipGetLastError();
    }
    t.buf[r] = peers[r]->buf();
    t.flags[r] = peers[r]->flags();
  }
  publish_table(t, rank, n);
}

void PeerExchange::allreduce(const float* in, float* out, int64_t n, hipStream_t s, int algo) {
  if (!connected()) throw std::runtime_error("PeerExchange::allreduce: not connected");
  const int64_t cs = ((n + args_.nranks - 1) / args_.nranks + 3) / 4 * 4;
  const int64_t need = algo == 1 ? n + cs : n;
  if (n % 4 || need > half_)
    throw std::invalid_argument("PeerExchange::allreduce: n must be a multiple of 4 and fit the "
                                "exchange (" + std::to_string(half_) + " floats)");
  DSML_HIP_CHECK(hipSetDevice(device_));
  if (algo == 1)
    DSML_HIP_CHECK(xchg_allreduce2_f32(in, out, n, args_, ntiles_, ++seq_, s));
  else
    DSML_HIP_CHECK(xchg_allreduce_f32(in, out, n, args_, ntiles_, ++seq_, s));
}

void PeerExchange::reset(hipStream_t s) {
  seq_ = 0;
  DSML_HIP_CHECK(hipSetDevice(device_));
  DSML_HIP_CHECK(hipMemsetAsync(flags(), 0, (size_t)ntiles_ * sizeof(uint64_t), s));
  DSML_HIP_CHECK(hipMemsetAsync(err_, 0, sizeof(uint32_t), s));
  // the payload too: protocols that tag the data itself ({value, step} granules,
  // the persistent step) must not match a stale slot after a rewind
  DSML_HIP_CHECK(hipMemsetAsync(buf(), 0, (size_t)2 * (size_t)half_ * sizeof(float), s));
}

uint32_t PeerExchange::error(hipStream_t s) {
  uint32_t v = 0;
  DSML_HIP_CHECK(hipSetDevice(device_));
  DSML_HIP_CHECK(hipMemcpyAsync(&v, err_, sizeof(v), hipMemcpyDeviceToHost, s));
  DSML_HIP_CHECK(hipStreamSynchronize(s));
  return v;
}

void PeerExchange::set_timeout_ms(double ms) {
  args_.timeout_ticks = (uint64_t)(ms * 1e5);  // s_memrealtime runs at 100 MHz
}

}  // namespace dsml
