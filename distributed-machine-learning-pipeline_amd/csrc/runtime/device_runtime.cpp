// DeviceArena / CopyEngine / StreamTable: the device-side runtime that backs
// the GPUDevice gRPC servicer on a real MI355X.
#include <cstring>

#include "runtime.h"

namespace dsml {

std::string hip_error_string(hipError_t e) { return std::string(hipGetErrorString(e)); }

// ---------------------------------------------------------------------------
// DeviceArena
// ---------------------------------------------------------------------------
DeviceArena::DeviceArena(int device, uint64_t size_bytes, uint64_t base_addr)
    : device_(device), base_(base_addr), size_(size_bytes) {
  if (size_bytes == 0) throw std::invalid_argument("DeviceArena: size must be > 0");
  DSML_HIP_CHECK(hipSetDevice(device_));
  DSML_HIP_CHECK(hipMalloc(&ptr_, size_));
  DSML_HIP_CHECK(hipMemset(ptr_, 0, size_));
}

DeviceArena::~DeviceArena() {
  if (ptr_) {
    (void)hipSetDevice(device_);
    (void)hipFree(ptr_);
  }
}

bool DeviceArena::contains(uint64_t addr, uint64_t nbytes) const {
  if (addr < base_) return false;
  const uint64_t off = addr - base_;
  if (off > size_) return false;
  return nbytes <= size_ - off;
}

void* DeviceArena::translate(uint64_t addr, uint64_t nbytes) const {
  if (!contains(addr, nbytes))
    throw std::out_of_range("memory address out of range: addr=" + std::to_string(addr) +
                            " bytes=" + std::to_string(nbytes) + " valid=[" +
                            std::to_string(base_) + "," + std::to_string(base_ + size_) + ")");
  return static_cast<uint8_t*>(ptr_) + (addr - base_);
}

void DeviceArena::record_extent(uint64_t addr, uint64_t nbytes) {
  std::lock_guard<std::mutex> g(mu_);
  extents_[addr] = nbytes;
}

uint64_t DeviceArena::extent(uint64_t addr) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = extents_.find(addr);
  return it == extents_.end() ? 0 : it->second;
}

// ---------------------------------------------------------------------------
// CopyEngine
// ---------------------------------------------------------------------------
CopyEngine::CopyEngine(int device, size_t staging_bytes) : device_(device) {
  DSML_HIP_CHECK(hipSetDevice(device_));
  half_ = staging_bytes / 2;
  if (half_ < 4096) half_ = 4096;
  for (int i = 0; i < 2; ++i) {
    DSML_HIP_CHECK(hipHostMalloc(&pin_up_[i], half_, hipHostMallocDefault));
    DSML_HIP_CHECK(hipHostMalloc(&pin_dn_[i], half_, hipHostMallocDefault));
    DSML_HIP_CHECK(hipEventCreateWithFlags(&ev_up_[i], hipEventDisableTiming));
    DSML_HIP_CHECK(hipEventCreateWithFlags(&ev_dn_[i], hipEventDisableTiming));
  }
  DSML_HIP_CHECK(hipStreamCreateWithFlags(&s_h2d_, hipStreamNonBlocking));
  DSML_HIP_CHECK(hipStreamCreateWithFlags(&s_d2h_, hipStreamNonBlocking));
  DSML_HIP_CHECK(hipStreamCreateWithFlags(&s_d2d_, hipStreamNonBlocking));
}

CopyEngine::~CopyEngine() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(s_h2d_);
  (void)hipStreamSynchronize(s_d2h_);
  (void)hipStreamSynchronize(s_d2d_);
  for (int i = 0; i < 2; ++i) {
    (void)hipHostFree(pin_up_[i]);
    (void)hipHostFree(pin_dn_[i]);
    (void)hipEventDestroy(ev_up_[i]);
    (void)hipEventDestroy(ev_dn_[i]);
  }
  (void)hipStreamDestroy(s_h2d_);
  (void)hipStreamDestroy(s_d2h_);
  (void)hipStreamDestroy(s_d2d_);
}

void CopyEngine::h2d(void* dst_dev, const void* src_host, size_t n) {
  std::lock_guard<std::mutex> g(mu_up_);
  DSML_HIP_CHECK(hipSetDevice(device_));
  const uint8_t* src = static_cast<const uint8_t*>(src_host);
  uint8_t* dst = static_cast<uint8_t*>(dst_dev);
  bool used[2] = {false, false};
  size_t off = 0;
  int buf = 0;
  while (off < n) {
    const size_t c = (n - off) < half_ ? (n - off) : half_;
    if (used[buf]) DSML_HIP_CHECK(hipEventSynchronize(ev_up_[buf]));  // staging reusable
    std::memcpy(pin_up_[buf], src + off, c);
    DSML_HIP_CHECK(hipMemcpyAsync(dst + off, pin_up_[buf], c, hipMemcpyHostToDevice, s_h2d_));
    DSML_HIP_CHECK(hipEventRecord(ev_up_[buf], s_h2d_));
    used[buf] = true;
    off += c;
    buf ^= 1;
  }
  DSML_HIP_CHECK(hipStreamSynchronize(s_h2d_));
  bytes_h2d_ += n;
}

void CopyEngine::d2h(void* dst_host, const void* src_dev, size_t n) {
  std::lock_guard<std::mutex> g(mu_dn_);
  DSML_HIP_CHECK(hipSetDevice(device_));
  const uint8_t* src = static_cast<const uint8_t*>(src_dev);
  uint8_t* dst = static_cast<uint8_t*>(dst_host);
  // Issue chunk c+1's DMA before copying chunk c out of staging.
  size_t off = 0, pend_off = 0, pend_n = 0;
  int buf = 0, pend_buf = -1;
  while (off < n || pend_buf >= 0) {
    int issued = -1;
    size_t c = 0;
    if (off < n) {
      c = (n - off) < half_ ? (n - off) : half_;
      DSML_HIP_CHECK(hipMemcpyAsync(pin_dn_[buf], src + off, c, hipMemcpyDeviceToHost, s_d2h_));
      DSML_HIP_CHECK(hipEventRecord(ev_dn_[buf], s_d2h_));
      issued = buf;
    }
    if (pend_buf >= 0) {
      DSML_HIP_CHECK(hipEventSynchronize(ev_dn_[pend_buf]));
      std::memcpy(dst + pend_off, pin_dn_[pend_buf], pend_n);
      pend_buf = -1;
    }
    if (issued >= 0) {
      pend_buf = issued;
      pend_off = off;
      pend_n = c;
      off += c;
      buf ^= 1;
    }
  }
  bytes_d2h_ += n;
}

void CopyEngine::d2d(void* dst_dev, const void* src_dev, size_t n) {
  std::lock_guard<std::mutex> g(mu_dd_);
  DSML_HIP_CHECK(hipSetDevice(device_));
  DSML_HIP_CHECK(hipMemcpyAsync(dst_dev, src_dev, n, hipMemcpyDeviceToDevice, s_d2d_));
  DSML_HIP_CHECK(hipStreamSynchronize(s_d2d_));
}

// ---------------------------------------------------------------------------
// StreamTable
// ---------------------------------------------------------------------------
StreamTable::StreamTable(DeviceArena* arena, CopyEngine* ce) : arena_(arena), ce_(ce) {}

StreamTable::~StreamTable() {
  for (auto& kv : streams_)
    if (kv.second.done) (void)hipEventDestroy(kv.second.done);
}

uint64_t StreamTable::begin_send(uint64_t send_addr, uint64_t num_bytes, uint32_t dst_rank) {
  std::lock_guard<std::mutex> g(mu_);
  const uint64_t id = next_id_++;
  StreamState st;
  st.send_addr = send_addr;
  st.num_bytes = num_bytes;
  st.dst_rank = dst_rank;
  st.initiated_send = true;
  streams_[id] = st;
  return id;
}

void StreamTable::begin_receive(uint64_t stream_id, uint64_t recv_addr, uint64_t num_bytes,
                                uint32_t src_rank) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = streams_.find(stream_id);
  if (it == streams_.end())
    throw std::invalid_argument("stream not found: " + std::to_string(stream_id));
  const uint64_t n = num_bytes ? num_bytes : it->second.num_bytes;
  if (!arena_->contains(recv_addr, n))
    throw std::out_of_range("receive buffer out of range: " + std::to_string(recv_addr));
  it->second.recv_addr = recv_addr;
  it->second.src_rank = src_rank;
  it->second.initiated_recv = true;
}

bool StreamTable::push_chunk(uint64_t stream_id, const void* data, uint64_t n) {
  StreamState* st;
  uint64_t dst;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = streams_.find(stream_id);
    if (it == streams_.end()) return false;
    st = &it->second;
    if (!st->initiated_recv || st->received + n > st->num_bytes) {
      st->status = XferStatus::kFailed;
      return false;
    }
    dst = st->recv_addr + st->received;
    st->received += n;
  }
  if (n) ce_->h2d(arena_->translate(dst, n), data, n);
  return true;
}

bool StreamTable::finish(uint64_t stream_id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = streams_.find(stream_id);
  if (it == streams_.end()) return false;
  StreamState& st = it->second;
  const bool ok = st.initiated_recv && st.received == st.num_bytes &&
                  st.status != XferStatus::kFailed;
  st.status = ok ? XferStatus::kSuccess : XferStatus::kFailed;
  if (ok) arena_->record_extent(st.recv_addr, st.num_bytes);
  return ok;
}

XferStatus StreamTable::status(uint64_t stream_id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = streams_.find(stream_id);
  if (it == streams_.end()) return XferStatus::kFailed;
  return it->second.status;
}

std::vector<uint8_t> StreamTable::read_send_buffer(uint64_t stream_id) {
  uint64_t addr, n;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = streams_.find(stream_id);
    if (it == streams_.end())
      throw std::invalid_argument("stream not found: " + std::to_string(stream_id));
    addr = it->second.send_addr;
    n = it->second.num_bytes;
  }
  std::vector<uint8_t> out(n);
  if (n) ce_->d2h(out.data(), arena_->translate(addr, n), n);
  return out;
}

void StreamTable::erase(uint64_t stream_id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = streams_.find(stream_id);
  if (it == streams_.end()) return;
  if (it->second.done) (void)hipEventDestroy(it->second.done);
  streams_.erase(it);
}

size_t StreamTable::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return streams_.size();
}

}  // namespace dsml
