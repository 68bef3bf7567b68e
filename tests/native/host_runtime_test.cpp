// Sanitizer test of the host-side runtime (built by tests/test_host_sanitizers.py
// with g++ -fsanitize=address,undefined, and -fsanitize=thread for the
// concurrent StreamTable section), against the host-only HIP stand-in in
// csrc/hostshim.  Covers: ring_plan.h schedules for every n <= 8 (all ranks
// simulated with RCCL's per-pair FIFO send/recv matching: no deadlock, exact
// sums), DeviceArena bounds (incl. overflow
// at the top of the address space), CopyEngine chunking at every staging
// boundary, and the StreamTable state machine single- and multi-threaded.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "runtime/runtime.h"

using namespace dsml;

static int g_fail = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                                  \
    }                                                                            \
  } while (0)

// ---- ring schedule: every rank simulated with RCCL p2p semantics -------------
// Each rank posts its group's sends, then completes the group once every
// receive of it can be matched; sends and receives match in FIFO order per
// (src, dst) pair (how ncclSend/ncclRecv pair up).  No progress = deadlock.
static void ring_sim(int n, int64_t count, int64_t align, int64_t chunk, int max_rings) {
  std::vector<std::vector<std::vector<RingXfer>>> plans(n);
  for (int r = 0; r < n; ++r) {
    plans[r] = ring_schedule(n, r, count, align, chunk, max_rings);
    // the pipelined form's dependencies only point backwards (ring_pipeline)
    const auto deps = ring_pipeline(plans[r]);
    CHECK(deps.size() == plans[r].size());
    for (size_t i = 0; i < deps.size(); ++i) {
      CHECK(deps[i].wait_reduce < (int)i && deps[i].slot_free < (int)i);
      CHECK(deps[i].slot == 0 || deps[i].slot == 1);
    }
  }
  std::vector<std::vector<double>> buf(n, std::vector<double>(count > 0 ? count : 0));
  std::vector<double> want(count > 0 ? count : 0, 0.0);
  for (int r = 0; r < n; ++r)
    for (int64_t i = 0; i < count; ++i) {
      buf[r][i] = (double)((r + 1) * 1000 + (i % 97));
      want[i] += buf[r][i];
    }
  if (n < 2) {
    for (int r = 0; r < n; ++r) CHECK(plans[r].empty());
    return;
  }
  std::vector<std::vector<std::vector<std::vector<double>>>> q(
      n, std::vector<std::vector<std::vector<double>>>(n));  // q[src][dst] = FIFO of payloads
  std::vector<std::vector<size_t>> head(n, std::vector<size_t>(n, 0));
  std::vector<size_t> pc(n, 0);
  std::vector<bool> posted(n, false);
  for (;;) {
    bool progress = false, done = true;
    for (int r = 0; r < n; ++r) {
      if (pc[r] >= plans[r].size()) continue;
      done = false;
      const auto& g = plans[r][pc[r]];
      if (!posted[r]) {
        for (const RingXfer& x : g)
          if (x.send_len > 0) {
            CHECK(x.send_peer >= 0 && x.send_peer < n && x.send_peer != r);
            CHECK(x.send_off >= 0 && x.send_off + x.send_len <= count && x.send_off % align == 0);
            if (x.send_peer < 0 || x.send_peer >= n || x.send_off + x.send_len > count) return;
            q[r][x.send_peer].emplace_back(buf[r].begin() + x.send_off,
                                           buf[r].begin() + x.send_off + x.send_len);
          }
        posted[r] = true;
        progress = true;
      }
      std::vector<int> need(n, 0);
      for (const RingXfer& x : g)
        if (x.recv_len > 0) {
          CHECK(x.recv_peer >= 0 && x.recv_peer < n && x.recv_peer != r);
          if (x.recv_peer < 0 || x.recv_peer >= n) return;
          need[x.recv_peer]++;
        }
      bool ready = true;
      for (int p = 0; p < n; ++p)
        if (q[p][r].size() - head[p][r] < (size_t)need[p]) ready = false;
      if (!ready) continue;
      for (const RingXfer& x : g) {
        if (x.recv_len <= 0) continue;
        const std::vector<double>& d = q[x.recv_peer][r][head[x.recv_peer][r]++];
        CHECK((int64_t)d.size() == x.recv_len);
        CHECK(x.recv_off >= 0 && x.recv_off + x.recv_len <= count && x.recv_off % align == 0);
        if ((int64_t)d.size() != x.recv_len || x.recv_off + x.recv_len > count) return;
        for (int64_t i = 0; i < x.recv_len; ++i) {
          if (x.reduce) buf[r][x.recv_off + i] += d[i];
          else buf[r][x.recv_off + i] = d[i];
        }
      }
      pc[r]++;
      posted[r] = false;
      progress = true;
    }
    if (done) break;
    if (!progress) {
      std::fprintf(stderr, "ring n=%d count=%lld chunk=%lld: deadlock\n", n, (long long)count,
                   (long long)chunk);
      ++g_fail;
      return;
    }
  }
  for (int s = 0; s < n; ++s)
    for (int d = 0; d < n; ++d) CHECK(head[s][d] == q[s][d].size());  // every send received
  for (int r = 0; r < n; ++r)
    for (int64_t i = 0; i < count; ++i)
      if (buf[r][i] != want[i]) {
        std::fprintf(stderr, "ring n=%d count=%lld chunk=%lld rings=%d rank %d elem %lld: %f != %f\n",
                     n, (long long)count, (long long)chunk, max_rings, r, (long long)i,
                     buf[r][i], want[i]);
        ++g_fail;
        return;
      }
}

static void test_rings() {
  for (int n = 1; n <= 8; ++n)
    for (int64_t count : {1LL, 3LL, 17LL, 1000LL, 4101LL})
      for (int64_t chunk : {0LL, 16LL, 64LL})
        for (int mr : {0, 1}) ring_sim(n, count, 4, chunk, mr);
  // directed rings never share a directed link
  for (int n = 2; n <= 8; ++n) {
    const auto rings = directed_rings(n, 0);
    std::vector<int> used(n * n, 0);
    for (const auto& rg : rings) {
      CHECK((int)rg.size() == n);
      for (int i = 0; i < n; ++i) used[rg[i] * n + rg[(i + 1) % n]]++;
    }
    for (int v : used) CHECK(v <= 1);
  }
}

// ---- DeviceArena --------------------------------------------------------------
static void test_arena() {
  DeviceArena a(0, 1 << 16);
  CHECK(a.min_addr() == 0x1000 && a.max_addr() == 0x1000 + (1 << 16));
  CHECK(a.contains(0x1000, 1 << 16));
  CHECK(!a.contains(0x1000, (1 << 16) + 1));
  CHECK(!a.contains(0xfff, 1));
  CHECK(a.contains(0x1000 + (1 << 16), 0));
  CHECK(!a.contains(UINT64_MAX - 4, 16));  // no wrap-around at the top
  CHECK(!a.contains(0x2000, UINT64_MAX));
  bool threw = false;
  try { (void)a.translate(0x1000 + (1 << 16) - 4, 8); } catch (const std::out_of_range&) { threw = true; }
  CHECK(threw);
  uint8_t* p = static_cast<uint8_t*>(a.translate(0x1000, 16));
  std::memset(p, 7, 16);
  a.record_extent(0x1000, 16);
  CHECK(a.extent(0x1000) == 16 && a.extent(0x2000) == 0);
}

// ---- CopyEngine chunking --------------------------------------------------------
static void test_copy_engine() {
  CopyEngine ce(0, 8192);  // half = 4096: multi-chunk pipelines on both directions
  DeviceArena a(0, 1 << 20);
  std::mt19937 rng(5);
  for (size_t n : {size_t(0), size_t(1), size_t(4095), size_t(4096), size_t(4097), size_t(8192),
                   size_t(12289), size_t(100003)}) {
    std::vector<uint8_t> src(n), back(n, 0);
    for (auto& b : src) b = (uint8_t)rng();
    void* dev = a.translate(0x1000, n);
    ce.h2d(dev, src.data(), n);
    ce.d2h(back.data(), dev, n);
    CHECK(src == back);
    void* dev2 = a.translate(0x1000 + (1 << 19), n);
    ce.d2d(dev2, dev, n);
    std::vector<uint8_t> b2(n, 0);
    ce.d2h(b2.data(), dev2, n);
    CHECK(b2 == src);
  }
  CHECK(ce.bytes_h2d() > 0 && ce.bytes_d2h() > 0);
}

// ---- StreamTable state machine ----------------------------------------------------
static void test_stream_table_serial() {
  DeviceArena a(0, 1 << 16);
  CopyEngine ce(0, 8192);
  StreamTable t(&a, &ce);
  const uint64_t id = t.begin_send(0x1000, 10, 1);
  CHECK(id >= 1);
  CHECK(t.status(id) == XferStatus::kInProgress);
  CHECK(!t.push_chunk(id, "abc", 3));  // receive not bound yet -> FAILED
  CHECK(t.status(id) == XferStatus::kFailed);
  const uint64_t id2 = t.begin_send(0x1000, 10, 1);
  bool threw = false;
  try { t.begin_receive(999, 0x2000, 10, 0); } catch (const std::invalid_argument&) { threw = true; }
  CHECK(threw);
  threw = false;
  try { t.begin_receive(id2, 0x1000 + (1 << 16) - 4, 10, 0); } catch (const std::out_of_range&) { threw = true; }
  CHECK(threw);
  t.begin_receive(id2, 0x2000, 10, 0);
  CHECK(t.push_chunk(id2, "chunk", 5));
  CHECK(t.push_chunk(id2, "chunk", 5));
  CHECK(!t.push_chunk(id2, "x", 1));  // overflow
  CHECK(!t.finish(id2));              // overflow marked it FAILED
  const uint64_t id3 = t.begin_send(0x2000, 10, 1);
  t.begin_receive(id3, 0x3000, 0, 0);  // numBytes 0: the send's count
  CHECK(t.push_chunk(id3, "0123456789", 10));
  CHECK(t.finish(id3));
  CHECK(t.status(id3) == XferStatus::kSuccess);
  const auto v = t.read_send_buffer(id3);
  CHECK(v.size() == 10);
  CHECK(t.status(12345) == XferStatus::kFailed);
  t.erase(id3);
  CHECK(t.status(id3) == XferStatus::kFailed);
  t.erase(999999);  // unknown: no-op
}

static void test_stream_table_threads() {
  DeviceArena a(0, 8 << 20);
  CopyEngine ce(0, 16384);
  StreamTable t(&a, &ce);
  constexpr int kThreads = 8, kStreams = 24, kChunk = 1000, kChunks = 5;
  std::atomic<int> ok{0};
  std::vector<std::thread> th;
  for (int w = 0; w < kThreads; ++w) {
    th.emplace_back([&, w] {
      for (int s = 0; s < kStreams; ++s) {
        const uint64_t dst = 0x1000 + (uint64_t)(w * kStreams + s) * kChunk * kChunks;
        const uint64_t id = t.begin_send(0x1000, kChunk * kChunks, (uint32_t)w);
        t.begin_receive(id, dst, 0, (uint32_t)w);
        std::vector<uint8_t> c(kChunk, (uint8_t)(w * 31 + s));
        bool good = true;
        for (int k = 0; k < kChunks; ++k) good &= t.push_chunk(id, c.data(), c.size());
        good &= t.finish(id);
        good &= t.status(id) == XferStatus::kSuccess;
        (void)t.size();
        if (good) ok++;
        if (s % 3 == 0) t.erase(id);
      }
    });
  }
  for (auto& x : th) x.join();
  CHECK(ok.load() == kThreads * kStreams);
  // every region holds its writer's byte
  for (int w = 0; w < kThreads; ++w)
    for (int s = 0; s < kStreams; ++s) {
      const uint64_t dst = 0x1000 + (uint64_t)(w * kStreams + s) * kChunk * kChunks;
      const uint8_t* p = static_cast<const uint8_t*>(a.translate(dst, kChunk * kChunks));
      for (int i = 0; i < kChunk * kChunks; i += 997) CHECK(p[i] == (uint8_t)(w * 31 + s));
    }
}

int main(int argc, char** argv) {
  const std::string what = argc > 1 ? argv[1] : "all";
  if (what == "all" || what == "serial") {
    test_rings();
    test_arena();
    test_copy_engine();
    test_stream_table_serial();
  }
  if (what == "all" || what == "threads") test_stream_table_threads();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host runtime OK (%s)\n", what.c_str());
  return 0;
}
