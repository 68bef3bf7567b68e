// Multi-ring all-reduce schedule over edge-disjoint Hamiltonian cycles.
//
// xGMI on an MI355X node is a full mesh of point-to-point links (7 per GPU), so
// one ring (the reference's algorithm, gpu_coordinator_server.go:338-356, or a
// naive ncclSend/ncclRecv ring) drives ONE outgoing link per GPU.  K_n splits
// into floor((n-1)/2) edge-disjoint Hamiltonian cycles; running each cycle in
// both directions gives 2*floor((n-1)/2) directed rings that never share a
// directed link (n = 8: 6 rings on 6 of the 7 links).  The buffer is cut into
// one slice per ring; every ring runs reduce-scatter + all-gather on its slice,
// and all rings' transfers of a step go into one ncclGroup.
//
// The schedule is pure index arithmetic (no RCCL), so it is unit-tested on the
// CPU by simulating every rank (tests/test_ring_plan.py).
#pragma once
#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace dsml {

struct RingXfer {
  int ring;
  int send_peer;       // -1: nothing to send
  int64_t send_off, send_len;  // elements
  int recv_peer;       // -1: nothing to receive
  int64_t recv_off, recv_len;
  bool reduce;         // reduce-scatter (receive into scratch, then reduce) vs all-gather (in place)
  int step = 0;        // step within its phase (0 .. n-2)
  int round = 0;       // chunk round within the step
};

// Undirected edge-disjoint Hamiltonian cycles of K_n (found by exhaustive
// search offline; any rank computes the same table).
inline std::vector<std::vector<int>> hamiltonian_cycles(int n) {
  switch (n) {
    case 3: return {{0, 1, 2}};
    case 4: return {{0, 1, 2, 3}};
    case 5: return {{0, 1, 2, 3, 4}, {0, 2, 4, 1, 3}};
    case 6: return {{0, 1, 2, 3, 4, 5}, {0, 2, 4, 1, 5, 3}};
    case 7: return {{0, 1, 2, 3, 4, 5, 6}, {0, 2, 4, 1, 6, 3, 5}, {0, 3, 1, 5, 2, 6, 4}};
    case 8: return {{0, 1, 2, 3, 4, 5, 6, 7}, {0, 2, 4, 1, 5, 7, 3, 6}, {0, 3, 1, 6, 4, 7, 2, 5}};
    default: {
      std::vector<int> c(n);
      for (int i = 0; i < n; ++i) c[i] = i;
      return {c};
    }
  }
}

// Directed rings: each cycle forward and reversed (n >= 3); n = 2 has one.
inline std::vector<std::vector<int>> directed_rings(int n, int max_rings) {
  std::vector<std::vector<int>> out;
  for (const auto& c : hamiltonian_cycles(n)) {
    out.push_back(c);
    if (n >= 3) {
      std::vector<int> r(c.rbegin(), c.rend());
      out.push_back(r);
    }
  }
  if (max_rings > 0 && (int)out.size() > max_rings) out.resize(max_rings);
  return out;
}

// Steps of the all-reduce for `rank`: each inner vector is one ncclGroup.
// count/align/chunk in elements; align divides every slice and segment start.
inline std::vector<std::vector<RingXfer>> ring_schedule(int n, int rank, int64_t count,
                                                        int64_t align, int64_t chunk,
                                                        int max_rings) {
  std::vector<std::vector<RingXfer>> steps;
  if (n < 2 || count <= 0) return steps;
  if (align < 1) align = 1;
  const auto rings = directed_rings(n, max_rings);
  const int R = (int)rings.size();
  auto up = [align](int64_t x) { return (x + align - 1) / align * align; };
  // slice k = [so[k], so[k+1]); segment j of slice k = [so[k] + off(j), ...)
  std::vector<int64_t> so(R + 1);
  const int64_t sl = up((count + R - 1) / R);
  for (int k = 0; k <= R; ++k) so[k] = std::min<int64_t>((int64_t)k * sl, count);
  auto seg = [&](int k, int j, int64_t* o, int64_t* len) {
    const int64_t len_k = so[k + 1] - so[k];
    const int64_t sg = up((len_k + n - 1) / n);
    const int64_t a = std::min<int64_t>((int64_t)j * sg, len_k);
    const int64_t b = std::min<int64_t>((int64_t)(j + 1) * sg, len_k);
    *o = so[k] + a;
    *len = b - a;
  };
  if (chunk <= 0) chunk = count;
  chunk = std::max<int64_t>(align, chunk / align * align);
  std::vector<int> pos(R), nxt(R), prv(R);
  for (int k = 0; k < R; ++k) {
    const auto& rg = rings[k];
    const int p = (int)(std::find(rg.begin(), rg.end(), rank) - rg.begin());
    if (p >= n) throw std::logic_error("rank missing from ring");
    pos[k] = p;
    nxt[k] = rg[(p + 1) % n];
    prv[k] = rg[(p + n - 1) % n];
  }
  auto mod = [n](int x) { return ((x % n) + n) % n; };
  for (int phase = 0; phase < 2; ++phase) {
    for (int st = 0; st < n - 1; ++st) {
      // segments per ring for this step, then split into chunk rounds
      std::vector<int64_t> s_off(R), s_len(R), r_off(R), r_len(R);
      int64_t rounds = 1;
      for (int k = 0; k < R; ++k) {
        const int si = phase == 0 ? mod(pos[k] - st) : mod(pos[k] + 1 - st);
        const int ri = phase == 0 ? mod(pos[k] - st - 1) : mod(pos[k] - st);
        seg(k, si, &s_off[k], &s_len[k]);
        seg(k, ri, &r_off[k], &r_len[k]);
        const int64_t m = std::max(s_len[k], r_len[k]);
        rounds = std::max<int64_t>(rounds, (m + chunk - 1) / chunk);
      }
      for (int64_t c = 0; c < rounds; ++c) {
        std::vector<RingXfer> g;
        for (int k = 0; k < R; ++k) {
          const int64_t o = c * chunk;
          const int64_t sn = std::max<int64_t>(0, std::min(chunk, s_len[k] - o));
          const int64_t rn = std::max<int64_t>(0, std::min(chunk, r_len[k] - o));
          if (sn == 0 && rn == 0) continue;
          g.push_back(RingXfer{k, sn ? nxt[k] : -1, s_off[k] + o, sn, rn ? prv[k] : -1,
                               r_off[k] + o, rn, phase == 0, st, (int)c});
        }
        if (!g.empty()) steps.push_back(std::move(g));
      }
    }
  }
  return steps;
}

// Pipelined execution of a schedule on two streams: the transfers (one
// ncclGroup per entry, comm stream) and the reduce-scatter's reduces (one
// launch per group, reduce stream), so chunk c's reduce overlaps chunk c+1's
// transfer.  Per group i:
//   wait_reduce: the group whose REDUCE must have finished before i's sends
//     (a reduce-scatter step sends what the previous step reduced; the first
//     all-gather step sends what the last reduce-scatter step reduced), -1 none;
//   slot: scratch slot (0 / 1, double buffered per ring) i's receives land in;
//   slot_free: the group whose reduce last read that slot, -1 none.
// Reduces run in issue order on their stream, so waiting for a later group's
// reduce also covers every earlier one.  Pure index arithmetic: simulated on
// the CPU against adversarial stream timings (tests/test_ring_plan.py).
struct RingDeps {
  int wait_reduce = -1;
  int slot = 0;
  int slot_free = -1;
};
inline std::vector<RingDeps> ring_pipeline(const std::vector<std::vector<RingXfer>>& plan) {
  const int G = (int)plan.size();
  std::vector<RingDeps> out(G);
  // (phase, step) -> group index of each round
  std::vector<std::vector<int>> rs, ag;
  for (int i = 0; i < G; ++i) {
    if (plan[i].empty()) continue;
    const RingXfer& x = plan[i][0];
    auto& tab = x.reduce ? rs : ag;
    if ((int)tab.size() <= x.step) tab.resize(x.step + 1);
    tab[x.step].push_back(i);
  }
  auto pick = [](const std::vector<int>& rounds, int c) {
    return rounds.empty() ? -1 : rounds[std::min<int>(c, (int)rounds.size() - 1)];
  };
  int last[2] = {-1, -1};
  int nred = 0;
  for (int i = 0; i < G; ++i) {
    if (plan[i].empty()) continue;
    const RingXfer& x = plan[i][0];
    if (x.reduce) {
      if (x.step > 0) out[i].wait_reduce = pick(rs[x.step - 1], x.round);
      out[i].slot = nred & 1;
      out[i].slot_free = last[nred & 1];
      last[nred & 1] = i;
      ++nred;
    } else if (x.step == 0 && !rs.empty()) {
      out[i].wait_reduce = pick(rs.back(), x.round);
    }
  }
  return out;
}

}  // namespace dsml
