// CPU check of zipkin_amd/csrc/zdl_xplan.h (the multi-GPU combines' host bookkeeping) against
// simulated ranks: compiled and run by tests/test_xplan.py. Prints "ok" or the first failure.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#include "../zipkin_amd/csrc/zdl_xplan.h"

using namespace zdl_xplan;

#define CHECK(x)                                                   \
  do {                                                             \
    if (!(x)) {                                                    \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #x);     \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

struct Entry {
  uint32_t cell;
  uint64_t call, err;
};

// Sparse lists: W ranks' sorted (cell, call, err) lists gathered by the plan into every
// receiver's buffer (memcpy for each transfer, a local copy for a rank's own list), then
// summed per cell: equals the sum of all lists, and every receiver holds the rank-order
// concatenation. The sends a rank posts match the receives posted for it (same count), which
// NCCL's grouped point-to-point calls require.
static void check_sparse(std::mt19937_64& r, int W, bool all) {
  std::vector<std::vector<Entry>> lists(W);
  std::vector<uint64_t> n(W);
  for (int k = 0; k < W; ++k) {
    const int len = (r() % 4 == 0) ? 0 : (int)(r() % 200);  // some ranks have nothing
    std::map<uint32_t, Entry> m;
    for (int i = 0; i < len; ++i) {
      const uint32_t cell = (uint32_t)(r() % 500);
      auto& e = m[cell];
      e.cell = cell;
      e.call += 1 + r() % 5;
      e.err += r() % 2;
    }
    for (auto& kv : m) lists[k].push_back(kv.second);
    n[k] = lists[k].size();
  }
  const Plan p = gather_plan(n.data(), W, all);
  CHECK((int)p.at.size() == W + 1 && p.at[0] == 0);
  uint64_t tot = 0;
  for (int k = 0; k < W; ++k) {
    CHECK(p.at[k] == tot);
    tot += n[k];
  }
  CHECK(p.total() == tot);
  std::vector<std::vector<Entry>> buf(W, std::vector<Entry>(tot, Entry{~0u, 0, 0}));
  std::vector<std::vector<int>> sent(W, std::vector<int>(W, 0)), recvd(W, std::vector<int>(W, 0));
  for (const Xfer& x : p.ops) {
    CHECK(x.n > 0 && x.n == n[x.src] && x.at == p.at[x.src]);
    CHECK(all || x.dst == 0);
    sent[x.src][x.dst] += 1;
    recvd[x.dst][x.src] += 1;
    std::copy(lists[x.src].begin(), lists[x.src].end(), buf[x.dst].begin() + x.at);
  }
  for (int a = 0; a < W; ++a)
    for (int b = 0; b < W; ++b) {
      CHECK(sent[a][b] == recvd[b][a]);
      CHECK(sent[a][b] == ((all || b == 0) && n[a] ? 1 : 0));
    }
  std::map<uint32_t, std::pair<uint64_t, uint64_t>> want;
  for (auto& l : lists)
    for (auto& e : l) {
      want[e.cell].first += e.call;
      want[e.cell].second += e.err;
    }
  for (int d = 0; d < W; ++d) {
    if (!all && d != 0) continue;
    uint64_t at = 0;
    for (int k = 0; k < W; ++k)
      for (auto& e : lists[k]) {
        CHECK(buf[d][at].cell == e.cell && buf[d][at].call == e.call && buf[d][at].err == e.err);
        ++at;
      }
    std::map<uint32_t, std::pair<uint64_t, uint64_t>> got;
    for (auto& e : buf[d]) {
      got[e.cell].first += e.call;
      got[e.cell].second += e.err;
    }
    CHECK(got == want);
  }
}

// A job's sparse reduce-scatter (comm_sum_sparse): each rank samples its sorted list, every rank
// derives the same range bounds (range_split), cuts its list into W slices by lower bound, the
// W x W slice lengths give every rank its slice_plan; the plans' sends and receives agree, the
// slices land where the receivers expect them, each rank's received runs summed per cell lie in
// its range, and the reduced ranges concatenated in rank order are the job's list: sorted, each
// cell once, with the summed counts.
static void check_reduce_scatter(std::mt19937_64& r, int W) {
  const uint32_t q = SPLIT_SAMPLES;
  const uint32_t span = 1 + (uint32_t)(r() % 3 == 0 ? 3 : (r() % 2 ? 500 : 4000000000u));
  std::vector<std::vector<Entry>> lists(W);
  for (int k = 0; k < W; ++k) {
    const int len = (r() % 4 == 0) ? 0 : (int)(r() % 300);
    std::map<uint32_t, Entry> m;
    for (int i = 0; i < len; ++i) {
      // skewed cells (a Zipf-like head), some shared by every rank
      const uint32_t cell = (r() % 3 == 0) ? (uint32_t)(r() % 4) : (uint32_t)(r() % span);
      auto& e = m[cell];
      e.cell = cell;
      e.call += 1 + r() % 5;
      e.err += r() % 2;
    }
    for (auto& kv : m) lists[k].push_back(kv.second);
  }
  std::vector<uint64_t> meta((size_t)W * (1 + q));
  for (int k = 0; k < W; ++k) {
    const uint64_t n = lists[k].size();
    meta[(size_t)k * (1 + q)] = n;
    for (uint32_t i = 0; i < q; ++i)  // k_x_samples
      meta[(size_t)k * (1 + q) + 1 + i] = n ? lists[k][((2 * (uint64_t)i + 1) * n) / (2 * (uint64_t)q)].cell : 0;
  }
  const std::vector<uint64_t> b = range_split(meta.data(), W, q);
  CHECK((int)b.size() == W + 1 && b[0] == 0 && b[W] == (1ull << 32));
  for (int k = 0; k < W; ++k) CHECK(b[k] <= b[k + 1]);
  std::vector<uint64_t> cnt((size_t)W * W);
  for (int k = 0; k < W; ++k)  // k_x_slices
    for (int j = 0; j < W; ++j) {
      auto lb = [&](uint64_t v) {
        return (uint64_t)(std::lower_bound(lists[k].begin(), lists[k].end(), v,
                                           [](const Entry& e, uint64_t x) { return (uint64_t)e.cell < x; }) -
                          lists[k].begin());
      };
      cnt[(size_t)k * W + j] = lb(b[j + 1]) - lb(b[j]);
    }
  std::vector<Plan> plans;
  for (int me = 0; me < W; ++me) plans.push_back(slice_plan(cnt.data(), W, me));
  std::vector<std::vector<Entry>> buf(W);
  for (int me = 0; me < W; ++me) buf[me].assign(plans[me].total(), Entry{~0u, 0, 0});
  for (int me = 0; me < W; ++me)
    for (const Xfer& x : plans[me].ops) {
      CHECK(x.n > 0 && (x.src == me || x.dst == me));
      if (x.src != me) {  // a receive: the sender's plan holds the same transfer
        bool found = false;
        for (const Xfer& y : plans[x.src].ops)
          if (y.src == x.src && y.dst == me) {
            CHECK(!found && y.n == x.n && y.at == x.at && y.from == x.from);
            found = true;
          }
        CHECK(found);
        continue;
      }
      CHECK(x.from + x.n <= lists[me].size() && x.at + x.n <= buf[x.dst].size());
      std::copy(lists[me].begin() + x.from, lists[me].begin() + x.from + x.n, buf[x.dst].begin() + x.at);
    }
  std::map<uint32_t, std::pair<uint64_t, uint64_t>> want;
  for (auto& l : lists)
    for (auto& e : l) {
      want[e.cell].first += e.call;
      want[e.cell].second += e.err;
    }
  std::vector<Entry> job;
  for (int me = 0; me < W; ++me) {
    std::map<uint32_t, Entry> red;  // sparse_add
    for (auto& e : buf[me]) {
      CHECK(e.cell != ~0u && e.cell >= b[me] && e.cell < b[me + 1]);
      auto& x = red[e.cell];
      x.cell = e.cell;
      x.call += e.call;
      x.err += e.err;
    }
    for (auto& kv : red) job.push_back(kv.second);
  }
  CHECK(job.size() == want.size());
  size_t i = 0;
  for (auto& kv : want) {
    CHECK(job[i].cell == kv.first && job[i].call == kv.second.first && job[i].err == kv.second.second);
    ++i;
  }
}

// Insertion order: each rank's first-seen ranks tagged by ord_tag, the element-wise MIN over
// the ranks, then sorting the non-empty cells by it gives DependencyLinker.merge's order over
// the ranks' link() lists concatenated in rank order.
static void check_ord(std::mt19937_64& r, int W) {
  const uint32_t S = 7;
  std::vector<std::vector<uint64_t>> first(W, std::vector<uint64_t>(S * S, ~0ull));
  std::vector<std::vector<uint32_t>> lists(W);  // each rank's link() order: cells by first rank
  for (int k = 0; k < W; ++k) {
    std::vector<std::pair<uint64_t, uint32_t>> v;
    for (uint32_t c = 0; c < S * S; ++c)
      if (r() % 3 == 0) {
        const uint64_t pos = r() % ORD_POS_LIMIT, bfs = r() % 1000, kk = r() % 2;
        first[k][c] = ((pos + bfs) << 1) | kk;  // ord_rank's layout
        v.push_back({first[k][c], c});
      }
    std::sort(v.begin(), v.end());
    for (auto& e : v) lists[k].push_back(e.second);
  }
  std::vector<uint64_t> red(S * S, ~0ull);
  for (int k = 0; k < W; ++k)
    for (uint32_t c = 0; c < S * S; ++c) red[c] = std::min(red[c], ord_tag(first[k][c], k));
  std::vector<std::pair<uint64_t, uint32_t>> v;
  for (uint32_t c = 0; c < S * S; ++c)
    if (red[c] != ~0ull) v.push_back({red[c], c});
  std::sort(v.begin(), v.end());
  std::vector<uint32_t> want;  // merge(): first-seen over the concatenation
  std::vector<bool> seen(S * S, false);
  for (int k = 0; k < W; ++k)
    for (uint32_t c : lists[k])
      if (!seen[c]) {
        seen[c] = true;
        want.push_back(c);
      }
  CHECK(v.size() == want.size());
  for (size_t i = 0; i < v.size(); ++i) CHECK(v[i].second == want[i]);
  CHECK(ord_tag(~0ull, W - 1) == ~0ull);
}

int main() {
  std::mt19937_64 r(12345);
  for (int it = 0; it < 300; ++it) {
    const int W = 1 + (int)(r() % 8);
    check_sparse(r, W, true);
    check_sparse(r, W, false);
    check_ord(r, W);
    check_reduce_scatter(r, W);
  }
  for (int W : {16, 64}) check_reduce_scatter(r, W);
  check_ord(r, ORD_MAX_WORLD);
  std::printf("ok\n");
  return 0;
}
