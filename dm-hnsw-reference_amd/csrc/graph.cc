// Dump parsing: the load half of the HBM shard manager.
//
// Replaces MemoryNode::store_or_load_index (src/memory_node.hh:130-209), which reads
// `index_m{M}_efc{efC}_node{i}_of{N}.dat` verbatim into the memory node's buffer, and the RemotePtr
// addressing every later rdma::read_* uses (src/remote_pointer.hh:7-29).  Instead of keeping 64-bit
// RemotePtrs (memory node | byte offset) in HBM, records are walked once and every list entry is translated to
// a dense u32 node index, so the device layout is index-addressed and the 8-byte, 4-mod-8-misaligned list
// entries of the reference layout (node.hh:17) become aligned 4-byte ones.
#include "graph.h"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <mutex>
#include <thread>

namespace shine {

namespace {
thread_local std::string g_last_error;

template <class T>
T load(const u8* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

template <class F>
void parallel_for(u64 n, u32 threads, F&& f) {
  if (threads == 0) threads = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
  if (n < 4096 || threads == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const u64 chunk = (n + threads - 1) / threads;
  for (u32 t = 0; t < threads; ++t) {
    const u64 lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo >= hi) break;
    ts.emplace_back([&f, lo, hi]() { f(lo, hi); });
  }
  for (auto& t : ts) t.join();
}
}  // namespace

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
const char* last_error() { return g_last_error.c_str(); }

int read_file(const std::string& path, std::vector<u8>& out) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f.good()) return set_error(2, "file \"" + path + "\" does not exist");  // memory_node.hh:161-164
  const std::streamsize n = f.tellg();
  f.seekg(0, std::ios::beg);
  out.resize(static_cast<size_t>(n));
  if (n > 0 && !f.read(reinterpret_cast<char*>(out.data()), n)) return set_error(2, "cannot read \"" + path + "\"");
  return 0;
}

int parse_dumps(const u8* const* bufs, const u64* sizes, u32 n, u32 dim, u32 M, int metric, u32 threads,
                HostGraph& G) {
  if (n == 0 || n > 65535) return set_error(1, "number of dumps must be in [1, 65535]");
  if (dim == 0 || dim > 4096) return set_error(1, "dim must be in [1, 4096]");
  if (M == 0 || M > 32) return set_error(1, "M must be in [1, 32] (level-0 lists hold 2M <= 64 entries)");
  G = HostGraph{};
  G.L.dim = dim;
  G.L.M = M;
  G.metric = metric;
  G.n_shards = n;
  const RecordLayout& L = G.L;
  const u32 M0 = 2 * M;

  // pass 1: walk the records of every memory node; offsets are increasing within a shard
  std::vector<std::vector<u64>> offs(n);
  std::vector<u64> start(n + 1, 0);
  for (u32 s = 0; s < n; ++s) {
    if (sizes[s] < 16) return set_error(3, "dump " + std::to_string(s + 1) + " is shorter than its 16-byte header");
    const u64 free_ptr = load<u64>(bufs[s]);  // memory_node.hh:61 — first free byte
    if (free_ptr < 16 || free_ptr > sizes[s])
      return set_error(3, "dump " + std::to_string(s + 1) + ": free_ptr " + std::to_string(free_ptr) +
                              " outside the file (" + std::to_string(sizes[s]) + " bytes)");
    u64 off = 16;
    while (off < free_ptr) {
      if (off + 16 > free_ptr) return set_error(3, "truncated record header in dump " + std::to_string(s + 1));
      const u32 level = load<u32>(bufs[s] + off + 12);
      if (level > 64) return set_error(3, "implausible level " + std::to_string(level) + " at offset " + std::to_string(off));
      const u64 rs = L.alloc_size(level);
      if (off + rs > free_ptr) return set_error(3, "record at offset " + std::to_string(off) + " runs past free_ptr");
      offs[s].push_back(off);
      off += rs;
    }
    start[s + 1] = start[s] + offs[s].size();
  }
  const u64 N = start[n];
  if (N == 0) return set_error(3, "the dumps hold no records");
  if (N >= kInvalid) return set_error(3, "more than 2^32-1 records");
  G.N = N;
  G.shard_start = start;

  auto translate = [&](u64 rp, u32& out) -> bool {  // RemotePtr → dense id (remote_pointer.hh:19-20)
    const u32 s = static_cast<u32>(rp >> 48);
    const u64 off = (rp << 16) >> 16;
    if (s >= n) return false;
    const auto& v = offs[s];
    auto it = std::lower_bound(v.begin(), v.end(), off);
    if (it == v.end() || *it != off) return false;
    out = static_cast<u32>(start[s] + (it - v.begin()));
    return true;
  };

  // entry point: node1's bytes 8..15 (rdma_reads.hh:74-99)
  const u64 ep_ptr = load<u64>(bufs[0] + 8);
  if (ep_ptr == 0) return set_error(3, "entry-point pointer is null: the index was never initialised");
  if (!translate(ep_ptr, G.ep)) return set_error(3, "entry-point pointer does not name a record");

  G.vec.resize(N * dim);
  G.uid.resize(N);
  G.level.resize(N);
  G.up_base.assign(N, kInvalid);
  G.adj0.assign(N * M0, kInvalid);

  // upper-level row allocation (prefix sum over levels, in dense order)
  u64 rows = 0;
  for (u32 s = 0; s < n; ++s)
    for (u64 i = 0; i < offs[s].size(); ++i) {
      const u64 g = start[s] + i;
      const u32 lv = load<u32>(bufs[s] + offs[s][i] + 12);
      G.level[g] = lv;
      if (lv > 0) {
        G.up_base[g] = static_cast<u32>(rows);
        rows += lv;
      }
    }
  if (rows >= kInvalid) return set_error(3, "too many upper-level lists");
  G.adjU.assign(rows * M, kInvalid);
  G.ep_level = G.level[G.ep];

  std::mutex err_mu;
  int err = 0;
  std::string err_msg;
  bool dup_any = false;
  // pass 2 (parallel over dense ids): copy components and translate lists
  parallel_for(N, threads, [&](u64 lo, u64 hi) {
    bool dup_local = false;
    for (u64 g = lo; g < hi; ++g) {
      const u32 s = static_cast<u32>(std::upper_bound(start.begin(), start.end(), g) - start.begin() - 1);
      const u64 off = offs[s][g - start[s]];
      const u8* rec = bufs[s] + off;
      G.uid[g] = load<u32>(rec + 8);
      std::memcpy(&G.vec[g * dim], rec + 16, 4ull * dim);
      const u32 lv = G.level[g];
      for (u32 l = 0; l <= lv; ++l) {
        const u8* lst = bufs[s] + L.list_offset(off, l);
        const u32 cnt = load<u32>(lst);
        const u32 cap = l == 0 ? M0 : M;
        u32* dst = l == 0 ? &G.adj0[g * M0] : &G.adjU[(static_cast<u64>(G.up_base[g]) + l - 1) * M];
        if (cnt > cap) {
          std::lock_guard<std::mutex> lk(err_mu);
          err = 3;
          err_msg = "neighbour list with " + std::to_string(cnt) + " > " + std::to_string(cap) + " entries";
          return;
        }
        for (u32 j = 0; j < cnt; ++j) {
          u32 d;
          if (!translate(load<u64>(lst + 4 + 8ull * j), d)) {
            std::lock_guard<std::mutex> lk(err_mu);
            err = 3;
            err_msg = "dangling RemotePtr in the neighbour list of uid " + std::to_string(G.uid[g]);
            return;
          }
          dst[j] = d;
        }
        for (u32 j = 1; j < cnt && !dup_local; ++j)
          for (u32 i = 0; i < j; ++i)
            if (dst[i] == dst[j]) { dup_local = true; break; }
      }
    }
    if (dup_local) {
      std::lock_guard<std::mutex> lk(err_mu);
      dup_any = true;
    }
  });
  if (err) return set_error(err, err_msg);
  G.lists_unique = !dup_any;
  return 0;
}

// Reachability of the parsed graph from the entry point (diagnostic for shine_graph_stats).  A level-0 search
// starts at the node the greedy descent ends on (hnsw.hh:279-294) and follows level-0 lists only
// (hnsw.hh:436-438), so a record no level-0 path from the entry point reaches can never be returned.
GraphReach graph_reach(const HostGraph& G) {
  GraphReach r;
  const u32 M0 = 2 * G.L.M, MU = G.L.M;
  r.num_nodes = G.N;
  std::vector<u8> seen(G.N, 0);
  std::vector<u32> stack;
  auto bfs = [&](bool all_levels) {
    std::fill(seen.begin(), seen.end(), 0);
    stack.assign(1, G.ep);
    seen[G.ep] = 1;
    u64 cnt = 1;
    while (!stack.empty()) {
      const u32 g = stack.back();
      stack.pop_back();
      auto visit = [&](u32 x) {
        if (x != kInvalid && !seen[x]) {
          seen[x] = 1;
          ++cnt;
          stack.push_back(x);
        }
      };
      for (u32 j = 0; j < M0; ++j) visit(G.adj0[static_cast<u64>(g) * M0 + j]);
      if (all_levels)
        for (u32 l = 1; l <= G.level[g]; ++l)
          for (u32 j = 0; j < MU; ++j) visit(G.adjU[(static_cast<u64>(G.up_base[g]) + l - 1) * MU + j]);
    }
    return cnt;
  };
  r.reachable_l0 = bfs(false);
  r.reachable_any = bfs(true);
  std::vector<u32> indeg(G.N, 0);
  u64 edges = 0;
  for (u64 g = 0; g < G.N; ++g) {
    u32 c = 0;
    for (u32 j = 0; j < M0; ++j) {
      const u32 x = G.adj0[g * M0 + j];
      if (x == kInvalid) continue;
      ++c;
      ++indeg[x];
    }
    edges += c;
    if (c == M0) ++r.full_lists_l0;
  }
  for (u64 g = 0; g < G.N; ++g)
    if (indeg[g] == 0 && g != G.ep) ++r.zero_indegree_l0;
  r.mean_degree_l0 = G.N ? static_cast<double>(edges) / static_cast<double>(G.N) : 0.0;
  r.max_level = G.ep_level;
  return r;
}

}  // namespace shine
