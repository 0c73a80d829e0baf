// Host-side index model: the reference's dump records (src/memory_node.hh:15-27, src/node/node.hh:10-19)
// re-laid out for HBM as dense, index-addressed arrays.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace shine {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using f32 = float;

constexpr u32 kInvalid = 0xFFFFFFFFu;

// Status propagation: every fallible function returns an int (SHINE_OK / SHINE_ERR_*) and records a
// message for shine_last_error() — the reference's lib_assert/exit(1) (utils.hh:17-23) becomes a status.
int set_error(int code, const std::string& msg);
const char* last_error();

// Reference record geometry (node.hh:44-54, rdma_atomics.hh:90-95).
struct RecordLayout {
  u32 dim = 0, M = 0;
  u64 size_until_components() const { return 16 + 4ull * dim; }
  u64 list0_size() const { return 4 + 8ull * 2 * M; }
  u64 listU_size() const { return 4 + 8ull * M; }
  u64 total_size(u32 level) const { return size_until_components() + list0_size() + level * listU_size(); }
  u64 alloc_size(u32 level) const {
    u64 s = total_size(level);
    while (s % 8 != 0) s += 4;
    return s;
  }
  u64 list_offset(u64 node_off, u32 lvl) const {  // node.cc:18-27
    u64 o = node_off + size_until_components();
    if (lvl > 0) o += list0_size() + (lvl - 1) * listU_size();
    return o;
  }
};

// Dense graph.  Node g (0..N-1) is the g-th record in dump order (node1's records first).
//   vec    [N][dim] f32                 components
//   adj0   [N][2M]  u32                 level-0 neighbour dense ids, list order kept, kInvalid padding
//   uid    [N]      u32                 the record's uid (query results are uids, hnsw.hh:302)
//   up_base[N]      u32                 row of the node's level-1 list in adjU (level l: up_base + l - 1)
//   adjU   [R][M]   u32                 upper-level lists, kInvalid padding
struct HostGraph {
  RecordLayout L;
  int metric = 0;
  u64 N = 0;
  std::vector<f32> vec;
  std::vector<u32> adj0, uid, up_base, adjU, level;
  u32 ep = kInvalid, ep_level = 0;
  bool lists_unique = true;  // no list holds the same neighbour twice (lets the kernel skip in-list dedup)
  u32 n_shards = 0;
  std::vector<u64> shard_start;  // [n_shards + 1]: dense ids of memory node s are shard_start[s] .. shard_start[s+1]-1
  u64 bytes_reference_node() const { return L.size_until_components(); }
};

// Parse dump images (one per memory node, in node1..nodeN order) into a HostGraph.  `threads` = 0 → auto.
int parse_dumps(const u8* const* bufs, const u64* sizes, u32 n, u32 dim, u32 M, int metric, u32 threads,
                HostGraph& out);

int read_file(const std::string& path, std::vector<u8>& out);

struct GraphReach {
  u64 num_nodes = 0, reachable_l0 = 0, reachable_any = 0, zero_indegree_l0 = 0, full_lists_l0 = 0;
  double mean_degree_l0 = 0;
  u32 max_level = 0;
};
GraphReach graph_reach(const HostGraph& G);

}  // namespace shine
