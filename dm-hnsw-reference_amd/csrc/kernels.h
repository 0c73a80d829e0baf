// Device-side argument blocks and host launchers for the gfx950 kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace shine {

struct DevGraph {
  const void* vec;        // [N][dim] f32 or f16
  const uint32_t* adj0;   // [N][M0]
  const uint32_t* uid;    // [N]
  const uint32_t* up_base;// [N]
  const uint32_t* adjU;   // [R][MU]
  const uint32_t* inv_uid;// [inv_size] uid → dense id (distance-batch API)
  uint32_t inv_size;
  uint32_t N, M0, MU, ep, ep_level, lists_unique;
  uint32_t pad_node;      // a node local to this GPU: unconditional loads of empty list slots read it
  // Sharded placements: where a device id's record lives, for the per-query read accounting (qstats words 8-11,
  // the rdma_reads_in_bytes analogue, rdma_reads.hh:12,46).  Id x belongs to stripe x / stripe_ids (computed as
  // umulhi(x, div_magic) >> div_shift, exact for x < 2^31); it is local when the stripe is `slot`, a cached copy
  // when x % stripe_ids < cached_rows, otherwise an xGMI read.  sharded = 0: every read is local (replica).
  uint32_t sharded, slot, stripe_ids, cached_rows, div_magic, div_shift;
  uint32_t cached_list_rows;  // lists of rows x % stripe_ids < cached_list_rows are cached (the arrays' cached
                              // prefixes are whole VM pages of each array, so the two row counts differ)
  // Dynamic record cache (SHINE_CACHE_DYNAMIC, the reference's cache::Cache, cache.hh:102-311): this GPU's arena of
  // record vectors, fixed during a call and updated between calls by the host's admission / eviction engine.
  // Kernels built with ACCT = 2 look every off-stripe vector read up in cslot: a hit reads the local arena row and
  // offers a cooling entry its second chance (cache.hh:128-132: the device id goes to rlog), a miss reads over xGMI
  // and is offered for admission through clog (entry point and upper levels always, level-0 reads while the cache is
  // not full or when their coin passes, hnsw.hh:447-448).
  const uint32_t* cslot;      // [id space]: arena slot of device id x with the entry's cooling flag in bit 31, or
                              // 0xFFFFFFFF (the flag travels with the slot: one dependent read for both)
  const uint32_t* cbits;      // [id space / 32]: bit x set while x is cached — read before cslot, so that a miss
                              // (most off-stripe reads) costs one read of a bitmap 1/32 of cslot's size, which stays
                              // in the caches, instead of a cslot read from HBM ahead of its xGMI read
  const void* cvec;           // [arena slots][row]: cached vectors, device row layout
  uint32_t* cool;             // [arena slots]: 1 while the entry is cooling (the host's copy; kernels read cslot's bit)
  unsigned long long* clog;   // admission candidates: (query << 32) | x | always << 31 | coin << 63
  uint32_t* clog_n;           // [0] candidates logged (may exceed clog_cap: the overflow is counted, not stored);
                              // [1] hits on cooling entries logged
  uint32_t* rlog;             // device ids of the hits on cooling entries, each arena slot once per log epoch
  uint32_t* rlogged;          // [arena slots]: the log epoch in which the slot's hit was logged (reset when it is filled)
  uint32_t clog_cap, rlog_cap;
  uint32_t dyn_epoch;         // log epoch: the logs' contents since the host last fetched and zeroed them
  uint32_t dyn_full;          // the cache was full when the call started: level-0 misses draw the coin
  uint32_t dyn_call;          // call counter (coin input)
  unsigned long long dyn_seed;
};

// Counter words of one call on a stream (SearchArgs::call_counters).
constexpr uint32_t kCallWords = 11;

// Per-query counter words (u32) written by the search kernels; include/shine_gpu.h SHINE_QS_*.
constexpr uint32_t kQsWords = 12;

struct SearchArgs {
  DevGraph g;
  const float* queries;   // [nq_total][dim]
  uint32_t nq;            // work items
  uint32_t k, ef, cap;    // cap: next_candidates capacity held in LDS
  uint32_t vis_cap;       // LDS visited hash-table entries (power of two; 0 = global bitmap variant)
  uint32_t vis_limit;     // entries allowed in the LDS table before the query is re-run with more LDS
  uint32_t* out_ids;      // [nq_total][k]
  float* out_dists;       // [nq_total][k] (nullable)
  uint32_t* qstats;       // [nq_total][kQsWords] (nullable)
  uint32_t* visited;      // [slots][words_per_slot] bitmaps, all-zero between queries
  uint64_t words_per_slot;
  uint32_t* vlog;         // [slots][log_cap] ids whose visited bit is set (for clearing)
  uint32_t log_cap;
  uint32_t* counter;      // work queue head (zeroed before every launch)
  const uint32_t* in_list;   // fixup passes: work items are in_list[0 .. *in_count)
  const uint32_t* in_count;
  uint32_t* out_list;        // queries that overflow here are appended for the next pass (nullable)
  uint32_t* out_count;
  unsigned long long* heaps; // global-heap pass: per-slot top / next heaps in HBM, heap_stride entries each
  uint64_t heap_stride;
  uint32_t* access;          // cache warmup (nullable): per device id, reads of the record (vector or list)
  uint32_t* call_counters;   // last pass of a call (nullable): the call's kCallWords counter words; the last workgroup
  uint32_t* host_counts;     // to finish copies words 4..6 to host_counts[0..2] (host memory), sets host_counts[3] = 1,
                             // copies words 3 and 8 to host_counts[4] and [5], the call's nq to [6], words 9 and 10 to
                             // [7] and [8], and zeroes the words for the next call
                             // on the stream (word 7 counts finished groups)
  uint32_t* call_out;        // last pass (nullable): call_out[0] = the queries the call's passes handed on (words 4..6
                             // summed), call_out[1] = 1 — a per-call copy (host_counts is the stream's, and a later call
                             // on the stream may overwrite it before the host reads it)
  uint32_t* vis_max;         // every pass (nullable): the call's counter word 3, the most nodes any query marked
                             // visited (atomicMax per query) — sizes the next call's visited tables
  uint32_t* next_max;        // exact passes (nullable): the call's counter word 10, the most next_candidates entries
                             // any query held (atomicMax per query; past the capacity: capacity + 1) — sizes the next
                             // call's reservation for them (capi.cc pick_shape)
  uint32_t* vis_sum;         // every pass (nullable): the call's counter word 8, the nodes its queries marked visited
                             // (atomicAdd per query; copied to host_counts[5]) — the mean sizes spilling tables
  unsigned long long* prof; // diagnostics (nullable): per-phase shader-clock totals, PROF kernel variant only
  uint32_t fast;            // 1: sorted-list kernel (SHINE_MODE_FAST; ef <= kFastMaxEf, vis_cap > 0)
  uint32_t sort_out;        // heap kernel writes ascending order (fast-mode fixup passes)
  uint32_t global_heaps;    // 1: heap kernel with both heaps in HBM (last fallback pass; vis_cap must be 0)
  uint32_t vis16;           // LDS visited table kind (kernels_impl.h VisitedLds<vis16>): 0 u32 linear probing, 1 u16
                            // quotient entries, 2 u16 two-choice buckets, 3 u32 two-choice buckets (replicas only)
  uint32_t vis_bits;        // ... bits of the id space the multiply permutes (vis_bits - log2(vis_cap) <= 10: buckets of 8, >= 3 distance bits)
  uint32_t vis_mul;         // ... odd multiplier
  uint32_t vis_mul_inv;     // ... its inverse mod 2^32 (decodes an entry back to its id when a table spills)
  // Fast kernel: a query that outgrows its LDS visited table spills it in place into one of spill_slots HBM bitmaps
  // (the `visited` bitmaps of the stream's fallback passes, words_per_slot words each, all zero between uses) and
  // goes on with its visited set there; spill_flags[i] = 1 while bitmap i is held.  spill_slots = 0: no spilling
  // (the query is handed on to the next pass instead).
  uint32_t* spill_flags;
  uint32_t spill_slots;
  uint32_t* spill_count;     // main pass (nullable): the call's counter word 9, queries that spilled (copied to
                             // host_counts[7]): a learned table that spills too often is grown (capi.cc)
  uint32_t spill_hash;       // 0: a spilled table goes to its slot as a bitmap over the id space; else to a hash table
                             // of spill_hash entries (a power of two <= words_per_slot) in the slot (kernels_impl.h
                             // SpillSet), where the id-space bitmap would outgrow an XCD's L2
};

struct DistArgs {
  DevGraph g;
  const float* queries;
  uint32_t nq;
  const uint32_t* node_uids;  // [nq][n_per]
  uint32_t n_per;
  float* out;                 // [nq][n_per]
};

// GPU batch builder (build_impl.h kernels, gpu_build.cc host side).  One batch = node ids batch_start ..
// batch_start + n_lists0 - 1 inserted against the graph as it stood before the batch.
struct BuildArgs {
  DevGraph g;                 // the graph being built: f32 rows (device layout), lists, ep / ep_level before the batch
  uint32_t* adj0w;            // writable views of g.adj0 / g.adjU
  uint32_t* adjUw;
  const float* base;          // the caller's rows, unpermuted [N][dim] (the batch's nodes as queries)
  uint32_t ef, M;             // ef_construction; neighbours a new node selects (select_heuristic(top, M), hnsw.hh:157)
  // candidate lists, ef entries each, ascending, INV-padded: rows 0 .. n_lists0-1 level 0 of the batch's nodes (the
  // fast search kernel's output), then n_listsU upper-level lists (build_upper_kernel)
  uint32_t* cand_ids;
  float* cand_d;
  uint32_t n_lists0, n_listsU, batch_start;
  const uint32_t* list_node;  // [n_listsU] node and level of upper list j
  const uint32_t* list_level;
  // upper-level beams: batch nodes whose insert searches levels >= 1
  const uint32_t* up_node;    // [n_up]
  const uint32_t* up_first;   // [n_up] index of the node's first upper list (global); up_first_base: the batch's first
  const uint32_t* up_levels;  // [n_up] L = min(level, top): lists at levels L .. 1, in that order
  uint32_t up_first_base, n_up, vis_cap;
  // reverse-edge requests [n_lists0 + n_listsU][M]: target row key (level 0: the node; level l: N + its upper row;
  // key_none: no request), the new node, its distance; req_pos = the position (the sort's values)
  uint32_t *req_key, *req_src, *req_pos;
  float* req_d;
  uint32_t key_none;
  // the requests sorted by key (stable): skey / sval (positions); seg[0 .. *nseg) the first position of every key
  const uint32_t* skey;
  const uint32_t* sval;
  uint32_t n_req;
  const uint32_t* seg;
  const uint32_t* nseg;
  uint32_t* work;             // prune work-queue head (zero before the launch)
  const uint32_t* row_owner;  // [upper rows] the node owning each
  unsigned long long* stats;  // [0] appended rows [1] pruned rows [2] pools truncated to 64 [3] upper beams stopped
};
enum BuildKernel { BUILD_UPPER = 0, BUILD_SELECT = 1, BUILD_PRUNE = 2 };

// bytes of one visited-table entry of SearchArgs::vis16's kind (u16 entries for kinds 1 and 2)
__host__ __device__ inline uint32_t vis_entry_bytes(uint32_t vis16) { return vis16 == 1 || vis16 == 2 ? 2u : 4u; }

// LDS layout of a search workgroup: top[ef] | next[cap] | visited table[vis_cap] (entry_bytes each) | scratch
// ids[64], dists[64]
__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
inline size_t search_lds_bytes(uint32_t ef, uint32_t cap, uint32_t vis_cap, uint32_t entry_bytes = 4) {
  return align16(8ull * ef) + align16(8ull * cap) + align16(static_cast<size_t>(entry_bytes) * vis_cap) + 64 * 4 * 2;
}

// LDS of the fast kernel: visited table[vis_cap] (entry_bytes each) | scratch ids[64], dists[64] | merge scratch
constexpr uint32_t kFastMaxEf = 512;
// list registers per lane of the fast kernel for this ef (1, 2, 4 or 8)
inline uint32_t fast_list_regs(uint32_t ef) { return ef <= 64 ? 1 : ef <= 128 ? 2 : ef <= 256 ? 4 : 8; }
// the merge scratch holds the 64 R list positions plus the cut and sink slots
inline size_t search_fast_lds_bytes(uint32_t vis_cap, uint32_t ef, uint32_t entry_bytes = 4) {
  return align16(static_cast<size_t>(entry_bytes) * vis_cap) + 64 * 4 * 2 + 8ull * (64 * fast_list_regs(ef) + 2);
}
// LDS a workgroup holds, for residency estimates: whole 1 KiB granules.  HIP's occupancy calculator rounds to 128 B,
// but the measured rates follow granules of at least 512 B: on the 100M-record index at ef = 128, 6,400 u32 entries
// (27,152 B: 6 wavefronts per CU by 128-byte rounding, 5 by 512) ran at 4.29 M QPS against 4.75-4.83 M for 6,144
// (26,128 B, 6 either way) and 4.33 M for 7,168 (5 either way) (profiles/r05/scale_cfg4_viscap*.jsonl,
// lds_occupancy.jsonl); 1 KiB keeps the sizing clear of the boundary either way.
inline size_t lds_alloc_bytes(size_t bytes) { return (bytes + 1023) / 1024 * 1024; }

// Device row layout of the vectors.  The reference's AVX2 kernels keep 8 accumulators: accumulator a sums the
// elements i ≡ a (mod 8) of the 16-aligned prefix in increasing i (distance.hh:11-76).  A distance kernel lane
// plays accumulators 2c and 2c+1 (c = 0..3) as the halves of a packed-FP32 pair, so the device row stores the
// prefix in 4-element chunks [acc 2c elem t, acc 2c+1 elem t, acc 2c elem t+1, acc 2c+1 elem t+1] (t even),
// ordered by (t/2, c):  element a + 8t lives at (t >> 1) * 16 + (a >> 1) * 4 + (t & 1) * 2 + (a & 1).
// One 16-byte load per lane (8 bytes for f16) then brings two ready-made pairs, and the 4 lanes of a vector read
// 64 contiguous bytes.  The scalar tail (elements DB..dim-1, distance.hh:112-115) follows unpermuted.
__host__ __device__ inline uint32_t permuted_index(uint32_t dim, uint32_t i) {
  const uint32_t db = dim >> 4 << 4;
  if (i >= db) return i;
  const uint32_t a = i & 7u, t = i >> 3;
  return (t >> 1) * 16u + (a >> 1) * 4u + (t & 1u) * 2u + (a & 1u);
}

// Byte rows (SHINE_ELEM_U8 / _I8): each lane's chunks are contiguous instead, chunk (t/2, c) at byte
// (c * NCH + t/2) * 4 with NCH = (dim >> 4) chunks per lane, so a lane reads dim/4 contiguous bytes (two 16-byte
// loads at dim 128) and the 4 lanes of a vector read the row's prefix as one 128-byte run; the tail follows at byte
// dim >> 4 << 4, and rows are padded to 16 bytes.
__host__ __device__ inline uint32_t permuted_index_bytes(uint32_t dim, uint32_t i) {
  const uint32_t db = dim >> 4 << 4;
  if (i >= db) return i;
  const uint32_t a = i & 7u, t = i >> 3, nch = dim >> 4;
  return ((a >> 1) * nch + (t >> 1)) * 4u + (t & 1u) * 2u + (a & 1u);
}
inline bool elem_is_byte(int elem) { return elem == 2 || elem == 3; }
// fp16 rows (config 5) keep the natural element order: their distances are judged by recall, not bitwise, and run on the
// matrix cores for inner products (kernels_impl.h pass_dists_mfma), which take each lane's 8 consecutive elements
__host__ __device__ inline uint32_t device_index(uint32_t dim, int elem, uint32_t i) {
  return elem == 2 || elem == 3 ? permuted_index_bytes(dim, i) : elem == 1 ? i : permuted_index(dim, i);
}
inline uint32_t elem_bytes(int elem) { return elem == 0 ? 4u : elem == 1 ? 2u : 1u; }
// bytes of one device row
inline uint64_t row_bytes(uint32_t dim, int elem) {
  return elem_is_byte(elem) ? (static_cast<uint64_t>(dim) + 15) / 16 * 16 : static_cast<uint64_t>(dim) * elem_bytes(elem);
}

bool dim_supported(uint32_t dim, int elem);

// The compiled vector dimensions: one translation unit each (kernels_dim.hip built with -DSHINE_DIM=D), so the
// kernel instantiations compile in parallel.  fp16 records (config 5) exist for 96, 128 and 200.
#define SHINE_DIMS(X) X(16) X(32) X(64) X(96) X(100) X(128) X(200) X(256)
#define SHINE_DECLARE_DIM(DD)                                                                                       \
  hipError_t launch_search_d##DD(int metric, int elem, uint32_t grid, const SearchArgs& a, hipStream_t s);          \
  hipError_t launch_distance_d##DD(int metric, int elem, const DistArgs& a, hipStream_t s);                        \
  hipError_t launch_build_d##DD(int which, int metric, uint32_t grid, const BuildArgs& a, hipStream_t s);
SHINE_DIMS(SHINE_DECLARE_DIM)
#undef SHINE_DECLARE_DIM
// byte rows: one translation unit per (dimension, signedness), kernels_dim.hip with -DSHINE_BYTES=2 (u8) / 3 (i8)
#define SHINE_BYTE_DIMS(X) X(100) X(128)
#define SHINE_DECLARE_BDIM(DD)                                                                                      \
  hipError_t launch_search_d##DD##_e2(int metric, uint32_t grid, const SearchArgs& a, hipStream_t s);              \
  hipError_t launch_search_d##DD##_e3(int metric, uint32_t grid, const SearchArgs& a, hipStream_t s);              \
  hipError_t launch_distance_d##DD##_e2(int metric, const DistArgs& a, hipStream_t s);                             \
  hipError_t launch_distance_d##DD##_e3(int metric, const DistArgs& a, hipStream_t s);
SHINE_BYTE_DIMS(SHINE_DECLARE_BDIM)
#undef SHINE_DECLARE_BDIM

// Returns hipSuccess or the launch error.  grid = number of persistent search slots (one wavefront each).
hipError_t launch_search(uint32_t dim, int metric, int elem, uint32_t grid, const SearchArgs& a, hipStream_t s);
hipError_t launch_distance(uint32_t dim, int metric, int elem, const DistArgs& a, hipStream_t s);
// GPU batch builder: one of BuildKernel over `grid` workgroups (f32 rows)
hipError_t launch_build(uint32_t dim, int metric, int which, uint32_t grid, const BuildArgs& a, hipStream_t s);

// Dimension-independent builder kernels (build_kernels.hip)
hipError_t launch_iota(uint32_t* out, uint64_t n, hipStream_t s);
// rows [n][dim] f32 unpermuted → device layout (kernels.h permuted_index) f32 / f16 / byte rows (elem 0 / 1 / 2 / 3);
// from_device_layout: the source is already f32 in the device layout (a layout change of the element type only)
hipError_t launch_rows_to_device(const float* src, void* dst, uint64_t n, uint32_t dim, int elem, bool from_device_layout,
                                 hipStream_t s);
// a batch's search counters: out[0] += distcomps, out[1] += searches that ended with a status
hipError_t launch_qstats_sum(const uint32_t* qs, uint32_t nq, unsigned long long* out, hipStream_t s);
// *flag |= 1 if any of `total` f32 components is not exactly a u8 (elem 2) / i8 (elem 3) value
hipError_t launch_fits_bytes(const float* src, uint64_t total, int elem, uint32_t* flag, hipStream_t s);
// segment starts of the sorted request keys (keys < key_none): seg[atomic] = i where key[i] != key[i-1]
hipError_t launch_segments(const uint32_t* skey, uint32_t n, uint32_t key_none, uint32_t* seg, uint32_t* nseg,
                           hipStream_t s);
// stable radix sort of (key, value) pairs on the low `bits` key bits; temp == nullptr: *temp_bytes = the need
hipError_t radix_sort_u32_pairs(void* temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                                const uint32_t* vals_in, uint32_t* vals_out, uint32_t n, uint32_t bits, hipStream_t s);

// Dynamic record cache updates between calls (capi.cc apply_dynamic), in order on one stream: drop the departing
// device ids from cslot; copy the admitted records' rows (row_bytes each, from the GPU's view of the vectors) into
// their arena slots and point cslot at them; set the cooling flags.  upd = [drop ids (n_drop) | (slot, id) pairs
// (n_fill) | (slot, flag) pairs (n_cool)].
hipError_t launch_cache_apply(const uint32_t* upd, uint32_t n_drop, uint32_t n_fill, uint32_t n_cool, uint32_t* cslot,
                              uint32_t* cbits, uint8_t* cvec, uint32_t* cool, uint32_t* rlogged, uint32_t* slot_id,
                              const uint8_t* vec, uint64_t row_bytes, hipStream_t s);

// Diagnostics: replay push / pop / push_k sequences through the device heap routines (one wavefront).
hipError_t launch_heap_replay(int is_max, const int32_t* ops, const float* vals, const uint32_t* ids, uint32_t n_ops,
                              uint32_t k, float* out_d, uint32_t* out_ids, uint32_t* out_n, hipStream_t s);

}  // namespace shine
