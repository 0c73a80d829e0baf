/*
 * shine_gpu.h — C ABI of the MI355X-native SHINE compute-node query engine.
 *
 * This is the drop-in boundary for the reference's query path.  The reference has no FFI: its seam is the
 * C++ template call `HNSW<Distance>::knn(q_id, span<f32>, thread)` (src/hnsw/hnsw.hh:253) reading remote
 * memory through `rdma::read_node / read_neighborlist / read_entry_point_ptr` (src/rdma/rdma_reads.hh:9-99)
 * from memory nodes that hold the dump `[free_ptr | ep_ptr | records...]` (src/memory_node.hh:15-27).
 * Each entry point below names the reference interface it replaces.
 *
 * Conventions: every function returns SHINE_OK (0) or a positive error code; nothing calls exit().  The
 * message for the last error on the calling thread is available from shine_last_error().  A handle may be
 * used by one host thread at a time; distinct handles are independent.  No torch / HIP C++ types cross the
 * boundary: streams are passed as `void*` (a hipStream_t, or NULL for the handle's own stream).
 */
#ifndef SHINE_GPU_H
#define SHINE_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHINE_OK 0
#define SHINE_ERR_ARG 1      /* invalid argument (also: ef < k, hnsw.hh:36) */
#define SHINE_ERR_IO 2       /* dump / file could not be read */
#define SHINE_ERR_FORMAT 3   /* malformed dump (record walks past free_ptr, dangling RemotePtr, ...) */
#define SHINE_ERR_HIP 4      /* HIP runtime error, or no usable gfx950 device */
#define SHINE_ERR_NOMEM 5    /* device memory exhausted */
#define SHINE_ERR_OVERFLOW 6 /* a query's candidate queue exceeded the largest supported capacity */

#define SHINE_METRIC_L2 0 /* L2Distance (src/hnsw/distance.hh:153-155), squared L2 */
#define SHINE_METRIC_IP 1 /* IPDistance (src/hnsw/distance.hh:157-161), 1 - <a,b> */

#define SHINE_ELEM_F32 0 /* element_t = f32 (src/common/types.hh:9) */
#define SHINE_ELEM_F16 1 /* vectors converted to fp16 at load (config 5); distances still accumulate in f32 */
/* Byte rows: lossless narrow storage of records whose every component is exactly a byte value, as the reference's
 * .u8bin / .i8bin inputs are before read_data converts them element-wise to f32 (read_data.hh:21-28,
 * deserializer.hh:24-44).  The kernels widen each byte back to f32 and run the same f32 distance arithmetic, so
 * results are bitwise those of SHINE_ELEM_F32; a record with any other component value is SHINE_ERR_ARG at open.
 * Rows are padded to 16 bytes.  Compiled for dim 100 and 128 (SPACEV-style i8, SIFT/BIGANN-style u8). */
#define SHINE_ELEM_U8 2  /* components in {0, ..., 255} */
#define SHINE_ELEM_I8 3  /* components in {-128, ..., 127} */
/* The narrowest lossless of U8, I8 and F32 for this index (never F16); shine_index_info.elem reports the choice. */
#define SHINE_ELEM_AUTO 4

/* Per-query counter layout (u32 words), identical in the oracle and on the GPU. */
#define SHINE_QS_DISTCOMPS 0     /* stats.distcomps                         (hnsw.hh:272,286,376,459) */
#define SHINE_QS_VISITED_UPPER 1 /* stats.visited_nodes, level > 0          (statistics.hh:164-170) */
#define SHINE_QS_VISITED_L0 2    /* stats.visited_nodes_l0                  (statistics.hh:164-170) */
#define SHINE_QS_LISTS_UPPER 3   /* stats.visited_neighborlists, level > 0  (hnsw.hh:359) */
#define SHINE_QS_LISTS_L0 4      /* stats.visited_neighborlists, level 0    (hnsw.hh:438) */
#define SHINE_QS_MAX_NEXT 5      /* exact mode: peak size of next_candidates (diagnostic) */
#define SHINE_QS_TIES 5          /* fast mode: equal-key events met (0 = result identical to exact mode) */
#define SHINE_QS_STATUS 6        /* 0 = ok, otherwise the SHINE_ERR_* that stopped this query */
#define SHINE_QS_NRESULT 7       /* number of ids written (< k only if the graph has fewer nodes) */
/* Reads of records outside the answering GPU's own stripe (sharded placements; 0 for a replica): the analogue of
 * rdma_reads_in_bytes / cache_hits / cache_misses (rdma_reads.hh:12,46; statistics.hh:148-175).  "remote" reads
 * cross xGMI, "cached" reads are served by this GPU's local copies of other stripes' hot records. */
#define SHINE_QS_REMOTE_VEC 8    /* vector reads over xGMI */
#define SHINE_QS_REMOTE_LIST 9   /* level-0 neighbour-list reads over xGMI */
#define SHINE_QS_CACHED_VEC 10   /* vector reads served by the local copies (cache hits) */
#define SHINE_QS_CACHED_LIST 11  /* level-0 list reads served by the local copies */
#define SHINE_QS_WORDS 12

typedef struct shine_index* shine_index_t;

/* Aggregates, named after the reference's CNStatistics / ThreadStatistics (statistics.hh:68-175). */
typedef struct shine_stats {
  uint64_t processed;             /* queries.processed */
  uint64_t distcomps;             /* queries.dist_comps */
  uint64_t visited_nodes;         /* queries.visited_nodes (levels > 0) */
  uint64_t visited_nodes_l0;      /* queries.visited_nodes_l0 */
  uint64_t visited_neighborlists; /* queries.visited_neighborlists (all levels) */
  uint64_t visited_neighborlists_l0;
  uint64_t rdma_reads_in_bytes;   /* bytes the reference would READ from memory nodes for the same search */
  uint64_t algorithmic_bytes;     /* roofline basis B_q summed over the batch */
  uint64_t overflow_retries;      /* queries re-run with a larger candidate-queue capacity */
  uint64_t remote_reads_in_bytes; /* bytes read over xGMI from other GPUs' stripes (device layout) */
  uint64_t cache_hits;            /* cache.hits_total: off-stripe record reads served by local copies */
  uint64_t cache_misses;          /* cache.misses_total: off-stripe record reads that crossed xGMI */
  double kernel_ms;               /* device time of the search launch(es), HIP events */
  /* The reference's cache counters (statistics.hh:159-173), where every node (vector) read is a cache lookup:
   * cache.hit_rate = node_cache_hits / node_reads. */
  uint64_t node_reads;            /* node reads: the entry point, upper-level neighbours, fresh level-0 neighbours */
  uint64_t node_cache_hits;       /* ... served by this GPU's cache (static copies or the dynamic cache) */
  uint64_t cache_admitted;        /* SHINE_CACHE_DYNAMIC: by the replays of earlier calls' logs that finished since the
                                     previous call reported (shine_cache_wait), records admitted ... */
  uint64_t cache_evicted;         /* ... evicted through the cooling table ... */
  uint64_t cache_rescued;         /* ... cooling entries given a second chance by a hit */
  uint64_t cache_log_dropped;     /* admission candidates past the log's capacity (not offered) */
} shine_stats;

typedef struct shine_index_info {
  uint64_t num_nodes;      /* records found in all dumps */
  uint64_t num_upper_rows; /* neighbour lists at levels >= 1 */
  uint64_t device_bytes;   /* HBM held by the index on each GPU */
  uint32_t dim, M, metric, elem;
  uint32_t max_level;      /* level of the entry point */
  uint32_t entry_uid;      /* uid of the entry point (ep_ptr in node1's dump, bytes 8..15) */
  uint32_t n_shards;       /* dump files (memory nodes) */
  uint32_t n_gpus;
  uint32_t placement;      /* SHINE_PLACE_* */
  uint32_t reserved0;
  uint64_t id_space;       /* device node-id range: num_nodes (replica) or n_gpus x ids_per_gpu (sharded) */
  double cache_fraction;   /* sharded: share of every other GPU's record vectors held in local HBM copies */
  uint32_t cus;            /* compute units of GPU slot 0 (hipDeviceProp_t), used to size the launches */
  uint32_t lds_per_cu;     /* LDS bytes per CU of GPU slot 0 */
} shine_index_info;

/* Placement of the records over the GPUs of a handle.
 * REPLICA: every GPU holds the whole index (the bench metric's index fits one GPU).
 * SHARDED: memory node s (dump s+1) lives in the HBM of GPU slot s % n_gpus only, as the reference places records
 *   on memory nodes (RemotePtr bits 63..48, remote_pointer.hh:9-22, rdma_atomics.hh:89).  Every GPU maps the
 *   level-0 records (vectors and lists) of all slots into one virtual range of its own (HIP virtual memory, peer
 *   access over xGMI): a search dereferences any record directly, local or remote, the way read_node /
 *   read_neighborlist dereference a RemotePtr (rdma_reads.hh:9-72).  Upper-level lists, uids and the entry point are replicated
 *   (about 1/M of the index; the reference's read_entry_point_ptr, rdma_reads.hh:74-99).  Queries are split over
 *   the slots like over compute nodes (id % G, read_data.hh:57-58); no collective is on the query path. */
#define SHINE_PLACE_REPLICA 0
#define SHINE_PLACE_SHARDED 1
/* SHARDED_REGIONS: as SHARDED, but GPU slot o owns region o of the space rather than memory nodes: balanced k-means
 *   (k = n_gpus; Kmeans::run_and_optimize, kmeans.hh:24-91) over the top-level nodes (Placement::fetch_level,
 *   placement.hh:78-106), every record in its closest region with at most 5 % imbalance, and shine_knn_batch routes
 *   each query to its closest region within per-batch limits that adapt to the slots' queues (QueryRouter,
 *   query_router.hh:106-151, 280-387), so that a search reads mostly its own GPU's HBM. */
#define SHINE_PLACE_SHARDED_REGIONS 2

/* Open the index from the memory nodes' dumps `index_m{M}_efc{efC}_node{i}_of{N}.dat`, i = 1..N, in that
 * order (replaces MemoryNode::store_or_load_index, memory_node.hh:130-209, plus the token/EP distribution,
 * compute_node.cc:258-268 and rdma_reads.hh:74-99).  dim / M / metric are not stored in the dump; they come
 * from the base file header and the file name, exactly as in the reference.  gpu_ids / n_gpus select the
 * device(s); NULL / 0 means device 0.  With n_gpus > 1 every GPU holds a full replica. */
int shine_open(const char* const* dump_paths, uint32_t n_dumps, uint32_t dim, uint32_t M, int metric, int elem,
               const int* gpu_ids, uint32_t n_gpus, shine_index_t* out);

/* Same, from dump images already in host memory (e.g. produced by shine_build). */
int shine_open_buffers(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim,
                       uint32_t M, int metric, int elem, const int* gpu_ids, uint32_t n_gpus, shine_index_t* out);

/* shine_open / shine_open_buffers with an explicit placement (SHINE_PLACE_*).  gpu_ids may repeat a device (e.g.
 * {0, 0}): each slot then owns its own stripe on that device, which exercises the sharded layout on one GPU.
 * cache_fraction (sharded only, in [0, 1]; each array's share rounded up to whole 2 MiB pages of that array, and
 * shine_index_info.cache_fraction reports the vectors' share after rounding) replaces the compute node's record cache
 * (cache::Cache, cache.hh:102-311, sized as a share of the index, compute_node.cc:40-56): each slot's records are
 * ordered hottest first (upper-level nodes, then level-0 in-degree; the reference always admits upper levels,
 * cache.hh:368) and every GPU keeps local copies of that leading share of every other GPU's records, so those
 * reads stay in local HBM instead of crossing xGMI.  Results do not depend on it. */
int shine_open_ex(const char* const* dump_paths, uint32_t n_dumps, uint32_t dim, uint32_t M, int metric, int elem,
                  const int* gpu_ids, uint32_t n_gpus, int placement, double cache_fraction, shine_index_t* out);
int shine_open_buffers_ex(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim,
                          uint32_t M, int metric, int elem, const int* gpu_ids, uint32_t n_gpus, int placement,
                          double cache_fraction, shine_index_t* out);

/* knn over a batch of host-resident queries (replaces the WorkerPool::process_queries → hnsw::schedule →
 * HNSW::knn loop, worker_pool.hh:78-89, scheduler.hh:19-102, hnsw.hh:253-307).  queries: nq × dim row-major.
 * query_ids (nullable): the queries' ids (HNSW::knn's q_id); query i is answered on GPU slot query_ids[i] % n_gpus
 * (the compute-node split, read_data.hh:57-58), or on slot i % n_gpus when NULL.
 * out_ids: nq × k uids, in the reference's result order (top_candidates heap-array order, hnsw.hh:300-303).
 * out_dists (nullable): nq × k.  stats (nullable): aggregates.  The signature is SURVEY.md §8b's.
 * Requires ef >= k (hnsw.hh:36).  Synchronous: every slot's batch is staged in pinned host memory mapped into the
 * GPU's address space (the kernels read the queries and write the results over PCIe themselves, no copy engine) and
 * enqueued before the call waits.  A slot's share beyond 1,024 queries (SHINE_HOST_CHUNK) runs as 1,024-query chunks
 * kept in flight on four streams of the slot, each staged just before its launch and copied out as soon as it is
 * done — the T threads x C coroutines of queries the reference keeps in flight (scheduler.hh:42-96,
 * compute_node.cc:354-386); not under the dynamic cache policy, whose logs are per launch. */
int shine_knn_batch(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                    uint32_t ef, uint32_t* out_ids, float* out_dists, shine_stats* stats);

/* Asynchronous shine_knn_batch_ex: routes, stages and enqueues the batch, then returns a request without waiting for
 * any search (the reference keeps T threads x C coroutines of queries in flight across its query loop,
 * worker_pool.hh:78-89, scheduler.hh:42-96; here a caller keeps several calls in flight).  The queries are copied
 * before the call returns, so their buffer may be reused at once; out_ids / out_dists / qstats (caller-owned, same
 * layout as shine_knn_batch_ex) are written by shine_wait and must stay valid until it returns.  Calls enqueued back
 * to back run concurrently, chunk by chunk, on every slot's host streams; results equal shine_knn_batch's, query by
 * query.  Under SHINE_CACHE_DYNAMIC the call completes before it returns (the cache replays calls in order).  Every
 * request is waited for exactly once; shine_close discards the ones never waited for. */
typedef struct shine_request* shine_request_t;
int shine_knn_batch_async(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                          uint32_t ef, uint32_t* out_ids, float* out_dists, uint32_t* qstats, shine_request_t* out);
/* Wait for a request, write its results and statistics (stats nullable), and free it: the call's status. */
int shine_wait(shine_request_t req, shine_stats* stats);

/* One-time setup before a measured query phase (the GPU side of the reference's compute-thread setup, outside its
 * query timer, compute_node.cc:354-380): on every slot the host streams, per-stream scratch and pinned staging for
 * calls of up to nq queries, and the search kernels' code loaded, by searching nq all-zero queries (results
 * discarded; the dynamic cache's logs of them are dropped). */
int shine_prepare(shine_index_t h, uint32_t nq, uint32_t k, uint32_t ef);

/* shine_knn_batch with the per-query counters as well: qstats (nullable) nq × SHINE_QS_WORDS, query i's row. */
int shine_knn_batch_ex(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                       uint32_t ef, uint32_t* out_ids, float* out_dists, uint32_t* qstats, shine_stats* stats);

/* Same with device-resident inputs/outputs on GPU `gpu_slot` of the handle, enqueued on `stream`
 * (hipStream_t; NULL = the handle's stream).  Asynchronous: returns after enqueue.  qstats (device,
 * nullable).  The pointers may also be pinned host memory the device can address (hipHostMalloc, torch
 * pin_memory): the kernels then read queries / write results over PCIe (zero copy; bench.py value_host_to_host).
 * Queries whose candidate queue overflowed are flagged in qstats[SHINE_QS_STATUS]; use
 * shine_knn_batch (or check qstats) when exactness under overflow must be guaranteed.
 * Batches enqueued on different streams run concurrently: the handle keeps its search scratch (work-queue
 * heads, fixup lists, visited bitmaps) per stream, so a serving loop may keep several batches in flight
 * (bench.py keeps four).  Calls on one stream are ordered as usual.
 * Stream lifetime: the handle keeps per-stream scratch keyed by the stream; a caller stream must stay valid until
 * shine_release_stream(h, stream) or shine_close(h), and must be released before it is destroyed if its handle
 * value may be reused while h is open. */
int shine_knn_batch_device(shine_index_t h, uint32_t gpu_slot, const float* d_queries, uint32_t nq, uint32_t k,
                           uint32_t ef, uint32_t* d_out_ids, float* d_out_dists, uint32_t* d_qstats, void* stream);

/* Wait for the work enqueued on `stream` and free the handle's scratch for it (every GPU slot). */
int shine_release_stream(shine_index_t h, void* stream);

/* Cache warmup (the reference's warmup split, compute_node.cc:116-131, feeding cache::Cache admission,
 * hnsw.hh:447-448): answers the warmup queries like shine_knn_batch while counting every record read, then re-ranks
 * each stripe — upper-level records first (always admitted, cache.hh:368), then level-0 records by warmup reads,
 * most first — and re-lays out the sharded arrays so the cached prefix every GPU copies holds the hottest records.
 * Results of later searches do not change; their cache_hits / cache_misses do.  No-op for a replica, one slot, or a
 * zero cache fraction.  On failure the handle keeps its previous layout but can no longer be re-ranked. */
int shine_cache_warmup(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                       uint32_t ef);

/* Cache policy of a sharded handle (the compute node's record cache, cache::Cache, cache.hh:24-311).
 * STATIC (default): the cache_fraction of shine_open_ex — each stripe's hottest records (static rank, or the warmup
 *   re-rank of shine_cache_warmup) copied once to every other GPU.
 * DYNAMIC: the reference's runtime policy.  Every GPU keeps an arena of ratio_percent % of estimate_index_size(N)
 *   over 16 + 4d bytes entries (compute_node.cc:40-56, hnsw.hh:309-321).  A search reads a cached record from the
 *   arena, any other off-stripe record over xGMI; after every shine_knn_batch the misses are admitted (entry point and
 *   upper levels always, level-0 records while the cache is not full, then with probability 0.01 — hnsw.hh:447-448,
 *   constants.hh:16), evicting through random cooling and the cooling table, and a hit on a cooling entry rescues it
 *   (cache.hh:128-132, 232-311, cooling_table.hh:52-98).  The cache is fixed during a call and updated between calls
 *   (stream-ordered before the next call on the slot's stream); random draws come from SplitMix64 seeded with
 *   `seed` + slot, so runs are reproducible (oracle/cache_ref.py restates the policy).  Results never depend on it.
 *   Needs a sharded handle of >= 2 slots opened with cache_fraction 0.  Device-API calls (shine_knn_batch_device)
 *   read the cache; their logged misses are applied by the next shine_cache_update or shine_knn_batch, which first
 *   wait for every stream of the device (the update rewrites arena rows a search in flight could be reading). */
#define SHINE_CACHE_STATIC 0
#define SHINE_CACHE_DYNAMIC 1
int shine_set_cache_policy(shine_index_t h, int policy, double ratio_percent, uint64_t seed);
/* Apply the misses and rescues logged since the last update (shine_knn_batch does this itself after every call). */
int shine_cache_update(shine_index_t h);
/* Pipelined policy (the default; SHINE_CACHE_LAG=0 replays inside each call instead): shine_knn_batch starts the
 * replay of the previous call's logs on the handle's worker threads and returns without waiting for it; the next call
 * (or any cache function) waits for it and enqueues its updates ahead of its own searches, so call n's admissions
 * serve from call n + 2 on either way.  This waits for such a replay and enqueues its updates now (a caller timing a
 * stream of calls ends its clock here).  The replay's statistics (cache_admitted / evicted / rescued) are reported by
 * the next shine_knn_batch. */
int shine_cache_wait(shine_index_t h);
/* Diagnostics: the uids GPU slot `slot`'s dynamic cache holds, ascending (*n = count; up to cap written), and the
 * device ids of uids (0xFFFFFFFF where a uid is not a record). */
int shine_cache_keys(shine_index_t h, uint32_t slot, uint32_t* uids, uint64_t cap, uint64_t* n);
int shine_device_ids(shine_index_t h, const uint32_t* uids, uint32_t n, uint32_t* out);
/* Diagnostics (host only): the dynamic cache's policy engine driven by explicit logs, for tests against its
 * restatement.  entries / seed as a GPU slot's cache; call c offers cand[cand_off[c] .. cand_off[c+1]) (triples
 * query, key, flags: bit 0 always, bit 1 coin) after rescuing resc[resc_off[c] .. resc_off[c+1]) (keys).  Writes the
 * final keys ascending (up to cap; *n = count) and counts[0..2] = admitted, evicted, rescued. */
int shine_selftest_cache(uint32_t entries, uint64_t seed, uint32_t n_calls, const uint32_t* cand_off,
                         const uint32_t* cand, const uint32_t* resc_off, const uint32_t* resc, uint32_t* keys,
                         uint64_t cap, uint64_t* n, uint64_t* counts);

/* The GPU slot each query of a batch is answered on: id % n_gpus, or for SHINE_PLACE_SHARDED_REGIONS the slot the
 * handle's query router picks (QueryRouter::run_routing, query_router.hh:280-387): the closest region whose count in
 * the current batch of 200 * n_gpus queries (LIMIT_PER_CN, constants.hh:25) is below its limit.  At every batch
 * boundary the limits are re-derived from the slots' queue sizes (update_limits, query_router.hh:106-151), modelled
 * from each slot's rate in its last call.  The router's state lives in the handle across calls, as the reference's
 * router lives for the whole query phase, so this call advances it like a shine_knn_batch would.  Host-only. */
int shine_route(shine_index_t h, const float* queries, uint32_t nq, uint32_t* out_slot);

/* Host-only planner behind SHINE_PLACE_SHARDED_REGIONS (no device needed): fetch_level(500) + balanced k-means.
 * centroids (nullable): capacity 2k x dim (k odd: 2k centroids merged in pairs); mapping (nullable, capacity 2k):
 * region of every centroid; n_centroids (nullable): k or 2k; region_of_uid (nullable): region of every record by
 * uid, capacity uid_capacity. */
int shine_plan_regions(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim, uint32_t M,
                       int metric, uint32_t k, uint32_t* region_of_uid, uint64_t uid_capacity, float* centroids,
                       uint32_t* mapping, uint32_t* n_centroids);

/* Host-only view plan of SHINE_PLACE_SHARDED (no device needed; the same plan shine_open_ex maps): for n_slots GPU
 * slots on gpu_ids (ids may repeat), a sharded array of stride_bytes per slot's stripe, whose leading cached_bytes every
 * other slot keeps a local copy of.  Every slot's view maps the whole id space, G x stride_bytes: its own stripe
 * (SHINE_VIEW_OWN), its local copies of the other stripes' hot prefixes (SHINE_VIEW_COPY) and the other stripes' cold
 * rows backed by their owners' HBM (SHINE_VIEW_PEER: xGMI reads between distinct GPUs) — the reference's RemotePtr
 * memory node (remote_pointer.hh:9-22) becomes the stripe, a remote read a peer load.  pieces (capacity cap_pieces;
 * nullable to count): every view's pieces, view by view in offset order.  access (nullable, n_slots x n_slots):
 * row o holds the n_access[o] devices granted access to view o.  peer_pairs (nullable, 2 x n_slots x n_slots): the
 * ordered (accessor, owner) device pairs that need a peer path, n_peer_pairs of them. */
#define SHINE_VIEW_OWN 0
#define SHINE_VIEW_COPY 1
#define SHINE_VIEW_PEER 2
typedef struct shine_view_piece {
  uint32_t view_slot;      /* the slot whose view holds the piece */
  uint32_t stripe;         /* the slot whose rows the piece holds */
  uint64_t offset;         /* in the view's virtual range */
  uint64_t size;
  int32_t backing_device;  /* the GPU whose allocation backs the piece */
  uint32_t kind;           /* SHINE_VIEW_* */
} shine_view_piece;
int shine_plan_sharded_views(const int* gpu_ids, uint32_t n_slots, uint64_t stride_bytes, uint64_t cached_bytes,
                             shine_view_piece* pieces, uint64_t cap_pieces, uint64_t* n_pieces, int* access,
                             uint32_t* n_access, int* peer_pairs, uint32_t* n_peer_pairs);

/* Kmeans<Distance> over n rows (kmeans.hh:10-378), host-only: balanced != 0 is run_and_optimize (balanced k-means,
 * c = 0.15, penalty factor 1.01, max size difference 1; odd k runs 2k clusters and merges the closest pairs),
 * balanced == 0 is run_kmeans with k clusters.  centroids: capacity 2k x dim; mapping: capacity 2k (centroid ->
 * region); n_centroids, region_sizes (k; rows per region after balancing) and iterations ([0] Lloyd, [1] balancing)
 * are nullable.  SHINE_ERR_ARG when n < the number of clusters (the reference asserts). */
int shine_kmeans(const float* rows, uint64_t n, uint32_t dim, int metric, uint32_t k, int balanced, float* centroids,
                 uint32_t* mapping, uint32_t* n_centroids, uint64_t* region_sizes, uint32_t* iterations);

/* QueryRouter::run_routing's decisions for a stream of nq queries over the given centroids (host-only): the region
 * of every query, with BALANCED_ROUTING limits and, when adaptive != 0, update_limits at every boundary of
 * 200 * k queries from the queue sizes the acks carry: row b of queue_sizes (n_rows x k; the last row repeats;
 * NULL = all zero, no update) at boundary b.  out_limits (nullable, k): the limits after the last boundary. */
int shine_router_run(const float* centroids, const uint32_t* mapping, uint32_t n_centroids, uint32_t k, uint32_t dim,
                     int metric, const float* queries, uint32_t nq, const uint32_t* queue_sizes, uint32_t n_rows,
                     int adaptive, uint32_t* out_region, uint64_t* out_limits);

/* Batched distance kernel: for query i and its n_per_query node uids node_uids[i*n_per_query + j], write
 * out[i*n_per_query + j] = Distance::dist(q_i, x_uid) (distance.hh:153-161).  Device pointers, async. */
int shine_distance_batch_device(shine_index_t h, uint32_t gpu_slot, const float* d_queries, uint32_t nq,
                                const uint32_t* d_node_uids, uint32_t n_per_query, float* d_out, void* stream);

/* Search modes.  EXACT (default): the reference's two std heaps replayed step for step — ids in heap-array
 * order, identical to HNSW::knn under distance ties.  FAST: one sorted candidate list per query held in
 * registers (ef <= 512; larger ef runs the exact kernel); same expansions, ids, distances and counters whenever
 * no two distances compare equal where the reference's heap layout would break the tie (qstats word
 * SHINE_QS_TIES counts such events, 0 = identical set), results in ascending distance order. */
#define SHINE_MODE_EXACT 0
#define SHINE_MODE_FAST 1
int shine_set_search_mode(shine_index_t h, int mode);

int shine_index_get_info(shine_index_t h, shine_index_info* out);

/* Total algorithmic bytes (roofline basis) for per-query counters produced by a search with this index. */
uint64_t shine_algorithmic_bytes(shine_index_t h, const uint32_t* qstats, uint32_t nq);

int shine_close(shine_index_t h);

/* Diagnostics: replay a sequence of heap operations (0 = push, 1 = pop, 2 = push_k with capacity k) through the
 * device heap routines the search kernel uses (on device 0) and return the final heap array.  is_max selects
 * heap::MaxHeapCompare / MinHeapCompare (heap.hh:15-21).  Tests compare it with libstdc++'s std::push_heap /
 * std::pop_heap on the same sequence. */
int shine_selftest_heap(int is_max, const int32_t* ops, const float* vals, const uint32_t* ids, uint32_t n_ops,
                        uint32_t k, float* out_d, uint32_t* out_ids, uint32_t* out_n);

const char* shine_last_error(void);

/* Provenance of this library: "src <hash of every source it was built from> git <head at build time>". */
const char* shine_build_id(void);

/* Host-only graph diagnostics over dump images (no device needed): how much of the index a search can reach.
 * A level-0 search follows level-0 lists only (hnsw.hh:436-438) from where the greedy descent ends, so a record
 * outside reachable_l0 can never be returned, whatever ef.  Used to tell an index property from a search bug. */
typedef struct shine_graph_stats {
  uint64_t num_nodes;
  uint64_t reachable_l0;     /* records reachable from the entry point along level-0 lists */
  uint64_t reachable_any;    /* ... along the lists of every level */
  uint64_t zero_indegree_l0; /* records no level-0 list names (entry point excluded) */
  uint64_t full_lists_l0;    /* records whose level-0 list holds 2M entries */
  double mean_degree_l0;
  uint32_t max_level;
  uint32_t reserved0;
} shine_graph_stats;
int shine_graph_stats_buffers(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim,
                              uint32_t M, shine_graph_stats* out);

/* ----------------------------------------------------------------------------------------------------------
 * Build path: a parallel CPU restatement of HNSW::insert (hnsw.hh:40-251) writing the
 * reference's dump layout.  threads == 1 reproduces the single-threaded insert order exactly.
 * -------------------------------------------------------------------------------------------------------- */
typedef struct shine_build* shine_build_t;
int shine_build(const float* base, uint64_t n, uint32_t dim, uint32_t M, uint32_t ef_construction, int metric,
                uint32_t n_shards, uint32_t seed, uint32_t threads, shine_build_t* out);
uint64_t shine_build_dump_size(shine_build_t b, uint32_t shard);
const uint8_t* shine_build_dump_data(shine_build_t b, uint32_t shard);
uint64_t shine_build_distcomps(shine_build_t b);
int shine_build_write(shine_build_t b, const char* dir, uint32_t M, uint32_t ef_construction); /* dump/ files */
int shine_build_free(shine_build_t b);

/* ----------------------------------------------------------------------------------------------------------
 * GPU batch build (SURVEY §8f row 2 at 10M-100M records): HNSW::insert (hnsw.hh:40-251) and select_heuristic
 * (:482-522) on one MI355X.  Levels are drawn exactly as shine_build draws them (std::mt19937(seed), hnsw.hh:48; the
 * first record takes level 0 and a record above the top level takes top + 1, :56-111).  Records are inserted in id
 * order in batches of consecutive ids, every record of a batch against the graph as it stood before the batch:
 * level-0 candidates come from the fast search kernel (knn with k = ef = ef_construction), upper levels from a beam
 * kernel, select_heuristic(M) gives each record its lists, and the reverse edges of a batch are applied per target
 * row (appended, or the row re-pruned with select_heuristic(m_max) over its old and new entries together).  A record
 * that raises the top level is inserted alone, so the entry-point protocol (:56-111, 234-248) is the reference's.
 * Deterministic for fixed inputs.  Batches hold floor(batch_fraction x records already inserted) records (at least 1,
 * at most max_batch; 0 / 0 = defaults 0.02 and 1 << 20).
 * base: n x dim f32 rows, on the host (base_on_device = 0) or in device memory of GPU gpu_id (1: read during the call
 * only).  The result stays on that GPU: open it as a search handle (shine_gpu_build_open) and / or write the reference's
 * dump layout (shine_gpu_build_dumps, memory node of each record drawn like shine_build's).
 * -------------------------------------------------------------------------------------------------------- */
typedef struct shine_gpu_builder* shine_gpu_build_t;
typedef struct shine_gpu_build_stats {
  uint64_t num_nodes;
  uint64_t num_upper_rows;       /* neighbour lists at levels >= 1 */
  uint64_t batches;
  uint64_t upper_lists;          /* upper-level candidate lists searched */
  uint64_t requests;             /* reverse-edge requests (selected neighbours) */
  uint64_t rows_appended;        /* target rows that took their new entries as appends */
  uint64_t rows_pruned;          /* target rows re-pruned with select_heuristic(m_max) */
  uint64_t pools_truncated;      /* re-prunes whose old + new entries exceeded 64 (the 64 closest were kept) */
  uint64_t upper_beams_stopped;  /* upper-level beams stopped by a full visited table */
  uint64_t search_failures;      /* level-0 searches that ended with a status (none expected) */
  uint64_t distcomps;            /* distance computations of the level-0 searches */
  uint32_t max_level, entry_uid;
  double ms_total;               /* wall time of shine_gpu_build */
  /* device time per phase, with SHINE_BUILD_PROFILE=1 (each batch then waits for its phases); else 0 */
  double ms_search, ms_upper, ms_select, ms_sort, ms_prune;
} shine_gpu_build_stats;
int shine_gpu_build(const float* base, int base_on_device, uint64_t n, uint32_t dim, uint32_t M,
                    uint32_t ef_construction, int metric, uint32_t seed, int gpu_id, double batch_fraction,
                    uint32_t max_batch, shine_gpu_build_t* out);
int shine_gpu_build_get_stats(shine_gpu_build_t b, shine_gpu_build_stats* out);
/* The reference's dump images ([free_ptr | ep_ptr | records], memory_node.hh:15-27, 185-201) of the built index over
 * n_shards memory nodes, in host memory (records in id order within each node). */
int shine_gpu_build_dumps(shine_gpu_build_t b, uint32_t n_shards);
uint64_t shine_gpu_build_dump_size(shine_gpu_build_t b, uint32_t shard);
const uint8_t* shine_gpu_build_dump_data(shine_gpu_build_t b, uint32_t shard);
/* <dir>/dump/index_m{M}_efc{efC}_node{i}_of{N}.dat (compute_node.cc:426-430) from shine_gpu_build_dumps' images */
int shine_gpu_build_write(shine_gpu_build_t b, const char* dir);
/* The built index as a search handle (replica on the build's GPU; elem F32, F16, U8 or I8, the last two only when every
 * component is exactly such a byte value).  The device arrays move into the handle: afterwards the build handle keeps
 * its dump images and statistics only. */
int shine_gpu_build_open(shine_gpu_build_t b, int elem, shine_index_t* out);
/* The built index under any placement of shine_open_ex (e.g. SHINE_PLACE_SHARDED over 8 GPUs): the records spread over
 * n_shards memory nodes exactly as shine_gpu_build_dumps spreads them, laid out as shine_open_buffers_ex lays out those
 * dumps — without writing or parsing them.  The build handle keeps its arrays (shine_gpu_build_open may follow). */
int shine_gpu_build_open_ex(shine_gpu_build_t b, uint32_t n_shards, int elem, const int* gpu_ids, uint32_t n_gpus,
                            int placement, double cache_fraction, shine_index_t* out);
int shine_gpu_build_free(shine_gpu_build_t b);

#ifdef __cplusplus
}
#endif

#endif /* SHINE_GPU_H */
