// C ABI (include/shine_gpu.h): the HBM shard manager and the batched query entry points.
//
// Replaces, on the query side: MemoryNode (src/memory_node.hh:40-209: buffer allocation + dump load),
// the remote-access token / entry-point distribution (compute_node.cc:258-268, rdma_reads.hh:74-99),
// WorkerPool::process_queries + hnsw::schedule (worker_pool.hh:78-89, scheduler.hh:19-102) and the per-query
// HNSW::knn coroutine (hnsw.hh:253-307).  One query per wavefront replaces one query per coroutine; the device
// work queue replaces the lock-free query queue (query_router.hh:393 / scheduler.hh:64-77).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <string>
#include <thread>
#include <vector>

#include "index_internal.h"

using namespace shine;

namespace {

DevGraph dev_graph(const shine_index* h, const Replica& r) {
  DevGraph g{};
  const bool sharded = h->placement != SHINE_PLACE_REPLICA;
  g.vec = sharded ? static_cast<const void*>(h->svec.view[r.slot].va) : r.vec.p;
  g.adj0 = sharded ? reinterpret_cast<const uint32_t*>(h->sadj0.view[r.slot].va) : r.adj0.p;
  g.uid = r.uid.p;
  g.up_base = r.up_base.p;
  g.adjU = r.adjU.p;
  g.inv_uid = r.inv_uid.p;
  g.inv_size = h->inv_size;
  g.pad_node = r.pad_node;
  g.N = static_cast<uint32_t>(h->id_space);
  g.M0 = h->M0;
  g.MU = h->M;
  g.ep = h->ep;
  g.ep_level = h->ep_level;
  g.lists_unique = h->lists_unique;
  g.sharded = h->placement != SHINE_PLACE_REPLICA && h->reps.size() > 1 ? 1u : 0u;
  g.slot = r.slot;
  g.stripe_ids = static_cast<uint32_t>(h->ids_per_slot);
  g.cached_rows = static_cast<uint32_t>(h->cached_rows);
  g.cached_list_rows = static_cast<uint32_t>(h->cached_list_rows);
  g.div_magic = h->div_magic;
  g.div_shift = h->div_shift;
  if (h->cache_policy == SHINE_CACHE_DYNAMIC && g.sharded && r.cslot.p) {
    g.cslot = r.cslot.p;
    g.cbits = r.cbits.p;
    g.cvec = r.cvec.p;
    g.cool = r.cool.p;
    g.clog = r.clog.p;
    g.clog_n = r.logn.p;
    g.rlog = r.rlog.p;
    g.clog_cap = r.clog_cap;
    g.rlog_cap = r.rlog_cap;
    g.rlogged = r.rlogged.p;
    g.dyn_epoch = r.log_epoch;
    g.dyn_full = r.dyn_full ? 1u : 0u;
    g.dyn_call = r.dyn_call;
    g.dyn_seed = h->cache_seed + r.slot;
  }
  return g;
}

// Division by the stripe size on the device: for x < 2^31, x / U == umulhi(x, m) >> (l - 1) with l = ceil(log2 U),
// m = floor(2^(31 + l) / U) + 1 (round-up reciprocal; m < 2^32 for U >= 2).  Checked on the host at every stripe
// boundary the id space has.
bool stripe_divider(uint64_t U, uint64_t slots, uint32_t& magic, uint32_t& shift) {
  if (U < 2 || U * slots > 0x80000000ull) return false;
  uint32_t l = 0;
  while ((1ull << l) < U) ++l;
  const unsigned __int128 m = ((static_cast<unsigned __int128>(1) << (31 + l)) / U) + 1;
  if (m >> 32) return false;
  magic = static_cast<uint32_t>(m);
  shift = l - 1;
  auto q = [&](uint64_t x) { return static_cast<uint32_t>((x * magic) >> 32) >> shift; };
  for (uint64_t o = 0; o < slots; ++o) {
    const uint64_t lo = o * U, hi = lo + U - 1;
    if (q(lo) != o || q(hi) != o) return false;
  }
  return true;
}

template <class T>
int upload(DevBuf<T>& dst, const T* src, size_t n, hipStream_t s) {
  if (int rc = dst.grow(std::max<size_t>(n, 1))) return rc;
  if (n) HIP_TRY(hipMemcpyAsync(dst.p, src, n * sizeof(T), hipMemcpyHostToDevice, s));
  return 0;
}

void release_state(IndexState* h) {
  for (auto& R : h->reps) {
    // The whole device drains: a caller stream may already be destroyed (include/shine_gpu.h: stream lifetime), so
    // its handle is never touched here.
    (void)hipSetDevice(R.device);
    (void)hipDeviceSynchronize();
    for (auto* b : {&R.adj0, &R.uid, &R.up_base, &R.adjU, &R.inv_uid}) b->release();
    for (auto& e : R.by_stream) e.second->release();
    R.by_stream.clear();
    R.main.release();
    R.release_dynamic();
    R.prof.release();
    R.vec.release();
    for (auto& st : R.stages_free) st->release();
    R.stages_free.clear();
    for (hipStream_t s : R.hstreams) (void)hipStreamDestroy(s);
    if (R.hfork) (void)hipEventDestroy(R.hfork);
    R.hstreams.clear();
    R.hfork = nullptr;
    if (R.ev0) (void)hipEventDestroy(R.ev0);
    if (R.ev1) (void)hipEventDestroy(R.ev1);
    if (R.stream) (void)hipStreamDestroy(R.stream);
  }
  h->svec.release();
  h->sadj0.release();
  h->reps.clear();
}

void release_index(shine_index* h) {
  release_state(h);
  delete h;
}

hipMemAllocationProp device_prop(int device) {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

// Allocate and map one sharded array (see ShardedArray), then fill nothing: the caller writes every slot's stripe
// through that slot's view and calls fill_copies.  Access is granted once per view, for every device of the handle,
// over a view without holes (per-piece grants on views with holes were refused by the driver).
int map_sharded(ShardedArray& A, uint64_t stride, size_t cached, const std::vector<int>& devs, size_t gran) {
  const size_t G = devs.size();
  // the plan (views.cc, host-only and tested on CPU): which allocation backs every piece of every view, and the
  // devices every view grants access to
  const ViewPlan P = plan_views(devs, stride, cached);
  A.stride = stride;
  A.cached = P.cached;
  A.hot.assign(G, 0);
  A.cold.assign(G, 0);
  A.copy.assign(G * G, 0);  // [o * G + q]: slot o's local copy of slot q's hot prefix
  for (size_t o = 0; o < G; ++o) {
    const hipMemAllocationProp prop = device_prop(devs[o]);
    if (A.cached) HIP_TRY(hipMemCreate(&A.hot[o], A.cached, &prop, 0));
    if (A.cached < stride) HIP_TRY(hipMemCreate(&A.cold[o], stride - A.cached, &prop, 0));
    for (size_t q = 0; q < G; ++q)
      if (A.cached && q != o) HIP_TRY(hipMemCreate(&A.copy[o * G + q], A.cached, &prop, 0));
  }
  A.view.resize(G);
  for (size_t o = 0; o < G; ++o) {
    StripedRange& V = A.view[o];
    V.bytes = G * stride;
    void* va = nullptr;
    HIP_TRY(hipMemAddressReserve(&va, V.bytes, gran, nullptr, 0));
    V.va = static_cast<char*>(va);
    for (const ViewPiece& p : P.pieces[o]) {
      // own stripe: this slot's hot / cold allocation; a copy: this slot's copy of the stripe's hot prefix; a peer
      // piece: the owner's cold allocation (on the owner's GPU)
      const hipMemGenericAllocationHandle_t backing = p.kind == 1 ? A.copy[o * G + p.stripe]
                                                      : p.hot     ? A.hot[p.stripe]
                                                                  : A.cold[p.stripe];
      HIP_TRY(hipMemMap(V.va + p.offset, p.size, 0, backing, 0));
      V.maps.emplace_back(p.offset, p.size);
    }
    std::vector<hipMemAccessDesc> acc(P.access[o].size());
    for (size_t i = 0; i < acc.size(); ++i) {
      acc[i].location.type = hipMemLocationTypeDevice;
      acc[i].location.id = P.access[o][i];
      acc[i].flags = hipMemAccessFlagsProtReadWrite;
    }
    const hipError_t e = hipMemSetAccess(V.va, V.bytes, acc.data(), acc.size());
    if (e != hipSuccess)
      return set_error(SHINE_ERR_HIP, std::string("hipMemSetAccess(") + std::to_string(V.bytes) + "-byte view, " +
                                          std::to_string(V.maps.size()) + " pieces): " + hipGetErrorString(e));
  }
  return 0;
}

// Refresh every slot's local copies of the other slots' hot prefixes from the owners' stripes.
int fill_copies(ShardedArray& A, const std::vector<int>& devs) {
  const size_t G = devs.size();
  if (!A.cached) return 0;
  for (size_t o = 0; o < G; ++o) {
    HIP_TRY(hipSetDevice(devs[o]));
    for (size_t q = 0; q < G; ++q)
      if (q != o)
        HIP_TRY(hipMemcpy(A.view[o].va + q * A.stride, A.view[q].va + q * A.stride, A.cached, hipMemcpyDeviceToDevice));
  }
  return 0;
}

// Every component is bit for bit the f32 image of a u8 (SHINE_ELEM_U8) / i8 (_I8) value (so -0.0 and NaN never
// fit): the byte rows then give the kernels exactly the f32 operands the reference's records hold.
bool fits_bytes(const std::vector<float>& v, int elem) {
  const float lo = elem == SHINE_ELEM_U8 ? 0.f : -128.f, hi = elem == SHINE_ELEM_U8 ? 255.f : 127.f;
  for (float x : v) {
    if (!(x >= lo && x <= hi)) return false;
    const float r = static_cast<float>(static_cast<int>(x));
    uint32_t a, b;
    std::memcpy(&a, &x, 4);
    std::memcpy(&b, &r, 4);
    if (a != b) return false;
  }
  return true;
}

// heat (nullable, indexed by graph node): warmup read counts that rank each stripe's level-0 records for the cache
int make_index(HostGraph G, int elem, const int* gpu_ids, uint32_t n_gpus, int placement, double cache_fraction,
               shine_index_t* out, const std::vector<uint32_t>* heat = nullptr) {
  if (!out) return set_error(SHINE_ERR_ARG, "out is NULL");
  if (elem < SHINE_ELEM_F32 || elem > SHINE_ELEM_AUTO)
    return set_error(SHINE_ERR_ARG, "elem must be one of SHINE_ELEM_F32 / _F16 / _U8 / _I8 / _AUTO");
  if (elem == SHINE_ELEM_AUTO || elem_is_byte(elem)) {
    // byte rows only where they reproduce every component bit for bit (so every distance is unchanged)
    if (elem == SHINE_ELEM_AUTO) {
      elem = SHINE_ELEM_F32;
      for (int b : {SHINE_ELEM_U8, SHINE_ELEM_I8})
        if (dim_supported(G.L.dim, b) && fits_bytes(G.vec, b)) {
          elem = b;
          break;
        }
    } else if (!fits_bytes(G.vec, elem)) {
      return set_error(SHINE_ERR_ARG, std::string("a record component is not exactly a ") +
                                          (elem == SHINE_ELEM_U8 ? "u8" : "i8") + " value: byte rows would change it");
    }
  }
  if (placement != SHINE_PLACE_REPLICA && placement != SHINE_PLACE_SHARDED && placement != SHINE_PLACE_SHARDED_REGIONS)
    return set_error(SHINE_ERR_ARG, "placement must be one of SHINE_PLACE_REPLICA / _SHARDED / _SHARDED_REGIONS");
  if (!(cache_fraction >= 0.0 && cache_fraction <= 1.0))
    return set_error(SHINE_ERR_ARG, "cache fraction must be in [0, 1]");
  if (!dim_supported(G.L.dim, elem))
    return set_error(SHINE_ERR_ARG, "dim " + std::to_string(G.L.dim) + " has no compiled kernel for this element type");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (ndev <= 0) return set_error(SHINE_ERR_HIP, "no HIP device");
  std::vector<int> devs;
  if (!gpu_ids || n_gpus == 0) devs.push_back(0);
  else devs.assign(gpu_ids, gpu_ids + n_gpus);
  for (int d : devs)
    if (d < 0 || d >= ndev) return set_error(SHINE_ERR_ARG, "gpu id " + std::to_string(d) + " out of range");
  const bool sharded = placement != SHINE_PLACE_REPLICA;
  // device shape from the runtime (CU count and LDS per CU size the launches; partitioned modes change both)
  std::vector<hipDeviceProp_t> props(devs.size());
  for (size_t i = 0; i < devs.size(); ++i) {
    HIP_TRY(hipGetDeviceProperties(&props[i], devs[i]));
    if (std::strncmp(props[i].gcnArchName, "gfx950", 6) != 0)
      return set_error(SHINE_ERR_HIP, "GPU " + std::to_string(devs[i]) + " is " + props[i].gcnArchName +
                                          "; the kernels are built for gfx950 (MI355X) only");
  }
  if (sharded) {  // every slot dereferences every other slot's stripe: each ordered pair needs a peer path (xGMI)
    for (const auto& [a, b] : plan_views(devs, 1, 0).peer_pairs) {
      int can = 0;
      HIP_TRY(hipDeviceCanAccessPeer(&can, a, b));
      if (!can)
        return set_error(SHINE_ERR_HIP, "GPU " + std::to_string(a) + " cannot access GPU " + std::to_string(b) +
                                            "'s memory (no peer path): the sharded placement needs all-to-all "
                                            "peer access");
    }
  }

  std::unique_ptr<shine_index> h(new shine_index);
  struct Guard {  // a failed open releases what it had already placed on the devices
    std::unique_ptr<shine_index>& p;
    ~Guard() {
      if (p) release_index(p.release());
    }
  } guard{h};
  h->dim = G.L.dim;
  h->M = G.L.M;
  h->M0 = 2 * G.L.M;
  h->metric = G.metric;
  h->elem = elem;
  h->N = G.N;
  h->upper_rows = G.adjU.size() / G.L.M;
  h->ep_level = G.ep_level;
  h->ep_uid = G.uid[G.ep];
  h->n_shards = G.n_shards;
  h->lists_unique = G.lists_unique ? 1 : 0;
  h->placement = placement;

  const uint32_t dim = G.L.dim, M0 = h->M0, S = G.n_shards;
  const uint32_t slots = static_cast<uint32_t>(devs.size());
  const uint64_t vrow = row_bytes(dim, elem), arow = 4ull * M0;
  const std::vector<uint64_t>& start = G.shard_start;

  // Device id space.  Replica: graph.cc's dense ids.  Sharded: slot o = s % slots owns memory node s; its records
  // are numbered o * U + rank, hottest first (upper-level nodes by level, then by level-0 in-degree: a static form
  // of the reference's cache admission, upper levels always, cache.hh:368), with U a whole number of VM pages of
  // rows, so that every slot's stripe starts on its own pages and its hot prefix is a page range.
  std::vector<uint64_t> owned(slots, 0);
  std::vector<std::vector<uint32_t>> order(sharded ? slots : 0);  // [slot]: its records (old ids), hottest first
  uint64_t U = G.N;
  size_t gran = 0;
  if (sharded) {
    if (placement == SHINE_PLACE_SHARDED_REGIONS) {  // balanced k-means regions of the top levels (placement.hh:22-61)
      if (plan_regions(G, slots, true, h->regions))
        return set_error(SHINE_ERR_ARG, "region placement: fewer top-level nodes than k-means clusters");
      h->router.init(slots);
      h->slot_rate.assign(slots, 0.0);
      const std::vector<uint32_t> region = assign_regions(G, h->regions, 0.05, 1);
      for (uint64_t g = 0; g < G.N; ++g) order[region[g]].push_back(static_cast<uint32_t>(g));
    } else {
      for (uint32_t s = 0; s < S; ++s)
        for (uint64_t g = start[s]; g < start[s + 1]; ++g) order[s % slots].push_back(static_cast<uint32_t>(g));
    }
    for (uint32_t o = 0; o < slots; ++o) owned[o] = order[o].size();
    for (int d : devs) {
      const hipMemAllocationProp prop = device_prop(d);
      size_t g = 0;
      HIP_TRY(hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended));
      gran = std::max(gran, g);
    }
    gran = std::max(gran, size_t(1) << 21);  // whole 2 MiB pages per piece (4 KiB pieces were refused access)
    uint64_t unit = 1;
    while ((unit * vrow) % gran != 0 || (unit * arow) % gran != 0) unit <<= 1;
    const uint64_t most = *std::max_element(owned.begin(), owned.end());
    U = std::max<uint64_t>(unit, (most + unit - 1) / unit * unit);
    if (U * slots >= 0x80000000ull)
      return set_error(SHINE_ERR_ARG, "sharded id space of " + std::to_string(U * slots) + " ids exceeds 2^31");
    if (!stripe_divider(U, slots, h->div_magic, h->div_shift))
      return set_error(SHINE_ERR_ARG, "no exact 32-bit divider for " + std::to_string(U) + " ids per stripe");
  }
  const uint64_t id_space = sharded ? U * slots : G.N;
  h->id_space = id_space;
  h->ids_per_slot = U;
  h->words_per_slot = (id_space + 31) / 32;
  std::vector<uint32_t> newid;
  if (sharded) {
    std::vector<uint32_t> indeg(G.N, 0);
    for (uint32_t x : G.adj0)
      if (x != kInvalid) ++indeg[x];
    newid.resize(G.N);
    for (uint32_t o = 0; o < slots; ++o) {
      std::stable_sort(order[o].begin(), order[o].end(), [&](uint32_t a, uint32_t b) {
        if (G.level[a] != G.level[b]) return G.level[a] > G.level[b];  // upper levels always admitted
        if (heat && (*heat)[a] != (*heat)[b]) return (*heat)[a] > (*heat)[b];  // warmup reads, most first
        return indeg[a] > indeg[b];
      });
      for (size_t i = 0; i < order[o].size(); ++i) newid[order[o][i]] = static_cast<uint32_t>(o * U + i);
    }
  }
  auto dev_id = [&](uint32_t g) -> uint32_t { return (!sharded || g == kInvalid) ? g : newid[g]; };
  h->ep = dev_id(G.ep);
  if (sharded) {  // every id a kernel can follow must name a record of its slot (never a hole, never past the space)
    auto real = [&](uint32_t d) { return d / U < slots && d % U < owned[d / U]; };
    bool ok = real(h->ep);
    for (uint32_t x : G.adj0) ok = ok && (x == kInvalid || real(newid[x]));
    for (uint32_t x : G.adjU) ok = ok && (x == kInvalid || real(newid[x]));
    if (!ok) return set_error(SHINE_ERR_FORMAT, "sharded layout: a list names an id outside the records");
  }

  // per-node arrays in device order (sharded: holes between the stripes stay kInvalid and are never referenced)
  std::vector<uint32_t> uid_s, upb_s, adjU_s;
  const std::vector<uint32_t>* uid_d = &G.uid;
  const std::vector<uint32_t>* upb_d = &G.up_base;
  const std::vector<uint32_t>* adjU_d = &G.adjU;
  if (sharded) {
    uid_s.assign(id_space, kInvalid);
    upb_s.assign(id_space, kInvalid);
    for (uint64_t g = 0; g < G.N; ++g) {
      uid_s[newid[g]] = G.uid[g];
      upb_s[newid[g]] = G.up_base[g];
    }
    adjU_s.resize(G.adjU.size());
    for (size_t i = 0; i < G.adjU.size(); ++i) adjU_s[i] = dev_id(G.adjU[i]);
    uid_d = &uid_s;
    upb_d = &upb_s;
    adjU_d = &adjU_s;
  }

  // uid → device id (for the distance-batch API); uids are the base-file positions, so dense-ish
  uint32_t max_uid = 0;
  for (uint32_t u : G.uid) max_uid = std::max(max_uid, u);
  h->inv_size = max_uid + 1;
  std::vector<uint32_t> inv(h->inv_size, kInvalid);
  for (uint64_t g = 0; g < G.N; ++g) inv[G.uid[g]] = dev_id(static_cast<uint32_t>(g));

  // rows in the device layout (kernels.h permuted_index / permuted_index_bytes / fp16 rows in natural order); config 5
  // converts records to fp16 at load, byte rows narrow them losslessly (checked above)
  std::vector<uint32_t> perm(dim);
  for (uint32_t i = 0; i < dim; ++i) perm[i] = device_index(dim, elem, i);
  std::vector<uint8_t> vbytes(G.N * vrow, 0);
  {
    float* fp = reinterpret_cast<float*>(vbytes.data());
    __half* hp = reinterpret_cast<__half*>(vbytes.data());
    for (uint64_t n = 0; n < G.N; ++n) {
      const float* src = G.vec.data() + n * dim;
      uint8_t* brow = vbytes.data() + n * vrow;
      for (uint32_t i = 0; i < dim; ++i) {
        if (elem == SHINE_ELEM_F16) hp[n * dim + perm[i]] = __float2half(src[i]);
        else if (elem_is_byte(elem)) brow[perm[i]] = static_cast<uint8_t>(static_cast<int>(src[i]));
        else fp[n * dim + perm[i]] = src[i];
      }
    }
  }
  const uint8_t* vsrc = vbytes.data();
  const size_t vlen = vbytes.size();

  uint32_t pad_default = 0;  // a mapped node for slots that own no records
  for (uint32_t o = 0; o < slots; ++o)
    if (sharded && owned[o] > 0) {
      pad_default = static_cast<uint32_t>(o * U);
      break;
    }
  h->reps.resize(slots);
  for (uint32_t r = 0; r < slots; ++r) {
    Replica& R = h->reps[r];
    R.device = devs[r];
    R.slot = r;
    R.cus = static_cast<uint32_t>(std::max(1, props[r].multiProcessorCount));
    R.lds_per_cu = static_cast<uint32_t>(props[r].maxSharedMemoryPerMultiProcessor > 0
                                             ? props[r].maxSharedMemoryPerMultiProcessor
                                             : props[r].sharedMemPerBlock);
    R.pad_node = sharded && owned[r] > 0 ? static_cast<uint32_t>(r * U) : pad_default;
    HIP_TRY(hipSetDevice(R.device));
    HIP_TRY(hipStreamCreateWithFlags(&R.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&R.ev0));
    HIP_TRY(hipEventCreate(&R.ev1));
    if (!sharded) {
      if (int rc = upload(R.vec, vsrc, vlen, R.stream)) return rc;
      if (int rc = upload(R.adj0, G.adj0.data(), G.adj0.size(), R.stream)) return rc;
    }
    if (int rc = upload(R.uid, uid_d->data(), uid_d->size(), R.stream)) return rc;
    if (int rc = upload(R.up_base, upb_d->data(), upb_d->size(), R.stream)) return rc;
    if (int rc = upload(R.adjU, adjU_d->data(), adjU_d->size(), R.stream)) return rc;
    if (int rc = upload(R.inv_uid, inv.data(), inv.size(), R.stream)) return rc;
    if (int rc = R.main.counter.grow(kCallWords)) return rc;
    HIP_TRY(hipStreamSynchronize(R.stream));
  }
  const uint64_t replicated = 4 * (uid_d->size() + upb_d->size() + adjU_d->size() + inv.size());
  if (sharded) {
    // the cached prefix of every stripe: the leading cache_fraction of each array's bytes, rounded up to whole VM
    // pages of that array.  A record counts as cached when its row lies wholly inside (a row straddling the edge
    // reads partly over xGMI and counts as remote).  Rounding the two arrays to a common row count instead would
    // cost whole stripes: 400-byte fp16 rows (cfg 5) meet a 2 MiB page only every 131,072 rows.
    auto hot_bytes = [&](uint64_t stride) {
      const uint64_t b = static_cast<uint64_t>(cache_fraction * static_cast<double>(stride) + 0.5);
      return std::min<uint64_t>(stride, (b + gran - 1) / gran * gran);
    };
    const uint64_t hot_v = slots > 1 ? hot_bytes(U * vrow) : 0, hot_a = slots > 1 ? hot_bytes(U * arow) : 0;
    h->cached_rows = hot_v / vrow;
    h->cached_list_rows = hot_a / arow;
    h->cache_fraction = static_cast<double>(hot_v) / static_cast<double>(U * vrow);
    h->cache_requested = cache_fraction;
    if (int rc = map_sharded(h->svec, U * vrow, hot_v, devs, gran)) return rc;
    if (int rc = map_sharded(h->sadj0, U * arow, hot_a, devs, gran)) return rc;
    std::vector<uint8_t> vb;
    std::vector<uint32_t> rows;
    for (uint32_t o = 0; o < slots; ++o) {
      const auto& ord = order[o];
      if (ord.empty()) continue;
      vb.resize(ord.size() * vrow);
      rows.resize(ord.size() * M0);
      for (size_t i = 0; i < ord.size(); ++i) {
        std::memcpy(&vb[i * vrow], vsrc + static_cast<uint64_t>(ord[i]) * vrow, vrow);
        for (uint32_t j = 0; j < M0; ++j) rows[i * M0 + j] = dev_id(G.adj0[static_cast<uint64_t>(ord[i]) * M0 + j]);
      }
      HIP_TRY(hipSetDevice(devs[o]));  // through slot o's own view: its stripe is local there
      HIP_TRY(hipMemcpy(h->svec.view[o].va + o * U * vrow, vb.data(), vb.size(), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(h->sadj0.view[o].va + o * U * arow, rows.data(), rows.size() * 4, hipMemcpyHostToDevice));
    }
    if (int rc = fill_copies(h->svec, devs)) return rc;
    if (int rc = fill_copies(h->sadj0, devs)) return rc;
    h->device_bytes = U * (vrow + arow) + (slots - 1) * (hot_v + hot_a) + replicated;
  } else {
    h->device_bytes = vlen + 4 * G.adj0.size() + replicated;
  }
  if (sharded) {
    h->devs = devs;
    h->uid_of_dev = std::move(uid_s);
    h->dev_of_uid = std::move(inv);
    if (h->cached_rows || h->cached_list_rows) {  // a warmup may re-rank the stripes: keep what it relays out
      h->dev_of = std::move(newid);
      h->host = std::move(G);
    }
  }
  *out = h.release();
  return SHINE_OK;
}

// Launch shapes and the pass chain.  Each search runs as up to three passes enqueued back to back on one stream,
// every pass handing the queries it could not hold to the next through a device list (no host round trip):
//   main    fast mode: the sorted-list kernel, visited table in LDS (PASS_FAST); exact mode: both std heaps and
//           the visited table in LDS, one wavefront per query up to 16 per CU (PASS_LDS).
//   light   visited set as a bitmap in HBM, heaps in a 16 KiB LDS share (kLightFixupLds), so its workgroups fit
//           beside the main pass of another batch in flight instead of waiting for a drained CU.
//   global  visited bitmap and both heaps in HBM: no capacity limit short of kGlobalNextCap entries, slow per
//           heap operation, sized for the few queries the light pass cannot hold.
// The whole-CU pass (16K-entry LDS table, PASS_WHOLE_CU) is reachable only through SHINE_DEBUG_START_MODE=1.
enum PassKind { PASS_LDS = 0, PASS_WHOLE_CU = 1, PASS_LIGHT = 2, PASS_GLOBAL = 3, PASS_FAST = 4 };

struct LaunchShape {
  uint32_t cap, grid, vis_cap, vis_limit;
  uint32_t waves;            // wavefronts per CU the LDS shares allow
  uint32_t tight;            // exact pass: 1 = the tight next_candidates room was taken (pick_shape)
  uint32_t vis16, vis_bits;  // fast kernel: u16 quotient visited entries over a vis_bits-bit id space
};

// spilled visited tables a main pass (fast or exact) may hold at once (SearchArgs::spill_flags)
constexpr uint32_t kSpillSlots = 64;
constexpr uint64_t kXcdL2Bytes = 4ull << 20;  // L2 of one XCD (MI355X_MICROARCH.md)
bool spill_enabled();

// the inverse of an odd multiplier mod 2^32 (Newton: each step doubles the correct low bits)
uint32_t inverse_odd(uint32_t m) {
  uint32_t x = m;  // correct to 3 bits: m * m == 1 (mod 8)
  for (int i = 0; i < 4; ++i) x *= 2u - m * x;
  return x;
}

uint32_t pow2_at_least(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

uint32_t log2_ceil(uint32_t x) {
  uint32_t l = 0;
  while ((1u << l) < x) ++l;
  return l;
}

int64_t env_int(const char* name, int64_t dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoll(e) : dflt;
}

// the main passes continue a query whose visited table overflows in an HBM bitmap (SHINE_DEBUG_NO_SPILL=1: hand it
// to the light pass instead, the round-2 behaviour)
bool spill_enabled() { return env_int("SHINE_DEBUG_NO_SPILL", 0) == 0; }

// A spilled table goes to a hash table in its spill slot (kernels_impl.h SpillSet) where the id-space bitmap would
// outgrow an XCD's L2 (> 32M ids); SHINE_SPILL_HASH = 0 / 1 forces the bitmap / the hash table (tests, A/B).
constexpr uint32_t kSpillHashMax = 65536;  // entries (256 KB): 8 x the largest table it takes over, load <= 1/2
bool spill_hashed(const shine_index* h) {
  const int64_t f = env_int("SHINE_SPILL_HASH", -1);
  return f == 1 || (f < 0 && 4ull * h->words_per_slot > kXcdL2Bytes);
}
// Hash entries for a main-pass table of vis_cap entries: 8 x, 16,384 to 65,536 (a spilled query hands itself on at
// half of it, beyond any query seen at these sizes).
uint32_t spill_hash_entries(uint32_t vis_cap) {
  return std::min<uint32_t>(kSpillHashMax, std::max<uint32_t>(16384, pow2_at_least(8 * std::max<uint32_t>(vis_cap, 1))));
}
// Two-choice u32 buckets (kernels_impl.h VisitedLds<3>) where the linear-probed u32 table would be used beyond L2 (the
// 26-27-bit id spaces of cfg 4 / cfg 5), at a load of SHINE_VT3_LOAD / 1000 (vt3_load_permille) at the mean query, grown to
// the largest table at the same wavefronts per CU: an insert is one read of both buckets and one compare-and-swap
// whatever the load, so the table runs fuller than the u32 rule's 0.45 and more wavefronts share a CU.  Compiled for
// replicas only (no read accounting); SHINE_VT3 = 0 turns it off, 1 forces it on the fast pass too (A/B).
bool vt3_usable(const shine_index* h) {
  const bool sharded = h->placement != SHINE_PLACE_REPLICA && h->reps.size() > 1;
  return !sharded && env_int("SHINE_VT3", 1) != 0;
}
// Loads measured on the 50M TTI-shaped index (profiles/r06/scale_cfg5_vt3_*.jsonl): fast 0.6 (7,488 entries, 5 wavefronts
// per CU) 1.41 M QPS, 0.7 (5,952, 6) 1.81 M, 0.85 (4,928, 7) 1.82 M once no call hands queries on; exact 0.6 0.63 M, 0.7
// 0.61 M (linear-probed u32 at 0.45: 1.42 M / 0.41 M).
uint32_t vt3_load_permille(bool fast) {
  const int64_t v = fast ? env_int("SHINE_VT3_LOAD", 700) : env_int("SHINE_VT3_EXACT_LOAD", env_int("SHINE_VT3_LOAD", 600));
  return static_cast<uint32_t>(std::min<int64_t>(950, std::max<int64_t>(100, v)));
}

// Words per spill / fallback slot: the id-space bitmap, or at least the largest hash table; a multiple of 4 words, so
// that every slot starts 16-byte aligned (spill_release clears a hash table with 16-byte stores from the slot base).
uint64_t slot_words(const shine_index* h) {
  const uint64_t w = spill_hashed(h) ? std::max<uint64_t>(h->words_per_slot, kSpillHashMax) : h->words_per_slot;
  return (w + 3) / 4 * 4;
}

// Fast mode: the sorted list lives in VGPRs, LDS holds only the visited table.  The table holds between pow2(40·ef)
// and pow2(48·ef) entries (a query visits ~5-20·ef nodes; one that fills 7/8 of it goes to the light pass).  The
// shape aims at the wavefronts of two batches being resident together (the next batch in flight runs beside this
// one instead of waiting for LDS): for each entry width — u32 keys, or u16 quotient entries (VisitedLds<1>) when
// the id space fits them — the largest table that allows that many wavefronts per CU is taken, and the width with
// more resident wavefronts, then the larger table, wins; u32 on a tie (its inserts take fewer LDS round trips:
// measured 8.7 M vs 6.0 M QPS at ef = 32, where both fit; 4.26 M vs 3.89 M at ef = 128, where only u16 does).
// Visited-table entries learned from the previous call on a stream: the most nodes one of its queries marked visited
// (queries the main pass handed on count in full: the fallback passes record them too), with room to spare (tables
// are used to 7/8 and the next batch may visit more: >= 1.625x), never below the floor a learned table that
// overflowed has set; 0 when there is nothing to learn from (first call on the stream, or the previous one ran at
// another ef).  Fixed shapes size tables
// from ef alone: DEEP-shaped 1M records at ef = 256 visit at most ~3.8K nodes, and 8K entries instead of 16K run
// 1.6-1.8x faster (profiles/r02/cfg3_table_size.txt); SIFT-shaped at ef = 32 outgrow the fixed 2K entries.
uint32_t learned_table(const Scratch& S) {
  if (!S.seen.p || !S.seen.p[3] || env_int("SHINE_DEBUG_NO_LEARN", 0)) return 0;
  const uint32_t vmax = S.seen.p[4];
  if (vmax == 0) return 0;
  return std::min<uint32_t>(16384, std::max<uint32_t>({1024u, S.table_floor, pow2_at_least(vmax + vmax / 2 + vmax / 8)}));
}

// With the in-place spill a table need only hold the typical query of the stream: pow2(1.25 x the previous call's
// mean visited count + 64) — a query beyond it spills and goes on in an HBM bitmap.  The mean, not the maximum: on the
// DEEP-shaped 10M index at ef = 256 a query visits 2.9K nodes on average but up to 7K (profiles/r02/
// config_lines_cfg3_10m_final.jsonl), and a table sized for the maximum holds half the wavefronts per CU.  Never below
// the floor a call that exhausted the spill bitmaps set.
// The previous call's mean visited count per query (0: nothing to learn from; see learned_mean_table)
uint32_t mean_visits(const Scratch& S) {
  if (!S.seen.p || !S.seen.p[3] || env_int("SHINE_DEBUG_NO_LEARN", 0)) return 0;
  const uint32_t nq = S.seen.p[6];
  return nq == 0 || nq >= (1u << 18) ? 0u : S.seen.p[5] / nq;
}

uint32_t learned_mean_table(const Scratch& S) {
  // (the visited sum is a u32 word of per-query counts capped at 16,384: calls of fewer than 2^18 queries cannot wrap
  // it — 2^18 x 2^14 is 2^32; seen[6] is the queries of the call that wrote the sum, which need not be the last one
  // enqueued)
  if (!S.seen.p || !S.seen.p[3] || env_int("SHINE_DEBUG_NO_LEARN", 0)) return 0;
  const uint32_t nq = S.seen.p[6];
  if (nq == 0 || nq >= (1u << 18)) return 0;
  const uint32_t mean = S.seen.p[5] / nq;
  if (mean == 0) return 0;
  return std::min<uint32_t>(16384, std::max<uint32_t>({1024u, S.table_floor, pow2_at_least(mean + mean / 4 + 64)}));
}

// The fast table where the spill target is HBM beyond L2 (large id spaces, see enqueue_search): u32 entries
// (VisitedLds<0>, any multiple of 64), sized for a load of 0.45 at the stream's mean query and then grown to the
// largest table that keeps the same wavefronts per CU.  A linear-probed table's probe chains, walked in lockstep by the
// wave's 32 list slots, lengthen with the load faster than residency pays for it: on the 100M-record index at ef = 128
// (mean 2,524 visits) 6,144 entries at 6 wavefronts per CU (load 0.41) ran at 4.75-4.83 M QPS, against 4.18 M for
// 5,120 at 7 (0.49, no query spilling in the timed batches), 3.35 M for 4,096 at 8 (0.62), 4.33 M for 7,168 at 5 and
// 3.79 M for 8,192 at 4; at d = 200, ef = 250 on 50M ids (mean 4,200) 9,536 entries at 4 per CU (0.44) ran at 1.45 M
// against 1.38 M for 7,488 at 5, 1.39 M for 8,192 at 4 and 1.21-1.24 M at 3 (profiles/r05/scale_cfg4_viscap*.jsonl,
// scale_cfg5_viscap*.jsonl).  The few queries that outgrow the table spill in place to the L2 hash set.
// SHINE_FAST_TABLE_POW2=1: the round-4 rule (the power of two 9/8 above the last call's worst query).
uint32_t learned_max_table(const Scratch& S, uint32_t ef, uint32_t lds_per_cu, uint32_t waves_wanted,
                           uint32_t load_permille = 450) {
  if (!S.seen.p || !S.seen.p[3] || env_int("SHINE_DEBUG_NO_LEARN", 0)) return 0;
  auto clampt = [&](uint64_t t) {
    return std::min<uint32_t>(16384, std::max<uint32_t>({1024u, S.table_floor, static_cast<uint32_t>(std::min<uint64_t>(t, 16384))}));
  };
  if (env_int("SHINE_FAST_TABLE_POW2", 0)) {
    const uint64_t vmax = S.seen.p[4];
    return vmax ? clampt(pow2_at_least(static_cast<uint32_t>(std::min<uint64_t>(16384, vmax * 9 / 8)))) : 0;
  }
  const uint32_t nq = S.seen.p[6];  // (the mean as learned_mean_table reads it)
  if (nq == 0 || nq >= (1u << 18) || S.seen.p[5] == 0) return 0;
  const uint64_t mean = S.seen.p[5] / nq;
  const uint64_t overhead = search_fast_lds_bytes(0, ef, 4);
  auto waves = [&](uint64_t t) { return lds_per_cu / lds_alloc_bytes(search_fast_lds_bytes(static_cast<uint32_t>(t), ef, 4)); };
  auto largest_at = [&](uint64_t w) -> uint64_t {  // the largest multiple of 64 entries holding w wavefronts per CU
    const uint64_t per = lds_per_cu / w / 1024 * 1024;
    return per > overhead + 256 ? (per - overhead) / 4 / 64 * 64 : 0;
  };
  const uint64_t want = (mean * 1000 / std::max<uint32_t>(100, load_permille) + 63) / 64 * 64;  // (0.45: the u32 rule)
  // (no more wavefronts per CU than two batches of this call's size put there: a small call takes a larger table)
  const uint64_t w = std::max<uint64_t>(1, std::min<uint64_t>(waves(want), waves_wanted));
  return clampt(std::max(want, largest_at(w)));
}

// The exact pass's learned table, with the in-place spill: just the previous call's worst query (eighths/8 × its
// visited count, SHINE_EXACT_LEARN_EIGHTHS, default 8), never below 2,048 entries (SHINE_EXACT_LEARN_MIN), which then
// replaces the fixed size in either direction — a query beyond it spills in place instead of being re-run.  At
// ef = 128 on the bench's index that is 4,096 entries and 11 wavefronts per CU instead of 8,192 and 7: 3.51 M against
// 2.38 M QPS (profiles/r03/exact_learned_scan.jsonl); at ef = 32 a 1,024-entry table spilled too often (9.7 M against
// 10.6 M), hence the floor.  No margin above the worst query: with 9/8 (rounds 3-4) a batch whose worst query visits
// 3,851 nodes put the next call on its stream on 8,192 entries, and that one slow launch set the time of a 20-step run
// (warmup 5: 3.19 M against 3.64 M QPS with 8/8; 200 steps: 3.74 M against 3.96 M, profiles/r05/k20_exact_eighths.jsonl)
// — the few queries past the table's 7/8 load spill in place.  The worst query of the slot's recent calls on all its
// streams (Replica::vmax_recent), as the fast table: one stream's last call flipped the 100M-record index's table
// between 4,096 and 8,192 entries (exact 1.29 M against 1.46 M QPS, profiles/r05/scale_cfg4_rule.jsonl).  Without the
// spill: learned_table (1.625 ×).
uint32_t learned_exact_table(const Scratch& S, uint32_t ef, uint32_t recent_vmax) {
  if (!spill_enabled()) return learned_table(S);
  if (!S.seen.p || !S.seen.p[3] || env_int("SHINE_DEBUG_NO_LEARN", 0)) return 0;
  const uint64_t vmax = std::max(S.seen.p[4], recent_vmax);
  if (vmax == 0) return 0;
  // at ef <= 32 the tables are small and a half-empty one probed faster than a fuller one (10.6 M against 9.7 M QPS
  // at ef = 32, profiles/r03/exact_learned_scan_floor.jsonl): the round-2 margin there
  const uint64_t eighths =
      static_cast<uint64_t>(std::max<int64_t>(6, env_int("SHINE_EXACT_LEARN_EIGHTHS", ef <= 32 ? 13 : 8)));
  const uint64_t want = std::min<uint64_t>(16384, vmax * eighths / 8);
  const uint32_t lo = static_cast<uint32_t>(std::max<int64_t>(1024, env_int("SHINE_EXACT_LEARN_MIN", 2048)));
  return std::min<uint32_t>(16384, std::max<uint32_t>({lo, S.table_floor, pow2_at_least(static_cast<uint32_t>(want))}));
}

LaunchShape pick_fast_shape(uint32_t nq, uint32_t ef, uint32_t cus, uint32_t lds_per_cu, uint64_t id_space,
                            uint32_t learned = 0, bool grow = false, bool byte_rows = false, uint32_t vt3_table = 0) {
  LaunchShape sh{};
  const uint32_t want = std::max<uint32_t>(1, std::min<uint32_t>(16, (nq + cus - 1) / cus));
  // Waves per CU the tables are sized for, in batches of `want`, and the table floor per ef.  f32 rows: two batches,
  // pow2(40·ef) entries.  Byte rows at ef > 64 move a quarter of the bytes per distance over long searches, so the
  // kernel is latency-bound there and residency pays: four batches (12-16 wavefronts per CU at batch 1,024) and
  // pow2(24·ef) entries, the few queries that outgrow them spilling in place (SearchArgs::spill_flags) — u8 rows at
  // ef = 128: 8.26-8.28 M against 7.78-7.79 M QPS; at ef = 48 the same policy lost 17 % (17.3 M against 20.8 M), f32
  // rows lose at ef = 128 (6.34 M against 6.69 M) (profiles/r03/ab1_merge_spill_tables.jsonl,
  // lib_probe_v16_tables.jsonl).  The environment overrides both (tuning).
  const bool wide_residency = byte_rows && ef > 64;
  const uint32_t target = std::min<uint32_t>(
      16, static_cast<uint32_t>(env_int("SHINE_FAST_TARGET_BATCHES", wide_residency ? 4 : 2)) * want);
  // with f32 rows a table below pow2(40·ef) entries costs more than its residency buys
  const uint32_t per_ef =
      static_cast<uint32_t>(std::max<int64_t>(1, env_int("SHINE_FAST_TABLE_PER_EF", wide_residency ? 24 : 40)));
  uint32_t lo = std::min<uint32_t>(16384, std::max<uint32_t>(2048, pow2_at_least(per_ef * ef)));
  // what the previous call's queries needed: a smaller table, or a larger one once the fixed size overflowed
  if (learned && (learned < lo || grow)) lo = learned;
  const uint32_t hi = std::min<uint32_t>(16384, std::max<uint32_t>(lo, pow2_at_least(48 * ef)));
  uint32_t bits = 14;
  while (bits < 32 && (1ull << bits) < id_space) ++bits;
  auto log2u = [](uint32_t x) { uint32_t l = 0; while ((1u << l) < x) ++l; return l; };
  auto table_for = [&](uint32_t entry_bytes) {
    const int64_t budget = static_cast<int64_t>(lds_per_cu / target) - static_cast<int64_t>(search_fast_lds_bytes(0, ef));
    uint32_t fit = 1024;
    while (static_cast<int64_t>(fit) * 2 * entry_bytes <= budget) fit *= 2;
    return std::max(lo, std::min(hi, fit));
  };
  auto resident = [&](uint32_t t, uint32_t entry_bytes) {
    return std::min<uint64_t>(target, lds_per_cu / lds_alloc_bytes(search_fast_lds_bytes(t, ef, entry_bytes)));
  };
  // test hook: the id space the u16 entries are sized for, widened (SHINE_DEBUG_VIS_BITS=24 puts a small index's ids
  // through the full 15-bit remainders of 4,096-entry two-choice tables)
  bits = std::max<uint32_t>(bits, static_cast<uint32_t>(std::min<int64_t>(31, env_int("SHINE_DEBUG_VIS_BITS", 0))));
  // u16 entries: in linear-probed buckets (VisitedLds<1>, >= 3 distance bits) where the id space allows, else in
  // two-choice buckets (VisitedLds<2>, a 15-bit remainder and a bucket bit); SHINE_DEBUG_VIS16 = 0 / 1 / 2 forces
  auto kind16 = [&](uint32_t t) -> uint32_t {
    return bits <= log2u(t) + 10 ? 1u : bits <= log2u(t) + 12 ? 2u : 0u;
  };
  const uint32_t t32 = table_for(4), t16 = pow2_at_least(table_for(2));  // (a learned size may not be a power of two)
  const int64_t force16 = env_int("SHINE_DEBUG_VIS16", -1);
  const bool can16 = force16 != 0 && kind16(t16) != 0 && (kind16(t16) == 1 || env_int("SHINE_TWO_CHOICE", 1) != 0);
  const uint64_t w32 = resident(t32, 4), w16 = can16 ? resident(t16, 2) : 0;
  // at equal residency the larger u16 table wins; in two-choice buckets only where it holds twice the u32 table's
  // entries (the u32 one is then the spilling half-size table): a two-choice lookup reads two buckets and plans its
  // insert, dearer than a u32 probe — TTI-shaped 50M: 16,384 two-choice entries ran at 1.35 M QPS against 8,192-9,216
  // u32 entries (the worst query's size) at 1.55 M, both 4 wavefronts per CU (profiles/r04/scale_v7); at 10M 8,192
  // two-choice entries against 4,096 u32 ones, 2.45 M against 2.14 M
  // (linear-probed u16 buckets win every tie: at ef <= 32 the round-1 rule took u32 tables on a tie, and u16 ran
  // 1.21-1.33x faster there — ef = 16 / 32: 18.5 M / 15.1 M QPS against 13.9 M / 12.5 M, profiles/r05/ef_floor.jsonl)
  const bool tie16 = w16 == w32 && (kind16(t16) == 1 ? t16 >= t32 : t16 >= 2 * t32);
  sh.vis16 = can16 && (w16 > w32 || tie16) ? kind16(t16) : 0;
  if (force16 >= 1 && can16) sh.vis16 = kind16(t16);  // test hook: force the u16 entries
  sh.vis_cap = sh.vis16 ? t16 : t32;
  const bool viscap_hook = std::getenv("SHINE_DEBUG_VISCAP") != nullptr;
  sh.vis_cap = static_cast<uint32_t>(env_int("SHINE_DEBUG_VISCAP", sh.vis_cap));  // test hook
  // a forced table size: the entries it allows (0: back to u32; u16 buckets need a power of two)
  if (sh.vis16) sh.vis16 = (sh.vis_cap & (sh.vis_cap - 1)) == 0 ? kind16(sh.vis_cap) : 0u;
  if (force16 == 2 && bits <= log2u(sh.vis_cap) + 12) sh.vis16 = 2;  // test hook: two-choice
  // two-choice u32 buckets: the learned table of vt3_usable indexes beyond L2 (enqueue_search) unless a test hook fixes
  // the table, or forced at any id space and table size (test hook SHINE_DEBUG_VIS16=3; whole buckets)
  if (vt3_table && force16 < 0 && !viscap_hook) {
    sh.vis16 = 3;
    sh.vis_cap = vt3_table;
  }
  if (force16 == 3) sh.vis16 = 3;
  if (sh.vis16 == 3) sh.vis_cap = std::max<uint32_t>(64, sh.vis_cap / 4 * 4);
  sh.vis_bits = std::max(bits, log2u(sh.vis_cap) + 1);
  const uint64_t need = lds_alloc_bytes(search_fast_lds_bytes(sh.vis_cap, ef, vis_entry_bytes(sh.vis16)));
  const uint32_t fit = std::max<uint32_t>(1, static_cast<uint32_t>(lds_per_cu / need));
  const uint32_t wpc = std::max<uint32_t>(1, std::min<uint32_t>({(nq + cus - 1) / cus, 16u, fit}));
  sh.cap = 0;
  // test hook: the table's load limit in 1/1000 (a query that visits more goes to the light pass)
  const int64_t load = env_int("SHINE_DEBUG_VISLOAD", 875);
  sh.vis_limit = static_cast<uint32_t>(std::min<int64_t>(sh.vis_cap - 64, static_cast<int64_t>(sh.vis_cap) * load / 1000));
  sh.grid = std::max<uint32_t>(1, std::min<uint32_t>(nq, cus * wpc));
  return sh;
}

// LDS share of the light pass.  next_candidates holds (16 KiB - top - 512 B) / 8 entries (>= 1,470 at ef <= 512);
// a query that outgrows it goes on to the global-heap pass.
constexpr uint64_t kLightFixupLds = 16384;

// Visited-bitmap slots the fallback passes may use on this index (kBitmapBudget of HBM per stream).
uint32_t bitmap_slot_cap(const shine_index* h) {
  const uint64_t per = std::max<uint64_t>(1, h->words_per_slot * 4);
  return static_cast<uint32_t>(std::max<uint64_t>(kGlobalSlots, std::min<uint64_t>(1u << 20, kBitmapBudget / per)));
}

// handed: queries the main pass handed on in an earlier call on this stream.  The light pass gets slots for twice
// that (at least one per CU, at most what LDS shares and bitmap memory allow): its workgroups of a call with few
// overflows exit at once, and a launch of thousands of them delays the stream's next batch (-7 % QPS at ef = 32).
// room8: next_candidates' room the exact pass reserves per wavefront, in eighths of ef (0: the fixed 5 ef with u16
// tables and 4 ef with u32); see pick_shape below
LaunchShape pick_shape_room(const shine_index* h, const Replica& R, uint32_t nq, uint32_t ef, int pass, uint32_t handed,
                            uint32_t learned, uint32_t learned_mean, uint32_t mean_visits, int64_t room8) {
  LaunchShape sh{};
  const uint64_t top_bytes = align16(8ull * ef);
  const uint32_t cus = R.cus, lds = R.lds_per_cu;
  if (pass == PASS_GLOBAL) {
    sh.vis_cap = 0;
    sh.cap = static_cast<uint32_t>(env_int("SHINE_DEBUG_GLOBAL_CAP", kGlobalNextCap));  // test hook
    sh.grid = std::max<uint32_t>(1, std::min<uint32_t>({nq, kGlobalSlots, bitmap_slot_cap(h)}));
    return sh;
  }
  uint32_t wpc = 1;
  uint64_t budget = lds;
  if (pass == PASS_LDS) {
    // u16 quotient entries (VisitedLds<1>) when the id space fits them and they let more wavefronts share a CU with
    // next_candidates still >= 5·ef entries (u32: 4·ef).  Tables of pow2(48·ef) entries, or the previous call's
    // most-visited query, sized for the wavefronts of two batches in flight.  Smaller tables for four batches
    // (pow2(24·ef): 4,096 entries and up to 11 wavefronts per CU at ef = 128 instead of 8,192 and 7), with the
    // in-place spill catching the queries that outgrow them, were slower: 1.76-1.84 M against 1.94 M QPS
    // (profiles/r03/ab1_merge_spill_tables.jsonl).  But where the table sized for the worst query leaves fewer than
    // four wavefronts per CU, the mean-sized one (learned_mean) is taken: DEEP-shaped 10M ids at ef = 256, 16,384
    // u16 entries and 3 wavefronts per CU against 4,096 u32 entries and 6, 0.48 M against 0.72 M QPS
    // (profiles/r03/config_lines_cfg3_10m*.jsonl).  Tuning hooks: the two env knobs.
    const uint32_t per_ef = static_cast<uint32_t>(std::max<int64_t>(1, env_int("SHINE_EXACT_TABLE_PER_EF", 48)));
    const uint32_t batches = static_cast<uint32_t>(std::max<int64_t>(1, env_int("SHINE_EXACT_TARGET_BATCHES", 3)));
    const uint32_t want = std::min<uint32_t>(batches * ((nq + cus - 1) / cus), 16u);
    uint32_t bits = 14;
    while (bits < 32 && (1ull << bits) < h->id_space) ++bits;
    bits = std::max<uint32_t>(bits, static_cast<uint32_t>(std::min<int64_t>(31, env_int("SHINE_DEBUG_VIS_BITS", 0))));
    // entry width and resident wavefronts for a table size.  u16 entries: linear-probed buckets (VisitedLds<1>), or
    // two-choice buckets (VisitedLds<2>) where the id space leaves no distance bits (two_choice).  The exact kernel's
    // insert has no look-ahead plan, so two-choice pays the guess, a read of both buckets and the swap: on the table
    // sized for the worst query it only lost (cfg 3: 8,192 entries, 0.89 M against 1.14 M QPS on u32), but on the
    // mean-sized table (below) its halved bytes put a seventh wavefront on each CU and make room for next_candidates:
    // 1.28 M against 1.14 M, and the hand-ons for next_candidates capacity drop from 6-13 to 0-1 per call
    // (profiles/r04/env_scan_cfg3_exact.jsonl).  SHINE_EXACT_TWO_CHOICE = 0 / 1 turns it off / on for both sizes.
    // next_candidates' room (pick_shape), reserved when wavefronts are counted; the leftover LDS goes to it in the end
    uint32_t next16 = 5 * ef, next32 = 4 * ef;
    if (room8 > 0) next16 = next32 = std::max<uint32_t>(static_cast<uint32_t>((room8 * ef + 7) / 8), ef + 2 * h->M0);
    auto fit = [&](uint32_t vis_cap, uint32_t& vis16, bool two_choice) {
      auto waves = [&](uint64_t need) {
        return std::max<uint32_t>(1, std::min<uint32_t>(want, static_cast<uint32_t>(lds / need)));
      };
      const uint32_t w32 = waves(search_lds_bytes(ef, next32, vis_cap, 4));
      const uint32_t w16 = waves(search_lds_bytes(ef, next16, vis_cap, 2));
      const int64_t tc = env_int("SHINE_EXACT_TWO_CHOICE", -1);
      const uint32_t kind = bits <= log2_ceil(vis_cap) + 10                                        ? 1u
                            : bits <= log2_ceil(vis_cap) + 12 && (tc == 1 || (tc < 0 && two_choice)) ? 2u
                                                                                                   : 0u;
      const int64_t force16 = env_int("SHINE_DEBUG_VIS16", -1);
      const bool can16 = force16 != 0 && kind != 0;
      vis16 = can16 && (w16 > w32 || force16 >= 1) ? kind : 0;
      if (force16 == 2 && bits <= log2_ceil(vis_cap) + 12) vis16 = 2;  // test hook: two-choice
      if (force16 == 3) vis16 = 3;                                       // test hook: two-choice u32 buckets
      return vis16 == 1 || vis16 == 2 ? w16 : w32;
    };
    sh.vis_cap = std::min<uint32_t>(16384, std::max<uint32_t>(1024, pow2_at_least(per_ef * ef)));
    // a learned size replaces the fixed one: with the spill in either direction, else only to shrink (or to grow
    // after a call that handed queries on)
    if (learned && (spill_enabled() || learned < sh.vis_cap || (handed != 0xFFFFFFFFu && handed > 0)))
      sh.vis_cap = learned;
    wpc = fit(sh.vis_cap, sh.vis16, false);
    if (wpc < 4 && learned_mean && learned_mean < sh.vis_cap && spill_enabled()) {
      uint32_t v16 = 0;
      const uint32_t w = fit(learned_mean, v16, true);
      if (w > wpc) {
        sh.vis_cap = learned_mean;
        sh.vis16 = v16;
        wpc = w;
      }
    }
    // Where spills go to the hash set beyond L2 (100M / 50M ids: u32 entries), the fast pass's table rule (learned_max_
    // table): load 0.45 at the mean query, grown to the largest u32 table at the same wavefronts per CU, next_candidates
    // keeping 5 · ef entries — taken only where it puts more wavefronts on a CU than the table above: 100M ids at
    // ef = 128, 6,528 entries and 5 per CU against 8,192 and 4, 1.51 M against 1.42 M QPS; at 50M ids and ef = 250 it
    // holds the same 3 per CU with less room for next_candidates and ran at 0.38 M against 0.41 M
    // (profiles/r05/scale_cfg{4,5}_exact_rule.jsonl).
    // Two-choice u32 buckets (vt3_usable) take the same rule at their higher load (SHINE_VT3_LOAD).
    const bool vt3 = vt3_usable(h);
    if (mean_visits && sh.vis16 == 0 && spill_enabled() && spill_hashed(h) && env_int("SHINE_EXACT_LOAD_RULE", 1)) {
      const uint64_t fixed = top_bytes + align16(8ull * std::min<uint32_t>(next16, 5 * ef)) + 512;
      auto waves = [&](uint64_t t) {
        return std::min<uint64_t>(want, lds / lds_alloc_bytes(fixed + align16(4ull * t)));
      };
      // (t0: the table at the load; w: the wavefronts it leaves; t: the largest table at w)
      auto rule = [&](uint32_t load_permille, uint64_t& t0, uint64_t& w, uint64_t& t) {
        t0 = (static_cast<uint64_t>(mean_visits) * 1000 / load_permille + 63) / 64 * 64;
        w = std::max<uint64_t>(1, waves(t0));
        const uint64_t per = lds / w / 1024 * 1024;
        t = per > fixed + 4096 ? std::min<uint64_t>(16384, (per - fixed) / 4 / 64 * 64) : 0;
      };
      uint64_t t0 = 0, w = 0, t = 0;
      rule(vt3 ? vt3_load_permille(false) : 450, t0, w, t);
      // two-choice tables where the load leaves 4 wavefronts per CU or fewer: a fuller table (0.72) for one more
      // wavefront — cfg 5 50M exact 0.75 -> 0.79 M; at cfg 4's 7 per CU 0.72 lost (1.81 against 1.90 M,
      // profiles/r06/exact/scale_cfg*_vt3_exact_load_scan.jsonl).  SHINE_VT3_EXACT_LOAD sets the load outright.
      if (vt3 && w <= 4 && !std::getenv("SHINE_VT3_EXACT_LOAD") && !std::getenv("SHINE_VT3_LOAD")) {
        uint64_t t0b = 0, wb = 0, tb = 0;
        rule(720, t0b, wb, tb);
        if (wb > w && tb >= t0b && tb >= 1024) {
          t0 = t0b;
          w = wb;
          t = tb;
        }
      }
      if (t >= t0 && t >= 1024 && w > wpc) {
        sh.vis_cap = static_cast<uint32_t>(t);
        sh.vis16 = vt3 ? 3u : 0u;
        wpc = static_cast<uint32_t>(w);
      }
    }
    // beyond L2 every u32 table of a replica takes two-choice buckets: an insert costs one read and one swap where a
    // linear probe chain grows with the load (the worst queries fill the tables learned from them)
    if (vt3 && sh.vis16 == 0 && spill_enabled() && spill_hashed(h)) sh.vis16 = 3;
    if (const char* e = std::getenv("SHINE_DEBUG_VISCAP")) {  // test hook
      sh.vis_cap = static_cast<uint32_t>(std::atoll(e));
      wpc = fit(sh.vis_cap, sh.vis16, false);
    }
    if (sh.vis16 == 3) sh.vis_cap = std::max<uint32_t>(64, sh.vis_cap / 4 * 4);  // whole buckets
    sh.vis_bits = std::max(bits, log2_ceil(sh.vis_cap) + 1);
    budget = (lds / wpc) & ~15u;
  } else if (pass == PASS_WHOLE_CU) {
    sh.vis_cap = 16384;
  } else {  // PASS_LIGHT: as many slots as the LDS shares allow, capped by the HBM its bitmaps take
    sh.vis_cap = 0;
    budget = kLightFixupLds;
    wpc = static_cast<uint32_t>(env_int("SHINE_DEBUG_LIGHT_WPC", std::max<uint32_t>(1, static_cast<uint32_t>(lds / kLightFixupLds))));
  }
  const int64_t vis_bytes = static_cast<int64_t>(align16(static_cast<uint64_t>(vis_entry_bytes(sh.vis16)) * sh.vis_cap));
  const int64_t cap = (static_cast<int64_t>(budget) - static_cast<int64_t>(top_bytes) - vis_bytes - 512) / 8;
  sh.cap = static_cast<uint32_t>(std::max<int64_t>(cap & ~1ll, 2));
  if (pass == PASS_LDS) sh.cap = static_cast<uint32_t>(std::max<int64_t>(1, env_int("SHINE_DEBUG_CAP", sh.cap)));
  if (pass == PASS_LIGHT) sh.cap = static_cast<uint32_t>(std::max<int64_t>(1, env_int("SHINE_DEBUG_LIGHT_CAP", sh.cap)));
  // linear probing stays short, and one expansion's fresh ids (up to M0) always find free slots: the u32 table's insert
  // has no overflow exit (a 64-entry table, forced by the test hook at M0 = 16, filled up and probed forever)
  sh.vis_limit = std::min<uint32_t>(sh.vis_cap / 8 * 7, sh.vis_cap > h->M0 ? sh.vis_cap - h->M0 : 0u);
  sh.grid = std::max<uint32_t>(1, std::min<uint32_t>(nq, cus * wpc));
  sh.waves = wpc;
  if (pass == PASS_LIGHT) {
    sh.grid = std::min(sh.grid, bitmap_slot_cap(h));
    // at least 64 slots: a call whose main pass hands on nothing launches few workgroups that exit at once (64
    // instead of one per CU: +0.8 % at ef = 128 with four batches in flight, profiles/r02/fallback_launch_cost.txt)
    const uint64_t floor_grid = static_cast<uint64_t>(std::max<int64_t>(1, env_int("SHINE_DEBUG_LIGHT_MIN_GRID", 64)));
    const uint64_t want = std::max<uint64_t>(floor_grid, (2ull * handed + 63) / 64 * 64);
    sh.grid = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(sh.grid, want)));
  }
  return sh;
}

// The exact pass's next_candidates room.  A query that outgrows the capacity is handed on to the next pass.  How
// large next_candidates grows depends on the data: the oracle's largest on a TTI-shaped index is 1.4 ef on average
// and 2.3 ef at most (ef = 128, 250), on a SIFT-shaped one 2.2 and 3.5 ef (ef = 128), 2.6 and 4.3 ef at ef = 64 — a
// heavy tail, so the most any recent query held (reported in call word 10) would reserve for the outliers.  The fixed
// 5 ef (u16 tables) / 4 ef (u32) stay where they leave more than 8 wavefronts per CU; at 8 or fewer 3 ef is taken
// unless it leaves fewer: another wavefront or two on each CU (cfg 3: 7 -> 9) or a larger table at the same count (cfg
// 5: 4 per CU, 7,104 -> ~7,900 two-choice u32 entries), the few queries past it handed on: exact cfg 5 (50M) 0.65-0.68
// -> 0.74 M, cfg 3 (10M) 1.34 -> 1.69 M, cfg 4 (100M) 1.52 -> 1.92 M QPS.  At the SIFT-shaped bench (11 wavefronts per
// CU) 3 ef cost 37 % (2.30 M against 3.62 M: its launches are short, and the hand-on pass after each one is not;
// profiles/r06/exact/).
// SHINE_EXACT_NEXT_EIGHTHS > 0: that room everywhere, < 0: the fixed sizes everywhere (tuning).
// The room is a cliff: at cfg 4, 3 ef hands on 3-4 % of a call's queries and runs at 1.90 M, 2.5 ef at 1.03 M and
// 2 ef at 0.51 M (profiles/r06/exact/scale_cfg4_100m_room_scan.jsonl).  So a stream whose call handed on more than 1/12
// of its queries with the tight room keeps the fixed room at that ef from then on (allow_tight, Scratch::tight_off_ef).
LaunchShape pick_shape(const shine_index* h, const Replica& R, uint32_t nq, uint32_t ef, int pass,
                       uint32_t handed = 0xFFFFFFFFu, uint32_t learned = 0, uint32_t learned_mean = 0,
                       uint32_t mean_visits = 0, bool allow_tight = true) {
  const int64_t room8 = env_int("SHINE_EXACT_NEXT_EIGHTHS", 0);
  if (pass != PASS_LDS || room8 != 0) {
    LaunchShape sh =
        pick_shape_room(h, R, nq, ef, pass, handed, learned, learned_mean, mean_visits, std::max<int64_t>(room8, 0));
    sh.tight = pass == PASS_LDS && room8 > 0 ? 1u : 0u;
    return sh;
  }
  LaunchShape fixed = pick_shape_room(h, R, nq, ef, pass, handed, learned, learned_mean, mean_visits, 0);
  fixed.tight = 0;
  if (fixed.waves > 8 || !allow_tight) return fixed;
  LaunchShape tight = pick_shape_room(h, R, nq, ef, pass, handed, learned, learned_mean, mean_visits, 24);
  tight.tight = 1;
  return tight.waves >= fixed.waves ? tight : fixed;
}

Scratch& scratch_for(Replica& R, hipStream_t s) {
  if (s == R.stream) return R.main;
  for (auto& e : R.by_stream)
    if (e.first == s) return *e.second;
  R.by_stream.emplace_back(s, std::make_unique<Scratch>());
  return *R.by_stream.back().second;
}

int ensure_bitmaps(shine_index* h, Scratch& S, hipStream_t s, uint32_t slots) {
  const uint64_t stride = slot_words(h);
  if (slots <= S.slots && stride == S.stride) return 0;
  HIP_TRY(hipStreamSynchronize(s));  // earlier calls on this stream may still read the old bitmaps
  S.visited.release();
  S.vlog.release();
  S.slots = 0;
  S.stride = stride;
  if (int rc = S.visited.grow(static_cast<size_t>(slots) * stride)) return rc;
  if (int rc = S.vlog.grow(static_cast<size_t>(slots) * kLogCap)) return rc;
  HIP_TRY(hipMemsetAsync(S.visited.p, 0, S.visited.n * sizeof(uint32_t), s));
  HIP_TRY(hipStreamSynchronize(s));
  S.slots = slots;
  return 0;
}

// Enqueue the pass chain on stream s (see PassKind).  Counter words of the call: queue head of pass i at [i],
// size of the list pass i hands on at [4 + i].  Everything stays on the device: asynchronous and still exact.
int enqueue_search(shine_index* h, Replica& R, const float* d_q, uint32_t nq, uint32_t k, uint32_t ef,
                   uint32_t* d_ids, float* d_dists, uint32_t* d_qs, hipStream_t s, uint32_t* d_access = nullptr,
                   uint32_t* d_call_out = nullptr) {
  Scratch& S = scratch_for(R, s);
  if (int rc = S.counter.grow(kCallWords)) return rc;
  if (S.ovf.n < 3ull * nq) HIP_TRY(hipStreamSynchronize(s));  // a reallocation must not pull the list from under
  if (int rc = S.ovf.grow(3ull * nq)) return rc;                // an earlier call on this stream
  if (!S.seen_dev) {
    if (int rc = S.seen.grow(12, hipHostMallocMapped | hipHostMallocPortable)) return rc;
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, S.seen.p, 0));
    S.seen_dev = static_cast<uint32_t*>(dp);
  }
  // the counter words start at zero: left so by the last call's last pass, else (first call, a failed call) set here
  if (!S.counters_zero) HIP_TRY(hipMemsetAsync(S.counter.p, 0, kCallWords * sizeof(uint32_t), s));
  S.counters_zero = false;
  const int start = static_cast<int>(env_int("SHINE_DEBUG_START_MODE", 0));  // test hook: the fallback passes alone
  const bool fast_mode = h->search_mode == SHINE_MODE_FAST;
  const bool fast_kernel = fast_mode && ef <= kFastMaxEf && h->M0 <= 64;
  const uint32_t handed = S.seen.p[3] ? S.seen.p[0] : 0;  // [3] = 1 once a call has written the counts
  // a learned table that handed queries on was too small — unless the pass spills its tables in place: then only the
  // exact pass hands queries on, for its next_candidates capacity, which a larger table would only shrink
  if (handed && S.last_learned && (S.last_fast || !spill_enabled()))
    S.table_floor = std::max(S.table_floor, pow2_at_least(2 * S.last_table));
  // Tuning hook (off by default): a learned fast table that sent more than SHINE_FAST_SPILL_PERMILLE / 1000 of its
  // call's queries to a spill bitmap is grown.  It cost 30 % at cfg 3 (10M ids, batch 4096), where residency matters
  // more than the spills (profiles/r04/scale_cfg3_cfg5_10m_v2_floor.jsonl), and did not help at 100M ids, where the
  // u32 table's load was the cost (profiles/r04/diag100m_*.jsonl).
  {
    const uint64_t spilled = S.seen.p[3] ? S.seen.p[7] : 0, seen_nq = S.seen.p[3] ? S.seen.p[6] : 0;
    const int64_t permille = env_int("SHINE_FAST_SPILL_PERMILLE", 0);
    if (permille > 0 && spilled && S.last_learned && S.last_fast && spilled * 1000 > seen_nq * static_cast<uint64_t>(permille))
      S.table_floor = std::max(S.table_floor, pow2_at_least(2 * S.last_table));
  }
  if (ef != S.last_ef) S.table_floor = 0;
  // the tight next_candidates room handed on too many of the last call's queries: the fixed room at this ef from now
  if (S.last_tight && ef == S.last_ef && S.seen.p[3] && handed * 12 > S.seen.p[6]) S.tight_off_ef = ef;
  if (ef != R.vmax_ef) {
    for (uint32_t& v : R.vmax_recent) v = 0;
    for (uint32_t& v : R.nmax_recent) v = 0;
    R.vmax_ef = ef;
  }
  if (ef == S.last_ef && S.seen.p && S.seen.p[3]) {  // the worst query of the stream's latest finished call
    R.nmax_recent[R.vmax_pos % 32] = S.seen.p[8];
    R.vmax_recent[R.vmax_pos++ % 32] = S.seen.p[4];
  }
  // the fast pass sizes its table for the mean query when it can spill in place; the exact pass keeps the maximum
  // (its tables sized from the mean ran slower, profiles/r03/ab1_merge_spill_tables.jsonl)
  const uint32_t learned = ef != S.last_ef ? 0 : learned_exact_table(S, ef, R.recent_vmax());
  const uint32_t mean_v = ef != S.last_ef ? 0 : mean_visits(S);
  // The fast table: sized for the previous call's mean query — the smallest power of two above 1.25x it (mean-sized,
  // spilling the rest, where the spill bitmap stays in an XCD's 4 MiB L2: at 10M ids the mean-sized table's residency
  // wins, cfg5-shaped 10M at ef = 250: 1.82 M against 1.59 M with the worst query's table, profiles/r04/
  // scale_cfg3_cfg5_10m_v6_maxtable.jsonl) or, beyond L2, the u32 table of learned_max_table (load 0.45 at the mean,
  // grown to its residency level), where it holds the wavefronts one batch puts on a CU.  SHINE_FAST_TABLE_MAX=0 / 1
  // forces either (tuning).
  uint32_t learned_fast = 0, learned_mean = 0, learned_vt3 = 0;
  if (ef == S.last_ef) {
    if (!spill_enabled()) {
      learned_fast = learned;
    } else {
      const uint64_t need = std::min<uint64_t>(16, (nq + R.cus - 1) / R.cus);
      const uint32_t mean_t = learned_mean_table(S),
                     max_t = learned_max_table(S, ef, R.lds_per_cu, static_cast<uint32_t>(std::min<uint64_t>(16, 2 * need)));
      const bool max_fits = max_t && R.lds_per_cu / lds_alloc_bytes(search_fast_lds_bytes(max_t, ef, 4)) >= need;
      // (the mean-sized power of two at 100M ids: 4,096 entries, load 0.62 at the mean, 3.39 M QPS, profiles/r05/
      // scale_cfg4_100m_hash_vs_bitmap.jsonl)
      const bool beyond_l2 = 4ull * h->words_per_slot > kXcdL2Bytes;
      const int64_t force = env_int("SHINE_FAST_TABLE_MAX", -1);
      learned_fast = (force == 1 || (force < 0 && max_fits && beyond_l2)) ? max_t : mean_t;
      learned_mean = mean_t;
      // Two-choice u32 buckets where the u32 rule leaves one wavefront per SIMD (the latency-bound regime: cfg 5's 50M
      // records at d = 200, ef = 250, 4 per CU): at load 0.7 they hold 6, 1.42 M -> 1.81 M QPS.  Where the u32 rule
      // already holds more (cfg 4's 100M records at ef = 128: 6 per CU), the fuller tables' extra wavefronts did not pay
      // for the two-bucket look-ahead probe: 4.57-4.70 M against 4.66-4.72 M at loads 0.5-0.6, 4.20 M at 0.7 and 8-10
      // per CU (profiles/r06/scale_cfg4_vt3_*.jsonl).  SHINE_VT3_BATCHES: the batches in flight whose wavefronts the
      // table may make room for (default 2).
      const uint64_t waves_u32 = max_t ? R.lds_per_cu / lds_alloc_bytes(search_fast_lds_bytes(max_t, ef, 4)) : 0;
      const int64_t vt3_force = env_int("SHINE_VT3", -1);
      if (beyond_l2 && force < 0 && vt3_usable(h) && (vt3_force == 1 || waves_u32 <= 4)) {
        const uint64_t batches = static_cast<uint64_t>(std::max<int64_t>(1, env_int("SHINE_VT3_BATCHES", 2)));
        learned_vt3 = learned_max_table(S, ef, R.lds_per_cu, static_cast<uint32_t>(std::min<uint64_t>(16, batches * need)),
                                        vt3_load_permille(true)) / 4 * 4;
      }
    }
  }
  S.last_ef = ef;
  S.last_nq = nq;
  int chain[3], n_pass = 0;
  if (start <= 0) chain[n_pass++] = fast_kernel ? PASS_FAST : PASS_LDS;
  else if (start == 1) chain[n_pass++] = PASS_WHOLE_CU;
  const bool main_only = env_int("SHINE_DEBUG_MAIN_ONLY", 0) != 0;  // measurement hook: no fallback passes
  if (start <= 2 && !main_only) chain[n_pass++] = PASS_LIGHT;
  if (!env_int("SHINE_DEBUG_NO_GLOBAL", 0) && !main_only) chain[n_pass++] = PASS_GLOBAL;  // measurement hook
  for (int i = 0; i < n_pass; ++i) {
    const int pass = chain[i];
    const LaunchShape sh =
        pass == PASS_FAST ? pick_fast_shape(nq, ef, R.cus, R.lds_per_cu, h->id_space, learned_fast, handed > 0,
                                          elem_is_byte(h->elem), learned_vt3)
                          : pick_shape(h, R, nq, ef, pass, handed, learned, learned_mean,
                                       i == 0 ? mean_v : 0u, S.tight_off_ef != ef);
    if (i == 0) {
      S.last_table = sh.vis_cap;
      S.last_fast = pass == PASS_FAST;
      S.last_tight = pass == PASS_LDS && sh.tight;
      // the table came from learning, not the fixed rule
      S.last_learned = (learned_fast != 0 && sh.vis_cap == learned_fast) || (learned_vt3 != 0 && sh.vis16 == 3) ||
                       (pass != PASS_FAST && learned != 0 && sh.vis_cap == learned);
      if (env_int("SHINE_DEBUG_SHAPE", 0))  // diagnostics: the main pass's shape and what it was learned from
        std::fprintf(stderr, "shape: pass %d nq %u ef %u table %u vis16 %u grid %u waves %u cap %u learned %u vmax %u "
                     "next_max %u handed %u floor %u spill_hash %u learned_fast %u\n",
                     pass, nq, ef, sh.vis_cap, sh.vis16, sh.grid, sh.waves, sh.cap, learned,
                     S.seen.p[3] ? S.seen.p[4] : 0u, R.recent_nmax(), handed, S.table_floor,
                     spill_hashed(h) ? spill_hash_entries(sh.vis_cap) : 0u, learned_fast);
    }
    SearchArgs a{};
    a.g = dev_graph(h, R);
    if (!a.g.vec || !a.g.adj0 || !a.g.uid || !a.g.up_base)
      return set_error(SHINE_ERR_HIP, "search launch: an index array is missing on this GPU slot");
    if (pass == PASS_LIGHT || pass == PASS_GLOBAL || pass == PASS_FAST || pass == PASS_LDS) {
      // the fallback passes' bitmaps; the main pass borrows them for its spilled tables (it runs first on the stream
      // and hands every one back zeroed)
      const uint32_t need = std::max<uint32_t>({pick_shape(h, R, nq, ef, PASS_LIGHT).grid,
                                                pick_shape(h, R, nq, ef, PASS_GLOBAL).grid, kSpillSlots});
      if (int rc = ensure_bitmaps(h, S, s, need)) return rc;
    }
    if ((pass == PASS_FAST || pass == PASS_LDS) && spill_enabled()) {
      if (!S.spill_flags.p) {
        if (int rc = S.spill_flags.grow(kSpillSlots)) return rc;
        HIP_TRY(hipMemsetAsync(S.spill_flags.p, 0, kSpillSlots * sizeof(uint32_t), s));
      }
      a.spill_flags = S.spill_flags.p;
      a.spill_slots = std::min<uint32_t>(kSpillSlots, S.slots);
    }
    if (pass == PASS_GLOBAL) {
      a.heap_stride = align16(8ull * ef) / 8 + sh.cap;
      const size_t want = static_cast<size_t>(sh.grid) * a.heap_stride;
      if (S.heaps.n < want) HIP_TRY(hipStreamSynchronize(s));
      if (int rc = S.heaps.grow(want)) return rc;
      a.heaps = S.heaps.p;
      a.global_heaps = 1;
    }
    a.queries = d_q;
    a.nq = nq;
    a.k = k;
    a.ef = ef;
    a.cap = sh.cap;
    a.vis_cap = sh.vis_cap;
    a.vis_limit = sh.vis_limit;
    a.out_ids = d_ids;
    a.out_dists = d_dists;
    a.qstats = d_qs;
    a.visited = S.visited.p;
    a.words_per_slot = S.stride;
    a.spill_hash = spill_hashed(h) ? spill_hash_entries(sh.vis_cap) : 0u;
    if (a.spill_hash) {  // test hook: a smaller hash table (a power of two, >= 256 entries)
      const int64_t hs = env_int("SHINE_DEBUG_SPILL_HASH", 0);
      if (hs >= 256 && hs <= kSpillHashMax && (hs & (hs - 1)) == 0) a.spill_hash = static_cast<uint32_t>(hs);
    }
    a.vlog = S.vlog.p;
    a.log_cap = kLogCap;
    a.counter = S.counter.p + i;
    a.vis_max = S.counter.p + 3;
    a.next_max = S.counter.p + 10;
    a.vis_sum = i == 0 ? S.counter.p + 8 : nullptr;  // the main pass's queries only: a hand-on counts once
    a.spill_count = i == 0 ? S.counter.p + 9 : nullptr;
    a.fast = pass == PASS_FAST ? 1u : 0u;
    a.vis16 = sh.vis16;
    a.vis_bits = sh.vis_bits;
    a.vis_mul = 0x9E3779B1u;  // odd: x -> x * mul mod 2^vis_bits permutes the id space
    a.vis_mul_inv = inverse_odd(a.vis_mul);
    a.sort_out = fast_mode ? 1u : 0u;
    a.access = d_access;
    if (i > 0) {
      a.in_list = S.ovf.p + static_cast<size_t>(i - 1) * nq;
      a.in_count = S.counter.p + 4 + (i - 1);
    }
    if (i == 0 && env_int("SHINE_PHASE_PROFILE", 0)) {
      if (int rc = R.prof.grow(24)) return rc;
      HIP_TRY(hipMemsetAsync(R.prof.p, 0, 24 * sizeof(unsigned long long), s));
      a.prof = R.prof.p;
    }
    if (i + 1 < n_pass) {
      a.out_list = S.ovf.p + static_cast<size_t>(i) * nq;
      a.out_count = S.counter.p + 4 + i;
    } else {
      a.call_counters = S.counter.p;
      a.host_counts = S.seen_dev;
      a.call_out = d_call_out;
    }
    hipError_t e = launch_search(h->dim, h->metric, h->elem, sh.grid, a, s);
    if (e != hipSuccess) return set_error(SHINE_ERR_HIP, std::string("search launch: ") + hipGetErrorString(e));
    if (env_int("SHINE_DEBUG_SYNC", 0)) {  // diagnostics: wait for every pass and name the one that failed
      e = hipStreamSynchronize(s);
      if (e != hipSuccess)
        return set_error(SHINE_ERR_HIP, "pass " + std::to_string(i) + " (kind " + std::to_string(pass) + ", grid " +
                                            std::to_string(sh.grid) + ", table " + std::to_string(sh.vis_cap) +
                                            ", vis16 " + std::to_string(sh.vis16) + "): " + hipGetErrorString(e));
    }
  }
  S.counters_zero = true;
  return 0;
}

int check_knn_args(shine_index* h, uint32_t k, uint32_t ef) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  if (k == 0) return set_error(SHINE_ERR_ARG, "k must be > 0");
  if (ef < k) return set_error(SHINE_ERR_ARG, "ef_search must be >= k");  // hnsw.hh:36
  if (ef > 4096) return set_error(SHINE_ERR_ARG, "ef_search must be <= 4096");
  return 0;
}

// Debug (SHINE_DEBUG_VALIDATE=1): read every slot's level-0 lists back through that slot's own view and check on the
// host that each entry names a record of the id space, before any search is launched on the layout.
int validate_views(shine_index* h) {
  if (h->placement == SHINE_PLACE_REPLICA) return 0;
  const uint64_t U = h->ids_per_slot, G = h->reps.size();
  std::vector<uint32_t> rows(U * h->M0), ub(h->id_space);
  for (uint64_t r = 0; r < G; ++r) {
    HIP_TRY(hipSetDevice(h->reps[r].device));
    HIP_TRY(hipMemcpy(ub.data(), h->reps[r].up_base.p, ub.size() * 4, hipMemcpyDeviceToHost));
    for (uint64_t o = 0; o < G; ++o) {
      HIP_TRY(hipMemcpy(rows.data(), h->sadj0.view[r].va + o * h->sadj0.stride, rows.size() * 4, hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < rows.size(); ++i) {
        const uint32_t x = rows[i];
        if (x != kInvalid && x >= h->id_space)
          return set_error(SHINE_ERR_FORMAT, "validate: slot " + std::to_string(r) + " sees id " + std::to_string(x) +
                                                 " in row " + std::to_string(o * U + i / h->M0));
      }
    }
    std::fprintf(stderr, "validate: slot %llu view ok (ep %u, ep up_base %u)\n", static_cast<unsigned long long>(r),
                 h->ep, ub[h->ep]);
  }
  return 0;
}

// The queue sizes the compute nodes' acks would carry at a batch boundary (query_router.hh:233-255, 304-311).  The
// host routes a whole call before any slot starts, so a slot's queue is modelled: the queries routed to it so far
// minus what it answers while the node as a whole answers all of them, at the per-slot rates of the last call.
void modelled_queues(const std::vector<double>& rate, const std::vector<uint64_t>& routed, std::vector<uint32_t>& q) {
  double total = 0, rsum = 0;
  for (size_t i = 0; i < routed.size(); ++i) {
    total += static_cast<double>(routed[i]);
    rsum += rate[i] > 0 ? rate[i] : 1.0;
  }
  const double t = total / rsum;
  for (size_t i = 0; i < routed.size(); ++i) {
    const double r = rate[i] > 0 ? rate[i] : 1.0;
    q[i] = static_cast<uint32_t>(std::llround(std::max(0.0, static_cast<double>(routed[i]) - r * t)));
  }
}

void route_batch(shine_index* h, const float* q, const uint32_t* ids, uint32_t nq, uint32_t* out) {
  const uint32_t G = static_cast<uint32_t>(h->reps.size());
  if (h->placement == SHINE_PLACE_SHARDED_REGIONS && G > 1) {  // QueryRouter::run_routing (query_router.hh:280-387)
    const std::vector<double>& rate = h->slot_rate;
    h->router.route(h->regions, q, nq, h->dim,
                    [&](const std::vector<uint64_t>& routed, std::vector<uint32_t>& p) { modelled_queues(rate, routed, p); },
                    out);
    return;
  }
  for (uint32_t i = 0; i < nq; ++i) out[i] = (ids ? ids[i] : i) % G;
}

void print_phase_profile(const shine_index* h, const Replica& R) {  // SHINE_PHASE_PROFILE diagnostics
  unsigned long long ph[24];
  if (hipMemcpy(ph, R.prof.p, sizeof(ph), hipMemcpyDeviceToHost) != hipSuccess) return;
  std::fprintf(stderr, "SHINE_PHASE_PROFILE entries:");
  for (int i = 12; i < 24; ++i) std::fprintf(stderr, " %llu", ph[i]);
  std::fprintf(stderr, "\n");
  if (h->search_mode == SHINE_MODE_FAST)  // entry counts 9..11: next = runner-up / fresh, mispredicted
    std::fprintf(stderr, "SHINE_PHASE_PROFILE cycles: setup %llu greedy %llu pick %llu - %llu predict+issue %llu "
                         "dist %llu merge %llu out %llu visited %llu\n",
                 ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], ph[6], ph[7], ph[8]);
  else
    std::fprintf(stderr, "SHINE_PHASE_PROFILE cycles: setup %llu greedy %llu pop %llu adj+visited %llu dist %llu "
                         "predict %llu accept-loop %llu out %llu next-push %llu top-pop %llu top-push %llu trim %llu\n",
                 ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], ph[6], ph[7], ph[8], ph[9], ph[10], ph[11]);
}

// B_q, with the record's stored element width (f32 4, f16 2, byte rows 1) and the f32 query
uint64_t bq_bytes(const shine_index* h, const uint32_t* qs) {
  const uint64_t e = elem_bytes(h->elem);
  return qs[SHINE_QS_DISTCOMPS] * h->dim * e + qs[SHINE_QS_LISTS_L0] * (4ull + 4ull * h->M0) +
         qs[SHINE_QS_LISTS_UPPER] * (4ull + 4ull * h->M) + 4ull * h->dim;
}

uint64_t ref_read_bytes(const shine_index* h, const uint32_t* qs) {  // rdma_reads.hh:12,46 accounting
  const uint64_t node = 16 + 4ull * h->dim;
  const uint64_t node_reads = qs[SHINE_QS_DISTCOMPS] > 0 ? qs[SHINE_QS_DISTCOMPS] - 1 : 0;
  return node_reads * node + qs[SHINE_QS_LISTS_L0] * (4ull + 8ull * h->M0) + qs[SHINE_QS_LISTS_UPPER] * (4ull + 8ull * h->M);
}

}  // namespace

namespace shine {

int search_enqueue(shine_index* h, uint32_t slot, const float* d_q, uint32_t nq, uint32_t k, uint32_t ef,
                   uint32_t* d_ids, float* d_dists, uint32_t* d_qs, hipStream_t s) {
  if (slot >= h->reps.size()) return set_error(SHINE_ERR_ARG, "gpu_slot out of range");
  return enqueue_search(h, h->reps[slot], d_q, nq, k, ef, d_ids, d_dists, d_qs, s);
}

void index_release(shine_index* h) { release_index(h); }

int index_from_graph(HostGraph&& G, int elem, const int* gpu_ids, uint32_t n_gpus, int placement, double cache_fraction,
                     shine_index_t* out) {
  return make_index(std::move(G), elem, gpu_ids, n_gpus, placement, cache_fraction, out);
}

}  // namespace shine

extern "C" {

const char* shine_last_error(void) { return last_error(); }

int shine_open_buffers_ex(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim,
                          uint32_t M, int metric, int elem, const int* gpu_ids, uint32_t n_gpus, int placement,
                          double cache_fraction, shine_index_t* out) {
  if (!dumps || !sizes) return set_error(SHINE_ERR_ARG, "dumps / sizes is NULL");
  if (metric != SHINE_METRIC_L2 && metric != SHINE_METRIC_IP) return set_error(SHINE_ERR_ARG, "metric must be 0 or 1");
  HostGraph G;
  if (int rc = parse_dumps(dumps, sizes, n_dumps, dim, M, metric, 0, G)) return rc;
  return make_index(std::move(G), elem, gpu_ids, n_gpus, placement, cache_fraction, out);
}

int shine_open_ex(const char* const* dump_paths, uint32_t n_dumps, uint32_t dim, uint32_t M, int metric, int elem,
                  const int* gpu_ids, uint32_t n_gpus, int placement, double cache_fraction, shine_index_t* out) {
  if (!dump_paths || n_dumps == 0) return set_error(SHINE_ERR_ARG, "no dump paths");
  std::vector<std::vector<uint8_t>> files(n_dumps);
  std::vector<const uint8_t*> ptrs(n_dumps);
  std::vector<uint64_t> sizes(n_dumps);
  for (uint32_t i = 0; i < n_dumps; ++i) {
    if (!dump_paths[i]) return set_error(SHINE_ERR_ARG, "dump path is NULL");
    if (int rc = read_file(dump_paths[i], files[i])) return rc;
    ptrs[i] = files[i].data();
    sizes[i] = files[i].size();
  }
  return shine_open_buffers_ex(ptrs.data(), sizes.data(), n_dumps, dim, M, metric, elem, gpu_ids, n_gpus, placement,
                               cache_fraction, out);
}

int shine_open_buffers(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim,
                       uint32_t M, int metric, int elem, const int* gpu_ids, uint32_t n_gpus, shine_index_t* out) {
  return shine_open_buffers_ex(dumps, sizes, n_dumps, dim, M, metric, elem, gpu_ids, n_gpus, SHINE_PLACE_REPLICA, 0.0,
                               out);
}

int shine_open(const char* const* dump_paths, uint32_t n_dumps, uint32_t dim, uint32_t M, int metric, int elem,
               const int* gpu_ids, uint32_t n_gpus, shine_index_t* out) {
  return shine_open_ex(dump_paths, n_dumps, dim, M, metric, elem, gpu_ids, n_gpus, SHINE_PLACE_REPLICA, 0.0, out);
}

int shine_set_search_mode(shine_index_t h, int mode) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  if (mode != SHINE_MODE_EXACT && mode != SHINE_MODE_FAST) return set_error(SHINE_ERR_ARG, "unknown search mode");
  if (mode == SHINE_MODE_FAST && h->id_space >= 0x80000000ull)
    return set_error(SHINE_ERR_ARG, "fast mode needs fewer than 2^31 node ids");
  std::lock_guard<std::mutex> lk(h->mu);
  h->search_mode = mode;
  return SHINE_OK;
}

int shine_index_get_info(shine_index_t h, shine_index_info* o) {
  if (!h || !o) return set_error(SHINE_ERR_ARG, "NULL argument");
  std::memset(o, 0, sizeof(*o));
  o->num_nodes = h->N;
  o->num_upper_rows = h->upper_rows;
  o->device_bytes = h->device_bytes;
  o->dim = h->dim;
  o->M = h->M;
  o->metric = static_cast<uint32_t>(h->metric);
  o->elem = static_cast<uint32_t>(h->elem);
  o->max_level = h->ep_level;
  o->entry_uid = h->ep_uid;
  o->n_shards = h->n_shards;
  o->n_gpus = static_cast<uint32_t>(h->reps.size());
  o->placement = static_cast<uint32_t>(h->placement);
  o->id_space = h->id_space;
  o->cache_fraction = h->cache_fraction;
  if (!h->reps.empty()) {
    o->cus = h->reps[0].cus;
    o->lds_per_cu = h->reps[0].lds_per_cu;
  }
  return SHINE_OK;
}

uint64_t shine_algorithmic_bytes(shine_index_t h, const uint32_t* qstats, uint32_t nq) {
  if (!h || !qstats) return 0;
  uint64_t t = 0;
  for (uint32_t i = 0; i < nq; ++i) t += bq_bytes(h, qstats + static_cast<size_t>(i) * SHINE_QS_WORDS);
  return t;
}

int shine_knn_batch_device(shine_index_t h, uint32_t gpu_slot, const float* d_queries, uint32_t nq, uint32_t k,
                           uint32_t ef, uint32_t* d_out_ids, float* d_out_dists, uint32_t* d_qstats, void* stream) {
  if (int rc = check_knn_args(h, k, ef)) return rc;
  if (gpu_slot >= h->reps.size()) return set_error(SHINE_ERR_ARG, "gpu_slot out of range");
  if (nq == 0) return SHINE_OK;
  if (!d_queries || !d_out_ids) return set_error(SHINE_ERR_ARG, "NULL device pointer");
  std::lock_guard<std::mutex> lk(h->mu);
  Replica& R = h->reps[gpu_slot];
  HIP_TRY(hipSetDevice(R.device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : R.stream;
  uint32_t* qs = d_qstats;
  if (!qs) {
    Scratch& S = scratch_for(R, s);
    if (S.qs.n < static_cast<size_t>(nq) * kQsWords) HIP_TRY(hipStreamSynchronize(s));
    if (int rc = S.qs.grow(static_cast<size_t>(nq) * kQsWords)) return rc;
    qs = S.qs.p;
  }
  if (h->cache_policy == SHINE_CACHE_DYNAMIC) R.dev_api_dirty = true;  // it reads the arena and logs into its buffers
  return enqueue_search(h, R, d_queries, nq, k, ef, d_out_ids, d_out_dists, qs, s);
}

}  // extern "C"

namespace {

// The dynamic cache between calls (SHINE_CACHE_DYNAMIC), in three steps per GPU slot:
//   fetch_logs      after a call's searches are done: its miss and rescue logs to the host, the device counts zeroed;
//   replay          host only (one thread per slot): the reference's policy (cache.cc) over the fetched logs, and the
//                   arena updates it makes (rows to copy in, device ids to drop, cooling flags);
//   enqueue_update  the updates uploaded and applied on the slot's stream, behind whatever is enqueued there.
// Pipelined (default): a call's logs are replayed during the NEXT call's searches and its updates are applied behind
// them, so the host's work hides behind the GPU's and a call's admissions serve from the call after next (the
// reference admits while its queries run; here at call granularity, one call later).  SHINE_CACHE_LAG=0: the
// updates of a call are applied before it returns (the round-3/4 behaviour: the host waits for the replay).
bool cache_lagged() { return env_int("SHINE_CACHE_LAG", 1) != 0; }

// Every slot's logs, the copies of all slots in flight together on their streams (counts first, then the logs they
// size) into pinned memory: two waits in all instead of three blocking copies per slot (24 round trips at 8 slots)
int fetch_logs(shine_index* h) {
  for (Replica& R : h->reps) {
    if (!R.logn.p || R.counts_inflight) continue;  // (knn_host enqueues the counts behind its searches)
    HIP_TRY(hipSetDevice(R.device));
    if (int rc = R.logn_h.grow(2)) return rc;
    HIP_TRY(hipMemcpyAsync(R.logn_h.p, R.logn.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, R.stream));
  }
  for (Replica& R : h->reps) {
    if (!R.logn.p) continue;
    HIP_TRY(hipSetDevice(R.device));
    HIP_TRY(hipStreamSynchronize(R.stream));
  }
  for (Replica& R : h->reps) {
    if (!R.logn.p) continue;
    HIP_TRY(hipSetDevice(R.device));
    const uint32_t n0 = std::min(R.logn_h.p[0], R.clog_cap), n1 = std::min(R.logn_h.p[1], R.rlog_cap);
    if (int rc = R.clog_h.grow(std::max<uint32_t>(n0, 1))) return rc;
    if (int rc = R.rlog_h.grow(std::max<uint32_t>(n1, 1))) return rc;
    if (n0) HIP_TRY(hipMemcpyAsync(R.clog_h.p, R.clog.p, n0 * sizeof(unsigned long long), hipMemcpyDeviceToHost, R.stream));
    if (n1) HIP_TRY(hipMemcpyAsync(R.rlog_h.p, R.rlog.p, n1 * sizeof(uint32_t), hipMemcpyDeviceToHost, R.stream));
    HIP_TRY(hipMemsetAsync(R.logn.p, 0, 2 * sizeof(uint32_t), R.stream));  // before the slot's next search
    ++R.log_epoch;  // searches enqueued from here on log into the emptied buffers: a new epoch
  }
  for (Replica& R : h->reps) {
    if (!R.logn.p) continue;
    HIP_TRY(hipSetDevice(R.device));
    HIP_TRY(hipStreamSynchronize(R.stream));
    const uint32_t c0 = R.logn_h.p[0], c1 = R.logn_h.p[1];
    const uint32_t n0 = std::min(c0, R.clog_cap), n1 = std::min(c1, R.rlog_cap);
    R.pend_clog.insert(R.pend_clog.end(), R.clog_h.p, R.clog_h.p + n0);
    R.pend_rlog.insert(R.pend_rlog.end(), R.rlog_h.p, R.rlog_h.p + n1);
    R.pend_lost += (c0 - n0) + (c1 - n1);
    R.counts_inflight = false;
  }
  return 0;
}

// Host only (no HIP call): safe on a thread per slot while the main thread waits.
void replay(const shine_index* h, Replica& R, shine_stats* agg) {
  if (R.rp_clog.empty() && R.rp_rlog.empty()) return;
  const auto t0 = std::chrono::steady_clock::now();
  // hits on cooling entries (by device id, every hit logged): each key once, deduplicated in an open-addressed set over
  // twice the log (a sort of the raw log was most of this step), then sorted by the engine
  std::vector<uint32_t> rescued_keys;
  {
    uint32_t rmask = 63;
    while (rmask + 1 < 2 * R.rp_rlog.size()) rmask = 2 * rmask + 1;
    std::vector<uint32_t> seen(rmask + 1, kInvalid);
    for (uint32_t x : R.rp_rlog) {
      if (x >= h->uid_of_dev.size()) continue;
      uint32_t q = (x * 0x9E3779B1u) & rmask;
      while (seen[q] != kInvalid && seen[q] != x) q = (q + 1) & rmask;
      if (seen[q] == x) continue;
      seen[q] = x;
      rescued_keys.push_back(h->uid_of_dev[x]);
    }
  }
  std::vector<CacheCandidate> cand(R.rp_clog.size());
  for (size_t i = 0; i < cand.size(); ++i) {
    const unsigned long long e = R.rp_clog[i];
    CacheCandidate& c = cand[i];
    c.query = static_cast<uint32_t>(e >> 32) & 0x7FFFFFFFu;
    c.dev_id = static_cast<uint32_t>(e) & 0x7FFFFFFFu;
    c.always = ((e >> 31) & 1ull) != 0;
    c.coin = (e >> 63) != 0;
    c.key = c.dev_id < h->uid_of_dev.size() ? h->uid_of_dev[c.dev_id] : kInvalid;
  }
  const uint64_t a0 = R.cache.admitted, e0 = R.cache.evicted, r0 = R.cache.rescued;
  std::vector<CacheUpdate> ups;
  std::vector<uint32_t> flagged;  // slots whose cooling flag the policy changed
  const size_t n_cand = cand.size(), n_resc = rescued_keys.size();
  const auto t1 = std::chrono::steady_clock::now();
  R.cache.apply_call(std::move(rescued_keys), std::move(cand), ups, flagged);
  const auto t2 = std::chrono::steady_clock::now();
  // one change per slot: the occupant at the call's start leaves cslot, the last one admitted is copied in (ups are in
  // slot-claim order; `at` maps a slot to its entry of `order`, open-addressed over twice the updates: a few KiB that
  // stay in cache, where an array over the arena's slots took a miss per update)
  std::vector<uint32_t> order, first_old, last_new;
  uint32_t amask = 63;
  while (amask + 1 < 2 * ups.size()) amask = 2 * amask + 1;
  std::vector<uint64_t> at(amask + 1, ~0ull);  // (slot << 32) | index
  for (const CacheUpdate& u : ups) {
    uint32_t p = (u.slot * 0x9E3779B1u) & amask;
    while (at[p] != ~0ull && static_cast<uint32_t>(at[p] >> 32) != u.slot) p = (p + 1) & amask;
    if (at[p] == ~0ull) {
      at[p] = (static_cast<uint64_t>(u.slot) << 32) | order.size();
      order.push_back(u.slot);
      first_old.push_back(u.old_dev);
      last_new.push_back(u.new_dev);
    } else {
      last_new[static_cast<uint32_t>(at[p])] = u.new_dev;
    }
  }
  // (every replay is uploaded before the next one: enqueue_update follows each replay_all)
  std::vector<uint32_t>& upd = R.upd_vec;
  std::vector<uint32_t> drop, fill;
  for (uint32_t i = 0; i < order.size(); ++i)
    if (first_old[i] != kInvalid) drop.push_back(first_old[i]);
  for (uint32_t i = 0; i < order.size(); ++i) {
    fill.push_back(order[i]);
    fill.push_back(last_new[i]);
  }
  // the engine's final cooling state of every slot this replay changed, each slot once (an open-addressed set over
  // twice the slots: a sort of the ~9K touched slots took a third of the updates' time)
  std::vector<uint32_t> cool;
  {
    const size_t nt = flagged.size() + order.size();
    uint32_t smask = 63;
    while (smask + 1 < 2 * nt) smask = 2 * smask + 1;
    std::vector<uint32_t> seen(smask + 1, kInvalid);
    cool.reserve(2 * nt);
    auto add = [&](uint32_t slot) {
      uint32_t q = (slot * 0x9E3779B1u) & smask;
      while (seen[q] != kInvalid && seen[q] != slot) q = (q + 1) & smask;
      if (seen[q] == slot) return;
      seen[q] = slot;
      cool.push_back(slot);
      cool.push_back(R.cache.cooling(slot) ? 1u : 0u);
    };
    for (uint32_t slot : flagged) add(slot);
    for (uint32_t slot : order) add(slot);
  }
  upd.clear();
  upd.insert(upd.end(), drop.begin(), drop.end());
  upd.insert(upd.end(), fill.begin(), fill.end());
  upd.insert(upd.end(), cool.begin(), cool.end());
  R.upd_drop = static_cast<uint32_t>(drop.size());
  R.upd_fill = static_cast<uint32_t>(fill.size() / 2);
  R.upd_cool = static_cast<uint32_t>(cool.size() / 2);
  if (env_int("SHINE_DEBUG_CACHE_TIMING", 0) > 1) {  // diagnostics: the replay's parts on this slot
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::fprintf(stderr, "replay slot %u: %zu candidates, %zu rescued keys, %zu updates: logs %.3f policy %.3f "
                 "(second chances %.3f, sort %.3f, admissions %.3f, %llu scan steps) updates %.3f ms\n", R.slot, n_cand,
                 n_resc, ups.size(), ms(t0, t1), ms(t1, t2), R.cache.ms_rescue, R.cache.ms_sort, R.cache.ms_admit,
                 static_cast<unsigned long long>(R.cache.scan_steps), ms(t2, std::chrono::steady_clock::now()));
  }
  if (agg) {
    agg->cache_admitted += R.cache.admitted - a0;
    agg->cache_evicted += R.cache.evicted - e0;
    agg->cache_rescued += R.cache.rescued - r0;
    agg->cache_log_dropped += R.rp_lost;
  }
  R.rp_clog.clear();
  R.rp_rlog.clear();
  R.rp_lost = 0;
}

// The replayed updates onto the slot's stream (from pinned host memory: the stream is synchronized before the next
// upload reuses it).  A device-API search on another stream of the slot may still read the arena: the device drains
// first then.
int enqueue_update(shine_index* h, Replica& R) {
  if (R.upd_vec.empty()) return 0;
  HIP_TRY(hipSetDevice(R.device));
  if (R.dev_api_dirty) {
    HIP_TRY(hipDeviceSynchronize());
    R.dev_api_dirty = false;
    // a count copy enqueued behind this call's own searches (knn_host) may predate entries the device-API searches
    // logged after it: the counts are copied again once the call's searches are done (fetch_logs)
    R.counts_inflight = false;
  }
  const size_t n = R.upd_vec.size();
  if (R.upd.n < n || R.upd_host.n < n) HIP_TRY(hipStreamSynchronize(R.stream));
  if (int rc = R.upd.grow(n)) return rc;
  if (int rc = R.upd_host.grow(n)) return rc;
  std::memcpy(R.upd_host.p, R.upd_vec.data(), n * sizeof(uint32_t));
  HIP_TRY(hipMemcpyAsync(R.upd.p, R.upd_host.p, n * sizeof(uint32_t), hipMemcpyHostToDevice, R.stream));
  hipError_t e = launch_cache_apply(R.upd.p, R.upd_drop, R.upd_fill, R.upd_cool, R.cslot.p, R.cbits.p, R.cvec.p,
                                    R.cool.p, R.rlogged.p, R.slot_id.p,
                                    reinterpret_cast<const uint8_t*>(h->svec.view[R.slot].va),
                                    row_bytes(h->dim, h->elem), R.stream);
  if (e != hipSuccess) return set_error(SHINE_ERR_HIP, std::string("cache update: ") + hipGetErrorString(e));
  R.upd_vec.clear();
  R.upd_drop = R.upd_fill = R.upd_cool = 0;
  return 0;
}

// The slots whose fetched logs await a replay, their logs handed to it (rp_*): the next call's logs can be fetched
// into pend_* while it runs.
std::vector<size_t> take_logs(shine_index* h) {
  std::vector<size_t> todo;
  for (size_t r = 0; r < h->reps.size(); ++r) {
    Replica& R = h->reps[r];
    if (R.pend_clog.empty() && R.pend_rlog.empty()) continue;
    R.rp_clog.swap(R.pend_clog);
    R.rp_rlog.swap(R.pend_rlog);
    R.pend_clog.clear();
    R.pend_rlog.clear();
    R.rp_lost = R.pend_lost;
    R.pend_lost = 0;
    todo.push_back(r);
  }
  return todo;
}

// replay on every slot with pending logs, one thread each from the handle's pool (8 slots of a 10M-record index filling
// their caches took ~0.3 s a call one after the other, profiles/r03/config_lines_cfg4_10m.jsonl).  The caller has
// waited for a replay still running (wait_replay).
void replay_all(shine_index* h, std::vector<shine_stats>& per) {
  const size_t G = h->reps.size();
  per.assign(G, shine_stats{});
  const std::vector<size_t> todo = take_logs(h);
  h->pool.run(todo.size(), [&](size_t i) { replay(h, h->reps[todo[i]], &per[todo[i]]); });
  for (Replica& R : h->reps) R.dyn_full = R.cache.full();
}

// Pipelined policy: the replay of the logs fetched so far starts on the pool and runs past the host call's return —
// through the call's searches, its collection and the caller's time until the next call — instead of holding the
// call until it ends (a replay of 8 slots took 2.1-2.6 ms against 1.6-1.8 ms of searches in the skew cell,
// profiles/r06/cache/skew8_replay_timing_inline.txt).  The next host call, and everything else that reads the engine or the
// arena's state, waits for it first (wait_replay).
void replay_launch(shine_index* h) {
  const std::vector<size_t> todo = take_logs(h);
  h->replay_per.assign(h->reps.size(), shine_stats{});
  if (todo.empty()) return;
  h->replay_busy = true;
  h->pool.launch(todo.size(), [h, todo](size_t i) { replay(h, h->reps[todo[i]], &h->replay_per[todo[i]]); });
}

// A replay started by replay_launch joined: its updates onto each slot's stream (behind the searches enqueued there
// so far, ahead of the next ones) and its statistics kept for the next call to report.  The host calls' order of
// updates and searches on a slot's stream is the same as with the replay inside the call: call n's updates land
// before call n + 2's searches.
int wait_replay(shine_index* h) {
  if (!h->replay_busy) return 0;
  h->pool.wait();
  h->replay_busy = false;
  const size_t G = h->reps.size();
  if (h->replay_unreported.size() != G) h->replay_unreported.assign(G, shine_stats{});
  for (size_t r = 0; r < G; ++r) {
    Replica& R = h->reps[r];
    R.dyn_full = R.cache.full();
    const shine_stats& p = h->replay_per[r];
    shine_stats& u = h->replay_unreported[r];
    u.cache_admitted += p.cache_admitted;
    u.cache_evicted += p.cache_evicted;
    u.cache_rescued += p.cache_rescued;
    u.cache_log_dropped += p.cache_log_dropped;
  }
  for (size_t r = 0; r < G; ++r)
    if (int rc = enqueue_update(h, h->reps[r])) return rc;
  return 0;
}

// Queries per chunk of a large host-API call (the bench's batch) and the chunks in flight per slot: four, as the bench
// keeps four batches in flight (2 -> 4 in flight: +27 % QPS, profiles/r02/inflight_scan_bucketed.jsonl).
constexpr uint32_t kHostChunk = 1024;
constexpr uint32_t kHostStreams = 4;

// The slot's host streams, created together on first use: streams created back to back take consecutive hardware
// queues of HIP's round-robin, so four chunks in flight run on four queues (two batches sharing a queue run back to
// back: DESIGN §4 "Hardware queues").
int ensure_host_streams(Replica& R) {
  if (!R.hstreams.empty()) return 0;
  const uint32_t n = static_cast<uint32_t>(std::max<int64_t>(1, env_int("SHINE_HOST_STREAMS", kHostStreams)));
  for (uint32_t i = 0; i < n; ++i) {
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    R.hstreams.push_back(s);
  }
  HIP_TRY(hipEventCreateWithFlags(&R.hfork, hipEventDisableTiming));
  return 0;
}

// A staging set of the slot's pool, large enough for n queries in chunks (a synchronous call gives it back before it
// returns; an asynchronous one when it is waited for).
int take_stage(Replica& R, uint32_t n, uint32_t k, uint32_t d, uint32_t n_chunks, std::unique_ptr<HostStage>& out) {
  if (!R.stages_free.empty()) {
    out = std::move(R.stages_free.back());
    R.stages_free.pop_back();
  } else {
    out = std::make_unique<HostStage>();
  }
  HostStage& S = *out;
  constexpr unsigned kMapped = hipHostMallocMapped | hipHostMallocPortable;
  auto dev = [](void* host, auto** dp) -> hipError_t { return hipHostGetDevicePointer(reinterpret_cast<void**>(dp), host, 0); };
  const size_t nq = std::max<uint32_t>(n, 1);
  if (S.hq.n < nq * d) {
    if (int rc = S.hq.grow(nq * d, kMapped)) return rc;
    HIP_TRY(dev(S.hq.p, &S.dq));
  }
  if (S.hids.n < nq * k) {
    if (int rc = S.hids.grow(nq * k, kMapped)) return rc;
    HIP_TRY(dev(S.hids.p, &S.dids));
  }
  if (S.hd.n < nq * k) {
    if (int rc = S.hd.grow(nq * k, kMapped)) return rc;
    HIP_TRY(dev(S.hd.p, &S.dd));
  }
  if (S.hqs.n < nq * kQsWords + 8) {
    if (int rc = S.hqs.grow(nq * kQsWords + 8, kMapped)) return rc;
    HIP_TRY(dev(S.hqs.p, &S.dqs));
  }
  if (S.hcnt.n < 2ull * std::max<uint32_t>(n_chunks, 1)) {
    if (int rc = S.hcnt.grow(2ull * std::max<uint32_t>(n_chunks, 1), kMapped)) return rc;
    HIP_TRY(dev(S.hcnt.p, &S.hcnt_dev));
  }
  std::memset(S.hcnt.p, 0, S.hcnt.n * sizeof(uint32_t));
  while (S.hchunk.size() < n_chunks) {  // timing events: the call's kernel_ms is its first start to its last chunk's end
    hipEvent_t ev = nullptr;
    HIP_TRY(hipEventCreate(&ev));
    S.hchunk.push_back(ev);
  }
  if (!S.ev0) HIP_TRY(hipEventCreate(&S.ev0));
  return 0;
}

void give_stage(Replica& R, std::unique_ptr<HostStage>& s) {
  if (s) R.stages_free.push_back(std::move(s));
}

}  // namespace

// One host-API call between its enqueue and its collection (shine_knn_batch runs both at once; shine_knn_batch_async
// returns in between and shine_wait collects).
struct shine_request {
  shine_index* h = nullptr;
  uint32_t nq = 0, k = 0;
  uint32_t* out_ids = nullptr;
  float* out_dists = nullptr;
  uint32_t* qstats = nullptr;
  std::vector<DevBuf<uint32_t>>* access = nullptr;
  std::vector<std::vector<uint32_t>> part;           // [slot] the call's query positions answered there
  std::vector<std::unique_ptr<HostStage>> stage;     // [slot] its staging (null: the slot has no queries)
  std::vector<uint8_t> chunked;                      // [slot] 1: chunks on the host streams, 0: one launch on R.stream
  std::vector<uint32_t> csize, nchunks;              // [slot] chunk size and count
  bool dynamic = false, lagged = false;
  bool rotate = false;                               // chunks start at the slot's next host stream (asynchronous
                                                     // calls in flight spread over the streams), else at stream 0
  std::vector<shine_stats> per;                      // statistics of replays finished since the last call's
  double replay_ms = 0;
  std::chrono::steady_clock::time_point t_enq, t_launched;  // (SHINE_DEBUG_CACHE_TIMING)
  int rc = SHINE_OK;                                 // an error already met (collected calls drain first)
  bool collected = false;
  shine_stats stats{};
};

namespace {

// Enqueue a host-API call: route its queries, stage each slot's share in that slot's pinned mapped staging and launch
// it, in chunks on the slot's host streams (SHINE_HOST_CHUNK, default 1,024 queries), or as one launch on the slot's
// own stream where the dynamic cache logs the call or a warmup counts its reads.  Returns before any search finishes.
int knn_enqueue(shine_index* h, shine_request& C, const float* queries, const uint32_t* query_ids, uint32_t ef) {
  const uint32_t G = static_cast<uint32_t>(h->reps.size());
  const size_t d = h->dim;
  const uint32_t nq = C.nq, k = C.k;
  if (env_int("SHINE_DEBUG_VALIDATE", 0))
    if (int rc = validate_views(h)) return rc;
  // queries are split over the slots as compute nodes split them, by id (read_data.hh:57-58: id % num_clients ==
  // client_id; the position stands in for the id when query_ids is NULL); a region-placed index routes them to
  // their region instead
  std::vector<uint32_t> dest(nq);
  route_batch(h, queries, query_ids, nq, dest.data());
  C.part.assign(G, {});
  for (uint32_t i = 0; i < nq; ++i) C.part[dest[i]].push_back(i);
  C.stage.resize(G);
  C.chunked.assign(G, 0);
  C.csize.assign(G, 0);
  C.nchunks.assign(G, 0);
  C.t_enq = std::chrono::steady_clock::now();
  C.dynamic = h->cache_policy == SHINE_CACHE_DYNAMIC && !C.access;
  C.lagged = C.dynamic && cache_lagged();
  // a replay still running from the previous call: joined, its updates enqueued ahead of this call's searches, its
  // statistics reported by this call
  {
    const auto t0 = std::chrono::steady_clock::now();
    if (int rc = wait_replay(h)) return rc;
    C.replay_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (C.dynamic) {
      C.per = std::move(h->replay_unreported);
      h->replay_unreported.clear();
    }
  }
  // on an error after the first enqueue, the slots already enqueued are drained before returning
  auto drain = [&](uint32_t upto, int rc) {
    for (uint32_t r = 0; r < upto; ++r) {
      if (C.part[r].empty()) continue;
      (void)hipSetDevice(h->reps[r].device);
      (void)hipStreamSynchronize(h->reps[r].stream);
      for (hipStream_t hs : h->reps[r].hstreams) (void)hipStreamSynchronize(hs);
    }
    return rc;
  };
  // Calls of more than `chunk` queries on a slot are split into chunks kept in flight (SHINE_HOST_CHUNK, default
  // 1,024: the bench's batch; 0 = never split).  Not while the dynamic cache logs a call (its replay orders admissions
  // by query within one launch) or a warmup counts reads: those run as one launch on the slot's own stream.
  const int64_t chunk_env = env_int("SHINE_HOST_CHUNK", kHostChunk);
  const uint32_t chunk = chunk_env <= 0 ? 0xFFFFFFFFu : static_cast<uint32_t>(std::min<int64_t>(chunk_env, 0x7FFFFFFF));
  for (uint32_t r = 0; r < G; ++r) {
    const uint32_t n = static_cast<uint32_t>(C.part[r].size());
    if (n == 0) continue;
    Replica& R = h->reps[r];
    HIP_TRY(hipSetDevice(R.device));
    // A synchronous call's share of at most one chunk runs as one launch on the slot's own stream too: the slots' own
    // streams were created together at open and take distinct hardware queues, where every slot's first host stream
    // can land on the same one (eight slots of one GPU ran their shares back to back: 3.1 against 1.35 ms a call)
    const bool own_stream = C.access || C.dynamic || (!C.rotate && n <= chunk);
    // chunks near `chunk` queries, and once there are at least as many as host streams, as many on every stream (the
    // call ends when its longest stream does: 10,000 queries as ten chunks of 1,024 left two of the four streams a
    // chunk behind); a call just past one chunk is not cut into launches too small to fill the GPU
    uint32_t m_chunk = n, n_chunks = 1;
    if (!own_stream) {
      if (int rc = ensure_host_streams(R)) return drain(r, rc);
      const uint64_t S = R.hstreams.size();
      uint64_t n_split = n <= chunk ? 1 : std::max<uint64_t>(1, (static_cast<uint64_t>(n) + chunk / 2) / chunk);
      if (n_split >= S) {  // the nearest multiple of S (a tie takes the larger chunks)
        const uint64_t q = n_split / S, rem = n_split % S;
        n_split = (q + (2 * rem > S ? 1 : 0)) * S;
      }
      m_chunk = static_cast<uint32_t>((n + n_split - 1) / n_split);
      n_chunks = (n + m_chunk - 1) / m_chunk;
    }
    C.csize[r] = m_chunk;
    C.nchunks[r] = n_chunks;
    // zero copy: the pinned staging is mapped into the GPU's address space; the kernels read the queries and write
    // ids, distances and counters over PCIe themselves.  Copy-engine transfers would add a cross-engine dependency
    // per batch (copy -> kernel -> copy) that held the host back until each kernel finished: 3.0 M against 6.1 M QPS
    // with four batches in flight (profiles/r02/host_leg_probe.jsonl)
    if (int rc = take_stage(R, n, k, static_cast<uint32_t>(d), n_chunks, C.stage[r])) return drain(r, rc);
    HostStage& S = *C.stage[r];
    const std::vector<uint32_t>& pr = C.part[r];
    // (the slot's share in call order from position lo on: one copy of the run instead of a copy per query)
    const bool identity = n == nq || pr[n - 1] - pr[0] == n - 1;
    auto stage = [&](uint32_t lo, uint32_t hi) {  // queries lo .. hi-1 of the slot into the staging
      if (identity) {
        std::memcpy(S.hq.p + static_cast<size_t>(lo) * d, queries + static_cast<size_t>(pr[lo]) * d,
                    static_cast<size_t>(hi - lo) * d * sizeof(float));
        return;
      }
      for (uint32_t j = lo; j < hi; ++j)
        std::memcpy(S.hq.p + static_cast<size_t>(j) * d, queries + static_cast<size_t>(pr[j]) * d, d * sizeof(float));
    };
    if (own_stream) {
      stage(0, n);
      HIP_TRY(hipEventRecord(S.ev0, R.stream));
      if (int rc = enqueue_search(h, R, S.dq, n, k, ef, S.dids, S.dd, S.dqs, R.stream, C.access ? (*C.access)[r].p : nullptr))
        return drain(r + 1, rc);
      HIP_TRY(hipEventRecord(S.hchunk[0], R.stream));
      if (C.dynamic && R.logn.p) {  // the log counts behind the searches, so they are home when the results are
        if (int rc = R.logn_h.grow(2)) return drain(r + 1, rc);
        HIP_TRY(hipMemcpyAsync(R.logn_h.p, R.logn.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, R.stream));
        R.counts_inflight = true;
      }
      continue;
    }
    // The chunks run on the slot's host streams, as a serving loop keeps batches in flight (the last, longest queries
    // of one chunk overlap the next chunks' first ones), after anything enqueued on the slot's own stream before the
    // call (the fork event).  Nothing joins them back: the call's chunk events are what its collection waits for, so
    // calls enqueued back to back (shine_knn_batch_async) overlap as chunks of one call do.  Each chunk is staged
    // just before its launch (the first starts after one chunk's copy, not the whole call's).
    HIP_TRY(hipEventRecord(S.ev0, R.stream));
    HIP_TRY(hipEventRecord(R.hfork, R.stream));
    for (hipStream_t hs : R.hstreams) HIP_TRY(hipStreamWaitEvent(hs, R.hfork, 0));
    // A synchronous call starts at stream 0, so that consecutive calls put their chunks on the same streams and each
    // stream's visited tables are learned from the calls before it (capi.cc learned_*_table: per stream); calls in
    // flight together start where the previous one stopped
    const uint64_t first = C.rotate ? R.hnext + R.slot : 0;  // (slots of one GPU start on different queues)
    if (C.rotate) R.hnext += n_chunks;
    for (uint32_t c = 0, off = 0; off < n; ++c, off += m_chunk) {
      const uint32_t m = std::min(m_chunk, n - off);
      hipStream_t hs = R.hstreams[(first + c) % R.hstreams.size()];
      stage(off, off + m);
      if (int rc = enqueue_search(h, R, S.dq + static_cast<size_t>(off) * d, m, k, ef, S.dids + static_cast<size_t>(off) * k,
                                  S.dd + static_cast<size_t>(off) * k, S.dqs + static_cast<size_t>(off) * kQsWords, hs,
                                  nullptr, S.hcnt_dev + 2ull * c))
        return drain(r + 1, rc);
      HIP_TRY(hipEventRecord(S.hchunk[c], hs));
    }
    C.chunked[r] = 1;
  }
  // Dynamic cache, pipelined: the previous call's logs are replayed while this call's searches run and past its
  // return; the next call enqueues the updates ahead of its searches (they serve from the call after this one on)
  C.t_launched = std::chrono::steady_clock::now();
  if (C.lagged) {
    replay_launch(h);
    // SHINE_CACHE_ASYNC=0: the replay joined inside the call, while its searches run (the round-5 pipeline; its
    // updates then land behind this call's searches, its statistics are reported by the next call)
    if (env_int("SHINE_CACHE_ASYNC", 1) == 0)
      if (int rc = wait_replay(h)) return drain(G, rc);
  }
  return SHINE_OK;
}

// Collect an enqueued call: each slot's results, chunk by chunk in order while later chunks still run, into the
// caller's arrays; the statistics; and, under the dynamic cache, the call's logs.  The staging goes back to the pool.
int knn_collect(shine_index* h, shine_request& C, shine_stats* stats) {
  const uint32_t G = static_cast<uint32_t>(h->reps.size());
  const uint32_t k = C.k;
  int rc = SHINE_OK;
  shine_stats agg{};
  const uint64_t e = elem_bytes(h->elem);
  auto give_all = [&]() {
    for (uint32_t r = 0; r < G && r < C.stage.size(); ++r) give_stage(h->reps[r], C.stage[r]);
  };
  // results of the slot's queries lo .. hi-1 out of the staging into the caller's arrays, and their counters
  auto collect = [&](uint32_t r, uint32_t lo, uint32_t hi) {
    const HostStage& S = *C.stage[r];
    const std::vector<uint32_t>& pr = C.part[r];
    const bool run = hi > lo && pr[hi - 1] - pr[lo] == hi - 1 - lo;  // queries in call order: bulk copies
    if (run) {
      std::memcpy(C.out_ids + static_cast<size_t>(pr[lo]) * k, S.hids.p + static_cast<size_t>(lo) * k,
                  static_cast<size_t>(hi - lo) * k * 4);
      if (C.out_dists)
        std::memcpy(C.out_dists + static_cast<size_t>(pr[lo]) * k, S.hd.p + static_cast<size_t>(lo) * k,
                    static_cast<size_t>(hi - lo) * k * 4);
    }
    for (size_t j = lo; j < hi; ++j) {
      const uint32_t qi = pr[j];
      if (!run) {
        std::memcpy(C.out_ids + static_cast<size_t>(qi) * k, S.hids.p + j * k, k * 4);
        if (C.out_dists) std::memcpy(C.out_dists + static_cast<size_t>(qi) * k, S.hd.p + j * k, k * 4);
      }
      const uint32_t* qs = S.hqs.p + j * kQsWords;
      if (C.qstats) std::memcpy(C.qstats + static_cast<size_t>(qi) * SHINE_QS_WORDS, qs, SHINE_QS_WORDS * 4);
      if (qs[SHINE_QS_STATUS] != 0 && rc == SHINE_OK)
        rc = set_error(static_cast<int>(qs[SHINE_QS_STATUS]),
                       "query " + std::to_string(qi) + " failed with status " + std::to_string(qs[SHINE_QS_STATUS]));
      agg.processed += qs[SHINE_QS_STATUS] == 0 ? 1 : 0;
      agg.distcomps += qs[SHINE_QS_DISTCOMPS];
      agg.visited_nodes += qs[SHINE_QS_VISITED_UPPER];
      agg.visited_nodes_l0 += qs[SHINE_QS_VISITED_L0];
      agg.visited_neighborlists += qs[SHINE_QS_LISTS_L0] + qs[SHINE_QS_LISTS_UPPER];
      agg.visited_neighborlists_l0 += qs[SHINE_QS_LISTS_L0];
      agg.rdma_reads_in_bytes += ref_read_bytes(h, qs);
      agg.algorithmic_bytes += bq_bytes(h, qs);
      agg.remote_reads_in_bytes += qs[SHINE_QS_REMOTE_VEC] * h->dim * e + qs[SHINE_QS_REMOTE_LIST] * 4ull * h->M0;
      agg.cache_hits += qs[SHINE_QS_CACHED_VEC] + qs[SHINE_QS_CACHED_LIST];
      agg.cache_misses += qs[SHINE_QS_REMOTE_VEC] + qs[SHINE_QS_REMOTE_LIST];
      // every node read is a cache lookup in the reference (hnsw.hh:524-548): distcomps less the top push (:285)
      agg.node_reads += qs[SHINE_QS_DISTCOMPS] > 0 ? qs[SHINE_QS_DISTCOMPS] - 1 : 0;
      agg.node_cache_hits += qs[SHINE_QS_CACHED_VEC];
    }
  };
  double kernel_ms = 0;
  uint64_t retries = 0;
  for (uint32_t r = 0; r < G; ++r) {
    const uint32_t n = static_cast<uint32_t>(C.part[r].size());
    if (n == 0) continue;
    Replica& R = h->reps[r];
    HIP_TRY(hipSetDevice(R.device));
    HostStage& S = *C.stage[r];
    float ms = 0;
    for (uint32_t c = 0, off = 0; off < n; ++c, off += C.csize[r]) {  // chunk by chunk, in order
      HIP_TRY(hipEventSynchronize(S.hchunk[c]));
      collect(r, off, std::min(n, off + C.csize[r]));
      float mc = 0;
      HIP_TRY(hipEventElapsedTime(&mc, S.ev0, S.hchunk[c]));
      ms = std::max(ms, mc);
      if (C.chunked[r]) {
        const volatile uint32_t* cc = S.hcnt.p + 2ull * c;
        if (cc[1]) retries += cc[0];
      }
    }
    if (!C.chunked[r]) {
      HIP_TRY(hipStreamSynchronize(R.stream));  // (the log counts' copy behind the searches)
      const uint32_t* cnt = R.main.seen.p;      // written by the call's last pass (finish_call)
      retries += cnt[0] + cnt[1] + cnt[2];      // queries handed on by each pass
    }
    kernel_ms = std::max(kernel_ms, static_cast<double>(ms));
    if (r < h->slot_rate.size() && ms > 0) h->slot_rate[r] = n / static_cast<double>(ms);
    if (env_int("SHINE_PHASE_PROFILE", 0) && R.prof.p) print_phase_profile(h, R);
  }
  give_all();
  agg.overflow_retries = retries;
  agg.kernel_ms = kernel_ms;
  if (C.dynamic) {
    // this call's logs to the host (device-API searches on other streams of a slot log into the same buffers: the
    // device drains first when one ran)
    const auto t0 = std::chrono::steady_clock::now();
    const auto t_coll = C.t_launched;
    for (uint32_t r = 0; r < G; ++r) {
      Replica& R = h->reps[r];
      HIP_TRY(hipSetDevice(R.device));
      if (!C.lagged || R.dev_api_dirty) {
        HIP_TRY(hipDeviceSynchronize());
        R.dev_api_dirty = false;
        R.counts_inflight = false;  // counted again after every stream's searches
      }
      ++R.dyn_call;  // the coin's call counter: one per host call
    }
    if (int e2 = fetch_logs(h)) return e2;
    if (!C.lagged) {  // the updates before the call returns
      std::vector<shine_stats> now;
      replay_all(h, now);
      C.per.insert(C.per.end(), now.begin(), now.end());
      for (uint32_t r = 0; r < G; ++r) {
        if (int e2 = enqueue_update(h, h->reps[r])) return e2;
        HIP_TRY(hipStreamSynchronize(h->reps[r].stream));
      }
    }
    for (const shine_stats& p : C.per) {
      agg.cache_admitted += p.cache_admitted;
      agg.cache_evicted += p.cache_evicted;
      agg.cache_rescued += p.cache_rescued;
      agg.cache_log_dropped += p.cache_log_dropped;
    }
    if (env_int("SHINE_DEBUG_CACHE_TIMING", 0)) {  // diagnostics: where the time between calls goes
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      auto d = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      std::fprintf(stderr, "cache timing: kernel %.3f ms, waited for the previous replay %.3f ms, enqueue %.3f ms, "
                   "launch to results %.3f ms, after the searches %.3f ms, admitted %llu (%s)\n", kernel_ms, C.replay_ms,
                   d(C.t_enq, C.t_launched), d(t_coll, t0), ms, static_cast<unsigned long long>(agg.cache_admitted),
                   C.lagged ? "pipelined" : "synchronous");
    }
  }
  if (stats) *stats = agg;
  return rc;
}

// shine_knn_batch with the handle locked.  access (nullable): per-slot device counters of record reads (warmup).
int knn_host(shine_index* h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k, uint32_t ef,
             uint32_t* out_ids, float* out_dists, uint32_t* qstats, shine_stats* stats,
             std::vector<DevBuf<uint32_t>>* access) {
  shine_request C;
  C.h = h;
  C.nq = nq;
  C.k = k;
  C.out_ids = out_ids;
  C.out_dists = out_dists;
  C.qstats = qstats;
  C.access = access;
  if (int rc = knn_enqueue(h, C, queries, query_ids, ef)) {
    for (uint32_t r = 0; r < C.stage.size(); ++r) give_stage(h->reps[r], C.stage[r]);
    return rc;
  }
  return knn_collect(h, C, stats);
}

}  // namespace

extern "C" {

int shine_knn_batch(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                    uint32_t ef, uint32_t* out_ids, float* out_dists, shine_stats* stats) {
  return shine_knn_batch_ex(h, queries, query_ids, nq, k, ef, out_ids, out_dists, nullptr, stats);
}

int shine_knn_batch_ex(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                       uint32_t ef, uint32_t* out_ids, float* out_dists, uint32_t* qstats, shine_stats* stats) {
  if (int rc = check_knn_args(h, k, ef)) return rc;
  if (stats) std::memset(stats, 0, sizeof(*stats));
  if (nq == 0) return SHINE_OK;
  if (!queries || !out_ids) return set_error(SHINE_ERR_ARG, "NULL host pointer");
  std::lock_guard<std::mutex> lk(h->mu);
  return knn_host(h, queries, query_ids, nq, k, ef, out_ids, out_dists, qstats, stats, nullptr);
}

int shine_knn_batch_async(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                          uint32_t ef, uint32_t* out_ids, float* out_dists, uint32_t* qstats, shine_request_t* out) {
  if (!out) return set_error(SHINE_ERR_ARG, "NULL request pointer");
  *out = nullptr;
  if (int rc = check_knn_args(h, k, ef)) return rc;
  if (nq > 0 && (!queries || !out_ids)) return set_error(SHINE_ERR_ARG, "NULL host pointer");
  std::lock_guard<std::mutex> lk(h->mu);
  auto C = std::make_unique<shine_request>();
  C->h = h;
  C->nq = nq;
  C->k = k;
  C->out_ids = out_ids;
  C->out_dists = out_dists;
  C->qstats = qstats;
  C->rotate = true;
  if (nq > 0) {
    const int rc = knn_enqueue(h, *C, queries, query_ids, ef);
    if (rc) {
      for (uint32_t r = 0; r < C->stage.size(); ++r) give_stage(h->reps[r], C->stage[r]);
      return rc;
    }
    // the dynamic cache replays a call's logs between calls, in call order: such a call is collected at once
    if (C->dynamic) {
      C->rc = knn_collect(h, *C, &C->stats);
      C->collected = true;
    }
  } else {
    C->collected = true;
  }
  h->requests.push_back(C.get());
  *out = C.release();
  return SHINE_OK;
}

int shine_wait(shine_request_t req, shine_stats* stats) {
  if (!req) return set_error(SHINE_ERR_ARG, "request is NULL");
  shine_index* h = req->h;
  int rc = SHINE_OK;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    if (!req->collected) {
      req->rc = knn_collect(h, *req, &req->stats);
      req->collected = true;
    }
    rc = req->rc;
    if (stats) *stats = req->stats;
    for (uint32_t r = 0; r < req->stage.size(); ++r) give_stage(h->reps[r], req->stage[r]);  // (an error path)
    h->requests.erase(std::remove(h->requests.begin(), h->requests.end(), req), h->requests.end());
  }
  delete req;
  return rc;  // (shine_last_error holds the message set when the call was collected)
}

int shine_prepare(shine_index_t h, uint32_t nq, uint32_t k, uint32_t ef) {
  if (int rc = check_knn_args(h, k, ef)) return rc;
  if (nq == 0) return SHINE_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  const size_t n = nq;
  std::vector<float> q(n * h->dim, 0.f);
  std::vector<uint32_t> ids(n * k);
  const bool dynamic = h->cache_policy == SHINE_CACHE_DYNAMIC;
  // The setup searches leave the cache as it was: the logs of earlier calls not replayed yet (a pipelined call's) are
  // set aside, so that the setup call does not replay them with its statistics discarded, and put back after it;
  // the setup's own logs are dropped and the coin's call count restored.
  struct Stash {
    std::vector<unsigned long long> clog;
    std::vector<uint32_t> rlog;
    uint64_t lost = 0;
    uint32_t call = 0;
  };
  std::vector<Stash> stash(h->reps.size());
  std::vector<shine_stats> unreported;
  if (dynamic) {
    if (int rc = wait_replay(h)) return rc;
    unreported.swap(h->replay_unreported);
    for (size_t r = 0; r < h->reps.size(); ++r) {
      Replica& R = h->reps[r];
      stash[r].clog.swap(R.pend_clog);
      stash[r].rlog.swap(R.pend_rlog);
      stash[r].lost = R.pend_lost;
      stash[r].call = R.dyn_call;
      R.pend_lost = 0;
    }
  }
  int rc = knn_host(h, q.data(), nullptr, nq, k, ef, ids.data(), nullptr, nullptr, nullptr, nullptr);
  if (rc == SHINE_OK && !dynamic) {
    // Calls kept in flight (shine_knn_batch_async) hold a staging set each and start at the next host stream: as many
    // setup calls in flight as a slot has host streams, so that every stream's scratch and every staging set a caller
    // keeping calls in flight needs exist before its timer starts (found on the first calls otherwise: 2.4 M against
    // 5.1 M QPS for the compute node's 10,000 queries in four calls, two in flight)
    size_t S = 1;
    for (const Replica& R : h->reps) S = std::max(S, R.hstreams.size());
    std::vector<std::unique_ptr<shine_request>> reqs;
    for (size_t i = 0; i < S && rc == SHINE_OK; ++i) {
      auto C = std::make_unique<shine_request>();
      C->h = h;
      C->nq = nq;
      C->k = k;
      C->out_ids = ids.data();
      C->rotate = true;
      rc = knn_enqueue(h, *C, q.data(), nullptr, ef);
      if (rc) {
        for (uint32_t r = 0; r < C->stage.size(); ++r) give_stage(h->reps[r], C->stage[r]);
        break;
      }
      reqs.push_back(std::move(C));
    }
    for (auto& C : reqs) {
      const int r2 = knn_collect(h, *C, nullptr);
      if (rc == SHINE_OK) rc = r2;
    }
  }
  if (dynamic) {
    for (size_t r = 0; r < h->reps.size(); ++r) {
      Replica& R = h->reps[r];
      R.pend_clog.swap(stash[r].clog);
      R.pend_rlog.swap(stash[r].rlog);
      R.pend_lost = stash[r].lost;
      R.dyn_call = stash[r].call;
    }
    h->replay_unreported.swap(unreported);
  }
  return rc;
}

int shine_cache_warmup(shine_index_t h, const float* queries, const uint32_t* query_ids, uint32_t nq, uint32_t k,
                       uint32_t ef) {
  if (int rc = check_knn_args(h, k, ef)) return rc;
  if (nq == 0) return SHINE_OK;
  if (!queries) return set_error(SHINE_ERR_ARG, "NULL host pointer");
  std::lock_guard<std::mutex> lk(h->mu);
  if (int rc = wait_replay(h)) return rc;
  const uint32_t G = static_cast<uint32_t>(h->reps.size());
  if (h->placement == SHINE_PLACE_REPLICA || G < 2 || (h->cached_rows == 0 && h->cached_list_rows == 0))
    return SHINE_OK;  // nothing is cached
  if (h->host.N == 0 || h->dev_of.size() != h->host.N)
    return set_error(SHINE_ERR_ARG, "the index's host graph is gone (an earlier warmup failed): reopen it");
  // 1. the warmup split, with every record read counted per slot (the reference's warmup run, compute_node.cc:116-131)
  std::vector<DevBuf<uint32_t>> access(G);
  auto free_access = [&]() {
    for (uint32_t r = 0; r < G; ++r) {
      (void)hipSetDevice(h->reps[r].device);
      access[r].release();
    }
  };
  for (uint32_t r = 0; r < G; ++r) {
    HIP_TRY(hipSetDevice(h->reps[r].device));
    if (int rc = access[r].grow(h->id_space)) return free_access(), rc;
    HIP_TRY(hipMemsetAsync(access[r].p, 0, h->id_space * 4, h->reps[r].stream));
  }
  std::vector<uint32_t> ids(static_cast<size_t>(nq) * k);
  if (int rc = knn_host(h, queries, query_ids, nq, k, ef, ids.data(), nullptr, nullptr, nullptr, &access))
    return free_access(), rc;
  // 2. admission ranking: reads summed over the slots, per graph node
  std::vector<uint32_t> part(h->id_space), heat(h->host.N, 0);
  for (uint32_t r = 0; r < G; ++r) {
    HIP_TRY(hipSetDevice(h->reps[r].device));
    HIP_TRY(hipMemcpy(part.data(), access[r].p, h->id_space * 4, hipMemcpyDeviceToHost));
    for (uint64_t g = 0; g < h->host.N; ++g) heat[g] += part[h->dev_of[g]];
  }
  free_access();
  // 3. the same stripes re-laid out hottest first (a new layout beside the old one, then moved in)
  shine_index_t nh = nullptr;
  const std::vector<int> devs = h->devs;
  // the host graph moves into the new layout; if building it fails, the handle keeps its old layout and no host graph
  // (a later warmup reports that instead of relaying out from emptied arrays)
  HostGraph hg = std::move(h->host);
  h->host = HostGraph{};
  h->dev_of.clear();
  if (int rc = make_index(std::move(hg), h->elem, devs.data(), static_cast<uint32_t>(devs.size()), h->placement,
                          h->cache_requested, &nh, &heat))
    return rc;
  nh->search_mode = h->search_mode;
  release_state(h);
  static_cast<IndexState&>(*h) = std::move(static_cast<IndexState&>(*nh));
  delete nh;  // its state was moved out: nothing left to release
  return SHINE_OK;
}

int shine_release_stream(shine_index_t h, void* stream) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  if (!stream) return SHINE_OK;  // the handle's own streams live as long as the handle
  std::lock_guard<std::mutex> lk(h->mu);
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (auto& R : h->reps) {
    for (auto it = R.by_stream.begin(); it != R.by_stream.end(); ++it) {
      if (it->first != s) continue;
      HIP_TRY(hipSetDevice(R.device));
      HIP_TRY(hipStreamSynchronize(s));
      it->second->release();
      R.by_stream.erase(it);
      break;
    }
  }
  return SHINE_OK;
}

int shine_route(shine_index_t h, const float* queries, uint32_t nq, uint32_t* out_slot) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  if (nq == 0) return SHINE_OK;
  if (!queries || !out_slot) return set_error(SHINE_ERR_ARG, "NULL host pointer");
  route_batch(h, queries, nullptr, nq, out_slot);
  return SHINE_OK;
}

int shine_plan_regions(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim, uint32_t M,
                       int metric, uint32_t k, uint32_t* region_of_uid, uint64_t uid_capacity, float* centroids,
                       uint32_t* mapping, uint32_t* n_centroids) {
  if (!dumps || !sizes) return set_error(SHINE_ERR_ARG, "dumps / sizes is NULL");
  if (k == 0) return set_error(SHINE_ERR_ARG, "k must be > 0");
  if (metric != SHINE_METRIC_L2 && metric != SHINE_METRIC_IP) return set_error(SHINE_ERR_ARG, "metric must be 0 or 1");
  HostGraph G;
  if (int rc = parse_dumps(dumps, sizes, n_dumps, dim, M, metric, 0, G)) return rc;
  Regions R;
  if (plan_regions(G, k, true, R)) return set_error(SHINE_ERR_ARG, "fewer top-level nodes than k-means clusters");
  if (centroids) std::memcpy(centroids, R.centroids.data(), R.centroids.size() * sizeof(float));
  if (mapping) std::memcpy(mapping, R.mapping.data(), R.mapping.size() * sizeof(uint32_t));
  if (n_centroids) *n_centroids = R.n_centroids();
  if (region_of_uid) {
    const std::vector<uint32_t> region = assign_regions(G, R, 0.05, 1);
    for (uint64_t g = 0; g < G.N; ++g) {
      if (G.uid[g] >= uid_capacity) return set_error(SHINE_ERR_ARG, "uid_capacity is below the largest uid + 1");
      region_of_uid[G.uid[g]] = region[g];
    }
  }
  return SHINE_OK;
}

int shine_kmeans(const float* rows, uint64_t n, uint32_t dim, int metric, uint32_t k, int balanced, float* centroids,
                 uint32_t* mapping, uint32_t* n_centroids, uint64_t* region_sizes, uint32_t* iterations) {
  if (!rows || !centroids || !mapping) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (k == 0 || dim == 0) return set_error(SHINE_ERR_ARG, "k and dim must be > 0");
  if (metric != SHINE_METRIC_L2 && metric != SHINE_METRIC_IP) return set_error(SHINE_ERR_ARG, "metric must be 0 or 1");
  KmeansInput in;
  in.metric = metric;
  in.dim = dim;
  in.rows.resize(n);
  for (uint64_t i = 0; i < n; ++i) in.rows[i] = rows + i * dim;
  Regions R;
  if (run_and_optimize(in, k, balanced != 0, R)) return set_error(SHINE_ERR_ARG, "fewer rows than k-means clusters");
  std::memcpy(centroids, R.centroids.data(), R.centroids.size() * sizeof(float));
  std::memcpy(mapping, R.mapping.data(), R.mapping.size() * sizeof(uint32_t));
  if (n_centroids) *n_centroids = R.n_centroids();
  if (region_sizes) std::memcpy(region_sizes, R.sizes.data(), R.sizes.size() * sizeof(uint64_t));
  if (iterations) {
    iterations[0] = R.iterations;
    iterations[1] = R.balance_iterations;
  }
  return SHINE_OK;
}

int shine_router_run(const float* centroids, const uint32_t* mapping, uint32_t n_centroids, uint32_t k, uint32_t dim,
                     int metric, const float* queries, uint32_t nq, const uint32_t* queue_sizes, uint32_t n_rows,
                     int adaptive, uint32_t* out_region, uint64_t* out_limits) {
  if (!centroids || !mapping || (!queries && nq) || (!out_region && nq)) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (k == 0 || n_centroids == 0 || dim == 0) return set_error(SHINE_ERR_ARG, "k, n_centroids and dim must be > 0");
  for (uint32_t i = 0; i < n_centroids; ++i)
    if (mapping[i] >= k) return set_error(SHINE_ERR_ARG, "mapping names a region >= k");
  Regions R;
  R.k = k;
  R.dim = dim;
  R.metric = metric;
  R.centroids.assign(centroids, centroids + static_cast<size_t>(n_centroids) * dim);
  R.mapping.assign(mapping, mapping + n_centroids);
  Router router;
  router.init(k);
  router.adaptive = adaptive != 0;
  uint32_t boundary = 0;
  router.route(R, queries, nq, dim,
               [&](const std::vector<uint64_t>&, std::vector<uint32_t>& p) {
                 if (queue_sizes && n_rows) {
                   const uint32_t row = std::min(boundary, n_rows - 1);
                   std::copy(queue_sizes + static_cast<size_t>(row) * k, queue_sizes + static_cast<size_t>(row + 1) * k,
                             p.begin());
                 }
                 ++boundary;
               },
               out_region);
  if (out_limits) std::copy(router.limits.begin(), router.limits.end(), out_limits);
  return SHINE_OK;
}

int shine_graph_stats_buffers(const uint8_t* const* dumps, const uint64_t* sizes, uint32_t n_dumps, uint32_t dim,
                              uint32_t M, shine_graph_stats* out) {
  if (!dumps || !sizes || !out) return set_error(SHINE_ERR_ARG, "NULL argument");
  HostGraph G;
  if (int rc = parse_dumps(dumps, sizes, n_dumps, dim, M, SHINE_METRIC_L2, 0, G)) return rc;
  const GraphReach r = graph_reach(G);
  std::memset(out, 0, sizeof(*out));
  out->num_nodes = r.num_nodes;
  out->reachable_l0 = r.reachable_l0;
  out->reachable_any = r.reachable_any;
  out->zero_indegree_l0 = r.zero_indegree_l0;
  out->full_lists_l0 = r.full_lists_l0;
  out->mean_degree_l0 = r.mean_degree_l0;
  out->max_level = r.max_level;
  return SHINE_OK;
}

int shine_distance_batch_device(shine_index_t h, uint32_t gpu_slot, const float* d_queries, uint32_t nq,
                                const uint32_t* d_node_uids, uint32_t n_per_query, float* d_out, void* stream) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  if (gpu_slot >= h->reps.size()) return set_error(SHINE_ERR_ARG, "gpu_slot out of range");
  if (nq == 0 || n_per_query == 0) return SHINE_OK;
  if (!d_queries || !d_node_uids || !d_out) return set_error(SHINE_ERR_ARG, "NULL device pointer");
  std::lock_guard<std::mutex> lk(h->mu);
  Replica& R = h->reps[gpu_slot];
  HIP_TRY(hipSetDevice(R.device));
  DistArgs a{};
  a.g = dev_graph(h, R);
  if (!a.g.vec || !a.g.inv_uid) return set_error(SHINE_ERR_HIP, "distance launch: an index array is missing");
  a.queries = d_queries;
  a.nq = nq;
  a.node_uids = d_node_uids;
  a.n_per = n_per_query;
  a.out = d_out;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : R.stream;
  hipError_t e = launch_distance(h->dim, h->metric, h->elem, a, s);
  if (e != hipSuccess) return set_error(SHINE_ERR_HIP, std::string("distance launch: ") + hipGetErrorString(e));
  return SHINE_OK;
}

int shine_selftest_heap(int is_max, const int32_t* ops, const float* vals, const uint32_t* ids, uint32_t n_ops,
                        uint32_t k, float* out_d, uint32_t* out_ids, uint32_t* out_n) {
  if (!ops || !vals || !ids || !out_d || !out_ids || !out_n) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (n_ops == 0 || n_ops > 16384) return set_error(SHINE_ERR_ARG, "n_ops must be in [1, 16384]");
  HIP_TRY(hipSetDevice(0));
  DevBuf<int32_t> dops;
  DevBuf<float> dvals, dd;
  DevBuf<uint32_t> dids, di, dn;
  auto cleanup = [&]() { dops.release(); dvals.release(); dd.release(); dids.release(); di.release(); dn.release(); };
  int rc = 0;
  if ((rc = dops.grow(n_ops)) || (rc = dvals.grow(n_ops)) || (rc = dids.grow(n_ops)) || (rc = dd.grow(n_ops + 1)) ||
      (rc = di.grow(n_ops + 1)) || (rc = dn.grow(1))) {
    cleanup();
    return rc;
  }
  hipError_t e = hipMemcpy(dops.p, ops, 4ull * n_ops, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dvals.p, vals, 4ull * n_ops, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dids.p, ids, 4ull * n_ops, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_heap_replay(is_max, dops.p, dvals.p, dids.p, n_ops, k, dd.p, di.p, dn.p, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out_n, dn.p, 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && *out_n) e = hipMemcpy(out_d, dd.p, 4ull * *out_n, hipMemcpyDeviceToHost);
  if (e == hipSuccess && *out_n) e = hipMemcpy(out_ids, di.p, 4ull * *out_n, hipMemcpyDeviceToHost);
  cleanup();
  if (e != hipSuccess) return set_error(SHINE_ERR_HIP, std::string("heap replay: ") + hipGetErrorString(e));
  return SHINE_OK;
}

int shine_set_cache_policy(shine_index_t h, int policy, double ratio_percent, uint64_t seed) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  if (int rc = wait_replay(h)) return rc;
  h->replay_unreported.clear();
  if (policy == SHINE_CACHE_STATIC) {
    for (auto& R : h->reps) {
      HIP_TRY(hipSetDevice(R.device));
      HIP_TRY(hipDeviceSynchronize());
      R.release_dynamic();
    }
    h->cache_policy = SHINE_CACHE_STATIC;
    return SHINE_OK;
  }
  if (policy != SHINE_CACHE_DYNAMIC) return set_error(SHINE_ERR_ARG, "unknown cache policy");
  if (h->placement == SHINE_PLACE_REPLICA || h->reps.size() < 2)
    return set_error(SHINE_ERR_ARG, "the dynamic cache needs a sharded placement over >= 2 GPU slots");
  if (h->cached_rows || h->cached_list_rows)
    return set_error(SHINE_ERR_ARG, "the handle holds a static cache (cache_fraction > 0): open it with 0");
  if (!(ratio_percent > 0.0 && ratio_percent <= 100.0)) return set_error(SHINE_ERR_ARG, "ratio must be in (0, 100]");
  const uint64_t entries = std::min<uint64_t>(cache_entries(h->N, h->M, h->dim, ratio_percent), 0x7FFFFFFFull);
  if (!RecordCache::size_ok(static_cast<uint32_t>(entries)))
    return set_error(SHINE_ERR_ARG, "the cache ratio gives " + std::to_string(entries) +
                                        " entries, no more than its cooling table holds (the reference's eviction "
                                        "would never end)");
  const uint64_t vrow = row_bytes(h->dim, h->elem);
  for (auto& R : h->reps) {
    HIP_TRY(hipSetDevice(R.device));
    HIP_TRY(hipDeviceSynchronize());
    R.release_dynamic();
    R.clog_cap = 1u << 22;
    // hits on cooling entries: each arena slot at most once per log epoch (kernels_impl.h count_vec_reads), and an
    // epoch's slots change occupant at most once (the updates between calls): twice the arena holds every entry
    R.rlog_cap = static_cast<uint32_t>(std::max<uint64_t>(4096, 2 * entries));
    int rc = 0;
    if ((rc = R.cslot.grow(h->id_space)) || (rc = R.cbits.grow((h->id_space + 31) / 32)) ||
        (rc = R.cvec.grow(entries * vrow)) || (rc = R.cool.grow(entries)) || (rc = R.rlogged.grow(entries)) ||
        (rc = R.slot_id.grow(entries)) ||
        (rc = R.clog.grow(R.clog_cap)) || (rc = R.rlog.grow(R.rlog_cap)) || (rc = R.logn.grow(2))) {
      R.release_dynamic();
      return rc;
    }
    HIP_TRY(hipMemsetAsync(R.cslot.p, 0xFF, h->id_space * sizeof(uint32_t), R.stream));
    HIP_TRY(hipMemsetAsync(R.cbits.p, 0, (h->id_space + 31) / 32 * sizeof(uint32_t), R.stream));
    HIP_TRY(hipMemsetAsync(R.cool.p, 0, entries * sizeof(uint32_t), R.stream));
    HIP_TRY(hipMemsetAsync(R.rlogged.p, 0xFF, entries * sizeof(uint32_t), R.stream));
    HIP_TRY(hipMemsetAsync(R.slot_id.p, 0xFF, entries * sizeof(uint32_t), R.stream));
    HIP_TRY(hipMemsetAsync(R.logn.p, 0, 2 * sizeof(uint32_t), R.stream));
    HIP_TRY(hipStreamSynchronize(R.stream));
    R.cache = RecordCache(static_cast<uint32_t>(entries), seed + R.slot, h->inv_size);  // keys: uids < inv_size
    R.dyn_full = R.cache.full();
  }
  h->cache_policy = SHINE_CACHE_DYNAMIC;
  h->cache_seed = seed;
  h->cache_entries_per_gpu = entries;
  return SHINE_OK;
}

int shine_cache_update(shine_index_t h) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->cache_policy != SHINE_CACHE_DYNAMIC) return SHINE_OK;
  if (int rc = wait_replay(h)) return rc;
  for (auto& R : h->reps) {  // every stream of the slot may have searched: wait for the device
    HIP_TRY(hipSetDevice(R.device));
    HIP_TRY(hipDeviceSynchronize());
    R.dev_api_dirty = false;
    R.counts_inflight = false;  // device-API searches may have logged since: counted again
  }
  if (int rc = fetch_logs(h)) return rc;
  std::vector<shine_stats> per;
  replay_all(h, per);  // every log not replayed yet (a pipelined call's, device-API searches')
  for (auto& R : h->reps) {
    if (int rc = enqueue_update(h, R)) return rc;
    HIP_TRY(hipStreamSynchronize(R.stream));
  }
  return SHINE_OK;
}

int shine_cache_wait(shine_index_t h) {
  if (!h) return set_error(SHINE_ERR_ARG, "index handle is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  return wait_replay(h);
}

int shine_cache_keys(shine_index_t h, uint32_t slot, uint32_t* uids, uint64_t cap, uint64_t* n) {
  if (!h || !n) return set_error(SHINE_ERR_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(h->mu);
  if (slot >= h->reps.size()) return set_error(SHINE_ERR_ARG, "gpu_slot out of range");
  if (int rc = wait_replay(h)) return rc;  // (the engine as the last call left it)
  const std::vector<uint32_t> keys = h->reps[slot].cache.keys();
  *n = keys.size();
  if (uids) std::copy(keys.begin(), keys.begin() + std::min<uint64_t>(cap, keys.size()), uids);
  return SHINE_OK;
}

int shine_device_ids(shine_index_t h, const uint32_t* uids, uint32_t n, uint32_t* out) {
  if (!h || (n && (!uids || !out))) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (h->dev_of_uid.empty()) return set_error(SHINE_ERR_ARG, "device ids are kept for sharded placements only");
  for (uint32_t i = 0; i < n; ++i) out[i] = uids[i] < h->dev_of_uid.size() ? h->dev_of_uid[uids[i]] : kInvalid;
  return SHINE_OK;
}

int shine_selftest_cache(uint32_t entries, uint64_t seed, uint32_t n_calls, const uint32_t* cand_off,
                         const uint32_t* cand, const uint32_t* resc_off, const uint32_t* resc, uint32_t* keys,
                         uint64_t cap, uint64_t* n, uint64_t* counts) {
  if (!cand_off || !resc_off || !n || !counts) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (!RecordCache::size_ok(entries)) return set_error(SHINE_ERR_ARG, "cache no larger than its cooling table");
  uint32_t key_space = 1;  // keys below the largest named + 1
  for (uint32_t i = cand_off[0]; i < cand_off[n_calls]; ++i) key_space = std::max(key_space, cand[3ull * i + 1] + 1);
  for (uint32_t i = resc_off[0]; i < resc_off[n_calls]; ++i) key_space = std::max(key_space, resc[i] + 1);
  RecordCache c(entries, seed, key_space);
  for (uint32_t call = 0; call < n_calls; ++call) {
    std::vector<uint32_t> rk(resc + resc_off[call], resc + resc_off[call + 1]);
    std::vector<CacheCandidate> cv;
    for (uint32_t i = cand_off[call]; i < cand_off[call + 1]; ++i) {
      const uint32_t* t = cand + 3ull * i;
      cv.push_back({t[0], t[1], t[1], (t[2] & 1u) != 0, (t[2] & 2u) != 0});
    }
    std::vector<CacheUpdate> ups;
    std::vector<uint32_t> flagged;
    c.apply_call(std::move(rk), std::move(cv), ups, flagged);
  }
  const std::vector<uint32_t> k = c.keys();
  *n = k.size();
  if (keys) std::copy(k.begin(), k.begin() + std::min<uint64_t>(cap, k.size()), keys);
  counts[0] = c.admitted;
  counts[1] = c.evicted;
  counts[2] = c.rescued;
  return SHINE_OK;
}

int shine_close(shine_index_t h) {
  if (!h) return SHINE_OK;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    (void)wait_replay(h);  // (its updates are dropped with the arena)
  }
  // requests never waited for: their staging goes back to the pools (freed, once the devices drain, with the rest)
  for (shine_request* q : h->requests) {
    for (uint32_t r = 0; r < q->stage.size() && r < h->reps.size(); ++r) give_stage(h->reps[r], q->stage[r]);
    delete q;
  }
  h->requests.clear();
  release_index(h);
  return SHINE_OK;
}

}  // extern "C"
