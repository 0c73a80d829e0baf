// GPU batch builder (include/shine_gpu.h shine_gpu_build*): HNSW::insert (src/hnsw/hnsw.hh:40-251)
// over batches of consecutive node ids on one MI355X, writing the graph straight into the search layout of capi.cc
// (an index handle in fast mode serves the level-0 candidate searches) and, on request, the reference's dump images
// (src/memory_node.hh:15-27, 185-201; records as rdma_writes.hh:75-171 writes them).
//
// Per batch, one stream, no host round trip (the host knows every level and so every batch's shape up front):
//   1. level-0 candidates: search_enqueue(k = ef = efC) — knn's greedy descent and search_level(efC, 0) (:129-154);
//   2. upper levels (records of level >= 1): build_upper_kernel — descent to level L + 1, beams at L .. 1 (:129-175);
//   3. build_select_kernel: select_heuristic(M) per list → own lists, reverse-edge requests (:155-180);
//   4. the requests sorted by target row (rocPRIM radix sort, stable), segment starts;
//   5. build_prune_kernel: per target row, append or re-prune with select_heuristic(m_max) (:180-225).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "index_internal.h"

using namespace shine;

namespace {

constexpr uint64_t kEntryNode = 0b10000000000000000;  // node.hh:30
constexpr uint32_t kUpperVisCap = 8192;                // LDS visited-table entries of build_upper_kernel (32 KiB)

int64_t env_int(const char* name, int64_t dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoll(e) : dflt;
}

// Host threads for host-side loops: OMP_NUM_THREADS when set (the GPU boxes grant 16 CPUs per GPU while the machine
// shows 256), else the hardware's, at most 16.
uint64_t host_threads() {
  const int64_t omp = env_int("OMP_NUM_THREADS", 0);
  if (omp > 0) return static_cast<uint64_t>(omp);
  return std::max<uint64_t>(1, std::min<uint64_t>(16, std::thread::hardware_concurrency()));
}

template <class T>
int upload_vec(DevBuf<T>& dst, const std::vector<T>& src, hipStream_t s) {
  if (int rc = dst.grow(std::max<size_t>(src.size(), 1))) return rc;
  if (!src.empty()) HIP_TRY(hipMemcpyAsync(dst.p, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return 0;
}

}  // namespace

struct shine_gpu_builder {
  uint32_t dim = 0, M = 0, M0 = 0, efc = 0, seed = 0;
  int metric = 0, device = 0;
  uint64_t N = 0, R = 0;
  std::vector<uint32_t> level;    // effective level of every record
  std::vector<uint32_t> up_base;  // first upper row (kInvalid at level 0)
  uint32_t ep = 0, ep_level = 0;
  shine_index* h = nullptr;       // the graph in the search layout (replica, fast mode) until shine_gpu_build_open
  shine_gpu_build_stats st{};
  std::vector<std::vector<uint8_t>> dumps;
  ~shine_gpu_builder() {
    if (h) index_release(h);
  }
};

namespace {

// Levels exactly as builder.cc / the oracle draw them (hnsw.hh:30, 34-35, 48) and as insert() assigns them: the first
// record takes level 0 (:63-76), a record drawn above the top level takes top + 1 and becomes the entry point (:98-111).
void draw_levels(uint64_t n, uint32_t M, uint32_t seed, std::vector<uint32_t>& eff, std::vector<uint8_t>& is_new) {
  std::mt19937 prng(seed);
  std::uniform_real_distribution<> uniform(0., 1.);
  const double nf = 1. / std::log(static_cast<double>(M));
  eff.assign(n, 0);
  is_new.assign(n, 0);
  uint32_t top = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t drawn = static_cast<uint32_t>(std::floor(-std::log(uniform(prng)) * nf));
    if (i == 0) continue;
    if (drawn > top) {
      eff[i] = ++top;
      is_new[i] = 1;
    } else {
      eff[i] = drawn;
    }
  }
}

// The internal search handle over the build arrays (replica on `device`, f32 rows, fast mode).
int make_build_handle(shine_gpu_builder* b, hipStream_t& stream_out) {
  hipDeviceProp_t prop{};
  HIP_TRY(hipGetDeviceProperties(&prop, b->device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_error(SHINE_ERR_HIP, std::string("GPU is ") + prop.gcnArchName + "; the kernels are built for gfx950 only");
  std::unique_ptr<shine_index> h(new shine_index);
  struct Guard {
    std::unique_ptr<shine_index>& p;
    ~Guard() {
      if (p) index_release(p.release());
    }
  } guard{h};
  h->dim = b->dim;
  h->M = b->M;
  h->M0 = b->M0;
  h->metric = b->metric;
  h->elem = SHINE_ELEM_F32;
  h->N = b->N;
  h->upper_rows = b->R;
  h->ep = 0;
  h->ep_level = 0;
  h->ep_uid = 0;
  h->n_shards = 1;
  h->lists_unique = 1;
  h->inv_size = static_cast<uint32_t>(b->N);
  h->id_space = b->N;
  h->ids_per_slot = b->N;
  h->words_per_slot = (b->N + 31) / 32;
  h->placement = SHINE_PLACE_REPLICA;
  h->search_mode = SHINE_MODE_FAST;
  h->reps.resize(1);
  Replica& R = h->reps[0];
  R.device = b->device;
  R.slot = 0;
  R.cus = static_cast<uint32_t>(std::max(1, prop.multiProcessorCount));
  R.lds_per_cu = static_cast<uint32_t>(prop.maxSharedMemoryPerMultiProcessor > 0 ? prop.maxSharedMemoryPerMultiProcessor
                                                                                 : prop.sharedMemPerBlock);
  R.pad_node = 0;
  HIP_TRY(hipSetDevice(R.device));
  HIP_TRY(hipStreamCreateWithFlags(&R.stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreate(&R.ev0));
  HIP_TRY(hipEventCreate(&R.ev1));
  const uint64_t N = b->N;
  if (int rc = R.vec.grow(N * b->dim * 4)) return rc;
  if (int rc = R.adj0.grow(N * b->M0)) return rc;
  if (int rc = R.adjU.grow(std::max<uint64_t>(1, b->R * b->M))) return rc;
  if (int rc = R.uid.grow(N)) return rc;
  if (int rc = R.inv_uid.grow(N)) return rc;
  if (int rc = upload_vec(R.up_base, b->up_base, R.stream)) return rc;
  if (int rc = R.main.counter.grow(kCallWords)) return rc;
  HIP_TRY(hipMemsetAsync(R.adj0.p, 0xFF, R.adj0.n * 4, R.stream));
  HIP_TRY(hipMemsetAsync(R.adjU.p, 0xFF, R.adjU.n * 4, R.stream));
  HIP_TRY(launch_iota(R.uid.p, N, R.stream));
  HIP_TRY(launch_iota(R.inv_uid.p, N, R.stream));
  h->device_bytes = N * b->dim * 4 + N * b->M0 * 4ull + b->R * b->M * 4ull + 12ull * N;
  stream_out = R.stream;
  b->h = h.release();
  return 0;
}

int run_build(shine_gpu_builder* b, const float* base, bool on_device, double frac, uint32_t max_batch) {
  const auto t_start = std::chrono::steady_clock::now();
  const uint64_t N = b->N;
  const uint32_t dim = b->dim, M = b->M, efc = b->efc;
  std::vector<uint8_t> is_new;
  draw_levels(N, M, b->seed, b->level, is_new);
  // upper rows, their owners, and the upper-level candidate lists of every record (levels L .. 1, L = min(level,
  // top before it))
  b->up_base.assign(N, kInvalid);
  std::vector<uint32_t> row_owner, UN, UF, UL, LN, LL;
  uint64_t rows = 0;
  uint32_t top = 0;
  UF.push_back(0);
  for (uint64_t i = 0; i < N; ++i) {
    const uint32_t lv = b->level[i];
    if (lv > 0) {
      b->up_base[i] = static_cast<uint32_t>(rows);
      for (uint32_t l = 0; l < lv; ++l) row_owner.push_back(static_cast<uint32_t>(i));
      rows += lv;
    }
    const uint32_t L = i == 0 ? 0 : std::min(lv, top);
    if (L > 0) {
      UN.push_back(static_cast<uint32_t>(i));
      UL.push_back(L);
      for (uint32_t l = L; l >= 1; --l) {
        LN.push_back(static_cast<uint32_t>(i));
        LL.push_back(l);
      }
      UF.push_back(static_cast<uint32_t>(LN.size()));
    }
    top = std::max(top, lv);
  }
  if (rows >= kInvalid || N + rows >= kInvalid) return set_error(SHINE_ERR_ARG, "too many upper-level rows");
  b->R = rows;
  b->st.num_nodes = N;
  b->st.num_upper_rows = rows;
  hipStream_t s = nullptr;
  if (int rc = make_build_handle(b, s)) return rc;
  Replica& RP = b->h->reps[0];

  // rows into the device layout; the caller's unpermuted rows are the batches' queries
  DevBuf<float> base_own;
  const float* base_dev = base;
  if (!on_device) {
    if (int rc = base_own.grow(N * dim)) return rc;
    HIP_TRY(hipMemcpyAsync(base_own.p, base, N * dim * 4, hipMemcpyHostToDevice, s));
    base_dev = base_own.p;
  }
  HIP_TRY(launch_rows_to_device(base_dev, RP.vec.p, N, dim, SHINE_ELEM_F32, false, s));

  // the batch schedule (host), and the largest batch's shape for the scratch
  struct Batch {
    uint64_t start, n;
    uint32_t u0, u1;  // upper records [u0, u1) of UN
  };
  std::vector<Batch> sched;
  {
    uint64_t i = 1;
    uint32_t u = 0;
    while (i < N) {
      uint64_t nb = std::min<uint64_t>(max_batch, std::max<uint64_t>(1, static_cast<uint64_t>(frac * static_cast<double>(i))));
      if (is_new[i]) {
        nb = 1;
      } else {
        uint64_t j = i + 1;
        while (j < i + nb && j < N && !is_new[j]) ++j;
        nb = std::min<uint64_t>(j, N) - i;
      }
      const uint64_t e = i + nb;
      const uint32_t u0 = u;
      while (u < UN.size() && UN[u] < e) ++u;
      sched.push_back({i, nb, u0, u});
      i = e;
    }
  }
  uint64_t max_nb = 1, max_lists = 1, max_up = 1;
  for (const Batch& B : sched) {
    const uint64_t nl = UF[B.u1] - UF[B.u0];
    max_nb = std::max(max_nb, B.n);
    max_up = std::max<uint64_t>(max_up, B.u1 - B.u0);
    max_lists = std::max(max_lists, B.n + nl);
  }
  const uint64_t max_req = max_lists * M;
  if (max_req >= 0x80000000ull) return set_error(SHINE_ERR_ARG, "max_batch too large");

  DevBuf<uint32_t> dUN, dUF, dUL, dLN, dLL, dOwner, cand_ids, qs, req_key, req_src, req_pos, skey, sval, seg, ctr;
  DevBuf<float> cand_d, req_d;
  DevBuf<unsigned long long> dstats;
  DevBuf<uint8_t> sort_tmp;
  int rc = 0;
  if ((rc = upload_vec(dUN, UN, s)) || (rc = upload_vec(dUF, UF, s)) || (rc = upload_vec(dUL, UL, s)) ||
      (rc = upload_vec(dLN, LN, s)) || (rc = upload_vec(dLL, LL, s)) || (rc = upload_vec(dOwner, row_owner, s)) ||
      (rc = cand_ids.grow(max_lists * efc)) || (rc = cand_d.grow(max_lists * efc)) || (rc = qs.grow(max_nb * kQsWords)) ||
      (rc = req_key.grow(max_req)) || (rc = req_src.grow(max_req)) || (rc = req_pos.grow(max_req)) ||
      (rc = req_d.grow(max_req)) || (rc = skey.grow(max_req)) || (rc = sval.grow(max_req)) || (rc = seg.grow(max_req)) ||
      (rc = ctr.grow(2)) || (rc = dstats.grow(8)))
    return rc;
  HIP_TRY(hipMemsetAsync(dstats.p, 0, 8 * sizeof(unsigned long long), s));
  const uint32_t key_none = static_cast<uint32_t>(N + rows);
  uint32_t bits = 1;
  while (bits < 32 && (1ull << bits) <= key_none) ++bits;
  size_t tmp_bytes = 0;
  HIP_TRY(radix_sort_u32_pairs(nullptr, &tmp_bytes, req_key.p, skey.p, req_pos.p, sval.p,
                               static_cast<uint32_t>(max_req), bits, s));
  if ((rc = sort_tmp.grow(tmp_bytes + 256))) return rc;

  const bool prof = env_int("SHINE_BUILD_PROFILE", 0) != 0;
  hipEvent_t ev[6] = {};
  if (prof)
    for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
  auto phase_ms = [&](int a, int z) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ev[a], ev[z]);
    return static_cast<double>(ms);
  };
  const uint32_t prune_grid = RP.cus * 16;
  shine_index* h = b->h;
  BuildArgs A{};
  A.adj0w = RP.adj0.p;
  A.adjUw = RP.adjU.p;
  A.base = base_dev;
  A.ef = efc;
  A.M = M;
  A.cand_ids = cand_ids.p;
  A.cand_d = cand_d.p;
  A.vis_cap = kUpperVisCap;
  A.req_key = req_key.p;
  A.req_src = req_src.p;
  A.req_pos = req_pos.p;
  A.req_d = req_d.p;
  A.key_none = key_none;
  A.skey = skey.p;
  A.sval = sval.p;
  A.seg = seg.p;
  A.nseg = ctr.p;
  A.work = ctr.p + 1;
  A.row_owner = dOwner.p;
  A.stats = dstats.p;
  uint64_t n_lists_total = 0, n_req_total = 0;
  for (size_t bi = 0; bi < sched.size(); ++bi) {
    const Batch& B = sched[bi];
    h->ep = b->ep;
    h->ep_level = b->ep_level;
    const uint32_t nb = static_cast<uint32_t>(B.n);
    if (prof) HIP_TRY(hipEventRecord(ev[0], s));
    if ((rc = search_enqueue(h, 0, base_dev + B.start * dim, nb, efc, efc, cand_ids.p, cand_d.p, qs.p, s))) return rc;
    HIP_TRY(launch_qstats_sum(qs.p, nb, dstats.p + 4, s));
    if (prof) HIP_TRY(hipEventRecord(ev[1], s));
    // the graph as the kernels see it (dev_graph of capi.cc, replica)
    A.g = DevGraph{};
    A.g.vec = RP.vec.p;
    A.g.adj0 = RP.adj0.p;
    A.g.uid = RP.uid.p;
    A.g.up_base = RP.up_base.p;
    A.g.adjU = RP.adjU.p;
    A.g.inv_uid = RP.inv_uid.p;
    A.g.inv_size = static_cast<uint32_t>(N);
    A.g.N = static_cast<uint32_t>(N);
    A.g.M0 = b->M0;
    A.g.MU = M;
    A.g.ep = b->ep;
    A.g.ep_level = b->ep_level;
    A.g.lists_unique = 1;
    A.batch_start = static_cast<uint32_t>(B.start);
    A.n_lists0 = nb;
    A.n_up = B.u1 - B.u0;
    A.up_first_base = UF[B.u0];
    A.n_listsU = UF[B.u1] - UF[B.u0];
    A.up_node = dUN.p + B.u0;
    A.up_first = dUF.p + B.u0;
    A.up_levels = dUL.p + B.u0;
    A.list_node = dLN.p + UF[B.u0];
    A.list_level = dLL.p + UF[B.u0];
    if (A.n_up) {
      hipError_t e = launch_build(dim, b->metric, BUILD_UPPER, A.n_up, A, s);
      if (e != hipSuccess) return set_error(SHINE_ERR_HIP, std::string("build upper launch: ") + hipGetErrorString(e));
    }
    if (prof) HIP_TRY(hipEventRecord(ev[2], s));
    const uint32_t n_lists = nb + A.n_listsU;
    {
      hipError_t e = launch_build(dim, b->metric, BUILD_SELECT, n_lists, A, s);
      if (e != hipSuccess) return set_error(SHINE_ERR_HIP, std::string("build select launch: ") + hipGetErrorString(e));
    }
    if (prof) HIP_TRY(hipEventRecord(ev[3], s));
    const uint32_t n_req = n_lists * M;
    size_t tb = sort_tmp.n;
    HIP_TRY(radix_sort_u32_pairs(sort_tmp.p, &tb, req_key.p, skey.p, req_pos.p, sval.p, n_req, bits, s));
    HIP_TRY(hipMemsetAsync(ctr.p, 0, 2 * sizeof(uint32_t), s));
    HIP_TRY(launch_segments(skey.p, n_req, key_none, seg.p, ctr.p, s));
    if (prof) HIP_TRY(hipEventRecord(ev[4], s));
    A.n_req = n_req;
    {
      hipError_t e = launch_build(dim, b->metric, BUILD_PRUNE, std::min<uint32_t>(prune_grid, n_req), A, s);
      if (e != hipSuccess) return set_error(SHINE_ERR_HIP, std::string("build prune launch: ") + hipGetErrorString(e));
    }
    if (prof) {
      HIP_TRY(hipEventRecord(ev[5], s));
      HIP_TRY(hipStreamSynchronize(s));
      b->st.ms_search += phase_ms(0, 1);
      b->st.ms_upper += phase_ms(1, 2);
      b->st.ms_select += phase_ms(2, 3);
      b->st.ms_sort += phase_ms(3, 4);
      b->st.ms_prune += phase_ms(4, 5);
    } else if ((bi & 63) == 63) {
      HIP_TRY(hipStreamSynchronize(s));  // keep the host's run-ahead bounded
    }
    if (env_int("SHINE_DEBUG_SYNC", 0)) {
      hipError_t e = hipStreamSynchronize(s);
      if (e != hipSuccess)
        return set_error(SHINE_ERR_HIP, "build batch " + std::to_string(bi) + " (start " + std::to_string(B.start) +
                                            ", n " + std::to_string(nb) + "): " + hipGetErrorString(e));
    }
    n_lists_total += A.n_listsU;
    n_req_total += n_req;
    if (is_new[B.start]) {  // a new top level: this record is the entry point now (hnsw.hh:234-248)
      b->ep = static_cast<uint32_t>(B.start);
      b->ep_level = b->level[B.start];
    }
  }
  HIP_TRY(hipStreamSynchronize(s));
  if (prof)
    for (auto& e : ev) (void)hipEventDestroy(e);
  unsigned long long stv[8];
  HIP_TRY(hipMemcpy(stv, dstats.p, sizeof(stv), hipMemcpyDeviceToHost));
  b->st.rows_appended = stv[0];
  b->st.rows_pruned = stv[1];
  b->st.pools_truncated = stv[2];
  b->st.upper_beams_stopped = stv[3];
  b->st.distcomps = stv[4];
  b->st.search_failures = stv[5];
  b->st.batches = sched.size();
  b->st.upper_lists = n_lists_total;
  b->st.requests = n_req_total;
  b->st.max_level = b->ep_level;
  b->st.entry_uid = b->ep;
  h->ep = b->ep;
  h->ep_level = b->ep_level;
  h->ep_uid = b->ep;
  for (auto* d : {&dUN, &dUF, &dUL, &dLN, &dLL, &dOwner, &cand_ids, &qs, &req_key, &req_src, &req_pos, &skey, &sval, &seg, &ctr})
    d->release();
  cand_d.release();
  req_d.release();
  dstats.release();
  sort_tmp.release();
  base_own.release();
  // the search handle's per-stream scratch is sized for the build's batches: drop it (a search re-creates it)
  RP.main.release();
  if (int rc2 = RP.main.counter.grow(kCallWords)) return rc2;
  b->st.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  if (b->st.search_failures) return set_error(SHINE_ERR_OVERFLOW, std::to_string(b->st.search_failures) +
                                                                  " level-0 candidate searches failed");
  return 0;
}

}  // namespace

extern "C" {

int shine_gpu_build(const float* base, int base_on_device, uint64_t n, uint32_t dim, uint32_t M,
                    uint32_t ef_construction, int metric, uint32_t seed, int gpu_id, double batch_fraction,
                    uint32_t max_batch, shine_gpu_build_t* out) {
  if (!out || !base) return set_error(SHINE_ERR_ARG, "NULL argument");
  *out = nullptr;
  if (n < 2 || n >= 0x7FFFFFFFull) return set_error(SHINE_ERR_ARG, "n must be in [2, 2^31-1)");
  if (M < 2 || M > 32 || ef_construction == 0 || ef_construction > kFastMaxEf)
    return set_error(SHINE_ERR_ARG, "invalid build parameters (2 <= M <= 32, 0 < efC <= 512)");
  if (metric != SHINE_METRIC_L2 && metric != SHINE_METRIC_IP) return set_error(SHINE_ERR_ARG, "metric must be 0 or 1");
  if (!dim_supported(dim, SHINE_ELEM_F32)) return set_error(SHINE_ERR_ARG, "dim " + std::to_string(dim) + " has no compiled kernel");
  if (batch_fraction < 0 || batch_fraction > 1) return set_error(SHINE_ERR_ARG, "batch_fraction must be in [0, 1]");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (gpu_id < 0 || gpu_id >= ndev) return set_error(SHINE_ERR_ARG, "gpu id out of range");
  std::unique_ptr<shine_gpu_builder> b(new shine_gpu_builder);
  b->dim = dim;
  b->M = M;
  b->M0 = 2 * M;
  b->efc = ef_construction;
  b->metric = metric;
  b->seed = seed;
  b->device = gpu_id;
  b->N = n;
  HIP_TRY(hipSetDevice(gpu_id));
  try {
    if (int rc = run_build(b.get(), base, base_on_device != 0, batch_fraction > 0 ? batch_fraction : 0.02,
                           max_batch ? max_batch : (1u << 20)))
      return rc;
  } catch (const std::bad_alloc&) {
    return set_error(SHINE_ERR_NOMEM, "out of host memory while building");
  }
  *out = b.release();
  return SHINE_OK;
}

int shine_gpu_build_get_stats(shine_gpu_build_t b, shine_gpu_build_stats* out) {
  if (!b || !out) return set_error(SHINE_ERR_ARG, "NULL argument");
  *out = b->st;
  return SHINE_OK;
}

int shine_gpu_build_dumps(shine_gpu_build_t b, uint32_t n_shards) {
  if (!b) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (!b->h) return set_error(SHINE_ERR_ARG, "the built arrays moved into an index handle (shine_gpu_build_open)");
  if (n_shards == 0 || n_shards > 65535) return set_error(SHINE_ERR_ARG, "n_shards must be in [1, 65535]");
  const uint64_t N = b->N;
  const uint32_t dim = b->dim, M = b->M, M0 = b->M0;
  Replica& R = b->h->reps[0];
  HIP_TRY(hipSetDevice(R.device));
  HIP_TRY(hipStreamSynchronize(R.stream));
  try {
    std::vector<float> vec(N * dim);
    std::vector<uint32_t> adj0(N * M0), adjU(b->R * M);
    HIP_TRY(hipMemcpy(vec.data(), R.vec.p, vec.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(adj0.data(), R.adj0.p, adj0.size() * 4, hipMemcpyDeviceToHost));
    if (!adjU.empty()) HIP_TRY(hipMemcpy(adjU.data(), R.adjU.p, adjU.size() * 4, hipMemcpyDeviceToHost));
    RecordLayout L;
    L.dim = dim;
    L.M = M;
    // memory node of every record: builder.cc's draw (the reference's std::random_device, compute_thread.hh:88)
    std::mt19937 shard_rng(b->seed ^ 0x9E3779B9u);
    std::uniform_int_distribution<uint32_t> sd(0, n_shards - 1);
    std::vector<uint32_t> shard(N);
    std::vector<uint64_t> off(N), fill(n_shards, 16);
    for (uint64_t i = 0; i < N; ++i) {
      shard[i] = sd(shard_rng);
      off[i] = fill[shard[i]];
      fill[shard[i]] += L.alloc_size(b->level[i]);
    }
    auto rptr = [&](uint32_t x) { return (static_cast<uint64_t>(shard[x]) << 48) | off[x]; };
    b->dumps.assign(n_shards, {});
    for (uint32_t s = 0; s < n_shards; ++s) {
      b->dumps[s].assign(fill[s], 0);
      std::memcpy(b->dumps[s].data(), &fill[s], 8);  // free_ptr (memory_node.hh:61)
    }
    const uint64_t ep_ptr = rptr(b->ep);
    std::memcpy(b->dumps[0].data() + 8, &ep_ptr, 8);  // rdma_reads.hh:74-99
    std::vector<uint32_t> perm(dim);
    for (uint32_t i = 0; i < dim; ++i) perm[i] = permuted_index(dim, i);
    // records write disjoint byte ranges: the loop runs on the process's CPU share (16 per GPU on the pool's boxes;
    // 100M records took a minute on one thread)
    auto write_records = [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; ++i) {
        uint8_t* p = b->dumps[shard[i]].data() + off[i];
        const uint64_t hdr = i == b->ep ? kEntryNode : 0;
        const uint32_t id = static_cast<uint32_t>(i), lv = b->level[i];
        std::memcpy(p, &hdr, 8);
        std::memcpy(p + 8, &id, 4);
        std::memcpy(p + 12, &lv, 4);
        float* c = reinterpret_cast<float*>(p + 16);
        const float* row = vec.data() + i * dim;
        for (uint32_t k = 0; k < dim; ++k) std::memcpy(c + k, row + perm[k], 4);
        for (uint32_t l = 0; l <= lv; ++l) {
          uint8_t* lp = b->dumps[shard[i]].data() + L.list_offset(off[i], l);
          const uint32_t* src = l == 0 ? &adj0[i * M0] : &adjU[(static_cast<uint64_t>(b->up_base[i]) + l - 1) * M];
          const uint32_t cap = l == 0 ? M0 : M;
          uint32_t cnt = 0;
          while (cnt < cap && src[cnt] != kInvalid) {
            const uint64_t rp = rptr(src[cnt]);
            std::memcpy(lp + 4 + 8ull * cnt, &rp, 8);
            ++cnt;
          }
          std::memcpy(lp, &cnt, 4);
        }
      }
    };
    const uint64_t nt = std::max<uint64_t>(1, std::min<uint64_t>({host_threads(), 64, N / 65536 + 1}));
    std::vector<std::thread> ts;
    for (uint64_t t = 0; t < nt; ++t) ts.emplace_back(write_records, N * t / nt, N * (t + 1) / nt);
    for (auto& t : ts) t.join();
  } catch (const std::bad_alloc&) {
    b->dumps.clear();
    return set_error(SHINE_ERR_NOMEM, "out of host memory for the dump images");
  }
  return SHINE_OK;
}

uint64_t shine_gpu_build_dump_size(shine_gpu_build_t b, uint32_t s) {
  return b && s < b->dumps.size() ? b->dumps[s].size() : 0;
}
const uint8_t* shine_gpu_build_dump_data(shine_gpu_build_t b, uint32_t s) {
  return b && s < b->dumps.size() ? b->dumps[s].data() : nullptr;
}

int shine_gpu_build_write(shine_gpu_build_t b, const char* dir) {
  if (!b || !dir) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (b->dumps.empty()) return set_error(SHINE_ERR_ARG, "no dump images: call shine_gpu_build_dumps first");
  const std::string d = std::string(dir) + "/dump";
  mkdir(dir, 0755);
  mkdir(d.c_str(), 0755);
  const size_t n = b->dumps.size();
  for (size_t i = 0; i < n; ++i) {  // compute_node.cc:426-430
    const std::string p = d + "/index_m" + std::to_string(b->M) + "_efc" + std::to_string(b->efc) + "_node" +
                          std::to_string(i + 1) + "_of" + std::to_string(n) + ".dat";
    std::ofstream f(p, std::ios::binary);
    if (!f.write(reinterpret_cast<const char*>(b->dumps[i].data()), static_cast<std::streamsize>(b->dumps[i].size())))
      return set_error(SHINE_ERR_IO, "cannot write " + p);
  }
  return SHINE_OK;
}

int shine_gpu_build_open(shine_gpu_build_t b, int elem, shine_index_t* out) {
  if (!b || !out) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (!b->h) return set_error(SHINE_ERR_ARG, "the built arrays already moved into an index handle");
  if (elem != SHINE_ELEM_F32 && elem != SHINE_ELEM_F16 && elem != SHINE_ELEM_U8 && elem != SHINE_ELEM_I8)
    return set_error(SHINE_ERR_ARG, "elem must be SHINE_ELEM_F32, _F16, _U8 or _I8");
  if (!dim_supported(b->dim, elem))
    return set_error(SHINE_ERR_ARG, "dim " + std::to_string(b->dim) + " has no compiled kernel for this element type");
  shine_index* h = b->h;
  Replica& R = h->reps[0];
  HIP_TRY(hipSetDevice(R.device));
  HIP_TRY(hipStreamSynchronize(R.stream));
  if (elem != SHINE_ELEM_F32) {
    const uint64_t N = b->N;
    if (elem_is_byte(elem)) {  // byte rows only where they reproduce every component exactly
      DevBuf<uint32_t> flag;
      if (int rc = flag.grow(1)) return rc;
      HIP_TRY(hipMemsetAsync(flag.p, 0, 4, R.stream));
      HIP_TRY(launch_fits_bytes(reinterpret_cast<const float*>(R.vec.p), N * b->dim, elem, flag.p, R.stream));
      uint32_t bad = 0;
      HIP_TRY(hipMemcpy(&bad, flag.p, 4, hipMemcpyDeviceToHost));
      flag.release();
      if (bad)
        return set_error(SHINE_ERR_ARG, std::string("a record component is not exactly a ") +
                                            (elem == SHINE_ELEM_U8 ? "u8" : "i8") + " value: byte rows would change it");
    }
    DevBuf<uint8_t> nv;
    if (int rc = nv.grow(N * row_bytes(b->dim, elem))) return rc;
    HIP_TRY(hipMemsetAsync(nv.p, 0, nv.n, R.stream));
    HIP_TRY(launch_rows_to_device(reinterpret_cast<const float*>(R.vec.p), nv.p, N, b->dim, elem, true, R.stream));
    HIP_TRY(hipStreamSynchronize(R.stream));
    R.vec.release();
    R.vec.p = nv.p;
    R.vec.n = nv.n;
    nv.p = nullptr;
    nv.n = 0;
    h->elem = elem;
    h->device_bytes = h->device_bytes - N * b->dim * 4 + R.vec.n;
  }
  h->search_mode = SHINE_MODE_EXACT;  // as every opened handle
  *out = h;
  b->h = nullptr;
  return SHINE_OK;
}

int shine_gpu_build_open_ex(shine_gpu_build_t b, uint32_t n_shards, int elem, const int* gpu_ids, uint32_t n_gpus,
                            int placement, double cache_fraction, shine_index_t* out) {
  if (!b || !out) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (!b->h) return set_error(SHINE_ERR_ARG, "the built arrays already moved into an index handle");
  if (n_shards == 0 || n_shards > 65535) return set_error(SHINE_ERR_ARG, "n_shards must be in [1, 65535]");
  const uint64_t N = b->N;
  const uint32_t dim = b->dim, M = b->M, M0 = b->M0;
  Replica& R = b->h->reps[0];
  HIP_TRY(hipSetDevice(R.device));
  HIP_TRY(hipStreamSynchronize(R.stream));
  try {
    // the records as the dump parser would lay them out (graph.cc parse_dumps): memory node s's records in id order,
    // node1's first, every list entry a dense id; memory nodes drawn as shine_gpu_build_dumps draws them
    std::mt19937 shard_rng(b->seed ^ 0x9E3779B9u);
    std::uniform_int_distribution<uint32_t> sd(0, n_shards - 1);
    std::vector<uint32_t> shard(N);
    std::vector<uint64_t> start(n_shards + 1, 0);
    for (uint64_t i = 0; i < N; ++i) {
      shard[i] = sd(shard_rng);
      ++start[shard[i] + 1];
    }
    for (uint32_t s = 0; s < n_shards; ++s) start[s + 1] += start[s];
    std::vector<uint32_t> dense(N);
    {
      std::vector<uint64_t> fill(start.begin(), start.end() - 1);
      for (uint64_t i = 0; i < N; ++i) dense[i] = static_cast<uint32_t>(fill[shard[i]]++);
    }
    std::vector<float> vdev(N * dim);
    std::vector<uint32_t> adj0(N * M0), adjU(b->R * M);
    HIP_TRY(hipMemcpy(vdev.data(), R.vec.p, vdev.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(adj0.data(), R.adj0.p, adj0.size() * 4, hipMemcpyDeviceToHost));
    if (!adjU.empty()) HIP_TRY(hipMemcpy(adjU.data(), R.adjU.p, adjU.size() * 4, hipMemcpyDeviceToHost));
    HostGraph G;
    G.L.dim = dim;
    G.L.M = M;
    G.metric = b->metric;
    G.N = N;
    G.n_shards = n_shards;
    G.shard_start = start;
    G.vec.resize(N * dim);
    G.uid.resize(N);
    G.level.resize(N);
    G.up_base.resize(N);
    G.adj0.assign(N * M0, kInvalid);
    std::vector<uint32_t> perm(dim);
    for (uint32_t k = 0; k < dim; ++k) perm[k] = permuted_index(dim, k);
    for (uint64_t i = 0; i < N; ++i) {
      const uint64_t g = dense[i];
      const float* row = vdev.data() + i * dim;
      float* dst = G.vec.data() + g * dim;
      for (uint32_t k = 0; k < dim; ++k) dst[k] = row[perm[k]];
      G.uid[g] = static_cast<uint32_t>(i);
      G.level[g] = b->level[i];
      G.up_base[g] = b->up_base[i];  // the upper rows keep the build's order: rows are reached through up_base only
      for (uint32_t j = 0; j < M0; ++j) {
        const uint32_t x = adj0[i * M0 + j];
        G.adj0[g * M0 + j] = x == kInvalid ? kInvalid : dense[x];
      }
    }
    G.adjU.resize(adjU.size());
    for (size_t j = 0; j < adjU.size(); ++j) G.adjU[j] = adjU[j] == kInvalid ? kInvalid : dense[adjU[j]];
    G.ep = dense[b->ep];
    G.ep_level = b->ep_level;
    G.lists_unique = true;
    std::vector<float>().swap(vdev);
    return index_from_graph(std::move(G), elem, gpu_ids, n_gpus, placement, cache_fraction, out);
  } catch (const std::bad_alloc&) {
    return set_error(SHINE_ERR_NOMEM, "out of host memory for the host graph");
  }
}

int shine_gpu_build_free(shine_gpu_build_t b) {
  delete b;
  return SHINE_OK;
}

}  // extern "C"
