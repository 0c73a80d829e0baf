// shine_compute_node — the reference's compute-node driver rebuilt on the C ABI (include/shine_gpu.h).
//
// Mirrors ComputeNode<Distance> (src/compute_node.cc:8-188) for one process that owns the GPUs of a node:
//   flags              IndexConfiguration (src/common/configuration.hh:55-113), same names, defaults and checks
//   read_dataset       base / queries / groundtruth / warmup files under --data-path (compute_node.cc:278-319),
//                      big-ann formats with the round-robin partial read (src/io/read_data.hh:8-78)
//   build or load      --store-index / --load-index / neither (compute_node.cc:79-101, memory_node.hh:130-209):
//                      shine_build (+ shine_build_write) or the dumps under <data-path>/dump
//   warmup             with --cache: the warmup queries run first and feed the cache admission (compute_node.cc:116-131)
//   run_queries        shine_prepare (setup, untimed), then the whole query set through shine_knn_batch (chunks in
//                      flight inside the library) with the queries' ids; query_results[q_id] is filled from
//                      out_ids (compute_thread.hh:77), the wall time of the whole phase is the query time
//   recall             compute_local_recall (compute_node.cc:579-600)
//   statistics         one JSON document on stdout under the reference's names (statistics.hh:122-130,
//                      compute_node.cc:549-556, 478-497): build / queries / cache / meta / hnsw_parameters / timings
// Transport flags of the RDMA deployment (--servers, --port, ...) have no meaning here; GPU placement flags are
// added (--gpus, --placement, --search-mode, --rows, --batch, --memory-nodes).  Errors print "[ERROR]: ..." and exit 1,
// as lib_assert / exit_with_help_message do (utils.hh:17-23, configuration.hh:88-113).
#include <algorithm>
#include <chrono>
#include <deque>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/shine_gpu.h"

namespace fs = std::filesystem;

namespace {

[[noreturn]] void fail(const std::string& msg) {
  std::cerr << "[ERROR]: " << msg << std::endl;
  std::exit(EXIT_FAILURE);
}

void check(int rc, const char* what) {
  if (rc != SHINE_OK) fail(std::string(what) + " failed (status " + std::to_string(rc) + "): " + shine_last_error());
}

void status(const std::string& msg) { std::cerr << "[STATUS]: " << msg << std::endl; }  // utils.cc:48-49

// ---- flags (configuration.hh:55-86) ------------------------------------------------------------------------
struct Config {
  std::string data_path, query_suffix, label;
  uint32_t num_threads = 0, num_coroutines = 4;
  int32_t seed = 1234;
  bool disable_thread_pinning = false;
  uint32_t ef_search = 0, ef_construction = 200, k = 0, m = 32;
  bool store_index = false, load_index = false, no_recall = false, ip_distance = false;
  uint32_t cache_size_ratio = 5;
  bool use_cache = false, routing = false;
  // compute-node split (read_data.hh:42-77): this process reads ids ≡ client_id (mod num_clients)
  uint32_t num_clients = 1, client_id = 0;
  // GPU placement (include/shine_gpu.h)
  std::vector<int> gpus{0};
  std::string placement = "replica", search_mode = "exact", rows = "f32", builder = "cpu";
  uint32_t batch = 0, memory_nodes = 1, calls_in_flight = 1;
};

const char* kHelp =
    "shine_compute_node — SHINE compute-node query path on MI355X (C ABI include/shine_gpu.h)\n"
    "  -d, --data-path DIR        base.{fbin,u8bin,i8bin} and queries/{query,groundtruth,warmup}-<suffix>.*\n"
    "  -q, --query-suffix S       query file suffix\n"
    "  -t, --threads N            host threads (index construction)\n"
    "  -C, --coroutines N         accepted for compatibility (default 4); batches replace coroutines\n"
    "  -p, --disable-thread-pinning\n"
    "      --seed N               PRNG seed (default 1234; -1 = random)\n"
    "      --label S              benchmark label\n"
    "  -s, --store-index          build the index and store the memory-node dumps under <data-path>/dump\n"
    "  -l, --load-index           load the memory-node dumps from <data-path>/dump\n"
    "      --cache                keep local copies of other GPUs' hot records (sharded placements)\n"
    "      --routing              route queries to the GPU owning their region (needs --cache)\n"
    "      --cache-ratio N        cache size in % of the index (default 5)\n"
    "      --no-recall            skip recall (no ground-truth file needed)\n"
    "      --ip-dist              inner-product distance instead of squared L2\n"
    "      --ef-search N          beam width during search\n"
    "      --ef-construction N    beam width during construction (default 200)\n"
    "  -k, --k N                  number of nearest neighbours\n"
    "  -m, --m N                  bidirectional connections (default 32)\n"
    "      --num-clients N / --client-id I   read queries with id % N == I (default 1 / 0)\n"
    "      --gpus LIST            GPU ids, comma separated (default 0)\n"
    "      --placement P          replica | sharded (default replica)\n"
    "      --memory-nodes N       memory-node dumps to build / load (default 1)\n"
    "      --search-mode M        exact (reference heap order) | fast (default exact)\n"
    "      --rows R               record storage in HBM: f32 | auto (u8 / i8 rows where every component is a byte\n"
    "                             value, bitwise the same results) (default f32)\n"
    "      --batch N              queries per shine_knn_batch call (default 0: the whole query set in one call, which\n"
    "                             the library runs as 1,024-query chunks kept in flight on four streams per GPU)\n"
    "      --calls-in-flight N    host calls kept in flight (shine_knn_batch_async / shine_wait; default 1: one\n"
    "                             synchronous call at a time; with N > 1 and --batch 0 the set goes out in 2N calls)\n"
    "      --builder B            cpu (parallel restatement of HNSW::insert) | gpu (shine_gpu_build, the batch\n"
    "                             builder on the first --gpus device) (default cpu)\n";

[[noreturn]] void exit_with_help(const std::string& msg) {
  std::cerr << "[ERROR]: " << msg << std::endl << kHelp;
  std::exit(EXIT_FAILURE);
}

uint64_t parse_uint(const std::string& flag, const std::string& v) {
  char* end = nullptr;
  errno = 0;
  const unsigned long long x = std::strtoull(v.c_str(), &end, 10);
  if (v.empty() || *end != '\0' || errno) exit_with_help("invalid value '" + v + "' for " + flag);
  return x;
}

Config parse(int argc, char** argv) {
  Config c;
  std::map<std::string, std::string> alias = {{"-d", "--data-path"}, {"-t", "--threads"},   {"-C", "--coroutines"},
                                              {"-p", "--disable-thread-pinning"},         {"-q", "--query-suffix"},
                                              {"-s", "--store-index"}, {"-l", "--load-index"}, {"-k", "--k"},
                                              {"-m", "--m"}};
  const std::vector<std::string> switches = {"--disable-thread-pinning", "--store-index", "--load-index", "--cache",
                                             "--routing", "--no-recall", "--ip-dist"};
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i], v;
    if (a == "-h" || a == "--help") {
      std::cout << kHelp;
      std::exit(EXIT_SUCCESS);
    }
    if (auto eq = a.find('='); a.rfind("--", 0) == 0 && eq != std::string::npos) {
      v = a.substr(eq + 1);
      a = a.substr(0, eq);
    }
    if (alias.count(a)) a = alias[a];
    const bool is_switch = std::find(switches.begin(), switches.end(), a) != switches.end();
    if (!is_switch && v.empty()) {
      if (i + 1 >= argc) exit_with_help("missing value for " + a);
      v = argv[++i];
    }
    if (a == "--data-path") c.data_path = v;
    else if (a == "--query-suffix") c.query_suffix = v;
    else if (a == "--label") c.label = v;
    else if (a == "--threads") c.num_threads = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--coroutines") c.num_coroutines = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--seed") c.seed = static_cast<int32_t>(std::stol(v));
    else if (a == "--ef-search") c.ef_search = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--ef-construction") c.ef_construction = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--k") c.k = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--m") c.m = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--cache-ratio") c.cache_size_ratio = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--num-clients") c.num_clients = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--client-id") c.client_id = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--batch") c.batch = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--calls-in-flight") c.calls_in_flight = std::max<uint32_t>(1, static_cast<uint32_t>(parse_uint(a, v)));
    else if (a == "--memory-nodes") c.memory_nodes = static_cast<uint32_t>(parse_uint(a, v));
    else if (a == "--placement") c.placement = v;
    else if (a == "--search-mode") c.search_mode = v;
    else if (a == "--rows") c.rows = v;
    else if (a == "--builder") c.builder = v;
    else if (a == "--gpus") {
      c.gpus.clear();
      std::stringstream ss(v);
      std::string tok;
      while (std::getline(ss, tok, ',')) c.gpus.push_back(static_cast<int>(parse_uint(a, tok)));
      if (c.gpus.empty()) exit_with_help("--gpus needs at least one id");
    } else if (a == "--disable-thread-pinning") c.disable_thread_pinning = true;
    else if (a == "--store-index") c.store_index = true;
    else if (a == "--load-index") c.load_index = true;
    else if (a == "--cache") c.use_cache = true;
    else if (a == "--routing") c.routing = true;
    else if (a == "--no-recall") c.no_recall = true;
    else if (a == "--ip-dist") c.ip_distance = true;
    else exit_with_help("unknown option " + a);
  }
  // validate_compute_node_options (configuration.hh:88-113)
  if (c.data_path.empty() || c.query_suffix.empty()) exit_with_help("Data path and query suffix cannot be empty");
  if (c.num_threads == 0 || c.ef_search == 0 || c.k == 0)
    exit_with_help("Parameters threads, ef-search, and k are required");
  if (c.store_index && c.load_index) exit_with_help("--store-index and --load-index cannot be used in conjunction");
  if (c.use_cache && c.cache_size_ratio == 0) exit_with_help("If --cache is set, --cache-ratio must be > 0");
  if (c.routing && !c.use_cache) exit_with_help("--routing can only be used in conjunction with --cache");
  // hnsw.hh:36
  if (c.ef_search < c.k) exit_with_help("ef_search must be >= k");
  if (c.num_clients == 0 || c.client_id >= c.num_clients) exit_with_help("--client-id must be < --num-clients");
  if (c.placement != "replica" && c.placement != "sharded") exit_with_help("--placement must be replica or sharded");
  if (c.search_mode != "exact" && c.search_mode != "fast") exit_with_help("--search-mode must be exact or fast");
  if (c.rows != "f32" && c.rows != "auto") exit_with_help("--rows must be f32 or auto");
  if (c.memory_nodes == 0) exit_with_help("--memory-nodes must be > 0");
  if (c.builder != "cpu" && c.builder != "gpu") exit_with_help("--builder must be cpu or gpu");
  return c;
}

// ---- big-ann files (read_data.hh:8-78, deserializer.hh:11-63) ------------------------------------------------
struct Database {  // io::Database (database.hh:8-51): [components | id] per slot, here two arrays
  uint32_t num_vectors_total = 0, dim = 0;
  std::vector<uint32_t> ids;
  std::vector<float> comps;
  std::vector<uint32_t> raw;  // .bin payload (ground truth), read whole
  uint32_t num_read() const { return static_cast<uint32_t>(ids.size()); }
};

void read_data(Database& db, const fs::path& file, uint32_t client_id, uint32_t num_clients, bool meta_only) {
  std::ifstream f(file, std::ios::binary);
  if (!f.good()) fail("file \"" + file.string() + "\" does not exist");  // deserializer.hh:15
  const std::string ext = file.extension().string();
  uint32_t csize = 0;
  if (ext == ".fbin" || ext == ".bin") csize = 4;
  else if (ext == ".u8bin" || ext == ".i8bin") csize = 1;
  else fail("unsupported file extension: " + ext);  // read_data.hh:31-33
  uint32_t hdr[2];
  if (!f.read(reinterpret_cast<char*>(hdr), 8)) fail("cannot read file " + file.string());
  db.num_vectors_total = hdr[0];
  db.dim = hdr[1];
  if (meta_only) return;
  if (ext == ".bin") {  // ground truth: read entirely (compute_node.cc:315-318)
    db.raw.resize(static_cast<size_t>(hdr[0]) * hdr[1]);
    if (!f.read(reinterpret_cast<char*>(db.raw.data()), static_cast<std::streamsize>(db.raw.size() * 4)))
      fail("cannot read file " + file.string());
    return;
  }
  // to_read = n / num_clients, +1 for client ids below the remainder (read_data.hh:42-49)
  uint32_t to_read = db.num_vectors_total / num_clients;
  if (client_id < db.num_vectors_total - to_read * num_clients) ++to_read;
  db.ids.reserve(to_read);
  db.comps.reserve(static_cast<size_t>(to_read) * db.dim);
  std::vector<char> row(static_cast<size_t>(db.dim) * csize);
  for (uint32_t id = 0; id < db.num_vectors_total; ++id) {
    if (id % num_clients != client_id) {
      f.seekg(static_cast<std::streamoff>(row.size()), std::ios::cur);  // Deserializer::jump
      continue;
    }
    if (!f.read(row.data(), static_cast<std::streamsize>(row.size()))) fail("cannot read file " + file.string());
    db.ids.push_back(id);
    for (uint32_t j = 0; j < db.dim; ++j) {  // deserializer.hh:24-44: bytes converted element-wise to f32
      float x;
      if (ext == ".fbin") std::memcpy(&x, row.data() + 4ull * j, 4);
      else if (ext == ".u8bin") x = static_cast<float>(static_cast<uint8_t>(row[j]));
      else x = static_cast<float>(static_cast<int8_t>(row[j]));
      db.comps.push_back(x);
    }
  }
}

fs::path find_stem(const fs::path& dir, const std::string& stem) {
  if (!fs::is_directory(dir)) return {};
  for (const auto& e : fs::directory_iterator(dir))
    if (e.path().stem() == stem) return e.path();
  return {};
}

// ---- timing (timing.hh:10-44) and a minimal JSON writer ----------------------------------------------------
struct Interval {
  std::string name;
  double ms = 0;
  std::chrono::steady_clock::time_point t0;
  void start() { t0 = std::chrono::steady_clock::now(); }
  void stop() { ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
};

struct Json {  // ordered object of already-encoded values
  std::vector<std::pair<std::string, std::string>> kv;
  template <class T>
  void num(const std::string& k, T v) {
    std::ostringstream o;
    o.precision(17);
    o << v;
    kv.emplace_back(k, o.str());
  }
  void str(const std::string& k, const std::string& v) {
    std::string e = "\"";
    for (char c : v) {
      if (c == '"' || c == '\\') e += '\\';
      e += c;
    }
    kv.emplace_back(k, e + "\"");
  }
  void obj(const std::string& k, const Json& j) { kv.emplace_back(k, j.dump(1)); }
  std::string dump(int depth = 0) const {
    const std::string pad(2 * (depth + 1), ' '), end(2 * depth, ' ');
    std::string s = "{\n";
    for (size_t i = 0; i < kv.size(); ++i)
      s += pad + "\"" + kv[i].first + "\": " + kv[i].second + (i + 1 < kv.size() ? ",\n" : "\n");
    return s + end + "}";
  }
};

// ---- the compute node ----------------------------------------------------------------------------------------
struct ComputeThread {  // compute_thread.hh:17-91: results and counters of the query phase
  // query_results[q_id] (:77) as one array the calls write into directly: row i holds the results of the query read
  // i-th, whose id is the database's ids[i] (allocated before the query timer, so the phase times no per-query
  // allocation — 10,000 map nodes and vectors took ~0.4 ms of a 2.3 ms phase)
  std::vector<uint32_t> results;
  shine_stats stats{};  // :82 (aggregated over batches)
};

void add(shine_stats& a, const shine_stats& b) {
  a.processed += b.processed;
  a.distcomps += b.distcomps;
  a.visited_nodes += b.visited_nodes;
  a.visited_nodes_l0 += b.visited_nodes_l0;
  a.visited_neighborlists += b.visited_neighborlists;
  a.visited_neighborlists_l0 += b.visited_neighborlists_l0;
  a.rdma_reads_in_bytes += b.rdma_reads_in_bytes;
  a.algorithmic_bytes += b.algorithmic_bytes;
  a.overflow_retries += b.overflow_retries;
  a.remote_reads_in_bytes += b.remote_reads_in_bytes;
  a.cache_hits += b.cache_hits;
  a.cache_misses += b.cache_misses;
  a.node_reads += b.node_reads;
  a.node_cache_hits += b.node_cache_hits;
  a.kernel_ms += b.kernel_ms;
}

std::string dump_path(const Config& c, uint32_t i) {  // compute_node.cc:428-430
  return (fs::path(c.data_path) / "dump" /
          ("index_m" + std::to_string(c.m) + "_efc" + std::to_string(c.ef_construction) + "_node" +
           std::to_string(i + 1) + "_of" + std::to_string(c.memory_nodes) + ".dat"))
      .string();
}

int run(const Config& c) {
  std::vector<Interval> timing;
  auto interval = [&](const std::string& name) -> Interval& {
    timing.push_back(Interval{name, 0.0, {}});
    return timing.back();
  };
  timing.reserve(8);  // references into it stay valid: at most 3 intervals are created
  Interval& t_build = interval("build_c" + std::to_string(c.client_id));
  Interval& t_query = interval("query_c" + std::to_string(c.client_id));

  // read_dataset (compute_node.cc:278-319)
  const fs::path data(c.data_path), qdir = fs::path(c.data_path) / "queries";
  const fs::path base_file = find_stem(data, "base"), query_file = find_stem(qdir, "query-" + c.query_suffix);
  const fs::path gt_file = find_stem(qdir, "groundtruth-" + c.query_suffix);
  const fs::path warm_file = find_stem(qdir, "warmup-" + c.query_suffix);
  if (base_file.empty() || query_file.empty()) fail("base or query file missing");
  Database base, queries, gt, warmup;
  read_data(base, base_file, 0, 1, c.load_index);  // the builder inserts every vector (one process)
  read_data(queries, query_file, c.client_id, c.num_clients, false);
  if (c.use_cache) {
    if (warm_file.empty()) fail("warmup file missing");
    read_data(warmup, warm_file, c.client_id, c.num_clients, false);
  }
  const bool compute_recall = !c.no_recall;
  if (compute_recall) {
    if (gt_file.empty()) fail("ground truth file missing");
    read_data(gt, gt_file, 0, 1, false);
    if (gt.dim < c.k) fail("ground truth holds fewer than k neighbours per query");
  }
  if (queries.dim != base.dim) fail("query and base dimensions differ");
  const uint32_t dim = base.dim;
  const int metric = c.ip_distance ? SHINE_METRIC_IP : SHINE_METRIC_L2;

  // build (+ store) or load (compute_node.cc:79-101; memory_node.hh:130-209)
  Json build_stats;
  std::vector<std::vector<uint8_t>> files;
  std::vector<const uint8_t*> ptrs;
  std::vector<uint64_t> sizes;
  shine_build_t b = nullptr;
  shine_gpu_build_t gb = nullptr;  // --builder gpu
  t_build.start();
  if (c.load_index) {
    status("load index from " + (fs::path(c.data_path) / "dump").string());
    for (uint32_t i = 0; i < c.memory_nodes; ++i) {
      std::ifstream f(dump_path(c, i), std::ios::binary | std::ios::ate);
      if (!f.good()) fail("file \"" + dump_path(c, i) + "\" does not exist");  // memory_node.hh:161-164
      files.emplace_back(static_cast<size_t>(f.tellg()));
      f.seekg(0);
      if (!f.read(reinterpret_cast<char*>(files.back().data()), static_cast<std::streamsize>(files.back().size())))
        fail("cannot read " + dump_path(c, i));
    }
    for (auto& f : files) {
      ptrs.push_back(f.data());
      sizes.push_back(f.size());
    }
    build_stats.num("dist_comps", 0);
  } else if (c.builder == "gpu") {
    // the GPU batch builder (shine_gpu_build): the same insert and select_heuristic, batches of records inserted
    // together on the first GPU; 100M records in about a minute instead of an hour
    status("**INSERT**: building the index on GPU " + std::to_string(c.gpus[0]));
    const uint32_t seed = c.seed == -1 ? static_cast<uint32_t>(std::random_device{}()) : static_cast<uint32_t>(c.seed);
    check(shine_gpu_build(base.comps.data(), 0, base.num_read(), dim, c.m, c.ef_construction, metric, seed, c.gpus[0],
                          0.0, 0, &gb),
          "shine_gpu_build");
    shine_gpu_build_stats gst{};
    check(shine_gpu_build_get_stats(gb, &gst), "shine_gpu_build_get_stats");
    if (c.store_index) {  // memory_node.hh:185-201: the dumps the reference's memory nodes would store
      check(shine_gpu_build_dumps(gb, c.memory_nodes), "shine_gpu_build_dumps");
      check(shine_gpu_build_write(gb, c.data_path.c_str()), "shine_gpu_build_write");
      for (uint32_t i = 0; i < c.memory_nodes; ++i) sizes.push_back(shine_gpu_build_dump_size(gb, i));
    }
    build_stats.num("dist_comps", gst.distcomps);
  } else {
    status("**INSERT**: building the index on " + std::to_string(c.num_threads) + " threads");
    const uint32_t seed = c.seed == -1 ? static_cast<uint32_t>(std::random_device{}()) : static_cast<uint32_t>(c.seed);
    check(shine_build(base.comps.data(), base.num_read(), dim, c.m, c.ef_construction, metric, c.memory_nodes, seed,
                      c.num_threads, &b),
          "shine_build");
    if (c.store_index) check(shine_build_write(b, c.data_path.c_str(), c.m, c.ef_construction), "shine_build_write");
    for (uint32_t i = 0; i < c.memory_nodes; ++i) {
      ptrs.push_back(shine_build_dump_data(b, i));
      sizes.push_back(shine_build_dump_size(b, i));
    }
    build_stats.num("dist_comps", shine_build_distcomps(b));
  }
  t_build.stop();
  uint64_t index_size = 0;
  for (uint64_t s : sizes) index_size += s;

  const int placement = c.placement == "replica" ? SHINE_PLACE_REPLICA
                        : c.routing               ? SHINE_PLACE_SHARDED_REGIONS
                                                  : SHINE_PLACE_SHARDED;
  const double cache_fraction = c.use_cache && placement != SHINE_PLACE_REPLICA ? c.cache_size_ratio / 100.0 : 0.0;
  const int elem = c.rows == "auto" ? SHINE_ELEM_AUTO : SHINE_ELEM_F32;
  shine_index_t h = nullptr;
  if (gb) {  // the built graph laid out directly, as its dumps would be (no dump written or parsed)
    if (placement == SHINE_PLACE_REPLICA && c.gpus.size() == 1 && elem == SHINE_ELEM_F32)
      check(shine_gpu_build_open(gb, elem, &h), "shine_gpu_build_open");  // the device arrays move into the handle
    else
      check(shine_gpu_build_open_ex(gb, c.memory_nodes, elem, c.gpus.data(), static_cast<uint32_t>(c.gpus.size()),
                                    placement, std::min(1.0, cache_fraction), &h),
            "shine_gpu_build_open_ex");
  } else {
    check(shine_open_buffers_ex(ptrs.data(), sizes.data(), c.memory_nodes, dim, c.m, metric, elem, c.gpus.data(),
                                static_cast<uint32_t>(c.gpus.size()), placement, std::min(1.0, cache_fraction), &h),
          "shine_open");
  }
  if (b) shine_build_free(b);
  if (gb) shine_gpu_build_free(gb);
  files.clear();
  check(shine_set_search_mode(h, c.search_mode == "fast" ? SHINE_MODE_FAST : SHINE_MODE_EXACT), "search mode");
  shine_index_info info{};
  check(shine_index_get_info(h, &info), "index info");
  build_stats.num("rdma_reads_in_bytes", 0);
  build_stats.num("rdma_writes_in_bytes", index_size);
  build_stats.num("remote_allocations", info.num_nodes);
  build_stats.num("index_size", index_size);
  build_stats.num("max_level", info.max_level);

  // queries per call: --batch, or the whole set in one call, or with calls in flight the set in 2N calls
  auto per_call_of = [&](uint32_t n_total) -> uint32_t {
    if (c.batch) return c.batch;
    if (c.calls_in_flight > 1) return std::max<uint32_t>(1, (n_total + 2 * c.calls_in_flight - 1) / (2 * c.calls_in_flight));
    return std::max<uint32_t>(1, n_total);
  };
  auto run_batches = [&](const Database& db, ComputeThread& th) {  // th.results sized by the caller
    const uint32_t per_call = per_call_of(db.num_read());
    if (c.calls_in_flight <= 1) {
      for (uint32_t s = 0; s < db.num_read(); s += per_call) {
        const uint32_t n = std::min(per_call, db.num_read() - s);
        shine_stats st{};
        check(shine_knn_batch(h, db.comps.data() + static_cast<size_t>(s) * db.dim, db.ids.data() + s, n, c.k,
                              c.ef_search, th.results.data() + static_cast<size_t>(s) * c.k, nullptr, &st),
              "shine_knn_batch");
        add(th.stats, st);
      }
      return;
    }
    // T threads x C coroutines keep queries in flight in the reference (worker_pool.hh:78-89, scheduler.hh:42-96):
    // here N host calls, the next enqueued before the oldest is waited for, so the GPU never drains between calls
    std::deque<shine_request_t> inflight;
    auto wait_oldest = [&]() {
      shine_stats st{};
      check(shine_wait(inflight.front(), &st), "shine_wait");
      inflight.pop_front();
      add(th.stats, st);
    };
    for (uint32_t s = 0; s < db.num_read(); s += per_call) {
      const uint32_t n = std::min(per_call, db.num_read() - s);
      shine_request_t req = nullptr;
      check(shine_knn_batch_async(h, db.comps.data() + static_cast<size_t>(s) * db.dim, db.ids.data() + s, n, c.k,
                                  c.ef_search, th.results.data() + static_cast<size_t>(s) * c.k, nullptr, nullptr, &req),
            "shine_knn_batch_async");
      inflight.push_back(req);
      if (inflight.size() >= c.calls_in_flight) wait_oldest();
    }
    while (!inflight.empty()) wait_oldest();
  };

  if (c.use_cache) {  // cache warmup (compute_node.cc:116-131): the warmup split runs first, then the cache is reset
    status("cache warmup");
    Interval& t_warm = interval("warmup_routing");
    t_warm.start();
    // the warmup split's record reads rank what every GPU caches (shine_cache_warmup; a no-op without a cache)
    check(shine_cache_warmup(h, warmup.comps.data(), warmup.ids.data(), warmup.num_read(), c.k, c.ef_search),
          "shine_cache_warmup");
    t_warm.stop();
  }

  // the compute threads' setup, outside the query timer (compute_node.cc:354-380): streams, scratch and staging for
  // the query phase's calls and the kernels' code, by a call over all-zero queries
  check(shine_prepare(h, std::max<uint32_t>(1, std::min(per_call_of(queries.num_read()), queries.num_read())),
                      c.k, c.ef_search),
        "shine_prepare");
  status("run queries");
  ComputeThread th;
  th.results.assign(static_cast<size_t>(queries.num_read()) * c.k, 0u);
  t_query.start();
  run_batches(queries, th);
  t_query.stop();
  status("processed queries: " + std::to_string(th.stats.processed));

  // compute_local_recall (compute_node.cc:579-600): set semantics against groundtruth[q_id][0:k]
  double recall = 0;
  if (compute_recall) {
    uint64_t true_results = 0;
    for (uint32_t i = 0; i < queries.num_read(); ++i) {
      const uint32_t q_id = queries.ids[i];
      if (q_id >= gt.num_vectors_total) fail("query id beyond the ground truth");
      const uint32_t* pos = gt.raw.data() + static_cast<size_t>(q_id) * gt.dim;
      for (uint32_t r = 0; r < c.k; ++r) {
        const uint32_t hit = th.results[static_cast<size_t>(i) * c.k + r];
        for (uint32_t j = 0; j < c.k; ++j)
          if (hit == pos[j]) {
            ++true_results;
            break;
          }
      }
    }
    recall = static_cast<double>(true_results) / static_cast<double>(th.stats.processed) / c.k;
    status("local recall: " + std::to_string(recall));
  }
  check(shine_close(h), "shine_close");

  // statistics (CNStatistics::convert, statistics.hh:122-143; compute_node.cc:549-556, 174-183)
  const double query_s = t_query.ms / 1000.0;
  Json qj;
  qj.num("dist_comps", th.stats.distcomps);
  qj.num("rdma_reads_in_bytes", th.stats.rdma_reads_in_bytes);
  qj.num("rdma_writes_in_bytes", 0);
  qj.num("recall", recall);
  qj.num("visited_nodes", th.stats.visited_nodes);
  qj.num("visited_nodes_l0", th.stats.visited_nodes_l0);
  qj.num("visited_neighborlists", th.stats.visited_neighborlists);
  qj.num("processed", th.stats.processed);
  qj.num("queries_per_sec", static_cast<uint64_t>(query_s > 0 ? th.stats.processed / query_s : 0));
  qj.str("compute_recall", compute_recall ? "true" : "false");
  Json cj;
  // statistics.hh:171-173: hits over every record lookup (a compute node reads every record remotely); the reads of
  // records another GPU holds are reported separately (off_stripe_*)
  const uint64_t reads = th.stats.node_reads, hits = th.stats.node_cache_hits;
  cj.num("hits_total", hits);
  cj.num("misses_total", reads - std::min(reads, hits));
  cj.num("hit_rate", reads ? static_cast<double>(hits) / static_cast<double>(reads) : 0.0);
  cj.num("off_stripe_hits_total", th.stats.cache_hits);
  cj.num("off_stripe_misses_total", th.stats.cache_misses);
  const uint64_t lookups = th.stats.cache_hits + th.stats.cache_misses;
  cj.num("off_stripe_hit_rate", lookups ? static_cast<double>(th.stats.cache_hits) / static_cast<double>(lookups) : 0.0);
  if (c.use_cache) cj.num("cache_size_ratio", c.cache_size_ratio);
  Json gj;  // not in the reference: the GPU side of the same run
  gj.num("device_bytes_per_gpu", info.device_bytes);
  gj.num("n_gpus", info.n_gpus);
  gj.str("placement", c.placement + (c.routing ? "+routing" : ""));
  gj.num("cache_fraction", info.cache_fraction);
  gj.str("search_mode", c.search_mode);
  gj.str("rows", info.elem == SHINE_ELEM_U8 ? "u8" : info.elem == SHINE_ELEM_I8 ? "i8" : "f32");
  gj.num("kernel_ms", th.stats.kernel_ms);
  gj.num("algorithmic_bytes", th.stats.algorithmic_bytes);
  gj.num("remote_reads_in_bytes", th.stats.remote_reads_in_bytes);
  gj.num("overflow_retries", th.stats.overflow_retries);
  Json meta;  // add_meta_statistics (compute_node.cc:478-497)
  meta.num("compute_nodes", c.num_clients);
  meta.num("memory_nodes", c.memory_nodes);
  meta.num("compute_threads", c.num_clients * c.num_threads);
  meta.num("coroutines_per_thread", c.num_coroutines);
  meta.str("threads_pinned", c.disable_thread_pinning ? "false" : "true");
  const fs::path pn = data.has_stem() ? data.stem() : data.parent_path().stem();
  meta.str("dataset", pn.string());
  meta.str("query_suffix", c.query_suffix);
  meta.str("zipf_parameter", c.query_suffix.size() > 1 ? c.query_suffix.substr(1, c.query_suffix.find_first_of('-') - 1)
                                                         : std::string());
  meta.num("timestamp", static_cast<uint64_t>(std::time(nullptr)));
  meta.str("label", c.label);
  Json hp;
  hp.num("k", c.k);
  hp.num("m", c.m);
  hp.num("ef_search", c.ef_search);
  hp.num("ef_construction", c.ef_construction);
  Json tj;
  for (const auto& t : timing) tj.num(t.name, t.ms);
  Json out;
  out.obj("build", build_stats);
  out.obj("queries", qj);
  out.obj("cache", cj);
  out.obj("gpu", gj);
  out.obj("meta", meta);
  out.obj("hnsw_parameters", hp);
  out.num("num_vectors", base.num_vectors_total);
  out.num("num_queries", queries.num_vectors_total);
  out.num("estimated_total_index_size", index_size);
  out.obj("timings", tj);
  std::cerr << std::endl << "statistics:" << std::endl;
  std::cout << out.dump() << std::endl;
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const Config c = parse(argc, argv);
  std::cerr << "data path: " << c.data_path << "\nquery suffix: " << c.query_suffix << "\nnumber of threads: "
            << c.num_threads << "\nK: " << c.k << "\nM: " << c.m << "\nef search: " << c.ef_search
            << "\nef construction: " << c.ef_construction << std::endl;
  return run(c);
}
