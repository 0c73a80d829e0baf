// gfx950 (CDNA4) kernels of the SHINE compute-node query path.
//
//   search_kernel   HNSW::knn (src/hnsw/hnsw.hh:253-307): greedy descent search_for_one (:331-393) and the
//                   level-0 best-first beam search search_level (:406-476), one query per wavefront,
//                   persistent workgroups pulling queries from a device work queue.
//   distance_kernel Distance::dist (src/hnsw/distance.hh:153-161) over gathered (query, node) pairs.
//
// Exactness.  Both kernels evaluate L2 / IP in exactly the oracle's floating-point order (oracle/oracle.cc):
// eight lanes of a wavefront play the eight AVX2 accumulators of L2SqrSIMD16ExtAVX / InnerProductSIMD16ExtAVX
// (distance.hh:11-76) — lane a owns elements i ≡ a (mod 8) of the 16-aligned prefix and runs the same fmaf
// chain — the eight partial sums are added left to right, then the scalar tail.  The two candidate queues are
// the reference's std::vector heaps (heap.hh) held in LDS and updated by lane 0 with the exact libstdc++
// push_heap / pop_heap algorithms (bits/stl_heap.h: __push_heap, __adjust_heap, __pop_heap), so ties between
// equal distances are broken exactly as on the CPU and the returned ids come out in the same heap-array
// order (hnsw.hh:300-303).
//
// Per expansion the wavefront: pops the closest candidate (lane 0), loads the 2M-entry adjacency row with
// one coalesced 128-/256-byte load (one u32 per lane), test-and-sets the visited bitmap with one atomicOr per
// lane (ballot + mbcnt give the fresh neighbours in list order), gathers the fresh neighbours' vectors
// (8 vectors per wave-instruction, 8 lanes × 32 B each), reduces, and lane 0 replays the reference's
// accept / push / push_k sequence over them in list order.
#include "kernels.h"

#include <hip/hip_fp16.h>

namespace shine {
namespace {

using u32 = uint32_t;
using u64 = uint64_t;
constexpr u32 INV = 0xFFFFFFFFu;
constexpr u32 ST_OVERFLOW = 6;  // SHINE_ERR_OVERFLOW
constexpr u32 ST_FORMAT = 3;    // SHINE_ERR_FORMAT

__device__ __forceinline__ float key(u64 e) { return __uint_as_float(static_cast<u32>(e)); }
__device__ __forceinline__ u32 eid(u64 e) { return static_cast<u32>(e >> 32); }
__device__ __forceinline__ u64 mk(float d, u32 id) { return (static_cast<u64>(id) << 32) | __float_as_uint(d); }

__device__ __forceinline__ u32 bcast(u32 v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float bcastf(float v) { return __uint_as_float(bcast(__float_as_uint(v))); }
__device__ __forceinline__ u64 bcast64(u64 v) {
  return (static_cast<u64>(bcast(static_cast<u32>(v >> 32))) << 32) | bcast(static_cast<u32>(v));
}
// Cross-lane LDS hand-off inside one wavefront: DS instructions of a wave execute in order, so only compiler
// code motion has to be stopped.
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__half x) { return __half2float(x); }

// ------------------------------------------------------------------------------------------------------------
// libstdc++ heap algorithms on an LDS array of packed {dist, id} entries (executed by lane 0 only).
//   MAXH = true : heap::MaxHeapCompare (lhs.distance < rhs.distance), heap.hh:15-17
//   MAXH = false: heap::MinHeapCompare (lhs.distance > rhs.distance), heap.hh:19-21
// ------------------------------------------------------------------------------------------------------------
template <bool MAXH>
__device__ __forceinline__ bool hcmp(float a, float b) {
  return MAXH ? (a < b) : (a > b);
}

// std::push_heap(first, first + n + 1) with h[n] = v   (std::__push_heap(first, n, 0, v))
template <bool MAXH>
__device__ __forceinline__ void heap_push(u64* h, int n, u64 v) {
  const float vd = key(v);
  int hole = n;
  while (hole > 0) {
    const int parent = (hole - 1) >> 1;
    const u64 pe = h[parent];
    if (!hcmp<MAXH>(key(pe), vd)) break;
    h[hole] = pe;
    hole = parent;
  }
  h[hole] = v;
}

// std::pop_heap(first, first + n) followed by pop_back  (std::__pop_heap → std::__adjust_heap(first, 0, n-1, v))
template <bool MAXH>
__device__ __forceinline__ void heap_pop(u64* h, int n) {
  if (n <= 1) return;
  const int len = n - 1;
  const u64 value = h[len];
  int hole = 0, second = 0;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (hcmp<MAXH>(key(h[second]), key(h[second - 1]))) second--;
    h[hole] = h[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    h[hole] = h[second - 1];
    hole = second - 1;
  }
  const float vd = key(value);
  while (hole > 0) {
    const int parent = (hole - 1) >> 1;
    const u64 pe = h[parent];
    if (!hcmp<MAXH>(key(pe), vd)) break;
    h[hole] = pe;
    hole = parent;
  }
  h[hole] = value;
}

// ------------------------------------------------------------------------------------------------------------
// Distance evaluation in the oracle's FP order.  Lane l: group g = l >> 3 evaluates one vector, a = l & 7 is
// the AVX2 accumulator it plays.  Up to NPB passes of 8 vectors have their loads in flight together.
// ------------------------------------------------------------------------------------------------------------
template <int D>
struct Geo {
  static constexpr int DB = D >> 4 << 4;  // elements handled by the SIMD16 kernel (qty16 << 4)
  static constexpr int PER = DB / 8;      // elements per accumulator lane
  static constexpr int TAIL = D - DB;     // scalar tail (distance.hh:112-115, 136-139)
  static constexpr int PERA = PER > 0 ? PER : 1;
  static constexpr int TAILA = TAIL > 0 ? TAIL : 1;
  static constexpr int NPB = PER == 0 ? 4 : (64 / PER < 1 ? 1 : (64 / PER > 4 ? 4 : 64 / PER));
};

template <int D>
struct QueryRegs {
  float qv[Geo<D>::PERA];
  float qt[Geo<D>::TAILA];
};

template <int D>
__device__ __forceinline__ void load_query(const float* __restrict__ q, int lane, QueryRegs<D>& Q) {
  using G = Geo<D>;
  const int a8 = lane & 7;
#pragma unroll
  for (int t = 0; t < G::PER; ++t) Q.qv[t] = q[a8 + 8 * t];
#pragma unroll
  for (int t = 0; t < G::TAIL; ++t) Q.qt[t] = q[G::DB + t];
}

// sc_d[j] = dist(q, vec[sc_ids[j]]) for j < n.  All 64 lanes must call it.
template <int D, int METRIC, typename E>
__device__ __forceinline__ void dist_list(const E* __restrict__ vec, const QueryRegs<D>& Q, const u32* sc_ids,
                                          float* sc_d, int n, int lane) {
  using G = Geo<D>;
  const int g8 = lane >> 3, a8 = lane & 7, base = lane & ~7;
  for (int p0 = 0; p0 < n; p0 += 8 * G::NPB) {
    float x[G::NPB][G::PERA];
    float xt[G::NPB][G::TAILA];
#pragma unroll
    for (int pp = 0; pp < G::NPB; ++pp) {
      const int slot = p0 + pp * 8 + g8;
      if (slot < n) {
        const E* row = vec + static_cast<u64>(sc_ids[slot]) * D;
#pragma unroll
        for (int t = 0; t < G::PER; ++t) x[pp][t] = to_f32(row[a8 + 8 * t]);
        if (a8 == 0) {
#pragma unroll
          for (int t = 0; t < G::TAIL; ++t) xt[pp][t] = to_f32(row[G::DB + t]);
        }
      }
    }
#pragma unroll
    for (int pp = 0; pp < G::NPB; ++pp) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < G::PER; ++t) {
        if constexpr (METRIC == 0) {
          const float df = Q.qv[t] - x[pp][t];
          acc = __builtin_fmaf(df, df, acc);
        } else {
          acc = __builtin_fmaf(Q.qv[t], x[pp][t], acc);
        }
      }
      float s = __shfl(acc, base);
#pragma unroll
      for (int j = 1; j < 8; ++j) s = s + __shfl(acc, base + j);
      const int slot = p0 + pp * 8 + g8;
      if (a8 == 0 && slot < n) {
        if constexpr (METRIC == 0) {
#pragma unroll
          for (int t = 0; t < G::TAIL; ++t) {
            const float df = Q.qt[t] - xt[pp][t];
            s = __builtin_fmaf(df, df, s);
          }
        } else {
          float tl = 0.f;
#pragma unroll
          for (int t = 0; t < G::TAIL; ++t) tl = __builtin_fmaf(Q.qt[t], xt[pp][t], tl);
          s = 1.0f - (s + tl);
        }
        sc_d[slot] = s;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// search kernel: one wavefront (= one workgroup) per persistent slot
// ------------------------------------------------------------------------------------------------------------
template <int D, int METRIC, typename E>
__global__ __launch_bounds__(64) void search_kernel(SearchArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u64* top = reinterpret_cast<u64*>(smem);      // MaxHeap top_candidates, capacity ef
  u64* nxt = top + A.ef;                         // MinHeap next_candidates, capacity cap
  u32* sc_ids = reinterpret_cast<u32*>(nxt + A.cap);  // fresh neighbours of the current expansion
  float* sc_d = reinterpret_cast<float*>(sc_ids + 64);

  const int lane = threadIdx.x;
  const E* __restrict__ vec = static_cast<const E*>(A.g.vec);
  const u32 M0 = A.g.M0, MU = A.g.MU;
  const int ef = static_cast<int>(A.ef), cap = static_cast<int>(A.cap);
  u32* __restrict__ vis = A.visited + static_cast<u64>(blockIdx.x) * A.words_per_slot;
  u32* __restrict__ vlog = A.vlog + static_cast<u64>(blockIdx.x) * A.log_cap;
  const u64 below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // lanes < this one

  for (;;) {
    u32 item = 0;
    if (lane == 0) item = atomicAdd(A.counter, 1u);
    item = bcast(item);
    if (item >= A.nq) break;
    const u32 qi = A.qmap ? A.qmap[item] : item;

    QueryRegs<D> Q;
    load_query<D>(A.queries + static_cast<u64>(qi) * D, lane, Q);

    u32 st_dist = 0, st_vup = 0, st_vl0 = 0, st_lup = 0, st_ll0 = 0, st_maxnext = 0, status = 0;

    // ---- entry point (hnsw.hh:256-272) -------------------------------------------------------------------
    const u32 ep = A.g.ep;
    if (lane == 0) sc_ids[0] = ep;
    wave_sync();
    dist_list<D, METRIC, E>(vec, Q, sc_ids, sc_d, 1, lane);
    wave_sync();
    float closest = sc_d[0];
    ++st_dist;
    if (A.g.ep_level > 0) ++st_vup; else ++st_vl0;

    // ---- greedy descent search_for_one (hnsw.hh:331-393) ------------------------------------------------
    u32 nn = ep;
    for (u32 level = A.g.ep_level; level > 0 && status == 0; --level) {
      bool changed;
      do {
        changed = false;
        const u32 ub = A.g.up_base[nn];
        if (ub == INV) { status = ST_FORMAT; break; }
        const u32* row = A.g.adjU + (static_cast<u64>(ub) + level - 1) * MU;
        u32 e = INV;
        if (static_cast<u32>(lane) < MU) e = row[lane];
        const bool valid = e != INV;
        const int cnt = __popcll(__ballot(valid));
        ++st_lup;
        st_vup += cnt;
        st_dist += cnt;
        if (valid) sc_ids[lane] = e;
        wave_sync();
        dist_list<D, METRIC, E>(vec, Q, sc_ids, sc_d, cnt, lane);
        wave_sync();
        // first neighbour (list order) attaining the minimum; adopted only if strictly closer (:378)
        float bd = (lane < cnt) ? sc_d[lane] : __builtin_inff();
        if (bd != bd) bd = __builtin_inff();  // NaN never compares less
        int bi = lane;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const float od = __shfl_xor(bd, off);
          const int oi = __shfl_xor(bi, off);
          if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
        }
        bd = bcastf(bd);
        bi = static_cast<int>(bcast(static_cast<u32>(bi)));
        if (bd < closest) {
          closest = bd;
          nn = sc_ids[bi];
          changed = true;
        }
        wave_sync();
      } while (changed);
    }

    // ---- top_candidates.push({nn, dist(q, nn)}) (hnsw.hh:285-286) ---------------------------------------
    ++st_dist;
    int ntop = 1, nnext = 1;
    u32 logpos = 0;
    bool log_overflow = false;
    if (status == 0) {
      const u64 e0 = mk(closest, nn);
      if (lane == 0) {
        top[0] = e0;
        nxt[0] = e0;  // search_level :412-415
        const u32 old = atomicOr(&vis[nn >> 5], 1u << (nn & 31));
        (void)old;
        vlog[0] = nn;
      }
      logpos = 1;
      st_maxnext = 1;

      // ---- search_level(q, ef, 0) (hnsw.hh:406-476) ---------------------------------------------------------
      while (nnext > 0) {
        u64 c = 0;
        int brk = 0;
        if (lane == 0) {
          c = nxt[0];  // next_candidates.top(); pop()  (:418-419)
          heap_pop<false>(nxt, nnext);
          brk = key(c) > key(top[0]);  // :421-426
        }
        c = bcast64(c);
        brk = static_cast<int>(bcast(static_cast<u32>(brk)));
        --nnext;
        if (brk) break;

        // neighbour list of the candidate at level 0 (:436-438)
        ++st_ll0;
        const u32* row = A.g.adj0 + static_cast<u64>(eid(c)) * M0;
        u32 e = INV;
        if (static_cast<u32>(lane) < M0) e = row[lane];
        bool cand = e != INV;
        if (!A.g.lists_unique) {  // first occurrence in list order wins (visited.insert order, :443)
          for (u32 j = 0; j < M0; ++j) {
            const u32 ej = __shfl(e, static_cast<int>(j));
            if (j < static_cast<u32>(lane) && ej == e) cand = false;
          }
        }
        bool fresh = false;
        if (cand) {  // visited.contains / insert (:441-443): one atomic test-and-set per lane
          const u32 bit = 1u << (e & 31);
          fresh = (atomicOr(&vis[e >> 5], bit) & bit) == 0;
        }
        const u64 fm = __ballot(fresh);
        const int nf = __popcll(fm);
        if (fresh) {
          const int r = __popcll(fm & below);
          sc_ids[r] = e;
          const u32 lp = logpos + r;
          if (lp < A.log_cap) vlog[lp] = e;
        }
        logpos += nf;
        if (logpos > A.log_cap) log_overflow = true;
        st_vl0 += nf;
        st_dist += nf;
        if (nf == 0) continue;
        wave_sync();
        dist_list<D, METRIC, E>(vec, Q, sc_ids, sc_d, nf, lane);
        wave_sync();

        // accept / push / push_k in list order (:456-465)
        int ovf = 0;
        if (lane == 0) {
          for (int j = 0; j < nf; ++j) {
            const float d = sc_d[j];
            const float farthest = key(top[0]);
            if (d < farthest || ntop < ef) {
              if (nnext >= cap) { ovf = 1; break; }
              const u64 en = mk(d, sc_ids[j]);
              heap_push<false>(nxt, nnext, en);
              ++nnext;
              if (ntop < ef) {  // heap.hh:34-41 push_k
                heap_push<true>(top, ntop, en);
                ++ntop;
              } else if (d < key(top[0])) {
                heap_pop<true>(top, ntop);
                heap_push<true>(top, ntop - 1, en);
              }
              if (static_cast<u32>(nnext) > st_maxnext) st_maxnext = nnext;
            }
          }
        }
        ntop = static_cast<int>(bcast(static_cast<u32>(ntop)));
        nnext = static_cast<int>(bcast(static_cast<u32>(nnext)));
        st_maxnext = bcast(st_maxnext);
        if (bcast(static_cast<u32>(ovf))) { status = ST_OVERFLOW; break; }
        wave_sync();
      }

      // ---- trim to k and emit in heap-array order (:296-303) ------------------------------------------------
      if (status == 0 && lane == 0) {
        while (ntop > static_cast<int>(A.k)) {
          heap_pop<true>(top, ntop);
          --ntop;
        }
      }
      ntop = static_cast<int>(bcast(static_cast<u32>(ntop)));
      wave_sync();
    }

    const u64 obase = static_cast<u64>(qi) * A.k;
    for (u32 i = lane; i < A.k; i += 64) {
      u32 id = INV;
      float d = 0.f;
      if (status == 0 && static_cast<int>(i) < ntop) {
        const u64 en = top[i];
        id = A.g.uid[eid(en)];
        d = key(en);
      }
      A.out_ids[obase + i] = id;
      if (A.out_dists) A.out_dists[obase + i] = d;
    }
    if (A.qstats && lane == 0) {
      u32* qs = A.qstats + static_cast<u64>(qi) * 8;
      qs[0] = st_dist;
      qs[1] = st_vup;
      qs[2] = st_vl0;
      qs[3] = st_lup;
      qs[4] = st_ll0;
      qs[5] = st_maxnext;
      qs[6] = status;
      qs[7] = status == 0 ? static_cast<u32>(ntop < static_cast<int>(A.k) ? ntop : A.k) : 0u;
    }

    // ---- visited_nodes.clear() (:475): clear exactly the words this query touched -------------------------
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!log_overflow) {
      for (u32 i = lane; i < logpos; i += 64) {
        const u32 id = __hip_atomic_load(&vlog[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vis[id >> 5] = 0u;
      }
    } else {
      for (u64 w = lane; w < A.words_per_slot; w += 64) vis[w] = 0u;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// ------------------------------------------------------------------------------------------------------------
// batched distance kernel: one wavefront per (query, 64-node chunk)
// ------------------------------------------------------------------------------------------------------------
template <int D, int METRIC, typename E>
__global__ __launch_bounds__(64) void distance_kernel(DistArgs A) {
  __shared__ u32 sc_ids[64];
  __shared__ float sc_d[64];
  const int lane = threadIdx.x;
  const u32 chunks = (A.n_per + 63) / 64;
  const u64 w = blockIdx.x;
  const u32 qi = static_cast<u32>(w / chunks), ch = static_cast<u32>(w % chunks);
  if (qi >= A.nq) return;
  QueryRegs<D> Q;
  load_query<D>(A.queries + static_cast<u64>(qi) * D, lane, Q);
  const u32 j = ch * 64 + lane;
  u32 dense = INV;
  if (j < A.n_per) {
    const u32 u = A.node_uids[static_cast<u64>(qi) * A.n_per + j];
    if (u < A.g.inv_size) dense = A.g.inv_uid[u];
  }
  const bool ok = dense != INV;
  const u64 om = __ballot(ok);
  const int n = __popcll(om);
  const u64 below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int r = __popcll(om & below);
  if (ok) sc_ids[r] = dense;
  wave_sync();
  dist_list<D, METRIC, E>(static_cast<const E*>(A.g.vec), Q, sc_ids, sc_d, n, lane);
  wave_sync();
  if (j < A.n_per) A.out[static_cast<u64>(qi) * A.n_per + j] = ok ? sc_d[r] : __builtin_nanf("");
}

template <int D, int METRIC, typename E>
hipError_t launch_search_t(uint32_t grid, const SearchArgs& a, hipStream_t s) {
  const size_t lds = search_lds_bytes(a.ef, a.cap);
  if (lds > 65536) {  // beyond the default dynamic-LDS limit: opt in (per device, so every launch)
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&search_kernel<D, METRIC, E>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((search_kernel<D, METRIC, E>), dim3(grid), dim3(64), lds, s, a);
  return hipGetLastError();
}

template <int D, int METRIC, typename E>
hipError_t launch_distance_t(const DistArgs& a, hipStream_t s) {
  const u64 chunks = (a.n_per + 63) / 64;
  const u64 grid = static_cast<u64>(a.nq) * chunks;
  if (grid == 0) return hipSuccess;
  if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((distance_kernel<D, METRIC, E>), dim3(static_cast<u32>(grid)), dim3(64), 0, s, a);
  return hipGetLastError();
}

#define SHINE_DIMS(X) X(16) X(32) X(64) X(96) X(100) X(128) X(200) X(256)

}  // namespace

bool dim_supported(uint32_t dim, int elem) {
#define SHINE_CASE(DD) \
  if (dim == DD) return true;
  if (elem == 0) {
    SHINE_DIMS(SHINE_CASE)
  } else if (dim == 96 || dim == 128 || dim == 200) {
    return true;
  }
#undef SHINE_CASE
  return false;
}

hipError_t launch_search(uint32_t dim, int metric, int elem, uint32_t grid, const SearchArgs& a, hipStream_t s) {
#define SHINE_CASE(DD)                                                                  \
  if (dim == DD) {                                                                      \
    return metric == 0 ? launch_search_t<DD, 0, float>(grid, a, s)                      \
                       : launch_search_t<DD, 1, float>(grid, a, s);                     \
  }
  if (elem == 0) {
    SHINE_DIMS(SHINE_CASE)
  }
#undef SHINE_CASE
#define SHINE_CASE16(DD)                                                                \
  if (dim == DD) {                                                                      \
    return metric == 0 ? launch_search_t<DD, 0, __half>(grid, a, s)                     \
                       : launch_search_t<DD, 1, __half>(grid, a, s);                    \
  }
  if (elem == 1) {
    SHINE_CASE16(96) SHINE_CASE16(128) SHINE_CASE16(200)
  }
#undef SHINE_CASE16
  return hipErrorInvalidValue;
}

hipError_t launch_distance(uint32_t dim, int metric, int elem, const DistArgs& a, hipStream_t s) {
#define SHINE_CASE(DD)                                                              \
  if (dim == DD) {                                                                  \
    return metric == 0 ? launch_distance_t<DD, 0, float>(a, s)                      \
                       : launch_distance_t<DD, 1, float>(a, s);                     \
  }
  if (elem == 0) {
    SHINE_DIMS(SHINE_CASE)
  }
#undef SHINE_CASE
#define SHINE_CASE16(DD)                                                            \
  if (dim == DD) {                                                                  \
    return metric == 0 ? launch_distance_t<DD, 0, __half>(a, s)                     \
                       : launch_distance_t<DD, 1, __half>(a, s);                    \
  }
  if (elem == 1) {
    SHINE_CASE16(96) SHINE_CASE16(128) SHINE_CASE16(200)
  }
#undef SHINE_CASE16
  return hipErrorInvalidValue;
}

}  // namespace shine
