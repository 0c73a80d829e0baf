// gfx950 kernels of the GPU batch builder (HNSW::insert, src/hnsw/hnsw.hh:40-251, and
// select_heuristic, :482-522), included by kernels_dim.hip after kernels_impl.h and instantiated per dimension for
// f32 rows (the reference's element_t, types.hh:9).  Host orchestration: gpu_build.cc.
//
// A batch of consecutive node ids is inserted against the graph as it stood before the batch:
//   * level 0: the fast search kernel itself (knn with k = ef = efC over the partial graph) yields every node's
//     efC best level-0 candidates, ascending — the search_level(efC, 0) of hnsw.hh:151-154;
//   * build_upper_kernel: nodes whose level is >= 1 also run the greedy descent (search_for_one, :129-143) and a
//     search_level(efC, l) beam at every level l = min(level, top) .. 1, each seeded by the previous level's closest;
//   * build_select_kernel: select_heuristic(M) (:482-522) over every candidate list → the node's own list at that
//     level, and one reverse-edge request per selected neighbour (:180-225);
//   * build_prune_kernel: the requests sorted by target row; a row that keeps room takes them as appended entries,
//     a row that would exceed m_max (2M at level 0, M above) is re-pruned with select_heuristic(m_max) over its old
//     entries and all its new ones together (the reference prunes once per incoming edge, :191-221).
// Distances are the search kernels' (dist_list: the reference's AVX2 accumulation order).
//
// Deliberate differences from the reference's insert (DESIGN §4 "GPU batch builder"), all by construction:
//   * records of one batch do not see each other (a batch is <= 2 % of the graph built so far);
//   * the level-0 beam of a record with upper levels starts from the greedy descent's node (the search kernel's
//     descent with ef = 1 through every level), not from the closest node of its own level-1 beam as hnsw.hh:227-230
//     leaves it: the level-0 searches of a whole batch run as one search-kernel launch before the upper beams, which
//     only ~1/M of the records run.  Its level-0 beam starts from a node no closer than the reference's; the GPU-built graph's
//     recall is within 1e-4 of the CPU builder's at 1M (profiles/r04/cmp1m_gpu_vs_cpu_build.jsonl);
//   * a row receiving several new entries in one batch is re-pruned once over all of them (the reference prunes per
//     incoming edge, :191-221).
#pragma once

#include "kernels_impl.h"

namespace shine {
namespace {

// A device row (f32, kernels.h permuted_index) as the "query" of dist_list: the lane's pairs {x[2c + 8t],
// x[2c + 1 + 8t]} sit side by side at (t >> 1) * 16 + c * 4 + (t & 1) * 2, the tail unpermuted.
template <int D>
__device__ __forceinline__ void load_query_row(const float* __restrict__ row, int lane, QueryRegs<D, float>& Q) {
  constexpr int DB = D >> 4 << 4, PER = DB / 8, TAIL = D - DB;
  const int c4 = lane & 3;
#pragma unroll
  for (int t = 0; t < PER; ++t) Q.q2[t] = *reinterpret_cast<const f32x2*>(row + (t >> 1) * 16 + c4 * 4 + (t & 1) * 2);
#pragma unroll
  for (int t = 0; t < TAIL; ++t) Q.qt[t] = row[DB + t];
}

// select_heuristic (hnsw.hh:482-522) over n candidates already in ascending order (cid / cd: ids and their distances
// to the base node; generic pointers, LDS or HBM).  Fewer than m candidates are all kept (:485); otherwise the
// closest is kept and each next one is kept unless a kept node is strictly closer to it than the base node is
// (:500-511), until m are kept.  sel / seld (LDS, 64 entries): the kept ids and distances, in order.  The distances
// from candidate c to the kept nodes are one dist_list with c as the query (symmetric, bitwise: the same products
// in the same accumulator order).
template <int D, int METRIC>
__device__ int heuristic(const float* __restrict__ vec, const u32* cid, const float* cd, int n, int m, u32* sel,
                         float* seld, float* sc_d, int lane) {
  if (n <= 0) return 0;
  if (n < m) {
    for (int i = lane; i < n; i += 64) {
      sel[i] = cid[i];
      seld[i] = cd[i];
    }
    wave_sync();
    return n;
  }
  if (lane == 0) {
    sel[0] = cid[0];
    seld[0] = cd[0];
  }
  wave_sync();
  int nsel = 1;
  for (int i = 1; i < n && nsel < m; ++i) {
    const u32 c = cid[i];
    const float dc = cd[i];
    QueryRegs<D, float> Qc;
    load_query_row<D>(vec + static_cast<u64>(c) * D, lane, Qc);
    dist_list<D, METRIC, float>(vec, Qc, sel, sc_d, nsel, lane);
    wave_sync();
    const bool rej = lane < nsel && sc_d[lane] < dc;
    if (__ballot(rej) == 0ull) {
      if (lane == 0) {
        sel[nsel] = c;
        seld[nsel] = dc;
      }
      ++nsel;
    }
    wave_sync();
  }
  return nsel;
}

__device__ __forceinline__ u32 row_key(const BuildArgs& A, u32 node, u32 level) {
  return level == 0 ? node : A.g.N + A.g.up_base[node] + level - 1;
}

// ---- upper levels -------------------------------------------------------------------------------------------
// One wavefront per batch node of level >= 1: EP distance, greedy descent over levels top .. L+1 (first minimum in
// list order, adopted only if strictly closer, hnsw.hh:364-384), then for l = L .. 1 a best-first beam of ef
// candidates over the level-l lists (hnsw.hh:406-476: the sorted list of the fast kernel — the smallest unexpanded
// entry is next; the loop ends when none is left), written as candidate list up_first[u] + (L - l).  The visited set
// is an exact LDS table; a beam that would overfill it stops early (counted in stats[3]).
template <int D, int METRIC>
__global__ __launch_bounds__(64) void build_upper_kernel(BuildArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int ef = static_cast<int>(A.ef);
  const int R = (ef + 63) >> 6;
  float* lk = reinterpret_cast<float*>(smem);
  u32* li = reinterpret_cast<u32*>(lk + 64 * R);
  u32* sc_ids = li + 64 * R;
  float* sc_d = reinterpret_cast<float*>(sc_ids + 64);
  u32* vt = reinterpret_cast<u32*>(sc_d + 64);
  const u32 vmask = A.vis_cap - 1;
  const u32 vlimit = A.vis_cap / 8 * 7 - 64;
  const float* __restrict__ vec = static_cast<const float*>(A.g.vec);
  const u32 MU = A.g.MU;
  const u64 below = lane == 0 ? 0ull : (~0ull >> (64 - lane));

  const u32 u = blockIdx.x;
  if (u >= A.n_up) return;
  const u32 q = A.up_node[u];
  const u32 L = A.up_levels[u];
  const u32 out0 = A.up_first[u] - A.up_first_base;
  QueryRegs<D, float> Q;
  load_query<D, float>(A.base + static_cast<u64>(q) * D, lane, Q);

  // EP + greedy descent to level L + 1
  u32 nn = A.g.ep;
  if (lane == 0) sc_ids[0] = nn;
  wave_sync();
  dist_list<D, METRIC, float>(vec, Q, sc_ids, sc_d, 1, lane);
  wave_sync();
  float closest = sc_d[0];
  wave_sync();
  for (u32 level = A.g.ep_level; level > L; --level) {
    bool changed;
    do {
      changed = false;
      const u32* row = A.g.adjU + (static_cast<u64>(A.g.up_base[nn]) + level - 1) * MU;
      const u32 e = static_cast<u32>(lane) < MU ? row[lane] : INV;
      const bool valid = e != INV;
      const u64 vm = __ballot(valid);
      const int cnt = __popcll(vm);
      if (valid) sc_ids[__popcll(vm & below)] = e;
      wave_sync();
      dist_list<D, METRIC, float>(vec, Q, sc_ids, sc_d, cnt, lane);
      wave_sync();
      float bd = lane < cnt ? sc_d[lane] : __builtin_inff();
      if (bd != bd) bd = __builtin_inff();
      const float mn = wave_min(bd);
      if (mn < closest) {
        const int bi = static_cast<int>(__builtin_ctzll(__ballot(bd == mn)));
        closest = mn;
        nn = sc_ids[bi];
        changed = true;
      }
      wave_sync();
    } while (changed);
  }

  u32 ent = nn;
  float ent_d = closest;
  u64 stopped = 0;
  for (u32 l = L; l >= 1; --l) {
    for (u32 i = lane; i < A.vis_cap; i += 64) vt[i] = INV;
    for (int r = 0; r < R; ++r) {
      lk[64 * r + lane] = __builtin_inff();
      li[64 * r + lane] = INV;
    }
    wave_sync();
    if (lane == 0) {
      vt[(ent * 0x9E3779B1u) & vmask] = ent;
      lk[0] = ent_d;
      li[0] = ent;
    }
    wave_sync();
    int cs = 1;
    u32 nvis = 1;
    for (;;) {
      int p = -1;
      for (int r = R - 1; r >= 0; --r) {
        const int pos = 64 * r + lane;
        const u64 m = __ballot(pos < cs && (li[pos] & EXPANDED) == 0u);
        if (m) p = 64 * r + static_cast<int>(__builtin_ctzll(m));
      }
      if (p < 0) break;
      if (nvis + MU > vlimit) {
        stopped = 1;
        break;
      }
      const u32 c = li[p];
      wave_sync();
      if (lane == 0) li[p] = c | EXPANDED;
      const u32* row = A.g.adjU + (static_cast<u64>(A.g.up_base[c]) + l - 1) * MU;
      const u32 e = static_cast<u32>(lane) < MU ? row[lane] : INV;
      bool fresh = false;
      if (e != INV) {
        u32 h = (e * 0x9E3779B1u) & vmask;
        for (;;) {
          const u32 old = atomicCAS(&vt[h], INV, e);
          if (old == INV) {
            fresh = true;
            break;
          }
          if (old == e) break;
          h = (h + 1) & vmask;
        }
      }
      const u64 fm = __ballot(fresh);
      const int nf = __popcll(fm);
      nvis += nf;
      if (fresh) sc_ids[__popcll(fm & below)] = e;
      wave_sync();
      if (nf == 0) continue;
      dist_list<D, METRIC, float>(vec, Q, sc_ids, sc_d, nf, lane);
      wave_sync();
      for (int i = 0; i < nf; ++i) {  // push / push_k in list order (hnsw.hh:461-465)
        const float d = sc_d[i];
        const u32 id = sc_ids[i];
        if (d != d) continue;
        if (cs == ef && !(d < lk[ef - 1])) continue;
        int rank = 0;  // entries at or below d stay ahead of it
        float kv[8];
        u32 iv[8];
        for (int r = 0; r < R; ++r) {
          const int pos = 64 * r + lane;
          kv[r] = lk[pos];
          iv[r] = li[pos];
          rank += __popcll(__ballot(pos < cs && kv[r] <= d));
        }
        wave_sync();
        for (int r = 0; r < R; ++r) {
          const int pos = 64 * r + lane;
          if (pos >= rank && pos < cs && pos + 1 < ef) {
            lk[pos + 1] = kv[r];
            li[pos + 1] = iv[r];
          }
        }
        wave_sync();
        if (lane == 0) {
          lk[rank] = d;
          li[rank] = id;
        }
        cs = cs < ef ? cs + 1 : ef;
        wave_sync();
      }
    }
    // candidate list of level l, ascending (ids without the expanded bit), INV-padded
    const u64 o = static_cast<u64>(A.n_lists0 + out0 + (L - l)) * A.ef;
    for (int r = 0; r < R; ++r) {
      const int pos = 64 * r + lane;
      if (pos < ef) {
        A.cand_ids[o + pos] = pos < cs ? (li[pos] & ~EXPANDED) : INV;
        A.cand_d[o + pos] = pos < cs ? lk[pos] : 0.f;
      }
    }
    ent = li[0] & ~EXPANDED;
    ent_d = lk[0];
    wave_sync();
  }
  if (lane == 0 && stopped) atomicAdd(&A.stats[3], 1ull);
}

// ---- select_heuristic(M) per candidate list → own lists + reverse-edge requests -------------------------------
template <int D, int METRIC>
__global__ __launch_bounds__(64) void build_select_kernel(BuildArgs A) {
  __shared__ u32 sel[64];
  __shared__ float seld[64], sc_d[64];
  const int lane = threadIdx.x;
  const u32 w = blockIdx.x;
  if (w >= A.n_lists0 + A.n_listsU) return;
  u32 node, level;
  if (w < A.n_lists0) {
    node = A.batch_start + w;
    level = 0;
  } else {
    node = A.list_node[w - A.n_lists0];
    level = A.list_level[w - A.n_lists0];
  }
  const u32* cid = A.cand_ids + static_cast<u64>(w) * A.ef;
  const float* cd = A.cand_d + static_cast<u64>(w) * A.ef;
  int n = 0;  // valid candidates: an INV-padded prefix
  for (u32 c = 0; c < A.ef; c += 64) {
    const u32 i = c + lane;
    n += __popcll(__ballot(i < A.ef && cid[i] != INV));
  }
  const float* __restrict__ vec = static_cast<const float*>(A.g.vec);
  const int nsel = heuristic<D, METRIC>(vec, cid, cd, n, static_cast<int>(A.M), sel, seld, sc_d, lane);
  const u32 len = level == 0 ? A.g.M0 : A.g.MU;
  u32* row = level == 0 ? A.adj0w + static_cast<u64>(node) * A.g.M0
                        : A.adjUw + (static_cast<u64>(A.g.up_base[node]) + level - 1) * A.g.MU;
  if (static_cast<u32>(lane) < len) row[lane] = lane < nsel ? sel[lane] : INV;
  if (static_cast<u32>(lane) < A.M) {
    const u64 pos = static_cast<u64>(w) * A.M + lane;
    A.req_key[pos] = lane < nsel ? row_key(A, sel[lane], level) : A.key_none;
    A.req_src[pos] = node;
    A.req_d[pos] = lane < nsel ? seld[lane] : 0.f;
    A.req_pos[pos] = static_cast<u32>(pos);
  }
}

// ---- reverse edges ------------------------------------------------------------------------------------------
__device__ __forceinline__ u64 shfl_xor64(u64 v, int m) {
  const u32 lo = static_cast<u32>(__shfl_xor(static_cast<int>(static_cast<u32>(v)), m));
  const u32 hi = static_cast<u32>(__shfl_xor(static_cast<int>(static_cast<u32>(v >> 32)), m));
  return (static_cast<u64>(hi) << 32) | lo;
}
__device__ __forceinline__ u64 shfl64(u64 v, int src) {
  const u32 lo = static_cast<u32>(__shfl(static_cast<int>(static_cast<u32>(v)), src));
  const u32 hi = static_cast<u32>(__shfl(static_cast<int>(static_cast<u32>(v >> 32)), src));
  return (static_cast<u64>(hi) << 32) | lo;
}
// bitonic sort of one key per lane, ascending in lane order
__device__ __forceinline__ u64 sort64(u64 v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const u64 o = shfl_xor64(v, j);
      const bool up = (lane & k) == 0 || k == 64;
      const bool lower = (lane & j) == 0;
      const u64 mn = v < o ? v : o, mx = v < o ? o : v;
      v = lower == up ? mn : mx;
    }
  }
  return v;
}
// a bitonic sequence (one key per lane) into ascending order
__device__ __forceinline__ u64 merge64(u64 v, int lane) {
#pragma unroll
  for (int j = 32; j > 0; j >>= 1) {
    const u64 o = shfl_xor64(v, j);
    const u64 mn = v < o ? v : o, mx = v < o ? o : v;
    v = (lane & j) == 0 ? mn : mx;
  }
  return v;
}
// (distance, id) as one ascending key: the distance's order-preserving image, then the id (ties by id, heap.hh:53-57)
__device__ __forceinline__ u64 dkey(float d, u32 id) { return (static_cast<u64>(sortable(d)) << 32) | id; }
__device__ __forceinline__ float dkey_dist(u64 k) {
  const u32 s = static_cast<u32>(k >> 32);
  return __uint_as_float((s & 0x80000000u) ? (s & 0x7FFFFFFFu) : ~s);
}

// One wavefront per target row (persistent; rows from the segment list of the sorted requests).  A row with room for
// all its new entries appends them in request order (node order: the reference's appends, hnsw.hh:184-188); otherwise
// its old entries (distances recomputed, :192-197) and the new ones are pooled, the 64 closest kept (by distance,
// then id), and select_heuristic(m_max) over them rewrites the row (:198-221).
template <int D, int METRIC>
__global__ __launch_bounds__(64) void build_prune_kernel(BuildArgs A) {
  __shared__ u32 cid[64], sel[64], sc_ids[64];
  __shared__ float cd[64], seld[64], sc_d[64];
  const int lane = threadIdx.x;
  const float* __restrict__ vec = static_cast<const float*>(A.g.vec);
  const u32 nseg = *A.nseg;
  u64 n_app = 0, n_prune = 0, n_trunc = 0;
  for (;;) {
    u32 item = 0;
    if (lane == 0) item = atomicAdd(A.work, 1u);
    item = bcast(item);
    if (item >= nseg) break;
    const u32 i0 = A.seg[item];
    const u32 key = A.skey[i0];
    u32 i1 = i0 + 1;
    for (u32 c = i0 + 1;; c += 64) {  // the segment's end: the first different key
      const u32 i = c + lane;
      const bool diff = i >= A.n_req || A.skey[i] != key;
      const u64 m = __ballot(diff);
      if (m) {
        i1 = c + static_cast<u32>(__builtin_ctzll(m));
        break;
      }
    }
    const u32 nin = i1 - i0;
    const bool l0 = key < A.g.N;
    const u32 target = l0 ? key : A.row_owner[key - A.g.N];
    const u32 mmax = l0 ? A.g.M0 : A.g.MU;
    u32* row = l0 ? A.adj0w + static_cast<u64>(key) * A.g.M0 : A.adjUw + static_cast<u64>(key - A.g.N) * A.g.MU;
    const u32 e = static_cast<u32>(lane) < mmax ? row[lane] : INV;
    const int cnt = __popcll(__ballot(e != INV));
    if (static_cast<u32>(cnt) + nin <= mmax) {
      for (u32 t = lane; t < nin; t += 64) row[cnt + t] = A.req_src[A.sval[i0 + t]];
      ++n_app;
      continue;
    }
    ++n_prune;
    QueryRegs<D, float> Qt;
    load_query_row<D>(vec + static_cast<u64>(target) * D, lane, Qt);
    if (lane < cnt) sc_ids[lane] = e;
    wave_sync();
    dist_list<D, METRIC, float>(vec, Qt, sc_ids, sc_d, cnt, lane);
    wave_sync();
    u64 best = sort64(lane < cnt ? dkey(sc_d[lane], e) : ~0ull, lane);
    for (u32 c = 0; c < nin; c += 64) {
      const u32 t = c + lane;
      u64 k = ~0ull;
      if (t < nin) {
        const u32 pos = A.sval[i0 + t];
        k = dkey(A.req_d[pos], A.req_src[pos]);
      }
      k = sort64(k, lane);
      k = shfl64(k, 63 - lane);  // descending
      best = merge64(best < k ? best : k, lane);
    }
    const int n = static_cast<int>(static_cast<u32>(cnt) + nin < 64u ? static_cast<u32>(cnt) + nin : 64u);
    if (static_cast<u32>(cnt) + nin > 64u) ++n_trunc;
    cid[lane] = static_cast<u32>(best);
    cd[lane] = dkey_dist(best);
    wave_sync();
    const int nsel = heuristic<D, METRIC>(vec, cid, cd, n, static_cast<int>(mmax), sel, seld, sc_d, lane);
    if (static_cast<u32>(lane) < mmax) row[lane] = lane < nsel ? sel[lane] : INV;
    wave_sync();
  }
  if (lane == 0) {
    if (n_app) atomicAdd(&A.stats[0], n_app);
    if (n_prune) atomicAdd(&A.stats[1], n_prune);
    if (n_trunc) atomicAdd(&A.stats[2], n_trunc);
  }
}

template <int D, int METRIC>
hipError_t launch_build_t(int which, uint32_t grid, const BuildArgs& a, hipStream_t s) {
  if (grid == 0) return hipSuccess;
  if (which == BUILD_UPPER) {
    const size_t lds = 8ull * ((a.ef + 63) / 64 * 64) + 512 + 4ull * a.vis_cap;
    const void* kern = reinterpret_cast<const void*>(&build_upper_kernel<D, METRIC>);
    if (lds > 65536) {
      hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((build_upper_kernel<D, METRIC>), dim3(grid), dim3(64), lds, s, a);
  } else if (which == BUILD_SELECT) {
    hipLaunchKernelGGL((build_select_kernel<D, METRIC>), dim3(grid), dim3(64), 0, s, a);
  } else if (which == BUILD_PRUNE) {
    hipLaunchKernelGGL((build_prune_kernel<D, METRIC>), dim3(grid), dim3(64), 0, s, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace
}  // namespace shine
