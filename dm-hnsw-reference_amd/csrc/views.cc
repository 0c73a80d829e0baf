// The sharded placement's view plan (views.h).
#include "views.h"

#include <algorithm>

#include "../../include/shine_gpu.h"
#include "graph.h"

namespace shine {

ViewPlan plan_views(const std::vector<int>& devs, uint64_t stride, uint64_t cached) {
  ViewPlan P;
  const size_t G = devs.size();
  P.stride = stride;
  P.cached = G > 1 ? std::min<uint64_t>(cached, stride) : 0;
  // access is granted once per view, for every device of the handle (per-piece grants on views with holes were
  // refused by the driver): every slot may be asked to read through any view of its own device
  std::vector<int> uniq(devs);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  P.pieces.assign(G, {});
  P.access.assign(G, uniq);
  for (size_t o = 0; o < G; ++o) {
    for (size_t q = 0; q < G; ++q) {
      const uint64_t base = q * stride;
      if (P.cached) {  // hot prefix: the owner's memory in its own view, the view slot's local copy in every other
        ViewPiece v;
        v.view_slot = static_cast<uint32_t>(o);
        v.stripe = static_cast<uint32_t>(q);
        v.offset = base;
        v.size = P.cached;
        v.backing_device = devs[o];  // own hot prefix or the local copy: both on the view's device
        v.kind = q == o ? 0u : 1u;
        v.hot = true;
        P.pieces[o].push_back(v);
      }
      if (P.cached < stride) {  // the cold rest: always the owner's allocation
        ViewPiece v;
        v.view_slot = static_cast<uint32_t>(o);
        v.stripe = static_cast<uint32_t>(q);
        v.offset = base + P.cached;
        v.size = stride - P.cached;
        v.backing_device = devs[q];
        v.kind = q == o ? 0u : 2u;
        P.pieces[o].push_back(v);
      }
    }
  }
  // every slot dereferences every other slot's stripe: each ordered pair of distinct devices needs a peer path
  for (int a : uniq)
    for (int b : uniq)
      if (a != b) P.peer_pairs.emplace_back(a, b);
  return P;
}

}  // namespace shine

extern "C" int shine_plan_sharded_views(const int* gpu_ids, uint32_t n_slots, uint64_t stride_bytes,
                                        uint64_t cached_bytes, shine_view_piece* pieces, uint64_t cap_pieces,
                                        uint64_t* n_pieces, int* access, uint32_t* n_access, int* peer_pairs,
                                        uint32_t* n_peer_pairs) {
  using namespace shine;
  if (!gpu_ids || n_slots == 0) return set_error(SHINE_ERR_ARG, "gpu_ids must name at least one slot");
  if (stride_bytes == 0) return set_error(SHINE_ERR_ARG, "stride_bytes must be > 0");
  const ViewPlan P = plan_views(std::vector<int>(gpu_ids, gpu_ids + n_slots), stride_bytes, cached_bytes);
  uint64_t n = 0;
  for (const auto& v : P.pieces)
    for (const ViewPiece& p : v) {
      if (pieces && n < cap_pieces)
        pieces[n] = shine_view_piece{p.view_slot, p.stripe, p.offset, p.size, p.backing_device, p.kind};
      ++n;
    }
  if (n_pieces) *n_pieces = n;
  if (pieces && n > cap_pieces) return set_error(SHINE_ERR_ARG, "pieces: capacity below the plan's pieces");
  for (uint32_t o = 0; o < n_slots; ++o) {
    if (n_access) n_access[o] = static_cast<uint32_t>(P.access[o].size());
    if (access)
      for (size_t j = 0; j < P.access[o].size(); ++j) access[static_cast<size_t>(o) * n_slots + j] = P.access[o][j];
  }
  if (n_peer_pairs) *n_peer_pairs = static_cast<uint32_t>(P.peer_pairs.size());
  if (peer_pairs)
    for (size_t i = 0; i < P.peer_pairs.size(); ++i) {
      peer_pairs[2 * i] = P.peer_pairs[i].first;
      peer_pairs[2 * i + 1] = P.peer_pairs[i].second;
    }
  return SHINE_OK;
}
