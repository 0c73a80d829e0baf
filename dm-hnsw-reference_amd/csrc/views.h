// The sharded placement's view plan (SHINE_PLACE_SHARDED): which physical allocation backs every piece of
// every GPU slot's virtual view of a sharded array, which devices each view grants access to, and which device pairs
// need a peer path.  Pure host code (no HIP call), so that the plan the multi-GPU open maps (capi.cc map_sharded) is
// testable on a machine without GPUs (tests/test_views.py through shine_plan_sharded_views).
//
// The reference places a record on memory node RemotePtr bits 63..48 (remote_pointer.hh:9-22) and a compute node
// reads every memory node over RDMA; here memory node s lives on slot s % G and every slot reads the other slots'
// stripes through its own view of the whole id space (read_data.hh:57-58 splits the queries over the slots).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace shine {

// One mapped piece of a view.  kind: 0 = the view's own stripe (its hot prefix or cold rest), 1 = the view slot's local
// copy of stripe `stripe`'s hot prefix (the cache of remote records), 2 = stripe `stripe`'s cold rows, backed by the
// owner's HBM (a peer read over xGMI when the owner is another GPU).
struct ViewPiece {
  uint32_t view_slot = 0, stripe = 0;
  uint64_t offset = 0, size = 0;  // in the view's virtual range
  int backing_device = 0;         // the GPU whose allocation backs the piece
  uint32_t kind = 0;
  bool hot = false;               // the piece is a hot prefix (own hot, or a local copy of another stripe's)
};

struct ViewPlan {
  uint64_t stride = 0;  // bytes of one slot's stripe in the view (U rows)
  uint64_t cached = 0;  // bytes of every stripe's hot prefix that the other slots copy (0 with one slot)
  std::vector<std::vector<ViewPiece>> pieces;  // [view slot]: its pieces in offset order, covering [0, G * stride)
  std::vector<std::vector<int>> access;        // [view slot]: devices granted read/write on the whole view
  std::vector<std::pair<int, int>> peer_pairs; // ordered (accessor, owner) device pairs that need a peer path
};

// slots G = devs.size(); slot o is on device devs[o] (devices may repeat: several slots of one GPU).
ViewPlan plan_views(const std::vector<int>& devs, uint64_t stride, uint64_t cached);

}  // namespace shine
