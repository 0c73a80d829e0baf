// gfx950 (CDNA4) kernels of the SHINE compute-node query path (device code and launch templates; included by
// kernels.hip and by one kernels_dim.hip translation unit per vector dimension, compiled in parallel).
//
//   search_kernel   HNSW::knn (src/hnsw/hnsw.hh:253-307): greedy descent search_for_one (:331-393) and the
//                   level-0 best-first beam search search_level (:406-476), one query per wavefront,
//                   persistent workgroups pulling queries from a device work queue.
//   distance_kernel Distance::dist (src/hnsw/distance.hh:153-161) over gathered (query, node) pairs.
//   heap_replay     diagnostics: the device heap routines driven by an op list (tests pin them to libstdc++).
//
// Exactness.  Distances are evaluated in exactly the oracle's floating-point order (oracle/oracle.cc): eight
// lanes of a wavefront play the eight AVX2 accumulators of L2SqrSIMD16ExtAVX / InnerProductSIMD16ExtAVX
// (distance.hh:11-76) — lane a owns elements i ≡ a (mod 8) of the 16-aligned prefix and runs the same fmaf
// chain — the eight partial sums are added left to right, then the scalar tail.  The two candidate queues are
// the reference's std::vector heaps (heap.hh) kept in LDS and updated with exactly the libstdc++ algorithms
// (bits/stl_heap.h: __push_heap, __adjust_heap, __pop_heap), so ties between equal distances are broken as on
// the CPU and results come out in the same heap-array order (hnsw.hh:300-303).
//
// Wave-parallel heap operations (one query = one wavefront, all 64 lanes cooperate on each operation):
//   push   the ancestors of the new slot are loaded in one LDS round, each lane compares its ancestor with the
//          new key, and the length of the run of moves (a ballot + ctz) fixes the final slot; the moved
//          ancestors are stored in one more round.  (std::__push_heap walks the same chain one level at a time.)
//   pop    std::__adjust_heap's hole walks from the root to a leaf always taking the child the comparator
//          prefers, independently of the value being re-inserted.  The walk is resolved five levels per LDS
//          round: 62 lanes load the 5-level subtree under the hole, 31 lanes compare sibling pairs, and the
//          ballot of "right child wins" bits is walked with scalar bit tests.  The final std::__push_heap of the
//          last element climbs back up that same path, so its stopping point is one more ballot, and all moves
//          are written in one round.
// Expansion step (search_level): pop the closest candidate; its 2M-entry adjacency row is one coalesced
// 128-/256-byte load (one u32 per lane), issued speculatively during the previous step's accept phase for the
// predicted next candidate; the visited test-and-set is an exact open-addressing hash table in LDS (CAS per
// lane); fresh neighbours' vectors are gathered 8 per wave-instruction group and reduced; the accept / push /
// push_k sequence (:456-465) is replayed in list order with the parallel heap operations.
#pragma once

#include "kernels.h"

#include <hip/hip_fp16.h>

#include <type_traits>

// v_writelane_b32 (this clang exposes readlane as a builtin but not writelane): `val` into lane `lane` of `old`
extern "C" __device__ int shine_writelane_i32(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

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
__device__ __forceinline__ u64 bcast64(u64 v) {
  return (static_cast<u64>(bcast(static_cast<u32>(v >> 32))) << 32) | bcast(static_cast<u32>(v));
}
// Cross-lane LDS hand-off inside one wavefront: DS instructions of a wave execute in order, so only compiler
// code motion has to be stopped.
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__half x) { return __half2float(x); }
__device__ __forceinline__ float to_f32(uint8_t x) { return static_cast<float>(x); }
__device__ __forceinline__ float to_f32(int8_t x) { return static_cast<float>(x); }

// ------------------------------------------------------------------------------------------------------------
// Heaps of packed {dist, id} entries in LDS.
//   MAXH = true : heap::MaxHeapCompare (lhs.distance < rhs.distance), heap.hh:15-17
//   MAXH = false: heap::MinHeapCompare (lhs.distance > rhs.distance), heap.hh:19-21
// ------------------------------------------------------------------------------------------------------------
template <bool MAXH>
__device__ __forceinline__ bool hcmp(float a, float b) {
  return MAXH ? (a < b) : (a > b);
}

// push_back(v) + std::push_heap on h[0..n]  ≡  std::__push_heap(h, n, 0, v).  Returns the new root given the
// old one (root0; ignored when n == 0).
template <bool MAXH>
__device__ __forceinline__ u64 heap_push(u64* h, int n, u64 v, u64 root0, int lane) {
  const float vd = key(v);
  const int L = 31 - __clz(n + 1);  // ancestors of slot n
  u64 ent = 0;
  bool c = false;
  if (lane < L) {  // lane t holds ancestor t+1
    ent = h[((n + 1) >> (lane + 1)) - 1];
    c = hcmp<MAXH>(key(ent), vd);  // parent moves down while comp(parent, value)
  }
  const u64 C = __ballot(c);
  const int s = static_cast<int>(__builtin_ctzll(~C));  // moves happen for the first s ancestors
  if (lane < s) h[lane == 0 ? n : ((n + 1) >> lane) - 1] = ent;
  const int fin = s == 0 ? n : ((n + 1) >> s) - 1;
  if (lane == 0) h[fin] = v;
  wave_sync();
  return fin == 0 ? v : root0;
}

// heap_push on next_candidates (min-heap `hn`, size nn) and on top_candidates (max-heap `ht`, size nt) in one LDS
// round: lanes 0..31 play hn's ancestors, lanes 32..63 ht's.  The two heaps are independent, so this is the two
// std::push_heap calls in either order, at the LDS latency of one.
__device__ __forceinline__ void heap_push2(u64* hn, int nn, u64* ht, int nt, u64 v, u64& root_n, u64& root_t,
                                           int lane) {
  const bool second = lane >= 32;
  const int l = lane & 31;
  u64* h = second ? ht : hn;
  const int n = second ? nt : nn;
  const float vd = key(v);
  const int L = 31 - __clz(n + 1);
  u64 ent = 0;
  bool c = false;
  if (l < L) {
    ent = h[((n + 1) >> (l + 1)) - 1];
    c = second ? hcmp<true>(key(ent), vd) : hcmp<false>(key(ent), vd);
  }
  const u64 C = __ballot(c);
  const int sn = static_cast<int>(__builtin_ctz(~static_cast<u32>(C)));
  const int st = static_cast<int>(__builtin_ctz(~static_cast<u32>(C >> 32)));
  const int s = second ? st : sn;
  if (l < s) h[l == 0 ? n : ((n + 1) >> l) - 1] = ent;
  const int fin = s == 0 ? n : ((n + 1) >> s) - 1;
  if (l == 0) h[fin] = v;
  wave_sync();
  const int fin_n = sn == 0 ? nn : ((nn + 1) >> sn) - 1, fin_t = st == 0 ? nt : ((nt + 1) >> st) - 1;
  if (fin_n == 0) root_n = v;
  if (fin_t == 0) root_t = v;
}

// General form (any keys, NaN included): the value's landing slot is found bottom-up like std::__push_heap.
// std::pop_heap on h[0..n) followed by pop_back  ≡  std::__adjust_heap(h, 0, n-1, h[n-1]).  Returns the new
// root (meaningless when n <= 1).
//
// The hole's walk is resolved six levels per LDS round: lane i plays internal node i+1 (1-based) of the
// 63-node window below the hole, reads both children's keys (adjacent slots: one ds_read2_b32) and votes
// "right child wins"; the walk then follows the ballot with scalar bit tests.
template <bool MAXH>
__device__ __forceinline__ u64 heap_pop_any(u64* h, int n, int lane) {
  if (n <= 1) return 0;
  const int len = n - 1;
  const u64 value = h[len];
  const float vk = key(value);
  const int lim = (len - 1) / 2;  // the hole has two children while hole < lim
  const u32* hk = reinterpret_cast<const u32*>(h);
  const int j1 = lane + 1;
  const int lj = 31 - __clz(j1);
  const int oj = j1 - (1 << lj);
  int pos = 0, L = 0, my_child = 0;  // lane t: the path's (t+1)-th node
  while (pos < lim) {
    const int a = ((pos + 1) << lj) - 1 + oj;  // this lane's node
    const int c1 = 2 * a + 1;
    bool right = false;
    if (lane < 63 && c1 + 1 < len) {
      const float lk = __uint_as_float(hk[2 * c1]);
      const float rk = __uint_as_float(hk[2 * c1 + 2]);
      right = !hcmp<MAXH>(rk, lk);  // libstdc++ takes the left child iff comp(right, left)
    }
    const u64 W = __ballot(right);
    int r1 = 1;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      if (pos >= lim) break;
      const int b = static_cast<int>((W >> (r1 - 1)) & 1ull);
      const int child = 2 * pos + 1 + b;
      if (lane == L) my_child = child;
      ++L;
      pos = child;
      r1 = 2 * r1 + b;
    }
  }
  if ((len & 1) == 0 && pos == (len - 2) / 2) {  // lone left child
    const int child = 2 * pos + 1;
    if (lane == L) my_child = child;
    ++L;
    pos = child;
  }
  // std::__push_heap(h, hole = path end, 0, value) climbs the same path
  u64 ent = 0;
  bool c = false;
  if (lane < L) {
    ent = h[my_child];
    c = hcmp<MAXH>(key(ent), vk);
  }
  const u64 C = __ballot(c);
  const u64 stay = ~C & (L >= 64 ? ~0ull : ((1ull << L) - 1));
  const int j = stay ? 64 - __clzll(stay) : 0;  // value lands on the path's j-th node
  const int pj = j == 0 ? 0 : __shfl(my_child, j - 1);
  if (lane < j) h[(my_child - 1) >> 1] = ent;  // path nodes above the landing slot shift up
  if (lane == 0) h[pj] = value;
  wave_sync();
  return j == 0 ? value : bcast64(ent);  // lane 0 holds the path's first node
}

// Per-lane constants of the pop window: lane i plays window node j = i + 1 (1-based, depth lj, offset oj within its
// depth); anc has bit (a - 1) set for every window ancestor a of j, dir holds at that bit the side (1 = right) the
// path takes from a towards j.  Lane 63 is outside the 63-node window.
struct PopLane {
  u64 anc = 0, dir = 0;
  int lj = 0, oj = 0;
  bool in_window = false;
  __device__ __forceinline__ explicit PopLane(int lane) {
    const int j1 = lane + 1;
    lj = 31 - __clz(j1);
    oj = j1 - (1 << lj);
    in_window = lane < 63;
    for (int t = 0; t < lj; ++t) {
      const int a = j1 >> (lj - t);
      anc |= 1ull << (a - 1);
      dir |= static_cast<u64>((j1 >> (lj - t - 1)) & 1) << (a - 1);
    }
  }
};

// Fast form for NaN-free heaps.  std::__adjust_heap's hole walks from the root towards the leaves, at every node
// into the child the comparator prefers (the right one unless comp(right, left)), while the node has a child; along
// any root-to-leaf path of a heap the keys are monotone, so the comparisons std::__push_heap makes on its way back
// up are false on a prefix of the path and true below it: every path node whose winning child the comparator does
// not rank past the value shifts that child up, the first one that does receives the value.  Each 6-level window
// costs one LDS round trip: lane i plays window node i+1, reads both children entries (adjacent slots: one
// ds_read2_b64) and votes for the right child; a lane knows it lies on the hole's path when the ballot agrees with
// the side of every one of its window ancestors (one masked compare against its PopLane constants: no serial walk),
// and the on-path lanes shift their winner up in place.
template <bool MAXH>
__device__ __forceinline__ u64 heap_pop(u64* h, int n, int lane, const PopLane& pl) {
  if (n <= 1) return 0;
  const int len = n - 1;
  const u64 value = h[len];
  const float vk = key(value);
  int P1 = 1;  // window root, 1-based heap index
  u64 root = value;
  for (int round = 0;; ++round) {
    const int a1 = (P1 << pl.lj) + pl.oj;  // this lane's node, 1-based
    const int c1 = 2 * a1 - 1;             // its left child, 0-based
    const bool has_child = pl.in_window && c1 < len;
    u64 le = 0, re = 0;
    if (has_child) {
      le = h[c1];
      re = h[c1 + 1];
    }
    const bool right = has_child && c1 + 1 < len && !hcmp<MAXH>(key(re), key(le));
    const u64 we = right ? re : le;  // the child the hole would move into
    const u64 W = __ballot(right);
    // on the path: every window ancestor sent the hole this lane's way; a hole there moves on iff the node has a child
    const bool hole = has_child && ((W ^ pl.dir) & pl.anc) == 0ull;
    const bool up = hole && !hcmp<MAXH>(key(we), vk);  // no move back down: the winner stays shifted up
    const u64 H = __ballot(hole), UP = __ballot(up);
    if (up) h[a1 - 1] = we;
    if (round == 0) root = UP & 1ull ? bcast64(we) : value;  // lane 0 is the root
    const u64 stop = H & ~UP;
    if (stop) {  // the first path node whose winner stays below the value receives it
      if (lane == static_cast<int>(__builtin_ctzll(stop))) h[a1 - 1] = value;
      break;
    }
    // every hole moved: the walk ends in the deepest hole's winner child, or goes on from it in the next window
    const int cw1 = 2 * a1 + (right ? 1 : 0);
    const int P = H ? __builtin_amdgcn_readlane(cw1, 63 - static_cast<int>(__clzll(H))) : P1;
    // no hole at window depth 5 (the path ended inside this window), or the deepest hole moved into a leaf (P has no
    // child: at ef = 128 every full pop ends so, and the next window would only place the value)
    if (!(H >> 31) || 2 * P > len) {
      if (lane == 0) h[P - 1] = value;
      break;
    }
    P1 = P;
  }
  wave_sync();
  return root;
}

// ------------------------------------------------------------------------------------------------------------
// Distance evaluation in the oracle's FP order.  A "pass" evaluates 16 vectors: lane l of the wavefront belongs
// to group g = l >> 2 (the vector, or slot) and plays the two AVX2 accumulators 2c and 2c+1, c = l & 3, as the
// two halves of a packed-FP32 register pair: each half runs the scalar fmaf chain of its accumulator
// (distance.hh:11-76), so v_pk_fma_f32 does two accumulators per instruction.  Rows are stored in the device
// layout of kernels.h (permuted_index): one 16-byte load (f32; 8 bytes for f16) brings elements t and t+1 of
// both of the lane's accumulators, already paired, and the 4 lanes of a group read 64 contiguous bytes.  The
// eight partial sums are folded left to right, ((((a0 + a1) + a2) ... ) + a7), by a 3-step DPP row_shr:1 chain
// that ends in the group's lane c = 3, which then adds the scalar tail.
// ------------------------------------------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int D, typename E>
struct Lay {
  static constexpr int DB = D >> 4 << 4;  // elements handled by the SIMD16 kernel (qty16 << 4)
  static constexpr int PER = DB / 8;      // elements per accumulator
  static constexpr int NCH = PER / 2;     // 4-element chunks per lane
  static constexpr int TAIL = D - DB;     // scalar tail (distance.hh:112-115, 136-139)
  static constexpr int TAILA = TAIL > 0 ? TAIL : 1;
  static_assert(DB >= 16, "dimension must be >= 16");
};

template <typename E>
constexpr bool kByte = std::is_same_v<E, uint8_t> || std::is_same_v<E, int8_t>;

template <int D, typename E = float, bool BYTES = kByte<E>>
struct QueryRegs {
  f32x2 q2[D / 16 * 2];  // {q[2c + 8t], q[2c + 1 + 8t]}, t < PER
  float qt[(D & 15) > 0 ? (D & 15) : 1];
};
// Byte rows also keep the query as bytes when every component is a byte value of the rows' kind (SIFT's u8 queries
// against u8 records): qb[u] packs the four components the lane's row word u pairs with (kernels.h
// permuted_index_bytes), qq is the lane's share of sum(q^2), qint says the whole query qualified (wave-uniform).
template <int D, typename E>
struct QueryRegs<D, E, true> {
  f32x2 q2[D / 16 * 2];
  float qt[(D & 15) > 0 ? (D & 15) : 1];
  u32 qb[D / 16 > 0 ? D / 16 : 1];
  int qq;
  bool qint;
};

// fp16 rows (natural order, see NbrBuf<D, __half>): the query for both distance paths — the MFMA operand of the inner
// product (lane l: A row l & 15, elements 32s + 8(l >> 4) .. +7 of every step s; row 0 the high halves of q * 2^e, row
// 1 the low halves q * 2^e - high, the other rows zero, so the product keeps ~21 bits of the f32 query; 2^e brings
// the largest component near 2^14, clear of fp16's subnormals) and the L2 path's f32 values (lane l: chunk l & 3 of
// every step).  Elements past D are zero.  (A kernel compiles only the part its metric reads.)
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
template <int D>
constexpr int kHalfSteps = (D + 31) / 32;  // 32-element steps of an fp16 row
template <int D>
struct QueryRegs<D, __half, false> {
  static constexpr int NS = kHalfSteps<D>;
  v8h a[NS];         // MFMA A fragments (inner product)
  float inv_scale;   // 2^-e
  float qv[NS][8];   // vector path (L2): this lane's chunk of every step, f32
};

template <int D, typename E>
__device__ __forceinline__ void load_query(const float* __restrict__ q, int lane, QueryRegs<D, E>& Q) {
  if constexpr (std::is_same_v<E, __half>) {
    constexpr int NS = kHalfSteps<D>;
    // the query's largest magnitude (every lane reads a strided share; a DPP max over the wave)
    float mx = 0.f;
    for (int i = lane; i < D; i += 64) mx = fmaxf(mx, fabsf(q[i]));
    {
      int x = __float_as_int(mx);
#define SHINE_DPP_MAX(CTRL, RM)                                                                                    \
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, CTRL, RM, 0xF, false))));
      SHINE_DPP_MAX(0x111, 0xF)
      SHINE_DPP_MAX(0x112, 0xF)
      SHINE_DPP_MAX(0x114, 0xF)
      SHINE_DPP_MAX(0x118, 0xF)
      SHINE_DPP_MAX(0x142, 0xA)
      SHINE_DPP_MAX(0x143, 0xC)
#undef SHINE_DPP_MAX
      mx = __int_as_float(__builtin_amdgcn_readlane(x, 63));
    }
    // 2^e with mx * 2^e in [2^13, 2^14): exact powers of two, so the scaling itself rounds nothing
    int e = 0;
    if (mx > 0.f && mx == mx && mx < __builtin_inff()) {
      int ex;
      (void)frexpf(mx, &ex);  // mx = f * 2^ex, f in [0.5, 1)
      e = 14 - ex;
      e = e > 100 ? 100 : (e < -100 ? -100 : e);
    }
    const float scale = ldexpf(1.f, e);
    Q.inv_scale = ldexpf(1.f, -e);
    const int m = lane & 15, kg = lane >> 4, c = lane & 3;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      v8h a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 32 * s + 8 * kg + j;
        const float v = (m < 2 && i < D) ? q[i] * scale : 0.f;
        const _Float16 hi = static_cast<_Float16>(v);
        a[j] = m == 0 ? hi : static_cast<_Float16>(v - static_cast<float>(hi));
      }
      Q.a[s] = a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 32 * s + 8 * c + j;
        Q.qv[s][j] = i < D ? q[i] : 0.f;
      }
    }
  } else {
  constexpr int DB = D >> 4 << 4, PER = DB / 8, TAIL = D - DB;
  const int c2 = 2 * (lane & 3);
#pragma unroll
  for (int t = 0; t < PER; ++t) Q.q2[t] = f32x2{q[c2 + 8 * t], q[c2 + 1 + 8 * t]};
#pragma unroll
  for (int t = 0; t < TAIL; ++t) Q.qt[t] = q[DB + t];
  if constexpr (kByte<E>) {
    constexpr bool U8 = std::is_same_v<E, uint8_t>;
    const float lo = U8 ? 0.f : -128.f, hi = U8 ? 255.f : 127.f;
    auto byte_ok = [&](float f) { return f == __builtin_rintf(f) && f >= lo && f <= hi; };
    bool ok = true;
    int qq = 0;
#pragma unroll
    for (int u = 0; u < PER / 2; ++u) {
      const float f[4] = {Q.q2[2 * u].x, Q.q2[2 * u].y, Q.q2[2 * u + 1].x, Q.q2[2 * u + 1].y};
      u32 w = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ok &= byte_ok(f[i]);
        const int v = static_cast<int>(f[i]);
        w |= (static_cast<u32>(v) & 0xFFu) << (8 * i);
        qq += v * v;
      }
      Q.qb[u] = w;
    }
#pragma unroll
    for (int t = 0; t < TAIL; ++t) ok &= byte_ok(Q.qt[t]);
    Q.qq = qq;
    Q.qint = __ballot(!ok) == 0ull;
  }
  }  // (f32 and byte rows)
}

// One chunk = elements (t, t+1) of accumulators (2c, 2c+1): f32 → 4 floats, f16 → 4 halves in 2 words, bytes →
// one word.
// elements of one device row (byte rows are padded to 16 bytes, kernels.h row_bytes)
template <int D, typename E>
constexpr int kRowElems = kByte<E> ? (D + 15) / 16 * 16 : D;

template <typename E>
struct ChunkT {
  using type = f32x4;
};
template <>
struct ChunkT<__half> {
  using type = uint2;
};

// The neighbour vectors of P passes (16 slots each) in VGPRs.  The scalar tail (distance.hh:112-115, d = 100 / 200) is
// loaded as whole 16-byte words, one load instruction per 16 bytes instead of one per element (d = 200 fp16 rows: 1
// load instead of 8 next to the lane's 12 chunk loads), and widened where lane c = 3 adds it.
template <int D, typename E, int P, bool BYTES = kByte<E>>
struct NbrBuf {
  using L = Lay<D, E>;
  static constexpr int TQ = L::TAIL > 0 ? (L::TAIL * static_cast<int>(sizeof(E)) + 15) / 16 : 1;
  static_assert(L::TAIL * sizeof(E) % 16 == 0, "the tail of a row must be whole 16-byte words");
  typename ChunkT<E>::type x[P][L::NCH];
  uint4 xt[P][TQ];
};
// Byte rows: the lane's NCH chunk words (contiguous in the row, kernels.h permuted_index_bytes) and the tail bytes
// as whole words; widened to f32 where the distances consume them.
template <int D, typename E, int P>
struct NbrBuf<D, E, P, true> {
  using L = Lay<D, E>;
  static constexpr int TW = L::TAIL > 0 ? (L::TAIL + 3) / 4 : 1;
  u32 x[P][L::NCH];
  u32 xt[P][TW];
};

// fp16 rows (config 5) are stored in natural element order (kernels.h row layout): fp16 records are judged by recall
// against the f32 oracle, not bitwise, so their sums need not follow the reference's eight-accumulator order.  A row is
// NS = ceil(D / 32) steps of 32 elements; a lane holds one 16-byte chunk (8 halves) per step, elements 32s + 8c ..
// 32s + 8c + 7 for its chunk index c (0..3); chunks past D are loaded from a valid address and masked to zero.  Inner
// product runs on the matrix cores (pass_dists_mfma: lane l takes slot l & 15 and chunk c = l >> 4, the B operand
// layout of v_mfma_f32_16x16x32_f16); L2 on the vector units (pass_dists: slot group g = l >> 2, chunk c = l & 3).
template <int D, int P>
struct NbrBuf<D, __half, P, false> {
  static constexpr int NS = kHalfSteps<D>;
  static_assert(D % 8 == 0, "fp16 rows are read in chunks of 8 elements");
  uint4 x[P][NS];
};
template <int METRIC, typename E>
constexpr bool kMfma = METRIC == 1 && std::is_same_v<E, __half>;
// chunk c of step s lies inside the row
template <int D>
__device__ __forceinline__ bool half_chunk_valid(int s, int c) { return 32 * s + 8 * c + 8 <= D; }
// this lane's chunks (index c) of one fp16 row: a chunk past the row reads the step's first chunk instead (always inside
// the row; its values are masked where the distances use them)
template <int D, int P>
__device__ __forceinline__ void load_half_row(NbrBuf<D, __half, P>& B, int p, const __half* __restrict__ row, int c) {
#pragma unroll
  for (int s = 0; s < kHalfSteps<D>; ++s) {
    const int off = half_chunk_valid<D>(s, c) ? 32 * s + 8 * c : 32 * s;
    B.x[p][s] = *reinterpret_cast<const uint4*>(row + off);
  }
}

// This lane's part of one byte row: NCH words at byte c4 * NCH * 4 in the widest aligned loads, then the tail words.
template <int D, typename E, int P>
__device__ __forceinline__ void load_byte_row(NbrBuf<D, E, P>& B, int p, const E* __restrict__ row, int c4) {
  using L = Lay<D, E>;
  constexpr int NCH = L::NCH;
  const unsigned char* rb = reinterpret_cast<const unsigned char*>(row);
  const unsigned char* base = rb + c4 * NCH * 4;
  if constexpr (NCH % 4 == 0) {
#pragma unroll
    for (int v = 0; v < NCH / 4; ++v) {
      const uint4 w = reinterpret_cast<const uint4*>(base)[v];
      B.x[p][4 * v] = w.x;
      B.x[p][4 * v + 1] = w.y;
      B.x[p][4 * v + 2] = w.z;
      B.x[p][4 * v + 3] = w.w;
    }
  } else if constexpr (NCH % 2 == 0) {
#pragma unroll
    for (int v = 0; v < NCH / 2; ++v) {
      const uint2 w = reinterpret_cast<const uint2*>(base)[v];
      B.x[p][2 * v] = w.x;
      B.x[p][2 * v + 1] = w.y;
    }
  } else {
#pragma unroll
    for (int v = 0; v < NCH; ++v) B.x[p][v] = reinterpret_cast<const u32*>(base)[v];
  }
  if constexpr (L::TAIL > 0) {
    const u32* tw = reinterpret_cast<const u32*>(rb + L::DB);
#pragma unroll
    for (int t = 0; t < NbrBuf<D, E, P>::TW; ++t) B.xt[p][t] = tw[t];
  }
}

// Off-stripe record x of a dynamic-cache view (DevGraph::cbits, cslot): its arena row when cached, else its xGMI row.
// A cslot word is the arena slot with the entry's cooling flag in bit 31 (kCool), INV when x is not cached.
constexpr u32 kCool = 0x80000000u;
__device__ __forceinline__ u32 read_class(const DevGraph& g, u32 x, u32 cached);
template <int D, typename E>
__device__ __forceinline__ const E* cached_row(const DevGraph& g, const E* row, u32 x) {
  if (read_class(g, x, 0u) == 2u && ((g.cbits[x >> 5] >> (x & 31)) & 1u)) {
    const u32 c = g.cslot[x];
    if (c != INV) return static_cast<const E*>(g.cvec) + static_cast<u64>(c & ~kCool) * kRowElems<D, E>;
  }
  return row;
}
// The cache word of a level-0 list entry, looked up once where the list arrives (the fast kernel carries it from the
// row request to the read accounting): INV for an empty slot, a record of this GPU's stripe, or one not cached.
__device__ __forceinline__ u32 cache_word(const DevGraph& g, u32 x) {
  return x != INV && read_class(g, x, 0u) == 2u ? g.cslot[x] : INV;
}
template <int D, typename E>
__device__ __forceinline__ const E* word_row(const DevGraph& g, const E* row, u32 w) {
  return w != INV ? static_cast<const E*>(g.cvec) + static_cast<u64>(w & ~kCool) * kRowElems<D, E> : row;
}

// Issue the loads of pass p: this lane's group evaluates node `id` (INV: nothing to load).  CACHE (the ACCT = 2 kernels
// of a dynamic-cache view): a cached off-stripe record is read from this GPU's arena, as the read accounting counts it.
template <int D, typename E, int P, bool CACHE = false>
__device__ __forceinline__ void issue_pass(NbrBuf<D, E, P>& B, int p, const E* __restrict__ vec, u32 id, int c4,
                                           const DevGraph* cg = nullptr) {
  using L = Lay<D, E>;
  if (id != INV) {
    const E* row = vec + static_cast<u64>(id) * kRowElems<D, E>;
    if constexpr (CACHE) row = cached_row<D, E>(*cg, row, id);
    if constexpr (kByte<E>) {
      load_byte_row<D, E, P>(B, p, row, c4);
    } else if constexpr (std::is_same_v<E, __half>) {
      load_half_row<D, P>(B, p, row, c4);
    } else {
      using C = typename ChunkT<E>::type;
#pragma unroll
      for (int u = 0; u < L::NCH; ++u) B.x[p][u] = *reinterpret_cast<const C*>(row + u * 16 + c4 * 4);
      if constexpr (L::TAIL > 0) {
        if (c4 == 3) {
#pragma unroll
          for (int t = 0; t < NbrBuf<D, E, P>::TQ; ++t) B.xt[p][t] = reinterpret_cast<const uint4*>(row + L::DB)[t];
        }
      }
    }
  }
}

// Unconditional form: always the same number of load instructions (an INV slot reads the local node `pad` and is
// ignored), so that the compiler's vmcnt bookkeeping stays exact across the software pipeline of search_fast_kernel.
template <int D, typename E, int P>
__device__ __forceinline__ void issue_row(NbrBuf<D, E, P>& B, int p, const E* __restrict__ row, int c4) {
  using L = Lay<D, E>;
  if constexpr (kByte<E>) {
    load_byte_row<D, E, P>(B, p, row, c4);
  } else if constexpr (std::is_same_v<E, __half>) {
    load_half_row<D, P>(B, p, row, c4);
  } else {
    using C = typename ChunkT<E>::type;
#pragma unroll
    for (int u = 0; u < L::NCH; ++u) B.x[p][u] = *reinterpret_cast<const C*>(row + u * 16 + c4 * 4);
    if constexpr (L::TAIL > 0) {
#pragma unroll
      for (int t = 0; t < NbrBuf<D, E, P>::TQ; ++t) B.xt[p][t] = reinterpret_cast<const uint4*>(row + L::DB)[t];
    }
  }
}

template <int D, typename E, int P>
__device__ __forceinline__ void issue_pass_u(NbrBuf<D, E, P>& B, int p, const E* __restrict__ vec, u32 id, u32 pad,
                                             int c4) {
  issue_row<D, E, P>(B, p, vec + static_cast<u64>(id == INV ? pad : id) * kRowElems<D, E>, c4);
}

// byte i of word w widened to f32 (exact): v_cvt_f32_ubyte{i} for u8, a sign-extending extract + convert for i8
template <typename E>
__device__ __forceinline__ float byte_f32(u32 w, int i) {
  if constexpr (std::is_same_v<E, uint8_t>) return static_cast<float>((w >> (8 * i)) & 0xFFu);
  else return static_cast<float>(static_cast<int>(w << (24 - 8 * i)) >> 24);
}

__device__ __forceinline__ float half_lo(u32 w) {
  return __half2float(__ushort_as_half(static_cast<unsigned short>(w & 0xFFFFu)));
}
__device__ __forceinline__ float half_hi(u32 w) { return __half2float(__ushort_as_half(static_cast<unsigned short>(w >> 16))); }
__device__ __forceinline__ f32x2 half2_to_f32x2(u32 w) {
  return f32x2{__half2float(__ushort_as_half(static_cast<unsigned short>(w & 0xFFFFu))),
               __half2float(__ushort_as_half(static_cast<unsigned short>(w >> 16)))};
}

// Left fold of a group's 8 accumulators (lane c holds 2c, 2c+1) into its lane c = 3.
__device__ __forceinline__ float fold8(f32x2 acc) {
  float s = acc.x + acc.y;
#pragma unroll
  for (int j = 1; j < 4; ++j)
    s = (__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x111, 0xF, 0xF, false)) + acc.x) + acc.y;
  return s;
}

template <int D, int METRIC, typename E>
__device__ __forceinline__ float add_tail(const QueryRegs<D, E>& Q, const float* xt, float s) {
  constexpr int TAIL = D & 15;
  if constexpr (METRIC == 0) {
#pragma unroll
    for (int t = 0; t < TAIL; ++t) {
      const float df = Q.qt[t] - xt[t];
      s = __builtin_fmaf(df, df, s);
    }
    return s;
  } else {
    float tl = 0.f;
#pragma unroll
    for (int t = 0; t < TAIL; ++t) tl = __builtin_fmaf(Q.qt[t], xt[t], tl);
    return 1.0f - (s + tl);
  }
}

template <int METRIC>
__device__ __forceinline__ f32x2 acc_step(f32x2 q, f32x2 x, f32x2 acc) {
  if constexpr (METRIC == 0) {
    const f32x2 df = q - x;
    return __builtin_elementwise_fma(df, df, acc);
  } else {
    return __builtin_elementwise_fma(q, x, acc);
  }
}

// Byte query against byte rows: every term of the reference's f32 sums is an integer and every partial sum stays
// below 2^24 (d <= 256: 256 x 255^2 < 2^24), so the f32 FMA chains are exact and equal the integer sums.  The
// integer sums are taken with v_dot4 (four byte products per instruction): L2 as sum(q^2) + sum(x^2) - 2 sum(q x),
// IP as sum(q x); the group's four lanes are added in lane 3 (DPP), the tail there too; converted once, exactly.
template <typename E>
__device__ __forceinline__ int dot4(u32 a, u32 b, int c) {
  if constexpr (std::is_same_v<E, uint8_t>) return static_cast<int>(__builtin_amdgcn_udot4(a, b, static_cast<u32>(c), false));
  else return __builtin_amdgcn_sdot4(static_cast<int>(a), static_cast<int>(b), c, false);
}

template <int D, int METRIC, typename E, int P>
__device__ __forceinline__ void pass_dists_int(const QueryRegs<D, E>& Q, const NbrBuf<D, E, P>& B, float (&out)[P]) {
  using L = Lay<D, E>;
  int v[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int qx = 0, xx = 0;
#pragma unroll
    for (int u = 0; u < L::NCH; ++u) {
      qx = dot4<E>(Q.qb[u], B.x[p][u], qx);
      if constexpr (METRIC == 0) xx = dot4<E>(B.x[p][u], B.x[p][u], xx);
    }
    v[p] = METRIC == 0 ? Q.qq + xx - 2 * qx : qx;
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int s = v[p] + __builtin_amdgcn_update_dpp(0, v[p], 0x111, 0xF, 0xF, false);  // row_shr:1
    s += __builtin_amdgcn_update_dpp(0, s, 0x112, 0xF, 0xF, false);                 // row_shr:2: lane 3 = 0+1+2+3
#pragma unroll
    for (int t = 0; t < L::TAIL; ++t) {
      const int q = static_cast<int>(Q.qt[t]), x = static_cast<int>(byte_f32<E>(B.xt[p][t >> 2], t & 3));
      s += METRIC == 0 ? (q - x) * (q - x) : q * x;
    }
    out[p] = METRIC == 0 ? static_cast<float>(s) : 1.0f - static_cast<float>(s);
  }
}

// out[p] = distance of the pass-p vector of this lane's group; valid in lanes c = 3.
template <int D, int METRIC, typename E, int P>
__device__ __forceinline__ void pass_dists(const QueryRegs<D, E>& Q, const NbrBuf<D, E, P>& B, float (&out)[P]) {
  using L = Lay<D, E>;
  if constexpr (std::is_same_v<E, __half>) {
    // fp16 rows on the vector units (natural order): the lane's chunk c = lane & 3 of every step, two accumulators per
    // slot (even / odd elements), then the group's four lanes summed into its lane 3 (DPP); chunks past D contribute 0
    const int c = static_cast<int>(threadIdx.x) & 3;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int st = 0; st < kHalfSteps<D>; ++st) {
        const bool ok = st < kHalfSteps<D> - 1 || D % 32 == 0 || half_chunk_valid<D>(st, c);
        const u32 w[4] = {B.x[p][st].x, B.x[p][st].y, B.x[p][st].z, B.x[p][st].w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const float x0 = ok ? half_lo(w[h]) : 0.f, x1 = ok ? half_hi(w[h]) : 0.f;
          if constexpr (METRIC == 0) {
            const float d0 = Q.qv[st][2 * h] - x0, d1 = Q.qv[st][2 * h + 1] - x1;
            a0 = __builtin_fmaf(d0, d0, a0);
            a1 = __builtin_fmaf(d1, d1, a1);
          } else {
            a0 = __builtin_fmaf(Q.qv[st][2 * h], x0, a0);
            a1 = __builtin_fmaf(Q.qv[st][2 * h + 1], x1, a1);
          }
        }
      }
      float v = a0 + a1;
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));  // row_shr:1
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xF, 0xF, false));  // row_shr:2
      out[p] = METRIC == 0 ? v : 1.0f - v;
    }
  } else {
  if constexpr (kByte<E>) {
    if (Q.qint) {  // byte query, byte rows: exact integer dot products (wave-uniform branch)
      pass_dists_int<D, METRIC, E, P>(Q, B, out);
      return;
    }
  }
  f32x2 acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) acc[p] = f32x2{0.f, 0.f};
#pragma unroll
  for (int u = 0; u < L::NCH; ++u) {
#pragma unroll
    for (int p = 0; p < P; ++p) {  // P independent chains interleaved
      f32x2 x0, x1;
      if constexpr (std::is_same_v<E, float>) {
        x0 = B.x[p][u].xy;
        x1 = B.x[p][u].zw;
      } else if constexpr (kByte<E>) {
        const u32 w = B.x[p][u];
        x0 = f32x2{byte_f32<E>(w, 0), byte_f32<E>(w, 1)};
        x1 = f32x2{byte_f32<E>(w, 2), byte_f32<E>(w, 3)};
      } else if constexpr (METRIC == 1) {
        // f16 rows, inner product: each accumulator's fmaf on the half widened in place (v_fma_mix_f32 with op_sel
        // picking the half: the widening is exact, one rounding as fmaf(q, float(x), acc)), 2 instructions per
        // word instead of 2 conversions and a packed FMA; same operands in the same order per accumulator
        const u32 w0 = B.x[p][u].x, w1 = B.x[p][u].y;
        acc[p].x = __builtin_fmaf(Q.q2[2 * u].x, half_lo(w0), acc[p].x);
        acc[p].y = __builtin_fmaf(Q.q2[2 * u].y, half_hi(w0), acc[p].y);
        acc[p].x = __builtin_fmaf(Q.q2[2 * u + 1].x, half_lo(w1), acc[p].x);
        acc[p].y = __builtin_fmaf(Q.q2[2 * u + 1].y, half_hi(w1), acc[p].y);
        continue;
      } else {
        x0 = half2_to_f32x2(B.x[p][u].x);
        x1 = half2_to_f32x2(B.x[p][u].y);
      }
      acc[p] = acc_step<METRIC>(Q.q2[2 * u], x0, acc[p]);
      acc[p] = acc_step<METRIC>(Q.q2[2 * u + 1], x1, acc[p]);
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if constexpr (kByte<E>) {
      float xt[L::TAILA];
#pragma unroll
      for (int t = 0; t < L::TAILA; ++t) xt[t] = L::TAIL > 0 ? byte_f32<E>(B.xt[p][t >> 2], t & 3) : 0.f;
      out[p] = add_tail<D, METRIC, E>(Q, xt, fold8(acc[p]));
    } else {
      float xt[L::TAILA];
      if constexpr (L::TAIL > 0) {
        E te[NbrBuf<D, E, P>::TQ * 16 / sizeof(E)];
        __builtin_memcpy(te, B.xt[p], sizeof(te));
#pragma unroll
        for (int t = 0; t < L::TAIL; ++t) xt[t] = to_f32(te[t]);
      } else {
        xt[0] = 0.f;
      }
      out[p] = add_tail<D, METRIC, E>(Q, xt, fold8(acc[p]));
    }
  }
  }  // (f32 and byte rows)
}

// Inner products of fp16 rows on the matrix cores: per pass p, lane l holds chunk l >> 4 of slot 16p + (l & 15) (the B
// operand of v_mfma_f32_16x16x32_f16: B[8(l >> 4) + j][l & 15]), the query's high and low halves are rows 0 and 1 of A
// (QueryRegs<D, __half>), and one MFMA per 32-element step accumulates C = A B; C[0][n] + C[1][n] (lane n, registers 0
// and 1) is slot 16p + n's product with the scaled query.  out[p] = 1 - <q, x> of slot 16p + lane in lanes 0..15.
template <int D, int P>
__device__ __forceinline__ void pass_dists_mfma(const QueryRegs<D, __half>& Q, const NbrBuf<D, __half, P>& B,
                                                float (&out)[P]) {
  const int c = static_cast<int>(threadIdx.x) >> 4;
  v4f acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) acc[p] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < kHalfSteps<D>; ++st) {
#pragma unroll
    for (int p = 0; p < P; ++p) {  // P independent accumulation chains interleaved
      uint4 w = B.x[p][st];
      // (only the last step can hold chunks past D: they were loaded from the step's first chunk)
      if (st == kHalfSteps<D> - 1 && D % 32 != 0 && !half_chunk_valid<D>(st, c)) w = make_uint4(0u, 0u, 0u, 0u);
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Q.a[st], __builtin_bit_cast(v8h, w), acc[p], 0, 0, 0);
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) out[p] = 1.0f - (acc[p][0] + acc[p][1]) * Q.inv_scale;
}

// slots p0 .. p0 + 16P - 1 of the list (those below n)
template <int D, int METRIC, typename E, int P, bool CACHE = false>
__device__ __forceinline__ void dist_chunk(const E* __restrict__ vec, const QueryRegs<D, E>& Q, const u32* sc_ids,
                                           float* sc_d, int p0, int n, int lane, const DevGraph* cg = nullptr) {
  if constexpr (kMfma<METRIC, E>) {  // fp16 inner products: lane l reads chunk l >> 4 of slot 16p + (l & 15)
    const int n16 = lane & 15, c = lane >> 4;
    NbrBuf<D, E, P> B;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int slot = p0 + 16 * p + n16;
      const u32 id = slot < n ? sc_ids[slot] : INV;
      if (id != INV) {
        const E* row = vec + static_cast<u64>(id) * D;
        if constexpr (CACHE) row = cached_row<D, E>(*cg, row, id);
        load_half_row<D, P>(B, p, row, c);
      } else {
#pragma unroll
        for (int st = 0; st < kHalfSteps<D>; ++st) B.x[p][st] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    float out[P];
    pass_dists_mfma<D, P>(Q, B, out);
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int slot = p0 + 16 * p + lane;
      if (lane < 16 && slot < n) sc_d[slot] = out[p];
    }
    return;
  }
  const int g4 = lane >> 2, c4 = lane & 3;
  NbrBuf<D, E, P> B;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int slot = p0 + 16 * p + g4;
    issue_pass<D, E, P, CACHE>(B, p, vec, slot < n ? sc_ids[slot] : INV, c4, cg);
  }
  float out[P];
  pass_dists<D, METRIC, E, P>(Q, B, out);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int slot = p0 + 16 * p + g4;
    if (c4 == 3 && slot < n) sc_d[slot] = out[p];
  }
}

// sc_d[j] = dist(q, vec[sc_ids[j]]) for j < n.  All 64 lanes must call it.  Two passes (32 slots) at a time while
// more than 16 remain, then one: a list of <= 16 fresh nodes (an upper-level
// list, most level-0 expansions of the heap kernel) costs one pass of VALU instead of two.
template <int D, int METRIC, typename E, bool CACHE = false>
__device__ __forceinline__ void dist_list(const E* __restrict__ vec, const QueryRegs<D, E>& Q, const u32* sc_ids,
                                          float* sc_d, int n, int lane, const DevGraph* cg = nullptr) {
  int p0 = 0;
  for (; n - p0 > 16; p0 += 32) dist_chunk<D, METRIC, E, 2, CACHE>(vec, Q, sc_ids, sc_d, p0, n, lane, cg);
  if (p0 < n) dist_chunk<D, METRIC, E, 1, CACHE>(vec, Q, sc_ids, sc_d, p0, n, lane, cg);
}

// Exact visited set (hashset_t<RemotePtr>, types.hh:14-15) on dense node ids.
//   VIS = 0: open-addressing table of u32 keys in LDS, linear probing, LDS compare-and-swap per lane.
//   VIS = 1: per-slot bitmap in HBM (atomicOr test-and-set) + a log of set ids for clearing (large-LDS fallback).
__device__ __forceinline__ u32 vhash(u32 key, u32 shift) { return (key * 0x9E3779B1u) >> shift; }

// ------------------------------------------------------------------------------------------------------------
// Read accounting (qstats words 8-11): the reads a search makes of records outside its GPU's own stripe, split
// into those served by the local copies (cache hits) and those that cross xGMI — the analogue of the
// reference's rdma_reads_in_bytes / cache_hits / cache_misses (rdma_reads.hh:12,46; statistics.hh:148-175).
// Counted per wave step with ballots; a replica index (sharded = 0) skips it on a uniform branch.  With
// A.access set (cache warmup), every record read is also counted per device id for the admission ranking.
// ------------------------------------------------------------------------------------------------------------
struct ReadCount {
  u32 vec_remote = 0, list_remote = 0, vec_cached = 0, list_cached = 0;
};

// 0 own stripe, 1 cached copy, 2 xGMI; `cached` = the array's cached rows per stripe (vectors or lists)
__device__ __forceinline__ u32 read_class(const DevGraph& g, u32 x, u32 cached) {
  const u32 s = __umulhi(x, g.div_magic) >> g.div_shift;
  const u32 r = x - s * g.stripe_ids;
  return s == g.slot ? 0u : (r < cached ? 1u : 2u);
}

// The coin of a level-0 miss once the cache is full (hnsw.hh:447-448, ADMISSION_RATIO = 0.01, constants.hh:16): a
// SplitMix64 hash of (seed, call, query, device id) below 0.01 * 2^24 in its top 24 bits (oracle/cache_ref.py).
__device__ __forceinline__ bool admission_coin(unsigned long long seed, u32 call, u32 q, u32 x) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (call + 1ull) + 0xC2B2AE3D27D4EB4Full * (q + 1ull) +
                         0x165667B19E3779F9ull * (x + 1ull);
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (z >> 40) < static_cast<unsigned long long>(0.01 * (1 << 24));
}

// vector reads of the lanes with `active` set (each reads record x; `always`: an entry-point or upper-level read,
// admitted without the coin).  ACCT = 0 (replica, no warmup) compiles the accounting out of the search loop; ACCT = 2
// adds the dynamic cache's lookups and logs (DevGraph::cslot).
// (w: the entry's cache word when the caller looked it up already, kNoWord to look it up here)
constexpr u32 kNoWord = 0xFFFFFFFEu;
template <int ACCT>
__device__ __forceinline__ void count_vec_reads(const SearchArgs& A, ReadCount& rc, bool active, u32 x, u32 qi = 0,
                                                bool always = false, u32 w = kNoWord) {
  if constexpr (!ACCT) return;
  if (A.g.sharded) {
    u32 c = active ? read_class(A.g, x, A.g.cached_rows) : 0u;
    if constexpr (ACCT == 2) {
      if (c == 2u) {
        const u32 word = w != kNoWord ? w : ((A.g.cbits[x >> 5] >> (x & 31)) & 1u) ? A.g.cslot[x] : INV;
        if (word != INV) {
          const u32 slot = word & ~kCool;
          c = 1u;
          // a hit on a cooling entry: its second chance (cache.hh:128-132) is the host's to give, so the hit is logged
          // by device id and the flag is left as the host engine set it: the flags on the device always equal the
          // engine's after its last update, which is what lets the updates trail the calls (capi.cc replay).  The
          // host takes each key once, so each slot logs once per log epoch (the plain read filters repeat hits
          // before the exchange that decides): the log holds at most one entry per arena slot and cannot overflow
          if (word & kCool) {
            const u32 ep = A.g.dyn_epoch;
            if (A.g.rlogged[slot] != ep && atomicExch(&A.g.rlogged[slot], ep) != ep) {
              const u32 i = atomicAdd(&A.g.clog_n[1], 1u);
              if (i < A.g.rlog_cap) A.g.rlog[i] = x;
            }
          }
        } else {
          const bool coin = admission_coin(A.g.dyn_seed, A.g.dyn_call, qi, x);
          if (always || !A.g.dyn_full || coin) {
            const u32 i = atomicAdd(&A.g.clog_n[0], 1u);
            if (i < A.g.clog_cap)
              A.g.clog[i] = (static_cast<unsigned long long>(qi) << 32) | x | (always ? 0x80000000ull : 0ull) |
                            (coin ? 0x8000000000000000ull : 0ull);
          }
        }
      }
    }
    rc.vec_remote += __popcll(__ballot(c == 2u));
    rc.vec_cached += __popcll(__ballot(c == 1u));
  }
  if (A.access && active) atomicAdd(&A.access[x], 1u);
}

// one neighbour-list read of record x (x uniform over the wave)
template <int ACCT>
__device__ __forceinline__ void count_list_read(const SearchArgs& A, ReadCount& rc, u32 x, int lane) {
  if constexpr (!ACCT) return;
  if (A.g.sharded) {
    const u32 c = read_class(A.g, x, A.g.cached_list_rows);
    rc.list_remote += c == 2u ? 1u : 0u;
    rc.list_cached += c == 1u ? 1u : 0u;
  }
  if (A.access && lane == 0) atomicAdd(&A.access[x], 1u);
}

__device__ __forceinline__ void write_read_counts(u32* qs, const ReadCount& rc) {
  qs[8] = rc.vec_remote;
  qs[9] = rc.list_remote;
  qs[10] = rc.vec_cached;
  qs[11] = rc.list_cached;
}

// ------------------------------------------------------------------------------------------------------------
// Wave-wide minimum on DPP: row_shr 1/2/4/8 inside each 16-lane row, then row_bcast15 / row_bcast31 — six VALU
// steps instead of a ds_bpermute butterfly.  Lanes that hold nothing must pass +inf; NaN never wins.
// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_min(float v) {
  int x = __float_as_int(v);
#define SHINE_DPP_MIN(CTRL, RM)                                                                        \
  x = __float_as_int(fminf(__int_as_float(x),                                                          \
                           __int_as_float(__builtin_amdgcn_update_dpp(0x7F800000, x, CTRL, RM, 0xF, false))));
  SHINE_DPP_MIN(0x111, 0xF)
  SHINE_DPP_MIN(0x112, 0xF)
  SHINE_DPP_MIN(0x114, 0xF)
  SHINE_DPP_MIN(0x118, 0xF)
  SHINE_DPP_MIN(0x142, 0xA)
  SHINE_DPP_MIN(0x143, 0xC)
#undef SHINE_DPP_MIN
  return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

// ------------------------------------------------------------------------------------------------------------
// Entry point + greedy descent, shared by both search kernels: HNSW::knn's EP read and distance
// (hnsw.hh:256-272) and search_for_one over levels ep_level..1 (hnsw.hh:331-393).  Counters: distcomps,
// visited_nodes (upper / L0 for the EP), visited_neighborlists (upper).  status = ST_FORMAT on a broken index.
// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ u32 sortable(float f) {  // order-preserving u32 image of a float (total order)
  const u32 b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

template <int D, int METRIC, typename E, int ACCT>
__device__ __forceinline__ void entry_and_descent(const SearchArgs& A, const E* __restrict__ vec,
                                                  const QueryRegs<D, E>& Q, u32* sc_ids, float* sc_d, int lane,
                                                  u32& nn, float& closest, u32& st_dist, u32& st_vup, u32& st_vl0,
                                                  u32& st_lup, u32& status, ReadCount& rc, u32 qi) {
  const u32 ep = A.g.ep;
  if (lane == 0) sc_ids[0] = ep;
  count_vec_reads<ACCT>(A, rc, lane == 0, ep, qi, true);
  wave_sync();
  dist_list<D, METRIC, E, ACCT == 2>(vec, Q, sc_ids, sc_d, 1, lane, &A.g);
  wave_sync();
  closest = sc_d[0];
  ++st_dist;
  if (A.g.ep_level > 0) ++st_vup; else ++st_vl0;
  nn = ep;
  const u32 MU = A.g.MU;
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
      count_vec_reads<ACCT>(A, rc, valid, e, qi, true);  // upper-level lists are replicated: only vectors can be remote
      wave_sync();
      dist_list<D, METRIC, E, ACCT == 2>(vec, Q, sc_ids, sc_d, cnt, lane, &A.g);
      wave_sync();
      // first neighbour (list order) attaining the minimum; adopted only if strictly closer (:378)
      float bd = (lane < cnt) ? sc_d[lane] : __builtin_inff();
      if (bd != bd) bd = __builtin_inff();  // NaN never compares less
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
}

// ------------------------------------------------------------------------------------------------------------
// search kernel: one wavefront (= one workgroup) per persistent slot
//   VIS   0: visited table in LDS, 1: visited bitmap in HBM
// ------------------------------------------------------------------------------------------------------------
// Phase stamps for the diagnostic (PROF) build: s_memtime with its lgkmcnt wait in one statement.
__device__ __forceinline__ u64 stamp() {
  u64 t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
template <bool PROF>
struct PhaseClock {  // empty unless PROF
  __device__ void start() {}
  __device__ void mark(int) {}
  __device__ void event(int) {}
  __device__ void flush(unsigned long long*, int) {}
};
template <>
struct PhaseClock<true> {  // lane i accumulates phase i: one compare and one 64-bit add per mark
  u64 acc = 0;
  u32 cnt = 0;
  u64 t_last = 0;
  int cur = 0;
  __device__ void start() { t_last = stamp(); }
  __device__ void mark(int i) {
    __builtin_amdgcn_sched_barrier(0);
    const u64 t = stamp();
    __builtin_amdgcn_sched_barrier(0);
    const int lane = static_cast<int>(threadIdx.x);
    if (lane == cur) acc += t - t_last;
    if (lane == i) ++cnt;
    t_last = t;
    cur = i;
  }
  __device__ void event(int i) {  // counts only (slots no phase uses)
    if (static_cast<int>(threadIdx.x) == i) ++cnt;
  }
  __device__ void flush(unsigned long long* out, int lane) {
    mark(0);
    if (out && lane < 12) {
      atomicAdd(&out[lane], static_cast<unsigned long long>(acc));
      atomicAdd(&out[12 + lane], static_cast<unsigned long long>(cnt));
    }
  }
};
#define PHASE(i) clk.mark(i);
#define EVENT(i) clk.event(i);

//   VIS   0: visited table in LDS; 1: visited bitmap in HBM; 2: visited bitmap and both heaps in HBM (the last
//         fallback pass: no capacity limit but the heap stride, ~µs per heap operation).  Heaps in HBM are
//         written by some lanes and read by others: a workgroup-scope fence orders every heap operation.
// ------------------------------------------------------------------------------------------------------------
// Exact visited set (hashset_t<RemotePtr>, types.hh:14-15) in the wave's LDS share (fast kernel; exact kernel VIS 0).
//   VT = 0: u32 keys, linear probing from a multiplicative hash (4 B per entry).
//   VT = 1: u16 quotient entries (2 B per entry): an odd multiply permutes the b-bit id space, the top t bits of
//           the image pick the home slot, and the entry keeps the other b - t bits plus the slot's distance from
//           home, so (slot, entry) names the id exactly.  Two entries share a 32-bit word; inserts are word-wide
//           compare-and-swaps whose first attempt assumes an empty word (one LDS round trip when it is).  Half the
//           LDS per wave lets two batches of 1,024 queries hold all their wavefronts on the CUs at once.  An id
//           that would land farther than 2^(16-(b-t)) - 2 slots from home stops the query (light pass re-runs it).
// ------------------------------------------------------------------------------------------------------------
template <int VT>
struct VisitedLds;

// VT = 0 tables hold any multiple of 64 entries: the home slot is the high word of hash x cap (v_mul_hi_u32), which for
// a power of two is the hash's top bits, the same slot as a shift; probing wraps at cap.  Large id spaces use that to
// size a table to its worst query without doubling it (100M ids at ef = 128: 6,144 entries, 6 wavefronts per CU,
// where 8,192 allow 4; capi.cc learned_max_table).
template <>
struct VisitedLds<0> {
  u32* t;
  u32 cap;
  __device__ __forceinline__ VisitedLds(void* base, const SearchArgs& A) : t(static_cast<u32*>(base)), cap(A.vis_cap) {}
  static constexpr u32 kBytes = 4;
  using Hint = u32;  // the id's home word
  static __device__ __forceinline__ Hint unknown() { return INV; }
  __device__ __forceinline__ u32 home(u32 x) const { return __umulhi(x * 0x9E3779B1u, cap); }
  __device__ __forceinline__ u32 next(u32 h) const { return h + 1 == cap ? 0u : h + 1; }
  __device__ __forceinline__ void clear(const SearchArgs& A, int lane) {
    uint4* t4 = reinterpret_cast<uint4*>(t);
    for (u32 i = lane; i < A.vis_cap / 4; i += 64) t4[i] = make_uint4(INV, INV, INV, INV);
  }
  __device__ __forceinline__ void insert_first(u32 x) { t[home(x)] = x; }  // the table is empty
  // f(x) for every id of the table (the entries are the ids themselves): the spill into HBM, and its release
  template <class F>
  __device__ __forceinline__ void for_each(F f, const SearchArgs& A, int lane) const {
    for (u32 i = lane; i < cap; i += 64) {
      const u32 x = t[i];
      if (x < A.g.N) f(x);
    }
  }
  __device__ __forceinline__ bool at_home(u32 x) const { return t[home(x)] == x; }
  // the word at x's home slot (one read); home_match: x sits at home in that word
  __device__ __forceinline__ u32 probe(u32 x) const { return t[home(x)]; }
  __device__ __forceinline__ bool home_match(u32 x, u32 w) const { return w == x; }
  // one exit from the probe loop (an early return per outcome compiles to a branchier loop and more live SGPRs).
  // hint: the home word as probe() read it since the last insert (INV: unknown), so a key found at home costs no
  // LDS operation and a home held by another key is skipped without a failed compare-and-swap
  __device__ __forceinline__ bool test_and_set(u32 x, bool& /*ovf*/, u32 hint = INV) {
    u32 h = home(x);
    bool fresh = false;
    if (hint == x) return false;
    if (hint != INV) h = next(h);  // slots are never freed: home still holds that other key
    for (;;) {
      const u32 old = atomicCAS(&t[h], INV, x);
      if (old == INV) {
        fresh = true;
        break;
      }
      if (old == x) break;
      h = next(h);
    }
    return fresh;
  }
};

template <>
struct VisitedLds<1> {
  u32* t;
  u32 bmask_b, mul, bmask, rbits, rmask, dbits, dmax;
  using Hint = uint4;  // a copy of the id's home bucket (4 words, 8 entries)
  __device__ __forceinline__ VisitedLds(void* base, const SearchArgs& A) : t(static_cast<u32*>(base)), mul(A.vis_mul) {
    const u32 tb = 31 - __clz(static_cast<int>(A.vis_cap >> 3));  // buckets of 8 entries
    bmask_b = (A.vis_cap >> 3) - 1;
    bmask = A.vis_bits >= 32 ? ~0u : (1u << A.vis_bits) - 1;
    rbits = A.vis_bits - tb;
    rmask = (1u << rbits) - 1;
    dbits = 16 - rbits;
    dmax = (1u << dbits) - 2;  // an all-ones entry is the empty marker
  }
  static constexpr u32 kBytes = 2;
  // not read yet: assume an empty bucket (a wrong guess costs one failed compare-and-swap and a read)
  static __device__ __forceinline__ Hint unknown() { return make_uint4(INV, INV, INV, INV); }
  __device__ __forceinline__ void clear(const SearchArgs& A, int lane) {
    uint4* t4 = reinterpret_cast<uint4*>(t);
    for (u32 i = lane; i < A.vis_cap / 8; i += 64) t4[i] = make_uint4(INV, INV, INV, INV);
  }
  __device__ __forceinline__ u32 image(u32 x) const { return (x * mul) & bmask; }
  // f(x) for every id of the table: entry (bucket b, remainder, distance d) names the id whose image is
  // ((b - d) << rbits) | remainder, and the inverse multiply maps the image back
  template <class F>
  __device__ __forceinline__ void for_each(F f, const SearchArgs& A, int lane) const {
    const u32 nw = A.vis_cap >> 1;  // two entries per word
    for (u32 i = lane; i < nw; i += 64) {
      const u32 w = t[i], b = i >> 2;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const u32 v = half ? (w >> 16) : (w & 0xFFFFu);
        if (v == 0xFFFFu) continue;
        const u32 home = (b - (v & ((1u << dbits) - 1u))) & bmask_b;
        const u32 x = (((home << rbits) | (v >> dbits)) * A.vis_mul_inv) & bmask;
        if (x < A.g.N) f(x);
      }
    }
  }
  __device__ __forceinline__ void insert_first(u32 x) {  // the table is empty: entry 0 of the home bucket
    const u32 h = image(x);
    t[(h >> rbits) * 4] = 0xFFFF0000u | ((h & rmask) << dbits);
  }
  __device__ __forceinline__ uint4 bucket(u32 b) const { return reinterpret_cast<const uint4*>(t)[b]; }
  // Branch-free bucket tests on both 16-bit halves of a word at once (SWAR): zero16(x) is non-zero iff a half of x
  // is zero (a borrow can flag the high half spuriously only when the low half is zero, so "any half" is exact).
  // Written with `|`, not `||`: short-circuit tests compiled to a cascade of exec-mask branches per entry.
  static __device__ __forceinline__ u32 zero16(u32 x) { return (x - 0x00010001u) & ~x & 0x80008000u; }
  static __device__ __forceinline__ bool has(u32 w, u32 e) { return zero16(w ^ (e * 0x00010001u)) != 0u; }
  static __device__ __forceinline__ bool has(const uint4& w, u32 e) {
    const u32 ee = e * 0x00010001u;
    return (zero16(w.x ^ ee) | zero16(w.y ^ ee) | zero16(w.z ^ ee) | zero16(w.w ^ ee)) != 0u;
  }
  // the bucket's first empty entry (0xFFFF) in bucket order: word j (-1: none) and half k (0 low, 1 high)
  static __device__ __forceinline__ void first_empty(const uint4& w, int& j, u32& k, u32& word) {
    const bool e0 = zero16(~w.x) != 0u, e1 = zero16(~w.y) != 0u, e2 = zero16(~w.z) != 0u, e3 = zero16(~w.w) != 0u;
    j = e0 ? 0 : e1 ? 1 : e2 ? 2 : e3 ? 3 : -1;
    word = e0 ? w.x : e1 ? w.y : e2 ? w.z : w.w;
    k = (word & 0xFFFFu) == 0xFFFFu ? 0u : 1u;
  }
  // the home bucket (one ds_read_b128); home_match: x sits in it
  __device__ __forceinline__ Hint probe(u32 x) const { return bucket(image(x) >> rbits); }
  __device__ __forceinline__ bool home_match(u32 x, const Hint& w) const {
    const u32 h = image(x);
    return has(w, (h & rmask) << dbits);
  }
  // The common case of test_and_set when `cur` IS x's home bucket as it stands (the look-ahead probe, no insert
  // since): the answer follows from `cur` alone — x sits in it (0), or the bucket has an empty entry, so x is absent
  // and fresh (1) — and the compare-and-swap recording x is issued without waiting for it (word pw, expected pexp,
  // its return in pold); finish() checks it after the distances.  2: a full bucket, use test_and_set.
  __device__ __forceinline__ int begin(u32 x, const Hint& cur, u32& pw, u32& pexp, u32& pold) {
    const u32 h = image(x);
    const u32 e = (h & rmask) << dbits;
    if (has(cur, e)) return 0;
    int j;
    u32 k;
    first_empty(cur, j, k, pexp);
    if (j < 0) return 2;
    pw = (h >> rbits) * 4 + static_cast<u32>(j);
    pold = atomicCAS(&t[pw], pexp, k ? ((pexp & 0xFFFFu) | (e << 16)) : ((pexp & 0xFFFF0000u) | e));
    return 1;
  }
  // another lane of the wave took that word first (two list entries, one home bucket): x is still absent and is
  // inserted again from its home bucket as it is now
  __device__ __forceinline__ void finish(u32 x, u32 pexp, u32 pold, bool& ovf) {
    if (pold != pexp) (void)test_and_set(x, ovf, bucket(image(x) >> rbits));
  }
  // Buckets of 8 entries, probed linearly: x's entry (its remainder and its bucket's distance from home) is looked for
  // in one bucket read at a time and goes to the bucket's first empty entry.  Entries are never removed, so a bucket
  // with an empty entry ends the search.  cur: the home bucket as last read (probe) or unknown().
  __device__ __forceinline__ bool test_and_set(u32 x, bool& ovf, Hint cur = unknown()) {
    const u32 h = image(x);
    u32 b = h >> rbits, disp = 0;
    const u32 rem = (h & rmask) << dbits;
    bool fresh = false;
    for (;;) {
      const u32 e = rem | disp;
      if (has(cur, e)) break;  // same bucket distance, same remainder: this id
      // first empty entry in bucket order: word j, high half k
      int j;
      u32 k, old_w;
      first_empty(cur, j, k, old_w);
      if (j >= 0) {
        const u32 want = k ? ((old_w & 0xFFFFu) | (e << 16)) : ((old_w & 0xFFFF0000u) | e);
        if (atomicCAS(&t[b * 4 + static_cast<u32>(j)], old_w, want) == old_w) {
          fresh = true;
          break;
        }
        cur = bucket(b);  // the bucket changed under us (or was not as guessed): read it
        continue;
      }
      b = (b + 1) & bmask_b;  // full bucket: the next one
      if (++disp > dmax) {
        ovf = true;
        break;
      }
      cur = bucket(b);
    }
    return fresh;
  }
};

// VT = 2: u16 entries in two-choice buckets, for id spaces too wide for VT = 1's distance bits (up to 2^(log2(cap) +
// 12) ids: 4,096 entries in 8 KiB at 24-bit ids, where VT = 1 needs 16,384).  The odd multiply permutes the b-bit id
// space; the top t bits of the image pick bucket b1, the other r = b - t <= 15 bits (the remainder) are stored with one
// bit naming the bucket the entry went to: b1, or b2 = b1 ^ alt(remainder), the less filled of the two when the id was
// inserted (b1 on a tie).  Entries fill a bucket in order and are never removed, so an id in b2 implies that b1 held an
// entry when it went there: a bucket b1 found empty answers "absent" alone.  The all-ones entry is the empty marker:
// at r = 15 the remainder 0x7FFF only ever goes to b1.  A lookup reads both buckets (two ds_read_b128 in flight
// together); both full is an overflow, and the query spills in place.  The look-ahead probe keeps no bucket copies
// (8 VGPRs live across the merge): it keeps the insert it would make, as three words — the word to swap (or "present"
// / "both full"), its expected value and its new value.
struct Plan2 {
  u32 pw, pexp, pnew;  // pw: the word to compare-and-swap, or kPresent / kFull / INV (not planned)
};
template <>
struct VisitedLds<2> {
  static constexpr u32 kPresent = 0xFFFFFFFEu, kFull = 0xFFFFFFFDu;
  u32* t;
  u32 bmask_b, mul, bmask, rbits, rmask, tb;
  using Hint = Plan2;
  __device__ __forceinline__ VisitedLds(void* base, const SearchArgs& A) : t(static_cast<u32*>(base)), mul(A.vis_mul) {
    tb = 31 - __clz(static_cast<int>(A.vis_cap >> 3));  // buckets of 8 entries
    bmask_b = (A.vis_cap >> 3) - 1;
    bmask = A.vis_bits >= 32 ? ~0u : (1u << A.vis_bits) - 1;
    rbits = A.vis_bits - tb;
    rmask = (1u << rbits) - 1;
  }
  static constexpr u32 kBytes = 2;
  static __device__ __forceinline__ Hint unknown() { return Plan2{INV, 0u, 0u}; }
  __device__ __forceinline__ void clear(const SearchArgs& A, int lane) {
    uint4* t4 = reinterpret_cast<uint4*>(t);
    for (u32 i = lane; i < A.vis_cap / 8; i += 64) t4[i] = make_uint4(INV, INV, INV, INV);
  }
  __device__ __forceinline__ u32 image(u32 x) const { return (x * mul) & bmask; }
  __device__ __forceinline__ u32 alt(u32 rem) const { return ((rem * 0x85EBCA6Bu) >> (32 - tb)) | 1u; }
  __device__ __forceinline__ u32 decode(u32 b, u32 v, const SearchArgs& A) const {
    const u32 rem = v >> 1;
    const u32 b1 = (v & 1u) ? (b ^ alt(rem)) & bmask_b : b;
    return (((b1 << rbits) | rem) * A.vis_mul_inv) & bmask;
  }
  template <class F>
  __device__ __forceinline__ void for_each(F f, const SearchArgs& A, int lane) const {
    const u32 nw = A.vis_cap >> 1;
    for (u32 i = lane; i < nw; i += 64) {
      const u32 w = t[i], b = i >> 2;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const u32 v = half ? (w >> 16) : (w & 0xFFFFu);
        if (v == 0xFFFFu) continue;
        const u32 x = decode(b, v, A);
        if (x < A.g.N) f(x);
      }
    }
  }
  __device__ __forceinline__ void insert_first(u32 x) {  // the table is empty: entry 0 of b1
    const u32 h = image(x);
    t[(h >> rbits) * 4] = 0xFFFF0000u | ((h & rmask) << 1);
  }
  __device__ __forceinline__ uint4 bucket(u32 b) const { return reinterpret_cast<const uint4*>(t)[b]; }
  // entries in a bucket (they fill it in order): 2 x the first word with an empty half, + 1 if its low half is taken
  static __device__ __forceinline__ u32 fill(const uint4& w) {
    int j;
    u32 k, word;
    VisitedLds<1>::first_empty(w, j, k, word);
    return j < 0 ? 8u : 2u * static_cast<u32>(j) + k;
  }
  // x against both buckets as they stand: present, both full, or the insert (the less filled bucket's first empty
  // entry) as a compare-and-swap to make
  __device__ __forceinline__ Hint probe(u32 x) const {
    const u32 h = image(x), rem = h & rmask, b1 = h >> rbits, b2 = (b1 ^ alt(rem)) & bmask_b;
    const uint4 w1 = bucket(b1), w2 = bucket(b2);
    const u32 e = rem << 1;
    // rem 0x7FFF never goes to b2 (its b2 entry would be the empty marker 0xFFFF, which any bucket with a free entry
    // "holds"): only b1 is looked at for it
    const bool in2 = rem != 0x7FFFu && VisitedLds<1>::has(w2, e | 1u);
    if (VisitedLds<1>::has(w1, e) || in2) return Plan2{kPresent, 0u, 0u};
    // each bucket's first empty entry once: its position is the bucket's fill (entries fill in order)
    int j1, j2;
    u32 k1, k2, o1, o2;
    VisitedLds<1>::first_empty(w1, j1, k1, o1);
    VisitedLds<1>::first_empty(w2, j2, k2, o2);
    const u32 f1 = j1 < 0 ? 8u : 2u * static_cast<u32>(j1) + k1, f2 = j2 < 0 ? 8u : 2u * static_cast<u32>(j2) + k2;
    const bool second = f2 < f1 && rem != 0x7FFFu;
    const int j = second ? j2 : j1;
    const u32 k = second ? k2 : k1, old = second ? o2 : o1;
    if (j < 0) return Plan2{kFull, 0u, 0u};
    const u32 ent = second ? (e | 1u) : e;
    return Plan2{(second ? b2 : b1) * 4 + static_cast<u32>(j), old,
                 k ? ((old & 0xFFFFu) | (ent << 16)) : ((old & 0xFFFF0000u) | ent)};
  }
  __device__ __forceinline__ bool home_match(u32 /*x*/, const Hint& p) const { return p.pw == kPresent; }
  // as VisitedLds<1>::begin, from the look-ahead probe's plan: 0 = present, 1 = compare-and-swap issued, 2 = both full
  __device__ __forceinline__ int begin(u32 /*x*/, const Hint& p, u32& pw, u32& pexp, u32& pold) {
    if (p.pw == kPresent) return 0;
    if (p.pw >= kFull) return 2;
    pw = p.pw;
    pexp = p.pexp;
    pold = atomicCAS(&t[pw], p.pexp, p.pnew);
    return 1;
  }
  __device__ __forceinline__ void finish(u32 x, u32 pexp, u32 pold, bool& ovf) {
    if (pold != pexp) (void)test_and_set(x, ovf, probe(x));
  }
  // p: a plan made since the last insert, or unknown() — then the guess that b1 is empty (its word 0 swapped from
  // all-empty: when that holds, x is in neither bucket), read and planned again when it fails
  __device__ __forceinline__ bool test_and_set(u32 x, bool& ovf, Hint p = unknown()) {
    if (p.pw == INV) {
      const u32 h = image(x);
      p = Plan2{(h >> rbits) * 4, INV, 0xFFFF0000u | ((h & rmask) << 1)};
    }
    for (;;) {
      if (p.pw == kPresent) return false;
      if (p.pw == kFull) {
        ovf = true;
        return false;
      }
      if (atomicCAS(&t[p.pw], p.pexp, p.pnew) == p.pexp) return true;
      p = probe(x);  // a word changed under us (or was not as guessed): read both buckets again
    }
  }
};

// VT = 3: u32 keys in two-choice buckets of 4 (16 bytes), for id spaces too wide for the u16 entries (26-27-bit ids:
// cfg 4's 100M, cfg 5's 50M records), where the linear-probed VT = 0 table needs a load of ~0.45 to keep its probe
// chains short: the wave's 32 list slots walk their chains in lockstep, so an expansion waits for its longest chain
// (DESIGN §4, round 5).  An id goes to the less filled of its two buckets b1, b2 (two multiplicative hashes; b1 on a
// tie), at the bucket's first empty word; when both are full, to the first bucket after b2 (wrapping) with an empty
// word.  Buckets fill in order and never empty, so a lookup reads b1 and b2 (two ds_read_b128 in flight together): the
// id in either, or an empty word in either (then the id is absent: it would have gone there), answers it; only when
// both are full does it walk on from b2 (rare below a load of ~0.6).  An id sits in b2 or beyond only if b1 held an
// entry then, so a guessed swap into an empty b1's word 0 that succeeds proves the id absent.  The lookup plans the
// insert (word, INV, id): an insert is one read and one compare-and-swap round trip in the common case, whatever the
// load, so the table runs fuller than the linear-probed one and more wavefronts share a CU.  A walk past kMaxWalk
// buckets is an overflow (the query spills in place).  Any multiple of 4 entries (homes by umulhi).
template <>
struct VisitedLds<3> {
  static constexpr u32 kPresent = 0xFFFFFFFEu, kFull = 0xFFFFFFFDu, kMaxWalk = 64;
  u32* t;
  u32 nb;
  using Hint = Plan2;
  __device__ __forceinline__ VisitedLds(void* base, const SearchArgs& A) : t(static_cast<u32*>(base)), nb(A.vis_cap >> 2) {}
  static constexpr u32 kBytes = 4;
  static __device__ __forceinline__ Hint unknown() { return Plan2{INV, 0u, 0u}; }
  __device__ __forceinline__ void clear(const SearchArgs& A, int lane) {
    uint4* t4 = reinterpret_cast<uint4*>(t);
    for (u32 i = lane; i < A.vis_cap / 4; i += 64) t4[i] = make_uint4(INV, INV, INV, INV);
  }
  __device__ __forceinline__ u32 b1(u32 x) const { return __umulhi(x * 0x9E3779B1u, nb); }
  __device__ __forceinline__ u32 b2(u32 x) const { return __umulhi(x * 0x85EBCA77u, nb); }
  template <class F>
  __device__ __forceinline__ void for_each(F f, const SearchArgs& A, int lane) const {
    for (u32 i = lane; i < A.vis_cap; i += 64) {
      const u32 x = t[i];
      if (x < A.g.N) f(x);
    }
  }
  __device__ __forceinline__ void insert_first(u32 x) { t[b1(x) * 4] = x; }
  __device__ __forceinline__ uint4 bucket(u32 b) const { return reinterpret_cast<const uint4*>(t)[b]; }
  // words in a bucket (they fill in order): the first empty word's index, 4 when full
  static __device__ __forceinline__ u32 fill(const uint4& w) {
    return w.x == INV ? 0u : w.y == INV ? 1u : w.z == INV ? 2u : w.w == INV ? 3u : 4u;
  }
  // (written with `|`: short-circuit tests compile to a cascade of exec-mask branches)
  static __device__ __forceinline__ bool has(const uint4& w, u32 x) {
    return (w.x == x) | (w.y == x) | (w.z == x) | (w.w == x);
  }
  __device__ __forceinline__ Hint probe(u32 x) const {
    const u32 h1 = b1(x), h2 = b2(x);
    const uint4 w1 = bucket(h1), w2 = bucket(h2);
    if (static_cast<int>(has(w1, x)) | static_cast<int>(has(w2, x))) return Plan2{kPresent, 0u, 0u};
    const u32 f1 = fill(w1), f2 = fill(w2);
    const bool second = f2 < f1;
    const u32 f = second ? f2 : f1;
    Plan2 p{(second ? h2 : h1) * 4 + f, INV, x};
    if (f >= 4u) {  // both full: the overflow walk from b2 on (one loop exit; see the probe loops above)
      p.pw = kFull;
      u32 b = h2;
      for (u32 i = 0; i < kMaxWalk; ++i) {
        b = b + 1 == nb ? 0u : b + 1;
        const uint4 w = bucket(b);
        if (has(w, x)) {
          p.pw = kPresent;
          break;
        }
        const u32 fb = fill(w);
        if (fb < 4u) {
          p.pw = b * 4 + fb;
          break;
        }
      }
    }
    return p;
  }
  __device__ __forceinline__ bool home_match(u32 /*x*/, const Hint& p) const { return p.pw == kPresent; }
  __device__ __forceinline__ int begin(u32 /*x*/, const Hint& p, u32& pw, u32& pexp, u32& pold) {
    if (p.pw == kPresent) return 0;
    if (p.pw >= kFull) return 2;
    pw = p.pw;
    pexp = p.pexp;
    pold = atomicCAS(&t[pw], p.pexp, p.pnew);
    return 1;
  }
  __device__ __forceinline__ void finish(u32 x, u32 pexp, u32 pold, bool& ovf) {
    if (pold != pexp) (void)test_and_set(x, ovf, probe(x));
  }
  __device__ __forceinline__ bool test_and_set(u32 x, bool& ovf, Hint p = unknown()) {
    if (p.pw == INV) p = Plan2{b1(x) * 4, INV, x};
    for (;;) {
      if (p.pw == kPresent) return false;
      if (p.pw == kFull) {
        ovf = true;
        return false;
      }
      if (atomicCAS(&t[p.pw], p.pexp, p.pnew) == p.pexp) return true;
      p = probe(x);  // a word changed under us (or was not as guessed): read the buckets again
    }
  }
};

// End of the last pass of a call: the last workgroup to finish publishes the queries every pass handed on (host
// memory: the next call sizes its light pass from them, shine_knn_batch reports them) and zeroes the call's counter
// words for the next call on this stream, so a call needs neither a memset nor a copy of its own.  No fence is
// needed: a workgroup counts itself finished only after the atomic that found the work queue empty has returned,
// the hand-on counts were final before this pass started, and the end-of-kernel release publishes the stores to
// the next kernel on the stream and to the host.  (An agent-scope fence per workgroup would write back L2 on every
// exit: -3 % QPS measured.)
__device__ __forceinline__ void finish_call(const SearchArgs& A, int lane) {
  if (!A.call_counters || lane != 0) return;
  u32* c = A.call_counters;
  if (atomicAdd(&c[7], 1u) != gridDim.x - 1) return;
  const u32 h0 = __atomic_load_n(&c[4], __ATOMIC_RELAXED), h1 = __atomic_load_n(&c[5], __ATOMIC_RELAXED),
            h2 = __atomic_load_n(&c[6], __ATOMIC_RELAXED);
  volatile u32* host = A.host_counts;
  host[0] = h0;
  host[1] = h1;
  host[2] = h2;
  host[4] = __atomic_load_n(&c[3], __ATOMIC_RELAXED);
  host[5] = __atomic_load_n(&c[8], __ATOMIC_RELAXED);
  host[6] = A.nq;  // the call the sum belongs to (several calls may be in flight on the stream)
  host[7] = __atomic_load_n(&c[9], __ATOMIC_RELAXED);
  host[8] = __atomic_load_n(&c[10], __ATOMIC_RELAXED);
  host[3] = 1u;
  if (A.call_out) {
    volatile u32* co = A.call_out;
    co[0] = h0 + h1 + h2;
    co[1] = 1u;
  }
#pragma unroll
  for (int i = 0; i < static_cast<int>(kCallWords); ++i) __atomic_store_n(&c[i], 0u, __ATOMIC_RELAXED);
}

// One of the stream's spill bitmaps for this wavefront (SearchArgs::spill_flags), or -1 when all are held.
__device__ __forceinline__ int claim_spill_bitmap(const SearchArgs& A, int lane) {
  if (A.spill_slots == 0) return -1;
  u32 got = INV;
  if (lane == 0) {
    if (A.spill_count) atomicAdd(A.spill_count, 1u);
    const u32 n = A.spill_slots;
    for (u32 i = 0, j = blockIdx.x % n; i < n; ++i, j = j + 1 == n ? 0u : j + 1)
      if (atomicCAS(&A.spill_flags[j], 0u, 1u) == 0u) {
        got = j;
        break;
      }
  }
  got = bcast(got);
  return got == INV ? -1 : static_cast<int>(got);
}

// Every bit a query sets in its spill bitmap after the spill is logged in the bitmap's vlog row (SearchArgs::vlog, free
// while the main pass runs: only the fallback passes use it, later on the stream), so that handing the bitmap back
// zeroes the table's ids and the logged ones only — O(visited) instead of the whole id space (12.5 MB per spilled query
// at 100M ids).  A log past log_cap falls back to zeroing every word.
__device__ __forceinline__ void spill_log(const SearchArgs& A, int sslot, u32& n, bool active, u32 id, int lane) {
  const u64 m = __ballot(active);
  if (!m) return;
  const u64 below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if (active) {
    const u32 pos = n + static_cast<u32>(__popcll(m & below));
    if (pos < A.log_cap) A.vlog[static_cast<u64>(sslot) * A.log_cap + pos] = id;
  }
  n += static_cast<u32>(__popcll(m));
}

// The visited set of a query whose LDS table overflowed (in-place spill): slot `sslot` of the stream's spill storage
// (SearchArgs::visited, words_per_slot words each, all zero between uses), used one of two ways.
//   * a bitmap over the id space (spill_hash == 0): one atomicOr per visit.  Cheap while the bitmap stays in an XCD's
//     L2 (1.25 MB at 10M ids); at 100M ids it is 12.5 MB, every visit of a spilled query missed to HBM, and the few
//     queries that spilled (0.3 %) set their batches' times: 2.37 M against 3.41 M QPS with tables twice the size
//     that never spill (profiles/r04/diag100m_tables_inflight.jsonl).
//   * an open-addressing hash table of spill_hash entries (a power of two, load kept <= 1/2) in the slot's first words
//     (spill_hash > 0): entry id + 1, 0 = empty (so the slot is all zero between uses, as the fallback passes' bitmaps
//     must be), linear probing from the multiplicative hash's top bits, one compare-and-swap per probe.  128 KB at
//     32,768 entries: it stays in L2 for the few queries that spill, whatever the id space.  The whole LDS table moves
//     in at the spill and every later visit of the query goes there (a lookup walking the frozen LDS table first was
//     40 % slower at cfg 3, profiles/r04/scale_cfg3_cfg5_10m_v3_hashspill_reverted.jsonl).
struct SpillSet {
  u32* p = nullptr;
  u32 hmask = 0, hshift = 0;  // hash entries - 1 and 32 - log2(entries); hmask == 0: bitmap
  __device__ __forceinline__ SpillSet() {}
  __device__ __forceinline__ SpillSet(const SearchArgs& A, int sslot)
      : p(A.visited + static_cast<u64>(sslot) * A.words_per_slot),
        hmask(A.spill_hash ? A.spill_hash - 1u : 0u),
        hshift(A.spill_hash ? static_cast<u32>(__clz(static_cast<int>(A.spill_hash))) + 1u : 0u) {}
  __device__ __forceinline__ bool hashed() const { return hmask != 0u; }
  // x recorded; true when it was not yet (ovf: a probe chain of 64, the query is handed on)
  __device__ __forceinline__ bool test_and_set(u32 x, bool& ovf) const {
    if (!hashed()) {
      const u32 bit = 1u << (x & 31);
      return (atomicOr(&p[x >> 5], bit) & bit) == 0u;
    }
    const u32 v = x + 1u;
    u32 h = (x * 0x9E3779B1u) >> hshift;
    bool fresh = false;
    for (u32 n = 0;; ++n) {  // one loop exit (see the probe loops above)
      const u32 old = atomicCAS(&p[h], 0u, v);
      if (old == 0u) {
        fresh = true;
        break;
      }
      if (old == v) break;
      if (n == 63) {
        ovf = true;
        break;
      }
      h = (h + 1u) & hmask;
    }
    return fresh;
  }
  __device__ __forceinline__ void set(u32 x) const {
    bool ovf = false;
    (void)test_and_set(x, ovf);
  }
};

// Hand the spill slot back all zero, then drop its flag (every lane stores the same flag word: see the fast kernel).
// Bitmap: the table's ids and the logged ones (spill_log); hash table: its words.
template <class VTab>
__device__ __forceinline__ void spill_release(const VTab& vt, const SearchArgs& A, int sslot, u32 n, int lane) {
  const SpillSet ss(A, sslot);
  u32* sb = ss.p;
  if (ss.hashed()) {
    uint4* s4 = reinterpret_cast<uint4*>(sb);
    for (u32 i = lane; i <= (ss.hmask >> 2); i += 64) s4[i] = make_uint4(0u, 0u, 0u, 0u);
  } else if (n > A.log_cap) {
    for (u64 w = lane; w < A.words_per_slot; w += 64) sb[w] = 0u;
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the log's stores, before its loads
    vt.for_each([sb](u32 x) { sb[x >> 5] = 0u; }, A, lane);
    const u32* lg = A.vlog + static_cast<u64>(sslot) * A.log_cap;
    for (u32 i = lane; i < n; i += 64) sb[__hip_atomic_load(&lg[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 5] = 0u;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __threadfence();
  __hip_atomic_store(&A.spill_flags[sslot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Move the LDS table into the spill slot (every id of it recorded there).
template <class VTab>
__device__ __forceinline__ void spill_table(const VTab& vt, const SpillSet& ss, const SearchArgs& A, int lane) {
  if (ss.hashed()) {
    const SpillSet s2 = ss;
    vt.for_each([s2](u32 x) { s2.set(x); }, A, lane);
  } else {
    u32* sb = ss.p;
    vt.for_each([sb](u32 x) { atomicOr(&sb[x >> 5], 1u << (x & 31)); }, A, lane);
  }
}

template <int D, int METRIC, typename E, int VIS, int ACCT, int VT = 0, bool PROF = false>
__global__ __launch_bounds__(64) void search_kernel(SearchArgs A) {
  PhaseClock<PROF> clk;
  clk.start();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ef = static_cast<int>(A.ef), cap = static_cast<int>(A.cap);
  const size_t top_b = align16(8ull * ef), next_b = align16(8ull * cap);
  u64* const gheap = VIS == 2 ? reinterpret_cast<u64*>(A.heaps) + static_cast<u64>(blockIdx.x) * A.heap_stride
                              : nullptr;
  u64* top = VIS == 2 ? gheap : reinterpret_cast<u64*>(smem);                   // MaxHeap top_candidates
  u64* nxt = VIS == 2 ? gheap + top_b / 8 : reinterpret_cast<u64*>(smem + top_b);  // MinHeap next_candidates
  unsigned char* vbase = VIS == 2 ? smem : smem + top_b + next_b;  // visited table (VIS = 0)
  VisitedLds<VT> vt(vbase, A);
  u32* sc_ids = reinterpret_cast<u32*>(vbase + (VIS == 0 ? A.vis_cap * VisitedLds<VT>::kBytes : 0u));  // fresh ids
  float* sc_d = reinterpret_cast<float*>(sc_ids + 64);
  auto hfence = []() {
    if constexpr (VIS == 2) __threadfence_block();
  };

  const int lane = threadIdx.x;
  const PopLane pl(lane);
  const E* __restrict__ vec = static_cast<const E*>(A.g.vec);
  const u32 M0 = A.g.M0;
  u32* __restrict__ vis = A.visited + (VIS >= 1 ? static_cast<u64>(blockIdx.x) * A.words_per_slot : 0ull);
  u32* __restrict__ vlog = A.vlog + (VIS >= 1 ? static_cast<u64>(blockIdx.x) * A.log_cap : 0ull);
  const u64 below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // lanes < this one

  const u32 n_items = A.in_count ? *A.in_count : A.nq;
  for (;;) {
    u32 item = 0;
    if (lane == 0) item = atomicAdd(A.counter, 1u);
    item = bcast(item);
    if (item >= n_items) break;
    const u32 qi = A.in_list ? A.in_list[item] : item;

    PHASE(0)
    QueryRegs<D, E> Q;
    load_query<D, E>(A.queries + static_cast<u64>(qi) * D, lane, Q);
    if (VIS == 0) vt.clear(A, lane);  // visited_nodes.clear()  (:475) — done up front for this query

    u32 st_dist = 0, st_vup = 0, st_vl0 = 0, st_lup = 0, st_ll0 = 0, st_maxnext = 0, status = 0;
    ReadCount rc;
    int sslot = -1;  // VIS == 0: the spill bitmap this query holds (wave-uniform), -1 = the LDS table
    u32 slog = 0;    // ids logged since the spill (spill_log)

    // ---- entry point + greedy descent (hnsw.hh:256-287) ---------------------------------------------------
    PHASE(1)
    u32 nn;
    float closest;
    entry_and_descent<D, METRIC, E, ACCT>(A, vec, Q, sc_ids, sc_d, lane, nn, closest, st_dist, st_vup, st_vl0, st_lup, status,
                                    rc, qi);

    // ---- top_candidates.push({nn, dist(q, nn)}) (hnsw.hh:285-286) ---------------------------------------
    ++st_dist;
    int ntop = 1, nnext = 1;
    u32 logpos = 0, nvis = 1;
    bool log_overflow = false;
    if (status == 0) {
      u64 troot = mk(closest, nn), nroot = troot;  // roots of top / next, kept in SGPRs
      bool nan_keys = closest != closest;            // a NaN key in either heap: general pop from now on
      if (lane == 0) {
        top[0] = troot;
        nxt[0] = troot;  // search_level :412-415
        if (VIS == 0) {
          vt.insert_first(nn);  // table is empty: the first probe slot is free
        } else {
          atomicOr(&vis[nn >> 5], 1u << (nn & 31));
          vlog[0] = nn;
        }
      }
      logpos = 1;
      st_maxnext = 1;
      hfence();
      wave_sync();

      u32 pre_id = INV;  // candidate whose adjacency row is in flight in pre_e
      u32 pre_e = INV;

      // ---- search_level(q, ef, 0) (hnsw.hh:406-476) ---------------------------------------------------------
      while (nnext > 0) {
        PHASE(2)
        const float ck = key(nroot), farthest0 = key(troot);  // next_candidates.top(); pop()  (:418-421)
        const u32 cid = eid(nroot);
        nroot = nan_keys ? heap_pop_any<false>(nxt, nnext, lane) : heap_pop<false>(nxt, nnext, lane, pl);
        hfence();
        --nnext;
        if (ck > farthest0) break;  // :421-426
        if (cid >= A.g.N) {  // a heap entry that is not a record: report it, never dereference it
          status = ST_FORMAT;
          break;
        }

        // neighbour list of the candidate at level 0 (:436-438)
        PHASE(3)
        ++st_ll0;
        count_list_read<ACCT>(A, rc, cid, lane);
        u32 e = INV;
        if (cid == pre_id) {
          e = pre_e;
        } else if (static_cast<u32>(lane) < M0) {
          e = A.g.adj0[static_cast<u64>(cid) * M0 + lane];
        }
        bool cand = e != INV;
        if (!A.g.lists_unique) {  // first occurrence in list order wins (visited.insert order, :443)
          for (u32 j = 0; j < M0; ++j) {
            const u32 ej = __shfl(e, static_cast<int>(j));
            if (j < static_cast<u32>(lane) && ej == e) cand = false;
          }
        }
        bool fresh = false, vovf = false;
        if (cand) {  // visited.contains / insert (:441-443)
          if (VIS == 0 && sslot < 0) {
            // the home word / bucket read first (every candidate lane's read in flight together): a visited id is
            // then answered in one LDS round trip and a fresh one swapped in two, where a blind swap assuming an
            // empty home costs an extra failed round trip once the table has filled
            fresh = vt.test_and_set(e, vovf, vt.probe(e));
          } else if (VIS == 0) {  // this query's spilled table: the HBM bitmap or hash table (SpillSet)
            fresh = SpillSet(A, sslot).test_and_set(e, vovf);
          } else {  // the fallback passes' HBM bitmap
            const u32 bit = 1u << (e & 31);
            fresh = (atomicOr(&vis[e >> 5], bit) & bit) == 0;
          }
        }
        if (VIS == 0 && sslot >= 0) {
          if (!SpillSet(A, sslot).hashed()) {
            spill_log(A, sslot, slog, fresh, e, lane);
          } else if (__ballot(vovf) || nvis + __popcll(__ballot(fresh)) > A.spill_hash / 2) {
            status = ST_OVERFLOW;  // the hash table is half full: the query is handed on to the light pass
            break;
          }
        }
        if constexpr (VIS == 0) {
          // In-place spill (as the fast kernel): the table is too full, or an id landed too far from its home
          // bucket — the table moves to an HBM bitmap and the query goes on there instead of being handed to the
          // light pass and re-run from scratch.  An insert that overflowed is tested against the bitmap.
          if (sslot < 0 && (__ballot(vovf) || nvis + __popcll(__ballot(fresh)) > A.vis_limit)) {
            sslot = claim_spill_bitmap(A, lane);
            if (sslot < 0) {
              status = ST_OVERFLOW;
              break;
            }
            const SpillSet ss(A, sslot);
            wave_sync();
            spill_table(vt, ss, A, lane);
            EVENT(3)
            bool hovf = false;
            if (vovf) fresh = ss.test_and_set(e, hovf);
            if (!ss.hashed()) spill_log(A, sslot, slog, vovf, e, lane);
            if (__ballot(hovf)) {
              status = ST_OVERFLOW;
              break;
            }
          }
        }
        const u64 fm = __ballot(fresh);
        const int nf = __popcll(fm);
        count_vec_reads<ACCT>(A, rc, fresh, e, qi);
        if (fresh) {
          const int r = __popcll(fm & below);
          sc_ids[r] = e;
          if (VIS >= 1) {
            const u32 lp = logpos + r;
            if (lp < A.log_cap) vlog[lp] = e;
          }
        }
        logpos += nf;
        nvis += nf;
        if (VIS >= 1 && logpos > A.log_cap) log_overflow = true;
        st_vl0 += nf;
        st_dist += nf;
        if (nf == 0) continue;
        PHASE(4)
        wave_sync();
        dist_list<D, METRIC, E, ACCT == 2>(vec, Q, sc_ids, sc_d, nf, lane, &A.g);
        wave_sync();
        PHASE(5)
        // lane j < nf holds fresh neighbour j (list order)
        const float my_d = lane < nf ? sc_d[lane] : __builtin_inff();
        const u32 my_id = lane < nf ? sc_ids[lane] : INV;
        if (__ballot(my_d != my_d)) nan_keys = true;

        // Speculative prefetch of the adjacency row of the candidate expected on top of next_candidates once
        // this step's pushes are done: a min-heap root changes only for a strictly smaller key, so the root
        // survives ties and, among the fresh keys, the first minimum in list order wins.
        {
          const float pd_l = (lane < nf && (my_d < farthest0 || ntop < ef) && my_d == my_d) ? my_d : __builtin_inff();
          const float pd = wave_min(pd_l);
          u32 pid = INV;
          if (nnext > 0 && !(pd < key(nroot))) {
            pid = eid(nroot);
          } else if (pd < __builtin_inff()) {
            const u64 hit = __ballot(pd_l == pd);
            pid = __builtin_amdgcn_readlane(static_cast<int>(my_id), static_cast<int>(__builtin_ctzll(hit)));
          }
          pre_id = pid < A.g.N ? pid : INV;
          if (pre_id != INV && static_cast<u32>(lane) < M0) pre_e = A.g.adj0[static_cast<u64>(pre_id) * M0 + lane];
        }

        // accept / push / push_k in list order (:456-465)
        PHASE(6)
        // keys that fail the accept test against the current top fail it later too (the farthest distance only
        // shrinks once the top is full), so only the lanes one ballot lets through are visited, in list order
        u64 pass = __ballot(lane < nf && (my_d < key(troot) || ntop < ef));
        while (pass) {
          const int j = static_cast<int>(__builtin_ctzll(pass));
          pass &= pass - 1;
          const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_d), j));
          if (d < key(troot) || ntop < ef) {
            if (nnext >= cap) {
              status = ST_OVERFLOW;
              st_maxnext = static_cast<u32>(cap) + 1u;  // (it needed more: the next call reserves more)
              break;
            }
            const u32 id = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(my_id), j));
            const u64 en = mk(d, id);
            // next_candidates.push (:462) and top_candidates.push_k (heap.hh:34-41) touch different heaps: the
            // pop of a full top goes first, then both pushes share one LDS round (heap_push2)
            if (ntop < ef) {
              PHASE(10)
              heap_push2(nxt, nnext, top, ntop, en, nroot, troot, lane);
              hfence();
              ++ntop;
            } else {  // d < top().distance holds: it is the accept test with the top full
              PHASE(9)
              troot = nan_keys ? heap_pop_any<true>(top, ntop, lane) : heap_pop<true>(top, ntop, lane, pl);
              hfence();
              PHASE(10)
              heap_push2(nxt, nnext, top, ntop - 1, en, nroot, troot, lane);
              hfence();
            }
            PHASE(6)
            ++nnext;
            if (static_cast<u32>(nnext) > st_maxnext) st_maxnext = nnext;
          }
        }
        if (status != 0) break;
      }

      // ---- trim to k and emit in heap-array order (:296-303) ------------------------------------------------
      PHASE(7)
      if (status == 0) {
        PHASE(11)
        while (ntop > static_cast<int>(A.k)) {
          if (nan_keys) heap_pop_any<true>(top, ntop, lane);
          else heap_pop<true>(top, ntop, lane, pl);
          hfence();
          --ntop;
        }
      }
    }

    const u64 obase = static_cast<u64>(qi) * A.k;
    for (u32 i = lane; i < A.k; i += 64) {
      u32 id = INV;
      float d = 0.f;
      u32 slot = i;
      if (status == 0 && static_cast<int>(i) < ntop) {
        const u64 en = top[i];
        id = A.g.uid[eid(en)];
        d = key(en);
        if (A.sort_out) {  // fast-mode fixup pass: ascending order (ties by heap position)
          const u32 si = sortable(d);
          slot = 0;
          for (int j = 0; j < ntop; ++j) {
            const u32 sj = sortable(key(top[j]));
            slot += (sj < si || (sj == si && static_cast<u32>(j) < i)) ? 1u : 0u;
          }
        }
      }
      A.out_ids[obase + slot] = id;
      if (A.out_dists) A.out_dists[obase + slot] = d;
    }
    if (status == ST_OVERFLOW && A.out_list && lane == 0) A.out_list[atomicAdd(A.out_count, 1u)] = qi;
    if (A.vis_max && lane == 0) atomicMax(A.vis_max, nvis);
    if (A.next_max && lane == 0) atomicMax(A.next_max, st_maxnext);
    // visited-table occupancy, for the next call's shape (capped at the largest table, so that the call's sum cannot
    // wrap below 2^18 queries)
    if (A.vis_sum && lane == 0) atomicAdd(A.vis_sum, nvis < 16384u ? nvis : 16384u);
    if (A.qstats && lane == 0) {
      u32* qs = A.qstats + static_cast<u64>(qi) * kQsWords;
      qs[0] = st_dist;
      qs[1] = st_vup;
      qs[2] = st_vl0;
      qs[3] = st_lup;
      qs[4] = st_ll0;
      qs[5] = A.sort_out ? 0u : st_maxnext;  // fast-mode fixup: exact, so no tie can have changed the set
      qs[6] = status;
      qs[7] = status == 0 ? static_cast<u32>(ntop < static_cast<int>(A.k) ? ntop : A.k) : 0u;
      write_read_counts(qs, rc);
    }

    if (VIS == 0 && sslot >= 0) spill_release(vt, A, sslot, slog, lane);  // the bitmap back all zero
    if (VIS >= 1) {  // visited_nodes.clear() (:475): clear exactly the words this query touched
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
  clk.flush(A.prof, lane);
  finish_call(A, lane);
}

// ------------------------------------------------------------------------------------------------------------
// Fast search kernel (SHINE_MODE_FAST).  The same traversal with a different candidate structure: one sorted
// list of the best ef candidates (key, id, expanded bit) held in VGPRs — position p in lane p % 64 of register
// p / 64 — instead of the two std::vector heaps.
//
// Equivalence: every entry pushed onto next_candidates is also pushed onto top_candidates (hnsw.hh:461-465), and
// with pairwise distinct distances an entry evicted from top has a key above every later farthest distance, so
// it is never expanded.  next_candidates' minimum is therefore the smallest unexpanded top entry, and the loop
// ends when none is left (the break at :424).  One expansion's accept / push / push_k sequence leaves top equal to
// the ef smallest of (top ∪ fresh).  Hence, when no two keys compare equal where the reference's tie-breaking
// could decide, this kernel expands the same nodes in the same order and returns the same ids, distances and
// counters.  The events where heap layout decides are counted in qstats word 5 (0 = identical result):
//   * a key inserted equal to an unexpanded one (which of the two next_candidates yields first),
//   * an eviction whose farthest entry had an equal twin (which one push_k pops, heap.hh:34-41),
//   * equal keys at positions k-1 and k at the end (which one the trim to k pops, hnsw.hh:296-299),
//   * NaN keys.
// A key equal to the farthest with the list full is rejected by both (:461 is strict).  Results are written
// in ascending distance order.  Costs: an insertion is two ballots per register plus one DPP wave_shr per
// register (no LDS), the next candidate is one ballot per register.
// ------------------------------------------------------------------------------------------------------------
constexpr u32 EXPANDED = 0x80000000u;  // id bit: this candidate has been expanded (ids < 2^31)

// ------------------------------------------------------------------------------------------------------------
// Pipelining.  The neighbour-vector loads of the NEXT expansion are issued before the current one's merge: once
// the distances of expansion t are known, the next candidate is already determined — the smaller of the runner-up
// unexpanded entry r (whose list was prefetched one expansion earlier) and the best accepted fresh key f* (merged
// order puts fresh keys first among equals, later list positions first).  For r the vectors are requested at once;
// for f* its list is loaded first.  Either way they land while the merge and the pick run.  A misprediction (only
// possible through ties or NaN keys) re-issues the loads for the picked candidate.  The one neighbour buffer is
// refilled as soon as the current distances have consumed it, and every list / vector load on the common path is
// unconditional, so every wait is an exact vmcnt that never covers the younger prefetches.
// ------------------------------------------------------------------------------------------------------------
// Slot layout of a neighbour list in the fast kernel: list slot 16p + g lives in lane 4g + p (p < P), so the lane
// group g that evaluates slot 16p + g in pass p finds the slot's id in its own lane p (a DPP quad broadcast) and the
// group's distance reaches the slot's lane the same way: no ds_bpermute between the pick, the vector loads and the
// merge.  List order is slot order, not lane order, wherever the reference's list order decides.
__device__ __forceinline__ u32 quad_bcast(u32 x, int p) {  // lane 4g + p's value to all of group g
  switch (p) {
    case 0: return static_cast<u32>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x00, 0xF, 0xF, false));
    case 1: return static_cast<u32>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x55, 0xF, 0xF, false));
    case 2: return static_cast<u32>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0xAA, 0xF, 0xF, false));
    default: return static_cast<u32>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0xFF, 0xF, 0xF, false));
  }
}

// w: the dynamic cache's word of this lane's entry (ACCT = 2: cache_word, looked up when the list arrived)
template <int D, int METRIC, typename E, int P, int ACCT>
__device__ __forceinline__ void issue_list(NbrBuf<D, E, P>& B, const E* __restrict__ vec, u32 e, u32 w, u32 pad, int c4,
                                           const DevGraph& g) {
  if constexpr (kMfma<METRIC, E>) {
    // fp16 inner products (pass_dists_mfma): lane l reads chunk l >> 4 of slot 16p + (l & 15), whose entry sits in lane
    // 4 (l & 15) + p of the list (one ds_bpermute per pass for the id, or the dynamic cache's resolved row address)
    const int lane = static_cast<int>(threadIdx.x), src = 4 * (lane & 15), c = lane >> 4;
    if constexpr (ACCT == 2) {
      const E* row = word_row<D, E>(g, vec + static_cast<u64>(e == INV ? pad : e) * kRowElems<D, E>, e == INV ? INV : w);
      const u64 rp = reinterpret_cast<u64>(row);
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const u64 lo = static_cast<u32>(__shfl(static_cast<int>(static_cast<u32>(rp)), src + p));
        const u64 hi = static_cast<u32>(__shfl(static_cast<int>(static_cast<u32>(rp >> 32)), src + p));
        load_half_row<D, P>(B, p, reinterpret_cast<const E*>((hi << 32) | lo), c);
      }
    } else {
      u32 sid[P];
#pragma unroll
      for (int p = 0; p < P; ++p) sid[p] = static_cast<u32>(__shfl(static_cast<int>(e), src + p));
#pragma unroll
      for (int p = 0; p < P; ++p) load_half_row<D, P>(B, p, vec + static_cast<u64>(sid[p] == INV ? pad : sid[p]) * D, c);
    }
    return;
  }
  if constexpr (ACCT == 2) {  // dynamic cache: each lane resolves its own list slot to a row, the groups share it
    const E* row = word_row<D, E>(g, vec + static_cast<u64>(e == INV ? pad : e) * kRowElems<D, E>, e == INV ? INV : w);
    const u64 rp = reinterpret_cast<u64>(row);
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const u64 lo = quad_bcast(static_cast<u32>(rp), p), hi = quad_bcast(static_cast<u32>(rp >> 32), p);
      issue_row<D, E, P>(B, p, reinterpret_cast<const E*>((hi << 32) | lo), c4);
    }
  } else {
    u32 sid[P];
#pragma unroll
    for (int p = 0; p < P; ++p) sid[p] = quad_bcast(e, p);
#pragma unroll
    for (int p = 0; p < P; ++p) issue_pass_u<D, E, P>(B, p, vec, sid[p], pad, c4);
  }
}


// Waves per SIMD the register allocation must allow (build-time tuning: 4 caps a wave at 128 VGPRs, so 16 wavefronts
// fit a CU when their LDS tables do).  The two-choice tables exist to put more wavefronts on a CU: at d <= 128 and
// ef <= 256 their kernels are held to 168 VGPRs (3 per SIMD; 173 unconstrained at d = 96, ef = 256, without spills
// at 168; at ef > 256 the same cap spills).
#ifndef SHINE_FAST_MIN_WAVES
#define SHINE_FAST_MIN_WAVES 1
#endif
// fp16 rows past d = 128 in two passes a list (cfg 5's TTI shape: MFMA inner products) are held to 256 registers (2
// per SIMD): unconstrained they took 236 VGPRs + 60 AGPRs, one wavefront per SIMD and 4 per CU whatever the visited
// tables left, and fit 225 without spilling (f32 rows at d = 200 spill at 256).
template <int D, int R, int VT, typename E = float, int P = 4>
constexpr int kFastWaves = VT == 2 && D <= 128 && R <= 4 && SHINE_FAST_MIN_WAVES < 3 ? 3
                           : std::is_same_v<E, __half> && D > 128 && P <= 2 && SHINE_FAST_MIN_WAVES < 2 ? 2
                                                                                                    : SHINE_FAST_MIN_WAVES;
template <int D, int METRIC, typename E, int R, int P, int ACCT, int VT, bool PROF = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kFastWaves<D, R, VT, E, P>))) void search_fast_kernel(
    SearchArgs A) {
  PhaseClock<PROF> clk;
  clk.start();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  VisitedLds<VT> vis(smem, A);                // visited table
  u32* sc_ids = reinterpret_cast<u32*>(smem + A.vis_cap * VisitedLds<VT>::kBytes);  // greedy-descent scratch
  float* sc_d = reinterpret_cast<float*>(sc_ids + 64);
  u64* mrg = reinterpret_cast<u64*>(sc_d + 64);  // merge scratch: (key, id) at merged positions 0 .. ef
  const int lane = threadIdx.x, g4 = lane >> 2, c4 = lane & 3;
  const E* __restrict__ vec = static_cast<const E*>(A.g.vec);
  const u32* __restrict__ adj0 = A.g.adj0;
  const u32 M0 = A.g.M0, pad = A.g.pad_node;
  const int ef = static_cast<int>(A.ef);
  const float INF = __builtin_inff();
  const u32 my_slot = 16u * static_cast<u32>(c4) + static_cast<u32>(g4);  // list slot of this lane (issue_list)
  const bool in_row = c4 < P && my_slot < M0;
  const u32 row_lane = in_row ? my_slot : 0u;
  // Unconditional, and never masked right after the load (that would wait for it): lanes without a slot hold a copy
  // of entry 0 and are excluded where the list is used (the visited test; they are never fresh).
  auto load_row = [&](u32 node) -> u32 { return adj0[static_cast<u64>(node < A.g.N ? node : pad) * M0 + row_lane]; };
  auto slot_of = [](int l) { return 16 * (l & 3) + (l >> 2); };

  const u32 n_items = A.in_count ? *A.in_count : A.nq;
  for (;;) {
    u32 item = 0;
    if (lane == 0) item = atomicAdd(A.counter, 1u);
    item = bcast(item);
    if (item >= n_items) break;
    const u32 qi = A.in_list ? A.in_list[item] : item;

    PHASE(0)
    QueryRegs<D, E> Q;
    load_query<D, E>(A.queries + static_cast<u64>(qi) * D, lane, Q);
    vis.clear(A, lane);
    u32 st_dist = 0, st_vup = 0, st_vl0 = 0, st_lup = 0, st_ll0 = 0, ties = 0, status = 0;
    ReadCount rc;
    PHASE(1)
    u32 nn;
    float closest;
    entry_and_descent<D, METRIC, E, ACCT>(A, vec, Q, sc_ids, sc_d, lane, nn, closest, st_dist, st_vup, st_vl0, st_lup, status,
                                    rc, qi);
    ++st_dist;  // top_candidates.push({nn, dist(q, nn)}) (hnsw.hh:285-286)

    float ck[R];  // candidate keys, ascending; +inf beyond the size
    u32 ci[R];    // candidate ids | EXPANDED; INV beyond the size
#pragma unroll
    for (int r = 0; r < R; ++r) {
      ck[r] = INF;
      ci[r] = INV;
    }
    int cs = 0;
    float cmax = INF;  // key at position ef - 1 once the list is full
    u32 nvis = 1;
    if (status == 0) {
      ck[0] = lane == 0 ? closest : INF;
      ci[0] = lane == 0 ? (nn | EXPANDED) : INV;  // popped right away (:418)
      cs = 1;
      if (closest != closest) ++ties;
      if (lane == 0) vis.insert_first(nn);
      wave_sync();
    }

    // pipeline state: the candidate's list `e` and its vectors in X (in flight); the runner-up r and its
    // prefetched list.  X is refilled for the next candidate as soon as the current distances have consumed it.
    NbrBuf<D, E, P> X;
    u32 e = load_row(status == 0 ? nn : pad);
    // ACCT = 2: the cache words of list e's entries (cache_word), looked up once per list and carried from its rows'
    // request to its read accounting; ncs: those of nrow, looked up after the distances, before the rows are requested
    u32 ecs = ACCT == 2 ? cache_word(A.g, e) : INV;
    u32 ncs = INV;
    issue_list<D, METRIC, E, P, ACCT>(X, vec, e, ecs, pad, c4, A.g);
    u32 r_id = INV;
    float r_key = INF;
    u32 nid = nn;
    u32 nrow = load_row(nn);
    u32 cur = nn;  // the candidate whose list `e` is
    bool ehint_known = false;  // ehint is e's home bucket as it stands (not a guess)
    typename VisitedLds<VT>::Hint ehint = VisitedLds<VT>::unknown();  // e's home word / bucket as probed one
                                                                      // expansion earlier (VisitedLds::test_and_set)
    // In-place spill (SearchArgs::spill_flags): once the table overflows, the query's visited set moves to an HBM
    // bitmap and the search goes on there (a global atomicOr per fresh id) instead of being re-run from scratch.
    // (Plain code, no lambda: a bitmap pointer assigned through a lambda's reference capture compiled to a constant
    // null base on this toolchain.)
    int sslot = -1;  // the bitmap this query holds (wave-uniform), -1 = the LDS table
    u32 slog = 0;    // ids logged since the spill (spill_log)

    while (status == 0) {
      ++st_ll0;  // read_neighborlist (:436-438)
      count_list_read<ACCT>(A, rc, cur, lane);
      PHASE(8)
      // ACCT = 2: the runner-up's cache words requested as soon as its list is home (it was the youngest load, so this
      // waits for e's vectors too, which the distances below need anyway): the lookup's round trip overlaps this
      // expansion's visited test and distances instead of holding the next rows' request back (PHASE(4))
      if constexpr (ACCT == 2) ncs = cache_word(A.g, nrow);
      bool cand = in_row && e != INV;
      if (!A.g.lists_unique) {  // first occurrence in list order wins (visited.insert order, :443)
#pragma unroll 1
        for (int j = 0; j < 4 * 16; ++j) {
          const u32 ej = __shfl(e, j);
          const u32 sj = static_cast<u32>(slot_of(j));
          if ((j & 3) < P && sj < M0 && sj < my_slot && ej == e) cand = false;
        }
      }
      // visited.contains / insert (:441-443); u16 table with e's home bucket known from the look-ahead probe: the
      // answer without an LDS round trip, the recording compare-and-swap checked after the distances (+1.2 % at
      // ef = 128, profiles/r02/lib_probe_deferred_insert.jsonl)
      bool fresh = false, vovf = false;
      u32 pw = INV, pexp = 0, pold = 0;
      if (sslot >= 0) {  // spilled: the HBM bitmap or hash table (SpillSet)
        const SpillSet ss(A, sslot);
        bool hovf = false;
        if (cand) fresh = ss.test_and_set(e, hovf);
        if (!ss.hashed()) {
          spill_log(A, sslot, slog, fresh, e, lane);
        } else if (__ballot(hovf) || nvis + __popcll(__ballot(fresh)) > A.spill_hash / 2) {
          status = ST_OVERFLOW;  // the hash table is half full: the query is handed on to the light pass
          break;
        }
      } else if constexpr (VT >= 1) {
        if (cand) {
          const int r = ehint_known ? vis.begin(e, ehint, pw, pexp, pold) : 2;
          fresh = r == 2 ? vis.test_and_set(e, vovf, ehint) : r == 1;
        }
      } else {
        if (cand) fresh = vis.test_and_set(e, vovf, ehint);
      }
      // the table is too full (or an id landed too far from home): spill it and go on in HBM.  Lanes whose insert
      // overflowed are tested against the bitmap; a deferred compare-and-swap that lost its word records its (fresh)
      // id there instead of retrying in the table.
      if (sslot < 0 && (__ballot(vovf) || nvis + __popcll(__ballot(fresh)) > A.vis_limit)) {
        const bool lost = pw != INV && pold != pexp;
        sslot = claim_spill_bitmap(A, lane);
        if (sslot < 0) {
          status = ST_OVERFLOW;
          break;
        }
        const SpillSet ss(A, sslot);
        wave_sync();
        spill_table(vis, ss, A, lane);
        EVENT(3)
        if (lost) ss.set(e);
        pw = INV;
        if (!ss.hashed()) spill_log(A, sslot, slog, lost || vovf, e, lane);
        bool hovf = false;
        if (vovf) {
          fresh = ss.test_and_set(e, hovf);
          vovf = false;
        }
        if (__ballot(hovf)) {
          status = ST_OVERFLOW;
          break;
        }
      }
      const u64 fm = __ballot(fresh);
      const int nf = __popcll(fm);
      count_vec_reads<ACCT>(A, rc, fresh, e, qi, false, ACCT == 2 ? ecs : kNoWord);
      nvis += nf;
      st_vl0 += nf;
      st_dist += nf;

      PHASE(5)
      float my_d = INF;  // distance of this lane's list slot
      u64 acc = 0;
      if (nf > 0) {
        float out[P];
        if constexpr (kMfma<METRIC, E>) {  // slot 16p + g's product is in lane g of pass p
          pass_dists_mfma<D, P>(Q, X, out);
#pragma unroll
          for (int p = 0; p < P; ++p) {
            const float v = __shfl(out[p], g4);
            if (c4 == p) my_d = v;
          }
        } else {
          pass_dists<D, METRIC, E, P>(Q, X, out);
#pragma unroll
          for (int p = 0; p < P; ++p) {  // the group's sum is complete in its lane 3 (fold8)
            const float v = __uint_as_float(quad_bcast(__float_as_uint(out[p]), 3));
            if (c4 == p) my_d = v;
          }
        }
        if (!fresh) my_d = INF;
        if (fresh && my_d != my_d) {  // NaN: the reference's comparisons are all false; no ordered slot exists here
          my_d = INF;
          ++ties;
        }
        acc = __ballot(fresh && (cs < ef || my_d < cmax));  // fresh keys that can enter (:461)
      }

      if constexpr (VT >= 1) {  // the deferred compare-and-swaps, before the table is probed again
        if (pw != INV) vis.finish(e, pexp, pold, vovf);
        if (__ballot(vovf)) {  // a retried insert overflowed: its id is fresh, record it in HBM
          sslot = claim_spill_bitmap(A, lane);
          if (sslot < 0) {
            status = ST_OVERFLOW;
            break;
          }
          const SpillSet ss(A, sslot);
          wave_sync();
          spill_table(vis, ss, A, lane);
          EVENT(3)
          if (vovf) ss.set(e);
          if (!ss.hashed()) spill_log(A, sslot, slog, vovf, e, lane);
        }
      }

      // ---- the next candidate, known before the merge ----------------------------------------------------------
      // the smaller of f* (best accepted fresh key; among equals the last list position, as merged) and the
      // runner-up r; its vectors are requested here, one issue point for every path, into the buffer the
      // distances above have just consumed
      PHASE(4)
      u32 pid = r_id;
      if (acc) {
        const float fstar = wave_min(((acc >> lane) & 1ull) ? my_d : INF);
        const u64 hit = acc & __ballot(my_d == fstar);
        if (r_id == INV || fstar <= r_key) {  // the last list slot among equals: highest p, then highest group
          int hl = 0;
#pragma unroll
          for (int p = 0; p < P; ++p) {
            const u64 m = hit & (0x1111111111111111ull << p);
            if (m) hl = 63 - static_cast<int>(__clzll(m));
          }
          pid = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(e), hl));
        }
      }
      if (pid == r_id) EVENT(9) else EVENT(10)
      const u32 prow = pid == r_id ? nrow : load_row(pid != INV ? pid : pad);  // a fresh f*: its list now
      // an entry already at its home slot of the visited table is not fresh: its row is not requested (one
      // read-only LDS probe; the visit proper still runs at the top of the next expansion)
      const bool probe = sslot < 0 && in_row && prow != INV;
      const typename VisitedLds<VT>::Hint pword = probe ? vis.probe(prow) : VisitedLds<VT>::unknown();
      const bool seen = probe && vis.home_match(prow, pword);
      const u32 pcs = ACCT == 2 ? (pid == r_id ? ncs : cache_word(A.g, prow)) : INV;
      issue_list<D, METRIC, E, P, ACCT>(X, vec, seen ? INV : prow, pcs, pad, c4, A.g);

      // ---- merge (:456-465 over the whole list at once) ----------------------------------------------------------
      PHASE(6)
      if (acc) {
        int shift[R];
#pragma unroll
        for (int r = 0; r < R; ++r) shift[r] = 0;
        int frank = 0;  // fresh lane: accepted keys ordered before it
        int fbase = 0;  // fresh lane: list entries below it
        // The merged order of the fresh keys as one 64-bit key per lane: the distance's order-preserving image (-0
        // made +0 first, so equal distances compare equal), then later list slots first.  One 64-bit compare per
        // accepted key instead of three float / slot compares and two mask operations.
        const u32 ohi = sortable(my_d + 0.0f), olo = 63u - my_slot;
        const u64 okey = (static_cast<u64>(ohi) << 32) | olo;
        u64 todo = acc;
        while (todo) {
          const int i = static_cast<int>(__builtin_ctzll(todo));
          todo ^= 1ull << i;
          const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_d), i));
          const u64 oi = (static_cast<u64>(static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(ohi), i))) << 32) |
                         static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(olo), i));
          // one compare per register serves both counts: the entries at or above d (shifted by this key) and, by
          // complement, the entries below it (neither d nor the list holds NaN)
          int at_or_above = 0;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const bool le = d <= ck[r];
            shift[r] += le ? 1 : 0;
            at_or_above += __popcll(__ballot(le));
          }
          frank += oi < okey ? 1 : 0;
          fbase = shine_writelane_i32(64 * R - at_or_above, i, fbase);
        }
        const int total = cs + __popcll(acc);
        const int hi = total < ef + 1 ? total : ef + 1;  // merged positions written: 0 .. hi-1
        const int sink = ef + 1;  // entries that fall past the cut are written to a scratch slot (no branches)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int p = 64 * r + lane;
          const int np = p + shift[r];
          mrg[(p < cs && np <= ef) ? np : sink] = (static_cast<u64>(ci[r]) << 32) | __float_as_uint(ck[r]);
        }
        {
          const int np = fbase + frank;
          mrg[(((acc >> lane) & 1ull) && np <= ef) ? np : sink] = (static_cast<u64>(e) << 32) | __float_as_uint(my_d);
        }
        wave_sync();
        cs = total < ef ? total : ef;
        bool tie = false;
        const u64 none = (static_cast<u64>(INV) << 32) | __float_as_uint(INF);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int p = 64 * r + lane;
          const int pc = p < ef ? p : ef;  // positions p, p + 1 in one ds_read2 (p + 1 <= sink)
          const u64 m0r = mrg[pc], m1r = mrg[pc + 1];
          tie |= p + 1 < hi && key(m0r) == key(m1r) &&
                 ((eid(m0r) & EXPANDED) == 0 || (eid(m1r) & EXPANDED) == 0 || p + 1 == ef);
          const u64 m0 = p < cs ? m0r : none;
          ck[r] = key(m0);
          ci[r] = eid(m0);
        }
        if (__ballot(tie)) ++ties;
        wave_sync();
        if (cs == ef) {
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (((ef - 1) >> 6) == r) cmax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ck[r]), (ef - 1) & 63));
        }
      }

      // ---- next_candidates.top(); pop() (:418-426) and the new runner-up -----------------------------------
      PHASE(2)
      u64 um[R];  // unexpanded entries (INV carries the EXPANDED bit)
#pragma unroll
      for (int r = 0; r < R; ++r) um[r] = __ballot(static_cast<int>(ci[r]) >= 0);
      int p1 = -1;
#pragma unroll
      for (int r = R - 1; r >= 0; --r) p1 = um[r] ? 64 * r + static_cast<int>(__builtin_ctzll(um[r])) : p1;
      if (p1 < 0) break;  // every candidate within the radius expanded: the break at :424
      const int r1 = p1 >> 6, l1 = p1 & 63;
      u32 c = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32 cr = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(ci[r]), l1));
        c = r == r1 ? cr : c;
        ci[r] = (r == r1 && lane == l1) ? (ci[r] | EXPANDED) : ci[r];
        um[r] = r == r1 ? (um[r] & (um[r] - 1)) : um[r];
      }
      int p2 = -1;
#pragma unroll
      for (int r = R - 1; r >= 0; --r) p2 = um[r] ? 64 * r + static_cast<int>(__builtin_ctzll(um[r])) : p2;
      u32 c2 = INV;
      float k2 = INF;
      {
        const int r2 = p2 >> 6, l2 = p2 & 63;  // p2 = -1: r2 = -1 matches no register
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const u32 cr = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(ci[r]), l2 & 63));
          const float kr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ck[r]), l2 & 63));
          c2 = r == r2 ? cr : c2;
          k2 = r == r2 ? kr : k2;
        }
      }
      u32 erow = prow, ecsn = pcs;
      if (c != pid) {  // mispredicted (ties / NaN keys): fetch the picked candidate's list and vectors
        EVENT(11)
        erow = c == nid ? nrow : load_row(c);
        if constexpr (ACCT == 2) ecsn = c == nid ? ncs : cache_word(A.g, erow);
        issue_list<D, METRIC, E, P, ACCT>(X, vec, erow, ecsn, pad, c4, A.g);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this rare path leaves nothing in flight behind the prefetch
      }
      nid = c2 != INV ? c2 : c;
      nrow = load_row(nid);  // unconditional: always the youngest load
      e = erow;
      ecs = ecsn;
      ehint = c != pid ? VisitedLds<VT>::unknown() : pword;  // the probe read prow's home bucket, no insert since
      ehint_known = c == pid && sslot < 0;
      cur = c;
      r_id = c2;
      r_key = k2;
    }

    PHASE(7)
    // top-k in ascending order; an equal pair straddling position k is decided by heap layout in the reference
    if (status == 0 && cs > static_cast<int>(A.k)) {
      const int k = static_cast<int>(A.k);
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (((k - 1) >> 6) == r) a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ck[r]), (k - 1) & 63));
        if ((k >> 6) == r) b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ck[r]), k & 63));
      }
      if (a == b) ++ties;
    }
    const u64 obase = static_cast<u64>(qi) * A.k;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 i = static_cast<u32>(64 * r + lane);
      if (i < A.k) {
        const bool ok = status == 0 && static_cast<int>(i) < cs && (ci[r] & ~EXPANDED) < A.g.N;
        A.out_ids[obase + i] = ok ? A.g.uid[ci[r] & ~EXPANDED] : INV;
        if (A.out_dists) A.out_dists[obase + i] = ok ? ck[r] : 0.f;
      }
    }
    if (status == ST_OVERFLOW && A.out_list && lane == 0) A.out_list[atomicAdd(A.out_count, 1u)] = qi;
    if (A.vis_max && lane == 0) atomicMax(A.vis_max, nvis);
    // visited-table occupancy, for the next call's shape (capped at the largest table, so that the call's sum cannot
    // wrap below 2^18 queries)
    if (A.vis_sum && lane == 0) atomicAdd(A.vis_sum, nvis < 16384u ? nvis : 16384u);
    if (A.qstats && lane == 0) {
      u32* qs = A.qstats + static_cast<u64>(qi) * kQsWords;
      qs[0] = st_dist;
      qs[1] = st_vup;
      qs[2] = st_vl0;
      qs[3] = st_lup;
      qs[4] = st_ll0;
      qs[5] = ties;
      qs[6] = status;
      qs[7] = status == 0 ? static_cast<u32>(cs < static_cast<int>(A.k) ? cs : A.k) : 0u;
      write_read_counts(qs, rc);
    }
    // Hand the bitmap back all zero: the stores land before the flag drops.  Every lane stores the same zero flag
    // (one dword): a lane-0 branch there, the last statement of the item loop, was jump-threaded into the next item's
    // lane-0 fetch, the wave split, lanes 1-63 ran an item without lane 0 and faulted
    // (tests/test_gpu_fast.py::test_fast_mode_spills_in_place_and_stays_exact).
    if (sslot >= 0) spill_release(vis, A, sslot, slog, lane);
  }
  clk.flush(A.prof, lane);
  finish_call(A, lane);
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
  QueryRegs<D, E> Q;
  load_query<D, E>(A.queries + static_cast<u64>(qi) * D, lane, Q);
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

// ------------------------------------------------------------------------------------------------------------
// heap replay (diagnostics): op 0 = push, 1 = pop, 2 = push_k(k)
// ------------------------------------------------------------------------------------------------------------
template <bool MAXH>
__global__ __launch_bounds__(64) void heap_replay_kernel(const int32_t* ops, const float* vals, const uint32_t* ids,
                                                         uint32_t n_ops, uint32_t k, float* out_d, uint32_t* out_ids,
                                                         uint32_t* out_n) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u64* h = reinterpret_cast<u64*>(smem);
  const int lane = threadIdx.x;
  const PopLane pl(lane);
  const bool any = (k & 0x80000000u) != 0;  // exercise the general pop instead of the fast one
  k &= 0x7FFFFFFFu;
  int n = 0;
  u64 root = 0;  // tracked exactly as the search kernel tracks it; checked against h[0] after every op
  bool root_ok = true;
  for (u32 i = 0; i < n_ops; ++i) {
    const u64 e = mk(vals[i], ids[i]);
    const int op = ops[i];
    if (op == 0) {
      root = heap_push<MAXH>(h, n, e, root, lane);
      ++n;
    } else if (op == 1) {
      if (n > 0) {
        root = any ? heap_pop_any<MAXH>(h, n, lane) : heap_pop<MAXH>(h, n, lane, pl);
        --n;
      }
    } else {
      if (n < static_cast<int>(k)) {
        root = heap_push<MAXH>(h, n, e, root, lane);
        ++n;
      } else if (hcmp<MAXH>(vals[i], key(root))) {
        root = any ? heap_pop_any<MAXH>(h, n, lane) : heap_pop<MAXH>(h, n, lane, pl);
        root = heap_push<MAXH>(h, n - 1, e, root, lane);
      }
    }
    if (n > 0 && bcast64(h[0]) != root) root_ok = false;
  }
  for (int i = lane; i < n; i += 64) {
    out_d[i] = key(h[i]);
    out_ids[i] = eid(h[i]);
  }
  if (lane == 0) *out_n = root_ok ? static_cast<u32>(n) : 0xFFFFFFFFu;
}

template <int D, int METRIC, typename E, int AC>
hipError_t launch_search_acct(uint32_t grid, const SearchArgs& a, hipStream_t s) {
  const size_t lds = search_lds_bytes(a.ef, a.cap, a.vis_cap, a.vis_cap > 0 ? vis_entry_bytes(a.vis16) : 4);
  auto run = [&](auto kern) -> hipError_t {
    if (lds > 65536) {  // beyond the default dynamic-LDS limit: opt in (per device, so every launch)
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, s, a);
    return hipGetLastError();
  };
  if (a.fast) {  // sorted-list kernel; the launcher's caller guarantees ef <= kFastMaxEf and a visited table in LDS
    const size_t lds_f = search_fast_lds_bytes(a.vis_cap, a.ef, vis_entry_bytes(a.vis16));
    auto runf = [&](auto kern) -> hipError_t {
      if (lds_f > 65536) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_f));
        if (e != hipSuccess) return e;
      }
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds_f, s, a);
      return hipGetLastError();
    };
    if (a.vis_cap == 0 || a.ef == 0 || a.ef > kFastMaxEf) return hipErrorInvalidValue;
    // P = passes of 16 list slots: 2 covers M0 <= 32 (M <= 16), 4 covers M0 <= 64
    if (a.g.M0 > 64) return hipErrorInvalidValue;
    const bool wide = a.g.M0 > 32;
    auto pick = [&](auto vt) -> hipError_t {
      constexpr int VT = decltype(vt)::value;
      if constexpr (!AC && D == 128 && METRIC == 0 && std::is_same_v<E, float>) {
        if (a.prof && !wide && a.ef > 64 && a.ef <= 128) return runf(search_fast_kernel<D, METRIC, E, 2, 2, AC, VT, true>);
      }
      if constexpr (!AC && D == 200 && METRIC == 1 && std::is_same_v<E, __half>) {  // cfg5's shape (fp16, IP, ef 250)
        if (a.prof && !wide && a.ef > 128 && a.ef <= 256) return runf(search_fast_kernel<D, METRIC, E, 4, 2, AC, VT, true>);
      }
      if (a.ef <= 64)
        return wide ? runf(search_fast_kernel<D, METRIC, E, 1, 4, AC, VT>) : runf(search_fast_kernel<D, METRIC, E, 1, 2, AC, VT>);
      if (a.ef <= 128)
        return wide ? runf(search_fast_kernel<D, METRIC, E, 2, 4, AC, VT>) : runf(search_fast_kernel<D, METRIC, E, 2, 2, AC, VT>);
      if (a.ef <= 256)
        return wide ? runf(search_fast_kernel<D, METRIC, E, 4, 4, AC, VT>) : runf(search_fast_kernel<D, METRIC, E, 4, 2, AC, VT>);
      return wide ? runf(search_fast_kernel<D, METRIC, E, 8, 4, AC, VT>) : runf(search_fast_kernel<D, METRIC, E, 8, 2, AC, VT>);
    };
    if (a.vis16 == 2) return pick(std::integral_constant<int, 2>{});
    if (a.vis16 == 3) {  // two-choice u32 buckets: compiled for replicas (no read accounting) only
      if constexpr (!AC) return pick(std::integral_constant<int, 3>{});
      else return hipErrorInvalidValue;
    }
    return a.vis16 ? pick(std::integral_constant<int, 1>{}) : pick(std::integral_constant<int, 0>{});
  }
  if constexpr (!AC && D == 128 && METRIC == 0 && std::is_same_v<E, float>) {
    if (a.prof && a.vis_cap > 0 && !a.vis16) return run(search_kernel<D, METRIC, E, 0, AC, 0, true>);
    if (a.prof && a.vis_cap > 0 && a.vis16 == 1) return run(search_kernel<D, METRIC, E, 0, AC, 1, true>);
  }
  if (a.global_heaps) {  // both heaps in HBM: only the scratch ids / distances stay in LDS
    if (a.vis_cap != 0 || !a.heaps || a.heap_stride < align16(8ull * a.ef) / 8 + a.cap) return hipErrorInvalidValue;
    hipLaunchKernelGGL((search_kernel<D, METRIC, E, 2, AC>), dim3(grid), dim3(64), 64 * 4 * 2, s, a);
    return hipGetLastError();
  }
  if (a.vis_cap > 0 && a.vis16 == 2) return run(search_kernel<D, METRIC, E, 0, AC, 2>);
  if (a.vis_cap > 0 && a.vis16 == 3) {
    if constexpr (!AC) return run(search_kernel<D, METRIC, E, 0, AC, 3>);
    else return hipErrorInvalidValue;
  }
  if (a.vis_cap > 0) return a.vis16 ? run(search_kernel<D, METRIC, E, 0, AC, 1>) : run(search_kernel<D, METRIC, E, 0, AC, 0>);
  return run(search_kernel<D, METRIC, E, 1, AC>);
}

// Read accounting (qstats words 8-11, cache-warmup counters) is compiled in only where it can count something.
template <int D, int METRIC, typename E>
hipError_t launch_search_t(uint32_t grid, const SearchArgs& a, hipStream_t s) {
  if (a.g.sharded && a.g.cslot) return launch_search_acct<D, METRIC, E, 2>(grid, a, s);  // dynamic cache
  if (a.g.sharded || a.access) return launch_search_acct<D, METRIC, E, 1>(grid, a, s);
  return launch_search_acct<D, METRIC, E, 0>(grid, a, s);
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

}  // namespace
}  // namespace shine
