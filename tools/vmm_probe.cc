// Diagnostics: which HIP virtual-memory mapping patterns this device / driver accepts (sharded placement).
// Build: hipcc -O1 tools/vmm_probe.cc -o tools/vmm_probe ; run on a GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

static void report(const char* what, hipError_t e) { std::printf("%-58s %s\n", what, hipGetErrorString(e)); }

static hipMemAllocationProp prop0() {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  return p;
}

// reserve `pieces` * stride, map `piece` bytes at each stride, set access per piece (or once for all)
static void trial(const char* name, size_t stride, size_t piece, int pieces, bool whole, size_t align = 0) {
  hipMemAllocationProp p = prop0();
  void* va = nullptr;
  hipError_t e = hipMemAddressReserve(&va, stride * pieces, align, nullptr, 0);
  if (e != hipSuccess) return report(name, e);
  std::vector<hipMemGenericAllocationHandle_t> hs(pieces);
  for (int i = 0; i < pieces && e == hipSuccess; ++i) {
    e = hipMemCreate(&hs[i], piece, &p, 0);
    if (e == hipSuccess) e = hipMemMap(static_cast<char*>(va) + i * stride, piece, 0, hs[i], 0);
  }
  hipMemAccessDesc d{};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  if (e == hipSuccess) {
    if (whole) e = hipMemSetAccess(va, stride * pieces, &d, 1);
    else
      for (int i = 0; i < pieces && e == hipSuccess; ++i) e = hipMemSetAccess(static_cast<char*>(va) + i * stride, piece, &d, 1);
  }
  if (e == hipSuccess) e = hipMemset(static_cast<char*>(va) + (pieces - 1) * stride, 1, piece);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  report(name, e);
  for (int i = 0; i < pieces; ++i) {
    (void)hipMemUnmap(static_cast<char*>(va) + i * stride, piece);
    (void)hipMemRelease(hs[i]);
  }
  (void)hipMemAddressFree(va, stride * pieces);
}

int main() {
  hipMemAllocationProp p = prop0();
  size_t gmin = 0, grec = 0;
  report("granularity (minimum)", hipMemGetAllocationGranularity(&gmin, &p, hipMemAllocationGranularityMinimum));
  report("granularity (recommended)", hipMemGetAllocationGranularity(&grec, &p, hipMemAllocationGranularityRecommended));
  std::printf("minimum %zu recommended %zu\n", gmin, grec);
  const size_t MB2 = size_t(1) << 21;
  trial("1 piece 2MB", MB2, MB2, 1, false);
  trial("2 pieces 2MB contiguous, access per piece", MB2, MB2, 2, false);
  trial("2 pieces 2MB, stride 4MB, access per piece", 2 * MB2, MB2, 2, false);
  trial("2 pieces 2MB contiguous, access once", MB2, MB2, 2, true);
  trial("2 pieces 4KB contiguous, access per piece", 4096, 4096, 2, false);
  trial("2 pieces 64KB, stride 128KB, access per piece", 131072, 65536, 2, false);
  trial("3 pieces 2MB contiguous, access per piece", MB2, MB2, 3, false);
  trial("2 pieces 2MB contiguous, reserve aligned 2MB", MB2, MB2, 2, false, MB2);
  trial("2 pieces 1024000 B, stride 1 MiB", 1 << 20, 1024000, 2, false);
  trial("2 pieces 1024000 B, stride 1 MiB, reserve aligned 4KB", 1 << 20, 1024000, 2, false, 4096);
  trial("2 pieces 4MB, stride 4MB, reserve aligned 2MB", 2 * MB2, 2 * MB2, 2, false, MB2);
  trial("2 pieces 131072 B contiguous", 131072, 131072, 2, false);
  trial("1 piece 256 MiB", size_t(256) << 20, size_t(256) << 20, 1, false, MB2);
  trial("2 pieces 256 MiB, stride 260 MiB, reserve aligned 2MB", size_t(260) << 20, size_t(256) << 20, 2, false, MB2);
  trial("2 pieces 64 MiB, stride 64 MiB", size_t(64) << 20, size_t(64) << 20, 2, false, MB2);
  trial("2 pieces 64 MiB, stride 66 MiB", size_t(66) << 20, size_t(64) << 20, 2, false, MB2);
  trial("2 pieces 32 MiB, stride 34 MiB", size_t(34) << 20, size_t(32) << 20, 2, false, MB2);
  trial("2 pieces 4 MiB, stride 6 MiB", size_t(6) << 20, size_t(4) << 20, 2, false, MB2);
  return 0;
}
