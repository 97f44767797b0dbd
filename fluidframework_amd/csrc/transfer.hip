// transfer.hip — device-side packing before a device -> host copy.
//
// Per-document results live in fixed-capacity slabs (catch-up ranges: 16 per flagged op; prop sets:
// the tier's table size), most of which a document never fills. Copying whole slabs moved up to ten
// times the bytes recorded (fmt_mt_fetch_catchup_all: the full slab region into a zeroed pageable
// vector, 0.18 GB/s end to end). gatherSpansKernel packs every document's used prefix into one dense
// buffer first (one wave per span, dword copies), so the D2H moves only what the host reads.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace fmt_kernels {

constexpr int kGatherWaves = 4;

__global__ __launch_bounds__(64 * kGatherWaves) void gatherSpansKernel(const GatherSpan* __restrict__ spans, uint32_t n,
                                                                       uint32_t* __restrict__ dst) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  for (uint32_t i = blockIdx.x * kGatherWaves + wave; i < n; i += gridDim.x * kGatherWaves) {
    const GatherSpan sp = spans[i];
    uint32_t* out = dst + sp.dstWord;
    for (uint32_t w = lane; w < sp.words; w += 64) out[w] = sp.src[w];
  }
}

hipError_t launchGatherSpans(const GatherSpan* spans, uint32_t n, uint32_t* dst, int numCUs, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t wanted = (n + kGatherWaves - 1) / kGatherWaves;
  const uint32_t cap = static_cast<uint32_t>(numCUs) * 8u;
  const uint32_t grid = wanted < cap ? wanted : cap;
  hipLaunchKernelGGL(gatherSpansKernel, dim3(grid), dim3(64 * kGatherWaves), 0, stream, spans, n, dst);
  return hipGetLastError();
}

}  // namespace fmt_kernels
