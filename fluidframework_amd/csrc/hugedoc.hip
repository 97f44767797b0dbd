// hugedoc.hip — replay of very large documents (BASELINE config 5, T3) for gfx950: one wavefront per
// document, its state in HBM (huge_engine.h), its LRU heap and group directory in LDS.
//
// A single document's ops form one dependency chain, so a document is replayed by one wave and
// several huge documents run side by side (one per workgroup / CU). What bounds a step is the latency
// of the dependent HBM/L2 round trips of one op (window pass, group scan, a slot list, one leaf
// block, the block/heap updates), not bandwidth.
#include <hip/hip_runtime.h>

#define FMT_HUGE_KERNEL 1  // (huge_engine.h: global-typed state pointers)
#include "huge_engine.h"
#include "kernels.h"

namespace fmt_kernels {

static_assert(sizeof(fmt_huge::HugeLds) <= 160 * 1024, "the huge-document LDS state must fit one CU's LDS");

// kWaves waves per workgroup: wave 0 replays; the others serve its window/slot passes. Adj: batches
// with annotate-adjust (huge_engine.h HugeDocT).
template <bool Adj, bool Rm>
__global__ __launch_bounds__(64 * fmt_huge::HugeDoc::kWaves) void hugeDocKernel(const fmt_huge::HugeState* __restrict__ states,
                                                                            const fmt_huge::HugeInputs* __restrict__ inputs,
                                                                            const HugeOut* __restrict__ outs, uint32_t count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));  // (scalar branch below)
  for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
    fmt_huge::HugeDocT<Adj, Rm> doc;
    doc.S = states[i];
    doc.L = reinterpret_cast<fmt_huge::HugeLds*>(lds);
    if (wave != 0) {
      doc.helperLoop(wave);
      continue;
    }
    doc.run(inputs[i]);
    doc.postExit();
    const HugeOut o = outs[i];
    const uint64_t t0 = fmt_huge::HugeDoc::clk();
    doc.writeOutputs(o.header, o.leaves, o.capLeaves, o.chars, o.capChars, o.props, o.legacy, o.leavesHi);
    doc.prof[6] += fmt_huge::HugeDoc::clk() - t0;
    doc.prof[23] = doc.textTop - doc.mergeLo;
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < fmt_huge::HugeDoc::kProf; k++) o.prof[k] = doc.prof[k];
  }
}

size_t hugeLdsBytes() { return sizeof(fmt_huge::HugeLds); }

hipError_t launchHugeDocs(const fmt_huge::HugeState* states, const fmt_huge::HugeInputs* inputs, const HugeOut* outs,
                          uint32_t count, bool adjust, bool rmOrder, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  const dim3 grid(count), block(64 * fmt_huge::HugeDoc::kWaves);
  const size_t lds = sizeof(fmt_huge::HugeLds);
  if (adjust && rmOrder) hipLaunchKernelGGL((hugeDocKernel<true, true>), grid, block, lds, stream, states, inputs, outs, count);
  else if (adjust) hipLaunchKernelGGL((hugeDocKernel<true, false>), grid, block, lds, stream, states, inputs, outs, count);
  else if (rmOrder) hipLaunchKernelGGL((hugeDocKernel<false, true>), grid, block, lds, stream, states, inputs, outs, count);
  else hipLaunchKernelGGL((hugeDocKernel<false, false>), grid, block, lds, stream, states, inputs, outs, count);
  return hipGetLastError();
}

}  // namespace fmt_kernels
