// digest.hip — per-document content digest of the converged merge-tree state (fmt_mt_state_digest).
//
// A 64-bit fingerprint of everything the parity tests compare field by field (tests/mt_compare.py):
// the header (status, collab window, counts, depth, visible length), every leaf in document order
// (stamps, remove-client set — tags 10 / 11 / 12 for short ids 64..127 / 128..191 / 192..253, only on leaves that have one — char
// offset, length, insert client, parent block ordinal, marker bit),
// each leaf's properties BY VALUE (document-local prop-set ids are not part of it) and the text. The
// definition is an order-sensitive sum of mixed elements, so one wave per document
// folds its leaves and units lane-parallel and reduces once:
//   elem(tag, i, w) = mix(mix((tag << 56) ^ i) ^ w),  digest = mix(Σ elem mod 2^64)
// mix = the splitmix64 finalizer. The oracle restates the same definition over its own state
// (oracle/capi.cpp orc_mt_replay_digest), which is how the bench ties full-size T1 to the oracle.
#include <hip/hip_runtime.h>

#include "../../include/fmt.h"
#include "kernels.h"

namespace fmt_kernels {

constexpr int kDigWaves = 4;

__device__ __forceinline__ uint64_t digMix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t digElem(uint64_t tag, uint64_t i, uint64_t w) {
  return digMix(digMix((tag << 56) ^ i) ^ w);
}

__global__ __launch_bounds__(64 * kDigWaves) void stateDigestKernel(const fmt_mt_doc_result* __restrict__ hdrs,
                                                                   const SumView* __restrict__ views, uint32_t nDocs,
                                                                   uint64_t* __restrict__ out) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  for (uint32_t d = blockIdx.x * kDigWaves + wave; d < nDocs; d += gridDim.x * kDigWaves) {
    const fmt_mt_doc_result h = hdrs[d];
    uint64_t acc = 0;
    if (h.status != FMT_OK) {  // a failed document: its status and failing seq only
      if (lane == 0)
        acc = digElem(1, 0, static_cast<uint32_t>(h.status)) + digElem(1, 1, static_cast<uint32_t>(h.fail_seq));
    } else {
      if (lane < 8) {
        const uint32_t f[8] = {static_cast<uint32_t>(h.status), static_cast<uint32_t>(h.cur_seq),
                               static_cast<uint32_t>(h.min_seq), h.n_leaves, h.n_chars, h.n_blocks, h.depth,
                               h.visible_len};
        uint32_t v = 0;
        for (int k = 0; k < 8; k++) v = k == lane ? f[k] : v;
        acc = digElem(1, static_cast<uint64_t>(lane), v);
      }
      const SumView V = views[d];
      for (uint32_t i = lane; i < h.n_leaves; i += 64) {
        const fmt_mt_leaf L = V.leaves[i];
        acc += digElem(2, i, static_cast<uint32_t>(L.ins_seq) | static_cast<uint64_t>(static_cast<uint32_t>(L.rm_seq)) << 32);
        acc += digElem(3, i, L.rm_clients);
        acc += digElem(4, i, L.char_off | static_cast<uint64_t>(L.len) << 32);
        acc += digElem(5, i, static_cast<uint16_t>(L.ins_client) | static_cast<uint64_t>(L.block) << 16 |
                                 static_cast<uint64_t>(L.pad) << 32);
        if (L.props == 0xFFFFu || L.props >= h.n_props) {
          acc += digElem(6, i, L.props == 0xFFFFu ? ~0ull : (1ull << 63) | L.props);  // (an id past the table: poisoned)
        } else {
          const fmt_mt_propset& P = V.props[L.props];
          const uint32_t n = P.n;
          acc += digElem(6, i, n);
          // (a wide set continues in the following records: tag 9 for entries 8 and up)
          for (uint32_t k = 0; k < n && k < FMT_MT_PROPS_KEYS_MAX && L.props + k / FMT_MT_PROPS_MAX < h.n_props; k++) {
            const uint32_t w = V.props[L.props + k / FMT_MT_PROPS_MAX].kv[k % FMT_MT_PROPS_MAX];
            acc += k < FMT_MT_PROPS_MAX ? digElem(7, static_cast<uint64_t>(i) * 8 + k, w) : digElem(9, static_cast<uint64_t>(i) * 64 + k, w);
          }
        }
      }
      if (V.rmHi != nullptr) {  // remove clients 64..127 (tag 10), 128..191 (11), 192..253 (12): leaves that have any
        for (uint32_t i = lane; i < h.n_leaves; i += 64) {
          for (int k = 0; k < 3; k++) {
            const uint64_t hi = V.rmHi[3 * static_cast<size_t>(i) + k];
            if (hi != 0) acc += digElem(10 + k, i, hi);
          }
        }
      }
      for (uint32_t u = lane; u < h.n_chars; u += 64) acc += digElem(8, u, V.chars[u]);
    }
    for (int off = 32; off > 0; off >>= 1) acc += static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(acc), off));
    if (lane == 0) out[d] = digMix(acc);
  }
}

hipError_t launchStateDigest(const fmt_mt_doc_result* hdrs, const SumView* views, uint32_t nDocs, uint64_t* out,
                             int numCUs, hipStream_t stream) {
  const uint32_t wanted = (nDocs + kDigWaves - 1) / kDigWaves;
  const uint32_t cap = static_cast<uint32_t>(numCUs) * 8u;
  const uint32_t grid = wanted < cap ? (wanted > 0 ? wanted : 1) : cap;
  hipLaunchKernelGGL(stateDigestKernel, dim3(grid), dim3(64 * kDigWaves), 0, stream, hdrs, views, nDocs, out);
  return hipGetLastError();
}

}  // namespace fmt_kernels
