// huge_ckpt.h — the large → huge tier checkpoint record (mt_engine.h Doc::saveHuge writes it,
// huge_engine.h HugeDoc::loadFromLarge reads it).
//
// A document (no local events; relative positions, annotate-adjust and remove-order recording since
// round 6: the marker list is rebuilt from the leaves, the PropertiesManager records and remove-order
// entries stay in their HBM slabs, kPmN / kRmN carry their counts) that the large tier is about to outgrow — an op that could add more leaves than its 2048 rows,
// more text than 131071 units, take its last blocks or prop sets, or that names a writer past 63 —
// stops before that op. The large tier then writes its result slabs as at the end of a replay
// (leaves in document order with stamps, remove-client sets, char offsets, prop-set ids; its text;
// its prop sets) plus this record: what the slabs do not say — the exact B+tree (every block's child
// count, parent, children and needsScour flag, block ids kept), each leaf's id and block, the LRU
// heap in its array order, the free-block list, the collab window and counters, and the live
// obliterates. The huge tier rebuilds the same tree from it in its paged layout and replays on from
// that op, instead of from the document's first op (the reference grows one tree without bound,
// mergeTree.ts:1484-1517).
#pragma once
#include <cstdint>

namespace fmt_ckpt {

constexpr int kLeaves = 2048;  // LargeTier rows x 64
constexpr int kBlocks = 1023;  // LargeTier::kMaxBlocks (block ids 0..1022)
constexpr int kHeap = 1024;    // LargeTier::kHeapCap + 1 entries (1-based heap, heap.ts)
constexpr int kObSlots = 64;   // fmt_mt::kObCap

// head words
enum : int {
  kNextLo = 0, kNextHi = 1, kN = 2, kNChars = 3, kRoot = 4, kNFree = 5, kHeapN = 6, kNProps = 7,
  kCurSeq = 8, kMinSeq = 9, kNextId = 10, kCuN = 11, kObCounts = 12 /* obSeqN | obStartN << 16 */,
  kObUsedLo = 13, kObUsedHi = 14, kPmN = 15 /* annotate-adjust: PropertiesManager records */,
  kRmN = 16 /* remove-order entries (leaf ids) in the document's slab */, kHeadWords = 17
};
// sections
constexpr int kLeafW4 = kHeadWords;             // [kLeaves] W4: leaf id | Marker << 23 | insert client << 24
constexpr int kLeafBlk = kLeafW4 + kLeaves;     // [kLeaves] the leaf's block id
constexpr int kBlk = kLeafBlk + kLeaves;        // [kBlocks x 10] count | leaf << 8 | (uint8)needsScour << 16,
constexpr int kBlkWords = 10;                   //   parent (0xFFFFFFFF: none), child[8]
constexpr int kHeapOff = kBlk + kBlkWords * kBlocks;  // [kHeap x 2] maxSeq, leaf id
constexpr int kFree = kHeapOff + 2 * kHeap;     // [kBlocks] free block ids, bottom of the stack first
constexpr int kOb = kFree + kBlocks;            // [kObSlots x 6] startId, endId, startOff, endOff, seq, client,
constexpr int kObSeq = kOb + 6 * kObSlots;      //   then seqOrdered and startOrdered (one slot id per word)
constexpr int kObStart = kObSeq + kObSlots;
constexpr int kWords = kObStart + kObSlots;
constexpr uint32_t kNoParent = 0xFFFFFFFFu;

// Internal header status of a document the large tier checkpointed for the huge tier (the runtime
// replaces it with the huge tier's result; never leaves the runtime).
constexpr int kStatusHuge = -35;

}  // namespace fmt_ckpt
