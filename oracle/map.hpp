// oracle/map.hpp — TEST INFRASTRUCTURE ONLY (parity oracle for the SharedMap LWW path).
//
// Restates the sequenced (remote) path of MapKernel (packages/dds/map/src/mapKernel.ts:706-853)
// with the JS Map semantics it relies on, and SharedMap.summarizeCore (map.ts:176-246).
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/fmt.h"

namespace orc {

// JS Map<string, value> restricted to the operations MapKernel uses: set keeps the position of an
// existing key, delete/clear drop it, a later set re-appends it (ECMAScript Map insertion order).
class MapState {
 public:
  // sparse: key -> item index in a hash map (any key pool, the sparse path's oracle) instead of a
  // dense table of key_bound entries
  explicit MapState(uint32_t keyBound, bool sparse = false)
      : slot_(sparse ? 0 : keyBound, -1), keyBound_(keyBound), sparse_(sparse) {}
  // mapKernel.ts:802-850 "set" remote branch: sequencedData.set(key, {value}).
  void set(uint32_t key, uint32_t value, uint32_t seq);
  // mapKernel.ts:761-801 "delete" remote branch: sequencedData.delete(key).
  void del(uint32_t key);
  // mapKernel.ts:708-760 "clear" remote branch: sequencedData.clear().
  void clear();
  // Live entries in Map iteration (insertion) order: (key, value, birth seq).
  struct Entry {
    uint32_t key, value, birth;
  };
  std::vector<Entry> entries() const;
  void toSlots(fmt_map_slot* out, uint32_t keyBound) const;

 private:
  struct Item {
    uint32_t key, value, birth;
    bool live;
  };
  int slotOf(uint32_t key) const;
  void setSlot(uint32_t key, int s);
  std::vector<int> slot_;   // key → index in items_, -1 if absent (dense)
  std::unordered_map<uint32_t, int> map_;  // the same, sparse
  uint32_t keyBound_;
  bool sparse_;
  std::vector<Item> items_; // append-only with tombstones; order = Map insertion order
};

// MapKernel's local-client pending state (mapKernel.ts:132-139) with the reference's own shapes: an
// ordered list of entries (a set "lifetime" holding its pending keySets, a delete, a clear), built by
// set / delete / clear (:388-538), emptied by the local branches of the message handlers (:706-853)
// and by rollback (:633-700). A submission is named by its event index (the localOpMetadata
// identity); the reference's asserts become a false return.
class PendingMap {
 public:
  enum Type : uint32_t { kLifetime = 0, kDelete = 1, kClear = 2 };
  struct KeySet {
    uint32_t value, sub;
  };
  struct Entry {
    uint32_t type, key;
    std::vector<KeySet> keySets;  // lifetimes
    uint32_t sub;                 // the submission that created the entry
  };
  void set(uint32_t key, uint32_t value, uint32_t sub);  // :402-447
  void del(uint32_t key, uint32_t sub);                  // :453-490
  void clear(uint32_t sub);                              // :495-538
  // process(op, local = true, metadata = sub): the handlers' local branches (:714-723, :771-787, :812-835)
  bool ack(uint32_t kind, uint32_t key, uint32_t sub);
  // rollback(op, metadata = sub) (:633-700)
  bool rollback(uint32_t kind, uint32_t key, uint32_t sub);
  // internalIterator (:176-240) over the sequenced entries (Map order) and the pending entries:
  // (key, optimistic value, sequenced birth or FMT_MAP_PENDING_BIRTH | creating submission)
  std::vector<MapState::Entry> iterate(const std::vector<MapState::Entry>& sequenced) const;

 private:
  std::vector<Entry> pending_;
};

// map.ts:176-246: header blob {"blobs":[...],"content":{...}} plus blobN for values ≥ 8 KiB and
// for each 16 KiB flush; object keys enumerate array indices first (OrdinaryOwnPropertyKeys).
struct MapSummary {
  std::string header;
  std::vector<std::string> blobs;  // blob0, blob1, ...
};
MapSummary summarizeMap(const std::vector<MapState::Entry>& entries,
                        const std::vector<std::string>& keyNames,
                        const std::vector<std::string>& valueJson);

}  // namespace orc
