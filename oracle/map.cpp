// oracle/map.cpp — TEST INFRASTRUCTURE ONLY. See map.hpp.
#include "map.hpp"

#include <algorithm>
#include <stdexcept>

#include "common.hpp"

namespace orc {

int MapState::slotOf(uint32_t key) const {
  if (!sparse_) return slot_.at(key);
  if (key >= keyBound_) throw std::out_of_range("key id >= key_bound");
  const auto it = map_.find(key);
  return it == map_.end() ? -1 : it->second;
}

void MapState::setSlot(uint32_t key, int s) {
  if (!sparse_) slot_[key] = s;
  else if (s < 0) map_.erase(key);
  else map_[key] = s;
}

void MapState::set(uint32_t key, uint32_t value, uint32_t seq) {
  const int s = slotOf(key);
  if (s >= 0 && items_[static_cast<size_t>(s)].live) {
    items_[static_cast<size_t>(s)].value = value;  // existing key keeps its position
    return;
  }
  setSlot(key, static_cast<int>(items_.size()));
  items_.push_back({key, value, seq, true});
}

void MapState::del(uint32_t key) {
  const int s = slotOf(key);
  if (s >= 0) items_[static_cast<size_t>(s)].live = false;
  setSlot(key, -1);
}

void MapState::clear() {
  for (auto& it : items_) {
    if (it.live) setSlot(it.key, -1);
    it.live = false;
  }
  items_.clear();
}

std::vector<MapState::Entry> MapState::entries() const {
  std::vector<Entry> out;
  for (const auto& it : items_)
    if (it.live) out.push_back({it.key, it.value, it.birth});
  return out;
}

void MapState::toSlots(fmt_map_slot* out, uint32_t keyBound) const {
  for (uint32_t k = 0; k < keyBound; k++) out[k] = {FMT_MAP_ABSENT, 0};
  for (const auto& it : items_)
    if (it.live) out[it.key] = {it.value, it.birth};
}

// ---------------------------------------------------------------- local-client pending state
void PendingMap::set(uint32_t key, uint32_t value, uint32_t sub) {
  // latestPendingEntry = findLast(pendingData, clear || entry.key === key) (:427-430)
  int latest = -1;
  for (int i = static_cast<int>(pending_.size()) - 1; i >= 0 && latest < 0; i--)
    if (pending_[i].type == kClear || pending_[i].key == key) latest = i;
  if (latest < 0 || pending_[latest].type != kLifetime) {  // a new lifetime (:431-437)
    pending_.push_back({kLifetime, key, {}, sub});
    latest = static_cast<int>(pending_.size()) - 1;
  }
  pending_[latest].keySets.push_back({value, sub});
}

void PendingMap::del(uint32_t key, uint32_t sub) { pending_.push_back({kDelete, key, {}, sub}); }

void PendingMap::clear(uint32_t sub) { pending_.push_back({kClear, 0, {}, sub}); }

bool PendingMap::ack(uint32_t kind, uint32_t key, uint32_t sub) {
  if (kind == FMT_MAP_CLEAR) {  // pendingData.shift() must be this clear (:714-723)
    if (pending_.empty() || pending_.front().type != kClear || pending_.front().sub != sub) return false;
    pending_.erase(pending_.begin());
    return true;
  }
  // findIndex(entry.type !== "clear" && entry.key === key) (:771-787, :812-835)
  size_t i = 0;
  while (i < pending_.size() && !(pending_[i].type != kClear && pending_[i].key == key)) i++;
  if (i == pending_.size()) return false;
  Entry& e = pending_[i];
  if (kind == FMT_MAP_DELETE) {
    if (e.type != kDelete || e.sub != sub) return false;
    pending_.erase(pending_.begin() + static_cast<long>(i));
    return true;
  }
  if (e.type != kLifetime || e.keySets.empty() || e.keySets.front().sub != sub) return false;
  e.keySets.erase(e.keySets.begin());  // keySets.shift()
  if (e.keySets.empty()) pending_.erase(pending_.begin() + static_cast<long>(i));
  return true;
}

bool PendingMap::rollback(uint32_t kind, uint32_t key, uint32_t sub) {
  if (kind == FMT_MAP_CLEAR) {  // pendingData.pop() must be this clear (:637-646)
    if (pending_.empty() || pending_.back().type != kClear || pending_.back().sub != sub) return false;
    pending_.pop_back();
    return true;
  }
  // findLastIndex(entry.type !== "clear" && entry.key === key) (:659-663)
  int i = static_cast<int>(pending_.size()) - 1;
  while (i >= 0 && !(pending_[i].type != kClear && pending_[i].key == key)) i--;
  if (i < 0) return false;
  Entry& e = pending_[i];
  if (e.type == kDelete) {
    if (kind != FMT_MAP_DELETE || e.sub != sub) return false;
    pending_.erase(pending_.begin() + i);
    return true;
  }
  if (kind != FMT_MAP_SET || e.keySets.empty() || e.keySets.back().sub != sub) return false;
  e.keySets.pop_back();
  if (e.keySets.empty()) pending_.erase(pending_.begin() + i);
  return true;
}

std::vector<MapState::Entry> PendingMap::iterate(const std::vector<MapState::Entry>& sequenced) const {
  std::vector<MapState::Entry> out;
  // getOptimisticLocalValue (:374-392) of a sequenced key with no pending delete / clear
  for (const auto& x : sequenced) {
    bool hidden = false;  // pendingData.some(clear || (delete && key === key)) (:190-195)
    for (const auto& e : pending_) hidden = hidden || e.type == kClear || (e.type == kDelete && e.key == x.key);
    if (hidden) continue;
    const Entry* latest = nullptr;
    for (const auto& e : pending_)
      if (e.type == kClear || e.key == x.key) latest = &e;
    out.push_back({x.key, latest == nullptr ? x.value : latest->keySets.back().value, x.birth});
  }
  for (size_t i = 0; i < pending_.size(); i++) {  // the pending lifetimes (:209-234)
    const Entry& e = pending_[i];
    if (e.type != kLifetime) continue;
    int lastDC = -1;  // findLastIndex(clear || (delete && key === e.key))
    for (size_t j = 0; j < pending_.size(); j++)
      if (pending_[j].type == kClear || (pending_[j].type == kDelete && pending_[j].key == e.key)) lastDC = static_cast<int>(j);
    if (static_cast<int>(i) <= lastDC) continue;
    bool inSeq = false;
    for (const auto& x : sequenced) inSeq = inSeq || x.key == e.key;
    if (inSeq && lastDC == -1) continue;
    out.push_back({e.key, e.keySets.back().value, FMT_MAP_PENDING_BIRTH | e.sub});
  }
  return out;
}

// String.prototype.length of a UTF-8 encoded text (UTF-16 code units).
static size_t utf16Length(const std::string& s) {
  size_t n = 0;
  for (size_t i = 0; i < s.size(); i++) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    if ((c & 0xC0) == 0x80) continue;  // continuation byte
    n += (c >= 0xF0) ? 2 : 1;
  }
  return n;
}

// JSON.stringify of {key: {"type":"Plain","value":<v>}} members in JS key order.
static void appendMember(std::string& out, bool& first, const std::string& key,
                         const std::string* value) {
  if (!first) out.push_back(',');
  first = false;
  jsonQuoteUtf8(out, key);
  out += ":{\"type\":\"Plain\"";
  if (value != nullptr) {
    out += ",\"value\":";
    out += *value;
  }
  out.push_back('}');
}

static std::vector<size_t> jsKeyOrder(const std::vector<MapState::Entry>& entries,
                                      const std::vector<std::string>& keyNames) {
  std::vector<std::pair<uint64_t, size_t>> idx;
  std::vector<size_t> rest;
  for (size_t i = 0; i < entries.size(); i++) {
    uint64_t v;
    if (isArrayIndexKey(keyNames.at(entries[i].key), &v)) idx.emplace_back(v, i);
    else rest.push_back(i);
  }
  std::sort(idx.begin(), idx.end());
  std::vector<size_t> order;
  for (auto& e : idx) order.push_back(e.second);
  for (size_t i : rest) order.push_back(i);
  return order;
}

MapSummary summarizeMap(const std::vector<MapState::Entry>& entries,
                        const std::vector<std::string>& keyNames,
                        const std::vector<std::string>& valueJson) {
  constexpr size_t kSeparateBlob = 8 * 1024;   // map.ts:190
  constexpr size_t kMaxBlob = 16 * 1024;       // map.ts:194
  const std::string kType = "Plain";
  MapSummary out;
  // getSerializedStorage iterates sequencedData (insertion order) into a plain object, so the
  // object — and everything derived from Object.entries(data) — enumerates array-index keys first.
  const std::vector<size_t> order = jsKeyOrder(entries, keyNames);
  std::vector<size_t> headerMembers;
  size_t currentSize = 0;
  auto flushHeader = [&](const std::vector<size_t>& members) {
    std::string j = "{";
    bool first = true;
    std::vector<MapState::Entry> sub;
    for (size_t i : members) sub.push_back(entries[i]);
    for (size_t k : jsKeyOrder(sub, keyNames)) {
      const auto& e = sub[k];
      const std::string* v = e.value == FMT_MAP_VALUE_UNDEFINED ? nullptr : &valueJson.at(e.value);
      appendMember(j, first, keyNames.at(e.key), v);
    }
    j.push_back('}');
    return j;
  };
  for (size_t i : order) {
    const auto& e = entries[i];
    const bool undef = e.value == FMT_MAP_VALUE_UNDEFINED;
    const size_t vlen = undef ? 0 : utf16Length(valueJson.at(e.value));
    if (!undef && vlen >= kSeparateBlob) {
      std::string j = "{";
      bool first = true;
      appendMember(j, first, keyNames.at(e.key), &valueJson.at(e.value));
      j.push_back('}');
      out.blobs.push_back(j);
    } else {
      currentSize += kType.size() + 21;
      currentSize += vlen;
      if (currentSize > kMaxBlob) {
        out.blobs.push_back(flushHeader(headerMembers));
        headerMembers.clear();
        currentSize = 0;
      }
      headerMembers.push_back(i);
    }
  }
  std::string h = "{\"blobs\":[";
  for (size_t b = 0; b < out.blobs.size(); b++) {
    if (b) h.push_back(',');
    h += "\"blob" + std::to_string(b) + "\"";
  }
  h += "],\"content\":";
  h += flushHeader(headerMembers);
  h.push_back('}');
  out.header = h;
  return out;
}

}  // namespace orc
