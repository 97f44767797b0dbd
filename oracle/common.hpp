// oracle/common.hpp — TEST INFRASTRUCTURE ONLY (parity oracle). Never linked into the product.
//
// Helpers shared by the CPU restatements: the XSadd PRNG and the `makeRandom` distributions of
// @fluid-private/stochastic-test-utils, and an ECMAScript-exact JSON writer for the subset of
// values the hot path serializes (strings, integers, pre-serialized JSON value texts).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

namespace orc {

// XSadd, packages/test/stochastic-test-utils/src/xsadd.ts:38-89. Seeds beyond those given are 0.
class XSadd {
 public:
  explicit XSadd(std::vector<uint32_t> seed) {
    seed.resize(4, 0);
    int32_t s[4];
    for (int i = 0; i < 4; i++) s[i] = static_cast<int32_t>(seed[i]);
    // LCG scramble with the Borosh-Niederreiter multiplier; repeat until the state is non-zero.
    for (int i = 1; i < 8 || (s[0] | s[1] | s[2] | s[3]) == 0; i++) {
      const uint32_t prev = static_cast<uint32_t>(s[(i - 1) & 3]);
      const uint32_t mixed = prev ^ (prev >> 30);
      const uint32_t term = static_cast<uint32_t>(i) + 0x6c078965u * mixed;  // imul wraps
      s[i & 3] = static_cast<int32_t>(static_cast<uint32_t>(s[i & 3]) ^ term);
    }
    x_ = static_cast<uint32_t>(s[0]);
    y_ = static_cast<uint32_t>(s[1]);
    z_ = static_cast<uint32_t>(s[2]);
    w_ = static_cast<uint32_t>(s[3]);
    for (int i = 0; i < 8; i++) uint32();
  }
  uint32_t uint32() {
    uint32_t t = x_;
    x_ = y_;
    y_ = z_;
    z_ = w_;
    t ^= t << 15;
    t ^= t >> 18;
    t ^= w_ << 11;
    w_ = t;
    return w_ + z_;
  }
  // Discards the weak low bits of both samples (xsadd.ts:82).
  double uint53() {
    const double hi = static_cast<double>(uint32() >> 6);
    const double lo = static_cast<double>(uint32() >> 5);
    return hi * 134217728.0 + lo;
  }
  double float64() { return uint53() / 9007199254740992.0; }

 private:
  uint32_t x_, y_, z_, w_;
};

// makeRandom, packages/test/stochastic-test-utils/src/random.ts:49-95 (integer/real/pick/string).
class Random {
 public:
  explicit Random(std::vector<uint32_t> seed) : eng_(std::move(seed)) {}
  // distributions/integer.ts:19-51 (division + rejection, inclusive bounds).
  int64_t integer(int64_t min, int64_t max) {
    const double range = static_cast<double>(max - min + 1);
    const double divisor = std::trunc(9007199254740992.0 / range);
    double r;
    do {
      r = eng_.uint53() / divisor;
    } while (r >= range);
    return static_cast<int64_t>(std::trunc(r)) + min;
  }
  // distributions/real.ts:14-21.
  double real(double min = 0, double max = 1) {
    const double a = eng_.float64();
    return (1 - a) * min + a * max;
  }
  bool boolean(double p = 0.5) { return eng_.float64() < p; }
  std::string string(int len) {
    static const char* kBase58 = "123456789abcdefghijkmnopqrstuvwxyzABCDEFGHJKLMNPQRSTUVWXYZ";
    std::string s;
    for (int i = 0; i < len; i++) s.push_back(kBase58[integer(0, 57)]);
    return s;
  }
  XSadd& engine() { return eng_; }

 private:
  XSadd eng_;
};

// ---------------------------------------------------------------------------------------------
// JSON (ECMAScript JSON.stringify semantics for strings and integers).
// ---------------------------------------------------------------------------------------------
inline void appendUtf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

// QuoteJSONString (ES2019 well-formed): short escapes, \u00xx for other controls, lone
// surrogates as \udxxx, everything else literal (UTF-8 encoded here).
inline void jsonQuoteUtf16(std::string& out, const char16_t* s, size_t n) {
  static const char* kHex = "0123456789abcdef";
  out.push_back('"');
  for (size_t i = 0; i < n; i++) {
    const uint32_t c = s[i];
    switch (c) {
      case '"': out += "\\\""; continue;
      case '\\': out += "\\\\"; continue;
      case '\b': out += "\\b"; continue;
      case '\f': out += "\\f"; continue;
      case '\n': out += "\\n"; continue;
      case '\r': out += "\\r"; continue;
      case '\t': out += "\\t"; continue;
      default: break;
    }
    if (c < 0x20) {
      out += "\\u00";
      out.push_back(kHex[c >> 4]);
      out.push_back(kHex[c & 15]);
    } else if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
      appendUtf8(out, 0x10000 + ((c - 0xD800) << 10) + (static_cast<uint32_t>(s[i + 1]) - 0xDC00));
      i++;
    } else if (c >= 0xD800 && c <= 0xDFFF) {
      out += "\\u";
      for (int sh = 12; sh >= 0; sh -= 4) out.push_back(kHex[(c >> sh) & 15]);
    } else {
      appendUtf8(out, c);
    }
  }
  out.push_back('"');
}

inline void jsonQuoteUtf8(std::string& out, const std::string& s) {
  // Decode UTF-8 to UTF-16 first so the escaping rules above apply uniformly.
  std::u16string u;
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
    else { cp = c & 0x07; n = 4; }
    for (int k = 1; k < n && i + k < s.size(); k++) cp = (cp << 6) | (static_cast<unsigned char>(s[i + k]) & 0x3F);
    i += n;
    if (cp >= 0x10000) {
      cp -= 0x10000;
      u.push_back(static_cast<char16_t>(0xD800 + (cp >> 10)));
      u.push_back(static_cast<char16_t>(0xDC00 + (cp & 0x3FF)));
    } else {
      u.push_back(static_cast<char16_t>(cp));
    }
  }
  jsonQuoteUtf16(out, u.data(), u.size());
}

inline void jsonInt(std::string& out, long long v) { out += std::to_string(v); }

// CanonicalNumericIndexString for array indices: "0" or [1-9][0-9]* with value < 2^32 - 1.
// JS objects enumerate such keys first, ascending (OrdinaryOwnPropertyKeys).
inline bool isArrayIndexKey(const std::string& k, uint64_t* value) {
  if (k.empty() || k.size() > 10) return false;
  if (k.size() > 1 && k[0] == '0') return false;
  uint64_t v = 0;
  for (char c : k) {
    if (c < '0' || c > '9') return false;
    v = v * 10 + static_cast<uint64_t>(c - '0');
  }
  if (v >= 4294967295ull) return false;
  if (value) *value = v;
  return true;
}

}  // namespace orc
