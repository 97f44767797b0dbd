// jsnum.h — JSON.stringify of a JS number on the host: ECMAScript Number::toString (ECMA-262
// §6.1.6.1.20) over the shortest round-trip digits, "null" for NaN / ±Infinity (SerializeJSONProperty),
// "0" for -0. The summary formatters write computed annotate-adjust values with it, so their bytes
// equal what the reference's serializer (shared-object-base/src/serializer.ts:120-123) writes.
#pragma once

#include <charconv>
#include <cmath>
#include <cstring>
#include <string>

namespace fmt_json {

// Writes at most `cap` bytes (no terminator) and returns the length (32 always suffices).
inline int jsNumber(double x, char* out, int cap) {
  char tmp[48];
  int n = 0;
  auto put = [&](char ch) {
    if (n < static_cast<int>(sizeof tmp)) tmp[n++] = ch;
  };
  if (std::isnan(x) || std::isinf(x)) {
    for (const char* p = "null"; *p; p++) put(*p);
  } else if (x == 0) {
    put('0');
  } else {
    if (x < 0) {
      put('-');
      x = -x;
    }
    // shortest digits d1.d2...dk e±E from to_chars (scientific), then the ECMAScript layout
    char sci[40];
    const auto r = std::to_chars(sci, sci + sizeof sci, x, std::chars_format::scientific);
    char digits[24];
    int k = 0, i = 0;
    const int len = static_cast<int>(r.ptr - sci);
    for (; i < len && sci[i] != 'e'; i++)
      if (sci[i] >= '0' && sci[i] <= '9') digits[k++] = sci[i];
    int e = 0;
    bool neg = false;
    for (i++; i < len; i++) {
      if (sci[i] == '-') neg = true;
      else if (sci[i] >= '0' && sci[i] <= '9') e = e * 10 + (sci[i] - '0');
    }
    if (neg) e = -e;
    while (k > 1 && digits[k - 1] == '0') k--;
    const int nn = e + 1;  // x = 0.d1...dk × 10^nn
    if (k <= nn && nn <= 21) {
      for (int t = 0; t < k; t++) put(digits[t]);
      for (int t = k; t < nn; t++) put('0');
    } else if (0 < nn && nn <= 21) {
      for (int t = 0; t < nn; t++) put(digits[t]);
      put('.');
      for (int t = nn; t < k; t++) put(digits[t]);
    } else if (-6 < nn && nn <= 0) {
      put('0');
      put('.');
      for (int t = 0; t < -nn; t++) put('0');
      for (int t = 0; t < k; t++) put(digits[t]);
    } else {
      put(digits[0]);
      if (k > 1) {
        put('.');
        for (int t = 1; t < k; t++) put(digits[t]);
      }
      put('e');
      put(nn - 1 >= 0 ? '+' : '-');
      const std::string es = std::to_string(nn - 1 >= 0 ? nn - 1 : 1 - nn);
      for (char ch : es) put(ch);
    }
  }
  const int w = n < cap ? n : cap;
  std::memcpy(out, tmp, static_cast<size_t>(w));
  return w;
}

inline std::string jsNumber(double x) {
  char b[48];
  return std::string(b, static_cast<size_t>(jsNumber(x, b, sizeof b)));
}

}  // namespace fmt_json
