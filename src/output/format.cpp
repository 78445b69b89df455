// format.cpp — reference-identical output framing.
//
//   Input Data:\n            (main.cu:166)
//   <input echoed verbatim>  (main.cu:180)
//   26 dashes\n              (main.cu:210)
//   word\tcount\n ...        (main.cu:213, first-occurrence order)
//   26 dashes\n              (main.cu:217)
//   Total Count:N\n          (main.cu:218)
//
// Counts are u64 (the reference's int overflows at 2^31).  `list_rows=false`
// and `top_k` exist for multi-GB inputs whose tables have millions of rows.
#include <algorithm>
#include <numeric>
#include <string>

#include "wc/wc.hpp"

namespace wc {

static const char kDashes[] = "--------------------------\n";

std::string format_output(const KeyTable& t, const uint8_t* echo, uint64_t echo_len, bool echo_input,
                          bool list_rows, uint64_t top_k) {
  std::string out;
  out.reserve(64 + (echo_input ? echo_len : 0) + (list_rows ? t.size() * 16 : 0));
  out += "Input Data:\n";
  if (echo_input && echo) out.append(reinterpret_cast<const char*>(echo), echo_len);
  out += kDashes;
  char num[32];
  auto row = [&](size_t i) {
    out += t.words[i];
    out += '\t';
    snprintf(num, sizeof num, "%llu\n", (unsigned long long)t.counts[i]);
    out += num;
  };
  if (list_rows) {
    if (top_k && top_k < t.size()) {
      std::vector<size_t> idx(t.size());
      std::iota(idx.begin(), idx.end(), 0);
      std::partial_sort(idx.begin(), idx.begin() + top_k, idx.end(), [&](size_t a, size_t b) {
        return t.counts[a] != t.counts[b] ? t.counts[a] > t.counts[b] : t.first_off[a] < t.first_off[b];
      });
      for (uint64_t k = 0; k < top_k; ++k) row(idx[k]);
    } else {
      for (size_t i = 0; i < t.size(); ++i) row(i);
    }
  }
  out += kDashes;
  snprintf(num, sizeof num, "%llu\n", (unsigned long long)t.total);
  out += "Total Count:";
  out += num;
  return out;
}

}  // namespace wc
