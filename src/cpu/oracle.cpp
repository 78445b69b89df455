// oracle.cpp — CPU word count paths.
//
// cpu::count: BASELINE config 1 ("test.txt word count on CPU reference path,
// single-thread std::map").  It keys a hash map by the word BYTES (not by the
// GPU's packed key) so it independently checks the GPU key scheme.
//
// cpu::count_reference_compat: reproduces the reference program's observable
// quirks for differential testing: fgets(…,100)
// records (main.cu:179), `strlen < 2` stops ALL input (main.cu:185-186), empty
// tokens for repeated delimiters (main.cu:188-194), CR ends the record
// (main.cu:195-196), the last token of an un-terminated line is dropped, and
// the reducer's asymmetric prefix compare (main.cu:57-67) with its
// inclusive scan (main.cu:81) against a zero-filled output slot.  It is a
// re-derivation of the behaviour, not a copy of the code, and has no capacity
// limits (the reference's overflows are undefined behaviour).
#include <string>
#include <string_view>
#include <unordered_map>

#include "../kernels/keys.hpp"
#include "wc/wc.hpp"

namespace wc {
namespace cpu {

KeyTable count(const uint8_t* text, uint64_t n, uint64_t global_base) {
  struct Ent {
    uint64_t count, first;
  };
  std::unordered_map<std::string_view, uint32_t> index;
  std::vector<std::string_view> words;
  std::vector<Ent> ents;
  const char* p = reinterpret_cast<const char*>(text);
  uint64_t i = 0;
  while (i < n) {
    while (i < n && is_delim((uint8_t)p[i])) ++i;
    if (i >= n) break;
    const uint64_t s = i;
    while (i < n && !is_delim((uint8_t)p[i])) ++i;
    std::string_view w(p + s, i - s);
    auto it = index.find(w);
    if (it == index.end()) {
      index.emplace(w, (uint32_t)words.size());
      words.push_back(w);
      ents.push_back({1, global_base + s});
    } else {
      ents[it->second].count++;
    }
  }
  KeyTable t;  // insertion order == first-occurrence order
  t.words.reserve(words.size());
  for (size_t k = 0; k < words.size(); ++k) {
    t.words.emplace_back(words[k]);
    t.counts.push_back(ents[k].count);
    t.first_off.push_back(ents[k].first);
    t.total += ents[k].count;
  }
  return t;
}

KeyTable count_reference_compat(const uint8_t* text, uint64_t n, std::string* echo) {
  // Split into fgets-style records of at most 99 bytes (a record ends after '\n').
  std::vector<std::string> tokens;
  uint64_t i = 0;
  while (i < n) {
    uint64_t e = i;
    while (e < n && e - i < 99 && text[e] != '\n') ++e;
    if (e < n && text[e] == '\n' && e - i < 99) ++e;
    std::string rec(reinterpret_cast<const char*>(text) + i, e - i);
    i = e;
    const size_t nul = rec.find('\0');  // strlen semantics
    if (nul != std::string::npos) rec.resize(nul);
    if (echo) echo->append(rec);  // printf("%s") of the record precedes the strlen < 2 check (main.cu:180-186)
    if (rec.size() < 2) break;
    std::string cur;
    for (char c : rec) {
      if (c == ' ' || c == '\r' || c == '\n') {
        tokens.push_back(cur);
        cur.clear();
        if (c == '\r') break;
      } else {
        cur.push_back(c);
      }
    }
  }
  // Reducer: output slots start zeroed; scan j = 0..nIndex inclusive with a
  // prefix test "new word is a prefix of the slot".
  std::vector<std::string> keys(1);  // slot nIndex is the zeroed next slot
  std::vector<uint64_t> cnts(1, 0);
  size_t used = 0;
  for (const std::string& w : tokens) {
    bool hit = false;
    for (size_t j = 0; j <= used && !hit; ++j) {
      if (keys[j].compare(0, w.size(), w) == 0 && keys[j].size() >= w.size()) {
        cnts[j]++;
        hit = true;
      }
    }
    if (hit) continue;
    // Append at nIndex: copies the bytes over whatever the slot held (no NUL
    // is written, so a longer stale word keeps its tail).
    std::string& slot = keys[used];
    if (slot.size() < w.size()) slot.resize(w.size());
    slot.replace(0, w.size(), w);
    cnts[used] = 1;
    ++used;
    keys.emplace_back();
    cnts.push_back(0);
  }
  KeyTable t;
  for (size_t j = 0; j < used; ++j) {
    t.words.push_back(keys[j]);
    t.counts.push_back(cnts[j]);
    t.first_off.push_back(j);
    t.total += cnts[j];
  }
  return t;
}

}  // namespace cpu
}  // namespace wc
