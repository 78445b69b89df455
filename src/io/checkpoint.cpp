// checkpoint.cpp — see checkpoint.hpp.
#include "io/checkpoint.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <unordered_map>

#include "common/hip_util.hpp"
#include "io/source.hpp"

namespace wc {
namespace {

constexpr char kMagic[8] = {'W', 'C', 'C', 'K', 'P', 'T', '0', '1'};

bool delim(uint8_t c) { return c == ' ' || c == '\r' || c == '\n'; }

struct Fnv {
  uint64_t h = 1469598103934665603ull;
  void add(const void* p, size_t n) {
    const auto* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  }
};

struct Writer {
  std::string buf;
  template <class T>
  void put(const T& v) { buf.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
  void bytes(const std::string& s) { buf.append(s); }
};

struct Reader {
  const std::string& buf;
  size_t pos = 0;
  template <class T>
  T get() {
    if (pos + sizeof(T) > buf.size()) fail("checkpoint truncated");
    T v;
    std::memcpy(&v, buf.data() + pos, sizeof(T));
    pos += sizeof(T);
    return v;
  }
  std::string bytes(size_t n) {
    if (pos + n > buf.size()) fail("checkpoint truncated");
    std::string s = buf.substr(pos, n);
    pos += n;
    return s;
  }
};

void pread_all(int fd, uint8_t* dst, uint64_t n, uint64_t off, const std::string& file) {
  if (pread_parallel(fd, dst, n, off) != n) fail("read failed (file shrank?): " + file);
}

}  // namespace

void merge_tables(KeyTable& acc, const KeyTable& add) {
  std::unordered_map<std::string, size_t> at;
  at.reserve(acc.size() + add.size());
  for (size_t i = 0; i < acc.size(); ++i) at.emplace(acc.words[i], i);
  bool reorder = false;
  for (size_t i = 0; i < add.size(); ++i) {
    auto it = at.find(add.words[i]);
    if (it == at.end()) {
      if (!acc.first_off.empty() && add.first_off[i] < acc.first_off.back()) reorder = true;
      at.emplace(add.words[i], acc.size());
      acc.words.push_back(add.words[i]);
      acc.counts.push_back(add.counts[i]);
      acc.first_off.push_back(add.first_off[i]);
    } else {
      const size_t j = it->second;
      acc.counts[j] += add.counts[i];
      if (add.first_off[i] < acc.first_off[j]) {
        acc.first_off[j] = add.first_off[i];
        reorder = true;
      }
    }
  }
  acc.total += add.total;
  if (!reorder) return;
  std::vector<size_t> idx(acc.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return acc.first_off[a] < acc.first_off[b]; });
  KeyTable o;
  o.total = acc.total;
  o.words.reserve(idx.size());
  o.counts.reserve(idx.size());
  o.first_off.reserve(idx.size());
  for (size_t i : idx) {
    o.words.push_back(std::move(acc.words[i]));
    o.counts.push_back(acc.counts[i]);
    o.first_off.push_back(acc.first_off[i]);
  }
  acc = std::move(o);
}

std::string checkpoint_path(const std::string& base, int rank, int world) {
  if (world <= 1) return base;
  return base + ".r" + std::to_string(rank) + "of" + std::to_string(world);
}

bool checkpoint_exists(const std::string& path) {
  struct stat s;
  return ::stat(path.c_str(), &s) == 0;
}

void save_checkpoint(const std::string& path, const Checkpoint& c) {
  Writer w;
  w.buf.append(kMagic, sizeof(kMagic));
  w.put<uint32_t>(2);  // format version (2: + prefix fingerprint)
  w.put(c.rank);
  w.put(c.world);
  w.put(c.intervals);
  w.put(c.input_size);
  w.put(c.begin);
  w.put(c.end);
  w.put(c.next);
  w.put(c.prefix_fp);
  w.put(c.table.total);
  w.put<uint64_t>(c.table.size());
  for (size_t i = 0; i < c.table.size(); ++i) {
    w.put<uint32_t>((uint32_t)c.table.words[i].size());
    w.put(c.table.counts[i]);
    w.put(c.table.first_off[i]);
    w.bytes(c.table.words[i]);
  }
  Fnv f;
  f.add(w.buf.data(), w.buf.size());
  w.put(f.h);

  const std::string tmp = path + ".tmp";
  const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) fail("cannot write checkpoint " + tmp);
  const char* p = w.buf.data();
  size_t n = w.buf.size();
  while (n) {
    const ssize_t k = ::write(fd, p, n);
    if (k <= 0) {
      ::close(fd);
      fail("checkpoint write failed: " + tmp);
    }
    p += k;
    n -= (size_t)k;
  }
  if (::fsync(fd) != 0 || ::close(fd) != 0) fail("checkpoint fsync failed: " + tmp);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) fail("checkpoint rename failed: " + path);
}

Checkpoint load_checkpoint(const std::string& path) {
  std::string buf;
  try {
    buf = read_file(path);
  } catch (const Error&) {
    fail("cannot open checkpoint " + path);
  }
  if (buf.size() < sizeof(kMagic) + 8 || std::memcmp(buf.data(), kMagic, sizeof(kMagic)) != 0)
    fail("not a wordcount checkpoint: " + path);
  Fnv f;
  f.add(buf.data(), buf.size() - 8);
  uint64_t want;
  std::memcpy(&want, buf.data() + buf.size() - 8, 8);
  if (f.h != want) fail("checkpoint checksum mismatch (corrupt file): " + path);
  const std::string body = buf.substr(0, buf.size() - 8);
  Reader r{body, sizeof(kMagic)};
  const uint32_t version = r.get<uint32_t>();
  if (version != 1 && version != 2) fail("unsupported checkpoint version: " + path);
  Checkpoint c;
  c.rank = r.get<uint32_t>();
  c.world = r.get<uint32_t>();
  c.intervals = r.get<uint32_t>();
  c.input_size = r.get<uint64_t>();
  c.begin = r.get<uint64_t>();
  c.end = r.get<uint64_t>();
  c.next = r.get<uint64_t>();
  c.prefix_fp = version >= 2 ? r.get<uint64_t>() : 0;  // 0: not recorded (version 1)
  c.table.total = r.get<uint64_t>();
  const uint64_t rows = r.get<uint64_t>();
  if (c.next < c.begin || c.next > c.end) fail("checkpoint offsets inconsistent: " + path);
  c.table.words.reserve(rows);
  c.table.counts.reserve(rows);
  c.table.first_off.reserve(rows);
  for (uint64_t i = 0; i < rows; ++i) {
    const uint32_t len = r.get<uint32_t>();
    c.table.counts.push_back(r.get<uint64_t>());
    c.table.first_off.push_back(r.get<uint64_t>());
    c.table.words.push_back(r.bytes(len));
  }
  if (r.pos != body.size()) fail("checkpoint has trailing bytes: " + path);
  return c;
}

uint64_t prefix_fingerprint(int fd, uint64_t begin, uint64_t next, const std::string& file) {
  Fnv f;
  const uint64_t n = next - begin;
  uint8_t b[4096];
  for (uint64_t i = 0; i < 256 && n >= 32; ++i) {
    const uint64_t off = begin + (n - 32) * i / 255;
    pread_all(fd, b, 32, off, file);
    f.add(reinterpret_cast<const char*>(b), 32);
  }
  const uint64_t tail = std::min<uint64_t>(n, sizeof(b));
  if (tail) {
    pread_all(fd, b, tail, next - tail, file);
    f.add(reinterpret_cast<const char*>(b), tail);
  }
  return f.h;
}

Checkpoint open_checkpoint(const std::string& path, bool resume, const std::string& file, uint64_t input_size,
                           uint64_t begin, uint64_t end, int rank, int world) {
  if (resume && checkpoint_exists(path)) {
    Checkpoint k = load_checkpoint(path);
    if (k.input_size != input_size || k.begin != begin || k.end != end || k.rank != (uint32_t)rank ||
        k.world != (uint32_t)world)
      fail("checkpoint " + path + " was written for another input or GPU count");
    if (k.prefix_fp) {
      const int fd = ::open(file.c_str(), O_RDONLY);
      if (fd < 0) fail("cannot open " + file);
      uint64_t fp = 0;
      try {
        fp = prefix_fingerprint(fd, k.begin, k.next, file);
      } catch (...) {
        ::close(fd);
        throw;
      }
      ::close(fd);
      if (fp != k.prefix_fp) fail("checkpoint " + path + ": the counted part of " + file + " changed since it was written");
    }
    std::fprintf(stderr, "wordcount: rank %d resumes at byte %llu of [%llu, %llu) (%u interval(s) done)\n", rank,
                 (unsigned long long)k.next, (unsigned long long)k.begin, (unsigned long long)k.end, k.intervals);
    return k;
  }
  Checkpoint k;
  k.input_size = input_size;
  k.begin = k.next = begin;
  k.end = end;
  k.rank = (uint32_t)rank;
  k.world = (uint32_t)world;
  return k;
}

void run_checkpointed(const std::string& file, Checkpoint& c, uint64_t interval, const std::string& path,
                      const std::function<KeyTable(const uint8_t*, uint64_t, uint64_t)>& count_interval) {
  WC_CHECK(interval > 0, "checkpoint interval must be positive");
  uint32_t stop_after = 0;
  if (const char* e = std::getenv("WC_CKPT_STOP_AFTER")) stop_after = (uint32_t)std::strtoul(e, nullptr, 10);
  const int fd = ::open(file.c_str(), O_RDONLY);
  if (fd < 0) fail("cannot open " + file);
  std::vector<uint8_t> buf;
  uint32_t written = 0;
  try {
    while (c.next < c.end) {
      // Interval [next, next+len): cut after its last delimiter so every token
      // lies in one interval; a word longer than the interval widens the read.
      uint64_t want = std::min(interval, c.end - c.next), len = 0;
      for (;;) {
        buf.resize(want);
        pread_all(fd, buf.data(), want, c.next, file);
        if (c.next + want == c.end) {
          len = want;
          break;
        }
        uint64_t cut = want;
        while (cut > 0 && !delim(buf[cut - 1])) --cut;
        if (cut) {
          len = cut;
          break;
        }
        want = std::min(want * 2, c.end - c.next);
      }
      merge_tables(c.table, count_interval(buf.data(), len, c.next));
      c.next += len;
      c.intervals++;
      if (!path.empty()) c.prefix_fp = prefix_fingerprint(fd, c.begin, c.next, file);
      if (!path.empty()) {
        save_checkpoint(path, c);
        WC_LOG(LOG_INFO, "checkpoint %s: rank %u interval %u, next byte %llu of %llu, %zu keys", path.c_str(), c.rank,
               c.intervals, (unsigned long long)c.next, (unsigned long long)c.end, c.table.size());
        if (stop_after && ++written == stop_after && c.next < c.end)
          fail("WC_CKPT_STOP_AFTER: stopped after " + std::to_string(written) + " checkpoint(s)");
      }
    }
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
}

}  // namespace wc
