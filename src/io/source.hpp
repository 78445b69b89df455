// source.hpp — input sources.
//
// Reference: main.cu:167-206 reads ./test.txt with fgets(…,100) into fixed
// records.  Here input is one logical byte stream; a rank (GPU) owns every
// token whose FIRST byte lies in its byte range [start, end), so
// shard_range() drops a leading partial token and extends past `end` to
// finish the last one.
#pragma once
#include <stdint.h>

#include <string>

#include "wc/wc.hpp"

namespace wc {

struct ShardRange {
  uint64_t begin = 0, end = 0;  // bytes to read; tokens owned start in [begin, end)
};

// Size of a file (throws on error).
uint64_t file_size(const std::string& path);
// Ownership-adjusted byte range of shard `rank` of `world` over a file.
ShardRange shard_range(const std::string& path, int rank, int world);
// Same over a memory buffer.
ShardRange shard_range_mem(const uint8_t* p, uint64_t n, int rank, int world);

// Reads [begin, end) of a file with pread (streams files larger than HBM/RAM).
class FileSource : public ChunkSource {
 public:
  FileSource(const std::string& path, uint64_t begin, uint64_t end);
  ~FileSource() override;
  uint64_t read(uint8_t* dst, uint64_t cap) override;

 private:
  int fd_ = -1;
  uint64_t pos_, end_;
};

// Replays a host-resident pool of self-contained chunks (each ends with a
// delimiter) until `total` bytes were produced: the 1 TB host-staged config.
class ReplaySource : public ChunkSource {
 public:
  ReplaySource(const uint8_t* pool, uint64_t pool_bytes, uint64_t total);
  uint64_t read(uint8_t* dst, uint64_t cap) override;

 private:
  const uint8_t* pool_;
  uint64_t pool_bytes_, total_, produced_ = 0, pos_ = 0;
};

std::string read_file(const std::string& path);

// pread of [off, off+n) into dst split over worker threads; returns the bytes
// read (short only at end of file), throws on a read error.
uint64_t pread_parallel(int fd, uint8_t* dst, uint64_t n, uint64_t off);

}  // namespace wc
