// checkpoint.hpp — checkpoint / resume of a long (host-staged) count.
//
// Reference: none — /root/reference/main.cu:133-162 is one in-memory pass and
// SURVEY §5.4 lists checkpointing as the optional extra for the 1 TB
// host-staged config.  Design: a rank walks its byte range in intervals that
// end on a delimiter; after each interval the engine's table is finalised
// (compact + first-occurrence sort on the GPU), folded into a host running
// table and written, together with the next byte offset, to a per-rank file
// (tmp + fsync + rename, so a crash leaves the previous checkpoint intact).
// Resume = load the table, skip to the saved offset, continue.  The key table
// is tiny next to the text (a 1M-word vocabulary is ~30 MB), so a checkpoint
// every few GiB costs well under 1 % of the run.
#pragma once
#include <stdint.h>

#include <functional>
#include <string>

#include "wc/wc.hpp"

namespace wc {

struct Checkpoint {
  uint64_t input_size = 0;      // size of the input (guards against resuming on another file)
  uint64_t begin = 0, end = 0;  // this rank's owned range
  uint64_t next = 0;            // first byte not yet counted (begin <= next <= end)
  uint32_t rank = 0, world = 1;
  uint32_t intervals = 0;       // intervals counted so far
  uint64_t prefix_fp = 0;       // fingerprint of the counted bytes [begin, next) (prefix_fingerprint)
  KeyTable table;               // running table, first-occurrence order
};

// Fingerprint of the bytes [begin, next) of an open input: FNV-1a-64 over 256
// evenly spaced 32-byte samples and the last 4 KiB before `next`.  A resume
// re-reads them, so an input modified in place (same size) is refused.
uint64_t prefix_fingerprint(int fd, uint64_t begin, uint64_t next, const std::string& file);

// Fold `add` into `acc`: counts add, first_off takes the min, rows stay in
// first-occurrence order (the output contract, main.cu:208-218).
void merge_tables(KeyTable& acc, const KeyTable& add);

// Atomic write (path.tmp -> fsync -> rename).  Format: "WCCKPT01" magic,
// fixed header, rows (u32 len, u64 count, u64 first_off, bytes), FNV-1a-64
// trailer over everything before it.
void save_checkpoint(const std::string& path, const Checkpoint& c);
// Throws wc::Error on a missing, truncated, corrupt or foreign file.
Checkpoint load_checkpoint(const std::string& path);
bool checkpoint_exists(const std::string& path);
// Per-rank file name: "<base>" for world 1, "<base>.r<rank>of<world>" otherwise.
std::string checkpoint_path(const std::string& base, int rank, int world);

// Rank `rank` of `world` over [begin, end) of `file` (input_size bytes): the
// checkpoint at `path` when `resume` and it exists (validated against the input
// size, range, rank, world and the fingerprint of the counted prefix; throws
// otherwise), else a fresh one.
Checkpoint open_checkpoint(const std::string& path, bool resume, const std::string& file, uint64_t input_size,
                           uint64_t begin, uint64_t end, int rank, int world);

// Counts [c.begin, c.end) of `file` in delimiter-aligned intervals of about
// `interval` bytes, starting at c.next (resume) and folding into c.table.
// `count_interval(host_ptr, len, global_base)` counts one interval and returns
// its table.  A checkpoint is written after every interval when `path` is
// non-empty.  Env WC_CKPT_STOP_AFTER=N (fault injection for tests) throws
// after the N-th checkpoint of this call is on disk, as a crash would.
void run_checkpointed(const std::string& file, Checkpoint& c, uint64_t interval, const std::string& path,
                      const std::function<KeyTable(const uint8_t*, uint64_t, uint64_t)>& count_interval);

}  // namespace wc
