// merge.cpp — cross-GPU merge of per-rank key tables.
//
// Keys are variable-length words, so per-rank tables are not index-aligned.
// Two protocols (Options::merge_mode), all device-side, RCCL over xGMI or loopback.
//
// SHUFFLE (default) — the MapReduce shuffle proper, W-way parallel merge work:
//  1. owner(key) = high bits of the placement hash; count rows / long-word
//     bytes per owner, all-gather the W x 2 count matrix (+ max offset)    tiny
//  2. pack rows (40 B) + long-word bytes by owner, RCCL all-to-all         ~V x 40 B
//  3. owner merges what it received in a global hash table (row-id claims,
//     device-scope count / min-offset atomics for the rows after the claiming
//     one, whose own values the compaction folds in) and compacts it
//  4. gather the merged rows + bytes to rank 0 (broadcast for all_ranks)   ~V x 40 B
// Each rank merges ~V/W keys instead of sorting all W x V, and only rank 0
// orders the final table; the merge is a few tens of microseconds of xGMI.
//
// DENSE (merge_mode 1) — the dictionary + dense-vector protocol of SURVEY §5.8:
//  1-3. as SHUFFLE: the owners build the dictionary union (each owner merges
//     only its ~V/W keys; no rank sorts the whole union)
//  4. owners' key counts all-gathered -> global id = owner base + compact index;
//     ids go back to the senders (reverse all-to-all, 4 B per row)
//  5. each rank scatters its local counts / first offsets into dense u64[V]
//     vectors by id; reduce-scatter(sum) + reduce-scatter(min), all-gather
//  6. dictionary rows + bytes gathered to rank 0 (broadcast for all_ranks)
// Every rank ends with identical id-indexed count vectors.  Ring
// reduce-scatter over 7 xGMI links moves ~V x 8 B x (W-1)/W per rank per vector.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../engine/engine_impl.hpp"
#include "comm.hpp"

namespace wc {

namespace {
template <class T>
T* take_aligned(DeviceArena& A, size_t n) {
  return A.take_n<T>(n ? n : 1);
}

// Pinned host words of one merge (W <= 64): async H2D copies from them need no
// host sync before the merge returns.  Fixed slots: max offset, source bases,
// own bytes, gather bases.
enum : size_t { HW_MX = 0, HW_BASE = 8, HW_OWNB = 160, HW_GBASE = 192, HW_SEG = 336, HW_WORDS = 512 };
uint64_t* host_words(Engine::Impl& im) {
  if (im.h_merge.size() < HW_WORDS * 8) im.h_merge.resize(HW_WORDS * 8);
  return reinterpret_cast<uint64_t*>(im.h_merge.data());
}
}  // namespace

// Small-vocabulary variant of the shuffle merge (see merge_cols_owner):
// pack all local rows (one "owner"), send them to rank 0, merge there.
// `cursor`: 4 zeroed device words (the owner plan's unused scatter cursor
// region, >= 4 words), so the one-owner pack needs no memset launch of its own:
// words 0-1 are the scatter cursor, words 2-3 its (zero) owner counts.
void merge_to_root(Engine::Impl& im, Comm& comm, const std::vector<uint64_t>& rank_rows,
                   const std::vector<uint64_t>& rank_bytes, uint64_t gmax_end, unsigned long long* cursor) {
  Range rg("wc_merge_root");
  hipStream_t s = im.s;
  const int W = comm.size(), R = comm.rank();
  const uint64_t n = im.cols.n;
  const uint64_t my_rows = rank_rows[R], my_bytes = rank_bytes[R];
  uint64_t rr = 0, rbt = 0;  // received by rank 0
  std::vector<size_t> zs(W, 0), sr(W, 0), sb(W, 0), ro_r(W, 0), rb_r(W, 0), ro_b(W, 0), rb_b(W, 0);
  uint64_t* base = host_words(im) + HW_BASE;  // row bases | byte bases per source
  for (int p = 0; p < W; ++p) {
    base[p] = rr;
    base[W + 1 + p] = rbt;
    ro_r[p] = rr * sizeof(MRow);
    ro_b[p] = rbt;
    if (R == 0) {
      rb_r[p] = rank_rows[p] * sizeof(MRow);
      rb_b[p] = rank_bytes[p];
    }
    rr += rank_rows[p];
    rbt += rank_bytes[p];
  }
  base[W] = rr;
  base[2 * W + 1] = rbt;
  sr[0] = my_rows * sizeof(MRow);
  sb[0] = my_bytes;
  if (R != 0) rr = rbt = 0;
  uint64_t T = 1024;
  while (T < 2 * rr) T <<= 1;
  DeviceArena& A = im.merge_mem;
  A.reserve((my_rows + 2 * rr) * sizeof(MRow) + my_bytes + rbt + T * (4 + 16) + rr * (5 * 8 + 4) +
            (2 * (size_t)W + 8) * 8 + 32 * 1024);
  MRow* send_rows = take_aligned<MRow>(A, my_rows);
  uint8_t* send_bytes = take_aligned<uint8_t>(A, my_bytes);
  MRow* recv_rows = take_aligned<MRow>(A, rr);
  uint8_t* recv_bytes = take_aligned<uint8_t>(A, rbt);
  // one owner: the scatter reads no owner count before its own (base 0)
  launch_owner_scatter(im.cols.k0, im.cols.k1, im.cols.cnt, im.cols.first, im.cols.sref_off, im.cols.sref_len,
                       im.cols_arena, n, 1u, cursor + 2, cursor, send_rows, send_bytes, nullptr, s);
  comm.group_begin();
  comm.alltoallv(send_rows, zs.data(), sr.data(), recv_rows, ro_r.data(), rb_r.data(), s);
  comm.alltoallv(send_bytes, zs.data(), sb.data(), recv_bytes, ro_b.data(), rb_b.data(), s);
  comm.group_end();
  KeyCols o;
  uint64_t* gb = host_words(im) + HW_GBASE;  // one output group (rows 0..G, byte base 0)
  gb[0] = gb[2] = 0;
  gb[3] = rbt;
  if (R == 0) {
    uint32_t* state = take_aligned<uint32_t>(A, T);
    unsigned long long* tcnt = take_aligned<unsigned long long>(A, T);
    unsigned long long* tfirst = take_aligned<unsigned long long>(A, T);
    MRow* merged = take_aligned<MRow>(A, rr);
    const size_t nbase = 2 * (size_t)W + 2;
    uint64_t* d_base = take_aligned<uint64_t>(A, nbase + 4);
    unsigned long long* d_m = take_aligned<unsigned long long>(A, 1);
    uint64_t* d_gbase = d_base + nbase;  // one group: row base 0 .. G, byte base 0
    const uint64_t G = rr;
    gb[1] = G;
    ZeroList z{};  // the owner table's state, the bases from page-locked host words: one launch
    z.add(state, T * 4);
    z.add(tcnt, T * 8);
    z.add(tfirst, T * 8, 0xFFFFFFFFu);
    z.add(d_m, 8);
    z.copy(d_base, base, nbase * 8);
    z.copy(d_gbase, gb, 4 * 8);
    launch_zero_regions(z, s);
    launch_mrow_insert(recv_rows, rr, recv_bytes, d_base, d_base + W + 1, (uint32_t)W, state, tcnt, tfirst, T, nullptr,
                       s);
    launch_mrow_compact(recv_rows, state, tcnt, tfirst, T, d_base, d_base + W + 1, (uint32_t)W, merged, d_m, nullptr,
                        s);
    // no host round trip: columns sized for the rows received (a bound of the
    // merged count), which stays on the device (KeyCols::dn) through the
    // first-occurrence sort; the finalize's last wait publishes it
    o.n = G;
    o.dn = d_m;
    o.k0 = take_aligned<uint64_t>(A, G);
    o.k1 = take_aligned<uint64_t>(A, G);
    o.cnt = take_aligned<uint64_t>(A, G);
    o.first = take_aligned<uint64_t>(A, G);
    o.sref_off = take_aligned<uint64_t>(A, G);
    o.sref_len = take_aligned<uint32_t>(A, G);
    launch_mrow_to_cols(merged, G, d_gbase, d_gbase + 2, 1u, o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, s,
                        reinterpret_cast<const uint64_t*>(d_m));
  }
  im.cols = o;  // still in flight: finalize waits under the comm watchdog
  im.cols_arena = recv_bytes;
  im.cols_arena_bytes = R == 0 ? rbt : 0;
  im.max_end = gmax_end;
}

// Step 1 of both protocols: rows / long-word bytes per (rank, owner), and the
// send / receive layouts of the owner exchange derived from them.  Count
// vector of one rank (C = 2W + 2 words): (rows, bytes) per owner, its max
// byte offset, and the flags of its last pass (nonzero: that pass needs
// recovery, so a speculative compaction behind it is void on EVERY rank).
struct OwnerPlan {
  int W = 1, R = 0;
  size_t C = 0;
  std::vector<unsigned long long> all;  // W x C
  uint64_t gmax_end = 0;
  bool any_flags = false;   // some rank's last pass needs recovery (all ranks redo)
  bool any_arena = false;   // some rank's key arena overflowed (all ranks fail)
  bool count_mismatch = false;  // some rank's row count != its owner-count sum (all ranks fail)
  std::vector<uint64_t> rank_rows, rank_bytes;
  uint64_t total_rows = 0, Gmax = 0, GBmax = 0;  // rows / bytes of all ranks (bounds of the merged table)
  std::vector<size_t> so_r, sb_r, so_b, sb_b, ro_r, rb_r, ro_b, rb_b;  // byte offsets / sizes
  uint64_t tr = 0, tb = 0, rr = 0, rbt = 0;                              // rows / bytes sent, received
  unsigned long long* d_cnt = nullptr;  // device: owner counts | scatter cursor
  unsigned long long* d_all = nullptr;  // device: the all-gathered W x C matrix
};

// Device half: owner counts of the compact columns (n rows, or *dn rows with
// n the bound), the max offset and (pass_flags) the last pass's flags, then the
// all-gather.  Nothing waits here.
void plan_enqueue(Engine::Impl& im, Comm& comm, uint64_t n, const uint64_t* dn, const uint32_t* pass_flags,
                  OwnerPlan& P) {
  hipStream_t s = im.s;
  P.W = comm.size();
  P.R = comm.rank();
  const int W = P.W;
  WC_CHECK(W <= (int)MERGE_MAX_RANKS, "merge supports at most 64 ranks");
  P.C = 2 * (size_t)W + 3;  // per owner (rows, bytes) | max offset | pass flags | row count
  const size_t C = P.C;
  DeviceArena& S = im.merge_small;  // small buffers: own arena
  S.reserve(((size_t)W * C + 2 * C + 16) * 8 + 8 * 1024);
  S.reset();
  P.d_cnt = take_aligned<unsigned long long>(S, 2 * C);
  P.d_all = take_aligned<unsigned long long>(S, (size_t)W * C);
  uint64_t* mx = host_words(im) + HW_MX;
  *mx = im.max_end;
  ZeroList z{};  // counts | max offset (from a page-locked host word) | cursor: one launch, disjoint regions
  z.add(P.d_cnt, 2 * (size_t)W * 8);
  z.add(P.d_cnt + 2 * W + 1, (2 * C - 2 * (size_t)W - 1) * 8);
  z.copy(P.d_cnt + 2 * W, mx, 8);
  launch_zero_regions(z, s);
  static const int fault_rank = std::getenv("WC_MERGE_FAULT_COUNT") ? std::atoi(std::getenv("WC_MERGE_FAULT_COUNT")) : -1;
  launch_owner_count(im.cols.k0, im.cols.k1, im.cols.sref_len, n, dn, pass_flags, (uint32_t)W, P.d_cnt, s,
                     P.R == fault_rank ? 1u : 0u);
  comm.allgather(P.d_cnt, P.d_all, C * 8, s);
}

void learn_caps(Engine::Impl& im, const OwnerPlan& P, const std::vector<unsigned long long>& owns, bool dense);

// Host half, from the all-gathered matrix (P.all).
void plan_finish(OwnerPlan& P) {
  const int W = P.W, R = P.R;
  const size_t C = P.C;
  P.rank_rows.assign(W, 0);
  P.rank_bytes.assign(W, 0);
  for (int r = 0; r < W; ++r) {
    P.gmax_end = std::max<uint64_t>(P.gmax_end, P.all[(size_t)r * C + 2 * W]);
    const unsigned long long f = P.all[(size_t)r * C + 2 * W + 1];
    if (f) P.any_flags = true;
    if (f & 2) P.any_arena = true;
    for (int p = 0; p < W; ++p) {
      P.rank_rows[r] += P.all[(size_t)r * C + 2 * p];
      P.rank_bytes[r] += P.all[(size_t)r * C + 2 * p + 1];
    }
    // rows counted vs the owner-count sum of the same rows: an owner-count /
    // gather consistency check (not an independent check of the compaction)
    if (P.all[(size_t)r * C + 2 * W + 2] != P.rank_rows[r]) P.count_mismatch = true;
    P.total_rows += P.rank_rows[r];
    P.GBmax += P.rank_bytes[r];
  }
  P.Gmax = P.total_rows;
  for (auto* v : {&P.so_r, &P.sb_r, &P.so_b, &P.sb_b, &P.ro_r, &P.rb_r, &P.ro_b, &P.rb_b}) v->assign(W, 0);
  const unsigned long long* mine = &P.all[(size_t)R * C];
  for (int p = 0; p < W; ++p) {
    P.so_r[p] = P.tr * sizeof(MRow);
    P.sb_r[p] = mine[2 * p] * sizeof(MRow);
    P.so_b[p] = P.tb;
    P.sb_b[p] = mine[2 * p + 1];
    P.tr += mine[2 * p];
    P.tb += mine[2 * p + 1];
    const unsigned long long* theirs = &P.all[(size_t)p * C];
    P.ro_r[p] = P.rr * sizeof(MRow);
    P.rb_r[p] = theirs[2 * R] * sizeof(MRow);
    P.ro_b[p] = P.rbt;
    P.rb_b[p] = theirs[2 * R + 1];
    P.rr += theirs[2 * R];
    P.rbt += theirs[2 * R + 1];
  }
}

namespace {

// Synchronous step 1 (compact columns already counted on the host).
OwnerPlan plan_owners(Engine::Impl& im, Comm& comm) {
  OwnerPlan P;
  plan_enqueue(im, comm, im.cols.n, nullptr, nullptr, P);
  P.all.resize((size_t)P.W * P.C);
  WC_HIP_CHECK(hipMemcpyAsync(P.all.data(), P.d_all, P.all.size() * 8, hipMemcpyDeviceToHost, im.s));
  comm.sync(im.s);
  plan_finish(P);
  if (P.count_mismatch) fail("owner plan: a rank's key count != its owner row counts");  // every rank sees it
  return P;
}

// Rows scaled from MRow (40 B) to element size `es` in the byte layouts of the
// row exchange (the dense merge's id return path).
std::vector<size_t> rescale(const std::vector<size_t>& v, size_t es) {
  std::vector<size_t> o(v.size());
  for (size_t i = 0; i < v.size(); ++i) o[i] = v[i] / sizeof(MRow) * es;
  return o;
}

}  // namespace

// Steps 2-4 of both protocols; the dense protocol (dense = true) then numbers
// the dictionary and reduces dense count vectors instead of using the owners'
// merged counts.
void merge_cols_owner(Engine::Impl& im, Comm& comm, bool all_ranks, bool dense, OwnerPlan& P) {
  Range rg(dense ? "wc_merge_dense" : "wc_merge_shuffle");
  hipStream_t s = im.s;
  const int W = P.W, R = P.R;
  const uint64_t n = im.cols.n;
  // Few keys in total: every rank sends its rows straight to rank 0, which
  // merges them alone — one exchange instead of two (owner exchange + gather)
  // and one host sync fewer.  WC_MERGE_ROOT_ROWS overrides the threshold.
  uint64_t root_max = MERGE_ROOT_MAX_ROWS;
  if (const char* e = std::getenv("WC_MERGE_ROOT_ROWS")) root_max = std::strtoull(e, nullptr, 10);
  static const bool planned_off =
      std::getenv("WC_MERGE_PLANNED") && std::atoi(std::getenv("WC_MERGE_PLANNED")) == 0;
  // with planned merges on, the exact merge takes the owner path: it learns
  // the caps the planned protocol needs (the root path has no owner counts)
  if (!dense && !all_ranks && P.total_rows <= root_max && (planned_off || std::getenv("WC_MERGE_ROOT_ROWS"))) {
    merge_to_root(im, comm, P.rank_rows, P.rank_bytes, P.gmax_end, P.d_cnt + P.C);
    return;
  }

  // 2. pack by owner and exchange
  const uint64_t tr = P.tr, tb = P.tb, rr = P.rr, rbt = P.rbt;
  uint64_t T = 1024;
  while (T < 2 * rr) T <<= 1;
  const uint64_t vpad_max = (P.Gmax + W - 1) / W * W + W;
  DeviceArena& A = im.merge_mem;
  A.reserve((tr + 2 * rr + P.Gmax) * sizeof(MRow) + tb + 2 * rbt + P.GBmax + T * (4 + 16) + P.Gmax * (5 * 8 + 4) +
            (4 * (size_t)W + 4) * 8 + 32 * 1024 +
            (dense ? (n + 2 * rr + T + tr) * 4 + vpad_max * 8 * 6 + 16 * 256 : 0));
  MRow* send_rows = take_aligned<MRow>(A, tr);
  uint8_t* send_bytes = take_aligned<uint8_t>(A, tb);
  MRow* recv_rows = take_aligned<MRow>(A, rr);
  uint8_t* recv_bytes = take_aligned<uint8_t>(A, rbt);
  uint32_t* send_pos = dense ? take_aligned<uint32_t>(A, n) : nullptr;
  launch_owner_scatter(im.cols.k0, im.cols.k1, im.cols.cnt, im.cols.first, im.cols.sref_off, im.cols.sref_len,
                       im.cols_arena, n, (uint32_t)W, P.d_cnt, P.d_cnt + P.C, send_rows, send_bytes, send_pos, s);
  comm.group_begin();  // rows and long-word bytes in one exchange
  comm.alltoallv(send_rows, P.so_r.data(), P.sb_r.data(), recv_rows, P.ro_r.data(), P.rb_r.data(), s);
  comm.alltoallv(send_bytes, P.so_b.data(), P.sb_b.data(), recv_bytes, P.ro_b.data(), P.rb_b.data(), s);
  comm.group_end();

  // 3. owner-side merge
  uint32_t* state = take_aligned<uint32_t>(A, T);
  unsigned long long* tcnt = take_aligned<unsigned long long>(A, T);
  unsigned long long* tfirst = take_aligned<unsigned long long>(A, T);
  MRow* merged = take_aligned<MRow>(A, rr);
  uint32_t* row_slot = dense ? take_aligned<uint32_t>(A, rr) : nullptr;
  uint32_t* slot_id = dense ? take_aligned<uint32_t>(A, T) : nullptr;
  uint64_t* d_base = take_aligned<uint64_t>(A, 2 * (size_t)W + 2);  // row / byte bases per source (then per owner)
  unsigned long long* d_m = take_aligned<unsigned long long>(A, 1);
  uint64_t* base = host_words(im) + HW_BASE;  // row | byte bases per source
  for (int p = 0; p < W; ++p) {
    base[p] = P.ro_r[p] / sizeof(MRow);
    base[W + 1 + p] = P.ro_b[p];
  }
  base[W] = rr;
  base[2 * W + 1] = rbt;
  {
    ZeroList z{};  // the owner table's state + the source bases (page-locked host words): one launch
    z.add(state, T * 4);
    z.add(tcnt, T * 8);
    z.add(tfirst, T * 8, 0xFFFFFFFFu);
    z.add(d_m, 8);
    z.copy(d_base, base, (2 * (size_t)W + 2) * 8);
    launch_zero_regions(z, s);
  }
  launch_mrow_insert(recv_rows, rr, recv_bytes, d_base, d_base + W + 1, (uint32_t)W, state, tcnt, tfirst, T, row_slot,
                     s);
  launch_mrow_compact(recv_rows, state, tcnt, tfirst, T, d_base, d_base + W + 1, (uint32_t)W, merged, d_m, slot_id, s);

  // 4. (merged rows, bytes) of every owner: the row count stays on the device
  // until this allgather, so one host sync serves both
  uint64_t* own_bytes = host_words(im) + HW_OWNB;
  *own_bytes = rbt;
  unsigned long long* d_own = take_aligned<unsigned long long>(A, 2);
  unsigned long long* d_owns = take_aligned<unsigned long long>(A, 2 * (size_t)W);
  {
    ZeroList z{};  // (merged rows, bytes): both copies in one launch
    z.copy(d_own, d_m, 8);
    z.copy(d_own + 1, own_bytes, 8);
    launch_zero_regions(z, s);
  }
  // dense: number each owner's dictionary (owner-local indices), return them to
  // the senders in the same RCCL launch as the (rows, bytes) all-gather, then
  // scatter the local counts into dense vectors sized for the bound (global id
  // = owner base from the gathered counts + index, on the device) — all
  // enqueued before the host waits for the counts
  uint32_t* ids = nullptr;
  uint32_t* ids_back = nullptr;
  uint64_t *vc = nullptr, *vf = nullptr;
  const uint64_t vpad_cap = (P.Gmax + W - 1) / W * W;
  if (dense) {
    ids = take_aligned<uint32_t>(A, rr);
    ids_back = take_aligned<uint32_t>(A, tr);
    launch_row_ids(row_slot, slot_id, rr, d_owns, 0u, ids, s);  // rank 0: no base
  }
  comm.group_begin();
  comm.allgather(d_own, d_owns, 16, s);
  if (dense) {
    const auto iro = rescale(P.ro_r, 4), irb = rescale(P.rb_r, 4), iso = rescale(P.so_r, 4), isb = rescale(P.sb_r, 4);
    comm.alltoallv(ids, iro.data(), irb.data(), ids_back, iso.data(), isb.data(), s);
  }
  comm.group_end();
  if (dense) {
    vc = take_aligned<uint64_t>(A, vpad_cap);
    vf = take_aligned<uint64_t>(A, vpad_cap);
    uint64_t* seg = host_words(im) + HW_SEG;  // send-row starts per owner
    for (int p = 0; p <= W; ++p) seg[p] = p < W ? P.so_r[p] / sizeof(MRow) : tr;
    uint64_t* d_seg = take_aligned<uint64_t>(A, (size_t)W + 1);
    ZeroList z{};
    if (vpad_cap) {
      z.add(vc, vpad_cap * 8);
      z.add(vf, vpad_cap * 8, 0xFFFFFFFFu);
    }
    z.copy(d_seg, seg, ((size_t)W + 1) * 8);
    launch_zero_regions(z, s);
    launch_scatter_ids(send_pos, ids_back, d_seg, d_owns, (uint32_t)W, im.cols.cnt, im.cols.first, n, vc, vf, s);
  }
  std::vector<unsigned long long> owns(2 * (size_t)W);
  WC_HIP_CHECK(hipMemcpyAsync(owns.data(), d_owns, owns.size() * 8, hipMemcpyDeviceToHost, s));
  comm.sync(s);
  learn_caps(im, P, owns, dense);  // the next merge of this shape runs planned
  const unsigned long long own[2] = {owns[2 * (size_t)R], rbt};
  std::vector<size_t> go_r(W, 0), gb_r(W, 0), go_b(W, 0), gb_b(W, 0), zs(W, 0);
  std::vector<size_t> sr(W, 0), sb(W, 0);
  uint64_t G = 0, GB = 0;
  uint64_t* gbase = host_words(im) + HW_GBASE;  // row | byte bases per owner in the gathered dictionary
  for (int p = 0; p < W; ++p) {
    gbase[p] = G;
    gbase[W + 1 + p] = GB;
    go_r[p] = G * sizeof(MRow);
    go_b[p] = GB;
    if (R == 0) {
      gb_r[p] = owns[2 * p] * sizeof(MRow);
      gb_b[p] = owns[2 * p + 1];
    }
    G += owns[2 * p];
    GB += owns[2 * p + 1];
  }
  gbase[W] = G;
  gbase[2 * W + 1] = GB;
  WC_CHECK(G < (1ull << 32), "merged dictionary exceeds 2^32 entries");

  // dense: the vectors' first vpad entries are reduce-scattered (sum, min) and
  // all-gathered below
  uint64_t* dcnt = nullptr;
  uint64_t* dfirst = nullptr;
  const uint64_t vpad = (G + W - 1) / W * W;
  if (dense) {
    WC_CHECK(vpad <= vpad_cap, "dense merge: dictionary above its bound");
    dcnt = take_aligned<uint64_t>(A, vpad);
    dfirst = take_aligned<uint64_t>(A, vpad);
  }

  // 5. gather the dictionary (merged rows + bytes) to rank 0 (broadcast for
  // all_ranks) — in the same RCCL launch as the dense reductions
  sr[0] = own[0] * sizeof(MRow);
  sb[0] = own[1];
  const bool have = R == 0 || all_ranks;
  MRow* grows = take_aligned<MRow>(A, G);
  uint8_t* gbytes = take_aligned<uint8_t>(A, GB);
  uint64_t* scnt = nullptr;
  uint64_t* sfirst = nullptr;
  if (dense && vpad) {
    scnt = take_aligned<uint64_t>(A, vpad / W);
    sfirst = take_aligned<uint64_t>(A, vpad / W);
  }
  comm.group_begin();
  if (dense && vpad) {
    comm.reduce_scatter_u64(vc, scnt, vpad / W, RedOp::Sum, s);
    comm.reduce_scatter_u64(vf, sfirst, vpad / W, RedOp::Min, s);
  }
  comm.alltoallv(merged, zs.data(), sr.data(), grows, go_r.data(), gb_r.data(), s);
  comm.alltoallv(recv_bytes, zs.data(), sb.data(), gbytes, go_b.data(), gb_b.data(), s);
  comm.group_end();
  comm.group_begin();
  if (dense && vpad) {
    comm.allgather(scnt, dcnt, vpad / W * 8, s);
    comm.allgather(sfirst, dfirst, vpad / W * 8, s);
  }
  if (all_ranks) {
    comm.broadcast(grows, G * sizeof(MRow), 0, s);
    comm.broadcast(gbytes, GB, 0, s);
  }
  comm.group_end();
  KeyCols o;
  o.n = have ? G : 0;
  if (have) {
    o.k0 = take_aligned<uint64_t>(A, G);
    o.k1 = take_aligned<uint64_t>(A, G);
    o.cnt = dense ? dcnt : take_aligned<uint64_t>(A, G);  // dense: id order == gathered row order
    o.first = dense ? dfirst : take_aligned<uint64_t>(A, G);
    o.sref_off = take_aligned<uint64_t>(A, G);
    o.sref_len = take_aligned<uint32_t>(A, G);
    uint64_t* d_gbase = take_aligned<uint64_t>(A, 2 * (size_t)W + 2);
    WC_HIP_CHECK(hipMemcpyAsync(d_gbase, gbase, (2 * (size_t)W + 2) * 8, hipMemcpyHostToDevice, s));
    launch_mrow_to_cols(grows, G, d_gbase, d_gbase + W + 1, (uint32_t)W, o.k0, o.k1, dense ? nullptr : o.cnt,
                        dense ? nullptr : o.first, o.sref_off, o.sref_len, s);
  }
  im.cols = o;  // still in flight: finalize waits under the comm watchdog
  im.cols_arena = gbytes;
  im.cols_arena_bytes = have ? GB : 0;
  im.max_end = P.gmax_end;
}

// Fixed exchange regions for the next planned merge, from an exact merge's
// all-gathered count matrix and merged-row counts (identical on every rank):
// the largest (rank -> owner) rows / bytes and owner merged rows, + 1/8 + 256.
void learn_caps(Engine::Impl& im, const OwnerPlan& P, const std::vector<unsigned long long>& owns, bool dense) {
  const int W = P.W;
  uint64_t rows = 0, bytes = 0, merged = 0;
  for (int p = 0; p < W; ++p)
    for (int o = 0; o < W; ++o) {
      rows = std::max<uint64_t>(rows, P.all[(size_t)p * P.C + 2 * o]);
      bytes = std::max<uint64_t>(bytes, P.all[(size_t)p * P.C + 2 * o + 1]);
    }
  for (int o = 0; o < W; ++o) merged = std::max<uint64_t>(merged, owns[2 * (size_t)o]);
  auto grow = [](uint64_t x) { return x + x / 8 + 256; };
  Engine::Impl::MergeCaps& c = im.merge_caps;
  c.valid = true;
  c.world = W;
  c.mode = dense ? 1u : 0u;
  c.rows = grow(rows);
  c.bytes = (grow(bytes) + 7) & ~7ull;
  c.merged = grow(merged);
  if (const char* e = std::getenv("WC_MERGE_CAP_ROWS")) {  // tests only: force region overflows (the redo path)
    c.rows = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
    c.merged = c.rows;
  }
  c.gmax_end = P.gmax_end;
}

// Planned merge (both protocols, SURVEY §5.8 with no host round trip): every
// exchange has sizes fixed in advance (Engine::Impl::MergeCaps) — owner o's
// rows from each rank in a region of caps.rows rows (+ caps.bytes bytes of
// long words), owner o's merged rows in a region of caps.merged rows for the
// gather (dense: padded ids o * caps.merged + index) — padding rows are empty
// keys that the owner merge skips.  Counts, decisions and the merged key count
// stay on the device: nothing here waits.  Each rank's word quad (merged rows,
// flags, max first offset, -) travels in ONE all-gather after the owner
// merge: its scatter sets the flags (a last pass needing recovery 1, an arena
// overflow 2, a region overflow 4), and wc_merge_check ORs every rank's into
// im.d_merge_flags (+ 4 for merged rows past their region or a first offset
// above the key width the order is sized for) — the finalize reads them after
// its last wait, and every rank redoes the merge with the exact protocol
// together when they are set.  (Before: an owner-count launch, a count-matrix
// all-gather and a check ahead of the scatter — one more collective.)
// Columns in: im.cols with n the bound and dn the device count.
// Wire-traffic accounting of one collective (Stats::merge_*): bytes this rank
// sends to each peer (vector over ranks; its own entry ignored).
void account(Engine::Impl& im, int R, const std::vector<size_t>& to_peer) {
  uint64_t mx = 0, tot = 0;
  for (size_t p = 0; p < to_peer.size(); ++p) {
    if ((int)p == R) continue;
    mx = std::max<uint64_t>(mx, to_peer[p]);
    tot += to_peer[p];
  }
  im.st.merge_collectives++;
  im.st.merge_sent_bytes += tot;
  im.st.merge_peer_bytes += mx;
}
void account_uniform(Engine::Impl& im, int R, int W, uint64_t bytes_each) {
  account(im, R, std::vector<size_t>((size_t)W, (size_t)bytes_each));
}

void merge_cols_planned(Engine::Impl& im, Comm& comm, bool all_ranks, bool dense, const uint32_t* pass_flags) {
  Range rg(dense ? "wc_merge_dense_planned" : "wc_merge_shuffle_planned");
  im.st.merge_collectives = 0;
  im.st.merge_sent_bytes = im.st.merge_peer_bytes = im.st.merge_root_recv_bytes = 0;
  hipStream_t s = im.s;
  const int W = comm.size(), R = comm.rank();
  WC_CHECK(W <= (int)MERGE_MAX_RANKS, "merge supports at most 64 ranks");
  const Engine::Impl::MergeCaps cp = im.merge_caps;
  const uint64_t Cr = cp.rows, Cb = cp.bytes, Gr = cp.merged;
  const uint64_t nb = im.cols.n;  // bound; the count is *dn
  const uint64_t* dn = reinterpret_cast<const uint64_t*>(im.cols.dn);
  DeviceArena& S = im.merge_small;
  S.reserve((8 * (size_t)W + 64) * 8 + 8 * 1024);
  S.reset();
  unsigned long long* d_cur = take_aligned<unsigned long long>(S, 2 * (size_t)W);  // scatter cursor per owner
  unsigned long long* d_owns = take_aligned<unsigned long long>(S, 4 * (size_t)W);
  unsigned long long* d_own = d_owns + 4 * (size_t)R;  // merged rows | flags | max offset | -, gathered in place
  unsigned long long* d_on = take_aligned<unsigned long long>(S, 1);
  im.d_merge_flags = take_aligned<uint32_t>(S, 2);
  // The bound every rank's gathered max first offset is checked against.  It
  // must be IDENTICAL on every rank — each rank decides "redo" from it on its
  // own, and a rank that disagrees skips the redo's collectives (a hang):
  // the caps' global max end (the last exact merge's), not this rank's own
  // max_end.  It is <= the width rank 0's order is sized for below
  // (max(max_end, gmax_end)), so a job that outgrows it redoes exactly, on
  // every rank together.
  const uint64_t key_bound = cp.gmax_end;

  DeviceArena& A = im.merge_mem;
  const uint64_t RR = (uint64_t)W * Cr, RB = (uint64_t)W * Cb, GR = (uint64_t)W * Gr;
  // the owner table: twice the learned merged-row cap (not the rows received:
  // at W ranks an owner receives ~W x its distinct keys, so 2 RR slots made the
  // zeroing and the compaction's scan W times larger than the keys need).  A
  // job with more distinct keys fills it: the insert's probes are bounded and
  // the compaction's count > Gr makes every rank redo the merge exactly.
  uint64_t T = 1024;
  while (T < 2 * std::min(RR, Gr)) T <<= 1;
  const bool have = R == 0 || all_ranks;
  // send + receive rows and bytes, the owner table (state + index), the
  // merged rows, the gathered rows and bytes, rank 0's columns, small words
  A.reserve(2 * RR * sizeof(MRow) + 2 * RB + T * (4 + 4) + Gr * sizeof(MRow) + (size_t)GR * sizeof(MRow) +
            (size_t)W * RB + (have ? GR * (5 * 8 + 4) : 0) + (4 * (size_t)W + 8) * 8 + 64 * 1024 +
            // dense: send_pos, ids, ids_back (u32); the padded vectors vc, vf (u64)
            (dense ? (nb + 2 * RR) * 4 + 2 * GR * 8 + 16 * 256 : 0));
  A.reset();
  // Nothing travels from a rank to itself: the scatter writes this rank's own
  // rows and bytes straight into its receive regions, rank 0's compaction
  // writes into region 0 of the gather buffer and its receive bytes ARE region
  // 0 of the gathered payload — so at W = 1 no collective moves data at all.
  MRow* grows = take_aligned<MRow>(A, GR);
  uint8_t* gbytes = take_aligned<uint8_t>(A, (uint64_t)W * RB);
  MRow* send_rows = take_aligned<MRow>(A, RR);
  uint8_t* send_bytes = take_aligned<uint8_t>(A, RB);
  MRow* recv_rows = take_aligned<MRow>(A, RR);
  uint8_t* recv_bytes = R == 0 ? gbytes : take_aligned<uint8_t>(A, RB);
  uint32_t* state = take_aligned<uint32_t>(A, T);     // claiming row + 1 per slot
  uint32_t* slot_idx = take_aligned<uint32_t>(A, T);  // its merged-row index + 1, once published
  // the owner's merged rows: the first Gr (more: counted, flagged, the merge is
  // redone) — count and (inverted) first offset words zeroed, added to by atomics
  MRow* merged = R == 0 ? grows : take_aligned<MRow>(A, Gr);
  uint64_t* d_base = take_aligned<uint64_t>(A, 2 * (size_t)W + 2);
  uint64_t* d_seg = take_aligned<uint64_t>(A, (size_t)W + 1);
  uint32_t* send_pos = dense ? take_aligned<uint32_t>(A, nb) : nullptr;
  // dense: each received row's owner-local id (written by the insert) and the ids that come back
  uint32_t* ids = dense ? take_aligned<uint32_t>(A, RR) : nullptr;
  uint32_t* ids_back = dense ? take_aligned<uint32_t>(A, RR) : nullptr;
  // dense: padded count / first-offset vectors (zeroed with everything else)
  uint64_t* vc = dense ? take_aligned<uint64_t>(A, GR) : nullptr;
  uint64_t* vf = dense ? take_aligned<uint64_t>(A, GR) : nullptr;
  {
    ZeroList z{};  // cursor, flags, padding rows, the owner table, the merged region, this rank's quad: ONE launch
    z.add(d_cur, 2 * (size_t)W * 8);
    z.add(im.d_merge_flags, 8);
    // padding rows read as K1_EMPTY: the send regions to peers, and this rank's own receive region
    if (R > 0) z.add(send_rows, (uint64_t)R * Cr * sizeof(MRow));
    if (R + 1 < W) z.add(send_rows + (uint64_t)(R + 1) * Cr, (uint64_t)(W - R - 1) * Cr * sizeof(MRow));
    z.add(recv_rows + (uint64_t)R * Cr, Cr * sizeof(MRow));
    z.add(state, T * 4);
    z.add(slot_idx, T * 4);
    z.add(merged, Gr * sizeof(MRow));
    z.add(d_own, 16);  // merged rows (wc_mrow_insert_emit adds), flags (the scatter ORs)
    if (im.cols.occ) z.add(reinterpret_cast<uint32_t*>(im.d_local_n), 8);  // the scatter counts the table's keys
    if (dense) {
      z.add(vc, GR * 8);
      z.add(vf, GR * 8, 0xFFFFFFFFu);
    }
    // (region bases and the max offset: written by the scatter's block 0).  The
    // same list as the last planned merge's was already applied by this job's
    // sampling launch (launch_pass): nothing since has touched these regions
    if (!(im.merge_zero_pre && same_fills(z, im.merge_zero_last) && im.merge_zero_gen == im.merge_arena_gen()))
      launch_zero_regions(z, s);
    im.merge_zero_last = z;
    im.merge_zero_last_valid = true;
    im.merge_zero_gen = im.merge_arena_gen();
    im.merge_zero_pre = false;
  }
  // 1. pack into the fixed regions (this rank's pass flags and region overflow
  // into its flag word) and exchange them whole
  // + the fixed-region bases per source (rows | bytes), the send-row starts per
  // owner (dense id return) and this rank's max first offset, from block 0
  const MergeSelf self{(uint32_t)R, recv_rows, recv_bytes, d_base, d_seg, d_own, im.max_end};
  launch_owner_scatter(im.cols.k0, im.cols.k1, im.cols.cnt, im.cols.first, im.cols.sref_off, im.cols.sref_len,
                       im.cols_arena, nb, (uint32_t)W, nullptr, d_cur, send_rows, send_bytes, send_pos, s, dn, Cr, Cb,
                       reinterpret_cast<uint32_t*>(d_own + 1), pass_flags, im.cols.occ,
                       im.cols.occ ? reinterpret_cast<unsigned long long*>(im.d_local_n) : nullptr, &self);
  std::vector<size_t> ro(W), rs(W, Cr * sizeof(MRow)), bo(W), bs(W, Cb), zs(W, 0), gr(W, 0), gb(W, 0), go(W), gbo(W);
  for (int p = 0; p < W; ++p) {
    ro[p] = (size_t)p * Cr * sizeof(MRow);
    bo[p] = (size_t)p * Cb;
  }
  rs[R] = 0;  // this rank's own region is already in place
  bs[R] = 0;
  comm.group_begin();
  comm.alltoallv(send_rows, ro.data(), rs.data(), recv_rows, ro.data(), rs.data(), s);
  comm.alltoallv(send_bytes, bo.data(), bs.data(), recv_bytes, bo.data(), bs.data(), s);
  comm.group_end();
  {
    std::vector<size_t> per(W);
    for (int p = 0; p < W; ++p) per[p] = rs[p] + bs[p];
    account(im, R, per);  // the owner exchange (rows + LONG bytes, one grouped launch)
  }
  // 2. owner merge (padding rows skipped), merged rows counted on the device into the quad
  // (+ dense: each row's owner-local id, this rank's own region straight into the returned ids)
  launch_mrow_insert_emit(recv_rows, RR, recv_bytes, d_base, d_base + W + 1, (uint32_t)W, state, slot_idx, T, merged,
                          d_own, Gr, ids, ids_back, (uint32_t)R, Cr, s);
  // 3. every rank's quad (+ dense: the owner-local ids back to the senders), the decision
  comm.group_begin();
  comm.allgather(d_own, d_owns, 32, s);
  if (dense) {
    std::vector<size_t> io(W), is(W, Cr * 4);
    for (int p = 0; p < W; ++p) io[p] = (size_t)p * Cr * 4;
    is[R] = 0;
    comm.alltoallv(ids, io.data(), is.data(), ids_back, io.data(), is.data(), s);
  }
  comm.group_end();
  account_uniform(im, R, W, 32 + (dense ? Cr * 4 : 0));  // the quads (+ dense: the ids back)
  if (!have) launch_merge_check(d_owns, (uint32_t)W, Gr, key_bound, im.d_merge_flags, s);  // else folded below
  // 4. dense: padded count / first-offset vectors, reduce-scattered (owner o's
  // slice = its ids) and all-gathered
  uint64_t *dcnt = nullptr, *dfirst = nullptr;
  if (dense) {
    // reduce-scatter and all-gather in place: owner R's reduced slice is
    // region R of the vectors, and the gathered vectors are the vectors
    uint64_t* scnt = vc + (uint64_t)R * Gr;
    uint64_t* sfirst = vf + (uint64_t)R * Gr;
    dcnt = vc;
    dfirst = vf;
    launch_scatter_ids(send_pos, ids_back, d_seg, d_owns, (uint32_t)W, im.cols.cnt, im.cols.first, nb, vc, vf, s, dn, Gr);
    comm.group_begin();
    comm.reduce_scatter_u64(vc, scnt, Gr, RedOp::Sum, s);
    comm.reduce_scatter_u64(vf, sfirst, Gr, RedOp::Min, s);
    comm.group_end();
    account_uniform(im, R, W, 2 * Gr * 8);  // reduce-scatter: owner p's slice of both vectors to p
    comm.group_begin();
    comm.allgather(scnt, dcnt, Gr * 8, s);
    comm.allgather(sfirst, dfirst, Gr * 8, s);
    comm.group_end();
    account_uniform(im, R, W, 2 * Gr * 8);  // all-gather: this rank's slice to every peer
  }
  // 5. every owner's merged region (+ its whole received byte payload) to rank 0
  for (int p = 0; p < W; ++p) {
    go[p] = (size_t)p * Gr * sizeof(MRow);
    gbo[p] = (size_t)p * RB;
    if (R == 0) {
      gr[p] = Gr * sizeof(MRow);
      gb[p] = RB;
    }
  }
  std::vector<size_t> sr(W, 0), sb(W, 0);
  sr[0] = Gr * sizeof(MRow);
  sb[0] = RB;
  if (R == 0) {  // rank 0's own region and payload are in place
    sr[0] = sb[0] = 0;
    gr[0] = gb[0] = 0;
  }
  comm.group_begin();
  comm.alltoallv(merged, zs.data(), sr.data(), grows, go.data(), gr.data(), s);
  comm.alltoallv(recv_bytes, zs.data(), sb.data(), gbytes, gbo.data(), gb.data(), s);
  comm.group_end();
  {
    std::vector<size_t> per(W, 0);
    per[0] = sr[0] + sb[0];
    account(im, R, per);  // the gather to rank 0
    if (R == 0)
      for (int p = 1; p < W; ++p) im.st.merge_root_recv_bytes += gr[p] + gb[p];
  }
  if (all_ranks) {
    comm.group_begin();
    comm.broadcast(grows, GR * sizeof(MRow), 0, s);
    comm.broadcast(gbytes, (uint64_t)W * RB, 0, s);
    comm.group_end();
    if (R == 0) account_uniform(im, R, W, GR * sizeof(MRow) + (uint64_t)W * RB);
  }
  KeyCols o;
  im.max_end = std::max(im.max_end, cp.gmax_end);  // the width the order below is sized for
  if (have) {
    o.n = GR;
    o.dn = d_on;
    o.k0 = take_aligned<uint64_t>(A, GR);
    o.k1 = take_aligned<uint64_t>(A, GR);
    o.cnt = take_aligned<uint64_t>(A, GR);
    o.first = take_aligned<uint64_t>(A, GR);
    o.sref_off = take_aligned<uint64_t>(A, GR);
    o.sref_len = take_aligned<uint32_t>(A, GR);
    // + the decision flags (wc_merge_check) and, when the sample sort will
    // order these rows, its exact key histogram: two launches fewer
    const bool hist = im.sample_order(GR);
    const uint32_t hm = fo_mbits(im.key_bits());
    launch_mrow_regions_to_cols(grows, (uint32_t)W, Gr, d_owns, RB, dcnt, dfirst, o.k0, o.k1, o.cnt, o.first,
                                o.sref_off, o.sref_len, d_on, s, im.d_merge_flags, key_bound,
                                hist ? im.d_fo_hist_cols : nullptr, hm);
    im.cols_hist_m = hist ? hm : 0;
  }
  im.cols = o;  // in flight: the finalize's last wait publishes the count and the flags
  im.cols_arena = gbytes;
  im.cols_arena_bytes = have ? (uint64_t)W * RB : 0;
  im.planned_active = true;
  im.st.merges_planned++;
}

// The planned merge launched right behind the pending last pass: device
// bucket offsets -> compaction sized to the table's capacity -> the planned
// protocol, nothing waited for.  Needs caps of this world size and protocol.
bool merge_cols_planned_speculative(Engine::Impl& im, Comm& comm, bool all_ranks) {
  const Engine::Impl::MergeCaps& cp = im.merge_caps;
  static const bool off = std::getenv("WC_MERGE_PLANNED") && std::atoi(std::getenv("WC_MERGE_PLANNED")) == 0;
  if (off || !cp.valid || cp.world != comm.size() || cp.mode != im.opt.merge_mode) return false;
  Range rg("wc_merge_planned_speculative");
  im.planned_pass = im.pend;
  im.pend.active = false;
  // the pass's counter publish stays held back: it rides in the finalize's
  // last publish (read after that wait) — one launch fewer
  const TableView& t = im.table();
  const size_t nb = (size_t)1 << t.log2_buckets;
  const uint64_t cap = (uint64_t)nb * TAB_SLOTS;
  DeviceArena& F = im.fin_mem;
  F.reserve(64 * 1024);
  F.reset();
  // no compaction: the owner scatter reads the table's slots (and counts its keys)
  KeyCols c;
  c.k0 = t.k0;
  c.k1 = t.k1;
  c.cnt = t.cnt;
  c.first = t.first;
  c.sref_off = t.sref_off;
  c.sref_len = t.sref_len;
  c.occ = t.occupancy;
  uint64_t* d_n = F.take_n<uint64_t>(2);
  c.n = cap;
  im.d_local_n = d_n;
  im.cols = c;
  im.cols_arena = im.d_arena;
  im.st.log2_buckets = t.log2_buckets;
  im.mark(Engine::Impl::EV_MERGE0);
  merge_cols_planned(im, comm, all_ranks, im.opt.merge_mode == 1, im.d_ctr->flags);
  return true;
}

void merge_cols(Engine::Impl& im, Comm& comm, bool all_ranks) {
  OwnerPlan P = plan_owners(im, comm);
  merge_cols_owner(im, comm, all_ranks, im.opt.merge_mode == 1, P);
}

// The merged finalize launched right behind the pending last pass (SURVEY
// §5.8 without the settle): device bucket offsets -> compaction sized to the
// table's capacity -> owner counts of the device-counted rows + this pass's
// flags -> all-gather -> one publish into page-locked memory, and ONE host
// wait for all of it (the pass's counters included).  A rank whose pass needs
// recovery flags it in its count vector, so every rank sees the same matrix
// and all of them fall back together (returns false; the caller recovers and
// runs the synchronous protocol).
bool merge_cols_speculative(Engine::Impl& im, Comm& comm, bool all_ranks) {
  Range rg("wc_merge_speculative");
  const Engine::Impl::PendingPass p = im.pend;
  im.pend.active = false;
  im.flush_pass_publish();
  hipStream_t s = im.s;
  const TableView& t = im.table();
  const size_t nb = (size_t)1 << t.log2_buckets;
  const uint64_t cap = (uint64_t)nb * TAB_SLOTS;
  DeviceArena& A = im.fin_mem;
  A.reserve((cap + 1) * (5 * 8 + 4) + nb * 8 + 64 * 1024);
  A.reset();
  KeyCols c;
  c.k0 = A.take_n<uint64_t>(cap + 1);
  c.k1 = A.take_n<uint64_t>(cap + 1);
  c.cnt = A.take_n<uint64_t>(cap + 1);
  c.first = A.take_n<uint64_t>(cap + 1);
  c.sref_off = A.take_n<uint64_t>(cap + 1);
  c.sref_len = A.take_n<uint32_t>(cap + 1);
  uint64_t* d_boff = A.take_n<uint64_t>(nb);
  uint64_t* d_n = A.take_n<uint64_t>(2);
  launch_bucket_offsets(t.occupancy, (uint32_t)nb, d_boff, d_n, s);
  launch_table_compact(t, d_boff, c.k0, c.k1, c.cnt, c.first, c.sref_off, c.sref_len, s, im.bounds(cap + 1));
  im.cols = c;
  im.cols_arena = im.d_arena;
  im.mark(Engine::Impl::EV_MERGE0);
  OwnerPlan P;
  plan_enqueue(im, comm, cap, d_n, im.d_ctr->flags, P);
  // one publish: the gathered matrix + the local key count, then a sequence word
  const size_t words = (size_t)P.W * P.C;
  if (im.h_plan.size() < (words + 4) * 8) {
    im.h_plan = PinnedBuffer(std::max<size_t>((words + 4) * 8, 4096));
    std::memset(im.h_plan.data(), 0, im.h_plan.size());
  }
  uint64_t* hp = reinterpret_cast<uint64_t*>(im.h_plan.data());
  PubList pl{};
  pl.add(hp, P.d_all, words * 8);
  pl.add(hp + words, d_n, 8);
  uint32_t* seq = reinterpret_cast<uint32_t*>(hp + words + 2);
  pl.seq_dst = seq;
  pl.seq = ++im.plan_seq;
  launch_publish(pl, s);
  // the peers' all-gather normally lands within microseconds: spin briefly,
  // then wait under the communicator's watchdog (a dead peer aborts, no hang)
  const double t0 = now_seconds();
  while (__atomic_load_n(seq, __ATOMIC_ACQUIRE) != im.plan_seq) {
    if (now_seconds() - t0 > 2e-3) {
      comm.sync(s);
      break;
    }
    __builtin_ia32_pause();
  }
  P.all.assign(hp, hp + words);
  plan_finish(P);
  // Decisions that end or redo the job come from the gathered matrix only, so
  // every rank takes them together: a rank whose key arena overflowed would
  // throw in complete_pass while the others entered the recovery's
  // collectives, and a row count that disagrees with its owner counts (a
  // compaction bug) used to throw on that rank alone — both fail every rank here
  if (P.any_arena)
    fail("key arena exhausted on a rank (" + std::to_string(im.opt.arena_bytes) + " bytes each); raise arena_bytes");
  if (P.count_mismatch) fail("speculative compaction: a rank's key count != its owner row counts");
  const bool clean = im.complete_pass(p.text, p.len, p.avail, p.base, p.prev, p.rb, p.blocks, true);
  if (!clean || P.any_flags) return false;  // every rank sees the same flags: all redo
  im.cols.n = P.all[(size_t)P.R * P.C + 2 * (size_t)P.W + 2];
  im.st.keys = im.cols.n;
  im.st.log2_buckets = t.log2_buckets;
  merge_cols_owner(im, comm, all_ranks, im.opt.merge_mode == 1, P);
  return true;
}

}  // namespace wc
