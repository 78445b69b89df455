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
//     device-scope count / min-offset atomics) and compacts it
//  4. gather the merged rows + bytes to rank 0 (broadcast for all_ranks)   ~V x 40 B
// Each rank merges ~V/W keys instead of sorting all W x V, and only rank 0
// orders the final table; the merge is a few tens of microseconds of xGMI.
//
// DENSE (merge_mode 1):
//  1. allgather per-rank (n_keys, arena bytes, max offset)              tiny
//  2. allgather the padded key columns (k0, k1, arena refs) + arenas    ~V x 28 B
//  3. every rank sorts the union by (k0, k1) (stable LSD radix) and
//     assigns global ids = rank of the key in that order -> identical
//     dictionary on every rank without any further exchange
//  4. scatter local counts / first offsets into dense u64[V] vectors
//  5. reduce-scatter(sum) counts, reduce-scatter(min) first offsets     V x 8 B each
//  6. all-gather the reduced slices                                     V x 8 B each
// Ring reduce-scatter over 7 xGMI links moves ~V x 8 B x (W-1)/W per rank:
// ~50 us for a million-word vocabulary, negligible next to the text scan.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../engine/engine_impl.hpp"
#include "comm.hpp"

namespace wc {

void merge_cols_dense(Engine::Impl& im, Comm& comm) {
  Range rg("wc_merge_dense");
  hipStream_t s = im.s;
  const int W = comm.size(), R = comm.rank();
  const uint64_t n = im.cols.n;

  // 1. metadata (small buffers: own arena, reserved once)
  DeviceArena& S = im.merge_small;
  S.reserve((size_t)(W + 1) * 4 * 8 + 1024);
  uint64_t* d_meta = S.take_n<uint64_t>((size_t)(W + 1) * 4);
  uint64_t meta[4] = {n, im.cols_arena_bytes, im.max_end, 0};
  WC_HIP_CHECK(hipMemcpyAsync(d_meta, meta, sizeof meta, hipMemcpyHostToDevice, s));
  comm.allgather(d_meta, d_meta + 4, 4 * 8, s);
  std::vector<uint64_t> all((size_t)W * 4);
  WC_HIP_CHECK(hipMemcpyAsync(all.data(), d_meta + 4, all.size() * 8, hipMemcpyDeviceToHost, s));
  comm.sync(s);
  uint64_t n_max = 1, a_max = 16, gmax_end = 0;
  for (int r = 0; r < W; ++r) {
    n_max = std::max(n_max, all[r * 4 + 0]);
    a_max = std::max(a_max, (all[r * 4 + 1] + 15) / 16 * 16);
    gmax_end = std::max(gmax_end, all[r * 4 + 2]);
  }
  const uint64_t m = (uint64_t)W * n_max;
  WC_CHECK(m < (1ull << 32), "merged dictionary exceeds 2^32 entries");
  const uint64_t vpad_max = (m + W - 1) / W * W;

  // 2. workspace
  DeviceArena& A = im.merge_mem;
  // every take_n below, in order (+ 256 B alignment slack per allocation)
  const size_t need = n_max * 28 + a_max + m * 28 + (size_t)W * a_max  // send + gathered columns
                      + m * (16 + 8) + radix_hist_words(m) * 4              // union sort
                      + m * (8 + 8) + vpad_max * 28                         // flags, ids, merged key columns
                      + vpad_max * 8 * 4 + 2 * (vpad_max / W) * 8           // dense vectors + slices
                      + 32 * 256 + 64 * 1024;
  A.reserve(need);
  A.reset();
  uint64_t* sk0 = A.take_n<uint64_t>(n_max);
  uint64_t* sk1 = A.take_n<uint64_t>(n_max);
  uint64_t* sso = A.take_n<uint64_t>(n_max);
  uint32_t* ssl = A.take_n<uint32_t>(n_max);
  uint8_t* sar = A.take_n<uint8_t>(a_max);
  uint64_t* K0 = A.take_n<uint64_t>(m);
  uint64_t* K1 = A.take_n<uint64_t>(m);
  uint64_t* SO = A.take_n<uint64_t>(m);
  uint32_t* SL = A.take_n<uint32_t>(m);
  uint8_t* AR = A.take_n<uint8_t>((size_t)W * a_max);
  launch_pad_u64(im.cols.k0, n, sk0, n_max, 0, s);
  launch_pad_u64(im.cols.k1, n, sk1, n_max, K1_EMPTY, s);
  launch_pad_u64(im.cols.sref_off, n, sso, n_max, 0, s);
  WC_HIP_CHECK(hipMemsetAsync(ssl, 0, n_max * 4, s));
  if (n) WC_HIP_CHECK(hipMemcpyAsync(ssl, im.cols.sref_len, n * 4, hipMemcpyDeviceToDevice, s));
  if (im.cols_arena_bytes)
    WC_HIP_CHECK(hipMemcpyAsync(sar, im.cols_arena, im.cols_arena_bytes, hipMemcpyDeviceToDevice, s));
  comm.allgather(sk0, K0, n_max * 8, s);
  comm.allgather(sk1, K1, n_max * 8, s);
  comm.allgather(sso, SO, n_max * 8, s);
  comm.allgather(ssl, SL, n_max * 4, s);
  comm.allgather(sar, AR, a_max, s);

  // 3. dictionary union: sort positions by (k0, k1), flag heads, scan -> ids
  uint64_t* keys = A.take_n<uint64_t>(m);
  uint64_t* tkeys = A.take_n<uint64_t>(m);
  uint32_t* pos = A.take_n<uint32_t>(m);
  uint32_t* tpos = A.take_n<uint32_t>(m);
  uint32_t* hist = A.take_n<uint32_t>(radix_hist_words(m));
  launch_iota_u32(pos, m, s);
  WC_HIP_CHECK(hipMemcpyAsync(keys, K1, m * 8, hipMemcpyDeviceToDevice, s));
  radix_sort_pairs(keys, pos, tkeys, tpos, hist, m, 64, s);
  launch_gather_u64(K0, pos, keys, m, s);
  radix_sort_pairs(keys, pos, tkeys, tpos, hist, m, 64, s);
  uint32_t* flag = A.take_n<uint32_t>(m);
  uint32_t* rep = A.take_n<uint32_t>(m);
  uint32_t* ex = A.take_n<uint32_t>(m);
  uint32_t* d_total = A.take_n<uint32_t>(1);
  launch_union_flags(pos, K0, K1, SO, SL, AR, n_max, a_max, flag, rep, m, s);
  launch_exclusive_scan_u32(flag, ex, m, d_total, s);
  uint32_t vg = 0;
  WC_HIP_CHECK(hipMemcpyAsync(&vg, d_total, 4, hipMemcpyDeviceToHost, s));
  comm.sync(s);
  const uint64_t vpad = std::max<uint64_t>(W, ((uint64_t)vg + W - 1) / W * W);
  uint32_t* id_of_pos = A.take_n<uint32_t>(m);
  KeyCols o;
  o.k0 = A.take_n<uint64_t>(vpad);
  o.k1 = A.take_n<uint64_t>(vpad);
  o.sref_off = A.take_n<uint64_t>(vpad);
  o.sref_len = A.take_n<uint32_t>(vpad);
  launch_union_assign(pos, flag, rep, ex, K0, K1, SO, SL, m, n_max, a_max, id_of_pos, o.k0, o.k1, o.sref_off,
                      o.sref_len, s);

  // 4-6. dense counts: scatter, reduce-scatter, all-gather
  uint64_t* dcnt = A.take_n<uint64_t>(vpad);
  uint64_t* dfirst = A.take_n<uint64_t>(vpad);
  uint64_t* scnt = A.take_n<uint64_t>(vpad / W);
  uint64_t* sfirst = A.take_n<uint64_t>(vpad / W);
  o.cnt = A.take_n<uint64_t>(vpad);
  o.first = A.take_n<uint64_t>(vpad);
  WC_HIP_CHECK(hipMemsetAsync(dcnt, 0, vpad * 8, s));
  launch_fill_u64(dfirst, ~0ull, vpad, s);
  launch_scatter_dense(id_of_pos + (size_t)R * n_max, im.cols.cnt, im.cols.first, dcnt, dfirst, n, s);
  comm.reduce_scatter_u64(dcnt, scnt, vpad / W, RedOp::Sum, s);
  comm.reduce_scatter_u64(dfirst, sfirst, vpad / W, RedOp::Min, s);
  comm.allgather(scnt, o.cnt, vpad / W * 8, s);
  comm.allgather(sfirst, o.first, vpad / W * 8, s);
  comm.sync(s);

  o.n = vg;
  im.cols = o;
  im.cols_arena = AR;
  im.cols_arena_bytes = (uint64_t)W * a_max;
  im.max_end = gmax_end;
}


namespace {
template <class T>
T* take_aligned(DeviceArena& A, size_t n) {
  return A.take_n<T>(n ? n : 1);
}
}  // namespace

// Small-vocabulary variant of the shuffle merge (see merge_cols_shuffle):
// pack all local rows (one "owner"), send them to rank 0, merge there.
void merge_to_root(Engine::Impl& im, Comm& comm, const std::vector<uint64_t>& rank_rows,
                   const std::vector<uint64_t>& rank_bytes, uint64_t gmax_end) {
  Range rg("wc_merge_root");
  hipStream_t s = im.s;
  const int W = comm.size(), R = comm.rank();
  const uint64_t n = im.cols.n;
  const uint64_t my_rows = rank_rows[R], my_bytes = rank_bytes[R];
  uint64_t rr = 0, rbt = 0;  // received by rank 0
  std::vector<size_t> zs(W, 0), sr(W, 0), sb(W, 0), ro_r(W, 0), rb_r(W, 0), ro_b(W, 0), rb_b(W, 0);
  std::vector<uint64_t> base(2 * (size_t)W + 2, 0);
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
  unsigned long long* d_cur = take_aligned<unsigned long long>(A, 4);  // zero counts (2) | cursor (2)
  WC_HIP_CHECK(hipMemsetAsync(d_cur, 0, 4 * 8, s));
  launch_owner_scatter(im.cols.k0, im.cols.k1, im.cols.cnt, im.cols.first, im.cols.sref_off, im.cols.sref_len,
                       im.cols_arena, n, 1u, d_cur, d_cur + 2, send_rows, send_bytes, s);
  comm.group_begin();
  comm.alltoallv(send_rows, zs.data(), sr.data(), recv_rows, ro_r.data(), rb_r.data(), s);
  comm.alltoallv(send_bytes, zs.data(), sb.data(), recv_bytes, ro_b.data(), rb_b.data(), s);
  comm.group_end();
  KeyCols o;
  uint64_t gb[4] = {0, 0, 0, rbt};  // one output group (rows 0..G, byte base 0); outlives its async H2D
  if (R == 0) {
    uint32_t* state = take_aligned<uint32_t>(A, T);
    unsigned long long* tcnt = take_aligned<unsigned long long>(A, T);
    unsigned long long* tfirst = take_aligned<unsigned long long>(A, T);
    MRow* merged = take_aligned<MRow>(A, rr);
    uint64_t* d_base = take_aligned<uint64_t>(A, base.size() + 4);
    unsigned long long* d_m = take_aligned<unsigned long long>(A, 1);
    WC_HIP_CHECK(hipMemcpyAsync(d_base, base.data(), base.size() * 8, hipMemcpyHostToDevice, s));
    WC_HIP_CHECK(hipMemsetAsync(state, 0, T * 4, s));
    WC_HIP_CHECK(hipMemsetAsync(tcnt, 0, T * 8, s));
    launch_fill_u64(reinterpret_cast<uint64_t*>(tfirst), ~0ull, T, s);
    WC_HIP_CHECK(hipMemsetAsync(d_m, 0, 8, s));
    launch_mrow_insert(recv_rows, rr, recv_bytes, d_base, d_base + W + 1, (uint32_t)W, state, tcnt, tfirst, T, s);
    launch_mrow_compact(recv_rows, state, tcnt, tfirst, T, d_base, d_base + W + 1, (uint32_t)W, merged, d_m, s);
    unsigned long long G = 0;
    WC_HIP_CHECK(hipMemcpyAsync(&G, d_m, 8, hipMemcpyDeviceToHost, s));
    comm.sync(s);
    o.n = G;
    o.k0 = take_aligned<uint64_t>(A, G);
    o.k1 = take_aligned<uint64_t>(A, G);
    o.cnt = take_aligned<uint64_t>(A, G);
    o.first = take_aligned<uint64_t>(A, G);
    o.sref_off = take_aligned<uint64_t>(A, G);
    o.sref_len = take_aligned<uint32_t>(A, G);
    uint64_t* d_gbase = d_base + base.size();  // one group: row base 0 .. G, byte base 0
    gb[1] = G;
    WC_HIP_CHECK(hipMemcpyAsync(d_gbase, gb, sizeof gb, hipMemcpyHostToDevice, s));
    launch_mrow_to_cols(merged, G, d_gbase, d_gbase + 2, 1u, o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, s);
  }
  comm.sync(s);  // also: base[] / gb[] are pageable host memory
  im.cols = o;
  im.cols_arena = recv_bytes;
  im.cols_arena_bytes = R == 0 ? rbt : 0;
  im.max_end = gmax_end;
}

void merge_cols_shuffle(Engine::Impl& im, Comm& comm, bool all_ranks) {
  Range rg("wc_merge_shuffle");
  hipStream_t s = im.s;
  const int W = comm.size(), R = comm.rank();
  WC_CHECK(W <= (int)MERGE_MAX_RANKS, "shuffle merge supports at most 64 ranks");
  const uint64_t n = im.cols.n;
  const size_t C = 2 * (size_t)W + 1;  // per rank: (rows, bytes) per owner + max offset

  // 1. owner counts, exchanged as a W x C matrix (small buffers: own arena)
  DeviceArena& S = im.merge_small;
  S.reserve(((size_t)W * C + 2 * C + 4 * (size_t)W + 16) * 8 + 8 * 1024);
  unsigned long long* d_cnt = take_aligned<unsigned long long>(S, 2 * C);  // counts | cursor
  unsigned long long* d_all = take_aligned<unsigned long long>(S, (size_t)W * C);
  WC_HIP_CHECK(hipMemsetAsync(d_cnt, 0, 2 * C * 8, s));
  const unsigned long long mx = im.max_end;
  WC_HIP_CHECK(hipMemcpyAsync(d_cnt + 2 * W, &mx, 8, hipMemcpyHostToDevice, s));
  launch_owner_count(im.cols.k0, im.cols.k1, im.cols.sref_len, n, (uint32_t)W, d_cnt, s);
  comm.allgather(d_cnt, d_all, C * 8, s);
  std::vector<unsigned long long> all((size_t)W * C);
  WC_HIP_CHECK(hipMemcpyAsync(all.data(), d_all, all.size() * 8, hipMemcpyDeviceToHost, s));
  comm.sync(s);
  uint64_t gmax_end = 0;
  for (int r = 0; r < W; ++r) gmax_end = std::max<uint64_t>(gmax_end, all[(size_t)r * C + 2 * W]);
  std::vector<uint64_t> rank_rows(W, 0), rank_bytes(W, 0);
  uint64_t total_rows = 0;
  for (int r = 0; r < W; ++r) {
    for (int p = 0; p < W; ++p) {
      rank_rows[r] += all[(size_t)r * C + 2 * p];
      rank_bytes[r] += all[(size_t)r * C + 2 * p + 1];
    }
    total_rows += rank_rows[r];
  }
  // Few keys in total: every rank sends its rows straight to rank 0, which
  // merges them alone — one exchange instead of two (owner exchange + gather)
  // and one host sync fewer.  WC_MERGE_ROOT_ROWS overrides the threshold.
  uint64_t root_max = MERGE_ROOT_MAX_ROWS;
  if (const char* e = std::getenv("WC_MERGE_ROOT_ROWS")) root_max = std::strtoull(e, nullptr, 10);
  if (!all_ranks && total_rows <= root_max) {
    merge_to_root(im, comm, rank_rows, rank_bytes, gmax_end);
    return;
  }

  // 2. pack by owner and exchange
  std::vector<size_t> so_r(W), sb_r(W), so_b(W), sb_b(W), ro_r(W), rb_r(W), ro_b(W), rb_b(W);
  size_t tr = 0, tb = 0, rr = 0, rbt = 0;
  for (int p = 0; p < W; ++p) {
    const unsigned long long* mine = &all[(size_t)R * C];
    so_r[p] = tr * sizeof(MRow);
    sb_r[p] = mine[2 * p] * sizeof(MRow);
    so_b[p] = tb;
    sb_b[p] = mine[2 * p + 1];
    tr += mine[2 * p];
    tb += mine[2 * p + 1];
    const unsigned long long* theirs = &all[(size_t)p * C];
    ro_r[p] = rr * sizeof(MRow);
    rb_r[p] = theirs[2 * R] * sizeof(MRow);
    ro_b[p] = rbt;
    rb_b[p] = theirs[2 * R + 1];
    rr += theirs[2 * R];
    rbt += theirs[2 * R + 1];
  }
  uint64_t T = 1024;
  while (T < 2 * rr) T <<= 1;
  // upper bounds of the gathered table: every row / byte of every rank
  uint64_t Gmax = 0, GBmax = 0;
  for (int r = 0; r < W; ++r)
    for (int p = 0; p < W; ++p) {
      Gmax += all[(size_t)r * C + 2 * p];
      GBmax += all[(size_t)r * C + 2 * p + 1];
    }
  DeviceArena& A = im.merge_mem;
  A.reserve((tr + 2 * rr + Gmax) * sizeof(MRow) + tb + 2 * rbt + GBmax + T * (4 + 16) + Gmax * (5 * 8 + 4) +
            (4 * (size_t)W + 4) * 8 + 32 * 1024);
  MRow* send_rows = take_aligned<MRow>(A, tr);
  uint8_t* send_bytes = take_aligned<uint8_t>(A, tb);
  MRow* recv_rows = take_aligned<MRow>(A, rr);
  uint8_t* recv_bytes = take_aligned<uint8_t>(A, rbt);
  launch_owner_scatter(im.cols.k0, im.cols.k1, im.cols.cnt, im.cols.first, im.cols.sref_off, im.cols.sref_len,
                       im.cols_arena, n, (uint32_t)W, d_cnt, d_cnt + C, send_rows, send_bytes, s);
  comm.group_begin();  // rows and long-word bytes in one exchange
  comm.alltoallv(send_rows, so_r.data(), sb_r.data(), recv_rows, ro_r.data(), rb_r.data(), s);
  comm.alltoallv(send_bytes, so_b.data(), sb_b.data(), recv_bytes, ro_b.data(), rb_b.data(), s);
  comm.group_end();

  // 3. owner-side merge
  uint32_t* state = take_aligned<uint32_t>(A, T);
  unsigned long long* tcnt = take_aligned<unsigned long long>(A, T);
  unsigned long long* tfirst = take_aligned<unsigned long long>(A, T);
  MRow* merged = take_aligned<MRow>(A, rr);
  uint64_t* d_base = take_aligned<uint64_t>(A, 2 * (size_t)W + 2);  // row / byte bases per source (then per owner)
  unsigned long long* d_m = take_aligned<unsigned long long>(A, 1);
  std::vector<uint64_t> base(2 * (size_t)W + 2);
  for (int p = 0; p < W; ++p) {
    base[p] = ro_r[p] / sizeof(MRow);
    base[W + 1 + p] = ro_b[p];
  }
  base[W] = rr;
  base[2 * W + 1] = rbt;
  WC_HIP_CHECK(hipMemcpyAsync(d_base, base.data(), base.size() * 8, hipMemcpyHostToDevice, s));
  WC_HIP_CHECK(hipMemsetAsync(state, 0, T * 4, s));
  WC_HIP_CHECK(hipMemsetAsync(tcnt, 0, T * 8, s));
  launch_fill_u64(reinterpret_cast<uint64_t*>(tfirst), ~0ull, T, s);
  WC_HIP_CHECK(hipMemsetAsync(d_m, 0, 8, s));
  launch_mrow_insert(recv_rows, rr, recv_bytes, d_base, d_base + W + 1, (uint32_t)W, state, tcnt, tfirst, T, s);
  launch_mrow_compact(recv_rows, state, tcnt, tfirst, T, d_base, d_base + W + 1, (uint32_t)W, merged, d_m, s);

  // 4. gather merged rows + bytes to rank 0 (and broadcast for all_ranks)
  // (merged rows, bytes) of every owner: the row count stays on the device
  // until this allgather, so one host sync serves both
  const unsigned long long own_bytes = rbt;
  unsigned long long* d_own = take_aligned<unsigned long long>(A, 2);
  unsigned long long* d_owns = take_aligned<unsigned long long>(A, 2 * (size_t)W);
  WC_HIP_CHECK(hipMemcpyAsync(d_own, d_m, 8, hipMemcpyDeviceToDevice, s));
  WC_HIP_CHECK(hipMemcpyAsync(d_own + 1, &own_bytes, 8, hipMemcpyHostToDevice, s));
  comm.allgather(d_own, d_owns, 16, s);
  std::vector<unsigned long long> owns(2 * (size_t)W);
  WC_HIP_CHECK(hipMemcpyAsync(owns.data(), d_owns, owns.size() * 8, hipMemcpyDeviceToHost, s));
  comm.sync(s);  // also: base[] / own_bytes are pageable host memory
  const unsigned long long own[2] = {owns[2 * (size_t)R], own_bytes};
  std::vector<size_t> go_r(W, 0), gb_r(W, 0), go_b(W, 0), gb_b(W, 0), zs(W, 0);
  std::vector<size_t> sr(W, 0), sb(W, 0);
  uint64_t G = 0, GB = 0;
  std::vector<uint64_t> gbase(2 * (size_t)W + 2);
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
  sr[0] = own[0] * sizeof(MRow);
  sb[0] = own[1];
  const bool have = R == 0 || all_ranks;
  MRow* grows = take_aligned<MRow>(A, G);
  uint8_t* gbytes = take_aligned<uint8_t>(A, GB);
  comm.group_begin();
  comm.alltoallv(merged, zs.data(), sr.data(), grows, go_r.data(), gb_r.data(), s);
  comm.alltoallv(recv_bytes, zs.data(), sb.data(), gbytes, go_b.data(), gb_b.data(), s);
  comm.group_end();
  if (all_ranks) {
    comm.group_begin();
    comm.broadcast(grows, G * sizeof(MRow), 0, s);
    comm.broadcast(gbytes, GB, 0, s);
    comm.group_end();
  }
  KeyCols o;
  o.n = have ? G : 0;
  if (have) {
    o.k0 = take_aligned<uint64_t>(A, G);
    o.k1 = take_aligned<uint64_t>(A, G);
    o.cnt = take_aligned<uint64_t>(A, G);
    o.first = take_aligned<uint64_t>(A, G);
    o.sref_off = take_aligned<uint64_t>(A, G);
    o.sref_len = take_aligned<uint32_t>(A, G);
    uint64_t* d_gbase = take_aligned<uint64_t>(A, gbase.size());
    WC_HIP_CHECK(hipMemcpyAsync(d_gbase, gbase.data(), gbase.size() * 8, hipMemcpyHostToDevice, s));
    launch_mrow_to_cols(grows, G, d_gbase, d_gbase + W + 1, (uint32_t)W, o.k0, o.k1, o.cnt, o.first, o.sref_off,
                        o.sref_len, s);
  }
  comm.sync(s);
  im.cols = o;
  im.cols_arena = gbytes;
  im.cols_arena_bytes = have ? GB : 0;
  im.max_end = gmax_end;
}

void merge_cols(Engine::Impl& im, Comm& comm, bool all_ranks) {
  if (im.opt.merge_mode == 1) merge_cols_dense(im, comm);
  else merge_cols_shuffle(im, comm, all_ranks);
}

}  // namespace wc
