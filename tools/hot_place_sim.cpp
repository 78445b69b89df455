// CPU model of the map's hot-table selection and placement (map.hip
// build_image / place_hot) on the synthetic generator's vocabulary: Poisson
// sample counts (~310k sampled tokens per GiB job), a slot budget, then one
// placement mode; prints the miss share and the per-bucket weight spread.
//   g++ -O2 -std=c++17 -Isrc -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
//       tools/hot_place_sim.cpp src/io/synth_host.cpp -o /tmp/hot_place_sim
//   /tmp/hot_place_sim SLOT_BUDGET MODE [VOCAB]
// MODE 0 greedy by count (the kernel's order), 1 two-word words first,
// 3 cuckoo (BFS displacement), 4 every selected word placed (the capacity
// bound), 5 / 6 tiered greedy + one- / two-level displacement repairs,
// 7 the kernel: BUDGET words by sampled count (not slots), tiered greedy,
// 8 slot-valued selection, 9 = 7 with two-word words first in each tier,
// 10 one image builder per job (greedy tiers + priority-eviction walks; built
// on the GPU in round 6 and dropped: its single block cost more than it saved),
// 11 the shipped round-6 placement: each of 256 partitions (8 groups; a
// word's two groups in its partition) places its own sampled words by count
// (SIM_REPAIR=1: + the one-level move of map.hip place_partition).
// SIM_ONE_SLOT8=1: 8-byte words as one-slot words; SIM_FIRST_SLOT8=1: only in
// an empty group's first slot.
// profiles/r5_session.md §12.
#include "io/synth_host.hpp"
#include "kernels/keys.hpp"
#include <cstdio>
#include <cmath>
#include <vector>
#include <random>
#include <algorithm>
#include <cstdlib>
using namespace wc;
int main(int argc, char** argv) {
  SynthSpec sp; sp.vocab = argc > 3 ? atoi(argv[3]) : 100000;
  HostVocab v = build_vocab(sp);
  const uint32_t n = sp.vocab, NG = 2048;
  const uint32_t BUDGET = argc > 1 ? atoi(argv[1]) : 3800;   // slots
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  const double SAMPLE = 310e3;
  std::vector<double> p(n); double z = 0;
  for (uint32_t i = 0; i < n; ++i) z += p[i] = 1.0 / std::pow(i + 1.0, sp.zipf_s);
  const double T = 158.6e6;
  std::mt19937_64 rng(7);
  std::vector<uint32_t> c(n), ph(n);
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t k0, k1; key_of(&v.bytes[v.off[i]], v.len[i], &k0, &k1);
    ph[i] = place_hash(k0, k1);
    std::poisson_distribution<int> pd(SAMPLE * p[i] / z);
    c[i] = pd(rng);
  }
  const uint32_t two_from = getenv("SIM_ONE_SLOT8") ? 9u : 8u;  // 8-byte words as one-slot words (raw k0 signature)
  auto slots = [&](uint32_t i) { return v.len[i] >= two_from ? 2u : 1u; };
  std::vector<uint32_t> cand; for (uint32_t i = 0; i < n; ++i) if (c[i]) cand.push_back(i);
  std::shuffle(cand.begin(), cand.end(), rng);
  // selection by value per slot (c / slots), budget in slots
  std::stable_sort(cand.begin(), cand.end(), [&](uint32_t a, uint32_t b) { return (double)c[a] / slots(a) > (double)c[b] / slots(b); });
  std::vector<uint32_t> take; uint32_t used = 0;
  if (mode == 8) {  // slot-valued selection: histogram key c / slots, each word weighing its slots, BUDGET slots
    std::vector<uint32_t> hist(4096, 0);
    for (auto i : cand) hist[std::min(c[i] / slots(i), 4095u)] += slots(i);
    uint32_t t = 4095, suf = 0;
    for (int b = 4095; b >= 1; --b) { if (suf + hist[b] > BUDGET) { t = b + 1; break; } suf += hist[b]; t = b; }
    for (auto i : cand) if (c[i] / slots(i) >= t) take.push_back(i);
  } else if (mode == 7 || mode == 9) {  // the kernel's selection (map.hip wave_count_threshold): BUDGET words by sampled count, ties at t - 1 while room
    std::vector<uint32_t> hist(4096, 0);
    for (auto i : cand) hist[std::min(c[i], 4095u)]++;
    uint32_t t = 4095, suf = 0;
    for (int b = 4095; b >= 1; --b) { if (suf + hist[b] > BUDGET) { t = b + 1; break; } suf += hist[b]; t = b; }
    uint32_t cum = 0; for (uint32_t b = t; b < 4096; ++b) cum += hist[b];
    uint32_t ties = t > 1 ? BUDGET - std::min(cum, BUDGET) : 0;
    for (auto i : cand) if (c[i] >= t) take.push_back(i);
    for (auto i : cand) if (c[i] + 1 == t && ties) { take.push_back(i); --ties; }
  } else {
    for (auto i : cand) { if (used + slots(i) > BUDGET) continue; used += slots(i); take.push_back(i); }
  }
  // placement order
  std::vector<uint32_t> ord = take;
  if (mode == 0) std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return c[a] > c[b]; });
  if (mode == 1) std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { if (slots(a) != slots(b)) return slots(a) > slots(b); return c[a] > c[b]; });
  std::vector<uint32_t> gocc(NG, 0);
  std::vector<uint32_t> gw0(NG, ~0u), gw1(NG, ~0u);  // one-slot words in the group (for cuckoo)
  std::vector<char> placed(n, 0);
  auto groups = [&](uint32_t i, uint32_t& g1, uint32_t& g2) { g1 = (ph[i] >> 20) & (NG - 1); g2 = g1 ^ (((ph[i] >> 8) & (NG - 1)) | 1u); };
  // mode 3: cuckoo (one-slot words kick one-slot occupants; two-word words take an empty group or relocate a lone one-slot occupant)
  std::vector<uint32_t> slot(2 * NG, ~0u);  // one-slot word per slot; two-word groups marked in gocc == 3
  auto try_insert1 = [&](uint32_t i) -> bool {
    // BFS over groups: a free slot reachable by moving one-slot occupants to their other group
    uint32_t g1, g2; groups(i, g1, g2);
    std::vector<int> prevg(NG, -2); std::vector<int> via(NG, -1);  // via: slot index whose occupant moved into this group
    std::vector<uint32_t> q;
    for (uint32_t g : {g1, g2}) if (gocc[g] != 3 && prevg[g] == -2) { prevg[g] = -1; q.push_back(g); }
    for (size_t h = 0; h < q.size() && h < 4000; ++h) {
      uint32_t g = q[h];
      for (int s = 0; s < 2; ++s) if (slot[2 * g + s] == ~0u) {
        // unwind: move occupants along the path
        uint32_t tg = g, ts = 2 * g + s;
        while (prevg[tg] != -1) {
          uint32_t from = via[tg];  // slot in previous group whose occupant goes to tg
          slot[ts] = slot[from]; gocc[tg]++; gocc[from / 2]--;
          slot[from] = ~0u; ts = from; tg = from / 2;
        }
        slot[ts] = i; gocc[tg]++;
        return true;
      }
      for (int s = 0; s < 2; ++s) {
        uint32_t j = slot[2 * g + s]; uint32_t h1, h2; groups(j, h1, h2); uint32_t alt = h1 == g ? h2 : h1;
        if (gocc[alt] == 3 || prevg[alt] != -2) continue;
        prevg[alt] = g; via[alt] = 2 * g + s; q.push_back(alt);
      }
    }
    return false;
  };
  std::vector<uint32_t> towner(NG, ~0u);
  if (mode == 4) { for (auto i : take) placed[i] = 1; ord.clear(); }
  if (mode >= 5 && mode != 10 && mode != 11) {
    // thresholds as the GPU: t from counts; tiers big=8t, mid=2t
    uint32_t mn = ~0u; for (auto i : take) mn = std::min(mn, c[i]);
    const uint32_t t = mn + 1, big = 8 * t, mid = 2 * t;
    std::vector<uint32_t> occ1(2 * NG, ~0u);  // one-slot occupants
    std::vector<char> two(NG, 0);
    auto free_slot = [&](uint32_t g) -> int { if (two[g]) return -1; for (int s = 0; s < 2; ++s) if (occ1[2*g+s] == ~0u) return s; return -1; };
    auto nocc = [&](uint32_t g) { return two[g] ? 2 : (occ1[2*g] != ~0u) + (occ1[2*g+1] != ~0u); };
    std::vector<uint32_t> failed;
    auto place = [&](uint32_t i) -> bool {
      uint32_t g1, g2; groups(i, g1, g2);
      if (slots(i) == 2) {
        for (uint32_t g : {g1, g2}) if (!two[g] && nocc(g) == 0) { two[g] = 1; towner[g] = i; return true; }
        return false;
      }
      if (getenv("SIM_FIRST_SLOT8") && v.len[i] == 8) {  // one-slot 8-byte word, first slot of an empty group only
        for (uint32_t g : {g1, g2}) if (!two[g] && nocc(g) == 0) { occ1[2*g] = i; return true; }
        return false;
      }
      if (nocc(g2) < nocc(g1)) std::swap(g1, g2);
      for (uint32_t g : {g1, g2}) { int s = free_slot(g); if (s >= 0) { occ1[2*g+s] = i; return true; } }
      return false;
    };
    auto repair = [&](uint32_t i) -> bool {  // move one occupant of g1/g2 to its alternate group
      uint32_t g1, g2; groups(i, g1, g2);
      for (uint32_t g : {g1, g2}) {
        if (two[g]) continue;
        if (slots(i) == 2 && nocc(g) != 1) continue;
        for (int s = 0; s < 2; ++s) {
          uint32_t j = occ1[2*g+s]; if (j == ~0u) continue;
          uint32_t h1, h2; groups(j, h1, h2); uint32_t alt = h1 == g ? h2 : h1;
          int fs = free_slot(alt);
          if (fs < 0 && mode == 6) {  // second level: an occupant of alt moves to its alternate
            for (int s2 = 0; s2 < 2 && fs < 0; ++s2) {
              uint32_t k = occ1[2*alt+s2]; if (k == ~0u || two[alt]) continue;
              uint32_t q1, q2; groups(k, q1, q2); uint32_t alt2 = q1 == alt ? q2 : q1;
              if (alt2 == g) continue;
              int f2 = free_slot(alt2); if (f2 < 0) continue;
              occ1[2*alt2+f2] = k; occ1[2*alt+s2] = ~0u; fs = s2;
            }
          }
          if (fs < 0) continue;
          occ1[2*alt+fs] = j; occ1[2*g+s] = ~0u;
          if (slots(i) == 2) { two[g] = 1; towner[g] = i; } else occ1[2*g+s] = i;
          return true;
        }
      }
      return false;
    };
    for (int pass = 0; pass < 3; ++pass) {
      std::vector<uint32_t> tier;
      for (auto i : take) { int tr = c[i] >= big ? 0 : (c[i] >= mid ? 1 : 2); if (tr == pass) tier.push_back(i); }
      std::shuffle(tier.begin(), tier.end(), rng);
      if (mode == 9) std::stable_sort(tier.begin(), tier.end(), [&](uint32_t a, uint32_t b) { return slots(a) > slots(b); });
      std::vector<uint32_t> f;
      for (auto i : tier) if (!place(i)) f.push_back(i);
      if (mode == 5 || mode == 6) for (auto i : f) repair(i);
    }
    for (uint32_t s = 0; s < 2 * NG; ++s) if (occ1[s] != ~0u) placed[occ1[s]] = 1;
    for (uint32_t g = 0; g < NG; ++g) if (towner[g] != ~0u) placed[towner[g]] = 1;
    ord.clear();
  }
  if (mode == 11) {
    // partition-local placement (round 6): group g1 = ph bits [20, 31), g2 = g1 ^
    // (bits [8, 11) | 1) — both in g1's partition of 8 groups (ph bits [23, 31)),
    // so each partition's 16 slots are placed by its own merge block: its
    // sampled words by count (value per slot with SIM_VALUE=1), greedy 2-choice
    take.clear();
    std::vector<std::vector<uint32_t>> part(256);
    for (auto i : cand) part[(ph[i] >> 23) & 255].push_back(i);
    auto g2of = [&](uint32_t i) { uint32_t g1 = (ph[i] >> 20) & (NG - 1); return g1 ^ (((ph[i] >> 8) & 7u) | 1u); };
    std::vector<uint32_t> occ(NG, 0);
    std::vector<std::vector<uint32_t>> who(NG);  // one-slot occupants
    const bool value = getenv("SIM_VALUE") != nullptr;
    const uint32_t TOP = getenv("SIM_TOP") ? atoi(getenv("SIM_TOP")) : 32;
    for (auto& P : part) {
      std::stable_sort(P.begin(), P.end(), [&](uint32_t a, uint32_t b) {
        if (value) return (double)c[a] / slots(a) > (double)c[b] / slots(b);
        return c[a] > c[b]; });
      if (P.size() > TOP) P.resize(TOP);
      for (auto i : P) {
        take.push_back(i);
        uint32_t g1 = (ph[i] >> 20) & (NG - 1), g2 = g2of(i);
        if (slots(i) == 2) {
          if (occ[g1] == 0) { occ[g1] = 2; placed[i] = 1; }
          else if (occ[g2] == 0) { occ[g2] = 2; placed[i] = 1; }
          continue;
        }
        if (occ[g2] < occ[g1]) std::swap(g1, g2);
        if (occ[g1] < 2) { occ[g1]++; placed[i] = 1; who[g1].push_back(i); }
        else if (occ[g2] < 2) { occ[g2]++; placed[i] = 1; who[g2].push_back(i); }
        else if (getenv("SIM_REPAIR")) {  // move a one-slot occupant of g1 / g2 to its other group
          bool done = false;
          for (uint32_t g : {g1, g2}) {
            if (done) break;
            for (size_t q = 0; q < who[g].size() && !done; ++q) {
              uint32_t o = who[g][q]; uint32_t a1 = (ph[o] >> 20) & (NG - 1), a2 = g2of(o), alt = a1 == g ? a2 : a1;
              if (occ[alt] < 2) { occ[alt]++; who[alt].push_back(o); who[g][q] = i; placed[i] = 1; done = true; }
            }
          }
        }
      }
    }
    ord.clear();
  }
  if (mode == 10) {
    // the round-6 image builder (map.hip build_image_once): BUDGET words by sampled
    // count (ties while room); per count tier (8t, 2t, rest): two-word words into an
    // empty group (2-choice) else evicting a lower-count two-word owner, then one-slot
    // words by a random walk that takes a free slot or evicts a lower-count one-slot
    // occupant (<= 64 moves), the last item of a walk dropped
    std::vector<uint32_t> hist(4096, 0);
    for (auto i : cand) hist[std::min(c[i], 4095u)]++;
    uint32_t t = 4095, suf = 0;
    for (int b = 4095; b >= 1; --b) { if (suf + hist[b] > BUDGET) { t = b + 1; break; } suf += hist[b]; t = b; }
    uint32_t cum = 0; for (uint32_t b = t; b < 4096; ++b) cum += hist[b];
    uint32_t ties = t > 1 ? BUDGET - std::min(cum, BUDGET) : 0;
    take.clear();
    for (auto i : cand) if (c[i] >= t) take.push_back(i);
    for (auto i : cand) if (c[i] + 1 == t && ties) { take.push_back(i); --ties; }
    const uint32_t tt = t, big = 8 * tt, mid = 2 * tt;
    std::vector<uint32_t> two(NG, ~0u), occ(2 * NG, ~0u);
    auto other = [&](uint32_t i, uint32_t g) { uint32_t g1, g2; groups(i, g1, g2); return g1 == g ? g2 : g1; };
    // one walk: place `item`, evicting strictly lower-count occupants; returns when placed or dropped
    auto walk = [&](uint32_t item) {
      for (int it = 0; it < 64; ++it) {
        uint32_t g1, g2; groups(item, g1, g2);
        auto nf = [&](uint32_t g) { return two[g] != ~0u ? 0 : (occ[2*g] == ~0u) + (occ[2*g+1] == ~0u); };
        if (slots(item) == 2) {
          bool done = false;
          for (uint32_t g : {g1, g2}) if (!done && nf(g) == 2) { two[g] = item; done = true; }
          if (done) return;
          // evict: a lower-count two-word owner, or a lone lower-count one-slot occupant
          uint32_t bg = ~0u, bc = ~0u;
          for (uint32_t g : {g1, g2}) {
            uint32_t o = two[g] != ~0u ? two[g] : (nf(g) == 1 ? (occ[2*g] != ~0u ? occ[2*g] : occ[2*g+1]) : ~0u);
            if (o != ~0u && c[o] < c[item] && c[o] < bc) { bc = c[o]; bg = g; }
          }
          if (bg == ~0u) return;
          uint32_t o = two[bg] != ~0u ? two[bg] : (occ[2*bg] != ~0u ? occ[2*bg] : occ[2*bg+1]);
          occ[2*bg] = occ[2*bg+1] = ~0u; two[bg] = item; item = o;
          continue;
        }
        if (nf(g2) > nf(g1)) std::swap(g1, g2);
        if (nf(g1) > 0) { occ[2*g1 + (occ[2*g1] == ~0u ? 0 : 1)] = item; return; }
        if (!getenv("SIM_NO_MOVE")) {  // a one-slot occupant with room in its other group moves there (nothing lost)
          bool moved = false;
          for (uint32_t g : {g1, g2}) {
            if (moved || two[g] != ~0u) continue;
            for (int h = 0; h < 2 && !moved; ++h) {
              uint32_t o = occ[2*g+h], alt = other(o, g);
              if (nf(alt) == 0) continue;
              occ[2*alt + (occ[2*alt] == ~0u ? 0 : 1)] = o; occ[2*g+h] = item; moved = true;
            }
          }
          if (moved) return;
        }
        // evict the lowest-count lower occupant: a one-slot word, or a two-word owner (its group then has a free half)
        uint32_t bs = ~0u, bc = ~0u; bool btwo = false;
        for (uint32_t g : {g1, g2}) {
          if (two[g] != ~0u) { if (c[two[g]] < c[item] && c[two[g]] < bc) { bc = c[two[g]]; bs = g; btwo = true; } continue; }
          for (int h = 0; h < 2; ++h) { uint32_t o = occ[2*g+h]; if (c[o] < c[item] && c[o] < bc) { bc = c[o]; bs = 2*g+h; btwo = false; } }
        }
        if (bs == ~0u) return;
        if (btwo) { uint32_t o = two[bs]; two[bs] = ~0u; occ[2*bs] = item; item = o; }
        else { uint32_t o = occ[bs]; occ[bs] = item; item = o; }
      }
    };
    for (int pass = 0; pass < 3; ++pass)
      for (int phase = 0; phase < 2; ++phase) {
        std::vector<uint32_t> tier;
        for (auto i : take) {
          int tr = c[i] >= big ? 0 : (c[i] >= mid ? 1 : 2);
          if (tr == pass && (slots(i) == 2) == (phase == 0)) tier.push_back(i);
        }
        std::shuffle(tier.begin(), tier.end(), rng);
        for (auto i0 : tier) walk(i0);
      }
    uint32_t n2 = 0, n1 = 0;
    for (uint32_t s = 0; s < 2 * NG; ++s) if (occ[s] != ~0u) { placed[occ[s]] = 1; ++n1; }
    for (uint32_t g = 0; g < NG; ++g) if (two[g] != ~0u) { placed[two[g]] = 1; ++n2; }
    if (getenv("SIM_DEBUG")) printf("two-word groups %u, one-slot words %u\n", n2, n1);
    ord.clear();
    (void)other;
  }
  if (mode == 3) {
    std::vector<uint32_t> o = take;
    std::stable_sort(o.begin(), o.end(), [&](uint32_t a, uint32_t b) { return c[a] > c[b]; });
    for (auto i : o) {
      uint32_t g1, g2; groups(i, g1, g2);
      if (slots(i) == 2) {
        bool done = false;
        for (uint32_t g : {g1, g2}) if (!done && gocc[g] == 0) { gocc[g] = 3; towner[g] = i; done = true; }
        for (uint32_t g : {g1, g2}) {
          if (done || gocc[g] != 1) continue;
          const int s0 = slot[2 * g] != ~0u ? 0 : 1;
          const uint32_t j = slot[2 * g + s0];
          slot[2 * g + s0] = ~0u; gocc[g] = 3;
          if (try_insert1(j)) { towner[g] = i; done = true; }
          else { gocc[g] = 1; slot[2 * g + s0] = j; }
        }
        continue;
      }
      try_insert1(i);
    }
    // placed = words in slots + two-word groups: recompute
    std::fill(placed.begin(), placed.end(), 0);
    for (uint32_t s = 0; s < 2 * NG; ++s) if (slot[s] != ~0u) placed[slot[s]] = 1;
    for (uint32_t g = 0; g < NG; ++g) if (towner[g] != ~0u) placed[towner[g]] = 1;
    ord.clear();
  }
  for (auto i : ord) {
    uint32_t g1, g2; groups(i, g1, g2);
    if (slots(i) == 2) {
      if (gocc[g1] == 0) { gocc[g1] = 2; placed[i] = 1; }
      else if (gocc[g2] == 0) { gocc[g2] = 2; placed[i] = 1; }
      else if (mode == 2) {  // try to evict a single one-slot word to its other group
        for (uint32_t g : {g1, g2}) {
          if (gocc[g] != 1 || gw0[g] == ~0u) continue;
          uint32_t j = gw0[g], h1, h2; groups(j, h1, h2); uint32_t alt = h1 == g ? h2 : h1;
          if (gocc[alt] < 2 && gw1[alt] == ~0u && (gocc[alt] == 0 || gw0[alt] != ~0u)) {
            if (gocc[alt] == 0) gw0[alt] = j; else gw1[alt] = j; gocc[alt]++;
            gocc[g] = 2; gw0[g] = ~0u; placed[i] = 1; break;
          }
        }
      }
      continue;
    }
    if (gocc[g2] < gocc[g1]) std::swap(g1, g2);
    uint32_t g = gocc[g1] < 2 ? g1 : (gocc[g2] < 2 ? g2 : ~0u);
    if (g == ~0u) continue;
    if (gocc[g] == 0) gw0[g] = i; else gw1[g] = i;
    gocc[g]++; placed[i] = 1;
  }
  double miss = 0; uint32_t np = 0, ns = 0;
  std::vector<double> w(64, 0);
  for (uint32_t i = 0; i < n; ++i) { np += placed[i]; if (placed[i]) ns += slots(i); if (!placed[i]) { double e = T * p[i] / z; miss += e; w[ph[i] & 63] += e; } }
  double mx = *std::max_element(w.begin(), w.end());
  printf("budget %u mode %d: taken %zu placed %u words / %u slots, miss %.2fM (%.1f%%), bucket max/mean %.3f\n", BUDGET, mode, take.size(), np, ns, miss / 1e6, 100 * miss / T, mx / (miss / 64));
}
