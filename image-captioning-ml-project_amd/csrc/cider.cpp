// CIDEr-D on the host: the SCST reward.
//
// Replaces src/evaluate/metrics.py:46-110 (pycocoevalcap's CiderD scorer, called by
// CaptioningTrainer._calculate_rewards, src/train/trainer.py:440-484).  pycocoevalcap is
// not installed here (and its Java tokenizer cannot run): this restates the published
// scorer (Vedantam et al. 2015; pycocoevalcap cider_scorer.py with the CiderD
// clipping and Gaussian length penalty) on token ids:
//
//   * n-grams n = 1..4 of each candidate and reference ("cooking");
//   * document frequency df(g) = number of corpus entries (images) whose reference set
//     contains g; ref_len = log(#images);
//   * vec_n(g) = tf(g) * (ref_len - log(max(1, df(g)))), norm_n = ||vec_n||,
//     "length" = number of bigrams (the scorer counts term frequencies of n == 2);
//   * sim_n(h, r) = sum_g min(vh(g), vr(g)) * vr(g) / (|vh| |vr|) * exp(-(lh - lr)^2 / (2 sigma^2));
//   * score = mean_n( sum_r sim_n(h, r) ) / #refs * 10.
//
// Each cooked sentence is a sorted vector of (n-gram key, weight), so a similarity is a
// merge join; candidates are scored on host threads.  The CPU restatement it is checked
// against lives in oracle/cider.py (tests/test_cider.py).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/capk.h"

namespace {

struct Key {
  uint64_t lo, hi;  // up to 4 int32 tokens of one n-gram order (unused slots 0)
  bool operator==(const Key& o) const { return lo == o.lo && hi == o.hi; }
  bool operator<(const Key& o) const { return lo < o.lo || (lo == o.lo && hi < o.hi); }
};
struct KeyHash {
  size_t operator()(const Key& k) const {
    uint64_t h = k.lo * 0x9E3779B97F4A7C15ull ^ (k.hi + 0x632BE59BD9B4E019ull + (k.lo << 6) + (k.lo >> 2));
    h ^= h >> 31;
    return (size_t)(h * 0xBF58476D1CE4E5B9ull);
  }
};

constexpr int NMAX = 4;

// one sentence: per order, sorted (key, term frequency)
struct Cooked {
  std::vector<std::pair<Key, double>> g[NMAX];
};

Key make_key(const int32_t* t, int n) {
  uint32_t w[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) w[i] = (uint32_t)t[i];
  return Key{(uint64_t)w[0] | ((uint64_t)w[1] << 32), (uint64_t)w[2] | ((uint64_t)w[3] << 32)};
}

void cook(const int32_t* t, int64_t len, int nmax, Cooked& c) {
  for (int n = 1; n <= nmax; ++n) {
    auto& v = c.g[n - 1];
    v.clear();
    if (len < n) continue;
    v.reserve(len - n + 1);
    for (int64_t i = 0; i + n <= len; ++i) v.push_back({make_key(t + i, n), 1.0});
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    size_t o = 0;  // merge duplicates -> term frequencies
    for (size_t i = 0; i < v.size(); ++i) {
      if (o > 0 && v[o - 1].first == v[i].first) v[o - 1].second += 1.0;
      else v[o++] = v[i];
    }
    v.resize(o);
  }
}

struct Vec {
  std::vector<std::pair<Key, double>> g[NMAX];
  double norm[NMAX];
  double length;
};

using DF = std::unordered_map<Key, double, KeyHash>;

void to_vec(const Cooked& c, const DF* df, double ref_len, int nmax, Vec& v) {
  v.length = 0.0;
  for (int n = 0; n < nmax; ++n) {
    v.g[n].resize(c.g[n].size());
    double nn = 0.0;
    for (size_t i = 0; i < c.g[n].size(); ++i) {
      const auto& kv = c.g[n][i];
      auto it = df[n].find(kv.first);
      const double d = std::log(std::max(1.0, it == df[n].end() ? 0.0 : it->second));
      const double w = kv.second * (ref_len - d);
      v.g[n][i] = {kv.first, w};
      nn += w * w;
      if (n == 1) v.length += kv.second;
    }
    v.norm[n] = std::sqrt(nn);
  }
}

void sim(const Vec& h, const Vec& r, int nmax, double sigma, double* out) {
  const double delta = h.length - r.length;
  const double pen = std::exp(-(delta * delta) / (2.0 * sigma * sigma));
  for (int n = 0; n < nmax; ++n) {
    double val = 0.0;
    const auto& a = h.g[n];
    const auto& b = r.g[n];
    size_t i = 0, j = 0;
    while (i < a.size() && j < b.size()) {
      if (a[i].first < b[j].first) ++i;
      else if (b[j].first < a[i].first) ++j;
      else {
        val += std::min(a[i].second, b[j].second) * b[j].second;
        ++i;
        ++j;
      }
    }
    if (h.norm[n] != 0.0 && r.norm[n] != 0.0) val /= h.norm[n] * r.norm[n];
    out[n] += val * pen;
  }
}

template <typename F>
void parallel_for(int64_t n, int threads, F&& f, int64_t min_n = 64) {
  if (threads <= 1 || n < min_n) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int64_t> next{0};
  std::vector<std::thread> pool;
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(16, n / (2 * (int64_t)threads)));
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&] {
      for (int64_t i; (i = next.fetch_add(chunk)) < n;)
        for (int64_t k = i; k < std::min(n, i + chunk); ++k) f(k);
    });
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" int capk_cider_d(int n_cand, const int32_t* cand_tok, const int64_t* cand_off, const int32_t* ref_tok,
                            const int64_t* ref_off, const int64_t* ref_img, int n_max, double sigma, int threads,
                            double* scores) {
  if (n_cand < 0 || n_max < 1 || n_max > NMAX || !scores || (n_cand > 0 && (!cand_off || !ref_off || !ref_img)))
    return CAPK_EINVAL;
  if (n_cand == 0) return CAPK_OK;
  if (threads <= 0) {
    // the process's CPU share, not the node's: a GPU box exposes every core of the node
    // (hardware_concurrency 256) to a 16-CPU cgroup, and one std::thread per core per
    // parallel_for costs more than the scoring itself
    threads = (int)std::max(1u, std::thread::hardware_concurrency());
    if (const char* e = getenv("OMP_NUM_THREADS")) threads = std::min(threads, std::max(1, atoi(e)));
    threads = std::min(threads, 16);
  }
  const int64_t n_ref = ref_img[n_cand];
  std::vector<Cooked> rc(n_ref);
  parallel_for(n_ref, threads, [&](int64_t r) { cook(ref_tok + ref_off[r], ref_off[r + 1] - ref_off[r], n_max, rc[r]); });
  // document frequency: once per image for every n-gram in the union of its references
  // (per order: each image's unique keys, all images' lists sorted together and counted)
  DF df[NMAX];
  parallel_for(
      n_max, std::min(threads, n_max), [&](int64_t n) {
    std::vector<Key> all, u;
    for (int i = 0; i < n_cand; ++i) {
      u.clear();
      for (int64_t r = ref_img[i]; r < ref_img[i + 1]; ++r)
        for (const auto& kv : rc[r].g[n]) u.push_back(kv.first);
      std::sort(u.begin(), u.end());
      u.erase(std::unique(u.begin(), u.end()), u.end());
      all.insert(all.end(), u.begin(), u.end());
    }
    std::sort(all.begin(), all.end());
    df[n].reserve(all.size());
    for (size_t i = 0; i < all.size();) {
      size_t j = i;
      while (j < all.size() && all[j] == all[i]) ++j;
      df[n].emplace(all[i], (double)(j - i));
      i = j;
    }
  }, 1);
  const double ref_len = std::log((double)n_cand);
  parallel_for(n_cand, threads, [&](int64_t i) {
    Cooked c;
    cook(cand_tok + cand_off[i], cand_off[i + 1] - cand_off[i], n_max, c);
    Vec vh, vr;
    to_vec(c, df, ref_len, n_max, vh);
    double acc[NMAX] = {0, 0, 0, 0};
    const int64_t nr = ref_img[i + 1] - ref_img[i];
    for (int64_t r = ref_img[i]; r < ref_img[i + 1]; ++r) {
      to_vec(rc[r], df, ref_len, n_max, vr);
      sim(vh, vr, n_max, sigma, acc);
    }
    double mean = 0.0;
    for (int n = 0; n < n_max; ++n) mean += acc[n];
    mean /= n_max;
    scores[i] = nr > 0 ? mean / (double)nr * 10.0 : 0.0;
  });
  return CAPK_OK;
}
