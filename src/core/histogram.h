// Log-linear latency histogram (HDR-style: 64 sub-buckets per power of two, ~1.6 %
// relative precision) for the load generator and the server --profile mode. Mergeable across threads/processes.
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

namespace hola {

class Histogram {
 public:
  static constexpr int kSub = 64;
  static constexpr int kOctaves = 42;  // up to ~2^42 ns (~73 min)
  static constexpr int kBins = kSub + kOctaves * kSub;

  Histogram() : h_(kBins, 0) {}
  static int bin_of(uint64_t v) {
    if (v < kSub) return int(v);
    int msb = 63 - __builtin_clzll(v);
    int sub = int((v >> (msb - 6)) & (kSub - 1));
    int b = kSub + (msb - 6) * kSub + sub;
    return b >= kBins ? kBins - 1 : b;
  }
  // Midpoint of the bin's value range.
  static uint64_t bin_value(int b) {
    if (b < kSub) return uint64_t(b);
    int oct = (b - kSub) / kSub, sub = (b - kSub) % kSub;
    int msb = oct + 6;
    uint64_t lo = (uint64_t(1) << msb) + (uint64_t(sub) << (msb - 6));
    return lo + ((uint64_t(1) << (msb - 6)) >> 1);
  }
  void add(uint64_t v) {
    ++h_[size_t(bin_of(v))];
    ++count_;
    sum_ += v;
    max_ = std::max(max_, v);
    min_ = std::min(min_, v);
  }
  void merge(const Histogram& o) {
    for (int i = 0; i < kBins; ++i) h_[size_t(i)] += o.h_[size_t(i)];
    count_ += o.count_;
    sum_ += o.sum_;
    max_ = std::max(max_, o.max_);
    min_ = std::min(min_, o.min_);
  }
  void reset() {
    std::fill(h_.begin(), h_.end(), 0);
    count_ = sum_ = max_ = 0;
    min_ = UINT64_MAX;
  }
  uint64_t count() const { return count_; }
  uint64_t max() const { return max_; }
  double mean() const { return count_ ? double(sum_) / double(count_) : 0; }
  uint64_t percentile(double p) const {
    if (!count_) return 0;
    uint64_t need = uint64_t(p / 100.0 * double(count_) + 0.5);
    if (need < 1) need = 1;
    if (need > count_) need = count_;
    uint64_t acc = 0;
    for (int i = 0; i < kBins; ++i) {
      acc += h_[size_t(i)];
      if (acc >= need) return std::min(bin_value(i), max_);
    }
    return max_;
  }
  // Sparse "bin:count,..." encoding for cross-process merging.
  std::string encode() const {
    std::string s;
    for (int i = 0; i < kBins; ++i)
      if (h_[size_t(i)]) {
        if (!s.empty()) s += ',';
        s += std::to_string(i) + ":" + std::to_string(h_[size_t(i)]);
      }
    return s;
  }

 private:
  std::vector<uint64_t> h_;
  uint64_t count_ = 0, sum_ = 0, max_ = 0, min_ = UINT64_MAX;
};

}  // namespace hola
