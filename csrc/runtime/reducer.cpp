// Gradient bucket assignment + readiness tracking for DistributedDataParallel.
//
// The reference gets this from torch's C++ Reducer behind `DDP(model, device_ids=[gpu_id])`
// (`PY1:35`, gradient all-reduce in `loss.backward()` `PY1:41`).  MI355X sizing: with 7
// point-to-point xGMI links a bucket should give every peer >= 1-4 MB per ring step, so buckets
// default to tens of MB while the first bucket stays small so the all-reduce starts early in backward.
#include <algorithm>
#include <stdexcept>

#include "runtime.h"

namespace pda_rt {

BucketReducer::BucketReducer(const std::vector<int64_t>& numels, const std::vector<int64_t>& elem_sizes,
                             const std::vector<int>& dtype_ids, int64_t bucket_cap_bytes, int64_t first_bucket_bytes,
                             int64_t align_elems, const std::vector<int64_t>& order) {
  const size_t P = numels.size();
  if (elem_sizes.size() != P || dtype_ids.size() != P) throw std::invalid_argument("reducer: size mismatch");
  param_bucket_.assign(P, -1);
  ready_.assign(P, 0);
  std::vector<int64_t> ord = order;
  if (ord.empty()) {  // default: reverse registration order (closest static guess of backward order)
    for (size_t i = 0; i < P; ++i) ord.push_back((int64_t)(P - 1 - i));
  }
  if (ord.size() != P) throw std::invalid_argument("reducer: order must list every parameter once");
  if (align_elems < 1) align_elems = 1;
  // one open bucket per dtype; the very first bucket is capped at first_bucket_bytes
  std::map<int, int> open;
  std::map<int, int64_t> open_bytes, open_cap;
  for (int64_t p : ord) {
    if (p < 0 || (size_t)p >= P || param_bucket_[p] != -1) throw std::invalid_argument("reducer: bad order");
    const int dt = dtype_ids[p];
    const int64_t bytes = numels[p] * elem_sizes[p];
    if (!open.count(dt) || (open_bytes[dt] > 0 && open_bytes[dt] + bytes > open_cap[dt])) {
      open_cap[dt] = buckets_.empty() ? first_bucket_bytes : bucket_cap_bytes;
      buckets_.push_back(Bucket());
      buckets_.back().dtype = dt;
      open[dt] = (int)buckets_.size() - 1;
      open_bytes[dt] = 0;
    }
    Bucket& b = buckets_[open[dt]];
    b.params.push_back(p);
    b.offsets.push_back(b.numel);
    b.numel += (numels[p] + align_elems - 1) / align_elems * align_elems;  // keep every view 16-B aligned
    open_bytes[dt] += bytes;
    param_bucket_[p] = open[dt];
  }
  prepare();
}

void BucketReducer::prepare() {
  std::fill(ready_.begin(), ready_.end(), 0);
  ready_order_.clear();
  for (auto& b : buckets_) b.pending = (int)b.params.size();
  next_launch_ = 0;
}

std::vector<int> BucketReducer::mark_ready(int64_t p) {
  std::vector<int> launch;
  if (p < 0 || (size_t)p >= ready_.size()) throw std::out_of_range("reducer: parameter index");
  if (ready_[p]) {
    throw std::runtime_error(
        "reducer: parameter " + std::to_string(p) +
        " produced a gradient twice in one iteration (reentrant backward / shared parameter used twice is not "
        "supported without no_sync)");
  }
  ready_[p] = 1;
  ready_order_.push_back(p);
  buckets_[param_bucket_[p]].pending--;
  while (next_launch_ < (int)buckets_.size() && buckets_[next_launch_].pending == 0) launch.push_back(next_launch_++);
  return launch;
}

std::vector<int> BucketReducer::flush_unready() {
  std::vector<int> launch;
  for (size_t p = 0; p < ready_.size(); ++p) {
    if (!ready_[p]) {
      auto l = mark_ready((int64_t)p);
      launch.insert(launch.end(), l.begin(), l.end());
    }
  }
  return launch;
}

std::vector<int64_t> BucketReducer::unready_params() const {
  std::vector<int64_t> out;
  for (size_t p = 0; p < ready_.size(); ++p)
    if (!ready_[p]) out.push_back((int64_t)p);
  return out;
}

}  // namespace pda_rt
