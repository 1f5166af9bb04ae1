// Host 64-ary sum tree (see runtime.h).
#include <algorithm>
#include <cmath>
#include <vector>

#include "runtime.h"

namespace {
constexpr int F = 64;

struct SumTree {
  int64_t cap;
  std::vector<int64_t> size;         // per level
  std::vector<std::vector<double>> lv;  // lv[0] = leaves, lv.back() = root (size 1)
};

void recompute(SumTree* t, int level, int64_t node) {
  // node is at `level`, recompute from children at level-1
  const auto& ch = t->lv[level - 1];
  const int64_t c0 = node * F, c1 = std::min<int64_t>(c0 + F, t->size[level - 1]);
  double s = 0.0;
  for (int64_t c = c0; c < c1; ++c) s += ch[c];
  t->lv[level][node] = s;
}
}  // namespace

extern "C" {

void* r2rt_sumtree_create(int64_t capacity) {
  if (capacity < 1) return nullptr;
  auto* t = new SumTree();
  t->cap = capacity;
  int64_t n = capacity;
  t->size.push_back(n);
  while (n > 1) {
    n = (n + F - 1) / F;
    t->size.push_back(n);
  }
  if (t->size.size() < 2) t->size.push_back(1);
  for (int64_t s : t->size) t->lv.emplace_back(s, 0.0);
  return t;
}

void r2rt_sumtree_destroy(void* p) { delete static_cast<SumTree*>(p); }

int64_t r2rt_sumtree_capacity(void* p) { return static_cast<SumTree*>(p)->cap; }

void r2rt_sumtree_set(void* p, const int64_t* idx, const double* val, int64_t n) {
  auto* t = static_cast<SumTree*>(p);
  std::vector<int64_t> dirty;
  dirty.reserve(n);
  for (int64_t i = 0; i < n; ++i) {
    if (idx[i] < 0 || idx[i] >= t->cap) continue;
    t->lv[0][idx[i]] = val[i] > 0.0 ? val[i] : 0.0;
    dirty.push_back(idx[i]);
  }
  for (size_t l = 1; l < t->lv.size(); ++l) {
    for (auto& d : dirty) d /= F;
    std::sort(dirty.begin(), dirty.end());
    dirty.erase(std::unique(dirty.begin(), dirty.end()), dirty.end());
    for (int64_t d : dirty) recompute(t, (int)l, d);
  }
}

void r2rt_sumtree_rebuild(void* p, const double* leaves) {
  auto* t = static_cast<SumTree*>(p);
  for (int64_t i = 0; i < t->cap; ++i) t->lv[0][i] = leaves[i] > 0.0 ? leaves[i] : 0.0;
  for (size_t l = 1; l < t->lv.size(); ++l)
    for (int64_t nd = 0; nd < t->size[l]; ++nd) recompute(t, (int)l, nd);
}

double r2rt_sumtree_total(void* p) { return static_cast<SumTree*>(p)->lv.back()[0]; }

double r2rt_sumtree_get(void* p, int64_t idx) {
  auto* t = static_cast<SumTree*>(p);
  return (idx >= 0 && idx < t->cap) ? t->lv[0][idx] : 0.0;
}

// u01: n uniforms in [0,1).  stratified: sample i targets [(i+u)/n, ...) of the total mass.
void r2rt_sumtree_sample(void* p, const double* u01, int64_t n, int stratified, int64_t* out_idx,
                         double* out_p) {
  auto* t = static_cast<SumTree*>(p);
  const double total = t->lv.back()[0];
  const int top = (int)t->lv.size() - 1;
  for (int64_t i = 0; i < n; ++i) {
    double u = (stratified ? (i + u01[i]) / (double)n : u01[i]) * total;
    int64_t node = 0;
    for (int l = top; l >= 1; --l) {
      const auto& ch = t->lv[l - 1];
      const int64_t c0 = node * F, c1 = std::min<int64_t>(c0 + F, t->size[l - 1]);
      int64_t pick = -1, last_nz = -1;
      for (int64_t c = c0; c < c1; ++c) {
        if (ch[c] <= 0.0) continue;
        last_nz = c;
        if (u < ch[c]) {
          pick = c;
          break;
        }
        u -= ch[c];
      }
      if (pick < 0) {  // float round-off past the end
        pick = last_nz >= 0 ? last_nz : c0;
        u = 0.0;
      }
      node = pick;
    }
    out_idx[i] = node;
    if (out_p) out_p[i] = total > 0.0 ? t->lv[0][node] / total : 0.0;
  }
}

int r2rt_version() { return 1; }
}
