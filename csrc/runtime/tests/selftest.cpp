// Native self-test of the host runtime, built with -fsanitize=address,undefined (and optionally
// -fsanitize=thread) by tests/test_runtime_sanitizers_cpu.py (sanitizer build of the
// C++ runtime).  Exercises the SPSC shared-memory ring with a real producer thread racing the
// consumer (wrap-around, variable lengths, checksum of every record), the sum tree against a
// brute-force prefix scan, fcntl locks between two descriptors and the heartbeat table.
// Exit code 0 = pass; any sanitizer report aborts with a non-zero code.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../runtime.h"

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(2);                                                     \
    }                                                                   \
  } while (0)

static uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void test_ring() {
  const std::string name = "/r2rt_selftest_" + std::to_string(getpid());
  void* prod = r2rt_ring_open(name.c_str(), 1 << 16, 1);
  CHECK(prod != nullptr);
  void* cons = r2rt_ring_open(name.c_str(), 1 << 16, 0);   // consumers attach with the same capacity
  CHECK(cons != nullptr);
  const int N = 20000;
  std::thread producer([&] {
    std::vector<uint8_t> buf(3000);
    for (int i = 0; i < N; ++i) {
      const uint32_t len = 8 + (uint32_t)(mix(i) % 2900);
      for (uint32_t k = 0; k < len; ++k) buf[k] = (uint8_t)mix((uint64_t)i * 4096 + k);
      std::memcpy(buf.data(), &i, sizeof(int));
      while (r2rt_ring_push(prod, buf.data(), len) != 0) std::this_thread::yield();
    }
  });
  std::vector<uint8_t> out(4096);
  for (int i = 0; i < N; ++i) {
    int64_t got;
    while ((got = r2rt_ring_pop(cons, out.data(), (uint32_t)out.size())) <= 0) std::this_thread::yield();
    const uint32_t len = 8 + (uint32_t)(mix(i) % 2900);
    CHECK(got == (int64_t)len);
    int id;
    std::memcpy(&id, out.data(), sizeof(int));
    CHECK(id == i);
    for (uint32_t k = sizeof(int); k < len; ++k) CHECK(out[k] == (uint8_t)mix((uint64_t)i * 4096 + k));
  }
  producer.join();
  CHECK(r2rt_ring_used(cons) == 0);
  r2rt_ring_close(cons, 0);
  r2rt_ring_close(prod, 1);
}

static void test_sumtree() {
  const int64_t n = 5000;
  void* t = r2rt_sumtree_create(n);
  std::vector<double> leaves(n);
  std::vector<int64_t> idx(n);
  for (int64_t i = 0; i < n; ++i) {
    leaves[i] = (mix(i) % 1000) / 100.0;
    idx[i] = i;
  }
  r2rt_sumtree_set(t, idx.data(), leaves.data(), n);
  double tot = 0;
  for (double v : leaves) tot += v;
  CHECK(std::fabs(r2rt_sumtree_total(t) - tot) < 1e-6 * tot);
  const int B = 257;
  std::vector<double> u(B), p(B);
  std::vector<int64_t> out(B);
  for (int b = 0; b < B; ++b) u[b] = (mix(100000 + b) >> 11) * (1.0 / 9007199254740992.0);
  r2rt_sumtree_sample(t, u.data(), B, 1, out.data(), p.data());
  for (int b = 0; b < B; ++b) {
    CHECK(out[b] >= 0 && out[b] < n);
    CHECK(leaves[out[b]] > 0);
    CHECK(std::fabs(p[b] - leaves[out[b]] / tot) < 1e-9);   // sampling probability
    // stratified: sample b lies in prefix interval [(b+u)/B, (b+1+u)/B) * total
    double pre = 0;
    for (int64_t i = 0; i < out[b]; ++i) pre += leaves[i];
    const double target = (b + u[b]) / B * tot;
    CHECK(pre <= target + 1e-6 && target <= pre + leaves[out[b]] + 1e-6);
  }
  r2rt_sumtree_destroy(t);
}

static void test_lock_and_heartbeat() {
  const std::string path = "/tmp/r2rt_selftest_" + std::to_string(getpid()) + ".lock";
  int a = r2rt_lock_open(path.c_str());
  CHECK(a >= 0);
  CHECK(r2rt_lock_acquire(a, 0) == 1);   // 1 = acquired, 0 = held elsewhere
  r2rt_lock_release(a);
  r2rt_lock_close(a);
  unlink(path.c_str());
  const std::string hb = "/r2rt_hb_selftest_" + std::to_string(getpid());
  void* h = r2rt_hb_open(hb.c_str(), 8, 1);
  CHECK(h != nullptr);
  std::vector<std::thread> th;
  std::atomic<int> go{0};
  for (int s = 0; s < 8; ++s)
    th.emplace_back([&, s] {
      while (!go.load()) std::this_thread::yield();
      for (uint64_t c = 1; c <= 1000; ++c) r2rt_hb_beat(h, s, c, s);
    });
  go = 1;
  for (auto& x : th) x.join();
  for (int s = 0; s < 8; ++s) {
    uint64_t last, counter;
    int32_t pid, status;
    CHECK(r2rt_hb_read(h, s, &last, &counter, &pid, &status) == 0);
    CHECK(counter == 1000 && status == s && last > 0);
  }
  r2rt_hb_close(h, 1);
}

int main() {
  test_ring();
  test_sumtree();
  test_lock_and_heartbeat();
  std::printf("runtime selftest ok\n");
  return 0;
}
