// Shared-memory SPSC ring, fcntl locks and heartbeat table (see runtime.h).
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <new>
#include <string>

#include "runtime.h"

namespace {

constexpr uint64_t RING_MAGIC = 0x52324432524e4731ull;  // "R2D2RNG1"
constexpr uint32_t WRAP = 0xFFFFFFFFu;

struct alignas(64) RingHdr {
  uint64_t magic;
  uint64_t capacity;                 // payload bytes (multiple of 8)
  alignas(64) std::atomic<uint64_t> head;  // bytes ever written (producer)
  alignas(64) std::atomic<uint64_t> tail;  // bytes ever consumed (consumer)
};

struct Ring {
  RingHdr* hdr;
  uint8_t* data;
  size_t map_len;
  std::string name;
};

inline uint64_t pad8(uint64_t x) { return (x + 7) & ~7ull; }

struct alignas(64) HbSlot {
  std::atomic<uint64_t> last_ns;
  std::atomic<uint64_t> counter;
  std::atomic<int32_t> pid;
  std::atomic<int32_t> status;
};

struct HbHdr {
  uint64_t magic;
  int32_t n_slots;
  int32_t pad;
};

struct Hb {
  HbHdr* hdr;
  HbSlot* slots;
  size_t map_len;
  std::string name;
};

void* map_shm(const std::string& name, size_t len, int create) {
  int fd = shm_open(name.c_str(), create ? (O_CREAT | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return nullptr;
  if (create && ftruncate(fd, (off_t)len) != 0) {
    close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  return p == MAP_FAILED ? nullptr : p;
}

}  // namespace

extern "C" {

void* r2rt_ring_open(const char* name, uint64_t capacity, int create) {
  capacity = pad8(capacity);
  const size_t len = sizeof(RingHdr) + capacity;
  void* p = map_shm(name, len, create);
  if (!p) return nullptr;
  auto* hdr = static_cast<RingHdr*>(p);
  if (create) {
    new (&hdr->head) std::atomic<uint64_t>(0);
    new (&hdr->tail) std::atomic<uint64_t>(0);
    hdr->capacity = capacity;
    std::atomic_thread_fence(std::memory_order_release);
    hdr->magic = RING_MAGIC;
  } else if (hdr->magic != RING_MAGIC || hdr->capacity != capacity) {
    munmap(p, len);
    return nullptr;
  }
  auto* r = new Ring{hdr, static_cast<uint8_t*>(p) + sizeof(RingHdr), len, name};
  return r;
}

// 0 = pushed, 1 = not enough space (retry later), -1 = record larger than the ring
int r2rt_ring_push(void* rp, const void* data, uint32_t len) {
  auto* r = static_cast<Ring*>(rp);
  const uint64_t cap = r->hdr->capacity;
  const uint64_t need = pad8(4 + (uint64_t)len);
  if (need + 8 > cap) return -1;
  const uint64_t head = r->hdr->head.load(std::memory_order_relaxed);
  const uint64_t tail = r->hdr->tail.load(std::memory_order_acquire);
  uint64_t pos = head % cap;
  uint64_t extra = 0;
  if (pos + need > cap) extra = cap - pos;  // skip to the start with a wrap marker
  if (head + extra + need - tail > cap) return 1;
  if (extra) {
    memcpy(r->data + pos, &WRAP, 4);
    pos = 0;
  }
  memcpy(r->data + pos, &len, 4);
  memcpy(r->data + pos + 4, data, len);
  r->hdr->head.store(head + extra + need, std::memory_order_release);
  return 0;
}

static int64_t ring_front(Ring* r, uint64_t* tail_io, uint64_t* pos_out) {
  const uint64_t cap = r->hdr->capacity;
  uint64_t tail = *tail_io;
  const uint64_t head = r->hdr->head.load(std::memory_order_acquire);
  if (tail == head) return -1;
  uint64_t pos = tail % cap;
  uint32_t len;
  if (cap - pos < 4) {  // too small for a marker: producer always skips these bytes
    tail += cap - pos;
    pos = 0;
  }
  memcpy(&len, r->data + pos, 4);
  if (len == WRAP) {
    tail += cap - pos;
    pos = 0;
    memcpy(&len, r->data + pos, 4);
  }
  *tail_io = tail;
  *pos_out = pos;
  return (int64_t)len;
}

int64_t r2rt_ring_peek(void* rp) {
  auto* r = static_cast<Ring*>(rp);
  uint64_t tail = r->hdr->tail.load(std::memory_order_relaxed), pos;
  return ring_front(r, &tail, &pos);
}

// returns record length, -1 if empty, -2 if maxlen too small (record left in place)
int64_t r2rt_ring_pop(void* rp, void* out, uint32_t maxlen) {
  auto* r = static_cast<Ring*>(rp);
  uint64_t tail = r->hdr->tail.load(std::memory_order_relaxed), pos;
  const int64_t len = ring_front(r, &tail, &pos);
  if (len < 0) return -1;
  if ((uint64_t)len > maxlen) return -2;
  memcpy(out, r->data + pos + 4, (size_t)len);
  r->hdr->tail.store(tail + pad8(4 + (uint64_t)len), std::memory_order_release);
  return len;
}

int64_t r2rt_ring_front(void* rp, const void** payload) {
  auto* r = static_cast<Ring*>(rp);
  uint64_t tail = r->hdr->tail.load(std::memory_order_relaxed), pos;
  const int64_t len = ring_front(r, &tail, &pos);
  if (len < 0) return -1;
  *payload = r->data + pos + 4;
  return len;
}

void r2rt_ring_release(void* rp) {
  auto* r = static_cast<Ring*>(rp);
  uint64_t tail = r->hdr->tail.load(std::memory_order_relaxed), pos;
  const int64_t len = ring_front(r, &tail, &pos);
  if (len < 0) return;
  r->hdr->tail.store(tail + pad8(4 + (uint64_t)len), std::memory_order_release);
}

uint64_t r2rt_ring_used(void* rp) {
  auto* r = static_cast<Ring*>(rp);
  return r->hdr->head.load(std::memory_order_acquire) - r->hdr->tail.load(std::memory_order_acquire);
}

// the whole mapping (header + payload): registered with the HIP runtime for zero-copy DMA
void* r2rt_ring_mapping(void* rp, uint64_t* len) {
  auto* r = static_cast<Ring*>(rp);
  *len = r->map_len;
  return r->hdr;
}

uint64_t r2rt_ring_capacity(void* rp) { return static_cast<Ring*>(rp)->hdr->capacity; }

void r2rt_ring_close(void* rp, int unlink_it) {
  auto* r = static_cast<Ring*>(rp);
  munmap(r->hdr, r->map_len);
  if (unlink_it) shm_unlink(r->name.c_str());
  delete r;
}

// ---------------------------------------------------------------- seqlock slot
struct alignas(64) SlotHdr {
  uint64_t magic;
  uint64_t bytes;
  alignas(64) std::atomic<uint64_t> seq;      // odd while a write is in progress
  std::atomic<int64_t> version;
};

struct Slot {
  SlotHdr* hdr;
  uint8_t* data;
  size_t map_len;
  std::string name;
};

void* r2rt_slot_open(const char* name, uint64_t bytes, int create) {
  const size_t len = sizeof(SlotHdr) + pad8(bytes);
  void* p = map_shm(name, len, create);
  if (!p) return nullptr;
  auto* hdr = static_cast<SlotHdr*>(p);
  if (create) {
    new (&hdr->seq) std::atomic<uint64_t>(0);
    new (&hdr->version) std::atomic<int64_t>(-1);
    hdr->bytes = bytes;
    std::atomic_thread_fence(std::memory_order_release);
    hdr->magic = RING_MAGIC + 2;
  } else if (hdr->magic != RING_MAGIC + 2 || hdr->bytes != bytes) {
    munmap(p, len);
    return nullptr;
  }
  return new Slot{hdr, static_cast<uint8_t*>(p) + sizeof(SlotHdr), len, name};
}

void r2rt_slot_write(void* sp, const void* data, uint64_t bytes, int64_t version) {
  auto* s = static_cast<Slot*>(sp);
  if (bytes > s->hdr->bytes) bytes = s->hdr->bytes;
  const uint64_t q = s->hdr->seq.load(std::memory_order_relaxed);
  s->hdr->seq.store(q + 1, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  memcpy(s->data, data, bytes);
  s->hdr->version.store(version, std::memory_order_relaxed);
  s->hdr->seq.store(q + 2, std::memory_order_release);
}

int r2rt_slot_read(void* sp, void* out, uint64_t bytes, int64_t have, int64_t* version) {
  auto* s = static_cast<Slot*>(sp);
  if (bytes > s->hdr->bytes) bytes = s->hdr->bytes;
  for (int attempt = 0; attempt < 64; ++attempt) {
    const uint64_t q0 = s->hdr->seq.load(std::memory_order_acquire);
    if (q0 & 1) {
      usleep(50);
      continue;
    }
    const int64_t v = s->hdr->version.load(std::memory_order_relaxed);
    if (v <= have) return 0;
    memcpy(out, s->data, bytes);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (s->hdr->seq.load(std::memory_order_relaxed) == q0) {
      *version = v;
      return 1;
    }
  }
  return -1;
}

int64_t r2rt_slot_version(void* sp) {
  return static_cast<Slot*>(sp)->hdr->version.load(std::memory_order_acquire);
}

void r2rt_slot_close(void* sp, int unlink_it) {
  auto* s = static_cast<Slot*>(sp);
  munmap(s->hdr, s->map_len);
  if (unlink_it) shm_unlink(s->name.c_str());
  delete s;
}

// ---------------------------------------------------------------- fcntl locks
int r2rt_lock_open(const char* path) { return open(path, O_CREAT | O_RDWR, 0644); }

int r2rt_lock_acquire(int fd, int blocking) {
  struct flock fl;
  memset(&fl, 0, sizeof(fl));
  fl.l_type = F_WRLCK;
  fl.l_whence = SEEK_SET;
  const int rc = fcntl(fd, blocking ? F_SETLKW : F_SETLK, &fl);
  if (rc == 0) return 1;
  return (errno == EACCES || errno == EAGAIN) ? 0 : -1;
}

int r2rt_lock_release(int fd) {
  struct flock fl;
  memset(&fl, 0, sizeof(fl));
  fl.l_type = F_UNLCK;
  fl.l_whence = SEEK_SET;
  return fcntl(fd, F_SETLK, &fl) == 0 ? 0 : -1;
}

void r2rt_lock_close(int fd) { close(fd); }

// ---------------------------------------------------------------- heartbeat table
uint64_t r2rt_now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

void* r2rt_hb_open(const char* name, int n_slots, int create) {
  const size_t len = sizeof(HbHdr) + 64 + sizeof(HbSlot) * (size_t)n_slots;
  void* p = map_shm(name, len, create);
  if (!p) return nullptr;
  auto* hdr = static_cast<HbHdr*>(p);
  auto* slots = reinterpret_cast<HbSlot*>(static_cast<uint8_t*>(p) + 64);
  if (create) {
    for (int i = 0; i < n_slots; ++i) {
      new (&slots[i].last_ns) std::atomic<uint64_t>(0);
      new (&slots[i].counter) std::atomic<uint64_t>(0);
      new (&slots[i].pid) std::atomic<int32_t>(0);
      new (&slots[i].status) std::atomic<int32_t>(0);
    }
    hdr->n_slots = n_slots;
    std::atomic_thread_fence(std::memory_order_release);
    hdr->magic = RING_MAGIC + 1;
  } else if (hdr->magic != RING_MAGIC + 1 || hdr->n_slots != n_slots) {
    munmap(p, len);
    return nullptr;
  }
  return new Hb{hdr, slots, len, name};
}

void r2rt_hb_beat(void* hp, int slot, uint64_t counter, int32_t status) {
  auto* h = static_cast<Hb*>(hp);
  if (slot < 0 || slot >= h->hdr->n_slots) return;
  HbSlot& s = h->slots[slot];
  s.pid.store((int32_t)getpid(), std::memory_order_relaxed);
  s.counter.store(counter, std::memory_order_relaxed);
  s.status.store(status, std::memory_order_relaxed);
  s.last_ns.store(r2rt_now_ns(), std::memory_order_release);
}

int r2rt_hb_read(void* hp, int slot, uint64_t* last_ns, uint64_t* counter, int32_t* pid,
                 int32_t* status) {
  auto* h = static_cast<Hb*>(hp);
  if (slot < 0 || slot >= h->hdr->n_slots) return -1;
  HbSlot& s = h->slots[slot];
  *last_ns = s.last_ns.load(std::memory_order_acquire);
  *counter = s.counter.load(std::memory_order_relaxed);
  *pid = s.pid.load(std::memory_order_relaxed);
  *status = s.status.load(std::memory_order_relaxed);
  return 0;
}

void r2rt_hb_close(void* hp, int unlink_it) {
  auto* h = static_cast<Hb*>(hp);
  munmap(h->hdr, h->map_len);
  if (unlink_it) shm_unlink(h->name.c_str());
  delete h;
}
}
